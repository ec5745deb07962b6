// Device-side restatement of the shading math on the BDPT / PT path:
// vector algebra (math/vector.cpp), frames (math/frame.cpp), samplers
// (sampler/sampler.cpp), Fresnel + BSDF (material/fresnel.cpp, bsdf.h, bsdf.cpp),
// AreaLight (scene/light.cpp), camera (scene/camera.cpp, math/transform.h).
//
// Every expression keeps the reference's float evaluation order; the
// translation units that include this file are built with -ffp-contract=off and
// HIP's default correctly-rounded f32 divide / sqrt, and the libm calls of the
// reference (cosf / sinf / powf) go through wr_libm.h, which returns glibc's
// float bit for bit, so every value equals the CPU oracle's.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "wr_libm.h"

namespace wrd {

#define WR_EPS 1e-3f
#define WR_INF 1e7f
#define WR_PI 3.14159274101257324f          /* (float)acos(-1.0) */
#define WR_INV_PI 0.318309873342514038f     /* 1.0f / WR_PI, rounded as the reference */

__device__ __forceinline__ int cmpf(float x) { return (x < -WR_EPS) ? -1 : (x > WR_EPS); }
__device__ __forceinline__ float smax(float a, float b) { return (a < b) ? b : a; }
__device__ __forceinline__ float smin(float a, float b) { return (b < a) ? b : a; }
__device__ __forceinline__ float clampv(float v, float lo, float hi) { return smin(hi, smax(v, lo)); }

struct V3 {
  float x, y, z;
};
__host__ __device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 mul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ float sqr_len(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ float length(V3 a) { return sqrtf(sqr_len(a)); }
__device__ __forceinline__ V3 normalize(V3 a) {  // vector.h:60-64
  float l = sqrtf(sqr_len(a));
  return v3(a.x / l, a.y / l, a.z / l);
}
__device__ __forceinline__ V3 div_guarded(V3 a, float s) {  // vector.cpp:36-41
  if (cmpf(s) == 0) return v3(WR_INF, WR_INF, WR_INF);
  return v3(a.x / s, a.y / s, a.z / s);
}
__device__ __forceinline__ bool near_eq(V3 a, V3 b) {  // vector.cpp:43-47
  return cmpf(a.x - b.x) == 0 && cmpf(a.y - b.y) == 0 && cmpf(a.z - b.z) == 0;
}
__device__ __forceinline__ bool black(V3 c) { return cmpf(c.x) == 0 && cmpf(c.y) == 0 && cmpf(c.z) == 0; }
__device__ __forceinline__ float luminance(V3 c) { return 0.2126f * c.x + 0.7152f * c.y + 0.0722f * c.z; }
__device__ __forceinline__ V3 div_plain(V3 c, float s) { return v3(c.x / s, c.y / s, c.z / s); }  // Color3 /

// ------------------------------------------------------------ counter RNG
// Stream key = mix(seed, iteration, subpath, path); draw j = hi32(mix(key + (j+1)*phi)).
// Identical to cr_stream_key / cr_stream_u32 of the oracle.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t stream_key(uint32_t seed, uint32_t iter, uint32_t sub, uint32_t path) {
  uint64_t a = mix64((static_cast<uint64_t>(seed) << 32) | iter);
  uint64_t b = mix64(((static_cast<uint64_t>(sub) << 32) | path) + 0x9E3779B97F4A7C15ull);
  return mix64(a ^ b);
}
struct Rng {
  uint64_t key;
  uint32_t ctr;
  __device__ __forceinline__ uint32_t u32() {
    return static_cast<uint32_t>(mix64(key + static_cast<uint64_t>(++ctr) * 0x9E3779B97F4A7C15ull) >> 32);
  }
  // rng.cpp:18-22
  __device__ __forceinline__ float f() { return static_cast<float>(u32() & 0xffffffu) / 16777216.0f; }
  __device__ __forceinline__ V3 v() {
    float a = f();
    float b = f();
    float c = f();
    return v3(a, b, c);
  }
};

// ------------------------------------------------------------ frames, samplers
struct Frame {
  V3 x, y, z;
};
__device__ __forceinline__ Frame frame_from_z(V3 z0) {  // frame.cpp:3-11
  Frame f;
  f.z = normalize(z0);
  V3 tx = (fabsf(f.z.x) > 0.99f) ? v3(0.f, 1.f, 0.f) : v3(1.f, 0.f, 0.f);
  f.y = normalize(cross(f.z, tx));
  f.x = cross(f.y, f.z);
  return f;
}
__device__ __forceinline__ V3 to_world(const Frame& f, V3 l) {
  return f.x * l.x + f.y * l.y + f.z * l.z;
}
__device__ __forceinline__ V3 to_local(const Frame& f, V3 w) { return v3(dot(w, f.x), dot(w, f.y), dot(w, f.z)); }

__device__ __forceinline__ V3 sample_triangle(V3 s, V3 a, V3 b, V3 c) {  // sampler.cpp:3-13
  V3 p1 = b - a, p2 = c - a;
  float u1 = sqrtf(s.x);
  float beta = 1.f - u1;
  float gamma = s.y * u1;
  return a + p1 * beta + p2 * gamma;
}
__device__ __forceinline__ V3 sample_rect_strat(V3 s, V3 v0, V3 v1, V3 v2, int cur, int len) {
  V3 p1 = v1 - v0, p2 = v2 - v0;  // sampler.cpp:28-42 (len = (int)sqrt(tot) given)
  int row = cur / len, col = cur % len;
  float a = (s.x + static_cast<float>(row)) / static_cast<float>(len);
  float b = (s.y + static_cast<float>(col)) / static_cast<float>(len);
  return v0 + p1 * a + p2 * b;
}
__device__ __forceinline__ V3 sample_cos_hemi(V3 s, float* pdf) {  // sampler.cpp:95-108
  float u1 = 2.f * WR_PI * s.x;
  float u2 = sqrtf(1.f - s.y);
  float sn, cs;
  wr_sincosf(u1, &sn, &cs);  // == glibc sinf(u1), cosf(u1)
  V3 r = v3(cs * u2, sn * u2, sqrtf(s.y));
  *pdf = r.z * WR_INV_PI;
  return normalize(r);
}
__device__ __forceinline__ V3 sample_pow_cos_hemi(V3 s, float power) {  // sampler.cpp:115-129
  float u1 = 2.f * WR_PI * s.x;
  float u2 = wr_powf(s.y, 1.f / (power + 1.f));
  float u3 = sqrtf(1.f - u2 * u2);
  float sn, cs;
  wr_sincosf(u1, &sn, &cs);
  return normalize(v3(cs * u3, sn * u3, u2));
}
__device__ __forceinline__ float pow_cos_pdf(V3 n, V3 d, float power) {  // sampler.cpp:131-136
  float c = clampv(dot(n, d), 0.f, 1.f);
  return (power + 1.f) * wr_powf(c, power) * (0.5f * WR_INV_PI);
}

// ------------------------------------------------------------ scene records
struct DLight {  // AreaLight (light.h:82-129)
  V3 p0, d1, d2, fx, fy, fz, le;
  float inv_area;
};
struct DMat {  // Material (material.h:7-31)
  V3 diffuse, phong, specular;
  float phong_exp, index;
};
struct DCam {
  V3 pos, fwd;
  float xres, yres, plane_dist;
  float w2r[16], r2w[16];
};

__device__ __forceinline__ V3 t_point(const float* m, V3 p) {  // transform.h:122-137
  float xp = m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3];
  float yp = m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7];
  float zp = m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11];
  float wp = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
  if (cmpf(wp - 1.0f) == 0) return v3(xp, yp, zp);
  return div_guarded(v3(xp, yp, zp), wp);
}
__device__ __forceinline__ bool check_raster(const DCam& c, float x, float y) {  // camera.cpp:31-35
  return cmpf(x) >= 0 && cmpf(y) >= 0 && cmpf(x - c.xres) < 0 && cmpf(y - c.yres) < 0;
}

// ------------------------------------------------------------ AreaLight
__device__ __forceinline__ V3 light_illuminance(const DLight& l, V3 pos, V3 r3, V3* dtl, float* dist,
                                                float* dpdf, float* epdf, float* cal) {  // light.cpp:4-38
  *epdf = 0;
  *cal = 0;
  V3 lp = sample_triangle(r3, l.p0, l.p0 + l.d1, l.p0 + l.d2);
  V3 d = lp - pos;
  *dist = length(d);
  d = div_guarded(d, *dist);
  *dtl = d;
  float cn = dot(l.fz, -d);
  if (cmpf(cn) <= 0) {
    *dpdf = 0;
    *epdf = 0;
    return v3(0.f, 0.f, 0.f);
  }
  *dpdf = l.inv_area * ((*dist) * (*dist)) / cn;
  *cal = cn;
  *epdf = l.inv_area * cn * WR_INV_PI;
  return l.le;
}
__device__ __forceinline__ V3 light_emit(const DLight& l, V3 dr, V3 pr, V3* pos, V3* dir, float* epdf,
                                         float* dpa, float* cal = nullptr) {  // light.cpp:40-67
  *pos = sample_triangle(pr, l.p0, l.p0 + l.d1, l.p0 + l.d2);
  V3 ld = sample_cos_hemi(dr, epdf);
  *epdf *= l.inv_area;
  ld.z = smax(ld.z, WR_EPS);
  Frame f{l.fx, l.fy, l.fz};
  *dir = to_world(f, ld);
  *dpa = l.inv_area;
  if (cal) *cal = ld.z;
  return l.le * ld.z;
}
__device__ __forceinline__ V3 light_radiance(const DLight& l, V3 rd, float* dpa, float* epdf) {  // light.cpp:69-100
  *dpa = 0;
  *epdf = 0;
  float cn = clampv(dot(l.fz, -rd), 0.f, 1.f);
  if (cmpf(cn) == 0) return v3(0.f, 0.f, 0.f);
  *dpa = l.inv_area;
  *epdf = clampv(dot(l.fz, -rd), 0.f, 1.f) * WR_INV_PI;
  *epdf *= l.inv_area;
  return l.le;
}

// ------------------------------------------------------------ BSDF
enum { T_REFL = 1, T_TRANS = 2, T_DIFF = 4, T_GLOSSY = 8, T_SPEC = 3 };

__device__ __forceinline__ float fresnel(float cos_i, float index) {  // fresnel.cpp:3-29
  if (cmpf(index) < 0) return 1.0f;
  float eta;
  if (cmpf(cos_i) < 0) {
    cos_i = -cos_i;
    eta = index;
  } else {
    eta = 1.0f / index;
  }
  float sin_t2 = (eta * eta) * (1.0f - cos_i * cos_i);
  float cos_t = sqrtf(smax(0.0f, 1.0f - sin_t2));
  float term1 = eta * cos_t;
  float par = (cos_i - term1) / (cos_i + term1);
  float term2 = eta * cos_i;
  float perp = (term2 - cos_t) / (term2 + cos_t);
  return 0.5f * (par * par + perp * perp);
}

struct Bsdf {
  int mat;     // 0 = invalid
  Frame fr;
  V3 wi;       // wiLocal
  bool delta;
  float cont, fres, pd, pg, pr, pt;
};

// BSDF::init (bsdf.h:66-89).  Emitter hits (mat < 0) get the pinned values of
// the oracle: probabilities 0, continueProb 0, isDelta false.
// The component / continuation probabilities of BSDF::init from the local
// wi and the material (the tail of bsdf_init; also how a stored vertex's
// BSDF is rebuilt, wr_bdpt.h stored_bsdf).
__device__ __forceinline__ void bsdf_probs(Bsdf& b, int hit_mat, const DMat* mats) {
  b.pd = b.pg = b.pr = b.pt = 0.f;
  b.cont = 0.f;
  b.fres = 1.f;
  b.delta = false;
  if (hit_mat > 0) {  // bsdf.cpp:24-55
    const DMat m = mats[hit_mat];
    b.fres = fresnel(b.wi.z, m.index);
    float pd = luminance(m.diffuse);
    float pg = luminance(m.phong);
    float pr = b.fres * luminance(m.specular);
    float pt = (1.f - b.fres) * 1.0f;
    float tot = pd + pg + pr + pt;
    if (cmpf(tot) > 0) {
      b.pd = pd / tot;
      b.pg = pg / tot;
      b.pr = pr / tot;
      b.pt = pt / tot;
      V3 refl = m.diffuse + m.phong + m.specular * b.fres;
      b.cont = smax(refl.x, smax(refl.y, refl.z)) + (1.f - b.fres);
      b.cont = clampv(b.cont, 0.f, 1.f);
    }
    b.delta = (cmpf(b.pd) == 0 && cmpf(b.pg) == 0);
  }
  b.mat = hit_mat;
}
__device__ __forceinline__ void bsdf_init(Bsdf& b, V3 wi, V3 n, int hit_mat, const DMat* mats) {
  b.mat = 0;
  b.fr = frame_from_z(n);
  b.wi = normalize(to_local(b.fr, wi));
  if (cmpf(b.wi.z) == 0) return;
  bsdf_probs(b, hit_mat, mats);
}

__device__ __forceinline__ V3 calc_diffuse(const Bsdf& b, const DMat& m, V3 wo, float* dp, float* rp) {
  if (cmpf(b.pd) == 0) return v3(0.f, 0.f, 0.f);  // bsdf.cpp:57-72
  if (cmpf(b.wi.z) <= 0 || cmpf(wo.z) <= 0) return v3(0.f, 0.f, 0.f);
  if (dp) *dp += b.pd * clampv(wo.z * WR_INV_PI, 0.0f, 1.0f);
  if (rp) *rp += b.pd * clampv(b.wi.z * WR_INV_PI, 0.0f, 1.0f);
  return m.diffuse * WR_INV_PI;
}
__device__ __forceinline__ V3 glossy_rho(const DMat& m, float c) {
  V3 rho = m.phong * (m.phong_exp + 2.f) * 0.5f * WR_INV_PI;
  return rho * wr_powf(c, m.phong_exp);
}
__device__ __forceinline__ V3 calc_glossy(const Bsdf& b, const DMat& m, V3 wo, float* dp, float* rp) {
  if (cmpf(b.pg) == 0) return v3(0.f, 0.f, 0.f);  // bsdf.cpp:74-100
  if (cmpf(b.wi.z) <= 0 || cmpf(wo.z) <= 0) return v3(0.f, 0.f, 0.f);
  V3 refl = v3(-b.wi.x, -b.wi.y, b.wi.z);
  float c = dot(refl, wo);
  if (cmpf(c) == 0) return v3(0.f, 0.f, 0.f);
  float pw = b.pg * pow_cos_pdf(refl, wo, m.phong_exp);
  if (dp) *dp += pw;
  if (rp) *rp += pw;
  return glossy_rho(m, c);
}
// BSDF::f (bsdf.cpp:102-126); dp / rp are always written (0 first)
__device__ __forceinline__ V3 bsdf_f(const Bsdf& b, const DMat* mats, V3 wo_w, float* cos_wo, float* dp,
                                     float* rp) {
  V3 res = v3(0.f, 0.f, 0.f);
  if (dp) *dp = 0.f;
  if (rp) *rp = 0.f;
  V3 wo = to_local(b.fr, wo_w);
  if (cmpf(wo.z * b.wi.z) < 0) return res;
  *cos_wo = fabsf(wo.z);
  if (b.mat < 0) return res;
  const DMat m = mats[b.mat];
  res = res + calc_diffuse(b, m, wo, dp, rp);
  res = res + calc_glossy(b, m, wo, dp, rp);
  return res;
}
__device__ __forceinline__ void pdf_glossy(const Bsdf& b, const DMat& m, V3 wo, float* dp, float* rp) {
  if (cmpf(b.pg) == 0) return;  // bsdf.cpp:143-163
  V3 refl = v3(-b.wi.x, -b.wi.y, b.wi.z);
  float c = dot(refl, wo);
  if (cmpf(c) == 0) return;
  float pw = b.pg * pow_cos_pdf(refl, wo, m.phong_exp);
  if (dp) *dp += pw;
  if (rp) *rp += pw;
}
// BSDF::pdf (bsdf.cpp:165-181)
__device__ __forceinline__ float bsdf_pdf(const Bsdf& b, const DMat* mats, V3 wo_w, bool rev) {
  V3 wo = to_local(b.fr, wo_w);
  if (cmpf(wo.z * b.wi.z) < 0) return 0;
  const DMat m = mats[b.mat];
  float dp = 0, rp = 0;
  if (cmpf(b.pd) != 0) {  // pdfDiffuse (bsdf.cpp:128-141)
    dp += b.pd * clampv(wo.z, 0.f, 1.f) * WR_INV_PI;
    rp += b.pd * clampv(b.wi.z, 0.f, 1.f) * WR_INV_PI;
  }
  pdf_glossy(b, m, wo, &dp, &rp);
  return rev ? rp : dp;
}
// BSDF::sample (bsdf.cpp:183-334)
__device__ __forceinline__ V3 bsdf_sample(const Bsdf& b, const DMat* mats, V3 r3, V3* wo_w, float* pdf,
                                          float* cos_wo, int* type) {
  const V3 zero = v3(0.f, 0.f, 0.f);
  int comp;
  if (r3.z < b.pd) comp = T_DIFF;
  else if (r3.z < b.pd + b.pg) comp = T_GLOSSY;
  else if (r3.z < b.pd + b.pg + b.pr) comp = T_REFL;
  else comp = T_TRANS;
  *type = comp;
  if (b.mat < 0) return zero;
  const DMat m = mats[b.mat];
  *pdf = 0;
  V3 res = zero;
  V3 wo = zero;
  if (comp == T_DIFF) {
    if (cmpf(b.wi.z) <= 0) return zero;
    float pw;
    wo = sample_cos_hemi(r3, &pw);
    *pdf += pw * b.pd;
    res = res + m.diffuse * WR_INV_PI;
    if (black(res)) return zero;
    res = res + calc_glossy(b, m, wo, pdf, nullptr);
  } else if (comp == T_GLOSSY) {
    wo = sample_pow_cos_hemi(r3, m.phong_exp);
    V3 refl = v3(-b.wi.x, -b.wi.y, b.wi.z);
    Frame f = frame_from_z(refl);
    wo = to_world(f, wo);
    float c = dot(refl, wo);
    V3 g = zero;
    if (cmpf(c) > 0) {
      pdf_glossy(b, m, wo, pdf, nullptr);
      g = glossy_rho(m, c);
    }
    res = res + g;
    if (black(res)) return zero;
    res = res + calc_diffuse(b, m, wo, pdf, nullptr);
  } else if (comp == T_REFL) {
    wo = v3(-b.wi.x, -b.wi.y, b.wi.z);
    *pdf += b.pr;
    res = res + div_plain(m.specular * b.fres, fabsf(wo.z));
    if (black(res)) return zero;
  } else {
    V3 t = zero;
    if (!(cmpf(m.index) < 0)) {
      float cos_i = b.wi.z, cos_t, eta;
      if (cmpf(cos_i) < 0) {
        eta = m.index;
        cos_i = -cos_i;
        cos_t = 1.f;
      } else {
        eta = 1.f / m.index;
        cos_t = -1.f;
      }
      float sin_i2 = 1.f - cos_i * cos_i;
      float sin_t2 = (eta * eta) * sin_i2;
      if (sin_t2 < 1.f) {
        cos_t *= sqrtf(clampv(1.f - sin_t2, 0.f, 1.f));
        wo = normalize(v3(-eta * b.wi.x, -eta * b.wi.y, cos_t));
        *pdf += b.pt;
        float v = (1.f - b.fres) / fabsf(cos_t);
        t = v3(v, v, v);
      }
    }
    res = res + t;
    if (black(res)) return zero;
  }
  *cos_wo = fabsf(wo.z);
  if (cmpf(*cos_wo) == 0) return zero;
  *wo_w = to_world(b.fr, wo);
  return res;
}

}  // namespace wrd
