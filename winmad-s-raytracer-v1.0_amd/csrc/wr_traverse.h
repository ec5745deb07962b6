// KD-tree closest-hit traversal on gfx950 -- KDtreeAccel::traverse
// (src/scene/KDtreeAccel.cpp:309-388) + Triangle::hit (src/geometry/triangle.cpp:22-87)
// + Sphere::hit (src/geometry/sphere.cpp:17-78).
//
// Layout in HBM (built by wr_device.cpp from wr::Scene):
//   nodes  uint2 per node, pre-order (left child = node + 1):
//            inner: x = split (float bits), y = right << 2 | axis (0..2)
//            leaf : x = first ref,          y = count << 2 | 3
//   refs   leaf primitive references, in the reference's objlist order, with the
//          triangle inlined so a test is one 40-byte gather:
//            ref_a = (p0.x, p0.y, p0.z, A)  ref_b = (B, C, D, E)  ref_c = (F, prim)
//          where A..F = p0 - p1, p0 - p2 exactly as Triangle::hit forms them.
//          Spheres: ref_c.y = -(prim + 1); geometry read from prim_sph.
//   stack  LDS, [depth][blockDim] columns of (node, tmin, tmax): one column per
//          lane, so a wave's push / pop hits 64 consecutive banks.
//
// Semantics kept from the reference: root-box clip, the belowFirst near/far rule,
// NO early exit (every leaf the ray crosses is visited), closest hit with the
// EPS tie rule `cmp(t - best) < 0` in leaf order (first-found wins).
#pragma once
#include "wr_devmath.h"

namespace wrd {

struct DevScene {
  const uint2* nodes;
  const float4* ref_a;
  const float4* ref_b;
  const float2* ref_c;
  const int* prim_mat;
  const int* prim_type;     // 0 triangle, 1 sphere
  const float4* prim_tri;   // (A, B, C, D) per primitive (winner normal)
  const float2* prim_tri2;  // (E, F)
  const float4* prim_sph;   // (cx, cy, cz, r)
  const float4* prim_sbox0; // (lx, ly, lz, rx) AABB after extend()
  const float2* prim_sbox1; // (ry, rz)
  V3 root_l, root_r;
  int max_stack;
  int nlights;
  const DLight* lights;
  const DMat* mats;
  DCam cam;
};

struct TraceCounters {  // algorithmic work, for the roofline's byte count
  uint32_t inner, leaves, refs;
};

// AABB::hit (AABB.cpp:9-32)
__device__ __forceinline__ bool box_hit(V3 l, V3 r, V3 o, V3 d, float& t1, float& t2) {
  float tmin = -WR_INF, tmax = WR_INF;
  const float lo[3] = {l.x, l.y, l.z}, hi[3] = {r.x, r.y, r.z}, oo[3] = {o.x, o.y, o.z},
              dd[3] = {d.x, d.y, d.z};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    float inv = 1.f / dd[i];
    float tn = (lo[i] - oo[i]) * inv;
    float tf = (hi[i] - oo[i]) * inv;
    if (tn > tf) {
      float t = tn;
      tn = tf;
      tf = t;
    }
    tmin = smax(tmin, tn);
    tmax = smin(tmax, tf);
    if (tmin > tmax) return false;
  }
  t1 = tmin;
  t2 = tmax;
  return true;
}

// Triangle::hit, returning t (or a value > every accepted t on rejection).
// The three quotients are the reference's correctly rounded divisions; the beta
// quotient is first screened with v_rcp_f32: a ray whose approximate beta lies
// clearly outside [-EPS, 1] (margin 1e-5 relative, far above the rcp error)
// would be rejected by the exact test too, so the screen never changes a result.
__device__ __forceinline__ bool tri_hit(float4 a, float4 b, float f, V3 o, V3 d, float rtmin, float rtmax,
                                        float& t_out) {
  const float A = a.w, B = b.x, C = b.y, D = b.z, E = b.w, F = f;
  const float G = d.x, H = d.y, I = d.z;
  const float J = a.x - o.x, K = a.y - o.y, L = a.z - o.z;
  const float EIHF = E * I - H * F;
  const float GFDI = G * F - D * I;
  const float DHEG = D * H - E * G;
  const float denom = A * EIHF + B * GFDI + C * DHEG;
  const float bnum = J * EIHF + K * GFDI + L * DHEG;
  const float ad = fabsf(denom);
  if (ad > 1e-30f && ad < 1e30f) {
    const float ba = bnum * __builtin_amdgcn_rcpf(denom);
    const float m = 1e-5f * fabsf(ba);
    if (ba < -WR_EPS - m || ba > 1.f + m) return false;
  }
  const float beta = bnum / denom;
  if (cmpf(beta) < 0 || beta > 1.f) return false;
  const float AKJB = A * K - J * B;
  const float JCAL = J * C - A * L;
  const float BLKC = B * L - K * C;
  const float gamma = (I * AKJB + H * JCAL + G * BLKC) / denom;
  if (cmpf(gamma) < 0 || beta + gamma > 1.f) return false;
  const float t = -(F * AKJB + E * JCAL + D * BLKC) / denom;
  if (cmpf(t) <= 0) return false;
  if (t < rtmin || t > rtmax) return false;
  t_out = t;
  return true;
}

// Sphere::hit (sphere.cpp:17-78): only t and the accept decision
__device__ __forceinline__ bool sph_hit(const DevScene& S, int prim, V3 o, V3 d, float rtmin, float rtmax,
                                        float& t_out, int* inside_out = nullptr) {
  float4 sb0 = S.prim_sbox0[prim];
  float2 sb1 = S.prim_sbox1[prim];
  float t1, t2;
  if (!box_hit(v3(sb0.x, sb0.y, sb0.z), v3(sb0.w, sb1.x, sb1.y), o, d, t1, t2)) return false;
  float4 cs = S.prim_sph[prim];
  V3 c = v3(cs.x, cs.y, cs.z);
  float rad = cs.w;
  V3 oc = c - o;
  bool inside = length(oc) < rad + WR_EPS;
  float l_oc = dot(oc, oc);
  float t_ca = dot(oc, d);
  if (cmpf(t_ca) < 0 && !inside) return false;
  float t_hc = rad * rad - l_oc + t_ca * t_ca;
  if (cmpf(t_hc) <= 0) return false;
  float dd = sqrtf(t_hc);
  float ta = t_ca - dd, tb = t_ca + dd;
  if (cmpf(tb) <= 0) return false;
  float t;
  int in;
  if (cmpf(ta) <= 0) {
    t = tb;
    in = 1;
  } else {
    t = ta;
    in = 0;
  }
  if (t < rtmin || t > rtmax) return false;
  t_out = t;
  if (inside_out) *inside_out = in;
  return true;
}

// Closest hit.  `stk_*` point at this lane's LDS column (stride = blockDim).
template <bool COUNT>
__device__ __forceinline__ int traverse(const DevScene& S, V3 o, V3 d, float rtmin, float rtmax, float& t_best,
                                        uint32_t* stk_node, float* stk_tmin, float* stk_tmax, int stride,
                                        TraceCounters& ctr) {
  t_best = WR_INF;
  float tmin, tmax;
  if (!box_hit(S.root_l, S.root_r, o, d, tmin, tmax)) return -1;
  const V3 inv = v3(1.f / d.x, 1.f / d.y, 1.f / d.z);
  int sp = 0;
  int best = -1;
  uint32_t node = 0;
  for (;;) {
    if (rtmax < tmin) break;
    const uint2 nd = S.nodes[node];
    const uint32_t axis = nd.y & 3u;
    if (axis != 3u) {
      if (COUNT) ++ctr.inner;
      const float split = __uint_as_float(nd.x);
      const float oa = axis == 0 ? o.x : (axis == 1 ? o.y : o.z);
      const float da = axis == 0 ? d.x : (axis == 1 ? d.y : d.z);
      const float ia = axis == 0 ? inv.x : (axis == 1 ? inv.y : inv.z);
      const float t = (split - oa) * ia;
      const bool below = (oa < split) || (oa == split && da <= 0);
      const uint32_t left = node + 1, right = nd.y >> 2;
      const uint32_t nearc = below ? left : right, farc = below ? right : left;
      if (t > tmax || t <= 0) {
        node = nearc;
      } else if (t < tmin) {
        node = farc;
      } else {
        stk_node[sp * stride] = farc;
        stk_tmin[sp * stride] = t;
        stk_tmax[sp * stride] = tmax;
        ++sp;
        node = nearc;
        tmax = t;
      }
    } else {
      const uint32_t first = nd.x, count = nd.y >> 2;
      if (COUNT) {
        ++ctr.leaves;
        ctr.refs += count;
      }
      for (uint32_t i = 0; i < count; ++i) {
        const float2 c = S.ref_c[first + i];
        const int prim = __float_as_int(c.y);
        float t;
        bool h;
        if (prim >= 0) {
          h = tri_hit(S.ref_a[first + i], S.ref_b[first + i], c.x, o, d, rtmin, rtmax, t);
        } else {
          h = sph_hit(S, -prim - 1, o, d, rtmin, rtmax, t);
        }
        if (h && cmpf(t - t_best) < 0) {
          t_best = t;
          best = prim >= 0 ? prim : -prim - 1;
        }
      }
      if (sp > 0) {
        --sp;
        node = stk_node[sp * stride];
        tmin = stk_tmin[sp * stride];
        tmax = stk_tmax[sp * stride];
      } else {
        break;
      }
    }
  }
  return best;
}

// Scene::intersect re-runs hit() on the winner (scene.cpp:25-27); from (t, prim)
// the intersection record is rebuilt with the same float operations.
struct Hit {
  float t;
  V3 p, n;
  int inside, mat;
};
__device__ __forceinline__ Hit rebuild_hit(const DevScene& S, int prim, float t, V3 o, V3 d) {
  Hit h;
  h.t = t;
  h.p = o + d * t;
  h.mat = S.prim_mat[prim];
  if (S.prim_type[prim] != 0) {
    float4 cs = S.prim_sph[prim];
    h.n = normalize(h.p - v3(cs.x, cs.y, cs.z));
    float tt;
    int in = 0;
    sph_hit(S, prim, o, d, 0.f, WR_INF, tt, &in);
    h.inside = in;
  } else {
    float4 g = S.prim_tri[prim];
    float2 g2 = S.prim_tri2[prim];
    // (p1 - p0) x (p2 - p0) == (p0 - p1) x (p0 - p2) exactly
    h.n = normalize(cross(v3(g.x, g.y, g.z), v3(g.w, g2.x, g2.y)));
    h.inside = (dot(d, h.n) < WR_EPS) ? 0 : 1;
  }
  return h;
}

}  // namespace wrd
