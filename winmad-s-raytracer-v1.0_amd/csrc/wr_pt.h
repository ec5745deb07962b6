// PathIntegrator::raytracing (pathIntegrator.cpp:29-148) + the stratified
// SurfaceIntegrator::render (surfaceIntegrator.cpp:14-46) as wavefront
// kernels: gen -> [trace -> resolve + shade] x (depth + 1).  Included by
// wr_render.hip inside its anonymous namespace.
#pragma once

// =============================================================== PT
// PT path state, one 32-byte record per path (the vertex kernel gathers it by
// path index): path weight, last BSDF pdf / specular flag, length, pixel, RNG counter
enum : int { PT_PW = 0, PT_LPDF = 3, PT_LSPEC = 4, PT_LEN = 5, PT_PIX = 6, PT_CTR = 7, PT_WORDS = 8 };
__device__ __forceinline__ float& ptf(float* s, int p, int k) { return s[size_t(p) * PT_WORDS + k]; }
__device__ __forceinline__ int& pti(float* s, int p, int k) {
  return reinterpret_cast<int*>(s)[size_t(p) * PT_WORDS + k];
}
__device__ __forceinline__ uint32_t& ptu(float* s, int p, int k) {
  return reinterpret_cast<uint32_t*>(s)[size_t(p) * PT_WORDS + k];
}
__device__ __forceinline__ V3 pld3(const float* s, int p, int k) {
  const float* r = s + size_t(p) * PT_WORDS + k;
  return v3(r[0], r[1], r[2]);
}
__device__ __forceinline__ void pst3(float* s, int p, int k, V3 v) {
  float* r = s + size_t(p) * PT_WORDS + k;
  r[0] = v.x;
  r[1] = v.y;
  r[2] = v.z;
}
struct PtBuf {
  int P = 0;
  float* st;  // PT_WORDS floats per path
  float *q_o[2], *q_d[2], *q_t[2];
  int *q_path[2], *q_prim[2];
  // NEE shadow rays, two buffers: those of step `slot` are [slot & 1], so a
  // step's resolve and the next vertex shading (writing [(slot + 1) & 1]) run
  // in one launch
  struct Sq {
    float *o, *d, *tgt, *val, *t, *cut;  // cut: occl_cut
    int *pix, *prim;
  } sq[2];
};
struct PtArgs {
  DevScene S;
  PtBuf T;
  DevCounters* ctr;
  StepCounters* sc;  // this sample's queue counters
  float* film;
  int W, H, P, spp, grid_len, max_depth;
  uint32_t seed, k;
};
struct PtGroup {
  PtArgs a[kGroup];
};

// SurfaceIntegrator::render per-sample setup (surfaceIntegrator.cpp:26-34)
__global__ void __launch_bounds__(kShadeBlock) WR_NO_PK_FP32 k_pt_gen(PtGroup G_) {
  const PtArgs& A = G_.a[blockIdx.y];
  const PtBuf& T = A.T;
  const DCam& cam = A.S.cam;
  const int P = A.P;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < P; p += gridDim.x * blockDim.x) {
    const int i = p / A.W, jj = p % A.W;
    Rng rng{stream_key(A.seed, A.k, 2, static_cast<uint32_t>(p)), 0};
    const V3 v0 = v3(static_cast<float>(jj) - 0.5f, static_cast<float>(i) - 0.5f, 0.f);
    const V3 v1 = v3(static_cast<float>(jj) + 0.5f, static_cast<float>(i) - 0.5f, 0.f);
    const V3 v2 = v3(static_cast<float>(jj) - 0.5f, static_cast<float>(i) + 0.5f, 0.f);
    const V3 pr = sample_rect_strat(rng.v(), v0, v1, v2, static_cast<int>(A.k), A.grid_len);
    const V3 wp = t_point(cam.r2w, v3(pr.x, pr.y, 0.f));
    const V3 d = normalize(wp - cam.pos);
    pst3(T.st, p, PT_PW, v3(1.f, 1.f, 1.f));
    ptf(T.st, p, PT_LPDF) = 1.f;
    pti(T.st, p, PT_LSPEC) = 1;
    pti(T.st, p, PT_LEN) = 1;
    pti(T.st, p, PT_PIX) = i * A.W + jj;
    ptu(T.st, p, PT_CTR) = rng.ctr;
    st3(T.q_o[0], P, p, cam.pos);  // Ray r(ray): no EPS offset for the primary ray
    st3(T.q_d[0], P, p, d);
    T.q_path[0][p] = p;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) A.sc->ext[0] = P;
}

// PathIntegrator::raytracing(ray, dep) for caller rays (wr_path_radiance): the
// path starts from the Ray object as given (o, d; no EPS offset, like the
// camera ray of k_pt_gen); output p is "pixel" p of an n x 1 film.
__global__ void __launch_bounds__(kShadeBlock) WR_NO_PK_FP32 k_pt_gen_rays(PtGroup G_, const wr_ray* rays) {
  const PtArgs& A = G_.a[blockIdx.y];
  const PtBuf& T = A.T;
  const int P = A.P;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < P; p += gridDim.x * blockDim.x) {
    const wr_ray r = rays[p];
    const V3 o = v3(r.o[0], r.o[1], r.o[2]), d = v3(r.d[0], r.d[1], r.d[2]);
    pst3(T.st, p, PT_PW, v3(1.f, 1.f, 1.f));
    ptf(T.st, p, PT_LPDF) = 1.f;
    pti(T.st, p, PT_LSPEC) = 1;
    pti(T.st, p, PT_LEN) = 1;
    pti(T.st, p, PT_PIX) = p;
    ptu(T.st, p, PT_CTR) = 0;
    st3(T.q_o[0], P, p, o);
    st3(T.q_d[0], P, p, d);
    T.q_path[0][p] = p;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) A.sc->ext[0] = P;
}

// One PathIntegrator::raytracing iteration (pathIntegrator.cpp:43-146)
__device__ __forceinline__ void pt_shade_body(const PtArgs& A, int slot, int bid, int nblk) {
  const PtBuf& T = A.T;
  const DevScene& S = A.S;
  const int P = A.P, cur = slot & 1, nxt = cur ^ 1;
  const int n = A.sc->ext[slot];
  if (bid == 0 && threadIdx.x == 0) atomicAdd(&A.ctr->closest, (unsigned long long)n);
  const int gstride = nblk * blockDim.x;
  const int nround = (n + gstride - 1) / gstride * gstride;
  const float lpp = 1.f / static_cast<float>(S.nlights);
  for (int j = bid * blockDim.x + threadIdx.x; j < nround; j += gstride) {
    bool ext = false, shadow = false;
    int p = -1, pix = -1;
    V3 e_o{}, e_d{}, s_o{}, s_d{}, s_tgt{}, s_val{};
    if (j < n) {
      p = T.q_path[cur][j];
      const int prim = T.q_prim[cur][j];
      if (prim >= 0) {
        const float t = T.q_t[cur][j];
        const V3 o = ld3(T.q_o[cur], P, j), d = ld3(T.q_d[cur], P, j);
        const Hit h = rebuild_hit(S, prim, t, o, d);
        Bsdf b;
        bsdf_init(b, -d, h.n, h.mat, S.mats);
        pix = pti(T.st, p, PT_PIX);
        if (b.mat != 0) {
          V3 pw = pld3(T.st, p, PT_PW);
          const int len = pti(T.st, p, PT_LEN);
          if (b.mat < 0) {  // (:53-73)
            const DLight L = S.lights[-b.mat - 1];
            float dpa, ep;
            const V3 c = light_radiance(L, d, &dpa, &ep);
            if (!black(c)) {
              float mw = 1.f;
              if (len > 1 && !pti(T.st, p, PT_LSPEC)) {
                const float dp = dpa * (t * t) / fabsf(b.wi.z);  // pdfAtoW
                const float lp = ptf(T.st, p, PT_LPDF);
                mw = lp / (lp + dp * lpp);
              }
              film_add(A.film, pix, mul(pw, c) * mw);
            }
          } else if (!(len > A.max_depth) && cmpf(b.cont) != 0) {
            Rng rng{stream_key(A.seed, A.k, 2, static_cast<uint32_t>(p)), ptu(T.st, p, PT_CTR)};
            if (!b.delta) {  // (:81-118)
              const int lid = min(static_cast<int>(rng.f() * static_cast<float>(S.nlights)), S.nlights - 1);
              const DLight L = S.lights[lid];
              V3 dtl;
              float dist = 0.f, dpdf = 0.f, ep, cal;
              const V3 illu = light_illuminance(L, h.p, rng.v(), &dtl, &dist, &dpdf, &ep, &cal);
              if (!black(illu)) {
                shadow = true;
                s_o = h.p + dtl * WR_EPS;
                s_d = normalize(dtl);
                s_tgt = h.p + dtl * (dist - WR_EPS);
                float bp, cw = 0.f;
                const V3 bf = bsdf_f(b, S.mats, dtl, &cw, &bp, nullptr);
                s_val = v3(0.f, 0.f, 0.f);
                if (!black(bf)) {
                  bp *= b.cont;
                  const float w = (dpdf * lpp) / ((dpdf * lpp) + bp);
                  const V3 c = mul(illu, bf) * (w * cw / (lpp * dpdf));
                  s_val = mul(c, pw);
                }
              }
            }
            float pdf = 0.f, cw = 0.f;
            int type;
            V3 dn = d;
            const V3 bf = bsdf_sample(b, S.mats, rng.v(), &dn, &pdf, &cw, &type);
            if (!black(bf)) {  // (:124-145)
              const float cp = b.cont;
              const int lspec = (type & T_SPEC) != 0;
              const float lpdf = pdf * cp;
              bool cont = true;
              if (cmpf(cp - 1.f) < 0) {
                if (cmpf(rng.f() - cp) > 0) cont = false;
                else pdf *= cp;
              }
              if (cont) {
                pw = mul(pw, bf) * (cw / pdf);
                ext = true;
                e_o = h.p + dn * WR_EPS;
                e_d = dn;  // r.dir stays un-normalised (:144-145)
                pst3(T.st, p, PT_PW, pw);
                pti(T.st, p, PT_LSPEC) = lspec;
                ptf(T.st, p, PT_LPDF) = lpdf;
                pti(T.st, p, PT_LEN) = len + 1;
              }
            }
            ptu(T.st, p, PT_CTR) = rng.ctr;
          }
        }
      }
    }
    const int ei = wave_append(&A.sc->ext[slot + 1], ext);
    if (ext) {
      st3(T.q_o[nxt], P, ei, e_o);
      st3(T.q_d[nxt], P, ei, e_d);
      T.q_path[nxt][ei] = p;
    }
    const int si = wave_append(&A.sc->sq[slot + 1], shadow);
    if (shadow) {
      const PtBuf::Sq& Q = T.sq[(slot + 1) & 1];
      st3(Q.o, P, si, s_o);
      st3(Q.d, P, si, s_d);
      st3(Q.tgt, P, si, s_tgt);
      st3(Q.val, P, si, s_val);
      Q.cut[si] = occl_cut(s_o, s_tgt, dot(s_tgt - s_o, s_d));
      Q.pix[si] = pix;
    }
  }
}

// NEE shadow rays of step `slot` after traversal (pathIntegrator.cpp:95-110):
// unoccluded => the queued contribution goes to the film
__device__ __forceinline__ void pt_resolve_body(const PtArgs& A, int slot, int bid, int nblk) {
  const PtBuf& T = A.T;
  const PtBuf::Sq& Q = T.sq[slot & 1];
  const int n = A.sc->sq[slot], P = A.P;
  const int gstride = nblk * blockDim.x;
  const int nround = (n + gstride - 1) / gstride * gstride;
  for (int j = bid * blockDim.x + threadIdx.x; j < nround; j += gstride) {
    bool is = false;
    if (j < n) {
      is = true;
      bool unocc = true;
      const int prim = Q.prim[j];
      if (prim >= 0) {
        const V3 o = ld3(Q.o, P, j), d = ld3(Q.d, P, j);
        unocc = near_eq(o + d * Q.t[j], ld3(Q.tgt, P, j));
      }
      if (unocc) film_add(A.film, Q.pix[j], ld3(Q.val, P, j));
    }
    wave_count(&A.ctr->shadow, is);
  }
}

// One PT step after its traversal: resolve the step's shadow rays (blocks
// [0, nres)) and shade its vertices (the rest, `shade` = 0 after the last
// bounce) -- they read and write different shadow-queue buffers.
// Register budget left to the compiler (106 VGPRs, 4 waves/SIMD).  Forcing more
// waves spills and loses: C3 2,738 (free) vs 2,763 (5, within noise), 2,617 (6),
// 2,603 (8) Mrays/s.
#ifndef WR_PT_WAVES
#define WR_PT_WAVES 1
#endif
__global__ void __launch_bounds__(kShadeBlock) __attribute__((amdgpu_waves_per_eu(WR_PT_WAVES, 8))) WR_NO_PK_FP32
k_pt_step(PtGroup G_, int slot, int nres, int shade) {
  const PtArgs& A = G_.a[blockIdx.y];
  if (static_cast<int>(blockIdx.x) < nres) pt_resolve_body(A, slot, blockIdx.x, nres);
  else if (shade) pt_shade_body(A, slot, blockIdx.x - nres, gridDim.x - nres);
}

__global__ void k_film_accumulate(float* dst, const float* src, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = dst[i] + src[i];
}
