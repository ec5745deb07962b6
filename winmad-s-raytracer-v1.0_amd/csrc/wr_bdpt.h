// BidirPathTracing::runIteration (surfaceIntegrator/bidirPathTracing.cpp:53-265)
// as wavefront kernels.  Two schedules (wr_render.hip, render_bdpt_one):
//   sequential: light pass gen -> [trace -> shade] x 9, then camera pass gen ->
//     [trace -> resolve + shade] x 11, as the reference orders them;
//   overlapped (default): both passes start together and bounce b of each is
//     traced by one launch (gen, then 11 steps).  A light vertex of length l
//     and a camera vertex of length c of the same path (the only pairing,
//     :130, :222-229) are connected by the vertex created second: the camera
//     side connects the light vertices stored so far (l <= c: the light
//     kernel of a step runs before the camera kernel), the light side the
//     camera vertices stored at earlier steps (c < l; camera vertices that
//     can still meet a later light vertex, c <= (maxlen - 2) / 2, are kept in
//     a small store, CV_*).  Every pair the reference connects (:219-257) is
//     connected once, with the same floats (connect_pair); only the order of
//     the film's float additions differs.
// Included by wr_render.hip inside its anonymous namespace (uses its device
// helpers: wave_append, ld3/st3, film_add, the counter slots).
#pragma once

// =============================================================== BDPT state
// Light / camera subpath state (bidirPathTracing.h:7-18), one 64-byte record
// per path: the vertex kernels gather it by path index (the queue's order), so
// a lane's state is one cache line instead of 15 words in 15 arrays.
enum : int {
  PS_O = 0, PS_D = 3, PS_THR = 6, PS_DVCM = 9, PS_DVC = 10, PS_LEN = 11, PS_NSPEC = 12, PS_CTR = 13,
  PS_VCOUNT = 14,  // light paths: stored light vertices
  PS_PIX = 14,     // camera paths: film pixel
  PS_DVM = 15,     // VCM: dVM (vertexcm.h:36)
  PS_CVCOUNT = 15, // (unused: BDPT keeps its counters in BQ_PACK)
  PS_WORDS = 16
};
__device__ __forceinline__ float& psf(float* s, int p, int k) { return s[size_t(p) * PS_WORDS + k]; }
__device__ __forceinline__ int& psi(float* s, int p, int k) {
  return reinterpret_cast<int*>(s)[size_t(p) * PS_WORDS + k];
}
__device__ __forceinline__ uint32_t& psu(float* s, int p, int k) {
  return reinterpret_cast<uint32_t*>(s)[size_t(p) * PS_WORDS + k];
}
__device__ __forceinline__ V3 ld3r(const float* s, int p, int k) {
  const float* r = s + size_t(p) * PS_WORDS + k;
  return v3(r[0], r[1], r[2]);
}
__device__ __forceinline__ void st3r(float* s, int p, int k, V3 v) {
  float* r = s + size_t(p) * PS_WORDS + k;
  r[0] = v.x;
  r[1] = v.y;
  r[2] = v.z;
}

// BDPT's own subpath record (VertexCM keeps PS_*): 32 bytes per path, half a
// PS record.  The subpath's origin and direction are not kept: the reference
// overwrites both in sampleScattering before any read (bidirPathTracing.cpp:
// 381-400 -- bsdf.sample writes the direction, origin = hitPos), and the next
// ray travels in the extension queue.  The small counters share one word:
//   BQ_PACK = len | nspec << 8 | stored vertices << 16 (light: light vertices,
//   camera: camera vertices of the overlapped schedule)
enum : int { BQ_THR = 0, BQ_DVCM = 3, BQ_DVC = 4, BQ_CTR = 5, BQ_PACK = 6, BQ_PIX = 7, BQ_WORDS = 8 };
__device__ __forceinline__ float& bqf(float* s, int p, int k) { return s[size_t(p) * BQ_WORDS + k]; }
__device__ __forceinline__ int& bqi(float* s, int p, int k) {
  return reinterpret_cast<int*>(s)[size_t(p) * BQ_WORDS + k];
}
__device__ __forceinline__ uint32_t& bqu(float* s, int p, int k) {
  return reinterpret_cast<uint32_t*>(s)[size_t(p) * BQ_WORDS + k];
}
__device__ __forceinline__ V3 bqld3(const float* s, int p, int k) {
  const float* r = s + size_t(p) * BQ_WORDS + k;
  return v3(r[0], r[1], r[2]);
}
__device__ __forceinline__ void bqst3(float* s, int p, int k, V3 v) {
  float* r = s + size_t(p) * BQ_WORDS + k;
  r[0] = v.x;
  r[1] = v.y;
  r[2] = v.z;
}
__device__ __forceinline__ int bq_pack(int len, int nspec, int cnt) { return len | (nspec << 8) | (cnt << 16); }
__device__ __forceinline__ int bq_len(int w) { return w & 255; }
__device__ __forceinline__ int bq_nspec(int w) { return (w >> 8) & 255; }
__device__ __forceinline__ int bq_count(int w) { return w >> 16; }
constexpr int kLightAlive = 0x80;  // BdptBuf::lvc

// BDPT's stored vertices (VertexCM keeps VS_*), light (B.vs) and camera (B.cv,
// overlapped schedule) alike: 64 bytes.  The geometric normal and the BSDF's
// probabilities are not stored: they are functions of the primitive (and, for
// a sphere, the position), the local wi and the material, and stored_bsdf
// rebuilds them with the operations the vertex itself ran (prim_normal,
// bsdf_probs), to the same floats.
//   BV_PACK = len | nspec << 8 | material << 16 (int16: emitters are < 0)
enum : int { BV_POS = 0, BV_WI = 3, BV_THR = 6, BV_DVCM = 9, BV_DVC = 10, BV_PRIM = 11, BV_PACK = 12, BV_PIX = 13,
             BV_WORDS = 16 };
__device__ __forceinline__ float& bvf(float* s, int i, int k) { return s[size_t(i) * BV_WORDS + k]; }
__device__ __forceinline__ int& bvi(float* s, int i, int k) {
  return reinterpret_cast<int*>(s)[size_t(i) * BV_WORDS + k];
}
__device__ __forceinline__ V3 bvld3(const float* s, int i, int k) {
  const float* r = s + size_t(i) * BV_WORDS + k;
  return v3(r[0], r[1], r[2]);
}
__device__ __forceinline__ void bvst3(float* s, int i, int k, V3 v) {
  float* r = s + size_t(i) * BV_WORDS + k;
  r[0] = v.x;
  r[1] = v.y;
  r[2] = v.z;
}
__device__ __forceinline__ int bv_pack(int len, int nspec, int mat) {
  return len | (nspec << 8) | static_cast<int>(static_cast<uint32_t>(mat) << 16);
}
__device__ __forceinline__ int bv_len(int w) { return w & 255; }
__device__ __forceinline__ int bv_nspec(int w) { return (w >> 8) & 255; }
__device__ __forceinline__ int bv_mat(int w) { return w >> 16; }  // arithmetic: the sign comes back
// one stored vertex: position, local wi, throughput, dVCM, dVC, primitive,
// (len, nspec, material) and the camera pixel
__device__ __forceinline__ void store_vertex(float* s, int i, V3 pos, const Bsdf& b, V3 thr, float dvcm, float dvc,
                                             int prim, int len, int nspec, int pix) {
  bvst3(s, i, BV_POS, pos);
  bvst3(s, i, BV_WI, b.wi);
  bvst3(s, i, BV_THR, thr);
  bvf(s, i, BV_DVCM) = dvcm;
  bvf(s, i, BV_DVC) = dvc;
  bvi(s, i, BV_PRIM) = prim;
  bvi(s, i, BV_PACK) = bv_pack(len, nspec, b.mat);
  bvi(s, i, BV_PIX) = pix;
}
// the BSDF of stored vertex i (BSDF::init at its hit, bsdf.h:66-89)
__device__ __forceinline__ Bsdf stored_bsdf(const DevScene& S, const float* s, int i, int pack) {
  Bsdf b;
  b.fr = frame_from_z(prim_normal(S, bvi(const_cast<float*>(s), i, BV_PRIM), bvld3(s, i, BV_POS)));
  b.wi = bvld3(s, i, BV_WI);
  bsdf_probs(b, bv_mat(pack), S.mats);
  return b;
}

// Stored light vertices (lightStates, bidirPathTracing.cpp:101-102), one
// 80-byte record per vertex slot k * P + p: the camera pass reads a path's
// vertices by path index (connectVertices, :219-257).
enum : int {
  VS_POS = 0, VS_N = 3, VS_WI = 6, VS_THR = 9, VS_DVCM = 12, VS_DVC = 13, VS_CONT = 14, VS_PD = 15, VS_PG = 16,
  VS_LEN = 17, VS_NSPEC = 18, VS_MAT = 19, VS_WORDS = 20
};
__device__ __forceinline__ float& vsf(float* s, int i, int k) { return s[size_t(i) * VS_WORDS + k]; }
__device__ __forceinline__ int& vsi(float* s, int i, int k) {
  return reinterpret_cast<int*>(s)[size_t(i) * VS_WORDS + k];
}
__device__ __forceinline__ V3 vld3(const float* s, int i, int k) {
  const float* r = s + size_t(i) * VS_WORDS + k;
  return v3(r[0], r[1], r[2]);
}
__device__ __forceinline__ void vst3(float* s, int i, int k, V3 v) {
  float* r = s + size_t(i) * VS_WORDS + k;
  r[0] = v.x;
  r[1] = v.y;
  r[2] = v.z;
}

// A camera vertex's direct-illumination record (getDirectIllumination,
// :484-608), one 64-byte record per path, finalised by its last resolved ray
enum : int {
  DR_NEE = 0, DR_NEEW = 3, DR_BSDF = 4, DR_THR = 7, DR_WLEN = 10, DR_FLAGS = 11, DR_LIGHT = 12, DR_PIX = 13,
  DR_STATE = 14, DR_WORDS = 16
};
__device__ __forceinline__ float& drf(float* s, int p, int k) { return s[size_t(p) * DR_WORDS + k]; }
__device__ __forceinline__ int& dri(float* s, int p, int k) {
  return reinterpret_cast<int*>(s)[size_t(p) * DR_WORDS + k];
}
__device__ __forceinline__ V3 drld3(const float* s, int p, int k) {
  const float* r = s + size_t(p) * DR_WORDS + k;
  return v3(r[0], r[1], r[2]);
}
__device__ __forceinline__ void drst3(float* s, int p, int k, V3 v) {
  float* r = s + size_t(p) * DR_WORDS + k;
  r[0] = v.x;
  r[1] = v.y;
  r[2] = v.z;
}

// Stored camera vertices of the overlapped schedule (BV_* records, slot
// j * P + p, j < kCvMax): what connectVertices (:610-665) reads of the camera
// side when a LATER light vertex of the path makes the connection.  Only
// vertices with length <= (maxlen - 2) / 2 can meet a later light vertex
// (c < l and l + 1 + c <= maxlen), so kCvMax = 4 slots for maxlen <= 10.
constexpr int kCvMax = (kVMax + 1 - 2) / 2;

struct BdptBuf {
  int P = 0, cap_sq = 0;
  float *ls, *cs;  // light / camera subpath state: BDPT BQ_WORDS, VertexCM PS_WORDS floats per path
  float* vs;       // stored light vertices: BDPT BV_WORDS, VertexCM VS_WORDS floats per record
                   // (sequential schedule: record k * P + p)
  float* cv;       // overlapped schedule: stored camera vertices, BV_WORDS floats per record
  // BDPT: stored light / camera vertices per path, one byte each -- what each
  // pass reads of the other's subpath (2 MB per 2M paths: L2-resident, where a
  // read of the other pass's record would be a line from HBM per vertex).
  // lvc's kLightAlive bit: the light subpath has an extension ray (a light
  // vertex of a greater length may still come)
  uint8_t *lvc, *cvc;
  // Overlapped schedule: the vertex stores are pools, sized by use rather than
  // by the worst case (the reference pushes only the vertices a path makes,
  // bidirPathTracing.cpp:101-102): vertex k of path p is record vidx[k * P +
  // p] of vs (cidx for cv), taken from the step counters' vpool / cpool; -1
  // when the pool was full.  A full pool or shadow queue sets the render's
  // overflow counter and the host renders again with pieces the worst case
  // fits (wr_render.hip, render_bdpt_one).  Null: records k * P + p.
  int* vidx;
  int* cidx;
  int vcap = 0, ccap = 0;
  // extension-ray queues (double buffered, SoA with stride qs).  Overlapped
  // schedule: qs = 2P, the light pass's rays of a bounce first (count
  // ext[b]), the camera pass's behind them (count ext[kCamSlot + b])
  int qs = 0;
  float *q_o[2], *q_d[2], *q_t[2];
  int *q_path[2], *q_prim[2];
  // shadow + aux closest-hit queue (splat / connection / NEE / DI-BSDF)
  // shadow / aux queue and DI records, two each: the ones of step `slot` are
  // [slot & 1], so a step's resolve and the next step's vertex shading (which
  // writes [(slot + 1) & 1]) can run in one launch
  struct Sq {
    float *o, *d, *tgt, *val, *t, *cut;  // cut: occl_cut (-INF for closest-hit DI-BSDF rays)
    int *meta, *pix, *prim;
  } sq[2];
  struct Di {
    float* r;  // DR_WORDS floats per path (DR_*); DR_STATE: rays still to resolve | DI_VIS | DI_SAME
  } di[2];
  // direct-illumination records (getDirectIllumination, :484-608)
};

struct BdptArgs {
  DevScene S;
  BdptBuf B;
  DevCounters* ctr;
  StepCounters* sc;  // this iteration's queue counters
  float* film;
  int W, H, P;     // film; P = W * H = lightPathNum (MIS, :55) -- global, whatever the piece
  int base, n;     // this piece of the iteration: global paths [base, base + n); buffers hold
                   // them at local index l = p - base (stride B.P >= n)
  uint32_t seed, iter;
  int ctl, maxlen, faithful;
  int overlap = 0;  // 1: the overlapped schedule (light splats into the step's sq, CV store, light-side connections)
  int untiled = 0;  // 1: camera paths in plain path order (a render redone with small pieces, BdptBuf)
};
// First queue index of the camera pass's extension rays of step `slot`
// (kCamSlot + bounce): overlapped, behind the light pass's rays of the same
// bounce, whose count is final once the step's light kernel has run
__device__ __forceinline__ int cam_ext_base(const BdptArgs& A, int slot) {
  return A.overlap ? A.sc->ext[slot - kCamSlot] : 0;
}
struct BdptGroup {
  BdptArgs a[kGroup];
};

__device__ __forceinline__ bool len_ok(int ctl, int L) { return ctl <= 0 || L == ctl; }

// record of stored light vertex k / camera vertex j of path p (-1: the pool was full)
__device__ __forceinline__ int lv_slot(const BdptBuf& B, int k, int p) {
  return B.vidx ? B.vidx[size_t(k) * B.P + p] : k * B.P + p;
}
__device__ __forceinline__ int cv_slot(const BdptBuf& B, int j, int p) {
  return B.cidx ? B.cidx[size_t(j) * B.P + p] : j * B.P + p;
}
// A pool record for this lane (called by the lanes that store, together:
// one atomic per wave); -1 and the overflow counter when the pool is full
__device__ __forceinline__ int pool_take(const BdptArgs& A, int* counter, int cap) {
  const int i = wave_append(counter, true);
  if (i < cap) return i;
  atomicAdd(&A.ctr->overflow, 1ull);
  return -1;
}
// a shadow / aux queue slot from wave_append: within the queue, or the overflow counter
__device__ __forceinline__ bool sq_fits(const BdptArgs& A, bool want, int si) {
  if (!want) return false;
  if (si < A.B.cap_sq) return true;
  atomicAdd(&A.ctr->overflow, 1ull);
  return false;
}
// Numerators of three MIS weights -- connectVertices (:658-664),
// getDirectIllumination's outer weight (:529) and connectToCamera's (:360):
// 1 in every product build.  scripts/perturbation_check.sh builds variants
// with 1.001 to show that the film parity gates (tests/_parity.py) catch a
// 1e-3 error in any of them.
#ifndef WR_TEST_CONN_W
#define WR_TEST_CONN_W 1.f
#endif
#ifndef WR_TEST_DI_W
#define WR_TEST_DI_W 1.f
#endif
#ifndef WR_TEST_SPLAT_W
#define WR_TEST_SPLAT_W 1.f
#endif

// generateLightSample (:267-311) + the first extension ray
__global__ void __launch_bounds__(kShadeBlock) WR_NO_PK_FP32 k_light_gen(BdptGroup G_) {
  const BdptArgs& A = G_.a[blockIdx.y];
  const BdptBuf& B = A.B;
  // (queues use the stride B.qs)
  const float lpp = 1.f / static_cast<float>(A.S.nlights);
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < A.n; p += gridDim.x * blockDim.x) {
    // local index p, global light path A.base + p (the RNG key pairs it with
    // the camera path of the same global index, :130, :222-229)
    Rng rng{stream_key(A.seed, A.iter, 0, static_cast<uint32_t>(A.base + p)), 0};
    const int id = min(static_cast<int>(rng.f() * static_cast<float>(A.S.nlights)), A.S.nlights - 1);
    const DLight L = A.S.lights[id];
    V3 pos, dir, rad;
    float epdf = 0.f, dpdf = 0.f;
    for (int tries = 0; tries < 64; ++tries) {
      // emit(..., rng.randVector3(), rng.randVector3(), ...): the reference's
      // compiler evaluates the second argument (posRand3) first
      V3 pr = rng.v();
      V3 dr = rng.v();
      rad = light_emit(L, dr, pr, &pos, &dir, &epdf, &dpdf);
      if (epdf > 1e-7f) break;
    }
    V3 thr = rad;
    epdf *= lpp;
    dpdf *= lpp;
    thr = div_plain(thr, epdf);
    bqst3(B.ls, p, BQ_THR, thr);
    bqf(B.ls, p, BQ_DVCM) = dpdf / epdf;
    bqf(B.ls, p, BQ_DVC) = 1.f / epdf;  // AreaLight::isDelta() == 0
    bqu(B.ls, p, BQ_CTR) = rng.ctr;
    bqi(B.ls, p, BQ_PACK) = bq_pack(1, 0, 0);  // pathLength 1, no specular vertex, no stored vertex
    B.lvc[p] = kLightAlive;  // no stored vertex, the first ray queued
    // Ray(origin + dir * EPS, dir) (:79-80)
    st3(B.q_o[0], B.qs, p, pos + dir * WR_EPS);
    st3(B.q_d[0], B.qs, p, normalize(dir));
    B.q_path[0][p] = p;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) A.sc->ext[0] = A.n;
}

// sampleScattering (:370-416).  Returns false when the subpath ends.
__device__ __forceinline__ bool sample_scatter(const DevScene& S, Rng& rng, const Bsdf& b, V3 hit, V3& o, V3& dir,
                                               V3& thr, float& dvcm, float& dvc, int& nspec) {
  float dpdf = 0.f, cos_wo = 0.f;
  int type;
  V3 wo = dir;
  const V3 f = bsdf_sample(b, S.mats, rng.v(), &wo, &dpdf, &cos_wo, &type);
  if (black(f)) return false;
  dir = wo;
  float rpdf = dpdf;
  if ((type & T_SPEC) == 0) rpdf = bsdf_pdf(b, S.mats, dir, true);
  const float cp = b.cont;
  if (rng.f() > cp) return false;
  dpdf *= cp;
  rpdf *= cp;
  if (type & T_SPEC) {
    ++nspec;
    dvcm = 0.f;
    dvc *= cos_wo;
  } else {
    dvc = (1.f / dpdf) * (dvcm + dvc * rpdf);
    dvcm = 1.f / dpdf;
  }
  o = hit;
  thr = mul(thr, f) * (cos_wo / dpdf);
  return true;
}

// connectVertices (:610-665) for one (camera vertex, stored light vertex)
// pair of path p: the camera vertex's BSDF b at hp with its state (cthr,
// cdvcm, cdvc, cnspec, length len) and light-vertex slot `slot` of length
// llen.  True when the shadow ray is cast (its contribution counts, or every
// ray is traced: faithful); sdir / stgt / sval then hold the ray and the value
// splatted if unoccluded.  One function for both sides of the overlapped
// schedule, so a pair's floats do not depend on which vertex came second.
__device__ __forceinline__ bool connect_pair(const BdptArgs& A, const Bsdf& b, V3 hp, V3 cthr, float cdvcm, float cdvc,
                                             int cnspec, int len, int slot, int llen, V3& sdir, V3& stgt, V3& sval,
                                             bool& counted) {
  const BdptBuf& B = A.B;
  const DevScene& S = A.S;
  bool shoot = false;
  const V3 lpos = bvld3(B.vs, slot, BV_POS);
  V3 dir = lpos - hp;
  const float d2 = sqr_len(dir);
  const float dist = sqrtf(d2);
  dir = div_guarded(dir, dist);
  float cos_c = 0.f, cdp, crp;
  const V3 cf = bsdf_f(b, S.mats, dir, &cos_c, &cdp, &crp);
  if (!black(cf)) {
    cdp *= b.cont;
    crp *= b.cont;
    const int lpk = bvi(B.vs, slot, BV_PACK);
    const Bsdf lb = stored_bsdf(S, B.vs, slot, lpk);
    float cos_l = 0.f, ldp, lrp;
    const V3 lf = bsdf_f(lb, S.mats, -dir, &cos_l, &ldp, &lrp);
    if (!black(lf)) {
      ldp *= lb.cont;
      lrp *= lb.cont;
      const float G = cos_l * cos_c / d2;
      if (!(cmpf(G) < 0)) {
        const float cdpa = cdp * fabsf(cos_l) / (dist * dist);
        const float ldpa = ldp * fabsf(cos_c) / (dist * dist);
        const V3 res = mul(cf, lf) * G;
        if (!black(res)) {
          const float wl = cdpa * (bvf(B.vs, slot, BV_DVCM) + lrp * bvf(B.vs, slot, BV_DVC));
          const float wc = ldpa * (cdvcm + crp * cdvc);
          const float w = WR_TEST_CONN_W / (wl + 1.f + wc);
          const bool counts = len_ok(A.ctl, llen + 1 + len);
          counted = counts;
          if (counts || A.faithful) {
            shoot = true;
            sdir = normalize(dir);
            stgt = hp + dir * dist;
            if (counts) {
              const float wlen = 1.f / (static_cast<float>(llen) + 1.f + static_cast<float>(len) -
                                        static_cast<float>(bv_nspec(lpk)) - static_cast<float>(cnspec));
              const V3 lthr = bvld3(B.vs, slot, BV_THR);
              sval = mul(mul(cthr, lthr), res * w) * wlen;
            }
          }
        }
      }
    }
  }
  return shoot;
}

// queue a connection's shadow ray (every lane of the wave calls it)
// A connection whose path length the control-length filter drops (:252-253)
// is still traced (faithful ray set, :244) but its outcome is never used: its
// entry carries the ray and kSqNoValue only (no target, value or pixel).
constexpr int kSqNoValue = 1 << 29;  // Sq meta: kind << 30 | kSqNoValue? | local path (< 2^29)
__device__ __forceinline__ void queue_connection(const BdptArgs& A, int qslot, bool shoot, bool counted, int p, int pix,
                                                 V3 hp, V3 sdir, V3 stgt, V3 sval) {
  const BdptBuf& B = A.B;
  const BdptBuf::Sq& Q = B.sq[qslot & 1];
  const int cap = B.cap_sq;
  const int si = wave_append(&A.sc->sq[qslot], shoot);
  if (sq_fits(A, shoot, si)) {
    st3(Q.o, cap, si, hp);
    st3(Q.d, cap, si, sdir);
    Q.cut[si] = occl_cut(hp, stgt, dot(stgt - hp, sdir));
    if (counted) {
      st3(Q.tgt, cap, si, stgt);
      st3(Q.val, cap, si, sval);
      Q.meta[si] = (SQ_CONN << 30) | p;
      Q.pix[si] = pix;
    } else {
      Q.meta[si] = (SQ_CONN << 30) | kSqNoValue | p;
    }
  }
}

// One light-subpath vertex (:77-128): path p's ray (o, d) hit prim at t
// (prim < 0: a miss, or a pending hard ray -- nothing to do).  Every lane of
// the wave calls it (queue appends).  oslot: the step whose queue gets the
// extension ray -- slot + 1, or slot + 2 for a deferred vertex (k_late_light).
__device__ __forceinline__ void light_vertex(const BdptArgs& A, int p, int prim, float t, V3 o, V3 d, int oslot) {
  const BdptBuf& B = A.B;
  const DevScene& S = A.S;
  const int P = B.P, nxt = oslot & 1;  // P: buffer stride (local paths)
  bool ext = false, splat = false;
  V3 e_o, e_d, s_o, s_d, s_val;
  int s_pix = -1;
  int lconn = 0, lslot = -1, llen = 0;  // overlapped: the stored vertex's slot, camera vertices to connect
  if (prim >= 0) {
    const Hit h = rebuild_hit(S, prim, t, o, d);
    Bsdf b;
    bsdf_init(b, -d, h.n, h.mat, S.mats);
    if (b.mat != 0) {
      float dvcm = bqf(B.ls, p, BQ_DVCM), dvc = bqf(B.ls, p, BQ_DVC);
      const int pk = bqi(B.ls, p, BQ_PACK);
      int len = bq_len(pk), nspec = bq_nspec(pk), nstored = bq_count(pk);
      V3 thr = bqld3(B.ls, p, BQ_THR);
      dvcm *= (t * t);  // pathLength > 1 || isFiniteLight: always for area lights (:94-97)
      dvcm /= fabsf(b.wi.z);
      dvc /= fabsf(b.wi.z);
      if (!b.delta) {  // lightStates.push_back (:101-102)
        const int k = nstored;
        int slot = k * P + p;
        if (B.vidx) {  // a pool record (the storing lanes of the wave take theirs together)
          slot = pool_take(A, &A.sc->vpool, B.vcap);
          B.vidx[size_t(k) * P + p] = slot;
        }
        if (slot >= 0) store_vertex(B.vs, slot, h.p, b, thr, dvcm, dvc, prim, len, nspec, -1);
        nstored = k + 1;
        if (A.overlap && slot >= 0) {  // the camera vertices stored at earlier steps (lengths < len)
          lslot = slot;
          llen = len;
          lconn = B.cvc[p];
        }
        if (len_ok(A.ctl, len + 1)) {  // connectToCamera (:105-120, :313-368)
          const DCam& cam = S.cam;
          const V3 ip = t_point(cam.w2r, h.p);
          if (check_raster(cam, ip.x, ip.y)) {
            V3 dtc = cam.pos - h.p;
            if (dot(-dtc, cam.fwd) > 0) {
              const float d2 = sqr_len(dtc);
              const float dist = sqrtf(d2);
              dtc = div_guarded(dtc, dist);
              float cos_to = 0.f, dp, rp;
              const V3 f = bsdf_f(b, S.mats, dtc, &cos_to, &dp, &rp);
              if (!black(f)) {
                rp *= b.cont;
                const float cos_at = dot(-dtc, cam.fwd);
                const float ipd = cam.plane_dist / cos_at;
                const float i2sa = (ipd * ipd) / cos_at;
                const float i2s = i2sa * fabsf(cos_to) / d2;
                const float pdf_a = i2s;
                const float s2i = 1.f / i2s;
                const V3 res = div_plain(mul(thr, f), static_cast<float>(A.P) * s2i);
#ifdef WR_DEBUG_PATH
                if (A.base + p == WR_DEBUG_PATH && A.iter == WR_DEBUG_ITER)
                  printf("[dbg gpu] len %d hit %a %a %a t %a prim %d thr %a %a %a f %a %a %a cos_to %a d2 %a i2s %a res %a %a %a black %d rp %a dvcm %a dvc %a\n",
                         len, h.p.x, h.p.y, h.p.z, t, prim, thr.x, thr.y, thr.z, f.x, f.y, f.z, cos_to, d2, i2s,
                         res.x, res.y, res.z, (int)black(res), rp, dvcm, dvc);
#endif
                if (!black(res)) {
                  const float wl = (pdf_a / static_cast<float>(A.P)) * (dvcm + rp * dvc);
                  const float w = WR_TEST_SPLAT_W / (wl + 1.f);
                  splat = true;
                  s_o = h.p;
                  s_d = normalize(dtc);  // occluded() -> Ray(p1, dir)
                  s_val = res * w;
                  s_pix = pix_index(static_cast<int>(ip.x), static_cast<int>(ip.y), A.H, A.W);
                } else {
                  // an EPS-black res is returned before the shadow test and the
                  // MIS weight (:354-355), and the caller adds it (:116-118)
                  film_add(A.film, pix_index(static_cast<int>(ip.x), static_cast<int>(ip.y), A.H, A.W), res);
                }
              }
            }
          }
        }
      }
      if (!(len + 2 > A.maxlen)) {  // (:123-127)
        Rng rng{stream_key(A.seed, A.iter, 0, static_cast<uint32_t>(A.base + p)), bqu(B.ls, p, BQ_CTR)};
        V3 lo{}, ld{};  // sampleScattering's origin and direction (outputs only)
        if (sample_scatter(S, rng, b, h.p, lo, ld, thr, dvcm, dvc, nspec)) {
          ext = true;
          ++len;
          e_o = lo + ld * WR_EPS;
          e_d = normalize(ld);
          bqst3(B.ls, p, BQ_THR, thr);
          bqf(B.ls, p, BQ_DVCM) = dvcm;
          bqf(B.ls, p, BQ_DVC) = dvc;
        }
        bqu(B.ls, p, BQ_CTR) = rng.ctr;
      }
      // len / nspec of the next vertex (when it scatters), the stored vertices
      if (ext || nstored != bq_count(pk)) bqi(B.ls, p, BQ_PACK) = bq_pack(len, nspec, nstored);
      const int lv = nstored | (ext ? kLightAlive : 0);
      if (lv != (bq_count(pk) | kLightAlive)) B.lvc[p] = static_cast<uint8_t>(lv);
    } else {  // an invalid BSDF ends the subpath (:86-88)
      B.lvc[p] &= static_cast<uint8_t>(~kLightAlive);
    }
  } else if (p >= 0) {  // a miss ends the subpath (:81-82)
    B.lvc[p] &= static_cast<uint8_t>(~kLightAlive);
  }
  const int ei = wave_append(&A.sc->ext[oslot], ext);
  if (ext) {
    st3(B.q_o[nxt], B.qs, ei, e_o);
    st3(B.q_d[nxt], B.qs, ei, e_d);
    B.q_path[nxt][ei] = p;
  }
  // sequential schedule: traced with the camera primaries; overlapped: with
  // the next step's extension rays, like the camera vertices' rays
  const int sslot = A.overlap ? kCamSlot + oslot : kCamSlot;
  const int si = wave_append(&A.sc->sq[sslot], splat);
  if (sq_fits(A, splat, si)) {
    const BdptBuf::Sq& Q = B.sq[sslot & 1];
    st3(Q.o, B.cap_sq, si, s_o);
    st3(Q.d, B.cap_sq, si, s_d);
    st3(Q.tgt, B.cap_sq, si, S.cam.pos);
    st3(Q.val, B.cap_sq, si, s_val);
    Q.cut[si] = occl_cut(s_o, S.cam.pos, dot(S.cam.pos - s_o, s_d));
    Q.meta[si] = (SQ_SPLAT << 30) | p;  // (the local path: diagnostics only)
    Q.pix[si] = s_pix;
  }
  // overlapped schedule: this light vertex connects to the path's camera
  // vertices stored at earlier steps (:219-257 reached from the camera side)
  if (A.overlap && __ballot(lconn > 0)) {
    for (int j = 0; __ballot(j < lconn); ++j) {
      bool shoot = false, counted = false;
      int pix = -1;
      V3 hp{}, sdir{}, stgt{}, sval{};
      const int cs = j < lconn ? cv_slot(B, j, p) : -1;
      if (cs >= 0) {
        const int cpk = bvi(B.cv, cs, BV_PACK);
        const int clen = bv_len(cpk);
        if (llen + 1 + clen > A.maxlen) {
          lconn = j;  // camera vertices are stored by increasing length
        } else {
          const Bsdf cb = stored_bsdf(S, B.cv, cs, cpk);
          hp = bvld3(B.cv, cs, BV_POS);
          pix = bvi(B.cv, cs, BV_PIX);
          shoot = connect_pair(A, cb, hp, bvld3(B.cv, cs, BV_THR), bvf(B.cv, cs, BV_DVCM), bvf(B.cv, cs, BV_DVC),
                               bv_nspec(cpk), clen, lslot, llen, sdir, stgt, sval, counted);
        }
      }
      queue_connection(A, sslot, shoot, counted, p, pix, hp, sdir, stgt, sval);
    }
  }
}

template <bool CAMERA>
__device__ __forceinline__ void late_vertex_body(const BdptArgs& A, const LateList& LL, const int* cnt, int slot,
                                                 int bid, int nblk);
// Blocks [0, gridDim.x - nlate) shade this step's vertices, the last nlate
// blocks the previous step's deferred ones (late_vertex_body).
__global__ void __launch_bounds__(kShadeBlock) WR_SHADE_OCC k_light_shade(BdptGroup G_, int slot, LateArgs L,
                                                                         int nlate) {
  const BdptArgs& A = G_.a[blockIdx.y];
  const int nmain = static_cast<int>(gridDim.x) - nlate;
  if (static_cast<int>(blockIdx.x) >= nmain) {
    late_vertex_body<false>(A, L.l[blockIdx.y], L.n[blockIdx.y], slot, blockIdx.x - nmain, nlate);
    return;
  }
  const BdptBuf& B = A.B;
  const int cur = slot & 1;
  const int n = A.sc->ext[slot];
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&A.ctr->closest, (unsigned long long)n);
  const int gstride = nmain * blockDim.x;
  const int nround = (n + gstride - 1) / gstride * gstride;  // whole waves reach the appends
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < nround; j += gstride) {
    int p = -1, prim = -1;
    float t = 0.f;
    V3 o = v3(0.f, 0.f, 0.f), d = v3(0.f, 0.f, 0.f);
    if (j < n) {
      p = B.q_path[cur][j];
      prim = B.q_prim[cur][j];
#ifdef WR_DEBUG_PATH
      if (A.base + p == WR_DEBUG_PATH && A.iter == WR_DEBUG_ITER) {
        const V3 o = ld3(B.q_o[cur], B.qs, j), d = ld3(B.q_d[cur], B.qs, j);
        printf("[dbg gpu] light step %d ray o %a %a %a d %a %a %a prim %d t %a\n", slot, o.x, o.y, o.z, d.x, d.y, d.z, prim,
               B.q_t[cur][j]);
      }
#endif
      if (prim >= 0) {
        t = B.q_t[cur][j];
        o = ld3(B.q_o[cur], B.qs, j);
        d = ld3(B.q_d[cur], B.qs, j);
      }
    }
    light_vertex(A, p, prim, t, o, d, slot + 1);
  }
}

// generateCameraSample (:418-452) + first extension ray, for queue entry s of
// the piece; returns the path's local index.  (VertexCM::generateCameraSample,
// vertexcm.cpp:446-479, is the same plus dVM = 0.)
template <bool VCM = false>
__device__ __forceinline__ int camera_gen_one(const BdptArgs& A, int s, int ebase = 0) {
  const BdptBuf& B = A.B;
  const DCam& cam = A.S.cam;
  // (queues use the stride B.qs)
  // queue order: 8x8 raster tiles per wave (coherent primary rays); the
  // path <-> pixel mapping stays the reference's (x = p / W, y = p % W, :422-423).
  // A tiled piece is whole 8-row bands (base and n multiples of 8 W), so the
  // tiles are the piece's own.
  const bool tiled = !A.untiled && (A.W % 8) == 0 && (A.H % 8) == 0;
  const int tiles_y = A.W / 8;
  int l;
  if (tiled) {
    const int t = s >> 6, w = s & 63;
    l = ((t / tiles_y) * 8 + (w >> 3)) * A.W + (t % tiles_y) * 8 + (w & 7);
  } else {
    l = s;
  }
  const int p = A.base + l;
  const int x = p / A.W, y = p % A.W;
  Rng rng{stream_key(A.seed, A.iter, 1, static_cast<uint32_t>(p)), 0};
  const V3 jit = rng.v();
  const float sx = static_cast<float>(x) + jit.x, sy = static_cast<float>(y) + jit.y;
  const V3 rp = t_point(cam.r2w, v3(sx, sy, 0.f));
  const V3 d = normalize(rp - cam.pos);  // Ray(pos, p - pos) (camera.cpp:37-42)
  const float cos_at = dot(cam.fwd, d);
  const float ipd = cam.plane_dist / cos_at;
  const float i2sa = (ipd * ipd) / cos_at;
  const int pix = pix_index(static_cast<int>(sx), static_cast<int>(sy), A.H, A.W);  // (:263)
  if (VCM) {
    st3r(B.cs, l, PS_O, cam.pos);
    st3r(B.cs, l, PS_D, d);
    st3r(B.cs, l, PS_THR, v3(1.f, 1.f, 1.f));
    psf(B.cs, l, PS_DVCM) = static_cast<float>(A.P) / i2sa;  // lightPathNum / cameraPdf
    psf(B.cs, l, PS_DVC) = 0.f;
    psi(B.cs, l, PS_LEN) = 1;
    psi(B.cs, l, PS_NSPEC) = 0;
    psu(B.cs, l, PS_CTR) = rng.ctr;
    psi(B.cs, l, PS_PIX) = pix;  // (VertexCM's camera gen sets PS_DVM after this)
  } else {
    bqst3(B.cs, l, BQ_THR, v3(1.f, 1.f, 1.f));
    bqf(B.cs, l, BQ_DVCM) = static_cast<float>(A.P) / i2sa;  // lightPathNum / cameraPdf
    bqf(B.cs, l, BQ_DVC) = 0.f;
    bqu(B.cs, l, BQ_CTR) = rng.ctr;
    bqi(B.cs, l, BQ_PACK) = bq_pack(1, 0, 0);  // no camera vertex stored yet
    bqi(B.cs, l, BQ_PIX) = pix;
    B.cvc[l] = 0;
  }
  const int e = ebase + s;  // overlapped: behind the light pass's first rays (cam_ext_base)
  st3(B.q_o[0], B.qs, e, cam.pos + d * WR_EPS);
  st3(B.q_d[0], B.qs, e, normalize(d));
  B.q_path[0][e] = l;
  return l;
}
__global__ void __launch_bounds__(kShadeBlock) WR_NO_PK_FP32 k_camera_gen(BdptGroup G_) {
  const BdptArgs& A = G_.a[blockIdx.y];
  const int eb = cam_ext_base(A, kCamSlot);
  for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < A.n; s += gridDim.x * blockDim.x) camera_gen_one(A, s, eb);
  if (blockIdx.x == 0 && threadIdx.x == 0) A.sc->ext[kCamSlot] = A.n;
}

// One camera-subpath vertex (:148-260): emitter hit, DI setup, vertex
// connections (shadow rays queued), scattering -- path p's ray (o, d) hit prim
// at t (prim < 0: a miss, or a pending hard ray: nothing).  Every lane of the
// wave calls it.  oslot: the step whose queues (shadow / aux, DI records,
// extension) get this vertex's rays -- slot + 1, or slot + 2 for a deferred
// vertex (k_late_camera).
// ebase: the queue index of the camera pass's first extension ray of step
// oslot (cam_ext_base, read once by the caller)
__device__ __forceinline__ void camera_vertex(const BdptArgs& A, int p, int prim, float t, V3 o, V3 d, int oslot,
                                              int ebase = 0) {
  const BdptBuf& B = A.B;
  const DevScene& S = A.S;
  const int P = B.P, nxt = oslot & 1, cap = B.cap_sq;  // P: buffer stride
  const float lpp = 1.f / static_cast<float>(S.nlights);
  const BdptBuf::Sq& Q = B.sq[oslot & 1];  // rays traced at step oslot
  const BdptBuf::Di& D = B.di[oslot & 1];
  bool live = false, ext = false, conn_phase = false, nee = false, dib = false;
  int pix = -1, nv = 0, len = 0, nspec = 0, cnspec = 0, pk = 0, ncv = 0;  // ncv: stored camera vertices
  V3 hp{}, thr{}, cthr{}, e_o{}, e_d{}, nee_tgt{}, nee_d{}, dib_o{}, dib_d{};
  float dvcm = 0.f, dvc = 0.f, cdvcm = 0.f, cdvc = 0.f;
  Bsdf b;
  b.mat = 0;
  if (prim >= 0) {
    const Hit h = rebuild_hit(S, prim, t, o, d);
    bsdf_init(b, -d, h.n, h.mat, S.mats);
    if (b.mat != 0) {
      hp = h.p;
      pix = bqi(B.cs, p, BQ_PIX);
      dvcm = bqf(B.cs, p, BQ_DVCM);
      dvc = bqf(B.cs, p, BQ_DVC);
      pk = bqi(B.cs, p, BQ_PACK);
      len = bq_len(pk);
      nspec = bq_nspec(pk);
      ncv = bq_count(pk);
      thr = bqld3(B.cs, p, BQ_THR);
      dvcm *= (t * t);  // (:180-182)
      dvcm /= fabsf(b.wi.z);
      dvc /= fabsf(b.wi.z);
      // this vertex's state, used by DI and the connections; the scatter
      // below updates thr / dvcm / dvc / nspec for the next vertex
      cthr = thr;
      cdvcm = dvcm;
      cdvc = dvc;
      cnspec = nspec;
      if (h.mat < 0) {  // hit an emitter (:184-199)
        if (len_ok(A.ctl, len)) {
          const DLight L = S.lights[-h.mat - 1];
          float dpa, ep;
          V3 r = light_radiance(L, d, &dpa, &ep);
          if (!black(r)) {
            if (len != 1) {  // getLightRadiance (:454-482)
              dpa *= lpp;
              ep *= lpp;
              const float wc = dpa * dvcm + ep * dvc;
              r = r * (1.f / (1.f + wc));
            }
            film_add(A.film, pix, mul(thr, r));
          }
        }
      } else if (len < A.maxlen) {
        live = true;
        Rng rng{stream_key(A.seed, A.iter, 1, static_cast<uint32_t>(A.base + p)), bqu(B.cs, p, BQ_CTR)};
        if (!b.delta && len_ok(A.ctl, len + 1)) {  // getDirectIllumination (:205-217, :484-608)
          const float wlen = 1.f / (static_cast<float>(len) + 1.f - static_cast<float>(nspec));
          const int lid = min(static_cast<int>(rng.f() * static_cast<float>(S.nlights)), S.nlights - 1);
          const DLight L = S.lights[lid];
          V3 dtl;
          float dist = 0.f, dpdf = 0.f, epdf = 0.f, cal = 0.f;
          const V3 illu = light_illuminance(L, hp, rng.v(), &dtl, &dist, &dpdf, &epdf, &cal);
          int flags = 0;
          V3 nee_val = v3(0.f, 0.f, 0.f), bsdf_val = v3(0.f, 0.f, 0.f);
          float nee_w = 0.f;
          if (!black(illu) && dpdf > 0) {
            float cos_to = 0.f, bdp, brp;
            const V3 bf = bsdf_f(b, S.mats, dtl, &cos_to, &bdp, &brp);
            if (!black(bf)) {
              bdp *= b.cont;
              brp *= b.cont;
              const V3 tmp = div_plain(mul(illu, bf) * cos_to, dpdf * lpp);
              if (!black(tmp)) {
                nee = true;
                flags |= DI_NEE;
                nee_d = normalize(dtl);
                nee_tgt = hp + dtl * dist;
                const float wl = bdp / (dpdf * lpp);
                const float wc = (epdf * cos_to / (dpdf * cal)) * (dvcm + brp * dvc);
                nee_w = WR_TEST_DI_W / (wl + 1.f + wc);
                nee_val = tmp * (dpdf / (dpdf + bdp));
              }
            }
          }
          V3 dtl2 = dtl;
          float dpdf2 = dpdf, cos_s = 0.f;
          int type;
          const V3 bf2 = bsdf_sample(b, S.mats, rng.v(), &dtl2, &dpdf2, &cos_s, &type);
          if (!black(bf2) && dpdf2 > 0) {
            float w = 1.f;
            V3 illu2 = illu;
            bool early = false;
            if (!(type & T_SPEC)) {
              float lpdf, ep2;
              illu2 = light_radiance(L, dtl2, &lpdf, &ep2);
              if (cmpf(lpdf) == 0) early = true;  // (:563-564) returns res unweighted
              else w = dpdf2 / (dpdf2 + lpdf);
            }
            if (early) {
              flags |= DI_EARLY;
            } else {
              dib = true;
              flags |= DI_BSDF;
              dib_o = hp + dtl2 * WR_EPS;
              dib_d = normalize(dtl2);
              if (!black(illu2)) bsdf_val = div_plain(mul(illu2, bf2) * cos_s, dpdf2) * w;
            }
          }
          // a record only when a ray will be resolved: with neither the NEE
          // nor the BSDF ray the contribution is exactly zero (:533-607)
          const int nrays = (nee ? 1 : 0) + (dib ? 1 : 0);
          if (nrays > 0) {
            dri(D.r, p, DR_FLAGS) = flags;
            drst3(D.r, p, DR_NEE, nee_val);
            drf(D.r, p, DR_NEEW) = nee_w;
            drst3(D.r, p, DR_BSDF, bsdf_val);
            drst3(D.r, p, DR_THR, thr);
            drf(D.r, p, DR_WLEN) = wlen;
            dri(D.r, p, DR_LIGHT) = lid;
            dri(D.r, p, DR_PIX) = pix;
            dri(D.r, p, DR_STATE) = nrays;
          }
        }
        if (!b.delta) {
          conn_phase = true;
          const int lv = B.lvc[p];
          nv = lv & ~kLightAlive;
          // overlapped schedule: a vertex a later light vertex may still meet
          // (len < l, l + 1 + len <= maxlen) is kept for that light vertex --
          // if the light subpath still has a ray (after this step's light
          // kernel: a vertex of length > len may come); else none will
          if (A.overlap && 2 * len + 2 <= A.maxlen && (lv & kLightAlive)) {
            const int j = ncv;
            int cs = j * P + p;
            if (B.cidx) {  // a pool record
              cs = pool_take(A, &A.sc->cpool, B.ccap);
              B.cidx[size_t(j) * P + p] = cs;
            }
            if (cs >= 0) store_vertex(B.cv, cs, hp, b, cthr, cdvcm, cdvc, prim, len, cnspec, pix);
            ncv = j + 1;
          }
        }
        V3 so{}, sd{};  // sampleScattering's origin and direction (outputs only)
        if (sample_scatter(S, rng, b, hp, so, sd, thr, dvcm, dvc, nspec)) {
          ext = true;
          e_o = so + sd * WR_EPS;
          e_d = normalize(sd);
        }
        bqu(B.cs, p, BQ_CTR) = rng.ctr;
        // the state for the NEXT vertex is committed below; the connections
        // use the values of THIS vertex (cthr, cdvcm, cdvc, cnspec)
      }
    }
  }
  // DI queue entries
  {
    const int ni = wave_append(&A.sc->sq[oslot], nee);
    if (sq_fits(A, nee, ni)) {
      st3(Q.o, cap, ni, hp);
      st3(Q.d, cap, ni, nee_d);
      st3(Q.tgt, cap, ni, nee_tgt);
      Q.cut[ni] = occl_cut(hp, nee_tgt, dot(nee_tgt - hp, nee_d));
      Q.meta[ni] = (SQ_NEE << 30) | p;
      Q.pix[ni] = pix;
    }
    const int bi = wave_append(&A.sc->sq[oslot], dib);
    if (sq_fits(A, dib, bi)) {
      st3(Q.o, cap, bi, dib_o);
      st3(Q.d, cap, bi, dib_d);
      Q.cut[bi] = -WR_INF;  // needs the closest hit (same light?)
      Q.meta[bi] = (SQ_DIB << 30) | p;
      Q.pix[bi] = pix;
    }
  }
  // vertex connections to the paired light subpath (:219-257)
  if (__ballot(conn_phase && nv > 0)) {
    for (int k = 0; __ballot(conn_phase && k < nv); ++k) {
      bool shoot = false, counted = false;
      V3 sdir{}, stgt{}, sval{};
      const int slot = conn_phase && k < nv ? lv_slot(B, k, p) : -1;
      if (slot >= 0) {
        const int llen = bv_len(bvi(B.vs, slot, BV_PACK));
        if (llen + 1 + len > A.maxlen) {
          nv = k;  // break (:237-239)
        } else {
          shoot = connect_pair(A, b, hp, cthr, cdvcm, cdvc, cnspec, len, slot, llen, sdir, stgt, sval, counted);
        }
      }
      queue_connection(A, oslot, shoot, counted, p, pix, hp, sdir, stgt, sval);
    }
  }
  if (live) {  // commit scattered state (:259-260) and the loop increment
    if (ext) {
      bqst3(B.cs, p, BQ_THR, thr);
      bqf(B.cs, p, BQ_DVCM) = dvcm;
      bqf(B.cs, p, BQ_DVC) = dvc;
      bqi(B.cs, p, BQ_PACK) = bq_pack(len + 1, nspec, ncv);
    } else if (ncv != bq_count(pk)) {
      bqi(B.cs, p, BQ_PACK) = bq_pack(len, nspec, ncv);
    }
    if (ncv != bq_count(pk)) B.cvc[p] = static_cast<uint8_t>(ncv);
  }
  const int ei = wave_append(&A.sc->ext[oslot], ext) + ebase;
  if (ext) {
    st3(B.q_o[nxt], B.qs, ei, e_o);
    st3(B.q_d[nxt], B.qs, ei, e_d);
    B.q_path[nxt][ei] = p;
  }
}

__device__ __forceinline__ void camera_shade_body(const BdptArgs& A, int slot, int bid, int nblk) {
  const BdptBuf& B = A.B;
  const int cur = slot & 1;
  const int n = A.sc->ext[slot], e0 = cam_ext_base(A, slot), eb = cam_ext_base(A, slot + 1);
  if (bid == 0 && threadIdx.x == 0) atomicAdd(&A.ctr->closest, (unsigned long long)n);
  const int gstride = nblk * blockDim.x;
  const int nround = (n + gstride - 1) / gstride * gstride;
  for (int j = bid * blockDim.x + threadIdx.x; j < nround; j += gstride) {
    int p = -1, prim = -1;
    float t = 0.f;
    V3 o = v3(0.f, 0.f, 0.f), d = v3(0.f, 0.f, 0.f);
    if (j < n) {
      const int e = e0 + j;
      p = B.q_path[cur][e];
      prim = B.q_prim[cur][e];
      if (prim >= 0) {
        t = B.q_t[cur][e];
        o = ld3(B.q_o[cur], B.qs, e);
        d = ld3(B.q_d[cur], B.qs, e);
      }
    }
    camera_vertex(A, p, prim, t, o, d, slot + 1, eb);
  }
}

// Deferred vertices (WR_TRACE_BVH, "deferred hard rays" in wr_render.hip):
// the paths whose step-(slot - 1) hit was settled off the critical path (by
// the blocks of step slot's search launch) are shaded one step late, by extra
// blocks of step slot's vertex launch, into the same queues as this step's
// vertices (step slot + 1).  Light vertices feed only their own path's camera
// connections (:130, :222-229) and every path keeps its own state, counters
// and random numbers, so the film is the one of the undeferred render.
template <bool CAMERA>
__device__ __forceinline__ void late_vertex_body(const BdptArgs& A, const LateList& LL, const int* cnt, int slot,
                                                 int bid, int nblk) {
  const int half = LL.cap >> 1;
  const int nt = min(cnt[0], half), n = nt + min(cnt[1], half);
  const int gstride = nblk * blockDim.x;
  const int nround = (n + gstride - 1) / gstride * gstride;
  for (int j = bid * blockDim.x + threadIdx.x; j < nround; j += gstride) {
    int p = -1, prim = -1;
    float t = 0.f;
    V3 o = v3(0.f, 0.f, 0.f), d = v3(0.f, 0.f, 0.f);
    if (j < n) {
      const int i = j < nt ? j : half + (j - nt);
      p = LL.pth[i];
      prim = LL.prim[i];
      t = LL.t[i];
      o = ld3(LL.o3, LL.cap, i);
      d = ld3(LL.d3, LL.cap, i);
    }
    if (CAMERA) camera_vertex(A, p, prim, t, o, d, slot + 1);
    else light_vertex(A, p, prim, t, o, d, slot + 1);
  }
}

// Light-tracing splats and camera-pass shadow / aux rays after traversal.
// Light-tracing splats and camera-pass shadow / aux rays of step `slot` after
// traversal.  A DI record is finalized (getDirectIllumination's combination,
// :533-607) by whichever of its rays is resolved last: each resolve adds
// (its result bit - 1) to the record's state word in one atomic.
__device__ __forceinline__ void sq_resolve_body(const BdptArgs& A, int slot, int bid, int nblk) {
  const BdptBuf& B = A.B;
  const DevScene& S = A.S;
  const BdptBuf::Sq& Q = B.sq[slot & 1];
  const BdptBuf::Di& D = B.di[slot & 1];
  const int cap = B.cap_sq, n = min(A.sc->sq[slot], cap);  // (appends past cap were dropped: overflow)
  const int gstride = nblk * blockDim.x;
  const int nround = (n + gstride - 1) / gstride * gstride;
  for (int j = bid * blockDim.x + threadIdx.x; j < nround; j += gstride) {
    bool is_shadow = false, is_closest = false;
    if (j < n) {
      const int meta = Q.meta[j];
      const int kind = (meta >> 30) & 3, p = meta & (kSqNoValue - 1);
      const int prim = Q.prim[j];
      const float t = Q.t[j];
      int di_bits = -1;  // >= 0: this ray belongs to DI record p
      if (meta & kSqNoValue) {  // a filtered connection: traced and counted, nothing to add
        is_shadow = true;
      } else if (kind == SQ_DIB) {  // DI BSDF-sampled ray: same light? (:570-596)
        is_closest = true;
        bool same = false;
        if (prim >= 0) {
          const int m = __float_as_int(S.prim_rec[2 * static_cast<size_t>(prim) + 1].z);
          same = m < 0 && -m - 1 == dri(D.r, p, DR_LIGHT);
        }
        di_bits = same ? DI_SAME : 0;
      } else {  // Scene::occluded: position equality (scene.cpp:55-69)
        is_shadow = true;
        bool unocc = true;
        if (prim >= 0) {
          const V3 o = ld3(Q.o, cap, j), d = ld3(Q.d, cap, j);
          unocc = near_eq(o + d * t, ld3(Q.tgt, cap, j));
        }
#ifdef WR_DEBUG_PATH
        if (kind == SQ_SPLAT && A.base + p == WR_DEBUG_PATH && A.iter == WR_DEBUG_ITER) {
          const V3 o = ld3(Q.o, cap, j), d = ld3(Q.d, cap, j), v = ld3(Q.val, cap, j);
          printf("[dbg gpu] splat o %a %a %a d %a %a %a prim %d t %a unocc %d val %a %a %a pix %d\n", o.x, o.y, o.z, d.x,
                 d.y, d.z, prim, t, (int)unocc, v.x, v.y, v.z, Q.pix[j]);
        }
#endif
        if (kind == SQ_NEE) {
          di_bits = unocc ? DI_VIS : 0;
        } else if (unocc) {
          film_add(A.film, Q.pix[j], ld3(Q.val, cap, j));
        }
      }
      if (di_bits >= 0) {
        const int st = atomicAdd(&dri(D.r, p, DR_STATE), di_bits - 1) + di_bits - 1;
        if ((st & DI_COUNT) == 0) {
          const int flags = dri(D.r, p, DR_FLAGS);
          V3 res = v3(0.f, 0.f, 0.f);
          float weight = 0.f;
          if ((flags & DI_NEE) && (st & DI_VIS)) {
            weight = drf(D.r, p, DR_NEEW);
            res = res + drld3(D.r, p, DR_NEE);
          }
          V3 di;
          if (flags & DI_EARLY) {
            di = res;
          } else {
            if ((flags & DI_BSDF) && (st & DI_SAME)) res = res + drld3(D.r, p, DR_BSDF);
            di = res * weight;
          }
          film_add(A.film, dri(D.r, p, DR_PIX), mul(drld3(D.r, p, DR_THR), di) * drf(D.r, p, DR_WLEN));
        }
      }
    }
    wave_count(&A.ctr->shadow, is_shadow);
    wave_count(&A.ctr->closest, is_closest);
  }
}

// One camera-pass step after its traversal: resolve the step's shadow / aux
// rays (blocks [0, nres)) and shade its camera vertices (the rest) -- they touch
// different queue / DI buffers.  The last step has no vertices (shade = 0).
// ... blocks [0, nres) resolve, then this step's vertices, then (the last
// nlate blocks) the previous step's deferred vertices.
__global__ void __launch_bounds__(kShadeBlock) WR_SHADE_OCC k_camera_step(BdptGroup G_, int slot, int nres,
                                                                         int shade, LateArgs L, int nlate) {
  const BdptArgs& A = G_.a[blockIdx.y];
  const int b = static_cast<int>(blockIdx.x), nmain = static_cast<int>(gridDim.x) - nlate;
  if (b < nres) sq_resolve_body(A, slot, b, nres);
  else if (b >= nmain) late_vertex_body<true>(A, L.l[blockIdx.y], L.n[blockIdx.y], slot, b - nmain, nlate);
  else if (shade) camera_shade_body(A, slot, b - nres, nmain - nres);
}
