// VertexCM (surfaceIntegrator/vertexcm.{h,cpp}) on the BDPT wavefront of
// wr_render.hip.  Included there, inside its anonymous namespace, after the
// BDPT kernels (it reuses BdptBuf / BdptArgs, camera_gen_one and
// sq_resolve_body).
//
//   light pass  : gen -> [trace -> shade] x 9                 (:67-140)
//   fix-up      : emitter-first light vertices (stale BSDF, below)
//   merge grid  : count -> exclusive scan -> scatter          (replaces :152)
//   camera pass : gen -> [trace -> resolve + shade + merge] x 11 (:157-283)
//
// The reference's point KD tree (scene/KDtree.h:88-175) answers
// searchInRadius with exactly the vertices v for which
// sqrtf(|x - v|^2) < radius (its pruning test |x[axis] - split| < radius is
// exact in float; tests/test_oracle.py checks this).  The GPU finds the same
// set in a hashed grid (cells of any size, WR_VCM_CELL x r'): the query visits
// every cell overlapping [x - r', x + r'] per axis with r' = r (1 + 2^-10),
// which holds every vertex the float test can accept (|fl(x - v)| <=
// fl-distance < r, and float subtraction, scaling and floor are monotone),
// applies the reference's test, and takes a vertex only in its own cell (a
// bucket may hold several cells).  Only the summation order of the merged
// contributions differs.

struct VcmBuf {
  // (dVM of the light / camera subpath state, vertexcm.h:36: word PS_DVM of
  // BdptBuf's path records)
  // Probabilities of the last non-emitter BSDF built on each light path (the
  // emitter-vertex quirk, k_vcm_light_shade): (pd, pg, continueProb, has one)
  float4* l_sb;
  float* v_dvm;    // [kVMax][P] beside BdptBuf's vertex store
  int* pending;    // light paths whose first vertex is an emitter
  int* cnt;        // [T + 1] vertices per grid bucket, then 0 after the scatter
  int* start;      // [T + 1] exclusive scan of cnt
  // merge records, bucket-sorted: the range scan reads only rpos
  float4* rpos;    // [kVMax * P] {pos, pathLength}
  float4* rdat;    // [kVMax * P][2] {wiWorld, continueProb}, {throughput, dVCM}
  float* rdvm;     // [kVMax * P] dVM
  // merge queries of a camera-pass step (vcm_merge_body), [2][field][P]: the
  // camera vertex's position, BSDF (normal, wiLocal, probabilities, matId) and
  // subpath state
  struct Mq {
    float *hp, *n, *wi, *thr, *dvcm, *dvm, *cont, *pd, *pg;
    int *mat, *len, *pix;
  } mq[2];
  void* scan_tmp;  // hipcub scan scratch
  size_t scan_bytes;
};

struct VcmArgs {
  BdptArgs a;  // S, B, counters, film, W / H / P, seed, iter, maxlen
  VcmBuf V;
  int minlen;
  float N;                               // lightSubPathNum (:49-51)
  float radius, vm_norm, mis_vm, mis_vc;  // (:53-64)
  V3 org;                                // grid origin (root box corner)
  float inv_cs, rq;                      // 1 / cell size, query half-width r (1 + 2^-10)
  float r2t;                             // sqrtf(s) < radius  <=>  s < r2t (exact, host-derived)
  uint32_t tmask;                        // T - 1
};
struct VcmGroup {
  VcmArgs a[kGroup];
};

__device__ __forceinline__ int vcm_cell(float x, float org, float inv_cs) {
  const float c = floorf((x - org) * inv_cs);
  return static_cast<int>(clampv(c, -1073741824.f, 1073741824.f));
}
// Buckets: a grid row (cy, cz) is hashed to a run of kRowW buckets, one per
// cx (mod kRowW), so the cells [x0, x1] of a row are one contiguous bucket
// range (two where cx wraps): a query reads one range per row.
constexpr int kRowBits = 10, kRowW = 1 << kRowBits;
__device__ __forceinline__ uint32_t vcm_row(int y, int z, uint32_t tmask) {
  return (((static_cast<uint32_t>(y) * 19349663u) ^ (static_cast<uint32_t>(z) * 83492791u)) << kRowBits) & tmask;
}
__device__ __forceinline__ uint32_t vcm_bucket(const VcmArgs& X, V3 p) {
  return vcm_row(vcm_cell(p.y, X.org.y, X.inv_cs), vcm_cell(p.z, X.org.z, X.inv_cs), X.tmask) |
         (static_cast<uint32_t>(vcm_cell(p.x, X.org.x, X.inv_cs)) & (kRowW - 1));
}

// generateLightSample (:287-330) + the first extension ray
__global__ void __launch_bounds__(kShadeBlock) WR_NO_PK_FP32 k_vcm_light_gen(VcmGroup G_) {
  const VcmArgs& X = G_.a[blockIdx.y];
  const BdptArgs& A = X.a;
  const BdptBuf& B = A.B;
  const VcmBuf& V = X.V;
  const int P = A.P;
  const float lpp = 1.f / static_cast<float>(A.S.nlights);
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < P; p += gridDim.x * blockDim.x) {
    Rng rng{stream_key(A.seed, A.iter, 0, static_cast<uint32_t>(p)), 0};
    const int id = min(static_cast<int>(rng.f() * static_cast<float>(A.S.nlights)), A.S.nlights - 1);
    const DLight L = A.S.lights[id];
    V3 pos, dir, rad;
    float epdf = 0.f, dpdf = 0.f, cal = 0.f;
    for (int tries = 0; tries < 64; ++tries) {  // posRand3 drawn first
      V3 pr = rng.v();
      V3 dr = rng.v();
      rad = light_emit(L, dr, pr, &pos, &dir, &epdf, &dpdf, &cal);
      if (epdf > 1e-7f) break;
    }
    V3 thr = rad;
    epdf = smax(epdf, 1e-7f);
    epdf *= lpp;
    dpdf *= lpp;
    thr = div_plain(thr, epdf);
    const float dvc = cal / epdf;  // AreaLight: finite, not delta -> cosAtLight
    st3r(B.ls, p, PS_O, pos);
    st3r(B.ls, p, PS_D, dir);
    st3r(B.ls, p, PS_THR, thr);
    psf(B.ls, p, PS_DVCM) = dpdf / epdf;
    psf(B.ls, p, PS_DVC) = dvc;
    psf(B.ls, p, PS_DVM) = dvc * X.mis_vc;
    psi(B.ls, p, PS_LEN) = 1;
    psu(B.ls, p, PS_CTR) = rng.ctr;
    psi(B.ls, p, PS_VCOUNT) = 0;
    V.l_sb[p] = make_float4(0.f, 0.f, 0.f, __int_as_float(0));
    st3(B.q_o[0], P, p, pos + dir * WR_EPS);  // Ray(origin + dir * EPS, dir) (:79-80)
    st3(B.q_d[0], P, p, normalize(dir));
    B.q_path[0][p] = p;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) A.sc->ext[0] = P;
}

// VertexCM::sampleScattering (:386-444)
__device__ __forceinline__ bool vcm_scatter(const VcmArgs& X, Rng& rng, const Bsdf& b, V3 hit, V3& o, V3& dir,
                                            V3& thr, float& dvcm, float& dvc, float& dvm) {
  float dpdf = 0.f, cos_wo = 0.f;
  int type;
  V3 wo = dir;
  const V3 f = bsdf_sample(b, X.a.S.mats, rng.v(), &wo, &dpdf, &cos_wo, &type);
  if (black(f)) return false;
  dir = wo;
  float rpdf = dpdf;
  if ((type & T_SPEC) == 0) rpdf = bsdf_pdf(b, X.a.S.mats, dir, true);
  const float cp = b.cont;
  if (rng.f() > cp) return false;
  dpdf *= cp;
  rpdf *= cp;
  if (type & T_SPEC) {
    dvcm = 0.f;
    dvc *= cos_wo;
    dvm *= cos_wo;
  } else {
    dvc = (cos_wo / dpdf) * (dvc * rpdf + dvcm + X.mis_vm);
    dvm = (cos_wo / dpdf) * (dvm * rpdf + dvcm * X.mis_vc + 1.f);
    dvcm = 1.f / dpdf;
  }
  o = hit;
  thr = mul(thr, f) * (cos_wo / dpdf);
  return true;
}

// One light-subpath vertex (:82-137): light-vertex store, connectToCamera
// (:332-384, splat ray queued with the camera primaries), scattering.
//
// Emitter hits: BSDF::init skips calcComponentProb for matId < 0 (bsdf.h:78-83),
// so componentProb / continueProb keep what the stack slot held -- the BSDF
// built before it in the reference's serial loop.  On a path's later vertex
// that is this path's previous vertex (l_s*); on its first vertex it is the
// last non-emitter BSDF of an earlier light path, known only after the whole
// pass: such vertices are stored provisionally and settled by k_vcm_fixup.
// Emitter vertices never connect (BSDF::f is black for matId < 0) and end the
// path (BSDF::sample too), but a non-delta one is merged (vertexcm.h:77-78).
__global__ void __launch_bounds__(kShadeBlock) WR_SHADE_OCC k_vcm_light_shade(VcmGroup G_, int slot) {
  const VcmArgs& X = G_.a[blockIdx.y];
  const BdptArgs& A = X.a;
  const BdptBuf& B = A.B;
  const VcmBuf& V = X.V;
  const DevScene& S = A.S;
  const int P = A.P, cur = slot & 1, nxt = cur ^ 1;
  const int n = A.sc->ext[slot];
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&A.ctr->closest, (unsigned long long)n);
  const int gstride = gridDim.x * blockDim.x;
  const int nround = (n + gstride - 1) / gstride * gstride;  // whole waves reach the appends
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < nround; j += gstride) {
    bool ext = false, splat = false, pend = false;
    V3 e_o, e_d, s_o, s_d, s_val;
    int s_pix = -1, p = -1;
    if (j < n) {
      p = B.q_path[cur][j];
      const int prim = B.q_prim[cur][j];
      if (prim >= 0) {
        const float t = B.q_t[cur][j];
        const V3 o = ld3(B.q_o[cur], P, j), d = ld3(B.q_d[cur], P, j);
        const Hit h = rebuild_hit(S, prim, t, o, d);
        Bsdf b;
        bsdf_init(b, -d, h.n, h.mat, S.mats);
        if (b.mat != 0) {
          int len = psi(B.ls, p, PS_LEN);
          if (b.mat < 0) {
            if (len > 1) {
              const float4 sb = V.l_sb[p];
              b.pd = sb.x;
              b.pg = sb.y;
              b.cont = sb.z;
              b.delta = (cmpf(b.pd) == 0 && cmpf(b.pg) == 0);
            } else {
              pend = true;  // decided by k_vcm_fixup
            }
          } else {
            V.l_sb[p] = make_float4(b.pd, b.pg, b.cont, __int_as_float(1));
          }
          float dvcm = psf(B.ls, p, PS_DVCM), dvc = psf(B.ls, p, PS_DVC), dvm = psf(B.ls, p, PS_DVM);
          V3 thr = ld3r(B.ls, p, PS_THR);
          // `pathLength > 1 || isFiniteLight == 1` (:94-95): isFiniteLight is a
          // signed 1-bit field (vertexcm.h:31) that reads back -1, so only the
          // path length counts -- unlike BDPT
          if (len > 1) dvcm *= (t * t);
          dvcm /= fabsf(b.wi.z);
          dvc /= fabsf(b.wi.z);
          dvm /= fabsf(b.wi.z);
          if (!b.delta) {  // lightVertices.push_back (:98-113)
            const int k = psi(B.ls, p, PS_VCOUNT);
            const int vs = k * P + p;
            vst3(B.vs, vs, VS_POS, h.p);
            vst3(B.vs, vs, VS_N, h.n);
            vst3(B.vs, vs, VS_WI, b.wi);
            vst3(B.vs, vs, VS_THR, thr);
            vsf(B.vs, vs, VS_DVCM) = dvcm;
            vsf(B.vs, vs, VS_DVC) = dvc;
            V.v_dvm[vs] = dvm;
            vsf(B.vs, vs, VS_CONT) = b.cont;
            vsf(B.vs, vs, VS_PD) = b.pd;
            vsf(B.vs, vs, VS_PG) = b.pg;
            vsi(B.vs, vs, VS_LEN) = len;
            vsi(B.vs, vs, VS_MAT) = b.mat;
            psi(B.ls, p, PS_VCOUNT) = k + 1;
            if (b.mat > 0 && len + 1 >= X.minlen) {  // connectToCamera (:116-127, :332-384)
              const DCam& cam = S.cam;
              const V3 ip = t_point(cam.w2r, h.p);
              if (check_raster(cam, ip.x, ip.y)) {
                V3 dtc = cam.pos - h.p;
                if (cmpf(dot(-dtc, cam.fwd)) > 0) {
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
                    const float wl = (i2s / X.N) * (X.mis_vm + dvcm + dvc * rp);
                    const float w = 1.f / (wl + 1.f);
                    const float s2i = 1.f / i2s;
                    const V3 res = div_plain(mul(thr, f) * w, X.N * s2i);
                    if (!black(res)) {
                      splat = true;
                      s_o = h.p;
                      s_d = normalize(dtc);  // occluded() -> Ray(p1, dir)
                      s_val = res;
                      s_pix = pix_index(static_cast<int>(ip.x), static_cast<int>(ip.y), A.H, A.W);
                    } else {  // EPS-black: returned unoccluded (vertexcm.cpp:375-376), added (:126-127)
                      film_add(A.film, pix_index(static_cast<int>(ip.x), static_cast<int>(ip.y), A.H, A.W), res);
                    }
                  }
                }
              }
            }
          }
          if (b.mat > 0 && !(len + 2 > A.maxlen)) {  // (:129-133); an emitter's sample is black
            Rng rng{stream_key(A.seed, A.iter, 0, static_cast<uint32_t>(p)), psu(B.ls, p, PS_CTR)};
            V3 lo = ld3r(B.ls, p, PS_O), ld = ld3r(B.ls, p, PS_D);
            if (vcm_scatter(X, rng, b, h.p, lo, ld, thr, dvcm, dvc, dvm)) {
              ext = true;
              ++len;
              e_o = lo + ld * WR_EPS;
              e_d = normalize(ld);
              st3r(B.ls, p, PS_O, lo);
              st3r(B.ls, p, PS_D, ld);
              st3r(B.ls, p, PS_THR, thr);
              psf(B.ls, p, PS_DVCM) = dvcm;
              psf(B.ls, p, PS_DVC) = dvc;
              psf(B.ls, p, PS_DVM) = dvm;
              psi(B.ls, p, PS_LEN) = len;
            }
            psu(B.ls, p, PS_CTR) = rng.ctr;
          }
        }
      }
    }
    const int pi = wave_append(&A.sc->vcm_pending, pend);
    if (pend) V.pending[pi] = p;
    const int ei = wave_append(&A.sc->ext[slot + 1], ext);
    if (ext) {
      st3(B.q_o[nxt], P, ei, e_o);
      st3(B.q_d[nxt], P, ei, e_d);
      B.q_path[nxt][ei] = p;
    }
    const int si = wave_append(&A.sc->sq[kCamSlot], splat);  // traced with the camera primaries
    if (splat) {
      const BdptBuf::Sq& Q = B.sq[kCamSlot & 1];
      st3(Q.o, B.cap_sq, si, s_o);
      st3(Q.d, B.cap_sq, si, s_d);
      st3(Q.tgt, B.cap_sq, si, S.cam.pos);
      st3(Q.val, B.cap_sq, si, s_val);
      Q.cut[si] = occl_cut(s_o, S.cam.pos, dot(S.cam.pos - s_o, s_d));
      Q.meta[si] = SQ_SPLAT << 30;
      Q.pix[si] = s_pix;
    }
  }
}

// Emitter vertices that are their path's first: the probabilities of the last
// non-emitter BSDF of the nearest earlier light path that built one (zero at
// the iteration's start), then isDelta from them (bsdf.h:86).  A delta one is
// dropped from the store.  Rare (a light path leaving one emitter and hitting
// another first); the backward walk is per entry.
__global__ void __launch_bounds__(kShadeBlock) k_vcm_fixup(VcmGroup G_) {
  const VcmArgs& X = G_.a[blockIdx.y];
  const BdptBuf& B = X.a.B;
  const VcmBuf& V = X.V;
  const int n = X.a.sc->vcm_pending;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int p = V.pending[i];
    int q = p - 1;
    while (q >= 0 && __float_as_int(V.l_sb[q].w) == 0) --q;
    float pd = 0.f, pg = 0.f, cont = 0.f;
    if (q >= 0) {
      const float4 sb = V.l_sb[q];
      pd = sb.x;
      pg = sb.y;
      cont = sb.z;
    }
    if (cmpf(pd) == 0 && cmpf(pg) == 0) {
      psi(B.ls, p, PS_VCOUNT) = 0;  // its only vertex (slot 0)
    } else {
      vsf(B.vs, p, VS_PD) = pd;
      vsf(B.vs, p, VS_PG) = pg;
      vsf(B.vs, p, VS_CONT) = cont;
    }
  }
}

// Merge grid, pass 1: vertices per bucket (and the total, for the stats)
__global__ void __launch_bounds__(kShadeBlock) k_vgrid_count(VcmGroup G_) {
  const VcmArgs& X = G_.a[blockIdx.y];
  const BdptBuf& B = X.a.B;
  const int P = X.a.P;
  const int gstride = gridDim.x * blockDim.x;
  const int nround = (P + gstride - 1) / gstride * gstride;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < nround; p += gstride) {
    const int nv = p < P ? psi(B.ls, p, PS_VCOUNT) : 0;
    for (int k = 0; k < nv; ++k) {
      const V3 pos = vld3(B.vs, k * P + p, VS_POS);
      atomicAdd(&X.V.cnt[vcm_bucket(X, pos)], 1);
    }
    const unsigned long long tot = wave_sum(static_cast<unsigned long long>(nv));
    if (lane_id() == 0 && tot) atomicAdd(&X.a.sc->vcm_nverts, static_cast<int>(tot));
  }
}

// Merge grid, pass 2 (after the exclusive scan cnt -> start): bucket-sorted
// merge records {pos, pathLength}, {wiWorld, continueProb}, {throughput, dVCM},
// {dVM} -- what RangeQuery::process reads of a light vertex (vertexcm.h:59-96).
__global__ void __launch_bounds__(kShadeBlock) k_vgrid_scatter(VcmGroup G_) {
  const VcmArgs& X = G_.a[blockIdx.y];
  const BdptBuf& B = X.a.B;
  const VcmBuf& V = X.V;
  const int P = X.a.P;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < P; p += gridDim.x * blockDim.x) {
    const int nv = psi(B.ls, p, PS_VCOUNT);
    for (int k = 0; k < nv; ++k) {
      const int vs = k * P + p;
      const V3 pos = vld3(B.vs, vs, VS_POS);
      const uint32_t h = vcm_bucket(X, pos);
      const int idx = V.start[h] + atomicSub(&V.cnt[h], 1) - 1;
      const Frame fr = frame_from_z(vld3(B.vs, vs, VS_N));
      const V3 ldir = to_world(fr, vld3(B.vs, vs, VS_WI));  // BSDF::wiWorld (bsdf.h:101-104)
      const V3 thr = vld3(B.vs, vs, VS_THR);
      V.rpos[idx] = make_float4(pos.x, pos.y, pos.z, __int_as_float(vsi(B.vs, vs, VS_LEN)));
      V.rdat[2 * static_cast<size_t>(idx)] = make_float4(ldir.x, ldir.y, ldir.z, vsf(B.vs, vs, VS_CONT));
      V.rdat[2 * static_cast<size_t>(idx) + 1] = make_float4(thr.x, thr.y, thr.z, vsf(B.vs, vs, VS_DVCM));
      V.rdvm[idx] = V.v_dvm[vs];
    }
  }
}

// Vertex merging at one camera vertex: KdTree::searchInRadius (KDtree.h:141-175)
// + RangeQuery::process (vertexcm.h:59-96).  Returns the contribution sum.
__device__ __forceinline__ V3 vcm_merge(const VcmArgs& X, const Bsdf& b, V3 hp, int len, float cdvcm, float cdvm,
                                        unsigned& found, unsigned& merged) {
  // (the reference skips the search when there are no light vertices at all)
  const VcmBuf& V = X.V;
  V3 acc = v3(0.f, 0.f, 0.f);
  const int x0 = vcm_cell(hp.x - X.rq, X.org.x, X.inv_cs), x1 = vcm_cell(hp.x + X.rq, X.org.x, X.inv_cs);
  const int y0 = vcm_cell(hp.y - X.rq, X.org.y, X.inv_cs), y1 = vcm_cell(hp.y + X.rq, X.org.y, X.inv_cs);
  const int z0 = vcm_cell(hp.z - X.rq, X.org.z, X.inv_cs), z1 = vcm_cell(hp.z + X.rq, X.org.z, X.inv_cs);
  const int ny = y1 - y0 + 1, nrow = ny * (z1 - z0 + 1);
  const bool whole = x1 - x0 >= kRowW - 1;
  const uint32_t a = static_cast<uint32_t>(x0) & (kRowW - 1), bx = static_cast<uint32_t>(x1) & (kRowW - 1);
  for (int k = 0; k < 2 * nrow; ++k) {  // row k / 2, part k % 2 (the wrapped tail of a row)
    const int cy = y0 + (k >> 1) % ny, cz = z0 + (k >> 1) / ny;
    const uint32_t row = vcm_row(cy, cz, X.tmask);
    uint32_t lo, hi;
    if (whole) {
      if (k & 1) continue;
      lo = row;
      hi = row | (kRowW - 1);
    } else if (a <= bx) {
      if (k & 1) continue;
      lo = row | a;
      hi = row | bx;
    } else {
      lo = (k & 1) ? row : (row | a);
      hi = (k & 1) ? (row | bx) : (row | (kRowW - 1));
    }
    const int i1 = V.start[hi + 1];
    for (int i = V.start[lo]; i < i1; ++i) {
      const float4 r0 = V.rpos[i];
      const V3 dd = hp - v3(r0.x, r0.y, r0.z);
      if (!(sqr_len(dd) < X.r2t)) continue;  // == sqrtf(|dd|^2) < radius (KDtree.h:171-173)
      // buckets are shared (hashed rows, cx mod kRowW): take the vertex only
      // from its own row and within this query's x cells
      const int vx = vcm_cell(r0.x, X.org.x, X.inv_cs);
      if (vcm_cell(r0.y, X.org.y, X.inv_cs) != cy || vcm_cell(r0.z, X.org.z, X.inv_cs) != cz || vx < x0 || vx > x1)
        continue;
      ++found;
      const int llen = __float_as_int(r0.w);
      if (llen + len > X.a.maxlen || llen + len < X.minlen) continue;
      const float4 r1 = V.rdat[2 * static_cast<size_t>(i)];
      float cos_c = 0.f, dp, rp;
      const V3 f = bsdf_f(b, X.a.S.mats, v3(r1.x, r1.y, r1.z), &cos_c, &dp, &rp);
      if (black(f)) continue;
      ++merged;
      const float4 r2 = V.rdat[2 * static_cast<size_t>(i) + 1];
      const float ldvm = V.rdvm[i];
      dp *= b.cont;
      rp *= r1.w;
      const float wl = r2.w * X.mis_vc + ldvm * dp;
      const float wc = cdvcm * X.mis_vc + cdvm * rp;
      const float w = 1.f / (wl + 1.f + wc);
      acc = acc + mul(f, v3(r2.x, r2.y, r2.z)) * w;
    }
  }
  return acc;
}

// generateCameraSample (:446-479)
__global__ void __launch_bounds__(kShadeBlock) WR_NO_PK_FP32 k_vcm_camera_gen(VcmGroup G_) {
  const VcmArgs& X = G_.a[blockIdx.y];
  for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < X.a.P; s += gridDim.x * blockDim.x) {
    const int p = camera_gen_one<true>(X.a, s);
    psf(X.a.B.cs, p, PS_DVM) = 0.f;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) X.a.sc->ext[kCamSlot] = X.a.P;
}

// One camera-subpath vertex (:166-281): emitter hit (getLightRadiance
// :481-514), NEE (getDirectIllumination :516-573, shadow ray queued), vertex
// connections to the paired light path (:575-636, shadow rays queued), vertex
// merging (inline), scattering.
__device__ __forceinline__ void vcm_camera_shade_body(const VcmArgs& X, int slot, int bid, int nblk) {
  const BdptArgs& A = X.a;
  const BdptBuf& B = A.B;
  const VcmBuf& V = X.V;
  const DevScene& S = A.S;
  const int P = A.P, cur = slot & 1, nxt = cur ^ 1, cap = B.cap_sq;
  const int n = A.sc->ext[slot];
  if (bid == 0 && threadIdx.x == 0) atomicAdd(&A.ctr->closest, (unsigned long long)n);
  const bool any_verts = A.sc->vcm_nverts > 0;
  const int gstride = nblk * blockDim.x;
  const int nround = (n + gstride - 1) / gstride * gstride;
  const float lpp = 1.f / static_cast<float>(S.nlights);
  const BdptBuf::Sq& Q = B.sq[(slot + 1) & 1];  // rays traced at the next step
  for (int j = bid * blockDim.x + threadIdx.x; j < nround; j += gstride) {
    bool ext = false, conn_phase = false, nee = false, query = false;
    int p = -1, pix = -1, nv = 0, len = 0;
    V3 hp{}, hn{}, thr{}, cthr{}, e_o{}, e_d{}, nee_tgt{}, nee_d{}, nee_val{};
    float dvcm = 0.f, dvc = 0.f, dvm = 0.f, cdvcm = 0.f, cdvc = 0.f, cdvm = 0.f;
    Bsdf b;
    b.mat = 0;
    if (j < n) {
      p = B.q_path[cur][j];
      const int prim = B.q_prim[cur][j];
      if (prim >= 0) {
        const float t = B.q_t[cur][j];
        const V3 o = ld3(B.q_o[cur], P, j), d = ld3(B.q_d[cur], P, j);
        const Hit h = rebuild_hit(S, prim, t, o, d);
        bsdf_init(b, -d, h.n, h.mat, S.mats);
        if (b.mat != 0) {
          hp = h.p;
          hn = h.n;
          pix = psi(B.cs, p, PS_PIX);
          dvcm = psf(B.cs, p, PS_DVCM);
          dvc = psf(B.cs, p, PS_DVC);
          dvm = psf(B.cs, p, PS_DVM);
          len = psi(B.cs, p, PS_LEN);
          thr = ld3r(B.cs, p, PS_THR);
          dvcm *= (t * t);  // (:190-193)
          dvcm /= fabsf(b.wi.z);
          dvc /= fabsf(b.wi.z);
          dvm /= fabsf(b.wi.z);
          cthr = thr;
          cdvcm = dvcm;
          cdvc = dvc;
          if (h.mat < 0) {  // (:195-209)
            if (len >= X.minlen) {
              const DLight L = S.lights[-h.mat - 1];
              float dpa, ep;
              V3 r = light_radiance(L, d, &dpa, &ep);
              if (!black(r)) {
                if (len != 1) {
                  dpa *= lpp;
                  ep *= lpp;
                  const float wc = dpa * dvcm + ep * dvc;
                  r = r * (1.f / (1.f + wc));
                }
                film_add(A.film, pix, mul(thr, r));
              }
            }
          } else if (len < A.maxlen) {
            Rng rng{stream_key(A.seed, A.iter, 1, static_cast<uint32_t>(p)), psu(B.cs, p, PS_CTR)};
            if (!b.delta && len + 1 >= X.minlen) {  // getDirectIllumination (:216-222, :516-573)
              const int lid = min(static_cast<int>(rng.f() * static_cast<float>(S.nlights)), S.nlights - 1);
              const DLight L = S.lights[lid];
              V3 dtl;
              float dist = 0.f, dpdf = 0.f, epdf = 0.f, cal = 0.f;
              const V3 illu = light_illuminance(L, hp, rng.v(), &dtl, &dist, &dpdf, &epdf, &cal);
              if (!black(illu)) {
                float cos_to = 0.f, bdp, brp;
                const V3 bf = bsdf_f(b, S.mats, dtl, &cos_to, &bdp, &brp);
                if (!black(bf)) {
                  bdp *= b.cont;  // AreaLight is not delta
                  brp *= b.cont;
                  const float wl = bdp / (lpp * dpdf);
                  const float wc = (epdf * cos_to / (dpdf * cal)) * (X.mis_vm + dvcm + dvc * brp);
                  const float w = 1.f / (wl + 1.f + wc);
                  const V3 res = mul(illu, bf) * (w * cos_to / (lpp * dpdf));
                  if (!black(res)) {
                    nee = true;
                    nee_d = normalize(dtl);
                    nee_tgt = hp + dtl * dist;
                    nee_val = mul(thr, res);
                  }
                }
              }
            }
            if (!b.delta) {
              conn_phase = true;
              nv = psi(B.ls, p, PS_VCOUNT);
              query = any_verts;  // vertex merging (:265-276): queued for the next launch
              cdvm = dvm;
            }
            V3 so = ld3r(B.cs, p, PS_O), sd = ld3r(B.cs, p, PS_D);
            if (vcm_scatter(X, rng, b, hp, so, sd, thr, dvcm, dvc, dvm)) {
              ext = true;
              e_o = so + sd * WR_EPS;
              e_d = normalize(sd);
              st3r(B.cs, p, PS_O, so);
              st3r(B.cs, p, PS_D, sd);
              st3r(B.cs, p, PS_THR, thr);
              psf(B.cs, p, PS_DVCM) = dvcm;
              psf(B.cs, p, PS_DVC) = dvc;
              psf(B.cs, p, PS_DVM) = dvm;
              psi(B.cs, p, PS_LEN) = len + 1;
            }
            psu(B.cs, p, PS_CTR) = rng.ctr;
          }
        }
      }
    }
    wave_count(&A.ctr->vm_queries, query);
    const int mi = wave_append(&A.sc->mq[slot], query);
    if (query) {
      const VcmBuf::Mq& M = V.mq[slot & 1];
      st3(M.hp, P, mi, hp);
      st3(M.n, P, mi, hn);
      st3(M.wi, P, mi, b.wi);
      st3(M.thr, P, mi, cthr);
      M.dvcm[mi] = cdvcm;
      M.dvm[mi] = cdvm;
      M.cont[mi] = b.cont;
      M.pd[mi] = b.pd;
      M.pg[mi] = b.pg;
      M.mat[mi] = b.mat;
      M.len[mi] = len;
      M.pix[mi] = pix;
    }
    const int ni = wave_append(&A.sc->sq[slot + 1], nee);
    if (nee) {  // resolved like a connection: value added when unoccluded
      st3(Q.o, cap, ni, hp);
      st3(Q.d, cap, ni, nee_d);
      st3(Q.tgt, cap, ni, nee_tgt);
      st3(Q.val, cap, ni, nee_val);
      Q.cut[ni] = occl_cut(hp, nee_tgt, dot(nee_tgt - hp, nee_d));
      Q.meta[ni] = (SQ_CONN << 30) | p;
      Q.pix[ni] = pix;
    }
    // vertex connections to the paired light path (:224-262)
    if (__ballot(conn_phase && nv > 0)) {
      for (int k = 0; __ballot(conn_phase && k < nv); ++k) {
        bool shoot = false;
        V3 sdir{}, stgt{}, sval{};
        if (conn_phase && k < nv) {
          const int vs = k * P + p;
          const int llen = vsi(B.vs, vs, VS_LEN);
          if (llen + 1 + len > A.maxlen) {
            nv = k;  // break (:242-244)
          } else if (llen + 1 + len >= X.minlen && vsi(B.vs, vs, VS_MAT) > 0) {  // emitter vertices: BSDF::f is black
            // connectVertices (:575-636)
            const V3 lpos = vld3(B.vs, vs, VS_POS);
            V3 dir = lpos - hp;
            const float d2 = sqr_len(dir);
            const float dist = sqrtf(d2);
            dir = div_guarded(dir, dist);
            float cos_c = 0.f, cdp, crp;
            const V3 cf = bsdf_f(b, S.mats, dir, &cos_c, &cdp, &crp);
            if (!black(cf)) {
              cdp *= b.cont;
              crp *= b.cont;
              Bsdf lb;
              lb.mat = vsi(B.vs, vs, VS_MAT);
              lb.fr = frame_from_z(vld3(B.vs, vs, VS_N));
              lb.wi = vld3(B.vs, vs, VS_WI);
              lb.pd = vsf(B.vs, vs, VS_PD);
              lb.pg = vsf(B.vs, vs, VS_PG);
              lb.cont = vsf(B.vs, vs, VS_CONT);
              float cos_l = 0.f, ldp, lrp;
              const V3 lf = bsdf_f(lb, S.mats, -dir, &cos_l, &ldp, &lrp);
              if (!black(lf)) {
                ldp *= lb.cont;
                lrp *= lb.cont;
                const float G = cos_l * cos_c / d2;
                if (!(cmpf(G) < 0)) {
                  const float cdpa = cdp * fabsf(cos_l) / (dist * dist);  // pdfWtoA (math.cpp:13-16)
                  const float ldpa = ldp * fabsf(cos_c) / (dist * dist);
                  const float wl = cdpa * (X.mis_vm + vsf(B.vs, vs, VS_DVCM) + vsf(B.vs, vs, VS_DVC) * lrp);
                  const float wc = ldpa * (X.mis_vm + cdvcm + cdvc * crp);
                  const float w = 1.f / (wl + 1.f + wc);
                  const V3 res = mul(cf, lf) * w * G;
                  if (!black(res)) {
                    shoot = true;
                    sdir = normalize(dir);
                    stgt = hp + dir * dist;
                    sval = mul(mul(cthr, vld3(B.vs, vs, VS_THR)), res);
                  }
                }
              }
            }
          }
        }
        const int si = wave_append(&A.sc->sq[slot + 1], shoot);
        if (shoot) {
          st3(Q.o, cap, si, hp);
          st3(Q.d, cap, si, sdir);
          st3(Q.tgt, cap, si, stgt);
          st3(Q.val, cap, si, sval);
          Q.cut[si] = occl_cut(hp, stgt, dot(stgt - hp, sdir));
          Q.meta[si] = (SQ_CONN << 30) | p;
          Q.pix[si] = pix;
        }
      }
    }
    const int ei = wave_append(&A.sc->ext[slot + 1], ext);
    if (ext) {
      st3(B.q_o[nxt], P, ei, e_o);
      st3(B.q_d[nxt], P, ei, e_d);
      B.q_path[nxt][ei] = p;
    }
  }
}

// Vertex merging of one camera-pass step's queued vertices (:265-276): one
// lane per query, outside the vertex kernel so that its long, divergent range
// scans run at the occupancy of a small kernel.
__device__ __forceinline__ void vcm_merge_body(const VcmArgs& X, int slot, int bid, int nblk) {
  const VcmBuf::Mq& M = X.V.mq[slot & 1];
  const int n = X.a.sc->mq[slot], P = X.a.P;
  const int gstride = nblk * blockDim.x;
  const int nround = (n + gstride - 1) / gstride * gstride;
  for (int j = bid * blockDim.x + threadIdx.x; j < nround; j += gstride) {
    unsigned found = 0, merged = 0;
    if (j < n) {
      Bsdf b;
      b.mat = M.mat[j];
      b.fr = frame_from_z(ld3(M.n, P, j));
      b.wi = ld3(M.wi, P, j);
      b.pd = M.pd[j];
      b.pg = M.pg[j];
      b.cont = M.cont[j];
      const V3 acc = vcm_merge(X, b, ld3(M.hp, P, j), M.len[j], M.dvcm[j], M.dvm[j], found, merged);
      film_add(X.a.film, M.pix[j], mul(ld3(M.thr, P, j), acc) * X.vm_norm);
    }
    const unsigned long long fs = wave_sum(found), ms = wave_sum(merged);
    if (lane_id() == 0 && fs) {
      atomicAdd(&X.a.ctr->vm_found, fs);
      atomicAdd(&X.a.ctr->vm_merged, ms);
    }
  }
}

// One camera-pass step after its traversal, three disjoint parts in one launch:
// blocks [0, nres) resolve the step's shadow rays, [nres, nres + nsh) shade its
// camera vertices (queueing merge queries into mq[slot & 1]), the rest merge
// the queries the previous step queued (mq[(slot - 1) & 1]; vertex merging
// only adds to the film, so it need not finish before this step's traversal).
__global__ void __launch_bounds__(kShadeBlock) WR_SHADE_OCC k_vcm_camera_step(VcmGroup G_, int slot, int nres,
                                                                             int nsh) {
  const VcmArgs& X = G_.a[blockIdx.y];
  const int bx = static_cast<int>(blockIdx.x);
  if (bx < nres) sq_resolve_body(X.a, slot, bx, nres);
  else if (bx < nres + nsh) vcm_camera_shade_body(X, slot, bx - nres, nsh);
  else vcm_merge_body(X, slot - 1, bx - nres - nsh, gridDim.x - nres - nsh);
}
