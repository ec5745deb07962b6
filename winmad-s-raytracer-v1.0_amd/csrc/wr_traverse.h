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

// Triangle::hit (triangle.cpp:22-87) inside the closest-hit loop.
// The reference forms beta, gamma and t with three correctly rounded divisions
// by `denom`; here the quotients are first estimated with one v_rcp_f32 and a
// candidate is dropped early only when the estimate proves the exact test would
// drop it too (margins 1e-5 relative, ~40x the estimate's error):
//   beta  < -EPS or > 1,  gamma < -EPS,  beta + gamma > 1,  t <= EPS,  t > tmax,
//   or t cannot improve the current best (cmp(t - best) < 0 impossible) -- a hit
//   that does not improve has no effect in the reference's leaf loop either.
// Survivors take the exact divisions, so accept / reject and t are bit-exact.
// Estimates are used only for |denom| in (1e-30, 1e30); NaN estimates fall through.
__device__ __forceinline__ bool tri_test(float4 a, float4 b, float f, V3 o, V3 d, float rtmin, float rtmax,
                                         float t_best, float& t_out) {
  const float A = a.w, B = b.x, C = b.y, D = b.z, E = b.w, F = f;
  const float G = d.x, H = d.y, I = d.z;
  const float J = a.x - o.x, K = a.y - o.y, L = a.z - o.z;
  const float EIHF = E * I - H * F;
  const float GFDI = G * F - D * I;
  const float DHEG = D * H - E * G;
  const float denom = A * EIHF + B * GFDI + C * DHEG;
  const float bnum = J * EIHF + K * GFDI + L * DHEG;
  const float AKJB = A * K - J * B;
  const float JCAL = J * C - A * L;
  const float BLKC = B * L - K * C;
  const float gnum = I * AKJB + H * JCAL + G * BLKC;
  const float tnum = -(F * AKJB + E * JCAL + D * BLKC);
  const float ad = fabsf(denom);
  if (ad > 1e-30f && ad < 1e30f) {
    const float r = __builtin_amdgcn_rcpf(denom);
    const float ba = bnum * r, ga = gnum * r, ta = tnum * r;
    const float mb = 1e-5f * fabsf(ba), mg = 1e-5f * fabsf(ga), mt = 1e-5f * fabsf(ta);
    if (ba < -WR_EPS - mb || ba > 1.f + mb) return false;
    if (ga < -WR_EPS - mg || ba + ga > 1.f + (mb + mg) + 1e-6f) return false;
    if (ta < WR_EPS - mt || ta > rtmax + mt) return false;
    if (ta - t_best > -WR_EPS + (mt + 1e-5f * fabsf(t_best))) return false;
  }
  const float beta = bnum / denom;
  if (cmpf(beta) < 0 || beta > 1.f) return false;
  const float gamma = gnum / denom;
  if (cmpf(gamma) < 0 || beta + gamma > 1.f) return false;
  const float t = tnum / denom;
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

// Persistent closest-hit traversal over a ray queue (one wave per workgroup).
//
// KDtreeAccel::traverse semantics per ray; the SIMT structure is GPU-specific:
//   * while-while: every live lane first descends inner nodes until it stands on
//     a leaf, then all lanes test their leaves together, then pop -- so the
//     expensive leaf loop runs with the wave full instead of interleaved with
//     inner-node steps of other lanes;
//   * lanes that finish their ray take the next one from a global counter (one
//     atomic per wave per refill), so a wave stays full until the queue drains;
//   * leaf references are prefetched one ahead (the 40-byte record of the next
//     triangle is in flight while the current one is tested).
// `rtmin3 / rtmax3` (optional) give per-ray [tmin, tmax]; default [0, INF].
template <bool COUNT, bool SPH>
__device__ __forceinline__ void trace_queue(const DevScene& S, const float* __restrict__ o3,
                                            const float* __restrict__ d3, int cap, int n,
                                            const float* __restrict__ rtmin_a, const float* __restrict__ rtmax_a,
                                            float* __restrict__ out_t, int* __restrict__ out_prim, int* fetch,
                                            uint32_t* stk_node, float* stk_tmin, float* stk_tmax, int stride,
                                            TraceCounters& ctr) {
  int r = -1;            // ray held by this lane (-1: none)
  bool pool = true;      // wave-uniform: queue not yet exhausted
  V3 o = v3(0.f, 0.f, 0.f), d = o, inv = o;
  float tmin = 0.f, tmax = 0.f, t_best = WR_INF, rtmin = 0.f, rtmax = WR_INF;
  int best = -1, sp = 0;
  uint32_t node = 0;
  for (;;) {
    // ---- refill idle lanes
    if (pool) {
      const bool idle = r < 0;
      if (__ballot(idle)) {
        const unsigned long long m = __ballot(idle);
        const int lane = __lane_id();
        const int leader = __ffsll(static_cast<unsigned long long>(m)) - 1;
        int base = 0;
        if (lane == leader) base = atomicAdd(fetch, __popcll(m));
        base = __shfl(base, leader);
        const int idx = base + __popcll(m & ((1ull << lane) - 1ull));
        if (idle) {
          if (idx < n) {
            r = idx;
            o = v3(o3[idx], o3[cap + idx], o3[2 * cap + idx]);
            d = v3(d3[idx], d3[cap + idx], d3[2 * cap + idx]);
            rtmin = rtmin_a ? rtmin_a[idx] : 0.f;
            rtmax = rtmax_a ? rtmax_a[idx] : WR_INF;
            t_best = WR_INF;
            best = -1;
            sp = 0;
            node = 0;
            if (!box_hit(S.root_l, S.root_r, o, d, tmin, tmax) || rtmax < tmin) {
              out_t[idx] = WR_INF;
              out_prim[idx] = -1;
              r = -1;
            } else {
              inv = v3(1.f / d.x, 1.f / d.y, 1.f / d.z);
            }
          }
        }
        if (__ballot(idle && idx >= n)) pool = false;
      }
    }
    if (!__ballot(r >= 0)) {
      if (!pool) break;
      continue;
    }
    if (r >= 0) {
      // ---- descend to a leaf (KDtreeAccel.cpp:325-358)
      uint2 nd = S.nodes[node];
      while ((nd.y & 3u) != 3u) {
        if (COUNT) ++ctr.inner;
        const uint32_t axis = nd.y & 3u;
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
        nd = S.nodes[node];
      }
      // ---- leaf: every primitive in objlist order, first-found wins (:359-373)
      const uint32_t first = nd.x, count = nd.y >> 2;
      if (COUNT) {
        ++ctr.leaves;
        ctr.refs += count;
      }
      if (count) {
        const uint32_t end = first + count;
        float4 a = S.ref_a[first], b = S.ref_b[first];
        float2 c = S.ref_c[first];
        for (uint32_t i = first; i < end;) {
          const float4 ca = a, cb = b;
          const float2 cc = c;
          ++i;
          const uint32_t j = i < end ? i : end - 1;
          a = S.ref_a[j];
          b = S.ref_b[j];
          c = S.ref_c[j];
          const int prim = __float_as_int(cc.y);
          float t;
          bool h;
          if (!SPH || prim >= 0) {
            h = tri_test(ca, cb, cc.x, o, d, rtmin, rtmax, t_best, t);
          } else {
            h = sph_hit(S, -prim - 1, o, d, rtmin, rtmax, t);
          }
          if (h && cmpf(t - t_best) < 0) {
            t_best = t;
            best = (!SPH || prim >= 0) ? prim : -prim - 1;
          }
        }
      }
      // ---- pop (:375-383); tmin only changes here, so the `ray.tmax < tmin`
      // check of :323 is evaluated after every pop
      bool done = true;
      if (sp > 0) {
        --sp;
        node = stk_node[sp * stride];
        tmin = stk_tmin[sp * stride];
        tmax = stk_tmax[sp * stride];
        done = rtmax < tmin;
      }
      if (done) {
        out_t[r] = t_best;
        out_prim[r] = best;
        r = -1;
      }
    }
  }
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
