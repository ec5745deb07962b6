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

// A ray queue: SoA origins / directions [3][cap], count on device, optional
// per-ray [tmin, tmax], and the (t, prim) outputs.
struct RayQueue {
  const float* o3;
  const float* d3;
  int cap;
  const int* count;
  const float* tmin;
  const float* tmax;
  float* out_t;
  int* out_prim;
};

// Per-wave LDS scratch of the traversal (one wave per workgroup, 64 lanes):
//   stack  [depth][64] x (node, tmin, tmax)
//   rays   origin, direction, [tmin, tmax], current best t of every lane
//   leaf   exclusive prefix of leaf sizes and first ref of every lane
//   res    kPairBatch pair results (t, or NaN for "no hit")
constexpr int kPairBatch = 256;
__host__ __device__ constexpr size_t trace_lds_bytes(int depth) {
  return size_t(4) * (3 * size_t(depth) * 64 + 9 * 64 + 2 * 64 + kPairBatch);
}

// Persistent closest-hit traversal over up to two ray queues (one wave per
// workgroup); queue `qa` is fetched first (the long shadow rays start early and
// overlap the extension rays of `qb` instead of forming a tail of their own).
//
// KDtreeAccel::traverse semantics per ray; the SIMT structure is GPU-specific:
//   * while-while: every live lane first descends inner nodes until it stands on
//     a leaf, then the wave tests all its leaves, then every lane pops;
//   * leaf pairs spread over the wave: the (ray, triangle) pairs of the 64 leaves
//     are numbered by a prefix sum and tested 64 at a time, so the expensive
//     triangle test runs at full SIMD width however unequal the leaves are; each
//     lane then walks ITS results in leaf order applying the reference's
//     order-dependent rule `cmp(t - best) < 0` (first found wins);
//   * lanes that finish their ray take the next one from a global counter (one
//     atomic per wave per refill), so a wave stays full until the queues drain.
template <bool COUNT, bool SPH>
__device__ __forceinline__ void trace_queue(const DevScene& S, const RayQueue& qa, const RayQueue& qb, int* fetch,
                                            uint32_t* lds, TraceCounters& ctr) {
  const int lane = __lane_id();
  const int depth = S.max_stack;
  uint32_t* stk_node = lds + lane;
  float* stk_tmin = reinterpret_cast<float*>(lds + depth * 64) + lane;
  float* stk_tmax = reinterpret_cast<float*>(lds + 2 * depth * 64) + lane;
  float* ray = reinterpret_cast<float*>(lds + 3 * depth * 64);  // [9][64]
  int* seg_start = reinterpret_cast<int*>(ray + 9 * 64);
  uint32_t* seg_first = reinterpret_cast<uint32_t*>(seg_start + 64);
  float* res = reinterpret_cast<float*>(seg_first + 64);
  const int na = qa.count ? *qa.count : 0;
  const int n = na + (qb.count ? *qb.count : 0);
  bool inb = false;      // the lane's ray comes from qb
  int r = -1;            // ray held by this lane (-1: none)
  bool pool = true;      // wave-uniform: queue not yet exhausted
  V3 o = v3(0.f, 0.f, 0.f), d = o, inv = o;
  float tmin = 0.f, tmax = 0.f, t_best = WR_INF, rtmax = WR_INF;
  int best = -1, sp = 0;
  uint32_t node = 0;
  for (;;) {
    // ---- refill idle lanes
    if (pool) {
      const bool idle = r < 0;
      const unsigned long long m = __ballot(idle);
      if (m) {
        const int leader = __ffsll(static_cast<unsigned long long>(m)) - 1;
        int base = 0;
        if (lane == leader) base = atomicAdd(fetch, __popcll(m));
        base = __shfl(base, leader);
        const int idx = base + __popcll(m & ((1ull << lane) - 1ull));
        if (idle && idx < n) {
          inb = idx >= na;
          const RayQueue& q = inb ? qb : qa;
          r = inb ? idx - na : idx;
          o = v3(q.o3[r], q.o3[q.cap + r], q.o3[2 * q.cap + r]);
          d = v3(q.d3[r], q.d3[q.cap + r], q.d3[2 * q.cap + r]);
          const float rtmin = q.tmin ? q.tmin[r] : 0.f;
          rtmax = q.tmax ? q.tmax[r] : WR_INF;
          t_best = WR_INF;
          best = -1;
          sp = 0;
          node = 0;
          if (!box_hit(S.root_l, S.root_r, o, d, tmin, tmax) || rtmax < tmin) {
            q.out_t[r] = WR_INF;
            q.out_prim[r] = -1;
            r = -1;
          } else {
            inv = v3(1.f / d.x, 1.f / d.y, 1.f / d.z);
            ray[0 * 64 + lane] = o.x;
            ray[1 * 64 + lane] = o.y;
            ray[2 * 64 + lane] = o.z;
            ray[3 * 64 + lane] = d.x;
            ray[4 * 64 + lane] = d.y;
            ray[5 * 64 + lane] = d.z;
            ray[6 * 64 + lane] = rtmin;
            ray[7 * 64 + lane] = rtmax;
          }
        }
        if (__ballot(idle && idx >= n)) pool = false;
      }
    }
    const bool act = r >= 0;
    if (!__ballot(act)) {
      if (!pool) break;
      continue;
    }
    // ---- descend to a leaf (KDtreeAccel.cpp:325-358)
    uint32_t first = 0, count = 0;
    if (act) {
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
          stk_node[sp * 64] = farc;
          stk_tmin[sp * 64] = t;
          stk_tmax[sp * 64] = tmax;
          ++sp;
          node = nearc;
          tmax = t;
        }
        nd = S.nodes[node];
      }
      first = nd.x;
      count = nd.y >> 2;
      if (COUNT) {
        ++ctr.leaves;
        ctr.refs += count;
      }
    }
    // ---- leaf phase (:359-373): number the wave's (ray, ref) pairs
    int incl = static_cast<int>(count);
    for (int off = 1; off < 64; off <<= 1) {
      const int v = __shfl_up(incl, off);
      if (lane >= off) incl += v;
    }
    const int excl = incl - static_cast<int>(count);
    const int total = __shfl(incl, 63);
    seg_start[lane] = excl;
    seg_first[lane] = first;
    ray[8 * 64 + lane] = t_best;
    int best_ref = -1;
    for (int base = 0; base < total; base += kPairBatch) {
      const int lim = min(total - base, kPairBatch);
      __syncthreads();
      for (int j = lane; j < lim; j += 64) {
        const int g = base + j;
        int L = 0;  // largest lane whose segment starts at or before g (owns pair g)
#pragma unroll
        for (int step = 32; step > 0; step >>= 1) {
          const int cand = L + step;
          if (cand <= 63 && seg_start[cand] <= g) L = cand;
        }
        const uint32_t ref = seg_first[L] + static_cast<uint32_t>(g - seg_start[L]);
        const V3 ro = v3(ray[0 * 64 + L], ray[1 * 64 + L], ray[2 * 64 + L]);
        const V3 rd = v3(ray[3 * 64 + L], ray[4 * 64 + L], ray[5 * 64 + L]);
        const float rmin = ray[6 * 64 + L], rmax = ray[7 * 64 + L], rbest = ray[8 * 64 + L];
        const float2 c = S.ref_c[ref];
        const int prim = __float_as_int(c.y);
        float t = __int_as_float(0x7fc00000);  // NaN: no hit
        float th;
        bool h;
        if (!SPH || prim >= 0) {
          h = tri_test(S.ref_a[ref], S.ref_b[ref], c.x, ro, rd, rmin, rmax, rbest, th);
        } else {
          h = sph_hit(S, -prim - 1, ro, rd, rmin, rmax, th);
        }
        if (h) t = th;
        res[j] = t;
      }
      __syncthreads();
      if (act) {  // this lane's pairs of the batch, in leaf order
        const int k0 = max(excl, base), k1 = min(excl + static_cast<int>(count), base + lim);
        for (int k = k0; k < k1; ++k) {
          const float t = res[k - base];
          if (t == t && cmpf(t - t_best) < 0) {
            t_best = t;
            best_ref = static_cast<int>(first) + (k - excl);
          }
        }
      }
    }
    if (act) {
      if (best_ref >= 0) {
        const int prim = __float_as_int(S.ref_c[best_ref].y);
        best = (!SPH || prim >= 0) ? prim : -prim - 1;
      }
      // ---- pop (:375-383); tmin only changes here, so the `ray.tmax < tmin`
      // check of :323 is evaluated after every pop
      bool done = true;
      if (sp > 0) {
        --sp;
        node = stk_node[sp * 64];
        tmin = stk_tmin[sp * 64];
        tmax = stk_tmax[sp * 64];
        done = rtmax < tmin;
      }
      if (done) {
        (inb ? qb : qa).out_t[r] = t_best;
        (inb ? qb : qa).out_prim[r] = best;
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
