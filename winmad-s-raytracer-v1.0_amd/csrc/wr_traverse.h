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
#include <type_traits>
#include "wr_devmath.h"

namespace wrd {

struct DevScene {
  // node i as (self, left child) and (right child): one pair of loads resolves
  // two levels of the descent.  self/child words: inner (split bits,
  // right << 2 | axis) with left = i + 1; leaf (first ref, count << 2 | 3)
  const uint4* nrec;
  const uint2* nrec_r;
  // three levels per record (WR_NODE_LEVELS = 3): node i's word, its two
  // children's and its four grandchildren's, 64 bytes:
  //   [4i] = (self, L)  [4i+1] = (R, LL)  [4i+2] = (LR, RL)  [4i+3] = (RR, 0)
  const uint4* nrec3;
  const float4* ref_a;
  const float4* ref_b;
  const float2* ref_c;
  const int* prim_mat;
  const int* prim_type;     // 0 triangle, 1 sphere
  const float4* prim_tri;   // (A, B, C, D) per primitive (winner normal)
  const float2* prim_tri2;  // (E, F)
  const float4* prim_sph;   // (cx, cy, cz, r)
  // the same per primitive as one 32-byte record (the vertex kernels gather it
  // by primitive): (A, B, C, D), (E, F, matId bits, type bits)
  const float4* prim_rec;
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
  uint32_t inner, leaves, refs, tests;
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
  // one combined screen predicate and one branch (divergent early returns cost
  // exec-mask bookkeeping per test); NaN estimates compare false and fall through
  const float ad = fabsf(denom);
  const float r = __builtin_amdgcn_rcpf(denom);
  const float ba = bnum * r, ga = gnum * r, ta = tnum * r;
  const float mb = 1e-5f * fabsf(ba), mg = 1e-5f * fabsf(ga), mt = 1e-5f * fabsf(ta);
  const bool drop = (ba < -WR_EPS - mb) | (ba > 1.f + mb) | (ga < -WR_EPS - mg) |
                    (ba + ga > 1.f + (mb + mg) + 1e-6f) | (ta < WR_EPS - mt) | (ta > rtmax + mt) |
                    (ta - t_best > -WR_EPS + (mt + 1e-5f * fabsf(t_best)));
  if (drop & (ad > 1e-30f) & (ad < 1e30f)) return false;
  // the reference's test, exactly (its early outs only skip work, never change
  // the outcome, so all three quotients are formed here)
  const float beta = bnum / denom;
  const float gamma = gnum / denom;
  const float t = tnum / denom;
  const bool beta_ok = !(cmpf(beta) < 0 || beta > 1.f);
  const bool gamma_ok = !(cmpf(gamma) < 0 || beta + gamma > 1.f);
  const bool t_ok = cmpf(t) > 0 && !(t < rtmin || t > rtmax);
  const bool ok = beta_ok && gamma_ok && t_ok;
  t_out = t;
  return ok;
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

// Hard rays taken off a render pipeline's critical path (WR_TRACE_BVH, BDPT
// extension rays; wr_render.hip, "deferred hard rays").  k_fast_resolve copies
// a deferrable ray it cannot settle into this list and marks its queue entry
// pending (out_prim = kPendingPrim: the vertex kernel skips it).  A side stream
// settles the list (k_late_hard) and shades the paths one step later.  A path
// is deferred at most once per pass (the queue's late_bit of delayed[path]).
// Records: tie entries at [0, n[0]), scan entries at [cap / 2, cap / 2 +
// n[1]), n = the queue's late_n (the step's counters).
struct LateList {
  int cap;
  const int* path;    // the queue's path index per entry
  uint8_t* delayed;   // per path (local index)
  float *o3, *d3;     // [3][cap]
  float* t1;          // the search's smallest hit (input of the resolution)
  int* p1;
  int* pth;           // path of the record
  int* tie;           // scan entries: a near-tie on a many-leaf primitive
  float* t;           // the settled answer (k_late_hard)
  int* prim;
};
constexpr int kPendingPrim = -2;

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
  // shadow rays (Scene::occluded, scene.cpp:55-69): a ray may stop as soon as
  // its best hit is below cut[k] -- see occl_cut.  nullptr / -INF: closest hit
  const float* cut;
  // deferrable hard rays (device pointer; nullptr: settled in the launch)
  const LateList* late;
  int* late_n;   // [2] this step's late-list counts
  int late_bit;  // the pass's bit of LateList::delayed
  // a second count (nullptr: none): the queue holds *count + *count2 rays (the
  // overlapped BDPT schedule: the light pass's rays, then the camera pass's)
  const int* count2;
};

// Scene::occluded(p1, dir, p2) answers "unoccluded" iff the closest hit is
// missing or its point equals p2 within EPS per component.  Best only
// decreases during the traversal, so once a hit at t < cut is accepted the
// closest hit's point lies at least cut's margin short of p2 along the ray --
// farther than EPS in the ray's largest direction component (>= 1/sqrt(3)),
// with room for the float error of both points (<= 7 * 2^-24 * M) -- and the
// answer is "occluded" whatever the rest of the traversal finds.  Exact: the
// occlusion result equals the full traversal's; only the returned (t, prim)
// can differ, and nothing else reads them.
__device__ __forceinline__ float occl_cut(V3 o, V3 tgt, float dist) {
  const float m = fmaxf(fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(tgt.x))),
                        fmaxf(fmaxf(fabsf(tgt.y), fabsf(tgt.z)), dist));
  return dist - 2.f * (WR_EPS + 1e-6f * m);
}

// The queues of one traversal launch, fetched in order (the shadow / aux queue
// of an iteration first: its long rays start early and overlap the extension
// rays instead of forming a tail of their own).
#ifndef WR_MAX_QUEUES
#define WR_MAX_QUEUES 4
#endif
constexpr int kMaxQueues = WR_MAX_QUEUES;
struct TraceQueues {
  RayQueue q[kMaxQueues];
  int n;
};

// Per-wave LDS scratch of the traversal (one wave per workgroup, 64 lanes):
//   stack  [depth][64] tmin (float) + [depth][64] node (u16 when the tree has
//          <= 65536 nodes, NARROW; u32 otherwise)
//   rays   per lane 8 floats (o.xyz, d.x | d.yz, tmin, tmax) + best t   (AoS, b128 reads)
//   leaf   per lane: exclusive prefix of its pair count; per leaf id
//          (lane * kLeavesPerRound + i): first ref and its offset in the lane's pairs
//   own    leaf id of each pair of the batch (bytes)
//   owner  per ray: (min hit key, smallest prim at it) and (min hit key, largest
//          prim at it) as 64-bit atomics, + a flag for hits in (min, min + 2 EPS]
#ifndef WR_PAIR_BATCH
#define WR_PAIR_BATCH 256
#endif
constexpr int kPairBatch = WR_PAIR_BATCH;  // multiple of 256
#ifndef WR_NODE_LEVELS
// tree levels resolved per dependent record load (2, 3 or 4); 3 over 2: C2
// 892 -> 911 Mrays/s; 4 (128-byte records, exact) loses 13-16 % on C2/C3
#define WR_NODE_LEVELS 3
#endif
static_assert(kPairBatch % 256 == 0, "the owner-table scan covers 4 bytes per lane per 256 slots");
static_assert(WR_NODE_LEVELS >= 2 && WR_NODE_LEVELS <= 4, "node record levels: 2, 3 or 4");
constexpr int kRecLevels = WR_NODE_LEVELS < 3 ? 3 : WR_NODE_LEVELS;  // nrec3 layout
constexpr int kRecU4 = kRecLevels == 4 ? 8 : 4;                      // uint4 per record
#ifndef WR_LEAVES_PER_ROUND
#define WR_LEAVES_PER_ROUND 4
#endif
// the walk of a round ends once every live lane holds WR_LEAVES_WAIT leaves
// (lanes that get there first walk on, up to kLeavesPerRound).  With 3-level
// node records and 16 pipelines, 1 beats 2 (C2 +1.8 %, C3 +0.9 %, VCM +1.7 %,
// C4 -0.7 %) and 3 (C2 -3.5 %); 3 leaves per round lose 5 %, 2 lose 8 %.
#ifndef WR_LEAVES_WAIT
#define WR_LEAVES_WAIT 1
#endif
#ifndef WR_PAIRS_IN_FLIGHT
#define WR_PAIRS_IN_FLIGHT 2
#endif
#ifndef WR_PAIRS_IN_FLIGHT_WIDE
#define WR_PAIRS_IN_FLIGHT_WIDE 4  // 32-bit-index trees (> 65536 nodes): C4 +4 % over 2
#endif
// (ray, triangle) records requested per lane per trip; torus-sized trees: 4
// costs C2 1.5 %
constexpr int kPairsInFlight = WR_PAIRS_IN_FLIGHT;
constexpr int kPairsInFlightWide = WR_PAIRS_IN_FLIGHT_WIDE;
static_assert(kPairBatch % (64 * kPairsInFlight) == 0 && kPairBatch % (64 * kPairsInFlightWide) == 0,
              "a batch is whole trips");
constexpr int kLeavesPerRound = WR_LEAVES_PER_ROUND;
#ifndef WR_RAY_GRAB
#define WR_RAY_GRAB 128  // 64: C2 -0.8 %, 256: -1 %
#endif
constexpr int kRayGrab = WR_RAY_GRAB;  // queue indices a wave reserves per atomic (>= 64)  // leaves a lane may collect per round
constexpr int kLeavesWait = WR_LEAVES_WAIT;           // the walk runs until every lane has this many
// leaf ids lane * kLeavesPerRound + i are stored in the byte-wide owner table
static_assert(64 * kLeavesPerRound <= 256, "owner table holds leaf ids in bytes: kLeavesPerRound <= 4");
static_assert(kLeavesWait >= 1 && kLeavesWait <= kLeavesPerRound, "kLeavesWait in 1..kLeavesPerRound");
// Per-ray mailbox of recently tested primitives (direct-mapped by prim id):
// a (ray, primitive) pair tested before -- the KD build duplicates straddling
// triangles into every leaf they touch (torus: 2.88 refs per triangle) -- is
// skipped.  A repeat cannot change the result: it yields the same t, and the
// earlier test either set best <= t or was rejected against a best that has
// only decreased since, so `cmp(t - best) < 0` fails again.  Measured on torus
// BDPT rays: 60 % of the reference's tests are repeats; an 8-entry mailbox
// catches 40 % of all tests (C4: 3,248 -> 819 tests per ray).  It is OFF (0):
// the filter pass (primitive load + mailbox per slot, then compaction) costs
// about what the skipped tests save -- the pair phase is bound by its
// dependent L2 round trips, not by the triangle arithmetic -- and the extra LDS
// lowers occupancy.  Measured (Mrays/s, 8 pipelines): C2 871 -> 702 (m8),
// C4 36.3 -> 34.5 (m8); scripts/build_variant.sh m8 -DWR_MAILBOX=8.
#ifndef WR_MAILBOX
#define WR_MAILBOX 0
#endif
constexpr int kMail = WR_MAILBOX;
static_assert((kMail & (kMail - 1)) == 0, "mailbox size: power of two");
// Where a pair's test reads its ray.  Default: the owner's 8-float record and
// best, kept in LDS (2.3 KB per wave).  DENSE: ds_bpermute from the owner
// lane's registers -- no LDS storage, so a torus wave fits the 8 KB of 20
// waves/CU (with <= 96 VGPRs) at the price of 9 permutes per pair.
__host__ __device__ constexpr size_t trace_lds_bytes(int depth, bool narrow, bool dense = false) {
  return size_t(depth) * 64 * (narrow ? 6 : 8) +
         size_t(4) * ((dense ? 0 : 8 * 64 + 64) + kLeavesPerRound * 64 + kLeavesPerRound * (narrow ? 32 : 64) +
                      kPairBatch / 4 + 4 * 64 + 16 + kMail * 64 + (kMail > 0 ? kPairBatch / 2 : 0));
}
// Ray prefetch: a lane holds the record of its next ray in registers, loaded
// one round ahead, so a refill does not wait on the queue load (never in the
// DENSE layout: no register room at 96 VGPRs).  Exact, but OFF: it costs C2
// 889 -> 828, VCM 796 -> 753, C4 41.4 -> 38.3 Mrays/s (127 VGPRs; vector
// loads retire in order, so the walk's first wait also waits for the prefetch).
#ifndef WR_RAY_PREFETCH
#define WR_RAY_PREFETCH 0
#endif
// value of v in lane `src` (all lanes of the wave active)
__device__ __forceinline__ float lane_get(float v, int src) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(v)));
}

// Persistent closest-hit traversal over the ray queues of one launch (one wave
// per workgroup), fetched in queue order.
//
// KDtreeAccel::traverse semantics per ray; the SIMT structure is GPU-specific:
//   * the reference never stops early (it walks to the far end of the root box
//     whatever it has hit), so a ray's sequence of leaves does not depend on its
//     hits.  Each round, every lane walks to its next leaf; lanes that get there
//     first walk on to a second one while the others are still descending
//     (up to kLeavesPerRound), and the round's leaves are tested together;
//   * leaf pairs spread over the wave: the (ray, triangle) pairs of the round
//     are numbered by a prefix sum and tested 64 at a time, so the triangle test
//     runs at full SIMD width however unequal the leaves are;
//   * first-found-wins (`cmp(t - best) < 0` in leaf order, :363-372) per ray
//     over its pairs of the round, concatenated in leaf order;
//   * lanes that finish their ray take the next one from a global counter (one
//     atomic per wave per refill), so a wave stays full until the queues drain.
// Wave64 inclusive scans on DPP (no LDS round trip, unlike __shfl_up's
// ds_bpermute): Hillis-Steele inside each 16-lane row (row_shr 1, 2, 4, 8;
// out-of-row sources read 0), then row 0's total into row 1 and row 2's into
// row 3 (row_bcast:15), then rows 0-1's total into rows 2-3 (row_bcast:31).
// Values must be >= 0 for the max scan (0 is its identity).  Full wave only.
__device__ __forceinline__ int wave_scan_add(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
  return v;
}
__device__ __forceinline__ int wave_scan_max(int v) {
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true));
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true));
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true));
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true));
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false));
  return v;
}
// value of lane - 1 (0 in lane 0): DPP wave_shr:1
__device__ __forceinline__ int wave_shr1(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xf, 0xf, true); }

// monotone int key of a float (signed-int order == float order, -0 < +0)
__device__ __forceinline__ int order_key(float f) {
  const int b = __float_as_int(f);
  return b >= 0 ? b : b ^ 0x7fffffff;
}
__device__ __forceinline__ float order_val(int k) { return __int_as_float(k >= 0 ? k : k ^ 0x7fffffff); }

// Diagnostic build only (STAMP = true, WR_TRACE_STAMPS=1): s_memtime at the
// phase boundaries, per-wave sums added to stamps[0..5] = refill, leaf walk,
// leaf setup, pair tests, first-found-wins decision, result write.  Never
// compiled into timed runs.
__device__ __forceinline__ uint64_t stamp_now() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

template <bool COUNT, bool SPH, bool NARROW, bool STAMP = false, bool CUT = false, bool DENSE = false>
__device__ __forceinline__ void trace_queue(const DevScene& S, const TraceQueues& Q, int* fetch,
                                            uint32_t* lds, TraceCounters& ctr,
                                            unsigned long long* stamps = nullptr) {
  uint64_t acc[6] = {0, 0, 0, 0, 0, 0};
  uint64_t ts = 0;
  if constexpr (STAMP) ts = stamp_now();
#define WR_STAMP(k)                       \
  if constexpr (STAMP) {                  \
    const uint64_t now_ = stamp_now();    \
    acc[k] += now_ - ts;                  \
    ts = now_;                            \
  }
  const int lane = __lane_id();
  const int depth = S.max_stack;
  using NodeIdx = typename std::conditional<NARROW, uint16_t, uint32_t>::type;
  float* stk_tmin = reinterpret_cast<float*>(lds) + lane;
  NodeIdx* stk_node = reinterpret_cast<NodeIdx*>(lds + depth * 64) + lane;
  // Stack entries hold (node, tmin) only: tmax changes only at a push
  // (tmax = t), so entry k's tmax is entry k-1's tmin and entry 0's is the
  // root-box tmax -- exactly the floats the reference's todo[] would hold.
  float4* ray4 = reinterpret_cast<float4*>(reinterpret_cast<char*>(lds) + size_t(depth) * 64 * (NARROW ? 6 : 8));
  float* rbest = reinterpret_cast<float*>(ray4 + (DENSE ? 0 : 2 * 64));  // [64]
  uint32_t* leaf_first = reinterpret_cast<uint32_t*>(rbest + (DENSE ? 0 : 64));  // [64 * kLeavesPerRound]
  // first pair of each leaf in the round's numbering (lane-local during the walk)
  using PairIdx = typename std::conditional<NARROW, uint16_t, uint32_t>::type;
  PairIdx* leaf_off = reinterpret_cast<PairIdx*>(leaf_first + kLeavesPerRound * 64);  // [64 * kLeavesPerRound]
  uint8_t* own = reinterpret_cast<uint8_t*>(leaf_off + kLeavesPerRound * 64);  // [kPairBatch]
  uint32_t* own32 = reinterpret_cast<uint32_t*>(own);
  unsigned long long* olo = reinterpret_cast<unsigned long long*>(own + kPairBatch);  // [64] key << 32 | prim
  unsigned long long* ohi = olo + 64;  // [64] (INT_MAX - key) << 32 | prim
  uint8_t* onear = reinterpret_cast<uint8_t*>(ohi + 64);  // [64]
  int* mail = reinterpret_cast<int*>(onear + 64);  // [64][kMail] prim keys tested per ray (0: empty)
  uint16_t* cslot = reinterpret_cast<uint16_t*>(mail + 64 * kMail);  // [kPairBatch] kept slots of the batch
  int qend[kMaxQueues];  // queue i holds launch indices [qend[i-1], qend[i])
  {
    int acc = 0;
#pragma unroll
    for (int i = 0; i < kMaxQueues; ++i) {
      // (capped: a shadow queue's appends past its capacity were dropped, BdptBuf)
      if (i < Q.n && Q.q[i].count) acc += min(*Q.q[i].count + (Q.q[i].count2 ? *Q.q[i].count2 : 0), Q.q[i].cap);
      qend[i] = acc;
    }
  }
  const int n = qend[kMaxQueues - 1];
  // waves past the ones the rays need leave before touching the cursor (trace_fast)
  if (static_cast<int>(blockIdx.x) * kRayGrab >= n) return;
  int qi = 0;            // queue of the lane's ray
  // field of queue q (selects, no dynamic indexing of the kernel argument)
  auto selq = [&](int q, auto field) {
    auto v = field(Q.q[0]);
#pragma unroll
    for (int i = 1; i < kMaxQueues; ++i)
      if (q == i) v = field(Q.q[i]);
    return v;
  };
  auto sel = [&](auto field) { return selq(qi, field); };
  // queue and index within it of launch index idx
  auto locate = [&](int idx, int& q, int& rr) {
    q = 0;
    int q0 = 0;
#pragma unroll
    for (int i = 0; i < kMaxQueues - 1; ++i)
      if (idx >= qend[i]) {
        q = i + 1;
        q0 = qend[i];
      }
    rr = idx - q0;
  };
  int r = -1;            // ray held by this lane (-1: none)
  bool pool = true;      // wave-uniform: queue not yet exhausted
  int pb = 0, pe = 0;    // wave-uniform: reserved queue indices [pb, pe)
  bool more = false;     // the lane's ray has nodes left to visit
  V3 o = v3(0.f, 0.f, 0.f), d = o, inv = o;
  float tmin = 0.f, tmax = 0.f, t_best = WR_INF, rtmax = WR_INF, root_tmax = 0.f, rcut = -WR_INF;
  float rtmin_v = 0.f, screen0 = WR_INF;  // the ray's tmin; its best at round start
  int best = -1, sp = 0;
  uint32_t node = 0;
  constexpr bool PF = WR_RAY_PREFETCH != 0 && !DENSE;
  constexpr int PIF = (NARROW || DENSE) ? kPairsInFlight : kPairsInFlightWide;  // DENSE: no room at 96 VGPRs
  int pidx = -1;  // PF: launch index of the prefetched ray (-1: none)
  V3 po = v3(0.f, 0.f, 0.f), pd = po;
  float ptn = 0.f, ptx = WR_INF, pcut = -WR_INF;
  // queue indices come from the wave's reservation [pb, pe), topped up kRayGrab
  // at a time (one global atomic per kRayGrab rays, not per refill)
  auto reserve = [&](bool want) -> int {
    const unsigned long long m = __ballot(want);
    const int need = __popcll(m);
    const int rank = __popcll(m & ((1ull << lane) - 1ull));
    int idx = pb + rank;
    if (need == 0) return idx;
    if (pe - pb < need) {
      int got = 0;
      if (lane == 0) got = atomicAdd(fetch, kRayGrab);
      got = __builtin_amdgcn_readlane(got, 0);
      const int rem = pe - pb;
      if (rank >= rem) idx = got + (rank - rem);
      pb = got + (need - rem);
      pe = got + kRayGrab;
    } else {
      pb += need;
    }
    return idx;
  };
  // PF: reserve the next ray of the lanes in `want` and issue its loads
  auto prefetch = [&](bool want) {
    const int idx = reserve(want);
    if (want) {
      pidx = -1;
      if (idx < n) {
        int q, rr;
        locate(idx, q, rr);
        pidx = idx;
        const float* o3 = selq(q, [](const RayQueue& x) { return x.o3; });
        const float* d3 = selq(q, [](const RayQueue& x) { return x.d3; });
        const int cap = selq(q, [](const RayQueue& x) { return x.cap; });
        const float* tmn = selq(q, [](const RayQueue& x) { return x.tmin; });
        const float* tmx = selq(q, [](const RayQueue& x) { return x.tmax; });
        po = v3(o3[rr], o3[cap + rr], o3[2 * cap + rr]);
        pd = v3(d3[rr], d3[cap + rr], d3[2 * cap + rr]);
        ptn = tmn ? tmn[rr] : 0.f;
        ptx = tmx ? tmx[rr] : WR_INF;
        if constexpr (CUT) {
          const float* cutp = selq(q, [](const RayQueue& x) { return x.cut; });
          pcut = cutp ? cutp[rr] : -WR_INF;
        }
      }
    }
    if (__ballot(want && idx >= n)) pool = false;
  };
  if constexpr (PF) prefetch(true);
  // one level of KDtreeAccelNode descent (:325-358) from inner node `at` (word w)
  auto step = [&](uint2 w, uint32_t at) -> uint32_t {
    if (COUNT) ++ctr.inner;
    const uint32_t axis = w.y & 3u;
    const float split = __uint_as_float(w.x);
    const float oa = axis == 0 ? o.x : (axis == 1 ? o.y : o.z);
    const float da = axis == 0 ? d.x : (axis == 1 ? d.y : d.z);
    const float ia = axis == 0 ? inv.x : (axis == 1 ? inv.y : inv.z);
    const float t = (split - oa) * ia;
    // predicates combined bitwise: one branch (the push) instead of a branch
    // per short-circuit
    const bool below = (oa < split) | ((oa == split) & (da <= 0));
    const uint32_t left = at + 1, right = w.y >> 2;
    const uint32_t nearc = below ? left : right, farc = below ? right : left;
    const bool go_near = (t > tmax) | (t <= 0);
    const bool go_far = !go_near & (t < tmin);
    if (!go_near & !go_far) {
      stk_node[sp * 64] = static_cast<NodeIdx>(farc);
      stk_tmin[sp * 64] = t;
      ++sp;
      tmax = t;
    }
    return go_far ? farc : nearc;
  };
  // t of one (ray, primitive) pair, NaN when Triangle::hit / Sphere::hit reject it
  // or (triangles) when it cannot beat `screen`, the ray's best at round start
  auto pair_t = [&](float4 a, float4 b, float2 c, V3 ro, V3 rd, float rt0, float rt1, float screen) -> float {
    const int prim = __float_as_int(c.y);
    float th = __int_as_float(0x7fc00000);
    bool h;
    if (!SPH || prim >= 0) {
      h = tri_test(a, b, c.x, ro, rd, rt0, rt1, screen, th);
    } else {
      h = sph_hit(S, -prim - 1, ro, rd, rt0, rt1, th);
    }
    return h ? th : __int_as_float(0x7fc00000);
  };
  for (;;) {
    // ---- refill idle lanes
    if (PF ? (pool || __ballot(pidx >= 0) != 0) : pool) {
      const bool idle = r < 0;
      if (__ballot(idle)) {
        int idx;
        bool take;
        if constexpr (PF) {  // the prefetched ray; the next one is requested below
          idx = pidx;
          take = idle && pidx >= 0;
        } else {
          idx = reserve(idle);
          take = idle && idx < n;
        }
        if (take) {
          locate(idx, qi, r);
          if constexpr (PF) {
            o = po;
            d = pd;
            rtmin_v = ptn;
            rtmax = ptx;
            if constexpr (CUT) rcut = pcut;
          } else {
            const float* o3 = sel([](const RayQueue& x) { return x.o3; });
            const float* d3 = sel([](const RayQueue& x) { return x.d3; });
            const int cap = sel([](const RayQueue& x) { return x.cap; });
            const float* tmn = sel([](const RayQueue& x) { return x.tmin; });
            const float* tmx = sel([](const RayQueue& x) { return x.tmax; });
            o = v3(o3[r], o3[cap + r], o3[2 * cap + r]);
            d = v3(d3[r], d3[cap + r], d3[2 * cap + r]);
            rtmin_v = tmn ? tmn[r] : 0.f;
            rtmax = tmx ? tmx[r] : WR_INF;
            if constexpr (CUT) {
              const float* cutp = sel([](const RayQueue& x) { return x.cut; });
              rcut = cutp ? cutp[r] : -WR_INF;
            }
          }
          const float rtmin = rtmin_v;
          t_best = WR_INF;
          best = -1;
          sp = 0;
          node = 0;
          const bool boxed = box_hit(S.root_l, S.root_r, o, d, tmin, tmax);
          root_tmax = tmax;
          more = true;
          if (!boxed || rtmax < tmin) {  // :312-313, and the :323 check before the root
            sel([](const RayQueue& x) { return x.out_t; })[r] = WR_INF;
            sel([](const RayQueue& x) { return x.out_prim; })[r] = -1;
            r = -1;
            more = false;
          } else {
            inv = v3(1.f / d.x, 1.f / d.y, 1.f / d.z);
            if constexpr (!DENSE) {
              ray4[2 * lane] = make_float4(o.x, o.y, o.z, d.x);
              ray4[2 * lane + 1] = make_float4(d.y, d.z, rtmin, rtmax);
            }
#pragma unroll
            for (int k = 0; k < kMail; ++k) mail[lane * kMail + k] = 0;
          }
        }
        if constexpr (PF) {
          if (pool) prefetch(take);
          else if (take) pidx = -1;
        } else if (__ballot(idle && idx >= n)) {
          pool = false;
        }
      }
    }
    WR_STAMP(0)
    const bool act = r >= 0;
    if (!__ballot(act)) {
      if (!pool && !(PF && __ballot(pidx >= 0))) break;  // PF: prefetched rays still to take
      continue;
    }
    // ---- walk to the next leaves (:321-358, pops :375-383).  One record pair
    // per iteration resolves up to two levels; the walk goes on while any lane
    // still has no leaf this round.
    // the round's leaves of this lane: first ref and pair offset, in LDS
    int nl = 0, count = 0;
    while (__ballot(more && nl < kLeavesWait)) {
      if (more && nl < kLeavesPerRound) {
#if WR_NODE_LEVELS == 4
        // 15 entries in 128 bytes: up to four descent steps per record
        const uint4* rp = S.nrec3 + 8 * static_cast<size_t>(node);
        const uint4 q0 = rp[0], q1 = rp[1], q2 = rp[2], q3 = rp[3], q4 = rp[4], q5 = rp[5], q6 = rp[6], q7 = rp[7];
        asm volatile("" : : "v"(q0.y), "v"(q1.x), "v"(q2.x), "v"(q3.x), "v"(q4.x), "v"(q5.x), "v"(q6.x), "v"(q7.x));
        uint2 nd = make_uint2(q0.x, q0.y);
        bool leaf = (nd.y & 3u) == 3u;
        if (!leaf) {
          const uint32_t a0 = node;
          node = step(nd, a0);
          const bool b1 = node != a0 + 1;  // went right
          nd = b1 ? make_uint2(q1.x, q1.y) : make_uint2(q0.z, q0.w);  // e2 : e1
          leaf = (nd.y & 3u) == 3u;
          if (!leaf) {
            const uint32_t a1 = node;
            node = step(nd, a1);
            const bool b2 = node != a1 + 1;
            // e3 = q1.zw, e4 = q2.xy, e5 = q2.zw, e6 = q3.xy
            nd = b1 ? (b2 ? make_uint2(q3.x, q3.y) : make_uint2(q2.z, q2.w))
                    : (b2 ? make_uint2(q2.x, q2.y) : make_uint2(q1.z, q1.w));
            leaf = (nd.y & 3u) == 3u;
            if (!leaf) {
              const uint32_t a2 = node;
              node = step(nd, a2);
              const bool b3 = node != a2 + 1;
              // e7 = q3.zw, e8 = q4.xy, e9 = q4.zw, e10 = q5.xy, e11 = q5.zw,
              // e12 = q6.xy, e13 = q6.zw, e14 = q7.xy
              const uint2 l0 = b3 ? make_uint2(q4.x, q4.y) : make_uint2(q3.z, q3.w);
              const uint2 l1 = b3 ? make_uint2(q5.x, q5.y) : make_uint2(q4.z, q4.w);
              const uint2 l2 = b3 ? make_uint2(q6.x, q6.y) : make_uint2(q5.z, q5.w);
              const uint2 l3 = b3 ? make_uint2(q7.x, q7.y) : make_uint2(q6.z, q6.w);
              nd = b1 ? (b2 ? l3 : l2) : (b2 ? l1 : l0);
              leaf = (nd.y & 3u) == 3u;
              if (!leaf) node = step(nd, node);
            }
          }
        }
#elif WR_NODE_LEVELS == 3
        const uint4* rp = S.nrec3 + 4 * static_cast<size_t>(node);
        const uint4 q0 = rp[0], q1 = rp[1], q2 = rp[2], q3 = rp[3];
        asm volatile("" : : "v"(q0.y), "v"(q1.x), "v"(q2.x), "v"(q3.x));
        uint2 nd = make_uint2(q0.x, q0.y);
        bool leaf = (nd.y & 3u) == 3u;
        if (!leaf) {
          const uint32_t at = node;
          node = step(nd, at);
          const bool lft = node == at + 1;
          nd = lft ? make_uint2(q0.z, q0.w) : make_uint2(q1.x, q1.y);
          leaf = (nd.y & 3u) == 3u;
          if (!leaf) {
            const uint32_t c = node;
            node = step(nd, c);
            const bool l2 = node == c + 1;
            nd = lft ? (l2 ? make_uint2(q1.z, q1.w) : make_uint2(q2.x, q2.y))
                     : (l2 ? make_uint2(q2.z, q2.w) : make_uint2(q3.x, q3.y));
            leaf = (nd.y & 3u) == 3u;
            if (!leaf) node = step(nd, node);
          }
        }
#else
        const uint4 q = S.nrec[node];
        const uint2 qr = S.nrec_r[node];
        // keep both loads in flight together: otherwise the second is sunk into
        // the inner-node branch and its latency is paid after the first's
        asm volatile("" : : "v"(q.y), "v"(qr.x), "v"(qr.y));
        uint2 nd = make_uint2(q.x, q.y);
        bool leaf = (nd.y & 3u) == 3u;
        if (!leaf) {
          const uint32_t at = node;
          node = step(nd, at);
          nd = node == at + 1 ? make_uint2(q.z, q.w) : qr;
          leaf = (nd.y & 3u) == 3u;
          if (!leaf) node = step(nd, node);
        }
#endif
        if (leaf) {
          leaf_first[lane * kLeavesPerRound + nl] = nd.x;
          leaf_off[lane * kLeavesPerRound + nl] = static_cast<PairIdx>(count);
          count += static_cast<int>(nd.y >> 2);
          ++nl;
          if (COUNT) {
            ++ctr.leaves;
            ctr.refs += nd.y >> 2;
          }
          // pop; tmin only changes here, so the `ray.tmax < tmin` check of :323
          // is evaluated after every pop
          if (sp > 0) {
            --sp;
            node = stk_node[sp * 64];
            tmin = stk_tmin[sp * 64];
            tmax = sp > 0 ? stk_tmin[(sp - 1) * 64] : root_tmax;
            more = !(rtmax < tmin);
          } else {
            more = false;
          }
        }
      }
    }
    WR_STAMP(1)
    // ---- leaf phase (:359-373): number the wave's (ray, ref) pairs
    const int incl = wave_scan_add(count);
    const int excl = incl - count;
    const int total = __builtin_amdgcn_readlane(incl, 63);
#pragma unroll
    for (int i = 0; i < kLeavesPerRound; ++i)  // nl <= kLeavesPerRound
      if (i < nl) leaf_off[lane * kLeavesPerRound + i] += static_cast<PairIdx>(excl);
    if constexpr (!DENSE) rbest[lane] = t_best;
    screen0 = t_best;
    // ref of pair k of the round, k in this lane's range [excl, excl + count)
    auto own_ref = [&](int k) -> uint32_t {
      int i = 0;
#pragma unroll
      for (int x = 1; x < kLeavesPerRound; ++x)
        if (x < nl && k >= static_cast<int>(leaf_off[lane * kLeavesPerRound + x])) i = x;
      return leaf_first[lane * kLeavesPerRound + i] +
             static_cast<uint32_t>(k - static_cast<int>(leaf_off[lane * kLeavesPerRound + i]));
    };
    for (int base = 0; base < total; base += kPairBatch) {
      const int lim = min(total - base, kPairBatch);
      const int k0 = max(excl, base), k1 = min(excl + count, base + lim);
      __syncthreads();
#pragma unroll
      for (int k = 0; k < kPairBatch / 256; ++k) own32[lane * (kPairBatch / 256) + k] = 0u;
      olo[lane] = ~0ull;
      ohi[lane] = 0ull;
      onear[lane] = 0;
      __syncthreads();
      // leaf table: each leaf marks its first slot in the batch, then a max-scan
      // over the batch in slot order (leaf ids increase with the slot)
      if (k0 < k1) {
        int s0 = static_cast<int>(leaf_off[lane * kLeavesPerRound]);
#pragma unroll
        for (int i = 0; i < kLeavesPerRound; ++i) {
          if (i < nl) {
            const int s1 = i + 1 < nl ? static_cast<int>(leaf_off[lane * kLeavesPerRound + i + 1]) : excl + count;
            const int a0 = max(s0, base), a1 = min(s1, base + lim);
            if (a0 < a1) own[a0 - base] = static_cast<uint8_t>(lane * kLeavesPerRound + i);
            s0 = s1;
          }
        }
      }
      __syncthreads();
      {
        // lane covers slots [lane * kPairBatch / 64, (lane + 1) * kPairBatch / 64)
        constexpr int kW = kPairBatch / 256;
        uint32_t m[4 * kW];
        uint32_t run = 0u;
#pragma unroll
        for (int k = 0; k < kW; ++k) {
          const uint32_t w = own32[lane * kW + k];
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            run = max(run, (w >> (8 * b)) & 0xffu);
            m[4 * k + b] = run;
          }
        }
        run = static_cast<uint32_t>(wave_scan_max(static_cast<int>(run)));
        const uint32_t prev = static_cast<uint32_t>(wave_shr1(static_cast<int>(run)));
#pragma unroll
        for (int k = 0; k < kW; ++k)
          own32[lane * kW + k] = max(m[4 * k], prev) | (max(m[4 * k + 1], prev) << 8) |
                                 (max(m[4 * k + 2], prev) << 16) | (max(m[4 * k + 3], prev) << 24);
      }
      __syncthreads();
      WR_STAMP(2)
      // Mailbox filter: each slot of the batch (j = lane + 64 k, in slot order,
      // i.e. leaf order per ray) reads its primitive and checks the ray's
      // mailbox; the pairs to test are compacted into cslot[0, nk).  The first
      // slot of a (ray, primitive) to be checked is kept and marks the
      // mailbox; later ones -- this batch or later -- are dropped.
      int nk = lim;
      if constexpr (kMail > 0) {
        nk = 0;
        uint32_t fref[kPairBatch / 64];
        int fown[kPairBatch / 64];
        float fprim[kPairBatch / 64];
#pragma unroll
        for (int k = 0; k < kPairBatch / 64; ++k) {
          const int j = min(lane + 64 * k, lim - 1);
          const int id = own[j];
          fown[k] = id / kLeavesPerRound;
          fref[k] = leaf_first[id] + static_cast<uint32_t>(base + j - static_cast<int>(leaf_off[id]));
        }
#pragma unroll
        for (int k = 0; k < kPairBatch / 64; ++k) fprim[k] = (lane + 64 * k < lim) ? S.ref_c[fref[k]].y : 0.f;
#pragma unroll
        for (int k = 0; k < kPairBatch / 64; ++k) {
          bool keep = false;
          if (lane + 64 * k < lim) {
            const int key = __float_as_int(fprim[k]) ^ static_cast<int>(0x80000000u);  // != 0 (empty)
            int* slot = mail + fown[k] * kMail + (key & (kMail - 1));
            keep = *slot != key;
            if (keep) *slot = key;
          }
          const unsigned long long m = __ballot(keep);
          if (keep) cslot[nk + __popcll(m & ((1ull << lane) - 1ull))] = static_cast<uint16_t>(lane + 64 * k);
          nk += __popcll(m);
        }
        __syncthreads();
      }
      // PIF pairs per lane per trip: c, c + 64, ... of the kept
      // slots; all their records are requested before the first test.  A lane
      // keeps the t of its own pairs ((c - lane) / 64) in registers.
      float tv[kPairBatch / 64];
#pragma unroll
      for (int k = 0; k < kPairBatch / 64; ++k) tv[k] = __int_as_float(0x7fc00000);  // NaN: no hit
#pragma unroll
      for (int tr = 0; tr < kPairBatch / (64 * PIF); ++tr) {
        const int c0 = lane + 64 * PIF * tr;
        if (64 * PIF * tr >= nk) break;  // wave-uniform
        uint32_t ref[PIF];
        int owner[PIF];
#pragma unroll
        for (int u = 0; u < PIF; ++u) {
          const int c = min(c0 + 64 * u, max(nk - 1, 0));
          const int j = kMail > 0 ? static_cast<int>(cslot[c]) : c;
          const int id = own[j];
          owner[u] = id / kLeavesPerRound;
          ref[u] = leaf_first[id] + static_cast<uint32_t>(base + j - static_cast<int>(leaf_off[id]));
        }
        float2 rc[PIF];
        float4 ra[PIF], rb[PIF];
#pragma unroll
        for (int u = 0; u < PIF; ++u) {
          rc[u] = S.ref_c[ref[u]];
          ra[u] = S.ref_a[ref[u]];
          rb[u] = S.ref_b[ref[u]];
        }
        // the owners' rays (converged wave: every source lane is active)
        float4 gx[PIF], gy[PIF];
        float gs[PIF];
        if constexpr (DENSE) {
#pragma unroll
          for (int u = 0; u < PIF; ++u) {
            const int L = owner[u];
            gx[u] = make_float4(lane_get(o.x, L), lane_get(o.y, L), lane_get(o.z, L), lane_get(d.x, L));
            gy[u] = make_float4(lane_get(d.y, L), lane_get(d.z, L), lane_get(rtmin_v, L), lane_get(rtmax, L));
            gs[u] = lane_get(screen0, L);
          }
        }
#pragma unroll
        for (int u = 0; u < PIF; ++u) {
          if (c0 + 64 * u >= nk) break;
          if (COUNT) ++ctr.tests;
          const int L = owner[u];
          const float4 x = DENSE ? gx[u] : ray4[2 * L], y = DENSE ? gy[u] : ray4[2 * L + 1];
          const float scr = DENSE ? gs[u] : rbest[L];
          const int prim = __float_as_int(rc[u].y);
          const float t = pair_t(ra[u], rb[u], rc[u], v3(x.x, x.y, x.z), v3(x.w, y.x, y.y), y.z, y.w, scr);
          if (t == t) {  // t > EPS > 0: the order key is the float's bits
            const unsigned long long key = static_cast<uint32_t>(__float_as_int(t));
            const unsigned long long pr = static_cast<uint32_t>((!SPH || prim >= 0) ? prim : -prim - 1);
            atomicMin(olo + L, (key << 32) | pr);
            atomicMax(ohi + L, ((0x7fffffffull - key) << 32) | pr);
          }
          tv[tr * PIF + u] = t;
        }
      }
      __syncthreads();
      // flag owners with a hit in (min, min + 2 EPS]
#pragma unroll
      for (int k = 0; k < kPairBatch / 64; ++k) {
        const int c = lane + 64 * k;
        const float t = tv[k];
        if (c < nk && t == t) {
          const int L = own[kMail > 0 ? static_cast<int>(cslot[c]) : c] / kLeavesPerRound;
          const float m = __int_as_float(static_cast<int>(olo[L] >> 32));
          if (t != m && t - m <= 2.f * WR_EPS) onear[L] = 1;
        }
      }
      __syncthreads();
      WR_STAMP(3)
      // first-found-wins (cmp(t - best) < 0, in leaf order, :367).  With m the
      // round's smallest hit (every hit t >= m, float rounding is monotone):
      //  * cmp(m - best) >= 0: no hit of the round can be taken -- no change;
      //  * else, if every other hit is more than 2 EPS above m and m is a single
      //    primitive (repeats of a triangle met in two leaves give the same t),
      //    m is taken when reached and nothing after it can replace it;
      //  * otherwise (a near-tie between different primitives) this owner
      //    replays its pairs in order, re-testing them (same inputs and screen
      //    => the same t as above).
      if (act && k0 < k1) {
        const unsigned long long lo = olo[lane];
        const float m = __int_as_float(static_cast<int>(lo >> 32));
        if (lo != ~0ull && cmpf(m - t_best) < 0) {
          const int pmin = static_cast<int>(lo & 0xffffffffull);
          const bool decided = onear[lane] == 0 && pmin == static_cast<int>(ohi[lane] & 0xffffffffull);
          if (decided) {
            t_best = m;
            best = pmin;
          }
          if (!decided) {
            const float screen = DENSE ? screen0 : rbest[lane];
            const float rtmin = DENSE ? rtmin_v : ray4[2 * lane + 1].z;
            for (int k = k0; k < k1; ++k) {
              const uint32_t ref = own_ref(k);
              const float2 c = S.ref_c[ref];
              const float t = pair_t(S.ref_a[ref], S.ref_b[ref], c, o, d, rtmin, rtmax, screen);
              if (t == t && cmpf(t - t_best) < 0) {
                t_best = t;
                const int cp = __float_as_int(c.y);
                best = (!SPH || cp >= 0) ? cp : -cp - 1;
              }
            }
          }
          if (CUT && t_best < rcut) more = false;  // occlusion settled (occl_cut)
        }
      }
      WR_STAMP(4)
    }
    if (act) {
      if (!more) {
        sel([](const RayQueue& x) { return x.out_t; })[r] = t_best;
        sel([](const RayQueue& x) { return x.out_prim; })[r] = best;
        r = -1;
      }
    }
    WR_STAMP(5)
  }
#undef WR_STAMP
  if constexpr (STAMP) {
    if (lane == 0)
      for (int k = 0; k < 6; ++k) atomicAdd(stamps + k, static_cast<unsigned long long>(acc[k]));
  }
}

// Scene::intersect re-runs hit() on the winner (scene.cpp:25-27); from (t, prim)
// the intersection record is rebuilt with the same float operations.
struct Hit {
  float t;
  V3 p, n;
  int inside, mat;
};
// The geometric normal of primitive prim at p (Triangle::hit / Sphere::hit):
// rebuild_hit's operations, for a stored vertex (wr_bdpt.h stored_bsdf).
__device__ __forceinline__ V3 prim_normal(const DevScene& S, int prim, V3 p) {
  const float4 r0 = S.prim_rec[2 * static_cast<size_t>(prim)], r1 = S.prim_rec[2 * static_cast<size_t>(prim) + 1];
  if (__float_as_int(r1.w) != 0) {
    const float4 cs = S.prim_sph[prim];
    return normalize(p - v3(cs.x, cs.y, cs.z));
  }
  return normalize(cross(v3(r0.x, r0.y, r0.z), v3(r0.w, r1.x, r1.y)));
}
__device__ __forceinline__ Hit rebuild_hit(const DevScene& S, int prim, float t, V3 o, V3 d) {
  Hit h;
  h.t = t;
  h.p = o + d * t;
  const float4 r0 = S.prim_rec[2 * static_cast<size_t>(prim)], r1 = S.prim_rec[2 * static_cast<size_t>(prim) + 1];
  h.mat = __float_as_int(r1.z);
  if (__float_as_int(r1.w) != 0) {
    float4 cs = S.prim_sph[prim];
    h.n = normalize(h.p - v3(cs.x, cs.y, cs.z));
    float tt;
    int in = 0;
    sph_hit(S, prim, o, d, 0.f, WR_INF, tt, &in);
    h.inside = in;
  } else {
    // (p1 - p0) x (p2 - p0) == (p0 - p1) x (p0 - p2) exactly
    h.n = normalize(cross(v3(r0.x, r0.y, r0.z), v3(r0.w, r1.x, r1.y)));
    h.inside = (dot(d, h.n) < WR_EPS) ? 0 : 1;
  }
  return h;
}

}  // namespace wrd
