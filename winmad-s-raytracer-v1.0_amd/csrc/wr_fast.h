// Verified-BVH closest hit on gfx950 (see wr_bvh.h for why its answers equal the
// reference's KDtreeAccel::traverse, src/scene/KDtreeAccel.cpp:309-388).
//
// Two launches over the same ray queues as k_trace:
//   k_trace_fast  every ray gets a closest-hit search over a binary BVH
//                 (64-byte nodes holding both children's boxes, 48-byte
//                 triangle records).  It keeps the smallest hit (t1, p1) --
//                 written as the ray's result -- and the smallest hit of any
//                 other triangle, t2, when within t1 + 2 EPS (per launch index
//                 into a scratch array).
//   k_fast_resolve one ray per lane, all lanes on the same code path
//                 (the rare cases below the first are listed and finished by a
//                 third launch, k_fast_hard):
//                 * no hit anywhere -> miss (the reference tests a subset);
//                 * cmp(t2 - t1) > 0 and p1 lies in a KD leaf the reference's
//                   traversal reaches (replay of its near / far rule down the
//                   leaf's root path, kd_member) -> (t1, p1) stands;
//                 * a near-tie (another hit within EPS of t1): every hit up to
//                   t1 + 3 EPS is collected by a second BVH search
//                   (bvh_collect), and the reference's first-found-wins rule is
//                   run over those it reaches, in the order it reaches them
//                   (resolve_tie);
//                 * otherwise (t1's triangle not reached, more near hits than
//                   the list holds, or hits in the band where unseen hits could
//                   interfere) the lane walks the reference's KD tree for the
//                   ray (kd_walk: KDtreeAccel::traverse statement for
//                   statement) and overwrites the result.
// Triangle tests are Triangle::hit exactly (tri_test: the rcp screen only skips
// tests whose exact outcome is a reject or a t beyond the window), so t1 is the
// reference's float.  The membership replay runs in its own launch because at
// the end of a lane's search it ran with a handful of lanes active (measured:
// 13 % VALU lane utilisation, most of it there).
#pragma once
#include <type_traits>
#include "wr_bvh.h"

namespace wrd {

struct FastScene {
  const float4* nodes;  // 4 per wrf::BNode (tie resolution's collection)
  const float4* nodes4;  // 4 per wrf::BNode4Q / 8 per wrf::BNode4 (wrf::BNode4S: the search when wide == 4)
  const float4* nodes8;  // 8 per wrf::BNode8 (the search when wide == 8)
  int wide;              // the search tree's width: 2 (nodes), 4 (nodes4) or 8 (nodes8)
  const float4* tris;   // 3 per wrf::TriRec
  const int* prim_leaf_off;
  const int* prim_leaf;
  const int* prim_leaf_pos;
  const uint2* path;
  const int* node_path;  // KD leaf node -> path record offset
  const float4* node_cell;  // 2 per KD node: cell lo, hi
  const float4* prim_rec;   // 8 per primitive (wrf::PrimRec): its first four leaves' cells and records
  V3 lo, hi;  // union of the (grown) triangle / sphere boxes
  // spheres in the tree (0: triangles only).  Their boxes are grown for ray
  // origins inside [org_lo, org_hi] (wr_bvh.cpp, sphere_grow); a ray from
  // outside takes the KD walk
  int sph;
  V3 org_lo, org_hi;
  int depth;   // stack entries of the KD walks and tie resolution (k_fast_hard, k_fast_verify)
  int sdepth;  // stack entries of the BVH search (k_trace_fast): the BVH's depth + 1
  int walk_wave;  // 1: the one-ray-per-wave resolutions walk the KD tree with the whole wave (kd_walk_wave)
  int pair;       // near-ties use the search's pair record: 2 = pair list (one per lane), 1 = tie list only, 0 = never
  int diag;   // WR_BVH_DIAG (measurement only): 1 = skip the KD walks, 8 = skip the replays, 16 = skip k_fast_resolve,
              // 32 = skip k_fast_hard, 64 its scan list, 128 its tie list (all wrong answers);
              // 2 = KD walk for every tie, 256 = every ray to k_fast_hard's KD walk (exact: a test of the walks)
};

struct FastCounters {  // algorithmic work (count_work)
  uint32_t nodes, tests, replay, fallback;
  uint32_t kinner, kleaves, krefs;           // KD walks of the fallback rays
  uint32_t max_nodes, max_tests, long_rays;  // per-ray tail: max visits, rays > 256 nodes
  uint32_t fb_tie;                            // near-ties resolved by visit order
  uint32_t why[4];                            // KD walks: many-leaf candidate, no visited hit, crowd, band
  // latency tail (count_work, 100 MHz ticks): k_fast_resolve membership,
  // k_fast_hard tie resolution and KD walk -- max and sum per ray -- and the
  // rays whose membership test scanned a many-leaf primitive's whole list
  uint32_t mem_max, mem_sum, tie_max, tie_sum, walk_max, walk_sum, scans;
  // WR_TIE_SPLIT (diagnostic build): the tie resolutions' ticks in bvh_collect and in
  // the first-leaf searches, and their second collect passes
  uint32_t tie_col, tie_leaf, tie_pass2, scan_t, pair_used;
  // kd_walk_wave (count_work): walks, their rounds and nodes, and fall-backs
  // to the serial walk (work stack or hit list outgrown)
  uint32_t ww_walks, ww_rounds, ww_nodes, ww_over;
};

// Per wave: the stack columns, 8 bytes per entry and lane (BVH: link + entry t;
// KD walk: node + tmin).
__host__ __device__ constexpr size_t fast_lds_bytes(int depth) { return size_t(depth) * 64 * 8; }
// The search's stack: link (4 bytes) + entry t rounded down to bfloat16 (2
// bytes).  A rounded-down entry t only lets more subtrees through the pop test
// (t_entry <= bound), never fewer, so the search still reports every hit it
// must; 6 instead of 8 bytes per entry raise the waves per CU the LDS allows.
// The first kLdsStack entries live in LDS, deeper ones (rare) in a per-lane
// global spill area, so that the 4-wide tree's worst case (3 entries per
// level) does not set the LDS size and with it the waves per CU.
#ifndef WR_BVH_LDS_STACK
#define WR_BVH_LDS_STACK 64  // the binary tree: never spills
#endif
#ifndef WR_BVH4_LDS_STACK
#define WR_BVH4_LDS_STACK 12  // the 4-wide tree (12 / 16 / 24 measured alike)
#endif
// The search tree's width is chosen per scene (FastScene::wide: the 4-wide
// tree for scenes whose nodes outgrow the L2, wrf::kWide4MinTris); the
// stack's LDS part per width.  Can it outgrow the LDS columns?  Not for the
// binary tree (kMaxBvhDepth + 1 entries fit), so its push / pop carry no
// spill branch: a generic pointer select between LDS and the spill area made
// the compiler emit flat loads (vmcnt + lgkmcnt waits) on every pop.
#ifndef WR_POP_TOGETHER
#define WR_POP_TOGETHER 1
#endif
#ifndef WR_LEAF_SCHED
#define WR_LEAF_SCHED 1
#endif
template <int W>
struct SearchStack {
  // the 8-wide tree keeps 16 (a ray's stack outgrows 12 entries for 2e-4 of
  // torus rays, 16 for none in 10^5: scripts/bvh_cost.cpp)
  static constexpr int lds = W == 4 ? WR_BVH4_LDS_STACK : W == 8 ? 16 : WR_BVH_LDS_STACK;
  static constexpr bool spills =
      (W == 8 ? 7 * wrf::kMaxBvhDepth + 1 : W == 4 ? 3 * wrf::kMaxBvhDepth + 1 : wrf::kMaxBvhDepth + 1) > lds;
};
__host__ __device__ constexpr int search_lds_stack(int wide) {
  return wide == 4 ? SearchStack<4>::lds : wide == 8 ? SearchStack<8>::lds : SearchStack<2>::lds;
}
__host__ __device__ constexpr size_t search_lds_bytes(int depth, int wide) {
  return size_t(depth < search_lds_stack(wide) ? depth : search_lds_stack(wide)) * 64 * 6;
}
// spill entries per lane for a search stack of `depth` entries
__host__ __device__ constexpr size_t search_spill_entries(int depth, int wide) {
  return depth > search_lds_stack(wide) ? size_t(depth - search_lds_stack(wide)) : 0;
}
// Speculative leaves (Aila & Laine 2009): a lane that has found its leaf keeps
// descending inner nodes while other lanes still look for theirs, and the
// leaf is tested (postponed) with theirs.  Extra nodes visited under a stale
// (larger) bound only add hits beyond the window, never drop one inside it.
#ifndef WR_BVH_SPEC
#define WR_BVH_SPEC 1
#endif
#ifndef WR_TIE_SPLIT
#define WR_TIE_SPLIT 0  // diagnostic: time the tie resolution's phases (count_work)
#endif
#ifndef WR_TIE_PASS2_CAP
#define WR_TIE_PASS2_CAP 1  // resolve_tie's second collection bounded by m + 3 EPS (0: unbounded)
#endif
// the tie resolution's leaf searches: calls (WR_HARD_CALL=__noinline__) or inlined
#ifndef WR_HARD_CALL
#define WR_HARD_CALL __forceinline__  // calls: 560-752 B of scratch per lane
#endif
__device__ __forceinline__ uint16_t t_down16(float t) {
  return static_cast<uint16_t>(__float_as_uint(fmaxf(t, 0.f)) >> 16);  // truncation: down for t >= 0
}
__device__ __forceinline__ float t_up32(uint16_t h) { return __uint_as_float(static_cast<uint32_t>(h) << 16); }

__device__ __forceinline__ float clamp_inv(float x) { return fminf(fmaxf(1.f / x, -1e30f), 1e30f); }

// KDtreeAccel::traverse reaches the leaf whose root path is rec[1..n]: the
// near / far rule (:331-357) and the `ray.tmax < tmin` stop (:323), evaluated
// with the reference's floats along that one path.  (tmin, tmax) = root clip.
// The record is read 8 entries (4 x 16 bytes) per round trip.  `key` gets the
// leaf's place in the ray's visit order: bit 63 - k is set when the path takes
// the far child at depth k.  The walk visits a node's near subtree before its
// far one, so for two visited leaves the smaller key is visited first (their
// paths part at a node where one goes near, the other far).
__device__ __forceinline__ bool kd_reaches(const uint2* rec, V3 o, V3 d, V3 inv, float tmin, float tmax, float rtmax,
                                           uint32_t& steps, unsigned long long& key) {
  key = 0ull;
  const int n = static_cast<int>(rec[0].x);
  const uint4* R = reinterpret_cast<const uint4*>(rec + 4);  // after the header
  for (int base = 0;; base += 8) {
    uint4 q[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) q[u] = R[base / 2 + u];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = base + j + 1;
      if (k > n) return true;
      const uint2 e = (j & 1) ? make_uint2(q[j / 2].z, q[j / 2].w) : make_uint2(q[j / 2].x, q[j / 2].y);
      ++steps;
      const uint32_t axis = e.y & 3u;
      const bool right = (e.y & 4u) != 0u;
      const float split = __uint_as_float(e.x);
      const float oa = axis == 0 ? o.x : (axis == 1 ? o.y : o.z);
      const float da = axis == 0 ? d.x : (axis == 1 ? d.y : d.z);
      const float ia = axis == 0 ? inv.x : (axis == 1 ? inv.y : inv.z);
      const float t = (split - oa) * ia;
      const bool below = (oa < split) | ((oa == split) & (da <= 0));
      const bool is_near = right != below;  // near = left iff below
      if (!is_near) key |= 1ull << (63 - min(k - 1, 63));
      const bool go_near = (t > tmax) | (t <= 0);
      const bool go_far = !go_near & (t < tmin);
      if (go_near) {
        if (!is_near) return false;
      } else if (go_far) {
        if (is_near) return false;
      } else if (is_near) {
        tmax = t;
      } else {
        tmin = t;  // popped later with tmin = t: the :323 check
        if (rtmax < tmin) return false;
      }
    }
    if (base + 8 >= n) return true;
  }
}

// The KD leaf whose cell holds point p (descent by p's coordinates, three
// levels per 64-byte record): its node index.
__device__ __forceinline__ uint32_t kd_locate_node(const DevScene& S, V3 p) {
  uint32_t node = 0;
  for (;;) {
    const uint4* rp = S.nrec3 + 4 * static_cast<size_t>(node);
    const uint4 q0 = rp[0], q1 = rp[1], q2 = rp[2], q3 = rp[3];
    // entries: 0 self, 1 L, 2 R, 3 LL, 4 LR, 5 RL, 6 RR (two per uint4)
    const uint2 e[7] = {make_uint2(q0.x, q0.y), make_uint2(q0.z, q0.w), make_uint2(q1.x, q1.y),
                        make_uint2(q1.z, q1.w), make_uint2(q2.x, q2.y), make_uint2(q2.z, q2.w),
                        make_uint2(q3.x, q3.y)};
    int h = 0;
    uint32_t at = node;
#pragma unroll
    for (int lev = 0; lev < 3; ++lev) {
      const uint2 w = e[h];
      if ((w.y & 3u) == 3u) return at;
      const uint32_t axis = w.y & 3u;
      const float split = __uint_as_float(w.x);
      const float pa = axis == 0 ? p.x : (axis == 1 ? p.y : p.z);
      const bool right = !(pa < split);
      at = right ? (w.y >> 2) : at + 1;
      h = 2 * h + (right ? 2 : 1);
      if (lev == 2) node = at;
    }
  }
}

// Does the reference's walk reach a leaf whose cell holds a point of the ray,
// o + d t with 0 < t <= rtmax, with room to spare -- without replaying its
// path?  The walk hands each node's float interval [a, b] down to the child
// that contains the ray's points there.  With the point at distance > delta
// from every face of the cell (delta_axis = 1e-6 x (|faces| + 2 |o| + |t d|)),
// each split's t = (split - o) * (1 / d) lies on the correct side of t despite
// its rounding (< 3 ulp relative: (split - o) and 1 / d rounded, then the
// product), and so do the root clip's slab t's; so every decision on the
// leaf's path (:331-357) keeps t inside the interval it passes on, and the
// leaf is visited.  (The exact point o + d t is within 2 ulp of the computed
// p.)
__device__ __forceinline__ bool cell_holds_with_margin(uint4 h0, uint4 h1, V3 o, V3 d, float t, V3 p) {
  const float lx = __uint_as_float(h0.z), ly = __uint_as_float(h0.w), lz = __uint_as_float(h1.x);
  const float hx = __uint_as_float(h1.y), hy = __uint_as_float(h1.z), hz = __uint_as_float(h1.w);
  const float mx = 1e-6f * (fabsf(lx) + fabsf(hx) + 2.f * fabsf(o.x) + fabsf(t * d.x));
  const float my = 1e-6f * (fabsf(ly) + fabsf(hy) + 2.f * fabsf(o.y) + fabsf(t * d.y));
  const float mz = 1e-6f * (fabsf(lz) + fabsf(hz) + 2.f * fabsf(o.z) + fabsf(t * d.z));
  return p.x - lx > mx && hx - p.x > mx && p.y - ly > my && hy - p.y > my && p.z - lz > mz && hz - p.z > mz;
}

// The witness: the middle of the ray's stretch inside the cell (in (0, rtmax]).
__device__ __forceinline__ bool cell_crossed_with_margin(uint4 h0, uint4 h1, V3 o, V3 d, V3 binv, float rtmax) {
  const float x0 = (__uint_as_float(h0.z) - o.x) * binv.x, x1 = (__uint_as_float(h1.y) - o.x) * binv.x;
  const float y0 = (__uint_as_float(h0.w) - o.y) * binv.y, y1 = (__uint_as_float(h1.z) - o.y) * binv.y;
  const float z0 = (__uint_as_float(h1.x) - o.z) * binv.z, z1 = (__uint_as_float(h1.w) - o.z) * binv.z;
  const float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), 0.f));
  const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), rtmax));
  if (!(tn < tf)) return false;
  const float tw = 0.5f * (tn + tf);
  return tw > 0.f && cell_holds_with_margin(h0, h1, o, d, tw, o + d * tw);
}

// The witness for a cell given as six floats.
__device__ __forceinline__ bool box_crossed_with_margin(float lx, float ly, float lz, float hx, float hy, float hz, V3 o,
                                                        V3 d, V3 binv, float rtmax) {
  const uint4 h0 = make_uint4(0u, 0u, __float_as_uint(lx), __float_as_uint(ly));
  const uint4 h1 = make_uint4(__float_as_uint(lz), __float_as_uint(hx), __float_as_uint(hy), __float_as_uint(hz));
  return cell_crossed_with_margin(h0, h1, o, d, binv, rtmax);
}

// Can the reference's walk reach the KD leaf whose cell is (h0.zw, h1) (the
// header of its path record)?  False only when the ray's LINE misses the cell
// grown by delta_a = 1e-5 x (|lo_a| + |hi_a| + 2 |o_a|) on every axis.  A leaf is
// reached only if its walk interval [tmin, tmax] stays non-empty (each near /
// far step of :331-357 keeps tmin <= tmax), and the interval's ends are float
// crossings of the cell's own faces (the root box and the splits on its path),
// each within 3 ulp of the exact crossing; missing the grown cell leaves a gap
// between the exact crossings far wider than that.  Rays with a near-zero
// direction component are never pruned.  Nor are rays whose root interval
// (tmax0) is not positive: an origin outside the root box, the ray pointing
// away.  The walk still runs for them (only `ray.tmax < tmin` stops it), every
// split crossing is then behind the origin (t <= 0: the near child only, the
// interval unchanged), so it ends in leaves whose cells the line need not
// meet -- and Triangle::hit's EPS-fattened test can still hit a triangle there
// at t > 0 (a wall met just outside the box; 20 of 600 K plane-grazing
// Cornell-box rays, tests/native/cell_filter_check.cpp).
__device__ __forceinline__ bool cell_may_be_reached(uint4 h0, uint4 h1, V3 o, V3 d, float tmax0) {
  if (!(tmax0 > 0.f)) return true;
  if (!(fabsf(d.x) > 1e-20f && fabsf(d.y) > 1e-20f && fabsf(d.z) > 1e-20f)) return true;
  const float lx = __uint_as_float(h0.z), ly = __uint_as_float(h0.w), lz = __uint_as_float(h1.x);
  const float hx = __uint_as_float(h1.y), hy = __uint_as_float(h1.z), hz = __uint_as_float(h1.w);
  const float mx = 1e-5f * (fabsf(lx) + fabsf(hx) + 2.f * fabsf(o.x)) + 1e-30f;
  const float my = 1e-5f * (fabsf(ly) + fabsf(hy) + 2.f * fabsf(o.y)) + 1e-30f;
  const float mz = 1e-5f * (fabsf(lz) + fabsf(hz) + 2.f * fabsf(o.z)) + 1e-30f;
  const float ix = 1.f / d.x, iy = 1.f / d.y, iz = 1.f / d.z;
  const float x0 = (lx - mx - o.x) * ix, x1 = (hx + mx - o.x) * ix;
  const float y0 = (ly - my - o.y) * iy, y1 = (hy + my - o.y) * iy;
  const float z0 = (lz - mz - o.z) * iz, z1 = (hz + mz - o.z) * iz;
  const float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
  const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
  return !(tn > tf);  // NaN: kept
}

// The membership replays (kd_member, scan_rays) skip leaves whose cell the
// ray's line misses, as the tie resolution does (WR_SCAN_CELL_FILTER=0: off).
#ifndef WR_SCAN_CELL_FILTER
#define WR_SCAN_CELL_FILTER 1
#endif
// Is the primitive whose KD leaves are prim_leaf[lb, lb + ln) tested by the
// reference's traversal of this ray?  kMember / kNotMember, or kScan: a
// many-leaf primitive whose located leaf proves nothing, left to the scan
// waves of k_fast_hard.  WR_RESOLVE_SCAN=1: such primitives are scanned here,
// by the lane (one leaf after another).
#ifndef WR_RESOLVE_SCAN
#define WR_RESOLVE_SCAN 0
#endif
constexpr int kNotMember = 0, kMember = 1, kScan = 2;
#ifndef WR_MEMBER_REFS
#define WR_MEMBER_REFS 0  // 1: kd_member tests the located leaf's references instead of a binary search of p1's leaf list (measured alike)
#endif
__device__ __forceinline__ int kd_member(const DevScene& S, const FastScene& F, int lb, int ln, V3 o, V3 d,
                                         float rtmax, float t_hit, uint32_t& steps, int p1) {
  float tmin, tmax;
  if (!box_hit(S.root_l, S.root_r, o, d, tmin, tmax) || rtmax < tmin) return kNotMember;  // :312-313, :323
  const V3 inv = v3(1.f / d.x, 1.f / d.y, 1.f / d.z);
  const V3 binv = v3(clamp_inv(d.x), clamp_inv(d.y), clamp_inv(d.z));
  const V3 p = o + d * t_hit;
  unsigned long long key;
  if (ln > 4) {
    // a big primitive (walls: hundreds of leaves): the leaf holding a point
    // just before the hit, else just after it (a hit on a wall lies on a split
    // plane, and the wall is in the leaves on one side of it only), found by
    // descent, then by binary search in the (ascending) list
    for (int side = 0; side < 2; ++side) {
      const float tp = side == 0 ? t_hit * 0.99999f - 1e-4f : t_hit * 1.00001f + 1e-4f;
      const uint32_t at = kd_locate_node(S, o + d * tp);
#if WR_MEMBER_REFS
      // does the located leaf list p1?  Its own references, 8 per round trip
      // (one for the usual leaf), instead of a binary search of p1's
      // ascending leaf list (~11 dependent loads for a floor's thousands)
      const uint4 w = S.nrec[at];
      const uint32_t first = w.x, cnt = w.y >> 2;
      bool listed = false;
      for (uint32_t j0 = 0; j0 < cnt && !listed; j0 += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int code = j0 + u < cnt ? __float_as_int(S.ref_c[first + j0 + u].y) : -1;
          const int pr = code >= 0 ? code : -code - 1;  // a sphere's ref: -(prim + 1)
          listed |= j0 + u < cnt && pr == p1;
        }
      }
      const int want = F.node_path[at];
#else
      const int want = F.node_path[at];
      int a = lb, b = lb + ln;
      while (a < b) {
        const int mid = (a + b) >> 1;
        if (F.prim_leaf[mid] < want) a = mid + 1;
        else b = mid;
      }
      const bool listed = a < lb + ln && F.prim_leaf[a] == want;
#endif
      if (listed) {
        const uint2* rec = F.path + want;
        const uint4 h0 = *reinterpret_cast<const uint4*>(rec);
        const uint4 h1 = *reinterpret_cast<const uint4*>(rec + 2);
        if (cell_crossed_with_margin(h0, h1, o, d, binv, rtmax)) return kMember;
        if (kd_reaches(rec, o, d, inv, tmin, tmax, rtmax, steps, key)) return kMember;
      }
    }
  }
#if !WR_RESOLVE_SCAN
  // a many-leaf primitive whose located leaf proved nothing: its whole leaf
  // list is scanned by one wave per ray in k_fast_hard (scan_fast) instead of
  // by this lane, which would hold the resolve wave for up to ~1 ms
  if (ln > 4) return kScan;
#endif
  if (ln >= 1 && ln <= 4) {
    // witnesses first, all of the primitive's leaves at once: the list
    // entries, then the cells, each set of loads in flight together
    int off[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) off[k] = F.prim_leaf[lb + min(k, ln - 1)];
    uint4 h0[4], h1[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint2* rec = F.path + off[k];
      h0[k] = *reinterpret_cast<const uint4*>(rec);
      h1[k] = *reinterpret_cast<const uint4*>(rec + 2);
    }
    bool seen = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) seen |= k < ln && cell_crossed_with_margin(h0[k], h1[k], o, d, binv, rtmax);
    if (seen) return kMember;
  }
  // replays: the leaves whose cell holds the hit point first (usually the one
  // reached), then the others
  for (int pass = 0; pass < 2; ++pass) {
    for (int k = lb; k < lb + ln; ++k) {
      const uint2* rec = F.path + F.prim_leaf[k];
      const uint4 h0 = *reinterpret_cast<const uint4*>(rec);
      const uint4 h1 = *reinterpret_cast<const uint4*>(rec + 2);
      const bool in = p.x >= __uint_as_float(h0.z) && p.y >= __uint_as_float(h0.w) && p.z >= __uint_as_float(h1.x) &&
                      p.x <= __uint_as_float(h1.y) && p.y <= __uint_as_float(h1.z) && p.z <= __uint_as_float(h1.w);
      if (pass == 0 && ln > 4 && cell_crossed_with_margin(h0, h1, o, d, binv, rtmax)) return kMember;
      if (in == (pass == 0) && (!WR_SCAN_CELL_FILTER || cell_may_be_reached(h0, h1, o, d, tmax)) &&
          kd_reaches(rec, o, d, inv, tmin, tmax, rtmax, steps, key))
        return kMember;
    }
  }
  return kNotMember;
}

// KDtreeAccel::traverse (KDtreeAccel.cpp:309-388) for one ray on one lane:
// root-box clip, the belowFirst near / far rule, the `ray.tmax < tmin` stop, no
// early exit, and `cmp(t - best) < 0` over every leaf's references in order.
// The stack holds (node, tmin) in LDS columns of stride 64; an entry's tmax is
// the previous entry's tmin (the root tmax for entry 0), the floats the
// reference's todo[] holds.
// One primitive of a KD leaf (refs: ref_c.y = prim, or -(prim + 1) for a
// sphere) or of a BVH leaf (TriRec: the same code in c.y): Triangle::hit
// (tri_test: the screen against t_best only drops what the exact test rejects
// or what cannot improve t_best) or Sphere::hit (sph_hit, sphere.cpp:17-78).
// prim gets the primitive.
__device__ __forceinline__ bool prim_test(const DevScene& S, float4 a, float4 b, float f, int code, V3 o, V3 d,
                                          float rtmin, float rtmax, float t_best, float& t, int& prim) {
  if (code >= 0) {
    prim = code;
    return tri_test(a, b, f, o, d, rtmin, rtmax, t_best, t);
  }
  prim = -code - 1;
  return sph_hit(S, prim, o, d, rtmin, rtmax, t);
}

template <bool COUNT>
__device__ __forceinline__ void kd_walk(const DevScene& S, V3 o, V3 d, float rtmin, float rtmax, int* stk_node,
                                        float* stk_tmin, float& t_best, int& best, FastCounters& ctr) {
  t_best = WR_INF;
  best = -1;
  float tmin, tmax;
  if (!box_hit(S.root_l, S.root_r, o, d, tmin, tmax) || rtmax < tmin) return;  // :312-313, :323
  const float root_tmax = tmax;
  const V3 inv = v3(1.f / d.x, 1.f / d.y, 1.f / d.z);
  uint32_t node = 0;
  int sp = 0;
  for (;;) {
    const uint4 w = S.nrec[node];  // (self, left child)
    if ((w.y & 3u) != 3u) {        // inner (:325-358)
      if (COUNT) ++ctr.kinner;
      const uint32_t axis = w.y & 3u;
      const float split = __uint_as_float(w.x);
      const float oa = axis == 0 ? o.x : (axis == 1 ? o.y : o.z);
      const float da = axis == 0 ? d.x : (axis == 1 ? d.y : d.z);
      const float ia = axis == 0 ? inv.x : (axis == 1 ? inv.y : inv.z);
      const float t = (split - oa) * ia;
      const bool below = (oa < split) | ((oa == split) & (da <= 0));
      const uint32_t left = node + 1, right = w.y >> 2;
      const uint32_t nearc = below ? left : right, farc = below ? right : left;
      if ((t > tmax) | (t <= 0)) {
        node = nearc;
      } else if (t < tmin) {
        node = farc;
      } else {
        stk_node[sp * 64] = static_cast<int>(farc);
        stk_tmin[sp * 64] = t;
        ++sp;
        node = nearc;
        tmax = t;
      }
      continue;
    }
    // leaf (:359-373): references in order, four records in flight
    const uint32_t first = w.x, cnt = w.y >> 2;
    if (COUNT) {
      ++ctr.kleaves;
      ctr.krefs += cnt;
    }
    for (uint32_t k0 = 0; k0 < cnt; k0 += 4) {
      float4 ra[4], rb[4];
      float2 rc[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t ref = first + min(k0 + u, cnt - 1);
        ra[u] = S.ref_a[ref];
        rb[u] = S.ref_b[ref];
        rc[u] = S.ref_c[ref];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (k0 + u >= cnt) break;
        float t;
        int prim;
        if (prim_test(S, ra[u], rb[u], rc[u].x, __float_as_int(rc[u].y), o, d, rtmin, rtmax, t_best, t, prim) &&
            cmpf(t - t_best) < 0) {
          t_best = t;
          best = prim;
        }
      }
    }
    if (sp == 0) return;  // :375-383
    --sp;
    node = static_cast<uint32_t>(stk_node[sp * 64]);
    tmin = stk_tmin[sp * 64];
    tmax = sp > 0 ? stk_tmin[(sp - 1) * 64] : root_tmax;
    if (rtmax < tmin) return;  // :323
  }
}

// kd_walk for one ray by a whole wave (every lane holds the ray; all lanes
// return the same answer).  The reference's walk has no early exit, so the
// leaves it reaches are fixed by the root clip, the near / far rule and the
// :323 stop, never by its hits; a node's (tmin, tmax) is a function of its
// root path (near child (tmin, t) or (tmin, tmax), far child (t, tmax): the
// popped todo entry's tmax is the entry below it, which is the parent's tmax);
// and the :323 stop at a popped far child ends the walk only after every entry
// below it would fail it too (their tmin are >= its own).  So the wave expands
// the crossed nodes up to 64 at a time from a work stack in LDS, and each
// reached leaf's references are tested by the lane that reached it.  A hit's
// place in the walk's order is its leaf's key (kd_reaches' bits, far child at
// depth k = bit 63 - k; the walk visits smaller keys first) with its position
// in the leaf in the key's free low bits.  Only each primitive's first hit in
// that order can matter -- the same ray and triangle give the same t, so a
// later repeat fails `cmp(t - best) < 0` whether the first was taken or not --
// and a floor or wall sits in hundreds of the leaves a ray crosses: the hits
// go to a hash table in LDS keyed by primitive, keeping the smallest order
// (atomicMin).  The reference's rule, first found wins, is then replayed over
// the primitives sorted by that order: kd_walk's answer.  A ray whose walk
// takes ~10^3 dependent loads on one lane takes ~ its tree depth plus its
// nodes / 64 in rounds here (C4: 40 rounds for 1,640 nodes).
// `lds`: the wave's `words` 32-bit words (the hard kernels' stack columns).
// Returns false, nothing written, when the work stack or the table outgrows
// them: the caller walks the ray the serial way.  Node indices < 2^26 (the
// depth shares their word) and KD depth <= 43 (the position's bits): the host
// checks, FastScene::walk_wave.
__device__ __forceinline__ uint32_t wave_add32(uint32_t v) {
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) v += __shfl_xor(v, sh);
  return v;
}
template <bool COUNT>
__device__ __forceinline__ bool kd_walk_wave(const DevScene& S, V3 o, V3 d, float rtmin, float rtmax, uint32_t* lds,
                                             int words, float& t_best, int& best, FastCounters& ctr) {
  const int lane = __lane_id();
  t_best = WR_INF;
  best = -1;
  float tmin0, tmax0;
  if (!box_hit(S.root_l, S.root_r, o, d, tmin0, tmax0) || rtmax < tmin0) return true;  // :312-313, :323
  const V3 inv = v3(1.f / d.x, 1.f / d.y, 1.f / d.z);
  // LDS: the table (order u64, primitive, t: 4 words a slot), then the work
  // stack (5 columns, at least as many entries as the table has slots: the
  // replay's sorted primitives go to its first two columns)
  const int lg = words >= 2048 ? 8 : 7, T = 1 << lg;
  const int cap = (words - 4 * T) / 5;
  if (cap < T || cap < 128) return false;
  unsigned long long* h_ord = reinterpret_cast<unsigned long long*>(lds);
  int* h_prim = reinterpret_cast<int*>(h_ord + T);
  float* h_t = reinterpret_cast<float*>(h_prim + T);
  uint32_t* s_node = reinterpret_cast<uint32_t*>(h_t + T);
  float* s_tmin = reinterpret_cast<float*>(s_node + cap);
  float* s_tmax = s_tmin + cap;
  uint32_t* s_khi = reinterpret_cast<uint32_t*>(s_tmax + cap);
  uint32_t* s_klo = s_khi + cap;
  for (int i = lane; i < T; i += 64) {
    h_ord[i] = ~0ull;
    h_prim[i] = -1;
  }
  if (lane == 0) {
    s_node[0] = 0u;
    s_tmin[0] = tmin0;
    s_tmax[0] = tmax0;
    s_khi[0] = 0u;
    s_klo[0] = 0u;
  }
  __syncthreads();  // one wave per block: orders the LDS writes for the other lanes
  int sp = 1;  // wave-uniform
  bool over = false, full = false;
  uint32_t rounds = 0;
  uint32_t ninner = 0, nleaves = 0, nrefs = 0;
  while (sp > 0) {
    // an entry taken pushes at most two: taking no more than the free room
    // keeps the stack within its columns (a long walk then narrows to the
    // room it has instead of failing over to the serial walk)
    const int take = max(1, min(min(sp, 64), cap - sp)), base = sp - take;
    ++rounds;
    const bool act = lane < take;
    uint32_t nd = 0, khi = 0, klo = 0;
    float tmin = 0.f, tmax = 0.f;
    if (act) {
      nd = s_node[base + lane];
      tmin = s_tmin[base + lane];
      tmax = s_tmax[base + lane];
      khi = s_khi[base + lane];
      klo = s_klo[base + lane];
    }
    __syncthreads();  // the entries are read before this round's pushes overwrite them
    const uint32_t node = nd & 0x03ffffffu, depth = nd >> 26;
    const uint4 w = act ? S.nrec[node] : make_uint4(0u, 0u, 0u, 0u);
    const bool leaf = act && (w.y & 3u) == 3u;
    // inner (:325-358): the children this node's walk goes on to
    int nc = 0;
    uint32_t c0 = 0, c1 = 0;
    float c0min = 0.f, c0max = 0.f, c1min = 0.f, c1max = 0.f;
    uint32_t c0hi = khi, c0lo = klo, c1hi = khi, c1lo = klo;
    if (act && !leaf) {
      if (COUNT) ++ninner;
      const uint32_t axis = w.y & 3u;
      const float split = __uint_as_float(w.x);
      const float oa = axis == 0 ? o.x : (axis == 1 ? o.y : o.z);
      const float da = axis == 0 ? d.x : (axis == 1 ? d.y : d.z);
      const float ia = axis == 0 ? inv.x : (axis == 1 ? inv.y : inv.z);
      const float t = (split - oa) * ia;
      const bool below = (oa < split) | ((oa == split) & (da <= 0));
      const uint32_t left = node + 1, right = w.y >> 2;
      const uint32_t nearc = below ? left : right, farc = below ? right : left;
      // the far child's key bit at this depth (a one-child step sets it or
      // not alike for every leaf below: only the order of two visited
      // children matters)
      const uint32_t fhi = depth < 32 ? (0x80000000u >> depth) : 0u, flo = depth < 32 ? 0u : (0x80000000u >> (depth - 32));
      const uint32_t cd = (depth + 1) << 26;
      if ((t > tmax) | (t <= 0)) {
        nc = 1;
        c0 = nearc | cd;
        c0min = tmin;
        c0max = tmax;
      } else if (t < tmin) {
        nc = 1;
        c0 = farc | cd;
        c0min = tmin;
        c0max = tmax;
        c0hi |= fhi;
        c0lo |= flo;
      } else {
        nc = 1;
        c0 = nearc | cd;
        c0min = tmin;
        c0max = t;
        if (!(rtmax < t)) {  // the far entry's :323 test at its pop
          nc = 2;
          c1 = farc | cd;
          c1min = t;
          c1max = tmax;
          c1hi |= fhi;
          c1lo |= flo;
        }
      }
    }
    // pushes: one or two entries per lane, packed by prefix counts
    const unsigned long long m1 = __ballot(nc >= 1), m2 = __ballot(nc == 2);
    const int pre = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m1 >> 32),
                                              __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m1), 0)) +
                    __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m2 >> 32),
                                              __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m2), 0));
    const int pushed = __popcll(m1) + __popcll(m2);
    if (base + pushed > cap) {
      over = true;
      break;
    }
    if (nc >= 1) {
      const int i = base + pre;
      s_node[i] = c0;
      s_tmin[i] = c0min;
      s_tmax[i] = c0max;
      s_khi[i] = c0hi;
      s_klo[i] = c0lo;
    }
    if (nc == 2) {
      const int i = base + pre + 1;
      s_node[i] = c1;
      s_tmin[i] = c1min;
      s_tmax[i] = c1max;
      s_khi[i] = c1hi;
      s_klo[i] = c1lo;
    }
    // leaf (:359-373): its references, four records in flight; each hit into
    // the table under its primitive, the smallest order kept
    if (leaf) {
      const uint32_t first = w.x, cnt = w.y >> 2;
      if (COUNT) {
        ++nleaves;
        nrefs += cnt;
      }
      const unsigned long long key = (static_cast<unsigned long long>(khi) << 32) | klo;
      for (uint32_t k0 = 0; k0 < cnt; k0 += 4) {
        float4 ra[4], rb[4];
        float2 rc[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t ref = first + min(k0 + u, cnt - 1);
          ra[u] = S.ref_a[ref];
          rb[u] = S.ref_b[ref];
          rc[u] = S.ref_c[ref];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (k0 + u >= cnt) break;
          float t;
          int prim;
          // t_best WR_INF: the exact Triangle::hit outcome (the screen drops
          // only what it proves rejected); the replay applies the rule
          if (prim_test(S, ra[u], rb[u], rc[u].x, __float_as_int(rc[u].y), o, d, rtmin, rtmax, WR_INF, t, prim) &&
              cmpf(t - WR_INF) < 0) {
            uint32_t h = (static_cast<uint32_t>(prim) * 2654435761u) >> (32 - lg);
            bool put = false;
            for (int probe = 0; probe < T && !put; ++probe) {
              const int was = atomicCAS(&h_prim[h], -1, prim);
              if (was == -1 || was == prim) {
                atomicMin(&h_ord[h], key | (k0 + u));
                h_t[h] = t;  // (every repeat writes the same t)
                put = true;
              }
              h = (h + 1) & static_cast<uint32_t>(T - 1);
            }
            full |= !put;
          }
        }
      }
    }
    sp = base + pushed;
    __syncthreads();  // this round's pushes and hits before the next round's reads
  }
  __syncthreads();
  full = __ballot(full) != 0ull;
  // the primitives hit, in walk order: each lane ranks its slots' entries
  // among all (orders are distinct: one primitive per leaf position), then
  // writes them sorted into the (finished) work stack's columns
  int nh = 0;
  if (!over && !full) {
    for (int i = lane; i < T; i += 64) {
      if (h_prim[i] < 0) continue;
      const unsigned long long a = h_ord[i];
      int rank = 0;
      for (int j = 0; j < T; ++j) rank += (h_prim[j] >= 0 && h_ord[j] < a) ? 1 : 0;
      s_tmin[rank] = h_t[i];
      s_node[rank] = static_cast<uint32_t>(h_prim[i]);
      ++nh;
    }
    nh = static_cast<int>(wave_add32(static_cast<uint32_t>(nh)));
  }
  if (COUNT) {
    const uint32_t a = wave_add32(ninner), b = wave_add32(nleaves);
    ctr.kinner += a;
    ctr.kleaves += b;
    ctr.krefs += wave_add32(nrefs);
    ctr.ww_walks += 1;
    ctr.ww_rounds += rounds;
    ctr.ww_nodes += a + b;
    ctr.ww_over += (over ? 1000u : 0u) + (full ? 1u : 0u);  // (stack x 1000 + table)
  }
  if (over || full) return false;
  __syncthreads();
  for (int j = 0; j < nh; ++j) {  // wave-uniform: the reference's leaf loop, primitive by primitive
    const float t = s_tmin[j];
    if (cmpf(t - t_best) < 0) {
      t_best = t;
      best = static_cast<int>(s_node[j]);
    }
  }
  return true;
}

// The kTie smallest triangle hits (Triangle::hit) with t <= cap of the ray over
// the BVH, as (t, prim) sorted by t: a search whose bound is the kTie-th
// smallest hit so far (and cap), with the main search's box margins.  Returns
// the number of hits <= cap found (> kTie: more exist beyond ct[kTie - 1]).
constexpr int kTie = 8;
#ifndef WR_TIE_LEAVES
#define WR_TIE_LEAVES 16
#endif
constexpr int kTieLeaves = WR_TIE_LEAVES;  // resolve_tie: replay up to this many KD leaves per candidate, else a pruned walk
#ifndef WR_TIE_WAVE_ALL
#define WR_TIE_WAVE_ALL 0  // 1: every near-tie to the one-ray-per-wave resolution
#endif
constexpr int kTieWaveLeaves = 65536;  // ... or, one ray per wave, up to this many leaves of all candidates (cell-filtered)
#ifndef WR_TIE_DEFER
// 1: in the one-ray-per-lane resolution, a near-tie with a many-leaf candidate
// is handed back (kTieDeferred) and resolved by the lane's whole wave
// afterwards (first_leaves_wave) instead of a pruned KD walk by the lane alone.
// Off: the longest tie drops 6.2 -> 0.76 ms, but the 16-pipeline run loses
// (C4 1,485 -> 1,176 Mrays/s)
#define WR_TIE_DEFER 0
#endif
constexpr int kTieDeferred = -1;
__device__ __forceinline__ int bvh_collect(const DevScene& S, const FastScene& F, V3 o, V3 d, float rtmin, float rtmax, float cap,
                                           int* stk_link, float* stk_t, float (&ct)[kTie], int (&cp)[kTie]) {
  rtmax = fminf(rtmax, cap);
#pragma unroll
  for (int j = 0; j < kTie; ++j) {
    ct[j] = WR_INF;
    cp[j] = -1;
  }
  const V3 binv = v3(clamp_inv(d.x), clamp_inv(d.y), clamp_inv(d.z));
  float dlen = sqrtf(d.x * d.x + d.y * d.y + d.z * d.z);
  if (!(dlen > 0.f)) dlen = 1.f;
  float tcap;
  {
    const float ax = (F.lo.x - o.x) * binv.x, bx = (F.hi.x - o.x) * binv.x;
    const float ay = (F.lo.y - o.y) * binv.y, by = (F.hi.y - o.y) * binv.y;
    const float az = (F.lo.z - o.z) * binv.z, bz = (F.hi.z - o.z) * binv.z;
    tcap = fmaxf(0.f, fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz)));
  }
  int found = 0, sp = 0, cur = 0;
  for (;;) {
    const float thi = fminf(rtmax, ct[kTie - 1]);
    const float g = wrf::kRayGrow * (fminf(thi, tcap) * dlen + 1.f);
    const float gt = g / dlen;
    if (cur >= 0) {
      const float4* np = F.nodes + 4 * static_cast<size_t>(cur);
      const float4 n0 = np[0], n1 = np[1], n2 = np[2];
      const int4 lk = *reinterpret_cast<const int4*>(np + 3);
      const float lo_t = rtmin - gt, hi_t = thi + gt;
      auto slab = [&](float lx, float ly, float lz, float hx, float hy, float hz, float& tn) {
        const float x0 = (lx - g - o.x) * binv.x, x1 = (hx + g - o.x) * binv.x;
        const float y0 = (ly - g - o.y) * binv.y, y1 = (hy + g - o.y) * binv.y;
        const float z0 = (lz - g - o.z) * binv.z, z1 = (hz + g - o.z) * binv.z;
        tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), lo_t));
        const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), hi_t));
        return tn <= tf;
      };
      float ta, tb;
      const bool ha = slab(n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, ta);
      const bool hb = slab(n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, tb);
      if (ha && hb) {
        const bool af = ta <= tb;
        stk_link[sp * 64] = af ? lk.y : lk.x;
        stk_t[sp * 64] = af ? tb : ta;
        ++sp;
        cur = af ? lk.x : lk.y;
        continue;
      }
      if (ha || hb) {
        cur = ha ? lk.x : lk.y;
        continue;
      }
    } else {
      const int l = ~cur;
      const int first = l >> 3, cnt = (l & 7) + 1;
      for (int j = 0; j < cnt; ++j) {
        const float4* tp = F.tris + 3 * static_cast<size_t>(first + j);
        float t;
        int npr;
        // screen: only hits below the current kTie-th can enter the list
        if (prim_test(S, tp[0], tp[1], tp[2].x, __float_as_int(tp[2].y), o, d, rtmin, rtmax,
                      fminf(ct[kTie - 1], rtmax) + WR_EPS + WR_EPS, t, npr) &&
            t <= rtmax) {
          ++found;
          float nt = t;
#pragma unroll
          for (int k = 0; k < kTie; ++k) {  // insertion, sorted by t
            const bool sw = nt < ct[k];
            const float tt = sw ? ct[k] : nt;
            const int pp = sw ? cp[k] : npr;
            if (sw) {
              ct[k] = nt;
              cp[k] = npr;
            }
            nt = tt;
            npr = pp;
          }
        }
      }
    }
    // pop the next subtree that can still hold one of the kTie smallest hits
    const float thi2 = fminf(rtmax, ct[kTie - 1]);
    const float gt2 = (wrf::kRayGrow * (fminf(thi2, tcap) * dlen + 1.f)) / dlen;
    cur = 0x7fffffff;
    while (sp > 0) {
      --sp;
      if (stk_t[sp * 64] <= thi2 + gt2) {
        cur = stk_link[sp * 64];
        break;
      }
    }
    if (cur == 0x7fffffff) return found;
  }
}

// The first leaf of primitive p that the reference's traversal visits, as its
// visit key (kd_reaches) and p's position in that leaf's list; key = ~0: p is
// not visited.  (pos < 256, so (key, pos) orders the visits of one ray.)
// The leaves are taken four at a time: their path offsets, then their headers
// (cells) in flight together -- a candidate's leaves mostly fail the cell
// test, and one at a time each cost two dependent round trips.
__device__ WR_HARD_CALL void first_leaf(const FastScene& F, int p, V3 o, V3 d, V3 inv, float tmin0, float tmax0,
                                        float rtmax, unsigned long long& key, int& pos, uint32_t& steps) {
  constexpr int U = 4;
  key = ~0ull;
  pos = 0;
  const int lb = F.prim_leaf_off[p], le = F.prim_leaf_off[p + 1];
  for (int k0 = lb; k0 < le; k0 += U) {
    int off[U];
    uint4 h0[U], h1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) off[u] = k0 + u < le ? F.prim_leaf[k0 + u] : F.prim_leaf[k0];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint2* rec = F.path + off[u];
      h0[u] = *reinterpret_cast<const uint4*>(rec);
      h1[u] = *reinterpret_cast<const uint4*>(rec + 2);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (k0 + u >= le) break;
      // a leaf whose cell the ray's line misses is never reached: no replay
      if (!cell_may_be_reached(h0[u], h1[u], o, d, tmax0)) continue;
      unsigned long long kk;
      if (!kd_reaches(F.path + off[u], o, d, inv, tmin0, tmax0, rtmax, steps, kk)) continue;
      const int pk = F.prim_leaf_pos[k0 + u];
      if (kk < key || (kk == key && pk < pos)) {
        key = kk;
        pos = pk;
      }
    }
  }
}

// first_leaf for the candidates cp[0, ncand) of ONE ray, with the wave's lanes
// sharing the work (every lane holds the same ray and list): the candidates'
// leaf lists are laid end to end and lane j takes entries j, j + 64, ..., four
// at a time with their loads in flight together.  A leaf whose cell the ray
// cannot reach (cell_may_be_reached) is dropped before its path replay --
// floors and walls sit in thousands of leaves, the ray meets a few.  Each lane
// keeps its smallest (key, pos) per candidate; one min-reduction over the
// lanes at the end.  Same answers as first_leaf per candidate.
__device__ __forceinline__ void first_leaves_wave(const FastScene& F, const int (&cp)[kTie], int ncand, V3 o, V3 d,
                                                  V3 inv, float tmin0, float tmax0, float rtmax,
                                                  unsigned long long (&key)[kTie], int (&pos)[kTie],
                                                  uint32_t& steps) {
  constexpr int U = 4;
  const int lane = __lane_id();
  int off[kTie + 1], lb[kTie];
  off[0] = 0;
#pragma unroll
  for (int c = 0; c < kTie; ++c) {
    lb[c] = c < ncand ? F.prim_leaf_off[cp[c]] : 0;
    off[c + 1] = off[c] + (c < ncand ? F.prim_leaf_off[cp[c] + 1] - lb[c] : 0);
    key[c] = ~0ull;
    pos[c] = 0x7fffffff;
  }
  const int total = off[kTie];
  for (int base = 0; base < total; base += 64 * U) {
    int k[U], mine[U], po[U];
    uint4 h0[U], h1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = base + u * 64 + lane;
      mine[u] = -1;
      k[u] = 0;
      if (j < total) {
        k[u] = lb[0] + j;
        mine[u] = 0;
#pragma unroll
        for (int c = 1; c < kTie; ++c)
          if (j >= off[c] && c < ncand) {
            mine[u] = c;
            k[u] = lb[c] + (j - off[c]);
          }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) po[u] = mine[u] >= 0 ? F.prim_leaf[k[u]] : 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint2* rec = F.path + po[u];
      h0[u] = *reinterpret_cast<const uint4*>(rec);
      h1[u] = *reinterpret_cast<const uint4*>(rec + 2);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      unsigned long long t;
      if (mine[u] >= 0 && cell_may_be_reached(h0[u], h1[u], o, d, tmax0) &&
          kd_reaches(F.path + po[u], o, d, inv, tmin0, tmax0, rtmax, steps, t)) {
        const int pk = F.prim_leaf_pos[k[u]];
#pragma unroll
        for (int c = 0; c < kTie; ++c)
          if (mine[u] == c && (t < key[c] || (t == key[c] && pk < pos[c]))) {
            key[c] = t;
            pos[c] = pk;
          }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < kTie; ++c) {
    if (c >= ncand) break;  // wave-uniform
    unsigned long long a = key[c];
    int b = pos[c];
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) {
      const unsigned long long a2 = __shfl_xor(a, sh);
      const int b2 = __shfl_xor(b, sh);
      const bool take = a2 < a || (a2 == a && b2 < b);
      a = take ? a2 : a;
      b = take ? b2 : b;
    }
    key[c] = a;
    pos[c] = a == ~0ull ? 0 : b;  // not visited: (~0, 0) as first_leaf leaves it
  }
#pragma unroll
  for (int c = 0; c < kTie; ++c)
    if (c >= ncand) pos[c] = 0;
}

// The first visited leaf of several primitives at once, by the reference's own
// walk (KDtreeAccel.cpp:309-388: root clip, near / far rule, the :323 stop)
// restricted to subtrees whose cell meets one of their boxes: a primitive is
// put in a child only when its box reaches into it by more than EPS
// (KDtreeAccel.cpp:138-157), so a subtree whose cell misses every box holds
// none of their leaves.  Leaves are numbered in visit order; at a leaf each
// unresolved primitive is looked up in its (ascending) leaf list.  want: mask
// of the candidates to find; vis / pos get (visit number, position in list).
__device__ WR_HARD_CALL void kd_first_leaves(const DevScene& S, const FastScene& F, V3 o, V3 d, float rtmax,
                                             const int* cp, unsigned want, int* stk_node, float* stk_tmin,
                                             int* vis, int* pos, uint32_t& steps) {
  float tmin, tmax;
  if (!box_hit(S.root_l, S.root_r, o, d, tmin, tmax) || rtmax < tmin) return;
  const float root_tmax = tmax;
  const V3 inv = v3(1.f / d.x, 1.f / d.y, 1.f / d.z);
  uint32_t node = 0;
  int sp = 0, visit = 0;
  for (;;) {
    const uint4 w = S.nrec[node];
    const float4 clo = F.node_cell[2 * node], chi = F.node_cell[2 * node + 1];
    ++steps;
    bool meets = false;
    for (int c = 0; c < kTie; ++c) {
      if (!((want >> c) & 1u)) continue;
      const float4 b0 = S.prim_sbox0[cp[c]];
      const float2 b1 = S.prim_sbox1[cp[c]];
      meets |= b0.x <= chi.x && b0.y <= chi.y && b0.z <= chi.z && b0.w >= clo.x && b1.x >= clo.y && b1.y >= clo.z;
    }
    bool pop = !meets;
    if (meets) {
      if ((w.y & 3u) != 3u) {  // inner (:325-358)
        const uint32_t axis = w.y & 3u;
        const float split = __uint_as_float(w.x);
        const float oa = axis == 0 ? o.x : (axis == 1 ? o.y : o.z);
        const float da = axis == 0 ? d.x : (axis == 1 ? d.y : d.z);
        const float ia = axis == 0 ? inv.x : (axis == 1 ? inv.y : inv.z);
        const float t = (split - oa) * ia;
        const bool below = (oa < split) | ((oa == split) & (da <= 0));
        const uint32_t left = node + 1, right = w.y >> 2;
        const uint32_t nearc = below ? left : right, farc = below ? right : left;
        if ((t > tmax) | (t <= 0)) {
          node = nearc;
        } else if (t < tmin) {
          node = farc;
        } else {
          stk_node[sp * 64] = static_cast<int>(farc);
          stk_tmin[sp * 64] = t;
          ++sp;
          node = nearc;
          tmax = t;
        }
        continue;
      }
      // leaf: which wanted primitives does it hold?  Its own reference list
      // (ref_c.y: the primitive, in the leaf's order) read 8 entries per
      // round trip -- one for the usual leaf -- instead of a binary search of
      // each candidate's ascending leaf list (~12 dependent loads per
      // candidate on the 1M-triangle tree); a primitive listed twice keeps its
      // first position, as prim_leaf_pos does
      ++visit;
      const uint32_t first = w.x, cnt = w.y >> 2;
      for (uint32_t j0 = 0; j0 < cnt && want; j0 += 8) {
        int pr[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int code = j0 + u < cnt ? __float_as_int(S.ref_c[first + j0 + u].y) : -1;
          pr[u] = code >= 0 || j0 + u >= cnt ? code : -code - 1;  // a sphere's ref: -(prim + 1)
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          for (int c = 0; c < kTie; ++c)
            if (((want >> c) & 1u) && pr[u] == cp[c]) {
              vis[c] = visit;
              pos[c] = static_cast<int>(j0) + u;
              want &= ~(1u << c);
            }
      }
      if (!want) return;
      pop = true;
    }
    if (pop) {
      if (sp == 0) return;  // :375-383
      --sp;
      node = static_cast<uint32_t>(stk_node[sp * 64]);
      tmin = stk_tmin[sp * 64];
      tmax = sp > 0 ? stk_tmin[(sp - 1) * 64] : root_tmax;
      if (rtmax < tmin) return;  // :323
    }
  }
}

// Resolution by visit order.  The reference's answer is first-found-wins
// (cmp(t - best) < 0) over the hits it visits, in visit order.  Let m be the
// smallest hit it visits.  Its winner lies within EPS of m (once m is reached
// either m is taken or best is already within EPS of it, and afterwards only t
// < best - EPS <= m could be taken).  A visited hit beyond m + 3 EPS, whenever
// it is the best, lets every hit up to m + 2 EPS through (their difference
// exceeds EPS), so with every hit up to m + 3 EPS known and no visited one
// between m + 1.5 EPS and m + 3 EPS, the rule run over the visited hits up to
// m + 1.5 EPS in visit order gives the reference's answer.  The kTie smallest
// hits of the scene (bvh_collect) hold all hits up to m + 3 EPS when fewer
// were found or the last one lies beyond.  Returns false when a condition
// fails (the caller walks the KD tree).
// WAVE: every lane of the wave holds the same ray (k_fast_hard's one ray per
// wave); the candidates' leaf replays are shared out (psteps: this lane's).
template <bool WAVE>
__device__ __forceinline__ bool resolve_tie(const DevScene& S, const FastScene& F, V3 o, V3 d, float rtmin,
                                            float rtmax, float t1, int* stk_link, float* stk_t, float& t_out,
                                            int& p_out, uint32_t& steps, uint32_t& psteps, int& dbg,
                                            uint32_t* split = nullptr, int p1 = -1, int2 pair = {-1, 0}) {
  float tmin0, tmax0;
  if (!box_hit(S.root_l, S.root_r, o, d, tmin0, tmax0) || rtmax < tmin0) return false;
  const V3 inv = v3(1.f / d.x, 1.f / d.y, 1.f / d.z);
  float ct[kTie];
  int cp[kTie];
  unsigned long long key[kTie];
  int pos[kTie];
  float m = WR_INF;
  int n = 0;
  // first the hits up to t1 + 3 EPS (t1 = the scene's smallest); if t1's
  // triangle is not visited, the hits up to m + 3 EPS, m = the smallest
  // visited hit of that window (WR_TIE_PASS2_CAP): every hit below t1 + 3 EPS
  // was in it, so no visited hit lies below m and m stays the smallest
  // visited -- the rule below needs every hit up to m + 3 EPS, no more.  Only
  // when no hit of the window is visited, the kTie smallest without a bound
  for (int pass = 0; pass < 2; ++pass) {
    const float cap = pass == 0 ? t1 + 3.f * WR_EPS : ((WR_TIE_PASS2_CAP && m < WR_INF) ? m + 3.f * WR_EPS : WR_INF);
#if WR_TIE_SPLIT
    const uint64_t a0 = wall_clock64();
#endif
    if (pass == 0 && pair.x >= 0 && p1 >= 0) {
      // the search's pair (kPairWindow): the first window holds exactly these
      // two hits, the collection's answer without the collection
#if WR_TIE_SPLIT
      if (split) ++split[3];
#endif
      n = 2;
#pragma unroll
      for (int j = 0; j < kTie; ++j) {
        ct[j] = j == 0 ? t1 : (j == 1 ? __int_as_float(pair.y) : WR_INF);
        cp[j] = j == 0 ? p1 : (j == 1 ? pair.x : -1);
      }
    } else {
      n = bvh_collect(S, F, o, d, rtmin, rtmax, cap, stk_link, stk_t, ct, cp);
    }
#if WR_TIE_SPLIT
    const uint64_t a1 = wall_clock64();
    if (split) {
      split[0] += static_cast<uint32_t>(a1 - a0);
      split[2] += pass;
    }
#endif
    m = WR_INF;
    const int ncand = min(n, kTie);
    // per candidate: its first visited leaf as a visit-order key (~0: none).
    // Primitives in many leaves (walls, floors): one walk of the KD tree
    // pruned to the candidates' boxes finds them all (keys = visit numbers);
    // otherwise each candidate's leaves are replayed (keys = far-child bits)
    bool big = false;
    int total = 0;
    for (int c = 0; c < ncand; ++c) {
      const int ln = F.prim_leaf_off[cp[c] + 1] - F.prim_leaf_off[cp[c]];
      big |= ln > kTieLeaves;
      total += ln;
    }
    // one ray per wave: the lanes replay every leaf of the candidates side by
    // side (up to kTieWaveLeaves of them, 128 rounds) instead of the walk
    if (WAVE && total <= kTieWaveLeaves) big = false;
    if (!WAVE && WR_TIE_DEFER && big) {  // the lane's wave resolves it together (hard_fast)
      dbg = kTieDeferred;
      return false;
    }
    if (big) {
      int vis[kTie], ps[kTie];
      for (int c = 0; c < kTie; ++c) {
        vis[c] = -1;
        ps[c] = 0;
      }
      kd_first_leaves(S, F, o, d, rtmax, cp, (1u << ncand) - 1u, stk_link, stk_t, vis, ps, steps);
#pragma unroll
      for (int c = 0; c < kTie; ++c) {
        key[c] = (c < ncand && vis[c] >= 0) ? static_cast<unsigned long long>(vis[c]) : ~0ull;
        pos[c] = ps[c];
      }
    } else if (WAVE) {
      first_leaves_wave(F, cp, ncand, o, d, inv, tmin0, tmax0, rtmax, key, pos, psteps);
    } else {
#pragma unroll
      for (int c = 0; c < kTie; ++c) {
        key[c] = ~0ull;
        pos[c] = 0;
        if (c < ncand) first_leaf(F, cp[c], o, d, inv, tmin0, tmax0, rtmax, key[c], pos[c], steps);
      }
    }
#if WR_TIE_SPLIT
    if (split) split[1] += static_cast<uint32_t>(wall_clock64() - a1);
#endif
#pragma unroll
    for (int c = 0; c < kTie; ++c)
      if (c < ncand && key[c] != ~0ull && m == WR_INF) m = ct[c];  // sorted by t: the first visited one
    if (pass == 0 && m == t1) break;  // the window t1 + 3 EPS is complete when n <= kTie
  }
  dbg = n;
  const int nc = min(n, kTie);
  if (m == WR_INF && n <= kTie) {  // every hit is known and none is visited: the reference misses
    t_out = WR_INF;
    p_out = -1;
    dbg |= 1 << 8;
    return true;
  }
  // m < 4096: fl(m + 3 EPS) is within EPS / 4 of m + 3 EPS
  if (!(m < 4096.f)) {
    dbg |= 3 << 16;
    return false;
  }
  const float lim = m + 3.f * WR_EPS;
  if (n > kTie && !(ct[kTie - 1] > lim)) {  // hits up to m + 3 EPS may be missing
    dbg |= 4 << 16;
    return false;
  }
  bool band = false;
#pragma unroll
  for (int c = 0; c < kTie; ++c)
    if (c < nc && key[c] != ~0ull && ct[c] <= lim && ct[c] - m > 1.5f * WR_EPS) band = true;  // exact difference
  if (band) {
    dbg |= 5 << 16;
    return false;
  }
  // first-found-wins over the visited candidates up to m + 1.5 EPS, in visit
  // order: each candidate's rank, then the rule rank by rank (compile-time
  // indices only: the lists stay in registers)
  bool use[kTie];
#pragma unroll
  for (int c = 0; c < kTie; ++c) use[c] = c < nc && key[c] != ~0ull && ct[c] - m <= 1.5f * WR_EPS;
  int rank[kTie];
#pragma unroll
  for (int c = 0; c < kTie; ++c) {
    rank[c] = 0;
#pragma unroll
    for (int e = 0; e < kTie; ++e)
      if (e != c && use[c] && use[e] && (key[e] < key[c] || (key[e] == key[c] && pos[e] < pos[c]))) ++rank[c];
  }
  float best = WR_INF;
  int win = -1;
#pragma unroll
  for (int k = 0; k < kTie; ++k) {
#pragma unroll
    for (int c = 0; c < kTie; ++c) {
      if (use[c] && rank[c] == k && cmpf(ct[c] - best) < 0) {
        best = ct[c];
        win = cp[c];
      }
    }
  }
  dbg |= 1 << 8;
  t_out = best;
  p_out = win;
  return true;
}

// launch index -> (queue, index in it), as k_trace numbers a launch's rays
struct QueueIndex {
  int qend[kMaxQueues];
  int n;
  __device__ __forceinline__ explicit QueueIndex(const TraceQueues& Q) {
    int acc = 0;
#pragma unroll
    for (int i = 0; i < kMaxQueues; ++i) {
      // (a shadow queue's count may pass its capacity: the appends past it were
      // dropped and the render is redone, BdptBuf)
      if (i < Q.n && Q.q[i].count) acc += min(*Q.q[i].count + (Q.q[i].count2 ? *Q.q[i].count2 : 0), Q.q[i].cap);
      qend[i] = acc;
    }
    n = acc;
  }
  __device__ __forceinline__ void locate(int idx, int& q, int& r) const {
    q = 0;
    int q0 = 0;
#pragma unroll
    for (int i = 0; i < kMaxQueues - 1; ++i)
      if (idx >= qend[i]) {
        q = i + 1;
        q0 = qend[i];
      }
    r = idx - q0;
  }
};
#ifndef WR_QFIELD_SGPR
#define WR_QFIELD_SGPR 1
#endif
#ifndef WR_QFIELD_GLOBAL
#define WR_QFIELD_GLOBAL 1
#endif
// a wave-uniform value forced into scalar registers (readfirstlane)
template <class T>
__device__ __forceinline__ T sgpr_value(T v) {
  if constexpr (sizeof(T) == 8) {
    unsigned long long u;
    __builtin_memcpy(&u, &v, 8);
    const unsigned lo = static_cast<unsigned>(__builtin_amdgcn_readfirstlane(static_cast<int>(u & 0xffffffffull)));
    const unsigned hi = static_cast<unsigned>(__builtin_amdgcn_readfirstlane(static_cast<int>(u >> 32)));
    u = (static_cast<unsigned long long>(hi) << 32) | lo;
    if constexpr (WR_QFIELD_GLOBAL && std::is_pointer_v<T>) {
      // queue arrays are global memory: the pointer is rebuilt in the global
      // address space, so that the loads and stores through it stay global
      // (a generic pointer makes them flat, which also wait on the LDS counter)
      using G = __attribute__((address_space(1))) std::remove_pointer_t<T>*;
      return (T)(reinterpret_cast<G>(u));
    } else {
      T r;
      __builtin_memcpy(&r, &u, 8);
      return r;
    }
  } else {
    static_assert(sizeof(T) == 4, "4- or 8-byte queue fields");
    int u;
    __builtin_memcpy(&u, &v, 4);
    u = __builtin_amdgcn_readfirstlane(u);
    T r;
    __builtin_memcpy(&r, &u, 4);
    return r;
  }
}
// A queue's field for the lane's queue q.  Each queue's value is uniform and
// taken into scalar registers before the per-lane select (WR_QFIELD_SGPR):
// left to itself the compiler turns the select into a per-lane load from the
// kernel-argument block, a vector-memory round trip before each ray's own
// loads (refill) and stores (results).
template <class Fn>
__device__ __forceinline__ auto qfield(const TraceQueues& Q, int q, Fn field) {
#if WR_QFIELD_SGPR
  auto v = sgpr_value(field(Q.q[0]));
#pragma unroll
  for (int i = 1; i < kMaxQueues; ++i) {
    const auto w = sgpr_value(field(Q.q[i]));
    if (q == i) v = w;
  }
#else
  auto v = field(Q.q[0]);
#pragma unroll
  for (int i = 1; i < kMaxQueues; ++i)
    if (q == i) v = field(Q.q[i]);
#endif
  return v;
}

// the search's near-tie mark on a hit primitive (queue out_prim, between the
// search and k_fast_resolve, which clears it; scenes have < 2^30 primitives)
constexpr int kTieMark = 1 << 30;
// ... and its grazing mark: the ray runs nearly in the plane of a triangle the
// search tested (tri_grazes), on a hit primitive, or kGrazeMiss for a ray
// without a hit (scenes have < 2^29 primitives)
constexpr int kGrazeMark = 1 << 29;
constexpr int kGrazeMiss = -3;
__device__ __forceinline__ int unmark(int p) {
  return p >= 0 ? (p & ~(kTieMark | kGrazeMark)) : (p == kGrazeMiss ? -1 : p);
}
__device__ __forceinline__ bool graze_marked(int p) { return p >= 0 ? (p & kGrazeMark) != 0 : p == kGrazeMiss; }
// Does the ray run inside the triangle's plane?  Triangle::hit's denominator
// (triangle.cpp:43-44) within kGrazeRel of the magnitude of its products (the
// direction nearly parallel to the plane) AND its t numerator within
// kGrazePlaneRel of its products' (the origin nearly on the plane).  There
// Cramer's rule divides rounding noise by rounding noise: the reference can
// accept a triangle of that plane at a noise t although the ray passes
// outside its grown box -- one the search never visits (the
// near-grazing case; the probe in tests/test_gpu_bvh.py found such rays only
// with the origin on the plane: a ray parallel to a plane but off it gets a
// t far beyond any other hit).  A ray inside a plane runs through the
// triangles of that plane near its origin, so the search tests one of them
// (the one the origin lies on) and the ray takes the KD walk.  A..F as in
// tri_test, p0 = a.xyz.
#ifndef WR_GRAZE_REL
#define WR_GRAZE_REL 1e-5f
#endif
#ifndef WR_GRAZE_PLANE_REL
#define WR_GRAZE_PLANE_REL 1e-3f
#endif
constexpr float kGrazeRel = WR_GRAZE_REL, kGrazePlaneRel = WR_GRAZE_PLANE_REL;
__device__ __forceinline__ bool tri_grazes(float4 a, float4 b, float f, V3 o, V3 dir) {
  const float A = a.w, B = b.x, C = b.y, D = b.z, E = b.w, F = f;
  const float G = dir.x, H = dir.y, I = dir.z;
  const float J = a.x - o.x, K = a.y - o.y, L = a.z - o.z;
  const float EIHF = E * I - H * F, GFDI = G * F - D * I, DHEG = D * H - E * G;
  const float den = A * EIHF + B * GFDI + C * DHEG;
  const float mag = fabsf(A) * (fabsf(E * I) + fabsf(H * F)) + fabsf(B) * (fabsf(G * F) + fabsf(D * I)) +
                    fabsf(C) * (fabsf(D * H) + fabsf(E * G));
  const float AKJB = A * K - J * B, JCAL = J * C - A * L, BLKC = B * L - K * C;
  const float tnum = F * AKJB + E * JCAL + D * BLKC;
  const float tmag = fabsf(F) * (fabsf(A * K) + fabsf(J * B)) + fabsf(E) * (fabsf(J * C) + fabsf(A * L)) +
                     fabsf(D) * (fabsf(B * L) + fabsf(K * C));
  return fabsf(den) <= kGrazeRel * mag && fabsf(tnum) <= kGrazePlaneRel * tmag;
}

// one atomic per wave: this lane's slot in a list (or -1 if !want)
__device__ __forceinline__ int fast_append(int* counter, bool want) {
  const unsigned long long m = __ballot(want);
  if (m == 0ull) return -1;
  const int lane = __lane_id();
  const int leader = __ffsll(static_cast<unsigned long long>(m)) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(counter, __popcll(m));
  base = __shfl(base, leader);
  return want ? base + __popcll(m & ((1ull << lane) - 1ull)) : -1;
}
// The resolve's first membership test (resolve_fast): is one of the first
// four KD leaf cells of the winner p1 (its PrimRec) crossed by the ray within
// the witness margin?  Then the reference's walk visits a leaf holding p1.
__device__ __forceinline__ bool first_cells_crossed(const FastScene& F, int p1, V3 o, V3 d, V3 binv, float rtmax) {
  const float4* pr = F.prim_rec + 8 * static_cast<size_t>(p1);
  const float4 c0 = pr[0], c1 = pr[1], c2 = pr[2], c3 = pr[3], c4 = pr[4], c5 = pr[5];
  return box_crossed_with_margin(c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, o, d, binv, rtmax) ||
         box_crossed_with_margin(c1.z, c1.w, c2.x, c2.y, c2.z, c2.w, o, d, binv, rtmax) ||
         box_crossed_with_margin(c3.x, c3.y, c3.z, c3.w, c4.x, c4.y, o, d, binv, rtmax) ||
         box_crossed_with_margin(c4.z, c4.w, c5.x, c5.y, c5.z, c5.w, o, d, binv, rtmax);
}

// RL (the resolve list): a finished ray whose answer needs no more -- a miss,
// or an unmarked winner that first_cells_crossed proves -- is settled here;
// the others (near-ties, grazing rays, winners proven by neither of those
// cells) are listed by launch index in rlist for k_fast_resolve, which then
// reads those rays only.  The test is the resolve's own, on the same floats.
template <bool COUNT, int W, bool SPH, bool RL = false>
__device__ __forceinline__ void trace_fast(const DevScene& S, const FastScene& F, const TraceQueues& Q, int* fetch,
                                           float* t2buf, int2* pairs, int2* spill, uint32_t* lds, FastCounters& ctr,
                                           int bid, int nblk,  // this block's index among the launch's nblk search blocks
                                           int* rlist = nullptr, int* rlist_n = nullptr) {
  constexpr int kLdsStack = SearchStack<W>::lds;
  constexpr bool kSearchSpills = SearchStack<W>::spills;
  const int lane = __lane_id();
  int* stk_link = reinterpret_cast<int*>(lds) + lane;
  uint16_t* stk_t = reinterpret_cast<uint16_t*>(reinterpret_cast<int*>(lds) + min(F.sdepth, kLdsStack) * 64) + lane;
  const size_t gl = static_cast<size_t>(nblk) * 64, gidx = static_cast<size_t>(bid) * 64 + lane;
  const QueueIndex QI(Q);
  const int n = QI.n;
  // Waves past the ones the rays need leave before touching the shared cursor:
  // the first reservations cover every index, and a launch of few rays (a
  // late bounce) no longer pays one device-scope atomic on a single address
  // per resident wave (5,120 of them: ~150 us per launch, measured)
  // A launch of at most one ray per resident lane reserves 64 at a time (one
  // ray per lane: the launch lasts one ray's traversal, not two)
#ifndef WR_GRAB_ADAPT
#define WR_GRAB_ADAPT 1
#endif
  const int grab = WR_GRAB_ADAPT && n <= 64 * nblk ? 64 : kRayGrab;
  if (bid * grab >= n) return;
  int r = -1, qi = 0, lidx = 0;
  bool pool = true;
  int pb = 0, pe = 0;
  V3 o = v3(0.f, 0.f, 0.f), d = o, binv = o;
  V3 cl = o, ch = o;  // slab offsets -(o + g) binv, -(o - g) binv for the current margin g
  float rtmin = 0.f, rtmax = WR_INF, t1 = WR_INF, t2 = WR_INF, tcap = 0.f, dlen = 1.f, olen = 0.f;
  float t3 = WR_INF;  // the third smallest hit (kPairWindow)
  int p2 = -1;        // the second smallest hit's primitive
  float lo_t = 0.f, hi_t = 0.f;
  int p1 = -1, sp = 0;
  bool gz = false;          // the ray grazes a tested triangle's plane (tri_grazes)
  uint32_t rn = 0, rt = 0;  // COUNT: this ray's node visits / tests
  int cur = 0;  // >= 0 inner node to visit; < 0 leaf link to test; kDone when finished
  int pl = 0;   // WR_BVH_SPEC: parked leaf link (< 0), or 0
  constexpr int kDone = 0x7fffffff;
  // RL: the listed rays gather in a 64-entry LDS buffer behind the stack and go
  // to rlist 64 at a time (one atomic per 64 listed rays, not per wave round)
  int* const lbuf = reinterpret_cast<int*>(lds) + search_lds_bytes(F.sdepth, W) / 4;
  int nlb = 0;
  bool listed = false;
  auto flush_list = [&]() {
    if (nlb == 0) return;
    int base = 0;
    if (lane == 0) base = atomicAdd(rlist_n, nlb);
    base = __builtin_amdgcn_readfirstlane(base);
    if (lane < nlb) rlist[base + lane] = lbuf[lane];
    nlb = 0;
  };
  auto reserve = [&](bool want) -> int {
    const unsigned long long m = __ballot(want);
    const int need = __popcll(m);
    const int rank = __popcll(m & ((1ull << lane) - 1ull));
    int idx = pb + rank;
    if (need == 0) return idx;
    if (pe - pb < need) {
      int got = 0;
      if (lane == 0) got = atomicAdd(fetch, grab);
      got = __builtin_amdgcn_readlane(got, 0);
      const int rem = pe - pb;
      if (rank >= rem) idx = got + (rank - rem);
      pb = got + (need - rem);
      pe = got + grab;
    } else {
      pb += need;
    }
    return idx;
  };
  // the search window: hits up to t1 + 3 EPS (the tie resolution's first
  // window: a near-tie whose window holds two hits leaves with both, kPairWindow),
  // and rtmax
  auto bound = [&]() { return fminf(rtmax, t1 + 3.f * WR_EPS); };
  // the ray's box margin g (space) and the node test's constants for it.  A
  // box face x is tested as fma(x, binv, -(o -+ g) binv): the product
  // (o -+ g) binv is rounded once, an error of < 1 ulp of |o| |binv| in t, i.e.
  // < 1.2e-7 |o| in space, covered by the 1e-6 |o| term of g
  auto margins = [&]() {
    const float tc = fminf(bound(), tcap);
    const float g = wrf::kRayGrow * (tc * dlen + 1.f) + 1e-6f * olen;
    const float gt = g / dlen;
    lo_t = rtmin - gt;
    hi_t = bound() + gt;
    cl = v3(-(o.x + g) * binv.x, -(o.y + g) * binv.y, -(o.z + g) * binv.z);
    ch = v3(-(o.x - g) * binv.x, -(o.y - g) * binv.y, -(o.z - g) * binv.z);
  };
  auto push = [&](int link, float t) {
    if (!kSearchSpills || sp < kLdsStack) {
      stk_link[sp * 64] = link;
      stk_t[sp * 64] = t_down16(t);
    } else {
      spill[static_cast<size_t>(sp - kLdsStack) * gl + gidx] = make_int2(link, __float_as_int(t));
    }
    ++sp;
  };
  auto pop = [&]() {
    cur = kDone;
    while (sp > 0) {
      --sp;
      int link;
      float te;
      if (!kSearchSpills || sp < kLdsStack) {
        link = stk_link[sp * 64];
        te = t_up32(stk_t[sp * 64]);
#if WR_POP_TOGETHER
        // the link is read with the entry's t, not after its test: one LDS
        // round trip per entry instead of two on the search's chain
        asm volatile("" : : "v"(link), "v"(te));
#endif
      } else {
        const int2 e = spill[static_cast<size_t>(sp - kLdsStack) * gl + gidx];
        link = e.x;
        te = __int_as_float(e.y);
      }
      if (te <= hi_t) {
        cur = link;
        break;
      }
    }
  };
  for (;;) {
    // ---- refill idle lanes
    if (pool) {
      const bool idle = r < 0;
      if (__ballot(idle)) {
        const int idx = reserve(idle);
        const bool take = idle && idx < n;
        if (take) {
          lidx = idx;
          QI.locate(idx, qi, r);
          const float* o3 = qfield(Q, qi, [](const RayQueue& x) { return x.o3; });
          const float* d3 = qfield(Q, qi, [](const RayQueue& x) { return x.d3; });
          const int cap = qfield(Q, qi, [](const RayQueue& x) { return x.cap; });
          const float* tmn = qfield(Q, qi, [](const RayQueue& x) { return x.tmin; });
          const float* tmx = qfield(Q, qi, [](const RayQueue& x) { return x.tmax; });
          o = v3(o3[r], o3[cap + r], o3[2 * cap + r]);
          d = v3(d3[r], d3[cap + r], d3[2 * cap + r]);
          rtmin = tmn ? tmn[r] : 0.f;
          rtmax = tmx ? tmx[r] : WR_INF;
          binv = v3(clamp_inv(d.x), clamp_inv(d.y), clamp_inv(d.z));
          dlen = sqrtf(d.x * d.x + d.y * d.y + d.z * d.z);
          if (!(dlen > 0.f)) dlen = 1.f;
          t1 = WR_INF;
          t2 = WR_INF;
          t3 = WR_INF;
          p1 = -1;
          p2 = -1;
          gz = false;
          sp = 0;
          cur = 0;
          rn = rt = 0;
          // exit of the union box: caps the search margin before the first hit
          const float ax = (F.lo.x - o.x) * binv.x, bx = (F.hi.x - o.x) * binv.x;
          const float ay = (F.lo.y - o.y) * binv.y, by = (F.hi.y - o.y) * binv.y;
          const float az = (F.lo.z - o.z) * binv.z, bz = (F.hi.z - o.z) * binv.z;
          tcap = fmaxf(0.f, fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz)));
          olen = fabsf(o.x) + fabsf(o.y) + fabsf(o.z);
          margins();
          // spheres: their boxes cover Sphere::hit's rounding for origins in
          // [org_lo, org_hi] only (wr_bvh.cpp): a ray from elsewhere (an API
          // caller's) takes the KD walk
          if (SPH) gz = !(o.x >= F.org_lo.x && o.y >= F.org_lo.y && o.z >= F.org_lo.z && o.x <= F.org_hi.x &&
                          o.y <= F.org_hi.y && o.z <= F.org_hi.z);
        }
        if (__ballot(idle && idx >= n)) pool = false;
      }
    }
    const bool act = r >= 0;
    if (!__ballot(act)) {
      if (!pool) break;
      continue;
    }
    // ---- inner nodes until this lane has a leaf (or is done).  WR_BVH_SPEC: a
    // leaf reached is parked in `pl` and the lane descends on (its next inner
    // nodes) until every lane has parked one or finished
    for (;;) {
#if WR_BVH_SPEC
      if (!__ballot(act && pl >= 0 && cur != kDone)) break;
      if (act && cur < 0 && pl >= 0) {
        pl = cur;
        pop();
      }
      const bool step = act && cur >= 0 && cur != kDone;
#else
      const bool step = act && cur >= 0 && cur != kDone;
      if (!__ballot(step)) break;
#endif
      if (step) {
        if (COUNT) {
          ++ctr.nodes;
          ++rn;
        }
        if constexpr (W == 4) {
        // a 4-wide node: the four boxes, then the hit children nearest first
        // (the nearest is visited next, the others pushed farthest first)
#if WR_BVH4_QUANT
        // wrf::BNode4Q: the child boxes decoded from bytes, fmaf(q, scale,
        // org) -- each contains the binary tree's box, bit for bit checked
        // by the build -- then tested as below; an unused slot never hits
        const float4* np = F.nodes4 + 4 * static_cast<size_t>(cur);
        const float4 h0 = np[0], h1 = np[1], h2 = np[2];
        const int4 lk = *reinterpret_cast<const int4*>(np + 3);
        const uint32_t qlx = __float_as_uint(h1.z), qly = __float_as_uint(h1.w), qlz = __float_as_uint(h2.x);
        const uint32_t qhx = __float_as_uint(h2.y), qhy = __float_as_uint(h2.z), qhz = __float_as_uint(h2.w);
        auto dq = [](uint32_t w, int k, float sc, float org) {
          return fmaf(static_cast<float>((w >> (8 * k)) & 255u), sc, org);
        };
        auto slabq = [&](int k, int link) {
          const float lx = dq(qlx, k, h0.w, h0.x), ly = dq(qly, k, h1.x, h0.y), lz = dq(qlz, k, h1.y, h0.z);
          const float hx = dq(qhx, k, h0.w, h0.x), hy = dq(qhy, k, h1.x, h0.y), hz = dq(qhz, k, h1.y, h0.z);
          const float x0 = fmaf(lx, binv.x, cl.x), x1 = fmaf(hx, binv.x, ch.x);
          const float y0 = fmaf(ly, binv.y, cl.y), y1 = fmaf(hy, binv.y, ch.y);
          const float z0 = fmaf(lz, binv.z, cl.z), z1 = fmaf(hz, binv.z, ch.z);
          const float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), lo_t));
          const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), hi_t));
          return (tn <= tf && link != wrf::kEmptyLink) ? tn : __int_as_float(0x7f800000);
        };
        float k0 = slabq(0, lk.x);
        float k1 = slabq(1, lk.y);
        float k2 = slabq(2, lk.z);
        float k3 = slabq(3, lk.w);
#else
        const float4* np = F.nodes4 + 8 * static_cast<size_t>(cur);
        const float4 bx0 = np[0], by0 = np[1], bz0 = np[2], bx1 = np[3], by1 = np[4], bz1 = np[5];
        const int4 lk = *reinterpret_cast<const int4*>(np + 6);
        auto slab4 = [&](float lx, float ly, float lz, float hx, float hy, float hz) {
          const float x0 = fmaf(lx, binv.x, cl.x), x1 = fmaf(hx, binv.x, ch.x);
          const float y0 = fmaf(ly, binv.y, cl.y), y1 = fmaf(hy, binv.y, ch.y);
          const float z0 = fmaf(lz, binv.z, cl.z), z1 = fmaf(hz, binv.z, ch.z);
          const float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), lo_t));
          const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), hi_t));
          return tn <= tf ? tn : __int_as_float(0x7f800000);  // miss: +inf (a hit's tn <= hi_t is finite)
        };
        float k0 = slab4(bx0.x, by0.x, bz0.x, bx1.x, by1.x, bz1.x);
        float k1 = slab4(bx0.y, by0.y, bz0.y, bx1.y, by1.y, bz1.y);
        float k2 = slab4(bx0.z, by0.z, bz0.z, bx1.z, by1.z, bz1.z);
        float k3 = slab4(bx0.w, by0.w, bz0.w, bx1.w, by1.w, bz1.w);
#endif
        int l0 = lk.x, l1 = lk.y, l2 = lk.z, l3 = lk.w;
        const int nh = (k0 < __int_as_float(0x7f800000)) + (k1 < __int_as_float(0x7f800000)) +
                       (k2 < __int_as_float(0x7f800000)) + (k3 < __int_as_float(0x7f800000));
        auto cswap = [](float& ta, int& la, float& tb, int& lb) {
          const bool s = tb < ta;
          const float t = s ? tb : ta;
          tb = s ? ta : tb;
          ta = t;
          const int l = s ? lb : la;
          lb = s ? la : lb;
          la = l;
        };
        cswap(k0, l0, k1, l1);
        cswap(k2, l2, k3, l3);
        cswap(k0, l0, k2, l2);
        cswap(k1, l1, k3, l3);
        cswap(k1, l1, k2, l2);
        if (nh == 0) {
          pop();
        } else {
          if (nh > 3) push(l3, k3);
          if (nh > 2) push(l2, k2);
          if (nh > 1) push(l1, k1);
          cur = l0;
        }
        } else if constexpr (W == 8) {
        // an 8-wide node (wrf::BNode8, one 128-byte line): the eight child
        // boxes decoded from bytes, fmaf(q, scale, org) -- the build made each
        // contain the binary tree's box, bit for bit checked -- and tested as
        // above; the children hit, nearest first: the nearest is visited next,
        // the others pushed farthest first
        const float4* np = F.nodes8 + 8 * static_cast<size_t>(cur);
        const float4 h0 = np[0], h1 = np[1];
        const int4 la = *reinterpret_cast<const int4*>(np + 2), lb = *reinterpret_cast<const int4*>(np + 3);
        const uint4 q0 = *reinterpret_cast<const uint4*>(np + 4), q1 = *reinterpret_cast<const uint4*>(np + 5),
                    q2 = *reinterpret_cast<const uint4*>(np + 6);
        const int nch = __float_as_int(h1.z);
        const float inf = __int_as_float(0x7f800000);
        float tk[8];
        int lk8[8] = {la.x, la.y, la.z, la.w, lb.x, lb.y, lb.z, lb.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int sh = 8 * (i & 3);
          auto dq = [&](uint32_t w, float sc, float org) {
            return fmaf(static_cast<float>((w >> sh) & 255u), sc, org);
          };
          const float lx = dq(i < 4 ? q0.x : q0.y, h0.w, h0.x), ly = dq(i < 4 ? q0.z : q0.w, h1.x, h0.y),
                      lz = dq(i < 4 ? q1.x : q1.y, h1.y, h0.z);
          const float hx = dq(i < 4 ? q1.z : q1.w, h0.w, h0.x), hy = dq(i < 4 ? q2.x : q2.y, h1.x, h0.y),
                      hz = dq(i < 4 ? q2.z : q2.w, h1.y, h0.z);
          const float x0 = fmaf(lx, binv.x, cl.x), x1 = fmaf(hx, binv.x, ch.x);
          const float y0 = fmaf(ly, binv.y, cl.y), y1 = fmaf(hy, binv.y, ch.y);
          const float z0 = fmaf(lz, binv.z, cl.z), z1 = fmaf(hz, binv.z, ch.z);
          const float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), lo_t));
          const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), hi_t));
          tk[i] = (tn <= tf && i < nch) ? tn : inf;  // miss: +inf (a hit's tn <= hi_t is finite)
        }
        auto cswap = [&](int a, int b) {
          const bool s = tk[b] < tk[a];
          const float t = s ? tk[b] : tk[a];
          tk[b] = s ? tk[a] : tk[b];
          tk[a] = t;
          const int l = s ? lk8[b] : lk8[a];
          lk8[b] = s ? lk8[a] : lk8[b];
          lk8[a] = l;
        };
        // 19-comparator sorting network for 8 keys
        cswap(0, 2); cswap(1, 3); cswap(4, 6); cswap(5, 7);
        cswap(0, 4); cswap(1, 5); cswap(2, 6); cswap(3, 7);
        cswap(0, 1); cswap(2, 3); cswap(4, 5); cswap(6, 7);
        cswap(2, 4); cswap(3, 5);
        cswap(1, 4); cswap(3, 6);
        cswap(1, 2); cswap(3, 4); cswap(5, 6);
        int nh = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) nh += tk[i] < inf ? 1 : 0;
        if (nh == 0) {
          pop();
        } else {
#pragma unroll
          for (int i = 7; i >= 1; --i)
            if (i < nh) push(lk8[i], tk[i]);
          cur = lk8[0];
        }
        } else {
        const float4* np = F.nodes + 4 * static_cast<size_t>(cur);
        const float4 n0 = np[0], n1 = np[1], n2 = np[2];
        const int4 lk = *reinterpret_cast<const int4*>(np + 3);
        auto slab = [&](float lx, float ly, float lz, float hx, float hy, float hz, float& tn) {
          const float x0 = fmaf(lx, binv.x, cl.x), x1 = fmaf(hx, binv.x, ch.x);
          const float y0 = fmaf(ly, binv.y, cl.y), y1 = fmaf(hy, binv.y, ch.y);
          const float z0 = fmaf(lz, binv.z, cl.z), z1 = fmaf(hz, binv.z, ch.z);
          tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), lo_t));
          const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), hi_t));
          return tn <= tf;
        };
        float ta, tb;
        const bool ha = slab(n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, ta);
        const bool hb = slab(n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, tb);
        if (ha && hb) {
          const bool af = ta <= tb;
          push(af ? lk.y : lk.x, af ? tb : ta);
          cur = af ? lk.x : lk.y;
        } else if (ha) {
          cur = lk.x;
        } else if (hb) {
          cur = lk.y;
        } else {
          pop();
        }
        }
      }
    }
    // ---- leaf: test its triangles (Triangle::hit), keep (t1, p1) and t2
#if WR_BVH_SPEC
    if (act && pl < 0) {
      const int l = ~pl;
      pl = 0;
#else
    if (act && cur < 0) {
      const int l = ~cur;
#endif
      const int first = l >> 3, cnt = (l & 7) + 1;
      // all records of the leaf requested before the first test
      float4 ta[wrf::kMaxLeaf], tb[wrf::kMaxLeaf], tc[wrf::kMaxLeaf];
#pragma unroll
      for (int j = 0; j < wrf::kMaxLeaf; ++j) {
        const float4* tp = F.tris + 3 * static_cast<size_t>(first + min(j, cnt - 1));
        ta[j] = tp[0];
        tb[j] = tp[1];
        tc[j] = tp[2];
      }
#if WR_LEAF_SCHED
      // every record load issued before the first test (the scheduler would
      // otherwise start the first test, and wait for its record, before the
      // second record's loads: two round trips per leaf instead of one)
      __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
      for (int j = 0; j < wrf::kMaxLeaf; ++j) {
        if (j >= cnt) break;
        if (COUNT) {
          ++ctr.tests;
          ++rt;
        }
        float t;
        int pr = __float_as_int(tc[j].y);
        bool hit;
        if (SPH && pr < 0) {  // a sphere: Sphere::hit, the same floats (no plane to graze)
          pr = -pr - 1;
          hit = sph_hit(S, pr, o, d, rtmin, rtmax, t);
        } else {
          gz |= tri_grazes(ta[j], tb[j], tc[j].x, o, d);
          // screen against t1 + 4 EPS: every hit with t <= t1 + 3 EPS survives
          hit = tri_test(ta[j], tb[j], tc[j].x, o, d, rtmin, rtmax, t1 + 4.f * WR_EPS, t);
        }
        if (hit) {
          if (t < t1) {
            t3 = t2;
            t2 = t1;
            p2 = p1;
            t1 = t;
            p1 = pr;
          } else if (t < t2) {
            t3 = t2;
            t2 = t;
            p2 = pr;
          } else if (t < t3) {
            t3 = t;
          }
        }
      }
      margins();
#if !WR_BVH_SPEC
      pop();
#endif
    }
    // ---- finished rays: the candidate goes to k_fast_resolve
    if (act && cur == kDone && pl >= 0) {
      if (COUNT) {
        ctr.max_nodes = max(ctr.max_nodes, rn);
        ctr.max_tests = max(ctr.max_tests, rt);
        ctr.long_rays += rn > 256u ? 1u : 0u;
      }
      // a near-tie (t2 within EPS of t1: the reference's first-found rule may
      // pick another hit) travels as a mark on p1 instead of t2 itself -- 4
      // bytes per ray less written here and read by k_fast_resolve.  The
      // diagnostic probes (F.diag) keep t2, as they may skip the kernels that
      // clear the mark.
      int po = p1;
      if (F.diag) {
        t2buf[lidx] = t2;
      } else if (p1 >= 0 && !(cmpf(t2 - t1) > 0 && cmpf(t1 - WR_INF) < 0)) {
        po = p1 | kTieMark;
        // every hit up to t1 + 3 EPS was seen (the window above): when the
        // third lies beyond the tie resolution's first window, its collection
        // would return exactly (t1, p1), (t2, p2) -- they travel with the ray
        const bool two = t3 > fminf(rtmax, t1 + 3.f * WR_EPS);
        pairs[lidx] = two ? make_int2(p2, __float_as_int(t2)) : make_int2(-1, 0);
      }
      if (gz) po = po >= 0 ? (po | kGrazeMark) : kGrazeMiss;
      qfield(Q, qi, [](const RayQueue& x) { return x.out_t; })[r] = p1 >= 0 ? t1 : WR_INF;
      qfield(Q, qi, [](const RayQueue& x) { return x.out_prim; })[r] = po;
      if constexpr (RL) {
        listed = po != p1;  // marked: a near-tie or a grazing ray
        if (!listed && p1 >= 0) listed = !first_cells_crossed(F, p1, o, d, binv, rtmax);
      }
      r = -1;
    }
    if constexpr (RL) {  // (wave-uniform) the listed rays into the wave's buffer
      const unsigned long long m = __ballot(listed);
      if (m) {
        const int k = __popcll(m);
        if (nlb + k > 64) flush_list();
        if (listed) lbuf[nlb + __popcll(m & ((1ull << lane) - 1ull))] = lidx;
        nlb += k;
        listed = false;
      }
    }
  }
  if constexpr (RL) flush_list();
}

// tie-list entries: launch index, | kWalkEntry for a ray the KD walk settles,
// | kTieEntry for a near-tie (its pair record is the search's)
constexpr int kWalkEntry = 1 << 30;
constexpr int kTieEntry = 1 << 29;
// k_fast_resolve: one ray per lane (grid-stride over the launch's indices).
// The rare rays it cannot settle (near-ties, t1 not reached) go to `hard` for
// k_fast_hard, so that their register-hungry code does not lower this
// kernel's occupancy.
template <bool COUNT>
__device__ __forceinline__ void resolve_fast(const DevScene& S, const FastScene& F, const TraceQueues& Q,
                                             const float* t2buf, int* hard, int* hard_n, int hcap,
                                             FastCounters& ctr, const int* rlist = nullptr,
                                             const int* rlist_n = nullptr) {
  const int lane = __lane_id();
  const QueueIndex QI(Q);
  // the search's list (RL), or every ray of the launch
  const int nr = rlist ? min(*rlist_n, QI.n) : QI.n;
  // the capacity diagnostics (wrong answers, never valid indices): the rays a
  // skipped kernel would settle keep the search's winner, its marks cleared
  // (a marked primitive would index past the scene in the vertex kernels)
  if (F.diag & 16) {
    for (int idx = blockIdx.x * 64 + lane; idx < QI.n; idx += gridDim.x * 64) {
      int q = 0, r = 0;
      QI.locate(idx, q, r);
      int* op = qfield(Q, q, [](const RayQueue& x) { return x.out_prim; });
      op[r] = unmark(op[r]);
    }
    return;
  }
  // every lane of the wave takes part in each list append (whole iterations)
  for (int base = blockIdx.x * 64; base < nr; base += gridDim.x * 64) {
    const int idx = base + lane < nr ? (rlist ? rlist[base + lane] : base + lane) : QI.n;
    bool need = false, scan = false, big_tie = false, walk = false, pair_tie = false, lane_pair = false;
    int q = 0, r = 0, p1 = -1;
    float t1 = WR_INF;
    V3 o = v3(0.f, 0.f, 0.f), d = v3(0.f, 0.f, 0.f);
    if (idx < QI.n) {
      QI.locate(idx, q, r);
      // every load that does not depend on p1 in flight at once
      const int pm = qfield(Q, q, [](const RayQueue& x) { return x.out_prim; })[r];
      p1 = unmark(pm);
      t1 = qfield(Q, q, [](const RayQueue& x) { return x.out_t; })[r];
      const float t2 = F.diag ? t2buf[idx] : 0.f;
      const float* o3 = qfield(Q, q, [](const RayQueue& x) { return x.o3; });
      const float* d3 = qfield(Q, q, [](const RayQueue& x) { return x.d3; });
      const int cap = qfield(Q, q, [](const RayQueue& x) { return x.cap; });
      const float* tmx = qfield(Q, q, [](const RayQueue& x) { return x.tmax; });
      o = v3(o3[r], o3[cap + r], o3[2 * cap + r]);
      d = v3(d3[r], d3[cap + r], d3[2 * cap + r]);
      const float rtmax = tmx ? tmx[r] : WR_INF;
      // p1's membership record: one line with its first four leaves' cells
      const float4* pr = F.prim_rec + 8 * static_cast<size_t>(max(p1, 0));
      const float4 c0 = pr[0], c1 = pr[1], c2 = pr[2], c3 = pr[3], c4 = pr[4], c5 = pr[5];
      if (graze_marked(pm) || (F.diag & 256)) {  // (diag 256: every ray, a test of the walks)
        // the ray runs within ~1e-5 (relative) of the plane of a triangle the
        // search tested (the winner among them): Cramer's rule is near its
        // rounding noise there, beyond the search margins' reach (DESIGN.md
        // 4b, margins) -- the KD walk settles it
        need = true;
        walk = true;
      } else if (p1 >= 0) {  // (no hit anywhere: a miss for the reference too)
        const bool tie = F.diag ? !(cmpf(t2 - t1) > 0 && cmpf(t1 - WR_INF) < 0) : (pm & kTieMark) != 0;
        if (tie) {
          // a tie on a many-leaf primitive (walls, floors: up to thousands of
          // leaves) is resolved by one wave (scan list, marked), the others
          // one per lane
          const bool big = WR_TIE_WAVE_ALL || F.prim_leaf_off[p1 + 1] - F.prim_leaf_off[p1] > kTieLeaves;
          need = !big;
          pair_tie = !F.diag && F.pair > 0;
          if (need && pair_tie && F.pair > 1) {
            const int2 pr2 = reinterpret_cast<const int2*>(hard + hcap)[idx];
            if (pr2.x >= 0 && F.prim_leaf_off[pr2.x + 1] - F.prim_leaf_off[pr2.x] <= kTieLeaves) {
              lane_pair = true;
              need = false;
            }
          }
          scan = big;
          big_tie = big;
        } else if (!(F.diag & 8)) {
          const V3 binv = v3(clamp_inv(d.x), clamp_inv(d.y), clamp_inv(d.z));
          const bool seen = box_crossed_with_margin(c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, o, d, binv, rtmax) ||
                            box_crossed_with_margin(c1.z, c1.w, c2.x, c2.y, c2.z, c2.w, o, d, binv, rtmax) ||
                            box_crossed_with_margin(c3.x, c3.y, c3.z, c3.w, c4.x, c4.y, o, d, binv, rtmax) ||
                            box_crossed_with_margin(c4.z, c4.w, c5.x, c5.y, c5.z, c5.w, o, d, binv, rtmax);
          if (!seen) {
            // the other leaves (more than four) and the replays
            uint32_t steps = 0;
            const uint64_t t0 = COUNT ? wall_clock64() : 0;
            const int lb = F.prim_leaf_off[p1], ln = F.prim_leaf_off[p1 + 1] - lb;
            const int m = kd_member(S, F, lb, ln, o, d, rtmax, t1, steps, p1);
            need = m == kNotMember;
            scan = m == kScan;
            if (COUNT) {
              ctr.replay += steps;
              const uint32_t dt = static_cast<uint32_t>(wall_clock64() - t0);
              ctr.mem_max = max(ctr.mem_max, dt);
              ctr.mem_sum += dt;
              ctr.scans += (ln > 4 && steps > 64) ? 1u : 0u;
            }
          }
        }
      }
    }
    // a deferrable queue (BDPT extension rays): the ray goes to the queue's
    // late list -- settled off the pipeline's critical path, its path shaded
    // one step later -- unless its path was deferred before in this pass.
    // Rare (0.1-0.5 % of rays): one atomic per listed ray.
    if ((need || scan) && !walk) {
      const LateList* LL = qfield(Q, q, [](const RayQueue& x) { return x.late; });
      if (LL) {
        const int pth = LL->path[r];
        const int bit = qfield(Q, q, [](const RayQueue& x) { return x.late_bit; });
        if (!(LL->delayed[pth] & bit)) {
          const int half = LL->cap >> 1;
          const int k = atomicAdd(qfield(Q, q, [](const RayQueue& x) { return x.late_n; }) + (scan ? 1 : 0), 1);
          if (k < half) {
            const int i = scan ? half + k : k;
            const int lc = LL->cap;
            LL->o3[i] = o.x;
            LL->o3[lc + i] = o.y;
            LL->o3[2 * lc + i] = o.z;
            LL->d3[i] = d.x;
            LL->d3[lc + i] = d.y;
            LL->d3[2 * lc + i] = d.z;
            LL->t1[i] = t1;
            LL->p1[i] = p1;
            LL->pth[i] = pth;
            LL->tie[i] = big_tie ? 1 : 0;
            LL->delayed[pth] = static_cast<uint8_t>(LL->delayed[pth] | bit);
            qfield(Q, q, [](const RayQueue& x) { return x.out_prim; })[r] = kPendingPrim;
            need = scan = false;
          }
        }
      }
    }
    if ((need && (F.diag & (32 | 128))) || (scan && (F.diag & (32 | 64)))) {  // (diagnostics, as above)
      qfield(Q, q, [](const RayQueue& x) { return x.out_prim; })[r] = p1;
      need = scan = false;
    }
    const int slot = fast_append(hard_n, need);
    if (need) hard[slot] = walk ? (idx | kWalkEntry) : (pair_tie ? (idx | kTieEntry) : idx);
    // near-ties the search's pair record covers, both candidates in few KD
    // leaves: the pair list (k_fast_hard, one per lane: lane_pair)
    const int pslot = fast_append(hard_n + 2, lane_pair);
    if (lane_pair) hard[3 * static_cast<size_t>(hcap) + pslot] = idx;
    // the scan list fills the same array from the top (a ray is in one list)
    const int sslot = fast_append(hard_n + 1, scan);
    if (scan) hard[hcap - 1 - sslot] = big_tie ? ~idx : idx;
  }
}

// k_fast_hard: the rays k_fast_resolve listed.  WAVE: one ray per wave --
// every lane holds the ray, runs the same (uniform) search and decision code,
// and the candidates' leaf replays are shared out across the lanes
// (first_leaves_wave); lane 0 writes the answer and the counts.  A wave then
// lasts as long as its own ray, not as long as the slowest of 64 divergent
// ones: a launch of a few hundred hard rays drops from 0.7-1.4 ms to ~0.5 ms,
// which the one-call API paths (wr_trace_closest & co.) wait for.  Inside the
// render pipelines the launch's latency overlaps the other pipelines' work,
// and there the one-ray-per-lane form uses far less of the machine (64
// rays per wave): measured C2 2,405 vs 2,287 Mrays/s at 64 iterations, so
// the pipelines keep WAVE = false.
// One listed ray's general resolution: the reference's rule over the visited
// hits near the smallest (resolve_tie), or failing that its KD walk.
// Returns false only when the one-lane form hands the ray back (kTieDeferred,
// or a KD walk when walk_wave: *hand_walk set; nothing written; hard_rays
// resolves it with the whole wave).  The callers' stack columns start at
// lds + lane: kd_walk_wave takes the wave's whole region.
template <bool COUNT, bool WAVE>
__device__ __forceinline__ bool settle_ray(const DevScene& S, const FastScene& F, V3 o, V3 d, float rtmin, float rtmax,
                                           float t1, int* stk_node, float* stk_tmin, float* outt, int* outp, int r,
                                           bool lead, FastCounters& ctr, bool walk = false,
                                           bool* hand_walk = nullptr, int p1 = -1, int2 pair = {-1, 0}) {
  float tb;
  int pb;
  if (!(F.diag & 2) && !walk) {
    uint32_t steps = 0, psteps = 0;
    int dbg = 0;
    const uint64_t c0 = COUNT ? wall_clock64() : 0;
    uint32_t split[4] = {0, 0, 0, 0};
    const bool done =
        resolve_tie<WAVE>(S, F, o, d, rtmin, rtmax, t1, stk_node, stk_tmin, tb, pb, steps, psteps, dbg, split, p1,
                          pair);
    if (!WAVE && dbg == kTieDeferred) {
      if (COUNT) ctr.replay += steps;
      return false;
    }
    if (COUNT) {
      ctr.replay += psteps;
      if (lead) {
        const uint32_t dt = static_cast<uint32_t>(wall_clock64() - c0);
        ctr.tie_max = max(ctr.tie_max, dt);
        ctr.tie_sum += dt;
        ctr.tie_col += split[0];
        ctr.tie_leaf += split[1];
        ctr.tie_pass2 += split[2];
        ctr.pair_used += split[3];
        ctr.replay += steps;
        ctr.fb_tie += done ? 1u : 0u;
        const int why = dbg >> 16;
        if (!done && why >= 2 && why <= 5) ++ctr.why[why - 2];
      }
    }
    if (F.diag & 4) {  // debug: the resolution record instead of the answer
      if (lead) outp[r] = -2 - dbg;
      return true;
    }
    if (done) {
      if (lead) {
        outt[r] = tb;
        outp[r] = pb;
      }
      return true;
    }
  }
  // unresolved (a crowd of hits near m, or visited hits in the band): the walk decides
  if (!WAVE && F.walk_wave && hand_walk) {  // by the lane's whole wave, afterwards
    *hand_walk = true;
    return false;
  }
  if (COUNT && lead) ++ctr.fallback;
  if (F.diag & 1) return true;
  const uint64_t c1 = COUNT ? wall_clock64() : 0;
  const uint32_t ki = ctr.kinner, kl = ctr.kleaves, kr = ctr.krefs;
  const bool waved = WAVE && F.walk_wave &&
                     kd_walk_wave<COUNT>(S, o, d, rtmin, rtmax, reinterpret_cast<uint32_t*>(stk_node - __lane_id()),
                                         F.depth * 128, tb, pb, ctr);
  if (!waved) kd_walk<COUNT>(S, o, d, rtmin, rtmax, stk_node, stk_tmin, tb, pb, ctr);
  if (COUNT) {
    if (!lead) {  // the wave walked one ray: counted once
      ctr.kinner = ki;
      ctr.kleaves = kl;
      ctr.krefs = kr;
    } else {
      const uint32_t dt = static_cast<uint32_t>(wall_clock64() - c1);
      ctr.walk_max = max(ctr.walk_max, dt);
      ctr.walk_sum += dt;
    }
  }
  if (lead) {
    outt[r] = tb;
    outp[r] = pb;
  }
  return true;
}

struct ListedRay {
  V3 o, d;
  float rtmin, rtmax, t1;
  int p1, r;
  float* outt;
  int* outp;
  bool walk;  // straight to the KD walk (k_fast_resolve's grazing winners)
  int2 pair;  // near-ties: the search's second hit (p2, t2 bits) when its first window holds two, else (-1, 0)
};

__device__ __forceinline__ ListedRay listed_ray(const TraceQueues& Q, const QueueIndex& QI, int idx) {
  ListedRay L;
  int q;
  QI.locate(idx, q, L.r);
  const int r = L.r;
  L.outp = qfield(Q, q, [](const RayQueue& x) { return x.out_prim; });
  L.outt = qfield(Q, q, [](const RayQueue& x) { return x.out_t; });
  L.t1 = L.outt[r];
  L.p1 = unmark(L.outp[r]);
  const float* o3 = qfield(Q, q, [](const RayQueue& x) { return x.o3; });
  const float* d3 = qfield(Q, q, [](const RayQueue& x) { return x.d3; });
  const int cap = qfield(Q, q, [](const RayQueue& x) { return x.cap; });
  const float* tmn = qfield(Q, q, [](const RayQueue& x) { return x.tmin; });
  const float* tmx = qfield(Q, q, [](const RayQueue& x) { return x.tmax; });
  L.o = v3(o3[r], o3[cap + r], o3[2 * cap + r]);
  L.d = v3(d3[r], d3[cap + r], d3[2 * cap + r]);
  L.rtmin = tmn ? tmn[r] : 0.f;
  L.rtmax = tmx ? tmx[r] : WR_INF;
  L.walk = false;
  L.pair = make_int2(-1, 0);
  return L;
}

// The tie list of one launch (hard_rays: count, ray getter), WAVE or one ray
// per lane with the hand-back above.
template <bool COUNT, bool WAVE, class Get>
__device__ __forceinline__ void hard_rays(const DevScene& S, const FastScene& F, int nh, Get get, int bid, int nb,
                                          uint32_t* lds, FastCounters& ctr) {
  const int lane = __lane_id();
  const bool lead = !WAVE || lane == 0;  // writes the answer, counts the uniform work
  int* stk_node = reinterpret_cast<int*>(lds) + lane;
  float* stk_tmin = reinterpret_cast<float*>(lds) + F.depth * 64 + lane;
  if (WAVE) {
    for (int i = bid; i < nh; i += nb) {
      const ListedRay L = get(i);
      settle_ray<COUNT, true>(S, F, L.o, L.d, L.rtmin, L.rtmax, L.t1, stk_node, stk_tmin, L.outt, L.outp, L.r, lead,
                              ctr, L.walk, nullptr, L.p1, L.pair);
    }
    return;
  }
  // one ray per lane; the rays a lane hands back (near-ties with a many-leaf
  // candidate) are then resolved one after another by the whole wave
  for (int base = bid * 64; base < nh; base += nb * 64) {  // wave-uniform
    const int i = base + lane;
    ListedRay L{};
    bool back = false, hw = false;
    if (i < nh) {
      L = get(i);
      back = !settle_ray<COUNT, false>(S, F, L.o, L.d, L.rtmin, L.rtmax, L.t1, stk_node, stk_tmin, L.outt, L.outp, L.r,
                                       true, ctr, L.walk, &hw, L.p1, L.pair);
    }
    for (unsigned long long m = __ballot(back); m != 0ull; m &= m - 1ull) {
      const int src = __ffsll(static_cast<unsigned long long>(m)) - 1;
      auto bf = [&](float x) { return __shfl(x, src); };
      auto bi = [&](int x) { return __shfl(x, src); };
      auto bp = [&](auto* x) {
        const uint64_t v = reinterpret_cast<uint64_t>(x);
        const uint32_t lo = __shfl(static_cast<uint32_t>(v), src), hi = __shfl(static_cast<uint32_t>(v >> 32), src);
        return reinterpret_cast<decltype(x)>((static_cast<uint64_t>(hi) << 32) | lo);
      };
      settle_ray<COUNT, true>(S, F, v3(bf(L.o.x), bf(L.o.y), bf(L.o.z)), v3(bf(L.d.x), bf(L.d.y), bf(L.d.z)),
                              bf(L.rtmin), bf(L.rtmax), bf(L.t1), stk_node, stk_tmin, bp(L.outt), bp(L.outp), bi(L.r),
                              lane == 0, ctr, bi(hw ? 1 : 0) != 0, nullptr, bi(L.p1), make_int2(bi(L.pair.x), bi(L.pair.y)));
    }
  }
}
template <bool COUNT, bool WAVE>
__device__ __forceinline__ void hard_fast(const DevScene& S, const FastScene& F, const TraceQueues& Q,
                                          const int* hard, const int* hard_n, const int2* pairs, int bid, int nb,
                                          uint32_t* lds, FastCounters& ctr) {
  const QueueIndex QI(Q);
  const int nh = (F.diag & (32 | 128)) ? 0 : hard_n[0];
  hard_rays<COUNT, WAVE>(S, F, nh, [&](int i) {
    const int e = hard[i];
    const int idx = e & ~(kWalkEntry | kTieEntry);
    ListedRay L = listed_ray(Q, QI, idx);
    L.walk = (e & kWalkEntry) != 0;
    if (pairs && (e & kTieEntry)) L.pair = pairs[idx];
    return L;
  }, bid, nb, lds, ctr);
}

// The pair list: near-ties whose 3-EPS window the search's pair record
// covers, both candidates in at most kTieLeaves KD leaves.  One per lane: the
// tie resolution then costs two candidates' leaf replays and no BVH search,
// and 64 of them share a wave (a near-tie per wave holds a wave per tie, and
// at one iteration's early steps those waves outnumber the slots the hard
// kernel's registers leave).  A ray the lane cannot settle (a walk) is
// resolved by its whole wave afterwards (hard_rays).
template <bool COUNT>
__device__ __forceinline__ void pair_fast(const DevScene& S, const FastScene& F, const TraceQueues& Q,
                                          const int* plist, const int* hard_n, const int2* pairs, int bid, int nb,
                                          uint32_t* lds, FastCounters& ctr) {
  const QueueIndex QI(Q);
  const int np = hard_n[2];
  hard_rays<COUNT, false>(S, F, np, [&](int i) {
    const int idx = plist[i];
    ListedRay L = listed_ray(Q, QI, idx);
    L.pair = pairs[idx];
    return L;
  }, bid, nb, lds, ctr);
}

// The scan list (k_fast_resolve's kScan rays and near-ties on many-leaf
// primitives, at the top of the list array): one ray per wave.  The lanes share out p1's leaves -- the witness for each
// leaf's cell, else the replay of its path -- and stop once one is reached;
// p1 then stands.  If none is, t1's triangle is not visited and the ray is
// settled in general by the same wave (settle_ray, one ray per wave).
template <bool COUNT, class Get>
__device__ __forceinline__ void scan_rays(const DevScene& S, const FastScene& F, int ns, Get get, int bid, int nb,
                                          uint32_t* lds, FastCounters& ctr) {
  const int lane = __lane_id();
  int* stk_node = reinterpret_cast<int*>(lds) + lane;
  float* stk_tmin = reinterpret_cast<float*>(lds) + F.depth * 64 + lane;
  for (int i = bid; i < ns; i += nb) {
    bool tie = false;  // a near-tie on a many-leaf primitive: straight to the general resolution
    const ListedRay L = get(i, tie);
    bool member = false;
    float tmin, tmax;
    uint32_t steps = 0;
#if WR_TIE_SPLIT
    const uint64_t s0 = wall_clock64();
#endif
    if (!tie && box_hit(S.root_l, S.root_r, L.o, L.d, tmin, tmax) && !(L.rtmax < tmin)) {  // :312-313, :323
      const V3 inv = v3(1.f / L.d.x, 1.f / L.d.y, 1.f / L.d.z);
      const V3 binv = v3(clamp_inv(L.d.x), clamp_inv(L.d.y), clamp_inv(L.d.z));
      const int lb = F.prim_leaf_off[L.p1], ln = F.prim_leaf_off[L.p1 + 1] - lb;
      // four leaves per lane and round, their loads in flight together; a
      // leaf whose cell the ray's line misses is not replayed
      // (cell_may_be_reached: floors and walls sit in hundreds of leaves)
      constexpr int U = 4;
      for (int base = 0; base < ln && !member; base += 64 * U) {  // wave-uniform
        int po[U];
        uint4 h0[U], h1[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int k = base + u * 64 + lane;
          po[u] = k < ln ? F.prim_leaf[lb + k] : -1;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint2* rec = F.path + max(po[u], 0);
          h0[u] = *reinterpret_cast<const uint4*>(rec);
          h1[u] = *reinterpret_cast<const uint4*>(rec + 2);
        }
        bool ok = false;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (ok || po[u] < 0) continue;
          unsigned long long key;
          ok = cell_crossed_with_margin(h0[u], h1[u], L.o, L.d, binv, L.rtmax) ||
               ((!WR_SCAN_CELL_FILTER || cell_may_be_reached(h0[u], h1[u], L.o, L.d, tmax)) &&
                kd_reaches(F.path + po[u], L.o, L.d, inv, tmin, tmax, L.rtmax, steps, key));
        }
        member = __ballot(ok) != 0ull;
      }
    }
    if (COUNT) {
      ctr.replay += steps;
      ctr.scans += lane == 0 ? 1u : 0u;
#if WR_TIE_SPLIT
      if (lane == 0) ctr.scan_t += static_cast<uint32_t>(wall_clock64() - s0);
#endif
    }
    if (member) {  // p1 stands (a queue entry holds it already; a late record gets it)
      if (lane == 0) {
        L.outt[L.r] = L.t1;
        L.outp[L.r] = L.p1;
      }
      continue;
    }
    settle_ray<COUNT, true>(S, F, L.o, L.d, L.rtmin, L.rtmax, L.t1, stk_node, stk_tmin, L.outt, L.outp, L.r,
                            lane == 0, ctr, false, nullptr, L.p1, L.pair);
  }
}
template <bool COUNT>
__device__ __forceinline__ void scan_fast(const DevScene& S, const FastScene& F, const TraceQueues& Q,
                                          const int* hard, const int* hard_n, int hcap, int bid, int nb, uint32_t* lds,
                                          FastCounters& ctr) {
  const QueueIndex QI(Q);
  const int ns = (F.diag & (32 | 64)) ? 0 : hard_n[1];
  scan_rays<COUNT>(S, F, ns, [&](int i, bool& tie) {
    const int e = hard[hcap - 1 - i];
    tie = e < 0;
    ListedRay L = listed_ray(Q, QI, tie ? ~e : e);
    if (tie && !F.diag && F.pair > 0) L.pair = reinterpret_cast<const int2*>(hard + hcap)[~e];  // (kPairWindow)
    return L;
  }, bid, nb, lds, ctr);
}

// A record of a late list (extension rays only: [0, inf) windows).
__device__ __forceinline__ ListedRay late_ray(const LateList& LL, int i) {
  ListedRay L;
  const int c = LL.cap;
  L.o = v3(LL.o3[i], LL.o3[c + i], LL.o3[2 * c + i]);
  L.d = v3(LL.d3[i], LL.d3[c + i], LL.d3[2 * c + i]);
  L.rtmin = 0.f;
  L.rtmax = WR_INF;
  L.t1 = LL.t1[i];
  L.p1 = LL.p1[i];
  L.r = i;
  L.outt = LL.t;
  L.outp = LL.prim;
  L.walk = false;
  L.pair = make_int2(-1, 0);
  return L;
}
// k_late_hard: a late list's tie entries (blocks [0, hard_blocks): one per
// wave up to wave_max entries, else one per lane on lane_blocks) and scan
// entries (the other blocks, one per wave).  Same resolutions as k_fast_hard.
template <bool COUNT>
__device__ __forceinline__ void late_hard(const DevScene& S, const FastScene& F, const LateList& LL, const int* n,
                                          int b, int nb, int hard_blocks, int lane_blocks, int wave_max,
                                          uint32_t* lds, FastCounters& ctr) {
  const int half = LL.cap >> 1;
  const int nt = min(n[0], half), ns = min(n[1], half);
  if (b < hard_blocks) {
    auto get = [&](int i) { return late_ray(LL, i); };
    if (nt <= wave_max)
      hard_rays<COUNT, true>(S, F, nt, get, b, hard_blocks, lds, ctr);
    else if (b < lane_blocks)
      hard_rays<COUNT, false>(S, F, nt, get, b, lane_blocks, lds, ctr);
  } else {
    scan_rays<COUNT>(S, F, ns, [&](int i, bool& tie) {
      tie = LL.tie[half + i] != 0;
      return late_ray(LL, half + i);
    }, b - hard_blocks, nb - hard_blocks, lds, ctr);
  }
}

// k_fast_verify (WR_BVH_VERIFY=1, validation only): the reference's KD walk
// for every ray of the launch, compared bit for bit with the BVH mode's answer.
__device__ __forceinline__ void verify_fast(const DevScene& S, const FastScene& F, const TraceQueues& Q, uint32_t* lds,
                                            uint32_t& rays, uint32_t& bad) {
  const int lane = __lane_id();
  int* stk_node = reinterpret_cast<int*>(lds) + lane;
  float* stk_tmin = reinterpret_cast<float*>(lds) + F.depth * 64 + lane;
  const QueueIndex QI(Q);
  FastCounters dummy{};
  for (int idx = blockIdx.x * 64 + lane; idx < QI.n; idx += gridDim.x * 64) {
    int q, r;
    QI.locate(idx, q, r);
    const float* o3 = qfield(Q, q, [](const RayQueue& x) { return x.o3; });
    const float* d3 = qfield(Q, q, [](const RayQueue& x) { return x.d3; });
    const int cap = qfield(Q, q, [](const RayQueue& x) { return x.cap; });
    const float* tmn = qfield(Q, q, [](const RayQueue& x) { return x.tmin; });
    const float* tmx = qfield(Q, q, [](const RayQueue& x) { return x.tmax; });
    const V3 o = v3(o3[r], o3[cap + r], o3[2 * cap + r]);
    const V3 d = v3(d3[r], d3[cap + r], d3[2 * cap + r]);
    float tb;
    int pb;
    kd_walk<false>(S, o, d, tmn ? tmn[r] : 0.f, tmx ? tmx[r] : WR_INF, stk_node, stk_tmin, tb, pb, dummy);
    const int p = qfield(Q, q, [](const RayQueue& x) { return x.out_prim; })[r];
    const float t = qfield(Q, q, [](const RayQueue& x) { return x.out_t; })[r];
    if (p == kPendingPrim) continue;  // deferred: checked by verify_late
    ++rays;
    if (p != pb || (pb >= 0 && __float_as_uint(t) != __float_as_uint(tb))) ++bad;
  }
}
// The same check for a late list's records (after k_late_hard).
__device__ __forceinline__ void verify_late(const DevScene& S, const FastScene& F, const LateList& LL, const int* n,
                                            uint32_t* lds, uint32_t& rays, uint32_t& bad) {
  const int lane = __lane_id();
  int* stk_node = reinterpret_cast<int*>(lds) + lane;
  float* stk_tmin = reinterpret_cast<float*>(lds) + F.depth * 64 + lane;
  FastCounters dummy{};
  const int half = LL.cap >> 1;
  const int nt = min(n[0], half), nall = nt + min(n[1], half);
  for (int j = blockIdx.x * 64 + lane; j < nall; j += gridDim.x * 64) {
    const int i = j < nt ? j : half + (j - nt);
    const ListedRay L = late_ray(LL, i);
    float tb;
    int pb;
    kd_walk<false>(S, L.o, L.d, L.rtmin, L.rtmax, stk_node, stk_tmin, tb, pb, dummy);
    const int p = LL.prim[i];
    const float t = LL.t[i];
    ++rays;
    if (p != pb || (pb >= 0 && __float_as_uint(t) != __float_as_uint(tb))) ++bad;
  }
}

}  // namespace wrd
