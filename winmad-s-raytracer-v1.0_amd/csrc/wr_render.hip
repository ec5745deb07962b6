// MI355X (gfx950) implementation of the reference's hot path behind the C ABI of
// include/winmad_rt.h (kernels in wr_traverse.h, wr_bdpt.h, wr_vcm.h, wr_pt.h;
// this file: shared device helpers, the runtime -- pipelines, work buffers,
// launches, timing -- and the C entry points):
//   * KD-tree closest-hit traversal (wr_traverse.h) as one generic queue kernel
//   * BidirPathTracing::runIteration (bidirPathTracing.cpp:53-265) as a wavefront:
//       light pass  : gen -> [trace -> shade] x 9 -> trace(splat rays) -> resolve
//       camera pass : gen -> [trace -> shade -> trace(shadow+aux) -> resolve -> DI] x 10
//     path state lives in SoA buffers sized for the whole frame; queues are
//     compacted with wave ballots + one atomic per wave
//   * PathIntegrator::raytracing (pathIntegrator.cpp:29-148), one sample index per
//     wavefront iteration
//
// Work is keyed by (iteration, path index) through the counter RNG, never by the
// device or launch geometry, so any sharding of iterations over GPUs renders the
// same film up to float summation order.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "winmad_rt.h"
#include "wr_scene.h"
#include "wr_traverse.h"
#include "wr_fast.h"

using namespace wrd;

// =============================================================== errors
static int fail(int code, const std::string& msg) { return wr::set_error(code, msg); }
// Hardware queues: one per render pipeline.  HIP gives a process
// GPU_MAX_HW_QUEUES queues (default 4; the GPU box exports 4), read once when
// HIP initialises, and pipelines beyond them share a queue and serialize
// (concurrent pipelines).  The library never writes the process
// environment by itself: a host that wants the measured configuration (16
// pipelines) asks for it with wr_request_hw_queues() before its first HIP call
// (example_main / tot_main do; bench.py and winmad_rt/native.py set the
// variable before HIP starts).  The count is latched by the library's first
// wr_create (the library's first HIP call, or later than the host's): pipelines
// are sized by that value from then on, and a wr_request_hw_queues after it
// changes nothing (HIP has read the variable by then).  A host that starts HIP
// itself (e.g. torch.cuda.is_available()) before asking gets the queues HIP
// saw only if it asks before that, which is what native.py does.
static std::atomic<int> g_hw_queues_latched{0};
static int hw_queues_env() {
  const char* q = std::getenv("GPU_MAX_HW_QUEUES");
  const int n = q ? std::atoi(q) : 0;
  return n > 0 ? n : 4;  // HIP's default
}
static int hw_queues_in_effect() {
  const int l = g_hw_queues_latched.load();
  return l > 0 ? l : hw_queues_env();
}
static int latch_hw_queues() {
  int expect = 0;
  g_hw_queues_latched.compare_exchange_strong(expect, hw_queues_env());
  return g_hw_queues_latched.load();
}

// Every C-ABI entry that selects a device (hipSetDevice) leaves the caller's
// current device as it found it: a multi-device render or reduce ends on its
// last device otherwise, and a PyTorch caller's next default-device work would
// run there.
struct DeviceGuard {
  int dev = -1;
  DeviceGuard() {
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  }
  ~DeviceGuard() {
    if (dev >= 0) (void)hipSetDevice(dev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};
#define HIPCHK(expr)                                                                          \
  do {                                                                                        \
    hipError_t e_ = (expr);                                                                   \
    if (e_ != hipSuccess) return fail(WR_E_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

// =============================================================== device helpers
namespace {

constexpr int kVMax = 9;       // light vertices per subpath (pathLength 1..9, :77-124)
constexpr int kTraceBlock = 64;  // one wave per workgroup: persistent traversal
constexpr int kShadeBlock = 256;
// The vertex kernels at <= 128 VGPRs (4 waves/SIMD, a few dwords spilled) run
// beside the other pipelines' traversal far better than at 132-146 VGPRs:
// measured 638 -> 693 Mrays/s (torus 1080p BDPT, 3 pipelines).
#ifndef WR_SHADE_WAVES
#define WR_SHADE_WAVES 4
#endif
// Scalar fp32 instead of v_pk_mul/add_f32: the pairing costs more register moves
// than it saves in this divergent, register-bound code (traversal 736 -> 791
// Mrays/s).  Results are identical (both are IEEE single-precision).  A gfx950
// target feature, so it is attached in the device pass only.
#ifdef __HIP_DEVICE_COMPILE__
#define WR_NO_PK_FP32 __attribute__((target("no-packed-fp32-ops")))
#else
#define WR_NO_PK_FP32
#endif
#define WR_SHADE_OCC __attribute__((amdgpu_waves_per_eu(WR_SHADE_WAVES, 8))) WR_NO_PK_FP32
// Iterations / samples a pipeline advances in lockstep (see struct Pipe).  The
// per-vertex kernels take the whole group (member = blockIdx.y).
#ifndef WR_GROUP
#define WR_GROUP 2
#endif
constexpr int kGroup = WR_GROUP;

// The late lists of one pipeline step (deferred hard rays, one per group member)
struct LateArgs {
  LateList l[kGroup];
  int* n[kGroup];
};

enum SqKind { SQ_SPLAT = 0, SQ_CONN = 1, SQ_NEE = 2, SQ_DIB = 3 };
enum DiFlag { DI_NEE = 1, DI_BSDF = 2, DI_EARLY = 4 };
// DI record state word: rays still to resolve (low byte) | results
enum DiState { DI_COUNT = 0xff, DI_VIS = 0x100, DI_SAME = 0x200 };

// Queue counters of one iteration / sample, one slot per step, cleared by a
// single memset at its start (no per-bounce counter resets).  BDPT: light
// bounce b uses slot b, camera bounce b slot kCamSlot + b; PT bounce b slot b.
constexpr int kSlots = 64;
constexpr int kCamSlot = 16;
struct StepCounters {
  int ext[kSlots];    // extension rays entering step `slot`
  int sq[kSlots];     // shadow / aux rays traced at step `slot` (light splats: slot 0 -> camera bounce 0)
  int di[kSlots];     // DI records finalized at step `slot`
  int fetch[kSlots];  // persistent-traversal cursor of the step's trace launch
  int vcm_pending;    // VCM: light paths whose first vertex is an emitter (k_vcm_fixup)
  int vcm_nverts;     // VCM: light vertices in the merge grid
  int mq[kSlots];     // VCM: merge queries queued at step `slot`
  int hard[kSlots][3];  // WR_TRACE_BVH: rays of step `slot` left to k_fast_hard (tie list, scan list, pair list)
  int rlist[kSlots];    // WR_TRACE_BVH: rays of step `slot` the search left to k_fast_resolve
  int late[kSlots][2];  // WR_TRACE_BVH: rays of step `slot` deferred (late list: ties, scans)
  int vpool, cpool;     // BDPT, overlapped: records taken from the light / camera vertex pools
};
struct DevCounters {
  int fetch;  // traversal cursor of the API path (wr_trace_closest / wr_occluded)
  int hard[3];  // API path: rays left to k_fast_hard (tie list, scan list, pair list)
  int rlist;    // API path: rays the search left to k_fast_resolve
  unsigned long long stamps[8];  // diagnostic build only (WR_TRACE_STAMPS=1)
  unsigned long long closest, shadow, inner, leaves, refs, tests;
  unsigned long long vm_queries, vm_found, vm_merged;  // VCM range queries / vertices in radius / merges
  unsigned long long bvh_nodes, bvh_tests, kd_replay, fallback;  // WR_TRACE_BVH work (count_work)
  unsigned long long verify_rays, verify_bad;                   // WR_BVH_VERIFY
  unsigned long long deferred;  // BDPT rays settled off the critical path (late lists)
  unsigned long long lat[12];  // WR_TRACE_BVH latency tail (FastCounters mem_max .. scans; max or sum; tie_col .. tie_pass2)
  unsigned long long ww[4];   // kd_walk_wave: walks, rounds, nodes, serial fall-backs
  unsigned long long overflow;  // BDPT: appends a full vertex pool / shadow queue dropped (the render is redone)
};

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// One atomic per wave: returns this lane's slot (or -1 if !want).
__device__ __forceinline__ int wave_append(int* counter, bool want) {
  const unsigned long long m = __ballot(want);
  if (m == 0ull) return -1;
  const int lane = lane_id();
  const int leader = __ffsll(static_cast<unsigned long long>(m)) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(counter, __popcll(m));
  base = __shfl(base, leader);
  return want ? base + __popcll(m & ((1ull << lane) - 1ull)) : -1;
}
__device__ __forceinline__ void wave_count(unsigned long long* counter, bool c) {
  const unsigned long long m = __ballot(c);
  if (m == 0ull) return;
  if (lane_id() == __ffsll(static_cast<unsigned long long>(m)) - 1) atomicAdd(counter, (unsigned long long)__popcll(m));
}
__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Queue entries (SoA x / y / z columns) are written by one kernel and read by
// the next one or two: with WR_QUEUE_NT they move with the non-temporal policy,
// leaving the L2 to the scene's nodes and triangles, which every search re-reads.
#ifndef WR_QUEUE_NT
#define WR_QUEUE_NT 1
#endif
__device__ __forceinline__ V3 ld3(const float* b, int stride, int i) {
#if WR_QUEUE_NT
  return v3(__builtin_nontemporal_load(b + i), __builtin_nontemporal_load(b + stride + i),
            __builtin_nontemporal_load(b + 2 * stride + i));
#else
  return v3(b[i], b[stride + i], b[2 * stride + i]);
#endif
}
__device__ __forceinline__ void st3(float* b, int stride, int i, V3 v) {
#if WR_QUEUE_NT
  __builtin_nontemporal_store(v.x, b + i);
  __builtin_nontemporal_store(v.y, b + stride + i);
  __builtin_nontemporal_store(v.z, b + 2 * stride + i);
#else
  b[i] = v.x;
  b[stride + i] = v.y;
  b[2 * stride + i] = v.z;
#endif
}
__device__ __forceinline__ void film_add(float* film, int pix, V3 v) {
  if (pix < 0) return;
  if (v.x != 0.f) atomicAdd(film + 3 * pix, v.x);
  if (v.y != 0.f) atomicAdd(film + 3 * pix + 1, v.y);
  if (v.z != 0.f) atomicAdd(film + 3 * pix + 2, v.z);
}
// ImageFilm::addColor bounds check (film.cpp:4-9) -> flat pixel or -1
__device__ __forceinline__ int pix_index(int h, int w, int H, int W) {
  return (h < 0 || h >= H || w < 0 || w >= W) ? -1 : h * W + w;
}

// =============================================================== trace kernels
// Generic persistent queue traversal: rays [3][cap] SoA, count on device.
template <bool COUNT, bool SPH, bool NARROW, bool STAMP = false, bool CUT = false, bool DENSE = false>
// Register budget: 4 waves/SIMD (<= 128 VGPRs) matches the LDS-limited 16
// waves/CU and fills the register file (BDPT at 96: C2 -0.8 %; the VCM camera
// pass, CUT, at 96: -1 %).  DENSE (PT): <= 96 VGPRs and no ray records in LDS
// -> 20 waves/CU on torus-sized trees.  C3 2,538 (4 waves) -> 2,620 (96 VGPRs,
// a shading wave of another pipeline fits beside the traversal) -> 2,697
// Mrays/s (DENSE); on BDPT DENSE loses (C2 -1 %), on VCM too (-1.3 %).
#ifndef WR_TRACE_WAVES_PER_EU
#define WR_TRACE_WAVES_PER_EU 4
#endif
#ifndef WR_TRACE_CUT_WAVES_PER_EU
#define WR_TRACE_CUT_WAVES_PER_EU 4
#endif
// wave issue priority of the traversal (s_setprio 0-3); 0 = hardware default
#ifndef WR_TRACE_PRIO
#define WR_TRACE_PRIO 0
#endif
__global__ void __launch_bounds__(kTraceBlock)
__attribute__((amdgpu_waves_per_eu(DENSE ? 5 : (CUT ? WR_TRACE_CUT_WAVES_PER_EU : WR_TRACE_WAVES_PER_EU), 8))) WR_NO_PK_FP32 k_trace(DevScene S, TraceQueues Q, DevCounters* ctr, int* fetch) {
  extern __shared__ uint32_t smem[];
#if WR_TRACE_PRIO > 0
  __builtin_amdgcn_s_setprio(WR_TRACE_PRIO);  // issue priority over co-resident vertex-kernel waves
#endif
  TraceCounters tc{0, 0, 0, 0};
  trace_queue<COUNT, SPH, NARROW, STAMP, CUT, DENSE>(S, Q, fetch, smem, tc, ctr->stamps);
  if (COUNT) {
    unsigned long long a = wave_sum(tc.inner), b = wave_sum(tc.leaves), c = wave_sum(tc.refs),
                       e = wave_sum(tc.tests);
    if (lane_id() == 0) {
      atomicAdd(&ctr->inner, a);
      atomicAdd(&ctr->leaves, b);
      atomicAdd(&ctr->refs, c);
      atomicAdd(&ctr->tests, e);
    }
  }
}

// Verified-BVH closest hit over the same queues (wr_fast.h): the search, then
// the one-ray-per-lane resolve (membership replay, KD walk of undecided rays).
// 4 waves/SIMD like k_trace.
template <bool COUNT>
__device__ __forceinline__ void fast_counts(DevCounters* ctr, const FastCounters& fc) {
  unsigned long long a = wave_sum(fc.nodes), b = wave_sum(fc.tests), c = wave_sum(fc.replay),
                     e = wave_sum(fc.fallback), ki = wave_sum(fc.kinner), kl = wave_sum(fc.kleaves),
                     kr = wave_sum(fc.krefs);
  if (lane_id() == 0) {
    atomicAdd(&ctr->bvh_nodes, a);
    atomicAdd(&ctr->bvh_tests, b);
    atomicAdd(&ctr->kd_replay, c);
    atomicAdd(&ctr->fallback, e);
    // the KD walks of undecided rays count as the reference traversal's work
    atomicAdd(&ctr->inner, ki);
    atomicAdd(&ctr->leaves, kl);
    atomicAdd(&ctr->refs, kr);
    atomicAdd(&ctr->tests, kr);
  }
  // diagnostic tail (stamps[5..7], WR_TRACE_LOG): max nodes / tests per ray, rays > 256 nodes
  atomicMax(&ctr->stamps[5], static_cast<unsigned long long>(fc.max_nodes));
  atomicMax(&ctr->stamps[6], static_cast<unsigned long long>(fc.max_tests));
  atomicAdd(&ctr->stamps[7], static_cast<unsigned long long>(fc.long_rays));
  atomicAdd(&ctr->stamps[4], static_cast<unsigned long long>(fc.fb_tie));
  for (int k = 0; k < 4; ++k) atomicAdd(&ctr->stamps[k], static_cast<unsigned long long>(fc.why[k]));
  const uint32_t lat[12] = {fc.mem_max, fc.mem_sum, fc.tie_max,   fc.tie_sum, fc.walk_max,  fc.walk_sum,
                            fc.scans,   fc.tie_col, fc.tie_leaf, fc.tie_pass2, fc.scan_t, fc.pair_used};
  for (int k = 0; k < 12; ++k) {
    if (k % 2 == 0 && k < 6) atomicMax(&ctr->lat[k], static_cast<unsigned long long>(lat[k]));
    else atomicAdd(&ctr->lat[k], static_cast<unsigned long long>(lat[k]));
  }
  if (lane_id() == 0) {  // (wave-uniform: counted by the walking wave's lane 0 only)
    const uint32_t ww[4] = {fc.ww_walks, fc.ww_rounds, fc.ww_nodes, fc.ww_over};
    for (int k = 0; k < 4; ++k)
      if (ww[k]) atomicAdd(&ctr->ww[k], static_cast<unsigned long long>(ww[k]));
  }
}
#ifndef WR_FAST_WAVES
#define WR_FAST_WAVES 4  // minimum waves per SIMD the search's registers must allow
#endif
// LATE: blocks [0, lblocks) settle the previous step's deferred hard rays
// (its late lists, late_hard) beside this step's search; they come first so
// that they are dispatched with the search's persistent blocks, not after them
// W: the search tree's width (FastScene::wide)
#ifndef WR_FAST4_WAVES
#define WR_FAST4_WAVES 5  // the 4-wide search: 98 VGPRs at 4, held to 96 for 5 waves per SIMD
#endif
// SPH: the tree holds spheres (FastScene::sph) -- a variant of its own, so
// that the triangle scenes' search keeps its registers
// RL: the search settles the rays whose winner's membership its first leaf
// cells prove (the resolve's first test) and lists the rest for k_fast_resolve
template <bool COUNT, bool LATE, int W, bool SPH, bool RL = false>
__global__ void __launch_bounds__(kTraceBlock)
__attribute__((amdgpu_waves_per_eu(W == 4 && !LATE ? WR_FAST4_WAVES : WR_FAST_WAVES, 8))) WR_NO_PK_FP32
k_trace_fast(DevScene S, FastScene F, TraceQueues Q, DevCounters* ctr, int* fetch, float* t2buf, int2* pairs,
             int2* spill, LateArgs L, int lblocks, int gn, int hblocks, int lane_blocks, int wave_max, int* rlist,
             int* rlist_n) {
  extern __shared__ uint32_t smem[];
  FastCounters fc{};
  const int b = static_cast<int>(blockIdx.x);
  if (LATE && b < lblocks) {
    const int per = lblocks / gn, m = b / per, bb = b % per;
    late_hard<COUNT>(S, F, L.l[m], L.n[m], bb, per, hblocks, lane_blocks, wave_max, smem, fc);
    if (bb == 0 && threadIdx.x == 0) {
      const int half = L.l[m].cap >> 1;
      atomicAdd(&ctr->deferred, static_cast<unsigned long long>(min(L.n[m][0], half) + min(L.n[m][1], half)));
    }
  } else {
    trace_fast<COUNT, W, SPH, RL>(S, F, Q, fetch, t2buf, pairs, spill, smem, fc, b - (LATE ? lblocks : 0),
                                  static_cast<int>(gridDim.x) - (LATE ? lblocks : 0), rlist, rlist_n);
  }
  if (COUNT) fast_counts<COUNT>(ctr, fc);
}
// the search kernel for a tree width (instantiated for 2 and 4; 8 when the
// library is built with WR_BVH_WIDE=8)
// RL: the search's per-wave buffer of listed rays (trace_fast)
constexpr size_t kRlistLds = 64 * sizeof(int);
using TraceFastKernel = void (*)(DevScene, FastScene, TraceQueues, DevCounters*, int*, float*, int2*, int2*, LateArgs,
                                 int, int, int, int, int, int*, int*);
template <bool COUNT, bool LATE>
TraceFastKernel trace_fast_kernel(int wide, bool sph = false, bool rl = false) {
#if WR_BVH_WIDE == 8
  if (wide == 8) return k_trace_fast<COUNT, LATE, 8, false>;  // (triangle scenes: the 8-wide tree is a build option)
#endif
  // (the deferred-hard-ray variants, LATE, are not built with spheres: defer_enabled)
  if (sph && !LATE) return wide == 4 ? k_trace_fast<COUNT, false, 4, true> : k_trace_fast<COUNT, false, 2, true>;
  // (the resolve list: triangle trees, no late lists)
  if (rl && !LATE)
    return wide == 4 ? k_trace_fast<COUNT, false, 4, false, true> : k_trace_fast<COUNT, false, 2, false, true>;
  return wide == 4 ? k_trace_fast<COUNT, LATE, 4, false> : k_trace_fast<COUNT, LATE, 2, false>;
}
#ifndef WR_RESOLVE_WAVES
#define WR_RESOLVE_WAVES 0  // > 0: the resolve's register budget as waves per SIMD (0: the compiler's choice, 101 VGPRs)
#endif
#if WR_RESOLVE_WAVES > 0
#define WR_RESOLVE_OCC __attribute__((amdgpu_waves_per_eu(WR_RESOLVE_WAVES, 8)))
#else
#define WR_RESOLVE_OCC
#endif
template <bool COUNT>
__global__ void __launch_bounds__(kTraceBlock) WR_NO_PK_FP32 WR_RESOLVE_OCC
k_fast_resolve(DevScene S, FastScene F, TraceQueues Q, DevCounters* ctr, const float* t2buf, int* hard, int* hard_n,
               int hcap, const int* rlist, const int* rlist_n) {
  FastCounters fc{};
  resolve_fast<COUNT>(S, F, Q, t2buf, hard, hard_n, hcap, fc, rlist, rlist_n);
  if (COUNT) fast_counts<COUNT>(ctr, fc);
}
// WR_HARD_WAVES: register budget of k_fast_hard as waves per SIMD (0: the
// compiler's choice).  Its waves live for the whole tie / scan work (up to ms)
// beside the other pipelines' search and vertex waves, so the VGPRs they hold
// are occupancy taken from those.
#ifndef WR_HARD_WAVES
#define WR_HARD_WAVES 0
#endif
#if WR_HARD_WAVES > 0
#define WR_HARD_OCC __attribute__((amdgpu_waves_per_eu(WR_HARD_WAVES, 8)))
#else
#define WR_HARD_OCC
#endif
// blocks [0, hard_blocks): the tie list; the rest: the scan list, one ray per
// wave.  WAVE: one tie per wave (the API paths).  Otherwise the launch adapts
// to the tie count it finds: up to wave_max ties (a late bounce's launch:
// its slowest tie is the step's latency) one per wave -- a wave lasts as long
// as its own tie, and the candidates' replays are shared by its lanes -- and
// more (full launches, where other pipelines hide the latency) one per lane
// on the first lane_blocks blocks.
template <bool COUNT, bool WAVE>
__global__ void __launch_bounds__(kTraceBlock) WR_NO_PK_FP32 WR_HARD_OCC
k_fast_hard(DevScene S, FastScene F, TraceQueues Q, DevCounters* ctr, const int* hard, const int* hard_n, int hcap,
            int hard_blocks, int lane_blocks, int wave_max, int pair_blocks) {
  extern __shared__ uint32_t smem[];
  FastCounters fc{};
  const int b = static_cast<int>(blockIdx.x);
  // the search's pair records and the pair list follow the lists (TraceSlot::t2)
  const int2* pairs = reinterpret_cast<const int2*>(hard + hcap);
  if (b >= hard_blocks && b < hard_blocks + pair_blocks) {
    pair_fast<COUNT>(S, F, Q, hard + 3 * static_cast<size_t>(hcap), hard_n, pairs, b - hard_blocks, pair_blocks, smem,
                     fc);
  } else if (b < hard_blocks) {
    if (WAVE || hard_n[0] <= wave_max)  // wave_max <= hard_blocks
      hard_fast<COUNT, true>(S, F, Q, hard, hard_n, pairs, b, hard_blocks, smem, fc);
    else if (b < lane_blocks)
      hard_fast<COUNT, false>(S, F, Q, hard, hard_n, pairs, b, lane_blocks, smem, fc);
  } else {
    const int s0 = hard_blocks + pair_blocks;
    scan_fast<COUNT>(S, F, Q, hard, hard_n, hcap, b - s0, static_cast<int>(gridDim.x) - s0, smem, fc);
  }
  if (COUNT) fast_counts<COUNT>(ctr, fc);
}

// WR_BVH_VERIFY: the late lists' answers against the KD walk
__global__ void __launch_bounds__(kTraceBlock) WR_NO_PK_FP32
k_late_verify(DevScene S, FastScene F, LateArgs L, DevCounters* ctr) {
  extern __shared__ uint32_t smem[];
  uint32_t rays = 0, bad = 0;
  verify_late(S, F, L.l[blockIdx.y], L.n[blockIdx.y], smem, rays, bad);
  const unsigned long long a = wave_sum(rays), b = wave_sum(bad);
  if (lane_id() == 0) {
    atomicAdd(&ctr->verify_rays, a);
    atomicAdd(&ctr->verify_bad, b);
  }
}

__global__ void __launch_bounds__(kTraceBlock) WR_NO_PK_FP32
k_fast_verify(DevScene S, FastScene F, TraceQueues Q, DevCounters* ctr) {
  extern __shared__ uint32_t smem[];
  uint32_t rays = 0, bad = 0;
  verify_fast(S, F, Q, smem, rays, bad);
  const unsigned long long a = wave_sum(rays), b = wave_sum(bad);
  if (lane_id() == 0) {
    atomicAdd(&ctr->verify_rays, a);
    atomicAdd(&ctr->verify_bad, b);
  }
}

// C-ABI traversal, before: AoS wr_ray -> SoA queue (occlusion rays re-normalised
// as Scene::occluded's Ray(p1, dir) does, scene.cpp:74)
__global__ void __launch_bounds__(256) k_api_prep(const wr_ray* rays, int n, int occ, float* o3, float* d3,
                                                  float* tmin, float* tmax, const float* targets, float* cut) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const wr_ray r = rays[i];
    const V3 o = v3(r.o[0], r.o[1], r.o[2]);
    V3 d = v3(r.d[0], r.d[1], r.d[2]);
    if (occ) {
      d = normalize(d);
      const V3 tg = v3(targets[3 * i], targets[3 * i + 1], targets[3 * i + 2]);
      cut[i] = occl_cut(o, tg, dot(tg - o, d));
    }
    st3(o3, n, i, o);
    st3(d3, n, i, d);
    tmin[i] = r.tmin;
    tmax[i] = r.tmax;
  }
}
// ... after: rebuild the Intersection (scene.cpp:25-27) or the occlusion answer
__global__ void __launch_bounds__(256) k_api_finish(DevScene S, const float* o3, const float* d3, const float* t,
                                                    const int* prim, const float* targets, int n, wr_hit* hits,
                                                    uint8_t* occ) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const V3 o = ld3(o3, n, i), d = ld3(d3, n, i);
    const int p = prim[i];
    if (occ) {
      const bool unocc = p < 0 || near_eq(o + d * t[i], v3(targets[3 * i], targets[3 * i + 1], targets[3 * i + 2]));
      occ[i] = unocc ? 0 : 1;
      continue;
    }
    wr_hit h;
    h.prim = p;
    if (p >= 0) {
      const Hit x = rebuild_hit(S, p, t[i], o, d);
      h.t = x.t;
      h.p[0] = x.p.x; h.p[1] = x.p.y; h.p[2] = x.p.z;
      h.n[0] = x.n.x; h.n[1] = x.n.y; h.n[2] = x.n.z;
      h.inside = x.inside;
      h.mat_id = x.mat;
    } else {
      h.t = WR_INF;
      h.p[0] = h.p[1] = h.p[2] = 0.f;
      h.n[0] = h.n[1] = h.n[2] = 0.f;
      h.inside = 0;
      h.mat_id = 0;
    }
    hits[i] = h;
  }
}

// =============================================================== BDPT, VCM, PT
#include "wr_bdpt.h"
#include "wr_vcm.h"
static_assert(sizeof(VcmGroup) <= 4000, "kernel argument block too large");
#include "wr_pt.h"

}  // namespace

// =============================================================== host side
struct wr_scene {
  wr::Scene s;
};

namespace {
// Device memory arena: bump allocation out of one hipMalloc per arena.
struct Arena {
  char* base = nullptr;
  size_t cap = 0, used = 0;
  int reserve(size_t bytes) {
    release();
    if (hipMalloc(&base, bytes) != hipSuccess) {
      base = nullptr;
      return fail(WR_E_HIP, "hipMalloc of " + std::to_string(bytes) + " bytes failed");
    }
    cap = bytes;
    used = 0;
    return WR_OK;
  }
  template <class T>
  T* take(size_t n) {
    size_t off = (used + 255) & ~size_t(255);
    used = off + n * sizeof(T);
    return reinterpret_cast<T*>(base + off);
  }
  void release() {
    if (base) (void)hipFree(base);
    base = nullptr;
    cap = used = 0;
  }
};

template <class Fn>
size_t measure(Fn fn) {  // bytes an arena layout needs
  Arena a;
  fn(a);
  return a.used + 256;
}
}  // namespace

// One render pipeline: a HIP stream with its own work buffers and queue
// counters.  Iterations (BDPT) / samples (PT) are dealt round-robin to the
// context's pipelines, so the long tail of one stream's late-bounce traversal
// launches (a launch lasts as long as its slowest ray) overlaps the full
// launches of another.  The film is a sum, so the result does not depend on the
// pipeline count (up to the order of float atomics).
#ifndef WR_MAX_PIPES
#define WR_MAX_PIPES 16
#endif
constexpr int kMaxPipes = WR_MAX_PIPES;
// Each pipeline advances a group of up to kGroup iterations / samples in
// lockstep: every traversal launch takes the queues of all of them, so the
// launch tail (its slowest ray) is paid once per group.
struct Pipe {
  hipStream_t stream = nullptr;
  DevCounters* ctr = nullptr;
  StepCounters* sc = nullptr;  // [kGroup]
  Arena work;
  size_t work_key = 0;  // P for which `work` is laid out
  int work_kind = 0;    // 1 bdpt, 2 pt, 3 vcm (bdpt + vcm buffers)
  int work_sets = 0;    // buffer sets laid out
  float work_pool = -1.f;  // the BDPT pool scale they were laid out with (bdpt_pool_scale)
  BdptBuf bb[kGroup]{};
  PtBuf pb[kGroup]{};
  VcmBuf vb[kGroup]{};
  float* t2buf = nullptr;  // WR_TRACE_BVH: per-ray t2 of the BVH search (launch index)
  int2* spill = nullptr;   // WR_TRACE_BVH: the search stack's spill area (fast_blocks x 64 lanes)
  size_t t2_cap = 0;
  std::vector<hipEvent_t> events;  // Timer marks (time_kernels)
  std::vector<int> ev_cat;
  size_t ev_used = 0;
  hipEvent_t done = nullptr;
  // deferred hard rays (BDPT, WR_TRACE_BVH): a step's late lists, settled and
  // shaded by extra blocks of the next step's launches
  Arena late_mem;
  size_t late_recs = 0, late_paths = 0;  // records per list, paths per member laid out
  LateList late_h[kGroup][2]{};          // host copies: [member][step parity]
  LateList* late_d = nullptr;            // device copies, same order
  uint8_t* delayed = nullptr;            // [kGroup][late_paths]
};

struct wr_context {
  int device = 0;
  hipStream_t stream = nullptr;  // API traversal, film set-up / return, joins the pipelines
  Pipe pipes[kMaxPipes];
  // torus 1080p BDPT, groups of 2 (Mrays/s): 4 pipelines / 4 queues 832,
  // 8 / 8 -> 864, 16 / 16 -> 894 (twice the memory of 8: ~5 GB per buffer set)
  int npipes = 4;
  hipEvent_t t_ref = nullptr;  // start of the current render (pipelines wait on it)
  hipEvent_t t_null = nullptr;  // the caller's legacy-stream work before a render
  DevScene ds{};
  Arena scene_mem;
  int64_t scene_bytes = 0;
  DevCounters* ctr = nullptr;  // API traversal
  float* film_tmp = nullptr;
  size_t film_tmp_n = 0;
  float* film_bak = nullptr;  // a device film as it was before a BDPT render (redone on pool overflow)
  size_t film_bak_n = 0;
  DevCounters* host_ctr = nullptr;  // pinned: the pipelines' counters after a render (finish_render)
  char* api_tmp = nullptr;  // wr_trace_closest / wr_occluded / wr_path_radiance scratch, grown on demand
  size_t api_tmp_n = 0;
  int grid = 2048;
  int cus = 256;
  float sph_r = 0.f;  // sceneSphere.sceneRadius (scene.cpp:483-487): VCM base radius
  float vcm_cell = 1.f;  // VCM merge-grid cell edge in query half-widths (WR_VCM_CELL); measured 2 -> 1: +4 %
  bool spheres = false;
  bool narrow = false;  // <= 65536 nodes, leaves <= 255 refs: 16-bit stack / pair offsets
  bool trace_log = false;  // WR_TRACE_LOG=1: per-launch ray counts and durations
  bool stamps = false;  // WR_TRACE_STAMPS=1: diagnostic traversal with phase stamps
  int trace_blocks = 4096;        // resident one-wave workgroups of the traversal
  int trace_blocks_dense = 4096;  // the same for the TRACE_DENSE layout
  bool api_dense = false;         // test knob WR_TRACE_DENSE=1: API launches in TRACE_DENSE
  bool no_cut = false;            // WR_TRACE_NO_CUT=1: shadow rays run to the end (no occl_cut)
  bool timing = false;
  // BDPT pieces (plan_pieces): at most piece_cap paths per buffer set, shares of
  // at least piece_min paths per pipeline (env WR_PIECE_CAP / WR_PIECE_MIN).
  // A short render runs on fewer, fuller pipelines: measured C2 Mrays/s for
  // piece_min 16 K / 384 K / 512 K / 640 K / 768 K / 1 M paths at 1 iteration
  // 656 / 771 / 951 / 1,002 / 868 / 841, at 4 iterations 1,559 / 1,585 /
  // 1,334 / 1,659 / 1,669 / 1,717; 20 and 256 iterations within noise
  // (profiles/r3/piece_min)
  int piece_cap = 1 << 21;
  int piece_min = 655360;
  // pipelines' k_fast_hard: launches with at most this many ties resolve them
  // one per wave (env WR_TIE_WAVE_MAX; 0: always one per lane).  Measured
  // (C2, profiles/r4/tie_wave_max): 512 -> 4096 lifts 1 iteration from
  // 1,182 to 1,328 Mrays/s and keeps 20 (2,766 -> 2,788); every tie one per
  // wave loses at 20 (2,432)
  int tie_wave_max = 4096;
  // k_fast_hard's scan-list waves (WR_SCAN_WAVES): 1,024 against 256, five runs each: C4 +1.3 %,
  // C2 20 it. +0.5 %, C3 and one iteration alike (profiles/r6/scan_waves*.txt)
  int scan_waves = 1024;
  // host threads issuing a render's launches (env WR_ISSUE_THREADS): the
  // pipelines are dealt out to them, each thread issues its pipelines' steps
  int issue_threads = 1;
  // verified-BVH traversal (wr_fast.h): built at wr_create for triangle scenes
  FastScene fs{};
  // a binary-tree scene's 4-wide tree, searched by renders whose pipelines
  // hold one group each (latency-bound: C2 at 1 iteration +6 %, -3 % at 20);
  // wide_now: the tree the current render searches (0: fs)
  int sdepth4 = 0;  // the 4-wide tree's search stack (search_scene)
  bool fs4_ok = false;
  bool lat_wide = true;  // env WR_BVH_WIDE_LAT=0: off
  int wide_now = 0;
  bool lat_now = false;  // the current BDPT render is latency-bound (see wide_now)
  Arena fast_mem;
  bool fast_ok = false;   // scene supports it
  bool fast_on = false;   // WR_TRACE_BVH mode selected
  int fast_blocks = 4096; // resident one-wave workgroups of k_trace_fast
  int resolve_blocks = 0; // k_fast_resolve's one-wave workgroups (0: fast_blocks; env WR_RESOLVE_GRID per CU)
  bool resolve_list = true;  // the search lists the rays the resolve must see (env WR_RESOLVE_LIST=0: all rays)
  bool verify = false;      // WR_BVH_VERIFY=1: every BVH answer checked against the KD walk
  // BDPT hard rays off the critical path (env WR_DEFER=1; off by default)
  int defer = -1;
  // BDPT light and camera passes overlapped (wr_bdpt.h; env WR_BDPT_OVERLAP=0: sequential)
  bool bdpt_overlap = true;
  float* api_t2 = nullptr;  // t2 scratch of the API path
  size_t api_t2_cap = 0;
  int2* api_spill = nullptr;  // the API path's search stack spill area
  // ---- several GPUs (wr_create_multi): this context drives devices[0], `subs`
  // the others; work is dealt to all of them and their films are summed on
  // devices[0] (RCCL reduce over xGMI when the devices are distinct)
  std::vector<wr_context*> subs;
  std::vector<ncclComm_t> dev_comms;  // one per device (ncclCommInitAll), empty: peer copies
  float* red_buf = nullptr;  // this device's film of a multi-device render
  size_t red_n = 0;
  float* stage_buf = nullptr;  // devices[0]: a peer film copied in before it is added
  size_t stage_n = 0;
  // ---- one process per GPU (wr_comm_init): this rank's communicator
  ncclComm_t comm = nullptr;
  int comm_ranks = 0, comm_rank = 0;
};

namespace {

// RCCL, bound at first use: the copy already in the process (PyTorch's) when
// its symbols are global, else ROCm's librccl.so.1.  Single-device contexts
// never load it.
struct RcclApi {
  bool ok = false;
  std::string why;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*init_all)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, int, ncclComm_t,
                         hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  ncclResult_t (*destroy)(ncclComm_t) = nullptr;
  const char* (*err_str)(ncclResult_t) = nullptr;
  ncclResult_t (*count)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*user_rank)(const ncclComm_t, int*) = nullptr;
};
const RcclApi& rccl() {
  static const RcclApi api = [] {
    RcclApi a;
    void* h = dlsym(RTLD_DEFAULT, "ncclCommInitRank") ? RTLD_DEFAULT : nullptr;
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char* e = dlerror();
      a.why = std::string("RCCL not loadable: ") + (e ? e : "librccl.so.1");
      return a;
    }
    auto sym = [&](auto& f, const char* name) {
      f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name));
      return f != nullptr;
    };
    a.ok = sym(a.get_unique_id, "ncclGetUniqueId") && sym(a.init_rank, "ncclCommInitRank") &&
           sym(a.init_all, "ncclCommInitAll") && sym(a.reduce, "ncclReduce") && sym(a.group_start, "ncclGroupStart") &&
           sym(a.group_end, "ncclGroupEnd") && sym(a.destroy, "ncclCommDestroy") && sym(a.err_str, "ncclGetErrorString") &&
           sym(a.count, "ncclCommCount") && sym(a.user_rank, "ncclCommUserRank");
    if (!a.ok) a.why = "RCCL lacks an entry point";
    return a;
  }();
  return api;
}
#define NCCLCHK(expr)                                                                           \
  do {                                                                                          \
    ncclResult_t r_ = (expr);                                                                   \
    if (r_ != ncclSuccess) return fail(WR_E_HIP, std::string(#expr ": ") + rccl().err_str(r_)); \
  } while (0)

// films of a multi-device render, summed on devices[0] (peer-copy path)
__global__ void __launch_bounds__(256) k_film_accumulate(float* dst, const float* src, size_t n) {
  for (size_t i = blockIdx.x * size_t(256) + threadIdx.x; i < n; i += size_t(gridDim.x) * 256) dst[i] += src[i];
}

// overlapped: the BDPT render's own layout (the camera pass's extension queues
// and the camera-vertex store); VertexCM's BDPT part runs the sequential
// schedule and goes without them
// Overlapped BDPT: the shadow / aux queues and the vertex pools per path of
// a buffer set (wr_bdpt.h, BdptBuf): what the reference scenes use is far
// below the worst case (torus: ~3 % of the 11 shadow rays a path may queue in
// one step; ~1 stored light vertex of 9), so they are sized by use and a
// render that fills one is redone with pieces the worst case fits (exact).
// Env WR_BDPT_POOL_SCALE scales all three (tests force small ones); 0: the
// worst case, no pools.
constexpr float kSqPerPath = 2.f, kVPoolPerPath = 2.f, kCPoolPerPath = 1.f;
float bdpt_pool_scale() {  // (read at every layout: a change re-lays out the buffers, ensure_work)
  const char* e = std::getenv("WR_BDPT_POOL_SCALE");
  return e ? std::max(0.f, static_cast<float>(std::atof(e))) : 1.f;
}
// capacity of a pool of `per` records per path, at least `floor` (a safe
// re-render piece of 64 paths fits), at most the worst case
int pool_cap(int P, float per, int worst, int floor) {
  const float s = bdpt_pool_scale();
  if (s <= 0.f) return worst * P;
  const double want = std::ceil(static_cast<double>(P) * per * s);
  return static_cast<int>(std::min<double>(static_cast<double>(worst) * P, std::max<double>(want, floor)));
}

void layout_bdpt(Arena& a, BdptBuf& B, int P, bool overlapped, bool vcm = false) {
  B.P = P;
  // shadow / aux rays queued by one step, per path: sequential schedule, a
  // camera vertex's <= kVMax connections + NEE + DI-BSDF (the light splats of
  // one path: <= kVMax); overlapped, at the step making vertices of length s:
  // camera side <= min(s, 9 - s) connections + NEE + DI-BSDF, light side
  // <= min(s - 1, 9 - s) connections + its splat: <= 11 as well.  Overlapped:
  // sized by use (kSqPerPath), the vertex stores pools (kVPoolPerPath,
  // kCPoolPerPath) -- 1.0 KB per path instead of 3.0 KB
  const bool pools = overlapped && bdpt_pool_scale() > 0.f;
  B.cap_sq = pools ? pool_cap(P, kSqPerPath, kVMax + 2, (kVMax + 2) * 64) : P * (kVMax + 2);
  B.vcap = pools ? pool_cap(P, kVPoolPerPath, kVMax, kVMax * 64) : kVMax * P;
  B.ccap = pools ? pool_cap(P, kCPoolPerPath, kCvMax, kCvMax * 64) : kCvMax * P;
  const size_t sP = P, sV = size_t(B.vcap), sQ = B.cap_sq;
  // subpath records: BDPT's 32-byte BQ_* (wr_bdpt.h), VertexCM's 64-byte PS_*
  const size_t rec = vcm ? PS_WORDS : BQ_WORDS;
  B.ls = a.take<float>(rec * sP);
  B.cs = a.take<float>(rec * sP);
  // stored vertices: BDPT's 64-byte BV_* records, VertexCM's 80-byte VS_*
  B.vs = a.take<float>((vcm ? VS_WORDS : BV_WORDS) * sV);
  B.cv = overlapped ? a.take<float>(BV_WORDS * size_t(B.ccap)) : nullptr;
  B.lvc = vcm ? nullptr : a.take<uint8_t>(sP);
  B.cvc = vcm ? nullptr : a.take<uint8_t>(sP);
  B.vidx = pools ? a.take<int>(size_t(kVMax) * P) : nullptr;
  B.cidx = pools ? a.take<int>(size_t(kCvMax) * P) : nullptr;
  // overlapped: an extension queue holds both passes' rays (light, then camera)
  B.qs = overlapped ? 2 * P : P;
  const size_t sE = B.qs;

  for (int q = 0; q < 2; ++q) {
    B.q_o[q] = a.take<float>(3 * sE);
    B.q_d[q] = a.take<float>(3 * sE);
    B.q_t[q] = a.take<float>(sE);
    B.q_path[q] = a.take<int>(sE);
    B.q_prim[q] = a.take<int>(sE);
  }
  for (int k = 0; k < 2; ++k) {
    BdptBuf::Sq& q = B.sq[k];
    q.o = a.take<float>(3 * sQ);
    q.d = a.take<float>(3 * sQ);
    q.tgt = a.take<float>(3 * sQ);
    q.val = a.take<float>(3 * sQ);
    q.t = a.take<float>(sQ);
    q.cut = a.take<float>(sQ);
    q.meta = a.take<int>(sQ);
    q.pix = a.take<int>(sQ);
    q.prim = a.take<int>(sQ);
    B.di[k].r = a.take<float>(DR_WORDS * sP);
  }
}

void layout_pt(Arena& a, PtBuf& T, int P) {
  T.P = P;
  const size_t sP = P;
  T.st = a.take<float>(PT_WORDS * sP);
  for (int q = 0; q < 2; ++q) {
    T.q_o[q] = a.take<float>(3 * sP);
    T.q_d[q] = a.take<float>(3 * sP);
    T.q_t[q] = a.take<float>(sP);
    T.q_path[q] = a.take<int>(sP);
    T.q_prim[q] = a.take<int>(sP);
  }
  for (int k = 0; k < 2; ++k) {
    PtBuf::Sq& Q = T.sq[k];
    Q.o = a.take<float>(3 * sP);
    Q.d = a.take<float>(3 * sP);
    Q.tgt = a.take<float>(3 * sP);
    Q.val = a.take<float>(3 * sP);
    Q.t = a.take<float>(sP);
    Q.cut = a.take<float>(sP);
    Q.pix = a.take<int>(sP);
    Q.prim = a.take<int>(sP);
  }
}

// VCM merge grid: 2^k buckets, at least twice the paths (light vertices
// average ~0.5-1 per path in the reference scenes)
uint32_t vcm_table(int P) {
  uint32_t t = kRowW;
  while (t < 2u * static_cast<uint32_t>(P)) t <<= 1;
  return t;
}
size_t vcm_scan_bytes(uint32_t T) {
  size_t b = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, b, static_cast<const int*>(nullptr), static_cast<int*>(nullptr),
                                         static_cast<int>(T + 1));
  return b;
}
void layout_vcm(Arena& a, VcmBuf& V, int P) {
  const size_t sP = P, sV = size_t(kVMax) * P;
  const uint32_t T = vcm_table(P);
  V.l_sb = a.take<float4>(sP);
  V.v_dvm = a.take<float>(sV);
  V.pending = a.take<int>(sP);
  V.cnt = a.take<int>(size_t(T) + 1);
  V.start = a.take<int>(size_t(T) + 1);
  V.rpos = a.take<float4>(sV);
  V.rdat = a.take<float4>(2 * sV);
  V.rdvm = a.take<float>(sV);
  for (int k = 0; k < 2; ++k) {
    VcmBuf::Mq& M = V.mq[k];
    M.hp = a.take<float>(3 * sP);
    M.n = a.take<float>(3 * sP);
    M.wi = a.take<float>(3 * sP);
    M.thr = a.take<float>(3 * sP);
    M.dvcm = a.take<float>(sP);
    M.dvm = a.take<float>(sP);
    M.cont = a.take<float>(sP);
    M.pd = a.take<float>(sP);
    M.pg = a.take<float>(sP);
    M.mat = a.take<int>(sP);
    M.len = a.take<int>(sP);
    M.pix = a.take<int>(sP);
  }
  V.scan_bytes = vcm_scan_bytes(T);
  V.scan_tmp = a.take<char>(V.scan_bytes);
}

// one buffer set of `kind` (into dst's set g, or only measured)
void layout_set(Arena& a, Pipe* dst, int g, int kind, int P) {
  BdptBuf b;
  PtBuf t;
  VcmBuf v;
  if (kind == 2) {
    layout_pt(a, dst ? dst->pb[g] : t, P);
    return;
  }
  layout_bdpt(a, dst ? dst->bb[g] : b, P, kind == 1, kind == 3);
  if (kind == 3) layout_vcm(a, dst ? dst->vb[g] : v, P);
}

int ensure_work(Pipe& p, int kind, int P, int sets) {
  // (a VCM layout holds the sequential BDPT layout only: no camera-pass queues)
  const bool same = p.work_kind == kind && p.work_pool == bdpt_pool_scale();
  if (same && p.work_key == static_cast<size_t>(P) && p.work_sets >= sets) return WR_OK;
  p.work_kind = 0;
  auto lay = [&](Arena& a, Pipe* dst) {
    for (int g = 0; g < sets; ++g) layout_set(a, dst, g, kind, P);
  };
  int rc = p.work.reserve(measure([&](Arena& a) { lay(a, nullptr); }));
  if (rc) return rc;
  lay(p.work, &p);
  p.work_kind = kind;
  p.work_key = P;
  p.work_sets = sets;
  p.work_pool = bdpt_pool_scale();
  return WR_OK;
}

// Work buffers for up to `want` pipelines, each with `sets` buffer sets (~2.5 KB
// per path for BDPT), kept within 3/4 of the device memory free now plus what
// the pipelines already hold: big films degrade to fewer pipelines instead of
// failing.  Every render lays out full groups on all pipelines that fit, so a
// short render (a warm-up) leaves the buffers of a long one in place.
int pipelines_that_fit(wr_context* c, int kind, int P, int sets, int want) {
  const size_t per = measure([&](Arena& a) {
    for (int g = 0; g < sets; ++g) layout_set(a, nullptr, g, kind, P);
  });
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return want;
  size_t held = 0;
  for (int i = 0; i < kMaxPipes; ++i) held += c->pipes[i].work.cap;
  const size_t budget = (free_b + held) / 4 * 3;
  const int fit = static_cast<int>(std::min<size_t>(static_cast<size_t>(want), std::max<size_t>(1, budget / per)));
  for (int i = fit; i < kMaxPipes; ++i) {  // memory-limited: free the rest
    c->pipes[i].work.release();
    c->pipes[i].work_kind = 0;
  }
  for (int i = 0; i < fit; ++i)
    if (ensure_work(c->pipes[i], kind, P, sets) != WR_OK) return 0;
  return fit;
}

// ---- launch helpers with optional per-launch HIP events (on the pipeline's stream)
// Flags of the library's events.  By default HIP records an event with a
// system-scope release (cache writeback for host visibility); the render's
// events only order and time work on this device, so they skip it
// (hipEventDisableSystemFence).  Env WR_EVENT_SYSTEM_FENCE=1 restores it.
unsigned ev_flags(unsigned base) {
  static const bool sys = [] {
    const char* e = std::getenv("WR_EVENT_SYSTEM_FENCE");
    return e && std::atoi(e) != 0;
  }();
  return sys ? base : (base | hipEventDisableSystemFence);
}

struct Timer {
  wr_context* c;
  Pipe* p;
  Timer(wr_context* cc, Pipe* pp) : c(cc), p(pp) {}
  void mark(int cat) {
    if (!c->timing || !p) return;
    if (p->ev_used >= p->events.size()) {
      hipEvent_t e;
      (void)hipEventCreateWithFlags(&e, ev_flags(hipEventDefault));
      p->events.push_back(e);
      p->ev_cat.push_back(0);
    }
    p->ev_cat[p->ev_used] = cat;
    (void)hipEventRecord(p->events[p->ev_used++], p->stream);
  }
};

RayQueue rq(const float* o3, const float* d3, int cap, const int* cnt, float* t, int* prim,
            const float* tmin = nullptr, const float* tmax = nullptr, const float* cut = nullptr,
            const LateList* late = nullptr, int* late_n = nullptr, int late_bit = 0, const int* cnt2 = nullptr) {
  return RayQueue{o3, d3, cap, cnt, tmin, tmax, t, prim, cut, late, late_n, late_bit, cnt2};
}
// a queue's ray count read back to the host (diagnostics only: synchronous)
int host_count(const RayQueue& q) {
  int k = 0, k2 = 0;
  if (q.count) (void)hipMemcpy(&k, q.count, sizeof(int), hipMemcpyDeviceToHost);
  if (q.count2) (void)hipMemcpy(&k2, q.count2, sizeof(int), hipMemcpyDeviceToHost);
  return k + k2;
}
// queues of one launch (empty `count` pointers are skipped)
struct QueueList {
  TraceQueues Q{};
  int max_rays = 0;
  void add(const RayQueue& q, int cap) {
    if (Q.n >= kMaxQueues) {  // a schedule asking for more queues than a launch takes: a build error
      std::fprintf(stderr, "winmad_rt: more than %d queues in one traversal launch\n", kMaxQueues);
      std::abort();
    }
    Q.q[Q.n++] = q;
    max_rays += cap;
  }
};

using TraceKernel = void (*)(DevScene, TraceQueues, DevCounters*, int*);
// cut: the launch's shadow rays may stop once occlusion is settled (occl_cut).
// Only PT, VCM and the API use it: BDPT launches carry 3 % shadow rays, and
// the check costs C2 1.5 % (measured).  TRACE_DENSE: cut + the 20-waves/CU
// layout (PT).
enum TraceMode { TRACE_PLAIN = 0, TRACE_CUT = 1, TRACE_DENSE = 2 };
#ifndef WR_BDPT_TRACE_MODE
// BDPT light / camera passes.  TRACE_DENSE without the cutoff (WR_DENSE_CUT
// false) measured C2 -2.5 % (-3.7 % with per-queue uniform branches)
#define WR_BDPT_TRACE_MODE TRACE_PLAIN
#endif
#ifndef WR_DENSE_CUT
#define WR_DENSE_CUT true  // TRACE_DENSE instances carry the occlusion cutoff
#endif
#ifndef WR_VCM_TRACE_MODE
#define WR_VCM_TRACE_MODE TRACE_CUT  // camera pass of VCM (TRACE_DENSE: -1.3 %)
#endif
TraceKernel trace_kernel(bool count, bool spheres, bool narrow, bool stamps, int mode = TRACE_PLAIN) {
  if (stamps) return narrow ? k_trace<false, false, true, true> : k_trace<false, false, false, true>;
  if (mode == TRACE_DENSE) {
    constexpr bool C = WR_DENSE_CUT;
    if (count) {
      if (spheres) return narrow ? k_trace<true, true, true, false, C, true> : k_trace<true, true, false, false, C, true>;
      return narrow ? k_trace<true, false, true, false, C, true> : k_trace<true, false, false, false, C, true>;
    }
    if (spheres) return narrow ? k_trace<false, true, true, false, C, true> : k_trace<false, true, false, false, C, true>;
    return narrow ? k_trace<false, false, true, false, C, true> : k_trace<false, false, false, false, C, true>;
  }
  if (mode == TRACE_CUT) {
    if (count) {
      if (spheres) return narrow ? k_trace<true, true, true, false, true> : k_trace<true, true, false, false, true>;
      return narrow ? k_trace<true, false, true, false, true> : k_trace<true, false, false, false, true>;
    }
    if (spheres) return narrow ? k_trace<false, true, true, false, true> : k_trace<false, true, false, false, true>;
    return narrow ? k_trace<false, false, true, false, true> : k_trace<false, false, false, false, true>;
  }
  if (count) {
    if (spheres) return narrow ? k_trace<true, true, true> : k_trace<true, true, false>;
    return narrow ? k_trace<true, false, true> : k_trace<true, false, false>;
  }
  if (spheres) return narrow ? k_trace<false, true, true> : k_trace<false, true, false>;
  return narrow ? k_trace<false, false, true> : k_trace<false, false, false>;
}

// The device counters of one traversal step: the persistent cursor (zero at
// the step's start: the iteration's counter memset, or the caller), and in
// WR_TRACE_BVH mode the per-ray t2 scratch of the BVH search (>= the launch's rays).
struct TraceSlot {
  int* fetch;
  float* t2;      // [t2_cap] t2 per launch index, then [t2_cap] the tie list (from the bottom) and the scan list (from the
                  // top), then [t2_cap] int2 pair records (kPairWindow), then [t2_cap] the pair list
  size_t t2_cap;
  int* hard_n;
  int2* spill;    // the search stack's spill area
  int* rlist_n;   // rays the search left to k_fast_resolve (their list: the t2 region)
};
TraceSlot tslot(Pipe& p, int slot) {
  return TraceSlot{&p.sc[0].fetch[slot], p.t2buf, p.t2_cap, &p.sc[0].hard[slot][0], p.spill, &p.sc[0].rlist[slot]};
}
// t2 scratch + hard-ray list of a pipeline for launches of up to `rays` rays
// search-stack spill entries per lane: the larger of the context's trees
size_t max_spill_entries(const wr_context* c) {
  size_t e = search_spill_entries(c->fs.sdepth, c->fs.wide);
  if (c->fs4_ok) e = std::max(e, search_spill_entries(c->sdepth4, 4));
  return e;
}
// the scene as the current render searches it: fs, or fs with its 4-wide
// tree (every other field -- KD stack depth, diagnostics -- is fs's own)
FastScene search_scene(const wr_context* c) {
  FastScene F = c->fs;
  // a latency-bound render keeps every near-tie one per wave (the pair list's
  // one per lane waits for its slowest lane: C2 at 1 iteration -4 %, while C4 at
  // 64 iterations gains 2.6 %, profiles/r6/pair_list/ab.txt)
  if (c->lat_now && F.pair > 1) F.pair = 1;
  if (c->wide_now == 4 && c->fs4_ok) {
    F.wide = 4;
    F.sdepth = c->sdepth4;
  }
  return F;
}
int ensure_t2(wr_context* c, Pipe& p, size_t rays) {
  if (!c->fast_on) return WR_OK;
  if (!p.spill && max_spill_entries(c) > 0)
    HIPCHK(hipMalloc(&p.spill, max_spill_entries(c) * size_t(c->fast_blocks) * 64 * sizeof(int2)));
  if (p.t2_cap >= rays) return WR_OK;
  if (p.t2buf) (void)hipFree(p.t2buf);
  p.t2buf = nullptr;
  p.t2_cap = 0;
  HIPCHK(hipMalloc(&p.t2buf, 5 * rays * sizeof(float)));  // t2 / list, hard lists, pair records (int2), pair list
  p.t2_cap = rays;
  return WR_OK;
}

// Late lists of a pipeline (deferred hard rays), `recs` records each, for
// buffer sets of `paths` paths.  The lists' queue path arrays are the
// pipeline's current BDPT buffers.
int ensure_late(Pipe& p, int paths, int recs) {
  if (p.late_recs < static_cast<size_t>(recs) || p.late_paths < static_cast<size_t>(paths)) {
    recs = std::max<int>(recs, static_cast<int>(p.late_recs));
    paths = std::max<int>(paths, static_cast<int>(p.late_paths));
    auto lay = [&](Arena& a, bool set) {
      for (int m = 0; m < kGroup; ++m)
        for (int k = 0; k < 2; ++k) {
          LateList L{};
          L.cap = recs;
          L.o3 = a.take<float>(3 * size_t(recs));
          L.d3 = a.take<float>(3 * size_t(recs));
          L.t1 = a.take<float>(recs);
          L.p1 = a.take<int>(recs);
          L.pth = a.take<int>(recs);
          L.tie = a.take<int>(recs);
          L.t = a.take<float>(recs);
          L.prim = a.take<int>(recs);
          if (set) p.late_h[m][k] = L;
        }
      uint8_t* dl = a.take<uint8_t>(size_t(kGroup) * paths);
      LateList* ld = a.take<LateList>(size_t(kGroup) * 2);
      if (set) {
        p.delayed = dl;
        p.late_d = ld;
      }
    };
    if (int rc = p.late_mem.reserve(measure([&](Arena& a) { lay(a, false); }))) return rc;
    lay(p.late_mem, true);
    p.late_recs = recs;
    p.late_paths = paths;
  }
  for (int m = 0; m < kGroup; ++m)
    for (int k = 0; k < 2; ++k) {
      LateList& L = p.late_h[m][k];
      L.path = p.bb[m].q_path[k];
      L.delayed = p.delayed + size_t(m) * p.late_paths;
    }
  HIPCHK(hipMemcpyAsync(p.late_d, p.late_h, sizeof(p.late_h), hipMemcpyHostToDevice, p.stream));
  return WR_OK;
}

// One persistent traversal launch over the queues of Q (max_rays bounds the
// grid).  WR_TRACE_BVH: the verified-BVH search + its resolve launch instead.
// Blocks of a fused search launch that settle the previous step's late lists:
// per group member kLateTieBlocks tie waves (one tie per wave up to that many,
// else one per lane on kLateLaneBlocks) and kLateScanBlocks scan waves
constexpr int kLateTieBlocks = 256, kLateLaneBlocks = 64, kLateScanBlocks = 64;
int trace_launch(wr_context* c, hipStream_t stream, DevCounters* ctr, const TraceSlot& ts, Timer& tm, bool count,
                 const TraceQueues& Q_, int max_rays, int mode = TRACE_PLAIN, bool hard_wave = false,
                 const LateArgs* late_prev = nullptr, int late_gn = 0) {
  int* fetch = ts.fetch;
  TraceQueues Q = Q_;
  if (c->no_cut)  // measurement knob: the same launches without the dead-work elision
    for (int i = 0; i < Q.n; ++i) Q.q[i].cut = nullptr;
  if (c->fast_on && !c->stamps && ts.t2 && static_cast<size_t>(max_rays) <= ts.t2_cap) {
    const FastScene F = search_scene(c);  // the render's search tree
    const int blocks = (max_rays + kTraceBlock - 1) / kTraceBlock;
    const int fgrid = std::max(1, std::min(c->fast_blocks, blocks));
    const size_t lds = fast_lds_bytes(c->fs.depth), slds = search_lds_bytes(F.sdepth, F.wide);
    // the search settles the rays its first membership test proves and lists
    // the rest for the resolve (in the t2 region: t2 is kept by diagnostics
    // only).  Measured (profiles/r5/resolve_list): C4 +5 %, C2 +1 %, VCM +1 %;
    // PT's dense launches -0.8 %, so they keep the resolve over every ray
    const bool rl = c->resolve_list && !F.diag && !late_prev && !F.sph && F.wide != 8 && mode != TRACE_DENSE;
    int* rlist = rl ? reinterpret_cast<int*>(ts.t2) : nullptr;
    int* rlist_n = rl ? ts.rlist_n : nullptr;
    const size_t rlds = slds + (rl ? kRlistLds : 0);
    // the search's pair records of near-ties (kPairWindow): after the lists
    int2* pairs = reinterpret_cast<int2*>(ts.t2 + 2 * ts.t2_cap);
    hipEvent_t f0 = nullptr, f1 = nullptr, fa = nullptr, fb = nullptr;
    if (c->trace_log) {
      (void)hipEventCreate(&f0);
      (void)hipEventCreate(&f1);
      (void)hipEventCreate(&fa);
      (void)hipEventCreate(&fb);
      (void)hipEventRecord(f0, stream);
    }
    if (late_prev) {  // + the previous step's deferred hard rays, beside the search
      const int lblocks = late_gn * (kLateTieBlocks + kLateScanBlocks);
      auto kf = count ? trace_fast_kernel<true, true>(F.wide, F.sph) : trace_fast_kernel<false, true>(F.wide, F.sph);
      hipLaunchKernelGGL(kf, dim3(lblocks + fgrid),
                         dim3(kTraceBlock), std::max(slds, lds), stream, c->ds, F, Q, ctr, fetch, ts.t2, pairs, ts.spill,
                         *late_prev, lblocks, late_gn, kLateTieBlocks, kLateLaneBlocks, kLateTieBlocks, nullptr, nullptr);
      if (c->verify)
        hipLaunchKernelGGL(k_late_verify, dim3(64, late_gn), dim3(kTraceBlock), lds, stream, c->ds, F, *late_prev,
                           ctr);
    } else {
      auto kf = count ? trace_fast_kernel<true, false>(F.wide, F.sph, rl)
                      : trace_fast_kernel<false, false>(F.wide, F.sph, rl);
      hipLaunchKernelGGL(kf, dim3(fgrid),
                         dim3(kTraceBlock), rlds, stream, c->ds, F, Q, ctr, fetch, ts.t2, pairs, ts.spill, LateArgs{}, 0,
                         1, 0, 0, 0, rlist, rlist_n);
    }
    if (c->trace_log) (void)hipEventRecord(fa, stream);
    int* hard = reinterpret_cast<int*>(ts.t2 + ts.t2_cap);
    hipLaunchKernelGGL(count ? k_fast_resolve<true> : k_fast_resolve<false>,
                       dim3(std::max(1, std::min(c->resolve_blocks > 0 ? c->resolve_blocks : c->fast_blocks, blocks))),
                       dim3(kTraceBlock), 0, stream, c->ds, F,
                       Q, ctr, ts.t2, hard, ts.hard_n, static_cast<int>(ts.t2_cap), rlist, rlist_n);
    if (c->trace_log) (void)hipEventRecord(fb, stream);
    // the hard rays are a few in 10^4: a small grid drains any count (one
    // ray per wave for the API calls: up to 2048 at once, 8 waves per CU)
    // (pipelines: up to c->tie_wave_max ties one per wave, more one per lane)
    const int lgrid = std::max(1, std::min(256, blocks));
    const int hgrid = hard_wave ? std::max(1, std::min(2048, max_rays))
                                : std::max(lgrid, std::min(c->tie_wave_max, max_rays));
    const int sgrid = std::max(1, std::min(c->scan_waves, max_rays));  // scan waves
    auto hk = hard_wave ? (count ? k_fast_hard<true, true> : k_fast_hard<false, true>)
                        : (count ? k_fast_hard<true, false> : k_fast_hard<false, false>);
    // the pair list (near-ties the search's pair record settles, one per lane)
    const int pgrid = (F.diag || F.pair < 2) ? 0 : lgrid;
    hipLaunchKernelGGL(hk, dim3(hgrid + pgrid + sgrid),
                       dim3(kTraceBlock), lds, stream, c->ds, F, Q, ctr, hard, ts.hard_n,
                       static_cast<int>(ts.t2_cap), hgrid, lgrid, std::min(hgrid, c->tie_wave_max), pgrid);
    if (c->verify)
      hipLaunchKernelGGL(k_fast_verify, dim3(std::max(1, std::min(c->fast_blocks, blocks))), dim3(kTraceBlock), lds,
                         stream, c->ds, F, Q, ctr);
    tm.mark(WR_K_TRACE);
    if (c->trace_log) {
      (void)hipEventRecord(f1, stream);
      (void)hipEventSynchronize(f1);
      int tot = 0;
      for (int i = 0; i < Q.n; ++i) tot += host_count(Q.q[i]);
      float ms = 0.f, ma = 0.f, mb = 0.f;
      int nhs[3] = {0, 0, 0};
      (void)hipMemcpy(nhs, ts.hard_n, 3 * sizeof(int), hipMemcpyDeviceToHost);
      const int nh = nhs[0], ns = nhs[1];
      (void)hipEventElapsedTime(&ms, f0, f1);
      (void)hipEventElapsedTime(&ma, f0, fa);
      (void)hipEventElapsedTime(&mb, fa, fb);
      std::fprintf(stderr,
                   "[wr bvh] %d rays  %.1f us (search %.1f, resolve %.1f, hard %.1f: %d + %d pair + %d scan rays)  grid %d\n",
                   tot, ms * 1e3f, ma * 1e3f, mb * 1e3f, (ms - ma - mb) * 1e3f, nh, nhs[2], ns, fgrid);
      (void)hipEventDestroy(f0);
      (void)hipEventDestroy(f1);
      (void)hipEventDestroy(fa);
      (void)hipEventDestroy(fb);
    }
    return WR_OK;
  }
  const bool dense = mode == TRACE_DENSE && !c->stamps;
  const size_t lds = trace_lds_bytes(c->ds.max_stack, c->narrow, dense);
  const int grid =
      std::max(1, std::min(dense ? c->trace_blocks_dense : c->trace_blocks, (max_rays + kTraceBlock - 1) / kTraceBlock));
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c->trace_log) {  // diagnostic (WR_TRACE_LOG=1): rays and duration of every launch
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, stream);
  }
  hipLaunchKernelGGL(trace_kernel(count, c->spheres, c->narrow, c->stamps, mode), dim3(grid), dim3(kTraceBlock), lds,
                     stream, c->ds, Q, ctr, fetch);
  tm.mark(WR_K_TRACE);
  if (c->trace_log) {
    (void)hipEventRecord(e1, stream);
    (void)hipEventSynchronize(e1);
    int tot = 0;
    for (int i = 0; i < Q.n; ++i) tot += host_count(Q.q[i]);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::fprintf(stderr, "[wr trace] %d queues, %d rays  %.1f us  grid %d\n", Q.n, tot, ms * 1e3f, grid);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
  return WR_OK;
}

int shade_grid(wr_context* c, int n) { return std::max(1, std::min(c->grid, (n + kShadeBlock - 1) / kShadeBlock)); }

// ---- BDPT work split.  A render is iterations x (W*H) paths; light path i
// pairs only with camera path i of the same iteration (:130, :222-229), MIS
// uses the global lightPathNum (:55), and splats are film atomics, so any
// partition of an iteration's path range renders the same film (up to the order
// of float atomics).  The render's path-iterations, flattened iteration-major,
// are split into one contiguous, equal share per pipeline (whole 8-row bands in
// the tiled camera order); a share is cut at iteration boundaries and into
// pieces of at most `cap` paths, and each pipeline runs its pieces in groups of
// kGroup.  Few iterations then still fill every pipeline (the reference's own
// default is 1 iteration, bidirPathTracing.cpp:9), and work buffers are sized by
// the piece, not the frame.
struct Piece {
  int iter;  // iteration index within the render
  int base;  // first global path
  int n;     // paths
};
struct PiecePlan {
  std::vector<std::vector<std::vector<Piece>>> per_pipe;  // [pipeline][group][member]
  int pipes() const { return std::max(1, static_cast<int>(per_pipe.size())); }
  int max_groups() const {
    size_t m = 0;
    for (const auto& v : per_pipe) m = std::max(m, v.size());
    return static_cast<int>(m);
  }
};
// a position in the flattened (iteration-major) path order, moved to the
// nearest whole unit of its iteration (an iteration's end is a boundary)
int64_t flat_round(int64_t f, int P, int unit) {
  const int64_t it = f / P, off = f % P;
  return it * P + std::min<int64_t>(P, (off + unit / 2) / unit * unit);
}
// [a, b) cut at iteration ends and into near-equal unit-aligned pieces of at
// most cap paths.  The stretch is counted in units (the last one may be
// partial: an iteration's end need not be unit-aligned) and each piece gets
// at most floor(cap / unit) of them, so no piece exceeds cap even when the
// stretch is not a multiple of the unit (cap is a whole number of units, or
// the frame itself).
void cut_pieces(int64_t a, int64_t b, int P, int unit, int cap, std::vector<Piece>& out) {
  const int64_t cap_units = std::max<int64_t>(1, cap / unit);
  while (a < b) {
    const int64_t it = a / P, off = a % P;
    const int64_t len = std::min<int64_t>(b - a, P - off);  // up to the iteration's end
    const int64_t units = (len + unit - 1) / unit;
    const int64_t cuts = (units + cap_units - 1) / cap_units;
    for (int64_t j = 0; j < cuts; ++j) {
      const int64_t lo = off + std::min(len, units * j / cuts * unit);
      const int64_t hi = off + std::min(len, units * (j + 1) / cuts * unit);
      if (hi > lo) out.push_back(Piece{static_cast<int>(it), static_cast<int>(lo), static_cast<int>(hi - lo)});
    }
    a += len;
  }
}
// The flattened path-iterations [lo, hi) (lo, hi whole units) over np
// pipelines, in groups of kGroup pieces.  (Splitting a short render's share
// unevenly into two groups per pipeline, so that the pipelines' late bounces
// fall at different times, measured worse: C2 at 20 iterations 2,292 ->
// 1,850 Mrays/s -- each extra group pays the bounce tails again.)
PiecePlan plan_pieces(int64_t lo, int64_t hi, int P, int unit, int cap, int np, int min_piece) {
  PiecePlan plan;
  const int64_t T = hi - lo;
  if (T <= 0) {
    plan.per_pipe.resize(1);
    return plan;
  }
  const int64_t shares = std::max<int64_t>(1, std::min<int64_t>(np, T / std::max(1, min_piece)));
  auto bound = [&](int64_t k) { return k == shares ? hi : flat_round(lo + k * T / shares, P, unit); };
  auto groups_of = [&](const std::vector<Piece>& pcs, std::vector<std::vector<Piece>>& gs) {
    for (size_t i = 0; i < pcs.size(); i += kGroup)
      gs.emplace_back(pcs.begin() + i, pcs.begin() + std::min(pcs.size(), i + kGroup));
  };
  for (int64_t k = 0; k < shares; ++k) {
    const int64_t a = bound(k), b = bound(k + 1);
    std::vector<Piece> pcs;
    cut_pieces(a, b, P, unit, cap, pcs);
    std::vector<std::vector<Piece>> gs;
    groups_of(pcs, gs);
    if (!gs.empty()) plan.per_pipe.push_back(std::move(gs));
  }
  if (plan.per_pipe.empty()) plan.per_pipe.resize(1);
  return plan;
}
// paths one buffer set holds: the frame, or WR_PIECE_CAP (default 2^21: a
// 1920x1080 frame is one piece, 4K frames are four) rounded up to whole units
int piece_capacity(const wr_context* c, int P, int unit) {
  const int64_t want = std::min<int64_t>(P, std::max<int64_t>(unit, c->piece_cap));
  return static_cast<int>(std::min<int64_t>(P, (want + unit - 1) / unit * unit));
}

double host_now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Start a render on `n` pipelines: they wait for the context stream's set-up
// (film clear) and clear their counters.
void begin_render(wr_context* c, int n, const int time_kernels) {
  // diagnostics: WR_TIME_KERNELS=0 drops the per-launch events of a timed call
  // (what the events themselves cost)
  static const bool no_events = [] {
    const char* e = std::getenv("WR_TIME_KERNELS");
    return e && std::atoi(e) == 0;
  }();
  c->timing = time_kernels != 0 && !no_events;
  // a device film may still be written by the caller's work on the legacy
  // null stream (e.g. torch's default stream zeroing it): the render's streams
  // are non-blocking, so order them after that work explicitly.  The null
  // stream is named as 0: the hipStreamLegacy handle ((hipStream_t)1) is not
  // understood by the older HIP runtime PyTorch loads first (segfault)
  (void)hipEventRecord(c->t_null, nullptr);
  (void)hipStreamWaitEvent(c->stream, c->t_null, 0);
  (void)hipEventRecord(c->t_ref, c->stream);
  for (int i = 0; i < n; ++i) {
    Pipe& p = c->pipes[i];
    p.ev_used = 0;
    (void)hipStreamWaitEvent(p.stream, c->t_ref, 0);
    (void)hipMemsetAsync(p.ctr, 0, sizeof(DevCounters), p.stream);
    Timer(c, &p).mark(WR_K_OTHER);
  }
}

// Join the pipelines into the context stream, wait, and add up the work
// counters and (time_kernels) the per-launch durations of every pipeline.
// stats->trace_wall_ms is the union of all traversal launch intervals.
int finish_render(wr_context* c, int n, wr_stats* st, double t0_host, unsigned long long* overflow = nullptr) {
  const double t_issued = host_now();
  for (int i = 0; i < n; ++i) {
    (void)hipEventRecord(c->pipes[i].done, c->pipes[i].stream);
    (void)hipStreamWaitEvent(c->stream, c->pipes[i].done, 0);
  }
  // every pipeline's counters to pinned host memory behind the render, one
  // synchronisation (16 synchronous copies took ~0.3 ms of a 60 ms render)
  if (!c->host_ctr) HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&c->host_ctr), kMaxPipes * sizeof(DevCounters), 0));
  for (int i = 0; i < n; ++i)
    HIPCHK(hipMemcpyAsync(&c->host_ctr[i], c->pipes[i].ctr, sizeof(DevCounters), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (std::getenv("WR_ISSUE_LOG"))  // diagnostics: host issue time vs the render's
    std::fprintf(stderr, "[wr issue] %d pipelines: issued in %.3f ms, done at %.3f ms\n", n,
                 (t_issued - t0_host) * 1e3, (host_now() - t0_host) * 1e3);
  HIPCHK(hipGetLastError());
  if (overflow) {  // (read whether or not stats are wanted)
    *overflow = 0;
    for (int i = 0; i < n; ++i) *overflow += c->host_ctr[i].overflow;
  }
  if (!st) return WR_OK;
  DevCounters sum{};
  for (int i = 0; i < n; ++i) {
    const DevCounters& h = c->host_ctr[i];
    sum.closest += h.closest;
    sum.shadow += h.shadow;
    sum.inner += h.inner;
    sum.leaves += h.leaves;
    sum.refs += h.refs;
    sum.tests += h.tests;
    sum.vm_queries += h.vm_queries;
    sum.vm_found += h.vm_found;
    sum.vm_merged += h.vm_merged;
    sum.bvh_nodes += h.bvh_nodes;
    sum.bvh_tests += h.bvh_tests;
    sum.kd_replay += h.kd_replay;
    sum.fallback += h.fallback;
    sum.verify_rays += h.verify_rays;
    sum.verify_bad += h.verify_bad;
    sum.deferred += h.deferred;
    for (int k = 0; k < 8; ++k) sum.stamps[k] += h.stamps[k];
  }
  st->closest_rays += static_cast<int64_t>(sum.closest);
  st->shadow_rays += static_cast<int64_t>(sum.shadow);
  st->inner_visits += static_cast<int64_t>(sum.inner);
  st->leaf_visits += static_cast<int64_t>(sum.leaves);
  st->prim_refs += static_cast<int64_t>(sum.refs);
  st->prim_tests += static_cast<int64_t>(sum.tests);
  st->vm_queries += static_cast<int64_t>(sum.vm_queries);
  st->vm_found += static_cast<int64_t>(sum.vm_found);
  st->vm_merged += static_cast<int64_t>(sum.vm_merged);
  st->bvh_nodes += static_cast<int64_t>(sum.bvh_nodes);
  st->bvh_tests += static_cast<int64_t>(sum.bvh_tests);
  st->kd_replay_steps += static_cast<int64_t>(sum.kd_replay);
  st->fallback_rays += static_cast<int64_t>(sum.fallback);
  st->verify_rays += static_cast<int64_t>(sum.verify_rays);
  st->verify_mismatches += static_cast<int64_t>(sum.verify_bad);
  st->pipelines = std::max<int64_t>(st->pipelines, n);
  st->deferred_rays += static_cast<int64_t>(sum.deferred);
  st->bvh_width = c->fast_on ? (c->wide_now ? c->wide_now : c->fs.wide) : 0;  // the tree this render searched
  if (c->trace_log && c->fast_on) {
    unsigned long long mx[3] = {0, 0, 0};
    for (int i = 0; i < n; ++i) {
      DevCounters h;
      HIPCHK(hipMemcpy(&h, c->pipes[i].ctr, sizeof h, hipMemcpyDeviceToHost));
      mx[0] = std::max(mx[0], h.stamps[5]);
      mx[1] = std::max(mx[1], h.stamps[6]);
      mx[2] += h.stamps[7];
    }
    unsigned long long ties = 0, why[4] = {0, 0, 0, 0}, lat[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < n; ++i) {
      DevCounters h;
      HIPCHK(hipMemcpy(&h, c->pipes[i].ctr, sizeof h, hipMemcpyDeviceToHost));
      ties += h.stamps[4];
      for (int k = 0; k < 4; ++k) why[k] += h.stamps[k];
      for (int k = 0; k < 12; ++k) lat[k] = (k % 2 == 0 && k < 6) ? std::max(lat[k], h.lat[k]) : lat[k] + h.lat[k];
    }
    std::fprintf(stderr,
                 "[wr bvh latency, us] membership max %.1f sum %.1f; ties max %.1f sum %.1f; walks max %.1f sum %.1f; "
                 "long many-leaf scans %llu\n",
                 lat[0] * 0.01, lat[1] * 0.01, lat[2] * 0.01, lat[3] * 0.01, lat[4] * 0.01, lat[5] * 0.01, lat[6]);
    if (lat[7] + lat[8])
      std::fprintf(stderr,
                   "[wr bvh tie split, us] collect %.1f, first leaves %.1f, second passes %llu, pair records used %llu; "
                   "scan membership %.1f\n",
                   lat[7] * 0.01, lat[8] * 0.01, lat[9], lat[11], lat[10] * 0.01);
    std::fprintf(stderr, "[wr bvh walks] many-leaf %llu, no visited hit %llu, crowd %llu, band %llu\n", why[0], why[1],
                 why[2], why[3]);
    unsigned long long ww[4] = {0, 0, 0, 0};
    for (int i = 0; i < n; ++i) {
      DevCounters h;
      HIPCHK(hipMemcpy(&h, c->pipes[i].ctr, sizeof h, hipMemcpyDeviceToHost));
      for (int k = 0; k < 4; ++k) ww[k] += h.ww[k];
    }
    std::fprintf(stderr, "[wr bvh wave walks] %llu walks, %.1f rounds and %.1f nodes per walk, %llu serial fall-backs\n",
                 ww[0], ww[0] ? double(ww[1]) / ww[0] : 0.0, ww[0] ? double(ww[2]) / ww[0] : 0.0, ww[3]);
    std::fprintf(stderr, "[wr bvh tail] max nodes/ray %llu, max tests/ray %llu, rays > 256 nodes %llu, ties resolved by visit order %llu\n",
                 mx[0], mx[1], mx[2], ties);
  }
  if (c->stamps) {
    static const char* names[6] = {"refill", "walk", "leaf-setup", "pair-tests", "decision", "write"};
    double tot = 0;
    for (int k = 0; k < 6; ++k) tot += static_cast<double>(sum.stamps[k]);
    std::fprintf(stderr, "[wr stamps]");
    for (int k = 0; k < 6; ++k) std::fprintf(stderr, " %s=%.1f%%", names[k], 100.0 * sum.stamps[k] / std::max(1.0, tot));
    std::fprintf(stderr, " (wave-cycles %.3g)\n", tot);
  }
  st->seconds += host_now() - t0_host;
  if (c->timing) {
    std::vector<std::pair<float, float>> spans;  // traversal launches, ms from t_ref
    // diagnostics: WR_TIMELINE=<file> appends every timed launch (pipeline,
    // category, start ms, end ms from the render's start), no profiler needed
    FILE* tl = nullptr;
    if (const char* e = std::getenv("WR_TIMELINE")) tl = std::fopen(e, "a");
    for (int i = 0; i < n; ++i) {
      const Pipe& p = c->pipes[i];
      float prev = 0.f;
      (void)hipEventElapsedTime(&prev, c->t_ref, p.events[0]);
      for (size_t k = 1; k < p.ev_used; ++k) {
        float at = 0.f;
        (void)hipEventElapsedTime(&at, c->t_ref, p.events[k]);
        const int cat = p.ev_cat[k];
        st->kernel_ms[cat] += at - prev;
        st->kernel_launches[cat] += 1;
        if (cat == WR_K_TRACE) spans.emplace_back(prev, at);
        if (tl) std::fprintf(tl, "%d,%d,%.4f,%.4f\n", i, cat, prev, at);
        prev = at;
      }
    }
    if (tl) std::fclose(tl);
    std::sort(spans.begin(), spans.end());
    double wall = 0.0, lo = 0.0, hi = -1.0;
    for (const auto& sp : spans) {
      if (sp.first > hi) {
        if (hi > lo) wall += hi - lo;
        lo = sp.first;
        hi = sp.second;
      } else {
        hi = std::max<double>(hi, sp.second);
      }
    }
    if (hi > lo) wall += hi - lo;
    st->trace_wall_ms += wall;
  }
  return WR_OK;
}


int check_device() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(WR_E_NODEVICE, "no HIP device visible");
  return WR_OK;
}

}  // namespace

// =============================================================== C ABI
extern "C" {

const char* wr_last_error(void) { return wr::last_error(); }
int wr_api_version(void) { return WR_API_VERSION; }

int wr_request_hw_queues(int n) {
  if (n < 1 || n > 32) return fail(WR_E_ARG, "hardware queues: 1..32");
  if (g_hw_queues_latched.load() > 0) return hw_queues_in_effect();  // HIP already read it
  if (hw_queues_in_effect() < n && setenv("GPU_MAX_HW_QUEUES", std::to_string(n).c_str(), 1) != 0)
    return fail(WR_E_ARG, "setenv GPU_MAX_HW_QUEUES failed");
  return hw_queues_in_effect();
}

int wr_scene_load(const char* path, wr_scene** out) {
  if (!path || !out) return fail(WR_E_ARG, "null argument");
  *out = nullptr;
  auto* s = new (std::nothrow) wr_scene();
  if (!s) return fail(WR_E_ARG, "out of host memory");
  std::string err;
  if (!wr::load_scene(path, s->s, err)) {
    delete s;
    return fail(WR_E_IO, err);
  }
  *out = s;
  return WR_OK;
}

int wr_scene_from_desc(const wr_scene_desc* d, wr_scene** out) {
  if (!d || !out) return fail(WR_E_ARG, "null argument");
  *out = nullptr;
  auto* s = new (std::nothrow) wr_scene();
  if (!s) return fail(WR_E_ARG, "out of host memory");
  wr::SceneArrays a{d->n_prims, d->prim_type, d->prim_data, d->prim_mat, d->n_lights, d->light_tri, d->light_le,
                    d->n_materials, d->materials, d->cam_pos, d->cam_fwd, d->cam_up, d->cam_xres, d->cam_yres,
                    d->cam_hfov};
  std::string err;
  if (!wr::scene_from_arrays(a, s->s, err)) {
    delete s;
    return fail(WR_E_ARG, err);
  }
  *out = s;
  return WR_OK;
}

int wr_scene_info_get(const wr_scene* sc, wr_scene_info* o) {
  if (!sc || !o) return fail(WR_E_ARG, "null argument");
  const wr::Scene& s = sc->s;
  std::memset(o, 0, sizeof *o);
  o->nprims = static_cast<int32_t>(s.prims.size());
  for (const auto& p : s.prims) (p.type == wr::kTri ? o->ntriangles : o->nspheres)++;
  o->nlights = static_cast<int32_t>(s.lights.size());
  o->nmaterials = static_cast<int32_t>(s.mats.size());
  o->kd_depth_max = s.dep_max;
  for (const auto& n : s.nodes) (n.axis >= 0 ? o->kd_inner : o->kd_leaves)++;
  o->kd_refs = static_cast<int64_t>(s.refs.size());
  o->kd_max_stack = s.max_stack;
  o->missing_files = s.missing_files;
  o->camera_xres = s.cam.xres;
  o->camera_yres = s.cam.yres;
  o->device_bytes = static_cast<int64_t>(s.nodes.size() * 24 + s.refs.size() * 40 + s.prims.size() * 64);
  return WR_OK;
}

int wr_scene_fingerprint(const wr_scene* sc, uint64_t* out) {
  if (!sc || !out) return fail(WR_E_ARG, "null argument");
  *out = wr::scene_fingerprint(sc->s);
  return WR_OK;
}

int wr_scene_dump(const wr_scene* sc, const char* path) {
  if (!sc || !path) return fail(WR_E_ARG, "null argument");
  std::string txt = wr::dump_scene(sc->s);
  FILE* f = std::fopen(path, "w");
  if (!f) return fail(WR_E_IO, std::string("cannot write ") + path);
  std::fwrite(txt.data(), 1, txt.size(), f);
  std::fclose(f);
  return WR_OK;
}

void wr_scene_free(wr_scene* s) { delete s; }

int wr_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int wr_create(const wr_scene* sc, int device, wr_context** out) {
  if (!sc || !out) return fail(WR_E_ARG, "null argument");
  *out = nullptr;
  latch_hw_queues();  // before the library's first HIP call: the value HIP reads
  if (int rc = check_device()) return rc;
  DeviceGuard dg;
  const wr::Scene& s = sc->s;
  if (s.prims.empty()) return fail(WR_E_SCENE, "scene has no primitives");
  for (const auto& p : s.prims)  // the reference would index materials[] out of range
    if (p.mat >= static_cast<int>(s.mats.size()))
      return fail(WR_E_SCENE, "primitive material id " + std::to_string(p.mat) + " has no <material>");
  HIPCHK(hipSetDevice(device));
  auto* c = new wr_context();
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->t_ref, ev_flags(hipEventDefault)) != hipSuccess ||
      hipEventCreateWithFlags(&c->t_null, ev_flags(hipEventDisableTiming)) != hipSuccess) {
    wr_destroy(c);
    return fail(WR_E_HIP, "hipStreamCreate failed");
  }
  // Pipeline 0 runs on the context stream: with GPU_MAX_HW_QUEUES = 4 (HIP's
  // default) a fifth stream would share a hardware queue with another and
  // serialize behind it (measured: 4 pipelines 648 Mrays/s on 5 streams, 734 on 4).
  for (Pipe& pp : c->pipes) {
    if (&pp == &c->pipes[0]) {
      pp.stream = c->stream;
      if (hipEventCreateWithFlags(&pp.done, ev_flags(hipEventDisableTiming)) != hipSuccess ||
          hipMalloc(&pp.ctr, sizeof(DevCounters)) != hipSuccess ||
          hipMalloc(&pp.sc, kGroup * sizeof(StepCounters)) != hipSuccess) {
        wr_destroy(c);
        return fail(WR_E_HIP, "pipeline stream / counters");
      }
      continue;
    }
    if (hipStreamCreateWithFlags(&pp.stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&pp.done, ev_flags(hipEventDisableTiming)) != hipSuccess ||
        hipMalloc(&pp.ctr, sizeof(DevCounters)) != hipSuccess ||
        hipMalloc(&pp.sc, kGroup * sizeof(StepCounters)) != hipSuccess) {
      wr_destroy(c);
      return fail(WR_E_HIP, "pipeline stream / counters");
    }
  }
  // one pipeline per hardware queue of this process (HIP's GPU_MAX_HW_QUEUES,
  // default 4; pipeline 0 shares the context stream), at most 16: streams that
  // share a hardware queue serialize behind each other
  c->npipes = std::max(1, std::min(kMaxPipes, latch_hw_queues()));
  if (const char* e = std::getenv("WR_PIPES")) c->npipes = std::max(1, std::min(kMaxPipes, std::atoi(e)));
  if (const char* e = std::getenv("WR_PIECE_CAP")) c->piece_cap = std::max(64, std::atoi(e));
  if (const char* e = std::getenv("WR_PIECE_MIN")) c->piece_min = std::max(1, std::atoi(e));
  if (const char* e = std::getenv("WR_TIE_WAVE_MAX")) c->tie_wave_max = std::max(0, std::atoi(e));
  if (const char* e = std::getenv("WR_SCAN_WAVES")) c->scan_waves = std::max(1, std::atoi(e));
  if (const char* e = std::getenv("WR_ISSUE_THREADS")) c->issue_threads = std::max(1, std::min(kMaxPipes, std::atoi(e)));
  if (const char* e = std::getenv("WR_DEFER")) c->defer = std::atoi(e) != 0 ? 1 : 0;
  if (const char* e = std::getenv("WR_BDPT_OVERLAP")) c->bdpt_overlap = std::atoi(e) != 0;
  if (const char* e = std::getenv("WR_RESOLVE_GRID")) c->resolve_blocks = std::max(0, std::atoi(e));  // per CU; scaled below
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) {
    // grid-stride vertex / resolve kernels: blocks per CU (knob WR_SHADE_GRID).
    // 2 = one resident round of both group members at 4 waves/SIMD; measured
    // against 8: C2 +0.9 %, C3 +1.9 %, VCM +1.3 % (16 and 32 lose 1-2 %).
    // With the path state in records (round 3) 1 does better again: C2 20 it.
    // +2.0 %, 256 it. +2.7 %, C4 +2.6 %, VCM +3 %, C3 -0.4 % (profiles/r3/shade_grid)
    int per_cu = 1;
    if (const char* e = std::getenv("WR_SHADE_GRID")) per_cu = std::max(1, std::min(64, std::atoi(e)));
    c->grid = std::max(256, prop.multiProcessorCount * per_cu);
  }

  // ---- flatten the tree + primitives into the HBM layout of wr_traverse.h
  const size_t nn = s.nodes.size(), nr = s.refs.size(), np = s.prims.size();
  std::vector<uint2> nodes(nn);
  for (size_t i = 0; i < nn; ++i) {
    const wr::KdNode& k = s.nodes[i];
    if (k.axis >= 0) {
      uint32_t bits;
      std::memcpy(&bits, &k.split, 4);
      nodes[i] = make_uint2(bits, (static_cast<uint32_t>(k.right) << 2) | static_cast<uint32_t>(k.axis));
    } else {
      nodes[i] = make_uint2(static_cast<uint32_t>(k.first), (static_cast<uint32_t>(k.count) << 2) | 3u);
    }
  }
  std::vector<uint4> nrec(nn);
  std::vector<uint2> nrec_r(nn, make_uint2(0u, 0u));
  for (size_t i = 0; i < nn; ++i) {
    const uint2 self = nodes[i];
    uint2 l = make_uint2(0u, 0u);
    if (s.nodes[i].axis >= 0) {
      l = nodes[i + 1];
      nrec_r[i] = nodes[static_cast<size_t>(s.nodes[i].right)];
    }
    nrec[i] = make_uint4(self.x, self.y, l.x, l.y);
  }
  // multi-level records (WR_NODE_LEVELS = 3 or 4): node i's subtree of
  // kRecLevels levels in heap order (entry 0 = i, entries 2h+1 / 2h+2 = the
  // children of entry h; 0 below a leaf), two entries per uint4
  std::vector<uint4> nrec3(kRecU4 * nn, make_uint4(0u, 0u, 0u, 0u));
  {
    constexpr int kEnt = (1 << kRecLevels) - 1;
    for (size_t i = 0; i < nn; ++i) {
      int64_t e[kEnt];
      e[0] = static_cast<int64_t>(i);
      for (int h = 0; 2 * h + 2 < kEnt; ++h) {
        e[2 * h + 1] = e[2 * h + 2] = -1;
        if (e[h] >= 0 && s.nodes[static_cast<size_t>(e[h])].axis >= 0) {
          e[2 * h + 1] = e[h] + 1;
          e[2 * h + 2] = s.nodes[static_cast<size_t>(e[h])].right;
        }
      }
      uint32_t* w = reinterpret_cast<uint32_t*>(&nrec3[kRecU4 * i]);
      for (int h = 0; h < kEnt; ++h) {
        const uint2 v = e[h] >= 0 ? nodes[static_cast<size_t>(e[h])] : make_uint2(0u, 0u);
        w[2 * h] = v.x;
        w[2 * h + 1] = v.y;
      }
    }
  }
  std::vector<float4> ra(nr), rb(nr);
  std::vector<float2> rcv(nr);
  for (size_t i = 0; i < nr; ++i) {
    const int pi = s.refs[i];
    const wr::Prim& p = s.prims[pi];
    if (p.type == wr::kTri) {
      // A..F exactly as Triangle::hit forms them (triangle.cpp:24-30)
      ra[i] = make_float4(p.p0.x, p.p0.y, p.p0.z, p.p0.x - p.p1.x);
      rb[i] = make_float4(p.p0.y - p.p1.y, p.p0.z - p.p1.z, p.p0.x - p.p2.x, p.p0.y - p.p2.y);
      float pb;
      std::memcpy(&pb, &pi, 4);
      rcv[i] = make_float2(p.p0.z - p.p2.z, pb);
    } else {
      ra[i] = make_float4(0, 0, 0, 0);
      rb[i] = make_float4(0, 0, 0, 0);
      int neg = -(pi + 1);
      float pb;
      std::memcpy(&pb, &neg, 4);
      rcv[i] = make_float2(0.f, pb);
    }
  }
  std::vector<int> pmat(np), ptype(np);
  std::vector<float4> ptri(np), psph(np), psb0(np);
  std::vector<float2> ptri2(np), psb1(np);
  for (size_t i = 0; i < np; ++i) {
    const wr::Prim& p = s.prims[i];
    pmat[i] = p.mat;
    ptype[i] = p.type;
    ptri[i] = make_float4(p.p0.x - p.p1.x, p.p0.y - p.p1.y, p.p0.z - p.p1.z, p.p0.x - p.p2.x);
    ptri2[i] = make_float2(p.p0.y - p.p2.y, p.p0.z - p.p2.z);
    psph[i] = make_float4(p.c.x, p.c.y, p.c.z, p.r);
    psb0[i] = make_float4(p.bl.x, p.bl.y, p.bl.z, p.br.x);
    psb1[i] = make_float2(p.br.y, p.br.z);
  }
  std::vector<DLight> lights(s.lights.size());
  for (size_t i = 0; i < lights.size(); ++i) {
    const wr::Light& l = s.lights[i];
    auto V = [](wr::F3 f) { return v3(f.x, f.y, f.z); };
    lights[i] = DLight{V(l.p0), V(l.d1), V(l.d2), V(l.fx), V(l.fy), V(l.fz), V(l.le), l.inv_area};
  }
  std::vector<DMat> mats(std::max<size_t>(1, s.mats.size()));
  for (size_t i = 0; i < s.mats.size(); ++i) {
    const wr::Material& m = s.mats[i];
    mats[i] = DMat{v3(m.diffuse.x, m.diffuse.y, m.diffuse.z), v3(m.phong.x, m.phong.y, m.phong.z),
                   v3(m.specular.x, m.specular.y, m.specular.z), m.phong_exp, m.index};
  }
  auto total = measure([&](Arena& a) {
    a.take<uint4>(nn); a.take<uint2>(nn); a.take<uint4>(kRecU4 * nn); a.take<float4>(nr); a.take<float4>(nr);
    a.take<float2>(nr);
    a.take<int>(np); a.take<int>(np); a.take<float4>(np); a.take<float2>(np); a.take<float4>(np);
    a.take<float4>(np); a.take<float2>(np); a.take<float4>(2 * np); a.take<DLight>(lights.size() + 1);
    a.take<DMat>(mats.size());
    a.take<DevCounters>(1);
  });
  if (int rc = c->scene_mem.reserve(total)) {
    delete c;
    return rc;
  }
  Arena& A = c->scene_mem;
  auto up = [&](auto* dst, const auto& v) {
    return hipMemcpy(dst, v.data(), v.size() * sizeof(v[0]), hipMemcpyHostToDevice);
  };
  DevScene& d = c->ds;
  uint4* dn = A.take<uint4>(nn);
  uint2* dnr = A.take<uint2>(nn);
  uint4* dn3 = A.take<uint4>(kRecU4 * nn);
  float4* dra = A.take<float4>(nr);
  float4* drb = A.take<float4>(nr);
  float2* drc = A.take<float2>(nr);
  int* dpm = A.take<int>(np);
  int* dpt = A.take<int>(np);
  float4* dptri = A.take<float4>(np);
  float2* dptri2 = A.take<float2>(np);
  float4* dpsph = A.take<float4>(np);
  float4* dpsb0 = A.take<float4>(np);
  float2* dpsb1 = A.take<float2>(np);
  float4* dprec = A.take<float4>(2 * np);
  std::vector<float4> prec(2 * np);
  for (size_t i = 0; i < np; ++i) {
    prec[2 * i] = ptri[i];
    float mb, tb;  // the int fields' bits (host code: no __int_as_float)
    std::memcpy(&mb, &pmat[i], 4);
    std::memcpy(&tb, &ptype[i], 4);
    prec[2 * i + 1] = make_float4(ptri2[i].x, ptri2[i].y, mb, tb);
  }
  DLight* dl = A.take<DLight>(lights.size() + 1);
  DMat* dm = A.take<DMat>(mats.size());
  c->ctr = A.take<DevCounters>(1);
  hipError_t e = hipSuccess;
  for (hipError_t x : {up(dn, nrec), up(dnr, nrec_r), up(dn3, nrec3), up(dra, ra), up(drb, rb), up(drc, rcv), up(dpm, pmat), up(dpt, ptype),
                       up(dptri, ptri), up(dptri2, ptri2), up(dpsph, psph), up(dpsb0, psb0), up(dpsb1, psb1), up(dprec, prec),
                       up(dm, mats)})
    if (x != hipSuccess) e = x;
  if (!lights.empty() && e == hipSuccess) e = up(dl, lights);
  if (e != hipSuccess) {
    wr_destroy(c);
    return fail(WR_E_HIP, std::string("scene upload: ") + hipGetErrorString(e));
  }
  d.nrec = dn;
  d.nrec_r = dnr;
  d.nrec3 = dn3;
  d.ref_a = dra;
  d.ref_b = drb;
  d.ref_c = drc;
  d.prim_mat = dpm;
  d.prim_type = dpt;
  d.prim_tri = dptri;
  d.prim_tri2 = dptri2;
  d.prim_sph = dpsph;
  d.prim_rec = dprec;
  d.prim_sbox0 = dpsb0;
  d.prim_sbox1 = dpsb1;
  d.root_l = v3(s.root_l.x, s.root_l.y, s.root_l.z);
  d.root_r = v3(s.root_r.x, s.root_r.y, s.root_r.z);
  d.max_stack = std::max(1, s.max_stack);
  c->sph_r = s.sph_r;
  d.nlights = static_cast<int>(s.lights.size());
  d.lights = dl;
  d.mats = dm;
  d.cam.pos = v3(s.cam.pos.x, s.cam.pos.y, s.cam.pos.z);
  d.cam.fwd = v3(s.cam.fwd.x, s.cam.fwd.y, s.cam.fwd.z);
  d.cam.xres = s.cam.xres;
  d.cam.yres = s.cam.yres;
  d.cam.plane_dist = s.cam.plane_dist;
  std::memcpy(d.cam.w2r, s.cam.w2r, sizeof d.cam.w2r);
  std::memcpy(d.cam.r2w, s.cam.r2w, sizeof d.cam.r2w);
  c->scene_bytes = static_cast<int64_t>(A.used);
  for (const auto& p : s.prims) c->spheres |= p.type != wr::kTri;
  if (const char* e = std::getenv("WR_TRACE_STAMPS")) c->stamps = std::atoi(e) != 0 && !c->spheres;
  if (const char* e = std::getenv("WR_TRACE_LOG")) c->trace_log = std::atoi(e) != 0;
  if (const char* e = std::getenv("WR_TRACE_DENSE")) c->api_dense = std::atoi(e) != 0;
  if (const char* e = std::getenv("WR_TRACE_NO_CUT")) c->no_cut = std::atoi(e) != 0;
  if (const char* e = std::getenv("WR_VCM_CELL")) c->vcm_cell = std::min(8.f, std::max(0.25f, (float)std::atof(e)));
  {
    // persistent traversal grid: the one-wave workgroups that fit at once (LDS stack
    // and registers); more would only queue behind the first wave of blocks
    // 16-bit stack nodes and 16-bit pair offsets (64 lanes x kLeavesPerRound
    // leaves x max leaf size < 65536)
    int max_leaf = 0;
    for (const auto& k : s.nodes)
      if (k.axis < 0) max_leaf = std::max(max_leaf, k.count);
    c->narrow = nn <= 65536 && static_cast<int64_t>(max_leaf) * 64 * kLeavesPerRound < 65536;
    // test knob: WR_TRACE_WIDE=1 runs the 32-bit-stack variant on any tree
    if (const char* e = std::getenv("WR_TRACE_WIDE")) c->narrow = c->narrow && std::atoi(e) == 0;
    auto resident = [&](int mode) {
      const size_t lds = trace_lds_bytes(d.max_stack, c->narrow, mode == TRACE_DENSE);
      int per_cu = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, trace_kernel(false, c->spheres, c->narrow, false, mode),
                                                       kTraceBlock, lds) != hipSuccess ||
          per_cu <= 0)
        per_cu = 8;
      // diagnostic: WR_TRACE_WAVES_PER_CU caps the resident traversal waves
      // (leaving room for the other pipelines' shading kernels)
      if (const char* e = std::getenv("WR_TRACE_WAVES_PER_CU")) per_cu = std::max(1, std::min(per_cu, std::atoi(e)));
      return per_cu;
    };
    c->cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    c->resolve_blocks *= c->cus;  // WR_RESOLVE_GRID was blocks per CU
    c->trace_blocks = c->cus * resident(TRACE_PLAIN);
    c->trace_blocks_dense = c->cus * resident(TRACE_DENSE);
  }
  // ---- verified-BVH traversal data (wr_bvh.h): BVH nodes, triangle records
  // in leaf order, and the KD root paths of every primitive's leaves
  {
    // the search tree's width: 4-wide for scenes whose binary tree outgrows
    // the L2 (its nodes then come from the Infinity Cache / HBM, and one
    // 128-byte node holds two of the binary tree's levels: C4 +5-8 %, while
    // L2-resident scenes lose 1-4 %: DESIGN.md 4b); WR_BVH_WIDE=2|4 forces
    int wide = WR_BVH_WIDE;
    if (wide == 2) {
      size_t tris = 0;
      for (const wr::Prim& p : s.prims) tris += p.type == wr::kTri ? 1 : 0;
      if (tris >= wrf::kWide4MinTris) wide = 4;
    }
    if (const char* e = std::getenv("WR_BVH_WIDE")) {
      const int w = std::atoi(e);
      if (w == 2 || w == 4 || (w == 8 && WR_BVH_WIDE == 8)) wide = w;
    }
    // the 8-wide search is instantiated for triangle leaves only: a scene with
    // spheres searches the 4-wide tree, whose kernels run the sphere test
    if (wide == 8)
      for (const wr::Prim& p : s.prims)
        if (p.type != wr::kTri) {
          wide = 4;
          break;
        }
    wrf::FastHost fh;
    wrf::build_fast(s, fh, wide, wide == 2);
    if (fh.ok) {
      const size_t fbn = fh.nodes.size(), ftr = fh.tris.size(), fpo = fh.prim_leaf_off.size(),
                   fpl = std::max<size_t>(1, fh.prim_leaf.size()), fpa = fh.path.size() / 2;
      const size_t fnp = fh.node_path.size();
      const size_t fbytes = measure([&](Arena& a) {
        a.take<wrf::BNode>(fbn); a.take<wrf::TriRec>(ftr); a.take<int>(fpo); a.take<int>(fpl); a.take<int>(fpl);
        a.take<uint2>(fpa); a.take<int>(fnp); a.take<float4>(2 * fnp); a.take<wrf::PrimRec>(fh.prim_rec.size());
        a.take<wrf::BNode4S>(fh.nodes4.size());
        a.take<wrf::BNode8>(fh.nodes8.size());
      });
      if (int rc = c->fast_mem.reserve(fbytes)) {
        wr_destroy(c);
        return rc;
      }
      Arena& F = c->fast_mem;
      auto* dno = F.take<wrf::BNode>(fbn);
      auto* dtr = F.take<wrf::TriRec>(ftr);
      int* dpo = F.take<int>(fpo);
      int* dpl = F.take<int>(fpl);
      int* dpp = F.take<int>(fpl);
      uint2* dpa = F.take<uint2>(fpa);
      int* dnp = F.take<int>(fnp);
      float4* dnc = F.take<float4>(2 * fnp);
      auto* dpr = F.take<wrf::PrimRec>(fh.prim_rec.size());
      auto* dn4 = F.take<wrf::BNode4S>(fh.nodes4.size());
      auto* dn8 = F.take<wrf::BNode8>(fh.nodes8.size());
      hipError_t fe = hipSuccess;
      for (hipError_t x : {hipMemcpy(dno, fh.nodes.data(), fbn * sizeof(wrf::BNode), hipMemcpyHostToDevice),
                           hipMemcpy(dtr, fh.tris.data(), ftr * sizeof(wrf::TriRec), hipMemcpyHostToDevice),
                           hipMemcpy(dpo, fh.prim_leaf_off.data(), fpo * sizeof(int), hipMemcpyHostToDevice),
                           hipMemcpy(dpl, fh.prim_leaf.data(), fh.prim_leaf.size() * sizeof(int), hipMemcpyHostToDevice),
                           hipMemcpy(dpp, fh.prim_leaf_pos.data(), fh.prim_leaf_pos.size() * sizeof(int),
                                     hipMemcpyHostToDevice),
                           hipMemcpy(dpa, fh.path.data(), fpa * sizeof(uint2), hipMemcpyHostToDevice),
                           hipMemcpy(dnp, fh.node_path.data(), fnp * sizeof(int), hipMemcpyHostToDevice),
                           hipMemcpy(dnc, fh.node_cell.data(), 8 * fnp * sizeof(float), hipMemcpyHostToDevice),
                           hipMemcpy(dpr, fh.prim_rec.data(), fh.prim_rec.size() * sizeof(wrf::PrimRec),
                                     hipMemcpyHostToDevice),
                           hipMemcpy(dn4, fh.nodes4.data(), fh.nodes4.size() * sizeof(wrf::BNode4S),
                                     hipMemcpyHostToDevice),
                           hipMemcpy(dn8, fh.nodes8.data(), fh.nodes8.size() * sizeof(wrf::BNode8),
                                     hipMemcpyHostToDevice)})
        if (x != hipSuccess) fe = x;
      if (fe != hipSuccess) {
        wr_destroy(c);
        return fail(WR_E_HIP, std::string("BVH upload: ") + hipGetErrorString(fe));
      }
      FastScene& fs = c->fs;
      fs.nodes = reinterpret_cast<const float4*>(dno);
      fs.tris = reinterpret_cast<const float4*>(dtr);
      fs.prim_leaf_off = dpo;
      fs.prim_leaf = dpl;
      fs.prim_leaf_pos = dpp;
      fs.path = dpa;
      fs.node_path = dnp;
      fs.node_cell = dnc;
      fs.prim_rec = reinterpret_cast<const float4*>(dpr);
      fs.nodes4 = reinterpret_cast<const float4*>(dn4);
      fs.nodes8 = reinterpret_cast<const float4*>(dn8);
      float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
      for (int k = 0; k < 3; ++k) {
        lo[k] = std::min(fh.nodes[0].b[k], fh.nodes[0].b[6 + k]);
        hi[k] = std::max(fh.nodes[0].b[3 + k], fh.nodes[0].b[9 + k]);
      }
      fs.lo = v3(lo[0], lo[1], lo[2]);
      fs.hi = v3(hi[0], hi[1], hi[2]);
      fs.sph = fh.spheres > 0 ? 1 : 0;
      fs.org_lo = v3(fh.org_lo[0], fh.org_lo[1], fh.org_lo[2]);
      fs.org_hi = v3(fh.org_hi[0], fh.org_hi[1], fh.org_hi[2]);
      // the search's stack holds BVH entries only; the hard rays' kernel walks
      // both trees
      fs.wide = wide;
      fs.sdepth = wide == 8 ? 7 * fh.depth8 + 1 : wide == 4 ? 3 * fh.depth4 + 1 : fh.depth + 1;
      if (wide == 2 && !fh.nodes4.empty()) {
        c->sdepth4 = 3 * fh.depth4 + 1;
        c->fs4_ok = true;
      }
      if (const char* e = std::getenv("WR_BVH_WIDE_LAT")) c->lat_wide = std::atoi(e) != 0;
      fs.depth = std::max(fh.depth + 1, d.max_stack + 1);
      // kd_walk_wave: node index and depth share a word, the leaf key and the
      // position in the leaf 64 bits (the key's lowest bit is 64 - dep_max, so
      // every leaf must hold fewer than 2^(64 - dep_max) references)
      size_t kd_max_leaf = 0;
      for (const auto& k : s.nodes)
        if (k.axis < 0) kd_max_leaf = std::max(kd_max_leaf, static_cast<size_t>(k.count));
      fs.walk_wave = s.nodes.size() < (size_t(1) << 26) && s.dep_max <= 43 &&
                             kd_max_leaf < (size_t(1) << (64 - std::max(s.dep_max, 0)))
                         ? 1
                         : 0;
      if (const char* e = std::getenv("WR_WALK_WAVE")) fs.walk_wave = fs.walk_wave && std::atoi(e) != 0;
      // near-ties and the search's pair record (kPairWindow): 2 = the pair list
      // (one per lane), 1 = the record in the tie list only, 0 = neither
      fs.pair = 2;
      if (const char* e = std::getenv("WR_PAIR_RECORD")) fs.pair = std::max(0, std::min(2, std::atoi(e)));
      c->fast_ok = true;
      if (const char* e = std::getenv("WR_RESOLVE_LIST")) c->resolve_list = std::atoi(e) != 0;
      int per_cu = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, trace_fast_kernel<false, false>(wide, fs.sph, c->resolve_list), kTraceBlock,
                                                       search_lds_bytes(fs.sdepth, wide) + (c->resolve_list ? kRlistLds : 0)) != hipSuccess ||
          per_cu <= 0)
        per_cu = 8;
      // diagnostic: WR_FAST_WAVES_PER_CU caps the search's resident waves
      if (const char* e = std::getenv("WR_FAST_WAVES_PER_CU")) per_cu = std::max(1, std::min(per_cu, std::atoi(e)));
      c->fast_blocks = c->cus * per_cu;
      // the verified BVH is the default traversal (same answers as the KD
      // walk); WR_TRACE_BVH=0 selects the walk
      c->fast_on = true;
      if (const char* e = std::getenv("WR_TRACE_BVH")) c->fast_on = std::atoi(e) != 0;
      if (const char* e = std::getenv("WR_BVH_DIAG")) fs.diag = std::atoi(e);
      if (const char* e = std::getenv("WR_BVH_VERIFY")) c->verify = std::atoi(e) != 0;
      if (c->trace_log)
        std::fprintf(stderr, "[wr bvh] nodes %zu tris %zu depth %d lds %zu B/wave, %d waves/CU -> grid %d; kd grid %d\n",
                     fbn, ftr, fs.sdepth, search_lds_bytes(fs.sdepth, wide), per_cu, c->fast_blocks, c->trace_blocks);
    }
  }
  *out = c;
  return WR_OK;
}

int wr_set_trace_mode(wr_context* c, int mode) {
  if (!c || (mode != WR_TRACE_REFERENCE && mode != WR_TRACE_BVH)) return fail(WR_E_ARG, "bad trace mode");
  if (mode == WR_TRACE_BVH && !c->fast_ok) return fail(WR_E_SCENE, "the scene has no verified BVH (empty, or too large)");
  c->fast_on = mode == WR_TRACE_BVH;
  for (wr_context* d : c->subs) d->fast_on = c->fast_on;
  return WR_OK;
}

int wr_set_pipelines(wr_context* c, int n) {
  if (!c || n < 1 || n > kMaxPipes) return fail(WR_E_ARG, "pipelines must be in 1.." + std::to_string(kMaxPipes));
  c->npipes = n;
  for (wr_context* d : c->subs) d->npipes = n;
  return WR_OK;
}

void wr_destroy(wr_context* c) {
  if (!c) return;
  DeviceGuard dg;
  for (wr_context* d : c->subs) wr_destroy(d);
  c->subs.clear();
  for (ncclComm_t m : c->dev_comms) (void)rccl().destroy(m);
  c->dev_comms.clear();
  if (c->comm) (void)rccl().destroy(c->comm);
  c->comm = nullptr;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (Pipe& p : c->pipes) {
    if (p.stream) (void)hipStreamSynchronize(p.stream);
    for (hipEvent_t e : p.events) (void)hipEventDestroy(e);
    if (p.done) (void)hipEventDestroy(p.done);
    p.late_mem.release();
    if (p.ctr) (void)hipFree(p.ctr);
    if (p.sc) (void)hipFree(p.sc);
    p.work.release();
    if (p.stream && p.stream != c->stream) (void)hipStreamDestroy(p.stream);
  }
  if (c->t_ref) (void)hipEventDestroy(c->t_ref);
  if (c->t_null) (void)hipEventDestroy(c->t_null);
  if (c->film_tmp) (void)hipFree(c->film_tmp);
  if (c->film_bak) (void)hipFree(c->film_bak);
  if (c->host_ctr) (void)hipHostFree(c->host_ctr);
  if (c->api_tmp) (void)hipFree(c->api_tmp);
  if (c->api_t2) (void)hipFree(c->api_t2);
  if (c->api_spill) (void)hipFree(c->api_spill);
  for (Pipe& p : c->pipes) {
    if (p.t2buf) (void)hipFree(p.t2buf);
    if (p.spill) (void)hipFree(p.spill);
  }
  if (c->red_buf) (void)hipFree(c->red_buf);
  if (c->stage_buf) (void)hipFree(c->stage_buf);
  c->fast_mem.release();
  c->scene_mem.release();
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

// the context's API scratch block, at least `bytes` (the stream is idle
// between API calls: every call ends with a stream synchronize)
static int api_scratch(wr_context* c, size_t bytes) {
  if (c->api_tmp_n >= bytes) return WR_OK;
  if (c->api_tmp) (void)hipFree(c->api_tmp);
  c->api_tmp = nullptr;
  c->api_tmp_n = 0;
  HIPCHK(hipMalloc(&c->api_tmp, bytes));
  c->api_tmp_n = bytes;
  return WR_OK;
}

static int trace_api(wr_context* c, const wr_ray* rays, const float* targets, int64_t n64, wr_hit* hits,
                     uint8_t* occ) {
  if (!c || (!rays && n64) || n64 < 0) return fail(WR_E_ARG, "bad argument");
  if (n64 == 0) return WR_OK;
  if (n64 > (1 << 28)) return fail(WR_E_ARG, "at most 2^28 rays per call");
  const int n = static_cast<int>(n64);
  HIPCHK(hipSetDevice(c->device));
  // one scratch block: rays, SoA queue, results, counters (kept on the
  // context: no allocation per call, nothing to free on an error return)
  const size_t nb = size_t(n);
  const size_t bytes = nb * (sizeof(wr_ray) + 4 * 14 + sizeof(wr_hit) + 1) + 16 * 256;
  if (int rc = api_scratch(c, bytes)) return rc;
  char* q = c->api_tmp;
  auto take = [&](size_t sz) { char* r = q; q += (sz + 255) & ~size_t(255); return r; };
  wr_ray* dr = reinterpret_cast<wr_ray*>(take(nb * sizeof(wr_ray)));
  float* o3 = reinterpret_cast<float*>(take(nb * 12));
  float* d3 = reinterpret_cast<float*>(take(nb * 12));
  float* tmn = reinterpret_cast<float*>(take(nb * 4));
  float* tmx = reinterpret_cast<float*>(take(nb * 4));
  float* tt = reinterpret_cast<float*>(take(nb * 4));
  int* pr = reinterpret_cast<int*>(take(nb * 4));
  float* dtg = reinterpret_cast<float*>(take(nb * 12));
  float* dcut = reinterpret_cast<float*>(take(nb * 4));
  wr_hit* dh = reinterpret_cast<wr_hit*>(take(nb * sizeof(wr_hit)));
  uint8_t* dox = reinterpret_cast<uint8_t*>(take(nb));
  int* cnt = reinterpret_cast<int*>(take(sizeof(int)));
  HIPCHK(hipMemcpyAsync(dr, rays, nb * sizeof(wr_ray), hipMemcpyHostToDevice, c->stream));
  if (occ) HIPCHK(hipMemcpyAsync(dtg, targets, nb * 12, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(cnt, &n, sizeof(int), hipMemcpyHostToDevice, c->stream));
  const int g = std::max(1, std::min(c->grid, (n + 255) / 256));
  hipLaunchKernelGGL(k_api_prep, dim3(g), dim3(256), 0, c->stream, dr, n, occ ? 1 : 0, o3, d3, tmn, tmx, dtg, dcut);
  c->timing = false;
  Timer tm(c, nullptr);
  HIPCHK(hipMemsetAsync(c->ctr, 0, sizeof(DevCounters), c->stream));
  if (c->fast_on && c->api_t2_cap < nb) {
    if (c->api_t2) (void)hipFree(c->api_t2);
    c->api_t2 = nullptr;
    c->api_t2_cap = 0;
    HIPCHK(hipMalloc(&c->api_t2, 5 * nb * sizeof(float)));  // as ensure_t2
    c->api_t2_cap = nb;
  }
  QueueList ql;
  ql.add(rq(o3, d3, n, cnt, tt, pr, tmn, tmx, occ ? dcut : nullptr), n);
  if (c->fast_on && !c->api_spill && max_spill_entries(c) > 0)
    HIPCHK(hipMalloc(&c->api_spill, max_spill_entries(c) * size_t(c->fast_blocks) * 64 * sizeof(int2)));
  const TraceSlot ts{&c->ctr->fetch, c->api_t2, c->api_t2_cap, &c->ctr->hard[0], c->api_spill, &c->ctr->rlist};
  trace_launch(c, c->stream, c->ctr, ts, tm, false, ql.Q, ql.max_rays,
               c->api_dense ? TRACE_DENSE : (occ != nullptr ? TRACE_CUT : TRACE_PLAIN), true);
  hipLaunchKernelGGL(k_api_finish, dim3(g), dim3(256), 0, c->stream, c->ds, o3, d3, tt, pr, dtg, n, dh,
                     occ ? dox : nullptr);
  HIPCHK(hipGetLastError());
  if (occ) HIPCHK(hipMemcpyAsync(occ, dox, nb, hipMemcpyDeviceToHost, c->stream));
  else HIPCHK(hipMemcpyAsync(hits, dh, nb * sizeof(wr_hit), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return WR_OK;
}

extern "C++" {
// ---- several devices: run fn(device context, index) on every device of c at
// once (devices[0] on the calling thread), first error wins
template <class Fn>
static int for_each_device(wr_context* c, Fn fn) {
  std::vector<wr_context*> dev{c};
  dev.insert(dev.end(), c->subs.begin(), c->subs.end());
  const int n = static_cast<int>(dev.size());
  std::vector<int> rc(n, WR_OK);
  std::vector<std::string> msg(n);
  std::vector<std::thread> th;
  for (int k = 1; k < n; ++k)
    th.emplace_back([&, k] {
      rc[k] = fn(dev[k], k);
      if (rc[k] != WR_OK) msg[k] = wr::last_error();
    });
  rc[0] = fn(dev[0], 0);
  if (rc[0] != WR_OK) msg[0] = wr::last_error();
  for (auto& t : th) t.join();
  for (int k = 0; k < n; ++k)
    if (rc[k] != WR_OK) return fail(rc[k], "device " + std::to_string(dev[k]->device) + ": " + msg[k]);
  return WR_OK;
}

}  // extern "C++"

static int trace_multi(wr_context* c, const wr_ray* rays, const float* targets, int64_t n, wr_hit* hits,
                       uint8_t* occ) {
  if (c->subs.empty() || n < 1024) return trace_api(c, rays, targets, n, hits, occ);
  const int64_t nd = 1 + static_cast<int64_t>(c->subs.size());
  return for_each_device(c, [&](wr_context* d, int k) {  // contiguous ray ranges
    const int64_t lo = n * k / nd, hi = n * (k + 1) / nd;
    return trace_api(d, rays + lo, targets ? targets + 3 * lo : nullptr, hi - lo, hits ? hits + lo : nullptr,
                     occ ? occ + lo : nullptr);
  });
}

int wr_trace_closest(wr_context* c, const wr_ray* rays, int64_t n, wr_hit* hits) {
  if (!hits && n) return fail(WR_E_ARG, "null hits");
  if (!c || (!rays && n) || n < 0) return fail(WR_E_ARG, "bad argument");
  DeviceGuard dg;
  return trace_multi(c, rays, nullptr, n, hits, nullptr);
}

int wr_occluded(wr_context* c, const wr_ray* rays, const float* targets, int64_t n, uint8_t* occluded) {
  if ((!targets || !occluded) && n) return fail(WR_E_ARG, "null targets / output");
  if (!c || (!rays && n) || n < 0) return fail(WR_E_ARG, "bad argument");
  DeviceGuard dg;
  return trace_multi(c, rays, targets, n, nullptr, occluded);
}

static int film_target(wr_context* c, float* film, int film_on_device, size_t nfloat, float** dev) {
  if (film_on_device) {
    *dev = film;
    return WR_OK;
  }
  if (c->film_tmp_n < nfloat) {
    if (c->film_tmp) (void)hipFree(c->film_tmp);
    c->film_tmp = nullptr;
    c->film_tmp_n = 0;
    HIPCHK(hipMalloc(&c->film_tmp, nfloat * sizeof(float)));
    c->film_tmp_n = nfloat;
  }
  HIPCHK(hipMemsetAsync(c->film_tmp, 0, nfloat * sizeof(float), c->stream));
  *dev = c->film_tmp;
  return WR_OK;
}

static int film_return(wr_context* c, float* film, int film_on_device, size_t nfloat) {
  if (film_on_device) return WR_OK;
  std::vector<float> tmp(nfloat);
  HIPCHK(hipMemcpyAsync(tmp.data(), c->film_tmp, nfloat * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  for (size_t i = 0; i < nfloat; ++i) film[i] = film[i] + tmp[i];
  return WR_OK;
}

// Issues one round of launches: step by step across the pipelines [0, np),
// on c->issue_threads host threads (pipeline i on thread i % T, each thread
// stepping through its own pipelines; their streams are independent).
// fn(pipeline, step) issues one step of one pipeline.
extern "C++" {
template <class Fn>
static int issue_round(wr_context* c, int live, int nsteps, Fn&& fn, int np) {
  const int T = std::min(c->issue_threads, std::max(1, live));
  auto run = [&](int t) -> int {
    for (int step = 0; step < nsteps; ++step)
      for (int pi = t; pi < np; pi += T)
        if (int rc = fn(pi, step)) return rc;
    return WR_OK;
  };
  if (T <= 1) return run(0);
  std::vector<int> rcs(T, WR_OK);
  std::vector<std::string> msg(T);  // wr_last_error is thread-local: carry it over
  std::vector<std::thread> th;
  th.reserve(T - 1);
  for (int t = 1; t < T; ++t)
    th.emplace_back([&, t] {
      const hipError_t e = hipSetDevice(c->device);
      if (e != hipSuccess) {
        rcs[t] = WR_E_HIP;
        msg[t] = std::string("issue thread hipSetDevice: ") + hipGetErrorString(e);
        return;
      }
      rcs[t] = run(t);
      if (rcs[t] != WR_OK) msg[t] = wr::last_error();
    });
  rcs[0] = run(0);
  if (rcs[0] != WR_OK) msg[0] = wr::last_error();
  for (auto& x : th) x.join();
  for (int t = 0; t < T; ++t)
    if (rcs[t] != WR_OK) return fail(rcs[t], msg[t]);
  return WR_OK;
}
}  // extern "C++"

// Deferred hard rays on np pipelines: env WR_DEFER=1 only.
static bool defer_enabled(const wr_context* c, int np) {
  (void)np;
  // off by default: measured slower (deferred hard rays); not
  // built for trees with spheres (no LATE search variant with spheres)
  return c->defer > 0 && !c->fs.sph;
}

// late-list records per group member and step parity (ties + scans) for pieces of `cap` paths
static int late_records(int cap) { return 2 * std::max(4096, cap / 32); }

static int check_bdpt(const wr_context* c, const wr_bdpt_params* prm, const float* film) {
  if (!c || !prm || !film) return fail(WR_E_ARG, "null argument");
  if (prm->width <= 0 || prm->height <= 0 || prm->iterations < 0) return fail(WR_E_ARG, "bad film size");
  if (static_cast<int64_t>(prm->width) * prm->height >= (1 << 30) / (kVMax + 2))
    return fail(WR_E_ARG, "film too large for one context");
  if (prm->max_path_length > kVMax + 1)
    return fail(WR_E_ARG, "max_path_length > 10 is not supported (light-vertex store sized for the reference's 10)");
  if (c->ds.nlights <= 0) return fail(WR_E_SCENE, "BDPT needs at least one area light");
  return WR_OK;
}
// camera-order unit of a BDPT piece: whole 8-row bands when the film is tiled
// (camera_gen_one), else 64 paths
static int bdpt_unit(const wr_bdpt_params* prm) {
  return ((prm->width % 8) == 0 && (prm->height % 8) == 0) ? 8 * prm->width : 64;
}
// One device: the flattened path-iterations [f_lo, f_hi) of the render
// (iteration iter_begin + f / P, path f % P; whole units).
static int render_bdpt_one(wr_context* c, const wr_bdpt_params* prm, int64_t f_lo, int64_t f_hi, float* film,
                           int film_on_device, wr_stats* st) {
  HIPCHK(hipSetDevice(c->device));
  const double t0 = host_now();
  const int P = prm->width * prm->height;
  // pieces of (iteration, path range) per pipeline, buffers sized for the largest
  const int unit = bdpt_unit(prm);
  const int cap = piece_capacity(c, P, unit);
  const int fit = pipelines_that_fit(c, 1, cap, kGroup, c->npipes);
  if (fit < 1) return WR_E_HIP;  // message set by the allocation
  const PiecePlan plan = plan_pieces(f_lo, f_hi, P, unit, cap, fit, c->piece_min);
  const int np = plan.pipes();
  // a render too short to fill the pipelines that fit, each holding one
  // group, is latency-bound: its searches take the 4-wide tree when the scene
  // has one beside the binary (DESIGN.md 4b, C2 at 1 iteration +2.3 %);
  // renders that fill the pipelines keep the binary (C2 at 20 iterations,
  // 16 pipelines of one group each: 4-wide -3 %)
  size_t most_groups = 0;
  for (const auto& pp : plan.per_pipe) most_groups = std::max(most_groups, pp.size());
  struct WideNow {
    wr_context* c;
    ~WideNow() {
      c->wide_now = 0;
      c->lat_now = false;
    }
  } wide_guard{c};
  c->lat_now = np < fit && most_groups <= 1;
  c->wide_now = (c->lat_now && c->fs4_ok && c->lat_wide) ? 4 : 0;
  // the buffer sets, queues and shadow-queue bounds below are laid out for `cap`
  // paths: a larger piece would write past them
  for (const auto& pp : plan.per_pipe)
    for (const auto& g : pp)
      for (const Piece& pc : g)
        if (pc.n > cap || pc.n <= 0)
          return fail(WR_E_ARG, "piece plan: a piece of " + std::to_string(pc.n) + " paths exceeds the buffer capacity " + std::to_string(cap));
  {  // WR_TRACE_BVH t2 scratch: a launch takes <= kGroup x (shadow / aux + extension) queues.
     // Laid out on every pipeline that fits, as the work buffers are: a short
     // render (a warm-up) on few of them leaves nothing to allocate to a long one
    const size_t cap_sq = size_t(c->pipes[0].bb[0].cap_sq);
    // (+ the camera pass's extension queue: the overlapped schedule traces both passes' at once)
    const size_t per = kGroup * (std::max(cap_sq, size_t(cap)) + 2 * size_t(cap));
    for (int i = 0; i < fit; ++i)
      if (int rc = ensure_t2(c, c->pipes[i], per)) return rc;
  }
  // Deferred hard rays: in BVH mode the extension rays a step's resolve cannot
  // settle (near-ties, membership scans: 0.1-0.5 % of them) go to a late list
  // instead of the step's k_fast_hard, so the step's vertex launch follows its
  // resolve without waiting for them.  The next step's search launch settles
  // them in extra blocks beside its search (late_hard), and its vertex launch
  // shades their paths in extra blocks, into the same queues as its own
  // vertices: a deferred path is one step behind, and the hard rays' latency
  // hides under the next search instead of lengthening the chain.  A path is
  // deferred once per pass, and each pass gets one step more (the light pass a
  // bounce step, the camera pass extension rays at its last step).
  // The overlapped schedule (wr_bdpt.h; WR_BDPT_OVERLAP=0: the sequential one,
  // which the deferred hard rays need)
  const bool overlap = c->bdpt_overlap && kMaxQueues >= 2 * kGroup && !(c->fast_on && !c->stamps && defer_enabled(c, np));
  const bool defer = !overlap && c->fast_on && !c->stamps && defer_enabled(c, np);
  if (defer)
    for (int i = 0; i < fit; ++i)
      if (int rc = ensure_late(c->pipes[i], cap, late_records(cap))) return rc;
  float* dfilm = nullptr;
  const size_t nf = size_t(P) * 3;
  if (int rc = film_target(c, film, film_on_device, nf, &dfilm)) return rc;
  // vertex pools and shadow queues sized by use (BdptBuf): a render that fills
  // one is redone from the film as it was before it.  A caller's device film is
  // copied first (after the caller's work on the null stream, before any
  // pipeline starts: begin_render orders them after the context stream); a
  // host film's device copy starts at zero
  const bool pooled = c->pipes[0].bb[0].vidx != nullptr;
  if (pooled && film_on_device) {
    if (c->film_bak_n < nf) {
      if (c->film_bak) (void)hipFree(c->film_bak);
      c->film_bak = nullptr;
      c->film_bak_n = 0;
      HIPCHK(hipMalloc(&c->film_bak, nf * sizeof(float)));
      c->film_bak_n = nf;
    }
    (void)hipEventRecord(c->t_null, nullptr);
    (void)hipStreamWaitEvent(c->stream, c->t_null, 0);
    HIPCHK(hipMemcpyAsync(c->film_bak, dfilm, nf * sizeof(float), hipMemcpyDeviceToDevice, c->stream));
  }
  const wr_stats st0 = st ? *st : wr_stats{};
  BdptArgs A0;
  A0.S = c->ds;
  A0.film = dfilm;
  A0.W = prm->width;
  A0.H = prm->height;
  A0.P = P;
  A0.seed = prm->seed;
  A0.ctl = prm->control_length;
  A0.maxlen = prm->max_path_length > 0 ? prm->max_path_length : 10;
  A0.faithful = prm->faithful;
  A0.overlap = overlap ? 1 : 0;
  const int maxlen = A0.maxlen;
  const bool count = prm->count_work != 0;
  // One group of pieces on one pipeline, issued step by step: step 0 clears
  // the counters and starts the light subpaths, steps 1 .. maxlen-1 are the
  // light bounces, step maxlen starts the camera subpaths, and steps
  // maxlen+1 .. 2 maxlen+1 are the camera bounces.
  struct GroupIssue {
    Pipe* pp = nullptr;
    BdptGroup GA;
    int gn = 0, nmax = 0;
    bool late[kSlots] = {};  // late work issued at step slot
  };
  // steps: light gen, light bounces b = 0 .. lb_n - 1, camera gen, camera bounces b = 0 .. maxlen;
  // overlapped: both gens, then bounces b = 0 .. maxlen of both passes together
  const int lb_n = maxlen - 1 + (defer ? 1 : 0);
  const int nsteps = overlap ? maxlen + 2 : lb_n + maxlen + 3;
  // The overlapped schedule: step 0 starts both subpaths of every path; step
  // b + 1 traces, per group member, the shadow / aux rays queued by the
  // vertices of bounce b - 1 (sq slot kCamSlot + b: light splats and
  // connections, camera DI rays and connections) and the extension queue of
  // bounce b: the light pass's rays (count ext[b]; b <= maxlen - 2) followed
  // by the camera pass's (count ext[kCamSlot + b]; b < maxlen) -- one queue,
  // so that a launch takes at most 2 x kGroup queues (more queues cost the
  // traversal kernels registers: WR_MAX_QUEUES 6 took k_trace_fast from 79 to
  // 95 VGPRs, 6 to 5 waves per SIMD).  Then it shades the light vertices of
  // bounce b and after them (same stream) resolves the step's shadow / aux
  // rays and shades its camera vertices, which append their extension rays
  // behind the light pass's final count.
  auto issue_overlap = [&](GroupIssue& G, int step) -> int {
    Pipe& pp = *G.pp;
    const hipStream_t sm = pp.stream;
    Timer tm(c, &pp);
    const int gn = G.gn;
    const BdptArgs* A = G.GA.a;
    const int g = shade_grid(c, G.nmax);
    if (step == 0) {
      HIPCHK(hipMemsetAsync(pp.sc, 0, gn * sizeof(StepCounters), sm));
      hipLaunchKernelGGL(k_light_gen, dim3(g, gn), dim3(kShadeBlock), 0, sm, G.GA);
      hipLaunchKernelGGL(k_camera_gen, dim3(g, gn), dim3(kShadeBlock), 0, sm, G.GA);
      tm.mark(WR_K_GEN);
      return WR_OK;
    }
    const int b = step - 1, slot = kCamSlot + b;
    const bool light = b <= maxlen - 2, more = b < maxlen;
    QueueList ql;
    for (int m = 0; m < gn; ++m) {
      const BdptBuf& B = pp.bb[m];
      const BdptBuf::Sq& Q = B.sq[slot & 1];
      ql.add(rq(Q.o, Q.d, B.cap_sq, &pp.sc[m].sq[slot], Q.t, Q.prim, nullptr, nullptr, Q.cut),
             std::min(A[m].n * (kVMax + 2), B.cap_sq));
      if (light || more)
        ql.add(rq(B.q_o[b & 1], B.q_d[b & 1], B.qs, &pp.sc[m].ext[b], B.q_t[b & 1], B.q_prim[b & 1], nullptr, nullptr,
                  nullptr, nullptr, nullptr, 0, &pp.sc[m].ext[slot]),
               2 * A[m].n);
    }
    trace_launch(c, sm, pp.ctr, tslot(pp, slot), tm, count, ql.Q, ql.max_rays, WR_BDPT_TRACE_MODE, false, nullptr,
                 gn);
    LateArgs L{};
    if (light) hipLaunchKernelGGL(k_light_shade, dim3(g, gn), dim3(kShadeBlock), 0, sm, G.GA, b, L, 0);
    const int nres = shade_grid(c, std::min(G.nmax * (kVMax + 2), pp.bb[0].cap_sq));
    hipLaunchKernelGGL(k_camera_step, dim3(nres + (more ? g : 0), gn), dim3(kShadeBlock), 0, sm, G.GA, slot, nres,
                       more ? 1 : 0, L, 0);
    tm.mark(WR_K_SHADE);
    return WR_OK;
  };
  auto issue = [&](GroupIssue& G, int step) -> int {
    if (overlap) return issue_overlap(G, step);
    Pipe& pp = *G.pp;
    const hipStream_t sm = pp.stream;
    Timer tm(c, &pp);
    const int gn = G.gn;
    const BdptArgs* A = G.GA.a;
    auto sq = [&](int m, int slot) {
      const BdptBuf::Sq& Q = pp.bb[m].sq[slot & 1];
      return rq(Q.o, Q.d, pp.bb[m].cap_sq, &pp.sc[m].sq[slot], Q.t, Q.prim, nullptr, nullptr, Q.cut);
    };
    // extension rays of step `slot`; bit: the pass's deferral bit (0: not deferrable)
    auto ext = [&](int m, int slot, int bit) {
      const BdptBuf& B = pp.bb[m];
      const int q = slot & 1;
      if (!bit) return rq(B.q_o[q], B.q_d[q], B.qs, &pp.sc[m].ext[slot], B.q_t[q], B.q_prim[q]);
      return rq(B.q_o[q], B.q_d[q], B.qs, &pp.sc[m].ext[slot], B.q_t[q], B.q_prim[q], nullptr, nullptr, nullptr,
                pp.late_d + 2 * m + q, pp.sc[m].late[slot], bit);
    };
    // the late lists of step slot - 1 (when it deferred): settled by extra
    // blocks of step slot's search launch, shaded by extra blocks of its vertex
    // launch, into the queues of step slot + 1
    auto late_of = [&](int slot, LateArgs& L) -> bool {
      if (slot < 1 || !G.late[slot - 1]) return false;
      const int k = (slot - 1) & 1;
      for (int m = 0; m < kGroup; ++m) {
        L.l[m] = pp.late_h[m][k];
        L.n[m] = pp.sc[m].late[slot - 1];
      }
      return true;
    };
    const int lg = std::max(1, std::min(shade_grid(c, G.nmax), 32));  // late-vertex blocks per member
    const int sq_max = std::min(G.nmax * (kVMax + 2), pp.bb[0].cap_sq);
    const int g = shade_grid(c, G.nmax);
    if (step == 0) {
      HIPCHK(hipMemsetAsync(pp.sc, 0, gn * sizeof(StepCounters), sm));
      if (defer) HIPCHK(hipMemsetAsync(pp.delayed, 0, kGroup * pp.late_paths, sm));
      for (bool& x : G.late) x = false;
      // ---------------- light pass (:67-131)
      hipLaunchKernelGGL(k_light_gen, dim3(g, gn), dim3(kShadeBlock), 0, sm, G.GA);
      tm.mark(WR_K_GEN);
    } else if (step <= lb_n) {
      const int b = step - 1;
      // deferrable up to the last regular bounce (a deferred path's next ray is
      // traced one step late: the extra step b = maxlen - 1 traces the last ones)
      const int bit = (defer && b <= maxlen - 2) ? 1 : 0;
      LateArgs L{};
      const bool lp = late_of(b, L);
      QueueList ql;
      for (int m = 0; m < gn; ++m) ql.add(ext(m, b, bit), A[m].n);
      trace_launch(c, sm, pp.ctr, tslot(pp, b), tm, count, ql.Q, ql.max_rays, WR_BDPT_TRACE_MODE, false,
                   lp ? &L : nullptr, gn);
      hipLaunchKernelGGL(k_light_shade, dim3(g + (lp ? lg : 0), gn), dim3(kShadeBlock), 0, sm, G.GA, b, L,
                         lp ? lg : 0);
      tm.mark(WR_K_SHADE);
      G.late[b] = bit != 0;
    } else if (step == lb_n + 1) {
      // ---------------- camera pass (:133-264).  The light pass's splat rays
      // (connectToCamera) ride along with the primary rays; afterwards each
      // bounce's shadow / aux rays ride along with the next bounce's extension rays.
      hipLaunchKernelGGL(k_camera_gen, dim3(g, gn), dim3(kShadeBlock), 0, sm, G.GA);
      tm.mark(WR_K_GEN);
    } else {
      const int b = step - lb_n - 2;
      const int slot = kCamSlot + b;
      const bool more = b < maxlen + (defer ? 1 : 0);  // extension rays of bounce b exist
      const int bit = (defer && b <= maxlen - 1) ? 2 : 0;
      LateArgs L{};
      const bool lp = late_of(slot, L);
      QueueList ql;
      for (int m = 0; m < gn; ++m) ql.add(sq(m, slot), std::min(A[m].n * (kVMax + 2), pp.bb[m].cap_sq));
      if (more)
        for (int m = 0; m < gn; ++m) ql.add(ext(m, slot, bit), A[m].n);
      trace_launch(c, sm, pp.ctr, tslot(pp, slot), tm, count, ql.Q, ql.max_rays, WR_BDPT_TRACE_MODE, false,
                   lp ? &L : nullptr, gn);
      // resolve this step's shadow / aux rays and shade its vertices (and the
      // previous step's deferred ones) in one launch
      const int nres = shade_grid(c, sq_max);
      hipLaunchKernelGGL(k_camera_step, dim3(nres + (more ? g : 0) + (lp ? lg : 0), gn), dim3(kShadeBlock), 0, sm,
                         G.GA, slot, nres, more ? 1 : 0, L, lp ? lg : 0);
      tm.mark(WR_K_SHADE);
      G.late[slot] = bit != 0;
    }
    return WR_OK;
  };
  // Round r takes every pipeline's r-th group, and the launches go out step by
  // step across the pipelines: each stream runs its own in order, and all of
  // them get their first launches at once instead of one pipeline's ~90
  // launches after another's (host issue time: ~2 us per call)
  unsigned long long overflow = 0;
  auto run = [&](const PiecePlan& pl) -> int {
  const int npl = pl.pipes();
  begin_render(c, npl, prm->time_kernels);
  std::vector<GroupIssue> round(npl);
  for (int r = 0; r < pl.max_groups(); ++r) {
    int live = 0;
    for (int pi = 0; pi < npl; ++pi) {
      GroupIssue& G = round[pi];
      G.gn = 0;
      if (r >= static_cast<int>(pl.per_pipe[pi].size())) continue;
      const std::vector<Piece>& grp = pl.per_pipe[pi][r];
      G.pp = &c->pipes[pi];
      G.gn = static_cast<int>(grp.size());
      G.nmax = 0;
      for (int m = 0; m < G.gn; ++m) {
        const Piece& pc = grp[m];
        BdptArgs& a = G.GA.a[m];
        a = A0;
        a.B = G.pp->bb[m];
        a.ctr = G.pp->ctr;
        a.sc = G.pp->sc + m;
        a.iter = static_cast<uint32_t>(prm->iter_begin + pc.iter);
        a.base = pc.base;
        a.n = pc.n;
        G.nmax = std::max(G.nmax, pc.n);
      }
      live += G.gn > 0;
    }
    if (!live) continue;
    if (int rc = issue_round(c, live, nsteps, [&](int pi, int step) {
          return round[pi].gn > 0 ? issue(round[pi], step) : WR_OK;
        }, npl))
      return rc;
  }
  HIPCHK(hipGetLastError());
  if (std::getenv("WR_ISSUE_LOG"))
    std::fprintf(stderr, "[wr issue] kernel args: BdptGroup %zu B, TraceQueues %zu B, DevScene %zu B, FastScene %zu B\n",
                 sizeof(BdptGroup), sizeof(TraceQueues), sizeof(DevScene), sizeof(c->fs));
  return finish_render(c, npl, st, t0, &overflow);
  };
  // an error after the first launch leaves a caller's device film as it was
  // before the render (its saved copy), not holding a partial render
  auto restore_film = [&](int rc) -> int {
    if (pooled && film_on_device) {
      (void)hipDeviceSynchronize();  // the pipelines' launches in flight
      (void)hipMemcpy(dfilm, c->film_bak, nf * sizeof(float), hipMemcpyDeviceToDevice);
    }
    return rc;
  };
  if (int rc = run(plan)) return restore_film(rc);
  if (overflow) {
    // A vertex pool or shadow queue filled up and appends were dropped: redo
    // the render from the film as it was, with pieces whose worst case fits
    // every pool (<= 11 shadow rays per path and step, 9 light and 4 camera
    // vertices per path), in the untiled camera order (64-path units; the
    // path <-> pixel map is the same), so the film is the one of an unbounded
    // render.  Rare: the pools hold several times what the reference scenes use.
    const BdptBuf& B = c->pipes[0].bb[0];
    const int safe = std::min({B.cap_sq / (kVMax + 2), B.vcap / kVMax, B.ccap / kCvMax, cap}) / 64 * 64;
    if (safe < 64) return restore_film(fail(WR_E_HIP, "BDPT pools too small for a 64-path piece"));
    if (film_on_device) HIPCHK(hipMemcpyAsync(dfilm, c->film_bak, nf * sizeof(float), hipMemcpyDeviceToDevice, c->stream));
    else HIPCHK(hipMemsetAsync(dfilm, 0, nf * sizeof(float), c->stream));
    if (st) *st = st0;
    A0.untiled = 1;
    overflow = 0;
    if (int rc = run(plan_pieces(f_lo, f_hi, P, 64, safe, fit, c->piece_min))) return restore_film(rc);
    // (env WR_TEST_REDO_FAIL=1: the test of this error path treats the redo as overflowed)
    if (overflow || std::getenv("WR_TEST_REDO_FAIL"))
      return restore_film(fail(WR_E_HIP, "BDPT pools overflowed with pieces the worst case fits"));
    if (st) st->redone += 1;
  }
  if (st) {
    for (int i = 0; i < np; ++i) st->work_bytes += static_cast<int64_t>(c->pipes[i].work.cap);
    st->work_paths += static_cast<int64_t>(np) * kGroup * cap;
  }
  return film_return(c, film, film_on_device, nf);
}

static int check_vcm(const wr_context* c, const wr_vcm_params* prm, const float* film) {
  if (!c || !prm || !film) return fail(WR_E_ARG, "null argument");
  if (prm->width <= 0 || prm->height <= 0 || prm->iterations < 0) return fail(WR_E_ARG, "bad film size");
  if (static_cast<int64_t>(prm->width) * prm->height >= (1 << 30) / (kVMax + 2))
    return fail(WR_E_ARG, "film too large for one context");
  if (prm->max_path_length < 1 || prm->max_path_length > kVMax + 1)
    return fail(WR_E_ARG, "max_path_length must be in 1..10 (light-vertex store sized for the reference's 10)");
  if (prm->min_path_length < 0 || !(prm->radius_factor > 0.f) || !(prm->radius_alpha <= 1.f))
    return fail(WR_E_ARG, "bad min_path_length / radius_factor / radius_alpha");
  if (c->ds.nlights <= 0) return fail(WR_E_SCENE, "VCM needs at least one area light");
  return WR_OK;
}
static int render_vcm_one(wr_context* c, const wr_vcm_params* prm, float* film, int film_on_device, wr_stats* st) {
  HIPCHK(hipSetDevice(c->device));
  const double t0 = host_now();
  const int P = prm->width * prm->height;
  const int ngroups = (prm->iterations + kGroup - 1) / kGroup;
  const int fit = pipelines_that_fit(c, 3, P, kGroup, c->npipes);
  if (fit < 1) return WR_E_HIP;  // message set by the allocation
  const int np = std::max(1, std::min(fit, ngroups));
  {  // WR_TRACE_BVH t2 scratch: a launch takes <= kGroup x (shadow / aux + extension) queues
    const size_t cap_sq = size_t(c->pipes[0].bb[0].cap_sq);
    const size_t per = kGroup * (std::max(cap_sq, size_t(P)) + size_t(P));
    for (int i = 0; i < fit; ++i)
      if (int rc = ensure_t2(c, c->pipes[i], per)) return rc;
  }
  float* dfilm = nullptr;
  const size_t nf = size_t(P) * 3;
  if (int rc = film_target(c, film, film_on_device, nf, &dfilm)) return rc;
  begin_render(c, np, prm->time_kernels);
  VcmArgs X0;
  BdptArgs& A0 = X0.a;
  A0.S = c->ds;
  A0.film = dfilm;
  A0.W = prm->width;
  A0.H = prm->height;
  A0.P = P;
  A0.seed = prm->seed;
  A0.ctl = 0;
  A0.maxlen = prm->max_path_length;
  A0.faithful = 1;
  // VCM renders whole iterations: every camera vertex merges with the light
  // vertices of the whole iteration (:152, :265-276)
  A0.base = 0;
  A0.n = P;
  X0.minlen = prm->min_path_length;
  X0.N = static_cast<float>(prm->height * prm->width);
  X0.org = c->ds.root_l;
  const uint32_t T = vcm_table(P);
  X0.tmask = T - 1;
  const float base_radius = prm->radius_factor * c->sph_r;  // VertexCM::init (:13)
  const int maxlen = A0.maxlen;
  const bool count = prm->count_work != 0;
  const int g = shade_grid(c, P);
  for (int gi = 0; gi < ngroups; ++gi) {
    Pipe& pp = c->pipes[gi % np];
    const hipStream_t sm = pp.stream;
    Timer tm(c, &pp);
    const int it0 = gi * kGroup, gn = std::min(kGroup, prm->iterations - it0);
    VcmGroup GA;
    for (int m = 0; m < gn; ++m) {
      VcmArgs& X = GA.a[m];
      X = X0;
      X.a.B = pp.bb[m];
      X.V = pp.vb[m];
      X.a.ctr = pp.ctr;
      X.a.sc = pp.sc + m;
      const int it = prm->iter_begin + it0 + m;
      X.a.iter = static_cast<uint32_t>(it);
      // runIteration's radius schedule and MIS factors (:50-64), host float
      float radius = base_radius;
      radius /= powf(static_cast<float>(it + 1), 0.5f * (1.f - prm->radius_alpha));
      radius = (radius < WR_EPS) ? WR_EPS : radius;
      const float r2 = radius * radius;
      X.radius = radius;
      X.vm_norm = 1.f / (r2 * WR_PI * X.N);
      const float eta = (WR_PI * r2) * X.N;
      X.mis_vm = eta;
      X.mis_vc = 1.f / eta;
      X.rq = radius * 1.0009765625f;
      // the first float s with sqrtf(s) >= radius: sqrtf is correctly rounded
      // and monotone on host and device, so `sqrtf(s) < radius` == `s < r2t`
      float t = r2;
      while (t > 0.f && std::sqrt(t) >= radius) t = std::nextafter(t, 0.f);
      while (!(std::sqrt(t) >= radius)) t = std::nextafter(t, INFINITY);
      X.r2t = t;
      X.inv_cs = 1.f / (c->vcm_cell * X.rq);
    }
    auto sq = [&](int m, int slot) {
      const BdptBuf::Sq& Q = pp.bb[m].sq[slot & 1];
      return rq(Q.o, Q.d, pp.bb[m].cap_sq, &pp.sc[m].sq[slot], Q.t, Q.prim, nullptr, nullptr, Q.cut);
    };
    auto ext = [&](int m, int slot) {
      const BdptBuf& B = pp.bb[m];
      const int q = slot & 1;
      return rq(B.q_o[q], B.q_d[q], P, &pp.sc[m].ext[slot], B.q_t[q], B.q_prim[q]);
    };
    const int sq_max = pp.bb[0].cap_sq;
    HIPCHK(hipMemsetAsync(pp.sc, 0, gn * sizeof(StepCounters), sm));
    // ---------------- light pass (:67-140)
    hipLaunchKernelGGL(k_vcm_light_gen, dim3(g, gn), dim3(kShadeBlock), 0, sm, GA);
    tm.mark(WR_K_GEN);
    for (int b = 0; b < maxlen - 1; ++b) {
      QueueList ql;
      for (int m = 0; m < gn; ++m) ql.add(ext(m, b), P);
      trace_launch(c, sm, pp.ctr, tslot(pp, b), tm, count, ql.Q, ql.max_rays);
      hipLaunchKernelGGL(k_vcm_light_shade, dim3(g, gn), dim3(kShadeBlock), 0, sm, GA, b);
      tm.mark(WR_K_SHADE);
    }
    // ---------------- light vertices -> merge grid (replaces the KdTree, :152)
    hipLaunchKernelGGL(k_vcm_fixup, dim3(64, gn), dim3(kShadeBlock), 0, sm, GA);
    for (int m = 0; m < gn; ++m) HIPCHK(hipMemsetAsync(pp.vb[m].cnt, 0, (size_t(T) + 1) * sizeof(int), sm));
    hipLaunchKernelGGL(k_vgrid_count, dim3(g, gn), dim3(kShadeBlock), 0, sm, GA);
    for (int m = 0; m < gn; ++m) {
      size_t bytes = pp.vb[m].scan_bytes;
      HIPCHK(hipcub::DeviceScan::ExclusiveSum(pp.vb[m].scan_tmp, bytes, pp.vb[m].cnt, pp.vb[m].start,
                                              static_cast<int>(T + 1), sm));
    }
    hipLaunchKernelGGL(k_vgrid_scatter, dim3(g, gn), dim3(kShadeBlock), 0, sm, GA);
    tm.mark(WR_K_OTHER);
    // ---------------- camera pass (:157-283)
    hipLaunchKernelGGL(k_vcm_camera_gen, dim3(g, gn), dim3(kShadeBlock), 0, sm, GA);
    tm.mark(WR_K_GEN);
    for (int b = 0; b <= maxlen; ++b) {
      const int slot = kCamSlot + b;
      const bool more = b < maxlen;
      QueueList ql;
      for (int m = 0; m < gn; ++m) ql.add(sq(m, slot), sq_max);
      if (more)
        for (int m = 0; m < gn; ++m) ql.add(ext(m, slot), P);
      trace_launch(c, sm, pp.ctr, tslot(pp, slot), tm, count, ql.Q, ql.max_rays, WR_VCM_TRACE_MODE);
      const int nres = shade_grid(c, sq_max);
      // + the merge queries of the previous step (none before the first)
      const int nsh = more ? g : 0, nmg = b > 0 ? g : 0;
      hipLaunchKernelGGL(k_vcm_camera_step, dim3(nres + nsh + nmg, gn), dim3(kShadeBlock), 0, sm, GA, slot, nres,
                         nsh);
      tm.mark(WR_K_SHADE);
    }
  }
  HIPCHK(hipGetLastError());
  if (int rc = finish_render(c, np, st, t0)) return rc;
  return film_return(c, film, film_on_device, nf);
}

static int check_radiance(const wr_context* c, const wr_ray* rays, int64_t n64, int32_t max_depth, const float* rgb) {
  if (!c || ((!rays || !rgb) && n64) || n64 < 0) return fail(WR_E_ARG, "bad argument");
  if (max_depth < 0 || max_depth > kSlots - 3) return fail(WR_E_ARG, "max_depth must be in 0..61");
  if (n64 > (1 << 26)) return fail(WR_E_ARG, "at most 2^26 rays per call");
  if (c->ds.nlights <= 0) return fail(WR_E_SCENE, "path tracing needs at least one area light");
  return WR_OK;
}
static int path_radiance_one(wr_context* c, const wr_ray* rays, int64_t n64, int32_t max_depth, uint32_t seed,
                             int32_t sample, float* rgb, wr_stats* st) {
  if (n64 == 0) return WR_OK;
  HIPCHK(hipSetDevice(c->device));
  const double t0 = host_now();
  const int P = static_cast<int>(n64);
  if (pipelines_that_fit(c, 2, P, 1, 1) < 1) return WR_E_HIP;
  if (int rc = ensure_t2(c, c->pipes[0], 2 * size_t(P))) return rc;
  Pipe& pp = c->pipes[0];  // the context stream
  const size_t nf = size_t(P) * 3;
  std::memset(rgb, 0, nf * sizeof(float));
  float* dfilm = nullptr;
  if (int rc = film_target(c, rgb, 0, nf, &dfilm)) return rc;
  if (int rc = api_scratch(c, size_t(P) * sizeof(wr_ray))) return rc;
  wr_ray* drays = reinterpret_cast<wr_ray*>(c->api_tmp);
  HIPCHK(hipMemcpyAsync(drays, rays, size_t(P) * sizeof(wr_ray), hipMemcpyHostToDevice, pp.stream));
  begin_render(c, 1, 0);
  PtGroup GA;
  PtArgs& A = GA.a[0];
  A.S = c->ds;
  A.T = pp.pb[0];
  A.ctr = pp.ctr;
  A.sc = pp.sc;
  A.film = dfilm;
  A.W = P;
  A.H = 1;
  A.P = P;
  A.spp = 1;
  A.grid_len = 1;
  A.max_depth = max_depth;
  A.seed = seed;
  A.k = static_cast<uint32_t>(sample);
  const hipStream_t sm = pp.stream;
  Timer tm(c, &pp);
  const int g = shade_grid(c, P);
  HIPCHK(hipMemsetAsync(pp.sc, 0, sizeof(StepCounters), sm));
  hipLaunchKernelGGL(k_pt_gen_rays, dim3(g, 1), dim3(kShadeBlock), 0, sm, GA, drays);
  for (int b = 0; b <= max_depth + 1; ++b) {
    const bool more = b <= max_depth;
    const PtBuf& T = pp.pb[0];
    const PtBuf::Sq& Q = T.sq[b & 1];
    QueueList ql;
    ql.add(rq(Q.o, Q.d, P, &pp.sc[0].sq[b], Q.t, Q.prim, nullptr, nullptr, Q.cut), P);
    if (more) ql.add(rq(T.q_o[b & 1], T.q_d[b & 1], P, &pp.sc[0].ext[b], T.q_t[b & 1], T.q_prim[b & 1]), P);
    trace_launch(c, sm, pp.ctr, tslot(pp, b), tm, false, ql.Q, ql.max_rays, TRACE_DENSE, true);
    const int nres = shade_grid(c, P);
    hipLaunchKernelGGL(k_pt_step, dim3(nres + (more ? g : 0), 1), dim3(kShadeBlock), 0, sm, GA, b, nres,
                       more ? 1 : 0);
    if (!more) break;
  }
  HIPCHK(hipGetLastError());
  if (int rc = finish_render(c, 1, st, t0)) return rc;
  return film_return(c, rgb, 0, nf);
}

static int check_path(const wr_context* c, const wr_path_params* prm, const float* film) {
  if (!c || !prm || !film) return fail(WR_E_ARG, "null argument");
  if (prm->width <= 0 || prm->height <= 0 || prm->spp <= 0) return fail(WR_E_ARG, "bad film size / spp");
  // path-state arrays are indexed up to 3 * P in 32-bit ints
  if (static_cast<int64_t>(prm->width) * prm->height >= (int64_t(1) << 31) / 4)
    return fail(WR_E_ARG, "film too large for one context");
  if (prm->max_depth < 0 || prm->max_depth > kSlots - 3) return fail(WR_E_ARG, "max_depth must be in 0..61");
  // sample k of the spp grid (surfaceIntegrator.cpp:26-32): only 0 <= k < spp exist
  if (prm->sample_begin < 0 || prm->sample_count < 0 ||
      static_cast<int64_t>(prm->sample_begin) + prm->sample_count > prm->spp ||
      prm->sample_begin > prm->spp)
    return fail(WR_E_ARG, "samples [sample_begin, sample_begin + sample_count) must lie in [0, spp)");
  if (c->ds.nlights <= 0) return fail(WR_E_SCENE, "path tracing needs at least one area light");
  return WR_OK;
}
static int render_path_one(wr_context* c, const wr_path_params* prm, float* film, int film_on_device, wr_stats* st) {
  HIPCHK(hipSetDevice(c->device));
  const double t0 = host_now();
  const int P = prm->width * prm->height;
  const int k0 = prm->sample_begin;
  const int k1 = prm->sample_count > 0 ? k0 + prm->sample_count : prm->spp;
  const int nk = std::max(0, k1 - k0);
  const int ngroups = (nk + kGroup - 1) / kGroup;
  const int fit = pipelines_that_fit(c, 2, P, kGroup, c->npipes);
  if (fit < 1) return WR_E_HIP;  // message set by the allocation
  const int np = std::max(1, std::min(fit, ngroups));
  {  // WR_TRACE_BVH t2 scratch: a launch takes <= kGroup x (shadow / aux + extension) queues
    const size_t cap_sq = size_t(c->pipes[0].bb[0].cap_sq);
    const size_t per = kGroup * (std::max(cap_sq, size_t(P)) + size_t(P));
    for (int i = 0; i < fit; ++i)
      if (int rc = ensure_t2(c, c->pipes[i], per)) return rc;
  }
  float* dfilm = nullptr;
  const size_t nf = size_t(P) * 3;
  if (int rc = film_target(c, film, film_on_device, nf, &dfilm)) return rc;
  begin_render(c, np, prm->time_kernels);
  PtArgs A0;
  A0.S = c->ds;
  A0.film = dfilm;
  A0.W = prm->width;
  A0.H = prm->height;
  A0.P = P;
  A0.spp = prm->spp;
  A0.grid_len = static_cast<int>(std::sqrt(static_cast<double>(prm->spp)));
  A0.max_depth = prm->max_depth;
  A0.seed = prm->seed;
  const bool count = prm->count_work != 0;
  const int g = shade_grid(c, P);
  for (int gi = 0; gi < ngroups; ++gi) {
    // a group of gn samples in lockstep on pipeline gi % np
    Pipe& pp = c->pipes[gi % np];
    const hipStream_t sm = pp.stream;
    Timer tm(c, &pp);
    const int gk = k0 + gi * kGroup, gn = std::min(kGroup, k1 - gk);
    PtGroup GA;
    PtArgs* A = GA.a;
    for (int m = 0; m < gn; ++m) {
      A[m] = A0;
      A[m].T = pp.pb[m];
      A[m].ctr = pp.ctr;
      A[m].sc = pp.sc + m;
      A[m].k = static_cast<uint32_t>(gk + m);
    }
    HIPCHK(hipMemsetAsync(pp.sc, 0, gn * sizeof(StepCounters), sm));
    hipLaunchKernelGGL(k_pt_gen, dim3(g, gn), dim3(kShadeBlock), 0, sm, GA);
    tm.mark(WR_K_GEN);
    for (int b = 0; b <= A0.max_depth + 1; ++b) {
      // NEE shadow rays of the previous vertex ride along with this bounce's rays
      const bool more = b <= A0.max_depth;
      const int q = b & 1;
      QueueList ql;
      for (int m = 0; m < gn; ++m) {
        const PtBuf& T = pp.pb[m];
        const PtBuf::Sq& Q = T.sq[b & 1];
        ql.add(rq(Q.o, Q.d, P, &pp.sc[m].sq[b], Q.t, Q.prim, nullptr, nullptr, Q.cut), P);
      }
      if (more)
        for (int m = 0; m < gn; ++m) {
          const PtBuf& T = pp.pb[m];
          ql.add(rq(T.q_o[q], T.q_d[q], P, &pp.sc[m].ext[b], T.q_t[q], T.q_prim[q]), P);
        }
      trace_launch(c, sm, pp.ctr, tslot(pp, b), tm, count, ql.Q, ql.max_rays, TRACE_DENSE);
      // resolve this step's shadow rays and shade its vertices in one launch
      const int nres = shade_grid(c, P);
      hipLaunchKernelGGL(k_pt_step, dim3(nres + (more ? g : 0), gn), dim3(kShadeBlock), 0, sm, GA, b, nres,
                         more ? 1 : 0);
      tm.mark(WR_K_SHADE);
      if (!more) break;
    }
  }
  HIPCHK(hipGetLastError());
  if (int rc = finish_render(c, np, st, t0)) return rc;
  return film_return(c, film, film_on_device, nf);
}


// ---- multi-device renders (wr_create_multi)
static void add_stats(wr_stats* d, const wr_stats& s) {
  d->closest_rays += s.closest_rays;
  d->shadow_rays += s.shadow_rays;
  d->inner_visits += s.inner_visits;
  d->leaf_visits += s.leaf_visits;
  d->prim_refs += s.prim_refs;
  for (int k = 0; k < WR_K_NUM; ++k) {
    d->kernel_ms[k] += s.kernel_ms[k];
    d->kernel_launches[k] += s.kernel_launches[k];
  }
  d->vm_queries += s.vm_queries;
  d->vm_found += s.vm_found;
  d->vm_merged += s.vm_merged;
  d->prim_tests += s.prim_tests;
  d->bvh_nodes += s.bvh_nodes;
  d->bvh_tests += s.bvh_tests;
  d->kd_replay_steps += s.kd_replay_steps;
  d->fallback_rays += s.fallback_rays;
  d->verify_rays += s.verify_rays;
  d->verify_mismatches += s.verify_mismatches;
  d->pipelines = std::max(d->pipelines, s.pipelines);
  d->deferred_rays += s.deferred_rays;
  d->bvh_width = std::max(d->bvh_width, s.bvh_width);
  d->work_bytes += s.work_bytes;
  d->work_paths += s.work_paths;
  d->redone += s.redone;
}

static int ensure_dev_film(wr_context* d, float** buf, size_t* have, size_t nf) {
  if (*have >= nf) return WR_OK;
  if (*buf) (void)hipFree(*buf);
  *buf = nullptr;
  *have = 0;
  HIPCHK(hipSetDevice(d->device));
  HIPCHK(hipMalloc(buf, nf * sizeof(float)));
  *have = nf;
  return WR_OK;
}

// films[k] (on device k) summed into films[0]: one RCCL reduce over the
// devices' communicators, or peer copies to devices[0] + an add kernel
static int reduce_films(wr_context* c, const std::vector<wr_context*>& dev, const std::vector<float*>& films,
                        size_t nf) {
  const int n = static_cast<int>(dev.size());
  if (n == 1) return WR_OK;
  if (static_cast<int>(c->dev_comms.size()) == n) {
    NCCLCHK(rccl().group_start());
    for (int k = 0; k < n; ++k) {
      HIPCHK(hipSetDevice(dev[k]->device));
      // in place on the root; the receive buffer is ignored elsewhere
      NCCLCHK(rccl().reduce(films[k], films[k], nf, ncclFloat32, ncclSum, 0, c->dev_comms[k], dev[k]->stream));
    }
    NCCLCHK(rccl().group_end());
    for (int k = 0; k < n; ++k) {
      HIPCHK(hipSetDevice(dev[k]->device));
      HIPCHK(hipStreamSynchronize(dev[k]->stream));
    }
    return WR_OK;
  }
  HIPCHK(hipSetDevice(c->device));
  const int g = static_cast<int>(std::min<size_t>(4096, (nf + 255) / 256));
  for (int k = 1; k < n; ++k) {
    const float* src = films[k];
    if (dev[k]->device != c->device) {
      if (int rc = ensure_dev_film(c, &c->stage_buf, &c->stage_n, nf)) return rc;
      HIPCHK(hipMemcpyPeerAsync(c->stage_buf, c->device, films[k], dev[k]->device, nf * sizeof(float), c->stream));
      src = c->stage_buf;
    }
    hipLaunchKernelGGL(k_film_accumulate, dim3(g), dim3(256), 0, c->stream, films[0], src, nf);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  return WR_OK;
}

extern "C++" {
// Every device renders its share (fn) into a film of its own (devices[0]:
// the caller's device film, if given), the films are summed on devices[0],
// and a host film gets the sum added.  Stats: counts summed, seconds = the
// call's wall time, trace_wall_ms = the largest device's.
template <class Fn>
static int multi_render(wr_context* c, size_t nf, float* film, int film_on_device, wr_stats* st, Fn fn) {
  const double t0 = host_now();
  std::vector<wr_context*> dev{c};
  dev.insert(dev.end(), c->subs.begin(), c->subs.end());
  const int n = static_cast<int>(dev.size());
  std::vector<float*> buf(n, nullptr);
  for (int k = 0; k < n; ++k) {
    if (k == 0 && film_on_device) {
      buf[0] = film;
      continue;
    }
    if (int rc = ensure_dev_film(dev[k], &dev[k]->red_buf, &dev[k]->red_n, nf)) return rc;
    HIPCHK(hipMemsetAsync(dev[k]->red_buf, 0, nf * sizeof(float), dev[k]->stream));
    buf[k] = dev[k]->red_buf;
  }
  std::vector<wr_stats> s(n);
  for (auto& x : s) std::memset(&x, 0, sizeof x);
  if (int rc = for_each_device(c, [&](wr_context* d, int k) { return fn(d, k, n, buf[k], &s[k]); })) return rc;
  if (int rc = reduce_films(c, dev, buf, nf)) return rc;
  if (!film_on_device) {
    std::vector<float> tmp(nf);
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpy(tmp.data(), buf[0], nf * sizeof(float), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < nf; ++i) film[i] = film[i] + tmp[i];
  }
  if (st) {
    double wall = 0.0;
    for (const auto& x : s) {
      add_stats(st, x);
      wall = std::max(wall, x.trace_wall_ms);
    }
    st->trace_wall_ms += wall;
    st->seconds += host_now() - t0;
  }
  return WR_OK;
}

}  // extern "C++"

// The work buffers every pipeline of one device needs for renders of this
// kind and film size: what the first render would allocate (SurfaceIntegrator::
// init's share of the set-up, surfaceIntegrator.h:14-34), so that render()
// itself only renders.
static int reserve_one(wr_context* c, int kind, int W, int H) {
  HIPCHK(hipSetDevice(c->device));
  const int P = W * H;
  int fit = 0, cap = P;
  if (kind == WR_INTEGRATOR_BDPT) {
    wr_bdpt_params prm{};
    prm.width = W;
    prm.height = H;
    cap = piece_capacity(c, P, bdpt_unit(&prm));
    fit = pipelines_that_fit(c, 1, cap, kGroup, c->npipes);
  } else {
    fit = pipelines_that_fit(c, kind == WR_INTEGRATOR_VCM ? 3 : 2, P, kGroup, c->npipes);
  }
  if (fit < 1) return WR_E_HIP;  // message set by the allocation
  const size_t cap_sq = size_t(c->pipes[0].bb[0].cap_sq);
  const size_t per = kGroup * (std::max(cap_sq, size_t(cap)) + 2 * size_t(cap));
  for (int i = 0; i < fit; ++i)
    if (int rc = ensure_t2(c, c->pipes[i], per)) return rc;
  if (kind == WR_INTEGRATOR_BDPT && c->fast_on && !c->stamps && defer_enabled(c, fit))
    for (int i = 0; i < fit; ++i)
      if (int rc = ensure_late(c->pipes[i], cap, late_records(cap))) return rc;
  HIPCHK(hipDeviceSynchronize());
  return WR_OK;
}

int wr_reserve(wr_context* c, int integrator, int32_t width, int32_t height) {
  if (!c) return fail(WR_E_ARG, "null argument");
  if (integrator < WR_INTEGRATOR_BDPT || integrator > WR_INTEGRATOR_PATH) return fail(WR_E_ARG, "bad integrator");
  if (width <= 0 || height <= 0) return fail(WR_E_ARG, "bad film size");
  if (static_cast<int64_t>(width) * height >= (1 << 30) / (kVMax + 2)) return fail(WR_E_ARG, "film too large for one context");
  DeviceGuard dg;
  if (int rc = reserve_one(c, integrator, width, height)) return rc;
  for (wr_context* d : c->subs)
    if (int rc = reserve_one(d, integrator, width, height)) return rc;
  return WR_OK;
}

int wr_render_bdpt(wr_context* c, const wr_bdpt_params* prm, float* film, int film_on_device, wr_stats* st) {
  if (int rc = check_bdpt(c, prm, film)) return rc;
  DeviceGuard dg;
  const int P = prm->width * prm->height;
  const int64_t T = static_cast<int64_t>(prm->iterations) * P;
  if (c->subs.empty()) return render_bdpt_one(c, prm, 0, T, film, film_on_device, st);
  // devices take equal contiguous shares of the flattened path-iterations:
  // a single iteration (the reference's default, bidirPathTracing.cpp:9)
  // still spreads over every device
  const int unit = bdpt_unit(prm);
  return multi_render(c, size_t(P) * 3, film, film_on_device, st,
                      [&](wr_context* d, int k, int n, float* buf, wr_stats* s) {
                        const int64_t lo = k == 0 ? 0 : flat_round(T * k / n, P, unit);
                        const int64_t hi = k == n - 1 ? T : flat_round(T * (k + 1) / n, P, unit);
                        return render_bdpt_one(d, prm, lo, hi, buf, 1, s);
                      });
}

int wr_render_vcm(wr_context* c, const wr_vcm_params* prm, float* film, int film_on_device, wr_stats* st) {
  if (int rc = check_vcm(c, prm, film)) return rc;
  DeviceGuard dg;
  if (c->subs.empty()) return render_vcm_one(c, prm, film, film_on_device, st);
  // whole iterations per device: an iteration's merge grid holds all of its
  // light vertices (vertexcm.cpp:152)
  const int I = prm->iterations;
  return multi_render(c, size_t(prm->width) * prm->height * 3, film, film_on_device, st,
                      [&](wr_context* d, int k, int n, float* buf, wr_stats* s) {
                        wr_vcm_params q = *prm;
                        const int lo = I * k / n, hi = I * (k + 1) / n;
                        if (hi <= lo) return static_cast<int>(WR_OK);
                        q.iter_begin = prm->iter_begin + lo;
                        q.iterations = hi - lo;
                        return render_vcm_one(d, &q, buf, 1, s);
                      });
}

int wr_render_path(wr_context* c, const wr_path_params* prm, float* film, int film_on_device, wr_stats* st) {
  if (int rc = check_path(c, prm, film)) return rc;
  DeviceGuard dg;
  if (c->subs.empty()) return render_path_one(c, prm, film, film_on_device, st);
  const int k0 = prm->sample_begin, k1 = prm->sample_count > 0 ? k0 + prm->sample_count : prm->spp;
  return multi_render(c, size_t(prm->width) * prm->height * 3, film, film_on_device, st,
                      [&](wr_context* d, int k, int n, float* buf, wr_stats* s) {
                        wr_path_params q = *prm;  // contiguous sample ranges of the spp grid
                        const int lo = k0 + (k1 - k0) * k / n, hi = k0 + (k1 - k0) * (k + 1) / n;
                        if (hi <= lo) return static_cast<int>(WR_OK);
                        q.sample_begin = lo;
                        q.sample_count = hi - lo;
                        return render_path_one(d, &q, buf, 1, s);
                      });
}

int wr_path_radiance(wr_context* c, const wr_ray* rays, int64_t n64, int32_t max_depth, uint32_t seed,
                     int32_t sample, float* rgb, wr_stats* st) {
  if (int rc = check_radiance(c, rays, n64, max_depth, rgb)) return rc;
  DeviceGuard dg;
  return path_radiance_one(c, rays, n64, max_depth, seed, sample, rgb, st);  // devices[0]
}

int wr_create_multi(const wr_scene* sc, const int* devices, int n, wr_context** out) {
  if (!sc || !devices || !out || n < 1 || n > 64) return fail(WR_E_ARG, "bad argument (1..64 devices)");
  *out = nullptr;
  if (int rc = check_device()) return rc;
  DeviceGuard dg;
  int have = 0;
  (void)hipGetDeviceCount(&have);
  for (int k = 0; k < n; ++k)
    if (devices[k] < 0 || devices[k] >= have)
      return fail(WR_E_ARG, "device " + std::to_string(devices[k]) + " not visible (" + std::to_string(have) + ")");
  // one context per device, created concurrently (scene upload + BVH build each)
  std::vector<wr_context*> ctx(n, nullptr);
  std::vector<int> rc(n, WR_OK);
  std::vector<std::string> msg(n);
  {
    std::vector<std::thread> th;
    for (int k = 0; k < n; ++k)
      th.emplace_back([&, k] {
        rc[k] = wr_create(sc, devices[k], &ctx[k]);
        if (rc[k] != WR_OK) msg[k] = wr::last_error();
      });
    for (auto& t : th) t.join();
  }
  for (int k = 0; k < n; ++k)
    if (rc[k] != WR_OK) {
      for (wr_context* x : ctx) wr_destroy(x);
      return fail(rc[k], "device " + std::to_string(devices[k]) + ": " + msg[k]);
    }
  wr_context* c = ctx[0];
  c->subs.assign(ctx.begin() + 1, ctx.end());
  // RCCL communicators over the devices when they are distinct (a device
  // listed twice -- tests on one GPU -- sums by copies); WR_MULTI_REDUCE=peer
  // forces the copies
  bool distinct = true;
  for (int a = 0; a < n; ++a)
    for (int b = a + 1; b < n; ++b) distinct = distinct && devices[a] != devices[b];
  const char* mode = std::getenv("WR_MULTI_REDUCE");
  const bool want = !(mode && std::string(mode) == "peer");
  if (n > 1 && distinct && want) {
    if (!rccl().ok) {
      wr_destroy(c);
      return fail(WR_E_HIP, rccl().why);
    }
    std::vector<ncclComm_t> comms(n, nullptr);
    const ncclResult_t r = rccl().init_all(comms.data(), n, devices);
    if (r != ncclSuccess) {
      wr_destroy(c);
      return fail(WR_E_HIP, std::string("ncclCommInitAll: ") + rccl().err_str(r));
    }
    c->dev_comms = comms;
  }
  *out = c;
  return WR_OK;
}

int wr_context_devices(const wr_context* c, int* devices, int max_n) {
  if (!c || max_n < 0 || (max_n > 0 && !devices)) return fail(WR_E_ARG, "bad argument");
  const int n = 1 + static_cast<int>(c->subs.size());
  for (int k = 0; k < n && k < max_n; ++k) devices[k] = k == 0 ? c->device : c->subs[k - 1]->device;
  return n;
}

// ---- one process per GPU: this rank's RCCL communicator and the film reduce
int wr_comm_unique_id(uint8_t id[128]) {
  if (!id) return fail(WR_E_ARG, "null argument");
  if (!rccl().ok) return fail(WR_E_HIP, rccl().why);
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  ncclUniqueId u;
  NCCLCHK(rccl().get_unique_id(&u));
  std::memcpy(id, &u, sizeof u);
  return WR_OK;
}

int wr_comm_init(wr_context* c, const uint8_t id[128], int nranks, int rank) {
  if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return fail(WR_E_ARG, "bad argument");
  if (!c->subs.empty()) return fail(WR_E_ARG, "a multi-device context reduces over its own devices");
  if (!rccl().ok) return fail(WR_E_HIP, rccl().why);
  DeviceGuard dg;
  HIPCHK(hipSetDevice(c->device));
  if (c->comm) (void)rccl().destroy(c->comm);
  c->comm = nullptr;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  NCCLCHK(rccl().init_rank(&c->comm, nranks, u, rank));
  c->comm_ranks = nranks;
  c->comm_rank = rank;
  return WR_OK;
}

int wr_comm_info(const wr_context* c, int* nranks, int* rank) {
  if (!c || !nranks || !rank) return fail(WR_E_ARG, "null argument");
  if (!c->comm) return fail(WR_E_ARG, "no communicator: call wr_comm_init first");
  // read back from the communicator itself (ncclCommCount / ncclCommUserRank),
  // not from what wr_comm_init was given
  NCCLCHK(rccl().count(c->comm, nranks));
  NCCLCHK(rccl().user_rank(c->comm, rank));
  return WR_OK;
}

int wr_film_reduce(wr_context* c, float* film, int64_t nfloat, int root) {
  if (!c || (!film && nfloat) || nfloat < 0) return fail(WR_E_ARG, "bad argument");
  if (!c->comm) return fail(WR_E_ARG, "no communicator: call wr_comm_init first");
  if (root < 0 || root >= c->comm_ranks) return fail(WR_E_ARG, "bad root rank");
  DeviceGuard dg;
  HIPCHK(hipSetDevice(c->device));
  // ordered after the caller's work on the legacy null stream, like a render
  (void)hipEventRecord(c->t_null, nullptr);
  (void)hipStreamWaitEvent(c->stream, c->t_null, 0);
  NCCLCHK(rccl().reduce(film, film, static_cast<size_t>(nfloat), ncclFloat32, ncclSum, root, c->comm, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return WR_OK;
}

}  // extern "C"
