/* winmad_rt.h -- C ABI of the MI355X-native BDPT / PT hot path.
 *
 * Drop-in boundary for winmad/Winmad-s-raytracer-v1.0 (paths below are relative
 * to /root/reference/Winmad-s-raytracer-v1.0/src).  The reference has no FFI;
 * its seam is the C++ class SurfaceIntegrator (surfaceIntegrator/surfaceIntegrator.h:14-34)
 * with Scene::intersect / Scene::occluded below it.  Each entry point names the
 * reference interface it replaces.  INTEGRATION.md shows the C++ / ctypes
 * bindings a maintainer adds on the reference side.
 *
 * Conventions (all functions):
 *   - return 0 on success, a negative WR_E* code on failure; never throw;
 *     the message of the last failure on this thread is wr_last_error();
 *   - plain pointers and sizes only; the caller owns every input / output buffer;
 *   - a wr_context is used by one host thread at a time; it owns its HIP streams
 *     on one device (wr_create) or on several (wr_create_multi).  Multi-GPU is
 *     either one process per GPU (wr_comm_* below) or one context over the
 *     node's GPUs (wr_create_multi); see DESIGN.md section 5.
 */
#ifndef WINMAD_RT_H
#define WINMAD_RT_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WR_API_VERSION 8

enum {
  WR_OK = 0,
  WR_E_ARG = -1,      /* bad argument                                  */
  WR_E_IO = -2,       /* scene / obj file unreadable or malformed      */
  WR_E_HIP = -3,      /* HIP runtime error (no device, OOM, launch)    */
  WR_E_SCENE = -4,    /* scene lacks what the call needs (lights, ...) */
  WR_E_NODEVICE = -5  /* the HIP extension found no gfx950 device       */
};

typedef struct wr_scene wr_scene;     /* host-side loaded scene + KD tree */
typedef struct wr_context wr_context; /* scene resident in HBM + stream  */

/* Ray (geometry/ray.h:6-32).  `d` is used as given: callers normalise it as
 * the Ray constructor does (ray.h:14-21).  The reference always has tmin = 0,
 * tmax = INF (1e7). */
typedef struct {
  float o[3];
  float d[3];
  float tmin, tmax;
} wr_ray; /* 32 bytes */

/* Intersection (geometry/intersection.h:6-19) + index of the winning primitive
 * in the reference's `Scene::objs` order (-1 = miss). */
typedef struct {
  float t;
  float p[3];
  float n[3];
  int32_t prim;
  int32_t inside;
  int32_t mat_id;
} wr_hit; /* 40 bytes */

typedef struct {
  int32_t nprims, ntriangles, nspheres, nlights, nmaterials;
  int32_t kd_depth_max;   /* depMax = int(1.2 ln N + 2) (KDtreeAccel.cpp:16) */
  int32_t kd_inner, kd_leaves;
  int64_t kd_refs;
  int32_t kd_max_stack;   /* traversal stack depth bound                    */
  int32_t missing_files;  /* .obj files the reference would silently skip   */
  float camera_xres, camera_yres;
  int64_t device_bytes;   /* bytes this scene occupies in HBM               */
} wr_scene_info;

/* BidirPathTracing knobs (bidirPathTracing.cpp:5-21). */
typedef struct {
  int32_t width, height;     /* Parameters WIDTH / HEIGHT; the film is height x width x 3   */
  int32_t iterations;        /* samples per pixel = iterations (hard-coded 1 in the reference) */
  int32_t iter_begin;        /* global index of the first iteration (RNG key; sharding)     */
  int32_t control_length;    /* 3 = reference filter; <= 0 accumulates every path length     */
  int32_t max_path_length;   /* 10 in the reference                                          */
  uint32_t seed;
  int32_t faithful;          /* 1: trace every ray the reference traces (default);
                                0: skip shadow rays whose contribution is filtered out       */
  int32_t time_kernels;      /* 1: HIP events around every launch -> wr_stats.kernel_ms      */
  int32_t count_work;        /* 1: per-traversal node / ref counters -> wr_stats              */
} wr_bdpt_params;

/* PathIntegrator knobs (pathIntegrator.cpp:3-15, parameters.para). */
typedef struct {
  int32_t width, height;
  int32_t spp;               /* SAMPLES_PER_PIXEL: the stratification grid (surfaceIntegrator.cpp:26-32) */
  int32_t max_depth;         /* MAX_TRACING_DEPTH                                          */
  int32_t sample_begin;      /* first sample index k rendered (RNG key; sharding), >= 0    */
  int32_t sample_count;      /* samples rendered by this call (0: spp - sample_begin);
                                negative, or sample_begin + sample_count > spp: WR_E_ARG    */
  uint32_t seed;
  int32_t time_kernels;
  int32_t count_work;
} wr_path_params;

/* VertexCM knobs (surfaceIntegrator/vertexcm.cpp:3-21, :47-66).  The merge
 * radius of global iteration i is
 *   max(radius_factor * sceneRadius / (i + 1)^(0.5 (1 - radius_alpha)), EPS). */
typedef struct {
  int32_t width, height;
  int32_t iterations;        /* hard-coded 1 in the reference (:7)                   */
  int32_t iter_begin;        /* global index of the first iteration (RNG key, radius) */
  int32_t min_path_length;   /* 0 in the reference                                    */
  int32_t max_path_length;   /* 10 in the reference; at most 10                      */
  float radius_factor;       /* 0.003: baseRadius = factor * sceneSphere.sceneRadius  */
  float radius_alpha;        /* 0.75                                                  */
  uint32_t seed;
  int32_t time_kernels;
  int32_t count_work;
} wr_vcm_params;

enum { WR_K_TRACE = 0, WR_K_SHADE = 1, WR_K_RESOLVE = 2, WR_K_GEN = 3, WR_K_OTHER = 4, WR_K_NUM = 8 };

typedef struct {
  int64_t closest_rays;      /* Scene::intersect traversals                 */
  int64_t shadow_rays;       /* Scene::occluded traversals                  */
  int64_t inner_visits;      /* count_work only                             */
  int64_t leaf_visits;
  int64_t prim_refs;         /* = triangle / sphere tests                   */
  double seconds;            /* host wall time of the call (stream synced)  */
  double kernel_ms[WR_K_NUM];      /* time_kernels only: summed launch durations */
  int64_t kernel_launches[WR_K_NUM];
  double trace_wall_ms;      /* time_kernels only: union of the traversal launch
                                intervals over all pipelines (launches overlap) */
  int64_t vm_queries;        /* VCM: range queries (KdTree::searchInRadius calls)  */
  int64_t vm_found;          /* VCM: light vertices found within the radius       */
  int64_t vm_merged;         /* VCM: RangeQuery::process merges (non-black BSDF)   */
  int64_t prim_tests;        /* count_work only: primitive tests run; < prim_refs
                                by the (ray, primitive) repeats skipped            */
  /* WR_TRACE_BVH only (wr_set_trace_mode), count_work: verified-BVH work.  The
   * KD counters above then cover only the fallback rays.                       */
  int64_t bvh_nodes;         /* BVH nodes visited (64-byte records)             */
  int64_t bvh_tests;         /* triangle tests of the BVH search                */
  int64_t kd_replay_steps;   /* KD path entries replayed (membership checks)    */
  int64_t fallback_rays;     /* rays handed to the faithful KD traversal        */
  /* WR_TRACE_BVH with env WR_BVH_VERIFY=1 (validation, slow): every ray is
   * traced again by the reference's KD walk and the two answers compared.     */
  int64_t verify_rays;
  int64_t verify_mismatches; /* (t, primitive) pairs that differ bit for bit      */
  int64_t pipelines;         /* render calls: the most concurrent pipelines one
                                device ran (API v6)                              */
  int64_t deferred_rays;     /* WR_TRACE_BVH BDPT: rays settled off the pipeline's
                                critical path, their paths shaded a step later
                                (deferred hard rays; API v6)        */
  int64_t bvh_width;         /* WR_TRACE_BVH: the search tree's width, 2 or 4 (4
                                from 2^18 triangles); 0: KD walk
                                (API v7)                                         */
  int64_t work_bytes;        /* render calls: device bytes of the work buffers the
                                pipelines of this call hold (API v8)              */
  int64_t work_paths;        /* ... and the paths they hold at once (buffer sets x
                                paths per set), so work_bytes / work_paths is the
                                memory per path in flight (API v8)               */
  int64_t redone;            /* BDPT: renders redone with smaller pieces because
                                a vertex pool or shadow queue sized by use filled
                                up (the film is the one of an unbounded render;
                                DESIGN.md 3; API v8)                              */
} wr_stats;

/* The reference's in-memory Scene (scene/scene.h:35-42) as flat host arrays,
 * for callers that build or already hold it instead of a .scene file.  The
 * caller keeps ownership; wr_scene_from_desc copies what it needs and builds
 * the KD tree (KDtreeAccel::init + buildTree, KDtreeAccel.cpp:12-307), so the
 * result is the scene wr_scene_load makes from a file with the same content. */
typedef struct {
  int32_t n_prims;             /* Scene::objs, in order (the KD tree's tie order)          */
  const int32_t* prim_type;    /* 0 Triangle (triangle.h:14-31), 1 Sphere (sphere.h:16-21) */
  const float* prim_data;      /* 9 floats each: triangle p0 p1 p2; sphere centre xyz, radius, 5 unused */
  const int32_t* prim_mat;     /* matId: >= 0 materials[]; < 0 emitter of AreaLight -matId-1
                                  (scene.cpp:412-427); 0 = black, ends paths                  */
  int32_t n_lights;            /* Scene::lights: AreaLight(p0, p1, p2, intensity) (light.h:90-103) */
  const float* light_tri;      /* 9 floats each: p0 p1 p2                                    */
  const float* light_le;       /* 3 floats each: intensity (RGB)                             */
  int32_t n_materials;         /* Scene::materials (material.h:7-31)                          */
  const float* materials;      /* 11 floats each: diffuse rgb, phong rgb, specular rgb, phongExp, refracIndex */
  float cam_pos[3], cam_fwd[3], cam_up[3]; /* Camera::setup (camera.cpp:3-29); fwd / up normalised there */
  float cam_xres, cam_yres;    /* raster size; the reference takes xRes from the XML height (scene.cpp:292-295) */
  float cam_hfov;              /* horizontal field of view, degrees                          */
} wr_scene_desc;

/* ---- scene (Scene::init, scene/scene.cpp:469-489 + loadScene :259-467) ---- */
int wr_scene_load(const char* scene_path, wr_scene** out);
/* Scene::init from the in-memory arrays above (WR_E_ARG on a malformed desc:
 * null arrays, bad type, an emitter matId without its light). */
int wr_scene_from_desc(const wr_scene_desc* desc, wr_scene** out);
int wr_scene_info_get(const wr_scene* scene, wr_scene_info* out);
/* 64-bit FNV-1a of what a render reads from the scene (primitives, lights,
 * materials, camera).  Checkpoints store it (with the integrator's settings)
 * so that a film is never resumed into a render of another scene. */
int wr_scene_fingerprint(const wr_scene* scene, uint64_t* out);
/* Text dump in the format of oracle/ref_driver.cpp `scene` (parity tests). */
int wr_scene_dump(const wr_scene* scene, const char* out_path);
void wr_scene_free(wr_scene* scene);

/* ---- device context ---- */
int wr_device_count(void);
int wr_create(const wr_scene* scene, int hip_device, wr_context** out);
/* Several GPUs of one node behind one context: the scene is uploaded to each
 * of devices[0..n) and every later call is shared out --
 *   wr_render_bdpt: equal contiguous shares of the render's path-iterations
 *     (iteration-major; one iteration still spreads over every device),
 *   wr_render_vcm: contiguous iteration ranges (a merge grid per iteration),
 *   wr_render_path: contiguous sample ranges of the spp grid,
 *   wr_trace_closest / wr_occluded: contiguous ray ranges;
 *   wr_path_radiance runs on devices[0].
 * The devices render concurrently into films of their own, which are summed on
 * devices[0] by one RCCL reduce over xGMI (a device listed twice, or env
 * WR_MULTI_REDUCE=peer: peer copies + an add kernel), then returned like a
 * single-device render (a device film lives on devices[0]).  The reference's
 * render loop over iterations (bidirPathTracing.cpp:25-26) is what is shared
 * out; the result equals one device's up to float summation order. */
int wr_create_multi(const wr_scene* scene, const int* hip_devices, int n_devices, wr_context** out);
/* Devices of a context (devices[0] first); returns their number, writes up to max_n. */
int wr_context_devices(const wr_context* ctx, int* devices, int max_n);
void wr_destroy(wr_context* ctx);

/* ---- one process per GPU: each rank renders its own
 * iterations into a device film; one reduce(sum) of the films over RCCL per
 * sample batch.  Rank 0 calls wr_comm_unique_id and hands the 128 bytes to the
 * other ranks (any channel: MPI, a file, torch.distributed); every rank then
 * calls wr_comm_init on its context. */
int wr_comm_unique_id(uint8_t id[128]);
int wr_comm_init(wr_context* ctx, const uint8_t id[128], int nranks, int rank);
/* Sum the ranks' device films (nfloat floats on the context's device) into
 * rank `root`'s film, in place; collective (every rank calls it).  Ordered
 * after the caller's work on the legacy null stream; returns when done. */
int wr_film_reduce(wr_context* ctx, float* film_dev, int64_t nfloat, int root);
/* The communicator's size and this rank, read back from RCCL (ncclCommCount,
 * ncclCommUserRank): a bench or driver checks the job really spans N ranks. */
int wr_comm_info(const wr_context* ctx, int* nranks, int* rank);
/* Concurrent render pipelines (HIP streams, each with its own work buffers,
 * ~5 GB per pair of iterations at 1080p): iterations / samples are dealt
 * round-robin to them so that one stream's late-bounce traversal tail overlaps
 * another's full launches.  1..16; default = the process's hardware queues
 * (GPU_MAX_HW_QUEUES, read when wr_create runs) up to 16, or env WR_PIPES.
 * GPU-specific scheduling; no reference counterpart. */
int wr_set_pipelines(wr_context* ctx, int n);
/* Ask HIP for n hardware queues (1..32) -- one per render pipeline -- by
 * raising GPU_MAX_HW_QUEUES to n (a larger value already set is kept).  HIP
 * reads the variable once, when it initialises: call this at the top of main(),
 * before the process's first HIP call and before other threads start (it
 * writes the process environment).  Returns the queue count in effect for
 * contexts created later, or WR_E_ARG.  The library never changes the
 * environment otherwise (API v8). */
int wr_request_hw_queues(int n);

/* Allocate now what renders of this integrator and film size on the context
 * will use -- every pipeline's work buffers (each device of a multi-device
 * context) -- instead of inside the first render call.  Optional; the
 * counterpart of the allocations SurfaceIntegrator::init makes before render()
 * (surfaceIntegrator/surfaceIntegrator.h:14-34).  Call after wr_set_pipelines /
 * wr_set_trace_mode (API v6). */
enum { WR_INTEGRATOR_BDPT = 0, WR_INTEGRATOR_VCM = 1, WR_INTEGRATOR_PATH = 2 };
int wr_reserve(wr_context* ctx, int integrator, int32_t width, int32_t height);

/* Traversal mode of every later call on the context.
 *   WR_TRACE_REFERENCE: the reference's KD tree, walked exactly as
 *     KDtreeAccel::traverse (scene/KDtreeAccel.cpp:309-388) walks it.
 *   WR_TRACE_BVH (default): a BVH search over the triangles and spheres for
 *     the smallest hit, accepted only when the winner is provably the
 *     reference's (unique within EPS, in a KD leaf the reference's traversal
 *     reaches, the ray not grazing a tested triangle's plane, its origin inside
 *     the region the sphere boxes are grown for); every other ray is traced in
 *     the reference mode.  Same rays, same (t, primitive) answers; see
 *     DESIGN.md 4b.  (Spheres: API v8.)
 * Env WR_TRACE_BVH=0 / 1 sets the mode at wr_create. */
enum { WR_TRACE_REFERENCE = 0, WR_TRACE_BVH = 1 };
int wr_set_trace_mode(wr_context* ctx, int mode);

/* ---- traversal ---- */
/* Scene::intersect (scene/scene.cpp:21-43) -> KDtreeAccel::traverse
 * (scene/KDtreeAccel.cpp:309-388).  Host arrays of n rays / hits. */
int wr_trace_closest(wr_context* ctx, const wr_ray* rays, int64_t n, wr_hit* hits);
/* Scene::occluded (scene/scene.cpp:55-81): a closest-hit traversal of
 * Ray(o, d) (d re-normalised as the Ray constructor does) whose answer is
 * "not occluded" iff it misses or its hit point equals targets[3k..3k+2]
 * within EPS per component. */
int wr_occluded(wr_context* ctx, const wr_ray* rays, const float* targets, int64_t n, uint8_t* occluded);

/* ---- integrators ---- */
/* BidirPathTracing::render (surfaceIntegrator/bidirPathTracing.cpp:23-27,
 * runIteration :53-265).  film: height*width*3 floats in ImageFilm layout
 * film[x_raster][y_raster] (pre-transpose), accumulated (+=), NOT scaled by
 * 1/iterations.  film_on_device != 0: `film` is a device pointer on the
 * context's device.  The render is ordered after all work submitted before the
 * call on the legacy null stream (torch's default stream); work on another
 * caller stream that writes the film must be synchronized by the caller first.
 * The call returns once the film holds the result (all streams synchronized). */
int wr_render_bdpt(wr_context* ctx, const wr_bdpt_params* p, float* film, int film_on_device, wr_stats* stats);
/* SurfaceIntegrator::render (surfaceIntegrator.cpp:14-46) + PathIntegrator::raytracing
 * (pathIntegrator.cpp:29-148).  film[height][width][3] accumulates the per-sample
 * radiance SUM (the reference's final film->scale(1/spp) is left to the caller). */
int wr_render_path(wr_context* ctx, const wr_path_params* p, float* film, int film_on_device, wr_stats* stats);

/* PathIntegrator::raytracing(const Ray& ray, int dep) (pathIntegrator.cpp:29-148),
 * the per-sample estimator SurfaceIntegrator::render calls, for a batch of
 * caller rays (o and d used as given, like a constructed Ray; tmin / tmax
 * ignored: the reference traces with 0 / INF).  rgb: n*3 floats, overwritten
 * with the radiance of each ray.  Ray k draws from the counter-RNG stream
 * (seed, sample, 2, k) -- the PT render's streams skip that stream's first
 * draw, which stratifies the pixel sample.  `dep` is unused by the reference
 * and has no counterpart. */
int wr_path_radiance(wr_context* ctx, const wr_ray* rays, int64_t n, int32_t max_depth, uint32_t seed,
                     int32_t sample, float* rgb, wr_stats* stats);

/* VertexCM::render (surfaceIntegrator/vertexcm.cpp:23-27, runIteration :47-285):
 * vertex connection + vertex merging.  The reference's point KD tree over the
 * light vertices (scene/KDtree.h) is replaced by a hash grid: searchInRadius
 * reports exactly the vertices with |x - v| < radius, and so does the grid.
 * film as wr_render_bdpt (pre-transpose, accumulated, not scaled). */
int wr_render_vcm(wr_context* ctx, const wr_vcm_params* p, float* film, int film_on_device, wr_stats* stats);

/* ---- output (ImageFilm::outputImage, scene/film.cpp:39-64; BDPT transpose
 * bidirPathTracing.cpp:29-46) ---- scale -> clamp [0,1] -> pow(1/gamma) ->
 * (uchar)(x*255.0); binary PPM (RGB).  transpose != 0 swaps [i][j] <-> [j][i]
 * first (square films only, as the reference). */
int wr_film_write_ppm(const float* film, int height, int width, float scale, float gamma, int transpose,
                      const char* path);
/* The same pipeline into the format the path's extension names, as the
 * reference's cvSaveImage(filename) does (film.cpp:63): .ppm, .bmp (24-bit),
 * .png (8-bit RGB); .pfm writes the scaled linear floats (no clamp / gamma).
 * Other extensions: WR_E_ARG. */
int wr_film_write_image(const float* film, int height, int width, float scale, float gamma, int transpose,
                        const char* path);

/* ---- film checkpoint / resume.  The reference keeps the film in
 * memory only while it loops over iterations (bidirPathTracing.cpp:23-27).
 * Iterations / samples are keyed by their global index, so a render resumes
 * exactly: load the film, render the indices [done, total) (iter_begin /
 * sample_begin = done) into it.  The file carries the accumulated, unscaled
 * film and a checksum; it is replaced atomically (write + rename). */
enum { WR_CKPT_BDPT = 1, WR_CKPT_VCM = 2, WR_CKPT_PT = 3 };
typedef struct {
  int32_t width, height;
  int32_t kind;         /* WR_CKPT_*                                         */
  int32_t done, total;  /* iterations (samples) summed in the film / wanted */
  uint32_t seed;
  uint32_t fingerprint[2]; /* (lo, hi) of a 64-bit hash of the scene
                              (wr_scene_fingerprint) and the integrator's
                              settings, set by the writer; a resume whose
                              own hash differs is refused.  0 = not recorded:
                              the C++ mirror (csrc/integrators.h) refuses such
                              a film too, e.g. one written before API v7 */
} wr_checkpoint_info; /* 32 bytes */
int wr_checkpoint_save(const char* path, const wr_checkpoint_info* info, const float* film);
/* film == NULL reads the header only; else film_floats must be height*width*3.
 * WR_E_IO for a missing, foreign, truncated or corrupt file. */
int wr_checkpoint_load(const char* path, wr_checkpoint_info* info, float* film, int64_t film_floats);

const char* wr_last_error(void);
int wr_api_version(void);

#ifdef __cplusplus
}
#endif
#endif /* WINMAD_RT_H */
