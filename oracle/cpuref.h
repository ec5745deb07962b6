/* cpuref -- CPU restatement of winmad/Winmad-s-raytracer-v1.0's BDPT / PT hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle: tests/, the smoke()
 * check in __graft_entry__.py and bench.py's cpu_baseline leg load it.  The
 * shipped renderer (winmad-s-raytracer-v1.0_amd/) never links or calls it.
 *
 * Pinned against the reference itself: oracle/_ref/refdrv (the reference's own
 * translation units, see oracle/Makefile) generated tests/golden/ fixtures; the
 * `-m "not gpu"` tests check this file against those fixtures bit for bit.
 *
 * Arithmetic mirrors the reference statement by statement (float, left-to-right,
 * no FMA contraction: build with -ffp-contract=off), so MT-serial mode replays the
 * reference's film exactly.  Counter mode swaps the single MT19937 stream for the
 * per-subpath counter RNG the HIP path uses (DESIGN.md "Counter RNG").
 */
#ifndef WINMAD_CPUREF_H
#define WINMAD_CPUREF_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cr_scene cr_scene;

enum { CR_RNG_MT = 0, CR_RNG_COUNTER = 1 };

typedef struct {
    int64_t closest_rays;  /* Scene::intersect traversals            */
    int64_t shadow_rays;   /* Scene::occluded traversals             */
    int64_t inner_visits;  /* KD inner nodes visited (all traversals) */
    int64_t leaf_visits;
    int64_t prim_refs;     /* leaf primitive references read          */
    int64_t tri_tests;     /* Triangle::hit calls inside traverse()   */
    int64_t sph_tests;
    double seconds;
    int64_t vm_queries;    /* VCM: KdTree::searchInRadius calls (camera vertices) */
    int64_t vm_found;      /* VCM: light vertices within the radius               */
    int64_t vm_merged;     /* VCM: RangeQuery::process merges (mergeNum)           */
    int64_t vm_emitter_first; /* VCM: light paths whose first vertex is an emitter
                                 (BSDF probabilities of the previous light path)      */
} cr_stats;

/* Load a .scene (scene.cpp:259-467) and build the KD tree (scene.cpp:469-489).
 * Returns NULL on error (message via cr_last_error). */
cr_scene* cr_scene_load(const char* path);
void cr_scene_free(cr_scene* s);
const char* cr_last_error(void);

int cr_scene_nobjs(const cr_scene* s);
int cr_scene_nlights(const cr_scene* s);
/* Text dump in the same format as `refdrv scene` (oracle/ref_driver.cpp). */
int cr_scene_dump(const cr_scene* s, const char* out_path);

/* Per ray (9 floats: origin, unnormalised dir, occlusion target):
 * Scene::intersect(Ray(o,d)) and Scene::occluded(o,d,target).
 * out_i[3*k] = prim (-1 miss), out_i[3*k+1] = inside, out_i[3*k+2] = matId,
 * out_f[7*k] = t, p(3), n(3), occ[k] = occluded.  Stats accumulate. */
void cr_trace(const cr_scene* s, const float* rays9, int64_t n, int32_t* out_i,
              float* out_f, uint8_t* occ, cr_stats* st);

/* BDPT (bidirPathTracing.cpp:5-665).  film: H*W*3 floats, film[x][y] layout of
 * ImageFilm (pre-transpose), ACCUMULATED (not scaled by 1/iterations).
 * Iterations [iter_begin, iter_begin + iterations).  Paths restricted to
 * [path_begin, path_end) (full frame: 0, W*H) -- used only to time a bounded
 * CPU sample.  control_length 3 = reference; <= 0 disables the length filter. */
/* debugging aid: log every traversal query (o, d, best t or -1, winner bits) */
void cr_set_ray_log(float* buf /* [cap][8] */, int64_t cap);
int64_t cr_ray_log_count(void);

int cr_render_bdpt(const cr_scene* s, int W, int H, int iter_begin, int iterations,
                   uint32_t seed, int rng_mode, int control_length, int64_t path_begin,
                   int64_t path_end, float* film, cr_stats* st);

/* VCM (vertexcm.cpp:47-285, KDtree.h): film[x][y] like BDPT, accumulated.
 * The reference: min 0, max 10, radius factor 0.003 (x sceneRadius), alpha 0.75,
 * iterations 1 (vertexcm.cpp:3-21).  The merge radius of iteration i (0-based,
 * global: iter_begin + k) is base / (i+1)^(0.5(1-alpha)) (:53-56). */
int cr_render_vcm(const cr_scene* s, int W, int H, int iter_begin, int iterations, uint32_t seed,
                  int rng_mode, int min_path_length, int max_path_length, float radius_factor,
                  float radius_alpha, int64_t path_begin, int64_t path_end, float* film, cr_stats* st);

/* PT (pathIntegrator.cpp:29-148 + surfaceIntegrator.cpp:14-46).  cr_render_pt:
 * all spp samples, film scaled by 1/spp.  cr_render_pt_samples: samples
 * [k_begin, k_begin + k_count) of the spp grid summed unscaled (one rank's
 * share of a sample-sharded render; counter RNG only unless the range is all). */
int cr_render_pt_samples(const cr_scene* s, int W, int H, int spp, int k_begin, int k_count, int max_depth,
                         uint32_t seed, int rng_mode, int64_t pix_begin, int64_t pix_end, float* film,
                         cr_stats* st);
int cr_render_pt(const cr_scene* s, int W, int H, int spp, int max_depth, uint32_t seed,
                 int rng_mode, int64_t pix_begin, int64_t pix_end, float* film, cr_stats* st);

/* PathIntegrator::raytracing per caller ray (rays6: o, d as given), counter RNG
 * stream (seed, sample, 2, k) from its first draw; out3: radiance per ray. */
int cr_pt_radiance(const cr_scene* s, const float* rays6, int64_t n, int max_depth, uint32_t seed,
                   uint32_t sample, float* out3, cr_stats* st);

/* Counter RNG (shared spec with the HIP path). */
uint64_t cr_stream_key(uint32_t seed, uint32_t iteration, uint32_t subpath, uint32_t path);
uint32_t cr_stream_u32(uint64_t key, uint32_t index);

/* MT19937 (rng.cpp) -- first n outputs for a seed. */
void cr_mt_outputs(uint32_t seed, int n, uint32_t* out);

/* Known-answer hooks for the component fixtures (tests/golden/kat_*). */
void cr_kat_sampler(const float* u, float power, float* out /* 3 cosh + pdf, 3 pcosh + pdf + pdf2 */);
void cr_kat_triangle(const float* u, const float* p012, float* out3);
void cr_kat_frame(const float* z, float* out9);
float cr_kat_fresnel(float cosi, float idx);
void cr_kat_strat(const float* u, int k, int tot, float* out3);
/* BSDF(wi, inter{n, matId}) then f / pdf / sample: returns valid flag.
 * out: isDelta, cosWi, contProb, fresnel, 4 probs, f(3), cosWo, dirPdf, revPdf,
 *      pdf(dir), pdf(rev), type, sample(3), wo(3), spdf, scos   (26 floats) */
int cr_kat_bsdf(const cr_scene* s, int matId, const float* n, const float* wi,
                const float* wo, const float* r3, float* out);
/* out: illuminance(3) dirToLight(3) dist dpdf epdf cal | emit(3) pos(3) dir(3) emp dpa cal
 *      | radiance(3) dpa epdf   (30 floats) */
void cr_kat_light(const cr_scene* s, int li, const float* pos, const float* r3,
                  const float* dr, const float* pr, const float* rd, float* out);
/* Point KD tree (KDtree.h:88-175) over pts[n][3]: per query, out4 = {found,
 * sum of found indices} by searchInRadius, then the same by brute force. */
void cr_kat_vkd(const float* pts, int n, const float* qs, int nq, float radius, int64_t* out4);
/* out: ray origin(3) dir(3), raster(3), check */
void cr_kat_camera(const cr_scene* s, float x, float y, const float* w, float* out10);

#ifdef __cplusplus
}
#endif
#endif
