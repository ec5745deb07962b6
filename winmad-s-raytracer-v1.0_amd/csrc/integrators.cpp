#include "integrators.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

namespace winmad {
namespace {
void ok(int rc) {
  if (rc != WR_OK) throw std::runtime_error(std::string("winmad_rt: ") + wr_last_error());
}
}  // namespace

void Parameters::load_parameters(const char* filename) {
  FILE* fp = std::fopen(filename, "r");
  if (!fp) throw std::runtime_error(std::string("cannot open parameter file ") + filename);
  int* slots[8] = {&MAX_TRACING_DEPTH, &SAMPLES_PER_PIXEL, &SAMPLES_OF_LIGHT, &SAMPLES_OF_HEMISPHERE,
                   &WIDTH, &HEIGHT, &PHONG_POWER_INDEX, &POINT_LIGHT_NUM};
  char tok[1024];
  int k = 0;
  while (k < 8 && std::fscanf(fp, "%1023s", tok) == 1) {
    if (tok[0] == '#') continue;  // read_int (parameters.cpp:9-20)
    *slots[k++] = std::atoi(tok);
  }
  for (; k < 8; ++k) *slots[k] = -1;  // read_int returns -1 at EOF
  std::fclose(fp);
}

SurfaceIntegrator::~SurfaceIntegrator() {
  if (ctx_) wr_destroy(ctx_);
  if (scene_) wr_scene_free(scene_);
}

void SurfaceIntegrator::load(const char* filename) {
  ok(wr_scene_load(filename, &scene_));
  if (devices.size() > 1)
    ok(wr_create_multi(scene_, devices.data(), static_cast<int>(devices.size()), &ctx_));
  else
    ok(wr_create(scene_, devices.empty() ? device : devices[0], &ctx_));
  if (traceMode >= 0) ok(wr_set_trace_mode(ctx_, traceMode));
  film.assign(static_cast<size_t>(height) * width * 3, 0.f);
  // the render's GPU work buffers now, as the reference's init allocates its
  // film and vertex arrays before render() (bidirPathTracing.cpp:5-21): the
  // render call then only renders
  if (reserveAtInit) ok(wr_reserve(ctx_, integrator_, width, height));
}

void SurfaceIntegrator::setTraceMode(int mode) {
  ok(wr_set_trace_mode(ctx_, mode));
  traceMode = mode;
}

void SurfaceIntegrator::reserve() { ok(wr_reserve(ctx_, integrator_, width, height)); }

// FNV-1a 64 of the scene's fingerprint and the integrator's settings: what a
// resumed film must have been rendered with, beyond the header's size, kind,
// total and seed
uint64_t SurfaceIntegrator::settingsHash(const std::vector<double>& settings) const {
  uint64_t scene = 0;
  ok(wr_scene_fingerprint(scene_, &scene));
  uint64_t h = 1469598103934665603ull;
  auto mix = [&h](const void* p, size_t n) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  };
  mix(&scene, sizeof scene);
  for (double v : settings) mix(&v, sizeof v);
  return h ? h : 1;  // 0 means "not recorded"
}

template <class Batch>
void SurfaceIntegrator::batched(int kind, int total, uint32_t seed, const std::vector<double>& settings, Batch batch) {
  int done = 0;
  stopped = false;
  const uint64_t fp = settingsHash(settings);
  wr_checkpoint_info want{width, height, kind, 0, total, seed, {uint32_t(fp), uint32_t(fp >> 32)}};
  if (!checkpointPath.empty()) {
    wr_checkpoint_info have{};
    if (FILE* f = std::fopen(checkpointPath.c_str(), "rb")) {  // resume
      std::fclose(f);
      ok(wr_checkpoint_load(checkpointPath.c_str(), &have, nullptr, 0));
      if (have.width != width || have.height != height || have.kind != kind || have.total != total ||
          have.seed != seed)
        throw std::runtime_error("checkpoint " + checkpointPath + " belongs to another render");
      // a film without a fingerprint (written before API v7, or saved with 0)
      // cannot be matched to a scene: refused like a foreign one
      if (have.fingerprint[0] == 0 && have.fingerprint[1] == 0)
        throw std::runtime_error("checkpoint " + checkpointPath +
                                 " carries no scene fingerprint (written before API v7 or without one); "
                                 "delete it to render from the start");
      if (have.fingerprint[0] != want.fingerprint[0] || have.fingerprint[1] != want.fingerprint[1])
        throw std::runtime_error("checkpoint " + checkpointPath +
                                 " was rendered from another scene or with other integrator settings");
      ok(wr_checkpoint_load(checkpointPath.c_str(), &have, film.data(), static_cast<int64_t>(film.size())));
      done = have.done;
    }
  }
  while (done < total) {
    int n = total - done;
    if (checkpointEvery > 0) n = std::min(n, checkpointEvery);
    if (stopAfter >= 0) n = std::min(n, stopAfter - done);
    if (n <= 0) {
      stopped = true;
      return;
    }
    batch(done, n);
    done += n;
    if (!checkpointPath.empty()) {
      want.done = done;
      ok(wr_checkpoint_save(checkpointPath.c_str(), &want, film.data()));
    }
  }
}

void BidirPathTracing::init(const char* filename, Parameters& para) {
  samplesPerPixel = para.SAMPLES_PER_PIXEL;  // stored, unused by BDPT (:11)
  integrator_ = WR_INTEGRATOR_BDPT;
  height = para.HEIGHT;
  width = para.WIDTH;
  load(filename);
}

void BidirPathTracing::render() {
  batched(WR_CKPT_BDPT, iterations, seed, {double(maxPathLength), double(controlLength)}, [&](int begin, int count) {  // :25-26
    wr_bdpt_params p{};
    p.width = width;
    p.height = height;
    p.iterations = count;
    p.iter_begin = begin;
    p.control_length = controlLength;
    p.max_path_length = maxPathLength;
    p.seed = seed;
    p.faithful = 1;
    ok(wr_render_bdpt(ctx_, &p, film.data(), 0, &stats));
  });
}

void BidirPathTracing::outputImage(const char* filename) {
  // The reference transposes in place assuming height == width (:31-44);
  // only square films are transposed here (non-square reference output is corrupt).
  ok(wr_film_write_image(film.data(), height, width, 1.f / iterations, 2.2f, height == width, filename));
}

void VertexCM::init(const char* filename, Parameters& para) {
  samplesPerPixel = para.SAMPLES_PER_PIXEL;  // stored, unused (:9)
  integrator_ = WR_INTEGRATOR_VCM;
  height = para.HEIGHT;
  width = para.WIDTH;
  load(filename);
}

void VertexCM::render() {
  batched(WR_CKPT_VCM, iterations, seed, {double(minPathLength), double(maxPathLength), double(baseRadiusFactor), double(radiusAlpha)}, [&](int begin, int count) {
    wr_vcm_params p{};
    p.width = width;
    p.height = height;
    p.iterations = count;
    p.iter_begin = begin;  // the merge radius follows the global iteration index (:53-58)
    p.min_path_length = minPathLength;
    p.max_path_length = maxPathLength;
    p.radius_factor = baseRadiusFactor;
    p.radius_alpha = radiusAlpha;
    p.seed = seed;
    ok(wr_render_vcm(ctx_, &p, film.data(), 0, &stats));
  });
}

void VertexCM::outputImage(const char* filename) {
  // transpose (square films only, :31-42), scale 1/iterations, gamma 2.2 (:44)
  ok(wr_film_write_image(film.data(), height, width, 1.f / iterations, 2.2f, height == width, filename));
}

void PathIntegrator::init(const char* filename, Parameters& para) {
  maxTracingDepth = para.MAX_TRACING_DEPTH;
  samplesPerPixel = para.SAMPLES_PER_PIXEL;
  samplesOfLight = para.SAMPLES_OF_LIGHT;
  samplesOfHemisphere = para.SAMPLES_OF_HEMISPHERE;
  integrator_ = WR_INTEGRATOR_PATH;
  height = para.HEIGHT;
  width = para.WIDTH;
  load(filename);
}

void PathIntegrator::render() {
  batched(WR_CKPT_PT, samplesPerPixel, seed, {double(maxTracingDepth), double(samplesOfLight), double(samplesOfHemisphere)}, [&](int begin, int count) {
    wr_path_params p{};
    p.width = width;
    p.height = height;
    p.spp = samplesPerPixel;
    p.max_depth = maxTracingDepth;
    p.sample_begin = begin;  // sample k of the stratification grid (surfaceIntegrator.cpp:26-32)
    p.sample_count = count;
    p.seed = seed;
    ok(wr_render_path(ctx_, &p, film.data(), 0, &stats));
  });
  if (stopped) return;
  const float inv = 1.f / samplesPerPixel;  // film->scale(1.f / samplesPerPixel) (:45)
  for (float& v : film) v = v * inv;
}

void PathIntegrator::raytracing(const wr_ray* rays, int64_t n, float* rgb, int sample) {
  ok(wr_path_radiance(ctx_, rays, n, maxTracingDepth, seed, sample, rgb, &stats));
}

void PathIntegrator::outputImage(const char* filename) {
  ok(wr_film_write_image(film.data(), height, width, 1.f, 2.2f, 0, filename));
}

}  // namespace winmad
