// C++ host mirror of the reference's integrator seam, over the C ABI.
//
// The reference's drop-in point is SurfaceIntegrator
// (src/surfaceIntegrator/surfaceIntegrator.h:14-34): main() picks an integrator by
// flag and calls init(scene, para) / render() / outputImage(path)
// (src/main.cpp:40-45 for -p, :65-70 for -bpt).  These classes keep those names
// and that call order; the work happens on the GPU through include/winmad_rt.h.
// Where the reference would crash (missing scene, no lights) these throw
// std::runtime_error carrying wr_last_error().
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "winmad_rt.h"

namespace winmad {

// src/parameters.h / parameters.cpp:22-34 -- 8 positional ints, '#' lines skipped
class Parameters {
 public:
  int MAX_TRACING_DEPTH = 7, SAMPLES_PER_PIXEL = 1, SAMPLES_OF_LIGHT = 8, SAMPLES_OF_HEMISPHERE = 4;
  int WIDTH = 512, HEIGHT = 512, PHONG_POWER_INDEX = 5, POINT_LIGHT_NUM = 400;
  void load_parameters(const char* filename);
};

class SurfaceIntegrator {
 public:
  int width = 0, height = 0, samplesPerPixel = 0;
  int device = 0;
  std::vector<int> devices;  // more than one: the GPUs of this node share the render (wr_create_multi)
  bool reserveAtInit = true;  // init() allocates the render's work buffers (wr_reserve)
  int traceMode = -1;        // -1: the library's default (WR_TRACE_BVH for triangle scenes); WR_TRACE_REFERENCE / WR_TRACE_BVH
  // Film checkpoint (the reference keeps the film in memory only,
  // bidirPathTracing.cpp:23-27): with a path set, render() resumes from a
  // matching checkpoint and saves one every checkpointEvery iterations
  // (samples) and at the end.  stopAfter >= 0 stops once that many are done
  // (an interruption, for tests); `stopped` then says the film is partial.
  std::string checkpointPath;
  int checkpointEvery = 0;
  int stopAfter = -1;
  bool stopped = false;
  std::vector<float> film;  // ImageFilm color[height][width] (r, g, b)
  wr_stats stats{};
  virtual ~SurfaceIntegrator();
  virtual void init(const char* filename, Parameters& para) = 0;
  virtual void render() = 0;
  virtual void outputImage(const char* filename) = 0;
  // wr_set_trace_mode after init (throws, e.g. WR_TRACE_BVH on a scene with spheres)
  void setTraceMode(int mode);
  // wr_reserve after init / setTraceMode: the render's GPU buffers now, so that
  // render() only renders (init() already does it unless reserveAtInit is false;
  // render() allocates whatever is missing otherwise)
  void reserve();

 protected:
  int integrator_ = WR_INTEGRATOR_BDPT;  // set by init: what reserve() allocates for
  wr_scene* scene_ = nullptr;
  wr_context* ctx_ = nullptr;
  void load(const char* filename);
  // the render loop in batches: renders [done, total) through batch(begin, count),
  // resuming from / saving checkpoints of `kind`
  template <class Batch>
  void batched(int kind, int total, uint32_t seed, const std::vector<double>& settings, Batch batch);
  // hash of the scene (wr_scene_fingerprint) and `settings`: stored in the
  // checkpoint, a resume with another scene or settings is refused
  uint64_t settingsHash(const std::vector<double>& settings) const;
};

// src/surfaceIntegrator/bidirPathTracing.{h,cpp}
class BidirPathTracing : public SurfaceIntegrator {
 public:
  int minPathLength = 0, maxPathLength = 10, controlLength = 3;
  int iterations = 1;  // bidirPathTracing.cpp:9
  uint32_t seed = 5489;
  void init(const char* filename, Parameters& para) override;  // :5-21
  void render() override;                                        // :23-27
  void outputImage(const char* filename) override;               // :29-46
};

// src/surfaceIntegrator/vertexcm.{h,cpp}
class VertexCM : public SurfaceIntegrator {
 public:
  int minPathLength = 0, maxPathLength = 10;
  int iterations = 1;            // vertexcm.cpp:7
  float baseRadiusFactor = 0.003f;  // baseRadius = 0.003 * sceneRadius (:13)
  float radiusAlpha = 0.75f;     // :14
  uint32_t seed = 5489;
  void init(const char* filename, Parameters& para) override;  // :3-21
  void render() override;                                        // :23-27
  void outputImage(const char* filename) override;               // :29-45
};

// src/surfaceIntegrator/pathIntegrator.{h,cpp} + SurfaceIntegrator::render
class PathIntegrator : public SurfaceIntegrator {
 public:
  int maxTracingDepth = 7, samplesOfLight = 8, samplesOfHemisphere = 4;
  uint32_t seed = 5489;
  void init(const char* filename, Parameters& para) override;  // pathIntegrator.cpp:3-15
  void render() override;                                        // surfaceIntegrator.cpp:14-46
  void outputImage(const char* filename) override;               // surfaceIntegrator.cpp:47-50
  // raytracing(const Ray&, int dep) (pathIntegrator.cpp:29-148) for a batch of
  // rays; rgb: n * 3 radiance values (dep is unused by the reference)
  void raytracing(const wr_ray* rays, int64_t n, float* rgb, int sample = 0);
};

}  // namespace winmad
