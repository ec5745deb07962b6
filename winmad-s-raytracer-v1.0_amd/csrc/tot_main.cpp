// wr_tot -- command-line twin of the reference's main() (src/main.cpp:29-97) for
// the GPU integrators:
//     wr_tot <scene> <out.ppm> -bpt|-vcm|-p [--params FILE] [--iterations N] [--seed S]
//            [--device D | --gpus N | --devices D0,D1,...] [--trace bvh|reference]
//            [--checkpoint FILE [--checkpoint-every N] [--stop-after N]] [--hw-queues N]
// Parameters come from src/parameters.para relative to the CWD, as in the
// reference (main.cpp:32), unless --params is given.  Writes time.txt like
// main.cpp:93-95 (seconds instead of clock ticks).
//
// Runs at the configuration bench.py measures: 16 hardware queues for the 16
// render pipelines (HIP and the GPU box default to 4; raised here before the
// first HIP call -- no re-exec), and the verified-BVH traversal for triangle
// scenes (--trace reference: the reference's KD walk; scenes with spheres
// always use it).  --gpus / --devices share the render over several GPUs of the
// node (wr_create_multi); --checkpoint resumes an interrupted render.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "integrators.h"

namespace {
std::vector<int> parse_list(const char* s) {
  std::vector<int> v;
  for (const char* p = s; *p;) {
    char* end = nullptr;
    v.push_back(static_cast<int>(std::strtol(p, &end, 10)));
    if (end == p) throw std::runtime_error(std::string("bad device list ") + s);
    p = (*end == ',') ? end + 1 : end;
  }
  return v;
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr,
                 "usage: %s <scene> <out.ppm> -bpt|-vcm|-p [--params F] [--iterations N] [--seed S] "
                 "[--device D | --gpus N | --devices D0,D1,..] [--trace bvh|reference] "
                 "[--checkpoint F [--checkpoint-every N] [--stop-after N]] [--hw-queues N]\n",
                 argv[0]);
    return 2;
  }
  const char* params = "src/parameters.para";
  const char* checkpoint = nullptr;
  int iterations = 1, device = 0, gpus = 0, every = 0, stop_after = -1, hw_queues = 16;
  std::vector<int> devices;
  unsigned seed = 5489;
  bool bvh = true;
  try {
    for (int i = 4; i + 1 < argc; i += 2) {
      const char* a = argv[i];
      const char* v = argv[i + 1];
      if (!std::strcmp(a, "--params")) params = v;
      else if (!std::strcmp(a, "--iterations")) iterations = std::atoi(v);
      else if (!std::strcmp(a, "--seed")) seed = static_cast<unsigned>(std::strtoul(v, nullptr, 10));
      else if (!std::strcmp(a, "--device")) device = std::atoi(v);
      else if (!std::strcmp(a, "--gpus")) gpus = std::atoi(v);
      else if (!std::strcmp(a, "--devices")) devices = parse_list(v);
      else if (!std::strcmp(a, "--trace")) bvh = std::strcmp(v, "reference") != 0;
      else if (!std::strcmp(a, "--checkpoint")) checkpoint = v;
      else if (!std::strcmp(a, "--checkpoint-every")) every = std::atoi(v);
      else if (!std::strcmp(a, "--stop-after")) stop_after = std::atoi(v);
      else if (!std::strcmp(a, "--hw-queues")) hw_queues = std::atoi(v);
      else throw std::runtime_error(std::string("unknown option ") + a);
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 2;
  }
  // before any HIP call: one hardware queue per render pipeline
  if (wr_request_hw_queues(hw_queues) < 0) {
    std::fprintf(stderr, "%s\n", wr_last_error());
    return 2;
  }
  if (gpus > 0 && devices.empty())
    for (int k = 0; k < gpus; ++k) devices.push_back(k);
  try {
    winmad::Parameters para;
    para.load_parameters(params);
    auto t0 = std::chrono::steady_clock::now();
    std::unique_ptr<winmad::SurfaceIntegrator> integ;
    if (!std::strcmp(argv[3], "-bpt")) {
      auto* b = new winmad::BidirPathTracing();
      b->iterations = iterations;
      b->seed = seed;
      integ.reset(b);
    } else if (!std::strcmp(argv[3], "-vcm")) {  // main.cpp:53-58
      auto* v = new winmad::VertexCM();
      v->iterations = iterations;
      v->seed = seed;
      integ.reset(v);
    } else if (!std::strcmp(argv[3], "-p")) {
      auto* p = new winmad::PathIntegrator();
      p->seed = seed;
      integ.reset(p);
    } else {
      std::printf("error!\n");  // main.cpp:88-91
      return 1;
    }
    integ->device = device;
    integ->devices = devices;
    integ->traceMode = WR_TRACE_REFERENCE;
    if (checkpoint) {
      integ->checkpointPath = checkpoint;
      integ->checkpointEvery = every;
      integ->stopAfter = stop_after;
    }
    integ->init(argv[1], para);
    if (bvh) {  // the verified BVH traversal where the scene allows it (triangles only)
      try {
        integ->setTraceMode(WR_TRACE_BVH);
      } catch (const std::exception&) {
        bvh = false;
      }
    }
    integ->reserve();  // the GPU work buffers, before the render (as init's allocations in the reference)
    integ->render();
    if (integ->stopped) {
      std::printf("stopped after --stop-after %d; checkpoint %s\n", stop_after, checkpoint);
      return 0;
    }
    integ->outputImage(argv[2]);
    double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (FILE* f = std::fopen("time.txt", "w")) {
      std::fprintf(f, "time = %.6f s\n", sec);
      std::fclose(f);
    }
    const wr_stats& s = integ->stats;
    std::printf("rays %lld (closest %lld, shadow %lld) in %.3f s: %.2f Mrays/s [trace %s, %zu GPU(s)]\n",
                static_cast<long long>(s.closest_rays + s.shadow_rays), static_cast<long long>(s.closest_rays),
                static_cast<long long>(s.shadow_rays), s.seconds,
                (s.closest_rays + s.shadow_rays) / s.seconds * 1e-6, bvh ? "bvh" : "reference",
                devices.size() > 1 ? devices.size() : size_t(1));
  } catch (const std::exception& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  }
  return 0;
}
