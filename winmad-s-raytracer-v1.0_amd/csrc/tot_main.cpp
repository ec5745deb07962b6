// wr_tot -- command-line twin of the reference's main() (src/main.cpp:29-97) for
// the two GPU integrators:
//     wr_tot <scene> <out.ppm> -bpt|-vcm|-p [--params FILE] [--iterations N] [--seed S] [--device D]
// Parameters come from src/parameters.para relative to the CWD, as in the
// reference (main.cpp:32), unless --params is given.  Writes time.txt like
// main.cpp:93-95 (seconds instead of clock ticks).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>

#include "integrators.h"

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s <scene> <out.ppm> -bpt|-vcm|-p [--params F] [--iterations N] [--seed S] [--device D]\n",
                 argv[0]);
    return 2;
  }
  const char* params = "src/parameters.para";
  int iterations = 1, device = 0;
  unsigned seed = 5489;
  for (int i = 4; i + 1 < argc; i += 2) {
    if (!std::strcmp(argv[i], "--params")) params = argv[i + 1];
    else if (!std::strcmp(argv[i], "--iterations")) iterations = std::atoi(argv[i + 1]);
    else if (!std::strcmp(argv[i], "--seed")) seed = static_cast<unsigned>(std::strtoul(argv[i + 1], nullptr, 10));
    else if (!std::strcmp(argv[i], "--device")) device = std::atoi(argv[i + 1]);
  }
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
    integ->init(argv[1], para);
    integ->render();
    integ->outputImage(argv[2]);
    double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (FILE* f = std::fopen("time.txt", "w")) {
      std::fprintf(f, "time = %.6f s\n", sec);
      std::fclose(f);
    }
    const wr_stats& s = integ->stats;
    std::printf("rays %lld (closest %lld, shadow %lld) in %.3f s: %.2f Mrays/s\n",
                static_cast<long long>(s.closest_rays + s.shadow_rays), static_cast<long long>(s.closest_rays),
                static_cast<long long>(s.shadow_rays), s.seconds,
                (s.closest_rays + s.shadow_rays) / s.seconds * 1e-6);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  }
  return 0;
}
