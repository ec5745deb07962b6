// Test infrastructure only (see ref_driver.cpp): the `vcm` command lives in its
// own translation unit because vertexcm.h and bidirPathTracing.h both define a
// file-scope `static FILE* fp` (vertexcm.h:10, bidirPathTracing.cpp's header),
// so they cannot be included together.
//
//   refdrv vcm SCENE PARA ITERS SEED OUT.f32 [RADIUS_FACTOR]
//       VertexCM::render, film pre-transpose.  RADIUS_FACTOR replaces init's 0.003
//       (vertexcm.cpp:13) through the public member baseRadius, so small test
//       films see enough merges.
#include "surfaceIntegrator/vertexcm.h"
#include <ctime>
#include <cstdlib>

int refdrv_vcm(int argc, char** argv, Parameters& para) {
    if (argc < 7) { fprintf(stderr, "usage: refdrv vcm SCENE PARA ITERS SEED OUT.f32\n"); return 2; }
    VertexCM* v = new VertexCM();
    v->init(argv[2], para);
    v->iterations = atoi(argv[4]);
    v->rng.seed((uint32_t)strtoul(argv[5], 0, 10));
    if (argc > 7) v->baseRadius = (float)atof(argv[7]) * v->scene.sceneSphere.sceneRadius;
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    v->render();
    clock_gettime(CLOCK_MONOTONIC, &b);
    FILE* f = fopen(argv[6], "wb");
    for (int i = 0; i < v->film->height; i++)
        for (int j = 0; j < v->film->width; j++) {
            float c[3] = {v->film->color[i][j].r, v->film->color[i][j].g, v->film->color[i][j].b};
            fwrite(c, sizeof(float), 3, f);
        }
    fclose(f);
    printf("render_seconds %.6f\n", (b.tv_sec - a.tv_sec) + 1e-9 * (b.tv_nsec - a.tv_nsec));
    return 0;
}
