/* cpuref CLI -- test infrastructure only (see cpuref.h).
 *   cpuref scene SCENE OUT.txt                         dump in refdrv format
 *   cpuref rays  SCENE CORPUS.f32                      like `refdrv rays`
 *   cpuref bdpt  SCENE W H ITERS SEED MODE OUT.f32 [CTL]
 *   cpuref pt    SCENE W H SPP DEPTH SEED MODE OUT.f32
 */
#include "cpuref.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static void hv(float x) { printf(" %a", (double)x); }

int main(int argc, char** argv) {
    if (argc < 3) { fprintf(stderr, "usage: see header\n"); return 2; }
    cr_scene* s = cr_scene_load(argv[2]);
    if (!s) { fprintf(stderr, "load failed: %s\n", cr_last_error()); return 1; }
    cr_stats st;
    memset(&st, 0, sizeof st);
    if (!strcmp(argv[1], "scene")) return cr_scene_dump(s, argv[3]);
    if (!strcmp(argv[1], "rays")) {
        FILE* f = fopen(argv[3], "rb");
        fseek(f, 0, SEEK_END);
        long n = ftell(f) / 36;
        fseek(f, 0, SEEK_SET);
        float* r = malloc(36 * n);
        if (fread(r, 36, n, f) != (size_t)n) return 1;
        fclose(f);
        int* oi = malloc(12 * n);
        float* of = malloc(28 * n);
        unsigned char* oc = malloc(n);
        cr_trace(s, r, n, oi, of, oc, &st);
        for (long k = 0; k < n; k++) {
            if (oi[3 * k] >= 0) {
                printf("%d", oi[3 * k]);
                for (int j = 0; j < 7; j++) hv(of[7 * k + j]);
                printf(" %d %d", oi[3 * k + 1], oi[3 * k + 2]);
            } else printf("-1");
            printf(" occ %d\n", oc[k]);
        }
        return 0;
    }
    if (!strcmp(argv[1], "bdpt") || !strcmp(argv[1], "pt")) {
        int W = atoi(argv[3]), H = atoi(argv[4]);
        float* film = calloc((size_t)W * H * 3, sizeof(float));
        int rc;
        const char* out;
        if (!strcmp(argv[1], "bdpt")) {
            int ctl = argc > 9 ? atoi(argv[9]) : 3;
            rc = cr_render_bdpt(s, W, H, 0, atoi(argv[5]), (unsigned)strtoul(argv[6], 0, 10), atoi(argv[7]), ctl,
                                0, (long long)W * H, film, &st);
            out = argv[8];
        } else {
            rc = cr_render_pt(s, W, H, atoi(argv[5]), atoi(argv[6]), (unsigned)strtoul(argv[7], 0, 10), atoi(argv[8]),
                              0, (long long)W * H, film, &st);
            out = argv[9];
        }
        if (rc) { fprintf(stderr, "%s\n", cr_last_error()); return 1; }
        FILE* f = fopen(out, "wb");
        fwrite(film, sizeof(float), (size_t)W * H * 3, f);
        fclose(f);
        printf("seconds %.4f closest %lld shadow %lld inner %lld leaves %lld refs %lld tris %lld\n", st.seconds,
               (long long)st.closest_rays, (long long)st.shadow_rays, (long long)st.inner_visits,
               (long long)st.leaf_visits, (long long)st.prim_refs, (long long)st.tri_tests);
        return 0;
    }
    return 2;
}
