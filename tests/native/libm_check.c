/* libm_check.c -- test program: the product's glibc-equal cosf / sinf / powf
 * (winmad-s-raytracer-v1.0_amd/csrc/wr_libm.h, the functions the GPU kernels
 * call; cos / sin checks cover wr_cosf, wr_sinf and wr_sincosf) against the glibc libm of this machine, over the inputs the renderer
 * gives them.  Prints one JSON object; every "diff" must be 0.
 *
 *   libm_check sampler            cos/sin(2*PI*k/2^24), all 2^24 k
 *                                 (sampler.cpp:97-100,121-125)
 *   libm_check range LO HI [STEP] cos/sin of every (STEP-th) float x in [LO, HI]
 *                                 (LO >= 0) and of -x
 *   libm_check powexp E [STEP]    powf(c, E) for every (STEP-th) float c in (0, 1]
 *                                 (bsdf.cpp:99, sampler.cpp:123,135) and
 *                                 powf(k/2^24, 1/(E+1)) for all k (sampler.cpp:119)
 *   libm_check powrand N SEED     powf of N random (x, y) pairs over all floats
 *
 * Built by tests/test_libm.py (strided, CPU suite) and scripts/libm_check_full.sh
 * (every input, profiles/r6/libm_check.json) with gcc -O2 -ffp-contract=off.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../../winmad-s-raytracer-v1.0_amd/csrc/wr_libm.h"

static int same(float a, float b) {
  uint32_t ua = wr_lm_asuint(a), ub = wr_lm_asuint(b);
  if (ua == ub) return 1;
  return isnan(a) && isnan(b);
}

static void report(const char* what, unsigned long long n, unsigned long long diff, float first_x,
                   float first_y) {
  printf("{\"check\": \"%s\", \"n\": %llu, \"diff\": %llu", what, n, diff);
  if (diff) printf(", \"first_x\": %.9g, \"first_y\": %.9g", first_x, first_y);
  printf("}\n");
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const float PI = 3.14159274101257324f; /* (float)acos(-1.0), math.h:16 */
  if (!strcmp(argv[1], "sampler")) {
    unsigned long long dc = 0, ds = 0;
    float fx = 0;
    for (uint32_t k = 0; k < (1u << 24); ++k) {
      volatile float s = (float)k / 16777216.0f; /* rng.cpp:18-22 */
      float u1 = 2.f * PI * s;
      float sv, cv;
      wr_sincosf(u1, &sv, &cv);
      if (!same(wr_cosf(u1), cosf(u1)) || !same(cv, cosf(u1))) { if (!dc) fx = u1; ++dc; }
      if (!same(wr_sinf(u1), sinf(u1)) || !same(sv, sinf(u1))) { if (!ds) fx = u1; ++ds; }
    }
    report("cos_sampler", 1u << 24, dc, fx, 0);
    report("sin_sampler", 1u << 24, ds, fx, 0);
  } else if (!strcmp(argv[1], "range") && argc >= 4) {
    /* every STEP-th float x in [LO, HI] (LO >= 0), and -x */
    uint32_t lo = wr_lm_asuint(strtof(argv[2], 0)), hi = wr_lm_asuint(strtof(argv[3], 0));
    uint32_t step = argc >= 5 ? (uint32_t)strtoul(argv[4], 0, 10) : 1;
    unsigned long long n = 0, dc = 0, ds = 0;
    float fx = 0;
    for (uint64_t u = lo; u <= hi; u += step) {
      for (int sg = 0; sg < 2; ++sg) {
        float x = wr_lm_asfloat((uint32_t)u | (sg ? 0x80000000u : 0u));
        float sv, cv;
        wr_sincosf(x, &sv, &cv);
        ++n;
        if (!same(wr_cosf(x), cosf(x)) || !same(cv, cosf(x))) { if (!dc && !ds) fx = x; ++dc; }
        if (!same(wr_sinf(x), sinf(x)) || !same(sv, sinf(x))) { if (!dc && !ds) fx = x; ++ds; }
      }
    }
    report("cos_range", n, dc, fx, 0);
    report("sin_range", n, ds, fx, 0);
  } else if (!strcmp(argv[1], "powexp") && argc >= 3) {
    float e = strtof(argv[2], 0);
    uint32_t step = argc >= 4 ? (uint32_t)strtoul(argv[3], 0, 10) : 1;
    unsigned long long n = 0, d = 0;
    float fx = 0;
    for (uint32_t u = 1; u <= 0x3f800000u; u += step) {
      float c = wr_lm_asfloat(u);
      ++n;
      if (!same(wr_powf(c, e), powf(c, e))) { if (!d) fx = c; ++d; }
    }
    report("pow_cos", n, d, fx, e);
    float ie = 1.f / (e + 1.f);
    n = 0; d = 0;
    for (uint32_t k = 0; k < (1u << 24); ++k) {
      volatile float s = (float)k / 16777216.0f;
      ++n;
      if (!same(wr_powf(s, ie), powf(s, ie))) { if (!d) fx = s; ++d; }
    }
    report("pow_sampler", n, d, fx, ie);
  } else if (!strcmp(argv[1], "powrand") && argc >= 4) {
    unsigned long long N = strtoull(argv[2], 0, 10), d = 0;
    uint64_t st = strtoull(argv[3], 0, 10) * 0x9E3779B97F4A7C15ull + 1;
    float fx = 0, fy = 0;
    for (unsigned long long i = 0; i < N; ++i) {
      st ^= st << 13; st ^= st >> 7; st ^= st << 17;
      float x = wr_lm_asfloat((uint32_t)st), y = wr_lm_asfloat((uint32_t)(st >> 32));
      if ((i & 3) == 0) x = fabsf(x);                       /* half the x positive */
      if ((i & 7) < 4) y = wr_lm_asfloat(0x3c000000u + ((uint32_t)(st >> 40) % 0x07000000u)); /* |y| in [2^-7, 2^7) */
      if (!same(wr_powf(x, y), powf(x, y))) { if (!d) { fx = x; fy = y; } ++d; }
    }
    report("pow_random", N, d, fx, fy);
  } else {
    return 2;
  }
  return 0;
}
