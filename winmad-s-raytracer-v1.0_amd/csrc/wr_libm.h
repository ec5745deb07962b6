/* wr_libm.h -- cosf / sinf / powf giving the same float, bit for bit, as the
 * glibc 2.35 x86-64 libm the reference links against.
 *
 * The reference takes every sampled direction and every Phong lobe through
 * libm: std::cos / std::sin of a float (sampler/sampler.cpp:100,123,125 ->
 * cosf / sinf) and std::pow of two floats (sampler.cpp:119,123,135,
 * material/bsdf.cpp:99 -> powf).  OCML's cosf / sinf / powf round differently
 * now and then, and a direction one ulp off sends a path elsewhere, so the GPU
 * film could only match the CPU film statistically.  These functions restate
 * the algorithms glibc 2.35 ships for the three calls (the Arm optimized-
 * routines single-precision code: sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c,
 * sincosf.h, sincosf_data.c, e_powf.c, e_powf_log2_data.c, e_exp2f_data.c):
 * the argument is widened to double, reduced, run through a short double
 * polynomial (a 16-entry log2 table and a 32-entry exp2 table for powf) and
 * rounded to float once.
 *
 * On x86-64 glibc picks, through an ifunc, the build of these files compiled
 * with -mfma -mavx2 (__sinf_fma, __cosf_fma, __powf_fma) whenever the CPU has
 * FMA -- every machine this project runs on.  GCC contracts each `a * b + c`
 * of that source into one fused multiply-add; the code below writes those
 * contractions out with an explicit fma() and leaves every other operation a
 * separately rounded double op (the translation units that include it are
 * built with -ffp-contract=off).  The table constants were checked against
 * the data of the libm in this image.
 *
 * Proof of equality: tests/native/libm_check.c runs these functions beside
 * glibc's over every input the renderer can give them (cos / sin of
 * 2*PI*k/2^24 for all 2^24 k, powf of every sampler value and of every float
 * cosine to the scenes' Phong exponents), every float in [-256, 256] and a
 * stride of all larger ones: 1.06e10 comparisons, 0 differences
 * (scripts/libm_check_full.sh -> profiles/r6/libm_check.json; a strided run
 * is the CPU test tests/test_libm.py).
 *
 * Usable from C (the CPU check, compiled with gcc) and from HIP device code.
 */
#ifndef WR_LIBM_H
#define WR_LIBM_H
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define WR_LIBM_FN __host__ __device__ static inline
#else
#define WR_LIBM_FN static inline
#endif

#define WR_LM_FMA(a, b, c) __builtin_fma((a), (b), (c))

WR_LIBM_FN uint32_t wr_lm_asuint(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  return u;
}
WR_LIBM_FN float wr_lm_asfloat(uint32_t u) {
  float f;
  __builtin_memcpy(&f, &u, 4);
  return f;
}
WR_LIBM_FN uint64_t wr_lm_asuint64(double f) {
  uint64_t u;
  __builtin_memcpy(&u, &f, 8);
  return u;
}
WR_LIBM_FN double wr_lm_asdouble(uint64_t u) {
  double f;
  __builtin_memcpy(&f, &u, 8);
  return f;
}

/* ------------------------------------------------------------------ sin/cos */
/* Top 12 bits of a float with the sign cleared (sincosf.h abstop12). */
WR_LIBM_FN uint32_t wr_lm_abstop12(float x) { return (wr_lm_asuint(x) >> 20) & 0x7ff; }

/* Cosine polynomial c0..c4 and sine polynomial s1..s3 (sincosf_data.c);
 * the second set is the first with the cosine polynomial negated, used for
 * quadrants 2 and 3. */
#define WR_SC_HPI_INV 0x1.45f306dc9c883p+23 /* 2/PI * 2^24 */
#define WR_SC_HPI 0x1.921fb54442d18p+0      /* PI/2 */
#define WR_SC_PI63 0x1.921fb54442d18p-62    /* 2PI * 2^-64 */
#define WR_SC_C0 0x1p0
#define WR_SC_C1 -0x1.ffffffd0c621cp-2
#define WR_SC_C2 0x1.55553e1068f19p-5
#define WR_SC_C3 -0x1.6c087e89a359dp-10
#define WR_SC_C4 0x1.99343027bf8c3p-16
#define WR_SC_S1 -0x1.555545995a603p-3
#define WR_SC_S2 0x1.1107605230bc4p-7
#define WR_SC_S3 -0x1.994eb3774cf24p-13

/* sincosf.h sinf_poly: sine polynomial for even n, cosine polynomial for odd
 * n; neg selects the negated cosine set. */
WR_LIBM_FN float wr_lm_sinf_poly(double x, double x2, int neg, int n) {
  if ((n & 1) == 0) {
    double x3 = x * x2;
    double s1 = WR_LM_FMA(x2, WR_SC_S3, WR_SC_S2);
    double x7 = x3 * x2;
    double s = WR_LM_FMA(x3, WR_SC_S1, x);
    return (float)WR_LM_FMA(x7, s1, s);
  } else {
    double c0 = neg ? -WR_SC_C0 : WR_SC_C0, c1 = neg ? -WR_SC_C1 : WR_SC_C1;
    double c2 = neg ? -WR_SC_C2 : WR_SC_C2, c3 = neg ? -WR_SC_C3 : WR_SC_C3;
    double c4 = neg ? -WR_SC_C4 : WR_SC_C4;
    double x4 = x2 * x2;
    double cc2 = WR_LM_FMA(x2, c4, c3);
    double cc1 = WR_LM_FMA(x2, c1, c0);
    double x6 = x4 * x2;
    double c = WR_LM_FMA(x4, c2, cc1);
    return (float)WR_LM_FMA(x6, cc2, c);
  }
}

/* sincosf.h reduce_fast: one multiply-subtract, |x| < 120.  The quadrant is
 * taken from 2/PI * 2^24 by an int conversion with explicit rounding. */
WR_LIBM_FN double wr_lm_reduce_fast(double x, int* np) {
  double r = x * WR_SC_HPI_INV;
  int n = ((int32_t)r + 0x800000) >> 24;
  *np = n;
  return WR_LM_FMA(-(double)n, WR_SC_HPI, x);
}

/* sincosf.h reduce_large: 4/PI to 192 bits (the bits of 2/PI shifted by a
 * byte per entry), 32x64-bit integer products. */
WR_LIBM_FN double wr_lm_reduce_large(uint32_t xi, int* np) {
  const uint32_t inv_pio4[24] = {
      0xa2u,       0xa2f9u,     0xa2f983u,   0xa2f9836eu, 0xf9836e4eu, 0x836e4e44u,
      0x6e4e4415u, 0x4e441529u, 0x441529fcu, 0x1529fc27u, 0x29fc2757u, 0xfc2757d1u,
      0x2757d1f5u, 0x57d1f534u, 0xd1f534ddu, 0xf534ddc0u, 0x34ddc0dbu, 0xddc0db62u,
      0xc0db6295u, 0xdb629599u, 0x6295993cu, 0x95993c43u, 0x993c4390u, 0x3c439041u};
  const uint32_t* arr = &inv_pio4[(xi >> 26) & 15];
  int shift = (xi >> 23) & 7;
  uint64_t n, res0, res1, res2;
  xi = (xi & 0xffffff) | 0x800000;
  xi <<= shift;
  res0 = (uint32_t)(xi * arr[0]);
  res1 = (uint64_t)xi * arr[4];
  res2 = (uint64_t)xi * arr[8];
  res0 = (res2 >> 32) | (res0 << 32);
  res0 += res1;
  n = (res0 + (1ULL << 61)) >> 62;
  res0 -= n << 62;
  double x = (double)(int64_t)res0;
  *np = (int)n;
  return x * WR_SC_PI63;
}

/* s_sinf.c */
WR_LIBM_FN float wr_sinf(float y) {
  double x = y;
  int n;
  const uint32_t top = wr_lm_abstop12(y);
  if (top < 0x3f4) { /* abstop12(pio4) */
    double s = x * x;
    if (top < 0x398) return y; /* |y| < 0x1p-12: sin y = y */
    return wr_lm_sinf_poly(x, s, 0, 0);
  } else if (top < 0x42f) { /* |y| < 120 */
    x = wr_lm_reduce_fast(x, &n);
    double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;
    return wr_lm_sinf_poly(x * s, x * x, (n & 2) != 0, n);
  } else if (top < 0x7f8) {
    uint32_t xi = wr_lm_asuint(y);
    int sign = (int)(xi >> 31);
    x = wr_lm_reduce_large(xi, &n);
    int q = (n + sign) & 3;
    double s = (q == 1 || q == 2) ? -1.0 : 1.0;
    return wr_lm_sinf_poly(x * s, x * x, (q & 2) != 0, n);
  }
  return (y - y) / (y - y); /* inf / nan: invalid */
}

/* s_cosf.c */
WR_LIBM_FN float wr_cosf(float y) {
  double x = y;
  int n;
  const uint32_t top = wr_lm_abstop12(y);
  if (top < 0x3f4) {
    double x2 = x * x;
    if (top < 0x398) return 1.0f;
    return wr_lm_sinf_poly(x, x2, 0, 1);
  } else if (top < 0x42f) {
    x = wr_lm_reduce_fast(x, &n);
    double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;
    return wr_lm_sinf_poly(x * s, x * x, (n & 2) != 0, n ^ 1);
  } else if (top < 0x7f8) {
    uint32_t xi = wr_lm_asuint(y);
    int sign = (int)(xi >> 31);
    x = wr_lm_reduce_large(xi, &n);
    int q = (n + sign) & 3;
    double s = (q == 1 || q == 2) ? -1.0 : 1.0;
    return wr_lm_sinf_poly(x * s, x * x, (q & 2) != 0, n ^ 1);
  }
  return (y - y) / (y - y);
}

/* sinf(y) and cosf(y) together, each bit for bit as wr_sinf / wr_cosf (the
 * samplers take both of one angle, sampler.cpp:100,125): one reduction, and
 * since both polynomials are odd / even in x and the negated cosine set is
 * the exact negation of the other, sin = +-S(x) or +-C(x^2) and cos the other,
 * with the signs glibc's quadrant tables give. */
WR_LIBM_FN void wr_sincosf(float y, float* sp, float* cp) {
  double x = y;
  int n = 0, q = 0;
  const uint32_t top = wr_lm_abstop12(y);
  if (top < 0x3f4) {
    if (top < 0x398) {
      *sp = y;
      *cp = 1.0f;
      return;
    }
  } else if (top < 0x42f) {
    x = wr_lm_reduce_fast(x, &n);
    q = n & 3;
  } else if (top < 0x7f8) {
    uint32_t xi = wr_lm_asuint(y);
    x = wr_lm_reduce_large(xi, &n);
    q = (n + (int)(xi >> 31)) & 3;
  } else {
    *sp = *cp = (y - y) / (y - y);
    return;
  }
  const double x2 = x * x;
  const float S = wr_lm_sinf_poly(x, x2, 0, 0); /* sine polynomial at +x */
  const float C = wr_lm_sinf_poly(x, x2, 0, 1); /* cosine polynomial    */
  const float Ss = (q == 1 || q == 2) ? -S : S; /* at x * sign[q]       */
  const float Cs = (q & 2) ? -C : C;            /* the negated set      */
  if (n & 1) {
    *sp = Cs;
    *cp = Ss;
  } else {
    *sp = Ss;
    *cp = Cs;
  }
}

/* --------------------------------------------------------------------- powf */
/* e_powf_log2_data.c: 16 subintervals of [0x3f330000, 2*0x3f330000), c near
 * the centre of each: invc = 1/c, logc = log2(c); log1p(r)/ln2 polynomial. */
WR_LIBM_FN double wr_lm_log2_inline(uint32_t ix) {
  const double invc_t[16] = {
      0x1.661ec79f8f3bep+0, 0x1.571ed4aaf883dp+0, 0x1.49539f0f010bp+0,  0x1.3c995b0b80385p+0,
      0x1.30d190c8864a5p+0, 0x1.25e227b0b8eap+0,  0x1.1bb4a4a1a343fp+0, 0x1.12358f08ae5bap+0,
      0x1.0953f419900a7p+0, 0x1p+0,               0x1.e608cfd9a47acp-1, 0x1.ca4b31f026aap-1,
      0x1.b2036576afce6p-1, 0x1.9c2d163a1aa2dp-1, 0x1.886e6037841edp-1, 0x1.767dcf5534862p-1};
  const double logc_t[16] = {
      -0x1.efec65b963019p-2, -0x1.b0b6832d4fca4p-2, -0x1.7418b0a1fb77bp-2, -0x1.39de91a6dcf7bp-2,
      -0x1.01d9bf3f2b631p-2, -0x1.97c1d1b3b7afp-3,  -0x1.2f9e393af3c9fp-3, -0x1.960cbbf788d5cp-4,
      -0x1.a6f9db6475fcep-5, 0x0p+0,                0x1.338ca9f24f53dp-4,  0x1.476a9543891bap-3,
      0x1.e840b4ac4e4d2p-3,  0x1.40645f0c6651cp-2,  0x1.88e9c2c1b9ff8p-2,  0x1.ce0a44eb17bccp-2};
  const double A0 = 0x1.27616c9496e0bp-2, A1 = -0x1.71969a075c67ap-2, A2 = 0x1.ec70a6ca7baddp-2,
               A3 = -0x1.7154748bef6c8p-1, A4 = 0x1.71547652ab82bp+0;
  uint32_t tmp = ix - 0x3f330000;
  int i = (int)((tmp >> 19) % 16);
  uint32_t top = tmp & 0xff800000;
  uint32_t iz = ix - top;
  int k = (int32_t)top >> 23;
  double invc = invc_t[i], logc = logc_t[i];
  double z = (double)wr_lm_asfloat(iz);
  double r = WR_LM_FMA(z, invc, -1.0);
  double y0 = logc + (double)k;
  double r2 = r * r;
  double y = WR_LM_FMA(A0, r, A1);
  double p = WR_LM_FMA(A2, r, A3);
  double r4 = r2 * r2;
  double q = WR_LM_FMA(A4, r, y0);
  q = WR_LM_FMA(p, r2, q);
  y = WR_LM_FMA(y, r4, q);
  return y;
}

/* e_exp2f_data.c: tab[i] = bits of 2^(i/32) minus i << 47; cubic for 2^r. */
WR_LIBM_FN double wr_lm_exp2_inline(double xd, uint32_t sign_bias) {
  const uint64_t T[32] = {
      0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
      0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
      0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
      0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
      0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
      0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
      0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
      0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};
  const double SHIFT = 0x1.8p+47; /* 0x1.8p52 / 32 */
  const double C0 = 0x1.c6af84b912394p-5, C1 = 0x1.ebfce50fac4f3p-3, C2 = 0x1.62e42ff0c52d6p-1;
  double kd = xd + SHIFT;
  uint64_t ki = wr_lm_asuint64(kd);
  kd -= SHIFT;
  double r = xd - kd;
  uint64_t t = T[ki % 32];
  uint64_t ski = ki + sign_bias;
  t += ski << (52 - 5);
  double s = wr_lm_asdouble(t);
  double z = WR_LM_FMA(C0, r, C1);
  double r2 = r * r;
  double y = WR_LM_FMA(C2, r, 1.0);
  y = WR_LM_FMA(z, r2, y);
  y = y * s;
  return y;
}

/* 0: not an integer, 1: odd integer, 2: even integer (e_powf.c checkint). */
WR_LIBM_FN int wr_lm_checkint(uint32_t iy) {
  int e = (int)(iy >> 23 & 0xff);
  if (e < 0x7f) return 0;
  if (e > 0x7f + 23) return 2;
  if (iy & ((1u << (0x7f + 23 - e)) - 1)) return 0;
  if (iy & (1u << (0x7f + 23 - e))) return 1;
  return 2;
}
WR_LIBM_FN int wr_lm_zeroinfnan(uint32_t ix) { return 2 * ix - 1 >= 2u * 0x7f800000 - 1; }

/* e_powf.c __powf.  Special cases as glibc's (quiet results; no errno). */
WR_LIBM_FN float wr_powf(float x, float y) {
  uint32_t sign_bias = 0;
  uint32_t ix = wr_lm_asuint(x), iy = wr_lm_asuint(y);
  if (ix - 0x00800000 >= 0x7f800000 - 0x00800000 || wr_lm_zeroinfnan(iy)) {
    if (wr_lm_zeroinfnan(iy)) {
      if (2 * iy == 0) return 1.0f;
      if (ix == 0x3f800000) return 1.0f;
      if (2 * ix > 2u * 0x7f800000 || 2 * iy > 2u * 0x7f800000) return x + y;
      if (2 * ix == 2 * 0x3f800000) return 1.0f;
      if ((2 * ix < 2 * 0x3f800000) == !(iy & 0x80000000)) return 0.0f;
      return y * y;
    }
    if (wr_lm_zeroinfnan(ix)) {
      float x2 = x * x;
      if ((ix & 0x80000000) && wr_lm_checkint(iy) == 1) x2 = -x2;
      return (iy & 0x80000000) ? 1.0f / x2 : x2;
    }
    if (ix & 0x80000000) { /* finite x < 0 */
      int yint = wr_lm_checkint(iy);
      if (yint == 0) return (x - x) / (x - x);
      if (yint == 1) sign_bias = 1u << (5 + 11);
      ix &= 0x7fffffff;
    }
    if (ix < 0x00800000) { /* subnormal x: normalise */
      ix = wr_lm_asuint(x * 0x1p23f);
      ix &= 0x7fffffff;
      ix -= 23 << 23;
    }
  }
  double logx = wr_lm_log2_inline(ix);
  double ylogx = (double)y * logx;
  if ((wr_lm_asuint64(ylogx) >> 47 & 0xffff) >= wr_lm_asuint64(126.0) >> 47) {
    if (ylogx > 0x1.fffffffd1d571p+6) /* overflow */
      return sign_bias ? -0x1p97f * 0x1p97f : 0x1p97f * 0x1p97f;
    if (ylogx <= -150.0) /* underflow */
      return sign_bias ? -0x1p-95f * 0x1p-95f : 0x1p-95f * 0x1p-95f;
  }
  return (float)wr_lm_exp2_inline(ylogx, sign_bias);
}

#endif /* WR_LIBM_H */
