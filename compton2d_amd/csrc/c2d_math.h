/*
 * c2d_math.h — deterministic fp64 elementary functions for the transport path.
 *
 * The reference calls libm for dlog/dexp/cos/acos (e.g. src/imctrk2d.f:153,
 * :414, :228, :477; src/compb_2d.f:85, :234; src/comtot2d.f:348, :392).
 * GPU ocml and host glibc differ in the last ulp, which would make a CPU
 * replay of a GPU packet history diverge at rare branch points.  These
 * routines restate the classic fdlibm/FreeBSD msun algorithms (public
 * domain, Sun Microsystems) using only IEEE +,-,*,/ and sqrt, all correctly
 * rounded on gfx950 and x86-64, so with contraction disabled
 * (-ffp-contract=off on both compilers) host and device return bit-identical
 * results.  Accuracy: < 1 ulp (log, exp, cos), < 2 ulp (acos) — checked
 * against glibc in tests/test_math_rng.py.
 */
#ifndef C2D_MATH_H
#define C2D_MATH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define C2D_HD __host__ __device__ __forceinline__
#else
#define C2D_HD static inline
#endif

/* The divisions of the series below (never by zero or a non-finite value on
 * the finite positive arguments the transport passes).  The fast transport
 * build may define it as a reciprocal-based division (~1 ulp); everything
 * else, the oracle included, keeps the IEEE quotient. */
#ifndef C2D_MDIV
#define C2D_MDIV(a, b) ((a) / (b))
#endif
/* a * b + c in the series' polynomial (Horner) steps: two roundings here;
 * the fast transport build may define it as one fused multiply-add */
#ifndef C2D_MADD
#define C2D_MADD(a, b, c) ((a) * (b) + (c))
#endif

C2D_HD uint64_t c2d_bits(double x) {
  uint64_t u;
  __builtin_memcpy(&u, &x, sizeof u);
  return u;
}
C2D_HD double c2d_from_bits(uint64_t u) {
  double x;
  __builtin_memcpy(&x, &u, sizeof x);
  return x;
}
C2D_HD int32_t c2d_hi(double x) { return (int32_t)(c2d_bits(x) >> 32); }
C2D_HD uint32_t c2d_lo(double x) { return (uint32_t)c2d_bits(x); }
C2D_HD double c2d_with_hi(double x, int32_t hi) {
  return c2d_from_bits(((uint64_t)(uint32_t)hi << 32) | (uint64_t)c2d_lo(x));
}
C2D_HD double c2d_with_lo0(double x) {
  return c2d_from_bits(c2d_bits(x) & 0xffffffff00000000ull);
}

/* natural log (fdlibm e_log.c) */
C2D_HD double c2d_log(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
               two54 = 1.80143985094819840000e+16,
               Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
               Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  int32_t hx = c2d_hi(x);
  uint32_t lx = c2d_lo(x);
  int32_t k = 0;
  if (hx < 0x00100000) {                     /* x < 2^-1022 */
    if (((hx & 0x7fffffff) | lx) == 0) return -two54 / 0.0;   /* -inf */
    if (hx < 0) return (x - x) / 0.0;                          /* NaN  */
    k -= 54;
    x *= two54;
    hx = c2d_hi(x);
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  int32_t i = (hx + 0x95f64) & 0x100000;
  x = c2d_with_hi(x, hx | (i ^ 0x3ff00000));
  k += (i >> 20);
  double f = x - 1.0;
  double dk;
  if ((0x000fffff & (2 + hx)) < 3) {        /* -2^-20 <= f < 2^-20 */
    if (f == 0.0) {
      if (k == 0) return 0.0;
      dk = (double)k;
      return dk * ln2_hi + dk * ln2_lo;
    }
    double R = f * f * (0.5 - 0.33333333333333333 * f);
    if (k == 0) return f - R;
    dk = (double)k;
    return dk * ln2_hi - ((R - dk * ln2_lo) - f);
  }
  double s = C2D_MDIV(f, 2.0 + f);
  dk = (double)k;
  double z = s * s;
  i = hx - 0x6147a;
  double w = z * z;
  int32_t j = 0x6b851 - hx;
  double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  i |= j;
  double R = t2 + t1;
  if (i > 0) {
    double hfsq = 0.5 * f * f;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  }
  if (k == 0) return f - s * (f - R);
  return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

/* c2d_log for finite x > 0 without branches: every path of c2d_log is
 * evaluated and the result selected, so a wavefront does not diverge.  The
 * k == 0 forms of c2d_log are the general forms with dk = 0 (0 * ln2 = 0,
 * a - b = -(b - a) exactly), so the result is bit-identical to c2d_log
 * (tests/test_math_rng.py). */
C2D_HD double c2d_log_pos(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
               two54 = 1.80143985094819840000e+16,
               Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
               Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  const int sub = c2d_hi(x) < 0x00100000;    /* x < 2^-1022 */
  x = sub ? x * two54 : x;
  int32_t hx = c2d_hi(x);
  int32_t k = (sub ? -54 : 0) + (hx >> 20) - 1023;
  hx &= 0x000fffff;
  const int32_t i = (hx + 0x95f64) & 0x100000;
  x = c2d_with_hi(x, hx | (i ^ 0x3ff00000));
  k += (i >> 20);
  const double f = x - 1.0;
  const double dk = (double)k;
  /* -2^-20 <= f < 2^-20 */
  const double Rs = f * f * (0.5 - 0.33333333333333333 * f);
  const double small = dk * ln2_hi - ((Rs - dk * ln2_lo) - f);
  const double s = C2D_MDIV(f, 2.0 + f);
  const double z = s * s;
  const double w = z * z;
  const double t1 = w * C2D_MADD(w, C2D_MADD(w, Lg6, Lg4), Lg2);
  const double t2 = z * C2D_MADD(w, C2D_MADD(w, C2D_MADD(w, Lg7, Lg5), Lg3), Lg1);
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  const double big_a = dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  const double big_b = dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
  const double big = ((hx - 0x6147a) | (0x6b851 - hx)) > 0 ? big_a : big_b;
  return ((0x000fffff & (2 + hx)) < 3) ? small : big;
}

/* exponential (fdlibm e_exp.c) */
C2D_HD double c2d_exp(double x) {
  const double o_threshold = 7.09782712893383973096e+02,
               u_threshold = -7.45133219101941108420e+02,
               ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10,
               invln2 = 1.44269504088896338700e+00, huge = 1.0e+300,
               twom1000 = 9.33263618503218878990e-302,
               P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
               P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
               P5 = 4.13813679705723846039e-08;
  double hi = 0.0, lo = 0.0;
  int32_t k = 0;
  int32_t hx = c2d_hi(x);
  int32_t xsb = (hx >> 31) & 1;
  hx &= 0x7fffffff;
  if (hx >= 0x40862E42) {                    /* |x| >= 709.78... */
    if (hx >= 0x7ff00000) {
      if (((hx & 0xfffff) | c2d_lo(x)) != 0) return x + x;   /* NaN */
      return (xsb == 0) ? x : 0.0;                           /* exp(+-inf) */
    }
    if (x > o_threshold) return huge * huge;
    if (x < u_threshold) return twom1000 * twom1000;
  }
  if (hx > 0x3fd62e42) {                     /* |x| > 0.5 ln2 */
    if (hx < 0x3FF0A2B2) {                   /* and |x| < 1.5 ln2 */
      hi = xsb ? x + ln2HI : x - ln2HI;
      lo = xsb ? -ln2LO : ln2LO;
      k = 1 - xsb - xsb;
    } else {
      k = (int32_t)(invln2 * x + (xsb ? -0.5 : 0.5));
      double t = (double)k;
      hi = x - t * ln2HI;
      lo = t * ln2LO;
    }
    x = hi - lo;
  } else if (hx < 0x3e300000) {              /* |x| < 2^-28 */
    if (huge + x > 1.0) return 1.0 + x;
  } else {
    k = 0;
  }
  double t = x * x;
  double c = x - t * C2D_MADD(t, C2D_MADD(t, C2D_MADD(t, C2D_MADD(t, P5, P4), P3), P2), P1);
  if (k == 0) return 1.0 - (C2D_MDIV(x * c, c - 2.0) - x);
  double y = 1.0 - ((lo - C2D_MDIV(x * c, 2.0 - c)) - hi);
  if (k >= -1021) return c2d_with_hi(y, (int32_t)((uint32_t)c2d_hi(y) + ((uint32_t)k << 20)));
  y = c2d_with_hi(y, (int32_t)((uint32_t)c2d_hi(y) + ((uint32_t)(k + 1000) << 20)));
  return y * twom1000;
}

/* c2d_exp without branches, bit for bit equal to it for every x (NaN and
 * infinities included): fdlibm's reduction with its own choice of k (0, +-1
 * or the rounded x/ln2), both final forms evaluated from one division
 * ((x c)/(c - 2) = -((x c)/(2 - c)) exactly), and the |x| < 2^-28, subnormal
 * and overflow/underflow results selected.  A wavefront whose lanes hold
 * arguments of different ranges runs one path instead of several. */
C2D_HD double c2d_exp_bf(double x) {
  const double o_threshold = 7.09782712893383973096e+02,
               u_threshold = -7.45133219101941108420e+02,
               ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10,
               invln2 = 1.44269504088896338700e+00, huge = 1.0e+300,
               twom1000 = 9.33263618503218878990e-302,
               P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
               P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
               P5 = 4.13813679705723846039e-08;
  const int32_t hx0 = c2d_hi(x);
  const int32_t xsb = (hx0 >> 31) & 1;
  const int32_t hx = hx0 & 0x7fffffff;
  /* the reduction on a clamped copy (the results of |x| > 800 and NaN are
   * replaced below; the clamp keeps the int conversion in range) */
  const double xr = (x > 800.0) ? 800.0 : ((x < -800.0) ? -800.0 : ((x == x) ? x : 0.0));
  const int32_t kg = (int32_t)(invln2 * xr + (xsb ? -0.5 : 0.5));
  const int32_t k = (hx > 0x3fd62e42) ? ((hx < 0x3FF0A2B2) ? (1 - xsb - xsb) : kg) : 0;
  const double t = (double)k;
  const double hi = xr - t * ln2HI, lo = t * ln2LO;
  const double xx = hi - lo;
  const double tt = xx * xx;
  const double c = xx - tt * (P1 + tt * (P2 + tt * (P3 + tt * (P4 + tt * P5))));
  const double q = (xx * c) / (2.0 - c);
  const double y = (k == 0) ? 1.0 - ((-q) - xx) : 1.0 - ((lo - q) - hi);
  const double yn = c2d_with_hi(y, (int32_t)((uint32_t)c2d_hi(y) + ((uint32_t)k << 20)));
  const double ys = c2d_with_hi(y, (int32_t)((uint32_t)c2d_hi(y) + ((uint32_t)(k + 1000) << 20))) * twom1000;
  double r = (k >= -1021) ? yn : ys;
  r = (hx < 0x3e300000) ? 1.0 + x : r;
  if (hx >= 0x40862E42) {                    /* |x| >= 709.78... (rare: a wave-uniform-ish branch) */
    if (hx >= 0x7ff00000)
      r = (((hx & 0xfffff) | c2d_lo(x)) != 0) ? x + x : ((xsb == 0) ? x : 0.0);
    else if (x > o_threshold)
      r = huge * huge;
    else if (x < u_threshold)
      r = twom1000 * twom1000;
  }
  return r;
}

/* kernels on [-pi/4, pi/4] (FreeBSD k_cos.c, k_sin.c) */
C2D_HD double c2d_kcos(double x, double y) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  double z = x * x;
  double w = z * z;
  double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
  double hz = 0.5 * z;
  w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + (z * r - x * y));
}

C2D_HD double c2d_ksin(double x, double y, int iy) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  double z = x * x;
  double w = z * z;
  double r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
  double v = z * x;
  if (iy == 0) return x + v * (S1 + z * r);
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

/* x -> n*pi/2 + (y0+y1) for |x| < 2^19*pi/2 (FreeBSD e_rem_pio2.c, medium case) */
C2D_HD int32_t c2d_rem_pio2(double x, double* y0, double* y1) {
  const double invpio2 = 6.36619772367581382433e-01,
               pio2_1 = 1.57079632673412561417e+00, pio2_1t = 6.07710050650619224932e-11,
               pio2_2 = 6.07710050630396597660e-11, pio2_2t = 2.02226624879595063154e-21,
               pio2_3 = 2.02226624871116645580e-21, pio2_3t = 8.47842766036889956997e-32,
               toint = 6755399441055744.0;   /* 0x1.8p52 */
  int32_t ix = c2d_hi(x) & 0x7fffffff;
  double fn = (x * invpio2 + toint) - toint;
  int32_t n = (int32_t)fn;
  double r = x - fn * pio2_1;
  double w = fn * pio2_1t;
  int32_t j = ix >> 20;
  double a = r - w;
  int32_t i = j - ((c2d_hi(a) >> 20) & 0x7ff);
  if (i > 16) {
    double t = r;
    w = fn * pio2_2;
    r = t - w;
    w = fn * pio2_2t - ((t - r) - w);
    a = r - w;
    i = j - ((c2d_hi(a) >> 20) & 0x7ff);
    if (i > 49) {
      t = r;
      w = fn * pio2_3;
      r = t - w;
      w = fn * pio2_3t - ((t - r) - w);
      a = r - w;
    }
  }
  *y0 = a;
  *y1 = (r - a) - w;
  return n;
}

C2D_HD double c2d_cos(double x) {
  int32_t ix = c2d_hi(x) & 0x7fffffff;
  if (ix <= 0x3fe921fb) {                    /* |x| ~< pi/4 */
    if (ix < 0x3e46a09e) return 1.0;         /* |x| < 2^-27 * sqrt(2) */
    return c2d_kcos(x, 0.0);
  }
  if (ix >= 0x7ff00000) return x - x;
  double y0, y1;
  int32_t n = c2d_rem_pio2(x, &y0, &y1);
  switch (n & 3) {
    case 0: return c2d_kcos(y0, y1);
    case 1: return -c2d_ksin(y0, y1, 1);
    case 2: return -c2d_kcos(y0, y1);
    default: return c2d_ksin(y0, y1, 1);
  }
}

/* arc cosine (fdlibm e_acos.c) */
C2D_HD double c2d_acos(double x) {
  const double pi = 3.14159265358979311600e+00, pio2_hi = 1.57079632679489655800e+00,
               pio2_lo = 6.12323399573676603587e-17,
               pS0 = 1.66666666666666657415e-01, pS1 = -3.25565818622400915405e-01,
               pS2 = 2.01212532134862925881e-01, pS3 = -4.00555345006794114027e-02,
               pS4 = 7.91534994289814532176e-04, pS5 = 3.47933107596021167570e-05,
               qS1 = -2.40339491173441421878e+00, qS2 = 2.02094576023350569471e+00,
               qS3 = -6.88283971605453293030e-01, qS4 = 7.70381505559019352791e-02;
  int32_t hx = c2d_hi(x);
  int32_t ix = hx & 0x7fffffff;
  if (ix >= 0x3ff00000) {                    /* |x| >= 1 */
    if (((ix - 0x3ff00000) | (int32_t)c2d_lo(x)) == 0) {
      if (hx > 0) return 0.0;
      return pi + 2.0 * pio2_lo;
    }
    return (x - x) / (x - x);
  }
  if (ix < 0x3fe00000) {                     /* |x| < 0.5 */
    if (ix <= 0x3c600000) return pio2_hi + pio2_lo;
    double z = x * x;
    double p = z * C2D_MADD(z, C2D_MADD(z, C2D_MADD(z, C2D_MADD(z, C2D_MADD(z, pS5, pS4), pS3), pS2), pS1), pS0);
    double q = C2D_MADD(z, C2D_MADD(z, C2D_MADD(z, C2D_MADD(z, qS4, qS3), qS2), qS1), 1.0);
    double r = C2D_MDIV(p, q);
    return pio2_hi - (x - (pio2_lo - x * r));
  } else if (hx < 0) {                       /* x < -0.5 */
    double z = (1.0 + x) * 0.5;
    double p = z * C2D_MADD(z, C2D_MADD(z, C2D_MADD(z, C2D_MADD(z, C2D_MADD(z, pS5, pS4), pS3), pS2), pS1), pS0);
    double q = C2D_MADD(z, C2D_MADD(z, C2D_MADD(z, C2D_MADD(z, qS4, qS3), qS2), qS1), 1.0);
    double s = __builtin_sqrt(z);
    double r = C2D_MDIV(p, q);
    double w = r * s - pio2_lo;
    return pi - 2.0 * (s + w);
  } else {                                   /* x > 0.5 */
    double z = (1.0 - x) * 0.5;
    double s = __builtin_sqrt(z);
    double df = c2d_with_lo0(s);
    double c = C2D_MDIV(z - df * df, s + df);
    double p = z * C2D_MADD(z, C2D_MADD(z, C2D_MADD(z, C2D_MADD(z, C2D_MADD(z, pS5, pS4), pS3), pS2), pS1), pS0);
    double q = C2D_MADD(z, C2D_MADD(z, C2D_MADD(z, C2D_MADD(z, qS4, qS3), qS2), qS1), 1.0);
    double r = C2D_MDIV(p, q);
    double w = r * s + c;
    return 2.0 * (df + w);
  }
}

/* x**y for x > 0 as used by file_sample (src/imcsurf2d_para.f:718-719). */
C2D_HD double c2d_pow(double x, double y) { return c2d_exp(y * c2d_log(x)); }

#endif /* C2D_MATH_H */
