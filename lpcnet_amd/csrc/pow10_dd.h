/*
 * pow10_dd.h -- 10^x in double, computed with double-double arithmetic from
 * IEEE-754 basic operations and fma only, so the host (gcc / hipcc host pass)
 * and the device (gfx950 v_fma_f64 ...) produce the same bits.
 *
 * Used for the band powers of lpc_from_cepstrum, freq.c:318
 *     Ex[i] = pow(10.f, Ex[i]) * compensation[i]   (double pow, float result)
 * The engine needs (float)(pow10_dd(E) * (double)comp) to equal
 * (float)(glibc pow(10, E) * (double)comp) for every float E and each of the
 * reference's compensation factors; oracle/checks/pow10_exhaustive.c checks
 * that over all 2^32 float bit patterns (tests/test_lpc.py runs it).  The
 * evaluation is accurate to far below one double ulp, so the only inputs where
 * a float rounding could differ from glibc's (0.52-ulp) pow are listed by that
 * check; there are none for the compensation factors of freq.c:50-53.
 *
 * Plain C/C++ (no libm): include from C, C++ or HIP.  Compile users with
 * -ffp-contract=off.
 */
#ifndef LPCNET_POW10_DD_H
#define LPCNET_POW10_DD_H

#if defined(__HIPCC__) || defined(__HIP__)
#define P10_HD __host__ __device__ __forceinline__
#define P10_FMA(a, b, c) __builtin_fma((a), (b), (c))
#else
#define P10_HD static inline
#define P10_FMA(a, b, c) __builtin_fma((a), (b), (c))
#endif

typedef struct {
  double hi, lo;
} p10_dd;

/* a + b exactly, |a| >= |b| not required */
P10_HD p10_dd p10_two_sum(double a, double b)
{
  const double s = a + b;
  const double bb = s - a;
  const double e = (a - (s - bb)) + (b - bb);
  p10_dd r;
  r.hi = s;
  r.lo = e;
  return r;
}

/* a + b exactly, requires |a| >= |b| (or a == 0) */
P10_HD p10_dd p10_fast_two_sum(double a, double b)
{
  const double s = a + b;
  p10_dd r;
  r.hi = s;
  r.lo = b - (s - a);
  return r;
}

P10_HD p10_dd p10_add(p10_dd x, p10_dd y)
{
  p10_dd s = p10_two_sum(x.hi, y.hi);
  p10_dd t = p10_two_sum(x.lo, y.lo);
  s.lo += t.hi;
  s = p10_fast_two_sum(s.hi, s.lo);
  s.lo += t.lo;
  return p10_fast_two_sum(s.hi, s.lo);
}

P10_HD p10_dd p10_mul(p10_dd x, p10_dd y)
{
  const double p = x.hi * y.hi;
  double e = P10_FMA(x.hi, y.hi, -p);
  e = P10_FMA(x.hi, y.lo, e);
  e = P10_FMA(x.lo, y.hi, e);
  return p10_fast_two_sum(p, e);
}

P10_HD p10_dd p10_mul_d(p10_dd x, double y)
{
  const double p = x.hi * y;
  double e = P10_FMA(x.hi, y, -p);
  e = P10_FMA(x.lo, y, e);
  return p10_fast_two_sum(p, e);
}

/* 2^n as a double, n in [-1022, 1023] */
P10_HD double p10_exp2i(int n)
{
  union {
    double d;
    unsigned long long u;
  } v;
  v.u = (unsigned long long)(n + 1023) << 52;
  return v.d;
}

/* 10^x.  NaN -> the NaN itself (quieted); +inf -> +inf; -inf -> +0;
 * overflow -> +inf; underflow -> a correctly scaled subnormal or +0. */
P10_HD double pow10_dd(double x)
{
  if (x != x) return x + x;
  if (x > 310.0) return x * 1e308; /* +inf (x may be +inf) */
  if (x < -330.0) return 0.0;
  /* log2(10) = L0 + L1 + L2 to ~160 bits (each the double nearest the remainder) */
  const double L0 = 3.321928094887362;
  const double L1 = 1.661617516973592e-16;
  const double L2 = 1.2215512178458181e-32;
  /* t = x * log2(10) as a double-double */
  const double p = x * L0;
  double e = P10_FMA(x, L0, -p);
  e = P10_FMA(x, L1, e);
  e = P10_FMA(x, L2, e);
  p10_dd t = p10_fast_two_sum(p, e);
  /* t = n + f, |f| <= 1/2 + tiny, f as a double-double; p - n is exact */
  const double n = __builtin_rint(t.hi);
  p10_dd f = p10_two_sum(t.hi - n, t.lo);
  /* g = f * ln 2 (ln 2 to 159 bits), |g| < 0.35; then g / 2^8 */
  p10_dd LN2;
  LN2.hi = 0.6931471805599453;
  LN2.lo = 2.3190468138462996e-17;
  p10_dd g = p10_mul(f, LN2);
  g.hi *= 0x1p-8;
  g.lo *= 0x1p-8;
  /* exp(g) - 1 for |g| < 0.0014 by Taylor to g^9/9! (next term < 2^-117),
   * Horner in double-double */
  /* 1/k! = hi + lo (hi the nearest double, lo the nearest double to the rest) */
  const double inv[8] = {2.48015873015873e-05, 0.0001984126984126984, 0.001388888888888889, 0.008333333333333333,
                         0.041666666666666664, 0.16666666666666666, 0.5, 1.0};
  const double inv_lo[8] = {2.1511947866775882e-23, 1.7209558293420705e-22, -5.300543954373577e-20,
                            1.1564823173178714e-19, 2.3129646346357427e-18, 9.25185853854297e-18, 0.0, 0.0};
  p10_dd s;
  s.hi = 2.7557319223985893e-06; /* 1/9! */
  s.lo = -1.858393274046472e-22;
  for (int k = 0; k < 8; k++) {
    s = p10_mul(s, g);
    p10_dd c;
    c.hi = inv[k];
    c.lo = inv_lo[k];
    s = p10_add(s, c);
  }
  s = p10_mul(s, g); /* exp(g) - 1 */
  /* (1 + s)^(2^8) via 8 squarings of 1 + s kept as 1 + s: (1+s)^2 = 1 + (2s + s^2) */
  for (int k = 0; k < 8; k++) {
    p10_dd s2 = p10_mul(s, s);
    p10_dd two_s;
    two_s.hi = 2.0 * s.hi;
    two_s.lo = 2.0 * s.lo;
    s = p10_add(two_s, s2);
  }
  p10_dd one;
  one.hi = 1.0;
  one.lo = 0.0;
  const p10_dd r = p10_add(one, s);
  const int ni = (int)n;
  /* scale by 2^n in two exact steps (no double rounding above the subnormal range) */
  if (ni > 1000) return (r.hi * p10_exp2i(1000)) * p10_exp2i(ni - 1000);
  if (ni < -1000) {
    /* result is subnormal: round once, from the double-double sum */
    return (r.hi * p10_exp2i(-1000)) * p10_exp2i(ni + 1000);
  }
  return r.hi * p10_exp2i(ni);
}

#endif
