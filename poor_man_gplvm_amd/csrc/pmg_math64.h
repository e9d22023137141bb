// f64 softplus, log and sigmoid for the Adam objective (fit_tuning_helper.py:63-81).
//
// The stop rule compares consecutive losses to tol = 1e-6 relative, so the loss must be
// evaluated to far better than f32 accuracy: a few-ulp f32 softplus / log moves a
// 5000-nat loss by ~1e-5, enough to move a stop decision whose relative change sits
// within 1e-3 of tol (tests/golden/em_small_stoprule.npz: body 985 at 9.9936e-7).  These
// are straight-line f64 evaluations (no tables, no branches) with errors of a few f64
// ulps, ~65 FMA-class operations per (row, neuron).
//
// Shared by the device kernels and the host unit test (oracle-free accuracy check against
// the C library: tests/test_math64.py builds it with g++).
#pragma once
#include <math.h>

#ifdef __HIPCC__
#define PMG_HD __host__ __device__ __forceinline__
#else
#define PMG_HD static inline
#endif

namespace pmg {

// e^x for x <= 0 (x >= -745: below that the result is 0 or subnormal and unused here)
PMG_HD double exp_neg64(double x) {
  const double kL2E = 1.4426950408889634074;
  const double kLn2Hi = 6.93147180369123816490e-01, kLn2Lo = 1.90821492927058770002e-10;
  x = x < -745.0 ? -745.0 : x;
  const double k = rint(x * kL2E);
  double r = fma(-k, kLn2Hi, x);        // exact (kLn2Hi has 32 significant bits, |k| < 2^11)
  r = fma(-k, kLn2Lo, r);               // |r| <= ln2 / 2
  // e^r, Taylor to degree 13 (|r|^14 / 14! < 2^-60 for |r| <= 0.347)
  double p = 1.0 / 6227020800.0;        // 1/13!
  p = fma(p, r, 1.0 / 479001600.0);
  p = fma(p, r, 1.0 / 39916800.0);
  p = fma(p, r, 1.0 / 3628800.0);
  p = fma(p, r, 1.0 / 362880.0);
  p = fma(p, r, 1.0 / 40320.0);
  p = fma(p, r, 1.0 / 5040.0);
  p = fma(p, r, 1.0 / 720.0);
  p = fma(p, r, 1.0 / 120.0);
  p = fma(p, r, 1.0 / 24.0);
  p = fma(p, r, 1.0 / 6.0);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return ldexp(p, (int)k);
}

// 2 atanh(s) = log((1 + s) / (1 - s)) for |s| <= 1/3: 2 s (1 + s^2/3 + s^4/5 + ...),
// 17 odd terms (s^36 / 37 < 2^-60 at s = 1/3)
PMG_HD double atanh2_series(double s) {
  const double z = s * s;
  double p = 1.0 / 35.0;
  p = fma(p, z, 1.0 / 33.0);
  p = fma(p, z, 1.0 / 31.0);
  p = fma(p, z, 1.0 / 29.0);
  p = fma(p, z, 1.0 / 27.0);
  p = fma(p, z, 1.0 / 25.0);
  p = fma(p, z, 1.0 / 23.0);
  p = fma(p, z, 1.0 / 21.0);
  p = fma(p, z, 1.0 / 19.0);
  p = fma(p, z, 1.0 / 17.0);
  p = fma(p, z, 1.0 / 15.0);
  p = fma(p, z, 1.0 / 13.0);
  p = fma(p, z, 1.0 / 11.0);
  p = fma(p, z, 1.0 / 9.0);
  p = fma(p, z, 1.0 / 7.0);
  p = fma(p, z, 1.0 / 5.0);
  p = fma(p, z, 1.0 / 3.0);
  const double s3 = s * z;
  return fma(2.0 * s3, p, 2.0 * s);
}

// a / b to ~1 ulp: v_rcp_f64 (or 1/b on the host) and two Newton steps, then one
// residual correction of the quotient
PMG_HD double div64(double a, double b) {
#ifdef __HIP_DEVICE_COMPILE__
  double r = __builtin_amdgcn_rcp(b);
#else
  double r = 1.0 / b;
#endif
  r = fma(r, fma(-b, r, 1.0), r);
  r = fma(r, fma(-b, r, 1.0), r);
  const double q = a * r;
  return fma(r, fma(-b, q, a), q);
}

// log1p(e) for 0 <= e <= 1: 2 atanh(e / (2 + e)) (2 + e is exact-rounded, the quotient
// carries ~1 ulp; no cancellation for small e)
PMG_HD double log1p_unit64(double e) { return atanh2_series(div64(e, 2.0 + e)); }

// log(x) for normal positive x: x = m 2^k with m in [sqrt(1/2), sqrt(2)), then
// 2 atanh((m - 1) / (m + 1)) (m - 1 exact by Sterbenz), + k ln 2 in two parts
PMG_HD double log64(double x) {
  int k;
  double m = frexp(x, &k);              // m in [0.5, 1)
  const bool lo = m < 0.70710678118654752440;
  m = lo ? 2.0 * m : m;
  k = lo ? k - 1 : k;
  const double t = atanh2_series(div64(m - 1.0, m + 1.0));
  const double kd = (double)k;
  return fma(kd, 6.93147180369123816490e-01, fma(kd, 1.90821492927058770002e-10, t));
}

// softplus(F) = max(F, 0) + log1p(e^-|F|), its log, and sigmoid(F) = (F >= 0 ? 1 : e) / (1 + e)
struct Softplus64 {
  double f, logf, sg;
};
PMG_HD Softplus64 softplus64(double F) {
  const double e = exp_neg64(-fabs(F));
  Softplus64 o;
  o.f = fmax(F, 0.0) + log1p_unit64(e);
  o.logf = log64(o.f + 1e-20);
  o.sg = div64(F >= 0.0 ? 1.0 : e, 1.0 + e);
  return o;
}

}  // namespace pmg
