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
#include <string.h>

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

// ---------------------------------------------------------------------------------
// Table-driven log for the hot loop (k_adam): 128 intervals of [1, 2), entry j holding
// (1 / c_j, -log(1 / c_j)) with c_j = 1 + (j + 1/2) / 128, except entry 0 = (1, 0) so that
// u in [1, 1 + 1/128) reduces EXACTLY to r = u - 1 (log1p of tiny arguments keeps its
// relative accuracy).  log x = k ln2 + (-log(1 / c_j)) + log1p(r), r = x 2^-k / c_j - 1 in
// one fma, |r| < 1/128, log1p(r) to degree 8 (r^9 / 9 < 2^-63 |r|).  The table is built on
// the device from log64 (log_tab_entry), so host and device share one definition.
// ---------------------------------------------------------------------------------
constexpr int kLogTab = 128;

PMG_HD void log_tab_entry(int j, double& invc, double& nlc) {
  if (j == 0) {
    invc = 1.0;
    nlc = 0.0;
    return;
  }
  invc = div64(1.0, 1.0 + (j + 0.5) / (double)kLogTab);
  nlc = -log64(invc);
}

// log x for normal positive x; tab[2 j] = 1 / c_j, tab[2 j + 1] = -log(1 / c_j)
PMG_HD double log_tab(double x, const double* tab) {
  int k;
  const double m = 2.0 * frexp(x, &k);          // [1, 2)
  const double kd = (double)(k - 1);
#ifdef __HIP_DEVICE_COMPILE__
  const int j = (int)((__double2hiint(m) >> 13) & (kLogTab - 1));
#else
  long long bits;
  memcpy(&bits, &m, 8);
  const int j = (int)((bits >> 45) & (kLogTab - 1));
#endif
  const double invc = tab[2 * j], nlc = tab[2 * j + 1];
  const double r = fma(m, invc, -1.0);
  double p = -1.0 / 8.0;
  p = fma(p, r, 1.0 / 7.0);
  p = fma(p, r, -1.0 / 6.0);
  p = fma(p, r, 1.0 / 5.0);
  p = fma(p, r, -1.0 / 4.0);
  p = fma(p, r, 1.0 / 3.0);
  p = fma(p, r, -1.0 / 2.0);
  const double lp = fma(r * r, p, r);            // log1p(r)
  const double hi = fma(kd, 6.93147180369123816490e-01, nlc);
  return hi + fma(kd, 1.90821492927058770002e-10, lp);
}

// log u for u in [1, 2) with the table of log_tab: no exponent split (k = 0)
PMG_HD double log_tab_unit(double u, const double* tab) {
#ifdef __HIP_DEVICE_COMPILE__
  const int j = (int)((__double2hiint(u) >> 13) & (kLogTab - 1));
#else
  long long bits;
  memcpy(&bits, &u, 8);
  const int j = (int)((bits >> 45) & (kLogTab - 1));
#endif
  const double invc = tab[2 * j], nlc = tab[2 * j + 1];
  const double r = fma(u, invc, -1.0);
  double p = -1.0 / 8.0;
  p = fma(p, r, 1.0 / 7.0);
  p = fma(p, r, -1.0 / 6.0);
  p = fma(p, r, 1.0 / 5.0);
  p = fma(p, r, -1.0 / 4.0);
  p = fma(p, r, 1.0 / 3.0);
  p = fma(p, r, -1.0 / 2.0);
  return nlc + fma(r * r, p, r);
}

// ---------------------------------------------------------------------------------
// Table-driven e^x (x <= 0) for the hot loop: x = (64 n + j) ln2 / 64 + r, |r| <= ln2 / 128,
// e^x = 2^n 2^(j/64) e^r with e^r to degree 6 (r^7 / 7! < 2^-64); entry j = 2^(j/64) is
// built from exp_neg64 (2 e^((j - 64) ln2 / 64)).  It sits after the log table: the k_adam
// LDS table and softplus_tab's `tab` hold both (kMathTab doubles).
// ---------------------------------------------------------------------------------
constexpr int kExpTab = 64;
constexpr int kMathTab = 2 * kLogTab + kExpTab;

PMG_HD double exp_tab_entry(int j) {
  return 2.0 * exp_neg64((double)(j - kExpTab) * (6.93147180559945309417e-01 / kExpTab));
}

// the whole table: log part (log_tab_entry) then exp part
PMG_HD void math_tab_entry(int q, double* tab) {
  if (q < kLogTab) log_tab_entry(q, tab[2 * q], tab[2 * q + 1]);
  else if (q < kLogTab + kExpTab) tab[2 * kLogTab + (q - kLogTab)] = exp_tab_entry(q - kLogTab);
}

PMG_HD double exp_neg_tab(double x, const double* et) {
  const double kL2E64 = 92.332482616893656;                 // 64 / ln 2
  const double kLn2Hi64 = 6.93147180369123816490e-01 / 64;  // 32 significant bits: k * it is exact
  const double kLn2Lo64 = 1.90821492927058770002e-10 / 64;
  x = x < -745.0 ? -745.0 : x;
  const double k = rint(x * kL2E64);
  double r = fma(-k, kLn2Hi64, x);
  r = fma(-k, kLn2Lo64, r);
  double p = 1.0 / 720.0;
  p = fma(p, r, 1.0 / 120.0);
  p = fma(p, r, 1.0 / 24.0);
  p = fma(p, r, 1.0 / 6.0);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  const int ki = (int)k;
  return ldexp(et[ki & (kExpTab - 1)] * p, ki >> 6);
}

// softplus, its log and the sigmoid with the table log and exp: log1p(e) = log(u) +
// (e - (u - 1)) / u, u = 1 + e rounded (u - 1 and e - (u - 1) are exact; the correction is
// below ulp(u), so an approximate reciprocal suffices); u in (1, 2], log 2 exactly at u = 2.
// The sigmoid is returned to f32 accuracy: it only scales the f32 gradient factor G.
// tab: kMathTab doubles (math_tab_entry).
struct SoftplusT {
  double f, logf;
  float sg;
};
PMG_HD SoftplusT softplus_tab(double F, const double* tab) {
  const double e = exp_neg_tab(-fabs(F), tab + 2 * kLogTab);
  const double u = 1.0 + e;
#ifdef __HIP_DEVICE_COMPILE__
  const double ru = __builtin_amdgcn_rcp(u);
#else
  const double ru = 1.0 / u;
#endif
  const double lu = u < 2.0 ? log_tab_unit(u, tab) : 6.93147180559945309417e-01;
  const double l1p = lu + (e - (u - 1.0)) * ru;
  SoftplusT o;
  o.f = fmax(F, 0.0) + l1p;
  o.logf = log_tab(o.f + 1e-20, tab);
  const float e32 = (float)e;
#ifdef __HIP_DEVICE_COMPILE__
  o.sg = (F >= 0.0 ? 1.0f : e32) * __builtin_amdgcn_rcpf(1.0f + e32);
#else
  o.sg = (F >= 0.0 ? 1.0f : e32) / (1.0f + e32);
#endif
  return o;
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
