// Accuracy check of poor_man_gplvm_amd/csrc/pmg_math64.h against the long-double C
// library (x87 80-bit: 11 more bits than f64), built and run by tests/test_math64.py.
// Prints one line: max errors in f64 ulps (log(f): in f64 eps relative to max(1, |log f|))
// of the series form (softplus64) and of the table form (softplus_tab).
#include <cmath>
#include <cstdio>
#include <random>

#include "pmg_math64.h"

static double ulps(double got, long double ref) {
  if (ref == 0) return got == 0 ? 0 : 1e30;
  const double r = std::fabs((double)ref);
  return (double)(std::fabs((long double)got - ref) / (std::nextafter(r, INFINITY) - r));
}
static double logerr(double got, long double ref) {
  return std::fabs(got - (double)ref) / std::fmax(1.0, std::fabs((double)ref)) / 1.1102230246251565e-16;
}

int main() {
  double tab[pmg::kMathTab];
  for (int q = 0; q < pmg::kLogTab + pmg::kExpTab; ++q) pmg::math_tab_entry(q, tab);
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> wide(-40, 40), narrow(-3, 3), lx(-350, 350);
  double ef = 0, el = 0, es = 0, ee = 0, eg = 0, tf = 0, tl = 0, ts = 0, tg = 0, te = 0;
  for (int i = 0; i < 1000000; ++i) {
    const double F = (i & 1) ? wide(g) : narrow(g);
    const pmg::Softplus64 o = pmg::softplus64(F);
    const pmg::SoftplusT t = pmg::softplus_tab(F, tab);
    const long double Fl = F, e = expl(-fabsl(Fl));
    const long double f = (Fl > 0 ? Fl : 0) + log1pl(e);
    const long double lf = logl(f + 1e-20L);
    const long double sg = 1.0L / (1.0L + expl(-Fl));
    ef = std::fmax(ef, ulps(o.f, f));
    el = std::fmax(el, logerr(o.logf, lf));
    es = std::fmax(es, ulps(o.sg, sg));
    tf = std::fmax(tf, ulps(t.f, f));
    tl = std::fmax(tl, logerr(t.logf, lf));
    ts = std::fmax(ts, std::fabs((double)t.sg - (double)sg) / (double)sg);
    ee = std::fmax(ee, ulps(pmg::exp_neg64(-std::fabs(F)), e));
    te = std::fmax(te, ulps(pmg::exp_neg_tab(-std::fabs(F), tab + 2 * pmg::kLogTab), e));
    const double x = std::exp(lx(g) * 2);
    eg = std::fmax(eg, ulps(pmg::log64(x), logl((long double)x)));
    tg = std::fmax(tg, logerr(pmg::log_tab(x, tab), logl((long double)x)));
  }
  std::printf("%.3f %.3f %.3f %.3f %.3f %.3f %.3f %.3e %.3f %.3f\n", ef, el, es, ee, eg, tf, tl, ts, tg, te);
  return 0;
}
