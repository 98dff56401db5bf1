// CPU check of the IPM kernels' fraction-to-boundary selection (cheeta-mpc_amd/csrc/step_ratio.hpp) at extreme
// fp32 magnitudes: slacks and directions near 1e-20 and 1e+20, where fp32 cross-products overflow or flush to 0.
// The selected ratio must equal the smallest v / (-d) over the candidates with d < 0 (reference: long double).
#include <cmath>
#include <cstdio>
#include <random>

#include "step_ratio.hpp"

template <typename T>
static int check(const T* v, const T* d, int n, const char* what) {
  cmpc::MinRatio<T> mr;
  long double best = 1e300L;
  for (int i = 0; i < n; ++i) {
    mr.cand(v[i], d[i]);
    if (d[i] < 0) best = std::fmin(best, (long double)v[i] / -(long double)d[i]);
  }
  const long double got = (long double)mr.value();
  const long double ref = (long double)(T)best;  // the kernels return the ratio in T
  const bool ok = (std::isinf((double)ref) && std::isinf((double)got)) ||
                  std::fabs((double)(got - ref)) <= 1e-6 * std::fabs((double)ref);
  if (!ok) std::printf("FAIL %s: got %.9Lg want %.9Lg\n", what, got, ref);
  return ok ? 0 : 1;
}

int main() {
  int fails = 0;
  {  // binding candidate with tiny slack and tiny step: fp32 products v*den ~ 1e-40 flush to 0
    const float v[4] = {1e-20f, 3e-20f, 1.0f, 2e-20f}, d[4] = {-2e-20f, -1e-20f, 0.5f, -1e-19f};
    fails += check(v, d, 4, "tiny");
  }
  {  // huge slacks and steps: fp32 products ~ 1e40 overflow to inf
    const float v[4] = {1e20f, 5e19f, 3e20f, 1e20f}, d[4] = {-1e20f, -1e19f, -1e21f, 4e20f};
    fails += check(v, d, 4, "huge");
  }
  {  // mixed: a tiny binding ratio among huge ones
    const float v[4] = {1e20f, 1e-20f, 2e20f, 7.0f}, d[4] = {-1e-20f, -1e20f, -3e20f, -1.0f};
    fails += check(v, d, 4, "mixed");
  }
  {  // no candidate with d < 0: full step (ratio >= 1)
    const float v[2] = {1e-20f, 1e20f}, d[2] = {1e-20f, 0.0f};
    cmpc::MinRatio<float> mr;
    for (int i = 0; i < 2; ++i) mr.cand(v[i], d[i]);
    if (!(mr.value() >= 1.0f)) {
      std::printf("FAIL none: %g\n", (double)mr.value());
      ++fails;
    }
  }
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> e(-30.0, 30.0);
  std::bernoulli_distribution neg(0.6);
  for (int t = 0; t < 20000; ++t) {  // random magnitudes over 1e-30 .. 1e30, fp32 and fp64
    float vf[8], df[8];
    double vd[8], dd[8];
    for (int i = 0; i < 8; ++i) {
      vd[i] = std::pow(10.0, e(rng));
      dd[i] = (neg(rng) ? -1.0 : 1.0) * std::pow(10.0, e(rng));
      vf[i] = (float)vd[i];
      df[i] = (float)dd[i];
    }
    fails += check(vf, df, 8, "random f32");
    fails += check(vd, dd, 8, "random f64");
    if (fails > 10) break;
  }
  std::printf(fails ? "step_ratio: %d failures\n" : "step_ratio: ok\n", fails);
  return fails ? 1 : 0;
}
