// The MPC tick through the HpipmInterface mirror (bench.py --ocp, the "tick" object): per tick, as
// MultipleShootingSolver::runImpl drives HPIPM (reference MultipleShootingSolver.cpp:275-277, :334-341):
//   resize(extractSizesFromProblem(...)) + solve(...) + getRiccatiFeedback(dynamics[0], cost[0])
// on problems whose sizes shift from tick to tick (the legged gait's event nodes, cheeta_mpc/ocp.py legged_problem
// with t0 advancing). Input: a binary file written by bench.py (int32 T, then per tick: int32 N, nx, has_rows,
// nu[N], nc[N+1] when has_rows; doubles x0[nx], rec[record size], crec[constraint record size] when has_rows —
// the packed forms of include/cmpc/cmpc.h). Output: one JSON line with the per-phase host times (ms; the median and
// the 90th percentile over the ticks after the first --warm) and the device time of the solve's kernel (HIP events,
// cmpc_ocp_last_solve_ms).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "hpipm_catkin/HpipmInterface.h"

using namespace ocs2;

namespace {

struct Tick {
  int N = 0, nx = 0;
  std::vector<int> nu, nc;
  vector_t x0;
  std::vector<VectorFunctionLinearApproximation> dyn, con;
  std::vector<ScalarFunctionQuadraticApproximation> cost;
  bool rows = false;
};

template <class T>
bool rd(FILE* f, T* p, size_t n) {
  return std::fread(p, sizeof(T), n, f) == n;
}

matrix_t take(const double*& p, int r, int c) {
  matrix_t m(r, c);
  for (int j = 0; j < c; ++j)
    for (int i = 0; i < r; ++i) m(i, j) = *p++;
  return m;
}
vector_t takev(const double*& p, int n) {
  vector_t v(n);
  for (int i = 0; i < n; ++i) v(i) = *p++;
  return v;
}

bool read_tick(FILE* f, Tick& t) {
  int h[3];
  if (!rd(f, h, 3)) return false;
  t.N = h[0];
  t.nx = h[1];
  t.rows = h[2] != 0;
  t.nu.resize((size_t)t.N);
  if (!rd(f, t.nu.data(), (size_t)t.N)) return false;
  t.nc.assign((size_t)t.N + 1, 0);
  if (t.rows && !rd(f, t.nc.data(), (size_t)t.N + 1)) return false;
  const int N = t.N, nx = t.nx;
  std::vector<double> x0((size_t)nx);
  if (!rd(f, x0.data(), (size_t)nx)) return false;
  const size_t rs = cmpc_ocp_record_size(N, nx, t.nu.data());
  std::vector<double> rec(rs);
  if (!rd(f, rec.data(), rs)) return false;
  std::vector<double> crec;
  if (t.rows) {
    crec.resize(cmpc_ocp_constraint_record_size(N, nx, t.nu.data(), t.nc.data()));
    if (!rd(f, crec.data(), crec.size())) return false;
  }
  t.x0 = vector_t(nx);
  for (int i = 0; i < nx; ++i) t.x0(i) = x0[(size_t)i];
  const double* p = rec.data();
  t.dyn.resize((size_t)N);
  for (int k = 0; k < N; ++k) {
    const int m = t.nu[(size_t)k];
    t.dyn[(size_t)k].dfdx = take(p, nx, nx);
    t.dyn[(size_t)k].dfdu = take(p, nx, m);
    t.dyn[(size_t)k].f = takev(p, nx);
  }
  t.cost.resize((size_t)N + 1);
  for (int k = 0; k <= N; ++k) {
    const int m = k < N ? t.nu[(size_t)k] : 0;
    auto& c = t.cost[(size_t)k];
    c.dfdxx = take(p, nx, nx);
    c.dfdux = take(p, m, nx);
    c.dfduu = take(p, m, m);
    c.dfdx = takev(p, nx);
    c.dfdu = takev(p, m);
  }
  if (t.rows) {
    const double* q = crec.data();
    t.con.resize((size_t)N + 1);
    for (int k = 0; k <= N; ++k) {
      const int g = t.nc[(size_t)k], m = k < N ? t.nu[(size_t)k] : 0;
      auto& c = t.con[(size_t)k];
      if (g == 0) {
        c.dfdx = matrix_t(0, nx);
        c.dfdu = matrix_t(0, m);
        c.f = vector_t(0);
        continue;
      }
      c.dfdx = take(q, g, nx);
      c.dfdu = take(q, g, m);
      c.f = takev(q, g);
    }
  }
  return true;
}

double pct(std::vector<double> v, double q) {
  if (v.empty()) return NAN;
  std::sort(v.begin(), v.end());
  const size_t i = std::min(v.size() - 1, (size_t)std::floor(q * (double)(v.size() - 1) + 0.5));
  return v[i];
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: hpipm_tick <ticks.bin> [warm]\n");
    return 2;
  }
  const int warm = argc > 2 ? std::atoi(argv[2]) : 5;
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  int T = 0;
  if (!rd(f, &T, 1) || T <= 0) return 2;
  std::vector<Tick> ticks((size_t)T);
  for (int t = 0; t < T; ++t)
    if (!read_tick(f, ticks[(size_t)t])) {
      std::fprintf(stderr, "hpipm_tick: short file at tick %d\n", t);
      return 2;
    }
  std::fclose(f);
  HpipmInterface hpipm;
  hpipm.enableDeviceTiming(true);
  std::vector<double> t_resize, t_solve, t_fb, t_tick, t_kernel;
  int ok = 0, allocs_warm = -1;
  using clk = std::chrono::steady_clock;
  auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  for (int t = 0; t < T; ++t) {
    Tick& k = ticks[(size_t)t];
    vector_array_t xs, us;
    const auto t0 = clk::now();
    hpipm.resize(hpipm_interface::extractSizesFromProblem(k.dyn, k.cost, k.rows ? &k.con : nullptr));
    const auto t1 = clk::now();
    const auto st = hpipm.solve(k.x0, k.dyn, k.cost, k.rows ? &k.con : nullptr, xs, us, false);
    const auto t2 = clk::now();
    const auto K = hpipm.getRiccatiFeedback(k.dyn[0], k.cost[0]);
    const auto t3 = clk::now();
    const double kern = hpipm.lastSolveDeviceMs();
    if (st == hpipm_status::SUCCESS && (int)K.size() == k.N) ++ok;
    if (t == warm - 1) allocs_warm = hpipm.deviceAllocations();
    if (t < warm) continue;
    t_resize.push_back(ms(t0, t1));
    t_solve.push_back(ms(t1, t2));
    t_fb.push_back(ms(t2, t3));
    t_tick.push_back(ms(t0, t3));
    t_kernel.push_back(kern);
  }
  // the same ticks again without keeping the exit factorisation: the keep's kernel cost, tick by tick
  std::vector<double> t_kernel_nokeep, t_keep_cost;
  {
    HpipmInterface h2;
    h2.enableDeviceTiming(true);
    h2.keepRiccati(false);
    for (int t = 0; t < T; ++t) {
      Tick& k = ticks[(size_t)t];
      vector_array_t xs, us;
      h2.resize(hpipm_interface::extractSizesFromProblem(k.dyn, k.cost, k.rows ? &k.con : nullptr));
      (void)h2.solve(k.x0, k.dyn, k.cost, k.rows ? &k.con : nullptr, xs, us, false);
      const double kern = h2.lastSolveDeviceMs();
      if (t < warm) continue;
      t_kernel_nokeep.push_back(kern);
      t_keep_cost.push_back(t_kernel[(size_t)(t - warm)] - kern);
    }
  }
  std::printf("{\"ticks\": %d, \"timed\": %zu, \"success\": %d, \"rows\": %s, "
              "\"tick_ms_median\": %.4f, \"tick_ms_p90\": %.4f, \"resize_ms_median\": %.4f, \"solve_ms_median\": %.4f, "
              "\"solve_ms_p90\": %.4f, \"feedback_ms_median\": %.4f, \"feedback_ms_p90\": %.4f, "
              "\"kernel_ms_median\": %.4f, \"host_over_kernel_ms_median\": %.4f, \"allocations_after_warmup\": %d, "
              "\"kernel_ms_median_nokeep\": %.4f, \"keep_cost_ms_median\": %.4f}\n",
              T, t_tick.size(), ok, ticks[0].rows ? "true" : "false", pct(t_tick, 0.5), pct(t_tick, 0.9),
              pct(t_resize, 0.5), pct(t_solve, 0.5), pct(t_solve, 0.9), pct(t_fb, 0.5), pct(t_fb, 0.9),
              pct(t_kernel, 0.5), pct(t_solve, 0.5) - pct(t_kernel, 0.5),
              hpipm.deviceAllocations() - allocs_warm, pct(t_kernel_nokeep, 0.5), pct(t_keep_cost, 0.5));
  return ok == T ? 0 : 1;
}
