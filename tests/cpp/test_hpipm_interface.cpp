// Built twice (tests/cpp/Makefile): against the hpipm_catkin stand-in types and against Eigen / ocs2_core-shaped
// types (mock_eigen, mock_ocs2), so it uses only the API both share (no zero-initialising constructors either).
// C++ mirror of the reference gtests ocs2_sqp/hpipm_catkin/test/testHpipmInterface.cpp (solve_and_check_dynamic
// :37-69, solve_after_resize :71-110, knownSolution :112-152, with_constraints :154-206, noInputs :208-256,
// retrieveRiccati :258-340) against the
// HpipmInterface
// mirror, whose solve runs on the MI355X engine. Random problems from a fixed-seed generator (ocs2's
// getRandomDynamics/getRandomCost are not vendored): uniform [-1,1) matrices, costs made positive definite.
#include <unistd.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "hpipm_catkin/HpipmInterface.h"
#ifdef CMPC_HAVE_OCS2_CORE
#include <ocs2_core/misc/LinearAlgebra.h>
#endif

using namespace ocs2;

static std::mt19937_64 rng(20221125);
static double U() { return std::uniform_real_distribution<double>(-1.0, 1.0)(rng); }

static matrix_t zeros(int r, int c) {
  matrix_t m(r, c);
  for (int j = 0; j < c; ++j)
    for (int i = 0; i < r; ++i) m(i, j) = 0.0;
  return m;
}
static matrix_t randm(int r, int c) {
  matrix_t m(r, c);
  for (int j = 0; j < c; ++j)
    for (int i = 0; i < r; ++i) m(i, j) = U();
  return m;
}
static vector_t randv(int n) {
  vector_t v(n);
  for (int i = 0; i < n; ++i) v[i] = U();
  return v;
}
static VectorFunctionLinearApproximation randomDynamics(int nx, int nu) {
  VectorFunctionLinearApproximation d;
  d.dfdx = randm(nx, nx);
  d.dfdu = randm(nx, nu);
  d.f = randv(nx);
  return d;
}
static ScalarFunctionQuadraticApproximation randomCost(int nx, int nu) {
  const int n = nx + nu;
  matrix_t M = randm(n, n), H(n, n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double s = (i == j) ? n : 0.0;
      for (int k = 0; k < n; ++k) s += M(i, k) * M(j, k);
      H(i, j) = s;
    }
  ScalarFunctionQuadraticApproximation c;
  c.dfdxx.resize(nx, nx);
  c.dfdux.resize(nu, nx);
  c.dfduu.resize(nu, nu);
  for (int i = 0; i < nx; ++i)
    for (int j = 0; j < nx; ++j) c.dfdxx(i, j) = H(i, j);
  for (int i = 0; i < nu; ++i)
    for (int j = 0; j < nx; ++j) c.dfdux(i, j) = H(nx + i, j);
  for (int i = 0; i < nu; ++i)
    for (int j = 0; j < nu; ++j) c.dfduu(i, j) = H(nx + i, nx + j);
  c.dfdx = randv(nx);
  c.dfdu = randv(nu);
  return c;
}
static vector_t mv(const matrix_t& A, const vector_t& x) {
  vector_t y(A.rows());
  for (int i = 0; i < A.rows(); ++i) {
    double s = 0;
    for (int j = 0; j < A.cols(); ++j) s += A(i, j) * x[j];
    y[i] = s;
  }
  return y;
}
static vector_t mtv(const matrix_t& A, const vector_t& x) {  // A' x
  vector_t y(A.cols());
  for (int j = 0; j < A.cols(); ++j) {
    double s = 0;
    for (int i = 0; i < A.rows(); ++i) s += A(i, j) * x[i];
    y[j] = s;
  }
  return y;
}
static double maxdiff(const vector_t& a, const vector_t& b) {
  double m = a.size() == b.size() ? 0.0 : 1e300;
  for (int i = 0; i < a.size() && i < b.size(); ++i) m = std::fmax(m, std::fabs(a[i] - b[i]));
  return m;
}

static double norm(const vector_t& v) {
  double s = 0.0;
  for (int i = 0; i < v.size(); ++i) s += v[i] * v[i];
  return std::sqrt(s);
}

static int failures = 0;
#define CHECK(cond, what)                                \
  do {                                                   \
    if (!(cond)) {                                       \
      std::printf("FAIL %s (%s:%d)\n", what, __FILE__, __LINE__); \
      ++failures;                                        \
    }                                                    \
  } while (0)

static void known_solution(bool no_inputs) {
  const int nx = 3, N = 5;
  std::vector<vector_t> xg{randv(nx)}, ug;
  std::vector<VectorFunctionLinearApproximation> sys;
  std::vector<ScalarFunctionQuadraticApproximation> cost;
  for (int k = 0; k < N; ++k) {
    const int nu = (no_inputs && k == 1) ? 0 : 2;
    ug.push_back(randv(nu));
    sys.push_back(randomDynamics(nx, nu));
    vector_t xn = sys[k].f;
    const vector_t ax = mv(sys[k].dfdx, xg[k]), bu = mv(sys[k].dfdu, ug[k]);
    for (int i = 0; i < nx; ++i) xn[i] += ax[i] + bu[i];
    xg.push_back(xn);
    cost.push_back(randomCost(nx, nu));
    const vector_t qx = mv(cost[k].dfdxx, xg[k]), su = mtv(cost[k].dfdux, ug[k]);
    for (int i = 0; i < nx; ++i) cost[k].dfdx[i] = -(qx[i] + su[i]);
    const vector_t ru = mv(cost[k].dfduu, ug[k]), sx = mv(cost[k].dfdux, xg[k]);
    for (int i = 0; i < nu; ++i) cost[k].dfdu[i] = -(ru[i] + sx[i]);
  }
  cost.push_back(randomCost(nx, 0));
  const vector_t qN = mv(cost[N].dfdxx, xg[N]);
  for (int i = 0; i < nx; ++i) cost[N].dfdx[i] = -qN[i];
  HpipmInterface hpipm(hpipm_interface::extractSizesFromProblem(sys, cost, nullptr));
  std::vector<vector_t> xs, us;
  const auto status = hpipm.solve(xg[0], sys, cost, nullptr, xs, us, false);
  CHECK(status == hpipm_status::SUCCESS, "knownSolution status");
  for (int k = 0; k <= N; ++k) CHECK(maxdiff(xs[(size_t)k], xg[(size_t)k]) < 1e-9, "knownSolution x");
  for (int k = 0; k < N; ++k) CHECK(maxdiff(us[(size_t)k], ug[(size_t)k]) < 1e-9, "knownSolution u");
}

static void dynamics_feasible(bool resize) {
  const int nx = 3, nu = 2, N = 5;
  const vector_t x0 = randv(nx);
  std::vector<VectorFunctionLinearApproximation> sys;
  std::vector<ScalarFunctionQuadraticApproximation> cost;
  for (int k = 0; k < N; ++k) {
    sys.push_back(randomDynamics(nx, nu));
    cost.push_back(randomCost(nx, nu));
  }
  cost.push_back(randomCost(nx, 0));
  HpipmInterface hpipm = resize ? HpipmInterface() : HpipmInterface(HpipmInterface::OcpSize(N, nx, nu));
  if (resize) hpipm.resize(HpipmInterface::OcpSize(N, nx, nu));
  std::vector<vector_t> xs, us;
  auto status = hpipm.solve(x0, sys, cost, nullptr, xs, us, false);
  if (resize) {
    hpipm.resize(HpipmInterface::OcpSize(N, nx, nu));
    status = hpipm.solve(x0, sys, cost, nullptr, xs, us, false);
  }
  CHECK(status == hpipm_status::SUCCESS, "dynamics status");
  CHECK(maxdiff(xs[0], x0) < 1e-15, "x0");
  for (int k = 0; k < N; ++k) {
    vector_t xn = sys[k].f;
    const vector_t ax = mv(sys[k].dfdx, xs[(size_t)k]), bu = mv(sys[k].dfdu, us[(size_t)k]);
    for (int i = 0; i < nx; ++i) xn[i] += ax[i] + bu[i];
    CHECK(maxdiff(xs[(size_t)k + 1], xn) < 1e-9, "dynamics feasibility");
  }
  // size mismatch throws like the reference (HpipmInterface.cpp:149-162)
  bool threw = false;
  try {
    std::vector<VectorFunctionLinearApproximation> shorter(sys.begin(), sys.end() - 1);
    hpipm.solve(x0, shorter, cost, nullptr, xs, us, false);
  } catch (const std::runtime_error&) {
    threw = true;
  }
  CHECK(threw, "size mismatch throws");
}

// Eigen's isApprox: |a - b| <= prec * min(|a|, |b|) (2-norms)
static bool is_approx(const vector_t& a, const vector_t& b, double prec) {
  if (a.size() != b.size()) return false;
  double d = 0, na = 0, nb = 0;
  for (int i = 0; i < a.size(); ++i) {
    d += (a[i] - b[i]) * (a[i] - b[i]);
    na += a[i] * a[i];
    nb += b[i] * b[i];
  }
  return std::sqrt(d) <= prec * std::sqrt(std::fmin(na, nb));
}
static VectorFunctionLinearApproximation randomConstraints(int nx, int nu, int nc) {
  VectorFunctionLinearApproximation c;
  c.dfdx = randm(nc, nx);
  c.dfdu = randm(nc, nu);
  c.f = randv(nc);
  return c;
}

// testHpipmInterface.cpp:154-206 with_constraints: one row per node, node 1 left empty, through getOCPSolution's
// non-projection branch (MultipleShootingSolver.cpp:275-277: resize from extractSizesFromProblem with constraints)
static void with_constraints() {
  const int nx = 3, nu = 2, nc = 1, N = 5;
  const vector_t x0 = randv(nx);
  std::vector<VectorFunctionLinearApproximation> sys, con;
  std::vector<ScalarFunctionQuadraticApproximation> cost;
  for (int k = 0; k < N; ++k) {
    sys.push_back(randomDynamics(nx, nu));
    cost.push_back(randomCost(nx, nu));
    con.push_back(randomConstraints(nx, nu, nc));
  }
  cost.push_back(randomCost(nx, 0));
  con.push_back(randomConstraints(nx, 0, nc));
  con[1] = VectorFunctionLinearApproximation();  // "Set one of the constraints to empty"
  HpipmInterface hpipm;
  hpipm.resize(hpipm_interface::extractSizesFromProblem(sys, cost, &con));
  vector_array_t xs, us;
  const auto status = hpipm.solve(x0, sys, cost, &con, xs, us, false);
  CHECK(status == hpipm_status::SUCCESS, "with_constraints status");
  CHECK(is_approx(xs[0], x0, 1e-15), "with_constraints x0");
  for (int k = 0; k < N; ++k) {
    vector_t xn = sys[k].f;
    const vector_t ax = mv(sys[k].dfdx, xs[(size_t)k]), bu = mv(sys[k].dfdu, us[(size_t)k]);
    for (int i = 0; i < nx; ++i) xn[i] += ax[i] + bu[i];
    CHECK(is_approx(xs[(size_t)k + 1], xn, 1e-9), "with_constraints dynamics");
  }
  for (int k = 0; k <= N; ++k) {
    if (con[(size_t)k].f.size() == 0) continue;
    vector_t r = mv(con[(size_t)k].dfdx, xs[(size_t)k]);
    if (k < N) {
      const vector_t du = mv(con[(size_t)k].dfdu, us[(size_t)k]);
      for (int i = 0; i < r.size(); ++i) r[i] += du[i];
    }
    for (int i = 0; i < r.size(); ++i) r[i] = -r[i];
    CHECK(is_approx(con[(size_t)k].f, r, 1e-9), "with_constraints constraint rows");
  }
  // the unconstrained solve of the same problem differs (the constraints bind)
  vector_array_t xu, uu;
  hpipm.resize(hpipm_interface::extractSizesFromProblem(sys, cost, nullptr));
  hpipm.solve(x0, sys, cost, nullptr, xu, uu, false);
  CHECK(maxdiff(uu[0], us[0]) > 1e-6, "constraints change the solution");
  // contradictory duplicate rows at one node: HPIPM's IPM cannot meet them and stops at MAX_ITER or MIN_STEP
  auto bad = con;
  bad[2].dfdx.resize(2, nx);
  bad[2].dfdu.resize(2, nu);
  bad[2].f.resize(2);
  for (int r = 0; r < 2; ++r) {
    for (int j = 0; j < nx; ++j) bad[2].dfdx(r, j) = con[2].dfdx(0, j);
    for (int j = 0; j < nu; ++j) bad[2].dfdu(r, j) = con[2].dfdu(0, j);
    bad[2].f[r] = con[2].f[0] + (r == 0 ? 0.0 : 1.0);
  }
  hpipm.resize(hpipm_interface::extractSizesFromProblem(sys, cost, &bad));
  {
    const auto st = hpipm.solve(x0, sys, cost, &bad, xu, uu, false);
    CHECK(st == hpipm_status::MAX_ITER || st == hpipm_status::MIN_STEP, "inconsistent rows");
  }
  // the same duplicate row, consistent: redundant, same solution as with one row
  bad[2].f[1] = bad[2].f[0];
  CHECK(hpipm.solve(x0, sys, cost, &bad, xu, uu, false) == hpipm_status::SUCCESS, "redundant rows status");
  double e = 0.0;
  for (int k = 0; k < N; ++k) e = std::fmax(e, maxdiff(uu[(size_t)k], us[(size_t)k]));
  CHECK(e < 1e-8, "redundant rows solution");
  std::printf("with_constraints ok (redundant-row max diff %.2e)\n", e);
}

// small dense helpers for the reference recursion (testHpipmInterface.cpp:280-304)
static matrix_t mm(const matrix_t& A, const matrix_t& B) {
  matrix_t C(A.rows(), B.cols());
  for (int i = 0; i < A.rows(); ++i)
    for (int j = 0; j < B.cols(); ++j) {
      double s = 0;
      for (int k = 0; k < A.cols(); ++k) s += A(i, k) * B(k, j);
      C(i, j) = s;
    }
  return C;
}
static matrix_t tr(const matrix_t& A) {
  matrix_t C(A.cols(), A.rows());
  for (int i = 0; i < A.rows(); ++i)
    for (int j = 0; j < A.cols(); ++j) C(j, i) = A(i, j);
  return C;
}
static matrix_t add(const matrix_t& A, const matrix_t& B, double sb = 1.0) {
  matrix_t C = A;
  for (int j = 0; j < C.cols(); ++j)
    for (int i = 0; i < C.rows(); ++i) C(i, j) += sb * B(i, j);
  return C;
}
static vector_t addv(const vector_t& a, const vector_t& b, double sb = 1.0) {
  vector_t c = a;
  for (int i = 0; i < c.size(); ++i) c[i] += sb * b[i];
  return c;
}
static matrix_t inv(const matrix_t& A) {  // Gauss-Jordan with partial pivoting (small, well conditioned)
  const int n = A.rows();
  matrix_t M = A, I = zeros(n, n);
  for (int i = 0; i < n; ++i) I(i, i) = 1.0;
  for (int c = 0; c < n; ++c) {
    int p = c;
    for (int r = c + 1; r < n; ++r)
      if (std::fabs(M(r, c)) > std::fabs(M(p, c))) p = r;
    for (int j = 0; j < n; ++j) {
      std::swap(M(c, j), M(p, j));
      std::swap(I(c, j), I(p, j));
    }
    const double d = M(c, c);
    for (int j = 0; j < n; ++j) {
      M(c, j) /= d;
      I(c, j) /= d;
    }
    for (int r = 0; r < n; ++r)
      if (r != c) {
        const double f = M(r, c);
        for (int j = 0; j < n; ++j) {
          M(r, j) -= f * M(c, j);
          I(r, j) -= f * I(c, j);
        }
      }
  }
  return I;
}
static double maxdiffm(const matrix_t& a, const matrix_t& b) {
  if (a.rows() != b.rows() || a.cols() != b.cols()) return 1e300;
  double m = 0.0;
  for (int j = 0; j < a.cols(); ++j)
    for (int i = 0; i < a.rows(); ++i) m = std::fmax(m, std::fabs(a(i, j) - b(i, j)));
  return m;
}

// testHpipmInterface.cpp:258-340 retrieveRiccati
static void retrieve_riccati() {
  const int nx = 3, nu = 2, N = 5;
  const vector_t x0 = randv(nx);
  std::vector<VectorFunctionLinearApproximation> sys;
  std::vector<ScalarFunctionQuadraticApproximation> cost;
  for (int k = 0; k < N; ++k) {
    sys.push_back(randomDynamics(nx, nu));
    cost.push_back(randomCost(nx, nu));
  }
  cost.push_back(randomCost(nx, 0));
  std::vector<matrix_t> SmG((size_t)N + 1), KG((size_t)N);
  std::vector<vector_t> svG((size_t)N + 1), kG((size_t)N);
  SmG[(size_t)N] = cost[(size_t)N].dfdxx;
  svG[(size_t)N] = cost[(size_t)N].dfdx;
  for (int k = N - 1; k >= 0; --k) {
    const matrix_t& Sm = SmG[(size_t)k + 1];
    const vector_t& sv = svG[(size_t)k + 1];
    const auto& A = sys[(size_t)k].dfdx;
    const auto& B = sys[(size_t)k].dfdu;
    const auto& b = sys[(size_t)k].f;
    const auto& c = cost[(size_t)k];
    const matrix_t P_BTSmA = add(c.dfdux, mm(tr(B), mm(Sm, A)));
    const matrix_t invR = inv(add(c.dfduu, mm(tr(B), mm(Sm, B))));
    const vector_t rr = addv(addv(c.dfdu, mtv(B, sv)), mtv(B, mv(Sm, b)));
    SmG[(size_t)k] = add(add(c.dfdxx, mm(tr(A), mm(Sm, A))), mm(tr(P_BTSmA), mm(invR, P_BTSmA)), -1.0);
    svG[(size_t)k] = addv(addv(addv(c.dfdx, mtv(A, sv)), mtv(A, mv(Sm, b))), mv(tr(P_BTSmA), mv(invR, rr)), -1.0);
    KG[(size_t)k] = add(zeros(nu, nx), mm(invR, P_BTSmA), -1.0);
    kG[(size_t)k] = mv(invR, rr);
    for (int i = 0; i < kG[(size_t)k].size(); ++i) kG[(size_t)k][i] = -kG[(size_t)k][i];
  }
  HpipmInterface hpipm(HpipmInterface::OcpSize(N, nx, nu));
  vector_array_t xs, us;
  const auto st = hpipm.solve(x0, sys, cost, nullptr, xs, us, false);
  CHECK(st == SUCCESS, "retrieveRiccati status");
  const auto K = hpipm.getRiccatiFeedback(sys[0], cost[0]);
  const auto kf = hpipm.getRiccatiFeedforward(sys[0], cost[0]);
  const auto ctg = hpipm.getRiccatiCostToGo(sys[0], cost[0]);
  double e = 0.0;
  for (int k = 0; k <= N; ++k) {
    e = std::fmax(e, maxdiffm(ctg[(size_t)k].dfdxx, SmG[(size_t)k]));
    e = std::fmax(e, maxdiff(ctg[(size_t)k].dfdx, svG[(size_t)k]));
    e = std::fmax(e, std::fabs(ctg[(size_t)k].f));
  }
  for (int k = 0; k < N; ++k) {
    e = std::fmax(e, maxdiffm(K[(size_t)k], KG[(size_t)k]));
    e = std::fmax(e, maxdiff(kf[(size_t)k], kG[(size_t)k]));
    // self-consistency u = K x + k
    e = std::fmax(e, maxdiff(us[(size_t)k], addv(mv(K[(size_t)k], xs[(size_t)k]), kf[(size_t)k])));
  }
  std::printf("retrieveRiccati max err %.3e\n", e);
  CHECK(e < 1e-9, "retrieveRiccati 1e-9");
}

// total cost of a trajectory: sum_k 1/2 x'Q x + u'S x + 1/2 u'R u + q'x + r'u (+ terminal)
static double total_cost(const std::vector<ScalarFunctionQuadraticApproximation>& cost, const vector_array_t& xs,
                         const vector_array_t& us) {
  double J = 0.0;
  for (size_t k = 0; k < cost.size(); ++k) {
    const auto& c = cost[k];
    const vector_t& x = xs[k];
    const vector_t qx = mv(c.dfdxx, x);
    for (int i = 0; i < x.size(); ++i) J += 0.5 * x[i] * qx[i] + c.dfdx[i] * x[i];
    if (k < us.size() && us[k].size() > 0) {
      const vector_t& u = us[k];
      const vector_t ru = mv(c.dfduu, u), sx = mv(c.dfdux, x);
      for (int i = 0; i < u.size(); ++i) J += 0.5 * u[i] * ru[i] + u[i] * sx[i] + c.dfdu[i] * u[i];
    }
  }
  return J;
}

// Riccati quantities after an equality-constrained solve (the non-projection branch of getOCPSolution followed by
// setPrimalSolution's getRiccatiFeedback, MultipleShootingSolver.cpp:275-277, :334-340). The device returns the
// barrier-weighted Riccati quantities of the interior-point solve at the returned point (cmpc_ocp_riccati): u_k =
// K_k x_k + k_k holds on the solution to the IPM's accuracy, and K_0 / the node-0 cost-to-go approach the exact
// derivatives of the constrained solution map as the rows' barrier weights grow (agreement ~1e-4 at HPIPM's default
// tolerances: rows with near-zero multipliers keep moderate weights). Node 0 carries no rows here: the reference
// rebuilds stage 0 from (dynamics0, cost0) alone (HpipmInterface.cpp:334-347, :376-389), which leaves out node-0 rows.
static void constrained_riccati() {
  const int nx = 3, nu = 2, N = 5;
  const vector_t x0 = randv(nx);
  std::vector<VectorFunctionLinearApproximation> sys, con;
  std::vector<ScalarFunctionQuadraticApproximation> cost;
  for (int k = 0; k < N; ++k) {
    sys.push_back(randomDynamics(nx, nu));
    cost.push_back(randomCost(nx, nu));
    con.push_back(randomConstraints(nx, nu, 1));
  }
  cost.push_back(randomCost(nx, 0));
  con.push_back(randomConstraints(nx, 0, 1));
  con[0] = VectorFunctionLinearApproximation();
  con[2] = VectorFunctionLinearApproximation();
  HpipmInterface hpipm(hpipm_interface::extractSizesFromProblem(sys, cost, &con));
  vector_array_t xs, us;
  CHECK(hpipm.solve(x0, sys, cost, &con, xs, us, false) == SUCCESS, "constrained riccati status");
  const auto K = hpipm.getRiccatiFeedback(sys[0], cost[0]);
  const auto kf = hpipm.getRiccatiFeedforward(sys[0], cost[0]);
  const auto ctg = hpipm.getRiccatiCostToGo(sys[0], cost[0]);
  double e_pol = 0.0, e_fd = 0.0, e_ctg = 0.0;
  for (int k = 0; k < N; ++k) e_pol = std::fmax(e_pol, maxdiff(us[(size_t)k], addv(mv(K[(size_t)k], xs[(size_t)k]), kf[(size_t)k])));
  const double J0 = total_cost(cost, xs, us);
  const double eps = 1e-3;
  for (int i = 0; i < nx; ++i) {
    vector_t x1 = x0;
    x1[i] += eps;
    vector_array_t x1s, u1s;
    hpipm.solve(x1, sys, cost, &con, x1s, u1s, false);
    for (int a = 0; a < nu; ++a) e_fd = std::fmax(e_fd, std::fabs((u1s[0][a] - us[0][a]) / eps - K[0](a, i)));
    // V(x0 + d) - V(x0) = s'd + x0'S d + 1/2 d'S d
    const double dJ = total_cost(cost, x1s, u1s) - J0;
    double pred = ctg[0].dfdx[i] * eps + 0.5 * ctg[0].dfdxx(i, i) * eps * eps;
    for (int c = 0; c < nx; ++c) pred += x0[c] * ctg[0].dfdxx(c, i) * eps;
    e_ctg = std::fmax(e_ctg, std::fabs(dJ - pred) / std::fmax(1.0, std::fabs(dJ)));
  }
  double e_sym = 0.0, smax = 1.0;
  for (int k = 0; k <= N; ++k)
    for (int i = 0; i < nx; ++i)
      for (int j = 0; j < nx; ++j) {
        e_sym = std::fmax(e_sym, std::fabs(ctg[(size_t)k].dfdxx(i, j) - ctg[(size_t)k].dfdxx(j, i)));
        smax = std::fmax(smax, std::fabs(ctg[(size_t)k].dfdxx(i, j)));
      }
  std::printf("constrained riccati: policy %.2e, fd K0 %.2e, cost-to-go %.2e, symmetry %.2e (of %.2e)\n", e_pol, e_fd,
              e_ctg, e_sym, smax);
  // u_k - K_k x_k - k_k is the feedforward of the Newton step at the returned point: its right-hand side is the
  // rows' residual (~1e-12) times their barrier weight (1e10+), so it sits near HPIPM's tolerances, not at rounding
  CHECK(e_pol < 1e-6, "constrained riccati u = K x + k");
  CHECK(e_fd < 1e-3, "constrained riccati K0 by finite differences");
  CHECK(e_ctg < 1e-3, "constrained riccati cost-to-go");
  CHECK(e_sym < 1e-12 * smax, "constrained riccati S symmetric");
}

// The legged-robot size (ocs2_legged_robot/config/mpc/task.info: 24 states, 24 inputs, dt 0.015 s over 1 s -> 67
// stages), the reference's constructions: knownSolution (1e-9), retrieveRiccati (closed-form recursion, 1e-9 relative)
// and with_constraints (12 rows per node, dynamics and rows isApprox 1e-9), with a solve-latency print.
static void legged_size() {
  const int nx = 24, nu = 24, N = 67;
  auto stable = [&](int r, int c, double dt) {
    matrix_t m = randm(r, c);
    for (int j = 0; j < c; ++j)
      for (int i = 0; i < r; ++i) m(i, j) = (i == j && r == c ? 1.0 : 0.0) + dt * m(i, j);
    return m;
  };
  std::vector<vector_t> xg{randv(nx)}, ug;
  std::vector<VectorFunctionLinearApproximation> sys;
  std::vector<ScalarFunctionQuadraticApproximation> cost;
  for (int k = 0; k < N; ++k) {
    ug.push_back(randv(nu));
    VectorFunctionLinearApproximation d;
    d.dfdx = stable(nx, nx, 0.015);
    d.dfdu = stable(nx, nu, 0.015);
    d.f = randv(nx);
    for (int i = 0; i < nx; ++i) d.f[i] *= 0.015;
    sys.push_back(d);
    vector_t xn = d.f;
    const vector_t ax = mv(d.dfdx, xg[(size_t)k]), bu = mv(d.dfdu, ug[(size_t)k]);
    for (int i = 0; i < nx; ++i) xn[i] += ax[i] + bu[i];
    xg.push_back(xn);
    cost.push_back(randomCost(nx, nu));
    const vector_t qx = mv(cost[(size_t)k].dfdxx, xg[(size_t)k]), su = mtv(cost[(size_t)k].dfdux, ug[(size_t)k]);
    for (int i = 0; i < nx; ++i) cost[(size_t)k].dfdx[i] = -(qx[i] + su[i]);
    const vector_t ru = mv(cost[(size_t)k].dfduu, ug[(size_t)k]), sx = mv(cost[(size_t)k].dfdux, xg[(size_t)k]);
    for (int i = 0; i < nu; ++i) cost[(size_t)k].dfdu[i] = -(ru[i] + sx[i]);
  }
  cost.push_back(randomCost(nx, 0));
  const vector_t qN = mv(cost[(size_t)N].dfdxx, xg[(size_t)N]);
  for (int i = 0; i < nx; ++i) cost[(size_t)N].dfdx[i] = -qN[i];
  HpipmInterface hpipm(HpipmInterface::OcpSize(N, nx, nu));
  vector_array_t xs, us;
  auto st = hpipm.solve(xg[0], sys, cost, nullptr, xs, us, false);  // first call: module load / first touch
  const auto t0 = std::chrono::steady_clock::now();
  const int reps = 20;
  for (int r = 0; r < reps; ++r) st = hpipm.solve(xg[0], sys, cost, nullptr, xs, us, false);
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / reps;
  CHECK(st == SUCCESS, "legged size status");
  double e = 0.0, sc = 1.0;
  for (int k = 0; k <= N; ++k) e = std::fmax(e, maxdiff(xs[(size_t)k], xg[(size_t)k]));
  for (int k = 0; k < N; ++k) e = std::fmax(e, maxdiff(us[(size_t)k], ug[(size_t)k]));
  // retrieveRiccati at this size
  std::vector<matrix_t> SmG((size_t)N + 1), KG((size_t)N);
  std::vector<vector_t> svG((size_t)N + 1), kG((size_t)N);
  SmG[(size_t)N] = cost[(size_t)N].dfdxx;
  svG[(size_t)N] = cost[(size_t)N].dfdx;
  for (int k = N - 1; k >= 0; --k) {
    const matrix_t& Sm = SmG[(size_t)k + 1];
    const vector_t& sv = svG[(size_t)k + 1];
    const auto& A = sys[(size_t)k].dfdx;
    const auto& B = sys[(size_t)k].dfdu;
    const auto& b = sys[(size_t)k].f;
    const auto& c = cost[(size_t)k];
    const matrix_t P = add(c.dfdux, mm(tr(B), mm(Sm, A)));
    const matrix_t invR = inv(add(c.dfduu, mm(tr(B), mm(Sm, B))));
    const vector_t rr = addv(addv(c.dfdu, mtv(B, sv)), mtv(B, mv(Sm, b)));
    SmG[(size_t)k] = add(add(c.dfdxx, mm(tr(A), mm(Sm, A))), mm(tr(P), mm(invR, P)), -1.0);
    // symmetrised: the plain recursion's antisymmetric rounding mode grows ~1.33x per stage here (4.7e-6 at stage 0
    // against an extended-precision recursion, tools/ric_probe.py); the symmetrised one stays at rounding level
    for (int i = 0; i < nx; ++i)
      for (int j = 0; j < i; ++j) {
        const double v = 0.5 * (SmG[(size_t)k](i, j) + SmG[(size_t)k](j, i));
        SmG[(size_t)k](i, j) = v;
        SmG[(size_t)k](j, i) = v;
      }
    svG[(size_t)k] = addv(addv(addv(c.dfdx, mtv(A, sv)), mtv(A, mv(Sm, b))), mv(tr(P), mv(invR, rr)), -1.0);
    KG[(size_t)k] = add(zeros(nu, nx), mm(invR, P), -1.0);
    kG[(size_t)k] = mv(invR, rr);
    for (int i = 0; i < nu; ++i) kG[(size_t)k][i] = -kG[(size_t)k][i];
  }
  const auto K = hpipm.getRiccatiFeedback(sys[0], cost[0]);
  const auto kf = hpipm.getRiccatiFeedforward(sys[0], cost[0]);
  const auto ctg = hpipm.getRiccatiCostToGo(sys[0], cost[0]);
  double er = 0.0;
  for (int k = 0; k <= N; ++k) {
    for (int i = 0; i < nx; ++i)
      for (int j = 0; j < nx; ++j) sc = std::fmax(sc, std::fabs(SmG[(size_t)k](i, j)));
    er = std::fmax(er, maxdiffm(ctg[(size_t)k].dfdxx, SmG[(size_t)k]));
    er = std::fmax(er, maxdiff(ctg[(size_t)k].dfdx, svG[(size_t)k]));
  }
  for (int k = 0; k < N; ++k) {
    er = std::fmax(er, maxdiffm(K[(size_t)k], KG[(size_t)k]));
    er = std::fmax(er, maxdiff(kf[(size_t)k], kG[(size_t)k]));
  }
  // with_constraints at this size: 12 rows per node (node 1 empty, node N state-only)
  std::vector<VectorFunctionLinearApproximation> con;
  for (int k = 0; k < N; ++k) con.push_back(randomConstraints(nx, nu, 12));
  con.push_back(randomConstraints(nx, 0, 12));
  con[1] = VectorFunctionLinearApproximation();
  HpipmInterface hc(hpipm_interface::extractSizesFromProblem(sys, cost, &con));
  vector_array_t xc, uc;
  auto stc = hc.solve(xg[0], sys, cost, &con, xc, uc, false);
  const auto t1 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; ++r) stc = hc.solve(xg[0], sys, cost, &con, xc, uc, false);
  const double msc = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count() / reps;
  CHECK(stc == SUCCESS, "legged size constrained status");
  double ec = 0.0;
  for (int k = 0; k < N; ++k) {
    vector_t xn = sys[(size_t)k].f;
    const vector_t ax = mv(sys[(size_t)k].dfdx, xc[(size_t)k]), bu = mv(sys[(size_t)k].dfdu, uc[(size_t)k]);
    for (int i = 0; i < nx; ++i) xn[i] += ax[i] + bu[i];
    ec = std::fmax(ec, maxdiff(xc[(size_t)k + 1], xn) / std::fmax(1e-300, norm(xn)));
    if (con[(size_t)k].f.size() > 0) {
      const vector_t r = addv(mv(con[(size_t)k].dfdx, xc[(size_t)k]), mv(con[(size_t)k].dfdu, uc[(size_t)k]));
      vector_t negf = con[(size_t)k].f;
      for (int i = 0; i < negf.size(); ++i) negf[i] = -negf[i];
      ec = std::fmax(ec, maxdiff(r, negf) / std::fmax(1e-300, norm(negf)));
    }
  }
  std::printf("legged size (nx %d, nu %d, N %d): known solution %.3e, riccati %.3e (of %.2e), constrained %.3e; "
              "host-path solve %.3f ms (no rows), %.3f ms (12 rows per node)\n", nx, nu, N, e, er, sc, ec, ms, msc);
  CHECK(e < 1e-9, "legged size knownSolution 1e-9");
  CHECK(er < 1e-9 * sc, "legged size retrieveRiccati 1e-9");
  CHECK(ec < 1e-9, "legged size with_constraints 1e-9");
}

// Per-node state dimensions (OcpSize::numStates[k], OcpSize.cpp:55-60; HPIPM takes nx[k] per node): a known
// solution (the knownSolution construction with nx changing along the horizon), the Riccati quantities against the
// closed-form recursion (retrieveRiccati's, with rectangular A_k), and an equality row at a node whose state is
// smaller than the largest.
static void varying_state_dims() {
  const int N = 5, nu = 2;
  const int nxk[N + 1] = {3, 4, 2, 3, 4, 3};
  std::vector<vector_t> xg{randv(nxk[0])}, ug;
  std::vector<VectorFunctionLinearApproximation> sys;
  std::vector<ScalarFunctionQuadraticApproximation> cost;
  for (int k = 0; k < N; ++k) {
    ug.push_back(randv(nu));
    VectorFunctionLinearApproximation d;
    d.dfdx = randm(nxk[k + 1], nxk[k]);
    d.dfdu = randm(nxk[k + 1], nu);
    d.f = randv(nxk[k + 1]);
    sys.push_back(d);
    vector_t xn = d.f;
    const vector_t ax = mv(d.dfdx, xg[(size_t)k]), bu = mv(d.dfdu, ug[(size_t)k]);
    for (int i = 0; i < nxk[k + 1]; ++i) xn[i] += ax[i] + bu[i];
    xg.push_back(xn);
    cost.push_back(randomCost(nxk[k], nu));
    const vector_t qx = mv(cost[(size_t)k].dfdxx, xg[(size_t)k]), su = mtv(cost[(size_t)k].dfdux, ug[(size_t)k]);
    for (int i = 0; i < nxk[k]; ++i) cost[(size_t)k].dfdx[i] = -(qx[i] + su[i]);
    const vector_t ru = mv(cost[(size_t)k].dfduu, ug[(size_t)k]), sx = mv(cost[(size_t)k].dfdux, xg[(size_t)k]);
    for (int i = 0; i < nu; ++i) cost[(size_t)k].dfdu[i] = -(ru[i] + sx[i]);
  }
  cost.push_back(randomCost(nxk[N], 0));
  const vector_t qN = mv(cost[(size_t)N].dfdxx, xg[(size_t)N]);
  for (int i = 0; i < nxk[N]; ++i) cost[(size_t)N].dfdx[i] = -qN[i];
  const auto size = hpipm_interface::extractSizesFromProblem(sys, cost, nullptr);
  CHECK(size.numStates[2] == 2 && size.numStates[4] == 4, "varying nx: extractSizesFromProblem");
  HpipmInterface hpipm(size);
  vector_array_t xs, us;
  auto st = hpipm.solve(xg[0], sys, cost, nullptr, xs, us, false);
  CHECK(st == SUCCESS, "varying nx status");
  double e = 0.0;
  for (int k = 0; k <= N; ++k) {
    CHECK(xs[(size_t)k].size() == nxk[k], "varying nx: x size");
    e = std::fmax(e, maxdiff(xs[(size_t)k], xg[(size_t)k]));
  }
  for (int k = 0; k < N; ++k) e = std::fmax(e, maxdiff(us[(size_t)k], ug[(size_t)k]));
  // Riccati quantities vs the closed-form recursion over rectangular A_k
  std::vector<matrix_t> SmG((size_t)N + 1), KG((size_t)N);
  std::vector<vector_t> svG((size_t)N + 1), kG((size_t)N);
  SmG[(size_t)N] = cost[(size_t)N].dfdxx;
  svG[(size_t)N] = cost[(size_t)N].dfdx;
  for (int k = N - 1; k >= 0; --k) {
    const matrix_t& Sm = SmG[(size_t)k + 1];
    const vector_t& sv = svG[(size_t)k + 1];
    const auto& A = sys[(size_t)k].dfdx;
    const auto& B = sys[(size_t)k].dfdu;
    const auto& b = sys[(size_t)k].f;
    const auto& c = cost[(size_t)k];
    const matrix_t P = add(c.dfdux, mm(tr(B), mm(Sm, A)));
    const matrix_t invR = inv(add(c.dfduu, mm(tr(B), mm(Sm, B))));
    const vector_t rr = addv(addv(c.dfdu, mtv(B, sv)), mtv(B, mv(Sm, b)));
    SmG[(size_t)k] = add(add(c.dfdxx, mm(tr(A), mm(Sm, A))), mm(tr(P), mm(invR, P)), -1.0);
    svG[(size_t)k] = addv(addv(addv(c.dfdx, mtv(A, sv)), mtv(A, mv(Sm, b))), mv(tr(P), mv(invR, rr)), -1.0);
    KG[(size_t)k] = add(zeros(nu, nxk[k]), mm(invR, P), -1.0);
    kG[(size_t)k] = mv(invR, rr);
    for (int i = 0; i < kG[(size_t)k].size(); ++i) kG[(size_t)k][i] = -kG[(size_t)k][i];
  }
  const auto K = hpipm.getRiccatiFeedback(sys[0], cost[0]);
  const auto kf = hpipm.getRiccatiFeedforward(sys[0], cost[0]);
  const auto ctg = hpipm.getRiccatiCostToGo(sys[0], cost[0]);
  double er = 0.0;
  for (int k = 0; k <= N; ++k) {
    CHECK(ctg[(size_t)k].dfdxx.rows() == nxk[k] && ctg[(size_t)k].dfdx.size() == nxk[k], "varying nx: S size");
    er = std::fmax(er, maxdiffm(ctg[(size_t)k].dfdxx, SmG[(size_t)k]));
    er = std::fmax(er, maxdiff(ctg[(size_t)k].dfdx, svG[(size_t)k]));
  }
  for (int k = 0; k < N; ++k) {
    CHECK(K[(size_t)k].rows() == nu && K[(size_t)k].cols() == nxk[k], "varying nx: K size");
    er = std::fmax(er, maxdiffm(K[(size_t)k], KG[(size_t)k]));
    er = std::fmax(er, maxdiff(kf[(size_t)k], kG[(size_t)k]));
  }
  // one equality row at node 2 (nx = 2): C dx + D du + e = 0 holds at the solution, u = K x + k
  std::vector<VectorFunctionLinearApproximation> cons((size_t)N + 1);
  for (int k = 0; k <= N; ++k) {
    cons[(size_t)k].dfdx = zeros(0, nxk[k]);
    cons[(size_t)k].dfdu = zeros(0, k < N ? nu : 0);
    cons[(size_t)k].f = vector_t(0);
  }
  cons[2] = randomConstraints(nxk[2], nu, 1);
  HpipmInterface hc(hpipm_interface::extractSizesFromProblem(sys, cost, &cons));
  vector_array_t xc, uc;
  st = hc.solve(xg[0], sys, cost, &cons, xc, uc, false);
  CHECK(st == SUCCESS, "varying nx constrained status");
  const vector_t cr = addv(addv(mv(cons[2].dfdx, xc[2]), mv(cons[2].dfdu, uc[2])), cons[2].f);
  double ec = std::fabs(cr[0]), ep = 0.0;
  for (int k = 0; k < N; ++k) {
    vector_t xn = sys[(size_t)k].f;
    const vector_t ax = mv(sys[(size_t)k].dfdx, xc[(size_t)k]), bu = mv(sys[(size_t)k].dfdu, uc[(size_t)k]);
    for (int i = 0; i < nxk[k + 1]; ++i) xn[i] += ax[i] + bu[i];
    ec = std::fmax(ec, maxdiff(xc[(size_t)k + 1], xn));
  }
  const auto Kc = hc.getRiccatiFeedback(sys[0], cost[0]);
  const auto kc = hc.getRiccatiFeedforward(sys[0], cost[0]);
  // u = K x + k with rows holds to the IPM's convergence tolerance (as in riccati_constrained: 1e-6)
  for (int k = 0; k < N; ++k) ep = std::fmax(ep, maxdiff(uc[(size_t)k], addv(mv(Kc[(size_t)k], xc[(size_t)k]), kc[(size_t)k])));
  std::printf("varying state dims: solution %.3e riccati %.3e constrained %.3e policy %.3e\n", e, er, ec, ep);
  CHECK(e < 1e-9 && er < 1e-9 && ec < 1e-8 && ep < 1e-6, "varying state dims");
}

// setRiccatiMinimumEigenvalue on the device path: stage 2 gets R = diag(1e-14, R11) with B_2's first column 0 and a
// small S row, so Lr_2(0,0) = sqrt(1e-14 + reg_prim) ~ 1e-6. Clamped to 1e-3, K_2's first row scales by one factor
// Lr_2(0,0) / 1e-3 and every other row and stage is unchanged (the reference's getRiccatiFeedback on a clamped Lr).
static void riccati_clamp_device() {
  const int nx = 3, nu = 2, N = 5;
  const vector_t x0 = randv(nx);
  std::vector<VectorFunctionLinearApproximation> sys;
  std::vector<ScalarFunctionQuadraticApproximation> cost;
  for (int k = 0; k < N; ++k) {
    sys.push_back(randomDynamics(nx, nu));
    cost.push_back(randomCost(nx, nu));
  }
  cost.push_back(randomCost(nx, 0));
  for (int i = 0; i < nx; ++i) sys[2].dfdu(i, 0) = 0.0;
  cost[2].dfduu(0, 0) = 1e-14;
  cost[2].dfduu(0, 1) = cost[2].dfduu(1, 0) = 0.0;
  for (int j = 0; j < nx; ++j) cost[2].dfdux(0, j) *= 1e-6;
  cost[2].dfdu[0] *= 1e-6;
  HpipmInterface hpipm(HpipmInterface::OcpSize(N, nx, nu));
  vector_array_t xs, us;
  CHECK(hpipm.solve(x0, sys, cost, nullptr, xs, us, false) == SUCCESS, "riccati clamp status");
  const auto Ku = hpipm.getRiccatiFeedback(sys[0], cost[0]);
  hpipm.setRiccatiMinimumEigenvalue(1e-3);
  const auto Kc = hpipm.getRiccatiFeedback(sys[0], cost[0]);
  double e_same = 0.0, rmin = 1e300, rmax = -1e300;
  for (int k = 0; k < N; ++k)
    for (int j = 0; j < nx; ++j)
      for (int a = 0; a < nu; ++a) {
        if (k == 2 && a == 0) {
          const double r = Kc[2](0, j) / Ku[2](0, j);
          rmin = std::fmin(rmin, r);
          rmax = std::fmax(rmax, r);
        } else {
          e_same = std::fmax(e_same, std::fabs(Kc[(size_t)k](a, j) - Ku[(size_t)k](a, j)) /
                                         std::fmax(1.0, std::fabs(Ku[(size_t)k](a, j))));
        }
      }
  const double want = std::sqrt(1e-14 + HpipmInterface::Settings().reg_prim) / 1e-3;
  std::printf("riccati clamp (device): other rows %.3e, clamped row factor [%.6e, %.6e] (want %.6e)\n", e_same, rmin,
              rmax, want);
  CHECK(e_same < 1e-12, "riccati clamp leaves unclamped rows");
  CHECK(std::fabs(rmin - want) < 1e-6 * want && std::fabs(rmax - want) < 1e-6 * want, "riccati clamp row factor");
}

#ifdef CMPC_HAVE_OCS2_CORE
// The getters' default clamp with ocs2_core on the include path (here the mock's ocs2_core/misc/LinearAlgebra.h): no
// minimum set, every getter clamps Lr through ocs2's LinearAlgebra::setTriangularMinimumEigenvalues with its own
// default (the reference's HpipmInterface.cpp:340, :357, :379, :419). Stage 2 gets R = diag(1e-24, R11), B_2's first
// column 0 and reg_prim = 0, so Lr_2(0,0) = 1e-12 lies below the default (1e-9 in the mock): K_2's first row scales by
// 1e-12 / 1e-9 against the unclamped getter (setRiccatiMinimumEigenvalue(0)), everything else is unchanged.
static void riccati_clamp_ocs2_default() {
  const int nx = 3, nu = 2, N = 5;
  const vector_t x0 = randv(nx);
  std::vector<VectorFunctionLinearApproximation> sys;
  std::vector<ScalarFunctionQuadraticApproximation> cost;
  for (int k = 0; k < N; ++k) {
    sys.push_back(randomDynamics(nx, nu));
    cost.push_back(randomCost(nx, nu));
  }
  cost.push_back(randomCost(nx, 0));
  for (int i = 0; i < nx; ++i) sys[2].dfdu(i, 0) = 0.0;
  cost[2].dfduu(0, 0) = 1e-24;
  cost[2].dfduu(0, 1) = cost[2].dfduu(1, 0) = 0.0;
  for (int j = 0; j < nx; ++j) cost[2].dfdux(0, j) *= 1e-12;
  cost[2].dfdu[0] *= 1e-12;
  HpipmInterface::Settings st;
  st.reg_prim = 0.0;
  HpipmInterface hpipm(HpipmInterface::OcpSize(N, nx, nu), st);
  vector_array_t xs, us;
  CHECK(hpipm.solve(x0, sys, cost, nullptr, xs, us, false) == SUCCESS, "ocs2 default clamp status");
  const int calls0 = LinearAlgebra::mockTriangularClampCalls();
  const auto Kd = hpipm.getRiccatiFeedback(sys[0], cost[0]);
  const int calls = LinearAlgebra::mockTriangularClampCalls() - calls0;
  hpipm.setRiccatiMinimumEigenvalue(0.0);
  const auto Ku = hpipm.getRiccatiFeedback(sys[0], cost[0]);
  double e_same = 0.0, rmin = 1e300, rmax = -1e300;
  for (int k = 0; k < N; ++k)
    for (int j = 0; j < nx; ++j)
      for (int a = 0; a < nu; ++a) {
        if (k == 2 && a == 0) {
          const double r = Kd[2](0, j) / Ku[2](0, j);
          rmin = std::fmin(rmin, r);
          rmax = std::fmax(rmax, r);
        } else {
          e_same = std::fmax(e_same, std::fabs(Kd[(size_t)k](a, j) - Ku[(size_t)k](a, j)) /
                                         std::fmax(1.0, std::fabs(Ku[(size_t)k](a, j))));
        }
      }
  std::printf("riccati clamp (ocs2 default): %d LinearAlgebra calls, other rows %.3e, clamped row factor [%.6e, %.6e]\n",
              calls, e_same, rmin, rmax);
  CHECK(calls == N, "the default getter clamps every stage through ocs2's LinearAlgebra");
  CHECK(e_same < 1e-12, "ocs2 default clamp leaves the other rows");
  CHECK(std::fabs(rmin - 1e-3) < 1e-6 && std::fabs(rmax - 1e-3) < 1e-6, "ocs2 default clamp row factor 1e-12 / 1e-9");
}
#endif

// An MPC loop's ticks through resize (MultipleShootingSolver.cpp:275-277 resizes every iteration): the sizes shift
// between the legged shapes (rows at some nodes, then none, nu changing), each tick's solution against a fresh
// interface; after the first round of shapes no device buffer is allocated again (cmpc_ocp_alloc_count).
static void resize_ticks() {
  const int nx = 6, N = 12;
  int allocs_after_warm = -1;
  HpipmInterface ticker;
  for (int tick = 0; tick < 12; ++tick) {
    const int nu = 3 + (tick % 3);
    const bool rows = (tick % 2) == 0;
    std::vector<VectorFunctionLinearApproximation> sys, con;
    std::vector<ScalarFunctionQuadraticApproximation> cost;
    for (int k = 0; k < N; ++k) {
      sys.push_back(randomDynamics(nx, nu));
      cost.push_back(randomCost(nx, nu));
      con.push_back(rows && k > 0 && (k + tick) % 3 ? randomConstraints(nx, nu, 1 + (k + tick) % 2)
                                                    : VectorFunctionLinearApproximation());
    }
    cost.push_back(randomCost(nx, 0));
    con.push_back(VectorFunctionLinearApproximation());
    const vector_t x0 = randv(nx);
    const auto size = hpipm_interface::extractSizesFromProblem(sys, cost, rows ? &con : nullptr);
    ticker.resize(size);
    vector_array_t xs, us, xf, uf;
    const auto st = ticker.solve(x0, sys, cost, rows ? &con : nullptr, xs, us, false);
    HpipmInterface fresh(size);
    const auto sf = fresh.solve(x0, sys, cost, rows ? &con : nullptr, xf, uf, false);
    const auto K = ticker.getRiccatiFeedback(sys[0], cost[0]);
    const auto Kf = fresh.getRiccatiFeedback(sys[0], cost[0]);
    double e = 0.0;
    for (int k = 0; k <= N; ++k) e = std::fmax(e, maxdiff(xs[(size_t)k], xf[(size_t)k]));
    for (int k = 0; k < N; ++k) e = std::fmax(e, std::fmax(maxdiff(us[(size_t)k], uf[(size_t)k]), maxdiffm(K[(size_t)k], Kf[(size_t)k])));
    CHECK(st == sf && e == 0.0, "resize tick equals a fresh interface");
    if (e != 0.0) std::printf("  tick %d: diff %.3e\n", tick, e);
    if (tick == 5) allocs_after_warm = ticker.deviceAllocations();
  }
  std::printf("resize ticks: allocations after the first six %d, after twelve %d\n", allocs_after_warm,
              ticker.deviceAllocations());
  CHECK(ticker.deviceAllocations() == allocs_after_warm, "resize ticks allocate nothing after the first shapes");
}

// solve(..., verbose = true) prints the reference's status block and its 17-column statistics table
// (HpipmInterface.cpp:457-503): one row per iteration 0..iter, the first ten columns the device solver's records.
static void verbose_table() {
  const int nx = 4, nu = 2, N = 6;
  std::vector<VectorFunctionLinearApproximation> sys, con;
  std::vector<ScalarFunctionQuadraticApproximation> cost;
  for (int k = 0; k < N; ++k) {
    sys.push_back(randomDynamics(nx, nu));
    cost.push_back(randomCost(nx, nu));
    con.push_back(k > 0 ? randomConstraints(nx, nu, 1) : VectorFunctionLinearApproximation());
  }
  cost.push_back(randomCost(nx, 0));
  con.push_back(VectorFunctionLinearApproximation());
  HpipmInterface hpipm(hpipm_interface::extractSizesFromProblem(sys, cost, &con));
  vector_array_t xs, us;
  std::fflush(stderr);
  FILE* tf = std::tmpfile();
  const int saved = dup(2);
  dup2(fileno(tf), 2);
  const auto st = hpipm.solve(randv(nx), sys, cost, &con, xs, us, true);
  std::fflush(stderr);
  dup2(saved, 2);
  close(saved);
  std::rewind(tf);
  std::string out;
  char buf[4096];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof buf, tf)) > 0) out.append(buf, n);
  std::fclose(tf);
  CHECK(st == hpipm_status::SUCCESS, "verbose solve status");
  CHECK(out.find("HPIPM returned with flag 0. -> QP solved!") != std::string::npos, "verbose status line");
  const size_t pi = out.find("ipm iter = ");
  CHECK(pi != std::string::npos, "verbose iteration line");
  const int iters = pi == std::string::npos ? -1 : std::atoi(out.c_str() + pi + 11);
  const size_t hi = out.find("lin res comp\n");
  CHECK(hi != std::string::npos && out.find("\tlq fact\t\titref pred\titref corr\tlin res stat") != std::string::npos,
        "verbose table header has the 17 columns");
  int rows = 0, bad = 0;
  double linmax = 0.0;
  size_t at = hi == std::string::npos ? out.size() : hi + 13;
  while (at < out.size()) {
    const size_t e = out.find('\n', at);
    const std::string line = out.substr(at, (e == std::string::npos ? out.size() : e) - at);
    at = e == std::string::npos ? out.size() : e + 1;
    if (line.empty()) continue;
    std::vector<double> v;
    const char* c = line.c_str();
    char* end = nullptr;
    for (double x = std::strtod(c, &end); end != c; x = std::strtod(c, &end)) {
      v.push_back(x);
      c = end;
    }
    // lin res stat / eq / ineq / comp (columns 13-16): the device's Newton-system residuals, finite and at rounding
    // level for every iteration that computed a direction, NaN for the exit row (no direction)
    bool lin_ok = v.size() == 17;
    for (int c = 13; lin_ok && c < 17; ++c) {
      if (rows < iters) {
        lin_ok = std::isfinite(v[(size_t)c]) && v[(size_t)c] <= 1e-6 * std::fmax(1.0, v[6]);
        linmax = std::fmax(linmax, v[(size_t)c]);
      } else {
        lin_ok = std::isnan(v[(size_t)c]);
      }
    }
    ++rows;
    if (v.size() != 17 || !std::isfinite(v[5]) || v[10] != 0.0 || v[11] != 0.0 || v[12] != 0.0 || !lin_ok) ++bad;
  }
  std::printf("verbose table: %d iterations, %d rows, %d malformed, largest lin res %.3e\n", iters, rows, bad, linmax);
  CHECK(rows == iters + 1 && bad == 0, "verbose table: iter + 1 rows of 17 columns");
}

int main() {
  dynamics_feasible(false);
  dynamics_feasible(true);
  known_solution(false);
  known_solution(true);
  with_constraints();
  retrieve_riccati();
  constrained_riccati();
  varying_state_dims();
  riccati_clamp_device();
#ifdef CMPC_HAVE_OCS2_CORE
  riccati_clamp_ocs2_default();
#endif
  resize_ticks();
  verbose_table();
  legged_size();
  std::printf("%s (%d failures)\n", failures ? "FAILED" : "PASSED", failures);
  return failures ? 1 : 0;
}
