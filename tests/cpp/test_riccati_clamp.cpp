// Host-only check of the Riccati getters' minimum-eigenvalue clamp (hpipm_interface::setTriangularMinimumEigenvalues
// and rederiveFeedback, include/hpipm_catkin/HpipmInterface.h; the reference clamps Lr in every getter,
// HpipmInterface.cpp:340, :357, :379, :419, and derives K = -Lr^-T Ls' at :361). A stage with a near-singular
// R + B'PB: R = diag(1e-14, 2, 3) and B's first column 0, so Lr(0, 0) = 1e-7. No device, no libcmpc.
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "hpipm_catkin/HpipmInterface.h"

int main() {
  const int m = 3, nx = 4;
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  // M = R + B'PB (column-major m x m), Nm = S + B'PA (m x nx): row/column 0 of M is (1e-14, 0, 0)
  double M[m * m] = {1e-14, 0, 0, 0, 2.0, 0.3, 0, 0.3, 3.0};
  std::vector<double> Nm((size_t)m * nx);
  for (auto& v : Nm) v = U(rng);
  // Cholesky M = L L' (lower, column-major)
  double L[m * m] = {0};
  for (int j = 0; j < m; ++j) {
    double d = M[j * m + j];
    for (int t = 0; t < j; ++t) d -= L[t * m + j] * L[t * m + j];
    L[j * m + j] = std::sqrt(d);
    for (int i = j + 1; i < m; ++i) {
      double s = M[j * m + i];
      for (int t = 0; t < j; ++t) s -= L[t * m + i] * L[t * m + j];
      L[j * m + i] = s / L[j * m + j];
    }
  }
  auto lsolve = [&](const double* F, double* c) {  // c <- F^-1 c
    for (int a = 0; a < m; ++a) {
      double s = c[a];
      for (int b = 0; b < a; ++b) s -= F[b * m + a] * c[b];
      c[a] = s / F[a * m + a];
    }
  };
  auto ltsolve = [&](const double* F, double* c) {  // c <- F^-T c
    for (int a = m - 1; a >= 0; --a) {
      double s = c[a];
      for (int b = a + 1; b < m; ++b) s -= F[a * m + b] * c[b];
      c[a] = s / F[a * m + a];
    }
  };
  // the device's quantities: K = -M^-1 Nm (through L), Ls' = L^-1 Nm
  std::vector<double> K((size_t)m * nx), LsT((size_t)m * nx);
  for (int j = 0; j < nx; ++j) {
    double c[m];
    for (int a = 0; a < m; ++a) c[a] = Nm[(size_t)j * m + a];
    lsolve(L, c);
    for (int a = 0; a < m; ++a) LsT[(size_t)j * m + a] = c[a];
    ltsolve(L, c);
    for (int a = 0; a < m; ++a) K[(size_t)j * m + a] = -c[a];
  }
  int fail = 0;
  // the clamp rule: diag >= min unchanged, small positive -> min, small negative -> -min
  {
    double A[4] = {0.5, 0.1, 0.0, -1e-9}, B[4] = {2.0, 0.0, 0.0, 3.0};
    const bool ca = ocs2::hpipm_interface::setTriangularMinimumEigenvalues(A, 2, 1e-3);
    const bool cb = ocs2::hpipm_interface::setTriangularMinimumEigenvalues(B, 2, 1e-3);
    if (!ca || cb || A[0] != 0.5 || A[3] != -1e-3 || A[1] != 0.1 || B[0] != 2.0 || B[3] != 3.0) {
      std::printf("clamp rule wrong\n");
      ++fail;
    }
  }
  const double minEig = 1e-3;
  double Lc[m * m];
  for (int i = 0; i < m * m; ++i) Lc[i] = L[i];
  if (!ocs2::hpipm_interface::setTriangularMinimumEigenvalues(Lc, m, minEig) || Lc[0] != minEig) {
    std::printf("near-singular stage not clamped\n");
    ++fail;
  }
  std::vector<double> Kc = K, work((size_t)m);
  ocs2::hpipm_interface::rederiveFeedback(L, Lc, Kc.data(), m, nx, work.data());
  // the reference's formula on the clamped factor: K = -Lc^-T Ls'
  double e = 0.0, e0 = 0.0;
  for (int j = 0; j < nx; ++j) {
    double c[m];
    for (int a = 0; a < m; ++a) c[a] = LsT[(size_t)j * m + a];
    ltsolve(Lc, c);
    for (int a = 0; a < m; ++a) {
      const double want = -c[a];
      e = std::fmax(e, std::fabs(Kc[(size_t)j * m + a] - want) / std::fmax(1.0, std::fabs(want)));
    }
    // closed form of the clamped row: -Nm(0, j) / (Lr(0, 0) minEig) = -Nm(0, j) / (1e-7 1e-3)
    const double row0 = -Nm[(size_t)j * m] / (1e-7 * minEig);
    e0 = std::fmax(e0, std::fabs(Kc[(size_t)j * m] - row0) / std::fabs(row0));
  }
  std::printf("riccati clamp: K vs -Lc^-T Ls' %.3e, clamped row vs closed form %.3e, unclamped row 0 %.3e\n", e, e0,
              K[0]);
  if (!(e < 1e-9) || !(e0 < 1e-9)) ++fail;
  std::printf("%s\n", fail ? "riccati_clamp: FAILED" : "riccati_clamp: ok");
  return fail ? 1 : 0;
}
