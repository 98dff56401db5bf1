/*
 * HpipmInterface.h — drop-in mirror of ocs2::HpipmInterface (reference
 * ocs2_sqp/hpipm_catkin/include/hpipm_catkin/HpipmInterface.h:49-128) whose solve runs on the MI355X engine
 * (a cmpc_ocp handle: the stage-wise OCP interior-point kernel, cmpc_ocp_solve_host).
 *
 * Value types come from hpipm_catkin/ocs2_types.h: the real ocs2_core / Eigen types when ocs2_core is on the include
 * path (then this header, OcpSize.h and HpipmInterfaceSettings.h replace the reference's three headers one for one),
 * else column-major stand-ins with the same member names. The implementation
 * (cheeta-mpc_amd/host/HpipmInterface.cpp) uses only the API both share and talks to the device through the C ABI.
 */
#pragma once

#include <memory>
#include <stdexcept>
#include <vector>

#include "cmpc/cmpc.h"
#include "hpipm_catkin/HpipmInterfaceSettings.h"
#include "hpipm_catkin/OcpSize.h"
#include "hpipm_catkin/ocs2_types.h"

namespace ocs2 {

namespace hpipm_interface {
/* LinearAlgebra::setTriangularMinimumEigenvalues (ocs2_core LinearAlgebra.cpp, called by every Riccati getter,
 * reference HpipmInterface.cpp:340, :357, :379, :419; ocs2_core is not in the reference tree, its published rule is
 * restated): each diagonal entry of the m x m triangular factor L (column-major) moves away from 0 to at least
 * minEigenValue in magnitude (d < 0: min(-minEig, d), else max(minEig, d)). Returns whether any entry changed. */
inline bool setTriangularMinimumEigenvalues(double* L, int m, double minEigenValue) {
  bool changed = false;
  for (int i = 0; i < m; ++i) {
    double& d = L[(size_t)i * m + i];
    const double c = d < 0.0 ? (d < -minEigenValue ? d : -minEigenValue) : (d > minEigenValue ? d : minEigenValue);
    changed = changed || c != d;
    d = c;
  }
  return changed;
}

/* K (m x nx, column-major) re-derived for the clamped factor Lc of the same stage, as getRiccatiFeedback derives it
 * from HPIPM's ric_Lr / ric_Ls (reference HpipmInterface.cpp:361, K = -Lr^-T Ls'): Ls' = -Lr' K recovers Ls' from the
 * unclamped factor Lr and the device's K, then K = -Lc^-T Ls'. work holds m doubles. */
inline void rederiveFeedback(const double* Lr, const double* Lc, double* K, int m, int nx, double* work) {
  for (int j = 0; j < nx; ++j) {
    double* Kj = K + (size_t)j * m;
    for (int a = 0; a < m; ++a) {  // Ls'(a, j) = -sum_{b >= a} Lr(b, a) K(b, j)
      double t = 0.0;
      for (int b = a; b < m; ++b) t -= Lr[(size_t)a * m + b] * Kj[b];
      work[a] = t;
    }
    for (int a = m - 1; a >= 0; --a) {  // Lc' y = Ls'(:, j)
      double t = work[a];
      for (int b = a + 1; b < m; ++b) t -= Lc[(size_t)a * m + b] * work[b];
      work[a] = t / Lc[(size_t)a * m + a];
    }
    for (int a = 0; a < m; ++a) Kj[a] = -work[a];
  }
}
}  // namespace hpipm_interface

class HpipmInterface {
 public:
  using OcpSize = hpipm_interface::OcpSize;
  using Settings = hpipm_interface::Settings;

  explicit HpipmInterface(OcpSize ocpSize = OcpSize(), const Settings& settings = Settings());
  ~HpipmInterface();
  /* Re-lays out the device handle for the new sizes (cmpc_ocp_reshape): the reference's MemoryBlock::reserve grows
   * HPIPM's memory only (HpipmInterface.cpp:46-67, :92-129) and so do the handle's device buffers and pinned staging;
   * a resize to sizes seen before allocates nothing. */
  void resize(OcpSize ocpSize);
  /* Solved on the device by the stage-wise OCP interior point method (cmpc_ocp_solve_host on the handle resize()
   * created): HPIPM's Mehrotra predictor-corrector over a Riccati factorisation per iteration (x0 eliminated, the
   * rows C dx + D du + e = 0 imposed as the reference's lg = ug rows, HpipmInterface.cpp:223-264). Settings are
   * HPIPM's (iter_max, alpha_min, mu0, tol_*, reg_prim; HpipmInterfaceSettings.h); statuses follow it: SUCCESS,
   * MAX_ITER, MIN_STEP (inconsistent rows end there, as in HPIPM), NAN_SOL.
   * The state dimension may change along the horizon (OcpSize::numStates[k], OcpSize.cpp:55-60): each node's state is
   * embedded in a zero-padded state of the largest dimension, whose padding never couples, and every output (state
   * trajectory, S_k, K_k) comes back in the node's own dimension.
   * verbose: the reference's status line, iteration count, max residuals and the per-iteration statistics table
   * (cmpc_ocp_get_residuals / cmpc_ocp_get_stats). */
  hpipm_status solve(const vector_t& x0, std::vector<VectorFunctionLinearApproximation>& dynamics,
                     std::vector<ScalarFunctionQuadraticApproximation>& cost,
                     std::vector<VectorFunctionLinearApproximation>* constraints, vector_array_t& stateTrajectory,
                     vector_array_t& inputTrajectory, bool verbose = false);

  /* Riccati quantities of the previously solved problem (reference HpipmInterface.h:93-123, .cpp:330-455):
   * the solve leaves HPIPM's barrier-weighted recursion at its exit point (cmpc_ocp_set_keep_riccati, the handle is
   * created with it) and cmpc_ocp_riccati_host copies S_k, s_k, K_k, k_k for k >= 1 and Lr_0 (it refactors on the
   * device when the solve left none); stage 0 is rebuilt from (dynamics0, cost0) with the reference's formulas, as
   * HPIPM eliminates x0. Cost-to-go f is 0, as in the reference. */
  std::vector<ScalarFunctionQuadraticApproximation> getRiccatiCostToGo(const VectorFunctionLinearApproximation& dynamics0,
                                                                       const ScalarFunctionQuadraticApproximation& cost0);
  matrix_array_t getRiccatiFeedback(const VectorFunctionLinearApproximation& dynamics0,
                                    const ScalarFunctionQuadraticApproximation& cost0);
  vector_array_t getRiccatiFeedforward(const VectorFunctionLinearApproximation& dynamics0,
                                       const ScalarFunctionQuadraticApproximation& cost0);

  /* The minimum eigenvalue the getters clamp Lr_k to. The reference always clamps, by ocs2_core's
   * LinearAlgebra::setTriangularMinimumEigenvalues with its default minimum (HpipmInterface.cpp:340, :357, :379, :419):
   * so does this mirror when ocs2_core is on the include path and no minimum is set. Setting a minimum replaces that
   * (0: no clamp, the device factor as it is: its pivot guard already zeroes a column whose pivot is <= 1e-200). With
   * the stand-in types (no ocs2_core) there is no ocs2 default: the clamp runs once a minimum is set
   * (hpipm_interface::setTriangularMinimumEigenvalues). A clamped stage's K_k is re-derived from the clamped factor as
   * getRiccatiFeedback derives it (:361), and stage 0 uses the clamped Lr_0. */
  void setRiccatiMinimumEigenvalue(double minEigenValue);
  /* Device allocations the interface's handle has made so far (cmpc_ocp_alloc_count; -1 without a handle). */
  int deviceAllocations() const;
  /* Extensions for timing the tick: HIP events around every solve's kernel (cmpc_ocp_enable_timing), and the last
   * solve's kernel time in ms (cmpc_ocp_last_solve_ms; NaN without a handle or with timing off). */
  void enableDeviceTiming(bool on);
  double lastSolveDeviceMs() const;
  /* Extension for measuring what keeping the exit factorisation costs: on (default) every solve leaves its exit Riccati
   * quantities for the getters (cmpc_ocp_set_keep_riccati); off, the getters refactorise on demand. */
  void keepRiccati(bool on);

 private:
  class Impl;
  std::unique_ptr<Impl> pImpl_;
};

}  // namespace ocs2
