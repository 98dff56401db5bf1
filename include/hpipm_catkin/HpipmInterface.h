/*
 * HpipmInterface.h — drop-in mirror of ocs2::HpipmInterface (reference
 * ocs2_sqp/hpipm_catkin/include/hpipm_catkin/HpipmInterface.h:49-128) whose solve runs on the MI355X engine
 * (cmpc_ocp_solve_batch_host / cmpc_ocp_solve_batch_eq_host: x0 elimination, condensing and a dense KKT solve on the
 * device).
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

class HpipmInterface {
 public:
  using OcpSize = hpipm_interface::OcpSize;
  using Settings = hpipm_interface::Settings;

  explicit HpipmInterface(OcpSize ocpSize = OcpSize(), const Settings& settings = Settings());
  ~HpipmInterface();
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
   * cmpc_ocp_riccati_host refactors at the returned point (HPIPM's barrier-weighted recursion at its exit) and gives
   * S_k, s_k, K_k, k_k for k >= 1 and Minv_0; stage 0 is rebuilt from (dynamics0, cost0) with the reference's formulas,
   * as HPIPM eliminates x0. Cost-to-go f is 0, as in the reference. */
  std::vector<ScalarFunctionQuadraticApproximation> getRiccatiCostToGo(const VectorFunctionLinearApproximation& dynamics0,
                                                                       const ScalarFunctionQuadraticApproximation& cost0);
  matrix_array_t getRiccatiFeedback(const VectorFunctionLinearApproximation& dynamics0,
                                    const ScalarFunctionQuadraticApproximation& cost0);
  vector_array_t getRiccatiFeedforward(const VectorFunctionLinearApproximation& dynamics0,
                                       const ScalarFunctionQuadraticApproximation& cost0);

 private:
  class Impl;
  std::unique_ptr<Impl> pImpl_;
};

}  // namespace ocs2
