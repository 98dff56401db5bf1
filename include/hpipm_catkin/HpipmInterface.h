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
  /* Solved on the device. constraints == nullptr: equality-free stages (cmpc_ocp_solve_batch_host); otherwise the
   * rows C dx + D du + e = 0 are imposed as the reference's lg = ug rows (HpipmInterface.cpp:223-264) by
   * cmpc_ocp_solve_batch_eq_host (x0-eliminated stage 0, redundant rows dropped, inconsistent rows -> INCONS_EQ,
   * where HPIPM's interior point method would stop at MAX_ITER or MIN_STEP instead: status parity unpinned).
   * The state dimension may change along the horizon (OcpSize::numStates[k], OcpSize.cpp:55-60): each node's state is
   * embedded in a zero-padded state of the largest dimension, whose padding never couples, and every output (state
   * trajectory, S_k, K_k) comes back in the node's own dimension.
   * Settings::reg_prim is added to the input Hessians (and the state Hessians of nodes 1..N); the other settings
   * parametrise an interior point method this direct solve does not run (HpipmInterfaceSettings.h).
   * verbose: the reference's status line, iteration count, max residuals and statistics table (one row: the
   * direct solve is iteration 0), residuals evaluated on the host from the returned trajectories. */
  hpipm_status solve(const vector_t& x0, std::vector<VectorFunctionLinearApproximation>& dynamics,
                     std::vector<ScalarFunctionQuadraticApproximation>& cost,
                     std::vector<VectorFunctionLinearApproximation>* constraints, vector_array_t& stateTrajectory,
                     vector_array_t& inputTrajectory, bool verbose = false);

  /* Riccati quantities of the previously solved problem (reference HpipmInterface.h:93-123, .cpp:330-455).
   * Unconstrained solve: the device recursion cmpc_ocp_riccati_batch_host. Equality-constrained solve: the exact
   * feedback of the constrained problem, which HPIPM's barrier-weighted recursion approaches at convergence: for
   * every stage k the tail problem k..N is solved on the device as a batch of nx + 1 problems (x_k = 0 and the unit
   * vectors; state-only rows of node k dropped, x_k being given there), so u_k = K_k x_k + k_k and the cost-to-go
   * 1/2 x' S_k x + s_k' x follows from the tail trajectories' affine maps. The reference rebuilds stage 0 from
   * (dynamics0, cost0) because HPIPM eliminates x0; here the recursion runs over stage 0 directly, so the arguments
   * must equal the stage-0 data of the last solve (size-checked). Cost-to-go f is 0, as in the reference. */
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
