/*
 * CentroidalMPC.h — Eigen-free mirror of the reference's public MPC class (reference CentroidalMPC.h:15-33,
 * NonlinearMPC.h:50-154), backed by the MI355X batched QP engine through the C ABI (cmpc/cmpc.h).
 *
 * Same constructor arguments, SetupMPC(), UpdateMPC(state, des_state, des_inputs) with the reference's flat
 * layouts (CentroidalMPC.cpp:284-323) and the same "mpc table invalid" std::runtime_error (:328-330). Differences:
 *   - UpdateMPC returns the contact forces (the reference returns an empty vector, :369): per leg i a 3 x N
 *     column-major block, legs concatenated — the order of the reference controller's contact_force_i outputs;
 *   - the IPOPT_SOLVER argument is accepted and ignored (the solver is the batched GPU interior point method);
 *   - nothing is printed (the reference prints the table and every output, :325, :357-362);
 *   - UpdateMPCBatch solves many robots' problems in one call (device-resident records, see cmpc_solve_batch).
 */
#pragma once

#include <cstdint>
#include <stdexcept>
#include <vector>

#include "cmpc/cmpc.h"

enum class IPOPT_SOLVER : unsigned int { MUMPS = 0, WSMP = 1, PARDISO = 2, MA27 = 3, MA57 = 4, MA77 = 5, MA86 = 6, MA97 = 7 };

namespace cheeta_mpc {
using VectorXd = std::vector<double>;
}

class CentroidalMPC {
 public:
  using VectorXd = cheeta_mpc::VectorXd;

  CentroidalMPC(double mass, int num_legs, int predict_horizon, double time_step, const VectorXd& weights,
                const VectorXd& mu, IPOPT_SOLVER ipopt_solver = IPOPT_SOLVER::MA97, int precision = CMPC_F64,
                int max_batch = 1);
  ~CentroidalMPC();
  CentroidalMPC(const CentroidalMPC&) = delete;
  CentroidalMPC& operator=(const CentroidalMPC&) = delete;

  void SetupMPC();
  VectorXd UpdateMPC(const VectorXd& state, const VectorXd& des_state, const VectorXd& des_inputs);
  void UpdateWeights(const VectorXd& weights);

  /* Batched extension: device pointers in cmpc_solve_batch's record layout, async on stream. */
  int UpdateMPCBatch(int B, const double* d_x0, const double* d_xref, const double* d_foot, const uint8_t* d_contact,
                     double* d_u, double* d_x, int* d_status, int* d_iters, void* stream);

  /* Feedback policy dU/dx0 of each QP at its solution d_u (cmpc_policy_batch; the condensed counterpart of
   * HpipmInterface::getRiccatiFeedback, HpipmInterface.cpp:330-455): d_K [B][N][L][3][13]. */
  int FeedbackPolicyBatch(int B, const double* d_x0, const double* d_xref, const double* d_foot,
                          const uint8_t* d_contact, const double* d_u, double act_tol, double* d_K, int* d_nfree,
                          int* d_status, void* stream);

  /* The 13-state record UpdateMPC builds from the reference's flat layouts (exposed for tests). */
  void PackRecord(const VectorXd& state, const VectorXd& des_state, const VectorXd& des_inputs, VectorXd& x0,
                  VectorXd& xref, VectorXd& foot, std::vector<uint8_t>& contact) const;

  int lastStatus() const { return last_status_; }
  int lastIterations() const { return last_iters_; }
  double currentTime() const { return current_time_; }
  const cmpc_model& model() const { return model_; }
  void setSettings(const cmpc_settings& s);

 private:
  cmpc_model model_;
  cmpc_settings settings_;
  int precision_;
  int max_batch_;
  cmpc_ctx* ctx_ = nullptr;
  double current_time_ = 0.0;
  int last_status_ = -1;
  int last_iters_ = 0;
};
