/*
 * CentroidalMPC.h — mirror of the reference's public MPC class (reference CentroidalMPC.h:15-33,
 * NonlinearMPC.h:50-154), backed by the MI355X batched QP engine through the C ABI (cmpc/cmpc.h).
 *
 * Same constructor arguments, SetupMPC(), UpdateMPC(state, des_state, des_inputs) with the reference's flat
 * layouts (CentroidalMPC.cpp:284-323) and the same "mpc table invalid" std::runtime_error (:328-330). The vector
 * arguments are templates over any contiguous double vector with data() / size() / resize() (Eigen::VectorXd, which
 * the reference takes, or std::vector<double>): the reference's caller (CentoidMPCTest.cpp) compiles against this
 * header with only the include swapped, and the library behind it (libcmpc.so, host/CentroidalMPC.cpp) sees raw
 * pointers only. Differences:
 *   - UpdateMPC returns the contact forces (the reference returns an empty vector, :369): per leg i a 3 x N
 *     column-major block, legs concatenated — the order of the reference controller's contact_force_i outputs;
 *   - the IPOPT_SOLVER argument is accepted and ignored (the solver is the batched GPU interior point method);
 *   - by default UpdateMPC solves the condensed QP of the hot path (lever arm at the reference CoM, later stance runs
 *     at the mean des foothold); setNonlinear(true) solves the reference's NLP instead (cmpc_nlp_solve_batch: SQP on
 *     the bilinear lever arm with the later runs' footholds as decision variables, CentroidalMPC.cpp:132-133,
 *     196-198, 218-221); FootPositions() returns the foot_pos output (:269-273) of the last call in both modes;
 *   - nothing is printed (the reference prints the table and every output, :325, :357-362);
 *   - UpdateMPCBatch solves many robots' problems in one call (device-resident records, see cmpc_solve_batch).
 */
#pragma once

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <vector>

#include "cmpc/cmpc.h"

#if !defined(CMPC_EIGEN_STANDIN) && __has_include(<Eigen/Dense>)
#include <Eigen/Dense>
#define CMPC_HAVE_EIGEN 1
#endif

enum class IPOPT_SOLVER : unsigned int { MUMPS = 0, WSMP = 1, PARDISO = 2, MA27 = 3, MA57 = 4, MA77 = 5, MA86 = 6, MA97 = 7 };

namespace cheeta_mpc {
#ifdef CMPC_HAVE_EIGEN
using VectorXd = Eigen::VectorXd;  // the reference's argument type (CentroidalMPC.h:26-32)
#else
using VectorXd = std::vector<double>;
#endif
}  // namespace cheeta_mpc

class CentroidalMPC {
 public:
  using VectorXd = cheeta_mpc::VectorXd;

  template <class Vec>
  CentroidalMPC(double mass, int num_legs, int predict_horizon, double time_step, const Vec& weights, const Vec& mu,
                IPOPT_SOLVER ipopt_solver = IPOPT_SOLVER::MA97, int precision = CMPC_F64, int max_batch = 1)
      : CentroidalMPC(mass, num_legs, predict_horizon, time_step, weights.data(), (size_t)weights.size(), mu.data(),
                      (size_t)mu.size(), ipopt_solver, precision, max_batch) {}
  /* the constructor proper: raw arrays (weights[(num_legs + 1) * 9], mu[num_legs]) */
  CentroidalMPC(double mass, int num_legs, int predict_horizon, double time_step, const double* weights,
                size_t n_weights, const double* mu, size_t n_mu, IPOPT_SOLVER ipopt_solver, int precision,
                int max_batch);
  ~CentroidalMPC();
  CentroidalMPC(const CentroidalMPC&) = delete;
  CentroidalMPC& operator=(const CentroidalMPC&) = delete;

  void SetupMPC();

  /* Returns the forces in the caller's vector type (per leg a 3 x N column-major block). */
  template <class Vec>
  Vec UpdateMPC(const Vec& state, const Vec& des_state, const Vec& des_inputs) {
    Vec out;
    out.resize((decltype(out.size()))OutputSize());
    UpdateMPCRaw(state.data(), (size_t)state.size(), des_state.data(), (size_t)des_state.size(), des_inputs.data(),
                 (size_t)des_inputs.size(), out.data());
    return out;
  }
  template <class Vec>
  void UpdateWeights(const Vec& weights) {
    UpdateWeightsRaw(weights.data(), (size_t)weights.size());
  }

  /* raw-array forms: out[OutputSize()] */
  int OutputSize() const { return model_.n_legs * 3 * model_.N; }
  void UpdateMPCRaw(const double* state, size_t n_state, const double* des_state, size_t n_des_state,
                    const double* des_inputs, size_t n_des_inputs, double* out);
  void UpdateWeightsRaw(const double* weights, size_t n);

  /* Batched extension: device pointers in cmpc_solve_batch's record layout, async on stream. */
  int UpdateMPCBatch(int B, const double* d_x0, const double* d_xref, const double* d_foot, const uint8_t* d_contact,
                     double* d_u, double* d_x, int* d_status, int* d_iters, void* stream);

  /* Batched NLP with the later runs' footholds as decision variables (cmpc_nlp_solve_batch): device pointers in
   * cmpc_solve_batch's record layout plus d_feet [B][N+1][L][3]; the SQP limits of setNonlinear. */
  int UpdateNLPBatch(int B, const double* d_x0, const double* d_xref, const double* d_foot, const uint8_t* d_contact,
                     double* d_u, double* d_feet, double* d_x, int* d_status, int* d_qp_iters, int* d_sqp_iters,
                     void* stream);

  /* Feedback policy dU/dx0 of each QP at its solution d_u (cmpc_policy_batch; the condensed counterpart of
   * HpipmInterface::getRiccatiFeedback, HpipmInterface.cpp:330-455): d_K [B][N][L][3][13]. */
  int FeedbackPolicyBatch(int B, const double* d_x0, const double* d_xref, const double* d_foot,
                          const uint8_t* d_contact, const double* d_u, double act_tol, double* d_K, int* d_nfree,
                          int* d_status, void* stream);

  /* The 13-state record UpdateMPC builds from the reference's flat layouts (exposed for tests). */
  template <class Vec>
  void PackRecord(const Vec& state, const Vec& des_state, const Vec& des_inputs, std::vector<double>& x0,
                  std::vector<double>& xref, std::vector<double>& foot, std::vector<uint8_t>& contact) const {
    PackRecordRaw(state.data(), (size_t)state.size(), des_state.data(), (size_t)des_state.size(), des_inputs.data(),
                  (size_t)des_inputs.size(), x0, xref, foot, contact);
  }
  void PackRecordRaw(const double* state, size_t n_state, const double* des_state, size_t n_des_state,
                     const double* des_inputs, size_t n_des_inputs, std::vector<double>& x0, std::vector<double>& xref,
                     std::vector<double>& foot, std::vector<uint8_t>& contact) const;

  /* Nonlinear mode: UpdateMPC solves the NLP with foothold variables (SQP: at most sqp_iter_max iterations,
   * ocs2's deltaTol = sqp_tol). */
  void setNonlinear(bool on, int sqp_iter_max = 10, double sqp_tol = 1e-6) {
    nonlinear_ = on;
    sqp_iter_max_ = sqp_iter_max;
    sqp_tol_ = sqp_tol;
  }
  bool nonlinear() const { return nonlinear_; }
  /* The controller's foot_pos outputs of the last UpdateMPC (CentroidalMPC.cpp:269-273): per leg a 3 x (N+1)
   * column-major block, legs concatenated. Node 0 and a stance run from step 0 at the current foot, free swing nodes
   * at des_foot_pos, a later stance run at its foothold (QP mode: the frozen mean of des_foot_pos over the run). */
  const std::vector<double>& FootPositions() const { return foot_pos_; }

  int lastStatus() const { return last_status_; }
  int lastIterations() const { return last_iters_; }  // IPM iterations (all SQP subproblems in nonlinear mode)
  int lastSqpIterations() const { return last_sqp_iters_; }
  double currentTime() const { return current_time_; }
  const cmpc_model& model() const { return model_; }
  void setSettings(const cmpc_settings& s);

 private:
  void FrozenFeet(const std::vector<double>& foot, const std::vector<uint8_t>& contact,
                  std::vector<double>& feet) const;
  cmpc_model model_;
  cmpc_settings settings_;
  int precision_;
  int max_batch_;
  cmpc_ctx* ctx_ = nullptr;
  double current_time_ = 0.0;
  int last_status_ = -1;
  int last_iters_ = 0;
  int last_sqp_iters_ = 0;
  bool nonlinear_ = false;
  int sqp_iter_max_ = 10;
  double sqp_tol_ = 1e-6;
  std::vector<double> foot_pos_;
};
