// CentroidalMPC.cpp — host mirror of the reference CentroidalMPC (CentroidalMPC.cpp:21-370) over the C ABI.
#include "cheeta_mpc/CentroidalMPC.h"

#include <cassert>
#include <cmath>
#include <cstring>
#include <string>

namespace {
void check(int r, const char* what) {
  if (r != CMPC_OK) throw std::runtime_error(std::string("[CentroidalMPC] ") + what + ": " + cmpc_error_string(r));
}
}  // namespace

CentroidalMPC::CentroidalMPC(double mass, int num_legs, int predict_horizon, double time_step, const double* weights,
                             size_t n_weights, const double* mu, size_t n_mu, IPOPT_SOLVER /*ipopt_solver*/,
                             int precision, int max_batch)
    : precision_(precision), max_batch_(max_batch) {
  // CentroidalMPC.cpp:24-25
  if (!(mass > 0 && num_legs > 0 && predict_horizon > 0)) throw std::invalid_argument("[CentroidalMPC] bad arguments");
  if ((int)n_mu != num_legs) throw std::invalid_argument("[CentroidalMPC] mu.size() != num_legs");
  if (num_legs != CMPC_MAX_LEGS) throw std::invalid_argument("[CentroidalMPC] this build supports num_legs == 4");
  if ((int)n_weights != (num_legs + 1) * 9) throw std::invalid_argument("[CentroidalMPC] weights size");
  cmpc_model_default(&model_, predict_horizon);
  model_.mass = mass;
  model_.dt = time_step;
  model_.n_legs = num_legs;
  for (int i = 0; i < num_legs; ++i) model_.mu[i] = mu[(size_t)i];
  for (int i = 0; i < CMPC_NUM_WEIGHTS; ++i) model_.weights[i] = weights[(size_t)i];
  model_.force_ub[4] = mass * 9.81 * num_legs;  // CentroidalMPC.cpp:183
  cmpc_settings_default(&settings_);
  current_time_ = 0.0;
}

CentroidalMPC::~CentroidalMPC() {
  if (ctx_) cmpc_destroy(ctx_);
}

void CentroidalMPC::SetupMPC() {
  if (ctx_) cmpc_destroy(ctx_);
  ctx_ = nullptr;
  check(cmpc_create(&model_, &settings_, precision_, max_batch_, nullptr, &ctx_), "cmpc_create");
}

void CentroidalMPC::UpdateWeightsRaw(const double* weights, size_t n) {
  if ((int)n != CMPC_NUM_WEIGHTS) throw std::invalid_argument("[CentroidalMPC] weights size");
  for (int i = 0; i < CMPC_NUM_WEIGHTS; ++i) model_.weights[i] = weights[(size_t)i];
  if (ctx_) check(cmpc_set_model(ctx_, &model_), "cmpc_set_model");
}

void CentroidalMPC::setSettings(const cmpc_settings& s) {
  settings_ = s;
  if (ctx_) check(cmpc_set_settings(ctx_, &settings_), "cmpc_set_settings");
}

void CentroidalMPC::PackRecordRaw(const double* state, size_t n_state, const double* des_state, size_t n_des_state,
                                  const double* des_inputs, size_t n_des_inputs, std::vector<double>& x0,
                                  std::vector<double>& xref, std::vector<double>& foot,
                                  std::vector<uint8_t>& contact) const {
  const int N = model_.N, L = model_.n_legs;
  if ((int)n_state < 9 + 3 * L || (int)n_des_state < 9 * (N + 1) || (int)n_des_inputs < L * (4 * N + 3))
    throw std::invalid_argument("[CentroidalMPC] input vector sizes");
  x0.assign(CMPC_NX, 0.0);
  for (int j = 0; j < 9; ++j) x0[(size_t)j] = state[(size_t)j];  // c, v, L (CentroidalMPC.cpp:284-286)
  x0[12] = -9.81;
  xref.assign((size_t)(N + 1) * CMPC_NX, 0.0);
  for (int k = 0; k <= N; ++k) {
    for (int b = 0; b < 3; ++b)  // des_com_pos | des_com_vel | des_angular_momentum, 3x(N+1) column-major (:297-299)
      for (int d = 0; d < 3; ++d) xref[(size_t)k * CMPC_NX + 3 * b + d] = des_state[(size_t)b * 3 * (N + 1) + 3 * k + d];
    xref[(size_t)k * CMPC_NX + 12] = -9.81;
  }
  foot.assign((size_t)(N + 1) * L * 3, 0.0);
  contact.assign((size_t)N * L, 0);
  for (int i = 0; i < L; ++i) {
    const size_t base = (size_t)i * (4 * N + 3);  // [contact_enable (N) | des_foot_pos 3x(N+1)] (:315-317)
    for (int k = 0; k < N; ++k) contact[(size_t)k * L + i] = des_inputs[base + k] > 0 ? 1 : 0;
    // node 0: cur_foot_pos = state[9+3i..] (:288-291), to which the reference pins foot_pos(:,0) (:165-167); its
    // des_foot_pos column only enters a constant tracking term. Nodes 1..N: des_foot_pos.
    for (int d = 0; d < 3; ++d) foot[(size_t)i * 3 + d] = state[(size_t)(9 + 3 * i + d)];
    for (int k = 1; k <= N; ++k)
      for (int d = 0; d < 3; ++d) foot[((size_t)k * L + i) * 3 + d] = des_inputs[base + N + 3 * k + d];
  }
}

void CentroidalMPC::UpdateMPCRaw(const double* state, size_t n_state, const double* des_state, size_t n_des_state,
                                 const double* des_inputs, size_t n_des_inputs, double* out) {
  if (!ctx_) throw std::runtime_error("[CentroidalMPC] SetupMPC() not called");
  const int N = model_.N, L = model_.n_legs;
  std::vector<double> x0, xref, foot;
  std::vector<uint8_t> contact;
  PackRecordRaw(state, n_state, des_state, n_des_state, des_inputs, n_des_inputs, x0, xref, foot, contact);
  for (int k = 0; k < N; ++k) {  // CentroidalMPC.cpp:326-330
    int ns = 0;
    for (int i = 0; i < L; ++i) ns += contact[(size_t)k * L + i];
    if (ns <= 0) throw std::runtime_error("mpc table invalid");
  }
  std::vector<double> u((size_t)N * CMPC_NU);
  std::vector<double> feet((size_t)(N + 1) * L * 3);
  int status = -1, iters = 0, sqp_iters = 0;
  if (nonlinear_) {
    check(cmpc_nlp_solve_batch_host(ctx_, 1, x0.data(), xref.data(), foot.data(), contact.data(), sqp_iter_max_,
                                    sqp_tol_, u.data(), feet.data(), nullptr, &status, &iters, &sqp_iters),
          "cmpc_nlp_solve_batch_host");
  } else {
    check(cmpc_solve_batch_host(ctx_, 1, x0.data(), xref.data(), foot.data(), contact.data(), u.data(), nullptr,
                                &status, &iters),
          "cmpc_solve_batch_host");
    FrozenFeet(foot, contact, feet);
  }
  last_status_ = status;
  last_iters_ = iters;
  last_sqp_iters_ = sqp_iters;
  foot_pos_.assign((size_t)L * 3 * (N + 1), 0.0);  // per leg 3 x (N+1) column-major (controller_ output order)
  for (int i = 0; i < L; ++i)
    for (int j = 0; j <= N; ++j)
      for (int d = 0; d < 3; ++d) foot_pos_[(size_t)i * 3 * (N + 1) + 3 * j + d] = feet[((size_t)j * L + i) * 3 + d];
  current_time_ += model_.dt;  // CentroidalMPC.cpp:368
  // per leg: contact_force_i as 3 x N column-major (controller_ output order)
  for (int i = 0; i < L; ++i)
    for (int k = 0; k < N; ++k)
      for (int d = 0; d < 3; ++d) out[(size_t)i * 3 * N + 3 * k + d] = u[((size_t)k * L + i) * 3 + d];
}

// foot_pos of the QP mode (cmpc.h cmpc_nlp_solve_batch semantics with the footholds frozen): node 0 and a run from
// step 0 at the current foot, a later run's nodes at p_s + sum_j (p_j - p_s) / cnt over its nodes s..e+1 (the
// lever-arm point the QP uses), free swing nodes at des_foot_pos.
void CentroidalMPC::FrozenFeet(const std::vector<double>& foot, const std::vector<uint8_t>& contact,
                               std::vector<double>& feet) const {
  const int N = model_.N, L = model_.n_legs;
  auto ct = [&](int k, int i) { return contact[(size_t)k * L + i] != 0; };
  for (int j = 0; j <= N; ++j)
    for (int i = 0; i < L; ++i) {
      const int k = (j < N && ct(j, i)) ? j : ((j > 0 && ct(j - 1, i)) ? j - 1 : -1);
      double* o = &feet[((size_t)j * L + i) * 3];
      const double* des = &foot[((size_t)j * L + i) * 3];
      for (int d = 0; d < 3; ++d) o[d] = des[d];
      if (j == 0 || k < 0) continue;
      int s = k;
      while (s > 0 && ct(s - 1, i)) --s;
      int e = k;
      while (e + 1 < N && ct(e + 1, i)) ++e;
      const double* ps = &foot[((size_t)s * L + i) * 3];
      for (int d = 0; d < 3; ++d) o[d] = ps[d];
      if (s == 0) continue;
      for (int d = 0; d < 3; ++d) {
        double acc = 0.0;
        for (int jj = s + 1; jj <= e + 1; ++jj) acc += foot[((size_t)jj * L + i) * 3 + d] - ps[d];
        o[d] = ps[d] + acc / (double)(e + 2 - s);
      }
    }
}

int CentroidalMPC::FeedbackPolicyBatch(int B, const double* d_x0, const double* d_xref, const double* d_foot,
                                       const uint8_t* d_contact, const double* d_u, double act_tol, double* d_K,
                                       int* d_nfree, int* d_status, void* stream) {
  if (!ctx_) return CMPC_ERR_ARG;
  return cmpc_policy_batch(ctx_, B, d_x0, d_xref, d_foot, d_contact, d_u, act_tol, d_K, d_nfree, d_status, stream);
}

int CentroidalMPC::UpdateMPCBatch(int B, const double* d_x0, const double* d_xref, const double* d_foot,
                                  const uint8_t* d_contact, double* d_u, double* d_x, int* d_status, int* d_iters,
                                  void* stream) {
  if (!ctx_) return CMPC_ERR_ARG;
  return cmpc_solve_batch(ctx_, B, d_x0, d_xref, d_foot, d_contact, d_u, d_x, d_status, d_iters, stream);
}

int CentroidalMPC::UpdateNLPBatch(int B, const double* d_x0, const double* d_xref, const double* d_foot,
                                  const uint8_t* d_contact, double* d_u, double* d_feet, double* d_x, int* d_status,
                                  int* d_qp_iters, int* d_sqp_iters, void* stream) {
  if (!ctx_) return CMPC_ERR_ARG;
  return cmpc_nlp_solve_batch(ctx_, B, d_x0, d_xref, d_foot, d_contact, sqp_iter_max_, sqp_tol_, d_u, d_feet, d_x,
                              d_status, d_qp_iters, d_sqp_iters, stream);
}
