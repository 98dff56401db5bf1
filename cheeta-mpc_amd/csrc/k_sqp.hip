// k_sqp.hip — device side of the batched Gauss-Newton SQP on the bilinear centroidal NLP.
//
// The reference's NLP keeps the lever arm bilinear, L+ = L + dt sum_i e_i (p_i - c) x f_i (CentroidalMPC.cpp:86),
// and IPOPT solves it; ocs2's SQP counterpart is MultipleShootingSolver::runImpl (MultipleShootingSolver.cpp:146-214)
// with its line search takeStep (:509-619). Here every QP of the batch iterates (cmpc_sqp_solve_batch, cmpc_api.cpp):
//   lin_j = (c_k, F_k = sum_i e_ik f_ik) of the nonlinear rollout of U_j   (k_sqp_init / k_sqp_step)
//   U_qp  = the condensed QP linearised at lin_j, warm-started from U_j  (the hot path itself, CondenseArgs::lin)
//   takeStep (:509-619) with zero constraint violation (single shooting: the rollout meets the dynamics, so the
//   merit is the NLP cost J, :447): alpha = 1, 1/2, ... while alpha >= alpha_min; Armijo J(U_j + alpha du) <
//   J(U_j) + armijoFactor alpha metric when the descent metric (:287-296) is negative, else J(U_j + alpha du) < J(U_j);
//   after a rejection the search stops once alpha |dx| and alpha |du| are both below deltaTol (:596-604);
//   checkConvergence (:620-645): no step, |J_new - J_j| < costTol, or alpha |dx|, alpha |du| < deltaTol
// with MultipleShootingSettings.h:42-54's defaults and deltaTol = sqp_tol. The restatement is
// oracle/cmpc_oracle.c:oracle_sqp_solve / oracle_nlp_rollout_cost / oracle_nlp_linstep; rollout, cost, linearised
// response and norms follow its floating-point order with contraction off, so the line-search decisions are the
// oracle's.
//
// One wave per QP: lanes 0..13 evaluate the fourteen trial steps 2^-m (2^-13 >= alpha_min = 1e-4 > 2^-14), lane 14
// the current iterate, lane 15 the linearised response |dx| and the descent metric, lane 16 |du|, each lane one whole
// sequential pass (13 states x N steps); the step, the convergence test and the next linearisation point are then
// lane-parallel over the 12 N inputs.
#include <hip/hip_runtime.h>

#include "cmpc/cmpc.h"
#include "cmpc_device.hpp"
#include "cmpc_kernels.hpp"

namespace cmpc {

namespace {

// line search / convergence settings of the SQP: MultipleShootingSettings.h:44-54 defaults (oracle/cmpc_oracle.h)
constexpr double SQP_ALPHA_MIN = 1e-4;  // 2^-13 is the last trial step (lanes 0..13)
constexpr double SQP_ARMIJO = 1e-4;
constexpr double SQP_COST_TOL = 1e-4;

#pragma clang fp contract(off)

// Foothold offset of the later run (s, leg) at the trial point D0 + alpha (D1 - D0) (D1 null: D0).
__device__ __forceinline__ void trial_offset(const double* D0, const double* D1, double alpha, int s, int leg,
                                             double o[3]) {
  for (int d = 0; d < 3; ++d) {
    const double a = D0[(s * NL + leg) * 3 + d];
    o[d] = D1 ? a + alpha * (D1[(s * NL + leg) * 3 + d] - a) : a;
  }
}

// Foot tracking cost of the later runs at the trial footholds D0 + alpha (D1 - D0), or (deriv) its derivative at D0
// along dD = D1 - D0: oracle foot_cost, same loop order (legs, runs by first step, nodes, components).
__device__ double foot_cost(const DevModel* M, const double* foot, const uint8_t* ct, const double* D0,
                            const double* D1, double alpha, bool deriv) {
  const int N = M->N;
  auto st = [ct](int k, int l) { return ct[k * NL + l] != 0; };
  double J = 0.0;
  for (int i = 0; i < NL; ++i)
    for (int s = 1; s < N; ++s) {
      int e = 0;
      if (!later_start(N, s, i, st, &e)) continue;
      double pb[3], dl[3];
      stance_point(foot, N, s, i, st, pb);
      trial_offset(D0, deriv ? nullptr : D1, alpha, s, i, dl);
      for (int j = s; j <= e + 1; ++j)
        for (int d = 0; d < 3; ++d) {
          const double ed = (pb[d] + dl[d]) - foot[(j * NL + i) * 3 + d];
          if (deriv)
            J += 2.0 * M->Wp[3 * i + d] * ed * (D1[(s * NL + i) * 3 + d] - dl[d]);
          else
            J += M->Wp[3 * i + d] * ed * ed;
        }
    }
  return J;
}

// Nonlinear rollout + NLP cost of the inputs u0 + alpha (u1 - u0) (u1 may be null: alpha unused) and, with footholds
// (D0 non-null), the later runs' footholds D0 + alpha (D1 - D0) in the lever arm plus their tracking cost. Writes
// lin [N][6] and x [(N+1)][13] when non-null. Mirrors oracle_nlp_rollout_cost_feet operation for operation.
__device__ double rollout_cost(const DevModel* M, const double* x0, const double* xref, const double* foot,
                               const uint8_t* ct, const double* u0, const double* u1, double alpha, double* lin,
                               double* xo, const double* D0 = nullptr, const double* D1 = nullptr) {
  const int N = M->N;
  const double dt = M->dt;
  double xs[NX], xn[NX];
  for (int s = 0; s < NX; ++s) xs[s] = x0[s];
  if (xo)
    for (int s = 0; s < NX; ++s) xo[s] = xs[s];
  double J = 0.0;
  double unext[NU];
  auto input = [&](int k, int j) -> double {
    const double a = u0[(size_t)k * NU + j];
    return u1 ? a + alpha * (u1[(size_t)k * NU + j] - a) : a;
  };
  for (int j = 0; j < NU; ++j) unext[j] = input(0, j);
  for (int k = 0; k < N; ++k) {
    double uk[NU];
    for (int j = 0; j < NU; ++j) uk[j] = unext[j];
    if (k + 1 < N)
      for (int j = 0; j < NU; ++j) unext[j] = input(k + 1, j);
    double F[3] = {0.0, 0.0, 0.0}, Tq[3] = {0.0, 0.0, 0.0};
    int ns = 0;
    for (int i = 0; i < NL; ++i) {
      if (!ct[k * NL + i]) continue;
      ++ns;
      double p[3];
      stance_point(foot, ct, N, k, i, p);
      if (D0) {
        const int s0 = run_start(k, i, [ct](int kk, int l) { return ct[kk * NL + l] != 0; });
        if (s0 > 0) {
          double dl[3];
          trial_offset(D0, D1, alpha, s0, i, dl);
          p[0] = p[0] + dl[0];
          p[1] = p[1] + dl[1];
          p[2] = p[2] + dl[2];
        }
      }
      const double* f = uk + 3 * i;
      const double rx = p[0] - xs[0], ry = p[1] - xs[1], rz = p[2] - xs[2];
      F[0] += f[0];
      F[1] += f[1];
      F[2] += f[2];
      Tq[0] += ry * f[2] - rz * f[1];
      Tq[1] += rz * f[0] - rx * f[2];
      Tq[2] += rx * f[1] - ry * f[0];
    }
    if (lin)
      for (int d = 0; d < 3; ++d) {
        lin[k * 6 + d] = xs[d];
        lin[k * 6 + 3 + d] = F[d];
      }
    for (int j = 0; j < NU; ++j) {
      const int i = j / 3;
      const double fd = (j % 3 == 2 && ct[k * NL + i] && ns > 0) ? M->mass * GRAV / (double)ns : 0.0;
      const double e = uk[j] - fd;
      J += M->Wf[j] * e * e;
      if (k + 1 < N) {
        const double r = unext[j] - uk[j];
        J += M->Wr[j] * r * r;
      }
    }
    double sp, cp;
    sincos(xref[k * NX + 11], &sp, &cp);
    const double RzT[9] = {cp, sp, 0.0, -sp, cp, 0.0, 0.0, 0.0, 1.0};
    for (int d = 0; d < 3; ++d) xn[d] = xs[d] + dt * xs[3 + d];
    xn[3] = xs[3] + dt * (F[0] / M->mass);
    xn[4] = xs[4] + dt * (F[1] / M->mass);
    xn[5] = xs[5] + dt * (xs[12] + F[2] / M->mass);
    for (int d = 0; d < 3; ++d) xn[6 + d] = xs[6 + d] + dt * Tq[d];
    for (int a = 0; a < 3; ++a) {
      double m = 0.0;
      for (int b = 0; b < 3; ++b) {
        double s2 = 0.0;
        for (int e = 0; e < 3; ++e) s2 += M->inv_inertia[a * 3 + e] * RzT[e * 3 + b];
        m += dt * s2 * xs[6 + b];
      }
      xn[9 + a] = xs[9 + a] + m;
    }
    xn[12] = xs[12];
    for (int s = 0; s < NX; ++s) xs[s] = xn[s];
    if (xo)
      for (int s = 0; s < NX; ++s) xo[(size_t)(k + 1) * NX + s] = xs[s];
    for (int s = 0; s < NX; ++s) {
      const double e = xs[s] - xref[(k + 1) * NX + s];
      J += 0.5 * M->qdiag[k + 1][s] * e * e;
    }
  }
  if (D0) J += foot_cost(M, foot, ct, D0, D1, alpha, false);
  return J;
}

// Linearised response of the rollout of u0 to du = u1 - u0 (and, with footholds, dD = D1 - D0) and the descent metric
// (MultipleShootingSolver.cpp:287-296): mirrors oracle_nlp_linstep_feet operation for operation. Returns |dx|
// (trajectoryNorm, :492-503) in dxn.
__device__ double linstep_metric(const DevModel* M, const double* x0, const double* xref, const double* foot,
                                 const uint8_t* ct, const double* u0, const double* u1, double* dxn,
                                 const double* D0 = nullptr, const double* D1 = nullptr) {
  const int N = M->N;
  const double dt = M->dt;
  double xs[NX], xn[NX], dx[NX], dn[NX];
  for (int s = 0; s < NX; ++s) {
    xs[s] = x0[s];
    dx[s] = 0.0;
  }
  double ss = 0.0, mt = 0.0;
  for (int k = 0; k < N; ++k) {
    const double* uk = u0 + (size_t)k * NU;
    double duk[NU];
    for (int j = 0; j < NU; ++j) duk[j] = u1[(size_t)k * NU + j] - uk[j];
    double F[3] = {0.0, 0.0, 0.0}, Tq[3] = {0.0, 0.0, 0.0}, dF[3] = {0.0, 0.0, 0.0}, dT[3] = {0.0, 0.0, 0.0};
    int ns = 0;
    for (int i = 0; i < NL; ++i) {
      if (!ct[k * NL + i]) continue;
      ++ns;
      double p[3], dp[3] = {0.0, 0.0, 0.0};
      stance_point(foot, ct, N, k, i, p);
      if (D0) {
        const int s0 = run_start(k, i, [ct](int kk, int l) { return ct[kk * NL + l] != 0; });
        if (s0 > 0)
          for (int d = 0; d < 3; ++d) {
            const double a = D0[(s0 * NL + i) * 3 + d];
            p[d] = p[d] + a;
            dp[d] = D1[(s0 * NL + i) * 3 + d] - a;
          }
      }
      const double* f = uk + 3 * i;
      const double* df = duk + 3 * i;
      const double rx = p[0] - xs[0], ry = p[1] - xs[1], rz = p[2] - xs[2];
      F[0] += f[0];
      F[1] += f[1];
      F[2] += f[2];
      Tq[0] += ry * f[2] - rz * f[1];
      Tq[1] += rz * f[0] - rx * f[2];
      Tq[2] += rx * f[1] - ry * f[0];
      dF[0] += df[0];
      dF[1] += df[1];
      dF[2] += df[2];
      const double q0 = dx[0] - dp[0], q1 = dx[1] - dp[1], q2 = dx[2] - dp[2];
      dT[0] += (ry * df[2] - rz * df[1]) - (q1 * f[2] - q2 * f[1]);
      dT[1] += (rz * df[0] - rx * df[2]) - (q2 * f[0] - q0 * f[2]);
      dT[2] += (rx * df[1] - ry * df[0]) - (q0 * f[1] - q1 * f[0]);
    }
    for (int j = 0; j < NU; ++j) {
      const int i = j / 3;
      const double fd = (j % 3 == 2 && ct[k * NL + i] && ns > 0) ? M->mass * GRAV / (double)ns : 0.0;
      double gu = 2.0 * M->Wf[j] * (uk[j] - fd);
      if (k > 0) gu += 2.0 * M->Wr[j] * (uk[j] - u0[(size_t)(k - 1) * NU + j]);
      if (k + 1 < N) gu -= 2.0 * M->Wr[j] * (u0[(size_t)(k + 1) * NU + j] - uk[j]);
      mt += gu * duk[j];
    }
    double sp, cp;
    sincos(xref[k * NX + 11], &sp, &cp);
    const double RzT[9] = {cp, sp, 0.0, -sp, cp, 0.0, 0.0, 0.0, 1.0};
    for (int d = 0; d < 3; ++d) {
      xn[d] = xs[d] + dt * xs[3 + d];
      dn[d] = dx[d] + dt * dx[3 + d];
    }
    xn[3] = xs[3] + dt * (F[0] / M->mass);
    xn[4] = xs[4] + dt * (F[1] / M->mass);
    xn[5] = xs[5] + dt * (xs[12] + F[2] / M->mass);
    dn[3] = dx[3] + dt * (dF[0] / M->mass);
    dn[4] = dx[4] + dt * (dF[1] / M->mass);
    dn[5] = dx[5] + dt * (dx[12] + dF[2] / M->mass);
    for (int d = 0; d < 3; ++d) {
      xn[6 + d] = xs[6 + d] + dt * Tq[d];
      dn[6 + d] = dx[6 + d] + dt * dT[d];
    }
    for (int a = 0; a < 3; ++a) {
      double m = 0.0, dm = 0.0;
      for (int b = 0; b < 3; ++b) {
        double s2 = 0.0;
        for (int e = 0; e < 3; ++e) s2 += M->inv_inertia[a * 3 + e] * RzT[e * 3 + b];
        m += dt * s2 * xs[6 + b];
        dm += dt * s2 * dx[6 + b];
      }
      xn[9 + a] = xs[9 + a] + m;
      dn[9 + a] = dx[9 + a] + dm;
    }
    xn[12] = xs[12];
    dn[12] = dx[12];
    for (int s = 0; s < NX; ++s) {
      xs[s] = xn[s];
      dx[s] = dn[s];
    }
    for (int s = 0; s < NX; ++s) {
      mt += M->qdiag[k + 1][s] * (xs[s] - xref[(k + 1) * NX + s]) * dx[s];
      ss += dx[s] * dx[s];
    }
  }
  if (D0) mt += foot_cost(M, foot, ct, D0, D1, 0.0, true);
  *dxn = sqrt(ss);
  return mt;
}

// U_j <- the cold QP's solution, lin <- its rollout; QPs the cold QP rejected are done from the start.
__global__ __launch_bounds__(64) void k_sqp_init(SqpArgs a) {
  const int q = blockIdx.x;
  const DevModel* M = a.model;
  const int N = M->N;
  const int nu = N * NU;
  for (int i = threadIdx.x; i < nu; i += 64) a.uj[(size_t)q * nu + i] = a.u[(size_t)q * nu + i];
  const double* ft = a.foot + (size_t)q * (N + 1) * NL * 3;
  const uint8_t* ct = a.contact + (size_t)q * N * NL;
  double* dj = a.dj ? a.dj + (size_t)q * nu : nullptr;
  if (dj)  // footholds start at clamp(0, lo, hi) (oracle_feet_init)
    for (int sl = threadIdx.x; sl < N * NL; sl += 64) {
      const int s0 = sl / NL, leg = sl % NL;
      auto st = [ct](int k, int l) { return ct[k * NL + l] != 0; };
      int e = 0;
      double pb[3];
      const bool run = later_start(N, s0, leg, st, &e);
      if (run) stance_point(ft, N, s0, leg, st, pb);
      for (int d = 0; d < 3; ++d) {
        double v = 0.0;
        if (run) {
          double lo, hi;
          foot_box_d(ft, s0, e, leg, d, pb, &lo, &hi);
          v = fmin(fmax(0.0, lo), hi);
        }
        dj[sl * 3 + d] = v;
      }
    }
  __syncthreads();
  if (threadIdx.x == 0) {
    a.done[q] = a.status[q] != CMPC_SUCCESS ? 1 : 0;
    a.sqp_iters[q] = 0;
    a.qp_iters[q] = a.iters ? a.iters[q] : 0;
    rollout_cost(M, a.x0 + (size_t)q * NX, a.xref + (size_t)q * (N + 1) * NX, ft, ct, a.u + (size_t)q * nu, nullptr,
                 0.0, a.lin + (size_t)q * N * 6, nullptr, dj);
  }
}

// One SQP step for every QP not yet done, after the QP at lin returned uq / status_q / iters_q.
__global__ __launch_bounds__(64) void k_sqp_step(SqpArgs a) {
  const int q = blockIdx.x;
  if (a.done[q]) return;
  const int lane = threadIdx.x;
  const DevModel* M = a.model;
  const int N = M->N;
  const int nu = N * NU;
  double* uj = a.uj + (size_t)q * nu;
  const double* uq = a.uq + (size_t)q * nu;
  double* dj = a.dj ? a.dj + (size_t)q * nu : nullptr;  // footholds (cmpc_nlp_solve_batch)
  const double* dq = a.dj ? a.dq + (size_t)q * nu : nullptr;
  const double* x0 = a.x0 + (size_t)q * NX;
  const double* xr = a.xref + (size_t)q * (N + 1) * NX;
  const double* ft = a.foot + (size_t)q * (N + 1) * NL * 3;
  const uint8_t* ct = a.contact + (size_t)q * N * NL;
  if (lane == 0) {
    a.sqp_iters[q] += 1;
    a.qp_iters[q] += a.iters_q[q];
  }
  if (a.status_q[q] != CMPC_SUCCESS) {  // keep U_j, report the subproblem's status (oracle_sqp_solve)
    if (lane == 0) {
      a.status[q] = a.status_q[q];
      a.done[q] = 1;
    }
    return;
  }
  // lanes m < 14: trial step alpha = 2^-m; lane 14: the current iterate; lane 15: |dx| and the descent metric;
  // lane 16: |du| (sequential, the oracle's order)
  double J = 0.0, aux = 0.0;
  if (lane < 14) {
    J = rollout_cost(M, x0, xr, ft, ct, uj, uq, ldexp(1.0, -lane), nullptr, nullptr, dj, dq);
  } else if (lane == 14) {
    J = rollout_cost(M, x0, xr, ft, ct, uj, nullptr, 0.0, nullptr, nullptr, dj, nullptr);
  } else if (lane == 15) {
    J = linstep_metric(M, x0, xr, ft, ct, uj, uq, &aux, dj, dq);
  } else if (lane == 16) {
    double s2 = 0.0;
    for (int i = 0; i < nu; ++i) {
      const double d = uq[i] - uj[i];
      s2 += d * d;
    }
    if (dj)
      for (int i = 0; i < nu; ++i) {
        const double d = dq[i] - dj[i];
        s2 += d * d;
      }
    aux = sqrt(s2);
  }
  const double J0 = __shfl(J, 14, 64);
  const double metric = __shfl(J, 15, 64), dxn = __shfl(aux, 15, 64), dun = __shfl(aux, 16, 64);
  const double tol = a.tol;
  // lane m: accepted (Armijo / decrease), and the early exit after a rejection at alpha = 2^-m (m >= 1)
  const double am = ldexp(1.0, -(lane < 14 ? lane : 0));
  const bool okm = lane < 14 && (metric < 0.0 ? (J < J0 + SQP_ARMIJO * am * metric) : (J < J0));
  const bool exm = lane >= 1 && lane < 14 && am * dxn < tol && am * dun < tol;
  const unsigned long long okb = __ballot(okm), exb = __ballot(exm);
  const int e = exb ? __ffsll((long long)exb) - 1 : 14;  // trials m >= e are never reached
  const unsigned long long reach = okb & ((1ull << e) - 1ull);
  const int ma = reach ? __ffsll((long long)reach) - 1 : -1;
  const double alpha = ma >= 0 ? ldexp(1.0, -ma) : 0.0;
  const double Jn = ma >= 0 ? __shfl(J, ma, 64) : J0;
  __syncthreads();
  if (alpha > 0.0)
    for (int i = lane; i < nu; i += 64) {
      uj[i] = uj[i] + alpha * (uq[i] - uj[i]);
      if (dj) dj[i] = dj[i] + alpha * (dq[i] - dj[i]);
    }
  const bool conv = alpha == 0.0 || fabs(Jn - J0) < SQP_COST_TOL || (alpha * dxn < tol && alpha * dun < tol);
  __syncthreads();
  if (lane == 0) {
    if (conv) a.done[q] = 1;
    rollout_cost(M, x0, xr, ft, ct, uj, nullptr, 0.0, a.lin + (size_t)q * N * 6, nullptr, dj);
  }
}

// Final outputs: u <- U_j, x <- its nonlinear rollout, status stays, iteration counts reported.
__global__ __launch_bounds__(64) void k_sqp_final(SqpArgs a) {
  const int q = blockIdx.x;
  const DevModel* M = a.model;
  const int N = M->N;
  const int nu = N * NU;
  for (int i = threadIdx.x; i < nu; i += 64) a.u[(size_t)q * nu + i] = a.uj[(size_t)q * nu + i];
  const double* ft = a.foot + (size_t)q * (N + 1) * NL * 3;
  const uint8_t* ct = a.contact + (size_t)q * N * NL;
  const double* dj = a.dj ? a.dj + (size_t)q * nu : nullptr;
  if (dj && a.feet)  // the controller's foot_pos output (oracle_feet_table)
    for (int sl = threadIdx.x; sl < (N + 1) * NL; sl += 64) {
      const int j = sl / NL, i = sl % NL;
      auto st = [ct](int k, int l) { return ct[k * NL + l] != 0; };
      const int k = (j < N && ct[j * NL + i]) ? j : ((j > 0 && ct[(j - 1) * NL + i]) ? j - 1 : -1);
      double p[3];
      if (j == 0 || k < 0) {
        for (int d = 0; d < 3; ++d) p[d] = ft[sl * 3 + d];
      } else {
        lever_point(ft, dj, N, k, i, st, p);
      }
      double* o = a.feet + ((size_t)q * (N + 1) * NL + sl) * 3;
      for (int d = 0; d < 3; ++d) o[d] = p[d];
    }
  __syncthreads();
  if (threadIdx.x == 0 && a.x)
    rollout_cost(M, a.x0 + (size_t)q * NX, a.xref + (size_t)q * (N + 1) * NX, ft, ct, a.u + (size_t)q * nu, nullptr,
                 0.0, nullptr, a.x + (size_t)q * (N + 1) * NX, dj);
}

// number of QPs not yet done -> count[0]
__global__ __launch_bounds__(256) void k_sqp_count(const int* done, int B, int* count) {
  int c = 0;
  for (int q = threadIdx.x; q < B; q += 256) c += done[q] ? 0 : 1;
  c = wave_sum(c);
  __shared__ int s[4];
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) count[0] = s[0] + s[1] + s[2] + s[3];
}

}  // namespace

int launch_sqp(int which, const SqpArgs& a, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  switch (which) {
    case 0: hipLaunchKernelGGL(k_sqp_init, dim3(B), dim3(64), 0, stream, a); break;
    case 1: hipLaunchKernelGGL(k_sqp_step, dim3(B), dim3(64), 0, stream, a); break;
    case 2: hipLaunchKernelGGL(k_sqp_final, dim3(B), dim3(64), 0, stream, a); break;
    case 3: hipLaunchKernelGGL(k_sqp_count, dim3(1), dim3(256), 0, stream, a.done, B, a.count); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace cmpc
