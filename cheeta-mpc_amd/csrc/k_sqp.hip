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
// sequential pass (13 states x N steps) over the QP's data staged in LDS by the whole wave first (View: the lever-arm
// points and Theta blocks precomputed once instead of per pass); the step, the convergence test and the next
// linearisation point are then lane-parallel over the 12 N inputs.
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

// One QP's read-only data, staged in LDS by the whole wave before the sequential per-lane passes (each lane's rollout
// is a long dependent chain; from LDS its operands arrive in tens of cycles instead of a global-load latency each):
// x0, xref, des foot table, contact flags, the lever-arm point of every stance (k, leg) (stance_point), the first step
// of its run, dt-free Theta blocks s2 = I_b^-1 R_z(psi_k)^T per step (the oracle's s2, same operations), and the
// iterate / QP solution forces and foothold offsets. Dynamic LDS, sqp_lds_bytes(N).
struct View {
  double *x0, *xr, *des, *pb, *S2, *u0, *u1, *D0, *D1;
  double* lt;  // k_sqp_step only: the CoM path c_k [N][3] of the rollouts of lanes 0..3 and 14 (trial_slot)
  uint8_t* ct;
  int* rs;
};

// k_sqp_step: the rollouts of alpha = 1, 1/2, 1/4, 1/8 (lanes 0..3) and of the current iterate (lane 14) keep their
// CoM path in View::lt (3 N doubles each: the LDS stays small enough for every QP of a 4096 batch to be resident)
constexpr int SQP_TRIALS = 5;
__device__ __forceinline__ int trial_slot(int lane) { return lane < 4 ? lane : (lane == 14 ? 4 : -1); }

__host__ __device__ inline size_t sqp_lds_doubles(int N, bool trial) {
  return 16 + (size_t)(N + 1) * (NX + NL * 3) + (size_t)N * (NL * 3 + 9 + 4 * NU) +
         (trial ? (size_t)SQP_TRIALS * N * 3 : 0);
}
__host__ __device__ inline size_t sqp_lds_bytes(int N, bool trial) {
  return sqp_lds_doubles(N, trial) * 8 + (size_t)N * NL * (sizeof(int) + 1);
}

__device__ View carve(unsigned char* sm, int N, bool trial) {
  View V;
  double* p = reinterpret_cast<double*>(sm);
  V.x0 = p; p += 16;
  V.xr = p; p += (N + 1) * NX;
  V.des = p; p += (N + 1) * NL * 3;
  V.pb = p; p += N * NL * 3;
  V.S2 = p; p += N * 9;
  V.u0 = p; p += N * NU;
  V.u1 = p; p += N * NU;
  V.D0 = p; p += N * NU;
  V.D1 = p; p += N * NU;
  V.lt = p; p += trial ? SQP_TRIALS * N * 3 : 0;
  V.rs = reinterpret_cast<int*>(p);
  V.ct = reinterpret_cast<uint8_t*>(V.rs + N * NL);
  return V;
}

// Stage QP q (every thread of the block calls: it syncs inside; u1 / D0 / D1 may be null: not staged). The caller
// syncs before reading.
__device__ View stage(const SqpArgs& a, int q, unsigned char* sm, const double* u0, const double* u1, const double* D0,
                      const double* D1, bool trial = false) {
  const DevModel* M = a.model;
  const int N = M->N, lane = threadIdx.x, nth = blockDim.x;
  View V = carve(sm, N, trial);
  const double* xr = a.xref + (size_t)q * (N + 1) * NX;
  const double* ft = a.foot + (size_t)q * (N + 1) * NL * 3;
  const uint8_t* ct = a.contact + (size_t)q * N * NL;
  for (int i = lane; i < NX; i += nth) V.x0[i] = a.x0[(size_t)q * NX + i];
  for (int i = lane; i < (N + 1) * NX; i += nth) V.xr[i] = xr[i];
  for (int i = lane; i < (N + 1) * NL * 3; i += nth) V.des[i] = ft[i];
  for (int i = lane; i < N * NL; i += nth) V.ct[i] = ct[i];
  for (int i = lane; i < N * NU; i += nth) {
    V.u0[i] = u0[i];
    if (u1) V.u1[i] = u1[i];
    if (D0) V.D0[i] = D0[i];
    if (D1) V.D1[i] = D1[i];
  }
  // lever-arm points and run starts from the LDS copies of the record (their loops walk back along a stance run: one
  // LDS latency per step instead of a global one)
  __syncthreads();
  const uint8_t* cl = V.ct;
  auto st = [cl](int k, int l) { return cl[k * NL + l] != 0; };
  for (int sl = lane; sl < N * NL; sl += nth) {
    const int k = sl / NL, i = sl % NL;
    double p[3] = {0.0, 0.0, 0.0};
    int s0 = 0;
    if (cl[sl]) {
      stance_point(V.des, N, k, i, st, p);
      s0 = run_start(k, i, st);
    }
    for (int d = 0; d < 3; ++d) V.pb[sl * 3 + d] = p[d];
    V.rs[sl] = s0;
  }
  for (int k = lane; k < N; k += nth) {
    double sp, cp;
    sincos(V.xr[k * NX + 11], &sp, &cp);
    const double RzT[9] = {cp, sp, 0.0, -sp, cp, 0.0, 0.0, 0.0, 1.0};
    for (int r = 0; r < 3; ++r)
      for (int b = 0; b < 3; ++b) {
        double s2 = 0.0;
        for (int e = 0; e < 3; ++e) s2 += M->inv_inertia[r * 3 + e] * RzT[e * 3 + b];
        V.S2[k * 9 + r * 3 + b] = s2;
      }
  }
  return V;
}

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
__device__ double foot_cost(const DevModel* M, const View& V, const double* D1, double alpha, bool deriv) {
  const int N = M->N;
  const uint8_t* ct = V.ct;
  auto st = [ct](int k, int l) { return ct[k * NL + l] != 0; };
  double J = 0.0;
  for (int i = 0; i < NL; ++i)
    for (int s = 1; s < N; ++s) {
      int e = 0;
      if (!later_start(N, s, i, st, &e)) continue;
      const double* pb = V.pb + (s * NL + i) * 3;  // stance_point of the run
      double dl[3];
      trial_offset(V.D0, deriv ? nullptr : D1, alpha, s, i, dl);
      for (int j = s; j <= e + 1; ++j)
        for (int d = 0; d < 3; ++d) {
          const double ed = (pb[d] + dl[d]) - V.des[(j * NL + i) * 3 + d];
          if (deriv)
            J += 2.0 * M->Wp[3 * i + d] * ed * (D1[(s * NL + i) * 3 + d] - dl[d]);
          else
            J += M->Wp[3 * i + d] * ed * ed;
        }
    }
  return J;
}

// Nonlinear rollout + NLP cost of the inputs u0 + alpha (u1 - u0) (has_u1 false: u0) and, with footholds (feet), the
// later runs' footholds D0 + alpha (D1 - D0) (has_u1 false: D0) in the lever arm plus their tracking cost. Writes
// lin [N][6] and x [(N+1)][13] when non-null. Mirrors oracle_nlp_rollout_cost_feet operation for operation.
__device__ double rollout_cost(const DevModel* M, const View& V, bool has_u1, double alpha, double* lin, double* xo,
                               bool feet, double* cpath = nullptr) {
  const int N = M->N;
  const double dt = M->dt;
  const double* u0 = V.u0;
  const double* u1 = has_u1 ? V.u1 : nullptr;
  const double* D1 = has_u1 ? V.D1 : nullptr;
  double xs[NX], xn[NX];
  for (int s = 0; s < NX; ++s) xs[s] = V.x0[s];
  if (xo)
    for (int s = 0; s < NX; ++s) xo[s] = xs[s];
  double J = 0.0;
  double unext[NU];
  auto input = [&](int k, int j) -> double {
    const double a = u0[k * NU + j];
    return u1 ? a + alpha * (u1[k * NU + j] - a) : a;
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
      if (!V.ct[k * NL + i]) continue;
      ++ns;
      double p[3];
      for (int d = 0; d < 3; ++d) p[d] = V.pb[(k * NL + i) * 3 + d];
      const int s0 = V.rs[k * NL + i];
      if (feet && s0 > 0) {
        double dl[3];
        trial_offset(V.D0, D1, alpha, s0, i, dl);
        p[0] = p[0] + dl[0];
        p[1] = p[1] + dl[1];
        p[2] = p[2] + dl[2];
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
    if (cpath)
      for (int d = 0; d < 3; ++d) cpath[k * 3 + d] = xs[d];
    for (int j = 0; j < NU; ++j) {
      const int i = j / 3;
      const double fd = (j % 3 == 2 && V.ct[k * NL + i] && ns > 0) ? M->mass * GRAV / (double)ns : 0.0;
      const double e = uk[j] - fd;
      J += M->Wf[j] * e * e;
      if (k + 1 < N) {
        const double r = unext[j] - uk[j];
        J += M->Wr[j] * r * r;
      }
    }
    for (int d = 0; d < 3; ++d) xn[d] = xs[d] + dt * xs[3 + d];
    xn[3] = xs[3] + dt * (F[0] / M->mass);
    xn[4] = xs[4] + dt * (F[1] / M->mass);
    xn[5] = xs[5] + dt * (xs[12] + F[2] / M->mass);
    for (int d = 0; d < 3; ++d) xn[6 + d] = xs[6 + d] + dt * Tq[d];
    for (int r = 0; r < 3; ++r) {
      double m = 0.0;
      for (int b = 0; b < 3; ++b) m += dt * V.S2[k * 9 + r * 3 + b] * xs[6 + b];
      xn[9 + r] = xs[9 + r] + m;
    }
    xn[12] = xs[12];
    for (int s = 0; s < NX; ++s) xs[s] = xn[s];
    if (xo)
      for (int s = 0; s < NX; ++s) xo[(size_t)(k + 1) * NX + s] = xs[s];
    for (int s = 0; s < NX; ++s) {
      const double e = xs[s] - V.xr[(k + 1) * NX + s];
      J += 0.5 * M->qdiag[k + 1][s] * e * e;
    }
  }
  if (feet) J += foot_cost(M, V, D1, alpha, false);
  return J;
}

// Linearised response of the rollout of u0 to du = u1 - u0 (and, with footholds, dD = D1 - D0) and the descent metric
// (MultipleShootingSolver.cpp:287-296): mirrors oracle_nlp_linstep_feet operation for operation. Returns |dx|
// (trajectoryNorm, :492-503) in dxn.
__device__ double linstep_metric(const DevModel* M, const View& V, double* dxn, bool feet) {
  const int N = M->N;
  const double dt = M->dt;
  const double* u0 = V.u0;
  const double* u1 = V.u1;
  double xs[NX], xn[NX], dx[NX], dn[NX];
  for (int s = 0; s < NX; ++s) {
    xs[s] = V.x0[s];
    dx[s] = 0.0;
  }
  double ss = 0.0, mt = 0.0;
  for (int k = 0; k < N; ++k) {
    const double* uk = u0 + k * NU;
    double duk[NU];
    for (int j = 0; j < NU; ++j) duk[j] = u1[k * NU + j] - uk[j];
    double F[3] = {0.0, 0.0, 0.0}, Tq[3] = {0.0, 0.0, 0.0}, dF[3] = {0.0, 0.0, 0.0}, dT[3] = {0.0, 0.0, 0.0};
    int ns = 0;
    for (int i = 0; i < NL; ++i) {
      if (!V.ct[k * NL + i]) continue;
      ++ns;
      double p[3], dp[3] = {0.0, 0.0, 0.0};
      for (int d = 0; d < 3; ++d) p[d] = V.pb[(k * NL + i) * 3 + d];
      const int s0 = V.rs[k * NL + i];
      if (feet && s0 > 0)
        for (int d = 0; d < 3; ++d) {
          const double a = V.D0[(s0 * NL + i) * 3 + d];
          p[d] = p[d] + a;
          dp[d] = V.D1[(s0 * NL + i) * 3 + d] - a;
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
      const double fd = (j % 3 == 2 && V.ct[k * NL + i] && ns > 0) ? M->mass * GRAV / (double)ns : 0.0;
      double gu = 2.0 * M->Wf[j] * (uk[j] - fd);
      if (k > 0) gu += 2.0 * M->Wr[j] * (uk[j] - u0[(k - 1) * NU + j]);
      if (k + 1 < N) gu -= 2.0 * M->Wr[j] * (u0[(k + 1) * NU + j] - uk[j]);
      mt += gu * duk[j];
    }
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
    for (int r = 0; r < 3; ++r) {
      double m = 0.0, dm = 0.0;
      for (int b = 0; b < 3; ++b) {
        const double s2 = V.S2[k * 9 + r * 3 + b];
        m += dt * s2 * xs[6 + b];
        dm += dt * s2 * dx[6 + b];
      }
      xn[9 + r] = xs[9 + r] + m;
      dn[9 + r] = dx[9 + r] + dm;
    }
    xn[12] = xs[12];
    dn[12] = dx[12];
    for (int s = 0; s < NX; ++s) {
      xs[s] = xn[s];
      dx[s] = dn[s];
    }
    for (int s = 0; s < NX; ++s) {
      mt += M->qdiag[k + 1][s] * (xs[s] - V.xr[(k + 1) * NX + s]) * dx[s];
      ss += dx[s] * dx[s];
    }
  }
  if (feet) mt += foot_cost(M, V, V.D1, 0.0, true);
  *dxn = sqrt(ss);
  return mt;
}

extern __shared__ __attribute__((aligned(16))) unsigned char sqp_lds[];

// Lab instrumentation (-DCMPC_SQP_STAMPS, lab/sqp_stamps.sh only, never in libcmpc.so): k_sqp_step's per-wave
// shader-clock cycles per phase (both waves) summed over every QP into sqp_stamp_acc (cmpc_sqp_debug_stamps):
// 0 staging, 1 the wave's own pass (wave 0: rollouts, wave 1: linearised response + |du|), 2 waiting for the other
// wave, 5 selection + update, 6 next linearisation point; 15 the number of waves.
#ifdef CMPC_SQP_STAMPS
__device__ unsigned long long sqp_stamp_acc[16];
#define SQ_DECL                                                 \
  unsigned long long sq_acc_[7] = {0, 0, 0, 0, 0, 0, 0};         \
  unsigned long long sq_prev_ = __builtin_amdgcn_s_memtime()
#define SQ(id)                                                  \
  do {                                                          \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    sq_acc_[id] += now_ - sq_prev_;                             \
    sq_prev_ = now_;                                            \
  } while (0)
#define SQ_STORE()                                                                      \
  do {                                                                                  \
    if ((threadIdx.x & 63) == 0) {                                                      \
      for (int k_ = 0; k_ < 7; ++k_) atomicAdd(&sqp_stamp_acc[k_ + 8 * (threadIdx.x >> 6)], sq_acc_[k_]); \
      atomicAdd(&sqp_stamp_acc[15], 1ull);                                              \
    }                                                                                   \
  } while (0)
#else
#define SQ_DECL (void)0
#define SQ(id) (void)0
#define SQ_STORE() (void)0
#endif

// U_j <- the cold QP's solution, lin <- its rollout; QPs the cold QP rejected are done from the start. With footholds
// the offsets start at clamp(0, lo, hi) (oracle_feet_init).
__global__ __launch_bounds__(64) void k_sqp_init(SqpArgs a) {
  const int q = blockIdx.x;
  const DevModel* M = a.model;
  const int N = M->N;
  const int nu = N * NU;
  const double* uc = a.u + (size_t)q * nu;
  for (int i = threadIdx.x; i < nu; i += 64) a.uj[(size_t)q * nu + i] = uc[i];
  View V = stage(a, q, sqp_lds, uc, nullptr, nullptr, nullptr);
  const bool feet = a.dj != nullptr;
  if (feet) {
    const double* ft = a.foot + (size_t)q * (N + 1) * NL * 3;
    const uint8_t* ct = a.contact + (size_t)q * N * NL;
    double* dj = a.dj + (size_t)q * nu;
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
        V.D0[sl * 3 + d] = v;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    a.done[q] = a.status[q] != CMPC_SUCCESS ? 1 : 0;
    a.sqp_iters[q] = 0;
    a.qp_iters[q] = a.iters ? a.iters[q] : 0;
    rollout_cost(M, V, false, 0.0, a.lin + (size_t)q * N * 6, nullptr, feet);
  }
}

// One SQP step for every QP not yet done, after the QP at lin returned uq / status_q / iters_q. Two waves: wave 0 runs
// the line search's rollouts, wave 1 (on another SIMD, at the same time) the linearised response and the step norm.
__global__ __launch_bounds__(128) void k_sqp_step(SqpArgs a) {
  const int q = blockIdx.x;
  if (a.done[q]) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const DevModel* M = a.model;
  const int N = M->N;
  const int nu = N * NU;
  double* uj = a.uj + (size_t)q * nu;
  const double* uq = a.uq + (size_t)q * nu;
  const bool feet = a.dj != nullptr;  // footholds (cmpc_nlp_solve_batch)
  double* dj = feet ? a.dj + (size_t)q * nu : nullptr;
  const double* dq = feet ? a.dq + (size_t)q * nu : nullptr;
  if (tid == 0) {
    a.sqp_iters[q] += 1;
    a.qp_iters[q] += a.iters_q[q];
  }
  if (a.status_q[q] != CMPC_SUCCESS) {  // keep U_j, report the subproblem's status (oracle_sqp_solve)
    if (tid == 0) {
      a.status[q] = a.status_q[q];
      a.done[q] = 1;
    }
    return;
  }
  __shared__ double xch[3];  // wave 1 -> wave 0: descent metric, |dx|, |du|
  __shared__ int xma;        // wave 0 -> all: the accepted trial (-1: none)
  SQ_DECL;
  View V = stage(a, q, sqp_lds, uj, uq, dj, dq, true);
  __syncthreads();
  SQ(0);
  // wave 0: lanes m < 14 trial step alpha = 2^-m, lane 14 the current iterate as the trial alpha = 0 (u0 + 0 (u1 - u0)
  // is u0 exactly, so one convergent pass serves both); wave 1: lane 0 |dx| and the descent metric, lane 1 |du|
  // (sequential, the oracle's order). Lanes 0..3 and 14 keep their rollout's CoM path: when the accepted trial is one
  // of them (or no step is taken) the next linearisation point is copied out instead of rolled out again (the iterate
  // u0 + alpha (u1 - u0) is formed by the same operations as the trial's inputs, so its rollout is the trial's bit for
  // bit; F_k is re-summed lane-parallel in the rollout's order)
  double J = 0.0;
  if (wave == 0) {
    const int ts = trial_slot(lane);
    double* cp = ts >= 0 ? V.lt + (size_t)ts * N * 3 : nullptr;
    if (lane < 15) J = rollout_cost(M, V, true, lane < 14 ? ldexp(1.0, -lane) : 0.0, nullptr, nullptr, feet, cp);
  } else if (lane == 0) {
    double dxn = 0.0;
    const double mt = linstep_metric(M, V, &dxn, feet);
    xch[0] = mt;
    xch[1] = dxn;
  } else if (lane == 1) {
    double s2 = 0.0;
    for (int i = 0; i < nu; ++i) {
      const double d = V.u1[i] - V.u0[i];
      s2 += d * d;
    }
    if (feet)
      for (int i = 0; i < nu; ++i) {
        const double d = V.D1[i] - V.D0[i];
        s2 += d * d;
      }
    xch[2] = sqrt(s2);
  }
  SQ(1);
  __syncthreads();
  SQ(2);
  const double tol = a.tol;
  if (wave == 0) {
    const double metric = xch[0], dxn = xch[1], dun = xch[2];
    const double J0 = __shfl(J, 14, 64);
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
    const bool conv = alpha == 0.0 || fabs(Jn - J0) < SQP_COST_TOL || (alpha * dxn < tol && alpha * dun < tol);
    if (lane == 0) {
      xma = ma;
      if (conv) a.done[q] = 1;
    }
  }
  __syncthreads();
  const int ma = xma;
  const double alpha = ma >= 0 ? ldexp(1.0, -ma) : 0.0;
  if (alpha > 0.0)
    for (int i = tid; i < nu; i += 128) {
      const double un = V.u0[i] + alpha * (V.u1[i] - V.u0[i]);
      uj[i] = un;
      V.u0[i] = un;
      if (feet) {
        const double dn = V.D0[i] + alpha * (V.D1[i] - V.D0[i]);
        dj[i] = dn;
        V.D0[i] = dn;
      }
    }
  __syncthreads();
  SQ(5);
  const int sel = trial_slot(ma >= 0 ? ma : 14);
  if (sel >= 0) {
    const double* cs = V.lt + (size_t)sel * N * 3;
    double* lo = a.lin + (size_t)q * N * 6;
    for (int i = tid; i < N * 6; i += 128) {
      const int k = i / 6, d = i % 6;
      double v;
      if (d < 3) {
        v = cs[k * 3 + d];
      } else {
        v = 0.0;
        for (int l = 0; l < NL; ++l)
          if (V.ct[k * NL + l]) v += V.u0[k * NU + 3 * l + (d - 3)];
      }
      lo[i] = v;
    }
  } else if (tid == 0) {
    rollout_cost(M, V, false, 0.0, a.lin + (size_t)q * N * 6, nullptr, feet);
  }
  SQ(6);
  SQ_STORE();
}

// Final outputs: u <- U_j, x <- its nonlinear rollout, the foot_pos table (footholds), status stays.
__global__ __launch_bounds__(64) void k_sqp_final(SqpArgs a) {
  const int q = blockIdx.x;
  const DevModel* M = a.model;
  const int N = M->N;
  const int nu = N * NU;
  const double* ujq = a.uj + (size_t)q * nu;
  for (int i = threadIdx.x; i < nu; i += 64) a.u[(size_t)q * nu + i] = ujq[i];
  const bool feet = a.dj != nullptr;
  View V = stage(a, q, sqp_lds, ujq, nullptr, feet ? a.dj + (size_t)q * nu : nullptr, nullptr);
  __syncthreads();
  if (feet && a.feet)  // the controller's foot_pos output (oracle_feet_table)
    for (int sl = threadIdx.x; sl < (N + 1) * NL; sl += 64) {
      const int j = sl / NL, i = sl % NL;
      const int k = (j < N && V.ct[j * NL + i]) ? j : ((j > 0 && V.ct[(j - 1) * NL + i]) ? j - 1 : -1);
      double p[3];
      if (j == 0 || k < 0) {
        for (int d = 0; d < 3; ++d) p[d] = V.des[sl * 3 + d];
      } else {
        for (int d = 0; d < 3; ++d) p[d] = V.pb[(k * NL + i) * 3 + d];
        const int s0 = V.rs[k * NL + i];
        if (s0 > 0)
          for (int d = 0; d < 3; ++d) p[d] = p[d] + V.D0[(s0 * NL + i) * 3 + d];
      }
      double* o = a.feet + ((size_t)q * (N + 1) * NL + sl) * 3;
      for (int d = 0; d < 3; ++d) o[d] = p[d];
    }
  if (threadIdx.x == 0 && a.x) rollout_cost(M, V, false, 0.0, nullptr, a.x + (size_t)q * (N + 1) * NX, feet);
}

// lin <- (c_k, F_k) of the nonlinear rollout of u (the point cmpc_sqp_policy_batch linearises the QP at).
__global__ __launch_bounds__(64) void k_sqp_lin(SqpArgs a) {
  const int q = blockIdx.x;
  const DevModel* M = a.model;
  const int N = M->N;
  View V = stage(a, q, sqp_lds, a.u + (size_t)q * N * NU, nullptr, nullptr, nullptr);
  __syncthreads();
  if (threadIdx.x == 0) rollout_cost(M, V, false, 0.0, a.lin + (size_t)q * N * 6, nullptr, false);
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
  if (a.N < 1 || a.N > MAXN) return -1;
  const size_t lds = sqp_lds_bytes(a.N, false);
  switch (which) {
    case 0: hipLaunchKernelGGL(k_sqp_init, dim3(B), dim3(64), lds, stream, a); break;
    case 1: hipLaunchKernelGGL(k_sqp_step, dim3(B), dim3(128), sqp_lds_bytes(a.N, true), stream, a); break;
    case 2: hipLaunchKernelGGL(k_sqp_final, dim3(B), dim3(64), lds, stream, a); break;
    case 3: hipLaunchKernelGGL(k_sqp_count, dim3(1), dim3(256), 0, stream, a.done, B, a.count); break;
    case 4: hipLaunchKernelGGL(k_sqp_lin, dim3(B), dim3(64), lds, stream, a); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace cmpc

#ifdef CMPC_SQP_STAMPS
extern "C" int cmpc_sqp_debug_stamps(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(cmpc::sqp_stamp_acc), sizeof(unsigned long long) * 16) != hipSuccess)
    return -2;
  if (reset) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(cmpc::sqp_stamp_acc), z, sizeof(z)) != hipSuccess) return -2;
  }
  return 0;
}
#endif
