// cmpc_device.hpp — device-side shared definitions for the CDNA4 (gfx950) kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cmpc/cmpc.h"

namespace cmpc {

constexpr int NX = CMPC_NX;  // 13-state SRBD
constexpr int NU = CMPC_NU;  // 12 contact-force inputs
constexpr int NL = CMPC_MAX_LEGS;
constexpr int MAXN = 63;           // longest horizon the device model table holds
constexpr int GAIT_HALF_PERIOD = 5;
constexpr double GRAV = 9.81;      // CentroidalMPC.cpp:70-73, :333
constexpr double THR0 = 1.0;       // IPM cold-start slack clip
constexpr double TAU = 0.995;      // fraction-to-boundary

// Model constants, derived once on the host (cmpc_set_model) and read through the scalar cache.
struct DevModel {
  int N, L;
  double mass, dt, dt_over_m;
  double inv_inertia[9];
  double mu[NL];
  double Wf[NU];             // force tracking weights   w[9+3L+3i+c]  (CentroidalMPC.cpp:223-225)
  double Wr[NU];             // force-rate weights       w[9+6L+3i+c]  (CentroidalMPC.cpp:227-231)
  double Wp[NU];             // foot position weights    w[9+3i+c]     (CentroidalMPC.cpp:218-221)
  double qdiag[MAXN + 1][NX];// 2*diag(Q_k) incl. squared CoM-z weight (CentroidalMPC.cpp:203-210)
  double ub[5];              // pyramid row upper bounds (CentroidalMPC.cpp:182-183)
};

// IPM settings (cmpc_settings, doubles widened for both precisions)
struct DevSettings {
  int iter_max;
  double alpha_min, mu0, tol_stat, tol_ineq, tol_comp, reg_prim;
};

// ---------------------------------------------------------------------------- wave-level helpers (wave64)

__device__ __forceinline__ double readlane(double x, int lane) {
  const int2 v = __builtin_bit_cast(int2, x);
  int2 r;
  r.x = __builtin_amdgcn_readlane(v.x, lane);
  r.y = __builtin_amdgcn_readlane(v.y, lane);
  return __builtin_bit_cast(double, r);
}
__device__ __forceinline__ float readlane(float x, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), lane));
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  return v;
}

// Accurate reciprocal square root: hardware estimate + Newton refinement (to ~1 ulp).
__device__ __forceinline__ double rsqrt_acc(double d) {
  double y = __builtin_amdgcn_rsq(d);
  double h = d * y;
  double r = fma(-h, y, 1.0);
  y = fma(0.5 * y, r, y);
  h = d * y;
  r = fma(-h, y, 1.0);
  y = fma(0.5 * y, r, y);
  return y;
}
__device__ __forceinline__ float rsqrt_acc(float d) {
  float y = __builtin_amdgcn_rsqf(d);
  float h = d * y;
  float r = fmaf(-h, y, 1.0f);
  return fmaf(0.5f * y, r, y);
}

// Lever-arm point of leg `leg` at a stance step k: the reference's foot_pos[leg] node k. A stance foot does not move
// (foot_pos+ = foot_pos + (1 - e) foot_vel dt, CentroidalMPC.cpp:93), so one position holds over a stance run's nodes
// s..e+1 (steps s..e in stance). Record node 0 is the current foot position (state[9+3i..], :288-291), to which the
// reference pins foot_pos(:,0) (:165-167): a run that starts at step 0 stays there. A later run (touch-down after a
// swing step) has a free position in the reference NLP; the QP freezes it at the minimiser of the foot tracking cost
// w9..w20 (:218-221) under the pinning, the mean of des_foot_pos over nodes s..e+1, formed as p_s + sum (p_j - p_s)/cnt
// so that a planted (constant) run returns p_s bit for bit. oracle_stance_point restates this operation for operation.
// st(k, leg) -> stance flag of step k.
template <typename StanceFn>
__device__ __forceinline__ void stance_point(const double* foot, int N, int k, int leg, StanceFn st, double p[3]) {
  int s = k;
  while (s > 0 && st(s - 1, leg)) --s;
  const double* ps = foot + (s * NL + leg) * 3;
  p[0] = ps[0];
  p[1] = ps[1];
  p[2] = ps[2];
  if (s == 0) return;
  int e = k;
  while (e + 1 < N && st(e + 1, leg)) ++e;
  double d0 = 0.0, d1 = 0.0, d2 = 0.0;
  for (int j = s + 1; j <= e + 1; ++j) {
    const double* pj = foot + (j * NL + leg) * 3;
    d0 += pj[0] - p[0];
    d1 += pj[1] - p[1];
    d2 += pj[2] - p[2];
  }
  const double cnt = (double)(e + 2 - s);
  p[0] += d0 / cnt;
  p[1] += d1 / cnt;
  p[2] += d2 / cnt;
}
// Same, stance flags from one QP's contact record [N][NL].
__device__ __forceinline__ void stance_point(const double* foot, const uint8_t* ct, int N, int k, int leg,
                                             double p[3]) {
  stance_point(foot, N, k, leg, [ct](int kk, int l) { return ct[kk * NL + l] != 0; }, p);
}

// Footholds as decision variables (cmpc_nlp_solve_batch; oracle/cmpc_oracle.c oracle_foot_box & co.): a LATER stance
// run of leg `leg` (first step s >= 1 after a swing step, last stance step e) holds one free foothold over its nodes
// s..e+1, p = pbar + delta with pbar = stance_point (the mean of des over the nodes); D [N][NL][3] holds delta at
// (s, leg). Step box of the NLP (CentroidalMPC.cpp:30-31, :196-198): lo_d = max_j (des_jd - pbar_d) + step_lb_d,
// hi_d = min_j (des_jd - pbar_d) + step_ub_d over j = s..e+1.
__device__ __forceinline__ double step_lb(int d) { return d < 2 ? CMPC_STEP_LB_XY : CMPC_STEP_LB_Z; }
__device__ __forceinline__ double step_ub(int d) { return d < 2 ? CMPC_STEP_UB_XY : CMPC_STEP_UB_Z; }

// First step of the stance run holding stance step k of leg (0: the pinned first run).
template <typename StanceFn>
__device__ __forceinline__ int run_start(int k, int leg, StanceFn st) {
  int s = k;
  while (s > 0 && st(s - 1, leg)) --s;
  return s;
}
// 1 when step s starts a later run of leg; *e = its last stance step.
template <typename StanceFn>
__device__ __forceinline__ bool later_start(int N, int s, int leg, StanceFn st, int* e) {
  if (s < 1 || s >= N || !st(s, leg) || st(s - 1, leg)) return false;
  int ee = s;
  while (ee + 1 < N && st(ee + 1, leg)) ++ee;
  *e = ee;
  return true;
}
// Box component d of the later run (s, leg) ending at e; pbar from stance_point.
__device__ __forceinline__ void foot_box_d(const double* des, int s, int e, int leg, int d, const double* pbar,
                                           double* lo, double* hi) {
  double mx = -__builtin_inf(), mn = __builtin_inf();
  for (int j = s; j <= e + 1; ++j) {
    const double v = des[(j * NL + leg) * 3 + d] - pbar[d];
    mx = v > mx ? v : mx;
    mn = v < mn ? v : mn;
  }
  *lo = mx + step_lb(d);
  *hi = mn + step_ub(d);
}
// Lever-arm point with the run's foothold offset: stance_point + D[s][leg] for a later run (D null: frozen).
template <typename StanceFn>
__device__ __forceinline__ void lever_point(const double* foot, const double* D, int N, int k, int leg, StanceFn st,
                                            double p[3]) {
  stance_point(foot, N, k, leg, st, p);
  if (!D) return;
  const int s = run_start(k, leg, st);
  if (s == 0) return;
  const double* dl = D + (s * NL + leg) * 3;
  p[0] = p[0] + dl[0];
  p[1] = p[1] + dl[1];
  p[2] = p[2] + dl[2];
}

// Friction pyramid row rho of F(mu) applied to (fx, fy, fz)  (CentroidalMPC.cpp:186-190)
template <typename T>
__device__ __forceinline__ T pyr_row(int rho, T mu, T fx, T fy, T fz) {
  const T mz = mu * fz;
  switch (rho) {
    case 0: return mz - fx;
    case 1: return mz + fx;
    case 2: return mz - fy;
    case 3: return mz + fy;
    default: return fz;
  }
}

// Issue priority falls with the QP's progress: 3 for iterations 0-1, 2 for 2-3, 1 for 4-5, 0 from 6 on. Two waves
// share a SIMD; at equal priority the older one takes the issue slots and the younger gets the leftovers, so the
// two slots of a SIMD drift apart (lab timeline, B = 4096: the older wave's QP 145 us, the younger's up to 230 us)
// and the launch ends with one wave per SIMD for ~60 us. Letting the less advanced QP win arbitration keeps the
// pair closer together: k_ipm64 0.411 -> 0.396 ms in the lab (per-iteration thirds and a round-aware variant measured
// within 1 % of this); iterates are bit-identical.
__device__ __forceinline__ void progress_prio(int it) {
  const int pr = 3 - min(3, it >> 1);
  if (pr == 3) __builtin_amdgcn_s_setprio(3);
  else if (pr == 2) __builtin_amdgcn_s_setprio(2);
  else if (pr == 1) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}

// Result scatter of one QP into the caller's arrays from the IPM kernel's epilogue (the fused path without rollout;
// k_misc.hip:expand_one is the stand-alone k_expand form; layout of CentroidalMPC.cpp:337-345): out_u[q] =
// [N][4][3] doubles, zero for swing legs and everywhere for a QP without a solution (n = 0), variable i at
// (tri_map[i / 3], i % 3); out_status[q], out_iters[q]. Every thread of the QP's group calls it (tid < nthr); thread
// i < n supplies variable i; buf: >= out_nu entries of LDS the group no longer reads; sync: the group's barrier.
template <typename T, typename Args, typename Sync>
__device__ __forceinline__ void scatter_result(const Args& a, int q, int n, T ui, int status, int iters, T* buf,
                                               int tid, int nthr, Sync sync) {
  const int nu = a.out_nu;
  for (int p = tid; p < nu; p += nthr) buf[p] = T(0);
  sync();
  if (tid < n) buf[a.tri_map[(size_t)q * (a.ld / 3) + tid / 3] * 3 + tid % 3] = ui;
  sync();
  double* uo = a.out_u + (size_t)q * nu;
  for (int p = tid; p < nu; p += nthr) uo[p] = (double)buf[p];
  if (tid == 0) {
    a.out_status[q] = status;
    if (a.out_iters) a.out_iters[q] = iters;
  }
}

}  // namespace cmpc
