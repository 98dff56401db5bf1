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

}  // namespace cmpc
