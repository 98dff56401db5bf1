#pragma once
// k_ipm128x.hpp — stage 2 of the hot path for the size class 64 < n <= 128 (pronk / all-stance at N <= 10, trot at
// N = 11..21): the same batched dense friction-pyramid QP and primal-dual Mehrotra predictor-corrector as k_ipm64
// (restated in oracle/cmpc_oracle.c:oracle_qp_ipm; settings and stopping rule of hpipm_interface::Settings,
// HpipmInterfaceSettings.h:44-57; replaces d_ocp_qp_ipm_solve at HpipmInterface.cpp:284), with k_ipm64's linear
// algebra spread over one workgroup of four waves.
//
// MI355X mapping — one workgroup of 4 waves per QP (fp64: two workgroups per CU, 2 waves per SIMD; fp32: four):
//   * the Newton matrix K (128 x 128, both triangles) lives in registers: wave w owns the row groups
//     R = 4 rho + w (rho = 0..7, cyclic, so every wave keeps rows below any pivot), lane l = 16a + b holding
//     K[16 rho + 4w + a][16c + b] in register 8 rho + c — 64 values per lane, as k_ipm64's tile per wave;
//   * elimination that builds L^-1 in place (k_ipm64): pivot s, every row i > s and column j != s:
//     K[i][j] -= K[i][s] K[s][j] / d_s. The row multipliers K[i][s] arrive by row_newbcast inside v_fmac_*_dpp
//     (column s sits in lane b = s % 16 of the lane's own 16-lane row); row s+1 is updated first by its owner wave
//     (look-ahead), published in LDS and read by all four waves after one workgroup barrier per pivot;
//   * the pivots run in 16-column chunks c0, a run-time loop (the unrolled code is one chunk long); after every
//     chunk the register tile is rotated by one row group and one column chunk, so the chunk's pivot row group is
//     always register row 0 and its DPP-source column chunk always register column 0 — compile-time register
//     indices under a run-time loop; eight rotations restore the order;
//   * the Newton matrix adds C' Sigma C + reg I from 3x3 block columns staged in LDS by the variable threads;
//   * solves K^-1 y = X' D^-1 X y (X = L^-1, X[i][j] = -S[i][j] / d_j from the strict lower part S): forward row
//     sums and backward column sums over the lower registers (c <= rho), partials reduced through LDS;
//   * one thread per variable (tid < 128) and per pyramid row (tid < 5 n / 3 <= 210); block reductions are DPP
//     wave reductions + 4 partials through LDS.
// Two-wave form (NW = 2, fp32, CMPC_W128=2): the same algorithm with wave w owning the row groups 2 rho + w
// (rows 8 rho + 4w + a, rho = 0..15: 128 tile registers per lane, 2 waves per SIMD), a chunk's pivot rows in register
// rows 0 and 1, the tile rotated by two register rows per chunk, and two pyramid rows per thread; half as many waves
// meet at each pair barrier and each brings twice the bulk FMAs.
#include <type_traits>

#include "cmpc_device.hpp"
#include "cmpc_kernels.hpp"
#include "srbd_condense.hpp"
#include "step_ratio.hpp"
#include "wave_dpp.hpp"

// In-kernel s_memtime stamps (wave 0's view), diagnostic builds only (-DCMPC_IPM_STAMPS; lab/run_lab.sh): per-QP
// cycles into IpmArgs::stamps[q][9]. Segments: 0 H + residuals, 1 Newton matrix, 2 elimination, 3 pivots/mask,
// 4 solves, 5 predictor rest, 6 corrector rest, 7 update, 8 total.
#ifdef CMPC_IPM_STAMPS
#define X_STAMP_DECL                                               \
  unsigned long long xs_acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0};       \
  const unsigned long long xs_t0_ = ipm128x::memtime();            \
  unsigned long long xs_prev_ = xs_t0_
#define X_STAMP(k)                                       \
  do {                                                   \
    const unsigned long long t_ = ipm128x::memtime();    \
    xs_acc_[k] += t_ - xs_prev_;                         \
    xs_prev_ = t_;                                       \
  } while (0)
#define X_STAMP_STORE(ptr, q)                                                   \
  do {                                                                          \
    const unsigned long long t_ = ipm128x::memtime();                           \
    if ((ptr) && threadIdx.x == 0) {                                            \
      for (int k_ = 0; k_ < 8; ++k_) (ptr)[(size_t)(q) * 9 + k_] = xs_acc_[k_]; \
      (ptr)[(size_t)(q) * 9 + 8] = t_ - xs_t0_;                                 \
    }                                                                           \
  } while (0)
#else
#define X_STAMP_DECL (void)0
#define X_STAMP(k) (void)0
#define X_STAMP_STORE(ptr, q) (void)0
#endif

// fp32 elimination bulk on packed FMAs (row_update2); 0 selects the DPP-FMA form (lab A/B builds only)
#ifndef CMPC_PK128
#define CMPC_PK128 1
#endif

namespace cmpc {
namespace ipm128x {
constexpr bool PACKED = CMPC_PK128 != 0;

__device__ __forceinline__ unsigned long long memtime() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

template <typename T>
struct Lim;
template <>
struct Lim<double> {
  static constexpr double pivot_min = 1e-200;
  static constexpr double mu_min = 1e-300;
};
template <>
struct Lim<float> {
  static constexpr float pivot_min = 1e-30f;
  static constexpr float mu_min = 1e-35f;
};

template <int B, int E, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    sfor<B + 1, E>(f);
  }
}

__device__ __forceinline__ double rcp_raw(double x) { return __builtin_amdgcn_rcp(x); }
__device__ __forceinline__ float rcp_raw(float x) { return __builtin_amdgcn_rcpf(x); }
template <typename T>
__device__ __forceinline__ T pivot_inv(T p) {
  T y = rcp_raw(p);
  const T e = fma(-p, y, T(1));
  y = fma(y, e, y);
  return p > T(Lim<T>::pivot_min) ? y : T(0);
}

// k += row_newbcast<B0>(src) * m
template <int B0, typename T>
__device__ __forceinline__ void dfma(T& k, const T& src, T m) {
  if constexpr (sizeof(T) == 8)
    asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(k) : "v"(src), "v"(m), "n"(B0));
  else
    asm volatile("s_nop 1\n\tv_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(k) : "v"(src), "v"(m), "n"(B0));
}
template <int B0, typename T>
__device__ __forceinline__ void dfma_nn(T& k, const T& src, T m) {  // no leading s_nop (caller ordered)
  if constexpr (sizeof(T) == 8)
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(k) : "v"(src), "v"(m), "n"(B0));
  else
    asm volatile("v_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(k) : "v"(src), "v"(m), "n"(B0));
}
template <int B0, typename T>
__device__ __forceinline__ void dfma_self(T& k, T m) {  // the DPP source itself (its lane B0 carries m = 0)
  if constexpr (sizeof(T) == 8)
    asm volatile("v_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "+v"(k) : "v"(m), "n"(B0));
  else
    asm volatile("v_fmac_f32_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "+v"(k) : "v"(m), "n"(B0));
}

__device__ __forceinline__ int olane() {
  int l = (int)threadIdx.x & 63;
  asm volatile("" : "+v"(l));
  return l;
}
__device__ __forceinline__ int owave() {
  int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  asm volatile("" : "+s"(w));
  return w;
}
__device__ __forceinline__ void cbar() { asm volatile("" ::: "memory"); }

// Partial-sum and pivot-row strides, padded so that every LDS access below is bank-conflict free under the MI355X
// banking rules (MI355X_MICROARCH.md §LDS: ds_write_b32 / ds_read_b32 in 32-lane groups on (a/4) mod 32,
// ds_write_b64 in 16-lane groups on (a/4) mod 32, ds_read_b64 in 32-lane groups on (a/4) mod 64):
//   row partials, partial b of row i at b * SR + i: a write instruction covers lanes (a, b) -> rows i0 + a, partials
//     b: (2b + a) mod 32 distinct for fp32 with SR = 2 mod 32; 2 b SR mod 32 distinct for fp64 with SR odd;
//   solve partials, partial p of variable i at p * SB + i: a write covers (p, p + 1) x 16 consecutive variables:
//     fp32 needs SB = 16 mod 32, fp64 (16-lane groups, one p) any SB;
//   pivot rows at row stride RB: a write covers rows (a, a + 1) x 16 consecutive columns: fp32 RB = 16 mod 32;
//   the backward-solve input z at row stride NR + 1 (fp64 writes 16 variables i, i % RG rows apart).
template <typename T>
struct LdsStride {
  static constexpr int SR = sizeof(T) == 4 ? 130 : 129;
  static constexpr int SB = sizeof(T) == 4 ? 144 : 129;
  static constexpr int RB = sizeof(T) == 4 ? 144 : 128;
  static constexpr int SCR = 16 * (SR > SB ? SR : SB);
};

template <typename T>
struct Lds {
  T scr[LdsStride<T>::SCR];  // row / column partial sums (16 per variable; layouts above)
  T rowbuf[2][2][LdsStride<T>::RB];  // pivot-pair rows broadcast (parity double buffer)
  T v[128];         // variable broadcast
  T z[144];         // backward-solve input, permuted [i % RG][i / RG] at row stride NR + 1
  T dg[128];        // pivots
  T w[256];         // pyramid-row broadcast (C' input, Newton block weights)
  T mut[43];        // friction coefficient per triple
  T red[4][4];
  T blk[3][144];     // Newton 3x3 block columns (row stride 16 mod 32: rows e, e + 1 read by one lane group)
  // parked per-row state (one pyramid row per thread)
  T p_lo[256], p_hi[256], p_rl[256], p_ru[256], p_itl[256], p_itu[256], p_rml[256], p_rmu[256];
  T p_tl[256], p_tu[256], p_ll[256], p_lu[256], p_u[128], p_rg[128];  // iterate parked across the elimination
  T p_res[3][256];  // this iteration's residual terms per thread (stat, ineq, comp), reduced at the exit
  T mu_st;          // this iteration's mu for the statistics row
};

}  // namespace ipm128x

// LDS of the 128 class; the fused kernel (k_solve128) runs the workgroup condensing first in the same bytes
template <typename T, bool FUSED>
struct Shared128 {
  ipm128x::Lds<T> ipm;
};
template <typename T>
struct Shared128<T, true> {
  union {
    ipm128x::Lds<T> ipm;
    srbd::SrbdLds<T, 128, 4> cond;
  };
};

// One QP on one workgroup of NW waves (NW = 4: the layout of the header; NW = 2, fp32 only: each wave owns every other
// row group, 128 tile registers per lane, two pyramid rows per thread). FUSED (k_solve128, cold-start
// cmpc_solve_batch, NW = 4): the workgroup condenses the QP first (srbd_condense_qp, which writes H, g and the pyramid
// data to the workspace) and the IPM reads them back after a workgroup barrier (same CU: no round trip through another
// launch); the LDS is one union of both phases.
//
// Layout constants: row group R = NW rho + w of wave w holds rows RG rho + 4 w + a (RG = 4 NW), register rho * 8 + c
// (NR = 32 / NW register rows); a 16-pivot chunk spans CR = 16 / RG register rows; thread tid serves pyramid rows
// tid + NT s (s < PR = 256 / NT).
template <typename T, int MINB, bool FUSED, int NW = 4>
__device__ __forceinline__ void ipm128x_body(const IpmArgs<T>& a, const CondenseArgs<T>* C, const int q) {
  using namespace ipm128x;
  static_assert(NW == 4 || NW == 2, "four or two waves per QP");
  static_assert(!FUSED || NW == 4, "the fused condensing runs on four waves");
  constexpr int NP = 128;
  constexpr int NT = 64 * NW;  // threads
  constexpr int NR = 32 / NW;  // register rows per wave
  constexpr int RG = 4 * NW;   // row stride of a wave's register rows
  constexpr int CR = 16 / RG;  // register rows per 16-pivot chunk
  constexpr int PR = 256 / NT; // pyramid-row slots per thread
  constexpr int NK = NR * 8;   // tile registers per lane
  // declared here, not in the kernel: as a reference from the kernel the LDS accesses lose their constant base
  __shared__ Shared128<T, FUSED> U;
  int n;
  if constexpr (FUSED) {
    // status and n of this QP come from the condensing itself (a uniform re-read of status / nvar would be a
    // scalar-cache load, which does not see the vector stores of this launch)
    n = srbd_condense_qp<T, 128, 4, true>(*C, q, &U.cond);
    if (n < 0) return;
    __syncthreads();  // H, g, pyramid data written by the whole workgroup; the IPM reuses the LDS bytes
  } else {
    if (a.status[q] != CMPC_SUCCESS) return;
    n = a.nvar[q];
  }
  if (n <= 64 || n > NP) return;  // served by another size class
  X_STAMP_DECL;
  const int ld = a.ld;
  const int nt = n / 3;
  const int m = 5 * nt;
  const DevSettings S = a.s;
  Lds<T>& L = U.ipm;

  const int tid = threadIdx.x;
  const int lane0 = tid & 63, wave0 = tid >> 6;
  const int la0 = lane0 >> 4, lb0 = lane0 & 15;

  // ---- variable role (tid < 128) and pyramid-row role (row tid + NT s < m)
  const bool isv = tid < NP;
  const bool var = tid < n;
  const T g_i = var ? a.g[(size_t)q * ld + tid] : T(0);
  const T mu_i = var ? a.tri_mu[(size_t)q * (ld / 3) + tid / 3] : T(0);
  T u_i = (a.warm && var) ? a.u[(size_t)q * ld + tid] : T(0), rg_i = T(0), du_i = T(0);
  auto rowj = [&](int s) { return tid + NT * s; };
  auto con = [&](int s) { return rowj(s) < m; };
#pragma unroll
  for (int s = 0; s < PR; ++s) {
    const int j = rowj(s);
    L.p_lo[j] = con(s) ? a.tri_lo[((size_t)q * (ld / 3) + j / 5) * 5 + j % 5] : T(0);
    L.p_hi[j] = con(s) ? a.tri_hi[((size_t)q * (ld / 3) + j / 5) * 5 + j % 5] : T(0);
  }
  if (tid < 43) L.mut[tid] = tid < nt ? a.tri_mu[(size_t)q * (ld / 3) + tid] : T(0);
  if (isv) L.v[tid] = u_i;
  __syncthreads();
  auto C_row = [&](int s) -> T {
    const int j = rowj(s), tj = j / 5;
    return con(s) ? pyr_row<T>(j % 5, L.mut[tj], L.v[3 * tj], L.v[3 * tj + 1], L.v[3 * tj + 2]) : T(0);
  };
  T tl[PR], tu[PR], ll[PR], lu[PR];
#pragma unroll
  for (int s = 0; s < PR; ++s) {
    const T cu0 = C_row(s);
    tl[s] = con(s) ? fmax(cu0 - L.p_lo[rowj(s)], T(THR0)) : T(1);
    tu[s] = con(s) ? fmax(L.p_hi[rowj(s)] - cu0, T(THR0)) : T(1);
    ll[s] = con(s) ? T(S.mu0) / tl[s] : T(0);
    lu[s] = con(s) ? T(S.mu0) / tu[s] : T(0);
  }
  T dtl[PR], dtu[PR], dll[PR], dlu[PR];
#pragma unroll
  for (int s = 0; s < PR; ++s) dtl[s] = dtu[s] = dll[s] = dlu[s] = T(0);
  __syncthreads();

  // the waves' partials in a fixed association (NW = 4: (0 + 1) + (2 + 3))
  auto red4 = [&](auto op, int k) -> T {
    if constexpr (NW == 4) return op(op(L.red[0][k], L.red[1][k]), op(L.red[2][k], L.red[3][k]));
    else return op(L.red[0][k], L.red[1][k]);
  };
  auto block_sum = [&](T r) -> T {
    r = wave_sum_dpp(r);
    if (lane0 == 0) L.red[wave0][0] = r;
    __syncthreads();
    const T o = red4([](T x, T y) { return x + y; }, 0);
    __syncthreads();
    return o;
  };
  auto block_min = [&](T r) -> T {
    r = wave_min_dpp(r);
    if (lane0 == 0) L.red[wave0][0] = r;
    __syncthreads();
    const T o = red4([](T x, T y) { return fmin(x, y); }, 0);
    __syncthreads();
    return o;
  };
  // (C' w)_i with w in L.w (caller synchronised)
  auto CT_var = [&]() -> T {
    if (!var) return T(0);
    const int t = tid / 3, dd = tid % 3;
    const T w0 = L.w[5 * t], w1 = L.w[5 * t + 1], w2 = L.w[5 * t + 2], w3 = L.w[5 * t + 3], w4 = L.w[5 * t + 4];
    return dd == 0 ? (w1 - w0) : (dd == 1 ? (w3 - w2) : (mu_i * (w0 + w1 + w2 + w3) + w4));
  };

  T K[NK];
  T invd_i = T(1);

  constexpr int SR = LdsStride<T>::SR, SB = LdsStride<T>::SB, RB = LdsStride<T>::RB, ZS = NR + 1;
  // row partial sums of the lane's rows into L.scr (partial b of row i at b * SR + i: conflict-free both ways);
  // FULL = all 8 chunks (H u), else the lower registers c <= (RG rho) / 16 (forward solve). Input chunk values in xc.
  auto row_partials = [&](const T (&xc)[8], auto full_) {
    constexpr bool full = decltype(full_)::value;
    const int ol = olane(), w = owave();
    const int a = ol >> 4, b = ol & 15;
    const int base = b * SR + 4 * w + a;  // row i = RG rho + 4w + a
    sfor<0, NR>([&](auto r_) {
      constexpr int rho = decltype(r_)::value;
      constexpr int ce = full ? 8 : (RG * rho) / 16 + 1;
      T p = K[rho * 8] * xc[0];
      sfor<1, ce>([&](auto c_) {
        constexpr int c = decltype(c_)::value;
        p = fma(K[rho * 8 + c], xc[c], p);
      });
      L.scr[base + RG * rho] = p;
    });
  };
  auto row_sum = [&]() -> T {  // variable tid's 16 partials (caller synchronised)
    T sv = T(0);
    if (isv) {
#pragma unroll
      for (int k = 0; k < 16; k += 2) sv += L.scr[k * SR + tid] + L.scr[(k + 1) * SR + tid];
    }
    return sv;
  };

  // K x = y for the thread's variable (y = 0 outside): see the header
  auto solve = [&](T& y) {
    if (isv) L.v[tid] = y * invd_i;
    __syncthreads();
    {
      const int ol = olane();
      const int b = ol & 15;
      T tc[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) tc[c] = L.v[b + 16 * c];
      row_partials(tc, std::false_type{});
    }
    __syncthreads();
    const T z = (y - row_sum()) * invd_i;
    if (isv) L.z[(tid % RG) * ZS + tid / RG] = z;
    __syncthreads();
    {
      const int ol = olane(), w = owave();
      const int a = ol >> 4, b = ol & 15;
      T zr[NR];
#pragma unroll
      for (int r = 0; r < NR; ++r) zr[r] = L.z[(4 * w + a) * ZS + r];
      sfor<0, 8>([&](auto c_) {
        constexpr int c = decltype(c_)::value;
        constexpr int r0 = c * CR;  // first register row whose diagonal chunk is c
        T qv = K[r0 * 8 + c] * zr[r0];
        sfor<r0 + 1, NR>([&](auto r_) {
          constexpr int rho = decltype(r_)::value;
          qv = fma(K[rho * 8 + c], zr[rho], qv);
        });
        L.scr[(4 * w + a) * SB + c * 16 + b] = qv;
      });
    }
    __syncthreads();
    T qs = T(0);
    if (isv) {
#pragma unroll
      for (int k = 0; k < RG; k += 2) qs += L.scr[k * SB + tid] + L.scr[(k + 1) * SB + tid];
    }
    y = var ? fma(-invd_i, qs, z) : T(0);
    __syncthreads();  // L.scr / L.v are rewritten next
  };

  const T* Hq = a.H + (size_t)q * ld * ld;  // class-packed 128 x 128 block (row-major) at the start of the slab
  int status = CMPC_MAX_ITER;
  int it = 0;

  auto direction = [&]() {
#pragma unroll
    for (int s = 0; s < PR; ++s) {
      const int j = rowj(s);
      const T rl = L.p_rl[j], ru = L.p_ru[j], itl = L.p_itl[j], itu = L.p_itu[j];
      const T rml = L.p_rml[j], rmu = L.p_rmu[j];
      L.w[j] = (rml + ll[s] * rl) * itl - (rmu + lu[s] * ru) * itu;
    }
    __syncthreads();
    const T ctw = CT_var();
    T y = var ? -rg_i - ctw : T(0);
    X_STAMP(5);
    solve(y);
    X_STAMP(4);
    du_i = y;
    if (isv) L.v[tid] = du_i;
    __syncthreads();
#pragma unroll
    for (int s = 0; s < PR; ++s) {
      const int j = rowj(s);
      const T rl = L.p_rl[j], ru = L.p_ru[j], itl = L.p_itl[j], itu = L.p_itu[j];
      const T rml = L.p_rml[j], rmu = L.p_rmu[j];
      const T cdu = C_row(s);
      dtl[s] = con(s) ? cdu + rl : T(0);
      dtu[s] = con(s) ? ru - cdu : T(0);
      dll[s] = -(rml + ll[s] * dtl[s]) * itl;
      dlu[s] = -(rmu + lu[s] * dtu[s]) * itu;
    }
    __syncthreads();  // L.v is rewritten next
  };
  // fraction-to-boundary ratio: the smallest v / (-d) over the thread's candidates with d < 0 is selected by
  // cross-multiplication (v, -d > 0) and divided once (k_ipm64: the per-candidate IEEE divisions cost ~3 %)
  auto max_step = [&]() -> T {
    MinRatio<T> mr;
#pragma unroll
    for (int s = 0; s < PR; ++s) {
      mr.cand(tl[s], dtl[s]);
      mr.cand(tu[s], dtu[s]);
      mr.cand(ll[s], dll[s]);
      mr.cand(lu[s], dlu[s]);
    }
    return block_min(mr.value());
  };

  // residual block maxima of the iteration whose terms are in L.p_res (written before a barrier) and its mu into a
  // statistics row; run by wave 0 only
  auto stats_res = [&](double* sr) {
    T r[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      T v = fmax(fmax(L.p_res[k][lane0], L.p_res[k][lane0 + 64]), fmax(L.p_res[k][lane0 + 128], L.p_res[k][lane0 + 192]));
      r[k] = wave_max_dpp(v);
    }
    if (lane0 == 0) {
      sr[5] = (double)L.mu_st;
      sr[6] = (double)r[0];
      sr[7] = 0.0;
      sr[8] = (double)r[1];
      sr[9] = (double)r[2];
    }
  };
  for (it = 0;; ++it) {
    progress_prio(it);  // cmpc_device.hpp (lab, n = 120 fp64: 3.94 -> 3.91 ms)
    // ---- H: NK loads per lane, 4 rows x 16 consecutive columns per instruction
    {
      const int ol = olane(), w = owave();
      const T* hp = Hq + (size_t)(4 * w + (ol >> 4)) * NP + (ol & 15);
#pragma unroll
      for (int rho = 0; rho < NR; ++rho)
#pragma unroll
        for (int c = 0; c < 8; ++c) K[rho * 8 + c] = hp[RG * rho * NP + 16 * c];
    }
    // ---- residuals: C u, H u
    if (isv) L.v[tid] = u_i;
    __syncthreads();
    T cu[PR];
#pragma unroll
    for (int s = 0; s < PR; ++s) cu[s] = C_row(s);
    {
      const int ol = olane();
      const int b = ol & 15;
      T uc[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) uc[c] = L.v[b + 16 * c];
      row_partials(uc, std::true_type{});
    }
    __syncthreads();
    const T hu = row_sum();
    T ms = T(0);
    bool fin_r = true, ok_r = true;
#pragma unroll
    for (int s = 0; s < PR; ++s) {
      const int j = rowj(s);
      const T lo = L.p_lo[j], hi = L.p_hi[j];
      const T rl = con(s) ? cu[s] - lo - tl[s] : T(0);
      const T ru = con(s) ? hi - cu[s] - tu[s] : T(0);
      L.p_rl[j] = rl;
      L.p_ru[j] = ru;
      const T ri = fmax(fabs(rl), fabs(ru));
      const T cl = tl[s] * ll[s], ch = tu[s] * lu[s];
      const T rc = con(s) ? fmax(cl, ch) : T(0);
      ms += con(s) ? cl + ch : T(0);
      L.w[j] = ll[s] - lu[s];
      L.p_res[1][j] = ri;  // this iteration's residual terms, reduced once at the exit
      L.p_res[2][j] = rc;
      fin_r = fin_r && isfinite(ri) && isfinite(rc);
      ok_r = ok_r && ri <= T(S.tol_ineq) && rc <= T(S.tol_comp);
    }
    __syncthreads();
    {
      const T ctw = CT_var();
      rg_i = isv ? hu + g_i - ctw : T(0);
    }
    const T rs = fabs(rg_i);
#pragma unroll
    for (int s = 0; s < PR; ++s) L.p_res[0][rowj(s)] = s == 0 ? rs : T(0);
    ms = block_sum(ms);
    const T mu = m > 0 ? ms / T(2 * m) : T(0);
    const bool st_on = a.stats && it < a.stats_cap;  // statistics row of this iteration (cmpc_enable_stats)
    auto st_row = [&]() { return a.stats + ((size_t)q * a.stats_cap + it) * CMPC_STAT_COLS; };
    if (st_on && tid == 0) L.mu_st = mu;  // the row's residual part is written at the end of the iteration / the exit
    // non-finite residual anywhere -> NAN_SOL; stopping rule as a block vote (max <= tol iff all <= tol)
    if (__syncthreads_or(!(isfinite(rs) && fin_r))) {
      status = CMPC_NAN_SOL;
      break;
    }
    if (__syncthreads_and(rs <= T(S.tol_stat) && ok_r)) {
      status = CMPC_SUCCESS;
      break;
    }
    if (it >= S.iter_max) {
      status = CMPC_MAX_ITER;
      break;
    }
    if (m > 0 && !(mu > T(Lim<T>::mu_min))) {
      status = CMPC_MIN_STEP;
      break;
    }
    X_STAMP(0);

    // ---- Newton matrix K = H + C' diag(lam_l/t_l + lam_u/t_u) C + reg I: thread j < 128 writes the 3x3 block
    //      column of variable j (rows t3 .. t3 + 2 of its triple), the tile adds it where entry (i, j) falls there
#pragma unroll
    for (int s = 0; s < PR; ++s) {
      const int j = rowj(s);
      const T itl = con(s) ? T(1) / tl[s] : T(0);
      const T itu = con(s) ? T(1) / tu[s] : T(0);
      L.p_itl[j] = itl;
      L.p_itu[j] = itu;
      L.w[j] = ll[s] * itl + lu[s] * itu;
    }
    __syncthreads();
    if (isv) {
      const int t = tid / 3, dd = tid % 3;
      T b0 = T(0), b1 = T(0), b2 = T(0);
      if (var) {
        const T s0 = L.w[5 * t], s1 = L.w[5 * t + 1], s2 = L.w[5 * t + 2], s3 = L.w[5 * t + 3], s4 = L.w[5 * t + 4];
        const T xx = s0 + s1, yy = s2 + s3, zz = mu_i * mu_i * (s0 + s1 + s2 + s3) + s4;
        const T xz = mu_i * (s1 - s0), yz = mu_i * (s3 - s2);
        b0 = dd == 0 ? xx : (dd == 1 ? T(0) : xz);
        b1 = dd == 0 ? T(0) : (dd == 1 ? yy : yz);
        b2 = dd == 0 ? xz : (dd == 1 ? yz : zz);
      }
      const T reg = T(S.reg_prim);
      L.blk[0][tid] = b0 + (dd == 0 ? reg : T(0));
      L.blk[1][tid] = b1 + (dd == 1 ? reg : T(0));
      L.blk[2][tid] = b2 + (dd == 2 ? reg : T(0));
    }
    __syncthreads();
    {
      const int ol = olane(), w = owave();
      const int a = ol >> 4, b = ol & 15;
      // entry (i, j) = (RG rho + 4w + a, 16c + b) is in j's triple iff 0 <= i - 3 (j / 3) <= 2: only registers
      // c = clo .. chi can hold such entries
      sfor<0, NR>([&](auto r_) {
        constexpr int rho = decltype(r_)::value;
        constexpr int lo_ = RG * rho - 17;
        constexpr int clo = lo_ <= 0 ? 0 : (lo_ + 15) / 16;
        constexpr int chi = (RG * rho + RG + 1) / 16 < 7 ? (RG * rho + RG + 1) / 16 : 7;
        sfor<clo, chi + 1>([&](auto c_) {
          constexpr int c = decltype(c_)::value;
          const int j = 16 * c + b;
          const int e = RG * rho + 4 * w + a - 3 * (j / 3);
          const bool in = e >= 0 && e <= 2;
          const T val = L.blk[in ? e : 0][j];
          K[rho * 8 + c] += in ? val : T(0);
        });
      });
    }
    X_STAMP(1);
    // park the per-thread iterate in LDS across the elimination (its registers hold the pivot pairs instead)
#pragma unroll
    for (int s = 0; s < PR; ++s) {
      const int j = rowj(s);
      L.p_tl[j] = tl[s];
      L.p_tu[j] = tu[s];
      L.p_ll[j] = ll[s];
      L.p_lu[j] = lu[s];
    }
    if (isv) {
      L.p_u[tid] = u_i;
      L.p_rg[tid] = rg_i;
    }
    // ---- elimination with L^-1 in place (see the header), 16-pivot chunks. The register tile is rotated by CR
    //      register rows and one column chunk after every chunk (K[rho][c] <- K[rho + CR][c + 1], indices mod NR
    //      and 8), so the chunk's pivot rows are always register rows 0 .. CR - 1 and the pivot column chunk always
    //      register column 0: compile-time register indices under a run-time chunk loop. Eight rotations restore
    //      the order.
    const int nch = (n + 15) >> 4;
    // Pivots in pairs (p = 16 c0 + 2 b, q = p + 1; both rows in the same wave and register row): one barrier and one
    // LDS round trip per pair. Row q gets pivot p from the broadcast copy (xq' = xq + K[q][p] mp, the look-ahead's
    // own FMA), its pivot from uniform LDS reads (d_q = K[q][q] + K[q][p] (-K[p][q] / d_p)): bit-identical to one
    // pivot at a time.
    T mp[8], mq[8];
    // lane coordinates are re-read (olane(): one opaque VALU op) at every use in the elimination: held across it, the
    // compiler spilled lb0 to scratch and reloaded it once per pivot pair (k_solve128<float>)
    // the pair's pivots and their reciprocals: scalar chain, started as soon as the pair's scalars are read so
    // that its latency (two reciprocals in sequence) runs under the bulk FMAs of the previous pair
    auto pair_piv = [&](T dp, T kqp, T kpq, T kqq, int s, T& invp, T& invq) {
      invp = pivot_inv(dp);
      const T dq = fma(kqp, -(kpq * invp), kqq);
      invq = pivot_inv(dq);
      if (tid == 0) {
        L.dg[s] = dp;
        L.dg[s + 1] = dq;
      }
    };
    // multipliers of the pair from the two broadcast rows
    auto pair_vec = [&](const T (&xp)[8], const T (&xq)[8], T kqp, T invp, T invq, auto tp_) {
      constexpr int tp = decltype(tp_)::value, tq = tp + 1;
      const int lbp = olane() & 15;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const T mv = -(xp[c] * invp);
        mp[c] = (c == 0 && lbp == tp) ? T(0) : mv;
        asm volatile("" : "+v"(mp[c]));
      }
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const T x2 = fma(kqp, mp[c], xq[c]);
        const T mv = -(x2 * invq);
        mq[c] = (c == 0 && lbp == tq) ? T(0) : mv;
        asm volatile("" : "+v"(mq[c]));
      }
    };
    // register row rho by the pair (source columns tp, tq of register chunk 0): pass p then pass q
    auto row_update2 = [&](auto rho_, auto tp_) {
      constexpr int rho = decltype(rho_)::value, tp = decltype(tp_)::value, tq = tp + 1;
      if constexpr (sizeof(T) == 4 && PACKED) {
        // fp32: the row multiplier K[i][p] is broadcast once into a register (v_mov_b32_dpp row_newbcast) and the 8
        // column chunks are updated as 4 packed pairs (v_pk_fma_f32, multiplier in both halves): 2 + 8 instructions
        // per register row and pair instead of 16 DPP FMAs (lab/micro/f32_issue.hip: 23.8 vs 10.9-15.3 FMA/clk per
        // SIMD at 4 waves). Column p itself carries mp[0] = 0 in lane p, as in the DPP form.
        typedef float f2 __attribute__((ext_vector_type(2)));
        auto pass = [&](auto tb_, const T (&mv)[8]) {
          constexpr int tb = decltype(tb_)::value;
          const float t = __builtin_bit_cast(
              float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, K[rho * 8]), 0x150 + tb, 0xf, 0xf, false));
          const f2 tt = {t, t};
#pragma unroll
          for (int cp = 0; cp < 4; ++cp) {
            f2 k = {K[rho * 8 + 2 * cp], K[rho * 8 + 2 * cp + 1]};
            const f2 mm = {mv[2 * cp], mv[2 * cp + 1]};
            k = __builtin_elementwise_fma(tt, mm, k);
            K[rho * 8 + 2 * cp] = k.x;
            K[rho * 8 + 2 * cp + 1] = k.y;
          }
        };
        pass(std::integral_constant<int, tp>{}, mp);
        pass(std::integral_constant<int, tq>{}, mq);
        return;
      }
      dfma<tp, T>(K[rho * 8 + 1], K[rho * 8], mp[1]);
      sfor<2, 8>([&](auto c_) {
        constexpr int c = decltype(c_)::value;
        dfma_nn<tp, T>(K[rho * 8 + c], K[rho * 8], mp[c]);
      });
      dfma_self<tp, T>(K[rho * 8], mp[0]);
      dfma<tq, T>(K[rho * 8 + 1], K[rho * 8], mq[1]);
      sfor<2, 8>([&](auto c_) {
        constexpr int c = decltype(c_)::value;
        dfma_nn<tq, T>(K[rho * 8 + c], K[rho * 8], mq[c]);
      });
      dfma_self<tq, T>(K[rho * 8], mq[0]);
    };
    auto read_pair = [&](int buf, T (&xp)[8], T (&xq)[8], T& dp, T& kqp, T& kpq, T& kqq, int tp) {
      const int lb = olane() & 15;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        xp[c] = L.rowbuf[buf][0][16 * c + lb];
        xq[c] = L.rowbuf[buf][1][16 * c + lb];
      }
      dp = L.rowbuf[buf][0][tp];
      kpq = L.rowbuf[buf][0][tp + 1];
      kqp = L.rowbuf[buf][1][tp];
      kqq = L.rowbuf[buf][1][tp + 1];
    };
    for (int c0 = 0; c0 < 8; ++c0) {
      if (c0 < nch) {
        // rows 16 c0, 16 c0 + 1 = wave 0, rows a = 0, 1 of register row 0: final (every earlier pivot applied)
        const int ol0 = olane();
        if (wave0 == 0 && (ol0 >> 4) < 2) {
#pragma unroll
          for (int c = 0; c < 8; ++c) L.rowbuf[0][ol0 >> 4][16 * c + (ol0 & 15)] = K[c];
        }
        __syncthreads();
        {
          T xp[8], xq[8], dp, kqp, kpq, kqq, invp, invq;
          read_pair(0, xp, xq, dp, kqp, kpq, kqq, 0);
          pair_piv(dp, kqp, kpq, kqq, 16 * c0, invp, invq);
          pair_vec(xp, xq, kqp, invp, invq, std::integral_constant<int, 0>{});
        }
        sfor<0, 8>([&](auto b_) {
          constexpr int b = decltype(b_)::value;
          constexpr int tp = 2 * b;  // pivots 16 c0 + tp, + tp + 1
          // next pair (b < 7): chunk row tp + 2 = RG r2 + 4 w2 + a2 (register row r2 of wave w2, rows a2, a2 + 1)
          constexpr int r2 = (tp + 2) / RG, w2 = ((tp + 2) % RG) / 4, a2 = (tp + 2) % 4;
          constexpr int nb = (b + 1) & 1;
          const int wv = owave();
          if constexpr (b < 7) {
            // the chunk's rows below the pair: the next pair's owner first, then its two rows to LDS
            if (wv == w2) {
              if constexpr (a2 == 2) {
                if ((olane() >> 4) >= 2) row_update2(std::integral_constant<int, r2>{}, std::integral_constant<int, tp>{});
              } else {
                row_update2(std::integral_constant<int, r2>{}, std::integral_constant<int, tp>{});
              }
              const int olw = olane();
              if ((olw >> 4) == a2 || (olw >> 4) == a2 + 1) {
#pragma unroll
                for (int c = 0; c < 8; ++c) L.rowbuf[nb][(olw >> 4) - a2][16 * c + (olw & 15)] = K[r2 * 8 + c];
              }
            }
            // every other chunk register row whose rows all lie below the pair
            sfor<0, CR>([&](auto rr_) {
              constexpr int rr = decltype(rr_)::value;
              if (RG * rr + 4 * wv >= tp + 2 && !(rr == r2 && wv == w2))
                row_update2(rr_, std::integral_constant<int, tp>{});
            });
          }
          // next pair published: its first row and pivot scalars are read here, landing while the bulk runs (the
          // second row after it: registers)
          T xp[8], xq[8], dp = T(0), kqp = T(0), kpq = T(0), kqq = T(0), invp = T(0), invq = T(0);
          if constexpr (b < 7) {
#ifdef X_BARRIER_STAMP  // diagnostic: time waiting at the pair barrier (segment 3)
            X_STAMP(2);
            __syncthreads();
            X_STAMP(3);
#else
            __syncthreads();
#endif
            const int lbx = olane() & 15;
#pragma unroll
            for (int c = 0; c < 8; ++c) xp[c] = L.rowbuf[nb][0][16 * c + lbx];
            dp = L.rowbuf[nb][0][tp + 2];
            kpq = L.rowbuf[nb][0][tp + 3];
            kqp = L.rowbuf[nb][1][tp + 2];
            kqq = L.rowbuf[nb][1][tp + 3];
            pair_piv(dp, kqp, kpq, kqq, 16 * c0 + tp + 2, invp, invq);
          }
          // bulk: register rows CR .. NR - 1 - CR c0 (row groups below the chunk), padding groups skipped
          sfor<CR, NR>([&](auto r_) {
            constexpr int rho = decltype(r_)::value;
            if (rho <= NR - 1 - CR * c0 && 16 * c0 + RG * rho < n) row_update2(r_, std::integral_constant<int, tp>{});
          });
          if constexpr (b < 7) {
            const int lby = olane() & 15;
#pragma unroll
            for (int c = 0; c < 8; ++c) xq[c] = L.rowbuf[nb][1][16 * c + lby];
            pair_vec(xp, xq, kqp, invp, invq, std::integral_constant<int, tp + 2>{});
          }
        });
        __syncthreads();  // rowbuf[0] is rewritten by the next chunk's first pair
      }
      // rotate: K[rho][c] <- K[rho + CR][c + 1]
      T K0[NK];
#pragma unroll
      for (int e = 0; e < NK; ++e) K0[e] = K[e];
#pragma unroll
      for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int c = 0; c < 8; ++c) K[r * 8 + c] = K0[((r + CR) % NR) * 8 + ((c + 1) & 7)];
    }
    X_STAMP(2);
#pragma unroll
    for (int s = 0; s < PR; ++s) {
      const int j = rowj(s);
      tl[s] = L.p_tl[j];
      tu[s] = L.p_tu[j];
      ll[s] = L.p_ll[j];
      lu[s] = L.p_lu[j];
    }
    if (isv) {
      u_i = L.p_u[tid];
      rg_i = L.p_rg[tid];
    }
    // pivots beyond the last chunk (n < 16 nch never leaves any: nch covers n) -> padding pivots are 1
    if (isv && tid >= 16 * nch) L.dg[tid] = T(1);
    __syncthreads();
    {
      const T d = isv ? L.dg[tid] : T(1);
      invd_i = pivot_inv(d);
      if (__syncthreads_or(isv && d != d)) {
        status = CMPC_NAN_SOL;
        break;
      }
    }
    // strict lower part only in the diagonal-straddling registers (rho, c = RG rho / 16): keep j < i
    {
      const int w = owave();
      sfor<0, NR>([&](auto r_) {
        constexpr int rho = decltype(r_)::value;
        constexpr int cd = (RG * rho) / 16, off = RG * rho - 16 * cd;
        K[rho * 8 + cd] = (lb0 < off + 4 * w + la0) ? K[rho * 8 + cd] : T(0);
      });
    }

    X_STAMP(3);
    // ---- predictor (affine scaling direction)
#pragma unroll
    for (int s = 0; s < PR; ++s) {
      L.p_rml[rowj(s)] = tl[s] * ll[s];
      L.p_rmu[rowj(s)] = tu[s] * lu[s];
    }
    direction();
    T alpha = fmin(T(1), max_step());
    if (m > 0) {
      T maff = T(0);
#pragma unroll
      for (int s = 0; s < PR; ++s)
        maff += con(s) ? (tl[s] + alpha * dtl[s]) * (ll[s] + alpha * dll[s]) +
                             (tu[s] + alpha * dtu[s]) * (lu[s] + alpha * dlu[s])
                       : T(0);
      maff = block_sum(maff) / T(2 * m);
      const T ratio = maff / mu;
      const T sigma = ratio * ratio * ratio;
      if (st_on && tid == 0) {
        double* sr = st_row();
        sr[0] = (double)alpha;
        sr[1] = (double)maff;
        sr[2] = (double)sigma;
      }
      // ---- corrector: rm = t.lam + dt_aff.dlam_aff - sigma mu
#pragma unroll
      for (int s = 0; s < PR; ++s) {
        L.p_rml[rowj(s)] = con(s) ? tl[s] * ll[s] + dtl[s] * dll[s] - sigma * mu : T(0);
        L.p_rmu[rowj(s)] = con(s) ? tu[s] * lu[s] + dtu[s] * dlu[s] - sigma * mu : T(0);
      }
      direction();
      alpha = fmin(T(1), T(TAU) * max_step());
    }
    X_STAMP(6);
    if (st_on && tid == 0) {
      double* sr = st_row();
      if (m == 0) sr[0] = sr[1] = sr[2] = __builtin_nan("");
      sr[3] = sr[4] = (double)alpha;
    }  // one step length for primal and dual
    if (alpha < T(S.alpha_min)) {
      status = CMPC_MIN_STEP;
      break;
    }
    u_i = fma(alpha, du_i, u_i);
#pragma unroll
    for (int s = 0; s < PR; ++s) {
      tl[s] = fma(alpha, dtl[s], tl[s]);
      tu[s] = fma(alpha, dtu[s], tu[s]);
      ll[s] = fma(alpha, dll[s], ll[s]);
      lu[s] = fma(alpha, dlu[s], lu[s]);
    }
    if (st_on && wave0 == 0) stats_res(st_row());  // this iteration's residuals, still in L.p_res
    X_STAMP(7);
  }

  const bool fin = !var || isfinite(u_i);
  if (__syncthreads_or(fin ? 0 : 1)) status = CMPC_NAN_SOL;
  if (isv && tid < ld) a.u[(size_t)q * ld + tid] = var ? u_i : T(0);
  if (tid == 0) {
    a.status[q] = status;
    a.iters[q] = it;
  }
  if (a.out_u) {  // the pyramid bounds in L.p_lo are dead by now
    __syncthreads();
    scatter_result<T>(a, q, n, u_i, status, it, L.p_lo, tid, NT, [] { __syncthreads(); });
  }
  if (a.stats && it < a.stats_cap) {  // the stopping iteration's row: residuals and mu, no step
    __syncthreads();
    if (wave0 == 0) {
      double* sr = a.stats + ((size_t)q * a.stats_cap + it) * CMPC_STAT_COLS;
      if (lane0 < 5) sr[lane0] = __builtin_nan("");
      stats_res(sr);
    }
  }
  if (a.res) {  // block max of the last residual terms (each thread reads back what it stored)
    T v0 = L.p_res[0][tid], v1 = L.p_res[1][tid], v2 = L.p_res[2][tid];
#pragma unroll
    for (int s = 1; s < PR; ++s) {
      v0 = fmax(v0, L.p_res[0][rowj(s)]);
      v1 = fmax(v1, L.p_res[1][rowj(s)]);
      v2 = fmax(v2, L.p_res[2][rowj(s)]);
    }
    const T r0 = wave_max_dpp(v0), r1 = wave_max_dpp(v1), r2 = wave_max_dpp(v2);
    __syncthreads();
    if (lane0 == 0) {
      L.red[wave0][0] = r0;
      L.red[wave0][1] = r1;
      L.red[wave0][2] = r2;
    }
    __syncthreads();
    if (tid == 0) {
      auto mx = [](T x, T y) { return fmax(x, y); };
      double* o = a.res + (size_t)q * 4;
      o[0] = (double)red4(mx, 0);
      o[1] = 0.0;
      o[2] = (double)red4(mx, 1);
      o[3] = (double)red4(mx, 2);
    }
  }
  X_STAMP_STORE(a.stamps, q);
}

template <typename T, int MINB, int NW = 4>  // MINB workgroups per CU: 2 (fp64, 2 waves per SIMD), 4 (fp32)
__global__ __launch_bounds__(64 * NW, MINB) void k_ipm128x(IpmArgs<T> a) {
  int q = blockIdx.x;
  if (a.qlist[1]) {  // compacted class list: real QPs first, the surplus workgroups exit
    if (q >= a.qcount[1]) return;
    q = a.qlist[1][q];
    if ((unsigned)q >= gridDim.x) return;  // grid = batch: a corrupt list entry cannot address past it
  }
  ipm128x_body<T, MINB, false, NW>(a, nullptr, q);
}

// Fused condensing + IPM of the 64 < n <= 128 class (cold-start cmpc_solve_batch): one launch over the class list
// k_class_lists built from k_solve64's nvar hints.
template <typename T, int MINB>
__global__ __launch_bounds__(256, MINB) void k_solve128(IpmArgs<T> a, CondenseArgs<T> c) {
  int q = blockIdx.x;
  if (q >= a.qcount[1]) return;
  q = a.qlist[1][q];
  if ((unsigned)q >= gridDim.x) return;  // grid = batch: a corrupt list entry cannot address past it
  ipm128x_body<T, MINB, true>(a, &c, q);
}

}  // namespace cmpc
