#pragma once
// k_ipm256.hpp — stage 2 of the hot path, workgroup-tiled IPM k_ipm_tiled<T, NT> for the size class
// 8 NT < n <= 16 NT: NT = 16 serves 128 < n <= 256 (all-stance horizons N = 11..21, e.g. pronk at N = 20: n = 240),
// (the 64 < n <= 128 class runs on k_ipm128x.hpp). Same batched dense friction-pyramid QP and the same primal-dual Mehrotra
// predictor-corrector as k_ipm_reg / k_ipm64 (restated in oracle/cmpc_oracle.c:oracle_qp_ipm; settings and stopping
// rule of hpipm_interface::Settings, HpipmInterfaceSettings.h:44-57); only the linear algebra is organised for a
// matrix too big for one wavefront's registers.
//
// MI355X mapping — one workgroup of NT / 2 waves per QP (NT = 16: 512 threads, 2 waves per SIMD):
//   * the Newton matrix K = H + C' Sigma C (256 x 256, symmetric) lives in registers as 136 lower 16x16 tiles in the
//     C/D layout of the 16x16x4 MFMA (v_mfma_f64_16x16x4_f64 / v_mfma_f32_16x16x4_f32): wave w owns the tile rows
//     w and 15 - w, 17 tiles each (balanced), "slot" s of wave w being tile (w, s) for s <= w, else
//     (15 - w, s - w - 1) — slot indices are compile-time, tile coordinates run-time;
//   * blocked right-looking Cholesky, 16-wide panels: the owner of tile row p factors the diagonal tile in registers
//     (column broadcast through LDS) and inverts the 16 x 16 factor; every wave then forms its panel tile
//     L_ip = A_ip L_pp^-T on the matrix cores and publishes it in an LDS panel (double-buffered by step parity);
//     the trailing update A_ij -= L_ip L_jp' is 4 MFMAs per tile with both operands read from that panel.
//     Two workgroup barriers per panel step;
//   * triangular solves by tile rows: forward with per-lane deferred partial sums (one 16-lane DPP reduction per
//     row tile), backward column-oriented by the owner of each tile row (permlane swaps across row groups);
//     the 16 inverted diagonal tiles stay in LDS for both sweeps;
//   * H u uses the tiles already loaded (rows: deferred 16-lane reductions; columns: permlane reductions), with
//     per-wave partial vectors summed in a fixed order, so results are run-to-run deterministic (no atomics);
//   * one thread per variable (tid < 256) and per pyramid row (tid < 5 n/3 <= 425): the constraint state stays in
//     registers; block reductions are DPP wave reductions + 8 partials through LDS.
#include <type_traits>

#include "cmpc_device.hpp"
#include "cmpc_kernels.hpp"
#include "step_ratio.hpp"
#include "wave_dpp.hpp"

namespace cmpc {
namespace ipm256 {

constexpr int PS = 17;           // LDS row stride of a 16 x 16 tile (bank-conflict padding)
constexpr int TS = 16 * PS;      // LDS tile size

template <typename T>
struct Mf;
template <>
struct Mf<double> {
  typedef double acc_t __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ acc_t run(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  // C/D layout of v_mfma_f64_16x16x4_f64: col = lane & 15, row = (lane >> 4) + 4 * reg
  static __device__ __forceinline__ int row(int lane, int k) { return (lane >> 4) + 4 * k; }
  static constexpr double pivot_min = 1e-200;
  static constexpr double mu_min = 1e-300;
};
template <>
struct Mf<float> {
  typedef float acc_t __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ acc_t run(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  // C/D layout of v_mfma_f32_16x16x4_f32: col = lane & 15, row = 4 * (lane >> 4) + reg
  static __device__ __forceinline__ int row(int lane, int k) { return 4 * (lane >> 4) + k; }
  static constexpr float pivot_min = 1e-30f;
  static constexpr float mu_min = 1e-35f;
};

template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// Lane / wave ids the compiler cannot hoist: every phase re-derives its lane offsets and slot coordinates from these,
// instead of keeping ~17 x 4 tile addresses live in VGPRs (and the slot coordinates in SGPRs) across the iteration.
__device__ __forceinline__ int opaque_lane() {
  int l = (int)threadIdx.x & 63;
  asm volatile("" : "+v"(l));
  return l;
}
__device__ __forceinline__ int opaque_wave() {
  int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  asm volatile("" : "+s"(w));
  return w;
}
#define IPM256_LOCAL_IDS                       \
  const int lane = ipm256::opaque_lane();      \
  const int wave = ipm256::opaque_wave();      \
  const int c16 = lane & 15, g4 = lane >> 4;   \
  (void)c16;                                   \
  (void)g4

// NT tile rows over W = NT / 2 waves, snake order: wave w owns tile rows w and NT - 1 - w (NT + 1 tiles)
template <int NT>
__device__ __forceinline__ int owner(int I) { return I < NT / 2 ? I : NT - 1 - I; }
template <int NT>
__device__ __forceinline__ int slot_I(int w, int s) { return s <= w ? w : NT - 1 - w; }
__device__ __forceinline__ int slot_J(int w, int s) { return s <= w ? s : s - w - 1; }

// one wave's LDS is in order; this orders the compiler and drains LDS before cross-lane reuse
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// sum inside each 16-lane row (every lane of the row gets it)
template <typename T>
__device__ __forceinline__ T row16_sum(T x) {
  x += wdpp::dpp<0xB1>(x);   // quad_perm [1,0,3,2]
  x += wdpp::dpp<0x4E>(x);   // quad_perm [2,3,0,1]
  x += wdpp::dpp<0x124>(x);  // row_ror:4
  x += wdpp::dpp<0x128>(x);  // row_ror:8
  return x;
}
// sum over the four 16-lane rows at the same position (lane & 15)
template <typename T>
__device__ __forceinline__ T cross4_sum(T x) {
  T p0, p1;
  wdpp::swap16(x, p0, p1);
  x = p0 + p1;
  wdpp::swap32(x, p0, p1);
  return p0 + p1;
}

template <typename T, int NT>
struct Lds {
  static constexpr int NP = 16 * NT, W = NT / 2, NTHR = 64 * W;
  T P[2][NT][TS];   // panel tiles of the current step (parity double buffer), row-major stride PS
  T Dinv[NT][TS];   // inverted diagonal factor tiles
  T dg[TS];         // diagonal tile factor (row-major) for the inversion
  T col[16];        // factor column broadcast
  T il[16];         // pivot reciprocals of the tile being factored
  T part[W][NP];    // per-wave partial vectors (H u)
  T vec[NP];        // broadcast vector (C x input, H u input, solve right-hand side / backward result)
  T y[NP];          // forward-solve result
  T acc[NP];        // backward-solve sums
  T tmp[16];
  T w[NTHR];        // constraint-side vector (C' input)
  T mut[NP / 3];    // friction coefficient per triple
  T red[W][4];
  int nanflag;
};

}  // namespace ipm256

template <typename T, int NT>
__global__ __launch_bounds__(32 * NT, 2) void k_ipm_tiled(IpmArgs<T> a) {  // 2 waves per SIMD
  using namespace ipm256;
  using MF = Mf<T>;
  using acc_t = typename MF::acc_t;
  constexpr int NP = 16 * NT;      // class size
  constexpr int W = NT / 2;        // waves per workgroup
  constexpr int NTHR = 64 * W;     // threads
  constexpr int SL = NT + 1;       // tiles (slots) per wave
  static_assert(5 * (NP / 3) <= NTHR, "one thread per pyramid row");

  int q = blockIdx.x;
  if (a.qlist[2]) {  // compacted class list: real QPs first, the surplus workgroups exit
    if (q >= a.qcount[2]) return;
    q = a.qlist[2][q];
    if ((unsigned)q >= gridDim.x) return;  // grid = batch: a corrupt list entry cannot address past it
  }
  if (a.status[q] != CMPC_SUCCESS) return;  // invalid contact table / too large: status already set
  const int n = a.nvar[q];
  if (n <= NP / 2 || n > NP) return;        // served by another size class
  const int ld = a.ld;
  const int nt = n / 3;
  const int m = 5 * nt;
  const DevSettings S = a.s;
  __shared__ Lds<T, NT> L;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c16 = lane & 15, g4 = lane >> 4;

  // ---- variable role (i = tid < 256) and pyramid-row role (j = tid < m); cold start as k_ipm_reg
  const int i = tid;
  const bool isv = tid < NP;
  const bool var = tid < n;
  const T g_i = var ? a.g[(size_t)q * ld + i] : T(0);
  const T mu_i = var ? a.tri_mu[(size_t)q * (ld / 3) + i / 3] : T(0);
  // cold start (warm_start = 0): u = 0; warm start: u from the workspace (cmpc_solve_batch_warm)
  T u_i = (a.warm && var) ? a.u[(size_t)q * ld + i] : T(0), rg_i = T(0), du_i = T(0);
  const int j = tid;
  const bool con = j < m;
  const int tj = j / 5, rj = j % 5;
  const T lo = con ? a.tri_lo[((size_t)q * (ld / 3) + tj) * 5 + rj] : T(0);
  const T hi = con ? a.tri_hi[((size_t)q * (ld / 3) + tj) * 5 + rj] : T(0);
  const T muj = con ? a.tri_mu[(size_t)q * (ld / 3) + tj] : T(0);
  if (isv) L.vec[tid] = u_i;
  __syncthreads();
  const T cu0 = con ? pyr_row<T>(rj, muj, L.vec[3 * tj], L.vec[3 * tj + 1], L.vec[3 * tj + 2]) : T(0);
  T tl = con ? fmax(cu0 - lo, T(THR0)) : T(1);
  T tu = con ? fmax(hi - cu0, T(THR0)) : T(1);
  T ll = con ? T(S.mu0) / tl : T(0);
  T lu = con ? T(S.mu0) / tu : T(0);
  T rl = T(0), ru = T(0), itl = T(0), itu = T(0), dtl = T(0), dtu = T(0), dll = T(0), dlu = T(0), rml = T(0),
    rmu = T(0);
  if (tid < NP / 3) L.mut[tid] = tid < nt ? a.tri_mu[(size_t)q * (ld / 3) + tid] : T(0);
  __syncthreads();  // every thread has read L.vec (initial C u) before the first iteration rewrites it

  // ---- block reduction of (max, max, max, sum)
  auto block_reduce = [&](T& r0, T& r1, T& r2, T& r3) {
    r0 = wave_max_dpp(r0);
    r1 = wave_max_dpp(r1);
    r2 = wave_max_dpp(r2);
    r3 = wave_sum_dpp(r3);
    if (lane == 0) {
      L.red[wave][0] = r0;
      L.red[wave][1] = r1;
      L.red[wave][2] = r2;
      L.red[wave][3] = r3;
    }
    __syncthreads();
    r0 = L.red[0][0], r1 = L.red[0][1], r2 = L.red[0][2], r3 = L.red[0][3];
#pragma unroll
    for (int v = 1; v < W; ++v) {
      r0 = fmax(r0, L.red[v][0]);
      r1 = fmax(r1, L.red[v][1]);
      r2 = fmax(r2, L.red[v][2]);
      r3 += L.red[v][3];
    }
    __syncthreads();
  };
  auto block_min = [&](T r) -> T {
    r = wave_min_dpp(r);
    if (lane == 0) L.red[wave][0] = r;
    __syncthreads();
    T o = L.red[0][0];
#pragma unroll
    for (int v = 1; v < W; ++v) o = fmin(o, L.red[v][0]);
    __syncthreads();
    return o;
  };
  auto block_sum = [&](T r) -> T {
    r = wave_sum_dpp(r);
    if (lane == 0) L.red[wave][0] = r;
    __syncthreads();
    T o = L.red[0][0];
#pragma unroll
    for (int v = 1; v < W; ++v) o += L.red[v][0];
    __syncthreads();
    return o;
  };
  // C x for this thread's pyramid row; x already in L.vec (caller synchronised)
  auto C_row = [&]() -> T {
    return con ? pyr_row<T>(rj, muj, L.vec[3 * tj], L.vec[3 * tj + 1], L.vec[3 * tj + 2]) : T(0);
  };
  // (C' w)_i with w already in L.w (caller synchronised)
  auto CT_var = [&]() -> T {
    if (!var) return T(0);
    const int t = i / 3, dd = i % 3;
    const T w0 = L.w[5 * t], w1 = L.w[5 * t + 1], w2 = L.w[5 * t + 2], w3 = L.w[5 * t + 3], w4 = L.w[5 * t + 4];
    return dd == 0 ? (w1 - w0) : (dd == 1 ? (w3 - w2) : (mu_i * (w0 + w1 + w2 + w3) + w4));
  };

  acc_t K[SL];

  // ---- (L L') x = b: b in L.vec (caller synchronised), x returned in L.vec (synchronised on return)
  auto chol_solve = [&]() {
    // forward L y = b, tile row by tile row; partial sums of the owned rows deferred per lane
    T pa0[4] = {T(0), T(0), T(0), T(0)}, pa1[4] = {T(0), T(0), T(0), T(0)};
    for (int J = 0; J < NT; ++J) {
      IPM256_LOCAL_IDS;
      if (wave == owner<NT>(J)) {
        const bool r0 = (J == wave);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const T t = row16_sum(r0 ? pa0[k] : pa1[k]);
          const int r = MF::row(lane, k);
          if (c16 == 0) L.tmp[r] = L.vec[16 * J + r] - t;
        }
        wave_sync();
        if (lane < 16) {
          const T* Di = &L.Dinv[J][lane * PS];
          T yr = T(0);
#pragma unroll
          for (int c = 0; c < 16; ++c) yr = c <= lane ? fma(Di[c], L.tmp[c], yr) : yr;
          L.y[16 * J + lane] = yr;
        }
      }
      __syncthreads();
      static_for<0, SL>([&](auto s_) {
        constexpr int s = decltype(s_)::value;
        const int I = slot_I<NT>(wave, s), Jt = slot_J(wave, s);
        if (Jt == J && I > J) {
          const T yc = L.y[16 * J + c16];
          if (s <= wave) {
#pragma unroll
            for (int k = 0; k < 4; ++k) pa0[k] = fma(K[s][k], yc, pa0[k]);
          } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) pa1[k] = fma(K[s][k], yc, pa1[k]);
          }
        }
      });
    }
    // backward L' x = y, by the owner of each tile row
    if (isv) L.acc[tid] = T(0);
    __syncthreads();
    for (int I = NT - 1; I >= 0; --I) {
      IPM256_LOCAL_IDS;
      if (wave == owner<NT>(I)) {
        if (lane < 16) L.tmp[lane] = L.y[16 * I + lane] - L.acc[16 * I + lane];
        wave_sync();
        if (lane < 16) {
          T xc = T(0);
#pragma unroll
          for (int r = 0; r < 16; ++r) xc = r >= lane ? fma(L.Dinv[I][r * PS + lane], L.tmp[r], xc) : xc;
          L.vec[16 * I + lane] = xc;
        }
        wave_sync();
        static_for<0, SL>([&](auto s_) {
          constexpr int s = decltype(s_)::value;
          const int It = slot_I<NT>(wave, s), J = slot_J(wave, s);
          if (It == I && J < I) {
            T p = T(0);
#pragma unroll
            for (int k = 0; k < 4; ++k) p = fma(K[s][k], L.vec[16 * I + MF::row(lane, k)], p);
            p = cross4_sum(p);
            if (lane < 16) L.acc[16 * J + lane] += p;
          }
        });
      }
      __syncthreads();
    }
  };

  const T* Hq = a.H + (size_t)q * ld * ld;  // class-packed 256 x 256 block (row-major) at the start of the slab
  int status = CMPC_MAX_ITER;
  int it = 0;

  // Newton direction for the complementarity targets rml / rmu
  auto direction = [&]() {
    L.w[tid] = (rml + ll * rl) * itl - (rmu + lu * ru) * itu;
    __syncthreads();
    const T ctw = CT_var();
    if (isv) L.vec[tid] = var ? -rg_i - ctw : T(0);
    __syncthreads();
    chol_solve();
    du_i = isv ? L.vec[tid] : T(0);
    const T cdu = C_row();
    dtl = con ? cdu + rl : T(0);
    dtu = con ? ru - cdu : T(0);
    dll = -(rml + ll * dtl) * itl;
    dlu = -(rmu + lu * dtu) * itu;
    __syncthreads();  // L.vec is rewritten next
  };
  // fraction-to-boundary ratio: the smallest v / (-d) over the thread's four candidates with d < 0 is selected by
  // cross-multiplication (v, -d > 0) and divided once (k_ipm64: the per-candidate IEEE divisions cost ~3 %)
  auto max_step = [&]() -> T {
    MinRatio<T> mr;
    auto cand = [&](T v, T d) { mr.cand(v, d); };
    cand(tl, dtl);
    cand(tu, dtu);
    cand(ll, dll);
    cand(lu, dlu);
    return block_min(mr.value());
  };

  for (it = 0;; ++it) {
    // ---- load H tiles (16 consecutive columns per row group: 128-B segments)
    {
    IPM256_LOCAL_IDS;
    static_for<0, SL>([&](auto s_) {
      constexpr int s = decltype(s_)::value;
      const int I = slot_I<NT>(wave, s), J = slot_J(wave, s);
      const T* hp = Hq + (size_t)(16 * I) * NP + 16 * J + c16;
#pragma unroll
      for (int k = 0; k < 4; ++k) K[s][k] = hp[(size_t)MF::row(lane, k) * NP];
    });
    }

    // ---- residuals: C u, H u
    if (isv) L.vec[tid] = u_i;
#pragma unroll
    for (int e = 0; e < NP; e += 64) L.part[wave][lane + e] = T(0);
    __syncthreads();
    const T cu = C_row();
    {
      IPM256_LOCAL_IDS;
      T pa0[4] = {T(0), T(0), T(0), T(0)}, pa1[4] = {T(0), T(0), T(0), T(0)};
      static_for<0, SL>([&](auto s_) {
        constexpr int s = decltype(s_)::value;
        const int I = slot_I<NT>(wave, s), J = slot_J(wave, s);
        const T uc = L.vec[16 * J + c16];
        if (s <= wave) {
#pragma unroll
          for (int k = 0; k < 4; ++k) pa0[k] = fma(K[s][k], uc, pa0[k]);
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) pa1[k] = fma(K[s][k], uc, pa1[k]);
        }
        if (I != J) {  // the mirrored upper tile: (H_IJ' u_I) lands on rows of tile row J
          T p = T(0);
#pragma unroll
          for (int k = 0; k < 4; ++k) p = fma(K[s][k], L.vec[16 * I + MF::row(lane, k)], p);
          p = cross4_sum(p);
          if (lane < 16) L.part[wave][16 * J + lane] += p;
        }
      });
      const int R0 = wave, R1 = NT - 1 - wave;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const T t0 = row16_sum(pa0[k]);
        const T t1 = row16_sum(pa1[k]);
        const int r = MF::row(lane, k);
        if (c16 == 0) {
          L.part[wave][16 * R0 + r] += t0;
          L.part[wave][16 * R1 + r] += t1;
        }
      }
    }
    __syncthreads();
    T hu = T(0);
    if (isv) {
#pragma unroll
      for (int v = 0; v < W; ++v) hu += L.part[v][tid];
    }
    T rs = T(0), ri = T(0), rc = T(0), ms = T(0);
    rl = con ? cu - lo - tl : T(0);
    ru = con ? hi - cu - tu : T(0);
    ri = fmax(fabs(rl), fabs(ru));
    {
      const T cl = tl * ll, ch = tu * lu;
      rc = con ? fmax(cl, ch) : T(0);
      ms = con ? cl + ch : T(0);
    }
    L.w[tid] = ll - lu;
    __syncthreads();
    {
      const T ctw = CT_var();
      rg_i = isv ? hu + g_i - ctw : T(0);
      rs = fabs(rg_i);
    }
    block_reduce(rs, ri, rc, ms);
    if (a.res && tid == 0) {  // block maxima of this iteration's residuals (the last write is the final one)
      double* o = a.res + (size_t)q * 4;
      o[0] = (double)rs;
      o[1] = 0.0;
      o[2] = (double)ri;
      o[3] = (double)rc;
    }
    const T mu = m > 0 ? ms / T(2 * m) : T(0);
    const bool st_on = a.stats && it < a.stats_cap;  // statistics row of this iteration (cmpc_enable_stats)
    auto st_row = [&]() { return a.stats + ((size_t)q * a.stats_cap + it) * CMPC_STAT_COLS; };
    if (st_on && tid == 0) {  // statistics row: residuals (block maxima) and mu now, the step below
      double* sr = st_row();
      for (int k = 0; k < 5; ++k) sr[k] = __builtin_nan("");
      sr[5] = (double)mu;
      sr[6] = (double)rs;
      sr[7] = 0.0;
      sr[8] = (double)ri;
      sr[9] = (double)rc;
    }
    if (!(isfinite(rs) && isfinite(ri) && isfinite(rc))) {
      status = CMPC_NAN_SOL;
      break;
    }
    if (rs <= T(S.tol_stat) && ri <= T(S.tol_ineq) && rc <= T(S.tol_comp)) {
      status = CMPC_SUCCESS;
      break;
    }
    if (it >= S.iter_max) {
      status = CMPC_MAX_ITER;
      break;
    }
    if (m > 0 && !(mu > T(MF::mu_min))) {
      status = CMPC_MIN_STEP;
      break;
    }

    // ---- Newton matrix K = H + C' diag(lam_l/t_l + lam_u/t_u) C + reg I (3x3 blocks on the triple diagonal)
    itl = con ? T(1) / tl : T(0);
    itu = con ? T(1) / tu : T(0);
    L.w[tid] = ll * itl + lu * itu;
    if (tid == 0) L.nanflag = 0;
    __syncthreads();
    {
    IPM256_LOCAL_IDS;
    static_for<0, SL>([&](auto s_) {
      constexpr int s = decltype(s_)::value;
      const int I = slot_I<NT>(wave, s), J = slot_J(wave, s);
      if (I - J <= 1) {
        const int gj = 16 * J + c16;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int gi = 16 * I + MF::row(lane, k);
          const int t = gi / 3;
          T add = T(0);
          if (gi < n && gj / 3 == t) {
            const int di = gi % 3, dj = gj % 3;
            const T s0 = L.w[5 * t], s1 = L.w[5 * t + 1], s2 = L.w[5 * t + 2], s3 = L.w[5 * t + 3],
                    s4 = L.w[5 * t + 4];
            const T mt = L.mut[t];
            const T xx = s0 + s1, yy = s2 + s3, zz = mt * mt * (s0 + s1 + s2 + s3) + s4;
            const T xz = mt * (s1 - s0), yz = mt * (s3 - s2);
            const int dsum = di + dj;
            add = di == dj ? (di == 0 ? xx : (di == 1 ? yy : zz)) : (dsum == 1 ? T(0) : (dsum == 2 ? xz : yz));
          }
          if (gi == gj) add += T(S.reg_prim);
          K[s][k] += add;
        }
      }
    });
    }

    // ---- blocked right-looking Cholesky
    for (int p = 0; p < NT; ++p) {
      const int buf = p & 1;
      IPM256_LOCAL_IDS;
      if (wave == owner<NT>(p)) {
        // diagonal tile (selected out of its slot once, so the factorisation code exists once); column s
        // broadcast through LDS
        acc_t D = K[0];
        static_for<1, SL>([&](auto s_) {
          constexpr int s = decltype(s_)::value;
          if (slot_I<NT>(wave, s) == p && slot_J(wave, s) == p) D = K[s];
        });
        static_for<0, 16>([&](auto c_) {
          constexpr int sc = decltype(c_)::value;
          if (c16 == sc) {
#pragma unroll
            for (int k = 0; k < 4; ++k) L.col[MF::row(lane, k)] = D[k];
          }
          wave_sync();
          const T d = L.col[sc];
          // BLASFEO-style guard as k_ipm_reg / oracle_qp_ipm: a lost pivot drops its direction; NaN recorded
          const T il0 = rsqrt_acc(fmax(d, T(MF::pivot_min)));
          const T il = d > T(MF::pivot_min) ? il0 : T(0);
          if (lane == 0) {
            L.il[sc] = il;
            if (d != d) L.nanflag = 1;
          }
          const T lc = c16 > sc ? L.col[c16] * il : T(0);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int r = MF::row(lane, k);
            const T lr = r > sc ? L.col[r] * il : T(0);
            D[k] = c16 == sc ? (r > sc ? lr : D[k]) : fma(-lr, lc, D[k]);
          }
          wave_sync();
        });
        // factor tile -> LDS, then invert it (lane c < 16 owns column c of L_pp^-1)
#pragma unroll
        for (int k = 0; k < 4; ++k) L.dg[MF::row(lane, k) * PS + c16] = D[k];
        wave_sync();
        if (lane < 16) {
          T X[16];
          static_for<0, 16>([&](auto r_) {
            constexpr int r = decltype(r_)::value;
            T v = r == lane ? T(1) : T(0);
            static_for<0, r>([&](auto k_) {
              constexpr int kk = decltype(k_)::value;
              v = fma(-L.dg[r * PS + kk], X[kk], v);
            });
            X[r] = v * L.il[r];
          });
#pragma unroll
          for (int r = 0; r < 16; ++r) L.Dinv[p][r * PS + lane] = X[r];
        }
      }
      // raw panel tiles A_ip (i > p) -> LDS
      static_for<0, SL>([&](auto s_) {
        constexpr int s = decltype(s_)::value;
        const int I = slot_I<NT>(wave, s), J = slot_J(wave, s);
        if (J == p && I > p) {
#pragma unroll
          for (int k = 0; k < 4; ++k) L.P[buf][I][MF::row(lane, k) * PS + c16] = K[s][k];
        }
      });
      __syncthreads();
      {
      IPM256_LOCAL_IDS;
      // L_ip = A_ip L_pp^-T on the matrix cores (A in the operand layout from LDS, B[k][j] = Linv[j][k])
      static_for<0, SL>([&](auto s_) {
        constexpr int s = decltype(s_)::value;
        const int I = slot_I<NT>(wave, s), J = slot_J(wave, s);
        if (J == p && I > p) {
          acc_t c = acc_t{T(0), T(0), T(0), T(0)};
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const int o = c16 * PS + 4 * kk + g4;
            c = MF::run(L.P[buf][I][o], L.Dinv[p][o], c);
          }
          K[s] = c;
#pragma unroll
          for (int k = 0; k < 4; ++k) L.P[buf][I][MF::row(lane, k) * PS + c16] = c[k];
        }
      });
      }
      __syncthreads();
      {
      IPM256_LOCAL_IDS;
      // trailing update A_ij -= L_ip L_jp' (i >= j > p)
      static_for<0, SL>([&](auto s_) {
        constexpr int s = decltype(s_)::value;
        const int I = slot_I<NT>(wave, s), J = slot_J(wave, s);
        if (J > p) {
          acc_t c = K[s];
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const int o = c16 * PS + 4 * kk + g4;
            c = MF::run(-L.P[buf][I][o], L.P[buf][J][o], c);
          }
          K[s] = c;
        }
      });
      }
    }
    __syncthreads();
    if (L.nanflag) {
      status = CMPC_NAN_SOL;
      break;
    }

    // ---- predictor (affine scaling direction)
    rml = tl * ll;
    rmu = tu * lu;
    direction();
    T alpha = fmin(T(1), max_step());
    if (m > 0) {
      T maff = con ? (tl + alpha * dtl) * (ll + alpha * dll) + (tu + alpha * dtu) * (lu + alpha * dlu) : T(0);
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
      rml = con ? tl * ll + dtl * dll - sigma * mu : T(0);
      rmu = con ? tu * lu + dtu * dlu - sigma * mu : T(0);
      direction();
      alpha = fmin(T(1), T(TAU) * max_step());
    }
    if (st_on && tid == 0) {
      double* sr = st_row();
      sr[3] = sr[4] = (double)alpha;
    }  // one step length for primal and dual
    if (alpha < T(S.alpha_min)) {
      status = CMPC_MIN_STEP;
      break;
    }
    u_i = fma(alpha, du_i, u_i);
    tl = fma(alpha, dtl, tl);
    tu = fma(alpha, dtu, tu);
    ll = fma(alpha, dll, ll);
    lu = fma(alpha, dlu, lu);
  }

  const bool fin = !var || isfinite(u_i);
  const int bad = __syncthreads_or(fin ? 0 : 1);
  if (bad) status = CMPC_NAN_SOL;
  if (isv && tid < ld) a.u[(size_t)q * ld + tid] = var ? u_i : T(0);
  if (tid == 0) {
    a.status[q] = status;
    a.iters[q] = it;
  }
  if (a.out_u) {  // the constraint-side vector L.w (NTHR >= 256 entries) is dead by now
    __syncthreads();
    scatter_result<T>(a, q, n, u_i, status, it, L.w, tid, NTHR, [] { __syncthreads(); });
  }
}

}  // namespace cmpc
