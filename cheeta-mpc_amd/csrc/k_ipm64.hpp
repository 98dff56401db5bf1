#pragma once
// k_ipm64.hpp — stage 2 of the hot path for condensed sizes n <= 64 (every trot QP at N <= 10): the batched dense
// friction-pyramid QP, primal-dual Mehrotra predictor-corrector interior point method. Replaces d_ocp_qp_ipm_solve
// (HPIPM, called at HpipmInterface.cpp:284) / IPOPT's Newton loop (CentroidalMPC.cpp:354) for the condensed
// centroidal QP; settings and stopping rule mirror hpipm_interface::Settings (HpipmInterfaceSettings.h:44-57).
// The iteration is the one restated in oracle/cmpc_oracle.c:oracle_qp_ipm; only the factorisation differs
// (LDL' with an explicit L^-1 here, Cholesky and triangular solves there), so the two agree to rounding.
//
//   min 1/2 u'Hu + g'u   s.t.  lo <= C u <= hi,   C = blkdiag_t F(mu_t) (5x3 pyramid per stance force triple)
//
// MI355X mapping — one wavefront (64 lanes) per QP, no workgroup barriers, 2 waves per SIMD (fp64):
//   * Newton matrix K = H + C' Sigma C in a 4 x 16-cyclic register tile: lane l = 16a + b holds
//     K[a + 4r][b + 16c] (r = 0..15, c = 0..3) in register e = 4r + c — 64 values per lane;
//   * LDL' elimination that also builds L^-1 in place. Step s, every row i > s and every column j != s:
//     K[i][j] -= K[i][s] K[s][j] / d_s. For j > s this is the right-looking LDL' update; for j < s the same
//     update accumulates the strict lower part S of the explicit inverse, X = L^-1 with X[i][j] = -S[i][j] / d_j
//     (column s is left as it is, so the row operations on the identity need no extra storage). The 16 row
//     multipliers K[i][s] of a lane live in its own 16-lane DPP row (column s sits in lane b = s % 16), so they
//     arrive through row_newbcast inside v_fmac_f64_dpp at no instruction cost (dpp_rows.hpp: dpp_rowf); only the
//     4 column multipliers K[s][j] / d_s come from LDS. One-step look-ahead: row s+1 is updated first, sent
//     through LDS and its pivot read and inverted before the bulk of step s, so both round trips overlap the FMAs;
//   * solves are K^-1 y = X' D^-1 X y: two matrix-vector products over the 40 registers of the strict lower part
//     (forward: row sums reduced through LDS; backward: column sums reduced through LDS), no serial sweeps and no
//     transpose of the factor (lab v6: 0.506 -> 0.449 ms per 4096 QPs, same iteration counts, 5e-16 vs v0);
//   * H u is formed from the tile once (first iteration) and then carried: H du = rhs - (C' Sigma C + reg I) du from
//     the last solve's right-hand side and the 3x3 blocks, so later iterations skip the 64-FMA product and its two
//     LDS reductions (lab: 1.8 % per launch, iterates within 1e-14 of the direct product, same iteration counts);
//   * vectors are lane-per-variable; the <= 105 pyramid rows are two slots per lane (j = lane + 64 cc) with the
//     primal-dual state in registers and per-iteration scratch in lane-private LDS;
//   * H is stored by the condensing kernel in the tile order (h_index, cmpc_kernels.hpp): 64 coalesced 512-B
//     row loads per iteration;
//   * lane-derived addresses come from an opaque lane id re-read every iteration (olane) so they are not hoisted
//     out of the loop as ~100 live VGPRs; lane masks use the plain id and are hoisted into SGPR pairs.
#include <type_traits>

#include "cmpc_device.hpp"
#include "cmpc_kernels.hpp"
#include "condense64.hpp"
#include "step_ratio.hpp"
#include "dpp_rows.hpp"
#include "wave_dpp.hpp"

// In-kernel s_memtime stamps, diagnostic builds only (-DCMPC_IPM_STAMPS; lab/run_lab.sh): per-QP cycles of each
// phase into IpmArgs::stamps[q][9]. Segments: 0 H + residuals, 1 Newton matrix, 2 LDL', 3 lower-part mask, 4 solves,
// 5 predictor rest, 6 corrector rest, 7 update, 8 total.
#ifdef CMPC_IPM_STAMPS
#define IPM_STAMP_DECL                                                    \
  unsigned long long st_acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0};              \
  const unsigned long long st_t0_ = ipm64::memtime();                   \
  unsigned long long st_prev_ = st_t0_
#define IPM_STAMP(k)                                      \
  do {                                                    \
    const unsigned long long t_ = ipm64::memtime();       \
    st_acc_[k] += t_ - st_prev_;                          \
    st_prev_ = t_;                                        \
  } while (0)
#define IPM_STAMP_STORE(ptr, q)                                                   \
  do {                                                                            \
    const unsigned long long t_ = ipm64::memtime();                               \
    if ((ptr) && threadIdx.x == 0) {                                              \
      for (int k_ = 0; k_ < 8; ++k_) (ptr)[(size_t)(q) * 9 + k_] = st_acc_[k_];   \
      (ptr)[(size_t)(q) * 9 + 8] = t_ - st_t0_;                                   \
    }                                                                             \
  } while (0)
#elif defined(CMPC_IPM_TIMELINE)
// diagnostic: per-QP wave start / end on the 100-MHz real-time counter and the hardware slot (HW_ID, XCC_ID)
#define IPM_STAMP_DECL                                                                      \
  unsigned long long tl_t0_;                                                                \
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(tl_t0_)::"memory")
#define IPM_STAMP(k) (void)0
#define IPM_STAMP_STORE(ptr, q)                                                             \
  do {                                                                                      \
    unsigned long long t_;                                                                  \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");          \
    unsigned hw_, xcc_;                                                                     \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));                       \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));                     \
    if ((ptr) && threadIdx.x == 0) {                                                        \
      (ptr)[(size_t)(q) * 9 + 0] = tl_t0_;                                                  \
      (ptr)[(size_t)(q) * 9 + 1] = t_;                                                      \
      (ptr)[(size_t)(q) * 9 + 2] = hw_;                                                     \
      (ptr)[(size_t)(q) * 9 + 3] = xcc_;                                                    \
    }                                                                                       \
  } while (0)
#else
#define IPM_STAMP_DECL (void)0
#define IPM_STAMP(k) (void)0
#define IPM_STAMP_STORE(ptr, q) (void)0
#endif

namespace cmpc {

namespace ipm64 {

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
  static constexpr double pivot_min = 1e-200;  // BLASFEO-style guard: smaller pivots drop their direction
  static constexpr double mu_min = 1e-300;     // mu underflow -> MIN_STEP instead of 0/0
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
template <int B, int E, typename F>
__device__ __forceinline__ void sfor_down(F&& f) {  // E-1 down to B
  if constexpr (B < E) {
    f(std::integral_constant<int, E - 1>{});
    sfor_down<B, E - 1>(f);
  }
}
// Compiler-only ordering of LDS accesses: one wave's DS instructions execute in order, so a read issued after a
// write (or a write after a read) in program order sees the right data without s_waitcnt.
__device__ __forceinline__ void cbar() { asm volatile("" ::: "memory"); }
__device__ __forceinline__ int olane() {
  int l = (int)threadIdx.x;
  asm volatile("" : "+v"(l));
  return l;
}
__device__ __forceinline__ bool uflag(bool b) { return __builtin_amdgcn_readfirstlane((int)b) != 0; }

__device__ __forceinline__ double rcp_raw(double x) { return __builtin_amdgcn_rcp(x); }
__device__ __forceinline__ float rcp_raw(float x) { return __builtin_amdgcn_rcpf(x); }
// reciprocal of a pivot: hardware estimate + one Newton step, 0 for pivots at or below the guard (and NaN)
template <typename T>
__device__ __forceinline__ T pivot_inv(T p) {
  T y = rcp_raw(p);
  const T e = fma(-p, y, T(1));
  y = fma(y, e, y);
  return p > T(Lim<T>::pivot_min) ? y : T(0);
}


// Strides of the partial-sum buffers, chosen so that every access is bank-conflict free under the MI355X rules
// (MI355X_MICROARCH.md §LDS; a ds_write_b64 covers 16 lanes of one row a = lane / 16, a ds_read_b64 32 lanes):
//   row partials: partial b of row i at b * RS + i (RS odd: 16 lanes b of one write on distinct banks; a read is 32
//     consecutive rows); column partials: partial a of column j at a * 64 + j; z at row stride ZS = 20 (the 16 lanes
//     of a write, (i % 4, i / 4), on 16 distinct bank pairs); block rows at stride 80 (rows e, e + 1 read by one lane
//     group half a bank row apart).
constexpr int RS = 65, ZS = 20, BS = 80;

template <typename T>
struct Lds {
  T v[64];          // lane-per-variable broadcast
  T w[128];         // pyramid-row broadcast
  T rowbuf[2][64];  // factorisation: row s of K as [c*16 + b]
  T dg[64];         // pivots d_s
  T z[4 * ZS];      // solve: z permuted as [i % 4][i / 4]
  T blk[3][BS];     // Newton 3x3 block rows
  T rl[128], ru[128], itl[128], itu[128], rml[128], rmu[128];  // lane-private pyramid-row scratch
  T scr[16 * RS];   // Hu and solve partial sums
};

}  // namespace ipm64

// LDS of the IPM; the fused kernel (k_solve64) runs the condensing first in the same bytes
template <typename T, bool FUSED>
struct IpmShared {
  ipm64::Lds<T> ipm;
};
template <typename T>
struct IpmShared<T, true> {
  union {
    ipm64::Lds<T> ipm;
    c64::C64Lds<T> cond;
  };
};

// Body of one QP on one wavefront. MODE 0 (k_ipm64): everything is read from the workspace a separate condensing
// launch filled. MODE 1 (k_solve64): the QP is condensed first by the same wave (condense64_qp, which also writes H
// and the QP data to the workspace for the later iterations and the other stages) and the first Newton matrix starts
// from the H the condensing leaves in registers. (An iteration-work-item form, k_solve64q, measured 7-17 % slower
// and was moved out of the library)
template <typename T, int WPE, int MODE>
__device__ __forceinline__ void ipm64_body(const IpmArgs<T>& A, const CondenseArgs<T>* C, int q) {
  // the LDS block is declared here, so its accesses keep a constant base (as a reference from the kernel,
  // ds_write2 / ds_read2 pairing is lost: +640 instructions, +3 % time)
  __shared__ IpmShared<T, (MODE > 0)> SH;
  constexpr bool FUSED = MODE > 0;
  using namespace ipm64;
  IPM_STAMP_DECL;
  Lds<T>& L = SH.ipm;
  T K[64];
  T g_v, mu_v;
  T lo[2], hi[2], muc[2];
  int n;
  if constexpr (FUSED) {
    {
      n = condense64_qp<T>(*C, q, SH.cond, K, g_v, mu_v);
      if (n < 0) {  // invalid contact table (status written) or a bigger class (nvar hint written)
        if (n == -2 && A.out_u)  // the rejected QP's result: zeros, INVALID_CONTACT, no iterations
          scatter_result<T>(A, q, 0, T(0), CMPC_INVALID_CONTACT, 0, SH.ipm.scr, olane(), 64,
                            [] { ipm64::cbar(); });
        if (n <= -3 && A.app_list && olane() == 0) {  // append to the bigger class's list
          const int cls = -3 - n <= 128 ? 1 : 2;
          const int pos = atomicAdd(&A.app_count[cls], 1);
          A.app_list[(size_t)cls * A.app_ld + pos] = q;
        }
        return;
      }
      // pyramid rows j = lane + 64 cc: the bounds and friction coefficients the condensing just wrote to the
      // workspace, taken from the model and its triple table in LDS before the IPM reuses those bytes
      const DevModel* M = C->model;
      const int lane_ = (int)threadIdx.x;
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        const int j = lane_ + 64 * cc;
        const bool on = j < 5 * (n / 3);
        lo[cc] = T(0);
        hi[cc] = on ? T(M->ub[j % 5]) : T(0);
        muc[cc] = on ? T(M->mu[SH.cond.tleg[j / 5]]) : T(0);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
  } else {
    if (A.status[q] != CMPC_SUCCESS) return;  // invalid contact table / too large: status already set
    n = A.nvar[q];
    if (n > 64) return;  // served by the 128 class
  }
  const int ld = A.ld;
  const int nt = n / 3;
  const int m = 5 * nt;
  const DevSettings S = A.s;
  int lane = (int)threadIdx.x;  // re-read opaquely at every iteration
  const int lane0 = (int)threadIdx.x;  // plain lane id: lane masks only (hoisted into SGPR pairs)

  // ---- lane-per-variable data
  const bool vin = lane < n;
  auto ldx = [&](const T* p) -> T { return *p; };
  if (!FUSED) {
    g_v = vin ? ldx(A.g + (size_t)q * ld + lane) : T(0);
    mu_v = vin ? ldx(A.tri_mu + (size_t)q * (ld / 3) + lane / 3) : T(0);
  }
  // cold start (warm_start = 0): u = 0; warm start: u from the workspace (previous solution, cmpc_solve_batch_warm)
  T u_v = (!FUSED && A.warm && vin) ? A.u[(size_t)q * ld + lane] : T(0);
  if (!FUSED && A.warm) L.v[lane] = u_v;
  cbar();
  // ---- pyramid rows j = lane + 64 cc: slacks of C u clipped at THR0, lam = mu0 / t
  T tl[2], tu[2], ll[2], lu[2];
#pragma unroll
  for (int cc = 0; cc < 2; ++cc) {
    const int j = lane + 64 * cc;
    const bool on = j < m;
    const int t = j / 5;
    if (!FUSED) {
      lo[cc] = on ? ldx(A.tri_lo + ((size_t)q * (ld / 3) + t) * 5 + j % 5) : T(0);
      hi[cc] = on ? ldx(A.tri_hi + ((size_t)q * (ld / 3) + t) * 5 + j % 5) : T(0);
      muc[cc] = on ? ldx(A.tri_mu + (size_t)q * (ld / 3) + t) : T(0);
    }
    T cu0 = T(0);
    if (!FUSED && A.warm && on) cu0 = pyr_row<T>(j % 5, muc[cc], L.v[3 * t], L.v[3 * t + 1], L.v[3 * t + 2]);
    tl[cc] = on ? fmax(cu0 - lo[cc], T(THR0)) : T(1);
    tu[cc] = on ? fmax(hi[cc] - cu0, T(THR0)) : T(1);
    ll[cc] = on ? T(S.mu0) / tl[cc] : T(0);
    lu[cc] = on ? T(S.mu0) / tu[cc] : T(0);
  }
  cbar();

  // C x for the lane's two pyramid rows, x already in L.v (CentroidalMPC.cpp:186-190)
  auto apply_C = [&](T (&out)[2]) {
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int j = lane + 64 * cc;
      const int t = j / 5;
      T v = T(0);
      if (j < m) v = pyr_row<T>(j % 5, muc[cc], L.v[3 * t], L.v[3 * t + 1], L.v[3 * t + 2]);
      out[cc] = v;
    }
  };
  // C' w, lane-per-variable
  auto apply_CT = [&](const T (&wv)[2]) -> T {
    L.w[lane] = wv[0];
    L.w[lane + 64] = wv[1];
    cbar();
    T v = T(0);
    if (vin) {
      const int t = lane / 3, dd = lane % 3;
      const T w0 = L.w[5 * t], w1 = L.w[5 * t + 1], w2 = L.w[5 * t + 2], w3 = L.w[5 * t + 3], w4 = L.w[5 * t + 4];
      v = dd == 0 ? (w1 - w0) : (dd == 1 ? (w3 - w2) : (mu_v * (w0 + w1 + w2 + w3) + w4));
    }
    cbar();
    return v;
  };

  T invd_v = T(1);
  T hu_v = T(0), rhs_v = T(0);
  T rg_v = T(0), du_v = T(0);
  T dtl[2], dtu[2], dll[2], dlu[2];

  // Solve K x = y with the eliminated tile (see the factorisation): strictly lower part S (X = L^-1 with
  // X[i][j] = -S[i][j] / d_j), pivots d. K^-1 = X' D^-1 X, so both halves are matrix-vector products over the
  // 40 lower registers (r >= 4c; the 16 diagonal-straddling ones were masked after the factorisation):
  //   forward  t = D^-1 y;  z = D^-1 (y - S t)            row sums: 16 partials per lane, reduced through LDS
  //   backward x = z - D^-1 (S' z)                         column sums: 4 partials per lane, reduced through LDS
  auto solve = [&](T& y) {
    const int ol = olane();
    const int ola = ol >> 4, olb = ol & 15;
    L.v[ol] = y * invd_v;
    cbar();
    T tc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) tc[c] = L.v[olb + 16 * c];
    cbar();
    {
      const int base = olb * RS + ola;  // row 4 r + ola, partial olb
      sfor<0, 16>([&](auto r_) {
        constexpr int r = decltype(r_)::value;
        T p = K[r * 4] * tc[0];
        sfor<1, r / 4 + 1>([&](auto c_) {
          constexpr int c = decltype(c_)::value;
          p = fma(K[r * 4 + c], tc[c], p);
        });
        L.scr[base + 4 * r] = p;
      });
    }
    cbar();
    T sv = T(0);
#pragma unroll
    for (int k = 0; k < 16; k += 2) sv += L.scr[k * RS + ol] + L.scr[(k + 1) * RS + ol];
    cbar();
    const T z = (y - sv) * invd_v;
    L.z[(ol & 3) * ZS + (ol >> 2)] = z;
    cbar();
    T zr[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) zr[r] = L.z[ola * ZS + r];
    cbar();
    sfor<0, 4>([&](auto c_) {
      constexpr int c = decltype(c_)::value;
      T q = K[(4 * c) * 4 + c] * zr[4 * c];
      sfor<4 * c + 1, 16>([&](auto r_) {
        constexpr int r = decltype(r_)::value;
        q = fma(K[r * 4 + c], zr[r], q);
      });
      L.scr[ola * 64 + c * 16 + olb] = q;
    });
    cbar();
    const T qs = (L.scr[ol] + L.scr[64 + ol]) + (L.scr[128 + ol] + L.scr[192 + ol]);
    cbar();
    y = fma(-invd_v, qs, z);
  };

  const T* Hq = A.H + (size_t)q * ld * ld;
  // H in tile order into the registers of the factor: the 40 stored rows (coalesced 512 B each), then the 24 strictly
  // upper registers as the mirrored elements of those rows (h_stored): register (r, c), c > r / 4, of lane
  // (a, b) is H[b + 16c][a + 4r] = stored register 16c + 4 (b >> 2) + (r >> 2), lane 16 (b & 3) + a + 4 (r & 3)
  auto load_H = [&]() {
    const int ln = olane();
    sfor<0, 64>([&](auto e_) {
      constexpr int e = decltype(e_)::value;
      if constexpr ((e & 3) <= (e >> 4)) K[e] = Hq[e * 64 + ln];
    });
    const int mt = ((ln & 15) >> 2) * 256 + (ln & 3) * 16 + (ln >> 4);
    sfor<0, 64>([&](auto e_) {
      constexpr int e = decltype(e_)::value, r = e >> 2, c = e & 3;
      if constexpr (c > (r >> 2)) K[e] = Hq[(16 * c + (r >> 2)) * 64 + 4 * (r & 3) + mt];
    });
  };

  // Newton direction for the complementarity targets in L.rml / L.rmu. After the iteration's last solve the factor
  // is dead: the next iteration's H is requested right there, so its latency hides behind the step-length work.
  auto direction = [&](auto last_, auto seg_) {
    constexpr bool last = decltype(last_)::value;
    constexpr int seg = decltype(seg_)::value;
    (void)seg;
    T wv[2];
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int j = lane + 64 * cc;
      wv[cc] = (L.rml[j] + ll[cc] * L.rl[j]) * L.itl[j] - (L.rmu[j] + lu[cc] * L.ru[j]) * L.itu[j];
    }
    const T ctw = apply_CT(wv);
    rhs_v = -rg_v - ctw;
    du_v = rhs_v;
    IPM_STAMP(seg);
    solve(du_v);
    IPM_STAMP(4);
    L.v[lane] = du_v;
    cbar();
    T cdu[2];
    apply_C(cdu);
    cbar();
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int j = lane + 64 * cc;
      dtl[cc] = cdu[cc] + L.rl[j];
      dtu[cc] = L.ru[j] - cdu[cc];
      dll[cc] = -(L.rml[j] + ll[cc] * dtl[cc]) * L.itl[j];
      dlu[cc] = -(L.rmu[j] + lu[cc] * dtu[cc]) * L.itu[j];
    }
  };
  // fraction-to-boundary ratio: the smallest v / (-d) over the lane's eight candidates with d < 0 is selected by
  // cross-multiplication (v, -d > 0) and divided once, instead of one IEEE division per candidate
  auto max_step = [&]() -> T {
    MinRatio<T> mr;
    auto cand = [&](T v, T d) { mr.cand(v, d); };
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      cand(tl[cc], dtl[cc]);
      cand(tu[cc], dtu[cc]);
      cand(ll[cc], dll[cc]);
      cand(lu[cc], dlu[cc]);
    }
    return wave_min_dpp(mr.value());
  };

  int status = CMPC_MAX_ITER;
  int it = 0;
  for (it = 0;; ++it) {
    progress_prio(it);  // cmpc_device.hpp
    if (!(FUSED && it == 0)) {
      // fused: iteration 0 starts from the condensing's registers; the rows it stored are re-read from iteration 1
      // on by the same lanes (the wait drains the stores before the first re-read)
      if (MODE == 1 && it == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      load_H();  // consumed first by Hu below: the pyramid residuals run while the 64 rows are in flight
    }
#ifdef H_WAIT_STAMP  // diagnostic: time to the last H row (segment 3)
    IPM_STAMP(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    IPM_STAMP(3);
#endif
    lane = olane();
    const int la = lane >> 4, lb = lane & 15;

    // ---- residuals that do not need H: C u, slack/complementarity residuals, C' lam
    L.v[lane] = u_v;
    cbar();
    T cu[2];
    apply_C(cu);
    T rs = T(0), ri = T(0), rc = T(0), ms = T(0);
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int j = lane + 64 * cc;
      const bool on = j < m;
      const T rl = on ? cu[cc] - lo[cc] - tl[cc] : T(0);
      const T ru = on ? hi[cc] - cu[cc] - tu[cc] : T(0);
      L.rl[j] = rl;
      L.ru[j] = ru;
      ri = fmax(ri, fmax(fabs(rl), fabs(ru)));
      const T cl = tl[cc] * ll[cc], ch = tu[cc] * lu[cc];
      rc = fmax(rc, fmax(cl, ch));
      ms += cl + ch;
    }
    T ctw;
    {
      const T wv[2] = {ll[0] - lu[0], ll[1] - lu[1]};
      ctw = apply_CT(wv);
    }
    // ---- Hu from the tile: 16 partial row sums per lane, reduced through LDS (partial b of row i at b * RS + i,
    //      conflict-free writes and row reads)
    T hu = hu_v;  // H u kept up to date incrementally; computed from the tile only at the first iteration
    if (it == 0) {
      T uc[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) uc[c] = L.v[lb + 16 * c];
      const int base = lb * RS + la;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        T p = K[r * 4] * uc[0];
        p = fma(K[r * 4 + 1], uc[1], p);
        p = fma(K[r * 4 + 2], uc[2], p);
        p = fma(K[r * 4 + 3], uc[3], p);
        L.scr[base + 4 * r] = p;
      }
      cbar();
#pragma unroll
      for (int k = 0; k < 16; k += 2) hu += L.scr[k * RS + lane] + L.scr[(k + 1) * RS + lane];
      cbar();
      hu_v = hu;
    }
    rg_v = vin ? hu + g_v - ctw : T(0);
    rs = fabs(rg_v);
    if (A.res_scr) {  // this iteration's residual terms, reduced once at the exit
      T* rp = A.res_scr + (size_t)q * 3 * 64 + lane;
      rp[0] = rs;
      rp[64] = ri;
      rp[128] = rc;
    }
    ms = wave_sum_dpp(ms);
    const T mu = m > 0 ? ms / T(2 * m) : T(0);
#ifdef CMPC_NO_STATS  // lab: the statistics code compiled out (A/B of its cost)
    constexpr bool st_on = false;
#else
    const bool st_on = A.stats && it < A.stats_cap;  // statistics row of this iteration (cmpc_enable_stats)
#endif
    auto st_row = [&]() { return A.stats + ((size_t)q * A.stats_cap + it) * CMPC_STAT_COLS; };
    if (st_on) {  // statistics row of this iteration: residuals and mu now, the step below (NaN if none is taken)
      const T r0 = wave_max_dpp(rs), r1 = wave_max_dpp(ri), r2 = wave_max_dpp(rc);
      if (lane == 0) {
        double* sr = st_row();
        for (int k = 0; k < 5; ++k) sr[k] = __builtin_nan("");
        sr[5] = (double)mu;
        sr[6] = (double)r0;
        sr[7] = 0.0;
        sr[8] = (double)r1;
        sr[9] = (double)r2;
      }
    }
    // a non-finite residual anywhere -> NAN_SOL; HPIPM's absolute stopping rule (tol_stat / tol_ineq / tol_comp)
    // as a wave vote: max over lanes <= tol iff every lane <= tol (no max-reductions needed)
    if (__any(!(isfinite(rs) && isfinite(ri) && isfinite(rc)))) {
      status = CMPC_NAN_SOL;
      break;
    }
    if (__all(rs <= T(S.tol_stat) && ri <= T(S.tol_ineq) && rc <= T(S.tol_comp))) {
      status = CMPC_SUCCESS;
      break;
    }
    if (it >= S.iter_max) {
      status = CMPC_MAX_ITER;
      break;
    }
    if (uflag(m > 0 && !(mu > T(Lim<T>::mu_min)))) {
      status = CMPC_MIN_STEP;
      break;
    }
    IPM_STAMP(0);

    // ---- Newton matrix K = H + C' diag(lam_l/t_l + lam_u/t_u) C + reg I: lane j writes the 3x3 block row of
    //      variable j, tile lanes add it where entry (i, j) falls in j's force triple
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int j = lane + 64 * cc;
      const bool on = j < m;
      const T itl = on ? T(1) / tl[cc] : T(0);
      const T itu = on ? T(1) / tu[cc] : T(0);
      L.itl[j] = itl;
      L.itu[j] = itu;
      L.w[j] = ll[cc] * itl + lu[cc] * itu;
    }
    cbar();
    {
      const int ti = lane / 3, dd = lane % 3;
      T b0 = T(0), b1 = T(0), b2 = T(0);
      if (vin) {
        const T s0 = L.w[5 * ti], s1 = L.w[5 * ti + 1], s2 = L.w[5 * ti + 2], s3 = L.w[5 * ti + 3], s4 = L.w[5 * ti + 4];
        const T xx = s0 + s1, yy = s2 + s3, zz = mu_v * mu_v * (s0 + s1 + s2 + s3) + s4;
        const T xz = mu_v * (s1 - s0), yz = mu_v * (s3 - s2);
        b0 = dd == 0 ? xx : (dd == 1 ? T(0) : xz);
        b1 = dd == 0 ? T(0) : (dd == 1 ? yy : yz);
        b2 = dd == 0 ? xz : (dd == 1 ? yz : zz);
      }
      const T reg = T(S.reg_prim);
      b0 += dd == 0 ? reg : T(0);
      b1 += dd == 1 ? reg : T(0);
      b2 += dd == 2 ? reg : T(0);
      L.blk[0][lane] = b0;
      L.blk[1][lane] = b1;
      L.blk[2][lane] = b2;
    }
    cbar();
    sfor<0, 4>([&](auto c_) {
      constexpr int c = decltype(c_)::value;
      // rows that can share a triple with some column of chunk c: local rows rlo..rhi
      constexpr int imin = 3 * ((16 * c) / 3);
      constexpr int imax0 = 3 * ((16 * c + 15) / 3) + 2;
      constexpr int imax = imax0 > 63 ? 63 : imax0;
      constexpr int rlo = imin / 4;
      constexpr int rhi = imax / 4;
      const int j = lb + 16 * c;
      const int t3 = 3 * (j / 3);
      const int e = (la - t3) & 3;  // the one row i = t3 + e of j's triple with i % 4 == a (none if e == 3)
      const int rstar = e <= 2 ? (t3 + e - la) >> 2 : -1;
      const T val = L.blk[e <= 2 ? e : 0][j];
      sfor<rlo, rhi + 1>([&](auto r_) {
        constexpr int r = decltype(r_)::value;
        K[r * 4 + c] += (rstar == r) ? val : T(0);
      });
    });
    cbar();
    IPM_STAMP(1);

    // ---- LDL' factorisation in the tile (see header)
    const bool full = uflag(n > 60);
    T piv = readlane(K[0], 0);
    T invd = pivot_inv(piv);
    T mm[4];
    {
      if (la == 0) {
#pragma unroll
        for (int c = 0; c < 4; ++c) L.rowbuf[0][c * 16 + lb] = K[c];
      }
      L.dg[0] = piv;
      cbar();
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const T mv = -(L.rowbuf[0][c * 16 + lb] * invd);
        mm[c] = (c == 0 && lb == 0) ? T(0) : mv;
      }
      cbar();
    }
    sfor<0, 63>([&](auto s_) {
      constexpr int s = decltype(s_)::value;
      constexpr int c0 = s / 16, b0 = s % 16, a0 = s % 4;
      constexpr int s1 = s + 1;
      constexpr int r1 = s1 / 4, a1 = s1 % 4, c1 = s1 / 16, b1 = s1 % 16;
      if constexpr (s1 >= 60) {
        // pivots 60..63 exist only for n > 60; padding rows keep S = 0 and get d = 1
        if (!full) {
          L.dg[s1] = T(1);
          return;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#ifdef LDL_SPLIT
      if constexpr (s == LDL_SPLIT) IPM_STAMP(2);
#endif
      const int la_m = lane0 >> 4, lb_m = lane0 & 15;  // masks and rowbuf addresses: hoisted, loop invariant
      // look-ahead local row r1 (holds row s+1); for a0 < 3 it is the partial row: rows a + 4 r1 > s iff a > a0
      if constexpr (a0 < 3) {
        if (la_m > a0)
          dpp_rowf<b0, c0, true, T>(K[r1 * 4], K[r1 * 4 + 1], K[r1 * 4 + 2], K[r1 * 4 + 3], mm[0], mm[1], mm[2], mm[3]);
      } else {
        dpp_rowf<b0, c0, true, T>(K[r1 * 4], K[r1 * 4 + 1], K[r1 * 4 + 2], K[r1 * 4 + 3], mm[0], mm[1], mm[2], mm[3]);
      }
      cbar();
      if (la_m == a1) {
#pragma unroll
        for (int c = 0; c < 4; ++c) L.rowbuf[s1 & 1][c * 16 + lb_m] = K[r1 * 4 + c];
      }
      cbar();
      T xn[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) xn[c] = L.rowbuf[s1 & 1][c * 16 + lb_m];
      cbar();
      const T pivn = readlane(K[r1 * 4 + c1], a1 * 16 + b1);
      T invdn = pivot_inv(pivn);
      asm volatile("" : "+v"(invdn));  // materialise the reciprocal here, ahead of the bulk rows
      sfor<r1 + 1, 16>([&](auto r_) {
        constexpr int r = decltype(r_)::value;
        if constexpr (((r - r1 - 1) & 3) == 0) __builtin_amdgcn_sched_barrier(0);
        if constexpr (r == 15) {
          if (full)  // rows 60..63 are padding when n <= 60 (every trot / bound QP at N = 10): S stays 0 there
            dpp_rowf<b0, c0, true, T>(K[r * 4], K[r * 4 + 1], K[r * 4 + 2], K[r * 4 + 3], mm[0], mm[1], mm[2], mm[3]);
        } else {
          dpp_rowf<b0, c0, false, T>(K[r * 4], K[r * 4 + 1], K[r * 4 + 2], K[r * 4 + 3], mm[0], mm[1], mm[2], mm[3]);
        }
      });
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const T mv = -(xn[c] * invdn);
        mm[c] = (c == c1 && lb_m == b1) ? T(0) : mv;
      }
      L.dg[s1] = pivn;
    });
    __builtin_amdgcn_sched_barrier(0);
    cbar();
#ifdef LDL_SPLIT
    IPM_STAMP(3);
#else
    IPM_STAMP(2);
#endif

    // ---- pivots -> 1/d_i (same reciprocal as the factorisation); a NaN pivot is NAN_SOL
    {
      const T d = L.dg[lane];
      invd_v = pivot_inv(d);
      if (uflag(__any(d != d))) {
        status = CMPC_NAN_SOL;
        break;
      }
    }
    // ---- keep only the strict lower part S in the 16 registers that straddle the diagonal (r = 4c .. 4c+3)
    {
      const int la_m = lane0 >> 4, lb_m = lane0 & 15;
      sfor<0, 4>([&](auto c_) {
        constexpr int c = decltype(c_)::value;
        sfor<4 * c, 4 * c + 4>([&](auto r_) {
          constexpr int r = decltype(r_)::value;
          K[r * 4 + c] = (lb_m + 16 * c < la_m + 4 * r) ? K[r * 4 + c] : T(0);
        });
      });
    }
    IPM_STAMP(3);

    // ---- predictor (affine scaling direction)
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int j = lane + 64 * cc;
      L.rml[j] = tl[cc] * ll[cc];
      L.rmu[j] = tu[cc] * lu[cc];
    }
    direction(std::false_type{}, std::integral_constant<int, 5>{});
    T alpha;
    if (m > 0) {
      alpha = fmin(T(1), max_step());
      T maff = T(0);
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        const int j = lane + 64 * cc;
        const bool on = j < m;
        const T v = (tl[cc] + alpha * dtl[cc]) * (ll[cc] + alpha * dll[cc]) +
                    (tu[cc] + alpha * dtu[cc]) * (lu[cc] + alpha * dlu[cc]);
        maff += on ? v : T(0);
      }
      maff = wave_sum_dpp(maff) / T(2 * m);
      const T ratio = maff / mu;
      const T sigma = ratio * ratio * ratio;
      if (st_on && lane == 0) {
        double* sr = st_row();
        sr[0] = (double)alpha;
        sr[1] = (double)maff;
        sr[2] = (double)sigma;
      }
      IPM_STAMP(5);
      // ---- corrector: rm = t.lam + dt_aff.dlam_aff - sigma mu
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        const int j = lane + 64 * cc;
        const bool on = j < m;
        L.rml[j] = on ? tl[cc] * ll[cc] + dtl[cc] * dll[cc] - sigma * mu : T(0);
        L.rmu[j] = on ? tu[cc] * lu[cc] + dtu[cc] * dlu[cc] - sigma * mu : T(0);
      }
      direction(std::false_type{}, std::integral_constant<int, 6>{});
      alpha = fmin(T(1), T(TAU) * max_step());
    } else {
      alpha = fmin(T(1), max_step());
    }
    IPM_STAMP(6);
    if (st_on && lane == 0) {
      double* sr = st_row();
      sr[3] = sr[4] = (double)alpha;
    }  // one step length for primal and dual
    if (uflag(alpha < T(S.alpha_min))) {
      status = CMPC_MIN_STEP;
      break;
    }
    u_v = fma(alpha, du_v, u_v);
    // H du = K du - (C' Sigma C + reg I) du = rhs - D du (D: the 3x3 blocks of this iteration, du still in L.v)
    {
      const int ln = olane();
      const int t3 = 3 * (ln / 3), e = ln - t3;
      T ddu = T(0);
      if (vin) {
#pragma unroll
        for (int d = 0; d < 3; ++d) ddu = fma(L.blk[e][t3 + d], L.v[t3 + d], ddu);
      }
      hu_v = fma(alpha, rhs_v - ddu, hu_v);
    }
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      tl[cc] = fma(alpha, dtl[cc], tl[cc]);
      tu[cc] = fma(alpha, dtu[cc], tu[cc]);
      ll[cc] = fma(alpha, dll[cc], ll[cc]);
      lu[cc] = fma(alpha, dlu[cc], lu[cc]);
    }
    IPM_STAMP(7);
  }

  lane = olane();
  const bool fin = isfinite(u_v);
  if (lane < ld) A.u[(size_t)q * ld + lane] = vin ? u_v : T(0);
  if (uflag(__any(!fin))) status = CMPC_NAN_SOL;
  if (lane == 0) {
    A.status[q] = status;
    A.iters[q] = it;
  }
  if (A.out_u) scatter_result<T>(A, q, n, u_v, status, it, L.scr, lane, 64, [] { cbar(); });
  if (A.res) {  // max over the lanes of the last residual terms (the same lanes stored them)
    const T* rp = A.res_scr + (size_t)q * 3 * 64 + lane;
    const T r0 = wave_max_dpp(rp[0]), r1 = wave_max_dpp(rp[64]), r2 = wave_max_dpp(rp[128]);
    if (lane == 0) {
      double* o = A.res + (size_t)q * 4;
      o[0] = (double)r0;
      o[1] = 0.0;
      o[2] = (double)r1;
      o[3] = (double)r2;
    }
  }
  IPM_STAMP_STORE(A.stamps, q);
}

template <typename T, int WPE>
__global__ __launch_bounds__(64, WPE) void k_ipm64(IpmArgs<T> A) {
  int q = blockIdx.x;
  if (A.qlist[0]) {  // compacted class list: real QPs first, the surplus workgroups exit
    if (q >= A.qcount[0]) return;
    q = A.qlist[0][q];
    if ((unsigned)q >= gridDim.x) return;  // grid = batch: a corrupt list entry cannot address past it
  }
  ipm64_body<T, WPE, 0>(A, nullptr, q);
}

// Fused stage 1 + stage 2 for the n <= 64 class (cmpc_solve_batch, cold start): one launch condenses and solves
// every QP of the class; QPs of the bigger classes only leave their nvar hint (k_class_lists, k_srbd_condense and
// the 128 / 256 IPM kernels follow).
template <typename T, int WPE>
__global__ __launch_bounds__(64, WPE) void k_solve64(IpmArgs<T> A, CondenseArgs<T> C) {
  if (A.app_reset && blockIdx.x == 0 && threadIdx.x < 3) A.app_reset[threadIdx.x] = 0;  // next call's counters
  ipm64_body<T, WPE, 1>(A, &C, (int)blockIdx.x);
}

}  // namespace cmpc
