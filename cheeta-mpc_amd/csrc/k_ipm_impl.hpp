#pragma once
// k_ipm_impl.hpp — stage 2 of the hot path for the size class 64 < n <= 128 (pronk / all-stance at N = 10, trot at
// N = 20): batched dense friction-pyramid QP, primal-dual Mehrotra predictor-corrector interior point method.
// Replaces d_ocp_qp_ipm_solve (HPIPM, called at HpipmInterface.cpp:284) / IPOPT's Newton loop (CentroidalMPC.cpp:354)
// for the condensed centroidal QP; settings and stopping rule mirror hpipm_interface::Settings
// (HpipmInterfaceSettings.h:44-57). The algorithm is restated line by line in oracle/cmpc_oracle.c:oracle_qp_ipm.
//
//   min 1/2 u'Hu + g'u   s.t.  lo <= C u <= hi,   C = blkdiag_a F(mu_a) (5x3 pyramid per stance force triple)
//
// MI355X mapping — one wavefront (64 lanes) per QP, no workgroup barriers:
//   - lane l owns rows l and l + 64 of the Newton matrix K = H + C' diag(lam/t) C, LOWER part only: row l in KA[64]
//     (columns 0..63), row l + 64 in KB[128] — 192 values per lane, so fp64 fits one wave's 512 registers without
//     spilling (a full-row layout would need 256 doubles per lane). Entries right of the diagonal hold finite
//     by-products and are never read;
//   - right-looking Cholesky in place, fully unrolled (every register index static): the scaled column s goes through
//     a 1-KB LDS line (uniform-address broadcast reads), the pivot through v_readlane;
//   - forward substitution: one v_readlane pair + two lane-parallel FMAs per step;
//   - backward substitution (L' x = y) by rows: x_k needs sum_{i>k} L_ik x_i, a wave reduction (DPP + permlane swaps)
//     of the lanes' own L_ik x_i — unknowns not yet solved are 0 so every lane can contribute unmasked;
//   - the per-constraint IPM state (slacks, multipliers, bounds, directions) is parked in LDS, lane-strided;
//   - H is streamed from HBM each iteration (class-packed, stride 128, symmetric so "row i" is read as column i:
//     every load is one contiguous 512-B line);
//   - scheduling barriers fence each phase and each 16-column chunk of the trailing update so the compiler cannot
//     stretch live ranges across the unrolled factorisation.
#include "cmpc_device.hpp"
#include "cmpc_kernels.hpp"
#include "wave_dpp.hpp"

#include <type_traits>

namespace cmpc {

namespace ipm128 {
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
__device__ __forceinline__ bool uniform_flag(bool b) { return __builtin_amdgcn_readfirstlane((int)b) != 0; }
// Lane id the compiler cannot CSE or hoist: every region recomputes its own lane-vs-index masks instead of keeping
// hundreds of 64-bit masks live in SGPRs across the iteration.
__device__ __forceinline__ int opaque_lane() {
  int l = (int)threadIdx.x;
  asm volatile("" : "+v"(l));
  return l;
}
__device__ __forceinline__ void sched_fence() { __builtin_amdgcn_sched_barrier(0); }
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}
// Single-wave workgroup: LDS is in order per wave; this orders the compiler and drains LDS before cross-lane reuse.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

constexpr int NMAX = 128;
constexpr int NTRI = NMAX / 3;
constexpr int MCP = ((5 * NTRI + 63) / 64) * 64;  // constraint rows, padded to lanes
constexpr int CPL = MCP / 64;                     // constraint rows per lane

template <typename T>
struct Lds {
  T v[NMAX];    // row-vector broadcast
  T col[NMAX];  // factor column broadcast
  T w[MCP];     // constraint-vector broadcast (C')
  T lo[MCP], hi[MCP], mu[MCP];
  T tl[MCP], tu[MCP], ll[MCP], lu[MCP];
  T rl[MCP], ru[MCP], itl[MCP], itu[MCP];
  T dtl[MCP], dtu[MCP], dll[MCP], dlu[MCP], rml[MCP], rmu[MCP];
};
}  // namespace ipm128

template <typename T, int WPE>
__global__ __launch_bounds__(64, WPE) void k_ipm128(IpmArgs<T> a) {
  using namespace ipm128;
  constexpr int CH = 16;  // trailing-update chunk (columns per scheduling region)

  const int q = blockIdx.x;
  if (a.status[q] != CMPC_SUCCESS) return;  // invalid contact table / too large: status already set
  const int n = a.nvar[q];
  if (n <= 64 || n > NMAX) return;          // served by another size class
  const int ld = a.ld;
  const int nt = n / 3;
  const int m = 5 * nt;
  const DevSettings S = a.s;
  __shared__ Lds<T> L;

  // ---- row data (row i = lane + 64 r)
  T g_r[2], mu_r[2], u_r[2];
  {
    const int lane = opaque_lane();
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = lane + 64 * r;
      g_r[r] = i < n ? a.g[(size_t)q * ld + i] : T(0);
      mu_r[r] = i < n ? a.tri_mu[(size_t)q * (ld / 3) + i / 3] : T(0);
      // cold start (warm_start = 0): u = 0; warm start: u from the workspace (cmpc_solve_batch_warm)
      u_r[r] = (a.warm && i < n) ? a.u[(size_t)q * ld + i] : T(0);
      L.v[i] = u_r[r];
    }
    wave_sync();
    // ---- constraint data (row j = lane + 64 c): slacks of C u clipped at THR0, lam = mu0 / t
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int j = lane + 64 * c;
      const bool on = j < m;
      const int t = j / 5;
      const T lo = on ? a.tri_lo[((size_t)q * (ld / 3) + t) * 5 + j % 5] : T(0);
      const T hi = on ? a.tri_hi[((size_t)q * (ld / 3) + t) * 5 + j % 5] : T(0);
      L.lo[j] = lo;
      L.hi[j] = hi;
      L.mu[j] = on ? a.tri_mu[(size_t)q * (ld / 3) + t] : T(0);
      const T cu0 = on ? pyr_row<T>(j % 5, L.mu[j], L.v[3 * t], L.v[3 * t + 1], L.v[3 * t + 2]) : T(0);
      const T tl = on ? fmax(cu0 - lo, T(THR0)) : T(1);
      const T tu = on ? fmax(hi - cu0, T(THR0)) : T(1);
      L.tl[j] = tl;
      L.tu[j] = tu;
      L.ll[j] = on ? T(S.mu0) / tl : T(0);
      L.lu[j] = on ? T(S.mu0) / tu : T(0);
    }
    wave_sync();
  }

  // out_c = C x_r  (pyramid rows of each triple), written to an LDS constraint array
  auto apply_C = [&](const T (&x)[2], T* out) {
    const int lane = opaque_lane();
    L.v[lane] = x[0];
    L.v[lane + 64] = x[1];
    wave_sync();
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int j = lane + 64 * c;
      const int t = j / 5;
      T v = T(0);
      if (j < m) v = pyr_row<T>(j % 5, L.mu[j], L.v[3 * t], L.v[3 * t + 1], L.v[3 * t + 2]);
      out[j] = v;
    }
    wave_sync();
  };
  // x_r = C' w, with w already in L.w
  auto apply_CT = [&](T (&x)[2]) {
    const int lane = opaque_lane();
    wave_sync();
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = lane + 64 * r;
      T v = T(0);
      if (i < n) {
        const int t = i / 3, dd = i % 3;
        const T w0 = L.w[5 * t], w1 = L.w[5 * t + 1], w2 = L.w[5 * t + 2], w3 = L.w[5 * t + 3], w4 = L.w[5 * t + 4];
        v = dd == 0 ? (w1 - w0) : (dd == 1 ? (w3 - w2) : (mu_r[r] * (w0 + w1 + w2 + w3) + w4));
      }
      x[r] = v;
    }
    wave_sync();
  };

  T KA[64];   // row lane,      columns 0..63
  T KB[128];  // row lane + 64, columns 0..127
  T invL[2], dg[2];

  // (L L') x = b with the in-place lower factor (L_ii = sqrt(d_i), 1 / L_ii = invL)
  auto chol_solve = [&](T (&y)[2]) {
    sched_fence();
    {
      // forward: y_k = y_k / L_kk broadcast, then y_i -= L_ik y_k for the rows below
      const int lane = opaque_lane();
      static_for<0, NMAX>([&](auto k_) {
        constexpr int k = decltype(k_)::value;
        constexpr int rk = k / 64, lk = k % 64;
        if constexpr (k % CH == 0) sched_fence();
        const T sv = readlane(y[rk] * invL[rk], lk);
        if constexpr (k < 64) y[0] = (lane == k) ? sv : ((lane > k) ? fma(-KA[k], sv, y[0]) : y[0]);
        y[1] = (lane + 64 == k) ? sv : ((lane + 64 > k) ? fma(-KB[k], sv, y[1]) : y[1]);
      });
    }
    sched_fence();
    {
      // backward, row k from the bottom: x_k = (y_k - sum_{i>k} L_ik x_i) / L_kk. The lanes' products use the
      // unknowns solved so far (x = 0 elsewhere), reduced over the wave; lane k (row k) then finishes x_k.
      const int lane = opaque_lane();
      T x0 = T(0), x1 = T(0);
      static_for<0, NMAX>([&](auto kk_) {
        constexpr int k = NMAX - 1 - decltype(kk_)::value;
        constexpr int rk = k / 64, lk = k % 64;
        if constexpr (k % CH == 0) sched_fence();
        T p = KB[k] * x1;
        if constexpr (k < 64) p = fma(KA[k], x0, p);
        const T s = wave_sum_dpp(p);
        if constexpr (rk == 0) {
          if (lane == lk) x0 = (y[0] - s) * invL[0];
        } else {
          if (lane == lk) x1 = (y[1] - s) * invL[1];
        }
      });
      y[0] = x0;
      y[1] = x1;
    }
    sched_fence();
  };

  const T* Hq = a.H + (size_t)q * ld * ld;  // class-packed NMAX x NMAX block at the start of the QP's slab
  int status = CMPC_MAX_ITER;
  int it = 0;
  T rg[2], du[2];

  // Newton direction for the complementarity targets in L.rml / L.rmu (constraint lanes)
  auto direction = [&]() {
    {
      const int lane = opaque_lane();
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int j = lane + 64 * c;
        L.w[j] = (L.rml[j] + L.ll[j] * L.rl[j]) * L.itl[j] - (L.rmu[j] + L.lu[j] * L.ru[j]) * L.itu[j];
      }
    }
    T ctw[2];
    apply_CT(ctw);
#pragma unroll
    for (int r = 0; r < 2; ++r) du[r] = -rg[r] - ctw[r];
    chol_solve(du);
    apply_C(du, L.w);  // C du -> L.w
    {
      const int lane = opaque_lane();
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int j = lane + 64 * c;
        const T cdu = L.w[j];
        const T dtl = cdu + L.rl[j], dtu = L.ru[j] - cdu;
        L.dtl[j] = dtl;
        L.dtu[j] = dtu;
        L.dll[j] = -(L.rml[j] + L.ll[j] * dtl) * L.itl[j];
        L.dlu[j] = -(L.rmu[j] + L.lu[j] * dtu) * L.itu[j];
      }
    }
  };
  auto max_step = [&]() -> T {
    const int lane = opaque_lane();
    T am = T(1e30);
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int j = lane + 64 * c;
      const T dtl = L.dtl[j], dtu = L.dtu[j], dll = L.dll[j], dlu = L.dlu[j];
      if (dtl < T(0)) am = fmin(am, -L.tl[j] / dtl);
      if (dtu < T(0)) am = fmin(am, -L.tu[j] / dtu);
      if (dll < T(0)) am = fmin(am, -L.ll[j] / dll);
      if (dlu < T(0)) am = fmin(am, -L.lu[j] / dlu);
    }
    return wave_min_dpp(am);
  };

  for (it = 0;; ++it) {
    sched_fence();
    // ---- stream H (class-packed, stride NMAX; symmetric: element (j, i) == (i, j); coalesced 8-B lanes)
    {
      const int lane = opaque_lane();
      const T* hp = Hq + lane;
      static_for<0, NMAX>([&](auto j_) {
        constexpr int j = decltype(j_)::value;
        if constexpr (j < 64) KA[j] = hp[j * NMAX];
        KB[j] = hp[j * NMAX + 64];
      });
    }
    sched_fence();

    // ---- residuals
    apply_C(u_r, L.w);  // C u -> L.w (kept until the constraint residuals below)
    T hu[2];
    {
      // H u: the freshly loaded registers hold H itself, full rows for l + 64 (KB) and columns 0..63 of row l (KA);
      // row l's columns 64..127 are re-read from H (symmetric: H[l][j] = H[j][l], again a 512-B line per load)
      const int lane = opaque_lane();
      L.v[lane] = u_r[0];
      L.v[lane + 64] = u_r[1];
      wave_sync();
      hu[0] = T(0);
      hu[1] = T(0);
      const T* hp = Hq + lane;
      static_for<0, 4>([&](auto c_) {
        constexpr int c = decltype(c_)::value;
        T e[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) e[t] = hp[(64 + 16 * c + t) * NMAX];
        static_for<0, 16>([&](auto t_) {
          constexpr int j = 16 * c + decltype(t_)::value;
          const T uj = L.v[j];
          hu[0] = fma(KA[j], uj, hu[0]);
          hu[1] = fma(KB[j], uj, hu[1]);
        });
        sched_fence();
#pragma unroll
        for (int t = 0; t < 16; ++t) {
          const T uj = L.v[64 + 16 * c + t];
          hu[0] = fma(e[t], uj, hu[0]);
          hu[1] = fma(KB[64 + 16 * c + t], uj, hu[1]);
        }
        sched_fence();
      });
      wave_sync();
    }
    T rs = T(0), ri = T(0), rc = T(0), ms = T(0);
    {
      const int lane = opaque_lane();
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int j = lane + 64 * c;
        const bool on = j < m;
        const T cu = L.w[j];
        const T tl = L.tl[j], tu = L.tu[j], ll = L.ll[j], lu = L.lu[j];
        const T rl = on ? cu - L.lo[j] - tl : T(0);
        const T ru = on ? L.hi[j] - cu - tu : T(0);
        L.rl[j] = rl;
        L.ru[j] = ru;
        ri = fmax(ri, fmax(fabs(rl), fabs(ru)));
        const T cl = tl * ll, ch = tu * lu;
        rc = fmax(rc, fmax(cl, ch));
        ms += cl + ch;
      }
      wave_sync();
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int j = lane + 64 * c;
        L.w[j] = L.ll[j] - L.lu[j];
      }
    }
    T ctw[2];
    apply_CT(ctw);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      rg[r] = hu[r] + g_r[r] - ctw[r];
      rs = fmax(rs, fabs(rg[r]));
    }
    rs = wave_max_dpp(rs);
    ri = wave_max_dpp(ri);
    rc = wave_max_dpp(rc);
    ms = wave_sum_dpp(ms);
    const T mu = m > 0 ? ms / T(2 * m) : T(0);
    if (uniform_flag(!(isfinite(rs) && isfinite(ri) && isfinite(rc)))) {
      status = CMPC_NAN_SOL;
      break;
    }
    if (uniform_flag(rs <= T(S.tol_stat) && ri <= T(S.tol_ineq) && rc <= T(S.tol_comp))) {
      status = CMPC_SUCCESS;
      break;
    }
    if (it >= S.iter_max) {
      status = CMPC_MAX_ITER;
      break;
    }
    // mu underflow (a stagnating primal residual below the precision of the bounds): stop instead of 0/0
    if (uniform_flag(m > 0 && !(mu > T(Lim<T>::mu_min)))) {
      status = CMPC_MIN_STEP;
      break;
    }

    // ---- Newton matrix K = H + C' diag(lam_l/t_l + lam_u/t_u) C + reg I  (3x3 blocks on the triple diagonal)
    {
      const int lane = opaque_lane();
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int j = lane + 64 * c;
        const bool on = j < m;
        const T itl = on ? T(1) / L.tl[j] : T(0);
        const T itu = on ? T(1) / L.tu[j] : T(0);
        L.itl[j] = itl;
        L.itu[j] = itu;
        L.w[j] = L.ll[j] * itl + L.lu[j] * itu;
      }
      wave_sync();
      T b[2][3];
      int ti[2];
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int i = lane + 64 * r;
        T b0 = T(0), b1 = T(0), b2 = T(0);
        ti[r] = i / 3;
        const int dd = i % 3;
        if (i < n) {
          const int t = ti[r];
          const T s0 = L.w[5 * t], s1 = L.w[5 * t + 1], s2 = L.w[5 * t + 2], s3 = L.w[5 * t + 3], s4 = L.w[5 * t + 4];
          const T mu_t = mu_r[r];
          const T xx = s0 + s1, yy = s2 + s3, zz = mu_t * mu_t * (s0 + s1 + s2 + s3) + s4;
          const T xz = mu_t * (s1 - s0), yz = mu_t * (s3 - s2);
          b0 = dd == 0 ? xx : (dd == 1 ? T(0) : xz);
          b1 = dd == 0 ? T(0) : (dd == 1 ? yy : yz);
          b2 = dd == 0 ? xz : (dd == 1 ? yz : zz);
        }
        const T reg = T(S.reg_prim);
        b[r][0] = b0 + (dd == 0 ? reg : T(0));
        b[r][1] = b1 + (dd == 1 ? reg : T(0));
        b[r][2] = b2 + (dd == 2 ? reg : T(0));
      }
      static_for<0, NTRI>([&](auto J_) {
        constexpr int J = decltype(J_)::value;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          if (3 * J + d < 64) KA[3 * J + d] += ti[0] == J ? b[0][d] : T(0);
          KB[3 * J + d] += ti[1] == J ? b[1][d] : T(0);
        }
      });
      wave_sync();
    }

    // ---- right-looking lower Cholesky, in place
    bool ok = true;
#pragma unroll
    for (int r = 0; r < 2; ++r) invL[r] = dg[r] = T(1);
    static_for<0, NMAX>([&](auto s_) {
      constexpr int s = decltype(s_)::value;
      constexpr int rs_ = s / 64, ls = s % 64;
      sched_fence();
      const int lane = opaque_lane();
      T d;
      if constexpr (rs_ == 0) d = readlane(KA[s], ls);
      else d = readlane(KB[s], ls);
      // BLASFEO-style guard: a pivot lost to cancellation (possible in fp32 late in the IPM) drops its direction
      // (inverse 0) instead of failing; mirrored in oracle_qp_ipm. Computed unconditionally, then selected.
      const T il0 = rsqrt_acc(fmax(d, T(Lim<T>::pivot_min)));
      const T il = d > T(Lim<T>::pivot_min) ? il0 : T(0);
      {
        const bool piv = lane == ls;
        invL[rs_] = piv ? il : invL[rs_];
        dg[rs_] = piv ? d : dg[rs_];
        asm volatile("" : "+v"(invL[rs_]), "+v"(dg[rs_]));
      }
      T bA = T(0), bB;
      if constexpr (s < 64) {
        const bool below = lane > s;
        bA = below ? KA[s] * il : T(0);
        KA[s] = below ? bA : KA[s];
        asm volatile("" : "+v"(KA[s]));
        L.col[lane] = bA;
      }
      {
        const bool below = lane + 64 > s;
        bB = below ? KB[s] * il : T(0);
        KB[s] = below ? bB : KB[s];
        asm volatile("" : "+v"(KB[s]));
        L.col[lane + 64] = bB;
      }
      wave_sync();
      static_for<s + 1, NMAX>([&](auto j_) {
        constexpr int j = decltype(j_)::value;
        if constexpr ((j - s - 1) % CH == 0) sched_fence();
        const T lj = L.col[j];
        if constexpr (s < 64 && j < 64) KA[j] = fma(-bA, lj, KA[j]);
        KB[j] = fma(-bB, lj, KB[j]);
      });
      sched_fence();
      wave_sync();
    });
    // NaN pivot -> NAN_SOL (checked once from the recorded pivots)
#pragma unroll
    for (int r = 0; r < 2; ++r) ok = ok && !(dg[r] != dg[r]);
    if (uniform_flag(__any(!ok))) {
      status = CMPC_NAN_SOL;
      break;
    }

    // ---- predictor (affine scaling direction)
    {
      const int lane = opaque_lane();
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int j = lane + 64 * c;
        L.rml[j] = L.tl[j] * L.ll[j];
        L.rmu[j] = L.tu[j] * L.lu[j];
      }
    }
    direction();
    T alpha = fmin(T(1), max_step());
    if (m > 0) {
      T maff = T(0);
      {
        const int lane = opaque_lane();
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const int j = lane + 64 * c;
          maff += (L.tl[j] + alpha * L.dtl[j]) * (L.ll[j] + alpha * L.dll[j]) +
                  (L.tu[j] + alpha * L.dtu[j]) * (L.lu[j] + alpha * L.dlu[j]);
        }
      }
      maff = wave_sum_dpp(maff) / T(2 * m);
      const T ratio = maff / mu;
      const T sigma = ratio * ratio * ratio;
      // ---- corrector: rm = t.lam + dt_aff.dlam_aff - sigma mu
      {
        const int lane = opaque_lane();
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          const int j = lane + 64 * c;
          const bool on = j < m;
          L.rml[j] = on ? L.tl[j] * L.ll[j] + L.dtl[j] * L.dll[j] - sigma * mu : T(0);
          L.rmu[j] = on ? L.tu[j] * L.lu[j] + L.dtu[j] * L.dlu[j] - sigma * mu : T(0);
        }
      }
      direction();
      alpha = fmin(T(1), T(TAU) * max_step());
    }
    if (uniform_flag(alpha < T(S.alpha_min))) {
      status = CMPC_MIN_STEP;
      break;
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) u_r[r] = fma(alpha, du[r], u_r[r]);
    {
      const int lane = opaque_lane();
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const int j = lane + 64 * c;
        L.tl[j] = fma(alpha, L.dtl[j], L.tl[j]);
        L.tu[j] = fma(alpha, L.dtu[j], L.tu[j]);
        L.ll[j] = fma(alpha, L.dll[j], L.ll[j]);
        L.lu[j] = fma(alpha, L.dlu[j], L.lu[j]);
      }
      wave_sync();
    }
  }

  bool fin = true;
  const int lane = opaque_lane();
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int i = lane + 64 * r;
    fin = fin && isfinite(u_r[r]);
    if (i < ld) a.u[(size_t)q * ld + i] = i < n ? u_r[r] : T(0);
  }
  if (uniform_flag(__any(!fin))) status = CMPC_NAN_SOL;
  if (lane == 0) {
    a.status[q] = status;
    a.iters[q] = it;
  }
}

}  // namespace cmpc
