#pragma once
// k_ipm_impl.hpp — stage 2 of the hot path: batched dense friction-pyramid QP, primal-dual Mehrotra predictor-corrector
// interior point method. Replaces d_ocp_qp_ipm_solve (HPIPM, called at HpipmInterface.cpp:284) / IPOPT's Newton loop
// (CentroidalMPC.cpp:354) for the condensed centroidal QP; settings and stopping rule mirror
// hpipm_interface::Settings (HpipmInterfaceSettings.h:44-57). The algorithm is restated line by line in
// oracle/cmpc_oracle.c:oracle_qp_ipm (the CPU checker).
//
//   min 1/2 u'Hu + g'u   s.t.  lo <= C u <= hi,   C = blkdiag_a F(mu_a) (5x3 pyramid per stance force triple)
//
// MI355X mapping — one wavefront (64 lanes) per QP, no workgroup barriers:
//   - lane i owns row i of the Newton matrix K = H + C' diag(lam/t) C (RPL = NMAX/64 rows per lane) in VGPRs;
//     the factor is computed in place by a right-looking Cholesky, fully unrolled so every register index is static;
//     column s of L is broadcast through a 512-B LDS line (wave-uniform ds_read_b128), the pivot through v_readlane;
//   - the factor keeps BOTH triangles: lane i holds L_ik (k < i) and U~_ik = L_ii L_ki (k > i), so the forward AND
//     the backward substitution are lane-parallel axpys driven by one v_readlane scalar per step — no transposes;
//   - the per-constraint IPM state (slacks, multipliers, bounds, directions) is parked in LDS, lane-strided, so the
//     VGPR budget is the Newton matrix plus a handful of row vectors (2 waves/SIMD in fp64);
//   - C and C' are applied through LDS broadcasts; H is streamed from HBM each iteration (class-packed, stride NMAX,
//     symmetric so "row i" is read as column i: every load instruction is one contiguous 512-B line);
//   - every reduction (residual norms, mu, step length) is a 64-lane butterfly; the loop exit is wave-uniform;
//   - scheduling barriers fence each phase and each 16-column chunk of the trailing update so the compiler cannot
//     stretch live ranges across the unrolled factorisation (it spills otherwise).
#include "cmpc_device.hpp"
#include "cmpc_kernels.hpp"
#include "lab_stamps.hpp"

#include <type_traits>

namespace {
using namespace cmpc;

template <typename T>
struct PIVOT_MIN;
template <>
struct PIVOT_MIN<double> {
  static constexpr double v = 1e-200;
};
template <>
struct PIVOT_MIN<float> {
  static constexpr float v = 1e-30f;
};
template <typename T>
struct MU_MIN;
template <>
struct MU_MIN<double> {
  static constexpr double v = 1e-300;
};
template <>
struct MU_MIN<float> {
  static constexpr float v = 1e-35f;
};
__device__ __forceinline__ bool uniform_flag(bool b) { return __builtin_amdgcn_readfirstlane((int)b) != 0; }
// Lane id the compiler cannot CSE or hoist: every region recomputes its own lane-vs-index masks instead of keeping
// ~200 64-bit masks live in SGPRs across the iteration.
__device__ __forceinline__ int opaque_lane() {
  int l = (int)threadIdx.x;
  asm volatile("" : "+v"(l));
  return l;
}
__device__ __forceinline__ void sched_fence() { __builtin_amdgcn_sched_barrier(0); }
// Compile-time loop: every index is a constant expression, so register arrays stay in VGPRs without relying on
// the loop unroller (which gives up on the triangular nest of the factorisation and demotes K to scratch).
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

template <typename T, int NMAX>
struct IpmLds {
  static constexpr int NTRI = NMAX / 3;
  static constexpr int MCP = ((5 * NTRI + 63) / 64) * 64;  // constraint rows, padded to lanes
  T v[NMAX];     // row-vector broadcast
  T col[NMAX];   // factor column broadcast
  T w[MCP];      // constraint-vector broadcast (C')
  T lo[MCP], hi[MCP], mu[MCP];
  T tl[MCP], tu[MCP], ll[MCP], lu[MCP];
  T rl[MCP], ru[MCP], itl[MCP], itu[MCP];
  T dtl[MCP], dtu[MCP], dll[MCP], dlu[MCP], rml[MCP], rmu[MCP];
};

template <typename T, int NMAX, int WPE>
__global__ __launch_bounds__(64, WPE) void k_ipm_reg(IpmArgs<T> a, unsigned long long* stamps) {
  STAMP_DECL;
  constexpr int RPL = NMAX / 64;                  // Newton-matrix rows per lane
  constexpr int NTRI = NMAX / 3;                  // force triples
  constexpr int CPL = IpmLds<T, NMAX>::MCP / 64;  // constraint rows per lane
  constexpr int LO_CLASS = NMAX == 64 ? -1 : NMAX / 2;
  constexpr int CH = 16;                          // trailing-update chunk (columns per scheduling region)

  const int q = blockIdx.x;
  if (a.status[q] != CMPC_SUCCESS) return;  // invalid contact table / too large: status already set
  const int n = a.nvar[q];
  if (n <= LO_CLASS || n > NMAX) return;    // served by another size class
  const int ld = a.ld;
  const int nt = n / 3;
  const int m = 5 * nt;
  const DevSettings S = a.s;
  __shared__ IpmLds<T, NMAX> L;

  // ---- row data (row i = lane + 64 r)
  T g_r[RPL], mu_r[RPL], u_r[RPL];
  {
    const int lane = opaque_lane();
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      const int i = lane + 64 * r;
      g_r[r] = i < n ? a.g[(size_t)q * ld + i] : T(0);
      mu_r[r] = i < n ? a.tri_mu[(size_t)q * (ld / 3) + i / 3] : T(0);
      u_r[r] = T(0);
    }
    // ---- constraint data (row j = lane + 64 c), cold start (warm_start = 0): u = 0, slacks clipped at THR0,
    //      lam = mu0 / t
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
      const T tl = on ? fmax(-lo, T(THR0)) : T(1);
      const T tu = on ? fmax(hi, T(THR0)) : T(1);
      L.tl[j] = tl;
      L.tu[j] = tu;
      L.ll[j] = on ? T(S.mu0) / tl : T(0);
      L.lu[j] = on ? T(S.mu0) / tu : T(0);
    }
  }

  // out_c = C x_r  (pyramid rows of each triple), written to an LDS constraint array
  auto apply_C = [&](const T (&x)[RPL], T* out) {
    const int lane = opaque_lane();
#pragma unroll
    for (int r = 0; r < RPL; ++r) L.v[lane + 64 * r] = x[r];
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
  auto apply_CT = [&](T (&x)[RPL]) {
    const int lane = opaque_lane();
    wave_sync();
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
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

  T K[RPL][NMAX];
  T invL[RPL], dg[RPL];

  // (L L') x = b with the in-place factor in K (see header comment)
  auto chol_solve = [&](T (&y)[RPL]) {
    sched_fence();
    {
      const int lane = opaque_lane();
#pragma unroll
      for (int k = 0; k < NMAX; ++k) {
        const int rk = k / 64, lk = k % 64;
        const T sv = readlane(y[rk] * invL[rk], lk);
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
          const int i = lane + 64 * r;
          y[r] = (i == k) ? sv : ((i > k) ? fma(-K[r][k], sv, y[r]) : y[r]);
        }
      }
    }
    sched_fence();
    // U~ x = D y, U~_ik = L_ii L_ki (k > i), U~_ii = L_ii^2, D = diag(L_ii)
#pragma unroll
    for (int r = 0; r < RPL; ++r) y[r] = y[r] * (dg[r] * invL[r]);
    {
      const int lane = opaque_lane();
#pragma unroll
      for (int k = NMAX - 1; k >= 0; --k) {
        const int rk = k / 64, lk = k % 64;
        const T sv = readlane(y[rk] * (invL[rk] * invL[rk]), lk);
#pragma unroll
        for (int r = 0; r < RPL; ++r) {
          const int i = lane + 64 * r;
          y[r] = (i == k) ? sv : ((i < k) ? fma(-K[r][k], sv, y[r]) : y[r]);
        }
      }
    }
    sched_fence();
  };

  const T* Hq = a.H + (size_t)q * ld * ld;  // class-packed NMAX x NMAX block at the start of the QP's slab
  int status = CMPC_MAX_ITER;
  int it = 0;
  T rg[RPL], du[RPL];

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
    T ctw[RPL];
    apply_CT(ctw);
#pragma unroll
    for (int r = 0; r < RPL; ++r) du[r] = -rg[r] - ctw[r];
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
    return wave_min(am);
  };

  for (it = 0;; ++it) {
    STAMP(7);
    sched_fence();
    // ---- stream H (class-packed, stride NMAX; symmetric: element (j, i) == (i, j); coalesced 8-B lanes)
    {
      const int lane = opaque_lane();
      const T* hp = Hq + lane;
      static_for<0, NMAX>([&](auto j_) {
        constexpr int j = decltype(j_)::value;
#pragma unroll
        for (int r = 0; r < RPL; ++r) K[r][j] = hp[j * NMAX + 64 * r];
      });
    }
    sched_fence();
    STAMP(0);

    // ---- residuals
    apply_C(u_r, L.w);  // C u -> L.w (kept until the constraint residuals below)
    T hu[RPL];
    {
      const int lane = opaque_lane();
#pragma unroll
      for (int r = 0; r < RPL; ++r) L.v[lane + 64 * r] = u_r[r];
      wave_sync();
#pragma unroll
      for (int r = 0; r < RPL; ++r) hu[r] = T(0);
      static_for<0, NMAX>([&](auto j_) {
        constexpr int j = decltype(j_)::value;
        if constexpr (j % CH == 0) sched_fence();
        const T uj = L.v[j];
#pragma unroll
        for (int r = 0; r < RPL; ++r) hu[r] = fma(K[r][j], uj, hu[r]);
      });
      sched_fence();
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
    T ctw[RPL];
    apply_CT(ctw);
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      rg[r] = hu[r] + g_r[r] - ctw[r];
      rs = fmax(rs, fabs(rg[r]));
    }
    rs = wave_max(rs);
    ri = wave_max(ri);
    rc = wave_max(rc);
    ms = wave_sum(ms);
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
    if (uniform_flag(m > 0 && !(mu > T(MU_MIN<T>::v)))) {
      status = CMPC_MIN_STEP;
      break;
    }

    STAMP(1);
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
#pragma unroll
      for (int r = 0; r < RPL; ++r) {
        const int i = lane + 64 * r;
        T b0 = T(0), b1 = T(0), b2 = T(0);
        const int ti = i / 3, dd = i % 3;
        if (i < n) {
          const T s0 = L.w[5 * ti], s1 = L.w[5 * ti + 1], s2 = L.w[5 * ti + 2], s3 = L.w[5 * ti + 3],
                  s4 = L.w[5 * ti + 4];
          const T mu_t = mu_r[r];
          const T xx = s0 + s1, yy = s2 + s3, zz = mu_t * mu_t * (s0 + s1 + s2 + s3) + s4;
          const T xz = mu_t * (s1 - s0), yz = mu_t * (s3 - s2);
          b0 = dd == 0 ? xx : (dd == 1 ? T(0) : xz);
          b1 = dd == 0 ? T(0) : (dd == 1 ? yy : yz);
          b2 = dd == 0 ? xz : (dd == 1 ? yz : zz);
        }
        const T reg = T(S.reg_prim);
        b0 += dd == 0 ? reg : T(0);
        b1 += dd == 1 ? reg : T(0);
        b2 += dd == 2 ? reg : T(0);
#pragma unroll
        for (int J = 0; J < NTRI; ++J) {
          const bool mine = (ti == J);
          K[r][3 * J + 0] += mine ? b0 : T(0);
          K[r][3 * J + 1] += mine ? b1 : T(0);
          K[r][3 * J + 2] += mine ? b2 : T(0);
        }
      }
      wave_sync();
    }

    STAMP(2);
    // ---- right-looking Cholesky, in place, both triangles kept (see header)
    bool ok = true;
#pragma unroll
    for (int r = 0; r < RPL; ++r) invL[r] = dg[r] = T(1);
    static_for<0, NMAX>([&](auto s_) {
      constexpr int s = decltype(s_)::value;
      sched_fence();
      const int lane = opaque_lane();
      constexpr int rs_ = s / 64, ls = s % 64;
      const T d = readlane(K[rs_][s], ls);
      // BLASFEO-style guard: a pivot lost to cancellation (possible in fp32 late in the IPM) drops its direction
      // (inverse 0) instead of failing; mirrored in oracle_qp_ipm.
      // (computed unconditionally then selected: a guarded call becomes a uniform branch per pivot, and the 128
      // basic blocks that makes wreck register allocation across the factorisation)
      const T il0 = rsqrt_acc(fmax(d, T(PIVOT_MIN<T>::v)));
      const T il = d > T(PIVOT_MIN<T>::v) ? il0 : T(0);
      T bsc[RPL];
#pragma unroll
      for (int r = 0; r < RPL; ++r) {
        const int i = lane + 64 * r;
        // The selects are pinned where they are computed (asm barrier): left alone, the compiler sinks them to their
        // first use in the substitutions and keeps 64 pivots + masks live across the whole factorisation (spills).
        if (r == rs_) {
          const bool piv = lane == ls;
          invL[r] = piv ? il : invL[r];
          dg[r] = piv ? d : dg[r];
          asm volatile("" : "+v"(invL[r]), "+v"(dg[r]));
        }
        const bool below = i > s;
        bsc[r] = below ? K[r][s] * il : T(0);
        K[r][s] = below ? bsc[r] : K[r][s];
        asm volatile("" : "+v"(K[r][s]));
        L.col[i] = bsc[r];
      }
      wave_sync();
      static_for<s + 1, NMAX>([&](auto j_) {
        constexpr int j = decltype(j_)::value;
        if constexpr ((j - s - 1) % CH == 0) sched_fence();
        const T lj = L.col[j];
#pragma unroll
        for (int r = 0; r < RPL; ++r) K[r][j] = fma(-bsc[r], lj, K[r][j]);
      });
      sched_fence();
      wave_sync();
    });
    // NaN pivot -> NAN_SOL (checked once from the recorded pivots: a per-step flag would keep all 64 pivots live)
#pragma unroll
    for (int r = 0; r < RPL; ++r) ok = ok && !(dg[r] != dg[r]);
    if (uniform_flag(__any(!ok))) {
      status = CMPC_NAN_SOL;
      break;
    }

    STAMP(3);
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
      maff = wave_sum(maff) / T(2 * m);
      const T ratio = maff / mu;
      const T sigma = ratio * ratio * ratio;
      STAMP(4);
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
    STAMP(5);
    if (uniform_flag(alpha < T(S.alpha_min))) {
      status = CMPC_MIN_STEP;
      break;
    }
#pragma unroll
    for (int r = 0; r < RPL; ++r) u_r[r] = fma(alpha, du[r], u_r[r]);
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
    STAMP(6);
  }

  bool fin = true;
  const int lane = opaque_lane();
#pragma unroll
  for (int r = 0; r < RPL; ++r) {
    const int i = lane + 64 * r;
    fin = fin && isfinite(u_r[r]);
    if (i < ld) a.u[(size_t)q * ld + i] = i < n ? u_r[r] : T(0);
  }
  if (uniform_flag(__any(!fin))) status = CMPC_NAN_SOL;
  if (lane == 0) {
    a.status[q] = status;
    a.iters[q] = it;
  }
  STAMP_STORE(stamps, q);
}

}  // namespace
