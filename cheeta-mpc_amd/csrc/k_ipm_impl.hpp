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
//     column s of L is broadcast through a 512-B LDS line (wave-uniform ds_read), the pivot through v_readlane;
//   - the factor keeps BOTH triangles: lane i holds L_ik (k < i) and U~_ik = L_ii L_ki (k > i), so the forward AND
//     the backward substitution are lane-parallel axpys driven by one v_readlane scalar per step — no transposes;
//   - constraint rows are lane-strided (CPL per lane); C and C' are applied through LDS broadcasts;
//   - H is streamed from HBM each iteration with coalesced 512-B row loads (symmetric, so "row i" = column i);
//   - every reduction (residual norms, mu, step length) is a 64-lane butterfly; the loop exit is wave-uniform.
#include "cmpc_device.hpp"
#include "cmpc_kernels.hpp"

namespace cmpc {

namespace {
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
__device__ __forceinline__ bool uniform_flag(bool b) {
  return __builtin_amdgcn_readfirstlane((int)b) != 0;
}
// Lane id the compiler cannot CSE or hoist: every region (factorisation, each substitution, C / C' application)
// recomputes its own lane-vs-index masks instead of keeping ~200 64-bit masks live in SGPRs across the iteration.
__device__ __forceinline__ int opaque_lane() {
  int l = (int)threadIdx.x;
  asm volatile("" : "+v"(l));
  return l;
}
template <typename T>
__device__ __forceinline__ T recip(T x) {
  return T(1) / x;
}
}  // namespace

template <typename T, int NMAX>
__global__ __launch_bounds__(64, (sizeof(T) == 4 && NMAX == 64) ? 2 : 1) void k_ipm_reg(IpmArgs<T> a) {
  constexpr int RPL = NMAX / 64;           // Newton-matrix rows per lane
  constexpr int NTRI = NMAX / 3;           // force triples
  constexpr int MC = 5 * NTRI;             // pyramid rows
  constexpr int CPL = (MC + 63) / 64;      // constraint rows per lane
  constexpr int LO_CLASS = NMAX == 64 ? -1 : NMAX / 2;

  const int q = blockIdx.x;
  const int lane0 = threadIdx.x;
  int lane = lane0;
  if (a.status[q] != CMPC_SUCCESS) return;  // invalid contact table / too large: status already set
  const int n = a.nvar[q];
  if (n <= LO_CLASS || n > NMAX) return;    // served by another size class
  const int ld = a.ld;
  const int nt = n / 3;
  const int m = 5 * nt;
  const DevSettings S = a.s;

  __shared__ T s_v[NMAX];
  __shared__ T s_c[CPL * 64];
  __shared__ T s_col[NMAX];

  // ---- row data (row i = lane + 64 r)
  T g_r[RPL], mu_r[RPL], u_r[RPL];
#pragma unroll
  for (int r = 0; r < RPL; ++r) {
    const int i = lane + 64 * r;
    g_r[r] = i < n ? a.g[(size_t)q * ld + i] : T(0);
    mu_r[r] = i < n ? a.tri_mu[(size_t)q * (ld / 3) + i / 3] : T(0);
    u_r[r] = T(0);
  }
  // ---- constraint data (row j = lane + 64 c)
  T lo_c[CPL], hi_c[CPL], mu_c[CPL], tl[CPL], tu[CPL], ll[CPL], lu[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int j = lane + 64 * c;
    const bool on = j < m;
    const int t = j / 5;
    lo_c[c] = on ? a.tri_lo[((size_t)q * (ld / 3) + t) * 5 + j % 5] : T(0);
    hi_c[c] = on ? a.tri_hi[((size_t)q * (ld / 3) + t) * 5 + j % 5] : T(0);
    mu_c[c] = on ? a.tri_mu[(size_t)q * (ld / 3) + t] : T(0);
    // cold start (warm_start = 0): u = 0, slacks clipped at THR0, lam = mu0 / t
    tl[c] = on ? fmax(-lo_c[c], T(THR0)) : T(1);
    tu[c] = on ? fmax(hi_c[c], T(THR0)) : T(1);
    ll[c] = on ? T(S.mu0) / tl[c] : T(0);
    lu[c] = on ? T(S.mu0) / tu[c] : T(0);
  }

  // y_c = C x_r (pyramid rows of each triple)
  auto apply_C = [&](const T (&x)[RPL], T (&y)[CPL]) {
    const int lane = opaque_lane();
#pragma unroll
    for (int r = 0; r < RPL; ++r) s_v[lane + 64 * r] = x[r];
    __syncthreads();
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int j = lane + 64 * c;
      const int t = j / 5;
      T v = T(0);
      if (j < m) v = pyr_row<T>(j % 5, mu_c[c], s_v[3 * t], s_v[3 * t + 1], s_v[3 * t + 2]);
      y[c] = v;
    }
    __syncthreads();
  };
  // x_r = C' w_c
  auto apply_CT = [&](const T (&w)[CPL], T (&x)[RPL]) {
    const int lane = opaque_lane();
#pragma unroll
    for (int c = 0; c < CPL; ++c) s_c[lane + 64 * c] = w[c];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      const int i = lane + 64 * r;
      T v = T(0);
      if (i < n) {
        const int t = i / 3, dd = i % 3;
        const T w0 = s_c[5 * t], w1 = s_c[5 * t + 1], w2 = s_c[5 * t + 2], w3 = s_c[5 * t + 3], w4 = s_c[5 * t + 4];
        v = dd == 0 ? (w1 - w0) : (dd == 1 ? (w3 - w2) : (mu_r[r] * (w0 + w1 + w2 + w3) + w4));
      }
      x[r] = v;
    }
    __syncthreads();
  };

  T K[RPL][NMAX];
  T invL[RPL], dg[RPL];

  // (L L') x = b with the in-place factor in K (see header comment)
  auto chol_solve = [&](const T (&b)[RPL], T (&x)[RPL]) {
    T y[RPL];
#pragma unroll
    for (int r = 0; r < RPL; ++r) y[r] = b[r];
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
    // U~ x = D y, U~_ik = L_ii L_ki (k > i), U~_ii = L_ii^2, D = diag(L_ii)
#pragma unroll
    for (int r = 0; r < RPL; ++r) y[r] = y[r] * (dg[r] * invL[r]);
    const int laneb = opaque_lane();
#pragma unroll
    for (int k = NMAX - 1; k >= 0; --k) {
      const int rk = k / 64, lk = k % 64;
      const int lane = laneb;
      const T sv = readlane(y[rk] * (invL[rk] * invL[rk]), lk);
#pragma unroll
      for (int r = 0; r < RPL; ++r) {
        const int i = lane + 64 * r;
        y[r] = (i == k) ? sv : ((i < k) ? fma(-K[r][k], sv, y[r]) : y[r]);
      }
    }
#pragma unroll
    for (int r = 0; r < RPL; ++r) x[r] = y[r];
  };

  const T* Hq = a.H + (size_t)q * ld * ld;  // class-packed NMAX x NMAX block at the start of the QP's slab
  int status = CMPC_MAX_ITER;
  int it = 0;
  T rg[RPL], rl[CPL], ru[CPL], itl[CPL], itu[CPL];
  T du[RPL], dtl[CPL], dtu[CPL], dll[CPL], dlu[CPL], rml[CPL], rmu[CPL];

  auto direction = [&]() {
    T wv[CPL], ctw[RPL], rhs[RPL], cdu[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) wv[c] = (rml[c] + ll[c] * rl[c]) * itl[c] - (rmu[c] + lu[c] * ru[c]) * itu[c];
    apply_CT(wv, ctw);
#pragma unroll
    for (int r = 0; r < RPL; ++r) rhs[r] = -rg[r] - ctw[r];
    chol_solve(rhs, du);
    apply_C(du, cdu);
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      dtl[c] = cdu[c] + rl[c];
      dtu[c] = ru[c] - cdu[c];
      dll[c] = -(rml[c] + ll[c] * dtl[c]) * itl[c];
      dlu[c] = -(rmu[c] + lu[c] * dtu[c]) * itu[c];
    }
  };
  auto max_step = [&]() -> T {
    T am = T(1e30);
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      if (dtl[c] < T(0)) am = fmin(am, -tl[c] / dtl[c]);
      if (dtu[c] < T(0)) am = fmin(am, -tu[c] / dtu[c]);
      if (dll[c] < T(0)) am = fmin(am, -ll[c] / dll[c]);
      if (dlu[c] < T(0)) am = fmin(am, -lu[c] / dlu[c]);
    }
    return wave_min(am);
  };

  for (it = 0;; ++it) {
    // Opaque copy of the lane id: keeps the lane-vs-index masks and row addresses from being hoisted out of the
    // iteration loop (LICM would otherwise pin ~200 loop-invariant 64-bit masks in SGPRs and spill them).
    lane = opaque_lane();
    // ---- stream H (class-packed, stride NMAX; symmetric: element (j, i) == (i, j); coalesced 8-B lanes)
    {
      const T* hp = Hq + lane;
#pragma unroll
      for (int j = 0; j < NMAX; ++j)
#pragma unroll
        for (int r = 0; r < RPL; ++r) K[r][j] = hp[j * NMAX + 64 * r];
    }

    // ---- residuals
    T cu[CPL], hu[RPL], ctw[RPL], wv[CPL];
    apply_C(u_r, cu);
#pragma unroll
    for (int r = 0; r < RPL; ++r) s_v[lane + 64 * r] = u_r[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RPL; ++r) hu[r] = T(0);
#pragma unroll
    for (int j = 0; j < NMAX; ++j) {
      const T uj = s_v[j];
#pragma unroll
      for (int r = 0; r < RPL; ++r) hu[r] = fma(K[r][j], uj, hu[r]);
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < CPL; ++c) wv[c] = ll[c] - lu[c];
    apply_CT(wv, ctw);
    T rs = T(0), ri = T(0), rc = T(0), ms = T(0);
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      rg[r] = hu[r] + g_r[r] - ctw[r];
      rs = fmax(rs, fabs(rg[r]));
    }
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const bool on = lane + 64 * c < m;
      rl[c] = on ? cu[c] - lo_c[c] - tl[c] : T(0);
      ru[c] = on ? hi_c[c] - cu[c] - tu[c] : T(0);
      ri = fmax(ri, fmax(fabs(rl[c]), fabs(ru[c])));
      const T cl = tl[c] * ll[c], ch = tu[c] * lu[c];
      rc = fmax(rc, fmax(cl, ch));
      ms += cl + ch;
    }
    rs = wave_max(rs);
    ri = wave_max(ri);
    rc = wave_max(rc);
    ms = wave_sum(ms);
    const T mu = m > 0 ? ms / T(2 * m) : T(0);
    if (uniform_flag<T>(!(isfinite(rs) && isfinite(ri) && isfinite(rc)))) {
      status = CMPC_NAN_SOL;
      break;
    }
    if (uniform_flag<T>(rs <= T(S.tol_stat) && ri <= T(S.tol_ineq) && rc <= T(S.tol_comp))) {
      status = CMPC_SUCCESS;
      break;
    }
    if (it >= S.iter_max) {
      status = CMPC_MAX_ITER;
      break;
    }

    // ---- Newton matrix K = H + C' diag(lam_l/t_l + lam_u/t_u) C + reg I  (3x3 blocks on the triple diagonal)
    T sg[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const bool on = lane + 64 * c < m;
      itl[c] = on ? recip(tl[c]) : T(0);
      itu[c] = on ? recip(tu[c]) : T(0);
      sg[c] = ll[c] * itl[c] + lu[c] * itu[c];
      s_c[lane + 64 * c] = sg[c];
    }
    __syncthreads();
    T bk[RPL][3];
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      const int i = lane + 64 * r;
      bk[r][0] = bk[r][1] = bk[r][2] = T(0);
      if (i < n) {
        const int t = i / 3, dd = i % 3;
        const T s0 = s_c[5 * t], s1 = s_c[5 * t + 1], s2 = s_c[5 * t + 2], s3 = s_c[5 * t + 3],
                s4 = s_c[5 * t + 4];
        const T mu_t = mu_r[r];
        const T xx = s0 + s1, yy = s2 + s3, zz = mu_t * mu_t * (s0 + s1 + s2 + s3) + s4;
        const T xz = mu_t * (s1 - s0), yz = mu_t * (s3 - s2);
        bk[r][0] = dd == 0 ? xx : (dd == 1 ? T(0) : xz);
        bk[r][1] = dd == 0 ? T(0) : (dd == 1 ? yy : yz);
        bk[r][2] = dd == 0 ? xz : (dd == 1 ? yz : zz);
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      const int i = lane + 64 * r;
      const int ti = i / 3;
      const int dd = i % 3;
      const T reg = T(S.reg_prim);
#pragma unroll
      for (int J = 0; J < NTRI; ++J) {
        const bool mine = (ti == J);
#pragma unroll
        for (int cc = 0; cc < 3; ++cc) {
          const T add = bk[r][cc] + (dd == cc ? reg : T(0));
          K[r][3 * J + cc] += mine ? add : T(0);
        }
      }
    }

    // ---- right-looking Cholesky, in place, both triangles kept (see header)
    bool ok = true;
#pragma unroll
    for (int r = 0; r < RPL; ++r) invL[r] = dg[r] = T(1);
    const int lanef = opaque_lane();
#pragma unroll
    for (int s = 0; s < NMAX; ++s) {
      const int lane = lanef;
      const int rs_ = s / 64, ls = s % 64;
      const T d = readlane(K[rs_][s], ls);
      ok = ok && !(d != d);  // NaN pivot -> NAN_SOL
      // BLASFEO-style guard: a pivot lost to cancellation (possible in fp32 late in the IPM) drops its direction
      // (inverse 0) instead of failing; mirrored in oracle_qp_ipm.
      const T il = d > T(PIVOT_MIN<T>::v) ? rsqrt_acc(d) : T(0);
      T bsc[RPL];
#pragma unroll
      for (int r = 0; r < RPL; ++r) {
        const int i = lane + 64 * r;
        if (r == rs_) {
          const bool piv = lane == ls;
          invL[r] = piv ? il : invL[r];
          dg[r] = piv ? d : dg[r];
          asm volatile("" : "+v"(invL[r]), "+v"(dg[r]));
        }
        const bool below = i > s;
        bsc[r] = below ? K[r][s] * il : T(0);
        K[r][s] = below ? bsc[r] : K[r][s];
        asm volatile("" : "+v"(K[r][s]));  // materialise the select here: do not keep the mask alive into the solves
        s_col[i] = bsc[r];
      }
      __syncthreads();
#pragma unroll
      for (int j = s + 1; j < NMAX; ++j) {
        const T lj = s_col[j];
#pragma unroll
        for (int r = 0; r < RPL; ++r) K[r][j] = fma(-bsc[r], lj, K[r][j]);
      }
      __syncthreads();
    }
    if (uniform_flag<T>(!ok)) {
      status = CMPC_NAN_SOL;
      break;
    }

    // ---- predictor (affine scaling direction)
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      rml[c] = tl[c] * ll[c];
      rmu[c] = tu[c] * lu[c];
    }
    direction();
    T alpha = fmin(T(1), max_step());
    if (m > 0) {
      T maff = T(0);
#pragma unroll
      for (int c = 0; c < CPL; ++c)
        maff += (tl[c] + alpha * dtl[c]) * (ll[c] + alpha * dll[c]) + (tu[c] + alpha * dtu[c]) * (lu[c] + alpha * dlu[c]);
      maff = wave_sum(maff) / T(2 * m);
      const T ratio = maff / mu;
      const T sigma = ratio * ratio * ratio;
      // ---- corrector
#pragma unroll
      for (int c = 0; c < CPL; ++c) {
        const bool on = lane + 64 * c < m;
        rml[c] = on ? tl[c] * ll[c] + dtl[c] * dll[c] - sigma * mu : T(0);
        rmu[c] = on ? tu[c] * lu[c] + dtu[c] * dlu[c] - sigma * mu : T(0);
      }
      direction();
      alpha = fmin(T(1), T(TAU) * max_step());
    }
    if (uniform_flag<T>(alpha < T(S.alpha_min))) {
      status = CMPC_MIN_STEP;
      break;
    }
#pragma unroll
    for (int r = 0; r < RPL; ++r) u_r[r] = fma(alpha, du[r], u_r[r]);
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      tl[c] = fma(alpha, dtl[c], tl[c]);
      tu[c] = fma(alpha, dtu[c], tu[c]);
      ll[c] = fma(alpha, dll[c], ll[c]);
      lu[c] = fma(alpha, dlu[c], lu[c]);
    }
  }

  bool fin = true;
#pragma unroll
  for (int r = 0; r < RPL; ++r) {
    const int i = lane + 64 * r;
    fin = fin && isfinite(u_r[r]);
    if (i < ld) a.u[(size_t)q * ld + i] = i < n ? u_r[r] : T(0);
  }
  if (uniform_flag<T>(__any(!fin))) status = CMPC_NAN_SOL;
  if (lane == 0) {
    a.status[q] = status;
    a.iters[q] = it;
  }
}

}  // namespace cmpc
