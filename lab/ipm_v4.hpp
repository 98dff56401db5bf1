#pragma once
// ipm_v4.hpp — lab variant (v3 + lane masks hoisted as SGPR constants, 1 Newton step on the pivot reciprocal;
// was v3: v2 + factor rows pre-scaled by 1/d_i so each sweep step is readlane + FMA;
// was v2: v1 + pipelined factorisation step: next row prefetched, fast pivot reciprocal pinned early,
// partial row exec-masked; stamps: 0 H+resid, 1 newton, 2 LDL', 3 transpose, 4 sweeps, 5 pred other, 6 corr other, 7 upd)
// was: ipm_v1.hpp — lab variant of the batched IPM (n <= 64 class), re-laid out for CDNA4:
//   * Newton matrix K in a 2D-cyclic 4 x 16 register layout: lane l = 16a + b holds K[a + 4r][b + 16c]
//     (r = 0..15, c = 0..3), so a rank-1 update needs only 4 broadcast values per lane from LDS (the row),
//     the other 16 come through DPP row_newbcast inside the 16-lane row;
//   * LDL' right-looking factorisation (no square roots), one-step look-ahead: row s+1 is updated first, written
//     to LDS and its pivot read before the bulk of step s, so the LDS round trip overlaps the FMAs;
//   * the factor is transposed once through LDS into row layout (lane i = row i) for the four triangular sweeps,
//     which save each finished unknown to LDS instead of masking every step;
//   * constraint state lives in registers (tl, tu, lam, directions) and lane-private LDS slots.
// H is read in the 2D order: H2[(r*4 + c)*64 + lane] (prepared by the lab's prep kernel).
#include "cmpc_device.hpp"
#include "cmpc_kernels.hpp"
#include "lab_stamps.hpp"
#include "dpp_rows.hpp"

#include <type_traits>

namespace {
using namespace cmpc;

template <typename T>
struct PMIN1;
template <>
struct PMIN1<double> {
  static constexpr double v = 1e-200;
};
template <>
struct PMIN1<float> {
  static constexpr float v = 1e-30f;
};
template <typename T>
struct MUMIN1;
template <>
struct MUMIN1<double> {
  static constexpr double v = 1e-300;
};
template <>
struct MUMIN1<float> {
  static constexpr float v = 1e-35f;
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
__device__ __forceinline__ void cbar() { asm volatile("" ::: "memory"); }
// lane id the compiler cannot CSE or hoist out of the iteration loop (keeps lane-derived masks and LDS addresses
// from piling up as loop invariants across the unrolled factorisation)
__device__ __forceinline__ int olane() {
  int l = (int)threadIdx.x;
  asm volatile("" : "+v"(l));
  return l;
}
__device__ __forceinline__ bool uflag(bool b) { return __builtin_amdgcn_readfirstlane((int)b) != 0; }

template <int LN>
__device__ __forceinline__ double bcast16(double x) {
  return __builtin_amdgcn_update_dpp(x, x, 0x150 + LN, 0xf, 0xf, true);
}
template <int LN>
__device__ __forceinline__ float bcast16(float x) {
  return __builtin_amdgcn_update_dpp(x, x, 0x150 + LN, 0xf, 0xf, true);
}

template <typename T>
struct Lds1 {
  T v[64];           // v-form broadcast
  T w[128];          // constraint-vector broadcast
  T rowbuf[2][64];   // factorisation: row s of K, [c*16 + b]
  T dg[64];          // pivots d_s
  T z[64];           // sweep results
  T blk[3][64];      // Newton 3x3 block rows
  T rl[128], ru[128], itl[128], itu[128], rml[128], rmu[128];  // lane-private constraint slots
  T scr[1024];       // Hu partials / factor transpose
};

// row-layout column k of lane i's row after the transpose, stored in the register the 2D layout used
__host__ __device__ constexpr int RIDX(int j) { return (j & 15) * 4 + (j >> 4); }

template <typename T, int NMAX, int WPE>
__global__ __launch_bounds__(64, WPE) void k_ipm_reg(IpmArgs<T> A, unsigned long long* stamps) {
  static_assert(NMAX == 64, "2D layout kernel serves the n <= 64 class");
  STAMP_DECL;
  const int q = blockIdx.x;
  if (A.status[q] != CMPC_SUCCESS) return;
  const int n = A.nvar[q];
  if (n > 64) return;
  const int ld = A.ld;
  const int nt = n / 3;
  const int m = 5 * nt;
  const DevSettings S = A.s;
  __shared__ Lds1<T> L;
  int lane = (int)threadIdx.x;  // re-read opaquely at the top of every iteration (see olane)
  const int lane0 = (int)threadIdx.x;  // plain lane id: only for lane masks (hoisted into SGPR pairs)

  // ---- v-form (lane i = variable i)
  const bool vin = lane < n;
  const T g_v = vin ? A.g[(size_t)q * ld + lane] : T(0);
  const T mu_v = vin ? A.tri_mu[(size_t)q * (ld / 3) + lane / 3] : T(0);
  T u_v = T(0);
  // ---- constraint slots j = lane + 64 cc
  T tl[2], tu[2], ll[2], lu[2], lo[2], hi[2], muc[2];
#pragma unroll
  for (int cc = 0; cc < 2; ++cc) {
    const int j = lane + 64 * cc;
    const bool on = j < m;
    const int t = j / 5;
    lo[cc] = on ? A.tri_lo[((size_t)q * (ld / 3) + t) * 5 + j % 5] : T(0);
    hi[cc] = on ? A.tri_hi[((size_t)q * (ld / 3) + t) * 5 + j % 5] : T(0);
    muc[cc] = on ? A.tri_mu[(size_t)q * (ld / 3) + t] : T(0);
    tl[cc] = on ? fmax(-lo[cc], T(THR0)) : T(1);
    tu[cc] = on ? fmax(hi[cc], T(THR0)) : T(1);
    ll[cc] = on ? T(S.mu0) / tl[cc] : T(0);
    lu[cc] = on ? T(S.mu0) / tu[cc] : T(0);
  }

  // C x (x in v-form), x already in L.v
  auto apply_C_v = [&](T (&out)[2]) {
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int j = lane + 64 * cc;
      const int t = j / 5;
      T v = T(0);
      if (j < m) v = pyr_row<T>(j % 5, muc[cc], L.v[3 * t], L.v[3 * t + 1], L.v[3 * t + 2]);
      out[cc] = v;
    }
  };
  // C' w -> v-form
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

  T K[64];
  T invd_v = T(1);
  T rg_v = T(0), du_v = T(0);
  T dtl[2], dtu[2], dll[2], dlu[2];

  // LDL' solve with the row-layout factor (K[RIDX(k)] = K[lane][k]); y: v-form rhs -> solution
  // LDL' solve with the row-scaled row-layout factor K'[i][k] = K[i][k] / d_i (K[RIDX(k)] = K'[lane][k]):
  //   forward  w = D^-1 rhs; z_k = w_k; w_i -= K'[i][k] z_k          (= D^-1 L^-1 rhs)
  //   backward v = z;        x_k = v_k; v_i -= K'[i][k] x_k (i < k)  (= L^-T z)
  // lanes past their own step receive garbage updates; their result was saved to LDS at that step.
  auto solve = [&](T& y) {
#ifndef LAB_NO_SOLVE
    T w = y * invd_v;
    sfor<0, 64>([&](auto k_) {
      constexpr int k = decltype(k_)::value;
      const T zk = readlane(w, k);
      L.z[k] = zk;
      w = fma(-K[RIDX(k)], zk, w);
    });
    cbar();
    w = L.z[lane];
    cbar();
    sfor_down<0, 64>([&](auto k_) {
      constexpr int k = decltype(k_)::value;
      const T xk = readlane(w, k);
      L.z[k] = xk;
      w = fma(-K[RIDX(k)], xk, w);
    });
    cbar();
    y = L.z[lane];
    cbar();
#endif
  };

  auto direction = [&](auto pc_) {
    constexpr int pc = decltype(pc_)::value;
    (void)pc;
    T wv[2];
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int j = lane + 64 * cc;
      wv[cc] = (L.rml[j] + ll[cc] * L.rl[j]) * L.itl[j] - (L.rmu[j] + lu[cc] * L.ru[j]) * L.itu[j];
    }
    const T ctw = apply_CT(wv);
    du_v = -rg_v - ctw;
    STAMP(pc);
    solve(du_v);
    STAMP(4);
    L.v[lane] = du_v;
    cbar();
    T cdu[2];
    apply_C_v(cdu);
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
  auto max_step = [&]() -> T {
    T am = T(1e30);
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      if (dtl[cc] < T(0)) am = fmin(am, -tl[cc] / dtl[cc]);
      if (dtu[cc] < T(0)) am = fmin(am, -tu[cc] / dtu[cc]);
      if (dll[cc] < T(0)) am = fmin(am, -ll[cc] / dll[cc]);
      if (dlu[cc] < T(0)) am = fmin(am, -lu[cc] / dlu[cc]);
    }
    return wave_min(am);
  };

  const T* Hq = A.H + (size_t)q * ld * ld;
  int status = CMPC_MAX_ITER;
  int it = 0;
  for (it = 0;; ++it) {
    lane = olane();
    const int la = lane >> 4, lb = lane & 15;
    // ---- H in 2D order (coalesced 512-B rows)
#pragma unroll
    for (int e = 0; e < 64; ++e) K[e] = Hq[e * 64 + lane];

    // ---- residuals: Hu through the 2D layout, partial sums reduced via LDS
    T hu = T(0);
    {
    const int lane = olane();
    const int la = lane >> 4, lb = lane & 15;
    L.v[lane] = u_v;
    cbar();
    T uc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) uc[c] = L.v[lb + 16 * c];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      T p = K[r * 4] * uc[0];
      p = fma(K[r * 4 + 1], uc[1], p);
      p = fma(K[r * 4 + 2], uc[2], p);
      p = fma(K[r * 4 + 3], uc[3], p);
      const int i = la + 4 * r;
      L.scr[i * 16 + ((((lb >> 1) + i) & 7) << 1) + (lb & 1)] = p;
    }
    cbar();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int idx = lane * 16 + (((k + lane) & 7) << 1);
      hu += L.scr[idx] + L.scr[idx + 1];
    }
    cbar();
    }
    T cu[2];
    apply_C_v(cu);  // L.v still holds u
    cbar();
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
    {
      T wv[2] = {ll[0] - lu[0], ll[1] - lu[1]};
      const T ctw = apply_CT(wv);
      rg_v = vin ? hu + g_v - ctw : T(0);
      rs = fabs(rg_v);
    }
    rs = wave_max(rs);
    ri = wave_max(ri);
    rc = wave_max(rc);
    ms = wave_sum(ms);
    const T mu = m > 0 ? ms / T(2 * m) : T(0);
    if (uflag(!(isfinite(rs) && isfinite(ri) && isfinite(rc)))) {
      status = CMPC_NAN_SOL;
      break;
    }
    if (uflag(rs <= T(S.tol_stat) && ri <= T(S.tol_ineq) && rc <= T(S.tol_comp))) {
      status = CMPC_SUCCESS;
      break;
    }
    if (it >= S.iter_max) {
      status = CMPC_MAX_ITER;
      break;
    }
    if (uflag(m > 0 && !(mu > T(MUMIN1<T>::v)))) {
      status = CMPC_MIN_STEP;
      break;
    }
    STAMP(0);

    // ---- Newton matrix K = H + C' diag(lam_l/t_l + lam_u/t_u) C + reg I
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
    // 2D add: entry (i, j) of lane (a, b) column c gets blk[i - 3(j/3)][j] when i is in j's triple
    sfor<0, 4>([&](auto c_) {
      const int ol = olane();
      const int la = ol >> 4, lb = ol & 15;
      constexpr int c = decltype(c_)::value;
      constexpr int imin = 3 * ((16 * c) / 3);
      constexpr int imax0 = 3 * ((16 * c + 15) / 3) + 2;
      constexpr int imax = imax0 > 63 ? 63 : imax0;
      constexpr int rlo = imin >= 3 ? (imin - 3 + 3) / 4 : 0;
      constexpr int rhi = imax / 4;
      const int j = lb + 16 * c;
      const int t3 = 3 * (j / 3);
      const int e = (la - t3) & 3;              // i = t3 + e has i % 4 == a
      const int rstar = e <= 2 ? (t3 + e - la) >> 2 : -1;
      const T val = L.blk[e <= 2 ? e : 0][j];
      sfor<rlo, rhi + 1>([&](auto r_) {
        constexpr int r = decltype(r_)::value;
        K[r * 4 + c] += (rstar == r) ? val : T(0);
      });
    });
    cbar();
    STAMP(1);

    // ---- LDL' factorisation (2D layout). Step s: look-ahead row r1 (holds row s+1) first, row s+1 to LDS and
    //      prefetched back, pivot s+1 and its reciprocal, then the bulk rows r1+1..15, then step s+1's multipliers.
    auto rcp_guard = [](T p) -> T {
      T y = __builtin_amdgcn_rcp(p);
      const T e = fma(-p, y, T(1));
      y = fma(y, e, y);
      return p > T(PMIN1<T>::v) ? y : T(0);
    };
    T piv = readlane(K[0], 0);
    T invd = rcp_guard(piv);
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
        mm[c] = c == 0 ? (lb > 0 ? mv : T(0)) : mv;
      }
      cbar();
    }
#ifndef LAB_NO_CHOL
    sfor<0, 63>([&](auto s_) {
      constexpr int s = decltype(s_)::value;
      constexpr int c0 = s / 16, b0 = s % 16, a0 = s % 4;
      constexpr int s1 = s + 1;
      constexpr int r1 = s1 / 4, a1 = s1 % 4, c1 = s1 / 16, b1 = s1 % 16;
      __builtin_amdgcn_sched_barrier(0);
      const int ol = olane();
      const int lb = ol & 15;
      const int la_m = lane0 >> 4, lb_m = lane0 & 15;  // masks: hoistable SGPR constants
      // look-ahead row r1: rows a + 4 r1; when a0 < 3 it is the partial row (rows > s only for a > a0)
      if constexpr (a0 < 3) {
        if (la_m > a0) dpp_row<b0, c0, true, T>(K[r1 * 4], K[r1 * 4 + 1], K[r1 * 4 + 2], K[r1 * 4 + 3], mm[0], mm[1], mm[2], mm[3]);
      } else {
        dpp_row<b0, c0, true, T>(K[r1 * 4], K[r1 * 4 + 1], K[r1 * 4 + 2], K[r1 * 4 + 3], mm[0], mm[1], mm[2], mm[3]);
      }
      cbar();
      if (la_m == a1) {
#pragma unroll
        for (int c = c1; c < 4; ++c) L.rowbuf[s1 & 1][c * 16 + lb] = K[r1 * 4 + c];
      }
      cbar();
      T xn[4];
#pragma unroll
      for (int c = c1; c < 4; ++c) xn[c] = L.rowbuf[s1 & 1][c * 16 + lb];
      cbar();
      const T pivn = readlane(K[r1 * 4 + c1], a1 * 16 + b1);
      T invdn = rcp_guard(pivn);
      asm volatile("" : "+v"(invdn));  // materialise the reciprocal here, before the bulk rows
      sfor<r1 + 1, 16>([&](auto r_) {
        constexpr int r = decltype(r_)::value;
        if constexpr (((r - r1 - 1) & 3) == 0) __builtin_amdgcn_sched_barrier(0);
        dpp_row<b0, c0, false, T>(K[r * 4], K[r * 4 + 1], K[r * 4 + 2], K[r * 4 + 3], mm[0], mm[1], mm[2], mm[3]);
      });
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int c = c1; c < 4; ++c) {
        const T mv = -(xn[c] * invdn);
        mm[c] = c == c1 ? (lb_m > b1 ? mv : T(0)) : mv;
      }
      L.dg[s1] = pivn;
    });
#endif
    __builtin_amdgcn_sched_barrier(0);
    cbar();
    STAMP(2);

    // ---- pivots -> 1/d (same reciprocal as the factorisation), NaN pivot -> NAN_SOL
    {
      const T d = L.dg[lane];
      T y = __builtin_amdgcn_rcp(d);
      const T e = fma(-d, y, T(1));
      y = fma(y, e, y);
      invd_v = d > T(PMIN1<T>::v) ? y : T(0);
      if (uflag(__any(d != d))) {
        status = CMPC_NAN_SOL;
        break;
      }
    }
    // ---- transpose the factor into row layout (lane i = row i), through LDS 16 columns at a time, scaling
    //      row i by 1/d_i on the way
    sfor<0, 4>([&](auto c_) {
      const int lane = olane();
      const int la = lane >> 4, lb = lane & 15;
      constexpr int c = decltype(c_)::value;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = la + 4 * r;
        L.scr[i * 16 + ((((lb >> 1) + i) & 7) << 1) + (lb & 1)] = K[r * 4 + c];
      }
      cbar();
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int idx = lane * 16 + (((k + lane) & 7) << 1);
        K[RIDX(16 * c + 2 * k)] = L.scr[idx] * invd_v;
        K[RIDX(16 * c + 2 * k + 1)] = L.scr[idx + 1] * invd_v;
      }
      cbar();
    });
    STAMP(3);

    // ---- predictor (affine scaling direction)
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int j = lane + 64 * cc;
      L.rml[j] = tl[cc] * ll[cc];
      L.rmu[j] = tu[cc] * lu[cc];
    }
    direction(std::integral_constant<int, 5>{});
    T alpha = fmin(T(1), max_step());
    if (m > 0) {
      T maff = T(0);
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        const int j = lane + 64 * cc;
        const bool on = j < m;
        const T v = (tl[cc] + alpha * dtl[cc]) * (ll[cc] + alpha * dll[cc]) +
                    (tu[cc] + alpha * dtu[cc]) * (lu[cc] + alpha * dlu[cc]);
        maff += on ? v : T(0);
      }
      maff = wave_sum(maff) / T(2 * m);
      const T ratio = maff / mu;
      const T sigma = ratio * ratio * ratio;
      STAMP(5);
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        const int j = lane + 64 * cc;
        const bool on = j < m;
        L.rml[j] = on ? tl[cc] * ll[cc] + dtl[cc] * dll[cc] - sigma * mu : T(0);
        L.rmu[j] = on ? tu[cc] * lu[cc] + dtu[cc] * dlu[cc] - sigma * mu : T(0);
      }
      direction(std::integral_constant<int, 6>{});
      alpha = fmin(T(1), T(TAU) * max_step());
    }
    STAMP(6);
    if (uflag(alpha < T(S.alpha_min))) {
      status = CMPC_MIN_STEP;
      break;
    }
    u_v = fma(alpha, du_v, u_v);
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      tl[cc] = fma(alpha, dtl[cc], tl[cc]);
      tu[cc] = fma(alpha, dtu[cc], tu[cc]);
      ll[cc] = fma(alpha, dll[cc], ll[cc]);
      lu[cc] = fma(alpha, dlu[cc], lu[cc]);
    }
    STAMP(7);
  }

  lane = olane();
  const bool fin = isfinite(u_v);
  if (lane < ld) A.u[(size_t)q * ld + lane] = vin ? u_v : T(0);
  if (uflag(__any(!fin))) status = CMPC_NAN_SOL;
  if (lane == 0) {
    A.status[q] = status;
    A.iters[q] = it;
  }
  STAMP_STORE(stamps, q);
}

// lab prep: class-packed row-major 64 x 64 H -> 2D order H2[(r*4 + c)*64 + lane] (in a separate buffer)
template <typename T>
__global__ void k_prep2d(const T* H, T* H2, const int* nvar, int ld) {
  const int q = blockIdx.x;
  const int lane = threadIdx.x;
  const int la = lane >> 4, lb = lane & 15;
  if (nvar[q] > 64) return;
  const T* hq = H + (size_t)q * ld * ld;
  T* oq = H2 + (size_t)q * ld * ld;
  for (int r = 0; r < 16; ++r)
    for (int c = 0; c < 4; ++c) oq[(r * 4 + c) * 64 + lane] = hq[(la + 4 * r) * 64 + lb + 16 * c];
}

}  // namespace
