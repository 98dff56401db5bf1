#pragma once
// k_ipm72.hpp — the 64 < n <= 72 size class on one wavefront: the subproblems of the NLP with footholds as decision
// variables on a trot horizon of N = 10 (cmpc_nlp_solve_batch: 60 forces and two to four foothold triples, n = 66 or
// 72), which the four-wave 128 class would otherwise serve at a quarter of the QPs per CU. The IPM is k_ipm64's (the
// iteration of oracle/cmpc_oracle.c:oracle_qp_ipm, HPIPM's stopping rule and settings), on the bordered Newton system
//     [K_AA  K_AB] [x_A]   [r_A]      A = variables 0..63: k_ipm64's 4 x 16-cyclic register tile and elimination
//     [K_AB' K_BB] [x_B] = [r_B]      B = variables 64..n-1, nb = n - 64 <= NB = 8: LDS
// solved through the Schur complement:
//   * K_AA is eliminated in the tile exactly as in k_ipm64 (LDL' with L^-1 in place, DPP row updates, look-ahead),
//     so K_AA^-1 = M' D^-1 M with M unit triangular;
//   * Y = M K_AB by nb forward half-solves (in place of K_AB) and S = K_BB - K_AB' K_AA^-1 K_AB = K_BB - Y' D^-1 Y (by
//     symmetry only k >= l): W = K_AA^-1 K_AB is never formed, which saves nb backward half-solves per iteration;
//   * S^-1 by Gauss-Jordan across the wave: lane 8k + l holds S[k][l], identity-padded to 8 x 8 (S is SPD as a Schur
//     complement of the SPD K: no pivoting);
//   * per right-hand side: z = D^-1 M r_A, x_B = S^-1 (r_B - Y' z), x_A = M' (z - D^-1 Y x_B) (one tile solve, split).
// Border variables live in a second per-lane slot (lane k carries variable 64 + k) next to k_ipm64's lane-per-variable
// slot. H comes from the class-128 block of the workspace (row-major, stride 128) the workgroup condensing wrote. The
// LDS stays under 20 KB, so 8 waves fit a CU as for k_ipm64: rowbuf and z share bytes, and the tile solve reduces its
// row partials in two halves through a 4 KB scratch (k_ipm64's 8 KB would leave 6 waves per CU).
// The iterates agree with the oracle's (Cholesky of the whole K) to rounding; statuses and iteration counts are
// checked against it (tests/test_ipm72.py).
#include "k_ipm64.hpp"

namespace cmpc {

// Lab instrumentation (-DCMPC_IPM72_STAMPS, lab/ipm72_stamps.sh only, never in libcmpc.so): per-wave shader-clock
// cycles per phase, summed over every QP into ipm72_stamp_acc (read by cmpc_ipm72_debug_stamps). Phases: 0 H +
// residuals, 1 Newton blocks, 2 LDL' of K_AA, 3 Y = M K_AB, 4 S, 5 S^-1, 6 predictor, 7 corrector, 8 update,
// 9 iterations, 10 total.
#ifdef CMPC_IPM72_STAMPS
__device__ unsigned long long ipm72_stamp_acc[16];
#define I72_DECL                                                  \
  unsigned long long i72_acc_[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}; \
  const unsigned long long i72_t0_ = __builtin_amdgcn_s_memtime();  \
  unsigned long long i72_prev_ = i72_t0_
#define I72(id)                                                   \
  do {                                                            \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    i72_acc_[id] += now_ - i72_prev_;                             \
    i72_prev_ = now_;                                             \
  } while (0)
#define I72_STORE(iters)                                                                  \
  do {                                                                                    \
    i72_acc_[9] = (unsigned long long)(iters);                                            \
    i72_acc_[10] = __builtin_amdgcn_s_memtime() - i72_t0_;                                \
    if (threadIdx.x == 0)                                                                 \
      for (int k_ = 0; k_ < 11; ++k_) atomicAdd(&ipm72_stamp_acc[k_], i72_acc_[k_]);      \
  } while (0)
#else
#define I72_DECL (void)0
#define I72(id) (void)0
#define I72_STORE(iters) (void)0
#endif

namespace ipm72 {

constexpr int NP = 128;  // row stride of the class-128 H block

constexpr int NB = 8;  // border variables at most (n <= 72)
constexpr int RS2 = 33;  // row stride of the half-tile partial sums

template <typename T>
struct Lds72 {
  T v[64 + NB];  // lane-per-variable broadcast
  T w[128];      // pyramid-row broadcast
  union {
    T rowbuf[2][64];     // factorisation: row s of K_AA as [c*16 + b]
    T z[4 * ipm64::ZS];  // tile solve (after the factorisation): z permuted as [i % 4][i / 4], row stride ZS
  };
  T dg[64];           // pivots of K_AA
  T blk[3][64 + NB];  // Newton 3x3 block rows
  T rl[128], ru[128], itl[128], itu[128], rml[128], rmu[128];  // lane-private pyramid-row scratch
  T scr[16 * RS2];    // H u and tile-solve partial sums (half the rows at a time: partial b of row il at b RS2 + il,
                      // RS2 odd, conflict-free as ipm64::RS); result scatter
  T kab[NB][64];      // K_AB columns, then W = K_AA^-1 K_AB
  T sb[NB * NB];      // S, then S^-1 (row-major 8 x 8, identity-padded)
  T hb[NB * NB];      // H_BB (row-major 8 x 8, zero-padded)
  T xb[NB];           // border vector exchange
};

// 16-lane row reduce-scatter: every lane holds p[0..15]; returns, in the lane at row position b = lane & 15, the sum of
// p[b] over the 16 lanes of its DPP row. Four pairwise exchanges whose lane flips (row_mirror 1111, row_half_mirror
// 0111, quad_perm 0010, 0001) are independent over GF(2): each halves the slots a lane keeps (the half whose slot
// bit equals the lane's), 15 adds per lane in place of 16 LDS partials, a barrier and 16 LDS reads.
template <typename T>
__device__ __forceinline__ T row_reduce_scatter16(const T (&p)[16], int b) {
  const bool b3 = (b & 8) != 0, b2 = (b & 4) != 0, b1 = (b & 2) != 0, b0 = (b & 1) != 0;
  T q8[8], q4[4], q2[2];
#pragma unroll
  for (int k = 0; k < 8; ++k) q8[k] = (b3 ? p[8 + k] : p[k]) + wdpp::dpp<0x140>(b3 ? p[k] : p[8 + k]);
#pragma unroll
  for (int k = 0; k < 4; ++k) q4[k] = (b2 ? q8[4 + k] : q8[k]) + wdpp::dpp<0x141>(b2 ? q8[k] : q8[4 + k]);
#pragma unroll
  for (int k = 0; k < 2; ++k) q2[k] = (b1 ? q4[2 + k] : q4[k]) + wdpp::dpp<0x4E>(b1 ? q4[k] : q4[2 + k]);
  return (b0 ? q2[1] : q2[0]) + wdpp::dpp<0xB1>(b0 ? q2[0] : q2[1]);
}

}  // namespace ipm72

template <typename T, int WPE>
__device__ __forceinline__ void ipm72_body(const IpmArgs<T>& A, int q) {
  __shared__ ipm72::Lds72<T> L;
  using namespace ipm64;
  constexpr int NP = ipm72::NP, NB = ipm72::NB;
  T K[64];
  if (A.status[q] != CMPC_SUCCESS) return;
  const int n = A.nvar[q];
  if (n <= 64 || n > 64 + NB) return;  // served by another size class
  const int nb = n - 64;
  const int ld = A.ld;
  const int nt = n / 3;
  const int m = 5 * nt;
  const DevSettings S = A.s;
  int lane = (int)threadIdx.x;         // re-read opaquely at every iteration
  const int lane0 = (int)threadIdx.x;  // plain lane id: lane masks only
  const bool bin = lane0 < nb;         // this lane also carries border variable 64 + lane
  const size_t qg = (size_t)q * ld, qt = (size_t)q * (ld / 3);
  const T* Hq = A.H + (size_t)q * ld * ld;

  // ---- lane-per-variable data: slot A (variable lane, always real: n > 64) and slot B (variable 64 + lane)
  const T g_v = A.g[qg + lane];
  const T g_b = bin ? A.g[qg + 64 + lane] : T(0);
  const T mu_v = A.tri_mu[qt + lane / 3];
  const T mu_b = bin ? A.tri_mu[qt + (64 + lane) / 3] : T(0);
  T u_v = A.warm ? A.u[qg + lane] : T(0);
  T u_b = (A.warm && bin) ? A.u[qg + 64 + lane] : T(0);
  L.v[lane] = u_v;
  if (lane < NB) L.v[64 + lane] = u_b;
  {  // H_BB (fixed for the whole solve), zero-padded to 8 x 8
    const int hk = lane >> 3, hl = lane & 7;
    L.hb[lane] = (hk < nb && hl < nb) ? Hq[(size_t)(64 + hk) * NP + 64 + hl] : T(0);
  }
  cbar();
  // ---- pyramid rows j = lane + 64 cc: slacks of C u clipped at THR0, lam = mu0 / t
  T lo[2], hi[2], muc[2], tl[2], tu[2], ll[2], lu[2];
#pragma unroll
  for (int cc = 0; cc < 2; ++cc) {
    const int j = lane + 64 * cc;
    const bool on = j < m;
    const int t = j / 5;
    lo[cc] = on ? A.tri_lo[(qt + t) * 5 + j % 5] : T(0);
    hi[cc] = on ? A.tri_hi[(qt + t) * 5 + j % 5] : T(0);
    muc[cc] = on ? A.tri_mu[qt + t] : T(0);
    T cu0 = T(0);
    if (A.warm && on) cu0 = pyr_row<T>(j % 5, muc[cc], L.v[3 * t], L.v[3 * t + 1], L.v[3 * t + 2]);
    tl[cc] = on ? fmax(cu0 - lo[cc], T(THR0)) : T(1);
    tu[cc] = on ? fmax(hi[cc] - cu0, T(THR0)) : T(1);
    ll[cc] = on ? T(S.mu0) / tl[cc] : T(0);
    lu[cc] = on ? T(S.mu0) / tu[cc] : T(0);
  }
  cbar();

  // C x for the lane's two pyramid rows, x (variables 0..n-1) already in L.v
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
  // C' w for variable lane (returned) and variable 64 + lane (vb, border lanes)
  auto apply_CT = [&](const T (&wv)[2], T& vb) -> T {
    L.w[lane] = wv[0];
    L.w[lane + 64] = wv[1];
    cbar();
    auto ct = [&](int var, T muv) -> T {
      const int t = var / 3, dd = var % 3;
      const T w0 = L.w[5 * t], w1 = L.w[5 * t + 1], w2 = L.w[5 * t + 2], w3 = L.w[5 * t + 3], w4 = L.w[5 * t + 4];
      return dd == 0 ? (w1 - w0) : (dd == 1 ? (w3 - w2) : (muv * (w0 + w1 + w2 + w3) + w4));
    };
    const T v = ct(lane, mu_v);
    vb = bin ? ct(64 + lane, mu_b) : T(0);
    cbar();
    return v;
  };

  T invd_v = T(1);
  T hu_v = T(0), rhs_v = T(0), rg_v = T(0), du_v = T(0);
  T hu_b = T(0), rhs_b = T(0), rg_b = T(0), du_b = T(0);
  T dtl[2], dtu[2], dll[2], dlu[2];

  // K_AA^-1 = M' D^-1 M with the eliminated tile (k_ipm64's solve over the 40 lower registers), in two halves:
  // fwd(y) = M y, bwd(z) = M' z
  auto fwd = [&](T y) -> T {
    const int ol = olane();
    const int ola = ol >> 4, olb = ol & 15;
    L.v[ol] = y * invd_v;
    cbar();
    T tc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) tc[c] = L.v[olb + 16 * c];
    // row partials of the 4 x 16-cyclic tile, reduced across each 16-lane row (ipm72::row_reduce_scatter16)
    T pr[16];
    sfor<0, 16>([&](auto r_) {
      constexpr int r = decltype(r_)::value;
      T acc = K[r * 4] * tc[0];
      sfor<1, r / 4 + 1>([&](auto c_) {
        constexpr int c = decltype(c_)::value;
        acc = fma(K[r * 4 + c], tc[c], acc);
      });
      pr[r] = acc;
    });
    L.scr[ola + 4 * olb] = ipm72::row_reduce_scatter16(pr, olb);  // row ola + 4 olb
    cbar();
    const T sv = L.scr[ol];
    cbar();
    return y - sv;
  };
  auto bwd = [&](T z) -> T {
    const int ol = olane();
    const int ola = ol >> 4, olb = ol & 15;
    L.z[(ol & 3) * ipm64::ZS + (ol >> 2)] = z;
    cbar();
    T zr[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) zr[r] = L.z[ola * ipm64::ZS + r];
    cbar();
    sfor<0, 4>([&](auto c_) {
      constexpr int c = decltype(c_)::value;
      T qv = K[(4 * c) * 4 + c] * zr[4 * c];
      sfor<4 * c + 1, 16>([&](auto r_) {
        constexpr int r = decltype(r_)::value;
        qv = fma(K[r * 4 + c], zr[r], qv);
      });
      L.scr[ola * 64 + c * 16 + olb] = qv;
    });
    cbar();
    const T qs = (L.scr[ol] + L.scr[64 + ol]) + (L.scr[128 + ol] + L.scr[192 + ol]);
    cbar();
    return fma(-invd_v, qs, z);
  };

  // H_AA into the tile (4 rows x 16 consecutive columns per load) and this lane's row of H_AB into hab (written to
  // L.kab with the Newton blocks, so no wait on the loads sits in front of the residual work)
  T hab[NB];
  auto load_H = [&]() {
    const int ln = olane();
    const T* hr = Hq + (size_t)ln * NP + 64;
#pragma unroll
    for (int k = 0; k < NB; ++k) hab[k] = k < nb ? hr[k] : T(0);
    const T* hp = Hq + (size_t)(ln >> 4) * NP + (ln & 15);
#pragma unroll
    for (int e = 0; e < 64; ++e) K[e] = hp[(e >> 2) * 4 * NP + (e & 3) * 16];
  };

  // Newton direction for the complementarity targets in L.rml / L.rmu (both slots); leaves du in L.v
  auto direction = [&]() {
    T wv[2];
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int j = lane + 64 * cc;
      wv[cc] = (L.rml[j] + ll[cc] * L.rl[j]) * L.itl[j] - (L.rmu[j] + lu[cc] * L.ru[j]) * L.itu[j];
    }
    T ctw_b;
    const T ctw = apply_CT(wv, ctw_b);
    rhs_v = -rg_v - ctw;
    rhs_b = bin ? -rg_b - ctw_b : T(0);
    // z = D^-1 M r_A; t = r_B - W' r_A = r_B - Y' z (lane k), then x_B = S^-1 t
    const T z = fwd(rhs_v) * invd_v;
    T tb = rhs_b;
    sfor<0, NB>([&](auto k_) {  // independent wave sums (zero beyond nb)
      constexpr int k = decltype(k_)::value;
      const T s = wave_sum_dpp((k < nb ? L.kab[k][lane] : T(0)) * z);
      tb = lane0 == k ? tb - s : tb;
    });
    if (lane < NB) L.xb[lane] = bin ? tb : T(0);
    cbar();
    T xk = T(0);
    if (bin)
      for (int l = 0; l < nb; ++l) xk = fma(L.sb[lane * NB + l], L.xb[l], xk);
    du_b = xk;
    cbar();
    if (lane < NB) L.xb[lane] = du_b;
    cbar();
    // x_A = K_AA^-1 (r_A - K_AB x_B) = M' (z - D^-1 Y x_B)
    T yx = T(0);
    for (int k = 0; k < nb; ++k) yx = fma(L.kab[k][lane], L.xb[k], yx);
    du_v = bwd(fma(-invd_v, yx, z));
    L.v[lane] = du_v;
    if (lane < NB) L.v[64 + lane] = du_b;
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
  auto max_step = [&]() -> T {
    MinRatio<T> mr;
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      mr.cand(tl[cc], dtl[cc]);
      mr.cand(tu[cc], dtu[cc]);
      mr.cand(ll[cc], dll[cc]);
      mr.cand(lu[cc], dlu[cc]);
    }
    return wave_min_dpp(mr.value());
  };

  int status = CMPC_MAX_ITER;
  int it = 0;
  I72_DECL;
  for (it = 0;; ++it) {
    progress_prio(it);
    load_H();
    lane = olane();
    const int la = lane >> 4, lb = lane & 15;

    // ---- residuals that do not need H
    L.v[lane] = u_v;
    if (lane < NB) L.v[64 + lane] = u_b;
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
    T ctw, ctw_b;
    {
      const T wv[2] = {ll[0] - lu[0], ll[1] - lu[1]};
      ctw = apply_CT(wv, ctw_b);
    }
    // ---- H u from H at the first iteration (then carried): tile rows + K_AB (raw H_AB in L.kab) + H_BB. Later
    // iterations write H_AB into L.kab only with the Newton blocks, so no wait on its loads sits in the residuals
    if (it == 0) {
#pragma unroll
      for (int k = 0; k < NB; ++k)
        if (k < nb) L.kab[k][lane] = hab[k];
      cbar();
      T hu = T(0);
      T uc[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) uc[c] = L.v[lb + 16 * c];
      const int base = lb * ipm72::RS2 + la;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int r = 8 * h; r < 8 * h + 8; ++r) {
          T p = K[r * 4] * uc[0];
          p = fma(K[r * 4 + 1], uc[1], p);
          p = fma(K[r * 4 + 2], uc[2], p);
          p = fma(K[r * 4 + 3], uc[3], p);
          L.scr[base + 4 * (r - 8 * h)] = p;
        }
        cbar();
        if ((lane >> 5) == h) {
          const int il = lane - 32 * h;
#pragma unroll
          for (int k = 0; k < 16; k += 2) hu += L.scr[k * ipm72::RS2 + il] + L.scr[(k + 1) * ipm72::RS2 + il];
        }
        cbar();
      }
      T hb = T(0);
      for (int k = 0; k < nb; ++k) {
        hu = fma(L.kab[k][lane], L.v[64 + k], hu);
        const T s = wave_sum_dpp(L.kab[k][lane] * u_v);
        hb = lane0 == k ? s : hb;
      }
      if (bin)
        for (int l = 0; l < nb; ++l) hb = fma(L.hb[lane * NB + l], L.v[64 + l], hb);
      hu_v = hu;
      hu_b = bin ? hb : T(0);
    }
    rg_v = hu_v + g_v - ctw;
    rg_b = bin ? hu_b + g_b - ctw_b : T(0);
    rs = fmax(fabs(rg_v), fabs(rg_b));
    if (A.res_scr) {  // this iteration's residual terms, reduced once at the exit
      T* rp = A.res_scr + (size_t)q * 3 * 64 + lane;
      rp[0] = rs;
      rp[64] = ri;
      rp[128] = rc;
    }
    ms = wave_sum_dpp(ms);
    const T mu = m > 0 ? ms / T(2 * m) : T(0);
    const bool st_on = A.stats && it < A.stats_cap;
    auto st_row = [&]() { return A.stats + ((size_t)q * A.stats_cap + it) * CMPC_STAT_COLS; };
    if (st_on) {
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

    I72(0);
    // ---- Newton matrix K = H + C' diag(lam_l/t_l + lam_u/t_u) C + reg I: 3x3 block rows of both slots
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
      const T reg = T(S.reg_prim);
      // column dd of variable var's triple block: entries (t3 + e, var), e = 0..2
      auto blkcol = [&](int var, T muv, T& b0, T& b1, T& b2) {
        const int ti = var / 3, dd = var % 3;
        const T s0 = L.w[5 * ti], s1 = L.w[5 * ti + 1], s2 = L.w[5 * ti + 2], s3 = L.w[5 * ti + 3], s4 = L.w[5 * ti + 4];
        const T xx = s0 + s1, yy = s2 + s3, zz = muv * muv * (s0 + s1 + s2 + s3) + s4;
        const T xz = muv * (s1 - s0), yz = muv * (s3 - s2);
        b0 = (dd == 0 ? xx : (dd == 1 ? T(0) : xz)) + (dd == 0 ? reg : T(0));
        b1 = (dd == 0 ? T(0) : (dd == 1 ? yy : yz)) + (dd == 1 ? reg : T(0));
        b2 = (dd == 0 ? xz : (dd == 1 ? yz : zz)) + (dd == 2 ? reg : T(0));
      };
      T b0, b1, b2;
      blkcol(lane, mu_v, b0, b1, b2);
      L.blk[0][lane] = b0;
      L.blk[1][lane] = b1;
      L.blk[2][lane] = b2;
      if (lane < NB) {
        b0 = b1 = b2 = T(0);
        if (bin) blkcol(64 + lane, mu_b, b0, b1, b2);
        L.blk[0][64 + lane] = b0;
        L.blk[1][64 + lane] = b1;
        L.blk[2][64 + lane] = b2;
      }
    }
    cbar();
    // K_AA: tile lanes add the block entries of their column's triple (as k_ipm64)
    sfor<0, 4>([&](auto c_) {
      constexpr int c = decltype(c_)::value;
      constexpr int imin = 3 * ((16 * c) / 3);
      constexpr int imax0 = 3 * ((16 * c + 15) / 3) + 2;
      constexpr int imax = imax0 > 63 ? 63 : imax0;
      constexpr int rlo = imin / 4;
      constexpr int rhi = imax / 4;
      const int j = lb + 16 * c;
      const int t3 = 3 * (j / 3);
      const int e = (la - t3) & 3;
      const int rstar = e <= 2 ? (t3 + e - la) >> 2 : -1;
      const T val = L.blk[e <= 2 ? e : 0][j];
      sfor<rlo, rhi + 1>([&](auto r_) {
        constexpr int r = decltype(r_)::value;
        K[r * 4 + c] += (rstar == r) ? val : T(0);
      });
    });
    // K_AB: row lane of border column k gets its block entry when both share a triple (only the triple 63..65)
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      const int t3k = 3 * ((64 + k) / 3);
      if (k < nb) L.kab[k][lane] = lane >= t3k ? hab[k] + L.blk[lane - t3k][64 + k] : hab[k];
    }
    {  // K_BB = H_BB + blocks into L.sb (identity-padded)
      const int hk = lane >> 3, hl = lane & 7;
      T s = hk == hl ? T(1) : T(0);
      if (hk < nb && hl < nb) {
        const int vk = 64 + hk, vl = 64 + hl, t3l = 3 * (vl / 3);
        s = L.hb[lane] + ((vk / 3 == vl / 3) ? L.blk[vk - t3l][vl] : T(0));
      }
      L.sb[lane] = s;
    }
    cbar();

    I72(1);
    // ---- LDL' of K_AA in the tile (k_ipm64's elimination; every pivot is real here)
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
      __builtin_amdgcn_sched_barrier(0);
      const int la_m = lane0 >> 4, lb_m = lane0 & 15;
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
      asm volatile("" : "+v"(invdn));
      sfor<r1 + 1, 16>([&](auto r_) {
        constexpr int r = decltype(r_)::value;
        if constexpr (((r - r1 - 1) & 3) == 0) __builtin_amdgcn_sched_barrier(0);
        dpp_rowf<b0, c0, r == 15, T>(K[r * 4], K[r * 4 + 1], K[r * 4 + 2], K[r * 4 + 3], mm[0], mm[1], mm[2], mm[3]);
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
    {
      const T d = L.dg[lane];
      invd_v = pivot_inv(d);
      if (uflag(__any(d != d))) {
        status = CMPC_NAN_SOL;
        break;
      }
    }
    I72(2);
    {  // strict lower part S only in the 16 registers that straddle the diagonal
      const int la_m = lane0 >> 4, lb_m = lane0 & 15;
      sfor<0, 4>([&](auto c_) {
        constexpr int c = decltype(c_)::value;
        sfor<4 * c, 4 * c + 4>([&](auto r_) {
          constexpr int r = decltype(r_)::value;
          K[r * 4 + c] = (lb_m + 16 * c < la_m + 4 * r) ? K[r * 4 + c] : T(0);
        });
      });
    }

    // ---- Y = M K_AB in place of K_AB (forward halves only: W = K_AA^-1 K_AB = M' D^-1 Y is never formed) and
    // S = K_BB - K_AB' W = K_BB - Y' D^-1 Y (by symmetry only k >= l)
    // all nb columns in one pass: row partials of the 4 x 16-cyclic tile reduced across each 16-lane row by
    // row_reduce_scatter16 (no LDS partials), one LDS exchange and barrier for every column together
    {
      const int ol = olane();
      const int ola = ol >> 4, olb = ol & 15;
      T ivc[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) ivc[c] = pivot_inv(L.dg[olb + 16 * c]);  // = invd_v of lane olb + 16 c
      sfor<0, NB>([&](auto l_) {
        constexpr int l = decltype(l_)::value;
        if (l < nb) {
          T tc[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) tc[c] = L.kab[l][olb + 16 * c] * ivc[c];
          T pr[16];
          sfor<0, 16>([&](auto r_) {
            constexpr int r = decltype(r_)::value;
            T acc = K[r * 4] * tc[0];
            sfor<1, r / 4 + 1>([&](auto c_) {
              constexpr int c = decltype(c_)::value;
              acc = fma(K[r * 4 + c], tc[c], acc);
            });
            pr[r] = acc;
          });
          L.scr[l * 64 + ola + 4 * olb] = ipm72::row_reduce_scatter16(pr, olb);  // row ola + 4 olb
        }
      });
      cbar();
      sfor<0, NB>([&](auto l_) {
        constexpr int l = decltype(l_)::value;
        if (l < nb) L.kab[l][ol] = L.kab[l][ol] - L.scr[l * 64 + ol];
      });
      cbar();
    }
    I72(3);
    // S -= Y' D^-1 Y: slot 8 k + l of the 8 x 8 block, products Y_max(k,l) (Y_min(k,l) / d) (so S stays exactly
    // symmetric), in four groups of 16 slots reduced across each 16-lane row (ipm72::row_reduce_scatter16), then the
    // four rows' partials through LDS; zero beyond nb
    {
      const int ol = olane();
      const int ola = ol >> 4, olb = ol & 15;
      T yv[NB], zv[NB];
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        yv[k] = k < nb ? L.kab[k][ol] : T(0);
        zv[k] = yv[k] * invd_v;
      }
      sfor<0, 4>([&](auto m_) {
        constexpr int m = decltype(m_)::value;
        T pr[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
          const int k = 2 * m + (t >> 3), l = t & 7;
          pr[t] = k >= l ? yv[k] * zv[l] : yv[l] * zv[k];
        }
        L.scr[ola * 64 + 16 * m + olb] = ipm72::row_reduce_scatter16(pr, olb);
      });
      cbar();
      const T sub = (L.scr[ol] + L.scr[64 + ol]) + (L.scr[128 + ol] + L.scr[192 + ol]);
      L.sb[ol] -= sub;
    }
    cbar();
    I72(4);
    {  // S^-1 by Gauss-Jordan across the wave (lane 8k + l holds S[k][l]); SPD: no pivoting
      const int gk = lane0 >> 3, gl = lane0 & 7;
      T s = L.sb[lane];
#pragma unroll
      for (int p = 0; p < NB; ++p) {
        const T pv = readlane(s, p * NB + p);
        const T inv = T(1) / pv;
        const T skp = __shfl(s, gk * NB + p, 64);
        const T spl = __shfl(s, p * NB + gl, 64);
        if (gk == p && gl == p) s = inv;
        else if (gk == p) s = spl * inv;
        else if (gl == p) s = -skp * inv;
        else s = fma(-skp * inv, spl, s);
      }
      if (uflag(__any(!isfinite(s)))) {
        status = CMPC_NAN_SOL;
        break;
      }
      L.sb[lane] = s;
      cbar();
    }

    I72(5);
    // ---- predictor (affine scaling direction)
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int j = lane + 64 * cc;
      L.rml[j] = tl[cc] * ll[cc];
      L.rmu[j] = tu[cc] * lu[cc];
    }
    direction();
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
      I72(6);
      // ---- corrector: rm = t.lam + dt_aff.dlam_aff - sigma mu
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        const int j = lane + 64 * cc;
        const bool on = j < m;
        L.rml[j] = on ? tl[cc] * ll[cc] + dtl[cc] * dll[cc] - sigma * mu : T(0);
        L.rmu[j] = on ? tu[cc] * lu[cc] + dtu[cc] * dlu[cc] - sigma * mu : T(0);
      }
      direction();
      alpha = fmin(T(1), T(TAU) * max_step());
    } else {
      alpha = fmin(T(1), max_step());
    }
    if (st_on && lane == 0) {
      double* sr = st_row();
      sr[3] = sr[4] = (double)alpha;
    }
    I72(7);
    if (uflag(alpha < T(S.alpha_min))) {
      status = CMPC_MIN_STEP;
      break;
    }
    u_v = fma(alpha, du_v, u_v);
    u_b = fma(alpha, du_b, u_b);
    // H du = rhs - (C' Sigma C + reg I) du for both slots (du in L.v, this iteration's blocks in L.blk)
    {
      const int ln = olane();
      auto ddu = [&](int var) -> T {
        const int t3 = 3 * (var / 3), e = var - t3;
        T r = T(0);
#pragma unroll
        for (int d = 0; d < 3; ++d) r = fma(L.blk[e][t3 + d], L.v[t3 + d], r);
        return r;
      };
      hu_v = fma(alpha, rhs_v - ddu(ln), hu_v);
      if (bin) hu_b = fma(alpha, rhs_b - ddu(64 + ln), hu_b);
    }
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      tl[cc] = fma(alpha, dtl[cc], tl[cc]);
      tu[cc] = fma(alpha, dtu[cc], tu[cc]);
      ll[cc] = fma(alpha, dll[cc], ll[cc]);
      lu[cc] = fma(alpha, dlu[cc], lu[cc]);
    }
    I72(8);
  }
  I72_STORE(it);

  lane = olane();
  const bool fin = isfinite(u_v) && isfinite(u_b);
  A.u[qg + lane] = u_v;
  if (bin) A.u[qg + 64 + lane] = u_b;
  for (int p = 64 + nb + lane; p < ld; p += 64) A.u[qg + p] = T(0);  // entries >= n are 0 (cmpc_qp_solve_batch)
  if (uflag(__any(!fin))) status = CMPC_NAN_SOL;
  if (lane == 0) {
    A.status[q] = status;
    A.iters[q] = it;
  }
  if (A.out_u) {  // direct epilogue: [N][4][3] forces (foothold triples map past 12 N and are not forces)
    const int nu = A.out_nu;
    T* buf = L.scr;
    for (int p = lane; p < nu; p += 64) buf[p] = T(0);
    cbar();
    const int i0 = A.tri_map[qt + lane / 3] * 3 + lane % 3;
    if (i0 < nu) buf[i0] = u_v;
    if (bin) {
      const int i1 = A.tri_map[qt + (64 + lane) / 3] * 3 + (64 + lane) % 3;
      if (i1 < nu) buf[i1] = u_b;
    }
    cbar();
    double* uo = A.out_u + (size_t)q * nu;
    for (int p = lane; p < nu; p += 64) uo[p] = (double)buf[p];
    if (lane == 0) {
      A.out_status[q] = status;
      if (A.out_iters) A.out_iters[q] = it;
    }
  }
  if (A.res) {
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
}

// One wave per QP of its list (run_ipm_classes splits 64 < n <= 72 off the 128 class: qlist[1] / qcount[1] here)
template <typename T, int WPE>
__global__ __launch_bounds__(64, WPE) void k_ipm72(IpmArgs<T> A) {
  int q = blockIdx.x;
  if (A.qlist[1]) {
    if (q >= A.qcount[1]) return;
    q = A.qlist[1][q];
    if ((unsigned)q >= gridDim.x) return;
  }
  ipm72_body<T, WPE>(A, q);
}

}  // namespace cmpc
