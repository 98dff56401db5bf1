#pragma once
// condense64.hpp — the n <= 64 condensing of one QP by one wavefront (stage 1 of the hot path), shared by the
// stand-alone kernel k_condense64 (k_condense64.hip) and the fused condense + IPM kernel k_solve64 (k_ipm64.hpp).
//
// SRBD linearisation, horizon propagation, dense condensing and friction-pyramid stacking. One wavefront per QP.
//
// Reference semantics (paths relative to the reference repo), identical to k_condense.hip:
//   dynamics  CentroidalMPC.cpp:85-92 forward Euler, lever arm linearised at r = p_{i,k} - c^ref_k, p the
//             stance foot position of stance_point (cmpc_device.hpp: :93 pinning, node 0 = current foot :165-167)
//   horizon   CentroidalMPC.cpp:159-176 multiple shooting -> condensed X = Aqp x0 + Bqp U
//   cost      CentroidalMPC.cpp:203-231 -> H = Bqp' Qbar Bqp + Rbar, g = Bqp' Qbar (Aqp x0 - Xref) + rbar (A.3)
//   f^des     CentroidalMPC.cpp:326-335 (m*9.81/n_stance, "mpc table invalid" when a step has no stance leg)
//   pyramid   CentroidalMPC.cpp:179-201; swing legs (0 <= F f <= 0) eliminated (A.4)
//
// MI355X mapping:
//   - lane c owns column c of Bqp (one stance force component) and propagates its 13-state image through the SRBD
//     transition with the A_k sparsity (13 FMAs per step); lanes 0..12 propagate the free response Aqp x0 and
//     publish Q_k (x_hat_k - xref_k) through LDS;
//   - each step the block row Bqp_k (13 x 64, padded to 16 rows) is staged in LDS twice (plain and Q_k-scaled) and
//     H += Bqp_k' Q_k Bqp_k runs on the matrix cores over the lower 16 x 16 tiles whose columns are already active
//     (v_mfma_f64_16x16x4_f64 / v_mfma_f32_16x16x4_f32), so the MFMA work follows the block-triangular Bqp;
//   - the f64 MFMA accumulator layout (lane 16g + col, register q <-> row g + 4q, column col) IS the 4 x 16-cyclic
//     tile of k_ipm64, so tile (I, J) register q is H register 4(4I + q) + J; for f32 the A-operand rows are
//     permuted so that the f32 layout (row 4g + q) lands on the same rows;
//   - upper tiles are the lower tiles transposed once through LDS; Rbar (force tracking + force-rate coupling) and
//     the identity padding are added per lane in the epilogue;
//   - H leaves as 64 coalesced 512-B rows per QP in the order k_ipm64 reads it (h_index).
// QPs with n > 64 are left to the bigger classes (k_condense.hip): their status is not written here, only nvar = n as
// a hint, so that k_srbd_condense can drop every QP this kernel finished without re-reading its contact table.
#include "cmpc_device.hpp"
#include "cmpc_kernels.hpp"

namespace cmpc {

namespace c64 {


constexpr int C64_MAXN = 21;  // n <= 64 with at least one stance leg per step needs N <= 21

template <typename T>
struct Mf64;
template <>
struct Mf64<double> {
  typedef double acc_t __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ acc_t run(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  // A-operand row read by lane column index col so that accumulator register q of lane (g, col) is row g + 4q
  static __device__ __forceinline__ int arow(int col) { return col; }
};
template <>
struct Mf64<float> {
  typedef float acc_t __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ acc_t run(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  // f32 C layout puts hardware row 4g + q in register q of lane g: feed actual row g + 4q there
  static __device__ __forceinline__ int arow(int col) { return (col >> 2) + 4 * (col & 3); }
};

template <typename T>
struct C64Lds {
  // Bqp_k rows 0..11 and Q_k Bqp_k rows 0..11: the MFMA contraction runs K = 12 (row 12, g_z, of Bqp is identically
  // zero and unweighted); keeping the LDS block at 18 KB (fp64) lets 8 one-wave workgroups share a CU's 160 KB
  // (at 22 KB with 16 staged rows only 7 fitted: 4096 QPs took three rounds of 1792 instead of two of 2048)
  T g[12][64];
  T qg[12][64];
  T tr[16][17];      // tile transpose (padded rows)
  double M[C64_MAXN][9];  // dt * I_b^-1 R_z(psi_k)^T (Theta rows of A_k)
  int tk[22], tleg[22];   // step and leg of each force triple
  int cb[C64_MAXN + 1];   // 3 * #triples of steps < k
  int nx[64], pv[64];     // next / previous variable of the same leg and component (force-rate pair), -1 none
  T dR[64], oR[64];       // Rbar diagonal and force-rate coupling per variable
  double xh[16];          // free response x_hat_k (lane s < 13 owns component s)
  T w[16];                // Q_k (x_hat_k - xref_k)
};

}  // namespace c64

// One QP's condensing (lane c owns Bqp column c). Writes H (tile order), g, the pyramid data, tri_map, status and
// nvar to the workspace exactly as the stand-alone kernel always did, and also hands the result to a fused caller:
// K = H in the 4 x 16-cyclic register tile of k_ipm64, g_out = g[lane], mu_out = the friction coefficient of the
// lane's force triple. Returns n, or < 0 when the IPM has nothing to do here: -2 invalid contact table (status
// written), -3 - n for n > 64 (left to the bigger classes with the nvar hint).
template <typename T>
__device__ __forceinline__ int condense64_qp(const CondenseArgs<T>& a, const int q, c64::C64Lds<T>& S, T (&K)[64],
                                             T& g_out, T& mu_out) {
  using namespace c64;

  using MF = Mf64<T>;
  using acc_t = typename MF::acc_t;
  const DevModel* __restrict__ M = a.model;
  const int lane = (int)threadIdx.x;  // one wave per QP
  const int g4 = lane >> 4, col = lane & 15;
  const int N = M->N;
  constexpr int L = NL;
  const int ld = a.ld;

  // ---- contact table: stance flags of (k, leg) in k-major order, two 64-bit ballots (N * L <= 84)
  const int ne = N * L;
  const uint8_t* ct = a.contact + (size_t)q * ne;
  const int e0 = lane < ne ? (ct[lane] ? 1 : 0) : 0;
  const int e1 = lane + 64 < ne ? (ct[lane + 64] ? 1 : 0) : 0;
  const unsigned long long b0 = __ballot(e0), b1 = __ballot(e1);
  const int nt = __popcll(b0) + __popcll(b1);
  const int n = 3 * nt;
  // steps without a stance leg -> "mpc table invalid" (CentroidalMPC.cpp:328-330)
  auto stance_bits = [&](int k) -> int {  // 4 flags of step k
    const int p = k * L;
    return p < 64 ? (int)((b0 >> p) & 15ull) : (int)((b1 >> (p - 64)) & 15ull);
  };
  bool invalid = false;
  for (int k = 0; k < N; ++k) invalid |= stance_bits(k) == 0;
  if (invalid) {
    if (lane == 0) {
      a.status[q] = CMPC_INVALID_CONTACT;
      a.nvar[q] = 0;
    }
    return -2;
  }
  if (n > 64) {  // a bigger class; the hint lets its condensing kernel skip every QP handled here at once
    if (lane == 0) a.nvar[q] = n;
    return -3 - n;
  }

  // ---- triples: t-th stance (k, leg) in k-major order
  {
    const int pre0 = __popcll(b0 & ((1ull << lane) - 1ull));
    const int pre1 = __popcll(b0) + __popcll(b1 & ((1ull << lane) - 1ull));
    if (e0) {
      S.tk[pre0] = lane / L;
      S.tleg[pre0] = lane % L;
    }
    if (e1) {
      S.tk[pre1] = (lane + 64) / L;
      S.tleg[pre1] = (lane + 64) % L;
    }
  }
  if (lane < N) {
    const double psi = a.xref[((size_t)q * (N + 1) + lane) * NX + 11];
    double sp, cp;
    sincos(psi, &sp, &cp);
    const double RzT[9] = {cp, sp, 0.0, -sp, cp, 0.0, 0.0, 0.0, 1.0};
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        double s = 0.0;
        for (int t = 0; t < 3; ++t) s += M->inv_inertia[r * 3 + t] * RzT[t * 3 + c];
        S.M[lane][r * 3 + c] = M->dt * s;
      }
  }
  if (lane <= N) {  // cb[k] = 3 * #stance (k', leg) with k' < k
    const int p = lane * L;
    int cnt = 0;
    if (p >= 64) cnt = __popcll(b0) + __popcll(b1 & ((p - 64 >= 64) ? ~0ull : ((1ull << (p - 64)) - 1ull)));
    else cnt = __popcll(b0 & ((1ull << p) - 1ull));
    S.cb[lane] = 3 * cnt;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");

  // ---- column c = lane: Rbar entries, force-rate partners, f^des linear term, lever arm
  const int c = lane;
  const bool colv = c < n;
  int kc = 0, d = 0, leg = 0;
  T gcol = T(0);
  double rx = 0, ry = 0, rz = 0;
  {
    int nx = -1, pv = -1;
    T dR = T(1), oR = T(0);  // padding: identity diagonal
    if (colv) {
      const int t = c / 3;
      d = c % 3;
      kc = S.tk[t];
      leg = S.tleg[t];
      const int j = 3 * leg + d;
      const int nb = (kc > 0) + (kc < N - 1);
      dR = T(2.0 * M->Wf[j] + 2.0 * M->Wr[j] * (double)nb);
      oR = T(-2.0 * M->Wr[j]);
      const int sb = stance_bits(kc);
      if (kc + 1 < N && ((stance_bits(kc + 1) >> leg) & 1)) {
        const int nsb = stance_bits(kc + 1);
        const int rank = __popc(nsb & ((1 << leg) - 1));
        nx = S.cb[kc + 1] + 3 * rank + d;
      }
      if (kc > 0 && ((stance_bits(kc - 1) >> leg) & 1)) {
        const int psb = stance_bits(kc - 1);
        const int rank = __popc(psb & ((1 << leg) - 1));
        pv = S.cb[kc - 1] + 3 * rank + d;
      }
      if (d == 2) gcol = T(-2.0 * M->Wf[j] * (M->mass * GRAV / (double)__popc(sb)));
      double p[3];
      stance_point(a.foot + (size_t)q * (N + 1) * L * 3, N, kc, leg,
                   [&](int k, int l) { return ((stance_bits(k) >> l) & 1) != 0; }, p);
      const double* cb = a.lin ? a.lin + ((size_t)q * N + kc) * 6 : a.xref + ((size_t)q * (N + 1) + kc) * NX;
      rx = p[0] - cb[0];
      ry = p[1] - cb[1];
      rz = p[2] - cb[2];
    }
    S.nx[c] = nx;
    S.pv[c] = pv;
    S.dR[c] = dR;
    S.oR[c] = oR;
  }

  // ---- free response x_hat = Aqp x0: lane s < 13 owns component s
  double xs = lane < NX ? a.x0[(size_t)q * NX + lane] : 0.0;
  T gam[NX];
#pragma unroll
  for (int s = 0; s < NX; ++s) gam[s] = T(0);

  acc_t acc[10];  // lower tiles (I, J), J <= I, index I(I+1)/2 + J
#pragma unroll
  for (int p = 0; p < 10; ++p) acc[p] = acc_t{T(0), T(0), T(0), T(0)};

  const T dt = T(M->dt);
  const T dtm = T(M->dt_over_m);
  const double* xrq = a.xref + (size_t)q * (N + 1) * NX;
  double xr_k = lane < NX ? xrq[NX + lane] : 0.0;          // xref_k[lane] and Qbar_k[lane] for the coming step
  double qd_k = lane < NX ? M->qdiag[1][lane] : 0.0;
  for (int k = 1; k <= N; ++k) {
    const int km = k - 1;
    // (a) gamma <- A_{k-1} gamma + B_{k-1}[:, c]
    const double* lk = a.lin ? a.lin + ((size_t)q * N + km) * 6 : nullptr;
    if (colv && kc <= km) {
      const T Lx = gam[6], Ly = gam[7], Lz = gam[8];
      if (lk) {  // L+ += dt F_bar x c (SQP linearisation)
        const T Fx = T(lk[3]), Fy = T(lk[4]), Fz = T(lk[5]);
        const T c0 = gam[0], c1 = gam[1], c2 = gam[2];
        gam[6] += dt * (Fy * c2 - Fz * c1);
        gam[7] += dt * (Fz * c0 - Fx * c2);
        gam[8] += dt * (Fx * c1 - Fy * c0);
      }
#pragma unroll
      for (int s = 0; s < 3; ++s) gam[s] += dt * gam[3 + s];
      gam[9] += T(S.M[km][0]) * Lx + T(S.M[km][1]) * Ly + T(S.M[km][2]) * Lz;
      gam[10] += T(S.M[km][3]) * Lx + T(S.M[km][4]) * Ly + T(S.M[km][5]) * Lz;
      gam[11] += T(S.M[km][6]) * Lx + T(S.M[km][7]) * Ly + T(S.M[km][8]) * Lz;
      gam[5] += dt * gam[12];
      if (kc == km) {
        gam[3 + d] += dtm;
        if (d == 0) {  // dt * [r]x e_d
          gam[7] += dt * T(rz);
          gam[8] -= dt * T(ry);
        } else if (d == 1) {
          gam[6] -= dt * T(rz);
          gam[8] += dt * T(rx);
        } else {
          gam[6] += dt * T(ry);
          gam[7] -= dt * T(rx);
        }
      }
    }
    // (b) free response x_hat_k = A_{k-1} x_hat_{k-1} and w_k = Q_k (x_hat_k - xref_k) (lanes s < 13)
    if (lane < 16) S.xh[lane] = xs;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (lane < NX) {
      const int s = lane;
      double xn = xs;
      if (s < 3) xn += M->dt * S.xh[s + 3];
      if (s == 5) xn += M->dt * S.xh[12];
      if (s >= 9 && s < 12) {
        const int r = s - 9;
        xn += S.M[km][r * 3 + 0] * S.xh[6] + S.M[km][r * 3 + 1] * S.xh[7] + S.M[km][r * 3 + 2] * S.xh[8];
      }
      if (lk && s >= 6 && s < 9) {  // dt F_bar x (c - c_bar)
        const double d0 = S.xh[0] - lk[0], d1 = S.xh[1] - lk[1], d2 = S.xh[2] - lk[2];
        const double cr = s == 6 ? lk[4] * d2 - lk[5] * d1 : (s == 7 ? lk[5] * d0 - lk[3] * d2 : lk[3] * d1 - lk[4] * d0);
        xn += M->dt * cr;
      }
      xs = xn;
      S.w[s] = T(qd_k * (xn - xr_k));
    }
    // next step's reference and weight, requested now so the loads are off the next step's critical path
    if (lane < NX && k < N) {
      xr_k = xrq[(k + 1) * NX + lane];
      qd_k = M->qdiag[k + 1][lane];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    {
      T accg = T(0);
#pragma unroll
      for (int s = 0; s < NX; ++s) {
        const double qd = M->qdiag[k][s];
        accg += gam[s] * S.w[s];
        if (s < 12) {
          S.g[s][lane] = gam[s];
          S.qg[s][lane] = T(qd) * gam[s];
        }
      }
      gcol += accg;  // (c) g += Bqp_k' w_k
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // (d) H += Bqp_k' Q_k Bqp_k over the active lower tiles
    const int ncols = S.cb[k];
    const int rowA = MF::arow(col);
#pragma unroll
    for (int I = 0; I < 4; ++I) {
      if (16 * I < ncols) {
        // K = 12: state row 12 (g_z) of Bqp is identically 0 (no input reaches it) and carries no weight
        // (Qbar_k[12] = 0) -- a fourth K-slab would add exact zeros
#pragma unroll
        for (int kk = 0; kk < 3; ++kk) {
          const int s = 4 * kk + g4;
          const T av = S.qg[s][16 * I + rowA];
#pragma unroll
          for (int J = 0; J <= I; ++J) {
            const T bv = S.g[s][16 * J + col];
            acc[I * (I + 1) / 2 + J] = MF::run(av, bv, acc[I * (I + 1) / 2 + J]);
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }

  // ---- H registers in the 4 x 16-cyclic order: lower tiles directly, upper tiles transposed through LDS
#pragma unroll
  for (int I = 0; I < 4; ++I)
#pragma unroll
    for (int J = 0; J <= I; ++J)
#pragma unroll
      for (int r = 0; r < 4; ++r) K[(4 * I + r) * 4 + J] = acc[I * (I + 1) / 2 + J][r];
#pragma unroll
  for (int I = 1; I < 4; ++I)
#pragma unroll
    for (int J = 0; J < I; ++J) {
      // tile (I, J): lane (g, col) reg r = H[16I + g + 4r][16J + col]; tile (J, I) at lane (g, col) reg r needs
      // H[16J + g + 4r][16I + col] = tile (I, J) entry (col, g + 4r)
#pragma unroll
      for (int r = 0; r < 4; ++r) S.tr[g4 + 4 * r][col] = acc[I * (I + 1) / 2 + J][r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
      for (int r = 0; r < 4; ++r) K[(4 * J + r) * 4 + I] = S.tr[col][g4 + 4 * r];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
  // ---- Rbar and identity padding: entry (i, j) = (a + 4r, b + 16cc) of this lane. Diagonal: dR[j] (1 for
  //      padding). Force-rate coupling oR[j] at (next(j), j) and (prev(j), j). Partners are 3..12 apart.
#pragma unroll
  for (int cc = 0; cc < 4; ++cc) {
    const int j = col + 16 * cc;
    const T dRj = S.dR[j], oRj = S.oR[j];
    const int nxj = S.nx[j], pvj = S.pv[j];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      constexpr int span = 12;
      // rows a + 4r can be within 12 of some column of this chunk only for these r
      if (4 * r + 3 >= 16 * cc - span && 4 * r <= 16 * cc + 15 + span) {
        const int i = g4 + 4 * r;
        T add = i == j ? dRj : T(0);
        add += (i == nxj || i == pvj) ? oRj : T(0);
        K[r * 4 + cc] += add;
      }
    }
  }

  // ---- outputs: H (class 64, tile order, the 40 lower-or-diagonal register rows: h_stored), g, pyramid data, status
  T* Hq = a.H + (size_t)q * ld * ld;
#pragma unroll
  for (int e = 0; e < 64; ++e)
    if ((e & 3) <= (e >> 4)) Hq[e * 64 + lane] = K[e];
  if (lane < ld) a.g[(size_t)q * ld + lane] = colv ? gcol : T(0);
  if (lane < ld / 3 && lane < 64 / 3) {
    const int t = lane;
    const bool on = t < nt;
    const int lg = on ? S.tleg[t] : 0;
    a.tri_mu[(size_t)q * (ld / 3) + t] = on ? T(M->mu[lg]) : T(0);
    for (int r = 0; r < 5; ++r) {
      a.tri_lo[((size_t)q * (ld / 3) + t) * 5 + r] = T(0);
      a.tri_hi[((size_t)q * (ld / 3) + t) * 5 + r] = T(M->ub[r]);
    }
    a.tri_map[(size_t)q * (ld / 3) + t] = on ? S.tk[t] * L + lg : -1;
  }
  if (lane == 0) {
    a.status[q] = CMPC_SUCCESS;
    a.nvar[q] = n;
  }
  g_out = colv ? gcol : T(0);
  mu_out = colv ? T(M->mu[leg]) : T(0);
  return n;
}

}  // namespace cmpc
