#pragma once
// srbd_condense.hpp — one QP's condensing by one workgroup (WAVES wavefronts): SRBD linearisation, horizon
// propagation, dense condensing and friction-pyramid stacking, for the workgroup size classes (n <= 128 / 256).
// Called by k_srbd_condense (k_condense.hip) and by the fused 128-class kernel k_solve128 (k_ipm128x.hpp), which
// runs the IPM on the same workgroup right after it.
//
// Reference semantics (paths relative to the reference repo):
//   dynamics  CentroidalMPC.cpp:85-92 forward Euler, lever arm linearised at r = p_{i,k} - c^ref_k, p the
//             stance foot position of stance_point (cmpc_device.hpp: :93 pinning, node 0 = current foot :165-167)
//   horizon   CentroidalMPC.cpp:159-176 multiple shooting -> condensed X = Aqp x0 + Bqp U
//   cost      CentroidalMPC.cpp:203-231 -> H = Bqp' Qbar Bqp + Rbar, g = Bqp' Qbar (Aqp x0 - Xref) + rbar (A.3)
//   f^des     CentroidalMPC.cpp:326-335 (m*9.81/n_stance, "mpc table invalid" when a step has no stance leg)
//   pyramid   CentroidalMPC.cpp:179-201; swing legs (0 <= F f <= 0) eliminated (A.4)
//
// MI355X mapping:
//   - column c of Bqp (one stance force component) lives in thread c: its 13-state image gamma is propagated through
//     the SRBD transition with the A_k sparsity pattern (13 FMAs/step, not a dense 13x13 product);
//   - every step k the block row Bqp_k (13 x n) is staged in LDS (double-buffered) and the rank-13 update
//     H += Bqp_k' Q_k Bqp_k runs on the matrix cores: v_mfma_f64_16x16x4_f64 (fp64) / v_mfma_f32_16x16x4_f32 (fp32),
//     16x16 lower tiles of H spread round-robin over the workgroup's wavefronts, accumulators in registers;
//   - tiles whose columns are still all-zero at step k (inputs of later steps) are skipped, so the MFMA work follows
//     the block-triangular structure of Bqp;
//   - Rbar (diagonal + force-rate off-diagonals) and the identity padding are folded into the accumulator epilogue.
#include "cmpc_device.hpp"
#include "cmpc_kernels.hpp"

namespace cmpc {

// Lab instrumentation (-DCMPC_COND_STAMPS on k_condense.hip only, lab/sqp_stamps.sh, never in libcmpc.so): wave 0 of
// the two-wave foothold instantiation (NMAX = 80) sums its shader-clock cycles per phase over every QP into
// cond_stamp_acc (cmpc_cond_debug_stamps): 0 record load + ballots, 1 per-step tables, 2 per-column setup, then per
// step 3 gamma update, 4 free response (thread 0), 5 block row + barrier, 6 g and MFMA H update; 7 epilogue; 15 QPs.
#ifdef CMPC_COND_STAMPS
__device__ unsigned long long cond_stamp_acc[16];
#define CD_DECL                                                  \
  unsigned long long cd_acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0};      \
  unsigned long long cd_prev_ = __builtin_amdgcn_s_memtime()
#define CD(id)                                                   \
  do {                                                           \
    if constexpr (NMAX == 80) {                                  \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
      cd_acc_[id] += now_ - cd_prev_;                            \
      cd_prev_ = now_;                                           \
    }                                                            \
  } while (0)
#define CD_STORE()                                                                   \
  do {                                                                               \
    if (NMAX == 80 && threadIdx.x == 0) {                                            \
      for (int k_ = 0; k_ < 8; ++k_) atomicAdd(&cond_stamp_acc[k_], cd_acc_[k_]);    \
      atomicAdd(&cond_stamp_acc[15], 1ull);                                          \
    }                                                                                \
  } while (0)
#else
#define CD_DECL (void)0
#define CD(id) (void)0
#define CD_STORE() (void)0
#endif

namespace srbd {

template <typename T>
struct Mfma;
template <>
struct Mfma<double> {
  typedef double acc_t __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ acc_t run(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  // C/D layout of v_mfma_f64_16x16x4_f64: col = lane&15, row = (lane>>4) + 4*reg
  static __device__ __forceinline__ int row(int lane, int reg) { return (lane >> 4) + 4 * reg; }
};
template <>
struct Mfma<float> {
  typedef float acc_t __attribute__((ext_vector_type(4)));
  static __device__ __forceinline__ acc_t run(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  // C/D layout of v_mfma_f32_16x16x4_f32: col = lane&15, row = 4*(lane>>4) + reg
  static __device__ __forceinline__ int row(int lane, int reg) { return 4 * (lane >> 4) + reg; }
};

__device__ __forceinline__ void tile_of(int idx, int& ti, int& tj) {
  ti = 0;
  while ((ti + 1) * (ti + 2) / 2 <= idx) ++ti;
  tj = idx - ti * (ti + 1) / 2;
}


// HN: the longest horizon the per-step arrays hold (MAXN; the small foothold instantiation k_srbd_condense<T, 80, 2,
// true, C64_HN> holds N <= 21 and fits four workgroups per CU)
template <typename T, int NMAX, int WAVES, bool FEET = false, int HN = MAXN>
struct SrbdLds {
  static constexpr int NTRI = NMAX / 3;
  static constexpr int FT = FEET ? NTRI : 1;  // foothold arrays only in the FEET instantiation (LDS of k_solve128)
  // Bqp block rows, double-buffered; row stride NMAX + 16 (16 mod 32 in fp32, half a 64-bank row in fp64): the MFMA
  // operand reads take rows s and s + 1 in one lane group, which then fall on disjoint banks
  static constexpr int GS = NMAX + 16;
  T s_G[2][16][GS];
  T s_w[2][16];
  T s_q[2][16];
  double s_xref[(HN + 1) * NX];
  double s_foot[(HN + 1) * NL * 3];
  double s_M[HN][9];
  uint8_t s_e[HN * NL];
  int s_ns[HN];
  int s_cb[HN + 1];  // 3 * #triples of steps < k
  int s_tk[NTRI], s_tleg[NTRI];
  int s_nt[HN];  // triples acting first at step k (stance legs + later runs starting at k)
  // foothold triples (CondenseArgs::dbar): force triple of each stance (k, leg), foothold flag, run end, box (delta)
  // and the run's mean des position
  int s_slot[FEET ? HN * NL : 1];
  int s_rs[FEET ? HN * NL : 1];            // first step of the run of each stance (k, leg)
  double s_fb[FEET ? HN * NU : 1];         // the iterate's forces f_bar [N][12] (CondenseArgs::ubar)
  double s_D[FEET ? HN * NU : 1];          // the iterate's foothold offsets [N][4][3] (CondenseArgs::dbar)
  uint8_t s_tf[FT];
  int s_te[FT];
  double s_blo[FT][3], s_bhi[FT][3], s_pbar[FT][3];
  T s_diagR[NMAX], s_offR[NMAX];
  int s_next[NMAX];
  int s_wtot[WAVES];
  int s_flag;
};

}  // namespace srbd

// One QP (workgroup of 64 * WAVES threads). EXT: the LDS block is the caller's (*ext, e.g. a union with the IPM's),
// else declared here. Writes H (class-packed), g, the pyramid data, tri_map, status and nvar to the workspace.
// Returns n when the QP was condensed here, -1 otherwise (invalid contact table / too large: status written; a
// bigger class: nvar hint; a smaller class: nothing).
// FEET: the instantiation that also serves CondenseArgs::dbar (foothold columns); without it dbar is ignored.
// NMAX = 80 (the small foothold instantiation) condenses n <= 72 only, the QPs k_ipm72 serves from rows / columns < 80
// of the class-128 block (CondenseArgs::h72 must be set); bigger ones are left to the 128 class.
template <typename T, int NMAX, int WAVES, bool EXT, bool FEET = false, int HN = MAXN>
__device__ __forceinline__ int srbd_condense_qp(const CondenseArgs<T>& a, int q,
                                                srbd::SrbdLds<T, NMAX, WAVES, FEET, HN>* ext) {
  using namespace srbd;
  constexpr int NT = NMAX / 16;              // 16x16 tiles per dimension
  constexpr int NLT = NT * (NT + 1) / 2;     // lower tiles
  constexpr int TPW = (NLT + WAVES - 1) / WAVES;
  constexpr int NTRI = NMAX / 3;
  constexpr int NTHR = 64 * WAVES;
  constexpr int NCAP = NMAX == 80 ? 72 : NMAX;  // largest n condensed here
  static_assert(NMAX <= NTHR, "one thread per column");
  using MF = Mfma<T>;
  using acc_t = typename MF::acc_t;
  const DevModel* __restrict__ M = a.model;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int N = M->N, L = NL;
  const int ld = a.ld;

  __shared__ SrbdLds<T, NMAX, WAVES, FEET, HN> Sl;  // stand-alone kernel: declared here (constant LDS base)
  SrbdLds<T, NMAX, WAVES, FEET, HN>& S = EXT ? *ext : Sl;

  CD_DECL;
  // ---- load the QP record into LDS
  const double* xr = a.xref + (size_t)q * (N + 1) * NX;
  const double* ft = a.foot + (size_t)q * (N + 1) * NL * 3;
  for (int i = tid; i < (N + 1) * NX; i += NTHR) S.s_xref[i] = xr[i];
  for (int i = tid; i < (N + 1) * NL * 3; i += NTHR) S.s_foot[i] = ft[i];
  if constexpr (FEET) {  // the iterate's forces and foothold offsets, read once (the per-step passes use LDS)
    if (a.dbar)
      for (int i = tid; i < N * NU; i += NTHR) {
        S.s_fb[i] = a.ubar[(size_t)q * N * NU + i];
        S.s_D[i] = a.dbar[(size_t)q * N * NU + i];
      }
  }
  for (int i = tid; i < 2 * 16 * S.GS; i += NTHR) (&S.s_G[0][0][0])[i] = T(0);
  if (tid < 32) (&S.s_w[0][0])[tid] = T(0), (&S.s_q[0][0])[tid] = T(0);
  if (tid == 0) S.s_flag = 0;
  const int ne = N * L;
  const bool feet = FEET && a.dbar != nullptr;
  int e = 0, fs = 0;
  if (tid < ne) {
    const uint8_t* ctq = a.contact + (size_t)q * ne;
    e = ctq[tid] ? 1 : 0;
    S.s_e[tid] = (uint8_t)e;
    fs = (feet && e && tid >= L && !ctq[tid - L]) ? 1 : 0;  // (k, leg) starts a later run
  }
  // ballot prefix over (k, leg) in k-major order -> triple index of each stance (k, leg); a later run's foothold
  // triple follows the force triple of its first (k, leg)
  const unsigned long long bal = __ballot(e), balf = __ballot(fs);
  const unsigned long long below = (1ull << lane) - 1ull;
  const int pre = __popcll(bal & below) + __popcll(balf & below);
  if (lane == 0) S.s_wtot[wave] = __popcll(bal) + __popcll(balf);
  __syncthreads();
  CD(0);
  int off = 0;
  for (int w = 0; w < wave; ++w) off += S.s_wtot[w];
  int nt = 0;
  for (int w = 0; w < WAVES; ++w) nt += S.s_wtot[w];
  if (e) {
    const int t = off + pre;
    if (FEET) {
      S.s_slot[tid] = t;
      S.s_rs[tid] = run_start(tid / L, tid % L, [&](int kk, int l) { return S.s_e[kk * L + l] != 0; });
    }
    if (t < NTRI) {
      S.s_tk[t] = tid / L;
      S.s_tleg[t] = tid % L;
      if (FEET) S.s_tf[t] = 0;
    }
    if (FEET && fs && t + 1 < NTRI) {
      const int k = tid / L, leg = tid % L;
      auto st = [&](int kk, int l) { return S.s_e[kk * L + l] != 0; };
      int ee = k;
      later_start(N, k, leg, st, &ee);
      S.s_tk[t + 1] = k;
      S.s_tleg[t + 1] = leg;
      S.s_tf[t + 1] = 1;
      S.s_te[t + 1] = ee;
      double pb[3];
      stance_point(S.s_foot, N, k, leg, st, pb);
      bool empty = false;
      for (int d = 0; d < 3; ++d) {
        double lo, hi;
        foot_box_d(S.s_foot, k, ee, leg, d, pb, &lo, &hi);
        S.s_pbar[t + 1][d] = pb[d];
        S.s_blo[t + 1][d] = lo;
        S.s_bhi[t + 1][d] = hi;
        empty = empty || !(lo <= hi);
      }
      if (empty) atomicOr(&S.s_flag, 2);
    }
    if (FEET && feet && tid < L) {  // a run from step 0 keeps the current foot at its nodes 1..e+1, inside the box
      int ee = 0;
      while (ee + 1 < N && S.s_e[(ee + 1) * L + tid]) ++ee;
      const double lb[3] = {CMPC_STEP_LB_XY, CMPC_STEP_LB_XY, CMPC_STEP_LB_Z};
      const double ub[3] = {CMPC_STEP_UB_XY, CMPC_STEP_UB_XY, CMPC_STEP_UB_Z};
      bool out = false;
      for (int j = 1; j <= ee + 1 && j <= N; ++j)
        for (int d = 0; d < 3; ++d) {
          const double v = (double)S.s_foot[tid * 3 + d] - (double)S.s_foot[(j * L + tid) * 3 + d];
          out = out || v < lb[d] || v > ub[d];
        }
      if (out) atomicOr(&S.s_flag, 2);
    }
  }
  if (tid < N) {
    int ns = 0, nf = 0;
    for (int i = 0; i < L; ++i) {
      ns += S.s_e[tid * L + i];
      nf += (feet && tid > 0 && S.s_e[tid * L + i] && !S.s_e[(tid - 1) * L + i]) ? 1 : 0;
    }
    S.s_ns[tid] = ns;
    S.s_nt[tid] = ns + nf;
    if (ns == 0) atomicOr(&S.s_flag, 1);
    // per-step M_k = dt * I_b^{-1} R_z(psi_k)^T  (Theta row of A_k)
    const double psi = S.s_xref[tid * NX + 11];
    double sp, cp;
    sincos(psi, &sp, &cp);
    const double RzT[9] = {cp, sp, 0.0, -sp, cp, 0.0, 0.0, 0.0, 1.0};
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        double s = 0.0;
        for (int t = 0; t < 3; ++t) s += M->inv_inertia[r * 3 + t] * RzT[t * 3 + c];
        S.s_M[tid][r * 3 + c] = M->dt * s;
      }
  }
  __syncthreads();
  CD(1);
  const int n = 3 * nt;
  int st = CMPC_SUCCESS;
  if (S.s_flag & 1) st = CMPC_INVALID_CONTACT;
  else if (S.s_flag & 2) st = CMPC_INFEASIBLE_STEP;
  else if (n > NCAP) {
    if (NMAX < CMPC_IPM_MAX_N) {  // a bigger class follows: leave the hint, not the status
      if (tid == 0) a.nvar[q] = n;
      return -1;
    }
    st = CMPC_TOO_LARGE;
  }
  if (st == CMPC_SUCCESS && n <= a.n_lo) return -1;  // served by a smaller class
  if (st != CMPC_SUCCESS) {
    if (tid == 0) {
      a.status[q] = st;
      a.nvar[q] = 0;
    }
    return -1;
  }
  if (tid == 0) {
    int acc = 0;
    for (int k = 0; k < N; ++k) {
      S.s_cb[k] = 3 * acc;
      acc += S.s_nt[k];
    }
    S.s_cb[N] = 3 * acc;
  }
  __syncthreads();

  // ---- per-column setup (thread c <-> column c)
  const int c = tid;
  const bool col = c < n;
  int kc = 0, d = 0, leg = 0;
  bool fcol = false;  // a foothold column (acts at steps kc..ke)
  int ke = 0;
  T gam[NX];
#pragma unroll
  for (int s = 0; s < NX; ++s) gam[s] = T(0);
  T gcol = T(0);
  double rx = 0, ry = 0, rz = 0;
  if (col) {
    const int t = c / 3;
    d = c % 3;
    kc = S.s_tk[t];
    leg = S.s_tleg[t];
    const int j = 3 * leg + d;
    auto stf = [&](int k, int l) { return S.s_e[k * L + l] != 0; };
    fcol = FEET && feet && S.s_tf[t];
    if (fcol) {  // foothold: 2 Wp cnt on the diagonal, 2 Wp sum_j (pbar - des_j) in g (oracle_condense_feet)
      ke = S.s_te[t];
      double gs = 0.0;
      for (int jn = kc; jn <= ke + 1; ++jn) gs += S.s_pbar[t][d] - S.s_foot[(jn * L + leg) * 3 + d];
      S.s_diagR[c] = T(2.0 * M->Wp[j] * (double)(ke + 2 - kc));
      S.s_offR[c] = T(0);
      S.s_next[c] = -1;
      gcol = T(2.0 * M->Wp[j] * gs);
    } else {
      const int nb = (kc > 0) + (kc < N - 1);
      S.s_diagR[c] = T(2.0 * M->Wf[j] + 2.0 * M->Wr[j] * (double)nb);
      S.s_offR[c] = T(-2.0 * M->Wr[j]);
      int nx = -1;
      if (kc + 1 < N && S.s_e[(kc + 1) * L + leg]) {
        if (FEET) {
          nx = 3 * S.s_slot[(kc + 1) * L + leg] + d;
        } else {
          int rank = 0;
          for (int i = 0; i < leg; ++i) rank += S.s_e[(kc + 1) * L + i];
          nx = S.s_cb[kc + 1] + 3 * rank + d;
        }
      }
      S.s_next[c] = nx;
      if (d == 2) gcol = T(-2.0 * M->Wf[j] * (M->mass * GRAV / (double)S.s_ns[kc]));
      double p[3];
      lever_point(S.s_foot, feet ? S.s_D : nullptr, N, kc, leg, stf, p);
      const double* cb = a.lin ? a.lin + ((size_t)q * N + kc) * 6 : S.s_xref + kc * NX;
      rx = p[0] - cb[0];
      ry = p[1] - cb[1];
      rz = p[2] - cb[2];
    }
  }
  // free response x_hat_k = Aqp x0 (thread 0)
  double xh[NX];
  if (tid == 0) {
    for (int s = 0; s < NX; ++s) xh[s] = a.x0[(size_t)q * NX + s];
  }

  acc_t acc[TPW];
#pragma unroll
  for (int p = 0; p < TPW; ++p) acc[p] = acc_t{T(0), T(0), T(0), T(0)};
  // this wave's lower tiles (slot p = tile wave + WAVES p, row-major lower order)
  // tile table (NMAX <= 128 only), packed 8 bits per tile (ti | tj << 4, 15 = no tile) in TW words: unpacked at each
  // use from an opaque copy, so the compiler cannot hoist 2 TPW tile addresses across the step loop (as unpacked
  // per-tile registers they were spilled to scratch in k_solve128<float>)
  constexpr int TT = NMAX <= 128 ? TPW : 1;
  constexpr int TW = (TT + 3) / 4;
  int tile_pk[TW];
#pragma unroll
  for (int w4 = 0; w4 < TW; ++w4) tile_pk[w4] = 0;
#pragma unroll
  for (int p = 0; p < TT; ++p) {
    const int idx = wave + p * WAVES;
    int ti = 15, tj = 15;
    if (idx < NLT) tile_of(idx, ti, tj);
    tile_pk[p >> 2] |= (ti | (tj << 4)) << (8 * (p & 3));
  }

  const T dt = T(M->dt);
  const T dtm = T(M->dt_over_m);
  CD(2);
  for (int k = 1; k <= N; ++k) {
    const int buf = k & 1;
    const int km = k - 1;
    // (a) gamma <- A_{k-1} gamma + B_{k-1}[:, c]
    const double* lk = a.lin ? a.lin + ((size_t)q * N + km) * 6 : nullptr;
    if (col && kc <= km) {
      T Lx = gam[6], Ly = gam[7], Lz = gam[8];
      if (lk) {  // L+ += dt F_bar x c (SQP linearisation)
        const T Fx = T(lk[3]), Fy = T(lk[4]), Fz = T(lk[5]);
        const T c0 = gam[0], c1 = gam[1], c2 = gam[2];
        gam[6] += dt * (Fy * c2 - Fz * c1);
        gam[7] += dt * (Fz * c0 - Fx * c2);
        gam[8] += dt * (Fx * c1 - Fy * c0);
      }
#pragma unroll
      for (int s = 0; s < 3; ++s) gam[s] += dt * gam[3 + s];
      gam[9] += T(S.s_M[km][0]) * Lx + T(S.s_M[km][1]) * Ly + T(S.s_M[km][2]) * Lz;
      gam[10] += T(S.s_M[km][3]) * Lx + T(S.s_M[km][4]) * Ly + T(S.s_M[km][5]) * Lz;
      gam[11] += T(S.s_M[km][6]) * Lx + T(S.s_M[km][7]) * Ly + T(S.s_M[km][8]) * Lz;
      gam[5] += dt * gam[12];
      if (fcol) {
        if (km <= ke) {  // dt e_d x f_bar_{leg, km}
          const double* fb = S.s_fb + km * NU + 3 * leg;
          if (d == 0) {
            gam[7] += dt * T(-fb[2]);
            gam[8] += dt * T(fb[1]);
          } else if (d == 1) {
            gam[6] += dt * T(fb[2]);
            gam[8] += dt * T(-fb[0]);
          } else {
            gam[6] += dt * T(-fb[1]);
            gam[7] += dt * T(fb[0]);
          }
        }
      } else if (kc == km) {
        gam[3 + d] += dtm;
        // dt * [r]x e_d
        if (d == 0) {
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
    CD(3);
    // (b) free response and weighted tracking error w_k = Q_k (x_hat_k - xref_k)
    if (tid == 0) {
      double xn[NX];
      for (int s = 0; s < 3; ++s) xn[s] = xh[s] + M->dt * xh[3 + s];
      for (int s = 3; s < 9; ++s) xn[s] = xh[s];
      xn[5] += M->dt * xh[12];
      for (int r = 0; r < 3; ++r)
        xn[9 + r] = xh[9 + r] + S.s_M[km][r * 3 + 0] * xh[6] + S.s_M[km][r * 3 + 1] * xh[7] + S.s_M[km][r * 3 + 2] * xh[8];
      if (lk) {  // dt F_bar x (c - c_bar)
        const double d0 = xh[0] - lk[0], d1 = xh[1] - lk[1], d2 = xh[2] - lk[2];
        xn[6] += M->dt * (lk[4] * d2 - lk[5] * d1);
        xn[7] += M->dt * (lk[5] * d0 - lk[3] * d2);
        xn[8] += M->dt * (lk[3] * d1 - lk[4] * d0);
      }
      if (feet)  // -dt D x f_bar of the later runs' stance legs
        for (int i = 0; i < L; ++i) {
          if (!S.s_e[km * L + i]) continue;
          const int s0 = S.s_rs[km * L + i];
          if (s0 == 0) continue;
          const double* dl = S.s_D + (s0 * NL + i) * 3;
          const double* fb = S.s_fb + km * NU + 3 * i;
          xn[6] -= M->dt * (dl[1] * fb[2] - dl[2] * fb[1]);
          xn[7] -= M->dt * (dl[2] * fb[0] - dl[0] * fb[2]);
          xn[8] -= M->dt * (dl[0] * fb[1] - dl[1] * fb[0]);
        }
      xn[12] = xh[12];
      for (int s = 0; s < NX; ++s) {
        xh[s] = xn[s];
        const double qd = M->qdiag[k][s];
        S.s_q[buf][s] = T(qd);
        S.s_w[buf][s] = T(qd * (xn[s] - S.s_xref[k * NX + s]));
      }
    }
    CD(4);
    // (c) stage block row Bqp_k
    if (c < NMAX) {
#pragma unroll
      for (int s = 0; s < NX; ++s) S.s_G[buf][s][c] = gam[s];
    }
    __syncthreads();
    CD(5);
    // (d) g += Bqp_k' w_k
    if (col) {
      T acc_g = T(0);
#pragma unroll
      for (int s = 0; s < NX; ++s) acc_g += gam[s] * S.s_w[buf][s];
      gcol += acc_g;
    }
    // (e) H += Bqp_k' Q_k Bqp_k on the matrix cores; tiles of not-yet-active columns skipped. The wave's tiles are
    //     in row-major order, so the active ones are a prefix (p < np). NMAX <= 128: K-slab outer, tiles inner, so
    //     consecutive MFMAs are independent accumulators and pipeline instead of waiting out each chain (the 256
    //     class keeps tile-outer order: its 17 tiles per wave leave no registers for the tile table)
    const int ncols = S.s_cb[k];
    if constexpr (NMAX <= 128) {
      int tpk[TW];
#pragma unroll
      for (int w4 = 0; w4 < TW; ++w4) {
        tpk[w4] = tile_pk[w4];
        asm volatile("" : "+v"(tpk[w4]));
      }
      auto tile_i = [&](int p) { return (tpk[p >> 2] >> (8 * (p & 3))) & 15; };
      auto tile_j = [&](int p) { return (tpk[p >> 2] >> (8 * (p & 3) + 4)) & 15; };
      int np = 0;
#pragma unroll
      for (int p = 0; p < TPW; ++p) np += (tile_i(p) != 15 && 16 * tile_i(p) < ncols) ? 1 : 0;
      // K = 12: Bqp row 12 (g_z) is identically 0 and unweighted, rows 13..15 are padding
#pragma unroll
      for (int s4 = 0; s4 < 3; ++s4) {
        const int s = 4 * s4 + (lane >> 4);
        const T qs = S.s_q[buf][s];
#pragma unroll
        for (int p = 0; p < TPW; ++p) {
          if (p < np) {
            const T av = qs * S.s_G[buf][s][16 * tile_i(p) + (lane & 15)];
            const T bv = S.s_G[buf][s][16 * tile_j(p) + (lane & 15)];
            acc[p] = MF::run(av, bv, acc[p]);
          }
        }
      }
    } else {
#pragma unroll
      for (int p = 0; p < TPW; ++p) {
        const int idx = wave + p * WAVES;
        if (idx < NLT) {
          int ti, tj;
          tile_of(idx, ti, tj);
          if (16 * ti < ncols) {
#pragma unroll
            for (int s4 = 0; s4 < 3; ++s4) {
              const int s = 4 * s4 + (lane >> 4);
              const T av = S.s_q[buf][s] * S.s_G[buf][s][16 * ti + (lane & 15)];
              const T bv = S.s_G[buf][s][16 * tj + (lane & 15)];
              acc[p] = MF::run(av, bv, acc[p]);
            }
          }
        }
      }
    }
    CD(6);
  }
  __syncthreads();

  // ---- epilogue: Rbar, identity padding, write the class-padded block of H, g and the pyramid data
  const int npad = ipm_class(n);
  const int hlim = (a.h72 && npad == 128 && n <= 72) ? 80 : npad;  // CondenseArgs::h72
  T* Hq = a.H + (size_t)q * ld * ld;
#pragma unroll
  for (int p = 0; p < TPW; ++p) {
    const int idx = wave + p * WAVES;
    if (idx < NLT) {
      int ti, tj;
      tile_of(idx, ti, tj);
      if (16 * ti < hlim) {
        const int cc = 16 * tj + (lane & 15);
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
          const int rr = 16 * ti + MF::row(lane, r4);
          T v = acc[p][r4];
          if (rr == cc) {
            v = rr < n ? v + S.s_diagR[rr] : T(1);
          } else {
            if (rr < n && S.s_next[rr] == cc) v += S.s_offR[rr];
            if (cc < n && S.s_next[cc] == rr) v += S.s_offR[cc];
          }
          Hq[h_index(npad, rr, cc)] = v;  // class-packed block in the order the IPM of class npad reads
          // classes 64 / 256: lower tiles only (h_stored); the NMAX = 128 kernels keep the unconditional mirror
          // (the run-time class test alone made k_solve128<float> 1.4 % slower)
          if (ti != tj && (NMAX == 128 || npad == 128)) Hq[h_index(npad, cc, rr)] = v;
        }
      }
    }
  }
  if (c < npad) a.g[(size_t)q * ld + c] = col ? gcol : T(0);
  if (tid < npad / 3) {
    const int t = tid;
    const bool on = t < nt;
    const bool ft = FEET && on && feet && S.s_tf[t];
    const int lg = on ? S.s_tleg[t] : 0;
    a.tri_mu[(size_t)q * (ld / 3) + t] = (on && !ft) ? T(M->mu[lg]) : T(0);
    for (int r = 0; r < 5; ++r) {
      double lo = 0.0, hi = M->ub[r];
      if (ft) {  // rows [-x, x, -y, y, z] of the step box
        const int dd = r < 4 ? r / 2 : 2;
        const bool neg = r == 0 || r == 2;
        lo = neg ? -S.s_bhi[t][dd] : S.s_blo[t][dd];
        hi = neg ? -S.s_blo[t][dd] : S.s_bhi[t][dd];
      }
      a.tri_lo[((size_t)q * (ld / 3) + t) * 5 + r] = T(lo);
      a.tri_hi[((size_t)q * (ld / 3) + t) * 5 + r] = T(hi);
    }
    a.tri_map[(size_t)q * (ld / 3) + t] = on ? (ft ? N * L : 0) + S.s_tk[t] * L + lg : -1;
  }
  if (tid == 0) {
    a.status[q] = CMPC_SUCCESS;
    a.nvar[q] = n;
  }
  CD(7);
  CD_STORE();
  return n;
}

}  // namespace cmpc
