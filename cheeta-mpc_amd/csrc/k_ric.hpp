#pragma once
// k_ric.hpp — the hot path in stage-wise form: SRBD linearisation + friction-pyramid QP + primal-dual Mehrotra IPM
// in ONE wavefront per QP, with the Newton systems solved by a Riccati recursion over the horizon instead of a dense
// factorisation of the condensed Hessian. This is how HPIPM solves the reference's OCP (d_ocp_qp_ipm_solve,
// HpipmInterface.cpp:282-284, ric_alg 0 HpipmInterfaceSettings.h:56); the condensed H is never formed (no condensing
// stage, no H round trip through the workspace). The iteration (residuals, stopping rule, predictor / corrector,
// fraction-to-boundary step) is the one of oracle/cmpc_oracle.c:qp_ipm_run and k_ipm64.hpp; only the Newton solve
// differs (oracle_riccati_solve_one restates this structured solve on the CPU; lab/ric_proto.py checks the slot-
// indexed recursion below against the condensed matrix, 2.5e-14).
//
// Newton system of the QP (H + C' Sigma C + reg I) du = b as an OCP over the stages:
//   z_k = [x_k (12: c, v, L, Theta; g_z is constant and never perturbed); up (12 slots 3 leg + d: the forces of step
//   k-1, which carry the force-rate coupling of CentroidalMPC.cpp:227-231)], input v_k = the stance slots of step k,
//   z_{k+1} = [A_k x_k + B_k v_k; v_k], z_0 = 0; stage Hessians Q_k = qdiag (k >= 1), R_k = 2 Wf + 2 Wr [k >= 1] +
//   the triple's 3x3 block (C' Sigma C + reg I), S_k = -2 Wr between v_k and up (same slot), up diagonal 2 Wr.
//   Backward: G = B~'P, Rt = R + G B~, Rt = L L' (lane-per-row Cholesky with the explicit inverse Li = L^-1),
//   St = S + G A~, Y = Li St, P_k = Q + A~'P A~ - Y'Y. Solve: h = -b + B~'p, w = Li h, p_k = A~'p - Y'w;
//   forward v = -Li'(w + Y z), z_{k+1} = A~ z + B~ v.
//
// MI355X mapping (one wave per QP, no workgroup barriers beyond the wave's own):
//   * P is held column-per-lane in two halves: lane (h, j) = 32 h + j holds rows 12 h .. 12 h + 11 of column j
//     (j < 24): the B~ and A~ products are combinations of the lane's own registers with uniform coefficients (the
//     lever arms and dt I^-1 R_z^T come from LDS as broadcasts), halves combined by one cross-half shuffle;
//   * Rt rows: lane (slot a, leg b) forms 3 entries from the G rows in LDS; the Cholesky runs lane-per-row with the
//     pivot row broadcast by readlane, and builds L^-1 alongside, so every later use of the factor (Y, both sweeps of
//     every solve) is a matrix-vector product instead of a serial substitution;
//   * the factors of every stage (Li 12 x 12, Y 12 x 24) go to a per-QP scratch slab (L2-resident between the
//     factorisation and the two solves of the same iteration);
//   * the IPM's vectors are lane-per-force-triple (t = lane + 64 c, c < TPL): the 5 pyramid rows of a triple are the
//     lane's own registers, so C u, C' lam and the 3x3 Newton blocks need no communication;
//   * the gradient H u + g at the start point is a rollout (13 states) and an adjoint sweep; later iterations carry
//     it (H du = rhs - (C' Sigma C + reg I) du, as k_ipm64).
#include "cmpc_device.hpp"
#include "cmpc_kernels.hpp"
#include "step_ratio.hpp"
#include "wave_dpp.hpp"

// Diagnostic builds only (-DCMPC_RIC_STAMPS, lab): s_memtime cycles per phase of each QP, written over row 0 of the
// statistics buffer (cmpc_enable_stats): [0] setup, [1] gradient, [2] factorisations, [3] solves, [4] the rest of the
// iterations, [5] total, [6] iterations.
#ifdef CMPC_RIC_STAMPS
#define RIC_STAMP_DECL                                 \
  unsigned long long rst_[6] = {0, 0, 0, 0, 0, 0};    \
  const unsigned long long rst0_ = ric::memtime();    \
  unsigned long long rprev_ = rst0_
#define RIC_STAMP(k)                             \
  do {                                           \
    const unsigned long long t_ = ric::memtime(); \
    rst_[k] += t_ - rprev_;                      \
    rprev_ = t_;                                 \
  } while (0)
#else
#define RIC_STAMP_DECL (void)0
#define RIC_STAMP(k) (void)0
#endif

namespace cmpc {

namespace ric {

__device__ __forceinline__ unsigned long long memtime() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

constexpr int ZS = 24;           // z slots: 12 state rows + 12 previous-force slots
constexpr int RS = 12 * 12 + 12 * ZS;  // scratch per stage: Li [12][12], Y [12][24]

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

template <typename T, int NR, int TPL, int FS>
struct Lds {
  T fac[FS];             // stage factors (compact): per stage Li packed lower, then the state columns of Y
  int foff[NR + 1];      // offset of stage k's factors in fac
  T wf2[12], wr2[12];    // 2 Wf, 2 Wr per force slot
  int sb[NR];            // stance mask of step k
  int cb[NR + 1];        // 3 * #triples before step k
  int tk[4 * NR], tleg[4 * NR];
  double lev[NR][4][3];  // lever arm p - c_bar of (step, leg)
  double Mth[NR][9];     // dt I_b^-1 R_z(psi_k)^T (Theta rows of A_k)
  T blk[4 * NR][5];      // Newton 3x3 block of each triple: xx, yy, zz, xz, yz (reg included)
  T bs[12 * NR];         // solve: right-hand side in condensed order, then the direction
  T wk[NR][12];          // solve: w_k of the backward sweep
  T vec[32];             // broadcast of the z-vector (p or z)
  T hv[16];              // broadcast of a slot vector
  T hv2[16];
  T itl[5][64 * TPL];    // 1 / t of the lane's pyramid rows (lane-private columns), kept across the factorisation
  T itu[5][64 * TPL];
  union {
    struct {
      T G[12][ZS];
      T Rt[12][12];
      T Pcol[6][12];
    } f;
    struct {
      double X[NR + 1][16];  // rollout, then the adjoint lambda_{k+1} in slot k + 1
      T uf[NR][12];
    } g;
  };
};

// Ordering of LDS traffic between the lanes of the one wave (the workgroup is one wave): LDS writes drained
// (lgkmcnt) before the other lanes read them. The factor store and every exchange live in LDS, so the fence has no
// outstanding global stores to wait for inside the iteration.
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

template <typename T>
__device__ __forceinline__ T shfl_x32(T v) {
  return __shfl_xor(v, 32, 64);
}

// compact index of force slot a (3 leg + d) among the stance slots of mask sk
__device__ __forceinline__ int cslot(int sk, int a) { return 3 * __popc(sk & ((1 << (a / 3)) - 1)) + a % 3; }

template <typename T>
__device__ __forceinline__ T pinv_sqrt(T d) {
  return d > T(Lim<T>::pivot_min) ? T(rsqrt_acc(d)) : T(0);
}

}  // namespace ric

// Body of one QP. TPL: force triples per lane (nt <= 64 TPL); NR: longest horizon the LDS block holds.
template <typename T, int TPL, int NR, int FS>
__device__ __forceinline__ void ric_body(const RicArgs<T>& A, const int q) {
  using namespace ric;
  __shared__ Lds<T, NR, TPL, FS> S;
  const DevModel* __restrict__ M = A.model;
  const int N = M->N;
  const int lane = (int)threadIdx.x;
  const DevSettings st = A.s;
  const T dt = T(M->dt), dtm = T(M->dt_over_m);
  RIC_STAMP_DECL;

  // ---- contact table: stance masks, triple offsets (k-major, legs ascending: the condensed variable order)
  int sbl = 0;
  if (lane < N) {
    const uint8_t* ct = A.contact + ((size_t)q * N + lane) * NL;
    sbl = (ct[0] ? 1 : 0) | (ct[1] ? 2 : 0) | (ct[2] ? 4 : 0) | (ct[3] ? 8 : 0);
  }
  const int nsl = __popc(sbl);
  int incl = nsl;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  const bool invalid = __any(lane < N && sbl == 0);
  const int nt = __shfl(incl, N - 1, 64);
  const int n = 3 * nt;
  const int ld = A.ld;
  auto finish_rejected = [&](int code) {
    if (lane == 0) {
      A.status[q] = code;
      A.nvar[q] = 0;
      A.iters[q] = 0;
    }
    if (A.out_u) {
      for (int p = lane; p < A.out_nu; p += 64) A.out_u[(size_t)q * A.out_nu + p] = 0.0;
      if (lane == 0) {
        A.out_status[q] = code;
        if (A.out_iters) A.out_iters[q] = 0;
      }
    }
    if (A.res && lane < 4) A.res[(size_t)q * 4 + lane] = __builtin_nan("");
  };
  if (invalid) {  // "mpc table invalid" (CentroidalMPC.cpp:328-330)
    finish_rejected(CMPC_INVALID_CONTACT);
    return;
  }
  if (nt > 64 * TPL || N > NR) {
    finish_rejected(CMPC_TOO_LARGE);
    return;
  }
  // factor storage per stage: m (m + 1) / 2 + 12 m (m = 3 n_stance)
  const int msl = 3 * nsl;
  int fsz = lane < N ? msl * (msl + 1) / 2 + 12 * msl : 0;
  int fpre = fsz;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(fpre, o, 64);
    if (lane >= o) fpre += v;
  }
  const int ftot = __shfl(fpre, N - 1, 64);
  if (ftot > FS) {
    finish_rejected(CMPC_TOO_LARGE);
    return;
  }
  if (lane < N) {
    S.sb[lane] = sbl;
    S.cb[lane] = 3 * (incl - nsl);
    S.foff[lane] = fpre - fsz;
  }
  if (lane == 0) S.cb[N] = 3 * nt;
  if (lane < 12) {
    S.wf2[lane] = T(2.0 * M->Wf[lane]);
    S.wr2[lane] = T(2.0 * M->Wr[lane]);
  }
  wsync();
  // triple table, lever arms (stance_point, cmpc_device.hpp) and the Theta rows of A_k
  for (int e = lane; e < NL * N; e += 64) {
    const int k = e >> 2, l = e & 3;
    const int sk = S.sb[k];
    if ((sk >> l) & 1) {
      const int t = S.cb[k] / 3 + __popc(sk & ((1 << l) - 1));
      S.tk[t] = k;
      S.tleg[t] = l;
      double p[3];
      stance_point(A.foot + (size_t)q * (N + 1) * NL * 3, N, k, l,
                   [&](int kk, int ll) { return ((S.sb[kk] >> ll) & 1) != 0; }, p);
      const double* cb = A.lin ? A.lin + ((size_t)q * N + k) * 6 : A.xref + ((size_t)q * (N + 1) + k) * NX;
      S.lev[k][l][0] = p[0] - cb[0];
      S.lev[k][l][1] = p[1] - cb[1];
      S.lev[k][l][2] = p[2] - cb[2];
      if (A.tri_map) A.tri_map[(size_t)q * (ld / 3) + t] = k * NL + l;
    }
  }
  if (lane < N) {
    const double psi = A.xref[((size_t)q * (N + 1) + lane) * NX + 11];
    double sp, cp;
    sincos(psi, &sp, &cp);
    const double RzT[9] = {cp, sp, 0.0, -sp, cp, 0.0, 0.0, 0.0, 1.0};
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        double s = 0.0;
        for (int t = 0; t < 3; ++t) s += M->inv_inertia[r * 3 + t] * RzT[t * 3 + c];
        S.Mth[lane][r * 3 + c] = M->dt * s;
      }
  }
  wsync();

  // ---- lane-per-triple data
  int tkv[TPL], tlv[TPL];
  bool ton[TPL];
  T mu_t[TPL];
#pragma unroll
  for (int c = 0; c < TPL; ++c) {
    const int t = lane + 64 * c;
    ton[c] = t < nt;
    tkv[c] = ton[c] ? S.tk[t] : 0;
    tlv[c] = ton[c] ? S.tleg[t] : 0;
    mu_t[c] = ton[c] ? T(M->mu[tlv[c]]) : T(0);
  }
  T ub[5];
#pragma unroll
  for (int r = 0; r < 5; ++r) ub[r] = T(M->ub[r]);
  auto pyr = [](T mu, const T* f, T* c5) {
    const T mz = mu * f[2];
    c5[0] = mz - f[0];
    c5[1] = mz + f[0];
    c5[2] = mz - f[1];
    c5[3] = mz + f[1];
    c5[4] = f[2];
  };
  auto pyrT = [](T mu, const T* w, T* f) {
    f[0] = w[1] - w[0];
    f[1] = w[3] - w[2];
    f[2] = mu * (w[0] + w[1] + w[2] + w[3]) + w[4];
  };

  T u[TPL][3];
#pragma unroll
  for (int c = 0; c < TPL; ++c)
#pragma unroll
    for (int d = 0; d < 3; ++d) u[c][d] = T(0);

  RIC_STAMP(0);
  // ---- H u + g at the start point (u = 0): rollout of the 13 states and the adjoint sweep (oracle ric_grad)
  T hug[TPL][3];
  {
    for (int e = lane; e < N * 12; e += 64) S.g.uf[e / 12][e % 12] = T(0);
    wsync();
#pragma unroll
    for (int c = 0; c < TPL; ++c)
      if (ton[c])
#pragma unroll
        for (int d = 0; d < 3; ++d) S.g.uf[tkv[c]][3 * tlv[c] + d] = u[c][d];
    double xs = lane < NX ? A.x0[(size_t)q * NX + lane] : 0.0;
    const double* xrq = A.xref + (size_t)q * (N + 1) * NX;
    const double dtd = M->dt, dtmd = M->dt_over_m;
    for (int k = 0; k < N; ++k) {
      if (lane < 16) S.g.X[k][lane] = lane < NX ? xs : 0.0;
      wsync();
      if (lane < NX) {
        const int s = lane;
        const double* X = S.g.X[k];
        const int sk = S.sb[k];
        double xn = xs;
        if (s < 3) xn += dtd * X[3 + s];
        if (s == 5) xn += dtd * X[12];
        if (s >= 3 && s < 6) {
          double f = 0.0;
          for (int l = 0; l < NL; ++l)
            if ((sk >> l) & 1) f += (double)S.g.uf[k][3 * l + s - 3];
          xn += dtmd * f;
        }
        if (s >= 6 && s < 9) {
          double tq = 0.0;
          for (int l = 0; l < NL; ++l)
            if ((sk >> l) & 1) {
              const double* r = S.lev[k][l];
              const double fx = S.g.uf[k][3 * l], fy = S.g.uf[k][3 * l + 1], fz = S.g.uf[k][3 * l + 2];
              tq += s == 6 ? r[1] * fz - r[2] * fy : (s == 7 ? r[2] * fx - r[0] * fz : r[0] * fy - r[1] * fx);
            }
          xn += dtd * tq;
        }
        if (s >= 9 && s < 12) {
          const double* Mk = S.Mth[k];
          const int r = s - 9;
          xn += Mk[3 * r] * X[6] + Mk[3 * r + 1] * X[7] + Mk[3 * r + 2] * X[8];
        }
        if (A.lin && s >= 6 && s < 9) {  // dt F_bar x (c - c_bar)
          const double* lk = A.lin + ((size_t)q * N + k) * 6;
          const double d0 = X[0] - lk[0], d1 = X[1] - lk[1], d2 = X[2] - lk[2];
          xn += dtd * (s == 6 ? lk[4] * d2 - lk[5] * d1 : (s == 7 ? lk[5] * d0 - lk[3] * d2 : lk[3] * d1 - lk[4] * d0));
        }
        xs = xn;
      }
      wsync();
    }
    if (lane < 16) S.g.X[N][lane] = lane < NX ? xs : 0.0;
    wsync();
    // adjoint: lambda_N = qdiag_N (X_N - xref_N); lambda_k = qdiag_k (X_k - xref_k) + A_k' lambda_{k+1}; slot k + 1
    // of S.g.X is overwritten with lambda_{k+1} once X_{k+1} has been used
    double lam = lane < NX ? M->qdiag[N][lane] * (xs - xrq[N * NX + lane]) : 0.0;
    for (int k = N - 1; k >= 0; --k) {
      const double xk = lane < NX ? S.g.X[k][lane] : 0.0;
      wsync();
      if (lane < 16) S.g.X[k + 1][lane] = lane < NX ? lam : 0.0;
      wsync();
      if (k > 0 && lane < NX) {
        const double* Lm = S.g.X[k + 1];
        const int s = lane;
        double ln = M->qdiag[k][s] * (xk - xrq[k * NX + s]) + lam;
        if (s >= 3 && s < 6) ln += dtd * Lm[s - 3];
        if (s == 12) ln += dtd * Lm[5];
        if (s >= 6 && s < 9) {
          const double* Mk = S.Mth[k];
          const int cc = s - 6;
          ln += Mk[cc] * Lm[9] + Mk[3 + cc] * Lm[10] + Mk[6 + cc] * Lm[11];
        }
        if (A.lin && s < 3) {  // (dt [F_bar]x)' lambda_L
          const double* lk = A.lin + ((size_t)q * N + k) * 6;
          const double Fx = lk[3], Fy = lk[4], Fz = lk[5];
          const double l6 = Lm[6], l7 = Lm[7], l8 = Lm[8];
          ln += dtd * (s == 0 ? (Fz * l7 - Fy * l8) : (s == 1 ? (Fx * l8 - Fz * l6) : (Fy * l6 - Fx * l7)));
        }
        lam = ln;
      }
    }
    wsync();
    // gradient of each triple: B_k' lambda_{k+1} + 2 Wf (u - f_des) + force-rate terms
#pragma unroll
    for (int c = 0; c < TPL; ++c) {
#pragma unroll
      for (int d = 0; d < 3; ++d) hug[c][d] = T(0);
      if (ton[c]) {
        const int k = tkv[c], l = tlv[c];
        const double* Lm = S.g.X[k + 1];
        const double* r = S.lev[k][l];
        const double cx = Lm[7] * r[2] - Lm[8] * r[1], cy = Lm[8] * r[0] - Lm[6] * r[2],
                     cz = Lm[6] * r[1] - Lm[7] * r[0];  // lambda_L x r
        const double cr[3] = {cx, cy, cz};
        const double fdz = M->mass * GRAV / (double)__popc(S.sb[k]);
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          const int j = 3 * l + d;
          const double uk = (double)S.g.uf[k][j];
          double acc = dtmd * Lm[3 + d] + dtd * cr[d];
          acc += 2.0 * M->Wf[j] * (uk - (d == 2 ? fdz : 0.0));
          if (k > 0) acc += 2.0 * M->Wr[j] * (uk - (double)S.g.uf[k - 1][j]);
          if (k < N - 1) acc -= 2.0 * M->Wr[j] * ((double)S.g.uf[k + 1][j] - uk);
          hug[c][d] = T(acc);
        }
      }
    }
    wsync();
  }

  RIC_STAMP(1);
  // ---- IPM state: pyramid rows of each triple, slacks clipped at THR0, lam = mu0 / t
  T tl[TPL][5], tu[TPL][5], ll[TPL][5], lu[TPL][5];
#pragma unroll
  for (int c = 0; c < TPL; ++c) {
    T cu0[5];
    pyr(mu_t[c], u[c], cu0);
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      tl[c][r] = ton[c] ? fmax(cu0[r], T(THR0)) : T(1);
      tu[c][r] = ton[c] ? fmax(ub[r] - cu0[r], T(THR0)) : T(1);
      ll[c][r] = ton[c] ? T(st.mu0) / tl[c][r] : T(0);
      lu[c][r] = ton[c] ? T(st.mu0) / tu[c][r] : T(0);
    }
  }
  const int m = 5 * nt;
  const int hh = lane >> 5, jj = lane & 31;
  const bool colv = jj < ZS;

  // ---- Riccati factorisation of the Newton matrix (blocks in S.blk); returns false on a NaN pivot. The factors of
  //      stage k stay in LDS (S.fac + S.foff[k], compact slot order): Li packed lower [m (m + 1) / 2], then the state
  //      columns of Y [m][12]. The previous-force columns of Y are not stored: St has one entry -2 Wr there (same
  //      slot, leg in stance at k - 1 and k), so Y[.][12 + c] = -2 Wr_c Li[.][c].
  auto factor = [&]() -> bool {
    T Pc[12];
#pragma unroll
    for (int r = 0; r < 12; ++r) Pc[r] = (hh == 0 && jj == r) ? T(M->qdiag[N][r]) : T(0);
    bool nanp = false;
    for (int k = N - 1; k >= 0; --k) {
      const int Sk = S.sb[k];
      const int Sp = k > 0 ? S.sb[k - 1] : 0;
      const int Sc = Sk & Sp;
      const int m = 3 * __popc(Sk);
      T* F = S.fac + S.foff[k];
      T* Yx = F + m * (m + 1) / 2;
      // columns c (0..2) and Theta (9..11) of P, rows 0..11, for A~'P A~
      if (hh == 0 && (jj < 3 || (jj >= 9 && jj < 12))) {
        const int pc = jj < 3 ? jj : jj - 6;
#pragma unroll
        for (int r = 0; r < 12; ++r) S.f.Pcol[pc][r] = Pc[r];
      }
      // 1. G = B~' P, column jj, rows = stance slots
#pragma unroll
      for (int l = 0; l < NL; ++l) {
        if ((Sk >> l) & 1) {
          const T rx = T(S.lev[k][l][0]), ry = T(S.lev[k][l][1]), rz = T(S.lev[k][l][2]);
#pragma unroll
          for (int d = 0; d < 3; ++d) {
            const T wx = d == 0 ? T(0) : (d == 1 ? -rz : ry);
            const T wy = d == 0 ? rz : (d == 1 ? T(0) : -rx);
            const T wz = d == 0 ? -ry : (d == 1 ? rx : T(0));
            const T xp = dtm * Pc[3 + d] + dt * (wx * Pc[6] + wy * Pc[7] + wz * Pc[8]);
            const T part = hh ? Pc[3 * l + d] : xp;
            const T gv = part + shfl_x32(part);
            if (hh == 0 && colv) S.f.G[3 * l + d][jj] = gv;
          }
        }
      }
      wsync();
      // 2. Rt = R_k + G B~: lane (slot a, leg b) forms Rt[a][3b .. 3b + 2]
      if (lane < 48) {
        const int a = lane % 12, lb = lane / 12;
        const int la = a / 3, da = a % 3;
        if (((Sk >> la) & 1) && ((Sk >> lb) & 1)) {
          const T rx = T(S.lev[k][lb][0]), ry = T(S.lev[k][lb][1]), rz = T(S.lev[k][lb][2]);
          const T g6 = S.f.G[a][6], g7 = S.f.G[a][7], g8 = S.f.G[a][8];
          const int tb = S.cb[k] / 3 + __popc(Sk & ((1 << lb) - 1));
#pragma unroll
          for (int db = 0; db < 3; ++db) {
            const T wx = db == 0 ? T(0) : (db == 1 ? -rz : ry);
            const T wy = db == 0 ? rz : (db == 1 ? T(0) : -rx);
            const T wz = db == 0 ? -ry : (db == 1 ? rx : T(0));
            T v = dtm * S.f.G[a][3 + db] + dt * (wx * g6 + wy * g7 + wz * g8) + S.f.G[a][12 + 3 * lb + db];
            if (la == lb) {
              const T* bk = S.blk[tb];
              // block (da, db): xx yy zz on the diagonal, xz / yz off it, xy = 0
              const T bv = da == db ? bk[da] : ((da + db == 2 && da != 1) ? bk[3] : ((da + db == 3) ? bk[4] : T(0)));
              v += bv;
              if (da == db) v += S.wf2[a] + (k >= 1 ? S.wr2[a] : T(0));
            }
            S.f.Rt[a][3 * lb + db] = v;
          }
        }
      }
      wsync();
      // 3. Cholesky Rt = L L' and Li = L^-1, lane a < 12 holds row a
      {
        T R[12], Iv[12];
#pragma unroll
        for (int b = 0; b < 12; ++b) {
          R[b] = (lane < 12 && ((Sk >> (b / 3)) & 1)) ? S.f.Rt[lane < 12 ? lane : 0][b] : T(0);
          Iv[b] = lane == b ? T(1) : T(0);
        }
#pragma unroll
        for (int p = 0; p < 12; ++p) {
          if ((Sk >> (p / 3)) & 1) {
            const T dp = readlane(R[p], p);
            nanp |= dp != dp;
            const T invs = pinv_sqrt(dp);
            const T lap = lane > p ? R[p] * invs : T(0);
#pragma unroll
            for (int c = 0; c <= p; ++c) Iv[c] = lane == p ? Iv[c] * invs : Iv[c];
#pragma unroll
            for (int b = p + 1; b < 12; ++b)
              if ((Sk >> (b / 3)) & 1) R[b] = fma(-lap, readlane(R[p], b) * invs, R[b]);
#pragma unroll
            for (int c = 0; c <= p; ++c)
              if ((Sk >> (c / 3)) & 1) Iv[c] = fma(-lap, readlane(Iv[c], p), Iv[c]);
          }
        }
        if (lane < 12 && ((Sk >> (lane / 3)) & 1)) {
          const int ap = cslot(Sk, lane);
#pragma unroll
          for (int c = 0; c < 12; ++c)
            if (c <= lane && ((Sk >> (c / 3)) & 1)) F[ap * (ap + 1) / 2 + cslot(Sk, c)] = Iv[c];
        }
      }
      if (k == 0) break;
      wsync();
      // 4. St = S_k + G A~ (column jj of z_k), Y = Li St
      T Yc[12];
      {
        T stc[12];
#pragma unroll
        for (int a = 0; a < 12; ++a) {
          T v = T(0);
          if ((Sk >> (a / 3)) & 1) {
            if (jj < 12) {
              v = S.f.G[a][jj];
              if (jj >= 3 && jj < 6) v = fma(dt, S.f.G[a][jj - 3], v);
              if (jj >= 6 && jj < 9) {
                const double* Mk = S.Mth[k];
                const int cc = jj - 6;
                v += T(Mk[cc]) * S.f.G[a][9] + T(Mk[3 + cc]) * S.f.G[a][10] + T(Mk[6 + cc]) * S.f.G[a][11];
              }
            } else if (jj < ZS) {
              const int sj = jj - 12;
              if (sj == a && ((Sp >> (sj / 3)) & 1)) v = -S.wr2[a];
            }
          }
          stc[a] = v;
        }
#pragma unroll
        for (int a = 0; a < 12; ++a) {
          T y = T(0);
          if ((Sk >> (a / 3)) & 1) {
            const int ap = cslot(Sk, a);
            const T* Lr = F + ap * (ap + 1) / 2;
#pragma unroll
            for (int c = 0; c <= a; ++c)
              if ((Sk >> (c / 3)) & 1) y = fma(Lr[cslot(Sk, c)], stc[c], y);
          }
          Yc[a] = y;
        }
      }
      if (hh == 0 && jj < 12) {
#pragma unroll
        for (int a = 0; a < 12; ++a)
          if ((Sk >> (a / 3)) & 1) Yx[cslot(Sk, a) * 12 + jj] = Yc[a];
      }
      wsync();
      // 5. P_k = Q_k + A~' P A~ - Y' Y (+ 2 Wr on the previous-force slots of the legs of step k - 1)
      T nc[12];
      if (hh == 0 && jj < 12) {
        T X[12];
        const double* Mk = S.Mth[k];
#pragma unroll
        for (int r = 0; r < 12; ++r) {
          T v = Pc[r];
          if (jj >= 3 && jj < 6) v = fma(dt, S.f.Pcol[jj - 3][r], v);
          if (jj >= 6 && jj < 9) {
            const int cc = jj - 6;
            v += T(Mk[cc]) * S.f.Pcol[3][r] + T(Mk[3 + cc]) * S.f.Pcol[4][r] + T(Mk[6 + cc]) * S.f.Pcol[5][r];
          }
          X[r] = v;
        }
#pragma unroll
        for (int r = 0; r < 12; ++r) {
          T v = X[r];
          if (r >= 3 && r < 6) v = fma(dt, X[r - 3], v);
          if (r >= 6 && r < 9) {
            const int cc = r - 6;
            v += T(Mk[cc]) * X[9] + T(Mk[3 + cc]) * X[10] + T(Mk[6 + cc]) * X[11];
          }
          if (r == jj) v += T(M->qdiag[k][r]);
          nc[r] = v;
        }
      } else {
#pragma unroll
        for (int r = 0; r < 12; ++r)
          nc[r] = (hh == 1 && jj >= 12 && jj < ZS && r == jj - 12 && ((Sp >> (r / 3)) & 1)) ? S.wr2[r] : T(0);
      }
      // rows of Y: state rows from Yx (hh = 0), previous-force rows -2 Wr_r Li[.][r] (hh = 1, legs of S_k and S_k-1)
#pragma unroll
      for (int a = 0; a < 12; ++a) {
        if ((Sk >> (a / 3)) & 1) {
          const T ya = Yc[a];
          const int ap = cslot(Sk, a);
#pragma unroll
          for (int r = 0; r < 12; ++r) {
            const bool upv = ((Sc >> (r / 3)) & 1) && r <= a;
            const int ad = hh == 0 ? m * (m + 1) / 2 + ap * 12 + r : ap * (ap + 1) / 2 + (upv ? cslot(Sk, r) : 0);
            const T sc = hh == 0 ? T(1) : (upv ? -S.wr2[r] : T(0));
            nc[r] = fma(-(F[ad] * sc), ya, nc[r]);
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 12; ++r) Pc[r] = colv ? nc[r] : T(0);
      wsync();
    }
    wsync();
    return !__any(nanp);
  };

  // ---- solve (H + C' Sigma C + reg I) x = b, b and x in the triple lanes' registers, with the stage factors in LDS
  auto solve = [&](T (&bx)[TPL][3]) {
#pragma unroll
    for (int c = 0; c < TPL; ++c)
      if (ton[c]) {
        const int t = lane + 64 * c;
#pragma unroll
        for (int d = 0; d < 3; ++d) S.bs[3 * t + d] = bx[c][d];
      }
    T pv = T(0);
    for (int k = N - 1; k >= 0; --k) {
      const int Sk = S.sb[k];
      const int Sp = k > 0 ? S.sb[k - 1] : 0;
      const int Sc = Sk & Sp;
      const int m = 3 * __popc(Sk);
      const T* F = S.fac + S.foff[k];
      const T* Yx = F + m * (m + 1) / 2;
      if (lane < ZS) S.vec[lane] = pv;
      wsync();
      T hva = T(0);
      const bool sa = lane < 12 && ((Sk >> (lane / 3)) & 1);
      const int ap = sa ? cslot(Sk, lane) : 0;
      if (sa) {
        const int l = lane / 3, d = lane % 3;
        const T rx = T(S.lev[k][l][0]), ry = T(S.lev[k][l][1]), rz = T(S.lev[k][l][2]);
        const T wx = d == 0 ? T(0) : (d == 1 ? -rz : ry);
        const T wy = d == 0 ? rz : (d == 1 ? T(0) : -rx);
        const T wz = d == 0 ? -ry : (d == 1 ? rx : T(0));
        const int t = S.cb[k] / 3 + __popc(Sk & ((1 << l) - 1));
        hva = -S.bs[3 * t + d] + dtm * S.vec[3 + d] + dt * (wx * S.vec[6] + wy * S.vec[7] + wz * S.vec[8]) +
              S.vec[12 + lane];
      }
      if (lane < 12) S.hv[lane] = hva;
      wsync();
      T wa = T(0);
      if (sa) {
        const T* Lr = F + ap * (ap + 1) / 2;
#pragma unroll
        for (int c = 0; c < 12; ++c)
          if (((Sk >> (c / 3)) & 1) && c <= lane) wa = fma(Lr[cslot(Sk, c)], S.hv[c], wa);
        S.wk[k][lane] = wa;
      }
      if (k == 0) break;
      if (lane < 12) S.hv2[lane] = wa;
      wsync();
      if (lane < ZS) {
        T v = T(0);
        if (lane < 12) {
          v = S.vec[lane];
          if (lane >= 3 && lane < 6) v = fma(dt, S.vec[lane - 3], v);
          if (lane >= 6 && lane < 9) {
            const double* Mk = S.Mth[k];
            const int cc = lane - 6;
            v += T(Mk[cc]) * S.vec[9] + T(Mk[3 + cc]) * S.vec[10] + T(Mk[6 + cc]) * S.vec[11];
          }
#pragma unroll
          for (int a = 0; a < 12; ++a)
            if ((Sk >> (a / 3)) & 1) v = fma(-Yx[cslot(Sk, a) * 12 + lane], S.hv2[a], v);
        } else {
          const int c = lane - 12;
          if ((Sc >> (c / 3)) & 1) {  // -(Y'w)[12 + c] = 2 Wr_c sum_a Li[a][c] w_a
            const int cp = cslot(Sk, c);
            T acc = T(0);
#pragma unroll
            for (int a = 0; a < 12; ++a)
              if (((Sk >> (a / 3)) & 1) && a >= c) {
                const int apa = cslot(Sk, a);
                acc = fma(F[apa * (apa + 1) / 2 + cp], S.hv2[a], acc);
              }
            v = S.wr2[c] * acc;
          }
        }
        pv = v;
      }
      wsync();
    }
    wsync();
    // forward sweep
    T zv = T(0);
    for (int k = 0; k < N; ++k) {
      const int Sk = S.sb[k];
      const int Sp = k > 0 ? S.sb[k - 1] : 0;
      const int Sc = Sk & Sp;
      const int m = 3 * __popc(Sk);
      const T* F = S.fac + S.foff[k];
      const T* Yx = F + m * (m + 1) / 2;
      if (lane < ZS) S.vec[lane] = zv;
      wsync();
      const bool sa = lane < 12 && ((Sk >> (lane / 3)) & 1);
      const int ap = sa ? cslot(Sk, lane) : 0;
      T ya = T(0);
      if (sa) {
        ya = S.wk[k][lane];
        if (k > 0) {
          const T* Yr = Yx + ap * 12;
#pragma unroll
          for (int j = 0; j < 12; ++j) ya = fma(Yr[j], S.vec[j], ya);
          const T* Lr = F + ap * (ap + 1) / 2;
#pragma unroll
          for (int c = 0; c < 12; ++c)
            if (((Sc >> (c / 3)) & 1) && c <= lane) ya = fma(-S.wr2[c] * Lr[cslot(Sk, c)], S.vec[12 + c], ya);
        }
      }
      if (lane < 12) S.hv[lane] = ya;
      wsync();
      T va = T(0);
      if (sa) {
#pragma unroll
        for (int p = 0; p < 12; ++p)
          if (((Sk >> (p / 3)) & 1) && p >= lane) {
            const int pp = cslot(Sk, p);
            va = fma(-F[pp * (pp + 1) / 2 + ap], S.hv[p], va);
          }
        const int l = lane / 3, d = lane % 3;
        const int t = S.cb[k] / 3 + __popc(Sk & ((1 << l) - 1));
        S.bs[3 * t + d] = va;
      }
      if (lane < 12) S.hv2[lane] = va;
      wsync();
      if (lane < ZS && k + 1 < N) {
        T v;
        if (lane < 12) {
          v = S.vec[lane];
          if (lane < 3) v = fma(dt, S.vec[3 + lane], v);
          if (lane >= 3 && lane < 6) {
            T f = T(0);
#pragma unroll
            for (int l = 0; l < NL; ++l)
              if ((Sk >> l) & 1) f += S.hv2[3 * l + lane - 3];
            v = fma(dtm, f, v);
          }
          if (lane >= 6 && lane < 9) {
            T tq = T(0);
#pragma unroll
            for (int l = 0; l < NL; ++l)
              if ((Sk >> l) & 1) {
                const T rx = T(S.lev[k][l][0]), ry = T(S.lev[k][l][1]), rz = T(S.lev[k][l][2]);
                const T fx = S.hv2[3 * l], fy = S.hv2[3 * l + 1], fz = S.hv2[3 * l + 2];
                tq += lane == 6 ? ry * fz - rz * fy : (lane == 7 ? rz * fx - rx * fz : rx * fy - ry * fx);
              }
            v = fma(dt, tq, v);
          }
          if (lane >= 9) {
            const double* Mk = S.Mth[k];
            const int r = lane - 9;
            v += T(Mk[3 * r]) * S.vec[6] + T(Mk[3 * r + 1]) * S.vec[7] + T(Mk[3 * r + 2]) * S.vec[8];
          }
        } else {
          v = ((Sk >> ((lane - 12) / 3)) & 1) ? S.hv2[lane - 12] : T(0);
        }
        zv = v;
      }
      wsync();
    }
#pragma unroll
    for (int c = 0; c < TPL; ++c)
      if (ton[c]) {
        const int t = lane + 64 * c;
#pragma unroll
        for (int d = 0; d < 3; ++d) bx[c][d] = S.bs[3 * t + d];
      }
    wsync();
  };

  int status = CMPC_MAX_ITER;
  int it = 0;
  T rs_last = T(0), ri_last = T(0), rc_last = T(0);
  T rl[TPL][5], ru[TPL][5], rml[TPL][5], rmu[TPL][5];
  T rg[TPL][3], rhs[TPL][3], du[TPL][3];
  T dtl[TPL][5], dtu[TPL][5], dll[TPL][5], dlu[TPL][5];

  auto direction = [&]() {
#pragma unroll
    for (int c = 0; c < TPL; ++c) {
      T wv[5], ctw[3];
#pragma unroll
      for (int r = 0; r < 5; ++r)
        wv[r] = (rml[c][r] + ll[c][r] * rl[c][r]) * S.itl[r][lane + 64 * c] -
                (rmu[c][r] + lu[c][r] * ru[c][r]) * S.itu[r][lane + 64 * c];
      pyrT(mu_t[c], wv, ctw);
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        rhs[c][d] = ton[c] ? -rg[c][d] - ctw[d] : T(0);
        du[c][d] = rhs[c][d];
      }
    }
    RIC_STAMP(4);
    solve(du);
    RIC_STAMP(3);
#pragma unroll
    for (int c = 0; c < TPL; ++c) {
      T cdu[5];
      pyr(mu_t[c], du[c], cdu);
#pragma unroll
      for (int r = 0; r < 5; ++r) {
        dtl[c][r] = cdu[r] + rl[c][r];
        dtu[c][r] = ru[c][r] - cdu[r];
        dll[c][r] = -(rml[c][r] + ll[c][r] * dtl[c][r]) * S.itl[r][lane + 64 * c];
        dlu[c][r] = -(rmu[c][r] + lu[c][r] * dtu[c][r]) * S.itu[r][lane + 64 * c];
      }
    }
  };
  auto max_step = [&]() -> T {
    MinRatio<T> mr;
#pragma unroll
    for (int c = 0; c < TPL; ++c)
      if (ton[c])
#pragma unroll
        for (int r = 0; r < 5; ++r) {
          mr.cand(tl[c][r], dtl[c][r]);
          mr.cand(tu[c][r], dtu[c][r]);
          mr.cand(ll[c][r], dll[c][r]);
          mr.cand(lu[c][r], dlu[c][r]);
        }
    return wave_min_dpp(mr.value());
  };

  for (it = 0;; ++it) {
    progress_prio(it);
    // ---- residuals
    T rs = T(0), ri = T(0), rc = T(0), ms = T(0);
#pragma unroll
    for (int c = 0; c < TPL; ++c) {
      T cu[5], wl[5], ctw[3];
      pyr(mu_t[c], u[c], cu);
#pragma unroll
      for (int r = 0; r < 5; ++r) {
        const T rlr = ton[c] ? cu[r] - tl[c][r] : T(0);
        const T rur = ton[c] ? ub[r] - cu[r] - tu[c][r] : T(0);
        ri = fmax(ri, fmax(fabs(rlr), fabs(rur)));
        const T cl = tl[c][r] * ll[c][r], ch = tu[c][r] * lu[c][r];
        if (ton[c]) {
          rc = fmax(rc, fmax(cl, ch));
          ms += cl + ch;
        }
        wl[r] = ll[c][r] - lu[c][r];
      }
      pyrT(mu_t[c], wl, ctw);
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        rg[c][d] = ton[c] ? hug[c][d] - ctw[d] : T(0);
        rs = fmax(rs, fabs(rg[c][d]));
      }
    }
    rs_last = rs;
    ri_last = ri;
    rc_last = rc;
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
    if (__all(rs <= T(st.tol_stat) && ri <= T(st.tol_ineq) && rc <= T(st.tol_comp))) {
      status = CMPC_SUCCESS;
      break;
    }
    if (it >= st.iter_max) {
      status = CMPC_MAX_ITER;
      break;
    }
    if (m > 0 && !(mu > T(Lim<T>::mu_min))) {
      status = CMPC_MIN_STEP;
      break;
    }
    // ---- Newton blocks C' diag(lam_l / t_l + lam_u / t_u) C + reg I of every triple
#pragma unroll
    for (int c = 0; c < TPL; ++c) {
      T sg[5];
#pragma unroll
      for (int r = 0; r < 5; ++r) {
        const T itlr = ton[c] ? T(1) / tl[c][r] : T(0);
        const T itur = ton[c] ? T(1) / tu[c][r] : T(0);
        S.itl[r][lane + 64 * c] = itlr;
        S.itu[r][lane + 64 * c] = itur;
        sg[r] = ll[c][r] * itlr + lu[c][r] * itur;
      }
      const T mv = mu_t[c];
      const T reg = T(st.reg_prim);
      if (ton[c]) {
        T* bk = S.blk[lane + 64 * c];
        bk[0] = sg[0] + sg[1] + reg;
        bk[1] = sg[2] + sg[3] + reg;
        bk[2] = mv * mv * (sg[0] + sg[1] + sg[2] + sg[3]) + sg[4] + reg;
        bk[3] = mv * (sg[1] - sg[0]);
        bk[4] = mv * (sg[3] - sg[2]);
      }
    }
    wsync();
    RIC_STAMP(4);
    if (!factor()) {
      status = CMPC_NAN_SOL;
      break;
    }
    RIC_STAMP(2);
    // slack residuals again (not kept across the factorisation: registers)
#pragma unroll
    for (int c = 0; c < TPL; ++c) {
      T cu[5];
      pyr(mu_t[c], u[c], cu);
#pragma unroll
      for (int r = 0; r < 5; ++r) {
        rl[c][r] = ton[c] ? cu[r] - tl[c][r] : T(0);
        ru[c][r] = ton[c] ? ub[r] - cu[r] - tu[c][r] : T(0);
      }
    }
    // ---- predictor (affine scaling)
#pragma unroll
    for (int c = 0; c < TPL; ++c)
#pragma unroll
      for (int r = 0; r < 5; ++r) {
        rml[c][r] = tl[c][r] * ll[c][r];
        rmu[c][r] = tu[c][r] * lu[c][r];
      }
    direction();
    T alpha;
    if (m > 0) {
      alpha = fmin(T(1), max_step());
      T maff = T(0);
#pragma unroll
      for (int c = 0; c < TPL; ++c)
        if (ton[c])
#pragma unroll
          for (int r = 0; r < 5; ++r)
            maff += (tl[c][r] + alpha * dtl[c][r]) * (ll[c][r] + alpha * dll[c][r]) +
                    (tu[c][r] + alpha * dtu[c][r]) * (lu[c][r] + alpha * dlu[c][r]);
      maff = wave_sum_dpp(maff) / T(2 * m);
      const T ratio = maff / mu;
      const T sigma = ratio * ratio * ratio;
      if (st_on && lane == 0) {
        double* sr = st_row();
        sr[0] = (double)alpha;
        sr[1] = (double)maff;
        sr[2] = (double)sigma;
      }
      // ---- corrector
#pragma unroll
      for (int c = 0; c < TPL; ++c)
#pragma unroll
        for (int r = 0; r < 5; ++r) {
          rml[c][r] = ton[c] ? tl[c][r] * ll[c][r] + dtl[c][r] * dll[c][r] - sigma * mu : T(0);
          rmu[c][r] = ton[c] ? tu[c][r] * lu[c][r] + dtu[c][r] * dlu[c][r] - sigma * mu : T(0);
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
    if (alpha < T(st.alpha_min)) {
      status = CMPC_MIN_STEP;
      break;
    }
    // ---- step; H du = rhs - (C' Sigma C + reg I) du keeps H u + g current
#pragma unroll
    for (int c = 0; c < TPL; ++c) {
      const T b[5] = {S.blk[ton[c] ? lane + 64 * c : 0][0], S.blk[ton[c] ? lane + 64 * c : 0][1],
                      S.blk[ton[c] ? lane + 64 * c : 0][2], S.blk[ton[c] ? lane + 64 * c : 0][3],
                      S.blk[ton[c] ? lane + 64 * c : 0][4]};
      const T dd0 = b[0] * du[c][0] + b[3] * du[c][2];
      const T dd1 = b[1] * du[c][1] + b[4] * du[c][2];
      const T dd2 = b[3] * du[c][0] + b[4] * du[c][1] + b[2] * du[c][2];
      const T dd[3] = {dd0, dd1, dd2};
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        u[c][d] = fma(alpha, du[c][d], u[c][d]);
        hug[c][d] = fma(alpha, rhs[c][d] - dd[d], hug[c][d]);
      }
#pragma unroll
      for (int r = 0; r < 5; ++r) {
        tl[c][r] = fma(alpha, dtl[c][r], tl[c][r]);
        tu[c][r] = fma(alpha, dtu[c][r], tu[c][r]);
        ll[c][r] = fma(alpha, dll[c][r], ll[c][r]);
        lu[c][r] = fma(alpha, dlu[c][r], lu[c][r]);
      }
    }
  }

  RIC_STAMP(4);
#ifdef CMPC_RIC_STAMPS
  if (A.stats && lane == 0) {
    double* o = A.stats + (size_t)q * A.stats_cap * CMPC_STAT_COLS;
    for (int k = 0; k < 5; ++k) o[k] = (double)rst_[k];
    o[5] = (double)(ric::memtime() - rst0_);
    o[6] = (double)it;
  }
#endif
  // ---- outputs: condensed u, status, iterations, residuals, (direct) the caller's [N][4][3] forces
  bool fin = true;
#pragma unroll
  for (int c = 0; c < TPL; ++c)
#pragma unroll
    for (int d = 0; d < 3; ++d) fin = fin && isfinite(u[c][d]);
  if (__any(!fin)) status = CMPC_NAN_SOL;
#pragma unroll
  for (int c = 0; c < TPL; ++c) {
    const int t = lane + 64 * c;
    if (A.u_ws && 3 * t < ld)
#pragma unroll
      for (int d = 0; d < 3; ++d)
        if (3 * t + d < ld) A.u_ws[(size_t)q * ld + 3 * t + d] = ton[c] ? u[c][d] : T(0);
  }
  if (lane == 0) {
    A.status[q] = status;
    A.iters[q] = it;
    A.nvar[q] = n;
  }
  if (A.res) {
    const T r0 = wave_max_dpp(rs_last), r1 = wave_max_dpp(ri_last), r2 = wave_max_dpp(rc_last);
    if (lane == 0) {
      double* o = A.res + (size_t)q * 4;
      o[0] = (double)r0;
      o[1] = 0.0;
      o[2] = (double)r1;
      o[3] = (double)r2;
    }
  }
  if (A.out_u) {
    double* uo = A.out_u + (size_t)q * A.out_nu;
    for (int p = lane; p < A.out_nu; p += 64) uo[p] = 0.0;
    __threadfence_block();
    wsync();
#pragma unroll
    for (int c = 0; c < TPL; ++c)
      if (ton[c])
#pragma unroll
        for (int d = 0; d < 3; ++d) uo[(tkv[c] * NL + tlv[c]) * 3 + d] = (double)u[c][d];
    if (lane == 0) {
      A.out_status[q] = status;
      if (A.out_iters) A.out_iters[q] = it;
    }
  }
}

template <typename T, int TPL, int NR, int FS, int WPE>
__global__ __launch_bounds__(64, WPE) void k_ric(RicArgs<T> A) {
  int q = (int)blockIdx.x;
  if (A.qlist) {  // class lists of the fused path: list 1 then list 2; the surplus workgroups exit
    const int c1 = A.qcount[0], c2 = A.qlist2 ? A.qcount[1] : 0;
    if (q < c1) q = A.qlist[q];
    else if (q < c1 + c2) q = A.qlist2[q - c1];
    else return;
    if ((unsigned)q >= gridDim.x) return;
  }
  ric_body<T, TPL, NR, FS>(A, q);
}

}  // namespace cmpc
