/*
 * ocp_ipm.c — CPU restatement of the OCP-QP interior-point method that ocs2::HpipmInterface drives
 * (reference ocs2_sqp/hpipm_catkin/src/HpipmInterface.cpp:166-301; HPIPM d_ocp_qp_ipm_solve, stage-wise Riccati
 * Newton steps, ric_alg = 0 classical recursion, HpipmInterfaceSettings.h:44-57).
 *
 * TEST INFRASTRUCTURE ONLY: the checker of the device solver cmpc_ocp_solve (csrc/k_ocp.hip). Nothing in the product
 * links or calls it. HPIPM@255ffdf is not vendored and cannot be fetched offline: this is the builder's
 * restatement of its published algorithm, pinned by the reference's own constructions (testHpipmInterface.cpp
 * knownSolution :112-152, with_constraints :154-206, noInputs :208-256, retrieveRiccati :258-340) and by a dense
 * full-space KKT solve of each Newton system (tests/test_ocp_ipm.py). Parity against the HPIPM binary is unpinned.
 *
 * Problem (x0 eliminated as HpipmInterface.cpp:177-208 does: node 0 has no state variable):
 *   min  sum_k 1/2 x_k'Q_k x_k + u_k'S_k x_k + 1/2 u_k'R_k u_k + q_k'x_k + r_k'u_k        (x_0 = x0 fixed)
 *   s.t. x_{k+1} = A_k x_k + B_k u_k + b_k                                               k = 0..N-1
 *        lg_k <= C_k x_k + D_k u_k <= ug_k,  lg = ug = -e_k (HpipmInterface.cpp:223-264)  k = 0..N
 * The rows are HPIPM's general constraints: two-sided inequalities with slacks t_l, t_u >= 0 and multipliers
 * l_l, l_u >= 0, so an equality row is an inequality pair of zero width and the IPM honours iter_max / tol_* /
 * alpha_min on it (an inconsistent set of rows ends at MAX_ITER or MIN_STEP, never at a direct-solve verdict).
 *
 * Iteration (identical to oracle_qp_ipm's, cmpc_oracle.c:qp_ipm_run, with the OCP's dynamics multipliers pi_k):
 *   residuals  r_g = [R u + S x + r + B'pi_k - D'(l_l - l_u);  Q x + S'u + q - pi_{k-1} + A'pi_k - C'(l_l - l_u)]
 *              r_b = A x + B u + b - x_{k+1};  r_l = c - lg - t_l,  r_u = ug - c - t_u  (c = C x + D u)
 *   stop       |r_g| <= tol_stat, |r_b| <= tol_eq, |r_l|,|r_u| <= tol_ineq, max t l <= tol_comp (absolute, inf-norm)
 *   Newton     [H + Gc' Sigma Gc + reg I] dz + G' dpi = -(r_g + Gc' w),  G dz = -r_b,
 *              Sigma = l_l / t_l + l_u / t_u, w = (r_ml + l_l r_l) / t_l - (r_mu + l_u r_u) / t_u,
 *              solved stage-wise (backward Riccati, forward rollout), Mehrotra predictor-corrector, one step
 *              length, tau = 0.995, cold start z = 0, pi = 0, t = max(slack, 1), l = mu0 / t.
 * Riccati (per stage, on the barrier-weighted Hessian): Lr Lr' = R~ + B'PB, Ls' = Lr^-1 (S~ + B'PA),
 * P_k = Q~ + A'PA - Ls Ls', K_k = -Lr^-T Ls', and the vector part of each right-hand side.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "cmpc_oracle.h"

#define OCP_THR0 1.0
#define OCP_TAU 0.995
#define CM(M, ld, r, c) ((M)[(size_t)(c) * (ld) + (r)]) /* column-major access */

static inline double dmaxo(double a, double b) { return a > b ? a : b; }
static inline double dmino(double a, double b) { return a < b ? a : b; }

typedef struct ocp_prob {
  int N, nx, nU, m;
  const int *nu, *nc;
  const double *rec, *crec, *x0;
  size_t *oA, *oB, *ob, *oQ, *oS, *oR, *oq, *or_, *oC, *oD, *oe, *oLr, *oLs, *oMi;
  int *cu, *cr;
  double reg;
} ocp_prob;

static void prob_init(ocp_prob* p, int N, int nx, const int* nu, const int* nc, const double* x0, const double* rec,
                      const double* crec, double reg) {
  p->N = N;
  p->nx = nx;
  p->nu = nu;
  p->nc = nc;
  p->x0 = x0;
  p->rec = rec;
  p->crec = crec;
  p->reg = reg;
  const size_t n1 = (size_t)N + 1;
  size_t* buf = (size_t*)calloc(14 * (n1 + 1), sizeof(size_t));
  size_t** dst[] = {&p->oA, &p->oB, &p->ob, &p->oQ, &p->oS, &p->oR, &p->oq, &p->or_, &p->oC, &p->oD, &p->oe,
                    &p->oLr, &p->oLs, &p->oMi};
  for (int i = 0; i < 14; ++i) *dst[i] = buf + (size_t)i * (n1 + 1);
  p->cu = (int*)calloc(2 * (n1 + 1), sizeof(int));
  p->cr = p->cu + n1 + 1;
  size_t o = 0;
  for (int k = 0; k < N; ++k) {
    p->oA[k] = o; o += (size_t)nx * nx;
    p->oB[k] = o; o += (size_t)nx * nu[k];
    p->ob[k] = o; o += (size_t)nx;
  }
  size_t ol = 0, os = 0;
  for (int k = 0; k <= N; ++k) {
    const int m = k < N ? nu[k] : 0;
    p->oQ[k] = o; o += (size_t)nx * nx;
    p->oS[k] = o; o += (size_t)m * nx;
    p->oR[k] = o; o += (size_t)m * m;
    p->oq[k] = o; o += (size_t)nx;
    p->or_[k] = o; o += (size_t)m;
    p->oLr[k] = ol;
    p->oMi[k] = ol;
    ol += (size_t)m * m;
    p->oLs[k] = os;
    os += (size_t)m * nx;
  }
  p->oLr[n1] = ol;
  p->oLs[n1] = os;
  size_t oc = 0;
  int nU = 0, mr = 0;
  for (int k = 0; k <= N; ++k) {
    const int m = k < N ? nu[k] : 0;
    const int r = nc ? nc[k] : 0;
    p->cu[k] = nU;
    nU += m;
    p->cr[k] = mr;
    mr += r;
    p->oC[k] = oc; oc += (size_t)r * nx;
    p->oD[k] = oc; oc += (size_t)r * m;
    p->oe[k] = oc; oc += (size_t)r;
  }
  p->cu[n1] = nU;
  p->cr[n1] = mr;
  p->nU = nU;
  p->m = mr;
}

static void prob_free(ocp_prob* p) {
  free(p->oA);
  free(p->cu);
}

/* c_k = C_k x_k + D_k u_k for every row (x_0 = x0) */
static void rows_eval(const ocp_prob* p, const double* x, const double* u, double* c) {
  for (int k = 0; k <= p->N; ++k) {
    const int r = p->nc ? p->nc[k] : 0, m = k < p->N ? p->nu[k] : 0;
    const double* C = p->crec + p->oC[k];
    const double* D = p->crec + p->oD[k];
    for (int j = 0; j < r; ++j) {
      double s = 0.0;
      for (int i = 0; i < p->nx; ++i) s += CM(C, r, j, i) * x[(size_t)k * p->nx + i];
      for (int i = 0; i < m; ++i) s += CM(D, r, j, i) * u[p->cu[k] + i];
      c[p->cr[k] + j] = s;
    }
  }
}

/* out_k += Gc_k' v (u part into ou, x part into ox), v per row */
static void rows_applyT(const ocp_prob* p, const double* v, double* ou, double* ox) {
  for (int k = 0; k <= p->N; ++k) {
    const int r = p->nc ? p->nc[k] : 0, m = k < p->N ? p->nu[k] : 0;
    const double* C = p->crec + p->oC[k];
    const double* D = p->crec + p->oD[k];
    for (int j = 0; j < r; ++j) {
      const double vj = v[p->cr[k] + j];
      for (int i = 0; i < p->nx; ++i) ox[(size_t)k * p->nx + i] += CM(C, r, j, i) * vj;
      for (int i = 0; i < m; ++i) ou[p->cu[k] + i] += CM(D, r, j, i) * vj;
    }
  }
}

/* Cholesky of a row-major n x n SPD matrix with the IPM pivot guard (cmpc_oracle.c:ipm_cholesky): pivot <= 1e-200
 * -> L_ii = 0, 1/L_ii = 0 (direction dropped). -1 on a NaN pivot. */
static int chol_guard(int n, double* A, double* invd) {
  for (int k = 0; k < n; ++k) {
    double d = A[k * n + k];
    for (int j = 0; j < k; ++j) d -= A[k * n + j] * A[k * n + j];
    if (d != d) return -1;
    const double il = d > 1e-200 ? 1.0 / sqrt(d) : 0.0;
    A[k * n + k] = d > 1e-200 ? sqrt(d) : 0.0;
    invd[k] = il;
    for (int i = k + 1; i < n; ++i) {
      double s = A[i * n + k];
      for (int j = 0; j < k; ++j) s -= A[i * n + j] * A[k * n + j];
      A[i * n + k] = s * il;
    }
    for (int j = k + 1; j < n; ++j) A[k * n + j] = 0.0;
  }
  return 0;
}
static void lsolve(int n, const double* L, const double* invd, double* b) { /* b <- L^-1 b */
  for (int i = 0; i < n; ++i) {
    double s = b[i];
    for (int j = 0; j < i; ++j) s -= L[i * n + j] * b[j];
    b[i] = s * invd[i];
  }
}
static void ltsolve(int n, const double* L, const double* invd, double* b) { /* b <- L^-T b */
  for (int i = n - 1; i >= 0; --i) {
    double s = b[i];
    for (int j = i + 1; j < n; ++j) s -= L[j * n + i] * b[j];
    b[i] = s * invd[i];
  }
}

typedef struct ocp_fact {
  double *P;    /* [(N+1)][nx][nx] row-major */
  double *Lr;   /* per stage nu x nu row-major lower */
  double *iLd;  /* per stage nu: 1 / Lr_ii */
  double *LsT;  /* per stage nu x nx row-major: Lr^-1 (S~ + B'PA) */
  double *p;    /* [(N+1)][nx] vector part of the last solve */
  double *l;    /* [nU] Lr^-1 (gu + B'v) of the last solve */
  double *sig;  /* [m] Sigma the factorisation used */
} ocp_fact;

/* Backward Riccati factorisation of the barrier-weighted Newton matrix (sig per row). 0 ok, -1 NaN pivot. */
static int ocp_factor(const ocp_prob* p, const double* sig, ocp_fact* F, double* wk) {
  const int N = p->N, nx = p->nx;
  double* PA = wk;                   /* nx x nx */
  double* PB = PA + nx * nx;         /* nx x 64 */
  double* Ruu = PB + (size_t)nx * 64; /* 64 x 64 */
  if (sig) memcpy(F->sig, sig, sizeof(double) * (size_t)(p->m ? p->m : 1));
  for (int k = N; k >= 0; --k) {
    const int m = k < N ? p->nu[k] : 0, r = p->nc ? p->nc[k] : 0;
    const double* Q = p->rec + p->oQ[k];
    const double* S = p->rec + p->oS[k];
    const double* R = p->rec + p->oR[k];
    const double* C = p->crec ? p->crec + p->oC[k] : NULL;
    const double* D = p->crec ? p->crec + p->oD[k] : NULL;
    const double* sg = sig + p->cr[k];
    double* Pk = F->P + (size_t)k * nx * nx;
    /* state block Q~ = Q + C' Sigma C + reg I */
    for (int i = 0; i < nx; ++i)
      for (int j = 0; j < nx; ++j) {
        double s = CM(Q, nx, i, j) + (i == j ? p->reg : 0.0);
        for (int t = 0; t < r; ++t) s += CM(C, r, t, i) * sg[t] * CM(C, r, t, j);
        Pk[i * nx + j] = s;
      }
    if (k == N) continue;
    const double* A = p->rec + p->oA[k];
    const double* Bm = p->rec + p->oB[k];
    const double* Pn = F->P + (size_t)(k + 1) * nx * nx;
    for (int i = 0; i < nx; ++i) {
      for (int j = 0; j < nx; ++j) {
        double s = 0.0;
        for (int t = 0; t < nx; ++t) s += Pn[i * nx + t] * CM(A, nx, t, j);
        PA[i * nx + j] = s;
      }
      for (int a = 0; a < m; ++a) {
        double s = 0.0;
        for (int t = 0; t < nx; ++t) s += Pn[i * nx + t] * CM(Bm, nx, t, a);
        PB[i * 64 + a] = s;
      }
    }
    double* Lr = F->Lr + p->oLr[k];
    double* iLd = F->iLd + p->cu[k];
    double* LsT = F->LsT + p->oLs[k];
    for (int a = 0; a < m; ++a) {
      for (int b = 0; b < m; ++b) {
        double s = CM(R, m, a, b) + (a == b ? p->reg : 0.0);
        for (int t = 0; t < r; ++t) s += CM(D, r, t, a) * sg[t] * CM(D, r, t, b);
        for (int t = 0; t < nx; ++t) s += CM(Bm, nx, t, a) * PB[t * 64 + b];
        Ruu[a * m + b] = s;
      }
      for (int j = 0; j < nx; ++j) {
        double s = CM(S, m, a, j);
        for (int t = 0; t < r; ++t) s += CM(D, r, t, a) * sg[t] * CM(C, r, t, j);
        for (int t = 0; t < nx; ++t) s += CM(Bm, nx, t, a) * PA[t * nx + j];
        LsT[a * nx + j] = s;
      }
    }
    memcpy(Lr, Ruu, sizeof(double) * (size_t)m * m);
    if (chol_guard(m, Lr, iLd) != 0) return -1;
    /* LsT <- Lr^-1 Mux, column by column */
    double col[64];
    for (int j = 0; j < nx; ++j) {
      for (int a = 0; a < m; ++a) col[a] = LsT[a * nx + j];
      lsolve(m, Lr, iLd, col);
      for (int a = 0; a < m; ++a) LsT[a * nx + j] = col[a];
    }
    /* P_k = Q~ + A'PA - Ls Ls', from its lower triangle (HPIPM keeps the lower one), mirrored */
    for (int i = 0; i < nx; ++i)
      for (int j = 0; j <= i; ++j) {
        double s = 0.0;
        for (int t = 0; t < nx; ++t) s += CM(A, nx, t, i) * PA[t * nx + j];
        for (int a = 0; a < m; ++a) s -= LsT[a * nx + i] * LsT[a * nx + j];
        Pk[i * nx + j] += s;
        if (j < i) Pk[j * nx + i] = Pk[i * nx + j];
      }
  }
  return 0;
}

/* One Newton solve with the current factorisation: right-hand side (gu, gx) (the step problem's linear term) and
 * dynamics offsets rb (x_0 fixed: dx_0 = 0 when abs == 0). Outputs du, dx (node 0 = 0), dpi; the vector parts in F. */
static void ocp_solve(const ocp_prob* p, ocp_fact* F, const double* gu, const double* gx, const double* rb,
                      double* du, double* dx, double* dpi) {
  const int N = p->N, nx = p->nx;
  double* pv = F->p;
  double v[64], gb[64];
  for (int i = 0; i < nx; ++i) pv[(size_t)N * nx + i] = gx[(size_t)N * nx + i];
  for (int k = N - 1; k >= 0; --k) {
    const int m = p->nu[k];
    const double* A = p->rec + p->oA[k];
    const double* Bm = p->rec + p->oB[k];
    const double* Pn = F->P + (size_t)(k + 1) * nx * nx;
    const double* pn = pv + (size_t)(k + 1) * nx;
    for (int i = 0; i < nx; ++i) {
      double s = pn[i];
      for (int t = 0; t < nx; ++t) s += Pn[i * nx + t] * rb[(size_t)k * nx + t];
      v[i] = s;
    }
    double* l = F->l + p->cu[k];
    for (int a = 0; a < m; ++a) {
      double s = gu[p->cu[k] + a];
      for (int t = 0; t < nx; ++t) s += CM(Bm, nx, t, a) * v[t];
      gb[a] = s;
    }
    memcpy(l, gb, sizeof(double) * (size_t)m);
    lsolve(m, F->Lr + p->oLr[k], F->iLd + p->cu[k], l);
    const double* LsT = F->LsT + p->oLs[k];
    for (int i = 0; i < nx; ++i) {
      double s = gx[(size_t)k * nx + i];
      for (int t = 0; t < nx; ++t) s += CM(A, nx, t, i) * v[t];
      for (int a = 0; a < m; ++a) s -= LsT[a * nx + i] * l[a];
      pv[(size_t)k * nx + i] = s;
    }
  }
  if (!du) return;
  for (int i = 0; i < nx; ++i) dx[i] = 0.0;
  for (int k = 0; k < N; ++k) {
    const int m = p->nu[k];
    const double* A = p->rec + p->oA[k];
    const double* Bm = p->rec + p->oB[k];
    const double* LsT = F->LsT + p->oLs[k];
    double* d = du + p->cu[k];
    for (int a = 0; a < m; ++a) {
      double s = F->l[p->cu[k] + a];
      for (int t = 0; t < nx; ++t) s += LsT[a * nx + t] * dx[(size_t)k * nx + t];
      d[a] = -s;
    }
    ltsolve(m, F->Lr + p->oLr[k], F->iLd + p->cu[k], d);
    for (int i = 0; i < nx; ++i) {
      double s = rb[(size_t)k * nx + i];
      for (int t = 0; t < nx; ++t) s += CM(A, nx, i, t) * dx[(size_t)k * nx + t];
      for (int a = 0; a < m; ++a) s += CM(Bm, nx, i, a) * d[a];
      dx[(size_t)(k + 1) * nx + i] = s;
    }
    const double* Pn = F->P + (size_t)(k + 1) * nx * nx;
    for (int i = 0; i < nx; ++i) {
      double s = pv[(size_t)(k + 1) * nx + i];
      for (int t = 0; t < nx; ++t) s += Pn[i * nx + t] * dx[(size_t)(k + 1) * nx + t];
      dpi[(size_t)k * nx + i] = s;
    }
  }
}

static double* stat_row_ocp(double* stats, int rows, int it) {
  return (stats && it < rows) ? stats + (size_t)it * 10 : NULL;
}

int oracle_ocp_ipm(int N, int nx, const int* nu, const int* nc, const double* x0, const double* rec,
                   const double* crec, const cmpc_settings* s, double* xout, double* uout, int* iters, double* res,
                   oracle_ocp_ric* ric, double* stats, int stats_rows) {
  if (N <= 0 || nx <= 0 || nx > 64) return CMPC_NAN_SOL;
  for (int k = 0; k < N; ++k)
    if (nu[k] < 0 || nu[k] > 64) return CMPC_NAN_SOL;
  ocp_prob p;
  prob_init(&p, N, nx, nu, nc, x0, rec, crec, s->reg_prim);
  const int nU = p.nU, m = p.m;
  const size_t nX = (size_t)(N + 1) * nx, nP = (size_t)N * nx, mm = (size_t)(m ? m : 1);
  const size_t nLr = p.oLr[N + 1] ? p.oLr[N + 1] : 1, nLs = p.oLs[N + 1] ? p.oLs[N + 1] : 1;
  const size_t nUu = (size_t)(nU ? nU : 1);
  size_t tot = nX + nUu + nP          /* x u pi */
               + nUu + nX + nP        /* rgu rgx rb */
               + 16 * mm              /* rows */
               + nUu + nX + nP        /* du dx dpi */
               + nUu + nX             /* gu gx */
               + (size_t)(N + 1) * nx * nx + nLr + nUu + nLs + nX + nUu + mm /* factor */
               + (size_t)nx * nx + (size_t)nx * 64 + 64 * 64; /* factor scratch */
  double* buf = (double*)calloc(tot, sizeof(double));
  double* q = buf;
  double *x = q; q += nX;
  double *u = q; q += nUu;
  double *pi = q; q += nP;
  double *rgu = q; q += nUu;
  double *rgx = q; q += nX;
  double *rb = q; q += nP;
  double *c = q; q += mm;
  double *lg = q; q += mm;
  double *ug = q; q += mm;
  double *tl = q; q += mm;
  double *tu = q; q += mm;
  double *ll = q; q += mm;
  double *lu = q; q += mm;
  double *rl = q; q += mm;
  double *ru = q; q += mm;
  double *rml = q; q += mm;
  double *rmu = q; q += mm;
  double *wv = q; q += mm;
  double *dc = q; q += mm;
  double *dtl = q; q += mm;
  double *dtu = q; q += mm;
  double *dll = q; q += mm;
  double *dlu = q; q += mm;
  double *du = q; q += nUu;
  double *dx = q; q += nX;
  double *dpi = q; q += nP;
  double *gu = q; q += nUu;
  double *gx = q; q += nX;
  ocp_fact F;
  F.P = q; q += (size_t)(N + 1) * nx * nx;
  F.Lr = q; q += nLr;
  F.iLd = q; q += nUu;
  F.LsT = q; q += nLs;
  F.p = q; q += nX;
  F.l = q; q += nUu;
  F.sig = q; q += mm;
  double* wk = q;
  double* sig = dll; /* Sigma is consumed by the factorisation before dll is written */
  /* bounds lg = ug = -e */
  for (int k = 0; k <= N; ++k) {
    const int r = nc ? nc[k] : 0;
    for (int j = 0; j < r; ++j) lg[p.cr[k] + j] = ug[p.cr[k] + j] = -crec[p.oe[k] + j];
  }
  /* cold start: u = 0, x = 0 (node 0 = x0), pi = 0; t = max(slack, THR0), lam = mu0 / t. warm_start != 0 (HPIPM's
   * primal warm start): x (nodes 1..N) and u start from the caller's xout / uout, slacks and multipliers by the
   * same rule from C x + D u */
  if (s->warm_start && xout && uout) {
    memcpy(x + nx, xout + nx, sizeof(double) * (nX - (size_t)nx));
    if (nU) memcpy(u, uout, sizeof(double) * (size_t)nU);
  }
  memcpy(x, x0, sizeof(double) * nx);
  rows_eval(&p, x, u, c);
  for (int j = 0; j < m; ++j) {
    tl[j] = dmaxo(c[j] - lg[j], OCP_THR0);
    tu[j] = dmaxo(ug[j] - c[j], OCP_THR0);
    ll[j] = s->mu0 / tl[j];
    lu[j] = s->mu0 / tu[j];
  }
  int status = CMPC_MAX_ITER, it = 0, factored = 0;
  double rs = 0, re = 0, ri = 0, rc = 0;
  for (it = 0;; ++it) {
    /* --- residuals --- */
    rows_eval(&p, x, u, c);
    for (int k = 0; k <= N; ++k) {
      const int mk = k < N ? nu[k] : 0;
      const double* Q = rec + p.oQ[k];
      const double* S = rec + p.oS[k];
      const double* R = rec + p.oR[k];
      const double* qv = rec + p.oq[k];
      const double* rv = rec + p.or_[k];
      const double* xk = x + (size_t)k * nx;
      for (int a = 0; a < mk; ++a) {
        double sacc = rv[a];
        for (int b = 0; b < mk; ++b) sacc += CM(R, mk, a, b) * u[p.cu[k] + b];
        for (int j = 0; j < nx; ++j) sacc += CM(S, mk, a, j) * xk[j];
        const double* Bm = rec + p.oB[k];
        for (int t = 0; t < nx; ++t) sacc += CM(Bm, nx, t, a) * pi[(size_t)k * nx + t];
        rgu[p.cu[k] + a] = sacc;
      }
      for (int i = 0; i < nx; ++i) {
        if (k == 0) {
          rgx[i] = 0.0;
          continue;
        }
        double sacc = qv[i] - pi[(size_t)(k - 1) * nx + i];
        for (int j = 0; j < nx; ++j) sacc += CM(Q, nx, i, j) * xk[j];
        for (int a = 0; a < mk; ++a) sacc += CM(S, mk, a, i) * u[p.cu[k] + a];
        if (k < N) {
          const double* A = rec + p.oA[k];
          for (int t = 0; t < nx; ++t) sacc += CM(A, nx, t, i) * pi[(size_t)k * nx + t];
        }
        rgx[(size_t)k * nx + i] = sacc;
      }
      if (k < N) {
        const double* A = rec + p.oA[k];
        const double* Bm = rec + p.oB[k];
        const double* bv = rec + p.ob[k];
        for (int i = 0; i < nx; ++i) {
          double sacc = bv[i] - x[(size_t)(k + 1) * nx + i];
          for (int j = 0; j < nx; ++j) sacc += CM(A, nx, i, j) * xk[j];
          for (int a = 0; a < mk; ++a) sacc += CM(Bm, nx, i, a) * u[p.cu[k] + a];
          rb[(size_t)k * nx + i] = sacc;
        }
      }
    }
    for (int j = 0; j < m; ++j) wv[j] = -(ll[j] - lu[j]);
    rows_applyT(&p, wv, rgu, rgx);
    for (int i = 0; i < nx; ++i) rgx[i] = 0.0; /* node 0 has no state variable */
    rs = 0.0;
    re = 0.0;
    ri = 0.0;
    rc = 0.0;
    double musum = 0.0;
    for (int i = 0; i < nU; ++i) rs = dmaxo(rs, fabs(rgu[i]));
    for (size_t i = nx; i < nX; ++i) rs = dmaxo(rs, fabs(rgx[i]));
    for (size_t i = 0; i < nP; ++i) re = dmaxo(re, fabs(rb[i]));
    for (int j = 0; j < m; ++j) {
      rl[j] = c[j] - lg[j] - tl[j];
      ru[j] = ug[j] - c[j] - tu[j];
      ri = dmaxo(ri, dmaxo(fabs(rl[j]), fabs(ru[j])));
      const double cl = tl[j] * ll[j], cu2 = tu[j] * lu[j];
      rc = dmaxo(rc, dmaxo(cl, cu2));
      musum += cl + cu2;
    }
    const double mu = m > 0 ? musum / (2.0 * m) : 0.0;
    double* sr = stat_row_ocp(stats, stats_rows, it);
    if (sr) {
      for (int k = 0; k < 5; ++k) sr[k] = NAN;
      sr[5] = mu;
      sr[6] = rs;
      sr[7] = re;
      sr[8] = ri;
      sr[9] = rc;
    }
    if (!isfinite(rs) || !isfinite(re) || !isfinite(ri) || !isfinite(rc)) {
      status = CMPC_NAN_SOL;
      break;
    }
    if (rs <= s->tol_stat && re <= s->tol_eq && ri <= s->tol_ineq && rc <= s->tol_comp) {
      status = CMPC_SUCCESS;
      break;
    }
    if (it >= s->iter_max) {
      status = CMPC_MAX_ITER;
      break;
    }
    if (m > 0 && !(mu > 1e-300)) {
      status = CMPC_MIN_STEP;
      break;
    }
    /* --- factorisation --- */
    for (int j = 0; j < m; ++j) sig[j] = ll[j] / tl[j] + lu[j] / tu[j];
    if (ocp_factor(&p, sig, &F, wk) != 0) {
      status = CMPC_NAN_SOL;
      break;
    }
    factored = 1;
    /* --- predictor (pass 0), corrector (pass 1) --- */
    double alpha = 1.0;
    for (int pass = 0; pass < 2; ++pass) {
      if (pass == 0) {
        for (int j = 0; j < m; ++j) {
          rml[j] = tl[j] * ll[j];
          rmu[j] = tu[j] * lu[j];
        }
      }
      for (int j = 0; j < m; ++j) wv[j] = (rml[j] + ll[j] * rl[j]) / tl[j] - (rmu[j] + lu[j] * ru[j]) / tu[j];
      memcpy(gu, rgu, sizeof(double) * (size_t)nU);
      memcpy(gx, rgx, sizeof(double) * nX);
      rows_applyT(&p, wv, gu, gx);
      for (int i = 0; i < nx; ++i) gx[i] = 0.0;
      ocp_solve(&p, &F, gu, gx, rb, du, dx, dpi);
      rows_eval(&p, dx, du, dc); /* dx_0 = 0 */
      double amax = 1e300;
      for (int j = 0; j < m; ++j) {
        dtl[j] = dc[j] + rl[j];
        dtu[j] = ru[j] - dc[j];
        dll[j] = -(rml[j] + ll[j] * dtl[j]) / tl[j];
        dlu[j] = -(rmu[j] + lu[j] * dtu[j]) / tu[j];
        if (dtl[j] < 0.0) amax = dmino(amax, -tl[j] / dtl[j]);
        if (dtu[j] < 0.0) amax = dmino(amax, -tu[j] / dtu[j]);
        if (dll[j] < 0.0) amax = dmino(amax, -ll[j] / dll[j]);
        if (dlu[j] < 0.0) amax = dmino(amax, -lu[j] / dlu[j]);
      }
      if (pass == 0) {
        alpha = dmino(1.0, amax);
        if (m == 0) {
          if (sr) sr[3] = sr[4] = alpha;
          break;
        }
        double maff = 0.0;
        for (int j = 0; j < m; ++j)
          maff += (tl[j] + alpha * dtl[j]) * (ll[j] + alpha * dll[j]) + (tu[j] + alpha * dtu[j]) * (lu[j] + alpha * dlu[j]);
        maff /= 2.0 * m;
        const double ratio = maff / mu;
        const double sigma = ratio * ratio * ratio;
        if (sr) {
          sr[0] = alpha;
          sr[1] = maff;
          sr[2] = sigma;
        }
        for (int j = 0; j < m; ++j) {
          rml[j] = tl[j] * ll[j] + dtl[j] * dll[j] - sigma * mu;
          rmu[j] = tu[j] * lu[j] + dtu[j] * dlu[j] - sigma * mu;
        }
      } else {
        alpha = dmino(1.0, OCP_TAU * amax);
        if (sr) sr[3] = sr[4] = alpha;
      }
    }
    if (alpha < s->alpha_min) {
      status = CMPC_MIN_STEP;
      break;
    }
    for (int i = 0; i < nU; ++i) u[i] += alpha * du[i];
    for (size_t i = nx; i < nX; ++i) x[i] += alpha * dx[i];
    for (size_t i = 0; i < nP; ++i) pi[i] += alpha * dpi[i];
    for (int j = 0; j < m; ++j) {
      tl[j] += alpha * dtl[j];
      tu[j] += alpha * dtu[j];
      ll[j] += alpha * dll[j];
      lu[j] += alpha * dlu[j];
    }
  }
  for (size_t i = 0; i < nX; ++i)
    if (!isfinite(x[i])) status = CMPC_NAN_SOL;
  for (int i = 0; i < nU; ++i)
    if (!isfinite(u[i])) status = CMPC_NAN_SOL;
  if (xout) memcpy(xout, x, sizeof(double) * nX);
  if (uout && nU) memcpy(uout, u, sizeof(double) * nU);
  if (iters) *iters = it;
  if (res) {
    res[0] = rs;
    res[1] = re;
    res[2] = ri;
    res[3] = rc;
  }
  /* Riccati quantities (getRiccati*, HpipmInterface.cpp:330-455) at the exit point: the barrier-weighted
   * factorisation with the exit iterate's Sigma = l_l / t_l + l_u / t_u (HPIPM reads ric_* off its last iteration's
   * factorisation; refactorising at the point returned keeps the policy consistent with it), and the vector parts of
   * the Newton step from that point (rows at fixed complementarity: w_r = l_l r_l / t_l - l_u r_u / t_u), which are
   * ~0 at convergence:
   *   K_k = -Lr^-T Ls',  k_k = u_k - K_k x_k + kff_k(step),  p_k = pi_{k-1} - P_k x_k + p_k(step)   (k >= 1),
   * the absolute-form feedforward and cost-to-go gradient of the Newton iterate evaluated without the Sigma-sized
   * cancellations of the absolute recursion (for equality rows Sigma reaches 1e10+). Stage 0 follows the reference's
   * own reconstruction (HpipmInterface.cpp:334-347, 376-389, 416-453) from the stage-0 data (record's A_0, B_0, b_0,
   * Q_0, S_0, R_0, q_0, r_0) and the factor Lr_0, by triangular solves as there:
   *   T1 = Lr_0^-1 (S_0 + B_0'P_1 A_0), v = p_1 + P_1 b_0, t2 = Lr_0^-1 (r_0 + B_0'v), K_0 = -Lr_0^-T T1,
   *   k_0 = -Lr_0^-T t2, P_0 = Q_0 + A_0'P_1 A_0 - T1'T1, p_0 = q_0 + A_0'v - T1't2. */
  (void)factored;
  if (ric && status != CMPC_NAN_SOL) {
    for (int j = 0; j < m; ++j) sig[j] = ll[j] / tl[j] + lu[j] / tu[j];
    if (ocp_factor(&p, sig, &F, wk) != 0) status = CMPC_NAN_SOL;
  }
  if (ric && status != CMPC_NAN_SOL) {
    for (int j = 0; j < m; ++j) wv[j] = ll[j] * rl[j] / tl[j] - lu[j] * ru[j] / tu[j];
    memcpy(gu, rgu, sizeof(double) * (size_t)nU);
    memcpy(gx, rgx, sizeof(double) * nX);
    rows_applyT(&p, wv, gu, gx);
    for (int i = 0; i < nx; ++i) gx[i] = 0.0;
    ocp_solve(&p, &F, gu, gx, rb, du, dx, dpi);
    double col[64];
    for (int k = 0; k < N; ++k) {
      const int mk = nu[k];
      const double* Lr = F.Lr + p.oLr[k];
      const double* iLd = F.iLd + p.cu[k];
      const double* LsT = F.LsT + p.oLs[k];
      double* Kk = ric->K + p.oLs[k];
      for (int j = 0; j < nx; ++j) { /* K = -Lr^-T Ls' */
        for (int a = 0; a < mk; ++a) col[a] = -LsT[a * nx + j];
        ltsolve(mk, Lr, iLd, col);
        for (int a = 0; a < mk; ++a) CM(Kk, mk, a, j) = col[a];
      }
      if (ric->Lr) /* HPIPM's ric_Lr: lower Cholesky factor, column-major out */
        for (int b = 0; b < mk; ++b)
          for (int a = 0; a < mk; ++a) CM(ric->Lr + p.oMi[k], mk, a, b) = Lr[a * mk + b];
      if (k >= 1) {
        for (int a = 0; a < mk; ++a) col[a] = -F.l[p.cu[k] + a];
        ltsolve(mk, Lr, iLd, col); /* step feedforward */
        for (int a = 0; a < mk; ++a) {
          double sacc = u[p.cu[k] + a] + col[a];
          for (int j = 0; j < nx; ++j) sacc -= CM(Kk, mk, a, j) * x[(size_t)k * nx + j];
          ric->k[p.cu[k] + a] = sacc;
        }
      }
    }
    for (int k = 1; k <= N; ++k) {
      const double* Pk = F.P + (size_t)k * nx * nx;
      for (int i = 0; i < nx; ++i) {
        double sacc = pi[(size_t)(k - 1) * nx + i] + F.p[(size_t)k * nx + i];
        for (int j = 0; j < nx; ++j) {
          sacc -= Pk[i * nx + j] * x[(size_t)k * nx + j];
          CM(ric->P + (size_t)k * nx * nx, nx, i, j) = Pk[i * nx + j];
        }
        ric->p[(size_t)k * nx + i] = sacc;
      }
    }
    { /* stage 0, the reference's reconstruction */
      const int m0 = nu[0];
      const double* A = rec + p.oA[0];
      const double* Bm = rec + p.oB[0];
      const double* bv = rec + p.ob[0];
      const double* Q = rec + p.oQ[0];
      const double* S = rec + p.oS[0];
      const double* q0 = rec + p.oq[0];
      const double* r0 = rec + p.or_[0];
      const double* P1 = ric->P + (size_t)nx * nx; /* column-major, symmetric */
      const double* p1 = ric->p + nx;
      double* PA = wk;                       /* nx x nx row-major: P_1 A_0 */
      double* Mux = PA + (size_t)nx * nx;    /* m0 x nx row-major */
      double v[64], gr[64];
      for (int i = 0; i < nx; ++i) {
        for (int j = 0; j < nx; ++j) {
          double sacc = 0.0;
          for (int t = 0; t < nx; ++t) sacc += CM(P1, nx, i, t) * CM(A, nx, t, j);
          PA[i * nx + j] = sacc;
        }
        double sacc = p1[i];
        for (int t = 0; t < nx; ++t) sacc += CM(P1, nx, i, t) * bv[t];
        v[i] = sacc;
      }
      double* T1 = Mux + (size_t)64 * nx; /* m0 x nx row-major: Lr_0^-1 Mux */
      double t2[64];
      for (int a = 0; a < m0; ++a) {
        for (int j = 0; j < nx; ++j) {
          double sacc = CM(S, m0, a, j);
          for (int t = 0; t < nx; ++t) sacc += CM(Bm, nx, t, a) * PA[t * nx + j];
          Mux[a * nx + j] = sacc;
        }
        double sacc = r0[a];
        for (int t = 0; t < nx; ++t) sacc += CM(Bm, nx, t, a) * v[t];
        gr[a] = sacc;
      }
      for (int j = 0; j < nx; ++j) { /* T1 = Lr^-1 Mux, K_0 = -Lr^-T T1 */
        for (int a = 0; a < m0; ++a) col[a] = Mux[a * nx + j];
        lsolve(m0, F.Lr, F.iLd, col);
        for (int a = 0; a < m0; ++a) T1[a * nx + j] = col[a];
        ltsolve(m0, F.Lr, F.iLd, col);
        for (int a = 0; a < m0; ++a) CM(ric->K, m0, a, j) = -col[a];
      }
      for (int a = 0; a < m0; ++a) t2[a] = gr[a];
      lsolve(m0, F.Lr, F.iLd, t2);
      for (int a = 0; a < m0; ++a) col[a] = t2[a];
      ltsolve(m0, F.Lr, F.iLd, col);
      for (int a = 0; a < m0; ++a) ric->k[a] = -col[a];
      for (int i = 0; i < nx; ++i) { /* P_0 = Q_0 + A_0'PA - T1'T1, p_0 = q_0 + A_0'v - T1't2 */
        for (int j = 0; j < nx; ++j) {
          double sacc = CM(Q, nx, i, j);
          for (int t = 0; t < nx; ++t) sacc += CM(A, nx, t, i) * PA[t * nx + j];
          for (int a = 0; a < m0; ++a) sacc -= T1[a * nx + i] * T1[a * nx + j];
          CM(ric->P, nx, i, j) = sacc;
        }
        double sacc = q0[i];
        for (int t = 0; t < nx; ++t) sacc += CM(A, nx, t, i) * v[t];
        for (int a = 0; a < m0; ++a) sacc -= T1[a * nx + i] * t2[a];
        ric->p[i] = sacc;
      }
    }
  }
  free(buf);
  prob_free(&p);
  return status;
}

/* Newton step of the first iteration from the cold start, for pinning the stage-wise solve against a dense KKT solve
 * of the same system (tests/test_ocp_ipm.py): du [nU], dx [(N+1) nx] (node 0 = 0), dpi [N nx]. */
int oracle_ocp_first_step(int N, int nx, const int* nu, const int* nc, const double* x0, const double* rec,
                          const double* crec, const cmpc_settings* s, double* du, double* dx, double* dpi,
                          double* sig_out, double* rhs_u, double* rhs_x, double* rb_out) {
  cmpc_settings s1 = *s;
  s1.iter_max = 1;
  s1.tol_stat = s1.tol_eq = s1.tol_ineq = s1.tol_comp = 0.0;
  ocp_prob p;
  prob_init(&p, N, nx, nu, nc, x0, rec, crec, s->reg_prim);
  const int nU = p.nU, m = p.m;
  const size_t nX = (size_t)(N + 1) * nx, nP = (size_t)N * nx, mm = (size_t)(m ? m : 1);
  const size_t nLr = p.oLr[N + 1] ? p.oLr[N + 1] : 1, nLs = p.oLs[N + 1] ? p.oLs[N + 1] : 1;
  const size_t nUu = (size_t)(nU ? nU : 1);
  double* buf = (double*)calloc(nX + nUu + 10 * mm + nUu + nX + nP + (size_t)(N + 1) * nx * nx + nLr + 2 * nUu +
                                    nLs + nX + mm + (size_t)nx * nx + (size_t)nx * 64 + 64 * 64,
                                sizeof(double));
  double* q = buf;
  double *x = q; q += nX;
  double *u = q; q += nUu;
  double *c = q; q += mm;
  double *tl = q; q += mm;
  double *tu = q; q += mm;
  double *ll = q; q += mm;
  double *lu = q; q += mm;
  double *wv = q; q += mm;
  double *sig = q; q += mm;
  q += 3 * mm;
  double *gu = q; q += nUu;
  double *gx = q; q += nX;
  double *rb = q; q += nP;
  ocp_fact F;
  F.P = q; q += (size_t)(N + 1) * nx * nx;
  F.Lr = q; q += nLr;
  F.iLd = q; q += nUu;
  F.l = q; q += nUu;
  F.LsT = q; q += nLs;
  F.p = q; q += nX;
  F.sig = q; q += mm;
  double* wk = q;
  memcpy(x, x0, sizeof(double) * nx);
  rows_eval(&p, x, u, c);
  for (int k = 0; k <= N; ++k) {
    const int r = nc ? nc[k] : 0;
    for (int j = 0; j < r; ++j) {
      const int jj = p.cr[k] + j;
      const double lgv = -crec[p.oe[k] + j];
      tl[jj] = dmaxo(c[jj] - lgv, OCP_THR0);
      tu[jj] = dmaxo(lgv - c[jj], OCP_THR0);
      ll[jj] = s->mu0 / tl[jj];
      lu[jj] = s->mu0 / tu[jj];
      const double rl = c[jj] - lgv - tl[jj], ru = lgv - c[jj] - tu[jj];
      /* predictor: rm = t lam, so w = lam_l (1 + r_l / t_l) - lam_u (1 + r_u / t_u) */
      wv[jj] = (tl[jj] * ll[jj] + ll[jj] * rl) / tl[jj] - (tu[jj] * lu[jj] + lu[jj] * ru) / tu[jj] - (ll[jj] - lu[jj]);
      sig[jj] = ll[jj] / tl[jj] + lu[jj] / tu[jj];
    }
  }
  /* r_g at z = 0, pi = 0: [r~; q] - Gc'(l_l - l_u); the step's linear term adds Gc' w */
  for (int k = 0; k <= N; ++k) {
    const int mk = k < N ? nu[k] : 0;
    for (int a = 0; a < mk; ++a) {
      double sacc = rec[p.or_[k] + a];
      if (k == 0)
        for (int j = 0; j < nx; ++j) sacc += CM(rec + p.oS[0], mk, a, j) * x0[j];
      gu[p.cu[k] + a] = sacc;
    }
    for (int i = 0; i < nx; ++i) gx[(size_t)k * nx + i] = k == 0 ? 0.0 : rec[p.oq[k] + i];
    if (k < N)
      for (int i = 0; i < nx; ++i) {
        double sacc = rec[p.ob[k] + i];
        if (k == 0)
          for (int j = 0; j < nx; ++j) sacc += CM(rec + p.oA[0], nx, i, j) * x0[j];
        rb[(size_t)k * nx + i] = sacc;
      }
  }
  rows_applyT(&p, wv, gu, gx);
  for (int i = 0; i < nx; ++i) gx[i] = 0.0;
  int st = ocp_factor(&p, sig, &F, wk);
  if (st == 0) ocp_solve(&p, &F, gu, gx, rb, du, dx, dpi);
  if (sig_out && m) memcpy(sig_out, sig, sizeof(double) * m);
  if (rhs_u && nU) memcpy(rhs_u, gu, sizeof(double) * nU);
  if (rhs_x) memcpy(rhs_x, gx, sizeof(double) * nX);
  if (rb_out) memcpy(rb_out, rb, sizeof(double) * nP);
  free(buf);
  prob_free(&p);
  return st;
}

/* Batch over problems with nthreads pthreads (bench.py's OCP cpu_baseline): problem b has x0 + b nx, rec + b rec_size,
 * crec + b crec_size; outputs x [b][(N+1) nx], u [b][nU], status / iters [b]. */
#include <pthread.h>
typedef struct ocp_batch_job {
  int N, nx, B, next_stride;
  const int *nu, *nc;
  const double *x0, *rec, *crec;
  size_t rs, cs;
  const cmpc_settings* s;
  double *x, *u;
  int *status, *iters;
  int nU, b0, b1;
} ocp_batch_job;

static void* ocp_batch_worker(void* arg) {
  ocp_batch_job* j = (ocp_batch_job*)arg;
  for (int b = j->b0; b < j->b1; ++b)
    j->status[b] = oracle_ocp_ipm(j->N, j->nx, j->nu, j->nc, j->x0 + (size_t)b * j->nx, j->rec + (size_t)b * j->rs,
                                  j->crec ? j->crec + (size_t)b * j->cs : NULL, j->s,
                                  j->x + (size_t)b * (j->N + 1) * j->nx, j->u + (size_t)b * (j->nU ? j->nU : 1),
                                  j->iters + b, NULL, NULL, NULL, 0);
  return NULL;
}

int oracle_ocp_ipm_batch(int B, int N, int nx, const int* nu, const int* nc, const double* x0, const double* rec,
                         size_t rec_size, const double* crec, size_t crec_size, const cmpc_settings* s, double* x,
                         double* u, int* status, int* iters, int nthreads) {
  int nU = 0;
  for (int k = 0; k < N; ++k) nU += nu[k];
  if (nthreads < 1) nthreads = 1;
  if (nthreads > B) nthreads = B;
  pthread_t th[256];
  ocp_batch_job jobs[256];
  if (nthreads > 256) nthreads = 256;
  for (int t = 0; t < nthreads; ++t) {
    ocp_batch_job j = {N, nx, B, 0, nu, nc, x0, rec, crec, rec_size, crec_size, s, x, u, status, iters, nU,
                       (int)((long)B * t / nthreads), (int)((long)B * (t + 1) / nthreads)};
    jobs[t] = j;
  }
  if (nthreads == 1) {
    ocp_batch_worker(&jobs[0]);
    return 0;
  }
  for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, ocp_batch_worker, &jobs[t]);
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  return 0;
}
