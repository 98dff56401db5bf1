/*
 * cmpc_oracle.c — CPU fp64 restatement of the reference hot path. TEST INFRASTRUCTURE ONLY (see cmpc_oracle.h).
 *
 * What each function follows in the reference (paths relative to /root/reference):
 *   oracle_consts_init   weights indexing CentroidalMPC.cpp:203-231 (force weights w[9+3L+3i+c], rate w[9+6L+3i+c]),
 *                        CoM-z weight (w2/2)e^{-k}+w2/2 squared by sumsqr (:203-206, :210), force_ub :182-183.
 *   oracle_srbd_dynamics forward-Euler centroidal map CentroidalMPC.cpp:85-92 (gravity :70-73), bilinear lever arm
 *                        linearised at r = p - c^ref, p = oracle_stance_point (:93 pinning, node 0 =
 *                        current foot :165-167, :288-291); Theta/g_z rows are the 13-state extension.
 *   oracle_condense*     multiple shooting of CentroidalMPC.cpp:159-176 eliminated into Aqp/Bqp (App. A.3);
 *                        f^des_z = m*9.81/n_stance with the "mpc table invalid" check CentroidalMPC.cpp:326-335;
 *                        friction pyramid rows CentroidalMPC.cpp:179-201 (swing legs eliminated, App. A.4).
 *   oracle_qp_ipm        primal-dual Mehrotra predictor-corrector with HPIPM's stopping rule and settings
 *                        (HpipmInterfaceSettings.h:44-57; d_ocp_qp_ipm_solve is [external] HPIPM@255ffdf).
 *   oracle_ocp_*         HpipmInterface::Impl::solve x0 elimination HpipmInterface.cpp:177-208; Riccati recursion of
 *                        testHpipmInterface.cpp:280-304.
 */
#include "cmpc_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define NX CMPC_NX
#define NU CMPC_NU
#define GRAV 9.81
#define GAIT_HALF_PERIOD 5
#define THR0 1.0
#define TAU 0.995

static inline double dmin(double a, double b) { return a < b ? a : b; }
static inline double dmax(double a, double b) { return a > b ? a : b; }

/* ------------------------------------------------------------------------------------------------ model */

void oracle_consts_init(const cmpc_model* m, oracle_consts* c) {
  memset(c, 0, sizeof(*c));
  const int L = m->n_legs;
  const double* w = m->weights;
  c->N = m->N;
  c->L = L;
  c->mass = m->mass;
  c->dt = m->dt;
  for (int i = 0; i < L; ++i) {
    c->mu[i] = m->mu[i];
    for (int d = 0; d < 3; ++d) {
      c->Wf[3 * i + d] = w[9 + 3 * L + 3 * i + d];
      c->Wr[3 * i + d] = w[9 + 6 * L + 3 * i + d];
      c->Wp[3 * i + d] = w[9 + 3 * i + d];
    }
  }
  for (int k = 0; k <= m->N && k < 64; ++k) {
    const double wz = (w[2] / 2.0) * exp(-(double)k) + w[2] / 2.0;
    double* q = c->qdiag[k];
    q[0] = 2.0 * w[0];
    q[1] = 2.0 * w[1];
    q[2] = 2.0 * (wz * wz);
    for (int j = 3; j < 9; ++j) q[j] = 2.0 * w[j];
    for (int j = 0; j < 3; ++j) q[9 + j] = 2.0 * m->theta_weights[j];
    q[12] = 0.0;
  }
  for (int j = 0; j < 5; ++j) c->force_ub[j] = m->force_ub[j];
  /* inverse of the body inertia (adjugate / determinant) */
  const double* I = m->inertia;
  const double a00 = I[4] * I[8] - I[5] * I[7], a01 = I[2] * I[7] - I[1] * I[8], a02 = I[1] * I[5] - I[2] * I[4];
  const double a10 = I[5] * I[6] - I[3] * I[8], a11 = I[0] * I[8] - I[2] * I[6], a12 = I[2] * I[3] - I[0] * I[5];
  const double a20 = I[3] * I[7] - I[4] * I[6], a21 = I[1] * I[6] - I[0] * I[7], a22 = I[0] * I[4] - I[1] * I[3];
  const double det = I[0] * a00 + I[1] * a10 + I[2] * a20;
  const double id = 1.0 / det;
  double* R = c->inv_inertia;
  R[0] = a00 * id; R[1] = a01 * id; R[2] = a02 * id;
  R[3] = a10 * id; R[4] = a11 * id; R[5] = a12 * id;
  R[6] = a20 * id; R[7] = a21 * id; R[8] = a22 * id;
}

/* Stance foot position of leg i at step k (the reference's foot_pos[i] node k). A stance foot does not move
 * (foot_pos+ = foot_pos + (1 - e) foot_vel dt, CentroidalMPC.cpp:93): one position holds over a stance run's nodes
 * s..e+1. Record node 0 is the current foot position (state[9+3i..], :288-291), to which foot_pos(:,0) is pinned
 * (:165-167), so a run starting at step 0 stays there. A later run (after a swing step) is frozen at the mean of
 * des_foot_pos over nodes s..e+1 (minimiser of the w9..w20 foot tracking cost :218-221 under the pinning), formed as
 * p_s + sum_j (p_j - p_s) / cnt. Same operations as the device's stance_point (cmpc_device.hpp). */
void oracle_stance_point(const double* foot, const uint8_t* contact, int N, int L, int k, int i, double p[3]) {
  int s = k;
  while (s > 0 && contact[(s - 1) * L + i]) --s;
  const double* ps = foot + ((size_t)s * L + i) * 3;
  p[0] = ps[0];
  p[1] = ps[1];
  p[2] = ps[2];
  if (s == 0) return;
  int e = k;
  while (e + 1 < N && contact[(e + 1) * L + i]) ++e;
  double d0 = 0.0, d1 = 0.0, d2 = 0.0;
  for (int j = s + 1; j <= e + 1; ++j) {
    const double* pj = foot + ((size_t)j * L + i) * 3;
    d0 += pj[0] - p[0];
    d1 += pj[1] - p[1];
    d2 += pj[2] - p[2];
  }
  const double cnt = (double)(e + 2 - s);
  p[0] += d0 / cnt;
  p[1] += d1 / cnt;
  p[2] += d2 / cnt;
}

void oracle_stance_feet(int N, int L, const double* foot, const uint8_t* contact, double* out) {
  memset(out, 0, sizeof(double) * (size_t)N * L * 3);
  for (int k = 0; k < N; ++k)
    for (int i = 0; i < L; ++i)
      if (contact[k * L + i]) oracle_stance_point(foot, contact, N, L, k, i, out + ((size_t)k * L + i) * 3);
}

void oracle_srbd_dynamics(const oracle_consts* c, const double* xref, const double* foot, const uint8_t* contact,
                          double* A, double* B) {
  oracle_srbd_dynamics_lin(c, xref, foot, contact, NULL, A, B, NULL);
}

/* lin [N][6] = (c_bar_k, F_bar_k): Taylor expansion of the bilinear dt sum_i e_ik (p_ik - c_k) x f_ik
 * (CentroidalMPC.cpp:86) at (c_bar, f_bar): lever arm p_ik - c_bar_k, A_k gains dt [F_bar_k]x in the L rows / c
 * columns, affine term b_k = -dt F_bar_k x c_bar_k. lin = NULL: (c_ref_k, 0), b = 0. b [N][13] may be NULL. */
void oracle_srbd_dynamics_lin(const oracle_consts* c, const double* xref, const double* foot, const uint8_t* contact,
                              const double* lin, double* A, double* B, double* b) {
  const int N = c->N, L = c->L;
  const double dt = c->dt;
  for (int k = 0; k < N; ++k) {
    if (b) {
      memset(b + (size_t)k * NX, 0, sizeof(double) * NX);
      if (lin) {
        const double* lk = lin + (size_t)k * 6;
        b[k * NX + 6] = -dt * (lk[4] * lk[2] - lk[5] * lk[1]);
        b[k * NX + 7] = -dt * (lk[5] * lk[0] - lk[3] * lk[2]);
        b[k * NX + 8] = -dt * (lk[3] * lk[1] - lk[4] * lk[0]);
      }
    }
    double* Ak = A + (size_t)k * NX * NX;
    double* Bk = B + (size_t)k * NX * NU;
    memset(Ak, 0, sizeof(double) * NX * NX);
    memset(Bk, 0, sizeof(double) * NX * NU);
    for (int i = 0; i < NX; ++i) Ak[i * NX + i] = 1.0;
    /* c+ = c + dt v */
    for (int d = 0; d < 3; ++d) Ak[d * NX + 3 + d] = dt;
    /* v_z+ = v_z + dt g_z */
    Ak[5 * NX + 12] = dt;
    /* Theta+ = Theta + dt * I_b^{-1} R_z(psi)^T L */
    const double psi = xref[k * NX + 11];
    const double cp = cos(psi), sp = sin(psi);
    const double RzT[9] = {cp, sp, 0.0, -sp, cp, 0.0, 0.0, 0.0, 1.0};
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) {
        double s = 0.0;
        for (int e = 0; e < 3; ++e) s += c->inv_inertia[a * 3 + e] * RzT[e * 3 + b];
        Ak[(9 + a) * NX + 6 + b] = dt * s;
      }
    if (lin) { /* L+ += dt [F_bar]x c */
      const double* F = lin + (size_t)k * 6 + 3;
      const double SF[9] = {0.0, -F[2], F[1], F[2], 0.0, -F[0], -F[1], F[0], 0.0};
      for (int a2 = 0; a2 < 3; ++a2)
        for (int b2 = 0; b2 < 3; ++b2) Ak[(6 + a2) * NX + b2] = dt * SF[a2 * 3 + b2];
    }
    /* inputs: v+ += dt/m f_i, L+ += dt [r_ik]x f_i for stance legs */
    const double* cb = lin ? lin + (size_t)k * 6 : xref + (size_t)k * NX;
    for (int i = 0; i < L; ++i) {
      if (!contact[k * L + i]) continue;
      double p[3];
      oracle_stance_point(foot, contact, N, L, k, i, p);
      const double rx = p[0] - cb[0], ry = p[1] - cb[1], rz = p[2] - cb[2];
      const double S[9] = {0.0, -rz, ry, rz, 0.0, -rx, -ry, rx, 0.0};
      for (int d = 0; d < 3; ++d) Bk[(3 + d) * NU + 3 * i + d] = dt / c->mass;
      for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) Bk[(6 + a) * NU + 3 * i + b] = dt * S[a * 3 + b];
    }
  }
}

static int fdes_and_check(const oracle_consts* c, const uint8_t* contact, double* fdes_z /* [N][L] */) {
  const int N = c->N, L = c->L;
  for (int k = 0; k < N; ++k) {
    int ns = 0;
    for (int i = 0; i < L; ++i) ns += contact[k * L + i] ? 1 : 0;
    if (ns <= 0) return CMPC_INVALID_CONTACT;
    for (int i = 0; i < L; ++i) fdes_z[k * L + i] = contact[k * L + i] ? c->mass * GRAV / (double)ns : 0.0;
  }
  return CMPC_SUCCESS;
}

int oracle_condense_full(const oracle_consts* c, const double* x0, const double* xref, const double* foot,
                         const uint8_t* contact, double* H, double* g) {
  return oracle_condense_full_lin(c, x0, xref, foot, contact, NULL, H, g);
}

int oracle_condense_full_lin(const oracle_consts* c, const double* x0, const double* xref, const double* foot,
                             const uint8_t* contact, const double* lin, double* H, double* g) {
  const int N = c->N, L = c->L, n = NU * N;
  double* fdes = (double*)malloc(sizeof(double) * N * L);
  const int st = fdes_and_check(c, contact, fdes);
  if (st != CMPC_SUCCESS) {
    free(fdes);
    return st;
  }
  double* A = (double*)malloc(sizeof(double) * N * NX * NX);
  double* B = (double*)malloc(sizeof(double) * N * NX * NU);
  double* bb = (double*)malloc(sizeof(double) * N * NX);
  oracle_srbd_dynamics_lin(c, xref, foot, contact, lin, A, B, bb);
  double* G = (double*)calloc((size_t)NX * n, sizeof(double));  /* block row of Bqp for x_k: 13 x 12N */
  double* G2 = (double*)malloc(sizeof(double) * NX * n);
  double xh[NX], xh2[NX], e[NX];
  memcpy(xh, x0, sizeof(xh));
  memset(H, 0, sizeof(double) * n * n);
  memset(g, 0, sizeof(double) * n);
  for (int k = 0; k < N; ++k) {
    const double* Ak = A + (size_t)k * NX * NX;
    const double* Bk = B + (size_t)k * NX * NU;
    /* G <- A_k G + [B_k at columns of step k]; xh <- A_k xh (free response, Aqp x0) */
    for (int r = 0; r < NX; ++r) {
      for (int j = 0; j < n; ++j) {
        double s = 0.0;
        for (int t = 0; t < NX; ++t) s += Ak[r * NX + t] * G[t * n + j];
        G2[r * n + j] = s;
      }
      for (int j = 0; j < NU; ++j) G2[r * n + NU * k + j] += Bk[r * NU + j];
      double s = 0.0;
      for (int t = 0; t < NX; ++t) s += Ak[r * NX + t] * xh[t];
      xh2[r] = s + bb[k * NX + r];
    }
    memcpy(G, G2, sizeof(double) * NX * n);
    memcpy(xh, xh2, sizeof(xh));
    /* node k+1 cost: H += G' Q G, g += G' Q (xh - xref) */
    const double* q = c->qdiag[k + 1];
    for (int r = 0; r < NX; ++r) e[r] = q[r] * (xh[r] - xref[(k + 1) * NX + r]);
    for (int a = 0; a < n; ++a) {
      double ga = 0.0;
      for (int r = 0; r < NX; ++r) ga += G[r * n + a] * e[r];
      g[a] += ga;
      for (int b = 0; b <= a; ++b) {
        double s = 0.0;
        for (int r = 0; r < NX; ++r) s += G[r * n + a] * q[r] * G[r * n + b];
        H[a * n + b] += s;
      }
    }
  }
  for (int a = 0; a < n; ++a)
    for (int b = a + 1; b < n; ++b) H[a * n + b] = H[b * n + a];
  /* R-bar: force tracking + force-rate (block tridiagonal), r-bar = -2 W_f f^des */
  for (int k = 0; k < N; ++k)
    for (int j = 0; j < NU; ++j) {
      const int idx = NU * k + j;
      const int nb = (k > 0) + (k < N - 1);
      H[idx * n + idx] += 2.0 * c->Wf[j] + 2.0 * c->Wr[j] * (double)nb;
      if (k < N - 1) {
        H[idx * n + idx + NU] += -2.0 * c->Wr[j];
        H[(idx + NU) * n + idx] += -2.0 * c->Wr[j];
      }
      if (j % 3 == 2) g[idx] += -2.0 * c->Wf[j] * fdes[k * L + j / 3];
    }
  free(fdes);
  free(A);
  free(B);
  free(bb);
  free(G);
  free(G2);
  return CMPC_SUCCESS;
}

int oracle_condense(const oracle_consts* c, const double* x0, const double* xref, const double* foot,
                    const uint8_t* contact, int ld, int* n_out, double* H, double* g, double* tri_mu, double* tri_lo,
                    double* tri_hi, int* tri_map) {
  return oracle_condense_lin(c, x0, xref, foot, contact, NULL, ld, n_out, H, g, tri_mu, tri_lo, tri_hi, tri_map);
}

int oracle_condense_lin(const oracle_consts* c, const double* x0, const double* xref, const double* foot,
                        const uint8_t* contact, const double* lin, int ld, int* n_out, double* H, double* g,
                        double* tri_mu, double* tri_lo, double* tri_hi, int* tri_map) {
  const int N = c->N, L = c->L, nf = NU * N;
  *n_out = 0;
  int idx[NU * 64];
  int nt = 0;
  for (int k = 0; k < N; ++k)
    for (int i = 0; i < L; ++i)
      if (contact[k * L + i]) {
        if (tri_map) tri_map[nt] = k * L + i;
        idx[nt++] = NU * k + 3 * i;
      }
  const int n = 3 * nt;
  {
    int ns_ok = 1;
    for (int k = 0; k < N; ++k) {
      int ns = 0;
      for (int i = 0; i < L; ++i) ns += contact[k * L + i] ? 1 : 0;
      if (ns == 0) ns_ok = 0;
    }
    if (!ns_ok) return CMPC_INVALID_CONTACT;
  }
  if (n > ld) return CMPC_TOO_LARGE;
  double* Hf = (double*)malloc(sizeof(double) * nf * nf);
  double* gf = (double*)malloc(sizeof(double) * nf);
  const int st = oracle_condense_full_lin(c, x0, xref, foot, contact, lin, Hf, gf);
  if (st != CMPC_SUCCESS) {
    free(Hf);
    free(gf);
    return st;
  }
  for (int a = 0; a < ld; ++a) {
    for (int b = 0; b < ld; ++b) {
      double v;
      if (a < n && b < n)
        v = Hf[(idx[a / 3] + a % 3) * nf + idx[b / 3] + b % 3];
      else
        v = (a == b) ? 1.0 : 0.0;
      H[(size_t)a * ld + b] = v;
    }
    g[a] = a < n ? gf[idx[a / 3] + a % 3] : 0.0;
  }
  for (int t = 0; t < ld / 3; ++t) {
    const int leg = t < nt ? (tri_map ? tri_map[t] % L : 0) : 0;
    if (tri_mu) tri_mu[t] = t < nt ? c->mu[leg] : 0.0;
    for (int r = 0; r < 5; ++r) {
      if (tri_lo) tri_lo[t * 5 + r] = 0.0;
      if (tri_hi) tri_hi[t * 5 + r] = c->force_ub[r];
    }
  }
  if (tri_mu && !tri_map) {
    /* recompute leg of each triple when no map was requested */
    int t = 0;
    for (int k = 0; k < N; ++k)
      for (int i = 0; i < L; ++i)
        if (contact[k * L + i]) tri_mu[t++] = c->mu[i];
  }
  *n_out = n;
  free(Hf);
  free(gf);
  return CMPC_SUCCESS;
}

/* ------------------------------------------------------------------------------------------------ dense LA */

int oracle_cholesky(int n, double* A, int lda) {
  for (int k = 0; k < n; ++k) {
    double d = A[k * lda + k];
    for (int j = 0; j < k; ++j) d -= A[k * lda + j] * A[k * lda + j];
    if (!(d > 0.0)) return -1;
    const double l = sqrt(d);
    A[k * lda + k] = l;
    for (int i = k + 1; i < n; ++i) {
      double s = A[i * lda + k];
      for (int j = 0; j < k; ++j) s -= A[i * lda + j] * A[k * lda + j];
      A[i * lda + k] = s / l;
    }
  }
  return 0;
}

void oracle_chol_solve(int n, const double* Lm, int lda, double* b) {
  for (int i = 0; i < n; ++i) {
    double s = b[i];
    for (int j = 0; j < i; ++j) s -= Lm[i * lda + j] * b[j];
    b[i] = s / Lm[i * lda + i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = b[i];
    for (int j = i + 1; j < n; ++j) s -= Lm[j * lda + i] * b[j];
    b[i] = s / Lm[i * lda + i];
  }
}

/* ------------------------------------------------------------------------------------------------ IPM */

/* friction pyramid F(mu) rows (CentroidalMPC.cpp:186-190) applied to one force triple */
static inline void pyr_apply(double mu, const double* f, double* c5) {
  c5[0] = -f[0] + mu * f[2];
  c5[1] = f[0] + mu * f[2];
  c5[2] = -f[1] + mu * f[2];
  c5[3] = f[1] + mu * f[2];
  c5[4] = f[2];
}
static inline void pyr_applyT(double mu, const double* w, double* f) {
  f[0] = -w[0] + w[1];
  f[1] = -w[2] + w[3];
  f[2] = mu * (w[0] + w[1] + w[2] + w[3]) + w[4];
}

/* The two operations the IPM needs from the QP's Hessian: the gradient H u + g, and solves with the Newton matrix
 * H + C' Sigma C + reg I. Dense (oracle_qp_ipm: Cholesky of the condensed H) or structured (oracle_riccati_solve_one:
 * rollout / adjoint and a Riccati recursion over the stages, HPIPM's approach); the iteration itself is shared. */
typedef struct qp_ops {
  void* ctx;
  void (*grad)(void* ctx, const double* u, double* hug);
  int (*factor)(void* ctx, int nt, const double* tri_mu, const double* ll, const double* lu, const double* tl,
                const double* tu, double reg);
  void (*solve)(void* ctx, double* b);
} qp_ops;

typedef struct ipm_ws {
  double *invd, *K, *rg, *rhs, *du, *cu, *cdu, *tl, *tu, *ll, *lu, *rl, *ru, *dtl, *dtu, *dll, *dlu, *rml, *rmu, *w;
} ipm_ws;

/* Cholesky with the kernels' pivot guard: a pivot <= 1e-200 gets inverse 0 (direction dropped, BLASFEO-style).
 * Stores 1/L_ii in invd. Returns -1 only on a NaN pivot. */
static int ipm_cholesky(int n, double* A, double* invd) {
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
  }
  return 0;
}
static void ipm_chol_solve(int n, const double* Lm, const double* invd, double* b) {
  for (int i = 0; i < n; ++i) {
    double s = b[i];
    for (int j = 0; j < i; ++j) s -= Lm[i * n + j] * b[j];
    b[i] = s * invd[i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = b[i];
    for (int j = i + 1; j < n; ++j) s -= Lm[j * n + i] * b[j];
    b[i] = s * invd[i];
  }
}

static void ipm_dir(int n, const qp_ops* ops, int nt, const double* tri_mu, ipm_ws* W) {
  const int m = 5 * nt;
  for (int j = 0; j < m; ++j)
    W->w[j] = (W->rml[j] + W->ll[j] * W->rl[j]) / W->tl[j] - (W->rmu[j] + W->lu[j] * W->ru[j]) / W->tu[j];
  for (int i = 0; i < n; ++i) W->rhs[i] = -W->rg[i];
  for (int t = 0; t < nt; ++t) {
    double f[3];
    pyr_applyT(tri_mu[t], W->w + 5 * t, f);
    for (int d = 0; d < 3; ++d) W->rhs[3 * t + d] -= f[d];
  }
  memcpy(W->du, W->rhs, sizeof(double) * n);
  ops->solve(ops->ctx, W->du);
  for (int t = 0; t < nt; ++t) pyr_apply(tri_mu[t], W->du + 3 * t, W->cdu + 5 * t);
  for (int j = 0; j < m; ++j) {
    W->dtl[j] = W->cdu[j] + W->rl[j];
    W->dtu[j] = W->ru[j] - W->cdu[j];
    W->dll[j] = -(W->rml[j] + W->ll[j] * W->dtl[j]) / W->tl[j];
    W->dlu[j] = -(W->rmu[j] + W->lu[j] * W->dtu[j]) / W->tu[j];
  }
}

static double ipm_maxstep(int m, const ipm_ws* W) {
  double a = 1e300;
  for (int j = 0; j < m; ++j) {
    if (W->dtl[j] < 0.0) a = dmin(a, -W->tl[j] / W->dtl[j]);
    if (W->dtu[j] < 0.0) a = dmin(a, -W->tu[j] / W->dtu[j]);
    if (W->dll[j] < 0.0) a = dmin(a, -W->ll[j] / W->dll[j]);
    if (W->dlu[j] < 0.0) a = dmin(a, -W->lu[j] / W->dlu[j]);
  }
  return a;
}

typedef struct dense_ops_ctx {
  int n, ld;
  const double *H, *g;
  double *K, *invd;
} dense_ops_ctx;

static void dense_grad(void* vc, const double* u, double* hug) {
  const dense_ops_ctx* d = (const dense_ops_ctx*)vc;
  for (int i = 0; i < d->n; ++i) {
    double acc = 0.0;
    for (int j = 0; j < d->n; ++j) acc += d->H[(size_t)i * d->ld + j] * u[j];
    hug[i] = acc + d->g[i];
  }
}

/* Newton matrix K = H + C' diag(lam/t) C + reg I, Cholesky */
static int dense_factor(void* vc, int nt, const double* tri_mu, const double* lla, const double* lua,
                        const double* tla, const double* tua, double reg) {
  dense_ops_ctx* d = (dense_ops_ctx*)vc;
  const int n = d->n;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) d->K[i * n + j] = d->H[(size_t)i * d->ld + j];
  for (int t = 0; t < nt; ++t) {
    const double* ll = lla + 5 * t;
    const double* lu = lua + 5 * t;
    const double* tl = tla + 5 * t;
    const double* tu = tua + 5 * t;
    double sg[5];
    for (int r = 0; r < 5; ++r) sg[r] = ll[r] / tl[r] + lu[r] / tu[r];
    const double mu_t = tri_mu[t];
    const int b = 3 * t;
    d->K[b * n + b] += sg[0] + sg[1];
    d->K[(b + 1) * n + b + 1] += sg[2] + sg[3];
    d->K[(b + 2) * n + b + 2] += mu_t * mu_t * (sg[0] + sg[1] + sg[2] + sg[3]) + sg[4];
    const double xz = mu_t * (-sg[0] + sg[1]), yz = mu_t * (-sg[2] + sg[3]);
    d->K[b * n + b + 2] += xz;
    d->K[(b + 2) * n + b] += xz;
    d->K[(b + 1) * n + b + 2] += yz;
    d->K[(b + 2) * n + b + 1] += yz;
  }
  for (int i = 0; i < n; ++i) d->K[i * n + i] += reg;
  return ipm_cholesky(n, d->K, d->invd);
}

static void dense_solve(void* vc, double* b) {
  const dense_ops_ctx* d = (const dense_ops_ctx*)vc;
  ipm_chol_solve(d->n, d->K, d->invd, b);
}

static int qp_ipm_run(int n, const qp_ops* ops, const double* tri_mu, const double* tri_lo, const double* tri_hi,
                      const cmpc_settings* s, double* u, double* lam_lo, double* lam_hi, int* iters, double* res,
                      double* stats, int stats_rows);

int oracle_qp_ipm(int n, int ld, const double* H, const double* g, const double* tri_mu, const double* tri_lo,
                  const double* tri_hi, const cmpc_settings* s, double* u, double* lam_lo, double* lam_hi, int* iters,
                  double* res) {
  return oracle_qp_ipm_stats(n, ld, H, g, tri_mu, tri_lo, tri_hi, s, u, lam_lo, lam_hi, iters, res, NULL, 0);
}

int oracle_qp_ipm_stats(int n, int ld, const double* H, const double* g, const double* tri_mu, const double* tri_lo,
                        const double* tri_hi, const cmpc_settings* s, double* u, double* lam_lo, double* lam_hi,
                        int* iters, double* res, double* stats, int stats_rows) {
  double* buf = (double*)calloc((size_t)n * n + (size_t)n + 1, sizeof(double));
  dense_ops_ctx d = {n, ld, H, g, buf, buf + (size_t)n * n};
  qp_ops ops = {&d, dense_grad, dense_factor, dense_solve};
  const int st = qp_ipm_run(n, &ops, tri_mu, tri_lo, tri_hi, s, u, lam_lo, lam_hi, iters, res, stats, stats_rows);
  free(buf);
  return st;
}

/* Per-iteration statistics row (cmpc_enable_stats; the columns of HPIPM's stat table, HpipmInterface.cpp:476-502):
 * alpha_aff, mu_aff, sigma, alpha_prim, alpha_dual, mu, res_stat, res_eq, res_ineq, res_comp; NaN for no step. */
static double* stat_row(double* stats, int rows, int it) { return (stats && it < rows) ? stats + (size_t)it * 10 : NULL; }

static int qp_ipm_run(int n, const qp_ops* ops, const double* tri_mu, const double* tri_lo, const double* tri_hi,
                      const cmpc_settings* s, double* u, double* lam_lo, double* lam_hi, int* iters, double* res,
                      double* stats, int stats_rows) {
  const int nt = n / 3, m = 5 * nt;
  ipm_ws W;
  double* buf = (double*)calloc(4 * (size_t)n + 1 + 15 * (size_t)(m + 1), sizeof(double));
  double* p = buf;
  W.K = NULL;
  W.invd = NULL;
  W.rg = p; p += n;
  W.rhs = p; p += n;
  W.du = p; p += n;
  double* hu = p; p += n;
  double** mv[] = {&W.cu, &W.cdu, &W.tl, &W.tu, &W.ll, &W.lu, &W.rl, &W.ru, &W.dtl, &W.dtu, &W.dll, &W.dlu,
                   &W.rml, &W.rmu, &W.w};
  for (int i = 0; i < 15; ++i) {
    *mv[i] = p;
    p += m + 1;
  }
  /* cold start (warm_start = 0): u = 0; warm start (HPIPM warm_start = 1, primal): u as given on entry.
   * Then slacks of C u clipped at THR0, lam = mu0 / t */
  if (!s->warm_start)
    for (int i = 0; i < n; ++i) u[i] = 0.0;
  for (int t = 0; t < nt; ++t) pyr_apply(tri_mu[t], u + 3 * t, W.cu + 5 * t);
  for (int j = 0; j < m; ++j) {
    W.tl[j] = dmax(W.cu[j] - tri_lo[j], THR0);
    W.tu[j] = dmax(tri_hi[j] - W.cu[j], THR0);
    W.ll[j] = s->mu0 / W.tl[j];
    W.lu[j] = s->mu0 / W.tu[j];
  }
  int status = CMPC_MAX_ITER, it = 0;
  double rs = 0, ri = 0, rc = 0;
  for (it = 0;; ++it) {
    /* residuals */
    for (int t = 0; t < nt; ++t) pyr_apply(tri_mu[t], u + 3 * t, W.cu + 5 * t);
    ops->grad(ops->ctx, u, hu); /* H u + g */
    for (int j = 0; j < m; ++j) W.w[j] = W.ll[j] - W.lu[j];
    for (int t = 0; t < nt; ++t) {
      double f[3];
      pyr_applyT(tri_mu[t], W.w + 5 * t, f);
      for (int d = 0; d < 3; ++d) W.rg[3 * t + d] = hu[3 * t + d] - f[d];
    }
    double musum = 0.0;
    rs = 0.0;
    ri = 0.0;
    rc = 0.0;
    for (int i = 0; i < n; ++i) rs = dmax(rs, fabs(W.rg[i]));
    for (int j = 0; j < m; ++j) {
      W.rl[j] = W.cu[j] - tri_lo[j] - W.tl[j];
      W.ru[j] = tri_hi[j] - W.cu[j] - W.tu[j];
      ri = dmax(ri, dmax(fabs(W.rl[j]), fabs(W.ru[j])));
      const double cl = W.tl[j] * W.ll[j], cu = W.tu[j] * W.lu[j];
      rc = dmax(rc, dmax(cl, cu));
      musum += cl + cu;
    }
    const double mu = m > 0 ? musum / (2.0 * m) : 0.0;
    double* sr = stat_row(stats, stats_rows, it);
    if (sr) {
      for (int k = 0; k < 5; ++k) sr[k] = NAN;
      sr[5] = mu;
      sr[6] = rs;
      sr[7] = 0.0;
      sr[8] = ri;
      sr[9] = rc;
    }
    if (!isfinite(rs) || !isfinite(ri) || !isfinite(rc)) {
      status = CMPC_NAN_SOL;
      break;
    }
    if (rs <= s->tol_stat && ri <= s->tol_ineq && rc <= s->tol_comp) {
      status = CMPC_SUCCESS;
      break;
    }
    if (it >= s->iter_max) {
      status = CMPC_MAX_ITER;
      break;
    }
    if (m > 0 && !(mu > 1e-300)) { /* mu underflow guard, as the kernels */
      status = CMPC_MIN_STEP;
      break;
    }
    if (ops->factor(ops->ctx, nt, tri_mu, W.ll, W.lu, W.tl, W.tu, s->reg_prim) != 0) {
      status = CMPC_NAN_SOL;
      break;
    }
    /* predictor (affine scaling) */
    for (int j = 0; j < m; ++j) {
      W.rml[j] = W.tl[j] * W.ll[j];
      W.rmu[j] = W.tu[j] * W.lu[j];
    }
    ipm_dir(n, ops, nt, tri_mu, &W);
    double alpha = dmin(1.0, ipm_maxstep(m, &W));
    if (m > 0) {
      double maff = 0.0;
      for (int j = 0; j < m; ++j)
        maff += (W.tl[j] + alpha * W.dtl[j]) * (W.ll[j] + alpha * W.dll[j]) +
                (W.tu[j] + alpha * W.dtu[j]) * (W.lu[j] + alpha * W.dlu[j]);
      maff /= 2.0 * m;
      const double ratio = maff / mu;
      const double sigma = ratio * ratio * ratio;
      if (sr) {
        sr[0] = alpha;
        sr[1] = maff;
        sr[2] = sigma;
      }
      /* corrector: rm = t.lam + dt_aff.dlam_aff - sigma mu */
      for (int j = 0; j < m; ++j) {
        W.rml[j] = W.tl[j] * W.ll[j] + W.dtl[j] * W.dll[j] - sigma * mu;
        W.rmu[j] = W.tu[j] * W.lu[j] + W.dtu[j] * W.dlu[j] - sigma * mu;
      }
      ipm_dir(n, ops, nt, tri_mu, &W);
      alpha = dmin(1.0, TAU * ipm_maxstep(m, &W));
    }
    if (sr) sr[3] = sr[4] = alpha;
    if (alpha < s->alpha_min) {
      status = CMPC_MIN_STEP;
      break;
    }
    for (int i = 0; i < n; ++i) u[i] += alpha * W.du[i];
    for (int j = 0; j < m; ++j) {
      W.tl[j] += alpha * W.dtl[j];
      W.tu[j] += alpha * W.dtu[j];
      W.ll[j] += alpha * W.dll[j];
      W.lu[j] += alpha * W.dlu[j];
    }
  }
  for (int i = 0; i < n; ++i)
    if (!isfinite(u[i])) status = CMPC_NAN_SOL;
  if (lam_lo) memcpy(lam_lo, W.ll, sizeof(double) * m);
  if (lam_hi) memcpy(lam_hi, W.lu, sizeof(double) * m);
  if (iters) *iters = it;
  if (res) {
    res[0] = rs;
    res[1] = 0.0;
    res[2] = ri;
    res[3] = rc;
  }
  free(buf);
  return status;
}

void oracle_qp_kkt(int n, int ld, const double* H, const double* g, const double* tri_mu, const double* tri_lo,
                   const double* tri_hi, const double* u, const double* lam_lo, const double* lam_hi, double* out) {
  const int nt = n / 3;
  double st = 0.0, pf = 0.0, cp = 0.0, dn = 0.0;
  for (int t = 0; t < nt; ++t) {
    double w[5], f[3], c5[5];
    for (int r = 0; r < 5; ++r) w[r] = lam_lo[5 * t + r] - lam_hi[5 * t + r];
    pyr_applyT(tri_mu[t], w, f);
    pyr_apply(tri_mu[t], u + 3 * t, c5);
    for (int d = 0; d < 3; ++d) {
      const int i = 3 * t + d;
      double acc = g[i] - f[d];
      for (int j = 0; j < n; ++j) acc += H[(size_t)i * ld + j] * u[j];
      st = dmax(st, fabs(acc));
    }
    for (int r = 0; r < 5; ++r) {
      const int j = 5 * t + r;
      pf = dmax(pf, dmax(tri_lo[j] - c5[r], c5[r] - tri_hi[j]));
      cp = dmax(cp, dmax(fabs(lam_lo[j] * (c5[r] - tri_lo[j])), fabs(lam_hi[j] * (tri_hi[j] - c5[r]))));
      dn = dmax(dn, dmax(-lam_lo[j], -lam_hi[j]));
    }
  }
  out[0] = st;
  out[1] = pf;
  out[2] = cp;
  out[3] = dn;
}

/* ------------------------------------------------------------------------------------------------ full path */

int oracle_solve_one(const oracle_consts* c, const cmpc_settings* s, const double* x0, const double* xref,
                     const double* foot, const uint8_t* contact, double* u, double* x, int* iters) {
  return oracle_solve_one_lin(c, s, x0, xref, foot, contact, NULL, u, x, iters);
}

int oracle_solve_one_lin(const oracle_consts* c, const cmpc_settings* s, const double* x0, const double* xref,
                         const double* foot, const uint8_t* contact, const double* lin, double* u, double* x,
                         int* iters) {
  const int N = c->N, ld = NU * N;
  double* H = (double*)malloc(sizeof(double) * ld * ld);
  double* g = (double*)malloc(sizeof(double) * ld);
  double* mu = (double*)malloc(sizeof(double) * ld);
  double* lo = (double*)malloc(sizeof(double) * 5 * ld);
  double* hi = (double*)malloc(sizeof(double) * 5 * ld);
  double* uc = (double*)malloc(sizeof(double) * ld);
  int* map = (int*)malloc(sizeof(int) * ld);
  int n = 0, it = 0;
  double* u_in = NULL;
  if (s->warm_start) { /* u holds the initial guess [N][L][3] on entry */
    u_in = (double*)malloc(sizeof(double) * N * NU);
    memcpy(u_in, u, sizeof(double) * N * NU);
  }
  memset(u, 0, sizeof(double) * N * NU);
  int st = oracle_condense_lin(c, x0, xref, foot, contact, lin, ld, &n, H, g, mu, lo, hi, map);
  if (st == CMPC_SUCCESS) {
    if (u_in)
      for (int t = 0; t < n / 3; ++t)
        for (int d = 0; d < 3; ++d) uc[3 * t + d] = u_in[map[t] * 3 + d];
    st = oracle_qp_ipm(n, ld, H, g, mu, lo, hi, s, uc, NULL, NULL, &it, NULL);
    for (int t = 0; t < n / 3; ++t)
      for (int d = 0; d < 3; ++d) u[map[t] * 3 + d] = uc[3 * t + d];
  }
  if (x) {
    /* rollout x_{k+1} = A_k x_k + B_k u_k */
    double* A = (double*)malloc(sizeof(double) * N * NX * NX);
    double* B = (double*)malloc(sizeof(double) * N * NX * NU);
    double* bb = (double*)malloc(sizeof(double) * N * NX);
    oracle_srbd_dynamics_lin(c, xref, foot, contact, lin, A, B, bb);
    memcpy(x, x0, sizeof(double) * NX);
    for (int k = 0; k < N; ++k)
      for (int r = 0; r < NX; ++r) {
        double acc = 0.0;
        for (int t = 0; t < NX; ++t) acc += A[(size_t)k * NX * NX + r * NX + t] * x[k * NX + t];
        for (int j = 0; j < NU; ++j) acc += B[(size_t)k * NX * NU + r * NU + j] * u[k * NU + j];
        x[(k + 1) * NX + r] = acc + bb[k * NX + r];
      }
    free(A);
    free(B);
    free(bb);
  }
  if (iters) *iters = it;
  free(H);
  free(g);
  free(mu);
  free(lo);
  free(hi);
  free(uc);
  free(map);
  free(u_in);
  return st;
}

typedef struct batch_job {
  const oracle_consts* c;
  const cmpc_settings* s;
  int B, tid, nthreads;
  const double *x0, *xref, *foot;
  const uint8_t* contact;
  double *u, *x;
  int *status, *iters;
} batch_job;

static void* batch_worker(void* arg) {
  batch_job* j = (batch_job*)arg;
  const int N = j->c->N, L = j->c->L;
  for (int q = j->tid; q < j->B; q += j->nthreads) {
    int it = 0;
    const int st = oracle_solve_one(j->c, j->s, j->x0 + (size_t)q * NX, j->xref + (size_t)q * (N + 1) * NX,
                                    j->foot + (size_t)q * (N + 1) * L * 3, j->contact + (size_t)q * N * L,
                                    j->u + (size_t)q * N * NU, j->x ? j->x + (size_t)q * (N + 1) * NX : NULL, &it);
    if (j->status) j->status[q] = st;
    if (j->iters) j->iters[q] = it;
  }
  return NULL;
}

int oracle_solve_batch(const cmpc_model* m, const cmpc_settings* s, int B, const double* x0, const double* xref,
                       const double* foot, const uint8_t* contact, double* u, double* x, int* status, int* iters,
                       int nthreads) {
  oracle_consts c;
  oracle_consts_init(m, &c);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  batch_job jobs[256];
  pthread_t th[256];
  for (int t = 0; t < nthreads; ++t) {
    batch_job jb = {&c, s, B, t, nthreads, x0, xref, foot, contact, u, x, status, iters};
    jobs[t] = jb;
  }
  if (nthreads == 1) {
    batch_worker(&jobs[0]);
    return 0;
  }
  for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  return 0;
}

/* ------------------------------------------------------------------------------------------------ generator */

static inline void mulhilo32(uint32_t a, uint32_t b, uint32_t* hi, uint32_t* lo) {
  const uint64_t p = (uint64_t)a * (uint64_t)b;
  *hi = (uint32_t)(p >> 32);
  *lo = (uint32_t)p;
}

void oracle_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo32(0xD2511F53u, c0, &hi0, &lo0);
    mulhilo32(0xCD9E8D57u, c2, &hi1, &lo1);
    const uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0;
    c1 = n1;
    c2 = n2;
    c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

/* uniform draw idx of QP gid in [0,1): 53-bit mantissa, exact on any IEEE host/device */
static double gen_uniform(uint64_t seed, uint64_t gid, int idx) {
  const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  const uint32_t ctr[4] = {(uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)(idx >> 1), 0x43504D43u /* "CMPC" */};
  uint32_t o[4];
  oracle_philox4x32_10(ctr, key, o);
  const uint64_t v = (idx & 1) ? ((uint64_t)o[3] << 32 | o[2]) : ((uint64_t)o[1] << 32 | o[0]);
  return (double)(v >> 11) * 0x1.0p-53;
}

static inline double urange(double a, double b, double u) { return fma(b - a, u, a); }

/* nominal feet of CentoidMPCTest.cpp:43-46 (lf, rf, rh, lh) */
static const double kNomFoot[4][2] = {{0.35, 0.052}, {0.35, -0.054}, {-0.37, -0.053}, {-0.36, 0.054}};

void oracle_generate(const cmpc_model* m, uint64_t seed, int64_t qp_offset, int B, int gait, double* x0,
                     double* xref, double* foot, uint8_t* contact) {
  const int N = m->N, L = m->n_legs;
  const double PI = 3.14159265358979323846;
  for (int q = 0; q < B; ++q) {
    const uint64_t gid = (uint64_t)(qp_offset + q);
    double U[32];
    for (int i = 0; i < 32; ++i) U[i] = gen_uniform(seed, gid, i);
    double* X0 = x0 + (size_t)q * NX;
    X0[0] = urange(-0.2, 0.2, U[0]);
    X0[1] = urange(-0.2, 0.2, U[1]);
    X0[2] = urange(0.12, 0.20, U[2]);
    X0[3] = urange(-1.0, 1.0, U[3]);
    X0[4] = urange(-1.0, 1.0, U[4]);
    X0[5] = urange(-0.2, 0.2, U[5]);
    for (int d = 0; d < 3; ++d) X0[6 + d] = urange(-0.1, 0.1, U[6 + d]);
    X0[9] = urange(-0.1, 0.1, U[9]);
    X0[10] = urange(-0.1, 0.1, U[10]);
    X0[11] = urange(-PI, PI, U[11]);
    X0[12] = -GRAV;
    const double vdx = urange(-1.0, 1.0, U[12]), vdy = urange(-1.0, 1.0, U[13]);
    const int h = GAIT_HALF_PERIOD;
    const int phase = (int)(U[22] * (double)(2 * h));
    int gsel = 0;
    if (gait == 1) gsel = (int)(U[23] * 3.0);
    uint8_t* C = contact + (size_t)q * N * L;
    for (int k = 0; k < N; ++k) {
      const int first = ((k + phase) % (2 * h)) < h;
      for (int i = 0; i < L; ++i) {
        int e;
        if (gsel == 0) /* trot: {lf, rh} / {rf, lh} (CentoidMPCTest.cpp:68-73) */
          e = first ? (i == 0 || i == 2) : (i == 1 || i == 3);
        else if (gsel == 1) /* bound: front {0,1} / hind {2,3} */
          e = first ? (i < 2) : (i >= 2);
        else /* pronk, stance phase: all legs */
          e = 1;
        C[k * L + i] = (uint8_t)e;
      }
    }
    double* XR = xref + (size_t)q * (N + 1) * NX;
    double* FT = foot + (size_t)q * (N + 1) * L * 3;
    for (int k = 0; k <= N; ++k) {
      double* xr = XR + k * NX;
      const double tk = (double)k * m->dt;
      xr[0] = fma(tk, vdx, X0[0]);
      xr[1] = fma(tk, vdy, X0[1]);
      xr[2] = 0.15;
      xr[3] = vdx;
      xr[4] = vdy;
      xr[5] = 0.0;
      for (int d = 6; d < 11; ++d) xr[d] = 0.0;
      xr[11] = X0[11];
      xr[12] = -GRAV;
    }
    /* planted feet: a node pinned by a stance run (step k or k-1 in stance) holds the foothold placed at the run's
     * touch-down step s around c^ref_s; swing nodes follow the body; node 0 (current foot) adds a +-1 cm offset */
    for (int k = 0; k <= N; ++k) {
      for (int i = 0; i < L; ++i) {
        const int st_k = k < N && C[k * L + i], st_p = k > 0 && C[(k - 1) * L + i];
        int s = k;
        if (st_k || st_p) {
          s = st_k ? k : k - 1;
          while (s > 0 && C[(s - 1) * L + i]) --s;
        }
        const double ts = (double)s * m->dt;
        const double cx = fma(ts, vdx, X0[0]), cy = fma(ts, vdy, X0[1]);
        double* p = FT + ((size_t)k * L + i) * 3;
        p[0] = (cx + kNomFoot[i & 3][0]) + urange(-0.03, 0.03, U[14 + 2 * (i & 3)]);
        p[1] = (cy + kNomFoot[i & 3][1]) + urange(-0.03, 0.03, U[15 + 2 * (i & 3)]);
        p[2] = 0.0;
        if (k == 0) {
          p[0] += urange(-0.01, 0.01, U[24 + 2 * (i & 3)]);
          p[1] += urange(-0.01, 0.01, U[25 + 2 * (i & 3)]);
        }
      }
    }
  }
}

/* ------------------------------------------------------------------------------------------------ generic OCP */

static void ocp_offsets(int N, int nx, const int* nu, size_t* offA, size_t* offB, size_t* offb, size_t* offQ,
                        size_t* offS, size_t* offR, size_t* offq, size_t* offr, size_t* total) {
  size_t o = 0;
  for (int k = 0; k < N; ++k) {
    offA[k] = o; o += (size_t)nx * nx;
    offB[k] = o; o += (size_t)nx * nu[k];
    offb[k] = o; o += (size_t)nx;
  }
  for (int k = 0; k <= N; ++k) {
    const int m = k < N ? nu[k] : 0;
    offQ[k] = o; o += (size_t)nx * nx;
    offS[k] = o; o += (size_t)m * nx;
    offR[k] = o; o += (size_t)m * m;
    offq[k] = o; o += (size_t)nx;
    offr[k] = o; o += (size_t)m;
  }
  *total = o;
}

size_t oracle_ocp_record_size(int N, int nx, const int* nu) {
  size_t o = 0;
  for (int k = 0; k < N; ++k) o += (size_t)nx * nx + (size_t)nx * nu[k] + nx;
  for (int k = 0; k <= N; ++k) {
    const int m = k < N ? nu[k] : 0;
    o += (size_t)nx * nx + (size_t)m * nx + (size_t)m * m + nx + m;
  }
  return o;
}

#define CM(M, ld, r, c) ((M)[(size_t)(c) * (ld) + (r)]) /* column-major access */

int oracle_ocp_condense(int N, int nx, const int* nu, const double* x0, const double* rec, double* H, double* g) {
  size_t offA[N], offB[N], offb[N], offQ[N + 1], offS[N + 1], offR[N + 1], offq[N + 1], offr[N + 1], tot;
  ocp_offsets(N, nx, nu, offA, offB, offb, offQ, offS, offR, offq, offr, &tot);
  int cu[N + 1];
  int nU = 0;
  for (int k = 0; k < N; ++k) {
    cu[k] = nU;
    nU += nu[k];
  }
  cu[N] = nU;
  memset(H, 0, sizeof(double) * nU * nU);
  memset(g, 0, sizeof(double) * nU);
  double* G = (double*)calloc((size_t)nx * (nU + 1), sizeof(double)); /* row-major nx x nU */
  double* G2 = (double*)malloc(sizeof(double) * nx * (nU + 1));
  double* xb = (double*)malloc(sizeof(double) * nx);
  double* xb2 = (double*)malloc(sizeof(double) * nx);
  double* tmp = (double*)malloc(sizeof(double) * nx);
  memcpy(xb, x0, sizeof(double) * nx);
  /* k = 0: only the linear term r0 + S0 x0 (HpipmInterface.cpp:205-208) and R0 */
  for (int k = 0; k <= N; ++k) {
    const int m = k < N ? nu[k] : 0;
    const double* Q = rec + offQ[k];
    const double* S = rec + offS[k];
    const double* R = rec + offR[k];
    const double* q = rec + offq[k];
    const double* r = rec + offr[k];
    if (k >= 1) {
      /* H += G' Q G; g += G' (Q xb + q) */
      for (int i = 0; i < nx; ++i) {
        double s = q[i];
        for (int j = 0; j < nx; ++j) s += CM(Q, nx, i, j) * xb[j];
        tmp[i] = s;
      }
      for (int a = 0; a < cu[k]; ++a) {
        double s = 0.0;
        for (int i = 0; i < nx; ++i) s += G[i * nU + a] * tmp[i];
        g[a] += s;
        for (int b = 0; b < cu[k]; ++b) {
          double h = 0.0;
          for (int i = 0; i < nx; ++i) {
            double qg = 0.0;
            for (int j = 0; j < nx; ++j) qg += CM(Q, nx, i, j) * G[j * nU + b];
            h += G[i * nU + a] * qg;
          }
          H[a * nU + b] += h;
        }
      }
    }
    if (m > 0) {
      /* g_k += S xb + r ; H_kk += R ; cross terms E'S G + G'S'E */
      for (int a = 0; a < m; ++a) {
        double s = r[a];
        for (int j = 0; j < nx; ++j) s += CM(S, m, a, j) * xb[j];
        g[cu[k] + a] += s;
        for (int b = 0; b < m; ++b) H[(cu[k] + a) * nU + cu[k] + b] += CM(R, m, a, b);
        if (k >= 1)
          for (int b = 0; b < cu[k]; ++b) {
            double sg = 0.0;
            for (int j = 0; j < nx; ++j) sg += CM(S, m, a, j) * G[j * nU + b];
            H[(cu[k] + a) * nU + b] += sg;
            H[b * nU + cu[k] + a] += sg;
          }
      }
    }
    if (k < N) {
      /* propagate: G <- A G + [B at columns of k]; xb <- A xb + b */
      const double* A = rec + offA[k];
      const double* Bm = rec + offB[k];
      const double* b = rec + offb[k];
      for (int i = 0; i < nx; ++i) {
        for (int a = 0; a < nU; ++a) {
          double s = 0.0;
          for (int j = 0; j < nx; ++j) s += CM(A, nx, i, j) * G[j * nU + a];
          G2[i * nU + a] = s;
        }
        for (int a = 0; a < m; ++a) G2[i * nU + cu[k] + a] += CM(Bm, nx, i, a);
        double s = b[i];
        for (int j = 0; j < nx; ++j) s += CM(A, nx, i, j) * xb[j];
        xb2[i] = s;
      }
      memcpy(G, G2, sizeof(double) * nx * nU);
      memcpy(xb, xb2, sizeof(double) * nx);
    }
  }
  free(G);
  free(G2);
  free(xb);
  free(xb2);
  free(tmp);
  return nU;
}

int oracle_ocp_solve(int N, int nx, const int* nu, const double* x0, const double* rec, double* x, double* u) {
  int nU = 0;
  for (int k = 0; k < N; ++k) nU += nu[k];
  double* H = (double*)malloc(sizeof(double) * (nU * nU + 1));
  double* g = (double*)malloc(sizeof(double) * (nU + 1));
  oracle_ocp_condense(N, nx, nu, x0, rec, H, g);
  int st = CMPC_SUCCESS;
  if (nU > 0) {
    if (oracle_cholesky(nU, H, nU) != 0) st = CMPC_NAN_SOL;
    for (int i = 0; i < nU; ++i) u[i] = -g[i];
    if (st == CMPC_SUCCESS) oracle_chol_solve(nU, H, nU, u);
  }
  size_t offA[N], offB[N], offb[N], offQ[N + 1], offS[N + 1], offR[N + 1], offq[N + 1], offr[N + 1], tot;
  ocp_offsets(N, nx, nu, offA, offB, offb, offQ, offS, offR, offq, offr, &tot);
  memcpy(x, x0, sizeof(double) * nx);
  int cu = 0;
  for (int k = 0; k < N; ++k) {
    const double* A = rec + offA[k];
    const double* Bm = rec + offB[k];
    const double* b = rec + offb[k];
    for (int i = 0; i < nx; ++i) {
      double s = b[i];
      for (int j = 0; j < nx; ++j) s += CM(A, nx, i, j) * x[k * nx + j];
      for (int a = 0; a < nu[k]; ++a) s += CM(Bm, nx, i, a) * u[cu + a];
      x[(k + 1) * nx + i] = s;
    }
    cu += nu[k];
  }
  for (int i = 0; i < (N + 1) * nx; ++i)
    if (!isfinite(x[i])) st = CMPC_NAN_SOL;
  for (int i = 0; i < nU; ++i)
    if (!isfinite(u[i])) st = CMPC_NAN_SOL;
  free(H);
  free(g);
  return st;
}

/* general inverse via Cholesky of an SPD matrix (n <= 64): out = M^{-1} */
static int spd_inverse(int n, const double* M, double* out) {
  double* Lm = (double*)malloc(sizeof(double) * (n * n + 1));
  memcpy(Lm, M, sizeof(double) * n * n);
  if (oracle_cholesky(n, Lm, n) != 0) {
    free(Lm);
    return -1;
  }
  double* e = (double*)malloc(sizeof(double) * (n + 1));
  for (int j = 0; j < n; ++j) {
    for (int i = 0; i < n; ++i) e[i] = (i == j) ? 1.0 : 0.0;
    oracle_chol_solve(n, Lm, n, e);
    for (int i = 0; i < n; ++i) out[i * n + j] = e[i];
  }
  free(e);
  free(Lm);
  return 0;
}

int oracle_ocp_riccati(int N, int nx, const int* nu, const double* rec, double* Sm, double* sv, double* K,
                       double* kff) {
  size_t offA[N], offB[N], offb[N], offQ[N + 1], offS[N + 1], offR[N + 1], offq[N + 1], offr[N + 1], tot;
  ocp_offsets(N, nx, nu, offA, offB, offb, offQ, offS, offR, offq, offr, &tot);
  size_t offK[N + 1];
  int offk[N + 1];
  size_t ok = 0;
  int okk = 0;
  for (int k = 0; k < N; ++k) {
    offK[k] = ok;
    ok += (size_t)nu[k] * nx;
    offk[k] = okk;
    okk += nu[k];
  }
  /* terminal */
  for (int i = 0; i < nx; ++i) {
    for (int j = 0; j < nx; ++j) Sm[(size_t)N * nx * nx + i * nx + j] = CM(rec + offQ[N], nx, i, j);
    sv[(size_t)N * nx + i] = rec[offq[N] + i];
  }
  double* SmA = (double*)malloc(sizeof(double) * nx * nx);
  double* Smb = (double*)malloc(sizeof(double) * nx);
  double* P = (double*)malloc(sizeof(double) * 64 * nx);
  double* Rt = (double*)malloc(sizeof(double) * 64 * 64);
  double* iR = (double*)malloc(sizeof(double) * 64 * 64);
  double* rr = (double*)malloc(sizeof(double) * 64);
  double* SmB = (double*)malloc(sizeof(double) * nx * 64);
  int st = 0;
  for (int k = N - 1; k >= 0; --k) {
    const int m = nu[k];
    const double* A = rec + offA[k];
    const double* Bm = rec + offB[k];
    const double* b = rec + offb[k];
    const double* Q = rec + offQ[k];
    const double* S = rec + offS[k];
    const double* R = rec + offR[k];
    const double* q = rec + offq[k];
    const double* r = rec + offr[k];
    const double* Sn = Sm + (size_t)(k + 1) * nx * nx;
    const double* sn = sv + (size_t)(k + 1) * nx;
    for (int i = 0; i < nx; ++i) {
      for (int j = 0; j < nx; ++j) {
        double s = 0.0;
        for (int t = 0; t < nx; ++t) s += Sn[i * nx + t] * CM(A, nx, t, j);
        SmA[i * nx + j] = s;
      }
      for (int a = 0; a < m; ++a) {
        double s = 0.0;
        for (int t = 0; t < nx; ++t) s += Sn[i * nx + t] * CM(Bm, nx, t, a);
        SmB[i * 64 + a] = s;
      }
      double s = 0.0;
      for (int t = 0; t < nx; ++t) s += Sn[i * nx + t] * b[t];
      Smb[i] = s;
    }
    /* P = S + B' Sm A (m x nx); Rt = R + B' Sm B; rr = r + B' sv + B' Sm b */
    for (int a = 0; a < m; ++a) {
      for (int j = 0; j < nx; ++j) {
        double s = CM(S, m, a, j);
        for (int t = 0; t < nx; ++t) s += CM(Bm, nx, t, a) * SmA[t * nx + j];
        P[a * nx + j] = s;
      }
      for (int c = 0; c < m; ++c) {
        double s = CM(R, m, a, c);
        for (int t = 0; t < nx; ++t) s += CM(Bm, nx, t, a) * SmB[t * 64 + c];
        Rt[a * m + c] = s;
      }
      double s = r[a];
      for (int t = 0; t < nx; ++t) s += CM(Bm, nx, t, a) * (sn[t] + Smb[t]);
      rr[a] = s;
    }
    if (m > 0 && spd_inverse(m, Rt, iR) != 0) st = -1;
    double* Sk = Sm + (size_t)k * nx * nx;
    double* sk = sv + (size_t)k * nx;
    for (int i = 0; i < nx; ++i) {
      for (int j = 0; j < nx; ++j) {
        double s = CM(Q, nx, i, j);
        for (int t = 0; t < nx; ++t) s += CM(A, nx, t, i) * SmA[t * nx + j];
        for (int a = 0; a < m; ++a)
          for (int c = 0; c < m; ++c) s -= P[a * nx + i] * iR[a * m + c] * P[c * nx + j];
        Sk[i * nx + j] = s;
      }
      double s = q[i];
      for (int t = 0; t < nx; ++t) s += CM(A, nx, t, i) * (sn[t] + Smb[t]);
      for (int a = 0; a < m; ++a)
        for (int c = 0; c < m; ++c) s -= P[a * nx + i] * iR[a * m + c] * rr[c];
      sk[i] = s;
    }
    for (int a = 0; a < m; ++a) {
      for (int j = 0; j < nx; ++j) {
        double s = 0.0;
        for (int c = 0; c < m; ++c) s -= iR[a * m + c] * P[c * nx + j];
        K[offK[k] + (size_t)a * nx + j] = s;
      }
      double s = 0.0;
      for (int c = 0; c < m; ++c) s -= iR[a * m + c] * rr[c];
      kff[offk[k] + a] = s;
    }
  }
  free(SmA);
  free(Smb);
  free(P);
  free(Rt);
  free(iR);
  free(rr);
  free(SmB);
  return st;
}

/* ---------------------------------------------------------------------------------------------- gait schedule */
/* GaitSchedule::getModeSchedule keeps a STANCE phase before the tiled template (GaitSchedule.cpp:78-101);
 * tileModeSequenceTemplate repeats (mode_i, switching_time_{i+1} - switching_time_i) from the start time (:106-127);
 * modeNumber2StanceLeg decodes ModeNumber bits {LF, RF, LH, RH} = {8, 4, 2, 1} (MotionPhaseDefinition.h:69-124).
 * The mode of step k is the one in force at t = t0 + k dt, intervals closed on the left. */
void oracle_gait_contact(const cmpc_gait* g, const int* leg_map, double t_start, double t0, double dt, int N,
                         uint8_t* contact) {
  static const int def_map[4] = {0, 1, 3, 2};
  const int* lm = leg_map ? leg_map : def_map;
  for (int k = 0; k < N; ++k) {
    const double t = t0 + (double)k * dt;
    int mode = 15; /* STANCE */
    if (!(t < t_start)) {
      const int M = g->n_modes;
      const double period = g->switching_time[M] - g->switching_time[0];
      const double tau = fmod(t - t_start, period) + g->switching_time[0];
      int i = 0;
      for (int j = 1; j < M; ++j)
        if (g->switching_time[j] <= tau) i = j;
      mode = g->mode[i];
    }
    for (int j = 0; j < 4; ++j) contact[k * 4 + lm[j]] = (uint8_t)((mode >> (3 - j)) & 1);
  }
}

/* ------------------------------------------------------------------------------------------------- SQP (§8f) */
/* Nonlinear SRBD rollout with the bilinear lever arm of CentroidalMPC.cpp:85-92 (L+ = L + dt sum_i e_i (p_i - c) x
 * f_i, c+ = c + dt v, v+ = v + dt (g e_z + sum_i e_i f_i / m)), Theta as the QP (A.2), and the NLP cost of
 * CentroidalMPC.cpp:203-231 in its sumsqr form: sum_k w (x_k - xref_k)^2 (Q-bar / 2) + sum w_f (f - f^des)^2 +
 * sum w_r (f_{k+1} - f_k)^2 over all legs (swing forces are 0). x [(N+1)][13] and lin [N][6] (c_k, sum_i e_ik f_ik)
 * may be NULL. Returns the cost. Floating-point order is the one k_sqp_step follows. */
double oracle_nlp_rollout_cost(const oracle_consts* c, const double* x0, const double* xref, const double* foot,
                               const uint8_t* contact, const double* u, double* x, double* lin) {
  return oracle_nlp_rollout_cost_feet(c, x0, xref, foot, contact, u, NULL, x, lin);
}

/* Lever-arm point of stance leg i at step k: oracle_stance_point, plus the foothold offset D [N][L][3] of its run
 * when the run is a later one (D indexed by the run's first step; D = NULL: frozen footholds). */
static void lever_point(const double* foot, const uint8_t* contact, const double* D, int N, int L, int k, int i,
                        double p[3]) {
  oracle_stance_point(foot, contact, N, L, k, i, p);
  if (!D) return;
  int s = k;
  while (s > 0 && contact[(s - 1) * L + i]) --s;
  if (s == 0) return;
  const double* dl = D + ((size_t)s * L + i) * 3;
  p[0] = p[0] + dl[0];
  p[1] = p[1] + dl[1];
  p[2] = p[2] + dl[2];
}

/* Foot tracking cost of the later stance runs (CentroidalMPC.cpp:218-221 over the run's nodes s..e+1; nodes of the
 * first run are pinned to the current foot and free swing nodes track exactly, so neither depends on a decision
 * variable): sum_i sum_runs sum_j sum_d Wp (pbar + D - des_j)^2, legs outer, runs by first step, nodes, components.
 * With dD != NULL returns instead the directional derivative sum 2 Wp (pbar + D - des_j) dD. */
static double foot_cost(const oracle_consts* c, const double* foot, const uint8_t* contact, const double* D,
                        const double* dD) {
  const int N = c->N, L = c->L;
  double J = 0.0;
  for (int i = 0; i < L; ++i)
    for (int s = 1; s < N; ++s) {
      if (!contact[s * L + i] || contact[(s - 1) * L + i]) continue;
      int e = s;
      while (e + 1 < N && contact[(e + 1) * L + i]) ++e;
      double pb[3];
      oracle_stance_point(foot, contact, N, L, s, i, pb);
      const double* dl = D + ((size_t)s * L + i) * 3;
      for (int j = s; j <= e + 1; ++j)
        for (int d = 0; d < 3; ++d) {
          const double ed = (pb[d] + dl[d]) - foot[((size_t)j * L + i) * 3 + d];
          if (dD)
            J += 2.0 * c->Wp[3 * i + d] * ed * dD[((size_t)s * L + i) * 3 + d];
          else
            J += c->Wp[3 * i + d] * ed * ed;
        }
    }
  return J;
}

/* Same, with the later runs' footholds as decision variables: pbar + D (D [N][L][3] by run start, NULL: frozen) in
 * the lever arm and the foot tracking cost of the later runs added after the rollout. */
double oracle_nlp_rollout_cost_feet(const oracle_consts* c, const double* x0, const double* xref, const double* foot,
                                    const uint8_t* contact, const double* u, const double* D, double* x, double* lin) {
  const int N = c->N, L = c->L;
  const double dt = c->dt;
  double xs[NX], xn[NX];
  memcpy(xs, x0, sizeof(xs));
  if (x) memcpy(x, x0, sizeof(double) * NX);
  double J = 0.0;
  for (int k = 0; k < N; ++k) {
    const double* uk = u + (size_t)k * NU;
    double F[3] = {0.0, 0.0, 0.0}, T[3] = {0.0, 0.0, 0.0};
    int ns = 0;
    for (int i = 0; i < L; ++i) {
      if (!contact[k * L + i]) continue;
      ++ns;
      double p[3];
      lever_point(foot, contact, D, N, L, k, i, p);
      const double* f = uk + 3 * i;
      const double rx = p[0] - xs[0], ry = p[1] - xs[1], rz = p[2] - xs[2];
      F[0] += f[0];
      F[1] += f[1];
      F[2] += f[2];
      T[0] += ry * f[2] - rz * f[1];
      T[1] += rz * f[0] - rx * f[2];
      T[2] += rx * f[1] - ry * f[0];
    }
    if (lin) {
      for (int d = 0; d < 3; ++d) {
        lin[k * 6 + d] = xs[d];
        lin[k * 6 + 3 + d] = F[d];
      }
    }
    /* force tracking and force rate */
    for (int j = 0; j < NU; ++j) {
      const int i = j / 3;
      const double fd = (j % 3 == 2 && contact[k * L + i] && ns > 0) ? c->mass * GRAV / (double)ns : 0.0;
      const double e = uk[j] - fd;
      J += c->Wf[j] * e * e;
      if (k + 1 < N) {
        const double r = u[(size_t)(k + 1) * NU + j] - uk[j];
        J += c->Wr[j] * r * r;
      }
    }
    const double psi = xref[k * NX + 11];
    const double cp = cos(psi), sp = sin(psi);
    const double RzT[9] = {cp, sp, 0.0, -sp, cp, 0.0, 0.0, 0.0, 1.0};
    for (int d = 0; d < 3; ++d) xn[d] = xs[d] + dt * xs[3 + d];
    xn[3] = xs[3] + dt * (F[0] / c->mass);
    xn[4] = xs[4] + dt * (F[1] / c->mass);
    xn[5] = xs[5] + dt * (xs[12] + F[2] / c->mass);
    for (int d = 0; d < 3; ++d) xn[6 + d] = xs[6 + d] + dt * T[d];
    for (int a = 0; a < 3; ++a) {
      double m = 0.0;
      for (int b = 0; b < 3; ++b) {
        double s2 = 0.0;
        for (int e = 0; e < 3; ++e) s2 += c->inv_inertia[a * 3 + e] * RzT[e * 3 + b];
        m += dt * s2 * xs[6 + b];
      }
      xn[9 + a] = xs[9 + a] + m;
    }
    xn[12] = xs[12];
    memcpy(xs, xn, sizeof(xs));
    if (x) memcpy(x + (size_t)(k + 1) * NX, xs, sizeof(double) * NX);
    for (int sI = 0; sI < NX; ++sI) {
      const double e = xs[sI] - xref[(k + 1) * NX + sI];
      J += 0.5 * c->qdiag[k + 1][sI] * e * e;
    }
  }
  if (D) J += foot_cost(c, foot, contact, D, NULL);
  return J;
}

/* Linearised response of the rollout of u to the step du (the QP's dx, single shooting: no defects) and the descent
 * metric of MultipleShootingSolver::getOCPSolution (MultipleShootingSolver.cpp:287-296): sum_k dJ/dx_k . dx_k +
 * dJ/du_k . du_k at u. Returns |dx| (trajectoryNorm, :492-503: the 2-norm over the whole trajectory) and the metric.
 * Jacobian of the step of oracle_nlp_rollout_cost at (x_k, u_k); floating-point order is the one k_sqp_step follows. */
void oracle_nlp_linstep(const oracle_consts* c, const double* x0, const double* xref, const double* foot,
                        const uint8_t* contact, const double* u, const double* du, double* dxnorm, double* metric) {
  oracle_nlp_linstep_feet(c, x0, xref, foot, contact, u, NULL, du, NULL, dxnorm, metric);
}

/* Same at the iterate (u, D) along (du, dD): d[(p - c) x f] = (p - c) x df - (dc - dp) x f, and the foot tracking
 * cost's derivative added to the metric after the rollout (D, dD NULL: frozen footholds). */
void oracle_nlp_linstep_feet(const oracle_consts* c, const double* x0, const double* xref, const double* foot,
                             const uint8_t* contact, const double* u, const double* D, const double* du,
                             const double* dD, double* dxnorm, double* metric) {
  const int N = c->N, L = c->L;
  const double dt = c->dt;
  double xs[NX], xn[NX], dx[NX], dn[NX];
  memcpy(xs, x0, sizeof(xs));
  memset(dx, 0, sizeof(dx));
  double ss = 0.0, mt = 0.0;
  for (int k = 0; k < N; ++k) {
    const double* uk = u + (size_t)k * NU;
    const double* duk = du + (size_t)k * NU;
    double F[3] = {0.0, 0.0, 0.0}, T[3] = {0.0, 0.0, 0.0}, dF[3] = {0.0, 0.0, 0.0}, dT[3] = {0.0, 0.0, 0.0};
    int ns = 0;
    for (int i = 0; i < L; ++i) {
      if (!contact[k * L + i]) continue;
      ++ns;
      double p[3], dp[3] = {0.0, 0.0, 0.0};
      lever_point(foot, contact, D, N, L, k, i, p);
      if (dD) {
        int s = k;
        while (s > 0 && contact[(s - 1) * L + i]) --s;
        if (s > 0)
          for (int d = 0; d < 3; ++d) dp[d] = dD[((size_t)s * L + i) * 3 + d];
      }
      const double* f = uk + 3 * i;
      const double* df = duk + 3 * i;
      const double rx = p[0] - xs[0], ry = p[1] - xs[1], rz = p[2] - xs[2];
      F[0] += f[0];
      F[1] += f[1];
      F[2] += f[2];
      T[0] += ry * f[2] - rz * f[1];
      T[1] += rz * f[0] - rx * f[2];
      T[2] += rx * f[1] - ry * f[0];
      dF[0] += df[0];
      dF[1] += df[1];
      dF[2] += df[2];
      /* d[(p - c) x f] = (p - c) x df - (dc - dp) x f */
      const double q0 = dx[0] - dp[0], q1 = dx[1] - dp[1], q2 = dx[2] - dp[2];
      dT[0] += (ry * df[2] - rz * df[1]) - (q1 * f[2] - q2 * f[1]);
      dT[1] += (rz * df[0] - rx * df[2]) - (q2 * f[0] - q0 * f[2]);
      dT[2] += (rx * df[1] - ry * df[0]) - (q0 * f[1] - q1 * f[0]);
    }
    (void)T;
    /* dJ/du_k . du_k: force tracking and both force-rate terms that hold u_k */
    for (int j = 0; j < NU; ++j) {
      const int i = j / 3;
      const double fd = (j % 3 == 2 && contact[k * L + i] && ns > 0) ? c->mass * GRAV / (double)ns : 0.0;
      double gu = 2.0 * c->Wf[j] * (uk[j] - fd);
      if (k > 0) gu += 2.0 * c->Wr[j] * (uk[j] - u[(size_t)(k - 1) * NU + j]);
      if (k + 1 < N) gu -= 2.0 * c->Wr[j] * (u[(size_t)(k + 1) * NU + j] - uk[j]);
      mt += gu * duk[j];
    }
    const double psi = xref[k * NX + 11];
    const double cp = cos(psi), sp = sin(psi);
    const double RzT[9] = {cp, sp, 0.0, -sp, cp, 0.0, 0.0, 0.0, 1.0};
    for (int d = 0; d < 3; ++d) {
      xn[d] = xs[d] + dt * xs[3 + d];
      dn[d] = dx[d] + dt * dx[3 + d];
    }
    xn[3] = xs[3] + dt * (F[0] / c->mass);
    xn[4] = xs[4] + dt * (F[1] / c->mass);
    xn[5] = xs[5] + dt * (xs[12] + F[2] / c->mass);
    dn[3] = dx[3] + dt * (dF[0] / c->mass);
    dn[4] = dx[4] + dt * (dF[1] / c->mass);
    dn[5] = dx[5] + dt * (dx[12] + dF[2] / c->mass);
    for (int d = 0; d < 3; ++d) {
      xn[6 + d] = xs[6 + d] + dt * T[d];
      dn[6 + d] = dx[6 + d] + dt * dT[d];
    }
    for (int a = 0; a < 3; ++a) {
      double m = 0.0, dm = 0.0;
      for (int b = 0; b < 3; ++b) {
        double s2 = 0.0;
        for (int e = 0; e < 3; ++e) s2 += c->inv_inertia[a * 3 + e] * RzT[e * 3 + b];
        m += dt * s2 * xs[6 + b];
        dm += dt * s2 * dx[6 + b];
      }
      xn[9 + a] = xs[9 + a] + m;
      dn[9 + a] = dx[9 + a] + dm;
    }
    xn[12] = xs[12];
    dn[12] = dx[12];
    memcpy(xs, xn, sizeof(xs));
    memcpy(dx, dn, sizeof(dx));
    /* dJ/dx_{k+1} . dx_{k+1} and |dx|^2 */
    for (int sI = 0; sI < NX; ++sI) {
      mt += c->qdiag[k + 1][sI] * (xs[sI] - xref[(k + 1) * NX + sI]) * dx[sI];
      ss += dx[sI] * dx[sI];
    }
  }
  if (D && dD) mt += foot_cost(c, foot, contact, D, dD);
  *dxnorm = sqrt(ss);
  *metric = mt;
}

/* Gauss-Newton SQP on the centroidal NLP (the role of MultipleShootingSolver::runImpl, MultipleShootingSolver.cpp:
 * 146-214, for this problem; single shooting, so the dynamics are met exactly and the merit is the NLP cost of the
 * nonlinear rollout, :447):
 *   U_0 = QP at the reference (lin = NULL);
 *   repeat: lin = (c_k, F_k) of the rollout of U_j; U_qp = QP at lin, warm-started from U_j; du = U_qp - U_j;
 *           takeStep (:509-619) with zero constraint violation: alpha = 1, 1/2, ... while alpha >= alpha_min; accept
 *           J(U_j + alpha du) < J(U_j) + armijoFactor alpha metric if metric < 0 (Armijo, :562-566), else
 *           J(U_j + alpha du) < J(U_j) (:567-571); after a rejection stop early once alpha |dx| and alpha |du| are
 *           both below deltaTol (:596-604);
 *           checkConvergence (:620-645): stop when no step was taken, when |J_new - J_j| < costTol, or when
 *           alpha |dx| and alpha |du| are both below deltaTol.
 * Settings are MultipleShootingSettings.h:42-54's defaults, deltaTol = sqp_tol. The pyramid constraints are linear in
 * f, so every trial point stays feasible. */
int oracle_sqp_solve(const oracle_consts* c, const cmpc_settings* s, int sqp_iter_max, double sqp_tol,
                     const double* x0, const double* xref, const double* foot, const uint8_t* contact, double* u,
                     double* x, int* qp_iters, int* sqp_iters) {
  const int N = c->N, nu = N * NU;
  double* uq = (double*)malloc(sizeof(double) * nu);
  double* ut = (double*)malloc(sizeof(double) * nu);
  double* du = (double*)malloc(sizeof(double) * nu);
  double* lin = (double*)malloc(sizeof(double) * N * 6);
  cmpc_settings sw = *s;
  sw.warm_start = 0;
  int it = 0, its = 0;
  int st = oracle_solve_one_lin(c, &sw, x0, xref, foot, contact, NULL, u, NULL, &it);
  int tot = it;
  if (st == CMPC_SUCCESS) {
    sw.warm_start = 1;
    for (its = 0; its < sqp_iter_max; ++its) {
      const double J0 = oracle_nlp_rollout_cost(c, x0, xref, foot, contact, u, NULL, lin);
      memcpy(uq, u, sizeof(double) * nu);
      const int sq = oracle_solve_one_lin(c, &sw, x0, xref, foot, contact, lin, uq, NULL, &it);
      tot += it;
      if (sq != CMPC_SUCCESS) {
        st = sq;
        break;
      }
      double dun2 = 0.0;
      for (int i = 0; i < nu; ++i) {
        du[i] = uq[i] - u[i];
        dun2 += du[i] * du[i];
      }
      const double dun = sqrt(dun2);
      double dxn = 0.0, metric = 0.0;
      oracle_nlp_linstep(c, x0, xref, foot, contact, u, du, &dxn, &metric);
      double alpha = 0.0, Jn = J0;
      for (double a = 1.0; a >= SQP_ALPHA_MIN;) {
        for (int i = 0; i < nu; ++i) ut[i] = u[i] + a * du[i];
        const double Jt = oracle_nlp_rollout_cost(c, x0, xref, foot, contact, ut, NULL, NULL);
        const int ok = metric < 0.0 ? (Jt < J0 + SQP_ARMIJO * a * metric) : (Jt < J0);
        if (ok) {
          alpha = a;
          Jn = Jt;
          break;
        }
        a *= SQP_ALPHA_DECAY;
        if (a * dxn < sqp_tol && a * dun < sqp_tol) break;
      }
      if (alpha > 0.0)
        for (int i = 0; i < nu; ++i) u[i] = u[i] + alpha * du[i];
      if (alpha == 0.0 || fabs(Jn - J0) < SQP_COST_TOL || (alpha * dxn < sqp_tol && alpha * dun < sqp_tol)) {
        ++its;
        break;
      }
    }
  }
  if (x) oracle_nlp_rollout_cost(c, x0, xref, foot, contact, u, x, NULL);
  if (qp_iters) *qp_iters = tot;
  if (sqp_iters) *sqp_iters = its;
  free(uq);
  free(ut);
  free(du);
  free(lin);
  return st;
}

/* ------------------------------------------------------------------------------ footholds as variables (§8 a5/f3) */
/* The reference's NLP optimises foot_pos[i] at every node (CentroidalMPC.cpp:132-133) under the swing dynamics
 * foot_pos+ = foot_pos + (1 - e) foot_vel dt (:93, :174-176), the pinning foot_pos(:,0) = current (:165-167), the step
 * box step_lb <= foot_pos - des_foot_pos <= step_ub at nodes 1..N (:196-198, :30-31) and the tracking cost (:218-221).
 * foot_vel is free and uncosted, so a swing node that starts no stance run tracks des exactly, a run that starts at
 * step 0 stays at the current foot, and each LATER stance run (first step s >= 1 after a swing step, last stance step
 * e) holds one free foothold p over its nodes s..e+1. It is parametrised as p = pbar + delta, pbar =
 * oracle_stance_point (the mean of des over the nodes), so the tracking cost is sum_j Wp (pbar + delta - des_j)^2 and
 * the box reads lo <= delta <= hi with lo_d = max_j (des_jd - pbar_d) + step_lb_d, hi_d = min_j (...) + step_ub_d.
 * D [N][L][3] holds delta at index (s, i) of each later run (other entries unused, kept 0). */

static const double STEP_LB[3] = {CMPC_STEP_LB_XY, CMPC_STEP_LB_XY, CMPC_STEP_LB_Z};
static const double STEP_UB[3] = {CMPC_STEP_UB_XY, CMPC_STEP_UB_XY, CMPC_STEP_UB_Z};

/* 1 when step s starts a later stance run of leg i; *e = its last stance step. */
static int later_start(const uint8_t* contact, int N, int L, int s, int i, int* e) {
  if (s < 1 || s >= N || !contact[s * L + i] || contact[(s - 1) * L + i]) return 0;
  int ee = s;
  while (ee + 1 < N && contact[(ee + 1) * L + i]) ++ee;
  if (e) *e = ee;
  return 1;
}

int oracle_foot_box(const double* foot, const uint8_t* contact, int N, int L, int s, int i, double pbar[3],
                    double lo[3], double hi[3], int* cnt) {
  int e = 0;
  if (!later_start(contact, N, L, s, i, &e)) return 0;
  oracle_stance_point(foot, contact, N, L, s, i, pbar);
  for (int d = 0; d < 3; ++d) {
    double mx = -INFINITY, mn = INFINITY;
    for (int j = s; j <= e + 1; ++j) {
      const double v = foot[((size_t)j * L + i) * 3 + d] - pbar[d];
      mx = v > mx ? v : mx;
      mn = v < mn ? v : mn;
    }
    lo[d] = mx + STEP_LB[d];
    hi[d] = mn + STEP_UB[d];
  }
  if (cnt) *cnt = e + 2 - s;
  return 1;
}

/* Feasible start of the footholds: delta = clamp(0, lo, hi) for every later run (D [N][L][3], zeros elsewhere). */
void oracle_feet_init(const oracle_consts* c, const double* foot, const uint8_t* contact, double* D) {
  const int N = c->N, L = c->L;
  memset(D, 0, sizeof(double) * (size_t)N * L * 3);
  for (int s = 1; s < N; ++s)
    for (int i = 0; i < L; ++i) {
      double pb[3], lo[3], hi[3];
      if (!oracle_foot_box(foot, contact, N, L, s, i, pb, lo, hi, NULL)) continue;
      for (int d = 0; d < 3; ++d) D[((size_t)s * L + i) * 3 + d] = fmin(fmax(0.0, lo[d]), hi[d]);
    }
}

/* The reference controller's foot_pos output [(N+1)][L][3] (:269-273) from D: node 0 and the first run's nodes the
 * current foot, a later run's nodes pbar + delta, a free swing node des. */
void oracle_feet_table(const oracle_consts* c, const double* foot, const uint8_t* contact, const double* D,
                       double* out) {
  const int N = c->N, L = c->L;
  for (int j = 0; j <= N; ++j)
    for (int i = 0; i < L; ++i) {
      double* o = out + ((size_t)j * L + i) * 3;
      const double* des = foot + ((size_t)j * L + i) * 3;
      const int k = (j < N && contact[j * L + i]) ? j : ((j > 0 && contact[(j - 1) * L + i]) ? j - 1 : -1);
      if (j == 0) {
        o[0] = des[0], o[1] = des[1], o[2] = des[2];
      } else if (k < 0) {
        o[0] = des[0], o[1] = des[1], o[2] = des[2];
      } else {
        lever_point(foot, contact, D, N, L, k, i, o);
      }
    }
}

/* Condensed QP of the SQP with footholds, linearised at lin = (c_bar_k, F_bar_k) and at the iterate's per-leg forces
 * ubar [N][L][3] and footholds D: variables in the device's order, for each step k and leg i the force triple of a
 * stance (k, i) (tri_map k L + i) and then, when (k, i) starts a later run, its foothold triple (tri_map N L + k L + i,
 * mu = 0, rows [-x, x, -y, y, z] bounded by the step box). Torque (p - c) x f linearised at (pbar + D, c_bar, f_bar):
 * (pbar + D - c_bar) x f + delta x f_bar - D x f_bar - c x F_bar + c_bar x F_bar, so a foothold column acts at each
 * step k of its run on the L rows with dt e_d x f_bar_ik, and b_k gains -dt sum D x f_bar_ik. Cost: the condensed
 * state and force terms as oracle_condense_full_lin, plus 2 Wp cnt on the foothold diagonal and
 * 2 Wp sum_j (pbar - des_j) in g. Status INVALID_CONTACT / TOO_LARGE as oracle_condense_lin, INFEASIBLE_STEP when a
 * later run's box is empty or the current foot of a run from step 0 lies outside the box at one of its nodes. */
int oracle_condense_feet(const oracle_consts* c, const double* x0, const double* xref, const double* foot,
                         const uint8_t* contact, const double* lin, const double* ubar, const double* D, int ld,
                         int* n_out, double* H, double* g, double* tri_mu, double* tri_lo, double* tri_hi,
                         int* tri_map) {
  const int N = c->N, L = c->L;
  const double dt = c->dt;
  *n_out = 0;
  for (int k = 0; k < N; ++k) {
    int ns = 0;
    for (int i = 0; i < L; ++i) ns += contact[k * L + i] ? 1 : 0;
    if (ns == 0) return CMPC_INVALID_CONTACT;
  }
  /* triple list */
  int nt = 0;
  int* code = (int*)malloc(sizeof(int) * (size_t)2 * N * L);
  for (int k = 0; k < N; ++k)
    for (int i = 0; i < L; ++i) {
      if (contact[k * L + i]) code[nt++] = k * L + i;
      if (later_start(contact, N, L, k, i, NULL)) code[nt++] = N * L + k * L + i;
    }
  const int n = 3 * nt;
  if (n > ld) {
    free(code);
    return CMPC_TOO_LARGE;
  }
  double flo[3 * 4 * 64], fhi[3 * 4 * 64];
  for (int t = 0; t < nt; ++t) {
    if (code[t] < N * L) continue;
    const int s = (code[t] - N * L) / L, i = (code[t] - N * L) % L;
    double pb[3];
    oracle_foot_box(foot, contact, N, L, s, i, pb, flo + 3 * t, fhi + 3 * t, NULL);
    for (int d = 0; d < 3; ++d)
      if (!(flo[3 * t + d] <= fhi[3 * t + d])) {
        free(code);
        return CMPC_INFEASIBLE_STEP;
      }
  }
  /* a run from step 0 keeps the current foot (node 0, pinned :165-167) at its nodes 1..e+1, each of which the step box
   * of :196-198 also bounds: a current foot outside it makes the reference NLP infeasible */
  for (int i = 0; i < L; ++i) {
    if (!contact[i]) continue;
    int e = 0;
    while (e + 1 < N && contact[(e + 1) * L + i]) ++e;
    for (int j = 1; j <= e + 1 && j <= N; ++j)
      for (int d = 0; d < 3; ++d) {
        const double v = foot[(size_t)i * 3 + d] - foot[((size_t)j * L + i) * 3 + d];
        if (v < STEP_LB[d] || v > STEP_UB[d]) {
          free(code);
          return CMPC_INFEASIBLE_STEP;
        }
      }
  }
  /* dynamics at the iterate: the force columns' lever arm pbar + D (a foot table whose later-run nodes hold it) */
  double* ft = (double*)malloc(sizeof(double) * (size_t)(N + 1) * L * 3);
  oracle_feet_table(c, foot, contact, D, ft);
  double* A = (double*)malloc(sizeof(double) * N * NX * NX);
  double* B = (double*)malloc(sizeof(double) * N * NX * NU);
  double* bb = (double*)malloc(sizeof(double) * N * NX);
  oracle_srbd_dynamics_lin(c, xref, ft, contact, lin, A, B, bb);
  for (int k = 0; k < N; ++k)
    for (int i = 0; i < L; ++i) {
      if (!contact[k * L + i]) continue;
      int s = k;
      while (s > 0 && contact[(s - 1) * L + i]) --s;
      if (s == 0) continue;
      const double* dl = D + ((size_t)s * L + i) * 3;
      const double* f = ubar + (size_t)k * NU + 3 * i;
      bb[k * NX + 6] -= dt * (dl[1] * f[2] - dl[2] * f[1]);
      bb[k * NX + 7] -= dt * (dl[2] * f[0] - dl[0] * f[2]);
      bb[k * NX + 8] -= dt * (dl[0] * f[1] - dl[1] * f[0]);
    }
  double* G = (double*)calloc((size_t)NX * n, sizeof(double));
  double* G2 = (double*)malloc(sizeof(double) * NX * (n > 0 ? n : 1));
  double xh[NX], xh2[NX], e[NX];
  memcpy(xh, x0, sizeof(xh));
  for (int a = 0; a < ld; ++a) {
    for (int b = 0; b < ld; ++b) H[(size_t)a * ld + b] = 0.0;
    g[a] = 0.0;
  }
  for (int k = 0; k < N; ++k) {
    const double* Ak = A + (size_t)k * NX * NX;
    const double* Bk = B + (size_t)k * NX * NU;
    for (int r = 0; r < NX; ++r) {
      for (int j = 0; j < n; ++j) {
        double sacc = 0.0;
        for (int t = 0; t < NX; ++t) sacc += Ak[r * NX + t] * G[t * n + j];
        G2[r * n + j] = sacc;
      }
      double sacc = 0.0;
      for (int t = 0; t < NX; ++t) sacc += Ak[r * NX + t] * xh[t];
      xh2[r] = sacc + bb[k * NX + r];
    }
    /* input columns acting at step k */
    for (int t = 0; t < nt; ++t) {
      if (code[t] < N * L) {
        if (code[t] / L != k) continue;
        const int i = code[t] % L;
        for (int r = 0; r < NX; ++r)
          for (int d = 0; d < 3; ++d) G2[r * n + 3 * t + d] += Bk[r * NU + 3 * i + d];
      } else {
        const int s = (code[t] - N * L) / L, i = (code[t] - N * L) % L;
        int ee = 0;
        later_start(contact, N, L, s, i, &ee);
        if (k < s || k > ee) continue;
        const double* f = ubar + (size_t)k * NU + 3 * i;
        /* dt e_d x f_bar: e_0 x f = (0, -fz, fy), e_1 x f = (fz, 0, -fx), e_2 x f = (-fy, fx, 0) */
        G2[7 * n + 3 * t + 0] += dt * -f[2];
        G2[8 * n + 3 * t + 0] += dt * f[1];
        G2[6 * n + 3 * t + 1] += dt * f[2];
        G2[8 * n + 3 * t + 1] += dt * -f[0];
        G2[6 * n + 3 * t + 2] += dt * -f[1];
        G2[7 * n + 3 * t + 2] += dt * f[0];
      }
    }
    memcpy(G, G2, sizeof(double) * NX * n);
    memcpy(xh, xh2, sizeof(xh));
    const double* q = c->qdiag[k + 1];
    for (int r = 0; r < NX; ++r) e[r] = q[r] * (xh[r] - xref[(k + 1) * NX + r]);
    for (int a = 0; a < n; ++a) {
      double ga = 0.0;
      for (int r = 0; r < NX; ++r) ga += G[r * n + a] * e[r];
      g[a] += ga;
      for (int b = 0; b <= a; ++b) {
        double sacc = 0.0;
        for (int r = 0; r < NX; ++r) sacc += G[r * n + a] * q[r] * G[r * n + b];
        H[(size_t)a * ld + b] += sacc;
      }
    }
  }
  /* force terms (R-bar, r-bar) and foothold tracking */
  for (int t = 0; t < nt; ++t) {
    if (code[t] < N * L) {
      const int k = code[t] / L, i = code[t] % L;
      int ns = 0;
      for (int l = 0; l < L; ++l) ns += contact[k * L + l] ? 1 : 0;
      const int nb = (k > 0) + (k < N - 1);
      int tn = -1; /* triple of (k + 1, i) */
      if (k + 1 < N && contact[(k + 1) * L + i])
        for (int u2 = t + 1; u2 < nt; ++u2)
          if (code[u2] == (k + 1) * L + i) tn = u2;
      for (int d = 0; d < 3; ++d) {
        const int j = 3 * i + d, a = 3 * t + d;
        H[(size_t)a * ld + a] += 2.0 * c->Wf[j] + 2.0 * c->Wr[j] * (double)nb;
        if (tn >= 0) H[(size_t)(3 * tn + d) * ld + a] += -2.0 * c->Wr[j];
        if (d == 2) g[a] += -2.0 * c->Wf[j] * (c->mass * GRAV / (double)ns);
      }
    } else {
      const int s = (code[t] - N * L) / L, i = (code[t] - N * L) % L;
      double pb[3], lo[3], hi[3];
      int cnt = 0, ee = 0;
      oracle_foot_box(foot, contact, N, L, s, i, pb, lo, hi, &cnt);
      later_start(contact, N, L, s, i, &ee);
      for (int d = 0; d < 3; ++d) {
        const int a = 3 * t + d;
        double gs = 0.0;
        for (int j = s; j <= ee + 1; ++j) gs += pb[d] - foot[((size_t)j * L + i) * 3 + d];
        H[(size_t)a * ld + a] += 2.0 * c->Wp[3 * i + d] * (double)cnt;
        g[a] += 2.0 * c->Wp[3 * i + d] * gs;
      }
    }
  }
  for (int a = 0; a < ld; ++a)
    for (int b = a + 1; b < ld; ++b) H[(size_t)a * ld + b] = H[(size_t)b * ld + a];
  for (int a = n; a < ld; ++a) H[(size_t)a * ld + a] = 1.0;
  for (int t = 0; t < ld / 3; ++t) {
    const int on = t < nt, foot_t = on && code[t] >= N * L;
    if (tri_map) tri_map[t] = on ? code[t] : -1;
    if (tri_mu) tri_mu[t] = (on && !foot_t) ? c->mu[code[t] % L] : 0.0;
    for (int r = 0; r < 5; ++r) {
      double lo = 0.0, hi = c->force_ub[r];
      if (foot_t) {
        const int d = r / 2 < 2 ? r / 2 : 2;
        const int neg = (r == 0 || r == 2);
        lo = neg ? -fhi[3 * t + d] : flo[3 * t + d];
        hi = neg ? -flo[3 * t + d] : fhi[3 * t + d];
      }
      if (tri_lo) tri_lo[t * 5 + r] = lo;
      if (tri_hi) tri_hi[t * 5 + r] = hi;
    }
  }
  *n_out = n;
  free(code);
  free(ft);
  free(A);
  free(B);
  free(bb);
  free(G);
  free(G2);
  return CMPC_SUCCESS;
}

/* One QP of the SQP with footholds: oracle_condense_feet at (lin, u, D), IPM warm-started from (u, D) when
 * s->warm_start, solution scattered back: u [N][L][3] (swing 0) and D (later-run entries). */
int oracle_solve_one_feet(const oracle_consts* c, const cmpc_settings* s, const double* x0, const double* xref,
                          const double* foot, const uint8_t* contact, const double* lin, double* u, double* D,
                          int* iters) {
  const int N = c->N, L = c->L, ld = NU * N;
  double* H = (double*)malloc(sizeof(double) * ld * ld);
  double* g = (double*)malloc(sizeof(double) * ld);
  double* mu = (double*)malloc(sizeof(double) * ld);
  double* lo = (double*)malloc(sizeof(double) * 5 * ld);
  double* hi = (double*)malloc(sizeof(double) * 5 * ld);
  double* uc = (double*)malloc(sizeof(double) * ld);
  int* map = (int*)malloc(sizeof(int) * ld);
  double* ub = (double*)malloc(sizeof(double) * N * NU);
  double* Db = (double*)malloc(sizeof(double) * N * NU);
  memcpy(ub, u, sizeof(double) * N * NU);
  memcpy(Db, D, sizeof(double) * N * NU);
  int n = 0, it = 0;
  int st = oracle_condense_feet(c, x0, xref, foot, contact, lin, ub, Db, ld, &n, H, g, mu, lo, hi, map);
  if (st == CMPC_SUCCESS) {
    for (int t = 0; t < n / 3; ++t) {
      const double* src = map[t] < N * L ? ub + map[t] * 3 : Db + (map[t] - N * L) * 3;
      for (int d = 0; d < 3; ++d) uc[3 * t + d] = s->warm_start ? src[d] : 0.0;
    }
    st = oracle_qp_ipm(n, ld, H, g, mu, lo, hi, s, uc, NULL, NULL, &it, NULL);
    memset(u, 0, sizeof(double) * N * NU);
    memset(D, 0, sizeof(double) * N * NU);
    for (int t = 0; t < n / 3; ++t) {
      double* dst = map[t] < N * L ? u + map[t] * 3 : D + (map[t] - N * L) * 3;
      for (int d = 0; d < 3; ++d) dst[d] = uc[3 * t + d];
    }
  }
  if (iters) *iters = it;
  free(H);
  free(g);
  free(mu);
  free(lo);
  free(hi);
  free(uc);
  free(map);
  free(ub);
  free(Db);
  return st;
}

/* oracle_sqp_solve with the later runs' footholds as decision variables (the reference's NLP, CentroidalMPC.cpp:
 * 132-133, 196-198, 218-221): U_0 = the QP at the reference linearisation (frozen footholds, where the foothold
 * columns vanish: F_bar = 0), D_0 = oracle_feet_init; each iteration solves oracle_solve_one_feet at the iterate and
 * line-searches (U, D) jointly, |du| over forces and footholds. feet [(N+1)][L][3] (may be NULL): oracle_feet_table of
 * the final D. */
int oracle_sqp_solve_feet(const oracle_consts* c, const cmpc_settings* s, int sqp_iter_max, double sqp_tol,
                          const double* x0, const double* xref, const double* foot, const uint8_t* contact, double* u,
                          double* D, double* feet, double* x, int* qp_iters, int* sqp_iters) {
  const int N = c->N, nu = N * NU;
  double* uq = (double*)malloc(sizeof(double) * nu);
  double* ut = (double*)malloc(sizeof(double) * nu);
  double* du = (double*)malloc(sizeof(double) * nu);
  double* Dq = (double*)malloc(sizeof(double) * nu);
  double* Dt = (double*)malloc(sizeof(double) * nu);
  double* dD = (double*)malloc(sizeof(double) * nu);
  double* lin = (double*)malloc(sizeof(double) * N * 6);
  cmpc_settings sw = *s;
  sw.warm_start = 0;
  int it = 0, its = 0;
  int st = oracle_solve_one_lin(c, &sw, x0, xref, foot, contact, NULL, u, NULL, &it);
  oracle_feet_init(c, foot, contact, D);
  int tot = it;
  if (st == CMPC_SUCCESS) {
    sw.warm_start = 1;
    for (its = 0; its < sqp_iter_max; ++its) {
      const double J0 = oracle_nlp_rollout_cost_feet(c, x0, xref, foot, contact, u, D, NULL, lin);
      memcpy(uq, u, sizeof(double) * nu);
      memcpy(Dq, D, sizeof(double) * nu);
      const int sq = oracle_solve_one_feet(c, &sw, x0, xref, foot, contact, lin, uq, Dq, &it);
      tot += it;
      if (sq != CMPC_SUCCESS) {
        st = sq;
        break;
      }
      double dun2 = 0.0;
      for (int i = 0; i < nu; ++i) {
        du[i] = uq[i] - u[i];
        dun2 += du[i] * du[i];
      }
      for (int i = 0; i < nu; ++i) {
        dD[i] = Dq[i] - D[i];
        dun2 += dD[i] * dD[i];
      }
      const double dun = sqrt(dun2);
      double dxn = 0.0, metric = 0.0;
      oracle_nlp_linstep_feet(c, x0, xref, foot, contact, u, D, du, dD, &dxn, &metric);
      double alpha = 0.0, Jn = J0;
      for (double a = 1.0; a >= SQP_ALPHA_MIN;) {
        for (int i = 0; i < nu; ++i) {
          ut[i] = u[i] + a * du[i];
          Dt[i] = D[i] + a * dD[i];
        }
        const double Jt = oracle_nlp_rollout_cost_feet(c, x0, xref, foot, contact, ut, Dt, NULL, NULL);
        const int ok = metric < 0.0 ? (Jt < J0 + SQP_ARMIJO * a * metric) : (Jt < J0);
        if (ok) {
          alpha = a;
          Jn = Jt;
          break;
        }
        a *= SQP_ALPHA_DECAY;
        if (a * dxn < sqp_tol && a * dun < sqp_tol) break;
      }
      if (alpha > 0.0)
        for (int i = 0; i < nu; ++i) {
          u[i] = u[i] + alpha * du[i];
          D[i] = D[i] + alpha * dD[i];
        }
      if (alpha == 0.0 || fabs(Jn - J0) < SQP_COST_TOL || (alpha * dxn < sqp_tol && alpha * dun < sqp_tol)) {
        ++its;
        break;
      }
    }
  }
  if (x) oracle_nlp_rollout_cost_feet(c, x0, xref, foot, contact, u, D, x, NULL);
  if (feet) oracle_feet_table(c, foot, contact, D, feet);
  if (qp_iters) *qp_iters = tot;
  if (sqp_iters) *sqp_iters = its;
  free(uq);
  free(ut);
  free(du);
  free(Dq);
  free(Dt);
  free(dD);
  free(lin);
  return st;
}

/* ------------------------------------------------------------------------------------------------ policy */

/* Null space of the active pyramid rows of one force triple (the condensed analogue of HPIPM's Riccati feedback at
 * the solution, HpipmInterface.cpp:330-455, in its mu -> 0 limit: an active row has Sigma = lambda / s -> inf, so
 * the triple may only move inside the null space of its active rows). Row r is active when its slack to lo = 0 or
 * to hi = ub[r] is <= tol. Active rows are orthonormalised in order r = 0..4 (modified Gram-Schmidt, a row whose
 * residual is below 1e-6 of its norm is dependent); the free directions are then taken greedily from e_0, e_1, e_2,
 * each time the unit vector with the largest residual against everything chosen so far. Z[a*3 + c] = component a of
 * free direction c. Returns the number of free directions (0..3). The device kernel k_policy applies the same rule. */
int oracle_policy_triple(double mu, const double* ub, const double* f, double tol, double* Z) {
  const double nr[5][3] = {{-1.0, 0.0, mu}, {1.0, 0.0, mu}, {0.0, -1.0, mu}, {0.0, 1.0, mu}, {0.0, 0.0, 1.0}};
  double Q[3][3];
  int nq = 0;
  for (int r = 0; r < 5 && nq < 3; ++r) {
    const double v = nr[r][0] * f[0] + nr[r][1] * f[1] + nr[r][2] * f[2];
    if (!(v <= tol || ub[r] - v <= tol)) continue;
    double w[3] = {nr[r][0], nr[r][1], nr[r][2]};
    const double n0 = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    for (int p = 0; p < nq; ++p) {
      const double d = Q[p][0] * w[0] + Q[p][1] * w[1] + Q[p][2] * w[2];
      for (int a = 0; a < 3; ++a) w[a] -= d * Q[p][a];
    }
    const double nw = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    if (!(nw > 1e-6 * n0)) continue;
    for (int a = 0; a < 3; ++a) Q[nq][a] = w[a] / nw;
    ++nq;
  }
  const int rank = nq;
  for (int c = 0; c < 3 - rank; ++c) {
    double best[3] = {0.0, 0.0, 0.0}, bn = -1.0;
    for (int e = 0; e < 3; ++e) {
      double w[3] = {0.0, 0.0, 0.0};
      w[e] = 1.0;
      for (int p = 0; p < nq; ++p) {
        const double d = Q[p][0] * w[0] + Q[p][1] * w[1] + Q[p][2] * w[2];
        for (int a = 0; a < 3; ++a) w[a] -= d * Q[p][a];
      }
      const double nw = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
      if (nw > bn) {
        bn = nw;
        for (int a = 0; a < 3; ++a) best[a] = w[a];
      }
    }
    for (int a = 0; a < 3; ++a) Q[nq][a] = best[a] / bn;
    for (int a = 0; a < 3; ++a) Z[a * 3 + c] = Q[nq][a];
    ++nq;
  }
  return 3 - rank;
}

/* dU/dx0 of the condensed QP at its solution u [N][L][3] (swing entries ignored): K [12N][13] row-major, row
 * 12k + 3i + a = d u_{k,i,a} / d x0. g(x0) = Bqp' Q (Aqp x0 - X_ref) + r is affine in x0 with slope
 * F = Bqp' Q Aqp (the free response of SURVEY App. A.3), H does not depend on x0, so on a fixed active set
 *   K = -Z (Z' H Z)^{-1} Z' F,   Z = blkdiag of the per-triple free directions (oracle_policy_triple);
 * swing rows are 0 (those forces are eliminated). This is the condensed counterpart of HPIPM's Riccati
 * feedback/feedforward getters (HpipmInterface.cpp:330-455) that ocs2 uses as the feedback policy
 * (MultipleShootingSolver.cpp:334-362, useFeedbackPolicy, MultipleShootingSettings.h:57). *n_free = dim(Z).
 * Returns CMPC_SUCCESS, CMPC_INVALID_CONTACT, or CMPC_NAN_SOL when Z' H Z is not positive definite. */
int oracle_policy(const oracle_consts* c, const double* xref, const double* foot, const uint8_t* contact,
                  const double* u, double act_tol, double* K, int* n_free) {
  return oracle_policy_lin(c, xref, foot, contact, NULL, u, act_tol, K, n_free);
}

/* Same for the QP linearised at lin [N][6] (oracle_srbd_dynamics_lin; NULL: the reference linearisation): the
 * feedback of the SQP's subproblem at its solution (ocs2 reads the Riccati gains of the last QP,
 * MultipleShootingSolver.cpp:334-362). The linearisation point is held fixed, as HPIPM's factorisation is. */
int oracle_policy_lin(const oracle_consts* c, const double* xref, const double* foot, const uint8_t* contact,
                      const double* lin, const double* u, double act_tol, double* K, int* n_free) {
  const int N = c->N, L = c->L, nf = NU * N;
  *n_free = 0;
  memset(K, 0, sizeof(double) * nf * NX);
  double* Hf = (double*)malloc(sizeof(double) * nf * nf);
  double* gf = (double*)malloc(sizeof(double) * nf);
  double x0z[NX] = {0};
  int st = oracle_condense_full_lin(c, x0z, xref, foot, contact, lin, Hf, gf);
  if (st != CMPC_SUCCESS) {
    free(Hf);
    free(gf);
    return st;
  }
  /* F = sum_k G_k' Q_{k+1} P_{k+1}, P_{k+1} = A_k P_k (P_0 = I), G_{k+1} = A_k G_k + [B_k at step k] */
  double* A = (double*)malloc(sizeof(double) * N * NX * NX);
  double* Bm = (double*)malloc(sizeof(double) * N * NX * NU);
  oracle_srbd_dynamics_lin(c, xref, foot, contact, lin, A, Bm, NULL);
  double* G = (double*)calloc((size_t)NX * nf, sizeof(double));
  double* G2 = (double*)malloc(sizeof(double) * NX * nf);
  double* F = (double*)calloc((size_t)nf * NX, sizeof(double));
  double P[NX * NX], P2[NX * NX];
  memset(P, 0, sizeof(P));
  for (int r = 0; r < NX; ++r) P[r * NX + r] = 1.0;
  for (int k = 0; k < N; ++k) {
    const double* Ak = A + (size_t)k * NX * NX;
    const double* Bk = Bm + (size_t)k * NX * NU;
    for (int r = 0; r < NX; ++r) {
      for (int j = 0; j < nf; ++j) {
        double s = 0.0;
        for (int t = 0; t < NX; ++t) s += Ak[r * NX + t] * G[t * nf + j];
        G2[r * nf + j] = s;
      }
      for (int j = 0; j < NU; ++j) G2[r * nf + NU * k + j] += Bk[r * NU + j];
      for (int j = 0; j < NX; ++j) {
        double s = 0.0;
        for (int t = 0; t < NX; ++t) s += Ak[r * NX + t] * P[t * NX + j];
        P2[r * NX + j] = s;
      }
    }
    memcpy(G, G2, sizeof(double) * NX * nf);
    memcpy(P, P2, sizeof(P));
    const double* q = c->qdiag[k + 1];
    for (int a = 0; a < NU * (k + 1); ++a)
      for (int j = 0; j < NX; ++j) {
        double s = 0.0;
        for (int r = 0; r < NX; ++r) s += G[r * nf + a] * q[r] * P[r * NX + j];
        F[a * NX + j] += s;
      }
  }
  /* free directions of every stance triple */
  int nt = 0;
  int* idx = (int*)malloc(sizeof(int) * N * L);
  int* off = (int*)malloc(sizeof(int) * (N * L + 1));
  double* Z = (double*)calloc((size_t)N * L * 9, sizeof(double));
  int* kt = (int*)malloc(sizeof(int) * N * L);
  int m = 0;
  for (int k = 0; k < N; ++k)
    for (int i = 0; i < L; ++i) {
      if (!contact[k * L + i]) continue;
      idx[nt] = NU * k + 3 * i;
      off[nt] = m;
      kt[nt] = oracle_policy_triple(c->mu[i], c->force_ub, u + ((size_t)k * L + i) * 3, act_tol, Z + nt * 9);
      m += kt[nt];
      ++nt;
    }
  double* Hr = (double*)malloc(sizeof(double) * (m > 0 ? m * m : 1));
  double* Y = (double*)malloc(sizeof(double) * (m > 0 ? m * NX : 1));
  for (int t1 = 0; t1 < nt; ++t1)
    for (int c1 = 0; c1 < kt[t1]; ++c1) {
      const int r1 = off[t1] + c1;
      for (int t2 = 0; t2 < nt; ++t2)
        for (int c2 = 0; c2 < kt[t2]; ++c2) {
          double s = 0.0;
          for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b)
              s += Z[t1 * 9 + a * 3 + c1] * Hf[(size_t)(idx[t1] + a) * nf + idx[t2] + b] * Z[t2 * 9 + b * 3 + c2];
          Hr[r1 * m + off[t2] + c2] = s;
        }
      for (int j = 0; j < NX; ++j) {
        double s = 0.0;
        for (int a = 0; a < 3; ++a) s += Z[t1 * 9 + a * 3 + c1] * F[(idx[t1] + a) * NX + j];
        Y[r1 * NX + j] = -s;
      }
    }
  st = CMPC_SUCCESS;
  if (m > 0 && oracle_cholesky(m, Hr, m) != 0) st = CMPC_NAN_SOL;
  if (st == CMPC_SUCCESS && m > 0) {
    double* col = (double*)malloc(sizeof(double) * m);
    for (int j = 0; j < NX; ++j) {
      for (int r = 0; r < m; ++r) col[r] = Y[r * NX + j];
      oracle_chol_solve(m, Hr, m, col);
      for (int r = 0; r < m; ++r) Y[r * NX + j] = col[r];
    }
    free(col);
    for (int t = 0; t < nt; ++t)
      for (int a = 0; a < 3; ++a)
        for (int j = 0; j < NX; ++j) {
          double s = 0.0;
          for (int cc = 0; cc < kt[t]; ++cc) s += Z[t * 9 + a * 3 + cc] * Y[(off[t] + cc) * NX + j];
          K[(size_t)(idx[t] + a) * NX + j] = s;
        }
  }
  *n_free = m;
  free(Hf); free(gf); free(A); free(Bm); free(G); free(G2); free(F);
  free(idx); free(off); free(Z); free(kt); free(Hr); free(Y);
  return st;
}

/* ------------------------------------------------------------------------------------------------ Riccati IPM */

/* The same QP solved the way HPIPM solves the reference's OCP (d_ocp_qp_ipm_solve, HpipmInterface.cpp:282-284;
 * ric_alg 0, HpipmInterfaceSettings.h:56): no condensing. The Newton system (H + C' Sigma C + reg I) du = b is the
 * KKT system of an OCP over the stages with state z_k = [x_k (13); u_{k-1} (12, the previous forces, which carry
 * the force-rate coupling of CentroidalMPC.cpp:227-231)], input v_k = the stance forces of step k, z_0 = 0:
 *   z_{k+1} = blkdiag(A_k, 0) z_k + [B_k S_k; S_k] v_k        (S_k: stance selection, 12 x 3 ns_k)
 *   stage   1/2 x'diag(q_k)x [k >= 1] + sum_j Wr_j (S v - u_prev)_j^2 [k >= 1] + sum_j Wf_j (S v)_j^2
 *           + 1/2 v'(C'Sigma C + reg I)v - b_k'v;            terminal 1/2 x_N'diag(q_N) x_N,
 * solved by the backward Riccati recursion and a forward sweep; H u + g is a rollout plus an adjoint sweep.
 * O(N (25^3 + 25^2 nu)) per iteration instead of O(n^3): an independent restatement of the same optimum (its
 * iterates agree with oracle_qp_ipm to rounding) and the CPU line closest to the reference's own solver. */
#define NZ (NX + NU)

typedef struct ric_ops_ctx {
  const oracle_consts* c;
  int N;
  const double *A, *B, *x0, *xref, *fdes; /* A [N][13][13], B [N][13][12], fdes [N][L] (z) */
  int nu[64], off[64], nst[64], legs[64][CMPC_MAX_LEGS];
  double *Bt; /* [N][NZ][12]  B~_k (first nu_k columns used) */
  double *St; /* [N][12][NZ] */
  double *Kf; /* [N][12][NZ] */
  double *Lr; /* [N][12][12] Cholesky of Rt_k, and Lri [N][12] = 1 / L_ii */
  double *Lri;
  double *P;  /* scratch [NZ][NZ] x 2 */
  int n;
} ric_ops_ctx;

static void ric_grad(void* vc, const double* u, double* hug) {
  const ric_ops_ctx* r = (const ric_ops_ctx*)vc;
  const oracle_consts* c = r->c;
  const int N = r->N, L = c->L;
  double* uf = (double*)calloc((size_t)N * NU, sizeof(double));
  double* X = (double*)malloc(sizeof(double) * (N + 1) * NX);
  for (int k = 0; k < N; ++k)
    for (int t = 0; t < r->nst[k]; ++t)
      for (int d = 0; d < 3; ++d) uf[k * NU + 3 * r->legs[k][t] + d] = u[r->off[k] + 3 * t + d];
  memcpy(X, r->x0, sizeof(double) * NX);
  for (int k = 0; k < N; ++k)
    for (int i = 0; i < NX; ++i) {
      double acc = 0.0;
      for (int t = 0; t < NX; ++t) acc += r->A[(size_t)k * NX * NX + i * NX + t] * X[k * NX + t];
      for (int j = 0; j < NU; ++j) acc += r->B[(size_t)k * NX * NU + i * NU + j] * uf[k * NU + j];
      X[(k + 1) * NX + i] = acc;
    }
  double lam[NX], lam2[NX], gk[NU];
  for (int i = 0; i < NX; ++i) lam[i] = c->qdiag[N][i] * (X[N * NX + i] - r->xref[N * NX + i]);
  for (int k = N - 1; k >= 0; --k) {
    for (int j = 0; j < NU; ++j) {
      double acc = 0.0;
      for (int i = 0; i < NX; ++i) acc += r->B[(size_t)k * NX * NU + i * NU + j] * lam[i];
      const double fd = (j % 3 == 2) ? r->fdes[k * L + j / 3] : 0.0;
      acc += 2.0 * c->Wf[j] * (uf[k * NU + j] - fd);
      if (k > 0) acc += 2.0 * c->Wr[j] * (uf[k * NU + j] - uf[(k - 1) * NU + j]);
      if (k < N - 1) acc -= 2.0 * c->Wr[j] * (uf[(k + 1) * NU + j] - uf[k * NU + j]);
      gk[j] = acc;
    }
    for (int t = 0; t < r->nst[k]; ++t)
      for (int d = 0; d < 3; ++d) hug[r->off[k] + 3 * t + d] = gk[3 * r->legs[k][t] + d];
    if (k > 0) {
      for (int i = 0; i < NX; ++i) {
        double acc = c->qdiag[k][i] * (X[k * NX + i] - r->xref[k * NX + i]);
        for (int t = 0; t < NX; ++t) acc += r->A[(size_t)k * NX * NX + t * NX + i] * lam[t];
        lam2[i] = acc;
      }
      memcpy(lam, lam2, sizeof(lam));
    }
  }
  free(uf);
  free(X);
}

static int ric_factor(void* vc, int nt, const double* tri_mu, const double* lla, const double* lua,
                      const double* tla, const double* tua, double reg) {
  ric_ops_ctx* r = (ric_ops_ctx*)vc;
  const oracle_consts* c = r->c;
  const int N = r->N;
  double* P = r->P;
  double* Pn = r->P + NZ * NZ;
  double PB[NZ * NU], PA[NZ * NX], Rt[NU * NU];
  (void)nt;
  memset(P, 0, sizeof(double) * NZ * NZ);
  for (int i = 0; i < NX; ++i) P[i * NZ + i] = c->qdiag[N][i];
  for (int k = N - 1; k >= 0; --k) {
    const int m = r->nu[k];
    const double* Ak = r->A + (size_t)k * NX * NX;
    const double* Bt = r->Bt + (size_t)k * NZ * NU;
    double* St = r->St + (size_t)k * NU * NZ;
    double* Kf = r->Kf + (size_t)k * NU * NZ;
    double* Lr = r->Lr + (size_t)k * NU * NU;
    double* Lri = r->Lri + (size_t)k * NU;
    for (int i = 0; i < NZ; ++i) {
      for (int j = 0; j < m; ++j) {
        double acc = 0.0;
        for (int t = 0; t < NZ; ++t) acc += P[i * NZ + t] * Bt[t * NU + j];
        PB[i * NU + j] = acc;
      }
      for (int j = 0; j < NX; ++j) {
        double acc = 0.0;
        for (int t = 0; t < NX; ++t) acc += P[i * NZ + t] * Ak[t * NX + j];
        PA[i * NX + j] = acc;
      }
    }
    /* Rt = R_k + B~' P B~, R_k = diag(2 Wf + 2 Wr [k >= 1]) + C'Sigma C + reg I on the stance triples */
    for (int a = 0; a < m; ++a)
      for (int b = 0; b < m; ++b) {
        double acc = 0.0;
        for (int t = 0; t < NZ; ++t) acc += Bt[t * NU + a] * PB[t * NU + b];
        Rt[a * NU + b] = acc;
      }
    for (int tt = 0; tt < r->nst[k]; ++tt) {
      const int tg = r->off[k] / 3 + tt, b = 3 * tt;
      const double* ll = lla + 5 * tg;
      const double* lu = lua + 5 * tg;
      const double* tl = tla + 5 * tg;
      const double* tu = tua + 5 * tg;
      double sg[5];
      for (int q = 0; q < 5; ++q) sg[q] = ll[q] / tl[q] + lu[q] / tu[q];
      const double mu_t = tri_mu[tg];
      Rt[b * NU + b] += sg[0] + sg[1];
      Rt[(b + 1) * NU + b + 1] += sg[2] + sg[3];
      Rt[(b + 2) * NU + b + 2] += mu_t * mu_t * (sg[0] + sg[1] + sg[2] + sg[3]) + sg[4];
      const double xz = mu_t * (-sg[0] + sg[1]), yz = mu_t * (-sg[2] + sg[3]);
      Rt[b * NU + b + 2] += xz;
      Rt[(b + 2) * NU + b] += xz;
      Rt[(b + 1) * NU + b + 2] += yz;
      Rt[(b + 2) * NU + b + 1] += yz;
      for (int d = 0; d < 3; ++d) {
        const int j = 3 * r->legs[k][tt] + d;
        Rt[(b + d) * NU + b + d] += 2.0 * c->Wf[j] + (k > 0 ? 2.0 * c->Wr[j] : 0.0) + reg;
      }
    }
    /* St = S_k + B~' P A~ (A~ = blkdiag(A_k, 0)); S_k = -2 Wr on the u_prev columns (k >= 1) */
    for (int a = 0; a < m; ++a) {
      for (int j = 0; j < NZ; ++j) {
        double acc = 0.0;
        if (j < NX)
          for (int t = 0; t < NZ; ++t) acc += Bt[t * NU + a] * PA[t * NX + j];
        St[a * NZ + j] = acc;
      }
      if (k > 0) {
        const int jl = 3 * r->legs[k][a / 3] + a % 3;
        St[a * NZ + NX + jl] += -2.0 * c->Wr[jl];
      }
    }
    /* Cholesky of Rt with the kernels' pivot guard */
    for (int a = 0; a < m; ++a)
      for (int b = 0; b < m; ++b) Lr[a * NU + b] = Rt[a * NU + b];
    for (int q = 0; q < m; ++q) {
      double d = Lr[q * NU + q];
      for (int j = 0; j < q; ++j) d -= Lr[q * NU + j] * Lr[q * NU + j];
      if (d != d) return -1;
      const double il = d > 1e-200 ? 1.0 / sqrt(d) : 0.0;
      Lr[q * NU + q] = d > 1e-200 ? sqrt(d) : 0.0;
      Lri[q] = il;
      for (int i = q + 1; i < m; ++i) {
        double sacc = Lr[i * NU + q];
        for (int j = 0; j < q; ++j) sacc -= Lr[i * NU + j] * Lr[q * NU + j];
        Lr[i * NU + q] = sacc * il;
      }
    }
    /* K = -Rt^{-1} St, column by column */
    for (int j = 0; j < NZ; ++j) {
      double col[NU];
      for (int a = 0; a < m; ++a) col[a] = St[a * NZ + j];
      for (int a = 0; a < m; ++a) {
        double sacc = col[a];
        for (int b = 0; b < a; ++b) sacc -= Lr[a * NU + b] * col[b];
        col[a] = sacc * Lri[a];
      }
      for (int a = m - 1; a >= 0; --a) {
        double sacc = col[a];
        for (int b = a + 1; b < m; ++b) sacc -= Lr[b * NU + a] * col[b];
        col[a] = sacc * Lri[a];
      }
      for (int a = 0; a < m; ++a) Kf[a * NZ + j] = -col[a];
    }
    /* P_k = Q_k + A~' P A~ + St' K */
    for (int i = 0; i < NZ; ++i)
      for (int j = 0; j < NZ; ++j) {
        double acc = 0.0;
        if (i < NX && j < NX)
          for (int t = 0; t < NX; ++t) acc += Ak[t * NX + i] * PA[t * NX + j];
        for (int a = 0; a < m; ++a) acc += St[a * NZ + i] * Kf[a * NZ + j];
        Pn[i * NZ + j] = acc;
      }
    if (k > 0) {
      for (int i = 0; i < NX; ++i) Pn[i * NZ + i] += c->qdiag[k][i];
      for (int j = 0; j < NU; ++j) Pn[(NX + j) * NZ + NX + j] += 2.0 * c->Wr[j];
    }
    for (int i = 0; i < NZ; ++i)
      for (int j = 0; j < i; ++j) {
        const double v = 0.5 * (Pn[i * NZ + j] + Pn[j * NZ + i]);
        Pn[i * NZ + j] = v;
        Pn[j * NZ + i] = v;
      }
    double* tmp = P;
    P = Pn;
    Pn = tmp;
  }
  return 0;
}

static void ric_solve(void* vc, double* bvec) {
  const ric_ops_ctx* r = (const ric_ops_ctx*)vc;
  const int N = r->N;
  double p[NZ], p2[NZ], z[NZ], z2[NZ];
  double* kff = (double*)malloc(sizeof(double) * N * NU);
  memset(p, 0, sizeof(p));
  for (int k = N - 1; k >= 0; --k) {
    const int m = r->nu[k];
    const double* Ak = r->A + (size_t)k * NX * NX;
    const double* Bt = r->Bt + (size_t)k * NZ * NU;
    const double* St = r->St + (size_t)k * NU * NZ;
    const double* Lr = r->Lr + (size_t)k * NU * NU;
    const double* Lri = r->Lri + (size_t)k * NU;
    double col[NU];
    for (int a = 0; a < m; ++a) {
      double acc = -bvec[r->off[k] + a];
      for (int t = 0; t < NZ; ++t) acc += Bt[t * NU + a] * p[t];
      col[a] = acc;
    }
    for (int a = 0; a < m; ++a) {
      double sacc = col[a];
      for (int b = 0; b < a; ++b) sacc -= Lr[a * NU + b] * col[b];
      col[a] = sacc * Lri[a];
    }
    for (int a = m - 1; a >= 0; --a) {
      double sacc = col[a];
      for (int b = a + 1; b < m; ++b) sacc -= Lr[b * NU + a] * col[b];
      col[a] = sacc * Lri[a];
    }
    for (int a = 0; a < m; ++a) kff[k * NU + a] = -col[a];
    for (int i = 0; i < NZ; ++i) {
      double acc = 0.0;
      if (i < NX)
        for (int t = 0; t < NX; ++t) acc += Ak[t * NX + i] * p[t];
      for (int a = 0; a < m; ++a) acc += St[a * NZ + i] * kff[k * NU + a];
      p2[i] = acc;
    }
    memcpy(p, p2, sizeof(p));
  }
  memset(z, 0, sizeof(z));
  for (int k = 0; k < N; ++k) {
    const int m = r->nu[k];
    const double* Ak = r->A + (size_t)k * NX * NX;
    const double* Bt = r->Bt + (size_t)k * NZ * NU;
    const double* Kf = r->Kf + (size_t)k * NU * NZ;
    double v[NU];
    for (int a = 0; a < m; ++a) {
      double acc = kff[k * NU + a];
      for (int j = 0; j < NZ; ++j) acc += Kf[a * NZ + j] * z[j];
      v[a] = acc;
      bvec[r->off[k] + a] = acc;
    }
    for (int i = 0; i < NZ; ++i) {
      double acc = 0.0;
      if (i < NX)
        for (int t = 0; t < NX; ++t) acc += Ak[i * NX + t] * z[t];
      for (int a = 0; a < m; ++a) acc += Bt[i * NU + a] * v[a];
      z2[i] = acc;
    }
    memcpy(z, z2, sizeof(z));
  }
  free(kff);
}

int oracle_riccati_solve_one(const oracle_consts* c, const cmpc_settings* s, const double* x0, const double* xref,
                             const double* foot, const uint8_t* contact, double* u, int* iters) {
  const int N = c->N, L = c->L;
  memset(u, 0, sizeof(double) * N * NU);
  if (iters) *iters = 0;
  if (N > 63) return CMPC_TOO_LARGE;
  double* fdes = (double*)malloc(sizeof(double) * N * L);
  int st = fdes_and_check(c, contact, fdes);
  if (st != CMPC_SUCCESS) {
    free(fdes);
    return st;
  }
  ric_ops_ctx r;
  memset(&r, 0, sizeof(r));
  r.c = c;
  r.N = N;
  r.x0 = x0;
  r.xref = xref;
  r.fdes = fdes;
  double* A = (double*)malloc(sizeof(double) * N * NX * NX);
  double* Bm = (double*)malloc(sizeof(double) * N * NX * NU);
  oracle_srbd_dynamics(c, xref, foot, contact, A, Bm);
  r.A = A;
  r.B = Bm;
  int n = 0;
  for (int k = 0; k < N; ++k) {
    r.off[k] = n;
    r.nst[k] = 0;
    for (int i = 0; i < L; ++i)
      if (contact[k * L + i]) r.legs[k][r.nst[k]++] = i;
    r.nu[k] = 3 * r.nst[k];
    n += r.nu[k];
  }
  r.n = n;
  double* mem = (double*)calloc((size_t)N * (NZ * NU * 3 + NU * NU + NU) + 2 * NZ * NZ, sizeof(double));
  r.Bt = mem;
  r.St = r.Bt + (size_t)N * NZ * NU;
  r.Kf = r.St + (size_t)N * NU * NZ;
  r.Lr = r.Kf + (size_t)N * NU * NZ;
  r.Lri = r.Lr + (size_t)N * NU * NU;
  r.P = r.Lri + (size_t)N * NU;
  for (int k = 0; k < N; ++k) /* B~_k = [B_k S_k; S_k] */
    for (int t = 0; t < r.nst[k]; ++t)
      for (int d = 0; d < 3; ++d) {
        const int a = 3 * t + d, j = 3 * r.legs[k][t] + d;
        for (int i = 0; i < NX; ++i) r.Bt[(size_t)k * NZ * NU + i * NU + a] = Bm[(size_t)k * NX * NU + i * NU + j];
        r.Bt[(size_t)k * NZ * NU + (NX + j) * NU + a] = 1.0;
      }
  const int nt = n / 3;
  double* mu = (double*)malloc(sizeof(double) * (nt + 1));
  double* lo = (double*)calloc(5 * (size_t)(nt + 1), sizeof(double));
  double* hi = (double*)malloc(sizeof(double) * 5 * (nt + 1));
  double* uc = (double*)calloc((size_t)n + 1, sizeof(double));
  for (int k = 0, t = 0; k < N; ++k)
    for (int q = 0; q < r.nst[k]; ++q, ++t) {
      mu[t] = c->mu[r.legs[k][q]];
      for (int j = 0; j < 5; ++j) hi[5 * t + j] = c->force_ub[j];
    }
  qp_ops ops = {&r, ric_grad, ric_factor, ric_solve};
  cmpc_settings s2 = *s;
  s2.warm_start = 0;
  int it = 0;
  st = qp_ipm_run(n, &ops, mu, lo, hi, &s2, uc, NULL, NULL, &it, NULL, NULL, 0);
  for (int k = 0; k < N; ++k)
    for (int t = 0; t < r.nst[k]; ++t)
      for (int d = 0; d < 3; ++d) u[(k * L + r.legs[k][t]) * 3 + d] = uc[r.off[k] + 3 * t + d];
  if (iters) *iters = it;
  free(fdes); free(A); free(Bm); free(mem); free(mu); free(lo); free(hi); free(uc);
  return st;
}

typedef struct ric_job {
  const oracle_consts* c;
  const cmpc_settings* s;
  int B, tid, nthreads;
  const double *x0, *xref, *foot;
  const uint8_t* contact;
  double* u;
  int *status, *iters;
} ric_job;

static void* ric_worker(void* arg) {
  ric_job* j = (ric_job*)arg;
  const int N = j->c->N, L = j->c->L;
  for (int q = j->tid; q < j->B; q += j->nthreads) {
    int it = 0;
    const int st = oracle_riccati_solve_one(j->c, j->s, j->x0 + (size_t)q * NX, j->xref + (size_t)q * (N + 1) * NX,
                                            j->foot + (size_t)q * (N + 1) * L * 3, j->contact + (size_t)q * N * L,
                                            j->u + (size_t)q * N * NU, &it);
    if (j->status) j->status[q] = st;
    if (j->iters) j->iters[q] = it;
  }
  return NULL;
}

int oracle_riccati_solve_batch(const cmpc_model* m, const cmpc_settings* s, int B, const double* x0,
                               const double* xref, const double* foot, const uint8_t* contact, double* u,
                               int* status, int* iters, int nthreads) {
  oracle_consts c;
  oracle_consts_init(m, &c);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  ric_job jobs[256];
  pthread_t th[256];
  for (int t = 0; t < nthreads; ++t) {
    ric_job jb = {&c, s, B, t, nthreads, x0, xref, foot, contact, u, status, iters};
    jobs[t] = jb;
  }
  if (nthreads == 1) {
    ric_worker(&jobs[0]);
    return 0;
  }
  for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, ric_worker, &jobs[t]);
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  return 0;
}

/* Stage-0 Riccati feedback of the unconstrained problem (Sigma = 0, no regularisation): rows of the stance forces of
 * step 0, columns x0 (K0 [L][3][13], swing rows 0) — the matrix HPIPM's getRiccatiFeedback(0) returns for the
 * reference's OCP (HpipmInterface.cpp:330-455, test retrieveRiccati testHpipmInterface.cpp:258-340) when no
 * inequality is active; the condensed policy of oracle_policy must equal it on such a QP. */
int oracle_riccati_gain0(const oracle_consts* c, const double* xref, const double* foot, const uint8_t* contact,
                         double* K0) {
  const int N = c->N, L = c->L;
  memset(K0, 0, sizeof(double) * NU * NX);
  double* fdes = (double*)malloc(sizeof(double) * N * L);
  int st = fdes_and_check(c, contact, fdes);
  if (st != CMPC_SUCCESS) {
    free(fdes);
    return st;
  }
  ric_ops_ctx r;
  memset(&r, 0, sizeof(r));
  r.c = c;
  r.N = N;
  double* A = (double*)malloc(sizeof(double) * N * NX * NX);
  double* Bm = (double*)malloc(sizeof(double) * N * NX * NU);
  oracle_srbd_dynamics(c, xref, foot, contact, A, Bm);
  r.A = A;
  r.B = Bm;
  int n = 0;
  for (int k = 0; k < N; ++k) {
    r.off[k] = n;
    for (int i = 0; i < L; ++i)
      if (contact[k * L + i]) r.legs[k][r.nst[k]++] = i;
    r.nu[k] = 3 * r.nst[k];
    n += r.nu[k];
  }
  double* mem = (double*)calloc((size_t)N * (NZ * NU * 3 + NU * NU + NU) + 2 * NZ * NZ, sizeof(double));
  r.Bt = mem;
  r.St = r.Bt + (size_t)N * NZ * NU;
  r.Kf = r.St + (size_t)N * NU * NZ;
  r.Lr = r.Kf + (size_t)N * NU * NZ;
  r.Lri = r.Lr + (size_t)N * NU * NU;
  r.P = r.Lri + (size_t)N * NU;
  for (int k = 0; k < N; ++k)
    for (int t = 0; t < r.nst[k]; ++t)
      for (int d = 0; d < 3; ++d) {
        const int a = 3 * t + d, j = 3 * r.legs[k][t] + d;
        for (int i = 0; i < NX; ++i) r.Bt[(size_t)k * NZ * NU + i * NU + a] = Bm[(size_t)k * NX * NU + i * NU + j];
        r.Bt[(size_t)k * NZ * NU + (NX + j) * NU + a] = 1.0;
      }
  const int nt = n / 3;
  double* zero = (double*)calloc(5 * (size_t)(nt + 1), sizeof(double));
  double* one = (double*)malloc(sizeof(double) * 5 * (nt + 1));
  double* mu = (double*)calloc((size_t)nt + 1, sizeof(double));
  for (int j = 0; j < 5 * (nt + 1); ++j) one[j] = 1.0;
  st = ric_factor(&r, nt, mu, zero, zero, one, one, 0.0) == 0 ? CMPC_SUCCESS : CMPC_NAN_SOL;
  for (int t = 0; t < r.nst[0]; ++t)
    for (int d = 0; d < 3; ++d)
      for (int j = 0; j < NX; ++j) K0[(3 * r.legs[0][t] + d) * NX + j] = r.Kf[(3 * t + d) * NZ + j];
  free(fdes); free(A); free(Bm); free(mem); free(zero); free(one); free(mu);
  return st;
}
