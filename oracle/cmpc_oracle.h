/*
 * cmpc_oracle.h — CPU fp64 restatement of the reference's CentroidalMPC / HpipmInterface hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in the product (cheeta-mpc_amd/) links, loads or calls this code; only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only as the checker / the CPU
 * baseline. Parity status: the reference's solver (CasADi/IPOPT, HPIPM@255ffdf/BLASFEO@ae6e2d1) is absent from the
 * image and cannot be built offline; this restatement is pinned by the reference's own
 * known-answer constructions (testHpipmInterface.cpp:112-152 knownSolution, :208-256 noInputs, :258-340
 * retrieveRiccati), by KKT certificates and by numpy golden vectors (tests/golden/). Parity against the HPIPM
 * binary itself is unpinned.
 */
#ifndef CMPC_ORACLE_H_
#define CMPC_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#include "cmpc/cmpc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Model constants derived once per model (weights re-indexed, Q diag per node, inverse inertia). */
typedef struct oracle_consts {
  int N, L;
  double mass, dt;
  double inv_inertia[9];
  double mu[CMPC_MAX_LEGS];
  double Wf[CMPC_NU]; /* force tracking weight per (leg, comp) */
  double Wr[CMPC_NU]; /* force-rate weight per (leg, comp) */
  double Wp[CMPC_NU]; /* foot position tracking weight per (leg, comp), w[9 + 3i + c] (CentroidalMPC.cpp:218-221) */
  double qdiag[64][CMPC_NX]; /* 2*diag(Q_k), k = 0..N (k = 0 unused) */
  double force_ub[5];
} oracle_consts;

void oracle_consts_init(const cmpc_model* m, oracle_consts* c);

/* Stance foot position of leg i at stance step k (foot record [(N+1)][L][3]: node 0 = current foot, nodes 1..N =
 * des_foot_pos; CentroidalMPC.cpp:93, :165-167, :288-291) and all of them: out [N][L][3] (0 for swing). */
void oracle_stance_point(const double* foot, const uint8_t* contact, int N, int L, int k, int i, double p[3]);
void oracle_stance_feet(int N, int L, const double* foot, const uint8_t* contact, double* out);

/* SRBD linearisation (SURVEY App. A.2 from CentroidalMPC.cpp:41-100): A [N][13][13], B [N][13][12] row-major. */
void oracle_srbd_dynamics(const oracle_consts* c, const double* xref, const double* foot, const uint8_t* contact,
                          double* A, double* B);

/* Linearisation at lin [N][6] = (c_bar_k, F_bar_k) (NULL: (c_ref_k, 0)); affine term b [N][13] (may be NULL). */
void oracle_srbd_dynamics_lin(const oracle_consts* c, const double* xref, const double* foot, const uint8_t* contact,
                              const double* lin, double* A, double* B, double* b);
int oracle_condense_full_lin(const oracle_consts* c, const double* x0, const double* xref, const double* foot,
                             const uint8_t* contact, const double* lin, double* Hfull, double* gfull);
int oracle_condense_lin(const oracle_consts* c, const double* x0, const double* xref, const double* foot,
                        const uint8_t* contact, const double* lin, int ld, int* n, double* H, double* g,
                        double* tri_mu, double* tri_lo, double* tri_hi, int* tri_map);
int oracle_solve_one_lin(const oracle_consts* c, const cmpc_settings* s, const double* x0, const double* xref,
                         const double* foot, const uint8_t* contact, const double* lin, double* u, double* x,
                         int* iters);
/* Nonlinear (bilinear lever arm) rollout + NLP cost; x [(N+1)][13], lin [N][6] outputs may be NULL. */
double oracle_nlp_rollout_cost(const oracle_consts* c, const double* x0, const double* xref, const double* foot,
                               const uint8_t* contact, const double* u, double* x, double* lin);
/* Gauss-Newton SQP on the bilinear NLP; u [N][L][3] out, x [(N+1)][13] nonlinear rollout. */
/* line search / convergence settings of the SQP: MultipleShootingSettings.h:44-54 defaults */
#define SQP_ALPHA_DECAY 0.5
#define SQP_ALPHA_MIN 1e-4
#define SQP_ARMIJO 1e-4
#define SQP_COST_TOL 1e-4
void oracle_nlp_linstep(const oracle_consts* c, const double* x0, const double* xref, const double* foot,
                        const uint8_t* contact, const double* u, const double* du, double* dxnorm, double* metric);
int oracle_sqp_solve(const oracle_consts* c, const cmpc_settings* s, int sqp_iter_max, double sqp_tol,
                     const double* x0, const double* xref, const double* foot, const uint8_t* contact, double* u,
                     double* x, int* qp_iters, int* sqp_iters);
/* Footholds of the later stance runs as decision variables (CentroidalMPC.cpp:132-133, 196-198, 218-221; see
 * cmpc_oracle.c): D [N][L][3] = foothold offsets from the run's mean des position, indexed by the run's first step. */
double oracle_nlp_rollout_cost_feet(const oracle_consts* c, const double* x0, const double* xref, const double* foot,
                                    const uint8_t* contact, const double* u, const double* D, double* x, double* lin);
void oracle_nlp_linstep_feet(const oracle_consts* c, const double* x0, const double* xref, const double* foot,
                             const uint8_t* contact, const double* u, const double* D, const double* du,
                             const double* dD, double* dxnorm, double* metric);
int oracle_foot_box(const double* foot, const uint8_t* contact, int N, int L, int s, int i, double pbar[3],
                    double lo[3], double hi[3], int* cnt);
void oracle_feet_init(const oracle_consts* c, const double* foot, const uint8_t* contact, double* D);
void oracle_feet_table(const oracle_consts* c, const double* foot, const uint8_t* contact, const double* D,
                       double* out);
int oracle_condense_feet(const oracle_consts* c, const double* x0, const double* xref, const double* foot,
                         const uint8_t* contact, const double* lin, const double* ubar, const double* D, int ld,
                         int* n_out, double* H, double* g, double* tri_mu, double* tri_lo, double* tri_hi,
                         int* tri_map);
int oracle_solve_one_feet(const oracle_consts* c, const cmpc_settings* s, const double* x0, const double* xref,
                          const double* foot, const uint8_t* contact, const double* lin, double* u, double* D,
                          int* iters);
int oracle_sqp_solve_feet(const oracle_consts* c, const cmpc_settings* s, int sqp_iter_max, double sqp_tol,
                          const double* x0, const double* xref, const double* foot, const uint8_t* contact, double* u,
                          double* D, double* feet, double* x, int* qp_iters, int* sqp_iters);

/* Full condensing over all 12N inputs (no elimination): Hfull [12N][12N], gfull [12N]. Returns 0 or
 * CMPC_INVALID_CONTACT. */
int oracle_condense_full(const oracle_consts* c, const double* x0, const double* xref, const double* foot,
                         const uint8_t* contact, double* Hfull, double* gfull);

/* Condensed QP restricted to stance forces (swing legs eliminated):
 *   *n = 3 * (#stance (k,i)); H [ld][ld] with identity padding; g [ld];
 *   tri_mu [ld/3], tri_lo/tri_hi [ld/3][5]; tri_map [ld/3] = k*L + i of each active triple.
 * Returns CMPC_SUCCESS, CMPC_INVALID_CONTACT or CMPC_TOO_LARGE. */
int oracle_condense(const oracle_consts* c, const double* x0, const double* xref, const double* foot,
                    const uint8_t* contact, int ld, int* n, double* H, double* g, double* tri_mu, double* tri_lo,
                    double* tri_hi, int* tri_map);

/* Dense friction-pyramid QP, Mehrotra predictor-corrector IPM (the algorithm the HIP kernels run).
 * H [ld][ld], n <= ld, n % 3 == 0. u [n] out; lam_lo/lam_hi [5n/3] out (may be NULL).
 * res[4] out (may be NULL): max |r_stat|, 0 (no equalities), max |r_ineq|, max comp. Returns status. */
int oracle_qp_ipm(int n, int ld, const double* H, const double* g, const double* tri_mu, const double* tri_lo,
                  const double* tri_hi, const cmpc_settings* s, double* u, double* lam_lo, double* lam_hi, int* iters,
                  double* res);
/* Same, also recording the per-iteration statistics table stats[rows][10] (columns of cmpc_enable_stats). */
int oracle_qp_ipm_stats(int n, int ld, const double* H, const double* g, const double* tri_mu, const double* tri_lo,
                        const double* tri_hi, const cmpc_settings* s, double* u, double* lam_lo, double* lam_hi,
                        int* iters, double* res, double* stats, int stats_rows);

/* Whole hot path for one QP: u [N][L][3] (zeros for swing), x [(N+1)][13] (may be NULL). */
/* u [N][L][3] out; with s->warm_start != 0 it is also the initial guess on entry (HPIPM warm_start = 1). */
int oracle_solve_one(const oracle_consts* c, const cmpc_settings* s, const double* x0, const double* xref,
                     const double* foot, const uint8_t* contact, double* u, double* x, int* iters);

/* Batch over QP-major records with nthreads pthreads (nthreads <= 1: serial). */
int oracle_solve_batch(const cmpc_model* m, const cmpc_settings* s, int B, const double* x0, const double* xref,
                       const double* foot, const uint8_t* contact, double* u, double* x, int* status, int* iters,
                       int nthreads);

/* KKT certificate of a QP solution: returns max of stationarity / primal infeasibility / |complementarity| /
 * dual negativity, each in out[0..3]. */
void oracle_qp_kkt(int n, int ld, const double* H, const double* g, const double* tri_mu, const double* tri_lo,
                   const double* tri_hi, const double* u, const double* lam_lo, const double* lam_hi, double* out);

/* Synthetic inputs (bit-identical to the device generator cmpc_generate_batch). */
void oracle_generate(const cmpc_model* m, uint64_t seed, int64_t qp_offset, int B, int gait, double* x0,
                     double* xref, double* foot, uint8_t* contact);
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

/* ---- Generic OCP-QP (HpipmInterface semantics), record layout as cmpc_ocp_record_size ---- */
size_t oracle_ocp_record_size(int N, int nx, const int* nu);
/* Condense: H [nU][nU], g [nU] with nU = sum nu_k (row-major), after x0 elimination (HpipmInterface.cpp:177-208). */
int oracle_ocp_condense(int N, int nx, const int* nu, const double* x0, const double* rec, double* H, double* g);
/* Solve by condensing + Cholesky; x [(N+1)][nx], u [nU]. Returns status. */
int oracle_ocp_solve(int N, int nx, const int* nu, const double* x0, const double* rec, double* x, double* u);
/* Discrete Riccati recursion (testHpipmInterface.cpp:280-304): Sm [(N+1)][nx][nx], sv [(N+1)][nx],
 * K [N][nu_k x nx] (row-major, packed by stage), kff [sum nu_k]. */
int oracle_ocp_riccati(int N, int nx, const int* nu, const double* rec, double* Sm, double* sv, double* K,
                       double* kff);

/* ---- Stage-wise OCP IPM (ocp_ipm.c): HPIPM's d_ocp_qp_ipm as HpipmInterface::solve drives it ----
 * nc [N+1] rows per node (NULL: none), crec as cmpc_ocp_constraint_record_size (C_k, D_k, e_k column-major; the rows
 * C x + D u + e = 0 are the two-sided general constraints lg = ug = -e, HpipmInterface.cpp:223-264). x [(N+1)][nx]
 * (node 0 = x0), u [sum nu_k]; res[4] = max |r_stat|, |r_eq|, |r_ineq|, max t lam at exit; stats [rows][10] as
 * cmpc_enable_stats (res_eq now the dynamics residual). ric (optional): Riccati quantities of the last factorisation
 * with the vector part in absolute form (see ocp_ipm.c), all column-major: P [(N+1)][nx][nx], p [(N+1)][nx],
 * K [sum nu_k nx] (stage blocks nu_k x nx), k [sum nu_k], Lr [sum nu_k^2] (HPIPM's ric_Lr: the lower
 * Cholesky factor of R~ + B'PB + D'Sigma D, column-major, may be NULL). */
typedef struct oracle_ocp_ric {
  double *P, *p, *K, *k, *Lr;
} oracle_ocp_ric;
int oracle_ocp_ipm(int N, int nx, const int* nu, const int* nc, const double* x0, const double* rec,
                   const double* crec, const cmpc_settings* s, double* x, double* u, int* iters, double* res,
                   oracle_ocp_ric* ric, double* stats, int stats_rows);
/* Batch of B problems of the same dimensions over nthreads pthreads (bench.py's cpu_baseline for the OCP path). */
int oracle_ocp_ipm_batch(int B, int N, int nx, const int* nu, const int* nc, const double* x0, const double* rec,
                         size_t rec_size, const double* crec, size_t crec_size, const cmpc_settings* s, double* x,
                         double* u, int* status, int* iters, int nthreads);
/* The cold start's first (predictor) Newton step, with the system's data for a dense cross-check. */
int oracle_ocp_first_step(int N, int nx, const int* nu, const int* nc, const double* x0, const double* rec,
                          const double* crec, const cmpc_settings* s, double* du, double* dx, double* dpi,
                          double* sig, double* rhs_u, double* rhs_x, double* rb);

/* Contact table of one QP from a gait template (cmpc.h cmpc_gait semantics): GaitSchedule.cpp:78-127 tiling,
 * MotionPhaseDefinition.h:69-124 stance legs, mode at the start of each interval (left-closed). contact [N][4]. */
void oracle_gait_contact(const cmpc_gait* g, const int* leg_map, double t_start, double t0, double dt, int N,
                         uint8_t* contact);

/* Small dense helpers exported for tests. */
int oracle_cholesky(int n, double* A, int lda);                       /* in place, lower; 0 ok, -1 not PD */
void oracle_chol_solve(int n, const double* L, int lda, double* b);   /* solves (L L^T) x = b in place */


/* Feedback policy dU/dx0 at a solution u [N][L][3] on its active set (act_tol = slack threshold, absolute):
 * K [12N][13] row-major; *n_free = reduced dimension. oracle_policy_triple: free directions of one triple. */
int oracle_policy_triple(double mu, const double* ub, const double* f, double tol, double* Z);
int oracle_policy(const oracle_consts* c, const double* xref, const double* foot, const uint8_t* contact,
                  const double* u, double act_tol, double* K, int* n_free);
int oracle_policy_lin(const oracle_consts* c, const double* xref, const double* foot, const uint8_t* contact,
                      const double* lin, const double* u, double act_tol, double* K, int* n_free);


/* The same QP solved without condensing, HPIPM-style: the shared Mehrotra IPM with its Newton systems solved by a
 * Riccati recursion over the stages (state [x; u_prev], 25) and H u + g by rollout + adjoint. Cold start only.
 * u [N][L][3] out. oracle_riccati_solve_batch: QP-major batch over nthreads pthreads. */
int oracle_riccati_solve_one(const oracle_consts* c, const cmpc_settings* s, const double* x0, const double* xref,
                             const double* foot, const uint8_t* contact, double* u, int* iters);
int oracle_riccati_solve_batch(const cmpc_model* m, const cmpc_settings* s, int B, const double* x0,
                               const double* xref, const double* foot, const uint8_t* contact, double* u,
                               int* status, int* iters, int nthreads);

/* Stage-0 Riccati feedback (unconstrained) of the OCP form: K0 [L][3][13] (HpipmInterface::getRiccatiFeedback(0)). */
int oracle_riccati_gain0(const oracle_consts* c, const double* xref, const double* foot, const uint8_t* contact,
                         double* K0);

#ifdef __cplusplus
}
#endif

#endif /* CMPC_ORACLE_H_ */
