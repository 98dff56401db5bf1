/*
 * cmpc.h — C ABI of the MI355X-native batched centroidal-MPC QP engine.
 *
 * This is the drop-in boundary. It replaces, for the CentroidalMPC hot path:
 *   - CentroidalMPC::UpdateMPC            (reference CentroidalMPC.cpp:278-370 / CentroidalMPC.h:32)
 *       → cmpc_solve_batch (B = 1 is one UpdateMPC call)
 *   - HpipmInterface::Impl::solve          (reference ocs2_sqp/hpipm_catkin/src/HpipmInterface.cpp:166-301)
 *       → cmpc_ocp_create (initializeMemory, :92-129) + cmpc_ocp_solve / cmpc_ocp_solve_host (stage-wise OCP
 *         interior-point method on the device, x0 eliminated as :177-208, constraint rows as :223-264) and
 *         cmpc_ocp_riccati (getRiccati*, :330-455)
 *   - hpipm_interface::Settings            (reference hpipm_catkin/include/hpipm_catkin/HpipmInterfaceSettings.h:44-57)
 *       → cmpc_settings
 *   - d_ocp_qp_ipm_get_status codes        (reference HpipmInterface.h:79-85, HpipmInterface.cpp:462-473)
 *       → enum cmpc_qp_status
 *
 * Conventions (mirroring HPIPM's C API, HpipmInterface.cpp:104-128, :282-284):
 *   - plain pointers + sizes, no C++ types, no exceptions across the ABI;
 *   - API functions return an int error code (CMPC_OK = 0, negative on error); per-QP solver outcome is an
 *     int status array with HPIPM's codes;
 *   - batch entry points take DEVICE pointers and an opaque hipStream_t (void*), and are asynchronous on it;
 *     the *_host variants take host pointers and synchronise;
 *   - batch input layouts are QP-major (one contiguous record per QP): one wavefront/workgroup serves one QP and
 *     reads its record coalesced.
 *
 * Per-QP record layouts (N = horizon, L = n_legs = 4):
 *   x0      [13]              = [c(3), v(3), L(3), Theta(3), g_z]        (c,v,L as CentroidalMPC.cpp:284-286)
 *   xref    [(N+1)][13]       node k = 0..N                              (des_state, CentroidalMPC.cpp:297-299, extended)
 *   foot    [(N+1)][L][3]     node 0: current foot position p_i (state[9+3i..], CentroidalMPC.cpp:288-291);
 *                             nodes 1..N: desired foot position p^des_{i,k} (des_inputs, :316-317). The reference
 *                             pins foot_pos(:,0) to the current position (:165-167), so des_foot_pos node 0 only adds
 *                             a constant and is not carried. Stance lever arms follow the reference's foot dynamics
 *                             (a stance foot does not move, :93): a stance run from step 0 acts at node 0; a later
 *                             run (nodes s..e+1, touch-down after a swing step) at the mean of p^des over its nodes.
 *   contact [N][L]  (uint8)   e_{i,k} in {0,1}                           (mpc_table, CentroidalMPC.cpp:315-335)
 *   u       [N][L][3]         world-frame contact forces (0 for swing legs)
 *   x       [(N+1)][13]       optional state rollout of the solution
 */
#ifndef CMPC_CMPC_H_
#define CMPC_CMPC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CMPC_NX 13
#define CMPC_MAX_LEGS 4
#define CMPC_NU (3 * CMPC_MAX_LEGS)
#define CMPC_NUM_WEIGHTS ((CMPC_MAX_LEGS + 1) * 9) /* 45, CentoidMPCTest.cpp:18 */

/* API return codes */
enum cmpc_error {
  CMPC_OK = 0,
  CMPC_ERR_ARG = -1,      /* bad argument (null pointer, size out of range) */
  CMPC_ERR_HIP = -2,      /* HIP runtime error */
  CMPC_ERR_SIZE = -3,     /* batch larger than the context's max_batch, or horizon mismatch */
  CMPC_ERR_NO_DEVICE = -4 /* no usable gfx950 device */
  /* cmpc_ocp: a solve on a handle whose last cmpc_ocp_reshape failed returns CMPC_ERR_ARG until a reshape succeeds */
};

/* Per-QP solver status. 0..4 keep HPIPM's hpipm_status order (HpipmInterface.h:79-85). */
enum cmpc_qp_status {
  CMPC_SUCCESS = 0,          /* QP solved */
  CMPC_MAX_ITER = 1,         /* maximum number of iterations reached */
  CMPC_MIN_STEP = 2,         /* minimum step length reached */
  CMPC_NAN_SOL = 3,          /* NaN in computations / non-finite solution (HpipmInterface.cpp:290-295) */
  CMPC_INCONS_EQ = 4,        /* inconsistent equality constraints (HPIPM's code; the interior-point solvers here end
                                inconsistent rows at MAX_ITER / MIN_STEP as HPIPM's OCP IPM does) */
  CMPC_INVALID_CONTACT = 5,  /* a horizon step has no stance leg: reference throws "mpc table invalid"
                                (CentroidalMPC.cpp:328-330) */
  CMPC_TOO_LARGE = 6,        /* condensed size exceeds what this build's kernels support */
  CMPC_INFEASIBLE_STEP = 7,  /* cmpc_nlp_solve_batch: the step box of CentroidalMPC.cpp:196-198 cannot be met: a
                                later stance run's foothold box is empty (des_foot_pos varies over the run by more
                                than the box), or a run from step 0 keeps the current foot (:165-167) outside the box
                                around des_foot_pos at one of its nodes */
  CMPC_GRID_TIMEOUT = 8      /* cmpc_ocp grid form only, internal: a grid barrier timed out (the problem's workgroups
                                were not all resident). The same cmpc_ocp_solve call re-solves such a problem on one
                                workgroup (cmpc_ocp_fallback_count), so no solve returns this code */
};

/* Foothold step box of the NLP (CentroidalMPC.cpp:30-31): step_lb <= foot_pos - des_foot_pos <= step_ub at every node
 * 1..N (CentroidalMPC.cpp:196-198). */
#define CMPC_STEP_LB_XY (-0.2)
#define CMPC_STEP_LB_Z (-0.1)
#define CMPC_STEP_UB_XY 0.2
#define CMPC_STEP_UB_Z 0.1

enum cmpc_precision { CMPC_F64 = 0, CMPC_F32 = 1 };

/* Interior-point settings. Field-for-field mirror of hpipm_interface::Settings (HpipmInterfaceSettings.h:44-57),
 * defaults identical (cmpc_settings_default). Validated by cmpc_create / cmpc_set_settings (CMPC_ERR_ARG otherwise):
 *   hpipm_mode  0..3 = HPIPM's SPEED_ABS, SPEED, BALANCE, ROBUST (same numbering as hpipm_catkin's hpipm_mode enum).
 *               As in HpipmInterface.cpp:131-144 the mode only selects defaults that the explicit fields below then
 *               override; the build runs one iteration (Mehrotra predictor-corrector) for every mode.
 *   pred_corr   must be 1 (the only iteration the build restates); 0 is rejected.
 *   ric_alg     0 or 1: HPIPM's classical / square-root Riccati factorisation choice. Both give the same iterates in
 *               exact arithmetic; the build's dense factorisation serves both.
 *   tol_eq      stopping tolerance on equality residuals: the centroidal QP has none; the OCP path (cmpc_ocp_solve)
 *               applies it to the dynamics residual.
 *   warm_start  0 or 1: 1 makes cmpc_solve_batch_warm start from the given inputs.
 *   iter_max >= 0; alpha_min, mu0, tol_* > 0; reg_prim >= 0. */
typedef struct cmpc_settings {
  int hpipm_mode;   /* 1 = SPEED (default, HpipmInterfaceSettings.h:45) */
  int iter_max;     /* 30 */
  double alpha_min; /* 1e-12 */
  double mu0;       /* 10 */
  double tol_stat;  /* 1e-6 */
  double tol_eq;    /* 1e-8 */
  double tol_ineq;  /* 1e-8 */
  double tol_comp;  /* 1e-8 */
  double reg_prim;  /* 1e-12 */
  int warm_start;   /* 0 */
  int pred_corr;    /* 1 */
  int ric_alg;      /* 0 */
} cmpc_settings;

/* Centroidal model (CentroidalMPC ctor args, CentroidalMPC.h:26-27, plus SRBD extensions of SURVEY App. A). */
typedef struct cmpc_model {
  int N;                              /* predict_horizon */
  int n_legs;                         /* num_legs (must be 4 in this build) */
  double mass;                        /* kg */
  double dt;                          /* time_step */
  double inertia[9];                  /* body inertia I_b, row-major (build extension, A.2) */
  double mu[CMPC_MAX_LEGS];           /* friction coefficient per leg */
  double weights[CMPC_NUM_WEIGHTS];   /* CentroidalMPC weight vector, same indexing as CentroidalMPC.cpp:203-231 */
  double force_ub[5];                 /* pyramid row upper bounds; default {5000,5000,5000,5000, m*9.81*n_legs}
                                         (CentroidalMPC.cpp:182-183) */
  double theta_weights[3];            /* Q weight on roll/pitch/yaw (build extension, default 0) */
} cmpc_model;

void cmpc_settings_default(cmpc_settings* s);
/* CentoidMPCTest.cpp:12-33 parameters (m = 8, dt = 0.01, mu = 0.8, the 45 weights) at horizon N. */
void cmpc_model_default(cmpc_model* m, int N);

typedef struct cmpc_ctx cmpc_ctx;

/* Device workspace bytes a context needs for max_batch QPs (HPIPM-style *_memsize). */
size_t cmpc_memsize(const cmpc_model* model, int precision, int max_batch);
/* Create a context on the current HIP device. dev_mem: caller-owned device buffer of cmpc_memsize bytes, or NULL
 * to let the context allocate (and free) it. */
int cmpc_create(const cmpc_model* model, const cmpc_settings* settings, int precision, int max_batch, void* dev_mem,
                cmpc_ctx** out);
int cmpc_destroy(cmpc_ctx* ctx);
int cmpc_set_settings(cmpc_ctx* ctx, const cmpc_settings* settings);
int cmpc_set_model(cmpc_ctx* ctx, const cmpc_model* model); /* horizon N must not change */
int cmpc_get_model(const cmpc_ctx* ctx, cmpc_model* out);
/* Leading dimension (padded max condensed size) of the context's H workspace. */
int cmpc_ctx_ld(const cmpc_ctx* ctx);
/* 1 when a cold-start cmpc_solve_batch runs the fused condensing + IPM kernel for the n <= 64 class, else 0
 * (= cmpc_get_path(ctx, CMPC_PATH_FUSED64)). */
int cmpc_ctx_fused(const cmpc_ctx* ctx);
/* Kernel path of a context, for A/B measurement and tests; the first three options give bit-identical results:
 *   CMPC_PATH_FUSED64   1 (default when N <= 21): cold-start solves condense and solve the n <= 64 class in one
 *                       launch; 0: a condensing launch, then the IPM launch. 1 is CMPC_ERR_ARG when N > 21.
 *   CMPC_PATH_FUSED128  1: the 64 < n <= 128 class condensed and solved in one launch on the fused path (default for
 *                       fp32 contexts); 0: two launches (default for fp64, where the fused form measured slower).
 *   CMPC_PATH_DIRECT    1 (default): on the fused path without a rollout the IPM kernels write u / status / iters;
 *                       0: through the scatter kernel.
 *   CMPC_PATH_RICCATI   0 (default): the condensed path above. 1: on the fused path, the n > 64 QPs are solved by the
 *                       stage-wise kernel (Riccati Newton solves over the horizon, no condensing, HPIPM's method);
 *                       2: every cold-start QP is (one launch). Results agree with the condensed path to rounding,
 *                       not bit for bit (a different factorisation of the same Newton systems). Needs N <= 21; 1 needs
 *                       CMPC_PATH_FUSED64 = 1, and CMPC_PATH_FUSED64 = 0 is refused while RICCATI is 1.
 *   CMPC_PATH_IPM72     1 (default): where the IPM runs as its own launch (warm starts, the SQP / NLP subproblems,
 *                       CMPC_PATH_FUSED64 = 0), QPs with 64 < n <= 72 (the NLP's trot subproblems at N = 10: 60 forces
 *                       and two to four foothold triples) are solved by a one-wave kernel on the bordered Newton system (Schur
 *                       complement of the 64 x 64 block); 0: by the four-wave 128 class. Results agree to rounding.
 * cmpc_set_path returns CMPC_ERR_ARG for an unknown option or a value out of range (0 / 1; 0 / 1 / 2 for
 * CMPC_PATH_RICCATI); cmpc_get_path returns the current value or CMPC_ERR_ARG. */
enum cmpc_path_option {
  CMPC_PATH_FUSED64 = 0,
  CMPC_PATH_FUSED128 = 1,
  CMPC_PATH_DIRECT = 2,
  CMPC_PATH_RICCATI = 3,
  CMPC_PATH_IPM72 = 4
};
int cmpc_set_path(cmpc_ctx* ctx, int option, int value);
int cmpc_get_path(const cmpc_ctx* ctx, int option);

/* Full hot path: SRBD linearisation -> condensing (H, g) -> friction/force-bound stacking -> batched IPM ->
 * scatter to [N][L][3] (zeros for swing legs) and optional rollout. Device pointers, async on stream.
 * d_x may be NULL. d_iters may be NULL. */
int cmpc_solve_batch(cmpc_ctx* ctx, int B, const double* d_x0, const double* d_xref, const double* d_foot,
                     const uint8_t* d_contact, double* d_u, double* d_x, int* d_status, int* d_iters, void* stream);
/* Same, host pointers; synchronous. */
/* Warm-started hot path (hpipm_interface::Settings::warm_start, HpipmInterfaceSettings.h:54; HPIPM's warm_start = 1,
 * primal): with settings.warm_start != 0 and d_u_init != NULL, the IPM of each QP starts from d_u_init
 * [B][N][L][3] (e.g. the previous MPC tick's solution shifted by cmpc_shift_inputs; swing entries ignored) with
 * slacks of C u clipped at 1 and lam = mu0 / t; otherwise identical to cmpc_solve_batch (cold start). d_u_init may
 * alias d_u. */
int cmpc_solve_batch_warm(cmpc_ctx* ctx, int B, const double* d_x0, const double* d_xref, const double* d_foot,
                          const uint8_t* d_contact, const double* d_u_init, double* d_u, double* d_x, int* d_status,
                          int* d_iters, void* stream);
/* Batched Gauss-Newton SQP on the bilinear centroidal NLP: the reference's NLP keeps the lever
 * arm (p_i - c) x f_i bilinear (CentroidalMPC.cpp:86). Per QP: U_0 = the QP at the reference linearisation (as
 * cmpc_solve_batch); then up to sqp_iter_max times: linearise at the nonlinear rollout of U_j (lever arm p - c_k,
 * dt F_k x (c - c_k) coupling), solve that QP warm-started from U_j, and step by ocs2's filter line search
 * (MultipleShootingSolver::takeStep, MultipleShootingSolver.cpp:509-619) in its zero-violation form (single shooting:
 * the rollout meets the dynamics, the merit is the NLP cost): alpha = 1, 1/2, ... >= alpha_min = 1e-4, Armijo
 * (armijoFactor 1e-4) on the descent metric grad J . [dx; du] (:287-296) when it is negative, else plain decrease;
 * the search ends early once alpha |dx| and alpha |du| are below deltaTol. A QP stops (checkConvergence, :620-645)
 * when no step is taken, when |J_new - J_j| < costTol = 1e-4, or when alpha |dx| and alpha |du| (2-norms over the
 * trajectory) are both below deltaTol = sqp_tol (ocs2 default 1e-6); the other settings are
 * MultipleShootingSettings.h:44-54's defaults. d_x (optional) receives the nonlinear rollout. d_qp_iters:
 * total IPM iterations, d_sqp_iters: SQP iterations (both optional). Synchronises the stream once per SQP iteration
 * (early exit when every QP has converged). */
int cmpc_sqp_solve_batch(cmpc_ctx* ctx, int B, const double* d_x0, const double* d_xref, const double* d_foot,
                         const uint8_t* d_contact, int sqp_iter_max, double sqp_tol, double* d_u, double* d_x,
                         int* d_status, int* d_qp_iters, int* d_sqp_iters, void* stream);
/* The reference's NLP with its foothold variables (CentroidalMPC.cpp:132-133: foot_pos[i] at every node, swing
 * dynamics :93 / :174-176, pinned node 0 :165-167, step box :196-198 with CMPC_STEP_LB/UB, tracking cost :218-221):
 * cmpc_sqp_solve_batch over the forces AND the footholds. foot_vel is free and uncosted, so a swing node that starts
 * no stance run tracks des_foot_pos exactly and a stance run from step 0 stays at the current foot; each later stance
 * run (first stance step s >= 1) holds one free foothold, a decision variable of every QP of the SQP (a foothold
 * triple with mu = 0 whose rows [-x, x, -y, y, z] carry the step box; its lever-arm columns dt e_d x f_bar act on
 * the angular momentum at each step of the run). The footholds start at the box-projected mean of des_foot_pos over
 * the run's nodes (the frozen footholds of cmpc_solve_batch), the forces at the cold QP's solution; the line search
 * and the convergence test cover both (|du| over forces and footholds). d_feet [B][N+1][L][3] (required): the
 * reference controller's foot_pos outputs (:269-273) — node 0 and the first run's nodes the current foot, a later
 * run's nodes its foothold, free swing nodes des_foot_pos. Status CMPC_INFEASIBLE_STEP when a run's box is empty
 * (the forces then stay at the last iterate). Condensing runs on the workgroup kernels (n grows by 3 per later run).
 * Oracle: oracle_sqp_solve_feet. */
int cmpc_nlp_solve_batch(cmpc_ctx* ctx, int B, const double* d_x0, const double* d_xref, const double* d_foot,
                         const uint8_t* d_contact, int sqp_iter_max, double sqp_tol, double* d_u, double* d_feet,
                         double* d_x, int* d_status, int* d_qp_iters, int* d_sqp_iters, void* stream);
/* Same, host pointers; synchronous (the CentroidalMPC mirror's nonlinear UpdateMPC). */
int cmpc_nlp_solve_batch_host(cmpc_ctx* ctx, int B, const double* x0, const double* xref, const double* foot,
                              const uint8_t* contact, int sqp_iter_max, double sqp_tol, double* u, double* feet,
                              double* x, int* status, int* qp_iters, int* sqp_iters);
/* Feedback policy of each QP at its solution d_u [B][N][L][3] (e.g. from cmpc_solve_batch): d_K [B][N][L][3][13]
 * = dU/dx0, the condensed counterpart of HpipmInterface::getRiccatiFeedback (HpipmInterface.cpp:330-455; ocs2 uses
 * it as the linear feedback policy, MultipleShootingSolver.cpp:334-362). K = -Z (Z'HZ)^{-1} Z' Bqp'Q Aqp, where Z
 * spans the directions of each stance force triple left free by its active pyramid rows (slack <= act_tol, absolute,
 * in N; act_tol <= 0 selects 1e-5 for fp64 contexts, 2e-3 for fp32): the mu -> 0 limit of HPIPM's K, i.e. the
 * derivative of the QP solution map on its active set. Swing rows are 0. d_nfree [B] (optional) = dim Z;
 * d_status [B]: CMPC_SUCCESS, the condensing status, or CMPC_NAN_SOL (Z'HZ not positive definite). Recomputes the
 * condensed QP into the context workspace; the first call (or a larger B) allocates a scratch slab and
 * synchronises the stream. */
int cmpc_policy_batch(cmpc_ctx* ctx, int B, const double* d_x0, const double* d_xref, const double* d_foot,
                      const uint8_t* d_contact, const double* d_u, double act_tol, double* d_K, int* d_nfree,
                      int* d_status, void* stream);
/* Same for the QP linearised at the nonlinear rollout of u (the SQP's subproblem at its solution: lever arm p - c_k,
 * dt F_k x c coupling; e.g. u from cmpc_sqp_solve_batch, which ends on a fixed point of that QP): the feedback ocs2
 * reads off the last QP of its SQP (MultipleShootingSolver.cpp:334-362), with the linearisation point held fixed.
 * Oracle: oracle_policy_lin. */
int cmpc_sqp_policy_batch(cmpc_ctx* ctx, int B, const double* d_x0, const double* d_xref, const double* d_foot,
                          const uint8_t* d_contact, const double* d_u, double act_tol, double* d_K, int* d_nfree,
                          int* d_status, void* stream);
/* Receding-horizon shift of a batch of solutions on the device: out[q][k] = u[q][min(k + shift, N - 1)] (the role of
 * MultipleShootingSolver::initializeStateInputTrajectories, MultipleShootingSolver.cpp:220-266, on a fixed grid).
 * d_u_out must not alias d_u. */
int cmpc_shift_inputs(int B, int N, const double* d_u, int shift, double* d_u_out, void* stream);
int cmpc_solve_batch_host(cmpc_ctx* ctx, int B, const double* x0, const double* xref, const double* foot,
                          const uint8_t* contact, double* u, double* x, int* status, int* iters);

/* Stage 1 alone (test/inspection hook): condensed QP in the context precision, widened to double.
 *   d_H [B][ld][ld] (padded rows/cols carry an identity), d_g [B][ld], d_n [B] (condensed size, 0 if invalid),
 *   d_status [B] (CMPC_SUCCESS, or CMPC_INVALID_CONTACT / CMPC_TOO_LARGE). */
int cmpc_condense_batch(cmpc_ctx* ctx, int B, const double* d_x0, const double* d_xref, const double* d_foot,
                        const uint8_t* d_contact, double* d_H, double* d_g, int* d_n, int* d_status, void* stream);
/* Same at an SQP linearisation point (test hook of the SQP / NLP subproblems): d_lin [B][N][6] (c_bar_k, F_bar_k) or
 * NULL; with d_dbar [B][N][L][3] (foothold offsets by run start) and d_ubar [B][N][L][3] (forces) the foothold
 * triples of cmpc_nlp_solve_batch are added (oracle_condense_feet). Optional outputs: d_tri_map [B][ld/3] (k L + leg,
 * N L + s L + leg for a foothold triple, -1 padding), d_tri_lo / d_tri_hi [B][ld/3][5]. */
int cmpc_condense_lin_batch(cmpc_ctx* ctx, int B, const double* d_x0, const double* d_xref, const double* d_foot,
                            const uint8_t* d_contact, const double* d_lin, const double* d_ubar, const double* d_dbar,
                            double* d_H, double* d_g, int* d_n, int* d_status, int* d_tri_map, double* d_tri_lo,
                            double* d_tri_hi, void* stream);

/* Generic batched dense friction-pyramid QP (stage 2 alone):
 *   min 1/2 u'Hu + g'u  s.t.  lo_j <= F(mu_a) u_{3a..3a+2} <= hi_j   (F as CentroidalMPC.cpp:186-190)
 * per QP q: n[q] (multiple of 3, <= ld), H [ld][ld] row-major (symmetric), g [ld], tri_mu [ld/3],
 * tri_lo/tri_hi [ld/3][5]. Outputs u [ld] (entries >= n are 0), status, iters. Inputs are double; solved in the
 * context precision. ld must equal cmpc_ctx_ld(ctx). */
int cmpc_qp_solve_batch(cmpc_ctx* ctx, int B, const double* d_H, const double* d_g, const int* d_n,
                        const double* d_tri_mu, const double* d_tri_lo, const double* d_tri_hi, double* d_u,
                        int* d_status, int* d_iters, void* stream);

/* Counter-based synthetic input generator (Philox4x32-10 keyed by seed, counter = global QP id), identical
 * bit-for-bit to oracle_generate(). gait: 0 = trot (configs 2-4), 1 = mixed trot/bound/pronk (config 5).
 * QP ids run qp_offset .. qp_offset+B-1, so sharding across GPUs leaves every QP's inputs unchanged. */
int cmpc_generate_batch(const cmpc_model* model, uint64_t seed, int64_t qp_offset, int B, int gait, double* d_x0,
                        double* d_xref, double* d_foot, uint8_t* d_contact, void* stream);

/* ---- Generic OCP-QP: the HpipmInterface::solve path (reference HpipmInterface.cpp:86-554) ----
 *   min sum_k [1/2 x'Q_k x + u'S_k x + 1/2 u'R_k u + q_k'x + r_k'u] + 1/2 x_N'Q_N x_N + q_N'x_N
 *   s.t. x_{k+1} = A_k x_k + B_k u_k + b_k (k = 0..N-1), x_0 given (eliminated, HpipmInterface.cpp:177-208),
 *        C_k x_k + D_k u_k + e_k = 0 (nc_k rows at node k = 0..N; the reference's lg = ug = -e rows, :223-264).
 * Constant (padded) nx, per-stage nu_k (nu_N = 0). All blocks COLUMN-major (Eigen's default, so ocs2 .data() passes
 * through). Per-problem OCP record (size cmpc_ocp_record_size):
 *   A_k (nx*nx), B_k (nx*nu_k), b_k (nx)                                 k = 0..N-1
 *   Q_k (nx*nx), S_k (nu_k*nx), R_k (nu_k*nu_k), q_k (nx), r_k (nu_k)    k = 0..N (S, R, r empty at N)
 * Per-problem constraint record (size cmpc_ocp_constraint_record_size):
 *   C_k (nc_k*nx), D_k (nc_k*nu_k), e_k (nc_k)                           k = 0..N
 * Outputs x [(N+1)][nx] (x[0] = x0), u [sum nu_k]. */
size_t cmpc_ocp_record_size(int N, int nx, const int* nu);
size_t cmpc_ocp_constraint_record_size(int N, int nx, const int* nu, const int* nc);

/* Solver handle: HPIPM's dim / qp / sol / ipm_arg / ipm_ws memory (HpipmInterface.cpp:92-129), i.e. the problem
 * dimensions (N, nx, nu[N], nc[N+1]; nc may be NULL = no rows), the settings and all device memory for up to
 * max_batch problems, allocated once here; a solve allocates nothing and synchronises nothing.
 * Sizes: nx <= 63, nu_k + nx + 1 <= 128, nc_k <= 64, nx + 1 + max nc_k <= 128, N <= 4096 (CMPC_ERR_ARG otherwise).
 * Algorithm (csrc/k_ocp.hip; checker oracle/ocp_ipm.c): HPIPM's OCP interior-point method — the rows are two-sided
 * general constraints lg = ug = -e with slacks and multipliers, Mehrotra predictor-corrector, one step length,
 * tau = 0.995, cold start (z = 0, pi = 0, t = max(slack, 1), lam = mu0 / t), stopping on the absolute residuals
 * |r_stat| <= tol_stat, |r_eq| <= tol_eq (dynamics), |r_ineq| <= tol_ineq (rows), max t lam <= tol_comp, iter_max /
 * alpha_min honoured (an inconsistent set of rows ends at MAX_ITER or MIN_STEP, as HPIPM's IPM does); every Newton
 * system solved stage-wise by a Riccati recursion on the barrier-weighted Hessian with reg_prim on the diagonal of
 * the stage Hessians. Without rows the first Newton step is the solution (iters = 1). Settings.warm_start != 0 starts
 * x, u from the caller's arrays (cmpc_ocp_solve below). The LDS bound of the batched kernels: the handle is refused
 * (CMPC_ERR_ARG, and cmpc_ocp_memsize returns 0) when 8 ((nx + 1)^2 + 2 (nx + 1 + max nc) nzp + 4 nzp + 256) bytes,
 * nzp = 64 or 128 by max (nu_k + nx + 1, nx + 1 + max nc), exceed 160 KB. */
typedef struct cmpc_ocp cmpc_ocp;
size_t cmpc_ocp_memsize(int N, int nx, const int* nu, const int* nc, int max_batch); /* device bytes */
int cmpc_ocp_create(int N, int nx, const int* nu, const int* nc, const cmpc_settings* settings, int max_batch,
                    cmpc_ocp** out);
int cmpc_ocp_destroy(cmpc_ocp* ocp);
int cmpc_ocp_set_settings(cmpc_ocp* ocp, const cmpc_settings* settings);
/* Form of the Riccati factorisation for batches of up to 256 problems (one problem per CU; the MPC tick's B = 1):
 * chain = 1 (default) takes the latency form (csrc/ocp_chain.hpp: the stage matrix formed by the workgroup, its input
 * pivots eliminated two per round by one wave on 4 x 4 register blocks while the other waves load the next stage,
 * the gains solved stage-parallel afterwards) wherever the dimensions fit it (nx <= 27, nu_k + nx + 1 <= 60,
 * nc_k <= 16, N <= 512);
 * chain = 0 the batched form (a Gauss-Jordan sweep on the full stage matrix). Both run the same iteration; statuses and iteration counts agree, trajectories to rounding.
 * cmpc_ocp_path returns 1 when small batches take the latency form. */
int cmpc_ocp_set_path(cmpc_ocp* ocp, int chain);
int cmpc_ocp_path(const cmpc_ocp* ocp);
/* Grid form of the latency path for batches of up to 32 problems (the MPC tick's B = 1): each problem runs on G
 * workgroups, one per CU (B G <= 256), every stage-parallel pass (residuals, right-hand sides, closed-loop matrices,
 * step directions, the rows) split over them by stage ranges, the serial chains (factorisation, forward rollout,
 * cost-to-go recursion) on the first, grid barriers between the phases; reductions in a fixed order, so the
 * iteration is the single-workgroup one up to the order of the sums. G = 0 (default) picks min(32, N, 256 / B); G = 1
 * turns the grid form off (one workgroup per problem). cmpc_ocp_grid returns the G a batch of B problems runs with
 * (0: one workgroup per problem). */
int cmpc_ocp_set_grid(cmpc_ocp* ocp, int G);
int cmpc_ocp_grid(const cmpc_ocp* ocp, int B);
/* Co-residency of the grid form. cmpc_ocp_grid caps G by the occupancy the kernel admits on the current device (one
 * workgroup per CU). Kernels of other streams can still hold CUs when a solve starts: each grid barrier waits at most
 * us microseconds (cmpc_ocp_set_grid_timeout; 0 = the default 50 ms), then the problem's grid drains and the same
 * cmpc_ocp_solve re-solves it on one workgroup (a second launch on the stream, which returns at once for problems
 * whose grid finished; the result is the one-workgroup form's: same statuses and iterations, trajectories to
 * rounding). cmpc_ocp_fallback_count returns how many problems took that fallback since the handle was created
 * (synchronises on the last solve). cmpc_ocp_debug_force_grid_timeout(ocp, 1) makes every grid barrier time out at
 * once (tests of the fallback). */
/* Partitioned factorisation of the grid form (csrc/ocp_part.hpp): the backward Riccati recursion split into S horizon
 * segments on the problem's first S workgroups — each middle segment factorised from a zero end value and summarised
 * by its closed-loop transition, offset and controllability Gramian, the exact boundary values combined backward on
 * one workgroup, then every segment refactorised from its exact end value — so the serial depth is ~2 N / S stages
 * plus S - 2 combines instead of N stages. The result is the serial chain's factorisation up to rounding: a pivot the
 * first pass drops, a NaN, or a combine that would cancel more than 5 digits (an unstable segment: its free-evolution
 * cost-to-go exceeds the optimal one by > 1e5) falls back to the serial chain for that factorisation, counted by
 * cmpc_ocp_partition_fallback_count (since the handle was created; synchronises on the last solve). The serial vector
 * recursions (the rollout, the corrector's cost-to-go) run as a partitioned affine scan over the same segments.
 * S = 0 (default): ~sqrt(N) without rows, ~sqrt(2 N) with rows, at most G and N; S = 1: the serial chain.
 * cmpc_ocp_segments returns the S a batch of B problems runs with. */
int cmpc_ocp_set_segments(cmpc_ocp* ocp, int S);
int cmpc_ocp_segments(const cmpc_ocp* ocp, int B);
int cmpc_ocp_partition_fallback_count(cmpc_ocp* ocp);
int cmpc_ocp_set_grid_timeout(cmpc_ocp* ocp, double us);
int cmpc_ocp_fallback_count(cmpc_ocp* ocp);
int cmpc_ocp_debug_force_grid_timeout(cmpc_ocp* ocp, int on);
/* New dimensions for an existing handle (HpipmInterface::resize, HpipmInterface.cpp:92-129): the layout arrays are
 * re-uploaded and a device (or pinned host) buffer is reallocated only when the new size exceeds its capacity, as
 * HPIPM's MemoryBlock::reserve grows only (:46-67); handles for up to 32 problems keep 25 % headroom from the first
 * allocation (50 % at a growth), so the MPC's shifting event nodes and per-stage input counts reallocate nothing.
 * Waits for the handle's last solve first. The Riccati quantities of an earlier solve are dropped.
 * cmpc_ocp_alloc_count returns the allocations the handle has made (device and pinned host). */
int cmpc_ocp_reshape(cmpc_ocp* ocp, int N, int nx, const int* nu, const int* nc);
int cmpc_ocp_alloc_count(const cmpc_ocp* ocp);
/* keep = 1: a grid-form solve (batches up to 32) also leaves the Riccati quantities of cmpc_ocp_riccati at its exit
 * point (the factorisation the solve ends on: without rows the last Newton step's, with rows refactorised at the
 * exit point's Sigma), so cmpc_ocp_riccati becomes a copy (HPIPM's getters read its workspace,
 * HpipmInterface.cpp:336-360, :378-394). Default 0 (cmpc_ocp_riccati refactorises on demand). */
int cmpc_ocp_set_keep_riccati(cmpc_ocp* ocp, int keep);
/* on = 1: every solve records HIP events around its launch; cmpc_ocp_last_solve_ms synchronises on the last one and
 * returns its device time. */
int cmpc_ocp_enable_timing(cmpc_ocp* ocp, int on);
int cmpc_ocp_last_solve_ms(cmpc_ocp* ocp, float* ms);
/* Pinned host staging of cmpc_ocp_solve_host for handles of up to 32 problems (NULL otherwise): a caller that packs
 * its records straight into these (sized for max_batch problems) saves the host copy into the staging. The pointers
 * are valid until the next cmpc_ocp_reshape or cmpc_ocp_destroy of the handle: a reshape may reallocate the staging
 * and moves the record offsets with the record size, so fetch them again after it. */
#define CMPC_OCP_STAGE_X0 0
#define CMPC_OCP_STAGE_REC 1
#define CMPC_OCP_STAGE_CREC 2
double* cmpc_ocp_staging(cmpc_ocp* ocp, int which);
/* Device pointers, asynchronous on stream: d_x0 [B][nx], d_rec [B][record], d_crec [B][constraint record] (NULL when
 * the handle has no rows), d_x [B][(N+1)][nx], d_u [B][sum nu], d_status [B] (HPIPM codes 0..3), d_iters [B] (may be
 * NULL). The records must stay valid until cmpc_ocp_riccati of this solve has run, if it is called. With
 * settings.warm_start != 0, d_x (nodes 1..N) and d_u are read first as the initial guess (HPIPM's primal warm start:
 * slacks and multipliers start by the cold-start rule from it), as cmpc_ocp_solve_host's x and u then are. */
int cmpc_ocp_solve(cmpc_ocp* ocp, int B, const double* d_x0, const double* d_rec, const double* d_crec, double* d_x,
                   double* d_u, int* d_status, int* d_iters, void* stream);
/* Host pointers: one copy in (records into the handle's device buffers), the solve, one copy back; synchronous. */
int cmpc_ocp_solve_host(cmpc_ocp* ocp, int B, const double* x0, const double* rec, const double* crec, double* x,
                        double* u, int* status, int* iters);
/* Riccati quantities of the last solve's B problems (HpipmInterface::getRiccatiCostToGo / Feedback / Feedforward,
 * HpipmInterface.cpp:330-455), from a barrier-weighted factorisation at the point the solve returned (HPIPM keeps its
 * last iteration's; equal without rows, where the solve is one Newton step):
 *   K_k = -(R~ + B'PB)^-1 (S~ + B'PA), P_k the barrier-weighted Riccati matrix (rows of node k weighted by
 *   Sigma = lam_l / t_l + lam_u / t_u), k_k = u_k - K_k x_k + (Newton feedforward at the returned point, ~0), and
 *   p_k = pi_{k-1} - P_k x_k + (Newton cost-to-go gradient at the returned point), k >= 1: the absolute-form
 *   quantities of the Newton iterate, formed without the Sigma-sized cancellations of the absolute recursion;
 *   stage 0 as the reference rebuilds it from stage-0 data by triangular solves with Lr_0 (HpipmInterface.cpp:334-347,
 *   :376-389, :416-453; here the record's A_0, B_0, b_0, Q_0, S_0, R_0, q_0, r_0): T1 = Lr_0^-1 (S_0 + B_0'P_1 A_0),
 *   t2 = Lr_0^-1 (r_0 + B_0'(p_1 + P_1 b_0)), K_0 = -Lr_0^-T T1, k_0 = -Lr_0^-T t2, P_0 = Q_0 + A_0'P_1 A_0 - T1'T1,
 *   p_0 = q_0 + A_0'(p_1 + P_1 b_0) - T1't2.
 * Per problem, column-major: d_P [(N+1)][nx*nx], d_p [(N+1)][nx], d_K [sum nu_k*nx] (stage blocks nu_k x nx),
 * d_k [sum nu_k], d_Lr [sum nu_k^2] (HPIPM's ric_Lr, d_ocp_qp_ipm_get_ric_Lr: the lower Cholesky factor of
 * R~ + B'PB + D'Sigma D, zero above the diagonal; may be NULL); d_status [B]: 0, or 3 (NaN in the factorisation / no
 * solve).
 * Asynchronous on stream; overwrites the handle's factorisation workspace. */
int cmpc_ocp_riccati(cmpc_ocp* ocp, int B, double* d_P, double* d_p, double* d_K, double* d_k, double* d_Lr,
                     int* d_status, void* stream);
int cmpc_ocp_riccati_host(cmpc_ocp* ocp, int B, double* P, double* p, double* K, double* k, double* Lr,
                          int* status);
/* The MPC tick's part (HpipmInterface::getRiccatiFeedback, HpipmInterface.cpp:330-362): of problem b, K [sum nu_k*nx]
 * and Lr [sum nu_k^2] of every stage and P_1 [nx*nx] (for the stage-0 rebuild), host buffers, synchronous. With
 * cmpc_ocp_set_keep_riccati on a grid-form solve these are copies of what the solve kept (without rows the solve
 * keeps only P_k, K_k, Lr_k — its last factorisation is the exit point's — and cmpc_ocp_riccati refactorises when the
 * vectors are asked for); otherwise problems 0..b are refactorised first (as cmpc_ocp_riccati). K_0 here is the
 * factorisation's stage-0 gain. status: 0, or 3. */
int cmpc_ocp_riccati_feedback_host(cmpc_ocp* ocp, int b, double* K, double* Lr, double* P1, int* status);
/* Final residuals of the last solve, d_res [B][4] = (max |r_stat|, |r_eq|, |r_ineq|, max t lam) as
 * d_ocp_qp_ipm_get_max_res_stat / _eq / _ineq / _comp (HpipmInterface.cpp:478-485); per-iteration statistics
 * d_stats [B][rows][CMPC_STAT_COLS] (rows = iter_max + 1 of the settings at create / set_settings; the columns of
 * cmpc_enable_stats, res_eq = the dynamics residual; rows past a problem's last iteration are NaN). Device pointers,
 * asynchronous. cmpc_ocp_stat_rows returns rows. */
int cmpc_ocp_get_residuals(cmpc_ocp* ocp, int B, double* d_res, void* stream);
int cmpc_ocp_stat_rows(const cmpc_ocp* ocp);
int cmpc_ocp_get_stats(cmpc_ocp* ocp, int B, double* d_stats, void* stream);
/* Same, host pointers, synchronous (the HpipmInterface mirror's verbose printout). */
int cmpc_ocp_get_residuals_host(cmpc_ocp* ocp, int B, double* res);
int cmpc_ocp_get_stats_host(cmpc_ocp* ocp, int B, double* stats);
/* on = 1: every solve also records, per problem and iteration, the residuals of the Newton system it solved at its
 * final direction (predictor, or corrector with rows): HPIPM's "lin res stat / eq / ineq / comp" statistics columns
 * (HpipmInterface.cpp:492-501), the inf-norms of H~dz + G'dpi - Gc'dlam + r_stat (H~ the factorised Hessian, reg_prim
 * on its diagonal), A dx + B du - dx+ + r_eq, Gc dz - dt + r_ineq and t dlam + lam dt + r_comp.
 * d_linres [B][rows][4] (rows as cmpc_ocp_stat_rows; a row without a direction — the exit iteration's and those after
 * it — is NaN). Off by default (it costs one more pass and, in the grid form, one grid barrier per iteration);
 * cmpc_ocp_get_linres* return CMPC_ERR_ARG while it is off. */
int cmpc_ocp_set_linres(cmpc_ocp* ocp, int on);
int cmpc_ocp_get_linres(cmpc_ocp* ocp, int B, double* d_linres, void* stream);
int cmpc_ocp_get_linres_host(cmpc_ocp* ocp, int B, double* linres);

/* One-shot host entry points (create, solve, destroy; kept from the 0.3 ABI): the equality-free problem
 * (cmpc_ocp_solve_batch_host), with rows (cmpc_ocp_solve_batch_eq_host; nc == NULL is CMPC_ERR_ARG), and its Riccati
 * quantities at x0 = 0 (cmpc_ocp_riccati_batch_host: Sm = P, sv = p, K, kff as cmpc_ocp_riccati, the recursion of
 * testHpipmInterface.cpp:280-304 with reg_prim on the Hessian diagonals; status: the solve's when it did not succeed
 * (an indefinite stage is no NaN: the guarded factorisation drops the direction, as BLASFEO's, and the IPM ends at
 * MAX_ITER), else 0 or 3 from the factorisation). */
int cmpc_ocp_solve_batch_host(int B, int N, int nx, const int* nu, const double* x0, const double* rec, double* x,
                              double* u, int* status);
int cmpc_ocp_solve_batch_eq_host(int B, int N, int nx, const int* nu, const int* nc, const double* x0,
                                 const double* rec, const double* crec, double* x, double* u, int* status);
int cmpc_ocp_riccati_batch_host(int B, int N, int nx, const int* nu, const double* rec, double* Sm, double* sv,
                                double* K, double* kff, int* status);

/* ---- Contact schedules from gait templates ----
 * A template is ocs2's ModeSequenceTemplate (gait.info: modeSequence + switchingTimes, ModeNumber encoding of
 * MotionPhaseDefinition.h:48-63, stance legs of modeNumber2StanceLeg :69-124, ocs2 leg order {LF, RF, LH, RH}).
 * Each QP q follows its own schedule: STANCE before t_start[q] (GaitSchedule's default initial stance phase,
 * GaitSchedule.cpp:78-101), then the template tiled from t_start[q] (tileModeSequenceTemplate, :106-127). Step k of
 * the horizon takes the mode at the start of its interval, t = t0 + k dt (post-event, as the SQP's
 * getIntervalStart, TimeDiscretization.cpp:38-44), with left-closed mode intervals. contact[q][k][leg_map[j]] is
 * the stance flag of ocs2 leg j. A step whose mode is FLY yields a row without stance leg, which the solver reports
 * as CMPC_INVALID_CONTACT ("mpc table invalid", CentroidalMPC.cpp:328-330). */
#define CMPC_GAIT_MAX_MODES 16
#define CMPC_GAIT_MAX_TEMPLATES 64
typedef struct cmpc_gait {
  int n_modes;                                    /* M >= 1 */
  int mode[CMPC_GAIT_MAX_MODES];                  /* ModeNumber 0 (FLY) .. 15 (STANCE) */
  double switching_time[CMPC_GAIT_MAX_MODES + 1]; /* M + 1 increasing times; period = t[M] - t[0] */
} cmpc_gait;
typedef struct cmpc_gait_table cmpc_gait_table;
/* The gait.info templates by name (stance, trot, standing_trot, flying_trot, pace, standing_pace, dynamic_walk,
 * static_walk, amble, lindyhop, skipping, pawup). CMPC_ERR_ARG for an unknown name. */
int cmpc_gait_builtin(const char* name, cmpc_gait* out);
/* Device copy of n templates; leg_map[j] = contact column of ocs2 leg j (NULL: {0, 1, 3, 2}, i.e. LF, RF, LH, RH
 * onto CentroidalMPC's lf, rf, rh, lh order of CentoidMPCTest.cpp:43-46). */
int cmpc_gait_table_create(const cmpc_gait* gaits, int n, const int* leg_map, cmpc_gait_table** out);
int cmpc_gait_table_destroy(cmpc_gait_table* table);
/* contact [B][N][4] (device) from per-QP template ids and start times (device arrays). Asynchronous on stream. An
 * id outside the table gives all-swing rows (-> CMPC_INVALID_CONTACT downstream). */
int cmpc_gait_contact_batch(const cmpc_gait_table* table, int B, const int* d_gait_id, const double* d_t_start,
                            double t0, double dt, int N, uint8_t* d_contact, void* stream);

/* ---- Multi-GPU result gather (north_star: "xGMI only for result gather, no RCCL reductions") ----
 * One process per GPU, each solving a contiguous QP-id shard (cheeta_mpc/shard.py). Rank 0 owns the gathered
 * buffer on its device and exports it (cmpc_ipc_export); every other rank maps it into its own address space
 * (cmpc_ipc_open: dmabuf IPC, peer access over xGMI) and copies its shard straight into place with
 * cmpc_gather_shard (a device-to-device copy issued on the rank's stream: a peer write over xGMI when the ranks sit on
 * different GPUs). No collective and no reduction runs on the data path; the caller orders the copies with a
 * barrier (exported handle before the opens, copies done before rank 0 reads). */
#define CMPC_IPC_HANDLE_BYTES 64
typedef struct cmpc_ipc_handle {
  unsigned char bytes[CMPC_IPC_HANDLE_BYTES];
} cmpc_ipc_handle;
int cmpc_ipc_export(void* d_ptr, cmpc_ipc_handle* out);
int cmpc_ipc_open(const cmpc_ipc_handle* handle, void** d_ptr);
int cmpc_ipc_close(void* d_ptr);
int cmpc_gather_shard(void* d_dst, size_t dst_offset_bytes, const void* d_src, size_t bytes, void* stream);

/* Per-stage device timing with HIP events recorded on the solve stream (used by bench.py for the roofline):
 * after cmpc_profile_begin, each cmpc_solve_batch records events around its three stages (condense, IPM, expand);
 * cmpc_profile_end synchronises and returns the summed milliseconds per stage and the number of calls. On the fused
 * path (cmpc_ctx_fused) the first stage is the fused condensing + IPM launch of the n <= 64 class and the second
 * the bigger classes (class lists, their condensing and their IPM). */
int cmpc_profile_begin(cmpc_ctx* ctx, int max_calls);
int cmpc_profile_end(cmpc_ctx* ctx, double* ms_condense, double* ms_ipm, double* ms_expand, int* calls);

/* Solver statistics of the last IPM run on this context (cmpc_solve_batch[_warm], cmpc_qp_solve_batch,
 * cmpc_sqp_solve_batch's last QP), mirroring d_ocp_qp_ipm_get_max_res_stat / _eq / _ineq / _comp as the reference
 * reads them after a solve (HpipmInterface.cpp:459-489): d_res[q][4] = inf-norms at the iterate where the IPM stopped
 * of the stationarity residual H u + g - C' lam, the equality residual (0: the condensed QP has no equality rows), the
 * inequality residual (C u - lo - t_lo, hi - C u - t_hi) and the largest complementarity product t lam. NaN for QPs
 * the IPM did not run (status INVALID_CONTACT / TOO_LARGE). Iteration counts come with the solve (d_iters). Device
 * pointer, async on stream. */
int cmpc_get_residuals(cmpc_ctx* ctx, int B, double* d_res, void* stream);

/* Per-iteration IPM statistics: the table HPIPM's printStatus prints from d_ocp_qp_ipm_get_stat after a solve
 * (HpipmInterface.cpp:457-502). After cmpc_enable_stats(ctx, rows) every IPM run records, per QP and iteration
 * it < rows, CMPC_STAT_COLS values: alpha_aff, mu_aff, sigma, alpha_prim, alpha_dual (one step length: equal), mu,
 * res_stat, res_eq (0), res_ineq, res_comp, with the residuals and mu taken at the top of iteration it and the step
 * quantities of the step taken from there (NaN where none was taken: the stopping row). Rows past a QP's last iteration
 * are not written. rows = 0 disables recording (the default) and frees the buffer; enabling allocates
 * max_batch * rows * CMPC_STAT_COLS doubles of device memory. cmpc_get_stats copies d_stats[B][rows][CMPC_STAT_COLS]
 * (device pointer, async on stream); CMPC_ERR_ARG when recording is off. */
#define CMPC_STAT_COLS 10
int cmpc_enable_stats(cmpc_ctx* ctx, int rows);
int cmpc_get_stats(cmpc_ctx* ctx, int B, double* d_stats, void* stream);

/* Human-readable names. */
const char* cmpc_status_string(int status);
const char* cmpc_error_string(int err);
/* Device properties used by the bench roofline (peak fp64 FLOP/s from the datasheet unless measured). */
int cmpc_device_info(int* num_cu, int* clock_khz, char* arch_name, int arch_len);
/* Version string of the build, ending in the sha256 prefix of the library's sources ("... src <16 hex>"). */
const char* cmpc_version(void);

#ifdef __cplusplus
}
#endif

#endif /* CMPC_CMPC_H_ */
