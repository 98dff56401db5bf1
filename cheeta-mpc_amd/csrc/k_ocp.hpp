// k_ocp.hpp — stage-wise OCP-QP interior-point solver (the HpipmInterface::solve path, reference
// ocs2_sqp/hpipm_catkin/src/HpipmInterface.cpp:166-301): shared layout of the device kernels (k_ocp.hip) and the
// host API (ocp_api.cpp).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>

namespace cmpc {

constexpr int OCP_NT = 256;       // threads per problem (one workgroup)
constexpr int OCP_ROWS = 17;      // per-row workspace arrays (see OcpLayout::row)
constexpr int OCP_MAX_NX = 63;    // nx + 1 <= 64
constexpr int OCP_ONE_PER_CU_MAX = 256;  // batches up to this size run one problem per CU (k_ocp_ipm<64, 1>)
constexpr int OCP_MAX_NG = 64;    // general-constraint rows per node
constexpr int OCP_MAX_N = 4096;   // stages

// Per-row arrays, in order, each [m] per problem (m = sum_k ng_k)
enum OcpRow { R_C = 0, R_LG, R_UG, R_TL, R_TU, R_LL, R_LU, R_RL, R_RU, R_RML, R_RMU, R_W, R_DTL, R_DTU, R_DLL, R_DLU, R_SIG };

// Problem dimensions (shared by every problem of a batch, HPIPM's d_ocp_qp_dim) and the per-problem workspace map.
// Device arrays are owned by the cmpc_ocp handle (allocated once in cmpc_ocp_create, as HpipmInterface::resize
// reserves HPIPM's memory, HpipmInterface.cpp:92-129).
struct OcpLayout {
  int N, nx, nU, m, nzp, ngmax, numax;
  int nK, nM;                    // sum nu_k nx, sum nu_k^2
  const int* nu;                 // [N+1], nu[N] = 0
  const int* ng;                 // [N+1]
  const int* cu;                 // [N+2] offsets of u_k in u
  const int* cr;                 // [N+2] offsets of node k's rows
  const int* cK;                 // [N+1] offsets of K_k (nu_k x nx, column-major)
  const int* cM;                 // [N+1] offsets of nu_k x nu_k blocks (Lf_k, Lr_k; column-major)
  const long long* orec;         // [N+1][8] record offsets: A, B, b (k < N), Q, S, R, q, r (k <= N)
  const long long* ocon;         // [N+1][4] constraint-record offsets: C, D, e, (pad)
  const int* ustage;             // [nU] stage of each input entry
  const int* rstage;             // [m] node of each row
  const int* cHp;                // [N+1] offsets of the stages' Hc images (ocp_chain.hpp; cHp[N] = per-problem size)
  long long rec_size, crec_size;
  // workspace (doubles) per problem: stride and array offsets
  long long ws_stride;
  long long o_x, o_u, o_pi, o_rgu, o_rgx, o_rb, o_gu, o_gx, o_du, o_dx, o_dpi, o_rows, o_P, o_pv, o_K, o_kf,
      o_Lf, o_Acl, o_h, o_y, o_bcl;  // o_Lf: the u-block's LDL' columns per stage (nu_k x nu_k, column-major)
};

// Grid form (k_ocp_grid, batches up to OCP_GRID_MAX_B): G workgroups per problem, one per CU, B G <= OCP_GRID_MAX_WG
constexpr int OCP_GRID_MAX_B = 32;
constexpr int OCP_GRID_MAX_G = 32;
constexpr int OCP_GRID_MAX_WG = 256;
constexpr int OCP_GRID_TIMEOUT = 8;  // status of a grid-form solve whose barrier timed out (= CMPC_GRID_TIMEOUT)
int ocp_grid_width(int N, int B, int want);  // G for a batch by the CU count (0: not the grid form)
int ocp_grid_for(const OcpLayout& L, int B, int want);  // the same, capped by the kernel's co-residency

// Segment buffer of the grid form's partitioned factorisation (ocp_part.hpp: seg_esz / seg_bsz), doubles
__host__ __device__ inline int seg_esz(int nx) { return (3 * nx * nx + 2 * nx + 1) & ~1; }
__host__ __device__ inline int seg_bsz(int nx) { return (nx * nx + nx + 1) & ~1; }

// Limits of the latency form of the factorisation (ocp_chain.hpp, small batches)
constexpr int OCP_CHAIN_MAX_NX = 27;
constexpr int OCP_CHAIN_MAX_NU = 36;
constexpr int OCP_CHAIN_MAX_N1 = 60;  // nu_k + nx + 1: two 4 x 4 blocks of the stage matrix per lane of wave 0

struct OcpSolveArgs {
  OcpLayout L;
  const double* x0;    // [B][nx]
  const double* rec;   // [B][rec_size]
  const double* crec;  // [B][crec_size] or nullptr (m == 0)
  double* ws;          // [B][ws_stride]
  double* x;           // [B][(N+1) nx]
  double* u;           // [B][nU]
  int* status;         // [B]
  int* iters;          // [B]
  double* res;         // [B][4]
  double* stats;       // [B][stat_rows][10] or nullptr
  double* linres;      // [B][stat_rows][4] or nullptr: HPIPM's lin res stat / eq / ineq / comp (cmpc_ocp_set_linres)
  int stat_rows;
  int iter_max;
  int warm;  // Settings.warm_start: x (nodes >= 1), u start from x / u (HPIPM's primal warm start)
  int par_res;  // residuals of all nodes at once (small batches, set by launch_ocp_ipm) or node by node staged
  int fast;     // latency form of the factorisation (ocp_chain.hpp; k_ocp_ipm<64, 1> only, set by launch_ocp_ipm)
  double* hp;   // [B][hp_stride] Hc images of the latency form (nullptr when the handle has none)
  long long hp_stride;
  int G;           // grid form: workgroups per problem (0: one workgroup per problem)
  unsigned* bar;   // grid form: [B][4] barrier counter, fail word (zero at allocation; every launch leaves them zero)
  double* gpart;   // grid form: [B][G][8] per-workgroup partials of the reductions
  long long grid_timeout;  // grid form: barrier wait bound in ticks of the 100-MHz real-time counter (< 0: time out
                           // at the first barrier, the debug switch of the fallback test)
  unsigned* fallbacks;     // grid form: count of problems re-solved by k_ocp_fallback (cmpc_ocp_fallback_count)
  double* seg;             // grid form: [B][seg_stride] segment elements and boundary values (ocp_part.hpp), or null
  long long seg_stride;
  int nseg;                // grid form: segments of the partitioned factorisation (0 auto, 1 the serial chain)
  int ric;         // grid form: the exit Riccati quantities into ricP .. ricst (cmpc_ocp_set_keep_riccati)
  double *ricP, *ricp, *ricK, *rick, *ricLr;
  int* ricst;
  double alpha_min, mu0, tol_stat, tol_eq, tol_ineq, tol_comp, reg;
};

// Riccati quantities at the exit point of the last solve (cmpc_ocp_riccati): P [(N+1)][nx][nx], p [(N+1)][nx],
// K [nK], k [nU], Lr [nM] (HPIPM's ric_Lr, lower) per problem (column-major blocks), status [B].
struct OcpRicArgs {
  OcpSolveArgs S;
  double *P, *p, *K, *k, *Lr;
  int* rstatus;
};

// LDS bytes of the kernels for a layout (the latency form's, 0 when the layout is outside its limits)
size_t ocp_lds_bytes(const OcpLayout& L);
size_t ocp_chain_lds_bytes(const OcpLayout& L, int numax);
// launch_ocp_ipm takes the latency form for B <= OCP_ONE_PER_CU_MAX when a.fast != 0 on entry (the handle has it)
int launch_ocp_ipm(const OcpSolveArgs& a, int B, hipStream_t stream);
int launch_ocp_ric(const OcpRicArgs& a, int B, hipStream_t stream);
#ifdef CMPC_OCP_CHAIN_LAB
int launch_ocp_chain_lab(const OcpSolveArgs& a, int B, hipStream_t stream);
#endif

}  // namespace cmpc
