// cmpc_kernels.hpp — internal host-side launcher declarations shared by the HIP translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cmpc_device.hpp"

namespace cmpc {

// largest condensed size served by an IPM size class (classes: n <= 64, 64 < n <= 128, 128 < n <= 256)
#define CMPC_IPM_MAX_N 256

// class-padded size of a condensed problem
// internal per-QP status of a QP the SQP no longer solves (CondenseArgs::skip); never returned to the caller
#define CMPC_STATUS_SKIPPED 100

__host__ __device__ inline int ipm_class(int n) { return n <= 64 ? 64 : (n <= 128 ? 128 : 256); }

// Position of H[i][j] inside a QP's class-packed block. Class 64 is stored in the 4 x 16-cyclic register order of
// k_ipm64 (element (i, j) is register 4*(i/4) + j/16 of lane 16*(i%4) + j%16), so each of that kernel's 64 loads
// is one contiguous 512-B row; classes 128 and 256 are row-major with stride npad.
__host__ __device__ inline int h_index(int npad, int i, int j) {
  return npad == 64 ? (((i >> 2) * 4 + (j >> 4)) * 64 + (i & 3) * 16 + (j & 15)) : i * npad + j;
}
// Classes 64 and 256 store only the lower-or-diagonal 16 x 16 tiles of H (h_stored: tile column <= tile row). The
// strictly upper tiles are exact transposes of the lower ones (the condensing builds them that way): k_ipm64 reads
// them as the mirrored elements of the 40 stored rows it loads anyway (20 KB instead of 32 KB of H per QP and
// iteration from MALL: headline PMC traffic 1.30 -> 0.73 GB per launch), k_ipm_tiled reads lower tiles only. Class
// 128 stays full: k_ipm128x's mirrored loads (16 rows per instruction) cost more time than the traffic they saved
// (configs 3 / 5: +5 % / +2.5 %, profiles/r03_hsym_ab.txt). Readers of an arbitrary element go through h_index_sym.
__host__ __device__ inline bool h_stored(int i, int j) { return (j >> 4) <= (i >> 4); }
__host__ __device__ inline int h_index_sym(int npad, int i, int j) {
  return (npad == 128 || h_stored(i, j)) ? h_index(npad, i, j) : h_index(npad, j, i);
}

// Per-QP workspace of one context (precision T), QP-major:
//   H [B][ld][ld], g [B][ld], tri_mu [B][ld/3], tri_lo/tri_hi [B][ld/3][5], tri_map [B][ld/3], nvar [B],
//   status [B], iters [B], u [B][ld]
template <typename T>
struct CondenseArgs {
  const DevModel* model;
  int ld;
  const double* x0;
  const double* xref;
  const double* foot;
  const uint8_t* contact;
  // SQP linearisation point [B][N][6] = (c_bar_k, F_bar_k = sum_i e_ik f_bar_ik), or null for (c_ref_k, 0): the
  // lever arm becomes p_ik - c_bar_k and L+ gains dt F_bar_k x (c_k - c_bar_k) (Taylor expansion of the bilinear
  // dt sum_i e_ik (p_ik - c_k) x f_ik of CentroidalMPC.cpp:86)
  const double* lin;
  // footholds as decision variables (cmpc_nlp_solve_batch; workgroup condensing only): dbar [B][N][NL][3] = the
  // iterate's foothold offsets by run start (cmpc_device.hpp lever_point), ubar [B][N][12] = the iterate's forces.
  // dbar != null adds one foothold triple per later stance run after the force triple of its first (step, leg):
  // columns dt e_d x f_bar_ik on the L rows at each step of the run, mu 0, rows [-x, x, -y, y, z] in the step box,
  // tri_map N L + s L + leg (oracle_condense_feet)
  const double* ubar;
  const double* dbar;
  // SQP: skip[q] != 0 marks a QP whose SQP has converged; it is not condensed (nvar 0 and, if it was SUCCESS, status
  // CMPC_STATUS_SKIPPED, so no IPM class, warm pack or list takes it). Null: every QP.
  const int* skip;
  T* H;
  T* g;
  T* tri_mu;
  T* tri_lo;
  T* tri_hi;
  int* tri_map;
  int* nvar;
  int* status;
  int n_lo;       // k_srbd_condense serves n_lo < n <= NMAX; when n_lo > 0 a smaller class ran first and left
                  // nvar[q] = n for every QP, so QPs with nvar[q] <= n_lo exit before any work
  const int* qlist;   // or null: workgroup b < *qcount serves QP qlist[b] (the class list of k_class_lists)
  const int* qcount;
  // k_ipm72 serves 64 < n <= 72 (cmpc_ctx::ipm72): the 128-class block of such a QP is written for rows and columns
  // < 80 only (k_ipm72 reads rows and columns < 72; the rest is the identity padding no kernel reads)
  int h72 = 0;
};

template <typename T>
struct IpmArgs {
  int ld;
  const T* H;
  const T* g;
  const T* tri_mu;
  const T* tri_lo;
  const T* tri_hi;
  const int* nvar;
  int* status;  // in: condense status (non-zero = skip); out: solver status
  int* iters;
  T* u;         // [B][ld]: out; in as the initial point when warm != 0
  int warm;     // warm start (hpipm_interface::Settings::warm_start, HpipmInterfaceSettings.h:54): u from a.u
  DevSettings s;
  unsigned long long* stamps;  // diagnostic builds only (-DCMPC_IPM_STAMPS): per-QP phase cycles, else null
  // final residuals (cmpc_get_residuals), or null: res[q][4] = (stat, eq = 0, ineq, comp) at the iterate where the
  // IPM stopped; res_scr [B][3][64] holds each lane's last (stat, ineq, comp) terms until the exit reduction
  // (k_ipm64 only: the 128 / 256 classes reduce in LDS)
  T* res_scr;
  double* res;
  // per-iteration statistics (cmpc_enable_stats), or null: stats[q][it][CMPC_STAT_COLS] for it < stats_cap
  double* stats;
  int stats_cap;
  // per-class QP lists (k_class_lists), or null: size class c's kernel maps workgroup b < qcount[c] to QP
  // qlist[c][b] and lets the rest exit, so a mixed batch dispatches the real QPs of a class first
  const int* qlist[3];
  const int* qcount;
  // result scatter in the kernel's epilogue (fused cold-start path without rollout: no k_expand launch), or
  // out_u = null: out_u[q] = [N][4][3] doubles (zero for swing legs), out_status[q], out_iters[q] (may be null);
  // tri_map[q][ld / 3] = k * 4 + leg of the QP's triple t (written by the condensing); out_nu = 12 N <= 256
  double* out_u;
  int* out_status;
  int* out_iters;
  const int* tri_map;
  int out_nu;
  // fused path (k_solve64), or app_list = null: a QP of a bigger class is appended to its class list,
  // app_list[c * app_ld + atomicAdd(&app_count[c], 1)] = q (c = 1: n <= 128, 2: n <= 256; order not fixed, each QP's
  // result does not depend on it), and workgroup 0 zeroes app_reset[0..2] (the next call's counters)
  int* app_list;
  int* app_count;
  int* app_reset;
  int app_ld;
};

// one size class of the workgroup condensing kernel: npad 128 (64 < n <= 128, or n <= 128 when n_lo = 0) or 256
template <typename T>
int launch_srbd_condense(const CondenseArgs<T>& a, int npad, int B, hipStream_t stream);
// n <= 64 QPs, one wavefront each (k_condense64.hip); QPs with n > 64 are left to launch_srbd_condense
template <typename T>
int launch_condense64(const CondenseArgs<T>& a, int B, hipStream_t stream);
#define CMPC_C64_MAXN 21

// Runs every IPM size class over the batch; each QP is served by the class matching its condensed size.
template <typename T>
int launch_ipm(const IpmArgs<T>& a, int B, hipStream_t stream);
int launch_ipm64(const IpmArgs<double>& a, int B, hipStream_t stream);   // n <= 64 (k_ipm64.hpp)
int launch_ipm64(const IpmArgs<float>& a, int B, hipStream_t stream);
// fused condensing + IPM of the n <= 64 class (k_solve64, k_ipm64.hpp); QPs with n > 64 only get their nvar hint
int launch_solve64(const IpmArgs<double>& a, const CondenseArgs<double>& c, int B, hipStream_t stream);
int launch_solve64(const IpmArgs<float>& a, const CondenseArgs<float>& c, int B, hipStream_t stream);
// fused workgroup condensing + IPM of the 64 < n <= 128 class over its class list (k_solve128, k_ipm128x.hpp)
int launch_solve128(const IpmArgs<double>& a, const CondenseArgs<double>& c, int B, hipStream_t stream);
int launch_solve128(const IpmArgs<float>& a, const CondenseArgs<float>& c, int B, hipStream_t stream);
int launch_ipm72(const IpmArgs<double>& a, int B, hipStream_t stream);   // 64 < n <= 72 (k_ipm72.hpp, one wave)
int launch_ipm72(const IpmArgs<float>& a, int B, hipStream_t stream);
int launch_ipm128(const IpmArgs<double>& a, int B, hipStream_t stream);  // 64 < n <= 128 (k_ipm128x.hpp, 4 waves)
int launch_ipm128(const IpmArgs<float>& a, int B, hipStream_t stream);   // 64 < n <= 128 (k_ipm128x.hpp, 4 waves)
int launch_ipm256(const IpmArgs<double>& a, int B, hipStream_t stream);  // 128 < n <= 256 (k_ipm256.hpp)
int launch_ipm256(const IpmArgs<float>& a, int B, hipStream_t stream);

// Stage-wise (Riccati) form of the whole hot path, one wavefront per QP (k_ric.hpp): SRBD linearisation, pyramid
// stacking and the Mehrotra IPM with Riccati Newton solves; no condensing, no H in the workspace. Writes the same
// per-QP outputs as condensing + IPM (u [B][ld] in condensed order, tri_map, nvar, status, iters, res, stats) and,
// when out_u is set, the caller's [N][4][3] forces directly.
template <typename T>
struct RicArgs {
  const DevModel* model;
  int N;               // horizon (host copy of model->N: picks the instantiation)
  int ld;
  const double* x0;
  const double* xref;
  const double* foot;
  const uint8_t* contact;
  const double* lin;   // SQP linearisation point [B][N][6] or null (CondenseArgs::lin)
  DevSettings s;
  T* u_ws;             // [B][ld] condensed-order solution, or null
  int* tri_map;        // [B][ld / 3] or null
  int* nvar;
  int* status;
  int* iters;
  double* out_u;       // direct scatter, or null
  int* out_status;
  int* out_iters;
  int out_nu;
  double* res;         // [B][4] or null
  double* stats;       // [B][stats_cap][CMPC_STAT_COLS] or null
  int stats_cap;
  // QP selection: null = workgroup b serves QP b; else QP qlist[b] for b < qcount[0], then qlist2[b - qcount[0]]
  // for b < qcount[0] + qcount[1] (qlist2 may be null)
  const int* qlist;
  const int* qlist2;
  const int* qcount;
};
#define CMPC_RIC_MAXN 21
// nmax: the largest condensed size of the QPs the launch can see (picks the LDS factor store and triples per lane)
template <typename T>
int launch_ric(const RicArgs<T>& a, int nmax, int grid, hipStream_t stream);

// res[q][4] of the QPs the IPM ran; NaN for the others (status 5 / 6)
int launch_residuals(const double* res_ws, const int* status, int B, double* out, hipStream_t stream);

struct ExpandArgs {
  const DevModel* model;
  int ld;
  const double* x0;
  const double* xref;
  const double* foot;
  const uint8_t* contact;
  const int* tri_map;
  const int* nvar;
  const int* status;
  const void* u_ws;  // T [B][ld]
  int precision;
  double* u;  // [B][N][L][3]
  double* x;  // [B][N+1][13] or null
  int* status_out;
  const int* iters_ws;
  int* iters_out;
  double* dq;  // [B][N][L][3] foothold offsets of the foothold triples (tri_map >= N L), or null
};
int launch_expand(const ExpandArgs& a, int B, hipStream_t stream);

int launch_generate(const cmpc_model& m, uint64_t seed, int64_t qp_offset, int B, int gait, double* x0, double* xref,
                    double* foot, uint8_t* contact, hipStream_t stream);

// test-hook layout conversions between user [B][ld][ld] double and the class-packed workspace
int launch_unpack_qp(const void* H_ws, const void* g_ws, const int* nvar, int precision, int ld, double* H, double* g,
                     int B, hipStream_t stream);
int launch_pack_qp(const double* H, const double* g, const double* tri_mu, const double* tri_lo, const double* tri_hi,
                   const int* nvar_in, int precision, int ld, void* H_ws, void* g_ws, void* mu_ws, void* lo_ws,
                   void* hi_ws, int* nvar_ws, int* status_ws, int B, hipStream_t stream);

// batched SQP on the bilinear NLP (k_sqp.hip)
struct SqpArgs {
  const DevModel* model;
  int N;               // horizon (host copy of model->N: sizes the kernels' LDS)
  const double* x0;
  const double* xref;
  const double* foot;
  const uint8_t* contact;
  double* u;           // [B][N][L][3]: in = the cold QP's solution (k_sqp_init), out = the SQP solution (final)
  double* x;           // [B][N+1][13] nonlinear rollout (final) or null
  int* status;         // [B] in: cold status; out: SQP status
  const int* iters;    // [B] cold QP iterations (may be null)
  double* uj;          // [B][N][12] iterate
  const double* uq;    // [B][N][12] QP solution at lin
  const int* status_q; // [B]
  const int* iters_q;  // [B]
  double* lin;         // [B][N][6]
  int* done;           // [B]
  int* qp_iters;       // [B] total IPM iterations
  int* sqp_iters;      // [B]
  int* count;          // [1] QPs not done (k_sqp_count)
  double tol;
  // footholds as decision variables (cmpc_nlp_solve_batch), all null for cmpc_sqp_solve_batch
  double* dj;          // [B][N][L][3] iterate's foothold offsets by run start (k_sqp_init: clamp(0, lo, hi))
  const double* dq;    // [B][N][L][3] the QP's foothold offsets (k_expand ExpandArgs::dq)
  double* feet;        // [B][N+1][L][3] foot_pos output (k_sqp_final) or null
};
// 0 init, 1 step, 2 final, 3 count, 4 lin <- the linearisation point (c_k, F_k) of the nonlinear rollout of u
int launch_sqp(int which, const SqpArgs& a, int B, hipStream_t stream);

// warm start: scatter a previous solution u_init [B][N][L][3] into the condensed order of each QP (tri_map)
// d_init [B][N][L][3] (or null): the foothold offsets for the foothold triples (tri_map >= N L)
int launch_pack_warm(const double* u_init, const int* tri_map, const int* nvar, const int* status, int precision,
                     int ld, int N, void* u_ws, int B, hipStream_t stream, const double* d_init = nullptr);
// receding-horizon shift of a solution: out[k] = in[min(k + shift, N - 1)] per QP
int launch_shift_inputs(const double* in, int N, int shift, double* out, int B, hipStream_t stream);

// per-class QP lists: lists [3][B] (ascending QP ids), counts [3]; one workgroup. by_status != 0: QPs with
// status == CMPC_SUCCESS, classed by nvar; by_status == 0: QPs with nvar > 0 (the condensing hints, written for every
// QP by the first condensing kernel). n_mid > 64: the 128 class is split, list 1 = n_mid < n <= 128 and a fourth
// list (lists + 3 B, count in counts[9]) = 64 < n <= n_mid (k_ipm72's QPs)
int launch_class_lists(const int* status, const int* nvar, int B, int by_status, int* lists, int* counts,
                       hipStream_t stream, int n_mid = 0);

// widen/narrow helpers used by the test hooks
int launch_convert_f32_to_f64(const float* in, double* out, size_t n, hipStream_t stream);
int launch_convert_f64_to_f32(const double* in, float* out, size_t n, hipStream_t stream);

// feedback policy dU/dx0 at a solution (k_policy.hip); reads the condensing workspace (H, tri_map, nvar, status)
template <typename T>
struct PolicyArgs {
  const DevModel* model;
  int ld;
  int q0;               // first QP of this launch (blockIdx.x + q0); scratch is indexed by blockIdx.x
  const double* xref;
  const double* foot;
  const uint8_t* contact;
  const double* u;      // [B][N][L][3] solution
  const T* H;
  const int* tri_map;
  const int* nvar;
  const int* status;    // condense status
  double act_tol;
  double* K;            // [B][12N][13]
  int* nfree;           // [B] or null
  int* status_out;      // [B]
  double* scratch;      // [launch QPs][stride]
  size_t stride;
  const double* lin;    // [B][N][6] linearisation point of the QP (CondenseArgs::lin) or null: the reference one
};
size_t policy_scratch_doubles(int N, int ld);
template <typename T>
int launch_policy(const PolicyArgs<T>& a, int nq, hipStream_t stream);

}  // namespace cmpc
