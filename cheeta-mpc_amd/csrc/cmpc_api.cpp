// cmpc_api.cpp — implementation of the C ABI (include/cmpc/cmpc.h): contexts, device workspace, launches.
//
// Ownership follows HPIPM's memsize/create pattern as wrapped by HpipmInterface (HpipmInterface.cpp:46-83, :104-128):
// the context owns (or borrows) one device slab sized by cmpc_memsize and re-uses it for every batch up to
// max_batch; no allocation happens on the solve path (graph-capturable). Settings map 1:1 onto
// hpipm_interface::Settings (HpipmInterfaceSettings.h:44-57). No exception crosses the ABI.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "cmpc/cmpc.h"
#include "cmpc_device.hpp"
#include "cmpc_kernels.hpp"
#include "src_hash.h"

using namespace cmpc;

struct cmpc_ctx {
  cmpc_model model;
  cmpc_settings settings;
  int precision;
  int max_batch;
  int ld;
  int device;
  DevModel* d_model;
  char* ws;
  bool own_ws;
  size_t ws_bytes;
  // typed views into ws
  void* H;
  void* g;
  void* tri_mu;
  void* tri_lo;
  void* tri_hi;
  void* u;
  int* tri_map;
  int* nvar;
  int* status;
  int* iters;
  int* qlist;   // [4][max_batch] per-class QP lists (k_class_lists; the fourth: 64 < n <= 72 for k_ipm72)
  int* qcount;  // [10]: k_class_lists' counts, the fused path's two alternating append counters, the fourth list's
  int fused_parity = 0;  // fused path: this call appends to qcount[3 + 3 parity] and zeroes the other slice
  // kernel path (cmpc_set_path; every choice gives bit-identical results):
  bool fused;     // cold-start cmpc_solve_batch runs the fused n <= 64 kernel (k_solve64); possible when N <= 21
  bool fused128;  // fused path: the 64 < n <= 128 class as one condensing + IPM launch (k_solve128)
  bool direct;    // fused path without rollout: the IPM kernels scatter the results (no k_expand)
  int ric = 0;    // stage-wise (Riccati) kernel k_ric: 0 off, 1 the n > 64 classes of the fused path, 2 every QP
  bool ipm72 = true;  // separate IPM launches: 64 < n <= 72 on the bordered one-wave kernel (k_ipm72)
  double *lin, *uj, *uq, *dj, *dq;
  int *stq, *itq, *done, *sqpi, *qpi, *cnt;
  void* res_scr;
  double* res;
  double* stats = nullptr;  // [max_batch][stats_rows][CMPC_STAT_COLS] (cmpc_enable_stats)
  int stats_rows = 0;
  // host-API staging (grown on demand, outside the async path)
  char* stage;
  size_t stage_bytes;
  // feedback-policy scratch (cmpc_policy_batch, grown on demand)
  double* pol = nullptr;
  size_t pol_bytes = 0;
  // stage profiling (cmpc_profile_begin/end)
  std::vector<hipEvent_t> prof_ev;
  int prof_max;
  int prof_calls;
  bool profiling;
};

namespace {

#define HIP_OK(expr)                      \
  do {                                    \
    if ((expr) != hipSuccess) return CMPC_ERR_HIP; \
  } while (0)

int ld_for(const cmpc_model& m) {
  const int nf = CMPC_NU * m.N;
  return nf <= 64 ? 64 : (nf <= 128 ? 128 : 256);
}

struct Layout {
  size_t H, g, mu, lo, hi, u, map, nvar, status, iters, qlist, qcount, lin, uj, uq, dj, dq, stq, itq, done, sqpi, qpi,
      cnt, res_scr, res, total;
};

Layout layout(int ld, int precision, int B, int N) {
  const size_t es = precision == CMPC_F64 ? 8 : 4;
  const size_t nt = (size_t)(ld / 3);
  Layout L;
  size_t o = 0;
  auto take = [&](size_t bytes) {
    const size_t at = o;
    o += (bytes + 255) & ~(size_t)255;
    return at;
  };
  L.H = take((size_t)B * ld * ld * es);
  L.g = take((size_t)B * ld * es);
  L.mu = take((size_t)B * nt * es);
  L.lo = take((size_t)B * nt * 5 * es);
  L.hi = take((size_t)B * nt * 5 * es);
  L.u = take((size_t)B * ld * es);
  L.map = take((size_t)B * nt * sizeof(int));
  L.nvar = take((size_t)B * sizeof(int));
  L.status = take((size_t)B * sizeof(int));
  L.iters = take((size_t)B * sizeof(int));
  L.qlist = take((size_t)4 * B * sizeof(int));  // [3]: k_ipm72's part of the 128 class (run_ipm_classes)
  L.qcount = take(10 * sizeof(int));  // [0..2] k_class_lists; [3..5], [6..8] appended by k_solve64 (call parity); [9]
  // SQP (cmpc_sqp_solve_batch): linearisation points, iterate, QP solution, per-QP flags and counters
  L.lin = take((size_t)B * MAXN * 6 * 8);
  L.uj = take((size_t)B * MAXN * NU * 8);
  L.uq = take((size_t)B * MAXN * NU * 8);
  L.dj = take((size_t)B * N * NU * 8);  // cmpc_nlp_solve_batch: foothold offsets of the iterate and of the QP
  L.dq = take((size_t)B * N * NU * 8);
  L.stq = take((size_t)B * sizeof(int));
  L.itq = take((size_t)B * sizeof(int));
  L.done = take((size_t)B * sizeof(int));
  L.sqpi = take((size_t)B * sizeof(int));
  L.qpi = take((size_t)B * sizeof(int));
  L.cnt = take(sizeof(int));
  L.res_scr = take((size_t)B * 3 * 64 * es);   // per-lane residual terms of k_ipm64's last IPM iteration
  L.res = take((size_t)B * 4 * sizeof(double));  // final residuals (cmpc_get_residuals)
  L.total = o;
  return L;
}

// Model constants (host derivation of SURVEY App. A; weights indexed as CentroidalMPC.cpp:203-231).
void derive_model(const cmpc_model& m, DevModel& d) {
  std::memset(&d, 0, sizeof(d));
  const int L = m.n_legs;
  const double* w = m.weights;
  d.N = m.N;
  d.L = L;
  d.mass = m.mass;
  d.dt = m.dt;
  d.dt_over_m = m.dt / m.mass;
  for (int i = 0; i < L; ++i) {
    d.mu[i] = m.mu[i];
    for (int c = 0; c < 3; ++c) {
      d.Wf[3 * i + c] = w[9 + 3 * L + 3 * i + c];
      d.Wr[3 * i + c] = w[9 + 6 * L + 3 * i + c];
      d.Wp[3 * i + c] = w[9 + 3 * i + c];
    }
  }
  for (int k = 0; k <= m.N && k <= MAXN; ++k) {
    const double wz = (w[2] / 2.0) * std::exp(-(double)k) + w[2] / 2.0;  // CentroidalMPC.cpp:205
    double* q = d.qdiag[k];
    q[0] = 2.0 * w[0];
    q[1] = 2.0 * w[1];
    q[2] = 2.0 * (wz * wz);  // sumsqr(weightCoMZ .* dz) squares the weight, :210
    for (int j = 3; j < 9; ++j) q[j] = 2.0 * w[j];
    for (int j = 0; j < 3; ++j) q[9 + j] = 2.0 * m.theta_weights[j];
    q[12] = 0.0;
  }
  for (int r = 0; r < 5; ++r) d.ub[r] = m.force_ub[r];
  const double* I = m.inertia;
  const double c00 = I[4] * I[8] - I[5] * I[7], c01 = I[5] * I[6] - I[3] * I[8], c02 = I[3] * I[7] - I[4] * I[6];
  const double det = I[0] * c00 + I[1] * c01 + I[2] * c02;
  const double inv = 1.0 / det;
  d.inv_inertia[0] = c00 * inv;
  d.inv_inertia[1] = (I[2] * I[7] - I[1] * I[8]) * inv;
  d.inv_inertia[2] = (I[1] * I[5] - I[2] * I[4]) * inv;
  d.inv_inertia[3] = c01 * inv;
  d.inv_inertia[4] = (I[0] * I[8] - I[2] * I[6]) * inv;
  d.inv_inertia[5] = (I[2] * I[3] - I[0] * I[5]) * inv;
  d.inv_inertia[6] = c02 * inv;
  d.inv_inertia[7] = (I[1] * I[6] - I[0] * I[7]) * inv;
  d.inv_inertia[8] = (I[0] * I[4] - I[1] * I[3]) * inv;
}

// hpipm_interface::Settings ranges (cmpc.h): modes 0..3, predictor-corrector only, positive tolerances.
bool settings_ok(const cmpc_settings& s) {
  return s.hpipm_mode >= 0 && s.hpipm_mode <= 3 && s.iter_max >= 0 && s.alpha_min > 0 && s.mu0 > 0 &&
         s.tol_stat > 0 && s.tol_eq > 0 && s.tol_ineq > 0 && s.tol_comp > 0 && s.reg_prim >= 0 &&
         (s.warm_start == 0 || s.warm_start == 1) && s.pred_corr == 1 && (s.ric_alg == 0 || s.ric_alg == 1);
}

bool model_ok(const cmpc_model* m) {
  return m && m->N >= 1 && m->N <= MAXN && m->n_legs == CMPC_MAX_LEGS && m->mass > 0 && m->dt > 0;
}

DevSettings dev_settings(const cmpc_settings& s) {
  DevSettings d;
  d.iter_max = s.iter_max;
  d.alpha_min = s.alpha_min;
  d.mu0 = s.mu0;
  d.tol_stat = s.tol_stat;
  d.tol_ineq = s.tol_ineq;
  d.tol_comp = s.tol_comp;
  d.reg_prim = s.reg_prim;
  return d;
}

template <typename T>
CondenseArgs<T> condense_args(cmpc_ctx* c, const double* x0, const double* xref, const double* foot,
                              const uint8_t* contact) {
  CondenseArgs<T> a;
  a.model = c->d_model;
  a.ld = c->ld;
  a.x0 = x0;
  a.xref = xref;
  a.foot = foot;
  a.contact = contact;
  a.lin = nullptr;
  a.ubar = nullptr;
  a.dbar = nullptr;
  a.skip = nullptr;
  a.H = (T*)c->H;
  a.g = (T*)c->g;
  a.tri_mu = (T*)c->tri_mu;
  a.tri_lo = (T*)c->tri_lo;
  a.tri_hi = (T*)c->tri_hi;
  a.tri_map = c->tri_map;
  a.nvar = c->nvar;
  a.status = c->status;
  a.n_lo = 0;
  a.h72 = c->ipm72 ? 1 : 0;
  a.qlist = nullptr;
  a.qcount = nullptr;
  return a;
}

template <typename T>
IpmArgs<T> ipm_args(cmpc_ctx* c) {
  IpmArgs<T> a;
  a.ld = c->ld;
  a.H = (const T*)c->H;
  a.g = (const T*)c->g;
  a.tri_mu = (const T*)c->tri_mu;
  a.tri_lo = (const T*)c->tri_lo;
  a.tri_hi = (const T*)c->tri_hi;
  a.nvar = c->nvar;
  a.status = c->status;
  a.iters = c->iters;
  a.u = (T*)c->u;
  a.warm = 0;
  a.s = dev_settings(c->settings);
  a.stamps = nullptr;
  a.res_scr = (T*)c->res_scr;
  a.res = c->res;
  a.stats = c->stats;
  a.stats_cap = c->stats_rows;
  for (int k = 0; k < 3; ++k) a.qlist[k] = nullptr;
  a.qcount = nullptr;
  a.out_u = nullptr;
  a.out_status = nullptr;
  a.out_iters = nullptr;
  a.tri_map = c->tri_map;
  a.out_nu = c->model.N * 12;
  a.app_list = nullptr;
  a.app_count = nullptr;
  a.app_reset = nullptr;
  a.app_ld = 0;
  return a;
}

// n <= 64 QPs go through the one-wave condensing kernel (possible only for N <= 21); the workgroup kernel serves
// the 128 and 256 classes. When the context holds more than one class, the first condensing kernel leaves
// nvar[q] = n (0 if rejected) for every QP; k_class_lists turns those hints into per-class lists, so each bigger
// class's kernel dispatches only its own QPs first, and the IPM reuses the same lists (*lists = true).
template <typename T>
int run_condense_t(cmpc_ctx* c, int B, const double* x0, const double* xref, const double* foot,
                   const uint8_t* contact, hipStream_t st, const double* lin, bool* lists, const double* ubar,
                   const double* dbar, const int* skip) {
  CondenseArgs<T> a = condense_args<T>(c, x0, xref, foot, contact);
  a.lin = lin;
  a.ubar = ubar;
  a.dbar = dbar;
  a.skip = skip;
  *lists = false;
  // the one-wave condensing has no foothold columns: with footholds every QP goes through the workgroup kernel
  const bool small = c->model.N <= CMPC_C64_MAXN && !dbar;
  // footholds, N <= 21, k_ipm72 on: the two-wave foothold condensing takes n <= 72 first (four workgroups per CU
  // against two for the 128 class's), the 128 class the rest of its list
  const bool feet72 = dbar && c->ipm72 && c->ld >= 128 && c->model.N <= CMPC_C64_MAXN;
  int r = small ? launch_condense64<T>(a, B, st) : 0;
  if (r == 0 && feet72) r = launch_srbd_condense<T>(a, 72, B, st);
  else if (r == 0 && !small) r = launch_srbd_condense<T>(a, c->ld < 128 ? 64 : 128, B, st);  // n_lo = 0: 64, 128
  if (r != 0 || c->ld < 128) return r;
  if (launch_class_lists(c->status, c->nvar, B, 0, c->qlist, c->qcount, st) != 0) return -2;
  *lists = true;
  if (small || feet72) {
    a.n_lo = feet72 ? 72 : 64;
    a.qlist = c->qlist + (size_t)1 * B;
    a.qcount = c->qcount + 1;
    r = launch_srbd_condense<T>(a, 128, B, st);
  }
  if (r == 0 && c->ld > 128) {
    a.n_lo = 128;
    a.qlist = c->qlist + (size_t)2 * B;
    a.qcount = c->qcount + 2;
    r = launch_srbd_condense<T>(a, 256, B, st);
  }
  return r;
}

int run_condense(cmpc_ctx* c, int B, const double* x0, const double* xref, const double* foot,
                 const uint8_t* contact, hipStream_t st, const double* lin = nullptr, bool* lists = nullptr,
                 const double* ubar = nullptr, const double* dbar = nullptr, const int* skip = nullptr) {
  bool dummy = false;
  if (!lists) lists = &dummy;
  int r;
  if (c->precision == CMPC_F64)
    r = run_condense_t<double>(c, B, x0, xref, foot, contact, st, lin, lists, ubar, dbar, skip);
  else
    r = run_condense_t<float>(c, B, x0, xref, foot, contact, st, lin, lists, ubar, dbar, skip);
  return r == 0 ? CMPC_OK : (r == -1 ? CMPC_ERR_ARG : CMPC_ERR_HIP);
}

// Size classes, in order on the caller's stream. When the context can hold more than one class (ld >= 128), the
// QPs of each class are first compacted into a list (k_class_lists), so each class kernel dispatches its own QPs
// first and its surplus workgroups exit at the end of the grid; without the lists a class's QPs sat between the
// other classes' early-exit workgroups (mixed gait, config 5: IPM 2.31 -> 1.85-1.89 ms). Measured against running
// the bigger classes concurrently on a forked side stream: +1.5 % on the mixed batch, -1.5..-2.5 % on the headline
// (events and an empty launch on the critical path), so the classes run back to back. (A fork of the fused path that
// built its lists off the contact tables and started beside k_solve64 measured config 5 +2 %, headline -2..3 %; it
// was removed)

template <typename T>
int run_ipm_classes(cmpc_ctx* c, const IpmArgs<T>& a, int B, hipStream_t st, bool lists_ready) {
  if (B <= 0) return 0;
  if (c->ld < 128) return launch_ipm<T>(a, B, st);  // one class
  // with k_ipm72 the lists are always rebuilt here, the 128 class split at n = 72 (list 3, count qcount[9])
  if ((c->ipm72 || !lists_ready) &&
      launch_class_lists(a.status, a.nvar, B, 1, c->qlist, c->qcount, st, c->ipm72 ? 72 : 0) != 0)
    return -2;
  IpmArgs<T> al = a;
  for (int k = 0; k < 3; ++k) al.qlist[k] = c->qlist + (size_t)k * B;
  al.qcount = c->qcount;
  int r = launch_ipm64(al, B, st);
  if (r == 0 && c->ipm72) {  // 64 < n <= 72 on one wave (the NLP's trot subproblems); list 1 holds n > 72 now
    IpmArgs<T> a72 = al;
    a72.qlist[1] = c->qlist + (size_t)3 * B;
    a72.qcount = c->qcount + 8;  // k_ipm72 reads qcount[1] = the fourth list's count, qcount[9]
    r = launch_ipm72(a72, B, st);
  }
  if (r == 0) r = launch_ipm128(al, B, st);
  if (r == 0 && c->ld >= 256) r = launch_ipm256(al, B, st);
  return r;
}

template <typename T>
RicArgs<T> ric_args(cmpc_ctx* c, const double* x0, const double* xref, const double* foot, const uint8_t* contact,
                    double* out_u, int* out_status, int* out_iters) {
  RicArgs<T> a;
  a.model = c->d_model;
  a.N = c->model.N;
  a.ld = c->ld;
  a.x0 = x0;
  a.xref = xref;
  a.foot = foot;
  a.contact = contact;
  a.lin = nullptr;
  a.s = dev_settings(c->settings);
  a.u_ws = (T*)c->u;
  a.tri_map = c->tri_map;
  a.nvar = c->nvar;
  a.status = c->status;
  a.iters = c->iters;
  a.out_u = out_u;
  a.out_status = out_status;
  a.out_iters = out_iters;
  a.out_nu = c->model.N * 12;
  a.res = c->res;
  a.stats = c->stats;
  a.stats_cap = c->stats_rows;
  a.qlist = nullptr;
  a.qlist2 = nullptr;
  a.qcount = nullptr;
  return a;
}

// Stage-wise path for every QP (CMPC_PATH_RICCATI = 2): one k_ric launch, no condensing.
template <typename T>
int run_ric_all_t(cmpc_ctx* c, int B, const double* x0, const double* xref, const double* foot,
                  const uint8_t* contact, hipStream_t st, double* out_u, int* out_status, int* out_iters) {
  RicArgs<T> ra = ric_args<T>(c, x0, xref, foot, contact, out_u, out_status, out_iters);
  return launch_ric<T>(ra, 12 * c->model.N, B, st);
}

// Fused path (cold-start cmpc_solve_batch, N <= 21): k_solve64 condenses and solves the whole n <= 64 class in one
// launch (the condensing's MFMA/latency-bound phase overlaps the IPM of the co-resident wave, and the first Newton
// matrix starts from the condensing's registers instead of an H round trip); the bigger classes follow as before:
// their nvar hints -> k_class_lists -> workgroup condensing -> their IPM kernels. ev1 (profiling) is recorded after
// the fused launch.
// out_u != null: every IPM kernel scatters its QPs' results into the caller's u / status / iters (no k_expand launch;
// the rejected QPs are written by k_solve64, which sees them first).
template <typename T>
int run_fused_t(cmpc_ctx* c, int B, const double* x0, const double* xref, const double* foot, const uint8_t* contact,
                hipStream_t st, hipEvent_t ev1, double* out_u, int* out_status, int* out_iters) {
  CondenseArgs<T> ca = condense_args<T>(c, x0, xref, foot, contact);
  ca.h72 = 0;  // the fused path's 128 class (k_solve128 / k_ipm128) reads the whole block
  IpmArgs<T> ia = ipm_args<T>(c);
  ia.out_u = out_u;
  ia.out_status = out_status;
  ia.out_iters = out_iters;
  // the bigger classes' lists are appended by the fused kernel itself (no k_class_lists launch); the counters of
  // this call were zeroed by the previous fused call (or at cmpc_create), this call zeroes the next call's
  int* cnt = c->qcount + 3 + 3 * c->fused_parity;
  if (c->ld >= 128) {
    ia.app_list = c->qlist;
    ia.app_count = cnt;
    ia.app_reset = c->qcount + 3 + 3 * (c->fused_parity ^ 1);
    ia.app_ld = B;
  }
  if (c->ld >= 128) {
    // Under stream capture the graph is replayed with this call's parity frozen, so nothing would re-zero this
    // slice between replays: the captured call zeroes it itself (a memset node); uncaptured calls keep relying on
    // the previous call's reset (no extra launch on the hot path).
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess) return -2;
    if (cs == hipStreamCaptureStatusActive && hipMemsetAsync(cnt, 0, 3 * sizeof(int), st) != hipSuccess) return -2;
  }
  if (launch_solve64(ia, ca, B, st) != 0) return -2;
  if (c->ld < 128) return 0;
  c->fused_parity ^= 1;
  if (ev1 && hipEventRecord(ev1, st) != hipSuccess) return -2;
  IpmArgs<T> al = ia;
  al.app_list = nullptr;
  al.app_count = al.app_reset = nullptr;
  for (int k = 0; k < 3; ++k) al.qlist[k] = c->qlist + (size_t)k * B;  // list 0 unused here
  al.qcount = cnt;
  if (c->ric == 1) {  // stage-wise kernel over the appended lists (n <= 128 first, then n > 128)
    RicArgs<T> ra = ric_args<T>(c, x0, xref, foot, contact, out_u, out_status, out_iters);
    ra.qlist = c->qlist + (size_t)1 * B;
    ra.qcount = cnt + 1;
    const int nfull = 12 * c->model.N;
    if (nfull <= 128) {  // one launch over both lists
      ra.qlist2 = c->qlist + (size_t)2 * B;
      return launch_ric<T>(ra, nfull, B, st);
    }
    ra.qlist2 = nullptr;
    if (launch_ric<T>(ra, 128, B, st) != 0) return -2;
    ra.qlist = c->qlist + (size_t)2 * B;
    ra.qcount = cnt + 2;
    return launch_ric<T>(ra, nfull, B, st);
  }
  ca.n_lo = 64;
  ca.qlist = c->qlist + (size_t)1 * B;
  ca.qcount = cnt + 1;
  // 64 < n <= 128: condensing and IPM in one launch (k_solve128), or (CMPC_FUSED128=0) two
  int r = c->fused128 ? launch_solve128(al, ca, B, st) : launch_srbd_condense<T>(ca, 128, B, st);
  if (r == 0 && !c->fused128) r = launch_ipm128(al, B, st);
  if (r == 0 && c->ld > 128) {
    ca.n_lo = 128;
    ca.qlist = c->qlist + (size_t)2 * B;
    ca.qcount = cnt + 2;
    r = launch_srbd_condense<T>(ca, 256, B, st);
    if (r == 0) r = launch_ipm256(al, B, st);
  }
  return r;
}

// lists_ready: the condensing of this call built the class lists (run_condense), else they are built here
int run_ipm(cmpc_ctx* c, int B, hipStream_t st, int warm, bool lists_ready) {
  int r;
  if (c->precision == CMPC_F64) {
    IpmArgs<double> a = ipm_args<double>(c);
    a.warm = warm;
    r = run_ipm_classes<double>(c, a, B, st, lists_ready);
  } else {
    IpmArgs<float> a = ipm_args<float>(c);
    a.warm = warm;
    r = run_ipm_classes<float>(c, a, B, st, lists_ready);
  }
  return r == 0 ? CMPC_OK : CMPC_ERR_HIP;
}

int ensure_stage(cmpc_ctx* c, size_t bytes) {
  if (c->stage_bytes >= bytes) return CMPC_OK;
  if (c->stage) (void)hipFree(c->stage);
  c->stage = nullptr;
  c->stage_bytes = 0;
  HIP_OK(hipMalloc((void**)&c->stage, bytes));
  c->stage_bytes = bytes;
  return CMPC_OK;
}


}  // namespace

extern "C" {

void cmpc_settings_default(cmpc_settings* s) {
  if (!s) return;
  s->hpipm_mode = 1;  // SPEED (HpipmInterfaceSettings.h:45)
  s->iter_max = 30;
  s->alpha_min = 1e-12;
  s->mu0 = 1e1;
  s->tol_stat = 1e-6;
  s->tol_eq = 1e-8;
  s->tol_ineq = 1e-8;
  s->tol_comp = 1e-8;
  s->reg_prim = 1e-12;
  s->warm_start = 0;
  s->pred_corr = 1;
  s->ric_alg = 0;
}

void cmpc_model_default(cmpc_model* m, int N) {
  if (!m) return;
  std::memset(m, 0, sizeof(*m));
  // CentoidMPCTest.cpp:12-33
  static const double w[CMPC_NUM_WEIGHTS] = {1,   1,   100, 0.5, 0.5, 0,   2,   2,   8,   0.2, 0.2, 0.2,
                                             0.3, 0.3, 0.3, 0.1, 0.1, 0.1, 0.2, 0.2, 0.2, 0.3, 0.3, 0.3,
                                             0.1, 0.1, 0.1, 0.2, 0.2, 0.2, 0.3, 0.3, 0.3, 0.1, 0.1, 0.1,
                                             0.2, 0.2, 0.2, 0.3, 0.3, 0.3, 0.1, 0.1, 0.1};
  m->N = N;
  m->n_legs = CMPC_MAX_LEGS;
  m->mass = 8.0;
  m->dt = 0.01;
  const double I[9] = {0.07, 0, 0, 0, 0.26, 0, 0, 0, 0.28};
  std::memcpy(m->inertia, I, sizeof(I));
  for (int i = 0; i < CMPC_MAX_LEGS; ++i) m->mu[i] = 0.8;
  std::memcpy(m->weights, w, sizeof(w));
  for (int r = 0; r < 4; ++r) m->force_ub[r] = 5000.0;       // CentroidalMPC.cpp:182-183
  m->force_ub[4] = m->mass * 9.81 * m->n_legs;
}

size_t cmpc_memsize(const cmpc_model* model, int precision, int max_batch) {
  if (!model_ok(model) || max_batch <= 0) return 0;
  return layout(ld_for(*model), precision, max_batch, model->N).total;
}

int cmpc_create(const cmpc_model* model, const cmpc_settings* settings, int precision, int max_batch, void* dev_mem,
                cmpc_ctx** out) {
  if (!out || !model_ok(model) || max_batch <= 0 || (precision != CMPC_F64 && precision != CMPC_F32) ||
      (settings && !settings_ok(*settings)))
    return CMPC_ERR_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return CMPC_ERR_NO_DEVICE;
  cmpc_ctx* c = new (std::nothrow) cmpc_ctx();
  if (!c) return CMPC_ERR_ARG;
  c->model = *model;
  if (settings) c->settings = *settings;
  else cmpc_settings_default(&c->settings);
  c->precision = precision;
  c->max_batch = max_batch;
  c->ld = ld_for(*model);
  // default kernel path (cmpc_set_path): the fused n <= 64 kernel whenever it can serve the horizon; the fused 128
  // class for fp32 only (config 3: 2.267 -> 2.243 ms; fp64 measured slower fused: config 5 class stage 1.615 ->
  // 1.657 ms, all-stance 4.19 -> 4.29 ms); results scattered by the IPM kernels
  c->fused = model->N <= CMPC_C64_MAXN;
  c->fused128 = precision == CMPC_F32;
  c->direct = true;
  (void)hipGetDevice(&c->device);
  const Layout L = layout(c->ld, precision, max_batch, c->model.N);
  c->ws_bytes = L.total;
  if (dev_mem) {
    c->ws = (char*)dev_mem;
    c->own_ws = false;
  } else {
    if (hipMalloc((void**)&c->ws, L.total) != hipSuccess) {
      delete c;
      return CMPC_ERR_HIP;
    }
    c->own_ws = true;
  }
  c->H = c->ws + L.H;
  c->g = c->ws + L.g;
  c->tri_mu = c->ws + L.mu;
  c->tri_lo = c->ws + L.lo;
  c->tri_hi = c->ws + L.hi;
  c->u = c->ws + L.u;
  c->tri_map = (int*)(c->ws + L.map);
  c->nvar = (int*)(c->ws + L.nvar);
  c->status = (int*)(c->ws + L.status);
  c->iters = (int*)(c->ws + L.iters);
  c->lin = (double*)(c->ws + L.lin);
  c->dj = (double*)(c->ws + L.dj);
  c->dq = (double*)(c->ws + L.dq);
  c->uj = (double*)(c->ws + L.uj);
  c->uq = (double*)(c->ws + L.uq);
  c->stq = (int*)(c->ws + L.stq);
  c->itq = (int*)(c->ws + L.itq);
  c->done = (int*)(c->ws + L.done);
  c->sqpi = (int*)(c->ws + L.sqpi);
  c->qpi = (int*)(c->ws + L.qpi);
  c->cnt = (int*)(c->ws + L.cnt);
  c->res_scr = c->ws + L.res_scr;
  c->res = (double*)(c->ws + L.res);
  c->qlist = (int*)(c->ws + L.qlist);
  c->qcount = (int*)(c->ws + L.qcount);
  if (hipMemset(c->qcount, 0, 10 * sizeof(int)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    if (c->own_ws) (void)hipFree(c->ws);
    delete c;
    return CMPC_ERR_HIP;
  }
  if (hipMalloc((void**)&c->d_model, sizeof(DevModel)) != hipSuccess) {
    if (c->own_ws) (void)hipFree(c->ws);
    delete c;
    return CMPC_ERR_HIP;
  }
  const int r = cmpc_set_model(c, model);
  if (r != CMPC_OK) {
    cmpc_destroy(c);
    return r;
  }
  *out = c;
  return CMPC_OK;
}

int cmpc_destroy(cmpc_ctx* c) {
  if (!c) return CMPC_ERR_ARG;
  if (c->own_ws && c->ws) (void)hipFree(c->ws);
  if (c->d_model) (void)hipFree(c->d_model);
  if (c->stats) (void)hipFree(c->stats);
  if (c->stage) (void)hipFree(c->stage);
  if (c->pol) (void)hipFree(c->pol);
  for (hipEvent_t e : c->prof_ev) (void)hipEventDestroy(e);
  delete c;
  return CMPC_OK;
}

int cmpc_set_settings(cmpc_ctx* c, const cmpc_settings* s) {
  if (!c || !s || !settings_ok(*s)) return CMPC_ERR_ARG;
  c->settings = *s;
  return CMPC_OK;
}

int cmpc_set_model(cmpc_ctx* c, const cmpc_model* m) {
  if (!c || !model_ok(m) || m->N != c->model.N) return CMPC_ERR_ARG;
  c->model = *m;
  DevModel d;
  derive_model(*m, d);
  HIP_OK(hipMemcpy(c->d_model, &d, sizeof(d), hipMemcpyHostToDevice));
  return CMPC_OK;
}

int cmpc_get_model(const cmpc_ctx* c, cmpc_model* out) {
  if (!c || !out) return CMPC_ERR_ARG;
  *out = c->model;
  return CMPC_OK;
}

int cmpc_ctx_ld(const cmpc_ctx* c) { return c ? c->ld : 0; }
int cmpc_ctx_fused(const cmpc_ctx* c) { return c && c->fused ? 1 : 0; }

static int set_ric_path(cmpc_ctx* c, int value);
int cmpc_set_path(cmpc_ctx* c, int option, int value) {
  if (c && option == CMPC_PATH_RICCATI) return set_ric_path(c, value);
  if (!c || (value != 0 && value != 1)) return CMPC_ERR_ARG;
  switch (option) {
    case CMPC_PATH_FUSED64:
      if (value && c->model.N > CMPC_C64_MAXN) return CMPC_ERR_ARG;  // the one-wave condensing holds N <= 21
      if (!value && c->ric == 1) return CMPC_ERR_ARG;  // RICCATI = 1 runs on the fused path: set RICCATI first
      c->fused = value != 0;
      return CMPC_OK;
    case CMPC_PATH_FUSED128:
      c->fused128 = value != 0;
      return CMPC_OK;
    case CMPC_PATH_DIRECT:
      c->direct = value != 0;
      return CMPC_OK;
    case CMPC_PATH_IPM72:
      c->ipm72 = value != 0;
      return CMPC_OK;
    default:
      return CMPC_ERR_ARG;
  }
}

// CMPC_PATH_RICCATI takes 0 / 1 / 2 (cmpc.h)
static int set_ric_path(cmpc_ctx* c, int value) {
  if (value < 0 || value > 2) return CMPC_ERR_ARG;
  if (value > 0) {
    if (c->model.N > CMPC_RIC_MAXN) return CMPC_ERR_ARG;
    if (value == 1 && !c->fused) return CMPC_ERR_ARG;
  }
  c->ric = value;
  return CMPC_OK;
}

int cmpc_get_path(const cmpc_ctx* c, int option) {
  if (!c) return CMPC_ERR_ARG;
  switch (option) {
    case CMPC_PATH_FUSED64: return c->fused ? 1 : 0;
    case CMPC_PATH_FUSED128: return c->fused128 ? 1 : 0;
    case CMPC_PATH_DIRECT: return c->direct ? 1 : 0;
    case CMPC_PATH_RICCATI: return c->ric;
    case CMPC_PATH_IPM72: return c->ipm72 ? 1 : 0;
    default: return CMPC_ERR_ARG;
  }
}

int cmpc_enable_stats(cmpc_ctx* c, int rows) {
  if (!c || rows < 0 || rows > 4096) return CMPC_ERR_ARG;
  if (c->stats) (void)hipFree(c->stats);
  c->stats = nullptr;
  c->stats_rows = 0;
  if (rows == 0) return CMPC_OK;
  if (hipMalloc((void**)&c->stats, (size_t)c->max_batch * rows * CMPC_STAT_COLS * sizeof(double)) != hipSuccess) {
    c->stats = nullptr;
    return CMPC_ERR_HIP;
  }
  c->stats_rows = rows;
  return CMPC_OK;
}

int cmpc_get_stats(cmpc_ctx* c, int B, double* d_stats, void* stream) {
  if (!c || B < 0 || B > c->max_batch || !c->stats || (B > 0 && !d_stats)) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  HIP_OK(hipMemcpyAsync(d_stats, c->stats, (size_t)B * c->stats_rows * CMPC_STAT_COLS * sizeof(double),
                        hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return CMPC_OK;
}

int cmpc_get_residuals(cmpc_ctx* c, int B, double* d_res, void* stream) {
  if (!c || B < 0 || B > c->max_batch || (B > 0 && !d_res)) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  return launch_residuals(c->res, c->status, B, d_res, (hipStream_t)stream) == 0 ? CMPC_OK : CMPC_ERR_HIP;
}

int cmpc_solve_batch(cmpc_ctx* c, int B, const double* x0, const double* xref, const double* foot,
                     const uint8_t* contact, double* u, double* x, int* status, int* iters, void* stream) {
  return cmpc_solve_batch_warm(c, B, x0, xref, foot, contact, nullptr, u, x, status, iters, stream);
}

int cmpc_solve_batch_warm(cmpc_ctx* c, int B, const double* x0, const double* xref, const double* foot,
                          const uint8_t* contact, const double* u_init, double* u, double* x, int* status, int* iters,
                          void* stream) {
  if (!c || B < 0 || B > c->max_batch || !x0 || !xref || !foot || !contact || !u || !status) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  hipStream_t st = (hipStream_t)stream;
  hipEvent_t* ev = nullptr;
  if (c->profiling && c->prof_calls < c->prof_max) ev = &c->prof_ev[(size_t)4 * c->prof_calls++];
  if (ev) HIP_OK(hipEventRecord(ev[0], st));
  const int warm = (u_init && c->settings.warm_start != 0) ? 1 : 0;
  // fused path without rollout: the IPM kernels write u / status / iters themselves (no k_expand)
  const bool direct = c->direct && !warm && (c->fused || c->ric == 2) && x == nullptr && c->model.N * 12 <= 256;
  if (!warm && c->ric == 2) {
    double* du = direct ? u : nullptr;
    int* ds = direct ? status : nullptr;
    int* di = direct ? iters : nullptr;
    const int rr = c->precision == CMPC_F64 ? run_ric_all_t<double>(c, B, x0, xref, foot, contact, st, du, ds, di)
                                            : run_ric_all_t<float>(c, B, x0, xref, foot, contact, st, du, ds, di);
    if (rr != 0) return CMPC_ERR_HIP;
    if (ev) HIP_OK(hipEventRecord(ev[1], st));
  } else if (!warm && c->fused) {
    double* du = direct ? u : nullptr;
    int* ds = direct ? status : nullptr;
    int* di = direct ? iters : nullptr;
    const int rf = c->precision == CMPC_F64
                       ? run_fused_t<double>(c, B, x0, xref, foot, contact, st, ev ? ev[1] : nullptr, du, ds, di)
                       : run_fused_t<float>(c, B, x0, xref, foot, contact, st, ev ? ev[1] : nullptr, du, ds, di);
    if (rf != 0) return CMPC_ERR_HIP;
  } else {
    bool lists = false;
    int r = run_condense(c, B, x0, xref, foot, contact, st, nullptr, &lists);
    if (r != CMPC_OK) return r;
    if (warm && launch_pack_warm(u_init, c->tri_map, c->nvar, c->status, c->precision, c->ld, c->model.N, c->u, B,
                                 st) != 0)
      return CMPC_ERR_HIP;
    if (ev) HIP_OK(hipEventRecord(ev[1], st));
    r = run_ipm(c, B, st, warm, lists);
    if (r != CMPC_OK) return r;
  }
  if (ev) HIP_OK(hipEventRecord(ev[2], st));
  if (direct) {
    if (ev) HIP_OK(hipEventRecord(ev[3], st));
    return CMPC_OK;
  }
  ExpandArgs e;
  e.model = c->d_model;
  e.ld = c->ld;
  e.x0 = x0;
  e.xref = xref;
  e.foot = foot;
  e.contact = contact;
  e.tri_map = c->tri_map;
  e.nvar = c->nvar;
  e.status = c->status;
  e.u_ws = c->u;
  e.precision = c->precision;
  e.u = u;
  e.x = x;
  e.status_out = status;
  e.iters_ws = c->iters;
  e.iters_out = iters;
  e.dq = nullptr;
  if (launch_expand(e, B, st) != 0) return CMPC_ERR_HIP;
  if (ev) HIP_OK(hipEventRecord(ev[3], st));
  return CMPC_OK;
}

}  // extern "C"

namespace {

// Shared SQP driver of cmpc_sqp_solve_batch (feet false) and cmpc_nlp_solve_batch (feet true: the later runs'
// footholds are decision variables, dj/dq carry them, feet_out the foot_pos table).
int sqp_run(cmpc_ctx* c, int B, const double* x0, const double* xref, const double* foot, const uint8_t* contact,
            int sqp_iter_max, double sqp_tol, double* u, double* x, int* status, int* qp_iters, int* sqp_iters,
            void* stream, bool feet, double* feet_out) {
  if (!c || B < 0 || B > c->max_batch || !x0 || !xref || !foot || !contact || !u || !status || sqp_iter_max < 0 ||
      !(sqp_tol >= 0.0))
    return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  hipStream_t st = (hipStream_t)stream;
  // U_0: the QP at the reference linearisation, cold (oracle_sqp_solve)
  int r = cmpc_solve_batch_warm(c, B, x0, xref, foot, contact, nullptr, u, nullptr, status, c->qpi, stream);
  if (r != CMPC_OK) return r;
  SqpArgs a;
  a.model = c->d_model;
  a.N = c->model.N;
  a.x0 = x0;
  a.xref = xref;
  a.foot = foot;
  a.contact = contact;
  a.u = u;
  a.x = x;
  a.status = status;
  a.iters = c->qpi;
  a.uj = c->uj;
  a.uq = c->uq;
  a.status_q = c->stq;
  a.iters_q = c->itq;
  a.lin = c->lin;
  a.done = c->done;
  a.qp_iters = c->qpi;  // the cold iterations (written there by the solve above) accumulate in place
  a.sqp_iters = c->sqpi;
  a.count = c->cnt;
  a.tol = sqp_tol;
  a.dj = feet ? c->dj : nullptr;
  a.dq = feet ? c->dq : nullptr;
  a.feet = feet ? feet_out : nullptr;
  if (launch_sqp(0, a, B, st) != 0) return CMPC_ERR_HIP;
  for (int it = 0; it < sqp_iter_max; ++it) {
    bool lists = false;
    // QPs whose SQP has converged are not condensed or solved again (CondenseArgs::skip = done)
    r = run_condense(c, B, x0, xref, foot, contact, st, c->lin, &lists, feet ? c->uj : nullptr,
                     feet ? c->dj : nullptr, c->done);
    if (r != CMPC_OK) return r;
    if (launch_pack_warm(c->uj, c->tri_map, c->nvar, c->status, c->precision, c->ld, c->model.N, c->u, B, st,
                         feet ? c->dj : nullptr) != 0)
      return CMPC_ERR_HIP;
    r = run_ipm(c, B, st, 1, lists);
    if (r != CMPC_OK) return r;
    ExpandArgs e;
    e.model = c->d_model;
    e.ld = c->ld;
    e.x0 = x0;
    e.xref = xref;
    e.foot = foot;
    e.contact = contact;
    e.tri_map = c->tri_map;
    e.nvar = c->nvar;
    e.status = c->status;
    e.u_ws = c->u;
    e.precision = c->precision;
    e.u = c->uq;
    e.x = nullptr;
    e.status_out = c->stq;
    e.iters_ws = c->iters;
    e.iters_out = c->itq;
    e.dq = feet ? c->dq : nullptr;
    if (launch_expand(e, B, st) != 0) return CMPC_ERR_HIP;
    if (launch_sqp(1, a, B, st) != 0) return CMPC_ERR_HIP;
    // early exit once every QP has converged (one 4-byte read-back per SQP iteration)
    if (launch_sqp(3, a, B, st) != 0) return CMPC_ERR_HIP;
    int left = 0;
    HIP_OK(hipMemcpyAsync(&left, c->cnt, sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    if (left == 0) break;
  }
  if (launch_sqp(2, a, B, st) != 0) return CMPC_ERR_HIP;
  if (qp_iters) HIP_OK(hipMemcpyAsync(qp_iters, c->qpi, (size_t)B * sizeof(int), hipMemcpyDeviceToDevice, st));
  if (sqp_iters) HIP_OK(hipMemcpyAsync(sqp_iters, c->sqpi, (size_t)B * sizeof(int), hipMemcpyDeviceToDevice, st));
  return CMPC_OK;
}

}  // namespace

extern "C" {

int cmpc_sqp_solve_batch(cmpc_ctx* c, int B, const double* x0, const double* xref, const double* foot,
                         const uint8_t* contact, int sqp_iter_max, double sqp_tol, double* u, double* x, int* status,
                         int* qp_iters, int* sqp_iters, void* stream) {
  return sqp_run(c, B, x0, xref, foot, contact, sqp_iter_max, sqp_tol, u, x, status, qp_iters, sqp_iters, stream,
                 false, nullptr);
}

int cmpc_nlp_solve_batch(cmpc_ctx* c, int B, const double* x0, const double* xref, const double* foot,
                         const uint8_t* contact, int sqp_iter_max, double sqp_tol, double* u, double* feet,
                         double* x, int* status, int* qp_iters, int* sqp_iters, void* stream) {
  if (!feet) return CMPC_ERR_ARG;
  return sqp_run(c, B, x0, xref, foot, contact, sqp_iter_max, sqp_tol, u, x, status, qp_iters, sqp_iters, stream,
                 true, feet);
}

}  // extern "C"

namespace {

// Feedback policy of the QPs linearised at lin ([B][N][6] in the context workspace, or null: the reference
// linearisation) at their solutions u.
int policy_run(cmpc_ctx* c, int B, const double* x0, const double* xref, const double* foot, const uint8_t* contact,
               const double* u, double act_tol, double* K, int* nfree, int* status, void* stream, const double* lin) {
  hipStream_t st = (hipStream_t)stream;
  int r = run_condense(c, B, x0, xref, foot, contact, st, lin);
  if (r != CMPC_OK) return r;
  // scratch for at most `chunk` QPs per launch; launches on one stream reuse it in order
  const size_t stride = policy_scratch_doubles(c->model.N, c->ld);
  const int chunk = B < 2048 ? B : 2048;
  const size_t bytes = stride * sizeof(double) * (size_t)chunk;
  if (c->pol_bytes < bytes) {
    HIP_OK(hipStreamSynchronize(st));
    if (c->pol) (void)hipFree(c->pol);
    c->pol = nullptr;
    c->pol_bytes = 0;
    HIP_OK(hipMalloc((void**)&c->pol, bytes));
    c->pol_bytes = bytes;
  }
  if (!(act_tol > 0.0)) act_tol = c->precision == CMPC_F64 ? 1e-5 : 2e-3;
  for (int q0 = 0; q0 < B; q0 += chunk) {
    const int nq = B - q0 < chunk ? B - q0 : chunk;
    int rr;
    if (c->precision == CMPC_F64) {
      PolicyArgs<double> a{c->d_model, c->ld, q0, xref, foot, contact, u, (const double*)c->H, c->tri_map, c->nvar,
                           c->status, act_tol, K, nfree, status, c->pol, stride, lin};
      rr = launch_policy<double>(a, nq, st);
    } else {
      PolicyArgs<float> a{c->d_model, c->ld, q0, xref, foot, contact, u, (const float*)c->H, c->tri_map, c->nvar,
                          c->status, act_tol, K, nfree, status, c->pol, stride, lin};
      rr = launch_policy<float>(a, nq, st);
    }
    if (rr != 0) return CMPC_ERR_HIP;
  }
  return CMPC_OK;
}

}  // namespace

extern "C" {

int cmpc_policy_batch(cmpc_ctx* c, int B, const double* x0, const double* xref, const double* foot,
                      const uint8_t* contact, const double* u, double act_tol, double* K, int* nfree, int* status,
                      void* stream) {
  if (!c || B < 0 || B > c->max_batch || !x0 || !xref || !foot || !contact || !u || !K || !status)
    return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  return policy_run(c, B, x0, xref, foot, contact, u, act_tol, K, nfree, status, stream, nullptr);
}

int cmpc_sqp_policy_batch(cmpc_ctx* c, int B, const double* x0, const double* xref, const double* foot,
                          const uint8_t* contact, const double* u, double act_tol, double* K, int* nfree, int* status,
                          void* stream) {
  if (!c || B < 0 || B > c->max_batch || !x0 || !xref || !foot || !contact || !u || !K || !status)
    return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  SqpArgs a{};
  a.model = c->d_model;
  a.N = c->model.N;
  a.x0 = x0;
  a.xref = xref;
  a.foot = foot;
  a.contact = contact;
  a.u = const_cast<double*>(u);  // read only by k_sqp_lin
  a.lin = c->lin;
  if (launch_sqp(4, a, B, (hipStream_t)stream) != 0) return CMPC_ERR_HIP;
  return policy_run(c, B, x0, xref, foot, contact, u, act_tol, K, nfree, status, stream, c->lin);
}

int cmpc_shift_inputs(int B, int N, const double* d_u, int shift, double* d_u_out, void* stream) {
  if (B < 0 || N < 1 || shift < 0 || !d_u || !d_u_out || d_u == d_u_out) return CMPC_ERR_ARG;
  return launch_shift_inputs(d_u, N, shift, d_u_out, B, (hipStream_t)stream) == 0 ? CMPC_OK : CMPC_ERR_HIP;
}

static_assert(sizeof(cmpc_ipc_handle) == sizeof(hipIpcMemHandle_t), "IPC handle size");

int cmpc_ipc_export(void* d_ptr, cmpc_ipc_handle* out) {
  if (!d_ptr || !out) return CMPC_ERR_ARG;
  hipIpcMemHandle_t h;
  HIP_OK(hipIpcGetMemHandle(&h, d_ptr));
  std::memcpy(out->bytes, &h, sizeof(h));
  return CMPC_OK;
}

int cmpc_ipc_open(const cmpc_ipc_handle* handle, void** d_ptr) {
  if (!handle || !d_ptr) return CMPC_ERR_ARG;
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle->bytes, sizeof(h));
  *d_ptr = nullptr;
  HIP_OK(hipIpcOpenMemHandle(d_ptr, h, hipIpcMemLazyEnablePeerAccess));
  return CMPC_OK;
}

int cmpc_ipc_close(void* d_ptr) {
  if (!d_ptr) return CMPC_ERR_ARG;
  HIP_OK(hipIpcCloseMemHandle(d_ptr));
  return CMPC_OK;
}

int cmpc_gather_shard(void* d_dst, size_t dst_offset_bytes, const void* d_src, size_t bytes, void* stream) {
  if (!d_dst || (!d_src && bytes > 0)) return CMPC_ERR_ARG;
  if (bytes == 0) return CMPC_OK;
  HIP_OK(hipMemcpyAsync((char*)d_dst + dst_offset_bytes, d_src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return CMPC_OK;
}

int cmpc_profile_begin(cmpc_ctx* c, int max_calls) {
  if (!c || max_calls <= 0) return CMPC_ERR_ARG;
  for (hipEvent_t e : c->prof_ev) (void)hipEventDestroy(e);
  c->prof_ev.assign((size_t)4 * max_calls, nullptr);
  for (auto& e : c->prof_ev) HIP_OK(hipEventCreate(&e));
  c->prof_max = max_calls;
  c->prof_calls = 0;
  c->profiling = true;
  return CMPC_OK;
}

int cmpc_profile_end(cmpc_ctx* c, double* ms_condense, double* ms_ipm, double* ms_expand, int* calls) {
  if (!c || !c->profiling) return CMPC_ERR_ARG;
  double acc[3] = {0, 0, 0};
  for (int k = 0; k < c->prof_calls; ++k) {
    hipEvent_t* ev = &c->prof_ev[(size_t)4 * k];
    HIP_OK(hipEventSynchronize(ev[3]));
    for (int j = 0; j < 3; ++j) {
      float ms = 0.f;
      HIP_OK(hipEventElapsedTime(&ms, ev[j], ev[j + 1]));
      acc[j] += ms;
    }
  }
  if (ms_condense) *ms_condense = acc[0];
  if (ms_ipm) *ms_ipm = acc[1];
  if (ms_expand) *ms_expand = acc[2];
  if (calls) *calls = c->prof_calls;
  c->profiling = false;
  return CMPC_OK;
}

int cmpc_solve_batch_host(cmpc_ctx* c, int B, const double* x0, const double* xref, const double* foot,
                          const uint8_t* contact, double* u, double* x, int* status, int* iters) {
  if (!c || B < 0 || B > c->max_batch || !x0 || !xref || !foot || !contact || !u || !status) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  const int N = c->model.N;
  const size_t n_x0 = (size_t)B * CMPC_NX, n_xr = (size_t)B * (N + 1) * CMPC_NX,
               n_ft = (size_t)B * (N + 1) * CMPC_MAX_LEGS * 3, n_ct = (size_t)B * N * CMPC_MAX_LEGS,
               n_u = (size_t)B * N * CMPC_NU, n_xo = x ? n_xr : 0;
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t bytes = al(n_x0 * 8) + al(n_xr * 8) + al(n_ft * 8) + al(n_ct) + al(n_u * 8) + al(n_xo * 8) +
                       2 * al((size_t)B * sizeof(int));
  int r = ensure_stage(c, bytes);
  if (r != CMPC_OK) return r;
  char* p = c->stage;
  double* d_x0 = (double*)p; p += al(n_x0 * 8);
  double* d_xr = (double*)p; p += al(n_xr * 8);
  double* d_ft = (double*)p; p += al(n_ft * 8);
  uint8_t* d_ct = (uint8_t*)p; p += al(n_ct);
  double* d_u = (double*)p; p += al(n_u * 8);
  double* d_xo = x ? (double*)p : nullptr; p += al(n_xo * 8);
  int* d_st = (int*)p; p += al((size_t)B * sizeof(int));
  int* d_it = (int*)p;
  HIP_OK(hipMemcpy(d_x0, x0, n_x0 * 8, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_xr, xref, n_xr * 8, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_ft, foot, n_ft * 8, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_ct, contact, n_ct, hipMemcpyHostToDevice));
  r = cmpc_solve_batch(c, B, d_x0, d_xr, d_ft, d_ct, d_u, d_xo, d_st, d_it, nullptr);
  if (r != CMPC_OK) return r;
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpy(u, d_u, n_u * 8, hipMemcpyDeviceToHost));
  if (x) HIP_OK(hipMemcpy(x, d_xo, n_xo * 8, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(status, d_st, (size_t)B * sizeof(int), hipMemcpyDeviceToHost));
  if (iters) HIP_OK(hipMemcpy(iters, d_it, (size_t)B * sizeof(int), hipMemcpyDeviceToHost));
  return CMPC_OK;
}

int cmpc_condense_batch(cmpc_ctx* c, int B, const double* x0, const double* xref, const double* foot,
                        const uint8_t* contact, double* H, double* g, int* n, int* status, void* stream) {
  if (!c || B < 0 || B > c->max_batch || !H || !g || !n || !status) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  hipStream_t st = (hipStream_t)stream;
  int r = run_condense(c, B, x0, xref, foot, contact, st);
  if (r != CMPC_OK) return r;
  if (launch_unpack_qp(c->H, c->g, c->nvar, c->precision, c->ld, H, g, B, st) != 0) return CMPC_ERR_HIP;
  HIP_OK(hipMemcpyAsync(n, c->nvar, (size_t)B * sizeof(int), hipMemcpyDeviceToDevice, st));
  HIP_OK(hipMemcpyAsync(status, c->status, (size_t)B * sizeof(int), hipMemcpyDeviceToDevice, st));
  return CMPC_OK;
}

int cmpc_nlp_solve_batch_host(cmpc_ctx* c, int B, const double* x0, const double* xref, const double* foot,
                              const uint8_t* contact, int sqp_iter_max, double sqp_tol, double* u, double* feet,
                              double* x, int* status, int* qp_iters, int* sqp_iters) {
  if (!c || B < 0 || B > c->max_batch || !x0 || !xref || !foot || !contact || !u || !feet || !status)
    return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  const int N = c->model.N;
  const size_t n_x0 = (size_t)B * CMPC_NX, n_xr = (size_t)B * (N + 1) * CMPC_NX,
               n_ft = (size_t)B * (N + 1) * CMPC_MAX_LEGS * 3, n_ct = (size_t)B * N * CMPC_MAX_LEGS,
               n_u = (size_t)B * N * CMPC_NU, n_xo = x ? n_xr : 0;
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t bytes = al(n_x0 * 8) + al(n_xr * 8) + 2 * al(n_ft * 8) + al(n_ct) + al(n_u * 8) + al(n_xo * 8) +
                       3 * al((size_t)B * sizeof(int));
  int r = ensure_stage(c, bytes);
  if (r != CMPC_OK) return r;
  char* p = c->stage;
  double* d_x0 = (double*)p; p += al(n_x0 * 8);
  double* d_xr = (double*)p; p += al(n_xr * 8);
  double* d_ft = (double*)p; p += al(n_ft * 8);
  double* d_fo = (double*)p; p += al(n_ft * 8);
  uint8_t* d_ct = (uint8_t*)p; p += al(n_ct);
  double* d_u = (double*)p; p += al(n_u * 8);
  double* d_xo = x ? (double*)p : nullptr; p += al(n_xo * 8);
  int* d_st = (int*)p; p += al((size_t)B * sizeof(int));
  int* d_qi = (int*)p; p += al((size_t)B * sizeof(int));
  int* d_si = (int*)p;
  HIP_OK(hipMemcpy(d_x0, x0, n_x0 * 8, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_xr, xref, n_xr * 8, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_ft, foot, n_ft * 8, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(d_ct, contact, n_ct, hipMemcpyHostToDevice));
  r = cmpc_nlp_solve_batch(c, B, d_x0, d_xr, d_ft, d_ct, sqp_iter_max, sqp_tol, d_u, d_fo, d_xo, d_st, d_qi, d_si,
                           nullptr);
  if (r != CMPC_OK) return r;
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpy(u, d_u, n_u * 8, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(feet, d_fo, n_ft * 8, hipMemcpyDeviceToHost));
  if (x) HIP_OK(hipMemcpy(x, d_xo, n_xo * 8, hipMemcpyDeviceToHost));
  HIP_OK(hipMemcpy(status, d_st, (size_t)B * sizeof(int), hipMemcpyDeviceToHost));
  if (qp_iters) HIP_OK(hipMemcpy(qp_iters, d_qi, (size_t)B * sizeof(int), hipMemcpyDeviceToHost));
  if (sqp_iters) HIP_OK(hipMemcpy(sqp_iters, d_si, (size_t)B * sizeof(int), hipMemcpyDeviceToHost));
  return CMPC_OK;
}

int cmpc_condense_lin_batch(cmpc_ctx* c, int B, const double* x0, const double* xref, const double* foot,
                            const uint8_t* contact, const double* lin, const double* ubar, const double* dbar,
                            double* H, double* g, int* n, int* status, int* tri_map, double* tri_lo, double* tri_hi,
                            void* stream) {
  if (!c || B < 0 || B > c->max_batch || !H || !g || !n || !status || (dbar && (!ubar || !lin))) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  hipStream_t st = (hipStream_t)stream;
  int r = run_condense(c, B, x0, xref, foot, contact, st, lin, nullptr, ubar, dbar);
  if (r != CMPC_OK) return r;
  if (launch_unpack_qp(c->H, c->g, c->nvar, c->precision, c->ld, H, g, B, st) != 0) return CMPC_ERR_HIP;
  HIP_OK(hipMemcpyAsync(n, c->nvar, (size_t)B * sizeof(int), hipMemcpyDeviceToDevice, st));
  HIP_OK(hipMemcpyAsync(status, c->status, (size_t)B * sizeof(int), hipMemcpyDeviceToDevice, st));
  const size_t nt = (size_t)B * (c->ld / 3);
  if (tri_map) HIP_OK(hipMemcpyAsync(tri_map, c->tri_map, nt * sizeof(int), hipMemcpyDeviceToDevice, st));
  const void* src[2] = {c->tri_lo, c->tri_hi};
  double* dst[2] = {tri_lo, tri_hi};
  for (int k = 0; k < 2; ++k) {
    if (!dst[k]) continue;
    if (c->precision == CMPC_F64) {
      HIP_OK(hipMemcpyAsync(dst[k], src[k], nt * 5 * 8, hipMemcpyDeviceToDevice, st));
    } else if (launch_convert_f32_to_f64((const float*)src[k], dst[k], nt * 5, st) != 0) {
      return CMPC_ERR_HIP;
    }
  }
  return CMPC_OK;
}

int cmpc_qp_solve_batch(cmpc_ctx* c, int B, const double* H, const double* g, const int* n, const double* tri_mu,
                        const double* tri_lo, const double* tri_hi, double* u, int* status, int* iters,
                        void* stream) {
  if (!c || B < 0 || B > c->max_batch || !H || !g || !n || !tri_mu || !tri_lo || !tri_hi || !u || !status)
    return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  hipStream_t st = (hipStream_t)stream;
  if (launch_pack_qp(H, g, tri_mu, tri_lo, tri_hi, n, c->precision, c->ld, c->H, c->g, c->tri_mu, c->tri_lo,
                     c->tri_hi, c->nvar, c->status, B, st) != 0)
    return CMPC_ERR_HIP;
  int r = run_ipm(c, B, st, 0, false);
  if (r != CMPC_OK) return r;
  const size_t nu = (size_t)B * c->ld;
  if (c->precision == CMPC_F64) {
    HIP_OK(hipMemcpyAsync(u, c->u, nu * 8, hipMemcpyDeviceToDevice, st));
  } else if (launch_convert_f32_to_f64((const float*)c->u, u, nu, st) != 0) {
    return CMPC_ERR_HIP;
  }
  HIP_OK(hipMemcpyAsync(status, c->status, (size_t)B * sizeof(int), hipMemcpyDeviceToDevice, st));
  if (iters) HIP_OK(hipMemcpyAsync(iters, c->iters, (size_t)B * sizeof(int), hipMemcpyDeviceToDevice, st));
  return CMPC_OK;
}

int cmpc_generate_batch(const cmpc_model* m, uint64_t seed, int64_t qp_offset, int B, int gait, double* x0,
                        double* xref, double* foot, uint8_t* contact, void* stream) {
  if (!model_ok(m) || B < 0 || !x0 || !xref || !foot || !contact || (gait != 0 && gait != 1)) return CMPC_ERR_ARG;
  return launch_generate(*m, seed, qp_offset, B, gait, x0, xref, foot, contact, (hipStream_t)stream) == 0
             ? CMPC_OK
             : CMPC_ERR_HIP;
}

}  // extern "C"

extern "C" {

const char* cmpc_status_string(int s) {
  switch (s) {
    case CMPC_SUCCESS: return "SUCCESS";
    case CMPC_MAX_ITER: return "MAX_ITER";
    case CMPC_MIN_STEP: return "MIN_STEP";
    case CMPC_NAN_SOL: return "NAN_SOL";
    case CMPC_INCONS_EQ: return "INCONS_EQ";
    case CMPC_INVALID_CONTACT: return "INVALID_CONTACT";
    case CMPC_TOO_LARGE: return "TOO_LARGE";
    case CMPC_INFEASIBLE_STEP: return "INFEASIBLE_STEP";
    case CMPC_GRID_TIMEOUT: return "GRID_TIMEOUT";
    default: return "UNKNOWN";
  }
}

const char* cmpc_error_string(int e) {
  switch (e) {
    case CMPC_OK: return "ok";
    case CMPC_ERR_ARG: return "invalid argument";
    case CMPC_ERR_HIP: return "HIP runtime error";
    case CMPC_ERR_SIZE: return "size out of range";
    case CMPC_ERR_NO_DEVICE: return "no HIP device";
    default: return "unknown error";
  }
}

int cmpc_device_info(int* num_cu, int* clock_khz, char* arch, int arch_len) {
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  hipDeviceProp_t p;
  HIP_OK(hipGetDeviceProperties(&p, dev));
  if (num_cu) *num_cu = p.multiProcessorCount;
  if (clock_khz) *clock_khz = p.clockRate;
  if (arch && arch_len > 0) {
    std::snprintf(arch, (size_t)arch_len, "%s", p.gcnArchName);
  }
  return CMPC_OK;
}

// CMPC_SRC_HASH: sha256 prefix of every source, header and build file of libcmpc.so, written by the Makefile
// (build/src_hash.h), so a bench line or test log names the exact source it ran
const char* cmpc_version(void) { return "cheeta-mpc-amd 0.4.0 (gfx950) src " CMPC_SRC_HASH; }

}  // extern "C"
