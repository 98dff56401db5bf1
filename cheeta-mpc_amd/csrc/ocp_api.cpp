// ocp_api.cpp — C ABI of the HpipmInterface::solve path (cmpc.h "Generic OCP-QP"): the cmpc_ocp handle owns the
// problem dimensions, the settings and every device buffer, sized once at creation as HpipmInterface's
// initializeMemory reserves HPIPM's memory (reference HpipmInterface.cpp:92-129); solves launch k_ocp_ipm
// (k_ocp.hip) and allocate nothing.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "cmpc/cmpc.h"
#include "k_ocp.hpp"

using cmpc::OcpLayout;

struct cmpc_ocp {
  int N = 0, nx = 0, nU = 0, m = 0, max_batch = 0, stat_rows = 0;
  std::vector<int> nu, ng;
  cmpc_settings s{};
  OcpLayout L{};
  size_t rec_size = 0, crec_size = 0;
  void* d_dims = nullptr;  // layout arrays
  double* d_ws = nullptr;  // [max_batch][ws_stride]
  // staging of the host entry points and the per-problem outputs the device path keeps
  double *d_x0 = nullptr, *d_rec = nullptr, *d_crec = nullptr, *d_x = nullptr, *d_u = nullptr, *d_res = nullptr,
         *d_stats = nullptr;
  int *d_status = nullptr, *d_iters = nullptr, *d_rst = nullptr;
  double *d_P = nullptr, *d_p = nullptr, *d_K = nullptr, *d_k = nullptr, *d_Lr = nullptr;
  hipStream_t stream = nullptr;
  // the last solve (for cmpc_ocp_riccati)
  int last_B = 0;
  const double *last_rec = nullptr, *last_crec = nullptr;
  int* last_status = nullptr;
};

namespace {

bool dims_ok(int N, int nx, const int* nu, const int* nc, int& nzp, int& ngmax) {
  if (N <= 0 || N > cmpc::OCP_MAX_N || nx <= 0 || nx > cmpc::OCP_MAX_NX || !nu) return false;
  int numax = 0;
  ngmax = 0;
  for (int k = 0; k < N; ++k) {
    if (nu[k] < 0) return false;
    numax = nu[k] > numax ? nu[k] : numax;
  }
  if (nc)
    for (int k = 0; k <= N; ++k) {
      if (nc[k] < 0 || nc[k] > cmpc::OCP_MAX_NG) return false;
      ngmax = nc[k] > ngmax ? nc[k] : ngmax;
    }
  const int need = std::max(numax + nx + 1, nx + 1 + ngmax);
  if (need > 128) return false;
  nzp = need <= 64 ? 64 : 128;
  return true;
}

bool settings_ok(const cmpc_settings* s) {
  return s && s->iter_max >= 0 && s->iter_max <= 1000 && s->alpha_min > 0 && s->mu0 > 0 && s->tol_stat > 0 &&
         s->tol_eq > 0 && s->tol_ineq > 0 && s->tol_comp > 0 && s->reg_prim >= 0 && s->pred_corr == 1 &&
         (s->ric_alg == 0 || s->ric_alg == 1) && s->hpipm_mode >= 0 && s->hpipm_mode <= 3;
}

// host image of the layout arrays; also fills the scalar fields of L (workspace map)
struct Dims {
  std::vector<int> nu, ng, cu, cr, cK, cM, ustage, rstage;
  std::vector<long long> orec, ocon;
};

Dims build_dims(int N, int nx, const int* nu, const int* nc, OcpLayout& L, size_t& rec_size, size_t& crec_size) {
  Dims d;
  const int NP = N + 1;
  d.nu.assign(nu, nu + N);
  d.nu.push_back(0);
  d.ng.assign((size_t)NP, 0);
  if (nc)
    for (int k = 0; k <= N; ++k) d.ng[(size_t)k] = nc[k];
  d.cu.assign((size_t)NP + 1, 0);
  d.cr.assign((size_t)NP + 1, 0);
  d.cK.assign((size_t)NP, 0);
  d.cM.assign((size_t)NP, 0);
  int nK = 0, nM = 0;
  for (int k = 0; k <= N; ++k) {
    d.cu[(size_t)k + 1] = d.cu[(size_t)k] + d.nu[(size_t)k];
    d.cr[(size_t)k + 1] = d.cr[(size_t)k] + d.ng[(size_t)k];
    d.cK[(size_t)k] = nK;
    d.cM[(size_t)k] = nM;
    nK += d.nu[(size_t)k] * nx;
    nM += d.nu[(size_t)k] * d.nu[(size_t)k];
  }
  const int nU = d.cu[(size_t)NP], m = d.cr[(size_t)NP];
  for (int k = 0; k < N; ++k)
    for (int a = 0; a < d.nu[(size_t)k]; ++a) d.ustage.push_back(k);
  for (int k = 0; k <= N; ++k)
    for (int j = 0; j < d.ng[(size_t)k]; ++j) d.rstage.push_back(k);
  d.orec.assign(8 * (size_t)NP, 0);  // [N+1][8]: A, B, b (k < N), Q, S, R, q, r
  long long o = 0;
  for (int k = 0; k < N; ++k) {
    d.orec[8 * (size_t)k + 0] = o; o += (long long)nx * nx;
    d.orec[8 * (size_t)k + 1] = o; o += (long long)nx * d.nu[(size_t)k];
    d.orec[8 * (size_t)k + 2] = o; o += nx;
  }
  for (int k = 0; k <= N; ++k) {
    const long long mk = d.nu[(size_t)k];
    d.orec[8 * (size_t)k + 3] = o; o += (long long)nx * nx;
    d.orec[8 * (size_t)k + 4] = o; o += mk * nx;
    d.orec[8 * (size_t)k + 5] = o; o += mk * mk;
    d.orec[8 * (size_t)k + 6] = o; o += nx;
    d.orec[8 * (size_t)k + 7] = o; o += mk;
  }
  rec_size = (size_t)o;
  d.ocon.assign(4 * (size_t)NP, 0);  // [N+1][4]: C, D, e, (pad)
  long long oc = 0;
  for (int k = 0; k <= N; ++k) {
    const long long g = d.ng[(size_t)k], mk = d.nu[(size_t)k];
    d.ocon[4 * (size_t)k + 0] = oc; oc += g * nx;
    d.ocon[4 * (size_t)k + 1] = oc; oc += g * mk;
    d.ocon[4 * (size_t)k + 2] = oc; oc += g;
  }
  crec_size = (size_t)oc;
  L.N = N;
  L.nx = nx;
  L.nU = nU;
  L.m = m;
  L.nK = nK;
  L.nM = nM;
  L.rec_size = (long long)rec_size;
  L.crec_size = (long long)crec_size;
  // workspace map (doubles per problem)
  const long long nX = (long long)NP * nx, nP = (long long)N * nx, nxx = (long long)nx * nx;
  long long w = 0;
  auto take = [&w](long long n) {
    const long long at = w;
    w += (n + 1) & ~1LL;  // keep every array 16-byte aligned
    return at;
  };
  L.o_x = take(nX);
  L.o_u = take(nU);
  L.o_pi = take(nP);
  L.o_rgu = take(nU);
  L.o_rgx = take(nX);
  L.o_rb = take(nP);
  L.o_gu = take(nU);
  L.o_gx = take(nX);
  L.o_du = take(nU);
  L.o_dx = take(nX);
  L.o_dpi = take(nP);
  L.o_rows = take((long long)cmpc::OCP_ROWS * m);
  L.o_P = take(NP * nxx);
  L.o_pv = take(nX);
  L.o_K = take(nK);
  L.o_kf = take(nU);
  L.o_Lf = take(nM);
  L.o_Acl = take((long long)N * nxx);
  L.o_h = take(nX);
  L.o_y = take(nP);
  L.o_bcl = take(nP);
  L.ws_stride = w;
  return d;
}

template <class T>
size_t vbytes(const std::vector<T>& v) {
  return sizeof(T) * v.size();
}

void free_all(cmpc_ocp* o) {
  for (void* p : {(void*)o->d_dims, (void*)o->d_ws, (void*)o->d_x0, (void*)o->d_rec, (void*)o->d_crec, (void*)o->d_x,
                  (void*)o->d_u, (void*)o->d_res, (void*)o->d_stats, (void*)o->d_status, (void*)o->d_iters,
                  (void*)o->d_rst, (void*)o->d_P, (void*)o->d_p, (void*)o->d_K, (void*)o->d_k, (void*)o->d_Lr})
    if (p) (void)hipFree(p);
  if (o->stream) (void)hipStreamDestroy(o->stream);
}

size_t per_problem_doubles(const cmpc_ocp* o) {
  const size_t NP = (size_t)o->N + 1, nx = (size_t)o->nx;
  return (size_t)o->L.ws_stride + nx + o->rec_size + o->crec_size + NP * nx + (size_t)std::max(o->nU, 1) + 4 +
         (size_t)o->stat_rows * CMPC_STAT_COLS + NP * nx * nx + NP * nx + (size_t)std::max(o->L.nK, 1) +
         (size_t)std::max(o->nU, 1) + (size_t)std::max(o->L.nM, 1) + 3;
}

int alloc_stats(cmpc_ocp* o) {
  if (o->d_stats) (void)hipFree(o->d_stats);
  o->d_stats = nullptr;
  o->stat_rows = o->s.iter_max + 1;
  return hipMalloc((void**)&o->d_stats, sizeof(double) * (size_t)o->max_batch * o->stat_rows * CMPC_STAT_COLS) ==
                 hipSuccess
             ? CMPC_OK
             : CMPC_ERR_HIP;
}

cmpc::OcpSolveArgs solve_args(cmpc_ocp* o, const double* x0, const double* rec, const double* crec, double* x,
                              double* u, int* status, int* iters) {
  cmpc::OcpSolveArgs a;
  a.par_res = 0;  // launch_ocp_ipm chooses by batch size
  a.L = o->L;
  a.x0 = x0;
  a.rec = rec;
  a.crec = o->m > 0 ? crec : nullptr;
  a.ws = o->d_ws;
  a.x = x;
  a.u = u;
  a.status = status;
  a.iters = iters;
  a.res = o->d_res;
  a.stats = o->d_stats;
  a.stat_rows = o->stat_rows;
  a.iter_max = o->s.iter_max;
  a.warm = (o->s.warm_start != 0 && x && u) ? 1 : 0;
  a.alpha_min = o->s.alpha_min;
  a.mu0 = o->s.mu0;
  a.tol_stat = o->s.tol_stat;
  a.tol_eq = o->s.tol_eq;
  a.tol_ineq = o->s.tol_ineq;
  a.tol_comp = o->s.tol_comp;
  a.reg = o->s.reg_prim;
  return a;
}

}  // namespace

extern "C" {

size_t cmpc_ocp_record_size(int N, int nx, const int* nu) {
  if (N <= 0 || nx <= 0 || !nu) return 0;
  size_t o = 0;
  for (int k = 0; k < N; ++k) o += (size_t)nx * nx + (size_t)nx * nu[k] + nx;
  for (int k = 0; k <= N; ++k) {
    const size_t m = k < N ? (size_t)nu[k] : 0;
    o += (size_t)nx * nx + m * nx + m * m + nx + m;
  }
  return o;
}

size_t cmpc_ocp_constraint_record_size(int N, int nx, const int* nu, const int* nc) {
  if (N <= 0 || nx <= 0 || !nu || !nc) return 0;
  size_t o = 0;
  for (int k = 0; k <= N; ++k) {
    const size_t m = k < N ? (size_t)nu[k] : 0;
    o += (size_t)nc[k] * (nx + m + 1);
  }
  return o;
}

size_t cmpc_ocp_memsize(int N, int nx, const int* nu, const int* nc, int max_batch) {
  int nzp = 0, ngmax = 0;
  if (!dims_ok(N, nx, nu, nc, nzp, ngmax) || max_batch <= 0) return 0;
  cmpc_ocp o;
  o.N = N;
  o.nx = nx;
  o.L.ngmax = ngmax;
  Dims d = build_dims(N, nx, nu, nc, o.L, o.rec_size, o.crec_size);
  o.nU = o.L.nU;
  o.stat_rows = 31;
  return sizeof(double) * per_problem_doubles(&o) * (size_t)max_batch + vbytes(d.nu) * 8 + vbytes(d.orec) +
         vbytes(d.ocon) + vbytes(d.ustage) + vbytes(d.rstage);
}

int cmpc_ocp_create(int N, int nx, const int* nu, const int* nc, const cmpc_settings* settings, int max_batch,
                    cmpc_ocp** out) {
  if (!out) return CMPC_ERR_ARG;
  *out = nullptr;
  int nzp = 0, ngmax = 0;
  if (!dims_ok(N, nx, nu, nc, nzp, ngmax) || max_batch <= 0) return CMPC_ERR_ARG;
  cmpc_settings s;
  cmpc_settings_default(&s);
  if (settings) s = *settings;
  if (!settings_ok(&s)) return CMPC_ERR_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return CMPC_ERR_NO_DEVICE;
  cmpc_ocp* o = new cmpc_ocp();
  o->N = N;
  o->nx = nx;
  o->max_batch = max_batch;
  o->s = s;
  o->L.nzp = nzp;
  o->L.ngmax = ngmax;
  Dims d = build_dims(N, nx, nu, nc, o->L, o->rec_size, o->crec_size);
  o->nu = d.nu;
  o->ng = d.ng;
  o->nU = o->L.nU;
  o->m = o->L.m;
  if (cmpc::ocp_lds_bytes(o->L) > 160 * 1024) {
    delete o;
    return CMPC_ERR_ARG;
  }
  // one device block for the layout arrays
  const size_t b_int = vbytes(d.nu) + vbytes(d.ng) + vbytes(d.cu) + vbytes(d.cr) + vbytes(d.cK) + vbytes(d.cM) +
                       vbytes(d.ustage) + vbytes(d.rstage) + 8 * sizeof(int);
  const size_t b_ll = vbytes(d.orec) + vbytes(d.ocon);
  int r = CMPC_OK;
  auto ck = [&r](hipError_t e) {
    if (e != hipSuccess) r = CMPC_ERR_HIP;
  };
  ck(hipMalloc(&o->d_dims, b_ll + b_int + 64));
  if (r == CMPC_OK) {
    std::vector<unsigned char> img(b_ll + b_int + 64, 0);
    size_t off = 0;
    auto put = [&](const void* src, size_t n) {
      std::memcpy(img.data() + off, src, n);
      const size_t at = off;
      off += (n + 7) & ~(size_t)7;
      return (const void*)((unsigned char*)o->d_dims + at);
    };
    o->L.orec = (const long long*)put(d.orec.data(), vbytes(d.orec));
    o->L.ocon = (const long long*)put(d.ocon.data(), vbytes(d.ocon));
    o->L.nu = (const int*)put(d.nu.data(), vbytes(d.nu));
    o->L.ng = (const int*)put(d.ng.data(), vbytes(d.ng));
    o->L.cu = (const int*)put(d.cu.data(), vbytes(d.cu));
    o->L.cr = (const int*)put(d.cr.data(), vbytes(d.cr));
    o->L.cK = (const int*)put(d.cK.data(), vbytes(d.cK));
    o->L.cM = (const int*)put(d.cM.data(), vbytes(d.cM));
    o->L.ustage = (const int*)put(d.ustage.data(), vbytes(d.ustage));
    o->L.rstage = (const int*)put(d.rstage.data(), vbytes(d.rstage));
    ck(hipMemcpy(o->d_dims, img.data(), img.size(), hipMemcpyHostToDevice));
  }
  const size_t B = (size_t)max_batch, NP = (size_t)N + 1;
  ck(hipMalloc((void**)&o->d_ws, sizeof(double) * B * (size_t)o->L.ws_stride));
  ck(hipMalloc((void**)&o->d_x0, sizeof(double) * B * nx));
  ck(hipMalloc((void**)&o->d_rec, sizeof(double) * B * o->rec_size));
  if (o->crec_size) ck(hipMalloc((void**)&o->d_crec, sizeof(double) * B * o->crec_size));
  ck(hipMalloc((void**)&o->d_x, sizeof(double) * B * NP * nx));
  ck(hipMalloc((void**)&o->d_u, sizeof(double) * B * (size_t)std::max(o->nU, 1)));
  ck(hipMalloc((void**)&o->d_res, sizeof(double) * B * 4));
  ck(hipMalloc((void**)&o->d_status, sizeof(int) * B));
  ck(hipMalloc((void**)&o->d_iters, sizeof(int) * B));
  ck(hipMalloc((void**)&o->d_rst, sizeof(int) * B));
  ck(hipMalloc((void**)&o->d_P, sizeof(double) * B * NP * nx * nx));
  ck(hipMalloc((void**)&o->d_p, sizeof(double) * B * NP * nx));
  ck(hipMalloc((void**)&o->d_K, sizeof(double) * B * (size_t)std::max(o->L.nK, 1)));
  ck(hipMalloc((void**)&o->d_k, sizeof(double) * B * (size_t)std::max(o->nU, 1)));
  ck(hipMalloc((void**)&o->d_Lr, sizeof(double) * B * (size_t)std::max(o->L.nM, 1)));
  if (r == CMPC_OK) r = alloc_stats(o);
  if (r == CMPC_OK) ck(hipStreamCreateWithFlags(&o->stream, hipStreamNonBlocking));
  if (r != CMPC_OK) {
    free_all(o);
    delete o;
    return r;
  }
  *out = o;
  return CMPC_OK;
}

int cmpc_ocp_destroy(cmpc_ocp* o) {
  if (!o) return CMPC_ERR_ARG;
  if (o->stream) (void)hipStreamSynchronize(o->stream);
  free_all(o);
  delete o;
  return CMPC_OK;
}

int cmpc_ocp_set_settings(cmpc_ocp* o, const cmpc_settings* s) {
  if (!o || !settings_ok(s)) return CMPC_ERR_ARG;
  const bool grow = s->iter_max + 1 != o->stat_rows;
  o->s = *s;
  return grow ? alloc_stats(o) : CMPC_OK;
}

int cmpc_ocp_solve(cmpc_ocp* o, int B, const double* d_x0, const double* d_rec, const double* d_crec, double* d_x,
                   double* d_u, int* d_status, int* d_iters, void* stream) {
  if (!o || B < 0 || B > o->max_batch || !d_x0 || !d_rec || !d_x || !d_u || !d_status) return CMPC_ERR_ARG;
  if (o->m > 0 && !d_crec) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  const cmpc::OcpSolveArgs a = solve_args(o, d_x0, d_rec, d_crec, d_x, d_u, d_status, d_iters);
  if (cmpc::launch_ocp_ipm(a, B, (hipStream_t)stream) != 0) return CMPC_ERR_HIP;
  o->last_B = B;
  o->last_rec = d_rec;
  o->last_crec = d_crec;
  o->last_status = d_status;
  return CMPC_OK;
}

int cmpc_ocp_solve_host(cmpc_ocp* o, int B, const double* x0, const double* rec, const double* crec, double* x,
                        double* u, int* status, int* iters) {
  if (!o || B < 0 || B > o->max_batch || !x0 || !rec || !x || (!u && o->nU > 0) || !status) return CMPC_ERR_ARG;
  if (o->m > 0 && !crec) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  const size_t NP = (size_t)o->N + 1;
  hipStream_t st = o->stream;
  int r = CMPC_OK;
  auto ck = [&r](hipError_t e) {
    if (e != hipSuccess) r = CMPC_ERR_HIP;
  };
  ck(hipMemcpyAsync(o->d_x0, x0, sizeof(double) * B * o->nx, hipMemcpyHostToDevice, st));
  ck(hipMemcpyAsync(o->d_rec, rec, sizeof(double) * B * o->rec_size, hipMemcpyHostToDevice, st));
  if (o->m > 0) ck(hipMemcpyAsync(o->d_crec, crec, sizeof(double) * B * o->crec_size, hipMemcpyHostToDevice, st));
  if (o->s.warm_start) {  // x, u are in / out: the initial guess (HPIPM's primal warm start)
    ck(hipMemcpyAsync(o->d_x, x, sizeof(double) * B * NP * o->nx, hipMemcpyHostToDevice, st));
    if (o->nU > 0) ck(hipMemcpyAsync(o->d_u, u, sizeof(double) * B * o->nU, hipMemcpyHostToDevice, st));
  }
  if (r != CMPC_OK) return r;
  r = cmpc_ocp_solve(o, B, o->d_x0, o->d_rec, o->d_crec, o->d_x, o->d_u, o->d_status, o->d_iters, st);
  if (r != CMPC_OK) return r;
  ck(hipMemcpyAsync(x, o->d_x, sizeof(double) * B * NP * o->nx, hipMemcpyDeviceToHost, st));
  if (o->nU > 0) ck(hipMemcpyAsync(u, o->d_u, sizeof(double) * B * o->nU, hipMemcpyDeviceToHost, st));
  ck(hipMemcpyAsync(status, o->d_status, sizeof(int) * B, hipMemcpyDeviceToHost, st));
  if (iters) ck(hipMemcpyAsync(iters, o->d_iters, sizeof(int) * B, hipMemcpyDeviceToHost, st));
  ck(hipStreamSynchronize(st));
  return r;
}

int cmpc_ocp_riccati(cmpc_ocp* o, int B, double* d_P, double* d_p, double* d_K, double* d_k, double* d_Lr_out,
                     int* d_status, void* stream) {
  if (!o || B <= 0 || B > o->last_B || !d_P || !d_p || !d_status || (o->nU > 0 && (!d_K || !d_k)) ||
      !o->last_rec || !o->last_status)
    return CMPC_ERR_ARG;
  cmpc::OcpRicArgs a;
  a.S = solve_args(o, nullptr, o->last_rec, o->last_crec, nullptr, nullptr, o->last_status, nullptr);
  a.P = d_P;
  a.p = d_p;
  a.K = o->nU > 0 ? d_K : o->d_K;
  a.k = o->nU > 0 ? d_k : o->d_k;
  a.Lr = d_Lr_out ? d_Lr_out : o->d_Lr;
  a.rstatus = d_status;
  return cmpc::launch_ocp_ric(a, B, (hipStream_t)stream) == 0 ? CMPC_OK : CMPC_ERR_HIP;
}

int cmpc_ocp_riccati_host(cmpc_ocp* o, int B, double* P, double* p, double* K, double* k, double* Lr,
                          int* status) {
  if (!o || B <= 0 || B > o->last_B || !P || !p || !status || (o->nU > 0 && (!K || !k))) return CMPC_ERR_ARG;
  hipStream_t st = o->stream;
  int r = cmpc_ocp_riccati(o, B, o->d_P, o->d_p, o->d_K, o->d_k, o->d_Lr, o->d_rst, st);
  if (r != CMPC_OK) return r;
  const size_t NP = (size_t)o->N + 1, nx = (size_t)o->nx;
  auto ck = [&r](hipError_t e) {
    if (e != hipSuccess) r = CMPC_ERR_HIP;
  };
  ck(hipMemcpyAsync(P, o->d_P, sizeof(double) * B * NP * nx * nx, hipMemcpyDeviceToHost, st));
  ck(hipMemcpyAsync(p, o->d_p, sizeof(double) * B * NP * nx, hipMemcpyDeviceToHost, st));
  if (o->nU > 0) {
    ck(hipMemcpyAsync(K, o->d_K, sizeof(double) * B * o->L.nK, hipMemcpyDeviceToHost, st));
    ck(hipMemcpyAsync(k, o->d_k, sizeof(double) * B * o->nU, hipMemcpyDeviceToHost, st));
  }
  if (Lr && o->L.nM > 0) ck(hipMemcpyAsync(Lr, o->d_Lr, sizeof(double) * B * o->L.nM, hipMemcpyDeviceToHost, st));
  ck(hipMemcpyAsync(status, o->d_rst, sizeof(int) * B, hipMemcpyDeviceToHost, st));
  ck(hipStreamSynchronize(st));
  return r;
}

int cmpc_ocp_get_residuals(cmpc_ocp* o, int B, double* d_res, void* stream) {
  if (!o || B < 0 || B > o->max_batch || !d_res) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  return hipMemcpyAsync(d_res, o->d_res, sizeof(double) * B * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream) ==
                 hipSuccess
             ? CMPC_OK
             : CMPC_ERR_HIP;
}

int cmpc_ocp_stat_rows(const cmpc_ocp* o) { return o ? o->stat_rows : CMPC_ERR_ARG; }

int cmpc_ocp_get_stats(cmpc_ocp* o, int B, double* d_stats, void* stream) {
  if (!o || B < 0 || B > o->max_batch || !d_stats) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  return hipMemcpyAsync(d_stats, o->d_stats, sizeof(double) * B * o->stat_rows * CMPC_STAT_COLS,
                        hipMemcpyDeviceToDevice, (hipStream_t)stream) == hipSuccess
             ? CMPC_OK
             : CMPC_ERR_HIP;
}

int cmpc_ocp_get_residuals_host(cmpc_ocp* o, int B, double* res) {
  if (!o || B < 0 || B > o->max_batch || !res) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  if (hipMemcpyAsync(res, o->d_res, sizeof(double) * B * 4, hipMemcpyDeviceToHost, o->stream) != hipSuccess ||
      hipStreamSynchronize(o->stream) != hipSuccess)
    return CMPC_ERR_HIP;
  return CMPC_OK;
}

int cmpc_ocp_get_stats_host(cmpc_ocp* o, int B, double* stats) {
  if (!o || B < 0 || B > o->max_batch || !stats) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  if (hipMemcpyAsync(stats, o->d_stats, sizeof(double) * B * o->stat_rows * CMPC_STAT_COLS, hipMemcpyDeviceToHost,
                     o->stream) != hipSuccess ||
      hipStreamSynchronize(o->stream) != hipSuccess)
    return CMPC_ERR_HIP;
  return CMPC_OK;
}

// ---- one-shot host entry points of the 0.3 ABI ----

int cmpc_ocp_solve_batch_host(int B, int N, int nx, const int* nu, const double* x0, const double* rec, double* x,
                              double* u, int* status) {
  if (B < 0 || !nu || !x0 || !rec || !x || !u || !status) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  cmpc_ocp* o = nullptr;
  int r = cmpc_ocp_create(N, nx, nu, nullptr, nullptr, B, &o);
  if (r != CMPC_OK) return r;
  r = cmpc_ocp_solve_host(o, B, x0, rec, nullptr, x, u, status, nullptr);
  cmpc_ocp_destroy(o);
  return r;
}

int cmpc_ocp_solve_batch_eq_host(int B, int N, int nx, const int* nu, const int* nc, const double* x0,
                                 const double* rec, const double* crec, double* x, double* u, int* status) {
  if (B < 0 || !nu || !nc || !x0 || !rec || !x || !u || !status) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  int m = 0;
  for (int k = 0; k <= N && N > 0; ++k) m += nc[k] > 0 ? nc[k] : 0;
  if (m > 0 && !crec) return CMPC_ERR_ARG;
  cmpc_ocp* o = nullptr;
  int r = cmpc_ocp_create(N, nx, nu, nc, nullptr, B, &o);
  if (r != CMPC_OK) return r;
  r = cmpc_ocp_solve_host(o, B, x0, rec, crec, x, u, status, nullptr);
  cmpc_ocp_destroy(o);
  return r;
}

int cmpc_ocp_riccati_batch_host(int B, int N, int nx, const int* nu, const double* rec, double* Sm, double* sv,
                                double* K, double* kff, int* status) {
  if (B < 0 || !nu || !rec || !Sm || !sv || !status) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  cmpc_ocp* o = nullptr;
  int r = cmpc_ocp_create(N, nx, nu, nullptr, nullptr, B, &o);
  if (r != CMPC_OK) return r;
  if (o->nU > 0 && (!K || !kff)) {
    cmpc_ocp_destroy(o);
    return CMPC_ERR_ARG;
  }
  std::vector<double> x0((size_t)B * nx, 0.0), x((size_t)B * (N + 1) * nx), u((size_t)B * std::max(o->nU, 1));
  std::vector<int> st((size_t)B);
  r = cmpc_ocp_solve_host(o, B, x0.data(), rec, nullptr, x.data(), u.data(), st.data(), nullptr);
  if (r == CMPC_OK) r = cmpc_ocp_riccati_host(o, B, Sm, sv, K, kff, nullptr, status);
  if (r == CMPC_OK)
    for (int b = 0; b < B; ++b)
      if (st[(size_t)b] != CMPC_SUCCESS) status[b] = st[(size_t)b];  // e.g. an indefinite stage: MAX_ITER
  cmpc_ocp_destroy(o);
  return r;
}

}  // extern "C"
