// ocp_api.cpp — C ABI of the HpipmInterface::solve path (cmpc.h "Generic OCP-QP"): the cmpc_ocp handle owns the
// problem dimensions, the settings and every device buffer. As HpipmInterface's MemoryBlock::reserve grows HPIPM's
// memory only (reference HpipmInterface.cpp:46-67, :92-129), every buffer has a capacity that only grows: a new size
// (cmpc_ocp_reshape, the mirror's resize) re-lays out the dimensions and offsets with one small upload and allocates
// only where it exceeds the capacity (with headroom for the MPC's shifting event nodes). Solves launch k_ocp_ipm /
// k_ocp_grid (k_ocp.hip) and allocate nothing; the host entry point copies through pinned staging buffers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "cmpc/cmpc.h"
#include "k_ocp.hpp"

using cmpc::OcpLayout;

namespace {
struct DBuf {  // device buffer with a grow-only capacity (bytes)
  void* p = nullptr;
  size_t cap = 0;
};
}  // namespace

struct cmpc_ocp {
  int N = 0, nx = 0, nU = 0, m = 0, max_batch = 0, stat_rows = 0;
  std::vector<int> nu, ng;
  cmpc_settings s{};
  OcpLayout L{};
  size_t rec_size = 0, crec_size = 0;
  DBuf dims, ws, x0, rec, crec, x, u, res, stats, status, iters, rst, P, p, K, k, Lr, hp, bar, gpart, fbk, seg, linres;
  long long hp_stride = 0;
  int hp_batch = 0, chain = 1;  // chain: cmpc_ocp_set_path (1 = the latency form where it applies, 0 = never)
  int grid = 0;                 // cmpc_ocp_set_grid: workgroups per problem of the grid form (0 auto, 1 off)
  int keep_ric = 0;             // cmpc_ocp_set_keep_riccati: the grid-form solve leaves the exit Riccati quantities
  long long grid_timeout = 5000000;  // cmpc_ocp_set_grid_timeout: barrier wait bound, 100-MHz ticks (50 ms)
  int force_timeout = 0;        // cmpc_ocp_debug_force_grid_timeout
  int broken = 0;               // a failed (re-)layout left the buffers inconsistent: solves are refused
  int nseg = 0;                 // cmpc_ocp_set_segments: segments of the grid form's factorisation (0 auto)
  int linres_on = 0;            // cmpc_ocp_set_linres: the solves record the Newton systems' residuals
  long long seg_stride = 0;     // doubles per problem of the segment buffer
  void* pin = nullptr;          // pinned host staging of cmpc_ocp_solve_host / _riccati_host (small batches)
  size_t pin_cap = 0;
  int allocs = 0;               // device / pinned allocations made (cmpc_ocp_alloc_count)
  int timing = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev_done = nullptr, ev_t0 = nullptr, ev_t1 = nullptr;  // the last solve's end; timing events
  // the last solve (for cmpc_ocp_riccati)
  int last_B = 0, ric_B = 0;  // ric_B: problems whose exit Riccati quantities the last solve left in P .. Lr
  int ric_full = 0;            // 1: P, p, K, k, Lr all kept (rows); 0: P_k (k >= 1), K, Lr only (factor-only)
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
  std::vector<int> nu, ng, cu, cr, cK, cM, ustage, rstage, cHp;
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
  d.cHp.assign((size_t)NP, 0);
  int nK = 0, nM = 0, numax = 0;
  for (int k = 0; k < N; ++k) {  // the latency form's Hc images: 2 x 2 lower blocks of the (nu_k + nx + 1) matrix
    const int n1 = d.nu[(size_t)k] + nx + 1, nb = (n1 + 1) / 2;
    d.cHp[(size_t)k + 1] = d.cHp[(size_t)k] + 4 * (nb * (nb + 1) / 2);
    numax = std::max(numax, d.nu[(size_t)k]);
  }
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
  L.numax = numax;
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
  for (DBuf* b : {&o->dims, &o->ws, &o->x0, &o->rec, &o->crec, &o->x, &o->u, &o->res, &o->stats, &o->status,
                  &o->iters, &o->rst, &o->P, &o->p, &o->K, &o->k, &o->Lr, &o->hp, &o->bar, &o->gpart, &o->fbk, &o->seg,
                  &o->linres})
    if (b->p) (void)hipFree(b->p);
  if (o->pin) (void)hipHostFree(o->pin);
  if (o->ev_done) (void)hipEventDestroy(o->ev_done);
  if (o->ev_t0) (void)hipEventDestroy(o->ev_t0);
  if (o->ev_t1) (void)hipEventDestroy(o->ev_t1);
  if (o->stream) (void)hipStreamDestroy(o->stream);
}

// Grow-only capacity: a buffer is reallocated only when a size exceeds it; handles for small batches (the MPC tick)
// take 25 % headroom at the first allocation and 50 % at a growth, so the event nodes and per-stage input counts that
// shift from tick to tick stay inside it
int grow(cmpc_ocp* o, DBuf& b, size_t need) {
  if (need <= b.cap) return CMPC_OK;
  const bool small = o->max_batch <= cmpc::OCP_GRID_MAX_B;
  const size_t want = b.cap == 0 ? need + (small ? need / 4 : 0) : need + need / 2;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  if (hipMalloc(&b.p, want) != hipSuccess) return CMPC_ERR_HIP;
  b.cap = want;
  ++o->allocs;
  return CMPC_OK;
}

// pinned staging bytes of the host entry points for B problems (inputs, then outputs, then the Riccati outputs)
struct PinMap {
  size_t x0, rec, crec, x, u, st, it, P, p, K, k, Lr, rst, total;
};
PinMap pin_map(const cmpc_ocp* o, int B) {
  PinMap m;
  const size_t NP = (size_t)o->N + 1, nx = (size_t)o->nx, b = (size_t)B;
  auto al = [](size_t n) { return (n + 63) & ~(size_t)63; };
  size_t at = 0;
  m.x0 = at, at += al(sizeof(double) * b * nx);
  m.rec = at, at += al(sizeof(double) * b * o->rec_size);
  m.crec = at, at += al(sizeof(double) * b * std::max<size_t>(o->crec_size, 1));
  m.x = at, at += al(sizeof(double) * b * NP * nx);
  m.u = at, at += al(sizeof(double) * b * (size_t)std::max(o->nU, 1));
  m.st = at, at += al(sizeof(int) * b);
  m.it = at, at += al(sizeof(int) * b);
  m.P = at, at += al(sizeof(double) * b * NP * nx * nx);
  m.p = at, at += al(sizeof(double) * b * NP * nx);
  m.K = at, at += al(sizeof(double) * b * (size_t)std::max(o->L.nK, 1));
  m.k = at, at += al(sizeof(double) * b * (size_t)std::max(o->nU, 1));
  m.Lr = at, at += al(sizeof(double) * b * (size_t)std::max(o->L.nM, 1));
  m.rst = at, at += al(sizeof(int) * b);
  m.total = at;
  return m;
}

int grow_pin(cmpc_ocp* o, size_t need) {
  if (need <= o->pin_cap) return CMPC_OK;
  const size_t want = o->pin_cap == 0 ? need + need / 4 : need + need / 2;
  if (o->pin) (void)hipHostFree(o->pin);
  o->pin = nullptr;
  o->pin_cap = 0;
  if (hipHostMalloc(&o->pin, want, hipHostMallocDefault) != hipSuccess) return CMPC_ERR_HIP;
  o->pin_cap = want;
  ++o->allocs;
  return CMPC_OK;
}

int alloc_stats(cmpc_ocp* o) {
  o->stat_rows = o->s.iter_max + 1;
  int r = grow(o, o->stats, sizeof(double) * (size_t)o->max_batch * o->stat_rows * CMPC_STAT_COLS);
  if (r == CMPC_OK && o->linres_on) r = grow(o, o->linres, sizeof(double) * (size_t)o->max_batch * o->stat_rows * 4);
  return r;
}

// (Re-)lay out the handle for dimensions (N, nx, nu, nc): every device buffer grows to the new size if it exceeds its
// capacity (nothing else is allocated), then the layout arrays are uploaded into the dims block and the new layout is
// committed. A failed growth leaves the handle marked broken (grow frees before it allocates), so later solves are
// refused instead of reading freed memory; the next successful layout repairs it.
int layout(cmpc_ocp* o, int N, int nx, const int* nu, const int* nc) {
  int nzp = 0, ngmax = 0;
  if (!dims_ok(N, nx, nu, nc, nzp, ngmax)) return CMPC_ERR_ARG;
  OcpLayout L{};
  L.nzp = nzp;
  L.ngmax = ngmax;
  size_t rec_size = 0, crec_size = 0;
  Dims d = build_dims(N, nx, nu, nc, L, rec_size, crec_size);
  if (cmpc::ocp_lds_bytes(L) > 160 * 1024) return CMPC_ERR_ARG;
  // work of an earlier layout may still be in flight on the device (its buffers and dims block are about to change)
  if (o->ev_done && hipEventSynchronize(o->ev_done) != hipSuccess) return CMPC_ERR_HIP;
  const size_t b_int = vbytes(d.nu) + vbytes(d.ng) + vbytes(d.cu) + vbytes(d.cr) + vbytes(d.cK) + vbytes(d.cM) +
                       vbytes(d.ustage) + vbytes(d.rstage) + vbytes(d.cHp) + 10 * 8;
  const size_t b_ll = vbytes(d.orec) + vbytes(d.ocon);
  const size_t B = (size_t)o->max_batch, NP = (size_t)N + 1, D = sizeof(double);
  const int nU = L.nU;
  int r = CMPC_OK;
  auto ck = [&r](int e) {
    if (r == CMPC_OK) r = e;
  };
  o->broken = 1;  // until the layout below is committed
  ck(grow(o, o->dims, b_ll + b_int + 64));
  ck(grow(o, o->ws, D * B * (size_t)L.ws_stride));
  ck(grow(o, o->x0, D * B * nx));
  ck(grow(o, o->rec, D * B * rec_size));
  ck(grow(o, o->crec, D * B * std::max<size_t>(crec_size, 1)));
  ck(grow(o, o->x, D * B * NP * nx));
  ck(grow(o, o->u, D * B * (size_t)std::max(nU, 1)));
  ck(grow(o, o->res, D * B * 4));
  ck(grow(o, o->status, sizeof(int) * B));
  ck(grow(o, o->iters, sizeof(int) * B));
  ck(grow(o, o->rst, sizeof(int) * B));
  ck(grow(o, o->P, D * B * NP * nx * nx));
  ck(grow(o, o->p, D * B * NP * nx));
  ck(grow(o, o->K, D * B * (size_t)std::max(L.nK, 1)));
  ck(grow(o, o->k, D * B * (size_t)std::max(nU, 1)));
  ck(grow(o, o->Lr, D * B * (size_t)std::max(L.nM, 1)));
  // the latency form (small batches: one problem per CU, or G per problem) where the dimensions fit it
  long long hp_stride = 0, seg_stride = 0;
  int hp_batch = 0;
  const size_t lc = cmpc::ocp_chain_lds_bytes(L, L.numax);
  if (lc > 0 && lc <= 160 * 1024) {
    hp_batch = std::min(o->max_batch, cmpc::OCP_ONE_PER_CU_MAX);
    hp_stride = ((long long)d.cHp[(size_t)N] + 1) & ~1LL;
    ck(grow(o, o->hp, D * (size_t)hp_batch * (size_t)hp_stride));
    // the grid form's segment elements and boundary values (ocp_part.hpp), per problem of a grid-sized batch
    seg_stride = (long long)cmpc::OCP_GRID_MAX_G * (cmpc::seg_esz(nx) + cmpc::seg_bsz(nx));
    if (o->max_batch <= cmpc::OCP_GRID_MAX_B) ck(grow(o, o->seg, D * (size_t)o->max_batch * (size_t)seg_stride));
    if (!o->bar.p && r == CMPC_OK) {
      // the grid barriers' words and the fallback counter start at zero (every launch leaves the words zero); a handle
      // created outside the latency form's limits gets them at its first layout inside them
      ck(grow(o, o->bar, sizeof(unsigned) * 4 * (size_t)cmpc::OCP_GRID_MAX_B));
      ck(grow(o, o->gpart, D * 8 * (size_t)cmpc::OCP_GRID_MAX_WG));
      ck(grow(o, o->fbk, sizeof(unsigned) * 4));
      if (r == CMPC_OK && (hipMemset(o->bar.p, 0, o->bar.cap) != hipSuccess ||
                           hipMemset(o->fbk.p, 0, o->fbk.cap) != hipSuccess))
        r = CMPC_ERR_HIP;
    }
  }
  if (r != CMPC_OK) return r;
  std::vector<unsigned char> img(b_ll + b_int + 64, 0);
  size_t off = 0;
  auto put = [&](const void* src, size_t n) {
    std::memcpy(img.data() + off, src, n);
    const size_t at = off;
    off += (n + 7) & ~(size_t)7;
    return (const void*)((unsigned char*)o->dims.p + at);
  };
  L.orec = (const long long*)put(d.orec.data(), vbytes(d.orec));
  L.ocon = (const long long*)put(d.ocon.data(), vbytes(d.ocon));
  L.nu = (const int*)put(d.nu.data(), vbytes(d.nu));
  L.ng = (const int*)put(d.ng.data(), vbytes(d.ng));
  L.cu = (const int*)put(d.cu.data(), vbytes(d.cu));
  L.cr = (const int*)put(d.cr.data(), vbytes(d.cr));
  L.cK = (const int*)put(d.cK.data(), vbytes(d.cK));
  L.cM = (const int*)put(d.cM.data(), vbytes(d.cM));
  L.ustage = (const int*)put(d.ustage.data(), vbytes(d.ustage));
  L.rstage = (const int*)put(d.rstage.data(), vbytes(d.rstage));
  L.cHp = (const int*)put(d.cHp.data(), vbytes(d.cHp));
  if (hipMemcpy(o->dims.p, img.data(), off, hipMemcpyHostToDevice) != hipSuccess) return CMPC_ERR_HIP;
  o->N = N;
  o->nx = nx;
  o->L = L;
  o->nu = d.nu;
  o->ng = d.ng;
  o->nU = nU;
  o->m = L.m;
  o->rec_size = rec_size;
  o->crec_size = crec_size;
  o->hp_stride = hp_stride;
  o->hp_batch = hp_batch;
  o->seg_stride = seg_stride;
  o->last_B = 0;  // the Riccati quantities of a solve of another layout are gone
  o->ric_B = 0;
  o->last_rec = o->last_crec = nullptr;
  o->last_status = nullptr;
  o->broken = 0;
  return CMPC_OK;
}

bool has_chain(const cmpc_ocp* o) { return o->chain && o->hp_batch > 0 && o->hp.p; }

cmpc::OcpSolveArgs solve_args(cmpc_ocp* o, const double* x0, const double* rec, const double* crec, double* x,
                              double* u, int* status, int* iters) {
  cmpc::OcpSolveArgs a{};
  a.par_res = 0;  // launch_ocp_ipm chooses by batch size
  a.L = o->L;
  a.x0 = x0;
  a.rec = rec;
  a.crec = o->m > 0 ? crec : nullptr;
  a.ws = (double*)o->ws.p;
  a.x = x;
  a.u = u;
  a.status = status;
  a.iters = iters;
  a.res = (double*)o->res.p;
  a.stats = (double*)o->stats.p;
  a.linres = o->linres_on ? (double*)o->linres.p : nullptr;
  a.stat_rows = o->stat_rows;
  a.iter_max = o->s.iter_max;
  a.warm = (o->s.warm_start != 0 && x && u) ? 1 : 0;
  a.fast = has_chain(o) ? 1 : 0;  // launch_ocp_ipm applies it to batches up to hp_batch
  a.hp = (double*)o->hp.p;
  a.hp_stride = o->hp_stride;
  a.G = o->grid;  // 0 auto; 1 disables the grid form (ocp_grid_width returns 0 below 2)
  a.bar = o->grid == 1 ? nullptr : (unsigned*)o->bar.p;
  a.gpart = (double*)o->gpart.p;
  a.grid_timeout = o->force_timeout ? -1 : o->grid_timeout;
  a.seg = (o->seg.p && o->seg_stride > 0) ? (double*)o->seg.p : nullptr;
  a.seg_stride = o->seg_stride;
  a.nseg = o->nseg;
  a.fallbacks = (unsigned*)o->fbk.p;
  // the exit Riccati quantities of the grid form (cmpc_ocp_set_keep_riccati) into the handle's arrays
  a.ric = o->keep_ric;
  a.ricP = (double*)o->P.p;
  a.ricp = (double*)o->p.p;
  a.ricK = (double*)o->K.p;
  a.rick = (double*)o->k.p;
  a.ricLr = (double*)o->Lr.p;
  a.ricst = (int*)o->rst.p;
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
  OcpLayout L{};
  L.nzp = nzp;
  L.ngmax = ngmax;
  size_t rec_size = 0, crec_size = 0;
  Dims d = build_dims(N, nx, nu, nc, L, rec_size, crec_size);
  if (cmpc::ocp_lds_bytes(L) > 160 * 1024) return 0;  // cmpc_ocp_create refuses these dimensions
  const size_t NP = (size_t)N + 1, B = (size_t)max_batch;
  const size_t per = (size_t)L.ws_stride + nx + rec_size + crec_size + NP * nx + (size_t)std::max(L.nU, 1) + 4 +
                     31 * CMPC_STAT_COLS + NP * nx * nx + NP * nx + (size_t)std::max(L.nK, 1) +
                     (size_t)std::max(L.nU, 1) + (size_t)std::max(L.nM, 1) + 3;
  const size_t hp = cmpc::ocp_chain_lds_bytes(L, L.numax) > 0
                        ? sizeof(double) * (size_t)std::min(max_batch, cmpc::OCP_ONE_PER_CU_MAX) *
                              (size_t)(d.cHp[(size_t)N] + 1)
                        : 0;
  return sizeof(double) * per * B + vbytes(d.nu) * 9 + vbytes(d.orec) + vbytes(d.ocon) + vbytes(d.ustage) +
         vbytes(d.rstage) + hp;
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
  o->max_batch = max_batch;
  o->s = s;
  int r = CMPC_OK;
  if (hipStreamCreateWithFlags(&o->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&o->ev_done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreate(&o->ev_t0) != hipSuccess || hipEventCreate(&o->ev_t1) != hipSuccess)
    r = CMPC_ERR_HIP;
  if (r == CMPC_OK) r = layout(o, N, nx, nu, nc);
  if (r == CMPC_OK) r = alloc_stats(o);
  if (r == CMPC_OK && max_batch <= cmpc::OCP_GRID_MAX_B) r = grow_pin(o, pin_map(o, max_batch).total);
  if (r != CMPC_OK) {
    free_all(o);
    delete o;
    return r;
  }
  *out = o;
  return CMPC_OK;
}

int cmpc_ocp_reshape(cmpc_ocp* o, int N, int nx, const int* nu, const int* nc) {
  if (!o) return CMPC_ERR_ARG;
  const int r = layout(o, N, nx, nu, nc);
  if (r != CMPC_OK) return r;
  return o->max_batch <= cmpc::OCP_GRID_MAX_B ? grow_pin(o, pin_map(o, o->max_batch).total) : CMPC_OK;
}

int cmpc_ocp_alloc_count(const cmpc_ocp* o) { return o ? o->allocs : CMPC_ERR_ARG; }

int cmpc_ocp_destroy(cmpc_ocp* o) {
  if (!o) return CMPC_ERR_ARG;
  if (o->ev_done) (void)hipEventSynchronize(o->ev_done);
  if (o->stream) (void)hipStreamSynchronize(o->stream);
  free_all(o);
  delete o;
  return CMPC_OK;
}

int cmpc_ocp_set_settings(cmpc_ocp* o, const cmpc_settings* s) {
  if (!o || !settings_ok(s)) return CMPC_ERR_ARG;
  if (o->ev_done) (void)hipEventSynchronize(o->ev_done);
  o->s = *s;
  return alloc_stats(o);
}

int cmpc_ocp_set_path(cmpc_ocp* o, int chain) {
  if (!o || chain < 0 || chain > 1) return CMPC_ERR_ARG;
  o->chain = chain;
  return CMPC_OK;
}

int cmpc_ocp_path(const cmpc_ocp* o) { return o ? (has_chain(o) ? 1 : 0) : CMPC_ERR_ARG; }

int cmpc_ocp_set_grid(cmpc_ocp* o, int G) {
  if (!o || G < 0 || G > cmpc::OCP_GRID_MAX_G) return CMPC_ERR_ARG;
  o->grid = G;
  return CMPC_OK;
}

int cmpc_ocp_grid(const cmpc_ocp* o, int B) {
  if (!o || B <= 0) return CMPC_ERR_ARG;
  if (!has_chain(o) || !o->bar.p || o->grid == 1 || B > o->hp_batch) return 0;
  return cmpc::ocp_grid_for(o->L, B, o->grid);
}

int cmpc_ocp_set_segments(cmpc_ocp* o, int S) {
  if (!o || S < 0 || S > cmpc::OCP_GRID_MAX_G) return CMPC_ERR_ARG;
  o->nseg = S;
  return CMPC_OK;
}

int cmpc_ocp_segments(const cmpc_ocp* o, int B) {
  const int G = cmpc_ocp_grid(o, B);
  if (G < 0) return G;
  if (G == 0 || !o->seg.p) return 1;
  int S = o->nseg > 0 ? o->nseg : (int)(std::sqrt((o->m > 0 ? 2.0f : 1.0f) * (float)o->N) + 0.5f);  // part_segments
  S = std::min(S, std::min(G, o->N));
  return S < 1 ? 1 : S;
}

int cmpc_ocp_set_grid_timeout(cmpc_ocp* o, double us) {
  if (!o || !(us >= 0.0) || us > 60e6) return CMPC_ERR_ARG;
  o->grid_timeout = us == 0.0 ? 5000000 : (long long)(us * 100.0);  // 100-MHz ticks; 0: the default 50 ms
  return CMPC_OK;
}

int cmpc_ocp_debug_force_grid_timeout(cmpc_ocp* o, int on) {
  if (!o || on < 0 || on > 1) return CMPC_ERR_ARG;
  o->force_timeout = on;
  return CMPC_OK;
}

int cmpc_ocp_fallback_count(cmpc_ocp* o) {
  if (!o) return CMPC_ERR_ARG;
  if (!o->fbk.p) return 0;
  unsigned n = 0;
  if (o->ev_done && hipEventSynchronize(o->ev_done) != hipSuccess) return CMPC_ERR_HIP;
  if (hipMemcpy(&n, o->fbk.p, sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess) return CMPC_ERR_HIP;
  return (int)n;
}

int cmpc_ocp_partition_fallback_count(cmpc_ocp* o) {
  if (!o) return CMPC_ERR_ARG;
  if (!o->fbk.p) return 0;
  unsigned n[2] = {0, 0};
  if (o->ev_done && hipEventSynchronize(o->ev_done) != hipSuccess) return CMPC_ERR_HIP;
  if (hipMemcpy(n, o->fbk.p, sizeof(n), hipMemcpyDeviceToHost) != hipSuccess) return CMPC_ERR_HIP;
  return (int)n[1];
}

int cmpc_ocp_set_keep_riccati(cmpc_ocp* o, int on) {
  if (!o || on < 0 || on > 1) return CMPC_ERR_ARG;
  o->keep_ric = on;
  return CMPC_OK;
}

int cmpc_ocp_enable_timing(cmpc_ocp* o, int on) {
  if (!o || on < 0 || on > 1) return CMPC_ERR_ARG;
  o->timing = on;
  return CMPC_OK;
}

int cmpc_ocp_last_solve_ms(cmpc_ocp* o, float* ms) {
  if (!o || !ms || !o->timing || o->last_B == 0) return CMPC_ERR_ARG;
  if (hipEventSynchronize(o->ev_t1) != hipSuccess || hipEventElapsedTime(ms, o->ev_t0, o->ev_t1) != hipSuccess)
    return CMPC_ERR_HIP;
  return CMPC_OK;
}

double* cmpc_ocp_staging(cmpc_ocp* o, int which) {
  if (!o || !o->pin || o->broken || o->max_batch > cmpc::OCP_GRID_MAX_B) return nullptr;
  const PinMap m = pin_map(o, o->max_batch);
  unsigned char* b = (unsigned char*)o->pin;
  switch (which) {
    case CMPC_OCP_STAGE_X0: return (double*)(b + m.x0);
    case CMPC_OCP_STAGE_REC: return (double*)(b + m.rec);
    case CMPC_OCP_STAGE_CREC: return (double*)(b + m.crec);
    default: return nullptr;
  }
}

int cmpc_ocp_solve(cmpc_ocp* o, int B, const double* d_x0, const double* d_rec, const double* d_crec, double* d_x,
                   double* d_u, int* d_status, int* d_iters, void* stream) {
  if (!o || B < 0 || B > o->max_batch || !d_x0 || !d_rec || !d_x || !d_u || !d_status || o->broken) return CMPC_ERR_ARG;
  if (o->m > 0 && !d_crec) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  const cmpc::OcpSolveArgs a = solve_args(o, d_x0, d_rec, d_crec, d_x, d_u, d_status, d_iters);
  hipStream_t st = (hipStream_t)stream;
  if (o->timing) (void)hipEventRecord(o->ev_t0, st);
  if (cmpc::launch_ocp_ipm(a, B, st) != 0) return CMPC_ERR_HIP;
  if (o->timing) (void)hipEventRecord(o->ev_t1, st);
  // the handle's getters (own stream) are ordered after this solve on the caller's stream
  if (hipEventRecord(o->ev_done, st) != hipSuccess) return CMPC_ERR_HIP;
  o->last_B = B;
  o->last_rec = d_rec;
  o->last_crec = d_crec;
  o->last_status = d_status;
  o->ric_B = (a.ric && !o->linres_on && cmpc_ocp_grid(o, B) > 0) ? B : 0;  // the statistics solve keeps none
  o->ric_full = o->L.m > 0 ? 1 : 0;  // without rows the kernel keeps the factorisation only (k_ocp.hip, exit block)
  return CMPC_OK;
}

int cmpc_ocp_solve_host(cmpc_ocp* o, int B, const double* x0, const double* rec, const double* crec, double* x,
                        double* u, int* status, int* iters) {
  if (!o || B < 0 || B > o->max_batch || !x0 || !rec || !x || (!u && o->nU > 0) || !status || o->broken)
    return CMPC_ERR_ARG;
  if (o->m > 0 && !crec) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  const size_t NP = (size_t)o->N + 1, D = sizeof(double);
  const size_t bx0 = D * B * o->nx, brec = D * B * o->rec_size, bcrec = D * B * o->crec_size,
               bx = D * B * NP * o->nx, bu = D * B * o->nU;
  hipStream_t st = o->stream;
  int r = CMPC_OK;
  auto ck = [&r](hipError_t e) {
    if (e != hipSuccess) r = CMPC_ERR_HIP;
  };
  const bool pinned = o->pin && B <= o->max_batch && o->max_batch <= cmpc::OCP_GRID_MAX_B;
  if (pinned) {  // through the pinned staging: the DMA runs from locked pages (a caller packing into
    // cmpc_ocp_staging's buffers skips the host copy)
    const PinMap m = pin_map(o, o->max_batch);
    unsigned char* b = (unsigned char*)o->pin;
    auto in = [&](size_t off, const void* src, size_t n, void* dev) {
      if (n == 0) return;
      if ((const void*)(b + off) != src) std::memcpy(b + off, src, n);
      ck(hipMemcpyAsync(dev, b + off, n, hipMemcpyHostToDevice, st));
    };
    in(m.x0, x0, bx0, o->x0.p);
    in(m.rec, rec, brec, o->rec.p);
    if (o->m > 0) in(m.crec, crec, bcrec, o->crec.p);
    if (o->s.warm_start) {  // x, u are in / out: the initial guess (HPIPM's primal warm start)
      in(m.x, x, bx, o->x.p);
      if (o->nU > 0) in(m.u, u, bu, o->u.p);
    }
    if (r != CMPC_OK) return r;
    r = cmpc_ocp_solve(o, B, (double*)o->x0.p, (double*)o->rec.p, (double*)o->crec.p, (double*)o->x.p,
                       (double*)o->u.p, (int*)o->status.p, (int*)o->iters.p, st);
    if (r != CMPC_OK) return r;
    ck(hipMemcpyAsync(b + m.x, o->x.p, bx, hipMemcpyDeviceToHost, st));
    if (o->nU > 0) ck(hipMemcpyAsync(b + m.u, o->u.p, bu, hipMemcpyDeviceToHost, st));
    ck(hipMemcpyAsync(b + m.st, o->status.p, sizeof(int) * B, hipMemcpyDeviceToHost, st));
    ck(hipMemcpyAsync(b + m.it, o->iters.p, sizeof(int) * B, hipMemcpyDeviceToHost, st));
    ck(hipStreamSynchronize(st));
    if (r != CMPC_OK) return r;
    std::memcpy(x, b + m.x, bx);
    if (o->nU > 0) std::memcpy(u, b + m.u, bu);
    std::memcpy(status, b + m.st, sizeof(int) * B);
    if (iters) std::memcpy(iters, b + m.it, sizeof(int) * B);
    return r;
  }
  ck(hipMemcpyAsync(o->x0.p, x0, bx0, hipMemcpyHostToDevice, st));
  ck(hipMemcpyAsync(o->rec.p, rec, brec, hipMemcpyHostToDevice, st));
  if (o->m > 0) ck(hipMemcpyAsync(o->crec.p, crec, bcrec, hipMemcpyHostToDevice, st));
  if (o->s.warm_start) {
    ck(hipMemcpyAsync(o->x.p, x, bx, hipMemcpyHostToDevice, st));
    if (o->nU > 0) ck(hipMemcpyAsync(o->u.p, u, bu, hipMemcpyHostToDevice, st));
  }
  if (r != CMPC_OK) return r;
  r = cmpc_ocp_solve(o, B, (double*)o->x0.p, (double*)o->rec.p, (double*)o->crec.p, (double*)o->x.p,
                     (double*)o->u.p, (int*)o->status.p, (int*)o->iters.p, st);
  if (r != CMPC_OK) return r;
  ck(hipMemcpyAsync(x, o->x.p, bx, hipMemcpyDeviceToHost, st));
  if (o->nU > 0) ck(hipMemcpyAsync(u, o->u.p, bu, hipMemcpyDeviceToHost, st));
  ck(hipMemcpyAsync(status, o->status.p, sizeof(int) * B, hipMemcpyDeviceToHost, st));
  if (iters) ck(hipMemcpyAsync(iters, o->iters.p, sizeof(int) * B, hipMemcpyDeviceToHost, st));
  ck(hipStreamSynchronize(st));
  return r;
}

int cmpc_ocp_riccati(cmpc_ocp* o, int B, double* d_P, double* d_p, double* d_K, double* d_k, double* d_Lr_out,
                     int* d_status, void* stream) {
  if (!o || o->broken || B <= 0 || B > o->last_B || !d_P || !d_p || !d_status || (o->nU > 0 && (!d_K || !d_k)) ||
      !o->last_rec || !o->last_status)
    return CMPC_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (hipStreamWaitEvent(st, o->ev_done, 0) != hipSuccess) return CMPC_ERR_HIP;  // after the solve's stream
  if (B <= o->ric_B && o->ric_full) {  // the solve left them (the grid form with keep_riccati): copies
    const size_t NP = (size_t)o->N + 1, nx = (size_t)o->nx, D = sizeof(double);
    int r = CMPC_OK;
    auto cp = [&](void* dst, const void* src, size_t n) {
      if (dst != src && n && hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, st) != hipSuccess) r = CMPC_ERR_HIP;
    };
    cp(d_P, o->P.p, D * B * NP * nx * nx);
    cp(d_p, o->p.p, D * B * NP * nx);
    if (o->nU > 0) {
      cp(d_K, o->K.p, D * B * o->L.nK);
      cp(d_k, o->k.p, D * B * o->nU);
    }
    if (d_Lr_out && o->L.nM > 0) cp(d_Lr_out, o->Lr.p, D * B * o->L.nM);
    cp(d_status, o->rst.p, sizeof(int) * B);
    return r;
  }
  cmpc::OcpRicArgs a;
  a.S = solve_args(o, nullptr, o->last_rec, o->last_crec, nullptr, nullptr, o->last_status, nullptr);
  a.P = d_P;
  a.p = d_p;
  a.K = o->nU > 0 ? d_K : (double*)o->K.p;
  a.k = o->nU > 0 ? d_k : (double*)o->k.p;
  a.Lr = d_Lr_out ? d_Lr_out : (double*)o->Lr.p;
  a.rstatus = d_status;
  if (cmpc::launch_ocp_ric(a, B, st) != 0) return CMPC_ERR_HIP;
  // the workspace's factorisation is the refactorised one now; refactorised into the handle's arrays, their first B
  // problems hold everything
  if (d_P == o->P.p && d_K == o->K.p && d_Lr_out == o->Lr.p && d_status == (int*)o->rst.p) {
    o->ric_B = B;
    o->ric_full = 1;
  } else {
    o->ric_B = 0;
  }
  return CMPC_OK;
}

int cmpc_ocp_riccati_feedback_host(cmpc_ocp* o, int b, double* K, double* Lr, double* P1, int* status) {
  if (!o || b < 0 || b >= o->last_B || !Lr || !P1 || !status || (o->nU > 0 && !K) || o->N < 1) return CMPC_ERR_ARG;
  hipStream_t st = o->stream;
  int r = CMPC_OK;
  if (b >= o->ric_B) {  // not kept by the solve: refactorise problems 0..b into the handle's arrays
    r = cmpc_ocp_riccati(o, b + 1, (double*)o->P.p, (double*)o->p.p, (double*)o->K.p, (double*)o->k.p,
                         (double*)o->Lr.p, (int*)o->rst.p, st);
    if (r != CMPC_OK) return r;
  } else if (hipStreamWaitEvent(st, o->ev_done, 0) != hipSuccess) {
    return CMPC_ERR_HIP;
  }
  const size_t NP = (size_t)o->N + 1, nx = (size_t)o->nx, D = sizeof(double);
  const size_t nK = (size_t)o->L.nK, nM = (size_t)o->L.nM;
  auto ck = [&r](hipError_t e) {
    if (e != hipSuccess) r = CMPC_ERR_HIP;
  };
  const bool pinned = o->pin && o->max_batch <= cmpc::OCP_GRID_MAX_B;
  unsigned char* pb = (unsigned char*)o->pin;
  const PinMap m = pinned ? pin_map(o, o->max_batch) : PinMap{};
  auto out = [&](void* dst, size_t off, const void* src, size_t n) {
    if (n) ck(hipMemcpyAsync(pinned ? (void*)(pb + off) : dst, src, n, hipMemcpyDeviceToHost, st));
  };
  if (nK) out(K, m.K, (const double*)o->K.p + (size_t)b * nK, D * nK);
  if (nM) out(Lr, m.Lr, (const double*)o->Lr.p + (size_t)b * nM, D * nM);
  out(P1, m.P, (const double*)o->P.p + (size_t)b * NP * nx * nx + nx * nx, D * nx * nx);
  out(status, m.rst, (const int*)o->rst.p + b, sizeof(int));
  ck(hipStreamSynchronize(st));
  if (r == CMPC_OK && pinned) {
    if (nK) std::memcpy(K, pb + m.K, D * nK);
    if (nM) std::memcpy(Lr, pb + m.Lr, D * nM);
    std::memcpy(P1, pb + m.P, D * nx * nx);
    std::memcpy(status, pb + m.rst, sizeof(int));
  }
  return r;
}

int cmpc_ocp_riccati_host(cmpc_ocp* o, int B, double* P, double* p, double* K, double* k, double* Lr,
                          int* status) {
  if (!o || B <= 0 || B > o->last_B || !P || !p || !status || (o->nU > 0 && (!K || !k))) return CMPC_ERR_ARG;
  hipStream_t st = o->stream;
  int r = cmpc_ocp_riccati(o, B, (double*)o->P.p, (double*)o->p.p, (double*)o->K.p, (double*)o->k.p,
                           (double*)o->Lr.p, (int*)o->rst.p, st);
  if (r != CMPC_OK) return r;
  const size_t NP = (size_t)o->N + 1, nx = (size_t)o->nx, D = sizeof(double);
  const size_t bP = D * B * NP * nx * nx, bp = D * B * NP * nx, bK = D * B * o->L.nK, bk = D * B * o->nU,
               bL = D * B * o->L.nM;
  auto ck = [&r](hipError_t e) {
    if (e != hipSuccess) r = CMPC_ERR_HIP;
  };
  const bool pinned = o->pin && o->max_batch <= cmpc::OCP_GRID_MAX_B;
  unsigned char* b = (unsigned char*)o->pin;
  const PinMap m = pinned ? pin_map(o, o->max_batch) : PinMap{};
  auto out = [&](void* dst, size_t off, const void* src, size_t n) {
    if (n) ck(hipMemcpyAsync(pinned ? (void*)(b + off) : dst, src, n, hipMemcpyDeviceToHost, st));
  };
  out(P, m.P, o->P.p, bP);
  out(p, m.p, o->p.p, bp);
  if (o->nU > 0) {
    out(K, m.K, o->K.p, bK);
    out(k, m.k, o->k.p, bk);
  }
  if (Lr && o->L.nM > 0) out(Lr, m.Lr, o->Lr.p, bL);
  out(status, m.rst, o->rst.p, sizeof(int) * B);
  ck(hipStreamSynchronize(st));
  if (r == CMPC_OK && pinned) {
    std::memcpy(P, b + m.P, bP);
    std::memcpy(p, b + m.p, bp);
    if (o->nU > 0) {
      std::memcpy(K, b + m.K, bK);
      std::memcpy(k, b + m.k, bk);
    }
    if (Lr && o->L.nM > 0) std::memcpy(Lr, b + m.Lr, bL);
    std::memcpy(status, b + m.rst, sizeof(int) * B);
  }
  return r;
}

int cmpc_ocp_get_residuals(cmpc_ocp* o, int B, double* d_res, void* stream) {
  if (!o || B < 0 || B > o->max_batch || !d_res) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  if (hipStreamWaitEvent((hipStream_t)stream, o->ev_done, 0) != hipSuccess) return CMPC_ERR_HIP;
  return hipMemcpyAsync(d_res, o->res.p, sizeof(double) * B * 4, hipMemcpyDeviceToDevice, (hipStream_t)stream) ==
                 hipSuccess
             ? CMPC_OK
             : CMPC_ERR_HIP;
}

int cmpc_ocp_stat_rows(const cmpc_ocp* o) { return o ? o->stat_rows : CMPC_ERR_ARG; }

int cmpc_ocp_set_linres(cmpc_ocp* o, int on) {
  if (!o || on < 0 || on > 1) return CMPC_ERR_ARG;
  if (o->ev_done) (void)hipEventSynchronize(o->ev_done);
  o->linres_on = on;
  return on ? alloc_stats(o) : CMPC_OK;
}

int cmpc_ocp_get_linres(cmpc_ocp* o, int B, double* d_linres, void* stream) {
  if (!o || B < 0 || B > o->max_batch || !d_linres || !o->linres_on) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  if (hipStreamWaitEvent((hipStream_t)stream, o->ev_done, 0) != hipSuccess) return CMPC_ERR_HIP;
  return hipMemcpyAsync(d_linres, o->linres.p, sizeof(double) * B * o->stat_rows * 4, hipMemcpyDeviceToDevice,
                        (hipStream_t)stream) == hipSuccess
             ? CMPC_OK
             : CMPC_ERR_HIP;
}

int cmpc_ocp_get_linres_host(cmpc_ocp* o, int B, double* linres) {
  if (!o || B < 0 || B > o->max_batch || !linres || !o->linres_on) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  if (hipStreamWaitEvent(o->stream, o->ev_done, 0) != hipSuccess ||
      hipMemcpyAsync(linres, o->linres.p, sizeof(double) * B * o->stat_rows * 4, hipMemcpyDeviceToHost, o->stream) !=
          hipSuccess ||
      hipStreamSynchronize(o->stream) != hipSuccess)
    return CMPC_ERR_HIP;
  return CMPC_OK;
}

int cmpc_ocp_get_stats(cmpc_ocp* o, int B, double* d_stats, void* stream) {
  if (!o || B < 0 || B > o->max_batch || !d_stats) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  if (hipStreamWaitEvent((hipStream_t)stream, o->ev_done, 0) != hipSuccess) return CMPC_ERR_HIP;
  return hipMemcpyAsync(d_stats, o->stats.p, sizeof(double) * B * o->stat_rows * CMPC_STAT_COLS,
                        hipMemcpyDeviceToDevice, (hipStream_t)stream) == hipSuccess
             ? CMPC_OK
             : CMPC_ERR_HIP;
}

int cmpc_ocp_get_residuals_host(cmpc_ocp* o, int B, double* res) {
  if (!o || B < 0 || B > o->max_batch || !res) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  if (hipStreamWaitEvent(o->stream, o->ev_done, 0) != hipSuccess ||
      hipMemcpyAsync(res, o->res.p, sizeof(double) * B * 4, hipMemcpyDeviceToHost, o->stream) != hipSuccess ||
      hipStreamSynchronize(o->stream) != hipSuccess)
    return CMPC_ERR_HIP;
  return CMPC_OK;
}

int cmpc_ocp_get_stats_host(cmpc_ocp* o, int B, double* stats) {
  if (!o || B < 0 || B > o->max_batch || !stats) return CMPC_ERR_ARG;
  if (B == 0) return CMPC_OK;
  if (hipStreamWaitEvent(o->stream, o->ev_done, 0) != hipSuccess ||
      hipMemcpyAsync(stats, o->stats.p, sizeof(double) * B * o->stat_rows * CMPC_STAT_COLS, hipMemcpyDeviceToHost,
                     o->stream) != hipSuccess ||
      hipStreamSynchronize(o->stream) != hipSuccess)
    return CMPC_ERR_HIP;
  return CMPC_OK;
}

#ifdef CMPC_OCP_CHAIN_LAB
// Lab only: time reps launches of the latency-form factorisation on the last solve's workspace (ms per launch)
int cmpc_ocp_debug_chain(cmpc_ocp* o, int B, int reps, float* ms) {
  if (!o || B <= 0 || B > o->last_B || !o->hp.p || reps <= 0 || !ms) return CMPC_ERR_ARG;
  cmpc::OcpSolveArgs a = solve_args(o, nullptr, o->last_rec, o->last_crec, nullptr, nullptr, (int*)o->rst.p, nullptr);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, o->stream);
  for (int r = 0; r < reps; ++r)
    if (cmpc::launch_ocp_chain_lab(a, B, o->stream) != 0) return CMPC_ERR_HIP;
  (void)hipEventRecord(e1, o->stream);
  (void)hipEventSynchronize(e1);
  float t = 0.f;
  (void)hipEventElapsedTime(&t, e0, e1);
  *ms = t / reps;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return CMPC_OK;
}
#endif

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
