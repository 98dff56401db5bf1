// ipm_lab.cpp — development harness for A/B timing of IPM kernel variants on identical condensed QPs.
// Not part of the product: it links libcmpc.so for input generation, condensing and packing (the product path),
// runs the product solve once as the reference, then times each lab variant with HIP events and checks its
// solution against the reference. Usage: ipm_lab [B] [reps]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#include "cmpc/cmpc.h"
#include "cmpc_kernels.hpp"

using namespace cmpc;
typedef int (*lab_fn)(const IpmArgs<double>*, int, hipStream_t, unsigned long long*);
typedef int (*lab_prep)(const IpmArgs<double>*, int, hipStream_t, IpmArgs<double>*);

#define LAB_VARIANTS_DECL
#include "variants.inc"
#undef LAB_VARIANTS_DECL

struct Var {
  const char* name;
  lab_fn fn;
  lab_prep prep;
  int stamps;
};
static Var VARS[] = {
#define LAB_VARIANTS_LIST
#include "variants.inc"
#undef LAB_VARIANTS_LIST
};

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)
#define CC(x)                                                            \
  do {                                                                   \
    int r_ = (x);                                                        \
    if (r_ != 0) {                                                       \
      fprintf(stderr, "cmpc error %d at %s:%d\n", r_, __FILE__, __LINE__); \
      exit(1);                                                           \
    }                                                                    \
  } while (0)

template <typename T>
T* dmalloc(size_t n) {
  T* p = nullptr;
  CK(hipMalloc((void**)&p, n * sizeof(T)));
  CK(hipMemset(p, 0, n * sizeof(T)));
  return p;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 4096;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const char* only = argc > 3 ? argv[3] : nullptr;
  const int N = 10;
  cmpc_model m;
  cmpc_model_default(&m, N);
  cmpc_settings s;
  cmpc_settings_default(&s);
  cmpc_ctx* ctx = nullptr;
  CC(cmpc_create(&m, &s, CMPC_F64, B, nullptr, &ctx));
  const int ld = cmpc_ctx_ld(ctx), nt = ld / 3;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  double* x0 = dmalloc<double>((size_t)B * 13);
  double* xref = dmalloc<double>((size_t)B * (N + 1) * 13);
  double* foot = dmalloc<double>((size_t)B * (N + 1) * 12);
  uint8_t* contact = dmalloc<uint8_t>((size_t)B * N * 4);
  CC(cmpc_generate_batch(&m, 20221125ull, 0, B, 0, x0, xref, foot, contact, st));
  // LAB_ALLSTANCE=1: every leg in stance (n = 120, the 64 < n <= 128 class)
  if (getenv("LAB_ALLSTANCE") && atoi(getenv("LAB_ALLSTANCE"))) CK(hipMemsetAsync(contact, 1, (size_t)B * N * 4, st));
  double* H = dmalloc<double>((size_t)B * ld * ld);
  double* g = dmalloc<double>((size_t)B * ld);
  int* n = dmalloc<int>(B);
  int* cst = dmalloc<int>(B);
  CC(cmpc_condense_batch(ctx, B, x0, xref, foot, contact, H, g, n, cst, st));
  std::vector<double> hmu((size_t)B * nt, m.mu[0]), hlo((size_t)B * nt * 5, 0.0), hhi((size_t)B * nt * 5);
  for (size_t t = 0; t < (size_t)B * nt; ++t)
    for (int r = 0; r < 5; ++r) hhi[t * 5 + r] = m.force_ub[r];
  double* mu = dmalloc<double>(hmu.size());
  double* lo = dmalloc<double>(hlo.size());
  double* hi = dmalloc<double>(hhi.size());
  CK(hipMemcpy(mu, hmu.data(), hmu.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(lo, hlo.data(), hlo.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(hi, hhi.data(), hhi.size() * 8, hipMemcpyHostToDevice));
  // reference: the product solve (libcmpc.so) on the same QPs
  double* uref = dmalloc<double>((size_t)B * ld);
  int* sref = dmalloc<int>(B);
  int* iref = dmalloc<int>(B);
  CC(cmpc_qp_solve_batch(ctx, B, H, g, n, mu, lo, hi, uref, sref, iref, st));
  CK(hipStreamSynchronize(st));
  std::vector<double> hu_ref((size_t)B * ld);
  std::vector<int> hs_ref(B), hi_ref(B), hn(B);
  CK(hipMemcpy(hu_ref.data(), uref, hu_ref.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hs_ref.data(), sref, B * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hi_ref.data(), iref, B * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hn.data(), n, B * 4, hipMemcpyDeviceToHost));
  double it_sum = 0;
  int nok = 0;
  for (int q = 0; q < B; ++q)
    if (hs_ref[q] == 0) it_sum += hi_ref[q], ++nok;
  printf("{\"ref\": {\"B\": %d, \"ld\": %d, \"success\": %d, \"mean_iters\": %.4f, \"n0\": %d}}\n", B, ld, nok,
         it_sum / (nok ? nok : 1), hn[0]);
  // lab workspace (product class-packed layout)
  double* Hw = dmalloc<double>((size_t)B * ld * ld);
  double* gw = dmalloc<double>((size_t)B * ld);
  double* muw = dmalloc<double>((size_t)B * nt);
  double* low = dmalloc<double>((size_t)B * nt * 5);
  double* hiw = dmalloc<double>((size_t)B * nt * 5);
  int* nw = dmalloc<int>(B);
  int* sw = dmalloc<int>(B);
  int* s0 = dmalloc<int>(B);
  int* iw = dmalloc<int>(B);
  double* uw = dmalloc<double>((size_t)B * ld);
  unsigned long long* stamps = dmalloc<unsigned long long>((size_t)B * 9);
  CC(launch_pack_qp(H, g, mu, lo, hi, n, CMPC_F64, ld, Hw, gw, muw, low, hiw, nw, s0, B, st));
  IpmArgs<double> a{};
  a.ld = ld;
  a.H = Hw;
  a.g = gw;
  a.tri_mu = muw;
  a.tri_lo = low;
  a.tri_hi = hiw;
  a.nvar = nw;
  a.status = sw;
  a.iters = iw;
  a.u = uw;
  a.s.iter_max = s.iter_max;
  a.s.alpha_min = s.alpha_min;
  a.s.mu0 = s.mu0;
  a.s.tol_stat = s.tol_stat;
  a.s.tol_ineq = s.tol_ineq;
  a.s.tol_comp = s.tol_comp;
  a.s.reg_prim = s.reg_prim;
  if (getenv("LAB_RES") && atoi(getenv("LAB_RES"))) {  // the product's residual export buffers (cmpc_get_residuals)
    a.res_scr = dmalloc<double>((size_t)B * 3 * 256);
    a.res = dmalloc<double>((size_t)B * 4);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<double> hu((size_t)B * ld);
  std::vector<int> hs(B), hit(B);
  std::vector<unsigned long long> hst((size_t)B * 9);
  // interleaved timing: every round launches each variant once (round-robin), after a warm-up of the GPU clock;
  // medians over rounds are robust to DVFS drift between variants
  std::vector<int> sel;
  const int nv = (int)(sizeof(VARS) / sizeof(VARS[0]));
  for (int i = 0; i < nv; ++i)
    if (!only || strstr(VARS[i].name, only)) sel.push_back(i);
  std::vector<IpmArgs<double>> vargs(nv);
  for (int i : sel) {
    CC(VARS[i].prep(&a, B, st, &vargs[i]));
    CK(hipStreamSynchronize(st));
  }
  const bool repack = getenv("LAB_REPACK") && atoi(getenv("LAB_REPACK"));  // H freshly written before every run
  auto run_once = [&](int i, bool with_stamps) -> float {
    if (repack) {
      CC(cmpc_condense_batch(ctx, B, x0, xref, foot, contact, H, g, n, cst, st));
      CC(launch_pack_qp(H, g, mu, lo, hi, n, CMPC_F64, ld, Hw, gw, muw, low, hiw, nw, s0, B, st));
    }
    CK(hipMemcpyAsync(sw, s0, B * 4, hipMemcpyDeviceToDevice, st));
    CK(hipMemsetAsync(uw, 0, (size_t)B * ld * 8, st));
    CK(hipEventRecord(e0, st));
    CC(VARS[i].fn(&vargs[i], B, st, with_stamps ? stamps : nullptr));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms;
  };
  for (int w = 0; w < 30; ++w)
    for (int i : sel) run_once(i, false);
  std::vector<std::vector<float>> times(nv);
  for (int r = 0; r < reps; ++r)
    for (int i : sel) times[i].push_back(run_once(i, false));
  for (int i : sel) {
    const Var& v = VARS[i];
    std::vector<float> t = times[i];
    std::sort(t.begin(), t.end());
    const float med = t[t.size() / 2], best = t[0];
    run_once(i, v.stamps != 0);  // final run: results (+ stamps)
    CK(hipMemcpy(hu.data(), uw, hu.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hs.data(), sw, B * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hit.data(), iw, B * 4, hipMemcpyDeviceToHost));
    double maxrel = 0;
    int same_it = 0, same_st = 0, bitexact = 0;
    for (int q = 0; q < B; ++q) {
      double sc = 1.0, d = 0.0;
      for (int k = 0; k < ld; ++k) sc = fmax(sc, fabs(hu_ref[(size_t)q * ld + k]));
      bool be = true;
      for (int k = 0; k < ld; ++k) {
        d = fmax(d, fabs(hu[(size_t)q * ld + k] - hu_ref[(size_t)q * ld + k]));
        be = be && hu[(size_t)q * ld + k] == hu_ref[(size_t)q * ld + k];
      }
      if (!(d / sc <= maxrel)) maxrel = d / sc;
      same_it += hit[q] == hi_ref[q];
      same_st += hs[q] == hs_ref[q];
      bitexact += be;
    }
    printf("{\"variant\": \"%s\", \"ms_median\": %.5f, \"ms_best\": %.5f, \"qps_ipm\": %.0f, \"max_rel_du\": %.3e, "
           "\"same_status\": %d, \"same_iters\": %d, \"bitexact\": %d",
           v.name, med, best, B / (med * 1e-3), maxrel, same_st, same_it, bitexact);
    if (v.stamps == 2) {  // timeline build: raw [start, end, HW_ID, XCC_ID] per QP to a file for offline analysis
      CK(hipMemcpy(hst.data(), stamps, hst.size() * 8, hipMemcpyDeviceToHost));
      char path[256];
      snprintf(path, sizeof(path), "%s/timeline_%s.bin", getenv("LAB_OUT") ? getenv("LAB_OUT") : ".", v.name);
      FILE* f = fopen(path, "wb");
      if (f) {
        fwrite(hst.data(), 8, hst.size(), f);
        fclose(f);
      }
    } else if (v.stamps) {
      CK(hipMemcpy(hst.data(), stamps, hst.size() * 8, hipMemcpyDeviceToHost));
      double seg[9] = {0}, its = 0;
      for (int q = 0; q < B; ++q) {
        if (hs[q] != 0) continue;
        for (int k = 0; k < 9; ++k) seg[k] += (double)hst[(size_t)q * 9 + k];
        its += hit[q];
      }
      static const char* names[9] = {"s0", "s1", "s2", "s3", "s4", "s5", "s6", "s7", "total"};
      printf(", \"cycles_per_iter\": {");
      for (int k = 0; k < 9; ++k) printf("%s\"%s\": %.0f", k ? ", " : "", names[k], seg[k] / (its > 0 ? its : 1));
      printf("}");
    }
    printf("}\n");
    fflush(stdout);
  }
  cmpc_destroy(ctx);
  return 0;
}
