/* asan_driver.c — host AddressSanitizer / UBSan run of the CPU oracle (test infrastructure; SURVEY section 5,
 * "race detection / sanitizers"). Built with -fsanitize=address,undefined by `make -C oracle asan` and run by
 * tests/test_sanitizers.py: every oracle entry point the tests use runs on generated inputs (trot and mixed gaits,
 * the 64 / 128 / 256 size classes, the Riccati restatement, the SQP, the feedback policy, the gait tables, the
 * generic OCP path); any out-of-bounds access, use after free or undefined behaviour aborts with a report. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cmpc_oracle.h"

#define CHECK(c)                                                 \
  do {                                                           \
    if (!(c)) {                                                  \
      fprintf(stderr, "asan_driver: check failed: %s (line %d)\n", #c, __LINE__); \
      return 1;                                                  \
    }                                                            \
  } while (0)

#define NX CMPC_NX
#define NU CMPC_NU
#define NL CMPC_MAX_LEGS

/* oracle_py.default_model / default_settings (CentoidMPCTest.cpp:12-33, HpipmInterfaceSettings.h:44-57) */
static void default_model(cmpc_model* m, int N) {
  static const double w[CMPC_NUM_WEIGHTS] = {1, 1, 100, 0.5, 0.5, 0, 2, 2, 8,
                                             0.2, 0.2, 0.2, 0.3, 0.3, 0.3, 0.1, 0.1, 0.1,
                                             0.2, 0.2, 0.2, 0.3, 0.3, 0.3, 0.1, 0.1, 0.1,
                                             0.2, 0.2, 0.2, 0.3, 0.3, 0.3, 0.1, 0.1, 0.1,
                                             0.2, 0.2, 0.2, 0.3, 0.3, 0.3, 0.1, 0.1, 0.1};
  memset(m, 0, sizeof(*m));
  m->N = N;
  m->n_legs = NL;
  m->mass = 8.0;
  m->dt = 0.01;
  m->inertia[0] = 0.07;
  m->inertia[4] = 0.26;
  m->inertia[8] = 0.28;
  for (int i = 0; i < NL; ++i) m->mu[i] = 0.8;
  memcpy(m->weights, w, sizeof(w));
  for (int i = 0; i < 4; ++i) m->force_ub[i] = 5000.0;
  m->force_ub[4] = 8.0 * 9.81 * NL;
}
static void default_settings(cmpc_settings* s) {
  memset(s, 0, sizeof(*s));
  s->hpipm_mode = 1;
  s->iter_max = 30;
  s->alpha_min = 1e-12;
  s->mu0 = 10.0;
  s->tol_stat = 1e-6;
  s->tol_eq = 1e-8;
  s->tol_ineq = 1e-8;
  s->tol_comp = 1e-8;
  s->reg_prim = 1e-12;
  s->pred_corr = 1;
}

static int run_batch(int N, int B, int gait, int all_stance) {
  cmpc_model m;
  default_model(&m, N);
  cmpc_settings s;
  default_settings(&s);
  double* x0 = calloc((size_t)B * NX, sizeof(double));
  double* xref = calloc((size_t)B * (N + 1) * NX, sizeof(double));
  double* foot = calloc((size_t)B * (N + 1) * NL * 3, sizeof(double));
  uint8_t* contact = calloc((size_t)B * N * NL, 1);
  double* u = calloc((size_t)B * N * NL * 3, sizeof(double));
  double* x = calloc((size_t)B * (N + 1) * NX, sizeof(double));
  double* ur = calloc((size_t)B * N * NL * 3, sizeof(double));
  int* st = calloc(B, sizeof(int));
  int* it = calloc(B, sizeof(int));
  int* str = calloc(B, sizeof(int));
  int* itr = calloc(B, sizeof(int));
  oracle_generate(&m, 20221125ull, 0, B, gait, x0, xref, foot, contact);
  if (all_stance) memset(contact, 1, (size_t)B * N * NL);
  CHECK(oracle_solve_batch(&m, &s, B, x0, xref, foot, contact, u, x, st, it, 2) == 0);
  CHECK(oracle_riccati_solve_batch(&m, &s, B, x0, xref, foot, contact, ur, str, itr, 2) == 0);
  for (int q = 0; q < B; ++q) CHECK(st[q] == str[q]);
  oracle_consts c;
  oracle_consts_init(&m, &c);
  /* SQP and policy on the first QP */
  {
    double* us = calloc((size_t)N * NL * 3, sizeof(double));
    int qi = 0, si = 0;
    (void)oracle_sqp_solve(&c, &s, 3, 1e-7, x0, xref, foot, contact, us, NULL, &qi, &si);
    free(us);
  }
  {
    const int n = NU * N;
    double* K = calloc((size_t)n * NX, sizeof(double));
    int nfree = 0;
    (void)oracle_policy(&c, xref, foot, contact, u, 1e-6, K, &nfree);
    free(K);
  }
  free(x0); free(xref); free(foot); free(contact); free(u); free(x); free(ur); free(st); free(it); free(str); free(itr);
  return 0;
}

int main(void) {
  if (run_batch(10, 16, 0, 0)) return 1;  /* trot, n = 60 */
  if (run_batch(10, 16, 1, 0)) return 1;  /* mixed gait, n <= 120 */
  if (run_batch(20, 2, 0, 1)) return 1;   /* all stance, n = 240 */
  /* gait tables */
  {
    cmpc_gait g;
    memset(&g, 0, sizeof(g));
    g.n_modes = 2;
    g.mode[0] = 9;  /* LF + RH */
    g.mode[1] = 6;  /* RF + LH */
    g.switching_time[0] = 0.0;
    g.switching_time[1] = 0.3;
    g.switching_time[2] = 0.6;
    uint8_t ct[10 * NL];
    const int leg_map[4] = {0, 1, 3, 2};
    oracle_gait_contact(&g, leg_map, 0.1, 0.0, 0.05, 10, ct);
  }
  printf("asan_driver ok\n");
  return 0;
}
