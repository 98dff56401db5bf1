// abi_sanitize.cpp — host AddressSanitizer / UBSan run of the C ABI's argument checking and of the host C++ mirrors
// (SURVEY section 5). Linked against lib/libcmpc_asan.so, whose host code (cmpc_api.cpp, host/*.cpp) is built with
// -fsanitize=address,undefined (`make -C cheeta-mpc_amd asan`); the device code is the ordinary build. Needs no GPU:
// every call here is rejected before any device work (or, without a device, with CMPC_ERR_NO_DEVICE), and the host
// mirrors' size checks and record packing run in full. Run by tests/test_sanitizers.py; exit 0 = every check held
// and the sanitizers reported nothing.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "cheeta_mpc/CentroidalMPC.h"
#include "cmpc/cmpc.h"
#include "hpipm_catkin/HpipmInterface.h"

static int fails = 0;
#define EXPECT(c)                                                        \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "abi_sanitize: FAILED %s (line %d)\n", #c, __LINE__); \
      ++fails;                                                           \
    }                                                                    \
  } while (0)

template <typename E, typename F>
static bool throws(F&& f) {
  try {
    f();
  } catch (const E&) {
    return true;
  } catch (...) {
    return false;
  }
  return false;
}

int main() {
  cmpc_settings s;
  cmpc_settings_default(&s);
  EXPECT(s.iter_max == 30 && s.pred_corr == 1 && s.tol_stat == 1e-6);
  cmpc_model m;
  cmpc_model_default(&m, 10);
  EXPECT(m.N == 10 && m.n_legs == 4 && m.mass == 8.0);

  // sizes and creation arguments
  EXPECT(cmpc_memsize(nullptr, CMPC_F64, 16) == 0);
  EXPECT(cmpc_memsize(&m, CMPC_F64, 0) == 0);
  EXPECT(cmpc_memsize(&m, CMPC_F64, 16) > 0);
  cmpc_ctx* ctx = nullptr;
  EXPECT(cmpc_create(&m, &s, CMPC_F64, 16, nullptr, nullptr) == CMPC_ERR_ARG);
  EXPECT(cmpc_create(&m, &s, 7, 16, nullptr, &ctx) == CMPC_ERR_ARG);
  EXPECT(cmpc_create(&m, &s, CMPC_F64, 0, nullptr, &ctx) == CMPC_ERR_ARG);
  cmpc_settings bad = s;
  bad.pred_corr = 0;
  EXPECT(cmpc_create(&m, &bad, CMPC_F64, 16, nullptr, &ctx) == CMPC_ERR_ARG);
  bad = s;
  bad.tol_stat = -1.0;
  EXPECT(cmpc_create(&m, &bad, CMPC_F64, 16, nullptr, &ctx) == CMPC_ERR_ARG);
  cmpc_model bm = m;
  bm.N = 0;
  EXPECT(cmpc_create(&bm, &s, CMPC_F64, 16, nullptr, &ctx) == CMPC_ERR_ARG);
  bm = m;
  bm.n_legs = 3;
  EXPECT(cmpc_create(&bm, &s, CMPC_F64, 16, nullptr, &ctx) == CMPC_ERR_ARG);

  // every context entry point rejects a null context
  double dbuf[64] = {0};
  int ibuf[8] = {0};
  uint8_t cbuf[64] = {0};
  EXPECT(cmpc_destroy(nullptr) == CMPC_ERR_ARG);
  EXPECT(cmpc_set_settings(nullptr, &s) == CMPC_ERR_ARG);
  EXPECT(cmpc_set_model(nullptr, &m) == CMPC_ERR_ARG);
  EXPECT(cmpc_get_model(nullptr, &m) == CMPC_ERR_ARG);
  EXPECT(cmpc_ctx_ld(nullptr) == 0 && cmpc_ctx_fused(nullptr) == 0);
  EXPECT(cmpc_solve_batch(nullptr, 1, dbuf, dbuf, dbuf, cbuf, dbuf, nullptr, ibuf, ibuf, nullptr) == CMPC_ERR_ARG);
  EXPECT(cmpc_solve_batch_warm(nullptr, 1, dbuf, dbuf, dbuf, cbuf, dbuf, dbuf, nullptr, ibuf, ibuf, nullptr) ==
         CMPC_ERR_ARG);
  EXPECT(cmpc_sqp_solve_batch(nullptr, 1, dbuf, dbuf, dbuf, cbuf, 3, 1e-7, dbuf, nullptr, ibuf, ibuf, ibuf,
                              nullptr) == CMPC_ERR_ARG);
  EXPECT(cmpc_solve_batch_host(nullptr, 1, dbuf, dbuf, dbuf, cbuf, dbuf, nullptr, ibuf, ibuf) == CMPC_ERR_ARG);
  EXPECT(cmpc_condense_batch(nullptr, 1, dbuf, dbuf, dbuf, cbuf, dbuf, dbuf, ibuf, ibuf, nullptr) == CMPC_ERR_ARG);
  EXPECT(cmpc_qp_solve_batch(nullptr, 1, dbuf, dbuf, ibuf, dbuf, dbuf, dbuf, dbuf, ibuf, ibuf, nullptr) ==
         CMPC_ERR_ARG);
  EXPECT(cmpc_get_residuals(nullptr, 1, dbuf, nullptr) == CMPC_ERR_ARG);
  EXPECT(cmpc_profile_begin(nullptr, 4) == CMPC_ERR_ARG);
  double ms[3];
  EXPECT(cmpc_profile_end(nullptr, &ms[0], &ms[1], &ms[2], ibuf) == CMPC_ERR_ARG);
  EXPECT(cmpc_generate_batch(nullptr, 1, 0, 1, 0, dbuf, dbuf, dbuf, cbuf, nullptr) == CMPC_ERR_ARG);
  EXPECT(cmpc_shift_inputs(-1, 10, dbuf, 1, dbuf, nullptr) == CMPC_ERR_ARG);

  // names: every code, and out-of-range ones
  for (int k = -2; k <= 8; ++k) EXPECT(cmpc_status_string(k) != nullptr && std::strlen(cmpc_status_string(k)) > 0);
  for (int k = -6; k <= 1; ++k) EXPECT(cmpc_error_string(k) != nullptr && std::strlen(cmpc_error_string(k)) > 0);
  EXPECT(cmpc_version() != nullptr);

  // gait templates (host tables)
  const char* names[] = {"stance", "trot", "standing_trot", "flying_trot", "pace", "standing_pace", "dynamic_walk",
                         "static_walk", "amble", "lindyhop", "skipping", "pawup"};
  for (const char* nm : names) {
    cmpc_gait g;
    EXPECT(cmpc_gait_builtin(nm, &g) == CMPC_OK && g.n_modes >= 1 && g.n_modes <= CMPC_GAIT_MAX_MODES);
  }
  cmpc_gait g0;
  EXPECT(cmpc_gait_builtin("no_such_gait", &g0) == CMPC_ERR_ARG);
  EXPECT(cmpc_gait_builtin(nullptr, &g0) == CMPC_ERR_ARG);
  EXPECT(cmpc_gait_table_create(nullptr, 1, nullptr, nullptr) == CMPC_ERR_ARG);

  // generic OCP records: sizes and argument checks
  const int nu3[3] = {2, 2, 2};
  EXPECT(cmpc_ocp_record_size(3, 4, nu3) > 0);
  const int nc4[4] = {1, 0, 2, 1};
  EXPECT(cmpc_ocp_constraint_record_size(3, 4, nu3, nc4) > 0);
  EXPECT(cmpc_ocp_constraint_record_size(3, 4, nu3, nullptr) == 0);
  EXPECT(cmpc_ocp_solve_batch_host(1, 3, 4, nullptr, dbuf, dbuf, dbuf, dbuf, ibuf) == CMPC_ERR_ARG);

  // HpipmInterface mirror: OcpSize extraction (OcpSize.cpp:35-75), size checks, record packing
  {
    using namespace ocs2;
    const int N = 3, nx = 4, nu = 2;
    std::vector<VectorFunctionLinearApproximation> dyn((size_t)N);
    std::vector<ScalarFunctionQuadraticApproximation> cost((size_t)N + 1);
    for (int k = 0; k < N; ++k) {
      dyn[(size_t)k].dfdx.resize(nx, nx);
      dyn[(size_t)k].dfdu.resize(nx, nu);
      dyn[(size_t)k].f.resize(nx);
      for (int i = 0; i < nx; ++i) dyn[(size_t)k].dfdx(i, i) = 1.0;
    }
    for (int k = 0; k <= N; ++k) {
      const int u = k < N ? nu : 0;
      auto& c = cost[(size_t)k];
      c.dfdx.resize(nx);
      c.dfdu.resize(u);
      c.dfdxx.resize(nx, nx);
      c.dfdux.resize(u, nx);
      c.dfduu.resize(u, u);
      for (int i = 0; i < nx; ++i) c.dfdxx(i, i) = 1.0;
      for (int i = 0; i < u; ++i) c.dfduu(i, i) = 1.0;
    }
    const auto sz = hpipm_interface::extractSizesFromProblem(dyn, cost, nullptr);
    EXPECT(sz.numStages == N && sz.numInputs[0] == nu && sz.numInputs[(size_t)N] == 0 && sz.numStates[0] == nx);
    EXPECT(sz == hpipm_interface::OcpSize(N, nx, nu));
    HpipmInterface hp(sz);
    hp.resize(sz);
    vector_t x0(nx);
    vector_array_t xs, us;
    std::vector<VectorFunctionLinearApproximation> dyn_short(dyn.begin(), dyn.end() - 1);
    EXPECT(throws<std::runtime_error>([&] { hp.solve(x0, dyn_short, cost, nullptr, xs, us); }));
    std::vector<VectorFunctionLinearApproximation> cons((size_t)N);  // wrong length: N instead of N + 1
    EXPECT(throws<std::runtime_error>([&] { hp.solve(x0, dyn, cost, &cons, xs, us); }));
    // a consistent problem packs its records on the host; the device call either runs (GPU) or reports no device
    try {
      (void)hp.solve(x0, dyn, cost, nullptr, xs, us);
    } catch (const std::exception&) {
    }
  }

  // CentroidalMPC mirror: constructor checks, record packing (CentroidalMPC.cpp:278-323), use before SetupMPC
  {
    using VectorXd = cheeta_mpc::VectorXd;
    VectorXd w((size_t)CMPC_NUM_WEIGHTS, 0.1), mu4(4, 0.8), mu3(3, 0.8);
    EXPECT(throws<std::invalid_argument>([&] { CentroidalMPC c(8.0, 4, 10, 0.01, w, mu3); }));
    EXPECT(throws<std::invalid_argument>([&] { CentroidalMPC c(-1.0, 4, 10, 0.01, w, mu4); }));
    CentroidalMPC mpc(8.0, 4, 10, 0.01, w, mu4);
    // reference layouts (CentroidalMPC.cpp:284-323): state 9 + 3L, des_state 9 (N + 1), des_inputs L (4N + 3) =
    // per leg [contact_enable (N) | des_foot_pos 3 x (N + 1)]
    VectorXd state(21, 0.0), des_state(9 * 11, 0.0), des_inputs(4 * (4 * 10 + 3), 0.0);
    for (int i = 0; i < 4; ++i)
      for (int k = 0; k < 10; ++k) des_inputs[(size_t)(i * 43 + k)] = (i + k) % 2;
    VectorXd x0, xref, foot;
    std::vector<uint8_t> contact;
    mpc.PackRecord(state, des_state, des_inputs, x0, xref, foot, contact);
    EXPECT((int)x0.size() == CMPC_NX && (int)contact.size() == 10 * 4 && contact[1] == 1 && contact[0] == 0);
    VectorXd short_inputs(10, 0.0);
    EXPECT(throws<std::invalid_argument>([&] { mpc.PackRecord(state, des_state, short_inputs, x0, xref, foot, contact); }));
    EXPECT(throws<std::runtime_error>([&] { (void)mpc.UpdateMPC(state, des_state, des_inputs); }));
  }

  if (fails) {
    std::fprintf(stderr, "abi_sanitize: %d check(s) failed\n", fails);
    return 1;
  }
  std::printf("abi_sanitize ok\n");
  return 0;
}
