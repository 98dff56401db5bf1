// C++ driver equivalent of the reference CentoidMPCTest.cpp:11-116 on the MI355X engine (CentroidalMPC mirror).
// Same model, weights, state, des_state (including the test's under-filled 54-of-63 layout), contact table and
// desired foot positions; prints the contact forces UpdateMPC returns (leg-major 3 x N blocks) for the pytest.
#include <cstdio>
#include <vector>

#include "cheeta_mpc/CentroidalMPC.h"

int main() {
  const double mass = 8, time_step = 0.01;
  const int num_legs = 4, horizon = 6;
  std::vector<double> mu = {0.8, 0.8, 0.8, 0.8};
  std::vector<double> weights = {1,   1,   100, 0.5, 0.5, 0,   2,   2,   8,   0.2, 0.2, 0.2, 0.3, 0.3, 0.3,
                                 0.1, 0.1, 0.1, 0.2, 0.2, 0.2, 0.3, 0.3, 0.3, 0.1, 0.1, 0.1, 0.2, 0.2, 0.2,
                                 0.3, 0.3, 0.3, 0.1, 0.1, 0.1, 0.2, 0.2, 0.2, 0.3, 0.3, 0.3, 0.1, 0.1, 0.1};
  CentroidalMPC mpc(mass, num_legs, horizon, time_step, weights, mu);
  mpc.SetupMPC();
  std::vector<double> state = {0, 0, 0.15, 0.1, 0, 0, 0, 0, 0.1, 0.35, 0.052, 0, 0.35, -0.054, 0,
                               -0.37, -0.053, 0, -0.36, 0.054, 0};
  std::vector<double> des_state(9 * (horizon + 1), 0.0);
  const double ds[] = {0.31, 0, 0.16, 0.32, 0, 0.168, 0.33, 0, 0.172, 0.33, 0, 0.18, 0.34, 0, 0.19, 0.348, 0, 0.2,
                       0.1,  0, 0,    0.09, 0, 0,     0.08, 0, 0,     0.06, 0, 0,    0.04, 0, 0,    0,     0, 0,
                       0,    0, 0.12, 0,    0, 0.14,  0,    0, 0.16,  0,    0, 0.18, 0,    0, 0.2,  0,     0, 0.22};
  for (int i = 0; i < 54; ++i) des_state[(size_t)i] = ds[i];
  const int table[6][4] = {{1, 0, 1, 0}, {1, 0, 1, 0}, {1, 0, 1, 0}, {0, 1, 0, 1}, {0, 1, 0, 1}, {0, 1, 0, 1}};
  const double feet[4][7][3] = {
      {{0.35, 0.052, 0}, {0.35, 0.052, 0}, {0.35, 0.052, 0}, {0.35, 0.052, 0}, {0.38, 0.052, 0}, {0.39, 0.052, 0},
       {0.42, 0.052, 0}},
      {{0.35, -0.054, 0}, {0.37, -0.052, 0}, {0.39, -0.052, 0}, {0.43, -0.052, 0}, {0.43, -0.052, 0},
       {0.43, -0.052, 0}, {0.43, -0.052, 0}},
      {{-0.37, -0.052, 0}, {-0.37, -0.052, 0}, {-0.37, -0.052, 0}, {-0.36, -0.052, 0}, {-0.34, -0.052, 0},
       {-0.30, -0.052, 0}, {-0.28, -0.052, 0}},
      {{-0.36, 0.053, 0}, {-0.34, 0.053, 0}, {-0.32, 0.053, 0}, {-0.31, 0.053, 0}, {-0.31, 0.052, 0},
       {-0.31, 0.052, 0}, {-0.31, 0.052, 0}}};
  std::vector<double> des_input((size_t)num_legs * (4 * horizon + 3), 0.0);
  for (int i = 0; i < num_legs; ++i) {
    const size_t base = (size_t)i * (4 * horizon + 3);
    for (int k = 0; k < horizon; ++k) des_input[base + k] = table[k][i];
    for (int k = 0; k <= horizon; ++k)
      for (int d = 0; d < 3; ++d) des_input[base + horizon + 3 * k + d] = feet[i][k][d];
  }
  const std::vector<double> f = mpc.UpdateMPC(state, des_state, des_input);
  std::printf("status %d iters %d\n", mpc.lastStatus(), mpc.lastIterations());
  for (int i = 0; i < num_legs; ++i)
    for (int k = 0; k < horizon; ++k)
      std::printf("force %d %d %.17g %.17g %.17g\n", i, k, f[(size_t)i * 3 * horizon + 3 * k],
                  f[(size_t)i * 3 * horizon + 3 * k + 1], f[(size_t)i * 3 * horizon + 3 * k + 2]);
  // the current foot positions state[9..20] are an input (CentroidalMPC.cpp:288-291, pinned as foot_pos(:,0) by
  // :165-167): move the rh foot (leg 2, in stance from step 0) 2 cm forward
  std::vector<double> state2 = state;
  state2[9 + 3 * 2] += 0.02;
  const std::vector<double> f2 = mpc.UpdateMPC(state2, des_state, des_input);
  std::printf("status2 %d\n", mpc.lastStatus());
  for (int i = 0; i < num_legs; ++i)
    for (int k = 0; k < horizon; ++k)
      std::printf("force2 %d %d %.17g %.17g %.17g\n", i, k, f2[(size_t)i * 3 * horizon + 3 * k],
                  f2[(size_t)i * 3 * horizon + 3 * k + 1], f2[(size_t)i * 3 * horizon + 3 * k + 2]);
  // foot_pos output of the QP mode (frozen later-run footholds), then the reference's NLP with the later runs'
  // footholds as decision variables (setNonlinear, cmpc_nlp_solve_batch)
  {
    const std::vector<double>& fp = mpc.FootPositions();
    for (int i = 0; i < num_legs; ++i)
      for (int j = 0; j <= horizon; ++j)
        std::printf("foot2 %d %d %.17g %.17g %.17g\n", i, j, fp[(size_t)i * 3 * (horizon + 1) + 3 * j],
                    fp[(size_t)i * 3 * (horizon + 1) + 3 * j + 1], fp[(size_t)i * 3 * (horizon + 1) + 3 * j + 2]);
  }
  mpc.setNonlinear(true, 10, 1e-7);
  const std::vector<double> f3 = mpc.UpdateMPC(state, des_state, des_input);
  std::printf("status3 %d sqp %d\n", mpc.lastStatus(), mpc.lastSqpIterations());
  for (int i = 0; i < num_legs; ++i)
    for (int k = 0; k < horizon; ++k)
      std::printf("force3 %d %d %.17g %.17g %.17g\n", i, k, f3[(size_t)(i * 3 * horizon + 3 * k)],
                  f3[(size_t)(i * 3 * horizon + 3 * k + 1)], f3[(size_t)(i * 3 * horizon + 3 * k + 2)]);
  {
    const std::vector<double>& fp = mpc.FootPositions();
    for (int i = 0; i < num_legs; ++i)
      for (int j = 0; j <= horizon; ++j)
        std::printf("foot3 %d %d %.17g %.17g %.17g\n", i, j, fp[(size_t)i * 3 * (horizon + 1) + 3 * j],
                    fp[(size_t)i * 3 * (horizon + 1) + 3 * j + 1], fp[(size_t)i * 3 * (horizon + 1) + 3 * j + 2]);
  }
  mpc.setNonlinear(false);
  // "mpc table invalid" (CentroidalMPC.cpp:328-330)
  std::vector<double> bad = des_input;
  for (int i = 0; i < num_legs; ++i) bad[(size_t)i * (4 * horizon + 3) + 2] = 0;
  try {
    mpc.UpdateMPC(state, des_state, bad);
    std::printf("invalid-table not detected\n");
    return 1;
  } catch (const std::runtime_error& e) {
    std::printf("caught %s\n", e.what());
  }
  std::printf("finished test\n");
  return 0;
}
