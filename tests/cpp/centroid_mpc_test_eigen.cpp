// The CentoidMPCTest.cpp:11-116 calls written as the reference writes them — Eigen::VectorXd arguments built with
// Zero() and comma initializers (including the under-filled 54-of-63 des_state), std::make_shared<CentroidalMPC> —
// compiled against cheeta_mpc/CentroidalMPC.h with Eigen on the include path (tests/cpp/mock_eigen: this image has
// no Eigen). Prints the same lines as centroid_mpc_test.cpp (the std::vector build); the GPU test compares the two.
#include <Eigen/Dense>
#include <cstdio>
#include <memory>

#include "cheeta_mpc/CentroidalMPC.h"

static_assert(std::is_same<CentroidalMPC::VectorXd, Eigen::VectorXd>::value, "Eigen build must use Eigen::VectorXd");

int main() {
  double mass = 8;
  double time_step = 0.01;
  int num_legs = 4;
  int horizon = 6;
  Eigen::VectorXd mu = Eigen::VectorXd::Zero(num_legs);
  mu << 0.8, 0.8, 0.8, 0.8;
  Eigen::VectorXd weights = Eigen::VectorXd::Zero((num_legs + 1) * 9);
  weights << 1, 1, 100, 0.5, 0.5, 0, 2, 2, 8,  // com pos, com vel, angular momentum
      0.2, 0.2, 0.2, 0.3, 0.3, 0.3, 0.1, 0.1, 0.1, 0.2, 0.2, 0.2, 0.3, 0.3, 0.3, 0.1, 0.1, 0.1, 0.2, 0.2, 0.2, 0.3,
      0.3, 0.3, 0.1, 0.1, 0.1, 0.2, 0.2, 0.2, 0.3, 0.3, 0.3, 0.1, 0.1, 0.1;
  std::shared_ptr<CentroidalMPC> mpc = std::make_shared<CentroidalMPC>(mass, num_legs, horizon, time_step, weights, mu);
  mpc->SetupMPC();
  Eigen::VectorXd state = Eigen::VectorXd::Zero(3 * (num_legs + 3));
  Eigen::VectorXd des_state = Eigen::VectorXd::Zero(9 * (horizon + 1));
  Eigen::VectorXd des_input = Eigen::VectorXd::Zero(num_legs * (4 * horizon + 3));
  state << 0, 0, 0.15, 0.1, 0, 0, 0, 0, 0.1, 0.35, 0.052, 0, 0.35, -0.054, 0, -0.37, -0.053, 0, -0.36, 0.054, 0;
  des_state << 0.31, 0, 0.16, 0.32, 0, 0.168, 0.33, 0, 0.172, 0.33, 0, 0.18, 0.34, 0, 0.19, 0.348, 0, 0.2,  // com pos
      0.1, 0, 0, 0.09, 0, 0, 0.08, 0, 0, 0.06, 0, 0, 0.04, 0, 0, 0, 0, 0,                              // com vel
      0, 0, 0.12, 0, 0, 0.14, 0, 0, 0.16, 0, 0, 0.18, 0, 0, 0.2, 0, 0, 0.22;                          // ang mom
  Eigen::MatrixXd mpc_table = Eigen::MatrixXd::Zero(horizon, num_legs);
  mpc_table << 1, 0, 1, 0, 1, 0, 1, 0, 1, 0, 1, 0, 0, 1, 0, 1, 0, 1, 0, 1, 0, 1, 0, 1;
  Eigen::VectorXd des_foot_pos[4];
  for (auto& v : des_foot_pos) v = Eigen::VectorXd::Zero((horizon + 1) * 3);
  des_foot_pos[0] << 0.35, 0.052, 0, 0.35, 0.052, 0, 0.35, 0.052, 0, 0.35, 0.052, 0, 0.38, 0.052, 0, 0.39, 0.052, 0,
      0.42, 0.052, 0;
  des_foot_pos[1] << 0.35, -0.054, 0, 0.37, -0.052, 0, 0.39, -0.052, 0, 0.43, -0.052, 0, 0.43, -0.052, 0, 0.43,
      -0.052, 0, 0.43, -0.052, 0;
  des_foot_pos[2] << -0.37, -0.052, 0, -0.37, -0.052, 0, -0.37, -0.052, 0, -0.36, -0.052, 0, -0.34, -0.052, 0, -0.30,
      -0.052, 0, -0.28, -0.052, 0;
  des_foot_pos[3] << -0.36, 0.053, 0, -0.34, 0.053, 0, -0.32, 0.053, 0, -0.31, 0.053, 0, -0.31, 0.052, 0, -0.31,
      0.052, 0, -0.31, 0.052, 0;
  for (int i = 0; i < num_legs; ++i) {  // [contact_enable (N) | des_foot_pos 3 x (N + 1)] per leg (CentroidalMPC.cpp:315-317)
    const int base = i * (4 * horizon + 3);
    for (int k = 0; k < horizon; ++k) des_input(base + k) = mpc_table(k, i);
    for (int e = 0; e < 3 * (horizon + 1); ++e) des_input(base + horizon + e) = des_foot_pos[i](e);
  }
  const Eigen::VectorXd f = mpc->UpdateMPC(state, des_state, des_input);
  std::printf("status %d iters %d\n", mpc->lastStatus(), mpc->lastIterations());
  for (int i = 0; i < num_legs; ++i)
    for (int k = 0; k < horizon; ++k)
      std::printf("force %d %d %.17g %.17g %.17g\n", i, k, f(i * 3 * horizon + 3 * k), f(i * 3 * horizon + 3 * k + 1),
                  f(i * 3 * horizon + 3 * k + 2));
  Eigen::VectorXd state2 = state;
  state2(9 + 3 * 2) += 0.02;
  const Eigen::VectorXd f2 = mpc->UpdateMPC(state2, des_state, des_input);
  std::printf("status2 %d\n", mpc->lastStatus());
  for (int i = 0; i < num_legs; ++i)
    for (int k = 0; k < horizon; ++k)
      std::printf("force2 %d %d %.17g %.17g %.17g\n", i, k, f2(i * 3 * horizon + 3 * k),
                  f2(i * 3 * horizon + 3 * k + 1), f2(i * 3 * horizon + 3 * k + 2));
  {
    const std::vector<double>& fp = mpc->FootPositions();
    for (int i = 0; i < num_legs; ++i)
      for (int j = 0; j <= horizon; ++j)
        std::printf("foot2 %d %d %.17g %.17g %.17g\n", i, j, fp[(size_t)i * 3 * (horizon + 1) + 3 * j],
                    fp[(size_t)i * 3 * (horizon + 1) + 3 * j + 1], fp[(size_t)i * 3 * (horizon + 1) + 3 * j + 2]);
  }
  mpc->setNonlinear(true, 10, 1e-7);
  const Eigen::VectorXd f3 = mpc->UpdateMPC(state, des_state, des_input);
  std::printf("status3 %d sqp %d\n", mpc->lastStatus(), mpc->lastSqpIterations());
  for (int i = 0; i < num_legs; ++i)
    for (int k = 0; k < horizon; ++k)
      std::printf("force3 %d %d %.17g %.17g %.17g\n", i, k, f3(i * 3 * horizon + 3 * k),
                  f3(i * 3 * horizon + 3 * k + 1), f3(i * 3 * horizon + 3 * k + 2));
  {
    const std::vector<double>& fp = mpc->FootPositions();
    for (int i = 0; i < num_legs; ++i)
      for (int j = 0; j <= horizon; ++j)
        std::printf("foot3 %d %d %.17g %.17g %.17g\n", i, j, fp[(size_t)i * 3 * (horizon + 1) + 3 * j],
                    fp[(size_t)i * 3 * (horizon + 1) + 3 * j + 1], fp[(size_t)i * 3 * (horizon + 1) + 3 * j + 2]);
  }
  mpc->setNonlinear(false);
  Eigen::VectorXd bad = des_input;
  for (int i = 0; i < num_legs; ++i) bad(i * (4 * horizon + 3) + 2) = 0;
  try {
    mpc->UpdateMPC(state, des_state, bad);
    std::printf("invalid-table not detected\n");
    return 1;
  } catch (const std::runtime_error& e) {
    std::printf("caught %s\n", e.what());
  }
  std::printf("finished test\n");
  return 0;
}
