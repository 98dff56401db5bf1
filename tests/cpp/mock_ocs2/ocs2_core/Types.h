// ocs2_core/Types.h stand-in for the source-compatibility test (tests/cpp/Makefile: test_hpipm_interface_ocs2): the
// value types as ocs2_core defines them — Eigen vectors / matrices and the linear / quadratic approximation structs
// with ocs2's member names — over the Eigen mock (tests/cpp/mock_eigen).
#pragma once

#include <Eigen/Dense>
#include <vector>

namespace ocs2 {

using scalar_t = double;
using vector_t = Eigen::VectorXd;
using matrix_t = Eigen::MatrixXd;
using vector_array_t = std::vector<vector_t>;
using matrix_array_t = std::vector<matrix_t>;

struct VectorFunctionLinearApproximation {
  vector_t f;
  matrix_t dfdx;
  matrix_t dfdu;
};

struct ScalarFunctionQuadraticApproximation {
  matrix_t dfdxx;
  matrix_t dfdux;
  matrix_t dfduu;
  vector_t dfdx;
  vector_t dfdu;
  scalar_t f = 0.0;
};

}  // namespace ocs2
