/*
 * OcpSize.h — hpipm_interface::OcpSize (reference ocs2_sqp/hpipm_catkin/include/hpipm_catkin/OcpSize.h:51-75,
 * src/OcpSize.cpp:35-75): per-node problem dimensions, N + 1 entries each, numInputs[N] = 0.
 */
#pragma once

#include <vector>

#include "hpipm_catkin/ocs2_types.h"

namespace ocs2 {
namespace hpipm_interface {

struct OcpSize {
  int numStages;
  std::vector<int> numInputs;
  std::vector<int> numStates;
  std::vector<int> numInputBoxConstraints;
  std::vector<int> numStateBoxConstraints;
  std::vector<int> numIneqConstraints;
  std::vector<int> numInputBoxSlack;
  std::vector<int> numStateBoxSlack;
  std::vector<int> numIneqSlack;
  explicit OcpSize(int N = 0, int nx = 0, int nu = 0)
      : numStages(N), numInputs(N + 1, nu), numStates(N + 1, nx), numInputBoxConstraints(N + 1, 0),
        numStateBoxConstraints(N + 1, 0), numIneqConstraints(N + 1, 0), numInputBoxSlack(N + 1, 0),
        numStateBoxSlack(N + 1, 0), numIneqSlack(N + 1, 0) {
    numInputs.back() = 0;
  }
};

bool operator==(const OcpSize& lhs, const OcpSize& rhs) noexcept;

/* Sizes from the problem data: numStates[k] = dfdx.cols() of stage k (rows of the last stage's dfdx for node N),
 * numInputs[k] = dfdu.cols(), numIneqConstraints[k] = rows of constraint k (OcpSize.cpp:49-75). */
OcpSize extractSizesFromProblem(const std::vector<VectorFunctionLinearApproximation>& dynamics,
                                const std::vector<ScalarFunctionQuadraticApproximation>& cost,
                                const std::vector<VectorFunctionLinearApproximation>* constraints);

}  // namespace hpipm_interface
}  // namespace ocs2
