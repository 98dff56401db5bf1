// ocs2_core/misc/LinearAlgebra.h stand-in for the source-compatibility test (tests/cpp/Makefile:
// test_hpipm_interface_ocs2): the one function the HpipmInterface getters call (reference HpipmInterface.cpp:340,
// :357, :379, :419), with ocs2_core's signature — the minimum defaults to numeric_traits::weakEpsilon<scalar_t>() —
// and its rule (a diagonal entry d of the lower factor becomes max(min, d), or min(-min, d) when negative). ocs2_core
// is not vendored: the default's value here (1e-9) stands in for the real one, which an ocs2 build takes from its
// own header. The call counter lets the test see that the mirror's getters take this path.
#pragma once

#include <algorithm>

#include <ocs2_core/Types.h>

namespace ocs2 {
namespace LinearAlgebra {

inline int& mockTriangularClampCalls() {
  static int n = 0;
  return n;
}

inline void setTriangularMinimumEigenvalues(matrix_t& Lr, scalar_t minEigenValue = 1e-9) {
  ++mockTriangularClampCalls();
  for (long i = 0; i < Lr.rows(); ++i) {
    scalar_t& d = Lr(i, i);
    d = d < 0.0 ? std::min(-minEigenValue, d) : std::max(minEigenValue, d);
  }
}

}  // namespace LinearAlgebra
}  // namespace ocs2
