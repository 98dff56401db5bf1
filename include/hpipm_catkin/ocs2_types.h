/*
 * ocs2_types.h — the value types the hpipm_catkin mirror is written against.
 *
 * With ocs2_core on the include path (an ocs2 / ocs2_legged_robot build: reference HpipmInterface.h:38 includes
 * <ocs2_core/Types.h>), the real ocs2 types are used: vector_t / matrix_t are Eigen::VectorXd / Eigen::MatrixXd and
 * VectorFunctionLinearApproximation / ScalarFunctionQuadraticApproximation come from ocs2_core, so MultipleShooting-
 * Solver and testHpipmInterface compile against this header unchanged. Without it (this image has neither Eigen nor
 * ocs2_core), column-major stand-ins with the same member names are defined. The implementation
 * (cheeta-mpc_amd/host/HpipmInterface.cpp) only touches the part of the API both share — rows(), cols(), size(),
 * data(), resize(), operator() and vector operator[] — and reaches the device through the C ABI (cmpc/cmpc.h), so an
 * integrator compiles it inside the hpipm_catkin target against ocs2_core.
 * Define CMPC_OCS2_STANDIN to force the stand-ins.
 *
 * hpipm_status / hpipm_mode: from HPIPM's hpipm_common.h when it is on the include path (reference
 * HpipmInterface.h:34-36), else with HPIPM's numbering.
 */
#pragma once

#include <vector>

#if !defined(CMPC_OCS2_STANDIN) && __has_include(<ocs2_core/Types.h>)
#include <ocs2_core/Types.h>
#define CMPC_HAVE_OCS2_CORE 1
#else
namespace ocs2 {

using scalar_t = double;

class vector_t {  // Eigen::VectorXd subset (column vector, contiguous)
 public:
  vector_t() = default;
  explicit vector_t(long n) : v_((size_t)n, 0.0) {}
  long size() const { return (long)v_.size(); }
  long rows() const { return (long)v_.size(); }
  long cols() const { return 1; }
  void resize(long n) { v_.assign((size_t)n, 0.0); }
  double* data() { return v_.data(); }
  const double* data() const { return v_.data(); }
  double& operator()(long i) { return v_[(size_t)i]; }
  double operator()(long i) const { return v_[(size_t)i]; }
  double& operator[](long i) { return v_[(size_t)i]; }
  double operator[](long i) const { return v_[(size_t)i]; }

 private:
  std::vector<double> v_;
};

class matrix_t {  // Eigen::MatrixXd subset (column-major, contiguous)
 public:
  matrix_t() = default;
  matrix_t(long rows, long cols) : r_(rows), c_(cols), a_((size_t)(rows * cols), 0.0) {}
  long rows() const { return r_; }
  long cols() const { return c_; }
  long size() const { return r_ * c_; }
  void resize(long rows, long cols) {
    r_ = rows;
    c_ = cols;
    a_.assign((size_t)(rows * cols), 0.0);
  }
  double* data() { return a_.data(); }
  const double* data() const { return a_.data(); }
  double& operator()(long i, long j) { return a_[(size_t)(j * r_ + i)]; }
  double operator()(long i, long j) const { return a_[(size_t)(j * r_ + i)]; }

 private:
  long r_ = 0, c_ = 0;
  std::vector<double> a_;
};

using vector_array_t = std::vector<vector_t>;
using matrix_array_t = std::vector<matrix_t>;

struct VectorFunctionLinearApproximation {  // f(x,u) ~ f + dfdx x + dfdu u
  matrix_t dfdx, dfdu;
  vector_t f;
};

struct ScalarFunctionQuadraticApproximation {  // f + dfdx'x + dfdu'u + 1/2 x'dfdxx x + u'dfdux x + 1/2 u'dfduu u
  matrix_t dfdxx, dfduu, dfdux;
  vector_t dfdx, dfdu;
  scalar_t f = 0.0;
};

}  // namespace ocs2
#endif

#if !defined(CMPC_OCS2_STANDIN) && __has_include(<hpipm_common.h>)
extern "C" {
#include <hpipm_common.h>
}
#else
#include "cmpc/cmpc.h"
enum hpipm_status { SUCCESS = CMPC_SUCCESS, MAX_ITER = CMPC_MAX_ITER, MIN_STEP = CMPC_MIN_STEP, NAN_SOL = CMPC_NAN_SOL,
                    INCONS_EQ = CMPC_INCONS_EQ };
enum hpipm_mode { SPEED_ABS = 0, SPEED = 1, BALANCE = 2, ROBUST = 3 };
#endif
