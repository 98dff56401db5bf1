/*
 * HpipmInterface.h — drop-in mirror of ocs2::HpipmInterface (reference
 * ocs2_sqp/hpipm_catkin/include/hpipm_catkin/HpipmInterface.h:49-128) whose solve runs on the MI355X engine
 * (cmpc_ocp_solve_batch_host: x0 elimination, condensing and dense Cholesky on the device).
 *
 * This image has no Eigen/ocs2_core, so the ocs2 value types are provided here as minimal column-major stand-ins
 * with the members HpipmInterface touches (dfdx, dfdu, f, dfdxx, dfdux, dfduu). Eigen's default storage is
 * column-major as well, so binding the real ocs2 types is a pointer pass-through.
 */
#pragma once

#include <memory>
#include <stdexcept>
#include <vector>

#include "cmpc/cmpc.h"

namespace ocs2 {

using scalar_t = double;

struct vector_t {
  std::vector<double> v;
  vector_t() = default;
  explicit vector_t(int n) : v((size_t)n, 0.0) {}
  int size() const { return (int)v.size(); }
  int rows() const { return (int)v.size(); }
  void resize(int n) { v.assign((size_t)n, 0.0); }
  double* data() { return v.data(); }
  const double* data() const { return v.data(); }
  double& operator()(int i) { return v[(size_t)i]; }
  double operator()(int i) const { return v[(size_t)i]; }
  double& operator[](int i) { return v[(size_t)i]; }
  double operator[](int i) const { return v[(size_t)i]; }
};

struct matrix_t {  // column-major, like Eigen::MatrixXd
  int r = 0, c = 0;
  std::vector<double> a;
  matrix_t() = default;
  matrix_t(int rows, int cols) : r(rows), c(cols), a((size_t)rows * cols, 0.0) {}
  int rows() const { return r; }
  int cols() const { return c; }
  void resize(int rows, int cols) {
    r = rows;
    c = cols;
    a.assign((size_t)rows * cols, 0.0);
  }
  double* data() { return a.data(); }
  const double* data() const { return a.data(); }
  double& operator()(int i, int j) { return a[(size_t)j * r + i]; }
  double operator()(int i, int j) const { return a[(size_t)j * r + i]; }
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

enum hpipm_status { SUCCESS = CMPC_SUCCESS, MAX_ITER = CMPC_MAX_ITER, MIN_STEP = CMPC_MIN_STEP, NAN_SOL = CMPC_NAN_SOL,
                    INCONS_EQ = CMPC_INCONS_EQ };
enum hpipm_mode { SPEED_ABS = 0, SPEED = 1, BALANCE = 2, ROBUST = 3 };

namespace ocs2 {
namespace hpipm_interface {

/* reference OcpSize.h:51-75 */
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
OcpSize extractSizesFromProblem(const std::vector<VectorFunctionLinearApproximation>& dynamics,
                                const std::vector<ScalarFunctionQuadraticApproximation>& cost,
                                const std::vector<VectorFunctionLinearApproximation>* constraints);

/* reference HpipmInterfaceSettings.h:44-57 */
struct Settings {
  hpipm_mode hpipmMode = hpipm_mode::SPEED;
  int iter_max = 30;
  scalar_t alpha_min = 1e-12;
  scalar_t mu0 = 1e1;
  scalar_t tol_stat = 1e-6;
  scalar_t tol_eq = 1e-8;
  scalar_t tol_ineq = 1e-8;
  scalar_t tol_comp = 1e-8;
  scalar_t reg_prim = 1e-12;
  int warm_start = 0;
  int pred_corr = 1;
  int ric_alg = 0;
};

}  // namespace hpipm_interface

class HpipmInterface {
 public:
  using OcpSize = hpipm_interface::OcpSize;
  using Settings = hpipm_interface::Settings;

  explicit HpipmInterface(OcpSize ocpSize = OcpSize(), const Settings& settings = Settings());
  ~HpipmInterface();
  void resize(OcpSize ocpSize);
  /* Solved on the device. constraints == nullptr: equality-free stages (cmpc_ocp_solve_batch_host); otherwise the
   * rows C dx + D du + e = 0 are imposed as the reference's lg = ug rows (HpipmInterface.cpp:223-264) by
   * cmpc_ocp_solve_batch_eq_host (x0-eliminated stage 0, redundant rows dropped, inconsistent rows -> INCONS_EQ). */
  hpipm_status solve(const vector_t& x0, std::vector<VectorFunctionLinearApproximation>& dynamics,
                     std::vector<ScalarFunctionQuadraticApproximation>& cost,
                     std::vector<VectorFunctionLinearApproximation>* constraints, vector_array_t& stateTrajectory,
                     vector_array_t& inputTrajectory, bool verbose = false);

  /* Riccati quantities of the previously solved problem (reference HpipmInterface.h:93-123, .cpp:330-455), from the
   * device recursion cmpc_ocp_riccati_batch_host. The reference rebuilds stage 0 from (dynamics0, cost0) because
   * HPIPM eliminates x0; the recursion here runs over stage 0 directly, so the arguments are accepted and must equal
   * the stage-0 data of the last solve (size-checked). Cost-to-go f is 0, as in the reference. */
  std::vector<ScalarFunctionQuadraticApproximation> getRiccatiCostToGo(const VectorFunctionLinearApproximation& dynamics0,
                                                                       const ScalarFunctionQuadraticApproximation& cost0);
  matrix_array_t getRiccatiFeedback(const VectorFunctionLinearApproximation& dynamics0,
                                    const ScalarFunctionQuadraticApproximation& cost0);
  vector_array_t getRiccatiFeedforward(const VectorFunctionLinearApproximation& dynamics0,
                                       const ScalarFunctionQuadraticApproximation& cost0);

 private:
  class Impl;
  std::unique_ptr<Impl> pImpl_;
};

}  // namespace ocs2
