// HpipmInterface.cpp — ocs2::HpipmInterface mirror (reference HpipmInterface.cpp:86-554) on the MI355X engine.
#include "hpipm_catkin/HpipmInterface.h"

#include <cmath>
#include <cstdio>
#include <string>

namespace ocs2 {
namespace hpipm_interface {

bool operator==(const OcpSize& l, const OcpSize& r) noexcept {  // OcpSize.cpp:35-47
  return l.numStages == r.numStages && l.numInputs == r.numInputs && l.numStates == r.numStates &&
         l.numInputBoxConstraints == r.numInputBoxConstraints && l.numStateBoxConstraints == r.numStateBoxConstraints &&
         l.numIneqConstraints == r.numIneqConstraints && l.numInputBoxSlack == r.numInputBoxSlack &&
         l.numStateBoxSlack == r.numStateBoxSlack && l.numIneqSlack == r.numIneqSlack;
}

OcpSize extractSizesFromProblem(const std::vector<VectorFunctionLinearApproximation>& dynamics,
                                const std::vector<ScalarFunctionQuadraticApproximation>& cost,
                                const std::vector<VectorFunctionLinearApproximation>* constraints) {
  (void)cost;  // OcpSize.cpp:49-75
  const int N = (int)dynamics.size();
  OcpSize s(N);
  for (int k = 0; k < N; ++k) {
    s.numStates[(size_t)k] = dynamics[(size_t)k].dfdx.cols();
    s.numInputs[(size_t)k] = dynamics[(size_t)k].dfdu.cols();
  }
  s.numStates[(size_t)N] = N > 0 ? dynamics[(size_t)N - 1].dfdx.rows() : 0;
  s.numInputs[(size_t)N] = 0;
  if (constraints)
    for (int k = 0; k <= N; ++k) s.numIneqConstraints[(size_t)k] = (*constraints)[(size_t)k].f.size();
  return s;
}

}  // namespace hpipm_interface

class HpipmInterface::Impl {
 public:
  Impl(OcpSize s, Settings st) : settings_(st) { initializeMemory(std::move(s)); }
  void initializeMemory(OcpSize s) {
    s.numStates[0] = 0;  // x0 eliminated (HpipmInterface.cpp:93-95)
    size_ = std::move(s);
  }
  hpipm_status solve(const vector_t& x0, std::vector<VectorFunctionLinearApproximation>& dyn,
                     std::vector<ScalarFunctionQuadraticApproximation>& cost,
                     std::vector<VectorFunctionLinearApproximation>* constraints, vector_array_t& xs, vector_array_t& us,
                     bool verbose) {
    const int N = size_.numStages;
    // verifySizes (HpipmInterface.cpp:146-164)
    if ((int)dyn.size() != N)
      throw std::runtime_error("[HpipmInterface] Inconsistent size of dynamics: " + std::to_string(dyn.size()) +
                               " with " + std::to_string(N) + " number of stages.");
    if ((int)cost.size() != N + 1)
      throw std::runtime_error("[HpipmInterface] Inconsistent size of cost: " + std::to_string(cost.size()) + " with " +
                               std::to_string(N + 1) + " nodes.");
    if (constraints != nullptr && (int)constraints->size() != N + 1)
      throw std::runtime_error("[HpipmInterface] Inconsistent size of constraints: " +
                               std::to_string(constraints->size()) + " with " + std::to_string(N + 1) + " nodes.");
    const int nx = x0.size();
    std::vector<int> nu((size_t)N);
    for (int k = 0; k < N; ++k) {
      nu[(size_t)k] = dyn[(size_t)k].dfdu.cols();
      if (dyn[(size_t)k].dfdx.rows() != nx || dyn[(size_t)k].dfdx.cols() != nx)
        throw std::runtime_error("[HpipmInterface] constant state dimension required");
    }
    const size_t rs = cmpc_ocp_record_size(N, nx, nu.data());
    std::vector<double> rec(rs);
    size_t o = 0;
    auto put = [&](const double* p, size_t n) {
      for (size_t i = 0; i < n; ++i) rec[o + i] = p ? p[i] : 0.0;
      o += n;
    };
    for (int k = 0; k < N; ++k) {
      const auto& d = dyn[(size_t)k];
      put(d.dfdx.data(), (size_t)nx * nx);
      put(d.dfdu.data(), (size_t)nx * nu[(size_t)k]);
      put(d.f.data(), (size_t)nx);
    }
    for (int k = 0; k <= N; ++k) {
      const auto& c = cost[(size_t)k];
      const size_t m = k < N ? (size_t)nu[(size_t)k] : 0;
      put(c.dfdxx.data(), (size_t)nx * nx);
      put(m ? c.dfdux.data() : nullptr, m * nx);
      put(m ? c.dfduu.data() : nullptr, m * m);
      put(c.dfdx.data(), (size_t)nx);
      put(m ? c.dfdu.data() : nullptr, m);
    }
    int nU = 0;
    for (int v : nu) nU += v;
    // === Constraints === C dx + D du + e = 0 per node, handed to the device as they come (the reference maps them to
    // HPIPM's lg = ug = -e, with the stage-0 rows bounded through x0, HpipmInterface.cpp:223-264); an empty node
    // (f.size() == 0) has no rows
    std::vector<int> nc((size_t)N + 1, 0);
    std::vector<double> crec;
    int nE = 0;
    if (constraints != nullptr) {
      for (int k = 0; k <= N; ++k) {
        const auto& c = (*constraints)[(size_t)k];
        const int rows = c.f.size();
        const int m = k < N ? nu[(size_t)k] : 0;
        if (rows == 0) continue;
        if (c.dfdx.rows() != rows || c.dfdx.cols() != nx || (m > 0 && (c.dfdu.rows() != rows || c.dfdu.cols() != m)))
          throw std::runtime_error("[HpipmInterface] constraint " + std::to_string(k) + " has inconsistent sizes");
        nc[(size_t)k] = rows;
        nE += rows;
        crec.insert(crec.end(), c.dfdx.a.begin(), c.dfdx.a.end());
        if (m > 0) crec.insert(crec.end(), c.dfdu.a.begin(), c.dfdu.a.end());
        crec.insert(crec.end(), c.f.v.begin(), c.f.v.end());
      }
    }
    std::vector<double> x((size_t)(N + 1) * nx), u((size_t)(nU > 0 ? nU : 1));
    int status = -1;
    const int r = nE > 0 ? cmpc_ocp_solve_batch_eq_host(1, N, nx, nu.data(), nc.data(), x0.data(), rec.data(),
                                                         crec.data(), x.data(), u.data(), &status)
                         : cmpc_ocp_solve_batch_host(1, N, nx, nu.data(), x0.data(), rec.data(), x.data(), u.data(),
                                                     &status);
    if (r != CMPC_OK) throw std::runtime_error(std::string("[HpipmInterface] device solve failed: ") + cmpc_error_string(r));
    xs.assign((size_t)N + 1, vector_t());
    for (int k = 0; k <= N; ++k) {
      xs[(size_t)k].resize(nx);
      for (int i = 0; i < nx; ++i) xs[(size_t)k][i] = k == 0 ? x0[i] : x[(size_t)k * nx + i];
    }
    us.assign((size_t)N, vector_t());
    int off = 0;
    for (int k = 0; k < N; ++k) {
      us[(size_t)k].resize(nu[(size_t)k]);
      for (int i = 0; i < nu[(size_t)k]; ++i) us[(size_t)k][i] = u[(size_t)off + i];
      off += nu[(size_t)k];
    }
    if (verbose) std::fprintf(stderr, "\n=== HPIPM (MI355X engine) ===\nstatus %d (%s)\n", status, cmpc_status_string(status));
    lastRec_ = std::move(rec);
    lastNu_ = nu;
    lastNx_ = nx;
    lastConstrained_ = nE > 0;
    riccatiValid_ = false;
    return (hpipm_status)status;
  }

  // Device Riccati recursion over the last problem, computed once per solve on first use.
  void riccati(const VectorFunctionLinearApproximation& dyn0, const ScalarFunctionQuadraticApproximation& cost0) {
    const int N = (int)lastNu_.size();
    if (N == 0) throw std::runtime_error("[HpipmInterface] no solved problem to take Riccati quantities from");
    if (dyn0.dfdx.rows() != lastNx_ || dyn0.dfdu.cols() != lastNu_[0] || cost0.dfdxx.rows() != lastNx_)
      throw std::runtime_error("[HpipmInterface] dynamics0 / cost0 do not match the last solved problem");
    if (lastConstrained_)
      throw std::runtime_error(
          "[HpipmInterface] Riccati quantities of an equality-constrained solve are not provided by this build");
    if (riccatiValid_) return;
    const int nx = lastNx_;
    int nU = 0;
    for (int v : lastNu_) nU += v;
    Sm_.assign((size_t)(N + 1) * nx * nx, 0.0);
    sv_.assign((size_t)(N + 1) * nx, 0.0);
    K_.assign((size_t)(nU > 0 ? nU : 1) * nx, 0.0);
    k_.assign((size_t)(nU > 0 ? nU : 1), 0.0);
    int st = -1;
    const int r = cmpc_ocp_riccati_batch_host(1, N, nx, lastNu_.data(), lastRec_.data(), Sm_.data(), sv_.data(),
                                              K_.data(), k_.data(), &st);
    if (r != CMPC_OK) throw std::runtime_error(std::string("[HpipmInterface] device Riccati failed: ") + cmpc_error_string(r));
    if (st != CMPC_SUCCESS) throw std::runtime_error("[HpipmInterface] Riccati recursion: R + B'PB not positive definite");
    riccatiValid_ = true;
  }
  std::vector<ScalarFunctionQuadraticApproximation> costToGo(const VectorFunctionLinearApproximation& d0,
                                                              const ScalarFunctionQuadraticApproximation& c0) {
    riccati(d0, c0);
    const int N = (int)lastNu_.size(), nx = lastNx_;
    std::vector<ScalarFunctionQuadraticApproximation> out((size_t)N + 1);
    for (int k = 0; k <= N; ++k) {
      out[(size_t)k].dfdxx.resize(nx, nx);
      out[(size_t)k].dfdx.resize(nx);
      for (int e = 0; e < nx * nx; ++e) out[(size_t)k].dfdxx.a[(size_t)e] = Sm_[(size_t)k * nx * nx + e];
      for (int i = 0; i < nx; ++i) out[(size_t)k].dfdx[i] = sv_[(size_t)k * nx + i];
      out[(size_t)k].f = 0.0;
    }
    return out;
  }
  matrix_array_t feedback(const VectorFunctionLinearApproximation& d0, const ScalarFunctionQuadraticApproximation& c0) {
    riccati(d0, c0);
    const int N = (int)lastNu_.size(), nx = lastNx_;
    matrix_array_t out((size_t)N);
    size_t o = 0;
    for (int k = 0; k < N; ++k) {
      const int m = lastNu_[(size_t)k];
      out[(size_t)k].resize(m, nx);
      for (int e = 0; e < m * nx; ++e) out[(size_t)k].a[(size_t)e] = K_[o + (size_t)e];
      o += (size_t)m * nx;
    }
    return out;
  }
  vector_array_t feedforward(const VectorFunctionLinearApproximation& d0, const ScalarFunctionQuadraticApproximation& c0) {
    riccati(d0, c0);
    const int N = (int)lastNu_.size();
    vector_array_t out((size_t)N);
    size_t o = 0;
    for (int k = 0; k < N; ++k) {
      const int m = lastNu_[(size_t)k];
      out[(size_t)k].resize(m);
      for (int i = 0; i < m; ++i) out[(size_t)k][i] = k_[o + (size_t)i];
      o += (size_t)m;
    }
    return out;
  }

 private:
  Settings settings_;
  OcpSize size_;
  std::vector<double> lastRec_;
  std::vector<int> lastNu_;
  int lastNx_ = 0;
  bool lastConstrained_ = false;
  bool riccatiValid_ = false;
  std::vector<double> Sm_, sv_, K_, k_;
};

HpipmInterface::HpipmInterface(OcpSize s, const Settings& st) : pImpl_(new Impl(std::move(s), st)) {}
HpipmInterface::~HpipmInterface() = default;
void HpipmInterface::resize(OcpSize s) { pImpl_->initializeMemory(std::move(s)); }
hpipm_status HpipmInterface::solve(const vector_t& x0, std::vector<VectorFunctionLinearApproximation>& dynamics,
                                   std::vector<ScalarFunctionQuadraticApproximation>& cost,
                                   std::vector<VectorFunctionLinearApproximation>* constraints, vector_array_t& x,
                                   vector_array_t& u, bool verbose) {
  return pImpl_->solve(x0, dynamics, cost, constraints, x, u, verbose);
}
std::vector<ScalarFunctionQuadraticApproximation> HpipmInterface::getRiccatiCostToGo(
    const VectorFunctionLinearApproximation& dynamics0, const ScalarFunctionQuadraticApproximation& cost0) {
  return pImpl_->costToGo(dynamics0, cost0);
}
matrix_array_t HpipmInterface::getRiccatiFeedback(const VectorFunctionLinearApproximation& dynamics0,
                                                  const ScalarFunctionQuadraticApproximation& cost0) {
  return pImpl_->feedback(dynamics0, cost0);
}
vector_array_t HpipmInterface::getRiccatiFeedforward(const VectorFunctionLinearApproximation& dynamics0,
                                                     const ScalarFunctionQuadraticApproximation& cost0) {
  return pImpl_->feedforward(dynamics0, cost0);
}

}  // namespace ocs2
