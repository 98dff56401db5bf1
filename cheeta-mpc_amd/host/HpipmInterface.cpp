// HpipmInterface.cpp — ocs2::HpipmInterface mirror (reference HpipmInterface.cpp:86-554) on the MI355X engine: the
// Impl owns a cmpc_ocp handle (device dimensions, settings and memory) created once; resize re-lays it out for the new
// sizes with grow-only buffers (cmpc_ocp_reshape), as the reference's MemoryBlock::reserve grows HPIPM's memory only
// (:46-67, :92-129). solve packs the problem straight into the handle's pinned staging and runs cmpc_ocp_solve_host
// (one copy in, the stage-wise interior-point kernel, one copy back); the solve also leaves the Riccati quantities of
// its exit point (cmpc_ocp_set_keep_riccati), so the getters copy them (HPIPM's read its workspace, :336-360).
//
// Written against the API the real ocs2 / Eigen types and the stand-ins of ocs2_types.h share (rows(), cols(),
// size(), data(), resize(), operator()), so an ocs2 build compiles this file inside its hpipm_catkin target against
// ocs2_core; the device is reached only through the C ABI (cmpc/cmpc.h).
#include "hpipm_catkin/HpipmInterface.h"

#ifdef CMPC_HAVE_OCS2_CORE
#include <ocs2_core/misc/LinearAlgebra.h>  // the reference's clamp (HpipmInterface.cpp:32), with ocs2_core's default
#endif

#include <algorithm>
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
    s.numStates[(size_t)k] = (int)dynamics[(size_t)k].dfdx.cols();
    s.numInputs[(size_t)k] = (int)dynamics[(size_t)k].dfdu.cols();
  }
  s.numStates[(size_t)N] = N > 0 ? (int)dynamics[(size_t)N - 1].dfdx.rows() : 0;
  s.numInputs[(size_t)N] = 0;
  if (constraints)
    for (int k = 0; k <= N; ++k) s.numIneqConstraints[(size_t)k] = (int)(*constraints)[(size_t)k].f.size();
  return s;
}

std::ostream& operator<<(std::ostream& stream, const Settings& s) {  // HpipmInterfaceSettings.cpp
  const Settings d;
  auto line = [&](const char* name, double v, bool changed) {
    stream << " #### '" << name << "'" << std::string(name[0] ? 20 - std::min<size_t>(20, std::string(name).size()) : 0, '.')
           << " " << v << (changed ? "" : "\t(default)") << "\n";
  };
  stream << "\n #### HPIPM Settings:";
  stream << "\n #### =============================================================================\n";
  line("mode", (double)s.hpipmMode, s.hpipmMode != d.hpipmMode);
  line("iter_max", s.iter_max, s.iter_max != d.iter_max);
  line("alpha_min", s.alpha_min, s.alpha_min != d.alpha_min);
  line("mu0", s.mu0, s.mu0 != d.mu0);
  line("tol_stat", s.tol_stat, s.tol_stat != d.tol_stat);
  line("tol_eq", s.tol_eq, s.tol_eq != d.tol_eq);
  line("tol_ineq", s.tol_ineq, s.tol_ineq != d.tol_ineq);
  line("tol_comp", s.tol_comp, s.tol_comp != d.tol_comp);
  line("reg_prim", s.reg_prim, s.reg_prim != d.reg_prim);
  line("warm_start", s.warm_start, s.warm_start != d.warm_start);
  line("pred_corr", s.pred_corr, s.pred_corr != d.pred_corr);
  line("ric_alg", s.ric_alg, s.ric_alg != d.ric_alg);
  stream << " #### =============================================================================" << std::endl;
  return stream;
}

}  // namespace hpipm_interface

namespace {

// one problem in the engine's packed forms (cmpc.h: OCP record [A,B,b] per stage then [Q,S,R,q,r] per node;
// constraint record [C,D,e] per node with rows), column-major blocks as Eigen stores them
struct Packed {
  int N = 0, nx = 0;        // nx: the padded state dimension, max over the nodes
  std::vector<int> nxk;     // the problem's own state dimension per node (OcpSize::numStates)
  std::vector<int> nu, nc;
};

}  // namespace

class HpipmInterface::Impl {
 public:
  Impl(OcpSize s, Settings st) : settings_(st) { initializeMemory(std::move(s), true); }
  ~Impl() { release(); }

  // HpipmInterface.cpp:92-129: x0 is eliminated (numStates[0] = 0); on a size change (:97-100) the device handle is
  // re-laid out (cmpc_ocp_reshape: one small upload, buffers reallocated only beyond their capacity) or, the first
  // time, created
  void initializeMemory(OcpSize s, bool force = false) {
    s.numStates[0] = 0;
    if (!force && s == size_) return;
    size_ = std::move(s);
    const int N = size_.numStages;
    if (N <= 0) return;
    int nx = 0;
    for (int k = 1; k <= N; ++k) nx = std::max(nx, size_.numStates[(size_t)k]);
    std::vector<int> nc(size_.numIneqConstraints.begin(), size_.numIneqConstraints.end());
    // without a visible device the handle is left to the first solve(), which then reports it (the host-side size
    // checks and record packing stay usable, as the reference's are without a solve)
    shape(N, nx, std::vector<int>(size_.numInputs.begin(), size_.numInputs.begin() + N), nc, /*defer_no_device=*/true);
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
    Packed& p = last_;
    sizes(p, x0, dyn, cost, constraints);
    // the handle must have the problem's dimensions: node 0's state (x0.size()) may exceed numStates[1..N], and rows
    // passed for nodes the size has none for (or without rows where it has some) re-shape it, as a resize would
    const std::vector<int>& nc = p.nc;
    if (!ocp_ || ocpN_ != N || ocpNx_ != p.nx || ocpNu_ != p.nu || ocpNc_ != nc) shape(N, p.nx, p.nu, nc);
    const int nx = p.nx;
    int nU = 0, m = 0;
    for (int v : p.nu) nU += v;
    for (int v : nc) m += v;
    // the records go straight into the handle's pinned staging (host buffers when it has none)
    const size_t rs = cmpc_ocp_record_size(N, nx, p.nu.data());
    double* rec = cmpc_ocp_staging(ocp_, CMPC_OCP_STAGE_REC);
    double* crec = m > 0 ? cmpc_ocp_staging(ocp_, CMPC_OCP_STAGE_CREC) : nullptr;
    double* x0p = cmpc_ocp_staging(ocp_, CMPC_OCP_STAGE_X0);
    if (!rec) {
      recbuf_.assign(rs, 0.0);
      rec = recbuf_.data();
    }
    if (m > 0 && !crec) {
      crecbuf_.assign(cmpc_ocp_constraint_record_size(N, nx, p.nu.data(), nc.data()), 0.0);
      crec = crecbuf_.data();
    }
    if (!x0p) {
      x0buf_.assign((size_t)nx, 0.0);
      x0p = x0buf_.data();
    }
    fill(p, dyn, cost, constraints, rec, crec);
    for (int i = 0; i < nx; ++i) x0p[i] = i < p.nxk[0] ? x0(i) : 0.0;
    // with Settings::warm_start the last solution of the same size is the initial guess (HPIPM keeps it in qp_sol)
    if (!settings_.warm_start || xbuf_.size() != (size_t)(N + 1) * nx) xbuf_.assign((size_t)(N + 1) * nx, 0.0);
    if (!settings_.warm_start || ubuf_.size() != (size_t)(nU > 0 ? nU : 1)) ubuf_.assign((size_t)(nU > 0 ? nU : 1), 0.0);
    int status = -1, iters = 0;
    // the verbose table's lin res columns: the device records the Newton systems' residuals for this solve only
    if (cmpc_ocp_set_linres(ocp_, verbose ? 1 : 0) != CMPC_OK)
      throw std::runtime_error("[HpipmInterface] cannot record the statistics");
    const int r = cmpc_ocp_solve_host(ocp_, 1, x0p, rec, crec, xbuf_.data(), ubuf_.data(), &status, &iters);
    if (r != CMPC_OK) throw std::runtime_error(std::string("[HpipmInterface] device solve failed: ") + cmpc_error_string(r));
    // getStateSolution / getInputSolution (:303-328): x[0] = x0, each node in its own dimension; non-finite -> NAN_SOL
    bool finite = true;
    xs.assign((size_t)N + 1, vector_t());
    for (int k = 0; k <= N; ++k) {
      const int xk = p.nxk[(size_t)k];
      xs[(size_t)k].resize(xk);
      for (int i = 0; i < xk; ++i) {
        xs[(size_t)k](i) = k == 0 ? x0(i) : xbuf_[(size_t)k * nx + i];
        finite = finite && std::isfinite(xs[(size_t)k](i));
      }
    }
    us.assign((size_t)N, vector_t());
    int off = 0;
    for (int k = 0; k < N; ++k) {
      us[(size_t)k].resize(p.nu[(size_t)k]);
      for (int i = 0; i < p.nu[(size_t)k]; ++i) {
        us[(size_t)k](i) = ubuf_[(size_t)off + i];
        finite = finite && std::isfinite(us[(size_t)k](i));
      }
      off += p.nu[(size_t)k];
    }
    if (verbose) printStatus(status, iters);
    riccatiValid_ = false;
    ricFb_ = false;
    if (!finite) return hpipm_status::NAN_SOL;
    return (hpipm_status)status;
  }

  // Riccati quantities of the last solve (cmpc_ocp_riccati: factorisation at the returned point), fetched once per
  // solve; stage 0 rebuilt from (dynamics0, cost0) as the reference does (HpipmInterface.cpp:334-347, 376-389, 416-453).
  // all = false (getRiccatiFeedback, the MPC's per-tick call): K, Lr and P_1 only (cmpc_ocp_riccati_feedback_host,
  // copies of what the solve kept); all = true: every quantity (cmpc_ocp_riccati_host).
  void riccati(const VectorFunctionLinearApproximation& dyn0, const ScalarFunctionQuadraticApproximation& cost0,
               bool all) {
    const Packed& p = last_;
    const int N = p.N;
    if (N == 0 || !ocp_) throw std::runtime_error("[HpipmInterface] no solved problem to take Riccati quantities from");
    if ((int)dyn0.dfdx.rows() != p.nxk[1] || (int)dyn0.dfdx.cols() != p.nxk[0] || (int)dyn0.dfdu.cols() != p.nu[0] ||
        (int)cost0.dfdxx.rows() != p.nxk[0])
      throw std::runtime_error("[HpipmInterface] dynamics0 / cost0 do not match the last solved problem");
    if (!riccatiValid_ && !(ricFb_ && !all)) {
      const int nx = p.nx;
      int nU = 0, nK = 0, nM = 0;
      for (int v : p.nu) {
        nU += v;
        nK += v * nx;
        nM += v * v;
      }
      Pm_.assign((size_t)(N + 1) * nx * nx, 0.0);
      pv_.assign((size_t)(N + 1) * nx, 0.0);
      K_.assign((size_t)(nK > 0 ? nK : 1), 0.0);
      k_.assign((size_t)(nU > 0 ? nU : 1), 0.0);
      Lr_.assign((size_t)(nM > 0 ? nM : 1), 0.0);
      int st = -1;
      const int r = all ? cmpc_ocp_riccati_host(ocp_, 1, Pm_.data(), pv_.data(), K_.data(), k_.data(), Lr_.data(), &st)
                        : cmpc_ocp_riccati_feedback_host(ocp_, 0, K_.data(), Lr_.data(), Pm_.data() + (size_t)nx * nx,
                                                         &st);
      if (r != CMPC_OK)
        throw std::runtime_error(std::string("[HpipmInterface] device Riccati failed: ") + cmpc_error_string(r));
      if (st != CMPC_SUCCESS) throw std::runtime_error("[HpipmInterface] Riccati factorisation: NaN pivot");
      if (clampActive()) clampFactors(nx);
      if (all) riccatiValid_ = true;
      ricFb_ = true;
    }
    stage0(dyn0, cost0, all || riccatiValid_);
  }

  int allocations() const { return ocp_ ? cmpc_ocp_alloc_count(ocp_) : -1; }
  void setKeep(bool on) {
    keep_ = on;
    if (ocp_) (void)cmpc_ocp_set_keep_riccati(ocp_, on ? 1 : 0);
  }
  void enableTiming(bool on) {
    timing_ = on;
    if (ocp_) (void)cmpc_ocp_enable_timing(ocp_, on ? 1 : 0);
  }
  double lastSolveMs() const {
    float ms = 0.f;
    if (!ocp_ || !timing_ || cmpc_ocp_last_solve_ms(ocp_, &ms) != CMPC_OK) return NAN;
    return ms;
  }

  void setMinimumEigenvalue(double v) {
    if (!(v >= 0.0)) throw std::invalid_argument("[HpipmInterface] minimum eigenvalue must be >= 0");
    minEig_ = v;
    minEigSet_ = true;
    riccatiValid_ = false;
    ricFb_ = false;
  }

  std::vector<ScalarFunctionQuadraticApproximation> costToGo(const VectorFunctionLinearApproximation& d0,
                                                              const ScalarFunctionQuadraticApproximation& c0) {
    riccati(d0, c0, true);
    const int N = last_.N, nx = last_.nx;
    std::vector<ScalarFunctionQuadraticApproximation> out((size_t)N + 1);
    for (int k = 0; k <= N; ++k) {  // node k's own nxk x nxk block of the padded P_k
      const int xk = last_.nxk[(size_t)k];
      out[(size_t)k].dfdxx.resize(xk, xk);
      out[(size_t)k].dfdx.resize(xk);
      for (int j = 0; j < xk; ++j)
        for (int i = 0; i < xk; ++i)
          out[(size_t)k].dfdxx(i, j) = k == 0 ? S0_[(size_t)j * xk + i] : Pm_[(size_t)k * nx * nx + (size_t)j * nx + i];
      for (int i = 0; i < xk; ++i) out[(size_t)k].dfdx(i) = k == 0 ? s0_[(size_t)i] : pv_[(size_t)k * nx + i];
      out[(size_t)k].f = 0.0;
    }
    return out;
  }
  matrix_array_t feedback(const VectorFunctionLinearApproximation& d0, const ScalarFunctionQuadraticApproximation& c0) {
    riccati(d0, c0, false);
    const int N = last_.N, nx = last_.nx;
    matrix_array_t out((size_t)N);
    size_t o = 0;
    for (int k = 0; k < N; ++k) {
      const int m = last_.nu[(size_t)k], xk = last_.nxk[(size_t)k];
      out[(size_t)k].resize(m, xk);  // the first nxk columns of the padded m x nx gain (column-major)
      if (k == 0) std::copy(K0_.begin(), K0_.end(), out[0].data());
      else std::copy(K_.begin() + (long)o, K_.begin() + (long)(o + (size_t)m * xk), out[(size_t)k].data());
      o += (size_t)m * nx;
    }
    return out;
  }
  vector_array_t feedforward(const VectorFunctionLinearApproximation& d0, const ScalarFunctionQuadraticApproximation& c0) {
    riccati(d0, c0, true);
    const int N = last_.N;
    vector_array_t out((size_t)N);
    size_t o = 0;
    for (int k = 0; k < N; ++k) {
      const int m = last_.nu[(size_t)k];
      out[(size_t)k].resize(m);
      if (k == 0) std::copy(k0_.begin(), k0_.end(), out[0].data());
      else std::copy(k_.begin() + (long)o, k_.begin() + (long)(o + (size_t)m), out[(size_t)k].data());
      o += (size_t)m;
    }
    return out;
  }

 private:
  void release() {
    if (ocp_) cmpc_ocp_destroy(ocp_);
    ocp_ = nullptr;
  }
  // the handle in the given dimensions: re-laid out (grow-only) when it exists, created otherwise
  void shape(int N, int nx, const std::vector<int>& nu, const std::vector<int>& nc, bool defer_no_device = false) {
    bool rows = false;
    for (int v : nc) rows = rows || v > 0;
    if (ocp_) {
      const int r = cmpc_ocp_reshape(ocp_, N, nx, nu.data(), rows ? nc.data() : nullptr);
      if (r != CMPC_OK)
        throw std::runtime_error(std::string("[HpipmInterface] cannot resize the device solver: ") + cmpc_error_string(r));
      ocpN_ = N;
      ocpNx_ = nx;
      ocpNu_ = nu;
      ocpNc_ = nc;
      riccatiValid_ = false;
      ricFb_ = false;
      return;
    }
    create(N, nx, nu, nc, defer_no_device);
  }
  void create(int N, int nx, const std::vector<int>& nu, const std::vector<int>& nc, bool defer_no_device = false) {
    release();
    cmpc_settings s;
    cmpc_settings_default(&s);
    s.hpipm_mode = (int)settings_.hpipmMode;
    s.iter_max = settings_.iter_max;
    s.alpha_min = settings_.alpha_min;
    s.mu0 = settings_.mu0;
    s.tol_stat = settings_.tol_stat;
    s.tol_eq = settings_.tol_eq;
    s.tol_ineq = settings_.tol_ineq;
    s.tol_comp = settings_.tol_comp;
    s.reg_prim = settings_.reg_prim;
    s.warm_start = settings_.warm_start;
    s.pred_corr = settings_.pred_corr;
    s.ric_alg = settings_.ric_alg;
    bool rows = false;
    for (int v : nc) rows = rows || v > 0;
    const int r = cmpc_ocp_create(N, nx, nu.data(), rows ? nc.data() : nullptr, &s, 1, &ocp_);
    if (r != CMPC_OK) {
      ocp_ = nullptr;
      if (defer_no_device && r == CMPC_ERR_NO_DEVICE) return;
      throw std::runtime_error(std::string("[HpipmInterface] cannot create the device solver: ") + cmpc_error_string(r));
    }
    // the MPC reads the feedback policy of every solve (MultipleShootingSolver.cpp:337-341, useFeedbackPolicy): the
    // solve leaves its exit Riccati quantities, the getters copy them
    (void)cmpc_ocp_set_keep_riccati(ocp_, keep_ ? 1 : 0);
    if (timing_) (void)cmpc_ocp_enable_timing(ocp_, 1);
    ocpN_ = N;
    ocpNx_ = nx;
    ocpNu_ = nu;
    ocpNc_ = nc;
  }

  // The problem's dimensions (the reference's verifySizes, HpipmInterface.cpp:146-164, per node), nodes embedded in the
  // padded state dimension (per-node nx, HPIPM's nx[k]: the padding rows and columns of A, B, b, Q, S, q and C are 0,
  // so padding states stay 0 and never couple)
  static void sizes(Packed& p, const vector_t& x0, const std::vector<VectorFunctionLinearApproximation>& dyn,
                    const std::vector<ScalarFunctionQuadraticApproximation>& cost,
                    const std::vector<VectorFunctionLinearApproximation>* constraints) {
    const int N = (int)dyn.size();
    p.N = N;
    p.nxk.assign((size_t)N + 1, 0);
    p.nxk[0] = (int)x0.size();
    p.nu.assign((size_t)N, 0);
    for (int k = 0; k < N; ++k) {
      const auto& d = dyn[(size_t)k];
      p.nu[(size_t)k] = (int)d.dfdu.cols();
      p.nxk[(size_t)k + 1] = (int)d.dfdx.rows();
      if ((int)d.dfdx.cols() != p.nxk[(size_t)k] || (int)d.f.size() != p.nxk[(size_t)k + 1] ||
          (p.nu[(size_t)k] > 0 && (int)d.dfdu.rows() != p.nxk[(size_t)k + 1]))
        throw std::runtime_error("[HpipmInterface] dynamics " + std::to_string(k) + " has inconsistent sizes");
    }
    for (int k = 0; k <= N; ++k) {
      const auto& c = cost[(size_t)k];
      const int m = k < N ? p.nu[(size_t)k] : 0;
      if ((int)c.dfdxx.rows() != p.nxk[(size_t)k] || (int)c.dfdxx.cols() != p.nxk[(size_t)k] ||
          (int)c.dfdx.size() != p.nxk[(size_t)k] ||
          (m > 0 && ((int)c.dfduu.rows() != m || (int)c.dfdux.rows() != m || (int)c.dfdux.cols() != p.nxk[(size_t)k])))
        throw std::runtime_error("[HpipmInterface] cost " + std::to_string(k) + " has inconsistent sizes");
    }
    p.nx = *std::max_element(p.nxk.begin(), p.nxk.end());
    p.nc.assign((size_t)N + 1, 0);
    if (constraints != nullptr) {
      for (int k = 0; k <= N; ++k) {
        const auto& c = (*constraints)[(size_t)k];
        const int rows = (int)c.f.size();
        const int m = k < N ? p.nu[(size_t)k] : 0;
        if (rows == 0) continue;
        const int xk = p.nxk[(size_t)k];
        if ((int)c.dfdx.rows() != rows || (int)c.dfdx.cols() != xk ||
            (m > 0 && ((int)c.dfdu.rows() != rows || (int)c.dfdu.cols() != m)))
          throw std::runtime_error("[HpipmInterface] constraint " + std::to_string(k) + " has inconsistent sizes");
        p.nc[(size_t)k] = rows;
      }
    }
  }

  // The problem in the engine's packed forms (cmpc.h: OCP record [A,B,b] per stage then [Q,S,R,q,r] per node;
  // constraint record [C,D,e] per node with rows), column-major blocks as Eigen stores them, into rec / crec
  static void fill(const Packed& p, const std::vector<VectorFunctionLinearApproximation>& dyn,
                   const std::vector<ScalarFunctionQuadraticApproximation>& cost,
                   const std::vector<VectorFunctionLinearApproximation>* constraints, double* rec, double* crec) {
    const int N = p.N, nx = p.nx;
    size_t o = 0;
    auto put = [&](const double* src, int r, int c, int R, int Cc) {  // column-major r x c block into an R x C slot
      for (int j = 0; j < Cc; ++j)
        for (int i = 0; i < R; ++i) rec[o + (size_t)j * R + i] = (src && i < r && j < c) ? src[(size_t)j * r + i] : 0.0;
      o += (size_t)R * Cc;
    };
    for (int k = 0; k < N; ++k) {
      const auto& d = dyn[(size_t)k];
      const int r = p.nxk[(size_t)k + 1], c = p.nxk[(size_t)k], m = p.nu[(size_t)k];
      put(d.dfdx.data(), r, c, nx, nx);
      put(m ? d.dfdu.data() : nullptr, r, m, nx, m);
      put(d.f.data(), r, 1, nx, 1);
    }
    for (int k = 0; k <= N; ++k) {  // raw cost blocks: reg_prim enters the device factorisation only
      const auto& c = cost[(size_t)k];
      const int m = k < N ? p.nu[(size_t)k] : 0, xk = p.nxk[(size_t)k];
      put(c.dfdxx.data(), xk, xk, nx, nx);
      put(m ? c.dfdux.data() : nullptr, m, xk, m, nx);
      put(m ? c.dfduu.data() : nullptr, m, m, m, m);
      put(c.dfdx.data(), xk, 1, nx, 1);
      put(m ? c.dfdu.data() : nullptr, m, 1, m, 1);
    }
    // === Constraints === C dx + D du + e = 0 per node, the reference's lg = ug = -e rows (HpipmInterface.cpp:223-264,
    // stage 0 bounded through x0 on the device); an empty node (f.size() == 0) has none
    if (constraints == nullptr || !crec) return;
    size_t oc = 0;
    for (int k = 0; k <= N; ++k) {
      const auto& c = (*constraints)[(size_t)k];
      const int rows = p.nc[(size_t)k];
      const int m = k < N ? p.nu[(size_t)k] : 0;
      if (rows == 0) continue;
      const int xk = p.nxk[(size_t)k];
      std::copy(c.dfdx.data(), c.dfdx.data() + (size_t)rows * xk, crec + oc);
      oc += (size_t)rows * xk;
      std::fill(crec + oc, crec + oc + (size_t)rows * (nx - xk), 0.0);  // padding state columns
      oc += (size_t)rows * (nx - xk);
      if (m > 0) {
        std::copy(c.dfdu.data(), c.dfdu.data() + (size_t)rows * m, crec + oc);
        oc += (size_t)rows * m;
      }
      std::copy(c.f.data(), c.f.data() + rows, crec + oc);
      oc += (size_t)rows;
    }
  }

  // LinearAlgebra::setTriangularMinimumEigenvalues(Lr) of every getter (HpipmInterface.cpp:340, :357, :379, :419), when
  // a minimum is set (setRiccatiMinimumEigenvalue): the diagonal of each Lr_k is moved away from 0 to at least the
  // minimum in magnitude (hpipm_interface::setTriangularMinimumEigenvalues); K_k (k >= 1) is re-derived from the
  // clamped factor as the reference's getRiccatiFeedback does, K_k = -Lr_c^-T Ls', with Ls' = -Lr' K_k of the
  // device's factor; stage 0 uses the clamped Lr_0. The feedforward of k >= 1 is read as the reference reads ric_k.
  // With ocs2_core on the include path and no minimum set, every getter clamps as the reference does, by ocs2's own
  // LinearAlgebra::setTriangularMinimumEigenvalues with its default minimum; setRiccatiMinimumEigenvalue(v) replaces
  // that by v (0: no clamp). With the stand-in types there is no ocs2 default to take: the clamp runs when a minimum
  // is set.
  bool clampActive() const {
#ifdef CMPC_HAVE_OCS2_CORE
    if (!minEigSet_) return true;
#endif
    return minEig_ > 0.0;
  }
  // the clamp of one stage's m x m lower factor (column-major) in place; returns whether a diagonal entry changed
  bool clampStage(double* Lc, int m) const {
#ifdef CMPC_HAVE_OCS2_CORE
    if (!minEigSet_) {
      matrix_t L(m, m);
      std::copy(Lc, Lc + (size_t)m * m, L.data());
      LinearAlgebra::setTriangularMinimumEigenvalues(L);
      bool changed = false;
      for (int i = 0; i < m; ++i) changed = changed || L.data()[(size_t)i * m + i] != Lc[(size_t)i * m + i];
      std::copy(L.data(), L.data() + (size_t)m * m, Lc);
      return changed;
    }
#endif
    return hpipm_interface::setTriangularMinimumEigenvalues(Lc, m, minEig_);
  }
  void clampFactors(int nx) {
    const Packed& p = last_;
    size_t oK = 0, oM = 0;
    std::vector<double> Lc, Ls;
    for (int k = 0; k < p.N; ++k) {
      const int m = p.nu[(size_t)k];
      double* Lr = Lr_.data() + oM;
      Lc.assign(Lr, Lr + (size_t)m * m);
      if (m > 0 && clampStage(Lc.data(), m) && k >= 1) {
        Ls.resize((size_t)m);
        hpipm_interface::rederiveFeedback(Lr, Lc.data(), K_.data() + oK, m, nx, Ls.data());
      }
      std::copy(Lc.begin(), Lc.end(), Lr);
      oK += (size_t)m * nx;
      oM += (size_t)m * m;
    }
  }

  // Stage 0 as the reference rebuilds it (HpipmInterface.cpp:334-347, :376-389, :416-453; x0 is not an HPIPM
  // variable), by triangular solves with Lr_0 of the device factorisation (HPIPM's ric_Lr(0)) and P_1, p_1 of node 1:
  //   T1 = Lr_0^-1 (S_0 + B_0'P_1 A_0), t2 = Lr_0^-1 (r_0 + B_0'(p_1 + P_1 b_0)), K_0 = -Lr_0^-T T1, k_0 = -Lr_0^-T t2,
  //   S_0 = Q_0 + A_0'P_1 A_0 - T1'T1, s_0 = q_0 + A_0'(p_1 + P_1 b_0) - T1't2.
  // Lr_0 is the clamped factor when setRiccatiMinimumEigenvalue set a minimum (clampFactors, the reference's
  // LinearAlgebra::setTriangularMinimumEigenvalues(Lr0), :340, :379, :419); without one, the device factorisation's
  // pivot guard stands (a pivot <= 1e-200 gives a zero column, whose solves contribute 0).
  // vectors = false (feedback only): K_0 alone (k_0, S_0, s_0 need p_1, not fetched)
  void stage0(const VectorFunctionLinearApproximation& d0, const ScalarFunctionQuadraticApproximation& c0,
              bool vectors) {
    const Packed& p = last_;
    const int nx = p.nx, x0n = p.nxk[0], x1n = p.nxk[1], m = p.nu[0];
    const double* P1 = Pm_.data() + (size_t)nx * nx;  // padded, column-major
    const double* p1 = pv_.data() + nx;
    const double* Lr = Lr_.data();                   // m x m column-major, lower
    auto A = [&](int i, int j) { return d0.dfdx.data()[(size_t)j * x1n + i]; };
    auto B = [&](int i, int a) { return d0.dfdu.data()[(size_t)a * x1n + i]; };
    std::vector<double> PA((size_t)x1n * x0n), v((size_t)x1n), T1((size_t)m * x0n), t2((size_t)m);
    for (int i = 0; i < x1n; ++i) {
      for (int j = 0; j < x0n; ++j) {
        double s = 0.0;
        for (int t = 0; t < x1n; ++t) s += P1[(size_t)t * nx + i] * A(t, j);
        PA[(size_t)i * x0n + j] = s;
      }
      double s = p1[i];
      for (int t = 0; t < x1n; ++t) s += P1[(size_t)t * nx + i] * d0.f.data()[t];
      v[(size_t)i] = s;
    }
    for (int a = 0; a < m; ++a) {
      for (int j = 0; j < x0n; ++j) {
        double s = c0.dfdux.data()[(size_t)j * m + a];
        for (int t = 0; t < x1n; ++t) s += B(t, a) * PA[(size_t)t * x0n + j];
        T1[(size_t)a * x0n + j] = s;
      }
      double s = c0.dfdu.data()[a];
      for (int t = 0; t < x1n; ++t) s += B(t, a) * v[(size_t)t];
      t2[(size_t)a] = s;
    }
    auto L = [&](int i, int j) { return Lr[(size_t)j * m + i]; };
    auto lsolve = [&](double* c, size_t cs) {  // c <- Lr^-1 c
      for (int a = 0; a < m; ++a) {
        double s = c[(size_t)a * cs];
        for (int b = 0; b < a; ++b) s -= L(a, b) * c[(size_t)b * cs];
        c[(size_t)a * cs] = L(a, a) > 0.0 ? s / L(a, a) : 0.0;
      }
    };
    auto ltsolve = [&](double* c, size_t cs) {  // c <- Lr^-T c
      for (int a = m - 1; a >= 0; --a) {
        double s = c[(size_t)a * cs];
        for (int b = a + 1; b < m; ++b) s -= L(b, a) * c[(size_t)b * cs];
        c[(size_t)a * cs] = L(a, a) > 0.0 ? s / L(a, a) : 0.0;
      }
    };
    K0_.assign((size_t)m * x0n, 0.0);
    k0_.assign((size_t)m, 0.0);
    std::vector<double> col((size_t)m);
    for (int j = 0; j < x0n; ++j) {
      lsolve(T1.data() + j, (size_t)x0n);
      for (int a = 0; a < m; ++a) col[(size_t)a] = T1[(size_t)a * x0n + j];
      ltsolve(col.data(), 1);
      for (int a = 0; a < m; ++a) K0_[(size_t)j * m + a] = -col[(size_t)a];
    }
    lsolve(t2.data(), 1);
    for (int a = 0; a < m; ++a) col[(size_t)a] = t2[(size_t)a];
    ltsolve(col.data(), 1);
    for (int a = 0; a < m; ++a) k0_[(size_t)a] = -col[(size_t)a];
    if (!vectors) return;
    S0_.assign((size_t)x0n * x0n, 0.0);
    s0_.assign((size_t)x0n, 0.0);
    for (int i = 0; i < x0n; ++i) {
      for (int j = 0; j < x0n; ++j) {
        double s = c0.dfdxx.data()[(size_t)j * x0n + i];
        for (int t = 0; t < x1n; ++t) s += A(t, i) * PA[(size_t)t * x0n + j];
        for (int a = 0; a < m; ++a) s -= T1[(size_t)a * x0n + i] * T1[(size_t)a * x0n + j];
        S0_[(size_t)j * x0n + i] = s;
      }
      double s = c0.dfdx.data()[i];
      for (int t = 0; t < x1n; ++t) s += A(t, i) * v[(size_t)t];
      for (int a = 0; a < m; ++a) s -= T1[(size_t)a * x0n + i] * t2[(size_t)a];
      s0_[(size_t)i] = s;
    }
  }

  // The reference's verbose printout (HpipmInterface.cpp:457-503): status line, iteration count, the final max
  // residuals (d_ocp_qp_ipm_get_max_res_*) and the per-iteration statistics table (d_ocp_qp_ipm_get_stat), from the
  // device solver's records (cmpc_ocp_get_residuals_host / cmpc_ocp_get_stats_host). The table has the reference's
  // 17 columns: the first ten are cmpc_enable_stats'; lq fact, itref pred and itref corr are 0 (the device solver is
  // the Riccati recursion of the SPEED mode the reference selects, HpipmInterfaceSettings.h:45: no LQ factorisation,
  // no iterative refinement); the four lin res columns are the device's residuals of each iteration's Newton system
  // at its final direction (cmpc_ocp_set_linres; what HPIPM prints there is unpinned: it is not vendored)
  void printStatus(int status, int iters) const {
    double res[4] = {NAN, NAN, NAN, NAN};
    const int rows = cmpc_ocp_stat_rows(ocp_);
    std::vector<double> stats((size_t)(rows > 0 ? rows : 1) * CMPC_STAT_COLS, NAN);
    std::vector<double> lin((size_t)(rows > 0 ? rows : 1) * 4, NAN);
    cmpc_ocp_get_residuals_host(ocp_, 1, res);
    if (rows > 0) cmpc_ocp_get_stats_host(ocp_, 1, stats.data());
    if (rows > 0) cmpc_ocp_get_linres_host(ocp_, 1, lin.data());
    std::fprintf(stderr, "\n=== HPIPM (MI355X engine) ===\n");
    std::fprintf(stderr, "HPIPM returned with flag %i. -> ", status);
    if (status == CMPC_SUCCESS) std::fprintf(stderr, "QP solved!\n");
    else if (status == CMPC_MAX_ITER) std::fprintf(stderr, "Solver failed! Maximum number of iterations reached\n");
    else if (status == CMPC_MIN_STEP) std::fprintf(stderr, "Solver failed! Minimum step length reached\n");
    else if (status == CMPC_NAN_SOL) std::fprintf(stderr, "Solver failed! NaN in computations\n");
    else if (status == CMPC_INCONS_EQ) std::fprintf(stderr, "Solver failed! Unconsistent equality constraints\n");
    else std::fprintf(stderr, "Solver failed! Unknown return flag\n");
    std::fprintf(stderr, "ipm iter = %d\n", iters);
    std::fprintf(stderr, "ipm residuals max: res_g = %e, res_b = %e, res_d = %e, res_m = %e\n", res[0], res[1], res[2],
                 res[3]);
    std::fprintf(stderr,
                 "\nalpha_aff\tmu_aff\t\tsigma\t\talpha_prim\talpha_dual\tmu\t\tres_stat\tres_eq\t\tres_ineq\tres_comp\tlq fact\t\titref "
                 "pred\titref corr\tlin res stat\tlin res eq\tlin res ineq\tlin res comp\n");
    for (int j = 0; j < iters + 1 && j < rows; ++j) {
      for (int i = 0; i < CMPC_STAT_COLS; ++i) std::fprintf(stderr, "%e\t", stats[(size_t)j * CMPC_STAT_COLS + i]);
      for (int i = 0; i < 3; ++i) std::fprintf(stderr, "%e\t", 0.0);  // lq fact, itref pred, itref corr
      for (int i = 0; i < 4; ++i) std::fprintf(stderr, "%e\t", lin[(size_t)j * 4 + i]);  // lin res stat/eq/ineq/comp
      std::fprintf(stderr, "\n");
    }
  }

  Settings settings_;
  OcpSize size_;
  cmpc_ocp* ocp_ = nullptr;  // the device solver (HPIPM's dim / qp / sol / arg / ws memory)
  int ocpN_ = 0, ocpNx_ = 0;
  std::vector<int> ocpNu_, ocpNc_;
  Packed last_;
  bool riccatiValid_ = false;  // every Riccati quantity of the last solve fetched
  bool ricFb_ = false;         // K, Lr, P_1 fetched
  double minEig_ = 0.0;     // setRiccatiMinimumEigenvalue (0: no clamp)
  bool minEigSet_ = false;  // a minimum was set (otherwise, with ocs2_core, ocs2's own default clamps)
  bool timing_ = false;  // enableDeviceTiming
  bool keep_ = true;     // keepRiccati
  std::vector<double> xbuf_, ubuf_, recbuf_, crecbuf_, x0buf_, Pm_, pv_, K_, k_, Lr_, K0_, k0_, S0_, s0_;
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
void HpipmInterface::setRiccatiMinimumEigenvalue(double minEigenValue) { pImpl_->setMinimumEigenvalue(minEigenValue); }
int HpipmInterface::deviceAllocations() const { return pImpl_->allocations(); }
void HpipmInterface::enableDeviceTiming(bool on) { pImpl_->enableTiming(on); }
double HpipmInterface::lastSolveDeviceMs() const { return pImpl_->lastSolveMs(); }
void HpipmInterface::keepRiccati(bool on) { pImpl_->setKeep(on); }

}  // namespace ocs2
