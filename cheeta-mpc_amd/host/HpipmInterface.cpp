// HpipmInterface.cpp — ocs2::HpipmInterface mirror (reference HpipmInterface.cpp:86-554) on the MI355X engine.
//
// Written against the API the real ocs2 / Eigen types and the stand-ins of ocs2_types.h share (rows(), cols(),
// size(), data(), resize(), operator()), so an ocs2 build compiles this file inside its hpipm_catkin target against
// ocs2_core; the device is reached only through the C ABI (cmpc/cmpc.h).
#include "hpipm_catkin/HpipmInterface.h"

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
  std::vector<double> rec, crec;
  std::vector<size_t> coff;  // start of node k's [C, D, e] in crec
};

double maxabs(double a, double b) { return std::fmax(a, std::fabs(b)); }

}  // namespace

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
    Packed p;
    p.N = N;
    // per-node state dimensions (OcpSize::numStates, HPIPM's nx[k]): node k's state is embedded in the first
    // nxk[k] components of a padded state of dimension nx = max_k nxk[k]; the padding rows and columns of A, B, b,
    // Q, S, q and C are 0, so padding states stay 0 and never couple (the device path takes one nx per problem)
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
    const int nx = p.nx;
    p.rec.assign(cmpc_ocp_record_size(N, nx, p.nu.data()), 0.0);
    size_t o = 0;
    // column-major r x c block (src may be null) into an R x C slot, zero padded
    auto put = [&](const double* src, int r, int c, int R, int Cc) {
      for (int j = 0; j < Cc; ++j)
        for (int i = 0; i < R; ++i) p.rec[o + (size_t)j * R + i] = (src && i < r && j < c) ? src[(size_t)j * r + i] : 0.0;
      o += (size_t)R * Cc;
    };
    for (int k = 0; k < N; ++k) {
      const auto& d = dyn[(size_t)k];
      const int r = p.nxk[(size_t)k + 1], c = p.nxk[(size_t)k], m = p.nu[(size_t)k];
      put(d.dfdx.data(), r, c, nx, nx);
      put(m ? d.dfdu.data() : nullptr, r, m, nx, m);
      put(d.f.data(), r, 1, nx, 1);
    }
    const double reg = settings_.reg_prim;
    for (int k = 0; k <= N; ++k) {
      const auto& c = cost[(size_t)k];
      const int m = k < N ? p.nu[(size_t)k] : 0, xk = p.nxk[(size_t)k];
      const size_t oq = o;
      put(c.dfdxx.data(), xk, xk, nx, nx);
      if (k > 0)  // HPIPM's primal regularisation; node 0's state is eliminated
        for (int i = 0; i < xk; ++i) p.rec[oq + (size_t)i * nx + i] += reg;
      put(m ? c.dfdux.data() : nullptr, m, xk, m, nx);
      const size_t orr = o;
      put(m ? c.dfduu.data() : nullptr, m, m, m, m);
      for (int i = 0; i < m; ++i) p.rec[orr + (size_t)i * m + i] += reg;
      put(c.dfdx.data(), xk, 1, nx, 1);
      put(m ? c.dfdu.data() : nullptr, m, 1, m, 1);
    }
    int nU = 0;
    for (int v : p.nu) nU += v;
    // === Constraints === C dx + D du + e = 0 per node, handed to the device as they come (the reference maps them to
    // HPIPM's lg = ug = -e, with the stage-0 rows bounded through x0, HpipmInterface.cpp:223-264); an empty node
    // (f.size() == 0) has no rows
    p.nc.assign((size_t)N + 1, 0);
    p.coff.assign((size_t)N + 2, 0);
    int nE = 0;
    if (constraints != nullptr) {
      for (int k = 0; k <= N; ++k) {
        const auto& c = (*constraints)[(size_t)k];
        const int rows = (int)c.f.size();
        const int m = k < N ? p.nu[(size_t)k] : 0;
        p.coff[(size_t)k] = p.crec.size();
        if (rows == 0) continue;
        const int xk = p.nxk[(size_t)k];
        if ((int)c.dfdx.rows() != rows || (int)c.dfdx.cols() != xk ||
            (m > 0 && ((int)c.dfdu.rows() != rows || (int)c.dfdu.cols() != m)))
          throw std::runtime_error("[HpipmInterface] constraint " + std::to_string(k) + " has inconsistent sizes");
        p.nc[(size_t)k] = rows;
        nE += rows;
        p.crec.insert(p.crec.end(), c.dfdx.data(), c.dfdx.data() + (size_t)rows * xk);
        p.crec.insert(p.crec.end(), (size_t)rows * (nx - xk), 0.0);  // padding state columns
        if (m > 0) p.crec.insert(p.crec.end(), c.dfdu.data(), c.dfdu.data() + (size_t)rows * m);
        p.crec.insert(p.crec.end(), c.f.data(), c.f.data() + rows);
      }
      p.coff[(size_t)N + 1] = p.crec.size();
    }
    std::vector<double> x((size_t)(N + 1) * nx), u((size_t)(nU > 0 ? nU : 1));
    std::vector<double> x0p((size_t)nx, 0.0);
    for (int i = 0; i < p.nxk[0]; ++i) x0p[(size_t)i] = x0(i);
    int status = -1;
    deviceSolve(p, nE > 0, 1, x0p.data(), x.data(), u.data(), &status);
    xs.assign((size_t)N + 1, vector_t());
    for (int k = 0; k <= N; ++k) {
      const int xk = p.nxk[(size_t)k];
      xs[(size_t)k].resize(xk);
      for (int i = 0; i < xk; ++i) xs[(size_t)k](i) = k == 0 ? x0(i) : x[(size_t)k * nx + i];
    }
    us.assign((size_t)N, vector_t());
    int off = 0;
    for (int k = 0; k < N; ++k) {
      us[(size_t)k].resize(p.nu[(size_t)k]);
      for (int i = 0; i < p.nu[(size_t)k]; ++i) us[(size_t)k](i) = u[(size_t)off + i];
      off += p.nu[(size_t)k];
    }
    if (verbose) printStatus(p, nE > 0, x0p.data(), x, u, status);
    last_ = std::move(p);
    lastConstrained_ = nE > 0;
    riccatiValid_ = false;
    return (hpipm_status)status;
  }

  // Device Riccati quantities of the last problem, computed once per solve on first use.
  void riccati(const VectorFunctionLinearApproximation& dyn0, const ScalarFunctionQuadraticApproximation& cost0) {
    const int N = last_.N;
    if (N == 0) throw std::runtime_error("[HpipmInterface] no solved problem to take Riccati quantities from");
    if ((int)dyn0.dfdx.rows() != last_.nxk[1] || (int)dyn0.dfdx.cols() != last_.nxk[0] ||
        (int)dyn0.dfdu.cols() != last_.nu[0] || (int)cost0.dfdxx.rows() != last_.nxk[0])
      throw std::runtime_error("[HpipmInterface] dynamics0 / cost0 do not match the last solved problem");
    if (riccatiValid_) return;
    const int nx = last_.nx;
    int nU = 0;
    for (int v : last_.nu) nU += v;
    Sm_.assign((size_t)(N + 1) * nx * nx, 0.0);
    sv_.assign((size_t)(N + 1) * nx, 0.0);
    K_.assign((size_t)(nU > 0 ? nU : 1) * nx, 0.0);
    k_.assign((size_t)(nU > 0 ? nU : 1), 0.0);
    if (lastConstrained_) {
      constrainedRiccati();
    } else {
      int st = -1;
      const int r = cmpc_ocp_riccati_batch_host(1, N, nx, last_.nu.data(), last_.rec.data(), Sm_.data(), sv_.data(),
                                                K_.data(), k_.data(), &st);
      if (r != CMPC_OK)
        throw std::runtime_error(std::string("[HpipmInterface] device Riccati failed: ") + cmpc_error_string(r));
      if (st != CMPC_SUCCESS) throw std::runtime_error("[HpipmInterface] Riccati recursion: R + B'PB not positive definite");
    }
    riccatiValid_ = true;
  }
  std::vector<ScalarFunctionQuadraticApproximation> costToGo(const VectorFunctionLinearApproximation& d0,
                                                              const ScalarFunctionQuadraticApproximation& c0) {
    riccati(d0, c0);
    const int N = last_.N, nx = last_.nx;
    std::vector<ScalarFunctionQuadraticApproximation> out((size_t)N + 1);
    for (int k = 0; k <= N; ++k) {  // node k's own nxk x nxk block of the padded S_k
      const int xk = last_.nxk[(size_t)k];
      out[(size_t)k].dfdxx.resize(xk, xk);
      out[(size_t)k].dfdx.resize(xk);
      for (int j = 0; j < xk; ++j)
        for (int i = 0; i < xk; ++i) out[(size_t)k].dfdxx(i, j) = Sm_[(size_t)k * nx * nx + (size_t)j * nx + i];
      for (int i = 0; i < xk; ++i) out[(size_t)k].dfdx(i) = sv_[(size_t)k * nx + i];
      out[(size_t)k].f = 0.0;
    }
    return out;
  }
  matrix_array_t feedback(const VectorFunctionLinearApproximation& d0, const ScalarFunctionQuadraticApproximation& c0) {
    riccati(d0, c0);
    const int N = last_.N, nx = last_.nx;
    matrix_array_t out((size_t)N);
    size_t o = 0;
    for (int k = 0; k < N; ++k) {
      const int m = last_.nu[(size_t)k], xk = last_.nxk[(size_t)k];
      out[(size_t)k].resize(m, xk);  // the first nxk columns of the padded m x nx gain (column-major)
      std::copy(K_.begin() + (long)o, K_.begin() + (long)(o + (size_t)m * xk), out[(size_t)k].data());
      o += (size_t)m * nx;
    }
    return out;
  }
  vector_array_t feedforward(const VectorFunctionLinearApproximation& d0, const ScalarFunctionQuadraticApproximation& c0) {
    riccati(d0, c0);
    const int N = last_.N;
    vector_array_t out((size_t)N);
    size_t o = 0;
    for (int k = 0; k < N; ++k) {
      const int m = last_.nu[(size_t)k];
      out[(size_t)k].resize(m);
      std::copy(k_.begin() + (long)o, k_.begin() + (long)(o + (size_t)m), out[(size_t)k].data());
      o += (size_t)m;
    }
    return out;
  }

 private:
  // B problems of the packed form p sharing its records but with their own x0 [B][nx]
  static void deviceSolve(const Packed& p, bool eq, int B, const double* x0, double* x, double* u, int* status) {
    std::vector<double> rec, crec;
    const double* rp = p.rec.data();
    const double* cp = p.crec.data();
    if (B > 1) {
      for (int b = 0; b < B; ++b) rec.insert(rec.end(), p.rec.begin(), p.rec.end());
      rp = rec.data();
      if (eq) {
        for (int b = 0; b < B; ++b) crec.insert(crec.end(), p.crec.begin(), p.crec.end());
        cp = crec.data();
      }
    }
    const int r = eq ? cmpc_ocp_solve_batch_eq_host(B, p.N, p.nx, p.nu.data(), p.nc.data(), x0, rp, cp, x, u, status)
                     : cmpc_ocp_solve_batch_host(B, p.N, p.nx, p.nu.data(), x0, rp, x, u, status);
    if (r != CMPC_OK) throw std::runtime_error(std::string("[HpipmInterface] device solve failed: ") + cmpc_error_string(r));
  }

  // offsets of node k's blocks inside the OCP record (cmpc.h layout)
  static void recOffsets(const Packed& p, std::vector<size_t>& dynOff, std::vector<size_t>& costOff) {
    dynOff.assign((size_t)p.N + 1, 0);
    costOff.assign((size_t)p.N + 2, 0);
    size_t o = 0;
    for (int k = 0; k < p.N; ++k) {
      dynOff[(size_t)k] = o;
      o += (size_t)p.nx * p.nx + (size_t)p.nx * p.nu[(size_t)k] + (size_t)p.nx;
    }
    dynOff[(size_t)p.N] = o;
    for (int k = 0; k <= p.N; ++k) {
      costOff[(size_t)k] = o;
      const size_t m = k < p.N ? (size_t)p.nu[(size_t)k] : 0;
      o += (size_t)p.nx * p.nx + m * p.nx + m * m + (size_t)p.nx + m;
    }
    costOff[(size_t)p.N + 1] = o;
  }

  // The tail problem of stages k..N-1 of the last problem (records and constraint rows copied; the state-only rows of
  // its first node dropped: that state is given).
  Packed tail(int k) const {
    const Packed& p = last_;
    std::vector<size_t> dynOff, costOff;
    recOffsets(p, dynOff, costOff);
    Packed t;
    t.N = p.N - k;
    t.nx = p.nx;
    t.nu.assign(p.nu.begin() + k, p.nu.end());
    t.rec.assign(p.rec.begin() + (long)dynOff[(size_t)k], p.rec.begin() + (long)dynOff[(size_t)p.N]);
    t.rec.insert(t.rec.end(), p.rec.begin() + (long)costOff[(size_t)k], p.rec.begin() + (long)costOff[(size_t)p.N + 1]);
    t.nc.assign((size_t)t.N + 1, 0);
    t.coff.assign((size_t)t.N + 2, 0);
    for (int j = k; j <= p.N; ++j) {
      const int rows = p.nc[(size_t)j];
      t.coff[(size_t)(j - k)] = t.crec.size();
      if (rows == 0) continue;
      const int m = j < p.N ? p.nu[(size_t)j] : 0;
      const double* C = p.crec.data() + p.coff[(size_t)j];
      const double* D = C + (size_t)rows * p.nx;
      const double* e = D + (size_t)rows * m;
      std::vector<int> keep;
      for (int i = 0; i < rows; ++i) {
        bool hasInput = false;
        for (int c = 0; c < m; ++c) hasInput = hasInput || D[(size_t)c * rows + i] != 0.0;
        if (j > k || hasInput) keep.push_back(i);
      }
      const int kr = (int)keep.size();
      if (kr == 0) continue;
      t.nc[(size_t)(j - k)] = kr;
      for (int c = 0; c < p.nx; ++c)
        for (int i : keep) t.crec.push_back(C[(size_t)c * rows + i]);
      for (int c = 0; c < m; ++c)
        for (int i : keep) t.crec.push_back(D[(size_t)c * rows + i]);
      for (int i : keep) t.crec.push_back(e[i]);
    }
    t.coff[(size_t)t.N + 1] = t.crec.size();
    return t;
  }

  // Feedback, feedforward and cost-to-go of the equality-constrained problem from the affine solution maps of its
  // tail problems: for stage k, solve the tail from x_k = 0 and x_k = e_i (one device batch of nx + 1 problems);
  // u_k = K_k x_k + k_k, and V_k(x) = sum_j l_j(Phi_j x + phi_j, K_j x + k_j) over the tail's trajectories gives
  // S_k = sum [Phi; K]' [Q S'; S R] [Phi; K] and s_k = sum [Phi; K]' ([Q S'; S R] [phi; kk] + [q; r]).
  void constrainedRiccati() {
    const Packed& p = last_;
    const int N = p.N, nx = p.nx;
    std::vector<size_t> dynOff, costOff;
    recOffsets(p, dynOff, costOff);
    size_t kOff = 0;
    for (int k = 0; k <= N; ++k) {
      const int Nt = N - k;
      const int B = nx + 1;
      std::vector<double> xt, ut;
      int nUt = 0;
      if (Nt > 0) {
        const Packed t = tail(k);
        for (int v : t.nu) nUt += v;
        std::vector<double> x0((size_t)B * nx, 0.0);
        for (int i = 0; i < nx; ++i) x0[(size_t)(i + 1) * nx + i] = 1.0;
        xt.assign((size_t)B * (Nt + 1) * nx, 0.0);
        ut.assign((size_t)B * (nUt > 0 ? nUt : 1), 0.0);
        std::vector<int> st((size_t)B, -1);
        bool eq = false;
        for (int v : t.nc) eq = eq || v > 0;
        deviceSolve(t, eq, B, x0.data(), xt.data(), ut.data(), st.data());
        for (int b = 0; b < B; ++b)
          if (st[(size_t)b] != CMPC_SUCCESS)
            throw std::runtime_error("[HpipmInterface] constrained Riccati: tail problem of stage " + std::to_string(k) +
                                     " has status " + cmpc_status_string(st[(size_t)b]));
      }
      const int ust = nUt > 0 ? nUt : 1;
      // trajectory maps of the tail: node j (0..Nt) state Phi_j x + phi_j, stage j input Kj x + kj
      auto xs = [&](int b, int j, int i) { return Nt > 0 ? xt[((size_t)b * (Nt + 1) + j) * nx + i] : (b == 0 ? 0.0 : (b - 1 == i ? 1.0 : 0.0)); };
      std::vector<int> uoff((size_t)Nt + 1, 0);
      for (int j = 0; j < Nt; ++j) uoff[(size_t)j + 1] = uoff[(size_t)j] + p.nu[(size_t)(k + j)];
      auto us = [&](int b, int j, int i) { return ut[(size_t)b * ust + uoff[(size_t)j] + i]; };
      if (k < N) {  // K_k (m x nx column-major) and k_k
        const int m = p.nu[(size_t)k];
        for (int c = 0; c < nx; ++c)
          for (int i = 0; i < m; ++i) K_[kOff + (size_t)c * m + i] = us(c + 1, 0, i) - us(0, 0, i);
        for (int i = 0; i < m; ++i) k_[(kOff / nx) + i] = us(0, 0, i);
        kOff += (size_t)m * nx;
      }
      // cost-to-go of node k
      double* S = Sm_.data() + (size_t)k * nx * nx;
      double* s = sv_.data() + (size_t)k * nx;
      for (int j = 0; j <= Nt; ++j) {
        const int node = k + j;
        const int m = node < N ? p.nu[(size_t)node] : 0;
        const double* Q = p.rec.data() + costOff[(size_t)node];
        const double* Sx = Q + (size_t)nx * nx;  // S: m x nx
        const double* R = Sx + (size_t)m * nx;
        const double* q = R + (size_t)m * m;
        const double* r = q + nx;
        const int nz = nx + m;
        // columns of [Phi; K] (c = 0..nx-1) and [phi; kk]
        std::vector<double> Z((size_t)nz * (nx + 1));
        for (int c = 0; c <= nx; ++c)
          for (int i = 0; i < nz; ++i) {
            const int b = c < nx ? c + 1 : 0;
            const double v = i < nx ? xs(b, j, i) : us(b, j, i - nx);
            const double v0 = i < nx ? xs(0, j, i) : us(0, j, i - nx);
            Z[(size_t)c * nz + i] = c < nx ? v - v0 : v0;
          }
        // W = [Q S'; S R] applied to each column
        auto Wz = [&](const double* z, double* out) {
          for (int i = 0; i < nx; ++i) {
            double a = 0.0;
            for (int c = 0; c < nx; ++c) a += Q[(size_t)c * nx + i] * z[c];
            for (int c = 0; c < m; ++c) a += Sx[(size_t)i * m + c] * z[nx + c];  // S'(i, c) = S(c, i)
            out[i] = a;
          }
          for (int i = 0; i < m; ++i) {
            double a = 0.0;
            for (int c = 0; c < nx; ++c) a += Sx[(size_t)c * m + i] * z[c];
            for (int c = 0; c < m; ++c) a += R[(size_t)c * m + i] * z[nx + c];
            out[nx + i] = a;
          }
        };
        std::vector<double> wz((size_t)nz);
        for (int c = 0; c <= nx; ++c) {
          Wz(Z.data() + (size_t)c * nz, wz.data());
          if (c < nx) {
            for (int a = 0; a < nx; ++a) {
              double acc = 0.0;
              for (int i = 0; i < nz; ++i) acc += Z[(size_t)a * nz + i] * wz[(size_t)i];
              S[(size_t)c * nx + a] += acc;
            }
          } else {
            for (int i = 0; i < nx; ++i) wz[(size_t)i] += q[i];
            for (int i = 0; i < m; ++i) wz[(size_t)nx + i] += r[i];
            for (int a = 0; a < nx; ++a) {
              double acc = 0.0;
              for (int i = 0; i < nz; ++i) acc += Z[(size_t)a * nz + i] * wz[(size_t)i];
              s[a] += acc;
            }
          }
        }
      }
    }
  }

  // The reference's verbose printout (HpipmInterface.cpp:457-503). The direct solve is iteration 0; its residuals
  // are evaluated here from the trajectories: res_b = dynamics and equality rows, res_g = stationarity in u of the
  // equality-free problem (adjoint sweep; with equality rows their multipliers are not returned, so NaN).
  void printStatus(const Packed& p, bool eq, const double* x0, const std::vector<double>& x, const std::vector<double>& u,
                   int status) const {
    const int N = p.N, nx = p.nx;
    std::vector<size_t> dynOff, costOff;
    recOffsets(p, dynOff, costOff);
    auto X = [&](int k, int i) { return k == 0 ? x0[i] : x[(size_t)k * nx + i]; };
    std::vector<int> uoff((size_t)N + 1, 0);
    for (int k = 0; k < N; ++k) uoff[(size_t)k + 1] = uoff[(size_t)k] + p.nu[(size_t)k];
    double resB = 0.0, resG = 0.0;
    for (int k = 0; k < N; ++k) {
      const int m = p.nu[(size_t)k];
      const double* A = p.rec.data() + dynOff[(size_t)k];
      const double* Bm = A + (size_t)nx * nx;
      const double* b = Bm + (size_t)nx * m;
      for (int i = 0; i < nx; ++i) {
        double v = b[i] - X(k + 1, i);
        for (int c = 0; c < nx; ++c) v += A[(size_t)c * nx + i] * X(k, c);
        for (int c = 0; c < m; ++c) v += Bm[(size_t)c * nx + i] * u[(size_t)uoff[(size_t)k] + c];
        resB = maxabs(resB, v);
      }
    }
    for (int k = 0; eq && k <= N; ++k) {
      const int rows = p.nc[(size_t)k];
      const int m = k < N ? p.nu[(size_t)k] : 0;
      const double* C = p.crec.data() + p.coff[(size_t)k];
      const double* D = C + (size_t)rows * nx;
      const double* e = D + (size_t)rows * m;
      for (int i = 0; i < rows; ++i) {
        double v = e[i];
        for (int c = 0; c < nx; ++c) v += C[(size_t)c * rows + i] * X(k, c);
        for (int c = 0; c < m; ++c) v += D[(size_t)c * rows + i] * u[(size_t)uoff[(size_t)k] + c];
        resB = maxabs(resB, v);
      }
    }
    if (eq) {
      resG = NAN;
    } else {  // lambda_N = Q x + q; g_u,k = R u + S x + r + B' lambda_{k+1}; lambda_k = Q x + S' u + q + A' lambda_{k+1}
      std::vector<double> lam((size_t)nx), ln((size_t)nx);
      {
        const double* Q = p.rec.data() + costOff[(size_t)N];
        const double* q = Q + (size_t)nx * nx;
        for (int i = 0; i < nx; ++i) {
          double v = q[i];
          for (int c = 0; c < nx; ++c) v += Q[(size_t)c * nx + i] * X(N, c);
          lam[(size_t)i] = v;
        }
      }
      for (int k = N - 1; k >= 0; --k) {
        const int m = p.nu[(size_t)k];
        const double* A = p.rec.data() + dynOff[(size_t)k];
        const double* Bm = A + (size_t)nx * nx;
        const double* Q = p.rec.data() + costOff[(size_t)k];
        const double* Sx = Q + (size_t)nx * nx;
        const double* R = Sx + (size_t)m * nx;
        const double* q = R + (size_t)m * m;
        const double* r = q + nx;
        const double* uk = u.data() + uoff[(size_t)k];
        for (int i = 0; i < m; ++i) {
          double v = r[i];
          for (int c = 0; c < m; ++c) v += R[(size_t)c * m + i] * uk[c];
          for (int c = 0; c < nx; ++c) v += Sx[(size_t)c * m + i] * X(k, c);
          for (int c = 0; c < nx; ++c) v += Bm[(size_t)i * nx + c] * lam[(size_t)c];
          resG = maxabs(resG, v);
        }
        for (int i = 0; i < nx; ++i) {
          double v = q[i];
          for (int c = 0; c < nx; ++c) v += Q[(size_t)c * nx + i] * X(k, c) + A[(size_t)i * nx + c] * lam[(size_t)c];
          for (int c = 0; c < m; ++c) v += Sx[(size_t)i * m + c] * uk[c];
          ln[(size_t)i] = v;
        }
        lam.swap(ln);
      }
    }
    std::fprintf(stderr, "\n=== HPIPM (MI355X engine, direct KKT solve) ===\n");
    std::fprintf(stderr, "HPIPM returned with flag %i. -> ", status);
    if (status == CMPC_SUCCESS) std::fprintf(stderr, "QP solved!\n");
    else if (status == CMPC_MAX_ITER) std::fprintf(stderr, "Solver failed! Maximum number of iterations reached\n");
    else if (status == CMPC_MIN_STEP) std::fprintf(stderr, "Solver failed! Minimum step length reached\n");
    else if (status == CMPC_NAN_SOL) std::fprintf(stderr, "Solver failed! NaN in computations\n");
    else if (status == CMPC_INCONS_EQ) std::fprintf(stderr, "Solver failed! Unconsistent equality constraints\n");
    else std::fprintf(stderr, "Solver failed! Unknown return flag\n");
    std::fprintf(stderr, "ipm iter = %d\n", 0);
    std::fprintf(stderr, "ipm residuals max: res_g = %e, res_b = %e, res_d = %e, res_m = %e\n", resG, resB, 0.0, 0.0);
    std::fprintf(stderr, "\nalpha_aff\tmu_aff\t\tsigma\t\talpha_prim\talpha_dual\tmu\t\tres_stat\tres_eq\t\tres_ineq\tres_comp\n");
    std::fprintf(stderr, "%e\t%e\t%e\t%e\t%e\t%e\t%e\t%e\t%e\t%e\t\n", (double)NAN, (double)NAN, (double)NAN, 1.0, 1.0, 0.0,
                 resG, resB, 0.0, 0.0);
  }

  Settings settings_;
  OcpSize size_;
  Packed last_;
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
