// k_policy.hip — feedback policy dU/dx0 of each condensed QP at its solution: the centroidal engine's counterpart
// of HpipmInterface::getRiccatiFeedback / getRiccatiFeedforward (HpipmInterface.cpp:330-455), which ocs2 turns into
// the linear feedback policy (MultipleShootingSolver::setPrimalSolution, MultipleShootingSolver.cpp:334-362,
// useFeedbackPolicy = true, MultipleShootingSettings.h:57). HPIPM reads its K off the last IPM factorisation
// (H + C' Sigma C); as mu -> 0, Sigma = lambda / s -> inf on active rows and -> 0 on inactive ones, so the limit is
// the derivative of the QP solution map on the active set, which is what this kernel returns:
//
//   K = -Z (Z' H Z)^{-1} Z' F,   F = dg/dx0 = Bqp' Q Aqp,   Z = blkdiag of per-triple free directions,
//
// restated in oracle/cmpc_oracle.c:oracle_policy (which builds F by a different route, forward block rows of Bqp;
// the kernel uses the adjoint recursion below). H is the condensed Hessian the condensing kernels left in the
// context workspace (class-packed, h_index).
//
// MI355X mapping: one 256-thread workgroup (4 waves) per QP; everything is small (N x 13 x 13 propagation, an
// m x m Cholesky with m <= n <= 256), so the per-QP working set sits in a global scratch slab that stays in L2 and
// the work is spread over the 256 lanes with a workgroup barrier between dependent phases. Not on the bench path.
//
//   forward  P_0 = I, P_{k+1} = A_k P_k                        (Aqp block rows, kept: (N+1) x 13 x 13)
//   backward Lam_N = Q_N P_N; rows of step j: F_j = B_j' Lam_{j+1}; Lam_j = Q_j P_j + A_j' Lam_{j+1}
#include "cmpc_device.hpp"
#include "cmpc_kernels.hpp"

namespace cmpc {

namespace {

constexpr int PT = 256;  // threads per QP

// Row-major A_k (13 x 13) into ab[0..168] and B_k (13 x 12) into ab[169..324]: the forward-Euler SRBD map of
// CentroidalMPC.cpp:85-92 with the lever arm frozen at p_{k,i} - c^ref_k (p: stance_point), or, with the SQP
// linearisation lk = (c_bar_k, F_bar_k), at p_{k,i} - c_bar_k plus dt [F_bar_k]x in the L rows / c columns
// (oracle_srbd_dynamics_lin). Entry-parallel over the workgroup.
__device__ void build_ab(const DevModel* M, const double* xr, const double* ft, const uint8_t* ct, int k,
                         const double* lk, double* ab) {
  const double dt = M->dt;
  const double psi = xr[k * NX + 11];
  const double cp = cos(psi), sp = sin(psi);
  for (int e = threadIdx.x; e < NX * (NX + NU); e += PT) {
    double v = 0.0;
    if (e < NX * NX) {
      const int r = e / NX, c = e % NX;
      if (r == c) v = 1.0;
      else if (lk && r >= 6 && r < 9 && c < 3) {  // L+ += dt F_bar x c
        const double* F = lk + 3;
        const double SF[9] = {0.0, -F[2], F[1], F[2], 0.0, -F[0], -F[1], F[0], 0.0};
        v = dt * SF[(r - 6) * 3 + c];
      } else if (r < 3 && c == r + 3) v = dt;
      else if (r == 5 && c == 12) v = dt;
      else if (r >= 9 && r < 12 && c >= 6 && c < 9) {
        const double RzT[9] = {cp, sp, 0.0, -sp, cp, 0.0, 0.0, 0.0, 1.0};
        const int a = r - 9, b = c - 6;
        double s = 0.0;
        for (int t = 0; t < 3; ++t) s += M->inv_inertia[a * 3 + t] * RzT[t * 3 + b];
        v = dt * s;
      }
    } else {
      const int r = (e - NX * NX) / NU, c = (e - NX * NX) % NU;
      const int i = c / 3, b = c % 3;
      if (ct[k * NL + i]) {
        if (r >= 3 && r < 6 && r - 3 == b) v = dt / M->mass;
        if (r >= 6 && r < 9) {
          double p[3];
          stance_point(ft, ct, M->N, k, i, p);
          const double* cb = lk ? lk : xr + (size_t)k * NX;
          const double rx = p[0] - cb[0], ry = p[1] - cb[1], rz = p[2] - cb[2];
          const double S[9] = {0.0, -rz, ry, rz, 0.0, -rx, -ry, rx, 0.0};
          v = dt * S[(r - 6) * 3 + b];
        }
      }
    }
    ab[e] = v;
  }
}

// Free directions of one force triple (oracle_policy_triple): orthonormal basis of the active pyramid rows in order
// r = 0..4, then greedy completion from e_0, e_1, e_2. Z[a * 3 + c]; returns the number of free directions.
__device__ int triple_basis(double mu, const double* ub, const double* f, double tol, double* Z) {
  const double nr[5][3] = {{-1.0, 0.0, mu}, {1.0, 0.0, mu}, {0.0, -1.0, mu}, {0.0, 1.0, mu}, {0.0, 0.0, 1.0}};
  double Q[3][3];
  int nq = 0;
  for (int r = 0; r < 5 && nq < 3; ++r) {
    const double v = nr[r][0] * f[0] + nr[r][1] * f[1] + nr[r][2] * f[2];
    if (!(v <= tol || ub[r] - v <= tol)) continue;
    double w[3] = {nr[r][0], nr[r][1], nr[r][2]};
    const double n0 = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    for (int p = 0; p < nq; ++p) {
      const double d = Q[p][0] * w[0] + Q[p][1] * w[1] + Q[p][2] * w[2];
      for (int a = 0; a < 3; ++a) w[a] -= d * Q[p][a];
    }
    const double nw = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    if (!(nw > 1e-6 * n0)) continue;
    for (int a = 0; a < 3; ++a) Q[nq][a] = w[a] / nw;
    ++nq;
  }
  const int rank = nq;
  for (int c = 0; c < 3 - rank; ++c) {
    double best[3] = {0.0, 0.0, 0.0}, bn = -1.0;
    for (int e = 0; e < 3; ++e) {
      double w[3] = {0.0, 0.0, 0.0};
      w[e] = 1.0;
      for (int p = 0; p < nq; ++p) {
        const double d = Q[p][0] * w[0] + Q[p][1] * w[1] + Q[p][2] * w[2];
        for (int a = 0; a < 3; ++a) w[a] -= d * Q[p][a];
      }
      const double nw = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
      if (nw > bn) {
        bn = nw;
        for (int a = 0; a < 3; ++a) best[a] = w[a];
      }
    }
    for (int a = 0; a < 3; ++a) Q[nq][a] = best[a] / bn;
    for (int a = 0; a < 3; ++a) Z[a * 3 + c] = Q[nq][a];
    ++nq;
  }
  return 3 - rank;
}

template <typename T>
__global__ __launch_bounds__(PT) void k_policy(PolicyArgs<T> a) {
  const int q = a.q0 + blockIdx.x;
  const int tid = threadIdx.x;
  const DevModel* M = a.model;
  const int N = M->N, nf = NU * N, ld = a.ld;
  double* Kq = a.K + (size_t)q * nf * NX;
  for (int e = tid; e < nf * NX; e += PT) Kq[e] = 0.0;
  const int st = a.status[q];
  if (st != CMPC_SUCCESS) {  // condensing rejected the QP (uniform over the workgroup)
    if (tid == 0) {
      a.status_out[q] = st;
      if (a.nfree) a.nfree[q] = 0;
    }
    return;
  }
  const int n = a.nvar[q], npad = ipm_class(n), nt = n / 3;
  const double* xr = a.xref + (size_t)q * (N + 1) * NX;
  const double* ft = a.foot + (size_t)q * (N + 1) * NL * 3;
  const uint8_t* ct = a.contact + (size_t)q * N * NL;
  double* P = a.scratch + (size_t)blockIdx.x * a.stride;  // [N+1][13][13]
  double* ab = P + (size_t)(N + 1) * NX * NX;             // A_k | B_k
  double* lam0 = ab + NX * (NX + NU);
  double* lam1 = lam0 + NX * NX;
  double* F = lam1 + NX * NX;                             // [12N][13]
  double* Z = F + (size_t)nf * NX;                        // [ld/3][9]
  double* Y = Z + (size_t)3 * ld;                         // [m][13]
  double* Hr = Y + (size_t)ld * NX;                       // [m][m]
  __shared__ int s_kt[CMPC_IPM_MAX_N / 3 + 1], s_off[CMPC_IPM_MAX_N / 3 + 1], s_idx[CMPC_IPM_MAX_N / 3 + 1];
  __shared__ short s_ct[CMPC_IPM_MAX_N], s_cc[CMPC_IPM_MAX_N];
  __shared__ int s_fail;

  // forward: Aqp block rows P_k
  for (int e = tid; e < NX * NX; e += PT) P[e] = (e / NX == e % NX) ? 1.0 : 0.0;
  for (int k = 0; k < N; ++k) {
    build_ab(M, xr, ft, ct, k, a.lin ? a.lin + ((size_t)q * N + k) * 6 : nullptr, ab);
    __syncthreads();
    const double* Pk = P + (size_t)k * NX * NX;
    double* Pn = P + (size_t)(k + 1) * NX * NX;
    for (int e = tid; e < NX * NX; e += PT) {
      const int r = e / NX, c = e % NX;
      double s = 0.0;
      for (int t = 0; t < NX; ++t) s += ab[r * NX + t] * Pk[t * NX + c];
      Pn[e] = s;
    }
    __syncthreads();
  }
  // backward adjoint: F rows of step j = B_j' Lam_{j+1}
  {
    const double* PN = P + (size_t)N * NX * NX;
    for (int e = tid; e < NX * NX; e += PT) lam0[e] = M->qdiag[N][e / NX] * PN[e];
  }
  double* lc = lam0;
  double* ln = lam1;
  for (int j = N - 1; j >= 0; --j) {
    build_ab(M, xr, ft, ct, j, a.lin ? a.lin + ((size_t)q * N + j) * 6 : nullptr, ab);
    __syncthreads();
    const double* Bj = ab + NX * NX;
    for (int e = tid; e < NU * NX; e += PT) {
      const int c = e / NX, col = e % NX;
      double s = 0.0;
      for (int r = 0; r < NX; ++r) s += Bj[r * NU + c] * lc[r * NX + col];
      F[(size_t)(NU * j + c) * NX + col] = s;
    }
    if (j > 0) {
      const double* Pj = P + (size_t)j * NX * NX;
      for (int e = tid; e < NX * NX; e += PT) {
        const int r = e / NX, col = e % NX;
        double s = M->qdiag[j][r] * Pj[e];
        for (int t = 0; t < NX; ++t) s += ab[t * NX + r] * lc[t * NX + col];
        ln[e] = s;
      }
    }
    __syncthreads();
    double* tmp = lc;
    lc = ln;
    ln = tmp;
  }

  // free directions of each stance triple (tri_map order = condensed variable order)
  if (tid < nt) {
    const int tm = a.tri_map[(size_t)q * (ld / 3) + tid];
    const int k = tm / NL, i = tm % NL;
    s_idx[tid] = NU * k + 3 * i;
    s_kt[tid] = triple_basis(M->mu[i], M->ub, a.u + ((size_t)(q * N + k) * NL + i) * 3, a.act_tol, Z + tid * 9);
  }
  __syncthreads();
  if (tid == 0) {
    int m = 0;
    for (int t = 0; t < nt; ++t) {
      s_off[t] = m;
      for (int c = 0; c < s_kt[t]; ++c, ++m) {
        s_ct[m] = (short)t;
        s_cc[m] = (short)c;
      }
    }
    s_off[nt] = m;
    s_fail = 0;
  }
  __syncthreads();
  const int m = s_off[nt];
  const T* Hq = a.H + (size_t)q * ld * ld;
  // reduced Hessian Z' H Z (lower triangle) and right-hand sides -Z' F
  for (int e = tid; e < m * m; e += PT) {
    const int r1 = e / m, r2 = e % m;
    if (r2 > r1) continue;
    const int t1 = s_ct[r1], c1 = s_cc[r1], t2 = s_ct[r2], c2 = s_cc[r2];
    double s = 0.0;
    for (int x = 0; x < 3; ++x) {
      double hz = 0.0;
      for (int y = 0; y < 3; ++y) hz += (double)Hq[h_index_sym(npad, 3 * t1 + x, 3 * t2 + y)] * Z[t2 * 9 + y * 3 + c2];
      s += Z[t1 * 9 + x * 3 + c1] * hz;
    }
    Hr[r1 * m + r2] = s;
  }
  for (int e = tid; e < m * NX; e += PT) {
    const int r = e / NX, col = e % NX;
    const int t = s_ct[r], c = s_cc[r];
    double s = 0.0;
    for (int x = 0; x < 3; ++x) s += Z[t * 9 + x * 3 + c] * F[(size_t)(s_idx[t] + x) * NX + col];
    Y[e] = -s;
  }
  __syncthreads();
  // right-looking Cholesky of the lower triangle
  for (int p = 0; p < m; ++p) {
    const double d = Hr[p * m + p];
    if (!(d > 0.0)) {
      if (tid == 0) s_fail = 1;
      break;  // d is read by every thread after the same barrier: uniform exit
    }
    const double l = sqrt(d);
    for (int i = p + 1 + tid; i < m; i += PT) Hr[i * m + p] = Hr[i * m + p] / l;
    __syncthreads();
    if (tid == 0) Hr[p * m + p] = l;
    const int w = m - p - 1;
    for (int e = tid; e < w * w; e += PT) {
      const int i = p + 1 + e / w, j = p + 1 + e % w;
      if (j <= i) Hr[i * m + j] -= Hr[i * m + p] * Hr[j * m + p];
    }
    __syncthreads();
  }
  __syncthreads();
  if (s_fail) {
    if (tid == 0) {
      a.status_out[q] = CMPC_NAN_SOL;
      if (a.nfree) a.nfree[q] = m;
    }
    return;
  }
  // 13 right-hand sides, one column per lane: L y = b, L' x = y
  if (tid < NX) {
    for (int i = 0; i < m; ++i) {
      double s = Y[i * NX + tid];
      for (int j = 0; j < i; ++j) s -= Hr[i * m + j] * Y[j * NX + tid];
      Y[i * NX + tid] = s / Hr[i * m + i];
    }
    for (int i = m - 1; i >= 0; --i) {
      double s = Y[i * NX + tid];
      for (int j = i + 1; j < m; ++j) s -= Hr[j * m + i] * Y[j * NX + tid];
      Y[i * NX + tid] = s / Hr[i * m + i];
    }
  }
  __syncthreads();
  // K rows of the stance forces: Z_t Y_t
  for (int e = tid; e < nt * 3 * NX; e += PT) {
    const int t = e / (3 * NX), x = (e / NX) % 3, col = e % NX;
    double s = 0.0;
    for (int c = 0; c < s_kt[t]; ++c) s += Z[t * 9 + x * 3 + c] * Y[(s_off[t] + c) * NX + col];
    Kq[(size_t)(s_idx[t] + x) * NX + col] = s;
  }
  if (tid == 0) {
    a.status_out[q] = CMPC_SUCCESS;
    if (a.nfree) a.nfree[q] = m;
  }
}

}  // namespace

size_t policy_scratch_doubles(int N, int ld) {
  const size_t nf = (size_t)NU * N;
  return (size_t)(N + 1) * NX * NX + NX * (NX + NU) + 2 * NX * NX + nf * NX + 3 * (size_t)ld + (size_t)ld * NX +
         (size_t)ld * ld;
}

template <typename T>
int launch_policy(const PolicyArgs<T>& a, int nq, hipStream_t stream) {
  if (nq <= 0) return 0;
  hipLaunchKernelGGL(k_policy<T>, dim3(nq), dim3(PT), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
template int launch_policy<double>(const PolicyArgs<double>&, int, hipStream_t);
template int launch_policy<float>(const PolicyArgs<float>&, int, hipStream_t);

}  // namespace cmpc
