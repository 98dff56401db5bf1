// k_ocp.hip — stage-wise OCP-QP interior-point solver on the device: the HpipmInterface::solve path (reference
// ocs2_sqp/hpipm_catkin/src/HpipmInterface.cpp:166-301) for problems of the ocs2_legged_robot size (nx = 24,
// nu_k <= 24, N ~ 70; ocs2_legged_robot/config/mpc/task.info:33, :102), batched.
//
// Algorithm: HPIPM's OCP IPM as restated by oracle/ocp_ipm.c (x0 eliminated, HpipmInterface.cpp:177-208; the
// constraint rows C x + D u + e = 0 as two-sided general constraints lg = ug = -e, :223-264; Mehrotra predictor-
// corrector, one step length, tau = 0.995, the Settings of HpipmInterfaceSettings.h:44-57 honoured). Every Newton
// system is solved stage-wise:
//   - factorisation (backward over the stages, the only heavy serial chain): per stage the augmented symmetric matrix
//       M = [B A rb; 0 0 1]' [P p; p' 0] [B A rb; 0 0 1] + [R~ S~' g_u; S~ Q~ g_x; g_u' g_x' 0] + Gc' Sigma Gc
//     (rows/columns u | x | rhs) is formed in a register tile (16 x 16 threads, each an R x R cyclic tile) and the
//     u block is eliminated by nu_k Gauss-Jordan sweep steps (one workgroup barrier each): the swept matrix holds
//     K = -M_uu^-1 M_ux, P_k = M_xx - M_xu M_uu^-1 M_ux, kff and p_k at once, and the pivot columns are the LDL'
//     factor of M_uu (kept: the corrector's feedforward and HPIPM's ric_Lr come from it by triangular solves);
//     P_k, p_k stay in LDS for the next stage, whose data was prefetched into registers during the sweep;
//   - everything else is stage-parallel (residuals, right-hand sides, A + B K, the row directions) except two cheap
//     serial nx x nx matrix-vector chains (forward dx_{k+1} = (A + BK) dx_k + bcl_k; backward
//     p_k = (A + BK)' p_{k+1} + h_k for the corrector's right-hand side).
// One workgroup of 256 threads per problem; problem-major workspace allocated once per cmpc_ocp handle.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

#include "k_ocp.hpp"

namespace cmpc {
namespace {

constexpr int NT = OCP_NT;
typedef double v4d __attribute__((ext_vector_type(4)));
constexpr double TAU_OCP = 0.995;  // fraction-to-boundary, as oracle/ocp_ipm.c

// Lab instrumentation (-DCMPC_OCP_STAMPS, lab/ocp_stamps.sh only, never in libcmpc.so): thread 0 of problem 0
// accumulates shader-clock cycles per phase (s_memtime) into a device array read by cmpc_ocp_debug_stamps.
#ifdef CMPC_OCP_STAMPS
// thread 0 of problem 0 accumulates in LDS (no global round trip on the timed path) and adds to the device array at
// the kernel's end
__device__ unsigned long long ocp_stamp_acc[48];
__shared__ unsigned long long ocp_stamp_lds[49];
#define OCP_STAMP(id)                                                         \
  do {                                                                        \
    if (blockIdx.x == 0 && threadIdx.x == 0) {                                \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime();           \
      ocp_stamp_lds[id] += now_ - ocp_stamp_lds[48];                          \
      ocp_stamp_lds[48] = now_;                                               \
    }                                                                         \
  } while (0)
// a span of one thread other than 0 (t, e.g. a helper wave's work): cycles between OCP_SPAN_BEGIN and OCP_SPAN_END
#define OCP_SPAN_BEGIN(var) const unsigned long long var = __builtin_amdgcn_s_memtime()
#define OCP_SPAN_END(id, var, t)                                                          \
  do {                                                                                    \
    if (blockIdx.x == 0 && threadIdx.x == (t)) ocp_stamp_lds[id] += __builtin_amdgcn_s_memtime() - (var); \
  } while (0)
// a span of thread 0 of workgroup blk, added straight to the device array (another workgroup's timeline)
#define OCP_SPANG_END(id, var, blk)                                                                          \
  do {                                                                                                       \
    if (blockIdx.x == (blk) && threadIdx.x == 0)                                                             \
      __hip_atomic_fetch_add(&ocp_stamp_acc[id], __builtin_amdgcn_s_memtime() - (var), __ATOMIC_RELAXED,     \
                             __HIP_MEMORY_SCOPE_AGENT);                                                      \
  } while (0)
#define OCP_STAMP_BEGIN()                                                     \
  do {                                                                        \
    if (blockIdx.x == 0 && threadIdx.x == 0) {                                \
      for (int i_ = 0; i_ < 48; ++i_) ocp_stamp_lds[i_] = 0;                  \
      ocp_stamp_lds[48] = __builtin_amdgcn_s_memtime();                       \
    }                                                                         \
  } while (0)
#define OCP_STAMP_END()                                                       \
  do {                                                                        \
    if (blockIdx.x == 0 && threadIdx.x == 0)                                  \
      for (int i_ = 0; i_ < 48; ++i_) ocp_stamp_acc[i_] += ocp_stamp_lds[i_]; \
  } while (0)
#else
#define OCP_STAMP(id) \
  do {                \
  } while (0)
#define OCP_STAMP_BEGIN() \
  do {                    \
  } while (0)
#define OCP_SPAN_BEGIN(var) \
  do {                      \
  } while (0)
#define OCP_SPAN_END(id, var, t) \
  do {                           \
  } while (0)
#define OCP_SPANG_END(id, var, blk) \
  do {                              \
  } while (0)
#define OCP_STAMP_END() \
  do {                  \
  } while (0)
#endif

__device__ __forceinline__ double nmax(double a, double b) {
  return (a != a || b != b) ? __builtin_nan("") : (a > b ? a : b);
}
struct OpMax {
  __device__ double operator()(double a, double b) const { return nmax(a, b); }
};
struct OpMin {
  __device__ double operator()(double a, double b) const { return a < b ? a : b; }
};
struct OpSum {
  __device__ double operator()(double a, double b) const { return a + b; }
};

template <class Op>
__device__ __forceinline__ double block_reduce(double v, double* red, Op op) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = red[0];
#pragma unroll
  for (int w = 1; w < NT / 64; ++w) r = op(r, red[w]);
  return r;
}

// Per-problem view: record blocks, constraint blocks and workspace arrays of problem q
struct View {
  const OcpLayout& L;
  const double* rec;
  const double* crec;
  double* ws;
  int NP;
  __device__ __forceinline__ View(const OcpSolveArgs& a, int q)
      : L(a.L),
        rec(a.rec + (long long)q * a.L.rec_size),
        crec(a.crec ? a.crec + (long long)q * a.L.crec_size : nullptr),
        ws(a.ws + (long long)q * a.L.ws_stride),
        NP(a.L.N + 1) {}
  __device__ const double* A(int k) const { return rec + L.orec[8 * k + 0]; }
  __device__ const double* Bm(int k) const { return rec + L.orec[8 * k + 1]; }
  __device__ const double* b(int k) const { return rec + L.orec[8 * k + 2]; }
  __device__ const double* Q(int k) const { return rec + L.orec[8 * k + 3]; }
  __device__ const double* S(int k) const { return rec + L.orec[8 * k + 4]; }
  __device__ const double* R(int k) const { return rec + L.orec[8 * k + 5]; }
  __device__ const double* q(int k) const { return rec + L.orec[8 * k + 6]; }
  __device__ const double* r(int k) const { return rec + L.orec[8 * k + 7]; }
  __device__ const double* C(int k) const { return crec + L.ocon[4 * k + 0]; }
  __device__ const double* D(int k) const { return crec + L.ocon[4 * k + 1]; }
  __device__ const double* e(int k) const { return crec + L.ocon[4 * k + 2]; }
  __device__ double* row(int i) const { return ws + L.o_rows + (long long)i * L.m; }
  __device__ double* x() const { return ws + L.o_x; }
  __device__ double* u() const { return ws + L.o_u; }
  __device__ double* pi() const { return ws + L.o_pi; }
  __device__ double* rgu() const { return ws + L.o_rgu; }
  __device__ double* rgx() const { return ws + L.o_rgx; }
  __device__ double* rb() const { return ws + L.o_rb; }
  __device__ double* gu() const { return ws + L.o_gu; }
  __device__ double* gx() const { return ws + L.o_gx; }
  __device__ double* du() const { return ws + L.o_du; }
  __device__ double* dx() const { return ws + L.o_dx; }
  __device__ double* dpi() const { return ws + L.o_dpi; }
  __device__ double* P(int k) const { return ws + L.o_P + (long long)k * L.nx * L.nx; }
  __device__ double* pv() const { return ws + L.o_pv; }
  __device__ double* K(int k) const { return ws + L.o_K + L.cK[k]; }
  __device__ double* kf() const { return ws + L.o_kf; }
  __device__ double* Lf(int k) const { return ws + L.o_Lf + L.cM[k]; }
  __device__ double* Acl(int k) const { return ws + L.o_Acl + (long long)k * L.nx * L.nx; }
  __device__ double* h() const { return ws + L.o_h; }
  __device__ double* y() const { return ws + L.o_y; }
  __device__ double* bcl() const { return ws + L.o_bcl; }
};

// LDS carve
struct Lds {
  double *Paug, *ABx, *Tx, *col, *vec, *red, *sgn;
  int np1, nrm, nzp;
};
__device__ __forceinline__ Lds carve(double* smem, const OcpLayout& L, int NZP) {
  Lds s;
  s.np1 = L.nx + 1;
  s.nrm = L.nx + 1 + L.ngmax;
  s.nzp = NZP;
  const int pa = (s.np1 * s.np1 + 1) & ~1;
  s.Paug = smem;
  s.ABx = s.Paug + pa;
  s.Tx = s.ABx + s.nrm * NZP;
  s.col = s.Tx + s.nrm * NZP;
  s.vec = s.col + 4 * NZP;
  s.red = s.vec + 128;
  s.sgn = s.red + 64;
  return s;
}

// Workgroup barrier for LDS traffic only: lgkmcnt(0) and s_barrier, without the vmcnt(0) of __syncthreads(), so the
// next stage's global prefetch (registers) stays in flight across the sweep's barriers instead of being waited for at
// the first one. Used inside the factorisation's stage loop, whose threads exchange data through LDS only.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// c = C x + D u for every row (node 0's x is x0; the step's dx node 0 is 0)
// s + sum_{c<n} a[c as] b[c] in that fma order (the loop's), the loads of 16 terms issued before their fmas: one
// L2 round trip per 16 terms instead of per 8 (the unrolled loop's batches)
__device__ __forceinline__ double dotb(double s, const double* a, int as, const double* b, int n) {
  for (int c0 = 0; c0 < n; c0 += 16) {
    double av[16], bv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int c = c0 + u < n ? c0 + u : n - 1;
      av[u] = a[(long long)c * as];
      bv[u] = b[c];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (c0 + u < n) s = fma(av[u], bv[u], s);
  }
  return s;
}
__device__ __forceinline__ void rows_value(const View& V, const double* xs, const double* us, double* out, int j0 = 0,
                                           int j1 = -1) {
  const OcpLayout& L = V.L;
  if (j1 < 0) j1 = L.m;
  for (int j = j0 + threadIdx.x; j < j1; j += NT) {
    const int k = L.rstage[j], jl = j - L.cr[k], g = L.ng[k], mk = L.nu[k];
    const double* C = V.C(k);
    const double* D = V.D(k);
    double s = dotb(0.0, C + jl, g, xs + (long long)k * L.nx, L.nx);
    s = dotb(s, D + jl, g, us + L.cu[k], mk);
    out[j] = s;
  }
}

// out_u += D' v, out_x += C' v (x part for nodes >= 1), per entry over the node's rows
__device__ __forceinline__ double gct_u(const View& V, int k, int a, const double* v) {
  const int g = V.L.ng[k];
  const double* D = V.D(k);
  const double* vk = v + V.L.cr[k];
  double s = 0.0;
  for (int j = 0; j < g; ++j) s = fma(D[(long long)a * g + j], vk[j], s);
  return s;
}
__device__ __forceinline__ double gct_x(const View& V, int k, int i, const double* v) {
  const int g = V.L.ng[k];
  const double* C = V.C(k);
  const double* vk = v + V.L.cr[k];
  double s = 0.0;
  for (int j = 0; j < g; ++j) s = fma(C[(long long)i * g + j], vk[j], s);
  return s;
}

// Stationarity and dynamics residuals at (x, u, pi, l_l - l_u); returns the local max of |r_g| (rs) and |r_b| (re)
__device__ __forceinline__ void residuals(const View& V, double& rs, double& re) {
  const OcpLayout& L = V.L;
  const int nx = L.nx, N = L.N;
  const double* x = V.x();
  const double* u = V.u();
  const double* pi = V.pi();
  double* wl = V.row(R_W);  // l_l - l_u, prepared by the caller
  const int nU = L.nU, nXr = N * nx;
  for (int it = threadIdx.x; it < nU + 2 * nXr; it += NT) {
    if (it < nU) {
      const int k = L.ustage[it], a = it - L.cu[k], mk = L.nu[k];
      const double* R = V.R(k);
      const double* S = V.S(k);
      const double* Bm = V.Bm(k);
      double s = V.r(k)[a];
      for (int c = 0; c < mk; ++c) s = fma(R[(long long)c * mk + a], u[L.cu[k] + c], s);
      for (int j = 0; j < nx; ++j) s = fma(S[(long long)j * mk + a], x[(long long)k * nx + j], s);
      for (int t = 0; t < nx; ++t) s = fma(Bm[(long long)a * nx + t], pi[(long long)k * nx + t], s);
      s -= gct_u(V, k, a, wl);
      V.rgu()[it] = s;
      rs = nmax(rs, fabs(s));
    } else if (it < nU + nXr) {
      const int e = it - nU, k = 1 + e / nx, i = e % nx, mk = L.nu[k];
      const double* Q = V.Q(k);
      const double* S = V.S(k);
      double s = V.q(k)[i] - pi[(long long)(k - 1) * nx + i];
      for (int j = 0; j < nx; ++j) s = fma(Q[(long long)j * nx + i], x[(long long)k * nx + j], s);
      for (int a = 0; a < mk; ++a) s = fma(S[(long long)i * mk + a], u[L.cu[k] + a], s);
      if (k < N) {
        const double* A = V.A(k);
        for (int t = 0; t < nx; ++t) s = fma(A[(long long)i * nx + t], pi[(long long)k * nx + t], s);
      }
      s -= gct_x(V, k, i, wl);
      V.rgx()[(long long)k * nx + i] = s;
      rs = nmax(rs, fabs(s));
    } else {
      const int e = it - nU - nXr, k = e / nx, i = e % nx, mk = L.nu[k];
      const double* A = V.A(k);
      const double* Bm = V.Bm(k);
      double s = V.b(k)[i] - x[(long long)(k + 1) * nx + i];
      for (int j = 0; j < nx; ++j) s = fma(A[(long long)j * nx + i], x[(long long)k * nx + j], s);
      for (int a = 0; a < mk; ++a) s = fma(Bm[(long long)a * nx + i], u[L.cu[k] + a], s);
      V.rb()[(long long)k * nx + i] = s;
      re = nmax(re, fabs(s));
    }
  }
}

// Residuals of every node at once: r_gu (u rows), r_gx (x rows, k >= 1) and r_b (dynamics, k < N) of node k depend on
// that node's data and the current iterate only, so all nodes' outputs are spread over the workgroup (slot e of node k
// at k P + e, P = nzp + nx >= nu_k + 2 nx) with operands straight from the L2-resident records / iterate and no
// barrier between nodes; each output is the same fma chain as the node-by-node form (bit-identical). Used for
// B <= OCP_PAR_RES_MAX (OcpSolveArgs::par_res). Node by node,
// with ~72 of 256 threads busy and two barriers per node, it held a B = 1 solve 21 % longer (projected; rows 16 %);
// its L2 traffic is ~2.5x the staged form's, which wins for full batches (-14 % solves/s at B = 256, -11 % at 1024
// with this form).
constexpr int OCP_PAR_RES_MAX = 64;
__device__ __forceinline__ void residuals_par(const View& V, double& rs, double& re, int n0 = 0, int n1 = -1) {
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, nx = L.nx, N = L.N;
  const double *x = V.x(), *u = V.u(), *pi = V.pi(), *wl = V.row(R_W);
  const int P = L.nzp + nx;
  if (n1 < 0) n1 = N + 1;
  for (int w = n0 * P + tid; w < n1 * P; w += NT) {
    const int k = w / P, e = w - k * P;
    const int mk = L.nu[k], g = L.ng[k];
    const int n1 = mk, n2 = k >= 1 ? nx : 0, n3 = k < N ? nx : 0;
    if (e >= n1 + n2 + n3) continue;
    const double* A = V.A(k);
    const double* Bm = V.Bm(k);
    const double* xk = x + (long long)k * nx;
    const double* uk = u + L.cu[k];
    const double* pk = pi + (long long)k * nx;
    const double* wk = wl + L.cr[k];
    if (e < n1) {
      const int a = e;
      const double *R = V.R(k), *Sm = V.S(k);
      double s = V.r(k)[a];
      s = dotb(s, R + a, mk, uk, mk);
      s = dotb(s, Sm + a, mk, xk, nx);
      s = dotb(s, Bm + a * nx, 1, pk, n3);
      double d = 0.0;
      if (g) d = dotb(d, V.D(k) + a * g, 1, wk, g);
      s -= d;
      V.rgu()[L.cu[k] + a] = s;
      rs = nmax(rs, fabs(s));
    } else if (e < n1 + n2) {
      const int i = e - n1;
      const double *Q = V.Q(k), *Sm = V.S(k);
      const double* pm = pi + (long long)(k - 1) * nx;
      double s = V.q(k)[i] - pm[i];
      s = dotb(s, Q + i, nx, xk, nx);
      s = dotb(s, Sm + i * mk, 1, uk, mk);
      s = dotb(s, A + i * nx, 1, pk, n3);
      double d = 0.0;
      if (g) d = dotb(d, V.C(k) + i * g, 1, wk, g);
      s -= d;
      V.rgx()[(long long)k * nx + i] = s;
      rs = nmax(rs, fabs(s));
    } else {
      const int i = e - n1 - n2;
      const double* xn = x + (long long)(k + 1) * nx;
      double s = V.b(k)[i] - xn[i];
      s = dotb(s, A + i, nx, xk, nx);
      s = dotb(s, Bm + i, nx, uk, mk);
      V.rb()[(long long)k * nx + i] = s;
      re = nmax(re, fabs(s));
    }
  }
  __syncthreads();
}

// The same residuals one node at a time, the node's matrices staged in LDS (ABx and Tx as one buffer): the
// transposed products (B'pi, A'pi, S'u, D'w, C'w) read LDS instead of strided global loads, and the next node's
// matrices are loaded into registers while this one computes. A node whose matrices exceed the staging (nu_k far
// above nx) reads them from global memory.
struct NodeMats {
  int nA, nB, nQ, nS, nR, nC, nD, oB, oQ, oS, oR, oC, oD, tot;
};
__device__ __forceinline__ NodeMats node_mats(const OcpLayout& L, int k) {
  NodeMats M;
  const int nx = L.nx, mk = L.nu[k], g = L.ng[k];
  M.nA = k < L.N ? nx * nx : 0;
  M.nB = k < L.N ? nx * mk : 0;
  M.nQ = nx * nx;
  M.nS = mk * nx;
  M.nR = mk * mk;
  M.nC = g * nx;
  M.nD = g * mk;
  M.oB = M.nA;
  M.oQ = M.oB + M.nB;
  M.oS = M.oQ + M.nQ;
  M.oR = M.oS + M.nS;
  M.oC = M.oR + M.nR;
  M.oD = M.oC + M.nC;
  M.tot = M.oD + M.nD;
  return M;
}
__device__ __forceinline__ double node_load(const View& V, const NodeMats& M, int k, int e) {
  const double* p = e < M.oB   ? V.A(k) + e
                    : e < M.oQ ? V.Bm(k) + (e - M.oB)
                    : e < M.oS ? V.Q(k) + (e - M.oQ)
                    : e < M.oR ? V.S(k) + (e - M.oS)
                    : e < M.oC ? V.R(k) + (e - M.oR)
                    : e < M.oD ? V.C(k) + (e - M.oC)
                               : V.D(k) + (e - M.oD);
  return *p;
}
// The node's vectors staged beside its matrices: r, q, b, x_k, u_k, pi_k, pi_{k-1}, x_{k+1}, w_k, so the node's
// products read LDS only (a global load inside the dot-product loops is a full memory latency per node at B = 1)
struct NodeVecs {
  int o_q, o_b, o_x, o_u, o_pk, o_pm, o_xn, o_w, tot;
};
__device__ __forceinline__ NodeVecs node_vecs(const OcpLayout& L, int k) {
  NodeVecs W;
  const int nx = L.nx, mk = L.nu[k], g = L.ng[k], nd = k < L.N ? nx : 0;
  W.o_q = mk;
  W.o_b = W.o_q + nx;
  W.o_x = W.o_b + nd;
  W.o_u = W.o_x + nx;
  W.o_pk = W.o_u + mk;
  W.o_pm = W.o_pk + nd;
  W.o_xn = W.o_pm + (k >= 1 ? nx : 0);
  W.o_w = W.o_xn + nd;
  W.tot = W.o_w + g;
  return W;
}
__device__ __forceinline__ double vec_load(const View& V, const NodeVecs& W, int k, int e) {
  const OcpLayout& L = V.L;
  const int nx = L.nx;
  const double* p = e < W.o_q    ? V.r(k) + e
                    : e < W.o_b  ? V.q(k) + (e - W.o_q)
                    : e < W.o_x  ? V.b(k) + (e - W.o_b)
                    : e < W.o_u  ? V.x() + (long long)k * nx + (e - W.o_x)
                    : e < W.o_pk ? V.u() + L.cu[k] + (e - W.o_u)
                    : e < W.o_pm ? V.pi() + (long long)k * nx + (e - W.o_pk)
                    : e < W.o_xn ? V.pi() + (long long)(k - 1) * nx + (e - W.o_pm)
                    : e < W.o_w  ? V.x() + (long long)(k + 1) * nx + (e - W.o_xn)
                                 : V.row(R_W) + L.cr[k] + (e - W.o_w);
  return *p;
}
__device__ __forceinline__ void residuals_staged(const View& V, const Lds& S, double& rs, double& re) {
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, nx = L.nx, N = L.N;
  const double *x = V.x(), *u = V.u(), *pi = V.pi(), *wl = V.row(R_W);
  double* buf = S.ABx;  // ABx and Tx are contiguous
  const int cap = 2 * S.nrm * S.nzp;
  constexpr int EPR = 16, EPV = 2;
  auto staged = [&](const NodeMats& M, const NodeVecs& W) {
    return M.tot + W.tot <= cap && M.tot <= EPR * NT && W.tot <= EPV * NT;
  };
  double pre[EPR], prv[EPV];
  {
    const NodeMats M0 = node_mats(L, 0);
    const NodeVecs W0 = node_vecs(L, 0);
    if (staged(M0, W0)) {
      for (int e = tid; e < M0.tot; e += NT) buf[e] = node_load(V, M0, 0, e);
      for (int e = tid; e < W0.tot; e += NT) buf[M0.tot + e] = vec_load(V, W0, 0, e);
    }
  }
  __syncthreads();
  for (int k = 0; k <= N; ++k) {
    const NodeMats M = node_mats(L, k);
    const NodeVecs W = node_vecs(L, k);
    const bool st = staged(M, W);
    const int mk = L.nu[k], g = L.ng[k];
    const NodeMats Mn = node_mats(L, k < N ? k + 1 : k);
    const NodeVecs Wn = node_vecs(L, k < N ? k + 1 : k);
    const bool pn = k < N && staged(Mn, Wn);
    if (pn) {
#pragma unroll
      for (int q = 0; q < EPR; ++q) {
        const int e = tid + NT * q;
        pre[q] = e < Mn.tot ? node_load(V, Mn, k + 1, e) : 0.0;
      }
#pragma unroll
      for (int q = 0; q < EPV; ++q) {
        const int e = tid + NT * q;
        prv[q] = e < Wn.tot ? vec_load(V, Wn, k + 1, e) : 0.0;
      }
    }
    const double* A = st ? buf : V.A(k);
    const double* Bm = st ? buf + M.oB : V.Bm(k);
    const double* Q = st ? buf + M.oQ : V.Q(k);
    const double* Sm = st ? buf + M.oS : V.S(k);
    const double* R = st ? buf + M.oR : V.R(k);
    const double* C = st ? buf + M.oC : (g ? V.C(k) : nullptr);
    const double* D = st ? buf + M.oD : (g ? V.D(k) : nullptr);
    const double* vb = buf + M.tot;
    const double* rk = st ? vb : V.r(k);
    const double* qk = st ? vb + W.o_q : V.q(k);
    const double* bk = st ? vb + W.o_b : V.b(k);
    const double* xk = st ? vb + W.o_x : x + (long long)k * nx;
    const double* uk = st ? vb + W.o_u : u + L.cu[k];
    const double* pk = st ? vb + W.o_pk : pi + (long long)k * nx;
    const double* pm = st ? vb + W.o_pm : pi + (long long)(k - 1) * nx;
    const double* xn = st ? vb + W.o_xn : x + (long long)(k + 1) * nx;
    const double* wk = st ? vb + W.o_w : wl + L.cr[k];
    const int n1 = mk, n2 = k >= 1 ? nx : 0, n3 = k < N ? nx : 0;
    for (int e = tid; e < n1 + n2 + n3; e += NT) {
      if (e < n1) {
        const int a = e;
        double s = rk[a];
        for (int c = 0; c < mk; ++c) s = fma(R[c * mk + a], uk[c], s);
        for (int j = 0; j < nx; ++j) s = fma(Sm[j * mk + a], xk[j], s);
        for (int t = 0; t < n3; ++t) s = fma(Bm[a * nx + t], pk[t], s);
        double d = 0.0;
        for (int j = 0; j < g; ++j) d = fma(D[a * g + j], wk[j], d);
        s -= d;
        V.rgu()[L.cu[k] + a] = s;
        rs = nmax(rs, fabs(s));
      } else if (e < n1 + n2) {
        const int i = e - n1;
        double s = qk[i] - pm[i];
        for (int j = 0; j < nx; ++j) s = fma(Q[j * nx + i], xk[j], s);
        for (int a = 0; a < mk; ++a) s = fma(Sm[i * mk + a], uk[a], s);
        for (int t = 0; t < n3; ++t) s = fma(A[i * nx + t], pk[t], s);
        double d = 0.0;
        for (int j = 0; j < g; ++j) d = fma(C[i * g + j], wk[j], d);
        s -= d;
        V.rgx()[(long long)k * nx + i] = s;
        rs = nmax(rs, fabs(s));
      } else {
        const int i = e - n1 - n2;
        double s = bk[i] - xn[i];
        for (int j = 0; j < nx; ++j) s = fma(A[j * nx + i], xk[j], s);
        for (int a = 0; a < mk; ++a) s = fma(Bm[a * nx + i], uk[a], s);
        V.rb()[(long long)k * nx + i] = s;
        re = nmax(re, fabs(s));
      }
    }
    if (k < N) {
      lds_barrier();  // every thread is done with node k's staging buffer
      if (pn) {
#pragma unroll
        for (int q = 0; q < EPR; ++q) {
          const int e = tid + NT * q;
          if (e < Mn.tot) buf[e] = pre[q];
        }
#pragma unroll
        for (int q = 0; q < EPV; ++q) {
          const int e = tid + NT * q;
          if (e < Wn.tot) buf[Mn.tot + e] = prv[q];
        }
      }
      lds_barrier();
    }
  }
  __syncthreads();
}

// Step right-hand side over stages [k0, k1) (u entries) and nodes [max(k0, 1), n1) (x entries)
__device__ __forceinline__ void step_rhs_range(const View& V, int k0, int k1, int n1) {
  const OcpLayout& L = V.L;
  const int nx = L.nx, u0 = L.cu[k0], u1 = L.cu[k1], x0 = (k0 > 1 ? k0 : 1) * nx, x1 = n1 * nx;
  const double* w = V.row(R_W);
  const int nu = u1 - u0, nxr = x1 > x0 ? x1 - x0 : 0;
  for (int it = threadIdx.x; it < nu + nxr; it += NT) {
    if (it < nu) {
      const int e = u0 + it, k = L.ustage[e], a = e - L.cu[k];
      V.gu()[e] = V.rgu()[e] + gct_u(V, k, a, w);
    } else {
      const int e = x0 + it - nu, k = e / nx, i = e - k * nx;
      V.gx()[e] = V.rgx()[e] + gct_x(V, k, i, w);
    }
  }
}

// Step right-hand side g = r_g + Gc' w (node 0 has no state entries)
__device__ __forceinline__ void step_rhs(const View& V) {
  const OcpLayout& L = V.L;
  const int nx = L.nx, nXr = L.N * nx;
  const double* w = V.row(R_W);
  for (int it = threadIdx.x; it < L.nU + nXr; it += NT) {
    if (it < L.nU) {
      const int k = L.ustage[it], a = it - L.cu[k];
      V.gu()[it] = V.rgu()[it] + gct_u(V, k, a, w);
    } else {
      const int e = it - L.nU, k = 1 + e / nx, i = e % nx;
      V.gx()[(long long)k * nx + i] = V.rgx()[(long long)k * nx + i] + gct_x(V, k, i, w);
    }
  }
}

// Stage k's augmented data rows (LDS image [nrk][NZP]): rows 0..nx-1 = [B A rb], row nx = [0 0 1],
// rows nx+1.. = [D C 0] (their T rows are Sigma times them). Element loads are branch-light: one address selected,
// one unconditional load (from a valid dummy address for the constant entries), then a select.
struct StagePtrs {
  const double *A, *B, *rb, *C, *D;
  int mk, nz, g;
};
__device__ __forceinline__ StagePtrs stage_ptrs(const View& V, int k) {
  StagePtrs P;
  const int nx = V.L.nx;
  P.mk = V.L.nu[k];
  P.nz = P.mk + nx;
  P.g = V.L.ng[k];
  P.A = V.A(k);
  P.B = V.Bm(k);
  P.rb = V.rb() + (long long)k * nx;
  P.C = P.g ? V.C(k) : P.rb;
  P.D = P.g ? V.D(k) : P.rb;
  return P;
}
__device__ __forceinline__ double stage_load(const StagePtrs& P, int nx, int r, int l) {
  const double* p = P.rb;
  double cst = 0.0;
  bool use = false;
  if (l <= P.nz) {
    if (r < nx) {
      use = true;
      p = l < P.mk ? P.B + (long long)l * nx + r : (l < P.nz ? P.A + (long long)(l - P.mk) * nx + r : P.rb + r);
    } else if (r == nx) {
      cst = l == P.nz ? 1.0 : 0.0;
    } else if (l < P.nz) {
      const int j = r - nx - 1;
      use = true;
      p = l < P.mk ? P.D + (long long)l * P.g + j : P.C + (long long)(l - P.mk) * P.g + j;
    }
  }
  const double v = *p;
  return use ? v : cst;
}

// Stage k's Hessian / right-hand-side block [R~ S~' g_u; S~ Q~ g_x; g_u' g_x' 0] (reg on the R and Q diagonals)
struct HPtrs {
  const double *R, *S, *Q, *gu, *gx;
  int mk, nz;
};
__device__ __forceinline__ HPtrs h_ptrs(const View& V, int k) {
  HPtrs H;
  H.mk = V.L.nu[k];
  H.nz = H.mk + V.L.nx;
  H.R = V.R(k);
  H.S = V.S(k);
  H.Q = V.Q(k);
  H.gu = V.gu() + V.L.cu[k];
  H.gx = V.gx() + (long long)k * V.L.nx;
  return H;
}
__device__ __forceinline__ double h_load(const HPtrs& H, int nx, int i, int l, double reg) {
  // (a select-only, branch-free form of this was measured 4-9 % slower on MI355X: more VGPRs, more spills)
  const double* p = H.gx;
  bool use = false;
  double add = 0.0;
  if (i <= H.nz && l <= H.nz && !(i == H.nz && l == H.nz)) {
    use = true;
    if (l == H.nz) {
      p = i < H.mk ? H.gu + i : H.gx + (i - H.mk);
    } else if (i == H.nz) {
      p = l < H.mk ? H.gu + l : H.gx + (l - H.mk);
    } else if (i < H.mk && l < H.mk) {
      p = H.R + (long long)l * H.mk + i;
      add = i == l ? reg : 0.0;
    } else if (i < H.mk) {
      p = H.S + (long long)(l - H.mk) * H.mk + i;
    } else if (l < H.mk) {
      p = H.S + (long long)(i - H.mk) * H.mk + l;
    } else {
      p = H.Q + (long long)(l - H.mk) * nx + (i - H.mk);
      add = i == l ? reg : 0.0;
    }
  }
  const double v = *p;
  return use ? v + add : 0.0;
}

template <int NZP>
struct StagePrefetch {
  static constexpr int EPT = NZP == 64 ? (64 * 64) / NT : 1;  // register prefetch for the 64 class only
  double v[EPT];
};


// Backward factorisation of the barrier-weighted Newton matrix with the right-hand side (gu, gx, rb) of ws.
// Writes P_k, pv_k (k = 0..N), K_k, kf_k and the LDL' columns Lf_k (k = 0..N-1). Returns false on a NaN pivot.
template <int NZP>
__device__ __forceinline__ bool factor_pass(const View& V, const Lds& S, double reg) {
  constexpr int R = NZP / 16;
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, ti = tid & 15, tj = tid >> 4;
  const int N = L.N, nx = L.nx, np1 = nx + 1;
  bool bad = false;
  // P_N = Q_N + reg I + C_N' Sigma C_N, p_N = g_x,N
  {
    const int g = L.ng[N];
    const double* Q = V.Q(N);
    const double* sig = V.row(R_SIG) + L.cr[N];
    for (int e = tid; e < np1 * np1; e += NT) {
      const int r = e / np1, c = e % np1;
      double val;
      if (r < nx && c < nx) {
        val = Q[(long long)c * nx + r] + (r == c ? reg : 0.0);
        const double* C = g ? V.C(N) : nullptr;
        for (int j = 0; j < g; ++j) val = fma(C[(long long)r * g + j] * sig[j], C[(long long)c * g + j], val);
        V.P(N)[(long long)c * nx + r] = val;
      } else if (r < nx) {
        val = V.gx()[(long long)N * nx + r];
        V.pv()[(long long)N * nx + r] = val;
      } else if (c < nx) {
        val = V.gx()[(long long)N * nx + c];
      } else {
        val = 0.0;
      }
      S.Paug[r * np1 + c] = val;
    }
    // stage N-1 data into LDS
    const StagePtrs P = stage_ptrs(V, N - 1);
    const int nrk = np1 + P.g;
    const double* sg = V.row(R_SIG) + L.cr[N - 1];
    for (int e = tid; e < nrk * NZP; e += NT) {
      const int r = e / NZP, l = e % NZP;
      const double v = stage_load(P, nx, r, l);
      S.ABx[e] = v;
      if (r > nx) S.Tx[e] = sg[r - nx - 1] * v;
    }
  }
  double hm[R][R];
  {
    const HPtrs H = h_ptrs(V, N - 1);
#pragma unroll
    for (int a = 0; a < R; ++a)
#pragma unroll
      for (int b = 0; b < R; ++b) hm[a][b] = h_load(H, nx, ti + 16 * a, tj + 16 * b, reg);
  }
  __syncthreads();
  OCP_STAMP(10);
  for (int k = N - 1; k >= 0; --k) {
    const int mk = L.nu[k], nz = mk + nx, nrk = np1 + L.ng[k];
    // --- T = Paug [B A rb; 0 0 1] (rows 0..nx) on v_mfma_f64_16x16x4_f64: wave w owns the 16-column blocks
    //     w, w + 4, .. and all (at most four) 16-row blocks of T, K = np1 in steps of 4; operands straight from LDS
    //     (A: Paug[16 rb + lane % 16][4 kk + lane / 16], 0 beyond np1; B: ABx[4 kk + lane / 16][16 cb + lane % 16]);
    //     C/D rows (lane / 16) + 4 reg, columns lane % 16. Four independent accumulator chains per wave: the
    //     dependent VALU form left each s-step waiting on its LDS loads (26 % of a B = 1 solve) ---
    {
      const int lane = tid & 63, wv = tid >> 6, lr = lane & 15, lk = lane >> 4;
      const int nrb = (np1 + 15) >> 4, nks = (np1 + 3) >> 2;
      for (int cb = wv; cb < NZP / 16; cb += 4) {
        v4d acc[4];
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) acc[rb] = v4d{0.0, 0.0, 0.0, 0.0};
        for (int kk = 0; kk < nks; ++kk) {
          const int s2 = 4 * kk + lk;
          const bool sin = s2 < np1;
          const double bv = sin ? S.ABx[s2 * NZP + 16 * cb + lr] : 0.0;
#pragma unroll
          for (int rb = 0; rb < 4; ++rb) {
            if (rb < nrb) {
              const int r = 16 * rb + lr;
              const double av = (sin && r < np1) ? S.Paug[r * np1 + s2] : 0.0;
              acc[rb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[rb], 0, 0, 0);
            }
          }
        }
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
          if (rb < nrb) {
#pragma unroll
            for (int q2 = 0; q2 < 4; ++q2) {
              const int r = 16 * rb + lk + 4 * q2;
              if (r < np1) S.Tx[r * NZP + 16 * cb + lr] = acc[rb][q2];
            }
          }
        }
      }
    }
    lds_barrier();
    OCP_STAMP(11);
    // --- M = H + ABx' Tx over the stage's nrk rows (register tile) ---
    double m[R][R];
#pragma unroll
    for (int a = 0; a < R; ++a)
#pragma unroll
      for (int b = 0; b < R; ++b) m[a][b] = hm[a][b];
    for (int r = 0; r < nrk; ++r) {
      double ai[R], tl[R];
#pragma unroll
      for (int a = 0; a < R; ++a) ai[a] = S.ABx[r * NZP + ti + 16 * a];
#pragma unroll
      for (int b = 0; b < R; ++b) tl[b] = S.Tx[r * NZP + tj + 16 * b];
#pragma unroll
      for (int a = 0; a < R; ++a)
#pragma unroll
        for (int b = 0; b < R; ++b) m[a][b] = fma(ai[a], tl[b], m[a][b]);
    }
    lds_barrier();  // ABx / Tx are free: the next stage's data goes there
    OCP_STAMP(12);
    // --- prefetch stage k-1 (its data rows, its H tile, its rows' Sigma) ---
    StagePrefetch<NZP> pf;
    const int kn = k - 1;
    double sgv = 0.0;
    if (kn >= 0) {
      const StagePtrs P = stage_ptrs(V, kn);
      const int nrn = np1 + P.g;
      if constexpr (NZP == 64) {
#pragma unroll
        for (int s2 = 0; s2 < StagePrefetch<NZP>::EPT; ++s2) {
          const int e = tid + NT * s2;
          pf.v[s2] = e < nrn * NZP ? stage_load(P, nx, e / NZP, e % NZP) : 0.0;
        }
      }
      sgv = tid < P.g ? V.row(R_SIG)[L.cr[kn] + tid] : 0.0;  // into S.sgn at the sweep's last barrier
      const HPtrs H = h_ptrs(V, kn);
#pragma unroll
      for (int a = 0; a < R; ++a)
#pragma unroll
        for (int b = 0; b < R; ++b) hm[a][b] = h_load(H, nx, ti + 16 * a, tj + 16 * b, reg);
    }
    OCP_STAMP(13);
    // --- Gauss-Jordan sweep of the u block, two pivots per barrier: columns j and j + 1 are published together
    //     (parity double buffer, [parity][column][NZP]) before pivot j; every thread forms column j + 1 after pivot j
    //     itself, by the owner's own FMA (bit-identical to one pivot per barrier), then applies both pivots ---
    if (mk > 0) {
      // owner threads of column c write it (all rows). The register column is picked by selects: written as
      // m[a][c >> 4] (or a branch per b) the compiler kept m in scratch for a dynamic index, and the reload's
      // vmcnt wait then also waited out the next stage's prefetch, every pivot pair
      auto publish = [&](int c, double* dst) {
        const int cb = c >> 4;
        double v[R];
#pragma unroll
        for (int a = 0; a < R; ++a) {
          double t = m[a][0];
#pragma unroll
          for (int b = 1; b < R; ++b) {
            double mb = m[a][b];
            asm volatile("" : "+v"(mb));  // no select-of-loads fold back into m[a][cb]
            t = cb == b ? mb : t;
          }
          v[a] = t;
        }
        if (c < mk && tj == (c & 15)) {
#pragma unroll
          for (int a = 0; a < R; ++a) dst[ti + 16 * a] = v[a];
        }
      };
      // one GJ step with the pivot column pc (all rows) of pivot p: m <- (mask p) - a a' / d, a_p = -1
      auto step = [&](int p, const double* pc, double dinv) {
        double ci[R], cl[R];
#pragma unroll
        for (int a = 0; a < R; ++a) {
          const int i = ti + 16 * a;
          ci[a] = i == p ? -1.0 : pc[i];
        }
#pragma unroll
        for (int b = 0; b < R; ++b) {
          const int l = tj + 16 * b;
          cl[b] = l == p ? -1.0 : pc[l];
        }
#pragma unroll
        for (int a = 0; a < R; ++a) {
          const int i = ti + 16 * a;
          const double f = -ci[a] * dinv;
#pragma unroll
          for (int b = 0; b < R; ++b) {
            const int l = tj + 16 * b;
            const double base = (i == p || l == p) ? 0.0 : m[a][b];
            m[a][b] = fma(f, cl[b], base);
          }
        }
      };
      publish(0, S.col);
      publish(1, S.col + NZP);
      lds_barrier();
      double* Lf = V.Lf(k);
      for (int j = 0; j < mk; j += 2) {
        const double* c0 = S.col + ((j >> 1) & 1) * 2 * NZP;
        const double* c1 = c0 + NZP;
        const double d0 = c0[j];
        bad = bad || (d0 != d0);
        const double dinv0 = d0 > 1e-200 ? 1.0 / d0 : 0.0;
        // the pivot columns of the Schur complement are the columns of L D (the LDL' factor of M_uu), rows p..mk-1
        if (tid >= j && tid < mk) Lf[(long long)j * mk + tid] = c0[tid];
        if (j + 1 < mk) {
          const double a1 = c0[j + 1];  // a_{j+1} of pivot j
          // column j + 1 after pivot j, at the rows this thread needs (its tile rows and columns) and at j + 1
          double e1[R], e2[R];
#pragma unroll
          for (int a = 0; a < R; ++a) {
            const int i = ti + 16 * a;
            const double ai = i == j ? -1.0 : c0[i];
            e1[a] = fma(-ai * dinv0, a1, i == j ? 0.0 : c1[i]);
          }
#pragma unroll
          for (int b = 0; b < R; ++b) {
            const int l = tj + 16 * b;
            const double al = l == j ? -1.0 : c0[l];
            e2[b] = fma(-al * dinv0, a1, l == j ? 0.0 : c1[l]);
          }
          const double d1 = fma(-a1 * dinv0, a1, c1[j + 1]);
          bad = bad || (d1 != d1);
          const double dinv1 = d1 > 1e-200 ? 1.0 / d1 : 0.0;
          if (tid > j && tid < mk) {
            const double at = c0[tid];
            Lf[(long long)(j + 1) * mk + tid] = fma(-at * dinv0, a1, c1[tid]);
          }
          step(j, c0, dinv0);
          // pivot j + 1 with the column formed above (a_{j+1} = -1)
#pragma unroll
          for (int a = 0; a < R; ++a) {
            const int i = ti + 16 * a;
            const double bi = i == j + 1 ? -1.0 : e1[a];
            const double f = -bi * dinv1;
#pragma unroll
            for (int b = 0; b < R; ++b) {
              const int l = tj + 16 * b;
              const double bl = l == j + 1 ? -1.0 : e2[b];
              const double base = (i == j + 1 || l == j + 1) ? 0.0 : m[a][b];
              m[a][b] = fma(f, bl, base);
            }
          }
        } else {
          step(j, c0, dinv0);
        }
        double* nb = S.col + (((j >> 1) + 1) & 1) * 2 * NZP;
        publish(j + 2, nb);
        publish(j + 3, nb + NZP);
        if (j + 2 >= mk && kn >= 0 && tid < L.ng[kn]) S.sgn[tid] = sgv;
        lds_barrier();
      }
    } else {
      if (kn >= 0 && tid < L.ng[kn]) S.sgn[tid] = sgv;
      lds_barrier();  // S.sgn visible to the stores below
    }
    OCP_STAMP(14);
    // --- next stage's data into LDS ---
    if (kn >= 0) {
      const int nrn = np1 + L.ng[kn];
      if constexpr (NZP == 64) {
#pragma unroll
        for (int s2 = 0; s2 < StagePrefetch<NZP>::EPT; ++s2) {
          const int e = tid + NT * s2;
          if (e < nrn * NZP) {
            S.ABx[e] = pf.v[s2];
            if (e / NZP > nx) S.Tx[e] = S.sgn[e / NZP - nx - 1] * pf.v[s2];
          }
        }
      } else {
        const StagePtrs P = stage_ptrs(V, kn);
        for (int e = tid; e < nrn * NZP; e += NT) {
          const int r = e / NZP;
          const double v = stage_load(P, nx, r, e % NZP);
          S.ABx[e] = v;
          if (r > nx) S.Tx[e] = S.sgn[r - nx - 1] * v;
        }
      }
    }
    OCP_STAMP(15);
    // --- outputs ---
    {
      double* Kk = V.K(k);
      double* kf = V.kf() + L.cu[k];
      double* Pk = V.P(k);
      double* pk = V.pv() + (long long)k * nx;
#pragma unroll
      for (int a = 0; a < R; ++a)
#pragma unroll
        for (int b = 0; b < R; ++b) {
          const int i = ti + 16 * a, l = tj + 16 * b;
          const double v = m[a][b];
          if (i < mk) {
            if (l >= mk && l < nz) Kk[(long long)(l - mk) * mk + i] = -v;
            else if (l == nz) kf[i] = -v;
          } else if (i < nz) {
            if (l >= mk && l < nz) {  // P_k from its lower triangle, mirrored (HPIPM keeps the lower one)
              if (i >= l) {
                Pk[(long long)(l - mk) * nx + (i - mk)] = v;
                Pk[(long long)(i - mk) * nx + (l - mk)] = v;
                S.Paug[(i - mk) * np1 + (l - mk)] = v;
                S.Paug[(l - mk) * np1 + (i - mk)] = v;
              }
            } else if (l == nz) {
              pk[i - mk] = v;
              S.Paug[(i - mk) * np1 + nx] = v;
            }
          } else if (i == nz) {
            if (l >= mk && l < nz) S.Paug[nx * np1 + (l - mk)] = v;
            else if (l == nz) S.Paug[nx * np1 + nx] = 0.0;
          }
        }
    }
    lds_barrier();
    OCP_STAMP(16);
  }
  return __syncthreads_or(bad) == 0;
}

// Closed-loop matrices Acl_k = A_k + B_k K_k (column-major, k = 1..N-1) and bcl_k = rb_k + B_k kf_k (k = 0..N-1), one
// stage at a time: B_k, K_k and kf_k staged in LDS (double buffer in ABx / Tx, one LDS barrier per stage; the next
// stage's operands are loaded into registers while this one computes) so that every product operand is an LDS read
// (B_k consecutive over the rows, K_k broadcast), A_k and rb_k coalesced global loads. A stage whose operands exceed
// the register staging (nu_k far above nx) reads them from global memory instead.
// Acl_k = A_k + B_k K_k (k >= 1, with_acl) and bcl_k = rb_k + B_k kff_k for every stage at once: no stage depends on
// another once the factorisation has produced K and kff, so the work is spread over all stages (4 x 4 blocks of Acl,
// 4-row blocks of bcl per thread, operands straight from the L2-resident records / workspace) with no barrier
// between stages; each entry is the same fma chain over a as the per-stage form, so the results are bit-identical
// (was one stage per barrier with LDS-staged operands: 11 % of a B = 1 solve)
__device__ __forceinline__ void acl_pass(const View& V, const Lds& S, bool with_acl, int k0 = 0, int k1 = -1,
                                         bool sync = true) {
  (void)S;
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, nx = L.nx, N = L.N;
  const int nb4 = (nx + 3) >> 2;
  const int pa = with_acl ? nb4 * nb4 : 0;  // Acl blocks per stage
  const int ps = pa + nb4;                  // + bcl blocks
  const double* kfv = V.kf();
  const double* rbv = V.rb();
  double* bclv = V.bcl();
  if (k1 < 0) k1 = N;
  for (int w = k0 * ps + tid; w < k1 * ps; w += NT) {
    const int k = w / ps, r = w - k * ps;
    const int mk = L.nu[k];
    const double* Bk = V.Bm(k);
    if (r < pa) {
      if (k == 0) continue;  // dx_0 = 0: Acl_0 is never used
      const int i0 = 4 * (r / nb4), c0 = 4 * (r - (r / nb4) * nb4);
      const double* Ak = V.A(k);
      const double* Kk = V.K(k);
      double acc[4][4];
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) {
          const int i = i0 + ii, c = c0 + cc;
          acc[ii][cc] = (i < nx && c < nx) ? Ak[c * nx + i] : 0.0;
        }
#pragma unroll 4
      for (int aa = 0; aa < mk; ++aa) {
        double bv[4], kv[4];
#pragma unroll
        for (int ii = 0; ii < 4; ++ii) bv[ii] = i0 + ii < nx ? Bk[aa * nx + i0 + ii] : 0.0;
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) kv[cc] = c0 + cc < nx ? Kk[(c0 + cc) * mk + aa] : 0.0;
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
#pragma unroll
          for (int cc = 0; cc < 4; ++cc) acc[ii][cc] = fma(bv[ii], kv[cc], acc[ii][cc]);
      }
      double* Ao = V.Acl(k);
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int cc = 0; cc < 4; ++cc)
          if (i0 + ii < nx && c0 + cc < nx) Ao[(c0 + cc) * nx + i0 + ii] = acc[ii][cc];
    } else {
      const int i0 = 4 * (r - pa);
      const double* kk = kfv + L.cu[k];
      double acc[4];
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) acc[ii] = i0 + ii < nx ? rbv[(long long)k * nx + i0 + ii] : 0.0;
#pragma unroll 4
      for (int aa = 0; aa < mk; ++aa) {
        const double kv = kk[aa];
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
          acc[ii] = fma(i0 + ii < nx ? Bk[aa * nx + i0 + ii] : 0.0, kv, acc[ii]);
      }
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
        if (i0 + ii < nx) bclv[(long long)k * nx + i0 + ii] = acc[ii];
    }
  }
  if (sync) __syncthreads();
}

// Serial forward sweep: dx_1 = bcl_0, dx_{k+1} = Acl_k dx_k + bcl_k (dx node 0 stays 0)
__device__ __forceinline__ void forward_pass(const View& V, const Lds& S) {
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, nx = L.nx, N = L.N, nxx = nx * nx;
  double* dx = V.dx();
  double* v0 = S.vec;
  double* v1 = S.vec + 64;
  if (tid < nx) {
    const double d = V.bcl()[tid];
    v0[tid] = d;
    dx[nx + tid] = d;
  }
  if (N > 1)
    for (int e = tid; e < nxx; e += NT) S.ABx[e] = V.Acl(1)[e];
  // bcl_k is loaded one stage ahead with Acl_{k+1}: no global latency at the head of a stage's chain
  double bn = (N > 1 && tid < nx) ? V.bcl()[(long long)nx + tid] : 0.0;
  __syncthreads();
  for (int k = 1; k < N; ++k) {
    double* cur = (k & 1) ? S.ABx : S.Tx;
    double* nxt = (k & 1) ? S.Tx : S.ABx;
    const double* vin = (k & 1) ? v0 : v1;
    double* vout = (k & 1) ? v1 : v0;
    double pre[16];
    const bool more = k + 1 < N;
    const double bk = bn;
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2) {
      const int e = tid + NT * s2;
      pre[s2] = (more && e < nxx) ? V.Acl(k + 1)[e] : 0.0;
    }
    if (more && tid < nx) bn = V.bcl()[(long long)(k + 1) * nx + tid];
    if (tid < nx) {
      double acc = bk;
#pragma unroll 8
      for (int c = 0; c < nx; ++c) acc = fma(cur[c * nx + tid], vin[c], acc);
      vout[tid] = acc;
      dx[(long long)(k + 1) * nx + tid] = acc;
    }
    if (more) {
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) {
        const int e = tid + NT * s2;
        if (e < nxx) nxt[e] = pre[s2];
      }
    }
    __syncthreads();
  }
}

// du_k = K_k dx_k + kf_k, dpi_k = P_{k+1} dx_{k+1} + p_{k+1}; then the row directions and the largest step
// (returns the local min over rows of the fraction-to-boundary step, 1e300 if none)
__device__ __forceinline__ double post_pass(const View& V, int k0 = 0, int k1 = -1, int n1 = -1) {
  const OcpLayout& L = V.L;
  const int nx = L.nx, N = L.N;
  const double* dx = V.dx();
  if (k1 < 0) k1 = N;
  if (n1 < 0) n1 = N + 1;
  const int u0 = L.cu[k0], nuR = L.cu[k1] - u0, r0 = L.cr[k0], r1 = L.cr[n1];
  for (int itr = threadIdx.x; itr < nuR + (k1 - k0) * nx; itr += NT) {
    const int it = itr < nuR ? u0 + itr : L.nU + k0 * nx + (itr - nuR);
    if (it < L.nU) {
      const int k = L.ustage[it], a = it - L.cu[k], mk = L.nu[k];
      double s = V.kf()[it];
      if (k > 0) {
        const double* Kk = V.K(k);
        for (int c = 0; c < nx; ++c) s = fma(Kk[(long long)c * mk + a], dx[(long long)k * nx + c], s);
      }
      V.du()[it] = s;
    } else {
      const int e = it - L.nU, k = e / nx, i = e % nx;
      const double* Pn = V.P(k + 1);
      double s = V.pv()[(long long)(k + 1) * nx + i];
      for (int t = 0; t < nx; ++t) s = fma(Pn[(long long)t * nx + i], dx[(long long)(k + 1) * nx + t], s);
      V.dpi()[(long long)k * nx + i] = s;
    }
  }
  __syncthreads();
  double amax = 1e300;
  if (r1 > r0) {
    double* dc = V.row(R_DTL);
    rows_value(V, dx, V.du(), dc, r0, r1);  // each thread reads back only its own rows below
    const double *rl = V.row(R_RL), *ru = V.row(R_RU), *tl = V.row(R_TL), *tu = V.row(R_TU), *ll = V.row(R_LL),
                 *lu = V.row(R_LU), *rml = V.row(R_RML), *rmu = V.row(R_RMU);
    double *dtl = V.row(R_DTL), *dtu = V.row(R_DTU), *dll = V.row(R_DLL), *dlu = V.row(R_DLU);
    for (int j = r0 + threadIdx.x; j < r1; j += NT) {
      const double c = dtl[j];
      const double a1 = c + rl[j], a2 = ru[j] - c;
      const double b1 = -(rml[j] + ll[j] * a1) / tl[j], b2 = -(rmu[j] + lu[j] * a2) / tu[j];
      dtl[j] = a1;
      dtu[j] = a2;
      dll[j] = b1;
      dlu[j] = b2;
      if (a1 < 0.0) amax = fmin(amax, -tl[j] / a1);
      if (a2 < 0.0) amax = fmin(amax, -tu[j] / a2);
      if (b1 < 0.0) amax = fmin(amax, -ll[j] / b1);
      if (b2 < 0.0) amax = fmin(amax, -lu[j] / b2);
    }
  }
  return amax;
}

// x = -M_uu^{-1} z from the sweep's LDL' columns F (column j holds d_j l_j on rows j..m-1; d_j = F[j][j]), with
// the sweep's guard (1/d -> 0 for d <= 1e-200). Triangular solves keep the IPM's benign ill-conditioning benign:
// an explicit inverse applied to z does not (its error grows with the barrier's Sigma and stalls the iteration).
__device__ __forceinline__ void ldl_solve(const double* __restrict__ F, int m, const double* __restrict__ z,
                                          double* __restrict__ x) {
  for (int i = 0; i < m; ++i) x[i] = z[i];
  for (int j = 0; j < m; ++j) {  // L D y = z, then y /= d
    const double d = F[(long long)j * m + j];
    const double dinv = d > 1e-200 ? 1.0 / d : 0.0;
    const double yj = x[j] * dinv;
    for (int i = j + 1; i < m; ++i) x[i] = fma(-F[(long long)j * m + i], yj, x[i]);
    x[j] = yj;
  }
  for (int j = m - 1; j >= 0; --j) {  // L' x = y
    const double d = F[(long long)j * m + j];
    const double dinv = d > 1e-200 ? 1.0 / d : 0.0;
    double s = x[j];
    for (int i = j + 1; i < m; ++i) s = fma(-F[(long long)j * m + i] * dinv, x[i], s);
    x[j] = s;
  }
  for (int i = 0; i < m; ++i) x[i] = -x[i];
}

#include "ocp_chain.hpp"

// LDS of the latency form: G images (two), T, Paug, the pivot-column buffers and the rows' Sigma (two), then red and
// vec; the other passes of the kernel see G0 / G1 as ABx / Tx (contiguous: the staged residuals' buffer)
__device__ __forceinline__ Lds carve_fast(double* smem, const OcpLayout& L, ChainLds& C) {
  const int ngr = CH_NRP + ((L.ngmax + 3) & ~3), ngp = (L.ngmax + 4) & ~3;  // rows in groups of four (chain_m)
  const int g1 = ngr * CH_GS > CH_MAXU * CH_FS ? ngr * CH_GS : CH_MAXU * CH_FS;
  C.G0 = smem;
  C.G1 = C.G0 + ngr * CH_GS;
  C.F1 = C.G1;  // the chain's second factor image (G1 is the other passes' scratch)
  C.T = C.G1 + g1;
  C.Pa = C.T + CH_NRP * CH_GS;
  C.C = C.Pa + CH_PS * CH_PS;
  C.sg0 = C.C + 256;
  C.sg1 = C.sg0 + ngp;
  C.Ml = C.sg1 + ngp + 64 + 128;
  C.Hc = C.Ml + CH_MR * CH_GS;
  C.gb = C.Hc + 4 * CH_MAXNT;
  C.Pa2 = C.gb + 64;
  C.F0 = C.Pa2 + CH_PS * CH_PS;
  C.desc = (int*)(C.F0 + CH_MAXU * CH_FS);
  Lds s;
  s.np1 = L.nx + 1;
  s.nrm = L.nx + 1 + L.ngmax;
  s.nzp = 64;
  s.Paug = C.Pa;
  s.ABx = C.G0;
  s.Tx = C.G1;
  s.col = C.C;
  s.red = C.sg1 + ngp;
  s.vec = s.red + 64;
  s.sgn = C.sg0;
  return s;
}

// ---- grid form (small batches): G workgroups per problem, stage ranges, grid barriers -----------------------------
// Workgroup g of problem q owns stages [k0, k1) and nodes [k0, n1) (n1 = k1, the last one N + 1), their rows
// [r0, r1) and inputs [u0, u1): every stage-parallel pass runs on the owned range; the serial chains (the
// factorisation, the forward rollout, the corrector's cost-to-go recursion) run on workgroup 0; grid barriers between
// the phases. Reductions (residual maxima, mu, the step length) go through per-workgroup partials read back in a fixed
// order by every workgroup, so all workgroups take the same decisions.
struct GridRange {
  int g, G, k0, k1, n1, u0, u1, r0, r1;
};
__device__ __forceinline__ GridRange grid_range(const OcpLayout& L, int g, int G) {
  GridRange R;
  R.g = g;
  R.G = G;
  R.k0 = (int)((long long)L.N * g / G);
  R.k1 = (int)((long long)L.N * (g + 1) / G);
  R.n1 = g == G - 1 ? L.N + 1 : R.k1;
  R.u0 = L.cu[R.k0];
  R.u1 = L.cu[R.k1];
  R.r0 = L.cr[R.k0];
  R.r1 = L.cr[R.n1];
  return R;
}

// Grid barrier of one problem's G workgroups (the hand-off recipe of the MI355X guide: every wave's stores drained,
// lane-0 agent release, a relaxed agent-scope arrive on a counter that is zero at the launch, a relaxed poll with
// s_sleep, one agent acquire). The wait is bounded in time (limit: ticks of the 100-MHz real-time counter,
// OcpSolveArgs::grid_timeout): on a timeout (or another workgroup's) the problem's fail word is set and every workgroup
// returns false at its next barrier, so the grid drains instead of hanging; the solve then reports
// CMPC_GRID_TIMEOUT and the fallback launch (k_ocp_fallback) re-solves the problem on one workgroup. A negative limit
// forces the timeout at the first barrier (cmpc_ocp_debug_force_grid_timeout).
__device__ __forceinline__ bool grid_sync(unsigned* bar, unsigned target, double* flag_lds, long long limit) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    bool good = __hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (limit < 0) {
      __hip_atomic_store(bar + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      good = false;
    }
    while (good && __hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (__hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) good = false;
      if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > limit) {
        __hip_atomic_store(bar + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        good = false;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    flag_lds[0] = good ? 1.0 : 0.0;
  }
  __syncthreads();
  return flag_lds[0] != 0.0;
}

// Every workgroup's nv partials (slot [g][0..nv)) reduced in workgroup order by lanes of wave 0, the same in every
// workgroup; ops: 0 max (NaN-propagating), 1 sum, 2 min. Result in out (LDS), valid after the trailing barrier.
__device__ __forceinline__ void grid_collect(const double* part, int G, int nv, const int* ops, double* out) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    for (int c = 0; c < nv; ++c) {
      const int op = ops[c];
      const double idv = op == 0 ? 0.0 : (op == 1 ? 0.0 : 1e300);
      double v = lane < G ? __hip_atomic_load(part + lane * 8 + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : idv;
      // fixed-order tree over the 64 lanes (identical in every workgroup)
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const double w = __shfl_xor(v, o, 64);
        v = op == 0 ? nmax(v, w) : (op == 1 ? ((lane & o) ? w + v : v + w) : (v < w ? v : w));
      }
      if (lane == 0) out[c] = v;
    }
  }
  __syncthreads();
}

#include "ocp_part.hpp"

// Corrector's backward vector pass split for the grid form: (a) y_k = P_{k+1} rb_k and h_k on the owned stages
// (p_N = g_x,N on the last workgroup), (b) the serial recursion p_k = Acl_k' p_{k+1} + h_k on workgroup 0, (c) the
// feedforward kf_k = -M_uu,k^{-1} (g_u,k + B_k'(y_k + p_{k+1})) on the owned stages. (a) + (b) + (c) = backward_vec_pass.
__device__ __forceinline__ void bwd_vec_a(const View& V, int k0, int k1, bool last) {
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, nx = L.nx, N = L.N;
  double* y = V.y();
  double* h = V.h();
  for (int it = k0 * nx + tid; it < k1 * nx; it += NT) {
    const int k = it / nx, i = it - k * nx;
    const double* Pn = V.P(k + 1);
    double s = 0.0;
#pragma unroll 8
    for (int t = 0; t < nx; ++t) s = fma(Pn[(long long)t * nx + i], V.rb()[(long long)k * nx + t], s);
    y[it] = s;
  }
  if (last)
    for (int it = tid; it < nx; it += NT) V.pv()[(long long)N * nx + it] = V.gx()[(long long)N * nx + it];
  __syncthreads();
  const int ka = k0 > 1 ? k0 : 1;
  for (int it = ka * nx + tid; it < k1 * nx; it += NT) {
    const int k = it / nx, i = it - k * nx, mk = L.nu[k];
    const double* Kk = V.K(k);
    const double* Ac = V.Acl(k);
    double s = V.gx()[(long long)k * nx + i];
#pragma unroll 8
    for (int a = 0; a < mk; ++a) s = fma(Kk[(long long)i * mk + a], V.gu()[L.cu[k] + a], s);
#pragma unroll 8
    for (int t = 0; t < nx; ++t) s = fma(Ac[(long long)i * nx + t], y[(long long)k * nx + t], s);
    h[(long long)k * nx + i] = s;
  }
}

// Corrector's serial cost-to-go recursion (backward_vec_pass part b): p_N = g_x,N, p_k = Acl_k' p_{k+1} + h_k
// (k = N-1..1); Acl_k' staged transposed in LDS (double buffer in ABx / Tx)
__device__ __forceinline__ void bwd_vec_b(const View& V, const Lds& S) {
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, nx = L.nx, N = L.N, nxx = nx * nx;
  double* h = V.h();
  double* pv = V.pv();
  double* v0 = S.vec;
  double* v1 = S.vec + 64;
  if (tid < nx) v0[tid] = V.gx()[(long long)N * nx + tid];
  if (N > 1)
    for (int e = tid; e < nxx; e += NT) {
      const int c = e / nx, r = e % nx;  // Acl col-major: e = c nx + r holds Acl(r, c); LDS [r][c]
      S.ABx[r * nx + c] = V.Acl(N - 1)[e];
    }
  __syncthreads();
  double hn = (N > 1 && tid < nx) ? h[(long long)(N - 1) * nx + tid] : 0.0;  // h_k one stage ahead, as bcl above
  for (int k = N - 1, t2 = 0; k >= 1; --k, ++t2) {
    double* cur = (t2 & 1) ? S.Tx : S.ABx;
    double* nxt = (t2 & 1) ? S.ABx : S.Tx;
    const double* vin = (t2 & 1) ? v1 : v0;
    double* vout = (t2 & 1) ? v0 : v1;
    double pre[16];
    const bool more = k - 1 >= 1;
    const double hk = hn;
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2) {
      const int e = tid + NT * s2;
      pre[s2] = (more && e < nxx) ? V.Acl(k - 1)[e] : 0.0;
    }
    if (more && tid < nx) hn = h[(long long)(k - 1) * nx + tid];
    if (tid < nx) {  // p_k[i] = sum_t Acl(t, i) p_{k+1}[t] + h_k[i]; cur[t * nx + i] = Acl(t, i)
      double acc = hk;
#pragma unroll 8
      for (int t = 0; t < nx; ++t) acc = fma(cur[t * nx + tid], vin[t], acc);
      vout[tid] = acc;
      pv[(long long)k * nx + tid] = acc;
    }
    if (more) {
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) {
        const int e = tid + NT * s2;
        if (e < nxx) {
          const int c = e / nx, r = e % nx;
          nxt[r * nx + c] = pre[s2];
        }
      }
    }
    __syncthreads();
  }
}

// Corrector's feedforward on stages [k0, k1) (backward_vec_pass part c): z_k = g_u + B'(y_k + p_{k+1}) into du
// (scratch), then kf_k = -M_uu,k^{-1} z_k by the LDL' factors
__device__ __forceinline__ void bwd_vec_c(const View& V, int k0, int k1) {
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, nx = L.nx;
  const double* y = V.y();
  const double* pv = V.pv();
  double* z = V.du();
  for (int it = L.cu[k0] + tid; it < L.cu[k1]; it += NT) {
    const int k = L.ustage[it], a = it - L.cu[k];
    const double* Bm = V.Bm(k);
    double s = V.gu()[it];
#pragma unroll 8
    for (int t = 0; t < nx; ++t)
      s = fma(Bm[(long long)a * nx + t], y[(long long)k * nx + t] + pv[(long long)(k + 1) * nx + t], s);
    z[it] = s;
  }
  __syncthreads();
  for (int k = k0 + tid; k < k1; k += NT) ldl_solve(V.Lf(k), L.nu[k], z + L.cu[k], V.kf() + L.cu[k]);
}

// Corrector's backward vector pass with the factorisation kept: y_k = P_{k+1} rb_k; h_k = g_x,k + K_k' g_u,k +
// Acl_k' y_k; p_N = g_x,N, p_k = Acl_k' p_{k+1} + h_k (serial, k = N-1..1); kf_k = -M_uu,k^{-1} (g_u,k + B_k'(y_k +
// p_{k+1})) by the LDL' factors
__device__ __forceinline__ void backward_vec_pass(const View& V, const Lds& S) {
  const int N = V.L.N;
  bwd_vec_a(V, 0, N, true);
  __syncthreads();
  bwd_vec_b(V, S);
  __syncthreads();
  bwd_vec_c(V, 0, N);
}

// Residuals of the Newton system an iteration solved, at its final direction (dz = (dx, du), dpi, the rows' dt, dl),
// HPIPM's "lin res" statistics (HpipmInterface.cpp:492-501, d_ocp_qp_ipm_get_stat columns 13-16): the inf-norms of
//   stat  H~ dz + G'dpi - Gc'(dl_l - dl_u) + r_g   (H~ the factorised Hessian: reg_prim on its diagonal),
//   eq    A_k dx_k + B_k du_k - dx_{k+1} + r_b,
//   ineq  Gc dz - dt_l + r_l,  -Gc dz - dt_u + r_u,
//   comp  t_l dl_l + l_l dt_l + r_ml,  t_u dl_u + l_u dt_u + r_mu
// over the nodes [n0, n1) and their rows [r0, r1) (local maxima; the caller reduces). r_g, r_b are the iteration's
// residuals (rgu / rgx / rb), r_m the final direction's complementarity right-hand side; c = Gc dz goes through R_W
// (free after the step's right-hand side).
__device__ __forceinline__ void lin_res(const View& V, double reg, int n0, int n1, double* o) {
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, nx = L.nx, N = L.N;
  const double *dx = V.dx(), *du = V.du(), *dpi = V.dpi();
  const double *dll = V.row(R_DLL), *dlu = V.row(R_DLU);
  const int P = L.nzp + nx;
  for (int w = n0 * P + tid; w < n1 * P; w += NT) {
    const int k = w / P, e = w - k * P;
    const int mk = L.nu[k], g = L.ng[k];
    const int m1 = mk, m2 = k >= 1 ? nx : 0, m3 = k < N ? nx : 0;
    if (e >= m1 + m2 + m3) continue;
    const double* A = V.A(k);
    const double* Bm = V.Bm(k);
    const double* dxk = dx + (long long)k * nx;
    const double* duk = du + L.cu[k];
    const double* dpk = dpi + (long long)k * nx;
    const int rk = L.cr[k];
    if (e < m1) {
      const int a = e;
      const double *R = V.R(k), *Sm = V.S(k);
      double s = fma(reg, duk[a], V.rgu()[L.cu[k] + a]);
      for (int c = 0; c < mk; ++c) s = fma(R[c * mk + a], duk[c], s);
      for (int j = 0; j < nx; ++j) s = fma(Sm[j * mk + a], dxk[j], s);
      for (int t = 0; t < m3; ++t) s = fma(Bm[a * nx + t], dpk[t], s);
      if (g) {
        const double* D = V.D(k);
        for (int j = 0; j < g; ++j) s = fma(-D[a * g + j], dll[rk + j] - dlu[rk + j], s);
      }
      o[0] = nmax(o[0], fabs(s));
    } else if (e < m1 + m2) {
      const int i = e - m1;
      const double *Q = V.Q(k), *Sm = V.S(k);
      double s = fma(reg, dxk[i], V.rgx()[(long long)k * nx + i] - dpi[(long long)(k - 1) * nx + i]);
      for (int j = 0; j < nx; ++j) s = fma(Q[j * nx + i], dxk[j], s);
      for (int a = 0; a < mk; ++a) s = fma(Sm[i * mk + a], duk[a], s);
      for (int t = 0; t < m3; ++t) s = fma(A[i * nx + t], dpk[t], s);
      if (g) {
        const double* C = V.C(k);
        for (int j = 0; j < g; ++j) s = fma(-C[i * g + j], dll[rk + j] - dlu[rk + j], s);
      }
      o[0] = nmax(o[0], fabs(s));
    } else {
      const int i = e - m1 - m2;
      double s = V.rb()[(long long)k * nx + i] - dx[(long long)(k + 1) * nx + i];
      for (int j = 0; j < nx; ++j) s = fma(A[j * nx + i], dxk[j], s);
      for (int a = 0; a < mk; ++a) s = fma(Bm[a * nx + i], duk[a], s);
      o[1] = nmax(o[1], fabs(s));
    }
  }
  const int r0 = L.cr[n0], r1 = L.cr[n1 < N + 1 ? n1 : N + 1];
  if (r1 > r0) {
    double* c = V.row(R_W);
    rows_value(V, dx, du, c, r0, r1);  // each thread reads back only its own rows
    const double *rl = V.row(R_RL), *ru = V.row(R_RU), *tl = V.row(R_TL), *tu = V.row(R_TU), *ll = V.row(R_LL),
                 *lu = V.row(R_LU), *rml = V.row(R_RML), *rmu = V.row(R_RMU), *dtl = V.row(R_DTL),
                 *dtu = V.row(R_DTU);
    for (int j = r0 + tid; j < r1; j += NT) {
      o[2] = nmax(o[2], nmax(fabs(c[j] + rl[j] - dtl[j]), fabs(ru[j] - c[j] - dtu[j])));
      o[3] = nmax(o[3], nmax(fabs(fma(tl[j], dll[j], fma(ll[j], dtl[j], rml[j]))),
                             fabs(fma(tu[j], dlu[j], fma(lu[j], dtu[j], rmu[j])))));
    }
  }
}

// (l_l - l_u) into R_W
__device__ __forceinline__ void load_lamdiff(const View& V) {
  double* w = V.row(R_W);
  const double *ll = V.row(R_LL), *lu = V.row(R_LU);
  for (int j = threadIdx.x; j < V.L.m; j += NT) w[j] = ll[j] - lu[j];
}

template <int NZP, int MINB, bool FAST, bool LINRES = false>
__device__ __forceinline__ void ipm_body(const OcpSolveArgs& a, int q, const Lds& S, const ChainLds& CS) {
  const View V(a, q);
  const OcpLayout& L = a.L;
  const int tid = threadIdx.x, nx = L.nx, N = L.N, m = L.m;
  double* x = V.x();
  double* u = V.u();
  constexpr bool fast = FAST;
  double* hp = fast ? a.hp + (long long)q * a.hp_stride : nullptr;
  if (fast) hp_build(V, hp, a.reg);  // the stages' constant Hessian blocks, once per solve (read after a barrier)
  // --- cold start ---
  for (int i = tid; i < (N + 1) * nx; i += NT) {  // warm: x (nodes >= 1), u from the caller's d_x / d_u
    x[i] = i < nx ? a.x0[(long long)q * nx + i] : (a.warm ? a.x[(long long)q * (N + 1) * nx + i] : 0.0);
    V.dx()[i] = 0.0;
    V.gx()[i] = 0.0;
    V.rgx()[i] = 0.0;
  }
  for (int i = tid; i < L.nU; i += NT) u[i] = a.warm ? a.u[(long long)q * L.nU + i] : 0.0;
  for (int i = tid; i < N * nx; i += NT) V.pi()[i] = 0.0;
  __syncthreads();
  {
    double* c = V.row(R_C);
    rows_value(V, x, u, c);
    double *lg = V.row(R_LG), *ug = V.row(R_UG), *tl = V.row(R_TL), *tu = V.row(R_TU), *ll = V.row(R_LL),
           *lu = V.row(R_LU);
    for (int j = tid; j < m; j += NT) {
      const int k = L.rstage[j];
      const double bnd = -V.e(k)[j - L.cr[k]];
      lg[j] = bnd;
      ug[j] = bnd;
      tl[j] = fmax(c[j] - bnd, 1.0);
      tu[j] = fmax(bnd - c[j], 1.0);
      ll[j] = a.mu0 / tl[j];
      lu[j] = a.mu0 / tu[j];
    }
  }
  __syncthreads();
  int status = 1, it = 0;
  double rs = 0, re = 0, ri = 0, rc = 0;
  OCP_STAMP(0);
  for (it = 0;; ++it) {
    // --- residuals ---
    rows_value(V, x, u, V.row(R_C));
    load_lamdiff(V);
    __syncthreads();
    double lrs = 0.0, lre = 0.0, lri = 0.0, lrc = 0.0, lmu = 0.0;
    if (MINB == 1 && a.par_res) residuals_par(V, lrs, lre);  // small batches: all nodes at once (latency)
    else residuals_staged(V, S, lrs, lre);                  // L2 traffic bounds bigger batches
    {
      const double *c = V.row(R_C), *lg = V.row(R_LG), *ug = V.row(R_UG), *tl = V.row(R_TL), *tu = V.row(R_TU),
                   *ll = V.row(R_LL), *lu = V.row(R_LU);
      double *rl = V.row(R_RL), *ru = V.row(R_RU);
      for (int j = tid; j < m; j += NT) {
        const double a1 = c[j] - lg[j] - tl[j], a2 = ug[j] - c[j] - tu[j];
        rl[j] = a1;
        ru[j] = a2;
        lri = nmax(lri, nmax(fabs(a1), fabs(a2)));
        const double c1 = tl[j] * ll[j], c2 = tu[j] * lu[j];
        lrc = nmax(lrc, nmax(c1, c2));
        lmu += c1 + c2;
      }
    }
    rs = block_reduce(lrs, S.red, OpMax());
    re = block_reduce(lre, S.red, OpMax());
    ri = block_reduce(lri, S.red, OpMax());
    rc = block_reduce(lrc, S.red, OpMax());
    const double musum = block_reduce(lmu, S.red, OpSum());
    const double mu = m > 0 ? musum / (2.0 * m) : 0.0;
    OCP_STAMP(1);
    double* sr = (a.stats && it < a.stat_rows) ? a.stats + ((long long)q * a.stat_rows + it) * 10 : nullptr;
    if (sr && tid == 0 && a.linres)
      for (int c = 0; c < 4; ++c) a.linres[((long long)q * a.stat_rows + it) * 4 + c] = __builtin_nan("");
    if (sr && tid == 0) {
      for (int c = 0; c < 5; ++c) sr[c] = __builtin_nan("");
      sr[5] = mu;
      sr[6] = rs;
      sr[7] = re;
      sr[8] = ri;
      sr[9] = rc;
    }
    if (!(isfinite(rs) && isfinite(re) && isfinite(ri) && isfinite(rc))) {
      status = 3;
      break;
    }
    if (rs <= a.tol_stat && re <= a.tol_eq && ri <= a.tol_ineq && rc <= a.tol_comp) {
      status = 0;
      break;
    }
    if (it >= a.iter_max) {
      status = 1;
      break;
    }
    if (m > 0 && !(mu > 1e-300)) {
      status = 2;
      break;
    }
    // --- predictor right-hand side and factorisation ---
    {
      const double *tl = V.row(R_TL), *tu = V.row(R_TU), *ll = V.row(R_LL), *lu = V.row(R_LU), *rl = V.row(R_RL),
                   *ru = V.row(R_RU);
      double *sig = V.row(R_SIG), *rml = V.row(R_RML), *rmu = V.row(R_RMU), *w = V.row(R_W);
      for (int j = tid; j < m; j += NT) {
        sig[j] = ll[j] / tl[j] + lu[j] / tu[j];
        rml[j] = tl[j] * ll[j];
        rmu[j] = tu[j] * lu[j];
        w[j] = (rml[j] + ll[j] * rl[j]) / tl[j] - (rmu[j] + lu[j] * ru[j]) / tu[j];
      }
    }
    __syncthreads();
    step_rhs(V);
    __syncthreads();
    OCP_STAMP(2);
    bool fok;
    if constexpr (FAST) {
      fok = chain_factor(V, CS, hp, a.reg);
      chain_gains(V, 0, N);
      __syncthreads();
    } else {
      fok = factor_pass<NZP>(V, S, a.reg);
    }
    if (!fok) {
      status = 3;
      break;
    }
    OCP_STAMP(17);
    acl_pass(V, S, true);
    __syncthreads();
    OCP_STAMP(3);
    if constexpr (FAST) chain_affine<false>(V, CS, S.vec, S.vec + 64);
    else forward_pass(V, S);
    OCP_STAMP(4);
    double amax = block_reduce(post_pass(V), S.red, OpMin());
    OCP_STAMP(5);
    double alpha = fmin(1.0, amax);
    if (m > 0) {
      // mu_aff and the corrector
      double lm = 0.0;
      const double *tl = V.row(R_TL), *tu = V.row(R_TU), *ll = V.row(R_LL), *lu = V.row(R_LU), *dtl = V.row(R_DTL),
                   *dtu = V.row(R_DTU), *dll = V.row(R_DLL), *dlu = V.row(R_DLU);
      for (int j = tid; j < m; j += NT)
        lm += (tl[j] + alpha * dtl[j]) * (ll[j] + alpha * dll[j]) + (tu[j] + alpha * dtu[j]) * (lu[j] + alpha * dlu[j]);
      const double maff = block_reduce(lm, S.red, OpSum()) / (2.0 * m);
      const double ratio = maff / mu;
      const double sigma = ratio * ratio * ratio;
      if (sr && tid == 0) {
        sr[0] = alpha;
        sr[1] = maff;
        sr[2] = sigma;
      }
      {
        const double *rl = V.row(R_RL), *ru = V.row(R_RU);
        double *rml = V.row(R_RML), *rmu = V.row(R_RMU), *w = V.row(R_W);
        for (int j = tid; j < m; j += NT) {
          rml[j] = tl[j] * ll[j] + dtl[j] * dll[j] - sigma * mu;
          rmu[j] = tu[j] * lu[j] + dtu[j] * dlu[j] - sigma * mu;
          w[j] = (rml[j] + ll[j] * rl[j]) / tl[j] - (rmu[j] + lu[j] * ru[j]) / tu[j];
        }
      }
      __syncthreads();
      step_rhs(V);
      __syncthreads();
      OCP_STAMP(6);
      if constexpr (FAST) {
        const int N = a.L.N;
        bwd_vec_a(V, 0, N, true);
        __syncthreads();
        chain_affine<true>(V, CS, S.vec, S.vec + 64);
        __syncthreads();
        bwd_vec_c(V, 0, N);
      } else {
        backward_vec_pass(V, S);
      }
      __syncthreads();
      OCP_STAMP(7);
      acl_pass(V, S, false);
      __syncthreads();
      if constexpr (FAST) chain_affine<false>(V, CS, S.vec, S.vec + 64);
      else forward_pass(V, S);
      OCP_STAMP(8);
      amax = block_reduce(post_pass(V), S.red, OpMin());
      OCP_STAMP(5);
      alpha = fmin(1.0, TAU_OCP * amax);
    }
    if (sr && tid == 0) sr[3] = sr[4] = alpha;
    if (LINRES && a.linres && it < a.stat_rows) {  // the Newton system's residuals at the final direction (cmpc_ocp_set_linres)
      double lr[4] = {0.0, 0.0, 0.0, 0.0};
      __syncthreads();
      lin_res(V, a.reg, 0, N + 1, lr);
      double* lo = a.linres + ((long long)q * a.stat_rows + it) * 4;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const double v = block_reduce(lr[c], S.red, OpMax());
        if (tid == 0) lo[c] = v;
      }
    }
    if (alpha < a.alpha_min) {
      status = 2;
      break;
    }
    // --- update ---
    for (int i = tid + nx; i < (N + 1) * nx; i += NT) x[i] = fma(alpha, V.dx()[i], x[i]);
    for (int i = tid; i < L.nU; i += NT) u[i] = fma(alpha, V.du()[i], u[i]);
    for (int i = tid; i < N * nx; i += NT) V.pi()[i] = fma(alpha, V.dpi()[i], V.pi()[i]);
    {
      double *tl = V.row(R_TL), *tu = V.row(R_TU), *ll = V.row(R_LL), *lu = V.row(R_LU);
      const double *dtl = V.row(R_DTL), *dtu = V.row(R_DTU), *dll = V.row(R_DLL), *dlu = V.row(R_DLU);
      for (int j = tid; j < m; j += NT) {
        tl[j] = fma(alpha, dtl[j], tl[j]);
        tu[j] = fma(alpha, dtu[j], tu[j]);
        ll[j] = fma(alpha, dll[j], ll[j]);
        lu[j] = fma(alpha, dlu[j], lu[j]);
      }
    }
    __syncthreads();
    OCP_STAMP(9);
  }
  // --- outputs ---
  bool fin = true;
  for (int i = tid; i < (N + 1) * nx; i += NT) {
    const double v = x[i];
    fin = fin && isfinite(v);
    a.x[(long long)q * (N + 1) * nx + i] = v;
  }
  for (int i = tid; i < L.nU; i += NT) {
    const double v = u[i];
    fin = fin && isfinite(v);
    a.u[(long long)q * L.nU + i] = v;
  }
  const bool allfin = __syncthreads_and(fin) != 0;
  if (tid == 0) {
    if (!allfin) status = 3;
    a.status[q] = status;
    if (a.iters) a.iters[q] = it;
    if (a.res) {
      a.res[(long long)q * 4 + 0] = rs;
      a.res[(long long)q * 4 + 1] = re;
      a.res[(long long)q * 4 + 2] = ri;
      a.res[(long long)q * 4 + 3] = rc;
    }
  }
  if (a.stats)  // rows after the last iteration: NaN (cmpc.h)
    for (int e = tid; e < (a.stat_rows - it - 1) * 10; e += NT)
      a.stats[((long long)q * a.stat_rows + it + 1) * 10 + e] = __builtin_nan("");
  if (a.linres)  // rows after the last iteration: NaN (the last one's is NaN unless it computed a direction)
    for (int e = tid; e < (a.stat_rows - it - 1) * 4; e += NT)
      a.linres[((long long)q * a.stat_rows + it + 1) * 4 + e] = __builtin_nan("");
}

// MINB workgroups per CU: 1 (the whole register file for one problem's chain: the lowest latency, B <= #CUs) or 2
// (bounded at 256 VGPRs, spilling some bookkeeping: 1.4-1.5x the solves/s of a full chip, 10 % slower per problem)
// Stage 0 of the Riccati getters, the reference's reconstruction (HpipmInterface.cpp:334-347, 376-389, 416-453) from
// node 1's P, p (in Po, po), stage 0's Lr (Lro) and the stage-0 record; writes P_0, p_0, K_0, k_0. Workgroup-wide.
__device__ __forceinline__ void ric_stage0(const View& V, const Lds& S, double* Po, double* po, double* Ko, double* ko,
                                           const double* Lro) {
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, nx = L.nx;
  // stage 0, the reference's reconstruction (HpipmInterface.cpp:334-347, 376-389, 416-453) from P_1, p_1, Lr_0 and the
  // stage-0 record: PA = P_1 A_0, v = p_1 + P_1 b_0, Mux = S_0 + B_0'PA, gr = r_0 + B_0'v, T1 = Lr_0^-1 Mux,
  // t2 = Lr_0^-1 gr, K_0 = -Lr_0^-T T1, k_0 = -Lr_0^-T t2, P_0 = Q_0 + A_0'PA - T1'T1, p_0 = q_0 + A_0'v - T1't2.
  // LDS: PA [nx][nx] in ABx, Mux / T1 [m0][nx] in Tx, v, gr / t2.
  {
    const int m0 = L.nu[0];
    const double* P1 = Po + (long long)nx * nx;
    const double* p1 = po + nx;
    const double* A = V.A(0);
    const double* Bm = V.Bm(0);
    double* PA = S.ABx;
    double* Mux = S.Tx;
    double* v = S.vec;
    double* gr = S.vec + 64;
    for (int e = tid; e < nx * nx; e += NT) {
      const int i = e / nx, j = e % nx;  // PA[i][j]
      double s = 0.0;
      for (int t = 0; t < nx; ++t) s = fma(P1[(long long)t * nx + i], A[(long long)j * nx + t], s);
      PA[i * nx + j] = s;
    }
    for (int i = tid; i < nx; i += NT) {
      double s = p1[i];
      for (int t = 0; t < nx; ++t) s = fma(P1[(long long)t * nx + i], V.b(0)[t], s);
      v[i] = s;
    }
    __syncthreads();
    for (int e = tid; e < m0 * nx + m0; e += NT) {
      if (e < m0 * nx) {
        const int a2 = e / nx, j = e % nx;
        double s = V.S(0)[(long long)j * m0 + a2];
        for (int t = 0; t < nx; ++t) s = fma(Bm[(long long)a2 * nx + t], PA[t * nx + j], s);
        Mux[a2 * nx + j] = s;
      } else {
        const int a2 = e - m0 * nx;
        double s = V.r(0)[a2];
        for (int t = 0; t < nx; ++t) s = fma(Bm[(long long)a2 * nx + t], v[t], s);
        gr[a2] = s;
      }
    }
    __syncthreads();
    // T1 = Lr_0^-1 Mux (in place, Tx), t2 = Lr_0^-1 gr (in place); K_0 = -Lr_0^-T T1, k_0 = -Lr_0^-T t2 (in place in
    // the outputs); one thread per right-hand side, the factor's guarded pivots (diag 0) contributing 0 as in HPIPM
    const double* Lr0 = Lro;
    for (int j = tid; j <= nx; j += NT) {
      double* c = j < nx ? Mux + j : gr;
      const int cs = j < nx ? nx : 1;
      double* o = j < nx ? Ko + (long long)j * m0 : ko;
      for (int a2 = 0; a2 < m0; ++a2) {
        double s = c[a2 * cs];
        for (int b = 0; b < a2; ++b) s = fma(-Lr0[(long long)b * m0 + a2], c[b * cs], s);
        const double d = Lr0[(long long)a2 * m0 + a2];
        c[a2 * cs] = d > 0.0 ? s / d : 0.0;
      }
      for (int a2 = m0 - 1; a2 >= 0; --a2) {
        double s = c[a2 * cs];
        for (int b = a2 + 1; b < m0; ++b) s = fma(-Lr0[(long long)a2 * m0 + b], o[b], s);
        const double d = Lr0[(long long)a2 * m0 + a2];
        o[a2] = d > 0.0 ? s / d : 0.0;
      }
      for (int a2 = 0; a2 < m0; ++a2) o[a2] = -o[a2];
    }
    __syncthreads();
    for (int e = tid; e < nx * nx + nx; e += NT) {
      if (e < nx * nx) {
        const int j = e / nx, i = e % nx;  // P_0 (i, j) = Q_0 + A_0'PA - T1'T1
        double s = V.Q(0)[(long long)j * nx + i];
        for (int t = 0; t < nx; ++t) s = fma(A[(long long)i * nx + t], PA[t * nx + j], s);
        for (int a2 = 0; a2 < m0; ++a2) s = fma(-Mux[a2 * nx + i], Mux[a2 * nx + j], s);
        Po[e] = s;
      } else {
        const int i = e - nx * nx;  // p_0 = q_0 + A_0'v - T1't2
        double s = V.q(0)[i];
        for (int t = 0; t < nx; ++t) s = fma(A[(long long)i * nx + t], v[t], s);
        for (int a2 = 0; a2 < m0; ++a2) s = fma(-Mux[a2 * nx + i], gr[a2], s);
        po[i] = s;
      }
    }
  }
}

// The IPM of ipm_body in the grid form: problem q on workgroups q G .. q G + G - 1 (see grid_range). Same iteration,
// same stopping rule, statistics and outputs; the latency-form factorisation (FAST) or factor_pass on workgroup 0.
template <bool FAST>
__device__ __forceinline__ void ipm_grid(const OcpSolveArgs& a, int q, int g, const Lds& S, const ChainLds& CS) {
  const View V(a, q);
  const OcpLayout& L = a.L;
  const int tid = threadIdx.x, nx = L.nx, N = L.N, m = L.m, G = a.G;
  const GridRange R = grid_range(L, g, G);
  const bool lead = g == 0, last = g == G - 1;
  unsigned* bar = a.bar + 4 * (long long)q;
  double* part = a.gpart + 8 * (long long)G * q;  // [G][8] partials of this problem
  // Slots: a workgroup may write its next partial while a slower one still reads the last collected values (the
  // barrier precedes the collect, not the next write), so partials collected back to back use different slots:
  // 0-4 residuals, 5 factorisation status / corrector step / exit checks, 6 predictor step, 7 mu_aff / finite check.
  double* mine = part + 8 * g;
  double* fl = S.red + 32;   // LDS: barrier flag [0], reduced values [1..8]
  double* red = S.red + 40;  // reduced partials
  unsigned nbar = 0;
  bool alive = true;
  auto sync = [&]() {
    if (alive) alive = grid_sync(bar, (++nbar) * (unsigned)G, fl, a.grid_timeout);
    return alive;
  };
  const int ops_res[5] = {0, 0, 0, 0, 1};
  const int ops_min[1] = {2};
  const int ops_sum[1] = {1};
  const int ops_max[1] = {0};
  double* x = V.x();
  double* u = V.u();
  double* hp = FAST ? a.hp + (long long)q * a.hp_stride : nullptr;
  // The factorisation (ocp_part.hpp): nseg segments of the horizon on workgroups 0 .. nseg-1 — P1 (the last segment
  // from the terminal node, the middle ones from a zero value function, then their elements), P2 (the combine on
  // workgroup 0), P3 (segments 0 .. nseg-2 from their end node's exact value) — or, with one segment, the serial
  // chain on workgroup 0. Leaves mine[5] = the NaN flag for the caller's barrier + collect. Partials: the first
  // pass's flags in slot 4, the combine's in slot 6 (both collected well before their next writers, see above).
  double* segq = a.seg ? a.seg + (long long)q * a.seg_stride : nullptr;
  const int nseg = (FAST && segq) ? part_segments(a.nseg, G, N, L.m) : 1;
  unsigned fgen = 0;  // partitioned factorisations so far (the generation of the level word's values)
  // segments of the partitioned affine scans (ocp_part.hpp): at most the steps N - 1 and what affine_bound stages
  const int naff = [&] {
    int Sa = nseg < N - 1 ? nseg : N - 1;
    const int cap = 1 + CH_SCRATCH / (nx * (nx + 1));
    return Sa > cap ? cap : Sa;
  }();
  // a serial vector recursion of the chain (the rollout, BWD = false, or the corrector's cost-to-go): on workgroup 0,
  // or as the partitioned scan (A: compositions, B: boundary values, C: the segments' own steps); false when a grid
  // barrier failed. The caller's barrier follows.
  auto affine_scan = [&](auto bwd) __attribute__((always_inline)) -> bool {
    constexpr bool BWD = decltype(bwd)::value;
    if constexpr (FAST) {
      if (naff <= 1) {
        if (lead) chain_affine<BWD>(V, CS, S.vec, S.vec + 64);
        return true;
      }
      const int n = N - 1, s0 = aff_begin(n, naff, g < naff ? g : naff), s1 = aff_begin(n, naff, g < naff ? g + 1 : naff);
      if (g < naff - 1) affine_comp<BWD>(V, CS, s0, s1, segq + g * seg_esz(nx));
      OCP_STAMP(34);
      if (!sync()) return false;
      OCP_STAMP(35);
      if (g >= 1 && g < naff) affine_bound<BWD>(V, CS, segq, naff, g, S.vec);
      if (g < naff) chain_affine<BWD>(V, CS, S.vec, S.vec + 64, s0, s1, g < naff - 1);
    } else if (lead) {
      if constexpr (BWD) bwd_vec_b(V, S);
      else forward_pass(V, S);
    }
    return true;
  };
  auto factor_grid = [&]() __attribute__((always_inline)) -> bool {
    if (nseg <= 1) {  // the serial chain on workgroup 0
      if (lead) {
        const bool fok = chain_factor(V, CS, hp, a.reg);
        if (tid == 0) mine[5] = fok ? 0.0 : 1.0;
      } else if (tid == 0) {
        mine[5] = 0.0;
      }
      return true;
    }
    // phase 0 = P1: the last segment from the terminal node, the middle ones from a zero end value (then their
    // elements); phase 1 = P2 on workgroup 0 with P3 behind it: segment g < nseg-1 refactorises from boundary g + 1's
    // exact value as soon as workgroup 0 has published it (segment 0, on workgroup 0, after the last combine);
    // phase 2 (a dropped pivot in the first pass, a NaN or a failed combine): the serial chain on workgroup 0. One
    // chain_factor call site (each inlined copy of the chain costs registers); workgroups g >= nseg only take part in
    // the barriers.
    const int cb = seg_begin(N, nseg, g < nseg ? g : nseg), ce = seg_begin(N, nseg, g < nseg ? g + 1 : nseg);
    const bool mid = g >= 1 && g < nseg - 1;
    unsigned* lvl = bar + 3;
    const unsigned gen = ++fgen;
    int f = 0;
    bool pok = true;
    for (int ph = 0; ph < 3; ++ph) {
      bool run;
      int k0 = cb, k1 = ce, term = CH_TERM_ZERO;
      const double* Pt = nullptr;
      if (ph == 0) {
        run = g >= 1 && g < nseg;
        if (g == nseg - 1) {
          k1 = N;
          term = CH_TERM_NODE;
        }
      } else if (ph == 1) {
        if (!pok) continue;
        run = g < nseg - 1;
        term = CH_TERM_GIVEN;
        Pt = segq + OCP_GRID_MAX_G * seg_esz(nx) + (g + 1) * seg_bsz(nx);
        bool cok = true;
        if (lead) {
          cok = seg_combine(V, CS, segq, nseg, N, lvl, gen);
          run = run && cok;
        } else if (run) {
          const int w = seg_wait(bar, lvl, gen * 64u + (unsigned)(nseg - g - 1), gen * 64u + SEG_FAIL, red,
                                 a.grid_timeout);
          if (w < 0) {
            alive = false;
            return false;
          }
          run = w > 0;
        }
        if (tid == 0) mine[6] = cok ? 0.0 : 1.0;
      } else {
        if (pok) break;
        run = lead;
        k0 = 0;
        k1 = N;
        term = CH_TERM_NODE;
        if (lead && tid == 0 && a.fallbacks)
          __hip_atomic_fetch_add(a.fallbacks + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      OCP_SPAN_BEGIN(t_ch);
      f = run ? chain_factor<true>(V, CS, hp, a.reg, k0, k1, term, Pt, Pt ? Pt + nx * nx : nullptr) : 0;
      OCP_SPANG_END(30, t_ch, 1);
      if (ph == 2) break;
      if (ph == 0) {
        OCP_SPAN_BEGIN(t_el);
        if (f == 0 && mid) f |= seg_element(V, CS, cb, ce, segq + g * seg_esz(nx));
        OCP_SPANG_END(31, t_el, 1);
        if (tid == 0) mine[4] = (double)f;
        if (!sync()) return false;
        grid_collect(part + 4, G, 1, ops_max, red);
        OCP_STAMP(18);
        pok = red[0] == 0.0;
      } else {
        if (!sync()) return false;
        grid_collect(part + 6, G, 1, ops_max, red);
        OCP_STAMP(19);
        pok = red[0] == 0.0;
      }
    }
    OCP_STAMP(29);
    if (tid == 0) mine[5] = (f & CH_NAN) ? 1.0 : 0.0;
    return true;
  };
  if (FAST) {  // this workgroup's stages' constant Hessian blocks (read by workgroup 0's chain after a barrier)
    const int e0 = L.cHp[R.k0], e1 = L.cHp[R.k1];
    int k = R.k0;
    for (int e = e0 + tid; e < e1; e += NT) {
      while (e >= L.cHp[k + 1]) ++k;
      const int le = e - L.cHp[k], tau = le >> 2, aa = (le >> 1) & 1, bb = le & 1;
      int bi, bj;
      ch_block(tau, bi, bj);
      const int i = 2 * bi + aa, l = 2 * bj + bb;
      const int mk = L.nu[k], nz = mk + nx;
      double v = 0.0;
      if (i >= l && i < nz && l < nz) {
        if (i < mk) v = V.R(k)[l * mk + i] + (i == l ? a.reg : 0.0);
        else if (l < mk) v = V.S(k)[(i - mk) * mk + l];
        else v = V.Q(k)[(l - mk) * nx + (i - mk)] + (i == l ? a.reg : 0.0);
      }
      hp[e] = v;
    }
  }
  // --- cold start on the owned nodes / stages / rows ---
  for (int i = R.k0 * nx + tid; i < R.n1 * nx; i += NT) {
    x[i] = i < nx ? a.x0[(long long)q * nx + i] : (a.warm ? a.x[(long long)q * (N + 1) * nx + i] : 0.0);
    V.dx()[i] = 0.0;
    V.gx()[i] = 0.0;
    V.rgx()[i] = 0.0;
  }
  for (int i = R.u0 + tid; i < R.u1; i += NT) u[i] = a.warm ? a.u[(long long)q * L.nU + i] : 0.0;
  for (int i = R.k0 * nx + tid; i < R.k1 * nx; i += NT) V.pi()[i] = 0.0;
  __syncthreads();
  {
    double* c = V.row(R_C);
    rows_value(V, x, u, c, R.r0, R.r1);
    double *lg = V.row(R_LG), *ug = V.row(R_UG), *tl = V.row(R_TL), *tu = V.row(R_TU), *ll = V.row(R_LL),
           *lu = V.row(R_LU);
    for (int j = R.r0 + tid; j < R.r1; j += NT) {
      const int k = L.rstage[j];
      const double bnd = -V.e(k)[j - L.cr[k]];
      lg[j] = bnd;
      ug[j] = bnd;
      tl[j] = fmax(c[j] - bnd, 1.0);
      tu[j] = fmax(bnd - c[j], 1.0);
      ll[j] = a.mu0 / tl[j];
      lu[j] = a.mu0 / tu[j];
    }
  }
  sync();  // every node's iterate before the first residuals
  OCP_STAMP(28);
  int status = 1, it = 0;
  double rs = 0, re = 0, ri = 0, rc = 0;
  // keep_riccati: the factorisation at the exit point (with rows; or without a step taken) runs through this loop's
  // factor phase once more (ric_pass), so the kernel carries one copy of the factorisation code
  bool ric_pass = false, rok = false;
  for (it = 0; alive; ++it) {
   double mu = 0.0;
   double* sr = nullptr;
   if (!ric_pass) {
    // --- residuals (owned nodes / rows), reduced over the grid ---
    rows_value(V, x, u, V.row(R_C), R.r0, R.r1);
    {
      double* w = V.row(R_W);
      const double *ll = V.row(R_LL), *lu = V.row(R_LU);
      for (int j = R.r0 + tid; j < R.r1; j += NT) w[j] = ll[j] - lu[j];
    }
    __syncthreads();
    double lrs = 0.0, lre = 0.0, lri = 0.0, lrc = 0.0, lmu = 0.0;
    residuals_par(V, lrs, lre, R.k0, R.n1);
    OCP_STAMP(32);
    {
      const double *c = V.row(R_C), *lg = V.row(R_LG), *ug = V.row(R_UG), *tl = V.row(R_TL), *tu = V.row(R_TU),
                   *ll = V.row(R_LL), *lu = V.row(R_LU);
      double *rl = V.row(R_RL), *ru = V.row(R_RU);
      for (int j = R.r0 + tid; j < R.r1; j += NT) {
        const double a1 = c[j] - lg[j] - tl[j], a2 = ug[j] - c[j] - tu[j];
        rl[j] = a1;
        ru[j] = a2;
        lri = nmax(lri, nmax(fabs(a1), fabs(a2)));
        const double c1 = tl[j] * ll[j], c2 = tu[j] * lu[j];
        lrc = nmax(lrc, nmax(c1, c2));
        lmu += c1 + c2;
      }
    }
    {
      // the five reductions in one pass (one barrier; the same wave trees and wave order as block_reduce)
      double v[5] = {lrs, lre, lri, lrc, lmu};
#pragma unroll
      for (int c = 0; c < 5; ++c)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const double w2 = __shfl_xor(v[c], o, 64);
          v[c] = c < 4 ? nmax(v[c], w2) : v[c] + w2;
        }
      __syncthreads();  // the previous users of S.red are done
      if ((tid & 63) == 0)
#pragma unroll
        for (int c = 0; c < 5; ++c) S.red[(tid >> 6) * 5 + c] = v[c];
      __syncthreads();
      if (tid == 0) {
#pragma unroll
        for (int c = 0; c < 5; ++c) {
          double r = S.red[c];
#pragma unroll
          for (int w = 1; w < NT / 64; ++w) r = c < 4 ? nmax(r, S.red[w * 5 + c]) : r + S.red[w * 5 + c];
          mine[c] = r;
        }
      }
    }
    if (!sync()) break;
    grid_collect(part, G, 5, ops_res, red);
    OCP_STAMP(1);
    rs = red[0];
    re = red[1];
    ri = red[2];
    rc = red[3];
    mu = m > 0 ? red[4] / (2.0 * m) : 0.0;
    sr = (lead && a.stats && it < a.stat_rows) ? a.stats + ((long long)q * a.stat_rows + it) * 10 : nullptr;
    if (sr && tid == 0 && a.linres)
      for (int c = 0; c < 4; ++c) a.linres[((long long)q * a.stat_rows + it) * 4 + c] = __builtin_nan("");
    if (sr && tid == 0) {
      for (int c = 0; c < 5; ++c) sr[c] = __builtin_nan("");
      sr[5] = mu;
      sr[6] = rs;
      sr[7] = re;
      sr[8] = ri;
      sr[9] = rc;
    }
    int ex = -1;
    if (!(isfinite(rs) && isfinite(re) && isfinite(ri) && isfinite(rc))) ex = 3;
    else if (rs <= a.tol_stat && re <= a.tol_eq && ri <= a.tol_ineq && rc <= a.tol_comp) ex = 0;
    else if (it >= a.iter_max) ex = 1;
    else if (m > 0 && !(mu > 1e-300)) ex = 2;
    if (ex >= 0) {
      status = ex;
      // the exit point's factorisation for keep_riccati: with rows at the exit point's Sigma; without rows the last
      // Newton step's factorisation is the exit point's (kept as it is), unless no step was taken
      if (!(a.ric && status != 3 && (m > 0 || it == 0))) break;
      ric_pass = true;
      {  // Sigma and the rows' step term at the exit iterate (complementarity kept), the step's right-hand side
        const double *tl = V.row(R_TL), *tu = V.row(R_TU), *ll = V.row(R_LL), *lu = V.row(R_LU), *rl = V.row(R_RL),
                     *ru = V.row(R_RU);
        double *sig = V.row(R_SIG), *w = V.row(R_W);
        for (int j = R.r0 + tid; j < R.r1; j += NT) {
          sig[j] = ll[j] / tl[j] + lu[j] / tu[j];
          w[j] = ll[j] * rl[j] / tl[j] - lu[j] * ru[j] / tu[j];
        }
      }
      __syncthreads();
      step_rhs_range(V, R.k0, R.k1, R.n1);
      if (!sync()) break;
    } else {
    // --- predictor right-hand side (owned rows / nodes) ---
    {
      const double *tl = V.row(R_TL), *tu = V.row(R_TU), *ll = V.row(R_LL), *lu = V.row(R_LU), *rl = V.row(R_RL),
                   *ru = V.row(R_RU);
      double *sig = V.row(R_SIG), *rml = V.row(R_RML), *rmu = V.row(R_RMU), *w = V.row(R_W);
      for (int j = R.r0 + tid; j < R.r1; j += NT) {
        sig[j] = ll[j] / tl[j] + lu[j] / tu[j];
        rml[j] = tl[j] * ll[j];
        rmu[j] = tu[j] * lu[j];
        w[j] = (rml[j] + ll[j] * rl[j]) / tl[j] - (rmu[j] + lu[j] * ru[j]) / tu[j];
      }
    }
    __syncthreads();
    step_rhs_range(V, R.k0, R.k1, R.n1);
    if (!sync()) break;
    }
   }
    OCP_STAMP(2);
    // --- factorisation: the partitioned chain over the grid (FAST; nseg = 1: the serial chain on workgroup 0) ---
    if constexpr (FAST) {
      if (!factor_grid()) break;
    } else if (lead) {
      const bool fok = factor_pass<64>(V, S, a.reg);
      if (tid == 0) mine[5] = fok ? 0.0 : 1.0;
    } else if (tid == 0) {
      mine[5] = 0.0;
    }
    if (!sync()) break;
    grid_collect(part + 5, G, 1, ops_max, red);
    OCP_STAMP(17);
    if (ric_pass) {
      rok = red[0] == 0.0;
      break;
    }
    if (red[0] != 0.0) {
      status = 3;
      break;
    }
    if constexpr (FAST) {  // the owned stages' gains from the chain's factor
      chain_gains(V, R.k0, R.k1);
      __syncthreads();
    }
    OCP_STAMP(33);
    acl_pass(V, S, true, R.k0, R.k1, true);
    if (!sync()) break;
    OCP_STAMP(3);
    if (!affine_scan(std::integral_constant<bool, false>{})) break;
    if (!sync()) break;
    OCP_STAMP(4);
    double amax = block_reduce(post_pass(V, R.k0, R.k1, R.n1), S.red, OpMin());
    if (m > 0) {
      if (tid == 0) mine[6] = amax;
      if (!sync()) break;
      grid_collect(part + 6, G, 1, ops_min, red);
      amax = red[0];
    }
    OCP_STAMP(5);
    double alpha = fmin(1.0, amax);
    if (m > 0) {
      // mu_aff and the corrector
      double lm = 0.0;
      const double *tl = V.row(R_TL), *tu = V.row(R_TU), *ll = V.row(R_LL), *lu = V.row(R_LU), *dtl = V.row(R_DTL),
                   *dtu = V.row(R_DTU), *dll = V.row(R_DLL), *dlu = V.row(R_DLU);
      for (int j = R.r0 + tid; j < R.r1; j += NT)
        lm += (tl[j] + alpha * dtl[j]) * (ll[j] + alpha * dll[j]) + (tu[j] + alpha * dtu[j]) * (lu[j] + alpha * dlu[j]);
      {
        const double v = block_reduce(lm, S.red, OpSum());
        if (tid == 0) mine[7] = v;
      }
      if (!sync()) break;
      grid_collect(part + 7, G, 1, ops_sum, red);
      const double maff = red[0] / (2.0 * m);
      const double ratio = maff / mu;
      const double sigma = ratio * ratio * ratio;
      if (sr && tid == 0) {
        sr[0] = alpha;
        sr[1] = maff;
        sr[2] = sigma;
      }
      {
        const double *rl = V.row(R_RL), *ru = V.row(R_RU);
        double *rml = V.row(R_RML), *rmu = V.row(R_RMU), *w = V.row(R_W);
        for (int j = R.r0 + tid; j < R.r1; j += NT) {
          rml[j] = tl[j] * ll[j] + dtl[j] * dll[j] - sigma * mu;
          rmu[j] = tu[j] * lu[j] + dtu[j] * dlu[j] - sigma * mu;
          w[j] = (rml[j] + ll[j] * rl[j]) / tl[j] - (rmu[j] + lu[j] * ru[j]) / tu[j];
        }
      }
      __syncthreads();
      step_rhs_range(V, R.k0, R.k1, R.n1);
      __syncthreads();
      OCP_STAMP(6);
      bwd_vec_a(V, R.k0, R.k1, last);
      if (!sync()) break;
      if (!affine_scan(std::integral_constant<bool, true>{})) break;
      if (!sync()) break;
      bwd_vec_c(V, R.k0, R.k1);
      __syncthreads();
      OCP_STAMP(7);
      acl_pass(V, S, false, R.k0, R.k1, true);
      if (!sync()) break;
      if (!affine_scan(std::integral_constant<bool, false>{})) break;
      if (!sync()) break;
      OCP_STAMP(8);
      {
        const double v = block_reduce(post_pass(V, R.k0, R.k1, R.n1), S.red, OpMin());
        if (tid == 0) mine[5] = v;
      }
      if (!sync()) break;
      grid_collect(part + 5, G, 1, ops_min, red);
      amax = red[0];
      alpha = fmin(1.0, TAU_OCP * amax);
    }
    if (sr && tid == 0) sr[3] = sr[4] = alpha;
    if (alpha < a.alpha_min) {
      status = 2;
      break;
    }
    // --- update (owned) ---
    for (int i = (R.k0 > 1 ? R.k0 : 1) * nx + tid; i < R.n1 * nx; i += NT) x[i] = fma(alpha, V.dx()[i], x[i]);
    for (int i = R.u0 + tid; i < R.u1; i += NT) u[i] = fma(alpha, V.du()[i], u[i]);
    for (int i = R.k0 * nx + tid; i < R.k1 * nx; i += NT) V.pi()[i] = fma(alpha, V.dpi()[i], V.pi()[i]);
    {
      double *tl = V.row(R_TL), *tu = V.row(R_TU), *ll = V.row(R_LL), *lu = V.row(R_LU);
      const double *dtl = V.row(R_DTL), *dtu = V.row(R_DTU), *dll = V.row(R_DLL), *dlu = V.row(R_DLU);
      for (int j = R.r0 + tid; j < R.r1; j += NT) {
        tl[j] = fma(alpha, dtl[j], tl[j]);
        tu[j] = fma(alpha, dtu[j], tu[j]);
        ll[j] = fma(alpha, dll[j], ll[j]);
        lu[j] = fma(alpha, dlu[j], lu[j]);
      }
    }
    if (!sync()) break;
    OCP_STAMP(9);
  }
  if (!alive) status = OCP_GRID_TIMEOUT;  // a barrier timed out: the grid drained; k_ocp_fallback re-solves
  // --- the exit point's Riccati quantities (cmpc_ocp_set_keep_riccati; k_ocp_ric's outputs, same formulas) ---
  if (a.ric && alive && status != 3) {
    // Without rows the last Newton step's factorisation is the exit point's (no Sigma): the solve keeps its P_k, K_k,
    // Lr_k only (factor-only; the exit point's p_k, kff_k and the stage-0 rebuild come from cmpc_ocp_riccati's
    // refactorisation when asked for, the MPC's feedback policy needs none of them). With rows (or when no step was
    // taken) the loop's last pass refactorised at the exit point (ric_pass) and everything is kept.
    const bool fonly = m == 0;
    const bool full = ric_pass;
    if (!full) rok = true;
    if (FAST && full) {
      chain_gains(V, R.k0, R.k1);
      __syncthreads();
    }
    const long long oP = (long long)q * (N + 1) * nx * nx, op = (long long)q * (N + 1) * nx;
    const long long oK = (long long)q * (L.nK > 0 ? L.nK : 1), ok2 = (long long)q * (L.nU > 0 ? L.nU : 1),
                    oM = (long long)q * (L.nM > 0 ? L.nM : 1);
    if (rok) {  // owned stages / nodes >= 1; the Lr factor of every owned stage
      for (int e = L.cK[R.k0] + tid; e < L.cK[R.k1]; e += NT) a.ricK[oK + e] = V.ws[L.o_K + e];
      for (int k = R.k0; k < R.k1; ++k) {
        const int mk = L.nu[k];
        const double* F = V.Lf(k);
        double* Lo = a.ricLr + oM + L.cM[k];
        for (int e = tid; e < mk * mk; e += NT) {
          const int j = e / mk, i = e - j * mk;
          const double d = F[(long long)j * mk + j];
          Lo[e] = (i >= j && d > 1e-200) ? F[e] / sqrt(d) : 0.0;
        }
      }
      for (int e = (R.k0 > 1 ? L.cu[R.k0] : L.cu[1]) + tid; !fonly && e < R.u1; e += NT) {
        const int k = L.ustage[e], a2 = e - L.cu[k], mk = L.nu[k];
        const double* Kk = V.K(k);
        double s2 = u[e] + V.kf()[e];
        for (int c = 0; c < nx; ++c) s2 = fma(-Kk[(long long)c * mk + a2], x[(long long)k * nx + c], s2);
        a.rick[ok2 + e] = s2;
      }
      const int na = R.k0 > 1 ? R.k0 : 1;
      for (int e = na * nx * nx + tid; e < R.n1 * nx * nx; e += NT) a.ricP[oP + e] = V.ws[L.o_P + e];
      for (int e = na * nx + tid; !fonly && e < R.n1 * nx; e += NT) {
        const int k = e / nx, i = e - k * nx;
        const double* Pk = V.P(k);
        double s2 = V.pi()[(long long)(k - 1) * nx + i] + V.pv()[e];
        for (int j = 0; j < nx; ++j) s2 = fma(-Pk[(long long)j * nx + i], x[(long long)k * nx + j], s2);
        a.ricp[op + e] = s2;
      }
    }
    sync();  // node 1's P, p and stage 0's Lr before the stage-0 reconstruction
    if (lead && rok && !fonly) ric_stage0(V, S, a.ricP + oP, a.ricp + op, a.ricK + oK, a.rick + ok2, a.ricLr + oM);
    if (lead && tid == 0) a.ricst[q] = rok ? 0 : 3;
  } else if (a.ric && lead && tid == 0) {
    a.ricst[q] = alive ? 3 : OCP_GRID_TIMEOUT;
  }
  // --- outputs (owned nodes / stages) ---
  bool fin = true;
  for (int i = R.k0 * nx + tid; i < R.n1 * nx; i += NT) {
    const double v = x[i];
    fin = fin && isfinite(v);
    a.x[(long long)q * (N + 1) * nx + i] = v;
  }
  for (int i = R.u0 + tid; i < R.u1; i += NT) {
    const double v = u[i];
    fin = fin && isfinite(v);
    a.u[(long long)q * L.nU + i] = v;
  }
  const bool allfin = __syncthreads_and(fin) != 0;
  if (tid == 0) mine[7] = allfin ? 0.0 : 1.0;
  const bool ok_end = sync();
  if (ok_end) grid_collect(part + 7, G, 1, ops_max, red);
  if (lead && tid == 0) {
    if (!ok_end) status = OCP_GRID_TIMEOUT;
    else if (red[0] != 0.0) status = 3;
    a.status[q] = status;
    if (a.iters) a.iters[q] = it;
    if (a.res) {
      a.res[(long long)q * 4 + 0] = rs;
      a.res[(long long)q * 4 + 1] = re;
      a.res[(long long)q * 4 + 2] = ri;
      a.res[(long long)q * 4 + 3] = rc;
    }
    if (a.stats)  // rows after the last iteration: NaN (cmpc.h)
      for (int r = it + 1; r < a.stat_rows; ++r)
        for (int c = 0; c < 10; ++c) a.stats[((long long)q * a.stat_rows + r) * 10 + c] = __builtin_nan("");
    if (a.linres)  // rows after the last iteration: NaN (the last one's is NaN unless it computed a direction)
      for (int r = it + 1; r < a.stat_rows; ++r)
        for (int c = 0; c < 4; ++c) a.linres[((long long)q * a.stat_rows + r) * 4 + c] = __builtin_nan("");
  }
  // the barrier words back to zero for the next launch (no memset launch before it): every workgroup counts itself
  // out after its last barrier; the last one out resets the counter, the fail word and the out-count (nobody polls
  // them any more by then)
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned out = __hip_atomic_fetch_add(bar + 2, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (out == (unsigned)G - 1) {
      __hip_atomic_store(bar + 0, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(bar + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(bar + 3, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(bar + 2, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Grid form: G workgroups per problem (B G <= 256, one per CU), launched as k_ocp_grid<FAST>
template <bool FAST>
__global__ __launch_bounds__(NT, 1) void k_ocp_grid(OcpSolveArgs a) {
  extern __shared__ double smem[];
  ChainLds CS{};
  const Lds S = FAST ? carve_fast(smem, a.L, CS) : carve(smem, a.L, 64);
  const int q = blockIdx.x / a.G, g = blockIdx.x - q * a.G;
  OCP_STAMP_BEGIN();
  ipm_grid<FAST>(a, q, g, S, CS);
  OCP_STAMP_END();
}

template <int NZP, int MINB, bool FAST>
__global__ __launch_bounds__(NT, MINB) void k_ocp_ipm(OcpSolveArgs a) {
  extern __shared__ double smem[];
  ChainLds CS{};
  const Lds S = FAST ? carve_fast(smem, a.L, CS) : carve(smem, a.L, NZP);
  OCP_STAMP_BEGIN();
  ipm_body<NZP, MINB, FAST>(a, blockIdx.x, S, CS);
  OCP_STAMP_END();
}

// The statistics solve (cmpc_ocp_set_linres: HPIPM's lin res columns of the verbose table): one workgroup per problem,
// the batched form's factorisation, the Newton systems' residuals recorded per iteration. A separate instantiation, so
// the solves' kernels carry none of it (the same iteration; trajectories equal the other forms' to rounding).
template <int NZP>
__global__ __launch_bounds__(NT, 1) void k_ocp_ipm_linres(OcpSolveArgs a) {
  extern __shared__ double smem[];
  ChainLds CS{};
  const Lds S = carve(smem, a.L, NZP);
  ipm_body<NZP, 1, false, true>(a, blockIdx.x, S, CS);
}

// Riccati quantities at the exit point (see k_ocp.hpp / cmpc.h cmpc_ocp_riccati) of problem q, one workgroup
template <int NZP>
__device__ __forceinline__ void ric_body(const OcpRicArgs& r, int q, const Lds& S) {
  const OcpSolveArgs& a = r.S;
  const OcpLayout& L = a.L;
  const int tid = threadIdx.x, nx = L.nx, N = L.N, m = L.m;
  const View V(a, q);
  if (a.status[q] == 3) {
    if (tid == 0) r.rstatus[q] = 3;
    return;
  }
  {
    const double *tl = V.row(R_TL), *tu = V.row(R_TU), *ll = V.row(R_LL), *lu = V.row(R_LU), *rl = V.row(R_RL),
                 *ru = V.row(R_RU);
    double *sig = V.row(R_SIG), *w = V.row(R_W);
    for (int j = tid; j < m; j += NT) {
      sig[j] = ll[j] / tl[j] + lu[j] / tu[j];
      w[j] = ll[j] * rl[j] / tl[j] - lu[j] * ru[j] / tu[j];
    }
  }
  __syncthreads();
  step_rhs(V);
  __syncthreads();
  const bool ok = factor_pass<NZP>(V, S, a.reg);
  const long long oP = (long long)q * (N + 1) * nx * nx, op = (long long)q * (N + 1) * nx;
  const long long oK = (long long)q * (L.nK > 0 ? L.nK : 1), ok2 = (long long)q * (L.nU > 0 ? L.nU : 1),
                  oM = (long long)q * (L.nM > 0 ? L.nM : 1);
  const double* x = V.x();
  const double* u = V.u();
  // stages k >= 1: K, k = u - K x + kf, P, p = pi_{k-1} - P x + pv
  for (int it = tid; it < L.nK; it += NT) r.K[oK + it] = V.ws[L.o_K + it];
  // Lr_k (HPIPM's ric_Lr): from the sweep's LDL' columns F (d_j = F(j, j)), Lr(i, j) = F(i, j) / sqrt(d_j) for i >= j,
  // 0 above the diagonal and in a guarded pivot's column
  for (int k = 0; k < N; ++k) {
    const int mk = L.nu[k];
    const double* F = V.Lf(k);
    double* Lo = r.Lr + oM + L.cM[k];
    for (int e = tid; e < mk * mk; e += NT) {
      const int j = e / mk, i = e % mk;
      const double d = F[(long long)j * mk + j];
      Lo[e] = (i >= j && d > 1e-200) ? F[e] / sqrt(d) : 0.0;
    }
  }
  for (int it = tid; it < L.nU; it += NT) {
    const int k = L.ustage[it], a2 = it - L.cu[k], mk = L.nu[k];
    if (k == 0) continue;
    const double* Kk = V.K(k);
    double s = u[it] + V.kf()[it];
    for (int c = 0; c < nx; ++c) s = fma(-Kk[(long long)c * mk + a2], x[(long long)k * nx + c], s);
    r.k[ok2 + it] = s;
  }
  for (int it = tid; it < N * nx * nx; it += NT) r.P[oP + (long long)nx * nx + it] = V.ws[L.o_P + (long long)nx * nx + it];
  for (int it = tid; it < N * nx; it += NT) {
    const int k = 1 + it / nx, i = it % nx;
    const double* Pk = V.P(k);
    double s = V.pi()[(long long)(k - 1) * nx + i] + V.pv()[(long long)k * nx + i];
    for (int j = 0; j < nx; ++j) s = fma(-Pk[(long long)j * nx + i], x[(long long)k * nx + j], s);
    r.p[op + (long long)k * nx + i] = s;
  }
  __syncthreads();
  ric_stage0(V, S, r.P + oP, r.p + op, r.K + oK, r.k + ok2, r.Lr + oM);
  if (tid == 0) r.rstatus[q] = ok ? 0 : 3;
}

template <int NZP>
__global__ __launch_bounds__(NT) void k_ocp_ric(OcpRicArgs r) {
  extern __shared__ double smem[];
  ric_body<NZP>(r, blockIdx.x, carve(smem, r.S.L, NZP));
}

// Fallback of the grid form, launched after k_ocp_grid on the same stream: a problem whose grid barriers timed out
// (status OCP_GRID_TIMEOUT: its workgroups were not all resident, e.g. another stream's kernels held the CUs) is
// re-solved by one workgroup in the latency form (ipm_body<64, 1, true>: the same iteration) and, when the solve keeps
// its Riccati quantities, refactorised at the exit point as k_ocp_ric does; every other problem's workgroup exits at
// its first instruction.
__global__ __launch_bounds__(NT, 1) void k_ocp_fallback(OcpSolveArgs a) {
  const int q = blockIdx.x;
  if (a.status[q] != OCP_GRID_TIMEOUT) return;
  extern __shared__ double smem[];
  ChainLds CS{};
  const Lds S = carve_fast(smem, a.L, CS);
  ipm_body<64, 1, true>(a, q, S, CS);
  if (a.ric) {
    __syncthreads();
    OcpRicArgs r;
    r.S = a;
    r.P = a.ricP;
    r.p = a.ricp;
    r.K = a.ricK;
    r.k = a.rick;
    r.Lr = a.ricLr;
    r.rstatus = a.ricst;
    ric_body<64>(r, q, carve(smem, a.L, 64));
  }
  if (threadIdx.x == 0 && a.fallbacks) __hip_atomic_fetch_add(a.fallbacks, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

#ifdef CMPC_OCP_CHAIN_LAB
// Lab only (lab/ocp_stamps.sh): the latency-form factorisation alone on the workspace of the last solve, for timing
// the chain in isolation (cmpc_ocp_debug_chain)
namespace {
__global__ __launch_bounds__(NT, 1) void k_ocp_chain_lab(OcpSolveArgs a) {
  extern __shared__ double smem[];
  ChainLds CS{};
  (void)carve_fast(smem, a.L, CS);
  const View V(a, blockIdx.x);
  double* hp = a.hp + (long long)blockIdx.x * a.hp_stride;
  hp_build(V, hp, a.reg);
  __syncthreads();
  if (!chain_factor(V, CS, hp, a.reg) && threadIdx.x == 0) a.status[blockIdx.x] = 3;
  chain_gains(V, 0, a.L.N);
}
}  // namespace
int launch_ocp_chain_lab(const OcpSolveArgs& a, int B, hipStream_t stream) {
  const size_t lc = ocp_chain_lds_bytes(a.L, a.L.numax);
  if (!lc || !a.hp) return -1;
  if (hipFuncSetAttribute((const void*)k_ocp_chain_lab, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lc) !=
      hipSuccess)
    return -1;
  hipLaunchKernelGGL(k_ocp_chain_lab, dim3(B), dim3(NT), lc, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
#endif

#ifdef CMPC_OCP_STAMPS
extern "C" int cmpc_ocp_debug_stamps(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ocp_stamp_acc), sizeof(unsigned long long) * 48) != hipSuccess) return -2;
  if (reset) {
    unsigned long long z[32] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(ocp_stamp_acc), z, sizeof(z)) != hipSuccess) return -2;
  }
  return 0;
}
#endif

size_t ocp_lds_bytes(const OcpLayout& L) {
  const int np1 = L.nx + 1, nrm = L.nx + 1 + L.ngmax;
  const size_t pa = (size_t)((np1 * np1 + 1) & ~1);
  return sizeof(double) * (pa + 2 * (size_t)nrm * L.nzp + 4 * (size_t)L.nzp + 128 + 64 + 64);
}

// CUs of the current device (cached per device: every workgroup of the grid needs a CU of its own)
static int device_cus() {
  static int ncu[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  const int slot = dev < 64 ? dev : 63;
  if (ncu[slot] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 1;
    ncu[slot] = n;
  }
  return ncu[slot];
}

int ocp_grid_width(int N, int B, int want) {
  if (B <= 0 || B > OCP_GRID_MAX_B) return 0;
  const int ncu = device_cus();
  const int cap = ncu < OCP_GRID_MAX_WG ? ncu : OCP_GRID_MAX_WG;
  int G = want > 0 ? want : OCP_GRID_MAX_G;
  if (G > N) G = N;
  if (G * B > cap) G = cap / B;
  if (G > OCP_GRID_MAX_G) G = OCP_GRID_MAX_G;
  return G >= 2 ? G : 0;
}

size_t ocp_chain_lds_bytes(const OcpLayout& L, int numax) {
  if (L.nzp != 64 || L.nx > OCP_CHAIN_MAX_NX || numax > OCP_CHAIN_MAX_NU || L.nx + numax + 1 > OCP_CHAIN_MAX_N1 ||
      L.ngmax > CH_MAXG || L.N > CH_MAXN)
    return 0;
  const size_t ngr = CH_NRP + (size_t)((L.ngmax + 3) & ~3), ngp = (size_t)((L.ngmax + 4) & ~3);
  const size_t g1 = std::max(ngr * CH_GS, (size_t)CH_MAXU * CH_FS);
  const size_t d = ngr * CH_GS + g1 + (size_t)CH_NRP * CH_GS + CH_PS * CH_PS + 256 + 2 * ngp + 64 + 128 +
                   (size_t)CH_MR * CH_GS + 4 * CH_MAXNT + 64 + CH_PS * CH_PS + (size_t)CH_MAXU * CH_FS;
  const size_t bytes = sizeof(double) * d + sizeof(int) * CH_DESC * (size_t)L.N;
  return bytes <= 160 * 1024 ? bytes : 0;  // beyond the LDS: the batched form
}

// G of the grid form for a batch of B problems of layout L (0: not the grid form): ocp_grid_width, capped by the
// co-residency the kernel's registers and LDS admit on the current device (one workgroup per CU at most is used; the
// occupancy query is cached per device and LDS size). Other streams' kernels can still hold CUs at the launch: the
// barriers' time bound and the fallback launch cover that.
int ocp_grid_for(const OcpLayout& L, int B, int want) {
  const size_t lc = ocp_chain_lds_bytes(L, L.numax);
  if (!lc) return 0;
  int G = ocp_grid_width(L.N, B, want);
  if (G == 0) return 0;
  const size_t lds = std::max(ocp_lds_bytes(L), lc);
  struct Occ {
    int dev;
    size_t lds;
    int per_cu;
  };
  static Occ cache[16];
  static int ncache = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  int per_cu = -1;
  for (int i = 0; i < ncache; ++i)
    if (cache[i].dev == dev && cache[i].lds == lds) per_cu = cache[i].per_cu;
  if (per_cu < 0) {
    per_cu = 0;
    if (hipFuncSetAttribute((const void*)k_ocp_grid<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) ==
            hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_ocp_grid<true>, NT, lds) != hipSuccess)
      per_cu = 0;
    cache[ncache < 16 ? ncache++ : 15] = Occ{dev, lds, per_cu};
  }
  const long long resident = (long long)std::min(per_cu, 1) * device_cus();
  if ((long long)B * G > resident) G = (int)(resident / B);
  if (G > OCP_GRID_MAX_G) G = OCP_GRID_MAX_G;
  return G >= 2 ? G : 0;
}

int launch_ocp_ipm(const OcpSolveArgs& a0, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  OcpSolveArgs a = a0;
  a.par_res = B <= OCP_PAR_RES_MAX ? 1 : 0;
  const size_t lc = ocp_chain_lds_bytes(a.L, a.L.numax);
  if (a.linres) {  // the statistics solve (k_ocp_ipm_linres)
    a.fast = 0;
    const size_t l0 = ocp_lds_bytes(a.L);
    const void* kf = a.L.nzp == 64 ? (const void*)k_ocp_ipm_linres<64> : (const void*)k_ocp_ipm_linres<128>;
    if (hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l0) != hipSuccess) return -1;
    if (a.L.nzp == 64) hipLaunchKernelGGL(k_ocp_ipm_linres<64>, dim3(B), dim3(NT), l0, stream, a);
    else hipLaunchKernelGGL(k_ocp_ipm_linres<128>, dim3(B), dim3(NT), l0, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  a.fast = (a0.fast && a0.hp && lc > 0 && B <= OCP_ONE_PER_CU_MAX) ? 1 : 0;
  size_t lds = ocp_lds_bytes(a.L);
  if (a.fast && lc > lds) lds = lc;
  const int G = a.fast && a.bar && a.gpart ? ocp_grid_for(a.L, B, a.G) : 0;
  if (G > 0) {  // grid form: G workgroups per problem, one per CU
    a.G = G;
    // the barrier words are zero at allocation and every launch leaves them zero (ipm_grid's last workgroup out)
    if (hipFuncSetAttribute((const void*)k_ocp_grid<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
        hipSuccess)
      return -1;
    hipLaunchKernelGGL(k_ocp_grid<true>, dim3(B * G), dim3(NT), lds, stream, a);
    // problems whose barriers timed out (status OCP_GRID_TIMEOUT) re-solved on one workgroup; the others exit at once
    if (hipFuncSetAttribute((const void*)k_ocp_fallback, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
        hipSuccess)
      return -1;
    hipLaunchKernelGGL(k_ocp_fallback, dim3(B), dim3(NT), lds, stream, a);
  } else if (a.fast) {  // the latency form (k_ocp_ipm<64, 1, true>): B <= OCP_ONE_PER_CU_MAX, one problem per CU
    if (hipFuncSetAttribute((const void*)k_ocp_ipm<64, 1, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
      return -1;
    hipLaunchKernelGGL((k_ocp_ipm<64, 1, true>), dim3(B), dim3(NT), lds, stream, a);
  } else if (a.L.nzp == 64) {
    // one problem per CU while the batch leaves CUs idle anyway, two per CU beyond (cmpc_ocp_solve's B)
    const bool two = B > OCP_ONE_PER_CU_MAX;
    const void* kf = two ? (const void*)k_ocp_ipm<64, 2, false> : (const void*)k_ocp_ipm<64, 1, false>;
    if (hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return -1;
    if (two)
      hipLaunchKernelGGL((k_ocp_ipm<64, 2, false>), dim3(B), dim3(NT), lds, stream, a);
    else
      hipLaunchKernelGGL((k_ocp_ipm<64, 1, false>), dim3(B), dim3(NT), lds, stream, a);
  } else {
    if (hipFuncSetAttribute((const void*)k_ocp_ipm<128, 1, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds) != hipSuccess)
      return -1;
    hipLaunchKernelGGL((k_ocp_ipm<128, 1, false>), dim3(B), dim3(NT), lds, stream, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_ocp_ric(const OcpRicArgs& a, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  const size_t lds = ocp_lds_bytes(a.S.L);
  if (a.S.L.nzp == 64) {
    if (hipFuncSetAttribute((const void*)k_ocp_ric<64>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
        hipSuccess)
      return -1;
    hipLaunchKernelGGL(k_ocp_ric<64>, dim3(B), dim3(NT), lds, stream, a);
  } else {
    if (hipFuncSetAttribute((const void*)k_ocp_ric<128>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
        hipSuccess)
      return -1;
    hipLaunchKernelGGL(k_ocp_ric<128>, dim3(B), dim3(NT), lds, stream, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cmpc
