// k_misc.hip — the small kernels around the hot path: synthetic input generation, result scatter/rollout,
// precision conversion, class lists, warm-start packing (the HpipmInterface::solve path is k_ocp.hip).
#include "cmpc_device.hpp"
#include "cmpc_kernels.hpp"

namespace cmpc {

// ------------------------------------------------------------------------------------------ generator
// Philox4x32-10 keyed by seed, counter = (global QP id, draw block, "CMPC"); bit-identical to oracle_generate().

__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n1 = lo1, n2 = hi0 ^ c[3] ^ k1, n3 = lo0;
    c[0] = n0;
    c[1] = n1;
    c[2] = n2;
    c[3] = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__device__ __forceinline__ double gen_uniform(uint64_t seed, uint64_t gid, int idx) {
  uint32_t c[4] = {(uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)(idx >> 1), 0x43504D43u};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const uint64_t v = (idx & 1) ? ((uint64_t)c[3] << 32 | c[2]) : ((uint64_t)c[1] << 32 | c[0]);
  return (double)(v >> 11) * 0x1.0p-53;
}

__device__ __forceinline__ double urange(double a, double b, double u) { return __builtin_fma(b - a, u, a); }

struct GenArgs {
  int N, L;
  double dt;
  uint64_t seed;
  int64_t qp_offset;
  int gait;
  double* x0;
  double* xref;
  double* foot;
  uint8_t* contact;
};

__global__ __launch_bounds__(256) void k_generate(GenArgs a, int B) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= B) return;
  const int N = a.N, L = a.L;
  const uint64_t gid = (uint64_t)(a.qp_offset + q);
  const double nom[4][2] = {{0.35, 0.052}, {0.35, -0.054}, {-0.37, -0.053}, {-0.36, 0.054}};
  const double PI = 3.14159265358979323846;
  double U[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) U[i] = gen_uniform(a.seed, gid, i);
  double* X0 = a.x0 + (size_t)q * NX;
  double x0v[NX];
  x0v[0] = urange(-0.2, 0.2, U[0]);
  x0v[1] = urange(-0.2, 0.2, U[1]);
  x0v[2] = urange(0.12, 0.20, U[2]);
  x0v[3] = urange(-1.0, 1.0, U[3]);
  x0v[4] = urange(-1.0, 1.0, U[4]);
  x0v[5] = urange(-0.2, 0.2, U[5]);
  for (int d = 0; d < 3; ++d) x0v[6 + d] = urange(-0.1, 0.1, U[6 + d]);
  x0v[9] = urange(-0.1, 0.1, U[9]);
  x0v[10] = urange(-0.1, 0.1, U[10]);
  x0v[11] = urange(-PI, PI, U[11]);
  x0v[12] = -GRAV;
  for (int s = 0; s < NX; ++s) X0[s] = x0v[s];
  const double vdx = urange(-1.0, 1.0, U[12]), vdy = urange(-1.0, 1.0, U[13]);
  // contact schedule first: the stance runs decide where the feet are planted
  const int h = GAIT_HALF_PERIOD;
  const int phase = (int)(U[22] * (double)(2 * h));
  const int gsel = a.gait == 1 ? (int)(U[23] * 3.0) : 0;
  uint8_t* C = a.contact + (size_t)q * N * L;
  for (int k = 0; k < N; ++k) {
    const bool first = ((k + phase) % (2 * h)) < h;
    for (int i = 0; i < L; ++i) {
      bool e;
      if (gsel == 0) e = first ? (i == 0 || i == 2) : (i == 1 || i == 3);  // trot (CentoidMPCTest.cpp:68-73)
      else if (gsel == 1) e = first ? (i < 2) : (i >= 2);                    // bound
      else e = true;                                                          // pronk, stance phase
      C[k * L + i] = (uint8_t)e;
    }
  }
  double* XR = a.xref + (size_t)q * (N + 1) * NX;
  double* FT = a.foot + (size_t)q * (N + 1) * L * 3;
  for (int k = 0; k <= N; ++k) {
    double* xr = XR + k * NX;
    const double tk = (double)k * a.dt;
    const double cx = __builtin_fma(tk, vdx, x0v[0]), cy = __builtin_fma(tk, vdy, x0v[1]);
    xr[0] = cx;
    xr[1] = cy;
    xr[2] = 0.15;
    xr[3] = vdx;
    xr[4] = vdy;
    xr[5] = 0.0;
    for (int d = 6; d < 11; ++d) xr[d] = 0.0;
    xr[11] = x0v[11];
    xr[12] = -GRAV;
  }
  // Feet: a node pinned by a stance run (step k or step k-1 in stance) holds the foothold planted at the run's
  // touch-down step s, nominal offset + per-leg perturbation around c^ref_s; a swing node follows the body. Node 0
  // is the measured current foot (cmpc.h record), the planted foothold plus a +-1 cm measurement offset.
  for (int k = 0; k <= N; ++k) {
    for (int i = 0; i < L; ++i) {
      const bool st_k = k < N && C[k * L + i], st_p = k > 0 && C[(k - 1) * L + i];
      int s = k;
      if (st_k || st_p) {
        s = st_k ? k : k - 1;
        while (s > 0 && C[(s - 1) * L + i]) --s;
      }
      const double ts = (double)s * a.dt;
      const double cx = __builtin_fma(ts, vdx, x0v[0]), cy = __builtin_fma(ts, vdy, x0v[1]);
      double* p = FT + ((size_t)k * L + i) * 3;
      p[0] = (cx + nom[i & 3][0]) + urange(-0.03, 0.03, U[14 + 2 * (i & 3)]);
      p[1] = (cy + nom[i & 3][1]) + urange(-0.03, 0.03, U[15 + 2 * (i & 3)]);
      p[2] = 0.0;
      if (k == 0) {
        p[0] += urange(-0.01, 0.01, U[24 + 2 * (i & 3)]);
        p[1] += urange(-0.01, 0.01, U[25 + 2 * (i & 3)]);
      }
    }
  }
}

int launch_generate(const cmpc_model& m, uint64_t seed, int64_t qp_offset, int B, int gait, double* x0, double* xref,
                    double* foot, uint8_t* contact, hipStream_t stream) {
  if (B <= 0) return 0;
  GenArgs a{m.N, m.n_legs, m.dt, seed, qp_offset, gait, x0, xref, foot, contact};
  hipLaunchKernelGGL(k_generate, dim3((B + 255) / 256), dim3(256), 0, stream, a, B);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ------------------------------------------------------------------------------------------ expand / rollout
// Scatter the condensed solution back to u[N][L][3] (zeros for swing legs, as the reference's 0 <= F f <= 0 rows
// force, CentroidalMPC.cpp:199) and roll the SRBD model forward (X = Aqp x0 + Bqp U) for the optional x output.

template <typename T>
__device__ void expand_one(const ExpandArgs& a, int q) {
  const DevModel* M = a.model;
  const int N = M->N, L = NL, ld = a.ld;
  const int tid = threadIdx.x;
  const int st = a.status[q];
  const int n = st == CMPC_TOO_LARGE || st == CMPC_INVALID_CONTACT ? 0 : a.nvar[q];
  const T* uw = reinterpret_cast<const T*>(a.u_ws) + (size_t)q * ld;
  double* uo = a.u + (size_t)q * N * NU;
  double* dqo = a.dq ? a.dq + (size_t)q * N * NU : nullptr;
  for (int i = tid; i < N * NU; i += blockDim.x) {
    uo[i] = 0.0;
    if (dqo) dqo[i] = 0.0;
  }
  __syncthreads();
  for (int t = tid; t < n / 3; t += blockDim.x) {
    const int kl = a.tri_map[(size_t)q * (ld / 3) + t];
    double* dst = kl < N * L ? uo + kl * 3 : dqo + (kl - N * L) * 3;  // foothold triples only with a.dq
    for (int d = 0; d < 3; ++d) dst[d] = (double)uw[3 * t + d];
  }
  if (tid == 0) {
    a.status_out[q] = st;
    if (a.iters_out) a.iters_out[q] = (st == CMPC_TOO_LARGE || st == CMPC_INVALID_CONTACT) ? 0 : a.iters_ws[q];
  }
  if (a.x == nullptr) return;
  __syncthreads();
  if (tid != 0) return;
  const double* xr = a.xref + (size_t)q * (N + 1) * NX;
  const double* ft = a.foot + (size_t)q * (N + 1) * L * 3;
  const uint8_t* ct = a.contact + (size_t)q * N * L;
  double* xo = a.x + (size_t)q * (N + 1) * NX;
  double x[NX];
  for (int s = 0; s < NX; ++s) xo[s] = x[s] = a.x0[(size_t)q * NX + s];
  for (int k = 0; k < N; ++k) {
    const double dt = M->dt;
    double xn[NX];
    for (int s = 0; s < 3; ++s) xn[s] = x[s] + dt * x[3 + s];
    for (int s = 3; s < 9; ++s) xn[s] = x[s];
    xn[5] += dt * x[12];
    double sp, cp;
    sincos(xr[k * NX + 11], &sp, &cp);
    const double RzT[9] = {cp, sp, 0.0, -sp, cp, 0.0, 0.0, 0.0, 1.0};
    for (int r = 0; r < 3; ++r) {
      double acc = 0.0;
      for (int c = 0; c < 3; ++c) {
        double mrc = 0.0;
        for (int t = 0; t < 3; ++t) mrc += M->inv_inertia[r * 3 + t] * RzT[t * 3 + c];
        acc += dt * mrc * x[6 + c];
      }
      xn[9 + r] = x[9 + r] + acc;
    }
    xn[12] = x[12];
    for (int i = 0; i < L; ++i) {
      if (!ct[k * L + i]) continue;
      const double* f = uo + (k * L + i) * 3;
      double p[3];
      stance_point(ft, ct, N, k, i, p);
      const double rx = p[0] - xr[k * NX + 0], ry = p[1] - xr[k * NX + 1], rz = p[2] - xr[k * NX + 2];
      for (int d = 0; d < 3; ++d) xn[3 + d] += M->dt_over_m * f[d];
      xn[6] += dt * (ry * f[2] - rz * f[1]);
      xn[7] += dt * (rz * f[0] - rx * f[2]);
      xn[8] += dt * (rx * f[1] - ry * f[0]);
    }
    for (int s = 0; s < NX; ++s) xo[(k + 1) * NX + s] = x[s] = xn[s];
  }
}

__global__ __launch_bounds__(64) void k_expand(ExpandArgs a) {
  const int q = blockIdx.x;
  if (a.precision == CMPC_F64) expand_one<double>(a, q);
  else expand_one<float>(a, q);
}

int launch_expand(const ExpandArgs& a, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(k_expand, dim3(B), dim3(64), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ------------------------------------------------------------------------------------------ size-class lists
// One workgroup of 16 waves walks the batch in 1024-QP tiles: per class a wave ballot gives each QP its rank inside
// the wave, wave totals through LDS give the tile offsets, so every list is in ascending QP order (deterministic).
__global__ __launch_bounds__(1024) void k_class_lists(const int* status, const int* nvar, int B, int by_status,
                                                      int n_mid, int* lists, int* counts) {
  __shared__ int s_wtot[4][16];
  __shared__ int s_base[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int ncls = n_mid > 64 ? 4 : 3;
  if (tid < 4) s_base[tid] = 0;
  // the next tile's hints are requested before this tile's scans, so the loads overlap the barriers
  int nv_next = tid < B ? nvar[tid] : 0;
  int st_next = (by_status && tid < B) ? status[tid] : CMPC_SUCCESS;
  __syncthreads();
  for (int q0 = 0; q0 < B; q0 += 1024) {
    const int q = q0 + tid;
    const int nv = nv_next, stv = st_next;
    if (q + 1024 < B) {
      nv_next = nvar[q + 1024];
      if (by_status) st_next = status[q + 1024];
    }
    int cls = -1;
    if (q < B && stv == CMPC_SUCCESS && (by_status || nv > 0)) {
      cls = nv <= 64 ? 0 : (nv <= 128 ? 1 : 2);
      if (cls == 1 && nv <= n_mid) cls = 3;
    }
    int pre = 0;
    const unsigned long long below = (1ull << lane) - 1ull;
    for (int c = 0; c < ncls; ++c) {
      const unsigned long long mask = __ballot(cls == c);
      if (cls == c) pre = __popcll(mask & below);
      if (lane == 0) s_wtot[c][w] = __popcll(mask);
    }
    __syncthreads();
    if (cls >= 0) {
      int off = s_base[cls];
      for (int v = 0; v < w; ++v) off += s_wtot[cls][v];
      lists[(size_t)cls * B + off + pre] = q;
    }
    __syncthreads();
    if (tid < ncls) {
      int t = 0;
      for (int v = 0; v < 16; ++v) t += s_wtot[tid][v];
      s_base[tid] += t;
    }
    __syncthreads();
  }
  if (tid < ncls) counts[tid < 3 ? tid : 9] = s_base[tid];
}

int launch_class_lists(const int* status, const int* nvar, int B, int by_status, int* lists, int* counts,
                       hipStream_t stream, int n_mid) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(k_class_lists, dim3(1), dim3(1024), 0, stream, status, nvar, B, by_status, n_mid, lists, counts);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ------------------------------------------------------------------------------------------ solver statistics
// cmpc_get_residuals: the IPM kernels' final residuals, NaN for QPs they did not run (status 5 / 6 or unset)
__global__ void k_residuals(const double* res, const int* status, int B, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 4 * B) return;
  const int st = status[i / 4];
  // CMPC_STATUS_SKIPPED: a converged SQP's QP, whose residuals are those of its last IPM run
  out[i] = ((st >= CMPC_SUCCESS && st <= CMPC_NAN_SOL) || st == CMPC_STATUS_SKIPPED) ? res[i] : __builtin_nan("");
}
int launch_residuals(const double* res_ws, const int* status, int B, double* out, hipStream_t stream) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(k_residuals, dim3((4 * B + 255) / 256), dim3(256), 0, stream, res_ws, status, B, out);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ------------------------------------------------------------------------------------------ conversions
__global__ void k_f32_to_f64(const float* in, double* out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = (double)in[i];
}
__global__ void k_f64_to_f32(const double* in, float* out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = (float)in[i];
}
static unsigned grid_for(size_t n) {
  size_t b = (n + 255) / 256;
  return (unsigned)(b > 4096 ? 4096 : (b == 0 ? 1 : b));
}
int launch_convert_f32_to_f64(const float* in, double* out, size_t n, hipStream_t stream) {
  hipLaunchKernelGGL(k_f32_to_f64, dim3(grid_for(n)), dim3(256), 0, stream, in, out, n);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
int launch_convert_f64_to_f32(const double* in, float* out, size_t n, hipStream_t stream) {
  hipLaunchKernelGGL(k_f64_to_f32, dim3(grid_for(n)), dim3(256), 0, stream, in, out, n);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}


}  // namespace cmpc

namespace cmpc {

// ------------------------------------------------------------------------------------------ test-hook layouts
template <typename T>
__global__ __launch_bounds__(256) void k_unpack_qp(const T* H_ws, const T* g_ws, const int* nvar, int ld, double* H,
                                                   double* g) {
  const int q = blockIdx.x;
  const int n = nvar[q];
  const int np = ipm_class(n);
  const T* hq = H_ws + (size_t)q * ld * ld;
  double* ho = H + (size_t)q * ld * ld;
  for (int e = threadIdx.x; e < ld * ld; e += blockDim.x) {
    const int r = e / ld, c = e % ld;
    // the padding rows / columns n.. are the identity (not stored for k_ipm72's QPs, CondenseArgs::h72)
    ho[e] = (r < n && c < n) ? (double)hq[h_index_sym(np, r, c)] : (r == c ? 1.0 : 0.0);
  }
  for (int i = threadIdx.x; i < ld; i += blockDim.x) g[(size_t)q * ld + i] = i < np ? (double)g_ws[(size_t)q * ld + i] : 0.0;
}

int launch_unpack_qp(const void* H_ws, const void* g_ws, const int* nvar, int precision, int ld, double* H, double* g,
                     int B, hipStream_t stream) {
  if (B <= 0) return 0;
  if (precision == CMPC_F64)
    hipLaunchKernelGGL(k_unpack_qp<double>, dim3(B), dim3(256), 0, stream, (const double*)H_ws, (const double*)g_ws,
                       nvar, ld, H, g);
  else
    hipLaunchKernelGGL(k_unpack_qp<float>, dim3(B), dim3(256), 0, stream, (const float*)H_ws, (const float*)g_ws, nvar,
                       ld, H, g);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

template <typename T>
__global__ __launch_bounds__(256) void k_pack_qp(const double* H, const double* g, const double* tri_mu,
                                                 const double* tri_lo, const double* tri_hi, const int* nvar_in, int ld,
                                                 T* H_ws, T* g_ws, T* mu_ws, T* lo_ws, T* hi_ws, int* nvar_ws,
                                                 int* status_ws) {
  const int q = blockIdx.x;
  const int n = nvar_in[q];
  const bool ok = n >= 0 && n <= ld && n <= CMPC_IPM_MAX_N && n % 3 == 0;
  const int np = ipm_class(n);
  const int nt = ld / 3;
  if (ok) {
    for (int e = threadIdx.x; e < np * np; e += blockDim.x) {
      const int r = e / np, c = e % np;
      T v;
      if (r < n && c < n) v = (T)H[(size_t)q * ld * ld + (size_t)r * ld + c];
      else v = r == c ? T(1) : T(0);
      H_ws[(size_t)q * ld * ld + h_index(np, r, c)] = v;
    }
    for (int i = threadIdx.x; i < ld; i += blockDim.x) g_ws[(size_t)q * ld + i] = i < n ? (T)g[(size_t)q * ld + i] : T(0);
    for (int t = threadIdx.x; t < nt; t += blockDim.x) {
      mu_ws[(size_t)q * nt + t] = (T)tri_mu[(size_t)q * nt + t];
      for (int r = 0; r < 5; ++r) {
        lo_ws[((size_t)q * nt + t) * 5 + r] = (T)tri_lo[((size_t)q * nt + t) * 5 + r];
        hi_ws[((size_t)q * nt + t) * 5 + r] = (T)tri_hi[((size_t)q * nt + t) * 5 + r];
      }
    }
  }
  if (threadIdx.x == 0) {
    nvar_ws[q] = ok ? n : 0;
    status_ws[q] = ok ? CMPC_SUCCESS : CMPC_TOO_LARGE;
  }
}

int launch_pack_qp(const double* H, const double* g, const double* tri_mu, const double* tri_lo, const double* tri_hi,
                   const int* nvar_in, int precision, int ld, void* H_ws, void* g_ws, void* mu_ws, void* lo_ws,
                   void* hi_ws, int* nvar_ws, int* status_ws, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  if (precision == CMPC_F64)
    hipLaunchKernelGGL(k_pack_qp<double>, dim3(B), dim3(256), 0, stream, H, g, tri_mu, tri_lo, tri_hi, nvar_in, ld,
                       (double*)H_ws, (double*)g_ws, (double*)mu_ws, (double*)lo_ws, (double*)hi_ws, nvar_ws,
                       status_ws);
  else
    hipLaunchKernelGGL(k_pack_qp<float>, dim3(B), dim3(256), 0, stream, H, g, tri_mu, tri_lo, tri_hi, nvar_in, ld,
                       (float*)H_ws, (float*)g_ws, (float*)mu_ws, (float*)lo_ws, (float*)hi_ws, nvar_ws, status_ws);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace cmpc

namespace cmpc {

// ------------------------------------------------------------------------------------------------ warm start
// Previous solution u_init [B][N][L][3] -> condensed order of each QP (the stance triples listed by tri_map), the
// initial point of the IPM when hpipm_interface::Settings::warm_start != 0 (HpipmInterfaceSettings.h:54). One
// thread per condensed variable slot; QPs rejected by the condensing (status != SUCCESS) are left alone.
template <typename T>
__global__ __launch_bounds__(256) void k_pack_warm(const double* u_init, const int* tri_map, const int* nvar,
                                                   const int* status, int ld, int N, T* u_ws, int B,
                                                   const double* d_init) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)B * ld) return;
  const int q = (int)(e / ld), i = (int)(e % ld);
  if (status[q] != CMPC_SUCCESS) return;
  const int n = nvar[q];
  T v = T(0);
  if (i < n) {
    const int km = tri_map[(size_t)q * (ld / 3) + i / 3];  // k * L + leg (N L + s L + leg: foothold)
    v = km < N * NL ? (T)u_init[(size_t)q * N * NU + (size_t)km * 3 + i % 3]
                    : (T)d_init[(size_t)q * N * NU + (size_t)(km - N * NL) * 3 + i % 3];
  }
  u_ws[e] = v;
}

int launch_pack_warm(const double* u_init, const int* tri_map, const int* nvar, const int* status, int precision,
                     int ld, int N, void* u_ws, int B, hipStream_t stream, const double* d_init) {
  if (B <= 0) return 0;
  const long total = (long)B * ld;
  const dim3 grid((unsigned)((total + 255) / 256));
  if (precision == CMPC_F64)
    hipLaunchKernelGGL((k_pack_warm<double>), grid, dim3(256), 0, stream, u_init, tri_map, nvar, status, ld, N,
                       (double*)u_ws, B, d_init);
  else
    hipLaunchKernelGGL((k_pack_warm<float>), grid, dim3(256), 0, stream, u_init, tri_map, nvar, status, ld, N,
                       (float*)u_ws, B, d_init);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Receding-horizon shift (the role of MultipleShootingSolver::initializeStateInputTrajectories,
// MultipleShootingSolver.cpp:220-266, for a fixed grid): out[q][k] = in[q][min(k + shift, N - 1)].
__global__ __launch_bounds__(256) void k_shift_inputs(const double* in, int N, int shift, double* out, int B) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)B * N * NU) return;
  const int q = (int)(e / (N * NU)), r = (int)(e % (N * NU));
  const int k = r / NU, j = r % NU;
  const int ks = k + shift < N ? k + shift : N - 1;
  out[e] = in[(size_t)q * N * NU + (size_t)ks * NU + j];
}

int launch_shift_inputs(const double* in, int N, int shift, double* out, int B, hipStream_t stream) {
  if (B <= 0) return 0;
  const long total = (long)B * N * NU;
  hipLaunchKernelGGL(k_shift_inputs, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, in, N, shift, out, B);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace cmpc
