// ocp_chain.hpp — latency form of the OCP Riccati factorisation (the HpipmInterface::solve path's only serial chain,
// reference HpipmInterface.cpp:282-284 -> HPIPM's backward Riccati recursion; restated by oracle/ocp_ipm.c:ocp_factor)
// for small batches: k_ocp_ipm<64, 1, true>. Included inside k_ocp.hip's anonymous namespace (uses NT, View,
// lds_barrier, OCP_STAMP).
//
// Per stage k (backward), with Paug = [P p; p' 0] of node k + 1 in LDS:
//   T = Paug [B A rb; 0 0 1]                            (nx + 1) x n1, 2 x 2 register blocks per thread
//   M = Hc_k + [B A rb; 0 0 1]' T + Gc' Sigma Gc        lower triangle only, 2 x 2 blocks (one to three per thread)
//   symmetric sweep (Gauss-Jordan on the lower triangle) of the nu_k input pivots, two per workgroup barrier: the
//   pivot pair's row / column of M is published after the previous round's update, every thread forms the pair's
//   2 x 2 pivot block and updates its blocks itself. After the sweep the lower triangle holds
//   [. ; -K' ; -kff' | P_k ; p_k'] (the x / rhs rows of the input columns are -M_xu M_uu^-1, the trailing block the
//   Schur complement), and the pivot columns at their pivot's round are the LDL' factor of
//   M_uu = R~ + B'PB + D'Sigma D (kept for the corrector's feedforward and HPIPM's ric_Lr).
// Hc_k = [R + reg I, S'; S, Q + reg I] (the constant part of the stage Hessian) is laid out once per solve in the
// chain's register-block order (hp_build), so a stage's prefetch is two 16-byte loads per block; A_k, B_k, rb_k, the
// rows C_k, D_k and their Sigma are loaded straight from the record / workspace one stage ahead into registers and
// written into the other half of a double-buffered LDS image at the end of the stage. The stage descriptors
// (dimensions, offsets) sit in an LDS table. No global load and no scalar load sits on the chain: every barrier inside
// it is an LDS-only barrier, so the prefetch stays in flight across the rounds. The number of register blocks per
// thread is uniform per stage (1..3 by n1) and compiled per count, so no LDS load sits behind a divergent branch.
// The other factorisation (factor_pass: a Gauss-Jordan sweep over the full 4 x 4-cyclic register tile, the stage's
// data addressed by pointer selects on the chain) stays for the batched instantiations.
#pragma once

constexpr int CH_GS = 66;    // row stride (doubles) of the G and T images (16-byte aligned rows)
constexpr int CH_PS = 28;    // row stride of Paug
constexpr int CH_NRP = 28;   // G image rows of [B A rb] / [0 0 1] (np1 = nx + 1 <= 28); the rows' block follows
constexpr int CH_MAXT = 3;   // 2 x 2 lower blocks per thread (n1 <= 64: at most 528 blocks)
constexpr int CH_MAXG = 16;  // rows per node of the fast path
constexpr int CH_MAXN = 512; // stages of the fast path (LDS descriptor table)
constexpr int CH_DESC = 8;   // ints per stage descriptor
typedef double d2v __attribute__((ext_vector_type(2)));

// 2 x 2 block tau of the lower triangle in row order: tau = bi (bi + 1) / 2 + bj, bj <= bi
__device__ __forceinline__ void ch_block(int tau, int& bi, int& bj) {
  int b = (int)((sqrtf(8.0f * (float)tau + 1.0f) - 1.0f) * 0.5f);
  while ((b + 1) * (b + 2) / 2 <= tau) ++b;
  while (b * (b + 1) / 2 > tau) --b;
  bi = b;
  bj = tau - b * (b + 1) / 2;
}

struct ChainLds {
  double *G0, *G1, *T, *Pa, *C, *sg0, *sg1;
  int* desc;  // [N][CH_DESC]: nu, ng, cu, cr, cHp, record offset of A, constraint-record offset of C, nt
};

// Hc image of every stage (once per solve): block tau of stage k at hp[cHp[k] + 4 tau + 2 a + b] = M(2 bi + a,
// 2 bj + b) for the constant part (R + reg I | S | Q + reg I), 0 in the rhs row / column and outside n1 and above
// the diagonal. One pass over all stages' blocks with no barrier.
__device__ __forceinline__ void hp_build(const View& V, double* hp, double reg) {
  const OcpLayout& L = V.L;
  const int nx = L.nx, N = L.N;
  const int tot = L.cHp[N];
  int k = 0;
  for (int e = threadIdx.x; e < tot; e += NT) {
    while (e >= L.cHp[k + 1]) ++k;
    const int le = e - L.cHp[k], tau = le >> 2, a = (le >> 1) & 1, b = le & 1;
    int bi, bj;
    ch_block(tau, bi, bj);
    const int i = 2 * bi + a, l = 2 * bj + b;
    const int mk = L.nu[k], nz = mk + nx;
    double v = 0.0;
    if (i >= l && i < nz && l < nz) {
      if (i < mk) v = V.R(k)[l * mk + i] + (i == l ? reg : 0.0);
      else if (l < mk) v = V.S(k)[(i - mk) * mk + l];
      else v = V.Q(k)[(l - mk) * nx + (i - mk)] + (i == l ? reg : 0.0);
    }
    hp[e] = v;
  }
}

// One stage's operands in registers (the prefetch of the next stage in the chain)
struct ChainRegs {
  double gv[8];              // [B A rb] image: row tid & 31, columns (tid >> 5) + 8 q
  double cv[4];              // rows' [D C] image: row tid & 15, columns (tid >> 4) + 16 q
  double sv;                 // Sigma of row tid (tid < ng)
  double hc[CH_MAXT][2][2];  // Hc blocks
  double gr[CH_MAXT][2];     // rhs-row entries (g_u, g_x) of a block in row nz
};

__device__ __forceinline__ void chain_fetch(const View& V, const int* d, int k, const int (&bi)[CH_MAXT],
                                            const int (&bj)[CH_MAXT], const double* hp, ChainRegs& R) {
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, nx = L.nx;
  const int mk = d[0], g = d[1], cu = d[2], cr = d[3], chp = d[4], nt = d[7];
  const int nz = mk + nx, n1 = nz + 1;
  const double* A = V.rec + d[5];
  const double* B = A + nx * nx;
  const double* rb = V.rb() + (long long)k * nx;
  {
    const int r = tid & 31, c0 = tid >> 5;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = c0 + 8 * q;
      const double* p = c < mk ? B + c * nx + r : (c < nz ? A + (c - mk) * nx + r : rb + r);
      R.gv[q] = (r < nx && c < n1) ? *p : 0.0;
    }
  }
  {
    const int r = tid & 15, c0 = tid >> 4;
    const double* C = V.crec ? V.crec + d[6] : rb;
    const double* D = C + g * nx;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c0 + 16 * q;
      const double* p = c < mk ? D + c * g + r : C + (c - mk) * g + r;
      R.cv[q] = (r < g && c < nz) ? *p : 0.0;
    }
  }
  R.sv = tid < g ? V.row(R_SIG)[cr + tid] : 0.0;
  const double* hk = hp + chp;
  const double* gu = V.gu() + cu;
  const double* gx = V.gx() + (long long)k * nx;
#pragma unroll
  for (int r = 0; r < CH_MAXT; ++r) {
    const int tau = tid + NT * r;
    const bool act = tau < nt;
    const d2v* h = (const d2v*)(hk + 4 * (act ? tau : 0));
    const d2v h0 = h[0], h1 = h[1];
    R.hc[r][0][0] = act ? h0.x : 0.0;
    R.hc[r][0][1] = act ? h0.y : 0.0;
    R.hc[r][1][0] = act ? h1.x : 0.0;
    R.hc[r][1][1] = act ? h1.y : 0.0;
    // the block holding row nz carries g there (the rhs column of the stage Hessian)
    const int arow = nz - 2 * bi[r];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int l = 2 * bj[r] + b;
      const bool on = act && (arow == 0 || arow == 1) && l < nz;
      const double* p = l < mk ? gu + l : gx + (l - mk);
      R.gr[r][b] = on ? *p : 0.0;
    }
  }
}

// Registers of a stage into the LDS image G (rows 0..nx-1 = [B A rb], row nx = e_nz, rows CH_NRP.. = [D C 0]) and sg;
// columns up to the even width w >= n1 (the odd pad column is zero)
__device__ __forceinline__ void chain_commit(const View& V, const int* d, const ChainRegs& R, double* G, double* sg) {
  const int tid = threadIdx.x, nx = V.L.nx;
  const int mk = d[0], g = d[1], nz = mk + nx, n1 = nz + 1, w = (n1 + 1) & ~1;
  {
    const int r = tid & 31, c0 = tid >> 5;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = c0 + 8 * q;
      if (r < nx && c < w) G[r * CH_GS + c] = R.gv[q];
    }
  }
  if (tid < w) G[nx * CH_GS + tid] = tid == nz ? 1.0 : 0.0;
  {
    const int r = tid & 15, c0 = tid >> 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c0 + 16 * q;
      if (r < g && c < w) G[(CH_NRP + r) * CH_GS + c] = R.cv[q];
    }
  }
  if (tid < g) sg[tid] = R.sv;
}

// Per-stage part after T for NS register blocks per thread: M, the symmetric sweep, the outputs. Returns the NaN flag.
template <int NS>
__device__ __forceinline__ bool chain_stage(const View& V, const ChainLds& S, int k, const int* d, const double* G,
                                            const double* sg, const int (&bi)[CH_MAXT], const int (&bj)[CH_MAXT],
                                            const ChainRegs& cur) {
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, nx = L.nx, np1 = nx + 1;
  const int mk = d[0], g = d[1], nt = d[7], nz = mk + nx, n1 = nz + 1;
  bool bad = false;
  double m[NS][2][2];
#pragma unroll
  for (int r = 0; r < NS; ++r)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) m[r][a][b] = cur.hc[r][a][b] + ((2 * bi[r] + a == nz) ? cur.gr[r][b] : 0.0);
  // --- M = Hc + G' T + Gc' Sigma Gc ---
#pragma unroll 5
  for (int s = 0; s < np1; ++s) {
    const double* gr = G + s * CH_GS;
    const double* tr = S.T + s * CH_GS;
#pragma unroll
    for (int r = 0; r < NS; ++r) {
      const d2v gv = *(const d2v*)(gr + 2 * bi[r]);
      const d2v tv = *(const d2v*)(tr + 2 * bj[r]);
      m[r][0][0] = fma(gv.x, tv.x, m[r][0][0]);
      m[r][0][1] = fma(gv.x, tv.y, m[r][0][1]);
      m[r][1][0] = fma(gv.y, tv.x, m[r][1][0]);
      m[r][1][1] = fma(gv.y, tv.y, m[r][1][1]);
    }
  }
  for (int s = 0; s < g; ++s) {
    const double sgs = sg[s];
    const double* gr = G + (CH_NRP + s) * CH_GS;
#pragma unroll
    for (int r = 0; r < NS; ++r) {
      const d2v gv = *(const d2v*)(gr + 2 * bi[r]);
      const d2v hv = *(const d2v*)(gr + 2 * bj[r]);
      const double u0 = sgs * hv.x, u1 = sgs * hv.y;
      m[r][0][0] = fma(gv.x, u0, m[r][0][0]);
      m[r][0][1] = fma(gv.x, u1, m[r][0][1]);
      m[r][1][0] = fma(gv.y, u0, m[r][1][0]);
      m[r][1][1] = fma(gv.y, u1, m[r][1][1]);
    }
  }
  OCP_STAMP(22);
  // --- symmetric sweep of the nu_k input pivots, two per round ---
  // publish(q): the pivot pair (2q, 2q + 1)'s row / column of M into the round's buffers c0 = M(., 2q),
  // c1 = M(., 2q + 1) (lower storage: rows below from block column q, columns left from block row q)
  auto publish = [&](int q, double* c0) {
    double* c1 = c0 + 64;
#pragma unroll
    for (int r = 0; r < NS; ++r) {
      if (tid + NT * r < nt) {
        if (bj[r] == q) {
#pragma unroll
          for (int a = 0; a < 2; ++a) {
            c0[2 * bi[r] + a] = m[r][a][0];
            if (bi[r] > q || a == 1) c1[2 * bi[r] + a] = m[r][a][1];
          }
        }
        if (bi[r] == q) {
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            if (bj[r] < q || b == 0) c0[2 * bj[r] + b] = m[r][0][b];
            c1[2 * bj[r] + b] = m[r][1][b];
          }
        }
      }
    }
  };
  if (mk > 0) {
    publish(0, S.C);
    lds_barrier();
    double* Lf = V.Lf(k);
    const int npair = (mk + 1) >> 1;
    for (int p = 0; p < npair; ++p) {
      const int j = 2 * p, j1 = j + 1;
      const bool two = j1 < mk;
      const double* c0 = S.C + (p & 1) * 128;
      const double* c1 = c0 + 64;
      const double d0 = c0[j], a1 = c0[j1], e1 = c1[j1];
      bad = bad || (d0 != d0);
      const double d0i = d0 > 1e-200 ? 1.0 / d0 : 0.0;
      const double l1 = a1 * d0i;
      const double d1 = fma(-a1, l1, e1);
      double d1i = 0.0;
      if (two) {
        bad = bad || (d1 != d1);
        d1i = d1 > 1e-200 ? 1.0 / d1 : 0.0;
      }
      // the LDL' factor of M_uu: pivot column j (rows j..), column j + 1 after pivot j (rows j + 1..)
      if (tid >= j && tid < mk) {
        Lf[j * mk + tid] = c0[tid];
        if (two && tid >= j1) Lf[j1 * mk + tid] = fma(-c0[tid], l1, c1[tid]);
      }
#pragma unroll
      for (int r = 0; r < NS; ++r) {
        const int i0 = 2 * bi[r], l0 = 2 * bj[r];
        const d2v ci0 = *(const d2v*)(c0 + i0), ci1 = *(const d2v*)(c1 + i0);
        const d2v cl0 = *(const d2v*)(c0 + l0), cl1 = *(const d2v*)(c1 + l0);
        // per index x: at = sweep-j vector (-1 at j), c1p = M'(x, j + 1), bt = sweep-(j + 1) vector (-1 at j + 1)
        double at[4], bt[4];
        const int xs[4] = {i0, i0 + 1, l0, l0 + 1};
        const double c0x[4] = {ci0.x, ci0.y, cl0.x, cl0.y}, c1x[4] = {ci1.x, ci1.y, cl1.x, cl1.y};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          at[t] = xs[t] == j ? -1.0 : c0x[t];
          const double c1p = fma(-at[t], l1, xs[t] == j ? 0.0 : c1x[t]);
          bt[t] = xs[t] == j1 ? -1.0 : c1p;
        }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int i = i0 + a, l = l0 + b;
            const double b1 = (i == j || l == j) ? 0.0 : m[r][a][b];
            double v = fma(-at[a] * d0i, at[2 + b], b1);
            if (two) {
              const double b2 = (i == j1 || l == j1) ? 0.0 : v;
              v = fma(-bt[a] * d1i, bt[2 + b], b2);
            }
            m[r][a][b] = v;
          }
      }
      if (p + 1 < npair) {
        publish(p + 1, S.C + ((p + 1) & 1) * 128);
        lds_barrier();
      }
    }
  }
  OCP_STAMP(23);
  // --- outputs: K_k = -(x rows of the input columns)', kff_k, P_k / p_k (global and Paug) ---
  {
    double* Kk = V.K(k);
    double* kf = V.kf() + d[2];
    double* Pk = V.P(k);
    double* pk = V.pv() + (long long)k * nx;
#pragma unroll
    for (int r = 0; r < NS; ++r) {
      if (!(tid + NT * r < nt)) continue;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int i = 2 * bi[r] + a, l = 2 * bj[r] + b;
          if (i < l || i >= n1 || i < mk) continue;
          const double v = m[r][a][b];
          const int I = i - mk;
          if (l < mk) {
            if (I < nx) Kk[I * mk + l] = -v;
            else kf[l] = -v;
          } else {
            const int J = l - mk;
            if (I < nx) {
              Pk[J * nx + I] = v;
              Pk[I * nx + J] = v;
              S.Pa[I * CH_PS + J] = v;
              S.Pa[J * CH_PS + I] = v;
            } else if (J < nx) {
              pk[J] = v;
              S.Pa[nx * CH_PS + J] = v;
              S.Pa[J * CH_PS + nx] = v;
            } else {
              S.Pa[nx * CH_PS + nx] = 0.0;
            }
          }
        }
    }
  }
  return bad;
}

// Backward factorisation of the barrier-weighted Newton matrix, latency form. Writes P_k, pv_k (k = 0..N), K_k, kf_k,
// and the LDL' columns Lf_k (k = 0..N-1), as factor_pass. Returns false on a NaN pivot.
__device__ __forceinline__ bool chain_factor(const View& V, const ChainLds& S, const double* hp, double reg) {
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, N = L.N, nx = L.nx, np1 = nx + 1;
  int bi[CH_MAXT], bj[CH_MAXT];
#pragma unroll
  for (int r = 0; r < CH_MAXT; ++r) ch_block(tid + NT * r, bi[r], bj[r]);
  bool bad = false;
  // stage descriptors into LDS
  for (int k = tid; k < N; k += NT) {
    int* dk = S.desc + CH_DESC * k;
    const int mk = L.nu[k], n1 = mk + nx + 1, nb = (n1 + 1) >> 1;
    dk[0] = mk;
    dk[1] = L.ng[k];
    dk[2] = L.cu[k];
    dk[3] = L.cr[k];
    dk[4] = L.cHp[k];
    dk[5] = (int)L.orec[8 * k + 0];
    dk[6] = (int)L.ocon[4 * k + 0];
    dk[7] = nb * (nb + 1) / 2;
  }
  // terminal node: P_N = Q_N + reg I + C_N' Sigma C_N, p_N = g_x,N; Paug's padding rows / columns zero
  {
    const int g = L.ng[N];
    const double* Q = V.Q(N);
    const double* sig = V.row(R_SIG) + L.cr[N];
    const double* C = g ? V.C(N) : nullptr;
    for (int e = tid; e < CH_PS * CH_PS; e += NT) {
      const int r = e / CH_PS, c = e - r * CH_PS;
      double val = 0.0;
      if (r < nx && c < nx) {
        val = Q[c * nx + r] + (r == c ? reg : 0.0);
        for (int j = 0; j < g; ++j) val = fma(C[r * g + j] * sig[j], C[c * g + j], val);
        V.P(N)[c * nx + r] = val;
      } else if (r < nx && c == nx) {
        val = V.gx()[(long long)N * nx + r];
        V.pv()[(long long)N * nx + r] = val;
      } else if (r == nx && c < nx) {
        val = V.gx()[(long long)N * nx + c];
      }
      S.Pa[e] = val;
    }
  }
  __syncthreads();  // descriptors
  ChainRegs cur;    // stage k's Hc blocks / rhs entries (its G image is in LDS)
  chain_fetch(V, S.desc + CH_DESC * (N - 1), N - 1, bi, bj, hp, cur);
  chain_commit(V, S.desc + CH_DESC * (N - 1), cur, S.G0, S.sg0);
  __syncthreads();
  OCP_STAMP(20);
  for (int k = N - 1; k >= 0; --k) {
    const int cb = (N - 1 - k) & 1;
    const double* G = cb ? S.G1 : S.G0;
    const double* sg = cb ? S.sg1 : S.sg0;
    const int* d = S.desc + CH_DESC * k;
    const int mk = d[0], nz = mk + nx, n1 = nz + 1, nb = (n1 + 1) >> 1, nt = d[7];
    // --- prefetch of stage k - 1 (registers; committed to the other image at the end of this stage) ---
    ChainRegs nxt;
    if (k > 0) chain_fetch(V, d - CH_DESC, k - 1, bi, bj, hp, nxt);
    // --- T = Paug [B A rb; 0 0 1]: 2 x 2 blocks over rows 0..np1 (Paug's odd pad row is zero), columns < 2 nb ---
    {
      const int nrp = (np1 + 1) >> 1, items = nrp * nb;
      const int w0 = tid, w1 = tid + NT;
      const int ws0 = w0 < items ? w0 : 0, ws1 = w1 < items ? w1 : 0;
      const int rp0 = ws0 / nb, cp0 = ws0 - rp0 * nb, rp1 = ws1 / nb, cp1 = ws1 - rp1 * nb;
      const double* pa0 = S.Pa + 2 * rp0;
      const double* gc0 = G + 2 * cp0;
      double t0[4] = {0.0, 0.0, 0.0, 0.0};
      if (items > NT) {  // uniform: two items per thread
        const double* pa1 = S.Pa + 2 * rp1;
        const double* gc1 = G + 2 * cp1;
        double t1[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 5
        for (int s = 0; s < np1; ++s) {
          const d2v p0 = *(const d2v*)(pa0 + s * CH_PS), g0 = *(const d2v*)(gc0 + s * CH_GS);
          const d2v p1 = *(const d2v*)(pa1 + s * CH_PS), g1 = *(const d2v*)(gc1 + s * CH_GS);
          t0[0] = fma(p0.x, g0.x, t0[0]);
          t0[1] = fma(p0.x, g0.y, t0[1]);
          t0[2] = fma(p0.y, g0.x, t0[2]);
          t0[3] = fma(p0.y, g0.y, t0[3]);
          t1[0] = fma(p1.x, g1.x, t1[0]);
          t1[1] = fma(p1.x, g1.y, t1[1]);
          t1[2] = fma(p1.y, g1.x, t1[2]);
          t1[3] = fma(p1.y, g1.y, t1[3]);
        }
        if (w1 < items) {
          double* t = S.T + (2 * rp1) * CH_GS + 2 * cp1;
          *(d2v*)t = d2v{t1[0], t1[1]};
          *(d2v*)(t + CH_GS) = d2v{t1[2], t1[3]};
        }
      } else {
#pragma unroll 5
        for (int s = 0; s < np1; ++s) {
          const d2v p0 = *(const d2v*)(pa0 + s * CH_PS), g0 = *(const d2v*)(gc0 + s * CH_GS);
          t0[0] = fma(p0.x, g0.x, t0[0]);
          t0[1] = fma(p0.x, g0.y, t0[1]);
          t0[2] = fma(p0.y, g0.x, t0[2]);
          t0[3] = fma(p0.y, g0.y, t0[3]);
        }
      }
      if (w0 < items) {
        double* t = S.T + (2 * rp0) * CH_GS + 2 * cp0;
        *(d2v*)t = d2v{t0[0], t0[1]};
        *(d2v*)(t + CH_GS) = d2v{t0[2], t0[3]};
      }
    }
    lds_barrier();
    OCP_STAMP(21);
    const int ns = (nt + NT - 1) / NT;
    if (ns == 1) bad = chain_stage<1>(V, S, k, d, G, sg, bi, bj, cur) || bad;
    else if (ns == 2) bad = chain_stage<2>(V, S, k, d, G, sg, bi, bj, cur) || bad;
    else bad = chain_stage<3>(V, S, k, d, G, sg, bi, bj, cur) || bad;
    // --- the prefetched stage k - 1 into the other image ---
    if (k > 0) {
      chain_commit(V, d - CH_DESC, nxt, cb ? S.G0 : S.G1, cb ? S.sg0 : S.sg1);
#pragma unroll
      for (int r = 0; r < CH_MAXT; ++r)
#pragma unroll
        for (int a = 0; a < 2; ++a) {
#pragma unroll
          for (int b = 0; b < 2; ++b) cur.hc[r][a][b] = nxt.hc[r][a][b];
          cur.gr[r][a] = nxt.gr[r][a];
        }
    }
    lds_barrier();
    OCP_STAMP(24);
  }
  return __syncthreads_or(bad) == 0;
}
