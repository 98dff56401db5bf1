// ocp_chain.hpp — latency form of the OCP Riccati factorisation (the HpipmInterface::solve path's only serial chain,
// reference HpipmInterface.cpp:282-284 -> HPIPM's backward Riccati recursion; restated by oracle/ocp_ipm.c:ocp_factor)
// for small batches: k_ocp_ipm<64, 1, true> and the grid form. Included inside k_ocp.hip's anonymous namespace (uses
// NT, View, lds_barrier, OCP_STAMP).
//
// Per stage k (backward), with Paug = [P p; p' 0] of node k + 1 in LDS:
//   (A) T = Paug [B A rb; 0 0 1]                        (nx + 1) x n1, 2 x 2 blocks, all four waves
//   (B) M = Hc_k + g + [B A rb; 0 0 1]' T + Gc' Sigma Gc lower triangle, 2 x 2 blocks, all four waves, into LDS
//   (C) wave 0 alone: the LDL' elimination of the nu_k input pivots, two per round, on 4 x 4 register blocks of M: the
//       pivot pair's columns are published to LDS and read back by the same wave (LDS instructions of one wave run
//       in order, so a round needs no barrier); the trailing entries take the pair's rank-2 update
//       M -= c0 c0' / d0 + c1~ c1~' / d1 (c1~ = c1 - c0 a1 / d0), the same fma sequence as the symmetric sweep of
//       factor_pass on the entries that stay live, so P_k = the x / rhs block of the result is that sweep's. The
//       pivot columns are the LDL' factor F = L D of M_uu = R~ + B'PB + D'Sigma D (Lf, HPIPM's ric_Lr) and of its
//       x / rhs rows (stored in K / kf and turned into K_k = -L_uu^-T L_xu', kff_k by chain_gains, stage-parallel,
//       after the chain).
//       Waves 1-3 meanwhile load stage k - 1's operands (A_k-1, B_k-1, rb, the rows C, D and Sigma, the Hc image,
//       g) and write them into the LDS images: their load latency is off the chain, and wave 0 issues no global
//       load, so nothing on the chain waits on the vector-memory counter.
// Hc_k = [R + reg I, S'; S, Q + reg I] (the constant part of the stage Hessian) is laid out once per solve in the
// 2 x 2 block order of (B) (hp_build). The stage descriptors (dimensions, offsets) sit in an LDS table. Three
// barriers per stage, all LDS-only.
// The other factorisation (factor_pass: a Gauss-Jordan sweep over the full 4 x 4-cyclic register tile) stays for the
// batched instantiations.
#pragma once

constexpr int CH_GS = 66;     // row stride (doubles) of the G, T and M images (16-byte aligned rows)
constexpr int CH_PS = 28;     // row stride of Paug
constexpr int CH_NRP = 28;    // G image rows of [B A rb] / [0 0 1] (np1 = nx + 1 <= 28); the rows' block follows
constexpr int CH_MAXT = 3;    // 2 x 2 lower blocks per thread in (B) (n1 <= 64: at most 528 blocks)
constexpr int CH_MAXNT = 528; // 2 x 2 lower blocks of a stage (Hc image)
constexpr int CH_MAXG = 16;   // rows per node of the fast path
constexpr int CH_MAXN = 512;  // stages of the fast path (LDS descriptor table)
constexpr int CH_DESC = 10;   // ints per stage descriptor
constexpr int CH_MR = 60;     // rows of the M image (n1 <= OCP_CHAIN_MAX_N1)
constexpr int CH_FS = 60;     // column stride of the factor image F (rows x of the pivot column j at F[j CH_FS + x])
constexpr int CH_MAXU = 36;   // pivot columns of the factor image (nu_k <= OCP_CHAIN_MAX_NU)
// LDS from ChainLds::Ml to the descriptor table (M image, Hc image, g, the second Paug, F0): scratch of the
// partitioned factorisation's element and combine steps (ocp_part.hpp) between chains
constexpr int CH_SCRATCH = CH_MR * CH_GS + 4 * CH_MAXNT + 64 + CH_PS * CH_PS + CH_MAXU * CH_FS;
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
  double *Ml, *Hc, *gb;  // M image (CH_MR x CH_GS), the stage's Hc image (4 CH_MAXNT), g of the stage (64)
  double *Pa2, *F0, *F1;  // the other Paug; the factor images of alternate stages (F1 aliases G1: unused by the chain)
  int* desc;  // [N][CH_DESC]: nu, ng, cu, cr, cHp, record offset of A, constraint-record offset of C, nt, cM, cK
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

// Waves 1-3 (t = threadIdx.x - 64 in [0, 192)): stage k's operands into the LDS images — G (rows 0..nx-1 = [B A rb],
// row nx = e_nz, rows CH_NRP.. = the rows' [D C 0]; columns up to the even width w >= n1, the pad column zero), sg
// (Sigma of the rows), Hc (the stage's Hc image, 4 nt doubles) and gb (g_u, g_x, then zeros up to w). Every load is
// issued before the first store, so one wait covers them.
__device__ __forceinline__ void chain_out(const View& V, const int* d, int k, const double* Pb, const double* Fb, int t,
                                          int nthr);
__device__ __forceinline__ void chain_load(const View& V, const int* d, int k, const double* hp, const ChainLds& S,
                                           const int* dout, const double* Pout, const double* Fout) {
  const OcpLayout& L = V.L;
  const int t = threadIdx.x - 64, nx = L.nx;
  const int mk = d[0], g = d[1], cu = d[2], cr = d[3], chp = d[4], nt = d[7];
  const int nz = mk + nx, n1 = nz + 1, w = (n1 + 1) & ~1;
  const double* A = V.rec + d[5];
  const double* B = A + nx * nx;
  const double* rb = V.rb() + (long long)k * nx;
  // unconditional loads (an out-of-range entry reads A_k[0]; zeroed at the store): a load whose value is selected
  // against 0 at the fetch would make the compiler wait for it there, one load at a time
  double gv[11], cv[6], hv[12], sv, gg;
  {
    const int r = t & 31, c0 = t >> 5;  // [B A rb]: row r, columns c0 + 6 q
#pragma unroll
    for (int q = 0; q < 11; ++q) {
      const int c = c0 + 6 * q;
      const bool on = r < nx && c < n1;
      const double* p = c < mk ? B + c * nx + r : (c < nz ? A + (c - mk) * nx + r : rb + r);
      gv[q] = *(on ? p : A);
    }
  }
  const double* C = V.crec ? V.crec + d[6] : rb;
  {
    const int r = t & 15, c0 = t >> 4;  // rows' [D C]: row r, columns c0 + 12 q
    const double* D = C + g * nx;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const int c = c0 + 12 * q;
      const bool on = r < g && c < nz;
      const double* p = c < mk ? D + c * g + r : C + (c - mk) * g + r;
      cv[q] = *(on ? p : A);
    }
  }
  sv = *(t < g ? V.row(R_SIG) + cr + t : A);
  gg = *(t < mk ? V.gu() + cu + t : (t < nz ? V.gx() + (long long)k * nx + t - mk : A));
  {
    const d2v* h = (const d2v*)(hp + chp);
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const int e = t + 192 * q;
      const d2v v = h[e < 2 * nt ? e : 0];
      hv[2 * q] = v.x;
      hv[2 * q + 1] = v.y;
    }
  }
  // stage k + 2's outputs (the chain's stage before the current one) to global memory while the loads are in flight
  if (dout) chain_out(V, dout, k + 2, Pout, Fout, t, 192);
  double* G = S.G0;
  {
    const int r = t & 31, c0 = t >> 5;
#pragma unroll
    for (int q = 0; q < 11; ++q) {
      const int c = c0 + 6 * q;
      if (r < nx && c < w) G[r * CH_GS + c] = c < n1 ? gv[q] : 0.0;
    }
  }
  if (t < w) G[nx * CH_GS + t] = t == nz ? 1.0 : 0.0;
  {
    const int r = t & 15, c0 = t >> 4;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const int c = c0 + 12 * q;
      if (r < ((g + 3) & ~3) && c < w) G[(CH_NRP + r) * CH_GS + c] = (r < g && c < nz) ? cv[q] : 0.0;
    }
  }
  if (t < ((g + 3) & ~3)) S.sg0[t] = t < g ? sv : 0.0;
  if (t < w) S.gb[t] = t < nz ? gg : 0.0;
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const int e = t + 192 * q;
    if (e < 2 * nt) *(d2v*)(S.Hc + 2 * e) = d2v{hv[2 * q], hv[2 * q + 1]};
  }
}

// Stage k's outputs from the LDS images to global memory (threads t of nthr): P_k, p_k from its Paug image Pb, the
// factor columns from Fb — u rows into Lf_k, x rows into K_k (row x of the column-major nu_k x nx block), the rhs row
// into kf_k (chain_gains turns the last two into the gains)
__device__ __forceinline__ void chain_out(const View& V, const int* d, int k, const double* Pb, const double* Fb, int t,
                                          int nthr) {
  const OcpLayout& L = V.L;
  const int nx = L.nx, np1 = nx + 1;
  const int mk = d[0], nz = mk + nx, n1 = nz + 1;
  double* Pk = V.P(k);
  double* pk = V.pv() + (long long)k * nx;
  for (int e = t; e < nx * np1; e += nthr) {
    const int I = e / np1, J = e - I * np1;
    const double v = Pb[J * CH_PS + I];
    if (J < nx) Pk[I * nx + J] = v;
    else pk[I] = v;
  }
  double* Lf = V.ws + L.o_Lf + d[8];
  double* Kx = V.ws + L.o_K + d[9];
  double* kx = V.kf() + d[2];
  for (int e = t; e < mk * n1; e += nthr) {
    const int j = e / n1, x = e - j * n1;
    if (x < j) continue;
    const double v = Fb[j * CH_FS + x];
    if (x < mk) Lf[j * mk + x] = v;
    else if (x < nz) Kx[(x - mk) * mk + j] = v;
    else kx[j] = v;
  }
}

// (B): M = Hc + g + G' T + Gc' Sigma Gc on NS 2 x 2 lower blocks per thread, into the M image
template <int NS>
__device__ __forceinline__ void chain_m(const ChainLds& S, int nx, const int* d, const int (&bi)[CH_MAXT],
                                        const int (&bj)[CH_MAXT]) {
  const int tid = threadIdx.x, np1 = nx + 1;
  const int mk = d[0], g = d[1], nt = d[7], nz = mk + nx;
  const double* G = S.G0;
  double m[NS][2][2];
#pragma unroll
  for (int r = 0; r < NS; ++r) {
    const int tau = tid + NT * r;
    const bool act = tau < nt;
    const d2v* h = (const d2v*)(S.Hc + 4 * (act ? tau : 0));
    const d2v h0 = h[0], h1 = h[1];
    const d2v gr = *(const d2v*)(S.gb + (act ? 2 * bj[r] : 0));
    m[r][0][0] = h0.x + (2 * bi[r] == nz ? gr.x : 0.0);
    m[r][0][1] = h0.y + (2 * bi[r] == nz ? gr.y : 0.0);
    m[r][1][0] = h1.x + (2 * bi[r] + 1 == nz ? gr.x : 0.0);
    m[r][1][1] = h1.y + (2 * bi[r] + 1 == nz ? gr.y : 0.0);
  }
  // groups of four rows, every load of a group issued before its fmas (the image's rows np1 .. np1 rounded up to 4
  // are zero, so are the rows' block's rows g .. g rounded up to 4 and their Sigma)
  const int np1r = (np1 + 3) & ~3, g4 = (g + 3) & ~3;
  for (int s = 0; s < np1r; s += 4) {
    d2v gv[4][NS], tv[4][NS];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int r = 0; r < NS; ++r) {
        gv[u][r] = *(const d2v*)(G + (s + u) * CH_GS + 2 * bi[r]);
        tv[u][r] = *(const d2v*)(S.T + (s + u) * CH_GS + 2 * bj[r]);
      }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int r = 0; r < NS; ++r) {
        m[r][0][0] = fma(gv[u][r].x, tv[u][r].x, m[r][0][0]);
        m[r][0][1] = fma(gv[u][r].x, tv[u][r].y, m[r][0][1]);
        m[r][1][0] = fma(gv[u][r].y, tv[u][r].x, m[r][1][0]);
        m[r][1][1] = fma(gv[u][r].y, tv[u][r].y, m[r][1][1]);
      }
  }
  for (int s = 0; s < g4; s += 4) {
    d2v gv[4][NS], hv[4][NS];
    double sgs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      sgs[u] = S.sg0[s + u];
#pragma unroll
      for (int r = 0; r < NS; ++r) {
        gv[u][r] = *(const d2v*)(G + (CH_NRP + s + u) * CH_GS + 2 * bi[r]);
        hv[u][r] = *(const d2v*)(G + (CH_NRP + s + u) * CH_GS + 2 * bj[r]);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int r = 0; r < NS; ++r) {
        const double u0 = sgs[u] * hv[u][r].x, u1 = sgs[u] * hv[u][r].y;
        m[r][0][0] = fma(gv[u][r].x, u0, m[r][0][0]);
        m[r][0][1] = fma(gv[u][r].x, u1, m[r][0][1]);
        m[r][1][0] = fma(gv[u][r].y, u0, m[r][1][0]);
        m[r][1][1] = fma(gv[u][r].y, u1, m[r][1][1]);
      }
  }
#pragma unroll
  for (int r = 0; r < NS; ++r) {
    if (tid + NT * r < nt) {
      double* o = S.Ml + (2 * bi[r]) * CH_GS + 2 * bj[r];
      *(d2v*)o = d2v{m[r][0][0], m[r][0][1]};
      *(d2v*)(o + CH_GS) = d2v{m[r][1][0], m[r][1][1]};
    }
  }
}

// One pair round of (C): pivots j, j + 1 (j = 4 jb + A0). Publishes the pair's columns (rows >= 4 jb, from the
// blocks of block column jb; the column offset A0 in the block is a template argument, so the publish needs no
// select), stores the factor's columns, and applies the rank-2 update to every entry (entries in processed rows /
// columns are dead: never read again). A missing second pivot (odd nu_k) has 1 / d1 = 0, which leaves the update's
// second term exactly 0.
template <int NB, int A0, bool WEAK>
__device__ __forceinline__ void chain_round(double (&m)[NB][4][4], const int (&bi)[NB], const int (&bj)[NB],
                                            const bool (&on)[NB], int j, int mk, int n1, double* c0, double* c1,
                                            double* F, bool& bad, bool& weak) {
  const int lane = threadIdx.x, j1 = j + 1, jb = j >> 2;
  const bool two = j1 < mk;
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    if (on[q] && bj[q] == jb) {
      double* o0 = c0 + 4 * bi[q];
      double* o1 = c1 + 4 * bi[q];
      *(d2v*)o0 = d2v{m[q][0][A0], m[q][1][A0]};
      *(d2v*)(o0 + 2) = d2v{m[q][2][A0], m[q][3][A0]};
      *(d2v*)o1 = d2v{m[q][0][A0 + 1], m[q][1][A0 + 1]};
      *(d2v*)(o1 + 2) = d2v{m[q][2][A0 + 1], m[q][3][A0 + 1]};
    }
  }
  __builtin_amdgcn_wave_barrier();
  const double d0 = c0[j], a1 = c0[j1], e1 = c1[j1];
  bad = bad || (d0 != d0);
  const double d0i = d0 > 1e-200 ? 1.0 / d0 : 0.0;
  const double l1 = a1 * d0i;
  const double d1 = fma(-a1, l1, e1);
  bad = bad || (two && d1 != d1);
  const double d1i = (two && d1 > 1e-200) ? 1.0 / d1 : 0.0;
  if (WEAK) weak = weak || !(d0 > 1e-200) || (two && !(d1 > 1e-200));
  // the factor's columns into the F image (rows >= j; chain_out reads column j + 1 from row j + 1)
  if (lane >= j && lane < n1) {
    const double v0 = c0[lane];
    F[j * CH_FS + lane] = v0;
    if (two) F[j1 * CH_FS + lane] = fma(-v0, l1, c1[lane]);
  }
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const d2v ri0 = *(const d2v*)(c0 + 4 * bi[q]), ri1 = *(const d2v*)(c0 + 4 * bi[q] + 2);
    const d2v si0 = *(const d2v*)(c1 + 4 * bi[q]), si1 = *(const d2v*)(c1 + 4 * bi[q] + 2);
    const d2v rl0 = *(const d2v*)(c0 + 4 * bj[q]), rl1 = *(const d2v*)(c0 + 4 * bj[q] + 2);
    const d2v sl0 = *(const d2v*)(c1 + 4 * bj[q]), sl1 = *(const d2v*)(c1 + 4 * bj[q] + 2);
    const double ci[4] = {ri0.x, ri0.y, ri1.x, ri1.y}, cl[4] = {rl0.x, rl0.y, rl1.x, rl1.y};
    const double ei[4] = {si0.x, si0.y, si1.x, si1.y}, el[4] = {sl0.x, sl0.y, sl1.x, sl1.y};
    double ui[4], vi[4], bl[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      ui[t] = -ci[t] * d0i;
      vi[t] = -fma(-ci[t], l1, ei[t]) * d1i;
      bl[t] = fma(-cl[t], l1, el[t]);
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) m[q][a][b] = fma(vi[a], bl[b], fma(ui[a], cl[b], m[q][a][b]));
  }
  __builtin_amdgcn_wave_barrier();
}

// A quad round of (C): pivots j .. j + 3 (j = 4 jb) in one publish — the whole block column jb — computing exactly
// what the two pair rounds (j, j + 1) and (j + 2, j + 3) compute: every lane forms the second pair's columns for its
// own rows and columns from the published pre-round values with the owners' fma sequence, and applies the two rank-2
// updates in the same order, so the results are bit-identical with half the publish / read-back latency chains.
template <int NB, bool WEAK>
__device__ __forceinline__ void chain_round4(double (&m)[NB][4][4], const int (&bi)[NB], const int (&bj)[NB],
                                             const bool (&on)[NB], int j, int n1, double* cb, double* F, bool& bad,
                                             bool& weak) {
  const int lane = threadIdx.x, jb = j >> 2;
  double* c0 = cb;
  double* c1 = cb + 64;
  double* c2 = cb + 128;
  double* c3 = cb + 192;
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    if (on[q] && bj[q] == jb) {
      const int o = 4 * bi[q];
      *(d2v*)(c0 + o) = d2v{m[q][0][0], m[q][1][0]};
      *(d2v*)(c0 + o + 2) = d2v{m[q][2][0], m[q][3][0]};
      *(d2v*)(c1 + o) = d2v{m[q][0][1], m[q][1][1]};
      *(d2v*)(c1 + o + 2) = d2v{m[q][2][1], m[q][3][1]};
      *(d2v*)(c2 + o) = d2v{m[q][0][2], m[q][1][2]};
      *(d2v*)(c2 + o + 2) = d2v{m[q][2][2], m[q][3][2]};
      *(d2v*)(c3 + o) = d2v{m[q][0][3], m[q][1][3]};
      *(d2v*)(c3 + o + 2) = d2v{m[q][2][3], m[q][3][3]};
    }
  }
  __builtin_amdgcn_wave_barrier();
  // the pivot block (rows j .. j + 3 of the four columns)
  const d2v q0a = *(const d2v*)(c0 + j), q0b = *(const d2v*)(c0 + j + 2);
  const d2v q1b = *(const d2v*)(c1 + j), q1c = *(const d2v*)(c1 + j + 2);
  const d2v q2b = *(const d2v*)(c2 + j + 2), q3b = *(const d2v*)(c3 + j + 2);
  // first pair, as chain_round
  const double d0 = q0a.x, a1 = q0a.y, e1 = q1b.y;
  bad = bad || (d0 != d0);
  const double d0i = d0 > 1e-200 ? 1.0 / d0 : 0.0;
  const double l1 = a1 * d0i;
  const double d1 = fma(-a1, l1, e1);
  bad = bad || (d1 != d1);
  const double d1i = d1 > 1e-200 ? 1.0 / d1 : 0.0;
  // the first pair's row / column vectors at index y (published pre-round values c0_y, c1_y)
  auto u_of = [&](double x0) { return -x0 * d0i; };
  auto p_of = [&](double x0, double x1) { return fma(-x0, l1, x1); };
  // pivots j + 2, j + 3 after the first pair's update (entries (j+2, j+2), (j+3, j+2), (j+3, j+3))
  const double cl2 = q0b.x, cl3 = q0b.y;                       // c0 at j + 2, j + 3
  const double bl2 = p_of(q0b.x, q1c.x), bl3 = p_of(q0b.y, q1c.y);  // c1~ at j + 2, j + 3
  const double u2 = u_of(q0b.x), u3 = u_of(q0b.y);
  const double v2 = -bl2 * d1i, v3 = -bl3 * d1i;
  const double e2 = fma(v2, bl2, fma(u2, cl2, q2b.x));  // M'(j+2, j+2)
  const double a3 = fma(v3, bl2, fma(u3, cl2, q2b.y));  // M'(j+3, j+2)
  const double e3 = fma(v3, bl3, fma(u3, cl3, q3b.y));  // M'(j+3, j+3)
  bad = bad || (e2 != e2);
  const double d2i = e2 > 1e-200 ? 1.0 / e2 : 0.0;
  const double l3 = a3 * d2i;
  const double d3 = fma(-a3, l3, e3);
  bad = bad || (d3 != d3);
  const double d3i = d3 > 1e-200 ? 1.0 / d3 : 0.0;
  if (WEAK) weak = weak || !(d0 > 1e-200) || !(d1 > 1e-200) || !(e2 > 1e-200) || !(d3 > 1e-200);
  // the factor's columns j .. j + 3 (rows >= j): c0, c1~, the updated column j + 2 and its c~ for j + 3
  if (lane >= j && lane < n1) {
    const double x0 = c0[lane], x1 = c1[lane], x2 = c2[lane], x3 = c3[lane];
    const double u = u_of(x0), pp = p_of(x0, x1), v = -pp * d1i;
    const double y2 = fma(v, bl2, fma(u, cl2, x2)), y3 = fma(v, bl3, fma(u, cl3, x3));
    F[j * CH_FS + lane] = x0;
    F[(j + 1) * CH_FS + lane] = pp;
    F[(j + 2) * CH_FS + lane] = y2;
    F[(j + 3) * CH_FS + lane] = fma(-y2, l3, y3);
  }
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    double x0[8], x1[8], x2[8], x3[8];
    {
      const int oi = 4 * bi[q], ol = 4 * bj[q];
      const d2v r0a = *(const d2v*)(c0 + oi), r0b = *(const d2v*)(c0 + oi + 2);
      const d2v r1a = *(const d2v*)(c1 + oi), r1b = *(const d2v*)(c1 + oi + 2);
      const d2v r2a = *(const d2v*)(c2 + oi), r2b = *(const d2v*)(c2 + oi + 2);
      const d2v r3a = *(const d2v*)(c3 + oi), r3b = *(const d2v*)(c3 + oi + 2);
      const d2v s0a = *(const d2v*)(c0 + ol), s0b = *(const d2v*)(c0 + ol + 2);
      const d2v s1a = *(const d2v*)(c1 + ol), s1b = *(const d2v*)(c1 + ol + 2);
      const d2v s2a = *(const d2v*)(c2 + ol), s2b = *(const d2v*)(c2 + ol + 2);
      const d2v s3a = *(const d2v*)(c3 + ol), s3b = *(const d2v*)(c3 + ol + 2);
      const double t0[8] = {r0a.x, r0a.y, r0b.x, r0b.y, s0a.x, s0a.y, s0b.x, s0b.y};
      const double t1[8] = {r1a.x, r1a.y, r1b.x, r1b.y, s1a.x, s1a.y, s1b.x, s1b.y};
      const double t2[8] = {r2a.x, r2a.y, r2b.x, r2b.y, s2a.x, s2a.y, s2b.x, s2b.y};
      const double t3[8] = {r3a.x, r3a.y, r3b.x, r3b.y, s3a.x, s3a.y, s3b.x, s3b.y};
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        x0[t] = t0[t];
        x1[t] = t1[t];
        x2[t] = t2[t];
        x3[t] = t3[t];
      }
    }
    // first pair: u (rows), c0 (columns), v (rows), c1~ (columns); second pair from the updated columns 2, 3
    double ui[4], cl[4], vi[4], bl[4], ui2[4], cl2v[4], vi2[4], bl2v[4];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const double u = u_of(x0[t]), pp = p_of(x0[t], x1[t]), v = -pp * d1i;
      const double y2 = fma(v, bl2, fma(u, cl2, x2[t])), y3 = fma(v, bl3, fma(u, cl3, x3[t]));
      const double pp2 = fma(-y2, l3, y3);
      if (t < 4) {
        ui[t] = u;
        vi[t] = v;
        ui2[t] = -y2 * d2i;
        vi2[t] = -pp2 * d3i;
      } else {
        cl[t - 4] = x0[t];
        bl[t - 4] = pp;
        cl2v[t - 4] = y2;
        bl2v[t - 4] = pp2;
      }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const double w = fma(vi[a], bl[b], fma(ui[a], cl[b], m[q][a][b]));
        m[q][a][b] = fma(vi2[a], bl2v[b], fma(ui2[a], cl2v[b], w));
      }
  }
  __builtin_amdgcn_wave_barrier();
}

// (C) on wave 0: NB 4 x 4 lower blocks of M per lane (block beta = lane + 64 q), the pair rounds, the outputs.
// Returns the pivots' flags: CH_NAN (a NaN pivot), CH_WEAK (a pivot the guard dropped, d <= 1e-200).
constexpr int CH_NAN = 1, CH_WEAK = 2;
template <int NB, bool WEAK>
__device__ __forceinline__ int chain_elim(const View& V, const ChainLds& S, int mk, double* F, double* PaW, int nxo = -1) {
  const OcpLayout& L = V.L;
  const int lane = threadIdx.x, nx = nxo >= 0 ? nxo : L.nx;  // nxo: the trailing block's size when not nx
  const int nz = mk + nx, n1 = nz + 1, nb4 = (n1 + 3) >> 2, nt4 = nb4 * (nb4 + 1) / 2;
  bool bad = false, weak = false;
  int bi[NB], bj[NB];
  bool on[NB];
  double m[NB][4][4];
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const int beta = lane + 64 * q;
    on[q] = beta < nt4;
    ch_block(on[q] ? beta : 0, bi[q], bj[q]);
    const double* src = S.Ml + (4 * bi[q]) * CH_GS + 4 * bj[q];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const d2v v0 = *(const d2v*)(src + a * CH_GS), v1 = *(const d2v*)(src + a * CH_GS + 2);
      m[q][a][0] = v0.x;
      m[q][a][1] = v0.y;
      m[q][a][2] = v1.x;
      m[q][a][3] = v1.y;
    }
    if (bi[q] == bj[q]) {  // the image holds the lower triangle: the diagonal block's upper part by symmetry
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = a + 1; b < 4; ++b) m[q][a][b] = m[q][b][a];
    }
  }
  double* c0 = S.C;
  double* c1 = S.C + 64;
  OCP_STAMP(27);
  for (int j = 0; j < mk; j += 4) {
    if (j + 4 <= mk) {
      chain_round4<NB, WEAK>(m, bi, bj, on, j, n1, S.C, F, bad, weak);
    } else {
      chain_round<NB, 0, WEAK>(m, bi, bj, on, j, mk, n1, c0, c1, F, bad, weak);
      if (j + 2 < mk) chain_round<NB, 2, WEAK>(m, bi, bj, on, j + 2, mk, n1, c0, c1, F, bad, weak);
    }
  }
  OCP_STAMP(23);
  // --- Paug of node k straight from the registers: the live entries (rows / columns >= nu_k, lower triangle of the
  // blocks) and their mirror into PaW (global P_k, p_k: chain_out on the helper waves, a stage later); the other
  // entries' stores go to a dummy slot, so the stores need no branch ---
  if ((mk & 1) == 0 && ((n1 + 3) & ~3) - mk <= CH_PS) {
    // nu_k even: every live pair of columns of a block is a 16-byte piece of a Paug row; each block writes its live
    // rows and, mirrored, its live columns in such pieces (diagonal blocks from their lower triangle, so Paug stays
    // exactly symmetric); the entries past n1 are written as zeros (Paug's pad rows / columns stay zero)
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      if (!on[q] || 4 * bj[q] + 4 <= mk) continue;
      const int I0 = 4 * bi[q] - mk, J0 = 4 * bj[q] - mk;
      const bool diag = bi[q] == bj[q];
      double w[4][4];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const double v = (diag && a < b) ? m[q][b][a] : m[q][a][b];
          const int I = I0 + a, J = J0 + b;
          w[a][b] = (I > nx || J > nx || (I == nx && J == nx)) ? 0.0 : v;
        }
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        if (I0 + a < 0) continue;
        if (J0 >= 0) *(d2v*)(PaW + (I0 + a) * CH_PS + J0) = d2v{w[a][0], w[a][1]};
        *(d2v*)(PaW + (I0 + a) * CH_PS + J0 + 2) = d2v{w[a][2], w[a][3]};
      }
      if (!diag) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          if (J0 + b < 0) continue;
          if (I0 >= 0) *(d2v*)(PaW + (J0 + b) * CH_PS + I0) = d2v{w[0][b], w[1][b]};
          *(d2v*)(PaW + (J0 + b) * CH_PS + I0 + 2) = d2v{w[2][b], w[3][b]};
        }
      }
    }
    return (bad ? CH_NAN : 0) | (weak ? CH_WEAK : 0);
  }
  double* dummy = S.C + 128 + lane;  // one slot per lane: a shared one would serialise the masked lanes' stores
#pragma unroll
  for (int q = 0; q < NB; ++q)
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int i = 4 * bi[q] + a, l = 4 * bj[q] + b;
        const bool live = on[q] && i >= l && l >= mk && i < n1;
        const int I = i - mk, J = l - mk;
        const double v = (I == nx && J == nx) ? 0.0 : m[q][a][b];
        *(live ? PaW + I * CH_PS + J : dummy) = v;
        *(live ? PaW + J * CH_PS + I : dummy) = v;
      }
  return (bad ? CH_NAN : 0) | (weak ? CH_WEAK : 0);
}

// K_k = -L_uu^-T L_xu', kff_k = -L_uu^-T l_r' for stages [k0, k1) from the LDL' factor F = L D the chain left (u rows
// in Lf, x / rhs rows in K / kf): thread per (stage, column); a guarded pivot (d <= 1e-200) has a zero column
__device__ __forceinline__ void chain_gains(const View& V, int k0, int k1) {
  const OcpLayout& L = V.L;
  const int nx = L.nx, np1 = nx + 1;
  for (int e = threadIdx.x; e < (k1 - k0) * np1; e += NT) {
    const int k = k0 + e / np1, c = e - (e / np1) * np1;
    const int mk = L.nu[k];
    if (mk == 0) continue;
    const double* F = V.Lf(k);
    double* x = c < nx ? V.K(k) + c * mk : V.kf() + L.cu[k];
    for (int a = mk - 1; a >= 0; --a) {
      const double da = F[a * mk + a];
      const double dai = da > 1e-200 ? 1.0 / da : 0.0;
      double s = x[a];
      for (int b = a + 1; b < mk; ++b) s = fma(F[a * mk + b], x[b], s);
      x[a] = -(s * dai);
    }
  }
}

// Backward factorisation of the barrier-weighted Newton matrix, latency form, over the stages [k0, k1) from the value
// function of node k1 given by term:
//   CH_TERM_NODE  node k1 = N: P_N = Q_N + reg I + C_N' Sigma C_N, p_N = g_x,N (written to P(N), pv(N));
//   CH_TERM_ZERO  V_k1 = 0 (a segment of the partitioned factorisation, ocp_part.hpp: its first pass);
//   CH_TERM_GIVEN V_k1(x) = x'Pt x / 2 + pt'x (Pt column-major nx x nx, pt [nx]; the partitioned form's second pass).
// Writes P_k, pv_k (k = k0..k1-1), the LDL' columns Lf_k and the factor's x / rhs rows (chain_gains turns them into
// K_k, kf_k). Returns the pivots' flags of all four waves (CH_NAN, CH_WEAK), workgroup-uniform.
// PART = false: the serial chain (k0 = 0, k1 = N, CH_TERM_NODE; no guarded-pivot flag), the form the solve's own loop
// inlines; PART = true: any range and end value (ocp_part.hpp, compiled in its own function).
constexpr int CH_TERM_NODE = 0, CH_TERM_ZERO = 1, CH_TERM_GIVEN = 2;
template <bool PART>
__device__ __forceinline__ int chain_factor(const View& V, const ChainLds& S, const double* hp, double reg, int k0,
                                            int k1, int term, const double* Pt, const double* pt) {
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, N = L.N, nx = L.nx, np1 = nx + 1;
  const int wave = tid >> 6;
  int bi[CH_MAXT], bj[CH_MAXT];
#pragma unroll
  for (int r = 0; r < CH_MAXT; ++r) ch_block(tid + NT * r, bi[r], bj[r]);
  int flags = 0;
  // stage descriptors into LDS
  for (int k = k0 + tid; k < k1; k += NT) {
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
    dk[8] = L.cM[k];
    dk[9] = L.cK[k];
  }
  // the value function of node k1 into Paug; Paug's padding rows / columns zero
  if (term == CH_TERM_NODE) {  // terminal node: P_N = Q_N + reg I + C_N' Sigma C_N, p_N = g_x,N
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
      S.Pa2[e] = 0.0;
    }
  } else {
    for (int e = tid; e < CH_PS * CH_PS; e += NT) {
      const int r = e / CH_PS, c = e - r * CH_PS;
      double val = 0.0;
      if (term == CH_TERM_GIVEN) {
        if (r < nx && c < nx) val = Pt[c * nx + r];
        else if (r < nx && c == nx) val = pt[r];
        else if (r == nx && c < nx) val = pt[c];
      }
      S.Pa[e] = val;
      S.Pa2[e] = 0.0;
    }
  }
  // the image's rows and T's rows np1 .. CH_NRP stay zero (the T and M loops run over rows in groups of four)
  for (int e = tid; e < (CH_NRP - np1) * CH_GS; e += NT) {
    S.G0[np1 * CH_GS + e] = 0.0;
    S.T[np1 * CH_GS + e] = 0.0;
  }
  __syncthreads();  // descriptors
  if (wave > 0) chain_load(V, S.desc + CH_DESC * (k1 - 1), k1 - 1, hp, S, nullptr, nullptr, nullptr);
  __syncthreads();
  OCP_STAMP(20);
  for (int k = k1 - 1; k >= k0; --k) {
    const int* d = S.desc + CH_DESC * k;
    const int mk = d[0], nz = mk + nx, n1 = nz + 1, nb = (n1 + 1) >> 1, nt = d[7];
    const int pb = (k1 - 1 - k) & 1;
    const double* PaR = pb ? S.Pa2 : S.Pa;  // Paug of node k + 1
    double* PaW = pb ? S.Pa : S.Pa2;        // Paug of node k
    double* Fw = (k & 1) ? S.F1 : S.F0;     // the factor image of stage k (stage k + 1's is the other)
    // --- (A) T = Paug [B A rb; 0 0 1]: 2 x 2 blocks over rows 0..np1 (Paug's odd pad row is zero), columns < 2 nb ---
    {
      const double* G = S.G0;
      const int nrp = (np1 + 1) >> 1, items = nrp * nb;
      const int w0 = tid, w1 = tid + NT;
      const int ws0 = w0 < items ? w0 : 0, ws1 = w1 < items ? w1 : 0;
      const int rp0 = ws0 / nb, cp0 = ws0 - rp0 * nb, rp1 = ws1 / nb, cp1 = ws1 - rp1 * nb;
      const double* pa0 = PaR + 2 * rp0;
      const double* gc0 = G + 2 * cp0;
      double t0[4] = {0.0, 0.0, 0.0, 0.0};
      const int np1r = (np1 + 3) & ~3;  // Paug's pad columns and the image's rows up to np1r are zero
      if (items > NT) {  // uniform: two items per thread
        const double* pa1 = PaR + 2 * rp1;
        const double* gc1 = G + 2 * cp1;
        double t1[4] = {0.0, 0.0, 0.0, 0.0};
        for (int s = 0; s < np1r; s += 4) {
          d2v p0[4], g0[4], p1[4], g1[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            p0[u] = *(const d2v*)(pa0 + (s + u) * CH_PS);
            g0[u] = *(const d2v*)(gc0 + (s + u) * CH_GS);
            p1[u] = *(const d2v*)(pa1 + (s + u) * CH_PS);
            g1[u] = *(const d2v*)(gc1 + (s + u) * CH_GS);
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            t0[0] = fma(p0[u].x, g0[u].x, t0[0]);
            t0[1] = fma(p0[u].x, g0[u].y, t0[1]);
            t0[2] = fma(p0[u].y, g0[u].x, t0[2]);
            t0[3] = fma(p0[u].y, g0[u].y, t0[3]);
            t1[0] = fma(p1[u].x, g1[u].x, t1[0]);
            t1[1] = fma(p1[u].x, g1[u].y, t1[1]);
            t1[2] = fma(p1[u].y, g1[u].x, t1[2]);
            t1[3] = fma(p1[u].y, g1[u].y, t1[3]);
          }
        }
        if (w1 < items) {
          double* t = S.T + (2 * rp1) * CH_GS + 2 * cp1;
          *(d2v*)t = d2v{t1[0], t1[1]};
          *(d2v*)(t + CH_GS) = d2v{t1[2], t1[3]};
        }
      } else {
        for (int s = 0; s < np1r; s += 4) {
          d2v p0[4], g0[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            p0[u] = *(const d2v*)(pa0 + (s + u) * CH_PS);
            g0[u] = *(const d2v*)(gc0 + (s + u) * CH_GS);
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            t0[0] = fma(p0[u].x, g0[u].x, t0[0]);
            t0[1] = fma(p0[u].x, g0[u].y, t0[1]);
            t0[2] = fma(p0[u].y, g0[u].x, t0[2]);
            t0[3] = fma(p0[u].y, g0[u].y, t0[3]);
          }
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
    // --- (B) M into the image ---
    const int ns = (nt + NT - 1) / NT;
    if (ns == 1) chain_m<1>(S, nx, d, bi, bj);
    else if (ns == 2) chain_m<2>(S, nx, d, bi, bj);
    else chain_m<3>(S, nx, d, bi, bj);
    lds_barrier();
    OCP_STAMP(22);
    // --- (C) wave 0: the elimination and the outputs; waves 1-3: stage k - 1's operands ---
    if (wave == 0) {
      const int nb4 = (n1 + 3) >> 2, nt4 = nb4 * (nb4 + 1) / 2;
      if (nt4 <= 64) flags |= chain_elim<1, PART>(V, S, d[0], Fw, PaW);
      else flags |= chain_elim<2, PART>(V, S, d[0], Fw, PaW);  // nt4 <= 120: n1 <= 60 (OCP_CHAIN_MAX_N1, ocp_chain_lds_bytes)
      OCP_STAMP(25);
    } else if (k > k0) {
      OCP_SPAN_BEGIN(t_load);
      // stage k - 1's operands; stage k + 1's outputs (its Paug and factor images, untouched in this stage)
      const bool out = k + 1 < k1;
      chain_load(V, d - CH_DESC, k - 1, hp, S, out ? d + CH_DESC : nullptr, PaR, (k & 1) ? S.F0 : S.F1);
      OCP_SPAN_END(26, t_load, 64);
    }
    lds_barrier();
    OCP_STAMP(24);
  }
  // the outputs of stages k0 + 1 (if not yet written: a one-stage range has none) and k0
  if (k1 - k0 > 1)
    chain_out(V, S.desc + CH_DESC * (k0 + 1), k0 + 1, ((k1 - k0) & 1) ? S.Pa : S.Pa2, ((k0 + 1) & 1) ? S.F1 : S.F0,
              tid, NT);
  chain_out(V, S.desc + CH_DESC * k0, k0, ((k1 - k0) & 1) ? S.Pa2 : S.Pa, (k0 & 1) ? S.F1 : S.F0, tid, NT);
  const int fl = (__syncthreads_or(flags & CH_NAN) ? CH_NAN : 0) | (__syncthreads_or(flags & CH_WEAK) ? CH_WEAK : 0);
  __syncthreads();  // every wave's global stores (chain_out) visible to the workgroup
  return fl;
}

// The whole horizon from the terminal node (the serial chain); returns false on a NaN pivot
__device__ __forceinline__ bool chain_factor(const View& V, const ChainLds& S, const double* hp, double reg) {
  return (chain_factor<false>(V, S, hp, reg, 0, V.L.N, CH_TERM_NODE, nullptr, nullptr) & CH_NAN) == 0;
}

// The Newton step's serial affine recursions on wave 0, their operands staged in LDS a chunk of stages ahead by waves
// 1-3 (the factorisation's images are free then):
//   BWD = false (forward rollout):       dx_1 = bcl_0, dx_{k+1} = Acl_k dx_k + bcl_k           (k = 1 .. N-1)
//   BWD = true  (corrector's cost-to-go): v_N = g_x,N, p_k = Acl_k' v_{k+1} + h_k, v_k = p_k    (k = N-1 .. 1)
// Each stage's slot holds the matrix in the order wave 0 reads it (lane r, column c at [c nx + r]: Acl_k as stored,
// or transposed for BWD) and the vector. Wave 0 keeps the running vector in LDS (v0 / v1, read back by the same wave:
// no barrier per stage); one workgroup barrier per chunk. The fma order per entry is the one of forward_pass /
// bwd_vec_b.
// The steps s = s0 .. s1 - 1 of the sequence (k = 1 + s forward, N - 1 - s backward; s1 < 0: to the end): s0 = 0 starts
// from the recursion's own initial value, s0 > 0 from the output row before step s0 (dx_{1 + s0} / p_{N - s0}, written
// by the caller); keep_last leaves the last step's output row alone (the partitioned scan's boundary value, owned by the
// caller: affine_grid).
template <bool BWD>
__device__ __forceinline__ void chain_affine(const View& V, const ChainLds& C, double* v0, double* v1, int s0 = 0,
                                             int s1 = -1, bool keep_last = false) {
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, nx = L.nx, N = L.N, nxx = nx * nx, wave = tid >> 6;
  const int SS = (nxx + nx + 1) & ~1;
  const int region = (int)((C.F0 + CH_MAXU * CH_FS) - C.Ml);
  int CK = region / (2 * SS);
  if (CK > 24 * 192 / SS) CK = 24 * 192 / SS;
  if (CK > 16) CK = 16;
  double* buf0 = C.Ml;
  double* buf1 = C.Ml + CK * SS;
  const int n = (s1 < 0 ? N - 1 : s1) - s0;  // steps of this range
  const double* vec = BWD ? V.h() : V.bcl();
  // waves 1-3: chunk c (steps s0 + c CK .. s0 + c CK + cnt - 1 of the sequence) into its buffer; all loads before any
  // store
  auto load = [&](int c) {
    const int t = tid - 64, j0 = c * CK;
    const int cnt = (n - j0) < CK ? (n - j0) : CK;
    const int tot = cnt * SS;
    double* dst = (c & 1) ? buf1 : buf0;
    double r[24];
    int idx[24];
    int j = 0, w = t;
    while (w >= SS) {
      w -= SS;
      ++j;
    }
#pragma unroll
    for (int q = 0; q < 24; ++q) {
      const int e = t + 192 * q;
      const bool on = e < tot;
      const int k = BWD ? N - 1 - (s0 + j0 + j) : 1 + s0 + j0 + j;
      const double* src = V.ws;  // an always valid address for the entries outside the chunk
      if (on) {
        if (w < nxx) {
          if (BWD) {
            const int cc = w / nx, rr = w - cc * nx;  // slot [cc nx + rr] = Acl_k(cc, rr) = stored [rr nx + cc]
            src = V.Acl(k) + rr * nx + cc;
          } else {
            src = V.Acl(k) + w;
          }
        } else if (w < nxx + nx) {
          src = vec + (long long)k * nx + (w - nxx);
        }
      }
      r[q] = *src;
      idx[q] = on ? j * SS + w : -1;
      w += 192;
      while (w >= SS) {
        w -= SS;
        ++j;
      }
    }
#pragma unroll
    for (int q = 0; q < 24; ++q)
      if (idx[q] >= 0) dst[idx[q]] = r[q];
  };
  if (wave == 0 && tid < nx) {
    double d;
    if (s0 == 0) {
      d = BWD ? V.gx()[(long long)N * nx + tid] : V.bcl()[tid];
      if (!BWD) V.dx()[nx + tid] = d;
    } else {
      d = BWD ? V.pv()[(long long)(N - s0) * nx + tid] : V.dx()[(long long)(1 + s0) * nx + tid];
    }
    v0[tid] = d;
  }
  if (wave > 0 && n > 0) load(0);
  __syncthreads();
  double* out = BWD ? V.pv() : V.dx();
  for (int c = 0, s = 0; c * CK < n; ++c) {
    if (wave == 0) {
      const double* b = (c & 1) ? buf1 : buf0;
      const int cnt = (n - c * CK) < CK ? (n - c * CK) : CK;
      for (int j = 0; j < cnt; ++j, ++s) {
        const double* M = b + j * SS;
        const double* vin = (s & 1) ? v1 : v0;
        double* vout = (s & 1) ? v0 : v1;
        const int k = BWD ? N - 1 - (s0 + s) : 1 + s0 + s;
        if (tid < nx) {
          double acc = M[nxx + tid];
#pragma unroll 8
          for (int cc = 0; cc < nx; ++cc) acc = fma(M[cc * nx + tid], vin[cc], acc);
          vout[tid] = acc;
          if (!(keep_last && s == n - 1)) out[(long long)(BWD ? k : k + 1) * nx + tid] = acc;
        }
        __builtin_amdgcn_wave_barrier();
      }
    } else if ((c + 1) * CK < n) {
      load(c + 1);
    }
    lds_barrier();
  }
  __syncthreads();  // wave 0's stores of the outputs visible to the workgroup (the LDS-only barriers above do not wait)
}
