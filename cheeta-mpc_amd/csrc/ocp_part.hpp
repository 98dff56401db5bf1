// ocp_part.hpp — partitioned (parallel-in-time) form of the latency factorisation for the grid form (k_ocp_grid): the
// backward Riccati recursion of the HpipmInterface::solve path (reference HpipmInterface.cpp:282-284 -> HPIPM's
// Riccati factorisation; restated serially by oracle/ocp_ipm.c:ocp_factor) split over S horizon segments, so that the
// chain is S times shorter. Included inside k_ocp.hip's anonymous namespace after ocp_chain.hpp.
//
// Segment s holds the stages [c_s, c_{s+1}) (seg_begin: the last segment 5/2 times the others) and runs on workgroup s
// of the problem's grid.
//   P1 (all segments at once): the last segment runs the chain from the terminal node: its values are exact. Every
//      middle segment (1 <= s <= S-2) runs the chain from a zero value function at its end node b = c_{s+1} (V^0) and
//      then forms its element: with the closed loop of that pass, Acl_k = A_k + B_k K^0_k, bcl_k = rb_k + B_k kff^0_k,
//        Phi = Acl_{b-1} ... Acl_a (a = c_s),  f = sum_k Phi(b, k+1) bcl_k,
//        W = sum_k Phi(b, k+1) B_k (M^0_uu,k)^-1 B_k' Phi(b, k+1)'   (the segment's controllability Gramian),
//      accumulated backward over the segment (Phi(b, k+1) = Acl_{b-1} ... Acl_{k+1}). Any input sequence of the
//      segment is u_k = K^0_k x_k + kff^0_k + v_k, its cost V^0_a(x_a) + sum v_k' M^0_uu,k v_k / 2 and its end state
//      x_b = Phi x_a + f + sum Phi(b, k+1) B_k v_k, so for the true value function V_b(x) = x'P_b x / 2 + p_b'x the
//      minimum over v gives V_a exactly:
//        P_a = P^0_a + Phi' P_b X_Phi,   p_a = p^0_a + Phi' P_b X_f + X_Phi' p_b,   [X_Phi X_f] = (I + W P_b)^-1 [Phi f].
//      With W = Gw Gw' (its Cholesky factor, formed by the segment's workgroup) and Woodbury, the same combine reads
//        P_a = D - C' N^-1 C,  p_a = e - C' N^-1 g,  N = I + Gw' P_b Gw,  C = Gw' P_b Phi,  D = P^0_a + Phi' P_b Phi,
//        g = Gw' h,  e = p^0_a + Phi' h,  h = P_b f + p_b,
//      i.e. the Schur complement of the symmetric positive definite pivot block N (eigenvalues >= 1) in
//        M = U' P_b U + [I 0 Gw'p_b; 0 P^0_a p^0_a + Phi'p_b; . . 0],  U = [Gw Phi f]:
//      exactly the elimination a chain stage performs (chain_elim on wave 0, nx pivots, no pivoting needed).
//   P2 (workgroup 0): that combine, backward from the last segment's value at c_{S-1} down to c_1 (S - 2 steps: two
//      products and one chain_elim each): the exact value function at every boundary.
//   P3 (segments 0 .. S-2 at once): the chain again over the segment from its end node's exact value: every stage's
//      P_k, p_k, LDL' factor and gains are the factorisation of the serial chain, up to rounding.
// The serial depth is ~2 N / S chain stages plus S - 2 combines instead of N stages. A pivot the first pass's guard
// dropped (M^0_uu singular without the future's cost) or a failed combine falls back to the serial chain, so the
// guarded-pivot behaviour is always the serial one's.
#pragma once

// Segment boundaries c_s, s = 0 .. S (c_0 = 0, c_S = N): the middle segments weigh one, the last one 5/2 — in P1 it
// runs only its chain (about 13 k cycles per stage at the legged size) while the middle ones run the chain and their
// element (about 33 k) — and segment 0 one half: its second pass is the only one that waits for the last combine (the
// others run behind the combines); at least one stage per segment
__device__ __forceinline__ int seg_begin(int N, int S, int s) {
  if (s <= 0) return 0;
  if (s >= S) return N;
  int c = (int)((long long)N * (10 * s - 5) / (10 * S + 10));
  if (c < s) c = s;
  if (c > N - (S - s)) c = N - (S - s);
  return c;
}

// Per-problem segment buffer (OcpSolveArgs::seg, doubles): element s (U = [Gw Phi f], column-major nx x (2 nx + 1),
// then P^0, p^0 of its start node) at
// s * seg_esz(nx); the boundary value of node c_j (P column-major, p) at OCP_GRID_MAX_G * seg_esz(nx) + j * seg_bsz(nx)
// (seg_esz / seg_bsz: k_ocp.hpp)

// Segments of the partitioned factorisation for a grid of G workgroups (want: cmpc_ocp_set_segments, 0 = auto): at
// most G and N; auto ~ sqrt(N) without rows, sqrt(2 N) with them (two chain passes of N / S stages and the segment
// elements against S - 2 combines; with rows the three affine scans per iteration also shorten with S; measured
// optimum at the legged size: 7-8 / 12-14)
__device__ __forceinline__ int part_segments(int want, int G, int N, int m) {
  int S = want > 0 ? want : (int)(sqrtf((m > 0 ? 2.0f : 1.0f) * (float)N) + 0.5f);
  if (S > G) S = G;
  if (S > N) S = N;
  return S < 1 ? 1 : S;
}

// 2 x 2 output block (i0, j0) of sum_{t<K} A(i, t) B(t, j), A(i, t) = A[i ai + t at], B(t, j) = B[t bt + j bj] (LDS
// operands), added to c. The loads of 8 consecutive t are issued before their fmas (one LDS round trip per 8 t: these
// small products are latency-bound with one wave per SIMD). A row / column past m / n reads row / column m-1 / n-1
// (the caller does not store it); the fma order over t is fixed, so the (i, j) entry of one block and the (j, i) entry
// of the transposed product's block are the same fma chain.
__device__ __forceinline__ void blk2(const double* A, int ai, int at, const double* B, int bt, int bj, int i0, int j0,
                                     int m, int n, int K, double (&c)[2][2]) {
  const int i1 = i0 + 1 < m ? i0 + 1 : i0, j1 = j0 + 1 < n ? j0 + 1 : j0;
  for (int t0 = 0; t0 < K; t0 += 8) {
    double a0[8], a1[8], b0[8], b1[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int t = t0 + u < K ? t0 + u : K - 1;
      a0[u] = A[i0 * ai + t * at];
      a1[u] = A[i1 * ai + t * at];
      b0[u] = B[t * bt + j0 * bj];
      b1[u] = B[t * bt + j1 * bj];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (t0 + u < K) {
        c[0][0] = fma(a0[u], b0[u], c[0][0]);
        c[0][1] = fma(a0[u], b1[u], c[0][1]);
        c[1][0] = fma(a1[u], b0[u], c[1][0]);
        c[1][1] = fma(a1[u], b1[u], c[1][1]);
      }
    }
  }
}
// store a 2 x 2 block into a column-major m x n array (leading dimension ld) where it lies inside
__device__ __forceinline__ void st2(double* C, int ld, int i0, int j0, int m, int n, const double (&c)[2][2]) {
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
      if (i0 + x < m && j0 + y < n) C[(j0 + y) * ld + i0 + x] = c[x][y];
}

// One 16 x 16 tile (rows r0 .., columns c0 ..) of sum_{t<K} A(i, t) B(t, j) added to acc on v_mfma_f64_16x16x4f64 (one
// wave): A(i, t) = A[i ai + t at], B(t, j) = B[t bt + j bj] (LDS), rows >= m / columns >= n / t >= K read as zero; the
// loads of up to 7 k-steps (t < 28) issued before their mfmas. acc[q] is the entry (r0 + (lane >> 4) + 4 q,
// c0 + (lane & 15)).
__device__ __forceinline__ v4d mtile(const double* A, int ai, int at, const double* B, int bt, int bj, int r0, int c0,
                                     int m, int n, int K, v4d acc) {
  const int lane = threadIdx.x & 63, lr = lane & 15, lk = lane >> 4;
  const int i = r0 + lr, j = c0 + lr, nks = (K + 3) >> 2;
  for (int k0 = 0; k0 < nks; k0 += 7) {
    double av[7], bv[7];
#pragma unroll
    for (int kk = 0; kk < 7; ++kk) {
      const int t = 4 * (k0 + kk) + lk;
      const bool tv = k0 + kk < nks && t < K;
      av[kk] = (tv && i < m) ? A[i * ai + t * at] : 0.0;
      bv[kk] = (tv && j < n) ? B[t * bt + j * bj] : 0.0;
    }
#pragma unroll
    for (int kk = 0; kk < 7; ++kk)
      if (k0 + kk < nks) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[kk], bv[kk], acc, 0, 0, 0);
  }
  return acc;
}

// P1 of a middle segment [a, b) after its chain from V_b = 0 (workgroup-wide), from the factor the chain left (LDL'
// columns F = L D of M^0_uu,k in Lf_k, its x rows F_x and rhs row F_r in K_k / kf_k): with Yd_k = B_k L_k^-T D_k^-1
// (nx x nu_k, row-wise forward substitution; a guarded pivot's column 0),
//   Acl_k = A_k + B_k K^0_k = A_k - Yd_k F_x',  bcl_k = rb_k + B_k kff^0_k = rb_k - Yd_k F_r',
//   B_k (M^0_uu,k)^-1 B_k' = Ys_k Ys_k',  Ys_k = Yd_k D_k^1/2,
// and backward over the stages Phi <- Phi Acl_k, f += Phi bcl_k, W += Gs Gs' (Gs = Phi Ys_k). The stages go in chunks of
// up to SEG_CHUNK: a chunk's operands [A | B | rb | F | F_x | F_r] come into LDS (region B, ChainLds::Ml) in one pass of
// loads, then its Yd (one thread per (stage, row)), Acl and bcl are formed for all its stages at once (in place of A,
// B, rb), and the accumulation takes one phase per stage (Phi Acl, Phi Ys, Phi bcl and the previous stage's W update
// side by side, 2 x 2 register blocks). Phi, W, f and the Gs double buffer in region A (from ChainLds::G0). Finally
// W = Gw Gw' by chain_elim on wave 0 (nx pivots of [W 0; 0 0] with a 4-wide zero trailing block, so one 4 x 4 block
// per lane; a dropped pivot leaves a zero column). Writes U = [Gw
// Phi f] to el. Returns chain_elim's NaN flag.
constexpr int SEG_CHUNK = 9;  // stages per chunk: Yd takes one thread per (stage, row), 9 * 27 <= NT
__device__ __forceinline__ int seg_element(const View& V, const ChainLds& CS, int a, int b, double* el) {
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, nx = L.nx, nxx = nx * nx, hb = (nx + 1) >> 1;
  const int numax = L.numax > 0 ? L.numax : 1;
  const int ssz = (nxx + 2 * nx * numax + nx + numax * numax + numax + 1) & ~1;  // one stage's slot (<= 4032 doubles)
  int cmax = CH_SCRATCH / ssz;
  if (cmax > SEG_CHUNK) cmax = SEG_CHUNK;
  double* Ph0 = CS.G0;  // region A
  double* Ph1 = Ph0 + nxx;
  double* Wm = Ph1 + nxx;
  double* fv = Wm + nxx;
  double* Gs0 = fv + 32;
  double* Gs1 = Gs0 + nx * numax;
  double* Op = CS.Ml;  // region B: the chunk's stage slots
  for (int e = tid; e < nxx; e += NT) {
    const int i = e % nx, j = e / nx;
    Ph0[e] = i == j ? 1.0 : 0.0;
    Wm[e] = 0.0;
  }
  if (tid < nx) fv[tid] = 0.0;
  int cur = 0, mprev = 0;  // Phi buffer; nu of the stage whose Gs waits for its W update
  for (int ce = b; ce > a; ce -= cmax) {
    const int cb = ce - cmax > a ? ce - cmax : a, nc = ce - cb;
    OCP_SPAN_BEGIN(t_f);
    // (1) the chunk's operands: flat over the stage slots, 16 loads per thread in flight per round; each stage's six
    // source pointers and nu_k first into an LDS table (ChainLds::C, free until the Cholesky at the end), so an
    // element's address costs LDS reads instead of dependent global reads of the layout arrays
    long long* ptab = (long long*)CS.C;  // [slot][8]: A, B, rb, F (Lf), F_x (K), F_r (kf), nu_k
    if (tid < nc) {
      const int k = cb + tid;
      long long* pt = ptab + tid * 8;
      pt[0] = (long long)V.A(k);
      pt[1] = (long long)V.Bm(k);
      pt[2] = (long long)(V.rb() + (long long)k * nx);
      pt[3] = (long long)V.Lf(k);
      pt[4] = (long long)V.K(k);
      pt[5] = (long long)(V.kf() + L.cu[k]);
      pt[6] = L.nu[k];
    }
    __syncthreads();
    {
      int s0 = tid / ssz, o0 = tid - s0 * ssz;
      const int tot = nc * ssz;
      for (int base = 0; base < tot; base += 16 * NT) {
        double r[16];
        int sl[16], ol[16];
        int sx = s0, ox = o0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          sl[i] = sx;
          ol[i] = ox;
          const long long* pt = ptab + (sx < nc ? sx : nc - 1) * 8;
          const int mk = (int)pt[6];
          const int oB = nxx, oR = oB + nx * mk, oF = oR + nx, oX = oF + mk * mk, oL = oX + nx * mk, oe = oL + mk;
          const int seg = ox < oB ? 0 : ox < oR ? 1 : ox < oF ? 2 : ox < oX ? 3 : ox < oL ? 4 : 5;
          const int o = ox - (seg == 0 ? 0 : seg == 1 ? oB : seg == 2 ? oR : seg == 3 ? oF : seg == 4 ? oX : oL);
          const double* src = (const double*)pt[seg] + o;
          r[i] = (sx < nc && ox < oe) ? *src : 0.0;
          ox += NT;
          while (ox >= ssz) {
            ox -= ssz;
            ++sx;
          }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (sl[i] < nc) Op[sl[i] * ssz + ol[i]] = r[i];
        s0 = sx;
        o0 = ox;
      }
    }
    __syncthreads();
    OCP_SPANG_END(10, t_f, 1);
    OCP_SPAN_BEGIN(t_1);
    // (2) Yd of every stage of the chunk: thread (stage, row r), in place of B (8 terms per LDS round trip)
    if (tid < nc * nx) {
      const int sl = tid / nx, r = tid - sl * nx, mk = (int)ptab[sl * 8 + 6];
      double* O = Op + sl * ssz;
      double* Yd = O + nxx;
      const double* F = Yd + nx * mk + nx;
      for (int q = 0; q < mk; ++q) {
        double s2 = Yd[q * nx + r];
        for (int c0 = 0; c0 < q; c0 += 8) {
          double fq[8], yc[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int c = c0 + u < q ? c0 + u : q - 1;
            fq[u] = F[c * mk + q];
            yc[u] = Yd[c * nx + r];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (c0 + u < q) s2 = fma(-fq[u], yc[u], s2);
        }
        const double d = F[q * mk + q];
        Yd[q * nx + r] = d > 1e-200 ? s2 / d : 0.0;
      }
    }
    __syncthreads();
    OCP_SPANG_END(11, t_1, 1);
    OCP_SPAN_BEGIN(t_2);
    // (3) Acl = A - Yd F_x' in place of A, bcl = rb - Yd F_r' in place of rb (2 x 2 blocks of every stage)
    for (int w = tid; w < nc * (hb * hb + hb); w += NT) {
      const int sl = w / (hb * hb + hb), v = w - sl * (hb * hb + hb), mk = (int)ptab[sl * 8 + 6];
      double* O = Op + sl * ssz;
      const double* Yd = O + nxx;
      double* rb = O + nxx + nx * mk;
      const double* Fx = rb + nx + mk * mk;
      const double* Fr = Fx + nx * mk;
      const bool isA = v < hb * hb;
      const int i0 = isA ? 2 * (v % hb) : 2 * (v - hb * hb), j0 = isA ? 2 * (v / hb) : 0, n = isA ? nx : 1;
      double* C = isA ? O : rb;
      double c[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
      blk2(Yd, 1, nx, isA ? Fx : Fr, 1, isA ? mk : 0, i0, j0, nx, n, mk, c);
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          const int i = i0 + x < nx ? i0 + x : nx - 1, j = j0 + y < n ? j0 + y : n - 1;
          c[x][y] = C[j * nx + i] - c[x][y];
        }
      st2(C, nx, i0, j0, nx, n, c);
    }
    __syncthreads();
    OCP_SPANG_END(12, t_2, 1);
    OCP_SPAN_BEGIN(t_3);
    // (4) backward over the chunk's stages, one phase each: Phi [Acl_k Yd_k bcl_k] (one nx x (nx + nu_k + 1) product:
    // Phi Acl_k, Gs = Phi Yd_k D^1/2, f += Phi bcl_k) and the W update of the stage before (its Gs from the last phase),
    // 16 x 16 tiles on the matrix cores, tile w + 4 v on wave w
    for (int k = ce - 1; k >= cb; --k) {
      const int mk = (int)ptab[(k - cb) * 8 + 6], LX = nx + mk + 1;
      const double* X = Op + (k - cb) * ssz;  // [Acl | Yd | bcl], column-major, ld nx
      const double* F = X + nx * LX;
      const double* Ph = cur ? Ph1 : Ph0;
      double* Pn = cur ? Ph0 : Ph1;
      double* Gn = cur ? Gs1 : Gs0;
      const double* Gp = cur ? Gs0 : Gs1;
      const int nt = (nx + 15) >> 4, nP = nt * ((LX + 15) >> 4), nW = mprev > 0 ? nt * nt : 0;
      const int lane = tid & 63, lr = lane & 15, lk = lane >> 4;
      for (int w = tid >> 6; w < nP + nW; w += 4) {
        if (w < nP) {
          const int r0 = 16 * (w % nt), c0 = 16 * (w / nt), j = c0 + lr;
          const v4d acc = mtile(Ph, 1, nx, X, 1, nx, r0, c0, nx, LX, nx, v4d{0.0, 0.0, 0.0, 0.0});
          const int qd = (j >= nx && j < nx + mk) ? j - nx : 0;
          const double d = F[qd * mk + qd], sd = d > 1e-200 ? sqrt(d) : 0.0;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int i = r0 + lk + 4 * q;
            if (i < nx) {
              if (j < nx) Pn[j * nx + i] = acc[q];
              else if (j < nx + mk) Gn[(j - nx) * nx + i] = acc[q] * sd;
              else if (j == nx + mk) fv[i] += acc[q];
            }
          }
        } else {
          const int v = w - nP, r0 = 16 * (v % nt), c0 = 16 * (v / nt), j = c0 + lr;
          v4d acc;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int i = r0 + lk + 4 * q;
            acc[q] = (i < nx && j < nx) ? Wm[j * nx + i] : 0.0;
          }
          acc = mtile(Gp, 1, nx, Gp, nx, 1, r0, c0, nx, nx, mprev, acc);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int i = r0 + lk + 4 * q;
            if (i < nx && j < nx) Wm[j * nx + i] = acc[q];
          }
        }
      }
      mprev = mk;
      cur ^= 1;
      __syncthreads();
    }
    OCP_SPANG_END(13, t_3, 1);
  }
  // the last stage's W update, then M = [W 0; 0 0] (lower triangle, rows / columns up to the 4 x 4 blocks' pad)
  const double* Gp = cur ? Gs0 : Gs1;
  const int n1 = 2 * nx + 1, np = (n1 + 3) & ~3;
  if (mprev > 0) {
    const int nt = (nx + 15) >> 4, lane = tid & 63, lr = lane & 15, lk = lane >> 4;
    for (int v = tid >> 6; v < nt * nt; v += 4) {
      const int r0 = 16 * (v % nt), c0 = 16 * (v / nt), j = c0 + lr;
      v4d acc;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = r0 + lk + 4 * q;
        acc[q] = (i < nx && j < nx) ? Wm[j * nx + i] : 0.0;
      }
      acc = mtile(Gp, 1, nx, Gp, nx, 1, r0, c0, nx, nx, mprev, acc);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = r0 + lk + 4 * q;
        if (i < nx && j < nx) Wm[j * nx + i] = acc[q];
      }
    }
  }
  __syncthreads();
  for (int e = tid; e < np * np; e += NT) {
    const int i = e / np, j = e - i * np;
    CS.Ml[i * CH_GS + j] = (i < nx && j < nx) ? Wm[j * nx + i] : 0.0;
  }
  __syncthreads();
  OCP_SPAN_BEGIN(t_c);
  int fl = 0;
  if (tid < 64) fl = chain_elim<1, false>(V, CS, nx, CS.F0, CS.Pa2, 3);  // trailing block of 3 + 1 zeros: NB = 1
  fl = __syncthreads_or(fl & CH_NAN) ? CH_NAN : 0;
  OCP_SPANG_END(13, t_c, 1);
  // U = [Gw Phi f]: Gw(x, j) = F(x, j) / sqrt(d_j) below the diagonal (0 for a dropped pivot); then this pass's
  // P^0_a, p^0_a (the combine reads them here: the segment's second pass overwrites the workspace's while P2 runs)
  const double* Ph = cur ? Ph1 : Ph0;
  const double* P0 = V.P(a);
  const double* p0 = V.pv() + (long long)a * nx;
  for (int e = tid; e < 3 * nxx + 2 * nx; e += NT) {
    double v;
    if (e < nxx) {
      const int x = e % nx, j = e / nx;
      const double d = CS.F0[j * CH_FS + j];
      v = (x >= j && d > 1e-200) ? CS.F0[j * CH_FS + x] / sqrt(d) : 0.0;
    } else if (e < 2 * nxx + nx) {
      v = e < 2 * nxx ? Ph[e - nxx] : fv[e - 2 * nxx];
    } else {
      const int o = e - (2 * nxx + nx);
      v = o < nxx ? P0[o] : p0[o - nxx];
    }
    el[e] = v;
  }
  __syncthreads();
  return fl;
}

// P2 on one workgroup: the exact value function at the boundaries c_{S-1} .. c_1 into the segment buffer (the last
// segment's own P, p at c_{S-1}; then the combine per middle segment, see the header): T = P_b U (+ p_b on the f
// column: h), the M image's lower triangle T' U + [I; P^0_a; p^0_a], both as 16 x 16 tiles on the matrix cores (U and T
// kept row-major, so that each tile's loads are unit-stride across its lanes); chain_elim of its nx pivots on wave 0;
// its Paug image is [P_a p_a]. Region A holds U, T, P_b, p_b; region B the chain's M image, factor and Paug images.
// Returns false on a NaN or dropped pivot (then the serial chain runs).
// Boundary values published by P2 while P3 runs behind it (the pipelined form): workgroup 0 stores, per
// factorisation gen, gen * 64 + (S - s) into the problem's level word once boundary s is in the segment buffer
// (SEG_FAIL: a combine failed), with the grid barrier's hand-off (every thread's stores drained, one agent release);
// segment g's workgroup waits for boundary g + 1 (time-bounded like grid_sync: a timeout fails the grid).
constexpr unsigned SEG_FAIL = 63;
__device__ __forceinline__ void seg_publish(unsigned* lvl, unsigned val) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_store(lvl, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// 1: the boundary is there; 0: a combine failed; -1: the grid failed or the wait timed out (the grid fail word set)
__device__ __forceinline__ int seg_wait(unsigned* bar, unsigned* lvl, unsigned target, unsigned failv, double* flag_lds,
                                        long long limit) {
  if (threadIdx.x == 0) {
    int r = 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned v;
    while ((v = __hip_atomic_load(lvl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < target) {
      if (__hip_atomic_load(bar + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
          (long long)(__builtin_amdgcn_s_memrealtime() - t0) > limit) {
        __hip_atomic_store(bar + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        r = -1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (r == 1 && v == failv) r = 0;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    flag_lds[0] = (double)r;
  }
  __syncthreads();
  return (int)flag_lds[0];
}

constexpr double SEG_CANCEL = 1e5;  // largest max D_ii / max P_a,ii a combine may leave (about 1e-11 relative error)
__device__ __forceinline__ bool seg_combine(const View& V, const ChainLds& CS, double* sq, int S, int N, unsigned* lvl,
                                            unsigned gen) {
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, nx = L.nx, nxx = nx * nx;
  const int LU = 2 * nx + 1, np = (LU + 3) & ~3, nt = (nx + 15) >> 4, nu4 = (LU + 15) >> 4;
  const int lane = tid & 63, lr = lane & 15, lk = lane >> 4;
  const int esz = seg_esz(nx), bsz = seg_bsz(nx);
  double* bnd = sq + OCP_GRID_MAX_G * esz;
  double* Ut = CS.G0;        // U = [Gw Phi f] row-major: U(t, j) at t LU + j
  double* Tt = Ut + nx * LU; // T = P_b U (+ p_b on column 2 nx), row-major
  double* Pb = Tt + nx * LU;
  double* pb = Pb + nxx;
  double* P0s = pb + 32;  // P^0_a, p^0_a of the boundary (column-major, then the vector)
  double* Ml = CS.Ml;
  // the next combine's element and P^0 / p^0 in registers: their global loads (written by other workgroups) overlap
  // the current combine
  double rel[6], rp0[3];
  auto prefetch = [&](int s) {
    const double* el = sq + s * esz;
    const double* P0 = el + nx * LU;  // the segment's first-pass P^0, p^0 at its start node (seg_element)
    const double* p0 = P0 + nxx;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int e = tid + NT * i;
      rel[i] = e < nx * LU ? el[e] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int e = tid + NT * i;
      rp0[i] = e < nxx ? P0[e] : (e < nxx + nx ? p0[e - nxx] : 0.0);
    }
  };
  if (S > 2) prefetch(S - 2);
  {
    const int cl = seg_begin(N, S, S - 1);
    const double* P = V.P(cl);
    const double* p = V.pv() + (long long)cl * nx;
    double* bo = bnd + (S - 1) * bsz;
    for (int e = tid; e < nxx + nx; e += NT) {
      const double v = e < nxx ? P[e] : p[e - nxx];
      if (e < nxx) Pb[e] = v;
      else pb[e - nxx] = v;
      bo[e] = v;
    }
    for (int e = tid; e < np * np; e += NT) {  // the image's pad rows / columns stay zero
      const int i = e / np, j = e - i * np;
      if (i >= LU || j >= LU) Ml[i * CH_GS + j] = 0.0;
    }
  }
  if (lvl) seg_publish(lvl, gen * 64u + 1u);
  bool ok = true;
  for (int s = S - 2; s >= 1; --s) {
#pragma unroll
    for (int i = 0; i < 6; ++i) {  // U (column-major in the segment buffer) transposed into Ut
      const int e = tid + NT * i, j = e / nx, t = e - j * nx;
      if (e < nx * LU) Ut[t * LU + j] = rel[i];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int e = tid + NT * i;
      if (e < nxx + nx) P0s[e] = rp0[i];
    }
    if (s > 1) prefetch(s - 1);
    __syncthreads();
    OCP_SPAN_BEGIN(t_a);
    for (int w = tid >> 6; w < nt * nu4; w += 4) {
      const int r0 = 16 * (w % nt), c0 = 16 * (w / nt), j = c0 + lr;
      v4d acc = mtile(Pb, 1, nx, Ut, LU, 1, r0, c0, nx, LU, nx, v4d{0.0, 0.0, 0.0, 0.0});
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = r0 + lk + 4 * q;
        if (i < nx && j < LU) Tt[i * LU + j] = acc[q] + (j == 2 * nx ? pb[i] : 0.0);
      }
    }
    __syncthreads();
    // M(i, j), i >= j: T(:, i)' U(:, j) + (i == j < nx) + P^0_a / p^0_a in the x rows (lower 16 x 16 tiles)
    const double* P0 = P0s;
    const double* p0 = P0s + nxx;
    for (int w = tid >> 6; w < nu4 * (nu4 + 1) / 2; w += 4) {
      int rb = 0;
      while ((rb + 1) * (rb + 2) / 2 <= w) ++rb;
      const int cb = w - rb * (rb + 1) / 2, r0 = 16 * rb, c0 = 16 * cb, j = c0 + lr;
      v4d acc;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = r0 + lk + 4 * q;
        double v = (i == j && i < nx) ? 1.0 : 0.0;
        if (i >= nx && i < 2 * nx && j >= nx && j < 2 * nx) v = P0[(j - nx) * nx + (i - nx)];
        else if (i == 2 * nx && j >= nx && j < 2 * nx) v = p0[j - nx];
        acc[q] = v;
      }
      acc = mtile(Tt, 1, LU, Ut, LU, 1, r0, c0, LU, LU, nx, acc);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = r0 + lk + 4 * q;
        if (i < LU && j <= i) Ml[i * CH_GS + j] = acc[q];
      }
    }
    __syncthreads();
    OCP_SPANG_END(14, t_a, 0);
    OCP_SPAN_BEGIN(t_g);
    int fl = 0;
    if (tid < 64) {
      fl = chain_elim<2, true>(V, CS, nx, CS.F0, CS.Pa2);
      // cancellation guard: P_a = D - C'N^-1 C loses log10(max D_ii / max P_a,ii) digits; past SEG_CANCEL the combine
      // is refused and the serial chain runs
      double dm = 0.0, am = 0.0;
      if (tid < nx) {
        dm = Ml[(nx + tid) * CH_GS + nx + tid];
        am = CS.Pa2[tid * CH_PS + tid];
      }
      for (int o = 32; o > 0; o >>= 1) {
        dm = fmax(dm, __shfl_xor(dm, o));
        am = fmax(am, __shfl_xor(am, o));
      }
      if (!(dm <= SEG_CANCEL * am)) fl |= CH_WEAK;
    }
    ok = ok && !__syncthreads_or(fl);
    OCP_SPANG_END(15, t_g, 0);
    if (!ok) {
      if (lvl) seg_publish(lvl, gen * 64u + SEG_FAIL);
      break;
    }
    OCP_SPAN_BEGIN(t_p);
    double* bo = bnd + s * bsz;
    for (int e = tid; e < nxx + nx; e += NT) {
      const int I = e < nxx ? e % nx : e - nxx, J = e < nxx ? e / nx : nx;
      const double v = CS.Pa2[I * CH_PS + J];
      if (e < nxx) Pb[e] = v;
      else pb[e - nxx] = v;
      bo[e] = v;
    }
    if (lvl) seg_publish(lvl, gen * 64u + (unsigned)(S - s));
    __syncthreads();
    OCP_SPANG_END(16, t_p, 0);
  }
  return ok;
}

// ---- the partitioned affine scan (the grid form's serial vector recursions: chain_affine's forward rollout
// dx_{k+1} = Acl_k dx_k + bcl_k and the corrector's p_k = Acl_k' p_{k+1} + h_k) ----
// Step s of the sequence maps y_s to y_{s+1} = M_s y_s + c_s (forward: M_s = Acl_{1+s}, c_s = bcl_{1+s}; backward:
// M_s = Acl_{N-1-s}', c_s = h_{N-1-s}); segment g owns the steps [a_g, a_{g+1}), a_g = floor(n g / S), n = N - 1.
//   A: every segment composes its steps' affine maps, [Psi_g psi_g] = M_{a_{g+1}-1} .. M_{a_g} [I 0] + ..., into the
//      segment buffer (affine_comp, on the matrix cores);
//   B: every segment g >= 1 carries the boundary values y_{a_h} = Psi_{h-1} y_{a_{h-1}} + psi_{h-1} (h = 1 .. g, from
//      the recursion's initial value) up to its own, into its first output row (affine_bound);
//   C: every segment runs its steps from its boundary value (chain_affine over the range; the last output row, the
//      next segment's boundary value, stays as that segment's B wrote it). One grid barrier between A and B.
// The serial depth is ~2 n / S steps plus S - 1 matrix-vector products instead of n steps.
__device__ __forceinline__ int aff_begin(int n, int S, int g) { return (int)((long long)n * g / S); }

// A for one segment (workgroup-wide): the steps' matrices and offsets staged in LDS in chunks (region B), the
// composition on the matrix cores ([Psi psi] double-buffered in region A, one 16 x 16 tile per wave per step), the
// result [Psi psi] (column-major nx x (nx + 1)) to dst
template <bool BWD>
__device__ __forceinline__ void affine_comp(const View& V, const ChainLds& CS, int s0, int s1, double* dst) {
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, nx = L.nx, N = L.N, nxx = nx * nx, LX = nx + 1;
  const int SS = (nxx + nx + 1) & ~1, cmax = CH_SCRATCH / SS;
  const int nt = (nx + 15) >> 4, nc = (LX + 15) >> 4, lane = tid & 63, lr = lane & 15, lk = lane >> 4;
  const double* vec = BWD ? V.h() : V.bcl();
  double* X0 = CS.G0;
  double* X1 = X0 + nx * LX;
  for (int e = tid; e < nx * LX; e += NT) {
    const int i = e % nx, j = e / nx;
    X0[e] = i == j ? 1.0 : 0.0;
  }
  int cur = 0;
  for (int cb = s0; cb < s1; cb += cmax) {
    const int ce = cb + cmax < s1 ? cb + cmax : s1, cnt = ce - cb;
    {  // the chunk's [M_s (as stored: Acl_k column-major) | c_s], 16 loads per thread before their stores
      int sx = tid / SS, ox = tid - sx * SS;
      for (int base = 0; base < cnt * SS; base += 16 * NT) {
        double r[16];
        int sl[16], ol[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          sl[i] = sx;
          ol[i] = ox;
          const int k = BWD ? N - 1 - (cb + sx) : 1 + cb + sx;
          const double* src = ox < nxx ? V.Acl(k) + ox : (ox < nxx + nx ? vec + (long long)k * nx + (ox - nxx) : nullptr);
          r[i] = (sx < cnt && src) ? *src : 0.0;
          ox += NT;
          while (ox >= SS) {
            ox -= SS;
            ++sx;
          }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (sl[i] < cnt) CS.Ml[sl[i] * SS + ol[i]] = r[i];
      }
    }
    __syncthreads();
    for (int s = 0; s < cnt; ++s) {
      const double* M = CS.Ml + s * SS;
      const double* Xc = cur ? X1 : X0;
      double* Xn = cur ? X0 : X1;
      for (int w = tid >> 6; w < nt * nc; w += 4) {
        const int r0 = 16 * (w % nt), c0 = 16 * (w / nt), j = c0 + lr;
        v4d acc;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = r0 + lk + 4 * q;
          acc[q] = (j == nx && i < nx) ? M[nxx + i] : 0.0;
        }
        // forward M(i, t) = Acl(i, t) at [t nx + i]; backward M(i, t) = Acl(t, i) at [i nx + t]
        acc = mtile(M, BWD ? nx : 1, BWD ? 1 : nx, Xc, 1, nx, r0, c0, nx, LX, nx, acc);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = r0 + lk + 4 * q;
          if (i < nx && j < LX) Xn[j * nx + i] = acc[q];
        }
      }
      cur ^= 1;
      __syncthreads();
    }
  }
  const double* Xc = cur ? X1 : X0;
  for (int e = tid; e < nx * LX; e += NT) dst[e] = Xc[e];
  __syncthreads();
}

// B on every segment's workgroup g >= 1: y at the start of segments 1 .. g from the recursion's initial value through
// the compositions (staged in LDS region B: g nx (nx + 1) doubles; wave 0, y in LDS), its own one into its output
// row (the one its steps start from; the segment before leaves that row alone), so C follows without a grid barrier
template <bool BWD>
__device__ __forceinline__ void affine_bound(const View& V, const ChainLds& CS, const double* sq, int S, int g,
                                             double* y) {
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, nx = L.nx, N = L.N, n = N - 1, esz = seg_esz(nx), LX = nx + 1;
  double* out = BWD ? V.pv() : V.dx();
  double* Ps = CS.Ml;  // [g][nx (nx + 1)]
  const int tot = g * nx * LX;
  for (int e = tid; e < tot; e += NT) {
    const int h = e / (nx * LX), o = e - h * (nx * LX);
    Ps[e] = sq[(long long)h * esz + o];
  }
  if (tid < nx) y[tid] = BWD ? V.gx()[(long long)N * nx + tid] : V.bcl()[tid];
  __syncthreads();
  if (tid < 64) {
    for (int h = 1; h <= g; ++h) {
      const double* P = Ps + (h - 1) * nx * LX;
      if (tid < nx) {
        double acc = P[nx * nx + tid];
        for (int c0 = 0; c0 < nx; c0 += 8) {
          double pv[8], yv[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int c = c0 + u < nx ? c0 + u : nx - 1;
            pv[u] = P[c * nx + tid];
            yv[u] = y[c];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (c0 + u < nx) acc = fma(pv[u], yv[u], acc);
        }
        __builtin_amdgcn_wave_barrier();
        y[tid] = acc;
        if (h == g) {
          const int a = aff_begin(n, S, g);
          out[(long long)(BWD ? N - a : 1 + a) * nx + tid] = acc;
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  __syncthreads();
}
