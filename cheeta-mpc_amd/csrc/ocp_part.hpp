// ocp_part.hpp — partitioned (parallel-in-time) form of the latency factorisation for the grid form (k_ocp_grid): the
// backward Riccati recursion of the HpipmInterface::solve path (reference HpipmInterface.cpp:282-284 -> HPIPM's
// Riccati factorisation; restated serially by oracle/ocp_ipm.c:ocp_factor) split over S horizon segments, so that the
// chain is S times shorter. Included inside k_ocp.hip's anonymous namespace after ocp_chain.hpp.
//
// Segment s holds the stages [c_s, c_{s+1}), c_s = floor(N s / S), and runs on workgroup s of the problem's grid.
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
//   P2 (workgroup 0): that combine, backward from the last segment's value at c_{S-1} down to c_1 (S - 2 steps, each a
//      Gauss-Jordan solve of the nx x nx system with partial pivoting): the exact value function at every boundary.
//   P3 (segments 0 .. S-2 at once): the chain again over the segment from its end node's exact value: every stage's
//      P_k, p_k, LDL' factor and gains are the factorisation of the serial chain, up to rounding.
// The serial depth is ~2 N / S chain stages plus S - 2 combines instead of N stages. A pivot the first pass's guard
// dropped (M^0_uu singular without the future's cost) or a failed combine falls back to the serial chain, so the
// guarded-pivot behaviour is always the serial one's.
#pragma once

__device__ __forceinline__ int seg_begin(int N, int S, int s) { return (int)((long long)N * s / S); }

// Per-problem segment buffer (OcpSolveArgs::seg, doubles): element s (Phi, W column-major nx x nx, f [nx]) at
// s * seg_esz(nx); the boundary value of node c_j (P column-major, p) at OCP_GRID_MAX_G * seg_esz(nx) + j * seg_bsz(nx)
// (seg_esz / seg_bsz: k_ocp.hpp)

// Segments of the partitioned factorisation for a grid of G workgroups (want: cmpc_ocp_set_segments, 0 = auto): at
// most G and N; auto ~ sqrt(2 N) (two chain passes of N / S stages plus S - 2 combines of about a stage each)
__device__ __forceinline__ int part_segments(int want, int G, int N) {
  int S = want > 0 ? want : (int)(sqrtf(2.0f * (float)N) + 0.5f);
  if (S > G) S = G;
  if (S > N) S = N;
  return S < 1 ? 1 : S;
}

// P1 of a middle segment [a, b) after its chain from V_b = 0 (workgroup-wide; scr: LDS scratch of ChainLds::Ml):
// the gains and closed loop of the pass (chain_gains, acl_pass into the workspace, overwritten by P3), Yt_k =
// B_k L_k^-T D_k^-1/2 into K_k's storage (M^0_uu,k = L D L' from the LDL' columns F = L D, guarded pivots 0), then
// Phi, f, W by the backward accumulation, into el
__device__ __forceinline__ void seg_element(const View& V, const Lds& S, double* scr, int a, int b, double* el) {
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, nx = L.nx, nxx = nx * nx;
  chain_gains(V, a, b);
  __syncthreads();
  acl_pass(V, S, true, a, b, true);
  {
    // one (stage, row) item per thread, its y in an LDS slot (the items in chunks that fit the scratch)
    const int slot = L.numax > 0 ? L.numax : 1, items = (b - a) * nx;
    const int chunk = CH_SCRATCH / slot < NT ? CH_SCRATCH / slot : NT;
    for (int base = 0; base < items; base += chunk) {
      const int e = base + tid;
      if (tid < chunk && e < items) {
        const int k = a + e / nx, r = e - (e / nx) * nx, mk = L.nu[k];
        const double* __restrict__ F = V.Lf(k);
        const double* __restrict__ Bk = V.Bm(k);
        double* __restrict__ Yt = V.K(k);
        double* yd = scr + tid * slot;  // y_c / d_c
        for (int qq = 0; qq < mk; ++qq) {  // y L' = b (L(q, c) = F(q, c) / d_c): y_q = b_q - sum_{c<q} F(q, c) y_c / d_c
          double s = Bk[qq * nx + r];
          for (int c = 0; c < qq; ++c) s = fma(-F[c * mk + qq], yd[c], s);
          const double d = F[qq * mk + qq];
          const double di = d > 1e-200 ? 1.0 / d : 0.0;
          yd[qq] = s * di;
          Yt[r * mk + qq] = s * sqrt(di);
        }
      }
      __syncthreads();
    }
  }
  // backward accumulation over the segment's stages; each stage's operands [Acl_k | Yt_k | bcl_k] staged in LDS, the
  // next stage's loaded into registers meanwhile (no global latency inside the products)
  const int osz = nxx + nx * (L.numax > 0 ? L.numax : 1) + nx;  // <= 1728 doubles (nx <= 27, numax <= 36)
  double* Ph0 = scr;
  double* Ph1 = Ph0 + nxx;
  double* Wm = Ph1 + nxx;
  double* fv = Wm + nxx;
  double* Gm = fv + 32;  // [CH_MAXU][nx]
  double* Op0 = Gm + CH_MAXU * 27;
  double* Op1 = Op0 + osz;
  constexpr int PRE = 7;  // ceil(1728 / NT)
  auto fetch = [&](int k, double (&r)[PRE]) {
    const int mk = L.nu[k], nA = nxx, nY = nx * mk;
    const double* Ac = V.Acl(k);
    const double* Yt = V.K(k);
    const double* bc = V.bcl() + (long long)k * nx;
#pragma unroll
    for (int i = 0; i < PRE; ++i) {
      const int e = tid + NT * i;
      const double* src = e < nA ? Ac + e : (e < nA + nY ? Yt + (e - nA) : (e < nA + nY + nx ? bc + (e - nA - nY) : Ac));
      r[i] = *src;
    }
  };
  auto stash = [&](int k, const double (&r)[PRE], double* Op) {
    const int tot = nxx + nx * L.nu[k] + nx;
#pragma unroll
    for (int i = 0; i < PRE; ++i) {
      const int e = tid + NT * i;
      if (e < tot) Op[e] = r[i];
    }
  };
  double pre[PRE];
  fetch(b - 1, pre);
  for (int e = tid; e < nxx; e += NT) {
    const int i = e % nx, j = e / nx;
    Ph0[e] = i == j ? 1.0 : 0.0;
    Wm[e] = 0.0;
  }
  if (tid < nx) fv[tid] = 0.0;
  stash(b - 1, pre, Op0);
  __syncthreads();
  int cur = 0;
  for (int k = b - 1; k >= a; --k) {
    const int mk = L.nu[k];
    const double* Ph = cur ? Ph1 : Ph0;  // Phi(b, k + 1), column-major
    double* Pn = cur ? Ph0 : Ph1;
    const double* Op = cur ? Op1 : Op0;
    double* On = cur ? Op0 : Op1;
    const double* Ac = Op;
    const double* Yt = Op + nxx;
    const double* bc = Yt + nx * mk;
    if (k > a) fetch(k - 1, pre);
    const int nG = nx * mk;
    for (int e = tid; e < nxx + nG + nx; e += NT) {
      if (e < nxx) {  // Phi(b, k) = Phi(b, k + 1) Acl_k
        const int i = e % nx, j = e / nx;
        double s = 0.0;
#pragma unroll 8
        for (int t = 0; t < nx; ++t) s = fma(Ph[t * nx + i], Ac[j * nx + t], s);
        Pn[e] = s;
      } else if (e < nxx + nG) {  // G = Phi(b, k + 1) Yt_k
        const int e2 = e - nxx, i = e2 % nx, qq = e2 / nx;
        double s = 0.0;
#pragma unroll 8
        for (int t = 0; t < nx; ++t) s = fma(Ph[t * nx + i], Yt[t * mk + qq], s);
        Gm[qq * nx + i] = s;
      } else {  // f += Phi(b, k + 1) bcl_k
        const int i = e - nxx - nG;
        double s = fv[i];
#pragma unroll 8
        for (int t = 0; t < nx; ++t) s = fma(Ph[t * nx + i], bc[t], s);
        fv[i] = s;
      }
    }
    __syncthreads();
    for (int e = tid; e < nxx; e += NT) {  // W += G G' (the same fma order for (i, j) and (j, i): exactly symmetric)
      const int i = e % nx, j = e / nx;
      double s = Wm[e];
      for (int qq = 0; qq < mk; ++qq) s = fma(Gm[qq * nx + i], Gm[qq * nx + j], s);
      Wm[e] = s;
    }
    if (k > a) stash(k - 1, pre, On);
    cur ^= 1;
    __syncthreads();
  }
  const double* Ph = cur ? Ph1 : Ph0;
  for (int e = tid; e < 2 * nxx + nx; e += NT) el[e] = e < nxx ? Ph[e] : (e < 2 * nxx ? Wm[e - nxx] : fv[e - 2 * nxx]);
  __syncthreads();
}

// P2 on one workgroup: the exact value function at the boundaries c_{S-1} .. c_1 into the segment buffer (the last
// segment's own P, p at c_{S-1}; then the combine per middle segment). scr: LDS scratch of ChainLds::Ml (9080
// doubles: the layout below needs 11 nx^2 + 7 nx + 64 <= 8272 for nx <= 27). Returns false on a zero or non-finite
// pivot of a combine's solve.
__device__ __forceinline__ bool seg_combine(const View& V, double* scr, double* sq, int S, int N) {
  const OcpLayout& L = V.L;
  const int tid = threadIdx.x, nx = L.nx, nxx = nx * nx, LW = 2 * nx + 2;
  const int esz = seg_esz(nx), bsz = seg_bsz(nx);
  double* bnd = sq + OCP_GRID_MAX_G * esz;
  double* A0 = scr;             // [nx][LW] row-major: I + W P_b | Phi | f
  double* A1 = A0 + nx * LW;    // Gauss-Jordan double buffer
  double* Pb = A1 + nx * LW;    // P_b (column-major), p_b
  double* pb = Pb + nxx;
  double* Pa = pb + 32;         // P_a, p_a
  double* pa = Pa + nxx;
  double* Ph = pa + 32;         // Phi
  double* Wm = Ph + nxx;        // W
  double* Y = Wm + nxx;         // P_b X (column-major nx x (nx + 1))
  double* Z = Y + nxx + nx;     // Phi' P_b X_Phi
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
  }
  bool ok = true;
  for (int s = S - 2; s >= 1; --s) {
    const int cs = seg_begin(N, S, s);
    const double* el = sq + s * esz;
    for (int e = tid; e < 2 * nxx; e += NT) {
      if (e < nxx) Ph[e] = el[e];
      else Wm[e - nxx] = el[e];
    }
    __syncthreads();
    // A = [I + W P_b | Phi | f]
    for (int e = tid; e < nx * (2 * nx + 1); e += NT) {
      const int i = e / (2 * nx + 1), j = e - i * (2 * nx + 1);
      double v;
      if (j < nx) {
        v = i == j ? 1.0 : 0.0;
#pragma unroll 8
        for (int t = 0; t < nx; ++t) v = fma(Wm[t * nx + i], Pb[j * nx + t], v);
      } else if (j < 2 * nx) {
        v = Ph[(j - nx) * nx + i];
      } else {
        v = el[2 * nxx + i];
      }
      A0[i * LW + j] = v;
    }
    __syncthreads();
    // Gauss-Jordan with partial pivoting (the pivot row found by every thread from the same LDS column: no extra
    // barrier); row k takes the pivot row scaled, the pivot row the old row k eliminated, columns < k are never read
    double* Ac = A0;
    double* An = A1;
    for (int k = 0; k < nx; ++k) {
      int p = k;
      double best = fabs(Ac[k * LW + k]);
      for (int i = k + 1; i < nx; ++i) {
        const double v = fabs(Ac[i * LW + k]);
        if (v > best) {
          best = v;
          p = i;
        }
      }
      const double piv = Ac[p * LW + k];
      ok = ok && piv != 0.0 && isfinite(piv);
      const double pinv = 1.0 / piv;
      const int wc = 2 * nx + 1 - k;
      for (int e = tid; e < nx * wc; e += NT) {
        const int i = e / wc, j = k + (e - i * wc);
        const double rk = Ac[p * LW + j] * pinv;
        double v = rk;
        if (i != k) {
          const int src = i == p ? k : i;
          v = fma(-Ac[src * LW + k], rk, Ac[src * LW + j]);
        }
        An[i * LW + j] = v;
      }
      __syncthreads();
      double* t = Ac;
      Ac = An;
      An = t;
    }
    // Y = P_b [X_Phi X_f]
    for (int e = tid; e < nxx + nx; e += NT) {
      const int i = e % nx, j = e / nx;
      double v = 0.0;
#pragma unroll 8
      for (int t = 0; t < nx; ++t) v = fma(Pb[t * nx + i], Ac[t * LW + nx + j], v);
      Y[j * nx + i] = v;
    }
    __syncthreads();
    // Z = Phi' Y_Phi; p_a = p^0_a + Phi' Y_f + X_Phi' p_b
    const double* P0 = V.P(cs);
    const double* p0 = V.pv() + (long long)cs * nx;
    for (int e = tid; e < nxx + nx; e += NT) {
      if (e < nxx) {
        const int i = e % nx, j = e / nx;
        double v = 0.0;
#pragma unroll 8
        for (int t = 0; t < nx; ++t) v = fma(Ph[i * nx + t], Y[j * nx + t], v);
        Z[e] = v;
      } else {
        const int i = e - nxx;
        double v = 0.0, w = 0.0;
#pragma unroll 8
        for (int t = 0; t < nx; ++t) {
          v = fma(Ph[i * nx + t], Y[nxx + t], v);
          w = fma(Ac[t * LW + nx + i], pb[t], w);
        }
        pa[i] = p0[i] + (v + w);
      }
    }
    __syncthreads();
    double* bo = bnd + s * bsz;
    for (int e = tid; e < nxx + nx; e += NT) {
      if (e < nxx) {
        const int i = e % nx, j = e / nx;
        const double v = P0[e] + 0.5 * (Z[e] + Z[i * nx + j]);  // symmetric by construction
        Pa[e] = v;
        bo[e] = v;
      } else {
        bo[e] = pa[e - nxx];
      }
    }
    __syncthreads();
    for (int e = tid; e < nxx + nx; e += NT) {
      if (e < nxx) Pb[e] = Pa[e];
      else pb[e - nxx] = pa[e - nxx];
    }
    __syncthreads();
  }
  __syncthreads();  // the boundary stores (global) ordered before the grid barrier's release
  return __syncthreads_and(ok) != 0;
}
