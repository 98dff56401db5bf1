"""Prototype of the stage-wise (Riccati) Newton solve of k_ric (cheeta-mpc_amd/csrc/k_ric.hpp), in numpy.

Lab tool, not product code: it restates, step for step and with the kernel's slot indexing, what one wavefront does
per stage, and checks it against the condensed QP of the CPU oracle:
  * solve(b) == (H + D + reg I)^-1 b with H from oracle_condense and D the 3x3 pyramid blocks of every force triple;
  * grad(u) == H u + g (rollout + adjoint).

State of the Newton system at stage k: z_k = [x_k (12: c, v, L, Theta; g_z is constant and dropped); up (12 slots:
the forces of step k-1, slot 3 leg + d)]. Inputs v_k: the stance slots of step k.
Run: python lab/ric_proto.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle_py as op  # noqa: E402

NXR, NZ, NS = 12, 24, 12


def setup(model, x0, xref, foot, contact):
    c = op.consts(model)
    N = model.N
    A, B = op.srbd_dynamics(model, xref, foot, contact)
    sb = [int(sum(int(contact[k, l]) << l for l in range(4))) for k in range(N)]
    feet = op.stance_feet(foot, contact)
    lev = np.zeros((N, 4, 3))
    for k in range(N):
        for l in range(4):
            if sb[k] >> l & 1:
                lev[k, l] = feet[k, l] - xref[k, :3]
    M = A[:, 9:12, 6:9].copy()  # Theta rows of A_k: dt I^-1 Rz^T
    tri = []  # (k, leg) in k-major order
    cb = [0]
    for k in range(N):
        for l in range(4):
            if sb[k] >> l & 1:
                tri.append((k, l))
        cb.append(3 * len(tri))
    return dict(c=c, N=N, A=A, B=B, sb=sb, lev=lev, M=M, tri=tri, cb=cb, dt=model.dt, dtm=model.dt / model.mass,
                qd=np.array([[c.qdiag[k][i] for i in range(13)] for k in range(N + 1)]),
                Wf=np.array([c.Wf[j] for j in range(12)]), Wr=np.array([c.Wr[j] for j in range(12)]))


def lv(r, d):
    """column d of [r]x (dt omitted): L-rows of B for force component d."""
    rx, ry, rz = r
    return [(0.0, rz, -ry), (-rz, 0.0, rx), (ry, -rx, 0.0)][d]


def tri_index(S, k, leg):
    sb = S["sb"][k]
    return S["cb"][k] // 3 + bin(sb & ((1 << leg) - 1)).count("1")


def factor(S, blk, reg):
    """Backward sweep. blk[t] = 3x3 block of triple t (C' Sigma C). Returns per-stage (Linv, Y)."""
    N, dt, dtm = S["N"], S["dt"], S["dtm"]
    P = np.zeros((NZ, NZ))
    P[:NXR, :NXR] = np.diag(S["qd"][N][:NXR])
    out = [None] * N
    for k in range(N - 1, -1, -1):
        Sk = S["sb"][k]
        Sp = S["sb"][k - 1] if k > 0 else 0
        lev = S["lev"][k]
        act = [3 * l + d for l in range(4) if Sk >> l & 1 for d in range(3)]
        # 1. G = B~' P  (row per slot a; lane j = column j)
        G = np.zeros((NS, NZ))
        for a in act:
            l, d = divmod(a, 3)
            w = lv(lev[l], d)
            G[a] = dtm * P[3 + d] + dt * (w[0] * P[6] + w[1] * P[7] + w[2] * P[8]) + P[12 + a]
        # 2. Rt = R_k + G B~
        Rt = np.zeros((NS, NS))
        for a in act:
            for b in act:
                lb, db = divmod(b, 3)
                w = lv(lev[lb], db)
                Rt[a, b] = dtm * G[a, 3 + db] + dt * (w[0] * G[a, 6] + w[1] * G[a, 7] + w[2] * G[a, 8]) + G[a, 12 + b]
            la, da = divmod(a, 3)
            Rt[a, a] += 2 * S["Wf"][a] + (2 * S["Wr"][a] if k >= 1 else 0.0)
            t = tri_index(S, k, la)
            for db in range(3):
                Rt[a, 3 * la + db] += blk[t][da, db]
            Rt[a, a] += reg
        # 3. Cholesky + explicit inverse over the active slots (lane a holds row a; right-looking)
        R = Rt.copy()
        Inv = np.eye(NS)
        Linv = np.zeros((NS, NS))
        for p in act:
            dp = R[p, p]
            invs = 1.0 / np.sqrt(dp) if dp > 1e-200 else 0.0
            l = R[:, p] * invs  # column p of L (rows > p valid)
            Inv[p] *= invs  # row p of L^-1 final
            for a in act:
                if a > p:
                    R[a] -= l[a] * l  # only entries b > p matter
                    Inv[a] -= l[a] * Inv[p]
        for a in act:
            Linv[a] = Inv[a]
        if k == 0:
            out[k] = (Linv, None)
            continue
        # 4. St = S_k + G A~ on z_k, Y = Linv St
        St = np.zeros((NS, NZ))
        for a in act:
            St[a, :NXR] = G[a, :NXR]
            for d in range(3):
                St[a, 3 + d] += dt * G[a, d]
            for s in range(3):
                St[a, 6 + s] += sum(S["M"][k][r, s] * G[a, 9 + r] for r in range(3))
            la = a // 3
            if Sp >> la & 1:
                St[a, 12 + a] += -2 * S["Wr"][a]
        Y = Linv @ St
        out[k] = (Linv, Y)
        # 5. P_k = Q + A~' P A~ - Y'Y (+ 2 Wr on the up slots of the legs of step k-1)
        Pn = np.zeros((NZ, NZ))
        X = P[:NXR, :NXR].copy()
        PA = X.copy()
        for d in range(3):
            PA[:, 3 + d] += dt * X[:, d]
        for s in range(3):
            PA[:, 6 + s] += sum(S["M"][k][r, s] * X[:, 9 + r] for r in range(3))
        APA = PA.copy()
        for d in range(3):
            APA[3 + d] += dt * PA[d]
        for s in range(3):
            APA[6 + s] += sum(S["M"][k][r, s] * PA[9 + r] for r in range(3))
        Pn[:NXR, :NXR] = APA + np.diag(S["qd"][k][:NXR])
        for l in range(4):
            if Sp >> l & 1:
                for d in range(3):
                    Pn[12 + 3 * l + d, 12 + 3 * l + d] += 2 * S["Wr"][3 * l + d]
        Pn -= Y.T @ Y
        P = Pn
    return out


def solve(S, fac, b):
    """(H + D + reg I) du = b, b in condensed (triple) order."""
    N, dt, dtm = S["N"], S["dt"], S["dtm"]
    p = np.zeros(NZ)
    W = [None] * N
    for k in range(N - 1, -1, -1):
        Sk = S["sb"][k]
        Sp = S["sb"][k - 1] if k > 0 else 0
        lev = S["lev"][k]
        act = [3 * l + d for l in range(4) if Sk >> l & 1 for d in range(3)]
        Linv, Y = fac[k]
        h = np.zeros(NS)
        for a in act:
            l, d = divmod(a, 3)
            w = lv(lev[l], d)
            t = tri_index(S, k, l)
            h[a] = -b[3 * t + d] + dtm * p[3 + d] + dt * (w[0] * p[6] + w[1] * p[7] + w[2] * p[8]) + p[12 + a]
        w = Linv @ h
        W[k] = w
        if k == 0:
            break
        pn = np.zeros(NZ)
        pn[:NXR] = p[:NXR]
        for d in range(3):
            pn[3 + d] += dt * p[d]
        for s in range(3):
            pn[6 + s] += sum(S["M"][k][r, s] * p[9 + r] for r in range(3))
        pn -= Y.T @ w
        for l in range(4):
            if not (Sp >> l & 1):
                pn[12 + 3 * l:15 + 3 * l] = 0.0
        p = pn
    du = np.zeros(S["cb"][-1])
    z = np.zeros(NZ)
    for k in range(N):
        Sk = S["sb"][k]
        lev = S["lev"][k]
        act = [3 * l + d for l in range(4) if Sk >> l & 1 for d in range(3)]
        Linv, Y = fac[k]
        y = W[k] + (Y @ z if Y is not None else 0.0)
        v = -(Linv.T @ y)
        for a in act:
            l, d = divmod(a, 3)
            du[3 * tri_index(S, k, l) + d] = v[a]
        zn = np.zeros(NZ)
        x = z[:NXR]
        zn[:NXR] = x
        zn[0:3] += dt * x[3:6]
        zn[9:12] += S["M"][k] @ x[6:9]
        for l in range(4):
            if Sk >> l & 1:
                f = v[3 * l:3 * l + 3]
                zn[3:6] += dtm * f
                zn[6:9] += dt * np.cross(lev[l], f)
                zn[12 + 3 * l:15 + 3 * l] = f
        z = zn
    return du


def grad(S, x0, xref, u):
    """H u + g by rollout (13 states incl. g_z) and adjoint, u in condensed order."""
    N, dt, dtm = S["N"], S["dt"], S["dtm"]
    m = dtm and dt / dtm
    uf = np.zeros((N, 12))
    for t, (k, l) in enumerate(S["tri"]):
        uf[k, 3 * l:3 * l + 3] = u[3 * t:3 * t + 3]
    X = np.zeros((N + 1, 13))
    X[0] = x0
    for k in range(N):
        x = X[k]
        xn = x.copy()
        xn[0:3] += dt * x[3:6]
        xn[5] += dt * x[12]
        xn[9:12] += S["M"][k] @ x[6:9]
        for l in range(4):
            if S["sb"][k] >> l & 1:
                f = uf[k, 3 * l:3 * l + 3]
                xn[3:6] += dtm * f
                xn[6:9] += dt * np.cross(S["lev"][k][l], f)
        X[k + 1] = xn
    lam = S["qd"][N] * (X[N] - xref[N])
    out = np.zeros(S["cb"][-1])
    for k in range(N - 1, -1, -1):
        ns = bin(S["sb"][k]).count("1")
        for l in range(4):
            if S["sb"][k] >> l & 1:
                gl = dtm * lam[3:6] + dt * np.cross(lam[6:9], S["lev"][k][l])
                for d in range(3):
                    j = 3 * l + d
                    fd = m * 9.81 / ns if d == 2 else 0.0
                    acc = gl[d] + 2 * S["Wf"][j] * (uf[k, j] - fd)
                    if k > 0:
                        acc += 2 * S["Wr"][j] * (uf[k, j] - uf[k - 1, j])
                    if k < N - 1:
                        acc -= 2 * S["Wr"][j] * (uf[k + 1, j] - uf[k, j])
                    out[3 * tri_index(S, k, l) + d] = acc
        if k > 0:
            ln = S["qd"][k] * (X[k] - xref[k])
            ln += lam
            ln[3:6] += dt * lam[0:3]
            ln[12] += dt * lam[5]
            ln[6:9] += S["M"][k].T @ lam[9:12]
            lam = ln
    return out


def check(N=10, gait=0, seed=5, nq=6, theta=0.0):
    model = op.default_model(N)
    for j in range(3):
        model.theta_weights[j] = theta
    x0, xref, foot, contact = op.generate(model, seed, nq, gait=gait)
    worst = 0.0
    for q in range(nq):
        S = setup(model, x0[q], xref[q], foot[q], contact[q])
        n, H, g, mu, lo, hi, mp, st = op.condense(model, x0[q], xref[q], foot[q], contact[q])
        assert st == 0 and n == S["cb"][-1]
        H = H[:n, :n]
        g = g[:n]
        rng = np.random.default_rng(q)
        nt = n // 3
        blk = []
        D = np.zeros((n, n))
        for t in range(nt):
            Z = rng.normal(size=(3, 3))
            bk = Z @ Z.T * 10.0 ** rng.uniform(-3, 3)
            blk.append(bk)
            D[3 * t:3 * t + 3, 3 * t:3 * t + 3] = bk
        reg = 1e-12
        fac = factor(S, blk, reg)
        b = rng.normal(size=n)
        du = solve(S, fac, b)
        ref = np.linalg.solve(H + D + reg * np.eye(n), b)
        e1 = np.max(np.abs(du - ref)) / np.max(np.abs(ref))
        u = rng.normal(size=n) * 10
        e2 = np.max(np.abs(grad(S, x0[q], xref[q], u) - (H @ u + g))) / np.max(np.abs(H @ u + g))
        worst = max(worst, e1, e2)
        print(f"N={N} gait={gait} q={q} n={n}: solve rel err {e1:.2e}, grad rel err {e2:.2e}")
    return worst


if __name__ == "__main__":
    w = max(check(10, 0), check(10, 2), check(20, 0), check(10, 0, theta=3.0), check(6, 1))
    print("worst", w)
    assert w < 1e-9
