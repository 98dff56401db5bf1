"""Riccati quantities of an unconstrained legged-size OCP (the construction of tests/cpp/test_hpipm_interface.cpp's
legged_size: A, B = I + 0.015 U, random costs, known solution) against the closed-form recursion of retrieveRiccati
(testHpipmInterface.cpp:280-304): per quantity, the largest error and its stage. Oracle always; device with --gpu."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "cheeta-mpc_amd", "python"))
import oracle_py as op  # noqa: E402


def problem(seed=1, nx=24, nu=24, N=67):
    rng = np.random.default_rng(seed)
    U = lambda *s: rng.uniform(-1, 1, s)  # noqa: E731
    A = [np.eye(nx) + 0.015 * U(nx, nx) for _ in range(N)]
    B = [np.eye(nx, nu) + 0.015 * U(nx, nu) for _ in range(N)]
    b = [0.015 * U(nx) for _ in range(N)]

    def rc(n):
        M = U(n, n)
        return M @ M.T + n * np.eye(n)
    H = [rc(nx + nu) for _ in range(N)] + [rc(nx)]
    xg, ug, q, r = [U(nx)], [], [], []
    for k in range(N):
        ug.append(U(nu))
        xg.append(b[k] + A[k] @ xg[k] + B[k] @ ug[k])
        Q, S, R = H[k][:nx, :nx], H[k][nx:, :nx], H[k][nx:, nx:]
        q.append(-(Q @ xg[k] + S.T @ ug[k]))
        r.append(-(R @ ug[k] + S @ xg[k]))
    q.append(-H[N] @ xg[N])
    return dict(N=N, nx=nx, nu=[nu] * N, nc=None, x0=xg[0], A=A, B=B, b=b,
                Q=[h[:nx, :nx] for h in H], S=[h[nx:, :nx] for h in H[:N]] + [np.zeros((0, nx))],
                R=[h[nx:, nx:] for h in H[:N]] + [np.zeros((0, 0))], q=q, r=r + [np.zeros(0)])


def closed_form(p):
    N = p["N"]
    Sm, sv = [None] * (N + 1), [None] * (N + 1)
    K, kk = [None] * N, [None] * N
    Sm[N], sv[N] = p["Q"][N], p["q"][N]
    for k in range(N - 1, -1, -1):
        A, B, b = p["A"][k], p["B"][k], p["b"][k]
        P = p["S"][k] + B.T @ Sm[k + 1] @ A
        Rt = p["R"][k] + B.T @ Sm[k + 1] @ B
        rr = p["r"][k] + B.T @ (sv[k + 1] + Sm[k + 1] @ b)
        K[k] = -np.linalg.solve(Rt, P)
        kk[k] = -np.linalg.solve(Rt, rr)
        Sm[k] = p["Q"][k] + A.T @ Sm[k + 1] @ A + P.T @ K[k]
        if "--plain" not in sys.argv:  # symmetrised (the plain recursion's antisymmetric rounding mode grows)
            Sm[k] = 0.5 * (Sm[k] + Sm[k].T)
        sv[k] = p["q"][k] + A.T @ (sv[k + 1] + Sm[k + 1] @ b) + K[k].T @ rr
    return Sm, sv, K, kk


def report(tag, P, pv, K, kf, ref):
    Sm, sv, Kc, kc = ref
    for name, a, b in (("S", P, Sm), ("s", pv, sv), ("K", K, Kc), ("k", kf, kc)):
        errs = [float(np.abs(np.asarray(a[k]) - b[k]).max()) for k in range(len(b))]
        kmax = int(np.argmax(errs))
        print(f"{tag:7s} {name}: max err {errs[kmax]:.3e} at stage {kmax} (|ref| {np.abs(b[kmax]).max():.3e}); "
              f"stage 0 {errs[0]:.3e}, stage 1 {errs[1]:.3e}")


if __name__ == "__main__":
    p = problem()
    ref = closed_form(p)
    from cheeta_mpc import ocp as gen  # noqa: E402
    rec, _ = gen.pack(p)
    o = op.ocp_ipm(p["N"], p["nx"], p["nu"], p["x0"], rec, ric=True)
    print("oracle status", o["status"], "iters", o["iters"])
    report("oracle", o["P"], o["p"], o["K"], o["k"], ref)
    if "--gpu" in sys.argv:
        import cheeta_mpc as cm
        s = cm.OcpSolver(p["N"], p["nx"], p["nu"], None, max_batch=1)
        x, u, st, it = s.solve(p["x0"][None], rec[None], None)
        P, pv, K, kf, Lr, rst = s.riccati(1)
        print("device status", st[0], "iters", it[0], "ric", rst[0])
        report("device", P[0], pv[0], K[0], kf[0], ref)
