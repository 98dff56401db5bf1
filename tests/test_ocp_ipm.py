"""HpipmInterface::solve path at the size of its real caller.

The reference's HpipmInterface (ocs2_sqp/hpipm_catkin/src/HpipmInterface.cpp:166-301) hands the OCP to HPIPM's
interior-point method: x0 eliminated (:177-208), the equality rows as two-sided general constraints lg = ug
(:223-264), Riccati Newton steps (ric_alg, HpipmInterfaceSettings.h:56), the Settings' iter_max / tol_* honoured.
Its caller MultipleShootingSolver runs it on the legged robot: nx = 24, nu = 24 (projected: 10-12, 0 at event
nodes), N ~ 70 (ocs2_legged_robot/config/mpc/task.info:33, :40, :102).

Oracle: oracle/ocp_ipm.c (oracle_ocp_ipm), the builder's restatement of HPIPM's OCP IPM (HPIPM itself is not
vendored: parity against its binary is unpinned). It is pinned here on the CPU by
  - its first Newton step against a dense full-space KKT solve of the same system,
  - the reference's own constructions (testHpipmInterface.cpp: knownSolution :112-152, with_constraints :154-206,
    noInputs :208-256, retrieveRiccati :258-340 at 1e-9), at the reference's sizes and at the legged-robot size,
  - the exact constrained solution (np_ref.ocp_eq_fullspace) and the exact constrained feedback of the tail problems.
The device (cmpc_ocp_solve / cmpc_ocp_riccati, csrc/k_ocp.hip) must match the oracle: statuses and iteration counts
equal, trajectories and Riccati quantities to 1e-9 relative (rounding of a different factorisation: Gauss-Jordan
sweeps on the device, Cholesky in the oracle).
"""
import numpy as np
import pytest

import np_ref
from cheeta_mpc import ocp as ocpgen
from test_oracle import random_ocp


def _small(seed, N=5, nx=3, nu=None, nc=None, rows=True):
    rng = np.random.default_rng(seed)
    nu = list(nu or [2] * N)
    nc = list(nc or ([1, 0] + [1] * (N - 1))[: N + 1]) if rows else None
    A, B, b, Q, S, R, q, r = random_ocp(rng, N, nx, nu)
    p = dict(N=N, nx=nx, nu=nu, nc=nc, x0=rng.uniform(-1, 1, nx), A=A, B=B, b=b, Q=Q, S=S, R=R, q=q, r=r)
    Cc, D, e = [], [], []
    for k in range(N + 1):
        m = nu[k] if k < N else 0
        g = nc[k] if nc else 0
        Cc.append(rng.uniform(-1, 1, (g, nx)))
        D.append(rng.uniform(-1, 1, (g, m)))
        e.append(rng.uniform(-1, 1, g))
    p.update(Cc=Cc, D=D, e=e)
    return p


def _known(p, rows_hold=True, seed=0):
    """knownSolution (testHpipmInterface.cpp:112-152): q, r make a random rollout the optimum; with rows_hold the rows
    are satisfied there (then it is the constrained optimum too)."""
    rng = np.random.default_rng(seed + 1000)
    N = p["N"]
    xs, us = [p["x0"]], []
    for k in range(N):
        us.append(rng.uniform(-1, 1, p["nu"][k]))
        xs.append(p["b"][k] + p["A"][k] @ xs[k] + p["B"][k] @ us[k])
        p["q"][k] = -(p["Q"][k] @ xs[k] + p["S"][k].T @ us[k])
        p["r"][k] = -(p["R"][k] @ us[k] + p["S"][k] @ xs[k])
    p["q"][N] = -p["Q"][N] @ xs[N]
    if rows_hold and p.get("nc"):
        for k in range(N + 1):
            if p["nc"][k]:
                p["e"][k] = -(p["Cc"][k] @ xs[k] + (p["D"][k] @ us[k] if k < N else 0.0))
    p["xs"], p["us"] = np.array(xs), us
    return p


def _oracle(op, p, **kw):
    rec, crec = ocpgen.pack(p)
    return op.ocp_ipm(p["N"], p["nx"], p["nu"], p["x0"], rec, nc=p.get("nc"), crec=crec, **kw)


def _split(p, u):
    offs = np.cumsum([0] + list(p["nu"]))
    return [u[offs[k]:offs[k + 1]] for k in range(p["N"])]


def _closed_form_riccati(p, reg=0.0):
    """testHpipmInterface.cpp:280-304 (unconstrained discrete Riccati recursion)."""
    N = p["N"]
    Sm, sv, K, kf = [None] * (N + 1), [None] * (N + 1), [None] * N, [None] * N
    Sm[N], sv[N] = p["Q"][N], p["q"][N]
    for k in range(N - 1, -1, -1):
        A, B, b = p["A"][k], p["B"][k], p["b"][k]
        Q, R, P, q, r = p["Q"][k], p["R"][k], p["S"][k], p["q"][k], p["r"][k]
        PBSA = P + B.T @ Sm[k + 1] @ A
        iR = np.linalg.inv(R + reg * np.eye(len(r)) + B.T @ Sm[k + 1] @ B) if len(r) else np.zeros((0, 0))
        rr = r + B.T @ sv[k + 1] + B.T @ Sm[k + 1] @ b
        Sm[k] = Q + A.T @ Sm[k + 1] @ A - PBSA.T @ iR @ PBSA
        Sm[k] = 0.5 * (Sm[k] + Sm[k].T)  # the plain recursion's antisymmetric rounding mode grows along N
        sv[k] = q + A.T @ sv[k + 1] + A.T @ Sm[k + 1] @ b - PBSA.T @ iR @ rr
        K[k] = -iR @ PBSA
        kf[k] = -iR @ rr
    return Sm, sv, K, kf


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(1.0, np.abs(b).max())) if a.size else 0.0


# ------------------------------------------------------------------------------------------------- oracle (CPU)

def _dense_first_step(p, sig, gu, gx, rb):
    """The cold start's Newton system [H + Gc'Sigma Gc + reg I, G'; G, 0] [dz; dpi] = [-g; -rb] assembled densely."""
    N, nx, nu = p["N"], p["nx"], p["nu"]
    reg = 1e-12
    xo, uo, n = {}, {}, 0
    for k in range(N + 1):
        if k >= 1:
            xo[k] = n
            n += nx
        if k < N:
            uo[k] = n
            n += nu[k]
    H = np.zeros((n, n))
    g = np.zeros(n)
    row0 = 0
    for k in range(N + 1):
        m = nu[k] if k < N else 0
        us = slice(uo[k], uo[k] + m) if k < N else None
        if k >= 1:
            xs = slice(xo[k], xo[k] + nx)
            H[xs, xs] += p["Q"][k] + reg * np.eye(nx)
            g[xs] += gx[k]
        if m:
            H[us, us] += p["R"][k] + reg * np.eye(m)
            g[us] += gu[k]
            if k >= 1:
                H[us, xs] += p["S"][k]
                H[xs, us] += p["S"][k].T
        gk = p["nc"][k] if p.get("nc") else 0
        if gk:
            s = sig[row0:row0 + gk]
            row0 += gk
            Gk = np.zeros((gk, n))
            if k >= 1:
                Gk[:, xs] = p["Cc"][k]
            if m:
                Gk[:, us] = p["D"][k]
            H += Gk.T @ (s[:, None] * Gk)
    G = np.zeros((N * nx, n))
    for k in range(N):
        G[k * nx:(k + 1) * nx, xo[k + 1]:xo[k + 1] + nx] = -np.eye(nx)
        if k >= 1:
            G[k * nx:(k + 1) * nx, xo[k]:xo[k] + nx] = p["A"][k]
        if nu[k]:
            G[k * nx:(k + 1) * nx, uo[k]:uo[k] + nu[k]] = p["B"][k]
    Kkt = np.block([[H, G.T], [G, np.zeros((N * nx, N * nx))]])
    sol = np.linalg.solve(Kkt, np.concatenate([-g, -np.concatenate(rb)]))
    du = np.concatenate([sol[uo[k]:uo[k] + nu[k]] for k in range(N)])
    dx = np.array([np.zeros(nx)] + [sol[xo[k]:xo[k] + nx] for k in range(1, N + 1)])
    return du, dx, sol[n:].reshape(N, nx)


@pytest.mark.parametrize("shape", [dict(N=5, nx=3), dict(N=6, nx=4, nu=[3, 0, 3, 2, 3, 3], nc=[2, 0, 1, 2, 0, 1, 2])])
def test_oracle_first_step_is_the_dense_newton_step(op, shape):
    p = _small(3, **shape)
    rec, crec = ocpgen.pack(p)
    fs = op.ocp_first_step(p["N"], p["nx"], p["nu"], p["x0"], rec, nc=p["nc"], crec=crec)
    assert fs["status"] == 0
    gu = _split(p, fs["rhs_u"])
    du, dx, dpi = _dense_first_step(p, fs["sig"], gu, fs["rhs_x"], list(fs["rb"]))
    assert _rel(fs["du"], du) < 1e-10
    assert _rel(fs["dx"], dx) < 1e-10
    assert _rel(fs["dpi"], dpi) < 1e-10


@pytest.mark.parametrize("nu", [[2] * 5, [2, 0, 2, 2, 2]])
def test_oracle_unconstrained_is_one_newton_step(op, nu):
    """solve_and_check_dynamic / noInputs (testHpipmInterface.cpp:37-69, :208-256): without rows the IPM's first
    Newton step is the solution; equals the condensed solve (oracle_ocp_solve) and the dynamics hold."""
    p = _small(5, nu=nu, rows=False)
    rec, _ = ocpgen.pack(p)
    r = op.ocp_ipm(p["N"], p["nx"], p["nu"], p["x0"], rec)
    assert r["status"] == 0 and r["iters"] == 1
    xc, uc, st = op.ocp_solve(p["N"], p["nx"], p["nu"], p["x0"], rec)
    assert st == 0 and _rel(r["u"], uc) < 1e-10 and _rel(r["x"], xc) < 1e-10
    for k, uk in enumerate(_split(p, r["u"])):
        assert np.allclose(r["x"][k + 1], p["A"][k] @ r["x"][k] + p["B"][k] @ uk + p["b"][k], rtol=1e-12, atol=1e-12)


def test_oracle_retrieve_riccati(op):
    """retrieveRiccati (testHpipmInterface.cpp:258-340): S, s, K, k equal the discrete recursion at 1e-9 and
    u = K x + k along the solution."""
    p = _small(8, rows=False)
    r = _oracle(op, p, ric=True)
    Sm, sv, K, kf = _closed_form_riccati(p)
    for k in range(p["N"] + 1):
        assert _rel(r["P"][k], Sm[k]) < 1e-9 and _rel(r["p"][k], sv[k]) < 1e-9
    us = _split(p, r["u"])
    for k in range(p["N"]):
        assert _rel(r["K"][k], K[k]) < 1e-9 and _rel(r["k"][k], kf[k]) < 1e-9
        assert np.allclose(us[k], r["K"][k] @ r["x"][k] + r["k"][k], atol=1e-9)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_with_constraints(op, seed):
    """with_constraints (testHpipmInterface.cpp:154-206): nc = 1 per node, node 1 empty, node N state-only; the IPM
    converges (HPIPM's stopping rule) to the exact constrained solution (np_ref full-space KKT) and the reference's
    isApprox checks hold at 1e-9."""
    p = _small(seed)
    r = _oracle(op, p)
    assert r["status"] == 0 and 3 <= r["iters"] <= 30
    x, u, _ = np_ref.ocp_eq_fullspace(p["N"], p["nx"], p["nu"], p["x0"], p["A"], p["B"], p["b"], p["Q"], p["S"],
                                      p["R"], p["q"], p["r"], Cc=p["Cc"], D=p["D"], e=p["e"])
    assert _rel(r["x"], x) < 1e-9 and _rel(r["u"], np.concatenate(u)) < 1e-9
    us = _split(p, r["u"])
    for k in range(p["N"]):
        xn = p["A"][k] @ r["x"][k] + p["B"][k] @ us[k] + p["b"][k]
        assert np.linalg.norm(r["x"][k + 1] - xn) <= 1e-9 * np.linalg.norm(xn)
        if p["nc"][k]:
            v = -(p["Cc"][k] @ r["x"][k] + p["D"][k] @ us[k])
            assert np.linalg.norm(p["e"][k] - v) <= 1e-9 * np.linalg.norm(p["e"][k])


def test_oracle_inconsistent_rows_end_at_max_iter_or_min_step(op):
    """HPIPM's OCP IPM treats lg = ug rows as inequalities: contradictory rows cannot be met, the IPM runs out of
    iterations (MAX_ITER) or steps (MIN_STEP) within iter_max; a consistent duplicate row changes nothing."""
    p = _small(21)
    base = _oracle(op, p)
    q = dict(p)
    q["nc"] = list(p["nc"])
    q["nc"][2] = 2
    q["Cc"], q["D"], q["e"] = list(p["Cc"]), list(p["D"]), list(p["e"])
    q["Cc"][2] = np.vstack([p["Cc"][2], p["Cc"][2]])
    q["D"][2] = np.vstack([p["D"][2], p["D"][2]])
    q["e"][2] = np.concatenate([p["e"][2], p["e"][2]])
    dup = _oracle(op, q)
    assert base["status"] == 0 and dup["status"] == 0
    assert _rel(dup["u"], base["u"]) < 1e-8
    q["e"][2] = np.concatenate([p["e"][2], p["e"][2] + 1.0])
    for it_max in (30, 12):
        bad = _oracle(op, q, settings=op.default_settings(iter_max=it_max))
        assert bad["status"] in (1, 2) and bad["iters"] <= it_max
        assert bad["res"][2] > 1e-3  # the rows stay violated


def _tail_feedback(p, k, eps=1.0):
    """Exact du_k/dx_k of the equality-constrained tail problem k..N (np_ref full-space solve from x_k = 0 and the
    unit vectors; the state-only rows of node k dropped, x_k being given), the limit of the barrier-weighted K_k."""
    N, nx = p["N"], p["nx"]
    sl = lambda a: list(a[k:])  # noqa: E731
    Cc, D, e = sl(p["Cc"]), sl(p["D"]), sl(p["e"])
    if p["nc"][k]:
        keep = np.abs(D[0]).sum(axis=1) > 0
        Cc[0], D[0], e[0] = Cc[0][keep], D[0][keep], e[0][keep]
    args = (N - k, nx, p["nu"][k:], None, sl(p["A"]), sl(p["B"]), sl(p["b"]), sl(p["Q"]), sl(p["S"]), sl(p["R"]),
            sl(p["q"]), sl(p["r"]))
    u0 = np_ref.ocp_eq_fullspace(*args[:3], np.zeros(nx), *args[4:], Cc=Cc, D=D, e=e)[1][0]
    K = np.zeros((len(u0), nx))
    for i in range(nx):
        xi = np.zeros(nx)
        xi[i] = eps
        K[:, i] = (np_ref.ocp_eq_fullspace(*args[:3], xi, *args[4:], Cc=Cc, D=D, e=e)[1][0] - u0) / eps
    return K


def test_oracle_constrained_riccati(op):
    """After an equality-constrained solve: K_k (k >= 1) is the barrier-weighted feedback at the exit point, which
    approaches the exact constrained feedback of the tail problem as Sigma -> inf on the rows (a row whose multiplier
    is ~0 keeps a moderate Sigma = l / t at the exit point, so the agreement is ~1e-4, not 1e-9: a property of the
    interior-point method, HPIPM's included); u_k = K_k x_k + k_k holds at the returned point to the IPM's accuracy."""
    p = _small(2)
    r = _oracle(op, p, ric=True)
    assert r["status"] == 0
    us = _split(p, r["u"])
    for k in range(1, p["N"]):
        assert np.abs(us[k] - (r["K"][k] @ r["x"][k] + r["k"][k])).max() < 1e-8
        assert _rel(r["K"][k], _tail_feedback(p, k)) < 1e-3


@pytest.mark.parametrize("projected", [True, False])
def test_oracle_legged_size_known_solution(op, projected):
    """knownSolution at the ocs2_legged_robot size (nx = 24, N = 70 with three event nodes; projected: nu 10 / 12 / 0
    and no rows; else nu = 24 and 12-14 equality rows per node, satisfied at the known solution)."""
    p = ocpgen.legged_problem(7, projected=projected, known_solution=True, rows_hold=True, cost="random")
    assert p["N"] == 70 and p["nx"] == 24
    r = _oracle(op, p)
    assert r["status"] == 0
    assert r["iters"] == 1 if projected else r["iters"] <= 30
    assert _rel(r["x"], p["xs"]) < 1e-9
    assert _rel(r["u"], np.concatenate(p["us"])) < 1e-9


def test_oracle_legged_constrained_matches_fullspace(op):
    """The legged-size problem with binding rows (random e): the IPM's solution equals the exact full-space solve."""
    p = ocpgen.legged_problem(11, projected=False)
    r = _oracle(op, p)
    assert r["status"] == 0
    x, u, _ = np_ref.ocp_eq_fullspace(p["N"], p["nx"], p["nu"], p["x0"], p["A"], p["B"], p["b"], p["Q"], p["S"],
                                      p["R"], p["q"], p["r"], Cc=p["Cc"], D=p["D"], e=p["e"])
    assert _rel(r["x"], x) < 1e-8 and _rel(r["u"], np.concatenate(u)) < 1e-8


def test_oracle_stats_table(op):
    """Per-iteration statistics: rows 0..iters, residual columns equal to the exit residuals on the last row."""
    p = _small(4)
    r = _oracle(op, p, stats_rows=31)
    st = r["stats"]
    it = r["iters"]
    assert np.all(np.isnan(st[it + 1:]))
    assert np.allclose(st[it, 6:], r["res"], rtol=0, atol=0)
    assert np.all(np.isnan(st[it, :5]))
    assert np.all(st[:it, 3] > 0) and np.all(st[:it, 3] <= 1)


# ------------------------------------------------------------------------------------------------- device (GPU)

def _device_batch(cm, ps, settings=None):
    p0 = ps[0]
    recs, crecs = zip(*[ocpgen.pack(p) for p in ps])
    solver = cm.OcpSolver(p0["N"], p0["nx"], p0["nu"], p0.get("nc"), settings=settings, max_batch=len(ps))
    x, u, st, it = solver.solve(np.array([p["x0"] for p in ps]), np.array(recs),
                                np.array(crecs) if p0.get("nc") else None)
    return solver, x, u, st, it


def _check_vs_oracle(op, ps, x, u, st, it, settings=None, tol=1e-9):
    for i, p in enumerate(ps):
        r = _oracle(op, p, settings=settings)
        assert st[i] == r["status"], (i, st[i], r["status"])
        assert it[i] == r["iters"], (i, it[i], r["iters"])
        assert _rel(x[i], r["x"]) < tol, (i, _rel(x[i], r["x"]))
        assert _rel(u[i], r["u"]) < tol, (i, _rel(u[i], r["u"]))


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [dict(N=5, nx=3), dict(N=6, nx=4, nu=[3, 0, 3, 2, 3, 3], nc=[2, 0, 1, 2, 0, 1, 2]),
                                   dict(N=5, nx=3, rows=False), dict(N=5, nx=3, nu=[2, 0, 2, 2, 2], rows=False)])
def test_device_small_shapes_match_oracle(cm, op, shape):
    ps = [_small(40 + i, **shape) for i in range(6)]
    _, x, u, st, it = _device_batch(cm, ps)
    _check_vs_oracle(op, ps, x, u, st, it)


@pytest.mark.gpu
@pytest.mark.parametrize("projected", [True, False])
def test_device_legged_size_matches_oracle(cm, op, projected):
    """nx = 24, N = 70 (67 intervals + 3 event nodes), projected (nu 10 / 12 / 0, no rows) or with the 12-14 equality
    rows per node (nu = 24): a batch of 6 seeded problems, device vs oracle."""
    ps = [ocpgen.legged_problem(100 + i, projected=projected) for i in range(6)]
    _, x, u, st, it = _device_batch(cm, ps)
    assert np.all(st == 0)
    _check_vs_oracle(op, ps, x, u, st, it, tol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("projected", [True, False])
def test_device_legged_known_solution(cm, op, projected):
    ps = [ocpgen.legged_problem(200 + i, projected=projected, known_solution=True, rows_hold=True, cost="random")
          for i in range(3)]
    _, x, u, st, it = _device_batch(cm, ps)
    for i, p in enumerate(ps):
        assert st[i] == 0
        assert _rel(x[i], p["xs"]) < 1e-9 and _rel(u[i], np.concatenate(p["us"])) < 1e-9


@pytest.mark.gpu
def test_device_with_constraints_reference_properties(cm, op):
    ps = [_small(60 + i) for i in range(4)]
    _, x, u, st, it = _device_batch(cm, ps)
    for i, p in enumerate(ps):
        assert st[i] == 0
        us = _split(p, u[i])
        for k in range(p["N"]):
            xn = p["A"][k] @ x[i][k] + p["B"][k] @ us[k] + p["b"][k]
            assert np.linalg.norm(x[i][k + 1] - xn) <= 1e-9 * np.linalg.norm(xn)
            if p["nc"][k]:  # to the IPM's accuracy (tol_eq 1e-8): absolute below unit-size e
                v = -(p["Cc"][k] @ x[i][k] + p["D"][k] @ us[k])
                assert np.linalg.norm(p["e"][k] - v) <= 1e-9 * max(1.0, np.linalg.norm(p["e"][k]))


@pytest.mark.gpu
def test_device_inconsistent_rows_status(cm, op):
    p = _small(21)
    q = dict(p)
    q["nc"] = list(p["nc"])
    q["nc"][2] = 2
    q["Cc"], q["D"], q["e"] = list(p["Cc"]), list(p["D"]), list(p["e"])
    q["Cc"][2] = np.vstack([p["Cc"][2], p["Cc"][2]])
    q["D"][2] = np.vstack([p["D"][2], p["D"][2]])
    q["e"][2] = np.concatenate([p["e"][2], p["e"][2] + 1.0])
    for it_max in (30, 12):
        s = cm.default_settings(iter_max=it_max)
        _, x, u, st, it = _device_batch(cm, [q], settings=s)
        r = _oracle(op, q, settings=op.default_settings(iter_max=it_max))
        assert st[0] in (1, 2) and st[0] == r["status"] and it[0] == r["iters"] <= it_max


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["small", "legged_projected", "legged_rows"])
def test_device_riccati_matches_oracle(cm, op, case):
    """cmpc_ocp_riccati vs the oracle's Riccati quantities (P, p, K, k, Lr per stage) at 1e-9; without rows also vs
    the closed-form recursion of retrieveRiccati (testHpipmInterface.cpp:280-304) and u = K x + k."""
    if case == "small":
        ps = [_small(70 + i, rows=False) for i in range(3)]
    elif case == "legged_projected":
        ps = [ocpgen.legged_problem(300 + i, projected=True) for i in range(3)]
    else:
        ps = [ocpgen.legged_problem(310 + i, projected=False) for i in range(3)]
    solver, x, u, st, it = _device_batch(cm, ps)
    P, pv, K, kf, Lr, rst = solver.riccati(len(ps))
    assert np.all(rst == 0)
    # With rows the factorisation at the exit point weights them by Sigma = lam / t with t ~ 1e-10: each
    # implementation's slacks carry ~1e-16 |C x + D u| of rounding, i.e. ~1e-6 of t, into the weights of the
    # constrained directions (1e10+), and P, p, Lr, K, k are formed by eliminations across those weights: device and
    # oracle agree to 1e-4 of each quantity's largest entry there (measured 1e-5), and the Sigma-free checks carry the
    # parity: the policy on the solution (below) and, in the C++ mirror, K_0 against finite differences of the solve.
    # Without rows everything agrees to 1e-9 / 1e-8.
    rows = ps[0].get("nc") is not None
    tS = 1e-4 if rows else 1e-9
    for i, p in enumerate(ps):
        r = _oracle(op, p, ric=True)
        N = p["N"]
        for k in range(1, N + 1):
            assert _rel(P[i][k], r["P"][k]) < tS, ("P", k)
            assert _rel(pv[i][k], r["p"][k]) < max(tS, 1e-8), ("p", k)
            assert np.array_equal(P[i][k], P[i][k].T), ("P symmetric (lower triangle mirrored)", k)
        for k in range(N):
            assert _rel(Lr[i][k], r["Lr"][k]) < tS, ("Lr", k)
            if k > 0:
                assert _rel(K[i][k], r["K"][k]) < (tS if rows else 1e-9), ("K", k)
                assert _rel(kf[i][k], r["k"][k]) < (tS if rows else 1e-8), ("k", k)
        if rows:  # the policy on the solution (u - K x - k is the exit point's Newton feedforward, near tolerance)
            us = _split(p, u[i])
            for k in range(1, N):
                assert np.allclose(us[k], K[i][k] @ x[i][k] + kf[i][k], atol=1e-6), ("policy", k)
            continue  # stage 0 rebuilt from P_1 (above) and the record: the same Sigma sensitivity
        # stage 0, the reference's reconstruction (HpipmInterface.cpp:416-453): P_0 = Q_0 + A_0'P_1 A_0 - T1'T1 and
        # p_0 cancel terms of the size of A_0'P_1 A_0 (with rows at node 1 P_1 carries their barrier weight, 1e10+), and
        # K_0, k_0 are solves with M_0 = Lr_0 Lr_0' (node-0 rows' weight inside): both implementations' rounding is
        # amplified alike, so the bound is 1e-9 of the cancelled terms and 1e-15 cond(M_0) for the solves (equal to
        # 1e-9 relative when there are no rows)
        A0, b0 = p["A"][0], p["b"][0]
        sP = np.abs(A0.T @ r["P"][1] @ A0).max() + np.abs(p["Q"][0]).max()
        sp = np.abs(A0.T @ (r["p"][1] + r["P"][1] @ b0)).max() + np.abs(p["q"][0]).max()
        assert np.abs(P[i][0] - r["P"][0]).max() <= 1e-9 * max(sP, np.abs(r["P"][0]).max(), 1.0), "P_0"
        assert np.abs(pv[i][0] - r["p"][0]).max() <= 1e-9 * max(sp, np.abs(r["p"][0]).max(), 1.0), "p_0"
        if p["nu"][0]:
            kap = np.linalg.cond(r["Lr"][0] @ r["Lr"][0].T)
            assert _rel(K[i][0], r["K"][0]) <= 1e-9 + 1e-15 * kap, ("K_0", kap)
            assert _rel(kf[i][0], r["k"][0]) <= 1e-8 + 1e-15 * kap, ("k_0", kap)
        if p.get("nc") is None:
            Sm, sv, Kc, kc = _closed_form_riccati(p)
            us = _split(p, u[i])
            for k in range(N):
                assert _rel(K[i][k], Kc[k]) < 1e-8 and _rel(kf[i][k], kc[k]) < 1e-7
                assert np.allclose(us[k], K[i][k] @ x[i][k] + kf[i][k], atol=1e-8)


@pytest.mark.gpu
def test_device_residuals_and_stats_match_oracle(cm, op):
    ps = [_small(80 + i) for i in range(3)]
    solver, x, u, st, it = _device_batch(cm, ps)
    res = solver.residuals(len(ps))
    stats = solver.stats(len(ps))
    for i, p in enumerate(ps):
        r = _oracle(op, p, stats_rows=solver.stat_rows)
        # final residuals sit at rounding level (1e-12): agreement to 1e-10 absolute, 1e-6 relative above it
        assert np.allclose(res[i], r["res"], rtol=1e-6, atol=1e-10)
        n = solver.stat_rows  # every row: those after the last iteration are NaN on both sides (cmpc.h)
        a, b = stats[i][:n], r["stats"][:n]
        assert np.array_equal(np.isnan(a), np.isnan(b))
        fin = ~np.isnan(b)
        assert np.allclose(a[fin], b[fin], rtol=1e-6, atol=1e-10)


@pytest.mark.gpu
def test_device_pointer_entry_equals_host_entry(cm, op):
    """cmpc_ocp_solve (device pointers, caller's stream) and cmpc_ocp_solve_host give identical results."""
    ps = [ocpgen.legged_problem(400 + i, projected=False) for i in range(4)]
    solver, x, u, st, it = _device_batch(cm, ps)
    recs, crecs = zip(*[ocpgen.pack(p) for p in ps])
    B = len(ps)
    dx0 = cm.DeviceArray.from_host(np.array([p["x0"] for p in ps]))
    drec = cm.DeviceArray.from_host(np.array(recs))
    dcrec = cm.DeviceArray.from_host(np.array(crecs))
    dx = cm.DeviceArray((B, ps[0]["N"] + 1, 24), np.float64)
    du = cm.DeviceArray((B, solver.nU), np.float64)
    dst = cm.DeviceArray((B,), np.int32)
    dit = cm.DeviceArray((B,), np.int32)
    solver.solve_device(B, dx0, drec, dcrec, dx, du, dst, dit)
    assert np.array_equal(dx.host(), x) and np.array_equal(du.host(), u)
    assert np.array_equal(dst.host(), st) and np.array_equal(dit.host(), it)


@pytest.mark.gpu
def test_device_getters_ordered_after_stream_solve(cm, op):
    """cmpc_ocp_solve on the caller's (non-blocking) stream, then riccati / residuals / stats on the handle with no
    synchronisation in between: the handle's getters wait on an event recorded after the solve, so they
    read the finished workspace — equal to the same getters after a full device synchronisation."""
    import ctypes as C
    ps = [ocpgen.legged_problem(410 + i, projected=False) for i in range(3)]
    recs, crecs = zip(*[ocpgen.pack(p) for p in ps])
    B, p0 = len(ps), ps[0]
    H = cm.hip()
    stream = C.c_void_p()
    assert H.hipStreamCreateWithFlags(C.byref(stream), 1) == 0  # hipStreamNonBlocking
    dx0 = cm.DeviceArray.from_host(np.array([p["x0"] for p in ps]))
    drec = cm.DeviceArray.from_host(np.array(recs))
    dcrec = cm.DeviceArray.from_host(np.array(crecs))
    out = []
    for sync in (False, True):
        s = cm.OcpSolver(p0["N"], p0["nx"], p0["nu"], p0.get("nc"), max_batch=B)
        dx = cm.DeviceArray((B, p0["N"] + 1, p0["nx"]), np.float64)
        du = cm.DeviceArray((B, s.nU), np.float64)
        dst, dit = cm.DeviceArray((B,), np.int32), cm.DeviceArray((B,), np.int32)
        s.solve_device(B, dx0, drec, dcrec, dx, du, dst, dit, stream)
        if sync:
            H.hipDeviceSynchronize()
        ric = s.riccati(B)
        res = s.residuals(B)
        out.append((ric, res, dst.host()))
        s.close()
    H.hipStreamDestroy(stream)
    (r0, e0, s0), (r1, e1, s1) = out
    assert np.array_equal(s0, s1) and np.all(s0 == 0)
    assert np.array_equal(e0, e1)
    assert np.array_equal(r0[0], r1[0]) and np.array_equal(r0[1], r1[1]) and np.array_equal(r0[5], r1[5])
    for b in range(B):
        for k in range(p0["N"]):
            assert np.array_equal(r0[2][b][k], r1[2][b][k]) and np.array_equal(r0[4][b][k], r1[4][b][k])


@pytest.mark.gpu
@pytest.mark.parametrize("projected", [True, False])
def test_device_staging_views_equal_copies(cm, op, projected):
    """The host path with the problem written into the handle's pinned staging (OcpSolver.staging(): no host copy,
    as the C++ mirror packs it) gives the same solution bit for bit as from ordinary arrays."""
    p = ocpgen.legged_problem(420, projected=projected)
    rec, crec = ocpgen.pack(p)
    s = cm.OcpSolver(p["N"], p["nx"], p["nu"], p.get("nc"), max_batch=1)
    x1, u1, st1, it1 = s.solve(p["x0"][None], rec[None], crec[None] if crec is not None else None)
    stg = s.staging()
    assert stg is not None
    sx0, srec, screc = stg
    sx0[0] = p["x0"]
    srec[0] = rec
    if screc is not None:
        screc[0] = crec
    x2, u2, st2, it2 = s.solve(sx0[:1], srec[:1], screc[:1] if screc is not None else None)
    s.close()
    assert st1[0] == st2[0] == 0 and it1[0] == it2[0]
    assert np.array_equal(x1, x2) and np.array_equal(u1, u2)


def _device_batch_path(cm, ps, chain, grid=0):
    p0 = ps[0]
    recs, crecs = zip(*[ocpgen.pack(p) for p in ps])
    solver = cm.OcpSolver(p0["N"], p0["nx"], p0["nu"], p0.get("nc"), max_batch=len(ps))
    solver.set_path(chain)
    solver.set_grid(grid)
    x, u, st, it = solver.solve(np.array([p["x0"] for p in ps]), np.array(recs),
                                np.array(crecs) if p0.get("nc") else None)
    return solver, x, u, st, it


@pytest.mark.gpu
@pytest.mark.parametrize("projected", [False, True])
def test_device_two_per_cu_instantiation_equals_one_per_cu(cm, op, projected):
    """Batches above 256 run k_ocp_ipm<64, 2> (bounded at 256 VGPRs) with the node-by-node staged residuals, batches up
    to 64 k_ocp_ipm<64, 1> with every node's residuals at once (OcpSolveArgs::par_res): with the batched form of the
    factorisation in both (cmpc_ocp_set_path(0)) the same fma chains, so the same problems give bit-identical
    results either way."""
    ps = [ocpgen.legged_problem(500 + i, projected=projected) for i in range(8)]
    _, x1, u1, st1, it1 = _device_batch_path(cm, ps, 0)
    big = [ps[i % 8] for i in range(264)]
    _, x2, u2, st2, it2 = _device_batch_path(cm, big, 0)
    for i in range(264):
        j = i % 8
        assert st2[i] == st1[j] and it2[i] == it1[j]
        assert np.array_equal(x2[i], x1[j]) and np.array_equal(u2[i], u1[j])


@pytest.mark.gpu
@pytest.mark.parametrize("projected", [True, False])
def test_device_grid_form_equals_one_workgroup(cm, op, projected):
    """Batches of up to 32 run in the grid form (G workgroups per problem, stage ranges, grid barriers, reductions in
    a fixed order): statuses and iterations equal to the single-workgroup latency form and to the oracle, trajectories
    to rounding (the sums of mu and of the step's complementarity are ordered differently), for the automatic width,
    an uneven G = 7 and G = 2."""
    ps = [ocpgen.legged_problem(540 + i, projected=projected) for i in range(3)]
    s1, x1, u1, st1, it1 = _device_batch_path(cm, ps, 1, grid=1)
    assert s1.grid(3) == 0
    _check_vs_oracle(op, ps, x1, u1, st1, it1)
    for G in (0, 7, 2):
        sg, xg, ug, stg, itg = _device_batch_path(cm, ps, 1, grid=G)
        assert sg.grid(3) == (min(32, ps[0]["N"], 256 // 3) if G == 0 else G)
        assert np.array_equal(stg, st1) and np.array_equal(itg, it1), G
        for i in range(len(ps)):
            assert _rel(xg[i], x1[i]) < 1e-10 and _rel(ug[i], u1[i]) < 1e-10, G
        _check_vs_oracle(op, ps, xg, ug, stg, itg)


@pytest.mark.gpu
@pytest.mark.parametrize("projected", [True, False])
def test_device_latency_form_equals_batched_form(cm, op, projected):
    """Small batches take the latency form of the factorisation (ocp_chain.hpp: LDL' on 4 x 4 lower blocks, gains by
    back substitution); the batched form (Gauss-Jordan sweep) is the other factorisation of the same Newton systems:
    statuses and iteration counts equal, trajectories to rounding, both against the oracle at 1e-9; a batch of 264
    (above the latency form's 256) takes the batched form and equals the small batch to rounding as well."""
    ps = [ocpgen.legged_problem(520 + i, projected=projected) for i in range(6)]
    s1, x1, u1, st1, it1 = _device_batch_path(cm, ps, 1)
    assert s1.path == 1
    s0, x0, u0, st0, it0 = _device_batch_path(cm, ps, 0)
    assert s0.path == 0
    assert np.array_equal(st1, st0) and np.array_equal(it1, it0)
    for i in range(len(ps)):
        assert _rel(x1[i], x0[i]) < 1e-10 and _rel(u1[i], u0[i]) < 1e-10
    _check_vs_oracle(op, ps, x1, u1, st1, it1)
    big = [ps[i % 6] for i in range(264)]
    _, x2, u2, st2, it2 = _device_batch_path(cm, big, 1)
    for i in range(264):
        j = i % 6
        assert st2[i] == st1[j] and it2[i] == it1[j]
        assert _rel(x2[i], x1[j]) < 1e-10 and _rel(u2[i], u1[j]) < 1e-10


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [False, True])
def test_device_wide_stage_class_matches_oracle(cm, op, rows):
    """nu_k + nx + 1 > 64 takes the NZP = 128 instantiation (k_ocp_ipm<128, 1>): nx = 20, nu_k up to 50."""
    shape = dict(N=4, nx=20, nu=[50, 30, 45, 10], nc=[0, 6, 3, 4, 2] if rows else None, rows=rows)
    ps = [_small(90 + i, **shape) for i in range(3)]
    solver, x, u, st, it = _device_batch(cm, ps)
    _check_vs_oracle(op, ps, x, u, st, it)


@pytest.mark.gpu
@pytest.mark.parametrize("case", [
    # (shape, latency form expected): the chain's bound nu_k + nx + 1 <= 60 (OCP_CHAIN_MAX_N1), one past it, the NZP
    # = 64 / 128 instantiation boundary, the shortest horizon and a one-state system
    (dict(N=6, nx=24, nu=[35] * 6), 1),
    (dict(N=6, nx=24, nu=[35] * 6, rows=False), 1),
    (dict(N=6, nx=24, nu=[35, 0, 12, 35, 20, 35], nc=[2, 0, 3, 1, 4, 2, 1]), 1),
    (dict(N=6, nx=24, nu=[36] * 6), 0),
    (dict(N=6, nx=24, nu=[36] * 6, rows=False), 0),
    (dict(N=4, nx=20, nu=[43] * 4), 0),
    (dict(N=4, nx=20, nu=[44, 43, 44, 10]), 0),
    (dict(N=1, nx=3, nu=[2]), 1),
    (dict(N=8, nx=1, nu=[1] * 8), 1),
], ids=["n1_60", "n1_60_norows", "n1_60_mixed", "n1_61", "n1_61_norows", "n1_64", "n1_65", "N1", "nx1"])
def test_device_dimension_boundaries_match_oracle(cm, op, case):
    """The dimension limits of the device paths: the latency form takes nu_k + nx + 1 <= 60 and hands anything wider to
    the batched form (cmpc_ocp_path), the batched form switches to its NZP = 128 instantiation past 64; each side of
    each limit, the one-stage horizon and nx = 1 against the oracle (status, iterations, x / u at 1e-9)."""
    shape, chain = case
    ps = [_small(700 + i, **shape) for i in range(3)]
    solver, x, u, st, it = _device_batch(cm, ps)
    assert solver.path == chain
    _check_vs_oracle(op, ps, x, u, st, it)


def test_oracle_warm_start_from_solution(op):
    """HPIPM's primal warm start (warm_start = 1): from the converged x, u the IPM needs no more iterations than cold
    and lands on the same solution."""
    p = _small(33)
    r = _oracle(op, p)
    s = op.default_settings()
    s.warm_start = 1
    rec, crec = ocpgen.pack(p)
    w = op.ocp_ipm(p["N"], p["nx"], p["nu"], p["x0"], rec, nc=p["nc"], crec=crec, settings=s,
                   guess=(r["x"], r["u"]))
    assert w["status"] == 0 and w["iters"] <= r["iters"]
    assert _rel(w["u"], r["u"]) < 1e-8


@pytest.mark.gpu
def test_device_warm_start_matches_oracle(cm, op):
    """The same warm start on the device (cmpc_ocp_solve_host with x, u in / out): statuses, iterations and the
    solution equal the oracle's from the same guess (a perturbed solution of the legged problem with rows)."""
    ps = [ocpgen.legged_problem(600 + i, projected=False) for i in range(3)]
    p0 = ps[0]
    s = cm.default_settings()
    s.warm_start = 1
    recs, crecs = zip(*[ocpgen.pack(p) for p in ps])
    solver = cm.OcpSolver(p0["N"], p0["nx"], p0["nu"], p0.get("nc"), settings=s, max_batch=len(ps))
    rng = np.random.default_rng(5)
    guesses = []
    for p in ps:
        r = _oracle(op, p)
        guesses.append((r["x"] + 1e-3 * rng.standard_normal(r["x"].shape), r["u"] + 1e-3 * rng.standard_normal(r["u"].shape)))
    gx = np.array([g[0] for g in guesses])
    gu = np.array([g[1] for g in guesses])
    x, u, st, it = solver.solve(np.array([p["x0"] for p in ps]), np.array(recs), np.array(crecs), guess=(gx, gu))
    so = op.default_settings()
    so.warm_start = 1
    for i, p in enumerate(ps):
        w = op.ocp_ipm(p["N"], p["nx"], p["nu"], p["x0"], recs[i], nc=p["nc"], crec=crecs[i], settings=so,
                       guess=guesses[i])
        assert st[i] == w["status"] and it[i] == w["iters"], (i, st[i], w["status"], it[i], w["iters"])
        assert _rel(x[i], w["x"]) < 1e-9 and _rel(u[i], w["u"]) < 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("projected", [True, False])
def test_device_keep_riccati_equals_refactorisation(cm, op, projected):
    """cmpc_ocp_set_keep_riccati: the grid-form solve leaves the exit point's Riccati quantities (HPIPM's getters read
    its workspace, HpipmInterface.cpp:336-360), so cmpc_ocp_riccati is a copy: equal to the on-demand refactorisation
    (k_ocp_ric) of the same solve, without rows to rounding (the factorisation is the last Newton step's), with rows to
    the Sigma-conditioning bound of test_device_riccati_matches_oracle; and the oracle's."""
    ps = [ocpgen.legged_problem(320 + i, projected=projected) for i in range(3)]
    p0 = ps[0]
    recs, crecs = zip(*[ocpgen.pack(p) for p in ps])
    out = []
    for keep in (1, 0):
        solver = cm.OcpSolver(p0["N"], p0["nx"], p0["nu"], p0.get("nc"), max_batch=len(ps))
        solver.set_keep_riccati(keep)
        x, u, st, it = solver.solve(np.array([p["x0"] for p in ps]), np.array(recs),
                                    np.array(crecs) if p0.get("nc") else None)
        assert np.all(st == 0)
        out.append(solver.riccati(len(ps)))
    (P1, p1, K1, k1, L1, r1), (P0, p0_, K0, k0, L0, r0) = out
    assert np.all(r1 == 0) and np.all(r0 == 0)
    rows = p0.get("nc") is not None
    tS = 1e-4 if rows else 1e-9
    for i, p in enumerate(ps):
        r = _oracle(op, p, ric=True)
        for k in range(1, p["N"] + 1):
            assert _rel(P1[i][k], P0[i][k]) < tS and _rel(P1[i][k], r["P"][k]) < tS, ("P", k)
            assert _rel(p1[i][k], p0_[i][k]) < max(tS, 1e-8), ("p", k)
        for k in range(p["N"]):
            assert _rel(L1[i][k], L0[i][k]) < tS, ("Lr", k)
            assert _rel(K1[i][k], K0[i][k]) < tS and _rel(k1[i][k], k0[i][k]) < max(tS, 1e-8), ("K, k", k)


@pytest.mark.gpu
@pytest.mark.parametrize("projected", [True, False])
def test_device_riccati_feedback_equals_full(cm, op, projected):
    """cmpc_ocp_riccati_feedback_host (the MPC tick's getRiccatiFeedback part: K, Lr of every stage, P_1): copies of
    what a keep_riccati solve left — without rows the solve keeps its last factorisation only — equal to the full
    cmpc_ocp_riccati (which refactorises without rows) to rounding, and the same from a solve that kept nothing."""
    p = ocpgen.legged_problem(330, projected=projected)
    rec, crec = ocpgen.pack(p)
    res = []
    for keep in (1, 0):
        h = cm.OcpSolver(p["N"], p["nx"], p["nu"], p.get("nc"), max_batch=1)
        h.set_keep_riccati(keep)
        x, u, st, it = h.solve(p["x0"][None], rec[None], crec[None] if crec is not None else None)
        assert st[0] == 0
        fb = h.riccati_feedback(0)
        full = h.riccati(1)
        res.append((fb, full))
        h.close()
    tS = 1e-4 if not projected else 1e-9
    for (K, M, P1, s), (P, pv, Kf, kf, Mf, rst) in res:
        assert s == 0 and rst[0] == 0
        assert _rel(P1, P[0][1]) < tS
        for k in range(1, p["N"]):
            assert _rel(K[k], Kf[0][k]) < tS and _rel(M[k], Mf[0][k]) < tS, k
    (K1, M1, P11, _), _ = res[0]
    (K0, M0, P10, _), _ = res[1]
    assert _rel(P11, P10) < tS
    for k in range(p["N"]):
        assert _rel(K1[k], K0[k]) < tS and _rel(M1[k], M0[k]) < tS, k


@pytest.mark.gpu
def test_device_reshape_ticks_allocate_nothing(cm, op):
    """The MPC tick on one handle (HpipmInterface::resize + solve + getRiccatiFeedback, MultipleShootingSolver.cpp:276,
    :337-341): 50 ticks of the legged problem with the event nodes moving as the gait advances (N 70 / 71, the inputs
    per stage 10 / 12 / 0 shifting), reshaped on one handle with the exit Riccati kept: after the handle's first
    allocation no device or pinned allocation happens, and every tick's solution and Riccati quantities equal a fresh
    handle's bit for bit."""
    h = None
    base = None
    for t in range(50):
        p = ocpgen.legged_problem(700 + t, projected=True, t0=0.015 * t)
        rec, _ = ocpgen.pack(p)
        if h is None:
            h = cm.OcpSolver(p["N"], p["nx"], p["nu"], None, max_batch=1)
            h.set_keep_riccati(1)
            base = h.alloc_count
        else:
            h.reshape(p["N"], p["nx"], p["nu"])
        x, u, st, it = h.solve(p["x0"][None], rec[None])
        ric = h.riccati(1)
        assert h.alloc_count == base, (t, h.alloc_count, base)
        f = cm.OcpSolver(p["N"], p["nx"], p["nu"], None, max_batch=1)
        f.set_keep_riccati(1)
        xf, uf, stf, itf = f.solve(p["x0"][None], rec[None])
        rf = f.riccati(1)
        f.close()
        assert st[0] == 0 and stf[0] == 0 and it[0] == itf[0]
        assert np.array_equal(x, xf) and np.array_equal(u, uf), t
        assert np.array_equal(ric[0], rf[0]) and np.array_equal(ric[1], rf[1]), t
        for k in range(p["N"]):
            assert np.array_equal(ric[2][0][k], rf[2][0][k]) and np.array_equal(ric[3][0][k], rf[3][0][k]), (t, k)


@pytest.mark.gpu
def test_device_reshape_across_path_limits(cm, op):
    """One handle reshaped across the paths' dimension limits and back (latency form at nu_k + nx + 1 = 60, batched
    form at 61, the NZP = 128 class at 65, a one-stage horizon, the legged problem with rows): every solve equals a
    fresh handle's bit for bit, the path is the one the new dimensions select, and the results match the oracle."""
    shapes = [(dict(N=6, nx=24, nu=[35] * 6), 1), (dict(N=6, nx=24, nu=[36] * 6), 0),
              (dict(N=4, nx=20, nu=[44, 43, 44, 10]), 0), (dict(N=1, nx=3, nu=[2]), 1),
              (dict(N=6, nx=24, nu=[35] * 6, rows=False), 1)]
    h = None
    for t, (shape, chain) in enumerate(shapes + shapes[::-1]):
        ps = [_small(760 + 10 * t + i, **shape) for i in range(2)]
        recs, crecs = zip(*[ocpgen.pack(p) for p in ps])
        p0 = ps[0]
        crec = np.array(crecs) if p0.get("nc") else None
        if h is None:
            h = cm.OcpSolver(p0["N"], p0["nx"], p0["nu"], p0.get("nc"), max_batch=2)
        else:
            h.reshape(p0["N"], p0["nx"], p0["nu"], p0.get("nc"))
        x, u, st, it = h.solve(np.array([p["x0"] for p in ps]), np.array(recs), crec)
        assert h.path == chain, t
        f, xf, uf, stf, itf = _device_batch(cm, ps)
        f.close()
        assert np.array_equal(st, stf) and np.array_equal(it, itf), t
        for i in range(len(ps)):
            assert np.array_equal(x[i], xf[i]) and np.array_equal(u[i], uf[i]), (t, i)
        _check_vs_oracle(op, ps, x, u, st, it)
    h.close()
