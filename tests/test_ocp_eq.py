"""Equality-constrained OCP path: HpipmInterface::solve with constraints != nullptr.

The reference hands the rows C_k dx + D_k du + e_k = 0 to HPIPM as lg = ug = -e, with the stage-0 rows bounded through
x0 (ocs2_sqp/hpipm_catkin/src/HpipmInterface.cpp:223-264); MultipleShootingSolver::getOCPSolution takes that branch
whenever projection is off (ocs2_sqp/ocs2_sqp/src/MultipleShootingSolver.cpp:274-277). Its gtest
(testHpipmInterface.cpp:154-206, with_constraints) checks dynamics feasibility and the constraint rows at 1e-9 with
one node left empty.

Oracle: oracle/np_ref.py:ocp_eq_fullspace, a dense KKT solve in the full (x, u) space (no condensing, no Schur
complement), pinned here by (a) the reference test's own properties, (b) agreement with the C oracle's condensed
solve when there are no constraints, (c) the knownSolution construction (testHpipmInterface.cpp:112-152) with rows
that hold at the known solution. The device (cmpc_ocp_solve_batch_eq_host) must match it at 1e-9.
"""
import numpy as np
import pytest

import np_ref
from test_oracle import random_ocp


def _random_constraints(rng, N, nx, nu, nc):
    Cc, D, e = [], [], []
    for k in range(N + 1):
        m = nu[k] if k < N else 0
        Cc.append(rng.uniform(-1, 1, (nc[k], nx)))
        D.append(rng.uniform(-1, 1, (nc[k], m)))
        e.append(rng.uniform(-1, 1, nc[k]))
    return Cc, D, e


def _problem(seed, N=5, nx=3, nu=None, nc=None):
    rng = np.random.default_rng(seed)
    nu = nu or [2] * N
    nc = nc or [1, 0, 1, 1, 1, 1][: N + 1]
    A, B, b, Q, S, R, q, r = random_ocp(rng, N, nx, nu)
    Cc, D, e = _random_constraints(rng, N, nx, nu, nc)
    x0 = rng.uniform(-1, 1, nx)
    return dict(N=N, nx=nx, nu=nu, nc=nc, x0=x0, A=A, B=B, b=b, Q=Q, S=S, R=R, q=q, r=r, Cc=Cc, D=D, e=e)


def _full(p, with_con=True):
    kw = dict(Cc=p["Cc"], D=p["D"], e=p["e"]) if with_con else {}
    return np_ref.ocp_eq_fullspace(p["N"], p["nx"], p["nu"], p["x0"], p["A"], p["B"], p["b"], p["Q"], p["S"], p["R"],
                                   p["q"], p["r"], **kw)


def _check_reference_properties(p, x, u, tol=1e-9):
    """testHpipmInterface.cpp:192-205: x0, dynamics feasibility and the constraint rows (isApprox, relative)."""
    def approx(a, b):
        return np.linalg.norm(a - b) <= tol * min(np.linalg.norm(a), np.linalg.norm(b))
    assert approx(x[0], p["x0"])
    for k in range(p["N"]):
        assert approx(x[k + 1], p["A"][k] @ x[k] + p["B"][k] @ u[k] + p["b"][k])
    for k in range(p["N"] + 1):
        if p["nc"][k]:
            Du = p["D"][k] @ u[k] if k < p["N"] else 0.0
            assert approx(p["e"][k], -(p["Cc"][k] @ x[k] + Du))


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fullspace_oracle_has_reference_properties(seed):
    p = _problem(seed)
    x, u, res = _full(p)
    assert res < 1e-12
    _check_reference_properties(p, x, u)
    # the rows bind: the unconstrained optimum is a different point
    _, uu, _ = _full(p, with_con=False)
    assert max(np.abs(a - c).max() for a, c in zip(u, uu)) > 1e-6


def test_fullspace_oracle_matches_c_oracle_without_constraints(op):
    p = _problem(7)
    x, u, _ = _full(p, with_con=False)
    rec = op.ocp_pack(p["N"], p["nx"], p["nu"], p["A"], p["B"], p["b"], p["Q"], p["S"], p["R"], p["q"], p["r"])
    xc, uc, st = op.ocp_solve(p["N"], p["nx"], p["nu"], p["x0"], rec)
    assert st == 0
    assert np.abs(xc - x).max() < 1e-10
    assert np.abs(uc - np.concatenate(u)).max() < 1e-10


def _known_solution_problem(seed, N=5, nx=3):
    """knownSolution (testHpipmInterface.cpp:112-152) plus constraint rows that hold at the known solution: the
    unconstrained minimiser satisfies them, so it is the constrained minimiser too (multipliers 0)."""
    p = _problem(seed, N, nx)
    rng = np.random.default_rng(seed + 100)
    xs = [p["x0"]]
    us = []
    for k in range(N):
        us.append(rng.uniform(-1, 1, p["nu"][k]))
        xs.append(p["b"][k] + p["A"][k] @ xs[k] + p["B"][k] @ us[k])
        p["q"][k] = -(p["Q"][k] @ xs[k] + p["S"][k].T @ us[k])
        p["r"][k] = -(p["R"][k] @ us[k] + p["S"][k] @ xs[k])
    p["q"][N] = -p["Q"][N] @ xs[N]
    for k in range(N + 1):
        if p["nc"][k]:
            Du = p["D"][k] @ us[k] if k < N else 0.0
            p["e"][k] = -(p["Cc"][k] @ xs[k] + Du)
    return p, np.array(xs), us


def test_fullspace_oracle_known_solution():
    p, xs, us = _known_solution_problem(11)
    x, u, _ = _full(p)
    assert np.abs(x - xs).max() < 1e-9
    assert np.abs(np.concatenate(u) - np.concatenate(us)).max() < 1e-9


def _device(cm, op, ps):
    N, nx, nu, nc = ps[0]["N"], ps[0]["nx"], ps[0]["nu"], ps[0]["nc"]
    recs = np.array([op.ocp_pack(N, nx, nu, p["A"], p["B"], p["b"], p["Q"], p["S"], p["R"], p["q"], p["r"])
                     for p in ps])
    crecs = np.array([op.ocp_constraint_pack(N, nx, nu, nc, p["Cc"], p["D"], p["e"]) for p in ps])
    x0s = np.array([p["x0"] for p in ps])
    return cm.ocp_solve_eq(N, nx, nu, nc, x0s, recs, crecs)


@pytest.mark.gpu
def test_device_with_constraints_matches_fullspace(cm, op):
    """with_constraints shape (nc = 1 per node, node 1 empty, node N state-only) and a wider case (two rows at some
    nodes, a stage without inputs), batched: device vs the full-space oracle at 1e-9, plus the reference properties."""
    for shape in (dict(N=5, nx=3, nu=[2] * 5, nc=[1, 0, 1, 1, 1, 1]),
                  dict(N=6, nx=4, nu=[3, 0, 3, 2, 3, 3], nc=[2, 0, 1, 2, 0, 1, 2])):
        ps = [_problem(50 + i, **shape) for i in range(6)]
        x, u, st = _device(cm, op, ps)
        assert np.all(st == 0)
        for i, p in enumerate(ps):
            xr, ur, _ = _full(p)
            ur = np.concatenate(ur)
            assert np.abs(x[i] - xr).max() <= 1e-9 * max(1.0, np.abs(xr).max())
            assert np.abs(u[i] - ur).max() <= 1e-9 * max(1.0, np.abs(ur).max())
            offs = np.cumsum([0] + list(p["nu"]))
            _check_reference_properties(p, x[i], [u[i][offs[k]:offs[k + 1]] for k in range(p["N"])])


@pytest.mark.gpu
def test_device_known_solution_with_constraints(cm, op):
    p, xs, us = _known_solution_problem(12)
    x, u, st = _device(cm, op, [p])
    assert st[0] == 0
    assert np.abs(x[0] - xs).max() < 1e-9
    assert np.abs(u[0] - np.concatenate(us)).max() < 1e-9


@pytest.mark.gpu
def test_device_redundant_and_inconsistent_rows(cm, op):
    """A duplicated row: consistent -> SUCCESS with the single-row solution; contradictory -> MAX_ITER or MIN_STEP
    (HPIPM's OCP IPM treats the lg = ug rows as inequalities and runs out of iterations / steps on them)."""
    p = _problem(21)
    x1, u1, st1 = _device(cm, op, [p])
    q = dict(p)
    q["nc"] = list(p["nc"])
    q["nc"][2] = 2
    q["Cc"] = list(p["Cc"])
    q["D"] = list(p["D"])
    q["e"] = list(p["e"])
    q["Cc"][2] = np.vstack([p["Cc"][2], p["Cc"][2]])
    q["D"][2] = np.vstack([p["D"][2], p["D"][2]])
    q["e"][2] = np.concatenate([p["e"][2], p["e"][2]])
    x2, u2, st2 = _device(cm, op, [q])
    assert st1[0] == 0 and st2[0] == 0
    assert np.abs(u2 - u1).max() < 1e-8
    q["e"][2] = np.concatenate([p["e"][2], p["e"][2] + 1.0])
    _, _, st3 = _device(cm, op, [q])
    assert st3[0] in (1, 2)  # CMPC_MAX_ITER / CMPC_MIN_STEP


@pytest.mark.gpu
def test_device_eq_without_rows_equals_unconstrained(cm, op):
    """nc = 0 everywhere through the eq entry point is the plain solve."""
    p = _problem(31, nc=[0] * 6)
    x, u, st = _device(cm, op, [p])
    rec = op.ocp_pack(p["N"], p["nx"], p["nu"], p["A"], p["B"], p["b"], p["Q"], p["S"], p["R"], p["q"], p["r"])
    x2, u2, st2 = cm.ocp_solve(p["N"], p["nx"], p["nu"], p["x0"][None], rec[None])
    assert st[0] == 0 and st2[0] == 0
    assert np.array_equal(u, u2) and np.array_equal(x, x2)
