"""The partitioned (parallel-in-time) Riccati factorisation of the grid form (csrc/ocp_part.hpp) on the
HpipmInterface::solve path (reference HpipmInterface.cpp:282-284: HPIPM's backward Riccati recursion, restated serially
by oracle/ocp_ipm.c). The horizon is split into S segments: the middle ones factorised from a zero end value and
summarised by (Phi, f, W), the exact boundary values combined backward, every segment refactorised from its exact end
value. The factorisation is the serial chain's up to rounding, so the solve must keep the oracle's statuses and
iteration counts and its x / u at 1e-9, for S = 1 (the serial chain), 2 (no combine), 8 and the automatic S; the kept
Riccati quantities (cmpc_ocp_set_keep_riccati) equal the refactorisation of the one-workgroup form. A stage whose
input Hessian is singular without the future's cost (R = 0, reg_prim = 0) makes the first pass drop a pivot: the
factorisation then falls back to the serial chain, as does a combine that would cancel more than 5 digits (unstable
segments). The serial vector recursions (the rollout, the corrector's cost-to-go) run as a partitioned affine scan over
the same segments (compositions, boundary values, the segments' own steps)."""
import numpy as np
import pytest

from cheeta_mpc import ocp as ocpgen
from test_ocp_ipm import _check_vs_oracle, _device_batch_path, _rel, _small

pytestmark = pytest.mark.gpu


def _seg_begin(N, S, s):
    """Segment boundary c_s of csrc/ocp_part.hpp:seg_begin (segment 0 weighs 1/2, the last one 5/2)."""
    if s <= 0:
        return 0
    if s >= S:
        return N
    return min(max(N * (10 * s - 5) // (10 * S + 10), s), N - (S - s))


def _solve(h, ps):
    recs, crecs = zip(*[ocpgen.pack(p) for p in ps])
    return h.solve(np.array([p["x0"] for p in ps]), np.array(recs), np.array(crecs) if ps[0].get("nc") else None)


@pytest.mark.parametrize("projected", [True, False])
def test_device_partitioned_factorisation_matches_oracle(cm, op, projected):
    ps = [ocpgen.legged_problem(580 + i, projected=projected) for i in range(2)]
    p0 = ps[0]
    s1, x1, u1, st1, it1 = _device_batch_path(cm, ps, 1, grid=1)
    ric1 = s1.riccati(2)
    rows = p0.get("nc") is not None
    tS = 1e-4 if rows else 1e-9
    for S in (1, 2, 8, 0):
        h = cm.OcpSolver(p0["N"], p0["nx"], p0["nu"], p0.get("nc"), max_batch=2)
        h.set_segments(S)
        h.set_keep_riccati(1)
        want = S if S else int(np.sqrt((2.0 if rows else 1.0) * p0["N"]) + 0.5)
        assert h.segments(2) == min(want, h.grid(2)), S
        x, u, st, it = _solve(h, ps)
        assert np.array_equal(st, st1) and np.array_equal(it, it1), S
        _check_vs_oracle(op, ps, x, u, st, it)
        for i in range(2):
            assert _rel(x[i], x1[i]) < 1e-9 and _rel(u[i], u1[i]) < 1e-9, (S, i, _rel(x[i], x1[i]), _rel(u[i], u1[i]))
        P, pv, K, kf, Lr, rst = h.riccati(2)
        assert np.all(rst == 0)
        for i in range(2):
            for k in range(1, p0["N"] + 1):
                assert _rel(P[i][k], ric1[0][i][k]) < tS, (S, "P", k, _rel(P[i][k], ric1[0][i][k]))
            for k in range(1, p0["N"]):
                assert _rel(K[i][k], ric1[2][i][k]) < tS, (S, "K", k)
                assert _rel(Lr[i][k], ric1[4][i][k]) < tS, (S, "Lr", k)
        assert h.fallback_count == 0
        assert h.partition_fallbacks == 0, S  # the partitioned form ran (no serial-chain fallback)
        h.close()


@pytest.mark.parametrize("S", [2, 3, 5])
def test_device_partitioned_small_shapes(cm, op, S):
    """Short horizons (N = 5, nx = 3, rows and mixed nu with a zero-input stage) down to one-stage segments."""
    for shape in (dict(N=5, nx=3), dict(N=6, nx=4, nu=[3, 0, 3, 2, 3, 3], nc=[2, 0, 1, 2, 0, 1, 2]),
                  dict(N=5, nx=3, nu=[2, 0, 2, 2, 2], rows=False)):
        ps = [_small(860 + i, **shape) for i in range(3)]
        p0 = ps[0]
        h = cm.OcpSolver(p0["N"], p0["nx"], p0["nu"], p0.get("nc"), max_batch=3)
        h.set_segments(S)
        assert h.segments(3) == min(S, p0["N"])
        x, u, st, it = _solve(h, ps)
        _check_vs_oracle(op, ps, x, u, st, it)
        h.close()


def test_device_partitioned_dropped_pivot_falls_back_to_the_serial_chain(cm, op):
    """R_k = 0 at the last stage of a middle segment with reg_prim = 0: the first pass (zero end value) meets M^0_uu = 0 there and the guard
    drops the pivot, so the partitioned factorisation falls back to the serial chain (counted): the result equals
    S = 1's to rounding (the rollouts stay partitioned) and the oracle's."""
    p = ocpgen.legged_problem(590, projected=True)
    N = p["N"]
    # the last stage of a middle segment (S = 8): its first-pass end value is 0, so M^0_uu = R_k = 0 there
    k = next(_seg_begin(N, 8, s + 1) - 1 for s in (4, 3, 5, 2, 1) if p["nu"][_seg_begin(N, 8, s + 1) - 1] > 0)
    p["R"][k] = np.zeros_like(p["R"][k])
    p["S"][k] = np.zeros_like(p["S"][k])
    p["r"][k] = np.zeros_like(p["r"][k])
    s = cm.default_settings()
    s.reg_prim = 0.0
    out = []
    for S in (1, 8):
        h = cm.OcpSolver(N, p["nx"], p["nu"], None, settings=s, max_batch=1)
        h.set_segments(S)
        out.append(_solve(h, [p]))
        if S == 8:
            assert h.partition_fallbacks >= 1
        h.close()
    (x1, u1, st1, it1), (x8, u8, st8, it8) = out
    assert np.array_equal(st1, st8) and np.array_equal(it1, it8)
    assert _rel(x8, x1) < 1e-9 and _rel(u8, u1) < 1e-9
    _check_vs_oracle(op, [p], x8, u8, st8, it8, settings=op.default_settings(reg_prim=0.0))


def test_device_partitioned_unstable_segments_fall_back_to_the_serial_chain(cm, op):
    """Strongly unstable dynamics (A scaled by 3: a 9-stage segment amplifies by ~2e4): the combine's Woodbury form
    P_a = D - C'N^-1 C would subtract two terms 1e5+ times larger than P_a (D = P^0_a + Phi'P_b Phi), so the
    cancellation guard refuses it and the factorisation runs on the serial chain (counted): S = 1's result to
    rounding, the oracle's at its tolerance."""
    p = ocpgen.legged_problem(592, projected=True)
    p["A"] = [3.0 * np.asarray(a) for a in p["A"]]
    out = []
    for S in (1, 8):
        h = cm.OcpSolver(p["N"], p["nx"], p["nu"], None, max_batch=1)
        h.set_segments(S)
        out.append(_solve(h, [p]))
        if S == 8:
            assert h.partition_fallbacks >= 1
        h.close()
    (x1, u1, st1, it1), (x8, u8, st8, it8) = out
    assert np.array_equal(st1, st8) and np.array_equal(it1, it8)
    assert _rel(x8, x1) < 1e-9 and _rel(u8, u1) < 1e-9
    _check_vs_oracle(op, [p], x8, u8, st8, it8)


@pytest.mark.parametrize("grid", [0, 1])
def test_device_linres_statistics(cm, op, grid):
    """cmpc_ocp_set_linres: per iteration the residuals of the Newton system at the final direction (HPIPM's lin res
    stat / eq / ineq / comp columns, HpipmInterface.cpp:492-501), in the grid form and the one-workgroup form: finite
    and at rounding level (relative to the iteration's own residuals) for every iteration that computed a direction,
    NaN for the exit row and after it; the solve's result the same to rounding (the recording solve runs the batched
    form's factorisation: same iterations and statuses, x and u at 1e-10)."""
    ps = [ocpgen.legged_problem(595 + i, projected=False) for i in range(2)]
    p0 = ps[0]
    h = cm.OcpSolver(p0["N"], p0["nx"], p0["nu"], p0.get("nc"), max_batch=2)
    h.set_grid(grid)
    x0, u0, st0, it0 = _solve(h, ps)
    h.set_linres(1)
    x, u, st, it = _solve(h, ps)
    assert np.array_equal(it, it0) and np.array_equal(st, st0)
    assert _rel(x, x0) < 1e-10 and _rel(u, u0) < 1e-10
    lr = h.linres(2)
    stats = h.stats(2)
    for i in range(2):
        n = it[i]
        assert np.all(np.isfinite(lr[i][:n])), lr[i][:n]
        assert np.all(np.isnan(lr[i][n:]))
        scale = np.maximum(1.0, np.nanmax(stats[i][:n, 6:10], axis=1))
        assert np.all(lr[i][:n].max(axis=1) <= 1e-6 * scale), (lr[i][:n], scale)
    h.close()
