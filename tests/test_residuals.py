"""Solver statistics (cmpc_get_residuals): the final residual inf-norms per QP, mirroring the reference's reads of
d_ocp_qp_ipm_get_max_res_stat / _eq / _ineq / _comp after a solve (HpipmInterface.cpp:459-489). Each size class's
kernel (fused k_solve64 n <= 64, k_ipm128x, k_ipm_tiled n <= 256) is checked against the residuals the CPU oracle's
IPM (oracle/cmpc_oracle.c:qp_ipm_run, res[4]) reports for the same condensed QP, plus the stopping-rule semantics
(SUCCESS => every residual within its tolerance; MAX_ITER at a tiny iter_max => not) and NaN for QPs the IPM skipped.
Parity note: the oracle is this repo's restatement; HPIPM's own statistics are unpinned."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20221125
ABS = 1e-9  # residuals are differences of O(1e3) terms at iterates equal to ~1e-15 relative


def oracle_res(op, mo, so, x0, xref, foot, contact):
    out = []
    for q in range(x0.shape[0]):
        n, H, g, mu, lo, hi, _, st = op.condense(mo, x0[q], xref[q], foot[q], contact[q])
        assert st == 0
        _, _, _, s, it, res = op.qp_ipm(n, H, g, mu, lo, hi, so)
        out.append((s, it, res))
    return out


def check_against_oracle(eng, cm, op, N, B, contact_fn=None, gait=0, settings=None):
    m, mo = cm.default_model(N), op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=gait)
    if contact_fn is not None:
        contact[:] = contact_fn(contact)
    u, _, st, it = eng.solve(x0, xref, foot, contact, want_x=False)
    res = eng.residuals(B)
    so = settings or op.default_settings()
    ref = oracle_res(op, mo, so, x0, xref, foot, contact)
    for q in range(B):
        s, itr, rr = ref[q]
        assert st[q] == s, (q, st[q], s)
        assert abs(int(it[q]) - itr) <= 1, (q, it[q], itr)
        assert res[q, 1] == 0.0
        np.testing.assert_allclose(res[q], rr, rtol=1e-6, atol=ABS, err_msg=f"QP {q}")
    return res, st


def test_residuals_fused_class64_match_oracle(cm, op):
    N, B = 10, 16
    eng = cm.Engine(cm.default_model(N), precision=cm.F64, max_batch=B)
    assert cm.lib().cmpc_ctx_fused(eng.ctx) == 1
    res, st = check_against_oracle(eng, cm, op, N, B)
    s = cm.default_settings()
    ok = st == 0
    assert ok.all()
    assert np.all(res[ok, 0] <= s.tol_stat) and np.all(res[ok, 2] <= s.tol_ineq) and np.all(res[ok, 3] <= s.tol_comp)


def test_residuals_class128_and_256_match_oracle(cm, op):
    # N = 10 all-stance: n = 120 (k_ipm128x); N = 20 all-stance: n = 240 (k_ipm_tiled)
    for N, B in ((10, 6), (20, 2)):
        eng = cm.Engine(cm.default_model(N), precision=cm.F64, max_batch=B)
        res, st = check_against_oracle(eng, cm, op, N, B, contact_fn=lambda c: np.ones_like(c))
        assert np.all(st == 0)


def test_residuals_fused_equals_separate_launches(cm, op):
    N, B = 10, 64
    mo = op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=1)  # mixed gait: n <= 64 and 64 < n <= 128 QPs
    eng_f = cm.Engine(cm.default_model(N), precision=cm.F64, max_batch=B)
    eng_s = cm.Engine(cm.default_model(N), precision=cm.F64, max_batch=B, path={cm.PATH_FUSED64: 0})
    assert cm.lib().cmpc_ctx_fused(eng_f.ctx) == 1 and cm.lib().cmpc_ctx_fused(eng_s.ctx) == 0
    uf, _, sf, itf = eng_f.solve(x0, xref, foot, contact, want_x=False)
    rf = eng_f.residuals(B)
    us, _, ss, its = eng_s.solve(x0, xref, foot, contact, want_x=False)
    rs = eng_s.residuals(B)
    # the fused kernel runs the same condensing and IPM code: results are bit-identical
    assert np.array_equal(sf, ss) and np.array_equal(itf, its)
    assert np.array_equal(uf, us)
    assert np.array_equal(rf, rs)


def test_residuals_max_iter_and_skipped(cm, op):
    N, B = 10, 8
    s = cm.default_settings()
    s.iter_max = 2
    eng = cm.Engine(cm.default_model(N), settings=s, precision=cm.F64, max_batch=B)
    mo = op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=0)
    contact[3, 4, :] = 0  # a step without a stance leg: INVALID_CONTACT, the IPM never runs
    _, _, st, it = eng.solve(x0, xref, foot, contact, want_x=False)
    res = eng.residuals(B)
    assert st[3] == 5 and np.all(np.isnan(res[3]))
    run = np.arange(B) != 3
    assert np.all(st[run] == 1) and np.all(it[run] == 2)
    # stopped by the iteration cap: at least one residual above its tolerance for every such QP
    d = cm.default_settings()
    above = (res[run, 0] > d.tol_stat) | (res[run, 2] > d.tol_ineq) | (res[run, 3] > d.tol_comp)
    assert above.all(), res[run]


@pytest.mark.parametrize("feet", [False, True])
def test_residuals_after_sqp(cm, op, feet):
    """After cmpc_sqp_solve_batch / cmpc_nlp_solve_batch the residuals are those of each QP's last subproblem, also
    for QPs whose SQP converged early and were skipped by later iterations; NaN for a rejected contact table."""
    N, B = 10, 32
    m, mo = cm.default_model(N), op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=1)
    contact[5, 3, :] = 0  # "mpc table invalid"
    eng = cm.Engine(m, precision=0, max_batch=B)
    if feet:
        u, _, _, st, qi, si = eng.nlp_solve(x0, xref, foot, contact, sqp_iter_max=10, sqp_tol=1e-7)
    else:
        u, _, st, qi, si = eng.sqp_solve(x0, xref, foot, contact, sqp_iter_max=10, sqp_tol=1e-7)
    res = eng.residuals(B)
    s = cm.default_settings()
    assert st[5] == 5 and np.all(np.isnan(res[5]))
    ok = np.arange(B) != 5
    assert np.all(st[ok] == 0) and len(set(si[ok].tolist())) > 1  # QPs converge after different SQP iterations
    assert np.all(res[ok, 0] <= s.tol_stat) and np.all(res[ok, 2] <= s.tol_ineq) and np.all(res[ok, 3] <= s.tol_comp)
