"""Stage-wise (Riccati) form of the hot path (k_ric.hpp, CMPC_PATH_RICCATI) against the CPU oracle.

The kernel solves the same QP as the condensed path with the IPM iteration of oracle_qp_ipm, but its
Newton systems go through a Riccati recursion over the stages (HPIPM's method for the reference's OCP,
HpipmInterface.cpp:282-284) instead of a dense factorisation of the condensed H; oracle_riccati_solve_one is the CPU
restatement of that structure. Bars as the condensed path's: statuses equal, iterations within 1, forces within 1e-8
relative (fp64) / 2e-3 (fp32, tolerances of the fp32 settings) of the fp64 oracle."""
import numpy as np
import pytest

SEED = 20221125


def _settings(cm, precision):
    return cm.default_settings() if precision == 0 else cm.default_settings(tol_stat=1e-3, tol_ineq=1e-3, tol_comp=1e-4)


def _solve(cm, N, B, gait, precision, ric, seed=SEED, fused=None):
    m = cm.default_model(N)
    path = {cm.PATH_RICCATI: ric}
    if fused is not None:
        path[cm.PATH_FUSED64] = fused
    eng = cm.Engine(m, settings=_settings(cm, precision), precision=precision, max_batch=B, path=path)
    x0, xref, foot, contact = cm.generate_device(m, seed, B, gait=gait)
    u = cm.DeviceArray((B, N, 4, 3), np.float64)
    st = cm.DeviceArray((B,), np.int32)
    it = cm.DeviceArray((B,), np.int32)
    eng.solve_device(B, x0, xref, foot, contact, u, None, st, it)
    cm.hip().hipDeviceSynchronize()
    return (x0.host(), xref.host(), foot.host(), contact.host()), u.host(), st.host(), it.host(), eng


@pytest.mark.gpu
@pytest.mark.parametrize("N,gait,precision,ric", [(10, 0, 0, 2), (10, 1, 0, 2), (10, 1, 0, 1), (6, 1, 0, 2),
                                                   (16, 1, 0, 2), (20, 1, 0, 2), (20, 1, 0, 1), (20, 0, 1, 2),
                                                   (20, 0, 1, 1), (10, 1, 1, 2)])
def test_ric_matches_oracle(cm, op, N, gait, precision, ric):
    B = 96
    inputs, u, st, it, _ = _solve(cm, N, B, gait, precision, ric)
    mo = op.default_model(N)
    so = op.default_settings() if precision == 0 else op.tight_settings()
    ur, _, sr, itr = op.solve_batch(mo, so, *inputs, nthreads=8, want_x=False)
    assert np.array_equal(st, sr)
    err = np.abs(u - ur).reshape(B, -1).max(1) / np.maximum(1.0, np.abs(ur).reshape(B, -1).max(1))
    assert err.max() < (1e-8 if precision == 0 else 2e-3), err.max()
    assert np.all(u[inputs[3] == 0] == 0.0)
    if precision == 0:
        assert np.abs(it - itr).max() <= 1


@pytest.mark.gpu
@pytest.mark.parametrize("N,gait,precision", [(10, 0, 0), (10, 1, 0), (20, 0, 1)])
def test_ric_full_batch_equals_condensed(cm, N, gait, precision):
    """Configs 2, 5 and 3 at B = 4096: the stage-wise path (every QP, and the bigger classes only) agrees with the
    condensed path to rounding on every QP."""
    B = 4096
    _, u0, s0, i0, _ = _solve(cm, N, B, gait, precision, 0)
    for ric in (1, 2):
        _, u1, s1, i1, _ = _solve(cm, N, B, gait, precision, ric)
        assert np.array_equal(s0, s1)
        err = np.abs(u1 - u0).reshape(B, -1).max(1) / np.maximum(1.0, np.abs(u0).reshape(B, -1).max(1))
        assert err.max() < (1e-9 if precision == 0 else 2e-3), (ric, err.max())
        if precision == 0:
            assert np.abs(i1 - i0).max() <= 1


@pytest.mark.gpu
def test_ric_rejects_invalid_contact_and_rollout(cm, op):
    """A step without a stance leg is INVALID_CONTACT with zero forces (CentroidalMPC.cpp:328-330); with a rollout
    requested the results go through the scatter kernel (condensed-order u, tri_map, nvar written by k_ric)."""
    N, B = 10, 8
    m = cm.default_model(N)
    eng = cm.Engine(m, precision=0, max_batch=B, path={cm.PATH_RICCATI: 2})
    x0, xref, foot, contact = (a.host() for a in cm.generate_device(m, SEED, B, gait=1))
    contact[3, 4] = 0
    u, x, st, it = eng.solve(x0, xref, foot, contact, want_x=True)
    ur, xr, sr, _ = op.solve_batch(op.default_model(N), op.default_settings(), x0, xref, foot, contact, nthreads=4)
    assert st[3] == 5 and np.all(u[3] == 0.0)
    assert np.array_equal(st, sr)
    ok = sr == 0
    assert np.abs(u[ok] - ur[ok]).max() / max(1.0, np.abs(ur[ok]).max()) < 1e-8
    assert np.abs(x[ok] - xr[ok]).max() / max(1.0, np.abs(xr[ok]).max()) < 1e-8


@pytest.mark.gpu
def test_ric_residuals_and_stats(cm, op):
    """Final residuals (cmpc_get_residuals) and the per-iteration statistics rows of the stage-wise kernel against
    the oracle IPM's (res of oracle_qp_ipm, stat table of oracle_qp_ipm_stats), as for the condensed classes."""
    N, B = 10, 16
    m = cm.default_model(N)
    eng = cm.Engine(m, precision=0, max_batch=B, path={cm.PATH_RICCATI: 2})
    eng.enable_stats(32)
    x0, xref, foot, contact = (a.host() for a in cm.generate_device(m, SEED, B, gait=1))
    u, _, st, it = eng.solve(x0, xref, foot, contact, want_x=False)
    res = eng.residuals(B)
    stats = eng.stats(B)
    mo = op.default_model(N)
    for q in range(B):
        n, H, g, mu, lo, hi, mp, cst = op.condense(mo, x0[q], xref[q], foot[q], contact[q])
        uo, sto, ito, reso, tab = op.qp_ipm_stats(n, H, g, mu, lo, hi, op.default_settings(), 32)
        assert sto == st[q] and ito == it[q]
        assert np.allclose(res[q], reso, rtol=1e-6, atol=1e-9)
        rows = ito + 1
        assert np.allclose(stats[q, :rows, 5:], tab[:rows, 5:], rtol=1e-6, atol=1e-9, equal_nan=True)
