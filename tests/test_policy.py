"""Feedback policy dU/dx0 of the condensed QP (SURVEY §8f rank 1 for the centroidal engine; the condensed counterpart
of HpipmInterface::getRiccatiFeedback, HpipmInterface.cpp:330-455, consumed as ocs2's feedback policy at
MultipleShootingSolver.cpp:334-362). The oracle (oracle_policy) is pinned here by central finite differences of its own
QP solution map (tight IPM tolerances), on batches with and without active pyramid / force-bound rows; the device
kernel (k_policy) is checked against the oracle fed the same solution u, so both see the same active set."""
import numpy as np
import pytest

SEED = 20221125


def _model(op, N, ub4=None):
    m = op.default_model(N)
    if ub4 is not None:
        m.force_ub[4] = ub4  # normal-force bound below m g / n_stance: upper rows become active
    return m


def _fd_policy(op, m, s, x0, xref, foot, contact, h=1e-4):
    X = np.repeat(x0[None], 26, 0)
    for j in range(13):
        X[2 * j, j] += h
        X[2 * j + 1, j] -= h
    R = lambda a: np.repeat(a[None], 26, 0)
    uu, _, st, _ = op.solve_batch(m, s, X, R(xref), R(foot), R(contact), nthreads=8, want_x=False)
    assert np.all(st == 0)
    return np.moveaxis((uu[0::2] - uu[1::2]) / (2 * h), 0, -1)  # [N, L, 3, 13]


@pytest.mark.parametrize("N,gait,ub4,nfree_lt_n", [(10, 0, None, False), (10, 1, None, False), (10, 1, 15.0, True),
                                                    (20, 0, 15.0, True)])
def test_oracle_policy_matches_finite_differences(op, N, gait, ub4, nfree_lt_n):
    m = _model(op, N, ub4)
    s = op.tight_settings()
    x0, xref, foot, contact = op.generate(m, SEED, 3, gait=gait)
    u, _, st, _ = op.solve_batch(m, s, x0, xref, foot, contact, nthreads=8, want_x=False)
    assert np.all(st == 0)
    for q in range(3):
        K, nfree, pst = op.policy(m, xref[q], foot[q], contact[q], u[q])
        assert pst == 0
        n = 3 * int(contact[q].sum())
        assert (nfree < n) == nfree_lt_n
        fd = _fd_policy(op, m, s, x0[q], xref[q], foot[q], contact[q])
        assert np.abs(fd - K).max() / max(1.0, np.abs(K).max()) < 1e-7
        # swing rows are exactly zero
        assert np.all(K[contact[q] == 0] == 0.0)


def test_oracle_policy_triple_free_directions(op):
    mu, ub = 0.8, np.array([5000.0] * 4 + [50.0])
    tol = 1e-6
    # interior: all three directions free
    Z = op.policy_triple(mu, ub, np.array([1.0, -2.0, 20.0]), tol)
    assert Z.shape == (3, 3) and np.allclose(Z.T @ Z, np.eye(3))
    # zero force: all five lower rows active (rank 3), nothing free
    assert op.policy_triple(mu, ub, np.zeros(3), tol).shape == (3, 0)
    # on facet 0 (mu fz - fx = 0): two free directions orthogonal to its normal
    Z = op.policy_triple(mu, ub, np.array([8.0, 1.0, 10.0]), tol)
    assert Z.shape == (3, 2) and np.allclose(np.array([-1.0, 0.0, mu]) @ Z, 0.0)
    # edge of facets 0 and 2: one free direction along (mu, mu, 1)
    Z = op.policy_triple(mu, ub, np.array([8.0, 8.0, 10.0]), tol)
    d = np.array([mu, mu, 1.0]) / np.linalg.norm([mu, mu, 1.0])
    assert Z.shape == (3, 1) and np.isclose(abs(float(d @ Z[:, 0])), 1.0)
    # normal-force upper bound: fz fixed, fx / fy free
    Z = op.policy_triple(mu, ub, np.array([1.0, 1.0, 50.0]), tol)
    assert Z.shape == (3, 2) and np.allclose(Z[2], 0.0)


def test_oracle_policy_is_linear_response(op):
    """On a fixed active set the solution is affine in x0: u(x0 + d) - u(x0) = K d for a small d."""
    m = _model(op, 10, 15.0)
    s = op.tight_settings()
    x0, xref, foot, contact = op.generate(m, SEED + 7, 2, gait=1)
    u, _, _, _ = op.solve_batch(m, s, x0, xref, foot, contact, nthreads=4, want_x=False)
    d = 1e-3 * np.random.default_rng(0).standard_normal(x0.shape)
    d[:, 12] = 0.0
    u2, _, _, _ = op.solve_batch(m, s, x0 + d, xref, foot, contact, nthreads=4, want_x=False)
    for q in range(2):
        K, _, _ = op.policy(m, xref[q], foot[q], contact[q], u[q])
        assert np.abs(u2[q] - u[q] - K @ d[q]).max() < 1e-7 * max(1.0, np.abs(K).max())


def _device_vs_oracle(cm, op, N, gait, ub4, B, precision, all_stance=False):
    m = cm.default_model(N)
    mo = _model(op, N, ub4)
    if ub4 is not None:
        m.force_ub[4] = ub4
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=gait)
    if all_stance:
        contact[:] = 1
    settings = (cm.default_settings() if precision == 0 else
                cm.default_settings(tol_stat=1e-3, tol_ineq=1e-3, tol_comp=1e-4))  # fp32 settings of bench.py
    eng = cm.Engine(m, settings=settings, precision=precision, max_batch=B)
    u, _, st, _ = eng.solve(x0, xref, foot, contact, want_x=False)
    assert np.all(st == 0)
    K, nfree, pst = eng.policy(x0, xref, foot, contact, u)
    assert np.all(pst == 0)
    tol = 1e-5 if precision == 0 else 2e-3
    worst = 0.0
    for q in range(B):
        Kr, nfr, sr = op.policy(mo, xref[q], foot[q], contact[q], u[q], 1e-5 if precision == 0 else 2e-3)
        assert sr == 0 and nfr == nfree[q]
        worst = max(worst, float(np.abs(K[q] - Kr).max() / max(1.0, np.abs(Kr).max())))
    assert worst < (1e-9 if precision == 0 else tol), worst
    return nfree


@pytest.mark.gpu
@pytest.mark.parametrize("N,gait,ub4,B,all_stance", [(10, 0, None, 64, False), (10, 0, 15.0, 32, True),
                                                      (10, 1, 15.0, 48, False), (20, 0, 15.0, 16, False),
                                                      (20, 0, None, 8, True)])
def test_device_policy_matches_oracle_fp64(cm, op, N, gait, ub4, B, all_stance):
    """Class 64 (trot N=10), 128 (all-stance N=10 / trot N=20), 256 (all-stance N=20); mixed gaits; active bounds."""
    nfree = _device_vs_oracle(cm, op, N, gait, ub4, B, 0, all_stance)
    if ub4 is not None:
        assert nfree.max() > 0


@pytest.mark.gpu
def test_device_policy_fp32(cm, op):
    _device_vs_oracle(cm, op, 20, 0, None, 16, 1)


@pytest.mark.gpu
def test_device_policy_invalid_contact(cm, op):
    N, B = 10, 4
    m, mo = cm.default_model(N), op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=0)
    u, _, _, _ = op.solve_batch(mo, op.default_settings(), x0, xref, foot, contact, nthreads=4, want_x=False)
    contact[1, 3, :] = 0  # a step with no stance leg ("mpc table invalid", CentroidalMPC.cpp:328-330)
    eng = cm.Engine(m, precision=0, max_batch=B)
    K, nfree, st = eng.policy(x0, xref, foot, contact, u)
    assert st[1] == 5 and nfree[1] == 0 and np.all(K[1] == 0.0)
    assert st[0] == 0 and st[2] == 0 and nfree[0] > 0


@pytest.mark.parametrize("N,gait", [(10, 0), (10, 1), (20, 0)])
def test_oracle_policy_equals_riccati_feedback_when_unconstrained(op, N, gait):
    """SURVEY §8c property: the condensed solution's sensitivity equals the Riccati u = K x + k of the OCP form.
    On QPs with no active row (every slack >= 1 at the default bounds) the condensed policy's step-0 rows equal the
    stage-0 Riccati feedback (HpipmInterface::getRiccatiFeedback(0), HpipmInterface.cpp:330-455) of the
    unconstrained OCP."""
    m = op.default_model(N)
    x0, xref, foot, contact = op.generate(m, SEED, 4, gait=gait)
    u, _, st, _ = op.solve_batch(m, op.default_settings(), x0, xref, foot, contact, nthreads=4, want_x=False)
    for q in range(4):
        K, nfree, pst = op.policy(m, xref[q], foot[q], contact[q], u[q])
        assert pst == 0 and nfree == 3 * int(contact[q].sum())  # nothing active
        K0, rst = op.riccati_gain0(m, xref[q], foot[q], contact[q])
        assert rst == 0
        assert np.abs(K[0] - K0).max() / max(1.0, np.abs(K0).max()) < 1e-9


@pytest.mark.parametrize("ub4", [None, 15.0])
def test_oracle_policy_at_sqp_linearisation_matches_finite_differences(op, ub4):
    """The feedback of the QP linearised at the SQP solution (oracle_policy_lin): central differences of that QP's
    solution map in x0 with the linearisation point held fixed, as HPIPM's factorisation of the last QP is."""
    N = 10
    m = _model(op, N, ub4)
    s = op.tight_settings()
    x0, xref, foot, contact = op.generate(m, SEED + 3, 2, gait=1)
    for q in range(2):
        u = op.sqp_solve(m, s, x0[q], xref[q], foot[q], contact[q], sqp_iter_max=20, sqp_tol=1e-10)[0]
        lin = op.nlp_rollout_cost(m, x0[q], xref[q], foot[q], contact[q], u)[2]
        uq, st, _ = op.solve_one_lin(m, s, x0[q], xref[q], foot[q], contact[q], lin)
        assert st == 0
        K, nfree, pst = op.policy(m, xref[q], foot[q], contact[q], uq, lin=lin)
        assert pst == 0
        h = 1e-4
        fd = np.zeros_like(K)
        for j in range(12):
            dp, dm = x0[q].copy(), x0[q].copy()
            dp[j] += h
            dm[j] -= h
            up = op.solve_one_lin(m, s, dp, xref[q], foot[q], contact[q], lin)[0]
            um = op.solve_one_lin(m, s, dm, xref[q], foot[q], contact[q], lin)[0]
            fd[..., j] = (up - um) / (2 * h)
        assert np.abs(fd[..., :12] - K[..., :12]).max() / max(1.0, np.abs(K).max()) < 1e-6
        # differs from the policy of the reference-linearised QP
        K0 = op.policy(m, xref[q], foot[q], contact[q], uq)[0]
        assert np.abs(K - K0).max() > 1e-6 * max(1.0, np.abs(K).max())


@pytest.mark.gpu
@pytest.mark.parametrize("N,gait,ub4", [(10, 1, 15.0), (20, 0, None)])
def test_device_sqp_policy_matches_oracle(cm, op, N, gait, ub4):
    """cmpc_sqp_policy_batch at the device SQP's solution against oracle_policy_lin at the same u, linearised at its
    nonlinear rollout (classes 64 / 128 at N = 10 mixed, 128 at N = 20)."""
    B = 16
    m, mo = cm.default_model(N), _model(op, N, ub4)
    if ub4 is not None:
        m.force_ub[4] = ub4
    x0, xref, foot, contact = op.generate(mo, SEED + 5, B, gait=gait)
    eng = cm.Engine(m, precision=0, max_batch=B)
    u, _, st, _, _ = eng.sqp_solve(x0, xref, foot, contact, sqp_iter_max=10, sqp_tol=1e-7, want_x=False)
    assert np.all(st == 0)
    K, nfree, pst = eng.sqp_policy(x0, xref, foot, contact, u)
    K0 = eng.policy(x0, xref, foot, contact, u)[0]
    for q in range(B):
        lin = op.nlp_rollout_cost(mo, x0[q], xref[q], foot[q], contact[q], u[q])[2]
        Kr, nfr, sr = op.policy(mo, xref[q], foot[q], contact[q], u[q], lin=lin)
        assert pst[q] == sr == 0 and nfree[q] == nfr
        assert np.abs(K[q] - Kr).max() / max(1.0, np.abs(Kr).max()) < 1e-9, q
    assert np.abs(K - K0).max() > 1e-6  # not the reference-linearised QP's policy
