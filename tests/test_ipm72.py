"""The 64 < n <= 72 class on one wave (k_ipm72.hpp: the bordered Newton system through the Schur complement of its
64 x 64 block) against the oracle's IPM (oracle_qp_ipm: Cholesky of the whole Newton matrix) and against the
four-wave 128 class it replaces (CMPC_PATH_IPM72 = 0), n = 66 / 69 / 72 (border of 2 / 5 / 8 variables).
Results agree to rounding (different factorisations of the same Newton systems); statuses and iteration counts are
equal."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20221125


def rel_err(u, ur):
    return np.abs(u - ur).max() / max(1.0, np.abs(ur).max())


def contact_with(N, B, n_triples, rng):
    """Contact tables with exactly n_triples stance legs, at least one per step (a step without one is
    INVALID_CONTACT, CentroidalMPC.cpp:328-330)."""
    c = np.zeros((B, N, 4), np.uint8)
    for q in range(B):
        c[q, np.arange(N), rng.integers(0, 4, size=N)] = 1
        free = np.flatnonzero(c[q].reshape(-1) == 0)
        c[q].reshape(-1)[rng.choice(free, size=n_triples[q] - N, replace=False)] = 1
    return c


def test_qp_hook_bordered_class_matches_oracle(cm, op):
    N, B = 6, 12
    m, mo = cm.default_model(N), op.default_model(N)
    rng = np.random.default_rng(7)
    x0, xref, foot, _ = op.generate(mo, SEED, B, gait=0)
    contact = contact_with(N, B, [22, 23, 24] * 4, rng)
    engs = {v: cm.Engine(m, precision=0, max_batch=B, path={cm.PATH_IPM72: v}) for v in (1, 0)}
    ld = engs[1].ld
    assert ld == 128
    Hs, gs, ns, mus, los, his, refs = [], [], [], [], [], [], []
    for q in range(B):
        n, H, g, mu, lo, hi, mp, st = op.condense(mo, x0[q], xref[q], foot[q], contact[q], ld=ld)
        assert 64 < n <= 72
        Hs.append(H); gs.append(g); ns.append(n); mus.append(mu); los.append(lo); his.append(hi)
        refs.append(op.qp_ipm(n, H, g, mu, lo, hi, op.default_settings()))
    out = {v: e.qp_solve(np.array(Hs), np.array(gs), np.array(ns, np.int32), np.array(mus), np.array(los),
                         np.array(his)) for v, e in engs.items()}
    for q in range(B):
        ur, st_r, it_r = refs[q][0], refs[q][3], refs[q][4]
        for v, (u, st, it) in out.items():
            assert st[q] == st_r == 0, (v, q)
            assert it[q] == it_r, (v, q, it[q], it_r)
            assert rel_err(u[q, :ns[q]], ur) < 1e-9, (v, q)
            assert np.all(u[q, ns[q]:] == 0)


@pytest.mark.parametrize("warm", [0, 1])
def test_solve_bordered_class_matches_oracle(cm, op, warm):
    """cmpc_solve_batch with separate IPM launches (CMPC_PATH_FUSED64 = 0), cold and warm, n = 66 / 69 / 72."""
    N, B = 6, 12
    m, mo = cm.default_model(N), op.default_model(N)
    rng = np.random.default_rng(11)
    x0, xref, foot, _ = op.generate(mo, SEED, B, gait=0)
    contact = contact_with(N, B, [22, 23, 24] * 4, rng)
    s = cm.default_settings(warm_start=warm)
    so = op.default_settings(warm_start=warm)
    u0 = None
    if warm:
        u0 = op.solve_batch(mo, so, x0, xref, foot, contact, want_x=False, u_init=np.zeros((B, N, 4, 3)))[0]
        u0 = u0 + 0.5 * rng.standard_normal(u0.shape) * (contact[..., None] > 0)
    ur, _, st_r, it_r = op.solve_batch(mo, so, x0, xref, foot, contact, want_x=False, u_init=u0)
    for v in (1, 0):
        eng = cm.Engine(m, s, precision=0, max_batch=B, path={cm.PATH_FUSED64: 0, cm.PATH_IPM72: v})
        u, _, st, it = eng.solve(x0, xref, foot, contact, want_x=False, u_init=u0)
        assert np.array_equal(st, st_r) and np.all(st == 0), v
        assert np.array_equal(it, it_r), (v, it, it_r)
        for q in range(B):
            assert rel_err(u[q], ur[q]) < 1e-9, (v, q)


@pytest.mark.parametrize("prec", [0, 1])
def test_nlp_bordered_class_matches_128_class(cm, op, prec):
    """The NLP's trot subproblems (n = 66 / 72) on k_ipm72 and on the 128 class: the same SQP."""
    N, B = 10, 64
    m, mo = cm.default_model(N), op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=0)
    settings = cm.default_settings() if prec == 0 else cm.default_settings(tol_stat=1e-3, tol_ineq=1e-3,
                                                                           tol_comp=1e-4)
    res = {}
    for v in (1, 0):
        eng = cm.Engine(m, settings, precision=prec, max_batch=B, path={cm.PATH_IPM72: v})
        res[v] = eng.nlp_solve(x0, xref, foot, contact, sqp_iter_max=10, sqp_tol=1e-7, want_x=False)
    (u1, f1, _, s1, q1, i1), (u0, f0, _, s0, q0, i0) = res[1], res[0]
    assert np.all(s1 == 0) and np.array_equal(s1, s0)
    tol = 1e-8 if prec == 0 else 2e-3
    for q in range(B):
        assert rel_err(u1[q], u0[q]) < tol, q
        assert np.abs(f1[q] - f0[q]).max() < tol, q
    if prec == 0:
        assert np.array_equal(i1, i0)
        assert np.abs(q1.astype(int) - q0.astype(int)).max() <= 1


def test_every_class_in_one_batch(cm, op):
    """One N = 20 batch with n = 60 / 66 / 69 / 72 / 120 / 240 through the separate IPM launches (k_class_lists with
    the 128 class split at 72: lists 0..3 at once, k_ipm64 / k_ipm72 / k_ipm128x / k_ipm_tiled), against the oracle."""
    N = 20
    m, mo = cm.default_model(N), op.default_model(N)
    rng = np.random.default_rng(5)
    sizes = [20, 22, 23, 24, 40, 80] * 3
    B = len(sizes)
    x0, xref, foot, _ = op.generate(mo, SEED, B, gait=0)
    contact = contact_with(N, B, sizes, rng)
    ur, _, st_r, it_r = op.solve_batch(mo, op.default_settings(), x0, xref, foot, contact, want_x=False)
    eng = cm.Engine(m, precision=0, max_batch=B, path={cm.PATH_FUSED64: 0})
    assert eng.ld == 256
    u, _, st, it = eng.solve(x0, xref, foot, contact, want_x=False)
    assert np.array_equal(st, st_r) and np.all(st == 0), (st, st_r)
    assert np.array_equal(it, it_r), (it, it_r)
    for q in range(B):
        assert rel_err(u[q], ur[q]) < 1e-8, q


def test_bordered_class_non_finite_input(cm, op):
    """A NaN in the gradient of an n = 66 / 72 QP gives the oracle's status (NAN_SOL) on both kernels; its neighbours
    in the batch are unaffected."""
    N, B = 6, 6
    m, mo = cm.default_model(N), op.default_model(N)
    rng = np.random.default_rng(3)
    x0, xref, foot, _ = op.generate(mo, SEED, B, gait=0)
    contact = contact_with(N, B, [22, 24] * 3, rng)
    Hs, gs, ns, mus, los, his = [], [], [], [], [], []
    for q in range(B):
        n, H, g, mu, lo, hi, mp, st = op.condense(mo, x0[q], xref[q], foot[q], contact[q], ld=128)
        Hs.append(H); gs.append(g); ns.append(n); mus.append(mu); los.append(lo); his.append(hi)
    gs[1][5] = np.nan   # tile variable (n = 72)
    gs[2][65] = np.nan  # border variable (n = 66)
    ref = [op.qp_ipm(ns[q], Hs[q], gs[q], mus[q], los[q], his[q], op.default_settings()) for q in range(B)]
    st_r = np.array([r[3] for r in ref])
    assert st_r[1] == st_r[2] == 3 and np.all(np.delete(st_r, [1, 2]) == 0)
    for v in (1, 0):
        eng = cm.Engine(m, precision=0, max_batch=B, path={cm.PATH_IPM72: v})
        u, st, it = eng.qp_solve(np.array(Hs), np.array(gs), np.array(ns, np.int32), np.array(mus), np.array(los),
                                 np.array(his))
        assert np.array_equal(st, st_r), (v, st, st_r)
        for q in np.nonzero(st_r == 0)[0]:
            assert rel_err(u[q, :ns[q]], ref[q][0]) < 1e-9, (v, q)
