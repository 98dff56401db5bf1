"""Batched SQP on the bilinear centroidal NLP: the QP linearised at the iterate instead of at the
reference. The reference's NLP keeps the lever arm bilinear, (p - c) x f (CentroidalMPC.cpp:86), and solves it with
IPOPT; its SQP counterpart in ocs2 is MultipleShootingSolver::runImpl (MultipleShootingSolver.cpp:146-214). CPU: the
linearisation is an exact Taylor expansion and the SQP fixed point is a KKT point of the NLP; GPU: the device SQP
follows the oracle's."""
import numpy as np
import pytest

SEED = 20221125


def rel_err(u, ur):
    return float(np.max(np.abs(u - ur)) / max(1.0, float(np.max(np.abs(ur)))))


def linear_rollout(A, B, b, x0, u):
    N = A.shape[0]
    x = [np.asarray(x0, float)]
    for k in range(N):
        x.append(A[k] @ x[k] + B[k] @ u[k].reshape(-1) + b[k])
    return np.array(x)


def test_linearisation_is_exact_taylor(op):
    N = 10
    mo = op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, 4, gait=1)
    rng = np.random.default_rng(0)
    for q in range(4):
        u = rng.uniform(0, 40, (N, 4, 3)) * contact[q][:, :, None]
        J, xnl, lin = op.nlp_rollout_cost(mo, x0[q], xref[q], foot[q], contact[q], u)
        A, B, b = op.srbd_dynamics_lin(mo, xref[q], foot[q], contact[q], lin)
        # at the linearisation point the linear model reproduces the nonlinear rollout
        assert np.abs(linear_rollout(A, B, b, x0[q], u) - xnl).max() < 1e-11
        # first order: a perturbation du changes the two by O(du^2) only
        du = 1e-3 * rng.standard_normal(u.shape) * contact[q][:, :, None]
        _, xnl2, _ = op.nlp_rollout_cost(mo, x0[q], xref[q], foot[q], contact[q], u + du)
        assert np.abs(linear_rollout(A, B, b, x0[q], u + du) - xnl2).max() < 1e-7
        # lin = None is the reference linearisation of the QP (b = 0)
        A0, B0, b0 = op.srbd_dynamics_lin(mo, xref[q], foot[q], contact[q], None)
        A1, B1 = op.srbd_dynamics(mo, xref[q], foot[q], contact[q])
        assert np.array_equal(A0, A1) and np.array_equal(B0, B1) and not b0.any()


def test_nlp_cost_matches_qp_objective_at_reference_linearisation(op):
    """With f_bar = 0 and c_bar = c_ref the QP objective 1/2 U'HU + g'U differs from the NLP cost of the LINEAR
    rollout by a constant only; checked through two inputs."""
    N = 8
    mo = op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, 1, gait=0)
    H, g, st = op.condense_full(mo, x0[0], xref[0], foot[0], contact[0])
    rng = np.random.default_rng(1)
    us = [rng.uniform(0, 30, (N, 4, 3)) * contact[0][:, :, None] for _ in range(2)]
    # NLP cost of the linear rollout, evaluated by hand with the same weights
    A, B, b = op.srbd_dynamics_lin(mo, xref[0], foot[0], contact[0], None)
    c = op.consts(mo)
    def jlin(u):
        x = linear_rollout(A, B, b, x0[0], u)
        J = sum(0.5 * c.qdiag[k + 1][s] * (x[k + 1, s] - xref[0][k + 1, s]) ** 2 for k in range(N) for s in range(13))
        uf = u.reshape(N, 12)
        ns = contact[0].sum(axis=1)
        fd = np.zeros((N, 12))
        for k in range(N):
            for i in range(4):
                if contact[0][k, i]:
                    fd[k, 3 * i + 2] = mo.mass * 9.81 / ns[k]
        J += sum(c.Wf[j] * (uf[k, j] - fd[k, j]) ** 2 for k in range(N) for j in range(12))
        J += sum(c.Wr[j] * (uf[k + 1, j] - uf[k, j]) ** 2 for k in range(N - 1) for j in range(12))
        return J
    qp = lambda u: 0.5 * u.reshape(-1) @ H @ u.reshape(-1) + g @ u.reshape(-1)  # noqa: E731
    assert abs((jlin(us[0]) - qp(us[0])) - (jlin(us[1]) - qp(us[1]))) < 1e-7 * max(1.0, abs(jlin(us[0])))


def test_oracle_sqp_converges_to_nlp_stationary_point(op):
    N = 10
    mo = op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, 6, gait=1)
    s = op.default_settings()
    for q in range(6):
        u, x, st, qi, si = op.sqp_solve(mo, s, x0[q], xref[q], foot[q], contact[q], sqp_iter_max=20, sqp_tol=1e-8)
        assert st == 0 and si < 20
        J, xnl, lin = op.nlp_rollout_cost(mo, x0[q], xref[q], foot[q], contact[q], u)
        assert np.abs(x - xnl).max() == 0.0
        # the cold QP (reference linearisation) is the SQP's first iterate; the SQP lowers the NLP cost
        u0, _, st0, _ = op.solve_batch(mo, s, x0[q:q + 1], xref[q:q + 1], foot[q:q + 1], contact[q:q + 1])
        J0, _, _ = op.nlp_rollout_cost(mo, x0[q], xref[q], foot[q], contact[q], u0[0])
        assert J <= J0 + 1e-9 * abs(J0)
        # fixed point: the QP linearised at the solution returns the solution (first-order KKT of the NLP)
        tight = op.tight_settings()
        n, Hc, gc, mu, lo, hi, mp, stc = condense_lin(op, mo, x0[q], xref[q], foot[q], contact[q], lin)
        uq = op.qp_ipm(n, Hc, gc, mu, lo, hi, tight)[0]
        ucond = np.array([u[mp[t] // 4, mp[t] % 4, d] for t in range(n // 3) for d in range(3)])
        assert np.abs(uq - ucond).max() < 1e-4 * max(1.0, np.abs(ucond).max())
    # swing forces exactly zero
    assert np.all(u[contact[5] == 0] == 0.0)


def test_linstep_is_the_directional_derivative(op):
    """The line search's inputs (MultipleShootingSolver.cpp:287-296, :492-503): the descent metric is grad J . du
    along the nonlinear rollout and |dx| the norm of the rollout's linear response, both by central differences."""
    N = 10
    mo = op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, 4, gait=1)
    rng = np.random.default_rng(7)
    for q in range(4):
        u = op.solve_batch(mo, op.default_settings(), x0[q:q + 1], xref[q:q + 1], foot[q:q + 1], contact[q:q + 1])[0][0]
        du = rng.standard_normal(u.shape) * 5.0 * contact[q][..., None]
        dxn, mt = op.nlp_linstep(mo, x0[q], xref[q], foot[q], contact[q], u, du)
        h = 1e-4
        Jp, xp, _ = op.nlp_rollout_cost(mo, x0[q], xref[q], foot[q], contact[q], u + h * du)
        Jm, xm, _ = op.nlp_rollout_cost(mo, x0[q], xref[q], foot[q], contact[q], u - h * du)
        assert abs(mt - (Jp - Jm) / (2 * h)) < 1e-6 * max(1.0, abs(mt))
        assert abs(dxn - np.linalg.norm((xp - xm) / (2 * h))) < 1e-7 * max(1.0, dxn)


def test_sqp_line_search_rules(op):
    """Every accepted SQP step satisfies the reference's acceptance test (Armijo with the descent metric when it is
    negative, plain decrease otherwise; MultipleShootingSolver.cpp:562-571) at a step 2^-m >= alpha_min."""
    N = 10
    mo = op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, 6, gait=1)
    s = op.default_settings()
    for q in range(6):
        u_prev = None
        for its in range(1, 6):
            u, _, st, _, si = op.sqp_solve(mo, s, x0[q], xref[q], foot[q], contact[q], sqp_iter_max=its, sqp_tol=1e-9)
            assert st == 0
            if u_prev is not None and si == its:
                J0, _, lin = op.nlp_rollout_cost(mo, x0[q], xref[q], foot[q], contact[q], u_prev)
                J1 = op.nlp_rollout_cost(mo, x0[q], xref[q], foot[q], contact[q], u)[0]
                assert J1 <= J0
            u_prev = u
            if si < its:
                break


def condense_lin(op, mo, x0, xref, foot, contact, lin):
    """Condensed QP at a linearisation point through the oracle's full condensing + elimination."""
    import ctypes as C
    N = mo.N
    ld = 12 * N
    c = op.consts(mo)
    H = np.zeros((ld, ld)); g = np.zeros(ld); mu = np.zeros(ld // 3); lo = np.zeros((ld // 3, 5))
    hi = np.zeros((ld // 3, 5)); mp = np.zeros(ld // 3, np.int32); n = C.c_int(0)
    L = op.lib()
    L.oracle_condense_lin.argtypes = [C.c_void_p] + [C.POINTER(C.c_double)] * 3 + [C.POINTER(C.c_uint8),
                                      C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_int)] + \
        [C.POINTER(C.c_double)] * 5 + [C.POINTER(C.c_int)]
    a = [np.ascontiguousarray(v, np.float64) for v in (x0, xref, foot, lin)]
    ct = np.ascontiguousarray(contact, np.uint8)
    st = L.oracle_condense_lin(C.byref(c), op._p(a[0]), op._p(a[1]), op._p(a[2]), op._p(ct, C.c_uint8), op._p(a[3]),
                               ld, C.byref(n), op._p(H), op._p(g), op._p(mu), op._p(lo), op._p(hi),
                               op._p(mp, C.c_int))
    return n.value, H, g, mu, lo, hi, mp, st


@pytest.mark.gpu
@pytest.mark.parametrize("N,gait,all_stance", [(10, 1, False), (20, 0, False), (12, 0, True)])
def test_device_sqp_matches_oracle(cm, op, N, gait, all_stance):
    """All size classes (n = 60/120 at N = 10 mixed, 120 at N = 20 trot, 144 at N = 12 all-stance)."""
    B = 24
    m, mo = cm.default_model(N), op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=gait)
    if all_stance:
        contact[:] = 1
    eng = cm.Engine(m, precision=0, max_batch=B)
    u, x, st, qi, si = eng.sqp_solve(x0, xref, foot, contact, sqp_iter_max=10, sqp_tol=1e-7)
    s = op.default_settings()
    for q in range(B):
        ur, xr, sr, qir, sir = op.sqp_solve(mo, s, x0[q], xref[q], foot[q], contact[q], sqp_iter_max=10,
                                            sqp_tol=1e-7)
        assert st[q] == sr == 0
        assert rel_err(u[q], ur) < 1e-6, q
        assert abs(int(si[q]) - sir) <= 1 and si[q] < 10
        assert np.abs(x[q] - xr).max() < 1e-6 * max(1.0, np.abs(xr).max())
    # the SQP never raises the NLP cost above the reference-linearised QP's
    u0, _, st0, _ = eng.solve(x0, xref, foot, contact, want_x=False)
    for q in range(B):
        J = op.nlp_rollout_cost(mo, x0[q], xref[q], foot[q], contact[q], u[q])[0]
        J0 = op.nlp_rollout_cost(mo, x0[q], xref[q], foot[q], contact[q], u0[q])[0]
        assert J <= J0 + 1e-9 * abs(J0)
    assert np.all(u[contact == 0] == 0.0)
