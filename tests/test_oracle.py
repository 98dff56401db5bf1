"""CPU suite: the oracle (oracle/cmpc_oracle.c) pinned against the reference's own known-answer constructions and the
numpy golden fixtures (tests/golden/, made by the independent restatement oracle/np_ref.py).

Reference tests mirrored (ocs2_sqp/hpipm_catkin/test/testHpipmInterface.cpp):
  solve_and_check_dynamic :37-69   knownSolution :112-152   noInputs :208-256   retrieveRiccati :258-340
Properties of SURVEY §8c: dynamics consistency, KKT certificate, friction rows satisfied, swing forces exactly 0,
"mpc table invalid" status, generator known answers.
"""
import glob
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def load(name):
    with np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


GOLDEN = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "c*.npz")))


def test_philox_known_answers(op):
    kat = load("philox4x32_10_kat")["kat"]
    for row in kat:
        out = op.philox([int(x) for x in row[:4]], [int(x) for x in row[4:6]])
        assert out == [int(x) for x in row[6:]]


def test_generator_shard_invariance_and_ranges(op):
    m = op.default_model(10)
    full = op.generate(m, 20221125, 64, gait=1)
    half = op.generate(m, 20221125, 32, gait=1, offset=32)
    for f, h in zip(full, half):
        assert np.array_equal(f[32:], h)
    x0, xref, foot, contact = full
    assert np.all(x0[:, 12] == -9.81) and np.all((x0[:, 2] >= 0.12) & (x0[:, 2] <= 0.2))
    assert np.all(contact.sum(axis=2) >= 2)  # trot/bound/pronk always keep >= 2 stance legs


@pytest.mark.parametrize("name", GOLDEN)
def test_condense_matches_golden(op, name):
    z = load(name)
    m = op.default_model(int(z["N"]))
    for q in range(z["x0"].shape[0]):
        H, g, st = op.condense_full(m, z["x0"][q], z["xref"][q], z["foot"][q], z["contact"][q])
        assert st == 0
        assert rel(H, z["H_full"][q]) < 1e-12
        assert rel(g, z["g_full"][q]) < 1e-12


@pytest.mark.parametrize("name", GOLDEN)
def test_solve_matches_golden(op, name):
    z = load(name)
    m = op.default_model(int(z["N"]))
    u, x, st, it = op.solve_batch(m, op.tight_settings(), z["x0"], z["xref"], z["foot"], z["contact"])
    assert np.all(st == 0)
    for q in range(u.shape[0]):
        assert rel(u[q], z["u"][q]) < 1e-9
    # HPIPM default settings (tol_stat 1e-6, tol_comp 1e-8) are inside the north-star 1e-5 gate
    u2, _, st2, _ = op.solve_batch(m, op.default_settings(), z["x0"], z["xref"], z["foot"], z["contact"])
    assert np.all(st2 == 0)
    assert max(rel(u2[q], z["u"][q]) for q in range(u.shape[0])) < 1e-6


def test_dynamics_consistency_and_rollout(op):
    import np_ref
    m = op.default_model(10)
    x0, xref, foot, contact = op.generate(m, 7, 4, gait=1)
    u, x, st, _ = op.solve_batch(m, op.default_settings(), x0, xref, foot, contact)
    M = np_ref.model_arrays(m)
    for q in range(4):
        A, B = op.srbd_dynamics(m, xref[q], foot[q], contact[q])
        xs = x0[q].copy()
        for k in range(10):
            xs = A[k] @ xs + B[k] @ u[q, k].reshape(-1)
            assert np.allclose(xs, x[q, k + 1], rtol=0, atol=1e-12)
        _, _, Aqp, Bqp = np_ref.condense_full(M, x0[q], xref[q], foot[q], contact[q])
        X = Aqp @ x0[q] + Bqp @ u[q].reshape(-1)
        assert np.allclose(X, x[q, 1:].reshape(-1), rtol=0, atol=1e-11)


def test_constraints_and_swing(op):
    m = op.default_model(10)
    x0, xref, foot, contact = op.generate(m, 11, 32, gait=1)
    u, _, st, _ = op.solve_batch(m, op.default_settings(), x0, xref, foot, contact)
    assert np.all(st == 0)
    assert np.all(u[contact == 0] == 0.0)  # 0 <= F f <= 0 for swing legs (CentroidalMPC.cpp:199)
    f = u[contact == 1]
    mu = 0.8
    tol = 1e-6
    assert np.all(mu * f[:, 2] - np.abs(f[:, 0]) >= -tol)
    assert np.all(mu * f[:, 2] - np.abs(f[:, 1]) >= -tol)
    assert np.all(f[:, 2] >= -tol) and np.all(f[:, 2] <= 8 * 9.81 * 4 + tol)


def test_kkt_certificate(op):
    m = op.default_model(10)
    x0, xref, foot, contact = op.generate(m, 3, 6, gait=1)
    for q in range(6):
        n, H, g, mu, lo, hi, mp, st = op.condense(m, x0[q], xref[q], foot[q], contact[q])
        u, ll, lu, st, it, res = op.qp_ipm(n, H, g, mu, lo, hi, op.tight_settings())
        assert st == 0
        kkt = op.qp_kkt(n, H, g, mu, lo, hi, u, ll, lu)
        assert kkt[0] < 1e-9 and kkt[1] < 1e-10 and kkt[2] < 1e-9 and kkt[3] <= 0.0


def test_invalid_contact_table(op):
    m = op.default_model(10)
    x0, xref, foot, contact = op.generate(m, 5, 3, gait=0)
    contact[2, 4, :] = 0  # a flight step: reference throws "mpc table invalid" (CentroidalMPC.cpp:328-330)
    u, _, st, _ = op.solve_batch(m, op.default_settings(), x0, xref, foot, contact)
    assert list(st) == [0, 0, 5]
    assert np.all(u[2] == 0)


def test_known_solution_recovered_with_pyramid_rows(op):
    """SURVEY §8c known-solution construction on the condensed QP: pick U* strictly inside every friction pyramid,
    set g = -H U*, and the IPM (pyramid rows present, all inactive at U*) returns U*."""
    m = op.default_model(10)
    x0, xref, foot, contact = op.generate(m, 17, 4, gait=1)
    rng = np.random.default_rng(4)
    for q in range(4):
        n, H, g, mu, lo, hi, mp, st = op.condense(m, x0[q], xref[q], foot[q], contact[q])
        assert st == 0
        t = n // 3
        fz = rng.uniform(10.0, 60.0, t)
        fx = rng.uniform(-0.3, 0.3, t) * mu[:t] * fz
        fy = rng.uniform(-0.3, 0.3, t) * mu[:t] * fz
        us = np.stack([fx, fy, fz], axis=1).reshape(-1)
        g2 = g.copy()
        g2[:n] = -H[:n, :n] @ us
        u, ll, lu, st2, it, res = op.qp_ipm(n, H, g2, mu, lo, hi, op.tight_settings())
        assert st2 == 0
        assert np.abs(u - us).max() < 1e-8 * max(1.0, np.abs(us).max())


def test_fdes_sums_to_weight(op):
    """f^des_z = m 9.81 / n_stance per stance leg (CentroidalMPC.cpp:326-335) sums to m g per step. With
    every state weight 0 the condensed gradient is r-bar = -2 W_f f^des alone."""
    m = op.default_model(10)
    for j in range(9):
        m.weights[j] = 0.0
    x0, xref, foot, contact = op.generate(m, 23, 3, gait=1)
    L = 4
    for q in range(3):
        H, g, st = op.condense_full(m, x0[q], xref[q], foot[q], contact[q])
        assert st == 0
        N = m.N
        for k in range(N):
            fz = [-g[12 * k + 3 * i + 2] / (2.0 * m.weights[9 + 3 * L + 3 * i + 2]) for i in range(L)]
            assert abs(sum(fz) - m.mass * 9.81) < 1e-9
            for i in range(L):
                assert (fz[i] == 0.0) == (contact[q][k, i] == 0)


def test_unconstrained_is_newton_step(op):
    # with no inequality rows the IPM is one Newton step: H u = -g
    rng = np.random.default_rng(0)
    n = 9
    A = rng.standard_normal((n, n))
    H = A @ A.T + n * np.eye(n)
    g = rng.standard_normal(n)
    ld = 12
    Hp = np.eye(ld)
    Hp[:n, :n] = H
    gp = np.zeros(ld)
    gp[:n] = g
    mu = np.full(ld // 3, 0.8)
    lo = np.full((ld // 3, 5), -1e9)
    hi = np.full((ld // 3, 5), 1e9)
    u, ll, lu, st, it, res = op.qp_ipm(n, Hp, gp, mu, lo, hi, op.tight_settings())
    assert st == 0
    assert np.allclose(u, np.linalg.solve(H, -g), atol=1e-8)


# ---------------------------------------------------------------------------- HpipmInterface known answers

def random_ocp(rng, N, nx, nu_list):
    A, B, b, Q, S, R, q, r = [], [], [], [], [], [], [], []
    for k in range(N):
        nu = nu_list[k]
        A.append(rng.uniform(-1, 1, (nx, nx)))
        B.append(rng.uniform(-1, 1, (nx, nu)))
        b.append(rng.uniform(-1, 1, nx))
    for k in range(N + 1):
        nu = nu_list[k] if k < N else 0
        Mx = rng.uniform(-1, 1, (nx + nu, nx + nu))
        Hk = Mx @ Mx.T + (nx + nu) * np.eye(nx + nu)  # getRandomCost: positive definite
        Q.append(Hk[:nx, :nx])
        S.append(Hk[nx:, :nx])
        R.append(Hk[nx:, nx:])
        q.append(rng.uniform(-1, 1, nx))
        r.append(rng.uniform(-1, 1, nu))
    return A, B, b, Q, S, R, q, r


def test_hpipm_known_solution(op):
    """testHpipmInterface.cpp:112-152 (and noInputs :208-256 with nu_1 = 0)."""
    rng = np.random.default_rng(42)
    for nu_list in ([2, 2, 2, 2, 2], [2, 0, 2, 2, 2]):
        N, nx = 5, 3
        A, B, b, Q, S, R, q, r = random_ocp(rng, N, nx, nu_list)
        xs = [rng.uniform(-1, 1, nx)]
        us = []
        for k in range(N):
            us.append(rng.uniform(-1, 1, nu_list[k]))
            xs.append(b[k] + A[k] @ xs[k] + B[k] @ us[k])
            q[k] = -(Q[k] @ xs[k] + S[k].T @ us[k])
            r[k] = -(R[k] @ us[k] + S[k] @ xs[k])
        q[N] = -Q[N] @ xs[N]
        rec = op.ocp_pack(N, nx, nu_list, A, B, b, Q, S, R, q, r)
        x, u, st = op.ocp_solve(N, nx, nu_list, xs[0], rec)
        assert st == 0
        assert np.allclose(x, np.array(xs), atol=1e-9)
        assert np.allclose(u, np.concatenate(us), atol=1e-9)


def test_hpipm_dynamics_feasible(op):
    """testHpipmInterface.cpp:37-69."""
    rng = np.random.default_rng(3)
    N, nx, nu = 5, 3, [2] * 5
    A, B, b, Q, S, R, q, r = random_ocp(rng, N, nx, nu)
    x0 = rng.uniform(-1, 1, nx)
    x, u, st = op.ocp_solve(N, nx, nu, x0, op.ocp_pack(N, nx, nu, A, B, b, Q, S, R, q, r))
    assert st == 0
    assert np.allclose(x[0], x0)
    for k in range(N):
        assert np.allclose(x[k + 1], A[k] @ x[k] + B[k] @ u[2 * k:2 * k + 2] + b[k], atol=1e-12)


def test_hpipm_riccati(op):
    """testHpipmInterface.cpp:258-340: closed-form Riccati recursion vs the oracle's, and u = K x + k."""
    rng = np.random.default_rng(5)
    N, nx, nu = 5, 3, [2] * 5
    A, B, b, Q, S, R, q, r = random_ocp(rng, N, nx, nu)
    rec = op.ocp_pack(N, nx, nu, A, B, b, Q, S, R, q, r)
    Sm, sv, K, kff, st = op.ocp_riccati(N, nx, nu, rec)
    assert st == 0
    Sg, sg = Q[N], q[N]
    for k in range(N - 1, -1, -1):
        P = S[k] + B[k].T @ Sg @ A[k]
        iR = np.linalg.inv(R[k] + B[k].T @ Sg @ B[k])
        rr = r[k] + B[k].T @ sg + B[k].T @ Sg @ b[k]
        Sn = Q[k] + A[k].T @ Sg @ A[k] - P.T @ iR @ P
        sn = q[k] + A[k].T @ sg + A[k].T @ Sg @ b[k] - P.T @ iR @ rr
        assert np.allclose(K[k], -iR @ P, atol=1e-9)
        assert np.allclose(kff[k], -iR @ rr, atol=1e-9)
        assert np.allclose(Sm[k], Sn, atol=1e-9) and np.allclose(sv[k], sn, atol=1e-9)
        Sg, sg = Sn, sn
    x0 = rng.uniform(-1, 1, nx)
    x, u, st = op.ocp_solve(N, nx, nu, x0, rec)
    for k in range(N):
        assert np.allclose(u[2 * k:2 * k + 2], K[k] @ x[k] + kff[k], atol=1e-9)


@pytest.mark.parametrize("N,gait,ub4,all_stance", [(10, 0, None, False), (10, 1, None, False), (10, 1, 15.0, False),
                                                    (20, 0, None, False), (20, 0, 15.0, True), (6, 0, None, False)])
def test_riccati_ipm_matches_condensed_ipm(op, N, gait, ub4, all_stance):
    """The HPIPM-style restatement (no condensing: Riccati over [x; u_prev] stages, rollout/adjoint gradient) runs the
    same Mehrotra iteration as the condensed oracle, so statuses and iteration counts agree exactly and the forces to
    rounding: the condensing (H, g, swing elimination, force-rate coupling) is pinned against the OCP form HPIPM
    solves for the reference (HpipmInterface.cpp:166-301)."""
    m = op.default_model(N)
    if ub4 is not None:
        m.force_ub[4] = ub4
    s = op.default_settings()
    x0, xref, foot, contact = op.generate(m, 20221125, 64, gait=gait)
    if all_stance:
        contact[:] = 1
    u, _, st, it = op.solve_batch(m, s, x0, xref, foot, contact, nthreads=8, want_x=False)
    ur, sr, itr = op.riccati_solve_batch(m, s, x0, xref, foot, contact, nthreads=8)
    assert np.array_equal(st, sr) and np.all(st == 0)
    assert np.array_equal(it, itr)
    assert np.abs(u - ur).max() / max(1.0, np.abs(u).max()) < 1e-12


def test_riccati_ipm_invalid_contact(op):
    m = op.default_model(10)
    x0, xref, foot, contact = op.generate(m, 20221125, 2, gait=0)
    contact[1, 4, :] = 0
    ur, sr, _ = op.riccati_solve_batch(m, op.default_settings(), x0, xref, foot, contact)
    assert sr[0] == 0 and sr[1] == 5 and np.all(ur[1] == 0.0)


def test_stance_feet_matches_numpy_restatement(op):
    """oracle_stance_point (C scans) vs np_ref.stance_feet (numpy run boundaries) on random contact tables: the
    reference's foot dynamics (CentroidalMPC.cpp:93) with foot_pos(:,0) pinned to the state's feet (:165-167)."""
    import np_ref
    rng = np.random.default_rng(5)
    for N in (1, 2, 6, 10, 20):
        for _ in range(40):
            contact = (rng.random((N, 4)) < 0.6).astype(np.uint8)
            foot = rng.normal(size=(N + 1, 4, 3))
            P = op.stance_feet(foot, contact)
            R = np_ref.stance_feet(foot, contact)
            assert np.max(np.abs(P - R)) < 1e-14
            for i in range(4):
                run0 = 0
                while run0 < N and contact[run0, i]:
                    run0 += 1
                # the initial stance run acts at the current foot position, bit for bit
                assert np.array_equal(P[:run0, i], np.broadcast_to(foot[0, i], (run0, 3)))
                assert np.all(P[contact[:, i] == 0, i] == 0.0)


def test_planted_feet_are_exact(op):
    """A stance run whose des_foot_pos is constant (the generator plants feet) acts at that foothold exactly."""
    m = op.default_model(10)
    x0, xref, foot, contact = op.generate(m, 20221125, 32, gait=1)
    for q in range(32):
        P = op.stance_feet(foot[q], contact[q])
        for k in range(10):
            for i in range(4):
                if not contact[q, k, i]:
                    continue
                s = k
                while s > 0 and contact[q, s - 1, i]:
                    s -= 1
                assert np.array_equal(P[k, i], foot[q, s, i])


def test_current_foot_position_is_an_input(op):
    """UpdateMPC's state[9..20] (CentroidalMPC.cpp:288-291) moves U; the des_foot_pos nodes of the initial stance run
    do not (the reference pins those nodes to the current foot, :165-167 with :93)."""
    m = op.default_model(10)
    x0, xref, foot, contact = op.generate(m, 20221125, 4, gait=0)
    s = op.tight_settings()
    u0, _, st0, _ = op.solve_batch(m, s, x0, xref, foot, contact)
    f1 = foot.copy()
    f1[:, 0, :, 0] += 0.02  # current feet 2 cm forward
    u1, _, st1, _ = op.solve_batch(m, s, x0, xref, f1, contact)
    assert np.all(st0 == 0) and np.all(st1 == 0)
    assert rel(u1, u0) > 1e-4
    f2 = foot.copy()
    for q in range(4):
        for i in range(4):
            k = 0
            while k < 10 and contact[q, k, i]:
                k += 1
            if k > 0:  # initial stance run: nodes 1..k pinned to node 0 in the reference
                f2[q, 1:k + 1, i, :2] += 0.05
    u2, _, _, _ = op.solve_batch(m, s, x0, xref, f2, contact)
    assert np.array_equal(u2, u0)
