"""Footholds of the later stance runs as decision variables of the NLP: the reference optimises
foot_pos at every node (CentroidalMPC.cpp:132-133) under the swing dynamics (:93, :174-176), the pinning of node 0
(:165-167), the step box (:196-198, :30-31) and the tracking cost (:218-221). CPU: the oracle's condensed QP with
foothold columns is the first-order model of the NLP (gradient = NLP gradient by central differences), its linearised
step is the directional derivative, and the SQP with footholds ends at a KKT point inside the box with a cost no
higher than the frozen-foothold SQP's."""
import numpy as np
import pytest

SEED = 20221125
NL = 4


def later_runs(contact):
    N, L = contact.shape
    out = []
    for s in range(1, N):
        for i in range(L):
            if contact[s, i] and not contact[s - 1, i]:
                e = s
                while e + 1 < N and contact[e + 1, i]:
                    e += 1
                out.append((s, i, e))
    return out


def pack(mp, n, u, D, N):
    z = np.zeros(n)
    for t in range(n // 3):
        c = mp[t]
        src = u.reshape(N * NL, 3)[c] if c < N * NL else D.reshape(N * NL, 3)[c - N * NL]
        z[3 * t:3 * t + 3] = src
    return z


def unpack(mp, n, z, N):
    u, D = np.zeros((N * NL, 3)), np.zeros((N * NL, 3))
    for t in range(n // 3):
        c = mp[t]
        if c < N * NL:
            u[c] = z[3 * t:3 * t + 3]
        else:
            D[c - N * NL] = z[3 * t:3 * t + 3]
    return u.reshape(N, NL, 3), D.reshape(N, NL, 3)


@pytest.mark.parametrize("gait", [1, 2])
def test_foothold_qp_gradient_is_nlp_gradient(op, gait):
    N = 10
    mo = op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, 3, gait=gait)
    rng = np.random.default_rng(3)
    checked = 0
    for q in range(3):
        runs = later_runs(contact[q])
        u = rng.uniform(0, 40, (N, NL, 3)) * contact[q][:, :, None]
        D = np.zeros((N, NL, 3))
        for (s, i, e) in runs:
            D[s, i] = rng.uniform(-0.05, 0.05, 3)
        J, _, lin = op.nlp_rollout_cost_feet(mo, x0[q], xref[q], foot[q], contact[q], u, D)
        n, H, g, mu, lo, hi, mp, st = op.condense_feet(mo, x0[q], xref[q], foot[q], contact[q], lin, u, D)
        assert st == 0
        assert n == 3 * (int(contact[q].sum()) + len(runs))
        z = pack(mp, n, u, D, N)
        grad_qp = H[:n, :n] @ z + g[:n]
        h = 1e-5
        for a in range(n):
            dz = np.zeros(n)
            dz[a] = h
            up, Dp = unpack(mp, n, z + dz, N)
            um, Dm = unpack(mp, n, z - dz, N)
            Jp = op.nlp_rollout_cost_feet(mo, x0[q], xref[q], foot[q], contact[q], up, Dp)[0]
            Jm = op.nlp_rollout_cost_feet(mo, x0[q], xref[q], foot[q], contact[q], um, Dm)[0]
            fd = (Jp - Jm) / (2 * h)
            assert abs(fd - grad_qp[a]) < 1e-5 * max(1.0, abs(fd)), (q, a, fd, grad_qp[a])
        # foothold triples: mu 0 and the step box rows [-x, x, -y, y, z]
        for t in range(n // 3):
            if mp[t] >= N * NL:
                s, i = divmod(mp[t] - N * NL, NL)
                pb, blo, bhi, cnt = op.foot_box(foot[q], contact[q], s, i)
                assert mu[t] == 0.0
                assert np.allclose(lo[t], [-bhi[0], blo[0], -bhi[1], blo[1], blo[2]])
                assert np.allclose(hi[t], [-blo[0], bhi[0], -blo[1], bhi[1], bhi[2]])
                checked += 1
    assert checked > 0


def test_foothold_linstep_is_directional_derivative(op):
    N = 10
    mo = op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, 3, gait=1)
    rng = np.random.default_rng(11)
    for q in range(3):
        u = rng.uniform(0, 40, (N, NL, 3)) * contact[q][:, :, None]
        D, dD = np.zeros((N, NL, 3)), np.zeros((N, NL, 3))
        for (s, i, e) in later_runs(contact[q]):
            D[s, i] = rng.uniform(-0.05, 0.05, 3)
            dD[s, i] = rng.standard_normal(3) * 0.1
        du = rng.standard_normal(u.shape) * 5.0 * contact[q][..., None]
        dxn, mt = op.nlp_linstep_feet(mo, x0[q], xref[q], foot[q], contact[q], u, D, du, dD)
        h = 1e-5
        Jp, xp, _ = op.nlp_rollout_cost_feet(mo, x0[q], xref[q], foot[q], contact[q], u + h * du, D + h * dD)
        Jm, xm, _ = op.nlp_rollout_cost_feet(mo, x0[q], xref[q], foot[q], contact[q], u - h * du, D - h * dD)
        assert abs(mt - (Jp - Jm) / (2 * h)) < 1e-6 * max(1.0, abs(mt))
        assert abs(dxn - np.linalg.norm((xp - xm) / (2 * h))) < 1e-6 * max(1.0, dxn)
        # D = 0, dD = 0 reproduce the frozen-foothold functions' linearised step exactly
        z = np.zeros_like(D)
        assert op.nlp_linstep_feet(mo, x0[q], xref[q], foot[q], contact[q], u, z, du, z) == \
            op.nlp_linstep(mo, x0[q], xref[q], foot[q], contact[q], u, du)


def test_frozen_rollout_is_the_zero_offset_rollout(op):
    """With D = 0 the lever arm is the frozen one: same trajectory bit for bit, cost higher by the later runs' foot
    tracking at the mean position."""
    N = 10
    mo = op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, 2, gait=1)
    c = op.consts(mo)
    rng = np.random.default_rng(5)
    for q in range(2):
        u = rng.uniform(0, 40, (N, NL, 3)) * contact[q][:, :, None]
        J0, x0r, l0 = op.nlp_rollout_cost(mo, x0[q], xref[q], foot[q], contact[q], u)
        J1, x1r, l1 = op.nlp_rollout_cost_feet(mo, x0[q], xref[q], foot[q], contact[q], u, np.zeros((N, NL, 3)))
        assert np.array_equal(x0r, x1r) and np.array_equal(l0, l1)
        jf = 0.0
        for (s, i, e) in later_runs(contact[q]):
            pb = op.foot_box(foot[q], contact[q], s, i)[0]
            for j in range(s, e + 2):
                jf += sum(c.Wp[3 * i + d] * (pb[d] - foot[q][j, i, d]) ** 2 for d in range(3))
        assert abs((J1 - J0) - jf) < 1e-12 * max(1.0, J1)


@pytest.mark.parametrize("gait", [1, 2])
def test_oracle_sqp_with_footholds(op, gait):
    N = 10
    mo = op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, 4, gait=gait)
    s = op.default_settings()
    tight = op.tight_settings()
    moved = 0
    for q in range(4):
        runs = later_runs(contact[q])
        u, D, feet, x, st, qi, si = op.sqp_solve_feet(mo, s, x0[q], xref[q], foot[q], contact[q], sqp_iter_max=20,
                                                      sqp_tol=1e-8)
        assert st == 0 and si < 20
        J, xnl, lin = op.nlp_rollout_cost_feet(mo, x0[q], xref[q], foot[q], contact[q], u, D)
        assert np.abs(x - xnl).max() == 0.0
        # box respected, unused entries zero
        used = np.zeros((N, NL), bool)
        for (s0, i, e) in runs:
            pb, lo, hi, cnt = op.foot_box(foot[q], contact[q], s0, i)
            assert np.all(D[s0, i] >= lo - 1e-9) and np.all(D[s0, i] <= hi + 1e-9)
            used[s0, i] = True
            moved += int(np.abs(D[s0, i]).max() > 1e-6)
            for j in range(s0, e + 2):  # the run's nodes hold its foothold
                assert np.array_equal(feet[j, i], pb + D[s0, i])
        assert not D[~used].any()
        # node 0 and the first runs at the current foot, free swing nodes at des
        assert np.array_equal(feet[0], foot[q][0])
        for i in range(NL):
            for j in range(1, N + 1):
                in_stance = (j < N and contact[q][j, i]) or contact[q][j - 1, i]
                if not in_stance:
                    assert np.array_equal(feet[j, i], foot[q][j, i])
        # more freedom than the frozen-foothold SQP: no higher NLP cost
        uf = op.sqp_solve(mo, s, x0[q], xref[q], foot[q], contact[q], sqp_iter_max=20, sqp_tol=1e-8)[0]
        Jf = op.nlp_rollout_cost_feet(mo, x0[q], xref[q], foot[q], contact[q], uf, op.feet_init(mo, foot[q], contact[q]))[0]
        assert J <= Jf + 1e-6 * abs(Jf)
        # fixed point: the foothold QP linearised at the solution returns it (first-order KKT of the NLP)
        n, H, g, mu, lo, hi, mp, stc = op.condense_feet(mo, x0[q], xref[q], foot[q], contact[q], lin, u, D)
        zq = op.qp_ipm(n, H, g, mu, lo, hi, tight)[0]
        z = pack(mp, n, u, D, N)
        assert np.abs(zq - z).max() < 1e-4 * max(1.0, np.abs(z).max())
    assert moved > 0  # the footholds do move off the frozen mean


def test_empty_step_box_is_reported(op):
    N = 10
    mo = op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, 1, gait=1)
    runs = later_runs(contact[0])
    assert runs
    s0, i, e = runs[0]
    foot2 = foot[0].copy()
    foot2[e + 1, i, 0] += 0.5  # des varies over the run by more than the 0.4 m box
    u, D, feet, x, st, qi, si = op.sqp_solve_feet(mo, op.default_settings(), x0[0], xref[0], foot2, contact[0])
    assert st == 7  # CMPC_INFEASIBLE_STEP
    n, *_, stc = op.condense_feet(mo, x0[0], xref[0], foot2, contact[0], np.zeros((N, 6)), u, D)
    assert stc == 7


def _first_run_leg(contact):
    """A leg in stance at step 0 and the last node of that run (e + 1)."""
    N = contact.shape[0]
    for i in range(NL):
        if contact[0, i]:
            e = 0
            while e + 1 < N and contact[e + 1, i]:
                e += 1
            return i, min(e + 1, N)
    return None


def test_current_foot_outside_step_box_is_reported(op):
    """the step box of CentroidalMPC.cpp:196-198 also binds the nodes of a stance run from step 0, where
    foot_pos is pinned to the current foot (:165-167); a current foot 0.5 m off des_foot_pos there makes the reference
    NLP infeasible: INFEASIBLE_STEP (oracle condensing and SQP)."""
    N = 10
    mo = op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, 1, gait=0)
    i, j = _first_run_leg(contact[0])
    foot2 = foot[0].copy()
    foot2[j, i, 1] += 0.5  # des at a node of the first run, 0.5 m from the planted current foot
    u, D, feet, x, st, qi, si = op.sqp_solve_feet(mo, op.default_settings(), x0[0], xref[0], foot2, contact[0])
    assert st == 7
    n, *_, stc = op.condense_feet(mo, x0[0], xref[0], foot2, contact[0], np.zeros((N, 6)), u, D)
    assert stc == 7
    u, D, feet, x, st, qi, si = op.sqp_solve_feet(mo, op.default_settings(), x0[0], xref[0], foot[0], contact[0])
    assert st == 0


# ------------------------------------------------------------------------------------------------ device (gpu)

def rel_err(u, ur):
    return float(np.max(np.abs(u - ur)) / max(1.0, float(np.max(np.abs(ur)))))


@pytest.mark.gpu
@pytest.mark.parametrize("N,gait", [(10, 1), (10, 2), (20, 1), (5, 1)])
def test_device_foothold_condensing_matches_oracle(cm, op, N, gait):
    """cmpc_condense_lin_batch with foothold columns vs oracle_condense_feet (classes 64 / 128 / 256 and the
    one-class context N = 5): same triple order and boxes, H and g to 1e-11."""
    B = 8
    m, mo = cm.default_model(N), op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=gait)
    rng = np.random.default_rng(N + gait)
    u = rng.uniform(0, 40, (B, N, NL, 3)) * contact[..., None]
    D = np.zeros((B, N, NL, 3))
    lin = np.zeros((B, N, 6))
    for q in range(B):
        for (s, i, e) in later_runs(contact[q]):
            D[q, s, i] = rng.uniform(-0.05, 0.05, 3)
        lin[q] = op.nlp_rollout_cost_feet(mo, x0[q], xref[q], foot[q], contact[q], u[q], D[q])[2]
    eng = cm.Engine(m, precision=0, max_batch=B)
    H, g, n, st, mp, lo, hi = eng.condense_lin(x0, xref, foot, contact, lin, u, D)
    for q in range(B):
        nr, Hr, gr, mur, lor, hir, mpr, sr = op.condense_feet(mo, x0[q], xref[q], foot[q], contact[q], lin[q], u[q],
                                                               D[q], ld=eng.ld)
        assert st[q] == sr == 0 and n[q] == nr
        t = nr // 3
        assert np.array_equal(mp[q, :t], mpr[:t])
        assert np.allclose(lo[q, :t], lor[:t], rtol=0, atol=1e-15) and np.allclose(hi[q, :t], hir[:t], rtol=0,
                                                                                  atol=1e-15)
        sc = max(1.0, np.abs(Hr[:nr, :nr]).max())
        assert np.abs(H[q, :nr, :nr] - Hr[:nr, :nr]).max() < 1e-11 * sc
        assert np.abs(g[q, :nr] - gr[:nr]).max() < 1e-11 * max(1.0, np.abs(gr[:nr]).max())
    # frozen footholds (no dbar): the hook reproduces cmpc_condense_batch
    H0, g0, n0, st0, *_ = eng.condense_lin(x0, xref, foot, contact)
    H1, g1, n1, st1 = eng.condense(x0, xref, foot, contact)
    assert np.array_equal(H0, H1) and np.array_equal(g0, g1) and np.array_equal(n0, n1)


@pytest.mark.gpu
@pytest.mark.parametrize("N,gait,prec", [(10, 1, 0), (10, 2, 0), (20, 1, 0), (10, 1, 1), (20, 1, 1)])
def test_device_nlp_matches_oracle(cm, op, N, gait, prec):
    B = 16
    m, mo = cm.default_model(N), op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=gait)
    # fp32: the IPM tolerances fp32 reaches (as test_full_size's fp32 configs)
    settings = cm.default_settings() if prec == 0 else cm.default_settings(tol_stat=1e-3, tol_ineq=1e-3,
                                                                           tol_comp=1e-4)
    eng = cm.Engine(m, settings, precision=prec, max_batch=B)
    u, feet, x, st, qi, si = eng.nlp_solve(x0, xref, foot, contact, sqp_iter_max=10, sqp_tol=1e-7)
    s = op.default_settings()
    for q in range(B):
        ur, Dr, feetr, xr, sr, qir, sir = op.sqp_solve_feet(mo, s, x0[q], xref[q], foot[q], contact[q],
                                                            sqp_iter_max=10, sqp_tol=1e-7)
        assert st[q] == sr == 0
        if prec == 0:
            assert rel_err(u[q], ur) < 1e-6, q
            assert np.abs(feet[q] - feetr).max() < 1e-8, q
            assert abs(int(si[q]) - sir) <= 1 and si[q] < 10
            assert np.abs(x[q] - xr).max() < 1e-6 * max(1.0, np.abs(xr).max())
        else:  # fp32 QPs inside an fp64 line search: the NLP cost matches the fp64 oracle's to 1e-3
            J = op.nlp_rollout_cost_feet(mo, x0[q], xref[q], foot[q], contact[q], u[q],
                                         feet_offsets(op, mo, foot[q], contact[q], feet[q]))[0]
            Jr = op.nlp_rollout_cost_feet(mo, x0[q], xref[q], foot[q], contact[q], ur, Dr)[0]
            assert abs(J - Jr) < 1e-3 * abs(Jr)
        # feet table semantics: node 0 current, free swing nodes des, boxes respected
        assert np.array_equal(feet[q][0], foot[q][0])
        for (s0, i, e) in later_runs(contact[q]):
            pb, blo, bhi, cnt = op.foot_box(foot[q], contact[q], s0, i)
            dl = feet[q][s0, i] - pb
            assert np.all(dl >= blo - 1e-6) and np.all(dl <= bhi + 1e-6)
    assert np.all(u[contact == 0] == 0.0)


def feet_offsets(op, mo, foot, contact, feet):
    D = np.zeros((mo.N, NL, 3))
    for (s, i, e) in later_runs(contact):
        D[s, i] = feet[s, i] - op.foot_box(foot, contact, s, i)[0]
    return D


@pytest.mark.gpu
def test_device_nlp_empty_step_box(cm, op):
    N, B = 10, 4
    m, mo = cm.default_model(N), op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=1)
    runs = later_runs(contact[1])
    s0, i, e = runs[0]
    foot[1, e + 1, i, 0] += 0.5
    eng = cm.Engine(m, precision=0, max_batch=B)
    u, feet, x, st, qi, si = eng.nlp_solve(x0, xref, foot, contact)
    assert st[1] == 7 and all(st[q] == 0 for q in (0, 2, 3))
    # the current foot outside the box at a node of a run from step 0 (QP 2)
    i, j = _first_run_leg(contact[2])
    foot[2, j, i, 1] += 0.5
    u, feet, x, st, qi, si = eng.nlp_solve(x0, xref, foot, contact)
    assert st[1] == 7 and st[2] == 7 and all(st[q] == 0 for q in (0, 3))


@pytest.mark.gpu
def test_device_nlp_short_horizon_and_invalid_table(cm, op):
    """N = 5 (a one-class context, ld = 64, so the foothold QPs run in the workgroup condensing's 64 class) against
    the oracle, with one QP whose contact table has a flight step: INVALID_CONTACT ("mpc table invalid",
    CentroidalMPC.cpp:328-330), zero forces, the others unaffected."""
    N, B = 5, 12
    m, mo = cm.default_model(N), op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=1)
    contact[3, 2, :] = 0
    eng = cm.Engine(m, precision=0, max_batch=B)
    assert eng.ld == 64
    u, feet, x, st, qi, si = eng.nlp_solve(x0, xref, foot, contact, sqp_iter_max=10, sqp_tol=1e-7)
    s = op.default_settings()
    for q in range(B):
        ur, Dr, feetr, xr, sr, qir, sir = op.sqp_solve_feet(mo, s, x0[q], xref[q], foot[q], contact[q],
                                                            sqp_iter_max=10, sqp_tol=1e-7)
        assert st[q] == sr
        if q == 3:
            assert sr == 5 and not u[q].any()
            continue
        assert sr == 0
        assert rel_err(u[q], ur) < 1e-6, q
        assert np.abs(feet[q] - feetr).max() < 1e-8, q
