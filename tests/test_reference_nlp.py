"""The reference's NLP transcribed literally (CentroidalMPC.cpp:102-234: every variable of the CasADi Opti problem --
com_pos, com_vel, angular_momentum at nodes 0..N, foot_pos at nodes 0..N and foot_vel, contact_force at steps 0..N-1
per leg -- with the multiple-shooting dynamics :159-176, the x0 / foot pinning :162-167, the step box :196-198, the
friction pyramid :199 and the cost :203-231) and solved by scipy's SLSQP in place of IPOPT, against the oracle's SQP
with foothold variables (oracle_sqp_solve_feet). This pins the reduced formulation the engine solves (footholds of
the later stance runs only, swing nodes at des_foot_pos, the bilinear lever arm in the rollout) against the
reference's own problem statement, independently of the restatement's algebra. CPU only."""
import numpy as np
import pytest

SEED = 20221125
NL = 4
G = 9.81


def ref_nlp(mo, x0, xref, foot, contact, fix_feet=None):
    """Objective / constraints of the reference NLP over z = [c, v, L (3 x (N+1) each), per leg: p (3 x (N+1)),
    pv (3 x N), f (3 x N)]; returns (f, df, eq constraints list, ineq constraints list, unpack). fix_feet
    [(N+1)][L][3]: foot_pos additionally pinned at every node (the frozen-foothold problem of cmpc_sqp_solve_batch)."""
    torch = pytest.importorskip("torch")
    N, dt, m = mo.N, mo.dt, mo.mass
    w = np.array(mo.weights[:45])
    mu = np.array(mo.mu[:4])
    ub = np.array(mo.force_ub[:5])
    nS = 3 * (N + 1)
    sizes = [nS, nS, nS] + [nS, 3 * N, 3 * N] * NL
    offs = np.cumsum([0] + sizes)
    nz = offs[-1]
    T = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64)  # noqa: E731
    X0, XR, FT, CT = T(x0), T(xref), T(foot), T(contact.astype(np.float64))
    step_lb = torch.tensor([-0.2, -0.2, -0.1], dtype=torch.float64)
    step_ub = torch.tensor([0.2, 0.2, 0.1], dtype=torch.float64)

    def unpack(z):
        parts = [z[offs[i]:offs[i + 1]] for i in range(len(sizes))]
        c, v, L = (p.reshape(N + 1, 3) for p in parts[:3])
        legs = [(parts[3 + 3 * i].reshape(N + 1, 3), parts[4 + 3 * i].reshape(N, 3), parts[5 + 3 * i].reshape(N, 3))
                for i in range(NL)]
        return c, v, L, legs

    wz = torch.tensor([(w[2] / 2) * np.exp(-k) + w[2] / 2 for k in range(N + 1)], dtype=torch.float64)
    ns = contact.sum(axis=1)
    fdes = np.zeros((NL, N, 3))
    for k in range(N):
        for i in range(NL):
            if contact[k, i]:
                fdes[i, k, 2] = m * G / ns[k]
    FD = T(fdes)
    # des_foot_pos node 0 only enters a constant term (:218-221); nodes 1..N are the record's des
    def cost(z):
        c, v, L, legs = unpack(z)
        dc, dv, dL = c - XR[:, 0:3], v - XR[:, 3:6], L - XR[:, 6:9]
        J = w[0] * (dc[:, 0] ** 2).sum() + w[1] * (dc[:, 1] ** 2).sum() + ((wz * dc[:, 2]) ** 2).sum()
        J = J + w[3] * (dv[:, 0] ** 2).sum() + w[4] * (dv[:, 1] ** 2).sum() + w[5] * (dv[:, 2] ** 2).sum()
        J = J + w[6] * (dL[:, 0] ** 2).sum() + w[7] * (dL[:, 1] ** 2).sum() + w[8] * (dL[:, 2] ** 2).sum()
        for i, (p, pv, f) in enumerate(legs):
            dp = p[1:] - FT[1:, i, :]
            for d in range(3):
                J = J + w[9 + 3 * i + d] * (dp[:, d] ** 2).sum()
                J = J + w[9 + 3 * NL + 3 * i + d] * ((f[:, d] - FD[i, :, d]) ** 2).sum()
                J = J + w[9 + 6 * NL + 3 * i + d] * ((f[1:, d] - f[:-1, d]) ** 2).sum()
        return J

    def eq(z):
        c, v, L, legs = unpack(z)
        out = [c[0] - X0[0:3], v[0] - X0[3:6], L[0] - X0[6:9]]
        acc = torch.zeros(N, 3, dtype=torch.float64)
        acc[:, 2] = -G
        tq = torch.zeros(N, 3, dtype=torch.float64)
        for i, (p, pv, f) in enumerate(legs):
            e = CT[:, i:i + 1]
            acc = acc + e * f / m
            tq = tq + e * torch.cross(p[:-1] - c[:-1], f, dim=1)
            out.append(p[0] - FT[0, i, :])
            out.append((p[1:] - (p[:-1] + (1 - e) * pv * dt)).reshape(-1))
        out.append((c[1:] - (c[:-1] + v[:-1] * dt)).reshape(-1))
        out.append((v[1:] - (v[:-1] + acc * dt)).reshape(-1))
        out.append((L[1:] - (L[:-1] + tq * dt)).reshape(-1))
        if fix_feet is not None:  # foot_vel pinned so that the swing integrator lands on the fixed positions
            FF = T(fix_feet)
            for i, (p, pv, f) in enumerate(legs):
                out.append((pv - (FF[1:, i, :] - FF[:-1, i, :]) / dt).reshape(-1))
        return torch.cat([o.reshape(-1) for o in out])

    Fm = [torch.tensor([[-1, 0, mu[i]], [1, 0, mu[i]], [0, -1, mu[i]], [0, 1, mu[i]], [0, 0, 1]],
                       dtype=torch.float64) for i in range(NL)]
    UB = T(ub)

    def ineq(z):  # >= 0
        c, v, L, legs = unpack(z)
        out = []
        for i, (p, pv, f) in enumerate(legs):
            dp = p[1:] - FT[1:, i, :]
            out += [(dp - step_lb).reshape(-1), (step_ub - dp).reshape(-1)]
            r = f @ Fm[i].T  # N x 5
            out += [r.reshape(-1), (UB[None, :] * CT[:, i:i + 1] - r).reshape(-1)]
        return torch.cat(out)

    def wrap(fn):
        def val(z):
            return fn(torch.as_tensor(z, dtype=torch.float64)).detach().numpy()

        def jac(z):
            zt = torch.as_tensor(z, dtype=torch.float64)
            return torch.autograd.functional.jacobian(fn, zt, vectorize=True).detach().numpy()
        return val, jac

    return nz, wrap(cost), wrap(eq), wrap(ineq), lambda z: unpack(torch.as_tensor(z, dtype=torch.float64))


def initial_guess(op, mo, x0, xref, foot, contact, nz, unpack):
    """The oracle's frozen-foothold QP solution, its rollout and the feet table, packed into z."""
    N, dt = mo.N, mo.dt
    u, x, st, _ = op.solve_batch(mo, op.default_settings(), x0[None], xref[None], foot[None], contact[None])
    feet = op.feet_table(mo, foot, contact, np.zeros((N, NL, 3)))
    parts = [x[0][:, 0:3], x[0][:, 3:6], x[0][:, 6:9]]
    for i in range(NL):
        pv = np.zeros((N, 3))
        for k in range(N):
            if not contact[k, i]:
                pv[k] = (feet[k + 1, i] - feet[k, i]) / dt
        parts += [feet[:, i, :], pv, u[0][:, i, :]]
    z = np.concatenate([np.asarray(p).reshape(-1) for p in parts])
    assert z.size == nz
    return z


@pytest.mark.parametrize("case", ["centoid_mpc_test", "trot", "mixed"])
def test_reference_nlp_matches_oracle_sqp_with_footholds(op, case):
    from scipy.optimize import minimize
    import os
    N = 6
    mo = op.default_model(N)
    if case == "centoid_mpc_test":
        with np.load(os.path.join(os.path.dirname(__file__), "golden", "centoid_mpc_test_N6.npz")) as z:
            x0, xref, foot, contact = z["x0"][0], z["xref"][0], z["foot"][0], z["contact"][0]
    else:
        x0, xref, foot, contact = (a[0] for a in op.generate(mo, SEED + 7, 1, gait=0 if case == "trot" else 1))
    nz, (fv, fj), (ev, ej), (iv, ij), unpack = ref_nlp(mo, x0, xref, foot, contact)
    z0 = initial_guess(op, mo, x0, xref, foot, contact, nz, unpack)
    res = minimize(fv, z0, jac=fj, method="SLSQP",
                   constraints=[{"type": "eq", "fun": ev, "jac": ej}, {"type": "ineq", "fun": iv, "jac": ij}],
                   options={"ftol": 1e-12, "maxiter": 500})
    assert res.success, res.message
    assert np.abs(ev(res.x)).max() < 1e-9 and iv(res.x).min() > -1e-9
    c, v, L, legs = unpack(res.x)
    f_ref = np.stack([legs[i][2].numpy() for i in range(NL)], axis=1)  # [N][L][3]
    p_ref = np.stack([legs[i][0].numpy() for i in range(NL)], axis=1)  # [N+1][L][3]
    # the reference optimum is a KKT point of the engine's formulation: the foothold QP linearised there returns it
    D_ref = np.zeros((N, NL, 3))
    for s0 in range(1, N):
        for i in range(NL):
            box = op.foot_box(foot, contact, s0, i)
            if box is not None:
                D_ref[s0, i] = p_ref[s0, i] - box[0]
    lin = op.nlp_rollout_cost_feet(mo, x0, xref, foot, contact, f_ref, D_ref)[2]
    n, H, g, mu_t, lo, hi, mp, stc = op.condense_feet(mo, x0, xref, foot, contact, lin, f_ref, D_ref)
    assert stc == 0
    zq = op.qp_ipm(n, H, g, mu_t, lo, hi, op.tight_settings())[0]
    zr = np.array([(f_ref.reshape(N * NL, 3)[c] if c < N * NL else D_ref.reshape(N * NL, 3)[c - N * NL])[d]
                   for c in mp[:n // 3] for d in range(3)])
    scale = max(1.0, np.abs(f_ref).max())
    assert np.abs(zq - zr).max() < 1e-5 * scale, np.abs(zq - zr).max()
    # the SQP (ocs2's settings; it stops at |J_new - J| < costTol = 1e-4) lands on it
    u, D, feet, x, st, qi, si = op.sqp_solve_feet(mo, op.default_settings(), x0, xref, foot, contact,
                                                  sqp_iter_max=50, sqp_tol=1e-10)
    assert st == 0
    assert np.abs(u - f_ref).max() < 2e-5 * scale, np.abs(u - f_ref).max()
    # footholds: every node of a stance run (the swing nodes' positions are free in the reference and track des)
    for i in range(NL):
        for j in range(1, N + 1):
            in_run = (j < N and contact[j, i]) or contact[j - 1, i]
            if in_run:
                assert np.abs(feet[j, i] - p_ref[j, i]).max() < 2e-5, (i, j)
            else:
                assert np.abs(p_ref[j, i] - foot[j, i]).max() < 2e-5, (i, j)
    # the states: the oracle's nonlinear rollout is the reference's trajectory
    assert np.abs(x[:, 0:3] - c.numpy()).max() < 1e-5 and np.abs(x[:, 6:9] - L.numpy()).max() < 1e-4


def test_reference_nlp_with_frozen_footholds_matches_oracle_sqp(op):
    """The same literal problem with foot_pos pinned at the frozen footholds (current foot / the run's mean des / des
    on swing nodes) is what cmpc_sqp_solve_batch solves: SLSQP's optimum vs oracle_sqp_solve."""
    from scipy.optimize import minimize
    N = 6
    mo = op.default_model(N)
    x0, xref, foot, contact = (a[0] for a in op.generate(mo, SEED + 11, 1, gait=1))
    fixed = op.feet_table(mo, foot, contact, np.zeros((N, NL, 3)))
    nz, (fv, fj), (ev, ej), (iv, ij), unpack = ref_nlp(mo, x0, xref, foot, contact, fix_feet=fixed)
    z0 = initial_guess(op, mo, x0, xref, foot, contact, nz, unpack)
    res = minimize(fv, z0, jac=fj, method="SLSQP",
                   constraints=[{"type": "eq", "fun": ev, "jac": ej}, {"type": "ineq", "fun": iv, "jac": ij}],
                   options={"ftol": 1e-12, "maxiter": 500})
    assert res.success, res.message
    f_ref = np.stack([unpack(res.x)[3][i][2].numpy() for i in range(NL)], axis=1)
    u, x, st, qi, si = op.sqp_solve(mo, op.default_settings(), x0, xref, foot, contact, sqp_iter_max=50, sqp_tol=1e-10)
    assert st == 0
    assert np.abs(u - f_ref).max() < 2e-5 * max(1.0, np.abs(f_ref).max()), np.abs(u - f_ref).max()
