"""Warm start across MPC ticks (hpipm_interface::Settings::warm_start, HpipmInterfaceSettings.h:54,
HPIPM warm_start = 1: primal initial guess, slacks of C u clipped, lam = mu0 / t). The oracle restates the warm
initial point (oracle_qp_ipm); the device kernels of all three size classes must follow it iteration for iteration."""
import numpy as np
import pytest

SEED = 20221125


def rel_err(u, ur):
    return float(np.max(np.abs(u - ur)) / max(1.0, float(np.max(np.abs(ur)))))


def test_oracle_warm_start_same_optimum_fewer_iterations(op):
    N, B = 10, 24
    mo = op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=1)
    cold = op.default_settings()
    warm = op.default_settings(warm_start=1)
    u, _, st, it = op.solve_batch(mo, cold, x0, xref, foot, contact, nthreads=4, want_x=False)
    assert np.all(st == 0)
    rng = np.random.default_rng(1)
    guess = u * (1.0 + 0.05 * rng.standard_normal(u.shape))
    uw, _, stw, itw = op.solve_batch(mo, warm, x0, xref, foot, contact, nthreads=4, want_x=False, u_init=guess)
    assert np.all(stw == 0)
    assert max(rel_err(uw[q], u[q]) for q in range(B)) < 1e-6
    assert itw.mean() < it.mean()
    # warm_start = 0 ignores the guess
    uc, _, _, itc = op.solve_batch(mo, cold, x0, xref, foot, contact, nthreads=4, want_x=False, u_init=guess)
    assert np.array_equal(uc, u) and np.array_equal(itc, it)


@pytest.mark.gpu
@pytest.mark.parametrize("N,all_stance", [(10, False), (10, True), (20, True)])
def test_device_warm_start_matches_oracle(cm, op, N, all_stance):
    """n = 60 (k_ipm64), 120 (128 class), 240 (256 class)."""
    B = 32
    m, mo = cm.default_model(N), op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=0)
    if all_stance:
        contact[:] = 1
    cold = op.default_settings()
    u, _, st, it = op.solve_batch(mo, cold, x0, xref, foot, contact, nthreads=8, want_x=False)
    rng = np.random.default_rng(2)
    guess = u * (1.0 + 0.05 * rng.standard_normal(u.shape)) + 0.5 * rng.standard_normal(u.shape)
    ws = op.default_settings(warm_start=1)
    ur, _, sr, itr = op.solve_batch(mo, ws, x0, xref, foot, contact, nthreads=8, want_x=False, u_init=guess)
    eng = cm.Engine(m, settings=cm.default_settings(warm_start=1), precision=0, max_batch=B)
    ud, _, sd, itd = eng.solve(x0, xref, foot, contact, want_x=False, u_init=guess)
    assert np.all(sd == sr) and np.all(sd == 0)
    assert np.abs(itd - itr).max() <= 1
    assert max(rel_err(ud[q], ur[q]) for q in range(B)) < 1e-6
    assert itd.mean() < it.mean()
    # same engine, warm_start = 0 -> the guess is ignored (cold path)
    eng.set_settings(cm.default_settings())
    uc, _, sc, itc = eng.solve(x0, xref, foot, contact, want_x=False, u_init=guess)
    assert np.all(itc == it) or np.abs(itc - it).max() <= 1


@pytest.mark.gpu
def test_shift_inputs_and_closed_loop_ticks(cm, op):
    """Receding horizon: tick t+1 starts from tick t's solution shifted one step (cmpc_shift_inputs)."""
    N, B = 10, 64
    m, mo = cm.default_model(N), op.default_model(N)
    u = np.random.default_rng(3).standard_normal((B, N, 4, 3))
    s = cm.shift_inputs(u, 1)
    assert np.array_equal(s[:, :-1], u[:, 1:]) and np.array_equal(s[:, -1], u[:, -1])
    assert np.array_equal(cm.shift_inputs(u, 0), u)
    # tick 0 (cold) and tick 1 = the same robots one step later: x0 <- rollout x1, references shifted
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=0)
    eng = cm.Engine(m, settings=cm.default_settings(warm_start=1), precision=0, max_batch=B)
    u0, x, st0, it0 = eng.solve(x0, xref, foot, contact)
    assert np.all(st0 == 0)
    x1 = x[:, 1]
    xref1 = np.concatenate([xref[:, 1:], xref[:, -1:]], axis=1)
    foot1 = np.concatenate([foot[:, 1:], foot[:, -1:]], axis=1)
    contact1 = np.concatenate([contact[:, 1:], contact[:, :1]], axis=1)
    cold = eng.solve(x1, xref1, foot1, contact1)
    guess = cm.shift_inputs(u0, 1)
    warm = eng.solve(x1, xref1, foot1, contact1, u_init=guess)
    eng.set_settings(cm.default_settings())
    cold = eng.solve(x1, xref1, foot1, contact1)
    assert np.all(warm[2] == 0) and np.all(cold[2] == 0)
    assert max(rel_err(warm[0][q], cold[0][q]) for q in range(B)) < 1e-5
    assert warm[3].mean() < cold[3].mean()
