"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle on identical inputs.

Bars: bit-exact for the integer/byte work (input generator); fp64 contact forces within 1e-5 relative to
max(|u_ref|_inf, 1) (north_star), checked far tighter in practice; fp32 within 2e-3 relative.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20221125


def rel_err(u, ur):
    return float(np.max(np.abs(u - ur)) / max(1.0, float(np.max(np.abs(ur)))))


@pytest.mark.parametrize("gait", [0, 1])
def test_generator_bit_exact(cm, op, gait):
    for N in (10, 20):
        m = cm.default_model(N)
        mo = op.default_model(N)
        B = 257
        d = cm.generate_device(m, SEED, B, gait=gait, offset=12345)
        ho = op.generate(mo, SEED, B, gait=gait, offset=12345)
        for a, b in zip(d, ho):
            got = a.host()
            assert got.dtype == b.dtype
            assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(b).view(np.uint8)), "generator mismatch"


def test_generator_shard_invariance(cm):
    m = cm.default_model(10)
    full = [a.host() for a in cm.generate_device(m, SEED, 64, gait=1, offset=0)]
    part = [a.host() for a in cm.generate_device(m, SEED, 32, gait=1, offset=32)]
    for f, p in zip(full, part):
        assert np.array_equal(f[32:], p)


@pytest.mark.parametrize("precision", [0, 1])
@pytest.mark.parametrize("gait", [0, 1])
def test_condense_matches_oracle(cm, op, precision, gait):
    N = 10
    m = cm.default_model(N)
    mo = op.default_model(N)
    eng = cm.Engine(m, precision=precision, max_batch=64)
    x0, xref, foot, contact = op.generate(mo, SEED, 24, gait=gait)
    H, g, n, st = eng.condense(x0, xref, foot, contact)
    tol = 1e-12 if precision == 0 else 2e-5
    for q in range(24):
        nq, Hr, gr, mu, lo, hi, mp, sto = op.condense(mo, x0[q], xref[q], foot[q], contact[q], ld=eng.ld)
        assert st[q] == sto == 0
        assert n[q] == nq
        scale_h = np.abs(Hr[:nq, :nq]).max()
        scale_g = max(1.0, np.abs(gr[:nq]).max())
        assert np.abs(H[q, :nq, :nq] - Hr[:nq, :nq]).max() / scale_h < tol
        assert np.abs(g[q, :nq] - gr[:nq]).max() / scale_g < tol


def test_solve_fp64_trot_matches_oracle(cm, op):
    N = 10
    m, mo = cm.default_model(N), op.default_model(N)
    B = 128
    eng = cm.Engine(m, precision=0, max_batch=B)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=0)
    u, x, st, it = eng.solve(x0, xref, foot, contact)
    ur, xr, sr, itr = op.solve_batch(mo, op.default_settings(), x0, xref, foot, contact, nthreads=8)
    assert np.all(st == 0) and np.all(sr == 0)
    for q in range(B):
        assert rel_err(u[q], ur[q]) < 1e-5
    err = max(rel_err(u[q], ur[q]) for q in range(B))
    assert err < 1e-8, err
    assert np.abs(x - xr).max() < 1e-8
    # swing legs exactly zero (reference 0 <= F f <= 0 rows, CentroidalMPC.cpp:199)
    assert np.all(u[contact == 0] == 0.0)


def test_solve_fp64_mixed_gait_ragged(cm, op):
    N = 10
    m, mo = cm.default_model(N), op.default_model(N)
    B = 96
    eng = cm.Engine(m, precision=0, max_batch=B)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=1)
    u, x, st, it = eng.solve(x0, xref, foot, contact)
    ur, xr, sr, itr = op.solve_batch(mo, op.default_settings(), x0, xref, foot, contact, nthreads=8)
    nvar = 3 * contact.reshape(B, -1).sum(axis=1)
    assert set(np.unique(nvar)) >= {60, 120}
    assert np.all(st == sr)
    err = max(rel_err(u[q], ur[q]) for q in range(B))
    assert err < 1e-8, err


def test_solve_fp32_n20(cm, op):
    N = 20
    m, mo = cm.default_model(N), op.default_model(N)
    B = 64
    s = cm.default_settings(tol_stat=1e-3, tol_ineq=1e-4, tol_comp=1e-4)
    eng = cm.Engine(m, settings=s, precision=1, max_batch=B)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=0)
    u, x, st, it = eng.solve(x0, xref, foot, contact)
    ur, xr, sr, itr = op.solve_batch(mo, op.tight_settings(), x0, xref, foot, contact, nthreads=8)
    assert np.all(sr == 0)
    assert np.mean(st == 0) > 0.95
    err = max(rel_err(u[q], ur[q]) for q in range(B) if st[q] == 0)
    assert err < 2e-3, err


def test_invalid_contact_status(cm, op):
    N = 10
    m, mo = cm.default_model(N), op.default_model(N)
    eng = cm.Engine(m, precision=0, max_batch=8)
    x0, xref, foot, contact = op.generate(mo, SEED, 4, gait=0)
    contact[1, 3, :] = 0  # a flight step: reference throws "mpc table invalid" (CentroidalMPC.cpp:328-330)
    u, x, st, it = eng.solve(x0, xref, foot, contact)
    assert st[1] == 5 and np.all(u[1] == 0)
    assert st[0] == 0 and st[2] == 0 and st[3] == 0


def test_centoid_mpc_test_inputs(cm, op):
    import np_ref
    for N in (6, 10):
        m, mo = cm.default_model(N), op.default_model(N)
        x0, xref, foot, contact = np_ref.centoid_test_inputs(N)
        eng = cm.Engine(m, precision=0, max_batch=1)
        u, x, st, it = eng.solve(x0[None], xref[None], foot[None], contact[None])
        ur = np_ref.solve(np_ref.model_arrays(mo), x0, xref, foot, contact)
        assert st[0] == 0
        assert rel_err(u[0], ur) < 1e-8
