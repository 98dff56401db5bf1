"""BASELINE.json configs at their full sizes on the device (B = 4096; config 4's per-GPU share B = 32768), checked
through size-independent properties: every QP succeeds, iteration counts stay in the oracle's range, swing forces
are exactly zero, stance forces satisfy the friction pyramid / normal-force bounds (CentroidalMPC.cpp:179-201) to the
IPM tolerance, the normal forces of each step carry the body weight on average, and a seeded sample of QPs matches
the CPU oracle (the full batch would take the oracle minutes). Inputs come from the device generator, which is
bit-identical to the oracle's (test_gpu_parity.py::test_generator_bit_exact)."""
import numpy as np
import pytest

SEED = 20221125


def _run(cm, N, B, gait, precision, seed=SEED):
    m = cm.default_model(N)
    s = cm.default_settings() if precision == 0 else cm.default_settings(tol_stat=1e-3, tol_ineq=1e-3, tol_comp=1e-4)
    eng = cm.Engine(m, settings=s, precision=precision, max_batch=B)
    x0, xref, foot, contact = cm.generate_device(m, seed, B, gait=gait)
    u = cm.DeviceArray((B, N, 4, 3), np.float64)
    st = cm.DeviceArray((B,), np.int32)
    it = cm.DeviceArray((B,), np.int32)
    eng.solve_device(B, x0, xref, foot, contact, u, None, st, it)
    cm.hip().hipDeviceSynchronize()
    return (x0.host(), xref.host(), foot.host(), contact.host()), u.host(), st.host(), it.host()


def _check_properties(u, st, it, contact, mu=0.8, ub=(5000.0,) * 4 + (8.0 * 9.81 * 4,), tol=1e-6):
    assert np.all(st == 0)
    assert it.min() >= 3 and it.max() <= 30
    assert np.all(u[contact == 0] == 0.0)
    f = u[contact == 1]
    rows = np.stack([mu * f[:, 2] - f[:, 0], mu * f[:, 2] + f[:, 0], mu * f[:, 2] - f[:, 1], mu * f[:, 2] + f[:, 1],
                     f[:, 2]], 1)
    assert rows.min() >= -tol * max(1.0, np.abs(f).max())
    assert (np.array(ub)[None] - rows).min() >= -tol * max(1.0, np.abs(f).max())
    # stance normal forces carry the weight (force tracking to m g / n_stance, CentroidalMPC.cpp:326-335)
    fz_step = u[..., 2].sum(axis=2)  # [B, N]
    assert abs(fz_step.mean() / (8.0 * 9.81) - 1.0) < 0.25


def _sample_vs_oracle(op, N, inputs, u, st, it, idx, tol, iters_exact):
    x0, xref, foot, contact = (a[idx] for a in inputs)
    mo = op.default_model(N)
    ur, _, sr, itr = op.solve_batch(mo, op.default_settings() if tol < 1e-4 else op.tight_settings(), x0, xref, foot,
                                    contact, nthreads=8, want_x=False)
    assert np.all(sr == 0)
    err = np.abs(u[idx] - ur).reshape(len(idx), -1).max(1) / np.maximum(1.0, np.abs(ur).reshape(len(idx), -1).max(1))
    assert err.max() < tol, err.max()
    if iters_exact:
        assert np.abs(it[idx] - itr).max() <= 1


@pytest.mark.gpu
@pytest.mark.parametrize("name,N,B,gait,precision", [("config2_trot_f64", 10, 4096, 0, 0),
                                                      ("config3_trot_n20_f32", 20, 4096, 0, 1),
                                                      ("config5_mixed_f64", 10, 4096, 1, 0),
                                                      ("config4_share_b32768_f64", 10, 32768, 0, 0)])
def test_full_size_config(cm, op, name, N, B, gait, precision):
    inputs, u, st, it = _run(cm, N, B, gait, precision)
    _check_properties(u, st, it, inputs[3], tol=1e-6 if precision == 0 else 2e-3)
    idx = np.sort(np.random.default_rng(B + N + gait).choice(B, 48, replace=False))
    _sample_vs_oracle(op, N, inputs, u, st, it, idx, 1e-8 if precision == 0 else 2e-3, precision == 0)


@pytest.mark.gpu
def test_batch_edges(cm, op):
    """B = 0 is a no-op; B = max_batch is accepted; B > max_batch is CMPC_ERR_ARG; a single QP (B = 1, the
    UpdateMPC call) equals its row of a larger batch bit for bit."""
    N = 10
    m = cm.default_model(N)
    eng = cm.Engine(m, precision=0, max_batch=8)
    x0, xref, foot, contact = cm.generate_device(m, SEED, 8)
    u = cm.DeviceArray((8, N, 4, 3), np.float64)
    st = cm.DeviceArray((8,), np.int32)
    it = cm.DeviceArray((8,), np.int32)
    L = cm.lib()
    assert L.cmpc_solve_batch(eng.ctx, 0, x0.ptr, xref.ptr, foot.ptr, contact.ptr, u.ptr, None, st.ptr, it.ptr,
                              None) == 0
    assert L.cmpc_solve_batch(eng.ctx, 9, x0.ptr, xref.ptr, foot.ptr, contact.ptr, u.ptr, None, st.ptr, it.ptr,
                              None) == -1
    eng.solve_device(8, x0, xref, foot, contact, u, None, st, it)
    cm.hip().hipDeviceSynchronize()
    u8, st8 = u.host(), st.host()
    assert np.all(st8 == 0)
    hx = [a.host() for a in (x0, xref, foot, contact)]
    for q in (0, 5):
        u1, _, s1, _ = eng.solve(*(a[q:q + 1] for a in hx), want_x=False)
        assert s1[0] == 0 and np.array_equal(u1[0], u8[q])
