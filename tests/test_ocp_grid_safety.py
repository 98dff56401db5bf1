"""The grid form of the HpipmInterface::solve path (batches up to 32, the MPC tick's B = 1) when the device is shared.

The grid form runs one problem on G workgroups that meet at grid barriers, so it needs them all resident at once.
cmpc_ocp_grid caps G by the kernel's occupancy on the device; kernels of other streams can still hold CUs when a tick
starts. Each barrier therefore waits a bounded time (cmpc_ocp_set_grid_timeout), a timed-out grid drains with the
internal status CMPC_GRID_TIMEOUT (never NAN_SOL, which the caller would read as a numerical failure:
MultipleShootingSolver.cpp:283-285 throws on it), and the same cmpc_ocp_solve re-solves such a problem on one
workgroup (k_ocp_fallback). The status contract of HpipmInterface.cpp:290-300 holds throughout: the caller sees the
solver's own status.

Checked here against the oracle (oracle/ocp_ipm.c) and against the one-workgroup form bit for bit.
"""
import ctypes as C

import numpy as np
import pytest

from cheeta_mpc import ocp as ocpgen
from test_ocp_ipm import _check_vs_oracle, _device_batch, _device_batch_path, _rel, _small

pytestmark = pytest.mark.gpu


def _solve(h, ps):
    recs, crecs = zip(*[ocpgen.pack(p) for p in ps])
    return h.solve(np.array([p["x0"] for p in ps]), np.array(recs), np.array(crecs) if ps[0].get("nc") else None)


@pytest.mark.parametrize("projected", [True, False])
def test_device_forced_grid_timeout_falls_back_once(cm, op, projected):
    """Every grid barrier forced to time out (the debug switch): the grid drains at its first barrier and the fallback
    launch re-solves each problem on one workgroup — SUCCESS, the one-workgroup form's result bit for bit, the oracle's
    at 1e-9, one fallback per problem; the kept Riccati quantities are the fallback's (refactorised at the exit point),
    equal to the one-workgroup solve's refactorisation. With the switch off again the grid form runs and nothing falls
    back."""
    ps = [ocpgen.legged_problem(560 + i, projected=projected) for i in range(2)]
    p0 = ps[0]
    s1, x1, u1, st1, it1 = _device_batch_path(cm, ps, 1, grid=1)
    ric1 = s1.riccati(2)
    h = cm.OcpSolver(p0["N"], p0["nx"], p0["nu"], p0.get("nc"), max_batch=2)
    h.set_keep_riccati(1)
    assert h.grid(2) >= 2
    assert h.fallback_count == 0
    h.force_grid_timeout(1)
    x, u, st, it = _solve(h, ps)
    assert h.fallback_count == 2
    assert np.all(st == 0) and np.array_equal(st, st1) and np.array_equal(it, it1)
    assert np.array_equal(x, x1) and np.array_equal(u, u1)
    _check_vs_oracle(op, ps, x, u, st, it)
    P, pv, K, kf, Lr, rst = h.riccati(2)
    assert np.all(rst == 0)
    tS = 1e-4 if p0.get("nc") else 1e-9
    for i in range(2):
        for k in range(1, p0["N"] + 1):
            assert _rel(P[i][k], ric1[0][i][k]) < tS, ("P", k)
        for k in range(1, p0["N"]):
            assert _rel(K[i][k], ric1[2][i][k]) < tS and _rel(Lr[i][k], ric1[4][i][k]) < tS, ("K, Lr", k)
    Kf, Mf, P1, sf = h.riccati_feedback(1)
    assert sf == 0 and _rel(P1, ric1[0][1][1]) < tS
    h.force_grid_timeout(0)
    x2, u2, st2, it2 = _solve(h, ps)
    assert h.fallback_count == 2  # the grid form ran
    assert np.array_equal(st2, st1) and np.array_equal(it2, it1)
    for i in range(2):
        assert _rel(x2[i], x1[i]) < 1e-10 and _rel(u2[i], u1[i]) < 1e-10
    h.close()


def test_device_grid_solve_beside_a_long_centroidal_batch(cm, op):
    """A B = 1 tick through the grid form while a long centroidal batch (four 65536-QP calls, ~30 ms) occupies the
    device from another stream: SUCCESS with the oracle's result, whether the grid found its CUs or timed out (1 ms
    bound here) and fell back; the centroidal batch is unaffected (statuses equal to a solve alone)."""
    H = cm.hip()
    N, B = 10, 65536
    model = cm.default_model(N)
    eng = cm.Engine(model, cm.default_settings(), precision=cm.F64, max_batch=B)
    x0, xref, foot, contact = cm.generate_device(model, 99, B, gait=0)
    u = cm.DeviceArray((B, N, 4, 3), np.float64)
    st = cm.DeviceArray((B,), np.int32)
    it = cm.DeviceArray((B,), np.int32)
    eng.solve_device(B, x0, xref, foot, contact, u, None, st, it, None)
    cm._hchk(H.hipDeviceSynchronize(), "hipDeviceSynchronize")
    st_alone = st.host().copy()
    p = ocpgen.legged_problem(570, projected=False)
    h = cm.OcpSolver(p["N"], p["nx"], p["nu"], p.get("nc"), max_batch=1)
    h.set_grid_timeout(1000.0)
    assert h.grid(1) >= 2
    stream = C.c_void_p()
    cm._hchk(H.hipStreamCreateWithFlags(C.byref(stream), 1), "hipStreamCreateWithFlags")
    try:
        results = []
        for rep in range(3):
            for _ in range(4):
                eng.solve_device(B, x0, xref, foot, contact, u, None, st, it, stream)
            results.append(_solve(h, [p]))  # the handle's own stream, while the batch runs
            cm._hchk(H.hipStreamSynchronize(stream), "hipStreamSynchronize")
            assert np.array_equal(st.host(), st_alone), rep
        for x1, u1, st1, it1 in results:
            _check_vs_oracle(op, [p], x1, u1, st1, it1)
        print(f"grid beside the batch: {h.fallback_count} of {len(results)} ticks fell back")
    finally:
        H.hipStreamDestroy(stream)
        h.close()
        eng.close()


def test_device_reshape_into_latency_limits_zeroes_barriers(cm, op):
    """A handle created outside the latency form's limits (nx = 28 > 27: no grid form, no barrier words) and reshaped
    into them gets its grid barrier words allocated then, zeroed (they were zeroed only at create): the
    grid-form solves on it equal a fresh handle's bit for bit and the oracle's, with no fallback."""
    wide = [_small(780 + i, N=5, nx=28, nu=[6] * 5) for i in range(2)]
    h = cm.OcpSolver(wide[0]["N"], wide[0]["nx"], wide[0]["nu"], wide[0].get("nc"), max_batch=2)
    assert h.grid(2) == 0
    xw, uw, stw, itw = _solve(h, wide)
    _check_vs_oracle(op, wide, xw, uw, stw, itw)
    for t in range(3):
        ps = [ocpgen.legged_problem(790 + 10 * t + i, projected=bool(t % 2)) for i in range(2)]
        p0 = ps[0]
        h.reshape(p0["N"], p0["nx"], p0["nu"], p0.get("nc"))
        assert h.grid(2) >= 2
        x, u, st, it = _solve(h, ps)
        f, xf, uf, stf, itf = _device_batch(cm, ps)
        f.close()
        assert np.array_equal(st, stf) and np.array_equal(it, itf), t
        assert np.array_equal(x, xf) and np.array_equal(u, uf), t
        _check_vs_oracle(op, ps, x, u, st, it)
    assert h.fallback_count == 0
    h.close()


def test_device_staging_views_invalidated_by_reshape(cm, op):
    """cmpc_ocp_staging's pointers are valid until the next reshape / destroy (cmpc.h): the Python views handed out
    before a reshape become read-only and a solve refuses them; views fetched again after the reshape work."""
    p = ocpgen.legged_problem(800, projected=True)
    rec, _ = ocpgen.pack(p)
    h = cm.OcpSolver(p["N"], p["nx"], p["nu"], None, max_batch=1)
    sx0, srec, _ = h.staging()
    sx0[0] = p["x0"]
    srec[0] = rec
    x1, u1, st1, _ = h.solve(sx0[:1], srec[:1])
    q = ocpgen.legged_problem(801, projected=True, t0=0.015)
    qrec, _ = ocpgen.pack(q)
    h.reshape(q["N"], q["nx"], q["nu"])
    assert not srec.flags.writeable
    with pytest.raises(RuntimeError):
        h.solve(q["x0"][None], srec[:1])
    tx0, trec, _ = h.staging()
    tx0[0] = q["x0"]
    trec[0] = qrec
    x2, u2, st2, _ = h.solve(tx0[:1], trec[:1])
    xr, ur, str_, _ = h.solve(q["x0"][None], qrec[None])
    assert st1[0] == st2[0] == str_[0] == 0
    assert np.array_equal(x2, xr) and np.array_equal(u2, ur)
    h.close()
