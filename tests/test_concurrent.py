"""Contexts solving on separate streams at once (the pipelined serving form of bench.py --inflight K): every context
owns its workspace, class lists and counters (cmpc_api.cpp: layout), so batches in flight on different streams must
give exactly the results each gives alone. Checked bit for bit against the same batches solved one at a time, which
the parity tests tie to the oracle."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 424242


def _batch(cm, model, seed, B, gait, offset):
    x0, xref, foot, contact = cm.generate_device(model, seed, B, gait=gait, offset=offset)
    return x0, xref, foot, contact


@pytest.mark.parametrize("precision", [0, 1])
def test_contexts_in_flight_on_separate_streams_bit_exact(cm, precision):
    N = 10 if precision == 0 else 20
    B = 1024
    model = cm.default_model(N)
    # fp32 at the tolerances bench.py uses for config 3
    settings = cm.default_settings() if precision == 0 else cm.default_settings(tol_stat=1e-3, tol_ineq=1e-3,
                                                                                 tol_comp=1e-4)
    H = cm.hip()
    # three batches of different gaits (the mixed one runs the n <= 64 and the 128 class in one call)
    batches = [_batch(cm, model, SEED + k, B, gait, k * B) for k, gait in enumerate((0, 1, 0))]
    K = len(batches)
    outs = [(cm.DeviceArray((B, N, 4, 3), np.float64), cm.DeviceArray((B,), np.int32), cm.DeviceArray((B,), np.int32))
            for _ in range(K)]

    # alone: one context, each batch solved and synchronised before the next
    solo = cm.Engine(model, settings, precision=precision, max_batch=B)
    ref = []
    for k in range(K):
        u, st, it = outs[k]
        solo.solve_device(B, *batches[k], u, None, st, it, None)
        H.hipDeviceSynchronize()
        ref.append((u.host().copy(), st.host().copy(), it.host().copy()))
        u.zero()
        st.zero()
        it.zero()
    H.hipDeviceSynchronize()

    # in flight: one context and one stream per batch, all launched before any synchronisation, three rounds
    engs = [cm.Engine(model, settings, precision=precision, max_batch=B) for _ in range(K)]
    streams = []
    for _ in range(K):
        sh = C.c_void_p()
        cm._hchk(H.hipStreamCreate(C.byref(sh)), "hipStreamCreate")
        streams.append(sh)
    try:
        for _ in range(3):
            for k in range(K):
                u, st, it = outs[k]
                engs[k].solve_device(B, *batches[k], u, None, st, it, streams[k])
        for sh in streams:
            cm._hchk(H.hipStreamSynchronize(sh), "hipStreamSynchronize")
        for k in range(K):
            u, st, it = outs[k]
            assert np.array_equal(st.host(), ref[k][1]), k
            assert np.array_equal(it.host(), ref[k][2]), k
            assert np.array_equal(u.host(), ref[k][0]), k
        for k in range(K):  # the batches really solve (not all-failed statuses)
            assert (ref[k][1] == 0).mean() > 0.9, (k, np.bincount(ref[k][1]))
    finally:
        for sh in streams:
            H.hipStreamDestroy(sh)
