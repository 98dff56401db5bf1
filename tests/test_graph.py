"""The hot path under HIP stream capture (MI355X guide: capture launch-bound loops in hipGraphs): cmpc_solve_batch is
captured once into a graph and the graph replayed; every replay reproduces the direct call bit for bit, on a mixed
batch that uses the fused n <= 64 kernel's appended class lists (whose counters must be re-zeroed inside the graph)."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20221125


def test_solve_batch_graph_replay_bit_exact(cm, op):
    N, B = 10, 512
    m, mo = cm.default_model(N), op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=1)  # mixed: n <= 64 and 64 < n <= 128
    eng = cm.Engine(m, precision=0, max_batch=B)
    u_ref, _, st_ref, it_ref = eng.solve(x0, xref, foot, contact, want_x=False)
    assert len(set((3 * contact.reshape(B, -1).sum(axis=1)).tolist())) > 1
    H = cm.hip()
    H.hipStreamBeginCapture.argtypes = [C.c_void_p, C.c_int]
    H.hipStreamEndCapture.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
    H.hipGraphInstantiate.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_void_p, C.c_char_p, C.c_size_t]
    H.hipGraphLaunch.argtypes = [C.c_void_p, C.c_void_p]
    H.hipGraphExecDestroy.argtypes = [C.c_void_p]
    H.hipGraphDestroy.argtypes = [C.c_void_p]
    d = [cm.DeviceArray.from_host(np.asarray(a, t)) for a, t in
         ((x0, np.float64), (xref, np.float64), (foot, np.float64), (contact, np.uint8))]
    u = cm.DeviceArray((B, N, 4, 3), np.float64)
    st = cm.DeviceArray((B,), np.int32)
    it = cm.DeviceArray((B,), np.int32)
    s = C.c_void_p()
    assert H.hipStreamCreate(C.byref(s)) == 0
    graph, exe = C.c_void_p(), C.c_void_p()
    assert H.hipStreamBeginCapture(s, 0) == 0  # hipStreamCaptureModeGlobal
    rc = cm.lib().cmpc_solve_batch(eng.ctx, B, d[0].ptr, d[1].ptr, d[2].ptr, d[3].ptr, u.ptr, None, st.ptr, it.ptr, s)
    assert H.hipStreamEndCapture(s, C.byref(graph)) == 0 and rc == 0
    assert H.hipGraphInstantiate(C.byref(exe), graph, None, None, 0) == 0
    for _ in range(5):
        u.zero()
        assert H.hipGraphLaunch(exe, s) == 0
        assert H.hipStreamSynchronize(s) == 0
        assert np.array_equal(u.host(), u_ref) and np.array_equal(st.host(), st_ref) and np.array_equal(it.host(), it_ref)
    # direct calls on the same context after the replays still agree
    u2, _, st2, _ = eng.solve(x0, xref, foot, contact, want_x=False)
    assert np.array_equal(u2, u_ref) and np.array_equal(st2, st_ref)
    H.hipGraphExecDestroy(exe)
    H.hipGraphDestroy(graph)
