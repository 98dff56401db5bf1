"""Result scatter in the IPM kernels' epilogues (fused cold-start path without rollout: k_solve64, k_ipm128x and
k_ipm_tiled write u[N][4][3], status and iterations themselves; no k_expand launch) against the k_expand path
(cmpc_set_path(CMPC_PATH_DIRECT, 0)): identical outputs, bit for bit, on batches that reach every size class (N = 10 and
N = 20 mixed gaits: n <= 64, 64 < n <= 128, 128 < n <= 256) and carry rejected QPs (a step without a stance leg:
INVALID_CONTACT, zero forces, zero iterations)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20221125


def _solve(cm, N, B, gait, direct, invalid=()):
    m = cm.default_model(N)
    eng = cm.Engine(m, precision=cm.F64, max_batch=B, path={cm.PATH_DIRECT: direct})
    x0, xref, foot, contact = cm.generate_device(m, SEED, B, gait=gait)
    if invalid:
        c = contact.host()
        for q in invalid:
            c[q, N // 2, :] = 0  # one step in flight: "mpc table invalid" (CentroidalMPC.cpp:328-330)
        contact = cm.DeviceArray.from_host(c)
    u = cm.DeviceArray((B, N, 4, 3), np.float64)
    u.upload(np.full((B, N, 4, 3), 7.0))  # stale values: every entry must be written
    st = cm.DeviceArray((B,), np.int32)
    it = cm.DeviceArray((B,), np.int32)
    eng.solve_device(B, x0, xref, foot, contact, u, None, st, it)
    cm.hip().hipDeviceSynchronize()
    return u.host(), st.host(), it.host()


@pytest.mark.parametrize("N,B,gait", [(10, 300, 1), (20, 96, 1), (10, 64, 0)])
def test_direct_results_equal_expand_path(cm, N, B, gait):
    bad = (3, 17, B - 1)
    u0, st0, it0 = _solve(cm, N, B, gait, direct=False, invalid=bad)
    u1, st1, it1 = _solve(cm, N, B, gait, direct=True, invalid=bad)
    np.testing.assert_array_equal(st1, st0)
    np.testing.assert_array_equal(it1, it0)
    np.testing.assert_array_equal(u1, u0)
    assert np.all(st1[list(bad)] == 5)  # INVALID_CONTACT
    assert np.all(u1[list(bad)] == 0.0) and np.all(it1[list(bad)] == 0)
    assert np.all(st1[[q for q in range(B) if q not in bad]] == 0)


def test_repeated_calls_with_class_lists(cm):
    """The fused path appends the bigger classes' QPs to lists with two alternating counter sets (each call zeroes
    the next call's): repeated calls, a warm-start (unfused, k_class_lists) call and a rollout call in between, and
    a smaller batch must all give the first call's results."""
    N, B = 20, 96
    m = cm.default_model(N)
    eng = cm.Engine(m, precision=cm.F64, max_batch=B)
    x0, xref, foot, contact = cm.generate_device(m, SEED, B, gait=1)

    def run(Bc=B, u_init=None, x=None):
        u = cm.DeviceArray((Bc, N, 4, 3), np.float64)
        st = cm.DeviceArray((Bc,), np.int32)
        it = cm.DeviceArray((Bc,), np.int32)
        eng.solve_device(Bc, x0, xref, foot, contact, u, x, st, it, u_init=u_init)
        cm.hip().hipDeviceSynchronize()
        return u, st.host(), it.host()

    u_ref, st_ref, it_ref = run()
    assert np.all(st_ref == 0)
    uh = u_ref.host()
    for k in range(3):
        u, st, it = run()
        np.testing.assert_array_equal(st, st_ref)
        np.testing.assert_array_equal(it, it_ref)
        np.testing.assert_array_equal(u.host(), uh)
        if k == 0:
            run(u_init=u_ref)  # warm start: the unfused path with k_class_lists
        if k == 1:
            run(x=cm.DeviceArray((B, N + 1, 13), np.float64))  # rollout: k_expand after the fused kernels
    u, st, it = run(Bc=40)
    np.testing.assert_array_equal(st, st_ref[:40])
    np.testing.assert_array_equal(u.host(), uh[:40])
