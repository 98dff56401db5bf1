"""Opt-in work-item form of the fused n <= 64 path (k_solve64q, CMPC_ITEMS=1 at cmpc_create; k_ipm64.hpp): every
IPM iteration of a QP is one item of a per-CU FIFO in LDS, parking the QP's state in the workspace between items.
Each item runs the same arithmetic as k_solve64 (one wave per QP, cmpc_solve_batch), so the two paths must agree
QP by QP: same status, same iteration count, forces equal to fp64 rounding. Checked at one item per iteration and
at several iterations per item (CMPC_ITEMS_PERIOD), on uniform and mixed-gait batches (ragged n per QP, several
workgroups), and at the headline size."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20221125


def _solve(cm, N, B, gait, monkeypatch, items, period=None):
    monkeypatch.setenv("CMPC_ITEMS", "1" if items else "0")
    if period is not None:
        monkeypatch.setenv("CMPC_ITEMS_PERIOD", str(period))
    else:
        monkeypatch.delenv("CMPC_ITEMS_PERIOD", raising=False)
    m = cm.default_model(N)
    eng = cm.Engine(m, precision=cm.F64, max_batch=B)
    assert cm.lib().cmpc_ctx_fused(eng.ctx) == 1
    x0, xref, foot, contact = cm.generate_device(m, SEED, B, gait=gait)
    u = cm.DeviceArray((B, N, 4, 3), np.float64)
    st = cm.DeviceArray((B,), np.int32)
    it = cm.DeviceArray((B,), np.int32)
    eng.solve_device(B, x0, xref, foot, contact, u, None, st, it)
    cm.hip().hipDeviceSynchronize()
    return u.host(), st.host(), it.host()


@pytest.mark.parametrize("N,B,gait,period", [(6, 37, 0, None), (10, 600, 1, None), (10, 600, 1, 3),
                                             (10, 4096, 0, None)])
def test_items_match_fused_kernel(cm, monkeypatch, N, B, gait, period):
    u0, st0, it0 = _solve(cm, N, B, gait, monkeypatch, items=False)
    u1, st1, it1 = _solve(cm, N, B, gait, monkeypatch, items=True, period=period)
    np.testing.assert_array_equal(st1, st0)
    np.testing.assert_array_equal(it1, it0)
    scale = max(1.0, float(np.abs(u0).max()))
    np.testing.assert_allclose(u1, u0, rtol=0, atol=1e-9 * scale)
