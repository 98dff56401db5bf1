"""Fused condensing + IPM of the 64 < n <= 128 class (k_solve128: srbd_condense_qp and the k_ipm128x body on one
workgroup, LDS as one union; default for fp32, CMPC_FUSED128=1 forces it for fp64) against the two-launch path
(k_srbd_condense<T,128,4> + k_ipm128x, CMPC_FUSED128=0): the same arithmetic, so statuses, iteration counts and
forces are identical, on all-stance (n = 120), N = 20 trot (n = 120) and mixed-gait batches."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20221125


def _solve(cm, N, B, gait, precision, monkeypatch, fused, all_stance=False):
    monkeypatch.setenv("CMPC_FUSED128", "1" if fused else "0")
    m = cm.default_model(N)
    s = cm.default_settings() if precision == cm.F64 else cm.default_settings(tol_stat=1e-3, tol_ineq=1e-3,
                                                                               tol_comp=1e-4)
    eng = cm.Engine(m, settings=s, precision=precision, max_batch=B)
    x0, xref, foot, contact = cm.generate_device(m, SEED, B, gait=gait)
    if all_stance:
        contact = cm.DeviceArray.from_host(np.ones_like(contact.host()))
    u = cm.DeviceArray((B, N, 4, 3), np.float64)
    st = cm.DeviceArray((B,), np.int32)
    it = cm.DeviceArray((B,), np.int32)
    eng.solve_device(B, x0, xref, foot, contact, u, None, st, it)
    cm.hip().hipDeviceSynchronize()
    return u.host(), st.host(), it.host()


@pytest.mark.parametrize("N,B,gait,prec,all_stance", [(10, 48, 0, "F64", True), (10, 200, 1, "F64", False),
                                                      (20, 64, 0, "F32", False), (10, 48, 0, "F32", True)])
def test_fused128_equals_two_launches(cm, monkeypatch, N, B, gait, prec, all_stance):
    p = getattr(cm, prec)
    u0, st0, it0 = _solve(cm, N, B, gait, p, monkeypatch, False, all_stance)
    u1, st1, it1 = _solve(cm, N, B, gait, p, monkeypatch, True, all_stance)
    assert np.all(st0 == 0)
    np.testing.assert_array_equal(st1, st0)
    np.testing.assert_array_equal(it1, it0)
    np.testing.assert_array_equal(u1, u0)


@pytest.mark.parametrize("N,B,gait,prec,all_stance", [(10, 300, 1, "F64", False), (20, 96, 0, "F32", False),
                                                      (12, 64, 1, "F64", False), (10, 4096, 0, "F64", False)])
def test_forked_bigger_classes_equal_serial(cm, monkeypatch, N, B, gait, prec, all_stance):
    """CMPC_FORK=1: the bigger classes run on a side stream beside k_solve64 from class lists built off the contact
    tables; the same kernels solve the same QPs, so statuses, iteration counts and forces equal the serial path bit for
    bit (mixed gait with rejected tables, N = 20 fp32, N = 12 with the 256 class, the headline batch)."""
    p = getattr(cm, prec)
    m = cm.default_model(N)
    s = cm.default_settings() if p == cm.F64 else cm.default_settings(tol_stat=1e-3, tol_ineq=1e-3, tol_comp=1e-4)
    x0, xref, foot, contact = cm.generate_device(m, SEED, B, gait=gait)
    ct = contact.host()
    ct[1] = 0  # rejected tables: no stance leg at any step
    ct[3, 2] = 0
    contact = cm.DeviceArray.from_host(ct)
    out = {}
    for fork in ("0", "1"):
        monkeypatch.setenv("CMPC_FORK", fork)
        eng = cm.Engine(m, settings=s, precision=p, max_batch=B)
        for rep in range(2):  # repeated calls reuse the lists and the side stream
            u = cm.DeviceArray((B, N, 4, 3), np.float64)
            st = cm.DeviceArray((B,), np.int32)
            it = cm.DeviceArray((B,), np.int32)
            eng.solve_device(B, x0, xref, foot, contact, u, None, st, it)
            cm.hip().hipDeviceSynchronize()
            out[(fork, rep)] = (u.host(), st.host(), it.host())
    u0, st0, it0 = out[("0", 1)]
    assert st0[1] == 5 and st0[3] == 5
    for key in (("1", 0), ("1", 1), ("0", 0)):
        u1, st1, it1 = out[key]
        np.testing.assert_array_equal(st1, st0)
        np.testing.assert_array_equal(it1, it0)
        np.testing.assert_array_equal(u1, u0)
