"""Fused condensing + IPM of the 64 < n <= 128 class (k_solve128: srbd_condense_qp and the k_ipm128x body on one
workgroup, LDS as one union; default for fp32, cmpc_set_path(CMPC_PATH_FUSED128, 1) forces it for fp64) against the two-launch path
(k_srbd_condense<T,128,4> + k_ipm128x, CMPC_PATH_FUSED128 = 0): the same arithmetic, so statuses, iteration counts and
forces are identical, on all-stance (n = 120), N = 20 trot (n = 120) and mixed-gait batches."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20221125


def _solve(cm, N, B, gait, precision, fused, all_stance=False):
    m = cm.default_model(N)
    s = cm.default_settings() if precision == cm.F64 else cm.default_settings(tol_stat=1e-3, tol_ineq=1e-3,
                                                                               tol_comp=1e-4)
    eng = cm.Engine(m, settings=s, precision=precision, max_batch=B, path={cm.PATH_FUSED128: fused})
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
def test_fused128_equals_two_launches(cm, N, B, gait, prec, all_stance):
    p = getattr(cm, prec)
    u0, st0, it0 = _solve(cm, N, B, gait, p, False, all_stance)
    u1, st1, it1 = _solve(cm, N, B, gait, p, True, all_stance)
    assert np.all(st0 == 0)
    np.testing.assert_array_equal(st1, st0)
    np.testing.assert_array_equal(it1, it0)
    np.testing.assert_array_equal(u1, u0)
