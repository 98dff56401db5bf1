"""GPU parity of the 64 < n <= 128 size class (k_ipm128x, four waves per QP) at condensed sizes chosen to hit its
edges: just above the one-wave class (n = 66, 69), the chunk boundaries of its 16-pivot loop (n = 96, 111, 112) and
the class top (n = 126, 128 - 2 = the largest multiple of 3), with ld = 256 (N = 12) so the class-packed block sits
in a bigger slab. Oracle: oracle/cmpc_oracle.c (same algorithm, Cholesky); bars as test_gpu_parity.py.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20221125
SIZES = [66, 69, 72, 81, 96, 99, 111, 114, 120, 126]


def rel_err(u, ur):
    return float(np.max(np.abs(u - ur)) / max(1.0, float(np.max(np.abs(ur)))))


def contacts_for_sizes(N, sizes, seed=3):
    """One contact table per requested n = 3 * (#stance leg-steps): every step keeps a stance leg, the rest of the
    stance flags are spread at random (reproducible)."""
    rng = np.random.default_rng(seed)
    out = np.zeros((len(sizes), N, 4), np.uint8)
    for b, n in enumerate(sizes):
        t = n // 3
        assert N <= t <= 4 * N
        c = out[b]
        c[np.arange(N), rng.integers(0, 4, N)] = 1
        free = np.argwhere(c == 0)
        pick = free[rng.permutation(len(free))[: t - N]]
        c[pick[:, 0], pick[:, 1]] = 1
        assert int(c.sum()) == t
    return out


@pytest.mark.parametrize("precision", [0, 1])
def test_class128_sizes_match_oracle(cm, op, precision):
    N = 12
    m, mo = cm.default_model(N), op.default_model(N)
    B = len(SIZES)
    if precision == 0:
        s = cm.default_settings()
        so = op.default_settings()
    else:
        s = cm.default_settings(tol_stat=1e-3, tol_ineq=1e-3, tol_comp=1e-4)  # fp32: ulp(5000 N bound) = 4.9e-4
        so = op.tight_settings()
    eng = cm.Engine(m, settings=s, precision=precision, max_batch=B)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=0)
    contact[:] = contacts_for_sizes(N, SIZES)
    nvar = 3 * contact.reshape(B, -1).sum(axis=1)
    assert list(nvar) == SIZES
    u, x, st, it = eng.solve(x0, xref, foot, contact)
    ur, xr, sr, itr = op.solve_batch(mo, so, x0, xref, foot, contact, nthreads=8)
    assert np.all(sr == 0) and np.all(st == 0), (st, sr)
    err = max(rel_err(u[q], ur[q]) for q in range(B))
    if precision == 0:
        assert err < 1e-8, err
        assert np.abs(it - itr).max() <= 1, (it, itr)
    else:
        assert err < 2e-3, err
    assert np.all(u[contact == 0] == 0.0)
