"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracle on identical inputs.

Bars: bit-exact for the integer/byte work (input generator); fp64 contact forces within 1e-5 relative to
max(|u_ref|_inf, 1) (north_star), checked far tighter in practice; fp32 within 2e-3 relative.
"""
import pathlib

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
    s = cm.default_settings(tol_stat=1e-3, tol_ineq=1e-3, tol_comp=1e-4)  # fp32: ulp(5000 N bound) = 4.9e-4
    eng = cm.Engine(m, settings=s, precision=1, max_batch=B)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=0)
    u, x, st, it = eng.solve(x0, xref, foot, contact)
    ur, xr, sr, itr = op.solve_batch(mo, op.tight_settings(), x0, xref, foot, contact, nthreads=8)
    assert np.all(sr == 0)
    assert np.all(st == 0)
    err = max(rel_err(u[q], ur[q]) for q in range(B) if st[q] == 0)
    assert err < 2e-3, err


def _ragged_contacts(rng, B, N, p_stance):
    """Random per-QP contact tables (every step keeps >= 1 stance leg): condensed sizes spread over all three IPM
    size classes (n <= 64, 64 < n <= 128, 128 < n <= 256)."""
    c = (rng.random((B, N, 4)) < p_stance[:, None, None]).astype(np.uint8)
    for b in range(B):
        for k in range(N):
            if not c[b, k].any():
                c[b, k, rng.integers(4)] = 1
    return c


@pytest.mark.parametrize("precision", [0, 1])
def test_condense_large_class_matches_oracle(cm, op, precision):
    """256 class (128 < n <= 256): all-stance N = 20 gives n = 240 (SURVEY §8 a2/a3 sizes)."""
    N = 20
    m, mo = cm.default_model(N), op.default_model(N)
    eng = cm.Engine(m, precision=precision, max_batch=8)
    assert eng.ld == 256
    x0, xref, foot, contact = op.generate(mo, SEED, 6, gait=0)
    contact[:] = 1
    H, g, n, st = eng.condense(x0, xref, foot, contact)
    tol = 1e-12 if precision == 0 else 2e-5
    for q in range(6):
        nq, Hr, gr, mu, lo, hi, mp, sto = op.condense(mo, x0[q], xref[q], foot[q], contact[q], ld=eng.ld)
        assert st[q] == sto == 0 and n[q] == nq == 240
        assert np.abs(H[q, :nq, :nq] - Hr[:nq, :nq]).max() / np.abs(Hr[:nq, :nq]).max() < tol
        assert np.abs(g[q, :nq] - gr[:nq]).max() / max(1.0, np.abs(gr[:nq]).max()) < tol


def test_solve_fp64_large_class_all_stance(cm, op):
    N = 20
    m, mo = cm.default_model(N), op.default_model(N)
    B = 16
    eng = cm.Engine(m, precision=0, max_batch=B)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=0)
    contact[:] = 1
    u, x, st, it = eng.solve(x0, xref, foot, contact)
    ur, xr, sr, itr = op.solve_batch(mo, op.default_settings(), x0, xref, foot, contact, nthreads=8)
    assert np.all(sr == 0) and np.all(st == 0)
    err = max(rel_err(u[q], ur[q]) for q in range(B))
    assert err < 1e-6, err
    assert np.abs(it - itr).max() <= 1


def test_solve_fp64_ragged_all_classes(cm, op):
    N = 20
    m, mo = cm.default_model(N), op.default_model(N)
    B = 48
    rng = np.random.default_rng(7)
    eng = cm.Engine(m, precision=0, max_batch=B)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=0)
    contact[:] = _ragged_contacts(rng, B, N, np.linspace(0.2, 1.0, B))
    nvar = 3 * contact.reshape(B, -1).sum(axis=1)
    assert nvar.min() <= 64 and ((nvar > 64) & (nvar <= 128)).any() and nvar.max() > 128
    u, x, st, it = eng.solve(x0, xref, foot, contact)
    ur, xr, sr, itr = op.solve_batch(mo, op.default_settings(), x0, xref, foot, contact, nthreads=8)
    assert np.all(st == sr)
    ok = st == 0
    assert ok.mean() > 0.9
    err = max(rel_err(u[q], ur[q]) for q in range(B) if ok[q])
    assert err < 1e-6, err
    assert np.all(u[contact == 0] == 0.0)


def test_solve_fp32_large_class(cm, op):
    N = 20
    m, mo = cm.default_model(N), op.default_model(N)
    B = 16
    s = cm.default_settings(tol_stat=1e-3, tol_ineq=1e-3, tol_comp=1e-4)
    eng = cm.Engine(m, settings=s, precision=1, max_batch=B)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=0)
    contact[:] = 1
    u, x, st, it = eng.solve(x0, xref, foot, contact)
    ur, xr, sr, itr = op.solve_batch(mo, op.tight_settings(), x0, xref, foot, contact, nthreads=8)
    assert np.all(sr == 0) and np.all(st == 0)
    err = max(rel_err(u[q], ur[q]) for q in range(B))
    assert err < 2e-3, err


def test_too_large_status(cm, op):
    """n > 256 (all-stance N = 22: n = 264) -> TOO_LARGE (6), other QPs of the batch unaffected."""
    N = 22
    m, mo = cm.default_model(N), op.default_model(N)
    eng = cm.Engine(m, precision=0, max_batch=4)
    x0, xref, foot, contact = op.generate(mo, SEED, 3, gait=0)
    contact[1] = 1
    u, x, st, it = eng.solve(x0, xref, foot, contact)
    assert st[1] == 6 and np.all(u[1] == 0)
    ur, xr, sr, itr = op.solve_batch(mo, op.default_settings(), x0[[0, 2]], xref[[0, 2]], foot[[0, 2]],
                                     contact[[0, 2]], nthreads=2)
    assert st[0] == 0 and st[2] == 0
    assert max(rel_err(u[q], ur[k]) for k, q in enumerate((0, 2))) < 1e-6


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


# ---------------------------------------------------------------------------- golden fixtures on the device

import glob  # noqa: E402
import os  # noqa: E402
import subprocess  # noqa: E402

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
GOLDEN = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "c*.npz")))


def _load(name):
    with np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("name", GOLDEN)
def test_device_matches_golden_fp64(cm, name):
    z = _load(name)
    N = int(z["N"])
    m = cm.default_model(N)
    eng = cm.Engine(m, precision=0, max_batch=z["x0"].shape[0])
    u, x, st, it = eng.solve(z["x0"], z["xref"], z["foot"], z["contact"])
    assert np.all(st == 0)
    err = max(rel_err(u[q], z["u"][q]) for q in range(u.shape[0]))
    assert err < 1e-6, err   # HPIPM default tolerances; the north-star gate is 1e-5
    # condensed Hessian / gradient of stance rows against the numpy restatement
    H, g, n, stc = eng.condense(z["x0"], z["xref"], z["foot"], z["contact"])
    for q in range(u.shape[0]):
        idx = [12 * k + 3 * i + d for k in range(N) for i in range(4) if z["contact"][q, k, i] for d in range(3)]
        Hr = z["H_full"][q][np.ix_(idx, idx)]
        assert n[q] == len(idx)
        assert np.abs(H[q, :n[q], :n[q]] - Hr).max() / np.abs(Hr).max() < 1e-12


def test_generator_matches_golden_inputs(cm):
    z = _load("config5_mixed_N10")
    m = cm.default_model(10)
    d = [a.host() for a in cm.generate_device(m, SEED, z["x0"].shape[0], gait=1)]
    for got, key in zip(d, ("x0", "xref", "foot", "contact")):
        assert np.array_equal(got, z[key])


def test_qp_solve_hook_matches_oracle(cm, op):
    N = 10
    m, mo = cm.default_model(N), op.default_model(N)
    eng = cm.Engine(m, precision=0, max_batch=16)
    ld = eng.ld
    x0, xref, foot, contact = op.generate(mo, SEED, 16, gait=1)
    Hs, gs, ns, mus, los, his, refs = [], [], [], [], [], [], []
    for q in range(16):
        n, H, g, mu, lo, hi, mp, st = op.condense(mo, x0[q], xref[q], foot[q], contact[q], ld=ld)
        Hs.append(H); gs.append(g); ns.append(n); mus.append(mu); los.append(lo); his.append(hi)
        refs.append(op.qp_ipm(n, H, g, mu, lo, hi, op.default_settings())[0])
    u, st, it = eng.qp_solve(np.array(Hs), np.array(gs), np.array(ns, np.int32), np.array(mus), np.array(los),
                             np.array(his))
    assert np.all(st == 0)
    for q in range(16):
        assert rel_err(u[q, :ns[q]], refs[q]) < 1e-8
        assert np.all(u[q, ns[q]:] == 0)


def test_hpipm_interface_path_on_device(cm, op):
    """testHpipmInterface.cpp:112-152 known solution through the device OCP path (batched)."""
    from test_oracle import random_ocp
    rng = np.random.default_rng(42)
    recs, x0s, xgs, ugs = [], [], [], []
    N, nx, nu = 5, 3, [2, 0, 2, 2, 2]
    for b in range(8):
        A, B, bb, Q, S, R, q, r = random_ocp(rng, N, nx, nu)
        xs = [rng.uniform(-1, 1, nx)]
        us = []
        for k in range(N):
            us.append(rng.uniform(-1, 1, nu[k]))
            xs.append(bb[k] + A[k] @ xs[k] + B[k] @ us[k])
            q[k] = -(Q[k] @ xs[k] + S[k].T @ us[k])
            r[k] = -(R[k] @ us[k] + S[k] @ xs[k])
        q[N] = -Q[N] @ xs[N]
        recs.append(op.ocp_pack(N, nx, nu, A, B, bb, Q, S, R, q, r))
        x0s.append(xs[0]); xgs.append(np.array(xs)); ugs.append(np.concatenate(us))
    x, u, st = cm.ocp_solve(N, nx, nu, np.array(x0s), np.array(recs))
    assert np.all(st == 0)
    assert np.abs(x - np.array(xgs)).max() < 1e-9
    assert np.abs(u - np.array(ugs)).max() < 1e-9


def test_riccati_on_device_matches_recursion(cm, op):
    """testHpipmInterface.cpp:258-340 retrieveRiccati: device recursion vs the closed-form one (1e-9) and vs the
    oracle's, batched over problems with ragged inputs (nu_k = 0 stages included); u = K x + k self-consistency."""
    from test_oracle import random_ocp
    rng = np.random.default_rng(11)
    N, nx, nu = 6, 4, [3, 0, 2, 3, 1, 3]
    recs, probs = [], []
    for b in range(5):
        A, B, bb, Q, S, R, q, r = random_ocp(rng, N, nx, nu)
        recs.append(op.ocp_pack(N, nx, nu, A, B, bb, Q, S, R, q, r))
        probs.append((A, B, bb, Q, S, R, q, r))
    Sm, sv, K, kff, st = cm.ocp_riccati(N, nx, nu, np.array(recs))
    assert np.all(st == 0)
    for b, (A, B, bb, Q, S, R, q, r) in enumerate(probs):
        Sg, sg = Q[N], q[N]
        assert np.abs(Sm[b, N] - Sg).max() < 2e-12  # reg_prim (1e-12) on the diagonal
        for k in range(N - 1, -1, -1):
            m = nu[k]
            if m:
                P = S[k] + B[k].T @ Sg @ A[k]
                iR = np.linalg.inv(R[k] + B[k].T @ Sg @ B[k])
                rr = r[k] + B[k].T @ sg + B[k].T @ Sg @ bb[k]
                Sn = Q[k] + A[k].T @ Sg @ A[k] - P.T @ iR @ P
                sn = q[k] + A[k].T @ sg + A[k].T @ Sg @ bb[k] - P.T @ iR @ rr
                assert np.abs(K[b][k] - (-iR @ P)).max() < 1e-9
                assert np.abs(kff[b][k] - (-iR @ rr)).max() < 1e-9
            else:
                Sn = Q[k] + A[k].T @ Sg @ A[k]
                sn = q[k] + A[k].T @ sg + A[k].T @ Sg @ bb[k]
            assert np.abs(Sm[b, k] - Sn).max() < 1e-9 and np.abs(sv[b, k] - sn).max() < 1e-9
            Sg, sg = Sn, sn
        Smo, svo, Ko, ko, sto = op.ocp_riccati(N, nx, nu, recs[b])
        assert sto == 0 and np.abs(Sm[b] - Smo).max() < 1e-9
        x0 = rng.uniform(-1, 1, nx)
        x, u, _ = op.ocp_solve(N, nx, nu, x0, recs[b])
        o = 0
        for k in range(N):
            assert np.allclose(u[o:o + nu[k]], K[b][k] @ x[k] + kff[b][k], atol=1e-9)
            o += nu[k]


def test_riccati_not_pd_status(cm, op):
    from test_oracle import random_ocp
    rng = np.random.default_rng(3)
    N, nx, nu = 3, 2, [2, 2, 2]
    A, B, bb, Q, S, R, q, r = random_ocp(rng, N, nx, nu)
    R[1] = -1000.0 * np.eye(2)  # R + B'Sm B indefinite at stage 1
    rec = op.ocp_pack(N, nx, nu, A, B, bb, Q, S, R, q, r)
    *_, st = cm.ocp_riccati(N, nx, nu, rec[None])
    # the factorisation guards non-positive pivots as BLASFEO's dpotrf does (inverse 0, no NaN): the IPM cannot meet
    # stationarity along the dropped direction and ends at MAX_ITER, as the oracle's does
    r = op.ocp_ipm(N, nx, nu, np.zeros(nx), rec)
    assert st[0] == r["status"] == 1


@pytest.fixture(scope="module")
def cpp_bins(cm):
    """The C++ mirrors, prebuilt in-tree by __graft_entry__.build() (make is a no-op when they are current)."""
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp")
    subprocess.check_call(["make", "-s", "-C", here])
    return pathlib.Path(here) / "bin"


def test_cpp_hpipm_interface_mirror(cpp_bins):
    r = subprocess.run([str(cpp_bins / "test_hpipm_interface")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASSED" in r.stdout
    assert "varying state dims" in r.stdout  # OcpSize::numStates per node (OcpSize.cpp:55-60)


def test_cpp_hpipm_interface_mirror_ocs2_types(cpp_bins):
    """The same gtest mirror compiled against Eigen / ocs2_core-shaped value types (tests/cpp/mock_eigen, mock_ocs2:
    private storage, uninitialised sizing constructors): the include swap a real ocs2 build makes (reference
    HpipmInterface.h:38); includes the Riccati quantities after an equality-constrained solve."""
    r = subprocess.run([str(cpp_bins / "test_hpipm_interface_ocs2")], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASSED" in r.stdout and "constrained riccati" in r.stdout


def test_cpp_centroidal_mpc_eigen_driver_equals_vector_driver(cpp_bins):
    """CentoidMPCTest.cpp's calls written with Eigen::VectorXd, comma initializers and make_shared (the reference's
    own style) against cheeta_mpc/CentroidalMPC.h print exactly what the std::vector build prints."""
    a = subprocess.run([str(cpp_bins / "centroid_mpc_test")], capture_output=True, text=True, timeout=120)
    b = subprocess.run([str(cpp_bins / "centroid_mpc_test_eigen")], capture_output=True, text=True, timeout=120)
    assert a.returncode == 0 and b.returncode == 0, a.stdout + a.stderr + b.stdout + b.stderr
    assert a.stdout == b.stdout


def test_cpp_centroidal_mpc_driver(cpp_bins, op):
    """CentoidMPCTest.cpp equivalent through the C++ CentroidalMPC mirror vs the numpy golden (literal quirk)."""
    r = subprocess.run([str(cpp_bins / "centroid_mpc_test")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "caught mpc table invalid" in r.stdout
    z = _load("centoid_mpc_test_N6")
    u, u2, u3 = np.zeros((6, 4, 3)), np.zeros((6, 4, 3)), np.zeros((6, 4, 3))
    feet2, feet3 = np.zeros((7, 4, 3)), np.zeros((7, 4, 3))
    for line in r.stdout.splitlines():
        if line.startswith("status"):
            assert line.split()[1] == "0"
        if line.startswith("force"):
            tag, i, k, fx, fy, fz = line.split()
            {"force": u, "force2": u2, "force3": u3}[tag][int(k), int(i)] = [float(fx), float(fy), float(fz)]
        if line.startswith("foot"):
            tag, i, j, px, py, pz = line.split()
            {"foot2": feet2, "foot3": feet3}[tag][int(j), int(i)] = [float(px), float(py), float(pz)]
    assert "status3 0" in r.stdout
    assert rel_err(u, z["u"][0]) < 1e-6
    # second call: state[9+6] (rh foot x) moved 2 cm -> the record's node 0 moves, U changes, oracle agrees
    foot2 = z["foot"].copy()
    foot2[0, 0, 2, 0] += 0.02
    mo = op.default_model(6)
    ur2, _, sr2, _ = op.solve_batch(mo, op.tight_settings(), z["x0"], z["xref"], foot2, z["contact"])
    assert sr2[0] == 0
    assert rel_err(u2, ur2[0]) < 1e-6
    assert rel_err(u2, u) > 1e-4
    # QP mode's foot_pos output: the frozen footholds (node 0 current, later runs at the mean des, swing des)
    assert np.array_equal(feet2, op.feet_table(mo, foot2[0], z["contact"][0], np.zeros((6, 4, 3))))
    # setNonlinear(true): the reference's NLP with the later runs' footholds as variables (oracle_sqp_solve_feet)
    ur3, Dr3, feetr3, _, sr3, _, _ = op.sqp_solve_feet(mo, op.default_settings(), z["x0"][0], z["xref"][0],
                                                       z["foot"][0], z["contact"][0], sqp_iter_max=10, sqp_tol=1e-7)
    assert sr3 == 0 and np.abs(Dr3).max() > 1e-4  # the footholds move
    assert rel_err(u3, ur3) < 1e-6
    assert np.abs(feet3 - feetr3).max() < 1e-8


@pytest.mark.gpu
@pytest.mark.parametrize("N,gait", [(10, 0), (10, 1), (20, 0)])
def test_device_matches_riccati_restatement(cm, op, N, gait):
    """The device hot path (condensing + size-class IPM) against the HPIPM-style OCP restatement of the same QP
    (oracle_riccati_solve_batch: no condensing, Riccati Newton steps): statuses equal, iterations within 1,
    forces within the north star's 1e-5 (measured ~1e-15)."""
    B = 128
    m, mo = cm.default_model(N), op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=gait)
    eng = cm.Engine(m, precision=0, max_batch=B)
    u, _, st, it = eng.solve(x0, xref, foot, contact, want_x=False)
    ur, sr, itr = op.riccati_solve_batch(mo, op.default_settings(), x0, xref, foot, contact, nthreads=8)
    assert np.array_equal(st, sr) and np.all(st == 0)
    assert np.abs(it - itr).max() <= 1
    assert np.abs(u - ur).max() / max(1.0, np.abs(ur).max()) < 1e-9


@pytest.mark.gpu
def test_long_horizon_mixed_classes(cm, op):
    """N = 25 (no one-wave condensing: the first workgroup condensing kernel serves n <= 128 and leaves hints, the class
    lists then route 128 < n <= 256 to the 256 class): trot / bound (n = 150) solve and match the oracle, pronk
    (n = 300 > 256) is TOO_LARGE, on one mixed batch."""
    N, B = 25, 24
    m, mo = cm.default_model(N), op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=1)
    n = 3 * contact.reshape(B, -1).sum(axis=1)
    assert (n > 256).any() and ((n > 128) & (n <= 256)).any()
    eng = cm.Engine(m, precision=0, max_batch=B)
    u, _, st, it = eng.solve(x0, xref, foot, contact, want_x=False)
    assert np.all(st[n > 256] == 6) and np.all(u[n > 256] == 0)
    ok = n <= 256
    assert np.all(st[ok] == 0)
    ur, _, sr, itr = op.solve_batch(mo, op.default_settings(), x0[ok], xref[ok], foot[ok], contact[ok], nthreads=8,
                                    want_x=False)
    assert np.all(sr == 0)
    assert max(rel_err(a, b) for a, b in zip(u[ok], ur)) < 1e-6


@pytest.mark.parametrize("gait", [0, 1])
def test_device_foot_semantics(cm, op, gait):
    """Stance lever arms on the device follow the reference's foot dynamics (CentroidalMPC.cpp:93, :165-167,
    :288-291) exactly as the oracle: moving the current feet (record node 0) moves U and the device tracks the oracle;
    moving the des_foot_pos nodes of an initial stance run changes nothing, bit for bit; a later run acts at the mean
    of its nodes (perturbed, non-planted feet) and still matches the oracle."""
    N, B = 10, 64
    m, mo = cm.default_model(N), op.default_model(N)
    x0, xref, foot, contact = op.generate(mo, SEED, B, gait=gait)
    eng = cm.Engine(m, precision=0, max_batch=B)
    H0, g0, n0, st0 = eng.condense(x0, xref, foot, contact)
    f2 = foot.copy()
    for q in range(B):
        for i in range(4):
            k = 0
            while k < N and contact[q, k, i]:
                k += 1
            if k > 0:
                f2[q, 1:k + 1, i, :2] += 0.05
    H2, g2, n2, st2 = eng.condense(x0, xref, f2, contact)
    assert np.array_equal(H2, H0) and np.array_equal(g2, g0)
    rng = np.random.default_rng(3)
    f1 = foot + rng.uniform(-0.02, 0.02, foot.shape) * np.array([1.0, 1.0, 0.0])  # every node moves: means matter
    u1, _, s1, _ = eng.solve(x0, xref, f1, contact, want_x=False)
    ur1, _, sr1, _ = op.solve_batch(mo, op.default_settings(), x0, xref, f1, contact, nthreads=8, want_x=False)
    u0, _, _, _ = eng.solve(x0, xref, foot, contact, want_x=False)
    assert np.array_equal(s1, sr1) and np.all(s1 == 0)
    assert max(rel_err(u1[q], ur1[q]) for q in range(B)) < 1e-9
    assert rel_err(u1, u0) > 1e-4
