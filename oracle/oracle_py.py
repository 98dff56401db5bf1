"""ctypes binding of the CPU oracle (oracle/liboracle.so) plus the shared model/settings structs.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the
product (cheeta-mpc_amd/). See oracle/cmpc_oracle.h for what the oracle restates and how it is pinned.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
NX, NU, NL = 13, 12, 4

# CentoidMPCTest.cpp:19-33 weight vector (ordering as the code reads it, CentroidalMPC.cpp:203-231)
TEST_WEIGHTS = [1, 1, 100, 0.5, 0.5, 0, 2, 2, 8,
                0.2, 0.2, 0.2, 0.3, 0.3, 0.3, 0.1, 0.1, 0.1,
                0.2, 0.2, 0.2, 0.3, 0.3, 0.3, 0.1, 0.1, 0.1,
                0.2, 0.2, 0.2, 0.3, 0.3, 0.3, 0.1, 0.1, 0.1,
                0.2, 0.2, 0.2, 0.3, 0.3, 0.3, 0.1, 0.1, 0.1]
STATUS = {0: "SUCCESS", 1: "MAX_ITER", 2: "MIN_STEP", 3: "NAN_SOL", 4: "INCONS_EQ", 5: "INVALID_CONTACT",
          6: "TOO_LARGE", 7: "INFEASIBLE_STEP"}


class Model(C.Structure):
    _fields_ = [("N", C.c_int), ("n_legs", C.c_int), ("mass", C.c_double), ("dt", C.c_double),
                ("inertia", C.c_double * 9), ("mu", C.c_double * 4), ("weights", C.c_double * 45),
                ("force_ub", C.c_double * 5), ("theta_weights", C.c_double * 3)]


class Settings(C.Structure):
    _fields_ = [("hpipm_mode", C.c_int), ("iter_max", C.c_int), ("alpha_min", C.c_double), ("mu0", C.c_double),
                ("tol_stat", C.c_double), ("tol_eq", C.c_double), ("tol_ineq", C.c_double),
                ("tol_comp", C.c_double), ("reg_prim", C.c_double), ("warm_start", C.c_int),
                ("pred_corr", C.c_int), ("ric_alg", C.c_int)]


def default_model(N=10):
    """CentoidMPCTest.cpp:12-33 (m=8, dt=0.01, mu=0.8, 45 weights); inertia diag(0.07,0.26,0.28)."""
    m = Model()
    m.N = N
    m.n_legs = NL
    m.mass = 8.0
    m.dt = 0.01
    for i, v in enumerate([0.07, 0, 0, 0, 0.26, 0, 0, 0, 0.28]):
        m.inertia[i] = v
    for i in range(4):
        m.mu[i] = 0.8
    for i, v in enumerate(TEST_WEIGHTS):
        m.weights[i] = float(v)
    for i in range(4):
        m.force_ub[i] = 5000.0
    m.force_ub[4] = 8.0 * 9.81 * NL
    return m


def default_settings(**kw):
    """hpipm_interface::Settings defaults (HpipmInterfaceSettings.h:44-57)."""
    s = Settings(hpipm_mode=1, iter_max=30, alpha_min=1e-12, mu0=10.0, tol_stat=1e-6, tol_eq=1e-8, tol_ineq=1e-8,
                 tol_comp=1e-8, reg_prim=1e-12, warm_start=0, pred_corr=1, ric_alg=0)
    for k, v in kw.items():
        setattr(s, k, v)
    return s


def tight_settings():
    return default_settings(tol_stat=1e-10, tol_ineq=1e-10, tol_comp=1e-11, iter_max=50)


_lib = None
_LIBNAME = os.environ.get("CMPC_ORACLE_LIB", "liboracle.so")


def select_build(name):
    """Choose the oracle build before first use: "liboracle.so" (the checker, -ffp-contract=off) or
    "liboracle_fast.so" (bench.py's cpu_baseline: -O3, FMA contraction)."""
    global _LIBNAME
    if _lib is not None and name != _LIBNAME:
        raise RuntimeError("oracle library already loaded as " + _LIBNAME)
    _LIBNAME = name


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(HERE, _LIBNAME)
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", HERE])
        L = C.CDLL(path)
        P = C.POINTER
        d, i, u8 = P(C.c_double), P(C.c_int), P(C.c_uint8)
        L.oracle_solve_batch.argtypes = [P(Model), P(Settings), C.c_int, d, d, d, u8, d, d, i, i, C.c_int]
        L.oracle_generate.argtypes = [P(Model), C.c_uint64, C.c_int64, C.c_int, C.c_int, d, d, d, u8]
        L.oracle_qp_ipm.argtypes = [C.c_int, C.c_int, d, d, d, d, d, P(Settings), d, d, d, i, d]
        L.oracle_qp_ipm_stats.argtypes = [C.c_int, C.c_int, d, d, d, d, d, P(Settings), d, d, d, i, d, d, C.c_int]
        L.oracle_qp_kkt.argtypes = [C.c_int, C.c_int, d, d, d, d, d, d, d, d, d]
        L.oracle_ocp_record_size.restype = C.c_size_t
        L.oracle_ocp_record_size.argtypes = [C.c_int, C.c_int, i]
        L.oracle_ocp_condense.argtypes = [C.c_int, C.c_int, i, d, d, d, d]
        L.oracle_ocp_solve.argtypes = [C.c_int, C.c_int, i, d, d, d, d]
        L.oracle_ocp_riccati.argtypes = [C.c_int, C.c_int, i, d, d, d, d, d]
        L.oracle_ocp_ipm.argtypes = [C.c_int, C.c_int, i, i, d, d, d, P(Settings), d, d, i, d, C.c_void_p, d,
                                     C.c_int]
        L.oracle_ocp_ipm_batch.argtypes = [C.c_int, C.c_int, C.c_int, i, i, d, d, C.c_size_t, d, C.c_size_t,
                                           P(Settings), d, d, i, i, C.c_int]
        L.oracle_ocp_first_step.argtypes = [C.c_int, C.c_int, i, i, d, d, d, P(Settings), d, d, d, d, d, d, d]
        L.oracle_gait_contact.argtypes = [C.c_void_p, i, C.c_double, C.c_double, C.c_double, C.c_int,
                                          C.POINTER(C.c_uint8)]
        L.oracle_gait_contact.restype = None
        L.oracle_cholesky.argtypes = [C.c_int, d, C.c_int]
        L.oracle_nlp_rollout_cost.argtypes = [C.c_void_p, d, d, d, u8, d, d, d]
        L.oracle_nlp_rollout_cost.restype = C.c_double
        L.oracle_sqp_solve.argtypes = [C.c_void_p, P(Settings), C.c_int, C.c_double, d, d, d, u8, d, d, i, i]
        L.oracle_nlp_linstep.argtypes = [C.c_void_p, d, d, d, u8, d, d, d, d]
        L.oracle_nlp_linstep.restype = None
        L.oracle_srbd_dynamics_lin.argtypes = [C.c_void_p, d, d, u8, d, d, d, d]
        L.oracle_srbd_dynamics_lin.restype = None
        L.oracle_policy.argtypes = [C.c_void_p, d, d, u8, d, C.c_double, d, i]
        L.oracle_policy_lin.argtypes = [C.c_void_p, d, d, u8, d, d, C.c_double, d, i]
        L.oracle_solve_one_lin.argtypes = [C.c_void_p, P(Settings), d, d, d, u8, d, d, d, i]
        L.oracle_policy_triple.argtypes = [C.c_double, d, d, C.c_double, d]
        L.oracle_riccati_solve_batch.argtypes = [P(Model), P(Settings), C.c_int, d, d, d, u8, d, i, i, C.c_int]
        L.oracle_riccati_gain0.argtypes = [C.c_void_p, d, d, u8, d]
        L.oracle_philox4x32_10.argtypes = [P(C.c_uint32), P(C.c_uint32), P(C.c_uint32)]
        L.oracle_stance_feet.argtypes = [C.c_int, C.c_int, d, u8, d]
        L.oracle_stance_feet.restype = None
        L.oracle_nlp_rollout_cost_feet.argtypes = [C.c_void_p, d, d, d, u8, d, d, d, d]
        L.oracle_nlp_rollout_cost_feet.restype = C.c_double
        L.oracle_nlp_linstep_feet.argtypes = [C.c_void_p, d, d, d, u8, d, d, d, d, d, d]
        L.oracle_nlp_linstep_feet.restype = None
        L.oracle_foot_box.argtypes = [d, u8, C.c_int, C.c_int, C.c_int, C.c_int, d, d, d, i]
        L.oracle_feet_init.argtypes = [C.c_void_p, d, u8, d]
        L.oracle_feet_init.restype = None
        L.oracle_feet_table.argtypes = [C.c_void_p, d, u8, d, d]
        L.oracle_feet_table.restype = None
        L.oracle_condense_feet.argtypes = [C.c_void_p, d, d, d, u8, d, d, d, C.c_int, i, d, d, d, d, d, i]
        L.oracle_solve_one_feet.argtypes = [C.c_void_p, P(Settings), d, d, d, u8, d, d, d, i]
        L.oracle_sqp_solve_feet.argtypes = [C.c_void_p, P(Settings), C.c_int, C.c_double, d, d, d, u8, d, d, d, d,
                                            i, i]
        _lib = L
    return _lib


class _Consts(C.Structure):
    _fields_ = [("N", C.c_int), ("L", C.c_int), ("mass", C.c_double), ("dt", C.c_double),
                ("inv_inertia", C.c_double * 9), ("mu", C.c_double * 4), ("Wf", C.c_double * 12),
                ("Wr", C.c_double * 12), ("Wp", C.c_double * 12), ("qdiag", (C.c_double * 13) * 64),
                ("force_ub", C.c_double * 5)]


def _p(a, t=C.c_double):
    return a.ctypes.data_as(C.POINTER(t))


def consts(model):
    L = lib()
    c = _Consts()
    L.oracle_consts_init(C.byref(model), C.byref(c))
    return c


def stance_feet(foot, contact):
    """Foot position behind every stance force [N][4][3] of one QP (oracle_stance_feet; 0 for swing)."""
    foot = np.ascontiguousarray(foot, np.float64)
    contact = np.ascontiguousarray(contact, np.uint8)
    N = contact.shape[0]
    out = np.zeros((N, NL, 3))
    lib().oracle_stance_feet(N, NL, _p(foot), _p(contact, C.c_uint8), _p(out))
    return out


def generate(model, seed, B, gait=0, offset=0):
    N = model.N
    x0 = np.zeros((B, NX))
    xref = np.zeros((B, N + 1, NX))
    foot = np.zeros((B, N + 1, NL, 3))
    contact = np.zeros((B, N, NL), dtype=np.uint8)
    lib().oracle_generate(C.byref(model), seed, offset, B, gait, _p(x0), _p(xref), _p(foot), _p(contact, C.c_uint8))
    return x0, xref, foot, contact


def solve_batch(model, settings, x0, xref, foot, contact, nthreads=1, want_x=True, u_init=None):
    """u_init [B,N,L,3]: initial guess, used when settings.warm_start != 0."""
    B = x0.shape[0]
    N = model.N
    x0, xref, foot = (np.ascontiguousarray(a, dtype=np.float64) for a in (x0, xref, foot))
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    u = np.zeros((B, N, NL, 3)) if u_init is None else np.array(u_init, dtype=np.float64).reshape(B, N, NL, 3)
    x = np.zeros((B, N + 1, NX)) if want_x else None
    st = np.zeros(B, dtype=np.int32)
    it = np.zeros(B, dtype=np.int32)
    lib().oracle_solve_batch(C.byref(model), C.byref(settings), B, _p(x0), _p(xref), _p(foot),
                             _p(contact, C.c_uint8), _p(u), _p(x) if want_x else None, _p(st, C.c_int),
                             _p(it, C.c_int), nthreads)
    return u, x, st, it


def condense(model, x0, xref, foot, contact, ld=None):
    """Condensed QP of one problem: (n, H[ld,ld], g[ld], mu[ld/3], lo[ld/3,5], hi[ld/3,5], map, status)."""
    N = model.N
    ld = ld or NU * N
    c = consts(model)
    H = np.zeros((ld, ld))
    g = np.zeros(ld)
    mu = np.zeros(ld // 3)
    lo = np.zeros((ld // 3, 5))
    hi = np.zeros((ld // 3, 5))
    mp = np.zeros(ld // 3, dtype=np.int32)
    n = C.c_int(0)
    x0, xref, foot = (np.ascontiguousarray(a, dtype=np.float64) for a in (x0, xref, foot))
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    st = lib().oracle_condense(C.byref(c), _p(x0), _p(xref), _p(foot), _p(contact, C.c_uint8), ld, C.byref(n),
                               _p(H), _p(g), _p(mu), _p(lo), _p(hi), _p(mp, C.c_int))
    return n.value, H, g, mu, lo, hi, mp, st


def condense_full(model, x0, xref, foot, contact):
    N = model.N
    c = consts(model)
    n = NU * N
    H = np.zeros((n, n))
    g = np.zeros(n)
    x0, xref, foot = (np.ascontiguousarray(a, dtype=np.float64) for a in (x0, xref, foot))
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    st = lib().oracle_condense_full(C.byref(c), _p(x0), _p(xref), _p(foot), _p(contact, C.c_uint8), _p(H), _p(g))
    return H, g, st


def srbd_dynamics(model, xref, foot, contact):
    N = model.N
    c = consts(model)
    A = np.zeros((N, NX, NX))
    B = np.zeros((N, NX, NU))
    xref, foot = (np.ascontiguousarray(a, dtype=np.float64) for a in (xref, foot))
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    lib().oracle_srbd_dynamics(C.byref(c), _p(xref), _p(foot), _p(contact, C.c_uint8), _p(A), _p(B))
    return A, B


def srbd_dynamics_lin(model, xref, foot, contact, lin):
    """A, B, b of the dynamics linearised at lin [N,6] = (c_bar, F_bar) (None: the reference, b = 0)."""
    N = model.N
    c = consts(model)
    A = np.zeros((N, NX, NX))
    B = np.zeros((N, NX, NU))
    b = np.zeros((N, NX))
    xref, foot = (np.ascontiguousarray(a, dtype=np.float64) for a in (xref, foot))
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    ln = None if lin is None else np.ascontiguousarray(lin, np.float64)
    lib().oracle_srbd_dynamics_lin(C.byref(c), _p(xref), _p(foot), _p(contact, C.c_uint8),
                                   _p(ln) if ln is not None else None, _p(A), _p(B), _p(b))
    return A, B, b


def nlp_rollout_cost(model, x0, xref, foot, contact, u):
    """Nonlinear (bilinear lever arm) rollout and NLP cost of one QP: (J, x [N+1,13], lin [N,6])."""
    N = model.N
    c = consts(model)
    x = np.zeros((N + 1, NX))
    lin = np.zeros((N, 6))
    x0, xref, foot, u = (np.ascontiguousarray(a, dtype=np.float64) for a in (x0, xref, foot, u))
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    J = lib().oracle_nlp_rollout_cost(C.byref(c), _p(x0), _p(xref), _p(foot), _p(contact, C.c_uint8), _p(u), _p(x),
                                      _p(lin))
    return J, x, lin


def nlp_linstep(model, x0, xref, foot, contact, u, du):
    """Linearised response of the rollout of u to du: (|dx| over the trajectory, descent metric grad J . [dx; du])."""
    c = consts(model)
    x0, xref, foot, u, du = (np.ascontiguousarray(a, dtype=np.float64) for a in (x0, xref, foot, u, du))
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    dxn, mt = C.c_double(0.0), C.c_double(0.0)
    lib().oracle_nlp_linstep(C.byref(c), _p(x0), _p(xref), _p(foot), _p(contact, C.c_uint8), _p(u), _p(du),
                             C.byref(dxn), C.byref(mt))
    return dxn.value, mt.value


def sqp_solve(model, settings, x0, xref, foot, contact, sqp_iter_max=10, sqp_tol=1e-7):
    """Gauss-Newton SQP of one QP on the bilinear NLP: (u [N,L,3], x [N+1,13], status, qp_iters, sqp_iters)."""
    N = model.N
    c = consts(model)
    u = np.zeros((N, NL, 3))
    x = np.zeros((N + 1, NX))
    x0, xref, foot = (np.ascontiguousarray(a, dtype=np.float64) for a in (x0, xref, foot))
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    qi, si = C.c_int(0), C.c_int(0)
    st = lib().oracle_sqp_solve(C.byref(c), C.byref(settings), sqp_iter_max, sqp_tol, _p(x0), _p(xref), _p(foot),
                                _p(contact, C.c_uint8), _p(u), _p(x), C.byref(qi), C.byref(si))
    return u, x, st, qi.value, si.value


def _f64(*a):
    return tuple(np.ascontiguousarray(v, dtype=np.float64) for v in a)


def nlp_rollout_cost_feet(model, x0, xref, foot, contact, u, D):
    """nlp_rollout_cost with the later runs' footholds pbar + D (D [N,L,3] by run start): (J, x, lin)."""
    N = model.N
    c = consts(model)
    x = np.zeros((N + 1, NX))
    lin = np.zeros((N, 6))
    x0, xref, foot, u, D = _f64(x0, xref, foot, u, D)
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    J = lib().oracle_nlp_rollout_cost_feet(C.byref(c), _p(x0), _p(xref), _p(foot), _p(contact, C.c_uint8), _p(u),
                                           _p(D), _p(x), _p(lin))
    return J, x, lin


def nlp_linstep_feet(model, x0, xref, foot, contact, u, D, du, dD):
    c = consts(model)
    x0, xref, foot, u, D, du, dD = _f64(x0, xref, foot, u, D, du, dD)
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    dxn, mt = C.c_double(0.0), C.c_double(0.0)
    lib().oracle_nlp_linstep_feet(C.byref(c), _p(x0), _p(xref), _p(foot), _p(contact, C.c_uint8), _p(u), _p(D),
                                  _p(du), _p(dD), C.byref(dxn), C.byref(mt))
    return dxn.value, mt.value


def foot_box(foot, contact, s, i):
    """(pbar, lo, hi, cnt) of the later run of leg i starting at step s, or None."""
    N, L = contact.shape
    foot = np.ascontiguousarray(foot, dtype=np.float64)
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    pb, lo, hi, cnt = np.zeros(3), np.zeros(3), np.zeros(3), C.c_int(0)
    ok = lib().oracle_foot_box(_p(foot), _p(contact, C.c_uint8), N, L, s, i, _p(pb), _p(lo), _p(hi), C.byref(cnt))
    return (pb, lo, hi, cnt.value) if ok else None


def feet_init(model, foot, contact):
    c = consts(model)
    foot = np.ascontiguousarray(foot, dtype=np.float64)
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    D = np.zeros((model.N, NL, 3))
    lib().oracle_feet_init(C.byref(c), _p(foot), _p(contact, C.c_uint8), _p(D))
    return D


def feet_table(model, foot, contact, D):
    c = consts(model)
    foot, D = _f64(foot, D)
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    out = np.zeros((model.N + 1, NL, 3))
    lib().oracle_feet_table(C.byref(c), _p(foot), _p(contact, C.c_uint8), _p(D), _p(out))
    return out


def condense_feet(model, x0, xref, foot, contact, lin, ubar, D, ld=None):
    """Condensed QP of the SQP with footholds: (n, H, g, mu, lo, hi, tri_map, status), H [ld, ld]."""
    N = model.N
    ld = ld or 12 * N
    c = consts(model)
    H, g = np.zeros((ld, ld)), np.zeros(ld)
    mu, lo, hi = np.zeros(ld // 3), np.zeros((ld // 3, 5)), np.zeros((ld // 3, 5))
    mp = np.zeros(ld // 3, np.int32)
    n = C.c_int(0)
    x0, xref, foot, lin, ubar, D = _f64(x0, xref, foot, lin, ubar, D)
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    st = lib().oracle_condense_feet(C.byref(c), _p(x0), _p(xref), _p(foot), _p(contact, C.c_uint8), _p(lin),
                                    _p(ubar), _p(D), ld, C.byref(n), _p(H), _p(g), _p(mu), _p(lo), _p(hi),
                                    _p(mp, C.c_int))
    return n.value, H, g, mu, lo, hi, mp, st


def solve_one_feet(model, settings, x0, xref, foot, contact, lin, u, D):
    """One foothold QP at (lin, u, D), warm-started from (u, D) when settings.warm_start: (u, D, status, iters)."""
    c = consts(model)
    x0, xref, foot, lin = _f64(x0, xref, foot, lin)
    u, D = (np.array(v, dtype=np.float64) for v in (u, D))
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    it = C.c_int(0)
    st = lib().oracle_solve_one_feet(C.byref(c), C.byref(settings), _p(x0), _p(xref), _p(foot),
                                     _p(contact, C.c_uint8), _p(lin), _p(u), _p(D), C.byref(it))
    return u, D, st, it.value


def sqp_solve_feet(model, settings, x0, xref, foot, contact, sqp_iter_max=10, sqp_tol=1e-7):
    """SQP with the later runs' footholds as variables: (u, D, feet [N+1,L,3], x, status, qp_iters, sqp_iters)."""
    N = model.N
    c = consts(model)
    u, D = np.zeros((N, NL, 3)), np.zeros((N, NL, 3))
    feet, x = np.zeros((N + 1, NL, 3)), np.zeros((N + 1, NX))
    x0, xref, foot = _f64(x0, xref, foot)
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    qi, si = C.c_int(0), C.c_int(0)
    st = lib().oracle_sqp_solve_feet(C.byref(c), C.byref(settings), sqp_iter_max, sqp_tol, _p(x0), _p(xref),
                                     _p(foot), _p(contact, C.c_uint8), _p(u), _p(D), _p(feet), _p(x), C.byref(qi),
                                     C.byref(si))
    return u, D, feet, x, st, qi.value, si.value


def qp_ipm_stats(n, H, g, mu, lo, hi, settings, rows):
    """qp_ipm plus the per-iteration statistics table [rows, 10] (columns of cmpc_enable_stats; NaN = not written)."""
    ld = H.shape[0]
    H, g, mu, lo, hi = (np.ascontiguousarray(a, dtype=np.float64) for a in (H, g, mu, lo, hi))
    u = np.zeros(max(n, 1))
    m = max(5 * (n // 3), 1)
    ll = np.zeros(m)
    lu = np.zeros(m)
    it = C.c_int(0)
    res = np.zeros(4)
    stats = np.full((rows, 10), np.nan)
    st = lib().oracle_qp_ipm_stats(n, ld, _p(H), _p(g), _p(mu), _p(lo), _p(hi), C.byref(settings), _p(u), _p(ll),
                                   _p(lu), C.byref(it), _p(res), _p(stats), rows)
    return u[:n], st, it.value, res, stats


def qp_ipm(n, H, g, mu, lo, hi, settings):
    ld = H.shape[0]
    H, g, mu, lo, hi = (np.ascontiguousarray(a, dtype=np.float64) for a in (H, g, mu, lo, hi))
    u = np.zeros(max(n, 1))
    m = max(5 * (n // 3), 1)
    ll = np.zeros(m)
    lu = np.zeros(m)
    it = C.c_int(0)
    res = np.zeros(4)
    st = lib().oracle_qp_ipm(n, ld, _p(H), _p(g), _p(mu), _p(lo), _p(hi), C.byref(settings), _p(u), _p(ll), _p(lu),
                             C.byref(it), _p(res))
    return u[:n], ll[:5 * (n // 3)], lu[:5 * (n // 3)], st, it.value, res


def qp_kkt(n, H, g, mu, lo, hi, u, ll, lu):
    ld = H.shape[0]
    out = np.zeros(4)
    H, g, mu, lo, hi, u, ll, lu = (np.ascontiguousarray(a, dtype=np.float64) for a in (H, g, mu, lo, hi, u, ll, lu))
    lib().oracle_qp_kkt(n, ld, _p(H), _p(g), _p(mu), _p(lo), _p(hi), _p(u), _p(ll), _p(lu), _p(out))
    return out


# ---- generic OCP-QP (HpipmInterface semantics) -------------------------------------------------------------

def ocp_pack(N, nx, nu, A, B, b, Q, S, R, q, r):
    """Pack per-stage lists into the column-major record of cmpc_ocp_record_size."""
    parts = []
    for k in range(N):
        parts += [np.asarray(A[k]).reshape(nx, nx).flatten(order="F"),
                  np.asarray(B[k]).reshape(nx, nu[k]).flatten(order="F"), np.asarray(b[k]).reshape(nx)]
    for k in range(N + 1):
        m = nu[k] if k < N else 0
        parts += [np.asarray(Q[k]).reshape(nx, nx).flatten(order="F"),
                  np.asarray(S[k]).reshape(m, nx).flatten(order="F") if m else np.zeros(0),
                  np.asarray(R[k]).reshape(m, m).flatten(order="F") if m else np.zeros(0),
                  np.asarray(q[k]).reshape(nx), np.asarray(r[k]).reshape(m) if m else np.zeros(0)]
    return np.concatenate(parts).astype(np.float64)


def ocp_constraint_pack(N, nx, nu, nc, Cc, D, e):
    """Pack per-node equality constraints C_k x + D_k u + e_k = 0 into the column-major record of
    cmpc_ocp_constraint_record_size (k = 0..N; D_N empty)."""
    parts = []
    for k in range(N + 1):
        m = nu[k] if k < N else 0
        if nc[k] == 0:
            continue
        parts += [np.asarray(Cc[k]).reshape(nc[k], nx).flatten(order="F"),
                  np.asarray(D[k]).reshape(nc[k], m).flatten(order="F") if m else np.zeros(0),
                  np.asarray(e[k]).reshape(nc[k])]
    return np.concatenate(parts).astype(np.float64) if parts else np.zeros(0)


def ocp_solve(N, nx, nu, x0, rec):
    nua = np.asarray(nu, dtype=np.int32)
    nU = int(nua.sum())
    x = np.zeros((N + 1) * nx)
    u = np.zeros(max(nU, 1))
    st = lib().oracle_ocp_solve(N, nx, _p(nua, C.c_int), _p(np.ascontiguousarray(x0, dtype=np.float64)), _p(rec),
                                _p(x), _p(u))
    return x.reshape(N + 1, nx), u[:nU], st


def ocp_condense(N, nx, nu, x0, rec):
    nua = np.asarray(nu, dtype=np.int32)
    nU = int(nua.sum())
    H = np.zeros((max(nU, 1), max(nU, 1)))
    g = np.zeros(max(nU, 1))
    lib().oracle_ocp_condense(N, nx, _p(nua, C.c_int), _p(np.ascontiguousarray(x0, dtype=np.float64)), _p(rec),
                              _p(H), _p(g))
    return H[:nU, :nU], g[:nU]


def ocp_riccati(N, nx, nu, rec):
    nua = np.asarray(nu, dtype=np.int32)
    Sm = np.zeros((N + 1, nx, nx))
    sv = np.zeros((N + 1, nx))
    K = np.zeros(max(int(sum(nu[k] * nx for k in range(N))), 1))
    kff = np.zeros(max(int(nua[:N].sum()), 1))
    st = lib().oracle_ocp_riccati(N, nx, _p(nua, C.c_int), _p(rec), _p(Sm), _p(sv), _p(K), _p(kff))
    Ks, ks, o, ok = [], [], 0, 0
    for k in range(N):
        Ks.append(K[o:o + nu[k] * nx].reshape(nu[k], nx))
        ks.append(kff[ok:ok + nu[k]])
        o += nu[k] * nx
        ok += nu[k]
    return Sm, sv, Ks, ks, st


class OcpRic(C.Structure):
    _fields_ = [("P", C.POINTER(C.c_double)), ("p", C.POINTER(C.c_double)), ("K", C.POINTER(C.c_double)),
                ("k", C.POINTER(C.c_double)), ("Lr", C.POINTER(C.c_double))]


def ocp_ipm(N, nx, nu, x0, rec, nc=None, crec=None, settings=None, ric=False, stats_rows=0, guess=None):
    """Stage-wise OCP IPM (oracle/ocp_ipm.c). Returns dict: x [(N+1),nx], u [nU], status, iters, res [4], and with
    ric=True P [(N+1),nx,nx], p [(N+1),nx], K (list of nu_k x nx), k (list), Lr (list, lower); stats [rows,10]."""
    s = settings if settings is not None else default_settings()
    nua = np.asarray(list(nu) + [0], dtype=np.int32)
    nU = int(nua[:N].sum())
    nca = None if nc is None else np.asarray(nc, dtype=np.int32)
    crec_a = None if crec is None or nca is None or int(nca.sum()) == 0 else np.ascontiguousarray(crec, np.float64)
    if crec_a is None:
        nca = None
    x = np.zeros((N + 1) * nx)
    u = np.zeros(max(nU, 1))
    if guess is not None:  # initial guess (x [(N+1), nx], u [nU]); read when settings.warm_start != 0
        x[:] = np.asarray(guess[0], np.float64).reshape(-1)
        u[:nU] = np.asarray(guess[1], np.float64).reshape(-1)[:nU]
    it = C.c_int(0)
    res = np.zeros(4)
    st_rows = np.full((max(stats_rows, 1), 10), np.nan)
    out = {}
    r = None
    if ric:
        nK = max(int(sum(nu[k] * nx for k in range(N))), 1)
        nM = max(int(sum(nu[k] * nu[k] for k in range(N))), 1)
        P = np.zeros((N + 1) * nx * nx)
        pv = np.zeros((N + 1) * nx)
        K = np.zeros(nK)
        kk = np.zeros(max(nU, 1))
        Mi = np.zeros(nM)
        r = OcpRic(_p(P), _p(pv), _p(K), _p(kk), _p(Mi))
    status = lib().oracle_ocp_ipm(N, nx, _p(nua, C.c_int), _p(nca, C.c_int) if nca is not None else None,
                                  _p(np.ascontiguousarray(x0, dtype=np.float64)), _p(np.ascontiguousarray(rec)),
                                  _p(crec_a) if crec_a is not None else None, C.byref(s), _p(x), _p(u),
                                  C.byref(it), _p(res), C.byref(r) if r is not None else None,
                                  _p(st_rows) if stats_rows else None, stats_rows)
    out.update(x=x.reshape(N + 1, nx), u=u[:nU], status=status, iters=it.value, res=res)
    if stats_rows:
        out["stats"] = st_rows
    if ric:
        Ks, ks, Ms, o, om, ok = [], [], [], 0, 0, 0
        for k in range(N):
            m = nu[k]
            Ks.append(K[o:o + m * nx].reshape(nx, m).T.copy())
            ks.append(kk[ok:ok + m].copy())
            Ms.append(Mi[om:om + m * m].reshape(m, m).T.copy())
            o += m * nx
            om += m * m
            ok += m
        out.update(P=P.reshape(N + 1, nx, nx).transpose(0, 2, 1).copy(), p=pv.reshape(N + 1, nx), K=Ks, k=ks, Lr=Ms)
    return out


def ocp_ipm_batch(N, nx, nu, x0, rec, nc=None, crec=None, settings=None, nthreads=1):
    """oracle_ocp_ipm over a batch (x0 [B,nx], rec [B,rec_size], crec [B,crec_size]) on nthreads pthreads."""
    s = settings if settings is not None else default_settings()
    x0 = np.ascontiguousarray(x0, np.float64)
    B = x0.shape[0]
    rec = np.ascontiguousarray(rec, np.float64).reshape(B, -1)
    nua = np.asarray(list(nu) + [0], dtype=np.int32)
    nU = int(nua[:N].sum())
    nca = None if nc is None else np.asarray(nc, dtype=np.int32)
    cr = None if nca is None or int(nca.sum()) == 0 else np.ascontiguousarray(crec, np.float64).reshape(B, -1)
    if cr is None:
        nca = None
    x = np.zeros((B, N + 1, nx))
    u = np.zeros((B, max(nU, 1)))
    st = np.zeros(B, np.int32)
    it = np.zeros(B, np.int32)
    lib().oracle_ocp_ipm_batch(B, N, nx, _p(nua, C.c_int), _p(nca, C.c_int) if nca is not None else None, _p(x0),
                               _p(rec), rec.shape[1], _p(cr) if cr is not None else None,
                               cr.shape[1] if cr is not None else 0, C.byref(s), _p(x), _p(u), _p(st, C.c_int),
                               _p(it, C.c_int), int(nthreads))
    return x, u[:, :nU], st, it


def ocp_first_step(N, nx, nu, x0, rec, nc=None, crec=None, settings=None):
    s = settings if settings is not None else default_settings()
    nua = np.asarray(list(nu) + [0], dtype=np.int32)
    nU = int(nua[:N].sum())
    nca = None if nc is None else np.asarray(nc, dtype=np.int32)
    m = 0 if nca is None else int(nca.sum())
    du, dx, dpi = np.zeros(max(nU, 1)), np.zeros((N + 1) * nx), np.zeros(N * nx)
    sig, ru, rx, rb = np.zeros(max(m, 1)), np.zeros(max(nU, 1)), np.zeros((N + 1) * nx), np.zeros(N * nx)
    st = lib().oracle_ocp_first_step(N, nx, _p(nua, C.c_int), _p(nca, C.c_int) if m else None,
                                     _p(np.ascontiguousarray(x0, dtype=np.float64)), _p(np.ascontiguousarray(rec)),
                                     _p(np.ascontiguousarray(crec, np.float64)) if m else None, C.byref(s), _p(du),
                                     _p(dx), _p(dpi), _p(sig), _p(ru), _p(rx), _p(rb))
    return dict(status=st, du=du[:nU], dx=dx.reshape(N + 1, nx), dpi=dpi.reshape(N, nx), sig=sig[:m], rhs_u=ru[:nU],
                rhs_x=rx.reshape(N + 1, nx), rb=rb.reshape(N, nx))


def gait_contact(gait, t_start, t0, dt, N, leg_map=None):
    """Contact table [N,4] of one QP; gait is a cheeta_mpc.Gait (same struct layout as cmpc_gait)."""
    out = np.zeros((N, 4), np.uint8)
    lm = None if leg_map is None else np.ascontiguousarray(leg_map, np.int32)
    lib().oracle_gait_contact(C.byref(gait), _p(lm, C.c_int) if lm is not None else None, t_start, t0, dt, N,
                              _p(out, C.c_uint8))
    return out


def riccati_solve_batch(model, settings, x0, xref, foot, contact, nthreads=1):
    """The QP solved HPIPM-style (no condensing, Riccati Newton steps): (u [B,N,L,3], status, iters)."""
    B = x0.shape[0]
    N = model.N
    x0, xref, foot = (np.ascontiguousarray(a, dtype=np.float64) for a in (x0, xref, foot))
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    u = np.zeros((B, N, NL, 3))
    st = np.zeros(B, dtype=np.int32)
    it = np.zeros(B, dtype=np.int32)
    lib().oracle_riccati_solve_batch(C.byref(model), C.byref(settings), B, _p(x0), _p(xref), _p(foot),
                                     _p(contact, C.c_uint8), _p(u), _p(st, C.c_int), _p(it, C.c_int), nthreads)
    return u, st, it


def riccati_gain0(model, xref, foot, contact):
    """Unconstrained stage-0 Riccati feedback of the OCP form: (K0 [L,3,13], status)."""
    c = consts(model)
    K0 = np.zeros((NL, 3, NX))
    xref, foot = (np.ascontiguousarray(a, dtype=np.float64) for a in (xref, foot))
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    st = lib().oracle_riccati_gain0(C.byref(c), _p(xref), _p(foot), _p(contact, C.c_uint8), _p(K0))
    return K0, st


def policy(model, xref, foot, contact, u, act_tol=1e-5, lin=None):
    """Feedback policy dU/dx0 of one QP at its solution u [N,L,3] (oracle_policy; lin [N,6]: the QP linearised
    there, oracle_policy_lin): (K [N,L,3,13], n_free, status)."""
    N = model.N
    c = consts(model)
    K = np.zeros((N, NL, 3, NX))
    nfree = C.c_int(0)
    xref, foot, u = (np.ascontiguousarray(a, dtype=np.float64) for a in (xref, foot, u))
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    ln = None if lin is None else np.ascontiguousarray(lin, dtype=np.float64)
    st = lib().oracle_policy_lin(C.byref(c), _p(xref), _p(foot), _p(contact, C.c_uint8),
                                 _p(ln) if ln is not None else None, _p(u), act_tol, _p(K), C.byref(nfree))
    return K, nfree.value, st


def solve_one_lin(model, settings, x0, xref, foot, contact, lin, u_init=None):
    """One QP linearised at lin [N,6] (oracle_solve_one_lin): (u [N,L,3], status, iters)."""
    N = model.N
    c = consts(model)
    u = np.zeros((N, NL, 3)) if u_init is None else np.array(u_init, dtype=np.float64).reshape(N, NL, 3)
    x0, xref, foot, lin = _f64(x0, xref, foot, lin)
    contact = np.ascontiguousarray(contact, dtype=np.uint8)
    it = C.c_int(0)
    st = lib().oracle_solve_one_lin(C.byref(c), C.byref(settings), _p(x0), _p(xref), _p(foot),
                                    _p(contact, C.c_uint8), _p(lin), _p(u), None, C.byref(it))
    return u, st, it.value


def policy_triple(mu, ub, f, tol):
    Z = np.zeros((3, 3))
    ub, f = (np.ascontiguousarray(a, dtype=np.float64) for a in (ub, f))
    k = lib().oracle_policy_triple(mu, _p(ub), _p(f), tol, _p(Z))
    return Z[:, :k]


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().oracle_philox4x32_10(c, k, o)
    return list(o)
