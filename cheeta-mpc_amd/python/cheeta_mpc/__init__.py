"""ctypes bindings of the cheeta-mpc-amd C ABI (include/cmpc/cmpc.h) plus minimal HIP device-memory plumbing.

The product is libcmpc.so (HIP kernels for gfx950 + the C ABI). This module only marshals arguments: it never
computes a solution itself and raises if the native library is missing, so nothing here can silently fall back to
a CPU path. Device memory is managed with the HIP runtime directly (libamdhip64, the one libcmpc.so links); PyTorch
is not needed on the solve path.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.abspath(os.path.join(_HERE, "..", ".."))
LIB_PATH = os.environ.get("CMPC_LIB") or os.path.join(PKG_ROOT, "lib", "libcmpc.so")  # CMPC_LIB: lab builds only

NX, NU, NL = 13, 12, 4
F64, F32 = 0, 1
# kernel-path options of a context (cmpc_set_path; the first three give bit-identical results; PATH_RICCATI: 0 off,
# 1 the n > 64 classes of the fused path, 2 every QP through the stage-wise kernel; PATH_IPM72: 64 < n <= 72 on the bordered
# one-wave kernel where the IPM runs as its own launch)
PATH_FUSED64, PATH_FUSED128, PATH_DIRECT, PATH_RICCATI, PATH_IPM72 = 0, 1, 2, 3, 4
STATUS = {0: "SUCCESS", 1: "MAX_ITER", 2: "MIN_STEP", 3: "NAN_SOL", 4: "INCONS_EQ", 5: "INVALID_CONTACT",
          6: "TOO_LARGE", 7: "INFEASIBLE_STEP"}

# CentoidMPCTest.cpp:19-33
TEST_WEIGHTS = [1, 1, 100, 0.5, 0.5, 0, 2, 2, 8,
                0.2, 0.2, 0.2, 0.3, 0.3, 0.3, 0.1, 0.1, 0.1,
                0.2, 0.2, 0.2, 0.3, 0.3, 0.3, 0.1, 0.1, 0.1,
                0.2, 0.2, 0.2, 0.3, 0.3, 0.3, 0.1, 0.1, 0.1,
                0.2, 0.2, 0.2, 0.3, 0.3, 0.3, 0.1, 0.1, 0.1]


class Model(C.Structure):
    _fields_ = [("N", C.c_int), ("n_legs", C.c_int), ("mass", C.c_double), ("dt", C.c_double),
                ("inertia", C.c_double * 9), ("mu", C.c_double * 4), ("weights", C.c_double * 45),
                ("force_ub", C.c_double * 5), ("theta_weights", C.c_double * 3)]


class Settings(C.Structure):
    _fields_ = [("hpipm_mode", C.c_int), ("iter_max", C.c_int), ("alpha_min", C.c_double), ("mu0", C.c_double),
                ("tol_stat", C.c_double), ("tol_eq", C.c_double), ("tol_ineq", C.c_double),
                ("tol_comp", C.c_double), ("reg_prim", C.c_double), ("warm_start", C.c_int),
                ("pred_corr", C.c_int), ("ric_alg", C.c_int)]


GAIT_MAX_MODES = 16


class IpcHandle(C.Structure):
    """cmpc_ipc_handle (hipIpcMemHandle_t bytes)."""
    _fields_ = [("bytes", C.c_ubyte * 64)]


class Gait(C.Structure):
    """cmpc_gait: ocs2 ModeSequenceTemplate (gait.info modeSequence + switchingTimes)."""
    _fields_ = [("n_modes", C.c_int), ("mode", C.c_int * GAIT_MAX_MODES),
                ("switching_time", C.c_double * (GAIT_MAX_MODES + 1))]


_lib = None
_hip = None


def lib():
    """Load libcmpc.so; raises if it has not been built (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libcmpc.so not found at {LIB_PATH}; run `make -C cheeta-mpc_amd` (or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    P = C.POINTER
    vp, d, i, u8 = C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p
    L.cmpc_settings_default.argtypes = [P(Settings)]
    L.cmpc_settings_default.restype = None
    L.cmpc_model_default.argtypes = [P(Model), C.c_int]
    L.cmpc_model_default.restype = None
    L.cmpc_memsize.argtypes = [P(Model), C.c_int, C.c_int]
    L.cmpc_memsize.restype = C.c_size_t
    L.cmpc_create.argtypes = [P(Model), P(Settings), C.c_int, C.c_int, vp, P(vp)]
    L.cmpc_destroy.argtypes = [vp]
    L.cmpc_set_settings.argtypes = [vp, P(Settings)]
    L.cmpc_set_model.argtypes = [vp, P(Model)]
    L.cmpc_get_model.argtypes = [vp, P(Model)]
    L.cmpc_ctx_ld.argtypes = [vp]
    L.cmpc_ctx_fused.argtypes = [vp]
    L.cmpc_set_path.argtypes = [vp, C.c_int, C.c_int]
    L.cmpc_get_path.argtypes = [vp, C.c_int]
    L.cmpc_get_residuals.argtypes = [vp, C.c_int, d, vp]
    L.cmpc_enable_stats.argtypes = [vp, C.c_int]
    L.cmpc_get_stats.argtypes = [vp, C.c_int, d, vp]
    L.cmpc_solve_batch.argtypes = [vp, C.c_int, d, d, d, u8, d, d, i, i, vp]
    L.cmpc_solve_batch_warm.argtypes = [vp, C.c_int, d, d, d, u8, d, d, d, i, i, vp]
    L.cmpc_sqp_solve_batch.argtypes = [vp, C.c_int, d, d, d, u8, C.c_int, C.c_double, d, d, i, i, i, vp]
    L.cmpc_nlp_solve_batch.argtypes = [vp, C.c_int, d, d, d, u8, C.c_int, C.c_double, d, d, d, i, i, i, vp]
    L.cmpc_condense_lin_batch.argtypes = [vp, C.c_int, d, d, d, u8, d, d, d, d, d, i, i, i, d, d, vp]
    L.cmpc_policy_batch.argtypes = [vp, C.c_int, d, d, d, u8, d, C.c_double, d, i, i, vp]
    L.cmpc_sqp_policy_batch.argtypes = [vp, C.c_int, d, d, d, u8, d, C.c_double, d, i, i, vp]
    L.cmpc_shift_inputs.argtypes = [C.c_int, C.c_int, d, C.c_int, d, vp]
    L.cmpc_solve_batch_host.argtypes = [vp, C.c_int, d, d, d, u8, d, d, i, i]
    L.cmpc_condense_batch.argtypes = [vp, C.c_int, d, d, d, u8, d, d, i, i, vp]
    L.cmpc_qp_solve_batch.argtypes = [vp, C.c_int, d, d, i, d, d, d, d, i, i, vp]
    L.cmpc_generate_batch.argtypes = [P(Model), C.c_uint64, C.c_int64, C.c_int, C.c_int, d, d, d, u8, vp]
    L.cmpc_ocp_record_size.argtypes = [C.c_int, C.c_int, i]
    L.cmpc_ocp_record_size.restype = C.c_size_t
    L.cmpc_ocp_solve_batch_host.argtypes = [C.c_int, C.c_int, C.c_int, i, d, d, d, d, i]
    L.cmpc_ocp_constraint_record_size.argtypes = [C.c_int, C.c_int, i, i]
    L.cmpc_ocp_constraint_record_size.restype = C.c_size_t
    L.cmpc_ocp_solve_batch_eq_host.argtypes = [C.c_int, C.c_int, C.c_int, i, i, d, d, d, d, d, i]
    L.cmpc_gait_builtin.argtypes = [C.c_char_p, P(Gait)]
    L.cmpc_gait_table_create.argtypes = [P(Gait), C.c_int, i, P(vp)]
    L.cmpc_gait_table_destroy.argtypes = [vp]
    L.cmpc_gait_contact_batch.argtypes = [vp, C.c_int, i, d, C.c_double, C.c_double, C.c_int, u8, vp]
    L.cmpc_ocp_riccati_batch_host.argtypes = [C.c_int, C.c_int, C.c_int, i, d, d, d, d, d, i]
    L.cmpc_ocp_memsize.argtypes = [C.c_int, C.c_int, i, i, C.c_int]
    L.cmpc_ocp_memsize.restype = C.c_size_t
    L.cmpc_ocp_create.argtypes = [C.c_int, C.c_int, i, i, P(Settings), C.c_int, P(vp)]
    L.cmpc_ocp_destroy.argtypes = [vp]
    L.cmpc_ocp_set_settings.argtypes = [vp, P(Settings)]
    L.cmpc_ocp_set_path.argtypes = [vp, C.c_int]
    L.cmpc_ocp_path.argtypes = [vp]
    L.cmpc_ocp_set_grid.argtypes = [vp, C.c_int]
    L.cmpc_ocp_grid.argtypes = [vp, C.c_int]
    L.cmpc_ocp_reshape.argtypes = [vp, C.c_int, C.c_int, i, i]
    L.cmpc_ocp_alloc_count.argtypes = [vp]
    L.cmpc_ocp_set_keep_riccati.argtypes = [vp, C.c_int]
    L.cmpc_ocp_enable_timing.argtypes = [vp, C.c_int]
    L.cmpc_ocp_last_solve_ms.argtypes = [vp, P(C.c_float)]
    L.cmpc_ocp_set_linres.argtypes = [vp, C.c_int]
    L.cmpc_ocp_get_linres_host.argtypes = [vp, C.c_int, d]
    L.cmpc_ocp_set_segments.argtypes = [vp, C.c_int]
    L.cmpc_ocp_segments.argtypes = [vp, C.c_int]
    L.cmpc_ocp_set_grid_timeout.argtypes = [vp, C.c_double]
    L.cmpc_ocp_fallback_count.argtypes = [vp]
    L.cmpc_ocp_partition_fallback_count.argtypes = [vp]
    L.cmpc_ocp_debug_force_grid_timeout.argtypes = [vp, C.c_int]
    L.cmpc_ocp_staging.argtypes = [vp, C.c_int]
    L.cmpc_ocp_staging.restype = d
    L.cmpc_ocp_solve.argtypes = [vp, C.c_int, d, d, d, d, d, i, i, vp]
    L.cmpc_ocp_solve_host.argtypes = [vp, C.c_int, d, d, d, d, d, i, i]
    L.cmpc_ocp_riccati.argtypes = [vp, C.c_int, d, d, d, d, d, i, vp]
    L.cmpc_ocp_riccati_host.argtypes = [vp, C.c_int, d, d, d, d, d, i]
    L.cmpc_ocp_riccati_feedback_host.argtypes = [vp, C.c_int, d, d, d, i]
    L.cmpc_ocp_get_residuals.argtypes = [vp, C.c_int, d, vp]
    L.cmpc_ocp_stat_rows.argtypes = [vp]
    L.cmpc_ocp_get_stats.argtypes = [vp, C.c_int, d, vp]
    L.cmpc_ipc_export.argtypes = [vp, P(IpcHandle)]
    L.cmpc_ipc_open.argtypes = [P(IpcHandle), P(vp)]
    L.cmpc_ipc_close.argtypes = [vp]
    L.cmpc_gather_shard.argtypes = [vp, C.c_size_t, vp, C.c_size_t, vp]
    L.cmpc_status_string.argtypes = [C.c_int]
    L.cmpc_status_string.restype = C.c_char_p
    L.cmpc_error_string.argtypes = [C.c_int]
    L.cmpc_error_string.restype = C.c_char_p
    L.cmpc_device_info.argtypes = [P(C.c_int), P(C.c_int), C.c_char_p, C.c_int]
    L.cmpc_version.restype = C.c_char_p
    _lib = L
    return L


def hip():
    """HIP runtime (the libamdhip64 libcmpc.so is linked against)."""
    global _hip
    if _hip is None:
        lib()
        H = C.CDLL("libamdhip64.so.7", mode=C.RTLD_GLOBAL)
        H.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        H.hipFree.argtypes = [C.c_void_p]
        H.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        H.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
        H.hipDeviceSynchronize.argtypes = []
        H.hipStreamCreate.argtypes = [C.POINTER(C.c_void_p)]
        H.hipStreamSynchronize.argtypes = [C.c_void_p]
        H.hipStreamDestroy.argtypes = [C.c_void_p]
        H.hipEventCreate.argtypes = [C.POINTER(C.c_void_p)]
        H.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
        H.hipEventSynchronize.argtypes = [C.c_void_p]
        H.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
        H.hipEventDestroy.argtypes = [C.c_void_p]
        H.hipGetDeviceCount.argtypes = [C.POINTER(C.c_int)]
        H.hipSetDevice.argtypes = [C.c_int]
        H.hipGetErrorString.restype = C.c_char_p
        _hip = H
    return _hip


def _chk(r, what):
    if r != 0:
        raise RuntimeError(f"{what} failed: {r} {lib().cmpc_error_string(r).decode() if r < 0 else ''}")


def _hchk(r, what):
    if r != 0:
        raise RuntimeError(f"{what} failed: hipError {r} {hip().hipGetErrorString(r).decode()}")


def device_pci_id(dev):
    """PCI identity "domain:bus:device.function" of HIP device dev (distinguishes physical GPUs across ranks)."""
    H = hip()
    H.hipDeviceGetPCIBusId.argtypes = [C.c_char_p, C.c_int, C.c_int]
    buf = C.create_string_buffer(64)
    _hchk(H.hipDeviceGetPCIBusId(buf, 64, int(dev)), "hipDeviceGetPCIBusId")
    return buf.value.decode()


def device_count():
    n = C.c_int(0)
    if hip().hipGetDeviceCount(C.byref(n)) != 0:
        return 0
    return n.value


class DeviceArray:
    """A device allocation with a numpy shape/dtype (H2D/D2H via hipMemcpy)."""

    def __init__(self, shape, dtype):
        self.shape = tuple(int(s) for s in shape)
        self.dtype = np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        self.ptr = C.c_void_p()
        _hchk(hip().hipMalloc(C.byref(self.ptr), max(self.nbytes, 1)), "hipMalloc")

    @classmethod
    def from_host(cls, a):
        a = np.ascontiguousarray(a)
        d = cls(a.shape, a.dtype)
        d.upload(a)
        return d

    def upload(self, a):
        a = np.ascontiguousarray(a, dtype=self.dtype)
        assert a.nbytes == self.nbytes
        _hchk(hip().hipMemcpy(self.ptr, a.ctypes.data_as(C.c_void_p), self.nbytes, 1), "hipMemcpy H2D")

    def zero(self):
        _hchk(hip().hipMemset(self.ptr, 0, self.nbytes), "hipMemset")

    def host(self):
        out = np.empty(self.shape, dtype=self.dtype)
        _hchk(hip().hipDeviceSynchronize(), "hipDeviceSynchronize")
        _hchk(hip().hipMemcpy(out.ctypes.data_as(C.c_void_p), self.ptr, self.nbytes, 2), "hipMemcpy D2H")
        return out

    def __del__(self):
        try:
            if self.ptr and _hip is not None:
                _hip.hipFree(self.ptr)
        except Exception:
            pass


def default_model(N=10):
    m = Model()
    lib().cmpc_model_default(C.byref(m), N)
    return m


def default_settings(**kw):
    s = Settings()
    lib().cmpc_settings_default(C.byref(s))
    for k, v in kw.items():
        setattr(s, k, v)
    return s


class Engine:
    """One cmpc context (device workspace for max_batch QPs of horizon model.N)."""

    def __init__(self, model, settings=None, precision=F64, max_batch=4096, path=None):
        """path: {PATH_* option: 0 / 1} applied with cmpc_set_path after creation (A/B tests; default path if None)."""
        self.model = model
        self.settings = settings or default_settings()
        self.precision = precision
        self.max_batch = max_batch
        self.ctx = C.c_void_p()
        _chk(lib().cmpc_create(C.byref(model), C.byref(self.settings), precision, max_batch, None,
                               C.byref(self.ctx)), "cmpc_create")
        self.ld = lib().cmpc_ctx_ld(self.ctx)
        for k, v in (path or {}).items():
            self.set_path(k, v)

    def set_path(self, option, value):
        _chk(lib().cmpc_set_path(self.ctx, option, int(value)), "cmpc_set_path")

    def get_path(self, option):
        return lib().cmpc_get_path(self.ctx, option)

    def close(self):
        if self.ctx:
            lib().cmpc_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_settings(self, s):
        self.settings = s
        _chk(lib().cmpc_set_settings(self.ctx, C.byref(s)), "cmpc_set_settings")

    # ---- device-pointer entry points (async on stream)
    def solve_device(self, B, x0, xref, foot, contact, u, x, status, iters, stream=None, u_init=None):
        """u_init (DeviceArray [B,N,L,3], may be u itself): warm start when settings.warm_start != 0."""
        _chk(lib().cmpc_solve_batch_warm(self.ctx, B, x0.ptr, xref.ptr, foot.ptr, contact.ptr,
                                         u_init.ptr if u_init is not None else None, u.ptr,
                                         x.ptr if x is not None else None, status.ptr,
                                         iters.ptr if iters is not None else None, stream), "cmpc_solve_batch_warm")

    # ---- host convenience
    def solve(self, x0, xref, foot, contact, want_x=True, u_init=None):
        B = x0.shape[0]
        N = self.model.N
        d = {k: DeviceArray.from_host(v) for k, v in
             dict(x0=np.asarray(x0, np.float64), xref=np.asarray(xref, np.float64),
                  foot=np.asarray(foot, np.float64), contact=np.asarray(contact, np.uint8)).items()}
        u = DeviceArray((B, N, NL, 3), np.float64)
        if u_init is not None:
            u.upload(np.asarray(u_init, np.float64).reshape(B, N, NL, 3))
        x = DeviceArray((B, N + 1, NX), np.float64) if want_x else None
        st = DeviceArray((B,), np.int32)
        it = DeviceArray((B,), np.int32)
        self.solve_device(B, d["x0"], d["xref"], d["foot"], d["contact"], u, x, st, it,
                          u_init=u if u_init is not None else None)
        return u.host(), (x.host() if want_x else None), st.host(), it.host()

    def residuals(self, B):
        """Final residuals of the last IPM run, [B, 4] = (stat, eq, ineq, comp) (cmpc_get_residuals)."""
        r = DeviceArray((B, 4), np.float64)
        _chk(lib().cmpc_get_residuals(self.ctx, B, r.ptr, None), "cmpc_get_residuals")
        _hchk(hip().hipDeviceSynchronize(), "hipDeviceSynchronize")
        return r.host()

    STAT_COLS = ("alpha_aff", "mu_aff", "sigma", "alpha_prim", "alpha_dual", "mu", "res_stat", "res_eq", "res_ineq",
                 "res_comp")

    def enable_stats(self, rows):
        """Record the per-iteration statistics table of every following IPM run (cmpc_enable_stats); 0 disables."""
        _chk(lib().cmpc_enable_stats(self.ctx, rows), "cmpc_enable_stats")
        self.stats_rows = rows

    def stats(self, B):
        """[B, rows, 10] per-iteration statistics of the last IPM run (columns STAT_COLS; cmpc_get_stats)."""
        r = DeviceArray((B, self.stats_rows, len(self.STAT_COLS)), np.float64)
        _chk(lib().cmpc_get_stats(self.ctx, B, r.ptr, None), "cmpc_get_stats")
        _hchk(hip().hipDeviceSynchronize(), "hipDeviceSynchronize")
        return r.host()

    def sqp_solve(self, x0, xref, foot, contact, sqp_iter_max=10, sqp_tol=1e-6, want_x=True):
        """Batched SQP on the bilinear NLP (cmpc_sqp_solve_batch): (u, x, status, qp_iters, sqp_iters). sqp_tol is
        ocs2's deltaTol (MultipleShootingSettings.h:43, default 1e-6): the bound on alpha |dx| and alpha |du|."""
        B = x0.shape[0]
        N = self.model.N
        d = {k: DeviceArray.from_host(v) for k, v in
             dict(x0=np.asarray(x0, np.float64), xref=np.asarray(xref, np.float64),
                  foot=np.asarray(foot, np.float64), contact=np.asarray(contact, np.uint8)).items()}
        u = DeviceArray((B, N, NL, 3), np.float64)
        x = DeviceArray((B, N + 1, NX), np.float64) if want_x else None
        st = DeviceArray((B,), np.int32)
        qi = DeviceArray((B,), np.int32)
        si = DeviceArray((B,), np.int32)
        _chk(lib().cmpc_sqp_solve_batch(self.ctx, B, d["x0"].ptr, d["xref"].ptr, d["foot"].ptr, d["contact"].ptr,
                                        sqp_iter_max, sqp_tol, u.ptr, x.ptr if want_x else None, st.ptr, qi.ptr,
                                        si.ptr, None), "cmpc_sqp_solve_batch")
        _hchk(hip().hipDeviceSynchronize(), "hipDeviceSynchronize")
        return u.host(), (x.host() if want_x else None), st.host(), qi.host(), si.host()

    def nlp_solve(self, x0, xref, foot, contact, sqp_iter_max=10, sqp_tol=1e-6, want_x=True):
        """The NLP with the later runs' footholds as decision variables (cmpc_nlp_solve_batch):
        (u, feet [B,N+1,L,3], x, status, qp_iters, sqp_iters)."""
        B = x0.shape[0]
        N = self.model.N
        d = {k: DeviceArray.from_host(v) for k, v in
             dict(x0=np.asarray(x0, np.float64), xref=np.asarray(xref, np.float64),
                  foot=np.asarray(foot, np.float64), contact=np.asarray(contact, np.uint8)).items()}
        u = DeviceArray((B, N, NL, 3), np.float64)
        feet = DeviceArray((B, N + 1, NL, 3), np.float64)
        x = DeviceArray((B, N + 1, NX), np.float64) if want_x else None
        st = DeviceArray((B,), np.int32)
        qi = DeviceArray((B,), np.int32)
        si = DeviceArray((B,), np.int32)
        _chk(lib().cmpc_nlp_solve_batch(self.ctx, B, d["x0"].ptr, d["xref"].ptr, d["foot"].ptr, d["contact"].ptr,
                                        sqp_iter_max, sqp_tol, u.ptr, feet.ptr, x.ptr if want_x else None, st.ptr,
                                        qi.ptr, si.ptr, None), "cmpc_nlp_solve_batch")
        _hchk(hip().hipDeviceSynchronize(), "hipDeviceSynchronize")
        return u.host(), feet.host(), (x.host() if want_x else None), st.host(), qi.host(), si.host()

    def condense_lin(self, x0, xref, foot, contact, lin=None, ubar=None, dbar=None):
        """Condensed QP at a linearisation point (cmpc_condense_lin_batch): (H, g, n, status, tri_map, lo, hi)."""
        B = x0.shape[0]
        nt = self.ld // 3
        d = [DeviceArray.from_host(np.asarray(a, t)) if a is not None else None for a, t in
             ((x0, np.float64), (xref, np.float64), (foot, np.float64), (contact, np.uint8), (lin, np.float64),
              (ubar, np.float64), (dbar, np.float64))]
        H = DeviceArray((B, self.ld, self.ld), np.float64)
        g = DeviceArray((B, self.ld), np.float64)
        n = DeviceArray((B,), np.int32)
        st = DeviceArray((B,), np.int32)
        mp = DeviceArray((B, nt), np.int32)
        lo = DeviceArray((B, nt, 5), np.float64)
        hi = DeviceArray((B, nt, 5), np.float64)
        p = [a.ptr if a is not None else None for a in d]
        _chk(lib().cmpc_condense_lin_batch(self.ctx, B, *p, H.ptr, g.ptr, n.ptr, st.ptr, mp.ptr, lo.ptr, hi.ptr,
                                           None), "cmpc_condense_lin_batch")
        _hchk(hip().hipDeviceSynchronize(), "hipDeviceSynchronize")
        return H.host(), g.host(), n.host(), st.host(), mp.host(), lo.host(), hi.host()

    def policy(self, x0, xref, foot, contact, u, act_tol=0.0):
        """Feedback policy dU/dx0 at the solution u [B,N,L,3] (cmpc_policy_batch): (K [B,N,L,3,13], nfree, status).
        act_tol <= 0 selects the precision default."""
        B = x0.shape[0]
        N = self.model.N
        d = [DeviceArray.from_host(np.asarray(a, t)) for a, t in
             ((x0, np.float64), (xref, np.float64), (foot, np.float64), (contact, np.uint8),
              (np.asarray(u, np.float64).reshape(B, N, NL, 3), np.float64))]
        K = DeviceArray((B, N, NL, 3, NX), np.float64)
        nf = DeviceArray((B,), np.int32)
        st = DeviceArray((B,), np.int32)
        _chk(lib().cmpc_policy_batch(self.ctx, B, d[0].ptr, d[1].ptr, d[2].ptr, d[3].ptr, d[4].ptr, act_tol, K.ptr,
                                     nf.ptr, st.ptr, None), "cmpc_policy_batch")
        _hchk(hip().hipDeviceSynchronize(), "hipDeviceSynchronize")
        return K.host(), nf.host(), st.host()

    def sqp_policy(self, x0, xref, foot, contact, u, act_tol=0.0):
        """Feedback policy of the QP linearised at the nonlinear rollout of u (cmpc_sqp_policy_batch)."""
        B = x0.shape[0]
        N = self.model.N
        d = [DeviceArray.from_host(np.asarray(a, t)) for a, t in
             ((x0, np.float64), (xref, np.float64), (foot, np.float64), (contact, np.uint8),
              (np.asarray(u, np.float64).reshape(B, N, NL, 3), np.float64))]
        K = DeviceArray((B, N, NL, 3, NX), np.float64)
        nf = DeviceArray((B,), np.int32)
        st = DeviceArray((B,), np.int32)
        _chk(lib().cmpc_sqp_policy_batch(self.ctx, B, d[0].ptr, d[1].ptr, d[2].ptr, d[3].ptr, d[4].ptr, act_tol,
                                         K.ptr, nf.ptr, st.ptr, None), "cmpc_sqp_policy_batch")
        _hchk(hip().hipDeviceSynchronize(), "hipDeviceSynchronize")
        return K.host(), nf.host(), st.host()

    def condense(self, x0, xref, foot, contact):
        B = x0.shape[0]
        d = [DeviceArray.from_host(np.asarray(a, t)) for a, t in
             ((x0, np.float64), (xref, np.float64), (foot, np.float64), (contact, np.uint8))]
        H = DeviceArray((B, self.ld, self.ld), np.float64)
        g = DeviceArray((B, self.ld), np.float64)
        n = DeviceArray((B,), np.int32)
        st = DeviceArray((B,), np.int32)
        _chk(lib().cmpc_condense_batch(self.ctx, B, d[0].ptr, d[1].ptr, d[2].ptr, d[3].ptr, H.ptr, g.ptr, n.ptr,
                                       st.ptr, None), "cmpc_condense_batch")
        return H.host(), g.host(), n.host(), st.host()

    def qp_solve(self, H, g, n, mu, lo, hi):
        B = H.shape[0]
        ld = self.ld
        assert H.shape == (B, ld, ld)
        d = [DeviceArray.from_host(np.ascontiguousarray(a, t)) for a, t in
             ((H, np.float64), (g, np.float64), (n, np.int32), (mu, np.float64), (lo, np.float64), (hi, np.float64))]
        u = DeviceArray((B, ld), np.float64)
        st = DeviceArray((B,), np.int32)
        it = DeviceArray((B,), np.int32)
        _chk(lib().cmpc_qp_solve_batch(self.ctx, B, *[a.ptr for a in d], u.ptr, st.ptr, it.ptr, None),
             "cmpc_qp_solve_batch")
        return u.host(), st.host(), it.host()


def generate_device(model, seed, B, gait=0, offset=0, stream=None):
    N = model.N
    x0 = DeviceArray((B, NX), np.float64)
    xref = DeviceArray((B, N + 1, NX), np.float64)
    foot = DeviceArray((B, N + 1, NL, 3), np.float64)
    contact = DeviceArray((B, N, NL), np.uint8)
    _chk(lib().cmpc_generate_batch(C.byref(model), seed, offset, B, gait, x0.ptr, xref.ptr, foot.ptr, contact.ptr,
                                   stream), "cmpc_generate_batch")
    return x0, xref, foot, contact


def ocp_solve(N, nx, nu, x0, rec):
    """Batched generic OCP-QP (HpipmInterface semantics) on the device; x0 [B,nx], rec [B,record]."""
    x0 = np.ascontiguousarray(np.atleast_2d(x0), np.float64)
    rec = np.ascontiguousarray(np.atleast_2d(rec), np.float64)
    B = x0.shape[0]
    nua = np.ascontiguousarray(nu, np.int32)
    nU = int(nua.sum())
    x = np.zeros((B, N + 1, nx))
    u = np.zeros((B, max(nU, 1)))
    st = np.zeros(B, np.int32)
    vp = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    _chk(lib().cmpc_ocp_solve_batch_host(B, N, nx, vp(nua), vp(x0), vp(rec), vp(x), vp(u), vp(st)),
         "cmpc_ocp_solve_batch_host")
    return x, u[:, :nU], st


def ocp_solve_eq(N, nx, nu, nc, x0, rec, crec):
    """ocp_solve with equality constraints C_k x_k + D_k u_k + e_k = 0 (nc_k rows at node k = 0..N); crec [B,record]
    as cmpc_ocp_constraint_record_size (cmpc.h)."""
    x0 = np.ascontiguousarray(np.atleast_2d(x0), np.float64)
    rec = np.ascontiguousarray(np.atleast_2d(rec), np.float64)
    crec = np.ascontiguousarray(np.atleast_2d(crec), np.float64)
    B = x0.shape[0]
    nua = np.ascontiguousarray(nu, np.int32)
    nca = np.ascontiguousarray(nc, np.int32)
    nU = int(nua.sum())
    x = np.zeros((B, N + 1, nx))
    u = np.zeros((B, max(nU, 1)))
    st = np.zeros(B, np.int32)
    vp = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    _chk(lib().cmpc_ocp_solve_batch_eq_host(B, N, nx, vp(nua), vp(nca), vp(x0), vp(rec), vp(crec), vp(x), vp(u),
                                            vp(st)), "cmpc_ocp_solve_batch_eq_host")
    return x, u[:, :nU], st


def _dp(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


class OcpSolver:
    """cmpc_ocp handle (the HpipmInterface::solve path, cmpc.h): dimensions N, nx, nu [N], nc [N+1] (None: no rows),
    settings and device memory for max_batch problems, allocated once."""

    def __init__(self, N, nx, nu, nc=None, settings=None, max_batch=1):
        self.N, self.nx = int(N), int(nx)
        self.nu = np.ascontiguousarray(list(nu)[:N], dtype=np.int32)
        self.nc = None if nc is None else np.ascontiguousarray(list(nc), dtype=np.int32)
        self.nU = int(self.nu.sum())
        self.m = 0 if self.nc is None else int(self.nc.sum())
        self.nK = int(self.nu.sum()) * self.nx
        self.nM = int((self.nu.astype(np.int64) ** 2).sum())
        self.settings = settings or default_settings()
        self.max_batch = int(max_batch)
        self.h = C.c_void_p()
        _chk(lib().cmpc_ocp_create(self.N, self.nx, _dp(self.nu), _dp(self.nc), C.byref(self.settings), self.max_batch,
                                   C.byref(self.h)), "cmpc_ocp_create")
        self.rec_size = int(lib().cmpc_ocp_record_size(self.N, self.nx, _dp(self.nu)))
        self.crec_size = (int(lib().cmpc_ocp_constraint_record_size(self.N, self.nx, _dp(self.nu), _dp(self.nc)))
                          if self.nc is not None else 0)
        self.stat_rows = lib().cmpc_ocp_stat_rows(self.h)
        self._views = []  # staging views handed out since the last reshape (cmpc.h: valid until reshape / destroy)
        self._stale = []  # (address, bytes) of staging blocks a reshape or close invalidated

    def _invalidate_staging(self):
        # cmpc_ocp_staging's pointers die with a reshape (the pin block may be reallocated, the record offsets move) or
        # the handle: the views handed out become read-only, and solve() refuses arrays inside the old blocks
        for v in self._views:
            self._stale.append((v.ctypes.data, v.nbytes))
            try:
                v.flags.writeable = False
            except ValueError:
                pass
        self._views = []

    def _check_not_stale(self, *arrays):
        for a in arrays:
            if a is None or not self._stale:
                continue
            lo, hi = a.ctypes.data, a.ctypes.data + a.nbytes
            for addr, n in self._stale:
                if lo < addr + n and addr < hi:
                    raise RuntimeError("OcpSolver: an input lies in staging invalidated by reshape()/close(); "
                                       "call staging() again")

    def close(self):
        if self.h:
            self._invalidate_staging()
            lib().cmpc_ocp_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_settings(self, s):
        self.settings = s
        _chk(lib().cmpc_ocp_set_settings(self.h, C.byref(s)), "cmpc_ocp_set_settings")
        self.stat_rows = lib().cmpc_ocp_stat_rows(self.h)

    def set_path(self, chain):
        """cmpc_ocp_set_path: 1 = the latency form of the factorisation for batches <= 256 (default, where the
        dimensions fit it), 0 = the batched form everywhere."""
        _chk(lib().cmpc_ocp_set_path(self.h, int(chain)), "cmpc_ocp_set_path")

    @property
    def path(self):
        return int(lib().cmpc_ocp_path(self.h))

    def set_grid(self, G):
        """cmpc_ocp_set_grid: workgroups per problem of the grid form (0 auto, 1 off)."""
        _chk(lib().cmpc_ocp_set_grid(self.h, int(G)), "cmpc_ocp_set_grid")

    def grid(self, B):
        return int(lib().cmpc_ocp_grid(self.h, int(B)))

    def set_segments(self, S):
        """cmpc_ocp_set_segments: segments of the grid form's partitioned factorisation (0 auto, 1 the serial chain)."""
        _chk(lib().cmpc_ocp_set_segments(self.h, int(S)), "cmpc_ocp_set_segments")

    def segments(self, B):
        return int(lib().cmpc_ocp_segments(self.h, int(B)))

    def set_grid_timeout(self, us):
        """cmpc_ocp_set_grid_timeout: the grid barriers' wait bound in microseconds (0: the default 50 ms)."""
        _chk(lib().cmpc_ocp_set_grid_timeout(self.h, float(us)), "cmpc_ocp_set_grid_timeout")

    def force_grid_timeout(self, on):
        """cmpc_ocp_debug_force_grid_timeout: every grid barrier times out at once (the fallback's test switch)."""
        _chk(lib().cmpc_ocp_debug_force_grid_timeout(self.h, int(on)), "cmpc_ocp_debug_force_grid_timeout")

    @property
    def fallback_count(self):
        """Problems re-solved on one workgroup after a grid-barrier timeout since the handle was created."""
        n = int(lib().cmpc_ocp_fallback_count(self.h))
        if n < 0:
            _chk(n, "cmpc_ocp_fallback_count")
        return n

    @property
    def partition_fallbacks(self):
        """Factorisations of the partitioned form that fell back to the serial chain since the handle was created."""
        n = int(lib().cmpc_ocp_partition_fallback_count(self.h))
        if n < 0:
            _chk(n, "cmpc_ocp_partition_fallback_count")
        return n

    def reshape(self, N, nx, nu, nc=None):
        """cmpc_ocp_reshape: new dimensions on the same handle (grow-only buffers, HpipmInterface::resize)."""
        nu_a = np.ascontiguousarray(list(nu)[:N], dtype=np.int32)
        nc_a = None if nc is None else np.ascontiguousarray(list(nc), dtype=np.int32)
        self._invalidate_staging()
        _chk(lib().cmpc_ocp_reshape(self.h, int(N), int(nx), _dp(nu_a), _dp(nc_a)), "cmpc_ocp_reshape")
        self.N, self.nx, self.nu, self.nc = int(N), int(nx), nu_a, nc_a
        self.nU = int(nu_a.sum())
        self.m = 0 if nc_a is None else int(nc_a.sum())
        self.nK = self.nU * self.nx
        self.nM = int((nu_a.astype(np.int64) ** 2).sum())
        self.rec_size = int(lib().cmpc_ocp_record_size(self.N, self.nx, _dp(nu_a)))
        self.crec_size = (int(lib().cmpc_ocp_constraint_record_size(self.N, self.nx, _dp(nu_a), _dp(nc_a)))
                          if nc_a is not None else 0)

    @property
    def alloc_count(self):
        return int(lib().cmpc_ocp_alloc_count(self.h))

    def set_keep_riccati(self, on):
        _chk(lib().cmpc_ocp_set_keep_riccati(self.h, int(on)), "cmpc_ocp_set_keep_riccati")

    def enable_timing(self, on):
        _chk(lib().cmpc_ocp_enable_timing(self.h, int(on)), "cmpc_ocp_enable_timing")

    def last_solve_ms(self):
        ms = C.c_float()
        _chk(lib().cmpc_ocp_last_solve_ms(self.h, C.byref(ms)), "cmpc_ocp_last_solve_ms")
        return float(ms.value)

    def staging(self):
        """numpy views of the handle's pinned staging (cmpc_ocp_staging): x0 [max_batch, nx], rec [max_batch,
        rec_size], crec [max_batch, crec_size] or None; a solve whose inputs are these views copies nothing on the host
        (the records are written in place, as the C++ mirror packs them). None when the handle has no staging.
        The views are valid until the next reshape() or close() (cmpc.h): those make them read-only, and solve() refuses
        inputs inside invalidated staging — fetch them again."""
        out = []
        for which, n in ((0, self.nx), (1, self.rec_size), (2, self.crec_size if self.m else 0)):
            if n == 0:
                out.append(None)
                continue
            ptr = lib().cmpc_ocp_staging(self.h, which)
            if not ptr:
                return None
            arr = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_double)), shape=(self.max_batch * n,))
            view = arr.reshape(self.max_batch, n)
            self._views.append(view)
            lo, hi = view.ctypes.data, view.ctypes.data + view.nbytes  # the live staging is not stale (a reshape
            self._stale = [(ad, m) for ad, m in self._stale if not (lo < ad + m and ad < hi)]  # may keep the block)
            out.append(view)
        return tuple(out)

    def solve(self, x0, rec, crec=None, guess=None):
        """Host path (cmpc_ocp_solve_host): x0 [B,nx], rec [B,rec_size], crec [B,crec_size]; guess = (x, u), the
        initial guess read when the settings' warm_start is set. Returns x [B,N+1,nx], u [B,nU], status [B], iters."""
        self._check_not_stale(*(a for a in (x0, rec, crec) if isinstance(a, np.ndarray)))
        x0 = np.ascontiguousarray(np.atleast_2d(x0), np.float64)
        B = x0.shape[0]
        rec = np.ascontiguousarray(rec, np.float64).reshape(B, self.rec_size)
        cr = None if self.m == 0 else np.ascontiguousarray(crec, np.float64).reshape(B, self.crec_size)
        x = np.zeros((B, self.N + 1, self.nx))
        u = np.zeros((B, max(self.nU, 1)))
        if guess is not None:
            x[:] = np.asarray(guess[0], np.float64).reshape(B, self.N + 1, self.nx)
            u[:, :self.nU] = np.asarray(guess[1], np.float64).reshape(B, self.nU)
        st = np.zeros(B, np.int32)
        it = np.zeros(B, np.int32)
        _chk(lib().cmpc_ocp_solve_host(self.h, B, _dp(x0), _dp(rec), _dp(cr), _dp(x), _dp(u), _dp(st), _dp(it)),
             "cmpc_ocp_solve_host")
        return x, u[:, :self.nU], st, it

    def solve_device(self, B, x0, rec, crec, x, u, status, iters, stream=None):
        _chk(lib().cmpc_ocp_solve(self.h, B, x0.ptr, rec.ptr, crec.ptr if crec is not None else None, x.ptr, u.ptr,
                                  status.ptr, iters.ptr if iters is not None else None, stream), "cmpc_ocp_solve")

    def riccati(self, B):
        """cmpc_ocp_riccati_host of the last solve: P [B,N+1,nx,nx], p [B,N+1,nx], K (B lists of nu_k x nx), k, Lr (HPIPM's
        ric_Lr, lower), status [B]."""
        N, nx = self.N, self.nx
        P = np.zeros((B, (N + 1) * nx * nx))
        p = np.zeros((B, (N + 1) * nx))
        K = np.zeros((B, max(self.nK, 1)))
        k = np.zeros((B, max(self.nU, 1)))
        M = np.zeros((B, max(self.nM, 1)))
        st = np.zeros(B, np.int32)
        _chk(lib().cmpc_ocp_riccati_host(self.h, B, _dp(P), _dp(p), _dp(K), _dp(k), _dp(M), _dp(st)),
             "cmpc_ocp_riccati_host")
        Ks, ks, Ms = [], [], []
        for b in range(B):
            kb, kk, mb, o, ok, om = [], [], [], 0, 0, 0
            for s in range(N):
                m = int(self.nu[s])
                kb.append(K[b, o:o + m * nx].reshape(nx, m).T.copy())
                kk.append(k[b, ok:ok + m].copy())
                mb.append(M[b, om:om + m * m].reshape(m, m).T.copy())
                o += m * nx
                ok += m
                om += m * m
            Ks.append(kb)
            ks.append(kk)
            Ms.append(mb)
        return (P.reshape(B, N + 1, nx, nx).transpose(0, 1, 3, 2).copy(), p.reshape(B, N + 1, nx), Ks, ks, Ms, st)

    def riccati_feedback(self, b=0):
        """cmpc_ocp_riccati_feedback_host of problem b: K (list of nu_k x nx), Lr (list, lower), P_1 [nx, nx], status."""
        N, nx = self.N, self.nx
        K = np.zeros(max(self.nK, 1))
        M = np.zeros(max(self.nM, 1))
        P1 = np.zeros(nx * nx)
        st = np.zeros(1, np.int32)
        _chk(lib().cmpc_ocp_riccati_feedback_host(self.h, b, _dp(K), _dp(M), _dp(P1), _dp(st)),
             "cmpc_ocp_riccati_feedback_host")
        Ks, Ms, o, om = [], [], 0, 0
        for s in range(N):
            m = int(self.nu[s])
            Ks.append(K[o:o + m * nx].reshape(nx, m).T.copy())
            Ms.append(M[om:om + m * m].reshape(m, m).T.copy())
            o += m * nx
            om += m * m
        return Ks, Ms, P1.reshape(nx, nx).T.copy(), int(st[0])

    def residuals(self, B):
        d = DeviceArray((B, 4), np.float64)
        _chk(lib().cmpc_ocp_get_residuals(self.h, B, d.ptr, None), "cmpc_ocp_get_residuals")
        return d.host()

    def set_linres(self, on):
        """cmpc_ocp_set_linres: record each iteration's Newton-system residuals (HPIPM's lin res statistics)."""
        _chk(lib().cmpc_ocp_set_linres(self.h, int(on)), "cmpc_ocp_set_linres")

    def linres(self, B):
        out = np.zeros((B, self.stat_rows, 4))
        _chk(lib().cmpc_ocp_get_linres_host(self.h, B, _dp(out)), "cmpc_ocp_get_linres_host")
        return out

    def stats(self, B):
        d = DeviceArray((B, self.stat_rows, 10), np.float64)
        _chk(lib().cmpc_ocp_get_stats(self.h, B, d.ptr, None), "cmpc_ocp_get_stats")
        return d.host()


def ocp_riccati(N, nx, nu, rec):
    """Batched device Riccati recursion of the OCP (HpipmInterface::getRiccati*): returns Sm [B,N+1,nx,nx],
    sv [B,N+1,nx], K (per problem a list of nu_k x nx arrays), kff (per problem a list of nu_k vectors), status [B]."""
    rec = np.ascontiguousarray(np.atleast_2d(rec), np.float64)
    B = rec.shape[0]
    nua = np.ascontiguousarray(nu, np.int32)
    nU = int(nua.sum())
    Sm = np.zeros((B, N + 1, nx * nx))
    sv = np.zeros((B, N + 1, nx))
    K = np.zeros((B, max(nU * nx, 1)))
    kff = np.zeros((B, max(nU, 1)))
    st = np.zeros(B, np.int32)
    vp = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    _chk(lib().cmpc_ocp_riccati_batch_host(B, N, nx, vp(nua), vp(rec), vp(Sm), vp(sv), vp(K), vp(kff), vp(st)),
         "cmpc_ocp_riccati_batch_host")
    Sm = Sm.reshape(B, N + 1, nx, nx).transpose(0, 1, 3, 2)  # column-major blocks
    Ks, ks = [], []
    for b in range(B):
        o, ok, Kb, kb = 0, 0, [], []
        for k in range(N):
            m = int(nua[k])
            Kb.append(K[b, o:o + m * nx].reshape(nx, m).T)
            kb.append(kff[b, ok:ok + m])
            o += m * nx
            ok += m
        Ks.append(Kb)
        ks.append(kb)
    return Sm, sv, Ks, ks, st


def gait_builtin(name):
    g = Gait()
    _chk(lib().cmpc_gait_builtin(name.encode(), C.byref(g)), f"cmpc_gait_builtin({name})")
    return g


class GaitTable:
    """Device table of gait templates (cmpc_gait_table); contact() fills a [B,N,4] device contact table."""

    def __init__(self, gaits, leg_map=None):
        arr = (Gait * len(gaits))(*gaits)
        self.ptr = C.c_void_p()
        lm = None if leg_map is None else (C.c_int * 4)(*leg_map)
        _chk(lib().cmpc_gait_table_create(arr, len(gaits), C.cast(lm, C.POINTER(C.c_int)) if lm else None,
                                          C.byref(self.ptr)), "cmpc_gait_table_create")

    def contact_device(self, B, gait_id, t_start, t0, dt, N, contact, stream=None):
        _chk(lib().cmpc_gait_contact_batch(self.ptr, B, gait_id.ptr, t_start.ptr, t0, dt, N, contact.ptr, stream),
             "cmpc_gait_contact_batch")

    def contact(self, gait_id, t_start, t0, dt, N):
        gid = DeviceArray.from_host(np.ascontiguousarray(gait_id, np.int32))
        ts = DeviceArray.from_host(np.ascontiguousarray(t_start, np.float64))
        B = gid.shape[0]
        out = DeviceArray((B, N, 4), np.uint8)
        self.contact_device(B, gid, ts, t0, dt, N, out)
        _hchk(hip().hipDeviceSynchronize(), "hipDeviceSynchronize")
        return out.host()

    def __del__(self):
        try:
            if self.ptr:
                lib().cmpc_gait_table_destroy(self.ptr)
        except Exception:
            pass


def shift_inputs(u, shift=1):
    """Receding-horizon shift on the device (cmpc_shift_inputs): out[:, k] = u[:, min(k + shift, N - 1)]."""
    u = np.ascontiguousarray(u, np.float64)
    B, N = u.shape[0], u.shape[1]
    din = DeviceArray.from_host(u)
    dout = DeviceArray(u.shape, np.float64)
    _chk(lib().cmpc_shift_inputs(B, N, din.ptr, shift, dout.ptr, None), "cmpc_shift_inputs")
    _hchk(hip().hipDeviceSynchronize(), "hipDeviceSynchronize")
    return dout.host()


def device_info():
    cu, clk = C.c_int(0), C.c_int(0)
    arch = C.create_string_buffer(64)
    _chk(lib().cmpc_device_info(C.byref(cu), C.byref(clk), arch, 64), "cmpc_device_info")
    return cu.value, clk.value, arch.value.decode()
