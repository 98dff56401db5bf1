"""Quick GPU timing of cmpc_ocp_solve on legged-size problems (device pointers, HIP events on the solve stream).
Usage: python tools/ocp_probe.py [B ...]; phase stamps of a lab build (lab/ocp_stamps.sh):
CMPC_LIB=lab/_stamps/libcmpc_ocpstamps.so python tools/ocp_probe.py --stamps"""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cheeta-mpc_amd", "python"))
import cheeta_mpc as cm  # noqa: E402
from cheeta_mpc import ocp as gen  # noqa: E402


def run(projected, B, reps=int(os.environ.get("OCP_REPS", "5"))):
    H = cm.hip()
    ps = [gen.legged_problem(1000 + (i % 16), projected=projected) for i in range(B)]
    p0 = ps[0]
    recs, crecs = zip(*[gen.pack(p) for p in ps])
    s = cm.OcpSolver(p0["N"], p0["nx"], p0["nu"], p0.get("nc"), max_batch=B)
    s.set_path(int(os.environ.get("OCP_CHAIN", "1")))
    s.set_grid(int(os.environ.get("OCP_GRID", "0")))
    s.set_segments(int(os.environ.get("OCP_SEGS", "0")))
    dx0 = cm.DeviceArray.from_host(np.array([p["x0"] for p in ps]))
    drec = cm.DeviceArray.from_host(np.array(recs))
    dcrec = cm.DeviceArray.from_host(np.array(crecs)) if not projected else None
    dx = cm.DeviceArray((B, p0["N"] + 1, p0["nx"]), np.float64)
    du = cm.DeviceArray((B, max(s.nU, 1)), np.float64)
    dst = cm.DeviceArray((B,), np.int32)
    dit = cm.DeviceArray((B,), np.int32)
    stream = C.c_void_p()
    H.hipStreamCreate(C.byref(stream))
    e0, e1 = C.c_void_p(), C.c_void_p()
    H.hipEventCreate(C.byref(e0))
    H.hipEventCreate(C.byref(e1))
    s.solve_device(B, dx0, drec, dcrec, dx, du, dst, dit, stream)  # warm-up
    H.hipStreamSynchronize(stream)
    H.hipEventRecord(e0, stream)
    for _ in range(reps):
        s.solve_device(B, dx0, drec, dcrec, dx, du, dst, dit, stream)
    H.hipEventRecord(e1, stream)
    H.hipEventSynchronize(e1)
    ms = C.c_float()
    H.hipEventElapsedTime(C.byref(ms), e0, e1)
    st, it = dst.host(), dit.host()
    # host entry point (PCIe-inclusive) at this B
    t = time.perf_counter()
    s.solve(np.array([p["x0"] for p in ps]), np.array(recs), np.array(crecs) if not projected else None)
    th = (time.perf_counter() - t) * 1e3
    per = ms.value / reps
    print(f"{'projected' if projected else 'rows     '} B={B:5d} N={p0['N']} nx=24 nu={sorted(set(p0['nu']))} "
          f"kernel {per:8.3f} ms/solve ({B / per * 1e3:9.0f} solves/s), iters {it.mean():.2f}, "
          f"status ok {np.mean(st == 0):.2f}; host path {th:.2f} ms; path {s.path} grid {s.grid(B)} segments "
          f"{s.segments(B)} fallbacks {s.fallback_count} serial fallbacks {s.partition_fallbacks}", flush=True)


if __name__ == "__main__" and "--stamps" not in sys.argv and "--chain" not in sys.argv:
    Bs = [int(a) for a in sys.argv[1:]] or [1, 64, 256, 1024]
    for proj in (True, False):
        for B in Bs:
            run(proj, B)


def stamps(projected, B=1):
    """Per-phase cycles of problem 0 (lab build: CMPC_LIB=lab/_stamps/libcmpc_ocpstamps.so)."""
    L = cm.lib()
    L.cmpc_ocp_debug_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    buf = (C.c_ulonglong * 48)()
    ps = [gen.legged_problem(1000 + i, projected=projected) for i in range(B)]
    p0 = ps[0]
    recs, crecs = zip(*[gen.pack(p) for p in ps])
    s = cm.OcpSolver(p0["N"], p0["nx"], p0["nu"], p0.get("nc"), max_batch=B)
    s.set_path(int(os.environ.get("OCP_CHAIN", "1")))
    s.set_grid(int(os.environ.get("OCP_GRID", "0")))
    s.set_segments(int(os.environ.get("OCP_SEGS", "0")))
    x0 = np.array([p["x0"] for p in ps])
    s.solve(x0, np.array(recs), np.array(crecs) if not projected else None)
    L.cmpc_ocp_debug_stamps(buf, 1)
    x, u, st, it = s.solve(x0, np.array(recs), np.array(crecs) if not projected else None)
    L.cmpc_ocp_debug_stamps(buf, 1)
    names = {1: "residuals", 2: "rhs", 10: "[wg1 el:fetch]", 11: "[wg1 el:Yd]", 12: "[wg1 el:Acl,bcl]",
             13: "[wg1 el:accum+Gw]", 14: "[wg0 comb:products]", 15: "[wg0 comb:elim]", 16: "[wg0 comb:out]", 20: "chain:init", 21: "chain:T", 22: "chain:M",
             23: "chain:elim", 24: "chain:out", 25: "chain:outw0", 26: "[w1 load span]", 27: "chain:e-load", 28: "grid prologue", 17: "fact:exit", 3: "acl", 4: "forward",
             5: "post", 6: "corr rhs", 7: "backward", 8: "acl+forward (corr)", 9: "update", 18: "part:P1+wait",
             19: "part:combine+wait", 29: "part:P3", 30: "[wg1 chain spans]", 31: "[wg1 element spans]",
             32: "residuals: compute", 33: "acl: gains", 34: "scan: compose", 35: "scan: barrier"}
    tot = sum(buf[i] for i in names if i not in (10, 11, 12, 13, 14, 15, 16, 26, 30, 31))  # spans (other timelines)
    print(f"stamps {'projected' if projected else 'rows'} B={B} iters {it[0]} total {tot} cycles")
    for i, n in names.items():
        print(f"  {n:22s} {buf[i]:12d}  {100.0 * buf[i] / max(tot, 1):5.1f} %")


def chain_only(projected, B=1, reps=50):
    """The latency-form factorisation alone (lab build: CMPC_LIB=lab/_stamps/libcmpc_ocpchain.so), ms per launch."""
    L = cm.lib()
    L.cmpc_ocp_debug_chain.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_float)]
    ps = [gen.legged_problem(1000 + i, projected=projected) for i in range(B)]
    p0 = ps[0]
    recs, crecs = zip(*[gen.pack(p) for p in ps])
    s = cm.OcpSolver(p0["N"], p0["nx"], p0["nu"], p0.get("nc"), max_batch=B)
    dx0 = cm.DeviceArray.from_host(np.array([p["x0"] for p in ps]))
    drec = cm.DeviceArray.from_host(np.array(recs))
    dcrec = cm.DeviceArray.from_host(np.array(crecs)) if not projected else None
    dx = cm.DeviceArray((B, p0["N"] + 1, p0["nx"]), np.float64)
    du = cm.DeviceArray((B, max(s.nU, 1)), np.float64)
    dst = cm.DeviceArray((B,), np.int32)
    s.solve_device(B, dx0, drec, dcrec, dx, du, dst, None)
    cm.hip().hipDeviceSynchronize()
    ms = C.c_float()
    L.cmpc_ocp_debug_chain(s.h, B, 3, C.byref(ms))
    r = L.cmpc_ocp_debug_chain(s.h, B, reps, C.byref(ms))
    print(f"chain-only {'projected' if projected else 'rows'} B={B}: rc {r} {ms.value * 1e3:.1f} us per factorisation "
          f"({ms.value * 1e3 / p0['N']:.2f} us per stage)", flush=True)


if __name__ == "__main__" and "--stamps" in sys.argv:
    stamps(True)
    stamps(False)
if __name__ == "__main__" and "--chain" in sys.argv:
    chain_only(True)
    chain_only(False)
