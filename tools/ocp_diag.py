"""GPU diagnostic of the grid form's options (segments, keep_riccati, linres): solve a legged problem for each and
report failures with the HIP error string. Usage: python tools/ocp_diag.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cheeta-mpc_amd", "python"))
import cheeta_mpc as cm  # noqa: E402
from cheeta_mpc import ocp as gen  # noqa: E402

H = cm.hip()
H.hipGetErrorString.restype = __import__("ctypes").c_char_p
for projected in (True, False):
    ps = [gen.legged_problem(580 + i, projected=projected) for i in range(2)]
    p0 = ps[0]
    recs, crecs = zip(*[gen.pack(p) for p in ps])
    for S in (1, 2, 8, 0):
        for keep in (0, 1):
            for lr in (0, 1):
                h = cm.OcpSolver(p0["N"], p0["nx"], p0["nu"], p0.get("nc"), max_batch=2)
                h.set_segments(S)
                h.set_keep_riccati(keep)
                h.set_linres(lr)
                try:
                    x, u, st, it = h.solve(np.array([p["x0"] for p in ps]), np.array(recs),
                                           np.array(crecs) if not projected else None)
                    msg = f"ok st {st.tolist()} it {it.tolist()}"
                except Exception as e:  # noqa: BLE001
                    err = H.hipGetLastError()
                    msg = f"FAIL {e} last hip error {err} {H.hipGetErrorString(err).decode()}"
                print(f"{'proj' if projected else 'rows'} S={S} keep={keep} linres={lr}: {msg}", flush=True)
                h.close()
