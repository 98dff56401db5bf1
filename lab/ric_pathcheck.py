"""Lab check (round 5): Riccati refactorisation (cmpc_ocp_riccati, k_ocp_ric) after solves on each path of the OCP
IPM (batched / latency form, grid off / on) against the oracle, legged problem with rows, B = 3."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cheeta-mpc_amd", "python"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import cheeta_mpc as cm  # noqa: E402
import oracle_py as op  # noqa: E402
from cheeta_mpc import ocp as ocpgen  # noqa: E402


def rel(a, b):
    return float(np.abs(a - b).max() / max(1.0, np.abs(b).max())) if np.size(a) else 0.0


ps = [ocpgen.legged_problem(310 + i, projected=False) for i in range(3)]
p0 = ps[0]
recs, crecs = zip(*[ocpgen.pack(p) for p in ps])
refs = [op.ocp_ipm(p["N"], p["nx"], p["nu"], p["x0"], ocpgen.pack(p)[0], nc=p.get("nc"), crec=ocpgen.pack(p)[1],
                   ric=True) for p in ps]
for path, grid, keep in ((0, 1, 0), (1, 1, 0), (1, 0, 0), (1, 2, 0), (1, 0, 1)):
    s = cm.OcpSolver(p0["N"], p0["nx"], p0["nu"], p0.get("nc"), max_batch=3)
    s.set_path(path)
    s.set_grid(grid)
    s.set_keep_riccati(keep)
    x, u, st, it = s.solve(np.array([p["x0"] for p in ps]), np.array(recs), np.array(crecs))
    P, pv, K, kf, Lr, rst = s.riccati(3)
    for i, r in enumerate(refs):
        lr = [rel(Lr[i][k], r["Lr"][k]) for k in range(p0["N"])]
        pm = max(rel(P[i][k], r["P"][k]) for k in range(1, p0["N"] + 1))
        print(f"path {path} grid {grid} (G {s.grid(3)}) keep {keep} prob {i}: st {st[i]}/{r['status']} it {it[i]}/{r['iters']} "
              f"x {rel(x[i], r['x']):.2e} u {rel(u[i], r['u']):.2e} P {pm:.2e} Lr0 {lr[0]:.2e} Lr max {max(lr):.2e} "
              f"(k {int(np.argmax(lr))}) rst {rst[i]}", flush=True)
