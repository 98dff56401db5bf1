"""Device vs oracle per-iteration statistics of one legacy with_constraints problem (tests/test_ocp_eq.py seed 54)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("cheeta-mpc_amd/python", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import cheeta_mpc as cm  # noqa: E402
import oracle_py as op  # noqa: E402
from cheeta_mpc import ocp as gen  # noqa: E402
from test_ocp_eq import _problem  # noqa: E402

np.set_printoptions(linewidth=200, precision=4)
for seed in (54, 50):
    p = _problem(seed, N=5, nx=3, nu=[2] * 5, nc=[1, 0, 1, 1, 1, 1])
    rec, crec = gen.pack(p)
    s = cm.OcpSolver(p["N"], p["nx"], p["nu"], p["nc"], max_batch=1)
    x, u, st, it = s.solve(p["x0"][None], rec[None], crec[None])
    dstats = s.stats(1)[0]
    r = op.ocp_ipm(p["N"], p["nx"], p["nu"], p["x0"], rec, nc=p["nc"], crec=crec, stats_rows=s.stat_rows)
    print("seed", seed, "device", st[0], it[0], "oracle", r["status"], r["iters"])
    print("device stats\n", dstats[:max(it[0], r["iters"]) + 1])
    print("oracle stats\n", r["stats"][:max(it[0], r["iters"]) + 1])
    print("u dev", u[0])
    print("u ora", r["u"])
