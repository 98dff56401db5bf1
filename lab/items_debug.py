"""Lab: one small cmpc_solve_batch through the work-item kernel (k_solve64q), printing as it goes (debugging aid)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cheeta-mpc_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import cheeta_mpc as cm
import oracle_py as op
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
N = 10
print("start", B, flush=True)
m = cm.default_model(N)
eng = cm.Engine(m, precision=cm.F64, max_batch=B)
print("engine", cm.lib().cmpc_ctx_fused(eng.ctx), flush=True)
x0, xref, foot, contact = (a.host() for a in cm.generate_device(m, 20221125, B, gait=0))
t = time.time()
u, x, st, it = eng.solve(x0, xref, foot, contact, want_x=False)
print("solved in", time.time() - t, "status", np.bincount(st), "iters", np.bincount(it), flush=True)
ur, _, sr, itr = op.solve_batch(op.default_model(N), op.default_settings(), x0, xref, foot, contact, nthreads=4)
print("max rel du", float(np.max(np.abs(u - ur)) / max(1.0, float(np.max(np.abs(ur))))), "same iters", int((it == itr).sum()), flush=True)
