"""Lab (GPU): per-QP comparison of the stage-wise path modes against the oracle (debugging aid)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cheeta-mpc_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import cheeta_mpc as cm  # noqa: E402
import oracle_py as op  # noqa: E402

N, B, gait = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
mo = op.default_model(N)
x0, xref, foot, ct = op.generate(mo, 20221125, B, gait=gait)
n = ct.reshape(B, -1).sum(1) * 3
ur, _, sr, itr = op.solve_batch(mo, op.default_settings(), x0, xref, foot, ct, nthreads=8, want_x=False)
for ric in (1, 2):
    eng = cm.Engine(cm.default_model(N), precision=0, max_batch=B, path={cm.PATH_RICCATI: ric})
    for rep in range(2):
        u, _, st, it = eng.solve(x0, xref, foot, ct, want_x=False)
        err = np.abs(u - ur).reshape(B, -1).max(1) / np.maximum(1.0, np.abs(ur).reshape(B, -1).max(1))
        bad = np.nonzero((st != sr) | (err > 1e-8))[0]
        print(f"ric={ric} rep={rep}: bad {len(bad)}:", [(int(q), int(n[q]), int(st[q]), int(it[q]), int(itr[q]),
                                                        float(f"{err[q]:.2e}")) for q in bad[:8]], flush=True)
# the n = 240 QPs alone through mode 2
sel = np.nonzero(n == n.max())[0]
eng = cm.Engine(cm.default_model(N), precision=0, max_batch=len(sel), path={cm.PATH_RICCATI: 2})
u, _, st, it = eng.solve(x0[sel], xref[sel], foot[sel], ct[sel], want_x=False)
err = np.abs(u - ur[sel]).reshape(len(sel), -1).max(1) / np.maximum(1.0, np.abs(ur[sel]).reshape(len(sel), -1).max(1))
print("mode2 largest only: bad", int(((st != sr[sel]) | (err > 1e-8)).sum()), "of", len(sel))
