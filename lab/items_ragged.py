"""Lab: the ragged N = 20 batch of tests/test_gpu_parity.py with and without the work-item kernel, per-QP diff."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cheeta-mpc_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import cheeta_mpc as cm
import oracle_py as op
from test_gpu_parity import _ragged_contacts
N, B = 20, 48
m, mo = cm.default_model(N), op.default_model(N)
rng = np.random.default_rng(7)
x0, xref, foot, contact = op.generate(mo, 20221125, B, gait=0)
contact[:] = _ragged_contacts(rng, B, N, np.linspace(0.2, 1.0, B))
nvar = 3 * contact.reshape(B, -1).sum(axis=1)
res = {}
for flag in ("1", "0"):
    os.environ["CMPC_ITEMS"] = flag
    eng = cm.Engine(m, precision=0, max_batch=B)
    res[flag] = eng.solve(x0, xref, foot, contact)
u1, _, s1, i1 = res["1"]
u0, _, s0, i0 = res["0"]
for q in range(B):
    d = float(np.max(np.abs(u1[q] - u0[q])))
    if d > 0 or s1[q] != s0[q] or i1[q] != i0[q]:
        print(q, "n", nvar[q], "st", s1[q], s0[q], "it", i1[q], i0[q], "maxdiff", d, "max|u1|", float(np.abs(u1[q]).max()),
              "max|u0|", float(np.abs(u0[q]).max()))
print("done")
