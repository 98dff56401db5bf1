"""Lab (GPU): per-phase cycles of k_ric from the stamps build (lab/build_ric_stamps.sh), CMPC_LIB pointing at it.
Prints the mean cycles per QP of setup / gradient / factorisations / solves / rest / total and per iteration."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CMPC_LIB", os.path.join(ROOT, "lab", "build", "libcmpc_ricst.so"))
sys.path.insert(0, os.path.join(ROOT, "cheeta-mpc_amd", "python"))
import cheeta_mpc as cm  # noqa: E402


def run(N, gait, prec, B=4096, allst=False, reps=3):
    m = cm.default_model(N)
    s = cm.default_settings() if prec == 0 else cm.default_settings(tol_stat=1e-3, tol_ineq=1e-3, tol_comp=1e-4)
    eng = cm.Engine(m, settings=s, precision=prec, max_batch=B, path={cm.PATH_RICCATI: 2})
    eng.enable_stats(1)
    x0, xref, foot, contact = cm.generate_device(m, 20221125, B, gait=gait)
    if allst:
        contact.upload(np.ones((B, N, 4), np.uint8))
    u = cm.DeviceArray((B, N, 4, 3), np.float64)
    st = cm.DeviceArray((B,), np.int32)
    it = cm.DeviceArray((B,), np.int32)
    for _ in range(reps):
        eng.solve_device(B, x0, xref, foot, contact, u, None, st, it)
    cm.hip().hipDeviceSynchronize()
    S = eng.stats(B)[:, 0, :7]
    names = ["setup", "grad", "factor", "solve", "rest", "total"]
    iters = S[:, 6]
    out = {n: float(S[:, i].mean()) for i, n in enumerate(names)}
    out["per_iter"] = {n: float((S[:, i] / np.maximum(iters, 1)).mean()) for i, n in enumerate(names) if i >= 2}
    out["iters"] = float(iters.mean())
    print(f"N={N} gait={gait} prec={prec} allstance={allst}:", {k: (round(v) if isinstance(v, float) else
                                                                    {a: round(b) for a, b in v.items()})
                                                               for k, v in out.items()}, flush=True)


if __name__ == "__main__":
    run(10, 0, 0)
    run(10, 0, 0, allst=True)
    run(20, 0, 1)
    run(10, 0, 0, B=512)
