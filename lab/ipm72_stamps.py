"""Lab (GPU): per-phase cycles of k_ipm72 over one batched NLP solve (trot N = 10, B = 4096), from the stamps build
(lab/ipm72_stamps.sh), CMPC_LIB=lab/_stamps/libcmpc_ipm72stamps.so."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cheeta-mpc_amd", "python"))
import cheeta_mpc as cm  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
gait = int(sys.argv[2]) if len(sys.argv) > 2 else 0
L = cm.lib()
L.cmpc_ipm72_debug_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
buf = (C.c_ulonglong * 16)()
m = cm.default_model(10)
eng = cm.Engine(m, precision=cm.F64, max_batch=B)
x0, xref, foot, contact = (a.host() for a in cm.generate_device(m, 20221125, B, gait=gait))
eng.nlp_solve(x0, xref, foot, contact)
L.cmpc_ipm72_debug_stamps(buf, 1)
for rep in range(2):
    eng.nlp_solve(x0, xref, foot, contact)
    L.cmpc_ipm72_debug_stamps(buf, 1)
    names = ["H+residuals", "Newton blocks", "LDL' K_AA", "Y = M K_AB", "S", "S^-1", "predictor", "corrector",
             "update"]
    its = buf[9]
    tot = buf[10]
    print(f"rep {rep}: {its} IPM iterations over the k_ipm72 waves, {tot / max(its, 1):.0f} cycles per iteration (wave)")
    for k, n in enumerate(names):
        print(f"  {n:14s} {buf[k] / max(its, 1):9.0f} cycles/iter  {100.0 * buf[k] / max(tot, 1):5.1f} %")
