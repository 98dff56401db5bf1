"""Lab (GPU): per-phase cycles of k_sqp_step and of the two-wave foothold condensing over one batched NLP solve
(trot N = 10, B = 4096), from the stamps build (lab/sqp_stamps.sh), CMPC_LIB=lab/_stamps/libcmpc_nlpstamps.so."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cheeta-mpc_amd", "python"))
import cheeta_mpc as cm  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
L = cm.lib()
SQ = ["staging", "own pass", "wait for the other wave", "-", "-", "selection + update", "next lin point"]
fns = {"k_sqp_step wave 0 (rollouts)": (L.cmpc_sqp_debug_stamps, SQ),
       "k_sqp_step wave 1 (lin. response, |du|)": (L.cmpc_sqp_debug_stamps, SQ),
       "condense80 (wave 0)": (L.cmpc_cond_debug_stamps, ["record + ballots", "per-step tables", "column setup",
                                                           "gamma update", "free response (t0)", "block row + barrier",
                                                           "g + MFMA", "epilogue"])}
for f, _ in fns.values():
    f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
m = cm.default_model(10)
eng = cm.Engine(m, precision=cm.F64, max_batch=B)
x0, xref, foot, contact = (a.host() for a in cm.generate_device(m, 20221125, B, gait=0))
eng.nlp_solve(x0, xref, foot, contact)
buf = (C.c_ulonglong * 16)()
for f, _ in fns.values():
    f(buf, 1)
eng.nlp_solve(x0, xref, foot, contact)
sq = (C.c_ulonglong * 16)()
L.cmpc_sqp_debug_stamps(sq, 1)
cd = (C.c_ulonglong * 16)()
L.cmpc_cond_debug_stamps(cd, 1)
for name, (f, names) in fns.items():
    src, off, cnt = (cd, 0, cd[15]) if f is L.cmpc_cond_debug_stamps else (sq, 8 if "wave 1" in name else 0, sq[15] // 2)
    n = max(cnt, 1)
    tot = sum(src[off + k] for k in range(len(names)))
    print(f"{name}: {cnt} QPs, {tot / n:.0f} cycles each")
    for k, nm in enumerate(names):
        print(f"  {nm:26s} {src[off + k] / n:9.0f}  {100.0 * src[off + k] / max(tot, 1):5.1f} %")
