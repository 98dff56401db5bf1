#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (tools_gpu_pmc.sh: <dir>/p1, p2, ...) into per-dispatch means per kernel, and
derive the utilisation figures DESIGN.md quotes. Units follow MI355X_MICROARCH.md: SQ_WAVE_CYCLES, SQ_BUSY_CYCLES,
SQ_WAIT_* and SQ_ACTIVE_INST_* count quad-cycles (x4 = shader cycles); SQ_VALU_MFMA_BUSY_CYCLES counts cycles;
SQ_INSTS_* are wave-instructions summed over the dispatch; GRBM_GUI_ACTIVE is summed over the 8 XCDs.

  python pmc_summary.py <dir> [--json out.json]     (out.json: {"lib_md5": ..., "kernels": {name: ...}})
"""
import collections
import csv
import glob
import json
import os
import sys

KEYS = ("k_solve64", "k_solve128", "k_ipm64", "k_ipm128x", "k_ipm_tiled", "k_condense64", "k_srbd_condense", "k_ocp")


def load(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for p in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        with open(p) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"]
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
                vals[k]["_duration_s"].append(dur)
                meta[k] = {"vgpr": int(r["VGPR_Count"]), "agpr": int(r["Accum_VGPR_Count"]),
                           "sgpr": int(r["SGPR_Count"]), "lds": int(r["LDS_Block_Size"]),
                           "scratch": int(r["Scratch_Size"]), "grid": int(r["Grid_Size"]),
                           "wg": int(r["Workgroup_Size"])}
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}, meta


def derive(c):
    out = {}
    g = c.get
    if g("SQ_WAVE_CYCLES") and g("SQ_ACTIVE_INST_VALU") is not None:
        out["valu_active_per_wave_cycle"] = g("SQ_ACTIVE_INST_VALU") / g("SQ_WAVE_CYCLES")
    if g("SQ_WAVE_CYCLES") and g("SQ_WAIT_INST_ANY") is not None:
        out["issue_stall_frac"] = g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES")
    if g("SQ_WAVE_CYCLES") and g("SQ_WAIT_ANY") is not None:
        out["waitcnt_frac"] = g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES")
    if g("SQ_BUSY_CYCLES") and g("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
        # MFMA busy: cycles, summed over the SIMDs; SQ_BUSY_CYCLES: quad-cycles of the SQ (per SE), so the ratio is
        # reported raw and interpreted in DESIGN.md
        out["mfma_busy_cycles"] = g("SQ_VALU_MFMA_BUSY_CYCLES")
    if g("GRBM_GUI_ACTIVE") and g("_duration_s"):
        out["clock_ghz"] = g("GRBM_GUI_ACTIVE") / 8.0 / g("_duration_s") / 1e9
    if g("SQ_INSTS_VALU") and g("SQ_WAVES"):
        out["valu_insts_per_wave"] = g("SQ_INSTS_VALU") / g("SQ_WAVES")
    return out


def main():
    d = sys.argv[1]
    vals, meta = load(d)
    res = {}
    for k, c in vals.items():
        if not any(s in k for s in KEYS):
            continue
        res[k] = {"counters": c, "derived": derive(c), "resources": meta.get(k, {})}
        print(k)
        print("  resources", meta.get(k, {}))
        for cn in sorted(c):
            print(f"  {cn:34s} {c[cn]:.6g}")
        for dn, dv in res[k]["derived"].items():
            print(f"  = {dn:32s} {dv:.4g}")
    if "--json" in sys.argv:
        # stamped with the libcmpc.so md5 of this tree, so bench.py reports the MFMA figures only for the build the
        # counters were taken on
        import hashlib
        lib = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lib", "libcmpc.so")
        with open(lib, "rb") as f:
            md5 = hashlib.md5(f.read()).hexdigest()
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump({"lib_md5": md5, "kernels": res}, f, indent=1)


if __name__ == "__main__":
    main()
