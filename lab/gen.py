#!/usr/bin/env python3
"""Generates variants.inc (driver table) and variants.mk (build rules) from variants.txt (lab harness only).
variants.txt: one variant per line: <name> <header> <wpe> <stamps 0|1> [extra -D flags...]"""
import os
here = os.path.dirname(os.path.abspath(__file__))
rows = []
for line in open(os.path.join(here, "variants.txt")):
    line = line.split("#", 1)[0].split()
    if line:
        rows.append(line)
with open(os.path.join(here, "variants.inc"), "w") as f:
    f.write("#ifdef LAB_VARIANTS_DECL\n")
    for r in rows:
        f.write(f'extern "C" int {r[0]}(const cmpc::IpmArgs<double>*, int, hipStream_t, unsigned long long*);\n')
        f.write(f'extern "C" int {r[0]}_prep(const cmpc::IpmArgs<double>*, int, hipStream_t, cmpc::IpmArgs<double>*);\n')
    f.write("#endif\n#ifdef LAB_VARIANTS_LIST\n")
    for r in rows:
        f.write(f'{{"{r[0]}", {r[0]}, {r[0]}_prep, {r[3]}}},\n')
    f.write("#endif\n")
with open(os.path.join(here, "variants.mk"), "w") as f:
    objs = " ".join(f"build/{r[0]}.o" for r in rows)
    f.write(f"OBJS = {objs}\n")
    for r in rows:
        st = "-DLAB_STAMPS" if r[3] == "1" else ""
        extra = " ".join(r[4:])
        st = {"1": "-DLAB_STAMPS -DCMPC_IPM_STAMPS", "2": "-DCMPC_IPM_TIMELINE"}.get(r[3], "")
        f.write(f"build/{r[0]}.o: ipm_variant.hip {r[1]} lab_stamps.hpp ../cheeta-mpc_amd/csrc/k_ipm64.hpp ../cheeta-mpc_amd/csrc/k_ipm128x.hpp\n\t@mkdir -p build\n"
                f"\t$(HIPCC) $(FLAGS) -DLAB_HDR={r[1]} -DLAB_FN={r[0]} -DLAB_WPE={r[2]} {st} {extra} -c $< -o $@\n")
