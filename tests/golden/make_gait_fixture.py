#!/usr/bin/env python3
"""Writes tests/golden/gait_templates.json: the gait templates of the reference's
ocs2_legged_robot/config/command/gait.info (modeSequence + switchingTimes per gait, in the file's list order),
parsed from the boost-info text. Run in the build container (the reference is not on the GPU box); the JSON is the
fixture that pins cmpc_gait_builtin (tests/test_gait.py)."""
import json
import os
import re
import sys

SRC = "/root/reference/ocs2_legged_robot/config/command/gait.info"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gait_templates.json")


def parse(text):
    text = re.sub(r";[^\n]*", "", text)  # comments
    toks = re.findall(r"\{|\}|\[\d+\]|[^\s{}\[\]]+", text)
    pos = 0

    def block():
        nonlocal pos
        out, key = {}, None
        while pos < len(toks):
            t = toks[pos]
            pos += 1
            if t == "}":
                return out
            if t == "{":
                out[key] = block()
                key = None
            elif key is None:
                key = t
            else:
                out[key] = t
                key = None
        return out

    return block()


def main():
    d = parse(open(sys.argv[1] if len(sys.argv) > 1 else SRC).read())
    names = [d["list"][k] for k in sorted(d["list"], key=lambda s: int(s[1:-1]))]
    gaits = []
    for n in names:
        g = d[n]
        ms = [g["modeSequence"][k] for k in sorted(g["modeSequence"], key=lambda s: int(s[1:-1]))]
        st = [float(g["switchingTimes"][k]) for k in sorted(g["switchingTimes"], key=lambda s: int(s[1:-1]))]
        gaits.append({"name": n, "modeSequence": ms, "switchingTimes": st})
    with open(OUT, "w") as f:
        json.dump({"source": "ocs2_legged_robot/config/command/gait.info", "gaits": gaits}, f, indent=1)
    print(f"wrote {OUT}: {len(gaits)} gaits")


if __name__ == "__main__":
    main()
