#!/usr/bin/env python3
"""Summarise the rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools_gpu_round.sh) into per-launch HBM bytes.

Corrections follow /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section):
  * FETCH_SIZE and WRITE_SIZE are reported in KiB per dispatch;
  * on gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced streaming read (16 B/lane) -> x2.
    The IPM and condensing kernels read H / inputs as 16-B-per-lane coalesced rows, so the x2 applies to them;
  * WRITE_SIZE is exact for 16-B-per-lane streaming stores.
The two counters come from separate passes (they cannot share one: FETCH_SIZE uses 3 TCC counters, WRITE_SIZE 2).

  python pmc_traffic.py <gpurun_out dir> <out.json> [bench args]
bench.py reads the JSON back (roofline.traffic) for the dominant kernel.
"""
import collections
import csv
import json
import os
import sys


def per_kernel(path):
    d = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            d[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in d.items()}


def main():
    src, out = sys.argv[1], sys.argv[2]
    fetch = per_kernel(os.path.join(src, "pmc_FETCH_SIZE", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(src, "pmc_WRITE_SIZE", "run_counter_collection.csv"))
    res = {}
    for k in sorted(set(fetch) | set(write)):
        fb = fetch.get(k, 0.0) * 1024.0 * 2.0  # KiB -> B, gfx950 half-count correction for wide streaming reads
        wb = write.get(k, 0.0) * 1024.0
        res[k] = {"fetch_bytes": fb, "write_bytes": wb, "hbm_bytes": fb + wb}
    lib = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lib", "libcmpc.so")
    import hashlib
    with open(lib, "rb") as f:
        md5 = hashlib.md5(f.read()).hexdigest()  # bench.py reports the traffic only for this exact build
    with open(out, "w") as f:
        json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), per-launch mean; "
                             "FETCH_SIZE x2 (gfx950 wide-read correction)", "lib_md5": md5,
                   "bench_args": sys.argv[3] if len(sys.argv) > 3 else "", "kernels": res}, f, indent=1)
    for k, v in res.items():
        print(f"{v['hbm_bytes'] / 1e6:12.2f} MB  {k}")


if __name__ == "__main__":
    main()
