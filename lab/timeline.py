#!/usr/bin/env python3
"""Lab analysis of a timeline build (CMPC_IPM_TIMELINE): per-QP [start, end, HW_ID, XCC_ID] on the 100-MHz clock ->
kernel span, wave durations, waves per SIMD, concurrency over time. Usage: timeline.py <timeline_*.bin>"""
import sys
import numpy as np
a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 9)
t0, t1, hw, xcc = a[:, 0].astype(np.int64), a[:, 1].astype(np.int64), a[:, 2], a[:, 3]
ok = t0 > 0
t0, t1, hw, xcc = t0[ok], t1[ok], hw[ok], xcc[ok]
base = t0.min()
s, e = (t0 - base) * 1e-2, (t1 - base) * 1e-2  # us
dur = e - s
print(f"span {e.max():.1f} us; wave dur mean {dur.mean():.1f} min {dur.min():.1f} max {dur.max():.1f}; "
      f"ideal (sum dur / slots) {dur.sum() / 2048:.1f}")
slot = ((xcc * 8 + ((hw >> 13) & 7)) * 2 + ((hw >> 12) & 1)) * 64 + ((hw >> 8) & 15) * 4 + ((hw >> 4) & 3)
_, cnt = np.unique(slot, return_counts=True)
print("waves per SIMD", dict(enumerate(np.bincount(cnt))) )
print("end quantiles", np.round(np.percentile(e, [0, 10, 25, 50, 75, 90, 99, 100]), 1))
ts = np.linspace(0, e.max(), 30)
print("concurrency", [int(((s <= t) & (e > t)).sum()) for t in ts])
