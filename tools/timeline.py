#!/usr/bin/env python3
"""Summarise a per-wave timeline written by libcse ($CSE_TIMELINE with
CSE_AFFINE_VARIANT=47): 8 u64 per wave =
  [0] real-time clock at entry (100 MHz)   [1] shader clock at entry
  [2] shader clock when the gather landed  [3] after the functor + loss
  [4] staging reads landed (first store)   [5] after the last store issued
  [6] real-time clock at exit              [7] XCC_ID << 32 | HW_ID
"""
import sys

import numpy as np

t = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8).astype(np.int64)
t = t[t[:, 1] != 0]
n = len(t)
d_gather = t[:, 2] - t[:, 1]
d_compute = t[:, 3] - t[:, 2]
d_stage = t[:, 4] - t[:, 3]
d_store = t[:, 5] - t[:, 4]
d_total = t[:, 5] - t[:, 1]
real = (t[:, 6] - t[:, 0]) * 10.0  # ns
print(f"waves {n}")
for name, d in [("gather (cycles)", d_gather), ("compute", d_compute), ("staging", d_stage),
                ("store issue", d_store), ("wave total", d_total)]:
    q = np.percentile(d, [5, 50, 95])
    print(f"{name:16s} mean {d.mean():9.0f}  p5 {q[0]:9.0f}  p50 {q[1]:9.0f}  p95 {q[2]:9.0f}")
print(f"wave lifetime (real, ns) mean {real.mean():.0f} p50 {np.median(real):.0f} p95 {np.percentile(real, 95):.0f}")
t0, t1 = t[:, 0].min(), t[:, 6].max()
print(f"kernel span (real) {(t1 - t0) * 10 / 1e3:.1f} us")
# concurrency: waves alive at each 1 us bin
bins = np.arange(t0, t1 + 100, 100)
alive = np.zeros(len(bins))
starts = np.searchsorted(bins, t[:, 0])
ends = np.searchsorted(bins, t[:, 6])
np.add.at(alive, starts, 1)
np.add.at(alive, ends, -1)
alive = np.cumsum(alive)
print(f"waves alive: mean {alive[:-1].mean():.0f} max {alive.max():.0f} (chip holds 256 CUs x waves/CU)")
xcc = t[:, 7] >> 32
print("waves per XCC:", np.bincount(xcc.astype(np.int64), minlength=8))
