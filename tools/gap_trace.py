#!/usr/bin/env python3
"""Per-kernel durations and the idle gaps between consecutive dispatches
from a rocprofv3 kernel trace (--kernel-trace --output-format csv).

usage: gap_trace.py <rocprof output dir> [--last N]

Considers the last N dispatches (default: all), sorted by start time; for
each kernel name prints count, mean duration (us) and the mean gap (us)
between the end of the previous dispatch and its start; and the sum of
busy and idle time.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 0
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    if last:
        rows = rows[-last:]
    stats = defaultdict(lambda: [0, 0.0, 0.0])
    busy = idle = 0.0
    prev_end = None
    for s, e, name in rows:
        short = name.split("(")[0][:90]
        st = stats[short]
        st[0] += 1
        st[1] += (e - s) / 1e3
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        st[2] += max(gap, 0.0)
        busy += (e - s) / 1e3
        idle += max(gap, 0.0)
        prev_end = max(prev_end or e, e)
    for k, (n, dur, gap) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:6d}  dur {dur / n:9.2f} us  gap before {gap / n:7.2f} us  {k}")
    span = (rows[-1][1] - rows[0][0]) / 1e3 if rows else 0
    print(f"dispatches {len(rows)}  span {span:.1f} us  busy {busy:.1f} us  idle {idle:.1f} us")


if __name__ == "__main__":
    main()
