#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output for the evaluate kernel.

usage: pmc_summary.py <rocprof output dir> [kernel substring] [--json out.json]

Reads every *counter_collection.csv / *kernel_stats.csv / *kernel_trace.csv
under the directory and prints per-dispatch averages of each counter for
dispatches whose kernel name contains the substring (default
EvaluateGroupKernel).  HBM bytes follow MI355X_MICROARCH.md §HBM:
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the
bytes of a wide coalesced read, so the read side is doubled (the
correction the guide prescribes); WRITE_SIZE is exact for 16-B stores.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "EvaluateGroupKernel"
    out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    per = defaultdict(lambda: defaultdict(float))
    durations = []
    names = set()
    for f in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True):
        with open(f) as fh:
            rows = list(csv.DictReader(fh))
        if not rows:
            continue
        if "Counter_Name" in rows[0]:
            for r in rows:
                if sub in r.get("Kernel_Name", ""):
                    names.add(r["Kernel_Name"])
                    per[r["Counter_Name"]][r.get("Dispatch_Id") or r.get("Correlation_Id")] += float(r["Counter_Value"])
        elif "Start_Timestamp" in rows[0] and "Kernel_Name" in rows[0]:
            for r in rows:
                if sub in r["Kernel_Name"]:
                    names.add(r["Kernel_Name"])
                    durations.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    res = {"kernels": sorted(names)}
    if durations:
        res["dispatches"] = len(durations)
        res["avg_ms"] = sum(durations) / len(durations)
    for c, vals in sorted(per.items()):
        v = list(vals.values())
        res[c] = sum(v) / len(v)
    if "FETCH_SIZE" in res:
        res["hbm_read_bytes_per_launch"] = 2 * res["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in res:
        res["hbm_write_bytes_per_launch"] = res["WRITE_SIZE"] * 1024
    if "FETCH_SIZE" in res and "WRITE_SIZE" in res:
        res["hbm_bytes_per_launch"] = res["hbm_read_bytes_per_launch"] + res["hbm_write_bytes_per_launch"]
    print(json.dumps(res, indent=1))
    if out_json:
        old = {}
        if os.path.exists(out_json):
            with open(out_json) as fh:
                old = json.load(fh)
        old.update({k: v for k, v in res.items() if k != "kernels"})
        old.setdefault("kernels", res["kernels"])
        with open(out_json, "w") as fh:
            json.dump(old, fh, indent=1)


if __name__ == "__main__":
    main()
