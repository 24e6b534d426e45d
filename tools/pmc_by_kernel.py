#!/usr/bin/env python3
"""Per-kernel-name average of every counter in rocprofv3 CSV output dirs.
usage: pmc_by_kernel.py <dir> [<dir> ...]"""
import csv, glob, os, sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[r["Kernel_Name"]][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for k in sorted(vals):
    short = k.split("(")[0][:60]
    items = ", ".join(f"{c}={sum(v.values())/len(v):.4g}" for c, v in sorted(vals[k].items()))
    print(f"{short}: {items}")
