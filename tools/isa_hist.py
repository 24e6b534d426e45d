"""Instruction histogram of one kernel in a hipcc -S listing.
usage: python tools/isa_hist.py build/isa/cse_evaluator.s <symbol-substring>"""
import collections
import re
import sys

path, pat = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = None
for i, l in enumerate(lines):
    if re.match(r"^_Z\S*:", l) and pat in l.split(":")[0]:
        start = i
        break
assert start is not None, "symbol not found"
body = []
for l in lines[start + 1:]:
    if l.startswith("\t.section") or re.match(r"^\.Lfunc_end", l):
        break
    body.append(l)
ops = [l.split()[0] for l in body if l.startswith("\t") and not l.strip().startswith((".", ";"))]
c = collections.Counter(ops)
cls = collections.Counter()
for op, n in c.items():
    k = ("v_fp64" if op.startswith("v_") and ("f64" in op) else
         "valu_other" if op.startswith("v_") else
         "salu" if op.startswith("s_") else
         "lds" if op.startswith("ds_") else
         "vmem" if op.startswith(("global_", "buffer_", "flat_")) else "other")
    cls[k] += n
print(lines[start].split(":")[0])
print("total", sum(c.values()), dict(cls))
for op, n in c.most_common(40):
    print(f"{n:6d} {op}")
