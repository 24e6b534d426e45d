#!/usr/bin/env python3
"""Per-kernel fingerprints of the product's device code (tools only).

Compiles each product TU (ceres-solver-cuda_amd/csrc/*.hip) to gfx950
assembly with the product flags (no -DCSE_TUNING), splits the assembly per
function, strips label names and comments, and prints one line per kernel:
<sha1 of the normalised body> <instruction count> <demangled name>.

Used to check that a refactor of csrc/ (removing A/B switches, moving launch
code) leaves the shipped kernels' machine code unchanged:
    python tools/isa_fingerprint.py > before.txt   # on the old tree
    python tools/isa_fingerprint.py > after.txt
    diff before.txt after.txt
"""
import hashlib
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "ceres-solver-cuda_amd")
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-fno-signed-zeros", "-ffinite-math-only",
         "-munsafe-fp-atomics", "-w", "--cuda-device-only", "-S"]


def functions(asm):
    cur, body = None, []
    for line in asm.splitlines():
        m = re.match(r"^([A-Za-z_.$][\w.$]*):", line)
        if m and not m.group(1).startswith(".L") and cur is None:
            cur, body = m.group(1), []
            continue
        if cur is not None:
            if line.startswith(".Lfunc_end"):
                yield cur, body
                cur = None
                continue
            s = line.split(";")[0].strip()
            if not s or s.startswith("."):
                continue
            s = re.sub(r"\.LBB\d+_\d+", "L", s)
            body.append(s)


def main():
    srcs = sys.argv[1:] or ["csrc/cse_evaluator.hip", "csrc/jet_kernels.hip", "csrc/multi_device.hip"]
    names = []
    with tempfile.TemporaryDirectory() as td:
        outs = [os.path.join(td, "k%d.s" % i) for i in range(len(srcs))]
        procs = [subprocess.Popen(["/opt/rocm/bin/hipcc"] + FLAGS + ["-o", o, os.path.join(PKG, s)],
                                  cwd=PKG) for s, o in zip(srcs, outs)]
        if any(p.wait() for p in procs):
            sys.exit("compile failed")
        asm = "\n".join(open(o).read() for o in outs)
    if True:
        for name, body in functions(asm):
            h = hashlib.sha1("\n".join(body).encode()).hexdigest()[:16]
            names.append((name, h, len(body)))
    mangled = [n for n, _, _ in names]
    dem = subprocess.run(["c++filt"], input="\n".join(mangled),
                         capture_output=True, text=True).stdout.splitlines()
    for (n, h, c), d in sorted(zip(names, dem), key=lambda t: t[1]):
        print(h, c, d)


if __name__ == "__main__":
    main()
