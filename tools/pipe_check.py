#!/usr/bin/env python3
"""Equality of tuning variants against the shipped kernel (variant 0)
on problems of assorted shapes: ragged block counts (n mod 64 != 0), block
counts that put the F cells off a 64-byte sector (n mod 4 != 0), fewer
chunks than workgroups, and a mid-size problem.  Tuning build only.

  python tools/pipe_check.py --variants 40,41,42
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ceres-solver-cuda_amd"))

import numpy as np  # noqa: E402

from ceres_amd import _cse  # noqa: E402

_cse.use_library(os.path.join(REPO, "ceres-solver-cuda_amd", "lib", "libcse_tuning.so"))

import ceres_amd as ca  # noqa: E402
from ceres_amd import bal  # noqa: E402


def run(prog, variant):
    os.environ["CSE_TUNE_VARIANT"] = str(variant)
    ev = ca.Evaluator(prog, device=0)
    out = [ev.evaluate(residuals=True, gradient=False, jacobian=True) for _ in range(2)]
    ev.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="40")
    args = ap.parse_args()
    shapes = [(5, 300, 1000), (7, 2000, 7603), (16, 22106, 83718), (40, 30000, 150001),
              (120, 200000, 1000002), (1000, 600000, 3000005)]
    losses = {"huber": ca.Loss.huber(1.0), "trivial": ca.Loss.trivial()}
    bad = 0
    for C, P, O in shapes:
        for lname, loss in losses.items():
            prog = bal.synthetic_program((C, P, O), loss=loss, seed=O)
            ref = run(prog, 0)[0]
            for v in args.variants.split(","):
                outs = run(prog, int(v))
                for k, got in enumerate(outs):
                    # Cost and residuals bit-equal; Jacobian values within a few
                    # ulps (the kernels contract FMAs differently).
                    jd = np.abs(got[4] - ref[4])
                    jok = bool(np.all(jd <= 1e-14 * np.abs(ref[4]) + 1e-15 * np.abs(ref[4]).max()))
                    same = (got[0] == ref[0] and got[1] == ref[1]
                            and np.array_equal(got[2], ref[2]) and jok)
                    if k == 0:
                        print(f"  jacobian: {int((jd > 0).sum())} of {jd.size} values differ, max "
                              f"rel {float((jd / np.maximum(np.abs(ref[4]), 1e-300)).max()):.2e}")
                    if not same:
                        bad += 1
                        d = np.abs(got[4] - ref[4])
                        print(f"MISMATCH {C},{P},{O} {lname} variant {v} call {k}: cost "
                              f"{got[1]!r} vs {ref[1]!r}; residual diff "
                              f"{np.abs(got[2] - ref[2]).max()}; jac diff {d.max()} at "
                              f"{int(np.argmax(d))} of {d.size}", flush=True)
                print(f"{C},{P},{O} {lname} variant {v}: "
                      f"{'identical' if bad == 0 else 'checked'}", flush=True)
    print("ALL IDENTICAL" if bad == 0 else f"{bad} MISMATCHES")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
