#!/usr/bin/env python3
"""Output digests of the BSM residual+Jacobian evaluation over a set of edge
cases, for a bit-equality check of two builds of libcse.so (round 4: the
persistent software-pipelined kernel, CSE_PERSISTENT=1, against the
one-chunk-per-wave kernel).

  python tools/pers_check.py --lib lib/pers/libcse.so --out a.json
  python tools/pers_check.py --compare a.json b.json

Cases: fewer residuals than one wave, one chunk per wave (problem-16), a
little more than one chunk per wave, many chunks per wave (problem-1778),
a ragged last chunk, odd chunk counts per wave, three losses, and states
with non-finite values (the kernel's slow path).  NaN payloads are
canonicalised before hashing."""
import argparse
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ceres-solver-cuda_amd"))

import numpy as np  # noqa: E402


def cases():
    return [
        ("tiny", (8, 10, 50), "huber", False),
        ("p16", (16, 22106, 83718), "trivial", False),
        ("p16h", (16, 22106, 83718), "huber", False),
        ("ragged", (40, 70001, 64 * 3001 + 37), "cauchy", False),
        ("two", (60, 150000, 64 * 2048 * 2 + 64 * 5 + 1), "huber", False),
        ("p1778", (1778, 993923, 5001946), "huber", False),
        ("nan", (40, 70001, 64 * 3001 + 37), "huber", True),
    ]


def digest(a):
    a = np.asarray(a, np.float64).copy()
    a[np.isnan(a)] = np.nan
    return hashlib.sha1(a.view(np.uint64).tobytes()).hexdigest()


def run(args):
    from ceres_amd import _cse
    _cse.use_library(os.path.abspath(args.lib))
    import torch
    import ceres_amd as ca
    from ceres_amd import bal
    losses = {"trivial": ca.Loss.trivial(), "huber": ca.Loss.huber(1.0), "cauchy": ca.Loss.cauchy(1.0)}
    out = {}
    dev = torch.device("cuda", 0)
    for name, counts, loss, nan in cases():
        prog = bal.synthetic_program(counts, loss=losses[loss])
        st = prog.state.copy()
        if nan:
            st[3 * 17 + 1] = np.nan
            st[3 * 4001] = np.inf
            st[-9 * 3 + 2] = np.nan  # a camera: every residual of it
        f64 = torch.float64
        state = torch.from_numpy(st).to(dev)
        cost = torch.zeros(1, dtype=f64, device=dev)
        res = torch.empty(prog.num_residuals, dtype=f64, device=dev)
        jac = torch.empty(prog.num_jacobian_values, dtype=f64, device=dev)
        jac.fill_(7.0)
        ev = ca.Evaluator(prog, device=0)
        ev.evaluate_device(state.data_ptr(), cost.data_ptr(), res.data_ptr(), None, jac.data_ptr())
        rc = ev.wait()  # non-zero for a non-finite cost (the nan case)
        torch.cuda.synchronize()
        out[name] = {"rc": int(rc), "res": digest(res.cpu().numpy()), "jac": digest(jac.cpu().numpy()),
                     "cost": digest(cost.cpu().numpy()), "n": int(prog.num_residuals // 2)}
        print(name, out[name], flush=True)
        ev.close()
        del state, res, jac, cost
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib")
    ap.add_argument("--out")
    ap.add_argument("--compare", nargs=2)
    args = ap.parse_args()
    if args.compare:
        a, b = (json.load(open(p)) for p in args.compare)
        bad = [k for k in a if a[k] != b.get(k)]
        print("identical" if not bad else f"DIFFER: {bad}")
        sys.exit(1 if bad else 0)
    run(args)


if __name__ == "__main__":
    main()
