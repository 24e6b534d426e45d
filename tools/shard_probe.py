#!/usr/bin/env python3
"""Probe: rank 0's shard of an N-way cut, evaluated with output buffers at
different placements (exact-size torch allocations, oversized allocations,
shifted base addresses), to tell a size effect from an address effect.

    python tools/shard_probe.py --shards 2
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ceres-solver-cuda_amd"))

from ceres_amd import _cse  # noqa: E402

if "--lib" in sys.argv:  # another build of the same ABI (e.g. the previous commit's tuning lib)
    _cse.use_library(os.path.abspath(sys.argv[sys.argv.index("--lib") + 1]))

import ceres_amd as ca  # noqa: E402
from ceres_amd import bal, shard  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", type=int, default=2)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--fracs", default="", help="comma list: evaluate the first f*O blocks instead")
    ap.add_argument("--lib", default=None)
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    f64 = torch.float64
    counts = bal.CONFIGS["problem-13682-4456117"]
    arrays = bal.synthetic(*counts)
    if args.fracs:
        import numpy as np
        cams, pts, ci, pi, obs = arrays
        for f in [float(x) for x in args.fracs.split(",")]:
            S = int(len(ci) * f)
            last = int(pi[S - 1])
            S = int(np.searchsorted(pi, last, side="right"))
            prog = bal.program(cams, pts[:last + 1], ci[:S], pi[:S], obs[:S], loss=ca.Loss.huber(1.0))
            run(prog, {"exact": None}, f"frac {f:.3f} n={S}", args.steps, dev)
        return
    prog, sh = shard.shard_program(*arrays, 0, args.shards, loss=ca.Loss.huber(1.0))
    run(prog, None, f"shards {args.shards}", args.steps, dev)


def run(prog, only, label, steps, dev):
    import torch
    f64 = torch.float64
    stream = torch.cuda.current_stream(dev)
    ev = ca.Evaluator(prog, device=0, profile=True, stream=stream.cuda_stream)
    nbytes = ev.info().bytes_jacobian_eval
    state = torch.from_numpy(prog.state).to(dev)
    cost = torch.zeros(1, dtype=f64, device=dev)
    nr, nj = prog.num_residuals, prog.num_jacobian_values
    big_r = torch.empty(2 * nr + 4096, dtype=f64, device=dev)
    big_j = torch.empty(2 * nj + 4096, dtype=f64, device=dev)
    cases = {
        "exact": (torch.empty(nr, dtype=f64, device=dev), torch.empty(nj, dtype=f64, device=dev)),
        "oversized": (big_r[:nr], big_j[:nj]),
        "shift 1 MiB": (big_r[131072:131072 + nr], big_j[131072:131072 + nj]),
        "shift 64 MiB": (big_r[:nr], big_j[8 << 20:(8 << 20) + nj]),
        "shift half": (big_r[:nr], big_j[nj // 2:nj // 2 + nj]),
    }
    if only:
        cases = {k: v for k, v in cases.items() if k in only}
    for rnd in range(2):
        for name, (r, j) in cases.items():
            for _ in range(3):
                ev.evaluate_device(state.data_ptr(), cost.data_ptr(), r.data_ptr(), None, j.data_ptr())
            assert ev.wait() == 0
            ev.reset_kernel_stats()
            for _ in range(steps):
                ev.evaluate_device(state.data_ptr(), cost.data_ptr(), r.data_ptr(), None, j.data_ptr())
            assert ev.wait() == 0
            _, tot, n = ev.kernel_stats()
            ms = tot / n
            print(f"round {rnd} {label} {name:14s} jac@{j.data_ptr():#x} "
                  f"{ms:.4f} ms  frac {nbytes / ms / 1e6 / 8000:.3f}", flush=True)
    ev.close()


if __name__ == "__main__":
    main()
