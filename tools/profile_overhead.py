#!/usr/bin/env python3
"""Wall time per residual+Jacobian evaluation with and without the
evaluator's per-evaluation timing events (cse_options.profile), same
program, same buffers, interleaved rounds.

  python tools/profile_overhead.py --config problem-1778-993923 --format compressed_row
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ceres-solver-cuda_amd"))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="problem-13682-4456117")
    ap.add_argument("--format", default="block_sparse", choices=["block_sparse", "compressed_row"])
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    import torch
    import ceres_amd as ca
    from ceres_amd import bal
    prog = bal.synthetic_program(args.config, loss=ca.Loss.huber(1.0), format=args.format)
    dev = torch.device("cuda", 0)
    f64 = torch.float64
    stream = torch.cuda.current_stream(dev)
    state = torch.from_numpy(prog.state).to(dev)
    cost = torch.zeros(1, dtype=f64, device=dev)
    res = torch.empty(prog.num_residuals, dtype=f64, device=dev)
    jac = torch.empty(prog.num_jacobian_values, dtype=f64, device=dev)
    evs = {p: ca.Evaluator(prog, device=0, profile=p, stream=stream.cuda_stream) for p in (False, True)}
    out = {False: [], True: []}
    for _ in range(args.rounds):
        for p, ev in evs.items():
            for _ in range(3):
                ev.evaluate_device(state.data_ptr(), cost.data_ptr(), res.data_ptr(), None, jac.data_ptr())
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                ev.evaluate_device(state.data_ptr(), cost.data_ptr(), res.data_ptr(), None, jac.data_ptr())
            torch.cuda.synchronize()
            out[p].append((time.perf_counter() - t0) / args.steps * 1e3)
            assert ev.wait() == 0
    for p in (False, True):
        print(f"profile={p}: ms per evaluation {['%.4f' % v for v in out[p]]} median {np.median(out[p]):.4f}")


if __name__ == "__main__":
    main()
