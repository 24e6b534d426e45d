#!/usr/bin/env python3
"""Probe: one evaluation captured in a HIP graph (torch.cuda.CUDAGraph over
the launches libcse queues on the evaluator's stream) and replayed, against
the same evaluation issued call by call -- how much of a small evaluation's
time is host launch overhead and inter-kernel gaps.

    python tools/graph_probe.py [--steps 400]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ceres-solver-cuda_amd"))

import torch  # noqa: E402,F401  (first: libcse then shares torch's HIP runtime)

import ceres_amd as ca  # noqa: E402
from ceres_amd import bal, shard  # noqa: E402


def case(label, prog, steps, same_point):
    import torch
    dev = torch.device("cuda", 0)
    f64 = torch.float64
    torch.zeros(1, device=dev)  # initialise the runtime on the device first
    print("devices", torch.cuda.device_count(), [l.split()[-1] for l in open("/proc/self/maps")
                                                 if "amdhip64" in l][:1], flush=True)
    s = torch.cuda.Stream(dev)
    ev = ca.Evaluator(prog, device=0, profile=False, stream=s.cuda_stream)
    state = torch.from_numpy(prog.state).to(dev)
    cost = torch.zeros(1, dtype=f64, device=dev)
    r = torch.empty(prog.num_residuals, dtype=f64, device=dev)
    j = torch.empty(prog.num_jacobian_values, dtype=f64, device=dev)
    args = (state.data_ptr(), cost.data_ptr(), r.data_ptr(), None, j.data_ptr())
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        for _ in range(10):
            ev.evaluate_device(*args)
    assert ev.wait() == 0
    c_direct = float(cost.item())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        ev.evaluate_device(*args, new_evaluation_point=not same_point)
    torch.cuda.synchronize()
    for rnd in range(3):
        with torch.cuda.stream(s):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                ev.evaluate_device(*args, new_evaluation_point=not same_point)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            for _ in range(steps):
                g.replay()
            t3 = time.perf_counter()
            torch.cuda.synchronize()
            t4 = time.perf_counter()
        assert ev.wait() == 0
        print(f"{label:34s} round {rnd}: direct issue {(t1 - t0) / steps * 1e6:6.2f} wall "
              f"{(t2 - t0) / steps * 1e6:7.2f} us | graph issue {(t3 - t2) / steps * 1e6:6.2f} wall "
              f"{(t4 - t2) / steps * 1e6:7.2f} us | cost equal {float(cost.item()) == c_direct}",
              flush=True)
    ev.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    args = ap.parse_args()
    p16 = bal.program(*bal.synthetic(*bal.CONFIGS["problem-16-22106"]), loss=None)
    arrays = bal.synthetic(*bal.CONFIGS["problem-13682-4456117"])
    s8, _ = shard.shard_program(*arrays, 0, 8, loss=ca.Loss.huber(1.0))
    del arrays
    for sp in (False, True):
        case(f"problem-16 trivial BSM same={int(sp)}", p16, args.steps, sp)
        case(f"13682 shard 0/8 Huber same={int(sp)}", s8, max(args.steps // 4, 20), sp)


if __name__ == "__main__":
    main()
