#!/usr/bin/env python3
"""Diagnostic: does the hot kernel's time depend on the data it reads?

Builds the bench workload (problem-13682 shape, Huber, BSM), then times the
evaluator (HIP events, kernel_stats) with
  * the real synthetic inputs,
  * the camera ids replaced by a hash pattern (tools/membench's),
  * the state and observations zeroed,
so the differences isolate data/access-pattern effects from kernel shape.
Run on the GPU box: python tools/data_probe.py [variant ...]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ceres-solver-cuda_amd"))

import ceres_amd as ca  # noqa: E402
from ceres_amd import bal  # noqa: E402


def time_prog(prog, steps=20, layout="separate"):
    import torch
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    ev = ca.Evaluator(prog, device=0, profile=True, stream=stream.cuda_stream, check_finite=False)
    state = torch.from_numpy(prog.state).to(dev)
    cost = torch.zeros(1, dtype=torch.float64, device=dev)
    nr, nj = prog.num_residuals, prog.num_jacobian_values
    if layout == "one-buffer":
        buf = torch.empty(nr + nj + 64, dtype=torch.float64, device=dev)
        res, jac = buf[:nr], buf[nr + (-nr) % 16:][:nj]
    elif layout == "jac-first":
        jac = torch.empty(nj, dtype=torch.float64, device=dev)
        res = torch.empty(nr, dtype=torch.float64, device=dev)
    else:
        res = torch.empty(nr, dtype=torch.float64, device=dev)
        jac = torch.empty(nj, dtype=torch.float64, device=dev)
    for _ in range(3):
        ev.evaluate_device(state.data_ptr(), cost.data_ptr(), res.data_ptr(), None, jac.data_ptr())
    ev.wait()
    ev.reset_kernel_stats()
    for _ in range(steps):
        ev.evaluate_device(state.data_ptr(), cost.data_ptr(), res.data_ptr(), None, jac.data_ptr())
    ev.wait()
    _, total, n = ev.kernel_stats()
    ev.close()
    del state, res, jac
    torch.cuda.empty_cache()
    return total / n


def main():
    import torch
    torch.cuda.set_device(0)
    C, P, O = bal.CONFIGS["problem-13682-4456117"]
    cams, pts, ci, pi, obs = bal.synthetic(C, P, O)
    loss = ca.Loss.huber(1.0)
    i = np.arange(O, dtype=np.int64)
    h = ((i * 2654435761) & 0xFFFFFFFF) ^ (((i >> 7) * 40503) & 0xFFFFFFFF)
    hashed = (h % C).astype(ci.dtype)
    cases = [
        ("real", cams, pts, ci, obs),
        ("hashed camera ids", cams, pts, hashed, obs),
        ("zero state+obs", np.zeros_like(cams), np.zeros_like(pts), ci, np.zeros_like(obs)),
        ("sorted camera ids", cams, pts, np.sort(ci), obs),
    ]
    if os.environ.get("PROBE_LAYOUTS"):
        prog = bal.program(cams, pts, ci, pi, obs, loss=loss)
        for layout in ("separate", "one-buffer", "jac-first", "separate"):
            ms = time_prog(prog, layout=layout)
            print(f"{layout:24s} {ms:.4f} ms  {6.833e9 / ms / 1e6:.0f} GB/s", flush=True)
        return
    for name, c_, p_, ci_, o_ in cases:
        prog = bal.program(c_, p_, ci_, pi, o_, loss=loss)
        ms = time_prog(prog)
        print(f"{name:24s} {ms:.4f} ms  {6.833e9 / ms / 1e6:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
