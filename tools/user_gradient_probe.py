#!/usr/bin/env python3
"""Residual + Jacobian + gradient evaluations of a user functor kind against
the library kind of the same functor, on one problem-13682-shaped Program.

The library's SnavelyKind takes the fused gradient (points in the
evaluation, camera rows re-evaluated in camera order: gradient_mode 0).  A
user kind took the gradient post-passes over the written Jacobian until
ABI 5 (profiles/round6/r6v: 4.21 ms against 1.97); since, it takes the same
fused form through its own TU's launches (r6w).  Times
both (device-resident, HIP-event-free wall time over --steps evaluations)
with and without the gradient, and checks the gradients agree to 1e-13.

  python tools/user_gradient_probe.py
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ceres-solver-cuda_amd"))
import ceres_amd as ca  # noqa: E402
from ceres_amd import _cse, bal  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="problem-13682-4456117")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    lib = _cse.load_functor_library(os.path.join(REPO, "examples", "build", "libuser_functors.so"))
    lib.cse_example_kind_name.restype = C.c_char_p
    kinds = (C.c_int32 * 64)()
    n = lib.cse_example_register(kinds, 64)
    kind = {lib.cse_example_kind_name(i).decode(): kinds[i] for i in range(n)}[
        "SnavelyReprojectionError/Huber"]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    prog = bal.synthetic_program(args.config, loss=ca.Loss.huber(1.0))
    import copy
    import dataclasses
    uprog = copy.copy(prog)
    uprog.groups = [dataclasses.replace(g, kind=kind) for g in prog.groups]
    f64 = torch.float64
    state = torch.from_numpy(prog.state).to(dev)
    bufs = (torch.zeros(1, dtype=f64, device=dev), torch.empty(prog.num_residuals, dtype=f64, device=dev),
            torch.empty(prog.num_effective_parameters, dtype=f64, device=dev),
            torch.empty(prog.num_jacobian_values, dtype=f64, device=dev))
    evs = {"library": ca.Evaluator(prog, stream=stream.cuda_stream),
           "user": ca.Evaluator(uprog, stream=stream.cuda_stream)}
    out = {name: {} for name in evs}
    grads = {}
    for rnd in range(args.rounds):
        for name, ev in evs.items():
            for grad in (False, True):
                c, r, g, j = bufs
                gp = g.data_ptr() if grad else None
                for _ in range(5):
                    ev.evaluate_device(state.data_ptr(), c.data_ptr(), r.data_ptr(), gp, j.data_ptr())
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    ev.evaluate_device(state.data_ptr(), c.data_ptr(), r.data_ptr(), gp, j.data_ptr())
                torch.cuda.synchronize(dev)
                assert ev.wait() == 0
                ms = (time.perf_counter() - t0) / args.steps * 1e3
                out[name].setdefault("gradient" if grad else "no_gradient", []).append(round(ms, 4))
                if grad:
                    grads[name] = g.cpu().numpy().copy()
    for ev in evs.values():
        ev.close()
    a, b = grads["user"], grads["library"]
    out["gradient_rel_diff"] = float(np.linalg.norm(a - b) / np.linalg.norm(b))
    out["config"] = args.config
    print(json.dumps(out), flush=True)
    assert out["gradient_rel_diff"] <= 1e-13


if __name__ == "__main__":
    main()
