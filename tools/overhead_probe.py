#!/usr/bin/env python3
"""Probe: the fixed per-evaluation cost of small evaluations (launch and host
overhead), for BASELINE configs[1] (problem-16, no loss, BSM) and rank 0's
shard of an 8-way cut of problem-13682 (Huber, BSM).

Per case: host time to issue N cse_evaluate_device calls (no synchronisation
in between), wall time per evaluation once the stream has drained, and the
evaluation kernels' time (HIP events, profile=True).

    python tools/overhead_probe.py [--steps 400] [--lib path/to/libcse.so]
"""
import argparse
import ctypes as C
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ceres-solver-cuda_amd"))

from ceres_amd import _cse  # noqa: E402

if "--lib" in sys.argv:
    _cse.use_library(os.path.abspath(sys.argv[sys.argv.index("--lib") + 1]))

import ceres_amd as ca  # noqa: E402
from ceres_amd import bal, shard  # noqa: E402


def case(label, prog, steps, dev, profile, flags=None):
    import torch
    f64 = torch.float64
    stream = torch.cuda.current_stream(dev)
    ev = ca.Evaluator(prog, device=0, profile=profile, stream=stream.cuda_stream)
    state = torch.from_numpy(prog.state).to(dev)
    cost = torch.zeros(1, dtype=f64, device=dev)
    r = torch.empty(prog.num_residuals, dtype=f64, device=dev)
    j = torch.empty(prog.num_jacobian_values, dtype=f64, device=dev)
    L = _cse.lib()
    h = ev.handle
    args = (state.data_ptr(), cost.data_ptr(), r.data_ptr(), None, j.data_ptr())
    fn = L.cse_evaluate_device
    use_ex = flags is not None and hasattr(L, "cse_evaluate_device_ex")
    for _ in range(20):
        fn(h, *args)
    assert ev.wait() == 0
    out = {}
    for rnd in range(3):
        ev.reset_kernel_stats()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        if use_ex:
            ex = L.cse_evaluate_device_ex
            for _ in range(steps):
                ex(h, *args, flags)
        else:
            for _ in range(steps):
                fn(h, *args)
        t1 = time.perf_counter()
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        assert ev.wait() == 0
        kern = None
        if profile:
            _, tot, n = ev.kernel_stats()
            kern = tot / max(n, 1) * 1e3
        out = {"issue_us": (t1 - t0) / steps * 1e6, "wall_us": (t2 - t0) / steps * 1e6,
               "kernel_us": kern}
        print(f"{label:28s} profile={int(profile)} round {rnd}: issue {out['issue_us']:7.2f} us/call  "
              f"wall {out['wall_us']:7.2f} us/eval  kernels "
              f"{'-' if kern is None else f'{kern:7.2f} us'}", flush=True)
    ev.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--lib", default=None)
    ap.add_argument("--flags", type=int, default=None,
                    help="cse_evaluate_device_ex flags, when the library has it")
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    p16 = bal.program(*bal.synthetic(*bal.CONFIGS["problem-16-22106"]), loss=None)
    arrays = bal.synthetic(*bal.CONFIGS["problem-13682-4456117"])
    s8, _ = shard.shard_program(*arrays, 0, 8, loss=ca.Loss.huber(1.0))
    del arrays
    for prof in (False, True):
        case("problem-16 trivial BSM", p16, args.steps, dev, prof, args.flags)
        case("13682 shard 0 of 8 Huber", s8, max(args.steps // 4, 20), dev, prof, args.flags)


if __name__ == "__main__":
    main()
