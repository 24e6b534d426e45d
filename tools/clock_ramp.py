#!/usr/bin/env python3
"""The shader clock beside each headline evaluation after an idle phase.

profiles/round6/r6d/ramp_headline_dispatches.txt shows the headline kernel
at 1.38 ms on its first launch after bench.py's problem build, 1.49-1.59 ms
on the next four, and back at 1.33 ms after about twenty.  A plain copy of
the same bytes shows no such ramp (tools/ramp_probe.py).  This probe puts a
one-wave clock reading (tools/clock_probe.hip: s_memtime cycles over
s_memrealtime ticks at 100 MHz) on the evaluator's stream before every
evaluation of problem-13682 (Huber, BSM, residuals + Jacobian) and times
each evaluation with its own HIP events, for --launches launches after an
--idle second pause, twice.  One JSON line per phase.

  hipcc --offload-arch=gfx950 -O3 -fPIC -shared -o tools/build/libclockprobe.so tools/clock_probe.hip
  python tools/clock_ramp.py
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
from ceres_amd import bal  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="problem-13682-4456117")
    ap.add_argument("--idle", type=float, default=5.0)
    ap.add_argument("--launches", type=int, default=40)
    ap.add_argument("--iters", type=int, default=4000, help="probe loop length")
    ap.add_argument("--phases", type=int, default=2)
    args = ap.parse_args()
    lib = C.CDLL(os.path.join(REPO, "tools", "build", "libclockprobe.so"))
    lib.clock_probe_launch.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    prog = bal.synthetic_program(args.config, loss=ca.Loss.huber(1.0))
    ev = ca.Evaluator(prog, stream=stream.cuda_stream)
    f64 = torch.float64
    state = torch.from_numpy(prog.state).to(dev)
    cost = torch.zeros(1, dtype=f64, device=dev)
    res = torch.empty(prog.num_residuals, dtype=f64, device=dev)
    jac = torch.empty(prog.num_jacobian_values, dtype=f64, device=dev)
    probe = torch.zeros(args.launches * 3, dtype=torch.int64, device=dev)
    ev.evaluate_device(state.data_ptr(), cost.data_ptr(), res.data_ptr(), None, jac.data_ptr())
    assert ev.wait() == 0
    for phase in range(args.phases):
        time.sleep(args.idle)
        events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.launches)]
        for k, (a, b) in enumerate(events):
            lib.clock_probe_launch(probe.data_ptr() + 24 * k, args.iters, stream.cuda_stream)
            a.record(stream)
            ev.evaluate_device(state.data_ptr(), cost.data_ptr(), res.data_ptr(), None,
                               jac.data_ptr())
            b.record(stream)
        torch.cuda.synchronize(dev)
        assert ev.wait() == 0
        p = probe.cpu().numpy().reshape(-1, 3)
        mhz = p[:, 0] / (p[:, 1] / 100.0)  # cycles per microsecond
        ms = np.array([a.elapsed_time(b) for a, b in events])
        print(json.dumps({"phase": phase, "idle_s": args.idle, "config": args.config,
                          "eval_ms": [round(float(x), 4) for x in ms],
                          "sclk_mhz_before_eval": [round(float(x)) for x in mhz],
                          "corr_eval_ms_vs_sclk": round(float(np.corrcoef(ms, mhz)[0, 1]), 3)}),
              flush=True)
    ev.close()


if __name__ == "__main__":
    main()
