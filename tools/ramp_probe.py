#!/usr/bin/env python3
"""Is the first-launch ramp of the headline kernel the platform's or ours?

After an idle phase (the GPU does nothing for --idle seconds, as during
bench.py's problem build), time back-to-back launches of a plain
device-to-device copy (torch's copy kernel, no code of ours) with the same
bytes per launch as the headline evaluation (6.83 GB: 3.42 GB read + 3.42 GB
written), one HIP event pair per launch, then the same after a second idle
phase.  A ramp of the same shape as
profiles/round6/r6d/ramp_headline_dispatches.txt (first launch fast, the
next ones slower, back to steady state over a few tens of ms) in a kernel
that is not ours says the ramp is the GPU's clock / power management.

One JSON line per phase: durations in ms, in launch order.
"""
import argparse
import ctypes as C
import json
import os
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--idle", type=float, default=5.0)
    ap.add_argument("--launches", type=int, default=60)
    ap.add_argument("--gbytes", type=float, default=6.833, help="read + written per launch")
    ap.add_argument("--phases", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = int(args.gbytes * 1e9 / 2 / 8)
    src = torch.ones(n, dtype=torch.float64, device=dev)
    dst = torch.empty_like(src)
    # the shader clock before each copy (tools/clock_probe.hip), if built
    so = os.path.join(REPO, "tools", "build", "libclockprobe.so")
    lib = C.CDLL(so) if os.path.exists(so) else None
    if lib:
        lib.clock_probe_launch.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    probe = torch.zeros(args.launches * 3, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    torch.cuda.synchronize(dev)
    for phase in range(args.phases):
        time.sleep(args.idle)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.launches)]
        for k, (a, b) in enumerate(ev):
            if lib:
                lib.clock_probe_launch(probe.data_ptr() + 24 * k, 4000, stream.cuda_stream)
            a.record()
            dst.copy_(src)
            b.record()
        torch.cuda.synchronize(dev)
        ms = [a.elapsed_time(b) for a, b in ev]
        steady = sorted(ms[-20:])[10]
        p = probe.cpu().tolist()
        mhz = [round(p[3 * k] / (p[3 * k + 1] / 100.0)) if lib else None for k in range(args.launches)]
        print(json.dumps({"phase": phase, "idle_s": args.idle, "bytes_per_launch": 16 * n,
                          "ms": [round(x, 4) for x in ms],
                          "steady_ms_median_last20": round(steady, 4),
                          "first5_over_steady": [round(x / steady, 3) for x in ms[:5]],
                          "launches_above_2pct": sum(1 for x in ms if x > 1.02 * steady),
                          "sclk_mhz_before_copy": mhz}),
              flush=True)


if __name__ == "__main__":
    main()
