#!/usr/bin/env python3
"""cse_create_multi through host buffers (the reference's seam 2,
registered_cuda_evaluators.h:75-79): problem-13682, residuals + Jacobian
into one host buffer, k shards (all on device 0 when the box has one GPU),
with the caller's buffers page-locked (cse_host_register) or pageable (the
library stages the state through its own pinned buffer and the strips
through pinned bounce buffers).  Prints one JSON line per case.

  python tools/host_multi_probe.py --shards 1,2,8 --steps 3
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ceres-solver-cuda_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ceres_amd as ca  # noqa: E402
from ceres_amd import bal  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="problem-13682-4456117")
    ap.add_argument("--shards", default="1,2,8")
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    ndev = max(1, torch.cuda.device_count())
    prog = bal.synthetic_program(args.config, loss=ca.Loss.huber(1.0))
    hstate = np.array(prog.state)
    r = np.empty(prog.num_residuals)
    j = np.empty(prog.num_jacobian_values)
    ref = None
    for k in [int(x) for x in args.shards.split(",")]:
        devices = [i % ndev for i in range(k)]
        for pinned in (True, False):
            ev = ca.Evaluator(prog, devices=devices)
            if pinned:
                for a in (hstate, r, j):
                    ca.host_register(a)
            try:
                ok = ev.evaluate(hstate, residuals=True, gradient=False, jacobian=True, out=(r, None, j))
                assert ok[0]
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    ev.evaluate(hstate, residuals=True, gradient=False, jacobian=True, out=(r, None, j))
                e = (time.perf_counter() - t0) / args.steps
                h2d, d2h = ev.transfer_bytes()
                digest = (float(r[::9973].sum()), float(j[::99991].sum()))
                if ref is None:
                    ref = digest
            finally:
                ev.close()
                if pinned:
                    for a in (hstate, r, j):
                        ca.host_unregister(a)
            print(json.dumps({"shards": k, "devices": devices, "caller_pinned": pinned,
                              "ms_per_eval": e * 1e3, "evals_per_s": 1.0 / e,
                              "d2h_GBps": 8 * (prog.num_residuals + prog.num_jacobian_values) / e / 1e9,
                              "state_h2d_bytes": int(sum(h2d)), "strips_d2h_bytes": int(sum(d2h)),
                              "same_outputs_as_first_case": digest == ref}), flush=True)


if __name__ == "__main__":
    main()
