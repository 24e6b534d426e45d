#!/usr/bin/env python3
"""A/B timing of builds of the library in interleaved processes.

Loads lib/libcse.so or --lib PATH (e.g. the previous commit's build), builds
one problem-13682-shaped Program and times the residual+Jacobian evaluation
in rounds.  Rounds 2-5 also selected tuning variants of one build through
$CSE_TUNE_VARIANT (the tuning build, removed in round 6: the product reads no
environment variable, so --variants 0 is the only meaningful value now).
Every variant's residuals, Jacobian and cost are checked bit-equal to
variant 0's.

  python tools/ab_bench.py --lib other/libcse.so --variants 0 --rounds 3 --steps 20
"""
import argparse
import hashlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ceres-solver-cuda_amd"))

import numpy as np  # noqa: E402

from ceres_amd import _cse  # noqa: E402

_LIB = os.path.join(REPO, "ceres-solver-cuda_amd", "lib", "libcse.so")
if "--lib" in sys.argv:  # another build of the same ABI (e.g. the previous commit's)
    _LIB = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
_cse.use_library(_LIB)

import ceres_amd as ca  # noqa: E402
from ceres_amd import bal  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--config", default="problem-13682-4456117")
    ap.add_argument("--loss", default="huber")
    ap.add_argument("--out", default=None)
    ap.add_argument("--lib", default=None, help="library to load (default lib/libcse.so)")
    ap.add_argument("--mode", default="jacobian", choices=["jacobian", "gradient", "residual", "cost"])
    ap.add_argument("--format", default="block_sparse", choices=["block_sparse", "compressed_row"])
    ap.add_argument("--held-cameras", type=int, default=0,
                    help="hold the first K cameras constant (the const0 kernels)")
    ap.add_argument("--held-tail", type=int, default=0,
                    help="append one held camera observed by the last K blocks only (the "
                         "held-camera kernels on an otherwise aligned layout)")
    ap.add_argument("--jacobian-form", default="closed", choices=["closed", "jet"],
                    help="cse_options.jacobian_form of the evaluators (product kernels)")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="time rank 0's shard of an N-way point-bucket cut instead")
    args = ap.parse_args()
    import torch
    # "26s16": variant 26 with the slot-0 table repacked at a 16-double stride
    # (CSE_TUNE_CAMSTRIDE, read when the evaluator is created).
    variants = args.variants.split(",")
    loss = {"huber": ca.Loss.huber(1.0), "trivial": ca.Loss.trivial()}[args.loss]
    t0 = time.time()
    if args.shard_of > 1:
        from ceres_amd import shard
        prog = shard.shard_program(*bal.synthetic(*bal.CONFIGS[args.config]), 0, args.shard_of,
                                   loss=loss, format=args.format)[0]
    elif args.held_tail > 0:
        cams, pts, ci, pi, obs = bal.synthetic(*bal.CONFIGS[args.config])
        cams = np.vstack([cams, cams[:1]])
        ci = np.array(ci, copy=True)
        ci[-args.held_tail:] = len(cams) - 1
        prog = bal.program(cams, pts, ci, pi, obs, loss=loss, format=args.format,
                           constant_cameras=(len(cams) - 1,))
    else:
        prog = bal.synthetic_program(args.config, loss=loss, format=args.format,
                                     constant_cameras=tuple(range(args.held_cameras)))
    print(f"# built {args.config} in {time.time() - t0:.1f} s", flush=True)
    dev = torch.device("cuda", 0)
    f64 = torch.float64
    state = torch.from_numpy(prog.state).to(dev)
    cost = torch.zeros(1, dtype=f64, device=dev)
    res = torch.empty(prog.num_residuals, dtype=f64, device=dev)
    jac = torch.empty(prog.num_jacobian_values, dtype=f64, device=dev)
    grad = torch.empty(prog.num_effective_parameters, dtype=f64, device=dev)
    stream = torch.cuda.current_stream(dev)
    ref_hash = None
    times = {v: [] for v in variants}
    walls = {v: [] for v in variants}  # wall ms per evaluation (every launch)
    bytes_ = None
    for rnd in range(args.rounds):
        for v in variants:
            vv, _, cs = v.partition("s")
            os.environ["CSE_TUNE_VARIANT"] = vv
            if cs:
                os.environ["CSE_TUNE_CAMSTRIDE"] = cs
            else:
                os.environ.pop("CSE_TUNE_CAMSTRIDE", None)
            ev = ca.Evaluator(prog, device=0, profile=True, stream=stream.cuda_stream,
                              jacobian_form=args.jacobian_form)
            info = ev.info()
            bytes_ = {"jacobian": info.bytes_jacobian_eval, "residual": info.bytes_residual_eval,
                      "gradient": info.bytes_jacobian_eval + 8 * prog.num_effective_parameters,
                      "cost": info.bytes_residual_eval - 8 * prog.num_residuals}[args.mode]
            rp = res.data_ptr() if args.mode != "cost" else None
            jp = jac.data_ptr() if args.mode in ("jacobian", "gradient") else None
            gp = grad.data_ptr() if args.mode == "gradient" else None
            for _ in range(3):
                ev.evaluate_device(state.data_ptr(), cost.data_ptr(), rp, gp, jp)
            assert ev.wait() == 0
            if rnd == 0:
                h = hashlib.sha1()
                h.update(res.cpu().numpy().tobytes())
                h.update(jac[:: 97].cpu().numpy().tobytes())
                h.update(jac[-100000:].cpu().numpy().tobytes())
                h.update(cost.cpu().numpy().tobytes())
                if args.mode == "gradient":
                    h.update(grad.cpu().numpy().tobytes())
                digest = h.hexdigest()
                if ref_hash is None:
                    ref_hash = digest
                same = digest == ref_hash
                print(f"# variant {v}: outputs {'identical' if same else 'DIFFER'}", flush=True)
            ev.reset_kernel_stats()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                ev.evaluate_device(state.data_ptr(), cost.data_ptr(), rp, gp, jp)
            assert ev.wait() == 0
            torch.cuda.synchronize()
            walls[v].append((time.perf_counter() - t0) / args.steps * 1e3)
            _, total, n = ev.kernel_stats()
            ev.close()
            ms = total / n
            times[v].append(ms)
            print(f"round {rnd} variant {v}: {ms:.4f} ms  {bytes_ / ms / 1e6:.0f} GB/s  "
                  f"frac {bytes_ / ms / 1e6 / 8000:.3f}", flush=True)
    summary = {v: {"median_ms": float(np.median(t)), "min_ms": float(np.min(t)),
                   "median_wall_ms": float(np.median(walls[v])),
                   "frac_median": bytes_ / float(np.median(t)) / 1e6 / 8000} for v, t in times.items()}
    print(json.dumps({"mode": args.mode, "summary": summary}))
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"config": args.config, "loss": args.loss, "times_ms": times,
                       "summary": summary}, f, indent=1)


if __name__ == "__main__":
    main()
