#!/usr/bin/env python3
"""The general (table) kernel against the affine fast path on one problem.

Every functor shape the affine kernels do not take (user functors of other
shapes, manifolds given as explicit plus-Jacobians, ...) runs
EvaluateTableKernel.  This times both paths on the same BAL-shaped Program
(cse_options.force_general_layout), device-resident residuals + Jacobian +
cost, interleaved, and checks their outputs agree to 1e-13.

  python tools/general_path_probe.py --config problem-1778-993923 --rounds 3
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ceres-solver-cuda_amd"))
if "--lib" in sys.argv:  # another build of the same ABI (A/B)
    from ceres_amd import _cse  # noqa: E402
    _cse.use_library(os.path.abspath(sys.argv[sys.argv.index("--lib") + 1]))
import ceres_amd as ca  # noqa: E402
from ceres_amd import bal  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="problem-13682-4456117")
    ap.add_argument("--format", default="block_sparse", choices=["block_sparse", "compressed_row"])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--lib", default=None, help="load this build of libcse.so")
    ap.add_argument("--pose-reprojection", action="store_true",
                    help="the user functor PoseReprojectionError <2, 6, 3> of examples/"
                         "user_functors.hip (6-parameter poses, intrinsics in the functor) "
                         "on the same BAL structure, Huber")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    if args.pose_reprojection:
        import ctypes as C
        from ceres_amd import _cse
        lib = _cse.load_functor_library(os.path.join(REPO, "examples", "build",
                                                     "libuser_functors.so"))
        lib.cse_example_kind_name.restype = C.c_char_p
        kinds = (C.c_int32 * 64)()
        n = lib.cse_example_register(kinds, 64)
        kind = {lib.cse_example_kind_name(i).decode(): kinds[i] for i in range(n)}[
            "PoseReprojectionError/Huber"]
        cams, pts, ci, pi, obs = bal.synthetic(*bal.CONFIGS[args.config])
        m = len(ci)
        data = np.empty((m, 6))
        data[:, :2] = obs
        data[:, 2:] = (500.0, 500.0, 0.0, 0.0)
        prog = bal.program(np.ascontiguousarray(cams[:, :6]), pts, ci, pi, data, kind=kind,
                           loss=ca.Loss.huber(1.0), format=args.format)
    else:
        prog = bal.synthetic_program(args.config, loss=ca.Loss.huber(1.0), format=args.format)
    f64 = torch.float64
    state = torch.from_numpy(prog.state).to(dev)
    out = {}
    evs = {name: ca.Evaluator(prog, stream=stream.cuda_stream, force_general_layout=general)
           for name, general in (("affine", False), ("table", True))}
    bufs = {name: (torch.zeros(1, dtype=f64, device=dev),
                   torch.empty(prog.num_residuals, dtype=f64, device=dev),
                   torch.empty(prog.num_jacobian_values, dtype=f64, device=dev)) for name in evs}
    times = {name: [] for name in evs}
    for name, ev in evs.items():
        info = ev.info()
        out[name] = {"affine_groups": info.num_affine_groups}
    for rnd in range(args.rounds):
        for name, ev in evs.items():
            c, r, j = bufs[name]
            for _ in range(5):
                ev.evaluate_device(state.data_ptr(), c.data_ptr(), r.data_ptr(), None, j.data_ptr())
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(args.steps):
                ev.evaluate_device(state.data_ptr(), c.data_ptr(), r.data_ptr(), None, j.data_ptr())
            torch.cuda.synchronize(dev)
            assert ev.wait() == 0
            times[name].append((time.perf_counter() - t0) / args.steps * 1e3)
    a, t = bufs["affine"], bufs["table"]
    rel = lambda x, y: float(torch.linalg.norm(x - y) / torch.linalg.norm(y))
    for name in evs:
        out[name]["ms_per_eval"] = sorted(times[name])[len(times[name]) // 2]
        out[name]["rounds_ms"] = [round(x, 4) for x in times[name]]
    out["table_over_affine"] = out["table"]["ms_per_eval"] / out["affine"]["ms_per_eval"]
    out["rel_diff"] = {"cost": abs(float(a[0] - t[0])) / abs(float(t[0])),
                       "residuals": rel(a[1], t[1]), "jacobian": rel(a[2], t[2])}
    out["config"] = args.config
    out["functor"] = "PoseReprojectionError<2,6,3> (user)" if args.pose_reprojection else "Snavely<2,9,3>"
    # algorithmic bytes of the affine evaluation (cse_info), for its HBM rate
    info = evs["affine"].info()
    out["affine_bytes"] = info.bytes_jacobian_eval
    out["affine_GBps"] = info.bytes_jacobian_eval / (out["affine"]["ms_per_eval"] * 1e-3) / 1e9
    out["format"] = args.format
    for ev in evs.values():
        ev.close()
    print(json.dumps(out), flush=True)
    assert max(out["rel_diff"].values()) <= 1e-13


if __name__ == "__main__":
    main()
