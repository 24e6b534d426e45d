#!/usr/bin/env python3
"""Benchmark: residual+Jacobian evaluations/sec on BAL problem-13682 (MI355X).

One "step" = one residual+Jacobian evaluation of a problem-13682-shaped
Program (13,682 cameras, 4,456,117 points, 28,987,644 SnavelyReprojectionError
<2,9,3> residual blocks, HuberLoss(1.0), BlockSparseMatrix with the points
eliminated first: BASELINE.json configs[3]) through the C ABI's
device-resident entry point (cse_evaluate_device: residuals, Jacobian values
and cost written to HBM; inputs already resident when the clock starts).

Multi-GPU (one process per GPU, launched by torch.distributed.run):
  --scaling weak   (default) every rank evaluates its own problem-13682-sized
                   shard (a distinct seed) of an N x larger global problem;
                   the scalar cost is all-reduced over RCCL each step.
                   value = N * steps / time.
  --scaling strong the one problem-13682 is partitioned at point-bucket
                   boundaries (BASELINE.json configs[4]); each rank writes
                   its contiguous Jacobian strips; cost all-reduced over RCCL.
                   value = steps / time.

Data is synthetic (no BAL file is available offline; see
ceres_amd/bal.py for the generator), with the exact BAL header counts.
Rank 0 prints one JSON line; see DESIGN.md §5 for every field.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ceres-solver-cuda_amd"))

import ceres_amd as ca  # noqa: E402
from ceres_amd import bal, shard  # noqa: E402

PEAK_HBM_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "residual+Jacobian evaluations/sec on BAL problem-13682; achieved HBM GB/s"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="problem-13682-4456117", choices=list(bal.CONFIGS))
    ap.add_argument("--loss", default="huber", choices=["trivial", "huber", "cauchy"])
    ap.add_argument("--format", default="block_sparse", choices=["block_sparse", "compressed_row"])
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    ap.add_argument("--gradient", action="store_true", help="also produce the gradient J^T r")
    ap.add_argument("--gradient-mode", type=int, default=0, choices=[0, 1, 2],
                    help="cse_options.gradient_mode: 0 fused (default), 1 post-pass, 2 atomics")
    ap.add_argument("--mode", default="jacobian",
                    choices=["jacobian", "residual", "candidate", "spmv", "cgnr"],
                    help="jacobian: residual+Jacobian evaluation (the headline metric); "
                         "residual: residuals+cost only; candidate: the trust-region candidate "
                         "step, Plus(x, delta) then cost-only evaluation "
                         "(trust_region_minimizer.cc:770-788); spmv: one CGNR iteration's "
                         "products J p and J^T (J p) on the evaluated Jacobian (cgnr_solver.cc)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-blocks", type=int, default=0,
                    help="0 = the whole workload (about 1 s per eval on 16 cores)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, affinity)")
    ap.add_argument("--seed", type=int, default=0xCE2E5)
    ap.add_argument("--host-copy", action="store_true",
                    help="also time evaluations that copy the rank's residuals and Jacobian "
                         "strips to pinned host memory (the reference's D2H seam; reported "
                         "under 'host_copy', never as value)")
    return ap.parse_args()


def make_loss(name):
    return {"trivial": ca.Loss.trivial(), "huber": ca.Loss.huber(1.0),
            "cauchy": ca.Loss.cauchy(1.0)}[name]


def build_shard(args, rank, world):
    counts = bal.CONFIGS[args.config]
    loss = make_loss(args.loss)
    if args.scaling == "weak" or world == 1:
        cams, pts, ci, pi, obs = bal.synthetic(*counts, seed=args.seed + rank)
        prog = bal.program(cams, pts, ci, pi, obs, loss=loss, format=args.format)
        return prog, {"blocks": int(counts[2]), "strip": None}
    cams, pts, ci, pi, obs = bal.synthetic(*counts, seed=args.seed)
    prog, sh = shard.shard_program(cams, pts, ci, pi, obs, rank, world, loss=loss,
                                   format=args.format)
    strips = [[g, g + n] for _, g, n in sh.jacobian_strips()]
    return prog, {"blocks": sh.blocks[1] - sh.blocks[0], "strip": strips}


def cpu_baseline(args, threads):
    """The oracle (CPU restatement of Ceres' ProgramEvaluator, oracle/) on a
    bounded, point-bucket-aligned sample of the same workload."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_py as O
    counts = bal.CONFIGS[args.config]
    cams, pts, ci, pi, obs = bal.synthetic(*counts, seed=args.seed)
    S = min(args.cpu_sample_blocks or counts[2], counts[2])
    # Cut at a point-bucket boundary.
    last_pt = int(pi[S - 1])
    S = int(np.searchsorted(pi, last_pt, side="right"))
    np_ = last_pt + 1
    prog = bal.program(cams, pts[:np_], ci[:S], pi[:S], obs[:S], loss=make_loss(args.loss),
                       format=args.format)
    op = O.OracleProgram.from_program(prog)
    ev = op.evaluator(threads)
    r = np.empty(prog.num_residuals)
    j = np.empty(prog.num_jacobian_values)
    g = np.empty(prog.num_effective_parameters) if args.gradient else None
    ev.run(prog.state, None, r, g, j)  # warm-up
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        ok, _ = ev.run(prog.state, None, r, g, j)
        times.append(time.perf_counter() - t0)
        assert ok
    ev.close()
    t = float(np.median(times))
    blocks_per_s = S / t
    return {"value": blocks_per_s / counts[2], "unit": "evals/s", "cores": threads,
            "kind": "port",
            "sample": (f"all {S:,} residual blocks" if S == counts[2] else
                   f"first {S:,} of {counts[2]:,} residual blocks (point-bucket aligned)") +
                  f" of the same workload, residual+Jacobian{'+gradient' if args.gradient else ''}, "
                  f"median of 3 evals = {t * 1e3:.1f} ms; value = blocks/s / {counts[2]:,}",
            "blocks_per_sec": blocks_per_s}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    # One process per GPU.  (Ranks beyond the visible devices share them:
    # that only happens in a 1-GPU rehearsal of the multi-rank path, which
    # also sets CSE_DIST_BACKEND=gloo since RCCL needs distinct devices.)
    dev_index = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    backend = os.environ.get("CSE_DIST_BACKEND", "nccl")
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    t_build = time.perf_counter()
    prog, shard_info = build_shard(args, rank, world)
    build_s = time.perf_counter() - t_build

    stream = torch.cuda.current_stream(dev)
    ev = ca.Evaluator(prog, device=dev_index, profile=True, stream=stream.cuda_stream,
                      gradient_mode=args.gradient_mode)
    info = ev.info()
    f64 = torch.float64
    state = torch.from_numpy(prog.state).to(dev)
    cost = torch.zeros(1, dtype=f64, device=dev)
    res = torch.empty(prog.num_residuals, dtype=f64, device=dev)
    jac = torch.empty(prog.num_jacobian_values, dtype=f64, device=dev)
    grad = torch.empty(prog.num_effective_parameters, dtype=f64, device=dev) if args.gradient else None
    gptr = grad.data_ptr() if grad is not None else None

    if args.mode == "candidate":
        delta = torch.full((prog.num_effective_parameters,), 1e-6, dtype=f64, device=dev)
        cand = torch.empty_like(state)
    if args.mode in ("spmv", "cgnr"):
        ev.evaluate_device(state.data_ptr(), cost.data_ptr(), res.data_ptr(), None, jac.data_ptr())
        pvec = torch.ones(prog.num_effective_parameters, dtype=f64, device=dev)
        dvec = torch.full((prog.num_effective_parameters,), 0.5, dtype=f64, device=dev)
        jp = torch.zeros(prog.num_residuals, dtype=f64, device=dev)
        jtjp = torch.zeros(prog.num_effective_parameters, dtype=f64, device=dev)

    def step():
        if args.mode == "jacobian":
            ev.evaluate_device(state.data_ptr(), cost.data_ptr(), res.data_ptr(), gptr,
                               jac.data_ptr())
        elif args.mode == "residual":
            ev.evaluate_device(state.data_ptr(), cost.data_ptr(), res.data_ptr(), None, None)
        elif args.mode == "candidate":
            ev.plus_device(state.data_ptr(), delta.data_ptr(), cand.data_ptr())
            ev.evaluate_device(cand.data_ptr(), cost.data_ptr(), None, None, None)
        elif args.mode == "cgnr":  # one pass: J^T J p + D^2 p (cse_cgnr_multiply)
            ev.cgnr_multiply_device(jac.data_ptr(), dvec.data_ptr(), pvec.data_ptr(),
                                    jtjp.data_ptr())
            return
        else:
            ev.right_multiply_device(jac.data_ptr(), pvec.data_ptr(), jp.data_ptr())
            ev.left_multiply_device(jac.data_ptr(), jp.data_ptr(), jtjp.data_ptr())
            return
        if world > 1:
            dist.all_reduce(cost)  # RCCL over xGMI: the global cost

    for _ in range(args.warmup):
        step()
    status = ev.wait()
    if status != 0:
        raise SystemExit(f"rank {rank}: evaluation failed during warm-up (status {status})")
    ev.reset_kernel_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    status = ev.wait()
    last_ms, total_ms, launches = ev.kernel_stats()
    kernel_ms = total_ms / max(launches, 1)
    if args.mode in ("spmv", "cgnr"):  # no evaluate launches in the timed loop: the step time
        kernel_ms = elapsed / args.steps * 1e3
    if world > 1:
        t = torch.tensor([elapsed, kernel_ms], dtype=f64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms_max = float(t[0]), float(t[1])
        ok = torch.tensor([status], dtype=torch.int32, device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MAX)
        status = int(ok.item())
    else:
        kernel_ms_max = kernel_ms
    if status != 0:
        raise SystemExit(f"evaluation failed (status {status})")

    host_copy = None
    if args.host_copy:
        # The reference's seam: outputs handed back in host memory.  Each rank
        # copies its contiguous residual and Jacobian strips (shard.Shard) to
        # pinned buffers on the evaluator's stream.
        hres = torch.empty(prog.num_residuals, dtype=f64, pin_memory=True)
        hjac = torch.empty(prog.num_jacobian_values, dtype=f64, pin_memory=True)

        def step_host():
            step()
            hres.copy_(res, non_blocking=True)
            hjac.copy_(jac, non_blocking=True)

        step_host()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        th = time.perf_counter()
        for _ in range(args.steps):
            step_host()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        eh = time.perf_counter() - th
        if world > 1:
            t = torch.tensor([eh], dtype=f64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            eh = float(t[0])
        d2h = (prog.num_residuals + prog.num_jacobian_values) * 8
        host_copy = {
            "value": (world if (args.scaling == "weak" or world == 1) else 1) * args.steps / eh,
            "unit": "evals/s", "ms_per_step": eh / args.steps * 1e3,
            "d2h_bytes_per_rank": d2h, "d2h_GBps_per_rank": d2h * args.steps / eh / 1e9,
            "what": "device evaluation + D2H of the rank's residual and Jacobian strips into "
                    "pinned host memory, every step (PCIe-inclusive; not the headline value)"}

    # Compulsory bytes (SURVEY.md §8 d); the gradient adds its 8 B per
    # effective parameter written.
    bytes_per_launch = info.bytes_jacobian_eval + (8 * prog.num_effective_parameters
                                                   if args.gradient else 0)
    if args.mode == "residual":
        bytes_per_launch = info.bytes_residual_eval
    elif args.mode == "spmv":
        # J read twice, p/J p/J^T J p vectors; kernel_ms (events around the
        # evaluate launches only) does not apply, the step time does
        bytes_per_launch = 2 * 8 * prog.num_jacobian_values
    elif args.mode == "cgnr":
        # the normal operator's compulsory bytes: J once, p, D and y
        bytes_per_launch = 8 * prog.num_jacobian_values + 4 * 8 * prog.num_effective_parameters
    elif args.mode == "candidate":
        # the timed kernel is the cost-only evaluation (no residual stores);
        # Plus is in ms_per_step, not in kernel_ms_avg
        bytes_per_launch = info.bytes_residual_eval - 8 * prog.num_residuals
    achieved = bytes_per_launch / (kernel_ms * 1e-3) / 1e9
    weak = args.scaling == "weak" or world == 1
    value = (world if weak else 1) * args.steps / elapsed
    out = None
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            threads = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
            cpu = cpu_baseline(args, threads)
        traffic = None
        pmc_path = os.path.join(REPO, "profiles", f"pmc_{args.config}_{args.loss}_{args.format}.json")
        if os.path.exists(pmc_path):
            with open(pmc_path) as fh:
                pmc = json.load(fh)
            traffic = pmc.get("hbm_bytes_per_launch")
        C_, P_, O_ = bal.CONFIGS[args.config]
        out = {
            "metric": METRIC if args.mode == "jacobian" else
                      f"{args.mode} evaluations/sec on BAL {args.config} (not the headline)",
            "value": value,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if weak else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (BAL-shaped: exact header counts, seeded generator)",
            "config": {
                "workload": f"{args.config} SnavelyReprojectionError<2,9,3> "
                            f"{args.loss} {args.format} "
                            + {"jacobian": "residual+Jacobian", "residual": "residual+cost",
                               "candidate": "Plus + cost-only",
                               "spmv": "J p + J^T (J p)",
                               "cgnr": "J^T J p + D^2 p (one pass)"}[args.mode]
                            + f"{'+gradient' if args.gradient else ''}, device-resident",
                "cameras": C_, "points": P_, "observations": O_,
                "blocks_per_rank": shard_info["blocks"],
                "parallelism": ("replica shards per rank" if weak and world > 1 else
                                "point-bucket block sharding" if world > 1 else "single GPU"),
                "strip_rank0": shard_info["strip"],
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": PEAK_HBM_GBPS,
                "unit": "GB/s",
                "frac": achieved / PEAK_HBM_GBPS,
                "traffic": traffic,
                "algorithmic_bytes_per_launch": bytes_per_launch,
                "kernel_ms_avg": kernel_ms,
                "kernel_ms_avg_max_rank": kernel_ms_max,
                "kernel": "cse::EvaluateAffineChunks<SnavelyKind, loss, jacobian, layout, ...>",
                "traffic_source": "profiles/pmc_<config>_<loss>_<format>.json (rocprofv3 FETCH_SIZE/WRITE_SIZE)",
            },
            "cpu_baseline": cpu,
            "host_copy": host_copy,
            "speedup_vs_cpu": (value / world / cpu["value"]) if cpu else None,
            "build_s": build_s,
            "reference_published": {"value": 0.6455, "unit": "evals/s",
                                    "what": "V100 Jacobian&residual eval incl. H2D/D2H, no loss, "
                                            "README.md:189 (not the same metric)"},
        }
        print(json.dumps(out), flush=True)
    ev.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
