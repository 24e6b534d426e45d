"""Block-sharded evaluation through libcse.so in several ranks (configs[4]).

Two ranks share the one GPU of the test box (a real node gives each rank its
own device and RCCL; here gloo carries the exchange): each rank evaluates its
point-bucket shard with ceres_amd.distributed.ShardedEvaluator, all-reduces
the cost and the camera gradient rows, copies its residual and Jacobian
strips to pinned host memory (the reference's D2H seam), and sends them to
rank 0.  Rank 0 assembles the global arrays at the strips' global offsets and
checks them against the unsharded CPU oracle at the reference's tolerance
(tests/parity_util.py), for both Jacobian layouts, with the fused gradient.
"""
import os
import socket

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, fmt, counts, q, side_stream=False):
    import sys
    for p in (os.path.join(REPO, "ceres-solver-cuda_amd"), os.path.join(REPO, "oracle"),
              os.path.join(REPO, "tests")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    import ceres_amd as ca
    from ceres_amd import bal, distributed
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        C, P, Obs = counts
        cams, pts, ci, pi, obs = bal.synthetic(C, P, Obs, seed=33)
        loss = ca.Loss.huber(1.0)
        torch.cuda.set_device(0)
        # side_stream: the evaluator runs on a non-default stream, so the
        # exchange must be ordered against that stream.
        stream = torch.cuda.Stream() if side_stream else None
        se = distributed.ShardedEvaluator(cams, pts, ci, pi, obs, rank, world, device=0,
                                          loss=loss, format=fmt, gradient=True, stream=stream)
        for _ in range(2):  # the second evaluation re-uses every buffer
            se.evaluate()
        status = se.wait()
        hres, hjac = se.host_buffers()
        se.copy_strips_to_host(hres, hjac)
        torch.cuda.synchronize()
        lo, hi = se._cam_rows
        g = se.gradient.cpu().numpy()
        part = (se.shard, hres.numpy().copy(), hjac.numpy().copy(), g[:lo].copy(),
                g[lo:hi].copy(), float(se.cost.item()), status)
        se.close()
        parts = [None] * world
        dist.all_gather_object(parts, part)
        if rank == 0:
            import oracle_py as O
            from ceres_amd import shard
            from parity_util import assert_parity
            assert all(p[6] == 0 for p in parts)
            full = bal.program(cams, pts, ci, pi, obs, loss=loss, format=fmt)
            ref = O.OracleProgram.from_program(full).evaluate(full.state, num_threads=4)
            assert ref[0]
            J = shard.assemble([p[0] for p in parts], [p[2] for p in parts],
                               full.num_jacobian_values)
            assert not np.isnan(J).any()
            R = np.full(full.num_residuals, np.nan)
            for p in parts:
                r0, r1 = p[0].residual_strip
                R[r0:r1] = p[1]
            assert not np.isnan(R).any()
            # Every rank holds the same all-reduced cost and camera rows.
            assert len({p[5] for p in parts}) == 1
            assert all(np.array_equal(p[4], parts[0][4]) for p in parts)
            G = distributed.assemble_gradient([p[0] for p in parts], [p[3] for p in parts],
                                              parts[0][4], P, C)
            assert_parity((True, parts[0][5], R, G, J), ref, ("sharded", fmt, world))
            assert len({p[0].blocks for p in parts}) == world  # really cut
        q.put((rank, "ok"))
    except Exception as e:  # report to the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fmt,side_stream", [("block_sparse", False), ("compressed_row", False),
                                             ("block_sparse", True)])
def test_sharded_libcse_matches_unsharded_oracle(gpu, fmt, side_stream):
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    # Ragged shards: neither cut lands on a 64-block chunk boundary.
    counts = (20, 3001, 21113)
    procs = [ctx.Process(target=_worker, args=(r, world, port, fmt, counts, q, side_stream))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(100)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
    assert not alive, "a rank hung"
    results = dict(q.get(timeout=10) for _ in range(world))
    assert all(v == "ok" for v in results.values()), results
    assert all(p.exitcode == 0 for p in procs)
