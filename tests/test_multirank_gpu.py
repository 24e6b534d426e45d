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


def _rccl_worker(port, backend, fmt, counts, q):
    """One rank of a `backend` process group (world size 1) with the exchange
    forced on: every collective of ShardedEvaluator runs, and with one rank
    each all-reduce is the identity, so the outputs must equal a plain
    evaluation of the same shard bit for bit."""
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
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        C, P, Obs = counts
        cams, pts, ci, pi, obs = bal.synthetic(C, P, Obs, seed=41)
        loss = ca.Loss.huber(1.0)
        stream = torch.cuda.Stream()  # a non-default stream: ordering is exercised
        se = distributed.ShardedEvaluator(cams, pts, ci, pi, obs, 0, 1, device=0, loss=loss,
                                          format=fmt, gradient=True, stream=stream,
                                          exchange=True)
        assert se.exchange and se._host_reduce == (backend == "gloo")
        out = {}
        # overlapped cost all-reduces (async_op=True, one cost slot each), the
        # camera rows in order, then wait_exchange on the evaluator's stream
        costs = [torch.zeros(1, dtype=torch.float64, device=dev) for _ in range(3)]
        for c in costs:
            se.evaluate(cost=c, overlap=True)
        se.wait_exchange()
        assert se.wait() == 0
        torch.cuda.synchronize()
        out["overlap_costs"] = [float(c.item()) for c in costs]
        # ordered (overlap=False), the Jacobian at the same point too
        se.evaluate(overlap=False)
        se.evaluate(overlap=False, new_evaluation_point=False)
        assert se.wait() == 0
        torch.cuda.synchronize()
        out["cost"] = float(se.cost.item())
        out["r"] = se.residuals.cpu().numpy()
        out["j"] = se.jacobian.cpu().numpy()
        out["g"] = se.gradient.cpu().numpy()
        se.close()
        # the same shard through a plain evaluator (no collective at all)
        ev = ca.Evaluator(se.program, device=0)
        ok, c, r, g, j = ev.evaluate()
        ev.close()
        assert ok
        assert all(x == c for x in out["overlap_costs"]), (out["overlap_costs"], c)
        assert out["cost"] == c
        assert np.array_equal(out["r"], r) and np.array_equal(out["j"], j)
        assert np.array_equal(out["g"], g)
        np.save(os.path.join(os.environ.get("TMPDIR", "/tmp"), f"rccl1_{backend}_{fmt}_{port}.npy"),
                np.concatenate([[c], g[se._cam_rows[0]:se._cam_rows[1]]]))
        q.put(("ok", backend))
    except Exception as e:
        import traceback
        q.put((repr(e) + traceback.format_exc(), backend))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fmt", ["block_sparse", "compressed_row"])
def test_rccl_exchange_world_size_one(gpu, fmt):
    """The RCCL branch of ShardedEvaluator (distributed.py: device-tensor
    all_reduce, async_op=True with wait_exchange, the camera-row reduce on
    the evaluator's stream) executed once on the test box's GPU under an
    `nccl` process group of one rank, and the same under gloo; both must
    leave the plain evaluation's outputs unchanged."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    counts = (16, 2500, 12001)
    got = {}
    for backend in ("nccl", "gloo"):
        q = ctx.Queue()
        port = _free_port()
        p = ctx.Process(target=_rccl_worker, args=(port, backend, fmt, counts, q))
        p.start()
        p.join(100)
        if p.is_alive():
            p.kill()
            pytest.fail(f"{backend} rank hung")
        msg, b = q.get(timeout=10)
        assert msg == "ok", msg
        assert p.exitcode == 0
        path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"rccl1_{backend}_{fmt}_{port}.npy")
        got[backend] = np.load(path)
        os.remove(path)
    # RCCL and gloo exchanges give the same cost and camera rows
    assert np.array_equal(got["nccl"], got["gloo"])
