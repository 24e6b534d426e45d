"""Multi-process sharding on CPU with the gloo backend.

Each rank builds its shard of the same synthetic BAL problem with
ceres_amd.shard (point-bucket-aligned block ranges), evaluates it with the
CPU oracle (these tests run without a GPU; on the GPU box bench.py runs the
same shards through libcse.so and RCCL), all-reduces the cost and the camera
gradient, and gathers its Jacobian/residual strips.  Rank 0 checks that the
assembled strips and reduced values equal the unsharded evaluation.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _skewed(seed=21, C=12, P=700):
    """A BAL-shaped problem with ragged point buckets: most points seen by 2-4
    cameras, a few by many more (a rank's cut then lands far from its
    balanced target)."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "ceres-solver-cuda_amd"))
    from ceres_amd import bal
    cams, pts, ci, pi, obs = bal.synthetic(C, P, 3 * P, seed=seed)
    rng = np.random.default_rng(seed)
    per = rng.integers(2, 5, P)
    per[rng.choice(P, 6, replace=False)] = C  # heavy points: every camera
    ci2, pi2, obs2 = [], [], []
    for p in range(P):
        cs = rng.choice(C, per[p], replace=False)
        ci2.extend(cs)
        pi2.extend([p] * len(cs))
        obs2.extend(rng.normal(scale=50.0, size=(len(cs), 2)))
    return cams, pts, np.array(ci2, np.int32), np.array(pi2, np.int32), np.array(obs2)


def _worker(rank, world, port, fmt, q, held=(), skewed=False):
    import sys
    for p in (os.path.join(REPO, "ceres-solver-cuda_amd"), os.path.join(REPO, "oracle"),
              os.path.join(REPO, "tests")):
        sys.path.insert(0, p)
    import ceres_amd as ca
    from ceres_amd import bal, shard
    import oracle_py as O
    from parity_util import is_approx
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        C, P, Obs = 12, 700, 2600
        if skewed:
            cams, pts, ci, pi, obs = _skewed()
            Obs = len(ci)
        else:
            cams, pts, ci, pi, obs = bal.synthetic(C, P, Obs, seed=21)
        loss = ca.Loss.huber(1.0)
        prog, sh = shard.shard_program(cams, pts, ci, pi, obs, rank, world, loss=loss, format=fmt,
                                       constant_cameras=held)
        # The rank's blocks, points and strips are the point-bucket cut's
        # (what bench.py --gpus N reports as blocks_rank0 / strip_rank0).
        pc, bc = shard.point_bucket_cuts(pi, P, world)
        assert sh.blocks == (bc[rank], bc[rank + 1]) and sh.points == (pc[rank], pc[rank + 1])
        assert sh.residual_strip == (2 * bc[rank], 2 * bc[rank + 1])
        if fmt == "block_sparse" and not held:
            assert [g for _, g, _ in sh.jacobian_strips()] == [6 * bc[rank], 6 * Obs + 18 * bc[rank]]
        elif fmt == "compressed_row":
            assert sh.jacobian_strips() == [(0, 24 * bc[rank], 24 * (bc[rank + 1] - bc[rank]))]
        cs = prog.constant_state if prog.constant_state.size else None
        ok, cost, r, g, j = O.OracleProgram.from_program(prog).evaluate(prog.state, cs, num_threads=2)
        assert ok
        c = torch.tensor([cost], dtype=torch.float64)
        dist.all_reduce(c)
        pmap, cmap = shard.gradient_maps(sh, P, C - len(held))
        gcam = torch.from_numpy(g[cmap[0]:cmap[0] + cmap[2]].copy())
        dist.all_reduce(gcam)
        parts = [None] * world
        dist.all_gather_object(parts, (sh, r, j, g[pmap[0]:pmap[0] + pmap[2]].copy()))
        if rank == 0:
            full = bal.program(cams, pts, ci, pi, obs, loss=loss, format=fmt, constant_cameras=held)
            fcs = full.constant_state if full.constant_state.size else None
            okf, costf, rf, gf, jf = O.OracleProgram.from_program(full).evaluate(full.state, fcs,
                                                                              num_threads=2)
            assert okf
            assert abs(float(c.item()) - costf) <= 1e-12 * abs(costf)
            J = shard.assemble([p[0] for p in parts], [p[2] for p in parts], full.num_jacobian_values)
            assert not np.isnan(J).any()
            # Same per-block arithmetic on each side: the strips are bitwise equal.
            assert np.array_equal(J, jf)
            R = np.concatenate([p[1] for p in parts])
            assert np.array_equal(R, rf)
            G = np.concatenate([p[3] for p in parts] + [gcam.numpy()])
            assert is_approx(G, gf, 1e-13)
            sizes = [p[0].blocks[1] - p[0].blocks[0] for p in parts]
            assert sum(sizes) == Obs and min(sizes) > 0
            if not skewed:
                assert max(sizes) - min(sizes) <= 2 * (Obs // P + 1)
        q.put((rank, "ok"))
    except Exception as e:  # report to the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def _run(world, fmt, held=(), skewed=False):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fmt, q, held, skewed))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    results = dict(q.get() for _ in range(world))
    assert all(v == "ok" for v in results.values()), results
    assert all(p.exitcode == 0 for p in procs)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("fmt,held", [("block_sparse", ()), ("compressed_row", ()),
                                      ("block_sparse", (0, 5))])
def test_sharded_evaluation_matches_unsharded(world, fmt, held):
    # held: cameras held constant (their blocks have no F cell; Shard.f_cells)
    _run(world, fmt, held)


@pytest.mark.parametrize("fmt", ["block_sparse", "compressed_row"])
def test_eight_ranks_ragged_cuts(fmt):
    """BASELINE.json configs[4]'s rank count (8) over gloo, on a problem with
    ragged point buckets: the assembled strips equal the unsharded
    evaluation bit for bit and every rank's blocks / strips are the cut's."""
    _run(8, fmt, skewed=True)


def test_point_bucket_cuts_properties():
    import sys
    sys.path.insert(0, os.path.join(REPO, "ceres-solver-cuda_amd"))
    from ceres_amd import shard
    rng = np.random.default_rng(0)
    pt = np.sort(rng.integers(0, 1000, 20000))
    for world in (1, 2, 4, 8, 7):
        pc, bc = shard.point_bucket_cuts(pt, 1000, world)
        assert pc[0] == 0 and pc[-1] == 1000 and bc[0] == 0 and bc[-1] == len(pt)
        assert all(a <= b for a, b in zip(bc, bc[1:]))
        for r in range(1, world):
            # a cut never splits a point's observations
            if 0 < bc[r] < len(pt):
                assert pt[bc[r] - 1] < pt[bc[r]]
    with pytest.raises(ValueError):
        shard.point_bucket_cuts(pt[::-1], 1000, 2)
    # Cuts land on block indices that are multiples of 4 (sector-aligned
    # rank-local F cells) and stay close to the balanced target.
    for world in (2, 3, 8):
        pc, bc = shard.point_bucket_cuts(pt, 1000, world)
        assert all(b % 4 == 0 for b in bc[1:-1])
        for r in range(1, world):
            assert abs(bc[r] - len(pt) * r // world) <= 64 * 40


def test_point_bucket_cuts_small_and_skewed_problems():
    # alignment must never empty or overrun a rank.  About 100
    # points over 8 ranks, with a few heavy points (skewed buckets).
    import sys
    sys.path.insert(0, os.path.join(REPO, "ceres-solver-cuda_amd"))
    from ceres_amd import shard
    rng = np.random.default_rng(5)
    for trial in range(20):
        P = int(rng.integers(90, 120))
        counts = rng.integers(1, 4, P)
        counts[rng.integers(0, P, 3)] += rng.integers(10, 40, 3)
        pt = np.repeat(np.arange(P), counts)
        for world in (2, 3, 8):
            pc, bc = shard.point_bucket_cuts(pt, P, world)
            sizes = np.diff(bc)
            assert (sizes > 0).all(), (trial, world, bc)
            assert bc[0] == 0 and bc[-1] == len(pt) and pc[-1] == P
            for r in range(1, world):
                # each cut stays below the next rank's balanced target
                assert bc[r] < len(pt) * (r + 1) // world or bc[r] == bc[r - 1] + sizes[r - 1]
                if 0 < bc[r] < len(pt):
                    assert pt[bc[r] - 1] < pt[bc[r]]
