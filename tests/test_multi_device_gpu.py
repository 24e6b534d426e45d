"""GPU: BASELINE.json configs[4] -- problem-13682 cut into 8 point-bucket
shards -- and the single-process multi-device evaluator behind the C ABI.

Two forms of the 8-way cut, both checked against the *unsharded* oracle on
the whole problem (tests/parity_util.py tolerances):

  * cse_create_multi (include/cse.h): one evaluator over a device list; the
    library cuts the blocks itself, runs every shard on its device (here all
    eight on the test box's one GPU, device list [0] * 8) and copies each
    shard's residual and Jacobian strips into disjoint regions of the
    caller's one host buffer, as Ceres' host solve expects from
    RegisteredCUDAEvaluators::Evaluate (include/ceres/internal/
    registered_cuda_evaluators.h:75-79, registered_cuda_evaluators.cc:93-100);
    cost and gradient rows are summed over the shards in a fixed order.
  * ceres_amd.shard / the per-rank evaluators that bench.py --gpus 8 runs
    (one libcse.so evaluator per shard, shard.point_bucket_cuts with
    align=4), evaluated one after the other on the one GPU; residual and
    Jacobian strips placed at their global offsets, point gradient rows per
    shard, camera rows and cost summed over the shards (the all-reduce).

Small problems cover ragged shards, several shards per device, multiple
groups (residual_block_index), and the reference's mini bundle adjustment
(table path: manifold, constant blocks, three functor kinds).
"""
import numpy as np
import pytest

import ceres_amd as ca
from ceres_amd import bal, shard
import oracle_py as O
from parity_util import assert_parity

pytestmark = pytest.mark.gpu


def oracle_eval(prog, threads=16, **kw):
    op = O.OracleProgram.from_program(prog)
    return op.evaluate(prog.state, prog.constant_state if prog.constant_state.size else None,
                       num_threads=threads, **kw)


def multi_eval(prog, devices, **kw):
    ev = ca.Evaluator(prog, devices=devices)
    try:
        first, devs = ev.shard_info()
        return ev.evaluate(**kw), ev.info(), first, devs
    finally:
        ev.close()


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
@pytest.mark.parametrize("nshards", [1, 2, 3, 8])
def test_multi_device_small_bal(gpu, fmt, nshards):
    prog = bal.synthetic_program((20, 3001, 21113), loss=ca.Loss.huber(1.0), format=fmt, seed=33)
    ref = oracle_eval(prog, threads=8)
    got, info, first, devs = multi_eval(prog, [0] * nshards)
    assert list(devs) == [0] * nshards and first[0] == 0 and first[-1] == prog.num_residual_blocks
    assert len(first) == nshards + 1 and (np.diff(first) > 0).all()
    # point-bucket cuts: no point's blocks are split between shards
    pt = prog.groups[0].ids[:, 1]
    for c in first[1:-1]:
        assert pt[c - 1] != pt[c]
    assert info.num_affine_groups == 1
    assert info.num_residual_blocks == prog.num_residual_blocks
    assert_parity(got, ref, ("multi", fmt, nshards))
    # The same evaluator again: deterministic (fixed-order sums), and the
    # strips land in caller buffers passed explicitly (kept registered).
    ev = ca.Evaluator(prog, devices=[0] * nshards)
    bufs = (np.empty(prog.num_residuals), np.empty(prog.num_effective_parameters),
            np.empty(prog.num_jacobian_values))
    a = ev.evaluate(out=bufs)
    a = (a[0], a[1], a[2].copy(), a[3].copy(), a[4].copy())
    b = ev.evaluate(out=bufs)
    ev.close()
    assert a[1] == b[1] and all(np.array_equal(x, y) for x, y in zip(a[2:], b[2:]))
    assert_parity(a, ref)


def test_multi_device_shard_local_state_and_registered_buffers(gpu):
    """Each shard holds every camera it sees plus only its own point slice
    (SURVEY.md §8(e)): its device receives C*72 + P_shard*24 bytes of state
    per evaluation, not the whole state.  Buffers the caller page-locked
    (cse_host_register) take the asynchronous copies, others synchronous
    ones: both give the same bits.  Plus covers every parameter block."""
    C, P, O_ = 20, 3001, 21113
    prog = bal.synthetic_program((C, P, O_), loss=ca.Loss.huber(1.0), seed=8)
    ref = oracle_eval(prog, threads=8)
    n = 4
    ev = ca.Evaluator(prog, devices=[0] * n)
    first, _ = ev.shard_info()
    h2d, d2h = ev.transfer_bytes()
    pt = prog.groups[0].ids[:, 1]
    for k in range(n):
        b0, b1 = first[k], first[k + 1]
        npts = len(np.unique(pt[b0:b1]))
        ncam = len(np.unique(prog.groups[0].ids[b0:b1, 0]))
        assert h2d[k] == 8 * (3 * npts + 9 * ncam), k
        assert d2h[k] == 8 * (2 + 24) * (b1 - b0), k
    assert h2d.sum() < 8 * prog.num_parameters + n * 8 * 9 * C
    plain = ev.evaluate()
    state = np.array(prog.state)
    bufs = (np.empty(prog.num_residuals), np.empty(prog.num_effective_parameters),
            np.empty(prog.num_jacobian_values))
    for a in (state, bufs[0], bufs[2]):
        ca.host_register(a)
    try:
        pinned = ev.evaluate(state, out=bufs)
        again = ev.evaluate(state, out=bufs, new_evaluation_point=False)
    finally:
        for a in (state, bufs[0], bufs[2]):
            ca.host_unregister(a)
    with pytest.raises(ValueError, match="not an array registered"):
        ca.host_unregister(state)
    from ceres_amd import _cse
    assert _cse.lib().cse_host_unregister(state.ctypes.data) < 0  # the library's own registry
    assert "not registered" in _cse.lib().cse_last_error().decode()
    with pytest.raises(TypeError):
        ca.host_register(list(range(8)))  # only an ndarray, registered in place
    assert plain[1] == pinned[1] == again[1]
    assert all(np.array_equal(x, y) for x, y in zip(plain[2:], pinned[2:]))
    assert_parity(plain, ref, "shard-local multi")
    delta = np.random.default_rng(1).normal(size=prog.num_effective_parameters)
    out = ev.plus(prog.state, delta)
    ev.close()
    assert np.array_equal(out, prog.state + delta)


def test_multi_device_every_output_combination(gpu):
    prog = bal.synthetic_program((12, 900, 5003), loss=ca.Loss.cauchy(2.0), seed=4)
    ref = oracle_eval(prog, threads=8)
    for r, g, j in [(True, False, False), (False, True, False), (False, False, True),
                    (True, True, False), (False, False, False)]:
        ev = ca.Evaluator(prog, devices=[0, 0, 0])
        got = ev.evaluate(residuals=r, gradient=g, jacobian=j)
        ev.close()
        want = (ref[0], ref[1], ref[2] if r else None, ref[3] if g else None,
                ref[4] if j else None)
        assert_parity(got, want, ("outputs", r, g, j))


def test_multi_device_multiple_groups_and_table_path(gpu):
    # Interleaved groups (residual_block_index) and the mini bundle
    # adjustment of evaluator_cuda_test.cu.cc:232-459 (manifold, constants).
    from test_parity_gpu import mini_ba, small_bal
    prog = small_bal(C=20, P=800, O_=3000)
    g = prog.groups[0]
    idx = np.arange(g.n)
    odd = idx % 2 == 1
    prog.groups = [
        ca.ResidualGroup(g.kind, ca.Loss.huber(1.0), g.ids[odd], g.data[odd], idx[odd].astype(np.int64)),
        ca.ResidualGroup(g.kind, ca.Loss.trivial(), g.ids[~odd], g.data[~odd], idx[~odd].astype(np.int64)),
    ]
    prog.compile(ca.BLOCK_SPARSE, num_eliminate_blocks=800)
    ref = oracle_eval(prog, threads=8)
    got, info, _, _ = multi_eval(prog, [0, 0, 0])
    assert info.num_groups == 2
    assert_parity(got, ref, "multi groups")
    for fmt in (ca.BLOCK_SPARSE, ca.COMPRESSED_ROW):
        prog = mini_ba(fmt)
        ref = oracle_eval(prog, threads=1)
        got, info, first, _ = multi_eval(prog, [0, 0])
        assert info.num_groups >= 1
        assert_parity(got, ref, ("multi mini-BA", fmt))


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
def test_shard_strips_bit_identical_to_the_whole_problem(gpu, fmt):
    """A block's residuals and Jacobian do not depend on which blocks share
    its wave: the rotation form (series or the reference's) is chosen per
    lane (csrc/functors.hpp AngleAxisRotatePoint), so the strips of 8
    per-rank shards -- whose waves start at other blocks -- carry the same
    bits as the whole-problem evaluation.  Camera angles are mixed (about one
    camera in eight beyond theta^2 = 1, and tiny and zero angles), so many
    waves mix the two forms."""
    C, P = 40, 5000
    cams, pts, ci, pi, obs = bal.synthetic(C, P, 30011, seed=21)
    rng = np.random.default_rng(21)
    axis = rng.normal(size=(C, 3))
    axis /= np.linalg.norm(axis, axis=1)[:, None]
    theta = np.where(rng.random(C) < 0.125, rng.uniform(1.0, 3.0, C), rng.uniform(0.0, 1.0, C))
    theta[:3] = [0.0, 2.0 ** -30, 1.0 + 2.0 ** -52]
    cams = cams.copy()
    cams[:, 0:3] = axis * theta[:, None]
    obs = bal.project(cams, pts, ci, pi) + rng.normal(0.0, 1.0, (len(ci), 2))
    loss = ca.Loss.huber(1.0)
    full = bal.program(cams, pts, ci, pi, obs, loss=loss, format=fmt)
    ev = ca.Evaluator(full, device=0)
    ok, _, R, _, J = ev.evaluate(residuals=True, gradient=False, jacobian=True)
    ev.close()
    assert ok
    world = 8
    shards, jparts = [], []
    for rank in range(world):
        prog, sh = shard.shard_program(cams, pts, ci, pi, obs, rank, world, loss=loss, format=fmt)
        ev = ca.Evaluator(prog, device=0)
        ok, _, r, _, j = ev.evaluate(residuals=True, gradient=False, jacobian=True)
        ev.close()
        assert ok
        r0, r1 = sh.residual_strip
        assert np.array_equal(r, R[r0:r1]), (fmt, rank)
        shards.append(sh)
        jparts.append(j)
    Js = shard.assemble(shards, jparts, full.num_jacobian_values)
    assert np.array_equal(Js, J), fmt


def test_multi_device_refuses_device_pointer_calls(gpu):
    prog = bal.synthetic_program((8, 300, 1200), seed=2)
    ev = ca.Evaluator(prog, devices=[0, 0])
    with pytest.raises(RuntimeError, match="multi-device"):
        ev.evaluate_device(1, 1)
    assert ev.wait() == 0
    out = ev.plus(prog.state, np.ones(prog.num_effective_parameters))
    assert np.array_equal(out, prog.state + 1.0)
    ev.close()


# ---- configs[4] at its workload ------------------------------------------
@pytest.fixture(scope="module")
def problem_13682():
    return bal.synthetic(*bal.CONFIGS["problem-13682-4456117"])


@pytest.mark.slow
@pytest.mark.timeout(900)
def test_configs4_problem_13682_cse_create_multi_8_shards(gpu, problem_13682):
    cams, pts, ci, pi, obs = problem_13682
    prog = bal.program(cams, pts, ci, pi, obs, loss=ca.Loss.huber(1.0), format=ca.BLOCK_SPARSE)
    ev = ca.Evaluator(prog, devices=[0] * 8)
    first, devs = ev.shard_info()
    got = ev.evaluate(residuals=True, gradient=True, jacobian=True)
    info = ev.info()
    # Each shard's residual+Jacobian kernel without the gradient (the
    # kernel bench.py times), assembled into the caller's buffers.
    ok_ng, cost_ng, r_ng, _, j_ng = ev.evaluate(residuals=True, gradient=False, jacobian=True)
    ev.close()
    assert info.num_affine_groups == 1 and info.num_fused_gradient_groups == 1
    assert len(first) == 9 and (np.diff(first) > 0).all()
    assert all(c % 4 == 0 for c in first[1:-1])  # sector-aligned rank-local F cells
    for c in first[1:-1]:
        assert pi[c - 1] != pi[c]  # point-bucket cuts
    ref = oracle_eval(prog, threads=16, residuals=True, gradient=True, jacobian=True)
    rep = {}
    assert_parity(got, ref, "configs[4] cse_create_multi x8", report=rep)
    print("configs[4] (cse_create_multi, 8 shards) BSM Huber parity:", rep, "cuts", list(first))
    rep_ng = {}
    assert_parity((ok_ng, cost_ng, r_ng, None, j_ng), (ref[0], ref[1], ref[2], None, ref[4]),
                  "configs[4] cse_create_multi x8, no gradient", report=rep_ng)
    print("configs[4] (cse_create_multi, 8 shards), residual+Jacobian kernel:", rep_ng)


@pytest.mark.slow
@pytest.mark.timeout(900)
@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
def test_configs4_problem_13682_per_rank_shards(gpu, problem_13682, fmt):
    """The 8 ranks of bench.py --gpus 8 (ceres_amd.shard), one after the
    other on the one GPU, assembled at their global offsets."""
    cams, pts, ci, pi, obs = problem_13682
    world = 8
    loss = ca.Loss.huber(1.0)
    parts, parts_ng = [], []
    cost = cost_ng = 0.0
    cam_rows = None
    for rank in range(world):
        prog, sh = shard.shard_program(cams, pts, ci, pi, obs, rank, world, loss=loss, format=fmt)
        ev = ca.Evaluator(prog, device=0)
        ok, c, r, g, j = ev.evaluate(residuals=True, gradient=True, jacobian=True)
        info = ev.info()
        # The rank's timed evaluation (bench.py --gpus 8): residuals and
        # Jacobian, no gradient (EvaluateAffineChunksTwoRoundW1 / ...CrsW1).
        ok_ng, c_ng, r_ng, _, j_ng = ev.evaluate(residuals=True, gradient=False, jacobian=True)
        ev.close()
        assert ok and ok_ng and info.num_affine_groups == 1 and info.num_fused_gradient_groups == 1
        cost += c  # the all-reduce, in rank order
        cost_ng += c_ng
        npts = sh.points[1] - sh.points[0]
        rows = g[3 * npts:]
        cam_rows = rows.copy() if cam_rows is None else cam_rows + rows
        parts.append((sh, r, j, g[:3 * npts].copy()))
        parts_ng.append((r_ng, j_ng))
        del prog
    assert len({p[0].blocks for p in parts}) == world
    assert all(p[0].blocks[0] % 4 == 0 for p in parts)
    full = bal.program(cams, pts, ci, pi, obs, loss=loss, format=fmt)

    def assemble(res, jac):
        J = shard.assemble([p[0] for p in parts], jac, full.num_jacobian_values)
        assert not np.isnan(J).any()
        R = np.full(full.num_residuals, np.nan)
        for p, r in zip(parts, res):
            r0, r1 = p[0].residual_strip
            R[r0:r1] = r
        assert not np.isnan(R).any()
        return R, J

    R, J = assemble([p[1] for p in parts], [p[2] for p in parts])
    R_ng, J_ng = assemble([p[0] for p in parts_ng], [p[1] for p in parts_ng])
    del parts_ng
    from ceres_amd import distributed
    G = distributed.assemble_gradient([p[0] for p in parts], [p[3] for p in parts], cam_rows,
                                      pts.shape[0], cams.shape[0])
    del parts
    ref = oracle_eval(full, threads=16, residuals=True, gradient=True, jacobian=True)
    rep = {}
    assert_parity((True, cost, R, G, J), ref, ("configs[4] per-rank shards", fmt), report=rep)
    print(f"configs[4] (8 per-rank shards) {fmt} Huber parity:", rep)
    rep_ng = {}
    assert_parity((True, cost_ng, R_ng, None, J_ng), (ref[0], ref[1], ref[2], None, ref[4]),
                  ("configs[4] per-rank shards, no gradient", fmt), report=rep_ng)
    print(f"configs[4] (8 per-rank shards) {fmt} Huber, residual+Jacobian kernel:", rep_ng)


@pytest.mark.parametrize("nshards", [1, 3])
def test_plus_in_place_on_a_multi_device_evaluator(gpu, nshards):
    """cse_plus with out == state (Program::Plus(x, delta, x), program.cc:
    121-149) on cse_create_multi: every camera is held by several shards,
    each shard gathers its inputs before any writes, so the in-place result
    is bit-equal to separate buffers."""
    prog = bal.synthetic_program((20, 3001, 21113), loss=ca.Loss.huber(1.0), seed=35)
    rng = np.random.default_rng(9)
    delta = rng.normal(scale=1e-3, size=prog.num_effective_parameters)
    ev = ca.Evaluator(prog, devices=[0] * nshards)
    try:
        first, _ = ev.shard_info()
        if nshards > 1:  # cameras shared by several shards
            cams = [set(prog.groups[0].ids[first[k]:first[k + 1], 0]) for k in range(nshards)]
            assert cams[0] & cams[1]
        separate = ev.plus(prog.state, delta)
        x = prog.state.copy()
        same = ev.plus(x, delta, out=x)
        assert same is x
    finally:
        ev.close()
    assert np.array_equal(x, separate)
    assert np.array_equal(separate, prog.state + delta)  # no manifold: x + delta
