"""GPU parity: libcse.so (HIP, gfx950) against the CPU oracle.

Every test calls the product through the C ABI (ceres_amd -> libcse.so) and
the oracle (oracle/build/liboracle.so) on the same seeded inputs; the
tolerance is the reference's (tests/parity_util.py).  Covered, as the
reference's own tests do:
  * BAL-shaped problems: problem-16 (BSM, no loss), problem-1778 shape
    (CRS, Huber), Cauchy/scaled losses, both layouts on both paths;
  * the mini bundle-adjustment problem of evaluator_cuda_test.cu.cc:232-459
    (quaternion cameras on a ProductManifold, constant blocks, three
    functor types, Cauchy/Huber/no loss), BSM and CRS;
  * residual-only (cost) evaluation, every output combination, failures
    (non-finite outputs), empty and ragged problems, determinism, the
    device-pointer entry point.
"""
import math

import numpy as np
import pytest

import ceres_amd as ca
from ceres_amd import bal
import oracle_py as O
from parity_util import COST_RTOL, assert_parity, is_approx

pytestmark = pytest.mark.gpu


def oracle_eval(prog, threads=8, apply_loss=True, **kw):
    op = O.OracleProgram.from_program(prog, apply_loss_function=apply_loss)
    return op.evaluate(prog.state, prog.constant_state if prog.constant_state.size else None,
                       num_threads=threads, **kw)


def drop_gradient(out):
    """(ok, cost, r, g, j) without the gradient, for evaluations that did not
    request it."""
    ok, cost, r, _, j = out
    return ok, cost, r, None, j


def gpu_eval(prog, **kw):
    opts = {k: kw.pop(k) for k in list(kw) if k in ("force_general_layout", "apply_loss_function",
                                                    "check_finite")}
    ev = ca.Evaluator(prog, **opts)
    try:
        return ev.evaluate(**kw), ev.info()
    finally:
        ev.close()


def small_bal(C=16, P=600, O_=2300, loss=None, fmt=ca.BLOCK_SPARSE, seed=7):
    return bal.synthetic_program((C, P, O_), loss=loss, format=fmt, seed=seed)


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
@pytest.mark.parametrize("loss", [None, ca.Loss.huber(1.0), ca.Loss.cauchy(2.0),
                                  ca.Loss.huber(3.0).scaled_by(0.5),
                                  ca.Loss.trivial().scaled_by(2.0)])
def test_bal_small_all_losses_both_layouts(gpu, fmt, loss):
    prog = small_bal(loss=loss, fmt=fmt)
    ref = oracle_eval(prog)
    got, info = gpu_eval(prog)
    assert info.num_affine_groups == 1
    assert_parity(got, ref, (fmt, loss))
    got_general, info = gpu_eval(prog, force_general_layout=True)
    assert info.num_affine_groups == 0
    assert_parity(got_general, ref, (fmt, loss, "general"))
    # Same arithmetic, different store path: bit-identical residuals and
    # Jacobian (the gradient sums with atomics in arrival order).
    assert np.array_equal(got[2], got_general[2])
    assert np.array_equal(got[4], got_general[4])
    assert got[1] == got_general[1]


def test_problem_16_block_sparse_no_loss(gpu):
    # BASELINE.json configs[1]: problem-16-22106 shape, BSM, no loss.
    prog = bal.synthetic_program("problem-16-22106")
    ref = oracle_eval(prog)
    got, info = gpu_eval(prog)
    assert info.num_affine_groups == 1
    assert_parity(got, ref, "problem-16")


def test_problem_1778_compressed_row_huber(gpu):
    # BASELINE.json configs[2]: problem-1778-993923 shape, Huber, CRS.
    prog = bal.synthetic_program("problem-1778-993923", loss=ca.Loss.huber(1.0),
                                 format=ca.COMPRESSED_ROW)
    ref = oracle_eval(prog, threads=16)
    ev = ca.Evaluator(prog)
    try:
        got = ev.evaluate()
        # The timed evaluation of bench.py's secondary.configs2 (residuals and
        # Jacobian, no gradient: EvaluateAffineChunksTwoRoundCrsW1), the
        # Jacobian evaluation at an accepted point (trust_region_minimizer.cc:
        # 822-826).
        got_ng = ev.evaluate(residuals=True, gradient=False, jacobian=True)
    finally:
        ev.close()
    rep, rep_ng = {}, {}
    assert_parity(got, ref, "problem-1778", report=rep)
    assert_parity(drop_gradient(got_ng), drop_gradient(ref), "problem-1778 no gradient",
                  report=rep_ng)
    print("problem-1778 CRS Huber parity:", rep)
    print("problem-1778 CRS Huber parity, residual+Jacobian kernel:", rep_ng)
    del got, got_ng
    # The Jet<double, 12> form of the CRS kernel at full size
    # (cse_options.jacobian_form = CSE_JACOBIAN_JET: EvaluateAffineChunks
    # TwoRoundCrsW1<SnavelyJetKind, ...>), against the same oracle values.
    ev = ca.Evaluator(prog, jacobian_form="jet")
    try:
        got_jet = ev.evaluate(residuals=True, gradient=False, jacobian=True)
    finally:
        ev.close()
    rep_jet = {}
    assert_parity(drop_gradient(got_jet), drop_gradient(ref), "problem-1778 CRS Jet form",
                  report=rep_jet)
    print("problem-1778 CRS Huber parity, Jet<12> residual+Jacobian kernel:", rep_jet)


@pytest.mark.parametrize("combo", range(8))
def test_every_output_combination(gpu, combo):
    # evaluator_test.cc:207-218 CheckAllEvaluationCombinations.
    prog = small_bal(loss=ca.Loss.huber(1.0))
    kw = dict(residuals=bool(combo & 1), gradient=bool(combo & 2), jacobian=bool(combo & 4))
    ref = oracle_eval(prog, **kw)
    got, _ = gpu_eval(prog, **kw)
    assert_parity(got, ref, combo)


def test_apply_loss_function_false(gpu):
    # Evaluator::EvaluateOptions::apply_loss_function = false; the reference
    # kernel ignores it (a defect we do not replicate).
    prog = small_bal(loss=ca.Loss.cauchy(1.0))
    ref = oracle_eval(prog, apply_loss=False)
    got, _ = gpu_eval(prog, apply_loss_function=False)
    assert_parity(got, ref)


def quaternion_plus_jacobian(q):
    # QuaternionPlusJacobianImpl<CeresQuaternionOrder> (manifold.cc:63-80).
    w, x, y, z = q
    return np.array([[-x, -y, -z], [w, z, -y], [-z, w, x], [y, -x, w]])


def mini_ba(fmt):
    """internal/ceres/evaluator_cuda_test.cu.cc:232-330."""
    camera1 = [9.99946154126841180165e-01, 7.87061670168454075025e-03,
               -6.39535329165887445751e-03, -2.20038540935716883662e-03,
               -3.4093839577186584e-02, -1.0751387104921525e-01, 1.1202240291236032e+00,
               3.9975152639358436e+02, -3.1770643852803579e-07, 5.8820490534594022e-13]
    camera2 = [9.99877513605250900497e-01, 7.98833588996764563939e-03,
               -1.26117173449355086945e-02, -4.69987892415464365153e-03,
               -8.5667661408224093e-03, -1.2188049069425422e-01, 7.1901330750094605e-01,
               4.0201753385955931e+02, -3.7804765613385677e-07, 9.3074311683844792e-13]
    camera3 = [1.4846251175275622e-02, -2.1062899405576294e-02, -1.1669480098224182e-03,
               -2.4950970734443037e-02, -1.1398470545726247e-01, 9.2166020737027976e-01,
               4.0040175368358570e+02]
    point1 = [-6.1200015717226364e-01, 5.7175904776028286e-01, -1.8470812764548823e+00]
    point2 = [1.7074972220818254e+00, 9.5386921723786655e-01, -6.8771685779735616e+00]
    p = ca.ProblemCUDA()
    c1 = p.add_parameter_block(camera1)
    p1 = p.add_parameter_block(point1)
    c2 = p.add_parameter_block(camera2)
    p2 = p.add_parameter_block(point2)
    c3 = p.add_parameter_block(camera3)
    cauchy, huber = ca.Loss.cauchy(1.0), ca.Loss.huber(1.0)
    p.add_residual_block(ca.SNAVELY_QUATERNION_2_10_3, cauchy, [-3.326500e+02, 2.620900e+02], c1, p1)
    p.add_residual_block(ca.SNAVELY_QUATERNION_2_10_3, cauchy, [-1.997600e+02, 1.667000e+02], c2, p1)
    p.add_residual_block(ca.SNAVELY_QUATERNION_2_10_3, cauchy, [1.224100e+02, 6.554999e+01], c1, p2)
    p.add_residual_block(ca.SNAVELY_NO_DISTORTION_2_7_3, huber, [-2.530600e+02, 2.022700e+02], c3, p1)
    p.add_residual_block(ca.POINT_DISPLACEMENT_3_3, None, point1, p1)
    p.add_residual_block(ca.POINT_DISPLACEMENT_3_3, None, point2, p2)
    p.set_parameter_block_constant(c2)
    p.set_parameter_block_constant(p2)
    # ProductManifold<QuaternionManifold, EuclideanManifold<6>> on camera1.
    P = np.zeros((10, 9))
    P[:4, :3] = quaternion_plus_jacobian(camera1[:4])
    P[4:, 3:] = np.eye(6)
    p.set_plus_jacobian(c1, P)
    prog = p.program()
    prog.compile(fmt, num_eliminate_blocks=0)
    return prog


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
def test_evaluator_cuda_test_mini_bundle_adjustment(gpu, fmt):
    # EvaluateBundleAdjustmentProblem{BlockSparseMatrix,CompressedRowSparseMatrix}
    # (evaluator_cuda_test.cu.cc:451-459).
    prog = mini_ba(fmt)
    # The reduced program drops PointDisplacementError(point2): point2 is
    # constant (evaluator_cuda_test.cu.cc:322-330 -> 11 residuals).
    assert prog.num_residuals == 11
    ref = oracle_eval(prog, threads=1)
    got, info = gpu_eval(prog)
    assert info.num_groups == 3
    assert_parity(got, ref, fmt)
    assert abs(got[1] - ref[1]) <= 1e-13 * max(1.0, abs(ref[1]))


def test_non_finite_output_fails_the_evaluation(gpu):
    # ResidualBlock::Evaluate rejects non-finite outputs
    # (residual_block.cc:110-129); Evaluate then returns false.
    prog = small_bal()
    prog.state[5] = np.nan
    ref = oracle_eval(prog)
    got, _ = gpu_eval(prog)
    assert ref[0] is False and got[0] is False
    # A failed evaluation re-arms: the next good one succeeds.
    ev = ca.Evaluator(prog)
    ok, *_ = ev.evaluate()
    assert not ok
    good = prog.state.copy()
    good[5] = 0.25
    ok, cost, *_ = ev.evaluate(good)
    assert ok and math.isfinite(cost)
    ev.close()


def test_division_by_zero_depth_fails(gpu):
    # p_z == 0: the functor divides by zero -> inf -> rejected.
    cams, pts, ci, pi, obs = bal.synthetic(4, 30, 90, seed=3)
    cams[:, :3] = 0.0
    cams[:, 5] = 0.0
    pts[:, 2] = 0.0
    prog = bal.program(cams, pts, ci, pi, obs)
    ref = oracle_eval(prog)
    got, _ = gpu_eval(prog)
    assert ref[0] is False and got[0] is False


def _two_slot_problem(kind, loss, n=200, seed=5):
    """A small problem of one two-slot kind (Snavely-shaped) with a mix of
    small and large residuals, so that Huber's inlier and outlier branches
    both run."""
    rng = np.random.default_rng(seed)
    s0 = ca.FUNCTOR_SHAPES[kind][1][0]
    p = ca.ProblemCUDA()
    cams = []
    for c in range(4):
        if kind == ca.SNAVELY_QUATERNION_2_10_3:
            q = rng.normal(size=4)
            cam = np.concatenate([q / np.linalg.norm(q), [0.1, -0.2, -10.0], [800.0, 0.01, 0.001]])
        else:
            cam = np.concatenate([rng.normal(0, 0.05, 3), [0.1, -0.2, -10.0], [800.0, 0.01, 0.001]])
        cams.append(p.add_parameter_block(cam[:s0]))
    pts = [p.add_parameter_block(rng.uniform(-3, 3, 3)) for _ in range(n // 4)]
    for i in range(n):
        obs = rng.normal(0, 300.0, 2)
        p.add_residual_block(kind, loss, obs, cams[i % 4], pts[i // 4])
    prog = p.program()
    prog.compile(ca.BLOCK_SPARSE, num_eliminate_blocks=0)
    return prog


@pytest.mark.parametrize("kind", [ca.SNAVELY_2_9_3, ca.SNAVELY_NO_DISTORTION_2_7_3,
                                  ca.SNAVELY_QUATERNION_2_10_3, ca.POINT_DISPLACEMENT_3_3])
@pytest.mark.parametrize("loss", [None, ca.Loss.huber(1.0), ca.Loss.huber(1e6), ca.Loss.cauchy(1.0)])
@pytest.mark.parametrize("where", ["param-nan", "param-inf", "data-nan", "data-inf"])
def test_non_finite_inputs_fail_every_functor_and_loss(gpu, kind, loss, where):
    # The kernels are built with -ffinite-math-only; the evaluation must still
    # reject NaN/Inf outputs (residual_block.cc:146-152) on every functor and
    # every loss branch (Huber a = 1: outliers; a = 1e6: inliers), on both
    # the affine and the table path, as the CPU ProgramEvaluator does.
    if kind == ca.POINT_DISPLACEMENT_3_3:
        p = ca.ProblemCUDA()
        rng = np.random.default_rng(9)
        blocks = [p.add_parameter_block(rng.normal(size=3)) for _ in range(70)]
        for b in blocks:
            p.add_residual_block(kind, loss, rng.normal(size=3), b)
        prog = p.program()
        prog.compile(ca.BLOCK_SPARSE)
    else:
        prog = _two_slot_problem(kind, loss)
    bad = np.nan if where.endswith("nan") else np.inf
    if where.startswith("param"):
        prog.state[len(prog.state) // 2] = bad
    else:
        prog.groups[0].data[prog.groups[0].n // 3, 0] = bad
    ref = oracle_eval(prog, threads=1)
    assert ref[0] is False
    for general in (False, True):
        got, _ = gpu_eval(prog, force_general_layout=general)
        assert got[0] is False, (general, where)
        got, _ = gpu_eval(prog, force_general_layout=general, gradient=False, jacobian=False)
        assert got[0] is False, (general, where, "residuals only")


@pytest.mark.parametrize("n_obs", [1, 2, 63, 64, 65, 255, 256, 257, 1000])
def test_ragged_sizes(gpu, n_obs):
    n_pts = max(1, n_obs // 3)
    prog = small_bal(C=5, P=n_pts, O_=n_obs, loss=ca.Loss.huber(1.0), seed=n_obs)
    ref = oracle_eval(prog, threads=1)
    got, _ = gpu_eval(prog)
    assert_parity(got, ref, n_obs)


def test_empty_problem(gpu):
    p = ca.ProblemCUDA()
    p.add_parameter_block(np.ones(3))
    prog = p.program()
    prog.compile(ca.BLOCK_SPARSE)
    (ok, cost, r, g, j), _ = gpu_eval(prog)
    assert ok and cost == 0.0 and r.size == 0 and j.size == 0
    assert np.array_equal(g, np.zeros(3))


def test_residual_only_fast_path_and_determinism(gpu):
    prog = small_bal(C=40, P=5000, O_=30000, loss=ca.Loss.huber(1.0))
    ref = oracle_eval(prog, residuals=True, gradient=False, jacobian=False)
    ev = ca.Evaluator(prog)
    a = ev.evaluate(residuals=True, gradient=False, jacobian=False)
    b = ev.evaluate(residuals=True, gradient=False, jacobian=False)
    c = ev.evaluate(residuals=False, gradient=False, jacobian=False)
    assert_parity(a, ref)
    # Deterministic cost reduction: bit-identical run to run.
    assert a[1] == b[1] == c[1]
    assert np.array_equal(a[2], b[2])
    full = ev.evaluate()
    assert abs(full[1] - a[1]) <= 1e-12 * abs(a[1])
    ev.close()


def test_multiple_groups_of_one_kind(gpu):
    # Two registered types with different losses over interleaved blocks:
    # exercises the per-group launch, residual_block_index and the
    # cross-group cost sum.
    prog = small_bal(C=20, P=800, O_=3000)
    g = prog.groups[0]
    idx = np.arange(g.n)
    odd = idx % 2 == 1
    prog.groups = [
        ca.ResidualGroup(g.kind, ca.Loss.huber(1.0), g.ids[odd], g.data[odd], idx[odd].astype(np.int64)),
        ca.ResidualGroup(g.kind, ca.Loss.trivial(), g.ids[~odd], g.data[~odd], idx[~odd].astype(np.int64)),
    ]
    prog.compile(ca.BLOCK_SPARSE, num_eliminate_blocks=800)
    ref = oracle_eval(prog)
    got, info = gpu_eval(prog)
    assert info.num_groups == 2
    assert_parity(got, ref)


def test_device_entry_point_with_torch_buffers(gpu):
    import torch
    prog = small_bal(C=30, P=2000, O_=9000, loss=ca.Loss.huber(1.0))
    ref = oracle_eval(prog)
    dev = gpu
    ev = ca.Evaluator(prog, device=0)
    state = torch.from_numpy(prog.state).to(dev)
    cost = torch.zeros(1, dtype=torch.float64, device=dev)
    res = torch.empty(prog.num_residuals, dtype=torch.float64, device=dev)
    grad = torch.empty(prog.num_effective_parameters, dtype=torch.float64, device=dev)
    jac = torch.empty(prog.num_jacobian_values, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    ev.evaluate_device(state.data_ptr(), cost.data_ptr(), res.data_ptr(), grad.data_ptr(),
                       jac.data_ptr())
    assert ev.wait() == 0
    got = (True, float(cost.item()), res.cpu().numpy(), grad.cpu().numpy(), jac.cpu().numpy())
    assert_parity(got, ref)
    ev.close()


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_jet_jacobian_form(gpu, fmt, mode):
    """cse_options.jacobian_form = CSE_JACOBIAN_JET: the Snavely functor's
    Jacobian by forward-mode Jet<double, 12> (AutoDifferentiate,
    autodiff.h:314-381) on the same affine kernels, every gradient mode
    (3 runs as the post-pass 1), against the oracle; the closed-form
    default agrees with it to the parity bounds but not bit for bit (so the
    option really selects another instantiation)."""
    prog = small_bal(loss=ca.Loss.huber(1.0), fmt=fmt)
    ref = oracle_eval(prog)
    ev = ca.Evaluator(prog, jacobian_form="jet", gradient_mode=mode)
    try:
        got = ev.evaluate()
        info = ev.info()
        ng = ev.evaluate(residuals=True, gradient=False, jacobian=True)
        again = ev.evaluate(residuals=True, gradient=False, jacobian=True)
    finally:
        ev.close()
    assert info.num_affine_groups == 1
    assert info.num_fused_gradient_groups == (1 if mode == 0 else 0)
    assert_parity(got, ref, ("jet", fmt, mode))
    assert_parity(drop_gradient(ng), drop_gradient(ref), ("jet, no gradient", fmt))
    assert np.array_equal(ng[4], again[4]) and ng[1] == again[1]
    closed, _ = gpu_eval(prog, residuals=True, gradient=False, jacobian=True)
    assert not np.array_equal(closed[4], ng[4])
    assert is_approx(closed[4], ng[4])
    with pytest.raises(ValueError):
        ca.Evaluator(prog, jacobian_form="numeric")


def test_jet_jacobian_form_table_path(gpu):
    """Shapes the Jet instantiations do not cover run the table kernel with
    Jets: forced general layout, and held cameras (test_constant_gpu)."""
    prog = small_bal(loss=ca.Loss.cauchy(2.0))
    ref = oracle_eval(prog)
    ev = ca.Evaluator(prog, jacobian_form="jet", force_general_layout=True)
    try:
        got = ev.evaluate()
        info = ev.info()
    finally:
        ev.close()
    assert info.num_affine_groups == 0
    assert_parity(got, ref, "jet table")


@pytest.mark.slow
def test_problem_13682_full_size(gpu):
    # BASELINE.json configs[3]: problem-13682 shape, Huber, BSM: the full
    # evaluation against the oracle (16 host threads), plus the
    # size-independent property that the BSM E/F split tiles the values.
    prog = bal.synthetic_program("problem-13682-4456117", loss=ca.Loss.huber(1.0))
    O_ = prog.num_residual_blocks
    assert prog.num_jacobian_values == 24 * O_
    # The gradient comes from the fused deterministic path (gradient_mode 0),
    # as in a trust-region Jacobian evaluation; then the headline evaluation
    # bench.py times (residuals and Jacobian, no gradient: the group-store
    # kernel EvaluateAffineChunksGroupStore where GroupStoreEligible holds for
    # the output strips, else EvaluateAffineChunksTwoRoundW1; 28,987,644
    # blocks either way), as
    # TrustRegionMinimizer issues it at an accepted point
    # (trust_region_minimizer.cc:822-826).
    ev = ca.Evaluator(prog)
    try:
        got = ev.evaluate(residuals=True, gradient=True, jacobian=True)
        info = ev.info()
        got_ng = ev.evaluate(residuals=True, gradient=False, jacobian=True)
    finally:
        ev.close()
    assert info.num_affine_groups == 1 and info.num_fused_gradient_groups == 1
    ref = oracle_eval(prog, threads=16, residuals=True, gradient=True, jacobian=True)
    rep, rep_ng = {}, {}
    assert_parity(got, ref, "problem-13682", report=rep)
    del got
    assert_parity(drop_gradient(got_ng), drop_gradient(ref), "problem-13682 no gradient",
                  report=rep_ng)
    print("problem-13682 BSM Huber parity:", rep)
    print("problem-13682 BSM Huber parity, residual+Jacobian kernel:", rep_ng)
    del got_ng
    # The Jet<double, 12> instantiation of the same kernel (bench.py
    # secondary.jet; cse_options.jacobian_form = CSE_JACOBIAN_JET).
    ev = ca.Evaluator(prog, jacobian_form="jet")
    try:
        got_jet = ev.evaluate(residuals=True, gradient=False, jacobian=True)
    finally:
        ev.close()
    rep_jet = {}
    assert_parity(drop_gradient(got_jet), drop_gradient(ref), "problem-13682 Jet form",
                  report=rep_jet)
    print("problem-13682 BSM Huber parity, Jet<12> residual+Jacobian kernel:", rep_jet)
    del got_jet
    # Residuals + cost only at full size (bench.py secondary.residual_only),
    # and the cost alone, as ComputeCandidatePointAndEvaluateCost asks for
    # the trust-region candidate (trust_region_minimizer.cc:770-787).
    ev = ca.Evaluator(prog)
    try:
        ok, cost, r, g, j = ev.evaluate(residuals=True, gradient=False, jacobian=False)
        ok_c, cost_c, *_ = ev.evaluate(residuals=False, gradient=False, jacobian=False)
    finally:
        ev.close()
    assert ok_c and abs(cost_c - ref[1]) <= COST_RTOL * abs(ref[1])
    assert g is None and j is None
    rep_res = {}
    assert_parity((ok, cost, r, None, None), (ref[0], ref[1], ref[2], None, None),
                  "problem-13682 residual only", report=rep_res)
    print("problem-13682 BSM Huber parity, residual-only kernel:", rep_res)


def test_gradient_post_pass_deterministic_and_agrees_with_atomics(gpu):
    # Affine groups sum J^T r per parameter block in a fixed order (no
    # atomics): bit-identical run to run, and equal (to the tolerance) to the
    # in-kernel atomic path that serves gradient-without-Jacobian requests.
    prog = small_bal(C=24, P=3000, O_=20000, loss=ca.Loss.huber(1.0))
    ref = oracle_eval(prog)
    ev = ca.Evaluator(prog)
    a = ev.evaluate()
    b = ev.evaluate()
    atomic = ev.evaluate(residuals=False, gradient=True, jacobian=False)
    ev.close()
    assert_parity(a, ref)
    assert np.array_equal(a[3], b[3])
    assert is_approx(atomic[3], a[3], 1e-13)


def test_plus_on_device(gpu):
    # Evaluator::Plus -> Program::Plus (program.cc:121-149): without a
    # manifold ParameterBlock::Plus is x + delta (parameter_block.h:227-235),
    # bit for bit.
    prog = small_bal(C=8, P=300, O_=1200)
    ev = ca.Evaluator(prog)
    rng = np.random.default_rng(3)
    delta = rng.normal(size=prog.num_effective_parameters)
    out = ev.plus(prog.state, delta)
    assert np.array_equal(out, prog.state + delta)
    ev.close()


def test_plus_with_ragged_blocks_and_constants(gpu):
    p = ca.ProblemCUDA()
    rng = np.random.default_rng(11)
    cams = [p.add_parameter_block(rng.normal(size=7)) for _ in range(3)]
    pts = [p.add_parameter_block(rng.normal(size=3)) for _ in range(5)]
    for i, x in enumerate(pts):
        p.add_residual_block(ca.SNAVELY_NO_DISTORTION_2_7_3, None, [1.0, 2.0], cams[i % 3], x)
        p.add_residual_block(ca.POINT_DISPLACEMENT_3_3, None, [0.1, 0.2, 0.3], x)
    p.set_parameter_block_constant(cams[1])
    prog = p.program()
    prog.compile(ca.BLOCK_SPARSE)
    ev = ca.Evaluator(prog)
    delta = rng.normal(size=prog.num_effective_parameters)
    assert np.array_equal(ev.plus(prog.state, delta), prog.state + delta)
    ev.close()


def test_plus_refuses_manifolds(gpu):
    prog = mini_ba(ca.BLOCK_SPARSE)
    ev = ca.Evaluator(prog)
    with pytest.raises(RuntimeError, match="manifold"):
        ev.plus(prog.state, np.zeros(prog.num_effective_parameters))
    ev.close()
