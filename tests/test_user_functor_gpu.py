"""User AutoDiffCostFunction functors on the GPU (include/ceres_amd/
autodiff_cuda.h; the reference's usage model, README.md:19-33,
include/ceres/problem_cuda.h:110-160,423-474).

The example library (examples/user_functors.hip) compiles the reference's
own test functors and BundlerResidual in a user TU and registers their
kernels.  Checked here:
  * the reference's test functors (evaluator_cuda_test.cu.cc:84-230,
    autodiff_cost_function_cuda_test.cu.cc:40-51,123-139,224-230) as user
    kinds write the same bits as the library's kinds of the same functor,
    residuals and Jacobian, both layouts, both kernel paths (the library's
    Snavely kind in its Jet<double, 12> form, jacobian_form "jet");
  * BundlerResidual (bundle_adjustment_test_util.h:188-227, restated in the
    oracle) against the oracle with library and user losses (SoftLOne,
    Tolerant from loss_function.cc, as LossFunctionCUDA classes), every
    output, and at the problem-13682 size;
  * a functor that leaves an output unassigned fails the evaluation;
    a group whose loss differs from the kind's is refused.
Tolerance: tests/parity_util.py (the reference's isApprox 1e-13).
"""
import copy
import dataclasses

import numpy as np
import pytest

import ceres_amd as ca
from ceres_amd import _cse, bal
import oracle_py as O
from parity_util import assert_parity
import user_functors as U

pytestmark = pytest.mark.gpu


def with_kind(prog, kind, loss=None):
    p = copy.copy(prog)
    p.groups = [dataclasses.replace(g, kind=kind, loss=loss if loss is not None else g.loss)
                for g in prog.groups]
    return p


def evaluate(prog, **kw):
    opts = {k: kw.pop(k) for k in list(kw)
            if k in ("force_general_layout", "jacobian_form", "gradient_mode")}
    ev = ca.Evaluator(prog, **opts)
    try:
        return ev.evaluate(**kw), ev.info()
    finally:
        ev.close()


def assert_same_bits(a, b, what, gradient=False):
    ok_a, cost_a, r_a, g_a, j_a = a
    ok_b, cost_b, r_b, g_b, j_b = b
    assert ok_a == ok_b, what
    assert np.array_equal(r_a, r_b), (what, "residuals")
    assert np.array_equal(j_a, j_b), (what, "jacobian")
    assert cost_a == cost_b, (what, cost_a, cost_b)
    if gradient:
        assert np.array_equal(g_a, g_b), (what, "gradient")


def oracle(prog, kind_map=None, loss_map=None, threads=8, **kw):
    op = O.OracleProgram.from_program(prog, kind_map=kind_map, loss_map=loss_map)
    return op.evaluate(prog.state, prog.constant_state if prog.constant_state.size else None,
                       num_threads=threads, **kw)


def small(C=16, P=600, O_=2300, seed=7):
    return bal.synthetic(C, P, O_, seed=seed)


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
@pytest.mark.parametrize("loss_name,loss", [("Trivial", None), ("Huber", ca.Loss.huber(1.0)),
                                            ("Cauchy", ca.Loss.cauchy(2.0))])
def test_snavely_user_kind_equals_library_jet_kind(gpu, fmt, loss_name, loss):
    cams, pts, ci, pi, obs = small()
    lib_prog = bal.program(cams, pts, ci, pi, obs, loss=loss, format=fmt)
    user_prog = with_kind(lib_prog, U.kind("SnavelyReprojectionError/" + loss_name))
    for general in (False, True):
        a, ia = evaluate(lib_prog, jacobian_form="jet", force_general_layout=general, gradient=False)
        b, ib = evaluate(user_prog, force_general_layout=general, gradient=False)
        assert ia.num_affine_groups == ib.num_affine_groups == (0 if general else 1)
        assert_same_bits(a, b, (fmt, loss_name, general))
    ref = oracle(lib_prog)
    got, _ = evaluate(user_prog)
    assert_parity(got, ref, (fmt, loss_name))


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
@pytest.mark.parametrize("loss_name,loss", [("Trivial", None), ("Huber", ca.Loss.huber(1.0)),
                                            ("Cauchy", ca.Loss.cauchy(2.0))])
def test_user_kinds_take_the_fused_gradient(gpu, fmt, loss_name, loss):
    """ABI 5: a user kind of shape <NR, S0, 3> sums its gradient in
    gradient_mode 0 as the library's Snavely kinds do (the points in the
    Jacobian kernel, the camera rows by re-evaluation in camera order;
    cse_functor_ops.fused_points / camera_gradient).  Against the same kind's
    post-pass (mode 1) and the library kind: 1e-13; residuals and Jacobian
    bit-equal to the post-pass run's; a repeat evaluation bit-equal; mode 3
    (no fused form for user kinds) takes the post-pass."""
    cams, pts, ci, pi, obs = small()
    lib_prog = bal.program(cams, pts, ci, pi, obs, loss=loss, format=fmt)
    user_prog = with_kind(lib_prog, U.kind("SnavelyReprojectionError/" + loss_name))
    fused, i0 = evaluate(user_prog)
    again, _ = evaluate(user_prog)
    post, i1 = evaluate(user_prog, gradient_mode=1)
    mode3, i3 = evaluate(user_prog, gradient_mode=3)
    lib, il = evaluate(lib_prog)
    assert i0.num_fused_gradient_groups == 1 and il.num_fused_gradient_groups == 1
    assert i1.num_fused_gradient_groups == 0 and i3.num_fused_gradient_groups == 0
    assert_same_bits(fused, again, (fmt, loss_name, "repeat"), gradient=True)
    assert_same_bits(fused, post, (fmt, loss_name, "mode 1"))
    assert np.array_equal(mode3[3], post[3]), (fmt, loss_name, "mode 3")
    assert _close(fused[3], post[3]), np.linalg.norm(fused[3] - post[3])
    assert _close(fused[3], lib[3]), np.linalg.norm(fused[3] - lib[3])
    assert_parity(fused, oracle(lib_prog), (fmt, loss_name, "fused"))


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
def test_reference_test_functors_equal_library_kinds(gpu, fmt):
    cams, pts, ci, pi, obs = small(C=12, P=500, O_=2000, seed=11)
    # SnavelyReprojectionErrorNoRadialDistortion<2, 7, 3>
    p7 = bal.program(np.ascontiguousarray(cams[:, :7]), pts, ci, pi, obs,
                     kind=_cse.SNAVELY_NO_DISTORTION_2_7_3, format=fmt)
    # SnavelyReprojectionErrorWithQuaternions<2, 10, 3> (no manifold)
    p10 = bal.synthetic_program((12, 500, 2000), seed=11, quaternion=True, format=fmt)
    cases = [(p7, "SnavelyReprojectionErrorNoRadialDistortion/Trivial"),
             (p10, "SnavelyReprojectionErrorWithQuaternions/Trivial")]
    for prog, name in cases:
        ref_lib, info_lib = evaluate(prog, gradient=False)
        got, info = evaluate(with_kind(prog, U.kind(name)), gradient=False)
        assert info.num_affine_groups == info_lib.num_affine_groups == 1
        assert_same_bits(got, ref_lib, name)
        got_g, _ = evaluate(with_kind(prog, U.kind(name)))
        assert_parity(got_g, oracle(prog), name)


def point_problem(n=3000, seed=5):
    # PointDisplacementError<3, 3> blocks over scattered points, some shared.
    rng = np.random.default_rng(seed)
    pb = ca.ProblemCUDA()
    pts = [pb.add_parameter_block(rng.normal(size=3)) for _ in range(n // 3)]
    ids = rng.integers(0, len(pts), size=n)
    data = rng.normal(size=(n, 3))
    return pb, ids, data


def test_point_displacement_user_kind_equals_library(gpu):
    pb, ids, data = point_problem()
    pb.add_residual_blocks(_cse.POINT_DISPLACEMENT_3_3, None, ids[:, None], data)
    lib_prog = pb.program()
    lib_prog.compile(ca.BLOCK_SPARSE)
    user_prog = with_kind(lib_prog, U.kind("PointDisplacementError/Trivial"))
    a, _ = evaluate(lib_prog, gradient=False)
    b, _ = evaluate(user_prog, gradient=False)
    assert_same_bits(a, b, "point displacement")
    got, _ = evaluate(user_prog)
    assert_parity(got, oracle(lib_prog), "point displacement")


def test_general_path_functors_equal_library_test_kinds(gpu):
    # BinaryScalarCost<1, 2, 2> and TenParameterCost<1, 1 x 10>: the general
    # kernel (shapes outside the affine set).
    rng = np.random.default_rng(3)
    pb = ca.ProblemCUDA()
    xs = [pb.add_parameter_block(rng.normal(size=2)) for _ in range(40)]
    ones = [pb.add_parameter_block(rng.normal(size=1)) for _ in range(30)]
    n = 500
    # distinct blocks within each residual block (ProblemImpl::AddResidualBlock
    # refuses a block listed twice, problem_impl.cc:285-301)
    bil = np.stack([rng.choice(xs, 2, replace=False) for _ in range(n)])
    ten = np.stack([rng.choice(ones, 10, replace=False) for _ in range(n)])
    pb.add_residual_blocks(_cse.TEST_BILINEAR_1_2_2, None, bil, rng.normal(size=(n, 1)))
    pb.add_residual_blocks(_cse.TEST_TEN_PARAMETER_1_x10, None, ten, np.zeros((n, 1)))
    lib_prog = pb.program()
    lib_prog.compile(ca.COMPRESSED_ROW)
    user_prog = copy.copy(lib_prog)
    user_prog.groups = [dataclasses.replace(
        g, kind=U.kind("BinaryScalarCost/Trivial" if g.kind == _cse.TEST_BILINEAR_1_2_2
                       else "TenParameterCost/Trivial")) for g in lib_prog.groups]
    a, _ = evaluate(lib_prog)
    b, info = evaluate(user_prog)
    assert info.num_affine_groups == 0
    assert_same_bits(a, b, "general path")
    assert np.allclose(a[3], b[3], rtol=1e-13, atol=1e-13)  # gradient atomics: arrival order


def test_unassigned_output_fails_the_evaluation(gpu):
    # OnlyFillsOneOutputFunctor (autodiff_cost_function_cuda_test.cu.cc:224-230):
    # AutoDifferentiate's kImpossibleValue pre-fill is caught (autodiff.h:355-360).
    pb = ca.ProblemCUDA()
    x = pb.add_parameter_block(np.array([2.0]))
    pb.add_residual_blocks(U.kind("OnlyFillsOneOutputFunctor/Trivial"), None, [[x]], [[0.0]])
    prog = pb.program()
    prog.compile(ca.BLOCK_SPARSE)
    got, _ = evaluate(prog)
    assert got[0] is False


def test_loss_must_match_the_registered_kind(gpu):
    cams, pts, ci, pi, obs = small()
    prog = bal.program(cams, pts, ci, pi, obs, kind=U.kind("BundlerResidual/Trivial"),
                       loss=ca.Loss.huber(1.0))
    with pytest.raises(RuntimeError, match="loss kind"):
        ca.Evaluator(prog)


BUNDLER = {"Trivial": None, "Huber": ca.Loss.huber(1.0)}


def bundler_losses():
    return [("Trivial", None, None), ("Huber", ca.Loss.huber(1.0), None),
            ("SoftLOne", U.soft_l_one(2.0), (O.LOSS_SOFT_L_ONE, 2.0, 0.0)),
            ("Tolerant", U.tolerant(3.0, 2.0), (O.LOSS_TOLERANT, 3.0, 2.0)),
            ("SoftLOne", U.soft_l_one(2.0).scaled_by(0.5), (O.LOSS_SOFT_L_ONE, 2.0, 0.0))]


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
@pytest.mark.parametrize("case", range(5))
def test_bundler_residual_against_the_oracle(gpu, fmt, case):
    name, loss, oracle_loss = bundler_losses()[case]
    cams, pts, ci, pi, obs = small(seed=17 + case)
    prog = bal.program(cams, pts, ci, pi, obs, kind=U.kind("BundlerResidual/" + name), loss=loss,
                       format=fmt)
    kmap = {U.kind("BundlerResidual/" + name): O.BUNDLER_RESIDUAL_2_9_3}
    lmap = (lambda l: oracle_loss) if oracle_loss else None
    for combo in range(8):
        kw = dict(residuals=bool(combo & 1), gradient=bool(combo & 2), jacobian=bool(combo & 4))
        ref = oracle(prog, kmap, lmap, **kw)
        got, info = evaluate(prog, **kw)
        assert info.num_affine_groups == 1
        # the fused gradient (taken when residuals and Jacobian are written
        # too), the user loss object in CameraGradientKernel's arguments
        assert info.num_fused_gradient_groups == 1, combo
        assert_parity(got, ref, (fmt, name, combo))
    got, _ = evaluate(prog, force_general_layout=True)
    assert_parity(got, oracle(prog, kmap, lmap), (fmt, name, "general"))


def test_bundler_residual_problem_13682_full_size(gpu):
    # The user functor path at BASELINE.json configs[3]'s size (28,987,644
    # residual blocks, Huber, BlockSparseMatrix): residuals + Jacobian +
    # gradient, the timed residual+Jacobian evaluation (bench.py
    # secondary.user_functor), and the residual-only evaluation.
    k = U.kind("BundlerResidual/Huber")
    prog = with_kind(bal.synthetic_program("problem-13682-4456117", loss=ca.Loss.huber(1.0)), k)
    kmap = {k: O.BUNDLER_RESIDUAL_2_9_3}
    ev = ca.Evaluator(prog)
    try:
        got = ev.evaluate(residuals=True, gradient=True, jacobian=True)
        info = ev.info()
        got_ng = ev.evaluate(residuals=True, gradient=False, jacobian=True)
        got_r = ev.evaluate(residuals=True, gradient=False, jacobian=False)
    finally:
        ev.close()
    assert info.num_affine_groups == 1 and info.num_fused_gradient_groups == 1
    ref = oracle(prog, kmap, threads=16, residuals=True, gradient=True, jacobian=True)
    rep = {}
    assert_parity(got, ref, "BundlerResidual problem-13682", report=rep)
    del got
    ok, cost, r, _, j = ref
    assert_parity(got_ng, (ok, cost, r, None, j), "no gradient")
    assert_parity(got_r, (ok, cost, r, None, None), "residual only")
    print("BundlerResidual problem-13682 Huber parity:", rep)


def test_user_kind_on_a_multi_device_evaluator(gpu):
    # cse_create_multi over a user kind: 3 shards on device 0, the strips
    # assembled into one buffer, cost and gradient summed over shards.
    k = U.kind("BundlerResidual/SoftLOne")
    cams, pts, ci, pi, obs = small(C=20, P=2000, O_=9000, seed=23)
    prog = bal.program(cams, pts, ci, pi, obs, kind=k, loss=U.soft_l_one(2.0))
    one, _ = evaluate(prog)
    ev = ca.Evaluator(prog, devices=[0, 0, 0])
    try:
        multi = ev.evaluate()
    finally:
        ev.close()
    assert np.array_equal(one[2], multi[2]) and np.array_equal(one[4], multi[4])
    assert_parity(multi, one, "multi-device user kind")


# ---- Shapes outside the library's kinds on the affine kernels --------------
# PoseReprojectionError <2, 6, 3> (six doubles of functor data),
# PointToPlaneError <1, 6, 3>, RigidAlignmentError <3, 6> (examples/
# user_functors.h): each runs the affine kernels (cse::kAffineShape) and is
# checked against the general kernel, which evaluates the same functor one
# block per lane through the offset tables -- residuals, Jacobian (both
# layouts), cost, gradient, and the Jacobian operators.

def _scene(C, P, per_point, seed):
    rng = np.random.default_rng(seed)
    poses = np.concatenate([rng.normal(0, 0.05, (C, 3)),
                            np.stack([rng.normal(0, 1, C), rng.normal(0, 1, C),
                                      -10 + rng.normal(0, 1, C)], axis=1)], axis=1)
    pts = rng.uniform(-3, 3, (P, 3))
    ci = np.concatenate([rng.permutation(C)[:per_point] for _ in range(P)]).astype(np.int32)
    pi = np.repeat(np.arange(P, dtype=np.int32), per_point)
    return rng, poses, pts, ci, pi


def _pose_point_problem(name, seed=3, C=40, P=3000, per_point=5):
    """Points first (the Schur elimination group), then poses; residual
    blocks point-major, as bundle_adjuster orders them."""
    rng, poses, pts, ci, pi = _scene(C, P, per_point, seed)
    pb = ca.ProblemCUDA()
    pid = [pb.add_parameter_block(p) for p in pts]
    cid = [pb.add_parameter_block(c) for c in poses]
    ids = np.stack([np.asarray(cid)[ci], np.asarray(pid)[pi]], axis=1)
    n = len(ci)
    if name.startswith("PoseReprojectionError"):
        # u, v from the model plus noise; fx, fy, cx, cy per observation
        intr = np.stack([rng.uniform(400, 600, n), rng.uniform(400, 600, n),
                         rng.uniform(300, 340, n), rng.uniform(220, 260, n)], axis=1)
        uv = rng.normal(320, 50, (n, 2))
        data = np.concatenate([uv, intr], axis=1)
        loss = ca.Loss.huber(1.0) if name.endswith("Huber") else None
    else:  # PointToPlaneError
        nrm = rng.normal(size=(n, 3))
        nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
        data = np.concatenate([nrm, rng.normal(0, 2, (n, 1))], axis=1)
        loss = ca.Loss.cauchy(2.0)
    pb.add_residual_blocks(U.kind(name), loss, ids, data)
    return pb, P


def _rigid_problem(seed=5, C=64, per_pose=400):
    rng = np.random.default_rng(seed)
    pb = ca.ProblemCUDA()
    poses = np.concatenate([rng.normal(0, 0.1, (C, 3)), rng.normal(0, 1, (C, 3))], axis=1)
    cid = [pb.add_parameter_block(c) for c in poses]
    n = C * per_pose
    ids = np.repeat(np.asarray(cid, np.int32), per_pose)[:, None]
    data = np.concatenate([rng.uniform(-5, 5, (n, 3)), rng.uniform(-5, 5, (n, 3))], axis=1)
    pb.add_residual_blocks(U.kind("RigidAlignmentError/Trivial"), None, ids, data)
    return pb, 0


def _close(a, b, tol=1e-13):
    return np.linalg.norm(a - b) <= tol * max(np.linalg.norm(b), 1e-300)


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
@pytest.mark.parametrize("name", ["PoseReprojectionError/Trivial", "PoseReprojectionError/Huber",
                                  "PointToPlaneError/Cauchy", "RigidAlignmentError/Trivial"])
def test_other_shapes_on_the_affine_kernels(gpu, name, fmt):
    pb, n_elim = (_rigid_problem() if name.startswith("Rigid") else _pose_point_problem(name))
    prog = pb.program()
    prog.compile(fmt, num_eliminate_blocks=n_elim if fmt == ca.BLOCK_SPARSE else 0)
    fast, info_f = evaluate(prog)
    gen, info_g = evaluate(prog, force_general_layout=True)
    assert info_f.num_affine_groups == 1 and info_g.num_affine_groups == 0, name
    # <NR, 6, 3> with points sorted: the fused gradient (data of 6 and 4
    # doubles sorted into camera order by SortSlot0InputsAnyKernel)
    assert info_f.num_fused_gradient_groups == (0 if name.startswith("Rigid") else 1), name
    assert fast[0] and gen[0]
    assert abs(fast[1] - gen[1]) <= 1e-13 * abs(gen[1]), (name, fast[1], gen[1])
    for k, what in ((2, "residuals"), (3, "gradient"), (4, "jacobian")):
        assert np.isfinite(fast[k]).all(), (name, what)
        assert _close(fast[k], gen[k]), (name, what, np.linalg.norm(fast[k] - gen[k]))
    # residual-only and cost-only kernels of the shape
    r_only, _ = evaluate(prog, residuals=True, gradient=False, jacobian=False)
    assert _close(r_only[2], gen[2]) and abs(r_only[1] - gen[1]) <= 1e-13 * abs(gen[1])
    # J x and J^T x of the affine group against the dense Jacobian
    from test_spmv_gpu import dense_jacobian
    J = dense_jacobian(prog, gen[4])
    rng = np.random.default_rng(1)
    x = rng.normal(size=prog.num_effective_parameters)
    z = rng.normal(size=prog.num_residuals)
    import torch
    dev = torch.device("cuda", 0)
    ev = ca.Evaluator(prog, stream=torch.cuda.current_stream(dev).cuda_stream)
    try:
        dj = torch.from_numpy(fast[4]).to(dev)
        dx, dz = torch.from_numpy(x).to(dev), torch.from_numpy(z).to(dev)
        y = torch.zeros(prog.num_residuals, dtype=torch.float64, device=dev)
        w = torch.zeros(prog.num_effective_parameters, dtype=torch.float64, device=dev)
        ev.evaluate()  # the operators' plans
        ev.right_multiply_device(dj.data_ptr(), dx.data_ptr(), y.data_ptr())
        ev.left_multiply_device(dj.data_ptr(), dz.data_ptr(), w.data_ptr())
        torch.cuda.synchronize(dev)
    finally:
        ev.close()
    assert _close(y.cpu().numpy(), J @ x, 1e-12), name
    assert _close(w.cpu().numpy(), J.T @ z, 1e-12), name
