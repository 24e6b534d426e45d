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
    assert info.num_affine_groups == 1
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
