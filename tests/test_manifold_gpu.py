"""GPU: cameras on ProductManifold<QuaternionManifold, EuclideanManifold<6>>
on the affine (fast) kernels -- the problem bundle_adjuster --use_quaternions
--use_manifolds builds (examples/bundle_adjuster.cc:337-345; the reference's
mini-BA test uses the same manifold, evaluator_cuda_test.cu.cc:286).

The library takes the manifold as CSE_MANIFOLD_QUATERNION_EUCLIDEAN
(include/cse.h) and builds the plus-Jacobian in registers; the oracle takes
the reference's form, the explicit 10 x 9 matrix of every camera at the
evaluated state (Program.with_explicit_manifolds, as UpdatePlusJacobians
uploads, registered_cuda_evaluators.cc:139-160), and multiplies densely
(residual_block.cc:133-156).  Tolerances: tests/parity_util.py.

Covered: both Jacobian layouts, every loss, the three gradient modes (camera
re-evaluation, fused contributions, atomics), the table kernel on the same
descriptor (force_general_layout), the explicit-matrix descriptor on the
device, mixed groups (some cameras off the manifold: table path), the
Schur-ordered problem-13682 shape, and the multi-device evaluator.
"""
import numpy as np
import pytest

import ceres_amd as ca
from ceres_amd import _cse, bal
import oracle_py as O
from parity_util import assert_parity

pytestmark = pytest.mark.gpu


def oracle_eval(prog, threads=8, **kw):
    ex = prog.with_explicit_manifolds()
    op = O.OracleProgram.from_program(ex)
    return op.evaluate(ex.state, ex.constant_state if ex.constant_state.size else None,
                       num_threads=threads, **kw)


def gpu_eval(prog, **opts):
    ev = ca.Evaluator(prog, **opts)
    try:
        return ev.evaluate(), ev.info()
    finally:
        ev.close()


def quat_program(counts=(16, 700, 2900), loss=None, fmt=ca.BLOCK_SPARSE, seed=11):
    return bal.synthetic_program(counts, loss=loss, format=fmt, seed=seed,
                                 quaternion_manifold=True)


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
@pytest.mark.parametrize("loss", [None, ca.Loss.huber(1.0), ca.Loss.cauchy(2.0),
                                  ca.Loss.huber(3.0).scaled_by(0.5)])
def test_manifold_affine_path_matches_oracle(gpu, fmt, loss):
    prog = quat_program(loss=loss, fmt=fmt)
    assert prog.num_effective_parameters == 3 * 700 + 9 * 16
    ref = oracle_eval(prog)
    got, info = gpu_eval(prog)
    assert info.num_affine_groups == 1 and info.num_fused_gradient_groups == 1
    assert_parity(got, ref, (fmt, loss))
    # The table kernel on the same descriptor builds the same matrix.
    tab, info = gpu_eval(prog, force_general_layout=True)
    assert info.num_affine_groups == 0
    assert_parity(tab, ref, (fmt, loss, "table"))
    assert np.array_equal(got[2], tab[2])


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_manifold_every_gradient_mode(gpu, mode):
    prog = quat_program(loss=ca.Loss.huber(1.0), seed=5)
    ref = oracle_eval(prog)
    got, info = gpu_eval(prog, gradient_mode=mode)
    assert info.num_affine_groups == 1
    assert_parity(got, ref, ("gradient_mode", mode))


def test_explicit_matrix_descriptor_matches_device_built(gpu):
    """The reference's form on the device (explicit plus-Jacobians, table
    kernel) against the device-built manifold (affine kernel)."""
    prog = quat_program(loss=ca.Loss.cauchy(1.0), seed=21)
    ex = prog.with_explicit_manifolds()
    a, ia = gpu_eval(prog)
    b, ib = gpu_eval(ex)
    assert ia.num_affine_groups == 1 and ib.num_affine_groups == 0
    assert_parity(a, b, "explicit vs device-built")
    assert np.array_equal(a[2], b[2])
    # The product with the matrix equals the register form up to the sign of zeros.
    assert np.allclose(a[4], b[4], rtol=1e-13, atol=1e-300)


def test_mixed_manifold_group_takes_the_table_path(gpu):
    prog = quat_program(loss=ca.Loss.huber(1.0), seed=8)
    P = 700
    # cameras 0..7 on the manifold, 8..15 plain 10-parameter blocks
    prog.pb_manifold[P + 8:] = 0
    prog.pb_tangent[P + 8:] = 10
    prog.compile(ca.BLOCK_SPARSE, num_eliminate_blocks=P)
    ref = oracle_eval(prog)
    got, info = gpu_eval(prog)
    assert info.num_affine_groups == 0
    assert_parity(got, ref, "mixed")


def test_manifold_residual_and_cost_only(gpu):
    prog = quat_program(loss=ca.Loss.huber(1.0), seed=2)
    ref = oracle_eval(prog, residuals=True, gradient=False, jacobian=False)
    ev = ca.Evaluator(prog)
    got = ev.evaluate(residuals=True, gradient=False, jacobian=False)
    cost_only = ev.evaluate(residuals=False, gradient=False, jacobian=False)
    ev.close()
    assert_parity(got, ref, "residuals")
    assert cost_only[1] == got[1]


def test_manifold_multi_device(gpu):
    prog = quat_program(counts=(20, 3001, 21113), loss=ca.Loss.huber(1.0), seed=4)
    ref = oracle_eval(prog)
    ev = ca.Evaluator(prog, devices=[0, 0, 0])
    got = ev.evaluate()
    info = ev.info()
    ev.close()
    assert info.num_affine_groups == 1
    assert_parity(got, ref, "multi-device quaternion")


@pytest.mark.slow
@pytest.mark.timeout(900)
def test_problem_13682_quaternion_manifold(gpu):
    """BASELINE.json configs[1]'s problem-13682 with quaternion cameras on the
    manifold, Huber, BSM: the affine kernels against the oracle."""
    prog = bal.synthetic_program("problem-13682-4456117", loss=ca.Loss.huber(1.0),
                                 quaternion_manifold=True)
    got, info = gpu_eval(prog)
    assert info.num_affine_groups == 1 and info.num_fused_gradient_groups == 1
    ref = oracle_eval(prog, threads=16)
    rep = {}
    assert_parity(got, ref, "problem-13682 quaternion manifold", report=rep)
    print("problem-13682 quaternion-manifold parity:", rep)


def quaternion_plus_reference(x, delta):
    """ProductManifold<QuaternionManifold, EuclideanManifold<n>>::Plus as
    QuaternionPlusImpl (internal/ceres/manifold.cc:28-59) states it."""
    out = x.copy()
    d = delta[:3]
    m = np.abs(d).max()  # std::hypot(d0, d1, d2), libstdc++'s scaled form
    nd = m * np.sqrt(((np.abs(d) / m) ** 2).sum()) if m != 0.0 else 0.0
    if nd != 0.0:
        s = np.sin(nd) / nd
        w, a, b, c = np.cos(nd), s * d[0], s * d[1], s * d[2]
        q = x[:4]
        out[0] = w * q[0] - a * q[1] - b * q[2] - c * q[3]
        out[1] = w * q[1] + a * q[0] + b * q[3] - c * q[2]
        out[2] = w * q[2] - a * q[3] + b * q[0] + c * q[1]
        out[3] = w * q[3] + a * q[2] - b * q[1] + c * q[0]
    out[4:] = x[4:] + delta[3:]
    return out


def test_plus_on_the_quaternion_manifold(gpu):
    """cse_plus: quaternion cameras by QuaternionPlusImpl (zero rotation
    steps included), points by x + delta."""
    prog = quat_program(seed=17)
    P, C = 700, 16
    rng = np.random.default_rng(5)
    delta = rng.normal(0.0, 1e-3, prog.num_effective_parameters)
    delta[3 * P: 3 * P + 3] = 0.0  # camera 0: no rotation step
    ev = ca.Evaluator(prog)
    got = ev.plus(prog.state, delta)
    ev.close()
    want = np.empty_like(prog.state)
    want[:3 * P] = prog.state[:3 * P] + delta[:3 * P]
    for c in range(C):
        so, do = 3 * P + 10 * c, 3 * P + 9 * c
        want[so:so + 10] = quaternion_plus_reference(prog.state[so:so + 10], delta[do:do + 9])
    assert np.array_equal(got[:3 * P], want[:3 * P])
    assert np.array_equal(got[3 * P:3 * P + 10], want[3 * P:3 * P + 10])  # zero step: exact
    assert np.allclose(got, want, rtol=1e-14, atol=1e-15)


def test_quaternion_plus_tiny_and_huge_steps(gpu):
    """|delta| by the scaled hypot of the reference (std::hypot, manifold.cc:
    33-35): a rotation step of 1e-160 is not lost to underflow (it squares
    to zero), and one of 1e200 does not overflow to inf."""
    prog = quat_program(seed=3)
    P, C = 700, 16
    delta = np.zeros(prog.num_effective_parameters)
    steps = [np.array([1e-160, 0.0, 0.0]), np.array([3e-170, -4e-170, 0.0]),
             np.array([1e200, 0.0, 0.0]), np.array([0.0, 0.0, 0.0]),
             np.array([1e-310, 1e-310, 1e-310])]
    for c, st in enumerate(steps):
        delta[3 * P + 9 * c: 3 * P + 9 * c + 3] = st
    ev = ca.Evaluator(prog)
    got = ev.plus(prog.state, delta)
    ev.close()
    for c in range(len(steps)):
        so, do = 3 * P + 10 * c, 3 * P + 9 * c
        want = quaternion_plus_reference(prog.state[so:so + 10], delta[do:do + 9])
        g = got[so:so + 10]
        assert np.all(np.isfinite(g)), c
        assert np.allclose(g, want, rtol=1e-14, atol=1e-300), (c, g, want)


def test_bundle_adjuster_with_quaternion_manifolds(gpu):
    """bundle_adjuster --use_quaternions --use_manifolds: evaluations, Plus on
    the manifold and the iterative Schur solve all on the device."""
    from ceres_amd import bundle_adjuster
    c0, c1, rows = bundle_adjuster.main(["--synthetic", "problem-16-22106", "--robustify",
                                         "--use_quaternions", "--use_manifolds",
                                         "--point_sigma", "0.05", "--num_iterations", "4"])
    assert c1 < 0.9 * c0
    costs = [r[1] for r in rows] + [c1]
    assert all(b <= a for a, b in zip(costs, costs[1:]))
