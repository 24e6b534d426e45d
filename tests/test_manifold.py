"""CPU: the quaternion-manifold descriptor (CSE_MANIFOLD_QUATERNION_EUCLIDEAN,
include/cse.h) and its host-side helpers; the device parity tests are in
test_manifold_gpu.py."""
import ctypes

import numpy as np
import pytest

import ceres_amd as ca
from ceres_amd import _cse, bal
from ceres_amd.problem import quaternion_euclidean_plus_jacobian


def test_quaternion_cameras_are_unit_and_keep_the_rest():
    # AngleAxisToQuaternion (rotation.h:320-352) on the synthetic cameras.
    cams, _, _, _, _ = bal.synthetic(6, 40, 120, seed=3)
    cams[0, :3] = 0.0  # the theta == 0 branch
    q = bal.to_quaternion_cameras(cams)
    assert np.allclose((q[:, :4] ** 2).sum(1), 1.0)
    assert np.array_equal(q[0, :4], [1.0, 0.0, 0.0, 0.0])
    assert np.array_equal(q[:, 4:], cams[:, 3:9])
    # q = (cos(theta/2), sin(theta/2) axis)
    th = np.linalg.norm(cams[1:, :3], axis=1)
    assert np.allclose(q[1:, 0], np.cos(th / 2))
    assert np.allclose(q[1:, 1:4], cams[1:, :3] / th[:, None] * np.sin(th / 2)[:, None])


def test_plus_jacobian_matches_a_finite_difference_of_plus():
    """QuaternionManifold::Plus (manifold.cc:28-59) differentiated at 0 is
    the matrix quaternion_euclidean_plus_jacobian returns."""
    rng = np.random.default_rng(0)
    x = rng.normal(size=10)
    x[:4] /= np.linalg.norm(x[:4])

    def plus(x, d):
        n = np.linalg.norm(d[:3])
        out = x.copy()
        if n > 0:
            qd = np.concatenate([[np.cos(n)], np.sin(n) / n * d[:3]])
            w, a, b, c = qd
            W, X, Y, Z = x[:4]
            out[:4] = [w * W - a * X - b * Y - c * Z, w * X + a * W + b * Z - c * Y,
                       w * Y - a * Z + b * W + c * X, w * Z + a * Y - b * X + c * W]
        out[4:] = x[4:] + d[3:]
        return out

    P = quaternion_euclidean_plus_jacobian(x)
    h = 1e-7
    fd = np.stack([(plus(x, h * e) - plus(x, -h * e)) / (2 * h) for e in np.eye(9)], axis=1)
    assert P.shape == (10, 9)
    assert np.allclose(P, fd, atol=1e-8)


def test_with_explicit_manifolds_is_the_reference_form():
    prog = bal.synthetic_program((5, 60, 200), quaternion_manifold=True, seed=1)
    P = 60
    assert prog.pb_tangent[P:].tolist() == [9] * 5
    ex = prog.with_explicit_manifolds()
    assert ex.pb_manifold is None
    assert ex.num_effective_parameters == prog.num_effective_parameters
    for c in range(5):
        b = P + c
        off = int(prog.state_offset[b])
        want = quaternion_euclidean_plus_jacobian(prog.state[off:off + 10])
        got = ex.plus_jacobians[ex.pb_plus_jacobian[b]:ex.pb_plus_jacobian[b] + 90].reshape(10, 9)
        assert np.array_equal(got, want)
    assert (ex.pb_plus_jacobian[:P] == -1).all()


def _create(prog):
    L = _cse.lib()
    h = ctypes.c_void_p()
    d = prog.descriptor()
    return L.cse_create(ctypes.byref(d), None, ctypes.byref(h))


def test_malformed_manifold_blocks_are_rejected_without_a_gpu():
    # Validation precedes any HIP call.
    prog = bal.synthetic_program((4, 30, 90), quaternion_manifold=True)
    prog.pb_tangent[-1] = 10  # tangent must be size - 1
    assert _create(prog) == _cse.CSE_ERR_INVALID
    assert "quaternion manifold" in _cse.last_error()
    prog = bal.synthetic_program((4, 30, 90), quaternion_manifold=True)
    prog.pb_manifold[-1] = 7
    assert _create(prog) == _cse.CSE_ERR_INVALID
    assert "unknown manifold" in _cse.last_error()
    prog = bal.synthetic_program((4, 30, 90), quaternion_manifold=True)
    prog.pb_plus_jacobian[-1] = 0  # both forms at once
    prog.plus_jacobians = np.zeros(90)
    assert _create(prog) == _cse.CSE_ERR_INVALID


def test_problem_cuda_builder_sets_the_manifold():
    pc = ca.ProblemCUDA()
    cam = pc.add_parameter_block(np.r_[1.0, 0, 0, 0, np.zeros(6)])
    pt = pc.add_parameter_block(np.zeros(3))
    pc.set_quaternion_euclidean_manifold(cam)
    pc.add_residual_block(_cse.SNAVELY_QUATERNION_2_10_3, None, [1.0, 2.0], cam, pt)
    prog = pc.program()
    assert prog.pb_manifold.tolist() == [1, 0]
    assert prog.pb_tangent.tolist() == [9, 3]
    assert prog.num_effective_parameters == 12
