"""Pins the CPU oracle against independent golden vectors and the
reference's own known-answer tests.

* tests/golden/snavely_golden.json: sympy-derived Jacobians evaluated in
  mpmath at 50 digits (oracle/gen_golden.py) for SnavelyReprojectionError,
  the no-distortion and quaternion variants, and Trivial/Huber/Cauchy losses
  with the Triggs correction.  Tolerance: the reference's own
  ||x - x_ref|| <= 1e-13 * min(||x||, ||x_ref||) (Eigen isApprox,
  internal/ceres/evaluator_cuda_test.cu.cc:61,426-440).
* corrector_test.cc, loss_function_test.cc, rotation_test.cc known answers.
"""
import json
import math
import os

import numpy as np
import pytest

import oracle_py as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "snavely_golden.json")
TOL = 1e-13


def is_approx(x, y, tol=TOL):
    x, y = np.ravel(x), np.ravel(y)
    return np.linalg.norm(x - y) <= tol * min(np.linalg.norm(x), np.linalg.norm(y))


def residuals_close(r, r_exact, obs, tol=TOL):
    """r = predicted - observed cancels: an fp64 evaluation is accurate to
    eps * |predicted|, not eps * |r|, so the exact-value comparison scales
    the tolerance by the prediction's magnitude (scaled like r_exact by any
    loss correction)."""
    r, r_exact = np.ravel(r), np.ravel(r_exact)
    return np.linalg.norm(r - r_exact) <= tol * np.linalg.norm(obs) + tol * np.linalg.norm(r_exact)


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as fh:
        return json.load(fh)["cases"]


def _single_block_program(case, loss_kind, a):
    cam = np.array(case["camera"])
    kind = case["functor"]
    return O.OracleProgram(
        pb_size=[cam.size, 3], pb_tangent=[cam.size, 3], pb_constant=[0, 0],
        pb_plus_jacobian=[-1, -1], plus_jacobians=[0.0], rb_kind=[kind],
        rb_loss_kind=[loss_kind], rb_loss_a=[a], rb_loss_scale=[1.0], rb_loss_scaled=[0],
        rb_param_begin=[0, 2], rb_params=[0, 1], rb_data_begin=[0, 2], rb_data=case["obs"],
        jacobian_format=O.COMPRESSED_ROW, num_eliminate_blocks=0)


def test_golden_autodiff(golden):
    for case in golden:
        cam = np.array(case["camera"])
        ok, r, (Jc, Jp) = O.autodiff(case["functor"], case["obs"], [cam, case["point"]], 2,
                                     [cam.size, 3])
        assert ok
        J = np.hstack([Jc, Jp])
        assert residuals_close(r, case["residuals"], case["obs"]), case
        assert is_approx(J, case["jacobian"]), case


def test_golden_residual_block_with_losses(golden):
    for case in golden:
        cam = np.array(case["camera"])
        state = np.concatenate([cam, case["point"]])
        for L in case["losses"]:
            prog = _single_block_program(case, L["loss"], L["a"])
            ok, cost, r, g, j = prog.evaluate(state)
            assert ok
            scale = np.linalg.norm(L["residuals"]) / max(np.linalg.norm(case["residuals"]), 1e-300)
            pred = np.linalg.norm(case["obs"]) * max(scale, 1e-300)
            assert abs(cost - L["cost"]) <= 1e-13 * pred * np.linalg.norm(L["residuals"]) + \
                1e-13 * abs(L["cost"]), (case["functor"], L)
            assert residuals_close(r, L["residuals"], pred)
            # CRS row: columns sorted by parameter index = camera then point.
            # A robust loss scales J by sqrt(rho'(|r|^2)), which inherits the
            # cancellation error of r: 10x the plain tolerance there.
            assert is_approx(j.reshape(2, -1), L["jacobian"], TOL if L["loss"] == 0 else 10 * TOL)
            Jexp = np.array(L["jacobian"])
            g_exp = Jexp.T @ np.array(L["residuals"])
            assert np.linalg.norm(g - g_exp) <= 1e-13 * np.linalg.norm(Jexp) * pred


def test_golden_covers_both_rotation_branches_and_huber_regions(golden):
    zero = [c for c in golden if c["functor"] == 0 and not any(c["camera"][:3])]
    assert len(zero) >= 3
    huber = [(c["losses"][1]["residuals"], c["residuals"]) for c in golden]
    inlier = sum(1 for rc, r in huber if np.allclose(rc, r, rtol=0, atol=0))
    assert 0 < inlier < len(golden)


def test_corrector_known_answers():
    # internal/ceres/corrector_test.cc:56-135
    r0, j0 = math.sqrt(3.0), 10.0
    for rho in ([3.0, 0.1, -0.01], [3, 0.1, -0.1]):
        r, J = O.corrector(r0 * r0, rho, [r0], [[j0]])
        assert abs(r[0] - r0 * math.sqrt(rho[1])) < 1e-12
        assert abs(J[0, 0] - math.sqrt(rho[1]) * j0) < 1e-12
    r, J = O.corrector(0.0, [0.0, 0.1, -0.01], [0.0], [[10.0]])
    assert r[0] == 0.0 and abs(J[0, 0] - math.sqrt(0.1) * 10.0) < 1e-12


def test_corrector_gauss_newton_approximation():
    # corrector_test.cc:140-200: with rho'' > 0 the corrected normal
    # equations equal the robustified Gauss-Newton approximation
    # J^T (rho' + 2 rho'' r r^T) J and gradient rho' J^T r.
    rng = np.random.default_rng(5)
    for _ in range(10):
        r = rng.normal(size=3)
        J = rng.normal(size=(3, 4))
        sq = float(r @ r)
        rho = [sq, 0.1, 1.0 / sq / 10]
        rc, Jc = O.corrector(sq, rho, r, J)
        g_exp = rho[1] * J.T @ r
        H_exp = J.T @ (rho[1] * np.eye(3) + 2 * rho[2] * np.outer(r, r)) @ J
        assert np.allclose(Jc.T @ rc, g_exp, rtol=1e-10, atol=1e-12)
        assert np.allclose(Jc.T @ Jc, H_exp, rtol=1e-10, atol=1e-12)


def _fd_check(kind, a, s, scaled=False, scale=1.0):
    # loss_function_test.cc:45-74 (AssertLossFunctionIsValid)
    h = 1e-4
    rho = O.loss(kind, a, s, scaled, scale)
    fwd = O.loss(kind, a, s + h, scaled, scale)
    bwd = O.loss(kind, a, s - h, scaled, scale)
    assert abs((fwd[0] - bwd[0]) / (2 * h) - rho[1]) < 1e-6
    assert abs((fwd[0] - 2 * rho[0] + bwd[0]) / (h * h) - rho[2]) < 1e-6


def test_loss_functions_known_answers():
    for s in (0.357, 1.792):
        _fd_check(0, 1.0, s)
        for a in (0.7, 1.3):
            _fd_check(1, a, s)
            _fd_check(2, a, s)
            _fd_check(1, a, s, True, 10.0)   # ScaledLoss (loss_function_test.cc:193-234)
            _fd_check(2, a, s, True, 10.0)
    assert list(O.loss(0, 1.0, 0.0)) == [0.0, 1.0, 0.0]
    # Huber inlier region is the identity.
    assert list(O.loss(1, 2.0, 3.0)) == [3.0, 1.0, 0.0]


def test_rotation_known_answers():
    # rotation_test.cc: zero rotation is the identity; a rotation of pi/2
    # about z maps x to y; tiny angles agree with R = I + hat(w).
    pt = np.array([1.0, 2.0, 3.0])
    assert np.array_equal(O.angle_axis_rotate_point([0, 0, 0], pt), pt)
    out = O.angle_axis_rotate_point([0, 0, math.pi / 2], [1.0, 0, 0])
    assert np.allclose(out, [0, 1, 0], atol=1e-15)
    w = np.array([1e-20, -2e-20, 3e-20])
    assert np.allclose(O.angle_axis_rotate_point(w, pt), pt + np.cross(w, pt), rtol=1e-15)
    q = np.array([math.cos(math.pi / 4), 0, 0, math.sin(math.pi / 4)]) * 3.0
    assert np.allclose(O.quaternion_rotate_point(q, [1.0, 0, 0]), [0, 1, 0], atol=1e-15)


def test_jet_ops_known_answers():
    # jet_test.cc / jet_cuda_test.cu.cc: chain rule of the elementary ops.
    x = np.array([0.7, 1.0, 2.0, -1.0])
    y = np.array([-1.3, 0.5, 0.0, 3.0])
    z = np.array([2.2, 0.0, 1.0, 1.0])
    assert np.allclose(O.jet_op(0, x), [math.sin(0.7), *(math.cos(0.7) * x[1:])], rtol=1e-15)
    assert np.allclose(O.jet_op(1, x), [math.cos(0.7), *(-math.sin(0.7) * x[1:])], rtol=1e-15)
    assert np.allclose(O.jet_op(2, x), [math.sqrt(0.7), *(x[1:] / (2 * math.sqrt(0.7)))],
                       rtol=1e-15)
    hv = math.sqrt(0.7 ** 2 + 1.3 ** 2 + 2.2 ** 2)
    exp = [hv, *((0.7 * x[1:] - 1.3 * y[1:] + 2.2 * z[1:]) / hv)]
    assert np.allclose(O.jet_op(3, x, y, z), exp, rtol=1e-15)
    assert np.allclose(O.jet_op(4, y), [1.3, *(-y[1:])], rtol=1e-15)
    q = 0.7 / -1.3
    assert np.allclose(O.jet_op(5, x, y), [q, *((x[1:] - q * y[1:]) / -1.3)], rtol=1e-15)
    assert np.allclose(O.jet_op(6, x, y), [0.7 * -1.3, *(0.7 * y[1:] + x[1:] * -1.3)],
                       rtol=1e-15)
