"""Shared helpers for the GPU-vs-oracle parity tests.

Tolerance (stated once, used everywhere): the reference's own parity
criterion between its CPU and CUDA evaluators, Eigen isApprox with
kTolerance = 1e-13 per output vector
(internal/ceres/evaluator_cuda_test.cu.cc:61,426-440):
    ||x - x_ref|| <= 1e-13 * min(||x||, ||x_ref||)
and for the scalar cost |cost - cost_ref| <= 1e-12 * |cost_ref| (the
reference uses EXPECT_NEAR 1e-13 absolute on a 6-block problem; summing
millions of blocks in a different order needs a relative bound).
"""
import numpy as np

TOL = 1e-13
COST_RTOL = 1e-12


def is_approx(x, y, tol=TOL):
    x, y = np.ravel(x), np.ravel(y)
    nx, ny = np.linalg.norm(x), np.linalg.norm(y)
    if nx == 0 and ny == 0:
        return True
    return np.linalg.norm(x - y) <= tol * min(nx, ny)


def max_rel_err(x, y, floor=1e-8):
    x, y = np.ravel(x), np.ravel(y)
    m = np.abs(y) > floor
    if not m.any():
        return 0.0
    return float(np.max(np.abs(x[m] - y[m]) / np.abs(y[m])))


# Per-element bound, on top of the norm-wise one (a norm over millions of
# values dilutes a few bad elements by sqrt(n)):
#     |x_i - y_i| <= ELEM_RTOL * |y_i| + ELEM_ATOL * max_j |y_j|
# The absolute term covers entries that are small by cancellation (r =
# predicted - observed; Jacobian entries that are sums of terms of both
# signs), where FMA contraction and device-vs-libm sin/cos (1 ulp) move the
# last bits of the operands.
ELEM_RTOL = 1e-10
ELEM_ATOL = 1e-13


def elementwise_report(x, y):
    """max relative error over elements above 1e-6 * max|y|, max absolute
    error over max|y|, and the worst ratio to the per-element bound."""
    x, y = np.ravel(x), np.ravel(y)
    if y.size == 0:
        return {"max_rel_err": 0.0, "max_abs_err_over_max": 0.0, "bound_ratio": 0.0}
    ymax = float(np.max(np.abs(y)))
    d = np.abs(x - y)
    m = np.abs(y) > 1e-6 * ymax
    rel = float(np.max(d[m] / np.abs(y[m]))) if m.any() else 0.0
    bound = ELEM_RTOL * np.abs(y) + ELEM_ATOL * ymax
    ratio = float(np.max(d / np.where(bound > 0, bound, 1e-300)))
    return {"max_rel_err": rel, "max_abs_err_over_max": float(d.max()) / ymax if ymax else 0.0,
            "bound_ratio": ratio}


def assert_parity(gpu, ref, what="", report=None):
    """Norm-wise (the reference's isApprox) and per-element parity.  If
    `report` is a dict, it receives each output's elementwise_report."""
    ok_g, cost_g, r_g, g_g, j_g = gpu
    ok_r, cost_r, r_r, g_r, j_r = ref
    assert ok_g == ok_r, (what, ok_g, ok_r)
    if not ok_r:
        return
    assert abs(cost_g - cost_r) <= COST_RTOL * abs(cost_r) + 1e-300, (what, cost_g, cost_r)
    if report is not None:
        report["cost_rel_err"] = abs(cost_g - cost_r) / abs(cost_r) if cost_r else 0.0
    for name, a, b in (("residuals", r_g, r_r), ("gradient", g_g, g_r), ("jacobian", j_g, j_r)):
        if b is None:
            continue
        assert a is not None
        assert a.shape == b.shape, (what, name)
        assert np.isfinite(a).all(), (what, name)
        assert is_approx(a, b), (what, name, np.linalg.norm(a - b) / np.linalg.norm(b),
                                 max_rel_err(a, b))
        rep = elementwise_report(a, b)
        if report is not None:
            report[name] = rep
        assert rep["bound_ratio"] <= 1.0, (what, name, "per-element bound", rep)
