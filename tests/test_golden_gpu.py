"""GPU parity against the independent golden vectors.

tests/golden/snavely_golden.json holds sympy-derived residuals and
Jacobians evaluated in mpmath at 50 digits (oracle/gen_golden.py) for
SnavelyReprojectionError<2,9,3> (both rotation branches), the
no-distortion <2,7,3> and quaternion <2,10,3> variants, each under
Trivial/Huber/Cauchy losses with the Triggs correction.  This test runs
every (case, loss) pair as one residual block of one Program through the C
ABI (libcse.so, HIP) and checks it with the same tolerances the oracle is
pinned with (tests/test_oracle_golden.py): per-vector isApprox 1e-13
(evaluator_cuda_test.cu.cc:61,426-440); r = predicted - observed is
compared relative to |observed| because of its cancellation, and a
robust-loss-corrected Jacobian inherits that error (10x).
"""
import json
import os

import numpy as np
import pytest

import ceres_amd as ca

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "snavely_golden.json")
TOL = 1e-13


def _loss(kind, a):
    return {0: ca.Loss.trivial(), 1: ca.Loss.huber(a), 2: ca.Loss.cauchy(a)}[kind]


def _program(cases, fmt):
    p = ca.ProblemCUDA()
    rows = []
    for case in cases:
        for L in case["losses"]:
            c = p.add_parameter_block(case["camera"])
            x = p.add_parameter_block(case["point"])
            p.add_residual_block(case["functor"], _loss(L["loss"], L["a"]), case["obs"], c, x)
            rows.append((case, L))
    prog = p.program()
    prog.compile(fmt)
    return prog, rows


def _check(rows, r, g, j, cost, fmt):
    joff = goff = 0
    total = 0.0
    for k, (case, L) in enumerate(rows):
        n = len(case["camera"]) + 3
        obs = np.linalg.norm(case["obs"])
        scale = np.linalg.norm(L["residuals"]) / max(np.linalg.norm(case["residuals"]), 1e-300)
        pred = obs * max(scale, 1e-300)
        rk = r[2 * k:2 * k + 2]
        assert np.linalg.norm(rk - L["residuals"]) <= TOL * pred + TOL * np.linalg.norm(
            L["residuals"]), (k, case["functor"], L["loss"])
        Jexp = np.array(L["jacobian"])
        if fmt == ca.COMPRESSED_ROW:
            Jk = j[joff:joff + 2 * n].reshape(2, n)   # one row, columns by index
        else:
            # BlockJacobianWriter without elimination groups: a 2 x camera
            # cell then a 2 x 3 point cell, each row-major.
            nc = n - 3
            Jk = np.hstack([j[joff:joff + 2 * nc].reshape(2, nc),
                            j[joff + 2 * nc:joff + 2 * n].reshape(2, 3)])
        tol = TOL if L["loss"] == 0 else 10 * TOL
        assert np.linalg.norm(Jk - Jexp) <= tol * min(np.linalg.norm(Jk), np.linalg.norm(Jexp)), \
            (k, case["functor"], L["loss"])
        gk = g[goff:goff + n]
        assert np.linalg.norm(gk - Jexp.T @ np.array(L["residuals"])) <= \
            TOL * np.linalg.norm(Jexp) * pred
        joff += 2 * n
        goff += n
        total += L["cost"]
    assert abs(cost - total) <= 1e-12 * abs(total)


def _theta2(case):
    # angle-axis functors only (the quaternion kind has 10 camera values)
    cam = case["camera"]
    return sum(v * v for v in cam[:3]) if len(cam) in (7, 9) else 0.0


@pytest.mark.parametrize("fmt", [ca.COMPRESSED_ROW, ca.BLOCK_SPARSE])
@pytest.mark.parametrize("angles", ["all", "small", "large"])
def test_golden_vectors_on_gpu(gpu, fmt, angles):
    # "small" keeps the cases with theta^2 <= 1 (every wave takes the series
    # form of AngleAxisRotatePoint), "large" those with theta^2 > 1 (the
    # reference's form); "all" mixes them in one wave.
    with open(GOLDEN) as fh:
        cases = json.load(fh)["cases"]
    if angles == "small":
        cases = [c for c in cases if _theta2(c) <= 1.0]
    elif angles == "large":
        cases = [c for c in cases if _theta2(c) > 1.0]
    assert cases
    prog, rows = _program(cases, fmt)
    ev = ca.Evaluator(prog)
    try:
        ok, cost, r, g, j = ev.evaluate()
    finally:
        ev.close()
    assert ok
    _check(rows, r, g, j, cost, fmt)
