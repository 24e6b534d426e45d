"""GPU: evaluating at the same point (CSE_EVAL_SAME_POINT).

Ceres passes Evaluator::EvaluateOptions::new_evaluation_point = false when the
state equals the previous evaluation's (internal/ceres/evaluator.h:106-107):
TrustRegionMinimizer::HandleSuccessfulStep evaluates the Jacobian at the
candidate whose cost it has just evaluated (trust_region_minimizer.cc:822-826).
cse_evaluate_ex / cse_evaluate_device_ex then reuse the state already on the
device and the repacked slot-0 table instead of rebuilding them.  The outputs
must be bit-identical to a fresh evaluation at that point.
"""
import ctypes as C

import numpy as np
import pytest
import torch

import ceres_amd as ca
from ceres_amd import _cse, bal
import oracle_py as O
from parity_util import assert_parity

pytestmark = pytest.mark.gpu


def _same(a, b):
    assert a[0] == b[0] and a[1] == b[1]
    for x, y in zip(a[2:], b[2:]):
        assert (x is None) == (y is None)
        if x is not None:
            assert np.array_equal(x, y)


def _copy(out):
    return tuple(x.copy() if isinstance(x, np.ndarray) else x for x in out)


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
def test_host_path_same_point_is_bit_identical(gpu, fmt):
    prog = bal.synthetic_program((24, 3001, 20011), loss=ca.Loss.huber(1.0), format=fmt, seed=5)
    x = prog.state.copy()
    y = x + 1e-4 * np.random.default_rng(5).standard_normal(x.size)
    ev = ca.Evaluator(prog)
    try:
        fresh_y = _copy(ev.evaluate(y))
        ev.evaluate(x, residuals=True, gradient=False, jacobian=False)  # candidate at x
        # The Jacobian at x, from another buffer holding the same values.
        same = _copy(ev.evaluate(x.copy(), new_evaluation_point=False))
        fresh_x = _copy(ev.evaluate(x))
        _same(same, fresh_x)
        # The flag really reuses the uploaded state: handed y's buffer with
        # the flag, the evaluator still evaluates at x.
        stale = _copy(ev.evaluate(y, new_evaluation_point=False))
        _same(stale, fresh_x)
        again_y = _copy(ev.evaluate(y))
        _same(again_y, fresh_y)
    finally:
        ev.close()
    ref = O.OracleProgram.from_program(prog).evaluate(x, None, num_threads=8)
    assert_parity(same, ref, ("same point", fmt))


def test_device_path_same_point_skips_the_repack(gpu):
    prog = bal.synthetic_program((20, 2000, 12007), loss=ca.Loss.cauchy(2.0), seed=9)
    dev = torch.device("cuda", 0)
    f64 = torch.float64
    ev = ca.Evaluator(prog, device=0, stream=torch.cuda.current_stream(dev).cuda_stream)
    try:
        assert ev.info().num_affine_groups == 1
        x = torch.from_numpy(prog.state).to(dev)
        x2 = x.clone()
        cost = torch.zeros(1, dtype=f64, device=dev)
        r = torch.empty(prog.num_residuals, dtype=f64, device=dev)
        j = torch.empty(prog.num_jacobian_values, dtype=f64, device=dev)
        g = torch.empty(prog.num_effective_parameters, dtype=f64, device=dev)

        def run(state, new_point, residuals=True, jacobian=True, gradient=True):
            ev.evaluate_device(state.data_ptr(), cost.data_ptr(), r.data_ptr() if residuals else None,
                               g.data_ptr() if gradient else None, j.data_ptr() if jacobian else None,
                               new_evaluation_point=new_point)
            assert ev.wait() == 0
            return (True, float(cost.item()), r.cpu().numpy(), g.cpu().numpy(), j.cpu().numpy())

        fresh = run(x, True)
        run(x, True, jacobian=False, gradient=False)  # the candidate evaluation
        same = run(x2, False)  # another buffer, same values
        _same(same, fresh)
        # A first evaluation with the flag has nothing to reuse: it repacks.
        ev2 = ca.Evaluator(prog, device=0, stream=torch.cuda.current_stream(dev).cuda_stream)
        c2 = torch.zeros(1, dtype=f64, device=dev)
        ev2.evaluate_device(x.data_ptr(), c2.data_ptr(), new_evaluation_point=False)
        assert ev2.wait() == 0
        first = float(c2.item())
        ev2.evaluate_device(x.data_ptr(), c2.data_ptr())
        assert ev2.wait() == 0
        assert first == float(c2.item()) and np.isfinite(first)
        ev2.close()
    finally:
        ev.close()


def test_multi_device_same_point(gpu):
    prog = bal.synthetic_program((16, 1500, 9001), loss=ca.Loss.huber(1.0), seed=3)
    ev = ca.Evaluator(prog, devices=[0, 0, 0])
    try:
        x = prog.state.copy()
        fresh = _copy(ev.evaluate(x))
        same = _copy(ev.evaluate(x.copy(), new_evaluation_point=False))
        _same(same, fresh)
    finally:
        ev.close()


def test_unknown_flags_are_rejected(gpu):
    prog = bal.synthetic_program((4, 100, 400), seed=1)
    ev = ca.Evaluator(prog)
    try:
        cost = C.c_double(0.0)
        st = np.ascontiguousarray(prog.state)
        rc = _cse.lib().cse_evaluate_ex(ev.handle, st.ctypes.data_as(C.POINTER(C.c_double)),
                                        C.byref(cost), None, None, None, 6)
        assert rc == _cse.CSE_ERR_INVALID
        rc = _cse.lib().cse_evaluate_device_ex(ev.handle, 1, 1, None, None, None, 2)
        assert rc == _cse.CSE_ERR_INVALID
    finally:
        ev.close()
