"""The group-store kernel (csrc/group_store_kernel.hpp,
EvaluateAffineChunksGroupStore): four waves per workgroup over four
consecutive 64-block chunks, the workgroup's F cells, E cells and residuals
stored as long runs from one LDS image.  It runs for the Snavely BSM
residual+Jacobian evaluation when the residual, E and F bases sit on
64-byte sectors; the last, partial workgroup takes the slow tail per wave;
anything unaligned takes the one-wave kernel (EvaluateAffineChunksTwoRoundW1).

Checked here, against the oracle (the reference's tolerance,
tests/parity_util.py) and bit for bit against the table path
(force_general_layout, the same arithmetic through per-lane stores) and
against the one-wave kernel (the same device buffers shifted by 8 bytes, so
GroupStoreEligible fails):
  * block counts around every workgroup boundary (4, 60, 64, 68, 252, 256,
    260, ... blocks: 1 to 4 chunks in the last workgroup, ragged chunks);
  * every loss the kernel is instantiated for;
  * gradient_mode 2 (FP64 atomics in the kernel, as the reference's
    cuda_evaluator_kernel.h:149-160).
"""
import numpy as np
import pytest

import ceres_amd as ca
from ceres_amd import bal
import oracle_py as O
from parity_util import assert_parity

pytestmark = pytest.mark.gpu

# Workgroup = 4 chunks = 256 blocks.  The F cells start at 6 * O doubles,
# on a 64-byte sector when O % 4 == 0: those sizes take the group-store
# kernel (1 to 4 chunks in the last workgroup, ragged last chunks); the
# others the one-wave kernel, checked alike.
SIZES = [4, 60, 64, 68, 252, 256, 260, 512, 700, 1028, 1412, 1, 63, 65, 257]
LOSSES = [None, ca.Loss.huber(1.0), ca.Loss.cauchy(2.0)]


def _prog(n, loss, seed=11):
    cams = max(6, min(40, n // 8 + 2))
    pts = max(1, min(n, n // 5 + 1))
    return bal.synthetic_program((cams, pts, n), loss=loss, format=ca.BLOCK_SPARSE, seed=seed)


def _oracle(prog):
    op = O.OracleProgram.from_program(prog, apply_loss_function=True)
    return op.evaluate(prog.state, None, num_threads=8)


def _no_grad(out):
    ok, cost, r, _, j = out
    return ok, cost, r, None, j


def _device_eval(ev, prog, shift_doubles):
    """residuals + Jacobian into device buffers whose first element sits
    shift_doubles * 8 bytes past a 256-byte-aligned allocation."""
    import torch
    dev = torch.device("cuda", 0)
    s = shift_doubles
    state = torch.from_numpy(prog.state).to(dev)
    cost = torch.zeros(1, dtype=torch.float64, device=dev)
    res = torch.full((prog.num_residuals + s,), np.nan, dtype=torch.float64, device=dev)
    jac = torch.full((prog.num_jacobian_values + s,), np.nan, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    ev.evaluate_device(state.data_ptr(), cost.data_ptr(), res[s:].data_ptr(), None,
                       jac[s:].data_ptr())
    assert ev.wait() == 0
    return True, float(cost.item()), res[s:].cpu().numpy(), None, jac[s:].cpu().numpy()


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("loss", LOSSES, ids=["none", "huber", "cauchy"])
def test_group_store_sizes_against_oracle_and_table_path(gpu, n, loss):
    prog = _prog(n, loss)
    ref = _no_grad(_oracle(prog))
    ev = ca.Evaluator(prog)
    try:
        got = ev.evaluate(residuals=True, gradient=False, jacobian=True)
        assert ev.info().num_affine_groups == 1
    finally:
        ev.close()
    assert_parity(_no_grad(got), ref, ("group store", n))
    ev = ca.Evaluator(prog, force_general_layout=True)
    try:
        gen = ev.evaluate(residuals=True, gradient=False, jacobian=True)
        assert ev.info().num_affine_groups == 0
    finally:
        ev.close()
    assert np.array_equal(got[2], gen[2]), n
    assert np.array_equal(got[4], gen[4]), n
    assert got[1] == gen[1], n


@pytest.mark.parametrize("n", [260, 1028, 4096 + 76])
def test_group_store_bit_identical_to_the_one_wave_kernel(gpu, n):
    """The same device outputs at a 64-byte-aligned base (group store), 8
    bytes further (the one-wave kernel's sector-window tail) and 64 bytes
    further (group store again): equal bits, every output written."""
    prog = _prog(n, ca.Loss.huber(1.0))
    ref = _no_grad(_oracle(prog))
    ev = ca.Evaluator(prog, device=0)
    try:
        a = _device_eval(ev, prog, 0)
        b = _device_eval(ev, prog, 1)
        c = _device_eval(ev, prog, 8)  # 64 bytes: aligned again
    finally:
        ev.close()
    assert_parity(a, ref, ("aligned", n))
    for other in (b, c):
        assert np.array_equal(a[2], other[2])
        assert np.array_equal(a[4], other[4])
        assert a[1] == other[1]
    assert not np.isnan(a[4]).any() and not np.isnan(a[2]).any()


@pytest.mark.parametrize("n", [68, 1028])
def test_group_store_gradient_mode_2_atomics(gpu, n):
    """gradient_mode 2: the kernel adds J^T r with FP64 atomics, as the
    reference does; the gradient matches the oracle, the residuals and
    Jacobian are the no-gradient evaluation's bits."""
    prog = _prog(n, ca.Loss.huber(1.0))
    ref = _oracle(prog)
    ev = ca.Evaluator(prog, gradient_mode=2)
    try:
        got = ev.evaluate(residuals=True, gradient=True, jacobian=True)
        plain = ev.evaluate(residuals=True, gradient=False, jacobian=True)
    finally:
        ev.close()
    assert_parity(got, ref, ("mode 2", n))
    assert np.array_equal(got[2], plain[2])
    assert np.array_equal(got[4], plain[4])
