"""GPU parity of the gradient g = J^T r in its three forms (cse.h
cse_options.gradient_mode), against the CPU oracle's ProgramEvaluator
gradient (program_evaluator.h:134-290; the reference GPU kernel adds it with
atomics, cuda_evaluator_kernel.h:149-160):
  0  fused into the evaluation (cse::FusedGrad): slot-1 runs reduced in the
     wave, slot-0 rows by re-evaluation in camera order
     (cse::CameraGradientKernel);
  1  the fixed-order post-pass over the written Jacobian;
  2  in-kernel FP64 atomics;
  3  fused, slot-0 per-block contributions written in block order and summed
     in camera order (GradientContribKernel).
Modes 0, 1 and 3 are bit-deterministic; all three agree with the oracle to the
reference's tolerance (parity_util).  Cases cover the fused path's wave
boundaries: points whose runs span several waves, one-run waves, ragged
last chunks (down to one block), both Jacobian layouts and the losses.
"""
import numpy as np
import pytest

import ceres_amd as ca
from ceres_amd import bal
import oracle_py as O
from parity_util import assert_parity, is_approx

pytestmark = pytest.mark.gpu


def oracle_eval(prog, threads=8):
    op = O.OracleProgram.from_program(prog)
    return op.evaluate(prog.state, prog.constant_state if prog.constant_state.size else None,
                       num_threads=threads)


def run(prog, mode, repeat=1):
    ev = ca.Evaluator(prog, gradient_mode=mode)
    try:
        outs = [ev.evaluate() for _ in range(repeat)]
        return outs, ev.info()
    finally:
        ev.close()


def check_modes(prog):
    ref = oracle_eval(prog)
    (f0, f1), info = run(prog, 0, repeat=2)
    # Eligible: slot-1 ids sorted (always, point-major), slot-0 ids not
    # (a sorted slot 0 takes the post-pass's identity order instead).
    cams = prog.groups[0].ids[:, 0]
    assert info.num_fused_gradient_groups == (0 if np.all(np.diff(cams) >= 0) else 1)
    assert_parity(f0, ref, "fused")
    assert np.array_equal(f0[3], f1[3])  # deterministic
    (c0, c1), info_c = run(prog, 3, repeat=2)
    assert info_c.num_fused_gradient_groups == info.num_fused_gradient_groups
    assert_parity(c0, ref, "fused, contributions")
    assert np.array_equal(c0[3], c1[3])  # deterministic
    assert np.array_equal(f0[2], c0[2]) and np.array_equal(f0[4], c0[4]) and f0[1] == c0[1]
    assert is_approx(f0[3], c0[3], 1e-13)
    (p,), info_p = run(prog, 1)
    assert info_p.num_fused_gradient_groups == 0
    assert_parity(p, ref, "post-pass")
    (a,), _ = run(prog, 2)
    assert_parity(a, ref, "atomics")
    # Same residuals and Jacobian whatever the gradient mode; the gradients
    # agree to the tolerance (different summation orders).
    assert np.array_equal(f0[2], p[2]) and np.array_equal(f0[4], p[4])
    assert f0[1] == p[1]
    assert is_approx(f0[3], p[3], 1e-13)
    assert is_approx(f0[3], a[3], 1e-13)
    return f0


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
@pytest.mark.parametrize("loss", [None, ca.Loss.huber(1.0), ca.Loss.cauchy(2.0)])
def test_fused_gradient_matches_oracle(gpu, fmt, loss):
    prog = bal.synthetic_program((24, 3000, 20000), loss=loss, format=fmt, seed=11)
    check_modes(prog)


@pytest.mark.parametrize("n_obs", [4000, 4001, 4033, 4097])
def test_fused_gradient_runs_spanning_waves(gpu, n_obs):
    # 20 points seen by ~200 cameras each: every point's run covers several
    # whole waves (one-run waves), and 4097 = 64 * 64 + 1 leaves a last
    # chunk of one block.
    prog = bal.synthetic_program((210, 20, n_obs), loss=ca.Loss.huber(1.0), seed=n_obs)
    check_modes(prog)


@pytest.mark.parametrize("n_obs", [1, 2, 63, 64, 65, 130, 1000])
def test_fused_gradient_ragged(gpu, n_obs):
    prog = bal.synthetic_program((5, max(1, n_obs // 3), n_obs), loss=ca.Loss.huber(1.0),
                                 seed=n_obs)
    check_modes(prog)


def test_fused_gradient_needs_exclusive_points(gpu):
    # Two groups over the same points: the fused kernel stores point rows
    # (it does not add), so neither group may take it; the result is still
    # the oracle's.
    prog = bal.synthetic_program((20, 800, 3000), seed=3)
    g = prog.groups[0]
    half = g.n // 2
    idx = np.arange(g.n)
    prog.groups = [
        ca.ResidualGroup(g.kind, ca.Loss.huber(1.0), g.ids[:half], g.data[:half],
                         idx[:half].astype(np.int64)),
        ca.ResidualGroup(g.kind, ca.Loss.huber(1.0), g.ids[half:], g.data[half:],
                         idx[half:].astype(np.int64)),
    ]
    prog.compile(ca.BLOCK_SPARSE, num_eliminate_blocks=800)
    ref = oracle_eval(prog)
    (got,), info = run(prog, 0)
    assert info.num_groups == 2
    # A point seen by blocks on both sides of the split is shared.
    shared = set(g.ids[:half, 1]) & set(g.ids[half:, 1])
    if shared:
        assert info.num_fused_gradient_groups == 0
    assert_parity(got, ref, "two groups")


def _device_gradient(prog, fill=np.nan):
    """residuals + gradient + Jacobian through the device entry point, the
    gradient buffer filled with `fill` first (gradient_mode 0)."""
    import torch
    dev = torch.device("cuda", 0)
    ev = ca.Evaluator(prog, device=0)
    try:
        state = torch.from_numpy(prog.state).to(dev)
        cost = torch.zeros(1, dtype=torch.float64, device=dev)
        res = torch.empty(prog.num_residuals, dtype=torch.float64, device=dev)
        grad = torch.full((prog.num_effective_parameters,), fill, dtype=torch.float64, device=dev)
        jac = torch.empty(prog.num_jacobian_values, dtype=torch.float64, device=dev)
        torch.cuda.synchronize()
        ev.evaluate_device(state.data_ptr(), cost.data_ptr(), res.data_ptr(), grad.data_ptr(),
                           jac.data_ptr())
        assert ev.wait() == 0
        return (True, float(cost.item()), res.cpu().numpy(), grad.cpu().numpy(),
                jac.cpu().numpy()), ev.info()
    finally:
        ev.close()


def test_gradient_rows_written_once_into_a_dirty_buffer(gpu):
    """Every camera and point observed (Group::grad_exact): the fused
    gradient writes each row exactly once and the buffer is not zeroed
    first (CSE_GRAD_ASSIGN) -- a NaN-filled buffer comes back complete."""
    prog = bal.synthetic_program((24, 3000, 20000), loss=ca.Loss.huber(1.0), seed=11)
    assert len(np.unique(prog.groups[0].ids[:, 0])) == 24
    got, info = _device_gradient(prog)
    assert info.num_fused_gradient_groups == 1
    assert_parity(got, oracle_eval(prog), "assigned rows")


@pytest.mark.parametrize("drop_cams,drop_pts", [((7,), (100,)), ((23,), ()), ((0,), (0, 2999))])
def test_gradient_with_unobserved_parameter_blocks(gpu, drop_cams, drop_pts):
    """Cameras or points that no residual block uses (inside the id ranges
    or at their ends): their gradient rows are zero, so the buffer is zeroed
    first (grad_exact false) and the rest added -- a NaN-filled buffer comes
    back equal to the oracle."""
    cams, pts, ci, pi, obs = bal.synthetic(24, 3000, 20000, seed=5)
    keep = ~np.isin(ci, drop_cams) & ~np.isin(pi, drop_pts)
    prog = bal.program(cams, pts, ci[keep], pi[keep], obs[keep], loss=ca.Loss.huber(1.0))
    got, info = _device_gradient(prog)
    ref = oracle_eval(prog)
    assert_parity(got, ref, ("unobserved", drop_cams, drop_pts))
    P = pts.shape[0]
    g = got[3]
    for p in drop_pts:
        assert np.all(g[3 * p:3 * p + 3] == 0.0)
    cam0 = 3 * P
    for c in drop_cams:
        assert np.all(g[cam0 + 9 * c:cam0 + 9 * c + 9] == 0.0)
