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
