"""Host-side Jacobian layout builders (csrc/layout.cpp) on malformed input,
without a GPU: ProblemCUDA refuses a parameter block listed twice in one
residual block as ProblemImpl::AddResidualBlock does (problem_impl.cc:
285-301), and the C ABI's CRS builder, reached with such a block anyway,
returns CSE_ERR_INVALID with a cse_last_error text naming the block."""
import numpy as np
import pytest

import ceres_amd as ca
from ceres_amd import _cse


def _problem():
    pb = ca.ProblemCUDA()
    xs = [pb.add_parameter_block(np.full(2, float(i))) for i in range(4)]
    return pb, xs


def test_duplicate_block_refused_when_added():
    pb, xs = _problem()
    pb.add_residual_blocks(_cse.TEST_BILINEAR_1_2_2, None, [[xs[0], xs[1]]], [[1.0]])
    with pytest.raises(ValueError, match="duplicate parameter blocks in residual block 2"):
        pb.add_residual_blocks(_cse.TEST_BILINEAR_1_2_2, None,
                               [[xs[2], xs[3]], [xs[1], xs[1]]], [[1.0], [2.0]])
    with pytest.raises(ValueError, match="out of range"):
        pb.add_residual_block(_cse.TEST_BILINEAR_1_2_2, None, [1.0], xs[0], 17)


def test_crs_layout_reports_a_duplicate_block():
    pb, xs = _problem()
    pb.add_residual_blocks(_cse.TEST_BILINEAR_1_2_2, None, [[xs[0], xs[1]], [xs[2], xs[3]]],
                           [[1.0], [2.0]])
    pb._groups[0].ids[1] = [xs[3], xs[3]]  # past the facade's check
    prog = pb.program()
    with pytest.raises(RuntimeError, match="residual block 1 lists a parameter block twice"):
        prog.compile(ca.COMPRESSED_ROW)
