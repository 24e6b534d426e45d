"""ceres_amd: Python host side of the MI355X (gfx950) residual/Jacobian
evaluator for Ceres' ProblemCUDA / AutoDiffCostFunction residual blocks.

The compute path is libcse.so (HIP kernels behind the C ABI in
include/cse.h); this package builds Programs and calls it.  There is no
CPU fallback anywhere in the package.
"""
from . import _cse, bal
from ._cse import (LOSS_CAUCHY, LOSS_HUBER, LOSS_TRIVIAL, LOSS_USER, POINT_DISPLACEMENT_3_3,
                   SNAVELY_2_9_3, SNAVELY_NO_DISTORTION_2_7_3, SNAVELY_QUATERNION_2_10_3,
                   FUNCTOR_SHAPES, functor_shape, load_functor_library)
from .problem import (BLOCK_SPARSE, COMPRESSED_ROW, Evaluator, Loss, Program, ProblemCUDA,
                      ResidualGroup, host_register, host_unregister)

__all__ = ["bal", "Evaluator", "Loss", "Program", "ProblemCUDA", "ResidualGroup",
           "BLOCK_SPARSE", "COMPRESSED_ROW", "SNAVELY_2_9_3", "SNAVELY_NO_DISTORTION_2_7_3",
           "SNAVELY_QUATERNION_2_10_3", "POINT_DISPLACEMENT_3_3", "LOSS_TRIVIAL", "LOSS_HUBER",
           "LOSS_CAUCHY", "LOSS_USER", "FUNCTOR_SHAPES", "functor_shape", "load_functor_library",
           "host_register", "host_unregister"]
