"""User functor kinds without a GPU: the example library
(examples/user_functors.hip) registers its functors' kernels with libcse.so
(cse_register_functor), the shapes come back through cse_functor_shape, and
malformed launch tables are refused.  (Evaluation: test_user_functor_gpu.py.)"""
import ctypes as C

import pytest

from ceres_amd import _cse
import user_functors as U

NAMES = {
    "BundlerResidual/Trivial": (2, (9, 3), 2),
    "BundlerResidual/SoftLOne": (2, (9, 3), 2),
    "SnavelyReprojectionErrorNoRadialDistortion/Trivial": (2, (7, 3), 2),
    "SnavelyReprojectionErrorWithQuaternions/Trivial": (2, (10, 3), 2),
    "PointDisplacementError/Trivial": (3, (3,), 3),
    "BinaryScalarCost/Trivial": (1, (2, 2), 1),
    "TenParameterCost/Trivial": (1, (1,) * 10, 1),
    "PoseReprojectionError/Trivial": (2, (6, 3), 6),
    "PointToPlaneError/Cauchy": (1, (6, 3), 4),
    "RigidAlignmentError/Trivial": (3, (6,), 6),
}


def test_registration_shapes_and_idempotence():
    lib, kinds = U.library()
    assert len(kinds) == 17
    assert all(k >= _cse.FUNCTOR_USER_FIRST for k in kinds.values())
    assert len(set(kinds.values())) == len(kinds)
    for name, shape in NAMES.items():
        assert _cse.functor_shape(kinds[name]) == shape, name
    again = (C.c_int32 * 64)()
    assert lib.cse_example_register(again, 64) == len(kinds)
    assert sorted(again[:len(kinds)]) == sorted(kinds.values())


def test_unknown_kind_has_no_shape():
    L = _cse.lib()
    nr = C.c_int32()
    assert L.cse_functor_shape(999999, C.byref(nr), None, None, None) == _cse.CSE_ERR_UNSUPPORTED


class functor_ops(C.Structure):
    # include/cse.h cse_functor_ops (ABI 5), for the refusal checks only.
    _fields_ = [("abi_version", C.c_int32), ("num_residuals", C.c_int32),
                ("num_parameter_blocks", C.c_int32), ("sizes", C.c_int32 * 10),
                ("data_size", C.c_int32), ("loss_kind", C.c_int32), ("loss_size", C.c_int32),
                ("kernel_args_size", C.c_int32), ("gradient_args_size", C.c_int32),
                ("camera_gradient_args_size", C.c_int32), ("reserved", C.c_int32),
                ("kernel_args_tag", C.c_uint64), ("name", C.c_char_p), ("table", C.c_void_p * 2),
                ("affine", C.c_void_p * 8), ("multiply", C.c_void_p), ("gradient", C.c_void_p * 2),
                ("fused_points", C.c_void_p * 2), ("camera_gradient", C.c_void_p)]


def test_bad_launch_tables_are_refused():
    assert C.sizeof(functor_ops) == 224
    L = _cse.lib()
    k = C.c_int32(-1)
    o = functor_ops()
    o.abi_version = 3
    o.name = b"bad"
    assert L.cse_register_functor(C.byref(o), C.byref(k)) == _cse.CSE_ERR_INVALID
    assert "ABI" in _cse.last_error()
    o.abi_version = _cse.CSE_ABI_VERSION
    o.kernel_args_size = 8  # a TU built against other headers
    assert L.cse_register_functor(C.byref(o), C.byref(k)) == _cse.CSE_ERR_INVALID
    assert "layout" in _cse.last_error()
    assert k.value == -1
