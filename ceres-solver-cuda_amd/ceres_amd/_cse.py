"""ctypes binding of include/cse.h (the C ABI of libcse.so).

The library is loaded from ceres-solver-cuda_amd/lib/libcse.so (built by
`make` in ceres-solver-cuda_amd/ or __graft_entry__.build()).  There is no
fallback: if the library is missing, loading raises.  use_library() selects
another build of the same ABI before the first load (bench.py --lib tuning:
lib/libcse_tuning.so, the A/B build of tools/).
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.normpath(os.path.join(HERE, "..", "lib", "libcse.so"))

CSE_ABI_VERSION = 5

# cse_options.jacobian_form (cse_jacobian_form)
JACOBIAN_CLOSED_FORM = 0
JACOBIAN_JET = 1
CSE_OK = 0
CSE_EVALUATION_FAILED = 1
CSE_ERR_INVALID = -1
CSE_ERR_HIP = -2
CSE_ERR_OOM = -3
CSE_ERR_UNSUPPORTED = -4
EVAL_SAME_POINT = 1  # CSE_EVAL_SAME_POINT: new_evaluation_point == false

# cse_functor_kind
SNAVELY_2_9_3 = 0
SNAVELY_NO_DISTORTION_2_7_3 = 1
SNAVELY_QUATERNION_2_10_3 = 2
POINT_DISPLACEMENT_3_3 = 3
# Known-answer-test functors of the reference's own tests (cse.h).
TEST_LINEAR_3_2_3_4 = 100
TEST_LINEAR_3_4_3_2 = 101
TEST_LINEAR_2_2_3 = 102
TEST_LINEAR_3_2_4 = 103
TEST_LINEAR_4_3_4 = 104
TEST_BILINEAR_1_2_2 = 110
TEST_TEN_PARAMETER_1_x10 = 111
TEST_PARTIAL_OUTPUT_2_1 = 112

# (num_residuals, parameter block sizes, functor data size)
FUNCTOR_SHAPES = {
    SNAVELY_2_9_3: (2, (9, 3), 2),
    SNAVELY_NO_DISTORTION_2_7_3: (2, (7, 3), 2),
    SNAVELY_QUATERNION_2_10_3: (2, (10, 3), 2),
    POINT_DISPLACEMENT_3_3: (3, (3,), 3),
    TEST_LINEAR_3_2_3_4: (3, (2, 3, 4), 2),
    TEST_LINEAR_3_4_3_2: (3, (4, 3, 2), 2),
    TEST_LINEAR_2_2_3: (2, (2, 3), 2),
    TEST_LINEAR_3_2_4: (3, (2, 4), 2),
    TEST_LINEAR_4_3_4: (4, (3, 4), 2),
    TEST_BILINEAR_1_2_2: (1, (2, 2), 1),
    TEST_TEN_PARAMETER_1_x10: (1, (1,) * 10, 1),
    TEST_PARTIAL_OUTPUT_2_1: (2, (1,), 1),
}

# cse_schur_preconditioner
SCHUR_IDENTITY = 0
SCHUR_JACOBI = 1
SCHUR_SCHUR_JACOBI = 2

# cse_loss_kind
LOSS_TRIVIAL = 0
LOSS_HUBER = 1
LOSS_CAUCHY = 2
LOSS_USER = 3  # a user LossFunctionCUDA compiled into a user functor kind
USER_LOSS_BYTES = 64

# User functor kinds (cse_register_functor) are numbered from here.
FUNCTOR_USER_FIRST = 1000
MAX_PARAMETER_BLOCKS = 10

# cse_manifold_kind (include/cse.h)
MANIFOLD_MATRIX = 0
MANIFOLD_QUATERNION_EUCLIDEAN = 1


class cse_loss(C.Structure):
    _fields_ = [("kind", C.c_int32), ("scaled", C.c_int32), ("a", C.c_double),
                ("scale", C.c_double), ("user", C.c_double * (USER_LOSS_BYTES // 8))]


class cse_parameter_block(C.Structure):
    _fields_ = [("size", C.c_int32), ("tangent_size", C.c_int32),
                ("is_constant", C.c_int32), ("manifold", C.c_int32),
                ("state_offset", C.c_int64), ("delta_offset", C.c_int64),
                ("plus_jacobian_offset", C.c_int64)]


class cse_residual_group(C.Structure):
    _fields_ = [("functor_kind", C.c_int32), ("reserved", C.c_int32),
                ("loss", cse_loss), ("num_blocks", C.c_int64),
                ("residual_block_index", C.POINTER(C.c_int64)),
                ("first_residual_block", C.c_int64),
                ("parameter_block_ids", C.POINTER(C.c_int32)),
                ("functor_data", C.POINTER(C.c_double))]


class cse_problem_desc(C.Structure):
    _fields_ = [("abi_version", C.c_int32), ("num_groups", C.c_int32),
                ("groups", C.POINTER(cse_residual_group)),
                ("num_parameter_blocks", C.c_int64),
                ("parameter_blocks", C.POINTER(cse_parameter_block)),
                ("num_parameters", C.c_int64), ("num_effective_parameters", C.c_int64),
                ("num_constant_parameters", C.c_int64),
                ("constant_state", C.POINTER(C.c_double)),
                ("num_plus_jacobian_values", C.c_int64),
                ("plus_jacobians", C.POINTER(C.c_double)),
                ("num_residual_blocks", C.c_int64), ("num_residuals", C.c_int64),
                ("residual_layout", C.POINTER(C.c_int64)),
                ("jacobian_per_residual_layout", C.POINTER(C.c_int64)),
                ("jacobian_per_residual_offsets", C.POINTER(C.c_int64)),
                ("num_jacobian_per_residual_offsets", C.c_int64),
                ("num_jacobian_values", C.c_int64)]


class cse_options(C.Structure):
    _fields_ = [("device", C.c_int32), ("check_finite", C.c_int32),
                ("apply_loss_function", C.c_int32), ("force_general_layout", C.c_int32),
                ("profile", C.c_int32), ("use_stream", C.c_int32), ("stream", C.c_void_p),
                ("gradient_mode", C.c_int32), ("jacobian_form", C.c_int32)]


class cse_info(C.Structure):
    _fields_ = [("num_residual_blocks", C.c_int64), ("num_residuals", C.c_int64),
                ("num_parameters", C.c_int64), ("num_effective_parameters", C.c_int64),
                ("num_jacobian_values", C.c_int64), ("num_groups", C.c_int32),
                ("num_affine_groups", C.c_int32), ("device", C.c_int32),
                ("num_fused_gradient_groups", C.c_int32), ("bytes_jacobian_eval", C.c_int64),
                ("bytes_residual_eval", C.c_int64)]


P_i32 = C.POINTER(C.c_int32)
P_i64 = C.POINTER(C.c_int64)
P_f64 = C.POINTER(C.c_double)
P_pb = C.POINTER(cse_parameter_block)

# Every exported symbol of include/cse.h with its signature.
SIGNATURES = {
    "cse_default_options": (None, [C.POINTER(cse_options)]),
    "cse_create": (C.c_int, [C.POINTER(cse_problem_desc), C.POINTER(cse_options),
                             C.POINTER(C.c_void_p)]),
    "cse_evaluate": (C.c_int, [C.c_void_p, P_f64, P_f64, P_f64, P_f64, P_f64]),
    "cse_evaluate_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_void_p, C.c_void_p]),
    "cse_evaluate_ex": (C.c_int, [C.c_void_p, P_f64, P_f64, P_f64, P_f64, P_f64, C.c_uint32]),
    "cse_evaluate_device_ex": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_void_p, C.c_uint32]),
    "cse_wait": (C.c_int, [C.c_void_p]),
    "cse_set_plus_jacobians": (C.c_int, [C.c_void_p, P_f64]),
    "cse_plus_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "cse_plus": (C.c_int, [C.c_void_p, P_f64, P_f64, P_f64]),
    "cse_jacobian_right_multiply": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "cse_jacobian_left_multiply": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "cse_cgnr_multiply": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "cse_schur_structure": (C.c_int, [C.c_void_p, P_i64, P_i64]),
    "cse_schur_init": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_int]),
    "cse_schur_init_gradient": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                          C.c_void_p, C.c_int, C.c_void_p]),
    "cse_schur_multiply": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "cse_schur_precondition": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "cse_schur_back_substitute": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "cse_create_multi": (C.c_int, [C.POINTER(cse_problem_desc), C.POINTER(cse_options),
                                   P_i32, C.c_int32, C.POINTER(C.c_void_p)]),
    "cse_shard_info": (C.c_int, [C.c_void_p, P_i32, P_i64, P_i32]),
    "cse_shard_transfer_bytes": (C.c_int, [C.c_void_p, P_i64, P_i64]),
    "cse_host_register": (C.c_int, [C.c_void_p, C.c_size_t]),
    "cse_host_unregister": (C.c_int, [C.c_void_p]),
    "cse_destroy": (None, [C.c_void_p]),
    "cse_last_error": (C.c_char_p, []),
    "cse_get_info": (C.c_int, [C.c_void_p, C.POINTER(cse_info)]),
    "cse_kernel_stats": (C.c_int, [C.c_void_p, P_f64, P_f64, P_i64]),
    "cse_reset_kernel_stats": (C.c_int, [C.c_void_p]),
    "cse_block_sparse_layout": (C.c_int, [C.c_int64, P_pb, C.c_int64, P_i64, P_i32, P_i32,
                                          C.c_int64, P_i64, P_i64, P_i64, P_i64]),
    "cse_compressed_row_layout": (C.c_int, [C.c_int64, P_pb, C.c_int64, P_i64, P_i32, P_i32,
                                            P_i64, P_i64, P_i64, P_i64, P_i64, P_i64]),
    "cse_layout_offsets_count": (C.c_int64, [C.c_int64, P_pb, C.c_int64, P_i64, P_i32, P_i32]),
    "cse_register_functor": (C.c_int, [C.c_void_p, P_i32]),
    "cse_functor_shape": (C.c_int, [C.c_int32, P_i32, P_i32, P_i32, P_i32]),
    "cse_abi_version": (C.c_int, []),
    "cse_build_info": (C.c_char_p, []),
}

# Entry points an older build (tools/ A/B runs against a previous commit) may lack.
_SINCE_ROUND3 = {"cse_evaluate_ex", "cse_evaluate_device_ex"}
_DEFAULT_LIB = LIB_PATH

_lib = None


def use_library(path):
    """Load `path` (a build of the same ABI) instead of lib/libcse.so.  Must
    be called before the first lib() call."""
    global LIB_PATH
    if _lib is not None:
        raise RuntimeError("libcse already loaded from " + LIB_PATH)
    LIB_PATH = os.path.abspath(path)


def lib():
    """Load libcse.so once.  Raises if the HIP library has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libcse.so not found at {LIB_PATH}: build it with `make -C "
                f"ceres-solver-cuda_amd` (there is no CPU fallback)")
        handle = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if name in _SINCE_ROUND3 and LIB_PATH != _DEFAULT_LIB and not hasattr(handle, name):
                continue  # an older build loaded for an A/B (tools/)
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        if handle.cse_abi_version() != CSE_ABI_VERSION:
            raise RuntimeError("libcse.so ABI version mismatch")
        _lib = handle
    return _lib


def last_error():
    return lib().cse_last_error().decode()


def functor_shape(kind):
    """(num_residuals, parameter block sizes, functor data size) of a built-in
    or registered functor kind."""
    if kind in FUNCTOR_SHAPES:
        return FUNCTOR_SHAPES[kind]
    nr, nb, d = C.c_int32(), C.c_int32(), C.c_int32()
    sizes = (C.c_int32 * MAX_PARAMETER_BLOCKS)()
    check(lib().cse_functor_shape(int(kind), C.byref(nr), C.byref(nb), sizes, C.byref(d)),
          "cse_functor_shape")
    shape = (nr.value, tuple(sizes[:nb.value]), d.value)
    FUNCTOR_SHAPES[kind] = shape
    return shape


def load_functor_library(path):
    """Load a user functor library (a hipcc-built .so that includes
    ceres_amd/autodiff_cuda.h and links libcse.so) after libcse.so itself, so
    that its cse_register_functor calls reach this process's registry (the
    library binds to the loaded copy through libcse.so's SONAME)."""
    lib()
    return C.CDLL(os.path.abspath(path))


def check(rc, what):
    if rc < 0:
        raise RuntimeError(f"{what} failed ({rc}): {last_error()}")
    return rc
