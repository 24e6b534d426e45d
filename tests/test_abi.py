"""The C ABI library loads and exports every symbol include/cse.h declares
(no compute call: this runs without a GPU)."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "cse.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set(re.findall(r"\b(cse_[a-z_]+)\s*\(", text))
    return sorted(names)


def test_header_declares_the_boundary():
    names = declared_functions()
    for required in ("cse_create", "cse_evaluate", "cse_evaluate_device", "cse_destroy",
                     "cse_last_error", "cse_wait"):
        assert required in names


def test_library_exports_every_declared_symbol():
    from ceres_amd import _cse
    lib = ctypes.CDLL(_cse.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    # ... and the Python binding declares a signature for each of them.
    assert set(declared_functions()) == set(_cse.SIGNATURES)


def test_abi_version_and_build_info():
    from ceres_amd import _cse
    L = _cse.lib()
    assert L.cse_abi_version() == _cse.CSE_ABI_VERSION
    assert b"gfx950" in L.cse_build_info()


def test_struct_layouts_match_header():
    """ctypes mirrors of the descriptor structs have the C sizes."""
    from ceres_amd import _cse
    assert ctypes.sizeof(_cse.cse_loss) == 88  # ABI 4: 64 bytes of user loss object
    assert ctypes.sizeof(_cse.cse_parameter_block) == 40
    assert ctypes.sizeof(_cse.cse_residual_group) == 136
    assert ctypes.sizeof(_cse.cse_options) == 40


def test_create_rejects_bad_descriptors_without_a_gpu():
    """Validation happens before any HIP call: malformed input fails with
    CSE_ERR_INVALID and a message."""
    from ceres_amd import _cse
    L = _cse.lib()
    h = ctypes.c_void_p()
    assert L.cse_create(None, None, ctypes.byref(h)) == _cse.CSE_ERR_INVALID
    d = _cse.cse_problem_desc()
    d.abi_version = 999
    assert L.cse_create(ctypes.byref(d), None, ctypes.byref(h)) == _cse.CSE_ERR_INVALID
    assert "abi_version" in _cse.last_error()


def test_no_cpu_fallback_in_the_product():
    """The product package never imports the oracle or numpy math for the
    evaluation itself."""
    pkg = os.path.join(REPO, "ceres-solver-cuda_amd", "ceres_amd")
    for f in os.listdir(pkg):
        if f.endswith(".py"):
            src = open(os.path.join(pkg, f)).read()
            assert "oracle" not in src.replace("oracle/", ""), f


def test_product_library_reads_no_environment():
    """libcse.so has no getenv-selected kernels (round 6 removed the tuning
    build altogether): no CSE_* variable name is in its read-only data, and it
    imports no getenv at all."""
    from ceres_amd import _cse
    data = open(_cse.LIB_PATH, "rb").read()
    assert not re.findall(rb"CSE_[A-Z][A-Z_]+", data), re.findall(rb"CSE_[A-Z][A-Z_]+", data)[:5]
    import subprocess
    syms = subprocess.run(["nm", "-D", "--undefined-only", _cse.LIB_PATH], capture_output=True,
                          text=True, check=True).stdout
    assert "getenv" not in syms


def test_create_rejects_unknown_gradient_mode_without_a_gpu():
    """cse_options.gradient_mode has four meanings (0..3); anything else is
    refused before any HIP call instead of silently running as mode 1."""
    from ceres_amd import _cse
    L = _cse.lib()
    h = ctypes.c_void_p()
    d = _cse.cse_problem_desc()
    d.abi_version = _cse.CSE_ABI_VERSION
    layout = (ctypes.c_int64 * 1)(0)
    d.residual_layout = ctypes.cast(layout, _cse.P_i64)
    for mode in (-1, 4, 7):
        o = _cse.cse_options()
        L.cse_default_options(ctypes.byref(o))
        o.gradient_mode = mode
        assert L.cse_create(ctypes.byref(d), ctypes.byref(o), ctypes.byref(h)) == _cse.CSE_ERR_INVALID
        assert "gradient_mode" in _cse.last_error()
        assert not h.value


def test_create_multi_rejects_bad_device_lists_without_a_gpu():
    """cse_create_multi validates the descriptor and the device list before
    any HIP call."""
    from ceres_amd import _cse
    L = _cse.lib()
    h = ctypes.c_void_p()
    d = _cse.cse_problem_desc()
    d.abi_version = _cse.CSE_ABI_VERSION
    layout = (ctypes.c_int64 * 1)(0)
    d.residual_layout = ctypes.cast(layout, _cse.P_i64)
    assert L.cse_create_multi(ctypes.byref(d), None, None, 2, ctypes.byref(h)) == _cse.CSE_ERR_INVALID
    devs = (ctypes.c_int32 * 1)(0)
    assert L.cse_create_multi(ctypes.byref(d), None, devs, 0, ctypes.byref(h)) == _cse.CSE_ERR_INVALID
    assert "no devices" in _cse.last_error()
    bad = _cse.cse_problem_desc()
    bad.abi_version = 999
    assert L.cse_create_multi(ctypes.byref(bad), None, devs, 1, ctypes.byref(h)) == _cse.CSE_ERR_INVALID
    assert not h.value
