"""Shared helpers for the user functor tests: the example functor library
(examples/build/libuser_functors.so, examples/user_functors.hip) loaded into
this process's libcse.so, its kinds by name, and the user losses' bytes.

The library is built by `make -C examples` (__graft_entry__.build()); it is
user code, not the oracle."""
import ctypes as C
import os

from ceres_amd import _cse
import ceres_amd as ca

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "examples", "build", "libuser_functors.so")

_state = {}


def library():
    if "lib" not in _state:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} missing: make -C examples")
        lib = _cse.load_functor_library(LIB)
        lib.cse_example_register.restype = C.c_int
        lib.cse_example_kind_name.restype = C.c_char_p
        lib.cse_example_soft_l_one.argtypes = [C.c_double, C.c_void_p]
        lib.cse_example_tolerant.argtypes = [C.c_double, C.c_double, C.c_void_p]
        kinds = (C.c_int32 * 64)()
        n = lib.cse_example_register(kinds, 64)
        if n < 0:
            raise RuntimeError("cse_example_register: " + _cse.last_error())
        _state["lib"] = lib
        _state["kinds"] = {lib.cse_example_kind_name(i).decode(): kinds[i] for i in range(n)}
    return _state["lib"], _state["kinds"]


def kind(name):
    return library()[1][name]


def soft_l_one(a):
    """Loss for the */SoftLOne kinds: SoftLOneLossCUDA(a)'s bytes."""
    buf = (C.c_char * _cse.USER_LOSS_BYTES)()
    n = library()[0].cse_example_soft_l_one(a, buf)
    return ca.Loss.user_loss(bytes(buf)[:n])


def tolerant(a, b):
    """Loss for the */Tolerant kinds: TolerantLossCUDA(a, b)'s bytes."""
    buf = (C.c_char * _cse.USER_LOSS_BYTES)()
    n = library()[0].cse_example_tolerant(a, b, buf)
    return ca.Loss.user_loss(bytes(buf)[:n])
