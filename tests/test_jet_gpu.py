"""Device Jet parity (internal/ceres/jet_cuda_test.cu.cc:123-983, the
operations the library's functors use).

tests/hip/libjetops.so runs the library's Jet (csrc/jet.hpp, compiled with
the product kernels' -fno-signed-zeros -ffinite-math-only) on the GPU for the
reference test's operands x, y, z (:101-104) and the scalar 9.0; each result
is compared with the reference's jet.h formulas (include/ceres/jet.h:309-402,
533-537, 617-641, 742-760) evaluated here in IEEE double, with the test's
AreAlmostEqual at relative 1e-13 (:55-84).  Not covered: the Jet functions
the library does not implement (exp, log, pow, atan2, erf, Bessel, ...; no
functor on the path uses them) and /=.
"""
import ctypes as C
import math
import os

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "hip", "libjetops.so")
TOL = 1e-13

X = (2.3, -2.7, 1e-3)
Y = (1.7, 0.5, 1e2)
Z = (1e-6, 1e-4, 1e-2)
S = 9.0


def add(f, g): return (f[0] + g[0], f[1] + g[1], f[2] + g[2])                 # jet.h:324-327
def sub(f, g): return (f[0] - g[0], f[1] - g[1], f[2] - g[2])                 # :342-345
def neg(f): return (-f[0], -f[1], -f[2])                                      # :318-321
def mul(f, g): return (f[0] * g[0], f[0] * g[1] + f[1] * g[0], f[0] * g[2] + f[2] * g[0])  # :360


def div(f, g):  # :378-389
    inv = 1.0 / g[0]
    q = f[0] * inv
    return (q, (f[1] - q * g[1]) * inv, (f[2] - q * g[2]) * inv)


def adds(f, s): return (f[0] + s, f[1], f[2])                                 # :330-339
def subs(f, s): return (f[0] - s, f[1], f[2])                                 # :348-351
def ssub(s, f): return (s - f[0], -f[1], -f[2])                               # :354-356
def muls(f, s): return (f[0] * s, f[1] * s, f[2] * s)                         # :366-374


def divs(f, s):  # :400-403
    inv = 1.0 / s
    return (f[0] * inv, f[1] * inv, f[2] * inv)


def sdiv(s, g):  # :393-396
    m = -s / (g[0] * g[0])
    return (s / g[0], g[1] * m, g[2] * m)


def jsqrt(f):  # :617-621
    t = math.sqrt(f[0])
    two_inv = 1.0 / (2.0 * t)
    return (t, f[1] * two_inv, f[2] * two_inv)


def jabs(f):  # :535-537
    sgn = math.copysign(1.0, f[0])
    return (abs(f[0]), sgn * f[1], sgn * f[2])


def jsin(f): return (math.sin(f[0]), math.cos(f[0]) * f[1], math.cos(f[0]) * f[2])     # :638-640
def jcos(f): return (math.cos(f[0]), -math.sin(f[0]) * f[1], -math.sin(f[0]) * f[2])   # :625-627


def jhypot(x, y, z):  # :742-759
    t = math.hypot(x[0], y[0], z[0])
    return (t,) + tuple(x[0] / t * x[i] + y[0] / t * y[i] + z[0] / t * z[i] for i in (1, 2))


EXPECTED = [
    add(X, Y), sub(X, Y), mul(X, Y), neg(X), add(X, Y), sub(X, Y), mul(X, Y), div(X, Y),
    adds(X, S), adds(X, S), subs(X, S), ssub(S, X), muls(X, S), muls(X, S), divs(X, S),
    sdiv(S, X), jsqrt(X), jsqrt(Y), jabs(X), jabs(neg(X)), jsin(X), jcos(X), jsin(Z), jcos(Z),
    jhypot(X, Y, Z), jhypot(Z, neg(Y), X), jhypot(Z, Z, Z),
]


def almost_equal(x, y, tol=TOL):
    """AreAlmostEqual (jet_cuda_test.cu.cc:55-75)."""
    if math.isnan(x) and math.isnan(y):
        return True
    if math.isinf(x) and math.isinf(y):
        return math.copysign(1, x) == math.copysign(1, y)
    diff = abs(x - y)
    if x == 0.0 or y == 0.0:
        return diff <= tol
    return diff / max(abs(x), abs(y)) <= tol


def test_device_jet_matches_reference_formulas(gpu):
    assert os.path.exists(LIB), "build tests/hip/libjetops.so (__graft_entry__.build())"
    lib = C.CDLL(LIB)
    lib.jet_ops_names.restype = C.c_char_p
    lib.jet_ops_run.restype = C.c_int
    lib.jet_ops_run.argtypes = [C.POINTER(C.c_double)] * 3 + [C.c_double, C.POINTER(C.c_double)]
    names = lib.jet_ops_names().decode().split(";")
    arr = lambda t: (C.c_double * 3)(*t)
    out = (C.c_double * (3 * len(EXPECTED)))()
    n = lib.jet_ops_run(arr(X), arr(Y), arr(Z), S, out)
    assert n == len(EXPECTED)
    bad = []
    for i, exp in enumerate(EXPECTED):
        got = tuple(out[3 * i:3 * i + 3])
        if not all(almost_equal(g, e) for g, e in zip(got, exp)):
            bad.append((names[i] if i < len(names) else i, got, exp))
    assert not bad, bad


def test_device_sincos_polynomial_and_library_paths(gpu):
    """cse::SinCos (jet.hpp): the reduction-free polynomial on waves whose
    arguments all lie in [-pi/4, pi/4], the library sincos on the others.
    Both within 2 ulp of the host libm on a dense sweep, on the ends of the
    interval, on tiny and signed-zero arguments, and on waves that mix one
    large angle into small ones (those must take the library path)."""
    import numpy as np
    lib = C.CDLL(LIB)
    lib.sincos_run.restype = C.c_int
    lib.sincos_run.argtypes = [C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_double),
                               C.POINTER(C.c_double)]
    q = math.pi / 4
    small = np.concatenate([np.linspace(-q, q, 64 * 2000), [q, -q, np.nextafter(q, 0), 1e-300,
                                                             -1e-300, 0.0, 5e-9, -3e-5] * 8])
    small = small[: len(small) // 64 * 64]
    mixed = np.random.default_rng(3).uniform(-q, q, 64 * 64)
    mixed[::64] = np.random.default_rng(4).uniform(1.0, 40.0, 64)  # one big angle per wave
    big = np.random.default_rng(5).uniform(-1e4, 1e4, 64 * 64)
    x = np.ascontiguousarray(np.concatenate([small, mixed, big]))
    n = len(x)
    s = np.empty(n)
    c = np.empty(n)
    p = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
    assert lib.sincos_run(p(x), n, p(s), p(c)) == n
    ref_s = np.array([math.sin(v) for v in x])
    ref_c = np.array([math.cos(v) for v in x])
    ulp_s = np.spacing(np.abs(ref_s)) + 5e-324
    ulp_c = np.spacing(np.abs(ref_c)) + 5e-324
    assert np.max(np.abs(s - ref_s) / ulp_s) <= 2.0, np.max(np.abs(s - ref_s) / ulp_s)
    assert np.max(np.abs(c - ref_c) / ulp_c) <= 2.0, np.max(np.abs(c - ref_c) / ulp_c)
