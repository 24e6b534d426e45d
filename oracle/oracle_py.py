"""ctypes front end of the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker.  Never used by the product.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

BLOCK_SPARSE, COMPRESSED_ROW = 0, 1
LINEAR_TEST = 4

P_i32 = C.POINTER(C.c_int32)
P_i64 = C.POINTER(C.c_int64)
P_f64 = C.POINTER(C.c_double)


# oracle.h kinds/losses the GPU side reaches through user functor kinds
BUNDLER_RESIDUAL_2_9_3 = 5
LOSS_SOFT_L_ONE = 10
LOSS_TOLERANT = 11


class oracle_program(C.Structure):
    _fields_ = [("num_parameter_blocks", C.c_int64), ("pb_size", P_i32),
                ("pb_tangent_size", P_i32), ("pb_constant", P_i32),
                ("pb_plus_jacobian", P_i64), ("plus_jacobians", P_f64),
                ("num_residual_blocks", C.c_int64), ("rb_kind", P_i32),
                ("rb_loss_kind", P_i32), ("rb_loss_a", P_f64), ("rb_loss_scale", P_f64),
                ("rb_loss_scaled", P_i32), ("rb_param_begin", P_i64), ("rb_params", P_i32),
                ("rb_data_begin", P_i64), ("rb_data", P_f64), ("jacobian_format", C.c_int32),
                ("num_eliminate_blocks", C.c_int32), ("apply_loss_function", C.c_int32),
                ("rb_loss_b", P_f64)]


class oracle_sizes(C.Structure):
    _fields_ = [("num_parameters", C.c_int64), ("num_effective_parameters", C.c_int64),
                ("num_constant_parameters", C.c_int64), ("num_residuals", C.c_int64),
                ("num_jacobian_values", C.c_int64)]


_lib = None


def use_library(path):
    """Load `path` (another build of oracle.cpp, e.g. the -march=native CPU
    baseline of `make native`) instead of build/liboracle.so.  Must be
    called before the first lib() call."""
    global LIB_PATH
    if _lib is not None:
        raise RuntimeError("liboracle already loaded from " + LIB_PATH)
    LIB_PATH = os.path.abspath(path)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", HERE])
        L = C.CDLL(LIB_PATH)
        L.oracle_sizes_of.argtypes = [C.POINTER(oracle_program), C.POINTER(oracle_sizes)]
        L.oracle_evaluate.argtypes = [C.POINTER(oracle_program), P_f64, P_f64, C.c_int, P_f64,
                                      P_f64, P_f64, P_f64]
        L.oracle_create.argtypes = [C.POINTER(oracle_program), C.c_int]
        L.oracle_create.restype = C.c_void_p
        L.oracle_run.argtypes = [C.c_void_p, P_f64, P_f64, P_f64, P_f64, P_f64, P_f64]
        L.oracle_destroy.argtypes = [C.c_void_p]
        L.oracle_jacobian_offsets.argtypes = [C.POINTER(oracle_program), P_i64, P_i64, P_i64,
                                              P_i64]
        L.oracle_angle_axis_rotate_point.argtypes = [P_f64, P_f64, P_f64]
        L.oracle_quaternion_rotate_point.argtypes = [P_f64, P_f64, P_f64]
        L.oracle_loss.argtypes = [C.c_int, C.c_double, C.c_int, C.c_double, C.c_double, P_f64]
        L.oracle_loss_ab.argtypes = [C.c_int, C.c_double, C.c_double, C.c_int, C.c_double,
                                     C.c_double, P_f64]
        L.oracle_corrector.argtypes = [C.c_double, P_f64, C.c_int, C.c_int, P_f64, P_f64]
        L.oracle_autodiff.argtypes = [C.c_int, P_f64, C.POINTER(P_f64), P_f64, C.POINTER(P_f64)]
        L.oracle_jet_op.argtypes = [C.c_int, P_f64, P_f64, P_f64, P_f64]
        _lib = L
    return _lib


def _p(a, t):
    return None if a is None else a.ctypes.data_as(C.POINTER(t))


class OracleProgram:
    """Per-block arrays in program order for a ceres_amd Program (or raw
    arrays for hand-built KAT problems)."""

    def __init__(self, pb_size, pb_tangent, pb_constant, pb_plus_jacobian, plus_jacobians,
                 rb_kind, rb_loss_kind, rb_loss_a, rb_loss_scale, rb_loss_scaled, rb_param_begin,
                 rb_params, rb_data_begin, rb_data, jacobian_format, num_eliminate_blocks,
                 apply_loss_function=1, rb_loss_b=None):
        arr = lambda x, t: np.ascontiguousarray(np.asarray(x), t)
        self.a = dict(pb_size=arr(pb_size, np.int32), pb_tangent=arr(pb_tangent, np.int32),
                      pb_constant=arr(pb_constant, np.int32),
                      pb_pj=arr(pb_plus_jacobian, np.int64), pj=arr(plus_jacobians, np.float64),
                      kind=arr(rb_kind, np.int32), lk=arr(rb_loss_kind, np.int32),
                      la=arr(rb_loss_a, np.float64), ls=arr(rb_loss_scale, np.float64),
                      lsd=arr(rb_loss_scaled, np.int32), pbeg=arr(rb_param_begin, np.int64),
                      params=arr(rb_params, np.int32), dbeg=arr(rb_data_begin, np.int64),
                      data=arr(rb_data, np.float64),
                      lb=None if rb_loss_b is None else arr(rb_loss_b, np.float64))
        a = self.a
        self.s = oracle_program(len(a["pb_size"]), _p(a["pb_size"], C.c_int32),
                                _p(a["pb_tangent"], C.c_int32), _p(a["pb_constant"], C.c_int32),
                                _p(a["pb_pj"], C.c_int64), _p(a["pj"], C.c_double),
                                len(a["kind"]), _p(a["kind"], C.c_int32), _p(a["lk"], C.c_int32),
                                _p(a["la"], C.c_double), _p(a["ls"], C.c_double),
                                _p(a["lsd"], C.c_int32), _p(a["pbeg"], C.c_int64),
                                _p(a["params"], C.c_int32), _p(a["dbeg"], C.c_int64),
                                _p(a["data"], C.c_double), int(jacobian_format),
                                int(num_eliminate_blocks), int(apply_loss_function),
                                _p(a["lb"], C.c_double))

    @classmethod
    def from_program(cls, prog, apply_loss_function=True, kind_map=None, loss_map=None):
        """kind_map: functor kind -> oracle kind (user functor kinds);
        loss_map: Loss -> (oracle loss kind, a, b) for user losses."""
        # The reference's form: every manifold as its explicit plus-Jacobian
        # (Program.with_explicit_manifolds, at the Program's state).
        if getattr(prog, "pb_manifold", None) is not None and np.any(prog.pb_manifold):
            raise ValueError("OracleProgram: convert with prog.with_explicit_manifolds(state) first")
        nrb = prog.num_residual_blocks
        kind = np.zeros(nrb, np.int32)
        lk = np.zeros(nrb, np.int32)
        la = np.ones(nrb)
        ls = np.ones(nrb)
        lsd = np.zeros(nrb, np.int32)
        lb = np.zeros(nrb)
        nb = np.zeros(nrb, np.int64)
        nd = np.zeros(nrb, np.int64)
        for g in prog.groups:
            idx = g.index if g.index is not None else np.arange(g.first, g.first + g.n)
            kind[idx] = (kind_map or {}).get(g.kind, g.kind)
            lk[idx] = g.loss.kind
            la[idx] = g.loss.a
            if loss_map is not None and g.loss.kind == 3:  # LOSS_USER
                lk[idx], la[idx], lb[idx] = loss_map(g.loss)
            ls[idx] = g.loss.scale
            lsd[idx] = int(g.loss.scaled)
            nb[idx] = g.ids.shape[1]
            nd[idx] = g.data.shape[1]
        pbeg = np.zeros(nrb + 1, np.int64)
        np.cumsum(nb, out=pbeg[1:])
        dbeg = np.zeros(nrb + 1, np.int64)
        np.cumsum(nd, out=dbeg[1:])
        params = np.empty(int(pbeg[-1]), np.int32)
        data = np.empty(int(dbeg[-1]))
        for g in prog.groups:
            idx = g.index if g.index is not None else np.arange(g.first, g.first + g.n)
            params[(pbeg[idx][:, None] + np.arange(g.ids.shape[1])).ravel()] = g.ids.ravel()
            data[(dbeg[idx][:, None] + np.arange(g.data.shape[1])).ravel()] = g.data.ravel()
        fmt = BLOCK_SPARSE if prog.format == "block_sparse" else COMPRESSED_ROW
        return cls(prog.pb_size, prog.pb_tangent, prog.pb_constant, prog.pb_plus_jacobian,
                   prog.plus_jacobians if prog.plus_jacobians.size else np.zeros(1), kind, lk, la,
                   ls, lsd, pbeg, params, dbeg, data, fmt, prog.num_eliminate_blocks,
                   int(apply_loss_function), lb)

    def sizes(self):
        s = oracle_sizes()
        rc = lib().oracle_sizes_of(C.byref(self.s), C.byref(s))
        if rc:
            raise RuntimeError(f"oracle_sizes_of: {rc}")
        return s

    def evaluate(self, state, constant_state=None, num_threads=1, residuals=True, gradient=True,
                 jacobian=True):
        s = self.sizes()
        state = np.ascontiguousarray(state, np.float64)
        cs = np.ascontiguousarray(constant_state if constant_state is not None else np.zeros(1),
                                  np.float64)
        cost = C.c_double(-1.0)
        r = np.empty(s.num_residuals) if residuals else None
        g = np.empty(s.num_effective_parameters) if gradient else None
        j = np.empty(s.num_jacobian_values) if jacobian else None
        rc = lib().oracle_evaluate(C.byref(self.s), _p(state, C.c_double), _p(cs, C.c_double),
                                   int(num_threads), C.byref(cost), _p(r, C.c_double),
                                   _p(g, C.c_double), _p(j, C.c_double))
        if rc < 0:
            raise RuntimeError(f"oracle_evaluate: {rc}")
        return rc == 1, cost.value, r, g, j

    def evaluator(self, num_threads):
        """A prepared evaluator (layout + scratch built once): the CPU
        baseline times only run()."""
        return PreparedOracle(self, num_threads)

    def jacobian_offsets(self):
        s = self.sizes()
        nrb = len(self.a["kind"])
        lay = np.empty(nrb, np.int64)
        # upper bound: residuals x blocks per residual
        offs = np.full(int(s.num_residuals) * 8 + 1, -1, np.int64)
        rows = np.empty(int(s.num_residuals) + 1, np.int64)
        cols = np.empty(max(int(s.num_jacobian_values), 1), np.int64)
        rc = lib().oracle_jacobian_offsets(C.byref(self.s), _p(lay, C.c_int64),
                                           _p(offs, C.c_int64), _p(rows, C.c_int64),
                                           _p(cols, C.c_int64))
        if rc:
            raise RuntimeError(f"oracle_jacobian_offsets: {rc}")
        return lay, offs, rows, cols


class PreparedOracle:
    def __init__(self, prog, num_threads):
        self.prog = prog
        self.s = prog.sizes()
        self.h = lib().oracle_create(C.byref(prog.s), int(num_threads))
        if not self.h:
            raise RuntimeError("oracle_create failed")

    def run(self, state, constant_state=None, residuals=None, gradient=None, jacobian=None):
        cs = np.ascontiguousarray(constant_state if constant_state is not None else np.zeros(1))
        cost = C.c_double(-1.0)
        rc = lib().oracle_run(self.h, _p(state, C.c_double), _p(cs, C.c_double), C.byref(cost),
                              _p(residuals, C.c_double), _p(gradient, C.c_double),
                              _p(jacobian, C.c_double))
        return rc == 1, cost.value

    def close(self):
        if self.h:
            lib().oracle_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def angle_axis_rotate_point(aa, pt):
    out = np.empty(3)
    aa, pt = np.ascontiguousarray(aa, float), np.ascontiguousarray(pt, float)
    lib().oracle_angle_axis_rotate_point(_p(aa, C.c_double), _p(pt, C.c_double),
                                         _p(out, C.c_double))
    return out


def quaternion_rotate_point(q, pt):
    out = np.empty(3)
    q, pt = np.ascontiguousarray(q, float), np.ascontiguousarray(pt, float)
    lib().oracle_quaternion_rotate_point(_p(q, C.c_double), _p(pt, C.c_double),
                                         _p(out, C.c_double))
    return out


def loss(kind, a, s, scaled=False, scale=1.0, b=0.0):
    rho = np.empty(3)
    lib().oracle_loss_ab(kind, a, b, int(scaled), scale, s, _p(rho, C.c_double))
    return rho


def corrector(sq_norm, rho, residuals, jacobian):
    r = np.ascontiguousarray(residuals, float).copy()
    J = np.ascontiguousarray(jacobian, float).copy()
    rho = np.ascontiguousarray(rho, float)
    lib().oracle_corrector(sq_norm, _p(rho, C.c_double), J.shape[0], J.shape[1],
                           _p(r, C.c_double), _p(J, C.c_double))
    return r, J


def autodiff(kind, data, params, nres, sizes):
    data = np.ascontiguousarray(data, float)
    ps = [np.ascontiguousarray(p, float) for p in params]
    parr = (P_f64 * len(ps))(*[_p(p, C.c_double) for p in ps])
    jac = [np.empty(nres * s) for s in sizes]
    jarr = (P_f64 * len(jac))(*[_p(j, C.c_double) for j in jac])
    r = np.empty(nres)
    ok = lib().oracle_autodiff(kind, _p(data, C.c_double), parr, _p(r, C.c_double), jarr)
    return ok == 1, r, [j.reshape(nres, s) for j, s in zip(jac, sizes)]


def jet_op(op, x, y=None, z=None):
    f = lambda v: np.ascontiguousarray(v if v is not None else np.zeros(4), float)
    x, y, z = f(x), f(y), f(z)
    out = np.empty(4)
    lib().oracle_jet_op(op, _p(x, C.c_double), _p(y, C.c_double), _p(z, C.c_double),
                        _p(out, C.c_double))
    return out
