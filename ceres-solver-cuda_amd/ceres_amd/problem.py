"""Host-side Program model and evaluator for Python callers.

Mirrors the reference's ProblemCUDA surface (include/ceres/problem_cuda.h:85-486)
and the part of Ceres' Program the evaluator consumes:

  * ProblemCUDA.add_parameter_block / set_parameter_block_constant /
    set_plus_jacobian  (Problem::AddParameterBlock, SetParameterBlockConstant,
    SetManifold -> the manifold's PlusJacobian);
  * ProblemCUDA.add_residual_blocks(kind, loss, ids, data): a vectorised
    ProblemCUDA::AddResidualBlock<Functor, kR, Ns...>(cost, loss, x0, xs...)
    for many blocks of one (functor, loss) type at once — one
    "registered CUDA evaluator" (problem_cuda.h:462-468);
  * Program.compile(format, num_eliminate_blocks): parameter offsets
    (Program::SetParameterOffsetsAndIndex, program.cc:151-177) and the
    Jacobian layout of BlockJacobianWriter / CompressedRowJacobianWriter,
    built by the library's own C++ layout builders;
  * Evaluator: the ProgramEvaluatorCUDA seam (Evaluate(state, cost,
    residuals, gradient, jacobian_values)) over libcse.so.

Arrays, not per-block objects: a BAL problem-13682 has 29M residual blocks.
"""
import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import _cse
from ._cse import FUNCTOR_SHAPES, functor_shape

BLOCK_SPARSE = "block_sparse"
COMPRESSED_ROW = "compressed_row"


def _ptr(a, ctype):
    if a is None:
        return None
    return a.ctypes.data_as(C.POINTER(ctype))


@dataclass
class Loss:
    """LossFunctionCUDA (include/ceres/loss_function_cuda.h:62-150)."""
    kind: int = _cse.LOSS_TRIVIAL
    a: float = 1.0
    scaled: bool = False
    scale: float = 1.0
    # LOSS_USER: the user loss object's bytes (cse_loss.user), as produced by
    # the functor library that compiled the loss.
    user: bytes = b""

    @staticmethod
    def trivial():
        return Loss(_cse.LOSS_TRIVIAL)

    @staticmethod
    def huber(a):
        return Loss(_cse.LOSS_HUBER, float(a))

    @staticmethod
    def cauchy(a):
        return Loss(_cse.LOSS_CAUCHY, float(a))

    @staticmethod
    def user_loss(obj_bytes):
        """A user LossFunctionCUDA (CSE_LOSS_USER): its object bytes; only
        with a user functor kind registered with that loss type."""
        b = bytes(obj_bytes)
        if len(b) > _cse.USER_LOSS_BYTES:
            raise ValueError("user loss object larger than 64 bytes")
        return Loss(_cse.LOSS_USER, 0.0, False, 1.0, b)

    def scaled_by(self, s):
        return Loss(self.kind, self.a, True, float(s), self.user)

    def key(self):
        return (self.kind, self.a, self.scaled, self.scale, self.user)

    def describe(self):
        """The cse_loss of this loss."""
        d = _cse.cse_loss(self.kind, int(self.scaled), self.a, self.scale)
        if self.user:
            C.memmove(C.addressof(d.user), self.user, len(self.user))
        return d


@dataclass
class ResidualGroup:
    kind: int
    loss: Loss
    ids: np.ndarray            # (n, num blocks of kind) int32
    data: np.ndarray           # (n, data size) float64
    index: Optional[np.ndarray] = None  # (n,) int64 program order; None = contiguous
    first: int = 0

    @property
    def n(self):
        return int(self.ids.shape[0])


@dataclass
class Program:
    """A reduced Program: parameter blocks and residual groups in program order."""
    pb_size: np.ndarray
    pb_tangent: np.ndarray
    pb_constant: np.ndarray
    pb_plus_jacobian: np.ndarray
    plus_jacobians: np.ndarray
    groups: List[ResidualGroup]
    num_residual_blocks: int
    state: np.ndarray           # active parameter blocks, program order
    constant_state: np.ndarray  # constant parameter blocks
    # Set by compile().
    format: str = BLOCK_SPARSE
    num_eliminate_blocks: int = 0
    state_offset: np.ndarray = None
    delta_offset: np.ndarray = None
    residual_layout: np.ndarray = None
    jacobian_per_residual_layout: np.ndarray = None
    jacobian_per_residual_offsets: np.ndarray = None
    num_jacobian_values: int = 0
    crs_rows: np.ndarray = None
    crs_cols: np.ndarray = None
    # cse_manifold_kind per parameter block (None = all MANIFOLD_MATRIX).
    pb_manifold: np.ndarray = None
    _keep: list = field(default_factory=list)

    @property
    def num_parameter_blocks(self):
        return int(self.pb_size.shape[0])

    @property
    def num_parameters(self):
        return int(self.pb_size[self.pb_constant == 0].sum())

    @property
    def num_effective_parameters(self):
        return int(self.pb_tangent[self.pb_constant == 0].sum())

    @property
    def num_constant_parameters(self):
        return int(self.pb_size[self.pb_constant != 0].sum())

    def residuals_per_block(self):
        nres = np.zeros(self.num_residual_blocks, np.int32)
        for g in self.groups:
            idx = g.index if g.index is not None else np.arange(g.first, g.first + g.n)
            nres[idx] = functor_shape(g.kind)[0]
        return nres

    @property
    def num_residuals(self):
        return int(sum(functor_shape(g.kind)[0] * g.n for g in self.groups))

    def block_params_csr(self):
        """(param_begin[nrb+1], param_ids) in program order."""
        nrb = self.num_residual_blocks
        nb = np.zeros(nrb, np.int64)
        for g in self.groups:
            idx = g.index if g.index is not None else np.arange(g.first, g.first + g.n)
            nb[idx] = g.ids.shape[1]
        begin = np.zeros(nrb + 1, np.int64)
        np.cumsum(nb, out=begin[1:])
        ids = np.empty(int(begin[-1]), np.int32)
        for g in self.groups:
            idx = g.index if g.index is not None else np.arange(g.first, g.first + g.n)
            k = g.ids.shape[1]
            pos = begin[idx][:, None] + np.arange(k)[None, :]
            ids[pos.ravel()] = g.ids.ravel()
        return begin, ids

    def parameter_blocks_struct(self):
        npb = self.num_parameter_blocks
        arr = (_cse.cse_parameter_block * max(npb, 1))()
        rec = np.frombuffer(arr, dtype=np.dtype([("size", "<i4"), ("tangent_size", "<i4"),
                                                  ("is_constant", "<i4"), ("manifold", "<i4"),
                                                  ("state_offset", "<i8"),
                                                  ("delta_offset", "<i8"),
                                                  ("plus_jacobian_offset", "<i8")]),
                            count=max(npb, 1))
        if npb:
            rec["size"] = self.pb_size
            rec["tangent_size"] = self.pb_tangent
            rec["is_constant"] = self.pb_constant
            rec["manifold"] = 0 if self.pb_manifold is None else self.pb_manifold
            rec["state_offset"] = self.state_offset
            rec["delta_offset"] = self.delta_offset
            rec["plus_jacobian_offset"] = self.pb_plus_jacobian
        return arr

    def with_explicit_manifolds(self, state=None):
        """The same Program with every MANIFOLD_QUATERNION_EUCLIDEAN block
        given by its explicit plus-Jacobian matrix at `state` (default
        self.state): what the reference uploads for such a block
        (RegisteredCUDAEvaluators::UpdatePlusJacobians,
        registered_cuda_evaluators.cc:139-160, from
        ProductManifold<QuaternionManifold, EuclideanManifold<n>>::PlusJacobian).
        Checkers on the host take this form; the library builds the matrix itself."""
        import copy
        if self.pb_manifold is None or not np.any(self.pb_manifold):
            return self
        state = self.state if state is None else np.asarray(state, np.float64)
        out = copy.copy(self)
        pj_off = self.pb_plus_jacobian.copy()
        vals = [np.asarray(self.plus_jacobians, np.float64).ravel()]
        count = vals[0].size
        const = self.pb_constant != 0
        for b in np.flatnonzero(self.pb_manifold == _cse.MANIFOLD_QUATERNION_EUCLIDEAN):
            size = int(self.pb_size[b])
            src = self.constant_state if const[b] else state
            if self.state_offset is not None:
                off = int(self.state_offset[b])
            else:  # program order of the active / constant blocks
                sel = (const == const[b]) & (np.arange(len(const)) < b)
                off = int(self.pb_size[sel].sum())
            P = quaternion_euclidean_plus_jacobian(src[off:off + size])
            pj_off[b] = count
            vals.append(P.ravel())
            count += P.size
        out.pb_plus_jacobian = pj_off
        out.plus_jacobians = np.concatenate(vals)
        out.pb_manifold = None
        out._keep = []
        return out

    def compile(self, format=BLOCK_SPARSE, num_eliminate_blocks=0):
        """Offsets (program.cc:151-177) and the Jacobian layout tables."""
        self.format = format
        self.num_eliminate_blocks = int(num_eliminate_blocks)
        const = self.pb_constant != 0
        so = np.zeros(self.num_parameter_blocks, np.int64)
        do = np.full(self.num_parameter_blocks, -1, np.int64)
        act_sizes = np.where(const, 0, self.pb_size).astype(np.int64)
        act_tan = np.where(const, 0, self.pb_tangent).astype(np.int64)
        con_sizes = np.where(const, self.pb_size, 0).astype(np.int64)
        so_act = np.cumsum(act_sizes) - act_sizes
        so_con = np.cumsum(con_sizes) - con_sizes
        so[:] = np.where(const, so_con, so_act)
        do[:] = np.where(const, 0, np.cumsum(act_tan) - act_tan)
        self.state_offset, self.delta_offset = so, do
        pbs = self.parameter_blocks_struct()
        begin, ids = self.block_params_csr()
        nres = self.residuals_per_block()
        L = _cse.lib()
        nrb = self.num_residual_blocks
        count = L.cse_layout_offsets_count(self.num_parameter_blocks, pbs, nrb, _ptr(begin, C.c_int64),
                                           _ptr(ids, C.c_int32), _ptr(nres, C.c_int32))
        self.residual_layout = np.empty(nrb, np.int64)
        self.jacobian_per_residual_layout = np.empty(nrb, np.int64)
        self.jacobian_per_residual_offsets = np.empty(max(count, 1), np.int64)
        nvals = C.c_int64(0)
        if format == BLOCK_SPARSE:
            rc = L.cse_block_sparse_layout(
                self.num_parameter_blocks, pbs, nrb, _ptr(begin, C.c_int64), _ptr(ids, C.c_int32),
                _ptr(nres, C.c_int32), self.num_eliminate_blocks,
                _ptr(self.residual_layout, C.c_int64),
                _ptr(self.jacobian_per_residual_layout, C.c_int64),
                _ptr(self.jacobian_per_residual_offsets, C.c_int64), C.byref(nvals))
        elif format == COMPRESSED_ROW:
            self.crs_rows = np.empty(self.num_residuals + 1, np.int64)
            rc = L.cse_compressed_row_layout(
                self.num_parameter_blocks, pbs, nrb, _ptr(begin, C.c_int64), _ptr(ids, C.c_int32),
                _ptr(nres, C.c_int32), _ptr(self.residual_layout, C.c_int64),
                _ptr(self.jacobian_per_residual_layout, C.c_int64),
                _ptr(self.jacobian_per_residual_offsets, C.c_int64), C.byref(nvals),
                _ptr(self.crs_rows, C.c_int64), None)
        else:
            raise ValueError(format)
        _cse.check(rc, "layout")
        self.num_jacobian_offsets = int(count)
        self.num_jacobian_values = int(nvals.value)
        return self

    def descriptor(self):
        """cse_problem_desc over this program (arrays kept alive on self)."""
        assert self.residual_layout is not None, "compile() first"
        keep = []
        groups = (_cse.cse_residual_group * max(len(self.groups), 1))()
        for k, g in enumerate(self.groups):
            ids = np.ascontiguousarray(g.ids, np.int32)
            data = np.ascontiguousarray(g.data, np.float64)
            idx = None if g.index is None else np.ascontiguousarray(g.index, np.int64)
            keep += [ids, data, idx]
            groups[k].functor_kind = g.kind
            groups[k].loss = g.loss.describe()
            groups[k].num_blocks = g.n
            groups[k].residual_block_index = _ptr(idx, C.c_int64)
            groups[k].first_residual_block = g.first
            groups[k].parameter_block_ids = _ptr(ids, C.c_int32)
            groups[k].functor_data = _ptr(data, C.c_double)
        pbs = self.parameter_blocks_struct()
        cstate = np.ascontiguousarray(self.constant_state, np.float64)
        pj = np.ascontiguousarray(self.plus_jacobians, np.float64)
        keep += [groups, pbs, cstate, pj]
        d = _cse.cse_problem_desc()
        d.abi_version = _cse.CSE_ABI_VERSION
        d.num_groups = len(self.groups)
        d.groups = groups
        d.num_parameter_blocks = self.num_parameter_blocks
        d.parameter_blocks = pbs
        d.num_parameters = self.num_parameters
        d.num_effective_parameters = self.num_effective_parameters
        d.num_constant_parameters = self.num_constant_parameters
        d.constant_state = _ptr(cstate, C.c_double)
        d.num_plus_jacobian_values = int(pj.size)
        d.plus_jacobians = _ptr(pj, C.c_double)
        d.num_residual_blocks = self.num_residual_blocks
        d.num_residuals = self.num_residuals
        d.residual_layout = _ptr(self.residual_layout, C.c_int64)
        d.jacobian_per_residual_layout = _ptr(self.jacobian_per_residual_layout, C.c_int64)
        d.jacobian_per_residual_offsets = _ptr(self.jacobian_per_residual_offsets, C.c_int64)
        d.num_jacobian_per_residual_offsets = self.num_jacobian_offsets
        d.num_jacobian_values = self.num_jacobian_values
        self._keep = keep
        return d


def quaternion_euclidean_plus_jacobian(x):
    """PlusJacobian of ProductManifold<QuaternionManifold, EuclideanManifold<n>>
    at x (size 4 + n, tangent 3 + n): QuaternionPlusJacobianImpl
    (internal/ceres/manifold.cc:62-78, Ceres order w, x, y, z) and an
    identity, block-diagonal."""
    x = np.asarray(x, np.float64)
    size = x.size
    P = np.zeros((size, size - 1))
    w, qx, qy, qz = x[:4]
    P[:4, :3] = [[-qx, -qy, -qz], [w, qz, -qy], [-qz, w, qx], [qy, -qx, w]]
    P[4:, 3:] = np.eye(size - 4)
    return P


class ProblemCUDA:
    """Incremental builder with the reference's ProblemCUDA vocabulary."""

    def __init__(self):
        self._sizes, self._tangent, self._const, self._pj_off = [], [], [], []
        self._manifold = []
        self._values = []
        self._pj = []
        self._pj_count = 0
        self._groups = []
        self._nrb = 0

    def add_parameter_block(self, values):
        values = np.asarray(values, np.float64)
        self._sizes.append(values.size)
        self._tangent.append(values.size)
        self._const.append(0)
        self._pj_off.append(-1)
        self._manifold.append(0)
        self._values.append(values.copy())
        return len(self._sizes) - 1

    def set_parameter_block_constant(self, b):
        self._const[b] = 1

    def set_plus_jacobian(self, b, plus_jacobian):
        """Manifold for block b given by its PlusJacobian (size x tangent)."""
        pj = np.asarray(plus_jacobian, np.float64)
        assert pj.shape[0] == self._sizes[b]
        self._tangent[b] = pj.shape[1]
        self._pj_off[b] = self._pj_count
        self._pj.append(pj.ravel())
        self._pj_count += pj.size

    def set_quaternion_euclidean_manifold(self, b):
        """SetManifold(b, ProductManifold<QuaternionManifold,
        EuclideanManifold<size - 4>>): the library builds the plus-Jacobian
        from the block's value (MANIFOLD_QUATERNION_EUCLIDEAN)."""
        assert self._sizes[b] >= 4 and self._pj_off[b] < 0
        self._tangent[b] = self._sizes[b] - 1
        self._manifold[b] = _cse.MANIFOLD_QUATERNION_EUCLIDEAN

    def add_residual_blocks(self, kind, loss, ids, data):
        ids = np.ascontiguousarray(np.asarray(ids, np.int32).reshape(-1, len(functor_shape(kind)[1])))
        data = np.ascontiguousarray(np.asarray(data, np.float64).reshape(ids.shape[0], -1))
        n = ids.shape[0]
        if n and (ids.min() < 0 or ids.max() >= len(self._sizes)):
            raise ValueError("add_residual_blocks: parameter block id out of range")
        if n and ids.shape[1] > 1:
            # ProblemImpl::AddResidualBlock (problem_impl.cc:285-301) refuses a
            # parameter block listed twice in one residual block.
            srt = np.sort(ids, axis=1)
            dup = np.flatnonzero((srt[:, 1:] == srt[:, :-1]).any(axis=1))
            if dup.size:
                raise ValueError(f"add_residual_blocks: duplicate parameter blocks in residual "
                                 f"block {self._nrb + int(dup[0])}: {ids[dup[0]].tolist()}")
        self._groups.append(ResidualGroup(kind, loss or Loss.trivial(), ids, data, None, self._nrb))
        self._nrb += n
        return range(self._nrb - n, self._nrb)

    def add_residual_block(self, kind, loss, data, *blocks):
        return self.add_residual_blocks(kind, loss, [blocks], [data])[0]

    def program(self, group_by_type=True, reduce=True):
        """Program order = insertion order.  Blocks sharing (kind, loss) are
        merged into one group, like the per-type evaluator registry.

        reduce: drop residual blocks whose parameter blocks are all constant,
        as Program::CreateReducedProgram does before evaluation
        (program.cc RemoveFixedBlocks); their cost is the solver's fixed
        cost, not the evaluator's."""
        groups = self._groups
        const_flags = np.array(self._const, np.int32)
        if reduce:
            kept, nrb = [], 0
            for g in groups:
                live = ~np.all(const_flags[g.ids] != 0, axis=1)
                if live.any():
                    kept.append(ResidualGroup(g.kind, g.loss, g.ids[live], g.data[live], None, nrb))
                    nrb += int(live.sum())
            groups = kept
        else:
            nrb = self._nrb
        if group_by_type:
            merged = {}
            for g in groups:
                key = (g.kind,) + g.loss.key()
                idx = np.arange(g.first, g.first + g.n, dtype=np.int64)
                if key in merged:
                    m = merged[key]
                    m.ids = np.concatenate([m.ids, g.ids])
                    m.data = np.concatenate([m.data, g.data])
                    m.index = np.concatenate([m.index, idx])
                else:
                    merged[key] = ResidualGroup(g.kind, g.loss, g.ids, g.data, idx, 0)
            groups = list(merged.values())
            for g in groups:
                if np.array_equal(g.index, np.arange(g.index[0], g.index[0] + g.n)):
                    g.first, g.index = int(g.index[0]), None
        const = np.array(self._const, np.int32)
        values = self._values
        state = np.concatenate([v for v, c in zip(values, const) if not c] or [np.zeros(0)])
        cstate = np.concatenate([v for v, c in zip(values, const) if c] or [np.zeros(0)])
        pj = np.concatenate(self._pj) if self._pj else np.zeros(0)
        prog = Program(np.array(self._sizes, np.int32), np.array(self._tangent, np.int32), const,
                       np.array(self._pj_off, np.int64), pj, groups, nrb, state, cstate)
        if any(self._manifold):
            prog.pb_manifold = np.array(self._manifold, np.int32)
        return prog


# Arrays registered by host_register, by buffer address: the module keeps
# each one alive until host_unregister, so a registered address is never
# freed (and reused) while the library's registry still lists it.
_registered = {}


def host_register(arr):
    """Page-lock a C-contiguous numpy array in place for asynchronous
    transfers (cse_host_register) until host_unregister(arr); the
    multi-device evaluator copies into and out of such buffers without
    staging.  Only an existing ndarray is accepted (no conversion, so it is
    the caller's own buffer that is registered); the module holds a
    reference to it until it is unregistered."""
    if not isinstance(arr, np.ndarray):
        raise TypeError("host_register: a numpy.ndarray (registered in place, never a copy)")
    if not arr.flags.c_contiguous or arr.nbytes == 0:
        raise ValueError("host_register: a non-empty C-contiguous array")
    addr = arr.ctypes.data
    if addr in _registered:
        raise ValueError("host_register: this buffer is already registered")
    _cse.check(_cse.lib().cse_host_register(addr, arr.nbytes), "cse_host_register")
    _registered[addr] = arr
    return arr


def host_unregister(arr):
    if not isinstance(arr, np.ndarray) or arr.ctypes.data not in _registered:
        raise ValueError("host_unregister: not an array registered by host_register")
    addr = arr.ctypes.data
    _cse.check(_cse.lib().cse_host_unregister(addr), "cse_host_unregister")
    del _registered[addr]


class Evaluator:
    """ProgramEvaluatorCUDA seam over libcse.so (program_evaluator_cuda.h:65-183)."""

    def __init__(self, program, device=-1, check_finite=True, apply_loss_function=True,
                 force_general_layout=False, profile=False, stream=None, gradient_mode=0,
                 devices=None, jacobian_form="closed"):
        """devices: a list of HIP ordinals -> one evaluator over several
        devices (cse_create_multi: point-bucket shards, strips copied into
        the caller's one host buffer); repeats put several shards on one
        device.  Only the host-pointer calls work on it.
        jacobian_form: "closed" (the Snavely functor's closed-form Jacobian,
        the default) or "jet" (forward-mode Jet<double, 12>, as
        AutoDifferentiate; cse_options.jacobian_form)."""
        self.program = program
        self.desc = program.descriptor()
        opts = _cse.cse_options()
        L = _cse.lib()
        L.cse_default_options(C.byref(opts))
        opts.device = device
        opts.check_finite = int(check_finite)
        opts.apply_loss_function = int(apply_loss_function)
        opts.force_general_layout = int(force_general_layout)
        opts.profile = int(profile)
        # 0 = fused where eligible (else 1), 1 = post-pass, 2 = atomics (cse.h)
        opts.gradient_mode = int(gradient_mode)
        forms = {"closed": _cse.JACOBIAN_CLOSED_FORM, "jet": _cse.JACOBIAN_JET}
        if jacobian_form not in forms:
            raise ValueError(f"jacobian_form must be one of {sorted(forms)}")
        opts.jacobian_form = forms[jacobian_form]
        # stream: a hipStream_t handle (int) to run on -- 0 is the null stream
        # (torch's default stream); None = an evaluator-owned stream.
        opts.use_stream = int(stream is not None)
        opts.stream = stream if stream else None
        h = C.c_void_p()
        if devices is None:
            _cse.check(L.cse_create(C.byref(self.desc), C.byref(opts), C.byref(h)), "cse_create")
        else:
            if stream is not None:
                raise ValueError("a multi-device evaluator runs on its own per-device streams")
            devs = (C.c_int32 * len(devices))(*devices)
            _cse.check(L.cse_create_multi(C.byref(self.desc), C.byref(opts), devs, len(devices),
                                          C.byref(h)), "cse_create_multi")
        self.handle = h

    def close(self):
        if getattr(self, "handle", None):
            _cse.lib().cse_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self):
        inf = _cse.cse_info()
        _cse.check(_cse.lib().cse_get_info(self.handle, C.byref(inf)), "cse_get_info")
        return inf

    def shard_info(self):
        """(first block of each shard + the end, device of each shard)."""
        L = _cse.lib()
        n = C.c_int32()
        _cse.check(L.cse_shard_info(self.handle, C.byref(n), None, None), "cse_shard_info")
        first = np.empty(n.value + 1, np.int64)
        devs = np.empty(n.value, np.int32)
        _cse.check(L.cse_shard_info(self.handle, C.byref(n), _ptr(first, C.c_int64),
                                    _ptr(devs, C.c_int32)), "cse_shard_info")
        return first, devs

    def transfer_bytes(self):
        """Per shard: (state bytes copied to its device, strip bytes copied
        back) by one host-pointer evaluate (cse_shard_transfer_bytes)."""
        first, _ = self.shard_info()
        n = len(first) - 1
        h2d = np.empty(n, np.int64)
        d2h = np.empty(n, np.int64)
        _cse.check(_cse.lib().cse_shard_transfer_bytes(self.handle, _ptr(h2d, C.c_int64),
                                                        _ptr(d2h, C.c_int64)),
                   "cse_shard_transfer_bytes")
        return h2d, d2h

    def evaluate(self, state=None, residuals=True, gradient=True, jacobian=True, out=None,
                 new_evaluation_point=True):
        """Host-pointer Evaluate.  Returns (ok, cost, residuals, gradient, jacobian).
        out: optional (r, g, j) float64 arrays to write into (None entries are
        allocated), e.g. buffers kept across calls.  new_evaluation_point=False:
        the state equals the previous evaluation's (Evaluator::EvaluateOptions,
        evaluator.h:106-107; cse_evaluate_ex with CSE_EVAL_SAME_POINT)."""
        p = self.program
        state = np.ascontiguousarray(p.state if state is None else state, np.float64)
        cost = C.c_double(-1.0)
        ro, go, jo = out if out is not None else (None, None, None)
        r = (ro if ro is not None else np.empty(p.num_residuals)) if residuals else None
        g = (go if go is not None else np.empty(p.num_effective_parameters)) if gradient else None
        j = (jo if jo is not None else np.empty(p.num_jacobian_values)) if jacobian else None
        flags = 0 if new_evaluation_point else _cse.EVAL_SAME_POINT
        rc = _cse.lib().cse_evaluate_ex(self.handle, _ptr(state, C.c_double), C.byref(cost),
                                        _ptr(r, C.c_double), _ptr(g, C.c_double),
                                        _ptr(j, C.c_double), flags)
        _cse.check(rc, "cse_evaluate")
        return rc == _cse.CSE_OK, cost.value, r, g, j

    def evaluate_device(self, d_state, d_cost, d_residuals=None, d_gradient=None, d_jacobian=None,
                        new_evaluation_point=True):
        """Device-pointer Evaluate (integers = device addresses).  Async.
        new_evaluation_point=False: CSE_EVAL_SAME_POINT (see evaluate)."""
        if new_evaluation_point:
            rc = _cse.lib().cse_evaluate_device(self.handle, d_state, d_cost, d_residuals,
                                                d_gradient, d_jacobian)
        else:
            rc = _cse.lib().cse_evaluate_device_ex(self.handle, d_state, d_cost, d_residuals,
                                                   d_gradient, d_jacobian, _cse.EVAL_SAME_POINT)
        return _cse.check(rc, "cse_evaluate_device")

    def wait(self):
        return _cse.check(_cse.lib().cse_wait(self.handle), "cse_wait")

    def plus(self, state, delta, out=None):
        """Evaluator::Plus (program.cc:121-149) on the GPU, host arrays.
        out: the result array (C-contiguous float64, the state's size); it may
        be `state` itself (Plus(x, delta, x), as Ceres' line search and
        dogleg steps call it)."""
        state = np.ascontiguousarray(state, np.float64)
        delta = np.ascontiguousarray(delta, np.float64)
        if out is None:
            out = np.empty_like(state)
        elif (not isinstance(out, np.ndarray) or out.dtype != np.float64 or
              not out.flags.c_contiguous or out.size != state.size):
            raise ValueError("plus: out must be a C-contiguous float64 array of the state's size")
        _cse.check(_cse.lib().cse_plus(self.handle, _ptr(state, C.c_double),
                                       _ptr(delta, C.c_double), _ptr(out, C.c_double)), "cse_plus")
        return out

    def right_multiply_device(self, d_jacobian, d_x, d_y):
        """y += J x on the device (CudaSparseMatrix::RightMultiplyAndAccumulate)."""
        return _cse.check(_cse.lib().cse_jacobian_right_multiply(self.handle, d_jacobian, d_x, d_y),
                          "cse_jacobian_right_multiply")

    def left_multiply_device(self, d_jacobian, d_x, d_y):
        """y += J^T x on the device (CudaSparseMatrix::LeftMultiplyAndAccumulate)."""
        return _cse.check(_cse.lib().cse_jacobian_left_multiply(self.handle, d_jacobian, d_x, d_y),
                          "cse_jacobian_left_multiply")

    def cgnr_multiply_device(self, d_jacobian, d_D, d_x, d_y):
        """y += J^T (J x) + D.*D.*x on the device, d_D may be None
        (CudaCgnrLinearOperator::RightMultiplyAndAccumulate, cgnr_solver.cc:226-237)."""
        return _cse.check(_cse.lib().cse_cgnr_multiply(self.handle, d_jacobian, d_D, d_x, d_y),
                          "cse_cgnr_multiply")

    # ---- ITERATIVE_SCHUR (ImplicitSchurComplement on the device) ----------
    def schur_structure(self):
        """(num_cols_e, num_cols_f) of the Schur split; raises if the problem
        does not have the structure (cse_schur_structure)."""
        e, f = C.c_int64(), C.c_int64()
        _cse.check(_cse.lib().cse_schur_structure(self.handle, C.byref(e), C.byref(f)),
                   "cse_schur_structure")
        return e.value, f.value

    def schur_init_device(self, d_jacobian, d_D, d_b, d_rhs, preconditioner=_cse.SCHUR_JACOBI):
        """ImplicitSchurComplement::Init(A, D, b) + the preconditioner; writes
        the reduced right-hand side (num_cols_f) to d_rhs."""
        return _cse.check(_cse.lib().cse_schur_init(self.handle, d_jacobian, d_D, d_b, d_rhs,
                                                    int(preconditioner)), "cse_schur_init")

    def schur_init_gradient_device(self, d_jacobian, d_D, d_b, d_rhs, d_gradient,
                                   preconditioner=_cse.SCHUR_JACOBI):
        """schur_init_device plus the gradient g = J^T r (r = -b) into
        d_gradient, in the same pass (cse_schur_init_gradient)."""
        return _cse.check(_cse.lib().cse_schur_init_gradient(self.handle, d_jacobian, d_D, d_b,
                                                             d_rhs, int(preconditioner),
                                                             d_gradient),
                          "cse_schur_init_gradient")

    def schur_multiply_device(self, d_x, d_y):
        """y = S x (ImplicitSchurComplement::RightMultiplyAndAccumulate)."""
        return _cse.check(_cse.lib().cse_schur_multiply(self.handle, d_x, d_y),
                          "cse_schur_multiply")

    def schur_precondition_device(self, d_x, d_y):
        """y += M^-1 x for the preconditioner chosen at init."""
        return _cse.check(_cse.lib().cse_schur_precondition(self.handle, d_x, d_y),
                          "cse_schur_precondition")

    def schur_back_substitute_device(self, d_x, d_y):
        """y = [(E^T E + D_e^2)^-1 E^T (b - F x); x] (BackSubstitute)."""
        return _cse.check(_cse.lib().cse_schur_back_substitute(self.handle, d_x, d_y),
                          "cse_schur_back_substitute")

    def plus_device(self, d_state, d_delta, d_out):
        """Device-pointer Plus on the evaluator's stream.  Async."""
        return _cse.check(_cse.lib().cse_plus_device(self.handle, d_state, d_delta, d_out),
                          "cse_plus_device")

    def kernel_stats(self):
        last, total, n = C.c_double(), C.c_double(), C.c_int64()
        _cse.check(_cse.lib().cse_kernel_stats(self.handle, C.byref(last), C.byref(total),
                                               C.byref(n)), "cse_kernel_stats")
        return last.value, total.value, n.value

    def reset_kernel_stats(self):
        _cse.check(_cse.lib().cse_reset_kernel_stats(self.handle), "cse_reset_kernel_stats")
