"""The reference's evaluator known-answer tests
(internal/ceres/evaluator_test.cc:227-533), on the oracle and on the
product's host-side layout builders.

ParameterIgnoringCostFunction<kFactor, kR, Ns...> returns r_i = i + 1 and
Jacobian columns kFactor * (j + 1); the oracle's LINEAR_TEST functor
reproduces it exactly at the zero state the test evaluates at.  Every case
runs for each (Jacobian format, num_eliminate_blocks) the reference
instantiates (:560-580) and all 8 combinations of requested outputs
(:207-218), comparing the densified Jacobian with the expected matrix.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_py as O

SETTINGS = [(O.BLOCK_SPARSE, e) for e in range(5)] + [(O.COMPRESSED_ROW, 0)]


def make(blocks, residuals, constant=(), manifolds=None):
    """blocks: sizes in program order; residuals: (kFactor, kR, [block ids])."""
    manifolds = manifolds or {}
    sizes = list(blocks)
    tangent = list(blocks)
    pj_off = [-1] * len(blocks)
    pj = []
    for b, P in manifolds.items():
        P = np.asarray(P, float)
        tangent[b] = P.shape[1]
        pj_off[b] = len(pj)
        pj += list(P.ravel())
    const = [1 if b in constant else 0 for b in range(len(blocks))]
    kind, pbeg, params, dbeg, data = [], [0], [], [0], []
    for k_factor, nres, ids in residuals:
        kind.append(O.LINEAR_TEST)
        params += ids
        pbeg.append(len(params))
        data += [k_factor, nres]
        dbeg.append(len(data))
    n = len(residuals)

    def program(fmt, elim):
        return O.OracleProgram(sizes, tangent, const, pj_off, pj or [0.0], kind, [0] * n,
                               [1.0] * n, [1.0] * n, [0] * n, pbeg, params, dbeg, data, fmt, elim)
    return program


def densify(prog, values):
    s = prog.sizes()
    lay, offs, _, _ = prog.jacobian_offsets()
    a = prog.a
    dense = np.zeros((s.num_residuals, s.num_effective_parameters))
    delta = np.cumsum(np.where(a["pb_constant"] == 1, 0, a["pb_tangent"])) - \
        np.where(a["pb_constant"] == 1, 0, a["pb_tangent"])
    row = 0
    for i in range(len(a["kind"])):
        nres = int(a["data"][a["dbeg"][i] + 1])
        t = lay[i]
        for q in range(a["pbeg"][i], a["pbeg"][i + 1]):
            b = a["params"][q]
            if a["pb_constant"][b]:
                continue
            tan = a["pb_tangent"][b]
            for k in range(nres):
                dense[row + k, delta[b]:delta[b] + tan] = values[offs[t]:offs[t] + tan]
                t += 1
        row += nres
    return dense


def check_all(program, rows, cols, cost, residuals, gradient, jacobian):
    jacobian = np.asarray(jacobian, float).reshape(rows, cols)
    for fmt, elim in SETTINGS:
        prog = program(fmt, elim)
        s = prog.sizes()
        assert (s.num_residuals, s.num_effective_parameters) == (rows, cols)
        state = np.zeros(s.num_parameters)
        cstate = np.zeros(max(s.num_constant_parameters, 1))
        for combo in range(8):
            ok, c, r, g, j = prog.evaluate(state, cstate, residuals=bool(combo & 1),
                                           gradient=bool(combo & 2), jacobian=bool(combo & 4))
            assert ok
            assert c == cost
            if combo & 1:
                assert np.array_equal(r, residuals)
            if combo & 2:
                assert np.array_equal(g, gradient)
            if combo & 4:
                assert np.array_equal(densify(prog, j), jacobian), (fmt, elim)


def test_single_residual_problem():
    # evaluator_test.cc:227-253
    check_all(make([2, 3, 4], [(1, 3, [0, 1, 2])]), 3, 9, 7.0, [1, 2, 3],
              [6, 12, 6, 12, 18, 6, 12, 18, 24],
              [1, 2, 1, 2, 3, 1, 2, 3, 4] * 3)


def test_single_residual_problem_with_permuted_parameters():
    # evaluator_test.cc:255-290: cost function arguments (z, y, x)
    check_all(make([2, 3, 4], [(1, 3, [2, 1, 0])]), 3, 9, 7.0, [1, 2, 3],
              [6, 12, 6, 12, 18, 6, 12, 18, 24],
              [1, 2, 1, 2, 3, 1, 2, 3, 4] * 3)


def test_single_residual_problem_with_nuisance_parameters():
    # evaluator_test.cc:292-336: blocks a, x, b, y, c, z, d
    check_all(make([2, 2, 1, 3, 1, 4, 3], [(1, 3, [1, 3, 5])]), 3, 16, 7.0, [1, 2, 3],
              [0, 0, 6, 12, 0, 6, 12, 18, 0, 6, 12, 18, 24, 0, 0, 0],
              [0, 0, 1, 2, 0, 1, 2, 3, 0, 1, 2, 3, 4, 0, 0, 0] * 3)


MULTI = [(1, 2, [0, 1]), (2, 3, [0, 2]), (3, 4, [1, 2])]
MULTI_COST = (1 + 4 + 1 + 4 + 9 + 1 + 4 + 9 + 16) / 2.0
MULTI_RES = [1, 2, 1, 2, 3, 1, 2, 3, 4]


def test_multiple_residual_problem():
    # evaluator_test.cc:338-390
    J = ([1, 2, 1, 2, 3, 0, 0, 0, 0] * 2 + [2, 4, 0, 0, 0, 2, 4, 6, 8] * 3 +
         [0, 0, 3, 6, 9, 3, 6, 9, 12] * 4)
    check_all(make([2, 3, 4], MULTI), 9, 9, MULTI_COST, MULTI_RES,
              [15, 30, 33, 66, 99, 42, 84, 126, 168], J)


def test_multiple_residuals_with_manifolds():
    # evaluator_test.cc:392-454: SubsetManifold(3, {0}) on y,
    # SubsetManifold(4, {1}) on z, given by their plus-Jacobians.
    Py = [[0, 0], [1, 0], [0, 1]]
    Pz = [[1, 0, 0], [0, 0, 0], [0, 1, 0], [0, 0, 1]]
    J = ([1, 2, 2, 3, 0, 0, 0] * 2 + [2, 4, 0, 0, 2, 6, 8] * 3 + [0, 0, 6, 9, 3, 9, 12] * 4)
    check_all(make([2, 3, 4], MULTI, manifolds={1: Py, 2: Pz}), 9, 7, MULTI_COST, MULTI_RES,
              [15, 30, 66, 99, 42, 126, 168], J)


def test_multiple_residual_problem_with_some_constant_parameters():
    # evaluator_test.cc:456-518: z constant
    J = [1, 2, 1, 2, 3] * 2 + [2, 4, 0, 0, 0] * 3 + [0, 0, 3, 6, 9] * 4
    check_all(make([2, 3, 4], MULTI, constant={2}), 9, 5, MULTI_COST, MULTI_RES,
              [15, 30, 33, 66, 99], J)


def _product_offsets(program_fn, fmt, elim):
    """The product's layout builders (libcse.so, host code) on the same program."""
    from ceres_amd import _cse
    prog = program_fn(fmt, elim)
    a = prog.a
    npb = len(a["pb_size"])
    pbs = (_cse.cse_parameter_block * npb)()
    delta = 0
    so, cso = 0, 0
    for b in range(npb):
        pbs[b].size = int(a["pb_size"][b])
        pbs[b].tangent_size = int(a["pb_tangent"][b])
        pbs[b].is_constant = int(a["pb_constant"][b])
        pbs[b].plus_jacobian_offset = int(a["pb_pj"][b])
        if a["pb_constant"][b]:
            pbs[b].state_offset = cso
            cso += int(a["pb_size"][b])
        else:
            pbs[b].state_offset, pbs[b].delta_offset = so, delta
            so += int(a["pb_size"][b])
            delta += int(a["pb_tangent"][b])
    nrb = len(a["kind"])
    nres = np.array([int(a["data"][a["dbeg"][i] + 1]) for i in range(nrb)], np.int32)
    pbeg, params = a["pbeg"], a["params"]
    L = _cse.lib()
    P = lambda x, t: x.ctypes.data_as(C.POINTER(t))
    n = L.cse_layout_offsets_count(npb, pbs, nrb, P(pbeg, C.c_int64), P(params, C.c_int32),
                                   P(nres, C.c_int32))
    rl = np.empty(nrb, np.int64)
    lay = np.empty(nrb, np.int64)
    offs = np.empty(n, np.int64)
    nv = C.c_int64()
    if fmt == O.BLOCK_SPARSE:
        rc = L.cse_block_sparse_layout(npb, pbs, nrb, P(pbeg, C.c_int64), P(params, C.c_int32),
                                       P(nres, C.c_int32), elim, P(rl, C.c_int64),
                                       P(lay, C.c_int64), P(offs, C.c_int64), C.byref(nv))
        rows = cols = None
    else:
        s = prog.sizes()
        rows = np.empty(s.num_residuals + 1, np.int64)
        cols = np.empty(s.num_jacobian_values, np.int64)
        rc = L.cse_compressed_row_layout(npb, pbs, nrb, P(pbeg, C.c_int64), P(params, C.c_int32),
                                         P(nres, C.c_int32), P(rl, C.c_int64), P(lay, C.c_int64),
                                         P(offs, C.c_int64), C.byref(nv), P(rows, C.c_int64),
                                         P(cols, C.c_int64))
    assert rc == 0
    return prog, lay, offs, nv.value, rows, cols


@pytest.mark.parametrize("case", [
    make([2, 3, 4], [(1, 3, [0, 1, 2])]),
    make([2, 3, 4], [(1, 3, [2, 1, 0])]),
    make([2, 2, 1, 3, 1, 4, 3], [(1, 3, [1, 3, 5])]),
    make([2, 3, 4], MULTI),
    make([2, 3, 4], MULTI, constant={2}),
    make([2, 3, 4], MULTI, constant={0}),
    make([2, 3, 4], MULTI, manifolds={1: [[0, 0], [1, 0], [0, 1]]}),
])
def test_product_layout_builders_match_reference_writers(case):
    for fmt, elim in SETTINGS:
        prog, lay, offs, nv, rows, cols = _product_offsets(case, fmt, elim)
        olay, ooffs, orows, ocols = prog.jacobian_offsets()
        assert np.array_equal(lay, olay)
        assert np.array_equal(offs, ooffs[:len(offs)])
        assert nv == prog.sizes().num_jacobian_values
        if rows is not None:
            assert np.array_equal(rows, orows) and np.array_equal(cols, ocols)
