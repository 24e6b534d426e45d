"""The reference's own known answers, run through libcse.so (the HIP path).

* internal/ceres/evaluator_test.cc:227-553 -- the six EvaluatorTest problems
  (ParameterIgnoringCostFunction, as the library's TEST_LINEAR_* functor
  kinds, which reproduce the fake exactly at the zero state the test
  evaluates at), for every (Jacobian format, num_eliminate_blocks) setting
  of tests/test_evaluator_kat.py and all 8 combinations of requested outputs
  (CheckAllEvaluationCombinations, :207-218); the expected cost, residuals,
  gradient and densified Jacobian are the test's hard-coded values, compared
  exactly.  Plus EvaluatorAbortsForResidualsThatFailToEvaluate (:535-553).
* internal/ceres/autodiff_cost_function_cuda_test.cu.cc -- BilinearDifferentiationTest
  (:81-116: residual 10, J = [3 4] and [1 2]), ManyParameterAutodiffInstantiates
  (:141-222: residual 45, ten unit Jacobians) and
  PartiallyFilledResidualShouldFailEvaluation (:247-292: an unassigned
  output fails the evaluation), each as a one-block Program through the
  evaluator (the reference calls the cost function directly; here the
  autodiff runs inside the product kernel).
"""
import numpy as np
import pytest

import ceres_amd as ca
from ceres_amd import _cse

pytestmark = pytest.mark.gpu

# (format, num_eliminate_blocks): the settings tests/test_evaluator_kat.py
# runs on the oracle (evaluator_test.cc:560-580, minus the dense matrix).
SETTINGS = [(ca.BLOCK_SPARSE, e) for e in range(5)] + [(ca.COMPRESSED_ROW, 0)]

KIND_OF = {  # (kR, sizes) -> functor kind
    (3, (2, 3, 4)): _cse.TEST_LINEAR_3_2_3_4,
    (3, (4, 3, 2)): _cse.TEST_LINEAR_3_4_3_2,
    (2, (2, 3)): _cse.TEST_LINEAR_2_2_3,
    (3, (2, 4)): _cse.TEST_LINEAR_3_2_4,
    (4, (3, 4)): _cse.TEST_LINEAR_4_3_4,
}


def build(blocks, residuals, constant=(), manifolds=None, values=None, kinds=None,
          succeeds=True):
    """blocks: parameter block sizes in program order; residuals:
    (kFactor, kR, [block ids]).  Returns a function (format, elim) ->
    compiled Program."""
    manifolds = manifolds or {}

    def make(fmt, elim):
        p = ca.ProblemCUDA()
        ids = []
        for b, n in enumerate(blocks):
            v = np.zeros(n) if values is None else np.asarray(values[b], float)
            ids.append(p.add_parameter_block(v))
        for b, P in manifolds.items():
            p.set_plus_jacobian(ids[b], np.asarray(P, float))
        for k_factor, nres, bl in residuals:
            kind = KIND_OF[(nres, tuple(blocks[b] for b in bl))] if kinds is None else kinds
            data = [k_factor, 1.0 if succeeds else 0.0] if kinds is None else [k_factor]
            p.add_residual_block(kind, None, data, *[ids[b] for b in bl])
        for b in constant:
            p.set_parameter_block_constant(ids[b])
        prog = p.program(group_by_type=False)
        prog.compile(fmt, num_eliminate_blocks=elim)
        return prog
    return make


def densify(prog, values):
    """Dense J from the Program's layout tables (jacobian_per_residual_*,
    the reference's WriteJacobians addressing)."""
    begin, params = prog.block_params_csr()
    nres = prog.residuals_per_block()
    const = prog.pb_constant != 0
    dense = np.zeros((prog.num_residuals, prog.num_effective_parameters))
    offs = prog.jacobian_per_residual_offsets
    for i in range(prog.num_residual_blocks):
        row = prog.residual_layout[i]
        t = prog.jacobian_per_residual_layout[i]
        for q in range(begin[i], begin[i + 1]):
            b = params[q]
            if const[b]:
                continue
            d0, tan = prog.delta_offset[b], prog.pb_tangent[b]
            for k in range(nres[i]):
                dense[row + k, d0:d0 + tan] = values[offs[t]:offs[t] + tan]
                t += 1
    return dense


def check_all(make, rows, cols, cost, residuals, gradient, jacobian):
    jacobian = np.asarray(jacobian, float).reshape(rows, cols)
    for fmt, elim in SETTINGS:
        prog = make(fmt, elim)
        assert (prog.num_residuals, prog.num_effective_parameters) == (rows, cols)
        ev = ca.Evaluator(prog)
        try:
            assert ev.info().num_affine_groups == 0  # the general (table) kernel
            for combo in range(8):
                ok, c, r, g, j = ev.evaluate(residuals=bool(combo & 1), gradient=bool(combo & 2),
                                             jacobian=bool(combo & 4))
                assert ok, (fmt, elim, combo)
                assert c == cost, (fmt, elim, combo, c)
                if combo & 1:
                    assert np.array_equal(r, residuals), (fmt, elim, combo, r)
                if combo & 2:
                    assert np.array_equal(g, gradient), (fmt, elim, combo, g)
                if combo & 4:
                    assert np.array_equal(densify(prog, j), jacobian), (fmt, elim, combo)
        finally:
            ev.close()


def test_single_residual_problem(gpu):
    # evaluator_test.cc:227-253
    check_all(build([2, 3, 4], [(1, 3, [0, 1, 2])]), 3, 9, 7.0, [1, 2, 3],
              [6, 12, 6, 12, 18, 6, 12, 18, 24], [1, 2, 1, 2, 3, 1, 2, 3, 4] * 3)


def test_single_residual_problem_with_permuted_parameters(gpu):
    # evaluator_test.cc:255-290: cost function arguments (z, y, x)
    check_all(build([2, 3, 4], [(1, 3, [2, 1, 0])]), 3, 9, 7.0, [1, 2, 3],
              [6, 12, 6, 12, 18, 6, 12, 18, 24], [1, 2, 1, 2, 3, 1, 2, 3, 4] * 3)


def test_single_residual_problem_with_nuisance_parameters(gpu):
    # evaluator_test.cc:292-336: blocks a, x, b, y, c, z, d (a..d unused)
    check_all(build([2, 2, 1, 3, 1, 4, 3], [(1, 3, [1, 3, 5])]), 3, 16, 7.0, [1, 2, 3],
              [0, 0, 6, 12, 0, 6, 12, 18, 0, 6, 12, 18, 24, 0, 0, 0],
              [0, 0, 1, 2, 0, 1, 2, 3, 0, 1, 2, 3, 4, 0, 0, 0] * 3)


MULTI = [(1, 2, [0, 1]), (2, 3, [0, 2]), (3, 4, [1, 2])]
MULTI_COST = (1 + 4 + 1 + 4 + 9 + 1 + 4 + 9 + 16) / 2.0
MULTI_RES = [1, 2, 1, 2, 3, 1, 2, 3, 4]


def test_multiple_residual_problem(gpu):
    # evaluator_test.cc:338-390
    J = ([1, 2, 1, 2, 3, 0, 0, 0, 0] * 2 + [2, 4, 0, 0, 0, 2, 4, 6, 8] * 3 +
         [0, 0, 3, 6, 9, 3, 6, 9, 12] * 4)
    check_all(build([2, 3, 4], MULTI), 9, 9, MULTI_COST, MULTI_RES,
              [15, 30, 33, 66, 99, 42, 84, 126, 168], J)


def test_multiple_residuals_with_manifolds(gpu):
    # evaluator_test.cc:392-454: SubsetManifold(3, {0}) on y and
    # SubsetManifold(4, {1}) on z, given by their plus-Jacobians.
    Py = [[0, 0], [1, 0], [0, 1]]
    Pz = [[1, 0, 0], [0, 0, 0], [0, 1, 0], [0, 0, 1]]
    J = [1, 2, 2, 3, 0, 0, 0] * 2 + [2, 4, 0, 0, 2, 6, 8] * 3 + [0, 0, 6, 9, 3, 9, 12] * 4
    check_all(build([2, 3, 4], MULTI, manifolds={1: Py, 2: Pz}), 9, 7, MULTI_COST, MULTI_RES,
              [15, 30, 66, 99, 42, 126, 168], J)


def test_multiple_residual_problem_with_some_constant_parameters(gpu):
    # evaluator_test.cc:456-518: z constant
    J = [1, 2, 1, 2, 3] * 2 + [2, 4, 0, 0, 0] * 3 + [0, 0, 3, 6, 9] * 4
    check_all(build([2, 3, 4], MULTI, constant={2}), 9, 5, MULTI_COST, MULTI_RES,
              [15, 30, 33, 66, 99], J)


def test_evaluator_aborts_for_residuals_that_fail_to_evaluate(gpu):
    # evaluator_test.cc:535-553: ParameterIgnoringCostFunction<20, 3, 2, 3, 4>(false)
    make = build([2, 3, 4], [(20, 3, [0, 1, 2])], succeeds=False)
    for fmt, elim in SETTINGS:
        ev = ca.Evaluator(make(fmt, elim))
        try:
            for combo in range(8):
                ok, *_ = ev.evaluate(residuals=bool(combo & 1), gradient=bool(combo & 2),
                                     jacobian=bool(combo & 4))
                assert not ok, (fmt, elim, combo)
        finally:
            ev.close()


def one_block(kind, values, data):
    p = ca.ProblemCUDA()
    ids = [p.add_parameter_block(v) for v in values]
    p.add_residual_block(kind, None, data, *ids)
    prog = p.program()
    prog.compile(ca.COMPRESSED_ROW)
    return prog


def test_bilinear_differentiation(gpu):
    # autodiff_cost_function_cuda_test.cu.cc:81-116: x = (1, 2), y = (3, 4),
    # cost = x.y - 1 = 10, dcost/dx = (3, 4), dcost/dy = (1, 2).
    prog = one_block(_cse.TEST_BILINEAR_1_2_2, [[1.0, 2.0], [3.0, 4.0]], [1.0])
    ev = ca.Evaluator(prog)
    ok, cost, r, g, j = ev.evaluate(jacobian=False, gradient=False)
    assert ok and r[0] == 10.0 and cost == 50.0
    ok, cost, r, g, j = ev.evaluate()
    ev.close()
    assert ok and r[0] == 10.0
    assert np.array_equal(densify(prog, j), [[3.0, 4.0, 1.0, 2.0]])
    assert np.array_equal(g, [30.0, 40.0, 10.0, 20.0])


def test_many_parameter_autodiff_instantiates(gpu):
    # autodiff_cost_function_cuda_test.cu.cc:141-222: ten size-1 blocks
    # x_i = i, cost = sum = 45, every Jacobian 1.
    prog = one_block(_cse.TEST_TEN_PARAMETER_1_x10, [[float(i)] for i in range(10)], [0.0])
    ev = ca.Evaluator(prog)
    ok, cost, r, g, j = ev.evaluate(jacobian=False, gradient=False)
    assert ok and r[0] == 45.0
    ok, cost, r, g, j = ev.evaluate()
    ev.close()
    assert ok and r[0] == 45.0
    assert np.array_equal(densify(prog, j), np.ones((1, 10)))


@pytest.mark.parametrize("jacobian", [False, True])
def test_partially_filled_residual_fails_evaluation(gpu, jacobian):
    # autodiff_cost_function_cuda_test.cu.cc:247-292: the functor assigns
    # output[0] only; AutoDifferentiate's kImpossibleValue pre-fill is left in
    # output[1] and ResidualBlock::Evaluate rejects the block.
    prog = one_block(_cse.TEST_PARTIAL_OUTPUT_2_1, [[1.0]], [0.0])
    for check_finite in (True, False):
        ev = ca.Evaluator(prog, check_finite=check_finite)
        ok, *_ = ev.evaluate(jacobian=jacobian, gradient=jacobian)
        ev.close()
        assert not ok


def test_test_kinds_refuse_robust_losses(gpu):
    p = ca.ProblemCUDA()
    x = p.add_parameter_block([1.0, 2.0])
    y = p.add_parameter_block([3.0, 4.0])
    p.add_residual_block(_cse.TEST_BILINEAR_1_2_2, ca.Loss.huber(1.0), [1.0], x, y)
    prog = p.program()
    prog.compile(ca.COMPRESSED_ROW)
    with pytest.raises(RuntimeError, match="trivial loss"):
        ca.Evaluator(prog)
