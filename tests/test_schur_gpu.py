"""GPU: ITERATIVE_SCHUR's operators on the evaluator's Jacobian.

cse_schur_* replace ImplicitSchurComplement (internal/ceres/
implicit_schur_complement.cc) and the IDENTITY / JACOBI / SCHUR_JACOBI
preconditioners of IterativeSchurComplementSolver
(iterative_schur_complement_solver.cc:172-204, schur_jacobi_preconditioner.cc)
on the values the evaluator wrote in HBM.  Checked against dense numpy
formulas built from the Jacobian the evaluator returned:
    S   = F^T F + D_f^2 - F^T E (E^T E + D_e^2)^-1 E^T F
    rhs = F^T (b - E (E^T E + D_e^2)^-1 E^T b)
    back substitution y_e = (E^T E + D_e^2)^-1 E^T (b - F x)
on BAL-shaped problems with short point runs and with runs longer than a
wave (the big-run kernel, 64 and 65 rows at the boundary), and end to end:
a Jacobi-preconditioned CG on S plus back substitution solves
(J^T J + D^2) dx = J^T b like a dense solve.
"""
import numpy as np
import pytest

import ceres_amd as ca
from ceres_amd import _cse, bal

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from test_spmv_gpu import dense_jacobian  # noqa: E402

RTOL = 1e-12


def runs_problem(seed=3):
    """Points with 1 .. 130 observations (runs shorter and longer than a wave),
    each point seen by distinct cameras."""
    rng = np.random.default_rng(seed)
    counts = [1, 2, 70, 3, 130, 64, 65, 5, 4, 6, 63, 1, 66, 2] + list(rng.integers(1, 9, 120))
    C = 140
    P = len(counts)
    cams, pts, _, _, _ = bal.synthetic(C, P, P, seed=seed)
    ci = np.concatenate([rng.permutation(C)[:k] for k in counts]).astype(np.int32)
    pi = np.repeat(np.arange(P, dtype=np.int32), counts)
    obs = bal.project(cams, pts, ci, pi) + rng.normal(0, 1.0, (len(ci), 2))
    return bal.program(cams, pts, ci, pi, obs, loss=ca.Loss.huber(1.0))


def dense_schur(J, e_cols, D, b):
    E, F = J[:, :e_cols], J[:, e_cols:]
    De, Df = D[:e_cols], D[e_cols:]
    Minv = np.linalg.inv(E.T @ E + np.diag(De * De))
    S = F.T @ F + np.diag(Df * Df) - F.T @ E @ Minv @ E.T @ F
    rhs = F.T @ (b - E @ Minv @ (E.T @ b))
    return E, F, Minv, S, rhs


def block_inverse(A, size):
    out = np.zeros_like(A)
    for k in range(0, A.shape[0], size):
        out[k:k + size, k:k + size] = np.linalg.inv(A[k:k + size, k:k + size])
    return out


def close(a, b, tol=RTOL):
    return np.linalg.norm(a - b) <= tol * max(np.linalg.norm(b), 1e-300)


def user_kind_program(name="SnavelyReprojectionError/Huber"):
    """The BAL problem with a user functor kind of the Snavely shape
    (examples/user_functors.hip): the operators read only the Jacobian.
    (BundlerResidual's 9 x 9 camera blocks of F^T F reach condition numbers
    near 1e10 on this problem, beyond the preconditioner check's 1e-11.)"""
    import dataclasses
    import user_functors as U
    prog = bal.synthetic_program((10, 300, 1500), loss=ca.Loss.huber(1.0), seed=9)
    prog.groups = [dataclasses.replace(g, kind=U.kind(name)) for g in prog.groups]
    return prog


@pytest.mark.parametrize("which", ["bal", "runs", "quaternion", "user"])
@pytest.mark.parametrize("precond", [_cse.SCHUR_IDENTITY, _cse.SCHUR_JACOBI,
                                     _cse.SCHUR_SCHUR_JACOBI])
def test_schur_operators_match_dense(gpu, which, precond):
    # quaternion: cameras on ProductManifold<QuaternionManifold, EuclideanManifold<6>>
    # (9 tangent columns per f block, as the angle-axis camera).  user: the
    # Snavely functor as a user kind (its own TU) on the same operators.
    prog = (runs_problem() if which == "runs" else user_kind_program() if which == "user" else
            bal.synthetic_program((10, 300, 1500), loss=ca.Loss.huber(1.0), seed=9,
                                  quaternion_manifold=which == "quaternion"))
    dev = torch.device("cuda", 0)
    ev = ca.Evaluator(prog, stream=torch.cuda.current_stream(dev).cuda_stream)
    ok, cost, r, g, jv = ev.evaluate()
    assert ok
    J = dense_jacobian(prog, jv)
    n, m = prog.num_effective_parameters, prog.num_residuals
    e_cols, f_cols = ev.schur_structure()
    assert e_cols % 3 == 0 and e_cols + f_cols == n and f_cols % 9 == 0
    rng = np.random.default_rng(1)
    D = rng.uniform(0.1, 2.0, n)
    b = rng.normal(size=m)
    x = rng.normal(size=f_cols)
    y0 = rng.normal(size=f_cols)
    E, F, Minv, S, rhs = dense_schur(J, e_cols, D, b)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    dj, dD, db, dx = t(jv), t(D), t(b), t(x)
    drhs = torch.empty(f_cols, dtype=torch.float64, device=dev)
    dy = torch.empty(f_cols, dtype=torch.float64, device=dev)
    dy2 = torch.empty(f_cols, dtype=torch.float64, device=dev)
    dp = t(y0)
    dback = torch.empty(n, dtype=torch.float64, device=dev)
    ev.schur_init_device(dj.data_ptr(), dD.data_ptr(), db.data_ptr(), drhs.data_ptr(), precond)
    ev.schur_multiply_device(dx.data_ptr(), dy.data_ptr())
    ev.schur_multiply_device(dx.data_ptr(), dy2.data_ptr())
    ev.schur_precondition_device(dx.data_ptr(), dp.data_ptr())
    ev.schur_back_substitute_device(dx.data_ptr(), dback.data_ptr())
    torch.cuda.synchronize(dev)
    assert close(drhs.cpu().numpy(), rhs)
    assert close(dy.cpu().numpy(), S @ x)
    assert torch.equal(dy, dy2)  # fixed-order sums: bit-identical
    back = dback.cpu().numpy()
    assert close(back[:e_cols], Minv @ (E.T @ (b - F @ x)))
    assert np.array_equal(back[e_cols:], x)
    if precond == _cse.SCHUR_IDENTITY:
        P = np.eye(f_cols)
    elif precond == _cse.SCHUR_JACOBI:
        P = block_inverse(F.T @ F + np.diag(D[e_cols:] ** 2), 9)
    else:
        P = block_inverse(S, 9)
    assert close(dp.cpu().numpy(), y0 + P @ x, 1e-11)
    ev.close()


def test_schur_pcg_solve_matches_dense_normal_equations(gpu):
    """IterativeSchurComplementSolver end to end: PCG on S with the JACOBI
    preconditioner (ConjugateGradientsSolver), then back substitution."""
    prog = runs_problem(seed=8)
    dev = torch.device("cuda", 0)
    ev = ca.Evaluator(prog, stream=torch.cuda.current_stream(dev).cuda_stream)
    ok, cost, r, g, jv = ev.evaluate()
    J = dense_jacobian(prog, jv)
    n = prog.num_effective_parameters
    e_cols, f_cols = ev.schur_structure()
    rng = np.random.default_rng(2)
    D = np.sqrt(1e-2 * np.maximum(np.sum(J * J, axis=0), 1e-6))
    b = -r
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    dj, dD, db = t(jv), t(D), t(b)
    rhs = torch.empty(f_cols, dtype=torch.float64, device=dev)
    ev.schur_init_device(dj.data_ptr(), dD.data_ptr(), db.data_ptr(), rhs.data_ptr(),
                         _cse.SCHUR_JACOBI)
    xf = torch.zeros(f_cols, dtype=torch.float64, device=dev)
    res = rhs.clone()
    z = torch.zeros_like(res)
    ev.schur_precondition_device(res.data_ptr(), z.data_ptr())
    p = z.clone()
    rz = torch.dot(res, z)
    Ap = torch.empty_like(p)
    for _ in range(2000):
        ev.schur_multiply_device(p.data_ptr(), Ap.data_ptr())
        alpha = rz / torch.dot(p, Ap)
        xf += alpha * p
        res -= alpha * Ap
        if float(res.norm()) <= 1e-12 * float(rhs.norm()):
            break
        z.zero_()
        ev.schur_precondition_device(res.data_ptr(), z.data_ptr())
        rz_new = torch.dot(res, z)
        p = z + (rz_new / rz) * p
        rz = rz_new
    dx = torch.empty(n, dtype=torch.float64, device=dev)
    ev.schur_back_substitute_device(xf.data_ptr(), dx.data_ptr())
    torch.cuda.synchronize(dev)
    ref = np.linalg.solve(J.T @ J + np.diag(D * D), J.T @ b)
    got = dx.cpu().numpy()
    assert np.linalg.norm(got - ref) <= 1e-8 * np.linalg.norm(ref)
    ev.close()


def test_schur_refuses_other_structures(gpu):
    prog = bal.synthetic_program((10, 300, 1500), format=ca.COMPRESSED_ROW, seed=9)
    ev = ca.Evaluator(prog)
    with pytest.raises(RuntimeError, match="cse_schur_structure"):
        ev.schur_structure()
    ev.close()
    # a user kind of another camera size (<2, 7, 3>): not the operators' shape
    import dataclasses
    import user_functors as U
    cams, pts, ci, pi, obs = bal.synthetic(10, 300, 1500, seed=9)
    p7 = bal.program(np.ascontiguousarray(cams[:, :7]), pts, ci, pi, obs,
                     kind=_cse.SNAVELY_NO_DISTORTION_2_7_3)
    p7.groups = [dataclasses.replace(g, kind=U.kind("SnavelyReprojectionErrorNoRadialDistortion/Trivial"))
                 for g in p7.groups]
    ev = ca.Evaluator(p7)
    assert ev.info().num_fused_gradient_groups == 1  # the fused gradient, not the operators
    with pytest.raises(RuntimeError, match="Snavely-shaped"):
        ev.schur_structure()
    ev.close()


def test_schur_init_reports_singular_blocks_without_D(gpu):
    """with d_D = NULL a point seen by one residual block has a
    singular E^T E (rank 2).  The init must not spread NaN silently: the
    block's inverse is zero and the next cse_wait reports the failure; with
    a positive D the same problem factors cleanly."""
    prog = runs_problem()  # has points with a single observation
    dev = torch.device("cuda", 0)
    ev = ca.Evaluator(prog, stream=torch.cuda.current_stream(dev).cuda_stream)
    ok, cost, r, g, jv = ev.evaluate()
    assert ok
    e_cols, f_cols = ev.schur_structure()
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    dj, db = t(jv), t(-r)
    rhs = torch.empty(f_cols, dtype=torch.float64, device=dev)
    ev.schur_init_device(dj.data_ptr(), None, db.data_ptr(), rhs.data_ptr(), _cse.SCHUR_JACOBI)
    assert ev.wait() == _cse.CSE_EVALUATION_FAILED
    assert torch.isfinite(rhs).all()
    dD = t(np.full(prog.num_effective_parameters, 0.5))
    ev.schur_init_device(dj.data_ptr(), dD.data_ptr(), db.data_ptr(), rhs.data_ptr(),
                         _cse.SCHUR_JACOBI)
    assert ev.wait() == _cse.CSE_OK
    ev.close()


@pytest.mark.parametrize("which,with_D,precond",
                         [(w, d, _cse.SCHUR_JACOBI) for w in ("bal", "runs", "quaternion", "large")
                          for d in (True, False)] +
                         [(w, True, p) for w in ("bal", "runs")
                          for p in (_cse.SCHUR_IDENTITY, _cse.SCHUR_SCHUR_JACOBI)])
def test_schur_init_gradient_equals_evaluation_gradient(gpu, which, with_D, precond):
    """cse_schur_init_gradient: the init also writes
    g = J^T r (r = -b) -- what TrustRegionMinimizer::EvaluateGradientAndJacobian
    (trust_region_minimizer.cc:242-255) gets from the evaluator beside J --
    so the evaluation before it can skip its gradient.  g equals the
    evaluation's gradient (gradient_mode 0) to 1e-13 relative, per entry
    scaled by the gradient's max; rhs equals plain cse_schur_init's."""
    if which == "runs":
        prog = runs_problem()
    elif which == "large":
        prog = bal.synthetic_program((64, 20000, 90000), loss=ca.Loss.cauchy(2.0), seed=11)
    else:
        prog = bal.synthetic_program((10, 300, 1500), loss=ca.Loss.huber(1.0), seed=9,
                                     quaternion_manifold=which == "quaternion")
    dev = torch.device("cuda", 0)
    ev = ca.Evaluator(prog, stream=torch.cuda.current_stream(dev).cuda_stream)
    ok, cost, r, g, jv = ev.evaluate()
    assert ok
    n = prog.num_effective_parameters
    e_cols, f_cols = ev.schur_structure()
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    dj, db = t(jv), t(-r)
    dD = t(np.random.default_rng(2).uniform(0.1, 2.0, n)) if with_D else None
    D_ptr = dD.data_ptr() if with_D else None
    rhs0 = torch.empty(f_cols, dtype=torch.float64, device=dev)
    rhs1 = torch.full((f_cols,), np.nan, dtype=torch.float64, device=dev)
    dg = torch.full((n,), np.nan, dtype=torch.float64, device=dev)
    ev.schur_init_device(dj.data_ptr(), D_ptr, db.data_ptr(), rhs0.data_ptr(), precond)
    rc0 = ev.wait()
    ev.schur_init_gradient_device(dj.data_ptr(), D_ptr, db.data_ptr(), rhs1.data_ptr(),
                                  dg.data_ptr(), precond)
    rc1 = ev.wait()
    # without D the runs problem has singular point blocks: both inits say so
    assert rc0 == rc1
    got = dg.cpu().numpy()
    assert np.isfinite(got).all()
    scale = np.abs(g).max()
    assert np.abs(got - g).max() <= 1e-13 * scale
    assert close(got, g, 1e-13)
    a, b_ = rhs1.cpu().numpy(), rhs0.cpu().numpy()
    assert np.abs(a - b_).max() <= 1e-13 * np.abs(b_).max()
    # the gradient written here drives the next init too: a second call is
    # bit-identical (fixed-order sums)
    dg2 = torch.empty_like(dg)
    ev.schur_init_gradient_device(dj.data_ptr(), D_ptr, db.data_ptr(), rhs1.data_ptr(),
                                  dg2.data_ptr(), precond)
    ev.wait()
    assert torch.equal(dg, dg2)
    # the preconditioner built beside the gradient is the plain init's
    x = torch.from_numpy(np.random.default_rng(4).normal(size=f_cols)).to(dev)
    y0 = torch.zeros(f_cols, dtype=torch.float64, device=dev)
    y1 = torch.zeros(f_cols, dtype=torch.float64, device=dev)
    ev.schur_precondition_device(x.data_ptr(), y1.data_ptr())
    ev.schur_init_device(dj.data_ptr(), D_ptr, db.data_ptr(), rhs0.data_ptr(), precond)
    ev.schur_precondition_device(x.data_ptr(), y0.data_ptr())
    ev.wait()
    assert torch.equal(y0, y1)
    ev.close()


def test_schur_init_gradient_after_gradient_free_evaluation(gpu):
    """The intended sequence: cse_evaluate_device without a gradient pointer
    (no CameraGradientKernel), then cse_schur_init_gradient with b = -r; the
    gradient equals a full evaluation's."""
    prog = bal.synthetic_program((32, 4000, 20000), loss=ca.Loss.huber(1.0), seed=5)
    dev = torch.device("cuda", 0)
    ev = ca.Evaluator(prog, stream=torch.cuda.current_stream(dev).cuda_stream)
    ok, cost, r, g, jv = ev.evaluate()
    assert ok
    n, m = prog.num_effective_parameters, prog.num_residuals
    e_cols, f_cols = ev.schur_structure()
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    dx = t(prog.state)
    dcost = torch.empty(1, dtype=torch.float64, device=dev)
    dr = torch.empty(m, dtype=torch.float64, device=dev)
    dj = torch.empty(prog.num_jacobian_values, dtype=torch.float64, device=dev)
    ev.evaluate_device(dx.data_ptr(), dcost.data_ptr(), dr.data_ptr(), None, dj.data_ptr())
    assert ev.wait() == _cse.CSE_OK
    db = -dr
    dD = t(np.full(n, 0.25))
    rhs = torch.empty(f_cols, dtype=torch.float64, device=dev)
    dg = torch.empty(n, dtype=torch.float64, device=dev)
    ev.schur_init_gradient_device(dj.data_ptr(), dD.data_ptr(), db.data_ptr(), rhs.data_ptr(),
                                  dg.data_ptr(), _cse.SCHUR_JACOBI)
    assert ev.wait() == _cse.CSE_OK
    got = dg.cpu().numpy()
    assert np.abs(got - g).max() <= 1e-13 * np.abs(g).max()
    ev.close()
