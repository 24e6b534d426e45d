"""GPU: the Jacobian as a device linear operator.

cse_jacobian_right_multiply / cse_jacobian_left_multiply act on the values
the evaluator wrote, in HBM (the reference copies them to the host and back,
CudaSparseMatrix::CopyValuesFromCpu, cuda_sparse_matrix.h:77-96).  Checked
against a dense reconstruction of J from the layout tables
(BlockJacobianWriter / CompressedRowJacobianWriter addressing), on both
layouts, the affine and the table paths, constant blocks and manifolds; and
used end to end as the operator of a CGNR solve of the damped normal
equations (cgnr_solver.cc), compared with a dense solve.
"""
import numpy as np
import pytest

import ceres_amd as ca
from ceres_amd import bal

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def dense_jacobian(prog, values):
    """J[residual row, delta column] from the program's layout tables."""
    J = np.zeros((prog.num_residuals, prog.num_effective_parameters))
    begin, ids = prog.block_params_csr()
    nres = prog.residuals_per_block()
    for b in range(prog.num_residual_blocks):
        q = int(prog.jacobian_per_residual_layout[b])
        r0 = int(prog.residual_layout[b])
        for pid in ids[begin[b]:begin[b + 1]]:
            if prog.pb_constant[pid]:
                continue
            d0, t = int(prog.delta_offset[pid]), int(prog.pb_tangent[pid])
            for k in range(int(nres[b])):
                off = int(prog.jacobian_per_residual_offsets[q])
                q += 1
                J[r0 + k, d0:d0 + t] = values[off:off + t]
    return J


def device_check(prog, force_general=False, seed=0):
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    ev = ca.Evaluator(prog, force_general_layout=force_general, stream=stream)
    ok, cost, r, g, jvals = ev.evaluate()
    assert ok
    J = dense_jacobian(prog, jvals)
    rng = np.random.default_rng(seed)
    x = rng.normal(size=prog.num_effective_parameters)
    y0 = rng.normal(size=prog.num_residuals)
    f64 = torch.float64
    dj = torch.from_numpy(jvals).to(dev)
    dx = torch.from_numpy(x).to(dev)
    dy = torch.from_numpy(y0.copy()).to(dev)
    ev.right_multiply_device(dj.data_ptr(), dx.data_ptr(), dy.data_ptr())
    dz = torch.from_numpy(x.copy()).to(dev)
    dyl = torch.from_numpy(y0).to(dev)
    ev.left_multiply_device(dj.data_ptr(), dyl.data_ptr(), dz.data_ptr())
    torch.cuda.synchronize(dev)
    y = dy.cpu().numpy()
    z = dz.cpu().numpy()
    ev.close()
    ref_y = y0 + J @ x
    ref_z = x + J.T @ y0
    assert np.linalg.norm(y - ref_y) <= 1e-13 * np.linalg.norm(ref_y)
    assert np.linalg.norm(z - ref_z) <= 1e-13 * np.linalg.norm(ref_z)
    # J^T r with r the evaluator's residuals is the gradient it returned.
    return J, r, g, jvals


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
@pytest.mark.parametrize("general", [False, True])
def test_jacobian_multiply_matches_dense(gpu, fmt, general):
    prog = bal.synthetic_program((12, 400, 1600), loss=ca.Loss.huber(1.0), format=fmt, seed=5)
    J, r, g, _ = device_check(prog, force_general=general)
    assert np.linalg.norm(J.T @ r - g) <= 1e-13 * np.linalg.norm(g)


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
def test_jacobian_multiply_mini_ba(gpu, fmt):
    # Constant blocks and a ProductManifold camera: the table path, local
    # (tangent-space) Jacobian columns.
    from test_parity_gpu import mini_ba
    device_check(mini_ba(fmt))


@pytest.mark.parametrize("op", ["cgnr_multiply", "two_products"])
def test_cgnr_on_device_matches_dense_solve(gpu, op):
    # One Levenberg-Marquardt step's linear system, (J^T J + lam D) dx = -g
    # with D = diag(J^T J) (levenberg_marquardt_strategy.cc), solved by
    # Jacobi-preconditioned conjugate gradients on the normal equations
    # (cgnr_solver.cc): every J / J^T product through the device operator,
    # the values never leave HBM.  Compared with a dense solve.
    prog = bal.synthetic_program((6, 120, 500), loss=ca.Loss.huber(1.0), seed=9)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    ev = ca.Evaluator(prog, stream=stream)
    f64 = torch.float64
    n, m = prog.num_effective_parameters, prog.num_residuals
    state = torch.from_numpy(prog.state).to(dev)
    cost = torch.zeros(1, dtype=f64, device=dev)
    r = torch.empty(m, dtype=f64, device=dev)
    jac = torch.empty(prog.num_jacobian_values, dtype=f64, device=dev)
    g = torch.empty(n, dtype=f64, device=dev)
    ev.evaluate_device(state.data_ptr(), cost.data_ptr(), r.data_ptr(), g.data_ptr(),
                       jac.data_ptr())
    assert ev.wait() == 0
    J = dense_jacobian(prog, jac.cpu().numpy())
    lam = 1e-2
    Dh = np.einsum("ij,ij->j", J, J)
    D = torch.from_numpy(Dh).to(dev)

    sqrt_lam_d = torch.sqrt(lam * D)

    def normal_op(v):
        if op == "cgnr_multiply":  # one call: J^T J v + (sqrt(lam D))^2 v
            out = torch.zeros(n, dtype=f64, device=dev)
            ev.cgnr_multiply_device(jac.data_ptr(), sqrt_lam_d.data_ptr(), v.data_ptr(),
                                    out.data_ptr())
            return out
        Jv = torch.zeros(m, dtype=f64, device=dev)
        ev.right_multiply_device(jac.data_ptr(), v.data_ptr(), Jv.data_ptr())
        out = lam * D * v
        ev.left_multiply_device(jac.data_ptr(), Jv.data_ptr(), out.data_ptr())
        return out

    b = -g
    Minv = 1.0 / ((1.0 + lam) * D)
    x = torch.zeros(n, dtype=f64, device=dev)
    res = b.clone()
    z = Minv * res
    p = z.clone()
    rz = torch.dot(res, z)
    for _ in range(1000):
        Ap = normal_op(p)
        alpha = rz / torch.dot(p, Ap)
        x += alpha * p
        res -= alpha * Ap
        if res.norm() <= 1e-12 * b.norm():
            break
        z = Minv * res
        rz_new = torch.dot(res, z)
        p = z + (rz_new / rz) * p
        rz = rz_new
    ref = np.linalg.solve(J.T @ J + lam * np.diag(Dh), -(J.T @ r.cpu().numpy()))
    got = x.cpu().numpy()
    ev.close()
    assert np.linalg.norm(got - ref) <= 1e-8 * np.linalg.norm(ref)


def test_bundle_adjuster_driver_reduces_cost(gpu):
    # The f4 driver: Normalize + Perturb + Schur order + LM iterations whose
    # evaluations, Plus and CGNR products all run on the device.
    from ceres_amd import bundle_adjuster
    c0, c1, rows = bundle_adjuster.main(["--synthetic", "problem-16-22106", "--robustify",
                                         "--point_sigma", "0.05", "--num_iterations", "4"])
    # Normalize() scales the scene to a median absolute deviation of 100, so
    # point_sigma 0.05 is a small perturbation; the synthetic observations
    # carry 1 px noise and 5 % outliers, so the cost stays well above zero.
    assert c1 < 0.9 * c0
    costs = [r[1] for r in rows] + [c1]
    assert all(b <= a for a, b in zip(costs, costs[1:]))
    assert all(r[-1] for r in rows)


def test_bundle_adjuster_gradient_from_the_schur_init(gpu):
    """The iterative_schur driver evaluates without the gradient and takes
    g = Jᵀr from cse_schur_init_gradient; the cgnr driver takes it from the
    evaluation.  At the same (deterministically perturbed) start both report
    the same |g| and cost, and the Schur run's first step is accepted (its
    model decrease -(g·dx + |J dx|²/2) uses that g)."""
    from ceres_amd import bundle_adjuster
    base = ["--synthetic", "problem-16-22106", "--robustify", "--point_sigma", "0.05",
            "--num_iterations", "1"]
    _, _, rows_s = bundle_adjuster.main(base + ["--linear_solver", "iterative_schur"])
    _, _, rows_c = bundle_adjuster.main(base + ["--linear_solver", "cgnr"])
    (_, c0s, _, gs, _, _, _, acc_s), (_, c0c, _, gc, _, _, _, _) = rows_s[0], rows_c[0]
    assert c0s == c0c
    assert abs(gs - gc) <= 1e-12 * gc and gs > 0
    assert acc_s


def cgnr_op_check(prog, seed, with_d=True):
    """cse_cgnr_multiply against J^T J x + D^2 x from the dense J; fused and
    two-product paths; deterministic."""
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    ev = ca.Evaluator(prog, stream=stream)
    ok, cost, r, g, jvals = ev.evaluate()
    assert ok
    fused = ev.info().num_fused_gradient_groups
    J = dense_jacobian(prog, jvals)
    rng = np.random.default_rng(seed)
    x = rng.normal(size=prog.num_effective_parameters)
    y0 = rng.normal(size=prog.num_effective_parameters)
    D = rng.uniform(0.5, 2.0, size=prog.num_effective_parameters) if with_d else None
    dj = torch.from_numpy(jvals).to(dev)
    dx = torch.from_numpy(x).to(dev)
    dD = torch.from_numpy(D).to(dev) if with_d else None
    outs = []
    for _ in range(2):
        dy = torch.from_numpy(y0.copy()).to(dev)
        ev.cgnr_multiply_device(dj.data_ptr(), dD.data_ptr() if with_d else None, dx.data_ptr(),
                                dy.data_ptr())
        torch.cuda.synchronize(dev)
        outs.append(dy.cpu().numpy())
    # The two-product path of the same operator (right then left multiply).
    dz = torch.zeros(prog.num_residuals, dtype=torch.float64, device=dev)
    ev.right_multiply_device(dj.data_ptr(), dx.data_ptr(), dz.data_ptr())
    dy2 = torch.from_numpy(y0.copy()).to(dev)
    ev.left_multiply_device(dj.data_ptr(), dz.data_ptr(), dy2.data_ptr())
    torch.cuda.synchronize(dev)
    two = dy2.cpu().numpy() + (D * D * x if with_d else 0.0)
    ev.close()
    ref = y0 + J.T @ (J @ x) + (D * D * x if with_d else 0.0)
    assert np.array_equal(outs[0], outs[1])
    assert np.linalg.norm(outs[0] - ref) <= 1e-13 * np.linalg.norm(ref)
    assert np.linalg.norm(two - ref) <= 1e-13 * np.linalg.norm(ref)
    return fused


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
@pytest.mark.parametrize("shape", [(12, 400, 1600), (24, 3000, 20000), (210, 20, 4097),
                                   (5, 21, 65)])
def test_cgnr_operator_matches_dense(gpu, fmt, shape):
    prog = bal.synthetic_program(shape, loss=ca.Loss.huber(1.0), format=fmt, seed=shape[2])
    fused = cgnr_op_check(prog, seed=1, with_d=shape[2] % 2 == 0)
    cams = prog.groups[0].ids[:, 0]
    assert fused == (0 if np.all(np.diff(cams) >= 0) else 1)


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
def test_cgnr_operator_user_kind(gpu, fmt):
    # A user functor kind of the Snavely shape (BundlerResidual, its own TU)
    # takes the one-pass operator: it reads only the Jacobian.
    import dataclasses
    import user_functors as U
    prog = bal.synthetic_program((24, 3000, 20000), loss=ca.Loss.huber(1.0), format=fmt, seed=4)
    prog.groups = [dataclasses.replace(g, kind=U.kind("BundlerResidual/Huber")) for g in prog.groups]
    assert cgnr_op_check(prog, seed=3) == 1


def test_cgnr_operator_two_product_path(gpu):
    # The mini bundle-adjustment problem (manifolds, constant blocks, three
    # functor types): not eligible for the fused pass.
    from test_parity_gpu import mini_ba
    assert cgnr_op_check(mini_ba(ca.BLOCK_SPARSE), seed=2) == 0


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
def test_left_multiply_by_residuals_is_the_gradient(gpu, fmt):
    """A device CGNR step forms its right-hand side Jᵀ(−r) with
    cse_jacobian_left_multiply; with it the evaluation before needs no
    gradient either (as cse_schur_init_gradient for ITERATIVE_SCHUR):
    Jᵀr from the operator equals gradient_mode 0's gradient to 1e-13."""
    prog = bal.synthetic_program((24, 3000, 20000), loss=ca.Loss.huber(1.0), format=fmt, seed=12)
    dev = torch.device("cuda", 0)
    ev = ca.Evaluator(prog, stream=torch.cuda.current_stream(dev).cuda_stream)
    ok, cost, r, g, jv = ev.evaluate()
    assert ok
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    dj, dr = t(jv), t(r)
    dg = torch.zeros(prog.num_effective_parameters, dtype=torch.float64, device=dev)
    ev.left_multiply_device(dj.data_ptr(), dr.data_ptr(), dg.data_ptr())
    torch.cuda.synchronize(dev)
    got = dg.cpu().numpy()
    assert np.abs(got - g).max() <= 1e-13 * np.abs(g).max()
    ev.close()
