"""bundle_adjuster-style driver over the MI355X evaluator.

Mirrors the flow of examples/bundle_adjuster.cu.cc around the hot path:
read a BAL file (or build a synthetic one), Normalize(), Perturb(), put the
residual blocks in Schur order, and run Levenberg-Marquardt iterations
whose every evaluation is the HIP evaluator and whose linear solve is a
preconditioned CG on the device's implicit Schur complement
(--linear_solver iterative_schur, the reference benchmark's solver, with its
jacobi / schur_jacobi / identity preconditioners) or on the normal equations
(--linear_solver cgnr); no Jacobian value leaves HBM.  Prints a FullReport-style table of the evaluator timers
(solver.cc: "Residual only evaluation", "Jacobian & residual evaluation",
"Linear solver", "Plus").

The minimizer here is deliberately small (a driver that exercises the
path, not a port of Ceres' TrustRegionMinimizer, which stays Ceres'):
LM damping D = diag(J^T J) with Ceres' default radius policy
(levenberg_marquardt_strategy.cc: radius / (1 / 3 ... 2) updates), a
candidate accepted when the cost decreases.

    python -m ceres_amd.bundle_adjuster --synthetic problem-16-22106 \\
        --robustify --point_sigma 0.01 --num_iterations 5
"""
import argparse
import os
import sys
import time

import numpy as np

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import ceres_amd as ca  # noqa: E402
from ceres_amd import bal  # noqa: E402


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    src = ap.add_mutually_exclusive_group(required=True)
    src.add_argument("--input", help="BAL problem file (text)")
    src.add_argument("--synthetic", choices=list(bal.CONFIGS), help="synthetic BAL shape")
    ap.add_argument("--robustify", action="store_true", help="HuberLoss(1.0)")
    ap.add_argument("--use_quaternions", action="store_true",
                    help="10-parameter cameras {q, t, f, k1, k2} (bal_problem.cc:110-121)")
    ap.add_argument("--use_manifolds", action="store_true",
                    help="with --use_quaternions: every camera on ProductManifold<QuaternionManifold, "
                         "EuclideanManifold<6>> (bundle_adjuster.cc:337-345)")
    ap.add_argument("--format", default="block_sparse", choices=["block_sparse", "compressed_row"])
    ap.add_argument("--rotation_sigma", type=float, default=0.0)
    ap.add_argument("--translation_sigma", type=float, default=0.0)
    ap.add_argument("--point_sigma", type=float, default=0.0)
    ap.add_argument("--num_iterations", type=int, default=5)
    ap.add_argument("--max_linear_solver_iterations", type=int, default=500)
    ap.add_argument("--eta", type=float, default=1e-2, help="CG forcing tolerance")
    ap.add_argument("--initial_trust_region_radius", type=float, default=1e4)
    ap.add_argument("--linear_solver", default="iterative_schur", choices=["iterative_schur", "cgnr"],
                    help="iterative_schur (the reference benchmark's, README.md:143-184): PCG on "
                         "the implicit Schur complement (cse_schur_*); cgnr: PCG on the normal "
                         "equations (cse_cgnr_multiply)")
    ap.add_argument("--preconditioner", default="jacobi",
                    choices=["identity", "jacobi", "schur_jacobi"],
                    help="iterative_schur's preconditioner (bundle_adjuster.cc default: jacobi)")
    return ap.parse_args(argv)


class Timers:
    def __init__(self):
        self.t = {}

    def add(self, name, seconds):
        tot, n = self.t.get(name, (0.0, 0))
        self.t[name] = (tot + seconds, n + 1)

    def report(self):
        lines = ["Time (in seconds):"]
        for name, (tot, n) in self.t.items():
            lines.append(f"  {name:<34s}{tot:12.6f} ({n})")
        return "\n".join(lines)


def solve(args):
    import torch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    f64 = torch.float64
    timers = Timers()
    t0 = time.perf_counter()
    if args.input:
        cams, pts, ci, pi, obs = bal.read(args.input)
    else:
        C, P, O = bal.CONFIGS[args.synthetic]
        cams, pts, ci, pi, obs = bal.synthetic(C, P, O)
        cams, pts = cams.copy(), pts.copy()
    bal.normalize(cams, pts)
    bal.perturb(cams, pts, args.rotation_sigma, args.translation_sigma, args.point_sigma)
    order = bal.schur_residual_order(pi, pts.shape[0])
    loss = ca.Loss.huber(1.0) if args.robustify else None
    if args.use_quaternions:
        cams = bal.to_quaternion_cameras(cams)
    manifold = args.use_quaternions and args.use_manifolds
    if args.use_quaternions and not manifold and args.linear_solver == "iterative_schur":
        raise SystemExit("iterative_schur takes 9-column cameras: add --use_manifolds or use cgnr")
    prog = bal.program(cams, pts, ci[order], pi[order], obs[order], loss=loss, format=args.format,
                       quaternion_manifold=manifold)
    timers.add("Preprocessor", time.perf_counter() - t0)

    stream = torch.cuda.current_stream(dev).cuda_stream
    ev = ca.Evaluator(prog, device=0, stream=stream)
    n, m = prog.num_effective_parameters, prog.num_residuals
    x = torch.from_numpy(prog.state).to(dev)
    cand = torch.empty_like(x)
    cost = torch.zeros(1, dtype=f64, device=dev)
    ccost = torch.zeros(1, dtype=f64, device=dev)
    r = torch.empty(m, dtype=f64, device=dev)
    g = torch.empty(n, dtype=f64, device=dev)
    jac = torch.empty(prog.num_jacobian_values, dtype=f64, device=dev)

    def timed(name, fn):
        torch.cuda.synchronize(dev)
        s = time.perf_counter()
        out = fn()
        torch.cuda.synchronize(dev)
        timers.add(name, time.perf_counter() - s)
        return out

    # ITERATIVE_SCHUR takes g = J^T r from its own init (cse_schur_init_gradient,
    # every solve, before g is read); CGNR from the evaluation.
    grad_from_init = args.linear_solver == "iterative_schur"

    def jacobian_eval(new_point=True):
        # After an accepted step x holds the candidate just evaluated:
        # new_evaluation_point = false, as HandleSuccessfulStep passes
        # (trust_region_minimizer.cc:822-826).
        ev.evaluate_device(x.data_ptr(), cost.data_ptr(), r.data_ptr(),
                           None if grad_from_init else g.data_ptr(), jac.data_ptr(),
                           new_evaluation_point=new_point)
        return ev.wait()

    def normal_op(v, sqrt_lam_d):
        # (J^T J + lam D) v in one pass over J (cse_cgnr_multiply, the
        # CudaCgnrLinearOperator of cgnr_solver.cc:226-237).
        out = torch.zeros(n, dtype=f64, device=dev)
        ev.cgnr_multiply_device(jac.data_ptr(), sqrt_lam_d.data_ptr(), v.data_ptr(),
                                out.data_ptr())
        return out

    def cgnr(lam):
        # (J^T J + lam D) dx = -g by Jacobi-preconditioned CG on the normal
        # equations (cgnr_solver.cc), D = diag(J^T J).
        b = -g
        Minv = 1.0 / ((1.0 + lam) * D)
        sqrt_lam_d = torch.sqrt(lam * D)
        dx = torch.zeros(n, dtype=f64, device=dev)
        res = b.clone()
        z = Minv * res
        p = z.clone()
        rz = torch.dot(res, z)
        bn = b.norm()
        it = 0
        for it in range(1, args.max_linear_solver_iterations + 1):
            Ap = normal_op(p, sqrt_lam_d)
            alpha = rz / torch.dot(p, Ap)
            dx += alpha * p
            res -= alpha * Ap
            if res.norm() <= args.eta * bn:
                break
            z = Minv * res
            rz_new = torch.dot(res, z)
            p = z + (rz_new / rz) * p
            rz = rz_new
        return dx, it

    if args.linear_solver == "iterative_schur":
        e_cols, f_cols = ev.schur_structure()
        pre = {"identity": ca._cse.SCHUR_IDENTITY, "jacobi": ca._cse.SCHUR_JACOBI,
               "schur_jacobi": ca._cse.SCHUR_SCHUR_JACOBI}[args.preconditioner]
        rhs = torch.empty(f_cols, dtype=f64, device=dev)
        neg_r = torch.empty(m, dtype=f64, device=dev)

    def schur_solve(lam):
        # IterativeSchurComplementSolver (iterative_schur_complement_solver.cc:
        # 63-170): the augmented system [J; sqrt(lam diag(J^T J))] dx = [-r; 0]
        # reduced to S dx_f = rhs, PCG on S, then back substitution.
        torch.neg(r, out=neg_r)
        sqrt_lam_d = torch.sqrt(lam * D)
        ev.schur_init_gradient_device(jac.data_ptr(), sqrt_lam_d.data_ptr(), neg_r.data_ptr(),
                                      rhs.data_ptr(), g.data_ptr(), pre)
        xf = torch.zeros(f_cols, dtype=f64, device=dev)
        res = rhs.clone()
        z = torch.zeros_like(res)
        ev.schur_precondition_device(res.data_ptr(), z.data_ptr())
        p = z.clone()
        Ap = torch.empty_like(p)
        rz = torch.dot(res, z)
        bn = rhs.norm()
        it = 0
        for it in range(1, args.max_linear_solver_iterations + 1):
            ev.schur_multiply_device(p.data_ptr(), Ap.data_ptr())
            alpha = rz / torch.dot(p, Ap)
            xf += alpha * p
            res -= alpha * Ap
            if res.norm() <= args.eta * bn:
                break
            z.zero_()
            ev.schur_precondition_device(res.data_ptr(), z.data_ptr())
            rz_new = torch.dot(res, z)
            p = z + (rz_new / rz) * p
            rz = rz_new
        dx = torch.empty(n, dtype=f64, device=dev)
        ev.schur_back_substitute_device(xf.data_ptr(), dx.data_ptr())
        return dx, it

    status = timed("Jacobian & residual evaluation", jacobian_eval)
    if status != 0:
        raise SystemExit("initial evaluation failed")
    initial_cost = float(cost.item())
    radius = args.initial_trust_region_radius
    # LevenbergMarquardtStrategy (levenberg_marquardt_strategy.cc:157-170):
    # a rejected step divides the radius by decrease_factor and doubles it;
    # an accepted one resets it to 2.
    decrease_factor = 2.0
    max_radius = 1e16  # Solver::Options::max_trust_region_radius
    min_relative_decrease = 1e-3  # Solver::Options::min_relative_decrease
    rows = []
    D = torch.zeros(n, dtype=f64, device=dev)
    ones = torch.ones(m, dtype=f64, device=dev)
    jac2 = None  # squared Jacobian values, one buffer for the whole solve
    d_stale = True  # D follows J: recomputed after the initial and each accepted evaluation
    for it in range(args.num_iterations):
        # Jacobi scaling: diag(J^T J) = column sums of squared values, one
        # left-multiply of the squared Jacobian with a vector of ones.
        if d_stale:
            if jac2 is None:
                jac2 = torch.empty_like(jac)
            torch.mul(jac, jac, out=jac2)
            D.zero_()
            ev.left_multiply_device(jac2.data_ptr(), ones.data_ptr(), D.data_ptr())
            D.clamp_(min=1e-6)
            d_stale = False
        solver = schur_solve if args.linear_solver == "iterative_schur" else cgnr
        dx, cg_iters = timed("Linear solver", lambda: solver(1.0 / radius))
        timed("Plus", lambda: ev.plus_device(x.data_ptr(), dx.data_ptr(), cand.data_ptr()))

        def cand_eval():
            ev.evaluate_device(cand.data_ptr(), ccost.data_ptr(), None, None, None)
            return ev.wait()

        ok = timed("Residual only evaluation", cand_eval) == 0
        new_cost = float(ccost.item()) if ok else float("inf")
        old_cost = float(cost.item())
        # model decrease of the linearised problem: -(g.dx + 0.5 |J dx|^2)
        Jdx = torch.zeros(m, dtype=f64, device=dev)
        ev.right_multiply_device(jac.data_ptr(), dx.data_ptr(), Jdx.data_ptr())
        model = float(-(torch.dot(g, dx) + 0.5 * torch.dot(Jdx, Jdx)).item())
        rho = (old_cost - new_cost) / model if model > 0 else -1.0
        # TrustRegionMinimizer::IsStepSuccessful: relative decrease above
        # min_relative_decrease (trust_region_minimizer.cc).
        accepted = ok and rho > min_relative_decrease
        rows.append((it, old_cost, new_cost, float(g.norm().item()), float(dx.norm().item()),
                     radius, cg_iters, accepted))
        if accepted:
            x.copy_(cand)
            if timed("Jacobian & residual evaluation", lambda: jacobian_eval(False)) != 0:
                raise SystemExit(f"iteration {it}: Jacobian evaluation at the accepted point failed")
            d_stale = True
            radius = min(max_radius, radius / max(1.0 / 3.0, 1.0 - (2.0 * rho - 1.0) ** 3))
            decrease_factor = 2.0
        else:
            radius = radius / decrease_factor
            decrease_factor *= 2.0
    del jac2
    ev.close()
    print("iter      cost      cost_new   |gradient|    |step|    tr_radius  ls_iter  accepted")
    for it, c0, c1, gn, sn, rad, li, acc in rows:
        print(f"{it:4d} {c0:12.6e} {c1:12.6e} {gn:10.3e} {sn:10.3e} {rad:10.3e} {li:6d}   {acc}")
    print(f"\nInitial cost {initial_cost:.6e}  Final cost {float(cost.item()):.6e}")
    print(timers.report())
    return initial_cost, float(cost.item()), rows


def main(argv=None):
    return solve(parse(argv))


if __name__ == "__main__":
    main()
