#!/usr/bin/env python3
"""Golden vectors for the Snavely reprojection residual block, derived
independently of both the oracle and the HIP evaluator.

TEST INFRASTRUCTURE ONLY.  The model is written symbolically in sympy from
its definition (examples/snavely_reprojection_error.h:58-93,
include/ceres/rotation.h:830-899, the quaternion variant
rotation.h:753-798), differentiated symbolically, and evaluated with mpmath
at 50 significant digits.  The robust-loss correction follows the published
formulas (loss_function_cuda.h:62-113, corrector.h:82-213) evaluated in
mpmath as well.  Results are rounded to fp64 and written to
tests/golden/snavely_golden.json together with the inputs.

Run:  python oracle/gen_golden.py   (takes ~1 minute; deterministic)
"""
import json
import os
import sys

import mpmath
import numpy as np
import sympy as sp

mpmath.mp.dps = 50
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "tests", "golden", "snavely_golden.json")


def snavely_expr(kind):
    """Residual (2 expressions) and variables for a functor kind.

    kind 'aa'   : SnavelyReprojectionError<2,9,3>, Rodrigues branch
    kind 'aa0'  : same functor, theta == 0 Taylor branch (R = I + hat(aa))
    kind 'nod'  : SnavelyReprojectionErrorNoRadialDistortion<2,7,3>
    kind 'quat' : SnavelyReprojectionErrorWithQuaternions<2,10,3>
    """
    ox, oy = sp.symbols("ox oy")
    X = sp.Matrix(sp.symbols("X0:3"))
    if kind in ("aa", "aa0", "nod"):
        ncam = 9 if kind != "nod" else 7
        c = sp.symbols(f"c0:{ncam}")
        aa = sp.Matrix(c[0:3])
        if kind == "aa0":
            p = X + aa.cross(X)
        else:
            theta = sp.sqrt(aa.dot(aa))
            w = aa / theta
            p = (X * sp.cos(theta) + w.cross(X) * sp.sin(theta)
                 + w * w.dot(X) * (1 - sp.cos(theta)))
        p = p + sp.Matrix(c[3:6])
        xp, yp = -p[0] / p[2], -p[1] / p[2]
        f = c[6]
        if kind == "nod":
            px, py = f * xp, f * yp
        else:
            l1, l2 = c[7], c[8]
            r2 = xp * xp + yp * yp
            d = 1 + r2 * (l1 + l2 * r2)
            px, py = f * d * xp, f * d * yp
    else:
        c = sp.symbols("c0:10")
        q = sp.Matrix(c[0:4])
        qn = q / sp.sqrt(q.dot(q))
        w0, v = qn[0], sp.Matrix(qn[1:4])
        # Unit quaternion rotation: p = X + 2 w (v x X) + 2 v x (v x X)
        uv = v.cross(X) * 2
        p = X + w0 * uv + v.cross(uv)
        p = p + sp.Matrix(c[4:7])
        xp, yp = -p[0] / p[2], -p[1] / p[2]
        l1, l2, f = c[8], c[9], c[7]
        r2 = xp * xp + yp * yp
        d = 1 + r2 * (l1 + l2 * r2)
        px, py = f * d * xp, f * d * yp
    r = sp.Matrix([px - ox, py - oy])
    vars_ = list(c) + list(X)
    J = r.jacobian(vars_)
    return r, J, vars_, (ox, oy)


def loss_rho(kind, a, s):
    a = mpmath.mpf(a)
    if kind == 0:
        return [s, mpmath.mpf(1), mpmath.mpf(0)]
    if kind == 1:
        b = a * a
        if s > b:
            r = mpmath.sqrt(s)
            r1 = max(mpmath.mpf(sys.float_info.min), a / r)
            return [2 * a * r - b, r1, -r1 / (2 * s)]
        return [s, mpmath.mpf(1), mpmath.mpf(0)]
    b = a * a
    c = 1 / b
    sm = 1 + s * c
    inv = 1 / sm
    return [b * mpmath.log(sm), max(mpmath.mpf(sys.float_info.min), inv), -c * inv * inv]


def correct(rvec, Jmat, rho, sq):
    """Corrector (corrector.h:82-213) in mpmath."""
    sqrt_rho1 = mpmath.sqrt(rho[1])
    if sq == 0 or rho[2] <= 0:
        return [x * sqrt_rho1 for x in rvec], [[x * sqrt_rho1 for x in row] for row in Jmat]
    D = 1 + 2 * sq * rho[2] / rho[1]
    alpha = 1 - mpmath.sqrt(D)
    rs = sqrt_rho1 / (1 - alpha)
    asq = alpha / sq
    nrow, ncol = len(Jmat), len(Jmat[0])
    Jc = [[None] * ncol for _ in range(nrow)]
    for col in range(ncol):
        rtj = sum(Jmat[k][col] * rvec[k] for k in range(nrow))
        for k in range(nrow):
            Jc[k][col] = sqrt_rho1 * (Jmat[k][col] - asq * rvec[k] * rtj)
    return [x * rs for x in rvec], Jc


def make_cases(rng):
    cases = []
    # SURVEY.md §8(d) distributions plus edge rotations.
    def camera(aa):
        t = [rng.normal(), rng.normal(), -10 + rng.normal()]
        f = rng.uniform(400, 1200)
        return list(aa) + t + [f, rng.normal(0, 0.05), rng.normal(0, 0.01)]

    for i in range(48):
        if i < 4:
            aa = [0.0, 0.0, 0.0]
        elif i < 8:
            ax = rng.normal(size=3)
            aa = list(ax / np.linalg.norm(ax) * rng.uniform(2.0, 3.1))
        else:
            aa = list(rng.normal(0, 0.05, size=3))
        cam = camera(aa)
        pt = list(rng.uniform(-3, 3, size=3))
        cases.append(("snavely", cam, pt))
    for i in range(8):
        aa = [0.0, 0.0, 0.0] if i == 0 else list(rng.normal(0, 0.05, size=3))
        cam = camera(aa)[:7]
        pt = list(rng.uniform(-3, 3, size=3))
        cases.append(("nod", cam, pt))
    for i in range(8):
        q = rng.normal(size=4)
        q[0] = abs(q[0]) + 2.0
        q = q * rng.uniform(0.5, 2.0)   # not unit: QuaternionRotatePoint normalises
        cam = list(q) + [rng.normal(), rng.normal(), -10 + rng.normal(),
                         rng.uniform(400, 1200), rng.normal(0, 0.05), rng.normal(0, 0.01)]
        pt = list(rng.uniform(-3, 3, size=3))
        cases.append(("quat", cam, pt))
    return cases


def main():
    rng = np.random.default_rng(0xCE2E5)
    models = {k: snavely_expr(k) for k in ("aa", "aa0", "nod", "quat")}
    funcs = {}
    for k, (r, J, vars_, obs) in models.items():
        funcs[k] = (sp.lambdify(vars_ + list(obs), r, modules="mpmath"),
                    sp.lambdify(vars_ + list(obs), J, modules="mpmath"))
    out = []
    for idx, (kind, cam, pt) in enumerate(make_cases(rng)):
        if kind == "snavely":
            model = "aa0" if cam[0] == cam[1] == cam[2] == 0.0 else "aa"
            functor = 0
        elif kind == "nod":
            model = "aa0" if cam[0] == cam[1] == cam[2] == 0.0 else "aa"
            model = "nod" if model == "aa" else "nod0"
            functor = 1
        else:
            model, functor = "quat", 2
        if model == "nod0":
            # theta == 0 branch of the no-distortion functor.
            ox, oy = sp.symbols("ox oy")
            c = sp.symbols("c0:7")
            X = sp.Matrix(sp.symbols("X0:3"))
            p = X + sp.Matrix(c[0:3]).cross(X) + sp.Matrix(c[3:6])
            r = sp.Matrix([c[6] * (-p[0] / p[2]) - ox, c[6] * (-p[1] / p[2]) - oy])
            vars_ = list(c) + list(X)
            fr = sp.lambdify(vars_ + [ox, oy], r, modules="mpmath")
            fJ = sp.lambdify(vars_ + [ox, oy], r.jacobian(vars_), modules="mpmath")
        else:
            fr, fJ = funcs[model]
        args0 = [mpmath.mpf(x) for x in cam + pt]
        clean = fr(*(args0 + [mpmath.mpf(0), mpmath.mpf(0)]))
        # Observation = projection + noise; some outliers so Huber takes both
        # branches.
        noise = rng.normal(size=2) if idx % 5 else rng.uniform(-50, 50, size=2)
        obs = [float(clean[0]) + float(noise[0]), float(clean[1]) + float(noise[1])]
        args = args0 + [mpmath.mpf(obs[0]), mpmath.mpf(obs[1])]
        rv = [fr(*args)[i] for i in range(2)]
        Jm = fJ(*args)
        Jrows = [[Jm[i, j] for j in range(Jm.cols)] for i in range(2)]
        sq = rv[0] ** 2 + rv[1] ** 2
        entry = {"functor": functor, "camera": cam, "point": pt, "obs": obs,
                 "residuals": [float(x) for x in rv],
                 "jacobian": [[float(x) for x in row] for row in Jrows],
                 "losses": []}
        for loss_kind, a in ((0, 1.0), (1, 1.0), (1, 4.0), (2, 1.0), (2, 3.0)):
            rho = loss_rho(loss_kind, a, sq)
            if loss_kind == 0:
                rc, Jc = rv, Jrows
            else:
                rc, Jc = correct(rv, Jrows, rho, sq)
            entry["losses"].append({
                "loss": loss_kind, "a": a, "cost": float(rho[0] / 2),
                "residuals": [float(x) for x in rc],
                "jacobian": [[float(x) for x in row] for row in Jc]})
        out.append(entry)
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as fh:
        json.dump({"generator": "oracle/gen_golden.py", "dps": 50,
                   "seed": 0xCE2E5, "cases": out}, fh, indent=0)
    print(f"wrote {len(out)} cases to {OUT}")


if __name__ == "__main__":
    main()
