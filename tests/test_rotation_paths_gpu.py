"""GPU parity of both AngleAxisRotatePoint forms (csrc/functors.hpp).

The device evaluates a block's rotation as Rodrigues' formula with
sin(theta)/theta and (1 - cos(theta))/theta^2 as series in theta^2 when its
camera has theta^2 <= 1, and with the reference's form
(include/ceres/rotation.h:830-899: hypot, sin/cos, 1/theta) otherwise -- per
lane, so a block's outputs do not depend on the other blocks of its wave.  The
synthetic BAL generator draws small angles, so these tests set the camera
angle-axis vectors explicitly: all waves small (series only), all large
(reference form only), mixed waves, theta exactly 0 and tiny theta (the
reference's first-order branch and its neighbourhood), and the theta^2 = 1
boundary.  Each is checked against the oracle (which always follows the
reference's form) at the tolerances of tests/parity_util.py, on the affine
and the general path, with the gradient.
"""
import numpy as np
import pytest

import ceres_amd as ca
from ceres_amd import bal
import oracle_py as O
from parity_util import TOL, assert_parity, elementwise_report

pytestmark = pytest.mark.gpu

C, P, N_OBS = 96, 900, 4000


def _problem(angles, seed, loss, fmt, with_obs=False):
    cams, pts, ci, pi, _ = bal.synthetic(C, P, N_OBS, seed=seed)
    rng = np.random.default_rng(seed)
    axis = rng.normal(size=(C, 3))
    axis /= np.linalg.norm(axis, axis=1)[:, None]
    cams = cams.copy()
    cams[:, 0:3] = axis * np.asarray(angles, float)[:, None]
    obs = bal.project(cams, pts, ci, pi) + rng.normal(0.0, 1.0, (len(ci), 2))
    prog = bal.program(cams, pts, ci, pi, obs, loss=loss, format=fmt)
    return (prog, obs) if with_obs else prog


def _angles(kind, seed):
    rng = np.random.default_rng(100 + seed)
    if kind == "small":        # theta^2 <= 1 everywhere: the series form only
        # From 1e-3 up: below that the reference's form itself loses the
        # Jacobian to cancellation in 1 - cos(theta) (its error grows like
        # 1e-18 / theta), so tiny angles are checked against exact values
        # instead (test_tiny_angles_against_exact_values).
        a = rng.uniform(1e-3, 1.0, C)
        a[:2] = [0.0, 1.0]
    elif kind == "large":      # every wave sees theta^2 > 1: the reference form
        a = rng.uniform(1.0001, 3.14, C)
    elif kind == "mixed":      # some waves all small, some mixed
        a = np.where(rng.random(C) < 0.05, rng.uniform(1.0, 6.0, C), rng.uniform(0.0, 1.0, C))
        a[:3] = [0.0, 2.0 ** -30, 1.0 + 2.0 ** -52]
    else:                      # beyond pi: angle-axis vectors of any length
        a = rng.uniform(3.0, 12.0, C)
    return a


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
@pytest.mark.parametrize("kind", ["small", "large", "mixed", "beyond_pi"])
def test_rotation_forms_match_the_oracle(gpu, kind, fmt):
    # No loss, so r = predicted - observed and its cancellation can be
    # accounted for (the golden-vector tests' convention): the residuals are
    # held to 1e-13 |predicted| norm-wise plus the per-element bound.
    angles = _angles(kind, 3)
    prog, obs = _problem(angles, 3, None, fmt, with_obs=True)
    # Cameras with 0 < theta < 1e-3 take the series form (theta^2 <= 1),
    # while the oracle follows the reference's form, which loses the Jacobian
    # to cancellation below theta ~ 1e-6 (deviation 5): their
    # Jacobian cells and gradient rows are held to 1e-7 relative here, and
    # test_tiny_angles_against_exact_values pins the series form against
    # 40-digit values.
    tiny_cams = np.flatnonzero((angles > 0) & (angles < 1e-3))
    tiny = np.zeros(prog.num_effective_parameters, bool)
    for c in tiny_cams:
        tiny[3 * P + 9 * c: 3 * P + 9 * (c + 1)] = True
    tiny_j = np.zeros(prog.num_jacobian_values, bool)
    blocks = np.flatnonzero(np.isin(prog.groups[0].ids[:, 0] - P, tiny_cams))
    for b in blocks:  # the camera slot's two 9-value rows of each such block
        for k in range(2):
            o = prog.jacobian_per_residual_offsets[prog.jacobian_per_residual_layout[b] + k]
            tiny_j[o:o + 9] = True
    op = O.OracleProgram.from_program(prog, apply_loss_function=True)
    ref = op.evaluate(prog.state, None, num_threads=8)
    for general in (False, True):
        ev = ca.Evaluator(prog, force_general_layout=general)
        try:
            got = ev.evaluate()
        finally:
            ev.close()
        # Residuals, Jacobian, cost: the reference's isApprox 1e-13 and the
        # per-element bound.  The gradient g = J^T r of these problems cancels
        # to |g| ~ 1e-2 |J| |r| (random rotations, 4,000 blocks), where one
        # ulp on the operands already moves g by more than 1e-13 |g| (the
        # reference form on both sides gives 1.6e-13 for "large"), so it is
        # held to the first-order perturbation bound 1e-13 |J| |r| and the
        # per-element bound.
        ok, cost, r, g, j = got
        j_ref = ref[4]
        if tiny_j.any():
            jt, jt_ref = j[tiny_j], j_ref[tiny_j]
            assert np.linalg.norm(jt - jt_ref) <= 1e-7 * np.linalg.norm(jt_ref), (kind, fmt, general)
            nz = jt_ref != 0
            print(f"tiny-angle carve-out ({kind}, {fmt}, general={general}): "
                  f"{len(tiny_cams)} camera(s) with 0 < theta < 1e-3, worst Jacobian cell "
                  f"relative difference to the oracle "
                  f"{np.max(np.abs(jt[nz] - jt_ref[nz]) / np.abs(jt_ref[nz])):.2e} (held to 1e-7)")
            j, j_ref = j[~tiny_j], j_ref[~tiny_j]
        assert_parity((ok, cost, None, None, j), (ref[0], ref[1], None, None, j_ref),
                      (kind, fmt, general))
        pred = np.linalg.norm(ref[2] + obs.ravel())
        assert np.linalg.norm(r - ref[2]) <= TOL * pred, (kind, fmt, general)
        assert elementwise_report(r, ref[2])["bound_ratio"] <= 1.0, (kind, fmt, general)
        g_ref = ref[3]
        if tiny.any():
            gt, gt_ref = g[tiny], g_ref[tiny]
            assert np.linalg.norm(gt - gt_ref) <= 1e-7 * np.linalg.norm(gt_ref), \
                (kind, fmt, general, np.linalg.norm(gt - gt_ref) / np.linalg.norm(gt_ref))
            g, g_ref = g[~tiny], g_ref[~tiny]
        assert np.linalg.norm(g - g_ref) <= TOL * np.linalg.norm(ref[4]) * np.linalg.norm(ref[2]), \
            (kind, fmt, general, np.linalg.norm(g - g_ref) / np.linalg.norm(g_ref))
        assert elementwise_report(g, g_ref)["bound_ratio"] <= 1.0, (kind, fmt, general)


def _snavely_mp(mp, cam, pt, obs):
    """SnavelyReprojectionError in mpmath, Rodrigues written without the
    1 - cos(theta) cancellation: (1 - cos t) / t^2 = 2 sin(t/2)^2 / t^2."""
    aa = cam[0:3]
    t2 = sum(a * a for a in aa)
    t = mp.sqrt(t2)
    s = mp.sin(t) / t if t != 0 else mp.mpf(1)
    c = 2 * mp.sin(t / 2) ** 2 / t2 if t != 0 else mp.mpf("0.5")
    q = [aa[1] * pt[2] - aa[2] * pt[1], aa[2] * pt[0] - aa[0] * pt[2], aa[0] * pt[1] - aa[1] * pt[0]]
    m = [aa[1] * q[2] - aa[2] * q[1], aa[2] * q[0] - aa[0] * q[2], aa[0] * q[1] - aa[1] * q[0]]
    p = [pt[i] + s * q[i] + c * m[i] + cam[3 + i] for i in range(3)]
    xp, yp = -p[0] / p[2], -p[1] / p[2]
    r2 = xp * xp + yp * yp
    d = 1 + r2 * (cam[7] + cam[8] * r2)
    return [cam[6] * d * xp - obs[0], cam[6] * d * yp - obs[1]]


@pytest.mark.parametrize("fmt", [ca.BLOCK_SPARSE, ca.COMPRESSED_ROW])
def test_tiny_angles_against_exact_values(gpu, fmt):
    # theta = 0, 1e-150, 1e-12, 1e-9, 1e-6, 1e-3: residuals and Jacobian of
    # SnavelyReprojectionError<2,9,3> (no loss) against 40-digit values.  The
    # oracle (the reference's form in double) is only printed: at 1e-9 its
    # Jacobian is off by ~1e-9 (1 - cos(theta) rounds to 0).
    mp = pytest.importorskip("mpmath")
    mp.mp.dps = 40
    rng = np.random.default_rng(11)
    angles = [0.0, 1e-150, 1e-12, 1e-9, 1e-6, 1e-3]
    p = ca.ProblemCUDA()
    blocks = []
    for th in angles:
        axis = rng.normal(size=3)
        axis /= np.linalg.norm(axis)
        cam = np.concatenate([axis * th, rng.normal(0, 1, 2), [-10 + rng.normal()],
                              [rng.uniform(400, 1200)], rng.normal(0, [0.05, 0.01])])
        pt = rng.uniform(-3, 3, 3)
        obs = rng.normal(0, 5, 2)
        ci = p.add_parameter_block(cam)
        pi = p.add_parameter_block(pt)
        p.add_residual_block(ca.SNAVELY_2_9_3, None, obs, ci, pi)
        blocks.append((cam, pt, obs))
    prog = p.program()
    prog.compile(fmt)
    ev = ca.Evaluator(prog)
    try:
        ok, cost, r, g, j = ev.evaluate()
    finally:
        ev.close()
    assert ok
    op = O.OracleProgram.from_program(prog, apply_loss_function=True)
    ok_o, _, r_o, _, j_o = op.evaluate(prog.state, None, num_threads=1)
    worst = {"oracle": 0.0, "exact": 0.0, "oracle_at": None, "exact_at": None}
    for k, (cam, pt, obs) in enumerate(blocks):
        x = [mp.mpf(float(v)) for v in list(cam) + list(pt)]
        o = [mp.mpf(float(v)) for v in obs]
        f = lambda *v: _snavely_mp(mp, v[:9], v[9:], o)
        r_ex = np.array([float(v) for v in f(*x)])
        J_ex = np.zeros((2, 12))
        for col in range(12):
            for row in range(2):
                J_ex[row, col] = float(mp.diff(lambda t: f(*(x[:col] + [x[col] + t] + x[col + 1:]))[row], 0))
        if fmt == ca.COMPRESSED_ROW:
            Jk = j[24 * k:24 * k + 24].reshape(2, 12)
            Jo = j_o[24 * k:24 * k + 24].reshape(2, 12)
        else:
            Jk = np.hstack([j[24 * k:24 * k + 18].reshape(2, 9), j[24 * k + 18:24 * k + 24].reshape(2, 3)])
            Jo = np.hstack([j_o[24 * k:24 * k + 18].reshape(2, 9),
                            j_o[24 * k + 18:24 * k + 24].reshape(2, 3)])
        scale = np.linalg.norm(obs) + np.linalg.norm(r_ex)
        assert np.linalg.norm(r[2 * k:2 * k + 2] - r_ex) <= 1e-13 * scale, (angles[k], r[2 * k:2 * k + 2], r_ex)
        err = np.linalg.norm(Jk - J_ex) / np.linalg.norm(J_ex)
        print(f"theta {angles[k]:g}: GPU Jacobian rel err {err:.2e}, oracle (reference form) "
              f"{np.linalg.norm(Jo - J_ex) / np.linalg.norm(J_ex):.2e}")
        assert err <= 1e-13, (angles[k], err)
        if 0.0 < angles[k] < 1e-3:  # the carve-out: series form vs the reference's form
            nz = (Jo != 0) & (J_ex != 0)
            vo = float(np.max(np.abs(Jk[nz] - Jo[nz]) / np.abs(Jo[nz])))
            ve = float(np.max(np.abs(Jk[nz] - J_ex[nz]) / np.abs(J_ex[nz])))
            if vo > worst["oracle"]:
                worst["oracle"], worst["oracle_at"] = vo, angles[k]
            if ve > worst["exact"]:
                worst["exact"], worst["exact_at"] = ve, angles[k]
    print(f"tiny-angle parity report ({fmt}): worst Jacobian cell of a camera with "
          f"0 < theta < 1e-3, relative difference to the oracle (the reference's form) "
          f"{worst['oracle']:.2e} at theta {worst['oracle_at']:g}; to the 40-digit values "
          f"{worst['exact']:.2e} at theta {worst['exact_at']:g}")
    assert worst["exact"] <= 1e-12
