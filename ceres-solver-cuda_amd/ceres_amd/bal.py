"""BAL (Bundle Adjustment in the Large) problems for the evaluator.

* synthetic(C, P, O, seed): a BAL-shaped problem with exactly the header
  counts of a real BAL file; no BAL file is available
  offline.  Point-major observations, each point seen by floor/ceil(O/P)
  distinct cameras drawn uniformly without replacement; cameras
  aa ~ N(0, 0.05^2) (camera 0 exactly zero: the Taylor branch of
  AngleAxisRotatePoint), t = (N(0,1), N(0,1), -10 + N(0,1)),
  f ~ U[400, 1200], l1 ~ N(0, 0.05^2), l2 ~ N(0, 0.01^2); points
  ~ U[-3, 3]^3; obs = projection + N(0, 1) px, 5% outliers U(-50, 50) px.
* read(path): the BAL text format (examples/bal_problem.cc:72-132).
* program(...): the Ceres Program for bundle_adjuster's Schur setup
  (examples/bundle_adjuster.cu.cc:307-353 BuildProblem + the points-first
  elimination ordering): points are the E blocks (parameter blocks 0..P-1),
  cameras follow, residual blocks are grouped by point
  (reorder_program.cc:254-336).
"""
import os

import numpy as np

from . import _cse
from .problem import BLOCK_SPARSE, Loss, Program, ResidualGroup

# (cameras, points, observations) of the BAL files named in BASELINE.json.
CONFIGS = {
    "problem-16-22106": (16, 22106, 83718),
    "problem-1778-993923": (1778, 993923, 5001946),
    "problem-13682-4456117": (13682, 4456117, 28987644),
}


def project(cameras, points, cam_idx, pt_idx):
    """Snavely projection in numpy (generator only: observations are the
    model's prediction plus noise)."""
    cam = cameras[cam_idx]
    X = points[pt_idx]
    aa = cam[:, 0:3]
    theta = np.sqrt((aa * aa).sum(1))
    safe = np.where(theta > 0, theta, 1.0)
    w = aa / safe[:, None]
    ct, st = np.cos(theta), np.sin(theta)
    wx = np.cross(w, X)
    wd = (w * X).sum(1)
    rot = X * ct[:, None] + wx * st[:, None] + w * (wd * (1 - ct))[:, None]
    rot0 = X + np.cross(aa, X)
    p = np.where((theta > 0)[:, None], rot, rot0) + cam[:, 3:6]
    xp, yp = -p[:, 0] / p[:, 2], -p[:, 1] / p[:, 2]
    r2 = xp * xp + yp * yp
    d = 1.0 + r2 * (cam[:, 7] + cam[:, 8] * r2)
    return np.stack([cam[:, 6] * d * xp, cam[:, 6] * d * yp], 1)


def synthetic(num_cameras, num_points, num_observations, seed=0xCE2E5, outlier_fraction=0.05):
    """Returns (cameras[C,9], points[P,3], cam_idx[O], pt_idx[O], obs[O,2]) in
    point-major order.  If $CSE_BAL_CACHE names a directory, the arrays are
    cached there (profiling runs regenerate the same problem many times)."""
    cache = os.environ.get("CSE_BAL_CACHE")
    if cache:
        path = os.path.join(cache, f"bal_{num_cameras}_{num_points}_{num_observations}_"
                                   f"{seed}_{outlier_fraction}.npz")
        if os.path.exists(path):
            with np.load(path) as z:
                return z["cameras"], z["points"], z["cam_idx"], z["pt_idx"], z["obs"]
        out = _synthetic(num_cameras, num_points, num_observations, seed, outlier_fraction)
        os.makedirs(cache, exist_ok=True)
        tmp = path + f".{os.getpid()}.npz"
        np.savez(tmp, cameras=out[0], points=out[1], cam_idx=out[2], pt_idx=out[3], obs=out[4])
        os.replace(tmp, path)
        return out
    return _synthetic(num_cameras, num_points, num_observations, seed, outlier_fraction)


def _synthetic(num_cameras, num_points, num_observations, seed, outlier_fraction):
    C, P, O = int(num_cameras), int(num_points), int(num_observations)
    if O < P:
        raise ValueError("need at least one observation per point")
    rng = np.random.Generator(np.random.PCG64(seed))
    cameras = np.empty((C, 9))
    cameras[:, 0:3] = rng.normal(0.0, 0.05, (C, 3))
    cameras[0, 0:3] = 0.0
    cameras[:, 3:5] = rng.normal(0.0, 1.0, (C, 2))
    cameras[:, 5] = -10.0 + rng.normal(0.0, 1.0, C)
    cameras[:, 6] = rng.uniform(400.0, 1200.0, C)
    cameras[:, 7] = rng.normal(0.0, 0.05, C)
    cameras[:, 8] = rng.normal(0.0, 0.01, C)
    points = rng.uniform(-3.0, 3.0, (P, 3))

    base, extra = divmod(O, P)
    if base + (1 if extra else 0) > C:
        raise ValueError("more observations per point than cameras")
    counts = np.full(P, base, np.int64)
    counts[:extra] += 1
    cam_idx = np.empty(O, np.int32)
    pt_idx = np.repeat(np.arange(P, dtype=np.int32), counts)
    starts = np.zeros(P + 1, np.int64)
    np.cumsum(counts, out=starts[1:])
    for k, sel in ((base + 1, slice(0, extra)), (base, slice(extra, P))):
        npts = len(range(*sel.indices(P)))
        if npts == 0 or k == 0:
            continue
        m = _distinct_rows(rng, npts, k, C)
        first = starts[sel.start]
        cam_idx[first:first + npts * k] = m.ravel()
    obs = project(cameras, points, cam_idx, pt_idx)
    obs += rng.normal(0.0, 1.0, obs.shape)
    out = rng.random(O) < outlier_fraction
    obs[out] += rng.uniform(-50.0, 50.0, (int(out.sum()), 2))
    return cameras, points, cam_idx, pt_idx, obs


def _distinct_rows(rng, n, k, C):
    """n rows of k distinct integers in [0, C)."""
    if k * k > 4 * C:
        # Dense rows (most of the cameras per point, test shapes only):
        # rejection sampling would almost never draw k distinct values.
        return np.argsort(rng.random((n, C)), axis=1)[:, :k].astype(np.int32)
    m = rng.integers(0, C, (n, k), dtype=np.int32)
    while True:
        s = np.sort(m, axis=1)
        bad = (s[:, 1:] == s[:, :-1]).any(axis=1)
        nb = int(bad.sum())
        if nb == 0:
            return m
        m[bad] = rng.integers(0, C, (nb, k), dtype=np.int32)


def read(path):
    """BAL text file -> (cameras, points, cam_idx, pt_idx, obs) in file order."""
    with open(path) as fh:
        C, P, O = (int(x) for x in fh.readline().split())
        obs_rows = np.loadtxt(fh, max_rows=O)
        params = np.loadtxt(fh).ravel()
    cam_idx = obs_rows[:, 0].astype(np.int32)
    pt_idx = obs_rows[:, 1].astype(np.int32)
    obs = obs_rows[:, 2:4].copy()
    cameras = params[: 9 * C].reshape(C, 9)
    points = params[9 * C: 9 * C + 3 * P].reshape(P, 3)
    return cameras, points, cam_idx, pt_idx, obs


# --------------------------------------------------------------------------
# BALProblem::Normalize / Perturb (examples/bal_problem.cc:246-330), angle-axis
# cameras ([aa 3 | t 3 | f k1 k2]).
# --------------------------------------------------------------------------
def angle_axis_rotate(aa, pts):
    """AngleAxisRotatePoint (rotation.h:830-899), row-wise: Rodrigues, or
    the first-order form when theta^2 <= DBL_EPSILON."""
    aa = np.asarray(aa, np.float64)
    pts = np.asarray(pts, np.float64)
    th2 = np.einsum("ij,ij->i", aa, aa)
    big = th2 > np.finfo(np.float64).eps
    out = pts + np.cross(aa, pts)
    if big.any():
        th = np.sqrt(th2[big])
        w = aa[big] / th[:, None]
        c, s_ = np.cos(th)[:, None], np.sin(th)[:, None]
        p = pts[big]
        wxp = np.cross(w, p)
        tmp = np.einsum("ij,ij->i", w, p)[:, None] * (1.0 - c)
        out[big] = p * c + wxp * s_ + w * tmp
    return out


def _median(x):
    """Median() of bal_problem.cc:64-68: std::nth_element at size/2."""
    x = np.asarray(x, np.float64)
    return float(np.partition(x, x.size // 2)[x.size // 2])


def camera_to_angle_axis_and_center(cameras):
    """CameraToAngleAxisAndCenter: c = -R^T t."""
    aa = cameras[:, 0:3].copy()
    center = -angle_axis_rotate(-aa, cameras[:, 3:6])
    return aa, center


def angle_axis_and_center_to_camera(aa, center, cameras):
    """AngleAxisAndCenterToCamera: t = -R c (writes aa and t in place)."""
    cameras[:, 0:3] = aa
    cameras[:, 3:6] = -angle_axis_rotate(aa, center)


def normalize(cameras, points):
    """BALProblem::Normalize (bal_problem.cc:246-287): points and camera
    centers translated by the marginal median and scaled so the median
    absolute deviation (L1) is 100.  In place; returns (median, scale)."""
    median = np.array([_median(points[:, i]) for i in range(3)])
    mad = _median(np.abs(points - median).sum(axis=1))
    scale = 100.0 / mad
    points[:] = scale * (points - median)
    aa, center = camera_to_angle_axis_and_center(cameras)
    angle_axis_and_center_to_camera(aa, scale * (center - median), cameras)
    return median, scale


class _StdNormal:
    """libstdc++ std::normal_distribution<double> over std::mt19937
    (Marsaglia polar method; generate_canonical<double, 53> from two 32-bit
    draws), so Perturb reproduces the reference's noise bit for bit.  The
    reference binds a *copy* of its distribution for every PerturbPoint3
    call (bal_problem.cc:304,321,327), so the saved second value is dropped
    after each 3-vector: fresh() models that copy."""

    def __init__(self, bitgen):
        self.bg = bitgen

    def _canonical(self):
        u1, u2 = (float(v) for v in self.bg.random_raw(2))
        s = u1
        s += u2 * 4294967296.0
        r = s / 18446744073709551616.0
        return r if r < 1.0 else np.nextafter(1.0, 0.0)

    def draws(self, n, stddev):
        out, saved = [], None
        for _ in range(n):
            if saved is not None:
                out.append(saved * stddev)
                saved = None
                continue
            while True:
                x = 2.0 * self._canonical() - 1.0
                y = 2.0 * self._canonical() - 1.0
                r2 = x * x + y * y
                if not (r2 > 1.0 or r2 == 0.0):
                    break
            mult = np.sqrt(-2.0 * np.log(r2) / r2)
            saved = x * mult
            out.append(y * mult * stddev)
        return np.array(out)


def perturb(cameras, points, rotation_sigma, translation_sigma, point_sigma):
    """BALProblem::Perturb (bal_problem.cc:289-330), in place, with the
    reference's own random stream (std::mt19937, default seed 5489).  As in
    the reference, the rotation noise uses point_sigma as its standard
    deviation (bal_problem.cc:309-310) and is drawn only when
    rotation_sigma > 0."""
    if min(rotation_sigma, translation_sigma, point_sigma) < 0:
        raise ValueError("sigmas must be non-negative")
    bg = np.random.MT19937()
    bg._legacy_seeding(5489)
    nd = _StdNormal(bg)
    if point_sigma > 0:
        for i in range(points.shape[0]):
            points[i] += nd.draws(3, point_sigma)
    for i in range(cameras.shape[0]):
        aa, center = camera_to_angle_axis_and_center(cameras[i:i + 1])
        if rotation_sigma > 0.0:
            aa = aa + nd.draws(3, point_sigma)
        angle_axis_and_center_to_camera(aa, center, cameras[i:i + 1])
        if translation_sigma > 0.0:
            cameras[i, 3:6] += nd.draws(3, translation_sigma)


def schur_residual_order(pt_idx, num_points):
    """LexicographicallyOrderResidualBlocks (reorder_program.cc:254-336):
    bucket residual blocks by their E block (point), each bucket filled
    from the back.  Returns the permutation new_position -> old index."""
    pt_idx = np.asarray(pt_idx, np.int64)
    ends = np.cumsum(np.bincount(pt_idx, minlength=num_points))
    sort = np.argsort(pt_idx, kind="stable")
    sp = pt_idx[sort]
    # rank of each block among its point's blocks, in the old order
    rank = np.empty(len(pt_idx), np.int64)
    rank[sort] = np.arange(len(sp)) - np.searchsorted(sp, sp, side="left")
    new_pos = ends[pt_idx] - 1 - rank
    perm = np.empty(len(pt_idx), np.int64)
    perm[new_pos] = np.arange(len(pt_idx))
    return perm


def to_quaternion_cameras(cameras):
    """The 10-parameter cameras {q[4], t[3], f, k1, k2} of BALProblem with
    use_quaternions (examples/bal_problem.cc:110-121): each angle-axis
    rotation through AngleAxisToQuaternion (include/ceres/rotation.h:
    320-352), the rest copied."""
    cameras = np.asarray(cameras, np.float64)
    aa = cameras[:, :3]
    theta = np.sqrt((aa * aa).sum(axis=1))
    nz = theta != 0.0
    half = theta * 0.5
    k = np.where(nz, np.sin(half) / np.where(nz, theta, 1.0), 0.5)
    out = np.empty((cameras.shape[0], 10))
    out[:, 0] = np.where(nz, np.cos(half), 1.0)
    out[:, 1:4] = aa * k[:, None]
    out[:, 4:] = cameras[:, 3:9]
    return out


def program(cameras, points, cam_idx, pt_idx, obs, loss=None, kind=None,
            format=BLOCK_SPARSE, compile=True, quaternion_manifold=False, constant_cameras=()):
    """The Schur-ordered Program of a BAL problem (observations must
    already be point-major, as synthetic() returns and
    schur_residual_order() produces).  10-parameter (quaternion) cameras
    take SNAVELY_QUATERNION_2_10_3; quaternion_manifold puts each on
    ProductManifold<QuaternionManifold, EuclideanManifold<6>>, as
    bundle_adjuster --use_quaternions --use_manifolds does
    (examples/bundle_adjuster.cc:337-345).  constant_cameras: camera indices
    held constant (Problem::SetParameterBlockConstant, e.g. to fix the gauge):
    their values move to the constant state and they get no delta columns."""
    if kind is None:
        kind = _cse.SNAVELY_QUATERNION_2_10_3 if cameras.shape[1] == 10 else _cse.SNAVELY_2_9_3
    C, P = cameras.shape[0], points.shape[0]
    cam_size = cameras.shape[1]
    npb = P + C
    pb_size = np.empty(npb, np.int32)
    pb_size[:P] = 3
    pb_size[P:] = cam_size
    ids = np.empty((len(cam_idx), 2), np.int32)
    ids[:, 0] = P + np.asarray(cam_idx, np.int32)
    ids[:, 1] = pt_idx
    group = ResidualGroup(kind, loss or Loss.trivial(), ids, np.ascontiguousarray(obs, np.float64),
                          None, 0)
    const = np.zeros(npb, np.int32)
    cstate = np.zeros(0)
    if len(constant_cameras):
        cc = np.zeros(C, bool)
        cc[np.asarray(constant_cameras, np.int64)] = True
        const[P:] = cc
        state = np.concatenate([points.ravel(), cameras[~cc].ravel()])
        cstate = np.ascontiguousarray(cameras[cc].ravel(), np.float64)
    else:
        state = np.concatenate([points.ravel(), cameras.ravel()])
    prog = Program(pb_size, pb_size.copy(), const, np.full(npb, -1, np.int64),
                   np.zeros(0), [group], len(cam_idx), state, cstate)
    if quaternion_manifold:
        assert cam_size == 10, "quaternion cameras"
        prog.pb_manifold = np.zeros(npb, np.int32)
        prog.pb_manifold[P:] = _cse.MANIFOLD_QUATERNION_EUCLIDEAN
        prog.pb_tangent[P:] = 9
    if compile:
        prog.compile(format, num_eliminate_blocks=P)
    return prog


def synthetic_program(name_or_counts, loss=None, format=BLOCK_SPARSE, seed=0xCE2E5,
                      compile=True, quaternion=False, quaternion_manifold=False,
                      constant_cameras=()):
    """A synthetic BAL Program; quaternion: 10-parameter cameras
    (to_quaternion_cameras), optionally on the quaternion manifold."""
    counts = CONFIGS[name_or_counts] if isinstance(name_or_counts, str) else name_or_counts
    cams, pts, ci, pi, obs = synthetic(*counts, seed=seed)
    if quaternion or quaternion_manifold:
        cams = to_quaternion_cameras(cams)
    return program(cams, pts, ci, pi, obs, loss=loss, format=format, compile=compile,
                   quaternion_manifold=quaternion_manifold, constant_cameras=constant_cameras)
