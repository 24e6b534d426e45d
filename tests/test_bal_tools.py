"""BAL problem tools: BALProblem::Normalize / Perturb
restated in ceres_amd.bal (examples/bal_problem.cc:246-330).

* Perturb reproduces the reference's random stream: std::mt19937 (default
  seed) through libstdc++'s std::normal_distribution, a fresh distribution
  copy per 3-vector (std::bind copies it).  Pinned against the standard
  library itself (tests/cpp/std_normal_stream.cpp, compiled here).
* Normalize is a similarity of the world: every predicted observation is
  unchanged, the points' marginal median moves to 0 and their L1 median
  absolute deviation to 100.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from ceres_amd import bal

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def std_stream(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("stdn") / "std_normal_stream")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe,
                    os.path.join(HERE, "cpp", "std_normal_stream.cpp")], check=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    return np.array([[float(x) for x in line.split()] for line in out.strip().splitlines()])


def test_perturb_noise_stream_is_libstdcxx(std_stream):
    bg = np.random.MT19937()
    bg._legacy_seeding(5489)
    nd = bal._StdNormal(bg)
    rows = []
    for _ in range(4):
        rows.append(nd.draws(3, 0.5))
        rows.append(nd.draws(3, 2.0))
    np.testing.assert_array_equal(np.array(rows), std_stream)


def test_perturb_matches_reference_draw_order():
    cams, pts, ci, pi, obs = bal._synthetic(5, 7, 30, 1, 0.0)
    c0, p0 = cams.copy(), pts.copy()
    bal.perturb(cams, pts, rotation_sigma=0.1, translation_sigma=0.3, point_sigma=0.2)
    bg = np.random.MT19937()
    bg._legacy_seeding(5489)
    nd = bal._StdNormal(bg)
    pe = np.stack([nd.draws(3, 0.2) for _ in range(7)])
    np.testing.assert_array_equal(pts, p0 + pe)
    for i in range(5):
        rot = nd.draws(3, 0.2)   # the reference draws rotation noise with point_sigma
        tr = nd.draws(3, 0.3)
        aa, center = bal.camera_to_angle_axis_and_center(c0[i:i + 1])
        ref = c0[i:i + 1].copy()
        bal.angle_axis_and_center_to_camera(aa + rot, center, ref)
        ref[0, 3:6] += tr
        np.testing.assert_allclose(cams[i], ref[0], rtol=0, atol=1e-12)


def test_normalize_is_a_similarity():
    cams, pts, ci, pi, obs = bal._synthetic(9, 200, 900, 3, 0.0)
    before = bal.project(cams, pts, ci, pi)
    median, scale = bal.normalize(cams, pts)
    after = bal.project(cams, pts, ci, pi)
    assert np.allclose(after, before, rtol=1e-9, atol=1e-9)
    med = np.array([np.partition(pts[:, k], 100)[100] for k in range(3)])
    assert np.allclose(med, 0.0, atol=1e-9)
    mad = np.partition(np.abs(pts).sum(axis=1), 100)[100]
    assert abs(mad - 100.0) < 1e-9


def test_angle_axis_rotate_matches_projection_model():
    rng = np.random.default_rng(2)
    aa = rng.normal(scale=0.3, size=(50, 3))
    aa[0] = 0.0
    pts = rng.normal(size=(50, 3))
    out = bal.angle_axis_rotate(aa, pts)
    back = bal.angle_axis_rotate(-aa, out)
    np.testing.assert_allclose(back, pts, atol=1e-12)
    np.testing.assert_array_equal(out[0], pts[0])
