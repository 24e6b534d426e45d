"""The Snavely camera's residual and Jacobian written out by hand
(csrc/functors.hpp SnavelyJacobianByHand, what every Snavely kernel runs on
the device) against AutoDifferentiate through the seeded Jet<12> -- the
reference's form, include/ceres/internal/autodiff.h:314-381 and
examples/snavely_reprojection_error.h:58-93 -- compiled for the host.

200,000 random blocks over five angle classes (theta exactly 0, ~1e-6,
~0.3, ~1.5, ~3 rad).  Bound: 1e-12 of the row's largest entry for the
Jacobian, 1e-12 relative for the residual, except the ~1e-6 class, where
the reference's Rodrigues form itself loses the rotation partials to
cancellation (the carve-out of DESIGN.md section 6 item 5; the GPU tests
check that class against 40-digit values instead)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CPP = os.path.join(HERE, "cpp")


def test_snavely_jacobian_by_hand_matches_jets():
    subprocess.check_call(["make", "-s", "-C", CPP, "build/byhand_check"])
    out = subprocess.run([os.path.join(CPP, "build", "byhand_check")], capture_output=True,
                         text=True, timeout=300)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
