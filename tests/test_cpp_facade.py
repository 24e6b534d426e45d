"""The C++ ProblemCUDA facade: builds here (g++ against the C ABI; hipcc for
the user functor TU), runs its parity tests (tests/cpp/test_problem_cuda.cpp,
tests/cpp/test_user_facade.hip) on the GPU."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CPP = os.path.join(HERE, "cpp")


def build(name="test_problem_cuda"):
    subprocess.check_call(["make", "-s", "-C", CPP])
    return os.path.join(CPP, "build", name)


def test_facade_builds_and_links():
    exe = build()
    assert os.access(exe, os.X_OK)


@pytest.mark.gpu
def test_facade_mini_bundle_adjustment_parity(gpu):
    exe = build()
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "OK" in out.stdout


@pytest.mark.gpu
def test_user_functors_through_the_facade(gpu):
    """tests/cpp/test_user_facade.hip: the reference's test functors and
    BundlerResidual with a user loss, as user functors of a hipcc TU through
    ProblemCUDA::AddResidualBlock, against the oracle."""
    exe = build("test_user_facade")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "OK" in out.stdout
