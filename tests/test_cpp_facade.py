"""The C++ ProblemCUDA facade: builds here (g++ against the C ABI), runs its
parity test (tests/cpp/test_problem_cuda.cpp) on the GPU."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CPP = os.path.join(HERE, "cpp")


def build():
    subprocess.check_call(["make", "-s", "-C", CPP])
    return os.path.join(CPP, "build", "test_problem_cuda")


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
