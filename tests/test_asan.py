"""AddressSanitizer + UBSan runs of the host code (the
reference's SANITIZERS CMake option, CMakeLists.txt:156-158).

CPU: the layout builders (ceres-solver-cuda_amd/csrc/layout.cpp) and the
oracle (oracle/oracle.cpp) instrumented, tests/cpp/asan_driver.cpp part A.
GPU: the host half of libcse (descriptor validation, layout detection,
gradient and Schur plans, the multi-device sharding, error paths) and the
C++ ProblemCUDA facade instrumented, run against the device: asan_driver
part B and tests/cpp/test_problem_cuda.cpp.  The instrumented binaries are
built in this container (`make -C tests/cpp asan-hip`, by build()); device
code is never instrumented (GPU sanitizers are not available).  Leak
detection is off for the GPU runs: the HIP runtime keeps its allocations
until exit.
"""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CPP = os.path.join(HERE, "cpp")


def _run(exe, leaks):
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = f"detect_leaks={1 if leaks else 0}:abort_on_error=0"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    out = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    print(out.stdout[-3000:], out.stderr[-3000:])
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "OK" in out.stdout
    assert "ERROR: AddressSanitizer" not in out.stderr
    assert "runtime error" not in out.stderr


def test_asan_layout_builders_and_oracle():
    subprocess.check_call(["make", "-s", "-C", CPP, "asan-cpu"])
    _run(os.path.join(CPP, "build", "asan_cpu"), leaks=True)


@pytest.mark.gpu
@pytest.mark.parametrize("exe", ["asan_hip", "asan_facade"])
def test_asan_libcse_host_code_on_the_gpu(gpu, exe):
    path = os.path.join(CPP, "build", exe)
    assert os.path.exists(path), f"{path} not built (make -C tests/cpp asan-hip)"
    _run(path, leaks=False)
