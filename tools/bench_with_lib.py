#!/usr/bin/env python3
"""Run bench.py against another build of libcse.so (A/B of operator modes
that tools/ab_bench.py does not time, e.g. --mode schur / cgnr).

  python tools/bench_with_lib.py ceres-solver-cuda_amd/lib/NAME/libcse.so --mode schur --no-cpu-baseline
"""
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ceres-solver-cuda_amd"))

from ceres_amd import _cse  # noqa: E402

_cse.use_library(os.path.abspath(sys.argv[1]))
sys.argv = [os.path.join(REPO, "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
