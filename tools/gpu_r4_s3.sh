#!/bin/bash
# Round 4 session 3: the full GPU suite on the current build, then the
# held-camera A/B program under a kernel trace (where its extra time goes).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
T=${TAG:-r4s3}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=15 --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "pytest rc=$?"; tail -20 $OUT/pytest_gpu.txt; exit 1; }
tail -2 $OUT/pytest_gpu.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_ab_held -o run --output-format csv -- python3 tools/ab_bench.py --lib ceres-solver-cuda_amd/lib/libcse.so --variants 0 --rounds 1 --steps 10 --held-cameras 1 > $OUT/ab_held.txt 2>&1 || { echo "trace rc=$?"; tail -5 $OUT/ab_held.txt; exit 1; }
tail -2 $OUT/ab_held.txt
