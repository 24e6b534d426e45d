#!/bin/bash
# Round 4: the camera-gradient point copy (CSE_POINT_COPY) -- gradient tests
# on the product build, same-box A/B of lib/prev (no copy) vs lib/alt (copy),
# then per-kernel PMC of the alt build's gradient evaluation.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
OUT=gpurun_out/${TAG:-r4g}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gradient_gpu.py tests/test_constant_gpu.py tests/test_asan.py \
  tests/test_manifold_gpu.py tests/test_same_point_gpu.py tests/test_schur_gpu.py -m "gpu" -x -q \
  --timeout 300 --timeout-method thread -k "not problem_13682" > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
TAG=${TAG:-r4g}/ab MODE=gradient bash tools/gpu_ab_alt.sh || exit 1
BENCH_ARGS="--lib ceres-solver-cuda_amd/lib/alt/libcse.so --gradient --no-cpu-baseline --no-secondary --steps 5 --warmup 1" \
  bash tools/gpu_pmc_kernels.sh ${TAG:-r4g}/pmc_alt || exit 1
timeout -k 10 120 tools/membench3 10 > gpurun_out/${TAG:-r4g}/membench3.txt 2>&1 || { echo "membench3 rc=$?"; tail -5 gpurun_out/${TAG:-r4g}/membench3.txt; exit 1; }
cat gpurun_out/${TAG:-r4g}/membench3.txt
