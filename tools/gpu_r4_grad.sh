#!/bin/bash
# Round 4 session: (1) GPU tests of the changed areas on the product build;
# (2) same-box A/Bs: gradient evaluation without / with the camera-gradient
# point copy (lib/pc0 vs the product), held-camera Jacobian evaluation before
# / after the sector-aligned held-camera tail (lib/h0 vs lib/h1); (3) PMC of
# the product's gradient evaluation; (4) membench3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
T=${TAG:-r4g}
OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_constant_gpu.py tests/test_gradient_gpu.py tests/test_asan.py \
  tests/test_manifold_gpu.py tests/test_same_point_gpu.py tests/test_schur_gpu.py tests/test_multi_device_gpu.py \
  -m "gpu" -x -q --timeout 300 --timeout-method thread -k "not problem_13682 and not configs4" > $OUT/pytest.txt 2>&1 \
  || { echo "pytest rc=$?"; tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
cp ceres-solver-cuda_amd/lib/libcse.so ceres-solver-cuda_amd/lib/pc1.so 2>/dev/null; mkdir -p ceres-solver-cuda_amd/lib/pc1 && mv ceres-solver-cuda_amd/lib/pc1.so ceres-solver-cuda_amd/lib/pc1/libcse.so
TAG=$T/ab_grad MODE=gradient PREV=pc0 ALT=pc1 bash tools/gpu_ab_alt.sh || exit 1
TAG=$T/ab_held MODE=jacobian PREV=h0 ALT=h1 ABFLAGS="--held-cameras 1" bash tools/gpu_ab_alt.sh || exit 1
TAG=$T/ab_plain MODE=jacobian PREV=h0 ALT=h1 bash tools/gpu_ab_alt.sh || exit 1
BENCH_ARGS="--gradient --no-cpu-baseline --no-secondary --steps 5 --warmup 1" \
  bash tools/gpu_pmc_kernels.sh $T/pmc_grad || exit 1
timeout -k 10 120 tools/membench3 10 > $OUT/membench3.txt 2>&1 || { echo "membench3 rc=$?"; tail -5 $OUT/membench3.txt; exit 1; }
cat $OUT/membench3.txt
