#!/bin/bash
# Unmasked fused-gradient stores (lib/g1 vs g0) and the all-lanes cost
# partial (lib/pa vs g1); gradient and held-camera tests on the product build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
T=${TAG:-r4s4}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gradient_gpu.py tests/test_constant_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
TAG=$T/ab_grad MODE=gradient PREV=g0 ALT=g1 bash tools/gpu_ab_alt.sh || exit 1
TAG=$T/ab_partial MODE=jacobian PREV=g1 ALT=pa bash tools/gpu_ab_alt.sh || exit 1
