#!/bin/bash
# Exec-masked stores ahead of the unmasked windows: held-camera side slots
# first (lib/s1 vs h4), fused-gradient rows/entries first (lib/gf vs s1).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
T=${TAG:-r4s5}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gradient_gpu.py tests/test_constant_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
TAG=$T/ab_held MODE=jacobian PREV=h4 ALT=s1 ABFLAGS="--held-cameras 1" bash tools/gpu_ab_alt.sh || exit 1
TAG=$T/ab_grad MODE=gradient PREV=s1 ALT=gf bash tools/gpu_ab_alt.sh || exit 1
TAG=$T/ab_plain MODE=jacobian PREV=h4 ALT=s1 bash tools/gpu_ab_alt.sh || exit 1
