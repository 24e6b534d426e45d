#!/bin/bash
# Round 4: held-camera whole-sector windows -- the held-camera and multi-device
# GPU tests on the product build, then same-box A/B of the held-camera
# Jacobian evaluation (lib/h0: round-3 kernel, lib/h1: this build) with the
# unheld evaluation as the control, and the held bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
T=${TAG:-r4h}
OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_constant_gpu.py tests/test_multi_device_gpu.py -m "gpu" -x -q \
  --timeout 300 --timeout-method thread -k "not configs4" > $OUT/pytest.txt 2>&1 \
  || { echo "pytest rc=$?"; tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
TAG=$T/ab_held MODE=jacobian PREV=h0 ALT=h1 ABFLAGS="--held-cameras 1" bash tools/gpu_ab_alt.sh || exit 1
TAG=$T/ab_held_grad MODE=gradient PREV=h0 ALT=h1 ABFLAGS="--held-cameras 1" bash tools/gpu_ab_alt.sh || exit 1
TAG=$T/ab_plain MODE=jacobian PREV=h0 ALT=h1 bash tools/gpu_ab_alt.sh || exit 1
