#!/bin/bash
# Held cameras, unmasked window stores for whole chunks (lib/h4 = product
# build): the held-camera GPU tests, then plain/held/held-tail A/B against h3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
T=${TAG:-r4h4}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_constant_gpu.py tests/test_multi_device_gpu.py tests/test_gradient_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
TAG=$T/probe VARIANTS="plain:h4: tail:h3:--held-tail=64 tail:h4:--held-tail=64 held:h3:--held-cameras=1 held:h4:--held-cameras=1" bash tools/gpu_r4_held_probe2.sh || exit 1
TAG=$T/ab_held_grad MODE=gradient PREV=h3 ALT=h4 ABFLAGS="--held-cameras 1" bash tools/gpu_ab_alt.sh || exit 1
