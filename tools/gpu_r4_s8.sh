#!/bin/bash
# The shipped build (by-hand Snavely Jacobian, BSM capped at 12 waves per CU):
# full GPU suite, bit-equality over pers_check's cases against lib/b12, the
# held-camera cap A/B (lib/hc12 vs ship), and the bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
T=${TAG:-r4s8}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
TAG=$T/probe VARIANTS="plain:jet: plain:ship: held:ship:--held-cameras=1 held:hc12:--held-cameras=1" bash tools/gpu_r4_held_probe2.sh || exit 1
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -5 $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
