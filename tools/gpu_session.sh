#!/bin/bash
# One GPU session (run under gpurun from the repo root): the -m gpu tests,
# then optional A/B timing of tuning variants.  Usage:
#   tools/gpu_session.sh TAG [VARIANTS]
# Stops at the first GPU fault / abort / timeout (exit codes other than the
# test runner's 0/1).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
TAG=${1:-s}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
grep -E "FAILED|Error" $OUT/pytest_gpu.txt | head -20
if [ -n "$2" ]; then
  timeout -k 10 600 python -u tools/ab_bench.py --variants "$2" --rounds 3 --steps 20 --out $OUT/ab.json > $OUT/ab.txt 2>&1
  rc2=$?
  tail -12 $OUT/ab.txt
  [ $rc2 -ne 0 ] && { echo "ab rc=$rc2"; exit $rc2; }
fi
exit $rc
