#!/bin/bash
# One GPU session (run under gpurun from the repo root): optionally the slow
# (full-size) GPU tests, then in-process A/B runs of tuning variants per mode.
#   tools/gpu_variants.sh TAG SLOW(0|1) MODE:VARIANTS [MODE:VARIANTS ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
TAG=$1; SLOW=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$SLOW" = 1 ]; then
  timeout -k 10 500 python -u -m pytest tests -m "gpu and slow" -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest_slow.txt 2>&1
  rc=$?
  tail -3 $OUT/pytest_slow.txt
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|max_rel" $OUT/pytest_slow.txt | head -20; echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
for mv in "$@"; do
  m=${mv%%:*}; v=${mv#*:}
  timeout -k 10 400 python -u tools/ab_bench.py --variants $v --rounds 3 --steps 20 --mode $m \
    --out $OUT/ab_$m.json > $OUT/ab_$m.txt 2>&1 || { echo "ab rc=$? ($m)"; tail -5 $OUT/ab_$m.txt; exit 1; }
  grep -E "^# variant|summary" $OUT/ab_$m.txt
done
exit 0
