#!/bin/bash
# One GPU session (run under gpurun from the repo root): the -m gpu tests of
# the working tree, then an A/B of two tuning builds of libcse
# (lib/prev/libcse_tuning.so = the previous commit, lib/libcse_tuning.so =
# the working tree), alternating processes on one box, for the given modes.
#   tools/gpu_ab_libs.sh TAG [MODES] [ROUNDS]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
TAG=${1:-ab}
MODES=${2:-jacobian,residual}
ROUNDS=${3:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.txt
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $OUT/pytest_gpu.txt | head -20; echo "pytest rc=$rc: stopping"; exit $rc; fi
PREV=ceres-solver-cuda_amd/lib/prev/libcse_tuning.so
for r in $(seq 1 $ROUNDS); do
  for m in ${MODES//,/ }; do
    for which in prev new; do
      lib=ceres-solver-cuda_amd/lib/libcse_tuning.so
      [ $which = prev ] && lib=$PREV
      timeout -k 10 200 python -u tools/ab_bench.py --lib $lib --variants 0 --rounds 2 --steps 20 \
        --mode $m > $OUT/ab_${m}_${which}_$r.txt 2>&1 || { echo "ab rc=$? ($m $which)"; tail -5 $OUT/ab_${m}_${which}_$r.txt; exit 1; }
      echo "$m $which r$r: $(grep median_ms $OUT/ab_${m}_${which}_$r.txt | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["summary"]["0"]["median_ms"])')"
    done
  done
done
exit 0
