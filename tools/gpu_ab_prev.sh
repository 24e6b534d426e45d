#!/bin/bash
# One GPU session (run under gpurun from the repo root): the fast -m gpu
# tests of the working tree, the small-evaluation overhead probe, then an A/B
# of two product builds, lib/prev/libcse.so (a previous commit) against
# lib/libcse.so (the working tree), alternating processes on one box.
#   tools/gpu_ab_prev.sh TAG [MODES] [ROUNDS] [PROBE_FLAGS]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
TAG=${1:-abprev}
MODES=${2:-jacobian,residual}
ROUNDS=${3:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
L=ceres-solver-cuda_amd/lib
timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.txt
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $OUT/pytest_gpu.txt | head -20; echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u tools/overhead_probe.py > $OUT/probe_new.txt 2>&1 || { echo "probe rc=$?"; tail -5 $OUT/probe_new.txt; exit 1; }
grep "round 2" $OUT/probe_new.txt
timeout -k 10 300 python -u tools/overhead_probe.py --flags 1 > $OUT/probe_new_same_point.txt 2>&1 || { echo "probe rc=$?"; tail -5 $OUT/probe_new_same_point.txt; exit 1; }
grep "round 2" $OUT/probe_new_same_point.txt
for r in $(seq 1 $ROUNDS); do
  for m in ${MODES//,/ }; do
    for which in prev new; do
      lib=$L/libcse.so
      [ $which = prev ] && lib=$L/prev/libcse.so
      timeout -k 10 200 python -u tools/ab_bench.py --lib $lib --variants 0 --rounds 2 --steps 20 \
        --mode $m > $OUT/ab_${m}_${which}_$r.txt 2>&1 || { echo "ab rc=$? ($m $which)"; tail -5 $OUT/ab_${m}_${which}_$r.txt; exit 1; }
      echo "$m $which r$r: $(tail -1 $OUT/ab_${m}_${which}_$r.txt | python -c 'import sys,json; d=json.loads(sys.stdin.read())["summary"]["0"]; print(round(d["median_ms"],4), "wall", round(d["median_wall_ms"],4))')"
    done
  done
done
exit 0
