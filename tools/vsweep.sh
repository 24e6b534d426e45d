#!/bin/bash
# Bench-only variant sweep of the hot kernel (run under gpurun from the repo
# root): VARIANTS="0 49 50" bash tools/vsweep.sh TAG.  Stops at the first
# bench that crashes or times out.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
OUT=gpurun_out/vsweep_${1:-x}
mkdir -p $OUT
for v in ${VARIANTS:-0}; do
  export CSE_AFFINE_VARIANT=$v
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps ${STEPS:-30} --warmup 3 ${BENCH_ARGS:-} > $OUT/bench_v$v.log 2>&1
  brc=$?
  line=$(grep '^{' $OUT/bench_v$v.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print('%.4f ms  %.0f GB/s  frac %.3f  value %.1f' % (r['kernel_ms_avg'], r['achieved'], r['frac'], d['value']))" 2>/dev/null)
  echo "v$v rc=$brc $line" | tee -a $OUT/sweep.txt
  if [ $brc -ne 0 ]; then echo "stopping: bench rc $brc" >> $OUT/sweep.txt; exit 1; fi
done
