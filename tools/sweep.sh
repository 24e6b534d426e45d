#!/bin/bash
# Variant sweep of the hot kernel (run under gpurun from the repo root).
# Each variant: a parity subset (small BAL, BSM) and a short bench; the
# kernel's average time and achieved GB/s are collected in sweep.txt.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
OUT=gpurun_out/sweep_${1:-r01}
mkdir -p $OUT
VARIANTS=${VARIANTS:-"0 1 2 3 4 5 6 7 8 9"}
for v in $VARIANTS; do
  for wg in ${WGS:-"-1"}; do
    tag="v${v}_wg${wg}"
    if [ "$wg" = "-1" ]; then unset CSE_WG_PER_CU; else export CSE_WG_PER_CU=$wg; fi
    export CSE_AFFINE_VARIANT=$v
    timeout -k 10 300 python -m pytest tests/test_parity_gpu.py -q -x -k "bal_small and block_sparse" > $OUT/parity_$tag.log 2>&1
    prc=$?
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --warmup 3 > $OUT/bench_$tag.log 2>&1
    brc=$?
    line=$(grep '^{' $OUT/bench_$tag.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print('%.4f ms  %.0f GB/s  frac %.3f  value %.1f' % (r['kernel_ms_avg'], r['achieved'], r['frac'], d['value']))" 2>/dev/null)
    echo "$tag parity_rc=$prc bench_rc=$brc $line" | tee -a $OUT/sweep.txt
    if [ $brc -ne 0 ] && [ $brc -ne 1 ]; then echo "stopping: bench rc $brc" >> $OUT/sweep.txt; exit 1; fi
  done
done
