#!/bin/bash
# A/B of two product builds (run under gpurun from the repo root):
# lib/libcse.so (the working tree's default) against lib/alt/libcse.so (the
# same source with a compile-time setting changed), alternating processes on
# one box; then the alternative build replaces the default for the gradient
# parity tests and the full-size 13682 test.
#   tools/gpu_ab_product.sh TAG [MODES] [ROUNDS]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
TAG=${1:-abp}
MODES=${2:-gradient}
ROUNDS=${3:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
L=ceres-solver-cuda_amd/lib
for r in $(seq 1 $ROUNDS); do
  for m in ${MODES//,/ }; do
    for which in base alt; do
      lib=$L/libcse.so
      [ $which = alt ] && lib=$L/alt/libcse.so
      timeout -k 10 200 python -u tools/ab_bench.py --lib $lib --variants 0 --rounds 2 --steps 20 \
        --mode $m > $OUT/ab_${m}_${which}_$r.txt 2>&1 || { echo "ab rc=$? ($m $which)"; tail -5 $OUT/ab_${m}_${which}_$r.txt; exit 1; }
      echo "$m $which r$r: $(tail -1 $OUT/ab_${m}_${which}_$r.txt | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["summary"]["0"]["median_ms"])')"
    done
  done
done
cp $L/alt/libcse.so $L/libcse.so
timeout -k 10 300 python -u -m pytest tests/test_gradient_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_grad_alt.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest_grad_alt.txt; exit 1; }
tail -1 $OUT/pytest_grad_alt.txt
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -k 13682 -x -q -s --timeout 240 --timeout-method thread > $OUT/pytest_13682_alt.txt 2>&1 || { echo "pytest13682 rc=$?"; tail -30 $OUT/pytest_13682_alt.txt; exit 1; }
tail -1 $OUT/pytest_13682_alt.txt
