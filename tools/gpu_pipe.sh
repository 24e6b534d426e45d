#!/bin/bash
# Pipelined-kernel session: bit-equality on assorted shapes, then a same-box
# A/B of the hot kernel (variant 0 = shipped) on problem-13682.
#   tools/gpu_pipe.sh TAG VARIANTS
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-pipe}
VARS=${2:-40,41,42}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u tools/pipe_check.py --variants $VARS > $OUT/check.txt 2>&1
rc=$?; tail -3 $OUT/check.txt; [ $rc -eq 0 ] || { echo "check rc=$rc"; exit 1; }
timeout -k 10 400 python -u tools/ab_bench.py --variants 0,$VARS --rounds 3 --steps 20 > $OUT/ab.txt 2>&1
rc=$?; grep -E "variant|summary" $OUT/ab.txt | tail -20; [ $rc -eq 0 ] || { echo "ab rc=$rc"; exit 1; }
