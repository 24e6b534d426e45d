#!/bin/bash
# A/B of several product builds (run under gpurun from the repo root):
# lib/libcse.so and lib/alt<k>/libcse.so, alternating processes on one box.
#   tools/gpu_ab_multi.sh TAG MODES ROUNDS ALT1 [ALT2 ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
TAG=$1; MODES=$2; ROUNDS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
L=ceres-solver-cuda_amd/lib
for r in $(seq 1 $ROUNDS); do
  for m in ${MODES//,/ }; do
    for which in base "$@"; do
      lib=$L/libcse.so
      [ $which != base ] && lib=$L/$which/libcse.so
      timeout -k 10 200 python -u tools/ab_bench.py --lib $lib --variants 0 --rounds 2 --steps 20 \
        --mode $m $AB_ARGS > $OUT/ab_${m}_${which}_$r.txt 2>&1 || { echo "ab rc=$? ($m $which)"; tail -5 $OUT/ab_${m}_${which}_$r.txt; exit 1; }
      echo "$m $which r$r: $(tail -1 $OUT/ab_${m}_${which}_$r.txt | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["summary"]["0"]["median_ms"], "wall", d["summary"]["0"]["median_wall_ms"])')"
    done
  done
done
