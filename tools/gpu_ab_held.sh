#!/bin/bash
# A/B of lib/prev/libcse.so (before) and lib/libcse.so (after) on the
# held-camera problem (tools/ab_bench.py --held-cameras), alternating
# processes on one box.   tools/gpu_ab_held.sh TAG [HELD] [ROUNDS]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-abheld}; HELD=${2:-1}; ROUNDS=${3:-3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for which in prev new; do
    lib=ceres-solver-cuda_amd/lib/libcse.so
    [ $which = prev ] && lib=ceres-solver-cuda_amd/lib/prev/libcse.so
    timeout -k 10 200 python -u tools/ab_bench.py --lib $lib --variants 0 --rounds 2 --steps 20 \
      --mode jacobian --held-cameras $HELD > $OUT/ab_${which}_$r.txt 2>&1 || { echo "ab rc=$? ($which)"; tail -5 $OUT/ab_${which}_$r.txt; exit 1; }
    echo "$which r$r: $(grep median_ms $OUT/ab_${which}_$r.txt | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["summary"]["0"]["median_ms"])')"
  done
done
