#!/bin/bash
# bench.py --mode M of lib/prev/libcse.so against lib/$ALT/libcse.so,
# alternating processes on one box (run under gpurun from the repo root):
#   TAG=... ALT=alt2 MODES=schur,cgnr bash tools/gpu_ab_modes.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
OUT=gpurun_out/${TAG:-abm}; mkdir -p $OUT; L=ceres-solver-cuda_amd/lib
for r in 1 2; do for m in ${MODES//,/ }; do for which in prev ${ALT:-alt}; do
  timeout -k 10 200 python -u bench.py --lib $L/$which/libcse.so --mode $m --no-secondary --no-cpu-baseline \
    --steps 30 --warmup 3 > $OUT/${m}_${which}_$r.json 2> $OUT/${m}_${which}_$r.err || { echo "bench rc=$? ($m $which)"; tail -5 $OUT/${m}_${which}_$r.err; exit 1; }
  echo "$m $which r$r: $(python -c "import json; d=json.load(open('$OUT/${m}_${which}_$r.json')); print(round(d['ms_per_step'],4), 'ms')")"
done; done; done
