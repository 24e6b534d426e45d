#!/bin/bash
# Profile the evaluate kernel on the GPU box (run from the repo root under
# gpurun).  Kernel trace + stats in one run; every PMC group in its own run
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
TAG=${1:-r01}
ARGS=${BENCH_ARGS:-"--no-cpu-baseline --steps 10 --warmup 2"}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit 1
i=0
for group in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group -d $OUT/pmc$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc$i.log 2>&1 || echo "pmc group $i failed" >> $OUT/errors.txt
done
for d in $OUT/trace $OUT/pmc*; do
  [ -d "$d" ] && python3 tools/pmc_summary.py "$d" EvaluateAffine --json $OUT/summary.json > /dev/null
done
python3 tools/pmc_summary.py $OUT/trace EvaluateAffine > $OUT/trace_summary.json
cat $OUT/summary.json
