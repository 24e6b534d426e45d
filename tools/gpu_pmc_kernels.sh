#!/bin/bash
# Per-kernel PMC passes (FETCH_SIZE, WRITE_SIZE, L2 hits/misses) plus a
# kernel trace of one bench.py command (run under gpurun from the repo root).
#   BENCH_ARGS="--gradient --no-secondary ..." tools/gpu_pmc_kernels.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
TAG=${1:-pmc}
ARGS=${BENCH_ARGS:-"--no-cpu-baseline --no-secondary --steps 5 --warmup 1"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $OUT/trace.log; exit 1; }
i=0
for group in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $group -d $OUT/pmc$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc$i.log 2>&1 || { echo "pmc group $i rc=$?"; tail -3 $OUT/pmc$i.log; exit 1; }
done
find $OUT/trace -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
python3 tools/pmc_by_kernel.py $OUT/pmc1 $OUT/pmc2 $OUT/pmc3 $OUT/pmc4 $OUT/pmc5 > $OUT/pmc_by_kernel.txt
cat $OUT/pmc_by_kernel.txt
head -8 $OUT/kernel_stats.csv | cut -c1-200
