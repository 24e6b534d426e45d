#!/bin/bash
# Counters behind a kernel's floor: issue/wait split of the waves (SQ),
# L2 requests and hits (TCC), texture-addresser and -data busy (TA/TD) and
# the memory-side bytes, per kernel, for one bench.py command.
#   BENCH_ARGS="--mode residual ..." tools/gpu_pmc_floor.sh TAG
#   PROG="tools/general_path_probe.py --rounds 1" tools/gpu_pmc_floor.sh TAG  (another program)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-floor}
ARGS=${BENCH_ARGS:-"--mode residual --no-cpu-baseline --no-secondary --steps 5 --warmup 1"}
RUN=${PROG:-"bench.py $ARGS"}
export CSE_BAL_CACHE=/tmp/cse_bal_cache
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $RUN > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $OUT/trace.log; exit 1; }
i=0
for group in "FETCH_SIZE" "WRITE_SIZE" \
    "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum" \
    "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES" \
    "SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT" \
    "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_LOAD_WAVEFRONT_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $group -d $OUT/pmc$i -o run --output-format csv -- python3 $RUN > $OUT/pmc$i.log 2>&1 || { echo "pmc group $i ($group) rc=$?"; tail -3 $OUT/pmc$i.log; }
done
find $OUT/trace -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
python3 tools/pmc_by_kernel.py $OUT/pmc* > $OUT/pmc_by_kernel.txt
cut -c1-900 $OUT/pmc_by_kernel.txt
head -6 $OUT/kernel_stats.csv | cut -c1-160
