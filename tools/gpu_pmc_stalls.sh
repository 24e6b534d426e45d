#!/bin/bash
# Texture-pipe stall counters (TA/TD/TCP) per kernel for one bench.py
# command: is the vector-memory path saturated or waiting on L2?
#   BENCH_ARGS="--mode residual ..." tools/gpu_pmc_stalls.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-stalls}
ARGS=${BENCH_ARGS:-"--mode residual --no-cpu-baseline --no-secondary --steps 5 --warmup 1"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for group in \
    "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
    "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum TCP_GATE_EN1_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $group -d $OUT/pmc$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc$i.log 2>&1 || { echo "pmc group $i ($group) rc=$?"; tail -3 $OUT/pmc$i.log; }
done
python3 tools/pmc_by_kernel.py $OUT/pmc* > $OUT/pmc_by_kernel.txt
grep -E "EvaluateAffine|Schur|Cgnr|CameraGrad|GradientContrib" $OUT/pmc_by_kernel.txt | cut -c1-1200
