#!/bin/bash
# Round 4 evidence: full GPU suite + bench + rocprof (final_checks.sh), the
# other configurations, a kernel trace of configs[2], and the cost of the
# evaluator's timing events.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
N=${N:-1}
TAG=r4final$N bash tools/final_checks.sh || exit 1
TAG=r4configs$N CONFIGS="--config problem-16-22106 --loss trivial --format block_sparse --warmup 2000 --steps 2000
--config problem-1778-993923 --loss huber --format compressed_row --warmup 300 --steps 300
--config problem-1778-993923 --loss huber --format block_sparse --warmup 300 --steps 300
--config problem-13682-4456117 --loss huber --format compressed_row
--held-cameras 1
--gradient" bash tools/run_configs.sh || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4trace1778_$N -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary --config problem-1778-993923 --format compressed_row --steps 20 > gpurun_out/r4trace1778_$N.txt 2>&1 || exit 1
for c in "--config problem-1778-993923 --format compressed_row" "--config problem-13682-4456117"; do
  timeout -k 10 200 python -u tools/profile_overhead.py $c || exit 1
done
