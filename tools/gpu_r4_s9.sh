#!/bin/bash
# Round 4, shipped build: per-kernel PMC of the headline (HBM traffic JSON
# for bench.py's roofline.traffic), the other configurations, a kernel
# trace of configs[2].
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
T=${TAG:-r4s9}; OUT=gpurun_out/$T; mkdir -p $OUT
bash tools/gpu_pmc_kernels.sh $T/pmc > /dev/null || exit 1
python3 tools/pmc_traffic_json.py gpurun_out/$T/pmc/pmc1 gpurun_out/$T/pmc/pmc2 EvaluateAffineChunksTwoRoundW1 gpurun_out/$T/pmc_problem-13682-4456117_huber_block_sparse.json "round 4 shipped build (by-hand Snavely Jacobian, 12 waves per CU), tools/gpu_r4_s9.sh" || exit 1
cat gpurun_out/$T/pmc_problem-13682-4456117_huber_block_sparse.json
TAG=$T/configs CONFIGS="--config problem-16-22106 --loss trivial --format block_sparse --warmup 2000 --steps 2000
--config problem-1778-993923 --loss huber --format compressed_row --warmup 300 --steps 300
--config problem-1778-993923 --loss huber --format block_sparse --warmup 300 --steps 300
--config problem-13682-4456117 --loss huber --format compressed_row
--loss trivial
--loss cauchy
--held-cameras 1
--camera quaternion
--gradient
--mode residual" bash tools/run_configs.sh || exit 1
