#!/bin/bash
# Round 4 final evidence on the shipped build: full GPU suite + bench +
# rocprof (final_checks.sh), the quaternion and held-camera configurations
# interleaved with the headline, configs[2], a kernel trace of configs[2].
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
TAG=${TAG:-r4final2} bash tools/final_checks.sh || exit 1
TAG=${TAG:-r4final2}/probe VARIANTS="plain:: held::--held-cameras=1" bash tools/gpu_r4_held_probe2.sh || exit 1
TAG=${TAG:-r4final2}/configs CONFIGS="--config problem-1778-993923 --loss huber --format compressed_row --warmup 300 --steps 300
--config problem-16-22106 --loss trivial --format block_sparse --warmup 2000 --steps 2000
--config problem-13682-4456117 --loss huber --format compressed_row
--camera quaternion
--held-cameras 1
--gradient" bash tools/run_configs.sh || exit 1
T=${TAG:-r4final2}
bash tools/gpu_pmc_kernels.sh $T/pmc > /dev/null || exit 1
python3 tools/pmc_traffic_json.py gpurun_out/$T/pmc/pmc1 gpurun_out/$T/pmc/pmc2 EvaluateAffineChunksTwoRoundW1 gpurun_out/$T/pmc_problem-13682-4456117_huber_block_sparse.json "round 4 final build (by-hand Snavely Jacobian, E-F-residual tail, 16 waves per CU), tools/gpu_r4_final2.sh" || exit 1
