#!/bin/bash
# Round 4 final evidence on the shipped build: full GPU suite + bench +
# rocprof (final_checks.sh), the quaternion and held-camera configurations
# interleaved with the headline, configs[2], a kernel trace of configs[2].
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
TAG=r4final2 bash tools/final_checks.sh || exit 1
TAG=r4final2/probe VARIANTS="plain:: held::--held-cameras=1" bash tools/gpu_r4_held_probe2.sh || exit 1
TAG=r4final2/configs CONFIGS="--config problem-1778-993923 --loss huber --format compressed_row --warmup 300 --steps 300
--camera quaternion
--held-cameras 1" bash tools/run_configs.sh || exit 1
