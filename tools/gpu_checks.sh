# One GPU call's checks (run under gpurun from the repo root).  Edit per call.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
mkdir -p gpurun_out
set -o pipefail
VARIANTS="0 60 45 46 0 60 45 46" bash tools/vsweep.sh s5
