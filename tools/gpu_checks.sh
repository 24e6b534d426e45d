# One GPU call's checks (run under gpurun from the repo root).  Edit per call.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err; echo "bench rc=$?"; cat gpurun_out/bench_default.json
bash tools/gpu_profile.sh r03 > gpurun_out/profile_r03.log 2>&1; echo "profile rc=$?"; tail -30 gpurun_out/profile_r03.log
