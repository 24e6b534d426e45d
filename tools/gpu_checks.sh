# One GPU call's checks (run under gpurun from the repo root).  Edit per call.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
mkdir -p gpurun_out
set -o pipefail
PYTHONPATH=ceres-solver-cuda_amd timeout -k 10 300 python -u -m ceres_amd.bundle_adjuster --synthetic problem-13682-4456117 --robustify --point_sigma 0.01 --num_iterations 5 > gpurun_out/ba_13682.txt 2>&1 || { echo "ba rc=$?"; tail -20 gpurun_out/ba_13682.txt; exit 1; }
tail -22 gpurun_out/ba_13682.txt
for sc in weak strong; do
  CSE_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --scaling $sc --gradient > gpurun_out/dist_$sc.json 2> gpurun_out/dist_$sc.err || { echo "dist $sc rc=$?"; tail -20 gpurun_out/dist_$sc.err; exit 1; }
  grep '^{' gpurun_out/dist_$sc.json | cut -c1-400
done
