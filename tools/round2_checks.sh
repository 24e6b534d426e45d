#!/bin/bash
# GPU tests, a 13682-scale driver run and an SpMV profile (run under gpurun).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python ceres-solver-cuda_amd/ceres_amd/bundle_adjuster.py --synthetic problem-13682-4456117 \
  --robustify --point_sigma 0.05 --num_iterations 3 --max_linear_solver_iterations 50 > gpurun_out/ba13682.txt 2>&1
tail -12 gpurun_out/ba13682.txt
mkdir -p gpurun_out/rps
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rps -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 --mode spmv > /dev/null 2>&1
