#!/bin/bash
# Gradient path check (run under gpurun from the repo root): the gradient
# parity tests, the full-size 13682 parity test (fused gradient), the
# gradient-inclusive bench line in modes 0 and 3, and a rocprofv3 kernel
# summary of the mode-0 gradient evaluation.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
OUT=gpurun_out/${1:-grad}
mkdir -p $OUT
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gradient_gpu.py tests/test_multirank_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_grad.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest_grad.txt; exit 1; }
tail -2 $OUT/pytest_grad.txt
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -k 13682 -x -q -s --timeout 240 --timeout-method thread > $OUT/pytest_13682.txt 2>&1 || { echo "pytest13682 rc=$?"; tail -30 $OUT/pytest_13682.txt; exit 1; }
tail -2 $OUT/pytest_13682.txt
for m in 0 3; do
  timeout -k 10 300 python bench.py --gradient --gradient-mode $m --no-cpu-baseline --no-secondary --steps 30 > $OUT/bench_grad_m$m.json 2> $OUT/bench_grad_m$m.err || { echo "bench rc=$?"; tail -20 $OUT/bench_grad_m$m.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_grad_m$m.json')); print('mode $m', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --gradient --no-cpu-baseline --no-secondary --steps 30 --warmup 3 > $OUT/bench_under_rocprof.json 2> $OUT/trace.err || { echo "rocprof rc=$?"; tail -20 $OUT/trace.err; exit 1; }
find $OUT/trace -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
head -8 $OUT/kernel_stats.csv | cut -c1-200
