#!/bin/bash
# Round-end checks (run under gpurun from the repo root): GPU tests, the
# default bench line, and a rocprofv3 kernel-trace summary of the same bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
OUT=gpurun_out/${TAG:-final}
mkdir -p $OUT
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=15 --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo "pytest rc=$?"; tail -20 $OUT/pytest_gpu.txt; exit 1; }
tail -2 $OUT/pytest_gpu.txt
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 30 --warmup 3 > $OUT/bench_under_rocprof.json 2> $OUT/trace.err || { echo "rocprof rc=$?"; tail -20 $OUT/trace.err; exit 1; }
find $OUT/trace -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
head -6 $OUT/kernel_stats.csv
