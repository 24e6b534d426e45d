#!/bin/bash
# One parameterised GPU runner (under gpurun, from the repo root): a list of
# steps, each one quoted argument "<kind> <args...>", run in order; the first
# failing step ends the run.  Output under gpurun_out/$TAG/.
#
#   TAG=r5a bash tools/gpu_run.sh \
#     "tests tests/test_parity_gpu.py -k full_size" \
#     "suite" \
#     "bench" "bench --gradient --no-secondary" \
#     "rocprof --no-cpu-baseline --steps 30 --warmup 3" \
#     "rocprof-tests tests/test_parity_gpu.py -m slow" \
#     "ab 3 jacobian plain:: jet::--jacobian-form=jet" \
#     "configs" "pmc" "membench"
#
# Kinds:
#   suite                 the whole -m gpu suite (the driver's GPUTEST command)
#   tests ARGS            pytest ARGS (-v -s, per-test timeout 900 s)
#   bench ARGS            python bench.py ARGS -> bench_<n>.json
#   rocprof ARGS          the same under rocprofv3 --kernel-trace --stats
#   rocprof-tests ARGS    pytest ARGS under rocprofv3 --kernel-trace --stats
#   ab ROUNDS MODE LIB:FLAGS ...
#                         tools/ab_bench.py, interleaved processes: LIB is a
#                         directory under ceres-solver-cuda_amd/lib (empty =
#                         lib/libcse.so), FLAGS extra ab_bench flags with '='
#                         between flag and value and ',' between flags
#   configs [LIST]        tools/run_configs.sh (LIST: newline-separated args)
#   pmc [BENCH_ARGS]      per-kernel PMC passes (tools/gpu_pmc_kernels.sh); with
#                         no BENCH_ARGS (the headline) also its HBM traffic JSON
#   cmd ...               any other command, under a 600 s limit
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
TAG=${TAG:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
L=ceres-solver-cuda_amd/lib
n=0

summ() {  # the ab_bench summary line of one file
  tail -1 "$1" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read())["summary"]; print(" ".join("%s=%.4f(wall %.4f)" % (k, v["median_ms"], v["median_wall_ms"]) for k, v in d.items()))'
}

for step in "$@"; do
  n=$((n+1))
  read -r kind args <<< "$step"
  echo "== [$n] $kind $args"
  case $kind in
    suite)
      timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --durations=15 --timeout 900 \
        --timeout-method thread > $OUT/pytest_gpu_$n.txt 2>&1 || { echo "suite rc=$?"; tail -30 $OUT/pytest_gpu_$n.txt; exit 1; }
      tail -3 $OUT/pytest_gpu_$n.txt ;;
    tests)
      timeout -k 10 ${TEST_TIMEOUT:-1100} python -u -m pytest $args -x -v -s --timeout 900 \
        --timeout-method thread > $OUT/pytest_$n.txt 2>&1 || { echo "tests rc=$?"; tail -40 $OUT/pytest_$n.txt; exit 1; }
      grep -E "PASSED|FAILED|ERROR|passed|failed|parity" $OUT/pytest_$n.txt | tail -40 ;;
    bench)
      timeout -k 10 400 python bench.py $args > $OUT/bench_$n.json 2> $OUT/bench_$n.err || { echo "bench rc=$?"; tail -20 $OUT/bench_$n.err; exit 1; }
      cut -c1-400 $OUT/bench_$n.json ;;
    rocprof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace_$n -o run --output-format csv \
        -- python3 bench.py $args > $OUT/rocprof_bench_$n.json 2> $OUT/rocprof_$n.err || { echo "rocprof rc=$?"; tail -20 $OUT/rocprof_$n.err; exit 1; }
      find $OUT/trace_$n -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_$n.csv \;
      head -8 $OUT/kernel_stats_$n.csv | cut -c1-220 ;;
    rocprof-tests)
      timeout -k 10 ${TEST_TIMEOUT:-1100} rocprofv3 --kernel-trace --stats -d $OUT/trace_$n -o run --output-format csv \
        -- python3 -u -m pytest $args -x -v -s --timeout 900 --timeout-method thread > $OUT/pytest_$n.txt 2>&1 || { echo "rocprof-tests rc=$?"; tail -40 $OUT/pytest_$n.txt; exit 1; }
      grep -E "PASSED|FAILED|ERROR|passed|failed|parity" $OUT/pytest_$n.txt | tail -40
      find $OUT/trace_$n -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_$n.csv \;
      find $OUT/trace_$n -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace_$n.csv \;
      head -12 $OUT/kernel_stats_$n.csv | cut -c1-220 ;;
    ab)
      read -r rounds mode libs <<< "$args"
      for r in $(seq 1 $rounds); do
        for v in $libs; do
          IFS=: read name lib flags <<< "$v"
          lp=$L/libcse.so; [ -n "$lib" ] && lp=$L/$lib/libcse.so
          f=$OUT/ab_${n}_${name}_$r.txt
          fl=${flags//=/ }
          timeout -k 10 300 python -u tools/ab_bench.py --lib $lp --variants 0 --rounds 2 --steps 20 \
            --mode $mode ${fl//,/ } > $f 2>&1 || { echo "ab $v rc=$?"; tail -5 $f; exit 1; }
          echo "$name r$r: $(summ $f)"
        done
      done ;;
    configs)
      if [ -n "$args" ]; then CONFIGS="$args" TAG=$TAG/configs_$n bash tools/run_configs.sh || exit 1
      else TAG=$TAG/configs_$n bash tools/run_configs.sh || exit 1; fi ;;
    pmc)
      BENCH_ARGS=${args:-"--no-cpu-baseline --no-secondary --steps 5 --warmup 1"} \
        bash tools/gpu_pmc_kernels.sh $TAG/pmc_$n > /dev/null || exit 1
      cat $OUT/pmc_$n/pmc_by_kernel.txt | head -40
      if [ -z "$args" ]; then  # the headline: its HBM traffic JSON for bench.py
        python3 tools/pmc_traffic_json.py $OUT/pmc_$n/pmc1 $OUT/pmc_$n/pmc2 EvaluateAffineChunksGroupStore \
          $OUT/pmc_problem-13682-4456117_huber_block_sparse.json "tools/gpu_run.sh pmc, $TAG" || exit 1
      fi ;;
    cmd)
      timeout -k 10 600 bash -c "$args" > $OUT/cmd_$n.txt 2>&1 || { echo "cmd rc=$?"; tail -20 $OUT/cmd_$n.txt; exit 1; }
      tail -30 $OUT/cmd_$n.txt ;;
    *) echo "unknown step kind: $kind"; exit 2 ;;
  esac
done
