# One GPU call's checks (run under gpurun from the repo root).  Edit per call.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
mkdir -p gpurun_out
set -o pipefail
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
CSE_VALUES_VARIANT=1 timeout -k 10 300 $T tests/test_parity_gpu.py -m gpu -k "residual_only or every_output or ragged or all_losses" > gpurun_out/pytest_values1.log 2>&1 || { echo "values1 tests rc=$?"; tail -30 gpurun_out/pytest_values1.log; exit 1; }
tail -2 gpurun_out/pytest_values1.log
OUT=gpurun_out/values.txt
: > $OUT
for mode in residual candidate; do
  for cfg in "0 16" "1 8" "1 16" "1 24" "1 32"; do
    set -- $cfg
    CSE_VALUES_VARIANT=$1 CSE_VALUES_WAVES=$2 timeout -k 10 240 python bench.py --no-cpu-baseline --mode $mode --steps 50 --warmup 5 > gpurun_out/v.json 2> gpurun_out/v.err || { echo "bench rc=$? $mode $cfg"; tail -5 gpurun_out/v.err; exit 1; }
    echo "$mode variant=$1 waves=$2 $(grep '^{' gpurun_out/v.json | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print('kernel %.4f ms  %.0f GB/s  frac %.3f  ms/step %.4f' % (r['kernel_ms_avg'], r['achieved'], r['frac'], d['ms_per_step']))")" | tee -a $OUT
  done
done
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench rc=$?"; exit 1; }
cat gpurun_out/bench_default.json
