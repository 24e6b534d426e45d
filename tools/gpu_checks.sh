# One GPU call's checks (run under gpurun from the repo root).  Edit per call.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
mkdir -p gpurun_out
set -o pipefail
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_spmv_gpu.py tests/test_gradient_gpu.py -m gpu > gpurun_out/pytest_spmv.log 2>&1 || { echo "spmv tests rc=$?"; tail -40 gpurun_out/pytest_spmv.log; exit 1; }
tail -2 gpurun_out/pytest_spmv.log
timeout -k 10 600 $T tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
OUT=gpurun_out/cgnr.txt
: > $OUT
for args in "--mode spmv" "--mode cgnr" "--mode spmv --format compressed_row" "--mode cgnr --format compressed_row"; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 --warmup 3 $args > gpurun_out/v.json 2> gpurun_out/v.err || { echo "bench rc=$? $args"; tail -5 gpurun_out/v.err; exit 1; }
  echo "[$args] $(grep '^{' gpurun_out/v.json | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print('kernel %.4f ms  %.0f GB/s  frac %.3f  ms/step %.4f' % (r['kernel_ms_avg'], r['achieved'], r['frac'], d['ms_per_step']))")" | tee -a $OUT
done
