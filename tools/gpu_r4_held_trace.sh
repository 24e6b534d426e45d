set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
OUT=gpurun_out/r4ht; mkdir -p $OUT
for v in plain tail; do
  case $v in plain) F="";; tail) F="--held-tail 64";; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --stats -d $OUT/$v -o run --output-format csv -- python3 tools/ab_bench.py --lib ceres-solver-cuda_amd/lib/libcse.so --variants 0 --rounds 1 --steps 10 $F > $OUT/$v.txt 2>&1 || { echo "$v rc=$?"; tail -5 $OUT/$v.txt; exit 1; }
  grep "round 0" $OUT/$v.txt
done
