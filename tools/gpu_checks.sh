# One GPU call's checks (run under gpurun from the repo root).  Edit per call.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
mkdir -p gpurun_out
for v in 57 58; do
  CSE_AFFINE_VARIANT=$v timeout -k 10 120 python tools/debug_variant.py > gpurun_out/debug_v$v.txt 2>&1; rc=$?; echo "debug v$v rc=$rc"; cat gpurun_out/debug_v$v.txt
  [ $rc -ne 0 ] && exit 1
done
CSE_STREAM_WAVES=8 VARIANTS="0 57 58" bash tools/vsweep.sh st8b || exit 1
CSE_STREAM_WAVES=6 VARIANTS="58" bash tools/vsweep.sh st6b || exit 1
