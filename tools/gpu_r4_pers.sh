#!/bin/bash
# Round 4: the persistent software-pipelined BSM Jacobian kernel -- outputs
# bit-equal to the one-chunk-per-wave kernel over tools/pers_check.py's edge
# cases (lib/base vs lib/pers, CSE_PERSISTENT=1), then the same-box A/B of
# the problem-13682 Jacobian evaluation.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
T=${TAG:-r4p}
OUT=gpurun_out/$T; mkdir -p $OUT
L=ceres-solver-cuda_amd/lib
for w in ${PREV:-base} ${ALT:-pers}; do
  timeout -k 10 300 python -u tools/pers_check.py --lib $L/$w/libcse.so --out $OUT/check_$w.json \
    > $OUT/check_$w.txt 2>&1 || { echo "check $w rc=$?"; tail -20 $OUT/check_$w.txt; exit 1; }
done
python tools/pers_check.py --compare $OUT/check_${PREV:-base}.json $OUT/check_${ALT:-pers}.json | tee $OUT/compare.txt
TAG=$T/ab MODE=jacobian PREV=${PREV:-base} ALT=${ALT:-pers} bash tools/gpu_ab_alt.sh || exit 1
