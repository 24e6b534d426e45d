#!/bin/bash
# The Snavely Jacobian by hand (lib/bh = product) against the seeded Jets
# (lib/jet), and by hand with the F cells staged in half-wave rounds (lib/fh,
# 5 waves per SIMD): the full GPU suite on the product build, then A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
T=${TAG:-r4s6}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo "pytest rc=$?"; tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
timeout -k 10 300 python -u tools/pers_check.py --lib ceres-solver-cuda_amd/lib/bh/libcse.so --out $OUT/check_bh.json > $OUT/check_bh.txt 2>&1 || { echo "check rc=$?"; tail -5 $OUT/check_bh.txt; exit 1; }
timeout -k 10 300 python -u tools/pers_check.py --lib ceres-solver-cuda_amd/lib/fh/libcse.so --out $OUT/check_fh.json > $OUT/check_fh.txt 2>&1 || { echo "check rc=$?"; tail -5 $OUT/check_fh.txt; exit 1; }
python tools/pers_check.py --compare $OUT/check_bh.json $OUT/check_fh.json | tee $OUT/compare_bh_fh.txt
TAG=$T/ab_jac MODE=jacobian PREV=jet ALT=bh bash tools/gpu_ab_alt.sh || exit 1
TAG=$T/ab_jac_fh MODE=jacobian PREV=bh ALT=fh bash tools/gpu_ab_alt.sh || exit 1
TAG=$T/ab_grad MODE=gradient PREV=jet ALT=fh bash tools/gpu_ab_alt.sh || exit 1
TAG=$T/ab_crs MODE=jacobian PREV=jet ALT=fh ABFLAGS="--format compressed_row" bash tools/gpu_ab_alt.sh || exit 1
