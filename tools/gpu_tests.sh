#!/bin/bash
# Run a selection of GPU tests under a time limit.
#   tools/gpu_tests.sh TAG TIMEOUT pytest-args...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; TO=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 $TO python -u -m pytest "$@" -x -v -s --timeout 900 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|parity:" $OUT/pytest.txt | tail -40
exit $rc
