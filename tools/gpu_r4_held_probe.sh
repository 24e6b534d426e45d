#!/bin/bash
# Round 4: where the held-camera kernel's extra time comes from.  Same
# library, interleaved processes: every camera active; one held camera
# observed only by the last 64 blocks (the held-camera kernel on an aligned
# layout); camera 0 held (every later chunk shifted).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
OUT=gpurun_out/${TAG:-r4hp}; mkdir -p $OUT
LIB=${LIB:-ceres-solver-cuda_amd/lib/libcse.so}
for r in 1 2 3; do
  for v in plain tail held; do
    case $v in plain) F="";; tail) F="--held-tail 64";; held) F="--held-cameras 1";; esac
    timeout -k 10 200 python -u tools/ab_bench.py --lib $LIB --variants 0 --rounds 2 --steps 20 $F > $OUT/${v}_$r.txt 2>&1 || { echo "$v rc=$?"; tail -5 $OUT/${v}_$r.txt; exit 1; }
    echo "$v r$r: $(tail -1 $OUT/${v}_$r.txt | python -c 'import sys,json; d=json.loads(sys.stdin.read())["summary"]["0"]; print(round(d["median_ms"],4), "wall", round(d["median_wall_ms"],4))')"
  done
done
