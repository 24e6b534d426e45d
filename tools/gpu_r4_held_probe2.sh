#!/bin/bash
# Held-camera kernel: chunk-bound loads sunk next to the gather (lib/h3)
# against lib/h2, held camera 0 and held tail, with the unheld control.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
OUT=gpurun_out/${TAG:-r4hp2}; mkdir -p $OUT
L=ceres-solver-cuda_amd/lib
for r in 1 2 3; do
  for v in ${VARIANTS:-plain:h3: held:h2:--held-cameras=1 held:h3:--held-cameras=1 tail:h3:--held-tail=64}; do
    IFS=: read name lib flag <<< "$v"
    timeout -k 10 200 python -u tools/ab_bench.py --lib $L/$lib/libcse.so --variants 0 --rounds 2 --steps 20 ${flag/=/ } > $OUT/${name}_${lib}_$r.txt 2>&1 || { echo "$v rc=$?"; tail -5 $OUT/${name}_${lib}_$r.txt; exit 1; }
    echo "$name $lib r$r: $(tail -1 $OUT/${name}_${lib}_$r.txt | python -c 'import sys,json; d=json.loads(sys.stdin.read())["summary"]["0"]; print(round(d["median_ms"],4), "wall", round(d["median_wall_ms"],4))')"
  done
done
