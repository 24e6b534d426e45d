# A/B of lib/$PREV/libcse.so against lib/$ALT/libcse.so (default prev, alt: a
# build with one compile-time setting changed), alternating processes on one
# box: TAG=... MODE=... [PREV=... ALT=...] bash tools/gpu_ab_alt.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
OUT=gpurun_out/${TAG:-s3}; mkdir -p $OUT; L=ceres-solver-cuda_amd/lib
for r in 1 2 3; do for which in ${PREV:-prev} ${ALT:-alt}; do
  lib=$L/$which/libcse.so
  timeout -k 10 200 python -u tools/ab_bench.py --lib $lib --variants 0 --rounds 2 --steps 20 --mode $MODE ${ABFLAGS} > $OUT/ab_${MODE}_${which}_$r.txt 2>&1 || { echo "ab rc=$?"; tail -5 $OUT/ab_${MODE}_${which}_$r.txt; exit 1; }
  echo "$MODE $which r$r: $(tail -1 $OUT/ab_${MODE}_${which}_$r.txt | python -c 'import sys,json; d=json.loads(sys.stdin.read())["summary"]["0"]; print(round(d["median_ms"],4), "wall", round(d["median_wall_ms"],4))')"
done; done
