# Interleaved bench.py runs of the operator modes over several builds of
# libcse.so (bench.py --lib): LIBS (names under lib/, "" = lib/libcse.so)
# and MODES from the environment.
LIBS=${LIBS:-"libcse.so cpo0/libcse.so"}
MODES=${MODES:-"schur cgnr"}
for r in 1 2 3; do for l in $LIBS; do for m in $MODES; do
  echo "$r $l $m $(timeout -k 10 120 python bench.py --lib ceres-solver-cuda_amd/lib/$l --mode $m --no-cpu-baseline --no-secondary --steps 50 --warmup 5 2>/dev/null | cut -c1-300)" || exit 1
done; done; done
