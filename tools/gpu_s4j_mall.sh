cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
OUT=gpurun_out/s4j; mkdir -p $OUT
for n in 16 8; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/t$n -o run --output-format csv -- python3 bench.py --shard-of $n --gradient --no-secondary --no-cpu-baseline --steps 10 --warmup 2 > $OUT/b$n.json 2> $OUT/b$n.err || { echo "rc=$?"; tail -5 $OUT/b$n.err; exit 1; }
find $OUT/t$n -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_$n.csv \;
head -5 $OUT/kernel_stats_$n.csv | cut -c1-150
done
