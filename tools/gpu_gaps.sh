#!/bin/bash
# Kernel trace of small evaluations (launch overheads): problem-16
# (configs[1]) and rank 0's shard of an 8-way cut of problem-13682.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-gaps}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/p16 -o run --output-format csv -- python3 bench.py --config problem-16-22106 --loss trivial --no-secondary --no-cpu-baseline --steps 200 --warmup 20 > $OUT/p16.json 2> $OUT/p16.err || exit 1
python3 tools/gap_trace.py $OUT/p16 --last 400 > $OUT/p16_gaps.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/s8 -o run --output-format csv -- python3 bench.py --shard-of 8 --no-secondary --no-cpu-baseline --steps 50 --warmup 5 > $OUT/s8.json 2> $OUT/s8.err || exit 1
python3 tools/gap_trace.py $OUT/s8 --last 100 > $OUT/s8_gaps.txt
cat $OUT/p16_gaps.txt $OUT/s8_gaps.txt
python3 -c "import json; [print(f, json.load(open('$OUT/'+f))['ms_per_step'], json.load(open('$OUT/'+f))['roofline']['kernel_ms_avg']) for f in ('p16.json','s8.json')]"
