#!/bin/bash
# Bench lines for the other BASELINE.json configs, layouts, losses and the
# gradient (run under gpurun from the repo root).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export CSE_BAL_CACHE=/tmp/cse_bal_cache
OUT=gpurun_out/${TAG:-configs}.txt
: > $OUT
while read -r args; do
  [ -z "$args" ] && continue
  echo "== $args" >> $OUT
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary $args > gpurun_out/cfg.json 2>gpurun_out/cfg.err || { echo "rc=$?" >> $OUT; tail -3 gpurun_out/cfg.err >> $OUT; cat $OUT; exit 1; }
  grep '^{' gpurun_out/cfg.json | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); r=d['roofline']; print('%.1f %s  kernel %.4f ms  %.0f GB/s  frac %.3f  ms/step %.4f' % (d['value'], d['unit'], r['kernel_ms_avg'], r['achieved'], r['frac'], d['ms_per_step']))" >> $OUT
done <<LIST
${CONFIGS:---config problem-16-22106 --loss trivial --format block_sparse
--config problem-1778-993923 --loss huber --format compressed_row
--config problem-1778-993923 --loss huber --format block_sparse
--config problem-13682-4456117 --loss huber --format compressed_row
--gradient
--loss trivial
--loss cauchy}
LIST
cat $OUT
