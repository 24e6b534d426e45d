#!/bin/bash
# One gpurun session made of named steps, each under its own time limit:
#   tools/gpu_steps.sh TAG STEP [STEP ...]
# Steps:
#   tests      pytest -m "gpu and not slow"
#   slow       pytest -m slow -s (full-size parity, prints max_rel_err)
#   bench      bench.py (the driver's default line)
#   bench2     bench.py --gpus 2 (a 2-rank rehearsal of configs[4] on one GPU)
#   prof       rocprofv3 --kernel-trace --stats of a short bench.py run
#   ab:V,V,..  tools/ab_bench.py over tuning variants (lib/libcse_tuning.so)
#   py:FILE    python -u FILE (a tools/ script)
# Output goes to gpurun_out/TAG/.  A step that ends with a fault, an abort,
# a segfault or a time limit stops the session (no further GPU step).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 3
export CSE_BAL_CACHE=/tmp/cse_bal_cache
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
for s in "$@"; do
  case "$s" in
    tests)  timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -v --timeout 120 \
              --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1; rc=$?
            tail -3 "$OUT/pytest_gpu.txt"; grep -E "FAILED|Error" "$OUT/pytest_gpu.txt" | head -20 ;;
    slow)   timeout -k 10 900 python -u -m pytest tests -m slow -x -v -s --timeout 600 \
              --timeout-method thread > "$OUT/pytest_slow.txt" 2>&1; rc=$?
            grep -E "parity:|passed|failed|FAILED" "$OUT/pytest_slow.txt" | tail -8 ;;
    bench)  timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
            tail -c 3000 "$OUT/bench.json"; tail -5 "$OUT/bench.err" ;;
    bench2) timeout -k 10 600 python -u bench.py --gpus 2 --steps 10 --no-cpu-baseline \
              > "$OUT/bench2.json" 2> "$OUT/bench2.err"; rc=$?
            tail -c 2500 "$OUT/bench2.json"; tail -5 "$OUT/bench2.err" ;;
    bm:*)   # bm:MODE -- bench.py --mode MODE (no CPU baseline, no secondary legs)
            m=${s#bm:}
            timeout -k 10 300 python -u bench.py --mode $m --no-cpu-baseline --no-secondary --steps 20 \
              > "$OUT/bench_$m.json" 2> "$OUT/bench_$m.err"; rc=$?
            python3 -c "import json,sys; b=json.loads(open('$OUT/bench_$m.json').read().strip().splitlines()[-1]); print('$m', round(b['ms_per_step'],4), 'ms', round(b['roofline']['frac'],4))" ;;
    shard:*) # shard:N -- bench.py --shard-of N (rank 0's per-GPU work of an N-way run)
            m=${s#shard:}
            timeout -k 10 300 python -u bench.py --shard-of $m --no-cpu-baseline --no-secondary --steps 50 \
              > "$OUT/bench_shard$m.json" 2> "$OUT/bench_shard$m.err"; rc=$?
            python3 -c "import json,sys; b=json.loads(open('$OUT/bench_shard$m.json').read().strip().splitlines()[-1]); print('shard of $m', round(b['ms_per_step'],4), 'ms/step', round(b['roofline']['kernel_ms_avg'],4), 'ms kernel', round(b['roofline']['frac'],4))" ;;
    prof)   mkdir -p "$OUT/prof"
            timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run \
              --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary --steps 10 \
              --warmup 2 > "$OUT/prof_bench.json" 2> "$OUT/prof.err"; rc=$?
            tail -c 1500 "$OUT/prof_bench.json" ;;
    pmc:*)  # pmc:MODE[:extra bench args with commas]: one rocprofv3 --pmc pass per
            # counter group (MI355X_MICROARCH.md block limits), then a summary
            m=${s#pmc:}; mode=${m%%:*}; extra=""; [ "$m" != "$mode" ] && extra=$(echo "${m#*:}" | tr ',' ' ')
            P="$OUT/pmc_$mode"; mkdir -p "$P"; rc=0
            rocprofv3 -L > "$P/counters_list.txt" 2>&1 || true
            i=0
            for group in "FETCH_SIZE" "WRITE_SIZE" \
                "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU" \
                "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
                "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum" \
                "TA_BUSY_avr TD_BUSY_avr" "SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS"; do
              i=$((i+1))
              timeout -s KILL 120 rocprofv3 --pmc $group -d "$P/g$i" -o run --output-format csv -- \
                python3 bench.py --no-cpu-baseline --no-secondary --steps 10 --warmup 2 --mode $mode $extra \
                > "$P/g$i.log" 2>&1 || echo "group $i ($group) rc=$?" >> "$P/errors.txt"
            done
            for d in "$P"/g*; do [ -d "$d" ] && python3 tools/pmc_summary.py "$d" Evaluate --json "$P/summary.json" > /dev/null; done
            cat "$P/summary.json"; cat "$P/errors.txt" 2>/dev/null ;;
    ab*:*)  # ab:V,V,.. (Jacobian) or abres:V,.. / abcost:V,.. (residual / cost-only);
            # abprev:/abprevres: the same on lib/libcse_prev_tuning.so
            kind=${s%%:*}; mode=jacobian; lib=""; tag=$kind
            case "$kind" in *res) mode=residual ;; *cost) mode=cost ;; esac
            case "$kind" in abprev*) lib="--lib ceres-solver-cuda_amd/lib/libcse_prev_tuning.so" ;; esac
            timeout -k 10 600 python -u tools/ab_bench.py --variants "${s#*:}" --rounds ${AB_ROUNDS:-3} \
              --steps 20 --mode $mode $lib --out "$OUT/$tag.json" > "$OUT/$tag.txt" 2>&1; rc=$?
            tail -6 "$OUT/$tag.txt" ;;
    py:*)   f=${s#py:}; b=$(basename "$f" .py)
            timeout -k 10 600 python -u "$f" > "$OUT/$b.txt" 2>&1; rc=$?
            tail -20 "$OUT/$b.txt" ;;
    *)      echo "unknown step $s"; rc=2 ;;
  esac
  echo "== step $s rc=$rc"
  if [ "$rc" -ne 0 ]; then
    case "$s" in tests|slow) fatal "$rc" && exit "$rc" ;; *) exit "$rc" ;; esac
  fi
done
exit 0
