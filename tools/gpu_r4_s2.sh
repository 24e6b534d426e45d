#!/bin/bash
# Round 4 session 2: held-camera chunk bounds loaded early (lib/h2 vs h1),
# the 1024-slice cost reduction (lib/r2 vs h2) at problem-13682 and at
# configs[2] (problem-1778 CRS), per-kernel PMC of the held and unheld
# evaluations, and the bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=${TAG:-r4s2}
TAG=$T/ab_held MODE=jacobian PREV=h1 ALT=h2 ABFLAGS="--held-cameras 1" bash tools/gpu_ab_alt.sh || exit 1
TAG=$T/ab_red MODE=jacobian PREV=h2 ALT=r2 bash tools/gpu_ab_alt.sh || exit 1
TAG=$T/ab_red1778 MODE=jacobian PREV=h2 ALT=r2 ABFLAGS="--config problem-1778-993923 --format compressed_row" bash tools/gpu_ab_alt.sh || exit 1
BENCH_ARGS="--no-cpu-baseline --no-secondary --steps 5 --warmup 1 --held-cameras 1 --lib ceres-solver-cuda_amd/lib/h2/libcse.so" bash tools/gpu_pmc_kernels.sh $T/pmc_held > /dev/null || exit 1
BENCH_ARGS="--no-cpu-baseline --no-secondary --steps 5 --warmup 1 --lib ceres-solver-cuda_amd/lib/h2/libcse.so" bash tools/gpu_pmc_kernels.sh $T/pmc_plain > /dev/null || exit 1
grep -h "EvaluateAffine\|Fixup\|Repack\|Finalize" gpurun_out/$T/pmc_held/pmc_by_kernel.txt gpurun_out/$T/pmc_plain/pmc_by_kernel.txt | cut -c1-400
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > gpurun_out/$T/bench.txt 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/$T/bench.txt; exit 1; }
tail -1 gpurun_out/$T/bench.txt | cut -c1-600
