#!/bin/bash
# Waves per CU for the by-hand kernels: BSM Jacobian capped at 11/12/13
# (LDS padding, lib/b11 b12 b13) against the Jets (lib/jet); the fused
# gradient's points kernel at 12/16 waves per CU (fp12, fp16), 5 per SIMD
# (fp5) or uncapped (fh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r4s7}/bsm VARIANTS="plain:jet: plain:b11: plain:b12: plain:b13:" bash tools/gpu_r4_held_probe2.sh || exit 1
TAG=${TAG:-r4s7}/grad VARIANTS="g:jet:--mode=gradient g:fh:--mode=gradient g:fp12:--mode=gradient g:fp16:--mode=gradient g:fp5:--mode=gradient" bash tools/gpu_r4_held_probe2.sh || exit 1
