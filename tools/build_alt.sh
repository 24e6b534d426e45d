#!/bin/bash
# Build a variant of the product library into lib/NAME/libcse.so with extra
# compile-time definitions (A/B runs: tools/gpu_run.sh "ab ...").
#   tools/build_alt.sh NAME -DMACRO=VALUE ...
set -e
cd "$(dirname "$0")/../ceres-solver-cuda_amd"
NAME=$1; shift
mkdir -p build/$NAME lib/$NAME
make -s build/layout.o build/multi_device.o build/jet_kernels.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-signed-zeros -ffinite-math-only \
  -munsafe-fp-atomics -Wall -Wno-unused-function "$@" -c -o build/$NAME/cse_evaluator.o csrc/cse_evaluator.hip
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib/$NAME/libcse.so build/$NAME/cse_evaluator.o \
  build/jet_kernels.o build/multi_device.o build/layout.o
