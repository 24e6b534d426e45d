// clock_probe.hip -- the shader clock at a moment, from the GPU itself.
// One wave spins a fixed dependent-ALU loop and reads the core-clock counter
// (s_memtime: shader cycles) and the constant 100 MHz counter
// (s_memrealtime) before and after: core cycles / (wall ticks / 100 MHz) is
// the SCLK the wave ran at.  Launched between evaluations on the same
// stream (tools/clock_ramp.py).  Diagnostic only; not part of libcse.so.
//   hipcc --offload-arch=gfx950 -O3 -fPIC -shared -o tools/build/libclockprobe.so tools/clock_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(64) void ClockProbeKernel(unsigned long long* out, int iters) {
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  float x = (float)threadIdx.x;
  for (int i = 0; i < iters; ++i) x = x * 1.0000001f + 1e-7f;
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  const unsigned long long w1 = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  if (threadIdx.x == 0) {
    out[0] = c1 - c0;
    out[1] = w1 - w0;
    out[2] = x > 1e30f ? 1ull : 0ull;  // keeps the loop
  }
}

extern "C" int clock_probe_launch(unsigned long long* d_out, int iters, void* stream) {
  hipLaunchKernelGGL(ClockProbeKernel, dim3(1), dim3(64), 0, (hipStream_t)stream, d_out, iters);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
