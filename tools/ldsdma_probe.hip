// Probe: where does global_load_lds of size 4 / 12 / 16 put lane l's bytes?
// hipcc --offload-arch=gfx950 -O2 -o tools/ldsdma_probe tools/ldsdma_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __attribute__((noinline)) void Dma(const char* src, double* lds, int size, int lane) {
  if (size == 4) __builtin_amdgcn_global_load_lds(src + 4 * lane, lds, 4, 0, 0);
  if (size == 12) __builtin_amdgcn_global_load_lds(src + 12 * lane, lds, 12, 0, 2);
  if (size == 16) __builtin_amdgcn_global_load_lds(src + 16 * lane, lds, 16, 0, 0);
}

__global__ void probe(const double* src, double* out, int size) {
  __shared__ double buf[64 * 2 + 8];
  const int lane = threadIdx.x;
  for (int i = lane; i < 64 * 2 + 8; i += 64) buf[i] = -1.0;
  __syncthreads();
  Dma(reinterpret_cast<const char*>(src), buf, size, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = lane; i < 64 * 2 + 8; i += 64) out[i] = buf[i];
}

int main() {
  uint8_t h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = (uint8_t)(i & 255);
  double *d_src, *d_out;
  if (hipMalloc(&d_src, 4096) || hipMalloc(&d_out, 4096)) return 1;
  if (hipMemcpy(d_src, h, 4096, hipMemcpyHostToDevice)) return 1;
  for (int size : {4, 12, 16}) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d_src, d_out, size);
    uint8_t o[(64 * 2 + 8) * 8];
    if (hipMemcpy(o, d_out, sizeof(o), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    int bad = 0;
    for (int i = 0; i < 64 * size; ++i) bad += o[i] != (uint8_t)(i & 255);
    printf("size %2d: lane*size layout %s (%d of %d bytes differ); bytes 0..47:", size,
           bad ? "NO" : "yes", bad, 64 * size);
    for (int i = 0; i < 48; ++i) printf(" %02x", o[i]);
    printf("\n");
  }
  return hipDeviceSynchronize() != hipSuccess;
}
