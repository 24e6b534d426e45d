// jet_ops.hip -- device side of tests/test_jet_gpu.py (test code, not
// product): the library's Jet (ceres-solver-cuda_amd/csrc/jet.hpp), built
// with the product kernels' flags, applied on the GPU to the operands of
// internal/ceres/jet_cuda_test.cu.cc:101-104.  The test compares each result
// with the reference's jet.h formulas evaluated on the host at the
// reference's relative tolerance 1e-13 (jet_cuda_test.cu.cc:55-84).
#include <hip/hip_runtime.h>

#include "../../ceres-solver-cuda_amd/csrc/jet.hpp"

using J = cse::Jet<2>;

// Results in the order jet_ops_names() lists them; each is (a, v0, v1).
__global__ void JetOpsKernel(J x, J y, J z, double s, J* out) {
  int k = 0;
  // CompoundOperators (:88-121) minus /= (not in the library's Jet).
  J t = x;
  t += y;
  out[k++] = t;
  t = x;
  t -= y;
  out[k++] = t;
  t = x;
  t *= y;
  out[k++] = t;
  // UnitaryOperators (:195-233): unary minus.
  out[k++] = -x;
  // BinaryOperators (:235-273).
  out[k++] = x + y;
  out[k++] = x - y;
  out[k++] = x * y;
  out[k++] = x / y;
  // BinaryOperatorsWithScalar (:275-324).
  out[k++] = x + s;
  out[k++] = s + x;
  out[k++] = x - s;
  out[k++] = s - x;
  out[k++] = x * s;
  out[k++] = s * x;
  out[k++] = x / s;
  out[k++] = s / x;
  // MathFunctions (:561-689), the ones the library's functors use.
  out[k++] = cse::jsqrt(x);
  out[k++] = cse::jsqrt(y);
  out[k++] = cse::jabs(x);
  out[k++] = cse::jabs(-x);
  J sn, cs;
  cse::jsincos(x, &sn, &cs);
  out[k++] = sn;
  out[k++] = cs;
  cse::jsincos(z, &sn, &cs);
  out[k++] = sn;
  out[k++] = cs;
  out[k++] = cse::jhypot(x, y, z);
  out[k++] = cse::jhypot(z, -y, x);
  out[k++] = cse::jhypot(z, z, z);
}

extern "C" {

const char* jet_ops_names(void) {
  return "x+=y;x-=y;x*=y;-x;x+y;x-y;x*y;x/y;x+s;s+x;x-s;s-x;x*s;s*x;x/s;s/x;"
         "sqrt(x);sqrt(y);abs(x);abs(-x);sin(x);cos(x);sin(z);cos(z);"
         "hypot(x,y,z);hypot(z,-y,x);hypot(z,z,z)";
}

// x, y, z: (a, v0, v1) each; out: 3 doubles per result.  Returns the number
// of results, or -1 on a HIP error.
int jet_ops_run(const double* x, const double* y, const double* z, double s, double* out) {
  constexpr int kResults = 27;
  J jx, jy, jz;
  jx.a = x[0], jx.v[0] = x[1], jx.v[1] = x[2];
  jy.a = y[0], jy.v[0] = y[1], jy.v[1] = y[2];
  jz.a = z[0], jz.v[0] = z[1], jz.v[1] = z[2];
  J* d = nullptr;
  if (hipMalloc(&d, kResults * sizeof(J)) != hipSuccess) return -1;
  hipLaunchKernelGGL(JetOpsKernel, dim3(1), dim3(1), 0, 0, jx, jy, jz, s, d);
  J h[kResults];
  const bool ok = hipGetLastError() == hipSuccess &&
                  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess;
  (void)hipFree(d);
  if (!ok) return -1;
  for (int i = 0; i < kResults; ++i) {
    out[3 * i] = h[i].a;
    out[3 * i + 1] = h[i].v[0];
    out[3 * i + 2] = h[i].v[1];
  }
  return kResults;
}

// sin and cos of n arguments through cse::SinCos, 64 per wave: the
// library's reduction-free polynomial serves waves whose arguments are all
// within pi/4, the library sincos every other wave.
__global__ void SinCosKernel(const double* x, int n, double* s, double* c) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  cse::SinCos(x[i], s + i, c + i);
}

int sincos_run(const double* x, int n, double* s, double* c) {
  double* d = nullptr;
  if (hipMalloc(&d, 3 * (size_t)n * sizeof(double)) != hipSuccess) return -1;
  bool ok = hipMemcpy(d, x, n * sizeof(double), hipMemcpyHostToDevice) == hipSuccess;
  hipLaunchKernelGGL(SinCosKernel, dim3((n + 255) / 256), dim3(256), 0, 0, d, n, d + n, d + 2 * n);
  ok = ok && hipGetLastError() == hipSuccess &&
       hipMemcpy(s, d + n, n * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess &&
       hipMemcpy(c, d + 2 * n, n * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess;
  (void)hipFree(d);
  return ok ? n : -1;
}

}  // extern "C"
