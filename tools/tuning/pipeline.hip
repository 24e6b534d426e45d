// pipeline.hip -- instantiations and launchers of the persistent
// wave-specialised BlockSparse kernel (pipeline_kernel.hpp); built with
// -mllvm -disable-machine-licm (see pipeline_launch.h).
#include "pipeline_launch.h"

#include <algorithm>
#include <cstdio>
#include <vector>

#include "pipeline_kernel.hpp"

namespace cse {

template <int kLoss, int kStoreWaves, int kOpt>
void LaunchPipelinedSnavely(const GroupArgs& a, hipStream_t s) {
  const int64_t chunks = (a.n + kWave - 1) / kWave;
  const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(a.num_cus, chunks));
  hipLaunchKernelGGL((EvaluateAffinePipelined<SnavelyKind, kLoss, kStoreWaves, kOpt>), dim3((unsigned)grid),
                     dim3(kPipeThreads), 0, s, a);
}

#define CSE_PIPE_INST(L, W) template void LaunchPipelinedSnavely<L, W, 0>(const GroupArgs&, hipStream_t);
#define CSE_PIPE_INST2(L, W, O) template void LaunchPipelinedSnavely<L, W, O>(const GroupArgs&, hipStream_t);
CSE_PIPE_INST(kLossTrivial, 4)
CSE_PIPE_INST(kLossHuber, 4)
#ifdef CSE_TUNING
// Tuning build: the kernel with per-wave cycle accounting (s_memtime around
// each phase), summed over launches and printed every 23 launches.
template <int kLoss, int kStoreWaves, int kOpt>
void LaunchPipelinedSnavelyProbe(const GroupArgs& a0, hipStream_t s) {
  static unsigned long long* buf = nullptr;
  static int launches = 0;
  const int nwaves = a0.num_cus * kPipeWaves;
  if (!buf) {
    (void)hipMalloc(&buf, (size_t)nwaves * 8 * sizeof(unsigned long long));
    (void)hipMemset(buf, 0, (size_t)nwaves * 8 * sizeof(unsigned long long));
  }
  GroupArgs a = a0;
  a.probe = buf;
  const int64_t chunks = (a.n + kWave - 1) / kWave;
  const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(a.num_cus, chunks));
  hipLaunchKernelGGL((EvaluateAffinePipelined<SnavelyKind, kLoss, kStoreWaves, kOpt | 1>),
                     dim3((unsigned)grid), dim3(kPipeThreads), 0, s, a);
  if (++launches % 23 != 0) return;
  (void)hipStreamSynchronize(s);
  std::vector<unsigned long long> h((size_t)nwaves * 8);
  (void)hipMemcpy(h.data(), buf, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  constexpr int NC = kPipeWaves - kStoreWaves;
  double cs[6] = {0}, ss[6] = {0};
  for (int b = 0; b < grid; ++b)
    for (int w = 0; w < kPipeWaves; ++w)
      for (int k = 0; k < 6; ++k) (w < NC ? cs : ss)[k] += (double)h[((size_t)b * kPipeWaves + w) * 8 + k];
  fprintf(stderr,
          "# probe (%d launches, store waves %d) compute per chunk [cycles]: wait-inputs %.0f "
          "read+issue %.0f evaluate %.0f wait-slot %.0f write-slot %.0f | store per chunk: "
          "wait-fill %.0f read-slot %.0f issue-stores %.0f\n",
          launches, kStoreWaves, cs[0] / cs[5], cs[1] / cs[5], cs[2] / cs[5], cs[3] / cs[5],
          cs[4] / cs[5], ss[0] / ss[5], ss[1] / ss[5], ss[2] / ss[5]);
}
#define CSE_PROBE_INST(L, W, O) template void LaunchPipelinedSnavelyProbe<L, W, O>(const GroupArgs&, hipStream_t);
CSE_PROBE_INST(kLossHuber, 4, 0)
CSE_PROBE_INST(kLossTrivial, 4, 0)
CSE_PROBE_INST(kLossHuber, 8, 0)
CSE_PROBE_INST(kLossTrivial, 8, 0)
CSE_PROBE_INST(kLossHuber, 8, 2)
CSE_PROBE_INST(kLossTrivial, 8, 2)
CSE_PIPE_INST2(kLossTrivial, 8, 2)
CSE_PIPE_INST2(kLossHuber, 8, 2)
CSE_PIPE_INST2(kLossTrivial, 4, 2)
CSE_PIPE_INST2(kLossHuber, 4, 2)
CSE_PIPE_INST2(kLossTrivial, 6, 2)
CSE_PIPE_INST2(kLossHuber, 6, 2)
CSE_PIPE_INST(kLossTrivial, 6)
CSE_PIPE_INST(kLossHuber, 6)
CSE_PIPE_INST(kLossTrivial, 8)
CSE_PIPE_INST(kLossHuber, 8)
CSE_PIPE_INST(kLossTrivial, 3)
CSE_PIPE_INST(kLossHuber, 3)
CSE_PIPE_INST(kLossTrivial, 2)
CSE_PIPE_INST(kLossHuber, 2)
#endif
#undef CSE_PIPE_INST
#undef CSE_PIPE_INST2

// Residual-only / cost-only streamed kernel: kWG waves per workgroup,
// kPerCu workgroups per CU (the LDS input buffers: 8 KiB a wave).
template <int kLoss, int kWG, int kPerCu>
void LaunchResidualStreamedSnavely(const GroupArgs& a, hipStream_t s) {
  const int64_t chunks = (a.n + kWave - 1) / kWave;
  const int64_t grid =
      std::max<int64_t>(1, std::min<int64_t>((int64_t)a.num_cus * kPerCu, (chunks + kWG - 1) / kWG));
  if (a.residuals)
    hipLaunchKernelGGL((EvaluateResidualStreamed<SnavelyKind, kLoss, true, kWG>), dim3((unsigned)grid),
                       dim3(kWG * kWave), 0, s, a);
  else
    hipLaunchKernelGGL((EvaluateResidualStreamed<SnavelyKind, kLoss, false, kWG>), dim3((unsigned)grid),
                       dim3(kWG * kWave), 0, s, a);
}
#define CSE_RES_INST(L, G, C) template void LaunchResidualStreamedSnavely<L, G, C>(const GroupArgs&, hipStream_t);
CSE_RES_INST(kLossHuber, 8, 2)
CSE_RES_INST(kLossTrivial, 8, 2)
CSE_RES_INST(kLossHuber, 16, 1)
CSE_RES_INST(kLossTrivial, 16, 1)
CSE_RES_INST(kLossHuber, 4, 4)
CSE_RES_INST(kLossTrivial, 4, 4)
#undef CSE_RES_INST

}  // namespace cse
