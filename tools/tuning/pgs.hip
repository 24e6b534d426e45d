// pgs.hip -- instantiations and launchers of the persistent pipelined
// group-store kernel (pgs_kernel.hpp); built with -mllvm
// -disable-machine-licm (see pgs_launch.h).
#include "pgs_launch.h"

#include <algorithm>

#include "pgs_kernel.hpp"

namespace cse {

template <int kLoss>
void LaunchGroupStorePipelinedSnavely(const GroupArgs& a, hipStream_t s) {
  const int64_t nfull = a.n / (4 * kWave);
  const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(nfull, 3LL * std::max(1, a.num_cus)));
  hipLaunchKernelGGL((EvaluateGroupStorePipelined<SnavelyKind, kLoss>), dim3((unsigned)grid),
                     dim3(kBlockThreads), 0, s, a, nfull);
}

template void LaunchGroupStorePipelinedSnavely<kLossTrivial>(const GroupArgs&, hipStream_t);
template void LaunchGroupStorePipelinedSnavely<kLossHuber>(const GroupArgs&, hipStream_t);
template void LaunchGroupStorePipelinedSnavely<kLossCauchy>(const GroupArgs&, hipStream_t);

}  // namespace cse
