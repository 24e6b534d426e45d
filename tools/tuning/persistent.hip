// persistent.hip -- instantiations and launchers of the persistent
// software-pipelined BSM Jacobian kernel (persistent_kernel.hpp); built with
// -mllvm -disable-machine-licm (see persistent_launch.h).
#include "persistent_launch.h"

#include <algorithm>

#include "persistent_kernel.hpp"

namespace cse {

template <int kLoss>
void LaunchPersistentSnavely(const GroupArgs& a, hipStream_t s) {
  const int64_t chunks = (a.n + kWave - 1) / kWave;
  const int64_t waves = std::max<int64_t>(1, std::min<int64_t>(chunks, 8LL * std::max(1, a.num_cus)));
  hipLaunchKernelGGL((EvaluateAffinePersistent<SnavelyKind, kLoss>), dim3((unsigned)waves), dim3(kWave), 0, s, a);
}

template void LaunchPersistentSnavely<kLossTrivial>(const GroupArgs&, hipStream_t);
template void LaunchPersistentSnavely<kLossHuber>(const GroupArgs&, hipStream_t);
template void LaunchPersistentSnavely<kLossCauchy>(const GroupArgs&, hipStream_t);

}  // namespace cse
