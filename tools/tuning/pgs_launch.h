// pgs_launch.h -- host launcher of the persistent pipelined group-store
// kernel (pgs_kernel.hpp), compiled in its own TU (pgs.hip) with MachineLICM
// off, as the other persistent kernels of the tuning build.
#ifndef CSE_PGS_LAUNCH_H_
#define CSE_PGS_LAUNCH_H_

#include <hip/hip_runtime.h>

#include "../../ceres-solver-cuda_amd/csrc/kernel_common.hpp"

namespace cse {

// Snavely<2,9,3> BSM residuals + Jacobian (GroupStoreEligible groups), loss
// kind kLoss.  Grid: three 4-wave workgroups per CU, each walking quads.
template <int kLoss>
void LaunchGroupStorePipelinedSnavely(const GroupArgs& a, hipStream_t s);

}  // namespace cse

#endif  // CSE_PGS_LAUNCH_H_
