// persistent_launch.h -- host launchers of the persistent software-pipelined
// BSM Jacobian kernel (persistent_kernel.hpp), compiled in their own TU
// (persistent.hip) with MachineLICM off: in the persistent loop the
// optimiser otherwise hoists the functor's FP64 constants and per-lane
// addresses out of the loop and spills them, and every spill reload costs a
// compiler vmcnt(0) that drains the software pipeline.
#ifndef CSE_PERSISTENT_LAUNCH_H_
#define CSE_PERSISTENT_LAUNCH_H_

#include <hip/hip_runtime.h>

#include "../../ceres-solver-cuda_amd/csrc/kernel_common.hpp"

namespace cse {

// Snavely<2,9,3> BSM residuals + Jacobian, loss kind kLoss (0 trivial, 1
// Huber, 2 Cauchy).  Grid: min(chunks, 8 waves per CU) single-wave
// workgroups, each walking chunks blockIdx.x, +gridDim.x, ...
template <int kLoss>
void LaunchPersistentSnavely(const GroupArgs& a, hipStream_t s);

}  // namespace cse

#endif  // CSE_PERSISTENT_LAUNCH_H_
