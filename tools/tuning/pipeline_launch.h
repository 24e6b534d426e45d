// pipeline_launch.h -- host launchers of the persistent wave-specialised
// BlockSparse kernel (pipeline_kernel.hpp), compiled in their own TU
// (csrc/pipeline.hip) with MachineLICM off: in a persistent loop the
// optimiser would otherwise hoist the functor's FP64 constants and per-lane
// addresses out of the loop and spill them (95 VGPRs of scratch).
#ifndef CSE_PIPELINE_LAUNCH_H_
#define CSE_PIPELINE_LAUNCH_H_

#include <hip/hip_runtime.h>

#include "../../ceres-solver-cuda_amd/csrc/kernel_common.hpp"

namespace cse {

// Snavely<2,9,3> BSM residual+Jacobian, loss kind kLoss (0 trivial, 1
// Huber, 2 Cauchy), kStoreWaves store waves per workgroup.  Grid: one
// workgroup per CU (a.num_cus), at most one per chunk.
template <int kLoss, int kStoreWaves, int kOpt = 0>
void LaunchPipelinedSnavely(const GroupArgs& a, hipStream_t s);
template <int kLoss, int kWG, int kPerCu>
void LaunchResidualStreamedSnavely(const GroupArgs& a, hipStream_t s);
#ifdef CSE_TUNING
template <int kLoss, int kStoreWaves, int kOpt = 0>
void LaunchPipelinedSnavelyProbe(const GroupArgs& a, hipStream_t s);
#endif

}  // namespace cse

#endif  // CSE_PIPELINE_LAUNCH_H_
