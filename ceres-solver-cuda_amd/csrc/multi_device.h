// multi_device.h -- internal interface of the single-process multi-device
// evaluator behind cse_create_multi (include/cse.h).
//
// One Ceres host solve calls one evaluator with host pointers
// (RegisteredCUDAEvaluators::Evaluate, include/ceres/internal/
// registered_cuda_evaluators.h:75-79) and expects every output in its own
// buffers (registered_cuda_evaluators.cc:93-100).  CseMulti cuts the
// Program's residual blocks into contiguous shards at point-bucket
// boundaries, gives each shard an ordinary evaluator on its
// device, and on each Evaluate copies every shard's residual and Jacobian
// strips straight into disjoint regions of the caller's one residual and
// values buffers (asynchronously when the caller page-locked them), while the cost and the gradient rows
// are summed over the shards in a fixed order on the host.
#ifndef CSE_MULTI_DEVICE_H_
#define CSE_MULTI_DEVICE_H_

#include <stddef.h>
#include <stdint.h>

#include <string>

#include "../../include/cse.h"

struct CseMulti;

// Records msg as the thread's last error (cse_last_error) and returns code.
int CseFail(int code, const std::string& msg);
// Residuals, parameter blocks and functor-data doubles per residual block of
// a functor kind; false for an unknown kind (cse_evaluator.hip).
bool CseKindShape(int kind, int* num_residuals, int* num_blocks, int* data_size);

int MultiCreate(const cse_problem_desc* desc, const cse_options* options, const int32_t* devices,
                int32_t num_devices, CseMulti** out);
void MultiDestroy(CseMulti* m);
int MultiEvaluate(CseMulti* m, const double* state, double* cost, double* residuals,
                  double* gradient, double* jacobian_values, bool same_point);
int MultiInfo(CseMulti* m, cse_info* info);
int MultiShardInfo(CseMulti* m, int32_t* num_shards, int64_t* first_block, int32_t* devices);
int MultiSetPlusJacobians(CseMulti* m, const double* plus_jacobians);
int MultiPlus(CseMulti* m, const double* state, const double* delta, double* state_plus_delta);
int MultiTransferBytes(CseMulti* m, int64_t* state_h2d, int64_t* strips_d2h);
int CseHostRegister(void* p, size_t bytes);
int CseHostUnregister(void* p);
int MultiKernelStats(CseMulti* m, double* last_ms, double* total_ms, int64_t* launches);
int MultiResetKernelStats(CseMulti* m);

#endif  // CSE_MULTI_DEVICE_H_
