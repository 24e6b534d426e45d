// jet_kernels.h -- launchers of the Snavely<2,9,3> kernels with the Jacobian
// by forward-mode Jet<double, 12> (cse::SnavelyJetKind), selected per
// evaluator by cse_options.jacobian_form = CSE_JACOBIAN_JET.  They are
// instantiated in their own TU (jet_kernels.hip), compiled beside
// cse_evaluator.hip.  Loss kinds: cse::kLossTrivial / kLossHuber / kLossCauchy.
#ifndef CSE_JET_KERNELS_H_
#define CSE_JET_KERNELS_H_

#include <hip/hip_runtime.h>

#include "evaluate_kernel.hpp"

namespace cse {

using JetLaunchFn = void (*)(const GroupArgs&, int64_t num_wg, hipStream_t);

// Residuals + Jacobian on the affine kernels (no held cameras): the
// BlockSparseMatrix (crs = false, EvaluateAffineChunksTwoRoundW1) or
// CompressedRowSparseMatrix (EvaluateAffineChunksTwoRoundCrsW1) form.
JetLaunchFn JetSnavelyJacobian(int loss, bool crs);
// The fused gradient's points kernel (gradient_mode 0).
JetLaunchFn JetSnavelyFusedPoints(int loss, bool crs);
// The general (table) kernel, residuals and Jacobian.
JetLaunchFn JetSnavelyTable(int loss);
// CameraGradientKernel with the camera partials by Jet<9>, kWPB waves per
// workgroup, one chunk per wave.
void LaunchJetCameraGradient(int loss, const CamGradArgs& g, int64_t nslots, hipStream_t s);

}  // namespace cse

#endif  // CSE_JET_KERNELS_H_
