// jet_kernels.hip -- the Snavely<2,9,3> kernels with the Jacobian by
// forward-mode Jet<double, 12> (AutoDifferentiate, autodiff.h:314-381), the
// form every other AutoDiffCostFunction kind takes; the product's default for
// this functor is the closed form (SnavelyJacobianByHand, functors.hpp).
// Same kernels, same store tails, same settings as cse_evaluator.hip's;
// only the functor type differs.  One TU of its own so both compile in
// parallel.
#include "jet_kernels.h"

namespace cse {
namespace {

using K = SnavelyJetKind;

template <int L, bool Crs>
void LaunchJac(const GroupArgs& a, int64_t num_wg, hipStream_t s) {
  (void)num_wg;
  const int64_t chunks = (a.n + kWave - 1) / kWave;
  if constexpr (Crs)
    hipLaunchKernelGGL((EvaluateAffineChunksTwoRoundCrsW1<K, L, 2, ShippedTune>), dim3((unsigned)chunks),
                       dim3(kWave), 0, s, a);
  else
    hipLaunchKernelGGL((EvaluateAffineChunksTwoRoundW1<K, L, 2, ShippedTune>), dim3((unsigned)chunks),
                       dim3(kWave), 0, s, a);
}

template <int L, bool Crs>
void LaunchPoints(const GroupArgs& a, int64_t num_wg, hipStream_t s) {
  (void)num_wg;
  const int64_t chunks = (a.n + kWave - 1) / kWave;
  hipLaunchKernelGGL((EvaluateAffineChunksFusedPointsW1<K, L, Crs, PointsOnlyTune>), dim3((unsigned)chunks),
                     dim3(kWave), 0, s, a);
}

template <int L>
void LaunchTable(const GroupArgs& a, int64_t num_wg, hipStream_t s) {
  hipLaunchKernelGGL((EvaluateTableKernel<K, L, true>), dim3((unsigned)num_wg), dim3(kBlockThreads), 0, s, a);
}


}  // namespace

JetLaunchFn JetSnavelyJacobian(int loss, bool crs) {
  switch (loss) {
    case kLossHuber: return crs ? &LaunchJac<kLossHuber, true> : &LaunchJac<kLossHuber, false>;
    case kLossCauchy: return crs ? &LaunchJac<kLossCauchy, true> : &LaunchJac<kLossCauchy, false>;
    default: return crs ? &LaunchJac<kLossTrivial, true> : &LaunchJac<kLossTrivial, false>;
  }
}

JetLaunchFn JetSnavelyFusedPoints(int loss, bool crs) {
  switch (loss) {
    case kLossHuber: return crs ? &LaunchPoints<kLossHuber, true> : &LaunchPoints<kLossHuber, false>;
    case kLossCauchy: return crs ? &LaunchPoints<kLossCauchy, true> : &LaunchPoints<kLossCauchy, false>;
    default: return crs ? &LaunchPoints<kLossTrivial, true> : &LaunchPoints<kLossTrivial, false>;
  }
}

JetLaunchFn JetSnavelyTable(int loss) {
  switch (loss) {
    case kLossHuber: return &LaunchTable<kLossHuber>;
    case kLossCauchy: return &LaunchTable<kLossCauchy>;
    default: return &LaunchTable<kLossTrivial>;
  }
}

void LaunchJetCameraGradient(int loss, const CamGradArgs& g, int64_t nslots, hipStream_t s) {
  constexpr int W = kWavesPerBlock;
  const dim3 grid((unsigned)((nslots + W - 1) / W));
  switch (loss) {
    case kLossHuber:
      hipLaunchKernelGGL((CameraGradientKernel<K, kLossHuber, W>), grid, dim3(W * kWave), 0, s, g);
      break;
    case kLossCauchy:
      hipLaunchKernelGGL((CameraGradientKernel<K, kLossCauchy, W>), grid, dim3(W * kWave), 0, s, g);
      break;
    default:
      hipLaunchKernelGGL((CameraGradientKernel<K, kLossTrivial, W>), grid, dim3(W * kWave), 0, s, g);
  }
}

}  // namespace cse
