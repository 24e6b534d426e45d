// launch.hpp -- host-side launches of the evaluator kernels for one functor
// kind, in their shipped settings (grid, workgroup size, tuning struct).
//
// Shared by the library (cse_evaluator.hip) and by user functor kinds, whose
// kernels are instantiated in the user's hipcc TU
// (include/ceres_amd/autodiff_cuda.h) the way the reference instantiates
// EvaluateKernel<CostFunctor, LossFunctionCUDA, kR, Ns...> in the user's nvcc
// TU (include/ceres/internal/autodiff_residual_block_cuda_evaluator.h:
// 183-271, cuda_evaluator_kernel.h:297-422).  Every function here launches
// exactly the kernel the library launches for the same (kind, loss, layout,
// outputs); the Snavely camera's specialised kernels (group store, fused
// gradient, held cameras) are chosen in cse_evaluator.hip and never reach
// these.
#ifndef CSE_LAUNCH_HPP_
#define CSE_LAUNCH_HPP_

#include <hip/hip_runtime.h>

#include "operator_kernels.hpp"

namespace cse {

inline int64_t Chunks(int64_t n) { return (n + kWave - 1) / kWave; }

// The general kernel: one residual block per lane, offsets through the
// descriptor's tables (EvaluateTableKernel).
template <class K, int L, bool J>
void LaunchTableKernel(const GroupArgs& a, int64_t num_wg, hipStream_t s) {
  hipLaunchKernelGGL((EvaluateTableKernel<K, L, J>), dim3((unsigned)num_wg), dim3(kBlockThreads), 0, s,
                     a);
}

// The affine kernel: one 64-block chunk per wave, 4 waves per workgroup.
// kCoop 2: slot 0 by LDS-DMA from the repacked table; 1: 8-byte pieces from
// the state.
template <class K, int L, bool J, bool Crs, int kCoop, class T = ShippedTune>
void LaunchAffineChunks(const GroupArgs& a, int64_t num_wg, hipStream_t s) {
  hipLaunchKernelGGL((EvaluateAffineChunks<K, L, J, Crs, kCoop, T>), dim3((unsigned)num_wg),
                     dim3(kBlockThreads), 0, s, a);
}

// The residual+Jacobian evaluation of two-slot kinds with the LDS-DMA
// gather: two half-wave staging rounds, one wave per workgroup
// (BlockSparseMatrix: EvaluateAffineChunksTwoRoundW1; CompressedRow:
// EvaluateAffineChunksTwoRoundCrsW1).
template <class K, int L, int kCoop, class T = ShippedTune>
void LaunchTwoRoundW1(const GroupArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((EvaluateAffineChunksTwoRoundW1<K, L, kCoop, T>), dim3((unsigned)Chunks(a.n)),
                     dim3(kWave), 0, s, a);
}
template <class K, int L, int kCoop, class T = ShippedTune>
void LaunchTwoRoundCrsW1(const GroupArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((EvaluateAffineChunksTwoRoundCrsW1<K, L, kCoop, T>), dim3((unsigned)Chunks(a.n)),
                     dim3(kWave), 0, s, a);
}

// The affine evaluation of a (non-Snavely) kind: the kernel the library's
// Pick chooses for (layout, outputs, gather).
template <class K, int L, bool Crs, bool J, bool kDma>
void LaunchAffine(const GroupArgs& a, int64_t num_wg, hipStream_t s) {
  if constexpr (J && kDma && !Crs && kTwoRoundBsm<K>) {
    LaunchTwoRoundW1<K, L, 2>(a, s);
  } else if constexpr (J && kDma && Crs) {
    LaunchTwoRoundCrsW1<K, L, 2>(a, s);
  } else {
    LaunchAffineChunks<K, L, J, Crs, kDma ? 2 : 1>(a, num_wg, s);
  }
}

// J x (affine or table) and J^T x (table; affine groups use the gradient
// post-pass for it).  which: 0 = J x affine, 1 = J x table, 2 = J^T x table.
template <class K>
void LaunchMultiplyKernel(const GroupArgs& a, int which, const double* x, double* y, hipStream_t s) {
  const dim3 grid((unsigned)((a.n + kBlockThreads - 1) / kBlockThreads));
  if constexpr (KindTraits<K>::NB <= 2) {
    if (which == 0) {
      hipLaunchKernelGGL(RightMultiplyAffineKernel<K>, grid, dim3(kBlockThreads), 0, s, a, x, y);
      return;
    }
  }
  if (which == 2)
    hipLaunchKernelGGL((MultiplyTableKernel<K, true>), grid, dim3(kBlockThreads), 0, s, a, x, y);
  else
    hipLaunchKernelGGL((MultiplyTableKernel<K, false>), grid, dim3(kBlockThreads), 0, s, a, x, y);
}

// The gradient post-pass over one slot (GradArgs; NR residuals, S columns):
// form 0 = identity order, contiguous block ranges (points); 1 = chunks of
// at most kGradChunk blocks, one wave each, then the ordered chunk reduce
// (cameras); 2 = one lane per parameter block.
enum GradForm { kGradRange = 0, kGradChunked = 1, kGradPerBlock = 2 };
template <int NR, int S>
void LaunchGradientSlot(const GradArgs& ga, const GradChunks& ch, int form, hipStream_t s) {
  if (form == kGradRange) {
    hipLaunchKernelGGL((GradientRangeKernel<NR, S>), dim3((unsigned)((ga.count + kWave - 1) / kWave)),
                       dim3(kWave), 0, s, ga);
  } else if (form == kGradChunked) {
    const dim3 grid((unsigned)((ch.nchunks + kWavesPerBlock - 1) / kWavesPerBlock));
    if (ch.nchunks > 0)
      hipLaunchKernelGGL((GradientLanesKernel<NR, S>), grid, dim3(kBlockThreads), 0, s, ga, ch);
    hipLaunchKernelGGL((GradientChunkReduceKernel<S>),
                       dim3((unsigned)((ga.count + kBlockThreads - 1) / kBlockThreads)),
                       dim3(kBlockThreads), 0, s, ga, ch);
  } else {
    hipLaunchKernelGGL((GradientSlotKernel<NR, S, false>),
                       dim3((unsigned)((ga.count + kBlockThreads - 1) / kBlockThreads)),
                       dim3(kBlockThreads), 0, s, ga);
  }
}

// The fused gradient (gradient_mode 0) of a two-slot kind whose slot 1 has
// 3 parameters, the form the library's Snavely kinds take: the Jacobian
// kernel that also sums the slot-1 rows of its sorted blocks
// (EvaluateAffineChunksFusedPointsW1, one wave per workgroup), and the
// slot-0 rows by re-evaluation in slot-0 order (CameraGradientKernel).
template <class K>
constexpr bool kFusedGradShape = KindTraits<K>::NB == 2 && KindTraits<K>::S1 == 3;

template <class K, int L, bool Crs>
void LaunchFusedPointsKernel(const GroupArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((EvaluateAffineChunksFusedPointsW1<K, L, Crs>), dim3((unsigned)Chunks(a.n)), dim3(kWave),
                     0, s, a);
}

template <class K, int L>
void LaunchCameraGradient(const CamGradArgs& g, int64_t nslots, hipStream_t s) {
  constexpr int W = kWavesPerBlock;
  hipLaunchKernelGGL((CameraGradientKernel<K, L, W>), dim3((unsigned)((nslots + W - 1) / W)), dim3(W * kWave), 0,
                     s, g);
}

}  // namespace cse

#endif  // CSE_LAUNCH_HPP_
