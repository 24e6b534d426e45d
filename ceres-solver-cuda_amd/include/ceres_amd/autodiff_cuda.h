// autodiff_cuda.h -- user AutoDiffCostFunction functors on the gfx950
// evaluator (hipcc TUs only).
//
// The reference lets any functor
//   struct F { template <typename T> HOST_DEVICE bool operator()(const T* x0,
//              ..., T* residuals) const; ... };
// be evaluated on the GPU: ProblemCUDA::AddResidualBlock<F, kR, Ns...>
// instantiates EvaluateKernel<F, LossFunctionCUDA, kR, Ns...> in the user's
// nvcc TU and registers an AutoDiffResidualBlockCUDAEvaluator per type
// (include/ceres/problem_cuda.h:423-474, README.md:19-33).  This header does
// the same for libcse.so: including it in a TU compiled with
//   hipcc --offload-arch=gfx950 -O3 -fno-signed-zeros -ffinite-math-only
// (the flags of the library's own kernels; without them the kernels are
// correct but slower) makes ProblemCUDA::AddResidualBlock accept any
// functor, and RegisterAutoDiffFunctor<F, Loss, kR, Ns...>() returns a kind
// for the C ABI (cse_residual_group.functor_kind).
//
// What the TU instantiates for (F, Loss, kR, Ns...): the library's general
// kernel (EvaluateTableKernel, any shape up to 10 parameter blocks), and for
// the shapes the affine kernels take (cse::kAffineShape: one or two blocks,
// at most three residuals, slot 0 at most 16 values, slot 1 at most 8) the
// coalesced affine kernels with the LDS-DMA camera gather, their gradient
// post-passes and J x / J^T x -- the same kernels, same settings, as a
// built-in kind of that shape -- and for two-block shapes whose second block
// has 3 parameters (<NR, S0, 3>: cameras and points) the fused gradient of
// the library's Snavely kinds (cse::kFusedGradShape: the Jacobian kernel
// summing the point rows, CameraGradientKernel the camera rows; ABI 5).
// The Jacobian is always by Jet<double,
// sum Ns> (AutoDifferentiate, include/ceres/internal/autodiff.h:314-381).
//
// Functor requirements (as the reference's, README.md:19-50): every member
// function the evaluation calls is __host__ __device__ (HOST_DEVICE); the
// functor is trivially copyable (it is copied to the device bytewise, one
// copy per residual block, at most alignment 8); the math it calls on T is
// Ceres' Jet surface (sqrt, sin, atan2, pow, comparisons, ..., cse::Jet's
// hidden friends) and the rotation helpers below.
#ifndef CERES_AMD_AUTODIFF_CUDA_H_
#define CERES_AMD_AUTODIFF_CUDA_H_

#ifndef __HIPCC__
#error "ceres_amd/autodiff_cuda.h instantiates gfx950 kernels: compile this file with hipcc"
#endif

#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>
#include <typeinfo>

#include "../../csrc/functors.hpp"
#include "../../csrc/launch.hpp"
#include "../../csrc/user_kind.hpp"
#include "problem_cuda.h"

#ifndef HOST_DEVICE
#define HOST_DEVICE __host__ __device__
#endif

namespace ceres_amd {

// The dual number the functor sees for T (Ceres' Jet<double, N>).
template <int N>
using Jet = cse::Jet<N>;

// include/ceres/rotation.h on double and Jet (the library's own forms:
// AngleAxisRotatePoint as documented in csrc/functors.hpp).
using cse::AngleAxisRotatePoint;
using cse::QuaternionRotatePoint;

// UnitQuaternionRotatePoint (include/ceres/rotation.h:753-774).
template <typename T>
HOST_DEVICE inline void UnitQuaternionRotatePoint(const T q[4], const T pt[3], T result[3]) {
  T uv0 = q[2] * pt[2] - q[3] * pt[1];
  T uv1 = q[3] * pt[0] - q[1] * pt[2];
  T uv2 = q[1] * pt[1] - q[2] * pt[0];
  uv0 += uv0;
  uv1 += uv1;
  uv2 += uv2;
  result[0] = pt[0] + q[0] * uv0;
  result[1] = pt[1] + q[0] * uv1;
  result[2] = pt[2] + q[0] * uv2;
  result[0] += q[2] * uv2 - q[3] * uv1;
  result[1] += q[3] * uv0 - q[1] * uv2;
  result[2] += q[1] * uv1 - q[2] * uv0;
}

namespace autodiff_internal {

// The LossKind the kernels apply for loss type L (ScaledLossCUDA stripped by
// BaseLoss already): the library's three by their kind, anything else as a
// user loss compiled into the kernels.
template <typename L>
struct LossCode {
  static constexpr int value = cse::kLossUser;
  using user = L;
};
template <>
struct LossCode<TrivialLossCUDA> {
  static constexpr int value = cse::kLossTrivial;
  using user = void;
};
template <>
struct LossCode<HuberLossCUDA> {
  static constexpr int value = cse::kLossHuber;
  using user = void;
};
template <>
struct LossCode<CauchyLossCUDA> {
  static constexpr int value = cse::kLossCauchy;
  using user = void;
};

inline const cse::GroupArgs& Args(const void* p) { return *static_cast<const cse::GroupArgs*>(p); }

template <class K, int L, bool J>
void TableLaunch(const void* a, int64_t num_wg, void* s) {
  cse::LaunchTableKernel<K, L, J>(Args(a), num_wg, (hipStream_t)s);
}
template <class K, int L, bool Crs, bool J, bool Dma>
void AffineLaunch(const void* a, int64_t num_wg, void* s) {
  cse::LaunchAffine<K, L, Crs, J, Dma>(Args(a), num_wg, (hipStream_t)s);
}
template <class K>
void MultiplyLaunch(const void* a, int32_t which, const double* x, double* y, void* s) {
  cse::LaunchMultiplyKernel<K>(Args(a), which, x, y, (hipStream_t)s);
}
template <int NR, int S>
void GradientLaunch(const void* ga, const void* ch, int32_t form, void* s) {
  cse::LaunchGradientSlot<NR, S>(*static_cast<const cse::GradArgs*>(ga),
                                 *static_cast<const cse::GradChunks*>(ch), form, (hipStream_t)s);
}

template <class K, int L, bool Crs>
void FusedPointsLaunch(const void* a, int64_t num_wg, void* s) {
  (void)num_wg;
  cse::LaunchFusedPointsKernel<K, L, Crs>(Args(a), (hipStream_t)s);
}
template <class K, int L>
void CameraGradientLaunch(const void* g, int64_t nslots, void* s) {
  cse::LaunchCameraGradient<K, L>(*static_cast<const cse::CamGradArgs*>(g), nslots, (hipStream_t)s);
}

template <class K, int L>
cse_functor_ops MakeOps(const char* name) {
  using Tr = cse::KindTraits<K>;
  cse_functor_ops o{};
  o.abi_version = CSE_ABI_VERSION;
  o.num_residuals = Tr::NR;
  o.num_parameter_blocks = Tr::NB;
  for (int j = 0; j < Tr::NB; ++j) o.parameter_block_sizes[j] = K::kSizes[j];
  o.data_size = Tr::D;
  o.loss_kind = L;
  if constexpr (L == cse::kLossUser) o.loss_size = (int32_t)sizeof(typename K::UserLoss);
  o.kernel_args_size = (int32_t)sizeof(cse::GroupArgs);
  o.gradient_args_size = (int32_t)sizeof(cse::GradArgs);
  o.kernel_args_tag = cse::kGroupArgsTag;
  o.name = name;
  o.table[0] = &TableLaunch<K, L, false>;
  o.table[1] = &TableLaunch<K, L, true>;
  o.multiply = &MultiplyLaunch<K>;
  if constexpr (cse::kAffineShape<K>) {
    o.affine[0][0][0] = &AffineLaunch<K, L, false, false, false>;
    o.affine[0][0][1] = &AffineLaunch<K, L, false, false, true>;
    o.affine[0][1][0] = &AffineLaunch<K, L, false, true, false>;
    o.affine[0][1][1] = &AffineLaunch<K, L, false, true, true>;
    o.affine[1][0][0] = &AffineLaunch<K, L, true, false, false>;
    o.affine[1][0][1] = &AffineLaunch<K, L, true, false, true>;
    o.affine[1][1][0] = &AffineLaunch<K, L, true, true, false>;
    o.affine[1][1][1] = &AffineLaunch<K, L, true, true, true>;
    o.gradient[0] = &GradientLaunch<Tr::NR, K::kSizes[0]>;
    if constexpr (Tr::NB > 1) o.gradient[1] = &GradientLaunch<Tr::NR, K::kSizes[Tr::NB > 1 ? 1 : 0]>;
    if constexpr (cse::kFusedGradShape<K>) {
      o.fused_points[0] = &FusedPointsLaunch<K, L, false>;
      o.fused_points[1] = &FusedPointsLaunch<K, L, true>;
      o.camera_gradient = &CameraGradientLaunch<K, L>;
      o.camera_gradient_args_size = (int32_t)sizeof(cse::CamGradArgs);
    }
  }
  return o;
}

}  // namespace autodiff_internal

// Registers (once per process) the kernels of functor F with loss type Loss
// (TrivialLossCUDA, HuberLossCUDA, CauchyLossCUDA or a user loss class;
// ScaledLossCUDA<L> uses L's kernels) and returns its kind.  Throws on a
// registration error (cse_last_error()).
template <typename F, typename Loss, int kNumResiduals, int... Ns>
int32_t RegisterAutoDiffFunctor(const char* name = nullptr) {
  using LC = autodiff_internal::LossCode<typename BaseLoss<Loss>::type>;
  using K = cse::UserKind<F, typename LC::user, kNumResiduals, Ns...>;
  const std::string label = name ? std::string(name) : std::string(typeid(K).name());
  const cse_functor_ops ops = autodiff_internal::MakeOps<K, LC::value>(label.c_str());
  int32_t kind = -1;
  if (cse_register_functor(&ops, &kind) != CSE_OK)
    throw std::runtime_error(std::string("cse_register_functor: ") + cse_last_error());
  return kind;
}

// ProblemCUDA's hook (problem_cuda.h): the kind of (F, Loss), registered on
// first use.
template <typename F, typename Loss, int kNumResiduals, int... Ns>
struct UserFunctorKind {
  using K = cse::UserKind<F, typename autodiff_internal::LossCode<Loss>::user, kNumResiduals, Ns...>;
  static constexpr int kDataSize = K::kDataSize;
  static int32_t Kind() {
    static const int32_t kind = RegisterAutoDiffFunctor<F, Loss, kNumResiduals, Ns...>();
    return kind;
  }
};

}  // namespace ceres_amd

#endif  // CERES_AMD_AUTODIFF_CUDA_H_
