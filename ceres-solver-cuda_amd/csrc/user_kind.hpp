// user_kind.hpp -- a user's AutoDiffCostFunction functor as a kernel kind.
//
// The reference evaluates any functor F with
//   template <typename T> bool operator()(const T* x0, ..., T* residuals) const
// on the GPU (AutoDiffCostFunctionCUDA<F, kR, Ns...>::Evaluate,
// include/ceres/autodiff_cost_function_cuda.h:55-71: the functor on plain
// doubles without Jacobians, through AutoDifferentiate on
// Jet<double, sum Ns> with them).  UserKind<F, UserLoss, kR, Ns...> gives F
// the compile-time shape and the Evaluate / EvaluateFlat entry points the
// library's kernels call, so the same kernels (EvaluateAffineChunks*,
// EvaluateTableKernel) run it.  Instantiated in the user's hipcc TU by
// include/ceres_amd/autodiff_cuda.h.
//
// The functor object travels as per-block functor data, its bytes in
// ceil(sizeof(F) / 8) doubles (the reference copies one functor per block to
// the device, autodiff_residual_block_cuda_evaluator.h:96-133), so F must be
// trivially copyable with alignment at most 8.
#ifndef CSE_USER_KIND_HPP_
#define CSE_USER_KIND_HPP_

#include <type_traits>
#include <utility>

#include "kernel_common.hpp"

namespace cse {

// Functor-declared kMayLeaveOutputs (the functor may leave outputs
// unassigned; AutoDifferentiate's kImpossibleValue check then applies, on
// the general kernel).
template <class F, class = void>
struct FunctorMayLeaveOutputs {
  static constexpr bool value = false;
};
template <class F>
struct FunctorMayLeaveOutputs<F, decltype((void)F::kMayLeaveOutputs)> {
  static constexpr bool value = F::kMayLeaveOutputs;
};

template <class F, class UL, int kR, int... Ns>
struct UserKind {
  static_assert(sizeof...(Ns) >= 1 && sizeof...(Ns) <= kMaxSlots,
                "between 1 and 10 parameter blocks (the reference's StaticParameterDims bound)");
  static_assert(kR >= 1, "static number of residuals");
  static_assert(std::is_trivially_copyable<F>::value,
                "the functor is copied to the device bytewise: it must be trivially copyable");
  static_assert(alignof(F) <= alignof(double), "functor alignment above 8 bytes");
  using Functor = F;
  using UserLoss = UL;  // void: a library loss (LossKind)
  static constexpr int kNumResiduals = kR;
  static constexpr int kNumBlocks = (int)sizeof...(Ns);
  static constexpr int kSizes[kNumBlocks] = {Ns...};
  static constexpr int kSize0 = kSizes[0];
  static constexpr int kSize1 = kNumBlocks > 1 ? kSizes[kNumBlocks > 1 ? 1 : 0] : 0;
  static constexpr int kDataSize = sizeof(F) <= sizeof(double) ? 1 : (int)((sizeof(F) + 7) / 8);
  static constexpr bool kMayLeaveOutputs = FunctorMayLeaveOutputs<F>::value;

  // The functor rebuilt from its data doubles.
  struct Holder {
    alignas(F) unsigned char bytes[sizeof(F)];
    CSE_HD explicit Holder(const double* d) { __builtin_memcpy(bytes, d, sizeof(F)); }
    CSE_HD const F& get() const { return *reinterpret_cast<const F*>(bytes); }
  };

  // Two-slot entry (affine kernels): slot 0 at x0, slot 1 at x1.
  template <typename T>
  static CSE_HD bool Evaluate(const double* d, const T* x0, const T* x1, T* r) {
    const Holder h(d);
    if constexpr (kNumBlocks == 1) {
      (void)x1;
      return h.get()(x0, r);
    } else {
      return h.get()(x0, x1, r);
    }
  }

  // Flat entry (general kernel): the blocks concatenated in slot order.
  template <typename T>
  static CSE_HD bool EvaluateFlat(const double* d, const T* x, T* r) {
    const Holder h(d);
    return Call(h.get(), x, r, std::make_integer_sequence<int, kNumBlocks>{});
  }

 private:
  template <int J>
  static constexpr int Offset() {
    int o = 0;
    for (int b = 0; b < J; ++b) o += kSizes[b];
    return o;
  }
  template <typename T, int... Js>
  static CSE_HD bool Call(const F& f, const T* x, T* r, std::integer_sequence<int, Js...>) {
    return f((x + Offset<Js>())..., r);
  }
};

// The shapes the affine kernels take for a user kind: the host's bound
// (DetectAffine: one or two parameter blocks, at most three residuals),
// slot sizes within one 128-byte row of the repacked slot-0 table
// (PackedRowDoubles: at most 16 doubles) and 8 for slot 1, functors that
// assign every output.  The library's own kinds cover <2, 9|7|10, 3> and
// <3, 3> against the oracle; tests/test_user_functor_gpu.py checks the other
// shapes of examples/user_functors.hip (<2, 6, 3> with six doubles of data,
// <1, 6, 3>, <3, 6>) against the general kernel, which runs the same functor
// one block per lane.  Other shapes run the general kernel.
template <class K>
constexpr bool kAffineShape =
    !K::kMayLeaveOutputs && K::kNumResiduals <= 3 && K::kNumBlocks <= 2 && K::kSize0 <= 16 &&
    (K::kNumBlocks == 1 || K::kSize1 <= 8) && K::kDataSize <= 32;

}  // namespace cse

#endif  // CSE_USER_KIND_HPP_
