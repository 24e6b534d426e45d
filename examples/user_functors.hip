// user_functors.hip -- user AutoDiffCostFunction functors and losses on the
// gfx950 evaluator, as a user of the reference would write them
// (README.md:19-50): plain templated functors, compiled here with hipcc
// against ceres_amd/autodiff_cuda.h, their kernels registered with
// libcse.so through cse_register_functor.  Built into
// examples/build/libuser_functors.so; tests/test_user_functor_gpu.py and
// bench.py's secondary.user_functor line load it.
//
// The functors restate, by their published definitions:
//   BundlerResidual            internal/ceres/bundle_adjustment_test_util.h:188-227
//   SnavelyReprojectionError   examples/snavely_reprojection_error.h:54-105
//   ...NoRadialDistortion,     internal/ceres/evaluator_cuda_test.cu.cc:84-230
//   ...WithQuaternions, PointDisplacementError
//   BinaryScalarCost,          internal/ceres/autodiff_cost_function_cuda_test.cu.cc:
//   TenParameterCost,          40-51, 123-139, 224-230
//   OnlyFillsOneOutputFunctor
// three functors of other shapes (PoseReprojectionError <2, 6, 3> with six
// doubles of data, PointToPlaneError <1, 6, 3>, RigidAlignmentError <3, 6>),
// and two losses of internal/ceres/loss_function.cc as LossFunctionCUDA
// classes: SoftLOneLoss (:66-73) and TolerantLoss (:93-118, rho'' > 0: the
// Corrector's full branch).
#include "user_functors.h"

#include <cstring>



namespace {

using namespace ceres_amd;
struct Entry {
  const char* name;
  int32_t (*reg)(const char*);
};
template <typename F, typename L, int kR, int... Ns>
int32_t Reg(const char* name) {
  return RegisterAutoDiffFunctor<F, L, kR, Ns...>(name);
}
// The order is the interface: cse_example_kind_name(i) / kinds[i].
const Entry kEntries[] = {
    {"BundlerResidual/Trivial", &Reg<user::BundlerResidual, TrivialLossCUDA, 2, 9, 3>},
    {"BundlerResidual/Huber", &Reg<user::BundlerResidual, HuberLossCUDA, 2, 9, 3>},
    {"BundlerResidual/SoftLOne", &Reg<user::BundlerResidual, user::SoftLOneLossCUDA, 2, 9, 3>},
    {"BundlerResidual/Tolerant", &Reg<user::BundlerResidual, user::TolerantLossCUDA, 2, 9, 3>},
    {"SnavelyReprojectionError/Trivial", &Reg<user::SnavelyReprojectionError, TrivialLossCUDA, 2, 9, 3>},
    {"SnavelyReprojectionError/Huber", &Reg<user::SnavelyReprojectionError, HuberLossCUDA, 2, 9, 3>},
    {"SnavelyReprojectionError/Cauchy", &Reg<user::SnavelyReprojectionError, CauchyLossCUDA, 2, 9, 3>},
    {"SnavelyReprojectionErrorNoRadialDistortion/Trivial",
     &Reg<user::SnavelyReprojectionErrorNoRadialDistortion, TrivialLossCUDA, 2, 7, 3>},
    {"SnavelyReprojectionErrorWithQuaternions/Trivial",
     &Reg<user::SnavelyReprojectionErrorWithQuaternions, TrivialLossCUDA, 2, 10, 3>},
    {"PointDisplacementError/Trivial", &Reg<user::PointDisplacementError, TrivialLossCUDA, 3, 3>},
    {"BinaryScalarCost/Trivial", &Reg<user::BinaryScalarCost, TrivialLossCUDA, 1, 2, 2>},
    {"TenParameterCost/Trivial",
     &Reg<user::TenParameterCost, TrivialLossCUDA, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1>},
    {"OnlyFillsOneOutputFunctor/Trivial", &Reg<user::OnlyFillsOneOutputFunctor, TrivialLossCUDA, 2, 1>},
    {"PoseReprojectionError/Trivial", &Reg<user::PoseReprojectionError, TrivialLossCUDA, 2, 6, 3>},
    {"PoseReprojectionError/Huber", &Reg<user::PoseReprojectionError, HuberLossCUDA, 2, 6, 3>},
    {"PointToPlaneError/Cauchy", &Reg<user::PointToPlaneError, CauchyLossCUDA, 1, 6, 3>},
    {"RigidAlignmentError/Trivial", &Reg<user::RigidAlignmentError, TrivialLossCUDA, 3, 6>},
};
constexpr int kNumEntries = (int)(sizeof(kEntries) / sizeof(kEntries[0]));

}  // namespace

extern "C" {

// Registers every kind above; kinds[i] receives entry i's kind.  Returns the
// number of kinds, or -1 (cse_last_error() says why).
int cse_example_register(int32_t* kinds, int32_t capacity) {
  if (capacity < kNumEntries) return -1;
  try {
    for (int i = 0; i < kNumEntries; ++i) kinds[i] = kEntries[i].reg(kEntries[i].name);
  } catch (const std::exception&) {
    return -1;
  }
  return kNumEntries;
}

const char* cse_example_kind_name(int32_t i) { return i >= 0 && i < kNumEntries ? kEntries[i].name : nullptr; }

// The user losses' object bytes (cse_loss.user): SoftLOne(a), Tolerant(a, b).
int cse_example_soft_l_one(double a, void* out) {
  const user::SoftLOneLossCUDA l(a);
  std::memcpy(out, &l, sizeof(l));
  return (int)sizeof(l);
}
int cse_example_tolerant(double a, double b, void* out) {
  const user::TolerantLossCUDA l(a, b);
  std::memcpy(out, &l, sizeof(l));
  return (int)sizeof(l);
}

}  // extern "C"
