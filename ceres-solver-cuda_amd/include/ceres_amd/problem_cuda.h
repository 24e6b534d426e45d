// problem_cuda.h -- C++ host facade with the reference's ProblemCUDA surface.
//
// Mirrors include/ceres/problem_cuda.h (ProblemCUDA::AddResidualBlock<F, kR,
// Ns...>(cost, loss, x0, xs...), SetParameterBlockConstant, SetManifold, ...)
// and the evaluator seam of internal/ceres/program_evaluator_cuda.h
// (Evaluate(state, cost, residuals, gradient, jacobian_values)), on top of
// the C ABI in include/cse.h.  Header-only; link libcse.so.
//
// Residual functors: AddResidualBlock<F, kR, Ns...> takes any
// AutoDiffCostFunction-style functor (template <typename T> bool
// operator()(const T*..., T*) const), by value or wrapped in an
// AutoDiffCostFunction<F, kR, Ns...>, as the reference does
// (problem_cuda.h:110-160,423-474).  The library's own kinds
// (SnavelyReprojectionError, ...WithQuaternions, ...NoRadialDistortion,
// PointDisplacementError below) are pre-instantiated in libcse.so and work
// from any C++ compiler; any other functor has its kernels instantiated in
// the caller's TU, which must then be compiled with hipcc for gfx950 and
// include ceres_amd/autodiff_cuda.h (the reference likewise compiles user
// functors with nvcc, README.md:19-33).
//
// Differences from the reference, on purpose:
//  * manifolds are given by their PlusJacobian (the only thing the
//    evaluator uses, cuda_evaluator_kernel.h:355-371), recomputed from the
//    current state on every Evaluate;
//  * loss objects are small value types, owned by the problem.
#ifndef CERES_AMD_PROBLEM_CUDA_H_
#define CERES_AMD_PROBLEM_CUDA_H_

#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <numeric>
#include <stdexcept>
#include <string>
#include <tuple>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../../include/cse.h"

namespace ceres_amd {

// ---------------------------------------------------------------------------
// Loss functions (include/ceres/loss_function_cuda.h:62-150).  The library's
// three are described to the C ABI by kind and parameter; any other class
// with __host__ __device__ void Evaluate(double s, double rho[3]) const is a
// user loss (CSE_LOSS_USER): it is compiled into the user functor kind's
// kernels and its object travels as bytes (trivially copyable, at most
// CSE_USER_LOSS_BYTES).
// ---------------------------------------------------------------------------
struct TrivialLossCUDA {
  cse_loss Describe() const { return cse_loss{CSE_LOSS_TRIVIAL, 0, 1.0, 1.0}; }
};
struct HuberLossCUDA {
  explicit HuberLossCUDA(double a) : a(a) {}
  cse_loss Describe() const { return cse_loss{CSE_LOSS_HUBER, 0, a, 1.0}; }
  double a;
};
struct CauchyLossCUDA {
  explicit CauchyLossCUDA(double a) : a(a) {}
  cse_loss Describe() const { return cse_loss{CSE_LOSS_CAUCHY, 0, a, 1.0}; }
  double a;
};
template <typename L, typename = void>
struct HasDescribe : std::false_type {};
template <typename L>
struct HasDescribe<L, decltype((void)std::declval<const L&>().Describe())> : std::true_type {};

// The C-ABI description of a loss object (library or user loss).
template <typename L>
cse_loss DescribeLoss(const L& loss) {
  if constexpr (HasDescribe<L>::value) {
    return loss.Describe();
  } else {
    static_assert(std::is_trivially_copyable<L>::value && sizeof(L) <= CSE_USER_LOSS_BYTES,
                  "a user LossFunctionCUDA must be trivially copyable and at most 64 bytes");
    cse_loss l{};
    l.kind = CSE_LOSS_USER;
    l.a = 0.0;
    l.scale = 1.0;
    std::memcpy(l.user, &loss, sizeof(L));
    return l;
  }
}

template <typename LossFunctionCUDA>
struct ScaledLossCUDA {
  ScaledLossCUDA(const LossFunctionCUDA& rho, double a) : rho(rho), a(a) {}
  cse_loss Describe() const {
    cse_loss l = DescribeLoss(rho);
    l.scaled = 1;
    l.scale = a;
    return l;
  }
  LossFunctionCUDA rho;
  double a;
};

// The loss the kernels are compiled for: ScaledLossCUDA<L> applies L's rho
// and scales at run time (cse_loss.scaled), so its kernels are L's.
template <typename L>
struct BaseLoss {
  using type = L;
};
template <typename L>
struct BaseLoss<ScaledLossCUDA<L>> {
  using type = typename BaseLoss<L>::type;
};

// ---------------------------------------------------------------------------
// Residual functors available as gfx950 kernels.  Each carries its kind and
// the per-block constants the kernel needs (its "functor data").
// ---------------------------------------------------------------------------
struct SnavelyReprojectionError {  // examples/snavely_reprojection_error.h:54-105
  static constexpr cse_functor_kind kKind = CSE_FUNCTOR_SNAVELY_2_9_3;
  SnavelyReprojectionError(double observed_x, double observed_y)
      : observed_x(observed_x), observed_y(observed_y) {}
  void Pack(double* out) const { out[0] = observed_x; out[1] = observed_y; }
  double observed_x, observed_y;
};
struct SnavelyReprojectionErrorWithQuaternions {  // ibid. :112-175
  static constexpr cse_functor_kind kKind = CSE_FUNCTOR_SNAVELY_QUATERNION_2_10_3;
  SnavelyReprojectionErrorWithQuaternions(double observed_x, double observed_y)
      : observed_x(observed_x), observed_y(observed_y) {}
  void Pack(double* out) const { out[0] = observed_x; out[1] = observed_y; }
  double observed_x, observed_y;
};
struct SnavelyReprojectionErrorNoRadialDistortion {  // evaluator_cuda_test.cu.cc:112-150
  static constexpr cse_functor_kind kKind = CSE_FUNCTOR_SNAVELY_NO_DISTORTION_2_7_3;
  SnavelyReprojectionErrorNoRadialDistortion(double observed_x, double observed_y)
      : observed_x(observed_x), observed_y(observed_y) {}
  void Pack(double* out) const { out[0] = observed_x; out[1] = observed_y; }
  double observed_x, observed_y;
};
struct PointDisplacementError {  // evaluator_cuda_test.cu.cc:84-110
  static constexpr cse_functor_kind kKind = CSE_FUNCTOR_POINT_DISPLACEMENT_3_3;
  PointDisplacementError(double x, double y, double z) : x_(x), y_(y), z_(z) {}
  void Pack(double* out) const { out[0] = x_; out[1] = y_; out[2] = z_; }
  double x_, y_, z_;
};

// Shape of each kind, checked against the template arguments of
// AddResidualBlock<F, kNumResiduals, Ns...>.
template <typename F> struct FunctorShape;
// A functor type the library has pre-instantiated (it carries kKind).
template <typename F, typename = void>
struct IsLibraryFunctor : std::false_type {};
template <typename F>
struct IsLibraryFunctor<F, decltype((void)F::kKind)> : std::true_type {};
template <typename L>
constexpr bool kIsLibraryLoss = HasDescribe<typename BaseLoss<L>::type>::value;

// The functor kind of a user functor type with loss type L: defined by
// ceres_amd/autodiff_cuda.h (hipcc TUs only), which instantiates and
// registers the kernels (cse_register_functor) on first use.  A TU without
// that header can add residual blocks of the library's kinds only.
template <typename F, typename L, int kNumResiduals, int... Ns>
struct UserFunctorKind;

// AutoDiffCostFunction<F, kNumResiduals, Ns...> (include/ceres/
// autodiff_cost_function.h): owns the functor; ProblemCUDA::AddResidualBlock
// takes it as the reference's takes its CostFunction* (problem_cuda.h:
// 443-450) and owns it afterwards.
template <typename CostFunctor, int kNumResiduals, int... Ns>
class AutoDiffCostFunction {
 public:
  explicit AutoDiffCostFunction(CostFunctor* functor) : functor_(functor) {}
  const CostFunctor& functor() const { return *functor_; }

 private:
  std::unique_ptr<CostFunctor> functor_;
};
template <> struct FunctorShape<SnavelyReprojectionError> {
  static constexpr int kR = 2, kData = 2; static constexpr int kSizes[2] = {9, 3}; static constexpr int kNb = 2;
};
template <> struct FunctorShape<SnavelyReprojectionErrorWithQuaternions> {
  static constexpr int kR = 2, kData = 2; static constexpr int kSizes[2] = {10, 3}; static constexpr int kNb = 2;
};
template <> struct FunctorShape<SnavelyReprojectionErrorNoRadialDistortion> {
  static constexpr int kR = 2, kData = 2; static constexpr int kSizes[2] = {7, 3}; static constexpr int kNb = 2;
};
template <> struct FunctorShape<PointDisplacementError> {
  static constexpr int kR = 3, kData = 3; static constexpr int kSizes[2] = {3, 0}; static constexpr int kNb = 1;
};

// ---------------------------------------------------------------------------
// Manifolds, described by their PlusJacobian (ambient x tangent, row-major).
// ---------------------------------------------------------------------------
class Manifold {
 public:
  virtual ~Manifold() = default;
  virtual int AmbientSize() const = 0;
  virtual int TangentSize() const = 0;
  virtual void PlusJacobian(const double* x, double* jacobian) const = 0;
  // cse_manifold_kind the library can build on the device from the block's
  // value; CSE_MANIFOLD_MATRIX = upload PlusJacobian every evaluation.
  virtual int DeviceKind() const { return CSE_MANIFOLD_MATRIX; }
};

template <int N>
class EuclideanManifold : public Manifold {
 public:
  int AmbientSize() const override { return N; }
  int TangentSize() const override { return N; }
  void PlusJacobian(const double*, double* J) const override {
    for (int r = 0; r < N; ++r)
      for (int c = 0; c < N; ++c) J[r * N + c] = r == c ? 1.0 : 0.0;
  }
};

// QuaternionManifold (Ceres order w, x, y, z): internal/ceres/manifold.cc:63-80.
class QuaternionManifold : public Manifold {
 public:
  int AmbientSize() const override { return 4; }
  int TangentSize() const override { return 3; }
  void PlusJacobian(const double* x, double* J) const override {
    const double j[12] = {-x[1], -x[2], -x[3], x[0],  x[3], -x[2],
                          -x[3], x[0],  x[1],  x[2], -x[1], x[0]};
    std::memcpy(J, j, sizeof(j));
  }
};

// SubsetManifold: holds the listed coordinates constant.
class SubsetManifold : public Manifold {
 public:
  SubsetManifold(int size, const std::vector<int>& constant) : size_(size), keep_() {
    std::vector<bool> c(size, false);
    for (int k : constant) c.at(k) = true;
    for (int k = 0; k < size; ++k)
      if (!c[k]) keep_.push_back(k);
  }
  int AmbientSize() const override { return size_; }
  int TangentSize() const override { return (int)keep_.size(); }
  void PlusJacobian(const double*, double* J) const override {
    const int t = TangentSize();
    std::fill(J, J + size_ * t, 0.0);
    for (int c = 0; c < t; ++c) J[keep_[c] * t + c] = 1.0;
  }

 private:
  int size_;
  std::vector<int> keep_;
};

template <typename M>
struct IsEuclideanManifold : std::false_type {};
template <int N>
struct IsEuclideanManifold<EuclideanManifold<N>> : std::true_type {};

// ProductManifold<M1, M2>: block-diagonal plus-Jacobian.
template <typename M1, typename M2>
class ProductManifold : public Manifold {
 public:
  // ProductManifold<QuaternionManifold, EuclideanManifold<n>> (the
  // --use_quaternions --use_manifolds camera): built on the device.
  int DeviceKind() const override {
    return std::is_same<M1, QuaternionManifold>::value && IsEuclideanManifold<M2>::value
               ? CSE_MANIFOLD_QUATERNION_EUCLIDEAN
               : CSE_MANIFOLD_MATRIX;
  }
  int AmbientSize() const override { return m1_.AmbientSize() + m2_.AmbientSize(); }
  int TangentSize() const override { return m1_.TangentSize() + m2_.TangentSize(); }
  void PlusJacobian(const double* x, double* J) const override {
    const int a1 = m1_.AmbientSize(), t1 = m1_.TangentSize();
    const int a2 = m2_.AmbientSize(), t2 = m2_.TangentSize(), T = t1 + t2;
    std::vector<double> J1(a1 * t1), J2(a2 * t2);
    m1_.PlusJacobian(x, J1.data());
    m2_.PlusJacobian(x + a1, J2.data());
    std::fill(J, J + (a1 + a2) * T, 0.0);
    for (int r = 0; r < a1; ++r)
      for (int c = 0; c < t1; ++c) J[r * T + c] = J1[r * t1 + c];
    for (int r = 0; r < a2; ++r)
      for (int c = 0; c < t2; ++c) J[(a1 + r) * T + t1 + c] = J2[r * t2 + c];
  }

 private:
  M1 m1_;
  M2 m2_;
};

using ResidualBlockId = int64_t;

enum class JacobianFormat { kBlockSparse, kCompressedRow };

class EvaluatorCUDA;

// ---------------------------------------------------------------------------
// ProblemCUDA (include/ceres/problem_cuda.h:85-486).
// ---------------------------------------------------------------------------
class ProblemCUDA {
 public:
  ProblemCUDA() = default;
  ProblemCUDA(const ProblemCUDA&) = delete;
  ProblemCUDA& operator=(const ProblemCUDA&) = delete;

  // Problem::AddParameterBlock: repeated calls with the same pointer are ignored.
  void AddParameterBlock(double* values, int size) { Block(values, size); }
  void AddParameterBlock(double* values, int size, const Manifold* manifold) {
    Block(values, size);
    SetManifold(values, manifold);
  }

  template <typename CostFunctor, int kNumResiduals, int... Ns, typename LossFunctionCUDA,
            typename... Ts>
  ResidualBlockId AddResidualBlock(const CostFunctor& functor, const LossFunctionCUDA* loss,
                                   double* x0, Ts*... xs) {
    static_assert(sizeof...(Ts) + 1 == sizeof...(Ns), "one pointer per parameter block");
    static_assert(kNumResiduals >= 1, "the number of residuals must be static");
    constexpr int sizes[] = {Ns...};
    double* ptrs[] = {x0, xs...};
    Residual res;
    res.nres = kNumResiduals;
    if constexpr (IsLibraryFunctor<CostFunctor>::value && kIsLibraryLoss<LossFunctionCUDA>) {
      // A kind pre-instantiated in libcse.so.
      using S = FunctorShape<CostFunctor>;
      static_assert(S::kR == kNumResiduals, "kNumResiduals does not match the functor");
      static_assert(sizeof...(Ns) == S::kNb, "parameter block count does not match the functor");
      for (int j = 0; j < S::kNb; ++j)
        if (sizes[j] != S::kSizes[j]) throw std::invalid_argument("parameter block size mismatch");
      res.kind = CostFunctor::kKind;
      res.data.resize(S::kData);
      functor.Pack(res.data.data());
    } else {
      // Any other functor (or a library functor with a user loss): its
      // kernels are instantiated in this TU (ceres_amd/autodiff_cuda.h).
      // (An incomplete UserFunctorKind here means this TU lacks
      // ceres_amd/autodiff_cuda.h, or is not compiled with hipcc.)
      static_assert(!IsLibraryFunctor<CostFunctor>::value,
                    "the library's functor kinds take the library's losses");
      using U = UserFunctorKind<CostFunctor, typename BaseLoss<LossFunctionCUDA>::type,
                                kNumResiduals, Ns...>;
      res.kind = (cse_functor_kind)U::Kind();
      res.data.assign(U::kDataSize, 0.0);
      std::memcpy(res.data.data(), &functor, sizeof(CostFunctor));
    }
    res.loss = loss ? DescribeLoss(*loss) : TrivialLossCUDA().Describe();
    for (int j = 0; j < (int)sizeof...(Ns); ++j) res.blocks.push_back(Block(ptrs[j], sizes[j]));
    residuals_.push_back(std::move(res));
    return (ResidualBlockId)residuals_.size() - 1;
  }

  // The reference's form (problem_cuda.h:110-144): a cost function wrapping
  // the functor; the problem takes ownership of it.
  template <typename CostFunctor, int kNumResiduals, int... Ns, typename LossFunctionCUDA,
            typename... Ts>
  ResidualBlockId AddResidualBlock(AutoDiffCostFunction<CostFunctor, kNumResiduals, Ns...>* cost,
                                   const LossFunctionCUDA* loss, double* x0, Ts*... xs) {
    cost_functions_.emplace_back(cost, [](void* p) {
      delete static_cast<AutoDiffCostFunction<CostFunctor, kNumResiduals, Ns...>*>(p);
    });
    return AddResidualBlock<CostFunctor, kNumResiduals, Ns...>(cost->functor(), loss, x0, xs...);
  }
  template <typename CostFunctor, int kNumResiduals, int... Ns, typename... Ts>
  ResidualBlockId AddResidualBlock(AutoDiffCostFunction<CostFunctor, kNumResiduals, Ns...>* cost,
                                   std::nullptr_t, double* x0, Ts*... xs) {
    return AddResidualBlock<CostFunctor, kNumResiduals, Ns...>(
        cost, static_cast<const TrivialLossCUDA*>(nullptr), x0, xs...);
  }

  // nullptr loss = TrivialLossCUDA (problem_cuda.h:146-160).
  template <typename CostFunctor, int kNumResiduals, int... Ns, typename... Ts>
  ResidualBlockId AddResidualBlock(const CostFunctor& functor, std::nullptr_t, double* x0,
                                   Ts*... xs) {
    return AddResidualBlock<CostFunctor, kNumResiduals, Ns...>(
        functor, static_cast<const TrivialLossCUDA*>(nullptr), x0, xs...);
  }

  void SetParameterBlockConstant(const double* values) { At(values).constant = true; }
  void SetParameterBlockVariable(double* values) { At(values).constant = false; }
  bool IsParameterBlockConstant(const double* values) const { return At(values).constant; }
  void SetManifold(double* values, const Manifold* manifold) {
    Param& p = At(values);
    if (manifold && manifold->AmbientSize() != p.size)
      throw std::invalid_argument("manifold ambient size does not match the block");
    p.manifold = manifold;
  }
  bool HasManifold(const double* values) const { return At(values).manifold != nullptr; }

  int NumParameterBlocks() const { return (int)params_.size(); }
  int NumResidualBlocks() const { return (int)residuals_.size(); }
  int NumParameters() const {
    int n = 0;
    for (auto& p : params_) n += p.size;
    return n;
  }
  int NumResiduals() const {
    int n = 0;
    for (auto& r : residuals_) n += r.nres;
    return n;
  }
  int ParameterBlockSize(const double* values) const { return At(values).size; }
  int ParameterBlockTangentSize(const double* values) const {
    const Param& p = At(values);
    return p.manifold ? p.manifold->TangentSize() : p.size;
  }

  // Points-first (Schur) ordering, like bundle_adjuster's SetOrdering with
  // points in elimination group 0: the listed blocks come first in the
  // program and are the E blocks of the BlockSparseMatrix.
  void SetEliminationGroup(const std::vector<double*>& first) { elimination_ = first; }

 private:
  friend class EvaluatorCUDA;
  struct Param {
    double* values;
    int size;
    bool constant = false;
    const Manifold* manifold = nullptr;
  };
  struct Residual {
    cse_functor_kind kind;
    cse_loss loss;
    int nres;
    std::vector<int> blocks;
    std::vector<double> data;
  };
  int Block(double* values, int size) {
    auto it = index_.find(values);
    if (it != index_.end()) {
      if (params_[it->second].size != size)
        throw std::invalid_argument("parameter block re-added with a different size");
      return it->second;
    }
    params_.push_back(Param{values, size});
    index_[values] = (int)params_.size() - 1;
    return (int)params_.size() - 1;
  }
  Param& At(const double* v) {
    auto it = index_.find(const_cast<double*>(v));
    if (it == index_.end()) throw std::invalid_argument("unknown parameter block");
    return params_[it->second];
  }
  const Param& At(const double* v) const {
    auto it = index_.find(const_cast<double*>(v));
    if (it == index_.end()) throw std::invalid_argument("unknown parameter block");
    return params_[it->second];
  }
  std::vector<Param> params_;
  std::map<double*, int> index_;
  std::vector<Residual> residuals_;
  std::vector<double*> elimination_;
  std::vector<std::unique_ptr<void, void (*)(void*)>> cost_functions_;
};

// ---------------------------------------------------------------------------
// EvaluatorCUDA: the reduced Program of a ProblemCUDA plus the gfx950
// evaluator (ProgramEvaluatorCUDA, program_evaluator_cuda.h:65-183).
// ---------------------------------------------------------------------------
class EvaluatorCUDA {
 public:
  struct Options {
    JacobianFormat format = JacobianFormat::kBlockSparse;
    int device = -1;
    bool check_finite = true;
    bool apply_loss_function = true;
    // Let the library build the plus-Jacobians it knows (Manifold::DeviceKind)
    // instead of uploading them every evaluation.
    bool device_manifolds = true;
  };

  EvaluatorCUDA(ProblemCUDA& problem, const Options& options) : problem_(problem) {
    Build(options);
  }
  ~EvaluatorCUDA() {
    if (ev_) cse_destroy(ev_);
  }
  EvaluatorCUDA(const EvaluatorCUDA&) = delete;
  EvaluatorCUDA& operator=(const EvaluatorCUDA&) = delete;

  int NumParameters() const { return (int)num_parameters_; }
  int NumEffectiveParameters() const { return (int)num_effective_; }
  int NumResiduals() const { return (int)num_residuals_; }
  int NumResidualBlocks() const { return (int)program_residuals_.size(); }
  int64_t NumJacobianValues() const { return num_jacobian_values_; }
  // CompressedRowSparseMatrix structure (format kCompressedRow only).
  const std::vector<int64_t>& crs_rows() const { return crs_rows_; }
  const std::vector<int64_t>& crs_cols() const { return crs_cols_; }

  // Program::ParameterBlocksToStateVector / StateVectorToParameterBlocks.
  void ParameterBlocksToStateVector(double* state) const {
    for (size_t k = 0; k < order_.size(); ++k) {
      const auto& p = problem_.params_[order_[k]];
      if (!p.constant) std::memcpy(state + state_offset_[k], p.values, sizeof(double) * p.size);
    }
  }
  void StateVectorToParameterBlocks(const double* state) {
    for (size_t k = 0; k < order_.size(); ++k) {
      auto& p = problem_.params_[order_[k]];
      if (!p.constant) std::memcpy(p.values, state + state_offset_[k], sizeof(double) * p.size);
    }
  }

  // Evaluator::Evaluate (internal/ceres/evaluator.h:61-170) through
  // RegisteredCUDAEvaluators::Evaluate's seam: any output may be nullptr.
  // Returns false when a residual block failed (non-finite output).
  bool Evaluate(const double* state, double* cost, double* residuals, double* gradient,
                double* jacobian_values) {
    if (num_plus_jacobian_values_ > 0) {
      RefreshPlusJacobians(state);
      Check(cse_set_plus_jacobians(ev_, plus_jacobians_.data()), "cse_set_plus_jacobians");
    }
    const int rc = cse_evaluate(ev_, state, cost, residuals, gradient, jacobian_values);
    if (rc < 0) Check(rc, "cse_evaluate");
    return rc == CSE_OK;
  }

  cse_evaluator* handle() { return ev_; }

 private:
  static void Check(int rc, const char* what) {
    if (rc < 0) throw std::runtime_error(std::string(what) + ": " + cse_last_error());
  }

  void Build(const Options& o) {
    auto& P = problem_.params_;
    // Program order: the elimination group first, then insertion order.
    std::vector<int> order;
    std::vector<bool> placed(P.size(), false);
    for (double* v : problem_.elimination_) {
      const int i = problem_.index_.at(v);
      if (!placed[i]) order.push_back(i), placed[i] = true;
    }
    const int num_eliminate = (int)order.size();
    for (size_t i = 0; i < P.size(); ++i)
      if (!placed[i]) order.push_back((int)i);
    order_ = order;
    std::vector<int> program_index(P.size());
    for (size_t k = 0; k < order.size(); ++k) program_index[order[k]] = (int)k;

    // Offsets (Program::SetParameterOffsetsAndIndex, program.cc:151-177).
    pbs_.resize(order.size());
    state_offset_.resize(order.size());
    int64_t so = 0, dof = 0, cso = 0;
    for (size_t k = 0; k < order.size(); ++k) {
      const auto& p = P[order[k]];
      cse_parameter_block& b = pbs_[k];
      b.size = p.size;
      b.tangent_size = p.manifold ? p.manifold->TangentSize() : p.size;
      b.is_constant = p.constant;
      b.manifold = p.manifold && o.device_manifolds ? p.manifold->DeviceKind() : CSE_MANIFOLD_MATRIX;
      b.plus_jacobian_offset = -1;
      if (p.constant) {
        b.state_offset = cso;
        b.delta_offset = 0;
        for (int q = 0; q < p.size; ++q) constant_state_.push_back(p.values[q]);
        cso += p.size;
      } else {
        b.state_offset = so;
        b.delta_offset = dof;
        so += p.size;
        dof += b.tangent_size;
        if (p.manifold && b.manifold == CSE_MANIFOLD_MATRIX) {
          b.plus_jacobian_offset = num_plus_jacobian_values_;
          num_plus_jacobian_values_ += (int64_t)p.size * b.tangent_size;
        }
      }
      state_offset_[k] = b.state_offset;
    }
    num_parameters_ = so;
    num_effective_ = dof;
    plus_jacobians_.assign(num_plus_jacobian_values_, 0.0);

    // Reduced program: residual blocks with at least one active block
    // (Program::CreateReducedProgram), in insertion order.
    for (size_t r = 0; r < problem_.residuals_.size(); ++r) {
      bool live = false;
      for (int b : problem_.residuals_[r].blocks) live = live || !P[b].constant;
      if (live) program_residuals_.push_back((int)r);
    }
    const int64_t nrb = (int64_t)program_residuals_.size();
    std::vector<int64_t> begin(nrb + 1, 0);
    std::vector<int32_t> ids, nres(nrb);
    for (int64_t i = 0; i < nrb; ++i) {
      const auto& R = problem_.residuals_[program_residuals_[i]];
      for (int b : R.blocks) ids.push_back(program_index[b]);
      begin[i + 1] = (int64_t)ids.size();
      nres[i] = R.nres;
      num_residuals_ += R.nres;
    }
    const int64_t npb = (int64_t)pbs_.size();
    const int64_t count =
        cse_layout_offsets_count(npb, pbs_.data(), nrb, begin.data(), ids.data(), nres.data());
    residual_layout_.resize(nrb);
    jac_layout_.resize(nrb);
    jac_offsets_.resize(std::max<int64_t>(count, 1));
    if (o.format == JacobianFormat::kBlockSparse) {
      Check(cse_block_sparse_layout(npb, pbs_.data(), nrb, begin.data(), ids.data(), nres.data(),
                                    num_eliminate, residual_layout_.data(), jac_layout_.data(),
                                    jac_offsets_.data(), &num_jacobian_values_),
            "cse_block_sparse_layout");
    } else {
      crs_rows_.resize(num_residuals_ + 1);
      // Values count first, then columns.
      Check(cse_compressed_row_layout(npb, pbs_.data(), nrb, begin.data(), ids.data(), nres.data(),
                                      residual_layout_.data(), jac_layout_.data(),
                                      jac_offsets_.data(), &num_jacobian_values_, crs_rows_.data(),
                                      nullptr),
            "cse_compressed_row_layout");
      crs_cols_.resize(num_jacobian_values_);
      Check(cse_compressed_row_layout(npb, pbs_.data(), nrb, begin.data(), ids.data(), nres.data(),
                                      residual_layout_.data(), jac_layout_.data(),
                                      jac_offsets_.data(), &num_jacobian_values_, crs_rows_.data(),
                                      crs_cols_.data()),
            "cse_compressed_row_layout");
    }

    // One group per (functor kind, loss): the per-type evaluator registry
    // (problem_cuda.h:462-468, registered_cuda_evaluators.cc:294-298).
    using UserBytes = std::array<double, CSE_USER_LOSS_BYTES / 8>;
    std::map<std::tuple<int, int, double, int, double, UserBytes>, GroupStorage> groups;
    for (int64_t i = 0; i < nrb; ++i) {
      const auto& R = problem_.residuals_[program_residuals_[i]];
      UserBytes ub;
      std::memcpy(ub.data(), R.loss.user, sizeof(ub));
      auto key = std::make_tuple((int)R.kind, R.loss.kind, R.loss.a, R.loss.scaled, R.loss.scale, ub);
      GroupStorage& g = groups[key];
      g.g.functor_kind = R.kind;
      g.g.loss = R.loss;
      g.index.push_back(i);
      for (int b : R.blocks) g.ids.push_back(program_index[b]);
      g.data.insert(g.data.end(), R.data.begin(), R.data.end());
    }
    for (auto& kv : groups) group_storage_.push_back(std::move(kv.second));
    std::vector<cse_residual_group> gs;
    for (auto& g : group_storage_) {
      g.g.reserved = 0;
      g.g.num_blocks = (int64_t)g.index.size();
      g.g.residual_block_index = g.index.data();
      g.g.first_residual_block = 0;
      g.g.parameter_block_ids = g.ids.data();
      g.g.functor_data = g.data.data();
      gs.push_back(g.g);
    }
    cse_problem_desc d{};
    d.abi_version = CSE_ABI_VERSION;
    d.num_groups = (int32_t)gs.size();
    d.groups = gs.data();
    d.num_parameter_blocks = npb;
    d.parameter_blocks = pbs_.data();
    d.num_parameters = num_parameters_;
    d.num_effective_parameters = num_effective_;
    d.num_constant_parameters = cso;
    d.constant_state = constant_state_.data();
    d.num_plus_jacobian_values = num_plus_jacobian_values_;
    d.plus_jacobians = plus_jacobians_.data();
    d.num_residual_blocks = nrb;
    d.num_residuals = num_residuals_;
    d.residual_layout = residual_layout_.data();
    d.jacobian_per_residual_layout = jac_layout_.data();
    d.jacobian_per_residual_offsets = jac_offsets_.data();
    d.num_jacobian_per_residual_offsets = count;
    d.num_jacobian_values = num_jacobian_values_;
    cse_options opts;
    cse_default_options(&opts);
    opts.device = o.device;
    opts.check_finite = o.check_finite;
    opts.apply_loss_function = o.apply_loss_function;
    Check(cse_create(&d, &opts, &ev_), "cse_create");
  }

  // RegisteredCUDAEvaluators::UpdatePlusJacobians: the plus-Jacobian of
  // every manifold block at the current state.
  void RefreshPlusJacobians(const double* state) {
    for (size_t k = 0; k < order_.size(); ++k) {
      const auto& p = problem_.params_[order_[k]];
      if (p.constant || !p.manifold || pbs_[k].plus_jacobian_offset < 0) continue;
      p.manifold->PlusJacobian(state + state_offset_[k],
                               plus_jacobians_.data() + pbs_[k].plus_jacobian_offset);
    }
  }

  struct GroupStorage {
    cse_residual_group g;
    std::vector<int64_t> index;
    std::vector<int32_t> ids;
    std::vector<double> data;
  };
  ProblemCUDA& problem_;
  cse_evaluator* ev_ = nullptr;
  std::vector<int> order_;
  std::vector<int64_t> state_offset_;
  std::vector<cse_parameter_block> pbs_;
  std::vector<double> constant_state_;
  std::vector<double> plus_jacobians_;
  int64_t num_plus_jacobian_values_ = 0;
  int64_t num_parameters_ = 0, num_effective_ = 0, num_residuals_ = 0, num_jacobian_values_ = 0;
  std::vector<int> program_residuals_;
  std::vector<int64_t> residual_layout_, jac_layout_, jac_offsets_, crs_rows_, crs_cols_;
  std::vector<GroupStorage> group_storage_;
};

}  // namespace ceres_amd

#endif  // CERES_AMD_PROBLEM_CUDA_H_
