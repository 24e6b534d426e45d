// loss.hpp -- robust losses and the Triggs correction, fused into the
// evaluate kernel.
//
// Losses: include/ceres/loss_function_cuda.h:62-150 (Trivial, Huber,
// Cauchy, Scaled).  Correction: include/ceres/internal/corrector.h:82-213.
#ifndef CSE_LOSS_HPP_
#define CSE_LOSS_HPP_

#include <cfloat>
#include <type_traits>

#include "jet.hpp"

namespace cse {

// kLossUser: a LossFunctionCUDA type compiled into a user-registered
// functor kind (include/ceres_amd/autodiff_cuda.h); its state travels as
// kUserLossDoubles doubles of bytes (GroupArgs::user_loss).
enum LossKind { kLossTrivial = 0, kLossHuber = 1, kLossCauchy = 2, kLossUser = 3 };
constexpr int kUserLossDoubles = 8;

// The loss type a kind carries for kLossUser (K::UserLoss), else void.
template <class K, class = void>
struct UserLossOf {
  using type = void;
};
template <class K>
struct UserLossOf<K, decltype((void)sizeof(typename K::UserLoss))> {
  using type = typename K::UserLoss;
};

struct LossParams {
  double a;
  double scale;
  int scaled;
};

// rho(s) = (rho0, rho1, rho2).  kLossUser: K's UserLoss object, rebuilt
// from its bytes (user), evaluates rho (its Evaluate(s, rho), the
// LossFunctionCUDA contract of include/ceres/loss_function_cuda.h:62-94).
template <int kLoss, class K = void>
CSE_HD void EvaluateLoss(const LossParams& lp, double s, double rho[3],
                         const double* user = nullptr) {
  if constexpr (kLoss == kLossUser) {
    using UL = typename UserLossOf<K>::type;
    static_assert(!std::is_void<UL>::value, "kLossUser needs a kind with a UserLoss type");
    static_assert(sizeof(UL) <= kUserLossDoubles * sizeof(double), "user loss too large");
    alignas(UL) unsigned char buf[sizeof(UL)];
    __builtin_memcpy(buf, user, sizeof(UL));
    reinterpret_cast<const UL*>(buf)->Evaluate(s, rho);
  } else if constexpr (kLoss == kLossHuber) {
    const double a = lp.a, b = a * a;
    if (s > b) {
      // loss_function_cuda.h:72-87 with one division: 1/r serves rho1 and
      // rho2 = -rho1 / (2 s) = -0.5 rho1 / r^2.
      const double r = sqrt(s);
      const double r_inv = 1.0 / r;
      rho[0] = 2.0 * a * r - b;
      rho[1] = fmax(DBL_MIN, a * r_inv);
      rho[2] = -0.5 * rho[1] * (r_inv * r_inv);
    } else {
      rho[0] = s;
      rho[1] = 1.0;
      rho[2] = 0.0;
    }
  } else if constexpr (kLoss == kLossCauchy) {
    const double b = lp.a * lp.a;
    const double c = 1.0 / b;
    const double sum = 1.0 + s * c;
    const double inv = 1.0 / sum;
    rho[0] = b * log(sum);
    rho[1] = fmax(DBL_MIN, inv);
    rho[2] = -c * (inv * inv);
  } else {
    rho[0] = s;
    rho[1] = 1.0;
    rho[2] = 0.0;
  }
  if (lp.scaled) {
    rho[0] *= lp.scale;
    rho[1] *= lp.scale;
    rho[2] *= lp.scale;
  }
}

// Corrector: residuals *= sqrt(rho1)/(1-alpha); J = sqrt(rho1) (J -
// alpha/|r|^2 r r^T J) where alpha solves 0.5 a^2 - a - rho2/rho1 |r|^2 = 0.
// With rho2 <= 0 (every Huber outlier, every Cauchy point) alpha = 0 and
// both reduce to scaling by sqrt(rho1).
struct Corrector {
  double sqrt_rho1;
  double residual_scaling;
  double alpha_sq_norm;

  CSE_HD Corrector(double sq_norm, const double rho[3]) {
    sqrt_rho1 = sqrt(rho[1]);
    if (sq_norm == 0.0 || rho[2] <= 0.0) {
      residual_scaling = sqrt_rho1;
      alpha_sq_norm = 0.0;
    } else {
      const double D = 1.0 + 2.0 * sq_norm * rho[2] / rho[1];
      const double alpha = 1.0 - sqrt(D);
      residual_scaling = sqrt_rho1 / (1.0 - alpha);
      alpha_sq_norm = alpha / sq_norm;
    }
  }

  // J is kR x kCols row-major, corrected in place; r is uncorrected.
  template <int kR, int kCols>
  CSE_HD void CorrectJacobian(const double* r, double* J) const {
    if (alpha_sq_norm == 0.0) {
#pragma unroll
      for (int i = 0; i < kR * kCols; ++i) J[i] *= sqrt_rho1;
      return;
    }
#pragma unroll
    for (int c = 0; c < kCols; ++c) {
      double rtj = 0.0;
#pragma unroll
      for (int k = 0; k < kR; ++k) rtj += J[k * kCols + c] * r[k];
#pragma unroll
      for (int k = 0; k < kR; ++k)
        J[k * kCols + c] = sqrt_rho1 * (J[k * kCols + c] - alpha_sq_norm * r[k] * rtj);
    }
  }

  template <int kR>
  CSE_HD void CorrectResiduals(double* r) const {
#pragma unroll
    for (int k = 0; k < kR; ++k) r[k] *= residual_scaling;
  }
};

}  // namespace cse

#endif  // CSE_LOSS_HPP_
