// oracle.cpp -- CPU restatement of Ceres' ProgramEvaluator for the
// AutoDiffCostFunction residual blocks that ProblemCUDA registers.
//
// TEST INFRASTRUCTURE ONLY (see oracle.h).  Written from the reference's
// behaviour, not copied: every function cites the file:line it restates.
// Compiled with -ffp-contract=off so the arithmetic is the plain IEEE
// sequence the reference's host build (x86-64, no FMA) performs.

#include "oracle.h"

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <limits>
#include <thread>
#include <utility>
#include <vector>

namespace oracle {

// ---------------------------------------------------------------------------
// Jet<double, N>: include/ceres/jet.h:222-305 (struct), 309-402 (operators),
// 533-575 (abs/copysign), 617-641 (sqrt/cos/sin), 742-760 (hypot).
// ---------------------------------------------------------------------------
template <int N>
struct Jet {
  double a;
  double v[N];
  Jet() : a(0.0) { for (int i = 0; i < N; ++i) v[i] = 0.0; }
  explicit Jet(double value) : a(value) { for (int i = 0; i < N; ++i) v[i] = 0.0; }
  // jet.h:247-252: a = value, v = unit vector k.
  Jet(double value, int k) : a(value) {
    for (int i = 0; i < N; ++i) v[i] = 0.0;
    v[k] = 1.0;
  }
};

template <int N> Jet<N> operator-(const Jet<N>& f) {          // jet.h:318-321
  Jet<N> r; r.a = -f.a;
  for (int i = 0; i < N; ++i) r.v[i] = -f.v[i];
  return r;
}
template <int N> Jet<N> operator+(const Jet<N>& f, const Jet<N>& g) {  // :324-327
  Jet<N> r; r.a = f.a + g.a;
  for (int i = 0; i < N; ++i) r.v[i] = f.v[i] + g.v[i];
  return r;
}
template <int N> Jet<N> operator+(const Jet<N>& f, double s) {  // :330-333
  Jet<N> r = f; r.a = f.a + s; return r;
}
template <int N> Jet<N> operator+(double s, const Jet<N>& f) {  // :336-339
  Jet<N> r = f; r.a = f.a + s; return r;
}
template <int N> Jet<N> operator-(const Jet<N>& f, const Jet<N>& g) {  // :342-345
  Jet<N> r; r.a = f.a - g.a;
  for (int i = 0; i < N; ++i) r.v[i] = f.v[i] - g.v[i];
  return r;
}
template <int N> Jet<N> operator-(const Jet<N>& f, double s) {  // :348-351
  Jet<N> r = f; r.a = f.a - s; return r;
}
template <int N> Jet<N> operator-(double s, const Jet<N>& f) {  // :354-357
  Jet<N> r; r.a = s - f.a;
  for (int i = 0; i < N; ++i) r.v[i] = -f.v[i];
  return r;
}
template <int N> Jet<N> operator*(const Jet<N>& f, const Jet<N>& g) {  // :360-363
  Jet<N> r; r.a = f.a * g.a;
  for (int i = 0; i < N; ++i) r.v[i] = f.a * g.v[i] + f.v[i] * g.a;
  return r;
}
template <int N> Jet<N> operator*(const Jet<N>& f, double s) {  // :366-369
  Jet<N> r; r.a = f.a * s;
  for (int i = 0; i < N; ++i) r.v[i] = f.v[i] * s;
  return r;
}
template <int N> Jet<N> operator*(double s, const Jet<N>& f) {  // :372-375
  return f * s;
}
template <int N> Jet<N> operator/(const Jet<N>& f, const Jet<N>& g) {  // :378-390
  const double g_a_inverse = 1.0 / g.a;
  const double f_a_by_g_a = f.a * g_a_inverse;
  Jet<N> r; r.a = f_a_by_g_a;
  for (int i = 0; i < N; ++i) r.v[i] = (f.v[i] - f_a_by_g_a * g.v[i]) * g_a_inverse;
  return r;
}
template <int N> Jet<N> operator/(double s, const Jet<N>& g) {  // :393-397
  const double minus_s_g_a_inverse2 = -s / (g.a * g.a);
  Jet<N> r; r.a = s / g.a;
  for (int i = 0; i < N; ++i) r.v[i] = g.v[i] * minus_s_g_a_inverse2;
  return r;
}
template <int N> Jet<N> operator/(const Jet<N>& f, double s) {  // :400-404
  const double s_inverse = 1.0 / s;
  return f * s_inverse;
}
template <int N> Jet<N> jsqrt(const Jet<N>& f) {  // jet.h:622-627
  const double tmp = std::sqrt(f.a);
  const double two_a_inverse = 1.0 / (2.0 * tmp);
  Jet<N> r; r.a = tmp;
  for (int i = 0; i < N; ++i) r.v[i] = f.v[i] * two_a_inverse;
  return r;
}
template <int N> Jet<N> jcos(const Jet<N>& f) {  // jet.h:630-633
  Jet<N> r; r.a = std::cos(f.a);
  const double m = -std::sin(f.a);
  for (int i = 0; i < N; ++i) r.v[i] = m * f.v[i];
  return r;
}
template <int N> Jet<N> jsin(const Jet<N>& f) {  // jet.h:643-646
  Jet<N> r; r.a = std::sin(f.a);
  const double c = std::cos(f.a);
  for (int i = 0; i < N; ++i) r.v[i] = c * f.v[i];
  return r;
}
template <int N> Jet<N> jabs(const Jet<N>& f) {  // jet.h:533-537
  Jet<N> r; r.a = std::fabs(f.a);
  const double s = std::copysign(1.0, f.a);
  for (int i = 0; i < N; ++i) r.v[i] = s * f.v[i];
  return r;
}
// Three-argument hypot (jet.h:742-760).  The host build of the reference
// uses std::hypot for the value (rotation.h:832-835 selects std:: off-device).
template <int N> Jet<N> jhypot(const Jet<N>& x, const Jet<N>& y, const Jet<N>& z) {
  const double tmp = std::hypot(x.a, y.a, z.a);
  const double cx = x.a / tmp, cy = y.a / tmp, cz = z.a / tmp;
  Jet<N> r; r.a = tmp;
  for (int i = 0; i < N; ++i) r.v[i] = cx * x.v[i] + cy * y.v[i] + cz * z.v[i];
  return r;
}

// Scalar overloads so the functors below are written once for T in
// {double, Jet<N>} exactly like the reference's templated functors.
inline double jsqrt(double x) { return std::sqrt(x); }
inline double jcos(double x) { return std::cos(x); }
inline double jsin(double x) { return std::sin(x); }
inline double jabs(double x) { return std::fabs(x); }
inline double jhypot(double x, double y, double z) { return std::hypot(x, y, z); }
inline double value_of(double x) { return x; }
template <int N> double value_of(const Jet<N>& x) { return x.a; }

// ---------------------------------------------------------------------------
// Rotations: include/ceres/rotation.h
// ---------------------------------------------------------------------------
// AngleAxisRotatePoint, rotation.h:830-899.
template <typename T>
void AngleAxisRotatePoint(const T aa[3], const T pt[3], T result[3]) {
  const T theta = jhypot(aa[0], aa[1], aa[2]);
  if (std::fpclassify(value_of(theta)) != FP_ZERO) {
    const T costheta = jcos(theta);
    const T sintheta = jsin(theta);
    const T theta_inverse = T(1.0) / theta;
    const T w[3] = {aa[0] * theta_inverse, aa[1] * theta_inverse,
                    aa[2] * theta_inverse};
    const T w_cross_pt[3] = {w[1] * pt[2] - w[2] * pt[1],
                             w[2] * pt[0] - w[0] * pt[2],
                             w[0] * pt[1] - w[1] * pt[0]};
    const T tmp = (w[0] * pt[0] + w[1] * pt[1] + w[2] * pt[2]) * (T(1.0) - costheta);
    result[0] = pt[0] * costheta + w_cross_pt[0] * sintheta + w[0] * tmp;
    result[1] = pt[1] * costheta + w_cross_pt[1] * sintheta + w[1] * tmp;
    result[2] = pt[2] * costheta + w_cross_pt[2] * sintheta + w[2] * tmp;
  } else {
    // First order Taylor expansion at theta == 0 (rotation.h:873-898).
    const T w_cross_pt[3] = {aa[1] * pt[2] - aa[2] * pt[1],
                             aa[2] * pt[0] - aa[0] * pt[2],
                             aa[0] * pt[1] - aa[1] * pt[0]};
    result[0] = pt[0] + w_cross_pt[0];
    result[1] = pt[1] + w_cross_pt[1];
    result[2] = pt[2] + w_cross_pt[2];
  }
}

// UnitQuaternionRotatePoint, rotation.h:753-774.
template <typename T>
void UnitQuaternionRotatePoint(const T q[4], const T pt[3], T result[3]) {
  T uv0 = q[2] * pt[2] - q[3] * pt[1];
  T uv1 = q[3] * pt[0] - q[1] * pt[2];
  T uv2 = q[1] * pt[1] - q[2] * pt[0];
  uv0 = uv0 + uv0;
  uv1 = uv1 + uv1;
  uv2 = uv2 + uv2;
  result[0] = pt[0] + q[0] * uv0;
  result[1] = pt[1] + q[0] * uv1;
  result[2] = pt[2] + q[0] * uv2;
  result[0] = result[0] + (q[2] * uv2 - q[3] * uv1);
  result[1] = result[1] + (q[3] * uv0 - q[1] * uv2);
  result[2] = result[2] + (q[1] * uv1 - q[2] * uv0);
}

// QuaternionRotatePoint, rotation.h:776-798.
template <typename T>
void QuaternionRotatePoint(const T q[4], const T pt[3], T result[3]) {
  const T scale = T(1) / jsqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  const T unit[4] = {scale * q[0], scale * q[1], scale * q[2], scale * q[3]};
  UnitQuaternionRotatePoint(unit, pt, result);
}

// ---------------------------------------------------------------------------
// Functors
// ---------------------------------------------------------------------------
// SnavelyReprojectionError, examples/snavely_reprojection_error.h:58-93.
template <typename T>
void Snavely(const double* obs, const T* camera, const T* point, T* residuals) {
  T p[3];
  AngleAxisRotatePoint(camera, point, p);
  p[0] = p[0] + camera[3];
  p[1] = p[1] + camera[4];
  p[2] = p[2] + camera[5];
  const T xp = -p[0] / p[2];
  const T yp = -p[1] / p[2];
  const T& l1 = camera[7];
  const T& l2 = camera[8];
  const T r2 = xp * xp + yp * yp;
  const T distortion = 1.0 + r2 * (l1 + l2 * r2);
  const T& focal = camera[6];
  const T predicted_x = focal * distortion * xp;
  const T predicted_y = focal * distortion * yp;
  residuals[0] = predicted_x - obs[0];
  residuals[1] = predicted_y - obs[1];
}

// SnavelyReprojectionErrorNoRadialDistortion,
// internal/ceres/evaluator_cuda_test.cu.cc:117-144.
template <typename T>
void SnavelyNoDistortion(const double* obs, const T* camera, const T* point,
                         T* residuals) {
  T p[3];
  AngleAxisRotatePoint(camera, point, p);
  p[0] = p[0] + camera[3];
  p[1] = p[1] + camera[4];
  p[2] = p[2] + camera[5];
  const T xp = -p[0] / p[2];
  const T yp = -p[1] / p[2];
  const T& focal = camera[6];
  const T predicted_x = focal * xp;
  const T predicted_y = focal * yp;
  residuals[0] = predicted_x - obs[0];
  residuals[1] = predicted_y - obs[1];
}

// SnavelyReprojectionErrorWithQuaternions,
// examples/snavely_reprojection_error.h:118-158.
template <typename T>
void SnavelyQuaternion(const double* obs, const T* camera, const T* point,
                       T* residuals) {
  T p[3];
  QuaternionRotatePoint(camera, point, p);
  p[0] = p[0] + camera[4];
  p[1] = p[1] + camera[5];
  p[2] = p[2] + camera[6];
  const T xp = -p[0] / p[2];
  const T yp = -p[1] / p[2];
  const T& l1 = camera[8];
  const T& l2 = camera[9];
  const T r2 = xp * xp + yp * yp;
  const T distortion = 1.0 + r2 * (l1 + l2 * r2);
  const T& focal = camera[7];
  const T predicted_x = focal * distortion * xp;
  const T predicted_y = focal * distortion * yp;
  residuals[0] = predicted_x - obs[0];
  residuals[1] = predicted_y - obs[1];
}

// PointDisplacementError, internal/ceres/evaluator_cuda_test.cu.cc:84-110.
template <typename T>
void PointDisplacement(const double* xyz, const T* point, T* residuals) {
  residuals[0] = std::fabs(xyz[0]) - jabs(point[0]);
  residuals[1] = std::fabs(xyz[1]) - jabs(point[1]);
  residuals[2] = std::fabs(xyz[2]) - jabs(point[2]);
}

// BundlerResidual (internal/ceres/bundle_adjustment_test_util.h:188-227):
// Snavely's camera with the focal length applied before the perspective
// division and the distortion after it.
template <typename T>
void BundlerResidual(const double* uv, const T* camera, const T* point, T* residuals) {
  T p[3];
  AngleAxisRotatePoint(camera, point, p);
  p[0] = p[0] + camera[3];
  p[1] = p[1] + camera[4];
  p[2] = p[2] + camera[5];
  const T& focal = camera[6];
  const T& l1 = camera[7];
  const T& l2 = camera[8];
  const T xp = -focal * p[0] / p[2];
  const T yp = -focal * p[1] / p[2];
  const T r2 = xp * xp + yp * yp;
  const T distortion = T(1.0) + r2 * (l1 + l2 * r2);
  residuals[0] = distortion * xp - uv[0];
  residuals[1] = distortion * yp - uv[1];
}

struct KindInfo {
  int num_residuals;
  int num_blocks;
  int sizes[2];
  int data_size;
};

static bool kind_info(int kind, KindInfo* k) {
  switch (kind) {
    case ORACLE_SNAVELY_2_9_3: *k = {2, 2, {9, 3}, 2}; return true;
    case ORACLE_SNAVELY_NO_DISTORTION_2_7_3: *k = {2, 2, {7, 3}, 2}; return true;
    case ORACLE_SNAVELY_QUATERNION_2_10_3: *k = {2, 2, {10, 3}, 2}; return true;
    case ORACLE_POINT_DISPLACEMENT_3_3: *k = {3, 1, {3, 0}, 3}; return true;
    case ORACLE_BUNDLER_RESIDUAL_2_9_3: *k = {2, 2, {9, 3}, 2}; return true;
    default: return false;
  }
}

// AutoDifferentiate<kNumResiduals, StaticParameterDims<Ns...>>
// (include/ceres/internal/autodiff.h:314-381): seed a Jet per parameter with
// the unit vector of its position (Make1stOrderPerturbation, :185-199), run
// the functor, take the 0th and 1st order parts row-major (:376-378).
template <int NR, int N0, int N1, typename F>
bool AutoDiff2(F f, const double* const* params, double* residuals,
               double** jacobians) {
  constexpr int N = N0 + N1;
  Jet<N> x0[N0], x1[N1 > 0 ? N1 : 1], out[NR];
  for (int j = 0; j < N0; ++j) x0[j] = Jet<N>(params[0][j], j);
  for (int j = 0; j < N1; ++j) x1[j] = Jet<N>(params[1][j], N0 + j);
  f(x0, x1, out);
  for (int i = 0; i < NR; ++i) residuals[i] = out[i].a;
  if (jacobians) {
    if (jacobians[0])
      for (int i = 0; i < NR; ++i)
        for (int j = 0; j < N0; ++j) jacobians[0][i * N0 + j] = out[i].v[j];
    if (N1 > 0 && jacobians[1])
      for (int i = 0; i < NR; ++i)
        for (int j = 0; j < N1; ++j) jacobians[1][i * N1 + j] = out[i].v[N0 + j];
  }
  return true;
}

// One cost function evaluation (AutoDiffCostFunction::Evaluate,
// include/ceres/autodiff_cost_function.h:201-217).  Without jacobians the
// functor runs on plain doubles, as the reference does.
static bool CostEvaluate(int kind, const double* data, const int32_t* sizes,
                         int nblocks, int nres, const double* const* params,
                         double* residuals, double** jacobians) {
  switch (kind) {
    case ORACLE_SNAVELY_2_9_3:
      if (!jacobians) { Snavely<double>(data, params[0], params[1], residuals); return true; }
      return AutoDiff2<2, 9, 3>(
          [&](const Jet<12>* c, const Jet<12>* p, Jet<12>* r) { Snavely(data, c, p, r); },
          params, residuals, jacobians);
    case ORACLE_SNAVELY_NO_DISTORTION_2_7_3:
      if (!jacobians) { SnavelyNoDistortion<double>(data, params[0], params[1], residuals); return true; }
      return AutoDiff2<2, 7, 3>(
          [&](const Jet<10>* c, const Jet<10>* p, Jet<10>* r) { SnavelyNoDistortion(data, c, p, r); },
          params, residuals, jacobians);
    case ORACLE_SNAVELY_QUATERNION_2_10_3:
      if (!jacobians) { SnavelyQuaternion<double>(data, params[0], params[1], residuals); return true; }
      return AutoDiff2<2, 10, 3>(
          [&](const Jet<13>* c, const Jet<13>* p, Jet<13>* r) { SnavelyQuaternion(data, c, p, r); },
          params, residuals, jacobians);
    case ORACLE_BUNDLER_RESIDUAL_2_9_3:
      if (!jacobians) { BundlerResidual<double>(data, params[0], params[1], residuals); return true; }
      return AutoDiff2<2, 9, 3>(
          [&](const Jet<12>* c, const Jet<12>* p, Jet<12>* r) { BundlerResidual(data, c, p, r); },
          params, residuals, jacobians);
    case ORACLE_POINT_DISPLACEMENT_3_3:
      if (!jacobians) { PointDisplacement<double>(data, params[0], residuals); return true; }
      return AutoDiff2<3, 3, 0>(
          [&](const Jet<3>* p, const Jet<3>*, Jet<3>* r) { PointDisplacement(data, p, r); },
          params, residuals, jacobians);
    case ORACLE_LINEAR_TEST: {
      // ParameterIgnoringCostFunction<kFactor, kNumResiduals, Ns...>
      // (internal/ceres/evaluator_test.cc:58-100) written as the linear
      // functor r_i = (i+1) + kFactor * sum_k sum_j (j+1) x_k[j], whose value
      // at the zero state and Jacobian are exactly what the fake returns.
      const double k_factor = data[0];
      double acc = 0.0;
      for (int b = 0; b < nblocks; ++b)
        for (int j = 0; j < sizes[b]; ++j) acc += (j + 1) * params[b][j];
      for (int i = 0; i < nres; ++i) residuals[i] = (i + 1) + k_factor * acc;
      if (jacobians)
        for (int b = 0; b < nblocks; ++b)
          if (jacobians[b])
            for (int i = 0; i < nres; ++i)
              for (int j = 0; j < sizes[b]; ++j)
                jacobians[b][i * sizes[b] + j] = k_factor * (j + 1);
      return true;
    }
    default:
      return false;
  }
}

// ---------------------------------------------------------------------------
// Losses: include/ceres/loss_function_cuda.h:62-150 (identical formulas to
// the host HuberLoss/CauchyLoss in internal/ceres/loss_function.cc:50-80).
// ---------------------------------------------------------------------------
static void Loss(int kind, double a, int scaled, double scale, double s,
                 double rho[3], double b_param = 0.0) {
  switch (kind) {
    case ORACLE_LOSS_SOFT_L_ONE: {  // loss_function.cc:66-73 (b = a^2, c = 1/b)
      const double b = a * a, c = 1 / b;
      const double sum = 1.0 + s * c;
      const double tmp = std::sqrt(sum);
      rho[0] = 2.0 * b * (tmp - 1.0);
      rho[1] = std::max(std::numeric_limits<double>::min(), 1.0 / tmp);
      rho[2] = -(c * rho[1]) / (2.0 * sum);
      break;
    }
    case ORACLE_LOSS_TOLERANT: {  // loss_function.cc:87-118
      const double bb = b_param, c = bb * std::log(1.0 + std::exp(-a / bb));
      const double x = (s - a) / bb;
      if (x > 36.7) {
        rho[0] = s - a - c;
        rho[1] = 1.0;
        rho[2] = 0.0;
      } else {
        const double e_x = std::exp(x);
        rho[0] = bb * std::log(1.0 + e_x) - c;
        rho[1] = std::max(std::numeric_limits<double>::min(), e_x / (1.0 + e_x));
        rho[2] = 0.5 / (bb * (1.0 + std::cosh(x)));
      }
      break;
    }
    case ORACLE_LOSS_HUBER: {
      const double b = a * a;
      if (s > b) {
        const double r = std::sqrt(s);
        rho[0] = 2.0 * a * r - b;
        rho[1] = std::max(std::numeric_limits<double>::min(), a / r);
        rho[2] = -rho[1] / (2.0 * s);
      } else {
        rho[0] = s; rho[1] = 1.0; rho[2] = 0.0;
      }
      break;
    }
    case ORACLE_LOSS_CAUCHY: {
      const double b = a * a;
      const double c = 1 / b;
      const double sum = 1.0 + s * c;
      const double inv = 1.0 / sum;
      rho[0] = b * std::log(sum);
      rho[1] = std::max(std::numeric_limits<double>::min(), inv);
      rho[2] = -c * (inv * inv);
      break;
    }
    default:
      rho[0] = s; rho[1] = 1.0; rho[2] = 0.0;
  }
  if (scaled) {
    // ScaledLossCUDA (loss_function_cuda.h:115-150); the Trivial
    // specialisation gives the same numbers as scaling (s, 1, 0).
    if (kind == ORACLE_LOSS_TRIVIAL) {
      rho[0] = scale * s; rho[1] = scale; rho[2] = 0.0;
    } else {
      rho[0] *= scale; rho[1] *= scale; rho[2] *= scale;
    }
  }
}

// Corrector, include/ceres/internal/corrector.h:82-213.
struct Corrector {
  double sqrt_rho1, residual_scaling, alpha_sq_norm;
  Corrector(double sq_norm, const double rho[3]) {
    sqrt_rho1 = std::sqrt(rho[1]);
    if ((sq_norm == 0.0) || (rho[2] <= 0.0)) {
      residual_scaling = sqrt_rho1;
      alpha_sq_norm = 0.0;
      return;
    }
    const double D = 1.0 + 2.0 * sq_norm * rho[2] / rho[1];
    const double alpha = 1.0 - std::sqrt(D);
    residual_scaling = sqrt_rho1 / (1 - alpha);
    alpha_sq_norm = alpha / sq_norm;
  }
  void CorrectResiduals(int n, double* r) const {
    for (int i = 0; i < n; ++i) r[i] *= residual_scaling;
  }
  void CorrectJacobian(int rows, int cols, const double* r, double* J) const {
    if (alpha_sq_norm == 0.0) {
      for (int i = 0; i < rows * cols; ++i) J[i] *= sqrt_rho1;
      return;
    }
    for (int c = 0; c < cols; ++c) {
      double r_transpose_j = 0.0;
      for (int k = 0; k < rows; ++k) r_transpose_j += J[k * cols + c] * r[k];
      for (int k = 0; k < rows; ++k)
        J[k * cols + c] = sqrt_rho1 * (J[k * cols + c] - alpha_sq_norm * r[k] * r_transpose_j);
    }
  }
};

static bool AllFinite(int n, const double* x) {
  for (int i = 0; i < n; ++i)
    if (!std::isfinite(x[i])) return false;
  return true;
}

// ---------------------------------------------------------------------------
// Program: offsets (program.cc:151-177) and Jacobian layouts.
// ---------------------------------------------------------------------------
struct Prepared {
  const oracle_program* p;
  std::vector<int64_t> state_offset;  // active: into state; constant: into constant_state
  std::vector<int64_t> delta_offset;  // active only
  std::vector<int64_t> active_index;  // program index among active blocks, -1 constant
  std::vector<int64_t> residual_offset;
  std::vector<int> num_res;
  int64_t num_parameters = 0, num_effective = 0, num_constant = 0, num_residuals = 0;
  // BSM: per residual block, position of each active cell (jacobian_layout_).
  std::vector<int64_t> cell_begin;  // [nrb+1] into cell_pos
  std::vector<int64_t> cell_pos;
  // CRS: row pointers.
  std::vector<int64_t> crs_rows;
  int64_t num_jacobian_values = 0;
  int max_scratch = 0;
};

static int Prepare(const oracle_program* p, Prepared* P) {
  P->p = p;
  const int64_t npb = p->num_parameter_blocks;
  P->state_offset.assign(npb, 0);
  P->delta_offset.assign(npb, -1);
  P->active_index.assign(npb, -1);
  int64_t so = 0, dof = 0, cso = 0, ai = 0;
  for (int64_t i = 0; i < npb; ++i) {
    if (p->pb_constant[i]) {
      P->state_offset[i] = cso;
      cso += p->pb_size[i];
    } else {
      P->state_offset[i] = so;
      P->delta_offset[i] = dof;
      P->active_index[i] = ai++;
      so += p->pb_size[i];
      dof += p->pb_tangent_size[i];
    }
  }
  P->num_parameters = so;
  P->num_effective = dof;
  P->num_constant = cso;

  const int64_t nrb = p->num_residual_blocks;
  P->residual_offset.assign(nrb, 0);
  P->num_res.assign(nrb, 0);
  int64_t ro = 0;
  for (int64_t i = 0; i < nrb; ++i) {
    int nres;
    if (p->rb_kind[i] == ORACLE_LINEAR_TEST) {
      nres = (int)p->rb_data[p->rb_data_begin[i] + 1];
    } else {
      KindInfo k;
      if (!kind_info(p->rb_kind[i], &k)) return -1;
      nres = k.num_residuals;
      if (p->rb_param_begin[i + 1] - p->rb_param_begin[i] != k.num_blocks) return -2;
      for (int j = 0; j < k.num_blocks; ++j)
        if (p->pb_size[p->rb_params[p->rb_param_begin[i] + j]] != k.sizes[j]) return -3;
    }
    P->num_res[i] = nres;
    P->residual_offset[i] = ro;
    ro += nres;
  }
  P->num_residuals = ro;

  // Scratch for plus-jacobian products: ambient jacobians per block.
  for (int64_t i = 0; i < nrb; ++i) {
    int s = 0;
    for (int64_t q = p->rb_param_begin[i]; q < p->rb_param_begin[i + 1]; ++q)
      s += P->num_res[i] * p->pb_size[p->rb_params[q]];
    P->max_scratch = std::max(P->max_scratch, s);
  }

  if (p->jacobian_format == ORACLE_BLOCK_SPARSE) {
    // BuildJacobianLayout (block_jacobian_writer.cc:62-150): E cells (active
    // index < num_eliminate_blocks) first, in residual order, then F cells.
    int64_t f_block_pos = 0;
    for (int64_t i = 0; i < nrb; ++i)
      for (int64_t q = p->rb_param_begin[i]; q < p->rb_param_begin[i + 1]; ++q) {
        const int32_t b = p->rb_params[q];
        if (!p->pb_constant[b] && P->active_index[b] < p->num_eliminate_blocks)
          f_block_pos += (int64_t)P->num_res[i] * p->pb_tangent_size[b];
      }
    int64_t e_block_pos = 0;
    P->cell_begin.assign(nrb + 1, 0);
    P->cell_pos.clear();
    for (int64_t i = 0; i < nrb; ++i) {
      P->cell_begin[i] = (int64_t)P->cell_pos.size();
      for (int64_t q = p->rb_param_begin[i]; q < p->rb_param_begin[i + 1]; ++q) {
        const int32_t b = p->rb_params[q];
        if (p->pb_constant[b]) continue;
        const int64_t cell = (int64_t)P->num_res[i] * p->pb_tangent_size[b];
        if (P->active_index[b] < p->num_eliminate_blocks) {
          P->cell_pos.push_back(e_block_pos);
          e_block_pos += cell;
        } else {
          P->cell_pos.push_back(f_block_pos);
          f_block_pos += cell;
        }
      }
    }
    P->cell_begin[nrb] = (int64_t)P->cell_pos.size();
    P->num_jacobian_values = f_block_pos;
  } else {
    // CompressedRowJacobianWriter::CreateJacobian
    // (compressed_row_jacobian_writer.cc:93-193): a row holds the active
    // blocks' columns sorted by block index.
    P->crs_rows.assign(ro + 1, 0);
    int64_t row_pos = 0;
    for (int64_t i = 0; i < nrb; ++i) {
      int64_t nd = 0;
      for (int64_t q = p->rb_param_begin[i]; q < p->rb_param_begin[i + 1]; ++q) {
        const int32_t b = p->rb_params[q];
        if (!p->pb_constant[b]) nd += p->pb_tangent_size[b];
      }
      for (int r = 0; r < P->num_res[i]; ++r)
        P->crs_rows[row_pos + r + 1] = P->crs_rows[row_pos + r] + nd;
      row_pos += P->num_res[i];
    }
    P->num_jacobian_values = P->crs_rows[ro];
  }
  return 0;
}

// Active blocks of residual block i, sorted by program index, paired with
// their argument position (GetOrderedParameterBlocks,
// compressed_row_jacobian_writer.cc:71-91).
static void OrderedBlocks(const Prepared& P, int64_t i,
                          std::vector<std::pair<int64_t, int>>* out) {
  const oracle_program* p = P.p;
  out->clear();
  int arg = 0;
  for (int64_t q = p->rb_param_begin[i]; q < p->rb_param_begin[i + 1]; ++q, ++arg) {
    const int32_t b = p->rb_params[q];
    if (!p->pb_constant[b]) out->push_back({P.active_index[b], arg});
  }
  std::sort(out->begin(), out->end());
}

// ResidualBlock::Evaluate (internal/ceres/residual_block.cc:68-204).
// jacobians[j] is null for constant blocks (BlockEvaluatePreparer,
// block_evaluate_preparer.cc:48-75) and points at tangent-sized storage.
static bool EvaluateResidualBlock(const Prepared& P, int64_t i,
                                  const double* state, const double* cstate,
                                  bool apply_loss, double* cost, double* residuals,
                                  double** jacobians, double* scratch) {
  const oracle_program* p = P.p;
  const int nb = (int)(p->rb_param_begin[i + 1] - p->rb_param_begin[i]);
  const int nres = P.num_res[i];
  const double* params[8];
  int32_t sizes[8];
  double* global_jac[8];
  for (int j = 0; j < nb; ++j) {
    const int32_t b = p->rb_params[p->rb_param_begin[i] + j];
    params[j] = (p->pb_constant[b] ? cstate : state) + P.state_offset[b];
    sizes[j] = p->pb_size[b];
  }
  double* sc = scratch;
  if (jacobians) {
    for (int j = 0; j < nb; ++j) {
      const int32_t b = p->rb_params[p->rb_param_begin[i] + j];
      if (jacobians[j] != nullptr && p->pb_plus_jacobian[b] >= 0) {
        global_jac[j] = sc;
        sc += nres * p->pb_size[b];
      } else {
        global_jac[j] = jacobians[j];
      }
    }
  }
  double** eval_jac = jacobians ? global_jac : nullptr;
  const double* data = p->rb_data + p->rb_data_begin[i];
  if (!CostEvaluate(p->rb_kind[i], data, sizes, nb, nres, params, residuals, eval_jac))
    return false;
  // IsEvaluationValid (residual_block_utils.cc): everything requested finite.
  if (!AllFinite(nres, residuals)) return false;
  if (eval_jac)
    for (int j = 0; j < nb; ++j)
      if (eval_jac[j] && !AllFinite(nres * sizes[j], eval_jac[j])) return false;

  double squared_norm = 0.0;
  for (int k = 0; k < nres; ++k) squared_norm += residuals[k] * residuals[k];

  // Apply the plus-jacobian (residual_block.cc:133-156):
  // jacobians[j] = global_jacobians[j] * PlusJacobian (MatrixMatrixMultiply,
  // kOperation = 0 i.e. assignment).
  if (jacobians) {
    for (int j = 0; j < nb; ++j) {
      const int32_t b = p->rb_params[p->rb_param_begin[i] + j];
      if (jacobians[j] && p->pb_plus_jacobian[b] >= 0) {
        const int size = p->pb_size[b], tan = p->pb_tangent_size[b];
        const double* pj = p->plus_jacobians + p->pb_plus_jacobian[b];
        for (int r = 0; r < nres; ++r)
          for (int c = 0; c < tan; ++c) {
            double s = 0.0;
            for (int k = 0; k < size; ++k) s += global_jac[j][r * size + k] * pj[k * tan + c];
            jacobians[j][r * tan + c] = s;
          }
      }
    }
  }

  if (p->rb_loss_kind[i] == ORACLE_LOSS_TRIVIAL && !p->rb_loss_scaled[i]) {
    *cost = 0.5 * squared_norm;
    return true;
  }
  if (!apply_loss) {
    *cost = 0.5 * squared_norm;
    return true;
  }
  double rho[3];
  Loss(p->rb_loss_kind[i], p->rb_loss_a[i], p->rb_loss_scaled[i], p->rb_loss_scale[i],
       squared_norm, rho, p->rb_loss_b ? p->rb_loss_b[i] : 0.0);
  *cost = 0.5 * rho[0];
  Corrector correct(squared_norm, rho);
  if (jacobians)
    for (int j = 0; j < nb; ++j)
      if (jacobians[j]) {
        const int32_t b = p->rb_params[p->rb_param_begin[i] + j];
        correct.CorrectJacobian(nres, p->pb_tangent_size[b], residuals, jacobians[j]);
      }
  correct.CorrectResiduals(nres, residuals);
  return true;
}

// ParallelFor with kWorkBlocksPerThread = 4 contiguous chunks handed out
// dynamically (parallel_invoke.h:165-260, parallel_for.h:73-87).
template <typename F>
static void ParallelFor(int64_t start, int64_t end, int num_threads, F&& fn) {
  if (start >= end) return;
  if (num_threads <= 1 || end - start == 1) {
    for (int64_t i = start; i < end; ++i) fn(0, i);
    return;
  }
  const int64_t num_work_blocks = std::min<int64_t>(end - start, (int64_t)num_threads * 4);
  const int64_t base = (end - start) / num_work_blocks;
  const int64_t num_p1 = (end - start) % num_work_blocks;
  std::atomic<int64_t> next(0);
  auto task = [&](int tid) {
    while (true) {
      const int64_t b = next.fetch_add(1);
      if (b >= num_work_blocks) break;
      const int64_t cs = start + b * base + std::min(b, num_p1);
      const int64_t ce = cs + base + (b < num_p1 ? 1 : 0);
      for (int64_t i = cs; i < ce; ++i) fn(tid, i);
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < num_threads; ++t) pool.emplace_back(task, t);
  task(0);
  for (auto& th : pool) th.join();
}

}  // namespace oracle

using namespace oracle;

extern "C" int oracle_sizes_of(const oracle_program* p, oracle_sizes* out) {
  Prepared P;
  const int rc = Prepare(p, &P);
  if (rc) return rc;
  out->num_parameters = P.num_parameters;
  out->num_effective_parameters = P.num_effective;
  out->num_constant_parameters = P.num_constant;
  out->num_residuals = P.num_residuals;
  out->num_jacobian_values = P.num_jacobian_values;
  return 0;
}

// ProgramEvaluator (internal/ceres/program_evaluator.h:86-290): the layout
// and per-thread scratch are built once at construction, Evaluate() is the
// per-iteration hot path (the CPU baseline times only Evaluate()).
struct Evaluator {
  struct Scratch {
    double cost = 0.0;
    std::vector<double> gradient, residuals, jac, eval;
  };
  Prepared P;
  std::vector<Scratch> scratch;
  int num_threads = 1;

  int Init(const oracle_program* p, int threads) {
    const int rc = Prepare(p, &P);
    if (rc) return rc;
    num_threads = threads < 1 ? 1 : threads;
    int max_nres = 0, max_der = 0;
    for (int64_t i = 0; i < p->num_residual_blocks; ++i) {
      max_nres = std::max(max_nres, P.num_res[i]);
      int d = 0;
      for (int64_t q = p->rb_param_begin[i]; q < p->rb_param_begin[i + 1]; ++q)
        d += P.num_res[i] * p->pb_tangent_size[p->rb_params[q]];
      max_der = std::max(max_der, d);
    }
    scratch.resize(num_threads);
    for (auto& s : scratch) {
      s.gradient.assign(P.num_effective, 0.0);
      s.residuals.assign(max_nres, 0.0);
      s.jac.assign(max_der + 1, 0.0);
      s.eval.assign(P.max_scratch + max_nres + 1, 0.0);
    }
    return 0;
  }

  int Evaluate(const double* state, const double* constant_state, double* cost,
               double* residuals, double* gradient, double* jacobian_values) {
    const oracle_program* p = P.p;
    const bool want_jac = jacobian_values != nullptr;
    const bool want_grad = gradient != nullptr;
    if (residuals) std::fill(residuals, residuals + P.num_residuals, 0.0);
    if (want_jac) std::fill(jacobian_values, jacobian_values + P.num_jacobian_values, 0.0);
    for (auto& s : scratch) {
      s.cost = 0.0;
      if (want_grad) std::fill(s.gradient.begin(), s.gradient.end(), 0.0);
    }
    std::atomic<bool> abort(false);
    ParallelFor(0, p->num_residual_blocks, num_threads, [&](int tid, int64_t i) {
      if (abort) return;
      Scratch& s = scratch[tid];
      double* block_residuals = residuals ? residuals + P.residual_offset[i] : s.residuals.data();
      double* block_jac[8] = {nullptr};
      const int nb = (int)(p->rb_param_begin[i + 1] - p->rb_param_begin[i]);
      const bool need_jac = want_jac || want_grad;
      if (need_jac) {
        // Cells are evaluated into scratch (ScratchEvaluatePreparer) and
        // then written by the layout below; for BSM this is numerically
        // identical to BlockEvaluatePreparer writing in place.
        double* cur = s.jac.data();
        for (int j = 0; j < nb; ++j) {
          const int32_t b = p->rb_params[p->rb_param_begin[i] + j];
          if (p->pb_constant[b]) continue;
          block_jac[j] = cur;
          cur += P.num_res[i] * p->pb_tangent_size[b];
        }
      }
      double block_cost;
      if (!EvaluateResidualBlock(P, i, state, constant_state, p->apply_loss_function != 0,
                                 &block_cost, block_residuals, need_jac ? block_jac : nullptr,
                                 s.eval.data())) {
        abort = true;
        return;
      }
      s.cost += block_cost;
      const int nres = P.num_res[i];
      if (want_jac) {
        if (p->jacobian_format == ORACLE_BLOCK_SPARSE) {
          int k = 0;
          for (int j = 0; j < nb; ++j) {
            if (!block_jac[j]) continue;
            const int32_t b = p->rb_params[p->rb_param_begin[i] + j];
            const int64_t pos = P.cell_pos[P.cell_begin[i] + k++];
            std::memcpy(jacobian_values + pos, block_jac[j],
                        sizeof(double) * nres * p->pb_tangent_size[b]);
          }
        } else {
          // CompressedRowJacobianWriter::Write (:195-238).
          std::pair<int64_t, int> ob[8];
          int nob = 0;
          int arg = 0;
          for (int64_t q = p->rb_param_begin[i]; q < p->rb_param_begin[i + 1]; ++q, ++arg) {
            const int32_t b = p->rb_params[q];
            if (!p->pb_constant[b]) ob[nob++] = {P.active_index[b], arg};
          }
          std::sort(ob, ob + nob);
          int64_t col_pos = 0;
          for (int e = 0; e < nob; ++e) {
            const int a = ob[e].second;
            const int32_t b = p->rb_params[p->rb_param_begin[i] + a];
            const int tan = p->pb_tangent_size[b];
            for (int r = 0; r < nres; ++r)
              std::memcpy(jacobian_values + P.crs_rows[P.residual_offset[i] + r] + col_pos,
                          block_jac[a] + r * tan, sizeof(double) * tan);
            col_pos += tan;
          }
        }
      }
      if (want_grad) {
        // MatrixTransposeVectorMultiply into the thread's gradient scratch.
        for (int j = 0; j < nb; ++j) {
          if (!block_jac[j]) continue;
          const int32_t b = p->rb_params[p->rb_param_begin[i] + j];
          const int tan = p->pb_tangent_size[b];
          double* g = s.gradient.data() + P.delta_offset[b];
          for (int c = 0; c < tan; ++c) {
            double acc = 0.0;
            for (int r = 0; r < nres; ++r) acc += block_jac[j][r * tan + c] * block_residuals[r];
            g[c] += acc;
          }
        }
      }
    });
    if (abort) return 0;
    *cost = 0.0;
    if (want_grad) std::fill(gradient, gradient + P.num_effective, 0.0);
    for (int t = 0; t < num_threads; ++t) {
      *cost += scratch[t].cost;
      if (want_grad)
        for (int64_t k = 0; k < P.num_effective; ++k) gradient[k] += scratch[t].gradient[k];
    }
    return 1;
  }
};

extern "C" void* oracle_create(const oracle_program* p, int num_threads) {
  Evaluator* e = new Evaluator();
  if (e->Init(p, num_threads)) {
    delete e;
    return nullptr;
  }
  return e;
}

extern "C" int oracle_run(void* h, const double* state, const double* constant_state,
                          double* cost, double* residuals, double* gradient,
                          double* jacobian_values) {
  return static_cast<Evaluator*>(h)->Evaluate(state, constant_state, cost, residuals, gradient,
                                              jacobian_values);
}

extern "C" void oracle_destroy(void* h) { delete static_cast<Evaluator*>(h); }

extern "C" int oracle_evaluate(const oracle_program* p, const double* state,
                               const double* constant_state, int num_threads,
                               double* cost, double* residuals, double* gradient,
                               double* jacobian_values) {
  Evaluator e;
  const int rc = e.Init(p, num_threads);
  if (rc) return rc;
  return e.Evaluate(state, constant_state, cost, residuals, gradient, jacobian_values);
}

extern "C" int oracle_jacobian_offsets(const oracle_program* p, int64_t* per_residual_layout,
                                       int64_t* per_residual_offsets, int64_t* crs_rows,
                                       int64_t* crs_cols) {
  Prepared P;
  const int rc = Prepare(p, &P);
  if (rc) return rc;
  int64_t pos = 0;
  for (int64_t i = 0; i < p->num_residual_blocks; ++i) {
    per_residual_layout[i] = pos;
    const int nres = P.num_res[i];
    if (p->jacobian_format == ORACLE_BLOCK_SPARSE) {
      int k = 0;
      for (int64_t q = p->rb_param_begin[i]; q < p->rb_param_begin[i + 1]; ++q) {
        const int32_t b = p->rb_params[q];
        if (p->pb_constant[b]) continue;
        const int64_t cell = P.cell_pos[P.cell_begin[i] + k++];
        for (int r = 0; r < nres; ++r)
          per_residual_offsets[pos++] = cell + (int64_t)r * p->pb_tangent_size[b];
      }
    } else {
      // CreateJacobianPerResidualLayout (:240-300): entry
      // [pos + r + nres * active_arg] = row start + column position.
      std::vector<std::pair<int64_t, int>> ob;
      OrderedBlocks(P, i, &ob);
      std::vector<int> active_arg_of(8, -1);
      {
        int aa = 0;
        int arg = 0;
        for (int64_t q = p->rb_param_begin[i]; q < p->rb_param_begin[i + 1]; ++q, ++arg)
          if (!p->pb_constant[p->rb_params[q]]) active_arg_of[arg] = aa++;
      }
      for (int r = 0; r < nres; ++r) {
        int64_t col_pos = 0;
        for (auto& e : ob) {
          const int32_t b = p->rb_params[p->rb_param_begin[i] + e.second];
          per_residual_offsets[pos + r + nres * active_arg_of[e.second]] =
              P.crs_rows[P.residual_offset[i] + r] + col_pos;
          col_pos += p->pb_tangent_size[b];
        }
      }
      pos += (int64_t)ob.size() * nres;
    }
  }
  if (p->jacobian_format == ORACLE_COMPRESSED_ROW && crs_rows) {
    for (int64_t r = 0; r <= P.num_residuals; ++r) crs_rows[r] = P.crs_rows[r];
    if (crs_cols) {
      std::vector<std::pair<int64_t, int>> ob;
      for (int64_t i = 0; i < p->num_residual_blocks; ++i) {
        OrderedBlocks(P, i, &ob);
        for (int r = 0; r < P.num_res[i]; ++r) {
          int64_t col_pos = 0;
          const int64_t row_start = P.crs_rows[P.residual_offset[i] + r];
          for (auto& e : ob) {
            const int32_t b = p->rb_params[p->rb_param_begin[i] + e.second];
            for (int c = 0; c < p->pb_tangent_size[b]; ++c)
              crs_cols[row_start + col_pos + c] = P.delta_offset[b] + c;
            col_pos += p->pb_tangent_size[b];
          }
        }
      }
    }
  }
  return 0;
}

extern "C" void oracle_angle_axis_rotate_point(const double aa[3], const double pt[3],
                                               double out[3]) {
  AngleAxisRotatePoint<double>(aa, pt, out);
}

extern "C" void oracle_quaternion_rotate_point(const double q[4], const double pt[3],
                                               double out[3]) {
  QuaternionRotatePoint<double>(q, pt, out);
}

extern "C" void oracle_loss(int kind, double a, int scaled, double scale, double s,
                            double rho[3]) {
  Loss(kind, a, scaled, scale, s, rho);
}

extern "C" void oracle_loss_ab(int kind, double a, double b, int scaled, double scale, double s,
                               double rho[3]) {
  Loss(kind, a, scaled, scale, s, rho, b);
}

extern "C" void oracle_corrector(double sq_norm, const double rho[3], int num_rows,
                                 int num_cols, double* residuals, double* jacobian) {
  Corrector c(sq_norm, rho);
  if (jacobian) c.CorrectJacobian(num_rows, num_cols, residuals, jacobian);
  if (residuals) c.CorrectResiduals(num_rows, residuals);
}

extern "C" int oracle_autodiff(int kind, const double* data, const double* const* params,
                               double* residuals, double** jacobians) {
  KindInfo k;
  if (!kind_info(kind, &k)) return -1;
  int32_t sizes[2] = {k.sizes[0], k.sizes[1]};
  return CostEvaluate(kind, data, sizes, k.num_blocks, k.num_residuals, params, residuals,
                      jacobians)
             ? 1
             : 0;
}

extern "C" void oracle_jet_op(int op, const double* x, const double* y, const double* z,
                              double* out) {
  auto load = [](const double* s) {
    Jet<3> j;
    j.a = s[0];
    for (int i = 0; i < 3; ++i) j.v[i] = s[1 + i];
    return j;
  };
  Jet<3> a = load(x), r;
  switch (op) {
    case 0: r = jsin(a); break;
    case 1: r = jcos(a); break;
    case 2: r = jsqrt(a); break;
    case 3: r = jhypot(a, load(y), load(z)); break;
    case 4: r = jabs(a); break;
    case 5: r = a / load(y); break;
    case 6: r = a * load(y); break;
    default: r = a;
  }
  out[0] = r.a;
  for (int i = 0; i < 3; ++i) out[1 + i] = r.v[i];
}
