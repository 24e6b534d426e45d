// user_functors.h -- the example user functors and LossFunctionCUDA
// classes (see user_functors.hip for what each restates); header-only so
// that a test TU can use them through ProblemCUDA::AddResidualBlock.
#ifndef CSE_EXAMPLES_USER_FUNCTORS_H_
#define CSE_EXAMPLES_USER_FUNCTORS_H_

#include <cfloat>
#include <cmath>

#include "ceres_amd/autodiff_cuda.h"

namespace user {

using ceres_amd::AngleAxisRotatePoint;
using ceres_amd::QuaternionRotatePoint;

struct BundlerResidual {
  BundlerResidual(double u, double v) : u(u), v(v) {}
  template <typename T>
  HOST_DEVICE bool operator()(const T* const camera, const T* const point, T* residuals) const {
    T p[3];
    AngleAxisRotatePoint(camera, point, p);
    p[0] += camera[3];
    p[1] += camera[4];
    p[2] += camera[5];
    const T& focal = camera[6];
    const T& l1 = camera[7];
    const T& l2 = camera[8];
    T xp = -focal * p[0] / p[2];
    T yp = -focal * p[1] / p[2];
    T r2 = xp * xp + yp * yp;
    T distortion = T(1.0) + r2 * (l1 + l2 * r2);
    residuals[0] = distortion * xp - u;
    residuals[1] = distortion * yp - v;
    return true;
  }
  double u, v;
};

struct SnavelyReprojectionError {
  HOST_DEVICE SnavelyReprojectionError(double observed_x, double observed_y)
      : observed_x(observed_x), observed_y(observed_y) {}
  template <typename T>
  HOST_DEVICE bool operator()(const T* const camera, const T* const point, T* residuals) const {
    T p[3];
    AngleAxisRotatePoint(camera, point, p);
    p[0] += camera[3];
    p[1] += camera[4];
    p[2] += camera[5];
    const T xp = -p[0] / p[2];
    const T yp = -p[1] / p[2];
    const T& l1 = camera[7];
    const T& l2 = camera[8];
    const T r2 = xp * xp + yp * yp;
    const T distortion = 1.0 + r2 * (l1 + l2 * r2);
    const T& focal = camera[6];
    const T predicted_x = focal * distortion * xp;
    const T predicted_y = focal * distortion * yp;
    residuals[0] = predicted_x - observed_x;
    residuals[1] = predicted_y - observed_y;
    return true;
  }
  double observed_x, observed_y;
};

struct SnavelyReprojectionErrorNoRadialDistortion {
  SnavelyReprojectionErrorNoRadialDistortion(double observed_x, double observed_y)
      : observed_x(observed_x), observed_y(observed_y) {}
  template <typename T>
  HOST_DEVICE bool operator()(const T* const camera, const T* const point, T* residuals) const {
    T p[3];
    AngleAxisRotatePoint(camera, point, p);
    p[0] += camera[3];
    p[1] += camera[4];
    p[2] += camera[5];
    const T xp = -p[0] / p[2];
    const T yp = -p[1] / p[2];
    const T& focal = camera[6];
    const T predicted_x = focal * xp;
    const T predicted_y = focal * yp;
    residuals[0] = predicted_x - observed_x;
    residuals[1] = predicted_y - observed_y;
    return true;
  }
  double observed_x, observed_y;
};

struct SnavelyReprojectionErrorWithQuaternions {
  HOST_DEVICE SnavelyReprojectionErrorWithQuaternions(double observed_x, double observed_y)
      : observed_x(observed_x), observed_y(observed_y) {}
  template <typename T>
  HOST_DEVICE bool operator()(const T* const camera, const T* const point, T* residuals) const {
    T p[3];
    QuaternionRotatePoint(camera, point, p);
    p[0] += camera[4];
    p[1] += camera[5];
    p[2] += camera[6];
    const T xp = -p[0] / p[2];
    const T yp = -p[1] / p[2];
    const T& l1 = camera[8];
    const T& l2 = camera[9];
    const T r2 = xp * xp + yp * yp;
    const T distortion = 1.0 + r2 * (l1 + l2 * r2);
    const T& focal = camera[7];
    const T predicted_x = focal * distortion * xp;
    const T predicted_y = focal * distortion * yp;
    residuals[0] = predicted_x - observed_x;
    residuals[1] = predicted_y - observed_y;
    return true;
  }
  double observed_x, observed_y;
};

struct PointDisplacementError {
  PointDisplacementError(double x, double y, double z) : x_(x), y_(y), z_(z) {}
  template <typename T>
  HOST_DEVICE bool operator()(const T* const point, T* residuals) const {
    residuals[0] = abs(x_) - abs(point[0]);
    residuals[1] = abs(y_) - abs(point[1]);
    residuals[2] = abs(z_) - abs(point[2]);
    return true;
  }
  double x_, y_, z_;
};

class BinaryScalarCost {
 public:
  HOST_DEVICE explicit BinaryScalarCost(double a) : a_(a) {}
  template <typename T>
  HOST_DEVICE bool operator()(const T* const x, const T* const y, T* cost) const {
    cost[0] = x[0] * y[0] + x[1] * y[1] - T(a_);
    return true;
  }

 private:
  double a_;
};

struct TenParameterCost {
  template <typename T>
  HOST_DEVICE bool operator()(const T* const x0, const T* const x1, const T* const x2,
                              const T* const x3, const T* const x4, const T* const x5,
                              const T* const x6, const T* const x7, const T* const x8,
                              const T* const x9, T* cost) const {
    cost[0] = *x0 + *x1 + *x2 + *x3 + *x4 + *x5 + *x6 + *x7 + *x8 + *x9;
    return true;
  }
};

struct OnlyFillsOneOutputFunctor {
  static constexpr bool kMayLeaveOutputs = true;  // AutoDifferentiate's unassigned-output check
  template <typename T>
  HOST_DEVICE bool operator()(const T* x, T* output) const {
    output[0] = x[0];
    return true;
  }
};

// Three functors of shapes outside the library's own kinds, the kind a
// user brings: they run on the affine kernels through
// ceres_amd/autodiff_cuda.h (tests/test_user_functor_gpu.py checks each
// against the general kernel).
//
// Reprojection with a pose block (angle-axis, translation: 6) and a point
// (3); the pinhole intrinsics travel in the functor (6 doubles of data).
struct PoseReprojectionError {
  PoseReprojectionError(double u, double v, double fx, double fy, double cx, double cy)
      : u(u), v(v), fx(fx), fy(fy), cx(cx), cy(cy) {}
  template <typename T>
  HOST_DEVICE bool operator()(const T* const pose, const T* const point, T* residuals) const {
    T p[3];
    AngleAxisRotatePoint(pose, point, p);
    p[0] += pose[3];
    p[1] += pose[4];
    p[2] += pose[5];
    residuals[0] = fx * p[0] / p[2] + cx - u;
    residuals[1] = fy * p[1] / p[2] + cy - v;
    return true;
  }
  double u, v, fx, fy, cx, cy;
};

// Signed distance of a point (3), moved by a pose (6), to a plane n.x = d:
// one residual, the plane in the functor (4 doubles).
struct PointToPlaneError {
  PointToPlaneError(double nx, double ny, double nz, double d) : nx(nx), ny(ny), nz(nz), d(d) {}
  template <typename T>
  HOST_DEVICE bool operator()(const T* const pose, const T* const point, T* residuals) const {
    T q[3];
    AngleAxisRotatePoint(pose, point, q);
    residuals[0] = nx * (q[0] + pose[3]) + ny * (q[1] + pose[4]) + nz * (q[2] + pose[5]) - d;
    return true;
  }
  double nx, ny, nz, d;
};

// Rigid alignment: a source point moved by one pose block (6) against its
// target, three residuals; both points in the functor (6 doubles).
struct RigidAlignmentError {
  RigidAlignmentError(const double* src, const double* dst)
      : sx(src[0]), sy(src[1]), sz(src[2]), tx(dst[0]), ty(dst[1]), tz(dst[2]) {}
  template <typename T>
  HOST_DEVICE bool operator()(const T* const pose, T* residuals) const {
    const T s[3] = {T(sx), T(sy), T(sz)};
    T q[3];
    AngleAxisRotatePoint(pose, s, q);
    residuals[0] = q[0] + pose[3] - tx;
    residuals[1] = q[1] + pose[4] - ty;
    residuals[2] = q[2] + pose[5] - tz;
    return true;
  }
  double sx, sy, sz, tx, ty, tz;
};

// SoftLOneLoss (internal/ceres/loss_function.cc:66-73) as a LossFunctionCUDA.
class SoftLOneLossCUDA {
 public:
  HOST_DEVICE explicit SoftLOneLossCUDA(double a) : b_(a * a), c_(1 / b_) {}
  HOST_DEVICE void Evaluate(double s, double rho[3]) const {
    const double sum = 1.0 + s * c_;
    const double tmp = sqrt(sum);
    rho[0] = 2.0 * b_ * (tmp - 1.0);
    rho[1] = fmax(DBL_MIN, 1.0 / tmp);
    rho[2] = -(c_ * rho[1]) / (2.0 * sum);
  }

 private:
  double b_, c_;
};

// TolerantLoss (internal/ceres/loss_function.cc:93-118).
class TolerantLossCUDA {
 public:
  HOST_DEVICE TolerantLossCUDA(double a, double b) : a_(a), b_(b), c_(b * log(1.0 + exp(-a / b))) {}
  HOST_DEVICE void Evaluate(double s, double rho[3]) const {
    const double x = (s - a_) / b_;
    constexpr double kLog2Pow53 = 36.7;
    if (x > kLog2Pow53) {
      rho[0] = s - a_ - c_;
      rho[1] = 1.0;
      rho[2] = 0.0;
    } else {
      const double e_x = exp(x);
      rho[0] = b_ * log(1.0 + e_x) - c_;
      rho[1] = fmax(DBL_MIN, e_x / (1.0 + e_x));
      rho[2] = 0.5 / (b_ * (1.0 + cosh(x)));
    }
  }

 private:
  double a_, b_, c_;
};

}  // namespace user

#endif  // CSE_EXAMPLES_USER_FUNCTORS_H_
