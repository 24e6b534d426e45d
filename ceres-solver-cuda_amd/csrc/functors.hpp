// functors.hpp -- residual functors pre-instantiated in the gfx950 library.
//
// Each functor kind carries its shape (kNumResiduals, parameter block
// sizes, functor-data size) as compile-time traits and one templated
// Evaluate(data, params, residuals) written for T in {double, Jet<N>}, the
// same contract as a Ceres AutoDiffCostFunction functor
// (include/ceres/autodiff_cost_function.h:201-217).
#ifndef CSE_FUNCTORS_HPP_
#define CSE_FUNCTORS_HPP_

#include <type_traits>

#include "jet.hpp"

namespace cse {

// Every kind also offers EvaluateFlat(data, x, r) over its parameter blocks
// concatenated in slot order (x = [block 0 | block 1 | ...]); the general
// (table) kernel calls that form, which covers kinds with any number of
// parameter blocks.  Two-slot kinds forward to their Evaluate.
#define CSE_FLAT_FROM_TWO_SLOTS                                              \
  template <typename T>                                                      \
  static CSE_HD bool EvaluateFlat(const double* d, const T* x, T* r) {       \
    return Evaluate(d, x, x + kSize0, r);                                    \
  }

// The Rodrigues factors as functions of u = theta^2:
//   s(u) = sin(theta) / theta,   c(u) = (1 - cos(theta)) / theta^2,
// and their u-derivatives, from their Taylor series (coefficients
// (-1)^n / (2n+1)! and (-1)^n / (2n+2)!, rounded to double).  For
// 0 <= u <= 1 the terms fall by a factor u / 6 or more and the first one
// left out is below 1e-17 of the sum, so each is within an ulp or two.
CSE_HD void RodriguesFactors(double u, double* s, double* c, double* ds, double* dc) {
  *s = 1.0 + u * (-0.16666666666666666 + u * (0.0083333333333333332 + u * (-0.00019841269841269841 +
       u * (2.7557319223985893e-06 + u * (-2.505210838544172e-08 + u * (1.6059043836821613e-10 +
       u * (-7.6471637318198164e-13 + u * 2.8114572543455206e-15)))))));
  *c = 0.5 + u * (-0.041666666666666664 + u * (0.0013888888888888889 + u * (-2.4801587301587302e-05 +
       u * (2.7557319223985888e-07 + u * (-2.08767569878681e-09 + u * (1.1470745597729725e-11 +
       u * (-4.7794773323873853e-14 + u * 1.5619206968586225e-16)))))));
  *ds = -0.16666666666666666 + u * (0.016666666666666666 + u * (-0.00059523809523809529 +
        u * (1.1022927689594357e-05 + u * (-1.2526054192720859e-07 + u * (9.6354263020929685e-10 +
        u * (-5.3530146122738714e-12 + u * 2.2491658034764165e-14))))));
  *dc = -0.041666666666666664 + u * (0.0027777777777777779 + u * (-7.4404761904761911e-05 +
        u * (1.1022927689594355e-06 + u * (-1.043837849393405e-08 + u * (6.882447358637835e-11 +
        u * (-3.3456341326711696e-13 + u * 1.249536557486898e-15))))));
}
CSE_HD void RodriguesFactors(double u, double* s, double* c) {
  double ds, dc;
  RodriguesFactors(u, s, c, &ds, &dc);  // the derivatives are dead code here
}
template <int N>
CSE_HD void RodriguesFactors(const Jet<N>& u, Jet<N>* s, Jet<N>* c) {
  double ds, dc;
  RodriguesFactors(u.a, &s->a, &c->a, &ds, &dc);
#pragma unroll
  for (int i = 0; i < N; ++i) {
    s->v[i] = ds * u.v[i];
    c->v[i] = dc * u.v[i];
  }
}

// y = R(angle_axis) x  (include/ceres/rotation.h:830-899): Rodrigues away
// from theta == 0, the first-order form R = I + hat(w) exactly at zero so
// Jets still carry the right derivatives.
//
// On the device, a lane whose theta^2 <= 1 (rotations of up to 57 degrees,
// the usual BAL camera) evaluates the same rotation as
//   R x = x + s(theta^2) (w x x) + c(theta^2) (w x (w x x)),  w = angle_axis,
// Rodrigues' formula with sin(theta)/theta and (1 - cos(theta))/theta^2 as
// series in theta^2 (RodriguesFactors): no square root, no division, no
// sine or cosine, and the cross products of the seeded Jets carry their
// partials as plain copies.  At theta == 0 it is exactly the reference's
// first-order form (s = 1, c = 1/2, and the c term vanishes with its
// derivatives), so both branches of the reference are covered.  The form is
// chosen per lane, from the block's own camera: a block's outputs do not
// depend on which blocks share its wave (a sharded evaluation writes the
// same bits as the whole-problem one, and the camera-order gradient
// re-evaluation takes the same form as the point-order evaluation).  A wave
// whose lanes all fall on one side runs that form alone (the other is
// skipped on an empty exec mask); a mixed wave runs both.
template <typename T>
CSE_HD void AngleAxisRotatePoint(const T aa[3], const T pt[3], T out[3]) {
#ifdef __HIP_DEVICE_COMPILE__
  {
    const T u = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
    if (value_of(u) <= 1.0) {
      T s, c;
      RodriguesFactors(u, &s, &c);
      const T q[3] = {aa[1] * pt[2] - aa[2] * pt[1],
                      aa[2] * pt[0] - aa[0] * pt[2],
                      aa[0] * pt[1] - aa[1] * pt[0]};
      const T m[3] = {aa[1] * q[2] - aa[2] * q[1],
                      aa[2] * q[0] - aa[0] * q[2],
                      aa[0] * q[1] - aa[1] * q[0]};
      out[0] = pt[0] + s * q[0] + c * m[0];
      out[1] = pt[1] + s * q[1] + c * m[1];
      out[2] = pt[2] + s * q[2] + c * m[2];
      return;
    }
  }
#endif
  const T theta = jhypot(aa[0], aa[1], aa[2]);
  if (value_of(theta) != 0.0) {
    T sintheta, costheta;
    jsincos(theta, &sintheta, &costheta);
    const T theta_inverse = T(1.0) / theta;
    const T w[3] = {aa[0] * theta_inverse, aa[1] * theta_inverse, aa[2] * theta_inverse};
    const T w_cross_pt[3] = {w[1] * pt[2] - w[2] * pt[1],
                             w[2] * pt[0] - w[0] * pt[2],
                             w[0] * pt[1] - w[1] * pt[0]};
    const T tmp = (w[0] * pt[0] + w[1] * pt[1] + w[2] * pt[2]) * (T(1.0) - costheta);
    out[0] = pt[0] * costheta + w_cross_pt[0] * sintheta + w[0] * tmp;
    out[1] = pt[1] * costheta + w_cross_pt[1] * sintheta + w[1] * tmp;
    out[2] = pt[2] * costheta + w_cross_pt[2] * sintheta + w[2] * tmp;
  } else {
    out[0] = pt[0] + (aa[1] * pt[2] - aa[2] * pt[1]);
    out[1] = pt[1] + (aa[2] * pt[0] - aa[0] * pt[2]);
    out[2] = pt[2] + (aa[0] * pt[1] - aa[1] * pt[0]);
  }
}

// y = R(q) x for a not necessarily unit quaternion
// (include/ceres/rotation.h:753-798).
template <typename T>
CSE_HD void QuaternionRotatePoint(const T q[4], const T pt[3], T out[3]) {
  const T scale = T(1.0) / jsqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  const T u[4] = {scale * q[0], scale * q[1], scale * q[2], scale * q[3]};
  T uv0 = u[2] * pt[2] - u[3] * pt[1];
  T uv1 = u[3] * pt[0] - u[1] * pt[2];
  T uv2 = u[1] * pt[1] - u[2] * pt[0];
  uv0 += uv0;
  uv1 += uv1;
  uv2 += uv2;
  out[0] = pt[0] + u[0] * uv0;
  out[1] = pt[1] + u[0] * uv1;
  out[2] = pt[2] + u[0] * uv2;
  out[0] += u[2] * uv2 - u[3] * uv1;
  out[1] += u[3] * uv0 - u[1] * uv2;
  out[2] += u[1] * uv1 - u[2] * uv0;
}

// Pinhole camera with the Bundler sign convention, optional radial
// distortion (examples/snavely_reprojection_error.h:58-93).
template <bool kDistortion, typename T>
CSE_HD void Project(const T p[3], const T& focal, const T* l, const double* obs, T* r) {
  T xp, yp;
  if constexpr (std::is_same<T, double>::value) {
    const double neg_inv = -1.0 / p[2];  // one division for both coordinates
    xp = p[0] * neg_inv;
    yp = p[1] * neg_inv;
  } else {  // Jet division already shares 1 / p[2].a
    xp = -p[0] / p[2];
    yp = -p[1] / p[2];
  }
  if constexpr (kDistortion) {
    const T r2 = xp * xp + yp * yp;
    const T distortion = 1.0 + r2 * (l[0] + l[1] * r2);
    r[0] = focal * distortion * xp - obs[0];
    r[1] = focal * distortion * yp - obs[1];
  } else {
    r[0] = focal * xp - obs[0];
    r[1] = focal * yp - obs[1];
  }
}

// SnavelyReprojectionError<2, 9, 3>: camera = {aa[3], t[3], f, l1, l2}.
struct SnavelyKind {
  static constexpr int kNumResiduals = 2;
  static constexpr int kNumBlocks = 2;
  static constexpr int kSize0 = 9, kSize1 = 3;
  static constexpr int kSizes[2] = {9, 3};
  static constexpr int kDataSize = 2;
  template <typename T>
  static CSE_HD bool Evaluate(const double* obs, const T* camera, const T* point, T* r) {
    T p[3];
    AngleAxisRotatePoint(camera, point, p);
    p[0] += camera[3];
    p[1] += camera[4];
    p[2] += camera[5];
    Project<true>(p, camera[6], camera + 7, obs, r);
    return true;
  }
  CSE_FLAT_FROM_TWO_SLOTS
};

// The same functor with its Jacobian by forward-mode Jet<double, 12>, as
// AutoDifferentiate computes it (include/ceres/internal/autodiff.h:314-381;
// AutoDiffCostFunction, autodiff_cost_function_cuda.h:55-71), instead of
// SnavelyJacobianByHand: cse_options.jacobian_form = CSE_JACOBIAN_JET.  A
// distinct type so that the kernels' by-hand dispatch (is_same<K,
// SnavelyKind>) passes it by; instantiated in its own TU (jet_kernels.hip).
struct SnavelyJetKind : SnavelyKind {};

// SnavelyReprojectionError's residuals and Jacobian blocks written out by
// hand (the product rule the seeded Jet<12> applies, collected into 3x3
// matrices): J0 = dr/d[aa, t, f, l1, l2] (2 x 9), J1 = dr/dX (2 x 3), both
// row-major.  The primal follows Evaluate<double> operation for operation.
// With p = X + s q + c m + t, q = aa x X, m = aa x q, u = |aa|^2,
// s(u) = sin(theta)/theta, c(u) = (1 - cos(theta))/theta^2:
//   dp/dX  = R = (1 - c u) I + s [aa]x + c aa aa^T,
//   dp/daa = G = w aa^T + c (aa.X) I - [z]x,
//            w = 2 (s' q + c' m) - c X,  z = s X + c q   (s' = ds/du),
// exact for every theta: at theta == 0 (s, c, s', c') = (1, 1/2, -1/6, -1/24)
// give R = I and G = -[X]x, the reference's first-order form.  Then with
// (xp, yp) = -p_xy / p_z, D = 1 + r2 (l1 + l2 r2):
//   dr/dp = A B,  A = f (D I + (2 l1 + 4 l2 r2) x x^T),  B = [ni I | ni x],
// ni = -1/p_z, and J0 = [H G | H | D x | f r2 x | f r2^2 x], J1 = H R.
CSE_HD bool SnavelyJacobianByHand(const double* obs, const double* cam, const double* X, double* r,
                                  double* J0, double* J1) {
  const double a0 = cam[0], a1 = cam[1], a2 = cam[2];
  const double u = a0 * a0 + a1 * a1 + a2 * a2;
  double s, c, ds, dc, p[3];
  // q = aa x X and m = aa x q (the series form's vectors; also G's)
  const double q0 = a1 * X[2] - a2 * X[1], q1 = a2 * X[0] - a0 * X[2], q2 = a0 * X[1] - a1 * X[0];
  const double m0 = a1 * q2 - a2 * q1, m1 = a2 * q0 - a0 * q2, m2 = a0 * q1 - a1 * q0;
  if (u <= 1.0) {
    RodriguesFactors(u, &s, &c, &ds, &dc);
    p[0] = X[0] + s * q0 + c * m0;
    p[1] = X[1] + s * q1 + c * m1;
    p[2] = X[2] + s * q2 + c * m2;
  } else {  // AngleAxisRotatePoint's Rodrigues branch for the value
    const double theta = jhypot(a0, a1, a2);
    double st, ct;
    jsincos(theta, &st, &ct);
    const double ti = 1.0 / theta;
    const double w0 = a0 * ti, w1 = a1 * ti, w2 = a2 * ti;
    const double x0 = w1 * X[2] - w2 * X[1], x1 = w2 * X[0] - w0 * X[2], x2 = w0 * X[1] - w1 * X[0];
    const double tmp = (w0 * X[0] + w1 * X[1] + w2 * X[2]) * (1.0 - ct);
    p[0] = X[0] * ct + x0 * st + w0 * tmp;
    p[1] = X[1] * ct + x1 * st + w1 * tmp;
    p[2] = X[2] * ct + x2 * st + w2 * tmp;
    s = st * ti;
    c = (1.0 - ct) / u;
    ds = (ct - s) / (2.0 * u);
    dc = (s - 2.0 * c) / (2.0 * u);
  }
  p[0] += cam[3];
  p[1] += cam[4];
  p[2] += cam[5];
  // Project<true, double>
  const double ni = -1.0 / p[2];
  const double xp = p[0] * ni, yp = p[1] * ni;
  const double f = cam[6], l1 = cam[7], l2 = cam[8];
  const double r2 = xp * xp + yp * yp;
  const double D = 1.0 + r2 * (l1 + l2 * r2);
  r[0] = f * D * xp - obs[0];
  r[1] = f * D * yp - obs[1];
  // H = dr/dp
  const double fD = f * D, fg = f * (2.0 * l1 + 4.0 * l2 * r2);
  const double A00 = fD + fg * xp * xp, A01 = fg * xp * yp, A11 = fD + fg * yp * yp;
  double H[2][3];
  H[0][0] = A00 * ni;
  H[0][1] = A01 * ni;
  H[0][2] = (A00 * xp + A01 * yp) * ni;
  H[1][0] = A01 * ni;
  H[1][1] = A11 * ni;
  H[1][2] = (A01 * xp + A11 * yp) * ni;
  // R and G
  const double cu1 = 1.0 - c * u;
  const double R[3][3] = {{cu1 + c * a0 * a0, c * a0 * a1 - s * a2, c * a0 * a2 + s * a1},
                          {c * a1 * a0 + s * a2, cu1 + c * a1 * a1, c * a1 * a2 - s * a0},
                          {c * a2 * a0 - s * a1, c * a2 * a1 + s * a0, cu1 + c * a2 * a2}};
  const double d = a0 * X[0] + a1 * X[1] + a2 * X[2], cd = c * d;
  const double w0 = 2.0 * (ds * q0 + dc * m0) - c * X[0];
  const double w1 = 2.0 * (ds * q1 + dc * m1) - c * X[1];
  const double w2 = 2.0 * (ds * q2 + dc * m2) - c * X[2];
  const double z0 = s * X[0] + c * q0, z1 = s * X[1] + c * q1, z2 = s * X[2] + c * q2;
  const double G[3][3] = {{w0 * a0 + cd, w0 * a1 + z2, w0 * a2 - z1},
                          {w1 * a0 - z2, w1 * a1 + cd, w1 * a2 + z0},
                          {w2 * a0 + z1, w2 * a1 - z0, w2 * a2 + cd}};
  const double xy[2] = {xp, yp};
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    double* row = J0 + 9 * k;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      row[j] = H[k][0] * G[0][j] + H[k][1] * G[1][j] + H[k][2] * G[2][j];
      row[3 + j] = H[k][j];
      J1[3 * k + j] = H[k][0] * R[0][j] + H[k][1] * R[1][j] + H[k][2] * R[2][j];
    }
    row[6] = D * xy[k];
    row[7] = f * r2 * xy[k];
    row[8] = f * r2 * r2 * xy[k];
  }
  return true;
}

// SnavelyReprojectionErrorNoRadialDistortion<2, 7, 3>
// (internal/ceres/evaluator_cuda_test.cu.cc:112-150).
struct SnavelyNoDistortionKind {
  static constexpr int kNumResiduals = 2;
  static constexpr int kNumBlocks = 2;
  static constexpr int kSize0 = 7, kSize1 = 3;
  static constexpr int kSizes[2] = {7, 3};
  static constexpr int kDataSize = 2;
  template <typename T>
  static CSE_HD bool Evaluate(const double* obs, const T* camera, const T* point, T* r) {
    T p[3];
    AngleAxisRotatePoint(camera, point, p);
    p[0] += camera[3];
    p[1] += camera[4];
    p[2] += camera[5];
    Project<false>(p, camera[6], camera, obs, r);
    return true;
  }
  CSE_FLAT_FROM_TWO_SLOTS
};

// SnavelyReprojectionErrorWithQuaternions<2, 10, 3>: camera =
// {q[4], t[3], f, l1, l2} (examples/snavely_reprojection_error.h:112-175).
struct SnavelyQuaternionKind {
  static constexpr int kNumResiduals = 2;
  static constexpr int kNumBlocks = 2;
  static constexpr int kSize0 = 10, kSize1 = 3;
  static constexpr int kSizes[2] = {10, 3};
  static constexpr int kDataSize = 2;
  template <typename T>
  static CSE_HD bool Evaluate(const double* obs, const T* camera, const T* point, T* r) {
    T p[3];
    QuaternionRotatePoint(camera, point, p);
    p[0] += camera[4];
    p[1] += camera[5];
    p[2] += camera[6];
    Project<true>(p, camera[7], camera + 8, obs, r);
    return true;
  }
  CSE_FLAT_FROM_TWO_SLOTS
};

// One row of an ambient Jacobian (kS columns) of a block on
// ProductManifold<QuaternionManifold, EuclideanManifold<kS - 4>> times the
// manifold's plus-Jacobian: the 4 x 3 QuaternionPlusJacobianImpl of
// q = x[0..4) (internal/ceres/manifold.cc:62-78, Ceres order w, x, y, z)
// and an identity for the Euclidean part, block-diagonal
// (product_manifold.h).  out has kS - 1 columns.  Each sum adds the nonzero
// terms in the order of the dense product (residual_block.cc:133-156), so
// the result equals that product with the explicit matrix up to the sign of
// zeros.
template <int kS>
CSE_HD void QuaternionEuclideanTangentRow(const double* x, const double* amb, double* out) {
  static_assert(kS >= 4, "quaternion first");
  const double w = x[0], qx = x[1], qy = x[2], qz = x[3];
  const double P[4][3] = {{-qx, -qy, -qz}, {w, qz, -qy}, {-qz, w, qx}, {qy, -qx, w}};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    double s = 0.0;
#pragma unroll
    for (int m = 0; m < 4; ++m) s += amb[m] * P[m][c];
    out[c] = s;
  }
#pragma unroll
  for (int c = 3; c < kS - 1; ++c) out[c] = amb[c + 1];
}

// SnavelyQuaternionKind with its camera on ProductManifold<QuaternionManifold,
// EuclideanManifold<6>> (CSE_MANIFOLD_QUATERNION_EUCLIDEAN; the
// --use_quaternions --use_manifolds problem of examples/bundle_adjuster.cc:
// 337-345): the affine kernels gather the 10 ambient camera values
// (kAmbient0) and write the 9 tangent Jacobian columns (kSize0), as the
// 9-parameter Snavely camera.  Affine kernels only (no flat form).
struct SnavelyQuaternionTangentKind {
  static constexpr int kNumResiduals = 2;
  static constexpr int kNumBlocks = 2;
  static constexpr int kSize0 = 9, kSize1 = 3;
  static constexpr int kAmbient0 = 10;
  static constexpr int kSizes[2] = {9, 3};
  static constexpr int kDataSize = 2;
  static constexpr bool kAffineOnly = true;
  template <typename T>
  static CSE_HD bool Evaluate(const double* obs, const T* camera, const T* point, T* r) {
    return SnavelyQuaternionKind::Evaluate(obs, camera, point, r);
  }
  static CSE_HD void TangentRow(const double* x0, const double* amb, double* out) {
    QuaternionEuclideanTangentRow<10>(x0, amb, out);
  }
};

// PointDisplacementError<3, 3> (internal/ceres/evaluator_cuda_test.cu.cc:84-110).
struct PointDisplacementKind {
  static constexpr int kNumResiduals = 3;
  static constexpr int kNumBlocks = 1;
  static constexpr int kSize0 = 3, kSize1 = 0;
  static constexpr int kSizes[1] = {3};
  static constexpr int kDataSize = 3;
  template <typename T>
  static CSE_HD bool Evaluate(const double* xyz, const T* point, const T*, T* r) {
    r[0] = fabs(xyz[0]) - jabs(point[0]);
    r[1] = fabs(xyz[1]) - jabs(point[1]);
    r[2] = fabs(xyz[2]) - jabs(point[2]);
    return true;
  }
  template <typename T>
  static CSE_HD bool EvaluateFlat(const double* xyz, const T* x, T* r) {
    return Evaluate(xyz, x, x, r);
  }
};

// ---------------------------------------------------------------------------
// Functors of the reference's own known-answer tests.  They are built into
// the library so that those tests run through the product kernels (the
// general/table path; cse_functor_kind values 100+).  Not used by BAL.
// ---------------------------------------------------------------------------

// ParameterIgnoringCostFunction<kFactor, kR, Ns...>
// (internal/ceres/evaluator_test.cc:58-100) written as the linear functor
//   r_i = (i + 1) + kFactor * sum_b sum_j (j + 1) x_b[j]:
// at the zero state the reference's test evaluates at, its value i + 1 and
// its Jacobian columns kFactor * (j + 1) are exactly what the fake returns.
// data = {kFactor, succeeds}; succeeds == 0 makes the functor return false
// (EvaluatorAbortsForResidualsThatFailToEvaluate, :535-553).
template <int kR, int... Ns>
struct LinearTestKind {
  static constexpr int kNumResiduals = kR;
  static constexpr int kNumBlocks = sizeof...(Ns);
  static constexpr bool kTestOnly = true;
  static constexpr int kSizes[kNumBlocks] = {Ns...};
  static constexpr int kSize0 = kSizes[0], kSize1 = kNumBlocks > 1 ? kSizes[1] : 0;
  static constexpr int kDataSize = 2;
  template <typename T>
  static CSE_HD bool EvaluateFlat(const double* d, const T* x, T* r) {
    T acc(0.0);
    int q = 0;
#pragma unroll
    for (int b = 0; b < kNumBlocks; ++b)
#pragma unroll
      for (int j = 0; j < kSizes[b]; ++j, ++q) acc = acc + (double)(j + 1) * x[q];
#pragma unroll
    for (int i = 0; i < kR; ++i) r[i] = (double)(i + 1) + d[0] * acc;
    return d[1] != 0.0;
  }
};

// BinaryScalarCost (internal/ceres/autodiff_cost_function_cuda_test.cu.cc:40-51):
// cost = x0 y0 + x1 y1 - a, parameter blocks x[2], y[2]; data = {a}.
struct BilinearTestKind {
  static constexpr bool kTestOnly = true;
  static constexpr int kNumResiduals = 1;
  static constexpr int kNumBlocks = 2;
  static constexpr int kSizes[2] = {2, 2};
  static constexpr int kSize0 = 2, kSize1 = 2;
  static constexpr int kDataSize = 1;
  template <typename T>
  static CSE_HD bool EvaluateFlat(const double* d, const T* x, T* r) {
    r[0] = x[0] * x[2] + x[1] * x[3] - d[0];
    return true;
  }
};

// TenParameterCost (autodiff_cost_function_cuda_test.cu.cc:123-139): ten
// parameter blocks of size one, cost = x0 + ... + x9.  The functor has no
// constants; its one data double is unused.
struct TenParameterTestKind {
  static constexpr bool kTestOnly = true;
  static constexpr int kNumResiduals = 1;
  static constexpr int kNumBlocks = 10;
  static constexpr int kSizes[10] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1};
  static constexpr int kSize0 = 1, kSize1 = 1;
  static constexpr int kDataSize = 1;
  template <typename T>
  static CSE_HD bool EvaluateFlat(const double*, const T* x, T* r) {
    r[0] = x[0] + x[1] + x[2] + x[3] + x[4] + x[5] + x[6] + x[7] + x[8] + x[9];
    return true;
  }
};

// OnlyFillsOneOutputFunctor (autodiff_cost_function_cuda_test.cu.cc:224-230):
// two residuals, only the first assigned.  AutoDifferentiate pre-fills the
// outputs with kImpossibleValue (include/ceres/internal/autodiff.h:355-360)
// and ResidualBlock::Evaluate rejects them (residual_block.cc:146-152,
// array_utils.cc:44-53), so the evaluation fails.
struct PartialOutputTestKind {
  static constexpr bool kTestOnly = true;
  static constexpr int kNumResiduals = 2;
  static constexpr int kNumBlocks = 1;
  static constexpr int kSizes[1] = {1};
  static constexpr int kSize0 = 1, kSize1 = 0;
  static constexpr int kDataSize = 1;
  static constexpr bool kMayLeaveOutputs = true;
  template <typename T>
  static CSE_HD bool EvaluateFlat(const double*, const T* x, T* r) {
    r[0] = x[0];
    return true;
  }
};

}  // namespace cse

#endif  // CSE_FUNCTORS_HPP_
