// jet.hpp -- forward-mode dual numbers for the gfx950 evaluator.
//
// Semantics follow Ceres' Jet<T, N> (include/ceres/jet.h:222-402 for the
// algebra, :533-537 abs, :617-646 sqrt/cos/sin, :742-760 three-argument
// hypot): a value `a` plus an N-vector of partials `v`.  Written for one
// wavefront lane per residual block: everything is a fixed-size, fully
// unrolled register array, never indexed at run time, so a Jet never
// spills to scratch.
//
// Structural zeros.  Seeds are unit vectors, so most partials of most
// intermediates are exact zeros at compile time (the rotation only sees the
// 3 angle-axis and 3 point partials, focal and distortion enter last).  The
// evaluator TU is compiled with -fno-signed-zeros -ffinite-math-only, which
// lets the compiler fold x*0 -> 0 and y+0 -> y on those lanes of the
// vector; for finite inputs this is bit-identical to the dense evaluation
// and removes roughly half of the FP64 work.
#ifndef CSE_JET_HPP_
#define CSE_JET_HPP_

#include <hip/hip_runtime.h>

namespace cse {

#define CSE_HD __host__ __device__ __forceinline__

template <int N>
struct Jet {
  double a;
  double v[N];

  CSE_HD Jet() : a(0.0) {
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = 0.0;
  }
  CSE_HD explicit Jet(double value) : a(value) {
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = 0.0;
  }
  // Value and every partial set to x (AutoDifferentiate's kImpossibleValue
  // pre-fill of the outputs, autodiff.h:355-360).
  static CSE_HD Jet Filled(double x) {
    Jet r; r.a = x;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = x;
    return r;
  }
  // The k-th infinitesimal seeded (autodiff.h:185-199).
  CSE_HD Jet(double value, int k) : a(value) {
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = (i == k) ? 1.0 : 0.0;
  }
  CSE_HD Jet& operator+=(const Jet& g) { return *this = *this + g; }
  CSE_HD Jet& operator-=(const Jet& g) { return *this = *this - g; }
  CSE_HD Jet& operator*=(const Jet& g) { return *this = *this * g; }

  friend CSE_HD Jet operator-(const Jet& f) {
    Jet r; r.a = -f.a;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = -f.v[i];
    return r;
  }
  friend CSE_HD Jet operator+(const Jet& f, const Jet& g) {
    Jet r; r.a = f.a + g.a;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = f.v[i] + g.v[i];
    return r;
  }
  friend CSE_HD Jet operator+(const Jet& f, double s) { Jet r = f; r.a = f.a + s; return r; }
  friend CSE_HD Jet operator+(double s, const Jet& f) { Jet r = f; r.a = f.a + s; return r; }
  friend CSE_HD Jet operator-(const Jet& f, const Jet& g) {
    Jet r; r.a = f.a - g.a;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = f.v[i] - g.v[i];
    return r;
  }
  friend CSE_HD Jet operator-(const Jet& f, double s) { Jet r = f; r.a = f.a - s; return r; }
  friend CSE_HD Jet operator-(double s, const Jet& f) {
    Jet r; r.a = s - f.a;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = -f.v[i];
    return r;
  }
  friend CSE_HD Jet operator*(const Jet& f, const Jet& g) {
    Jet r; r.a = f.a * g.a;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = f.a * g.v[i] + f.v[i] * g.a;
    return r;
  }
  friend CSE_HD Jet operator*(const Jet& f, double s) {
    Jet r; r.a = f.a * s;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = f.v[i] * s;
    return r;
  }
  friend CSE_HD Jet operator*(double s, const Jet& f) { return f * s; }
  // (a + u) / (b + v) = a/b + (u - (a/b) v) / b  (jet.h:378-390).
  friend CSE_HD Jet operator/(const Jet& f, const Jet& g) {
    const double g_inv = 1.0 / g.a;
    const double f_by_g = f.a * g_inv;
    Jet r; r.a = f_by_g;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = (f.v[i] - f_by_g * g.v[i]) * g_inv;
    return r;
  }
  // s / (b + v) = s/b - (s/b^2) v (jet.h:392-398), with one division: the
  // reciprocal of b is reused for the value and the partials.
  friend CSE_HD Jet operator/(double s, const Jet& g) {
    const double g_inv = 1.0 / g.a;
    Jet r; r.a = s * g_inv;
    const double m = -r.a * g_inv;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = g.v[i] * m;
    return r;
  }
  friend CSE_HD Jet operator/(const Jet& f, double s) { return f * (1.0 / s); }
};

// Scalar helpers so functors are written once for double and Jet.
CSE_HD double value_of(double x) { return x; }
template <int N> CSE_HD double value_of(const Jet<N>& x) { return x.a; }

CSE_HD double jsqrt(double x) { return sqrt(x); }
template <int N> CSE_HD Jet<N> jsqrt(const Jet<N>& f) {
  const double t = sqrt(f.a);
  const double two_a_inverse = 1.0 / (2.0 * t);
  Jet<N> r; r.a = t;
#pragma unroll
  for (int i = 0; i < N; ++i) r.v[i] = f.v[i] * two_a_inverse;
  return r;
}

CSE_HD double jabs(double x) { return fabs(x); }
template <int N> CSE_HD Jet<N> jabs(const Jet<N>& f) {
  const double s = copysign(1.0, f.a);
  Jet<N> r; r.a = fabs(f.a);
#pragma unroll
  for (int i = 0; i < N; ++i) r.v[i] = s * f.v[i];
  return r;
}

// sin and cos of one argument together (the reference calls sin and cos
// separately, jet.h:630-646).  On the device, when every lane of the wave has
// |x| <= pi/4 (angle-axis rotations of a few degrees, the usual BAL camera),
// no range reduction is needed and both come from the minimax polynomials of
// fdlibm's __kernel_sin / __kernel_cos (error below 1 ulp on [-pi/4, pi/4]):
// about 22 FP64 operations against about 50 for the library sincos, whose
// reduction step is an identity there.  The test is per lane, so a lane's
// result depends only on its own argument (a wave whose lanes all fall on one
// side runs that path alone).
CSE_HD void SinCosSmall(double x, double* s, double* c) {
  const double z = x * x, w = z * z;
  const double rs = 8.33333333332248946124e-03 + z * (-1.98412698298579493134e-04 +
                    z * 2.75573137070700676789e-06) +
                    z * w * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10);
  *s = x + (z * x) * (-1.66666666666666324348e-01 + z * rs);
  const double rc = z * (4.16666666666666019037e-02 + z * (-1.38888888888741095749e-03 +
                    z * 2.48015872894767294178e-05)) +
                    w * w * (-2.75573143513906633035e-07 + z * (2.08757232129817482790e-09 +
                    z * -1.13596475577881948265e-11));
  const double hz = 0.5 * z, one_m_hz = 1.0 - hz;
  *c = one_m_hz + (((1.0 - one_m_hz) - hz) + z * rc);
}
CSE_HD void SinCos(double x, double* s, double* c) {
#ifdef __HIP_DEVICE_COMPILE__
  if (fabs(x) <= 0.78539816339744828) {
    SinCosSmall(x, s, c);
    return;
  }
#endif
  sincos(x, s, c);
}
CSE_HD void jsincos(double x, double* s, double* c) { SinCos(x, s, c); }
template <int N> CSE_HD void jsincos(const Jet<N>& f, Jet<N>* s, Jet<N>* c) {
  double sa, ca;
  SinCos(f.a, &sa, &ca);
  s->a = sa;
  c->a = ca;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    s->v[i] = ca * f.v[i];
    c->v[i] = -sa * f.v[i];
  }
}

// |(x, y, z)| with the overflow-safe scaling of the reference's device
// hypot (include/ceres/internal/cudamath/cuda_math.h:48-63).
// Inside [2^-500, 2^500] no square can overflow or lose range, and the
// plain root of the sum of squares is used (no division); the scaled form
// serves the ends of the range.
CSE_HD double hypot3(double x, double y, double z) {
  const double px = fabs(x), py = fabs(y), pz = fabs(z);
  const double m = fmax(px, fmax(py, pz));
  if (m > 0x1p-500 && m < 0x1p500) return sqrt(x * x + y * y + z * z);
  if (m == 0.0) return 0.0;
  const double inv = 1.0 / m;
  const double sx = px * inv, sy = py * inv, sz = pz * inv;
  return m * sqrt(sx * sx + sy * sy + sz * sz);
}
CSE_HD double jhypot(double x, double y, double z) { return hypot3(x, y, z); }
template <int N> CSE_HD Jet<N> jhypot(const Jet<N>& x, const Jet<N>& y, const Jet<N>& z) {
  const double t = hypot3(x.a, y.a, z.a);
  const double t_inv = 1.0 / t;
  const double cx = x.a * t_inv, cy = y.a * t_inv, cz = z.a * t_inv;
  Jet<N> r; r.a = t;
#pragma unroll
  for (int i = 0; i < N; ++i) r.v[i] = cx * x.v[i] + cy * y.v[i] + cz * z.v[i];
  return r;
}

}  // namespace cse

#endif  // CSE_JET_HPP_
