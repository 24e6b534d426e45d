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
  friend CSE_HD Jet operator/(double s, const Jet& g) {
    const double m = -s / (g.a * g.a);
    Jet r; r.a = s / g.a;
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

// sin and cos of the same argument share one range reduction on the device
// (the reference calls sin and cos separately, jet.h:630-646).
CSE_HD void jsincos(double x, double* s, double* c) { sincos(x, s, c); }
template <int N> CSE_HD void jsincos(const Jet<N>& f, Jet<N>* s, Jet<N>* c) {
  double sa, ca;
  sincos(f.a, &sa, &ca);
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
CSE_HD double hypot3(double x, double y, double z) {
  const double px = fabs(x), py = fabs(y), pz = fabs(z);
  const double m = fmax(px, fmax(py, pz));
  if (m == 0.0) return 0.0;
  const double inv = 1.0 / m;
  const double sx = px * inv, sy = py * inv, sz = pz * inv;
  return m * sqrt(sx * sx + sy * sy + sz * sz);
}
CSE_HD double jhypot(double x, double y, double z) { return hypot3(x, y, z); }
template <int N> CSE_HD Jet<N> jhypot(const Jet<N>& x, const Jet<N>& y, const Jet<N>& z) {
  const double t = hypot3(x.a, y.a, z.a);
  const double cx = x.a / t, cy = y.a / t, cz = z.a / t;
  Jet<N> r; r.a = t;
#pragma unroll
  for (int i = 0; i < N; ++i) r.v[i] = cx * x.v[i] + cy * y.v[i] + cz * z.v[i];
  return r;
}

}  // namespace cse

#endif  // CSE_JET_HPP_
