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
#include <stdint.h>

#include <cmath>

namespace cse {

#define CSE_HD __host__ __device__ __forceinline__

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
  CSE_HD Jet& operator/=(const Jet& g) { return *this = *this / g; }
  CSE_HD Jet& operator+=(double s) { a += s; return *this; }
  CSE_HD Jet& operator-=(double s) { a -= s; return *this; }
  CSE_HD Jet& operator*=(double s) { return *this = *this * s; }
  CSE_HD Jet& operator/=(double s) { return *this = *this / s; }
  friend CSE_HD Jet operator+(const Jet& f) { return f; }

  // ---- The rest of Ceres' Jet surface (include/ceres/jet.h:405-1335), for
  // user functors (AddResidualBlock<F, ...>, include/ceres_amd/autodiff_cuda.h).
  // Hidden friends: found by argument-dependent lookup on a Jet only, so an
  // unqualified sqrt(x) on a double anywhere in namespace cse still means
  // ::sqrt.  The derivative formulas are the reference's, term for term.
#define CSE_JET_CMP(op)                                                                  \
  friend CSE_HD bool operator op(const Jet& f, const Jet& g) { return f.a op g.a; }      \
  friend CSE_HD bool operator op(const Jet& f, double s) { return f.a op s; }            \
  friend CSE_HD bool operator op(double s, const Jet& g) { return s op g.a; }
  CSE_JET_CMP(<)
  CSE_JET_CMP(<=)
  CSE_JET_CMP(>)
  CSE_JET_CMP(>=)
  CSE_JET_CMP(==)
  CSE_JET_CMP(!=)
#undef CSE_JET_CMP

  // a + s v (the reference's Jet(a, v) constructor with a scaled vector).
  static CSE_HD Jet Chain(double value, double s, const Jet& f) {
    Jet r; r.a = value;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = s * f.v[i];
    return r;
  }
  // a + s f.v + t g.v
  static CSE_HD Jet Chain2(double value, double s, const Jet& f, double t, const Jet& g) {
    Jet r; r.a = value;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = s * f.v[i] + t * g.v[i];
    return r;
  }

  friend CSE_HD Jet abs(const Jet& f) { return Chain(::fabs(f.a), ::copysign(1.0, f.a), f); }
  friend CSE_HD Jet copysign(const Jet& f, const Jet& g) {  // jet.h:560-575
    const double d = Bits(g.a) << 1 == 0 ? Infinity() : 0.0;
    const double sa = ::copysign(1.0, f.a), sb = ::copysign(1.0, g.a);
    return Chain2(::copysign(f.a, g.a), sa * sb, f, ::fabs(f.a) * d, g);
  }
  friend CSE_HD Jet log(const Jet& f) { return Chain(::log(f.a), 1.0 / f.a, f); }
  friend CSE_HD Jet log10(const Jet& f) { return Chain(::log10(f.a), 1.0 / (f.a * ::log(10.0)), f); }
  friend CSE_HD Jet log1p(const Jet& f) { return Chain(::log1p(f.a), 1.0 / (1.0 + f.a), f); }
  friend CSE_HD Jet exp(const Jet& f) {
    const double t = ::exp(f.a);
    return Chain(t, t, f);
  }
  friend CSE_HD Jet expm1(const Jet& f) {
    const double t = ::expm1(f.a);
    return Chain(t, t + 1.0, f);
  }
  friend CSE_HD Jet sqrt(const Jet& f) {
    const double t = ::sqrt(f.a);
    return Chain(t, 1.0 / (2.0 * t), f);
  }
  friend CSE_HD Jet cos(const Jet& f) { return Chain(::cos(f.a), -::sin(f.a), f); }
  friend CSE_HD Jet acos(const Jet& f) { return Chain(::acos(f.a), -1.0 / ::sqrt(1.0 - f.a * f.a), f); }
  friend CSE_HD Jet sin(const Jet& f) { return Chain(::sin(f.a), ::cos(f.a), f); }
  friend CSE_HD Jet asin(const Jet& f) { return Chain(::asin(f.a), 1.0 / ::sqrt(1.0 - f.a * f.a), f); }
  friend CSE_HD Jet tan(const Jet& f) {
    const double t = ::tan(f.a);
    return Chain(t, 1.0 + t * t, f);
  }
  friend CSE_HD Jet atan(const Jet& f) { return Chain(::atan(f.a), 1.0 / (1.0 + f.a * f.a), f); }
  friend CSE_HD Jet sinh(const Jet& f) { return Chain(::sinh(f.a), ::cosh(f.a), f); }
  friend CSE_HD Jet cosh(const Jet& f) { return Chain(::cosh(f.a), ::sinh(f.a), f); }
  friend CSE_HD Jet tanh(const Jet& f) {
    const double t = ::tanh(f.a);
    return Chain(t, 1.0 - t * t, f);
  }
  friend CSE_HD Jet floor(const Jet& f) { return Jet(::floor(f.a)); }
  friend CSE_HD Jet ceil(const Jet& f) { return Jet(::ceil(f.a)); }
  friend CSE_HD Jet cbrt(const Jet& f) { return Chain(::cbrt(f.a), 1.0 / (3.0 * ::cbrt(f.a * f.a)), f); }
  friend CSE_HD Jet exp2(const Jet& f) {
    const double t = ::exp2(f.a);
    return Chain(t, t * ::log(2.0), f);
  }
  friend CSE_HD Jet log2(const Jet& f) { return Chain(::log2(f.a), 1.0 / (f.a * ::log(2.0)), f); }
  friend CSE_HD Jet hypot(const Jet& x, const Jet& y) {
    const double t = ::hypot(x.a, y.a);
    return Chain2(t, x.a / t, x, y.a / t, y);
  }
  friend CSE_HD Jet hypot(const Jet& x, const Jet& y, const Jet& z) {
    const double t = hypot3(x.a, y.a, z.a);
    Jet r; r.a = t;
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = x.a / t * x.v[i] + y.a / t * y.v[i] + z.a / t * z.v[i];
    return r;
  }
  friend CSE_HD Jet fma(const Jet& x, const Jet& y, const Jet& z) {
    Jet r; r.a = ::fma(x.a, y.a, z.a);
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = y.a * x.v[i] + x.a * y.v[i] + z.v[i];
    return r;
  }
  // fmax / fmin (jet.h:800-840): NaNs are missing data, equal values give the
  // average of the two Jets.
  friend CSE_HD Jet fmax(const Jet& x, const Jet& y) {
    if (IsNan(x.a) || IsNan(y.a) || x.a != y.a) return IsNan(x.a) || x.a < y.a ? y : x;
    return (x + y) * 0.5;
  }
  friend CSE_HD Jet fmax(const Jet& x, double y) { return fmax(x, Jet(y)); }
  friend CSE_HD Jet fmax(double x, const Jet& y) { return fmax(Jet(x), y); }
  friend CSE_HD Jet fmin(const Jet& x, const Jet& y) {
    if (IsNan(x.a) || IsNan(y.a) || x.a != y.a) return IsNan(x.a) || x.a > y.a ? y : x;
    return (x + y) * 0.5;
  }
  friend CSE_HD Jet fmin(const Jet& x, double y) { return fmin(x, Jet(y)); }
  friend CSE_HD Jet fmin(double x, const Jet& y) { return fmin(Jet(x), y); }
  friend CSE_HD Jet fdim(const Jet& f, const Jet& g) {  // jet.h:842-851
    if (IsNan(f.a) || IsNan(g.a)) return Jet(QuietNan());
    return f.a > g.a ? f - g : Jet();
  }
  // 2 / sqrt(pi) written as the reference writes it (jet.h:856-868).
  friend CSE_HD Jet erf(const Jet& x) {
    const double e = ::exp(-x.a * x.a), c = 1.0 / ::sqrt(::atan(1.0));
    Jet r; r.a = ::erf(x.a);
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = x.v[i] * e * c;
    return r;
  }
  friend CSE_HD Jet erfc(const Jet& x) {
    const double e = ::exp(-x.a * x.a), c = 1.0 / ::sqrt(::atan(1.0));
    Jet r; r.a = ::erfc(x.a);
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = -x.v[i] * e * c;
    return r;
  }
  friend CSE_HD Jet BesselJ0(const Jet& f) { return Chain(::j0(f.a), -::j1(f.a), f); }
  friend CSE_HD Jet BesselJ1(const Jet& f) { return Chain(::j1(f.a), 0.5 * (::j0(f.a) - ::jn(2, f.a)), f); }
  friend CSE_HD Jet BesselJn(int n, const Jet& f) {
    return Chain(::jn(n, f.a), 0.5 * (::jn(n - 1, f.a) - ::jn(n + 1, f.a)), f);
  }
  friend CSE_HD Jet atan2(const Jet& g, const Jet& f) {  // jet.h:1165-1176
    const double t = 1.0 / (f.a * f.a + g.a * g.a);
    Jet r; r.a = ::atan2(g.a, f.a);
#pragma unroll
    for (int i = 0; i < N; ++i) r.v[i] = t * (-g.a * f.v[i] + f.a * g.v[i]);
    return r;
  }
  friend CSE_HD Jet norm(const Jet& f) { return Chain(f.a * f.a, 2.0 * f.a, f); }
  friend CSE_HD Jet pow(const Jet& f, double g) { return Chain(::pow(f.a, g), g * ::pow(f.a, g - 1.0), f); }
  // pow(double, Jet) and pow(Jet, Jet) with the reference's special cases
  // (jet.h:1195-1340).
  friend CSE_HD Jet pow(double f, const Jet& g) {
    if (f == 0.0 && g.a > 0.0) return Jet(0.0);
    if (f < 0.0 && g.a == ::floor(g.a)) {
      Jet r(::pow(f, g.a));
#pragma unroll
      for (int i = 0; i < N; ++i)
        if (g.v[i] != 0.0) r.v[i] = QuietNan();
      return r;
    }
    const double t = ::pow(f, g.a);
    return Chain(t, ::log(f) * t, g);
  }
  friend CSE_HD Jet pow(const Jet& f, const Jet& g) {
    if (f.a == 0.0 && g.a >= 1.0) return g.a > 1.0 ? Jet(0.0) : f;
    if (f.a < 0.0 && g.a == ::floor(g.a)) {
      Jet r = Chain(::pow(f.a, g.a), g.a * ::pow(f.a, g.a - 1.0), f);
#pragma unroll
      for (int i = 0; i < N; ++i)
        if (g.v[i] != 0.0) r.v[i] = QuietNan();
      return r;
    }
    const double t1 = ::pow(f.a, g.a), t2 = g.a * ::pow(f.a, g.a - 1.0), t3 = t1 * ::log(f.a);
    return Chain2(t1, t2, f, t3, g);
  }
  // Classification of the value (jet.h:1010-1110), by the bit pattern: the
  // evaluator TUs are built with -ffinite-math-only, under which the library
  // isfinite/isnan fold to constants.
  static CSE_HD uint64_t Bits(double x) { return __builtin_bit_cast(uint64_t, x); }
  static CSE_HD double QuietNan() { return __builtin_bit_cast(double, 0x7ff8000000000000ull); }
  static CSE_HD double Infinity() { return __builtin_bit_cast(double, 0x7ff0000000000000ull); }
  static CSE_HD bool IsNan(double x) { return (Bits(x) << 1) > (0x7ffull << 53); }
  friend CSE_HD bool isfinite(const Jet& f) { return ((Bits(f.a) >> 52) & 0x7ff) != 0x7ff; }
  friend CSE_HD bool isinf(const Jet& f) { return (Bits(f.a) << 1) == (0x7ffull << 53); }
  friend CSE_HD bool isnan(const Jet& f) { return IsNan(f.a); }
  friend CSE_HD bool isnormal(const Jet& f) {
    const uint64_t e = (Bits(f.a) >> 52) & 0x7ff;
    return e != 0 && e != 0x7ff;
  }
  friend CSE_HD bool signbit(const Jet& f) { return (Bits(f.a) >> 63) != 0; }
  friend CSE_HD int fpclassify(const Jet& f) {
    const uint64_t e = (Bits(f.a) >> 52) & 0x7ff, m = Bits(f.a) & ((1ull << 52) - 1);
    if (e == 0x7ff) return m ? FP_NAN : FP_INFINITE;
    if (e == 0) return m ? FP_SUBNORMAL : FP_ZERO;
    return FP_NORMAL;
  }
  friend CSE_HD bool isless(const Jet& f, const Jet& g) { return f.a < g.a; }
  friend CSE_HD bool isgreater(const Jet& f, const Jet& g) { return f.a > g.a; }
  friend CSE_HD bool islessequal(const Jet& f, const Jet& g) { return f.a <= g.a; }
  friend CSE_HD bool isgreaterequal(const Jet& f, const Jet& g) { return f.a >= g.a; }
  friend CSE_HD bool islessgreater(const Jet& f, const Jet& g) { return f.a < g.a || f.a > g.a; }
  friend CSE_HD bool isunordered(const Jet& f, const Jet& g) { return IsNan(f.a) || IsNan(g.a); }
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
