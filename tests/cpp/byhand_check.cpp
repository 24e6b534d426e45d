// The Snavely camera's Jacobian by hand (SnavelyJacobianByHand, the device
// path of every Snavely kernel) against AutoDifferentiate through Jet<12>
// (the reference's form, include/ceres/internal/autodiff.h:314-381), on the
// host: random cameras over the whole angle range, theta == 0 exactly, tiny
// and large angles.  Prints the worst relative differences; exits 1 above
// the bound.
#include <cmath>
#include <cstdio>
#include <random>

#include "functors.hpp"

using namespace cse;

int main() {
  std::mt19937_64 rng(0xC0FFEE);
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  double worst_j = 0.0, worst_r = 0.0, worst_kind[5] = {0, 0, 0, 0, 0};
  int n = 0;
  for (int t = 0; t < 200000; ++t) {
    double cam[9], X[3], obs[2];
    const int kind = t % 5;
    const double scale = kind == 0 ? 0.0 : kind == 1 ? 1e-6 : kind == 2 ? 0.3 : kind == 3 ? 1.5 : 3.0;
    for (int k = 0; k < 3; ++k) cam[k] = scale * U(rng);
    for (int k = 3; k < 6; ++k) cam[k] = U(rng);
    cam[5] -= 5.0;  // points in front of the camera (Bundler: -z)
    cam[6] = 500.0 + 100.0 * U(rng);
    cam[7] = 1e-2 * U(rng);
    cam[8] = 1e-3 * U(rng);
    for (int k = 0; k < 3; ++k) X[k] = 2.0 * U(rng);
    obs[0] = 10.0 * U(rng);
    obs[1] = 10.0 * U(rng);
    double r[2], J0[18], J1[6];
    SnavelyJacobianByHand(obs, cam, X, r, J0, J1);
    Jet<12> jc[9], jp[3], out[2];
    for (int k = 0; k < 9; ++k) jc[k] = Jet<12>(cam[k], k);
    for (int k = 0; k < 3; ++k) jp[k] = Jet<12>(X[k], 9 + k);
    SnavelyKind::Evaluate(obs, jc, jp, out);
    for (int k = 0; k < 2; ++k) {
      double rownorm = 0.0;
      for (int c = 0; c < 12; ++c) rownorm = std::fmax(rownorm, std::fabs(out[k].v[c]));
      for (int c = 0; c < 12; ++c) {
        const double got = c < 9 ? J0[9 * k + c] : J1[3 * k + c - 9];
        const double d = std::fabs(got - out[k].v[c]) / (rownorm > 0 ? rownorm : 1.0);
        if (d > worst_kind[kind]) worst_kind[kind] = d;
        if (kind != 1 && d > worst_j) worst_j = d;
      }
      const double dr = std::fabs(r[k] - out[k].a) / std::fmax(1.0, std::fabs(out[k].a));
      if (dr > worst_r) worst_r = dr;
    }
    ++n;
  }
  std::printf("per angle class (theta 0, ~1e-6, ~0.3, ~1.5, ~3): %.2e %.2e %.2e %.2e %.2e\n",
              worst_kind[0], worst_kind[1], worst_kind[2], worst_kind[3], worst_kind[4]);
  std::printf("byhand_check: %d blocks, worst Jacobian difference %.3e of the row's largest entry, "
              "worst residual difference %.3e\n", n, worst_j, worst_r);
  return worst_j <= 1e-12 && worst_r <= 1e-12 ? 0 : 1;
}
