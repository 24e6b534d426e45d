// Prints the noise stream of BALProblem::Perturb's random-number usage
// (examples/bal_problem.cc:58-62,289-330) with the C++ standard library's
// own std::mt19937 and std::normal_distribution: a fresh copy of the
// distribution per PerturbPoint3 call (std::bind copies it).  Used by
// tests/test_bal_tools.py to pin ceres_amd.bal.perturb's restatement.
// Not reference code: only the standard library's generators.
#include <cstdio>
#include <functional>
#include <random>

static void Draw3(std::function<double()> dist, double* out) {
  for (int i = 0; i < 3; ++i) out[i] = dist();
}

int main() {
  std::mt19937 prng;
  std::normal_distribution<double> a(0.0, 0.5), b(0.0, 2.0);
  double v[3];
  for (int k = 0; k < 4; ++k) {
    Draw3(std::bind(a, std::ref(prng)), v);
    std::printf("%.17g %.17g %.17g\n", v[0], v[1], v[2]);
    Draw3(std::bind(b, std::ref(prng)), v);
    std::printf("%.17g %.17g %.17g\n", v[0], v[1], v[2]);
  }
  return 0;
}
