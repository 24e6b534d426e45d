// C++ parity test of the ProblemCUDA facade (ceres-solver-cuda_amd/include/
// ceres_amd/problem_cuda.h) against the CPU oracle, restating
// internal/ceres/evaluator_cuda_test.cu.cc:232-459: a 6-residual-block
// bundle adjustment problem with three functor types, Cauchy/Huber/no loss,
// two constant blocks and a ProductManifold<Quaternion, Euclidean<6>>
// camera, evaluated into a BlockSparseMatrix and a CompressedRowSparseMatrix.
// Tolerance: the reference's kTolerance = 1e-13 (isApprox per vector).
//
// Needs a GPU (run by tests/test_cpp_facade.py under -m gpu).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ceres_amd/problem_cuda.h"
#include "oracle.h"

using namespace ceres_amd;

static int failures = 0;
#define EXPECT(cond)                                                 \
  do {                                                               \
    if (!(cond)) {                                                   \
      std::printf("FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                    \
    }                                                                \
  } while (0)

static bool IsApprox(const std::vector<double>& a, const std::vector<double>& b, double tol) {
  if (a.size() != b.size()) return false;
  double d = 0, na = 0, nb = 0;
  for (size_t i = 0; i < a.size(); ++i) {
    d += (a[i] - b[i]) * (a[i] - b[i]);
    na += a[i] * a[i];
    nb += b[i] * b[i];
  }
  return std::sqrt(d) <= tol * std::sqrt(std::min(na, nb));
}

static double camera1[10] = {9.99946154126841180165e-01,  7.87061670168454075025e-03,
                             -6.39535329165887445751e-03, -2.20038540935716883662e-03,
                             -3.4093839577186584e-02,     -1.0751387104921525e-01,
                             1.1202240291236032e+00,      3.9975152639358436e+02,
                             -3.1770643852803579e-07,     5.8820490534594022e-13};
static double camera2[10] = {9.99877513605250900497e-01,  7.98833588996764563939e-03,
                             -1.26117173449355086945e-02, -4.69987892415464365153e-03,
                             -8.5667661408224093e-03,     -1.2188049069425422e-01,
                             7.1901330750094605e-01,      4.0201753385955931e+02,
                             -3.7804765613385677e-07,     9.3074311683844792e-13};
static double camera3[7] = {1.4846251175275622e-02,  -2.1062899405576294e-02,
                            -1.1669480098224182e-03, -2.4950970734443037e-02,
                            -1.1398470545726247e-01, 9.2166020737027976e-01,
                            4.0040175368358570e+02};
static double point1[3] = {-6.1200015717226364e-01, 5.7175904776028286e-01,
                           -1.8470812764548823e+00};
static double point2[3] = {1.7074972220818254e+00, 9.5386921723786655e-01,
                           -6.8771685779735616e+00};

static void RunFormat(JacobianFormat format) {
  const bool crs = format == JacobianFormat::kCompressedRow;
  ProblemCUDA problem;
  ProductManifold<QuaternionManifold, EuclideanManifold<6>> camera_manifold;
  CauchyLossCUDA cauchy(1.0);
  HuberLossCUDA huber(1.0);
  // Parameter blocks in the order the reference's problem creates them.
  problem.AddResidualBlock<SnavelyReprojectionErrorWithQuaternions, 2, 10, 3>(
      SnavelyReprojectionErrorWithQuaternions(-3.326500e+02, 2.620900e+02), &cauchy, camera1, point1);
  problem.AddResidualBlock<SnavelyReprojectionErrorWithQuaternions, 2, 10, 3>(
      SnavelyReprojectionErrorWithQuaternions(-1.997600e+02, 1.667000e+02), &cauchy, camera2, point1);
  problem.AddResidualBlock<SnavelyReprojectionErrorWithQuaternions, 2, 10, 3>(
      SnavelyReprojectionErrorWithQuaternions(1.224100e+02, 6.554999e+01), &cauchy, camera1, point2);
  problem.AddResidualBlock<SnavelyReprojectionErrorNoRadialDistortion, 2, 7, 3>(
      SnavelyReprojectionErrorNoRadialDistortion(-2.530600e+02, 2.022700e+02), &huber, camera3,
      point1);
  problem.AddResidualBlock<PointDisplacementError, 3, 3>(
      PointDisplacementError(point1[0], point1[1], point1[2]), nullptr, point1);
  problem.AddResidualBlock<PointDisplacementError, 3, 3>(
      PointDisplacementError(point2[0], point2[1], point2[2]), nullptr, point2);
  problem.SetParameterBlockConstant(camera2);
  problem.SetParameterBlockConstant(point2);
  problem.SetManifold(camera1, &camera_manifold);

  EvaluatorCUDA::Options options;
  options.format = format;
  EvaluatorCUDA evaluator(problem, options);
  EXPECT(evaluator.NumResiduals() == 11);
  EXPECT(evaluator.NumResidualBlocks() == 5);
  std::vector<double> state(evaluator.NumParameters());
  evaluator.ParameterBlocksToStateVector(state.data());
  double cost = -1;
  std::vector<double> r(11), g(evaluator.NumEffectiveParameters());
  std::vector<double> J(evaluator.NumJacobianValues(), -1.0);
  EXPECT(evaluator.Evaluate(state.data(), &cost, r.data(), g.data(), J.data()));

  // The same reduced program, for the oracle.  Program order = insertion:
  // camera1, point1, camera2 (const), point2 (const), camera3.
  std::vector<int32_t> pb_size = {10, 3, 10, 3, 7}, pb_tan = {9, 3, 10, 3, 7};
  std::vector<int32_t> pb_const = {0, 0, 1, 1, 0};
  std::vector<int64_t> pb_pj = {0, -1, -1, -1, -1};
  std::vector<double> pj(90);
  camera_manifold.PlusJacobian(camera1, pj.data());
  std::vector<int32_t> kind = {ORACLE_SNAVELY_QUATERNION_2_10_3, ORACLE_SNAVELY_QUATERNION_2_10_3,
                               ORACLE_SNAVELY_QUATERNION_2_10_3,
                               ORACLE_SNAVELY_NO_DISTORTION_2_7_3, ORACLE_POINT_DISPLACEMENT_3_3};
  std::vector<int32_t> lk = {ORACLE_LOSS_CAUCHY, ORACLE_LOSS_CAUCHY, ORACLE_LOSS_CAUCHY,
                             ORACLE_LOSS_HUBER, ORACLE_LOSS_TRIVIAL};
  std::vector<double> la(5, 1.0), ls(5, 1.0);
  std::vector<int32_t> lsd(5, 0);
  std::vector<int64_t> pbeg = {0, 2, 4, 6, 8, 9};
  std::vector<int32_t> params = {0, 1, 2, 1, 0, 3, 4, 1, 1};
  std::vector<int64_t> dbeg = {0, 2, 4, 6, 8, 11};
  std::vector<double> data = {-3.326500e+02, 2.620900e+02, -1.997600e+02, 1.667000e+02,
                              1.224100e+02,  6.554999e+01, -2.530600e+02, 2.022700e+02,
                              point1[0],     point1[1],    point1[2]};
  oracle_program p{5, pb_size.data(), pb_tan.data(), pb_const.data(), pb_pj.data(), pj.data(),
                   5, kind.data(), lk.data(), la.data(), ls.data(), lsd.data(), pbeg.data(),
                   params.data(), dbeg.data(), data.data(),
                   crs ? ORACLE_COMPRESSED_ROW : ORACLE_BLOCK_SPARSE, 0, 1, nullptr};
  oracle_sizes sz;
  EXPECT(oracle_sizes_of(&p, &sz) == 0);
  EXPECT(sz.num_jacobian_values == evaluator.NumJacobianValues());
  std::vector<double> ostate(sz.num_parameters), cstate(sz.num_constant_parameters);
  const double* act[] = {camera1, point1, camera3};
  const int act_size[] = {10, 3, 7};
  for (int b = 0, o = 0; b < 3; o += act_size[b], ++b)
    for (int k = 0; k < act_size[b]; ++k) ostate[o + k] = act[b][k];
  for (int k = 0; k < 10; ++k) cstate[k] = camera2[k];
  for (int k = 0; k < 3; ++k) cstate[10 + k] = point2[k];
  EXPECT(ostate == state);
  double ocost = -1;
  std::vector<double> orr(11), og(sz.num_effective_parameters), oJ(sz.num_jacobian_values);
  EXPECT(oracle_evaluate(&p, ostate.data(), cstate.data(), 1, &ocost, orr.data(), og.data(),
                         oJ.data()) == 1);
  // Relative like the per-vector isApprox (the reference's absolute 1e-13,
  // evaluator_cuda_test.cu.cc:425, is ~36 ulp of this cost of 12.68).
  EXPECT(std::fabs(cost - ocost) <= 1e-13 * std::max(1.0, std::fabs(ocost)));
  EXPECT(IsApprox(r, orr, 1e-13));
  EXPECT(IsApprox(g, og, 1e-13));
  EXPECT(IsApprox(J, oJ, 1e-13));
  if (crs) {
    std::vector<int64_t> rows(12), cols(sz.num_jacobian_values);
    std::vector<int64_t> lay(5), offs(64);
    EXPECT(oracle_jacobian_offsets(&p, lay.data(), offs.data(), rows.data(), cols.data()) == 0);
    EXPECT(evaluator.crs_rows() == rows);
    EXPECT(evaluator.crs_cols() == cols);
  }
  std::printf("%s: cost %.15e (oracle %.15e)\n", crs ? "CRS" : "BSM", cost, ocost);
}

// The AddressSanitizer build (tests/cpp/Makefile asan-hip, CSE_ASAN_HIP) ends
// by _Exit after flushing: the HIP runtime's exit-time destructors trip the
// ASan runtime's device allocator after it has been torn down.
static int Finish(int rc) {
  std::fflush(stdout);
#ifdef CSE_ASAN_HIP
  std::_Exit(rc);
#endif
  return rc;
}

int main() {
  RunFormat(JacobianFormat::kBlockSparse);
  RunFormat(JacobianFormat::kCompressedRow);
  if (failures) {
    std::printf("%d failure(s)\n", failures);
    return Finish(1);
  }
  std::printf("OK\n");
  return Finish(0);
}
