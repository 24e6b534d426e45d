// C++ parity test of user functors through the ProblemCUDA facade
// (ceres_amd/problem_cuda.h + ceres_amd/autodiff_cuda.h, compiled with
// hipcc as the reference's user TU is compiled with nvcc, README.md:19-33):
//   1. the mini bundle adjustment of internal/ceres/evaluator_cuda_test.cu.cc:
//      232-459 (three functor types, Cauchy/Huber/no loss, two constant
//      blocks, a ProductManifold<Quaternion, Euclidean<6>> camera) with the
//      reference's *own* test functors as user functors
//      (examples/user_functors.h), against the oracle, BSM and CRS;
//   2. BundlerResidual (bundle_adjustment_test_util.h:188-227) with a user
//      LossFunctionCUDA (SoftLOneLoss) and ScaledLossCUDA<SoftLOne>, added
//      through the reference's form AddResidualBlock<F, 2, 9, 3>(
//      AutoDiffCostFunction*, loss, ...), against the oracle.
// Tolerance: the reference's kTolerance = 1e-13 (isApprox per vector).
// Needs a GPU (tests/test_cpp_facade.py under -m gpu).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../examples/user_functors.h"
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

static void MiniBundleAdjustment(JacobianFormat format) {
  const bool crs = format == JacobianFormat::kCompressedRow;
  ProblemCUDA problem;
  ProductManifold<QuaternionManifold, EuclideanManifold<6>> camera_manifold;
  CauchyLossCUDA cauchy(1.0);
  HuberLossCUDA huber(1.0);
  using Q = user::SnavelyReprojectionErrorWithQuaternions;
  using N = user::SnavelyReprojectionErrorNoRadialDistortion;
  using D = user::PointDisplacementError;
  problem.AddResidualBlock<Q, 2, 10, 3>(Q(-3.326500e+02, 2.620900e+02), &cauchy, camera1, point1);
  problem.AddResidualBlock<Q, 2, 10, 3>(Q(-1.997600e+02, 1.667000e+02), &cauchy, camera2, point1);
  problem.AddResidualBlock<Q, 2, 10, 3>(Q(1.224100e+02, 6.554999e+01), &cauchy, camera1, point2);
  problem.AddResidualBlock<N, 2, 7, 3>(N(-2.530600e+02, 2.022700e+02), &huber, camera3, point1);
  problem.AddResidualBlock<D, 3, 3>(D(point1[0], point1[1], point1[2]), nullptr, point1);
  problem.AddResidualBlock<D, 3, 3>(D(point2[0], point2[1], point2[2]), nullptr, point2);
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
  EXPECT(std::fabs(cost - ocost) <= 1e-13 * std::max(1.0, std::fabs(ocost)));
  EXPECT(IsApprox(r, orr, 1e-13));
  EXPECT(IsApprox(g, og, 1e-13));
  EXPECT(IsApprox(J, oJ, 1e-13));
  std::printf("mini BA, user functors, %s: cost %.15e (oracle %.15e)\n", crs ? "CRS" : "BSM", cost,
              ocost);
}

// A small BundlerResidual problem: nc cameras, np points, each point seen by
// 3 cameras; half the blocks SoftLOne(2), half ScaledLoss(SoftLOne(2), 0.5).
static void BundlerWithUserLoss(JacobianFormat format) {
  const bool crs = format == JacobianFormat::kCompressedRow;
  const int nc = 5, np = 40;
  std::vector<double> cams(9 * nc), pts(3 * np);
  for (int c = 0; c < nc; ++c) {
    double* k = &cams[9 * c];
    k[0] = 0.02 * std::sin(c + 1.0);
    k[1] = 0.03 * std::cos(c + 2.0);
    k[2] = c == 0 ? 0.0 : 0.01 * c;
    k[3] = 0.1 * c;
    k[4] = -0.2 + 0.05 * c;
    k[5] = -10.0 + 0.3 * c;
    k[6] = 500.0 + 30.0 * c;
    k[7] = 0.01 * (c - 2);
    k[8] = 0.001 * c;
  }
  for (int q = 0; q < 3 * np; ++q) pts[q] = 2.5 * std::sin(0.7 * q + 0.3);
  ProblemCUDA problem;
  user::SoftLOneLossCUDA soft(2.0);
  ScaledLossCUDA<user::SoftLOneLossCUDA> scaled(soft, 0.5);
  struct Obs { int c, p; double u, v; };
  std::vector<Obs> obs;
  for (int p = 0; p < np; ++p)
    for (int j = 0; j < 3; ++j) {
      const int c = (p + 2 * j) % nc;
      obs.push_back({c, p, 40.0 * std::sin(p + j), 30.0 * std::cos(2.0 * p - j)});
    }
  // Points first (the Schur elimination group), as bundle_adjuster orders.
  std::vector<double*> first;
  for (int p = 0; p < np; ++p) first.push_back(&pts[3 * p]);
  for (size_t i = 0; i < obs.size(); ++i) {
    using F = user::BundlerResidual;
    auto* cost = new AutoDiffCostFunction<F, 2, 9, 3>(new F(obs[i].u, obs[i].v));
    if (i % 2 == 0)
      problem.AddResidualBlock<F, 2, 9, 3>(cost, &soft, &cams[9 * obs[i].c], &pts[3 * obs[i].p]);
    else
      problem.AddResidualBlock<F, 2, 9, 3>(cost, &scaled, &cams[9 * obs[i].c], &pts[3 * obs[i].p]);
  }
  problem.SetEliminationGroup(first);
  EvaluatorCUDA::Options options;
  options.format = format;
  EvaluatorCUDA evaluator(problem, options);
  const int nrb = (int)obs.size();
  std::vector<double> state(evaluator.NumParameters());
  evaluator.ParameterBlocksToStateVector(state.data());
  double cost = -1;
  std::vector<double> r(2 * nrb), g(evaluator.NumEffectiveParameters()),
      J(evaluator.NumJacobianValues());
  EXPECT(evaluator.Evaluate(state.data(), &cost, r.data(), g.data(), J.data()));

  // Oracle: program order = the elimination group (points), then the
  // cameras in the order AddResidualBlock first saw them (ProblemImpl adds
  // a block at first use), residual blocks in insertion order.
  std::vector<int> cam_pos(nc, -1), cam_order;
  for (const Obs& o : obs)
    if (cam_pos[o.c] < 0) {
      cam_pos[o.c] = (int)cam_order.size();
      cam_order.push_back(o.c);
    }
  EXPECT((int)cam_order.size() == nc);
  const int npb = np + nc;
  std::vector<int32_t> pb_size(npb), pb_const(npb, 0), kind(nrb, ORACLE_BUNDLER_RESIDUAL_2_9_3);
  std::vector<int64_t> pb_pj(npb, -1);
  for (int b = 0; b < npb; ++b) pb_size[b] = b < np ? 3 : 9;
  std::vector<int32_t> lk(nrb, ORACLE_LOSS_SOFT_L_ONE), lsd(nrb);
  std::vector<double> la(nrb, 2.0), ls(nrb, 1.0), data(2 * nrb);
  std::vector<int64_t> pbeg(nrb + 1), dbeg(nrb + 1);
  std::vector<int32_t> params(2 * nrb);
  for (int i = 0; i < nrb; ++i) {
    lsd[i] = i % 2;
    ls[i] = i % 2 ? 0.5 : 1.0;
    params[2 * i] = np + cam_pos[obs[i].c];
    params[2 * i + 1] = obs[i].p;
    data[2 * i] = obs[i].u;
    data[2 * i + 1] = obs[i].v;
    pbeg[i + 1] = 2 * (i + 1);
    dbeg[i + 1] = 2 * (i + 1);
  }
  double pj0 = 0;
  oracle_program p{npb, pb_size.data(), pb_size.data(), pb_const.data(), pb_pj.data(), &pj0,
                   nrb, kind.data(), lk.data(), la.data(), ls.data(), lsd.data(), pbeg.data(),
                   params.data(), dbeg.data(), data.data(),
                   crs ? ORACLE_COMPRESSED_ROW : ORACLE_BLOCK_SPARSE, np, 1, nullptr};
  oracle_sizes sz;
  EXPECT(oracle_sizes_of(&p, &sz) == 0);
  EXPECT(sz.num_jacobian_values == evaluator.NumJacobianValues());
  std::vector<double> ostate(pts);
  for (int c : cam_order) ostate.insert(ostate.end(), &cams[9 * c], &cams[9 * c] + 9);
  EXPECT(ostate == state);
  double ocost = -1;
  std::vector<double> orr(2 * nrb), og(sz.num_effective_parameters), oJ(sz.num_jacobian_values);
  EXPECT(oracle_evaluate(&p, ostate.data(), nullptr, 1, &ocost, orr.data(), og.data(), oJ.data()) ==
         1);
  EXPECT(std::fabs(cost - ocost) <= 1e-13 * std::max(1.0, std::fabs(ocost)));
  EXPECT(IsApprox(r, orr, 1e-13));
  EXPECT(IsApprox(g, og, 1e-13));
  EXPECT(IsApprox(J, oJ, 1e-13));
  std::printf("BundlerResidual + SoftLOne user loss, %s: cost %.15e (oracle %.15e)\n",
              crs ? "CRS" : "BSM", cost, ocost);
}

// cse_register_functor's checks on the fused gradient's launches (ABI 5):
// the header fills them for <NR, S0, 3> shapes only, and a table with some
// of them missing, or built against another CamGradArgs, is refused.
static void FusedGradientRegistration() {
  using KB = cse::UserKind<user::BundlerResidual, void, 2, 9, 3>;
  using KR = cse::UserKind<user::RigidAlignmentError, void, 3, 6>;
  const cse_functor_ops ob = autodiff_internal::MakeOps<KB, cse::kLossTrivial>("fused check");
  const cse_functor_ops orr = autodiff_internal::MakeOps<KR, cse::kLossTrivial>("rigid check");
  EXPECT(ob.fused_points[0] && ob.fused_points[1] && ob.camera_gradient &&
         ob.camera_gradient_args_size > 0);
  EXPECT(!orr.fused_points[0] && !orr.fused_points[1] && !orr.camera_gradient &&
         orr.camera_gradient_args_size == 0);
  int32_t kind = -1;
  cse_functor_ops bad = ob;
  bad.camera_gradient = nullptr;
  EXPECT(cse_register_functor(&bad, &kind) == CSE_ERR_INVALID && kind == -1);
  bad = ob;
  bad.camera_gradient_args_size += 8;
  EXPECT(cse_register_functor(&bad, &kind) == CSE_ERR_INVALID && kind == -1);
  bad = orr;
  bad.fused_points[0] = ob.fused_points[0];
  bad.fused_points[1] = ob.fused_points[1];
  bad.camera_gradient = ob.camera_gradient;
  bad.camera_gradient_args_size = ob.camera_gradient_args_size;
  EXPECT(cse_register_functor(&bad, &kind) == CSE_ERR_INVALID && kind == -1);
  EXPECT(cse_register_functor(&ob, &kind) == CSE_OK && kind >= CSE_FUNCTOR_USER_FIRST);
}

int main() {
  FusedGradientRegistration();
  MiniBundleAdjustment(JacobianFormat::kBlockSparse);
  MiniBundleAdjustment(JacobianFormat::kCompressedRow);
  BundlerWithUserLoss(JacobianFormat::kBlockSparse);
  BundlerWithUserLoss(JacobianFormat::kCompressedRow);
  if (failures) {
    std::printf("%d failure(s)\n", failures);
    return 1;
  }
  std::printf("OK\n");
  return 0;
}
