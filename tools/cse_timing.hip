// cse_timing.hip -- torch-free timing of the evaluator on a problem-13682
// shaped workload (diagnostic tool, not part of the product).
//
// Builds the BAL shape in C++ (points first = the eliminated group, then
// cameras; ids: cameras by membench's hash, points in order), lays out a
// Schur-ordered BlockSparseMatrix with cse_block_sparse_layout, and times
// cse_evaluate_device with hipMalloc'd buffers.  Compare against bench.py to
// separate library effects from the Python/torch process.
//   build: hipcc --offload-arch=gfx950 -O2 -I include tools/cse_timing.hip \
//          -L ceres-solver-cuda_amd/lib -lcse -Wl,-rpath,<abs lib dir> -o tools/cse_timing
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "cse.h"

#define CK(x)                                                              \
  do {                                                                     \
    int rc_ = (x);                                                         \
    if (rc_ < 0) {                                                         \
      fprintf(stderr, "%s:%d rc %d: %s\n", __FILE__, __LINE__, rc_, cse_last_error()); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)
#define HK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

int main(int argc, char** argv) {
  const int64_t C = 13682, P = 4456117, O = 28987644;
  const int steps = argc > 1 ? atoi(argv[1]) : 20;
  std::vector<cse_parameter_block> pbs(P + C);
  for (int64_t p = 0; p < P; ++p) pbs[p] = {3, 3, 0, 0, 3 * p, 3 * p, -1};
  for (int64_t c = 0; c < C; ++c) pbs[P + c] = {9, 9, 0, 0, 3 * P + 9 * c, 3 * P + 9 * c, -1};
  std::vector<int32_t> ids(2 * O), nres(O, 2);
  std::vector<int64_t> begin(O + 1);
  std::vector<double> obs(2 * O);
  for (int64_t i = 0; i < O; ++i) {
    const unsigned h = (unsigned)(i * 2654435761u) ^ (unsigned)(i >> 7) * 40503u;
    ids[2 * i] = (int32_t)(P + h % C);
    ids[2 * i + 1] = (int32_t)((i * P) / O);
    begin[i] = 2 * i;
    obs[2 * i] = 100.0 * std::sin(0.001 * i);
    obs[2 * i + 1] = 100.0 * std::cos(0.001 * i);
  }
  begin[O] = 2 * O;
  std::vector<double> state(3 * P + 9 * C);
  for (int64_t p = 0; p < P; ++p) {
    state[3 * p] = std::sin(1.0 + p);
    state[3 * p + 1] = std::cos(2.0 + p);
    state[3 * p + 2] = std::sin(3.0 + 0.5 * p);
  }
  for (int64_t c = 0; c < C; ++c) {
    double* x = &state[3 * P + 9 * c];
    x[0] = 0.01 * std::sin(c);
    x[1] = 0.01 * std::cos(c);
    x[2] = 0.02 * std::sin(0.5 * c);
    x[3] = 0.1;
    x[4] = -0.2;
    x[5] = -10.0;
    x[6] = 800.0;
    x[7] = 1e-3;
    x[8] = 1e-4;
  }
  const int64_t noff = cse_layout_offsets_count(P + C, pbs.data(), O, begin.data(), ids.data(), nres.data());
  std::vector<int64_t> rl(O), jl(O), offs(noff);
  int64_t nvals = 0;
  CK(cse_block_sparse_layout(P + C, pbs.data(), O, begin.data(), ids.data(), nres.data(), P,
                             rl.data(), jl.data(), offs.data(), &nvals));
  // The layout builder takes blocks in program order: (camera, point) per
  // residual block -- the functor's slot order.
  cse_residual_group g{};
  g.functor_kind = CSE_FUNCTOR_SNAVELY_2_9_3;
  g.loss = {CSE_LOSS_HUBER, 0, 1.0, 1.0};
  g.num_blocks = O;
  g.residual_block_index = nullptr;
  g.first_residual_block = 0;
  g.parameter_block_ids = ids.data();
  g.functor_data = obs.data();
  cse_problem_desc d{};
  d.abi_version = CSE_ABI_VERSION;
  d.num_groups = 1;
  d.groups = &g;
  d.num_parameter_blocks = P + C;
  d.parameter_blocks = pbs.data();
  d.num_parameters = 3 * P + 9 * C;
  d.num_effective_parameters = 3 * P + 9 * C;
  d.num_residual_blocks = O;
  d.num_residuals = 2 * O;
  d.residual_layout = rl.data();
  d.jacobian_per_residual_layout = jl.data();
  d.jacobian_per_residual_offsets = offs.data();
  d.num_jacobian_per_residual_offsets = noff;
  d.num_jacobian_values = nvals;
  cse_options o;
  cse_default_options(&o);
  o.device = 0;
  o.profile = 1;
  o.check_finite = 0;
  cse_evaluator* ev = nullptr;
  CK(cse_create(&d, &o, &ev));
  cse_info info;
  CK(cse_get_info(ev, &info));
  double *dstate, *dcost, *dres, *djac;
  HK(hipMalloc(&dstate, state.size() * 8));
  HK(hipMalloc(&dcost, 8));
  HK(hipMalloc(&dres, 2 * O * 8));
  HK(hipMalloc(&djac, nvals * 8));
  HK(hipMemcpy(dstate, state.data(), state.size() * 8, hipMemcpyHostToDevice));
  for (int w = 0; w < 3; ++w) CK(cse_evaluate_device(ev, dstate, dcost, dres, nullptr, djac));
  CK(cse_wait(ev));
  CK(cse_reset_kernel_stats(ev));
  for (int s = 0; s < steps; ++s) CK(cse_evaluate_device(ev, dstate, dcost, dres, nullptr, djac));
  CK(cse_wait(ev));
  double last = 0, total = 0;
  int64_t n = 0;
  CK(cse_kernel_stats(ev, &last, &total, &n));
  const double ms = total / n;
  printf("affine groups %d  kernel %.4f ms  %.0f GB/s (algorithmic %.3f GB)\n", info.num_affine_groups,
         ms, info.bytes_jacobian_eval / (ms * 1e-3) / 1e9, info.bytes_jacobian_eval / 1e9);
  cse_destroy(ev);
  return 0;
}
