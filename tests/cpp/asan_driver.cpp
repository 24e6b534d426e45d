// ASan/UBSan driver for the host code (SURVEY.md §5 "Race detection /
// sanitizers"; the reference's SANITIZERS option, CMakeLists.txt:156-158):
// the layout builders (ceres-solver-cuda_amd/csrc/layout.cpp), the CPU oracle
// (oracle/oracle.cpp) and -- built with CSE_ASAN_HIP -- the host half of
// libcse (cse_evaluator.hip, multi_device.hip: descriptor validation, layout
// detection, plans, the multi-device sharding, the error paths), all
// instrumented.  Device code is not instrumented (GPU sanitizers are not
// available on this pool).
//
// Part A (CPU): a synthetic BAL-shaped problem; the layout builders' offsets
// must equal the oracle's writers (block_jacobian_writer.cc /
// compressed_row_jacobian_writer.cc restatements), and the oracle evaluates
// both formats on 1 and 3 threads (bit-identical).
// Part B (CSE_ASAN_HIP, needs a GPU): cse_create / cse_evaluate and
// cse_create_multi over {0, 0, 0} against the oracle (the reference's
// isApprox 1e-13), plus malformed descriptors.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/cse.h"
#include "../../oracle/oracle.h"

#ifdef CSE_ASAN_HIP
#include <hip/hip_runtime.h>
#endif

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

// A deterministic BAL-shaped problem: C cameras, P points, point-major
// observations (Schur order), parameter blocks points first then cameras.
struct Bal {
  int C, P;
  int64_t O;
  std::vector<double> state;     // points 3P, then cameras 9C
  std::vector<int32_t> cam, pt;  // per observation
  std::vector<double> obs;       // 2 per observation
};

static uint64_t lcg = 88172645463325252ull;
static double Uniform() {
  lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
  return (double)(lcg >> 11) * (1.0 / 9007199254740992.0);
}

static Bal MakeBal(int C, int P, int per_point) {
  Bal b{C, P, 0, {}, {}, {}, {}};
  for (int p = 0; p < P; ++p)
    for (int k = 0; k < 3; ++k) b.state.push_back(6.0 * Uniform() - 3.0);
  for (int c = 0; c < C; ++c) {
    const double cam[9] = {0.1 * (Uniform() - 0.5), 0.1 * (Uniform() - 0.5), 0.1 * (Uniform() - 0.5),
                           Uniform() - 0.5,         Uniform() - 0.5,         -10.0 + Uniform(),
                           400.0 + 800.0 * Uniform(), 0.01 * (Uniform() - 0.5), 0.001 * Uniform()};
    b.state.insert(b.state.end(), cam, cam + 9);
  }
  for (int p = 0; p < P; ++p) {
    const int n = 1 + p % per_point;
    for (int k = 0; k < n; ++k) {
      b.cam.push_back((p * 7 + k * 3) % C);
      b.pt.push_back(p);
      b.obs.push_back(200.0 * (Uniform() - 0.5));
      b.obs.push_back(200.0 * (Uniform() - 0.5));
    }
  }
  b.O = (int64_t)b.cam.size();
  return b;
}

struct Layout {
  std::vector<cse_parameter_block> pbs;
  std::vector<int64_t> begin, res_layout, jac_layout, jac_offsets;
  std::vector<int32_t> params, nres;
  int64_t num_values = 0;
};

static Layout BuildLayout(const Bal& b, bool crs) {
  Layout L;
  for (int p = 0; p < b.P; ++p) L.pbs.push_back({3, 3, 0, 0, 3LL * p, 3LL * p, -1});
  for (int c = 0; c < b.C; ++c)
    L.pbs.push_back({9, 9, 0, 0, 3LL * b.P + 9LL * c, 3LL * b.P + 9LL * c, -1});
  L.begin.push_back(0);
  for (int64_t i = 0; i < b.O; ++i) {
    L.params.push_back(b.P + b.cam[i]);
    L.params.push_back(b.pt[i]);
    L.begin.push_back(L.params.size());
    L.nres.push_back(2);
  }
  const int64_t npb = (int64_t)L.pbs.size();
  const int64_t count = cse_layout_offsets_count(npb, L.pbs.data(), b.O, L.begin.data(),
                                                 L.params.data(), L.nres.data());
  EXPECT(count == 4 * b.O);
  L.res_layout.resize(b.O);
  L.jac_layout.resize(b.O);
  L.jac_offsets.resize(count);
  if (!crs) {
    EXPECT(cse_block_sparse_layout(npb, L.pbs.data(), b.O, L.begin.data(), L.params.data(),
                                   L.nres.data(), b.P, L.res_layout.data(), L.jac_layout.data(),
                                   L.jac_offsets.data(), &L.num_values) == CSE_OK);
  } else {
    std::vector<int64_t> rows(2 * b.O + 1);
    EXPECT(cse_compressed_row_layout(npb, L.pbs.data(), b.O, L.begin.data(), L.params.data(),
                                     L.nres.data(), L.res_layout.data(), L.jac_layout.data(),
                                     L.jac_offsets.data(), &L.num_values, rows.data(),
                                     nullptr) == CSE_OK);
    std::vector<int64_t> cols(L.num_values);
    EXPECT(cse_compressed_row_layout(npb, L.pbs.data(), b.O, L.begin.data(), L.params.data(),
                                     L.nres.data(), L.res_layout.data(), L.jac_layout.data(),
                                     L.jac_offsets.data(), &L.num_values, rows.data(),
                                     cols.data()) == CSE_OK);
  }
  EXPECT(L.num_values == 24 * b.O);
  return L;
}

struct OracleInputs {
  std::vector<int32_t> size, tan, cst, kind, lk, lsd, params;
  std::vector<int64_t> pj, pbeg, dbeg;
  std::vector<double> la, ls, data;
  oracle_program p;
};

static void MakeOracle(const Bal& b, bool crs, OracleInputs* in) {
  for (int p = 0; p < b.P; ++p) in->size.push_back(3);
  for (int c = 0; c < b.C; ++c) in->size.push_back(9);
  in->tan = in->size;
  in->cst.assign(in->size.size(), 0);
  in->pj.assign(in->size.size(), -1);
  in->pbeg.push_back(0);
  in->dbeg.push_back(0);
  for (int64_t i = 0; i < b.O; ++i) {
    in->kind.push_back(ORACLE_SNAVELY_2_9_3);
    in->lk.push_back(ORACLE_LOSS_HUBER);
    in->la.push_back(1.0);
    in->ls.push_back(1.0);
    in->lsd.push_back(0);
    in->params.push_back(b.P + b.cam[i]);
    in->params.push_back(b.pt[i]);
    in->pbeg.push_back(in->params.size());
    in->data.push_back(b.obs[2 * i]);
    in->data.push_back(b.obs[2 * i + 1]);
    in->dbeg.push_back(in->data.size());
  }
  in->p = oracle_program{(int64_t)in->size.size(), in->size.data(), in->tan.data(), in->cst.data(),
                         in->pj.data(),   nullptr,         b.O,            in->kind.data(),
                         in->lk.data(),   in->la.data(),   in->ls.data(),  in->lsd.data(),
                         in->pbeg.data(), in->params.data(), in->dbeg.data(), in->data.data(),
                         crs ? ORACLE_COMPRESSED_ROW : ORACLE_BLOCK_SPARSE, b.P, 1};
}

struct Outputs {
  double cost = -1;
  std::vector<double> r, g, J;
};

static void RunFormat(const Bal& b, bool crs) {
  Layout L = BuildLayout(b, crs);
  OracleInputs in;
  MakeOracle(b, crs, &in);
  oracle_sizes sz;
  EXPECT(oracle_sizes_of(&in.p, &sz) == 0);
  EXPECT(sz.num_jacobian_values == L.num_values);
  // The layout builders restate the same writers as the oracle.
  std::vector<int64_t> olay(b.O), offs(4 * b.O), rows(crs ? 2 * b.O + 1 : 1), cols(crs ? L.num_values : 1);
  EXPECT(oracle_jacobian_offsets(&in.p, olay.data(), offs.data(), crs ? rows.data() : nullptr,
                                 crs ? cols.data() : nullptr) == 0);
  EXPECT(olay == L.jac_layout);
  EXPECT(offs == L.jac_offsets);
  Outputs o1, o3;
  for (Outputs* o : {&o1, &o3}) {
    o->r.resize(sz.num_residuals);
    o->g.resize(sz.num_effective_parameters);
    o->J.resize(sz.num_jacobian_values);
  }
  EXPECT(oracle_evaluate(&in.p, b.state.data(), nullptr, 1, &o1.cost, o1.r.data(), o1.g.data(),
                         o1.J.data()) == 1);
  EXPECT(oracle_evaluate(&in.p, b.state.data(), nullptr, 3, &o3.cost, o3.r.data(), o3.g.data(),
                         o3.J.data()) == 1);
  EXPECT(o1.r == o3.r && o1.J == o3.J);
  EXPECT(std::fabs(o1.cost - o3.cost) <= 1e-12 * std::fabs(o1.cost));
  std::printf("%s oracle: cost %.15e, %lld values\n", crs ? "CRS" : "BSM", o1.cost,
              (long long)L.num_values);

#ifdef CSE_ASAN_HIP
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    std::printf("no GPU: part B skipped\n");
    return;
  }
  cse_residual_group g{};
  g.functor_kind = CSE_FUNCTOR_SNAVELY_2_9_3;
  g.loss = cse_loss{CSE_LOSS_HUBER, 0, 1.0, 1.0};
  g.num_blocks = b.O;
  std::vector<int32_t> ids(2 * b.O);
  for (int64_t i = 0; i < b.O; ++i) {
    ids[2 * i] = b.P + b.cam[i];
    ids[2 * i + 1] = b.pt[i];
  }
  g.parameter_block_ids = ids.data();
  g.functor_data = b.obs.data();
  cse_problem_desc d{};
  d.abi_version = CSE_ABI_VERSION;
  d.num_groups = 1;
  d.groups = &g;
  d.num_parameter_blocks = (int64_t)L.pbs.size();
  d.parameter_blocks = L.pbs.data();
  d.num_parameters = sz.num_parameters;
  d.num_effective_parameters = sz.num_effective_parameters;
  d.num_residual_blocks = b.O;
  d.num_residuals = sz.num_residuals;
  d.residual_layout = L.res_layout.data();
  d.jacobian_per_residual_layout = L.jac_layout.data();
  d.jacobian_per_residual_offsets = L.jac_offsets.data();
  d.num_jacobian_per_residual_offsets = (int64_t)L.jac_offsets.size();
  d.num_jacobian_values = L.num_values;
  cse_options opts;
  cse_default_options(&opts);
  const int32_t devs[3] = {0, 0, 0};
  for (int multi = 0; multi < 2; ++multi) {
    cse_evaluator* ev = nullptr;
    const int rc = multi ? cse_create_multi(&d, &opts, devs, 3, &ev) : cse_create(&d, &opts, &ev);
    EXPECT(rc == CSE_OK);
    if (rc != CSE_OK) {
      std::printf("create: %s\n", cse_last_error());
      continue;
    }
    Outputs o;
    o.r.resize(sz.num_residuals);
    o.g.resize(sz.num_effective_parameters);
    o.J.resize(sz.num_jacobian_values);
    for (int rep = 0; rep < 2; ++rep)
      EXPECT(cse_evaluate(ev, b.state.data(), &o.cost, o.r.data(), o.g.data(), o.J.data()) == CSE_OK);
    if (multi) {
      // The caller-pinned path (cse_host_register): asynchronous strips,
      // the same values; per-shard transfer sizes.
      EXPECT(cse_host_register(o.r.data(), o.r.size() * sizeof(double)) == CSE_OK);
      EXPECT(cse_host_register(o.J.data(), o.J.size() * sizeof(double)) == CSE_OK);
      EXPECT(cse_evaluate(ev, b.state.data(), &o.cost, o.r.data(), o.g.data(), o.J.data()) == CSE_OK);
      EXPECT(cse_host_unregister(o.r.data()) == CSE_OK);
      EXPECT(cse_host_unregister(o.J.data()) == CSE_OK);
      EXPECT(cse_host_unregister(o.J.data()) == CSE_ERR_INVALID);
      int64_t h2d[3] = {0, 0, 0}, d2h[3] = {0, 0, 0};
      EXPECT(cse_shard_transfer_bytes(ev, h2d, d2h) == CSE_OK);
      EXPECT(h2d[0] > 0 && h2d[0] < sz.num_parameters * 8 && d2h[0] > 0);
    }
    EXPECT(std::fabs(o.cost - o1.cost) <= 1e-12 * std::fabs(o1.cost));
    EXPECT(IsApprox(o.r, o1.r, 1e-13));
    EXPECT(IsApprox(o.g, o1.g, 1e-13));
    EXPECT(IsApprox(o.J, o1.J, 1e-13));
    // Program::Plus in place (out == state, program.cc:121-149): bit-equal to
    // separate buffers; on the multi-device evaluator cameras are held by
    // several shards (MultiPlus gathers every input before writing).
    {
      std::vector<double> delta(sz.num_effective_parameters), sep(b.state.size());
      for (size_t k = 0; k < delta.size(); ++k) delta[k] = 1e-3 * std::sin(0.37 * (double)k);
      std::vector<double> x = b.state;
      EXPECT(cse_plus(ev, b.state.data(), delta.data(), sep.data()) == CSE_OK);
      EXPECT(cse_plus(ev, x.data(), delta.data(), x.data()) == CSE_OK);
      EXPECT(x == sep);
      bool plain = true;
      for (size_t k = 0; k < x.size(); ++k) plain = plain && sep[k] == b.state[k] + delta[k];
      EXPECT(plain);
    }
    int32_t n = 0;
    EXPECT(cse_shard_info(ev, &n, nullptr, nullptr) == CSE_OK && n == (multi ? 3 : 1));
    cse_info info;
    EXPECT(cse_get_info(ev, &info) == CSE_OK && info.num_residual_blocks == b.O);
    std::printf("%s %s: cost %.15e\n", crs ? "CRS" : "BSM", multi ? "cse_create_multi x3" : "cse_create",
                o.cost);
    cse_destroy(ev);
  }
  // Malformed descriptors are refused with a message, nothing leaks.
  cse_problem_desc bad = d;
  std::vector<int64_t> broken = L.jac_offsets;
  broken[5] = L.num_values;  // out of range
  bad.jacobian_per_residual_offsets = broken.data();
  cse_evaluator* ev = nullptr;
  EXPECT(cse_create(&bad, &opts, &ev) == CSE_ERR_INVALID && ev == nullptr);
  EXPECT(cse_create_multi(&bad, &opts, devs, 3, &ev) != CSE_OK && ev == nullptr);
  std::vector<int32_t> bad_ids = ids;
  bad_ids[7] = (int32_t)L.pbs.size();
  cse_residual_group bg = g;
  bg.parameter_block_ids = bad_ids.data();
  bad = d;
  bad.groups = &bg;
  EXPECT(cse_create(&bad, &opts, &ev) == CSE_ERR_INVALID && ev == nullptr);
#endif
}

// With the instrumented HIP build the process ends by _Exit after flushing:
// at exit the HIP runtime's static destructors free memory through the ASan
// runtime's device allocator after it has been torn down, and ASan's own
// CHECK fires there (sanitizer_allocator_device.h), outside this program.
static int Finish(int rc) {
  std::fflush(stdout);
  std::fflush(stderr);
#ifdef CSE_ASAN_HIP
  std::_Exit(rc);
#endif
  return rc;
}

int main() {
  const Bal b = MakeBal(9, 400, 7);
  RunFormat(b, false);
  RunFormat(b, true);
  if (failures) {
    std::printf("%d failure(s)\n", failures);
    return Finish(1);
  }
  std::printf("OK\n");
  return Finish(0);
}
