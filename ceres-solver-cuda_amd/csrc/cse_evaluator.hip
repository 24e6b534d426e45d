// cse_evaluator.hip -- the C ABI (include/cse.h) over the gfx950 kernels.
//
// Host side of the evaluator: validates and uploads the Program once
// (RegisteredCUDAEvaluators::Init, internal/ceres/registered_cuda_evaluators.cc:226-280),
// picks a layout policy per residual group, and runs one fused kernel per
// group plus one finalize kernel per evaluation
// (RegisteredCUDAEvaluators::Evaluate, :46-103).
//
// The library reads no environment variable and has no build-time
// alternatives: every kernel it can launch is the shipped one for its
// (functor, loss, outputs, layout).  The settings measured and not shipped
// are recorded in DESIGN.md §4.4 (and the git history before round 6).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../include/cse.h"
#include "group_store_kernel.hpp"
#include "jet_kernels.h"
#include "launch.hpp"
#include "multi_device.h"
#include "schur_kernels.hpp"

namespace cse {
std::string& LastError();  // layout.cpp: one per thread, shared by every entry point
}  // namespace cse

namespace {

int Fail(int code, const std::string& msg) {
  cse::LastError() = msg;
  return code;
}

// Entry points whose arguments are device pointers of one device.
#define CSE_SINGLE_DEVICE(ev, what)                                                         \
  do {                                                                                     \
    if ((ev) && (ev)->multi)                                                               \
      return Fail(CSE_ERR_UNSUPPORTED, std::string(what) +                                 \
                                           ": not available on a multi-device evaluator " \
                                           "(cse_create_multi): its outputs span devices"); \
  } while (0)

#define CSE_HIP(call)                                                              \
  do {                                                                             \
    hipError_t e_ = (call);                                                        \
    if (e_ != hipSuccess)                                                          \
      return Fail(CSE_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

// The functor kinds the library is built for.  Visit(kind, f) calls
// f(K{}) with the kind's functor type; returns false for an unknown kind.
using TestLinear3_234 = cse::LinearTestKind<3, 2, 3, 4>;
using TestLinear3_432 = cse::LinearTestKind<3, 4, 3, 2>;
using TestLinear2_23 = cse::LinearTestKind<2, 2, 3>;
using TestLinear3_24 = cse::LinearTestKind<3, 2, 4>;
using TestLinear4_34 = cse::LinearTestKind<4, 3, 4>;

// Internal kernel kinds (never in a descriptor): a group whose slot-0
// blocks carry a manifold the affine kernels build in registers.
constexpr int kKindQuaternionTangent = -100;  // SNAVELY_QUATERNION_2_10_3, slot 0 on
                                              // CSE_MANIFOLD_QUATERNION_EUCLIDEAN

template <class F>
bool VisitKind(int kind, F&& f) {
  switch (kind) {
    case kKindQuaternionTangent: f(cse::SnavelyQuaternionTangentKind{}); return true;
    case CSE_FUNCTOR_SNAVELY_2_9_3: f(cse::SnavelyKind{}); return true;
    case CSE_FUNCTOR_SNAVELY_NO_DISTORTION_2_7_3: f(cse::SnavelyNoDistortionKind{}); return true;
    case CSE_FUNCTOR_SNAVELY_QUATERNION_2_10_3: f(cse::SnavelyQuaternionKind{}); return true;
    case CSE_FUNCTOR_POINT_DISPLACEMENT_3_3: f(cse::PointDisplacementKind{}); return true;
    case CSE_FUNCTOR_TEST_LINEAR_3_2_3_4: f(TestLinear3_234{}); return true;
    case CSE_FUNCTOR_TEST_LINEAR_3_4_3_2: f(TestLinear3_432{}); return true;
    case CSE_FUNCTOR_TEST_LINEAR_2_2_3: f(TestLinear2_23{}); return true;
    case CSE_FUNCTOR_TEST_LINEAR_3_2_4: f(TestLinear3_24{}); return true;
    case CSE_FUNCTOR_TEST_LINEAR_4_3_4: f(TestLinear4_34{}); return true;
    case CSE_FUNCTOR_TEST_BILINEAR_1_2_2: f(cse::BilinearTestKind{}); return true;
    case CSE_FUNCTOR_TEST_TEN_PARAMETER_1_x10: f(cse::TenParameterTestKind{}); return true;
    case CSE_FUNCTOR_TEST_PARTIAL_OUTPUT_2_1: f(cse::PartialOutputTestKind{}); return true;
    default: return false;
  }
}

// Known-answer-test kinds: general path and trivial loss only.
bool IsTestKind(int kind) { return kind >= 100 && kind < CSE_FUNCTOR_USER_FIRST; }

// ---- User functor kinds (cse_register_functor): the kernels live in the
// user's TU (include/ceres_amd/autodiff_cuda.h); the library holds their
// launch tables.  Entries are never removed, so a pointer to one stays valid.
struct UserKindEntry {
  cse_functor_ops ops;
  std::string name;
};
std::mutex g_user_mu;
std::vector<UserKindEntry*> g_user_kinds;

const cse_functor_ops* UserOps(int kind) {
  if (kind < CSE_FUNCTOR_USER_FIRST) return nullptr;
  std::lock_guard<std::mutex> lock(g_user_mu);
  const size_t i = (size_t)(kind - CSE_FUNCTOR_USER_FIRST);
  return i < g_user_kinds.size() ? &g_user_kinds[i]->ops : nullptr;
}

bool IsUserKind(int kind) { return UserOps(kind) != nullptr; }

// Every affine kernel of a user kind present (the header builds all eight
// or none).
bool UserAffine(const cse_functor_ops* u) {
  bool all = true;
  for (int c = 0; c < 2; ++c)
    for (int j = 0; j < 2; ++j)
      for (int d = 0; d < 2; ++d) all = all && u->affine[c][j][d] != nullptr;
  return all;
}

struct KindShape {
  int nr = 0, nb = 0, data = 0;
  int sz[cse::kMaxSlots] = {};
  int s0 = 0, s1 = 0;  // sz[0], sz[1] (0 if absent): the two-slot affine path
  int x0 = 0;          // slot-0 values gathered (ambient; s0 is the Jacobian's columns)
};

bool ShapeOf(int kind, KindShape* k) {
  if (const cse_functor_ops* u = UserOps(kind)) {
    *k = KindShape{};
    k->nr = u->num_residuals;
    k->nb = u->num_parameter_blocks;
    k->data = u->data_size;
    for (int j = 0; j < k->nb; ++j) k->sz[j] = u->parameter_block_sizes[j];
    k->s0 = k->sz[0];
    k->s1 = k->nb > 1 ? k->sz[1] : 0;
    k->x0 = k->s0;
    return true;
  }
  return VisitKind(kind, [&](auto kd) {
    using K = decltype(kd);
    using Tr = cse::KindTraits<K>;
    k->nr = Tr::NR;
    k->nb = Tr::NB;
    k->data = Tr::D;
    for (int j = 0; j < Tr::NB; ++j) k->sz[j] = K::kSizes[j];
    k->s0 = k->sz[0];
    k->s1 = Tr::NB > 1 ? k->sz[1] : 0;
    k->x0 = Tr::X0;
  });
}

// Device buffer, move-only, freed on destruction.
template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr, o.n = 0; }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) {
      release();
      p = o.p, n = o.n;
      o.p = nullptr, o.n = 0;
    }
    return *this;
  }
  ~DevBuf() { release(); }
  int alloc(size_t count) {
    release();
    if (count == 0) return CSE_OK;
    if (hipMalloc(&p, count * sizeof(T)) != hipSuccess) {
      p = nullptr;
      return Fail(CSE_ERR_OOM, "hipMalloc of " + std::to_string(count * sizeof(T)) + " bytes failed");
    }
    n = count;
    return CSE_OK;
  }
  // Allocate on first use / grow; keeps the buffer when large enough.
  int ensure(size_t count) {
    if (p && n >= count) return CSE_OK;
    return alloc(count);
  }
  int upload(const T* h, size_t count, hipStream_t s) {
    int rc = alloc(count);
    if (rc) return rc;
    if (count && hipMemcpyAsync(p, h, count * sizeof(T), hipMemcpyHostToDevice, s) != hipSuccess)
      return Fail(CSE_ERR_HIP, "hipMemcpyAsync H2D failed");
    return CSE_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

struct Group {
  int kind = 0;
  const cse_functor_ops* user = nullptr;  // a registered user functor kind
  std::string user_name;
  KindShape shape{};
  cse_loss loss{};
  int64_t n = 0;
  bool affine = false;
  int policy = 0;
  int64_t partial_offset = 0;
  int64_t num_wg = 0;
  DevBuf<int32_t> ids;
  DevBuf<double> data;
  DevBuf<int64_t> gindex;  // only when not contiguous
  int64_t first = 0;
  // affine parameters
  int64_t state_base[2] = {0, 0};
  int64_t delta_base[2] = {0, 0};
  int64_t res_base = 0;
  int64_t jac_base[2][3] = {{0, 0, 0}, {0, 0, 0}};
  int64_t jac_stride[2] = {0, 0};
  // Repacked slot-0 table (affine path, small id ranges).
  int32_t slot0_lo = 0;
  int64_t slot0_count = 0;
  int slot0_stride = 0;
  int packed_stride = 0;  // row stride of the repacked slot-0 table (doubles)
  // The manifold DetectAffine chose for slot 0, taken from the first block
  // with an active slot 0 (held blocks carry no Jacobian columns, so their
  // own manifold does not matter).
  int slot0_manifold = CSE_MANIFOLD_MATRIX;
  DevBuf<double> packed0;
  // Gradient post-pass plan per slot (affine groups with a Jacobian layout).
  struct GradPlan {
    bool ready = false;
    bool wave = false;  // one wave (not one lane) per parameter block
    int32_t lo = 0;
    int64_t count = 0;
    DevBuf<int32_t> perm;  // empty = identity
    DevBuf<int64_t> off;
    // wave mode: chunks of at most cse::kGradChunk blocks
    DevBuf<int64_t> chunk_begin, chunk_off;
    DevBuf<int32_t> chunk_pb;  // parameter block (id) of each chunk
    DevBuf<int32_t> chunk_order;  // passes > 1: the chunks pass-major (BuildGradPlan)
    int passes = 1;
    DevBuf<double> chunk_partial;
    int64_t nchunks = 0;
    int64_t nperm = 0;  // blocks in the plan (all but those with a constant block)
    bool all_present = false;  // every id in [lo, lo + count) has a block
  } grad[2];
  // Gradient mode 0 writes every gradient row exactly once (grad_exact): one
  // group, no constant blocks, every camera and point id of its ranges
  // present and their rows tiling the effective parameters.  Then the tail
  // kernels assign instead of adding and the gradient is not zeroed first.
  bool grad_exact = false;
  // Constant slot-0 blocks on the affine path (BlockSparseMatrix): the
  // active-bit table over the slot-0 id range, each id's repack source
  // (state offset, or -1 - constant-state offset), and per 64-block chunk
  // the offset of its first F cell.
  bool const0 = false;
  DevBuf<uint32_t> act0;
  DevBuf<int64_t> src0, fbase, delta0;
  std::vector<int64_t> h_fbase;
  // Held-camera sectors (HeldSectorFixupKernel): each chunk's two side
  // slots and the previous chunk with F cells (BSM) or row blocks (CRS).
  DevBuf<double> side;
  DevBuf<int32_t> prev_seg;
  // Fused gradient (cse::FusedGrad): eligible groups, and their slot-1
  // boundary entries and slot-0 contributions (allocated on first use).
  bool fuse_ok = false;
  DevBuf<double> gside, gcontrib;
  // cse_options.jacobian_form = CSE_JACOBIAN_JET on a Snavely group: its
  // Jacobian kernels are the Jet<double, 12> instantiations (jet_kernels.h).
  bool jet = false;
  // Slot-0-sorted functor data and slot-1 ids (CameraGradientKernel; built
  // on first use).
  DevBuf<double> sdata;
  DevBuf<int32_t> sid1;
  bool sorted_ready = false;
  // Table policy: each 64-block chunk's store runs (BuildTableRuns), and
  // slot 0 plain in every block (DetectPlain0).
  DevBuf<int64_t> runs;
  bool plain0 = false;
  int64_t plain0_state_base = 0, plain0_delta_base = 0;
};

using LaunchFn = void (*)(const cse::GroupArgs&, int64_t num_wg, hipStream_t);

// Waves per workgroup of the CGNR and Schur chunk kernels (one chunk per
// wave either way); one wave per workgroup, as the Jacobian kernels are
// launched, measured slower: S x 2.363 -> 2.410 ms, CGNR 2.596 -> 2.614 ms
// (profiles/round3/w1c).
constexpr int kOperatorWavesPerWg = cse::kWavesPerBlock;

// Cost reduction: above this many per-wave partials, kPartialBlocks
// workgroups sum slices and the last of them finalises
// (ReduceFinalizeKernel); below, one FinalizeKernel.
constexpr int64_t kPartialsTwoPass = 4096;
constexpr int kPartialBlocks = 128;

// Layout policy of a group: 0 = table, 1 = affine packed cells (BSM),
// 2 = affine interleaved rows (CRS).
enum Policy { kTable = 0, kAffinePacked = 1, kAffineCrs = 2 };

template <class K, int L, bool J>
void LaunchTable(const cse::GroupArgs& a, int64_t num_wg, hipStream_t s) {
  cse::LaunchTableKernel<K, L, J>(a, num_wg, s);
}

// The affine kernel: one 64-block chunk per wave, 4 waves per workgroup
// (the residual-only and cost-only evaluations; one wave per workgroup
// measured 1 % slower for them, profiles/round3/w1).
template <class K, int L, bool J, bool Crs, int Co, class T = cse::ShippedTune>
void LaunchChunks(const cse::GroupArgs& a, int64_t num_wg, hipStream_t s) {
  cse::LaunchAffineChunks<K, L, J, Crs, Co, T>(a, num_wg, s);
}

// The BSM residual+Jacobian evaluation of two-slot kinds: one wave per
// workgroup (EvaluateAffineChunksTwoRoundW1); the Snavely camera's, when
// its outputs sit on 64-byte sectors, four-wave workgroups storing long
// runs (EvaluateAffineChunksGroupStore, group_store_kernel.hpp).
template <class K, class T>
constexpr bool kGroupStore = std::is_same<K, cse::SnavelyKind>::value &&
                             std::is_same<T, cse::ShippedTune>::value;

template <class K, int L, int Co, class T = cse::ShippedTune>
void LaunchTwoRound(const cse::GroupArgs& a, int64_t num_wg, hipStream_t s) {
  (void)num_wg;
  if constexpr (kGroupStore<K, T> && Co == 2) {
    if (cse::GroupStoreEligible(a)) {
      const int64_t chunks = cse::Chunks(a.n);
      hipLaunchKernelGGL((cse::EvaluateAffineChunksGroupStore<K, L>),
                         dim3((unsigned)((chunks + cse::kQuadWaves - 1) / cse::kQuadWaves)),
                         dim3(cse::kQuadWaves * cse::kWave), 0, s, a);
      return;
    }
  }
  cse::LaunchTwoRoundW1<K, L, Co, T>(a, s);
}

// The CRS residual+Jacobian evaluation: one wave per workgroup.
template <class K, int L, int Co, class T = cse::ShippedTune>
void LaunchTwoRoundCrs(const cse::GroupArgs& a, int64_t num_wg, hipStream_t s) {
  (void)num_wg;
  cse::LaunchTwoRoundCrsW1<K, L, Co, T>(a, s);
}

// The affine kernel with the fused gradient (Snavely groups): with the
// slot-0 contributions (gradient_mode 3) or points only (gradient_mode 0,
// slot 0 from CameraGradientKernel; one wave per workgroup).
template <class K, int L, bool Crs, class T = cse::ShippedTune>
void LaunchFused(const cse::GroupArgs& a, int64_t num_wg, hipStream_t s) {
  hipLaunchKernelGGL((cse::EvaluateAffineChunksFused<K, L, Crs, T>), dim3((unsigned)num_wg),
                     dim3(cse::kBlockThreads), 0, s, a);
}
template <class K, int L, bool Crs, class T = cse::PointsOnlyTune>
void LaunchFusedPoints(const cse::GroupArgs& a, int64_t num_wg, hipStream_t s) {
  (void)num_wg;
  hipLaunchKernelGGL((cse::EvaluateAffineChunksFusedPointsW1<K, L, Crs, T>), dim3((unsigned)cse::Chunks(a.n)),
                     dim3(cse::kWave), 0, s, a);
}

// Kinds with the fused gradient: the Snavely camera and the quaternion
// camera on its manifold (the same 2 x (9 + 3) Jacobian shape).
bool FusedKind(int kind) {
  return kind == CSE_FUNCTOR_SNAVELY_2_9_3 || kind == kKindQuaternionTangent;
}

// The Jacobian operators built for the Snavely shape (CgnrMultiplyKernel,
// the Schur kernels) read only the Jacobian's values, so they serve every
// fused-gradient group of that shape -- 2 residuals, blocks of 9 (tangent)
// and 3 -- the library's kinds and user kinds alike.
bool SnavelyShaped(const Group& G) {
  return G.shape.nb == 2 && G.shape.nr == 2 && G.shape.s0 == 9 && G.shape.s1 == 3;
}

// f(std::integral_constant<int, s0>) for the slot-0 sizes the fused
// gradient's tail is built for (1..16, the affine kernels' bound).
template <class F>
bool VisitSlot0Size(int s0, F&& f) {
  switch (s0) {
#define CSE_S0_CASE(n) \
  case n: f(std::integral_constant<int, n>{}); return true;
    CSE_S0_CASE(1) CSE_S0_CASE(2) CSE_S0_CASE(3) CSE_S0_CASE(4) CSE_S0_CASE(5) CSE_S0_CASE(6)
    CSE_S0_CASE(7) CSE_S0_CASE(8) CSE_S0_CASE(9) CSE_S0_CASE(10) CSE_S0_CASE(11) CSE_S0_CASE(12)
    CSE_S0_CASE(13) CSE_S0_CASE(14) CSE_S0_CASE(15) CSE_S0_CASE(16)
#undef CSE_S0_CASE
    default: return false;
  }
}

// User kinds that registered the fused gradient's launches (cse_functor_ops
// ABI 5: two slots, slot 1 of 3 parameters): gradient_mode 0's form only
// (points kernel, CameraGradientKernel, the tail); the other modes, the Jet
// form and the operators stay with the library's kinds.
bool UserFused(const Group& G) {
  return G.user && G.user->fused_points[0] && G.user->fused_points[1] && G.user->camera_gradient &&
         G.shape.nb == 2 && G.shape.s1 == 3 && G.shape.s0 >= 1 && G.shape.s0 <= 16;
}

template <class K>
LaunchFn PickFusedK(int loss, bool crs, bool points) {
  switch (loss) {
    case CSE_LOSS_HUBER:
      return points ? (crs ? &LaunchFusedPoints<K, cse::kLossHuber, true> : &LaunchFusedPoints<K, cse::kLossHuber, false>)
                    : (crs ? &LaunchFused<K, cse::kLossHuber, true> : &LaunchFused<K, cse::kLossHuber, false>);
    case CSE_LOSS_CAUCHY:
      return points ? (crs ? &LaunchFusedPoints<K, cse::kLossCauchy, true> : &LaunchFusedPoints<K, cse::kLossCauchy, false>)
                    : (crs ? &LaunchFused<K, cse::kLossCauchy, true> : &LaunchFused<K, cse::kLossCauchy, false>);
    default:
      return points ? (crs ? &LaunchFusedPoints<K, cse::kLossTrivial, true> : &LaunchFusedPoints<K, cse::kLossTrivial, false>)
                    : (crs ? &LaunchFused<K, cse::kLossTrivial, true> : &LaunchFused<K, cse::kLossTrivial, false>);
  }
}

template <class K, bool Crs>
LaunchFn PickFusedC0(int loss, bool points) {
  using TP = cse::PointsOnlyTuneC0;
  using TF = cse::ShippedTuneC0;
  switch (loss) {
    case CSE_LOSS_HUBER:
      return points ? &LaunchFusedPoints<K, cse::kLossHuber, Crs, TP> : &LaunchFused<K, cse::kLossHuber, Crs, TF>;
    case CSE_LOSS_CAUCHY:
      return points ? &LaunchFusedPoints<K, cse::kLossCauchy, Crs, TP> : &LaunchFused<K, cse::kLossCauchy, Crs, TF>;
    default:
      return points ? &LaunchFusedPoints<K, cse::kLossTrivial, Crs, TP> : &LaunchFused<K, cse::kLossTrivial, Crs, TF>;
  }
}

// points = true: the slot-1 rows only (gradient_mode 0, slot 0 from
// CameraGradientKernel); false: with the slot-0 contributions (mode 3).
// const0: groups with constant slot-0 blocks (BSM).
LaunchFn PickFused(int kind, int loss, int policy, bool points, bool const0 = false) {
  const bool crs = policy == kAffineCrs;
  if (const0) {
    if (kind == kKindQuaternionTangent)
      return crs ? PickFusedC0<cse::SnavelyQuaternionTangentKind, true>(loss, points)
                 : PickFusedC0<cse::SnavelyQuaternionTangentKind, false>(loss, points);
    return crs ? PickFusedC0<cse::SnavelyKind, true>(loss, points)
               : PickFusedC0<cse::SnavelyKind, false>(loss, points);
  }
  if (kind == kKindQuaternionTangent)
    return PickFusedK<cse::SnavelyQuaternionTangentKind>(loss, crs, points);
  return PickFusedK<cse::SnavelyKind>(loss, crs, points);
}

// Affine kernels: cooperative slot-0 gather by LDS-DMA from the repacked
// table (dma = true) or by 8-byte pieces straight from the state.
template <class K, int L, bool Crs>
LaunchFn PickAffine(bool jac, bool dma) {
  if constexpr (!Crs && cse::kTwoRoundBsm<K>) {
    // (the 8-byte-piece gather of kCoop 1 would spill at 128 VGPRs)
    if (jac && dma) return &LaunchTwoRound<K, L, 2>;
  }
  if constexpr (Crs) {
    // 1778 CRS 0.298 -> 0.285 ms, 13682 CRS 1.540 -> 1.480 ms (profiles/round2/s5k)
    if (jac && dma) return &LaunchTwoRoundCrs<K, L, 2>;
  }
  if (dma) return jac ? &LaunchChunks<K, L, true, Crs, 2> : &LaunchChunks<K, L, false, Crs, 2>;
  return jac ? &LaunchChunks<K, L, true, Crs, 1> : &LaunchChunks<K, L, false, Crs, 1>;
}

template <class K, int L>
LaunchFn PickJP(bool jac, int policy, bool dma) {
  if constexpr (cse::KindTraits<K>::NB <= 2 && cse::KindTraits<K>::NR <= 3) {
    switch (policy) {
      case kAffinePacked: return PickAffine<K, L, false>(jac, dma);
      case kAffineCrs: return PickAffine<K, L, true>(jac, dma);
      default: break;
    }
  }
  return jac ? &LaunchTable<K, L, true> : &LaunchTable<K, L, false>;
}


// const0: the group has constant slot-0 blocks (FusedKind kinds, the
// repacked table; DetectAffine): the Jacobian kernel with the packed F cells
// (BSM) or the packed row blocks of two widths (CRS).
LaunchFn PickConst0(int kind, int loss, bool jac, bool crs) {
  auto pick = [&](auto kd) -> LaunchFn {
    using K = decltype(kd);
    using T = cse::ShippedTuneC0;
    if (!jac) return nullptr;  // residual/cost kernels write no Jacobian: the usual ones
    if (crs) {
      switch (loss) {
        case CSE_LOSS_HUBER: return &LaunchTwoRoundCrs<K, cse::kLossHuber, 2, T>;
        case CSE_LOSS_CAUCHY: return &LaunchTwoRoundCrs<K, cse::kLossCauchy, 2, T>;
        default: return &LaunchTwoRoundCrs<K, cse::kLossTrivial, 2, T>;
      }
    }
    switch (loss) {
      case CSE_LOSS_HUBER: return &LaunchTwoRound<K, cse::kLossHuber, 2, T>;
      case CSE_LOSS_CAUCHY: return &LaunchTwoRound<K, cse::kLossCauchy, 2, T>;
      default: return &LaunchTwoRound<K, cse::kLossTrivial, 2, T>;
    }
  };
  if (kind == kKindQuaternionTangent) return pick(cse::SnavelyQuaternionTangentKind{});
  if (kind == CSE_FUNCTOR_SNAVELY_2_9_3) return pick(cse::SnavelyKind{});
  return nullptr;
}

LaunchFn Pick(int kind, int loss, bool jac, int policy, bool dma, bool const0 = false) {
  if (const0 && jac)
    return (policy == kAffinePacked || policy == kAffineCrs) && dma
               ? PickConst0(kind, loss, jac, policy == kAffineCrs)
               : nullptr;
  LaunchFn fn = nullptr;
  VisitKind(kind, [&](auto kd) {
    using K = decltype(kd);
    if constexpr (cse::AffineOnly<K>::value) {
      if (policy == kAffinePacked || policy == kAffineCrs) {
        const bool crs = policy == kAffineCrs;
        switch (loss) {
          case CSE_LOSS_HUBER: fn = crs ? PickAffine<K, cse::kLossHuber, true>(jac, dma) : PickAffine<K, cse::kLossHuber, false>(jac, dma); break;
          case CSE_LOSS_CAUCHY: fn = crs ? PickAffine<K, cse::kLossCauchy, true>(jac, dma) : PickAffine<K, cse::kLossCauchy, false>(jac, dma); break;
          default: fn = crs ? PickAffine<K, cse::kLossTrivial, true>(jac, dma) : PickAffine<K, cse::kLossTrivial, false>(jac, dma); break;
        }
      }
    } else if constexpr (cse::TestOnly<K>::value) {
      if (loss == CSE_LOSS_TRIVIAL)
        fn = jac ? &LaunchTable<K, cse::kLossTrivial, true> : &LaunchTable<K, cse::kLossTrivial, false>;
    } else {
      switch (loss) {
        case CSE_LOSS_HUBER: fn = PickJP<K, cse::kLossHuber>(jac, policy, dma); break;
        case CSE_LOSS_CAUCHY: fn = PickJP<K, cse::kLossCauchy>(jac, policy, dma); break;
        default: fn = PickJP<K, cse::kLossTrivial>(jac, policy, dma); break;
      }
    }
  });
  return fn;
}

}  // namespace

int CseFail(int code, const std::string& msg) { return Fail(code, msg); }

bool CseKindShape(int kind, int* num_residuals, int* num_blocks, int* data_size) {
  KindShape k;
  if (!ShapeOf(kind, &k)) return false;
  *num_residuals = k.nr;
  *num_blocks = k.nb;
  *data_size = k.data;
  return true;
}

struct cse_evaluator {
  // A multi-device evaluator (cse_create_multi) is a shell around CseMulti;
  // everything below is unused then.
  CseMulti* multi = nullptr;
  int device = 0;
  int num_cus = 256;  // compute units (grid caps of the Plus kernels)
  hipStream_t stream = nullptr;
  bool own_stream = false;
  cse_options opts{};
  int64_t num_parameter_blocks = 0, num_parameters = 0, num_effective = 0, num_constant = 0;
  int64_t num_residual_blocks = 0, num_residuals = 0, num_jacobian_values = 0;
  int64_t num_plus_jacobian_values = 0;
  bool has_layout = false;
  bool jac_covered = true;  // every Jacobian value is written by some block
  bool res_covered = true;
  int64_t bytes_jac = 0, bytes_res = 0;
  std::vector<Group> groups;
  int64_t total_wg = 0;
  bool any_general = false;
  DevBuf<cse::PbDev> pbs;
  DevBuf<double> cstate, plus_jac;
  DevBuf<int64_t> res_layout, jac_layout, jac_offsets;
  DevBuf<double> partials, partials2;
  // Program::Plus (cse_plus_device): runs of manifold-free state entries.
  bool plus_supported = true;
  std::vector<cse::PlusRun> plus_runs_host;
  DevBuf<cse::PlusRun> plus_runs;
  // CSE_MANIFOLD_QUATERNION_EUCLIDEAN blocks: Plus one block per thread.
  std::vector<cse::QuatPlusBlock> plus_quat_host;
  DevBuf<cse::QuatPlusBlock> plus_quat;
  DevBuf<double> h_delta, h_plus;
  DevBuf<int> status;  // [0] running flag, [1] last status, [2] reduce counter
  // Host-path buffers (allocated on first use).
  DevBuf<double> h_state, h_cost, h_res, h_jac, h_grad;
  DevBuf<double> cg_z;  // cse_cgnr_multiply's z = J x when it cannot fuse
  int* status_host = nullptr;  // pinned
  // Evaluate at the same point (CSE_EVAL_SAME_POINT): the packed slot-0
  // tables hold the state of the last evaluation queued without error, and
  // h_state the last host state uploaded (cleared by a device-pointer call).
  bool point_current = false;
  bool host_state_current = false;
  // Profiling: one (start, stop) event pair per evaluation around its
  // group kernels, folded lazily so timing never stalls the launch queue.
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending, pool;
  double last_ms = 0.0, total_ms = 0.0;
  int64_t launches = 0;
  // The implicit Schur complement (cse_schur_*): structure found at create
  // time, values and vectors bound by cse_schur_init.
  struct Schur {
    bool eligible = false;
    bool duplicates = false;  // an e block sees one f block twice
    int64_t e_cols = 0, f_cols = 0;
    int64_t f_col_base = 0;   // f index of camera id = f_col_base + 9 id
    int64_t nchunks = 0, nbig = 0;
    DevBuf<int64_t> chunk_begin, big;
    DevBuf<double> ete_inv, precond, partial, ub;
    bool ready = false;
    int preconditioner = CSE_SCHUR_IDENTITY;
    const double *jac = nullptr, *D = nullptr, *b = nullptr;
  } schur;
};

namespace {

int Validate(const cse_problem_desc* d) {
  if (!d) return Fail(CSE_ERR_INVALID, "null descriptor");
  if (d->abi_version != CSE_ABI_VERSION)
    return Fail(CSE_ERR_INVALID, "abi_version mismatch: descriptor " +
                                     std::to_string(d->abi_version) + ", library " +
                                     std::to_string(CSE_ABI_VERSION));
  if (d->num_groups < 0 || (d->num_groups > 0 && !d->groups))
    return Fail(CSE_ERR_INVALID, "bad groups");
  if (d->num_parameter_blocks < 0 || (d->num_parameter_blocks > 0 && !d->parameter_blocks))
    return Fail(CSE_ERR_INVALID, "bad parameter blocks");
  for (int64_t b = 0; b < d->num_parameter_blocks; ++b) {
    const cse_parameter_block& pb = d->parameter_blocks[b];
    if (pb.size <= 0 || pb.tangent_size < 0 || pb.tangent_size > pb.size)
      return Fail(CSE_ERR_INVALID, "parameter block " + std::to_string(b) + " has bad size");
    const int64_t lim = pb.is_constant ? d->num_constant_parameters : d->num_parameters;
    if (pb.state_offset < 0 || pb.state_offset + pb.size > lim)
      return Fail(CSE_ERR_INVALID, "parameter block " + std::to_string(b) + " state out of range");
    if (!pb.is_constant && (pb.delta_offset < 0 ||
                            pb.delta_offset + pb.tangent_size > d->num_effective_parameters))
      return Fail(CSE_ERR_INVALID, "parameter block " + std::to_string(b) + " delta out of range");
    if (pb.plus_jacobian_offset >= 0 &&
        pb.plus_jacobian_offset + (int64_t)pb.size * pb.tangent_size > d->num_plus_jacobian_values)
      return Fail(CSE_ERR_INVALID, "parameter block " + std::to_string(b) +
                                       " plus jacobian out of range");
    if (pb.manifold != CSE_MANIFOLD_MATRIX && pb.manifold != CSE_MANIFOLD_QUATERNION_EUCLIDEAN)
      return Fail(CSE_ERR_INVALID, "parameter block " + std::to_string(b) + ": unknown manifold " +
                                       std::to_string(pb.manifold));
    if (pb.manifold == CSE_MANIFOLD_QUATERNION_EUCLIDEAN &&
        (pb.size < 4 || pb.tangent_size != pb.size - 1 || pb.plus_jacobian_offset >= 0))
      return Fail(CSE_ERR_INVALID, "parameter block " + std::to_string(b) +
                                       ": the quaternion manifold needs size >= 4, tangent_size "
                                       "size - 1 and plus_jacobian_offset -1");
  }
  if (d->num_constant_parameters > 0 && !d->constant_state)
    return Fail(CSE_ERR_INVALID, "constant_state missing");
  if (d->num_plus_jacobian_values > 0 && !d->plus_jacobians)
    return Fail(CSE_ERR_INVALID, "plus_jacobians missing");
  if (d->num_residual_blocks < 0 || !d->residual_layout)
    return Fail(CSE_ERR_INVALID, "residual_layout missing");
  return CSE_OK;
}

// Is the group table-free?  Returns the Policy (see evaluate_kernel.hpp
// for the two affine shapes).
// CameraGradientKernel's passes: its point gathers (slot 1, a table of
// 8 s1 bytes per point) hit the Infinity Cache only while the table plus
// every byte streamed between two uses of a line fits in ~256 MiB
// (MI355X_MICROARCH.md, Infinity Cache).  In camera order a point's blocks
// are spread over the whole launch, between which the sorted functor data
// and slot-1 ids (8 data + 4 bytes a block) stream by: 107 + 580 MB at
// problem-13682.  Cut into passes of consecutive point ranges, taken one
// after the other, each pass touches 1/passes of both: passes = the total
// over kCamGradPassBytes, at most 64.  (Passes 8 times finer dealt to the
// XCDs measured no faster.)  The camera sums over written contributions
// (gradient_mode 3, the Schur and CGNR operators' F^T u) take the same
// plan's chunks pass-major too (GradientContribKernel's order).
constexpr double kCamGradPassBytes = 96e6;
int CamGradPasses(const cse_residual_group& g, const KindShape& k) {
  int32_t lo = INT32_MAX, hi = INT32_MIN;
  for (int64_t i = 0; i < g.num_blocks; ++i) {
    lo = std::min(lo, g.parameter_block_ids[i * k.nb + 1]);
    hi = std::max(hi, g.parameter_block_ids[i * k.nb + 1]);
  }
  if (g.num_blocks == 0) return 1;
  const double bytes = 8.0 * k.s1 * ((double)hi - lo + 1) + (8.0 * k.data + 4.0) * g.num_blocks;
  const int p = (int)std::ceil(bytes / kCamGradPassBytes);
  return std::max(1, std::min(64, p));
}

// Blocks of slot j listed per parameter block (stable counting sort): the
// gradient post-pass sums each parameter block's blocks in this order.
// cpb (may be null): the descriptor's parameter blocks; blocks whose slot-j
// parameter block is constant are left out (a held camera has no gradient
// row), which makes the plan a permutation of the other blocks only.
// passes > 1 (slot 0 of a two-slot kind): each parameter block's list is
// further ordered by pass, pass(i) = i * passes / n (block order: in a
// Schur-ordered problem, consecutive point ranges), and no chunk straddles
// two passes; chunk_order lists the chunks pass-major, the order in which
// CameraGradientKernel takes them (CamGradPasses).
int BuildGradPlan(const cse_residual_group& g, const KindShape& k, int j, Group::GradPlan* plan,
                  hipStream_t s, const cse_parameter_block* cpb = nullptr, int passes = 1) {
  const int64_t n = g.num_blocks;
  if (passes < 1 || n < passes) passes = 1;
  auto skip = [&](int64_t i) {
    return cpb && cpb[g.parameter_block_ids[i * k.nb + j]].is_constant;
  };
  auto pass_of = [&](int64_t i) { return (int)((__int128)i * passes / n); };
  int32_t lo = g.parameter_block_ids[j], hi = lo;
  for (int64_t i = 0; i < n; ++i) {
    lo = std::min(lo, g.parameter_block_ids[i * k.nb + j]);
    hi = std::max(hi, g.parameter_block_ids[i * k.nb + j]);
  }
  const int64_t count = (int64_t)hi - lo + 1;
  // Counting sort on (parameter block, pass): poff[p * passes + t].
  std::vector<int64_t> poff(count * passes + 1, 0);
  bool sorted = true;
  int64_t kept = 0, prev = INT64_MIN;
  for (int64_t i = 0; i < n; ++i) {
    if (skip(i)) {
      sorted = false;  // a permutation of the kept blocks, never the identity
      continue;
    }
    const int32_t id = g.parameter_block_ids[i * k.nb + j];
    ++poff[(id - lo) * passes + pass_of(i) + 1];
    if (id < prev) sorted = false;
    prev = id;
    ++kept;
  }
  plan->nperm = kept;
  for (int64_t p = 0; p < count * passes; ++p) poff[p + 1] += poff[p];
  std::vector<int64_t> off(count + 1);
  for (int64_t p = 0; p <= count; ++p) off[p] = poff[p * passes];
  plan->all_present = true;
  for (int64_t p = 0; p < count && plan->all_present; ++p) plan->all_present = off[p + 1] > off[p];
  int rc;
  if (!sorted) {
    std::vector<int32_t> perm(std::max<int64_t>(kept, 1));
    std::vector<int64_t> next(poff.begin(), poff.end() - 1);
    for (int64_t i = 0; i < n; ++i)
      if (!skip(i))
        perm[next[(g.parameter_block_ids[i * k.nb + j] - lo) * passes + pass_of(i)]++] = (int32_t)i;
    if ((rc = plan->perm.upload(perm.data(), perm.size(), s))) return rc;
    if (hipStreamSynchronize(s) != hipSuccess) return Fail(CSE_ERR_HIP, "hipStreamSynchronize failed");
  }
  if ((rc = plan->off.upload(off.data(), off.size(), s))) return rc;
  if (hipStreamSynchronize(s) != hipSuccess) return Fail(CSE_ERR_HIP, "hipStreamSynchronize failed");
  plan->lo = lo;
  plan->count = count;
  plan->wave = !sorted && n >= 32 * count;  // on average 32+ blocks per parameter block
  // Chunks: the wave-mode post-pass and the fused gradient's slot-0 pass.
  if (!sorted) {
    std::vector<int64_t> begin, coff(count + 1, 0);
    std::vector<int32_t> cpb, cpass;
    for (int64_t p = 0; p < count; ++p) {
      coff[p] = (int64_t)begin.size();
      for (int t = 0; t < passes; ++t)
        for (int64_t q = poff[p * passes + t]; q < poff[p * passes + t + 1]; q += cse::kGradChunk) {
          begin.push_back(q);
          cpb.push_back((int32_t)(lo + p));
          cpass.push_back(t);
        }
    }
    coff[count] = (int64_t)begin.size();
    plan->nchunks = (int64_t)begin.size();
    plan->passes = passes;
    if (passes > 1) {  // pass-major launch order, camera order within a pass
      std::vector<int32_t> order;
      order.reserve(begin.size());
      for (int t = 0; t < passes; ++t)
        for (int64_t c = 0; c < plan->nchunks; ++c)
          if (cpass[c] == t) order.push_back((int32_t)c);
      if ((rc = plan->chunk_order.upload(order.data(), order.size(), s))) return rc;
    }
    // Chunk c covers [begin[c], begin[c + 1]): a parameter block's last
    // chunk ends at off[p + 1], where the next non-empty one starts.
    begin.push_back(kept);
    if ((rc = plan->chunk_begin.upload(begin.data(), begin.size(), s))) return rc;
    if ((rc = plan->chunk_off.upload(coff.data(), coff.size(), s))) return rc;
    if (!cpb.empty() && (rc = plan->chunk_pb.upload(cpb.data(), cpb.size(), s))) return rc;
    const int size = j == 0 ? k.s0 : k.s1;
    if ((rc = plan->chunk_partial.alloc((size_t)std::max<int64_t>(1, plan->nchunks) * size)))
      return rc;
    if (hipStreamSynchronize(s) != hipSuccess) return Fail(CSE_ERR_HIP, "hipStreamSynchronize failed");
  }
  plan->ready = true;
  return CSE_OK;
}

// The post-pass form of a plan (cse::GradForm) and its chunk table.
int GradFormOf(const cse::GradArgs& ga, const Group::GradPlan& P) {
  if (ga.perm == nullptr) return cse::kGradRange;  // identity order: contiguous ranges (points)
  return P.wave ? cse::kGradChunked : cse::kGradPerBlock;  // many blocks per parameter block: chunks
}
cse::GradChunks GradChunksOf(const Group::GradPlan& P) {
  return cse::GradChunks{P.chunk_begin.p, P.chunk_off.p, P.chunk_partial.p, P.nchunks};
}

// Gradient post-pass kernels of the built-in shapes; a user kind brings its
// own (cse_functor_ops.gradient).
bool GradSupported(int nr, int size, const cse_functor_ops* user = nullptr, int slot = 0) {
  if (user) return user->gradient[slot] != nullptr;
  return (nr == 2 && (size == 9 || size == 3 || size == 7 || size == 10)) || (nr == 3 && size == 3);
}

bool LaunchGradPass(int nr, int size, const cse::GradArgs& ga, const Group::GradPlan& P,
                    hipStream_t s, const cse_functor_ops* user = nullptr, int slot = 0) {
  const int form = GradFormOf(ga, P);
  const cse::GradChunks ch = GradChunksOf(P);
  if (user) {
    if (!user->gradient[slot]) return false;
    user->gradient[slot](&ga, &ch, form, s);
    return true;
  }
  if (nr == 2 && size == 9) return cse::LaunchGradientSlot<2, 9>(ga, ch, form, s), true;
  if (nr == 2 && size == 3) return cse::LaunchGradientSlot<2, 3>(ga, ch, form, s), true;
  if (nr == 2 && size == 7) return cse::LaunchGradientSlot<2, 7>(ga, ch, form, s), true;
  if (nr == 2 && size == 10) return cse::LaunchGradientSlot<2, 10>(ga, ch, form, s), true;
  if (nr == 3 && size == 3) return cse::LaunchGradientSlot<3, 3>(ga, ch, form, s), true;
  return false;
}

int DetectAffine(const cse_problem_desc* d, const cse_residual_group& g, const KindShape& k,
                  Group* G) {
  const int64_t n = g.num_blocks;
  if (n == 0) return kTable;
  // The affine kernels take one or two slots, at most three residuals; a
  // user kind has them only for the shapes its header instantiates.
  if (k.nb > 2 || k.nr > 3 || IsTestKind(g.functor_kind)) return kTable;
  if (const cse_functor_ops* u = UserOps(g.functor_kind))
    if (!UserAffine(u)) return kTable;
  auto gidx = [&](int64_t i) {
    return g.residual_block_index ? g.residual_block_index[i] : g.first_residual_block + i;
  };
  // Ambient sizes (state offsets) and tangent sizes (delta offsets, the
  // Jacobian's columns).  Slot 0 of the quaternion camera may be on
  // CSE_MANIFOLD_QUATERNION_EUCLIDEAN (then in every block): the kernel kind
  // becomes kKindQuaternionTangent, which builds the plus-Jacobian itself.
  const int ambient[2] = {k.s0, k.s1};
  int sizes[2] = {k.s0, k.s1};
  int manifold[2] = {CSE_MANIFOLD_MATRIX, CSE_MANIFOLD_MATRIX};
  // The first block whose slot j is active (bases and the manifold come from it).
  int64_t first[2] = {-1, -1};
  for (int64_t i = 0; i < n && (first[0] < 0 || (k.nb > 1 && first[1] < 0)); ++i)
    for (int j = 0; j < k.nb; ++j)
      if (first[j] < 0 && !d->parameter_blocks[g.parameter_block_ids[i * k.nb + j]].is_constant)
        first[j] = i;
  for (int j = 0; j < k.nb; ++j)
    if (first[j] < 0) return kTable;
  if (g.functor_kind == CSE_FUNCTOR_SNAVELY_QUATERNION_2_10_3 &&
      d->parameter_blocks[g.parameter_block_ids[first[0] * k.nb]].manifold ==
          CSE_MANIFOLD_QUATERNION_EUCLIDEAN) {
    manifold[0] = CSE_MANIFOLD_QUATERNION_EUCLIDEAN;
    sizes[0] = k.s0 - 1;
  }
  G->slot0_manifold = manifold[0];
  // Constant slot-0 blocks (a held camera) are allowed for the kinds with the
  // constant-aware kernels (the 9-column cameras, cse::ShippedTuneC0).
  const bool const0_ok = k.nb == 2 && (g.functor_kind == CSE_FUNCTOR_SNAVELY_2_9_3 ||
                                       manifold[0] == CSE_MANIFOLD_QUATERNION_EUCLIDEAN);
  // Parameters: active (slot 0 may be constant, above), no explicit
  // plus-Jacobian, state/delta offsets affine in the id.
  for (int j = 0; j < k.nb; ++j) {
    const int32_t id0 = g.parameter_block_ids[first[j] * k.nb + j];
    const cse_parameter_block& pb0 = d->parameter_blocks[id0];
    G->state_base[j] = pb0.state_offset - (int64_t)ambient[j] * id0;
    G->delta_base[j] = pb0.delta_offset - (int64_t)sizes[j] * id0;
  }
  // With constant slot-0 blocks the active ones need not be affine either
  // (a held camera in the middle shifts the later ones' offsets): their values
  // come through the repacked table, their gradient rows through a table.
  G->const0 = false;
  for (int64_t i = 0; i < n && !G->const0; ++i)
    G->const0 = d->parameter_blocks[g.parameter_block_ids[i * k.nb]].is_constant != 0;
  if (G->const0 && !const0_ok) return kTable;
  for (int64_t i = 0; i < n; ++i)
    for (int j = 0; j < k.nb; ++j) {
      const int32_t id = g.parameter_block_ids[i * k.nb + j];
      const cse_parameter_block& pb = d->parameter_blocks[id];
      if (pb.is_constant) {
        if (j != 0 || pb.size != ambient[0]) return kTable;
        continue;
      }
      if (pb.plus_jacobian_offset >= 0 || pb.manifold != manifold[j] ||
          pb.tangent_size != sizes[j] || pb.size != ambient[j])
        return kTable;
      if (j == 0 && G->const0) continue;
      if (pb.state_offset != G->state_base[j] + (int64_t)ambient[j] * id) return kTable;
      if (pb.delta_offset != G->delta_base[j] + (int64_t)sizes[j] * id) return kTable;
    }
  // Slot-0 id range (the repacked table of the cooperative gather).
  int32_t lo = g.parameter_block_ids[0], hi = lo;
  for (int64_t i = 0; i < n; ++i) {
    lo = std::min(lo, g.parameter_block_ids[i * k.nb]);
    hi = std::max(hi, g.parameter_block_ids[i * k.nb]);
  }
  G->slot0_lo = lo;
  G->slot0_count = (int64_t)hi - lo + 1;
  G->slot0_stride = (sizes[0] + 1) & ~1;  // per-block slot-0 gradient contributions
  G->packed_stride = cse::PackedRowDoubles(ambient[0]);
  // Residuals.
  G->res_base = d->residual_layout[gidx(0)];
  for (int64_t i = 0; i < n; ++i)
    if (d->residual_layout[gidx(i)] != G->res_base + (int64_t)k.nr * i) return kTable;
  // Jacobian rows.
  if (!d->jacobian_per_residual_layout || !d->jacobian_per_residual_offsets) return kAffinePacked;
  const int64_t* L = d->jacobian_per_residual_layout;
  const int64_t* O = d->jacobian_per_residual_offsets;
  if (G->const0) {
    const int NR = k.nr, S0 = sizes[0], S1 = sizes[1];
    auto act = [&](int64_t i) {
      return !d->parameter_blocks[g.parameter_block_ids[i * k.nb]].is_constant;
    };
    const int64_t nchunks = (n + cse::kWave - 1) / cse::kWave;
    // BlockSparseMatrix: the E (slot 1) cells affine, kR x S1 packed at
    // e0 + kR*S1*i; the F cells of the blocks with an active camera packed in
    // block order from f0 (a constant camera has none; its block's first
    // active entries are the E rows).  Per chunk of 64 blocks: its first F
    // cell, then the end of the F cells.
    auto try_bsm = [&]() -> bool {
      const int64_t f0 = O[L[gidx(first[0])]];
      const int64_t e0 = O[L[gidx(0)] + (act(0) ? NR : 0)];
      std::vector<int64_t> fb;
      fb.reserve((size_t)nchunks + 1);
      int64_t rank = 0;
      for (int64_t i = 0; i < n; ++i) {
        if (i % cse::kWave == 0) fb.push_back(f0 + (int64_t)NR * S0 * rank);
        const int64_t base = L[gidx(i)];
        int a = 0;
        if (act(i)) {
          for (int r = 0; r < NR; ++r)
            if (O[base + r] != f0 + (int64_t)NR * S0 * rank + (int64_t)r * S0) return false;
          ++rank;
          a = 1;
        }
        for (int r = 0; r < NR; ++r)
          if (O[base + a * NR + r] != e0 + (int64_t)NR * S1 * i + (int64_t)r * S1) return false;
      }
      for (int r = 0; r < NR; ++r) {
        G->jac_base[0][r] = f0 + (int64_t)r * S0;
        G->jac_base[1][r] = e0 + (int64_t)r * S1;
      }
      G->jac_stride[0] = (int64_t)NR * S0;
      G->jac_stride[1] = (int64_t)NR * S1;
      fb.push_back(f0 + (int64_t)NR * S0 * rank);
      G->h_fbase = std::move(fb);
      return true;
    };
    // CompressedRowSparseMatrix (compressed_row_jacobian_writer.cc:145-185):
    // every block's rows packed in block order, NR x (S0 + S1) with an active
    // camera (camera and point at fixed columns of the row) and NR x S1 with
    // a held one (the point alone).  Per chunk: the offset of its first row,
    // then the end.
    auto try_crs = [&]() -> bool {
      const int N = S0 + S1;
      const int64_t b0 = L[gidx(first[0])];
      const int64_t cam0 = O[b0], pt0 = O[b0 + NR];
      const int64_t rb0 = std::min(cam0, pt0);
      const int camcol = (int)(cam0 - rb0), ptcol = (int)(pt0 - rb0);
      if (!((camcol == 0 && ptcol == S0) || (ptcol == 0 && camcol == S1))) return false;
      const int64_t r0 = rb0 - (int64_t)NR * S1 * first[0];
      std::vector<int64_t> cb;
      cb.reserve((size_t)nchunks + 1);
      int64_t pos = r0;
      for (int64_t i = 0; i < n; ++i) {
        if (i % cse::kWave == 0) cb.push_back(pos);
        const int64_t base = L[gidx(i)];
        if (act(i)) {
          for (int r = 0; r < NR; ++r)
            if (O[base + r] != pos + (int64_t)r * N + camcol ||
                O[base + NR + r] != pos + (int64_t)r * N + ptcol)
              return false;
          pos += (int64_t)NR * N;
        } else {
          for (int r = 0; r < NR; ++r)
            if (O[base + r] != pos + (int64_t)r * S1) return false;
          pos += (int64_t)NR * S1;
        }
      }
      cb.push_back(pos);
      for (int r = 0; r < NR; ++r) {
        G->jac_base[0][r] = r0 + (int64_t)r * N + camcol;
        G->jac_base[1][r] = r0 + (int64_t)r * N + ptcol;
      }
      G->jac_stride[0] = G->jac_stride[1] = (int64_t)NR * N;
      G->h_fbase = std::move(cb);
      return true;
    };
    if (try_bsm()) return kAffinePacked;
    if (try_crs()) return kAffineCrs;
    return kTable;
  }
  for (int j = 0; j < k.nb; ++j)
    for (int r = 0; r < k.nr; ++r) G->jac_base[j][r] = O[L[gidx(0)] + j * k.nr + r];
  for (int j = 0; j < k.nb; ++j)
    G->jac_stride[j] = n > 1 ? O[L[gidx(1)] + j * k.nr] - G->jac_base[j][0] : (int64_t)k.nr * sizes[j];
  for (int64_t i = 0; i < n; ++i)
    for (int j = 0; j < k.nb; ++j)
      for (int r = 0; r < k.nr; ++r)
        if (O[L[gidx(i)] + j * k.nr + r] != G->jac_base[j][r] + G->jac_stride[j] * i) return kTable;
  const int N = sizes[0] + sizes[1];
  // Shape 1: packed cells (BlockSparseMatrix).
  bool packed = true;
  for (int j = 0; j < k.nb; ++j) {
    if (G->jac_stride[j] != (int64_t)k.nr * sizes[j]) packed = false;
    for (int r = 0; r < k.nr; ++r)
      if (G->jac_base[j][r] != G->jac_base[j][0] + (int64_t)r * sizes[j]) packed = false;
  }
  if (packed && !(G->jac_stride[0] == (int64_t)k.nr * N && k.nb > 1)) return kAffinePacked;
  // Shape 2: interleaved rows (CompressedRowSparseMatrix): every slot has
  // stride kR*N, row r of the block starts at row0 + r*N and each slot sits
  // at a fixed column position inside the row, the slots tiling [0, N).
  int64_t row0 = G->jac_base[0][0];
  for (int j = 0; j < k.nb; ++j) row0 = std::min(row0, G->jac_base[j][0]);
  bool cover[32] = {false};
  for (int j = 0; j < k.nb; ++j) {
    if (G->jac_stride[j] != (int64_t)k.nr * N) return kTable;
    const int64_t col = G->jac_base[j][0] - row0;
    if (col < 0 || col + sizes[j] > N) return kTable;
    for (int c = 0; c < sizes[j]; ++c) {
      if (cover[col + c]) return kTable;
      cover[col + c] = true;
    }
    for (int r = 0; r < k.nr; ++r)
      if (G->jac_base[j][r] != row0 + (int64_t)r * N + col) return kTable;
  }
  return kAffineCrs;
}

cse::GroupArgs MakeArgs(cse_evaluator* ev, Group& G, const double* state, double* res,
                        double* jac, double* grad) {
  cse::GroupArgs a{};
  a.n = G.n;
  a.ids = G.ids.p;
  a.data = G.data.p;
  a.state = state;
  a.cstate = ev->cstate.p;
  a.pbs = ev->pbs.p;
  a.plus_jacobians = ev->plus_jac.p;
  for (int j = 0; j < 2; ++j) {
    a.state_base[j] = G.state_base[j];
    a.delta_base[j] = G.delta_base[j];
    a.jac_stride[j] = G.jac_stride[j];
    for (int r = 0; r < 3; ++r) a.jac_base[j][r] = G.jac_base[j][r];
  }
  a.res_base = G.res_base;
  a.packed0 = G.packed0.p;
  a.packed0_lo = G.slot0_lo;
  a.packed0_stride = G.packed_stride;
  a.act0_bits = G.act0.p;
  a.fbase = G.fbase.p;
  a.side = G.side.p;
  a.delta0 = G.delta0.p;
  a.gindex = G.gindex.p;
  a.first = G.first;
  a.residual_layout = ev->res_layout.p;
  a.jac_layout = ev->jac_layout.p;
  a.jac_offsets = ev->jac_offsets.p;
  a.residuals = res;
  a.jacobian = jac;
  a.gradient = grad;
  a.partials = ev->partials.p + G.partial_offset;
  a.status = ev->status.p;
  a.loss.a = G.loss.a;
  a.loss.scale = G.loss.scale;
  a.loss.scaled = G.loss.scaled;
  static_assert(sizeof(a.user_loss) == sizeof(G.loss.user), "user loss bytes");
  std::memcpy(a.user_loss, G.loss.user, sizeof(a.user_loss));
  a.apply_loss = ev->opts.apply_loss_function;
  a.check_finite = ev->opts.check_finite;
  a.table_runs = G.runs.p;
  a.plain0 = G.plain0 ? 1 : 0;
  a.plain0_state_base = G.plain0_state_base;
  a.plain0_delta_base = G.plain0_delta_base;
  return a;
}

// A table group whose slot-0 blocks are all plain: active, no manifold
// (plus_jacobian_offset -1), tangent size = size = the kind's, state and
// delta offsets affine in the id.  EvaluateTableKernel then forms their PbDev
// records instead of loading them: one cache line less per lane for a
// camera-like slot 0, whose lines the point stream evicts from L2 between
// uses.
void DetectPlain0(const cse_problem_desc* d, const cse_residual_group& g, Group* G) {
  const KindShape& k = G->shape;
  G->plain0 = false;
  if (G->affine || G->n == 0) return;
  const int S = k.sz[0];
  const int32_t id0 = g.parameter_block_ids[0];
  const int64_t sb = d->parameter_blocks[id0].state_offset - (int64_t)S * id0;
  const int64_t db = d->parameter_blocks[id0].delta_offset - (int64_t)S * id0;
  for (int64_t i = 0; i < G->n; ++i) {
    const int32_t id = g.parameter_block_ids[i * k.nb];
    const cse_parameter_block& p = d->parameter_blocks[id];
    if (p.is_constant || p.manifold != CSE_MANIFOLD_MATRIX || p.plus_jacobian_offset != -1 ||
        p.size != S || p.tangent_size != S || p.state_offset != sb + (int64_t)S * id ||
        p.delta_offset != db + (int64_t)S * id)
      return;
  }
  G->plain0 = true;
  G->plain0_state_base = sb;
  G->plain0_delta_base = db;
}

// The general kernel's store runs, found once per 64-block chunk (the
// wave's blocks) by the tests TableStores makes on the device: flags
// kTableRunFlagResiduals when the chunk's residuals are one run (NR apart),
// kTableRunFlagBsm / Crs when every slot is active in all or none of its
// blocks with one tangent size and its Jacobian rows form BlockSparseMatrix
// cell runs / CompressedRow row blocks; then the residual run's start and
// each active slot's first row.  [chunks][2 + nb]; shapes the kernel stages
// (kTableStaged: NR x N <= 32) only.
int BuildTableRuns(const cse_evaluator* ev, const cse_problem_desc* d, const cse_residual_group& g, Group* G,
                   hipStream_t s) {
  const KindShape& k = G->shape;
  int N = 0;
  for (int j = 0; j < k.nb; ++j) N += k.sz[j];
  if (G->affine || G->n == 0 || k.nr * N > 32) return CSE_OK;
  const int NB = k.nb, NR = k.nr, W = 2 + NB;
  const int64_t n = G->n, nch = (n + cse::kWave - 1) / cse::kWave;
  std::vector<int64_t> runs((size_t)(nch * W), 0);
  auto gidx = [&](int64_t i) { return g.residual_block_index ? g.residual_block_index[i] : g.first_residual_block + i; };
  auto pb = [&](int64_t i, int j) -> const cse_parameter_block& {
    return d->parameter_blocks[g.parameter_block_ids[i * NB + j]];
  };
  for (int64_t c = 0; c < nch; ++c) {
    const int64_t i0 = c * cse::kWave;
    const int nb = (int)std::min<int64_t>(cse::kWave, n - i0);
    int64_t* R = &runs[(size_t)(c * W)];
    const int64_t off0 = d->residual_layout[gidx(i0)];
    bool rr = true;
    for (int l = 1; rr && l < nb; ++l) rr = d->residual_layout[gidx(i0 + l)] == off0 + (int64_t)NR * l;
    if (rr) {
      R[0] |= cse::kTableRunFlagResiduals;
      R[1] = off0;
    }
    if (!ev->has_layout) continue;
    bool cst[CSE_MAX_PARAMETER_BLOCKS];
    int t[CSE_MAX_PARAMETER_BLOCKS];
    bool uniform = true;
    for (int j = 0; j < NB; ++j) {
      cst[j] = pb(i0, j).is_constant != 0;
      t[j] = pb(i0, j).tangent_size;
      for (int l = 1; uniform && l < nb; ++l) {
        const cse_parameter_block& p = pb(i0 + l, j);
        uniform = (p.is_constant != 0) == cst[j] && (cst[j] || p.tangent_size == t[j]);
      }
    }
    if (!uniform) continue;
    // Row (j, kk) of lane l: offsets[layout[gidx] + a NR + kk], a = slot j's
    // position among the active slots.
    auto row = [&](int l, int a, int kk) {
      return d->jacobian_per_residual_offsets[d->jacobian_per_residual_layout[gidx(i0 + l)] + (int64_t)a * NR + kk];
    };
    int64_t base[CSE_MAX_PARAMETER_BLOCKS] = {0};
    int64_t r0 = INT64_MAX;
    int w = 0, a = 0;
    for (int j = 0; j < NB; ++j) {
      if (cst[j]) continue;
      base[j] = row(0, a++, 0);
      r0 = std::min(r0, base[j]);
      w += t[j];
    }
    bool bsm = true, crs = true;
    a = 0;
    for (int j = 0; j < NB; ++j) {
      if (cst[j]) continue;
      for (int l = 0; l < nb && (bsm || crs); ++l)
        for (int kk = 0; kk < NR; ++kk) {
          const int64_t v = row(l, a, kk);
          bsm = bsm && v == base[j] + (int64_t)l * NR * t[j] + (int64_t)kk * t[j];
          crs = crs && v == base[j] + (int64_t)l * NR * w + (int64_t)kk * w;
        }
      ++a;
      const int64_t cj = base[j] - r0;
      crs = crs && cj >= 0 && cj + t[j] <= w;
      for (int j2 = 0; j2 < j; ++j2) {
        if (cst[j2]) continue;
        const int64_t c2 = base[j2] - r0;
        crs = crs && (cj + t[j] <= c2 || c2 + t[j2] <= cj);
      }
    }
    R[0] |= (bsm ? cse::kTableRunFlagBsm : 0) | (crs ? cse::kTableRunFlagCrs : 0);
    for (int j = 0; j < NB; ++j) R[2 + j] = base[j];
  }
  int rc = G->runs.upload(runs.data(), runs.size(), s);
  if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = Fail(CSE_ERR_HIP, "table runs upload failed");
  return rc;
}

int FoldTiming(cse_evaluator* ev) {
  for (auto& pr : ev->pending) {
    float ms = 0.f;
    CSE_HIP(hipEventSynchronize(pr.second));
    CSE_HIP(hipEventElapsedTime(&ms, pr.first, pr.second));
    ev->last_ms = ms;
    ev->total_ms += ms;
    ev->launches += 1;
    ev->pool.push_back(pr);
  }
  ev->pending.clear();
  return CSE_OK;
}

// After a fused kernel (the evaluator's FusedGrad or CgnrMultiplyKernel):
// add the slot-1 boundary entries and the slot-0 contributions, per
// parameter block in a fixed order, into out (delta offsets).
int LaunchFusedGradTail(const Group& G, double* out, hipStream_t s) {
  const int64_t entries = 2 * ((G.n + cse::kWave - 1) / cse::kWave);
  hipLaunchKernelGGL((cse::GradientBoundaryKernel<3>),
                     dim3((unsigned)((entries + cse::kBlockThreads - 1) / cse::kBlockThreads)),
                     dim3(cse::kBlockThreads), 0, s, G.gside.p, entries, out, G.delta_base[1]);
  const Group::GradPlan& P = G.grad[0];
  cse::GradArgs ga{};
  ga.count = P.count;
  ga.lo = P.lo;
  ga.grad = out;
  ga.delta_base = G.delta_base[0];
  ga.delta_tab = G.const0 ? G.delta0.p + (P.lo - G.slot0_lo) : nullptr;
  const cse::GradChunks ch{P.chunk_begin.p, P.chunk_off.p, P.chunk_partial.p, P.nchunks};
  if (P.nchunks > 0)
    hipLaunchKernelGGL((cse::GradientContribKernel<9, 10>),
                       dim3((unsigned)((P.nchunks + cse::kWavesPerBlock - 1) / cse::kWavesPerBlock)),
                       dim3(cse::kBlockThreads), 0, s, G.gcontrib.p, P.perm.p, ch,
                       P.chunk_order.p);
  hipLaunchKernelGGL((cse::GradientChunkReduceKernel<9>),
                     dim3((unsigned)((ga.count + cse::kBlockThreads - 1) / cse::kBlockThreads)),
                     dim3(cse::kBlockThreads), 0, s, ga, ch);
  CSE_HIP(hipGetLastError());
  return CSE_OK;
}

// gradient_mode 0: the slot-1 boundary entries as above, and the slot-0
// sums by re-evaluation in camera order (CameraGradientKernel), then
// GradientChunkReduceKernel.  The sorted inputs are built on first use
// (CamGradSortedInputs, on the evaluator's stream).
int CamGradSortedInputs(Group& G, hipStream_t s) {
  const Group::GradPlan& P = G.grad[0];
  const int D = G.shape.data;
  int rc;
  if (!G.sorted_ready) {  // set only once the copies have been queued
    if (D != 2 && !UserFused(G))
      return Fail(CSE_ERR_UNSUPPORTED, "camera-order gradient: 2 data doubles per block");
    if ((rc = G.sdata.alloc((size_t)G.n * D))) return rc;
    if ((rc = G.sid1.alloc((size_t)G.n))) return rc;
    const dim3 grid((unsigned)((G.n + cse::kBlockThreads - 1) / cse::kBlockThreads));
    if (D == 2)
      hipLaunchKernelGGL((cse::SortSlot0InputsKernel<2>), grid, dim3(cse::kBlockThreads), 0, s, G.ids.p,
                         G.data.p, P.perm.p, P.nperm, G.sdata.p, G.sid1.p);
    else
      hipLaunchKernelGGL((cse::SortSlot0InputsAnyKernel<>), grid, dim3(cse::kBlockThreads), 0, s, G.ids.p,
                         G.data.p, D, P.perm.p, P.nperm, G.sdata.p, G.sid1.p);
    CSE_HIP(hipGetLastError());
    G.sorted_ready = true;
  }
  return CSE_OK;
}

// Waves per workgroup of CameraGradientKernel (one chunk per wave).
constexpr int kCamGradWavesPerWg = cse::kWavesPerBlock;

// CameraGradientKernel: the per-chunk slot-0 sums into P.chunk_partial.
int LaunchCameraGradKernel(cse_evaluator* ev, Group& G, const double* state, hipStream_t s) {
  const Group::GradPlan& P = G.grad[0];
  cse::CamGradArgs cg{};
  cg.state = state;
  cg.state_base0 = G.state_base[0];
  cg.state_base1 = G.state_base[1];
  cg.sdata = G.sdata.p;
  cg.sid1 = G.sid1.p;
  cg.chunk_pb = P.chunk_pb.p;
  cg.chunk_begin = P.chunk_begin.p;
  cg.chunk_order = P.chunk_order.p;
  cg.partial = P.chunk_partial.p;
  cg.nchunks = P.nchunks;
  cg.nslots = P.nchunks;
  cg.loss.a = G.loss.a;
  cg.loss.scale = G.loss.scale;
  cg.loss.scaled = G.loss.scaled;
  cg.apply_loss = ev->opts.apply_loss_function;
  if (G.const0) {  // active cameras' state offsets need not be affine
    cg.packed0 = G.packed0.p;
    cg.packed_lo = G.slot0_lo;
    cg.packed_stride = G.packed_stride;
  }
  if (G.user) {  // the kind's own CameraGradientKernel (its TU), with its loss object
    static_assert(sizeof(cg.user_loss) == sizeof(G.loss.user), "user loss bytes");
    std::memcpy(cg.user_loss, G.loss.user, sizeof(cg.user_loss));
    if (P.nchunks > 0) G.user->camera_gradient(&cg, cg.nslots, s);
    CSE_HIP(hipGetLastError());
    return CSE_OK;
  }
  constexpr int W = kCamGradWavesPerWg;
  const dim3 grid((unsigned)((cg.nslots + W - 1) / W));
  if (P.nchunks > 0) {
    auto launch = [&](auto kd) {
      using K = decltype(kd);
      switch (G.loss.kind) {
        case CSE_LOSS_HUBER:
          hipLaunchKernelGGL((cse::CameraGradientKernel<K, cse::kLossHuber, W>), grid,
                             dim3(W * cse::kWave), 0, s, cg);
          break;
        case CSE_LOSS_CAUCHY:
          hipLaunchKernelGGL((cse::CameraGradientKernel<K, cse::kLossCauchy, W>), grid,
                             dim3(W * cse::kWave), 0, s, cg);
          break;
        default:
          hipLaunchKernelGGL((cse::CameraGradientKernel<K, cse::kLossTrivial, W>), grid,
                             dim3(W * cse::kWave), 0, s, cg);
      }
    };
    if (G.jet) cse::LaunchJetCameraGradient(G.loss.kind, cg, cg.nslots, s);
    else if (G.kind == kKindQuaternionTangent) launch(cse::SnavelyQuaternionTangentKind{});
    else launch(cse::SnavelyKind{});
  }
  CSE_HIP(hipGetLastError());
  return CSE_OK;
}

// After the points kernel and CameraGradientKernel: the slot-1 boundary
// entries, then the slot-0 rows from the chunk sums, in a fixed order.
// assign (grad_exact): the rows are written, not added to.  The boundary
// entries and the camera rows in one launch (GradientTailKernel).
int LaunchCameraGradReduce(Group& G, double* out, hipStream_t s, bool assign = false) {
  const Group::GradPlan& P = G.grad[0];
  const int64_t entries = 2 * ((G.n + cse::kWave - 1) / cse::kWave);
  const int64_t bwg = (entries + cse::kBlockThreads - 1) / cse::kBlockThreads;
  cse::GradArgs ga{};
  ga.count = P.count;
  ga.lo = P.lo;
  ga.grad = out;
  ga.delta_base = G.delta_base[0];
  ga.delta_tab = G.const0 ? G.delta0.p + (P.lo - G.slot0_lo) : nullptr;
  const cse::GradChunks ch{P.chunk_begin.p, P.chunk_off.p, P.chunk_partial.p, P.nchunks};
  const int64_t cwg = (ga.count + cse::kBlockThreads - 1) / cse::kBlockThreads;
  const dim3 grid((unsigned)(bwg + cwg));
  auto tail = [&](auto s0) {
    constexpr int S0 = decltype(s0)::value;
    if (assign)
      hipLaunchKernelGGL((cse::GradientTailKernel<3, S0, true>), grid, dim3(cse::kBlockThreads), 0, s, G.gside.p,
                         entries, G.delta_base[1], bwg, ga, ch);
    else
      hipLaunchKernelGGL((cse::GradientTailKernel<3, S0, false>), grid, dim3(cse::kBlockThreads), 0, s,
                         G.gside.p, entries, G.delta_base[1], bwg, ga, ch);
  };
  if (!VisitSlot0Size(G.shape.s0, tail))
    return Fail(CSE_ERR_UNSUPPORTED, "fused gradient: slot 0 of " + std::to_string(G.shape.s0) + " parameters");
  CSE_HIP(hipGetLastError());
  return CSE_OK;
}

// The implicit Schur complement's structure (cse_schur_*): one Snavely
// group on the fused-gradient path with the BlockSparseMatrix layout, its
// e blocks (slot 1, points) the leading columns [0, e_cols) and its f blocks
// (slot 0, cameras) the rest, as ITERATIVE_SCHUR's elimination ordering puts
// them (iterative_schur_complement_solver.cc:66-80).  The e-block runs are cut
// into wave chunks of whole runs; longer runs are listed as big.
int BuildSchurPlan(cse_evaluator* ev, const cse_problem_desc* d, hipStream_t s) {
  auto& S = ev->schur;
  S.eligible = false;
  if (ev->groups.size() != 1 || d->num_groups != 1) return CSE_OK;
  const Group& G = ev->groups[0];
  if (!G.fuse_ok || G.policy != kAffinePacked || !SnavelyShaped(G) ||
      !ev->has_layout || ev->num_constant > 0)
    return CSE_OK;
  const cse_residual_group& g = d->groups[0];
  const int32_t* ids = g.parameter_block_ids;
  const int64_t n = g.num_blocks;
  int32_t pmin = ids[1], pmax = ids[1], cmin = ids[0], cmax = ids[0];
  for (int64_t i = 0; i < n; ++i) {
    pmin = std::min(pmin, ids[2 * i + 1]);
    pmax = std::max(pmax, ids[2 * i + 1]);
    cmin = std::min(cmin, ids[2 * i]);
    cmax = std::max(cmax, ids[2 * i]);
  }
  const int64_t e_lo = G.delta_base[1] + 3LL * pmin, e_hi = G.delta_base[1] + 3LL * pmax + 3;
  const int64_t f_lo = G.delta_base[0] + 9LL * cmin, f_hi = G.delta_base[0] + 9LL * cmax + 9;
  if (e_lo < 0 || f_lo != e_hi || f_hi != ev->num_effective || e_lo != 0) return CSE_OK;
  S.e_cols = e_hi;
  S.f_cols = f_hi - f_lo;
  S.f_col_base = G.delta_base[0] - S.e_cols;
  // One pass over the runs of equal e block: small runs are packed into
  // chunks of at most a wave ([begin, end) pairs; chunks never straddle a
  // big run), big runs listed on their own.
  std::vector<int64_t> ranges, big;
  std::vector<int32_t> cams;
  bool dup = false;
  int64_t run_start = 0, chunk_lo = 0;
  for (int64_t i = 1; i <= n; ++i) {
    if (i < n && ids[2 * i + 1] == ids[2 * (i - 1) + 1]) continue;
    const int64_t len = i - run_start;  // the run [run_start, i)
    cams.assign(len, 0);
    for (int64_t k = 0; k < len; ++k) cams[k] = ids[2 * (run_start + k)];
    std::sort(cams.begin(), cams.end());
    dup = dup || std::adjacent_find(cams.begin(), cams.end()) != cams.end();
    if (len > cse::kWave) {
      if (run_start > chunk_lo) ranges.insert(ranges.end(), {chunk_lo, run_start});
      big.insert(big.end(), {run_start, i});
      chunk_lo = i;
    } else if (i - chunk_lo > cse::kWave) {
      ranges.insert(ranges.end(), {chunk_lo, run_start});
      chunk_lo = run_start;
    }
    run_start = i;
  }
  if (n > chunk_lo) ranges.insert(ranges.end(), {chunk_lo, n});
  std::vector<int64_t>& begins = ranges;
  S.duplicates = dup;
  S.nchunks = (int64_t)begins.size() / 2;
  S.nbig = (int64_t)big.size() / 2;
  int rc;
  if ((rc = S.chunk_begin.upload(begins.data(), begins.size(), s))) return rc;
  if ((rc = S.big.upload(big.data(), big.size(), s))) return rc;
  if (hipStreamSynchronize(s) != hipSuccess) return Fail(CSE_ERR_HIP, "Schur plan upload failed");
  S.eligible = true;
  return CSE_OK;
}

// How a group's gradient is summed in one evaluation (cse_options.
// gradient_mode, cse.h): grad_pass = a deterministic post-pass over the
// written residuals and Jacobian (the group has plans for all its slots),
// else in-kernel FP64 atomics (as the reference); fused = the fused form
// (FusedGrad); recompute = its slot-0 rows by CameraGradientKernel (modes 0
// and 1 on held-camera groups) rather than written contributions (mode 3).
struct GradPath {
  bool grad_pass = false, fused = false, recompute = false;
};
GradPath GradPathOf(const cse_evaluator* ev, const Group& G, bool grad, bool res, bool jac) {
  GradPath p;
  p.grad_pass = grad && res && jac && G.affine && ev->opts.gradient_mode != 2;
  for (int j = 0; j < G.shape.nb; ++j) p.grad_pass = p.grad_pass && G.grad[j].ready;
  const int mode = ev->opts.gradient_mode;
  // Mode 1 (post-pass) has no form over the packed F cells of a group with
  // constant slot-0 blocks: it takes mode 0's fused form (also fixed order).
  // The Jet form has no mode-3 kernel (contributions in block order): the
  // post-pass instead, as for groups without a fused form.
  p.fused = p.grad_pass && G.fuse_ok &&
            (mode == 0 || (!G.user && ((mode == 3 && !G.jet) || (mode == 1 && G.const0))));
  // Constant slot-0 blocks: no post-pass over the packed F cells (in-kernel
  // atomics instead, active cameras only).
  if (G.const0 && !p.fused) p.grad_pass = false;
  p.recompute = p.fused && mode != 3;
  return p;
}

// Enqueue one evaluation on ev->stream.
// same_point (CSE_EVAL_SAME_POINT): the state equals the previous
// evaluation's, so the packed slot-0 tables it built are still valid and the
// repack launches are skipped.
int Enqueue(cse_evaluator* ev, const double* d_state, double* d_cost, double* d_res,
            double* d_grad, double* d_jac, bool same_point = false) {
  if (d_jac && !ev->has_layout)
    return Fail(CSE_ERR_INVALID, "Jacobian requested but the descriptor had no Jacobian layout");
  const bool repack = !(same_point && ev->point_current);
  ev->point_current = false;  // set again once every launch below is queued
  const bool jets = d_jac || d_grad;
  std::pair<hipEvent_t, hipEvent_t> timing{nullptr, nullptr};
  if (ev->opts.profile) {
    if (ev->pool.empty()) {
      // Timing only: no system-scope fence (cache write-back and
      // invalidation) at either event, which cost ~7-10 us per evaluation
      // at the 8-way shard and problem-16 (profiles/round3/ov0).
      CSE_HIP(hipEventCreateWithFlags(&timing.first, hipEventDisableSystemFence));
      CSE_HIP(hipEventCreateWithFlags(&timing.second, hipEventDisableSystemFence));
    } else {
      timing = ev->pool.back();
      ev->pool.pop_back();
    }
    if (ev->pending.size() > 4096) {
      int rc = FoldTiming(ev);
      if (rc) return rc;
    }
  }
  // One grad_exact group whose gradient takes the fused form with the
  // camera rows recomputed (the fused points kernel, the camera rows and the
  // boundary rows then write every row exactly once): no zeroing pass, the
  // tail kernels assign.  The same predicate as the group loop below.
  const bool grad_assign =
      d_grad && ev->groups.size() == 1 && ev->groups[0].grad_exact &&
      GradPathOf(ev, ev->groups[0], d_grad != nullptr, d_res != nullptr, d_jac != nullptr).recompute;
  if (d_grad && ev->num_effective > 0 && !grad_assign)
    CSE_HIP(hipMemsetAsync(d_grad, 0, ev->num_effective * sizeof(double), ev->stream));
  if (d_jac && !ev->jac_covered && ev->num_jacobian_values > 0)
    CSE_HIP(hipMemsetAsync(d_jac, 0, ev->num_jacobian_values * sizeof(double), ev->stream));
  if (d_res && !ev->res_covered && ev->num_residuals > 0)
    CSE_HIP(hipMemsetAsync(d_res, 0, ev->num_residuals * sizeof(double), ev->stream));
  for (size_t g = 0; g < ev->groups.size(); ++g) {
    Group& G = ev->groups[g];
    if (G.n == 0) continue;
    const bool dma = G.packed0.p != nullptr;
    LaunchFn fn = nullptr;
    cse_kernel_launch_fn ufn = nullptr;  // a user kind's kernel (its own TU)
    if (G.user) {
      ufn = G.policy == kTable ? G.user->table[jets ? 1 : 0]
                               : G.user->affine[G.policy == kAffineCrs][jets ? 1 : 0][dma ? 1 : 0];
      if (!ufn) return Fail(CSE_ERR_UNSUPPORTED, "user functor kind " + G.user_name + " has no such kernel");
    } else {
      fn = Pick(G.kind, G.loss.kind, jets, G.policy, dma, G.const0);
      if (G.jet && jets)  // the Jet<double, 12> instantiations (cse_create kept only these shapes)
        fn = G.policy == kTable ? cse::JetSnavelyTable(G.loss.kind)
                                : cse::JetSnavelyJacobian(G.loss.kind, G.policy == kAffineCrs);
      if (!fn) return Fail(CSE_ERR_UNSUPPORTED, "no kernel for functor kind " + std::to_string(G.kind));
    }
    const GradPath gp = GradPathOf(ev, G, d_grad != nullptr, d_res != nullptr, d_jac != nullptr);
    const bool grad_pass = gp.grad_pass, fused = gp.fused, recompute = gp.recompute;
    cse::GroupArgs a = MakeArgs(ev, G, d_state, d_res, d_jac, grad_pass ? nullptr : d_grad);
    if (fused) {
      const int64_t chunks = (G.n + cse::kWave - 1) / cse::kWave;
      int rc;
      if ((rc = G.gside.ensure((size_t)(2 * chunks * 4)))) return rc;
      if (!recompute && (rc = G.gcontrib.ensure((size_t)G.n * G.slot0_stride))) return rc;
      a.gfused = d_grad;
      a.gside = G.gside.p;
      a.gcontrib = G.gcontrib.p;
      if (G.user)
        ufn = G.user->fused_points[G.policy == kAffineCrs];
      else
        fn = PickFused(G.kind, G.loss.kind, G.policy, recompute, G.const0);
      if (G.jet) fn = cse::JetSnavelyFusedPoints(G.loss.kind, G.policy == kAffineCrs);
    }
    if (timing.first && g == 0) CSE_HIP(hipEventRecord(timing.first, ev->stream));
    if (dma && repack) {
      const int pieces = (G.shape.x0 + 1) / 2;
      const int64_t total = G.slot0_count * pieces;
      hipLaunchKernelGGL(cse::RepackSlot0Kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                         ev->stream, d_state, G.state_base[0], G.shape.x0, G.packed_stride, pieces,
                         G.slot0_lo, G.slot0_count, G.packed0.p, G.src0.p, ev->cstate.p);
    }
    if (recompute) {
      const int rc = CamGradSortedInputs(G, ev->stream);
      if (rc) return rc;
    }
    if (ufn)
      ufn(&a, G.num_wg, ev->stream);
    else
      fn(a, G.num_wg, ev->stream);
    CSE_HIP(hipGetLastError());
    if (G.const0 && jets && d_jac && G.side.p) {
      // The 64-byte sectors two held-camera chunks share (the full chunks
      // stored their heads and tails in side slots), when the full chunks
      // took that tail: the same base alignment test as the kernel.
      if (cse::HeldWindowsAligned(d_res, G.res_base, d_jac, G.jac_base[1][0], G.h_fbase[0])) {
        const int64_t nchunks = (G.n + cse::kWave - 1) / cse::kWave;
        const int64_t threads = 4 * nchunks;
        hipLaunchKernelGGL(cse::HeldSectorFixupKernel,
                           dim3((unsigned)((threads + cse::kBlockThreads - 1) / cse::kBlockThreads)),
                           dim3(cse::kBlockThreads), 0, ev->stream, d_jac, G.fbase.p, G.side.p,
                           G.prev_seg.p, nchunks, G.n / cse::kWave);
        CSE_HIP(hipGetLastError());
      }
    }
    if (recompute) {
      // After the points kernel on the same stream (beside it on a second
      // stream measured 3.9 % slower, 2.23 vs 2.15 ms: profiles/round3/s2).
      int rc;
      if ((rc = LaunchCameraGradKernel(ev, G, d_state, ev->stream))) return rc;
      if ((rc = LaunchCameraGradReduce(G, d_grad, ev->stream, grad_assign))) return rc;
    } else if (fused) {
      const int rc = LaunchFusedGradTail(G, d_grad, ev->stream);
      if (rc) return rc;
    } else if (grad_pass) {
      const int sizes[2] = {G.shape.s0, G.shape.s1};
      for (int j = 0; j < G.shape.nb; ++j) {
        const Group::GradPlan& P = G.grad[j];
        cse::GradArgs ga{};
        ga.jac = d_jac;
        for (int r = 0; r < G.shape.nr && r < 3; ++r) ga.jrow[r] = G.jac_base[j][r];
        ga.jstride = G.jac_stride[j];
        ga.res = d_res;
        ga.res_base = G.res_base;
        ga.perm = P.perm.p;
        ga.off = P.off.p;
        ga.count = P.count;
        ga.lo = P.lo;
        ga.grad = d_grad;
        ga.delta_base = G.delta_base[j];
        if (!LaunchGradPass(G.shape.nr, sizes[j], ga, P, ev->stream, G.user, j))
          return Fail(CSE_ERR_UNSUPPORTED, "no gradient pass for this shape");
        CSE_HIP(hipGetLastError());
      }
    }
  }
  if (timing.first) {
    if (ev->groups.empty()) CSE_HIP(hipEventRecord(timing.first, ev->stream));
    CSE_HIP(hipEventRecord(timing.second, ev->stream));
    ev->pending.push_back(timing);
  }
  const double* parts = ev->partials.p;
  const int64_t nparts = ev->total_wg;
  if (nparts > kPartialsTwoPass) {
    // Fixed-order slices summed by kPartialBlocks workgroups, the last of
    // which adds the slice sums: one launch (ReduceFinalizeKernel).
    const int64_t per = (nparts + kPartialBlocks - 1) / kPartialBlocks;
    hipLaunchKernelGGL(cse::ReduceFinalizeKernel, dim3(kPartialBlocks), dim3(cse::kBlockThreads), 0,
                       ev->stream, parts, nparts, per, ev->partials2.p, ev->status.p + 2, d_cost,
                       ev->status.p, ev->status.p + 1);
  } else {
    hipLaunchKernelGGL(cse::FinalizeKernel, dim3(1), dim3(1024), 0, ev->stream, parts, nparts,
                       d_cost, ev->status.p, ev->status.p + 1);
  }
  CSE_HIP(hipGetLastError());
  ev->point_current = true;
  return CSE_OK;
}

}  // namespace

extern "C" {

void cse_default_options(cse_options* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->device = -1;
  o->check_finite = 1;
  o->apply_loss_function = 1;
}

const char* cse_last_error(void) { return cse::LastError().c_str(); }

int cse_abi_version(void) { return CSE_ABI_VERSION; }

const char* cse_build_info(void) {
#define CSE_STR2_(x) #x
#define CSE_STR_(x) CSE_STR2_(x)
  return "cse abi=" CSE_STR_(CSE_ABI_VERSION) " target=gfx950 built " __DATE__ " " __TIME__;
}

int cse_create(const cse_problem_desc* d, const cse_options* options, cse_evaluator** out) {
  if (!out) return Fail(CSE_ERR_INVALID, "null out");
  *out = nullptr;
  int rc = Validate(d);
  if (rc) return rc;
  cse_evaluator* ev = new (std::nothrow) cse_evaluator();
  if (!ev) return Fail(CSE_ERR_OOM, "host allocation failed");
  if (options) ev->opts = *options; else cse_default_options(&ev->opts);
  auto bail = [&](int code) { cse_destroy(ev); return code; };
  if (ev->opts.gradient_mode < 0 || ev->opts.gradient_mode > 3)
    return bail(Fail(CSE_ERR_INVALID, "gradient_mode " + std::to_string(ev->opts.gradient_mode) +
                                          " is not one of 0..3"));
  if (ev->opts.jacobian_form != CSE_JACOBIAN_CLOSED_FORM && ev->opts.jacobian_form != CSE_JACOBIAN_JET)
    return bail(Fail(CSE_ERR_INVALID, "jacobian_form " + std::to_string(ev->opts.jacobian_form) +
                                          " is not a cse_jacobian_form"));

  if (ev->opts.device >= 0) {
    const hipError_t e = hipSetDevice(ev->opts.device);
    if (e != hipSuccess)
      return bail(Fail(CSE_ERR_HIP, "hipSetDevice(" + std::to_string(ev->opts.device) +
                                        ") failed: " + hipGetErrorString(e)));
    ev->device = ev->opts.device;
  } else {
    if (hipGetDevice(&ev->device) != hipSuccess) return bail(Fail(CSE_ERR_HIP, "no HIP device"));
  }
  if (hipDeviceGetAttribute(&ev->num_cus, hipDeviceAttributeMultiprocessorCount, ev->device) !=
      hipSuccess)
    return bail(Fail(CSE_ERR_HIP, "hipDeviceGetAttribute failed"));
  if (ev->opts.stream || ev->opts.use_stream) {
    ev->stream = (hipStream_t)ev->opts.stream;
  } else {
    if (hipStreamCreateWithFlags(&ev->stream, hipStreamNonBlocking) != hipSuccess)
      return bail(Fail(CSE_ERR_HIP, "hipStreamCreate failed"));
    ev->own_stream = true;
  }
  hipStream_t s = ev->stream;
  ev->num_parameter_blocks = d->num_parameter_blocks;
  ev->num_parameters = d->num_parameters;
  ev->num_effective = d->num_effective_parameters;
  ev->num_constant = d->num_constant_parameters;
  ev->num_residual_blocks = d->num_residual_blocks;
  ev->num_residuals = d->num_residuals;
  ev->num_jacobian_values = d->num_jacobian_values;
  ev->num_plus_jacobian_values = d->num_plus_jacobian_values;
  ev->has_layout = d->jacobian_per_residual_layout && d->jacobian_per_residual_offsets;
  {
    // Plus runs: active blocks sorted by state offset, merged while
    // contiguous with a constant delta shift.
    std::vector<std::pair<int64_t, int64_t>> blocks;  // (state_offset, index)
    for (int64_t b = 0; b < d->num_parameter_blocks; ++b) {
      const cse_parameter_block& pb = d->parameter_blocks[b];
      if (pb.is_constant) continue;
      if (pb.manifold == CSE_MANIFOLD_QUATERNION_EUCLIDEAN) {
        ev->plus_quat_host.push_back({pb.state_offset, pb.delta_offset, pb.size, 0});
        continue;
      }
      if (pb.plus_jacobian_offset >= 0 || pb.tangent_size != pb.size) ev->plus_supported = false;
      blocks.emplace_back(pb.state_offset, b);
    }
    std::sort(blocks.begin(), blocks.end());
    for (const auto& e : blocks) {
      const cse_parameter_block& pb = d->parameter_blocks[e.second];
      const int64_t shift = pb.state_offset - pb.delta_offset;
      auto& R = ev->plus_runs_host;
      if (!R.empty() && R.back().state_begin + R.back().length == pb.state_offset &&
          R.back().delta_shift == shift)
        R.back().length += pb.size;
      else
        R.push_back({pb.state_offset, pb.size, shift});
    }
  }

  // Groups.
  int64_t covered_res = 0, covered_jac = 0;
  std::vector<char> seen(d->num_parameter_blocks, 0);
  // Which (group, slot) uses each parameter block: -1 none, -2 several.
  std::vector<int32_t> owner(d->num_parameter_blocks, -1);
  for (int gi = 0; gi < d->num_groups; ++gi) {
    const cse_residual_group& g = d->groups[gi];
    Group G;
    if (g.functor_kind < 0 || !ShapeOf(g.functor_kind, &G.shape))
      return bail(Fail(CSE_ERR_UNSUPPORTED, "unknown functor kind " + std::to_string(g.functor_kind)));
    if (g.loss.kind < CSE_LOSS_TRIVIAL || g.loss.kind > CSE_LOSS_USER)
      return bail(Fail(CSE_ERR_UNSUPPORTED, "unknown loss kind " + std::to_string(g.loss.kind)));
    if (IsTestKind(g.functor_kind) && (g.loss.kind != CSE_LOSS_TRIVIAL || g.loss.scaled))
      return bail(Fail(CSE_ERR_UNSUPPORTED, "test functor kinds take the trivial loss only"));
    G.user = UserOps(g.functor_kind);
    if (G.user) {
      // The kernels of a user kind apply the loss they were built with
      // (AutoDiffResidualBlockCUDAEvaluator<F, LossFunctionCUDA, ...>).
      {
        std::lock_guard<std::mutex> lock(g_user_mu);
        G.user_name = g_user_kinds[(size_t)(g.functor_kind - CSE_FUNCTOR_USER_FIRST)]->name;
      }
      if (g.loss.kind != G.user->loss_kind)
        return bail(Fail(CSE_ERR_INVALID, "group " + std::to_string(gi) + ": user functor kind " +
                                              G.user_name + " was registered with loss kind " +
                                              std::to_string(G.user->loss_kind) + ", the group has " +
                                              std::to_string(g.loss.kind)));
    } else if (g.loss.kind == CSE_LOSS_USER) {
      return bail(Fail(CSE_ERR_INVALID, "the user loss kind (3) needs a user functor kind registered with it"));
    }
    if (g.num_blocks < 0 || (g.num_blocks > 0 && (!g.parameter_block_ids || !g.functor_data)))
      return bail(Fail(CSE_ERR_INVALID, "group " + std::to_string(gi) + " arrays missing"));
    G.kind = g.functor_kind;
    G.loss = g.loss;
    G.n = g.num_blocks;
    G.first = g.first_residual_block;
    const KindShape& k = G.shape;
    for (int64_t i = 0; i < g.num_blocks; ++i) {
      const int64_t gidx = g.residual_block_index ? g.residual_block_index[i] : g.first_residual_block + i;
      if (gidx < 0 || gidx >= d->num_residual_blocks)
        return bail(Fail(CSE_ERR_INVALID, "residual block index out of range in group " + std::to_string(gi)));
      if (d->residual_layout[gidx] < 0 || d->residual_layout[gidx] + k.nr > d->num_residuals)
        return bail(Fail(CSE_ERR_INVALID, "residual_layout out of range"));
      covered_res += k.nr;
      for (int j = 0; j < k.nb; ++j) {
        const int32_t id = g.parameter_block_ids[i * k.nb + j];
        if (id < 0 || id >= d->num_parameter_blocks)
          return bail(Fail(CSE_ERR_INVALID, "parameter block id out of range in group " + std::to_string(gi)));
        const int want = k.sz[j];
        const cse_parameter_block& pb = d->parameter_blocks[id];
        if (pb.size != want)
          return bail(Fail(CSE_ERR_INVALID, "parameter block size does not match the functor"));
        if (!pb.is_constant) covered_jac += (int64_t)k.nr * pb.tangent_size;
        const int32_t tag = 2 * gi + j;
        if (owner[id] == -1) owner[id] = tag;
        else if (owner[id] != tag) owner[id] = -2;
        if (!seen[id]) {
          seen[id] = 1;
          ev->bytes_jac += 8LL * pb.size;
          ev->bytes_res += 8LL * pb.size;
        }
      }
      if (ev->has_layout) {
        const int64_t base = d->jacobian_per_residual_layout[gidx];
        int na = 0;
        for (int j = 0; j < k.nb; ++j)
          if (!d->parameter_blocks[g.parameter_block_ids[i * k.nb + j]].is_constant) ++na;
        if (base < 0 || base + (int64_t)na * k.nr > d->num_jacobian_per_residual_offsets)
          return bail(Fail(CSE_ERR_INVALID, "jacobian_per_residual_layout out of range"));
        int a = 0;
        for (int j = 0; j < k.nb; ++j) {
          const cse_parameter_block& pb = d->parameter_blocks[g.parameter_block_ids[i * k.nb + j]];
          if (pb.is_constant) continue;
          for (int r = 0; r < k.nr; ++r) {
            const int64_t off = d->jacobian_per_residual_offsets[base + a * k.nr + r];
            if (off < 0 || off + pb.tangent_size > d->num_jacobian_values)
              return bail(Fail(CSE_ERR_INVALID, "jacobian offset out of range"));
          }
          ++a;
        }
      }
    }
    const int64_t per_block = 8LL * k.data + 4LL * k.nb + 8LL * k.nr;
    ev->bytes_res += per_block * g.num_blocks;
    ev->bytes_jac += per_block * g.num_blocks;
    G.policy = ev->opts.force_general_layout ? kTable : DetectAffine(d, g, k, &G);
    G.affine = G.policy != kTable;
    if (!G.affine) G.const0 = false;  // DetectAffine may have set it before giving up
    if (G.affine && g.functor_kind == CSE_FUNCTOR_SNAVELY_QUATERNION_2_10_3 &&
        G.slot0_manifold == CSE_MANIFOLD_QUATERNION_EUCLIDEAN) {
      // Slot 0 on the quaternion manifold (DetectAffine checked every active
      // block; a held camera's own manifold is irrelevant): the kernel kind
      // with the tangent Jacobian (k follows G.shape).
      G.kind = kKindQuaternionTangent;
      ShapeOf(G.kind, &G.shape);
    }
    // Constant slot-0 blocks need the repacked table (their values come from
    // the constant state through it).
    if (G.const0 && G.slot0_count > (1 << 20)) {
      G.policy = kTable;
      G.affine = false;
      G.const0 = false;
      if (G.kind == kKindQuaternionTangent) {
        G.kind = g.functor_kind;
        ShapeOf(G.kind, &G.shape);
      }
    }
    // The Jet form of the Snavely functor (cse_options.jacobian_form) is
    // instantiated for the affine kernels with the LDS-DMA gather and without
    // held cameras, and for the table kernel: other Snavely groups take the
    // table path.
    G.jet = ev->opts.jacobian_form == CSE_JACOBIAN_JET && g.functor_kind == CSE_FUNCTOR_SNAVELY_2_9_3;
    if (G.jet && G.affine && (G.const0 || G.slot0_count <= 0 || G.slot0_count > (1 << 20))) {
      G.policy = kTable;
      G.affine = false;
      G.const0 = false;
    }
    // Table-path tables: also for const0 groups (their J products use the
    // table kernels).
    if (G.const0) ev->any_general = true;
    if (!G.affine) ev->any_general = true;
    if (G.affine) {
      const int64_t chunks = (g.num_blocks + cse::kWave - 1) / cse::kWave;
      G.num_wg = std::max<int64_t>(1, (chunks + cse::kWavesPerBlock - 1) / cse::kWavesPerBlock);
    } else {
      G.num_wg = (g.num_blocks + cse::kBlockThreads - 1) / cse::kBlockThreads;
    }
    // Every kernel writes one cost partial per wave.
    G.partial_offset = ev->total_wg;
    ev->total_wg += G.num_wg * cse::kWavesPerBlock;
    // The LDS-DMA gather reads slot 0 from a repacked copy refreshed every
    // evaluation; worth it while the slot-0 id range is small (BAL: the
    // cameras), otherwise gather 8-byte pieces from the state directly.
    if (G.affine && G.slot0_count > 0 && G.slot0_count <= (1 << 20) &&
        (rc = G.packed0.alloc((size_t)G.slot0_count * G.packed_stride)))
      return bail(rc);
    if (G.const0) {
      std::vector<uint32_t> bits((size_t)((G.slot0_count + 31) / 32), 0u);
      std::vector<int64_t> src((size_t)G.slot0_count, 0), dlt((size_t)G.slot0_count, -1);
      // Ids in the range that are not camera-sized rows in bounds (blocks no
      // block of the group uses) repack the first active camera (never read).
      const int64_t fallback = G.state_base[0] + (int64_t)k.x0 * G.slot0_lo;  // overwritten below
      int64_t first_active = -1;
      for (int64_t q = 0; q < G.slot0_count && first_active < 0; ++q) {
        const cse_parameter_block& pb = d->parameter_blocks[G.slot0_lo + q];
        if (!pb.is_constant && pb.size == k.x0) first_active = pb.state_offset;
      }
      for (int64_t q = 0; q < G.slot0_count; ++q) {
        const cse_parameter_block& pb = d->parameter_blocks[G.slot0_lo + q];
        const bool fits = pb.size == k.x0 && pb.state_offset >= 0 &&
                          pb.state_offset + k.x0 <= (pb.is_constant ? d->num_constant_parameters
                                                                    : d->num_parameters);
        if (!fits) {
          src[q] = first_active >= 0 ? first_active : fallback;
        } else if (pb.is_constant) {
          src[q] = -1 - pb.state_offset;
        } else {
          bits[q >> 5] |= 1u << (q & 31);
          src[q] = pb.state_offset;
          dlt[q] = pb.delta_offset;
        }
      }
      if ((rc = G.act0.upload(bits.data(), bits.size(), s))) return bail(rc);
      if ((rc = G.src0.upload(src.data(), src.size(), s))) return bail(rc);
      if ((rc = G.delta0.upload(dlt.data(), dlt.size(), s))) return bail(rc);
      if (!G.h_fbase.empty() && (rc = G.fbase.upload(G.h_fbase.data(), G.h_fbase.size(), s)))
        return bail(rc);
      if (!G.h_fbase.empty()) {
        const int64_t nchunks = (int64_t)G.h_fbase.size() - 1;
        std::vector<int32_t> prev((size_t)nchunks, -1);
        int32_t last = -1;
        for (int64_t c = 0; c < nchunks; ++c) {
          prev[c] = last;
          if (G.h_fbase[c + 1] > G.h_fbase[c]) last = (int32_t)c;
        }
        if ((rc = G.prev_seg.upload(prev.data(), prev.size(), s))) return bail(rc);
        if ((rc = G.side.alloc((size_t)nchunks * 16))) return bail(rc);
      }
      if (hipStreamSynchronize(s) != hipSuccess) return bail(Fail(CSE_ERR_HIP, "upload failed"));
    }
    if (G.affine && ev->has_layout) {
      const int sizes[2] = {k.s0, k.s1};
      for (int j = 0; j < k.nb; ++j)
        if (GradSupported(k.nr, sizes[j], G.user, j) &&
            (rc = BuildGradPlan(g, k, j, &G.grad[j], s,
                                j == 0 && G.const0 ? d->parameter_blocks : nullptr,
                                j == 0 && k.nb == 2 && (FusedKind(G.kind) || UserFused(G))
                                    ? CamGradPasses(g, k)
                                    : 1)))
          return bail(rc);
    }
    if ((rc = BuildTableRuns(ev, d, g, &G, s))) return bail(rc);
    DetectPlain0(d, g, &G);
    if (G.plain0) {
      // A plain slot 0 of a small id range (the cameras) is read from a
      // repacked copy, as the affine kernels read it (RepackSlot0Kernel, every
      // evaluation): one 128-byte row a lane instead of its values at an
      // 8-byte alignment.
      int32_t lo = INT32_MAX, hi = INT32_MIN;
      for (int64_t i = 0; i < g.num_blocks; ++i) {
        lo = std::min(lo, g.parameter_block_ids[i * k.nb]);
        hi = std::max(hi, g.parameter_block_ids[i * k.nb]);
      }
      const int64_t count = (int64_t)hi - lo + 1;
      if (k.sz[0] <= 16 && count <= (1 << 20)) {
        G.slot0_lo = lo;
        G.slot0_count = count;
        G.packed_stride = cse::PackedRowDoubles(k.sz[0]);
        G.state_base[0] = G.plain0_state_base;
        if ((rc = G.packed0.alloc((size_t)count * G.packed_stride))) return bail(rc);
      }
    }
    if ((rc = G.ids.upload(g.parameter_block_ids, (size_t)g.num_blocks * k.nb, s))) return bail(rc);
    if ((rc = G.data.upload(g.functor_data, (size_t)g.num_blocks * k.data, s))) return bail(rc);
    if ((!G.affine || G.const0) && g.residual_block_index &&
        (rc = G.gindex.upload(g.residual_block_index, (size_t)g.num_blocks, s)))
      return bail(rc);
    ev->groups.push_back(std::move(G));
  }
  ev->bytes_jac += 8LL * covered_jac;
  // Fused gradient eligibility: a Snavely group on the affine LDS-DMA path
  // whose slot-1 blocks are sorted (identity plan) and used by no other
  // group or slot (the fused kernel stores their rows, it does not add),
  // and whose slot-0 blocks have a chunked plan.
  for (int gi = 0; gi < (int)ev->groups.size(); ++gi) {
    Group& G = ev->groups[gi];
    bool ok = (FusedKind(G.kind) || UserFused(G)) && G.affine && G.n > 0 && G.packed0.p &&
              G.grad[0].ready && G.grad[0].perm.p && G.grad[0].nchunks > 0 && G.grad[1].ready &&
              G.grad[1].perm.p == nullptr;
    const cse_residual_group& g = d->groups[gi];
    for (int64_t i = 0; ok && i < g.num_blocks; ++i)
      ok = owner[g.parameter_block_ids[2 * i + 1]] == 2 * gi + 1;
    G.fuse_ok = ok;
    G.grad_exact = ok && ev->groups.size() == 1 && d->num_groups == 1 && !G.const0 &&
                   ev->num_constant == 0 && G.shape.s1 == 3 && G.grad[0].all_present &&
                   G.grad[1].all_present &&
                   G.shape.s0 * G.grad[0].count + 3 * G.grad[1].count == ev->num_effective;
  }
  if ((rc = BuildSchurPlan(ev, d, s))) return bail(rc);
  ev->res_covered = covered_res == d->num_residuals;
  ev->jac_covered = covered_jac == d->num_jacobian_values;

  // Program-level device state.
  if ((rc = ev->cstate.upload(d->constant_state, (size_t)d->num_constant_parameters, s))) return bail(rc);
  if ((rc = ev->plus_jac.upload(d->plus_jacobians, (size_t)d->num_plus_jacobian_values, s))) return bail(rc);
  if (ev->any_general) {
    std::vector<cse::PbDev> pbs(d->num_parameter_blocks);
    for (int64_t b = 0; b < d->num_parameter_blocks; ++b) {
      const cse_parameter_block& pb = d->parameter_blocks[b];
      const int64_t pj = pb.manifold == CSE_MANIFOLD_QUATERNION_EUCLIDEAN
                             ? cse::kPlusJacobianQuaternion
                             : pb.plus_jacobian_offset;
      pbs[b] = {pb.state_offset, pb.delta_offset, pj, pb.tangent_size, pb.is_constant};
    }
    if ((rc = ev->pbs.upload(pbs.data(), pbs.size(), s))) return bail(rc);
    if ((rc = ev->res_layout.upload(d->residual_layout, (size_t)d->num_residual_blocks, s))) return bail(rc);
    if (ev->has_layout) {
      if ((rc = ev->jac_layout.upload(d->jacobian_per_residual_layout, (size_t)d->num_residual_blocks, s)))
        return bail(rc);
      if ((rc = ev->jac_offsets.upload(d->jacobian_per_residual_offsets,
                                       (size_t)d->num_jacobian_per_residual_offsets, s)))
        return bail(rc);
    }
  }
  if ((rc = ev->partials.alloc(std::max<int64_t>(ev->total_wg, 1)))) return bail(rc);
  // Slots of groups that launch nothing (empty groups) must read as zero.
  if (hipMemsetAsync(ev->partials.p, 0, ev->partials.n * sizeof(double), s) != hipSuccess)
    return bail(Fail(CSE_ERR_HIP, "hipMemsetAsync failed"));
  if ((rc = ev->partials2.alloc(kPartialBlocks))) return bail(rc);
  // [0] running flag, [1] last status, [2] ReduceFinalizeKernel's counter
  if ((rc = ev->status.alloc(3))) return bail(rc);
  if (hipMemsetAsync(ev->status.p, 0, 3 * sizeof(int), s) != hipSuccess)
    return bail(Fail(CSE_ERR_HIP, "memset failed"));
  if (hipHostMalloc(&ev->status_host, sizeof(int)) != hipSuccess)
    return bail(Fail(CSE_ERR_HIP, "hipHostMalloc failed"));
  if (hipStreamSynchronize(s) != hipSuccess) return bail(Fail(CSE_ERR_HIP, "upload failed"));
  *out = ev;
  return CSE_OK;
}

int cse_evaluate_device_ex(cse_evaluator* ev, const double* d_state, double* d_cost,
                           double* d_residuals, double* d_gradient, double* d_jacobian_values,
                           uint32_t flags) {
  if (!ev || !d_cost) return Fail(CSE_ERR_INVALID, "null evaluator or cost");
  CSE_SINGLE_DEVICE(ev, "cse_evaluate_device");
  if (flags & ~(uint32_t)CSE_EVAL_SAME_POINT) return Fail(CSE_ERR_INVALID, "unknown evaluate flags");
  if (ev->num_parameters > 0 && !d_state) return Fail(CSE_ERR_INVALID, "null state");
  if (hipSetDevice(ev->device) != hipSuccess) return Fail(CSE_ERR_HIP, "hipSetDevice failed");
  ev->host_state_current = false;
  return Enqueue(ev, d_state, d_cost, d_residuals, d_gradient, d_jacobian_values,
                 (flags & CSE_EVAL_SAME_POINT) != 0);
}

int cse_evaluate_device(cse_evaluator* ev, const double* d_state, double* d_cost,
                        double* d_residuals, double* d_gradient, double* d_jacobian_values) {
  return cse_evaluate_device_ex(ev, d_state, d_cost, d_residuals, d_gradient, d_jacobian_values, 0);
}

int cse_wait(cse_evaluator* ev) {
  if (!ev) return Fail(CSE_ERR_INVALID, "null evaluator");
  if (ev->multi) return CSE_OK;  // cse_evaluate on it is synchronous
  CSE_HIP(hipMemcpyAsync(ev->status_host, ev->status.p + 1, sizeof(int), hipMemcpyDeviceToHost,
                         ev->stream));
  CSE_HIP(hipStreamSynchronize(ev->stream));
  if (ev->opts.profile) {
    int rc = FoldTiming(ev);
    if (rc) return rc;
  }
  return *ev->status_host ? CSE_EVALUATION_FAILED : CSE_OK;
}

int cse_evaluate_ex(cse_evaluator* ev, const double* state, double* cost, double* residuals,
                    double* gradient, double* jacobian_values, uint32_t flags) {
  if (!ev || !cost) return Fail(CSE_ERR_INVALID, "null evaluator or cost");
  if (flags & ~(uint32_t)CSE_EVAL_SAME_POINT) return Fail(CSE_ERR_INVALID, "unknown evaluate flags");
  const bool same_point = (flags & CSE_EVAL_SAME_POINT) != 0;
  if (ev->multi) {
    if (!state) return Fail(CSE_ERR_INVALID, "null state");
    return MultiEvaluate(ev->multi, state, cost, residuals, gradient, jacobian_values, same_point);
  }
  if (ev->num_parameters > 0 && !state) return Fail(CSE_ERR_INVALID, "null state");
  CSE_HIP(hipSetDevice(ev->device));
  int rc;
  if (!ev->h_state.p && (rc = ev->h_state.alloc(std::max<int64_t>(ev->num_parameters, 1)))) return rc;
  if (!ev->h_cost.p && (rc = ev->h_cost.alloc(1))) return rc;
  if (residuals && !ev->h_res.p && (rc = ev->h_res.alloc(std::max<int64_t>(ev->num_residuals, 1)))) return rc;
  if (gradient && !ev->h_grad.p && (rc = ev->h_grad.alloc(std::max<int64_t>(ev->num_effective, 1)))) return rc;
  if (jacobian_values && !ev->h_jac.p &&
      (rc = ev->h_jac.alloc(std::max<int64_t>(ev->num_jacobian_values, 1))))
    return rc;
  // At the same point the state uploaded for the previous host-pointer
  // evaluation is still in h_state (Evaluator::EvaluateOptions::
  // new_evaluation_point == false, trust_region_minimizer.cc:826).
  if (ev->num_parameters > 0 && !(same_point && ev->host_state_current)) {
    ev->host_state_current = false;
    CSE_HIP(hipMemcpyAsync(ev->h_state.p, state, ev->num_parameters * sizeof(double),
                           hipMemcpyHostToDevice, ev->stream));
  }
  rc = Enqueue(ev, ev->h_state.p, ev->h_cost.p, residuals ? ev->h_res.p : nullptr,
               gradient ? ev->h_grad.p : nullptr, jacobian_values ? ev->h_jac.p : nullptr, same_point);
  if (rc) return rc;
  ev->host_state_current = true;
  rc = cse_wait(ev);
  if (rc < 0) return rc;
  if (rc == CSE_EVALUATION_FAILED) return rc;
  CSE_HIP(hipMemcpy(cost, ev->h_cost.p, sizeof(double), hipMemcpyDeviceToHost));
  if (residuals && ev->num_residuals > 0)
    CSE_HIP(hipMemcpy(residuals, ev->h_res.p, ev->num_residuals * sizeof(double), hipMemcpyDeviceToHost));
  if (gradient && ev->num_effective > 0)
    CSE_HIP(hipMemcpy(gradient, ev->h_grad.p, ev->num_effective * sizeof(double), hipMemcpyDeviceToHost));
  if (jacobian_values && ev->num_jacobian_values > 0)
    CSE_HIP(hipMemcpy(jacobian_values, ev->h_jac.p, ev->num_jacobian_values * sizeof(double),
                      hipMemcpyDeviceToHost));
  return CSE_OK;
}

int cse_evaluate(cse_evaluator* ev, const double* state, double* cost, double* residuals,
                 double* gradient, double* jacobian_values) {
  return cse_evaluate_ex(ev, state, cost, residuals, gradient, jacobian_values, 0);
}

int cse_set_plus_jacobians(cse_evaluator* ev, const double* plus_jacobians) {
  if (!ev) return Fail(CSE_ERR_INVALID, "null evaluator");
  if (ev->multi) return MultiSetPlusJacobians(ev->multi, plus_jacobians);
  if (ev->num_plus_jacobian_values == 0) return CSE_OK;
  if (!plus_jacobians) return Fail(CSE_ERR_INVALID, "null plus_jacobians");
  CSE_HIP(hipSetDevice(ev->device));
  CSE_HIP(hipMemcpyAsync(ev->plus_jac.p, plus_jacobians, ev->num_plus_jacobian_values * sizeof(double),
                         hipMemcpyHostToDevice, ev->stream));
  CSE_HIP(hipStreamSynchronize(ev->stream));
  return CSE_OK;
}

extern "C++" {
namespace {

bool DispatchMultiply(int kind, const cse::GroupArgs& a, bool affine, bool left, const double* x,
                      double* y, hipStream_t s) {
  const int which = affine && !left ? 0 : left ? 2 : 1;
  return VisitKind(kind, [&](auto kd) { cse::LaunchMultiplyKernel<decltype(kd)>(a, which, x, y, s); });
}

int JacobianMultiply(cse_evaluator* ev, const double* J, const double* x, double* y, bool left) {
  if (!ev) return Fail(CSE_ERR_INVALID, "null evaluator");
  CSE_SINGLE_DEVICE(ev, "cse_jacobian_multiply");
  if (!ev->has_layout)
    return Fail(CSE_ERR_INVALID, "the descriptor had no Jacobian layout");
  if (!J || !x || !y) return Fail(CSE_ERR_INVALID, "null pointer");
  CSE_HIP(hipSetDevice(ev->device));
  for (auto& G : ev->groups) {
    if (G.n == 0) continue;
    // Groups with constant slot-0 blocks take the table kernels (their F
    // cells are not at affine offsets).
    const bool affine = G.affine && !G.const0;
    bool plans = affine;
    for (int j = 0; j < G.shape.nb; ++j) plans = plans && G.grad[j].ready;
    // MakeArgs wants non-const outputs; the kernels only read a.jacobian.
    cse::GroupArgs a = MakeArgs(ev, G, nullptr, nullptr, const_cast<double*>(J), nullptr);
    if (left && plans) {
      const int sizes[2] = {G.shape.s0, G.shape.s1};
      for (int j = 0; j < G.shape.nb; ++j) {
        const Group::GradPlan& P = G.grad[j];
        cse::GradArgs ga{};
        ga.jac = J;
        for (int r = 0; r < G.shape.nr && r < 3; ++r) ga.jrow[r] = G.jac_base[j][r];
        ga.jstride = G.jac_stride[j];
        ga.res = x;
        ga.res_base = G.res_base;
        ga.perm = P.perm.p;
        ga.off = P.off.p;
        ga.count = P.count;
        ga.lo = P.lo;
        ga.grad = y;
        ga.delta_base = G.delta_base[j];
        if (!LaunchGradPass(G.shape.nr, sizes[j], ga, P, ev->stream, G.user, j))
          return Fail(CSE_ERR_UNSUPPORTED, "no J^T x pass for this shape");
      }
    } else {
      if (!G.affine && !ev->any_general)
        return Fail(CSE_ERR_UNSUPPORTED, "table-path tables were not uploaded");
      if (G.user) {
        if (!G.user->multiply)
          return Fail(CSE_ERR_UNSUPPORTED, "user functor kind " + G.user_name + " has no multiply kernel");
        G.user->multiply(&a, affine && !left ? 0 : left ? 2 : 1, x, y, ev->stream);
      } else if (!DispatchMultiply(G.kind, a, affine, left, x, y, ev->stream))
        return Fail(CSE_ERR_UNSUPPORTED, "no multiply kernel for functor kind " +
                                             std::to_string(G.kind));
    }
    CSE_HIP(hipGetLastError());
  }
  return CSE_OK;
}

}  // namespace
}  // extern "C++"

int cse_jacobian_right_multiply(cse_evaluator* ev, const double* d_jacobian_values,
                                const double* d_x, double* d_y) {
  return JacobianMultiply(ev, d_jacobian_values, d_x, d_y, false);
}

int cse_jacobian_left_multiply(cse_evaluator* ev, const double* d_jacobian_values,
                               const double* d_x, double* d_y) {
  return JacobianMultiply(ev, d_jacobian_values, d_x, d_y, true);
}

int cse_cgnr_multiply(cse_evaluator* ev, const double* d_jacobian_values, const double* d_D,
                      const double* d_x, double* d_y) {
  if (!ev) return Fail(CSE_ERR_INVALID, "null evaluator");
  CSE_SINGLE_DEVICE(ev, "cse_cgnr_multiply");
  if (!ev->has_layout) return Fail(CSE_ERR_INVALID, "the descriptor had no Jacobian layout");
  if (!d_jacobian_values || !d_x || !d_y) return Fail(CSE_ERR_INVALID, "null pointer");
  CSE_HIP(hipSetDevice(ev->device));
  hipStream_t s = ev->stream;
  if (d_D && ev->num_effective > 0)
    hipLaunchKernelGGL(cse::DtDxpyKernel,
                       dim3((unsigned)((ev->num_effective + cse::kBlockThreads - 1) / cse::kBlockThreads)),
                       dim3(cse::kBlockThreads), 0, s, d_D, d_x, d_y, ev->num_effective);
  bool fused = true;
  for (auto& G : ev->groups) fused = fused && (G.n == 0 || (G.fuse_ok && !G.const0 && SnavelyShaped(G)));
  if (!fused) {
    // z = J x, then y += J^T z: the two products of CudaCgnrLinearOperator.
    int rc;
    if ((rc = ev->cg_z.ensure((size_t)std::max<int64_t>(ev->num_residuals, 1)))) return rc;
    CSE_HIP(hipMemsetAsync(ev->cg_z.p, 0, ev->num_residuals * sizeof(double), s));
    if ((rc = JacobianMultiply(ev, d_jacobian_values, d_x, ev->cg_z.p, false))) return rc;
    return JacobianMultiply(ev, d_jacobian_values, ev->cg_z.p, d_y, true);
  }
  for (auto& G : ev->groups) {
    if (G.n == 0) continue;
    const int64_t chunks = (G.n + cse::kWave - 1) / cse::kWave;
    int rc;
    if ((rc = G.gside.ensure((size_t)(2 * chunks * 4)))) return rc;
    if ((rc = G.gcontrib.ensure((size_t)G.n * G.slot0_stride))) return rc;
    cse::GroupArgs a = MakeArgs(ev, G, nullptr, nullptr, const_cast<double*>(d_jacobian_values),
                                nullptr);
    a.gside = G.gside.p;
    a.gcontrib = G.gcontrib.p;
    constexpr int W = kOperatorWavesPerWg;
    const dim3 grid((unsigned)((chunks + W - 1) / W));
    if (G.policy == kAffineCrs)
      hipLaunchKernelGGL((cse::CgnrMultiplyKernel<cse::SnavelyKind, true, W>), grid,
                         dim3(W * cse::kWave), 0, s, a, d_x, d_y);
    else
      hipLaunchKernelGGL((cse::CgnrMultiplyKernel<cse::SnavelyKind, false, W>), grid,
                         dim3(W * cse::kWave), 0, s, a, d_x, d_y);
    CSE_HIP(hipGetLastError());
    if ((rc = LaunchFusedGradTail(G, d_y, s))) return rc;
  }
  return CSE_OK;
}

// ---------------------------------------------------------------------------
// ITERATIVE_SCHUR on the device (schur_kernels.hpp)
// ---------------------------------------------------------------------------
extern "C++" {
namespace {

cse::SchurArgs MakeSchurArgs(cse_evaluator* ev, const double* x, double* y) {
  const Group& G = ev->groups[0];
  const auto& S = ev->schur;
  cse::SchurArgs a{};
  a.n = G.n;
  a.ids = G.ids.p;
  a.jac = S.jac;
  a.f_base = G.jac_base[0][0];
  a.e_base = G.jac_base[1][0];
  a.f_col_base = S.f_col_base;
  a.e_col_base = G.delta_base[1];
  a.e_cols = S.e_cols;
  a.D = S.D;
  a.b = S.b;
  a.b_base = G.res_base;
  a.x = x;
  a.ete_inv = S.ete_inv.p;
  a.contrib = G.gcontrib.p;
  a.y = y;
  a.chunk_begin = S.chunk_begin.p;
  a.nchunks = S.nchunks;
  a.big = S.big.p;
  a.nbig = S.nbig;
  a.status = ev->status.p + 1;  // read by cse_wait
  return a;
}

template <int kMode, bool kGrad = false>
void LaunchSchurPass(const cse::SchurArgs& a, hipStream_t s) {
  constexpr int W = kOperatorWavesPerWg;
  if (a.nchunks > 0)
    hipLaunchKernelGGL((cse::SchurChunkKernel<9, kMode, W, kGrad>), dim3((unsigned)((a.nchunks + W - 1) / W)),
                       dim3(W * cse::kWave), 0, s, a);
  if (a.nbig > 0)
    hipLaunchKernelGGL((cse::SchurBigKernel<9, kMode, kGrad>),
                       dim3((unsigned)((a.nbig + cse::kWavesPerBlock - 1) / cse::kWavesPerBlock)),
                       dim3(cse::kBlockThreads), 0, s, a);
}

// y (f vector) += the per-f-block sums of the contributions just written.
int SchurFTail(cse_evaluator* ev, double* y, hipStream_t s) {
  const Group& G = ev->groups[0];
  const Group::GradPlan& P = G.grad[0];
  cse::GradArgs ga{};
  ga.count = P.count;
  ga.lo = P.lo;
  ga.grad = y;
  ga.delta_base = ev->schur.f_col_base;
  const cse::GradChunks ch{P.chunk_begin.p, P.chunk_off.p, P.chunk_partial.p, P.nchunks};
  if (P.nchunks > 0)
    hipLaunchKernelGGL((cse::GradientContribKernel<9, 10>),
                       dim3((unsigned)((P.nchunks + cse::kWavesPerBlock - 1) / cse::kWavesPerBlock)),
                       dim3(cse::kBlockThreads), 0, s, G.gcontrib.p, P.perm.p, ch,
                       P.chunk_order.p);
  hipLaunchKernelGGL((cse::GradientChunkReduceKernel<9>),
                     dim3((unsigned)((ga.count + cse::kBlockThreads - 1) / cse::kBlockThreads)),
                     dim3(cse::kBlockThreads), 0, s, ga, ch);
  CSE_HIP(hipGetLastError());
  return CSE_OK;
}

// The init's camera-order pass and the per-camera finish (schur_kernels.hpp).
struct SchurCameraLaunch {
  cse::SchurArgs a;
  const Group::GradPlan* P;
  cse::GradChunks ch;
  const double* D;
  int64_t d_off;  // D index of the plan's first camera's first column
  double* precond;
  int* status;
  double* rhs;   // rhs row of the plan's first camera
  double* grad;  // gradient row of the plan's first camera (null: no gradient)
};

template <int kDiag, bool kGrad>
void LaunchSchurCameraPass(const SchurCameraLaunch& L, hipStream_t s) {
  const Group::GradPlan& P = *L.P;
  if (P.nchunks > 0)
    hipLaunchKernelGGL((cse::SchurCameraPassKernel<9, kDiag, kGrad>),
                       dim3((unsigned)((P.nchunks + cse::kWavesPerBlock - 1) / cse::kWavesPerBlock)),
                       dim3(cse::kBlockThreads), 0, s, L.a, P.perm.p, L.ch, P.chunk_order.p);
  if (P.count > 0)
    hipLaunchKernelGGL((cse::SchurCameraFinishKernel<9, kDiag, kGrad>),
                       dim3((unsigned)((P.count + 63) / 64)), dim3(64), 0, s, L.ch, P.count, L.D,
                       L.d_off, L.precond, L.status, L.rhs, L.grad);
}

int SchurCheck(cse_evaluator* ev, bool need_ready) {
  if (!ev) return Fail(CSE_ERR_INVALID, "null evaluator");
  CSE_SINGLE_DEVICE(ev, "cse_schur");
  if (!ev->schur.eligible)
    return Fail(CSE_ERR_UNSUPPORTED,
                "implicit Schur complement: needs one Snavely-shaped group (2 residuals, blocks of 9 and 3) "
                "on the affine BlockSparse path "
                "with its points (slot 1) as the leading e columns and its cameras after them");
  if (need_ready && !ev->schur.ready) return Fail(CSE_ERR_INVALID, "cse_schur_init has not run");
  CSE_HIP(hipSetDevice(ev->device));
  return CSE_OK;
}

}  // namespace
}  // extern "C++"

int cse_schur_structure(cse_evaluator* ev, int64_t* num_cols_e, int64_t* num_cols_f) {
  int rc = SchurCheck(ev, false);
  if (rc) return rc;
  if (num_cols_e) *num_cols_e = ev->schur.e_cols;
  if (num_cols_f) *num_cols_f = ev->schur.f_cols;
  return CSE_OK;
}

extern "C++" {
namespace {
int SchurInit(cse_evaluator* ev, const double* d_jacobian_values, const double* d_D, const double* d_b,
              double* d_rhs, int preconditioner, double* d_gradient) {
  int rc = SchurCheck(ev, false);
  if (rc) return rc;
  if (!d_jacobian_values || !d_b || !d_rhs) return Fail(CSE_ERR_INVALID, "null pointer");
  auto& S = ev->schur;
  if (preconditioner != CSE_SCHUR_IDENTITY && preconditioner != CSE_SCHUR_JACOBI &&
      preconditioner != CSE_SCHUR_SCHUR_JACOBI)
    return Fail(CSE_ERR_INVALID, "unknown preconditioner");
  if (preconditioner == CSE_SCHUR_SCHUR_JACOBI && S.duplicates)
    return Fail(CSE_ERR_UNSUPPORTED,
                "SCHUR_JACOBI: an e block sees one f block in two residual blocks");
  Group& G = ev->groups[0];
  hipStream_t s = ev->stream;
  const bool grad = d_gradient != nullptr;
  if ((rc = S.ete_inv.ensure((size_t)2 * S.e_cols))) return rc;
  if ((rc = G.gcontrib.ensure((size_t)G.n * G.slot0_stride))) return rc;  // the multiplies'
  if ((rc = S.ub.ensure((size_t)G.n * (grad ? 4 : 2)))) return rc;
  S.jac = d_jacobian_values;
  S.D = d_D;
  S.b = d_b;
  S.preconditioner = preconditioner;
  // Point order: M_p, u_b = b_b - E_b M_p E_b^T b (and the gradient's e
  // rows); then camera order: rhs = F^T u, the gradient's f rows -F^T b and
  // the preconditioner's F^T Q F, each F cell read once.  The status word
  // read by cse_wait reports a non-positive pivot (schur_kernels.hpp, PivotOk).
  CSE_HIP(hipMemsetAsync(ev->status.p + 1, 0, sizeof(int), s));
  CSE_HIP(hipMemsetAsync(d_rhs, 0, S.f_cols * sizeof(double), s));
  if (grad)  // rows of blocks without residual blocks stay 0
    CSE_HIP(hipMemsetAsync(d_gradient, 0, ev->num_effective * sizeof(double), s));
  cse::SchurArgs a = MakeSchurArgs(ev, nullptr, nullptr);
  a.ub = S.ub.p;
  a.grad = d_gradient;
  if (grad)
    LaunchSchurPass<cse::kSchurInit, true>(a, s);
  else
    LaunchSchurPass<cse::kSchurInit>(a, s);
  CSE_HIP(hipGetLastError());
  const Group::GradPlan& P = G.grad[0];
  const int diag = preconditioner == CSE_SCHUR_IDENTITY ? 0 : preconditioner == CSE_SCHUR_JACOBI ? 1 : 2;
  const int parts = (diag ? cse::SymCount<9>() : 0) + 9 * (grad ? 2 : 1);
  if ((rc = S.partial.ensure((size_t)std::max<int64_t>(1, P.nchunks) * parts))) return rc;
  if (diag && (rc = S.precond.ensure((size_t)81 * P.count))) return rc;
  const cse::GradChunks ch{P.chunk_begin.p, P.chunk_off.p, S.partial.p, P.nchunks};
  // d_off: D index of camera lo + p = e_cols + f index = e_cols + f_col_base + 9 (lo + p).
  const int64_t d_off = S.e_cols + S.f_col_base + 9LL * P.lo;
  double* rhs_p = d_rhs + S.f_col_base + 9LL * P.lo;
  double* grad_p = grad ? d_gradient + G.delta_base[0] + 9LL * P.lo : nullptr;
  int* status = ev->status.p + 1;
  const SchurCameraLaunch L{a, &P, ch, d_D, d_off, S.precond.p, status, rhs_p, grad_p};
  switch (diag * 2 + (grad ? 1 : 0)) {
    case 0: LaunchSchurCameraPass<0, false>(L, s); break;
    case 1: LaunchSchurCameraPass<0, true>(L, s); break;
    case 2: LaunchSchurCameraPass<1, false>(L, s); break;
    case 3: LaunchSchurCameraPass<1, true>(L, s); break;
    case 4: LaunchSchurCameraPass<2, false>(L, s); break;
    default: LaunchSchurCameraPass<2, true>(L, s); break;
  }
  CSE_HIP(hipGetLastError());
  S.ready = true;
  return CSE_OK;
}
}  // namespace
}  // extern "C++"

int cse_schur_init(cse_evaluator* ev, const double* d_jacobian_values, const double* d_D,
                   const double* d_b, double* d_rhs, int preconditioner) {
  return SchurInit(ev, d_jacobian_values, d_D, d_b, d_rhs, preconditioner, nullptr);
}

int cse_schur_init_gradient(cse_evaluator* ev, const double* d_jacobian_values, const double* d_D,
                            const double* d_b, double* d_rhs, int preconditioner,
                            double* d_gradient) {
  if (!d_gradient) return Fail(CSE_ERR_INVALID, "null gradient");
  return SchurInit(ev, d_jacobian_values, d_D, d_b, d_rhs, preconditioner, d_gradient);
}

int cse_schur_multiply(cse_evaluator* ev, const double* d_x, double* d_y) {
  int rc = SchurCheck(ev, true);
  if (rc) return rc;
  if (!d_x || !d_y) return Fail(CSE_ERR_INVALID, "null pointer");
  const auto& S = ev->schur;
  hipStream_t s = ev->stream;
  hipLaunchKernelGGL(cse::SchurDiagKernel,
                     dim3((unsigned)((S.f_cols + cse::kBlockThreads - 1) / cse::kBlockThreads)),
                     dim3(cse::kBlockThreads), 0, s, S.D, S.e_cols, d_x, d_y, S.f_cols);
  LaunchSchurPass<cse::kSchurMultiply>(MakeSchurArgs(ev, d_x, nullptr), s);
  CSE_HIP(hipGetLastError());
  return SchurFTail(ev, d_y, s);
}

int cse_schur_precondition(cse_evaluator* ev, const double* d_x, double* d_y) {
  int rc = SchurCheck(ev, true);
  if (rc) return rc;
  if (!d_x || !d_y) return Fail(CSE_ERR_INVALID, "null pointer");
  const auto& S = ev->schur;
  hipStream_t s = ev->stream;
  const unsigned grid = (unsigned)((S.f_cols + cse::kBlockThreads - 1) / cse::kBlockThreads);
  if (S.preconditioner == CSE_SCHUR_IDENTITY) {  // IdentityPreconditioner: y += x
    hipLaunchKernelGGL(cse::AxpyKernel, dim3(grid), dim3(cse::kBlockThreads), 0, s, d_x, d_y,
                       S.f_cols);
    CSE_HIP(hipGetLastError());
    return CSE_OK;
  }
  const Group::GradPlan& P = ev->groups[0].grad[0];
  // The cameras' f rows start at f index f_col_base + 9 lo.
  const int64_t off = S.f_col_base + 9LL * P.lo;
  hipLaunchKernelGGL((cse::SchurPrecondApplyKernel<9>), dim3(grid), dim3(cse::kBlockThreads), 0, s,
                     S.precond.p, d_x + off, d_y + off, 9LL * P.count);
  CSE_HIP(hipGetLastError());
  return CSE_OK;
}

int cse_schur_back_substitute(cse_evaluator* ev, const double* d_x, double* d_y) {
  int rc = SchurCheck(ev, true);
  if (rc) return rc;
  if (!d_x || !d_y) return Fail(CSE_ERR_INVALID, "null pointer");
  const auto& S = ev->schur;
  hipStream_t s = ev->stream;
  // e part: (E^T E + D_e^2)^-1 E^T (b - F x); f part: x.
  CSE_HIP(hipMemsetAsync(d_y, 0, S.e_cols * sizeof(double), s));
  LaunchSchurPass<cse::kSchurBack>(MakeSchurArgs(ev, d_x, d_y), s);
  CSE_HIP(hipGetLastError());
  CSE_HIP(hipMemcpyAsync(d_y + S.e_cols, d_x, S.f_cols * sizeof(double), hipMemcpyDeviceToDevice, s));
  return CSE_OK;
}

int cse_plus_device(cse_evaluator* ev, const double* d_state, const double* d_delta,
                    double* d_state_plus_delta) {
  if (!ev) return Fail(CSE_ERR_INVALID, "null evaluator");
  CSE_SINGLE_DEVICE(ev, "cse_plus_device");
  if (!ev->plus_supported)
    return Fail(CSE_ERR_UNSUPPORTED,
                "Plus on device: an active parameter block has an explicit plus-Jacobian manifold");
  if (ev->plus_runs_host.empty() && ev->plus_quat_host.empty()) return CSE_OK;
  if (!d_state || !d_delta || !d_state_plus_delta) return Fail(CSE_ERR_INVALID, "null pointer");
  CSE_HIP(hipSetDevice(ev->device));
  if (!ev->plus_runs_host.empty()) {
    if (!ev->plus_runs.p) {
      int rc = ev->plus_runs.upload(ev->plus_runs_host.data(), ev->plus_runs_host.size(), ev->stream);
      if (rc) return rc;
    }
    const int64_t n = ev->num_parameters;
    const unsigned grid = (unsigned)std::max<int64_t>(
        1, std::min<int64_t>((n + cse::kBlockThreads - 1) / cse::kBlockThreads, 8LL * ev->num_cus));
    hipLaunchKernelGGL(cse::PlusKernel, dim3(grid), dim3(cse::kBlockThreads), 0, ev->stream, d_state,
                       d_delta, d_state_plus_delta, ev->plus_runs.p, (int)ev->plus_runs_host.size());
  }
  if (!ev->plus_quat_host.empty()) {
    if (!ev->plus_quat.p) {
      int rc = ev->plus_quat.upload(ev->plus_quat_host.data(), ev->plus_quat_host.size(), ev->stream);
      if (rc) return rc;
    }
    const int64_t nq = (int64_t)ev->plus_quat_host.size();
    hipLaunchKernelGGL(cse::QuaternionPlusKernel,
                       dim3((unsigned)((nq + cse::kBlockThreads - 1) / cse::kBlockThreads)),
                       dim3(cse::kBlockThreads), 0, ev->stream, d_state, d_delta, d_state_plus_delta,
                       ev->plus_quat.p, nq);
  }
  CSE_HIP(hipGetLastError());
  return CSE_OK;
}

int cse_plus(cse_evaluator* ev, const double* state, const double* delta,
             double* state_plus_delta) {
  if (!ev) return Fail(CSE_ERR_INVALID, "null evaluator");
  if (ev->multi) return MultiPlus(ev->multi, state, delta, state_plus_delta);
  if (!ev->plus_supported)
    return Fail(CSE_ERR_UNSUPPORTED,
                "Plus on device: an active parameter block has an explicit plus-Jacobian manifold");
  if (ev->num_parameters == 0) return CSE_OK;
  if (!state || !delta || !state_plus_delta) return Fail(CSE_ERR_INVALID, "null pointer");
  CSE_HIP(hipSetDevice(ev->device));
  int rc;
  if ((rc = ev->h_state.ensure(ev->num_parameters))) return rc;
  if ((rc = ev->h_delta.ensure(std::max<int64_t>(1, ev->num_effective)))) return rc;
  if ((rc = ev->h_plus.ensure(ev->num_parameters))) return rc;
  CSE_HIP(hipMemcpyAsync(ev->h_state.p, state, ev->num_parameters * sizeof(double),
                         hipMemcpyHostToDevice, ev->stream));
  CSE_HIP(hipMemcpyAsync(ev->h_delta.p, delta, ev->num_effective * sizeof(double),
                         hipMemcpyHostToDevice, ev->stream));
  double* out = ev->h_plus.p;
  if ((rc = cse_plus_device(ev, ev->h_state.p, ev->h_delta.p, out))) return rc;
  CSE_HIP(hipMemcpyAsync(state_plus_delta, out, ev->num_parameters * sizeof(double),
                         hipMemcpyDeviceToHost, ev->stream));
  CSE_HIP(hipStreamSynchronize(ev->stream));
  return CSE_OK;
}

void cse_destroy(cse_evaluator* ev) {
  if (!ev) return;
  if (ev->multi) {
    MultiDestroy(ev->multi);
    delete ev;
    return;
  }
  (void)hipSetDevice(ev->device);
  if (ev->stream) (void)hipStreamSynchronize(ev->stream);
  if (ev->status_host) (void)hipHostFree(ev->status_host);
  for (auto& pr : ev->pending) ev->pool.push_back(pr);
  for (auto& pr : ev->pool) {
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  if (ev->own_stream && ev->stream) (void)hipStreamDestroy(ev->stream);
  delete ev;  // every DevBuf (groups, plans, tables, scratch) frees itself
}

int cse_create_multi(const cse_problem_desc* d, const cse_options* options, const int32_t* devices,
                     int32_t num_devices, cse_evaluator** out) {
  if (!out) return Fail(CSE_ERR_INVALID, "null out");
  *out = nullptr;
  int rc = Validate(d);
  if (rc) return rc;
  if (options && (options->gradient_mode < 0 || options->gradient_mode > 3))
    return Fail(CSE_ERR_INVALID, "gradient_mode " + std::to_string(options->gradient_mode) +
                                     " is not one of 0..3");
  cse_evaluator* ev = new (std::nothrow) cse_evaluator();
  if (!ev) return Fail(CSE_ERR_OOM, "host allocation failed");
  if ((rc = MultiCreate(d, options, devices, num_devices, &ev->multi))) {
    delete ev;
    return rc;
  }
  ev->device = devices[0];
  *out = ev;
  return CSE_OK;
}

int cse_shard_info(cse_evaluator* ev, int32_t* num_shards, int64_t* first_block, int32_t* devices) {
  if (!ev) return Fail(CSE_ERR_INVALID, "null evaluator");
  if (ev->multi) return MultiShardInfo(ev->multi, num_shards, first_block, devices);
  if (num_shards) *num_shards = 1;
  if (first_block) {
    first_block[0] = 0;
    first_block[1] = ev->num_residual_blocks;
  }
  if (devices) devices[0] = ev->device;
  return CSE_OK;
}

int cse_shard_transfer_bytes(cse_evaluator* ev, int64_t* state_h2d_bytes, int64_t* strips_d2h_bytes) {
  if (!ev) return Fail(CSE_ERR_INVALID, "null evaluator");
  if (ev->multi) return MultiTransferBytes(ev->multi, state_h2d_bytes, strips_d2h_bytes);
  if (state_h2d_bytes) state_h2d_bytes[0] = ev->num_parameters * (int64_t)sizeof(double);
  if (strips_d2h_bytes)
    strips_d2h_bytes[0] = (ev->num_residuals + ev->num_jacobian_values) * (int64_t)sizeof(double);
  return CSE_OK;
}

int cse_host_register(void* p, size_t bytes) { return CseHostRegister(p, bytes); }

int cse_host_unregister(void* p) { return CseHostUnregister(p); }

// Registration compares whole tables bytewise: no padding inside.
static_assert(offsetof(cse_functor_ops, kernel_args_tag) == 80 && sizeof(cse_functor_ops) == 224,
              "cse_functor_ops layout");

int cse_register_functor(const cse_functor_ops* ops, int32_t* kind) {
  if (!ops || !kind) return Fail(CSE_ERR_INVALID, "null functor table or kind");
  const std::string name = ops->name ? ops->name : "(unnamed)";
  if (ops->abi_version != CSE_ABI_VERSION)
    return Fail(CSE_ERR_INVALID, "functor " + name + ": built against ABI " +
                                     std::to_string(ops->abi_version) + ", the library is " +
                                     std::to_string(CSE_ABI_VERSION));
  if (ops->kernel_args_size != (int32_t)sizeof(cse::GroupArgs) ||
      ops->gradient_args_size != (int32_t)sizeof(cse::GradArgs) ||
      ops->kernel_args_tag != cse::kGroupArgsTag)
    return Fail(CSE_ERR_INVALID, "functor " + name +
                                     ": kernel argument layout differs from the library's (build "
                                     "the functor against the same ceres-solver-cuda_amd headers)");
  const bool fused = ops->fused_points[0] || ops->fused_points[1] || ops->camera_gradient;
  if (fused && (!ops->fused_points[0] || !ops->fused_points[1] || !ops->camera_gradient ||
                ops->camera_gradient_args_size != (int32_t)sizeof(cse::CamGradArgs)))
    return Fail(CSE_ERR_INVALID, "functor " + name +
                                     ": the fused gradient's launches come as all three, with the "
                                     "library's camera-gradient argument size");
  const int nb = ops->num_parameter_blocks;
  if (ops->num_residuals < 1 || nb < 1 || nb > CSE_MAX_PARAMETER_BLOCKS || ops->data_size < 1)
    return Fail(CSE_ERR_INVALID, "functor " + name + ": bad shape");
  for (int j = 0; j < nb; ++j)
    if (ops->parameter_block_sizes[j] < 1)
      return Fail(CSE_ERR_INVALID, "functor " + name + ": parameter block size < 1");
  if (ops->loss_kind < CSE_LOSS_TRIVIAL || ops->loss_kind > CSE_LOSS_USER ||
      (ops->loss_kind == CSE_LOSS_USER &&
       (ops->loss_size < 1 || ops->loss_size > CSE_USER_LOSS_BYTES)))
    return Fail(CSE_ERR_INVALID, "functor " + name + ": bad loss kind or size");
  if (!ops->table[0] || !ops->table[1])
    return Fail(CSE_ERR_INVALID, "functor " + name + ": the general kernels are required");
  bool any_affine = false;
  for (int c = 0; c < 2; ++c)
    for (int j = 0; j < 2; ++j)
      for (int d = 0; d < 2; ++d) any_affine = any_affine || ops->affine[c][j][d];
  if (any_affine && (!UserAffine(ops) || nb > 2 || ops->num_residuals > 3))
    return Fail(CSE_ERR_INVALID, "functor " + name + ": affine kernels must come as all eight, "
                                                     "for at most two blocks and three residuals");
  if (fused && (!any_affine || nb != 2 || ops->parameter_block_sizes[1] != 3 ||
                ops->parameter_block_sizes[0] > 16))
    return Fail(CSE_ERR_INVALID, "functor " + name + ": the fused gradient is for affine kinds of two "
                                                     "blocks, the second of 3 parameters");
  std::lock_guard<std::mutex> lock(g_user_mu);
  for (size_t i = 0; i < g_user_kinds.size(); ++i) {
    const UserKindEntry& e = *g_user_kinds[i];
    cse_functor_ops a = e.ops, b = *ops;
    a.name = b.name = nullptr;
    if (e.name == name && std::memcmp(&a, &b, sizeof(a)) == 0) {
      *kind = CSE_FUNCTOR_USER_FIRST + (int32_t)i;
      return CSE_OK;
    }
  }
  UserKindEntry* e = new (std::nothrow) UserKindEntry{*ops, name};
  if (!e) return Fail(CSE_ERR_OOM, "host allocation failed");
  e->ops.name = nullptr;  // the copy in e->name serves
  g_user_kinds.push_back(e);
  *kind = CSE_FUNCTOR_USER_FIRST + (int32_t)(g_user_kinds.size() - 1);
  return CSE_OK;
}

int cse_functor_shape(int32_t kind, int32_t* num_residuals, int32_t* num_parameter_blocks,
                      int32_t* parameter_block_sizes, int32_t* data_size) {
  KindShape k;
  if (!ShapeOf(kind, &k)) return Fail(CSE_ERR_UNSUPPORTED, "unknown functor kind " + std::to_string(kind));
  if (num_residuals) *num_residuals = k.nr;
  if (num_parameter_blocks) *num_parameter_blocks = k.nb;
  if (parameter_block_sizes)
    for (int j = 0; j < k.nb; ++j) parameter_block_sizes[j] = k.sz[j];
  if (data_size) *data_size = k.data;
  return CSE_OK;
}

int cse_get_info(cse_evaluator* ev, cse_info* info) {
  if (!ev || !info) return Fail(CSE_ERR_INVALID, "null argument");
  if (ev->multi) return MultiInfo(ev->multi, info);
  std::memset(info, 0, sizeof(*info));
  info->num_residual_blocks = ev->num_residual_blocks;
  info->num_residuals = ev->num_residuals;
  info->num_parameters = ev->num_parameters;
  info->num_effective_parameters = ev->num_effective;
  info->num_jacobian_values = ev->num_jacobian_values;
  info->num_groups = (int32_t)ev->groups.size();
  for (auto& G : ev->groups) {
    info->num_affine_groups += G.affine ? 1 : 0;
    info->num_fused_gradient_groups +=
        (G.fuse_ok && (ev->opts.gradient_mode == 0 ||
                       (!G.user && ((ev->opts.gradient_mode == 3 && !G.jet) ||
                                    (ev->opts.gradient_mode == 1 && G.const0)))))
            ? 1
            : 0;
  }
  info->device = ev->device;
  info->bytes_jacobian_eval = ev->bytes_jac;
  info->bytes_residual_eval = ev->bytes_res;
  return CSE_OK;
}

int cse_kernel_stats(cse_evaluator* ev, double* last_ms, double* total_ms, int64_t* launches) {
  if (!ev) return Fail(CSE_ERR_INVALID, "null evaluator");
  if (ev->multi) return MultiKernelStats(ev->multi, last_ms, total_ms, launches);
  if (!ev->opts.profile) return Fail(CSE_ERR_INVALID, "evaluator created without options.profile");
  int rc = FoldTiming(ev);
  if (rc) return rc;
  if (last_ms) *last_ms = ev->last_ms;
  if (total_ms) *total_ms = ev->total_ms;
  if (launches) *launches = ev->launches;
  return CSE_OK;
}

int cse_reset_kernel_stats(cse_evaluator* ev) {
  if (!ev) return Fail(CSE_ERR_INVALID, "null evaluator");
  if (ev->multi) return MultiResetKernelStats(ev->multi);
  int rc = FoldTiming(ev);
  if (rc) return rc;
  ev->last_ms = ev->total_ms = 0.0;
  ev->launches = 0;
  return CSE_OK;
}

}  // extern "C"
