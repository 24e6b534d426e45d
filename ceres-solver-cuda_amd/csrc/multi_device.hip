// multi_device.hip -- the single-process multi-device evaluator
// (cse_create_multi), host code only.  See multi_device.h.
//
// Sharding.  Residual blocks are independent, so the
// Program's blocks are cut into num_devices contiguous ranges of the global
// residual-block index, each cut moved forward to the next "bucket"
// boundary: a block whose bucket key (its last parameter block: the point of
// a Schur-ordered BAL problem) differs from the previous block's, and then
// on to a multiple of 4 blocks when one is found before the next range's
// target (the rank-local BlockSparseMatrix F cells then start on a 64-byte
// sector).  This is ceres_amd.shard.point_bucket_cuts
// restated for any descriptor.  Every cut is correct -- a parameter block
// shared by two shards simply gets gradient rows from both, and the host sums
// them -- the bucket cuts only keep each point's rows in one shard.
//
// Each shard becomes an ordinary evaluator (cse_create) of a sub-descriptor:
// the shard's blocks renumbered from 0, only the parameter blocks they use
// (renumbered in id order: every camera the shard sees plus its own points,
// SURVEY.md §8(e)), and the state, delta, residual and Jacobian-value offsets
// of those mapped onto compact local ranges.  Each local range is the union of
// the global offsets involved, kept as a list of global intervals (a
// Schur-ordered BlockSparse shard: its point slice and its cameras for the
// state, its E strip and its F strip for the values; CompressedRow: one), so
// one Evaluate moves every interval with one copy at its global position: the
// state slices host-to-device, the strips device-to-host.  Renumbering in id
// order and compacting in offset order keep an affine layout affine (a
// shard's points and cameras stay on the fast kernels).  Cost and gradient:
// per shard on its device, then summed over the shards in shard order
// (deterministic).  Parameter blocks no residual block uses go to shard 0, so
// Plus covers every active block.
//
// Host buffers.  Asynchronous copies need page-locked memory.  The caller
// pins a buffer explicitly (cse_host_register, or its own hipHostMalloc);
// the library never pins or caches a caller buffer by address (a freed
// buffer's address can be reused by the next allocation).  A buffer that is
// not pinned is copied synchronously.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "multi_device.h"

namespace {

#define MD_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess)                                                              \
      return CseFail(CSE_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

// A global range [begin, end) of an output array and its position in the
// shard's compact local array.
struct Interval {
  int64_t begin, end, local;
};

// Unions ranges that arrive as a few interleaved ascending streams (the rows
// of a block's cells in program order): each range first tries to extend one
// of the recently extended intervals.
class IntervalBuilder {
 public:
  void Add(int64_t b, int64_t e) {
    if (e <= b) return;
    for (size_t h = 0; h < hot_.size(); ++h) {
      auto& iv = ivs_[hot_[h]];
      if (iv.second == b) {
        iv.second = e;
        return;
      }
    }
    ivs_.push_back({b, e});
    if (hot_.size() < 8) hot_.push_back(ivs_.size() - 1);
    else hot_[next_++ % 8] = ivs_.size() - 1;
  }
  // Sorted, merged, with local positions; returns the local size.
  int64_t Finish(std::vector<Interval>* out) {
    std::sort(ivs_.begin(), ivs_.end());
    out->clear();
    for (const auto& iv : ivs_) {
      if (!out->empty() && iv.first <= out->back().end) {
        out->back().end = std::max(out->back().end, iv.second);
      } else {
        out->push_back({iv.first, iv.second, 0});
      }
    }
    int64_t local = 0;
    for (auto& iv : *out) {
      iv.local = local;
      local += iv.end - iv.begin;
    }
    return local;
  }

 private:
  std::vector<std::pair<int64_t, int64_t>> ivs_;
  std::vector<size_t> hot_;
  size_t next_ = 0;
};

// Local position of global offset g (g inside one of the intervals).
int64_t LocalOf(const std::vector<Interval>& ivs, int64_t g) {
  auto it = std::upper_bound(ivs.begin(), ivs.end(), g,
                             [](int64_t v, const Interval& iv) { return v < iv.begin; });
  const Interval& iv = *(it - 1);
  return iv.local + (g - iv.begin);
}

struct Shape {
  int nr = 0, nb = 0, data = 0;
};

}  // namespace

struct CseMulti {
  struct Shard {
    int device = 0;
    cse_evaluator* ev = nullptr;
    hipStream_t stream = nullptr;
    int64_t g0 = 0, g1 = 0;
    // Global -> local intervals: state (active parameter blocks the shard
    // uses), delta (their tangent columns: the gradient rows), residuals and
    // Jacobian values (the strips).
    std::vector<Interval> state_iv, res_iv, jac_iv, grad_iv;
    int64_t nstate = 0, nres = 0, njac = 0, ngrad = 0;
    // The plus-Jacobian values of the shard's parameter blocks, compacted
    // (global -> local intervals of the caller's plus_jacobians array).
    std::vector<Interval> pj_iv;
    int64_t npj = 0;
    // Pinned staging of the shard's state slices (allocated on first use):
    // one H2D copy per evaluation however many intervals the slices form.
    double* h_state = nullptr;
    double *d_state = nullptr, *d_cost = nullptr, *d_res = nullptr, *d_jac = nullptr,
           *d_grad = nullptr;
    double *h_cost = nullptr, *h_grad = nullptr;  // pinned
    // Plus staging (pinned, allocated on first use): local state, delta, result.
    double *h_x = nullptr, *h_d = nullptr, *h_o = nullptr;
  };
  std::vector<Shard> shards;
  int64_t num_parameters = 0, num_effective = 0, num_residuals = 0, num_jacobian_values = 0;
  int64_t num_residual_blocks = 0;
  bool has_layout = false;
  // Every shard's d_state holds the state of the last evaluation queued
  // without error (CSE_EVAL_SAME_POINT skips the copies).
  bool state_current = false;
};

namespace {

void ReleaseShard(CseMulti::Shard& s) {
  if (s.ev) cse_destroy(s.ev);
  s.ev = nullptr;
  (void)hipSetDevice(s.device);
  for (double* p : {s.d_state, s.d_cost, s.d_res, s.d_jac, s.d_grad})
    if (p) (void)hipFree(p);
  for (double* p : {s.h_cost, s.h_grad, s.h_x, s.h_d, s.h_o, s.h_state})
    if (p) (void)hipHostFree(p);
  if (s.stream) (void)hipStreamDestroy(s.stream);
  s = CseMulti::Shard{};
}

// Ranges page-locked through cse_host_register (library-wide).
std::mutex g_reg_mu;
std::vector<std::pair<uintptr_t, uintptr_t>> g_reg;  // [begin, end)

// Is host memory at p page-locked by the HIP runtime (hipHostMalloc or
// hipHostRegister, the caller's own)?
bool RuntimePinned(const void* p) {
  hipPointerAttribute_t at;
  const hipError_t e = hipPointerGetAttributes(&at, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return at.type == hipMemoryTypeHost;
}

// May [p, p + bytes) take asynchronous copies?  Inside one cse_host_register
// range, or inside ONE page-locked allocation of the caller's (hipHostMalloc
// or hipHostRegister): the runtime's address range of p must cover the
// whole buffer (a range over two pinned allocations with pageable memory
// between them is not pinned).
bool Pinned(const void* p, size_t bytes) {
  if (!p || bytes == 0) return false;
  const uintptr_t b = reinterpret_cast<uintptr_t>(p), e = b + bytes;
  {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    for (const auto& r : g_reg)
      if (b >= r.first && e <= r.second) return true;
  }
  if (!RuntimePinned(p)) return false;
  void* start = nullptr;
  size_t size = 0;
  if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR,
                             reinterpret_cast<hipDeviceptr_t>(const_cast<void*>(p))) != hipSuccess ||
      hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE,
                             reinterpret_cast<hipDeviceptr_t>(const_cast<void*>(p))) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  const uintptr_t rb = reinterpret_cast<uintptr_t>(start);
  return rb <= b && e <= rb + size;
}

// Cut positions in the global residual-block index (module comment).
std::vector<int64_t> BucketCuts(const std::vector<int64_t>& key, int n) {
  const int64_t nrb = (int64_t)key.size();
  std::vector<int64_t> cuts{0};
  for (int r = 1; r < n; ++r) {
    const int64_t target = nrb * r / n, next_target = nrb * (r + 1) / n;
    int64_t g = std::max(target, cuts.back());
    while (g < nrb && g > 0 && key[g] == key[g - 1]) ++g;
    // On to a multiple of 4 at a later boundary before the next target.
    int64_t h = g;
    for (int tries = 0; h < nrb && h % 4 != 0 && tries < 64; ++tries) {
      ++h;
      while (h < nrb && key[h] == key[h - 1]) ++h;
    }
    if (h % 4 == 0 && h < next_target) g = h;
    cuts.push_back(std::min(g, nrb));
  }
  cuts.push_back(nrb);
  return cuts;
}

// Sorted, merged intervals of [begin, end) ranges given in any order.
int64_t IntervalsOf(std::vector<std::pair<int64_t, int64_t>>& ranges, std::vector<Interval>* out) {
  std::sort(ranges.begin(), ranges.end());
  IntervalBuilder ib;
  for (const auto& r : ranges) ib.Add(r.first, r.second);
  return ib.Finish(out);
}

// The sub-descriptor of shard [g0, g1) and its evaluator.  used: the
// parameter blocks the shard's residual blocks use (shard 0 also gets the
// blocks no residual block uses).
int CreateShard(const cse_problem_desc* d, const cse_options* opts, CseMulti::Shard& s,
                const std::vector<Shape>& shapes, const std::vector<char>& used) {
  const int64_t g0 = s.g0, g1 = s.g1, nloc = g1 - g0;
  const bool has_layout = d->jacobian_per_residual_layout && d->jacobian_per_residual_offsets;
  // Shard-local parameter blocks: the used ones, renumbered in id order; the
  // active ones' state and delta ranges compacted in offset order.
  std::vector<int32_t> lid(d->num_parameter_blocks, -1);
  std::vector<cse_parameter_block> pbs;
  {
    std::vector<std::pair<int64_t, int64_t>> st, dl;
    for (int64_t b = 0; b < d->num_parameter_blocks; ++b) {
      if (!used[b]) continue;
      lid[b] = (int32_t)pbs.size();
      const cse_parameter_block& pb = d->parameter_blocks[b];
      pbs.push_back(pb);
      if (pb.is_constant) continue;
      st.push_back({pb.state_offset, pb.state_offset + pb.size});
      if (pb.tangent_size > 0) dl.push_back({pb.delta_offset, pb.delta_offset + pb.tangent_size});
    }
    s.nstate = IntervalsOf(st, &s.state_iv);
    s.ngrad = IntervalsOf(dl, &s.grad_iv);
    std::vector<std::pair<int64_t, int64_t>> pj;
    for (const auto& pb : pbs)
      if (pb.plus_jacobian_offset >= 0)
        pj.push_back({pb.plus_jacobian_offset,
                      pb.plus_jacobian_offset + (int64_t)pb.size * pb.tangent_size});
    s.npj = IntervalsOf(pj, &s.pj_iv);
    for (auto& pb : pbs) {
      if (pb.plus_jacobian_offset >= 0) pb.plus_jacobian_offset = LocalOf(s.pj_iv, pb.plus_jacobian_offset);
      if (pb.is_constant) continue;  // offsets into the (whole) constant state
      pb.state_offset = LocalOf(s.state_iv, pb.state_offset);
      if (pb.tangent_size > 0) pb.delta_offset = LocalOf(s.grad_iv, pb.delta_offset);
    }
  }
  // The shard's plus-Jacobian values only (cse_set_plus_jacobians refreshes
  // them through the same intervals).
  std::vector<double> pj_local;
  if (s.npj > 0 && d->plus_jacobians) {
    pj_local.resize((size_t)s.npj);
    for (const auto& iv : s.pj_iv)
      std::copy(d->plus_jacobians + iv.begin, d->plus_jacobians + iv.end, pj_local.begin() + iv.local);
  }
  // Groups restricted to the shard, renumbered from g0, ids mapped to the
  // shard's parameter blocks.
  std::vector<cse_residual_group> groups;
  std::vector<std::vector<int64_t>> idx_store;
  std::vector<std::vector<int32_t>> ids_store;
  std::vector<std::vector<double>> data_store;
  // Per local block: its group and index (for the layout passes).
  std::vector<int32_t> gr_of(nloc, -1);
  std::vector<int64_t> i_of(nloc, -1);
  for (int gi = 0; gi < d->num_groups; ++gi) {
    const cse_residual_group& g = d->groups[gi];
    const Shape& k = shapes[gi];
    const int ds = k.data;
    cse_residual_group sg = g;
    ids_store.emplace_back();
    auto& id = ids_store.back();
    if (!g.residual_block_index) {
      const int64_t lo = std::clamp<int64_t>(g0 - g.first_residual_block, 0, g.num_blocks);
      const int64_t hi = std::clamp<int64_t>(g1 - g.first_residual_block, 0, g.num_blocks);
      sg.num_blocks = hi - lo;
      sg.first_residual_block = g.first_residual_block + lo - g0;
      id.resize((size_t)((hi - lo) * k.nb));
      for (int64_t q = 0; q < (hi - lo) * k.nb; ++q) id[q] = lid[g.parameter_block_ids[k.nb * lo + q]];
      sg.functor_data = g.functor_data ? g.functor_data + (int64_t)ds * lo : nullptr;
      for (int64_t i = lo; i < hi; ++i) {
        gr_of[g.first_residual_block + i - g0] = gi;
        i_of[g.first_residual_block + i - g0] = i;
      }
    } else {
      idx_store.emplace_back();
      data_store.emplace_back();
      auto& ix = idx_store.back();
      auto& dt = data_store.back();
      for (int64_t i = 0; i < g.num_blocks; ++i) {
        const int64_t gg = g.residual_block_index[i];
        if (gg < g0 || gg >= g1) continue;
        ix.push_back(gg - g0);
        for (int j = 0; j < k.nb; ++j) id.push_back(lid[g.parameter_block_ids[(int64_t)k.nb * i + j]]);
        dt.insert(dt.end(), g.functor_data + (int64_t)ds * i, g.functor_data + (int64_t)ds * (i + 1));
        gr_of[gg - g0] = gi;
        i_of[gg - g0] = i;
      }
      sg.num_blocks = (int64_t)ix.size();
      sg.residual_block_index = ix.data();
      sg.first_residual_block = 0;
      sg.functor_data = dt.data();
    }
    sg.parameter_block_ids = id.data();
    groups.push_back(sg);
  }
  // Residual and Jacobian-value intervals of the shard.
  IntervalBuilder rb, jb;
  for (int64_t l = 0; l < nloc; ++l) {
    const int gi = gr_of[l];
    if (gi < 0) continue;
    const Shape& k = shapes[gi];
    const cse_residual_group& g = d->groups[gi];
    const int64_t gg = g0 + l;
    // The same checks as cse_create's: every range this shard hands back
    // must lie inside the caller's buffers.
    if (d->residual_layout[gg] < 0 || d->residual_layout[gg] + k.nr > d->num_residuals)
      return CseFail(CSE_ERR_INVALID, "residual_layout out of range");
    rb.Add(d->residual_layout[gg], d->residual_layout[gg] + k.nr);
    int a = 0;
    for (int j = 0; j < k.nb; ++j) {
      const int32_t pid = g.parameter_block_ids[(int64_t)k.nb * i_of[l] + j];
      const cse_parameter_block& pb = d->parameter_blocks[pid];
      if (pb.is_constant || !has_layout) continue;
      const int64_t base = d->jacobian_per_residual_layout[gg] + (int64_t)a * k.nr;
      if (base < 0 || base + k.nr > d->num_jacobian_per_residual_offsets)
        return CseFail(CSE_ERR_INVALID, "jacobian_per_residual_layout out of range");
      for (int r = 0; r < k.nr; ++r) {
        const int64_t off = d->jacobian_per_residual_offsets[base + r];
        if (off < 0 || off + pb.tangent_size > d->num_jacobian_values)
          return CseFail(CSE_ERR_INVALID, "jacobian offset out of range");
        jb.Add(off, off + pb.tangent_size);
      }
      ++a;
    }
  }
  s.nres = rb.Finish(&s.res_iv);
  s.njac = jb.Finish(&s.jac_iv);
  // Local layouts.
  std::vector<int64_t> res_layout(std::max<int64_t>(nloc, 1), 0), jac_layout, jac_offsets;
  if (has_layout) jac_layout.assign(std::max<int64_t>(nloc, 1), 0);
  for (int64_t l = 0; l < nloc; ++l) {
    const int gi = gr_of[l];
    if (gi < 0) continue;
    const Shape& k = shapes[gi];
    const cse_residual_group& g = d->groups[gi];
    const int64_t gg = g0 + l;
    res_layout[l] = LocalOf(s.res_iv, d->residual_layout[gg]);
    if (!has_layout) continue;
    jac_layout[l] = (int64_t)jac_offsets.size();
    int a = 0;
    for (int j = 0; j < k.nb; ++j) {
      const int32_t pid = g.parameter_block_ids[(int64_t)k.nb * i_of[l] + j];
      if (d->parameter_blocks[pid].is_constant) continue;
      const int64_t base = d->jacobian_per_residual_layout[gg] + (int64_t)a * k.nr;
      for (int r = 0; r < k.nr; ++r)
        jac_offsets.push_back(LocalOf(s.jac_iv, d->jacobian_per_residual_offsets[base + r]));
      ++a;
    }
  }
  cse_problem_desc sd = *d;
  sd.num_groups = (int32_t)groups.size();
  sd.groups = groups.data();
  sd.num_parameter_blocks = (int64_t)pbs.size();
  sd.parameter_blocks = pbs.data();
  sd.num_parameters = s.nstate;
  sd.num_effective_parameters = s.ngrad;
  sd.num_residual_blocks = nloc;
  sd.num_residuals = s.nres;
  sd.residual_layout = res_layout.data();
  sd.jacobian_per_residual_layout = has_layout ? jac_layout.data() : nullptr;
  sd.jacobian_per_residual_offsets = has_layout ? (jac_offsets.empty() ? jac_layout.data()
                                                                        : jac_offsets.data())
                                                : nullptr;
  sd.num_jacobian_per_residual_offsets = (int64_t)jac_offsets.size();
  sd.num_jacobian_values = s.njac;
  sd.num_plus_jacobian_values = s.npj;
  sd.plus_jacobians = s.npj > 0 ? pj_local.data() : nullptr;
  // Device, stream, buffers, then the shard's evaluator on that stream.
  MD_HIP(hipSetDevice(s.device));
  MD_HIP(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
  cse_options so = *opts;
  so.device = s.device;
  so.use_stream = 1;
  so.stream = s.stream;
  int rc = cse_create(&sd, &so, &s.ev);
  if (rc) return rc;
  auto dalloc = [&](double** p, int64_t n) -> hipError_t {
    return hipMalloc(reinterpret_cast<void**>(p), std::max<int64_t>(n, 1) * sizeof(double));
  };
  if (dalloc(&s.d_state, s.nstate) != hipSuccess || dalloc(&s.d_cost, 1) != hipSuccess ||
      dalloc(&s.d_res, s.nres) != hipSuccess || dalloc(&s.d_jac, has_layout ? s.njac : 0) != hipSuccess ||
      dalloc(&s.d_grad, s.ngrad) != hipSuccess)
    return CseFail(CSE_ERR_OOM, "multi-device: device allocation failed on device " +
                                    std::to_string(s.device));
  MD_HIP(hipHostMalloc(reinterpret_cast<void**>(&s.h_cost), sizeof(double)));
  MD_HIP(hipHostMalloc(reinterpret_cast<void**>(&s.h_grad),
                       std::max<int64_t>(s.ngrad, 1) * sizeof(double)));
  return CSE_OK;
}

}  // namespace

int MultiCreate(const cse_problem_desc* d, const cse_options* options, const int32_t* devices,
                int32_t n, CseMulti** out) {
  *out = nullptr;
  if (n <= 0 || !devices) return CseFail(CSE_ERR_INVALID, "cse_create_multi: no devices");
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
    return CseFail(CSE_ERR_HIP, "cse_create_multi: no HIP device");
  for (int k = 0; k < n; ++k)
    if (devices[k] < 0 || devices[k] >= count)
      return CseFail(CSE_ERR_INVALID, "cse_create_multi: device " + std::to_string(devices[k]) +
                                          " out of range (" + std::to_string(count) + " visible)");
  cse_options opts;
  if (options) opts = *options; else cse_default_options(&opts);
  if (opts.use_stream || opts.stream)
    return CseFail(CSE_ERR_INVALID, "cse_create_multi: streams are per device (use_stream must be 0)");
  std::vector<Shape> shapes(d->num_groups);
  // Bucket key per global residual block: its last parameter block.
  std::vector<int64_t> key(d->num_residual_blocks);
  for (int64_t g = 0; g < d->num_residual_blocks; ++g) key[g] = -1 - g;
  for (int gi = 0; gi < d->num_groups; ++gi) {
    const cse_residual_group& g = d->groups[gi];
    if (!CseKindShape(g.functor_kind, &shapes[gi].nr, &shapes[gi].nb, &shapes[gi].data))
      return CseFail(CSE_ERR_UNSUPPORTED, "unknown functor kind " + std::to_string(g.functor_kind));
    const int nb = shapes[gi].nb;
    for (int64_t i = 0; i < g.num_blocks; ++i) {
      const int64_t gg = g.residual_block_index ? g.residual_block_index[i] : g.first_residual_block + i;
      if (gg < 0 || gg >= d->num_residual_blocks)
        return CseFail(CSE_ERR_INVALID, "residual block index out of range");
      if (!g.parameter_block_ids)
        return CseFail(CSE_ERR_INVALID, "group " + std::to_string(gi) + " arrays missing");
      key[gg] = g.parameter_block_ids[(int64_t)nb * i + nb - 1];
    }
  }
  CseMulti* m = new (std::nothrow) CseMulti();
  if (!m) return CseFail(CSE_ERR_OOM, "host allocation failed");
  m->num_parameters = d->num_parameters;
  m->num_effective = d->num_effective_parameters;
  m->num_residuals = d->num_residuals;
  m->num_jacobian_values = d->num_jacobian_values;
  m->num_residual_blocks = d->num_residual_blocks;
  m->has_layout = d->jacobian_per_residual_layout && d->jacobian_per_residual_offsets;
  const std::vector<int64_t> cuts = BucketCuts(key, n);
  key.clear();
  key.shrink_to_fit();
  // Parameter blocks used by each shard (checked ids); shard 0 also takes
  // the blocks no residual block uses.
  std::vector<std::vector<char>> used(n, std::vector<char>(d->num_parameter_blocks, 0));
  std::vector<char> any(d->num_parameter_blocks, 0);
  for (int gi = 0; gi < d->num_groups; ++gi) {
    const cse_residual_group& g = d->groups[gi];
    const int nb = shapes[gi].nb;
    for (int64_t i = 0; i < g.num_blocks; ++i) {
      const int64_t gg = g.residual_block_index ? g.residual_block_index[i] : g.first_residual_block + i;
      const int k = (int)(std::upper_bound(cuts.begin(), cuts.end(), gg) - cuts.begin()) - 1;
      for (int j = 0; j < nb; ++j) {
        const int32_t pid = g.parameter_block_ids[(int64_t)nb * i + j];
        if (pid < 0 || pid >= d->num_parameter_blocks) {
          delete m;
          return CseFail(CSE_ERR_INVALID, "parameter block id out of range");
        }
        used[k][pid] = 1;
        any[pid] = 1;
      }
    }
  }
  for (int64_t b = 0; b < d->num_parameter_blocks; ++b)
    if (!any[b]) used[0][b] = 1;
  any.clear();
  any.shrink_to_fit();
  m->shards.resize(n);
  for (int k = 0; k < n; ++k) {
    m->shards[k].device = devices[k];
    m->shards[k].g0 = cuts[k];
    m->shards[k].g1 = cuts[k + 1];
    const int rc = CreateShard(d, &opts, m->shards[k], shapes, used[k]);
    std::vector<char>().swap(used[k]);
    if (rc) {
      MultiDestroy(m);
      return rc;
    }
  }
  *out = m;
  return CSE_OK;
}

void MultiDestroy(CseMulti* m) {
  if (!m) return;
  for (auto& s : m->shards) ReleaseShard(s);
  delete m;
}

namespace {

// Synchronises the streams of shards [0, upto): the copies queued on them
// read or write the caller's buffers, which must not be returned to the
// caller (and freed) while in flight.
void Drain(CseMulti* m, size_t upto) {
  for (size_t k = 0; k < upto && k < m->shards.size(); ++k) {
    auto& s = m->shards[k];
    if (!s.stream) continue;
    (void)hipSetDevice(s.device);
    (void)hipStreamSynchronize(s.stream);
  }
}

}  // namespace

// A page-locked caller state is copied slice by slice while it has at most
// this many slices; beyond, through the shard's staging in one copy.
constexpr size_t kDirectStateIntervals = 8;

int MultiEvaluate(CseMulti* m, const double* state, double* cost, double* residuals,
                  double* gradient, double* jac, bool same_point) {
  if (jac && !m->has_layout)
    return CseFail(CSE_ERR_INVALID, "Jacobian requested but the descriptor had no Jacobian layout");
  const bool async_state = Pinned(state, m->num_parameters * sizeof(double));
  const bool async_res = residuals && Pinned(residuals, m->num_residuals * sizeof(double));
  const bool async_jac = jac && Pinned(jac, m->num_jacobian_values * sizeof(double));
  // Queue every shard: its state slices H2D, evaluation, strips D2H (disjoint
  // regions of the caller's buffers), gradient rows and cost into pinned
  // staging.  Any error drains the shards queued so far before returning.
  const bool copy_state = !(same_point && m->state_current);
  m->state_current = false;
  size_t queued = 0;
#define MD_Q(call)                                                                         do {                                                                                       hipError_t e_ = (call);                                                                  if (e_ != hipSuccess) {                                                                    Drain(m, queued + 1);                                                                    return CseFail(CSE_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_));        }                                                                                      } while (0)
  for (auto& s : m->shards) {
    MD_Q(hipSetDevice(s.device));
    if (copy_state && s.nstate > 0) {
      if (async_state && s.state_iv.size() <= kDirectStateIntervals) {
        for (const auto& iv : s.state_iv)
          MD_Q(hipMemcpyAsync(s.d_state + iv.local, state + iv.begin, (iv.end - iv.begin) * sizeof(double),
                              hipMemcpyHostToDevice, s.stream));
      } else {
        // Many slices (a BAL shard's cameras), or pageable state: gathered on
        // the host into the shard's pinned staging, then one copy.  The
        // staging is free again: the previous call waited for every shard.
        if (!s.h_state)
          MD_Q(hipHostMalloc(reinterpret_cast<void**>(&s.h_state), s.nstate * sizeof(double)));
        for (const auto& iv : s.state_iv)
          std::memcpy(s.h_state + iv.local, state + iv.begin, (iv.end - iv.begin) * sizeof(double));
        MD_Q(hipMemcpyAsync(s.d_state, s.h_state, s.nstate * sizeof(double), hipMemcpyHostToDevice,
                            s.stream));
      }
    }
    int rc = cse_evaluate_device_ex(s.ev, s.d_state, s.d_cost, residuals ? s.d_res : nullptr,
                                    gradient ? s.d_grad : nullptr, jac ? s.d_jac : nullptr,
                                    same_point ? CSE_EVAL_SAME_POINT : 0u);
    if (rc) {
      Drain(m, queued + 1);
      return rc;
    }
    MD_Q(hipMemcpyAsync(s.h_cost, s.d_cost, sizeof(double), hipMemcpyDeviceToHost, s.stream));
    if (residuals && async_res)
      for (const auto& iv : s.res_iv)
        MD_Q(hipMemcpyAsync(residuals + iv.begin, s.d_res + iv.local,
                            (iv.end - iv.begin) * sizeof(double), hipMemcpyDeviceToHost, s.stream));
    if (jac && async_jac)
      for (const auto& iv : s.jac_iv)
        MD_Q(hipMemcpyAsync(jac + iv.begin, s.d_jac + iv.local, (iv.end - iv.begin) * sizeof(double),
                            hipMemcpyDeviceToHost, s.stream));
    if (gradient && s.ngrad > 0)
      MD_Q(hipMemcpyAsync(s.h_grad, s.d_grad, s.ngrad * sizeof(double), hipMemcpyDeviceToHost,
                          s.stream));
    ++queued;
  }
  m->state_current = true;
  // Wait for every shard (cse_wait synchronises the shard's stream, which
  // carries the copies too) and collect the statuses; every shard is waited
  // for even after an error.
  int status = CSE_OK, err = CSE_OK;
  for (auto& s : m->shards) {
    if (hipSetDevice(s.device) != hipSuccess) {
      if (!err) err = CseFail(CSE_ERR_HIP, "hipSetDevice failed");
      continue;
    }
    const int rc = cse_wait(s.ev);
    if (rc < 0) {
      if (!err) err = rc;
      (void)hipStreamSynchronize(s.stream);
      continue;
    }
    if (rc == CSE_EVALUATION_FAILED) status = rc;
    if (err) continue;
    // Caller buffers that are not page-locked: synchronous copies now.
    if (residuals && !async_res)
      for (const auto& iv : s.res_iv)
        if (hipMemcpy(residuals + iv.begin, s.d_res + iv.local, (iv.end - iv.begin) * sizeof(double),
                      hipMemcpyDeviceToHost) != hipSuccess && !err)
          err = CseFail(CSE_ERR_HIP, "hipMemcpy (residual strip) failed");
    if (jac && !async_jac)
      for (const auto& iv : s.jac_iv)
        if (hipMemcpy(jac + iv.begin, s.d_jac + iv.local, (iv.end - iv.begin) * sizeof(double),
                      hipMemcpyDeviceToHost) != hipSuccess && !err)
          err = CseFail(CSE_ERR_HIP, "hipMemcpy (Jacobian strip) failed");
  }
#undef MD_Q
  if (err) {
    m->state_current = false;
    return err;
  }
  if (status != CSE_OK) return status;
  // Cost and gradient: sums over the shards in shard order.
  double c = 0.0;
  for (auto& s : m->shards) c += *s.h_cost;
  *cost = c;
  if (gradient) {
    std::memset(gradient, 0, m->num_effective * sizeof(double));
    for (auto& s : m->shards)
      for (const auto& iv : s.grad_iv) {
        const double* src = s.h_grad + iv.local;
        double* dst = gradient + iv.begin;
        for (int64_t t = 0, len = iv.end - iv.begin; t < len; ++t) dst[t] += src[t];
      }
  }
  return CSE_OK;
}

int MultiInfo(CseMulti* m, cse_info* info) {
  std::memset(info, 0, sizeof(*info));
  bool first = true;
  for (auto& s : m->shards) {
    cse_info si;
    const int rc = cse_get_info(s.ev, &si);
    if (rc) return rc;
    if (first) {
      info->num_groups = si.num_groups;
      info->num_affine_groups = si.num_affine_groups;
      info->num_fused_gradient_groups = si.num_fused_gradient_groups;
      info->device = si.device;
      first = false;
    } else {
      info->num_affine_groups = std::min(info->num_affine_groups, si.num_affine_groups);
      info->num_fused_gradient_groups =
          std::min(info->num_fused_gradient_groups, si.num_fused_gradient_groups);
    }
    info->bytes_jacobian_eval += si.bytes_jacobian_eval;
    info->bytes_residual_eval += si.bytes_residual_eval;
  }
  info->num_residual_blocks = m->num_residual_blocks;
  info->num_residuals = m->num_residuals;
  info->num_parameters = m->num_parameters;
  info->num_effective_parameters = m->num_effective;
  info->num_jacobian_values = m->num_jacobian_values;
  return CSE_OK;
}

int MultiShardInfo(CseMulti* m, int32_t* num_shards, int64_t* first_block, int32_t* devices) {
  const int n = (int)m->shards.size();
  if (num_shards) *num_shards = n;
  if (first_block) {
    for (int k = 0; k < n; ++k) first_block[k] = m->shards[k].g0;
    first_block[n] = m->num_residual_blocks;
  }
  if (devices)
    for (int k = 0; k < n; ++k) devices[k] = m->shards[k].device;
  return CSE_OK;
}

int MultiSetPlusJacobians(CseMulti* m, const double* pj) {
  std::vector<double> local;
  for (auto& s : m->shards) {
    if (s.npj == 0) continue;
    if (!pj) return CseFail(CSE_ERR_INVALID, "null plus_jacobians");
    local.resize((size_t)s.npj);
    for (const auto& iv : s.pj_iv) std::copy(pj + iv.begin, pj + iv.end, local.begin() + iv.local);
    const int rc = cse_set_plus_jacobians(s.ev, local.data());
    if (rc) return rc;
  }
  return CSE_OK;
}

int MultiPlus(CseMulti* m, const double* state, const double* delta, double* out) {
  // Each shard applies Plus to the parameter blocks it holds (a camera seen
  // by several shards gets the same result from each); every active block
  // belongs to some shard (MultiCreate).  Local slices through pinned
  // staging, the shard's own cse_plus in between.
  // Every shard's inputs are gathered before any output is written, so `out`
  // may alias `state` (in-place Plus, as Program::Plus allows): a camera
  // held by two shards is read once, before either writes it.
  for (auto& s : m->shards) {
    if (s.nstate == 0) continue;
    MD_HIP(hipSetDevice(s.device));
    if (!s.h_x) MD_HIP(hipHostMalloc(reinterpret_cast<void**>(&s.h_x), s.nstate * sizeof(double)));
    if (!s.h_d)
      MD_HIP(hipHostMalloc(reinterpret_cast<void**>(&s.h_d), std::max<int64_t>(s.ngrad, 1) * sizeof(double)));
    if (!s.h_o) MD_HIP(hipHostMalloc(reinterpret_cast<void**>(&s.h_o), s.nstate * sizeof(double)));
    for (const auto& iv : s.state_iv)
      std::memcpy(s.h_x + iv.local, state + iv.begin, (iv.end - iv.begin) * sizeof(double));
    for (const auto& iv : s.grad_iv)
      std::memcpy(s.h_d + iv.local, delta + iv.begin, (iv.end - iv.begin) * sizeof(double));
  }
  for (auto& s : m->shards) {
    if (s.nstate == 0) continue;
    MD_HIP(hipSetDevice(s.device));
    const int rc = cse_plus(s.ev, s.h_x, s.h_d, s.h_o);
    if (rc) return rc;
  }
  for (auto& s : m->shards) {
    if (s.nstate == 0) continue;
    for (const auto& iv : s.state_iv)
      std::memcpy(out + iv.begin, s.h_o + iv.local, (iv.end - iv.begin) * sizeof(double));
  }
  return CSE_OK;
}

int MultiTransferBytes(CseMulti* m, int64_t* state_h2d, int64_t* strips_d2h) {
  for (size_t k = 0; k < m->shards.size(); ++k) {
    const auto& s = m->shards[k];
    if (state_h2d) state_h2d[k] = s.nstate * (int64_t)sizeof(double);
    if (strips_d2h) strips_d2h[k] = (s.nres + s.njac) * (int64_t)sizeof(double);
  }
  return CSE_OK;
}

int CseHostRegister(void* p, size_t bytes) {
  if (!p || bytes == 0) return CseFail(CSE_ERR_INVALID, "cse_host_register: empty range");
  const hipError_t e = hipHostRegister(p, bytes, hipHostRegisterPortable);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return CseFail(CSE_ERR_HIP, std::string("hipHostRegister: ") + hipGetErrorString(e));
  }
  std::lock_guard<std::mutex> lk(g_reg_mu);
  const uintptr_t b = reinterpret_cast<uintptr_t>(p);
  g_reg.push_back({b, b + bytes});
  return CSE_OK;
}

int CseHostUnregister(void* p) {
  {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    const uintptr_t b = reinterpret_cast<uintptr_t>(p);
    auto it = std::find_if(g_reg.begin(), g_reg.end(), [&](const auto& r) { return r.first == b; });
    if (it == g_reg.end())
      return CseFail(CSE_ERR_INVALID, "cse_host_unregister: not registered with cse_host_register");
    g_reg.erase(it);
  }
  const hipError_t e = hipHostUnregister(p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return CseFail(CSE_ERR_HIP, std::string("hipHostUnregister: ") + hipGetErrorString(e));
  }
  return CSE_OK;
}

int MultiKernelStats(CseMulti* m, double* last_ms, double* total_ms, int64_t* launches) {
  double l = 0.0, t = 0.0;
  int64_t n = 0;
  for (auto& s : m->shards) {
    double sl = 0.0, st = 0.0;
    int64_t sn = 0;
    const int rc = cse_kernel_stats(s.ev, &sl, &st, &sn);
    if (rc) return rc;
    l = std::max(l, sl);
    if (st > t) t = st, n = sn;
  }
  if (last_ms) *last_ms = l;
  if (total_ms) *total_ms = t;
  if (launches) *launches = n;
  return CSE_OK;
}

int MultiResetKernelStats(CseMulti* m) {
  for (auto& s : m->shards) {
    const int rc = cse_reset_kernel_stats(s.ev);
    if (rc) return rc;
  }
  return CSE_OK;
}
