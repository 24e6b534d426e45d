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
// the shard's blocks renumbered from 0, every parameter block, and the
// residual / Jacobian-value offsets of its blocks mapped onto a compact local
// range.  The local ranges are the union of the offsets the shard's blocks
// write, kept as a list of global intervals (a Schur-ordered BlockSparse
// shard: two, its E strip and its F strip; CompressedRow: one), so one
// Evaluate hands every interval back with one D2H copy into the caller's
// buffer at the interval's global position.  Cost and gradient: per shard on
// its device, then summed over the shards in shard order (deterministic).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
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
    std::vector<Interval> res_iv, jac_iv, grad_iv;
    int64_t nres = 0, njac = 0, ngrad = 0;
    double *d_state = nullptr, *d_cost = nullptr, *d_res = nullptr, *d_jac = nullptr,
           *d_grad = nullptr;
    double *h_cost = nullptr, *h_grad = nullptr;  // pinned
  };
  std::vector<Shard> shards;
  int64_t num_parameters = 0, num_effective = 0, num_residuals = 0, num_jacobian_values = 0;
  int64_t num_residual_blocks = 0;
  bool has_layout = false;
  // Every shard's d_state holds the state of the last evaluation queued
  // without error (CSE_EVAL_SAME_POINT skips the copies).
  bool state_current = false;
  // The caller's host buffers, page-locked on first use (one per role).
  struct Reg {
    void* p = nullptr;
    size_t bytes = 0;
    bool ok = false;
  } reg[3];  // state, residuals, Jacobian values
};

namespace {

void ReleaseShard(CseMulti::Shard& s) {
  if (s.ev) cse_destroy(s.ev);
  s.ev = nullptr;
  (void)hipSetDevice(s.device);
  for (double* p : {s.d_state, s.d_cost, s.d_res, s.d_jac, s.d_grad})
    if (p) (void)hipFree(p);
  for (double* p : {s.h_cost, s.h_grad})
    if (p) (void)hipHostFree(p);
  if (s.stream) (void)hipStreamDestroy(s.stream);
  s = CseMulti::Shard{};
}

// Page-locks the caller's buffer for role k (once per buffer; a new buffer
// replaces the previous registration of that role).  Returns whether async
// copies may use it; if registration fails the copies fall back to
// synchronous pageable ones.
bool Register(CseMulti* m, int k, const void* p, size_t bytes) {
  auto& r = m->reg[k];
  if (r.p == p && r.bytes == bytes) return r.ok;
  if (r.p && r.ok) (void)hipHostUnregister(r.p);
  r.p = const_cast<void*>(p);
  r.bytes = bytes;
  const hipError_t e = hipHostRegister(r.p, bytes, hipHostRegisterPortable);
  if (e == hipErrorHostMemoryAlreadyRegistered) {
    (void)hipGetLastError();
    r.ok = true;  // already pinned by the caller (hipHostMalloc): keep, never unregister
    r.p = nullptr;
    r.bytes = 0;
    return true;
  }
  r.ok = e == hipSuccess;
  if (!r.ok) (void)hipGetLastError();
  return r.ok;
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

// The sub-descriptor of shard [g0, g1) and its evaluator.
int CreateShard(const cse_problem_desc* d, const cse_options* opts, CseMulti::Shard& s,
                const std::vector<Shape>& shapes) {
  const int64_t g0 = s.g0, g1 = s.g1, nloc = g1 - g0;
  const bool has_layout = d->jacobian_per_residual_layout && d->jacobian_per_residual_offsets;
  // Groups restricted to the shard, renumbered from g0.
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
    if (!g.residual_block_index) {
      const int64_t lo = std::clamp<int64_t>(g0 - g.first_residual_block, 0, g.num_blocks);
      const int64_t hi = std::clamp<int64_t>(g1 - g.first_residual_block, 0, g.num_blocks);
      sg.num_blocks = hi - lo;
      sg.first_residual_block = g.first_residual_block + lo - g0;
      sg.parameter_block_ids = g.parameter_block_ids ? g.parameter_block_ids + (int64_t)k.nb * lo : nullptr;
      sg.functor_data = g.functor_data ? g.functor_data + (int64_t)ds * lo : nullptr;
      for (int64_t i = lo; i < hi; ++i) {
        gr_of[g.first_residual_block + i - g0] = gi;
        i_of[g.first_residual_block + i - g0] = i;
      }
    } else {
      idx_store.emplace_back();
      ids_store.emplace_back();
      data_store.emplace_back();
      auto& ix = idx_store.back();
      auto& id = ids_store.back();
      auto& dt = data_store.back();
      for (int64_t i = 0; i < g.num_blocks; ++i) {
        const int64_t gg = g.residual_block_index[i];
        if (gg < g0 || gg >= g1) continue;
        ix.push_back(gg - g0);
        id.insert(id.end(), g.parameter_block_ids + (int64_t)k.nb * i,
                  g.parameter_block_ids + (int64_t)k.nb * (i + 1));
        dt.insert(dt.end(), g.functor_data + (int64_t)ds * i, g.functor_data + (int64_t)ds * (i + 1));
        gr_of[gg - g0] = gi;
        i_of[gg - g0] = i;
      }
      sg.num_blocks = (int64_t)ix.size();
      sg.residual_block_index = ix.data();
      sg.first_residual_block = 0;
      sg.parameter_block_ids = id.data();
      sg.functor_data = dt.data();
    }
    groups.push_back(sg);
  }
  // Residual, Jacobian-value and gradient intervals of the shard.
  IntervalBuilder rb, jb;
  std::vector<char> used(d->num_parameter_blocks, 0);
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
      if (pid < 0 || pid >= d->num_parameter_blocks)
        return CseFail(CSE_ERR_INVALID, "parameter block id out of range");
      const cse_parameter_block& pb = d->parameter_blocks[pid];
      used[pid] = 1;
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
  {
    std::vector<std::pair<int64_t, int64_t>> gs;
    for (int64_t b = 0; b < d->num_parameter_blocks; ++b) {
      const cse_parameter_block& pb = d->parameter_blocks[b];
      if (used[b] && !pb.is_constant && pb.tangent_size > 0)
        gs.push_back({pb.delta_offset, pb.delta_offset + pb.tangent_size});
    }
    IntervalBuilder gb;
    std::sort(gs.begin(), gs.end());
    for (const auto& r : gs) gb.Add(r.first, r.second);
    s.ngrad = gb.Finish(&s.grad_iv);
  }
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
  sd.num_residual_blocks = nloc;
  sd.num_residuals = s.nres;
  sd.residual_layout = res_layout.data();
  sd.jacobian_per_residual_layout = has_layout ? jac_layout.data() : nullptr;
  sd.jacobian_per_residual_offsets = has_layout ? (jac_offsets.empty() ? jac_layout.data()
                                                                        : jac_offsets.data())
                                                : nullptr;
  sd.num_jacobian_per_residual_offsets = (int64_t)jac_offsets.size();
  sd.num_jacobian_values = s.njac;
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
  if (dalloc(&s.d_state, d->num_parameters) != hipSuccess || dalloc(&s.d_cost, 1) != hipSuccess ||
      dalloc(&s.d_res, s.nres) != hipSuccess || dalloc(&s.d_jac, has_layout ? s.njac : 0) != hipSuccess ||
      dalloc(&s.d_grad, d->num_effective_parameters) != hipSuccess)
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
  m->shards.resize(n);
  for (int k = 0; k < n; ++k) {
    m->shards[k].device = devices[k];
    m->shards[k].g0 = cuts[k];
    m->shards[k].g1 = cuts[k + 1];
    const int rc = CreateShard(d, &opts, m->shards[k], shapes);
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
  for (auto& r : m->reg)
    if (r.p && r.ok) (void)hipHostUnregister(r.p);
  delete m;
}

int MultiEvaluate(CseMulti* m, const double* state, double* cost, double* residuals,
                  double* gradient, double* jac, bool same_point) {
  if (jac && !m->has_layout)
    return CseFail(CSE_ERR_INVALID, "Jacobian requested but the descriptor had no Jacobian layout");
  const bool async_state = Register(m, 0, state, m->num_parameters * sizeof(double));
  const bool async_res = residuals && Register(m, 1, residuals, m->num_residuals * sizeof(double));
  const bool async_jac = jac && Register(m, 2, jac, m->num_jacobian_values * sizeof(double));
  // Queue every shard: state H2D, evaluation, strips D2H (disjoint regions of
  // the caller's buffers), gradient rows and cost into pinned staging.
  const bool copy_state = !(same_point && m->state_current);
  m->state_current = false;
  for (auto& s : m->shards) {
    MD_HIP(hipSetDevice(s.device));
    if (m->num_parameters > 0 && copy_state) {
      if (async_state)
        MD_HIP(hipMemcpyAsync(s.d_state, state, m->num_parameters * sizeof(double),
                              hipMemcpyHostToDevice, s.stream));
      else
        MD_HIP(hipMemcpy(s.d_state, state, m->num_parameters * sizeof(double), hipMemcpyHostToDevice));
    }
    int rc = cse_evaluate_device_ex(s.ev, s.d_state, s.d_cost, residuals ? s.d_res : nullptr,
                                    gradient ? s.d_grad : nullptr, jac ? s.d_jac : nullptr,
                                    same_point ? CSE_EVAL_SAME_POINT : 0u);
    if (rc) return rc;
    MD_HIP(hipMemcpyAsync(s.h_cost, s.d_cost, sizeof(double), hipMemcpyDeviceToHost, s.stream));
    if (residuals && async_res)
      for (const auto& iv : s.res_iv)
        MD_HIP(hipMemcpyAsync(residuals + iv.begin, s.d_res + iv.local,
                              (iv.end - iv.begin) * sizeof(double), hipMemcpyDeviceToHost, s.stream));
    if (jac && async_jac)
      for (const auto& iv : s.jac_iv)
        MD_HIP(hipMemcpyAsync(jac + iv.begin, s.d_jac + iv.local, (iv.end - iv.begin) * sizeof(double),
                              hipMemcpyDeviceToHost, s.stream));
    if (gradient)
      for (const auto& iv : s.grad_iv)
        MD_HIP(hipMemcpyAsync(s.h_grad + iv.local, s.d_grad + iv.begin,
                              (iv.end - iv.begin) * sizeof(double), hipMemcpyDeviceToHost, s.stream));
  }
  m->state_current = true;
  // Wait for every shard (cse_wait synchronises the shard's stream, which
  // carries the copies too) and collect the statuses.
  int status = CSE_OK;
  for (auto& s : m->shards) {
    MD_HIP(hipSetDevice(s.device));
    const int rc = cse_wait(s.ev);
    if (rc < 0) return rc;
    if (rc == CSE_EVALUATION_FAILED) status = rc;
    // Unregistered caller buffers: synchronous copies now.
    if (residuals && !async_res)
      for (const auto& iv : s.res_iv)
        MD_HIP(hipMemcpy(residuals + iv.begin, s.d_res + iv.local, (iv.end - iv.begin) * sizeof(double),
                         hipMemcpyDeviceToHost));
    if (jac && !async_jac)
      for (const auto& iv : s.jac_iv)
        MD_HIP(hipMemcpy(jac + iv.begin, s.d_jac + iv.local, (iv.end - iv.begin) * sizeof(double),
                         hipMemcpyDeviceToHost));
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
  for (auto& s : m->shards) {
    const int rc = cse_set_plus_jacobians(s.ev, pj);
    if (rc) return rc;
  }
  return CSE_OK;
}

int MultiPlus(CseMulti* m, const double* state, const double* delta, double* out) {
  return cse_plus(m->shards[0].ev, state, delta, out);
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
