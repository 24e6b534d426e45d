// layout.cpp -- host-side Jacobian layout builders exported through cse.h.
//
// For callers without Ceres' own writers (our C++ ProblemCUDA facade, the
// Python binding, FFI users).  They produce exactly the tables the
// reference's ProgramEvaluatorCUDA hands to RegisteredCUDAEvaluators::Init:
//   residual_layout             program_evaluator_cuda.h:159-170
//   BlockSparseMatrix           block_jacobian_writer.cc:62-160
//   CompressedRowSparseMatrix   compressed_row_jacobian_writer.cc:93-193,240-300
#include <algorithm>
#include <string>
#include <utility>
#include <vector>

#include "../../include/cse.h"

namespace cse {
// cse_last_error's text (cse_evaluator.hip), kept here so the layout
// builders can set it when they are linked without the evaluator.
std::string& LastError() {
  thread_local std::string text;
  return text;
}
}  // namespace cse

namespace {

int Invalid(const std::string& msg) {
  cse::LastError() = msg;
  return CSE_ERR_INVALID;
}

bool Active(const cse_parameter_block* pbs, int32_t id) { return !pbs[id].is_constant; }

// Program index among the active blocks (ParameterBlock::index() of the
// reduced program): active blocks are numbered in program order.
std::vector<int64_t> ActiveIndex(int64_t npb, const cse_parameter_block* pbs) {
  std::vector<int64_t> idx(npb, -1);
  int64_t k = 0;
  for (int64_t b = 0; b < npb; ++b)
    if (!pbs[b].is_constant) idx[b] = k++;
  return idx;
}

}  // namespace

extern "C" int64_t cse_layout_offsets_count(int64_t /*npb*/, const cse_parameter_block* pbs,
                                            int64_t nrb, const int64_t* param_begin,
                                            const int32_t* param_ids, const int32_t* nres) {
  int64_t count = 0;
  for (int64_t i = 0; i < nrb; ++i)
    for (int64_t q = param_begin[i]; q < param_begin[i + 1]; ++q)
      if (Active(pbs, param_ids[q])) count += nres[i];
  return count;
}

extern "C" int cse_block_sparse_layout(int64_t npb, const cse_parameter_block* pbs, int64_t nrb,
                                       const int64_t* param_begin, const int32_t* param_ids,
                                       const int32_t* nres, int64_t num_eliminate_blocks,
                                       int64_t* residual_layout, int64_t* per_residual_layout,
                                       int64_t* per_residual_offsets,
                                       int64_t* num_jacobian_values) {
  if (npb < 0 || nrb < 0 || !param_begin || !nres || !residual_layout)
    return Invalid("layout: negative count or missing table");
  const std::vector<int64_t> index = ActiveIndex(npb, pbs);
  auto is_e = [&](int32_t id) { return index[id] < num_eliminate_blocks; };
  // Pass 1: the E cells occupy [0, e_total); F cells follow.
  int64_t e_total = 0;
  for (int64_t i = 0; i < nrb; ++i)
    for (int64_t q = param_begin[i]; q < param_begin[i + 1]; ++q) {
      const int32_t id = param_ids[q];
      if (Active(pbs, id) && is_e(id)) e_total += (int64_t)nres[i] * pbs[id].tangent_size;
    }
  // Pass 2: place cells in residual order; each cell is row-major
  // nres x tangent, so row k of a cell starts at cell + k*tangent.
  int64_t e_pos = 0, f_pos = e_total, r_pos = 0, t = 0;
  for (int64_t i = 0; i < nrb; ++i) {
    residual_layout[i] = r_pos;
    r_pos += nres[i];
    if (per_residual_layout) per_residual_layout[i] = t;
    for (int64_t q = param_begin[i]; q < param_begin[i + 1]; ++q) {
      const int32_t id = param_ids[q];
      if (!Active(pbs, id)) continue;
      const int64_t tan = pbs[id].tangent_size;
      int64_t& pos = is_e(id) ? e_pos : f_pos;
      for (int k = 0; k < nres[i]; ++k, ++t) {
        if (per_residual_offsets) per_residual_offsets[t] = pos;
        pos += tan;
      }
    }
  }
  if (num_jacobian_values) *num_jacobian_values = f_pos;
  return CSE_OK;
}

extern "C" int cse_compressed_row_layout(int64_t npb, const cse_parameter_block* pbs, int64_t nrb,
                                         const int64_t* param_begin, const int32_t* param_ids,
                                         const int32_t* nres, int64_t* residual_layout,
                                         int64_t* per_residual_layout,
                                         int64_t* per_residual_offsets,
                                         int64_t* num_jacobian_values, int64_t* crs_rows,
                                         int64_t* crs_cols) {
  if (npb < 0 || nrb < 0 || !param_begin || !nres || !residual_layout)
    return Invalid("layout: negative count or missing table");
  const std::vector<int64_t> index = ActiveIndex(npb, pbs);
  int64_t row = 0, value = 0, t = 0;
  if (crs_rows) crs_rows[0] = 0;
  // (program index, active argument position) of a block's active
  // parameters, sorted by program index: the column order of its rows.
  std::vector<std::pair<int64_t, int>> order;
  std::vector<int32_t> order_id;
  for (int64_t i = 0; i < nrb; ++i) {
    residual_layout[i] = row;
    if (per_residual_layout) per_residual_layout[i] = t;
    order.clear();
    int a = 0;
    int64_t width = 0;
    for (int64_t q = param_begin[i]; q < param_begin[i + 1]; ++q) {
      const int32_t id = param_ids[q];
      if (!Active(pbs, id)) continue;
      order.push_back({index[id], a++});
      width += pbs[id].tangent_size;
    }
    std::sort(order.begin(), order.end());
    for (size_t m = 1; m < order.size(); ++m)
      if (order[m].first == order[m - 1].first)
        return Invalid("layout: residual block " + std::to_string(i) +
                       " lists a parameter block twice");
    // Map active argument -> parameter block id.
    order_id.assign(order.size(), -1);
    {
      int aa = 0;
      for (int64_t q = param_begin[i]; q < param_begin[i + 1]; ++q)
        if (Active(pbs, param_ids[q])) order_id[aa++] = param_ids[q];
    }
    for (int k = 0; k < nres[i]; ++k) {
      int64_t col = 0;
      for (const auto& e : order) {
        const int32_t id = order_id[e.second];
        const int tan = pbs[id].tangent_size;
        if (per_residual_offsets) per_residual_offsets[t + k + (int64_t)nres[i] * e.second] = value + col;
        if (crs_cols)
          for (int c = 0; c < tan; ++c) crs_cols[value + col + c] = pbs[id].delta_offset + c;
        col += tan;
      }
      value += width;
      if (crs_rows) crs_rows[row + k + 1] = value;
    }
    row += nres[i];
    t += (int64_t)order.size() * nres[i];
  }
  if (num_jacobian_values) *num_jacobian_values = value;
  return CSE_OK;
}
