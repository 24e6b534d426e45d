// operator_kernels.hpp -- the kernels around the evaluation: the gradient
// post-pass and the fused gradient's tails, the Jacobian as a linear
// operator (J x, J^T x, the CGNR normal operator), Program::Plus, the cost
// reduction and the slot-0 repack.
#ifndef CSE_OPERATOR_KERNELS_HPP_
#define CSE_OPERATOR_KERNELS_HPP_

#include "evaluate_kernel.hpp"

namespace cse {

// ---------------------------------------------------------------------------
// Gradient g = J^T r as a deterministic post-pass over the outputs just
// written (affine groups with residuals and Jacobian requested).  The
// reference adds J^T r with per-element FP64 atomics inside the evaluate
// kernel (cuda_evaluator_kernel.h:149-160); with ~2,100 observations per
// camera and 64 random addresses per wave instruction those atomics ran at
// 18 ms per evaluation here (0.05 of the HBM roofline).  Instead, for each
// slot, the blocks are listed per parameter block (counting sort at create
// time; identity for the points of a Schur-ordered problem) and every
// parameter block sums its blocks' J_b^T r_b in a fixed order:
//   kWaveMode = false: one lane per parameter block (few blocks each:
//                      points), true: one wave per parameter block (many
//                      blocks each: cameras), lanes strided over the blocks
//                      and a fixed xor-butterfly.
// ---------------------------------------------------------------------------
struct GradArgs {
  const double* jac;
  int64_t jrow[3];   // start of row k of the slot's cell for block 0
  int64_t jstride;   // per block
  const double* res;
  int64_t res_base;
  const int32_t* perm;  // blocks sorted by parameter block; null = identity
  const int64_t* off;   // [count + 1]
  int64_t count;        // parameter blocks lo .. lo + count - 1
  int32_t lo;
  double* grad;
  int64_t delta_base;   // delta offset of id = delta_base + S * id
  const int64_t* delta_tab;  // GradientChunkReduceKernel: [count] offsets instead (may be null)
};

template <int NR, int S, bool kWaveMode>
__global__ __launch_bounds__(kBlockThreads) void GradientSlotKernel(const GradArgs g) {
  double acc[S];
#pragma unroll
  for (int c = 0; c < S; ++c) acc[c] = 0.0;
  int64_t p;
  int64_t q0, q1, qs;
  if constexpr (kWaveMode) {
    p = ((int64_t)blockIdx.x * kBlockThreads + threadIdx.x) / kWave;
    if (p >= g.count) return;
    q0 = g.off[p] + (threadIdx.x & (kWave - 1));
    q1 = g.off[p + 1];
    qs = kWave;
  } else {
    p = (int64_t)blockIdx.x * kBlockThreads + threadIdx.x;
    if (p >= g.count) return;
    q0 = g.off[p];
    q1 = g.off[p + 1];
    qs = 1;
  }
  for (int64_t q = q0; q < q1; q += qs) {
    const int64_t b = g.perm ? (int64_t)g.perm[q] : q;
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const double rk = g.res[g.res_base + (int64_t)NR * b + k];
      const double* row = g.jac + g.jrow[k] + g.jstride * b;
#pragma unroll
      for (int c = 0; c < S; ++c) acc[c] += row[c] * rk;
    }
  }
  double* dst = g.grad + g.delta_base + (int64_t)S * (g.lo + p);
  if constexpr (kWaveMode) {
#pragma unroll
    for (int c = 0; c < S; ++c)
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) acc[c] += __shfl_xor(acc[c], off, kWave);
    if ((threadIdx.x & (kWave - 1)) == 0) {
#pragma unroll
      for (int c = 0; c < S; ++c) dst[c] += acc[c];
    }
  } else {
#pragma unroll
    for (int c = 0; c < S; ++c) dst[c] += acc[c];
  }
}

// Parameter blocks with many blocks (cameras): their block lists are cut
// into chunks of at most kGradChunk blocks, one wave per chunk
// (GradientLanesKernel), and GradientChunkReduceKernel adds each parameter
// block's chunk partials in order.  Deterministic, no atomics.  (An
// element-per-lane variant that reads whole cells per instruction measured
// 3-10 % slower: the random cells and residual pairs cost whole lines
// either way.)
constexpr int kGradChunk = 512;

struct GradChunks {
  const int64_t* begin;      // [nchunks + 1] chunk c covers perm[begin[c], begin[c+1])
  const int64_t* chunk_off;  // [count + 1] chunks of parameter block p
  double* partial;           // [nchunks][S]
  int64_t nchunks;
};

// Lane per block: each lane reads its blocks' whole cells
// (rows of S contiguous doubles) and residual pairs; S accumulators per
// lane, combined by a fixed xor-butterfly.
template <int NR, int S>
__global__ __launch_bounds__(kBlockThreads) void GradientLanesKernel(const GradArgs g,
                                                                     const GradChunks ch) {
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const int64_t cid = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  if (cid >= ch.nchunks) return;
  const int64_t q1 = ch.begin[cid + 1];
  double acc[S];
#pragma unroll
  for (int c = 0; c < S; ++c) acc[c] = 0.0;
  for (int64_t q = ch.begin[cid] + lane; q < q1; q += kWave) {
    const int64_t b = g.perm ? (int64_t)g.perm[q] : q;
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const double rk = g.res[g.res_base + (int64_t)NR * b + k];
      const double* row = g.jac + g.jrow[k] + g.jstride * b;
#pragma unroll
      for (int c = 0; c < S; ++c) acc[c] += row[c] * rk;
    }
  }
#pragma unroll
  for (int c = 0; c < S; ++c)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc[c] += __shfl_xor(acc[c], off, kWave);
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < S; ++c) ch.partial[cid * S + c] = acc[c];
  }
}

// kAssign: the row is written, not added to (the evaluator's grad_exact:
// every row of the gradient is written once and it is not zeroed first).
template <int S, bool kAssign>
__device__ __forceinline__ void ChunkReduceRow(const GradArgs& g, const GradChunks& ch, int64_t p) {
  if (p >= g.count) return;
  // A block without chunks adds nothing (and a constant one has no row).
  if (!kAssign && ch.chunk_off[p] == ch.chunk_off[p + 1]) return;
  double acc[S];
#pragma unroll
  for (int c = 0; c < S; ++c) acc[c] = 0.0;
  for (int64_t q = ch.chunk_off[p]; q < ch.chunk_off[p + 1]; ++q)
#pragma unroll
    for (int c = 0; c < S; ++c) acc[c] += ch.partial[q * S + c];
  double* dst = g.grad + (g.delta_tab ? g.delta_tab[p] : g.delta_base + (int64_t)S * (g.lo + p));
#pragma unroll
  for (int c = 0; c < S; ++c) {
    if (kAssign)
      dst[c] = acc[c];
    else
      dst[c] += acc[c];
  }
}

template <int S, bool kAssign = false>
__global__ __launch_bounds__(kBlockThreads) void GradientChunkReduceKernel(const GradArgs g,
                                                                           const GradChunks ch) {
  ChunkReduceRow<S, kAssign>(g, ch, (int64_t)blockIdx.x * kBlockThreads + threadIdx.x);
}

// Fused-gradient slot 0 (FusedGrad): each chunk of a parameter block's
// block list sums the blocks' written contributions (S of the SP doubles
// per block; two 64-byte sectors per block instead of the Jacobian cell
// and residual pair), a fixed butterfly, then GradientChunkReduceKernel.
// order (may be null): the chunks taken pass-major (BuildGradPlan), so the
// resident waves read the records of one block range at a time and the
// 64-byte sectors two neighbouring 80-byte records share are fetched once.
template <int S, int SP>
__global__ __launch_bounds__(kBlockThreads) void GradientContribKernel(const double* contrib,
                                                                       const int32_t* perm,
                                                                       const GradChunks ch,
                                                                       const int32_t* order) {
  static_assert(SP % 2 == 0 && SP >= S, "16-byte records");
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const int64_t slot = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  if (slot >= ch.nchunks) return;
  const int64_t cid = order ? (int64_t)order[slot] : slot;
  const int64_t q1 = ch.begin[cid + 1];
  double acc[S];
#pragma unroll
  for (int c = 0; c < S; ++c) acc[c] = 0.0;
  for (int64_t q = ch.begin[cid] + lane; q < q1; q += kWave) {
    const double2* rec = reinterpret_cast<const double2*>(contrib + (int64_t)SP * perm[q]);
#pragma unroll
    for (int h = 0; h < SP / 2; ++h) {
      const double2 v = rec[h];
      if (2 * h < S) acc[2 * h] += v.x;
      if (2 * h + 1 < S) acc[2 * h + 1] += v.y;
    }
  }
#pragma unroll
  for (int c = 0; c < S; ++c)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc[c] += __shfl_xor(acc[c], off, kWave);
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < S; ++c) ch.partial[cid * S + c] = acc[c];
  }
}

// Fused-gradient slot 1: the waves' boundary entries (sum[S], id) are in
// wave order, so their ids are non-decreasing; the first entry of each id
// adds that id's entries in order and adds the sum to the row (no interior
// run of any wave touched these rows).
template <int S, bool kAssign>
__device__ __forceinline__ void BoundaryEntry(const double* side, int64_t count, double* grad,
                                              int64_t delta_base, int64_t e) {
  static_assert(S <= 3, "entries hold 3 sums and the id");
  if (e >= count) return;
  // The entry, its predecessor's id and the next two entries in one round
  // trip (independent 16-byte loads; a key's entries are one to three in
  // practice: a point continued from the previous wave, and into the next),
  // then the rare longer runs entry by entry.  Summed in entry order from 0.
  const double2* s2 = reinterpret_cast<const double2*>(side);
  const double2 m0 = s2[2 * e], m1 = s2[2 * e + 1];
  const double kprev = e > 0 ? side[4 * (e - 1) + 3] : -1.0;
  double2 n0[2], n1[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int64_t f = e + 1 + t < count ? e + 1 + t : e;
    n0[t] = s2[2 * f];
    n1[t] = s2[2 * f + 1];
  }
  const double key = m1.y;
  if (e > 0 && kprev == key) return;
  double acc[S];
#pragma unroll
  for (int c = 0; c < S; ++c) acc[c] = 0.0;
  auto add = [&](const double2& v0, const double2& v1) {
    const double v[3] = {v0.x, v0.y, v1.x};
#pragma unroll
    for (int c = 0; c < S; ++c) acc[c] += v[c];
  };
  add(m0, m1);
  int64_t f = e + 1;
  bool more = true;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    if (more && f < count && n1[t].y == key) {
      add(n0[t], n1[t]);
      ++f;
    } else {
      more = false;
    }
  }
  if (more) {
    for (; f < count && side[4 * f + 3] == key; ++f)
#pragma unroll
      for (int c = 0; c < S; ++c) acc[c] += side[4 * f + c];
  }
  double* dst = grad + delta_base + (int64_t)S * (int64_t)key;
#pragma unroll
  for (int c = 0; c < S; ++c) {
    if (kAssign)
      dst[c] = acc[c];
    else
      dst[c] += acc[c];
  }
}

template <int S, bool kAssign = false>
__global__ __launch_bounds__(kBlockThreads) void GradientBoundaryKernel(const double* side,
                                                                        int64_t count,
                                                                        double* grad,
                                                                        int64_t delta_base) {
  BoundaryEntry<S, kAssign>(side, count, grad, delta_base, (int64_t)blockIdx.x * kBlockThreads + threadIdx.x);
}

// Gradient mode 0's tail in one launch: workgroups [0, boundary_wg) add the
// slot-1 boundary entries (GradientBoundaryKernel), the rest the slot-0
// chunk partials per camera (GradientChunkReduceKernel).  The two touch
// disjoint rows.
template <int S1, int S0, bool kAssign>
__global__ __launch_bounds__(kBlockThreads) void GradientTailKernel(const double* side, int64_t entries,
                                                                    int64_t delta_base1, int64_t boundary_wg,
                                                                    const GradArgs g, const GradChunks ch) {
  const int64_t b = blockIdx.x;
  if (b < boundary_wg)
    BoundaryEntry<S1, kAssign>(side, entries, g.grad, delta_base1, b * kBlockThreads + threadIdx.x);
  else
    ChunkReduceRow<S0, kAssign>(g, ch, (b - boundary_wg) * kBlockThreads + threadIdx.x);
}

// Identity order (the points of a Schur-ordered problem): one 64-thread
// workgroup per 64 consecutive parameter blocks, whose blocks form one
// contiguous range.  The range is walked in tiles of 64 blocks: all lanes
// form the products J[e] * r[k] element by element (contiguous loads), park
// them in LDS, and then thread t sums parameter block t's blocks of the
// tile in block, row order.
template <int NR, int S>
__global__ __launch_bounds__(kWave) void GradientRangeKernel(const GradArgs g) {
  constexpr int E = NR * S;
  constexpr int T = kWave;  // blocks per tile
  __shared__ double prod[T * E];
  const int lane = threadIdx.x;
  const int64_t p0 = (int64_t)blockIdx.x * kWave;
  const int64_t p = p0 + lane;
  const int64_t pend = p0 + kWave < g.count ? p0 + kWave : g.count;
  const int64_t B0 = g.off[p0], B1 = g.off[pend];
  const int64_t my0 = p < g.count ? g.off[p] : B1, my1 = p < g.count ? g.off[p + 1] : B1;
  double acc[S];
#pragma unroll
  for (int cc = 0; cc < S; ++cc) acc[cc] = 0.0;
  for (int64_t t0 = B0; t0 < B1; t0 += T) {
    const int nb = B1 - t0 < T ? (int)(B1 - t0) : T;
#pragma unroll
    for (int it = 0; it < E; ++it) {
      const int t = it * kWave + lane;  // element t of the tile
      const int bm = t / E, e = t - bm * E, k = e / S, cc = e - k * S;
      double v = 0.0;
      if (bm < nb) {
        const int64_t b = t0 + bm;
        v = g.jac[g.jrow[k] + g.jstride * b + cc] * g.res[g.res_base + (int64_t)NR * b + k];
      }
      prod[t] = v;
    }
    __syncthreads();
    const int64_t lo = my0 > t0 ? my0 : t0, hi = my1 < t0 + nb ? my1 : t0 + nb;
    for (int64_t b = lo; b < hi; ++b) {
      const int bm = (int)(b - t0);
#pragma unroll
      for (int k = 0; k < NR; ++k)
#pragma unroll
        for (int cc = 0; cc < S; ++cc) acc[cc] += prod[bm * E + k * S + cc];
    }
    __syncthreads();
  }
  if (p < g.count) {
    double* dst = g.grad + g.delta_base + (int64_t)S * (g.lo + p);
#pragma unroll
    for (int cc = 0; cc < S; ++cc) dst[cc] += acc[cc];
  }
}

// ---------------------------------------------------------------------------
// The Jacobian as a linear operator (cse_jacobian_right/left_multiply):
// y += J x and y += J^T x on the values this evaluator wrote.  The affine
// J^T x reuses the gradient post-pass kernels (x in place of r).
// ---------------------------------------------------------------------------
template <class K>
__global__ __launch_bounds__(kBlockThreads) void RightMultiplyAffineKernel(const GroupArgs a,
                                                                           const double* x,
                                                                           double* y) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, NB = Tr::NB, S0 = Tr::S0, S1 = Tr::S1;
  const int64_t i = (int64_t)blockIdx.x * kBlockThreads + threadIdx.x;
  if (i >= a.n) return;
  const int2 id = LoadIds<K>(a, i);
  const double* x0 = x + a.delta_base[0] + (int64_t)S0 * id.x;
  double acc[NR];
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    const double* row = a.jacobian + a.jac_base[0][k] + a.jac_stride[0] * i;
    double t = 0.0;
#pragma unroll
    for (int c = 0; c < S0; ++c) t += row[c] * x0[c];
    acc[k] = t;
  }
  if constexpr (NB == 2) {
    const double* x1 = x + a.delta_base[1] + (int64_t)S1 * id.y;
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const double* row = a.jacobian + a.jac_base[1][k] + a.jac_stride[1] * i;
#pragma unroll
      for (int c = 0; c < S1; ++c) acc[k] += row[c] * x1[c];
    }
  }
  double* yb = y + a.res_base + (int64_t)NR * i;
#pragma unroll
  for (int k = 0; k < NR; ++k) yb[k] += acc[k];
}

// Table path (any layout, constant blocks, tangent sizes): the reference's
// WriteJacobians addressing (cuda_evaluator_kernel.h:260-294).
template <class K, bool kLeft>
__global__ __launch_bounds__(kBlockThreads) void MultiplyTableKernel(const GroupArgs a,
                                                                     const double* x, double* y) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, NB = Tr::NB;
  const int64_t i = (int64_t)blockIdx.x * kBlockThreads + threadIdx.x;
  if (i >= a.n) return;
  const int64_t gi = a.gindex ? a.gindex[i] : a.first + i;
  const int64_t res = a.residual_layout[gi];
  int64_t q = a.jac_layout[gi];
  double acc[NR];
#pragma unroll
  for (int k = 0; k < NR; ++k) acc[k] = 0.0;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const PbDev pb = a.pbs[a.ids[i * NB + j]];
    if (pb.is_constant) continue;
    const int S = Tr::Size(j);
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const double* row = a.jacobian + a.jac_offsets[q++];
      for (int c = 0; c < S; ++c) {
        if (c >= pb.tangent_size) break;
        if constexpr (kLeft)
          unsafeAtomicAdd(y + pb.delta_offset + c, row[c] * x[res + k]);
        else
          acc[k] += row[c] * x[pb.delta_offset + c];
      }
    }
  }
  if constexpr (!kLeft) {
#pragma unroll
    for (int k = 0; k < NR; ++k) y[res + k] += acc[k];
  }
}

// The CGNR normal operator in one pass over J (cse_cgnr_multiply):
// y += J^T (J x), replacing CudaCgnrLinearOperator::RightMultiplyAndAccumulate
// (internal/ceres/cgnr_solver.cc:226-237), which runs z = J x and y += J^T z
// as two sparse products (two reads of J and a round trip of z).  One wave
// per 64-block chunk, as the evaluator:
//   * the wave's Jacobian image (BSM: its F then E segments; CRS: its rows)
//     comes in by LDS-DMA, 1 KiB per instruction, and each lane reads its
//     block's cells from LDS;
//   * z_b = J_b x (two values) stays in registers;
//   * slot 1 (points): E_b^T z_b through the fused gradient's segmented
//     scan -- interior runs add into y directly, the wave's first and last
//     runs go to boundary entries (GradientBoundaryKernel adds them);
//   * slot 0 (cameras): F_b^T z_b in block order (GradientContribKernel and
//     GradientChunkReduceKernel add them per camera, fixed order).
// Deterministic; the host requires the fused gradient's eligibility.
template <class K, bool kCrs, int kWPB = kWavesPerBlock>
__global__ __launch_bounds__(kWPB * kWave) void CgnrMultiplyKernel(const GroupArgs a,
                                                                   const double* x, double* y) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, N = Tr::N;
  static_assert(Tr::NB == 2 && NR == 2 && S1 == 3, "Snavely-shaped groups");
  constexpr int S0p = (S0 + 1) & ~1;
  constexpr int kImg = kWave * NR * N;        // doubles of one wave's Jacobian image
  constexpr int kPieces = kImg / (2 * kWave);  // 16-byte DMA pieces per lane
  static_assert(kImg % (2 * kWave) == 0 && (kWave * NR * S0) % (2 * kWave) == 0, "16-B pieces");
  __shared__ double img[kWPB][kImg];
  const int lane = threadIdx.x & (kWave - 1), wave = kWPB == 1 ? 0 : threadIdx.x / kWave;
  const int64_t nchunks = (a.n + kWave - 1) / kWave;
  const int64_t c = (int64_t)blockIdx.x * kWPB + wave;
  if (c >= nchunks) return;
  double* im = img[wave];
  const int64_t i0 = c * kWave;
  const int nw = a.n - i0 < kWave ? (int)(a.n - i0) : kWave;
  const bool active = lane < nw;
  const int64_t i = active ? i0 + lane : a.n - 1;
  const long long idw = __builtin_nontemporal_load(reinterpret_cast<const long long*>(a.ids) + i);
  const int id0 = (int)idw, id1 = (int)(idw >> 32);

  // Column c of row k of slot j for this lane's block, at LDS offset
  // off[j][k] + c (full chunks) -- or straight from HBM (the last chunk).
  const int64_t row0 = kCrs ? (a.jac_base[0][0] < a.jac_base[1][0] ? a.jac_base[0][0]
                                                                     : a.jac_base[1][0])
                            : 0;
  double F[NR * S0], E[NR * S1];
  if (nw == kWave) {
    if constexpr (kCrs) {
      const double* seg = a.jacobian + row0 + (int64_t)NR * N * i0;
#pragma unroll
      for (int k = 0; k < kPieces; ++k)
        __builtin_amdgcn_global_load_lds(seg + 2 * (k * kWave + lane), im + 2 * kWave * k, 16, 0, 0);
    } else {
      const double* segF = a.jacobian + a.jac_base[0][0] + a.jac_stride[0] * i0;
      const double* segE = a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * i0;
      constexpr int kF = kWave * NR * S0 / (2 * kWave);
#pragma unroll
      for (int k = 0; k < kF; ++k)
        __builtin_amdgcn_global_load_lds(segF + 2 * (k * kWave + lane), im + 2 * kWave * k, 16, 0, 0);
#pragma unroll
      for (int k = 0; k < kPieces - kF; ++k)
        __builtin_amdgcn_global_load_lds(segE + 2 * (k * kWave + lane), im + 2 * kWave * (kF + k),
                                         16, 0, 0);
    }
  }
  double xc[S0], xp[S1];
  {
    const double* x0 = x + a.delta_base[0] + (int64_t)S0 * id0;
    const double* x1 = x + a.delta_base[1] + (int64_t)S1 * id1;
#pragma unroll
    for (int k = 0; k < S0; ++k) xc[k] = x0[k];
#pragma unroll
    for (int k = 0; k < S1; ++k) xp[k] = x1[k];
  }
  if (nw == kWave) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const int f0 = kCrs ? (int)(a.jac_base[0][k] - row0) + NR * N * lane : NR * S0 * lane + S0 * k;
      const int e0 = kCrs ? (int)(a.jac_base[1][k] - row0) + NR * N * lane
                          : kWave * NR * S0 + NR * S1 * lane + S1 * k;
#pragma unroll
      for (int cc = 0; cc < S0; ++cc) F[k * S0 + cc] = im[f0 + cc];
#pragma unroll
      for (int cc = 0; cc < S1; ++cc) E[k * S1 + cc] = im[e0 + cc];
    }
  } else {
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      const double* rf = a.jacobian + a.jac_base[0][k] + a.jac_stride[0] * i;
      const double* re = a.jacobian + a.jac_base[1][k] + a.jac_stride[1] * i;
#pragma unroll
      for (int cc = 0; cc < S0; ++cc) F[k * S0 + cc] = rf[cc];
#pragma unroll
      for (int cc = 0; cc < S1; ++cc) E[k * S1 + cc] = re[cc];
    }
  }
  double z[NR];
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    double t = 0.0;
#pragma unroll
    for (int cc = 0; cc < S0; ++cc) t += F[k * S0 + cc] * xc[cc];
#pragma unroll
    for (int cc = 0; cc < S1; ++cc) t += E[k * S1 + cc] * xp[cc];
    z[k] = active ? t : 0.0;
  }
  // J_b^T z_b: FusedGrad with z in place of r (its J1 rows are S1p = S1 wide).
  FusedGrad<K> fg;
  fg.Compute(z, F, E, id1, active, lane, nw, c);
  if (fg.interior) {
    double* row = y + a.delta_base[1] + (int64_t)S1 * fg.key;
    row[0] += fg.g1[0];
    row[1] += fg.g1[1];
    row[2] += fg.g1[2];
  }
  if (fg.writer) {
    double4* e = reinterpret_cast<double4*>(a.gside + 4 * fg.entry);
    *e = make_double4(fg.g1[0], fg.g1[1], fg.g1[2], fg.g1[3]);
  }
  if (nw == 1 && lane == 0)
    *reinterpret_cast<double4*>(a.gside + 4 * (2 * c + 1)) = make_double4(0.0, 0.0, 0.0, fg.g1[3]);
  if (nw == kWave) {
    // Camera contributions: staged (the image has been read), 16-B pieces.
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < S0p / 2; ++j)
      reinterpret_cast<double2*>(im)[lane * (S0p / 2) + j] = make_double2(fg.g0[2 * j], fg.g0[2 * j + 1]);
    __builtin_amdgcn_wave_barrier();
    typedef double v2d __attribute__((ext_vector_type(2)));
    v2d* dst = reinterpret_cast<v2d*>(a.gcontrib + (int64_t)S0p * i0);
#pragma unroll
    for (int j = 0; j < S0p / 2; ++j)
      __builtin_nontemporal_store(reinterpret_cast<const v2d*>(im)[j * kWave + lane],
                                  dst + j * kWave + lane);
  } else if (active) {
    double* dst = a.gcontrib + (int64_t)S0p * i;
#pragma unroll
    for (int cc = 0; cc < S0p; ++cc) dst[cc] = fg.g0[cc];
  }
}

// y += D .* D .* x (CudaVector::DtDxpy, cgnr_solver.cc:236).
__global__ __launch_bounds__(kBlockThreads) void DtDxpyKernel(const double* D, const double* x,
                                                              double* y, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * kBlockThreads + threadIdx.x;
  if (i < n) y[i] += D[i] * D[i] * x[i];
}

// Program::Plus for manifold-free blocks: runs of consecutive state entries
// whose delta offset is a constant shift away (one run for a BAL problem).
struct PlusRun {
  int64_t state_begin;
  int64_t length;
  int64_t delta_shift;  // delta index = state index - delta_shift
};

__global__ __launch_bounds__(kBlockThreads) void PlusKernel(const double* x, const double* delta,
                                                            double* out, const PlusRun* runs,
                                                            int num_runs) {
  for (int r = 0; r < num_runs; ++r) {
    const PlusRun run = runs[r];
    for (int64_t t = (int64_t)blockIdx.x * kBlockThreads + threadIdx.x; t < run.length;
         t += (int64_t)gridDim.x * kBlockThreads) {
      const int64_t i = run.state_begin + t;
      out[i] = x[i] + delta[i - run.delta_shift];
    }
  }
}

// Program::Plus of the CSE_MANIFOLD_QUATERNION_EUCLIDEAN blocks, one block
// per thread: ProductManifold<QuaternionManifold, EuclideanManifold<n>>::Plus,
// i.e. QuaternionPlusImpl (internal/ceres/manifold.cc:28-59: the quaternion
// exp(delta) on the left of x, x unchanged when |delta| is zero) and x + delta
// for the Euclidean tail.
struct QuatPlusBlock {
  int64_t state_offset;
  int64_t delta_offset;
  int32_t size;
  int32_t pad;
};

__global__ __launch_bounds__(kBlockThreads) void QuaternionPlusKernel(const double* x,
                                                                      const double* delta,
                                                                      double* out,
                                                                      const QuatPlusBlock* blocks,
                                                                      int64_t n) {
  const int64_t b = (int64_t)blockIdx.x * kBlockThreads + threadIdx.x;
  if (b >= n) return;
  const QuatPlusBlock B = blocks[b];
  const double* q = x + B.state_offset;
  const double* d = delta + B.delta_offset;
  double* o = out + B.state_offset;
  // |delta| as std::hypot(d0, d1, d2) (manifold.cc:33), in libstdc++'s
  // scaled form: no underflow for tiny steps (|d| < 1e-154 would square to
  // zero and be skipped), no overflow for huge ones; zero exactly when the
  // three components are (the FP_ZERO test, :35).
  const double a0 = fabs(d[0]), a1 = fabs(d[1]), a2 = fabs(d[2]);
  const double m = fmax(a0, fmax(a1, a2));
  if (m == 0.0) {
    o[0] = q[0];
    o[1] = q[1];
    o[2] = q[2];
    o[3] = q[3];
  } else {
    double nd;
    {
#pragma clang fp contract(off)
      const double r0 = a0 / m, r1 = a1 / m, r2 = a2 / m;
      nd = m * sqrt(r0 * r0 + r1 * r1 + r2 * r2);
    }
    double sn, cs;
    sincos(nd, &sn, &cs);
    const double sbd = sn / nd;
    const double w = cs, a = sbd * d[0], bq = sbd * d[1], c = sbd * d[2];
    o[0] = w * q[0] - a * q[1] - bq * q[2] - c * q[3];
    o[1] = w * q[1] + a * q[0] + bq * q[3] - c * q[2];
    o[2] = w * q[2] - a * q[3] + bq * q[0] + c * q[1];
    o[3] = w * q[3] + a * q[2] - bq * q[1] + c * q[0];
  }
  for (int k = 4; k < B.size; ++k) o[k] = q[k] + d[k - 1];
}

// Held-camera groups (Tune::kConst0 Jacobian kernels): after a held block
// the packed F cells (BSM) or row blocks (CRS) of a chunk start inside a
// 64-byte sector.  Each full chunk stored only the whole sectors of its
// segment and put its head pieces (slots 0-3: at their positions in the
// sector before its first whole one) and its tail pieces (slots 4-7: at their
// positions in the sector after its last) into side[16 c ..]; here thread
// 4 c + pos assembles position pos of the sector chunk c shares with the
// previous chunk that has a segment (prev[c]): the tail of that chunk, then
// the head of c, each only if that chunk was full (c < nfull; a ragged last
// chunk writes its whole segment itself), so each such sector is written as
// one 64-byte piece instead of two partial writes.  The group's first
// segment wrote its head itself.
__global__ __launch_bounds__(kBlockThreads) void HeldSectorFixupKernel(double* jac, const int64_t* fbase,
                                                                       const double* side,
                                                                       const int32_t* prev,
                                                                       int64_t nchunks, int64_t nfull) {
  const int64_t t = (int64_t)blockIdx.x * kBlockThreads + threadIdx.x;
  const int64_t c = t >> 2;
  const int pos = (int)(t & 3);
  if (c >= nchunks || c == 0) return;
  const int64_t f0 = fbase[c];
  if (fbase[c + 1] == f0 || f0 == fbase[0]) return;  // no segment, or the first one
  const uintptr_t A0 = reinterpret_cast<uintptr_t>(jac + f0);
  const int hp = (int)(((64 - (A0 & 63)) & 63) >> 4);  // head pieces of c
  if (hp == 0) return;                                    // starts on a sector
  const int64_t pc = prev[c];
  const double* src = nullptr;
  if (pos < 4 - hp) {
    if (pc >= 0 && pc < nfull) src = side + 16 * pc + 8 + 2 * pos;
  } else if (c < nfull) {
    src = side + 16 * c + 2 * pos;
  }
  if (src) {
    double* S = reinterpret_cast<double*>(A0 & ~(uintptr_t)63);
    *reinterpret_cast<double2*>(S + 2 * pos) = *reinterpret_cast<const double2*>(src);
  }
}

// Sums the per-workgroup partials of every group in a fixed order, writes
// the cost, publishes the evaluation status and re-arms the status word
// for the next evaluation (replaces thrust::reduce + the abort-flag round
// trip, autodiff_residual_block_cuda_evaluator.h:241-265).
__global__ __launch_bounds__(1024) void FinalizeKernel(const double* partials, int64_t n,
                                                       double* cost, int* status,
                                                       int* status_out) {
  __shared__ double wsum[1024 / kWave];
  // Four independent accumulators per thread keep several loads in flight.
  double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
  const int64_t step = blockDim.x;
  int64_t k = threadIdx.x;
  for (; k + 3 * step < n; k += 4 * step) {
    v0 += partials[k];
    v1 += partials[k + step];
    v2 += partials[k + 2 * step];
    v3 += partials[k + 3 * step];
  }
  for (; k < n; k += step) v0 += partials[k];
  double v = (v0 + v1) + (v2 + v3);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  if ((threadIdx.x & (kWave - 1)) == 0) wsum[threadIdx.x / kWave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < (int)(blockDim.x / kWave); ++w) t += wsum[w];
    const int s = *status;
    *cost = s ? 0.0 : t;
    *status_out = s;
    *status = 0;
  }
}

// Many partials, one launch: workgroup b sums partials [b*per, (b+1)*per)
// in a fixed order and hands its sum over to
// whichever workgroup finishes last, which adds the G slice sums in slice
// order and finalises as FinalizeKernel does -- the same value, bit for bit,
// as a slice pass followed by FinalizeKernel over the 128 slice sums.  Hand-over (MI355X_MICROARCH.md, valid
// forms: one lane per storing workgroup, agent-scope atomic add, the last
// adder told by the returned value): the slice sum is stored write-through
// (sc1) and drained (vmcnt(0)) before the add; the last workgroup reads the
// sums with sc1 loads only after its add has returned.  The counter is left
// at 0 for the next launch.
__global__ __launch_bounds__(kBlockThreads) void ReduceFinalizeKernel(
    const double* partials, int64_t n, int64_t per, double* slices, int* counter, double* cost,
    int* status, int* status_out) {
  __shared__ double lds_sum[kWavesPerBlock];
  __shared__ int last;
  const int64_t begin = (int64_t)blockIdx.x * per;
  const int64_t end = begin + per < n ? begin + per : n;
  // The slice's values in the same order as one load per step, but eight
  // loads in flight at a time (a dependent load per add cost ~0.5 us each:
  // 7 us for the 14 per thread of problem-13682's 452,931 partials).
  double v = 0.0;
  int64_t k = begin + threadIdx.x;
  for (; k + 7 * kBlockThreads < end; k += 8 * kBlockThreads) {
    double x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = partials[k + u * kBlockThreads];
#pragma unroll
    for (int u = 0; u < 8; ++u) v += x[u];
  }
  for (; k < end; k += kBlockThreads) v += partials[k];
  const double t = WorkgroupSum(v, lds_sum);
  if (threadIdx.x == 0) {
    double* dst = slices + blockIdx.x;
    asm volatile("global_store_dwordx2 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" ::"v"(dst), "v"(t)
                 : "memory");
    const int old = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == (int)gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  double s = 0.0;
  if (threadIdx.x < gridDim.x) {
    const double* src = slices + threadIdx.x;
    asm volatile("global_load_dwordx2 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(s) : "v"(src)
                 : "memory");
  }
  __syncthreads();  // lds_sum is reused
  const double total = WorkgroupSum(s, lds_sum);
  if (threadIdx.x == 0) {
    const int st = *status;
    *cost = st ? 0.0 : total;
    *status_out = st;
    *status = 0;
    *counter = 0;
  }
}

// Copies slot-0 parameter blocks [lo, lo + count) of the state into the
// packed table (once per evaluation: 13,682 cameras = 1.1 MB for BAL
// problem-13682), one 16-byte piece per thread: the first `pieces` pieces of
// each row of `stride` doubles (the LDS-DMA gather reads no others).
// With src_off (groups with constant slot-0 blocks): row b comes from
// state + src_off[b] (active) or cstate + (-1 - src_off[b]) (constant).
__global__ __launch_bounds__(256) void RepackSlot0Kernel(const double* state, int64_t state_base,
                                                         int size, int stride, int pieces, int32_t lo,
                                                         int64_t count, double* packed,
                                                         const int64_t* src_off, const double* cstate) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t b = t / pieces;
  const int k = 2 * (int)(t - b * pieces);
  if (b >= count) return;
  const double* src;
  if (src_off) {
    const int64_t o = src_off[b];
    src = o >= 0 ? state + o : cstate + (-1 - o);
  } else {
    src = state + state_base + (int64_t)size * (lo + b);
  }
  const double x = src[k];
  // The padding double of an odd-sized row marks a constant block (1.0):
  // the constant-aware kernels read it with the row (AffineInputs::x0pad).
  const double y = k + 1 < size ? src[k + 1] : (src_off && src_off[b] < 0 ? 1.0 : 0.0);
  *reinterpret_cast<double2*>(packed + (int64_t)stride * b + k) = make_double2(x, y);
}

}  // namespace cse

#endif  // CSE_OPERATOR_KERNELS_HPP_
