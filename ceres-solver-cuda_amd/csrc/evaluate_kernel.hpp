// evaluate_kernel.hpp -- the fused residual/Jacobian/loss/cost kernels.
//
// One wavefront lane owns one residual block (the reference's
// EvaluateKernel, include/ceres/internal/cuda_evaluator_kernel.h:297-422,
// also maps one thread to one block).  Per lane, fused in one pass:
//   gather parameters -> Jet autodiff of the functor -> plus-Jacobian
//   product (manifolds) -> loss rho(|r|^2) and Corrector on J then r ->
//   residual/Jacobian stores -> gradient J^T r -> the wave's cost partial
//   (summed deterministically by FinalizeKernel).
//
// Two layout policies, chosen per residual group on the host:
//   affine  table-free: block i of the group writes its residuals at
//           res_base + kR*i and row k of slot j at jac_base[j][k] +
//           jac_stride[j]*i, and reads parameter block `id` of slot j at
//           state_base[j] + size_j*id.  This is what BlockJacobianWriter and
//           CompressedRowJacobianWriter produce for Schur-ordered BAL
//           problems.  Kernel: EvaluateAffineChunks (the hot path).
//   table   the reference's offset tables (residual_layout,
//           jacobian_per_residual_layout/offsets, per-block parameter-block
//           records): any layout, constant blocks, manifolds, any number of
//           parameter blocks per residual.  Kernel: EvaluateTableKernel.
#ifndef CSE_EVALUATE_KERNEL_HPP_
#define CSE_EVALUATE_KERNEL_HPP_

#include <type_traits>

#include "kernel_common.hpp"

namespace cse {

// Stage one wave's outputs in LDS and write each contiguous segment (the
// slow tail: a partial last chunk or unaligned segments).  The wave's
// blocks [i0, i0 + nw) are contiguous in every segment:
//   residuals: [res_base + kR*i0, + kR*nw)
//   kCrs = false (BlockSparseMatrix): slot j's packed cells at
//       [jac_base[j][0] + stride_j*i0, + kR*size_j*nw)
//   kCrs = true (CompressedRowSparseMatrix): whole blocks, kR rows of N
//       columns, at [row0 + kR*N*i0, + kR*N*nw)
//   kHalves (CRS): the rows staged and written for lanes [0, 32), then for
//       lanes [32, 64), through half the LDS.
//   kConst0 (BlockSparseMatrix): lanes with a constant slot-0 block (act0
//       false) have no F cell; the others' cells are packed in lane order from
//       fbase[c] (chunk c).
//       (Held-camera chunks staged here write their whole segment, head and
//       tail included; HeldSectorFixupKernel leaves those bytes alone.)
template <class K, bool kJac, bool kCrs, bool kHalves = false, bool kConst0 = false>
__device__ __forceinline__ void StageAndStore(const GroupArgs& a, double* st, int lane, bool active,
                                              int64_t i0, int nw, const double* r,
                                              const double* J0, const double* J1,
                                              bool act0 = true, int64_t c = 0) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, NB = Tr::NB, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p;
  constexpr int N = S0 + S1;
  if (nw <= 0) return;
  if (a.residuals && active) {
    double* dst = a.residuals + a.res_base + (int64_t)NR * (i0 + lane);
#pragma unroll
    for (int k = 0; k < NR; ++k) __builtin_nontemporal_store(r[k], dst + k);
  }
  if constexpr (kJac) {
    if (!a.jacobian) return;
    if constexpr (kCrs && kConst0) {
      // Held cameras, CompressedRowSparseMatrix: the chunk's row blocks are
      // packed from fbase[c] (NR x N with an active camera, NR x S1 with a
      // held one); each lane writes its own (the slow tail: ragged or
      // unaligned chunks), past the head a previous sector-aligned wave wrote.
      static_assert(NB == 2, "two slots");
      const uint64_t m_any = __ballot(active), m_act = __ballot(active && act0);
      auto below = [&](uint64_t mm) {
        return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32),
                                              __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
      };
      const int ob = NR * S1 * below(m_any) + NR * S0 * below(m_act);
      constexpr int skip = 0;
      if (active) {
        double* seg = a.jacobian + a.fbase[c];
        const int64_t row0 = a.jac_base[0][0] < a.jac_base[1][0] ? a.jac_base[0][0] : a.jac_base[1][0];
        const int camcol = (int)(a.jac_base[0][0] - row0), ptcol = (int)(a.jac_base[1][0] - row0);
        if (act0) {
#pragma unroll
          for (int k = 0; k < NR; ++k) {
#pragma unroll
            for (int cc = 0; cc < S0; ++cc) {
              const int o = ob + k * N + camcol + cc;
              if (o >= skip) seg[o] = J0[k * S0 + cc];
            }
#pragma unroll
            for (int cc = 0; cc < S1; ++cc) {
              const int o = ob + k * N + ptcol + cc;
              if (o >= skip) seg[o] = J1[k * S1p + cc];
            }
          }
        } else {
#pragma unroll
          for (int k = 0; k < NR; ++k)
#pragma unroll
            for (int cc = 0; cc < S1; ++cc) {
              const int o = ob + k * S1 + cc;
              if (o >= skip) seg[o] = J1[k * S1p + cc];
            }
        }
      }
    } else if constexpr (kCrs) {
      const int64_t row0 = a.jac_base[0][0] < a.jac_base[NB - 1][0] ? a.jac_base[0][0]
                                                                      : a.jac_base[NB - 1][0];
      constexpr int kParts = kHalves ? 2 : 1, kLanes = kWave / kParts;
#pragma unroll
      for (int h = 0; h < kParts; ++h) {
        const int lo = h * kLanes;
        const int cnt = nw - lo < kLanes ? nw - lo : kLanes;
        if (cnt <= 0) break;
        if (active && lane >= lo && lane < lo + kLanes) {
          double* row = st + (lane - lo) * NR * N;
#pragma unroll
          for (int k = 0; k < NR; ++k) {
            const int c0 = (int)(a.jac_base[0][k] - row0);
#pragma unroll
            for (int c = 0; c < S0; ++c) row[c0 + c] = J0[k * S0 + c];
            if constexpr (S1 > 0) {
              const int c1 = (int)(a.jac_base[1][k] - row0);
#pragma unroll
              for (int c = 0; c < S1; ++c) row[c1 + c] = J1[k * S1p + c];
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
        WaveStore(st, a.jacobian + row0 + (int64_t)NR * N * (i0 + lo), cnt * NR * N, lane);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
      }
    } else {
      // Two rounds through the same LDS (slot 0's cells, then slot 1's): the
      // fast tail may size the staging buffer for slot 0 alone.
      if constexpr (kConst0) {
        const uint64_t m = __ballot(active && act0);
        const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (active && act0) {
#pragma unroll
          for (int q = 0; q < NR * S0; ++q) st[rank * NR * S0 + q] = J0[q];
        }
        __builtin_amdgcn_wave_barrier();
        WaveStore(st, a.jacobian + a.fbase[c], __popcll(m) * NR * S0, lane);
      } else {
        if (active) {
#pragma unroll
          for (int q = 0; q < NR * S0; ++q) st[lane * NR * S0 + q] = J0[q];
        }
        __builtin_amdgcn_wave_barrier();
        WaveStore(st, a.jacobian + a.jac_base[0][0] + a.jac_stride[0] * i0, nw * NR * S0, lane);
      }
      if constexpr (S1 > 0) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (active) {
#pragma unroll
          for (int q = 0; q < NR * S1; ++q) st[lane * NR * S1 + q] = J1[q];
        }
        __builtin_amdgcn_wave_barrier();
        WaveStore(st, a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * i0, nw * NR * S1, lane);
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// Gradient g += J^T r with device-scope FP64 atomics (native
// global_atomic_add_f64), as cuda_evaluator_kernel.h:149-160.  J is kR x
// kCols row-major; columns >= t are not added (tangent size).
template <int kR, int kCols>
__device__ __forceinline__ void AddGradientSlot(double* g, int t, const double* r, const double* J) {
#pragma unroll
  for (int c = 0; c < kCols; ++c) {
    if (c >= t) break;
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < kR; ++k) s += J[k * kCols + c] * r[k];
    unsafeAtomicAdd(g + c, s);
  }
}

// Inputs of one block (affine path).
template <class K>
struct AffineInputs {
  double d[KindTraits<K>::D];
  double x0[KindTraits<K>::X0];  // ambient values
  double x0pad;                   // the repacked row's padding double (odd X0): 1.0 = constant
  double x1[KindTraits<K>::S1p];
  int32_t id0, id1;
};

template <class K>
__device__ __forceinline__ int2 LoadIds(const GroupArgs& a, int64_t i) {
  if constexpr (KindTraits<K>::NB == 2) {
    return *reinterpret_cast<const int2*>(a.ids + 2 * i);
  } else {
    return make_int2(a.ids[i], 0);
  }
}

// Functor data and slot 1 (the point): per-lane loads.  In Schur order
// consecutive blocks share points, so these coalesce.
template <class K, bool kNtLoads>
__device__ __forceinline__ void GatherDataAndSlot1(const GroupArgs& a, int64_t i, int2 id,
                                                   AffineInputs<K>* in) {
  using Tr = KindTraits<K>;
  constexpr int S1 = Tr::S1, D = Tr::D;
  if constexpr (kNtLoads) {
#pragma unroll
    for (int k = 0; k < D; ++k) in->d[k] = __builtin_nontemporal_load(a.data + i * D + k);
  } else if constexpr (D == 2) {
    const double2 v = *reinterpret_cast<const double2*>(a.data + 2 * i);
    in->d[0] = v.x;
    in->d[1] = v.y;
  } else {
#pragma unroll
    for (int k = 0; k < D; ++k) in->d[k] = a.data[i * D + k];
  }
  if constexpr (S1 > 0) {
    const double* p1 = a.state + a.state_base[1] + (int64_t)S1 * id.y;
#pragma unroll
    for (int k = 0; k < S1; ++k) in->x1[k] = kNtLoads ? __builtin_nontemporal_load(p1 + k) : p1[k];
  }
}

// Slot 0 (the camera) loaded wave-cooperatively from the state: the wave's
// 64 parameter blocks are fetched as 64*S0 consecutive 8-byte pieces, piece
// p by lane p % 64 of load p / 64, so each load instruction walks the bytes
// of a few whole blocks (~8 cache lines) instead of 64 scattered lines;
// then the pieces are redistributed through LDS (lds: 64*S0 doubles of
// this wave).  Used when the slot-0 id range is too large for the repacked
// table of GatherCoopDma.
template <class K>
__device__ __forceinline__ void GatherCoop(const GroupArgs& a, int64_t i, int2 id,
                                           AffineInputs<K>* in, double* lds, int lane) {
  constexpr int X0 = KindTraits<K>::X0;
  GatherDataAndSlot1<K, false>(a, i, id, in);
  const double* base0 = a.state + a.state_base[0];
  double piece[X0];
#pragma unroll
  for (int k = 0; k < X0; ++k) {
    const int p = k * kWave + lane;
    const int t = p / X0, q = p - t * X0;
    const int cid = __shfl(id.x, t, kWave);
    piece[k] = base0[(int64_t)X0 * cid + q];
  }
#pragma unroll
  for (int k = 0; k < X0; ++k) lds[k * kWave + lane] = piece[k];
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < X0; ++k) in->x0[k] = lds[lane * X0 + k];
  __builtin_amdgcn_wave_barrier();
  in->id0 = id.x;
  in->id1 = id.y;
}

// The same with slot 0 fetched by LDS-DMA (global_load_lds_dwordx4) from
// the line-aligned repacked table: piece p (16 B) of the wave's 64
// blocks by lane p % 64 of load p / 64; the hardware writes each lane's
// 16 B at lds + 16 * p, so the pieces land in block order without passing
// through VGPRs.  The once-read streams (ids, observations, points) load
// non-temporally (-1.3 %, profiles/r02).
template <class K>
__device__ __forceinline__ void GatherCoopDma(const GroupArgs& a, int64_t i, int2 id,
                                              AffineInputs<K>* in, double* lds, int lane) {
  using Tr = KindTraits<K>;
  constexpr int X0 = Tr::X0;
  constexpr int X0p = (X0 + 1) & ~1;  // doubles per block in the packed table
  constexpr int kPieces = X0p / 2;    // 16-byte pieces per block
  constexpr int kRow = PackedRowDoubles(X0);
  const int cid_own = id.x - a.packed0_lo;
#pragma unroll
  for (int k = 0; k < kPieces; ++k) {
    const int p = k * kWave + lane;
    const int t = p / kPieces, q = p - t * kPieces;
    const int cid = __shfl(cid_own, t, kWave);
    const double* src = a.packed0 + (int64_t)kRow * cid + 2 * q;
    __builtin_amdgcn_global_load_lds(src, lds + 2 * kWave * k, 16, 0, 0);
  }
  GatherDataAndSlot1<K, true>(a, i, id, in);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < X0; ++k) in->x0[k] = lds[lane * X0p + k];
  if constexpr (X0 < X0p) in->x0pad = lds[lane * X0p + X0];
  __builtin_amdgcn_wave_barrier();
  in->id0 = id.x;
  in->id1 = id.y;
}

// The same with the observation load issued before the ids are waited for
// (the residual-only and cost-only kernels).
template <class K>
__device__ __forceinline__ void GatherEarly(const GroupArgs& a, int64_t i, int2 id,
                                            AffineInputs<K>* in, double* lds, int lane) {
  using Tr = KindTraits<K>;
  constexpr int X0 = Tr::X0, S1 = Tr::S1, D = Tr::D;
  constexpr int X0p = (X0 + 1) & ~1;
  constexpr int kPieces = X0p / 2;
  static_assert(D == 2, "observation pairs");
  const double obs_x = __builtin_nontemporal_load(a.data + 2 * i);
  const double obs_y = __builtin_nontemporal_load(a.data + 2 * i + 1);
  const int cid_own = id.x - a.packed0_lo;
#pragma unroll
  for (int k = 0; k < kPieces; ++k) {
    const int p = k * kWave + lane;
    const int t = p / kPieces, q = p - t * kPieces;
    const int cid = __shfl(cid_own, t, kWave);
    const double* src = a.packed0 + (int64_t)PackedRowDoubles(X0) * cid + 2 * q;
    __builtin_amdgcn_global_load_lds(src, lds + 2 * kWave * k, 16, 0, 0);
  }
  if constexpr (S1 > 0) {
    const double* p1 = a.state + a.state_base[1] + (int64_t)S1 * id.y;
#pragma unroll
    for (int k = 0; k < S1; ++k) in->x1[k] = __builtin_nontemporal_load(p1 + k);
  }
  in->d[0] = obs_x;
  in->d[1] = obs_y;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < X0; ++k) in->x0[k] = lds[lane * X0p + k];
  __builtin_amdgcn_wave_barrier();
  in->id0 = id.x;
  in->id1 = id.y;
}

// Segmented inclusive scan over the wave's lanes, fixed order (Hillis-
// Steele).  Keys are non-decreasing across lanes, so key[l - off] == key[l]
// means the whole range between is one run; afterwards each run's last lane
// holds the run's sum.
template <int S>
__device__ __forceinline__ void SegmentedScan(double* v, int key, int lane) {
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const int ku = __shfl_up(key, off, kWave);
    double vu[S];
#pragma unroll
    for (int c = 0; c < S; ++c) vu[c] = __shfl_up(v[c], off, kWave);
    if (lane >= off && ku == key) {
#pragma unroll
      for (int c = 0; c < S; ++c) v[c] += vu[c];
    }
  }
}

// The fused gradient of one wave (EvaluateAffineChunksFused): the
// deterministic replacement of the reference's in-kernel atomics
// (cuda_evaluator_kernel.h:149-160, 189-217) for Schur-ordered groups.
//   Slot 1 (points): the group's blocks are sorted by their slot-1 id, so a
//   parameter block's blocks are one run of lanes.  SegmentedScan leaves
//   the run's J1^T r in its last lane.  A run that touches neither end of
//   the wave is this wave's alone: stored straight into the gradient (the
//   host grants the group exclusive ownership of its slot-1 blocks).  The
//   wave's first and last runs may continue in the neighbouring waves: they
//   go to two boundary entries per wave (sum, id), which
//   GradientBoundaryKernel adds up in wave order.  A one-run wave writes
//   its run to entry 2c and a zero to entry 2c + 1 (same id).
//   Slot 0 (cameras, random order): each block's J0^T r, padded to S0p
//   doubles, in block order, for GradientContribKernel.
template <class K>
struct FusedGrad {
  static constexpr int S0 = KindTraits<K>::S0, S1 = KindTraits<K>::S1;
  static constexpr int S0p = (S0 + 1) & ~1;
  double g0[S0p];
  double g1[4];  // S1 == 3 sums, then the id (exact as a double)
  bool interior = false, writer = false, run_end = false;
  int64_t entry = 0;
  int key = 0;

  __device__ __forceinline__ void Compute(const double* r, const double* J0, const double* J1,
                                          int id1, bool active, int lane, int nw, int64_t c) {
    using Tr = KindTraits<K>;
    constexpr int NR = Tr::NR;
#pragma unroll
    for (int cc = 0; cc < S0p; ++cc) {
      double s = 0.0;
      if (cc < S0) {
#pragma unroll
        for (int k = 0; k < NR; ++k) s += J0[k * S0 + cc] * r[k];
      }
      g0[cc] = s;
    }
    ComputePoints(r, J1, id1, active, lane, nw, c);
  }

  // The slot-1 (point) part alone (g0 untouched).
  __device__ __forceinline__ void ComputePoints(const double* r, const double* J1, int id1, bool active,
                                                int lane, int nw, int64_t c) {
    using Tr = KindTraits<K>;
    constexpr int NR = Tr::NR, S1p = Tr::S1p;
    static_assert(Tr::NB == 2 && S1 == 3, "fused gradient: two slots, the second of size 3");
#pragma unroll
    for (int cc = 0; cc < S1; ++cc) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < NR; ++k) s += J1[k * S1p + cc] * r[k];
      g1[cc] = active ? s : 0.0;
    }
    key = active ? id1 : 0x7fffffff;
    SegmentedScan<S1>(g1, key, lane);
    const int knext = __shfl_down(key, 1, kWave);
    run_end = active && (lane == nw - 1 || (lane < nw - 1 && knext != key));
    const int k0 = __shfl(key, 0, kWave);
    const int kl = __shfl(key, nw - 1, kWave);
    const bool single = k0 == kl;
    const bool zero_entry = single && lane == 0 && nw > 1;
    interior = active && run_end && key != k0 && key != kl;
    writer = active && ((run_end && key == k0) || lane == nw - 1 || zero_entry);
    entry = 2 * c + (single ? (zero_entry ? 1 : 0) : (lane == nw - 1 ? 1 : 0));
    if (zero_entry) g1[0] = g1[1] = g1[2] = 0.0;
    g1[3] = (double)key;
  }
};

// Waves per CU of the one-wave Jacobian kernels, capped through their LDS
// footprint (doubles a lane; 0 = no cap).  BSM: 20 (10 KiB, 16 waves per
// CU).  With the by-hand Snavely functor the kernel needs only 92 VGPRs and
// could keep 17 waves per CU resident (LDS-bound); how many should depends on
// how the resident waves' three output streams (F cells, E cells, residuals)
// interleave.  With the tail storing F, E, residuals: 1.400 ms at 12 waves
// per CU, 1.44 at 13-14, 1.50 at 16, 1.525 at 17 (profiles/round4/r4occ,
// r4occ2, r4s7; the Jet kernel 1.427 at 16).  Storing E first (E, F,
// residuals; ShippedTune's order 2): 1.346-1.354 at 12, 1.326-1.336 at 14,
// 1.314-1.321 at 16 (r4ord2), and 16 ahead of 15 and 17 on another box
// (r4ord3).  CRS (one output stream) is fastest uncapped (20 waves per CU).
constexpr int kStageMinLane = 20;
constexpr int kStageMinLaneCrs = 0;
// The fused gradient's points kernel (94 VGPRs by hand): capped at 16 waves
// per CU like the Jet kernel's register bound (uncapped, 17, the gradient
// evaluation took 2.157-2.163 ms against 2.119-2.124 for the Jet build,
// profiles/round4/r4grad2; capped at 16, 2.126-2.133 against 2.124-2.131,
// r4s7).
constexpr int kStageMinLaneFp = 20;
// The held-camera tail stores its E cells before its F window (held
// evaluation 1.435-1.439 against 1.462-1.471 ms with E after F, the unheld
// evaluation 1.425-1.427 on that box; profiles/round4/r4held5).
// The held-camera BSM kernel likewise: 1.444-1.447 ms capped at 12 against
// 1.51-1.54 uncapped (16 per CU; profiles/round4/r4s8).
// The residual-only and cost-only kernels (8 waves per SIMD, 60 VGPRs) are
// fastest uncapped: capped at 24 waves per CU alike, at 16 7-15 % slower
// (profiles/round4/r4res).
constexpr int kStageMinLaneRes = 0;
constexpr int kStageMinLaneC0 = 26;

// Can the wave take the back-to-back store tail?  Full chunk, 16-byte
// pieces that tile every segment exactly, 16-byte-aligned destinations.
template <class K, bool kJac, bool kCrs, bool kConst0 = false>
__device__ __forceinline__ bool FastTail(const GroupArgs& a, int64_t i0, int nw, int64_t c = 0) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, N = S0 + S1;
  if (nw != kWave) return false;
  if constexpr (NR % 2 != 0) return false;
  if constexpr (kJac) {
    if constexpr (kCrs) {
      if ((NR * N) % 2 != 0) return false;
    } else {
      if ((NR * S0) % 2 != 0 || (NR * S1) % 2 != 0) return false;
    }
  }
  uintptr_t m = 0;
  if (a.residuals) m |= reinterpret_cast<uintptr_t>(a.residuals + a.res_base + (int64_t)NR * i0);
  if (kJac && a.jacobian) {
    if constexpr (kCrs) {
      const int64_t row0 = a.jac_base[0][0] < a.jac_base[Tr::NB - 1][0] ? a.jac_base[0][0]
                                                                         : a.jac_base[Tr::NB - 1][0];
      m |= reinterpret_cast<uintptr_t>(a.jacobian + row0 + (int64_t)NR * N * i0);
    } else {
      m |= reinterpret_cast<uintptr_t>(
          a.jacobian + (kConst0 ? a.fbase[c] : a.jac_base[0][0] + a.jac_stride[0] * i0));
      if constexpr (S1 > 0)
        m |= reinterpret_cast<uintptr_t>(a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * i0);
    }
  }
  return (m & 15) == 0;
}

// Sector-aligned store windows.  A wave's output segment of kQ wave
// instructions (kQ * 64 pieces of 16 bytes) starts at some byte S; when S is
// not on a 64-byte HBM sector boundary (the BlockSparseMatrix F cells start
// at 6 * num_blocks doubles, so this depends on the block count), every 1 KiB
// store instruction would begin and end inside a sector, and each of its two
// partial sectors leaves the streaming L2 path as a separate masked write:
// the kernel then ran at 0.45 instead of 0.60-0.65 of 8 TB/s
// (profiles/round2/s3n/fracs.txt: bimodal in block count mod 4).  So the
// pieces are regrouped: the first hp pieces (hp = pieces to the next sector
// boundary, 0..3) and the last 4 - hp are the segment's partial sectors,
// stored by lanes 60..63 of the last instruction; every other instruction
// writes 1 KiB of whole sectors, starting hp pieces into the segment.  With
// hp = 0 this is the plain in-order tiling.
// kA: the alignment unit in bytes (64: an HBM sector; 128: an L2 line).
template <int kA = 64>
__device__ __forceinline__ int SectorHeadPieces(const double* seg) {
  constexpr uint32_t m = kA - 1;
  return (int)(((kA - ((uint32_t)reinterpret_cast<uintptr_t>(seg) & m)) & m) >> 4);
}
// Piece of the segment that `lane` stores in the last instruction.
template <int kQ, int kA = 64>
__device__ __forceinline__ int LastPiece(int lane, int hp) {
  constexpr int kEdge = kA / 16;  // lanes carrying the head and tail pieces
  const int k = lane - (kWave - kEdge);
  return k < 0 ? (kQ - 1) * kWave + lane + hp : (k < hp ? k : kQ * kWave - kEdge + k);
}
// The kQ pieces this lane stores, read back from the wave's staged segment.
template <int kQ, int kA = 64>
__device__ __forceinline__ void ReadSegmentPieces(const double* staged, int hp, int lane,
                                                  cse_v4i* q) {
  const double2* st2 = reinterpret_cast<const double2*>(staged);
#pragma unroll
  for (int j = 0; j < kQ - 1; ++j) {
    const double2 v = st2[j * kWave + lane + hp];
    q[j] = AsV4i(v.x, v.y);
  }
  const double2 v = st2[LastPiece<kQ, kA>(lane, hp)];
  q[kQ - 1] = AsV4i(v.x, v.y);
}
// The same for a segment staged in parts: only the pieces in [lo, hi) are
// read, from staged + 16 * (piece - lo) bytes (the others keep their value).
template <int kQ, int kA = 64>
__device__ __forceinline__ void ReadSegmentPiecesRange(const double* staged, int hp, int lane,
                                                       int lo, int hi, cse_v4i* q) {
  const double2* st2 = reinterpret_cast<const double2*>(staged);
#pragma unroll
  for (int j = 0; j < kQ; ++j) {
    const int p = j < kQ - 1 ? j * kWave + lane + hp : LastPiece<kQ, kA>(lane, hp);
    if (p >= lo && p < hi) {
      const double2 v = st2[p - lo];
      q[j] = AsV4i(v.x, v.y);
    }
  }
}

// Held-camera groups (Tune::kConst0): may full chunks take the sector-aligned
// tail?  The residual, E-cell and F-cell bases 16-byte aligned (the chunk
// segments then start on 64-byte sectors when the bases do).
// fb_first: a.fbase[0].
// The one test, on the host (whether HeldSectorFixupKernel must run after
// the kernel, cse_evaluator.hip) and in the kernel (whether full chunks take
// the sector-window tail), so the two can never disagree.
CSE_HD bool HeldWindowsAligned(const double* residuals, int64_t res_base, const double* jacobian,
                                      int64_t e_base, int64_t f_first) {
  uintptr_t m = 0;
  if (residuals) m |= reinterpret_cast<uintptr_t>(residuals + res_base);
  if (jacobian)
    m |= reinterpret_cast<uintptr_t>(jacobian + e_base) | reinterpret_cast<uintptr_t>(jacobian + f_first);
  return (m & 15) == 0;
}
__device__ __forceinline__ bool C0Aligned(const GroupArgs& a, int64_t fb_first) {
  return HeldWindowsAligned(a.residuals, a.res_base, a.jacobian, a.jac_base[1][0], fb_first);
}

// Pieces kJ.. of a wave segment as SegmentStoresFrom, lane `lane` of
// instruction j storing only when its piece j * 64 + lane is below P.
template <int kJ, int kCount>
__device__ __forceinline__ void SegmentStoresMasked(double* b0, double* b1, const cse_v4i* q, int lane,
                                                    int P) {
  if constexpr (kJ < kCount) {
    if (kJ * kWave + lane < P) StoreNt16<(kJ % 8) * 1024 - 4096>(kJ < 8 ? b0 : b1, q[kJ]);
    SegmentStoresMasked<kJ + 1, kCount>(b0, b1, q, lane, P);
  }
}

// Compile-time settings of the affine kernel (the four the product ships,
// below).  Measured alternatives of rounds 2-5 -- wave priorities, E cells
// from registers, one-round staging, LDS occupancy caps, 128-byte windows,
// early observation loads, register gathers, other table strides, own-row
// DMA, store cache policies, XCD-contiguous chunks, scalar id loads --
// were slower and are not in the tree (git history before
// round 6).
//   kOrder  the store tail's order: 0 F, E, residuals; 1 residuals, E, F;
//           2 E, F, residuals.
//   kNoContrib  fused gradient without the slot-0 contributions (the slot-0
//           sums come from CameraGradientKernel instead).
//   kConst0 the group has constant slot-0 blocks (BSM: their F cells are
//           packed, fbase).
template <int kOrder_, bool kNoContrib_ = false, bool kConst0_ = false>
struct Tune {
  static constexpr int kOrder = kOrder_;
  static constexpr bool kNoContrib = kNoContrib_;
  static constexpr bool kConst0 = kConst0_;
};

// Shipped: no priority changes (kPrio 2 was 1.5-2 % faster with the library
// sincos and divisions, profiles/round2/s1, s3c, and 2 % slower once the
// functor's FP64 work shrank, s3d); two-round E/F staging (9 KiB of LDS a
// wave), which with the kernel held to 128 VGPRs gives 4 waves per SIMD
// instead of 3.  That was neutral with the heavier functor (s3i, s3j) and is
// 2.5 % faster with the series rotation (s4n).
// The store tail's segment order E, F, residuals (2): with the BSM kernel at
// 12 waves per CU, 1.369-1.373 ms against 1.397-1.398 for 0 and 1.369-1.377
// for 1; CRS neutral; profiles/round4/r4ord.
using ShippedTune = Tune<2>;
// The fused gradient's points-only form (CameraGradientKernel adds slot 0).
// Its store order: residuals, E, F (1) -- gradient evaluation 1.965-1.970
// ms against 2.017-2.026 for F, E, residuals (0) and 1.976-1.978 for E, F,
// residuals (2), same box (profiles/round4/r4fpord).
using PointsOnlyTune = Tune<1, true>;
// The same for groups with constant slot-0 blocks (a held camera): a wave
// with one takes the slow tail, its F cells packed from fbase[c]; waves
// without take the fast tail from fbase[c].
using ShippedTuneC0 = Tune<0, false, true>;
using PointsOnlyTuneC0 = Tune<0, true, true>;

// Does the shipped BSM Jacobian kernel of kind K stage in two rounds (and so
// fit 4 workgroups per CU)?
template <class K>
constexpr bool kTwoRoundBsm = KindTraits<K>::S1 > 0;

// The hot kernel: one 64-block chunk per wave, every output store issued
// back to back at the very end of the wave (see the store primitives in
// kernel_common.hpp for why).  Here: the wave's cost is reduced first
// (cross-lane, no barrier), the Jacobian is staged through LDS and read
// back as 16-byte pieces in segment order, and then every store is an
// inline-asm global_store_dwordx4 whose operands stay live to the end.
//   kCoop 2: slot 0 gathered by LDS-DMA from the repacked table;
//         1: 8-byte pieces straight from the state.
//   kGradF: the fused gradient (FusedGrad).
//   kWPB: waves per workgroup (chunk c = workgroup * kWPB + wave either way,
//         so the per-wave partials keep their slots and their order).
template <class K, int kLoss, bool kJac, bool kCrs, int kCoop, bool kGradF = false,
          class T = ShippedTune, int kWPB = kWavesPerBlock>
__device__ __forceinline__ void AffineChunkBody(const GroupArgs& a) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p, N = S0 + S1;
  static_assert(!MayLeaveOutputs<K>::value, "affine kernels: functors that assign every output");
  // BSM: the F cells staged and read back, then the E cells in the same LDS
  // (two rounds); CRS rows staged in two halves of the wave (lanes [0, 32),
  // then [32, 64)).
  constexpr bool kTwo = kJac && !kCrs && S1 > 0;
  constexpr bool kTwoCrs = kJac && kCrs;
  constexpr int kOutLane = kJac ? (kCrs ? (NR * N + 1) / 2
                                        : kTwo ? NR * (S0 > S1 ? S0 : S1) : NR * (S0 + S1))
                                : 1;
  constexpr int kCoopLane = kCoop == 2 ? ((Tr::X0 + 1) & ~1) : Tr::X0;
  // StageAndStore's footprint (ragged chunks): whole rows (CRS) or one
  // slot's cells at a time (BSM).
  constexpr int kSlowLane = !kJac ? 1 : kCrs ? (kTwoCrs ? (NR * N + 1) / 2 : NR * N) : NR * (S0 > S1 ? S0 : S1);
  // the fused gradient's slot-0 contributions (mode 3), staged after the cells
  constexpr int kContribLane = kGradF && !T::kNoContrib ? 2 * (FusedGrad<K>::S0p / 2) : 0;
  constexpr int kOutLane1 = kContribLane > kOutLane ? kContribLane : kOutLane;
  constexpr int kStageLane0 = kCoopLane > kOutLane1 ? kCoopLane : kOutLane1;
  constexpr int kStageLane1 = kSlowLane > kStageLane0 ? kSlowLane : kStageLane0;
  // The LDS cap on waves per CU (kStageMinLane, above), for the
  // by-hand Snavely kernels only (the Jet-based quaternion kernel is
  // register-bound at 16 waves per CU and slower capped: 1.516 vs 1.38 ms,
  // r4s9); the fused gradient's points kernel measured neutral to it (r4s7).
  constexpr bool kByHand = std::is_same<K, SnavelyKind>::value;
  constexpr int kPadLane = !kJac ? (std::is_same<K, SnavelyKind>::value ? kStageMinLaneRes : 0)
                          : kWPB != 1 || !kByHand ? 0
                          : T::kConst0 ? (kGradF || kCrs ? 0 : kStageMinLaneC0)
                          : kGradF ? kStageMinLaneFp
                          : kCrs ? kStageMinLaneCrs : kStageMinLane;
  constexpr int kStageLane = kPadLane > kStageLane1 ? kPadLane : kStageLane1;
  __shared__ double stage[kWPB][kWave * kStageLane];

  constexpr bool kC0J = T::kConst0 && kJac;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = kWPB == 1 ? 0 : threadIdx.x / kWave;
  const int64_t num_chunks = (a.n + kWave - 1) / kWave;
  const int64_t c = (int64_t)blockIdx.x * kWPB + wave;
  double* partial_dst = a.partials + c;
  if (c >= num_chunks) {
    if (lane == 0) *partial_dst = 0.0;  // the group's partial slots are 4 per workgroup
    return;
  }
  double* st = stage[wave];
  const int64_t i0 = c * kWave;
  const int64_t rem = a.n - i0;
  const int nw = rem < kWave ? (int)rem : kWave;
  const bool active = lane < nw;
  const int64_t i = active ? i0 + lane : a.n - 1;
  // Held-camera groups: the chunk's packed-F bounds and the group's, loaded
  // here, before the gather's memory-clobbering asm, so that the scalar
  // loads' latency is in neither the gather nor the store tail.
  int64_t fb[5] = {0, 0, 0, 0, 0};
  if constexpr (kC0J) {  // fbase is set for every held-camera group
    fb[0] = a.fbase[c];
    fb[1] = a.fbase[c + 1];
    fb[2] = a.fbase[0];
    fb[3] = a.fbase[num_chunks];
    fb[4] = a.fbase[c + 2 < num_chunks ? c + 2 : num_chunks];
  }

  AffineInputs<K> in;
  if constexpr (kCoop == 2) {
    int2 id;
    if constexpr (Tr::NB == 2) {
      const long long b = __builtin_nontemporal_load(reinterpret_cast<const long long*>(a.ids) + i);
      id = make_int2((int)b, (int)(b >> 32));
    } else {
      id = LoadIds<K>(a, i);
    }
    if constexpr (!kJac && Tr::D == 2 && Tr::NB == 2) {
      // Residual-only and cost-only evaluations issue the observation load
      // with the ids load (1.5-2 % faster, profiles/round2/s4h; the
      // Jacobian kernel is 4 % slower that way, s4c).
      GatherEarly<K>(a, i, id, &in, st, lane);
    } else {
      GatherCoopDma<K>(a, i, id, &in, st, lane);
    }
  } else {
    GatherCoop<K>(a, i, LoadIds<K>(a, i), &in, st, lane);
  }
  // The chunk bounds' first use, after the gather: their scalar loads were
  // issued before it and have long arrived (without the pin the compiler
  // compares them right away and waits for them before the gather starts).
  if constexpr (kC0J) {
    if constexpr (kWPB == 1)  // uniform: SGPRs
      asm volatile("" : "+s"(fb[0]), "+s"(fb[1]), "+s"(fb[2]), "+s"(fb[3]), "+s"(fb[4]));
    else  // the wave index is not known uniform to the compiler
      asm volatile("" : "+v"(fb[0]), "+v"(fb[1]), "+v"(fb[2]), "+v"(fb[3]), "+v"(fb[4]));
  }
  double r[NR], J0[NR * S0], J1[NR * S1p];
  bool ok = EvaluateFunctor<K, kJac>(in.d, in.x0, in.x1, r, J0, J1);
  if (ok && a.check_finite) {
    bool bad = AnyNonFinite<NR>(r);
    if constexpr (kJac) bad = bad || AnyNonFinite<NR * S0>(J0) || AnyNonFinite<NR * S1>(J1);
    ok = !bad;
  }
  const double cost =
      LossAndCorrect<K, kLoss, kJac>(a.loss, a.apply_loss, r, J0, J1, a.residuals != nullptr,
                                     a.user_loss);
  bool act0 = true;  // slot-0 block active (T::kConst0: from its bit)
  if constexpr (T::kConst0) {
    static_assert(kCoop == 2, "constant slot-0 blocks: the repacked table");
    if constexpr ((Tr::X0 & 1) != 0) {
      act0 = in.x0pad == 0.0;  // the flag came with the row (RepackSlot0Kernel)
    } else {
      const uint32_t k0 = (uint32_t)(in.id0 - a.packed0_lo);
      act0 = ((a.act0_bits[k0 >> 5] >> (k0 & 31)) & 1u) != 0;
    }
  }
  if (kJac && a.gradient != nullptr && active) {
    if (act0)
      AddGradientSlot<NR, S0>(a.gradient + (T::kConst0 ? a.delta0[in.id0 - a.packed0_lo]
                                                        : a.delta_base[0] + (int64_t)S0 * in.id0),
                              S0, r, J0);
    if constexpr (S1 > 0)
      AddGradientSlot<NR, S1p>(a.gradient + a.delta_base[1] + (int64_t)S1 * in.id1, S1, r, J1);
  }
  // The wave's cost (WaveSumLane0: a fixed order) and failure flag, before
  // any store is queued.
  const double wsum = WaveSumLane0(active ? cost : 0.0);
  const bool failed = __ballot(active && !ok) != 0;
  int* status_dst = a.status;
  static_assert(!kGradF || kJac, "fused gradient: Jacobian kernels only");
  FusedGrad<K> fg;
  if constexpr (kGradF) fg.Compute(r, J0, J1, in.id1, active, lane, nw, c);

  if constexpr (kC0J) {
    if (nw == kWave && C0Aligned(a, fb[2])) {
      // ---- held-camera groups, full chunk: whole-sector windows ----
      // After a held block the packed F cells (BSM) or row blocks (CRS) no
      // longer start on 64-byte sectors.  The wave stores only the whole
      // sectors of its segment, [W0, W1) = [A0 rounded up, A1 rounded down),
      // and its head and tail pieces (up to three of 16 B each) into its two
      // 64-byte side slots, one store; HeldSectorFixupKernel then writes each
      // sector shared by two waves in one piece.  The group's first and last
      // non-empty segments write their outer ends directly.
      static_assert(NR == 2 && S1 > 0, "held-camera tail: two-slot kinds, two residuals");
      constexpr int kF = NR * S0;  // doubles per F cell (BSM)
      // BlockSparseMatrix: the F window, then the E cells.  CompressedRow:
      // one window over the chunk's row blocks (NR x (S1 + S0) with an active
      // camera, NR x S1 with a held one), staged in two halves of the wave.
      constexpr int kSegPieces = kCrs ? kWave * NR * (S0 + S1) / 2 : kWave * kF / 2;
      constexpr int kQF = (kSegPieces + kWave - 1) / kWave;
      constexpr int kPE = kCrs ? 0 : kWave * NR * S1 / 2;  // E pieces of a chunk (BSM)
      constexpr int kQE = kCrs ? 1 : (kPE + kWave - 1) / kWave;
      constexpr int kLdsPieces = kWave * kStageLane / 2;
      static_assert(kQF <= 16, "window: one or two base registers");
      const bool jacw = a.jacobian != nullptr;
      cse_v4i qf[kQF], qe[kQE], qs;
      double* wf0 = nullptr;
      double* wf1 = nullptr;
      double* we0 = nullptr;
      double* ws = nullptr;
      int P = 0;
      bool whole = false;  // every F store unmasked (below)
      if (jacw) {
        const int64_t fb0 = fb[0], fb1 = fb[1];
        const uintptr_t A0 = reinterpret_cast<uintptr_t>(a.jacobian + fb0);
        const uintptr_t A1 = reinterpret_cast<uintptr_t>(a.jacobian + fb1);
        const bool first = fb0 == fb[2], last = fb1 == fb[3];
        const uintptr_t W0 = first ? A0 : ((A0 + 63) & ~(uintptr_t)63);
        const uintptr_t W1 = last ? A1 : (A1 & ~(uintptr_t)63);
        P = W1 > W0 ? (int)((W1 - W0) >> 4) : 0;
        const int off = (int)((W0 - A0) >> 4);            // head pieces (not stored here)
        const int npc = (int)((A1 - A0) >> 4);            // pieces of the segment
        const int tp = W1 > W0 ? (int)((A1 - W1) >> 4) : 0;  // tail pieces
        // A chunk without held blocks (npc = the whole staged segment) whose
        // next chunk is full and has F cells: its window's store
        // instructions run unmasked.  The lanes past the window then write
        // the tail pieces and, past A1, the next segment's head pieces in
        // the one sector the two share (P >= kQF * 64 - 4 here), which
        // HeldSectorFixupKernel rewrites whole after this kernel.  Masked
        // (exec-branched) stores made the held-camera kernel 15 % slower.
        whole = npc == kQF * kWave && !last && (c + 2) * kWave <= a.n && fb[4] > fb1;
        // Side slots: lanes 0-3 the head sector's pieces at their positions
        // (the head is its last `off` pieces), lanes 4-7 the tail sector's.
        int sp = lane < 4 ? lane - (4 - off) : npc - tp + (lane - 4);
        sp = sp < 0 ? 0 : (sp < npc ? sp : (npc > 0 ? npc - 1 : 0));
        const double2* st2 = reinterpret_cast<const double2*>(st);
        if constexpr (kCrs) {
          constexpr int N = S0 + S1;
          const uint64_t m_any = __ballot(active), m_act = __ballot(active && act0);
          auto below = [&](uint64_t mm) {
            return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32),
                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
          };
          // this lane's row block inside the chunk's segment (doubles)
          const int ob = NR * S1 * below(m_any) + NR * S0 * below(m_act);
          const int64_t row0 = a.jac_base[0][0] < a.jac_base[1][0] ? a.jac_base[0][0] : a.jac_base[1][0];
          const int camcol = (int)(a.jac_base[0][0] - row0), ptcol = (int)(a.jac_base[1][0] - row0);
          constexpr int kHalf = kWave / 2;
          const int split = __builtin_amdgcn_readlane(ob, kHalf);  // where lane kHalf's block starts
          const int total = 2 * npc;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int lo = h == 0 ? 0 : split, hi = h == 0 ? split : total;
            if (active && (h == 0 ? lane < kHalf : lane >= kHalf)) {
              double* blk = st + (ob - lo);
              if (act0) {
#pragma unroll
                for (int k = 0; k < NR; ++k) {
#pragma unroll
                  for (int cc = 0; cc < S0; ++cc) blk[k * N + camcol + cc] = J0[k * S0 + cc];
#pragma unroll
                  for (int cc = 0; cc < S1; ++cc) blk[k * N + ptcol + cc] = J1[k * S1p + cc];
                }
              } else {
#pragma unroll
                for (int k = 0; k < NR; ++k)
#pragma unroll
                  for (int cc = 0; cc < S1; ++cc) blk[k * S1 + cc] = J1[k * S1p + cc];
              }
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int j = 0; j < kQF; ++j) {
              const int o = 2 * (off + j * kWave + lane);  // segment offset, doubles (even)
              if (o >= lo && o < hi) {
                int p = (o - lo) >> 1;
                p = p < kLdsPieces ? p : kLdsPieces - 1;
                const double2 v = st2[p];
                qf[j] = AsV4i(v.x, v.y);
              }
            }
            if (2 * sp >= lo && 2 * sp < hi) {
              int p = sp - (lo >> 1);
              p = p < kLdsPieces ? p : kLdsPieces - 1;
              const double2 v = st2[p];
              qs = AsV4i(v.x, v.y);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
          }
        } else {
          const uint64_t m = __ballot(active && act0);
          const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          if (active && act0) {
#pragma unroll
            for (int q = 0; q < kF; ++q) st[rank * kF + q] = J0[q];
          }
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int j = 0; j < kQF; ++j) {
            int p = off + j * kWave + lane;
            p = p < kLdsPieces ? p : kLdsPieces - 1;
            const double2 v = st2[p];
            qf[j] = AsV4i(v.x, v.y);
          }
          {
            const double2 v = st2[sp < kLdsPieces ? sp : kLdsPieces - 1];
            qs = AsV4i(v.x, v.y);
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_wave_barrier();
          if (active) {
#pragma unroll
            for (int k = 0; k < NR; ++k)
#pragma unroll
              for (int cc = 0; cc < S1; ++cc) st[lane * NR * S1 + k * S1 + cc] = J1[k * S1p + cc];
          }
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int j = 0; j < kQE; ++j) {
            int p = j * kWave + lane;
            p = p < kPE ? p : kPE - 1;
            const double2 v = st2[p];
            qe[j] = AsV4i(v.x, v.y);
          }
          we0 = a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * i0 + 2 * lane + 512;
        }
        double* fw = reinterpret_cast<double*>(W0);
        wf0 = fw + 2 * lane + 512;
        wf1 = fw + 2 * lane + 1536;
        ws = a.side + 16 * c + 2 * lane;
      }
      const cse_v4i qr = AsV4i(r[0], r[1]);
      double* rdst = a.residuals ? a.residuals + a.res_base + (int64_t)NR * (i0 + lane) : nullptr;
      cse_v4i sq[2];
      double *gp = nullptr, *sp = nullptr;
      // gradient_mode 3: the slot-0 contributions J0^T r of the chunk's own
      // blocks (10 doubles each, block order), staged like the cells.
      constexpr bool kContribC0 = kGradF && !T::kNoContrib;
      constexpr int kGQ = kContribC0 ? FusedGrad<K>::S0p / 2 : 1;  // pieces per block
      constexpr int kPC = kWave * kGQ;
      constexpr int kQC = kContribC0 ? (kPC + kWave - 1) / kWave : 1;
      cse_v4i qc[kQC];
      double* cb0 = nullptr;
      if constexpr (kContribC0) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (active) {
#pragma unroll
          for (int j = 0; j < kGQ; ++j)
            reinterpret_cast<double2*>(st)[lane * kGQ + j] = make_double2(fg.g0[2 * j], fg.g0[2 * j + 1]);
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < kQC; ++j) {
          int p = j * kWave + lane;
          p = p < kPC ? p : kPC - 1;
          const double2 v = reinterpret_cast<const double2*>(st)[p];
          qc[j] = AsV4i(v.x, v.y);
        }
        cb0 = a.gcontrib + (int64_t)(2 * kGQ) * i0 + 2 * lane + 512;
      }
      if constexpr (kGradF) {
        sq[0] = AsV4i(fg.g1[0], fg.g1[1]);
        sq[1] = AsV4i(fg.g1[2], fg.g1[3]);
        gp = a.gfused + a.delta_base[1] + 3LL * fg.key;
        sp = a.gside + 4 * fg.entry;
      }
      double* v_partial = partial_dst;
      double v_wsum = wsum;
      asm volatile("" : "+v"(v_partial), "+v"(v_wsum));
      asm volatile("" ::"v"(wf0), "v"(wf1), "v"(we0), "v"(ws), "v"(rdst));
      auto store_g = [&]() {  // the fused gradient's stores (rows and entries exec-masked)
        if constexpr (kGradF) {
          if constexpr (kContribC0) SegmentStoresMasked<0, kQC>(cb0, cb0, qc, lane, kPC);
          if (fg.interior) {
            StoreB64At<0>(gp, fg.g1[0]);
            StoreB64At<8>(gp, fg.g1[1]);
            StoreB64At<16>(gp, fg.g1[2]);
          }
          if (fg.writer) {
            StoreNt16<0, 1>(sp, sq[0]);
            StoreNt16<16, 1>(sp, sq[1]);
          }
        }
      };
      // ---- every store of the wave ----
      // The side slots (8 lanes) first, then the unmasked window.  (The
      // fused gradient's masked stores ahead of the window measured
      // neutral, profiles/round4/r4s5.)
      if (jacw && lane < 8) StoreNt16<0, 1>(ws, qs);
      if (jacw) {
        if constexpr (!kCrs) SegmentStoresMasked<0, kQE>(we0, we0, qe, lane, kPE);
        if (whole)
          SegmentStoresMasked<0, kQF>(wf0, wf1, qf, 0, kQF * kWave);  // no lane masked
        else
          SegmentStoresMasked<0, kQF>(wf0, wf1, qf, lane, P);
      }
      if (a.residuals) StoreNt16<0>(rdst, qr);  // a full chunk: every lane active
      store_g();
      if (lane == 0) {
        StoreB64(v_partial, v_wsum);
        if (failed) StoreB32(status_dst, 1);
      }
      if constexpr (kContribC0) {
        KeepAlive<kQC>(qc);
        asm volatile("" ::"v"(cb0));
      }
      KeepAlive<kQF>(qf);
      KeepAlive<kQE>(qe);
      asm volatile("" ::"v"(qr), "v"(qs), "v"(ws), "v"(wf0), "v"(wf1), "v"(we0), "v"(rdst),
                   "v"(v_partial), "v"(v_wsum));
      if constexpr (kGradF) {
        KeepAlive<2>(sq);
        asm volatile("" ::"v"(gp), "v"(sp), "v"(fg.g1[0]), "v"(fg.g1[1]), "v"(fg.g1[2]));
      }
      return;
    }
  }
  bool fast = FastTail<K, kJac, kCrs, T::kConst0>(a, i0, nw, c);
  if constexpr (kC0J) fast = false;  // full aligned chunks returned above
  if (!fast) {
    StageAndStore<K, kJac, kCrs, kTwoCrs, T::kConst0>(a, st, lane, active, i0, nw, r, J0, J1, act0, c);
    if constexpr (kGradF) {
      // The group's last, partial chunk: plain stores.
      constexpr int S0p = FusedGrad<K>::S0p;
      if (!T::kNoContrib && active) {
        double* cdst = a.gcontrib + (int64_t)S0p * (i0 + lane);
#pragma unroll
        for (int cc = 0; cc < S0p; ++cc) cdst[cc] = fg.g0[cc];
      }
      if (fg.interior) {
        double* g = a.gfused + a.delta_base[1] + 3LL * fg.key;
        g[0] = fg.g1[0];
        g[1] = fg.g1[1];
        g[2] = fg.g1[2];
      }
      if (fg.writer) {
#pragma unroll
        for (int q = 0; q < 4; ++q) a.gside[4 * fg.entry + q] = fg.g1[q];
      }
      if (nw == 1 && lane == 0) {  // a one-block wave: its zero entry
        double* e = a.gside + 4 * (2 * c + 1);
        e[0] = e[1] = e[2] = 0.0;
        e[3] = fg.g1[3];
      }
    }
    if (lane == 0) {
      *partial_dst = wsum;
      if (failed) *status_dst = 1;
    }
    return;
  }

  // Stage the Jacobian, read it back as 16-byte pieces in segment order.
  constexpr int kQ0 = kJac ? (kCrs ? NR * N / 2 : NR * S0 / 2) : 0;  // pieces per lane, seg 0 (F)
  constexpr int kQ1 = (kJac && !kCrs && S1 > 0) ? NR * S1 / 2 : 0;   // seg 1 (E cells)
  const bool jac = kJac && a.jacobian != nullptr;
  cse_v4i q0[kQ0 > 0 ? kQ0 : 1], q1[kQ1 > 0 ? kQ1 : 1];
  double* seg0 = nullptr;
  double* seg1 = nullptr;
  int hp0 = 0, hp1 = 0;  // pieces to the first sector boundary (SectorHeadPieces)
  if constexpr (kJac) {
    if (jac) {
      if constexpr (kCrs) {
        const int64_t row0 = a.jac_base[0][0] < a.jac_base[Tr::NB - 1][0]
                                 ? a.jac_base[0][0]
                                 : a.jac_base[Tr::NB - 1][0];
        // Lane `lane`'s row block at `row` (kTwoCrs: the half-wave's rows).
        auto stage_rows = [&](double* row) {
#pragma unroll
          for (int k = 0; k < NR; ++k) {
            const int c0 = (int)(a.jac_base[0][k] - row0);
#pragma unroll
            for (int cc = 0; cc < S0; ++cc) row[c0 + cc] = J0[k * S0 + cc];
            if constexpr (S1 > 0) {
              const int c1 = (int)(a.jac_base[1][k] - row0);
#pragma unroll
              for (int cc = 0; cc < S1; ++cc) row[c1 + cc] = J1[k * S1p + cc];
            }
          }
        };
        seg0 = a.jacobian + row0 + (int64_t)NR * N * i0;
        if constexpr (kTwoCrs) {
          // Lanes [0, 32) stage their rows (the segment's first half), every
          // lane reads the pieces that fall in it; then lanes [32, 64) and
          // the second half, in the same LDS.  FastTail guarantees NR * N
          // even, so the halves split on a piece boundary.
          constexpr int kHalf = kWave / 2 * NR * N / 2;  // pieces per half
          hp0 = SectorHeadPieces(seg0);
          if (lane < kWave / 2) stage_rows(st + lane * NR * N);
          __builtin_amdgcn_wave_barrier();
          ReadSegmentPiecesRange<kQ0>(st, hp0, lane, 0, kHalf, q0);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_wave_barrier();
          if (lane >= kWave / 2) stage_rows(st + (lane - kWave / 2) * NR * N);
          __builtin_amdgcn_wave_barrier();
          ReadSegmentPiecesRange<kQ0>(st, hp0, lane, kHalf, 2 * kHalf, q0);
        } else {
          stage_rows(st + lane * NR * N);
        }
      } else {
        double* st1 = st + kWave * NR * S0;
#pragma unroll
        for (int p = 0; p < NR * S0; ++p) st[lane * NR * S0 + p] = J0[p];
        if constexpr (S1 > 0) {
          if constexpr (!kTwo) {
#pragma unroll
            for (int k = 0; k < NR; ++k)
#pragma unroll
              for (int cc = 0; cc < S1; ++cc) st1[lane * NR * S1 + k * S1 + cc] = J1[k * S1p + cc];
          }
          seg1 = a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * i0;
        }
        seg0 = a.jacobian + (T::kConst0 ? a.fbase[c] : a.jac_base[0][0] + a.jac_stride[0] * i0);
      }
      if constexpr (!kTwoCrs) {
        __builtin_amdgcn_wave_barrier();
        hp0 = SectorHeadPieces(seg0);
        ReadSegmentPieces<kQ0>(st, hp0, lane, q0);
      }
      if constexpr (kQ1 > 0) {
        hp1 = SectorHeadPieces(seg1);
        if constexpr (kTwo) {
          // Second round: the E cells in the LDS the F pieces came from.
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int k = 0; k < NR; ++k)
#pragma unroll
            for (int cc = 0; cc < S1; ++cc) st[lane * NR * S1 + k * S1 + cc] = J1[k * S1p + cc];
          __builtin_amdgcn_wave_barrier();
          ReadSegmentPieces<kQ1>(st, hp1, lane, q1);
        } else {
          ReadSegmentPieces<kQ1>(st + kWave * NR * S0, hp1, lane, q1);
        }
      }
    }
  }
  // Fused gradient: the slot-0 contributions staged through the same LDS
  // (after the Jacobian pieces have been read back), the slot-1 entry.
  constexpr bool kContrib = kGradF && !T::kNoContrib;
  constexpr int kGQ = kContrib ? FusedGrad<K>::S0p / 2 : 1;
  static_assert(kGQ <= 8, "contribution pieces: one base register");
  cse_v4i gq[kGQ], sq[2];
  double *cb0 = nullptr, *gp = nullptr, *sp = nullptr;
  if constexpr (kGradF) {
    sq[0] = AsV4i(fg.g1[0], fg.g1[1]);
    sq[1] = AsV4i(fg.g1[2], fg.g1[3]);
    gp = a.gfused + a.delta_base[1] + 3LL * fg.key;
    sp = a.gside + 4 * fg.entry;
  }
  if constexpr (kContrib) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < kGQ; ++j)
      reinterpret_cast<double2*>(st)[lane * kGQ + j] = make_double2(fg.g0[2 * j], fg.g0[2 * j + 1]);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < kGQ; ++j) {
      const double2 v = reinterpret_cast<const double2*>(st)[j * kWave + lane];
      gq[j] = AsV4i(v.x, v.y);
    }
    cb0 = a.gcontrib + (int64_t)(2 * kGQ) * i0 + 2 * lane + 512;
  }
  // Residual pieces: the lane's own NR doubles (NR even; FastTail sends
  // odd NR to the staged tail, the array only has to exist).
  constexpr int kQr = NR / 2;
  cse_v4i qr[kQr > 0 ? kQr : 1];
#pragma unroll
  for (int k = 0; k < kQr; ++k) qr[k] = AsV4i(r[2 * k], r[2 * k + 1]);
  double* rdst = a.residuals ? a.residuals + a.res_base + (int64_t)NR * (i0 + lane) : nullptr;

  // Every address and the wave's scalar outputs are computed (and pinned by
  // the empty asm) before the first store: after it the wave runs only
  // stores and SALU, so nothing waits on the store queue.
  double *f0 = nullptr, *f1 = nullptr, *e0 = nullptr, *e1 = nullptr;
  double *flast = nullptr, *elast = nullptr;
  if (jac) {
    f0 = seg0 + 2 * (lane + hp0) + 512;
    f1 = seg0 + 2 * (lane + hp0) + 1536;
    flast = seg0 + 2 * LastPiece<(kQ0 > 0 ? kQ0 : 1)>(lane, hp0);
    if constexpr (kQ1 > 0) {
      e0 = seg1 + 2 * (lane + hp1) + 512;
      e1 = seg1 + 2 * (lane + hp1) + 1536;
      elast = seg1 + 2 * LastPiece<kQ1>(lane, hp1);
    }
  }
  // The partial's address and value in VGPRs now, not after the tail.
  double* v_partial = partial_dst;
  double v_wsum = wsum;
  asm volatile("" : "+v"(v_partial), "+v"(v_wsum));
  asm volatile("" ::"v"(f0), "v"(f1), "v"(e0), "v"(e1), "v"(rdst), "v"(flast), "v"(elast));

  // ---- every store of the wave, back to back ----
  auto store_f = [&]() {
    if (jac) {
      SegmentStoresFrom<0, (kQ0 > 0 ? kQ0 - 1 : 0)>(f0, f1, q0);
      if constexpr (kQ0 > 0) StoreNt16<0>(flast, q0[kQ0 - 1]);
    }
  };
  auto store_e = [&]() {
    if constexpr (kQ1 > 0) {
      if (!jac) return;
      SegmentStoresFrom<0, kQ1 - 1>(e0, e1, q1);
      StoreNt16<0>(elast, q1[kQ1 - 1]);
    }
  };
  auto store_r = [&]() {
    if (a.residuals) {  // a kernel argument: a scalar branch, no VALU after the stores
      if constexpr (kQr >= 1) StoreNt16<0>(rdst, qr[0]);
      if constexpr (kQr >= 2) StoreNt16<16>(rdst, qr[1]);
      if constexpr (kQr >= 3) StoreNt16<32>(rdst, qr[2]);
    }
  };
  auto store_g = [&]() {  // the fused gradient's rows and entries (exec-masked)
    if constexpr (kGradF) {
      if (fg.interior) {
        StoreB64At<0>(gp, fg.g1[0]);
        StoreB64At<8>(gp, fg.g1[1]);
        StoreB64At<16>(gp, fg.g1[2]);
      }
      if (fg.writer) {
        StoreNt16<0, 1>(sp, sq[0]);
        StoreNt16<16, 1>(sp, sq[1]);
      }
    }
  };
  if constexpr (T::kOrder == 1) {
    store_r();
    store_e();
    store_f();
  } else if constexpr (T::kOrder == 2) {
    store_e();
    store_f();
    store_r();
  } else {
    store_f();
    store_e();
    store_r();
  }
  if constexpr (kGradF) {
    if constexpr (kContrib) SegmentStoresFrom<0, kGQ>(cb0, cb0, gq);
  }
  store_g();
  // The cost partial (one per wave, lane 0) and the failure flag, last.
  if (lane == 0) {
    StoreB64(v_partial, v_wsum);
    if (failed) StoreB32(status_dst, 1);
  }
  KeepAlive<(kQ0 > 0 ? kQ0 : 1)>(q0);
  KeepAlive<(kQ1 > 0 ? kQ1 : 1)>(q1);
  KeepAlive<kQr>(qr);
  asm volatile("" ::"v"(f0), "v"(f1), "v"(e0), "v"(e1), "v"(rdst), "v"(v_partial), "v"(v_wsum),
               "v"(flast), "v"(elast));
  if constexpr (kGradF) {
    if constexpr (kContrib) KeepAlive<kGQ>(gq);
    KeepAlive<2>(sq);
    asm volatile("" ::"v"(cb0), "v"(gp), "v"(sp), "v"(fg.g1[0]), "v"(fg.g1[1]), "v"(fg.g1[2]));
  }
}

template <class K, int kLoss, bool kJac, bool kCrs, int kCoop, class T = ShippedTune>
__global__ __launch_bounds__(kBlockThreads) void EvaluateAffineChunks(const GroupArgs a) {
  AffineChunkBody<K, kLoss, kJac, kCrs, kCoop, false, T>(a);
}
// The shipped BSM Jacobian kernel of two-slot kinds: two-round staging (9
// KiB of LDS a wave) with one wave per workgroup (16 per CU): each wave is
// dispatched and retired on its own, so the CU's waves do not start and
// reach their store tails in groups of four (1.447-1.454 -> 1.422-1.427 ms
// against four-wave workgroups, profiles/round3/w1).  Held to 4 waves per
// SIMD (128 VGPRs); the held-camera (kConst0) forms and the Jet-based kinds
// likewise (at 5 the quaternion kinds spill 130-160 bytes a lane).
constexpr int kW1WavesPerEu = 4;
template <class K, class T>
constexpr int kW1Waves = kW1WavesPerEu;
template <class K, int kLoss, int kCoop, class T = ShippedTune>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(kW1Waves<K, T>))) void
EvaluateAffineChunksTwoRoundW1(const GroupArgs a) {
  static_assert(kTwoRoundBsm<K>, "two-slot kinds");
  AffineChunkBody<K, kLoss, true, false, kCoop, false, T, 1>(a);
}

// The shipped CRS Jacobian kernel: rows staged in two half-waves (6 KiB of
// LDS a wave, one wave per workgroup) and held to 4 waves per SIMD (128
// VGPRs), as the BSM kernel; one-round staging took 130 VGPRs (3 waves per
// SIMD).
template <class K, int kLoss, int kCoop, class T = ShippedTune>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(kW1Waves<K, T>))) void
EvaluateAffineChunksTwoRoundCrsW1(const GroupArgs a) {
  AffineChunkBody<K, kLoss, true, true, kCoop, false, T, 1>(a);
}

// The fused-gradient form of the hot kernel, held to 3 waves per SIMD
// (168 VGPRs): the LDS bound of 3 workgroups per CU.  Unbounded, the CRS
// form takes 170 VGPRs and drops to 2.
template <class K, int kLoss, bool kCrs, class T = ShippedTune>
__global__ __launch_bounds__(kBlockThreads) __attribute__((amdgpu_waves_per_eu(3))) void
EvaluateAffineChunksFused(const GroupArgs a) {
  AffineChunkBody<K, kLoss, true, kCrs, 2, true, T>(a);
}

// The fused gradient's points-only form: the slot-1 rows and boundary
// entries as above, no slot-0 contributions (CameraGradientKernel computes
// the slot-0 sums).  Without the contribution registers it fits 128 VGPRs
// and runs at 4 waves per SIMD (CRS with the half-wave staging: 2.33 ->
// 2.25 ms against 3 waves, profiles/round2/s5l), one wave per workgroup
// (gradient evaluation 2.147-2.153 -> 2.107-2.109 ms, profiles/round3/w1).
template <class K, int kLoss, bool kCrs, class T = PointsOnlyTune>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(kW1Waves<K, T>))) void
EvaluateAffineChunksFusedPointsW1(const GroupArgs a) {
  AffineChunkBody<K, kLoss, true, kCrs, 2, true, T, 1>(a);
}

// Slot-0 (camera) part of the fused gradient, by re-evaluation in camera
// order.  The evaluation kernel runs in block (point) order, in which a
// camera's ~2,100 blocks are spread over the whole problem; summing their
// J0^T r there needs a transposing round trip through HBM (2.3 GB written in
// block order, 5.8 GB of lines gathered back in camera order at
// problem-13682, GradientContribKernel).  Here each wave takes one chunk of
// at most kGradChunk consecutive entries of one camera's block list and
// evaluates those blocks again with the camera's partials only (Jet<X0>,
// the point a constant): the camera is uniform over the wave, the functor
// data and point ids stream in camera order from a copy sorted once at
// setup (SortSlot0InputsKernel), and only the 24-byte points are gathered
// (a 107 MB table, mostly served from the Infinity Cache).  Per block the
// loss and the Corrector are applied to r and J0 as in the evaluation
// (residual_block.cc:159-199), then J0^T r is added; lanes accumulate
// their blocks in list order and the wave sums by a fixed butterfly, so the
// chunk partials -- and, through GradientChunkReduceKernel, the gradient --
// are deterministic and in the same order as GradientContribKernel's.
// The reference adds the same products with atomics
// (cuda_evaluator_kernel.h:149-160).
struct CamGradArgs {
  const double* state;
  int64_t state_base0, state_base1;
  const double* sdata;         // [n][D] functor data, slot-0-sorted order
  const int32_t* sid1;         // [n] slot-1 ids, same order
  const int32_t* chunk_pb;     // [nchunks] slot-0 id of each chunk
  const int64_t* chunk_begin;  // [nchunks + 1]
  const int32_t* chunk_order;  // [nchunks] the order to take them in (null: 0, 1, ...)
  double* partial;             // [nchunks][S0]
  int64_t nchunks;
  int64_t nslots;              // waves launched; chunk_order[slot] < 0: none
  LossParams loss;
  int apply_loss;
  // Groups with constant slot-0 blocks: the camera from the repacked table
  // (row id - packed_lo), whose state offsets need not be affine.
  const double* packed0;
  int32_t packed_lo;
  int32_t packed_stride;
  double user_loss[kUserLossDoubles];  // a user kind's loss object (kLossUser)
};

// r and the slot-0 Jacobian (NR x S0, row-major) of one block, the slot-1
// parameters held constant (AutoDifferentiate with only slot 0 seeded; a
// slot-0 manifold maps the X0 ambient partials to the S0 tangent columns).
// The Snavely camera's by hand (SnavelyJacobianByHand), as the evaluation.
template <class K>
__device__ __forceinline__ void EvaluateSlot0(const double* d, const double* x0,
                                              const double* x1, double* r, double* J0) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, X0 = Tr::X0, S1 = Tr::S1;
  if constexpr (std::is_same<K, SnavelyKind>::value) {
    double J1[NR * S1];  // dead: the point's partials are not needed here
    SnavelyJacobianByHand(d, x0, x1, r, J0, J1);
    return;
  }
  Jet<X0> j0[X0], j1[S1], out[NR];
#pragma unroll
  for (int k = 0; k < X0; ++k) j0[k] = Jet<X0>(x0[k], k);
#pragma unroll
  for (int k = 0; k < S1; ++k) j1[k] = Jet<X0>(x1[k]);
  K::Evaluate(d, j0, j1, out);
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    r[k] = out[k].a;
    if constexpr (X0 == S0) {
#pragma unroll
      for (int c = 0; c < S0; ++c) J0[k * S0 + c] = out[k].v[c];
    } else {
      K::TangentRow(x0, out[k].v, J0 + k * S0);
    }
  }
}

// The camera rows are J0 formed (by hand for the Snavely camera) and
// contracted with the corrected residuals (a reverse sweep measured no
// faster); the sorted slot-1 ids and the functor data stream non-temporally.
// Waves per SIMD: the compiler's choice (158 VGPRs = 3 with the by-hand
// functor).
template <class K, int kLoss, int kWPB = kWavesPerBlock>
__global__ __launch_bounds__(kWPB * kWave) __attribute__((amdgpu_waves_per_eu(1))) void
CameraGradientKernel(const CamGradArgs g) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p, D = Tr::D;
  static_assert(Tr::NB == 2 && S1 > 0, "two-slot kinds");
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = kWPB == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int64_t slot = (int64_t)blockIdx.x * kWPB + wave;
  if (slot >= g.nslots) return;
  // Pass-major (BuildGradPlan): the resident waves gather from one point
  // range at a time, small enough to stay in the Infinity Cache.
  const int64_t cid = g.chunk_order ? (int64_t)g.chunk_order[slot] : slot;
  if (cid < 0) return;
  const int64_t q0 = g.chunk_begin[cid], q1 = g.chunk_begin[cid + 1];
  constexpr int X0 = Tr::X0;
  const double* cam = g.packed0 ? g.packed0 + (int64_t)g.packed_stride * (g.chunk_pb[cid] - g.packed_lo)
                                : g.state + g.state_base0 + (int64_t)X0 * g.chunk_pb[cid];
  double x0[X0];
#pragma unroll
  for (int k = 0; k < X0; ++k) x0[k] = cam[k];
  double acc[S0];
#pragma unroll
  for (int c = 0; c < S0; ++c) acc[c] = 0.0;
  // kU blocks per lane and step: their loads are all in flight before the
  // first is evaluated.  (1, 2 and 4 measured alike, profiles/round2/s5i:
  // the kernel is insensitive to its occupancy, 2 to 4 waves per SIMD.)
  constexpr int kU = 2;
  for (int64_t q = q0 + lane; q < q1; q += kU * kWave) {
    int64_t qb[kU];
    bool live[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      live[u] = q + u * kWave < q1;
      qb[u] = live[u] ? q + u * kWave : q;
    }
    double d[kU][D], x1[kU][S1];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
#pragma unroll
      for (int k = 0; k < D; ++k) d[u][k] = __builtin_nontemporal_load(g.sdata + qb[u] * D + k);
      const int32_t id1 = __builtin_nontemporal_load(g.sid1 + qb[u]);
      const double* p1 = g.state + g.state_base1 + (int64_t)S1 * id1;
#pragma unroll
      for (int k = 0; k < S1; ++k) x1[u][k] = p1[k];
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      double r[NR], J0[NR * S0], J1[NR * S1p];
      EvaluateSlot0<K>(d[u], x0, x1[u], r, J0);
#pragma unroll
      for (int k = 0; k < NR * S1p; ++k) J1[k] = 0.0;
      LossAndCorrect<K, kLoss, true>(g.loss, g.apply_loss, r, J0, J1, true, g.user_loss);
      if (live[u]) {
#pragma unroll
        for (int c = 0; c < S0; ++c) {
          double s = 0.0;
#pragma unroll
          for (int k = 0; k < NR; ++k) s += J0[k * S0 + c] * r[k];
          acc[c] += s;
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < S0; ++c)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc[c] += __shfl_xor(acc[c], off, kWave);
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < S0; ++c) g.partial[cid * S0 + c] = acc[c];
  }
}

// The slot-0-sorted copies CameraGradientKernel streams: functor data and
// slot-1 ids of block perm[q] at position q.  Once per evaluator.
template <int D>
__global__ __launch_bounds__(kBlockThreads) void SortSlot0InputsKernel(const int32_t* ids,
                                                                       const double* data,
                                                                       const int32_t* perm,
                                                                       int64_t n, double* sdata,
                                                                       int32_t* sid1) {
  const int64_t q = (int64_t)blockIdx.x * kBlockThreads + threadIdx.x;
  if (q >= n) return;
  const int64_t b = perm[q];
#pragma unroll
  for (int k = 0; k < D; ++k) sdata[q * D + k] = data[b * D + k];
  sid1[q] = ids[2 * b + 1];
}

// The same for D data doubles per block (user kinds; a template so that
// every TU including this header may instantiate it).
template <int kUnused = 0>
__global__ __launch_bounds__(kBlockThreads) void SortSlot0InputsAnyKernel(const int32_t* ids, const double* data,
                                                                          int D, const int32_t* perm, int64_t n,
                                                                          double* sdata, int32_t* sid1) {
  const int64_t q = (int64_t)blockIdx.x * kBlockThreads + threadIdx.x;
  if (q >= n) return;
  const int64_t b = perm[q];
  for (int k = 0; k < D; ++k) sdata[q * D + k] = data[b * D + k];
  sid1[q] = ids[2 * b + 1];
}

// The general kernel's output stores, for the whole wave.  When the wave's
// rows form contiguous runs -- residuals NR apart; BlockSparseMatrix cells
// of consecutive blocks (slot j's row k at cell + k t_j, cells NR t_j
// apart); or CompressedRow row blocks (a block's NR rows of W = sum t_j
// values whose slot segments tile the row, blocks NR W apart) -- the wave
// stages the rows in LDS and stores each run with consecutive lanes on
// consecutive doubles (one 512-byte span per store instruction instead of 64
// scattered rows; the scatter made the kernel L2-request bound, 5.9x the
// affine kernel's requests, profiles/round6/r6s).  Otherwise (blocks held
// constant in part of the wave, manifold tangent sizes that differ, other
// layouts) each lane scatters its rows through the offset tables as
// WriteJacobians does (cuda_evaluator_kernel.h:260-294).  A failed block's
// outputs are unspecified (the evaluation reports the failure), so the
// staged runs carry them along.  With a.table_runs (BuildTableRuns: the
// same tests, made once per chunk at cse_create) the wave takes its run
// starts from there and loads no per-block offsets (at two slots and two
// residuals 48 of the kernel's table bytes a block, profiles/round6/r6gen).
template <class K>
constexpr bool kTableStaged = KindTraits<K>::NR * KindTraits<K>::N <= 32;
constexpr int kTableRunFlagResiduals = 1, kTableRunFlagBsm = 2, kTableRunFlagCrs = 4;

template <class K, bool kJac>
__device__ __forceinline__ void TableStores(const GroupArgs& a, bool active, bool ok, int64_t gi,
                                            const PbDev* pb, const double* r, const double* J,
                                            double* st) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, NB = Tr::NB, N = Tr::N;
  constexpr bool kStaged = kTableStaged<K>;
  const int lane = threadIdx.x & (kWave - 1);
  const uint64_t act = __ballot(active);
  if (act == 0) return;
  const int nb = __popcll(act);  // the active lanes are a prefix of the wave
  // Every active lane satisfies c (wave-uniform).
  auto all = [&](bool c) { return __ballot(active && !c) == 0; };
  auto sync = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  };
  // This wave's chunk record (wave-uniform: scalar loads).
  const int64_t* run = nullptr;
  int64_t flags = 0;
  if constexpr (kStaged) {
    if (a.table_runs) {
      const int64_t c = (int64_t)blockIdx.x * kWavesPerBlock + __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
      run = a.table_runs + c * (2 + NB);
      flags = run[0];
    }
  }
  if (a.residuals) {
    const int64_t off = active && !(flags & kTableRunFlagResiduals) ? a.residual_layout[gi] : 0;
    const int64_t off0 = run ? run[1] : __shfl(off, 0, kWave);
    if (kStaged && (run ? (flags & kTableRunFlagResiduals) != 0 : all(off == off0 + (int64_t)NR * lane))) {
      if (active) {
#pragma unroll
        for (int k = 0; k < NR; ++k) st[lane * NR + k] = r[k];
      }
      sync();
      for (int p = lane; p < nb * NR; p += kWave) a.residuals[off0 + p] = st[p];
      sync();
    } else if (active && ok) {
#pragma unroll
      for (int k = 0; k < NR; ++k) a.residuals[off + k] = r[k];
    }
  }
  if constexpr (kJac) {
    if (!a.jacobian) return;
    // Row (j, k) of slot j's a-th active position goes to
    // values + offsets[layout[gi] + a NR + k].
    const int64_t q = active && !run ? a.jac_layout[gi] : 0;
    bool uniform = kStaged;
    bool cst[NB];
    int t[NB];
    int64_t row[NB][NR];
    int na = 0;  // active slots (wave-uniform when `uniform`)
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const bool c = active && pb[j].is_constant;
      const uint64_t m = __ballot(c);
      cst[j] = m != 0;
      uniform = uniform && (m == 0 || m == act);
      t[j] = __shfl(active ? pb[j].tangent_size : 0, 0, kWave);
      uniform = uniform && all(pb[j].is_constant || pb[j].tangent_size == t[j]);
#pragma unroll
      for (int k = 0; k < NR; ++k)
        row[j][k] = active && !cst[j] && !run ? a.jac_offsets[q + (int64_t)na * NR + k] : 0;
      if (!cst[j]) ++na;
    }
    bool bsm = run ? (flags & kTableRunFlagBsm) != 0 : uniform;
    bool crs = run ? (flags & kTableRunFlagCrs) != 0 : uniform;
    int64_t base[NB];
    int64_t r0 = INT64_MAX;
    int w = 0;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      base[j] = run ? run[2 + j] : __shfl(row[j][0], 0, kWave);
      if (cst[j]) continue;
      r0 = base[j] < r0 ? base[j] : r0;
      w += t[j];
    }
    if (uniform && !run) {
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        if (cst[j]) continue;
        bool b = true, c = true;
#pragma unroll
        for (int k = 0; k < NR; ++k) {
          b = b && row[j][k] == base[j] + (int64_t)lane * NR * t[j] + (int64_t)k * t[j];
          c = c && row[j][k] == base[j] + (int64_t)lane * NR * w + (int64_t)k * w;
        }
        bsm = bsm && all(b);
        crs = crs && all(c);
        // CompressedRow: the slot segments [base - r0, + t) tile [0, w)
        const int64_t cj = base[j] - r0;
        crs = crs && cj >= 0 && cj + t[j] <= w;
#pragma unroll
        for (int j2 = 0; j2 < j; ++j2) {
          if (cst[j2]) continue;
          const int64_t c2 = base[j2] - r0;
          crs = crs && (cj + t[j] <= c2 || c2 + t[j2] <= cj);
        }
      }
    }
    if (bsm) {
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        if (cst[j]) continue;
        const int cell = NR * t[j];
        if (active) {
#pragma unroll
          for (int k = 0; k < NR; ++k)
#pragma unroll
            for (int c = 0; c < Tr::Size(j); ++c)
              if (c < t[j]) st[lane * cell + k * t[j] + c] = J[k * N + Tr::Off(j) + c];
        }
        sync();
        for (int p = lane; p < nb * cell; p += kWave) a.jacobian[base[j] + p] = st[p];
        sync();
      }
    } else if (crs) {
      const int blk = NR * w;
      if (active) {
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          if (cst[j]) continue;
          const int cj = (int)(base[j] - r0);
#pragma unroll
          for (int k = 0; k < NR; ++k)
#pragma unroll
            for (int c = 0; c < Tr::Size(j); ++c)
              if (c < t[j]) st[lane * blk + k * w + cj + c] = J[k * N + Tr::Off(j) + c];
        }
      }
      sync();
      for (int p = lane; p < nb * blk; p += kWave) a.jacobian[r0 + p] = st[p];
      sync();
    } else if (active && ok) {
      int64_t qq = run ? a.jac_layout[gi] : q;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        if (pb[j].is_constant) continue;
        const int tj = pb[j].tangent_size;
#pragma unroll
        for (int k = 0; k < NR; ++k) {
          double* dst = a.jacobian + a.jac_offsets[qq++];
#pragma unroll
          for (int c = 0; c < Tr::Size(j); ++c)
            if (c < tj) dst[c] = J[k * N + Tr::Off(j) + c];
        }
      }
    }
  }
}

// The general (table) path for any kind, any number of parameter blocks;
// also runs affine groups when force_general_layout is set.  One block per
// lane, one launch-wide grid.  Per block, as ResidualBlock::Evaluate
// (internal/ceres/residual_block.cc:68-204) and the reference kernel
// (cuda_evaluator_kernel.h:297-422): parameters through the PbDev table
// (constant blocks from the constant state), autodiff, validity check
// (IsEvaluationValid: finite and assigned), ambient J times the
// plus-Jacobian for manifold blocks, loss and Corrector, gradient atomics,
// residuals and Jacobian rows scattered through the offset tables
// (WriteJacobians, :260-294).
// The local Jacobian (NR x N doubles) stays in registers: every index into
// it is a compile-time constant once the loops unroll (a `break` on the
// runtime tangent size in the gradient loop used to leave it in 208 bytes of
// scratch a lane; profiles/round6/r6o).  Outputs: TableStores.
template <class K, int kLoss, bool kJac>
__global__ __launch_bounds__(kBlockThreads) void EvaluateTableKernel(const GroupArgs a) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, NB = Tr::NB, N = Tr::N, D = Tr::D;
  static_assert(NB <= kMaxSlots, "too many parameter blocks");

  const int64_t i = (int64_t)blockIdx.x * kBlockThreads + threadIdx.x;
  const bool active = i < a.n;
  const bool want_grad = kJac && a.gradient != nullptr;
  double cost = 0.0;
  __shared__ double stage_all[kWavesPerBlock][kTableStaged<K> ? kWave * NR * N : 1];
  PbDev pb[NB] = {};
  double r[NR], J[NR * N];
  bool ok = false;
  int64_t gi = 0;

  if (active) {
    double d[D];
#pragma unroll
    for (int k = 0; k < D; ++k) d[k] = a.data[i * D + k];
    double x[N];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int32_t id = a.ids[i * NB + j];
      const double* p;
      if (j == 0 && a.plain0) {  // the record the table holds, without its cache line
        constexpr int S = Tr::Size(0);
        pb[0] = PbDev{a.plain0_state_base + (int64_t)S * id, a.plain0_delta_base + (int64_t)S * id, -1, S, 0};
        // the values from the repacked copy when there is one (one aligned
        // 128-byte row), else from the state
        p = a.packed0 ? static_cast<const double*>(__builtin_assume_aligned(
                            a.packed0 + (int64_t)a.packed0_stride * (id - a.packed0_lo), 16))
                      : a.state + pb[0].state_offset;
      } else {
        pb[j] = a.pbs[id];
        p = (pb[j].is_constant ? a.cstate : a.state) + pb[j].state_offset;
      }
#pragma unroll
      for (int c = 0; c < Tr::Size(j); ++c) x[Tr::Off(j) + c] = p[c];
    }
    ok = EvaluateFunctorFlat<K, kJac>(d, x, r, J);
    if (ok && a.check_finite) {
      bool bad = AnyNonFinite<NR>(r);
      if constexpr (kJac) bad = bad || AnyNonFinite<NR * N>(J);
      ok = !bad;
    }
    if constexpr (MayLeaveOutputs<K>::value) {
      bool bad = AnyImpossible<NR>(r);
      if constexpr (kJac) bad = bad || AnyImpossible<NR * N>(J);
      ok = ok && !bad;
    }
    if constexpr (kJac) {
      // Local Jacobian = ambient Jacobian * PlusJacobian
      // (cuda_evaluator_kernel.h:355-371; residual_block.cc:133-156), in
      // place: slot j keeps its tangent columns first.
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        constexpr int kMax = Tr::MaxSize();
        const int S = Tr::Size(j), o = Tr::Off(j);
        if (pb[j].plus_jacobian_offset == kPlusJacobianQuaternion) {
          // CSE_MANIFOLD_QUATERNION_EUCLIDEAN: the plus-Jacobian from the
          // block's value (QuaternionEuclideanTangentRow), in place.
          if constexpr (kMax >= 4) {
#pragma unroll
            for (int k = 0; k < NR; ++k) {
              double* row = J + k * N + o;
              const double* q = x + o;
              double L[3];
              const double P[4][3] = {{-q[1], -q[2], -q[3]}, {q[0], q[3], -q[2]},
                                      {-q[3], q[0], q[1]}, {q[2], -q[1], q[0]}};
#pragma unroll
              for (int c = 0; c < 3; ++c) {
                double s = 0.0;
#pragma unroll
                for (int m = 0; m < 4; ++m) s += row[m] * P[m][c];
                L[c] = s;
              }
#pragma unroll
              for (int c = 3; c < kMax - 1; ++c)
                if (c < S - 1) row[c] = row[c + 1];
              row[0] = L[0];
              row[1] = L[1];
              row[2] = L[2];
            }
          }
          continue;
        }
        if (pb[j].plus_jacobian_offset < 0) continue;
        const double* PJ = a.plus_jacobians + pb[j].plus_jacobian_offset;
        const int t = pb[j].tangent_size;
#pragma unroll
        for (int k = 0; k < NR; ++k) {
          double L[kMax];
#pragma unroll
          for (int c = 0; c < kMax; ++c) {
            double s = 0.0;
            if (c < t && c < S) {
#pragma unroll
              for (int m = 0; m < kMax; ++m)
                if (m < S) s += J[k * N + o + m] * PJ[m * t + c];
            }
            L[c] = s;
          }
#pragma unroll
          for (int c = 0; c < kMax; ++c)
            if (c < S) J[k * N + o + c] = L[c];
        }
      }
    }
    // Loss and Corrector over all N columns at once (the correction acts on
    // each column independently).
    {
      double sq = 0.0;
#pragma unroll
      for (int k = 0; k < NR; ++k) sq += r[k] * r[k];
      const bool robust = (kLoss != kLossTrivial || a.loss.scaled) && a.apply_loss;
      if (!robust) {
        cost = 0.5 * sq;
      } else {
        double rho[3];
        EvaluateLoss<kLoss, K>(a.loss, sq, rho, a.user_loss);
        const Corrector corr(sq, rho);
        if constexpr (kJac) corr.template CorrectJacobian<NR, N>(r, J);
        corr.template CorrectResiduals<NR>(r);
        cost = 0.5 * rho[0];
      }
    }
    if (!ok) {
      cost = 0.0;
      *a.status = 1;
    } else {
      if (want_grad) {
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          if (pb[j].is_constant) continue;
          double* g = a.gradient + pb[j].delta_offset;
          const int t = pb[j].tangent_size;
          // (c < t as a guard, not a break: the loop unrolls fully and J
          // stays in registers)
#pragma unroll
          for (int c = 0; c < Tr::Size(j); ++c) {
            if (c < t) {
              double s = 0.0;
#pragma unroll
              for (int k = 0; k < NR; ++k) s += J[k * N + Tr::Off(j) + c] * r[k];
              unsafeAtomicAdd(g + c, s);
            }
          }
        }
      }
    }
    gi = a.gindex ? a.gindex[i] : a.first + i;
  }
  TableStores<K, kJac>(a, active, ok, gi, pb, r, J, stage_all[threadIdx.x / kWave]);
  // One partial per wave (the wave's 64 blocks are the affine kernels'
  // chunk, so both paths sum the same partials in the same order).
  const double w = WaveSumLane0(cost);
  if ((threadIdx.x & (kWave - 1)) == 0)
    a.partials[(int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave] = w;
}

}  // namespace cse

#endif  // CSE_EVALUATE_KERNEL_HPP_
