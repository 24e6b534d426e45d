// evaluate_kernel.hpp -- the fused residual/Jacobian/loss/cost kernels.
//
// One wavefront lane owns one residual block (the reference's
// EvaluateKernel, include/ceres/internal/cuda_evaluator_kernel.h:297-422,
// also maps one thread to one block).  Per lane, fused in one pass:
//   gather parameters -> Jet autodiff of the functor -> plus-Jacobian
//   product (manifolds) -> loss rho(|r|^2) and Corrector on J then r ->
//   residual/Jacobian stores -> gradient J^T r -> cost into a per-workgroup
//   partial (summed deterministically by FinalizeKernel).
//
// Two layout policies, chosen per residual group on the host:
//   affine  table-free: block i of the group writes its residuals at
//           res_base + kR*i and row k of slot j at jac_base[j][k] +
//           jac_stride[j]*i, and reads parameter block `id` of slot j at
//           state_base[j] + size_j*id.  This is what BlockJacobianWriter and
//           CompressedRowJacobianWriter produce for Schur-ordered BAL
//           problems: per block the kernel reads only 8 B of ids and the
//           functor data.  Kernel: EvaluateAffinePersistent.
//   table   the reference's offset tables (residual_layout,
//           jacobian_per_residual_layout/offsets, per-block parameter-block
//           records): any layout, constant blocks, manifolds.
//           Kernel: EvaluateGroupKernel<..., kAffine = false>.
//
// EvaluateAffinePersistent is the hot path.  It is sized to the chip (a
// fixed number of workgroups per CU), each wave walks 64-block chunks and
// software-pipelines them: while chunk c is differentiated, the parameter
// gathers of chunk c+1 and the ids of chunk c+2 are in flight, so the two
// dependent HBM round trips (ids -> camera/point) never stall a wave.  Its
// outputs are staged through LDS so every wave writes its contiguous output
// segments with 16-byte-per-lane stores (1 KiB per wave instruction).
#ifndef CSE_EVALUATE_KERNEL_HPP_
#define CSE_EVALUATE_KERNEL_HPP_

#include <stdint.h>

#include "functors.hpp"
#include "jet.hpp"
#include "loss.hpp"

namespace cse {

constexpr int kBlockThreads = 256;
constexpr int kWave = 64;
constexpr int kWavesPerBlock = kBlockThreads / kWave;

// Device copy of a parameter block (table path).
struct PbDev {
  int64_t state_offset;
  int64_t delta_offset;
  int64_t plus_jacobian_offset;
  int32_t tangent_size;
  int32_t is_constant;
};

struct GroupArgs {
  int64_t n;
  const int32_t* ids;   // [n][kNumBlocks]
  const double* data;   // [n][kDataSize]
  const double* state;
  const double* cstate;
  const PbDev* pbs;
  const double* plus_jacobians;
  // Affine policy.
  int64_t state_base[2];
  int64_t delta_base[2];
  int64_t res_base;
  int64_t jac_base[2][3];
  int64_t jac_stride[2];
  // Slot-0 parameter blocks repacked at a 16-byte-aligned stride (the
  // affine path's cooperative LDS-DMA gather; see RepackSlot0Kernel).
  const double* packed0;
  int32_t packed0_lo;
  int32_t packed0_stride;  // doubles per block, even
  // Table policy.
  const int64_t* gindex;
  int64_t first;
  const int64_t* residual_layout;
  const int64_t* jac_layout;
  const int64_t* jac_offsets;
  // Outputs.
  double* residuals;
  double* jacobian;
  double* gradient;
  double* partials;
  int* status;
  uint64_t* timeline;  // diagnostics only ($CSE_TIMELINE): 8 u64 per wave, or null
  // Fused gradient (EvaluateAffineChunks<..., kGradF = true>, see
  // FusedGradient below): the gradient (delta offsets), the slot-1
  // wave-boundary entries [2 * chunks][4] and the slot-0 per-block
  // contributions J0^T r [n][S0p].
  double* gfused;
  double* gside;
  double* gcontrib;
  LossParams loss;
  int apply_loss;
  int check_finite;
};

template <class K>
struct KindTraits {
  static constexpr int NR = K::kNumResiduals;
  static constexpr int NB = K::kNumBlocks;
  static constexpr int S0 = K::kSize0;
  static constexpr int S1 = K::kSize1;
  static constexpr int S1p = S1 > 0 ? S1 : 1;
  static constexpr int N = S0 + S1;
  static constexpr int D = K::kDataSize;
};

// Any of x[0..n) NaN or infinite?  An integer test on the exponent field:
// the TU is compiled with -ffinite-math-only, which would fold isfinite().
template <int kCount>
CSE_HD bool AnyNonFinite(const double* x) {
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < kCount; ++i) {
    const uint64_t b = __builtin_bit_cast(uint64_t, x[i]);
    m = max(m, (uint32_t)(b >> 32) & 0x7ff00000u);
  }
  return m == 0x7ff00000u;
}

// Deterministic workgroup sum: xor-butterfly inside each wave, then the
// waves in a fixed order.  Returns the sum in thread 0.
__device__ __forceinline__ double WorkgroupSum(double v, double* lds) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  if (lane == 0) lds[wave] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; ++w) t += lds[w];
  }
  return t;
}

// Copy `count` doubles, staged contiguously in LDS by this wave, to global
// memory at dst with all 64 lanes: 16-byte stores when dst is 16-byte
// aligned (1 KiB per wave instruction), 8-byte stores otherwise.
template <bool kNt = true>
__device__ __forceinline__ void WaveStore(const double* lds, double* dst, int count, int lane) {
  if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    const int pairs = count >> 1;
    for (int t = lane; t < pairs; t += kWave) {
      const double2 v = *reinterpret_cast<const double2*>(lds + 2 * t);
      if constexpr (kNt) {
        __builtin_nontemporal_store(v.x, dst + 2 * t);
        __builtin_nontemporal_store(v.y, dst + 2 * t + 1);
      } else {
        *reinterpret_cast<double2*>(dst + 2 * t) = v;
      }
    }
    if ((count & 1) && lane == 0) dst[count - 1] = lds[count - 1];
  } else {
    for (int t = lane; t < count; t += kWave) dst[t] = lds[t];
  }
}

// WaveStore for a full 64-block chunk: kCount (compile time) doubles, all
// LDS reads issued before any global store so the wave waits for LDS once
// per segment instead of once per 1 KiB piece.  dst is 16-byte aligned.
template <int kCount, bool kNt = true>
__device__ __forceinline__ void WaveStoreFull(const double* lds, double* dst, int lane) {
  constexpr int kPairs = kCount / 2;
  constexpr int kIters = (kPairs + kWave - 1) / kWave;
  double2 v[kIters];
#pragma unroll
  for (int it = 0; it < kIters; ++it) {
    const int t = it * kWave + lane;
    if (kPairs % kWave == 0 || t < kPairs) v[it] = reinterpret_cast<const double2*>(lds)[t];
  }
#pragma unroll
  for (int it = 0; it < kIters; ++it) {
    const int t = it * kWave + lane;
    if (kPairs % kWave == 0 || t < kPairs) {
      if constexpr (kNt) {
        __builtin_nontemporal_store(v[it].x, dst + 2 * t);
        __builtin_nontemporal_store(v[it].y, dst + 2 * t + 1);
      } else {
        reinterpret_cast<double2*>(dst)[t] = v[it];
      }
    }
  }
  if constexpr (kCount % 2 != 0) {
    if (lane == 0) dst[kCount - 1] = lds[kCount - 1];
  }
}

template <int kCount, bool kNt>
__device__ __forceinline__ void WaveStoreAny(const double* lds, double* dst, int count, int lane) {
  if (count == kCount && (reinterpret_cast<uintptr_t>(dst) & 15) == 0)
    WaveStoreFull<kCount, kNt>(lds, dst, lane);
  else
    WaveStore<kNt>(lds, dst, count, lane);
}

// The functor on plain doubles (kJac = false) or through
// AutoDifferentiate (include/ceres/internal/autodiff.h:314-381): seed one
// Jet per parameter with its unit vector, run the functor, split the
// partials into the row-major per-block Jacobians.
template <class K, bool kJac>
CSE_HD bool EvaluateFunctor(const double* d, const double* x0, const double* x1, double* r,
                            double* J0, double* J1) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p, N = Tr::N;
  if constexpr (kJac) {
    Jet<N> j0[S0], j1[S1p], out[NR];
#pragma unroll
    for (int k = 0; k < S0; ++k) j0[k] = Jet<N>(x0[k], k);
#pragma unroll
    for (int k = 0; k < S1; ++k) j1[k] = Jet<N>(x1[k], S0 + k);
    const bool ok = K::Evaluate(d, j0, j1, out);
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      r[k] = out[k].a;
#pragma unroll
      for (int c = 0; c < S0; ++c) J0[k * S0 + c] = out[k].v[c];
#pragma unroll
      for (int c = 0; c < S1; ++c) J1[k * S1p + c] = out[k].v[S0 + c];
    }
    return ok;
  } else {
    return K::Evaluate(d, x0, x1, r);
  }
}

// Loss and correction (cuda_evaluator_kernel.h:373-407 /
// residual_block.cc:159-199).  Returns the block cost.
template <class K, int kLoss, bool kJac>
CSE_HD double LossAndCorrect(const LossParams& lp, bool apply_loss, double* r, double* J0,
                             double* J1) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p;
  double sq = 0.0;
#pragma unroll
  for (int k = 0; k < NR; ++k) sq += r[k] * r[k];
  const bool robust = (kLoss != kLossTrivial || lp.scaled) && apply_loss;
  if (!robust) return 0.5 * sq;
  double rho[3];
  EvaluateLoss<kLoss>(lp, sq, rho);
  const Corrector corr(sq, rho);
  if constexpr (kJac) {
    corr.template CorrectJacobian<NR, S0>(r, J0);
    if constexpr (S1 > 0) corr.template CorrectJacobian<NR, S1p>(r, J1);
  }
  corr.template CorrectResiduals<NR>(r);
  return 0.5 * rho[0];
}

// Stage one wave's outputs in LDS and write each contiguous segment.  The
// wave's blocks [i0, i0 + nw) are contiguous in every segment:
//   residuals: [res_base + kR*i0, + kR*nw)
//   kCrs = false (BlockSparseMatrix): slot j's packed cells at
//       [jac_base[j][0] + stride_j*i0, + kR*size_j*nw)
//   kCrs = true (CompressedRowSparseMatrix): whole blocks, kR rows of N
//       columns, at [row0 + kR*N*i0, + kR*N*nw)
template <class K, bool kJac, bool kCrs, bool kNt = true, bool kOneRound = false>
__device__ __forceinline__ void StageAndStore(const GroupArgs& a, double* st, int lane, bool active,
                                              int64_t i0, int nw, const double* r,
                                              const double* J0, const double* J1) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, NB = Tr::NB, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p, N = Tr::N;
  if (nw <= 0) return;
  if (a.residuals) {
    // Residuals are already lane-contiguous (kR doubles per block): each
    // lane stores its own, no staging.
    double* dst = a.residuals + a.res_base + (int64_t)NR * (i0 + lane);
    if (active) {
      if (NR == 2 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        __builtin_nontemporal_store(r[0], dst);
        __builtin_nontemporal_store(r[NR - 1], dst + 1);
      } else {
#pragma unroll
        for (int k = 0; k < NR; ++k) __builtin_nontemporal_store(r[k], dst + k);
      }
    }
  }
  if constexpr (kJac) {
    if (!a.jacobian) return;
    if constexpr (kCrs) {
      const int64_t row0 = a.jac_base[0][0] < a.jac_base[NB - 1][0] ? a.jac_base[0][0]
                                                                      : a.jac_base[NB - 1][0];
      if (active) {
#pragma unroll
        for (int k = 0; k < NR; ++k) {
          const int c0 = (int)(a.jac_base[0][k] - row0);
#pragma unroll
          for (int c = 0; c < S0; ++c) st[lane * NR * N + c0 + c] = J0[k * S0 + c];
          if constexpr (S1 > 0) {
            const int c1 = (int)(a.jac_base[1][k] - row0);
#pragma unroll
            for (int c = 0; c < S1; ++c) st[lane * NR * N + c1 + c] = J1[k * S1p + c];
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
      WaveStoreAny<kWave * NR * N, kNt>(st, a.jacobian + row0 + (int64_t)NR * N * i0, nw * NR * N,
                                        lane);
      __builtin_amdgcn_wave_barrier();
    } else if constexpr (kOneRound && S1 > 0) {
      // Both slots' cells staged at once, one LDS round trip.
      double* st1 = st + kWave * NR * S0;
      if (active) {
#pragma unroll
        for (int q = 0; q < NR * S0; ++q) st[lane * NR * S0 + q] = J0[q];
#pragma unroll
        for (int q = 0; q < NR * S1; ++q) st1[lane * NR * S1 + q] = J1[q];
      }
      __builtin_amdgcn_wave_barrier();
      WaveStoreAny<kWave * NR * S0, kNt>(st, a.jacobian + a.jac_base[0][0] + a.jac_stride[0] * i0,
                                         nw * NR * S0, lane);
      WaveStoreAny<kWave * NR * S1, kNt>(st1, a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * i0,
                                         nw * NR * S1, lane);
      __builtin_amdgcn_wave_barrier();
    } else {
      if (active) {
#pragma unroll
        for (int q = 0; q < NR * S0; ++q) st[lane * NR * S0 + q] = J0[q];
      }
      __builtin_amdgcn_wave_barrier();
      WaveStoreAny<kWave * NR * S0, kNt>(st, a.jacobian + a.jac_base[0][0] + a.jac_stride[0] * i0,
                                         nw * NR * S0, lane);
      __builtin_amdgcn_wave_barrier();
      if constexpr (S1 > 0) {
        if (active) {
#pragma unroll
          for (int q = 0; q < NR * S1; ++q) st[lane * NR * S1 + q] = J1[q];
        }
        __builtin_amdgcn_wave_barrier();
        WaveStoreAny<kWave * NR * S1, kNt>(st, a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * i0,
                                           nw * NR * S1, lane);
        __builtin_amdgcn_wave_barrier();
      }
    }
  }
}

// Gradient g += J^T r with device-scope FP64 atomics (native
// global_atomic_add_f64), as cuda_evaluator_kernel.h:149-160.
template <class K>
__device__ __forceinline__ void AddGradient(double* g0, double* g1, int t0, int t1,
                                            const double* r, const double* J0,
                                            const double* J1) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p;
  if (g0) {
#pragma unroll
    for (int c = 0; c < S0; ++c) {
      if (c >= t0) break;
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < NR; ++k) s += J0[k * S0 + c] * r[k];
      unsafeAtomicAdd(g0 + c, s);
    }
  }
  if (g1) {
#pragma unroll
    for (int c = 0; c < S1; ++c) {
      if (c >= t1) break;
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < NR; ++k) s += J1[k * S1p + c] * r[k];
      unsafeAtomicAdd(g1 + c, s);
    }
  }
}

// Inputs of one block (affine path).
template <class K>
struct AffineInputs {
  double d[KindTraits<K>::D];
  double x0[KindTraits<K>::S0];
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

template <class K>
__device__ __forceinline__ void Gather(const GroupArgs& a, int64_t i, int2 id, AffineInputs<K>* in) {
  using Tr = KindTraits<K>;
  constexpr int S0 = Tr::S0, S1 = Tr::S1, D = Tr::D;
  if constexpr (D == 2) {
    const double2 v = *reinterpret_cast<const double2*>(a.data + 2 * i);
    in->d[0] = v.x;
    in->d[1] = v.y;
  } else {
#pragma unroll
    for (int k = 0; k < D; ++k) in->d[k] = a.data[i * D + k];
  }
  const double* p0 = a.state + a.state_base[0] + (int64_t)S0 * id.x;
#pragma unroll
  for (int k = 0; k < S0; ++k) in->x0[k] = p0[k];
  if constexpr (S1 > 0) {
    const double* p1 = a.state + a.state_base[1] + (int64_t)S1 * id.y;
#pragma unroll
    for (int k = 0; k < S1; ++k) in->x1[k] = p1[k];
  }
  in->id0 = id.x;
  in->id1 = id.y;
}

// Per-lane (unstaged) stores of one block: the wave's stores of a segment
// then cover it with 8/16-byte pieces at the block stride.
template <class K, bool kJac, bool kCrs>
__device__ __forceinline__ void DirectStore(const GroupArgs& a, int64_t i, const double* r,
                                            const double* J0, const double* J1) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p;
  if (a.residuals) {
    double* dst = a.residuals + a.res_base + (int64_t)NR * i;
#pragma unroll
    for (int k = 0; k < NR; ++k) dst[k] = r[k];
  }
  if constexpr (kJac) {
    if (!a.jacobian) return;
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      double* d0 = a.jacobian + a.jac_base[0][k] + a.jac_stride[0] * i;
#pragma unroll
      for (int c = 0; c < S0; ++c) d0[c] = J0[k * S0 + c];
      if constexpr (S1 > 0) {
        double* d1 = a.jacobian + a.jac_base[1][k] + a.jac_stride[1] * i;
#pragma unroll
        for (int c = 0; c < S1; ++c) d1[c] = J1[k * S1p + c];
      }
    }
  }
}

// Gather with slot 0 (the camera) loaded wave-cooperatively: the wave's 64
// parameter blocks are fetched as 64*S0 consecutive 8-byte pieces, piece p
// by lane p % 64 of load p / 64, so each load instruction walks the bytes of
// a few whole blocks (~8 cache lines) instead of 64 scattered lines, then
// the pieces are redistributed through LDS (lds: 64*S0 doubles of this
// wave).  Slot 1 (the point) and the functor data are per-lane loads: in
// Schur order consecutive blocks share points, so those already coalesce.
template <class K>
__device__ __forceinline__ void GatherCoop(const GroupArgs& a, int64_t i, int2 id,
                                           AffineInputs<K>* in, double* lds, int lane) {
  using Tr = KindTraits<K>;
  constexpr int S0 = Tr::S0, S1 = Tr::S1, D = Tr::D;
  if constexpr (D == 2) {
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
    for (int k = 0; k < S1; ++k) in->x1[k] = p1[k];
  }
  const double* base0 = a.state + a.state_base[0];
  double piece[S0];
#pragma unroll
  for (int k = 0; k < S0; ++k) {
    const int p = k * kWave + lane;
    const int t = p / S0, q = p - t * S0;
    const int cid = __shfl(id.x, t, kWave);
    piece[k] = base0[(int64_t)S0 * cid + q];
  }
#pragma unroll
  for (int k = 0; k < S0; ++k) lds[k * kWave + lane] = piece[k];
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < S0; ++k) in->x0[k] = lds[lane * S0 + k];
  __builtin_amdgcn_wave_barrier();
  in->id0 = id.x;
  in->id1 = id.y;
}

// Cooperative slot-0 gather in 16-byte pieces through VGPRs from the
// repacked table (the register twin of GatherCoopDma).
template <class K>
__device__ __forceinline__ void GatherCoopPacked(const GroupArgs& a, int64_t i, int2 id,
                                                 AffineInputs<K>* in, double* lds, int lane) {
  using Tr = KindTraits<K>;
  constexpr int S0 = Tr::S0, S1 = Tr::S1, D = Tr::D;
  constexpr int S0p = (S0 + 1) & ~1;
  constexpr int kPieces = S0p / 2;
  const int cid_own = id.x - a.packed0_lo;
  double2 piece[kPieces];
#pragma unroll
  for (int k = 0; k < kPieces; ++k) {
    const int p = k * kWave + lane;
    const int t = p / kPieces, q = p - t * kPieces;
    const int cid = __shfl(cid_own, t, kWave);
    piece[k] = *reinterpret_cast<const double2*>(a.packed0 + (int64_t)S0p * cid + 2 * q);
  }
  if constexpr (D == 2) {
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
    for (int k = 0; k < S1; ++k) in->x1[k] = p1[k];
  }
#pragma unroll
  for (int k = 0; k < kPieces; ++k) reinterpret_cast<double2*>(lds)[k * kWave + lane] = piece[k];
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < S0; ++k) in->x0[k] = lds[lane * S0p + k];
  __builtin_amdgcn_wave_barrier();
  in->id0 = id.x;
  in->id1 = id.y;
}

// Same gather with slot 0 fetched by LDS-DMA (global_load_lds_dwordx4):
// slot-0 blocks are read from the 16-byte-aligned repacked table, piece p
// (16 B) of the wave's 64 blocks by lane p % 64 of load p / 64; the
// hardware writes each lane's 16 B at lds + 16 * p, so the pieces land in
// block order without passing through VGPRs.
template <class K, bool kNtLoads = false>
__device__ __forceinline__ void GatherCoopDma(const GroupArgs& a, int64_t i, int2 id,
                                              AffineInputs<K>* in, double* lds, int lane) {
  using Tr = KindTraits<K>;
  constexpr int S0 = Tr::S0, S1 = Tr::S1, D = Tr::D;
  constexpr int S0p = (S0 + 1) & ~1;  // doubles per block in the packed table
  constexpr int kPieces = S0p / 2;    // 16-byte pieces per block
  const int cid_own = id.x - a.packed0_lo;
#pragma unroll
  for (int k = 0; k < kPieces; ++k) {
    const int p = k * kWave + lane;
    const int t = p / kPieces, q = p - t * kPieces;
    const int cid = __shfl(cid_own, t, kWave);
    const double* src = a.packed0 + (int64_t)S0p * cid + 2 * q;
    __builtin_amdgcn_global_load_lds(src, lds + 2 * kWave * k, 16, 0, 0);
  }
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
    for (int k = 0; k < S1; ++k)
      in->x1[k] = kNtLoads ? __builtin_nontemporal_load(p1 + k) : p1[k];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < S0; ++k) in->x0[k] = lds[lane * S0p + k];
  __builtin_amdgcn_wave_barrier();
  in->id0 = id.x;
  in->id1 = id.y;
}

// The hot path: persistent, software-pipelined, table-free.
//   kPrefetch 2: gathers of chunk c+1 and ids of chunk c+2 in flight while
//                chunk c computes; 1: only the ids of chunk c+1; 0: none;
//                -1: not persistent (one chunk per wave, grid = all chunks).
//   kStage: LDS-staged 1 KiB-per-instruction stores vs per-lane stores.
//   kDebug (diagnostic builds only): 1 replaces the functor with a trivial
//   map of its inputs (memory-path floor), 2 skips the stores (compute
//   floor), 3 stores without the non-temporal hint.
template <class K, int kLoss, bool kJac, bool kCrs, int kPrefetch, bool kStage, int kDebug = 0,
          int kCoop = 0>
__device__ __forceinline__ void AffinePersistentBody(const GroupArgs& a) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p, N = Tr::N;
  constexpr int kOutLane = !kStage ? 1
                          : kJac ? (kCrs || kDebug == 4 ? NR * N : (NR * S0 > NR * S1 ? NR * S0 : NR * S1))
                                 : 1;
  // The staging buffer also holds the cooperative camera gather (used
  // before the outputs are staged).
  constexpr int kCoopLane = kCoop == 2 ? ((S0 + 1) & ~1) : kCoop == 1 ? S0 : 0;
  constexpr int kStageLane = kCoopLane > kOutLane ? kCoopLane : kOutLane;
  __shared__ double stage[kWavesPerBlock][kWave * kStageLane];
  __shared__ double lds_sum[kWavesPerBlock];

  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int64_t num_chunks = (a.n + kWave - 1) / kWave;
  const int64_t stride = (int64_t)gridDim.x * kWavesPerBlock;
  int64_t c = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  const bool want_grad = kJac && a.gradient != nullptr;
  double* st = stage[wave];
  double cost_acc = 0.0;
  bool all_ok = true;

  auto idx = [&](int64_t chunk) {
    const int64_t i = chunk * kWave + lane;
    return i < a.n ? i : a.n - 1;  // inactive lanes re-read the last block
  };
  AffineInputs<K> cur;
  int2 ids_next = make_int2(0, 0);
  if constexpr (kPrefetch == 2) {
    if (c < num_chunks) Gather<K>(a, idx(c), LoadIds<K>(a, idx(c)), &cur);
    if (c + stride < num_chunks) ids_next = LoadIds<K>(a, idx(c + stride));
  } else if constexpr (kPrefetch == 1) {
    if (c < num_chunks) ids_next = LoadIds<K>(a, idx(c));
  }

  for (; c < num_chunks; c += (kPrefetch < 0 ? num_chunks : stride)) {
    const int64_t cn = c + stride;
    AffineInputs<K> nxt;
    if constexpr (kPrefetch == 2) {
      if (cn < num_chunks) Gather<K>(a, idx(cn), ids_next, &nxt);
      if (cn + stride < num_chunks) ids_next = LoadIds<K>(a, idx(cn + stride));
    } else if constexpr (kPrefetch == 1) {
      Gather<K>(a, idx(c), ids_next, &cur);
      if (cn < num_chunks) ids_next = LoadIds<K>(a, idx(cn));
    } else if constexpr (kCoop == 2) {
      GatherCoopDma<K>(a, idx(c), LoadIds<K>(a, idx(c)), &cur, st, lane);
    } else if constexpr (kCoop == 1) {
      GatherCoop<K>(a, idx(c), LoadIds<K>(a, idx(c)), &cur, st, lane);
    } else {
      Gather<K>(a, idx(c), LoadIds<K>(a, idx(c)), &cur);
    }
    (void)cn;

    const int64_t i0 = c * kWave;
    const int64_t rem = a.n - i0;
    const int nw = rem < kWave ? (int)rem : kWave;
    const bool active = lane < nw;
    double r[NR], J0[NR * S0], J1[NR * S1p];
    bool ok = true;
    if constexpr (kDebug == 1) {
#pragma unroll
      for (int k = 0; k < NR; ++k) r[k] = cur.d[k % Tr::D] - cur.x1[k % S1p];
#pragma unroll
      for (int q = 0; q < NR * S0; ++q) J0[q] = cur.x0[q % S0] * cur.d[0];
#pragma unroll
      for (int q = 0; q < NR * S1p; ++q) J1[q] = cur.x1[q % S1p] * cur.d[1 % Tr::D];
    } else {
      ok = EvaluateFunctor<K, kJac>(cur.d, cur.x0, cur.x1, r, J0, J1);
    }
    if (ok && a.check_finite) {
      bool bad = AnyNonFinite<NR>(r);
      if constexpr (kJac) bad = bad || AnyNonFinite<NR * S0>(J0) || AnyNonFinite<NR * S1>(J1);
      ok = !bad;
    }
    double cost = LossAndCorrect<K, kLoss, kJac>(a.loss, a.apply_loss, r, J0, J1);
    if constexpr (kDebug == 2) {
#pragma unroll
      for (int q = 0; q < NR * S0; ++q) cost += J0[q];
#pragma unroll
      for (int q = 0; q < NR * S1p; ++q) cost += J1[q];
#pragma unroll
      for (int k = 0; k < NR; ++k) cost += r[k];
    }
    if (active) {
      all_ok = all_ok && ok;
      cost_acc += cost;
      if (want_grad)
        AddGradient<K>(a.gradient + a.delta_base[0] + (int64_t)S0 * cur.id0,
                       S1 > 0 ? a.gradient + a.delta_base[1] + (int64_t)S1 * cur.id1 : nullptr,
                       S0, S1, r, J0, J1);
    }
    if constexpr (kDebug == 2) {
    } else if constexpr (kStage) {
      StageAndStore<K, kJac, kCrs, kDebug != 3, kDebug == 4>(a, st, lane, active, i0, nw, r, J0,
                                                             J1);
    } else if (active) {
      DirectStore<K, kJac, kCrs>(a, i0 + lane, r, J0, J1);
    }
    if constexpr (kPrefetch == 2) cur = nxt;
  }
  if (!all_ok) *a.status = 1;
  const double t = WorkgroupSum(cost_acc, lds_sum);
  // Affine groups own kWavesPerBlock partial slots per workgroup
  // (EvaluateAffineChunks writes one per wave).
  if (threadIdx.x < kWavesPerBlock)
    a.partials[(int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x] = threadIdx.x == 0 ? t : 0.0;
}

template <class K, int kLoss, bool kJac, bool kCrs, int kPrefetch, bool kStage, int kMinWaves>
__global__ __launch_bounds__(kBlockThreads, kMinWaves) void EvaluateAffinePersistent(
    const GroupArgs a) {
  AffinePersistentBody<K, kLoss, kJac, kCrs, kPrefetch, kStage>(a);
}

// Same kernel without an occupancy request (the compiler's default target).
template <class K, int kLoss, bool kJac, bool kCrs, int kPrefetch, bool kStage, int kDebug = 0,
          int kCoop = 0>
__global__ __launch_bounds__(kBlockThreads) void EvaluateAffinePersistentD(const GroupArgs a) {
  AffinePersistentBody<K, kLoss, kJac, kCrs, kPrefetch, kStage, kDebug, kCoop>(a);
}

// ---------------------------------------------------------------------------
// The shipped hot kernel: one 64-block chunk per wave, every output store
// issued back to back at the very end of the wave.
//
// Why the tail is shaped this way (measured, tools/membench2.hip): on
// gfx950 a vector-memory store reads its address and data VGPRs after
// issue, when the store reaches the head of the CU's memory queue.  An
// instruction that overwrites one of those VGPRs before then stalls the
// wave until the store drains -- under a saturated write stream that is
// microseconds -- so a wave whose register allocator reuses a store's
// VGPRs for the next store's address (or for the cost reduction) issues
// its 13 stores one queue-drain at a time.  The same 6.8 GB memory path
// ran 1.64 ms with that interleaving and 1.24 ms with the stores back to
// back.  Here: the wave's cost is reduced first (cross-lane, no barrier),
// the Jacobian is staged through LDS, and then every store is an inline-asm
// global_store_dwordx4 whose operands stay live (so unclobbered) to the
// end of the kernel.
// ---------------------------------------------------------------------------

typedef int cse_v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ cse_v4i AsV4i(double a, double b) {
  const double2 v = make_double2(a, b);
  cse_v4i d;
  __builtin_memcpy(&d, &v, 16);
  return d;
}

// 16-byte store at base + kOff bytes (kOff in [-4096, 4095]).  kPol: the
// cache policy bits, 0 = nt sc1 (the default: streaming, not kept in the
// XCD's L2; 6-8 % faster than nt alone on the evaluator's stream,
// profiles/r02), 1 = none, 2 = sc1, 3 = sc0 sc1, 4 = nt, 5 = sc0 sc1 nt,
// 6 = sc0 nt (tuning variants).
template <int kOff, int kPol = 0>
__device__ __forceinline__ void StoreNt16(double* base, const cse_v4i& d) {
  static_assert(kOff >= -4096 && kOff <= 4095, "global offset out of range");
  if constexpr (kPol == 4)
    asm volatile("global_store_dwordx4 %0, %1, off offset:%2 nt" ::"v"(base), "v"(d), "i"(kOff)
                 : "memory");
  else if constexpr (kPol == 1)
    asm volatile("global_store_dwordx4 %0, %1, off offset:%2" ::"v"(base), "v"(d), "i"(kOff)
                 : "memory");
  else if constexpr (kPol == 2)
    asm volatile("global_store_dwordx4 %0, %1, off offset:%2 sc1" ::"v"(base), "v"(d), "i"(kOff)
                 : "memory");
  else if constexpr (kPol == 3)
    asm volatile("global_store_dwordx4 %0, %1, off offset:%2 sc0 sc1" ::"v"(base), "v"(d),
                 "i"(kOff)
                 : "memory");
  else if constexpr (kPol == 0)
    asm volatile("global_store_dwordx4 %0, %1, off offset:%2 sc1 nt" ::"v"(base), "v"(d),
                 "i"(kOff)
                 : "memory");
  else if constexpr (kPol == 5)
    asm volatile("global_store_dwordx4 %0, %1, off offset:%2 sc0 sc1 nt" ::"v"(base), "v"(d),
                 "i"(kOff)
                 : "memory");
  else
    asm volatile("global_store_dwordx4 %0, %1, off offset:%2 sc0 nt" ::"v"(base), "v"(d),
                 "i"(kOff)
                 : "memory");
}

template <int kJ, int kCount, int kPol = 0>
__device__ __forceinline__ void SegmentStoresFrom(double* b0, double* b1, const cse_v4i* q) {
  if constexpr (kJ < kCount) {
    StoreNt16<(kJ % 8) * 1024 - 4096, kPol>(kJ < 8 ? b0 : b1, q[kJ]);
    SegmentStoresFrom<kJ + 1, kCount, kPol>(b0, b1, q);
  }
}

// A wave's contiguous segment of kCount 16-byte pieces per lane: piece j
// of lane l at seg + 16 * (64 j + l) bytes (1 KiB per instruction).
template <int kCount>
__device__ __forceinline__ void SegmentStores(double* seg, int lane, const cse_v4i* q,
                                              double** keep0, double** keep1) {
  static_assert(kCount <= 16, "segment too long");
  double* b0 = seg + 2 * lane + 512;   // pieces 0..7 at offsets -4096..3072
  double* b1 = seg + 2 * lane + 1536;  // pieces 8..15
  SegmentStoresFrom<0, kCount>(b0, b1, q);
  *keep0 = b0;
  *keep1 = b1;
}

// Diagnostics ($CSE_TIMELINE): the shader clock / the 100 MHz real-time
// clock, read into SGPRs (SMEM, no vector-memory slot).
__device__ __forceinline__ uint64_t ShaderClock() {
  uint64_t t;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t));
  return t;
}
__device__ __forceinline__ uint64_t RealClock() {
  uint64_t t;
  asm volatile("s_memrealtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t));
  return t;
}

// Vector stores of one wave-uniform value, issued by the calling lanes
// (the caller masks to lane 0).  Both operands are VGPRs computed before
// the store tail, so nothing after the tail writes a VGPR a queued store
// still has to read.  kPol: 0 = default policy (the partial's line is
// shared by 16 waves and merges in L2), 1 = nt sc1 (as the output
// segments), 2 = sc1.
template <int kPol = 0>
__device__ __forceinline__ void StoreB64(double* addr, double value) {
  if constexpr (kPol == 1)
    asm volatile("global_store_dwordx2 %0, %1, off sc1 nt" ::"v"(addr), "v"(value) : "memory");
  else if constexpr (kPol == 2)
    asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(addr), "v"(value) : "memory");
  else
    asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(addr), "v"(value) : "memory");
}
__device__ __forceinline__ void StoreB32(int* addr, int value) {
  asm volatile("global_store_dword %0, %1, off" ::"v"(addr), "v"(value) : "memory");
}

// XCD-grouped cost-partial slots: workgroups are dealt round-robin over
// the 8 XCDs, so workgroups b, b + 8, b + 16, b + 24 (one XCD, running at
// about the same time) get one 128-byte line of partials together instead
// of sharing it with three other XCDs.  The slot space is a multiple of 8
// workgroups (the host reserves it; unused slots stay zero).
__device__ __forceinline__ int64_t PartialSlot(int64_t b, int64_t num_wg, int wave, int wpb) {
  const int64_t per_xcd = (num_wg + 7) / 8;
  return ((b & 7) * per_xcd + (b >> 3)) * wpb + wave;
}

// One double at addr + kOff bytes, default cache policy (the fused
// gradient's scattered slot-1 rows: neighbouring lanes share lines in L2).
template <int kOff>
__device__ __forceinline__ void StoreB64At(double* addr, double value) {
  asm volatile("global_store_dwordx2 %0, %1, off offset:%2" ::"v"(addr), "v"(value), "i"(kOff)
               : "memory");
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

// The fused gradient of one wave (EvaluateAffineChunks<..., kGradF>): the
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
  bool interior = false, writer = false;
  int64_t entry = 0;
  int key = 0;

  __device__ __forceinline__ void Compute(const double* r, const double* J0, const double* J1,
                                          int id1, bool active, int lane, int nw, int64_t c) {
    using Tr = KindTraits<K>;
    constexpr int NR = Tr::NR, S1p = Tr::S1p;
    static_assert(Tr::NB == 2 && S1 == 3, "fused gradient: two slots, the second of size 3");
#pragma unroll
    for (int cc = 0; cc < S0p; ++cc) {
      double s = 0.0;
      if (cc < S0) {
#pragma unroll
        for (int k = 0; k < NR; ++k) s += J0[k * S0 + cc] * r[k];
      }
      g0[cc] = s;
    }
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
    const bool run_end = lane == nw - 1 || (lane < nw - 1 && knext != key);
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

template <int kCount>
__device__ __forceinline__ void KeepAlive(const cse_v4i* q) {
#pragma unroll
  for (int j = 0; j < kCount; ++j) asm volatile("" ::"v"(q[j]));
}

// Can the wave take the back-to-back store tail?  Full chunk, 16-byte
// pieces that tile every segment exactly, 16-byte-aligned destinations.
template <class K, bool kJac, bool kCrs>
__device__ __forceinline__ bool FastTail(const GroupArgs& a, int64_t i0, int nw) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, N = Tr::N;
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
      m |= reinterpret_cast<uintptr_t>(a.jacobian + a.jac_base[0][0] + a.jac_stride[0] * i0);
      if constexpr (S1 > 0)
        m |= reinterpret_cast<uintptr_t>(a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * i0);
    }
  }
  return (m & 15) == 0;
}

// kTwoRound (BSM only): stage slot 0's cells, read them back, then slot
// 1's into the same LDS (18 instead of 24 doubles per lane: 4 instead of 3
// workgroups per CU).
// kDebug (diagnostic variants, wrong results by design), bit flags: 1
// replaces the functor by a trivial map of its inputs (memory-path floor),
// 2 skips every output store (compute floor), 4 skips the LDS transpose
// (each lane stores its own values at the coalesced positions).
template <class K, int kLoss, bool kJac, bool kCrs, int kCoop, bool kTwoRound = false,
          int kDebug = 0, int kWPB = kWavesPerBlock, bool kGradF = false>
__device__ __forceinline__ void AffineChunkBody(const GroupArgs& a) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p, N = Tr::N;
  constexpr int kOutLane = (kJac && (kDebug & 12) == 0)
                              ? (kCrs ? NR * N
                                      : kTwoRound ? (S0 > S1 ? NR * S0 : NR * S1)
                                                  : NR * (S0 + S1))
                              : 1;
  constexpr int kCoopLane = kCoop >= 2 ? ((S0 + 1) & ~1) : kCoop == 1 ? S0 : 0;
  constexpr int kStageLane = kCoopLane > kOutLane ? kCoopLane : kOutLane;
  __shared__ double stage[kWPB][kWave * kStageLane];

  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int64_t num_chunks = (a.n + kWave - 1) / kWave;
  // kDebug bit 131072 (tuning variant): XCD-contiguous chunk ranges --
  // workgroups are dealt round-robin over the 8 XCDs, so XCD x runs
  // workgroups x, x + 8, ...; remapped, XCD x walks one contiguous range.
  int64_t bid = blockIdx.x;
  if constexpr ((kDebug & 131072) != 0) {
    const int64_t per = (gridDim.x + 7) / 8;
    const int64_t x = bid & 7, k = bid >> 3;
    const int64_t full = gridDim.x - (per - 1) * 8;  // XCDs that get `per` workgroups
    bid = x < full ? x * per + k : full * per + (x - full) * (per - 1) + k;
  }
  int64_t c = bid * kWPB + wave;
  // kDebug bit 262144 (tuning variant): the 8 workgroups dispatched
  // together (one per XCD) interleave their chunks one by one instead of
  // taking kWPB consecutive chunks each.
  if constexpr ((kDebug & 262144) != 0) {
    const int64_t grp = bid >> 3, x = bid & 7;
    c = (grp * kWPB + wave) * 8 + x;
    if ((grp + 1) * 8 > gridDim.x) c = bid * kWPB + wave;  // the ragged last group: identity
  }
  double* partial_dst =
      a.partials + ((kDebug & 65536) ? PartialSlot(blockIdx.x, gridDim.x, wave, kWPB) : c);
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
  constexpr bool kTime = (kDebug & 2048) != 0;
  uint64_t tl[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if constexpr (kTime) {
    tl[0] = RealClock();
    tl[1] = ShaderClock();
  }

  AffineInputs<K> in;
  if constexpr (kCoop == 3) {
    GatherCoopPacked<K>(a, i, LoadIds<K>(a, i), &in, st, lane);
  } else if constexpr (kCoop == 2) {
    // Once-read streams (ids, observations, points) load non-temporally
    // (-1.3 %, profiles/r02); kDebug bit 512 turns that off for A/B runs.
    constexpr bool kNtLoads = (kDebug & 512) == 0;
    int2 id;
    if constexpr (kNtLoads && Tr::NB == 2) {
      const long long b = __builtin_nontemporal_load(reinterpret_cast<const long long*>(a.ids) + i);
      id = make_int2((int)b, (int)(b >> 32));
    } else {
      id = LoadIds<K>(a, i);
    }
    GatherCoopDma<K, kNtLoads>(a, i, id, &in, st, lane);
  } else if constexpr (kCoop == 1) {
    GatherCoop<K>(a, i, LoadIds<K>(a, i), &in, st, lane);
  } else {
    Gather<K>(a, i, LoadIds<K>(a, i), &in);
  }
  if constexpr (kTime) {
    // the gather has landed once its values are used
    asm volatile("" ::"v"(in.x0[0]), "v"(in.x1[0]), "v"(in.d[0]));
    tl[2] = ShaderClock();
  }
  double r[NR], J0[NR * S0], J1[NR * S1p];
  bool ok = true;
  if constexpr ((kDebug & 1) != 0) {
#pragma unroll
    for (int k = 0; k < NR; ++k) r[k] = in.d[k % Tr::D] - in.x1[k % S1p];
#pragma unroll
    for (int q = 0; q < NR * S0; ++q) J0[q] = in.x0[q % S0] * in.d[0];
#pragma unroll
    for (int q = 0; q < NR * S1p; ++q) J1[q] = in.x1[q % S1p] * in.d[1 % Tr::D];
  } else {
    ok = EvaluateFunctor<K, kJac>(in.d, in.x0, in.x1, r, J0, J1);
  }
  // kDebug bit 524288 (diagnostic): the functor evaluated a second time on
  // inputs the compiler cannot prove equal, its outputs folded in times an
  // opaque zero -- twice the FP64 work, the same results.
  double extra = 0.0;
  if constexpr ((kDebug & 524288) != 0) {
    double zero = 0.0;
    asm volatile("" : "+v"(zero));
    AffineInputs<K> in2 = in;
    in2.x1[0] += zero * r[0];
    double r2[NR], J02[NR * S0], J12[NR * S1p];
    EvaluateFunctor<K, kJac>(in2.d, in2.x0, in2.x1, r2, J02, J12);
    double s2 = 0.0;
#pragma unroll
    for (int k = 0; k < NR; ++k) s2 += r2[k];
#pragma unroll
    for (int q = 0; q < NR * S0; ++q) s2 += J02[q];
#pragma unroll
    for (int q = 0; q < NR * S1p; ++q) s2 += J12[q];
    extra = zero * s2;
  }
  if (ok && a.check_finite) {
    bool bad = AnyNonFinite<NR>(r);
    if constexpr (kJac) bad = bad || AnyNonFinite<NR * S0>(J0) || AnyNonFinite<NR * S1>(J1);
    ok = !bad;
  }
  double cost = LossAndCorrect<K, kLoss, kJac>(a.loss, a.apply_loss, r, J0, J1) + extra;
  if constexpr ((kDebug & 2) != 0) {
#pragma unroll
    for (int q = 0; q < NR * S0; ++q) cost += J0[q];
#pragma unroll
    for (int q = 0; q < NR * S1p; ++q) cost += J1[q];
#pragma unroll
    for (int k = 0; k < NR; ++k) cost += r[k];
  }
  if (kJac && a.gradient != nullptr && active)
    AddGradient<K>(a.gradient + a.delta_base[0] + (int64_t)S0 * in.id0,
                   S1 > 0 ? a.gradient + a.delta_base[1] + (int64_t)S1 * in.id1 : nullptr, S0, S1,
                   r, J0, J1);
  if constexpr (kTime) {
    asm volatile("" ::"v"(cost), "v"(r[0]), "v"(J0[0]));
    tl[3] = ShaderClock();
  }
  // The wave's cost (fixed xor-butterfly order) and failure flag, before
  // any store is queued.
  double wsum = active ? cost : 0.0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) wsum += __shfl_xor(wsum, off, kWave);
  const bool failed = __ballot(active && !ok) != 0;
  int* status_dst = a.status;
  static_assert(!kGradF || (kJac && kDebug == 0), "fused gradient: real Jacobian kernels only");
  FusedGrad<K> fg;
  if constexpr (kGradF) fg.Compute(r, J0, J1, in.id1, active, lane, nw, c);

  if constexpr ((kDebug & 2) != 0) {
    if (lane == 0) *partial_dst = wsum;
    return;
  }
  if (!FastTail<K, kJac, kCrs>(a, i0, nw)) {
    if constexpr ((kDebug & 12) == 0)
      StageAndStore<K, kJac, kCrs, true, !kTwoRound>(a, st, lane, active, i0, nw, r, J0, J1);
    if constexpr (kGradF) {
      // The group's last, partial chunk: plain stores.
      constexpr int S0p = FusedGrad<K>::S0p;
      if (active) {
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
  constexpr int kQ0 = kJac ? (kCrs ? NR * N / 2 : NR * S0 / 2) : 0;  // pieces per lane, seg 0
  constexpr int kQ1 = (kJac && !kCrs && S1 > 0) ? NR * S1 / 2 : 0;   // seg 1 (E cells)
  const bool jac = kJac && a.jacobian != nullptr;
  cse_v4i q0[kQ0 > 0 ? kQ0 : 1], q1[kQ1 > 0 ? kQ1 : 1];
  double* seg0 = nullptr;
  double* seg1 = nullptr;
  if constexpr (kJac && (kDebug & 8) != 0 && !kCrs) {
    // Diagnostic: one register quad (the wave's cost) for every store.
    if (jac) {
      const cse_v4i one = AsV4i(wsum, wsum);
#pragma unroll
      for (int j = 0; j < kQ0; ++j) q0[j] = one;
#pragma unroll
      for (int j = 0; j < kQ1; ++j) q1[j] = one;
      seg0 = a.jacobian + a.jac_base[0][0] + a.jac_stride[0] * i0;
      seg1 = a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * i0;
    }
  } else if constexpr (kJac && (kDebug & 4) != 0 && !kCrs) {
    if (jac) {
#pragma unroll
      for (int j = 0; j < kQ0; ++j) q0[j] = AsV4i(J0[2 * j], J0[2 * j + 1]);
#pragma unroll
      for (int j = 0; j < kQ1; ++j) q1[j] = AsV4i(J1[2 * j], J1[2 * j + 1]);
      seg0 = a.jacobian + a.jac_base[0][0] + a.jac_stride[0] * i0;
      seg1 = a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * i0;
    }
  } else if constexpr (kJac) {
    if (jac) {
      if constexpr (kCrs) {
        const int64_t row0 = a.jac_base[0][0] < a.jac_base[Tr::NB - 1][0]
                                 ? a.jac_base[0][0]
                                 : a.jac_base[Tr::NB - 1][0];
#pragma unroll
        for (int k = 0; k < NR; ++k) {
          const int c0 = (int)(a.jac_base[0][k] - row0);
#pragma unroll
          for (int cc = 0; cc < S0; ++cc) st[lane * NR * N + c0 + cc] = J0[k * S0 + cc];
          if constexpr (S1 > 0) {
            const int c1 = (int)(a.jac_base[1][k] - row0);
#pragma unroll
            for (int cc = 0; cc < S1; ++cc) st[lane * NR * N + c1 + cc] = J1[k * S1p + cc];
          }
        }
        seg0 = a.jacobian + row0 + (int64_t)NR * N * i0;
      } else if constexpr (kTwoRound) {
#pragma unroll
        for (int p = 0; p < NR * S0; ++p) st[lane * NR * S0 + p] = J0[p];
        seg0 = a.jacobian + a.jac_base[0][0] + a.jac_stride[0] * i0;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < kQ0; ++j) {
          const double2 v = reinterpret_cast<const double2*>(st)[j * kWave + lane];
          q0[j] = AsV4i(v.x, v.y);
        }
        if constexpr (S1 > 0) {
          // Every lane's reads of round 1 must land before round 2 writes.
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int k = 0; k < NR; ++k)
#pragma unroll
            for (int cc = 0; cc < S1; ++cc) st[lane * NR * S1 + k * S1 + cc] = J1[k * S1p + cc];
          seg1 = a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * i0;
        }
      } else {
        double* st1 = st + kWave * NR * S0;
#pragma unroll
        for (int p = 0; p < NR * S0; ++p) st[lane * NR * S0 + p] = J0[p];
        if constexpr (S1 > 0) {
#pragma unroll
          for (int k = 0; k < NR; ++k)
#pragma unroll
            for (int cc = 0; cc < S1; ++cc) st1[lane * NR * S1 + k * S1 + cc] = J1[k * S1p + cc];
          seg1 = a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * i0;
        }
        seg0 = a.jacobian + a.jac_base[0][0] + a.jac_stride[0] * i0;
      }
      __builtin_amdgcn_wave_barrier();
      if constexpr (kCrs || !kTwoRound) {
#pragma unroll
        for (int j = 0; j < kQ0; ++j) {
          const double2 v = reinterpret_cast<const double2*>(st)[j * kWave + lane];
          q0[j] = AsV4i(v.x, v.y);
        }
      }
      if constexpr (kQ1 > 0) {
        const double* st1 = kTwoRound ? st : st + kWave * NR * S0;
#pragma unroll
        for (int j = 0; j < kQ1; ++j) {
          const double2 v = reinterpret_cast<const double2*>(st1)[j * kWave + lane];
          q1[j] = AsV4i(v.x, v.y);
        }
      }
    }
  }
  // Fused gradient: the slot-0 contributions staged through the same LDS
  // (after the Jacobian pieces have been read back), the slot-1 entry.
  constexpr int kGQ = kGradF ? FusedGrad<K>::S0p / 2 : 1;
  static_assert(kGQ <= 8, "contribution pieces: one base register");
  cse_v4i gq[kGQ], sq[2];
  double *cb0 = nullptr, *gp = nullptr, *sp = nullptr;
  if constexpr (kGradF) {
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
    sq[0] = AsV4i(fg.g1[0], fg.g1[1]);
    sq[1] = AsV4i(fg.g1[2], fg.g1[3]);
    cb0 = a.gcontrib + (int64_t)(2 * kGQ) * i0 + 2 * lane + 512;
    gp = a.gfused + a.delta_base[1] + 3LL * fg.key;
    sp = a.gside + 4 * fg.entry;
  }
  // Residual pieces: the lane's own NR doubles (NR even).
  constexpr int kQr = NR / 2;
  cse_v4i qr[kQr];
#pragma unroll
  for (int k = 0; k < kQr; ++k) qr[k] = AsV4i(r[2 * k], r[2 * k + 1]);
  double* rdst = a.residuals ? a.residuals + a.res_base + (int64_t)NR * (i0 + lane) : nullptr;

  // Every address and the wave's scalar outputs are computed (and pinned by
  // the empty asm) before the first store: after it the wave runs only
  // stores and SALU, so nothing waits on the store queue.
  double *f0 = nullptr, *f1 = nullptr, *e0 = nullptr, *e1 = nullptr;
  if (jac) {
    f0 = seg0 + 2 * lane + 512;
    f1 = seg0 + 2 * lane + 1536;
    if constexpr (kQ1 > 0) {
      e0 = seg1 + 2 * lane + 512;
      e1 = seg1 + 2 * lane + 1536;
    }
  }
  // The partial's address and value in VGPRs now, not after the tail.
  double* v_partial = partial_dst;
  double v_wsum = wsum;
  asm volatile("" : "+v"(v_partial), "+v"(v_wsum));
  asm volatile("" ::"v"(f0), "v"(f1), "v"(e0), "v"(e1), "v"(rdst));
  if constexpr (kTime) {
    KeepAlive<(kQ0 > 0 ? kQ0 : 1)>(q0);  // staging reads landed
    KeepAlive<(kQ1 > 0 ? kQ1 : 1)>(q1);
    tl[4] = ShaderClock();
  }

  // ---- every store of the wave, back to back ----
  constexpr int kPol = (kDebug >> 4) & 15;  // tuning variants only; 0 = nt sc1
  constexpr int kPartPol = (kDebug >> 12) & 3;       // tuning variants only
  constexpr bool kPartFirst = (kDebug & 16384) != 0;  // tuning variant: partial first
  if (kPartFirst && lane == 0) StoreB64<kPartPol>(v_partial, v_wsum);
  if (jac) {
    SegmentStoresFrom<0, kQ0, kPol>(f0, f1, q0);
    if constexpr (kQ1 > 0) SegmentStoresFrom<0, kQ1, kPol>(e0, e1, q1);
  }
  if (a.residuals) {  // a kernel argument: a scalar branch, no VALU after the stores
    if constexpr (kQr >= 1) StoreNt16<0, kPol>(rdst, qr[0]);
    if constexpr (kQr >= 2) StoreNt16<16, kPol>(rdst, qr[1]);
    if constexpr (kQr >= 3) StoreNt16<32, kPol>(rdst, qr[2]);
  }
  if constexpr (kGradF) {
    SegmentStoresFrom<0, kGQ>(cb0, cb0, gq);
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
  // The cost partial (one per wave, lane 0) and the failure flag, last.
  if (lane == 0) {
    if (!kPartFirst && (kDebug & 32768) == 0) StoreB64<kPartPol>(v_partial, v_wsum);
    if (failed) StoreB32(status_dst, 1);
  }
  if constexpr (kTime) {
    tl[5] = ShaderClock();
    tl[6] = RealClock();
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    tl[7] = ((uint64_t)xcc << 32) | hw;
    uint64_t mine = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) mine = lane == k ? tl[k] : mine;
    if (lane < 8) a.timeline[8 * c + lane] = mine;
  }
  KeepAlive<(kQ0 > 0 ? kQ0 : 1)>(q0);
  KeepAlive<(kQ1 > 0 ? kQ1 : 1)>(q1);
  KeepAlive<kQr>(qr);
  asm volatile("" ::"v"(f0), "v"(f1), "v"(e0), "v"(e1), "v"(rdst), "v"(v_partial), "v"(v_wsum));
  if constexpr (kGradF) {
    KeepAlive<kGQ>(gq);
    KeepAlive<2>(sq);
    asm volatile("" ::"v"(cb0), "v"(gp), "v"(sp), "v"(fg.g1[0]), "v"(fg.g1[1]), "v"(fg.g1[2]));
  }
}

// ---------------------------------------------------------------------------
// Software-pipelined persistent variant (Snavely-shaped groups: two slots,
// the second of size 3, two functor doubles).  Per-wave timelines
// (tools/timeline.py, CSE_AFFINE_VARIANT=47) of the one-chunk-per-wave
// kernel show the gather waiting ~10k cycles behind the write stream, half
// of each wave's life; here every input of chunk c + W (ids, observations,
// points, cameras) is fetched by LDS-DMA while chunk c computes and stores,
// and the ids one step earlier still.  All vector-memory traffic of the
// loop is LDS-DMA or inline-asm stores, so the compiler tracks none of it
// and the waits are explicit: at the top of an iteration everything but the
// previous chunk's 13 stores must have landed (s_waitcnt vmcnt(13)).
// One wave per workgroup (no sibling waves holding a finished wave's slot),
// persistent over W = gridDim.x waves.
// ---------------------------------------------------------------------------
// LDS reads the compiler does not see: its waitcnt pass would otherwise
// put an s_waitcnt vmcnt(0) (LDS-DMA -> ds_read) at the top of the pipelined
// loop and drain the previous chunk's stores.  The caller waits lgkmcnt(0)
// itself (PipeLdsFence) before using the values.
__device__ __forceinline__ uint32_t LdsAddr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
template <int kOff>
__device__ __forceinline__ cse_v4i LdsRead128(uint32_t addr) {
  cse_v4i v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(kOff));
  return v;
}
template <int kOff>
__device__ __forceinline__ double LdsRead64(uint32_t addr) {
  double v;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(kOff));
  return v;
}
template <int kOff>
__device__ __forceinline__ int LdsRead32(uint32_t addr) {
  int v;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(kOff));
  return v;
}
__device__ __forceinline__ void V4iToDoubles(cse_v4i v, double* d) { __builtin_memcpy(d, &v, 16); }

// LDS-DMA issue helpers of EvaluateAffinePipelined.  gfx950's
// global_load_lds moves 1, 2, 4, 12 or 16 bytes per lane and writes lane l's
// bytes at lds + size * l -- except the 12-byte form, which writes at
// lds + 16 * l (measured, tools/ldsdma_probe.hip: a 4-byte hole after each
// lane's 12 bytes).  The ids go as two dword streams, the 24-byte points as
// 128 cooperative 12-byte halves (half h of point t at lds + 32 t + 16 h),
// the cameras as 16-byte pieces (GatherCoopDma).  (Plain functions: clang
// drops a kernel whose lambdas capture __shared__ arrays by reference.)
__device__ __forceinline__ int64_t PipeBlock(const GroupArgs& a, int64_t cc, int lane) {
  const int64_t i = cc * kWave + lane;
  return i < a.n ? i : a.n - 1;
}
__device__ __forceinline__ void PipeIssueIds(const GroupArgs& a, int64_t cc, int lane, int32_t* ids) {
  const int32_t* src = a.ids + 2 * PipeBlock(a, cc, lane);
  __builtin_amdgcn_global_load_lds(src, ids, 4, 0, 2);
  __builtin_amdgcn_global_load_lds(src + 1, ids + kWave, 4, 0, 2);
}
template <int S0p>
__device__ __forceinline__ void PipeIssueGather(const GroupArgs& a, int64_t cc, int lane, int2 id,
                                                double* cam, double* obs, double* pt) {
  constexpr int kPieces = S0p / 2;
  const int cid_own = id.x - a.packed0_lo;
#pragma unroll
  for (int k = 0; k < kPieces; ++k) {
    const int p = k * kWave + lane;
    const int t = p / kPieces, q = p - t * kPieces;
    const int cid = __shfl(cid_own, t, kWave);
    __builtin_amdgcn_global_load_lds(a.packed0 + (int64_t)S0p * cid + 2 * q, cam + 2 * kWave * k, 16,
                                     0, 0);
  }
  __builtin_amdgcn_global_load_lds(a.data + 2 * PipeBlock(a, cc, lane), obs, 16, 0, 2);
  const double* base = a.state + a.state_base[1];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int p = k * kWave + lane;
    const int pid = __shfl(id.y, p >> 1, kWave);
    const char* src = reinterpret_cast<const char*>(base + 3 * (int64_t)pid) + 12 * (p & 1);
    __builtin_amdgcn_global_load_lds(src, reinterpret_cast<char*>(pt) + 16 * kWave * k, 12, 0, 2);
  }
}

template <class K, int kLoss, bool kJac, bool kCrs>
__global__ __launch_bounds__(kWave) void EvaluateAffinePipelined(const GroupArgs a) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p, N = Tr::N;
  static_assert(Tr::NB == 2 && S1 == 3 && Tr::D == 2 && NR == 2, "Snavely-shaped groups only");
  constexpr int S0p = (S0 + 1) & ~1;
  constexpr int kOutLane = kJac ? (kCrs ? NR * N : NR * (S0 + S1)) : 1;
  constexpr int kQ0 = kJac ? (kCrs ? NR * N / 2 : NR * S0 / 2) : 0;
  constexpr int kQ1 = (kJac && !kCrs) ? NR * S1 / 2 : 0;
  __shared__ double in_cam[kWave * S0p];
  __shared__ double in_obs[kWave * 2];
  __shared__ double in_pt[4 * kWave];  // point t: halves at 32 t and 32 t + 16 bytes
  __shared__ int32_t in_ids[2 * kWave];  // id0 of the 64 blocks, then id1
  __shared__ double stage[kWave * kOutLane];

  const int lane = threadIdx.x;
  const int64_t nchunks = (a.n + kWave - 1) / kWave;
  const int64_t W = gridDim.x;
  int64_t c = blockIdx.x;
  if (c >= nchunks) return;
  // Prologue: ids(c), then gather(c) and ids(c + W).
  PipeIssueIds(a, c, lane, in_ids);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  int2 idc = make_int2(in_ids[lane], in_ids[kWave + lane]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  PipeIssueGather<S0p>(a, c, lane, idc, in_cam, in_obs, in_pt);
  PipeIssueIds(a, c + W < nchunks ? c + W : nchunks - 1, lane, in_ids);
  bool first = true;
  bool prev_fast = true;  // the previous chunk issued exactly kStores stores
  bool failed_any = false;
  constexpr int kStores = kQ0 + kQ1 + 2;  // vector stores per full chunk (+ the partial)
  static_assert(kStores <= 63, "vmcnt field");
  const bool exact = a.residuals != nullptr && (!kJac || a.jacobian != nullptr);
  // Cost-only (candidate) evaluations: the partial is the chunk's one store.
  const bool cost_only = !kJac && a.residuals == nullptr;

  for (; c < nchunks; c += W) {
    // Everything issued before the previous chunk's kStores stores has
    // landed (vmcnt counts in issue order).  With other output sets the
    // store count differs: the cost-only form waits for its one store, any
    // other waits for everything (correct, not pipelined).
    if (first || !prev_fast || !(exact || cost_only))
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (cost_only)
      asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kStores) : "memory");
    first = false;
    __builtin_amdgcn_wave_barrier();
    AffineInputs<K> in;
    in.id0 = idc.x;
    in.id1 = idc.y;
    int2 idn;
    {
      static_assert(S0p == 10, "camera read below assumes 5 pieces");
      const uint32_t acam = LdsAddr(in_cam) + 8 * S0p * lane;
      const uint32_t aobs = LdsAddr(in_obs) + 16 * lane;
      const uint32_t apt = LdsAddr(in_pt) + 32 * lane;
      const uint32_t aid = LdsAddr(in_ids) + 4 * lane;
      cse_v4i c0 = LdsRead128<0>(acam), c1 = LdsRead128<16>(acam), c2 = LdsRead128<32>(acam);
      cse_v4i c3 = LdsRead128<48>(acam), c4 = LdsRead128<64>(acam);
      cse_v4i ob = LdsRead128<0>(aobs);
      // x = bytes 0..7, y = 8..11 | 16..19, z = 20..27 (4-byte aligned).
      double p0 = LdsRead64<0>(apt);
      int y0 = LdsRead32<8>(apt), y1 = LdsRead32<16>(apt);
      int z0 = LdsRead32<20>(apt), z1 = LdsRead32<24>(apt);
      int i0 = LdsRead32<0>(aid), i1 = LdsRead32<4 * kWave>(aid);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4)
                   : : "memory");
      asm volatile("" : "+v"(ob), "+v"(p0), "+v"(y0), "+v"(y1), "+v"(z0), "+v"(z1), "+v"(i0),
                   "+v"(i1));
      const double p1 = __builtin_bit_cast(double, ((uint64_t)(uint32_t)y1 << 32) | (uint32_t)y0);
      const double p2 = __builtin_bit_cast(double, ((uint64_t)(uint32_t)z1 << 32) | (uint32_t)z0);
      double cam[10];
      V4iToDoubles(c0, cam);
      V4iToDoubles(c1, cam + 2);
      V4iToDoubles(c2, cam + 4);
      V4iToDoubles(c3, cam + 6);
      V4iToDoubles(c4, cam + 8);
#pragma unroll
      for (int k = 0; k < S0; ++k) in.x0[k] = cam[k];
      V4iToDoubles(ob, in.d);
      in.x1[0] = p0;
      in.x1[1] = p1;
      in.x1[2] = p2;
      idn = make_int2(i0, i1);
    }
    __builtin_amdgcn_wave_barrier();
    // Next chunk's inputs (clamped past the end: harmless re-reads).
    const int64_t cn = c + W < nchunks ? c + W : nchunks - 1;
    const int64_t cnn = c + 2 * W < nchunks ? c + 2 * W : nchunks - 1;
    PipeIssueGather<S0p>(a, cn, lane, idn, in_cam, in_obs, in_pt);
    PipeIssueIds(a, cnn, lane, in_ids);

    const int64_t i0 = c * kWave;
    const int64_t rem = a.n - i0;
    const int nw = rem < kWave ? (int)rem : kWave;
    const bool active = lane < nw;
    double r[NR], J0[NR * S0], J1[NR * S1p];
    bool ok = EvaluateFunctor<K, kJac>(in.d, in.x0, in.x1, r, J0, J1);
    if (ok && a.check_finite) {
      bool bad = AnyNonFinite<NR>(r);
      if constexpr (kJac) bad = bad || AnyNonFinite<NR * S0>(J0) || AnyNonFinite<NR * S1>(J1);
      ok = !bad;
    }
    const double cost = LossAndCorrect<K, kLoss, kJac>(a.loss, a.apply_loss, r, J0, J1);
    double wsum = active ? cost : 0.0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) wsum += __shfl_xor(wsum, off, kWave);
    failed_any = failed_any || (__ballot(active && !ok) != 0);
    double* v_partial = a.partials + c;
    double v_wsum = wsum;
    asm volatile("" : "+v"(v_partial), "+v"(v_wsum));

    if (!FastTail<K, kJac, kCrs>(a, i0, nw)) {
      // Only the group's last, partial chunk: the generic staged stores
      // (compiler-visible; nothing is waited on after them).
      StageAndStore<K, kJac, kCrs, true, true>(a, stage, lane, active, i0, nw, r, J0, J1);
      if (lane == 0) StoreB64(v_partial, v_wsum);
      idc = idn;
      prev_fast = false;
      continue;
    }
    const bool jac = kJac && a.jacobian != nullptr;
    cse_v4i q0[kQ0 > 0 ? kQ0 : 1], q1[kQ1 > 0 ? kQ1 : 1];
    double* seg0 = nullptr;
    double* seg1 = nullptr;
    if constexpr (kJac) {
      if (jac) {
        if constexpr (kCrs) {
          const int64_t row0 = a.jac_base[0][0] < a.jac_base[1][0] ? a.jac_base[0][0]
                                                                   : a.jac_base[1][0];
#pragma unroll
          for (int k = 0; k < NR; ++k) {
            const int c0 = (int)(a.jac_base[0][k] - row0);
            const int c1 = (int)(a.jac_base[1][k] - row0);
#pragma unroll
            for (int cc = 0; cc < S0; ++cc) stage[lane * NR * N + c0 + cc] = J0[k * S0 + cc];
#pragma unroll
            for (int cc = 0; cc < S1; ++cc) stage[lane * NR * N + c1 + cc] = J1[k * S1p + cc];
          }
          seg0 = a.jacobian + row0 + (int64_t)NR * N * i0;
        } else {
          double* st1 = stage + kWave * NR * S0;
#pragma unroll
          for (int p = 0; p < NR * S0; ++p) stage[lane * NR * S0 + p] = J0[p];
#pragma unroll
          for (int k = 0; k < NR; ++k)
#pragma unroll
            for (int cc = 0; cc < S1; ++cc) st1[lane * NR * S1 + k * S1 + cc] = J1[k * S1p + cc];
          seg0 = a.jacobian + a.jac_base[0][0] + a.jac_stride[0] * i0;
          seg1 = a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * i0;
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < kQ0; ++j) {
          const double2 v = reinterpret_cast<const double2*>(stage)[j * kWave + lane];
          q0[j] = AsV4i(v.x, v.y);
        }
        if constexpr (kQ1 > 0) {
          const double* st1 = stage + kWave * NR * S0;
#pragma unroll
          for (int j = 0; j < kQ1; ++j) {
            const double2 v = reinterpret_cast<const double2*>(st1)[j * kWave + lane];
            q1[j] = AsV4i(v.x, v.y);
          }
        }
      }
    }
    const cse_v4i qr = AsV4i(r[0], r[1]);
    double* rdst = a.residuals ? a.residuals + a.res_base + (int64_t)NR * (i0 + lane) : nullptr;
    double *f0 = nullptr, *f1 = nullptr, *e0 = nullptr, *e1 = nullptr;
    if (jac) {
      f0 = seg0 + 2 * lane + 512;
      f1 = seg0 + 2 * lane + 1536;
      if constexpr (kQ1 > 0) {
        e0 = seg1 + 2 * lane + 512;
        e1 = seg1 + 2 * lane + 1536;
      }
    }
    asm volatile("" ::"v"(f0), "v"(f1), "v"(e0), "v"(e1), "v"(rdst));
    // Exactly kStores vector stores per full chunk (one when cost-only) for
    // the wait at the top.
    if (jac) {
      SegmentStoresFrom<0, kQ0>(f0, f1, q0);
      if constexpr (kQ1 > 0) SegmentStoresFrom<0, kQ1>(e0, e1, q1);
    }
    if (a.residuals) StoreNt16<0>(rdst, qr);
    if (lane == 0) StoreB64(v_partial, v_wsum);
    KeepAlive<(kQ0 > 0 ? kQ0 : 1)>(q0);
    KeepAlive<(kQ1 > 0 ? kQ1 : 1)>(q1);
    asm volatile("" ::"v"(f0), "v"(f1), "v"(e0), "v"(e1), "v"(rdst), "v"(qr), "v"(v_partial),
                 "v"(v_wsum));
    idc = idn;
  }
  if (failed_any && lane == 0) StoreB32(a.status, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the wave ends
}

// ---------------------------------------------------------------------------
// EvaluateAffineStream: persistent, one wave per workgroup, every input of
// chunk c + W fetched by LDS-DMA while chunk c computes (as
// EvaluateAffinePipelined), built around two gfx950 behaviours that stall
// a persistent wave (tools/membench2.hip, tools/ldsdma_probe.hip):
//   * a vector-memory instruction reads its VGPR operands (address and
//     store data) when it reaches the head of the CU's memory queue, which
//     under the write stream is thousands of cycles after issue; rewriting
//     such a register first stalls the wave until then.  So the DMA address
//     registers of chunk c + W stay live until the wait that retires those
//     DMAs (top of the next chunk), the stores take their data from one of
//     kSets rotating accumulation-register sets (AgprSet<k>, loaded straight
//     from the LDS staging buffer), and their addresses are a constant lane
//     offset plus wave-uniform SGPR bases.
//   * the DMA of 12-byte pieces leaves a 4-byte hole per lane.
// BSM Snavely<2,9,3> with residuals and Jacobian requested (the headline
// workload); other shapes take EvaluateAffineChunks.
// ---------------------------------------------------------------------------
#include "agpr_sets.inc"

__device__ __forceinline__ uint64_t Uniform64(uint64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
  return ((uint64_t)hi << 32) | lo;
}

struct StreamDma {
  const void* cam[5];
  const void* obs;
  const void* pt[2];
  const void* ids[2];
};

__device__ __forceinline__ void StreamIssueIds(const GroupArgs& a, int64_t cc, int lane, int32_t* ids,
                                               StreamDma* d) {
  const int32_t* src = a.ids + 2 * PipeBlock(a, cc, lane);
  d->ids[0] = src;
  d->ids[1] = src + 1;
  __builtin_amdgcn_global_load_lds(src, ids, 4, 0, 2);
  __builtin_amdgcn_global_load_lds(src + 1, ids + kWave, 4, 0, 2);
}

__device__ __forceinline__ void StreamIssueGather(const GroupArgs& a, int64_t cc, int lane, int2 id,
                                                  double* cam, double* obs, double* pt,
                                                  StreamDma* d) {
  constexpr int kPieces = 5;  // Snavely camera: 10 doubles in the packed table
  const int cid_own = id.x - a.packed0_lo;
#pragma unroll
  for (int k = 0; k < kPieces; ++k) {
    const int p = k * kWave + lane;
    const int t = p / kPieces, q = p - t * kPieces;
    const int cid = __shfl(cid_own, t, kWave);
    const double* src = a.packed0 + (int64_t)10 * cid + 2 * q;
    d->cam[k] = src;
    __builtin_amdgcn_global_load_lds(src, cam + 2 * kWave * k, 16, 0, 0);
  }
  const double* so = a.data + 2 * PipeBlock(a, cc, lane);
  d->obs = so;
  __builtin_amdgcn_global_load_lds(so, obs, 16, 0, 2);
  const double* base = a.state + a.state_base[1];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int p = k * kWave + lane;
    const int pid = __shfl(id.y, p >> 1, kWave);
    const char* src = reinterpret_cast<const char*>(base + 3 * (int64_t)pid) + 12 * (p & 1);
    d->pt[k] = src;
    __builtin_amdgcn_global_load_lds(src, reinterpret_cast<char*>(pt) + 16 * kWave * k, 12, 0, 2);
  }
}

// The previous DMA batch has landed (the caller waited): its address
// registers may be rewritten from here on.
__device__ __forceinline__ void StreamRelease(const StreamDma& d) {
  asm volatile("" ::"v"(d.cam[0]), "v"(d.cam[1]), "v"(d.cam[2]), "v"(d.cam[3]), "v"(d.cam[4]),
               "v"(d.obs), "v"(d.pt[0]), "v"(d.pt[1]), "v"(d.ids[0]), "v"(d.ids[1]));
}

struct StreamLds {
  double* cam;
  double* obs;
  double* pt;
  int32_t* ids;
  double* stage;
};

struct StreamState {
  int64_t c;
  int2 idc;
  StreamDma dma;
  bool first;
  bool failed;
  uint32_t voff;   // 16 * lane: the store offset of every piece
  uint32_t voff2;  // 16 * lane + 5120
  uint32_t vzero;  // 0: the partial's offset
};

// One chunk with store set kSet.  Returns false when the wave is done.
// kSplit: stage F, pull it into the set, then stage E in the same LDS
// (9 instead of 12 KiB of staging per wave).
template <class K, int kLoss, int kSet, bool kSplit = false>
__device__ __forceinline__ bool StreamStep(const GroupArgs& a, StreamState& S, const StreamLds& L,
                                           int lane, int64_t nchunks, int64_t W) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p;
  constexpr int kStores = 14;  // 13 pieces + the partial, per full chunk
  if (S.c >= nchunks) return false;
  // Everything but the previous chunk's stores has landed, in issue order.
  if (S.first)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(kStores) : "memory");
  S.first = false;
  StreamRelease(S.dma);
  __builtin_amdgcn_wave_barrier();
  AffineInputs<K> in;
  in.id0 = S.idc.x;
  in.id1 = S.idc.y;
  int2 idn;
  {
    const uint32_t acam = LdsAddr(L.cam) + 80 * lane;
    const uint32_t aobs = LdsAddr(L.obs) + 16 * lane;
    const uint32_t apt = LdsAddr(L.pt) + 32 * lane;
    const uint32_t aid = LdsAddr(L.ids) + 4 * lane;
    cse_v4i c0 = LdsRead128<0>(acam), c1 = LdsRead128<16>(acam), c2 = LdsRead128<32>(acam);
    cse_v4i c3 = LdsRead128<48>(acam), c4 = LdsRead128<64>(acam);
    cse_v4i ob = LdsRead128<0>(aobs);
    double p0 = LdsRead64<0>(apt);
    int y0 = LdsRead32<8>(apt), y1 = LdsRead32<16>(apt);
    int z0 = LdsRead32<20>(apt), z1 = LdsRead32<24>(apt);
    int i0 = LdsRead32<0>(aid), i1 = LdsRead32<4 * kWave>(aid);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4)
                 : : "memory");
    asm volatile("" : "+v"(ob), "+v"(p0), "+v"(y0), "+v"(y1), "+v"(z0), "+v"(z1), "+v"(i0),
                 "+v"(i1));
    double cam[10];
    V4iToDoubles(c0, cam);
    V4iToDoubles(c1, cam + 2);
    V4iToDoubles(c2, cam + 4);
    V4iToDoubles(c3, cam + 6);
    V4iToDoubles(c4, cam + 8);
#pragma unroll
    for (int k = 0; k < S0; ++k) in.x0[k] = cam[k];
    V4iToDoubles(ob, in.d);
    in.x1[0] = p0;
    in.x1[1] = __builtin_bit_cast(double, ((uint64_t)(uint32_t)y1 << 32) | (uint32_t)y0);
    in.x1[2] = __builtin_bit_cast(double, ((uint64_t)(uint32_t)z1 << 32) | (uint32_t)z0);
    idn = make_int2(i0, i1);
  }
  __builtin_amdgcn_wave_barrier();
  // Next chunk's inputs (clamped past the end: harmless re-reads).
  const int64_t c = S.c;
  const int64_t cn = c + W < nchunks ? c + W : nchunks - 1;
  const int64_t cnn = c + 2 * W < nchunks ? c + 2 * W : nchunks - 1;
  StreamIssueGather(a, cn, lane, idn, L.cam, L.obs, L.pt, &S.dma);
  StreamIssueIds(a, cnn, lane, L.ids, &S.dma);

  const int64_t i0 = c * kWave;
  const int64_t rem = a.n - i0;
  const int nw = rem < kWave ? (int)rem : kWave;
  const bool active = lane < nw;
  double r[NR], J0[NR * S0], J1[NR * S1p];
  bool ok = EvaluateFunctor<K, true>(in.d, in.x0, in.x1, r, J0, J1);
  if (ok && a.check_finite) {
    const bool bad = AnyNonFinite<NR>(r) || AnyNonFinite<NR * S0>(J0) || AnyNonFinite<NR * S1>(J1);
    ok = !bad;
  }
  const double cost = LossAndCorrect<K, kLoss, true>(a.loss, a.apply_loss, r, J0, J1);
  double wsum = active ? cost : 0.0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) wsum += __shfl_xor(wsum, off, kWave);
  S.failed = S.failed || (__ballot(active && !ok) != 0);
  S.c = c + W;
  S.idc = idn;

  if (!FastTail<K, true, false>(a, i0, nw)) {
    // The group's last, partial chunk: the generic staged stores.
    // (Also every chunk when an output is not requested.)  The next step
    // waits for everything: its store count is not kStores.
    StageAndStore<K, true, false, true, true>(a, L.stage, lane, active, i0, nw, r, J0, J1);
    if (lane == 0) StoreB64(a.partials + c, wsum);
    S.first = true;
    return true;
  }
  // Stage the E and F cells (lane-major, as EvaluateAffineChunks), then
  // pull them into the store set as 16-byte pieces in segment order.
  double* st = L.stage;
  double* st1 = kSplit ? st : st + kWave * NR * S0;
#pragma unroll
  for (int p = 0; p < NR * S0; ++p) st[lane * NR * S0 + p] = J0[p];
  if constexpr (kSplit) {
    __builtin_amdgcn_wave_barrier();
    AgprSet<kSet>::LoadStageF(LdsAddr(st) + 16 * lane);  // waits for its reads
    __builtin_amdgcn_wave_barrier();
  }
#pragma unroll
  for (int k = 0; k < NR; ++k)
#pragma unroll
    for (int cc = 0; cc < S1; ++cc) st1[lane * NR * S1 + k * S1 + cc] = J1[k * S1p + cc];
  __builtin_amdgcn_wave_barrier();
  if constexpr (kSplit)
    AgprSet<kSet>::LoadStageE(LdsAddr(st) + 16 * lane);
  else
    AgprSet<kSet>::LoadStage(LdsAddr(st) + 16 * lane);
  AgprSet<kSet>::PutRes(r[0], r[1], wsum);
  // Wave-uniform bases, forced into SGPRs (the "s" constraint alone lets
  // the compiler hand a VGPR pair to the assembler here).
  const uint64_t f0 = Uniform64(reinterpret_cast<uint64_t>(a.jacobian + a.jac_base[0][0] +
                                                           a.jac_stride[0] * i0));
  const uint64_t e0 = Uniform64(reinterpret_cast<uint64_t>(a.jacobian + a.jac_base[1][0] +
                                                           a.jac_stride[1] * i0));
  const uint64_t r0 = Uniform64(reinterpret_cast<uint64_t>(a.residuals + a.res_base + (int64_t)NR * i0));
  const uint64_t p0 = Uniform64(reinterpret_cast<uint64_t>(a.partials + c));
  AgprSet<kSet>::StoreAll(S.voff, S.voff2, f0, e0, r0);
  if (lane == 0) AgprSet<kSet>::StorePartial(S.vzero, p0);
  // The staging buffer is rewritten by the next chunk only after these
  // LDS reads (in-order LDS queue; StoreAll waited lgkmcnt(0) anyway).
  return true;
}

template <class K, int kLoss, int kSets, bool kSplit>
__device__ __forceinline__ void AffineStreamBody(const GroupArgs& a) {
  using Tr = KindTraits<K>;
  static_assert(Tr::NB == 2 && Tr::S0 == 9 && Tr::S1 == 3 && Tr::D == 2 && Tr::NR == 2,
                "Snavely<2,9,3>-shaped groups only");
  __shared__ double in_cam[kWave * 10];
  __shared__ double in_obs[kWave * 2];
  __shared__ double in_pt[4 * kWave];
  __shared__ int32_t in_ids[2 * kWave];
  __shared__ double stage[kWave * (kSplit ? 18 : 24)];
  const StreamLds L{in_cam, in_obs, in_pt, in_ids, stage};

  const int lane = threadIdx.x;
  const int64_t nchunks = (a.n + kWave - 1) / kWave;
  const int64_t W = gridDim.x;
  StreamState S;
  S.c = blockIdx.x;
  if (S.c >= nchunks) return;
  S.first = true;
  S.failed = false;
  S.voff = 16u * lane;
  S.voff2 = 16u * lane + 5120u;
  S.vzero = 0u;
  asm volatile("" : "+v"(S.voff), "+v"(S.voff2), "+v"(S.vzero));
  // Prologue: ids(c), then gather(c) and ids(c + W).
  StreamIssueIds(a, S.c, lane, in_ids, &S.dma);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  S.idc = make_int2(in_ids[lane], in_ids[kWave + lane]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  StreamIssueGather(a, S.c, lane, S.idc, in_cam, in_obs, in_pt, &S.dma);
  StreamIssueIds(a, S.c + W < nchunks ? S.c + W : nchunks - 1, lane, in_ids, &S.dma);
  for (;;) {
    if (!StreamStep<K, kLoss, 0, kSplit>(a, S, L, lane, nchunks, W)) break;
    if constexpr (kSets > 1)
      if (!StreamStep<K, kLoss, 1, kSplit>(a, S, L, lane, nchunks, W)) break;
    if constexpr (kSets > 2)
      if (!StreamStep<K, kLoss, 2, kSplit>(a, S, L, lane, nchunks, W)) break;
    if constexpr (kSets > 3)
      if (!StreamStep<K, kLoss, 3, kSplit>(a, S, L, lane, nchunks, W)) break;
  }
  if (S.failed && lane == 0) StoreB32(a.status, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the wave ends
  asm volatile("" ::"v"(S.voff), "v"(S.voff2), "v"(S.vzero));
}

template <class K, int kLoss, int kSets>
__global__ __launch_bounds__(kWave) void EvaluateAffineStream(const GroupArgs a) {
  AffineStreamBody<K, kLoss, kSets, false>(a);
}

// Two waves per SIMD (256 registers per wave), two-round staging (17.5 KiB
// of LDS per wave: 8 waves per CU fit).
template <class K, int kLoss, int kSets>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(2, 2))) void
EvaluateAffineStream2(const GroupArgs a) {
  AffineStreamBody<K, kLoss, kSets, true>(a);
}

// Diagnostic only: tools/membench2.hip's m1 memory path (camera gather
// from the packed table, 13 stores of one register quad) on the
// evaluator's real buffers (BSM, Snavely shapes).  Wrong results by design.
// kStep walks it towards EvaluateAffineChunks one change at a time:
//   0 m1 as in membench (register gather, compiler stores, lane-0 partial)
//   1 + the shipped tail (asm stores at SegmentStoresFrom bases, lane-0 partial last)
//   2 + LDS-DMA camera gather (GatherCoopDma)
//   3 + distinct data per store (q[j] = v * j)
template <int kStep>
__global__ __launch_bounds__(kBlockThreads) void MembenchM1Kernel(const GroupArgs a) {
  __shared__ double lds[kWavesPerBlock][kWave * 10];
  const int lane = threadIdx.x & 63, wave = threadIdx.x / 64;
  const int64_t chunks = (a.n + 63) / 64;
  const int64_t c = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  if (c >= chunks) return;
  int64_t i = c * 64 + lane;
  if (i >= a.n) i = a.n - 1;
  double v;
  if constexpr (kStep >= 2) {
    AffineInputs<SnavelyKind> in;
    GatherCoopDma<SnavelyKind>(a, i, LoadIds<SnavelyKind>(a, i), &in, lds[wave], lane);
    v = in.d[0] + in.d[1] + in.x1[0] + in.x1[1] + in.x1[2];
#pragma unroll
    for (int k = 0; k < 9; ++k) v += in.x0[k];
  } else {
    const int2 id = *reinterpret_cast<const int2*>(a.ids + 2 * i);
    const double2 o = reinterpret_cast<const double2*>(a.data)[i];
    const double* pt = a.state + a.state_base[1] + 3L * id.y;
    v = o.x + o.y + pt[0] + pt[1] + pt[2];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int p = k * 64 + lane;
      const int t = p / 5, q = p % 5;
      const int cid = __shfl(id.x - a.packed0_lo, t, 64);
      const double2 w = *reinterpret_cast<const double2*>(a.packed0 + 10L * cid + 2 * q);
      *reinterpret_cast<double2*>(lds[wave] + t * 10 + 2 * q) = w;
    }
    __builtin_amdgcn_wave_barrier();
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 9; ++k) s += lds[wave][lane * 10 + k];
    __builtin_amdgcn_wave_barrier();
    v += s;
  }
  double* res = a.residuals + a.res_base;
  double* E = a.jacobian + a.jac_base[1][0];
  double* F = a.jacobian + a.jac_base[0][0];
  if constexpr (kStep == 0) {
    __builtin_nontemporal_store(v, res + 128 * c + 2 * lane);
    __builtin_nontemporal_store(v, res + 128 * c + 2 * lane + 1);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      __builtin_nontemporal_store(v, E + 384 * c + 128 * k + 2 * lane);
      __builtin_nontemporal_store(v, E + 384 * c + 128 * k + 2 * lane + 1);
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      __builtin_nontemporal_store(v, F + 1152 * c + 128 * k + 2 * lane);
      __builtin_nontemporal_store(v, F + 1152 * c + 128 * k + 2 * lane + 1);
    }
    if (lane == 0) a.partials[c] = 0.0;
  } else {
    cse_v4i q0[9], q1[3];
#pragma unroll
    for (int j = 0; j < 9; ++j) q0[j] = kStep >= 3 ? AsV4i(v * j, v * (j + 1)) : AsV4i(v, v);
#pragma unroll
    for (int j = 0; j < 3; ++j) q1[j] = kStep >= 3 ? AsV4i(v * (j + 9), v * j) : AsV4i(v, v);
    const cse_v4i qr = AsV4i(v, v);
    double* seg0 = F + 1152 * c;
    double* seg1 = E + 384 * c;
    double* rdst = res + 128 * c + 2 * lane;
    double* f0 = seg0 + 2 * lane + 512;
    double* f1 = seg0 + 2 * lane + 1536;
    double* e0 = seg1 + 2 * lane + 512;
    double* e1 = seg1 + 2 * lane + 1536;
    double* v_partial = a.partials + c;
    double v_zero = 0.0;
    asm volatile("" : "+v"(v_partial), "+v"(v_zero));
    asm volatile("" ::"v"(f0), "v"(f1), "v"(e0), "v"(e1), "v"(rdst));
    SegmentStoresFrom<0, 9>(f0, f1, q0);
    SegmentStoresFrom<0, 3>(e0, e1, q1);
    StoreNt16<0>(rdst, qr);
    if (lane == 0) StoreB64(v_partial, v_zero);
    KeepAlive<9>(q0);
    KeepAlive<3>(q1);
    asm volatile("" ::"v"(f0), "v"(f1), "v"(e0), "v"(e1), "v"(rdst), "v"(qr), "v"(v_partial),
                 "v"(v_zero));
  }
}

template <class K, int kLoss, bool kJac, bool kCrs, int kCoop, bool kTwoRound = false,
          int kDebug = 0, int kWPB = kWavesPerBlock, bool kGradF = false>
__global__ __launch_bounds__(kWave * kWPB) void EvaluateAffineChunks(const GroupArgs a) {
  AffineChunkBody<K, kLoss, kJac, kCrs, kCoop, kTwoRound, kDebug, kWPB, kGradF>(a);
}

// Diagnostic variants held to 3 waves per SIMD (the shipped kernel's).
template <class K, int kLoss, int kDebug>
__global__ __launch_bounds__(kBlockThreads) __attribute__((amdgpu_waves_per_eu(3))) void
EvaluateAffineChunksW3(const GroupArgs a) {
  AffineChunkBody<K, kLoss, true, false, 2, false, kDebug>(a);
}

// The fused-gradient form of the shipped kernel, held to 3 waves per SIMD
// (168 VGPRs): the LDS bound of 3 workgroups per CU.  Unbounded, the CRS
// form takes 170 VGPRs and drops to 2.
template <class K, int kLoss, bool kCrs>
__global__ __launch_bounds__(kBlockThreads) __attribute__((amdgpu_waves_per_eu(3))) void
EvaluateAffineChunksFused(const GroupArgs a) {
  AffineChunkBody<K, kLoss, true, kCrs, 2, false, 0, kWavesPerBlock, true>(a);
}

// The general (table) path; also runs affine groups when
// force_general_layout is set.  One block per lane, one launch-wide grid.
template <class K, int kLoss, bool kJac>
__global__ __launch_bounds__(kBlockThreads) void EvaluateGroupKernel(const GroupArgs a) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, NB = Tr::NB, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p;

  const int64_t i = (int64_t)blockIdx.x * kBlockThreads + threadIdx.x;
  const bool active = i < a.n;
  const bool want_jac = kJac && a.jacobian != nullptr;
  const bool want_grad = kJac && a.gradient != nullptr;
  double cost = 0.0;

  if (active) {
    int32_t id[2] = {0, 0};
    const int2 ii = LoadIds<K>(a, i);
    id[0] = ii.x;
    id[1] = ii.y;
    double d[Tr::D];
#pragma unroll
    for (int k = 0; k < Tr::D; ++k) d[k] = a.data[i * Tr::D + k];
    const double* p[2] = {nullptr, nullptr};
    int64_t delta[2] = {0, 0};
    int tan[2] = {S0, S1};
    bool cst[2] = {false, false};
    int64_t pjo[2] = {-1, -1};
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const PbDev pb = a.pbs[id[j]];
      p[j] = (pb.is_constant ? a.cstate : a.state) + pb.state_offset;
      delta[j] = pb.delta_offset;
      tan[j] = pb.tangent_size;
      cst[j] = pb.is_constant != 0;
      pjo[j] = pb.plus_jacobian_offset;
    }
    double x0[S0], x1[S1p];
#pragma unroll
    for (int k = 0; k < S0; ++k) x0[k] = p[0][k];
#pragma unroll
    for (int k = 0; k < S1; ++k) x1[k] = p[1][k];

    double r[NR], J0[NR * S0], J1[NR * S1p];
    bool ok = EvaluateFunctor<K, kJac>(d, x0, x1, r, J0, J1);
    if (ok && a.check_finite) {
      bool bad = AnyNonFinite<NR>(r);
      if constexpr (kJac) bad = bad || AnyNonFinite<NR * S0>(J0) || AnyNonFinite<NR * S1>(J1);
      ok = !bad;
    }
    if constexpr (kJac) {
      // Local Jacobian = ambient Jacobian * PlusJacobian
      // (cuda_evaluator_kernel.h:355-371; residual_block.cc:133-156).
      if (pjo[0] >= 0) {
        const double* PJ = a.plus_jacobians + pjo[0];
        const int t = tan[0];
        double L[NR * S0];
#pragma unroll
        for (int k = 0; k < NR; ++k)
#pragma unroll
          for (int c = 0; c < S0; ++c) {
            double s = 0.0;
            if (c < t) {
#pragma unroll
              for (int m = 0; m < S0; ++m) s += J0[k * S0 + m] * PJ[m * t + c];
            }
            L[k * S0 + c] = s;
          }
#pragma unroll
        for (int q = 0; q < NR * S0; ++q) J0[q] = L[q];
      }
      if (S1 > 0 && pjo[1] >= 0) {
        const double* PJ = a.plus_jacobians + pjo[1];
        const int t = tan[1];
        double L[NR * S1p];
#pragma unroll
        for (int k = 0; k < NR; ++k)
#pragma unroll
          for (int c = 0; c < S1; ++c) {
            double s = 0.0;
            if (c < t) {
#pragma unroll
              for (int m = 0; m < S1; ++m) s += J1[k * S1p + m] * PJ[m * t + c];
            }
            L[k * S1p + c] = s;
          }
#pragma unroll
        for (int q = 0; q < NR * S1p; ++q) J1[q] = L[q];
      }
    }
    cost = LossAndCorrect<K, kLoss, kJac>(a.loss, a.apply_loss, r, J0, J1);
    if (!ok) {
      cost = 0.0;
      *a.status = 1;
    } else {
      if (want_grad)
        AddGradient<K>(cst[0] ? nullptr : a.gradient + delta[0],
                       (S1 > 0 && !cst[1]) ? a.gradient + delta[1] : nullptr, tan[0], tan[1], r,
                       J0, J1);
      const int64_t gi = a.gindex ? a.gindex[i] : a.first + i;
      if (a.residuals) {
        double* dst = a.residuals + a.residual_layout[gi];
#pragma unroll
        for (int k = 0; k < NR; ++k) dst[k] = r[k];
      }
      if (want_jac) {
        // WriteJacobians (cuda_evaluator_kernel.h:260-294): row k of the
        // a-th active slot goes to values + offsets[layout[gi] + a*kR + k].
        int64_t q = a.jac_layout[gi];
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          if (cst[j]) continue;
#pragma unroll
          for (int k = 0; k < NR; ++k) {
            double* dst = a.jacobian + a.jac_offsets[q++];
            if (j == 0) {
#pragma unroll
              for (int c = 0; c < S0; ++c)
                if (c < tan[0]) dst[c] = J0[k * S0 + c];
            } else {
#pragma unroll
              for (int c = 0; c < S1; ++c)
                if (c < tan[1]) dst[c] = J1[k * S1p + c];
            }
          }
        }
      }
    }
  }
  // One partial per wave (the wave's 64 blocks are the affine kernels'
  // chunk, so both paths sum the same partials in the same order).
  double w = cost;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) w += __shfl_xor(w, off, kWave);
  if ((threadIdx.x & (kWave - 1)) == 0)
    a.partials[(int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave] = w;
}

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

template <int S>
__global__ __launch_bounds__(kBlockThreads) void GradientChunkReduceKernel(const GradArgs g,
                                                                           const GradChunks ch) {
  const int64_t p = (int64_t)blockIdx.x * kBlockThreads + threadIdx.x;
  if (p >= g.count) return;
  double acc[S];
#pragma unroll
  for (int c = 0; c < S; ++c) acc[c] = 0.0;
  for (int64_t q = ch.chunk_off[p]; q < ch.chunk_off[p + 1]; ++q)
#pragma unroll
    for (int c = 0; c < S; ++c) acc[c] += ch.partial[q * S + c];
  double* dst = g.grad + g.delta_base + (int64_t)S * (g.lo + p);
#pragma unroll
  for (int c = 0; c < S; ++c) dst[c] += acc[c];
}

// Fused-gradient slot 0 (FusedGrad): each chunk of a parameter block's
// block list sums the blocks' written contributions (S of the SP doubles
// per block; two 64-byte sectors per block instead of the Jacobian cell
// and residual pair), a fixed butterfly, then GradientChunkReduceKernel.
template <int S, int SP>
__global__ __launch_bounds__(kBlockThreads) void GradientContribKernel(const double* contrib,
                                                                       const int32_t* perm,
                                                                       const GradChunks ch) {
  static_assert(SP % 2 == 0 && SP >= S, "16-byte records");
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const int64_t cid = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  if (cid >= ch.nchunks) return;
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
template <int S>
__global__ __launch_bounds__(kBlockThreads) void GradientBoundaryKernel(const double* side,
                                                                        int64_t count,
                                                                        double* grad,
                                                                        int64_t delta_base) {
  static_assert(S <= 3, "entries hold 3 sums and the id");
  const int64_t e = (int64_t)blockIdx.x * kBlockThreads + threadIdx.x;
  if (e >= count) return;
  const double key = side[4 * e + 3];
  if (e > 0 && side[4 * (e - 1) + 3] == key) return;
  double acc[S];
#pragma unroll
  for (int c = 0; c < S; ++c) acc[c] = 0.0;
  for (int64_t f = e; f < count && side[4 * f + 3] == key; ++f)
#pragma unroll
    for (int c = 0; c < S; ++c) acc[c] += side[4 * f + c];
  double* dst = grad + delta_base + (int64_t)S * (int64_t)key;
#pragma unroll
  for (int c = 0; c < S; ++c) dst[c] += acc[c];
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
  constexpr int NR = Tr::NR, NB = Tr::NB, S0 = Tr::S0, S1 = Tr::S1;
  const int64_t i = (int64_t)blockIdx.x * kBlockThreads + threadIdx.x;
  if (i >= a.n) return;
  const int64_t gi = a.gindex ? a.gindex[i] : a.first + i;
  const int2 ii = LoadIds<K>(a, i);
  const int32_t ids[2] = {ii.x, ii.y};
  const int64_t res = a.residual_layout[gi];
  int64_t q = a.jac_layout[gi];
  double acc[NR];
#pragma unroll
  for (int k = 0; k < NR; ++k) acc[k] = 0.0;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const PbDev pb = a.pbs[ids[j]];
    if (pb.is_constant) continue;
    const int S = j == 0 ? S0 : S1;
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
template <class K, bool kCrs>
__global__ __launch_bounds__(kBlockThreads) void CgnrMultiplyKernel(const GroupArgs a,
                                                                    const double* x, double* y) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, N = Tr::N;
  static_assert(Tr::NB == 2 && NR == 2 && S1 == 3, "Snavely-shaped groups");
  constexpr int S0p = (S0 + 1) & ~1;
  constexpr int kImg = kWave * NR * N;        // doubles of one wave's Jacobian image
  constexpr int kPieces = kImg / (2 * kWave);  // 16-byte DMA pieces per lane
  static_assert(kImg % (2 * kWave) == 0 && (kWave * NR * S0) % (2 * kWave) == 0, "16-B pieces");
  __shared__ double img[kWavesPerBlock][kImg];
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const int64_t nchunks = (a.n + kWave - 1) / kWave;
  const int64_t c = (int64_t)blockIdx.x * kWavesPerBlock + wave;
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

// First pass of the cost reduction when there are many partials: workgroup
// b sums partials [b*per, (b+1)*per) in a fixed order.
__global__ __launch_bounds__(kBlockThreads) void PartialSumKernel(const double* partials,
                                                                  int64_t n, int64_t per,
                                                                  double* out) {
  __shared__ double lds_sum[kWavesPerBlock];
  const int64_t begin = (int64_t)blockIdx.x * per;
  const int64_t end = begin + per < n ? begin + per : n;
  double v = 0.0;
  for (int64_t k = begin + threadIdx.x; k < end; k += kBlockThreads) v += partials[k];
  const double t = WorkgroupSum(v, lds_sum);
  if (threadIdx.x == 0) out[blockIdx.x] = t;
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

// Copies slot-0 parameter blocks [lo, lo + count) of the state into the
// packed table at a 16-byte-aligned stride (once per evaluation: 13,682
// cameras = 1.1 MB for BAL problem-13682).
__global__ __launch_bounds__(256) void RepackSlot0Kernel(const double* state, int64_t state_base,
                                                         int size, int stride, int32_t lo,
                                                         int64_t count, double* packed) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t b = t / stride;
  const int k = (int)(t - b * stride);
  if (b >= count) return;
  packed[t] = k < size ? state[state_base + (int64_t)size * (lo + b) + k] : 0.0;
}

}  // namespace cse

#endif  // CSE_EVALUATE_KERNEL_HPP_
