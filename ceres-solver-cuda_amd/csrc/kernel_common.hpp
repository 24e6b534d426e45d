// kernel_common.hpp -- shared pieces of the gfx950 evaluator kernels.
//
// Kernel arguments, compile-time functor shapes, the autodiff of one
// residual block (include/ceres/internal/autodiff.h:314-381), the loss and
// Corrector step (cuda_evaluator_kernel.h:373-407 / residual_block.cc:
// 159-199), LDS-staged wave stores and the inline-asm store primitives.
#ifndef CSE_KERNEL_COMMON_HPP_
#define CSE_KERNEL_COMMON_HPP_

#include <stdint.h>

#include "functors.hpp"
#include "jet.hpp"
#include "loss.hpp"

namespace cse {

constexpr int kBlockThreads = 256;
constexpr int kWave = 64;
constexpr int kWavesPerBlock = kBlockThreads / kWave;
constexpr int kMaxSlots = 10;  // parameter blocks per residual block (table path)


// kImpossibleValue (internal/ceres/array_utils.h:52): the marker
// AutoDifferentiate pre-fills outputs with.
constexpr double kImpossibleValue = 1e302;

// Device copy of a parameter block (table path).  plus_jacobian_offset:
// >= 0 the explicit matrix, -1 none, kPlusJacobianQuaternion the
// CSE_MANIFOLD_QUATERNION_EUCLIDEAN manifold (built in registers).
constexpr int64_t kPlusJacobianQuaternion = -2;
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
  // Slot-0 parameter blocks repacked at a line-aligned stride (the affine
  // path's cooperative LDS-DMA gather; see RepackSlot0Kernel and
  // PackedRowDoubles).
  const double* packed0;
  int32_t packed0_lo;
  int32_t packed0_stride;  // doubles per row: PackedRowDoubles(S0)
  // Constant slot-0 blocks (a held camera, BlockSparseMatrix only): bit
  // (id - packed0_lo) of act0_bits set = active; the F cells of the active
  // blocks of chunk c start at fbase[c] (no cell for a constant block).
  const uint32_t* act0_bits;
  const int64_t* fbase;   // [chunks + 1] (64-block chunks), the last = end of the F cells
  // [chunks][16]: each full chunk's head and tail pieces of its F segment
  // (BSM) or row-block segment (CRS), in two 64-byte slots, for
  // HeldSectorFixupKernel.
  double* side;
  const int64_t* delta0;  // [slot-0 id - packed0_lo] delta offset of an active block
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
  // Fused gradient (EvaluateAffineChunksFused, see FusedGrad): the gradient
  // (delta offsets), the slot-1 wave-boundary entries [2 * chunks][4] and
  // the slot-0 per-block contributions J0^T r [n][S0p].
  double* gfused;
  double* gside;
  double* gcontrib;
  LossParams loss;
  int apply_loss;
  int check_finite;
  // kLossUser: the bytes of the group's loss object (cse_loss.user).
  double user_loss[kUserLossDoubles];
  // Table policy, found at cse_create (BuildTableRuns): per 64-block chunk
  // [flags, residual run start, first cell / row segment of each slot];
  // null = the kernel finds the runs from the offset tables.
  const int64_t* table_runs;
  // Table policy, slot 0 plain in every block (active, no manifold, tangent
  // size = size, state and delta offsets affine in the id; DetectPlain0):
  // its PbDev is formed from these, not loaded.
  int64_t plain0_state_base, plain0_delta_base;
  int32_t plain0;
};

// Layout tag of the argument blocks (GroupArgs, GradArgs, CamGradArgs),
// checked when a user functor kind registers kernels compiled in another TU
// (cse_register_functor): bump on any change to them.
constexpr uint64_t kGroupArgsTag = 0x6373654761310005ull;

// Compile-time shape of a functor kind: kR residuals, NB parameter blocks
// of sizes kSizes[0..NB) concatenated into N columns.
template <class K>
constexpr int SlotOffset(int j) {
  int o = 0;
  for (int b = 0; b < j; ++b) o += K::kSizes[b];
  return o;
}
template <class K>
constexpr int MaxSlotSize() {
  int m = 0;
  for (int b = 0; b < K::kNumBlocks; ++b) m = K::kSizes[b] > m ? K::kSizes[b] : m;
  return m;
}
// Values gathered for slot 0: K::kAmbient0 where the kind declares it (a
// slot-0 manifold: kSize0 is then the tangent size, the Jacobian's
// columns), else kSize0.
template <class K, class = void>
struct Ambient0 {
  static constexpr int value = K::kSize0;
};
template <class K>
struct Ambient0<K, decltype((void)K::kAmbient0)> {
  static constexpr int value = K::kAmbient0;
};
template <class K>
struct KindTraits {
  static constexpr int NR = K::kNumResiduals;
  static constexpr int NB = K::kNumBlocks;
  static constexpr int S0 = K::kSize0;   // slot-0 Jacobian columns (tangent)
  static constexpr int X0 = Ambient0<K>::value;  // slot-0 values (ambient)
  static constexpr int S1 = NB > 1 ? K::kSize1 : 0;
  static constexpr int S1p = S1 > 0 ? S1 : 1;
  static constexpr int D = K::kDataSize;
  static constexpr int N = SlotOffset<K>(NB);
  static constexpr int Size(int j) { return K::kSizes[j]; }
  static constexpr int Off(int j) { return SlotOffset<K>(j); }
  static constexpr int MaxSize() { return MaxSlotSize<K>(); }
};

// Does the kind declare that it may leave outputs unassigned?
template <class K, class = void>
struct MayLeaveOutputs {
  static constexpr bool value = false;
};
template <class K>
struct MayLeaveOutputs<K, decltype((void)K::kMayLeaveOutputs)> {
  static constexpr bool value = K::kMayLeaveOutputs;
};

// Is the kind one of the known-answer-test functors (general path, trivial
// loss only)?
template <class K, class = void>
struct TestOnly {
  static constexpr bool value = false;
};
template <class K>
struct TestOnly<K, decltype((void)K::kTestOnly)> {
  static constexpr bool value = K::kTestOnly;
};

// Does the kind run on the affine kernels only (no flat form for the
// table kernel)?
template <class K, class = void>
struct AffineOnly {
  static constexpr bool value = false;
};
template <class K>
struct AffineOnly<K, decltype((void)K::kAffineOnly)> {
  static constexpr bool value = K::kAffineOnly;
};

// Row stride (doubles) of the repacked slot-0 table that the LDS-DMA gather
// reads: the block's size rounded up to 16 bytes and then to a power of two
// up to 128 bytes, so that no row straddles a 128-byte L2 line (16 doubles
// for the 9-double BAL camera).  Each DMA instruction then touches one line
// per row instead of 1.5 on average: the residual-only evaluation of
// problem-13682 went from 0.487 to 0.420 ms (profiles/round2/s4e).
constexpr int PackedRowDoubles(int s) {
  const int p = (s + 1) & ~1;
  return p <= 2 ? 2 : p <= 4 ? 4 : p <= 8 ? 8 : p <= 16 ? 16 : p;
}

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

// Any of x[0..n) equal to kImpossibleValue (an unassigned output)?  Bit
// comparison, for the same reason.
template <int kCount>
CSE_HD bool AnyImpossible(const double* x) {
  bool any = false;
#pragma unroll
  for (int i = 0; i < kCount; ++i)
    any = any || __builtin_bit_cast(uint64_t, x[i]) == __builtin_bit_cast(uint64_t, kImpossibleValue);
  return any;
}

// x of lane (lane ^ kOff), kOff < 32, by ds_swizzle in bit mode (and mask
// 0x1f, xor mask kOff): no address VGPRs and no range checks, where
// __shfl_xor costs four VALU instructions per step.
template <int kOff>
__device__ __forceinline__ double SwizzleXor(double x) {
  static_assert(kOff > 0 && kOff < 32, "ds_swizzle bit mode acts within 32 lanes");
  constexpr int kPattern = (kOff << 10) | 0x1f;
  const int lo = __builtin_amdgcn_ds_swizzle(__double2loint(x), kPattern);
  const int hi = __builtin_amdgcn_ds_swizzle(__double2hiint(x), kPattern);
  return __hiloint2double(hi, lo);
}

// The sum of v over the wave's 64 lanes, in lane 0, in a fixed order:
// butterflies over lane ^ 1, 2, 4, 8, 16 (each 32-lane half's sum in all of
// its lanes), then lane 0's half plus lane 32's.  Every lane must be active.
// The affine and the table kernels both use it, so their per-wave cost
// partials are bit-identical.
__device__ __forceinline__ double WaveSumLane0(double v) {
  v += SwizzleXor<1>(v);
  v += SwizzleXor<2>(v);
  v += SwizzleXor<4>(v);
  v += SwizzleXor<8>(v);
  v += SwizzleXor<16>(v);
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), 32);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), 32);
  return v + __hiloint2double(hi, lo);
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
__device__ __forceinline__ void WaveStore(const double* lds, double* dst, int count, int lane) {
  if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    const int pairs = count >> 1;
    for (int t = lane; t < pairs; t += kWave) {
      const double2 v = *reinterpret_cast<const double2*>(lds + 2 * t);
      __builtin_nontemporal_store(v.x, dst + 2 * t);
      __builtin_nontemporal_store(v.y, dst + 2 * t + 1);
    }
    if ((count & 1) && lane == 0) dst[count - 1] = lds[count - 1];
  } else {
    for (int t = lane; t < count; t += kWave) dst[t] = lds[t];
  }
}

// AutoDifferentiate (include/ceres/internal/autodiff.h:314-381) for the
// two-slot affine kernels: seed one Jet per parameter with its unit vector,
// pre-fill the outputs with kImpossibleValue (:355-360), run the functor,
// split the partials into the row-major per-block Jacobians.  kJac = false
// runs the functor on plain doubles.  The Snavely camera's Jacobian is the
// same product rule written out once (SnavelyJacobianByHand); its Jet form
// is the distinct kind SnavelyJetKind (cse_options.jacobian_form).
template <class K, bool kJac>
CSE_HD bool EvaluateFunctor(const double* d, const double* x0, const double* x1, double* r,
                            double* J0, double* J1) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, X0 = Tr::X0, S1 = Tr::S1, S1p = Tr::S1p, N = X0 + S1;
  if constexpr (kJac) {
#ifdef __HIP_DEVICE_COMPILE__
    if constexpr (std::is_same<K, SnavelyKind>::value)
      return SnavelyJacobianByHand(d, x0, x1, r, J0, J1);
#endif
    Jet<N> j0[X0], j1[S1p], out[NR];
#pragma unroll
    for (int k = 0; k < X0; ++k) j0[k] = Jet<N>(x0[k], k);
#pragma unroll
    for (int k = 0; k < S1; ++k) j1[k] = Jet<N>(x1[k], X0 + k);
#pragma unroll
    for (int k = 0; k < NR; ++k) out[k] = Jet<N>::Filled(kImpossibleValue);
    const bool ok = K::Evaluate(d, j0, j1, out);
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      r[k] = out[k].a;
      if constexpr (X0 == S0) {
#pragma unroll
        for (int c = 0; c < S0; ++c) J0[k * S0 + c] = out[k].v[c];
      } else {  // slot-0 manifold: ambient row times the plus-Jacobian
        K::TangentRow(x0, out[k].v, J0 + k * S0);
      }
#pragma unroll
      for (int c = 0; c < S1; ++c) J1[k * S1p + c] = out[k].v[X0 + c];
    }
    return ok;
  } else {
#pragma unroll
    for (int k = 0; k < NR; ++k) r[k] = kImpossibleValue;
    return K::Evaluate(d, x0, x1, r);
  }
}

// The same over the concatenated parameter vector x[N] of any number of
// slots (the table kernel): J is kR x N row-major, slot j in columns
// [Off(j), Off(j) + Size(j)).
template <class K, bool kJac>
CSE_HD bool EvaluateFunctorFlat(const double* d, const double* x, double* r, double* J) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, N = Tr::N;
  if constexpr (kJac) {
#ifdef __HIP_DEVICE_COMPILE__
    // The same arithmetic as the affine kernels (EvaluateFunctor): the two
    // store paths write bit-identical Jacobians.
    if constexpr (std::is_same<K, SnavelyKind>::value) {
      double J0[18], J1[6];
      const bool ok = SnavelyJacobianByHand(d, x, x + 9, r, J0, J1);
#pragma unroll
      for (int k = 0; k < 2; ++k) {
#pragma unroll
        for (int c = 0; c < 9; ++c) J[k * N + c] = J0[9 * k + c];
#pragma unroll
        for (int c = 0; c < 3; ++c) J[k * N + 9 + c] = J1[3 * k + c];
      }
      return ok;
    }
#endif
    Jet<N> xj[N], out[NR];
#pragma unroll
    for (int k = 0; k < N; ++k) xj[k] = Jet<N>(x[k], k);
#pragma unroll
    for (int k = 0; k < NR; ++k) out[k] = Jet<N>::Filled(kImpossibleValue);
    const bool ok = K::EvaluateFlat(d, xj, out);
#pragma unroll
    for (int k = 0; k < NR; ++k) {
      r[k] = out[k].a;
#pragma unroll
      for (int c = 0; c < N; ++c) J[k * N + c] = out[k].v[c];
    }
    return ok;
  } else {
#pragma unroll
    for (int k = 0; k < NR; ++k) r[k] = kImpossibleValue;
    return K::EvaluateFlat(d, x, r);
  }
}

// Loss and correction (cuda_evaluator_kernel.h:373-407 /
// residual_block.cc:159-199) on r and the per-slot Jacobians J0 (kR x S0)
// and J1 (kR x S1).  Returns the block cost.  correct = false (a cost-only
// evaluation: no residual or Jacobian leaves the kernel) skips the
// Corrector, as ResidualBlock::Evaluate's early exit does when neither
// Jacobians nor residuals are output (residual_block.cc:175-179).
template <class K, int kLoss, bool kJac>
CSE_HD double LossAndCorrect(const LossParams& lp, bool apply_loss, double* r, double* J0,
                             double* J1, bool correct = true, const double* user_loss = nullptr) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p;
  double sq = 0.0;
#pragma unroll
  for (int k = 0; k < NR; ++k) sq += r[k] * r[k];
  const bool robust = (kLoss != kLossTrivial || lp.scaled) && apply_loss;
  if (!robust) return 0.5 * sq;
  double rho[3];
  EvaluateLoss<kLoss, K>(lp, sq, rho, user_loss);
  if (!kJac && !correct) return 0.5 * rho[0];
  const Corrector corr(sq, rho);
  if constexpr (kJac) {
    corr.template CorrectJacobian<NR, S0>(r, J0);
    if constexpr (S1 > 0) corr.template CorrectJacobian<NR, S1p>(r, J1);
  }
  corr.template CorrectResiduals<NR>(r);
  return 0.5 * rho[0];
}

// ---------------------------------------------------------------------------
// Inline-asm store primitives.  Why the affine kernel's stores are inline
// asm (measured, tools/membench2.hip): on gfx950 a vector-memory store
// reads its address and data VGPRs after issue, when the store reaches the
// head of the CU's memory queue.  An instruction that overwrites one of
// those VGPRs before then stalls the wave until the store drains -- under a
// saturated write stream that is microseconds -- so a wave whose register
// allocator reuses a store's VGPRs for the next store's address issues its
// stores one queue-drain at a time (1.64 ms against 1.24 ms for the same
// memory path with the stores back to back).  These stores take operands
// the compiler keeps live to the end of the kernel (KeepAlive).
// ---------------------------------------------------------------------------
typedef int cse_v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ cse_v4i AsV4i(double a, double b) {
  const double2 v = make_double2(a, b);
  cse_v4i d;
  __builtin_memcpy(&d, &v, 16);
  return d;
}

// 16-byte store at base + kOff bytes (kOff in [-4096, 4095]).  kPol: the
// cache policy, 0 = nt sc1 (streaming, not kept in the XCD's L2; 6-8 %
// faster than nt alone on the evaluator's output stream, profiles/r02),
// 1 = default policy (small scattered stores whose lines neighbours share).
template <int kOff, int kPol = 0>
__device__ __forceinline__ void StoreNt16(double* base, const cse_v4i& d) {
  static_assert(kOff >= -4096 && kOff <= 4095, "global offset out of range");
  static_assert(kPol == 0 || kPol == 1, "cache policies: 0 streaming, 1 default");
  if constexpr (kPol == 1)
    asm volatile("global_store_dwordx4 %0, %1, off offset:%2" ::"v"(base), "v"(d), "i"(kOff)
                 : "memory");
  else
    asm volatile("global_store_dwordx4 %0, %1, off offset:%2 sc1 nt" ::"v"(base), "v"(d),
                 "i"(kOff)
                 : "memory");
}

// Pieces kJ.. of a wave segment: piece j of lane l at b + 16 * (64 (j % 8))
// - 4096 bytes, b = b0 for j < 8 and b1 after (1 KiB per instruction).
template <int kJ, int kCount>
__device__ __forceinline__ void SegmentStoresFrom(double* b0, double* b1, const cse_v4i* q) {
  if constexpr (kJ < kCount) {
    StoreNt16<(kJ % 8) * 1024 - 4096>(kJ < 8 ? b0 : b1, q[kJ]);
    SegmentStoresFrom<kJ + 1, kCount>(b0, b1, q);
  }
}

// One double (8-byte vector store, default cache policy) from the calling
// lanes; the caller masks.  Both operands are VGPRs computed before the
// store tail.
__device__ __forceinline__ void StoreB64(double* addr, double value) {
  asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(addr), "v"(value) : "memory");
}
__device__ __forceinline__ void StoreB32(int* addr, int value) {
  asm volatile("global_store_dword %0, %1, off" ::"v"(addr), "v"(value) : "memory");
}
// One double at addr + kOff bytes, default cache policy (the fused
// gradient's scattered slot-1 rows: neighbouring lanes share lines in L2).
template <int kOff>
__device__ __forceinline__ void StoreB64At(double* addr, double value) {
  asm volatile("global_store_dwordx2 %0, %1, off offset:%2" ::"v"(addr), "v"(value), "i"(kOff)
               : "memory");
}

template <int kCount>
__device__ __forceinline__ void KeepAlive(const cse_v4i* q) {
#pragma unroll
  for (int j = 0; j < kCount; ++j) asm volatile("" ::"v"(q[j]));
}

}  // namespace cse

#endif  // CSE_KERNEL_COMMON_HPP_
