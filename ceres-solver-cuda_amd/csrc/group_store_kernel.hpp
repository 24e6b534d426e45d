// group_store_kernel.hpp -- the BlockSparseMatrix residual+Jacobian kernel
// of the Snavely camera with kW-wave workgroups over kW consecutive 64-block
// chunks (shipped: kW = 4, EvaluateAffineChunksGroupStore).  Each wave
// evaluates its chunk as EvaluateAffineChunksTwoRoundW1 does (LDS-DMA camera
// gather, the closed-form functor, loss and Corrector, cost partial in the
// same slot); then the workgroup's F cells, E cells and residuals are staged
// together in LDS, in output order, and written as long contiguous runs:
// the workgroup's four chunks own one 36 KiB F run, one 12 KiB E run and one
// 4 KiB residual run (block_jacobian_writer.cc:75-149: all E cells, then all
// F cells, in block order), 52 KiB of LDS (3 workgroups, 12 waves per CU),
// and the image [F | E | R] is cut into 13 KiB per wave (kSched 0): wave 0
// stores F[0, 13 KiB), wave 1 F[13, 26), wave 2 F[26, 36) and E[0, 3), wave
// 3 E[3, 12) and the residuals -- one or two runs a wave instead of three
// short segments (9, 3 and 1 KiB) per wave.
//
// Measured (same-process interleaved A/Bs against the
// one-wave-workgroup kernel, bit-identical outputs): -1.4 % to -2.4 % on
// six boxes (profiles/round5/r5a-r5d, r5f, r5g).  Other shapes of the
// tuning build (kW = 2, 3, 5, 6, 8; 8 waves per CU; waves 0-2 taking F in
// thirds and wave 3 E and R, kSched 1; two LDS phases; a persistent
// pipelined form; stores in flight capped per wave, kVm) were slower.
//
// Used when the group's residual, E and F bases are 64-byte aligned (then
// every workgroup's runs are: 9216, 3072 and 1024 bytes per chunk) and both
// outputs are requested; otherwise the one-wave kernel, whose sector-window
// tail handles any alignment.  The last, partial workgroup stores each
// chunk through the slow tail.  Gradient atomics (gradient_mode 2) as the
// one-wave kernel.  The CompressedRowSparseMatrix form (kCrs) is built only
// on request (-DCSE_GROUP_STORE_CRS=1): measured slower than the one-wave
// CRS kernel, as was a fused-gradient form (removed).
#ifndef CSE_GROUP_STORE_KERNEL_HPP_
#define CSE_GROUP_STORE_KERNEL_HPP_

#include "evaluate_kernel.hpp"

namespace cse {

// KiB per chunk of each output region (Snavely, BSM): F 9, E 3, residuals 1.
constexpr int kQuadFk = 9, kQuadEk = 3, kQuadRk = 1;

// One store run: N instructions of 1 KiB, the data in q[J0 .. J0 + N),
// base = the run's first byte + 4096 (+ 16 * lane); N <= 16.
template <int N, int J0>
__device__ __forceinline__ void QuadRun(double* base, const cse_v4i* q) {
  static_assert(N <= 16, "two base registers per run");
  if constexpr (N > 0) SegmentStoresFrom<0, N>(base, base + 1024, q + J0);
}

// Tuning build (kVm > 0): the same run with at most kVm of the wave's
// stores in flight (s_waitcnt vmcnt after each store past the kVm-th), so
// that a CU's memory queue holds fewer stores ahead of other waves' loads.
template <int kVm, int kJ, int kCount, int kDone>
__device__ __forceinline__ void QuadRunThrottled(double* b0, double* b1, const cse_v4i* q) {
  if constexpr (kJ < kCount) {
    StoreNt16<(kJ % 8) * 1024 - 4096, 0>(kJ < 8 ? b0 : b1, q[kJ]);
    if constexpr (kDone + kJ + 1 > kVm) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kVm) : "memory");
    QuadRunThrottled<kVm, kJ + 1, kCount, kDone>(b0, b1, q);
  }
}

// Wave w's part of the workgroup image [F | E | R] (KiB): [lo, hi).  The
// CompressedRowSparseMatrix form has one Jacobian region: kFk = 12, kEk = 0.
template <int kW, int kSched, int w, int kFk = kQuadFk, int kEk = kQuadEk>
struct QuadPart {
  static constexpr int F = kFk * kW, E = kEk * kW, R = kQuadRk * kW;
  static constexpr int T = F + E + R;
  static constexpr int lo = kSched == 1 ? (w < 3 ? w * F / 3 : F) : T * w / kW;
  static constexpr int hi = kSched == 1 ? (w < 3 ? (w + 1) * F / 3 : T) : T * (w + 1) / kW;
  static constexpr int N = hi - lo;
  // region r's overlap with [lo, hi): start (image KiB) and count
  static constexpr int rb(int r) { return r == 0 ? 0 : r == 1 ? F : F + E; }
  static constexpr int re(int r) { return r == 0 ? F : r == 1 ? F + E : T; }
  static constexpr int s(int r) { return lo > rb(r) ? lo : rb(r); }
  static constexpr int n(int r) { return (hi < re(r) ? hi : re(r)) - s(r) > 0 ? (hi < re(r) ? hi : re(r)) - s(r) : 0; }
};

// Read wave w's pieces from the workgroup image and store them, region by
// region (at most three runs).
template <int kW, int kSched, int w, int kFk, int kEk, int kVm>
__device__ __forceinline__ void QuadTail(const double* img, double* const bases[3], int lane,
                                         double* v_partial, double v_wsum, bool failed,
                                         int* status_dst) {
  using P = QuadPart<kW, kSched, w, kFk, kEk>;
  constexpr int N = P::N;
  static_assert(N > 0 && N <= 24, "pieces per wave");
  cse_v4i q[N];
  const double2* im2 = reinterpret_cast<const double2*>(img);
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const double2 v = im2[(P::lo + j) * kWave + lane];
    q[j] = AsV4i(v.x, v.y);
  }
  // run bases: region start + offset inside the region (KiB = 128 doubles)
  double* b0 = bases[0] + 128 * (P::s(0) - P::rb(0)) + 2 * lane + 512;
  double* b1 = bases[1] + 128 * (P::s(1) - P::rb(1)) + 2 * lane + 512;
  double* b2 = bases[2] + 128 * (P::s(2) - P::rb(2)) + 2 * lane + 512;
  asm volatile("" : "+v"(v_partial), "+v"(v_wsum));
  asm volatile("" ::"v"(b0), "v"(b1), "v"(b2));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if constexpr (kVm > 0) {
    QuadRunThrottled<kVm, 0, P::n(0), 0>(b0, b0 + 1024, q);
    QuadRunThrottled<kVm, 0, P::n(1), P::n(0)>(b1, b1 + 1024, q + P::n(0));
    QuadRunThrottled<kVm, 0, P::n(2), P::n(0) + P::n(1)>(b2, b2 + 1024, q + P::n(0) + P::n(1));
  } else {
    QuadRun<P::n(0), 0>(b0, q);
    QuadRun<P::n(1), P::n(0)>(b1, q);
    QuadRun<P::n(2), P::n(0) + P::n(1)>(b2, q);
  }
  if (lane == 0) {
    StoreB64(v_partial, v_wsum);
    if (failed) StoreB32(status_dst, 1);
  }
  KeepAlive<N>(q);
  asm volatile("" ::"v"(b0), "v"(b1), "v"(b2), "v"(v_partial), "v"(v_wsum));
}

template <int kW, int kSched, int kFk = kQuadFk, int kEk = kQuadEk, int kVm = 0, int w = 0>
__device__ __forceinline__ void QuadTailFor(int wave, const double* img, double* const bases[3], int lane,
                                            double* v_partial, double v_wsum, bool failed,
                                            int* status_dst) {
  if constexpr (w < kW) {
    if (wave == w) {
      QuadTail<kW, kSched, w, kFk, kEk, kVm>(img, bases, lane, v_partial, v_wsum, failed, status_dst);
      return;
    }
    QuadTailFor<kW, kSched, kFk, kEk, kVm, w + 1>(wave, img, bases, lane, v_partial, v_wsum, failed, status_dst);
  }
}

// Waves per SIMD the register allocation must allow: the LDS bound.
template <int kW, int kPadKiB>
constexpr int kQuadWavesPerEu = ((160 / (13 * kW + kPadKiB)) * kW + 3) / 4;

// kCrs: CompressedRowSparseMatrix values (block_jacobian_writer's CRS
// sibling, compressed_row_jacobian_writer.cc): a block's NR rows of N = 12
// columns are contiguous, so a workgroup's four chunks own one 48 KiB run of
// rows and one 4 KiB run of residuals; each lane stages its rows with the
// group's column offsets (camera and point columns in either order).
// kPrio (tuning): the wave at s_setprio kPrio from its start to its store
// tail, so that waves still loading issue ahead of waves storing.
template <class K, int kLoss, int kW, int kSched, int kPadKiB, bool kCrs = false, int kVm = 0, int kPrio = 0>
__global__ __launch_bounds__(kW * kWave) __attribute__((amdgpu_waves_per_eu(kQuadWavesPerEu<kW, kPadKiB>))) void
EvaluateAffineChunksGroupStore(const GroupArgs a) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p;
  constexpr int N = S0 + S1;
  static_assert(NR == 2 && S0 == 9 && S1 == 3, "Snavely-shaped kinds");
  // KiB per chunk of the Jacobian regions: BSM F 9 and E 3, CRS rows 12
  constexpr int kFk = kCrs ? kQuadFk + kQuadEk : kQuadFk, kEk = kCrs ? 0 : kQuadEk;
  constexpr int kImg = (13 * kW + kPadKiB) * 128;  // doubles
  __shared__ __attribute__((aligned(16))) double img[kImg];
  const int lane = threadIdx.x & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int64_t num_chunks = (a.n + kWave - 1) / kWave;
  const int64_t c = (int64_t)blockIdx.x * kW + w;
  const bool has = c < num_chunks;
  const int64_t i0 = c * kWave;
  const int64_t rem = a.n - i0;
  const int nw = !has ? 0 : rem < kWave ? (int)rem : kWave;
  const bool active = lane < nw;
  const int64_t i = active ? i0 + lane : (a.n > 0 ? a.n - 1 : 0);
  double* fw = img + w * (kFk * 128);  // this wave's F cells or rows (and its gather landing area)
  double* ew = img + kFk * kW * 128 + w * (NR * S1 * kWave);
  double* rw = img + (kFk + kEk) * kW * 128 + w * (NR * kWave);

  double r[NR], J0[NR * S0], J1[NR * S1p];
  bool ok = true;
  double cost = 0.0;
  if constexpr (kPrio > 0) __builtin_amdgcn_s_setprio(kPrio);
  if (has) {
    AffineInputs<K> in;
    const long long b = __builtin_nontemporal_load(reinterpret_cast<const long long*>(a.ids) + i);
    const int2 id = make_int2((int)b, (int)(b >> 32));
    GatherCoopDma<K>(a, i, id, &in, fw, lane);
    ok = EvaluateFunctor<K, true>(in.d, in.x0, in.x1, r, J0, J1);
    if (ok && a.check_finite)
      ok = !(AnyNonFinite<NR>(r) || AnyNonFinite<NR * S0>(J0) || AnyNonFinite<NR * S1>(J1));
    cost = LossAndCorrect<K, kLoss, true>(a.loss, a.apply_loss, r, J0, J1, a.residuals != nullptr);
    if (a.gradient != nullptr && active) {  // gradient_mode 2: FP64 atomics, as the reference
      AddGradientSlot<NR, S0>(a.gradient + a.delta_base[0] + (int64_t)S0 * in.id0, S0, r, J0);
      AddGradientSlot<NR, S1p>(a.gradient + a.delta_base[1] + (int64_t)S1 * in.id1, S1, r, J1);
    }
  }
  const double wsum = WaveSumLane0(active ? cost : 0.0);
  const bool failed = __ballot(active && !ok) != 0;
  double* v_partial = a.partials + c;
  const int64_t wg0 = (int64_t)blockIdx.x * kW * kWave;  // the workgroup's first block
  // CRS: the first row's offset (the slots' first columns, either order)
  const int64_t row0 = a.jac_base[0][0] < a.jac_base[1][0] ? a.jac_base[0][0] : a.jac_base[1][0];
  double* fbase = !a.jacobian ? nullptr
                  : kCrs      ? a.jacobian + row0 + (int64_t)NR * N * wg0
                              : a.jacobian + a.jac_base[0][0] + a.jac_stride[0] * wg0;
  double* ebase = kCrs || !a.jacobian ? fbase : a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * wg0;
  double* rbase = a.residuals ? a.residuals + a.res_base + (int64_t)NR * wg0 : nullptr;
  const bool full = wg0 + kW * kWave <= a.n;
  const bool fast = full && fbase && rbase &&
                    ((reinterpret_cast<uintptr_t>(fbase) | reinterpret_cast<uintptr_t>(ebase) |
                      reinterpret_cast<uintptr_t>(rbase)) & 63) == 0;
  if (fast) {
    // Stage the wave's cells in output order (every lane active here).
    if constexpr (kCrs) {
      double* row = fw + lane * NR * N;
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        const int c0 = (int)(a.jac_base[0][k] - row0), c1 = (int)(a.jac_base[1][k] - row0);
#pragma unroll
        for (int cc = 0; cc < S0; ++cc) row[c0 + cc] = J0[k * S0 + cc];
#pragma unroll
        for (int cc = 0; cc < S1; ++cc) row[c1 + cc] = J1[k * S1p + cc];
      }
    } else {
#pragma unroll
      for (int q = 0; q < NR * S0; q += 2)
        *reinterpret_cast<double2*>(fw + lane * NR * S0 + q) = make_double2(J0[q], J0[q + 1]);
#pragma unroll
      for (int q = 0; q < NR * S1; q += 2)
        *reinterpret_cast<double2*>(ew + lane * NR * S1 + q) = make_double2(J1[q], J1[q + 1]);
    }
    *reinterpret_cast<double2*>(rw + lane * NR) = make_double2(r[0], r[1]);
    if constexpr (kPrio > 0) __builtin_amdgcn_s_setprio(0);
    __syncthreads();
    double* const bases[3] = {fbase, ebase, rbase};
    QuadTailFor<kW, kSched, kFk, kEk, kVm>(w, img, bases, lane, v_partial, wsum, failed, a.status);
    return;
  }
  // The last (partial) workgroup or unaligned outputs: each wave its own
  // chunk through the slow tail, in its own F region (CRS: its 12 KiB of rows).
  __syncthreads();  // every wave's gather landing area is free again
  if (has) StageAndStore<K, true, kCrs>(a, fw, lane, active, i0, nw, r, J0, J1);
  if (lane == 0 && has) {  // slots past the last chunk stay 0 (zeroed at cse_create)
    *v_partial = wsum;
    if (failed) *a.status = 1;
  }
}

// Tuning build: the same with the image staged in two phases through 36 KiB
// (4 workgroups, 16 waves per CU): the F cells (each wave then stores its
// own chunk's 9 KiB F segment), then E and residuals in the same LDS (wave
// w < 3 stores a third of the E run, wave 3 the residuals).
template <class K, int kLoss>
__global__ __launch_bounds__(4 * kWave) __attribute__((amdgpu_waves_per_eu(4))) void
EvaluateAffineChunksGroupStore2P(const GroupArgs a) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p;
  static_assert(NR == 2 && S0 == 9 && S1 == 3, "Snavely-shaped kinds");
  constexpr int kW = 4;
  __shared__ __attribute__((aligned(16))) double img[kQuadFk * kW * 128];
  const int lane = threadIdx.x & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int64_t num_chunks = (a.n + kWave - 1) / kWave;
  const int64_t c = (int64_t)blockIdx.x * kW + w;
  const bool has = c < num_chunks;
  const int64_t i0 = c * kWave;
  const int64_t rem = a.n - i0;
  const int nw = !has ? 0 : rem < kWave ? (int)rem : kWave;
  const bool active = lane < nw;
  const int64_t i = active ? i0 + lane : (a.n > 0 ? a.n - 1 : 0);
  double* fw = img + w * (NR * S0 * kWave);
  double r[NR], J0[NR * S0], J1[NR * S1p];
  bool ok = true;
  double cost = 0.0;
  if (has) {
    AffineInputs<K> in;
    const long long b = __builtin_nontemporal_load(reinterpret_cast<const long long*>(a.ids) + i);
    GatherCoopDma<K>(a, i, make_int2((int)b, (int)(b >> 32)), &in, fw, lane);
    ok = EvaluateFunctor<K, true>(in.d, in.x0, in.x1, r, J0, J1);
    if (ok && a.check_finite)
      ok = !(AnyNonFinite<NR>(r) || AnyNonFinite<NR * S0>(J0) || AnyNonFinite<NR * S1>(J1));
    cost = LossAndCorrect<K, kLoss, true>(a.loss, a.apply_loss, r, J0, J1, a.residuals != nullptr);
  }
  const double wsum = WaveSumLane0(active ? cost : 0.0);
  const bool failed = __ballot(active && !ok) != 0;
  double* v_partial = a.partials + c;
  const int64_t wg0 = (int64_t)blockIdx.x * kW * kWave;
  double* fbase = a.jacobian ? a.jacobian + a.jac_base[0][0] + a.jac_stride[0] * wg0 : nullptr;
  double* ebase = a.jacobian ? a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * wg0 : nullptr;
  double* rbase = a.residuals ? a.residuals + a.res_base + (int64_t)NR * wg0 : nullptr;
  const bool full = wg0 + kW * kWave <= a.n;
  const bool fast = full && fbase && rbase &&
                    ((reinterpret_cast<uintptr_t>(fbase) | reinterpret_cast<uintptr_t>(ebase) |
                      reinterpret_cast<uintptr_t>(rbase)) & 63) == 0;
  if (fast) {
    const double2* im2 = reinterpret_cast<const double2*>(img);
    cse_v4i q[13];
    // phase 1: the wave's own F cells, read back as its 9 KiB segment
#pragma unroll
    for (int k = 0; k < NR * S0; k += 2)
      *reinterpret_cast<double2*>(fw + lane * NR * S0 + k) = make_double2(J0[k], J0[k + 1]);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const double2 v = im2[(9 * w + j) * kWave + lane];
      q[j] = AsV4i(v.x, v.y);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();  // every wave's F pieces are in registers
    // phase 2: E cells [0, 12 KiB) and residuals [12, 16 KiB) of the workgroup
#pragma unroll
    for (int k = 0; k < NR * S1; k += 2)
      *reinterpret_cast<double2*>(img + w * (NR * S1 * kWave) + lane * NR * S1 + k) =
          make_double2(J1[k], J1[k + 1]);
    *reinterpret_cast<double2*>(img + kQuadEk * kW * 128 + w * (NR * kWave) + lane * NR) =
        make_double2(r[0], r[1]);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const double2 v = im2[(4 * w + j) * kWave + lane];
      q[9 + j] = AsV4i(v.x, v.y);
    }
    double* f0 = fbase + 128 * 9 * w + 2 * lane + 512;
    double* s0 = (w < 3 ? ebase + 128 * 4 * w : rbase) + 2 * lane + 512;
    asm volatile("" : "+v"(v_partial));
    double v_wsum = wsum;
    asm volatile("" : "+v"(v_wsum));
    asm volatile("" ::"v"(f0), "v"(s0));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    QuadRun<9, 0>(f0, q);
    QuadRun<4, 9>(s0, q);
    if (lane == 0) {
      StoreB64(v_partial, v_wsum);
      if (failed) StoreB32(a.status, 1);
    }
    KeepAlive<13>(q);
    asm volatile("" ::"v"(f0), "v"(s0), "v"(v_partial), "v"(v_wsum));
    return;
  }
  __syncthreads();
  if (has) StageAndStore<K, true, false>(a, fw, lane, active, i0, nw, r, J0, J1);
  if (lane == 0 && has) {
    *v_partial = wsum;
    if (failed) *a.status = 1;
  }
}

// May the group take EvaluateAffineChunksGroupStore?  Both outputs, and the
// residual, E-cell and F-cell bases on 64-byte sectors.
// CRS: the residuals and the group's first row on 64-byte sectors (a block's
// NR x N rows are contiguous on the affine CRS path).
inline bool GroupStoreEligibleCrs(const GroupArgs& a) {
  if (!a.residuals || !a.jacobian) return false;
  const int64_t row0 = a.jac_base[0][0] < a.jac_base[1][0] ? a.jac_base[0][0] : a.jac_base[1][0];
  const uintptr_t m = reinterpret_cast<uintptr_t>(a.residuals + a.res_base) |
                      reinterpret_cast<uintptr_t>(a.jacobian + row0);
  return (m & 63) == 0;
}

inline bool GroupStoreEligible(const GroupArgs& a) {
  if (!a.residuals || !a.jacobian) return false;
  const uintptr_t m = reinterpret_cast<uintptr_t>(a.residuals + a.res_base) |
                      reinterpret_cast<uintptr_t>(a.jacobian + a.jac_base[0][0]) |
                      reinterpret_cast<uintptr_t>(a.jacobian + a.jac_base[1][0]);
  return (m & 63) == 0 && a.jac_stride[0] == 18 && a.jac_stride[1] == 6;
}

}  // namespace cse

#endif  // CSE_GROUP_STORE_KERNEL_HPP_
