// group_store_kernel.hpp -- the BlockSparseMatrix residual+Jacobian kernel
// of the Snavely camera with 4-wave workgroups over 4 consecutive 64-block
// chunks (EvaluateAffineChunksGroupStore).  Each wave
// evaluates its chunk as EvaluateAffineChunksTwoRoundW1 does (LDS-DMA camera
// gather, the closed-form functor, loss and Corrector, cost partial in the
// same slot); then the workgroup's F cells, E cells and residuals are staged
// together in LDS, in output order, and written as long contiguous runs:
// the workgroup's four chunks own one 36 KiB F run, one 12 KiB E run and one
// 4 KiB residual run (block_jacobian_writer.cc:75-149: all E cells, then all
// F cells, in block order), 52 KiB of LDS (3 workgroups, 12 waves per CU),
// and the image [F | E | R] is cut into 13 KiB per wave: wave 0
// stores F[0, 13 KiB), wave 1 F[13, 26), wave 2 F[26, 36) and E[0, 3), wave
// 3 E[3, 12) and the residuals -- one or two runs a wave instead of three
// short segments (9, 3 and 1 KiB) per wave.
//
// Measured (same-process interleaved A/Bs against the
// one-wave-workgroup kernel, bit-identical outputs): -1.4 % to -2.4 % on
// six boxes (profiles/round5/r5a-r5d, r5f, r5g).  Other shapes measured in
// rounds 5 (kW = 2, 3, 5, 6, 8; 8 waves per CU; F in thirds; two LDS
// phases; a persistent pipelined form; stores in flight capped per wave; a
// CompressedRowSparseMatrix form; a fused-gradient form) were slower and are
// not in the tree (git history before round 6).
//
// Used when the group's residual, E and F bases are 64-byte aligned (then
// every workgroup's runs are: 9216, 3072 and 1024 bytes per chunk) and both
// outputs are requested; otherwise the one-wave kernel, whose sector-window
// tail handles any alignment.  The last, partial workgroup stores each
// chunk through the slow tail.  Gradient atomics (gradient_mode 2) as the
// one-wave kernel.
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

// Waves per workgroup: 4 consecutive chunks, 52 KiB of LDS.
constexpr int kQuadWaves = 4;

// Wave w's part of the workgroup image [F | E | R] (KiB): [lo, hi), the
// image cut in kW equal parts.
template <int kW, int w, int kFk = kQuadFk, int kEk = kQuadEk>
struct QuadPart {
  static constexpr int F = kFk * kW, E = kEk * kW, R = kQuadRk * kW;
  static constexpr int T = F + E + R;
  static constexpr int lo = T * w / kW;
  static constexpr int hi = T * (w + 1) / kW;
  static constexpr int N = hi - lo;
  // region r's overlap with [lo, hi): start (image KiB) and count
  static constexpr int rb(int r) { return r == 0 ? 0 : r == 1 ? F : F + E; }
  static constexpr int re(int r) { return r == 0 ? F : r == 1 ? F + E : T; }
  static constexpr int s(int r) { return lo > rb(r) ? lo : rb(r); }
  static constexpr int n(int r) { return (hi < re(r) ? hi : re(r)) - s(r) > 0 ? (hi < re(r) ? hi : re(r)) - s(r) : 0; }
};

// Read wave w's pieces from the workgroup image and store them, region by
// region (at most three runs).
template <int kW, int w, int kFk, int kEk>
__device__ __forceinline__ void QuadTail(const double* img, double* const bases[3], int lane,
                                         double* v_partial, double v_wsum, bool failed,
                                         int* status_dst) {
  using P = QuadPart<kW, w, kFk, kEk>;
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
  QuadRun<P::n(0), 0>(b0, q);
  QuadRun<P::n(1), P::n(0)>(b1, q);
  QuadRun<P::n(2), P::n(0) + P::n(1)>(b2, q);
  if (lane == 0) {
    StoreB64(v_partial, v_wsum);
    if (failed) StoreB32(status_dst, 1);
  }
  KeepAlive<N>(q);
  asm volatile("" ::"v"(b0), "v"(b1), "v"(b2), "v"(v_partial), "v"(v_wsum));
}

template <int kW, int kFk = kQuadFk, int kEk = kQuadEk, int w = 0>
__device__ __forceinline__ void QuadTailFor(int wave, const double* img, double* const bases[3], int lane,
                                            double* v_partial, double v_wsum, bool failed,
                                            int* status_dst) {
  if constexpr (w < kW) {
    if (wave == w) {
      QuadTail<kW, w, kFk, kEk>(img, bases, lane, v_partial, v_wsum, failed, status_dst);
      return;
    }
    QuadTailFor<kW, kFk, kEk, w + 1>(wave, img, bases, lane, v_partial, v_wsum, failed, status_dst);
  }
}

// Waves per SIMD the register allocation must allow: the LDS bound (3
// workgroups of 52 KiB per CU: 12 waves, 3 per SIMD).
constexpr int kQuadWavesPerEu = ((160 / (13 * kQuadWaves)) * kQuadWaves + 3) / 4;

template <class K, int kLoss>
__global__ __launch_bounds__(kQuadWaves * kWave) __attribute__((amdgpu_waves_per_eu(kQuadWavesPerEu))) void
EvaluateAffineChunksGroupStore(const GroupArgs a) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p;
  static_assert(NR == 2 && S0 == 9 && S1 == 3, "Snavely-shaped kinds");
  constexpr int kW = kQuadWaves;
  constexpr int kFk = kQuadFk, kEk = kQuadEk;  // KiB per chunk of the F and E regions
  constexpr int kImg = 13 * kW * 128;  // doubles
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
  double* fbase = !a.jacobian ? nullptr : a.jacobian + a.jac_base[0][0] + a.jac_stride[0] * wg0;
  double* ebase = !a.jacobian ? fbase : a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * wg0;
  double* rbase = a.residuals ? a.residuals + a.res_base + (int64_t)NR * wg0 : nullptr;
  const bool full = wg0 + kW * kWave <= a.n;
  const bool fast = full && fbase && rbase &&
                    ((reinterpret_cast<uintptr_t>(fbase) | reinterpret_cast<uintptr_t>(ebase) |
                      reinterpret_cast<uintptr_t>(rbase)) & 63) == 0;
  if (fast) {
    // Stage the wave's cells in output order (every lane active here).
#pragma unroll
    for (int q = 0; q < NR * S0; q += 2)
      *reinterpret_cast<double2*>(fw + lane * NR * S0 + q) = make_double2(J0[q], J0[q + 1]);
#pragma unroll
    for (int q = 0; q < NR * S1; q += 2)
      *reinterpret_cast<double2*>(ew + lane * NR * S1 + q) = make_double2(J1[q], J1[q + 1]);
    *reinterpret_cast<double2*>(rw + lane * NR) = make_double2(r[0], r[1]);
    __syncthreads();
    double* const bases[3] = {fbase, ebase, rbase};
    QuadTailFor<kW, kFk, kEk>(w, img, bases, lane, v_partial, wsum, failed, a.status);
    return;
  }
  // The last (partial) workgroup or unaligned outputs: each wave its own
  // chunk through the slow tail, in its own F region.
  __syncthreads();  // every wave's gather landing area is free again
  if (has) StageAndStore<K, true, false>(a, fw, lane, active, i0, nw, r, J0, J1);
  if (lane == 0 && has) {  // slots past the last chunk stay 0 (zeroed at cse_create)
    *v_partial = wsum;
    if (failed) *a.status = 1;
  }
}

// May the group take EvaluateAffineChunksGroupStore?  Both outputs, and the
// residual, E-cell and F-cell bases on 64-byte sectors.

inline bool GroupStoreEligible(const GroupArgs& a) {
  if (!a.residuals || !a.jacobian) return false;
  const uintptr_t m = reinterpret_cast<uintptr_t>(a.residuals + a.res_base) |
                      reinterpret_cast<uintptr_t>(a.jacobian + a.jac_base[0][0]) |
                      reinterpret_cast<uintptr_t>(a.jacobian + a.jac_base[1][0]);
  return (m & 63) == 0 && a.jac_stride[0] == 18 && a.jac_stride[1] == 6;
}

}  // namespace cse

#endif  // CSE_GROUP_STORE_KERNEL_HPP_
