// quad_kernel.hpp -- tuning build only (-DCSE_TUNING): the BlockSparseMatrix
// residual+Jacobian kernel with kW-wave workgroups over kW consecutive
// 64-block chunks whose F cells, E cells and residuals are staged together in
// LDS and then written as long contiguous runs, each wave storing one to
// three runs of the workgroup's output instead of its own chunk's three
// segments.
//
// The hypothesis it tests: the shipped
// kernel (EvaluateAffineChunksTwoRoundW1) reaches 0.61-0.66 of 8 TB/s while a
// pure 16-B write stream of its bytes reaches 0.72-0.74, and the gap is the
// interleaving of every resident wave's three short output streams (9 KiB of
// F, 3 KiB of E, 1 KiB of residuals).  Here the workgroup's kW chunks own
// one contiguous 9 kW KiB F run, one 3 kW KiB E run and one kW KiB residual
// run (block_jacobian_writer.cc:75-149: all E cells, then all F cells, in
// block order), staged in 13 kW KiB of LDS; the image [F | E | R] is cut
// into 13 KiB per wave (kSched 0), or (kSched 1, kW = 4) waves 0-2 take F in
// thirds and wave 3 all of E and R (the schedule VERDICT r4 named).
// kPadKiB: extra LDS per workgroup (an occupancy limit).
// Outputs are bit-identical to the shipped kernel's (same functor, loss,
// cost partial per wave in the same slot).
#ifndef CSE_QUAD_KERNEL_HPP_
#define CSE_QUAD_KERNEL_HPP_

#include "../../ceres-solver-cuda_amd/csrc/evaluate_kernel.hpp"

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

// Wave w's part of the workgroup image [F | E | R] (KiB): [lo, hi).
template <int kW, int kSched, int w>
struct QuadPart {
  static constexpr int F = kQuadFk * kW, E = kQuadEk * kW, R = kQuadRk * kW;
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
template <int kW, int kSched, int w>
__device__ __forceinline__ void QuadTail(const double* img, double* const bases[3], int lane,
                                         double* v_partial, double v_wsum, bool failed,
                                         int* status_dst) {
  using P = QuadPart<kW, kSched, w>;
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

template <int kW, int kSched, int w = 0>
__device__ __forceinline__ void QuadTailFor(int wave, const double* img, double* const bases[3], int lane,
                                            double* v_partial, double v_wsum, bool failed,
                                            int* status_dst) {
  if constexpr (w < kW) {
    if (wave == w) {
      QuadTail<kW, kSched, w>(img, bases, lane, v_partial, v_wsum, failed, status_dst);
      return;
    }
    QuadTailFor<kW, kSched, w + 1>(wave, img, bases, lane, v_partial, v_wsum, failed, status_dst);
  }
}

// Waves per SIMD the register allocation must allow: the LDS bound.
template <int kW, int kPadKiB>
constexpr int kQuadWavesPerEu = ((160 / (13 * kW + kPadKiB)) * kW + 3) / 4;

template <class K, int kLoss, int kW, int kSched, int kPadKiB>
__global__ __launch_bounds__(kW * kWave) __attribute__((amdgpu_waves_per_eu(kQuadWavesPerEu<kW, kPadKiB>))) void
EvaluateAffineQuad(const GroupArgs a) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p;
  static_assert(NR == 2 && S0 == 9 && S1 == 3, "Snavely-shaped kinds");
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
  double* fw = img + w * (NR * S0 * kWave);  // this wave's F cells (and its gather landing area)
  double* ew = img + kQuadFk * kW * 128 + w * (NR * S1 * kWave);
  double* rw = img + (kQuadFk + kQuadEk) * kW * 128 + w * (NR * kWave);

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
  }
  const double wsum = WaveSumLane0(active ? cost : 0.0);
  const bool failed = __ballot(active && !ok) != 0;
  double* v_partial = a.partials + c;

  const int64_t wg0 = (int64_t)blockIdx.x * kW * kWave;  // the workgroup's first block
  double* fbase = a.jacobian ? a.jacobian + a.jac_base[0][0] + a.jac_stride[0] * wg0 : nullptr;
  double* ebase = a.jacobian ? a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * wg0 : nullptr;
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
    QuadTailFor<kW, kSched>(w, img, bases, lane, v_partial, wsum, failed, a.status);
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

}  // namespace cse

#endif  // CSE_QUAD_KERNEL_HPP_
