// quad_kernel.hpp -- tuning build only (-DCSE_TUNING): the BlockSparseMatrix
// residual+Jacobian kernel with four-wave workgroups over four consecutive
// 64-block chunks whose F cells, E cells and residuals are staged together in
// LDS and then written as long contiguous runs, each wave storing one or two
// runs of the workgroup's output instead of its own chunk's three segments.
//
// The hypothesis it tests: the shipped
// kernel (EvaluateAffineChunksTwoRoundW1) reaches 0.61-0.66 of 8 TB/s while a
// pure 16-B write stream of its bytes reaches 0.72-0.74, and the gap is the
// interleaving of every resident wave's three short output streams (9 KiB of
// F, 3 KiB of E, 1 KiB of residuals).  Here the workgroup's four chunks own
// one contiguous 36 KiB F run, one 12 KiB E run and one 4 KiB residual run
// (block_jacobian_writer.cc:75-149: all E cells, then all F cells, in block
// order), staged in 52 KiB of LDS (3 workgroups = 12 waves per CU), and
//   kSched 0: 13 store instructions per wave -- wave 0 F[0, 13 KiB), wave 1
//             F[13, 26), wave 2 F[26, 36) + E[0, 3), wave 3 E[3, 12) + R;
//   kSched 1: waves 0-2 F in thirds (12 KiB each), wave 3 all of E and R.
// Outputs are bit-identical to the shipped kernel's (same functor, loss,
// cost partial per wave in the same slot).
#ifndef CSE_QUAD_KERNEL_HPP_
#define CSE_QUAD_KERNEL_HPP_

#include "../../ceres-solver-cuda_amd/csrc/evaluate_kernel.hpp"

namespace cse {

constexpr int kQuadF = 36, kQuadE = 12, kQuadR = 4;  // KiB per workgroup (Snavely)

// One store run: N instructions of 1 KiB from region offset O KiB, the data
// in q[J0 .. J0 + N), base = the run's first byte + 4096 (+ 16 * lane).
template <int N, int J0>
__device__ __forceinline__ void QuadRun(double* base, const cse_v4i* q) {
  if constexpr (N > 0) SegmentStoresFrom<0, N>(base, base + 1024, q + J0);
}

// The runs of wave w under schedule kSched: (region, KiB offset, count) x 2.
// Regions: 0 F, 1 E, 2 residuals.
template <int kSched, int w>
struct QuadSched;
template <> struct QuadSched<0, 0> { static constexpr int r0 = 0, o0 = 0, n0 = 13, r1 = 0, o1 = 0, n1 = 0; };
template <> struct QuadSched<0, 1> { static constexpr int r0 = 0, o0 = 13, n0 = 13, r1 = 0, o1 = 0, n1 = 0; };
template <> struct QuadSched<0, 2> { static constexpr int r0 = 0, o0 = 26, n0 = 10, r1 = 1, o1 = 0, n1 = 3; };
template <> struct QuadSched<0, 3> { static constexpr int r0 = 1, o0 = 3, n0 = 9, r1 = 2, o1 = 0, n1 = 4; };
template <> struct QuadSched<1, 0> { static constexpr int r0 = 0, o0 = 0, n0 = 12, r1 = 0, o1 = 0, n1 = 0; };
template <> struct QuadSched<1, 1> { static constexpr int r0 = 0, o0 = 12, n0 = 12, r1 = 0, o1 = 0, n1 = 0; };
template <> struct QuadSched<1, 2> { static constexpr int r0 = 0, o0 = 24, n0 = 12, r1 = 0, o1 = 0, n1 = 0; };
template <> struct QuadSched<1, 3> { static constexpr int r0 = 1, o0 = 0, n0 = 12, r1 = 2, o1 = 0, n1 = 4; };

constexpr int QuadRegionKiB(int r) { return r == 0 ? 0 : r == 1 ? kQuadF : kQuadF + kQuadE; }

// Read wave w's pieces from the workgroup image and store them.
template <int kSched, int w>
__device__ __forceinline__ void QuadTail(const double* img, double* const bases[3], int lane,
                                         double* v_partial, double v_wsum, bool failed,
                                         int* status_dst) {
  using S = QuadSched<kSched, w>;
  constexpr int N = S::n0 + S::n1;
  cse_v4i q[N];
  const double2* im2 = reinterpret_cast<const double2*>(img);
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const int kib = j < S::n0 ? QuadRegionKiB(S::r0) + S::o0 + j : QuadRegionKiB(S::r1) + S::o1 + (j - S::n0);
    const double2 v = im2[kib * kWave + lane];
    q[j] = AsV4i(v.x, v.y);
  }
  double* b0 = bases[S::r0] + 128 * S::o0 + 2 * lane + 512;
  double* b1 = bases[S::r1] + 128 * S::o1 + 2 * lane + 512;
  asm volatile("" : "+v"(v_partial), "+v"(v_wsum));
  asm volatile("" ::"v"(b0), "v"(b1));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  QuadRun<S::n0, 0>(b0, q);
  QuadRun<S::n1, S::n0>(b1, q);
  if (lane == 0) {
    StoreB64(v_partial, v_wsum);
    if (failed) StoreB32(status_dst, 1);
  }
  KeepAlive<N>(q);
  asm volatile("" ::"v"(b0), "v"(b1), "v"(v_partial), "v"(v_wsum));
}

template <class K, int kLoss, int kSched>
__global__ __launch_bounds__(kBlockThreads) __attribute__((amdgpu_waves_per_eu(3))) void
EvaluateAffineQuad(const GroupArgs a) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p;
  static_assert(NR == 2 && S0 == 9 && S1 == 3, "Snavely-shaped kinds");
  constexpr int kImg = (kQuadF + kQuadE + kQuadR) * 128;  // doubles (52 KiB)
  __shared__ __attribute__((aligned(16))) double img[kImg];
  const int lane = threadIdx.x & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int64_t num_chunks = (a.n + kWave - 1) / kWave;
  const int64_t c = (int64_t)blockIdx.x * kWavesPerBlock + w;
  const bool has = c < num_chunks;
  const int64_t i0 = c * kWave;
  const int64_t rem = a.n - i0;
  const int nw = !has ? 0 : rem < kWave ? (int)rem : kWave;
  const bool active = lane < nw;
  const int64_t i = active ? i0 + lane : (a.n > 0 ? a.n - 1 : 0);
  double* fw = img + w * (NR * S0 * kWave);  // this wave's F cells (and its gather landing area)
  double* ew = img + kQuadF * 128 + w * (NR * S1 * kWave);
  double* rw = img + (kQuadF + kQuadE) * 128 + w * (NR * kWave);

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

  const int64_t wg0 = (int64_t)blockIdx.x * kWavesPerBlock * kWave;  // the workgroup's first block
  double* fbase = a.jacobian ? a.jacobian + a.jac_base[0][0] + a.jac_stride[0] * wg0 : nullptr;
  double* ebase = a.jacobian ? a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * wg0 : nullptr;
  double* rbase = a.residuals ? a.residuals + a.res_base + (int64_t)NR * wg0 : nullptr;
  const bool full = wg0 + kWavesPerBlock * kWave <= a.n;
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
    switch (w) {
      case 0: QuadTail<kSched, 0>(img, bases, lane, v_partial, wsum, failed, a.status); break;
      case 1: QuadTail<kSched, 1>(img, bases, lane, v_partial, wsum, failed, a.status); break;
      case 2: QuadTail<kSched, 2>(img, bases, lane, v_partial, wsum, failed, a.status); break;
      default: QuadTail<kSched, 3>(img, bases, lane, v_partial, wsum, failed, a.status); break;
    }
    return;
  }
  // The last (partial) workgroup or unaligned outputs: each wave its own
  // chunk through the slow tail, in its own F region.
  __syncthreads();  // every wave's gather landing area is free again
  if (has) StageAndStore<K, true, false>(a, fw, lane, active, i0, nw, r, J0, J1);
  if (lane == 0) {
    *v_partial = has ? wsum : 0.0;
    if (has && failed) *a.status = 1;
  }
}

}  // namespace cse

#endif  // CSE_QUAD_KERNEL_HPP_
