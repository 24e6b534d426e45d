// pipeline_kernel.hpp -- the hot BlockSparse kernel as a persistent,
// wave-specialised pipeline.
//
// Same work and same outputs (bit for bit) as EvaluateAffineChunksTwoRound:
// one lane per residual block, one 64-block chunk per wave iteration, the
// reference's EvaluateKernel per block (cuda_evaluator_kernel.h:297-422:
// gather, Jet autodiff, loss + Corrector, residual and Jacobian writes, one
// cost partial per chunk).  What changes is who does what, and when:
//
//   * One 1024-thread workgroup per CU, alive for the whole launch, taking
//     every G-th chunk (G workgroups).
//   * kCompute "compute" waves fetch and evaluate.  Every input of a chunk
//     (parameter ids, observations, the point, the camera) is moved by
//     LDS-DMA into the wave's own input buffer one iteration ahead, so the
//     loads of chunk j + kCompute are in flight while chunk j is evaluated
//     and the wave never waits on a dependent load chain.  A compute wave
//     writes no global memory: it stages its chunk's F cells, E cells and
//     residuals into an LDS slot and moves on.
//   * kStore "store" waves drain the slots: read the staged chunk back as
//     16-byte pieces in segment order (sector-aligned windows, as the
//     shipped kernel) and issue its 13 back-to-back `global_store_dwordx4 ...
//     sc1 nt`, plus the chunk's cost partial.  A store wave holds only one
//     chunk's store data in VGPRs; when it refills them it waits until the
//     hardware has read the previous chunk's stores ("store
//     tail"), which is the pipeline's back-pressure.
//
// The slots are handed over through two LDS sequence words per slot
// (filled, drained); chunk j uses slot j % kSlots, compute wave j % kCompute
// and store wave j % kStore, so every wave walks its chunks in increasing
// order and the smallest unfinished chunk can always make progress (no
// deadlock).  No workgroup barrier is used after the prologue.
//
// Chunks whose outputs cannot take the 16-byte store windows (a ragged last
// chunk, unaligned segments) are stored by their compute wave itself
// (StageAndStore), exactly as the shipped kernel does; the slot then carries
// only the hand-over.
#ifndef CSE_PIPELINE_KERNEL_HPP_
#define CSE_PIPELINE_KERNEL_HPP_

#include "../../ceres-solver-cuda_amd/csrc/evaluate_kernel.hpp"

namespace cse {

constexpr int kPipeThreads = 1024;
constexpr int kPipeWaves = kPipeThreads / kWave;
constexpr int kLdsBytes = 160 * 1024;

template <class K, int kStoreWaves>
struct PipeShape {
  using Tr = KindTraits<K>;
  static constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1;
  static constexpr int S0p = (S0 + 1) & ~1;
  static constexpr int kStore = kStoreWaves;
  static constexpr int kCompute = kPipeWaves - kStoreWaves;
  // Input buffer of a compute wave (doubles): the 64 cameras (S0p doubles
  // each, lane-major), 64 observations (2), 64 points (six 4-byte DMA
  // pieces), the 64 id pairs of the chunk after next (two 4-byte halves).
  static constexpr int kInCam = 0;
  static constexpr int kInObs = kInCam + kWave * S0p;
  static constexpr int kInPt = kInObs + kWave * 2;
  static constexpr int kInIds = kInPt + kWave * 3;
  static constexpr int kInDoubles = kInIds + kWave;
  // Output slot (doubles): F cells, E cells, residuals (lane-major, i.e. in
  // segment order), then a 16-byte header {partial, (failed, mode)}.
  static constexpr int kSlotF = 0;
  static constexpr int kSlotE = kSlotF + kWave * NR * S0;
  static constexpr int kSlotR = kSlotE + kWave * NR * S1;
  static constexpr int kSlotHdr = kSlotR + kWave * NR;
  static constexpr int kSlotDoubles = kSlotHdr + 2;
  static constexpr int kFixedBytes = 8 * kCompute * kInDoubles + 64;
  static constexpr int kSlots = (kLdsBytes - kFixedBytes) / (8 * kSlotDoubles);
  static_assert(kSlots >= 2, "LDS too small for the pipeline");
  static_assert(Tr::D == 2 && Tr::NB == 2 && S1 == 3 && NR % 2 == 0, "BAL-shaped two-slot kinds");
  static_assert((NR * S0) % 2 == 0 && (NR * S1) % 2 == 0, "16-byte pieces");
};

template <class K, int kStoreWaves>
struct alignas(16) PipeLds {
  using P = PipeShape<K, kStoreWaves>;
  double in[P::kCompute][P::kInDoubles];
  double slot[P::kSlots][P::kSlotDoubles];
  int fill_seq[P::kSlots];
  int drain_seq[P::kSlots];
};

// The hand-over words are read and written with inline-asm ds_read_b32 /
// ds_write_b32: a volatile C++ access would make the compiler wait for every
// outstanding vector-memory operation first (vmcnt(0): a store wave's queued
// stores, a compute wave's prefetch), which is exactly what the pipeline
// must not do.
__device__ __forceinline__ int PipeLoadWord(const int* word) {
  int v;
  const uint32_t addr = (uint32_t)reinterpret_cast<uintptr_t>(word);
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return v;
}
// Spin (with s_sleep) until the LDS word equals `want`; wave-uniform.
__device__ __forceinline__ void PipeWait(const int* word, int want) {
  while (__builtin_amdgcn_readfirstlane(PipeLoadWord(word)) != want) __builtin_amdgcn_s_sleep(1);
  asm volatile("" ::: "memory");
}
// Publish `value` in an LDS word after this wave's LDS accesses completed.
__device__ __forceinline__ void PipeSignal(int* word, int value, int lane) {
  const uint32_t addr = (uint32_t)reinterpret_cast<uintptr_t>(word);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) asm volatile("ds_write_b32 %0, %1" ::"v"(addr), "v"(value) : "memory");
  asm volatile("" ::: "memory");
}

// LDS-DMA of one chunk's inputs into a compute wave's buffer: the camera
// pieces from the repacked slot-0 table (piece p of the wave's 64 cameras by
// lane p % 64 of instruction p / 64, as GatherCoopDma), the observation
// (16 B), the point (24 B as six 4-byte pieces).
// (kTag: unique per calling kernel; one instantiation per kernel works round
// a host-side template instantiation failure of hipcc 7.2 when two kernels
// share one instantiation of this DMA loop.)
template <class K, int kStoreWaves, int kTag>
__device__ __forceinline__ void PipeIssueInputs(const GroupArgs& a, double* in, int64_t i,
                                                int cam_own, int pt_own, int lane) {
  using P = PipeShape<K, kStoreWaves>;
  constexpr int kPieces = P::S0p / 2;
  constexpr int kRow = PackedRowDoubles(P::S0);
#pragma unroll
  for (int k = 0; k < kPieces; ++k) {
    const int p = k * kWave + lane;
    const int t = p / kPieces, q = p - t * kPieces;
    const int cid = __shfl(cam_own, t, kWave);
    const double* src = a.packed0 + (int64_t)kRow * cid + 2 * q;
    __builtin_amdgcn_global_load_lds(src, in + P::kInCam + 2 * kWave * k, 16, 0, 0);
  }
  __builtin_amdgcn_global_load_lds(a.data + 2 * i, in + P::kInObs, 16, 0, 2);
  // The point as six 4-byte pieces (dword k of lane l at 256 k + 4 l bytes).
  const uint32_t* pt = reinterpret_cast<const uint32_t*>(a.state + a.state_base[1] + 3LL * pt_own);
#pragma unroll
  for (int k = 0; k < 6; ++k)
    __builtin_amdgcn_global_load_lds(pt + k, in + P::kInPt + (kWave / 2) * k, 4, 0, 2);
}
// The id pair of block i: the slot-0 id at in[kInIds] + 4 lane bytes, the
// slot-1 id 256 bytes further.
template <class K, int kStoreWaves>
__device__ __forceinline__ void PipeIssueIds(const GroupArgs& a, double* in, int64_t i) {
  using P = PipeShape<K, kStoreWaves>;
  const int32_t* src = a.ids + 2 * i;
  __builtin_amdgcn_global_load_lds(src, in + P::kInIds, 4, 0, 2);
  __builtin_amdgcn_global_load_lds(src + 1, in + P::kInIds + kWave / 2, 4, 0, 2);
}
template <class K, int kStoreWaves>
__device__ __forceinline__ void PipeReadIds(const double* in, int lane, int* cam, int* pt) {
  using P = PipeShape<K, kStoreWaves>;
  const int* ids = reinterpret_cast<const int*>(in + P::kInIds);
  *cam = ids[lane];
  *pt = ids[kWave + lane];
}

// kOpt (tuning): bit 0 cycle accounting (a.probe), bit 1 compute waves at
// s_setprio 3 (their DMA issue ahead of the store waves' stores).
template <class K, int kLoss, int kStoreWaves, int kOpt = 0>
__device__ __forceinline__ void PipeComputeWave(const GroupArgs& a, PipeLds<K, kStoreWaves>& L,
                                                int w, int lane0, int64_t c0, int64_t cstep, int nloc) {
  constexpr bool kProbe = kOpt & 1;
  if constexpr ((kOpt & 2) != 0) __builtin_amdgcn_s_setprio(3);
  unsigned long long pr[6] = {0, 0, 0, 0, 0, 0}, tp = 0;
  auto probe = [&](int k) {
    if constexpr (kProbe) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (k >= 0) pr[k] += t - tp;
      tp = t;
    }
  };
  using P = PipeShape<K, kStoreWaves>;
  using Tr = KindTraits<K>;
  constexpr int NR = P::NR, S0 = P::S0, S1 = P::S1, S1p = Tr::S1p;
  constexpr int NC = P::kCompute;
  double* in = L.in[w];
  // Block of `lane` in chunk jj (the last block for the lanes past the end).
  auto block_of = [&](int jj, int lane) -> int64_t {
    const int64_t i0 = (c0 + jj * cstep) * kWave;
    const int64_t rem = a.n - 1 - i0;
    return i0 + (lane < rem ? lane : rem);
  };
  int j = w;
  if (j >= nloc) return;
  // Prologue: the ids of the first chunk, then its inputs and the ids of
  // the next one.
  {
    const int64_t i = block_of(j, lane0);
    PipeIssueIds<K, kStoreWaves>(a, in, i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    int cam, pt;
    PipeReadIds<K, kStoreWaves>(in, lane0, &cam, &pt);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    PipeIssueInputs<K, kStoreWaves, kLoss + 16 * kOpt>(a, in, i, cam - a.packed0_lo, pt, lane0);
    if (j + NC < nloc) PipeIssueIds<K, kStoreWaves>(a, in, block_of(j + NC, lane0));
  }
  for (; j < nloc; j += NC) {
    // The lane index, opaque to the optimiser: every lane-derived address
    // is recomputed inside the iteration instead of being hoisted out of the
    // loop and kept live (and spilled) across the evaluation.
    int lane = lane0;
    asm volatile("" : "+v"(lane));
    probe(-1);
    // This chunk's inputs (and the next chunk's ids) have landed.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    probe(0);
    AffineInputs<K> x;
    {
      const double* cam = in + P::kInCam + lane * P::S0p;
#pragma unroll
      for (int k = 0; k < S0; ++k) x.x0[k] = cam[k];
      const double2 o = reinterpret_cast<const double2*>(in + P::kInObs)[lane];
      x.d[0] = o.x;
      x.d[1] = o.y;
      const uint32_t* h = reinterpret_cast<const uint32_t*>(in + P::kInPt) + lane;
      x.x1[0] = __hiloint2double((int)h[kWave], (int)h[0]);
      x.x1[1] = __hiloint2double((int)h[3 * kWave], (int)h[2 * kWave]);
      x.x1[2] = __hiloint2double((int)h[5 * kWave], (int)h[4 * kWave]);
    }
    const int jn = j + NC;
    int cam_n = 0, pt_n = 0;
    if (jn < nloc) PipeReadIds<K, kStoreWaves>(in, lane, &cam_n, &pt_n);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if (jn < nloc) {
      PipeIssueInputs<K, kStoreWaves, kLoss + 16 * kOpt>(a, in, block_of(jn, lane), cam_n - a.packed0_lo, pt_n,
                                             lane);
      if (jn + NC < nloc) PipeIssueIds<K, kStoreWaves>(a, in, block_of(jn + NC, lane));
    }
    probe(1);

    // Evaluate chunk j.
    const int64_t c = c0 + j * cstep;
    const int64_t i0 = c * kWave;
    const int64_t rem = a.n - i0;
    const int nw = rem < kWave ? (int)rem : kWave;
    const bool active = lane < nw;
    double r[NR], J0[NR * S0], J1[NR * S1p];
    bool ok = EvaluateFunctor<K, true>(x.d, x.x0, x.x1, r, J0, J1);
    if (ok && a.check_finite) {
      const bool bad = AnyNonFinite<NR>(r) || AnyNonFinite<NR * S0>(J0) || AnyNonFinite<NR * S1>(J1);
      ok = !bad;
    }
    const double cost = LossAndCorrect<K, kLoss, true>(a.loss, a.apply_loss, r, J0, J1, true);
    const double wsum = WaveSumLane0(active ? cost : 0.0);
    const bool failed = __ballot(active && !ok) != 0;
    probe(2);

    // Hand the chunk to its store wave through slot j % kSlots.
    const int s = j % P::kSlots;
    double* slot = L.slot[s];
    PipeWait(&L.drain_seq[s], j - P::kSlots);
    probe(3);
    const bool fast = FastTail<K, true, false>(a, i0, nw);
    if (fast) {
#pragma unroll
      for (int q = 0; q < NR * S0; q += 2)
        reinterpret_cast<double2*>(slot + P::kSlotF + lane * NR * S0)[q / 2] =
            make_double2(J0[q], J0[q + 1]);
#pragma unroll
      for (int k = 0; k < NR; ++k)
#pragma unroll
        for (int cc = 0; cc < S1; ++cc) slot[P::kSlotE + lane * NR * S1 + k * S1 + cc] = J1[k * S1p + cc];
      reinterpret_cast<double2*>(slot + P::kSlotR)[lane] = make_double2(r[0], r[1]);
    } else {
      // Ragged or unaligned: this wave stores the chunk itself.
      StageAndStore<K, true, false>(a, slot, lane, active, i0, nw, r, J0, J1);
      if (lane == 0) {
        a.partials[c] = wsum;
        if (failed) *a.status = 1;
      }
    }
    if (lane == 0) {
      slot[P::kSlotHdr] = wsum;
      reinterpret_cast<int*>(slot + P::kSlotHdr + 1)[0] = failed ? 1 : 0;
      reinterpret_cast<int*>(slot + P::kSlotHdr + 1)[1] = fast ? 1 : 0;
    }
    PipeSignal(&L.fill_seq[s], j, lane);
    probe(4);
    pr[5] += 1;
  }
  if constexpr (kProbe) {
    if (lane0 == 0) {
      unsigned long long* o = a.probe + (blockIdx.x * kPipeWaves + w) * 8;
#pragma unroll
      for (int k = 0; k < 6; ++k) o[k] += pr[k];
    }
  }
}

template <class K, int kStoreWaves, int kOpt = 0>
__device__ __forceinline__ void PipeStoreWave(const GroupArgs& a, PipeLds<K, kStoreWaves>& L,
                                              int v, int lane0, int64_t c0, int64_t cstep, int nloc) {
  constexpr bool kProbe = kOpt & 1;
  unsigned long long pr[6] = {0, 0, 0, 0, 0, 0}, tp = 0;
  auto probe = [&](int k) {
    if constexpr (kProbe) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (k >= 0) pr[k] += t - tp;
      tp = t;
    }
  };
  using P = PipeShape<K, kStoreWaves>;
  constexpr int NR = P::NR, S0 = P::S0, S1 = P::S1;
  constexpr int kQ0 = NR * S0 / 2, kQ1 = NR * S1 / 2;
  static_assert(kQ0 <= 16 && kQ1 <= 8 && NR == 2, "store windows of the BAL shapes");
  for (int j = v; j < nloc; j += P::kStore) {
    int lane = lane0;  // opaque, as in PipeComputeWave
    asm volatile("" : "+v"(lane));
    const int s = j % P::kSlots;
    const double* slot = L.slot[s];
    probe(-1);
    PipeWait(&L.fill_seq[s], j);
    probe(0);
    const int mode = __builtin_amdgcn_readfirstlane(reinterpret_cast<const int*>(slot + P::kSlotHdr + 1)[1]);
    if (mode == 0) {  // stored by the compute wave
      PipeSignal(&L.drain_seq[s], j, lane);
      continue;
    }
    const int64_t c = c0 + j * cstep;
    const int64_t i0 = c * kWave;
    double* seg0 = a.jacobian + a.jac_base[0][0] + a.jac_stride[0] * i0;
    double* seg1 = a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * i0;
    double* rdst = a.residuals + a.res_base + (int64_t)NR * (i0 + lane);
    const int hp0 = SectorHeadPieces<64>(seg0);
    const int hp1 = SectorHeadPieces<64>(seg1);
    cse_v4i q0[kQ0], q1[kQ1], qr;
    ReadSegmentPieces<kQ0, 64>(slot + P::kSlotF, hp0, lane, q0);
    ReadSegmentPieces<kQ1, 64>(slot + P::kSlotE, hp1, lane, q1);
    {
      const double2 v2 = reinterpret_cast<const double2*>(slot + P::kSlotR)[lane];
      qr = AsV4i(v2.x, v2.y);
    }
    double wsum = slot[P::kSlotHdr];
    const int failed = reinterpret_cast<const int*>(slot + P::kSlotHdr + 1)[0];
    PipeSignal(&L.drain_seq[s], j, lane);
    probe(1);
    double* f0 = seg0 + 2 * (lane + hp0) + 512;
    double* f1 = seg0 + 2 * (lane + hp0) + 1536;
    double* flast = seg0 + 2 * LastPiece<kQ0, 64>(lane, hp0);
    double* e0 = seg1 + 2 * (lane + hp1) + 512;
    double* elast = seg1 + 2 * LastPiece<kQ1, 64>(lane, hp1);
    double* v_partial = a.partials + c;
    asm volatile("" : "+v"(v_partial), "+v"(wsum));
    asm volatile("" ::"v"(f0), "v"(f1), "v"(e0), "v"(rdst), "v"(flast), "v"(elast));
    SegmentStoresFrom<0, kQ0 - 1>(f0, f1, q0);
    StoreNt16<0>(flast, q0[kQ0 - 1]);
    SegmentStoresFrom<0, kQ1 - 1>(e0, e0, q1);
    StoreNt16<0>(elast, q1[kQ1 - 1]);
    StoreNt16<0>(rdst, qr);
    if (lane == 0) {
      StoreB64(v_partial, wsum);
      if (failed) StoreB32(a.status, 1);
    }
    KeepAlive<kQ0>(q0);
    KeepAlive<kQ1>(q1);
    KeepAlive<1>(&qr);
    asm volatile("" ::"v"(f0), "v"(f1), "v"(e0), "v"(rdst), "v"(flast), "v"(elast), "v"(v_partial),
                 "v"(wsum));
    probe(2);
    pr[5] += 1;
  }
  if constexpr (kProbe) {
    if (lane0 == 0) {
      unsigned long long* o = a.probe + (blockIdx.x * kPipeWaves + P::kCompute + v) * 8;
#pragma unroll
      for (int k = 0; k < 6; ++k) o[k] += pr[k];
    }
  }
}

// The kernel: gridDim.x workgroups (one per CU).  Workgroup b takes the
// chunks b, b + G, b + 2 G, ... (G = gridDim.x), so that at any moment the
// chunks in flight on the whole chip form one narrow window of the outputs,
// as in the one-chunk-per-wave kernel: with contiguous per-workgroup ranges
// the 256 workgroups wrote 768 distant streams at once and the kernel ran at
// 3.7 instead of 4.7 TB/s (profiles/round3/pipe4).  Requires residuals and
// the Jacobian (BlockSparseMatrix, affine), no gradient; the host checks.
template <class K, int kLoss, int kStoreWaves, int kOpt = 0>
__global__ __launch_bounds__(kPipeThreads) void EvaluateAffinePipelined(const GroupArgs a) {
  using P = PipeShape<K, kStoreWaves>;
  __shared__ PipeLds<K, kStoreWaves> L;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int64_t num_chunks = (a.n + kWave - 1) / kWave;
  const int64_t c0 = blockIdx.x, cstep = gridDim.x;
  const int nloc = (int)((num_chunks - c0 + cstep - 1) / cstep);
  if (threadIdx.x < P::kSlots) {
    L.fill_seq[threadIdx.x] = (int)threadIdx.x - P::kSlots;
    L.drain_seq[threadIdx.x] = (int)threadIdx.x - P::kSlots;
  }
  __syncthreads();
  if (wave < P::kCompute)
    PipeComputeWave<K, kLoss, kStoreWaves, kOpt>(a, L, wave, lane, c0, cstep, nloc);
  else
    PipeStoreWave<K, kStoreWaves, kOpt>(a, L, wave - P::kCompute, lane, c0, cstep, nloc);
}

// ---------------------------------------------------------------------------
// Residual-only / cost-only evaluation (the trust-region candidate step,
// trust_region_minimizer.cc:770-788) as persistent prefetching waves.  The
// one-chunk-per-wave kernel spends most of a wave's life in two dependent
// load round trips (the ids, then the camera gather); here
// each wave walks its chunks c, c + W, c + 2W, ... (W waves in the grid)
// with every input moved by LDS-DMA: the ids two chunks ahead, the camera
// pieces, observation and point one chunk ahead, so a wave waits on no
// dependent chain.  Per chunk a wave writes its residuals (kResiduals) and
// its cost partial; the top-of-iteration wait leaves those kStores youngest
// operations in flight (s_waitcnt vmcnt(kStores)).
template <class K, int kLoss, bool kResiduals, int kWG>
__global__ __launch_bounds__(kWG * kWave) void EvaluateResidualStreamed(const GroupArgs a) {
  using P = PipeShape<K, 4>;  // the input-buffer layout only
  using Tr = KindTraits<K>;
  constexpr int NR = P::NR;
  static_assert(NR == 2, "one 16-byte residual store per lane");
  __shared__ alignas(16) double in_all[kWG][P::kInDoubles];
  const int lane0 = threadIdx.x & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  double* in = in_all[w];
  const int64_t num_chunks = (a.n + kWave - 1) / kWave;
  const int64_t W = (int64_t)gridDim.x * kWG;
  int64_t c = (int64_t)blockIdx.x * kWG + w;
  if (c >= num_chunks) return;
  auto block_of = [&](int64_t cc, int lane) -> int64_t {
    const int64_t i0 = cc * kWave;
    const int64_t rem = a.n - 1 - i0;
    return i0 + (lane < rem ? lane : rem);
  };
  {
    const int64_t i = block_of(c, lane0);
    PipeIssueIds<K, 4>(a, in, i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    int cam, pt;
    PipeReadIds<K, 4>(in, lane0, &cam, &pt);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    PipeIssueInputs<K, 4, 32 + 8 * kWG + kLoss + 4 * kResiduals>(a, in, i, cam - a.packed0_lo, pt, lane0);
    if (c + W < num_chunks) PipeIssueIds<K, 4>(a, in, block_of(c + W, lane0));
  }
  constexpr int kStores = kResiduals ? 2 : 1;  // residual pair + lane-0 partial
  bool first = true;
  for (; c < num_chunks; c += W) {
    int lane = lane0;
    asm volatile("" : "+v"(lane));
    if (first)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kStores) : "memory");
    first = false;
    __builtin_amdgcn_wave_barrier();
    AffineInputs<K> x;
    {
      const double* cam = in + P::kInCam + lane * P::S0p;
#pragma unroll
      for (int k = 0; k < P::S0; ++k) x.x0[k] = cam[k];
      const double2 o = reinterpret_cast<const double2*>(in + P::kInObs)[lane];
      x.d[0] = o.x;
      x.d[1] = o.y;
      const uint32_t* h = reinterpret_cast<const uint32_t*>(in + P::kInPt) + lane;
      x.x1[0] = __hiloint2double((int)h[kWave], (int)h[0]);
      x.x1[1] = __hiloint2double((int)h[3 * kWave], (int)h[2 * kWave]);
      x.x1[2] = __hiloint2double((int)h[5 * kWave], (int)h[4 * kWave]);
    }
    const int64_t cn = c + W;
    int cam_n = 0, pt_n = 0;
    if (cn < num_chunks) PipeReadIds<K, 4>(in, lane, &cam_n, &pt_n);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if (cn < num_chunks) {
      PipeIssueInputs<K, 4, 32 + 8 * kWG + kLoss + 4 * kResiduals>(a, in, block_of(cn, lane),
                                                         cam_n - a.packed0_lo, pt_n, lane);
      if (cn + W < num_chunks) PipeIssueIds<K, 4>(a, in, block_of(cn + W, lane));
    }
    const int64_t i0 = c * kWave;
    const int64_t rem = a.n - i0;
    const bool active = lane < rem;
    double r[NR], J0[1], J1[1];
    bool ok = EvaluateFunctor<K, false>(x.d, x.x0, x.x1, r, J0, J1);
    if (ok && a.check_finite) ok = !AnyNonFinite<NR>(r);
    const double cost = LossAndCorrect<K, kLoss, false>(a.loss, a.apply_loss, r, J0, J1, kResiduals);
    const double wsum = WaveSumLane0(active ? cost : 0.0);
    const bool failed = __ballot(active && !ok) != 0;
    double* v_partial = a.partials + c;
    double v_wsum = wsum;
    asm volatile("" : "+v"(v_partial), "+v"(v_wsum));
    if constexpr (kResiduals) {
      double* rdst = a.residuals + a.res_base + (int64_t)NR * (i0 + lane);
      const cse_v4i q = AsV4i(r[0], r[1]);
      if (active) StoreNt16<0>(rdst, q);
    }
    if (lane == 0) StoreB64(v_partial, v_wsum);
    if (failed && lane == 0) StoreB32(a.status, 1);  // younger still: only over-waits
  }
}

}  // namespace cse

#endif  // CSE_PIPELINE_KERNEL_HPP_
