// persistent_kernel.hpp -- the BlockSparseMatrix Jacobian kernel in a
// persistent, software-pipelined form (one wave per workgroup, two waves per
// SIMD, each wave walking chunks c, c + G, c + 2G, ... of the grid G).
//
// Why (round 4, tools/membench3.hip, profiles/round4): a wave of the
// one-chunk-per-wave kernel spends its life in two dependent load phases
// (the block ids, then the camera DMA, observations and points) that queue
// behind the CU's outstanding stores, and holds its VGPR slot until its own
// 13 stores have been read out of the queue.  Here each wave issues chunk
// c + G's loads before it evaluates chunk c, so they are in flight during the
// functor, and chunk c's stores come from a register set disjoint from chunk
// c - G's, so no instruction overwrites a store's VGPRs while it may still be
// queued (kernel_common.hpp).  Every vector-memory instruction of the loop is
// inline asm and the waits are explicit: at the top of a chunk
// `s_waitcnt vmcnt(14)` retires its loads while the previous chunk's 13 stores
// and partial (issued after them) may stay in flight.
//
// Outputs are bit-identical to the one-chunk kernel's (the same per-lane
// arithmetic, the same 64-block chunks, one cost partial per chunk).  Used
// for two-slot kinds on the BlockSparseMatrix affine path with residuals and
// the Jacobian requested, no gradient, no held cameras.
#ifndef CSE_PERSISTENT_KERNEL_HPP_
#define CSE_PERSISTENT_KERNEL_HPP_

#include "../../ceres-solver-cuda_amd/csrc/evaluate_kernel.hpp"

namespace cse {

typedef double cse_v2d __attribute__((ext_vector_type(2)));

// The next chunk's per-lane inputs, loading: observation pair, point, and
// this lane's (camera, point) ids of the chunk after that.
struct PersistNext {
  cse_v2d o;
  double p[3];
  long long id;
};

// One chunk's stores: F pieces (kQ0), E pieces (kQ1), the residual pair and
// the wave's cost partial; the segment bases are wave-uniform (SGPR pairs),
// the per-lane byte offsets are the same for every chunk (PersistOffsets).
template <int kQ0, int kQ1>
struct PersistSet {
  cse_v4i q0[kQ0], q1[kQ1], qr;
  double wsum;
  double *f, *e, *r, *part;  // uniform: F and E segments, residuals, partial slot
};

// Per-lane byte offsets of the store tail, relative to the segment bases:
// pieces 0-3 and 4-7 of the F segment (1 KiB apart), its last piece (the
// sector-regrouped one, LastPiece), the E pieces and last piece, the residual
// pair.  The segments of every 64-block chunk have the same alignment, so
// these are computed once per wave.
struct PersistOffsets {
  uint32_t f0, f4, flast, e0, elast, r, zero;
};

// 16-byte store at SGPR base + VGPR offset + kOff bytes, `sc1 nt` (the
// streaming policy of StoreNt16).
template <int kOff>
__device__ __forceinline__ void StoreSaddr16(double* base, uint32_t voff, const cse_v4i& d) {
  static_assert(kOff >= 0 && kOff <= 4095, "global offset out of range");
  asm volatile("global_store_dwordx4 %0, %1, %2 offset:%3 sc1 nt" ::"v"(voff), "v"(d), "s"(base),
               "i"(kOff)
               : "memory");
}
__device__ __forceinline__ void StoreSaddr8(double* base, uint32_t voff, double v) {
  asm volatile("global_store_dwordx2 %0, %1, %2" ::"v"(voff), "v"(v), "s"(base) : "memory");
}

__device__ __forceinline__ int64_t PersistBlock(int64_t c, int lane, int64_t n) {
  const int64_t i = c * kWave + lane;
  return i < n ? i : n - 1;
}

// Queues chunk cn's gather (camera rows by LDS-DMA into camb; observation and
// point into nx) and the ids of chunk cnn into nx->id: 10 vector-memory
// instructions, all inline asm (invisible to the compiler's wait counting).
template <class K>
__device__ __forceinline__ void PersistIssueGather(const GroupArgs& a, double* camb, int64_t cn,
                                                   int64_t cnn, long long id, int lane,
                                                   PersistNext* nx) {
  using Tr = KindTraits<K>;
  constexpr int X0 = Tr::X0, X0p = (X0 + 1) & ~1, kPieces = X0p / 2;
  constexpr int kRow = PackedRowDoubles(X0);
  const int cid_own = (int)id - a.packed0_lo, pid = (int)(id >> 32);
  const uint32_t lbase = (uint32_t)reinterpret_cast<uintptr_t>(camb);
#pragma unroll
  for (int k = 0; k < kPieces; ++k) {
    const int p = k * kWave + lane;
    const int t = p / kPieces, q = p - t * kPieces;
    const int cid = __shfl(cid_own, t, kWave);
    const double* src = a.packed0 + (int64_t)kRow * cid + 2 * q;
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(lbase + 2u * kWave * 8u * k);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0)
                 : "memory");
  }
  const int64_t n = a.n;
  const double* po = a.data + 2 * PersistBlock(cn, lane, n);
  asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(nx->o) : "v"(po) : "memory");
  const double* pt = a.state + a.state_base[1] + 3LL * pid;
  asm volatile("global_load_dwordx2 %0, %1, off nt" : "=v"(nx->p[0]) : "v"(pt) : "memory");
  asm volatile("global_load_dwordx2 %0, %1, off offset:8 nt" : "=v"(nx->p[1]) : "v"(pt) : "memory");
  asm volatile("global_load_dwordx2 %0, %1, off offset:16 nt" : "=v"(nx->p[2]) : "v"(pt) : "memory");
  const long long* pi = reinterpret_cast<const long long*>(a.ids) + PersistBlock(cnn, lane, n);
  asm volatile("global_load_dwordx2 %0, %1, off nt" : "=v"(nx->id) : "v"(pi) : "memory");
}

// Retires the gather queued one chunk ago: kCount vector-memory instructions
// were issued after it (the previous chunk's stores).  The loaded registers
// are marked as written here, so nothing reads them earlier.
template <int kCount>
__device__ __forceinline__ void PersistWait(PersistNext* nx) {
  asm volatile("s_waitcnt vmcnt(%4)"
               : "+v"(nx->o), "+v"(nx->p[0]), "+v"(nx->p[1]), "+v"(nx->p[2])
               : "n"(kCount)
               : "memory");
  asm volatile("" : "+v"(nx->id));
}

template <int kQ0, int kQ1>
__device__ __forceinline__ void PersistKeep(const PersistSet<kQ0, kQ1>& s) {
  KeepAlive<kQ0>(s.q0);
  KeepAlive<kQ1>(s.q1);
  asm volatile("" ::"v"(s.qr), "v"(s.wsum), "s"(s.f), "s"(s.e), "s"(s.r), "s"(s.part));
}

// The vector-memory instructions a fast chunk issues after its successor's
// gather: the F and E segments, the residual pair and the lane-0 partial.
template <class K>
constexpr int PersistStoreOps() {
  using Tr = KindTraits<K>;
  return Tr::NR * Tr::S0 / 2 + Tr::NR * Tr::S1 / 2 + Tr::NR / 2 + 1;
}

// One chunk: evaluate from `cur` and camb_cur, queue the successor's gather
// into nxt / camb_nxt, stage and store from `mine`, keep `prev` (the previous
// chunk's store registers) alive until all of it is done.
template <class K, int kLoss, int kQ0, int kQ1>
__device__ __forceinline__ void PersistChunk(const GroupArgs& a, int64_t c, int64_t stride,
                                             int64_t num_chunks, const double* camb_cur,
                                             double* camb_nxt, double* st, PersistNext* cur,
                                             PersistNext* nxt, PersistSet<kQ0, kQ1>* mine,
                                             const PersistSet<kQ0, kQ1>& prev,
                                             const PersistOffsets& off, int hp0, int hp1, int lane) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p, X0 = Tr::X0;
  constexpr int X0p = (X0 + 1) & ~1;
  const int64_t i0 = c * kWave;
  const int64_t rem = a.n - i0;
  const int nw = rem < kWave ? (int)rem : kWave;
  const bool active = lane < nw;
  double d[2], x0[X0], x1[3];
#pragma unroll
  for (int k = 0; k < X0; ++k) x0[k] = camb_cur[lane * X0p + k];
  d[0] = cur->o.x;
  d[1] = cur->o.y;
  x1[0] = cur->p[0];
  x1[1] = cur->p[1];
  x1[2] = cur->p[2];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  const int64_t cn = c + stride;
  if (cn < num_chunks) PersistIssueGather<K>(a, camb_nxt, cn, cn + stride, cur->id, lane, nxt);

  double r[NR], J0[NR * S0], J1[NR * S1p];
  bool ok = EvaluateFunctor<K, true>(d, x0, x1, r, J0, J1);
  if (ok && a.check_finite)
    ok = !(AnyNonFinite<NR>(r) || AnyNonFinite<NR * S0>(J0) || AnyNonFinite<NR * S1>(J1));
  const double cost = LossAndCorrect<K, kLoss, true>(a.loss, a.apply_loss, r, J0, J1, true);
  const double wsum = WaveSumLane0(active ? cost : 0.0);
  const bool failed = __ballot(active && !ok) != 0;
  double* partial_dst = a.partials + c;

  if (!FastTail<K, true, false>(a, i0, nw)) {
    // A ragged or misaligned chunk: plain staged stores (rare: the last one).
    StageAndStore<K, true, false>(a, st, lane, active, i0, nw, r, J0, J1);
    if (lane == 0) {
      *partial_dst = wsum;
      if (failed) *a.status = 1;
    }
    PersistKeep(prev);
    // `mine` is this chunk's set on every path, so its previous value (two
    // chunks back) is dead here too and needs no registers during the functor.
    *mine = PersistSet<kQ0, kQ1>{};
    return;
  }
  // Stage the F cells, then the E cells, through the same LDS; read back as
  // 16-byte pieces in segment order (sector-aligned windows, as the
  // one-chunk kernel).
#pragma unroll
  for (int p = 0; p < NR * S0; ++p) st[lane * NR * S0 + p] = J0[p];
  __builtin_amdgcn_wave_barrier();
  ReadSegmentPieces<kQ0, 64>(st, hp0, lane, mine->q0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < NR; ++k)
#pragma unroll
    for (int cc = 0; cc < S1; ++cc) st[lane * NR * S1 + k * S1 + cc] = J1[k * S1p + cc];
  __builtin_amdgcn_wave_barrier();
  ReadSegmentPieces<kQ1, 64>(st, hp1, lane, mine->q1);
  mine->qr = AsV4i(r[0], r[1]);
  mine->wsum = wsum;
  mine->f = a.jacobian + a.jac_base[0][0] + a.jac_stride[0] * i0;
  mine->e = a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * i0;
  mine->r = a.residuals + a.res_base + (int64_t)NR * i0;
  mine->part = partial_dst;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  asm volatile("" : "+v"(mine->wsum));
  // ---- the chunk's stores, back to back ----
  static_assert(kQ0 == 9 && kQ1 == 3, "the Snavely cells: 9 F pieces, 3 E pieces a lane");
  StoreSaddr16<0>(mine->f, off.f0, mine->q0[0]);
  StoreSaddr16<1024>(mine->f, off.f0, mine->q0[1]);
  StoreSaddr16<2048>(mine->f, off.f0, mine->q0[2]);
  StoreSaddr16<3072>(mine->f, off.f0, mine->q0[3]);
  StoreSaddr16<0>(mine->f, off.f4, mine->q0[4]);
  StoreSaddr16<1024>(mine->f, off.f4, mine->q0[5]);
  StoreSaddr16<2048>(mine->f, off.f4, mine->q0[6]);
  StoreSaddr16<3072>(mine->f, off.f4, mine->q0[7]);
  StoreSaddr16<0>(mine->f, off.flast, mine->q0[8]);
  StoreSaddr16<0>(mine->e, off.e0, mine->q1[0]);
  StoreSaddr16<1024>(mine->e, off.e0, mine->q1[1]);
  StoreSaddr16<0>(mine->e, off.elast, mine->q1[2]);
  StoreSaddr16<0>(mine->r, off.r, mine->qr);
  if (lane == 0) {
    StoreSaddr8(mine->part, off.zero, mine->wsum);
    if (failed) StoreB32(a.status, 1);
  }
  PersistKeep(prev);
}

template <class K, int kLoss>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(2))) void
EvaluateAffinePersistent(const GroupArgs a) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, X0 = Tr::X0;
  static_assert(Tr::NB == 2 && Tr::D == 2 && S1 == 3 && NR % 2 == 0 && (NR * S0) % 2 == 0 &&
                    (NR * S1) % 2 == 0 && !MayLeaveOutputs<K>::value,
                "persistent kernel: two-slot kinds with 3-double points and 2 data doubles");
  constexpr int kQ0 = NR * S0 / 2, kQ1 = NR * S1 / 2;
  constexpr int X0p = (X0 + 1) & ~1;
  static_assert(kQ0 <= 9 && kQ1 <= 8, "segment stores: two base registers");
  __shared__ alignas(16) double camb[2][kWave * X0p];
  __shared__ alignas(16) double st[kWave * NR * (S0 > S1 ? S0 : S1)];
  const int lane = threadIdx.x;
  const int64_t num_chunks = (a.n + kWave - 1) / kWave;
  const int64_t stride = gridDim.x;
  int64_t c = blockIdx.x;
  if (c >= num_chunks) return;
  PersistNext A, B;
  long long id0;
  {
    const long long* pi = reinterpret_cast<const long long*>(a.ids) + PersistBlock(c, lane, a.n);
    asm volatile("global_load_dwordx2 %0, %1, off nt\n\ts_waitcnt vmcnt(0)" : "=v"(id0) : "v"(pi)
                 : "memory");
  }
  PersistIssueGather<K>(a, camb[0], c, c + stride, id0, lane, &A);
  // The store tail's per-lane offsets: every chunk's segments have the
  // alignment of chunk 0's (64 blocks = a multiple of 64 bytes in each).
  const int hp0 = SectorHeadPieces<64>(a.jacobian + a.jac_base[0][0]);
  const int hp1 = SectorHeadPieces<64>(a.jacobian + a.jac_base[1][0]);
  PersistOffsets off;
  off.f0 = 16u * (lane + hp0);
  off.f4 = off.f0 + 4096u;
  off.flast = 16u * LastPiece<kQ0, 64>(lane, hp0);
  off.e0 = 16u * (lane + hp1);
  off.elast = 16u * LastPiece<kQ1, 64>(lane, hp1);
  off.r = 16u * lane;
  off.zero = 0u;
  asm volatile("" : "+v"(off.f0), "+v"(off.f4), "+v"(off.flast), "+v"(off.e0), "+v"(off.elast),
               "+v"(off.r), "+v"(off.zero));
  PersistSet<kQ0, kQ1> S0set{}, S1set{};
  PersistWait<0>(&A);
  __builtin_amdgcn_wave_barrier();
  constexpr int kOps = PersistStoreOps<K>();
  for (;;) {
    PersistChunk<K, kLoss, kQ0, kQ1>(a, c, stride, num_chunks, camb[0], camb[1], st, &A, &B, &S0set,
                                     S1set, off, hp0, hp1, lane);
    c += stride;
    if (c >= num_chunks) break;
    PersistWait<kOps>(&B);
    __builtin_amdgcn_wave_barrier();
    PersistChunk<K, kLoss, kQ0, kQ1>(a, c, stride, num_chunks, camb[1], camb[0], st, &B, &A, &S1set,
                                     S0set, off, hp0, hp1, lane);
    c += stride;
    if (c >= num_chunks) break;
    PersistWait<kOps>(&A);
    __builtin_amdgcn_wave_barrier();
  }
  PersistKeep(S0set);
  PersistKeep(S1set);
  asm volatile("" ::"v"(off.f0), "v"(off.f4), "v"(off.flast), "v"(off.e0), "v"(off.elast), "v"(off.r),
               "v"(off.zero));
}

}  // namespace cse

#endif  // CSE_PERSISTENT_KERNEL_HPP_
