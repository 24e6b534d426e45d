// pgs_kernel.hpp -- tuning build only: the group-store BSM kernel
// (csrc/group_store_kernel.hpp) in a persistent, software-pipelined form.
//
// Why (the round-5 phase stamps): a wave of the shipped
// kernels spends ~58 % of its life in two dependent load phases (the ids,
// then the camera LDS-DMA, observations and points) queued behind the CU's
// outstanding stores.  Here each workgroup walks quads q, q + G, ... (G =
// the grid, three workgroups per CU); within quad q each wave
//   evaluates its chunk from inputs that arrived during quad q - G,
//   stages F, E and residuals into the workgroup image, barrier, reads its
//   13 pieces, barrier (the image is free again),
//   issues quad q + G's gather (camera rows by LDS-DMA into its own F
//   region of the image, observation and point into registers) and the ids
//   of quad q + 2G, THEN its 13 stores,
//   and waits with `s_waitcnt vmcnt(13)`: the gather is complete, the stores
//   may stay in flight.
// So the loads are queued ahead of the wave's own stores and the ids are two
// quads ahead.  The 13 store registers are kept alive through the next
// quad's functor (one register set: the next quad's pieces are read only
// after its compute, by when the stores have long read them).
// Outputs are bit-identical to the shipped kernels'.  Full, 64-byte-aligned
// quads only (GroupStoreEligible); the last, partial quad goes through the
// slow tail.
#ifndef CSE_PGS_KERNEL_HPP_
#define CSE_PGS_KERNEL_HPP_

#include "../../ceres-solver-cuda_amd/csrc/group_store_kernel.hpp"

namespace cse {

typedef double pgs_v2d __attribute__((ext_vector_type(2)));

// Byte offsets inside a wave's F region (9 KiB) of the landing areas: camera
// rows [0, 5 KiB), observations, the points' two 12-byte pieces.
// (x, y) by one 16-byte piece a lane, z by two 4-byte pieces: widths whose
// lane-linear LDS layout is certain (16 and 4 bytes a lane).
constexpr uint32_t kPgsObsOff = 5 * 1024, kPgsXyOff = 6 * 1024, kPgsZloOff = 7 * 1024,
                   kPgsZhiOff = 7 * 1024 + 256,
                   // the ids of the chunk after next: (camera, point), 4 bytes a lane each
                   kPgsIdcOff = 7 * 1024 + 512, kPgsIdpOff = 7 * 1024 + 768;

// The observation pair and the point of `lane` from the landing areas.
__device__ __forceinline__ void PgsReadInputs(const double* fw, int lane, double* d, double* x1) {
  const char* b = reinterpret_cast<const char*>(fw);
  const double2 ob = *reinterpret_cast<const double2*>(b + kPgsObsOff + 16 * lane);
  d[0] = ob.x;
  d[1] = ob.y;
  const double2 xy = *reinterpret_cast<const double2*>(b + kPgsXyOff + 16 * lane);
  const uint32_t zlo = *reinterpret_cast<const uint32_t*>(b + kPgsZloOff + 4 * lane);
  const uint32_t zhi = *reinterpret_cast<const uint32_t*>(b + kPgsZhiOff + 4 * lane);
  x1[0] = xy.x;
  x1[1] = xy.y;
  x1[2] = __builtin_bit_cast(double, ((uint64_t)zhi << 32) | zlo);
}

// 16-byte store at SGPR base + VGPR offset + kOff bytes, `sc1 nt`.
template <int kOff>
__device__ __forceinline__ void PgsStore16(const double* base, uint32_t voff, const cse_v4i& d) {
  static_assert(kOff >= 0 && kOff <= 4095, "global offset out of range");
  asm volatile("global_store_dwordx4 %0, %1, %2 offset:%3 sc1 nt" ::"v"(voff), "v"(d), "s"(base), "i"(kOff)
               : "memory");
}

// Run stores: N 1-KiB instructions from q + J0, base = the run's first byte.
template <int J, int N, int J0>
__device__ __forceinline__ void PgsRun(const double* base, uint32_t voff, const cse_v4i* q) {
  if constexpr (J < N) {
    PgsStore16<(J % 4) * 1024>(base + 512 * (J / 4), voff, q[J0 + J]);
    PgsRun<J + 1, N, J0>(base, voff, q);
  }
}

template <int w>
__device__ __forceinline__ void PgsStores(double* const bases[3], uint32_t voff, const cse_v4i* q) {
  using P = QuadPart<4, 0, w>;
  const double* b0 = bases[0] + 128 * (P::s(0) - P::rb(0));
  const double* b1 = bases[1] + 128 * (P::s(1) - P::rb(1));
  const double* b2 = bases[2] + 128 * (P::s(2) - P::rb(2));
  PgsRun<0, P::n(0), 0>(b0, voff, q);
  PgsRun<0, P::n(1), P::n(0)>(b1, voff, q);
  PgsRun<0, P::n(2), P::n(0) + P::n(1)>(b2, voff, q);
}

// Queue chunk c's gather: camera rows by LDS-DMA into lds (5 pieces a row),
// the observation pair and the point into registers; and the ids of chunk
// cn (if cn >= 0).  All inline asm: invisible to the compiler's waits.
template <class K>
__device__ __forceinline__ void PgsIssueGather(const GroupArgs& a, double* lds, int64_t c, long long id,
                                               int64_t cn, int lane, pgs_v2d* o, double* p,
                                               long long* idn, uint32_t ids_lds) {
  using Tr = KindTraits<K>;
  constexpr int X0 = Tr::X0, X0p = (X0 + 1) & ~1, kPieces = X0p / 2;
  constexpr int kRow = PackedRowDoubles(X0);
  const int cid_own = (int)id - a.packed0_lo, pid = (int)(id >> 32);
  const uint32_t lbase = (uint32_t)reinterpret_cast<uintptr_t>(lds);
#pragma unroll
  for (int k = 0; k < kPieces; ++k) {
    const int pc = k * kWave + lane;
    const int t = pc / kPieces, qq = pc - t * kPieces;
    const int cid = __shfl(cid_own, t, kWave);
    const double* src = a.packed0 + (int64_t)kRow * cid + 2 * qq;
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(lbase + 2u * kWave * 8u * k);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0)
                 : "memory", "m0");
  }
  // The observation pair (16 B a lane) and the point (two 12-byte pieces a
  // lane) by LDS-DMA too, after the camera rows in the same region: no VGPR
  // holds them while they are in flight.
  // (An LDS-DMA instruction's immediate offset moves its LDS destination
  // too, so every source offset is in the address register, offset 0.)
  const double* po = a.data + 2 * (c * kWave + lane);
  const uint32_t mo = __builtin_amdgcn_readfirstlane(lbase + kPgsObsOff);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off nt" ::"v"(po), "s"(mo)
               : "memory", "m0");
  const double* pt = a.state + a.state_base[1] + 3LL * pid;
  const uint32_t mxy = __builtin_amdgcn_readfirstlane(lbase + kPgsXyOff);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off nt" ::"v"(pt), "s"(mxy)
               : "memory", "m0");
  const char* pz = reinterpret_cast<const char*>(pt) + 16;
  const uint32_t mzl = __builtin_amdgcn_readfirstlane(lbase + kPgsZloOff);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off nt" ::"v"(pz), "s"(mzl)
               : "memory", "m0");
  const uint32_t mzh = __builtin_amdgcn_readfirstlane(lbase + kPgsZhiOff);
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off nt" ::"v"(pz + 4), "s"(mzh)
               : "memory", "m0");
  (void)o;
  (void)p;
  (void)idn;
  if (cn >= 0) {  // into a second id slot (the current ids were read from the first)
    const int32_t* pi = a.ids + 2 * (cn * kWave + lane);
    const uint32_t mic = __builtin_amdgcn_readfirstlane(ids_lds + kPgsIdcOff);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off nt" ::"v"(pi), "s"(mic)
                 : "memory", "m0");
    const uint32_t mip = __builtin_amdgcn_readfirstlane(ids_lds + kPgsIdpOff);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off nt" ::"v"(pi + 1), "s"(mip)
                 : "memory", "m0");
  }
}

template <class K, int kLoss>
__global__ __launch_bounds__(kBlockThreads) __attribute__((amdgpu_waves_per_eu(3))) void
EvaluateGroupStorePipelined(const GroupArgs a, int64_t nfull) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p, X0 = Tr::X0;
  constexpr int X0p = (X0 + 1) & ~1;
  static_assert(NR == 2 && S0 == 9 && S1 == 3 && Tr::D == 2, "Snavely-shaped kinds");
  constexpr int kImg = 52 * 128;
  __shared__ __attribute__((aligned(16))) double img[kImg];
  const int lane = threadIdx.x & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  double* fw = img + w * (NR * S0 * kWave);
  double* ew = img + kQuadFk * 4 * 128 + w * (NR * S1 * kWave);
  double* rw = img + (kQuadFk + kQuadEk) * 4 * 128 + w * (NR * kWave);
  const int64_t G = gridDim.x;
  const uint32_t voff = 16u * lane;
  const uint32_t ids_lds = (uint32_t)reinterpret_cast<uintptr_t>(fw);
  int64_t q = blockIdx.x;
  long long idn = 0, idnn = 0;
  pgs_v2d o = {0.0, 0.0}, on = {0.0, 0.0};  // (unused: the inputs land in LDS)
  double pt[3] = {0, 0, 0}, ptn[3] = {0, 0, 0};
  cse_v4i qv[13];
#pragma unroll
  for (int j = 0; j < 13; ++j) qv[j] = cse_v4i{0, 0, 0, 0};
  if (q < nfull) {
    long long id0;
    const long long* pi = reinterpret_cast<const long long*>(a.ids) + (q * 4 + w) * kWave + lane;
    asm volatile("global_load_dwordx2 %0, %1, off nt\n\ts_waitcnt vmcnt(0)" : "=v"(id0) : "v"(pi) : "memory");
    PgsIssueGather<K>(a, fw, q * 4 + w, id0, q + G < nfull ? (q + G) * 4 + w : -1, lane, &o, pt, &idn,
                      ids_lds);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  for (; q < nfull; q += G) {
    const int64_t c = q * 4 + w;
    double d[2], x0[X0], x1[3];
#pragma unroll
    for (int k = 0; k < X0; ++k) x0[k] = fw[lane * X0p + k];
    PgsReadInputs(fw, lane, d, x1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    double r[NR], J0[NR * S0], J1[NR * S1p];
    bool ok = EvaluateFunctor<K, true>(d, x0, x1, r, J0, J1);
    if (ok && a.check_finite)
      ok = !(AnyNonFinite<NR>(r) || AnyNonFinite<NR * S0>(J0) || AnyNonFinite<NR * S1>(J1));
    const double cost = LossAndCorrect<K, kLoss, true>(a.loss, a.apply_loss, r, J0, J1, true);
    const double wsum = WaveSumLane0(cost);
    const bool failed = __ballot(!ok) != 0;
    // the next quad's ids (landed with this quad's inputs), before the
    // staging below overwrites the landing areas
    {
      const char* fb = reinterpret_cast<const char*>(fw);
      const uint32_t ic = *reinterpret_cast<const uint32_t*>(fb + kPgsIdcOff + 4 * lane);
      const uint32_t ip = *reinterpret_cast<const uint32_t*>(fb + kPgsIdpOff + 4 * lane);
      idn = (long long)(((uint64_t)ip << 32) | ic);
    }
    KeepAlive<13>(qv);  // the previous quad's stores may still be reading these
#pragma unroll
    for (int k = 0; k < NR * S0; k += 2)
      *reinterpret_cast<double2*>(fw + lane * NR * S0 + k) = make_double2(J0[k], J0[k + 1]);
#pragma unroll
    for (int k = 0; k < NR * S1; k += 2)
      *reinterpret_cast<double2*>(ew + lane * NR * S1 + k) = make_double2(J1[k], J1[k + 1]);
    *reinterpret_cast<double2*>(rw + lane * NR) = make_double2(r[0], r[1]);
    __syncthreads();
    {
      const double2* im2 = reinterpret_cast<const double2*>(img);
#pragma unroll
      for (int j = 0; j < 13; ++j) {
        const double2 v = im2[(13 * w + j) * kWave + lane];
        qv[j] = AsV4i(v.x, v.y);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    // the chunk's partial and failure flag, ahead of the loads below
    if (lane == 0) {
      StoreB64(a.partials + c, wsum);
      if (failed) StoreB32(a.status, 1);
    }
    // quad q + G's gather and the ids of q + 2G, ahead of this quad's stores
    const int64_t qn = q + G;
    if (qn < nfull)
      PgsIssueGather<K>(a, fw, qn * 4 + w, idn, qn + G < nfull ? (qn + G) * 4 + w : -1, lane, &on, ptn,
                        &idnn, ids_lds);
    const int64_t b0 = q * 4 * kWave;
    double* const bases[3] = {a.jacobian + a.jac_base[0][0] + a.jac_stride[0] * b0,
                              a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * b0,
                              a.residuals + a.res_base + (int64_t)NR * b0};
    switch (w) {
      case 0: PgsStores<0>(bases, voff, qv); break;
      case 1: PgsStores<1>(bases, voff, qv); break;
      case 2: PgsStores<2>(bases, voff, qv); break;
      default: PgsStores<3>(bases, voff, qv); break;
    }
    // the gather (older than the 13 stores) has landed
    asm volatile("s_waitcnt vmcnt(13)" ::: "memory");
  }
  KeepAlive<13>(qv);
  asm volatile("" ::"v"(voff));
  // The last, partial quad (if any): its workgroup, not pipelined.
  const int64_t nq = (a.n + 4 * kWave - 1) / (4 * kWave);
  if (nfull < nq && blockIdx.x == nfull % G) {
    const int64_t num_chunks = (a.n + kWave - 1) / kWave;
    const int64_t c = nfull * 4 + w;
    __syncthreads();
    if (c < num_chunks) {
      const int64_t i0 = c * kWave, rem = a.n - i0;
      const int nw = rem < kWave ? (int)rem : kWave;
      const bool active = lane < nw;
      const int64_t i = active ? i0 + lane : a.n - 1;
      AffineInputs<K> in;
      const long long b = __builtin_nontemporal_load(reinterpret_cast<const long long*>(a.ids) + i);
      GatherCoopDma<K>(a, i, make_int2((int)b, (int)(b >> 32)), &in, fw, lane);
      double r[NR], J0[NR * S0], J1[NR * S1p];
      bool ok = EvaluateFunctor<K, true>(in.d, in.x0, in.x1, r, J0, J1);
      if (ok && a.check_finite)
        ok = !(AnyNonFinite<NR>(r) || AnyNonFinite<NR * S0>(J0) || AnyNonFinite<NR * S1>(J1));
      const double cost = LossAndCorrect<K, kLoss, true>(a.loss, a.apply_loss, r, J0, J1, true);
      const double wsum = WaveSumLane0(active ? cost : 0.0);
      const bool failed = __ballot(active && !ok) != 0;
      StageAndStore<K, true, false>(a, fw, lane, active, i0, nw, r, J0, J1);
      if (lane == 0) {
        a.partials[c] = wsum;
        if (failed) *a.status = 1;
      }
    }
  }
}

}  // namespace cse

#endif  // CSE_PGS_KERNEL_HPP_
