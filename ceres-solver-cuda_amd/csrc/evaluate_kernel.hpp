// evaluate_kernel.hpp -- the fused residual/Jacobian/loss/cost kernel.
//
// One wavefront lane owns one residual block (the reference's
// EvaluateKernel, include/ceres/internal/cuda_evaluator_kernel.h:297-422,
// also maps one thread to one block).  Per lane, fused in one pass:
//   gather parameters -> Jet autodiff of the functor -> plus-Jacobian
//   product (manifolds) -> loss rho(|r|^2) and Corrector on J then r ->
//   residual/Jacobian stores -> gradient J^T r -> cost into a per-workgroup
//   partial (summed deterministically by cse_finalize_kernel).
//
// Two layout policies, chosen per residual group on the host:
//   kAffine = true   table-free: block i of the group writes its residuals
//                    at res_base + kR*i and row k of slot j at
//                    jac_base[j][k] + jac_stride[j]*i, and reads parameter
//                    block `id` at state_base[j] + size_j*id.  This is what
//                    BlockJacobianWriter and CompressedRowJacobianWriter
//                    produce for Schur-ordered BAL problems; the kernel then
//                    reads only 8 B of ids + functor data per block.
//   kAffine = false  the reference's offset tables (residual_layout,
//                    jacobian_per_residual_layout/offsets, per-block
//                    parameter-block records): any layout, constant blocks,
//                    manifolds.
// Wide outputs of the affine path are staged through LDS so each wave
// writes its contiguous output segments with 16-byte-per-lane stores.
#ifndef CSE_EVALUATE_KERNEL_HPP_
#define CSE_EVALUATE_KERNEL_HPP_

#include <stdint.h>

#include "functors.hpp"
#include "jet.hpp"
#include "loss.hpp"

namespace cse {

constexpr int kBlockThreads = 256;
constexpr int kWave = 64;

// Device copy of a parameter block (general path).
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
  LossParams loss;
  int apply_loss;
  int check_finite;
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

CSE_HD int64_t GlobalIndex(const GroupArgs& a, int64_t i) {
  return a.gindex ? a.gindex[i] : a.first + i;
}

// Deterministic workgroup sum: xor-butterfly inside each wave, then waves
// in a fixed order.  Returns the sum in thread 0.
__device__ __forceinline__ double WorkgroupSum(double v, double* lds4) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  if (lane == 0) lds4[wave] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 0; w < kBlockThreads / kWave; ++w) t += lds4[w];
  }
  return t;
}

// Copy `count` doubles (per-lane staged in LDS, contiguous) to global
// memory at dst with all 64 lanes cooperating.  16-byte stores when the
// destination is 16-byte aligned, 8-byte stores otherwise.
__device__ __forceinline__ void WaveStore(const double* lds, double* dst, int count, int lane) {
  if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    const int pairs = count >> 1;
    for (int t = lane; t < pairs; t += kWave) {
      const double2 v = *reinterpret_cast<const double2*>(lds + 2 * t);
      *reinterpret_cast<double2*>(dst + 2 * t) = v;
    }
    if ((count & 1) && lane == 0) dst[count - 1] = lds[count - 1];
  } else {
    for (int t = lane; t < count; t += kWave) dst[t] = lds[t];
  }
}

template <class K>
struct KindTraits {
  static constexpr int NR = K::kNumResiduals;
  static constexpr int NB = K::kNumBlocks;
  static constexpr int S0 = K::kSize0;
  static constexpr int S1 = K::kSize1;
  static constexpr int S1p = S1 > 0 ? S1 : 1;
  static constexpr int N = S0 + S1;
  static constexpr int D = K::kDataSize;
  // Doubles of Jacobian a block produces (all slots active, no manifold).
  static constexpr int kJacPerBlock = NR * N;
};

// The kernel.  kJac: Jacobian and/or gradient requested (Jets); otherwise
// the functor runs on plain doubles (the reference always runs Jets,
// cuda_evaluator_kernel.h:327-345).
template <class K, int kLoss, bool kJac, bool kAffine>
__global__ __launch_bounds__(kBlockThreads) void EvaluateGroupKernel(const GroupArgs a) {
  using Tr = KindTraits<K>;
  constexpr int NR = Tr::NR, NB = Tr::NB, S0 = Tr::S0, S1 = Tr::S1, S1p = Tr::S1p;
  constexpr int N = Tr::N, D = Tr::D;
  // LDS staging for the affine path's stores (per wave: its 64 blocks'
  // residuals and each slot's Jacobian cells).
  constexpr int kStage = kAffine ? (kJac ? kWave * NR * N : kWave * NR) : 1;
  __shared__ double stage[kBlockThreads / kWave][kStage];
  __shared__ double lds4[kBlockThreads / kWave];

  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x / kWave;
  const int64_t i = (int64_t)blockIdx.x * kBlockThreads + threadIdx.x;
  const bool active = i < a.n;
  const bool want_res = a.residuals != nullptr;
  const bool want_jac = kJac && a.jacobian != nullptr;
  const bool want_grad = kJac && a.gradient != nullptr;

  double cost = 0.0;
  double r[NR];
  double J0[NR * S0];
  double J1[NR * S1p];
  bool ok = true;

  // --- gather -------------------------------------------------------------
  int32_t id[2] = {0, 0};
  const double* p0 = nullptr;
  const double* p1 = nullptr;
  int64_t delta[2] = {0, 0};
  int tan[2] = {S0, S1};
  bool cst[2] = {false, false};
  int64_t pjo[2] = {-1, -1};
  double d[D];
  if (active) {
    if constexpr (NB == 2) {
      const int2 ii = *reinterpret_cast<const int2*>(a.ids + 2 * i);
      id[0] = ii.x;
      id[1] = ii.y;
    } else {
      id[0] = a.ids[i];
    }
#pragma unroll
    for (int k = 0; k < D; ++k) d[k] = a.data[i * D + k];
    if constexpr (kAffine) {
      p0 = a.state + a.state_base[0] + (int64_t)S0 * id[0];
      delta[0] = a.delta_base[0] + (int64_t)S0 * id[0];
      if constexpr (NB == 2) {
        p1 = a.state + a.state_base[1] + (int64_t)S1 * id[1];
        delta[1] = a.delta_base[1] + (int64_t)S1 * id[1];
      }
    } else {
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const PbDev pb = a.pbs[id[j]];
        const double* p = (pb.is_constant ? a.cstate : a.state) + pb.state_offset;
        if (j == 0) p0 = p; else p1 = p;
        delta[j] = pb.delta_offset;
        tan[j] = pb.tangent_size;
        cst[j] = pb.is_constant != 0;
        pjo[j] = pb.plus_jacobian_offset;
      }
    }
  }

  if (active) {
    double x0[S0], x1[S1p];
#pragma unroll
    for (int k = 0; k < S0; ++k) x0[k] = p0[k];
#pragma unroll
    for (int k = 0; k < S1; ++k) x1[k] = p1[k];

    // --- autodiff -----------------------------------------------------------
    if constexpr (kJac) {
      // AutoDifferentiate (include/ceres/internal/autodiff.h:314-381).
      Jet<N> j0[S0], j1[S1p], out[NR];
#pragma unroll
      for (int k = 0; k < S0; ++k) j0[k] = Jet<N>(x0[k], k);
#pragma unroll
      for (int k = 0; k < S1; ++k) j1[k] = Jet<N>(x1[k], S0 + k);
      ok = K::Evaluate(d, j0, j1, out);
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        r[k] = out[k].a;
#pragma unroll
        for (int c = 0; c < S0; ++c) J0[k * S0 + c] = out[k].v[c];
#pragma unroll
        for (int c = 0; c < S1; ++c) J1[k * S1p + c] = out[k].v[S0 + c];
      }
    } else {
      ok = K::Evaluate(d, x0, x1, r);
    }
    if (ok && a.check_finite) {
      bool bad = AnyNonFinite<NR>(r);
      if constexpr (kJac) bad = bad || AnyNonFinite<NR * S0>(J0) || AnyNonFinite<NR * S1>(J1);
      ok = !bad;
    }
    if (!ok) *a.status = 1;

    double sq = 0.0;
#pragma unroll
    for (int k = 0; k < NR; ++k) sq += r[k] * r[k];

    if constexpr (kJac && !kAffine) {
      // Local Jacobian = ambient Jacobian * PlusJacobian
      // (cuda_evaluator_kernel.h:355-371; residual_block.cc:133-156).
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        if (pjo[j] < 0) continue;
        const double* PJ = a.plus_jacobians + pjo[j];
        const int t = tan[j];
        constexpr int kS = 0;
        (void)kS;
        if (j == 0) {
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
        } else {
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
    }

    // --- loss and correction (cuda_evaluator_kernel.h:373-407) -------------
    const bool robust = (kLoss != kLossTrivial || a.loss.scaled) && a.apply_loss;
    if (!robust) {
      cost = 0.5 * sq;
    } else {
      double rho[3];
      EvaluateLoss<kLoss>(a.loss, sq, rho);
      cost = 0.5 * rho[0];
      const Corrector corr(sq, rho);
      if constexpr (kJac) {
        corr.template CorrectJacobian<NR, S0>(r, J0);
        if constexpr (S1 > 0) corr.template CorrectJacobian<NR, S1p>(r, J1);
      }
      corr.template CorrectResiduals<NR>(r);
    }
    if (!ok) cost = 0.0;

    // --- gradient g += J^T r (cuda_evaluator_kernel.h:149-160,409-414) ------
    if (want_grad && ok) {
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        if (cst[j]) continue;
        double* g = a.gradient + delta[j];
        if (j == 0) {
#pragma unroll
          for (int c = 0; c < S0; ++c) {
            if (c >= tan[0]) break;
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < NR; ++k) s += J0[k * S0 + c] * r[k];
            unsafeAtomicAdd(g + c, s);
          }
        } else {
#pragma unroll
          for (int c = 0; c < S1; ++c) {
            if (c >= tan[1]) break;
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < NR; ++k) s += J1[k * S1p + c] * r[k];
            unsafeAtomicAdd(g + c, s);
          }
        }
      }
    }
  }

  // --- stores --------------------------------------------------------------
  if constexpr (kAffine) {
    // Stage this wave's outputs in LDS, then write each contiguous segment
    // with all lanes.  Wave-uniform: every lane takes the same path, the
    // wave's block range [i0, i0 + nw) is contiguous in every segment.
    const int64_t i0 = (int64_t)blockIdx.x * kBlockThreads + wave * kWave;
    const int64_t rem = a.n - i0;
    const int nw = rem <= 0 ? 0 : (rem < kWave ? (int)rem : kWave);
    double* st = stage[wave];
    if (want_res && nw > 0) {
      if (active) {
#pragma unroll
        for (int k = 0; k < NR; ++k) st[lane * NR + k] = r[k];
      }
      __builtin_amdgcn_wave_barrier();
      WaveStore(st, a.residuals + a.res_base + (int64_t)NR * i0, nw * NR, lane);
      __builtin_amdgcn_wave_barrier();
    }
    if constexpr (kJac) {
      if (want_jac && nw > 0) {
        // Slot j occupies rows k at jac_base[j][k] + jac_stride[j]*i.  Two
        // shapes are contiguous per wave: a packed cell (rows adjacent,
        // stride = kR*size; BlockSparseMatrix) and interleaved rows
        // covering all slots (stride = kR*N; CompressedRowSparseMatrix).
        const bool crs = a.jac_stride[0] == (int64_t)NR * N;
        if (crs) {
          // Row k of block i = [slot in column order] at jac_base[.][k].
          // Build the block's kR*N doubles in memory order.
          const int64_t row0 = a.jac_base[0][0] < a.jac_base[NB - 1][0] ? a.jac_base[0][0]
                                                                          : a.jac_base[NB - 1][0];
          if (active) {
#pragma unroll
            for (int k = 0; k < NR; ++k) {
#pragma unroll
              for (int c = 0; c < S0; ++c)
                st[lane * NR * N + (int)(a.jac_base[0][k] - row0) + c] = J0[k * S0 + c];
#pragma unroll
              for (int c = 0; c < S1; ++c)
                st[lane * NR * N + (int)(a.jac_base[1][k] - row0) + c] = J1[k * S1p + c];
            }
          }
          __builtin_amdgcn_wave_barrier();
          WaveStore(st, a.jacobian + row0 + (int64_t)NR * N * i0, nw * NR * N, lane);
          __builtin_amdgcn_wave_barrier();
        } else {
          if (active) {
#pragma unroll
            for (int q = 0; q < NR * S0; ++q) st[lane * NR * S0 + q] = J0[q];
          }
          __builtin_amdgcn_wave_barrier();
          WaveStore(st, a.jacobian + a.jac_base[0][0] + a.jac_stride[0] * i0, nw * NR * S0, lane);
          __builtin_amdgcn_wave_barrier();
          if constexpr (S1 > 0) {
            if (active) {
#pragma unroll
              for (int q = 0; q < NR * S1; ++q) st[lane * NR * S1 + q] = J1[q];
            }
            __builtin_amdgcn_wave_barrier();
            WaveStore(st, a.jacobian + a.jac_base[1][0] + a.jac_stride[1] * i0, nw * NR * S1,
                      lane);
            __builtin_amdgcn_wave_barrier();
          }
        }
      }
    }
  } else if (active && ok) {
    const int64_t gi = GlobalIndex(a, i);
    if (want_res) {
      double* dst = a.residuals + a.residual_layout[gi];
#pragma unroll
      for (int k = 0; k < NR; ++k) dst[k] = r[k];
    }
    if (want_jac) {
      // WriteJacobians (cuda_evaluator_kernel.h:260-294): row k of the
      // a-th active slot goes to values + offsets[layout[gi] + a*kR + k].
      int64_t idx = a.jac_layout[gi];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        if (cst[j]) continue;
#pragma unroll
        for (int k = 0; k < NR; ++k) {
          double* dst = a.jacobian + a.jac_offsets[idx++];
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

  // --- cost partial --------------------------------------------------------
  const double t = WorkgroupSum(cost, lds4);
  if (threadIdx.x == 0) a.partials[blockIdx.x] = t;
}

// Sums the per-workgroup partials of every group in a fixed order, writes
// the cost, publishes the evaluation status and re-arms the status word
// for the next evaluation (replaces thrust::reduce + the abort-flag round
// trip, autodiff_residual_block_cuda_evaluator.h:241-265).
__global__ __launch_bounds__(1024) void FinalizeKernel(const double* partials, int64_t n,
                                                       double* cost, int* status,
                                                       int* status_out) {
  __shared__ double wsum[1024 / kWave];
  double v = 0.0;
  for (int64_t k = threadIdx.x; k < n; k += blockDim.x) v += partials[k];
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

}  // namespace cse

#endif  // CSE_EVALUATE_KERNEL_HPP_
