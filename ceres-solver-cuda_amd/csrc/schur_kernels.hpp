// schur_kernels.hpp -- the implicit Schur complement on the evaluator's
// BlockSparseMatrix: ITERATIVE_SCHUR's linear operator and preconditioners
// (internal/ceres/implicit_schur_complement.cc, iterative_schur_complement_
// solver.cc, schur_jacobi_preconditioner.cc), on the Jacobian values where the
// evaluator wrote them in HBM.
//
// Structure (a Schur-ordered BAL problem): residual block i has one f block
// (slot 0, the camera: an F cell of 2 x S0 at f_base + 2 S0 i) and one e
// block (slot 1, the point: an E cell of 2 x 3 at e_base + 6 i); blocks are
// sorted by e block, so each e block's rows are one contiguous run.  The
// host cuts the runs into wave chunks of whole runs (at most 64 blocks);
// runs longer than a wave are the "big" e blocks, one wave each.
//
// With M_p = (E_p^T E_p + D_p^2)^-1 (3 x 3 per e block) the Schur complement
// is S = F^T F + D_f^2 - F^T E M E^T F.  Every operation below is, per e
// block p and its rows b:
//     s_p = sum_b E_b^T z_b,   w_p = M_p s_p,   u_b = z_b - E_b w_p
// followed by the f-block sum y_c += sum_{b of c} F_b^T u_b, with
//     init (UpdateRhs, implicit_schur_complement.cc:240-273):  z_b = b_b,
//          and M_p computed and stored (AddDiagonalAndInvert, :190-214);
//          u_b (and b_b, for the gradient) are written per block and one
//          camera-order pass (SchurCameraPassKernel) forms F^T u, F^T b and
//          the preconditioner's F^T Q F together, reading each F cell once
//     multiply (RightMultiplyAndAccumulate, :101-141):  z_b = F_b x_c, the
//          blocks' F_b^T u_b written in block order and summed per f block
//          in a fixed order by GradientContribKernel +
//          GradientChunkReduceKernel, as the fused gradient's camera rows
//     back substitution (BackSubstitute, :216-238):  z_b = b_b - F_b x_c,
//          y_p = w_p, no f-block sum.
// All sums run in a fixed order: results are bit-identical run to run.
#ifndef CSE_SCHUR_KERNELS_HPP_
#define CSE_SCHUR_KERNELS_HPP_

#include "operator_kernels.hpp"

namespace cse {

enum SchurMode { kSchurInit = 0, kSchurMultiply = 1, kSchurBack = 2 };

struct SchurArgs {
  int64_t n;               // residual blocks
  const int32_t* ids;      // [n][2]: f block (slot 0), e block (slot 1)
  const double* jac;       // BlockSparseMatrix values
  int64_t f_base, e_base;  // cell of block i: F at f_base + 2 S0 i, E at e_base + 6 i
  int64_t f_col_base;      // f-vector index of f block id: f_col_base + S0 id
  int64_t e_col_base;      // e column of e block id: e_col_base + 3 id
  int64_t e_cols;          // D[e_cols + k] scales f column k
  const double* D;         // [e_cols + f_cols], may be null
  const double* b;         // right-hand side rows: block i's pair at b + b_base + 2 i
  int64_t b_base;
  const double* x;         // f vector (multiply, back substitution)
  double* ete_inv;         // M_p, packed upper triangle, at ete_inv + 2 * (e column of p)
  double* contrib;         // multiply: [n][S0p] F_b^T u_b
  double* ub;              // init: [n][2] u_b, or [n][4] u_b then b_b with the gradient
  double* grad;            // init with the gradient: the e rows of g = J^T r = -J^T b
  double* y;               // back substitution: the full solution (e part written)
  const int64_t* chunk_begin;  // [nchunks][2] begin, end: wave chunks of whole e-block runs
  int64_t nchunks;
  const int64_t* big;      // [nbig][2] runs longer than a wave
  int64_t nbig;
  int* status;             // set to 1 when a pivot of E^T E + D_e^2 is not positive
};

// A Cholesky pivot that can be factored: positive and finite.  Bit tests:
// the kernels are compiled with -ffinite-math-only, which folds NaN checks.
__device__ __forceinline__ bool PivotOk(double p) {
  const uint64_t b = __builtin_bit_cast(uint64_t, p);
  return (b >> 63) == 0 && b != 0 && ((b >> 52) & 0x7ff) != 0x7ff;
}

// Packed upper triangle of a symmetric 3 x 3: (00, 01, 02, 11, 12, 22).
// M = (A + diag(d^2))^-1 by the Cholesky factor, as the reference's
// m.selfadjointView<Upper>().llt().solve(Identity) (implicit_schur_
// complement.cc:207-211): A = L L^T, M = L^-T L^-1.  Returns false (and M =
// 0) when a pivot is not positive -- A + diag(d^2) singular or indefinite,
// e.g. a point seen by a single residual block with D = NULL.  Eigen's LLT
// would return NaN/Inf there; the caller raises the status word instead.
__device__ __forceinline__ bool InvertSpd3(const double* A, const double* d, double* M) {
  const double a00 = A[0] + d[0] * d[0], a11 = A[3] + d[1] * d[1], a22 = A[5] + d[2] * d[2];
  const double p0 = a00;
  const double l00 = sqrt(p0);
  const double i00 = 1.0 / l00;
  const double l10 = A[1] * i00, l20 = A[2] * i00;
  const double p1 = a11 - l10 * l10;
  const double l11 = sqrt(p1);
  const double i11 = 1.0 / l11;
  const double l21 = (A[4] - l20 * l10) * i11;
  const double p2 = a22 - l20 * l20 - l21 * l21;
  const double l22 = sqrt(p2);
  const double i22 = 1.0 / l22;
  if (!(PivotOk(p0) && PivotOk(p1) && PivotOk(p2))) {
#pragma unroll
    for (int k = 0; k < 6; ++k) M[k] = 0.0;
    return false;
  }
  // L^-1 (lower): rows (i00), (j10 i11), (j20 j21 i22).
  const double j10 = -l10 * i00 * i11;
  const double j21 = -l21 * i11 * i22;
  const double j20 = -(l20 * i00 + l21 * j10) * i22;
  M[0] = i00 * i00 + j10 * j10 + j20 * j20;
  M[1] = j10 * i11 + j20 * j21;
  M[2] = j20 * i22;
  M[3] = i11 * i11 + j21 * j21;
  M[4] = j21 * i22;
  M[5] = i22 * i22;
  return true;
}

__device__ __forceinline__ void SymMul3(const double* M, const double* s, double* w) {
  w[0] = M[0] * s[0] + M[1] * s[1] + M[2] * s[2];
  w[1] = M[1] * s[0] + M[3] * s[1] + M[4] * s[2];
  w[2] = M[2] * s[0] + M[4] * s[1] + M[5] * s[2];
}

// One block's cells and z_b.
template <int S0, int kMode>
__device__ __forceinline__ void SchurLoadBlock(const SchurArgs& a, int64_t i, int id0, double* F,
                                               double* E, double* z) {
  const double2* ep = reinterpret_cast<const double2*>(a.jac + a.e_base + 6 * i);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double2 v = ep[k];
    E[2 * k] = v.x;
    E[2 * k + 1] = v.y;
  }
  {
    const double2* fp = reinterpret_cast<const double2*>(a.jac + a.f_base + 2 * S0 * i);
#pragma unroll
    for (int k = 0; k < S0; ++k) {
      const double2 v = fp[k];
      F[2 * k] = v.x;
      F[2 * k + 1] = v.y;
    }
  }
  if constexpr (kMode != kSchurMultiply) {
    const double2 v = *reinterpret_cast<const double2*>(a.b + a.b_base + 2 * i);
    z[0] = v.x;
    z[1] = v.y;
  }
  if constexpr (kMode != kSchurInit) {
    const double* xc = a.x + a.f_col_base + (int64_t)S0 * id0;
    double f0 = 0.0, f1 = 0.0;
#pragma unroll
    for (int k = 0; k < S0; ++k) {
      const double xv = xc[k];
      f0 += F[k] * xv;
      f1 += F[S0 + k] * xv;
    }
    if constexpr (kMode == kSchurMultiply) {
      z[0] = f0;
      z[1] = f1;
    } else {
      z[0] -= f0;
      z[1] -= f1;
    }
  }
}

// E_b^T z (3) and, for init, E_b^T E_b (packed, 6).
__device__ __forceinline__ void SchurEProducts(const double* E, const double* z, double* s,
                                               double* A) {
#pragma unroll
  for (int k = 0; k < 3; ++k) s[k] = E[k] * z[0] + E[3 + k] * z[1];
  A[0] = E[0] * E[0] + E[3] * E[3];
  A[1] = E[0] * E[1] + E[3] * E[4];
  A[2] = E[0] * E[2] + E[3] * E[5];
  A[3] = E[1] * E[1] + E[4] * E[4];
  A[4] = E[1] * E[2] + E[4] * E[5];
  A[5] = E[2] * E[2] + E[5] * E[5];
}

// u_b = z_b - E_b w, then F_b^T u_b (S0 values, padded to S0p) to contrib.
template <int S0>
__device__ __forceinline__ void SchurContrib(const SchurArgs& a, int64_t i, const double* F,
                                             const double* E, const double* z, const double* w) {
  constexpr int S0p = (S0 + 1) & ~1;
  const double u0 = z[0] - (E[0] * w[0] + E[1] * w[1] + E[2] * w[2]);
  const double u1 = z[1] - (E[3] * w[0] + E[4] * w[1] + E[5] * w[2]);
  double2* dst = reinterpret_cast<double2*>(a.contrib + (int64_t)S0p * i);
#pragma unroll
  for (int k = 0; k < S0p / 2; ++k) {
    const double c0 = F[2 * k] * u0 + F[S0 + 2 * k] * u1;
    const double c1 = 2 * k + 1 < S0 ? F[2 * k + 1] * u0 + F[S0 + 2 * k + 1] * u1 : 0.0;
    dst[k] = make_double2(c0, c1);
  }
}

// Init: block i's u_b (and b_b) record.
template <bool kGrad>
__device__ __forceinline__ void SchurStoreU(const SchurArgs& a, int64_t i, const double* E,
                                            const double* z, const double* w) {
  const double u0 = z[0] - (E[0] * w[0] + E[1] * w[1] + E[2] * w[2]);
  const double u1 = z[1] - (E[3] * w[0] + E[4] * w[1] + E[5] * w[2]);
  double2* dst = reinterpret_cast<double2*>(a.ub + (kGrad ? 4 : 2) * i);
  dst[0] = make_double2(u0, u1);
  if constexpr (kGrad) dst[1] = make_double2(z[0], z[1]);
}

// One wave per chunk of whole e-block runs.  The chunk's F cells and E cells
// are contiguous in the BlockSparseMatrix and come in by LDS-DMA (16-byte
// pieces, up to 1 KiB per instruction), as CgnrMultiplyKernel's image; each
// lane reads its block's cells from LDS.  The contributions F_b^T u_b are
// staged through the same LDS and leave as contiguous 16-byte pieces.
// kWPB: waves per workgroup (chunk = workgroup * kWPB + wave).
// Init reads no F cell: it writes u_b per block for the camera pass.
// kGrad (kSchurInit only): also the gradient g = J^T r = -J^T b, its e rows
// written here (-E^T b per e block), b_b beside u_b for its f rows.
template <int S0, int kMode, int kWPB = kWavesPerBlock, bool kGrad = false>
__global__ __launch_bounds__(kWPB * kWave) void SchurChunkKernel(const SchurArgs a) {
  static_assert(!kGrad || kMode == kSchurInit, "the gradient comes with the init pass");
  constexpr int S0p = (S0 + 1) & ~1;
  constexpr int kRec = S0p;                 // doubles per contribution record
  constexpr int kF = 2 * S0;                // doubles per F cell
  // F cells (not for init), then E cells, of up to a wave of blocks: init's
  // smaller image lets more waves stay resident.
  constexpr int kFImg = kMode == kSchurInit ? 0 : kWave * kF;
  constexpr int kImg = kFImg + kWave * 6;
  static_assert(kF % 2 == 0 && (kMode == kSchurInit || kWave * kRec <= kImg),
                "16-byte pieces; contributions fit");
  __shared__ double img_all[kWPB][kImg];
  const int lane = threadIdx.x & (kWave - 1), wave = kWPB == 1 ? 0 : threadIdx.x / kWave;
  const int64_t c = (int64_t)blockIdx.x * kWPB + wave;
  if (c >= a.nchunks) return;
  double* im = img_all[wave];
  const int64_t i0 = a.chunk_begin[2 * c];
  const int nb = (int)(a.chunk_begin[2 * c + 1] - i0);
  const bool active = lane < nb;
  const int64_t i = active ? i0 + lane : i0;
  {
    const double* segF = a.jac + a.f_base + (int64_t)kF * i0;
    const double* segE = a.jac + a.e_base + 6LL * i0;
    const int pf = (kF / 2) * nb, pe = 3 * nb;  // 16-byte pieces
    if constexpr (kMode != kSchurInit) {
#pragma unroll
      for (int k = 0; k < kF / 2; ++k) {
        const int p = k * kWave + lane;
        if (p < pf) __builtin_amdgcn_global_load_lds(segF + 2 * p, im + 2 * kWave * k, 16, 0, 0);
      }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int p = k * kWave + lane;
      if (p < pe)
        __builtin_amdgcn_global_load_lds(segE + 2 * p, im + kFImg + 2 * kWave * k, 16, 0, 0);
    }
  }
  const long long idw = reinterpret_cast<const long long*>(a.ids)[i];
  const int id0 = (int)idw, id1 = (int)(idw >> 32);
  double z[2] = {0.0, 0.0};
  if constexpr (kMode != kSchurMultiply) {
    const double2 v = *reinterpret_cast<const double2*>(a.b + a.b_base + 2 * i);
    z[0] = v.x;
    z[1] = v.y;
  }
  double xc[S0];
  if constexpr (kMode != kSchurInit) {
    const double* xp = a.x + a.f_col_base + (int64_t)S0 * id0;
#pragma unroll
    for (int k = 0; k < S0; ++k) xc[k] = xp[k];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  double F[kF], E[6];
  if constexpr (kMode != kSchurInit) {
#pragma unroll
    for (int k = 0; k < kF / 2; ++k) {
      const double2 v = reinterpret_cast<const double2*>(im + kF * lane)[k];
      F[2 * k] = v.x;
      F[2 * k + 1] = v.y;
    }
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double2 v = reinterpret_cast<const double2*>(im + kFImg + 6 * lane)[k];
    E[2 * k] = v.x;
    E[2 * k + 1] = v.y;
  }
  if constexpr (kMode != kSchurInit) {
    double f0 = 0.0, f1 = 0.0;
#pragma unroll
    for (int k = 0; k < S0; ++k) {
      f0 += F[k] * xc[k];
      f1 += F[S0 + k] * xc[k];
    }
    z[0] = kMode == kSchurMultiply ? f0 : z[0] - f0;
    z[1] = kMode == kSchurMultiply ? f1 : z[1] - f1;
  }
  double s[3], A[6];
  SchurEProducts(E, z, s, A);
  if (!active) {
#pragma unroll
    for (int k = 0; k < 3; ++k) s[k] = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) A[k] = 0.0;
  }
  // Runs are whole inside the chunk: a segmented scan leaves each run's
  // sums in its last lane, which every lane of the run then reads.
  const int key = active ? id1 : -1;
  SegmentedScan<3>(s, key, lane);
  if constexpr (kMode == kSchurInit) SegmentedScan<6>(A, key, lane);
  const int knext = __shfl_down(key, 1, kWave);
  const bool is_end = lane == kWave - 1 || knext != key;
  const uint64_t ends = __ballot(is_end);
  const int e = (int)__builtin_ctzll(ends >> lane) + lane;
#pragma unroll
  for (int k = 0; k < 3; ++k) s[k] = __shfl(s[k], e, kWave);
  const int64_t ecol = a.e_col_base + 3LL * id1;
  if constexpr (kGrad) {  // the e block's gradient rows, -E^T b
    if (active && lane == e) {
#pragma unroll
      for (int k = 0; k < 3; ++k) a.grad[ecol + k] = -s[k];
    }
  }
  double M[6];
  if constexpr (kMode == kSchurInit) {
#pragma unroll
    for (int k = 0; k < 6; ++k) A[k] = __shfl(A[k], e, kWave);
    double d[3] = {0.0, 0.0, 0.0};
    if (a.D) {
#pragma unroll
      for (int k = 0; k < 3; ++k) d[k] = a.D[ecol + k];
    }
    const bool ok = InvertSpd3(A, d, M);
    if (active && lane == e && !ok) *a.status = 1;
    if (active && lane == e) {
      double* m = a.ete_inv + 2 * ecol;
#pragma unroll
      for (int k = 0; k < 6; ++k) m[k] = M[k];
    }
  } else {
    const double2* m = reinterpret_cast<const double2*>(a.ete_inv + 2 * ecol);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const double2 v = m[k];
      M[2 * k] = v.x;
      M[2 * k + 1] = v.y;
    }
  }
  double w[3];
  SymMul3(M, s, w);
  if constexpr (kMode == kSchurBack) {
    if (active && lane == e) {
      double* yp = a.y + ecol;
      yp[0] = w[0];
      yp[1] = w[1];
      yp[2] = w[2];
    }
  } else if constexpr (kMode == kSchurInit) {
    if (active) SchurStoreU<kGrad>(a, i, E, z, w);
  } else {
    // F_b^T u_b, staged over the consumed image, out as contiguous pieces.
    const double u0 = z[0] - (E[0] * w[0] + E[1] * w[1] + E[2] * w[2]);
    const double u1 = z[1] - (E[3] * w[0] + E[4] * w[1] + E[5] * w[2]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < S0p / 2; ++k) {
      const double c0 = F[2 * k] * u0 + F[S0 + 2 * k] * u1;
      const double c1 = 2 * k + 1 < S0 ? F[2 * k + 1] * u0 + F[S0 + 2 * k + 1] * u1 : 0.0;
      reinterpret_cast<double2*>(im + kRec * lane)[k] = make_double2(c0, c1);
    }
    __builtin_amdgcn_wave_barrier();
    typedef double v2d __attribute__((ext_vector_type(2)));
    v2d* dst = reinterpret_cast<v2d*>(a.contrib + (int64_t)kRec * i0);
    const int pc = (kRec / 2) * nb;
#pragma unroll
    for (int k = 0; k < kRec / 2; ++k) {
      const int p = k * kWave + lane;
      if (p < pc) __builtin_nontemporal_store(reinterpret_cast<const v2d*>(im)[p], dst + p);
    }
  }
}

// One wave per e block with more rows than a wave: the rows are walked
// twice, once for the sums and once for the contributions.
template <int S0, int kMode, bool kGrad = false>
__global__ __launch_bounds__(kBlockThreads) void SchurBigKernel(const SchurArgs a) {
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const int64_t q = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  if (q >= a.nbig) return;
  const int64_t i0 = a.big[2 * q], i1 = a.big[2 * q + 1];
  const int id1 = (int)(reinterpret_cast<const long long*>(a.ids)[i0] >> 32);
  double s[3] = {0.0, 0.0, 0.0}, A[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int64_t i = i0 + lane; i < i1; i += kWave) {
    const int id0 = (int)reinterpret_cast<const long long*>(a.ids)[i];
    double F[2 * S0], E[6], z[2], sb[3], Ab[6];
    SchurLoadBlock<S0, kMode>(a, i, id0, F, E, z);
    SchurEProducts(E, z, sb, Ab);
#pragma unroll
    for (int k = 0; k < 3; ++k) s[k] += sb[k];
    if constexpr (kMode == kSchurInit) {
#pragma unroll
      for (int k = 0; k < 6; ++k) A[k] += Ab[k];
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
    for (int k = 0; k < 3; ++k) s[k] += __shfl_xor(s[k], off, kWave);
    if constexpr (kMode == kSchurInit) {
#pragma unroll
      for (int k = 0; k < 6; ++k) A[k] += __shfl_xor(A[k], off, kWave);
    }
  }
  const int64_t ecol = a.e_col_base + 3LL * id1;
  if constexpr (kGrad) {
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) a.grad[ecol + k] = -s[k];
    }
  }
  double M[6];
  if constexpr (kMode == kSchurInit) {
    double d[3] = {0.0, 0.0, 0.0};
    if (a.D) {
#pragma unroll
      for (int k = 0; k < 3; ++k) d[k] = a.D[ecol + k];
    }
    const bool ok = InvertSpd3(A, d, M);
    if (lane == 0 && !ok) *a.status = 1;
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < 6; ++k) a.ete_inv[2 * ecol + k] = M[k];
    }
  } else {
#pragma unroll
    for (int k = 0; k < 6; ++k) M[k] = a.ete_inv[2 * ecol + k];
  }
  double w[3];
  SymMul3(M, s, w);
  if constexpr (kMode == kSchurBack) {
    if (lane == 0) {
      a.y[ecol] = w[0];
      a.y[ecol + 1] = w[1];
      a.y[ecol + 2] = w[2];
    }
  } else if constexpr (kMode == kSchurInit) {
    for (int64_t i = i0 + lane; i < i1; i += kWave) {
      const double* ep = a.jac + a.e_base + 6 * i;
      double E[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) E[k] = ep[k];
      const double2 v = *reinterpret_cast<const double2*>(a.b + a.b_base + 2 * i);
      const double z[2] = {v.x, v.y};
      SchurStoreU<kGrad>(a, i, E, z, w);
    }
  } else {
    for (int64_t i = i0 + lane; i < i1; i += kWave) {
      const int id0 = (int)reinterpret_cast<const long long*>(a.ids)[i];
      double F[2 * S0], E[6], z[2];
      SchurLoadBlock<S0, kMode>(a, i, id0, F, E, z);
      SchurContrib<S0>(a, i, F, E, z, w);
    }
  }
}

// y[k] = D[off + k]^2 x[k] (the D^2 x term of RightMultiplyAndAccumulate,
// assigned: the reference sets y before adding F^T y1), or 0 without D.
__global__ __launch_bounds__(kBlockThreads) void SchurDiagKernel(const double* D, int64_t off,
                                                                 const double* x, double* y,
                                                                 int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * kBlockThreads + threadIdx.x;
  if (k >= n) return;
  if (D) {
    const double d = D[off + k];
    y[k] = d * d * x[k];
  } else {
    y[k] = 0.0;
  }
}

// y += x.
__global__ __launch_bounds__(kBlockThreads) void AxpyKernel(const double* x, double* y, int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * kBlockThreads + threadIdx.x;
  if (k < n) y[k] += x[k];
}

// The init's camera-order pass, one wave per block list chunk (the camera
// plan of the gradient: chunks of at most kGradChunk rows of one f block,
// taken pass-major when `order` is given).  Over the chunk's rows k (two per
// residual block) it forms, for its f block,
//     F^T u          rhs = F^T (b - E M E^T b)
//     F^T b          (kGrad) the gradient's f rows, -F^T b
//     F^T Q F        (kDiag) the preconditioner's block, with
//   kDiag 1, JACOBI        Q_b = I: (F^T F + D_f^2)^-1, ImplicitSchurComplement's
//                 block_diagonal_FtF_inverse (implicit_schur_complement.cc:
//                 71-95, iterative_schur_complement_solver.cc:186-189);
//   kDiag 2, SCHUR_JACOBI  Q_b = I - E_b M_p E_b^T: the f-block diagonal of S
//                 (schur_jacobi_preconditioner.cc:89-98; exact when no e
//                 block sees one f block twice, which the host checks),
// as ONE matrix product on the matrix cores: C (16 x 16) += A^T B over the
// chunk's rows, A = [F rows] (9 of 16 columns), B = [rows of Q F | u | b]
// (columns 0-8, 9, 10): C[0:9, 0:9] = F^T Q F, C[0:9, 9] = F^T u,
// C[0:9, 10] = F^T b.  Per slab of 32 blocks, two lanes gather each block
// (half the F cell each; the second also u_b and b_b; for Q both read E_b
// and M_p and each writes one row of Q F) into the wave's LDS slab; 16
// v_mfma_f64_16x16x4_f64 then take the slab's 64 rows, four at a time
// (lane l supplies row 4s + l/16, column l % 16 of A and of B).  The
// accumulator is 4 doubles per lane instead of the 63 sums a lane-per-block
// form keeps (248 VGPRs, 2 waves per SIMD): 42 VGPRs and 7 waves per SIMD
// here (4 for SCHUR_JACOBI).  Fixed order: bit-identical run to run.  The chunk's
// sums go to partial[cid][kPart] (upper triangle, then F^T u, then F^T b).
// Each F cell is read once per init, here; the point-order pass read only
// the E cells.
template <int S0>
constexpr int SymCount() { return S0 * (S0 + 1) / 2; }

template <int S0, int kDiag, bool kGrad>
constexpr int SchurPartCount() { return (kDiag ? SymCount<S0>() : 0) + S0 + (kGrad ? S0 : 0); }

template <int S0, int kDiag, bool kGrad>
__global__ __launch_bounds__(kBlockThreads) void SchurCameraPassKernel(const SchurArgs a,
                                                                       const int32_t* perm,
                                                                       const GradChunks ch,
                                                                       const int32_t* order) {
  static_assert(S0 + 2 <= 16, "A^T B in one 16 x 16 f64 tile");
  constexpr int T = kDiag ? SymCount<S0>() : 0;
  constexpr int kPart = SchurPartCount<S0, kDiag, kGrad>();
  constexpr int kU = kGrad ? 4 : 2;
  constexpr int kG = kDiag == 2 ? S0 : 0;  // Q F columns after F
  constexpr int kW = S0 + kG + 2;          // doubles per LDS row: F | Q F | u | b
  constexpr int kSlab = kWave / 2;         // blocks per slab: two lanes per block
  constexpr int kRows = 2 * kSlab;         // rows per slab
  typedef double v4d __attribute__((ext_vector_type(4)));
  __shared__ double slab_all[kWavesPerBlock][kRows * kW];
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const int64_t slot = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  if (slot >= ch.nchunks) return;
  double* slab = slab_all[wave];
  const int64_t cid = order ? (int64_t)order[slot] : slot;
  const int64_t q0 = ch.begin[cid], q1 = ch.begin[cid + 1];
  const int col = lane & 15, rsub = lane >> 4;
  const int bl = lane & (kSlab - 1), h = lane / kSlab;  // block of the slab, half of its cell
  constexpr int kP0 = (S0 + 1) / 2;                      // 16-byte pieces of half 0
  v4d acc = {0.0, 0.0, 0.0, 0.0};
  for (int64_t qs = q0; qs < q1; qs += kSlab) {
    const int nb = (int)(q1 - qs < kSlab ? q1 - qs : kSlab);
    int64_t i = 0;
    if (bl < nb) {
      i = perm[qs + bl];
      // half 0: F doubles [0, 2 kP0); half 1: [2 kP0, 2 S0), u_b (and b_b).
      const double2* fp = reinterpret_cast<const double2*>(a.jac + a.f_base + 2 * S0 * i);
      double* r0 = slab + (2 * bl) * kW;
      if (h == 0) {
#pragma unroll
        for (int k = 0; k < kP0; ++k) {
          const double2 v = fp[k];
          const int d = 2 * k;
          r0[(d / S0) * kW + d % S0] = v.x;
          r0[((d + 1) / S0) * kW + (d + 1) % S0] = v.y;
        }
      } else {
#pragma unroll
        for (int k = kP0; k < S0; ++k) {
          const double2 v = fp[k];
          const int d = 2 * k;
          r0[(d / S0) * kW + d % S0] = v.x;
          r0[((d + 1) / S0) * kW + (d + 1) % S0] = v.y;
        }
        const double2* up = reinterpret_cast<const double2*>(a.ub + kU * i);
        const double2 u = up[0];
        r0[S0 + kG] = u.x;
        r0[kW + S0 + kG] = u.y;
        if constexpr (kGrad) {
          const double2 bb = up[1];
          r0[S0 + kG + 1] = bb.x;
          r0[kW + S0 + kG + 1] = bb.y;
        } else {
          r0[S0 + kG + 1] = 0.0;
          r0[kW + S0 + kG + 1] = 0.0;
        }
      }
    }
    if constexpr (kDiag == 2) {
      // Q F rows: half h writes row h of its block, from the F rows above.
      double q0v = 0.0, q1v = 0.0;
      if (bl < nb) {
        const int id1 = (int)(reinterpret_cast<const long long*>(a.ids)[i] >> 32);
        const double* m = a.ete_inv + 2 * (a.e_col_base + 3LL * id1);
        double M[6], E[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) M[k] = m[k];
        const double* ep = a.jac + a.e_base + 6 * i;
#pragma unroll
        for (int k = 0; k < 6; ++k) E[k] = ep[k];
        double me0[3], me1[3];
        SymMul3(M, E, me0);
        SymMul3(M, E + 3, me1);
        const double q00 = 1.0 - (E[0] * me0[0] + E[1] * me0[1] + E[2] * me0[2]);
        const double q01 = -(E[0] * me1[0] + E[1] * me1[1] + E[2] * me1[2]);
        const double q11 = 1.0 - (E[3] * me1[0] + E[4] * me1[1] + E[5] * me1[2]);
        q0v = h == 0 ? q00 : q01;
        q1v = h == 0 ? q01 : q11;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      if (bl < nb) {
        const double* f0 = slab + (2 * bl) * kW;
        double* g = slab + (2 * bl + h) * kW + S0;
#pragma unroll
        for (int k = 0; k < S0; ++k) g[k] = q0v * f0[k] + q1v * f0[kW + k];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    // A[m][k] = row k, column m (F); B[k][n] = row k, column n of [Q F | u | b]
    // (columns 0-8 of B are F's own for JACOBI; none for IDENTITY).
    const int bcol = col < S0 ? (kDiag == 0 ? -1 : kDiag == 2 ? S0 + col : col)
                              : col == S0 ? S0 + kG : (kGrad && col == S0 + 1) ? S0 + kG + 1 : -1;
    const int rows = 2 * nb;
#pragma unroll 4
    for (int s = 0; s < kRows / 4; ++s) {
      const int row = 4 * s + rsub;
      if (4 * s >= rows) break;
      const bool live = row < rows;
      const double av = live && col < S0 ? slab[row * kW + col] : 0.0;
      const double bv = live && bcol >= 0 ? slab[row * kW + bcol] : 0.0;
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
  // C[m][n]: m = lane / 16 + 4 r, n = lane % 16.
  double* out = ch.partial + cid * kPart;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = rsub + 4 * r, n = col;
    if (m >= S0) continue;
    if constexpr (kDiag != 0) {
      if (n < S0 && m <= n) out[m * S0 - m * (m - 1) / 2 + (n - m)] = acc[r];
    }
    if (n == S0) out[T + m] = acc[r];
    if constexpr (kGrad) {
      if (n == S0 + 1) out[T + S0 + m] = acc[r];
    }
  }
}

// Per f block p (thread p): its chunk partials summed in order; rhs rows
// (rhs_p, S0 of them, assigned) and, kGrad, the gradient rows (grad_p,
// -F^T b); kDiag: D^2 on the diagonal and the inverse by the Cholesky
// factor (llt().solve(Identity), as the reference's
// BlockRandomAccessDiagonalMatrix::Invert and AddDiagonalAndInvert) stored
// as a full S0 x S0 matrix.
template <int S0, int kDiag, bool kGrad>
__global__ __launch_bounds__(64) void SchurCameraFinishKernel(const GradChunks ch, int64_t count,
                                                              const double* D, int64_t d_off,
                                                              double* P, int* status, double* rhs,
                                                              double* grad) {
  constexpr int T = kDiag ? SymCount<S0>() : 0;
  constexpr int kPart = SchurPartCount<S0, kDiag, kGrad>();
  const int64_t p = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (p >= count) return;
  {
    double ru[S0], rb[S0];
#pragma unroll
    for (int k = 0; k < S0; ++k) ru[k] = rb[k] = 0.0;
    for (int64_t q = ch.chunk_off[p]; q < ch.chunk_off[p + 1]; ++q) {
      const double* part = ch.partial + q * kPart + T;
#pragma unroll
      for (int k = 0; k < S0; ++k) ru[k] += part[k];
      if constexpr (kGrad) {
#pragma unroll
        for (int k = 0; k < S0; ++k) rb[k] += part[S0 + k];
      }
    }
#pragma unroll
    for (int k = 0; k < S0; ++k) rhs[(int64_t)S0 * p + k] = ru[k];
    if constexpr (kGrad) {
#pragma unroll
      for (int k = 0; k < S0; ++k) grad[(int64_t)S0 * p + k] = -rb[k];
    }
  }
  if constexpr (kDiag != 0) {
    double L[S0][S0];
    {
      double acc[T];
#pragma unroll
      for (int t = 0; t < T; ++t) acc[t] = 0.0;
      for (int64_t q = ch.chunk_off[p]; q < ch.chunk_off[p + 1]; ++q)
#pragma unroll
        for (int t = 0; t < T; ++t) acc[t] += ch.partial[q * kPart + t];
      int t = 0;
#pragma unroll
      for (int r = 0; r < S0; ++r)
#pragma unroll
        for (int cc = r; cc < S0; ++cc) L[cc][r] = acc[t++];  // lower triangle of A
    }
    if (D) {
#pragma unroll
      for (int r = 0; r < S0; ++r) {
        const double d = D[d_off + (int64_t)S0 * p + r];
        L[r][r] += d * d;
      }
    }
    // In-place Cholesky: A = L L^T.  A pivot that is not positive (a camera
    // with no observation and D = NULL) raises the status word and leaves
    // the block's inverse zero.
    bool ok = true;
#pragma unroll
    for (int j = 0; j < S0; ++j) {
      double djj = L[j][j];
#pragma unroll
      for (int k = 0; k < j; ++k) djj -= L[j][k] * L[j][k];
      ok = ok && PivotOk(djj);
      const double ljj = sqrt(djj);
      const double inv = 1.0 / ljj;
      L[j][j] = ljj;
#pragma unroll
      for (int r = j + 1; r < S0; ++r) {
        double v = L[r][j];
#pragma unroll
        for (int k = 0; k < j; ++k) v -= L[r][k] * L[j][k];
        L[r][j] = v * inv;
      }
    }
    double* out = P + (int64_t)S0 * S0 * p;
    if (!ok) {
      *status = 1;
      for (int k = 0; k < S0 * S0; ++k) out[k] = 0.0;
      return;
    }
    // Columns of the inverse: L y = e_c, then L^T x = y.
#pragma unroll
    for (int cc = 0; cc < S0; ++cc) {
      double y[S0];
#pragma unroll
      for (int r = 0; r < S0; ++r) {
        double v = r == cc ? 1.0 : 0.0;
#pragma unroll
        for (int k = 0; k < r; ++k) v -= L[r][k] * y[k];
        y[r] = v / L[r][r];
      }
#pragma unroll
      for (int r = S0 - 1; r >= 0; --r) {
        double v = y[r];
#pragma unroll
        for (int k = r + 1; k < S0; ++k) v -= L[k][r] * y[k];
        y[r] = v / L[r][r];
      }
#pragma unroll
      for (int r = 0; r < S0; ++r) out[r * S0 + cc] = y[r];
    }
  }
}

// y += P x per f block (the preconditioner's RightMultiplyAndAccumulate),
// one thread per f-vector entry.
template <int S0>
__global__ __launch_bounds__(kBlockThreads) void SchurPrecondApplyKernel(const double* P,
                                                                         const double* x,
                                                                         double* y, int64_t n) {
  const int64_t k = (int64_t)blockIdx.x * kBlockThreads + threadIdx.x;
  if (k >= n) return;
  const int64_t p = k / S0;
  const int r = (int)(k - p * S0);
  const double* row = P + (int64_t)S0 * S0 * p + (int64_t)S0 * r;
  const double* xp = x + (int64_t)S0 * p;
  double v = 0.0;
#pragma unroll
  for (int cc = 0; cc < S0; ++cc) v += row[cc] * xp[cc];
  y[k] += v;
}

}  // namespace cse

#endif  // CSE_SCHUR_KERNELS_HPP_
