// membench2.hip -- store-flavour and staging-shape microbenchmarks for the
// evaluate kernel's output path on MI355X (diagnostic tool, not part of
// the product).  Shapes as tools/membench.hip (problem-13682).
//
//   wseq <flavour>   pure 16 B/lane streaming stores of the 6.03 GB output
//                    flavours: plain, nt, sc1, sc0sc1, ntsc1
//   dma80 +stage1    the shipped kernel's memory path: LDS-DMA camera gather
//                    from an 80-byte table, per-lane point/obs loads, one LDS
//                    round (E+F, 24 doubles per lane), residuals direct
//   dma80 +half      the same with half-wave staging rounds (12 KB -> 6 KB
//                    of LDS per wave)
//   dma80 +segs      no staging (coalesced stores of fake values): floor
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

constexpr int kO = 28987644, kC = 13682, kP = 4456117;
constexpr int kWave = 64;

typedef int v4i __attribute__((ext_vector_type(4)));

enum { kPlain = 0, kNt = 1, kSc1 = 2, kSc0Sc1 = 3, kNtSc1 = 4 };

template <int kF>
__device__ __forceinline__ void st16(double* p, double a, double b) {
  if constexpr (kF == kPlain) {
    *reinterpret_cast<double2*>(p) = make_double2(a, b);
  } else if constexpr (kF == kNt) {
    __builtin_nontemporal_store(a, p);
    __builtin_nontemporal_store(b, p + 1);
  } else {
    double2 v = make_double2(a, b);
    v4i d;
    __builtin_memcpy(&d, &v, 16);
    if constexpr (kF == kSc1)
      asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(d) : "memory");
    else if constexpr (kF == kSc0Sc1)
      asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(d) : "memory");
    else
      asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(d) : "memory");
  }
}

// The evaluator's 13 per-chunk stores as one asm block: no instruction the
// compiler schedules can overwrite a queued store's address or data VGPRs
// between them.  r: residual pair, e[3], f[9]: 16-byte pieces.
__device__ __forceinline__ v4i as4(double a, double b) {
  double2 v = make_double2(a, b);
  v4i d;
  __builtin_memcpy(&d, &v, 16);
  return d;
}
__device__ __forceinline__ void store13_nt(double* pr, double* pe, double* pf, const v4i& r,
                                           const v4i* e, const v4i* f) {
  double* pf2 = pf + 512;   // +4096 B: F pieces 0..7 at offsets -4096 .. 3072
  double* pf3 = pf + 1024;  // F piece 8
  asm volatile(
      "global_store_dwordx4 %0, %3, off nt\n"
      "global_store_dwordx4 %1, %4, off nt\n"
      "global_store_dwordx4 %1, %5, off offset:1024 nt\n"
      "global_store_dwordx4 %1, %6, off offset:2048 nt\n"
      "global_store_dwordx4 %2, %7, off offset:-4096 nt\n"
      "global_store_dwordx4 %2, %8, off offset:-3072 nt\n"
      "global_store_dwordx4 %2, %9, off offset:-2048 nt\n"
      "global_store_dwordx4 %2, %10, off offset:-1024 nt\n"
      "global_store_dwordx4 %2, %11, off nt\n"
      "global_store_dwordx4 %2, %12, off offset:1024 nt\n"
      "global_store_dwordx4 %2, %13, off offset:2048 nt\n"
      "global_store_dwordx4 %2, %14, off offset:3072 nt\n"
      "global_store_dwordx4 %16, %15, off nt\n" ::"v"(pr),
      "v"(pe), "v"(pf2), "v"(r), "v"(e[0]), "v"(e[1]), "v"(e[2]), "v"(f[0]), "v"(f[1]), "v"(f[2]),
      "v"(f[3]), "v"(f[4]), "v"(f[5]), "v"(f[6]), "v"(f[7]), "v"(f[8]), "v"(pf3)
      : "memory");
}

// Same as store13_nt with non-negative immediate offsets only (4 F bases).
__device__ __forceinline__ void store13_nt_pos(double* pr, double* pe, double* pf, const v4i& r,
                                               const v4i* e, const v4i* f) {
  double* pf1 = pf + 512;
  double* pf2 = pf + 1024;
  asm volatile(
      "global_store_dwordx4 %0, %3, off nt\n"
      "global_store_dwordx4 %1, %4, off nt\n"
      "global_store_dwordx4 %1, %5, off offset:1024 nt\n"
      "global_store_dwordx4 %1, %6, off offset:2048 nt\n"
      "global_store_dwordx4 %2, %7, off nt\n"
      "global_store_dwordx4 %2, %8, off offset:1024 nt\n"
      "global_store_dwordx4 %2, %9, off offset:2048 nt\n"
      "global_store_dwordx4 %2, %10, off offset:3072 nt\n"
      "global_store_dwordx4 %16, %11, off nt\n"
      "global_store_dwordx4 %16, %12, off offset:1024 nt\n"
      "global_store_dwordx4 %16, %13, off offset:2048 nt\n"
      "global_store_dwordx4 %16, %14, off offset:3072 nt\n"
      "global_store_dwordx4 %17, %15, off nt\n" ::"v"(pr),
      "v"(pe), "v"(pf), "v"(r), "v"(e[0]), "v"(e[1]), "v"(e[2]), "v"(f[0]), "v"(f[1]), "v"(f[2]),
      "v"(f[3]), "v"(f[4]), "v"(f[5]), "v"(f[6]), "v"(f[7]), "v"(f[8]), "v"(pf1), "v"(pf2)
      : "memory");
}

template <int kF>
__global__ __launch_bounds__(256) void write_seq(double* out, long n2) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < n2; t += stride)
    st16<kF>(out + 2 * t, (double)t, 1.0);
}

// Pure write stream with a chosen data pattern: 0 zeros, 1 one repeated
// value, 2 (index, 1.0), 3 pseudo-random 64-bit words, 4 random doubles
// with realistic exponents (|x| in [2^-8, 2^8)).
template <int kData>
__global__ __launch_bounds__(256) void write_data(double* out, long n2) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < n2; t += stride) {
    double a, b;
    if constexpr (kData == 0) {
      a = b = 0.0;
    } else if constexpr (kData == 1) {
      a = b = 1.5;
    } else if constexpr (kData == 2) {
      a = (double)t;
      b = 1.0;
    } else {
      unsigned long h0 = (unsigned long)t * 0x9E3779B97F4A7C15UL;
      h0 ^= h0 >> 29;
      unsigned long h1 = h0 * 0xBF58476D1CE4E5B9UL;
      h1 ^= h1 >> 32;
      if constexpr (kData == 4) {
        // sign random, exponent 1015..1030, mantissa random
        h0 = (h0 & 0x800FFFFFFFFFFFFFUL) | ((1015UL + ((h0 >> 52) & 15)) << 52);
        h1 = (h1 & 0x800FFFFFFFFFFFFFUL) | ((1015UL + ((h1 >> 52) & 15)) << 52);
      }
      a = __longlong_as_double((long)h0);
      b = __longlong_as_double((long)h1);
    }
    __builtin_nontemporal_store(a, out + 2 * t);
    __builtin_nontemporal_store(b, out + 2 * t + 1);
  }
}

__global__ __launch_bounds__(256) void read_stream(const double2* in, long n2, double* sink) {
  const long stride = (long)gridDim.x * blockDim.x;
  double s = 0.0;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < n2; t += stride) {
    const double2 v = in[t];
    s += v.x + v.y;
  }
  if (s == 12345.678) sink[0] = s;
}

// kMode 0: coalesced fake stores (no staging); 1: one LDS round E+F;
// 2: half-wave rounds.  kReg: camera pieces through VGPRs + ds_write
// instead of LDS-DMA.
template <int kMode, int kF, bool kReg = false>
__global__ __launch_bounds__(256) void dma80(const int2* ids, const double2* obs,
                                             const double* pts, const double* cam80, double* res,
                                             double* E, double* F, long n) {
  constexpr int kLane = kMode == 2 ? 12 : (kMode == 1 || kMode == 3) ? 24 : 10;
  __shared__ double lds[4][kWave * kLane];
  const int lane = threadIdx.x & 63, wave = threadIdx.x / 64;
  const long c = (long)blockIdx.x * 4 + wave;
  const long chunks = (n + 63) / 64;
  if (c >= chunks) return;
  double* st = lds[wave];
  long i = c * 64 + lane;
  if (i >= n) i = n - 1;
  const int2 id = ids[i];
  // Camera: 5 x 16-B pieces per camera by LDS-DMA.
  const double2 o = obs[i];
  const double* pt = pts + 3L * id.y;
  double x[3];
  if constexpr (kReg) {
    double2 pc[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int p = k * 64 + lane;
      const int t = p / 5, q = p - t * 5;
      const int cid = __shfl(id.x, t, 64);
      pc[k] = *reinterpret_cast<const double2*>(cam80 + 10L * cid + 2 * q);
    }
    x[0] = pt[0], x[1] = pt[1], x[2] = pt[2];
#pragma unroll
    for (int k = 0; k < 5; ++k) reinterpret_cast<double2*>(st)[k * 64 + lane] = pc[k];
  } else {
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int p = k * 64 + lane;
      const int t = p / 5, q = p - t * 5;
      const int cid = __shfl(id.x, t, 64);
      __builtin_amdgcn_global_load_lds(cam80 + 10L * cid + 2 * q, st + 128 * k, 16, 0, 0);
    }
    x[0] = pt[0], x[1] = pt[1], x[2] = pt[2];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_wave_barrier();
  double cam[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) cam[k] = st[lane * 10 + k];
  __builtin_amdgcn_wave_barrier();
  double v = o.x + o.y + x[0] + x[1] + x[2];
#pragma unroll
  for (int k = 0; k < 9; ++k) v += cam[k];
  // Outputs: residuals direct.
  st16<kF>(res + 128 * c + 2 * lane, v, v);
  double J[24];
#pragma unroll
  for (int q = 0; q < 24; ++q) J[q] = v * (q + 1);
  if constexpr (kMode == 0) {
#pragma unroll
    for (int k = 0; k < 3; ++k) st16<kF>(E + 384 * c + 128 * k + 2 * lane, J[2 * k], J[2 * k + 1]);
#pragma unroll
    for (int k = 0; k < 9; ++k)
      st16<kF>(F + 1152 * c + 128 * k + 2 * lane, J[6 + 2 * k], J[7 + 2 * k]);
  } else if constexpr (kMode == 1) {
    double* stE = st;
    double* stF = st + 64 * 6;
#pragma unroll
    for (int q = 0; q < 6; q += 2)
      *reinterpret_cast<double2*>(stE + lane * 6 + q) = make_double2(J[q], J[q + 1]);
#pragma unroll
    for (int q = 0; q < 18; q += 2)
      *reinterpret_cast<double2*>(stF + lane * 18 + q) = make_double2(J[6 + q], J[7 + q]);
    __builtin_amdgcn_wave_barrier();
    double2 e[3], f[9];
#pragma unroll
    for (int k = 0; k < 3; ++k) e[k] = reinterpret_cast<const double2*>(stE)[k * 64 + lane];
#pragma unroll
    for (int k = 0; k < 9; ++k) f[k] = reinterpret_cast<const double2*>(stF)[k * 64 + lane];
#pragma unroll
    for (int k = 0; k < 3; ++k) st16<kF>(E + 384 * c + 128 * k + 2 * lane, e[k].x, e[k].y);
#pragma unroll
    for (int k = 0; k < 9; ++k) st16<kF>(F + 1152 * c + 128 * k + 2 * lane, f[k].x, f[k].y);
    __builtin_amdgcn_wave_barrier();
  } else if constexpr (kMode == 3) {
    double* stE = st;
    double* stF = st + 64 * 6;
#pragma unroll
    for (int q = 0; q < 6; q += 2)
      *reinterpret_cast<double2*>(stE + lane * 6 + q) = make_double2(J[q], J[q + 1]);
#pragma unroll
    for (int q = 0; q < 18; q += 2)
      *reinterpret_cast<double2*>(stF + lane * 18 + q) = make_double2(J[6 + q], J[7 + q]);
    __builtin_amdgcn_wave_barrier();
    double2 e[3], f[9];
#pragma unroll
    for (int k = 0; k < 3; ++k) e[k] = reinterpret_cast<const double2*>(stE)[k * 64 + lane];
#pragma unroll
    for (int k = 0; k < 9; ++k) f[k] = reinterpret_cast<const double2*>(stF)[k * 64 + lane];
    double* pe = E + 384 * c + 2 * lane;
    double* pf = F + 1152 * c + 2 * lane;
#pragma unroll
    for (int k = 0; k < 3; ++k) st16<kF>(pe + 128 * k, e[k].x, e[k].y);
#pragma unroll
    for (int k = 0; k < 9; ++k) st16<kF>(pf + 128 * k, f[k].x, f[k].y);
#pragma unroll
    for (int k = 0; k < 3; ++k) asm volatile("" ::"v"(e[k].x), "v"(e[k].y));
#pragma unroll
    for (int k = 0; k < 9; ++k) asm volatile("" ::"v"(f[k].x), "v"(f[k].y));
    asm volatile("" ::"v"(pe), "v"(pf), "v"(v));
  } else {
    // Two rounds of 32 lanes: each round's E (32*6) and F (32*18) regions
    // are contiguous halves of the wave's segments.
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      double* stE = st;
      double* stF = st + 32 * 6;
      if ((lane >> 5) == h) {
        const int l = lane & 31;
#pragma unroll
        for (int q = 0; q < 6; q += 2)
          *reinterpret_cast<double2*>(stE + l * 6 + q) = make_double2(J[q], J[q + 1]);
#pragma unroll
        for (int q = 0; q < 18; q += 2)
          *reinterpret_cast<double2*>(stF + l * 18 + q) = make_double2(J[6 + q], J[7 + q]);
      }
      __builtin_amdgcn_wave_barrier();
      // E half: 96 pairs -> 1.5 instructions; F half: 288 pairs -> 4.5.
      double2 e[2], f[5];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int t = k * 64 + lane;
        if (t < 96) e[k] = reinterpret_cast<const double2*>(stE)[t];
      }
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const int t = k * 64 + lane;
        if (t < 288) f[k] = reinterpret_cast<const double2*>(stF)[t];
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int t = k * 64 + lane;
        if (t < 96) st16<kF>(E + 384 * c + 192 * h + 2 * t, e[k].x, e[k].y);
      }
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const int t = k * 64 + lane;
        if (t < 288) st16<kF>(F + 1152 * c + 576 * h + 2 * t, f[k].x, f[k].y);
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// tools/membench.hip's coop_gather<true, 1> (grid-stride loop, values
// folded into one register pair), for a same-process comparison.
template <int kVariant>
__global__ __launch_bounds__(256) void m1(const int2* ids, const double2* obs, const double* pts,
                                          const double* cams, double* res, double* E, double* F,
                                          double* sink, long chunks, long n) {
  __shared__ double lds[4][64 * 10];
  const int lane = threadIdx.x & 63, wave = threadIdx.x / 64;
  const long stride = (long)gridDim.x * 4;
  double acc = 0.0;
  for (long c = (long)blockIdx.x * 4 + wave; c < chunks; c += stride) {
    long i = c * 64 + lane;
    if (i >= n) i = n - 1;
    const int2 id = ids[i];
    const double2 o = obs[i];
    const double* pt = pts + 3L * id.y;
    double v = o.x + o.y + pt[0] + pt[1] + pt[2];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int p = k * 64 + lane;
      const int t = p / 5, q = p % 5;
      const int cid = __shfl(id.x, t, 64);
      const double2 w = *reinterpret_cast<const double2*>(cams + 10L * cid + 2 * q);
      *reinterpret_cast<double2*>(lds[wave] + t * 10 + 2 * q) = w;
    }
    __builtin_amdgcn_wave_barrier();
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 9; ++k) s += lds[wave][lane * 10 + k];
    __builtin_amdgcn_wave_barrier();
    v += s;
    if constexpr (kVariant == 20) v += lane * 1e-3;                 // lane-distinct
    if constexpr (kVariant == 21) v += (double)c * 1e-3;            // chunk-distinct
    if constexpr (kVariant == 22) v += __longlong_as_double(0x3FF0000000000000L | ((unsigned long)(i * 0x9E3779B97F4A7C15L) >> 12)) ;  // random mantissa
    if constexpr (kVariant == 30) {
      if (lane == 0) sink[1 + c] = v;  // per-wave 8-byte partial store
    }
    if constexpr (kVariant == 31) {  // one full 64-byte line per wave
      if (lane < 4) st16<kPlain>(sink + 8 * c + 2 * lane, lane == 0 ? v : 0.0, 0.0);
    }
    if constexpr (kVariant == 32) {  // one full 128-byte line per wave
      if (lane < 8) st16<kPlain>(sink + 16 * c + 2 * lane, lane == 0 ? v : 0.0, 0.0);
    }
    if constexpr (kVariant == 33) {  // 8-byte non-temporal
      if (lane == 0) __builtin_nontemporal_store(v, sink + 1 + c);
    }
    if constexpr (kVariant == 36) {  // partial stored BEFORE the big stores
      if (lane == 0) sink[1 + c] = v;
      asm volatile("" ::: "memory");
    }
    if constexpr (kVariant == 34) {  // 64-byte line, non-temporal
      if (lane < 4) st16<kNt>(sink + 8 * c + 2 * lane, lane == 0 ? v : 0.0, 0.0);
    }
    if constexpr (kVariant == 0 || kVariant >= 20) {  // (30+: same stores as 0)
      st16<kNt>(res + 128 * c + 2 * lane, v, v);
#pragma unroll
      for (int k = 0; k < 3; ++k) st16<kNt>(E + 384 * c + 128 * k + 2 * lane, v, v);
#pragma unroll
      for (int k = 0; k < 9; ++k) st16<kNt>(F + 1152 * c + 128 * k + 2 * lane, v, v);
    } else if constexpr (kVariant == 2) {
      // distinct values, all computed first, stores pinned in address order
      double J[24];
#pragma unroll
      for (int q = 0; q < 24; ++q) J[q] = v * (q + 1);
      asm volatile("" ::: "memory");
      st16<kNt>(res + 128 * c + 2 * lane, v, v);
      asm volatile("" ::: "memory");
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        st16<kNt>(E + 384 * c + 128 * k + 2 * lane, J[2 * k], J[2 * k + 1]);
        asm volatile("" ::: "memory");
      }
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        st16<kNt>(F + 1152 * c + 128 * k + 2 * lane, J[6 + 2 * k], J[7 + 2 * k]);
        asm volatile("" ::: "memory");
      }
    } else if constexpr (kVariant == 3) {
      // same value, scrambled order
      const int ord[9] = {1, 2, 0, 4, 3, 6, 5, 8, 7};
      st16<kNt>(res + 128 * c + 2 * lane, v, v);
      asm volatile("" ::: "memory");
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        st16<kNt>(E + 384 * c + 128 * ord[k] + 2 * lane, v, v);
        asm volatile("" ::: "memory");
      }
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        st16<kNt>(F + 1152 * c + 128 * ord[k] + 2 * lane, v, v);
        asm volatile("" ::: "memory");
      }
    } else if constexpr (kVariant == 5) {
      // distinct registers, integer-produced (bit patterns), no FP64
      st16<kNt>(res + 128 * c + 2 * lane, v, v);
      const long vb = __double_as_longlong(v);
#pragma unroll
      for (int k = 0; k < 3; ++k)
        st16<kNt>(E + 384 * c + 128 * k + 2 * lane, __longlong_as_double(vb | (2 * k + 1)),
                  __longlong_as_double(vb | (2 * k + 2)));
#pragma unroll
      for (int k = 0; k < 9; ++k)
        st16<kNt>(F + 1152 * c + 128 * k + 2 * lane, __longlong_as_double(vb | (2 * k + 7)),
                  __longlong_as_double(vb | (2 * k + 8)));
    } else if constexpr (kVariant == 6) {
      // distinct registers holding the SAME value (copies)
      double J[24];
#pragma unroll
      for (int q = 0; q < 24; ++q) J[q] = __builtin_amdgcn_readfirstlane(q) + v - __builtin_amdgcn_readfirstlane(q);
      st16<kNt>(res + 128 * c + 2 * lane, v, v);
#pragma unroll
      for (int k = 0; k < 3; ++k) st16<kNt>(E + 384 * c + 128 * k + 2 * lane, J[2 * k], J[2 * k + 1]);
#pragma unroll
      for (int k = 0; k < 9; ++k)
        st16<kNt>(F + 1152 * c + 128 * k + 2 * lane, J[6 + 2 * k], J[7 + 2 * k]);
    } else if constexpr (kVariant == 7) {
      // same register for all stores, but nonzero data (v + 1.5)
      const double u = v + 1.5;
      st16<kNt>(res + 128 * c + 2 * lane, u, u);
#pragma unroll
      for (int k = 0; k < 3; ++k) st16<kNt>(E + 384 * c + 128 * k + 2 * lane, u, u);
#pragma unroll
      for (int k = 0; k < 9; ++k) st16<kNt>(F + 1152 * c + 128 * k + 2 * lane, u, u);
    } else if constexpr (kVariant == 8) {
      // random-looking nonzero data, integer produced
      const long vb = __double_as_longlong(v) ^ (i * 0x9E3779B97F4A7C15L);
#pragma unroll
      for (int k = 0; k < 13; ++k) {
        const long x0 = vb * (2 * k + 1) ^ 0x3FF0000000000000L, x1 = vb * (2 * k + 3);
        double* dst = k == 0 ? res + 128 * c : k < 4 ? E + 384 * c + 128 * (k - 1) : F + 1152 * c + 128 * (k - 4);
        st16<kNt>(dst + 2 * lane, __longlong_as_double(x0), __longlong_as_double(x1));
      }
    } else if constexpr (kVariant == 9 || kVariant == 10 || kVariant == 11) {
      // same-register stores (fast path) plus independent work whose result
      // is not stored: 9 = 192 FP64 FMAs, 10 = 192 integer ops, 11 = 48 FMAs
      constexpr int kOps = kVariant == 11 ? 48 : 192;
      if constexpr (kVariant == 10) {
        unsigned x = (unsigned)lane, y = (unsigned)c;
#pragma unroll
        for (int k = 0; k < kOps; ++k) { x = (x ^ y) + 0x9E3779B9u; y = (y << 3) ^ x; }
        acc += (double)(x ^ y);
      } else {
        double x = v + lane, y = v * 0.5;
#pragma unroll
        for (int k = 0; k < kOps; k += 2) { x = __builtin_fma(x, 0.999, y); y = __builtin_fma(y, 0.998, x); }
        acc += x + y;
      }
      st16<kNt>(res + 128 * c + 2 * lane, v, v);
#pragma unroll
      for (int k = 0; k < 3; ++k) st16<kNt>(E + 384 * c + 128 * k + 2 * lane, v, v);
#pragma unroll
      for (int k = 0; k < 9; ++k) st16<kNt>(F + 1152 * c + 128 * k + 2 * lane, v, v);
    } else if constexpr (kVariant == 12) {
      // distinct registers by integer moves of the same value
      double J[24];
#pragma unroll
      for (int q = 0; q < 24; ++q) asm volatile("v_mov_b64 %0, %1" : "=v"(J[q]) : "v"(v));
      st16<kNt>(res + 128 * c + 2 * lane, v, v);
#pragma unroll
      for (int k = 0; k < 3; ++k) st16<kNt>(E + 384 * c + 128 * k + 2 * lane, J[2 * k], J[2 * k + 1]);
#pragma unroll
      for (int k = 0; k < 9; ++k)
        st16<kNt>(F + 1152 * c + 128 * k + 2 * lane, J[6 + 2 * k], J[7 + 2 * k]);
    } else if constexpr (kVariant == 13 || kVariant == 14) {
      // rotation among 2 (13) or 4 (14) register quads holding v
      constexpr int kQ = kVariant == 13 ? 2 : 4;
      double J[2 * kQ];
#pragma unroll
      for (int q = 0; q < 2 * kQ; ++q) asm volatile("v_mov_b64 %0, %1" : "=v"(J[q]) : "v"(v));
      st16<kNt>(res + 128 * c + 2 * lane, v, v);
#pragma unroll
      for (int k = 0; k < 3; ++k)
        st16<kNt>(E + 384 * c + 128 * k + 2 * lane, J[2 * (k % kQ)], J[2 * (k % kQ) + 1]);
#pragma unroll
      for (int k = 0; k < 9; ++k)
        st16<kNt>(F + 1152 * c + 128 * k + 2 * lane, J[2 * ((k + 3) % kQ)], J[2 * ((k + 3) % kQ) + 1]);
    } else if constexpr (kVariant == 15) {
      // distinct values, then every data register kept live past the
      // stores (no VALU may overwrite a queued store's VGPRs)
      double J[24];
#pragma unroll
      for (int q = 0; q < 24; ++q) J[q] = v * (q + 1);
      double* pr = res + 128 * c + 2 * lane;
      double* pe = E + 384 * c + 2 * lane;
      double* pf = F + 1152 * c + 2 * lane;
      st16<kNt>(pr, v, v);
#pragma unroll
      for (int k = 0; k < 3; ++k) st16<kNt>(pe + 128 * k, J[2 * k], J[2 * k + 1]);
#pragma unroll
      for (int k = 0; k < 9; ++k) st16<kNt>(pf + 128 * k, J[6 + 2 * k], J[7 + 2 * k]);
#pragma unroll
      for (int q = 0; q < 24; ++q) asm volatile("" ::"v"(J[q]));
      asm volatile("" ::"v"(pr), "v"(pe), "v"(pf), "v"(v));
    } else if constexpr (kVariant == 16) {
      // distinct values, stores as one asm block at the end
      v4i e[3], f[9];
#pragma unroll
      for (int k = 0; k < 3; ++k) e[k] = as4(v * (2 * k + 1), v * (2 * k + 2));
#pragma unroll
      for (int k = 0; k < 9; ++k) f[k] = as4(v * (2 * k + 7), v * (2 * k + 8));
      store13_nt(res + 128 * c + 2 * lane, E + 384 * c + 2 * lane, F + 1152 * c + 2 * lane,
                 as4(v, v), e, f);
    } else if constexpr (kVariant == 4) {
      // same value, 200 cycles of FP64 work spread between the stores
      double w = v;
      st16<kNt>(res + 128 * c + 2 * lane, v, v);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        w = w * 0.5 + v;
        st16<kNt>(E + 384 * c + 128 * k + 2 * lane, w, w);
      }
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        w = w * 0.5 + v;
        st16<kNt>(F + 1152 * c + 128 * k + 2 * lane, w, w);
      }
    } else {
      // distinct values per store
      st16<kNt>(res + 128 * c + 2 * lane, v, v);
#pragma unroll
      for (int k = 0; k < 3; ++k)
        st16<kNt>(E + 384 * c + 128 * k + 2 * lane, v * (2 * k + 1), v * (2 * k + 2));
#pragma unroll
      for (int k = 0; k < 9; ++k)
        st16<kNt>(F + 1152 * c + 128 * k + 2 * lane, v * (2 * k + 7), v * (2 * k + 8));
    }
  }
  if (acc == 12345.678) sink[0] = acc;
}

// Pure writes of the evaluator's 13 per-chunk stores (no loads): one data
// quad (kDistinct = false) or 13 distinct quads of the same value.
template <bool kDistinct>
__global__ __launch_bounds__(256) void wsegs(double* res, double* E, double* F, long chunks) {
  const int lane = threadIdx.x & 63;
  const long c = (long)blockIdx.x * 4 + threadIdx.x / 64;
  if (c >= chunks) return;
  const double v = (double)(c & 1);
  if constexpr (kDistinct) {
    double J[24];
#pragma unroll
    for (int q = 0; q < 24; ++q) asm volatile("v_mov_b64 %0, %1" : "=v"(J[q]) : "v"(v));
    st16<kNt>(res + 128 * c + 2 * lane, v, v);
#pragma unroll
    for (int k = 0; k < 3; ++k) st16<kNt>(E + 384 * c + 128 * k + 2 * lane, J[2 * k], J[2 * k + 1]);
#pragma unroll
    for (int k = 0; k < 9; ++k)
      st16<kNt>(F + 1152 * c + 128 * k + 2 * lane, J[6 + 2 * k], J[7 + 2 * k]);
  } else {
    st16<kNt>(res + 128 * c + 2 * lane, v, v);
#pragma unroll
    for (int k = 0; k < 3; ++k) st16<kNt>(E + 384 * c + 128 * k + 2 * lane, v, v);
#pragma unroll
    for (int k = 0; k < 9; ++k) st16<kNt>(F + 1152 * c + 128 * k + 2 * lane, v, v);
  }
}

// m1 without the grid-stride loop, and an explicit per-wave partial:
// kP 0 none, 1 lane-0 store after the big stores, 2 lane-0 store before,
// 3 all 64 lanes store 8 B (wave-wide, v / 64 each) after, 4 the partial in
// LDS only (no store).  All operands kept live to the end.
template <int kP>
__global__ __launch_bounds__(256) void m2(const int2* ids, const double2* obs, const double* pts,
                                          const double* cams, double* res, double* E, double* F,
                                          double* sink, long chunks, long n) {
  __shared__ double lds[4][64 * 10];
  const int lane = threadIdx.x & 63, wave = threadIdx.x / 64;
  const long c = (long)blockIdx.x * 4 + wave;
  if (c >= chunks) return;
  long i = c * 64 + lane;
  if (i >= n) i = n - 1;
  const int2 id = ids[i];
  const double2 o = obs[i];
  const double* pt = pts + 3L * id.y;
  double v = o.x + o.y + pt[0] + pt[1] + pt[2];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int p = k * 64 + lane;
    const int t = p / 5, q = p % 5;
    const int cid = __shfl(id.x, t, 64);
    const double2 w = *reinterpret_cast<const double2*>(cams + 10L * cid + 2 * q);
    *reinterpret_cast<double2*>(lds[wave] + t * 10 + 2 * q) = w;
  }
  __builtin_amdgcn_wave_barrier();
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < 9; ++k) s += lds[wave][lane * 10 + k];
  __builtin_amdgcn_wave_barrier();
  v += s;
  double* pr = res + 128 * c + 2 * lane;
  double* pe = E + 384 * c + 2 * lane;
  double* pf = F + 1152 * c + 2 * lane;
  double* pp = sink + 1 + c;
  double* pw = sink + 64 * c + lane;
  const v4i d = as4(v, v);
  if constexpr (kP == 2) {
    if (lane == 0) asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(pp), "v"(v) : "memory");
  }
  v4i e[3] = {d, d, d};
  v4i f[9] = {d, d, d, d, d, d, d, d, d};
  if constexpr (kP == 6 || kP == 7 || kP == 8) {
    // 12 distinct register quads: 6 = copies of d (same data), 7 = random
    // 64-bit words (distinct per lane and per store), 8 = same data in all
    // lanes of a store but distinct per store
    const unsigned long h0 = (unsigned long)i * 0x9E3779B97F4A7C15UL ^ __double_as_longlong(v);
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      v4i q;
      if constexpr (kP == 6) {
        q = d;
        asm volatile("v_mov_b32 %0, %0" : "+v"(q.x));  // a distinct copy the compiler must keep
      } else if constexpr (kP == 7) {
        const unsigned long a = (h0 + j) * 0xBF58476D1CE4E5B9UL, b = (h0 ^ (j * 77)) * 0x94D049BB133111EBUL;
        q = v4i{(int)a, (int)(a >> 32), (int)b, (int)(b >> 32)};
      } else {
        const unsigned long a = (c + j) * 0xBF58476D1CE4E5B9UL;
        q = v4i{(int)a, (int)(a >> 32), (int)(a >> 7), (int)(a >> 40)};
      }
      if (j < 3) e[j] = q; else f[j - 3] = q;
    }
  }
  if constexpr (kP == 5)
    store13_nt_pos(pr, pe, pf, d, e, f);
  else
    store13_nt(pr, pe, pf, d, e, f);
  if constexpr (kP == 1) {
    if (lane == 0) asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(pp), "v"(v) : "memory");
  }
  if constexpr (kP == 3) asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(pw), "v"(v) : "memory");
  if constexpr (kP == 4) {
    // lane-0 partial with the output segments' streaming policy
    if (lane == 0) asm volatile("global_store_dwordx2 %0, %1, off sc1 nt" ::"v"(pp), "v"(v) : "memory");
  }
  asm volatile("" ::"v"(pr), "v"(pe), "v"(pf), "v"(d), "v"(v));
#pragma unroll
  for (int j = 0; j < 3; ++j) asm volatile("" ::"v"(e[j]));
#pragma unroll
  for (int j = 0; j < 9; ++j) asm volatile("" ::"v"(f[j]));
}

__global__ void tiny(double* p) {
  if (threadIdx.x == 0) p[0] += 1.0;
}

__global__ void init_ids(int2* ids, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned h = (unsigned)(i * 2654435761u) ^ (unsigned)(i >> 7) * 40503u;
  ids[i] = make_int2((int)(h % kC), (int)((i * (long)kP) / n));
}

int main(int argc, char** argv) {
  int reps = 10;
  const long chunks = (kO + 63) / 64;
  double *big, *res, *E, *F, *pts, *cam80;
  int2* ids;
  double2* obs;
  CHECK(hipMalloc(&big, (128L + 384L + 1152L) * chunks * 8 + 4096));
  res = big;
  E = big + 128L * chunks;
  F = E + 384L * chunks;
  CHECK(hipMalloc(&pts, 3L * kP * 8));
  CHECK(hipMalloc(&cam80, 10L * kC * 8));
  CHECK(hipMalloc(&ids, (long)kO * 8));
  CHECK(hipMalloc(&obs, (long)kO * 16));
  CHECK(hipMemset(cam80, 0, 10L * kC * 8));
  CHECK(hipMemset(pts, 0, 3L * kP * 8));
  CHECK(hipMemset(obs, 0, (long)kO * 16));
  hipLaunchKernelGGL(init_ids, dim3((kO + 255) / 256), dim3(256), 0, 0, ids, (long)kO);
  CHECK(hipDeviceSynchronize());
  // Optional: the bench's real inputs (tools/dump_bal.py writes them).
  if (const char* dir = getenv("MB_INPUTS")) {
    auto load = [&](const char* name, void* dst, size_t bytes) {
      char path[512];
      snprintf(path, sizeof path, "%s/%s", dir, name);
      FILE* f = fopen(path, "rb");
      if (!f) { fprintf(stderr, "cannot open %s\n", path); exit(1); }
      void* h = malloc(bytes);
      if (fread(h, 1, bytes, f) != bytes) { fprintf(stderr, "short read %s\n", path); exit(1); }
      fclose(f);
      CHECK(hipMemcpy(dst, h, bytes, hipMemcpyHostToDevice));
      free(h);
    };
    load("ids.bin", ids, (size_t)kO * 8);
    load("obs.bin", obs, (size_t)kO * 16);
    load("pts.bin", pts, (size_t)kP * 24);
    load("cam80.bin", cam80, (size_t)kC * 80);
    printf("loaded real inputs from %s\n", dir);
  }
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const double wbytes = 208.0 * kO, rbytes = 24.0 * kO + 24.0 * kP + 72.0 * kC;
  auto run = [&](const char* name, double bytes, auto launch) {
    launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("%-30s %8.4f ms  %7.0f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
  };
  const long n2 = (128L + 384L + 1152L) * chunks / 2;
  const unsigned g = (unsigned)((chunks + 3) / 4);
  const char* fl[] = {"plain", "nt", "sc1", "sc0sc1", "ntsc1"};
  char nm[128];
#define WSEQ(F)                                                                        \
  snprintf(nm, sizeof nm, "wseq %s", fl[F]);                                          \
  run(nm, wbytes, [&] { hipLaunchKernelGGL(write_seq<F>, dim3(g), dim3(256), 0, 0, big, n2); });
  WSEQ(0) WSEQ(1)
#define WDATA(D, label) run(label, wbytes, [&] { hipLaunchKernelGGL(write_data<D>, dim3(g), dim3(256), 0, 0, big, n2); });
  WDATA(0, "wdata zeros") WDATA(1, "wdata const") WDATA(2, "wdata (t,1.0)")
  WDATA(3, "wdata random64") WDATA(4, "wdata random-doubles")
  WDATA(4, "wdata random-doubles") WDATA(0, "wdata zeros")
  run("read_stream (after random fill)", wbytes, [&] { hipLaunchKernelGGL(read_stream, dim3(g), dim3(256), 0, 0, (const double2*)big, n2, pts); });
  WDATA(0, "wdata zeros")
  run("read_stream (after zero fill)", wbytes, [&] { hipLaunchKernelGGL(read_stream, dim3(g), dim3(256), 0, 0, (const double2*)big, n2, pts); });
#define DMA(M, F, label)                                                                   \
  snprintf(nm, sizeof nm, "dma80 %s %s", label, fl[F]);                                   \
  run(nm, rbytes + wbytes, [&] {                                                          \
    hipLaunchKernelGGL((dma80<M, F>), dim3(g), dim3(256), 0, 0, ids, obs, pts, cam80, res, E, \
                       F_, (long)kO);                                                     \
  });
  double* F_ = F;
#define REG(M, F, label)                                                                   \
  snprintf(nm, sizeof nm, "reg80 %s %s", label, fl[F]);                                   \
  run(nm, rbytes + wbytes, [&] {                                                          \
    hipLaunchKernelGGL((dma80<M, F, true>), dim3(g), dim3(256), 0, 0, ids, obs, pts, cam80, res, \
                       E, F_, (long)kO);                                                  \
  });
  double* sink = nullptr;
  CHECK(hipMalloc(&sink, 512 * (2 + chunks)));
  CHECK(hipMemset(sink, 0, 512 * (2 + chunks)));
  run("m1 same-value", rbytes + wbytes, [&] {
    hipLaunchKernelGGL(m1<0>, dim3(g), dim3(256), 0, 0, ids, obs, pts, cam80, res, E, F_, sink, chunks, (long)kO);
  });
  for (int sh : {8, 4, 2, 16, 0}) {
    snprintf(nm, sizeof nm, "m1 same-value F+%dB", sh * 8);
    run(nm, rbytes + wbytes, [&] {
      hipLaunchKernelGGL(m1<0>, dim3(g), dim3(256), 0, 0, ids, obs, pts, cam80, res, E, F_ + sh, sink, chunks, (long)kO);
    });
    snprintf(nm, sizeof nm, "m1 same-value E,F+%dB", sh * 8);
    run(nm, rbytes + wbytes, [&] {
      hipLaunchKernelGGL(m1<0>, dim3(g), dim3(256), 0, 0, ids, obs, pts, cam80, res, E + sh, F_ + sh, sink, chunks, (long)kO);
    });
  }
  run("m1 distinct-values", rbytes + wbytes, [&] {
    hipLaunchKernelGGL(m1<1>, dim3(g), dim3(256), 0, 0, ids, obs, pts, cam80, res, E, F_, sink, chunks, (long)kO);
  });
  run("m1 distinct-ordered", rbytes + wbytes, [&] {
    hipLaunchKernelGGL(m1<2>, dim3(g), dim3(256), 0, 0, ids, obs, pts, cam80, res, E, F_, sink, chunks, (long)kO);
  });
  run("m1 same-scrambled", rbytes + wbytes, [&] {
    hipLaunchKernelGGL(m1<3>, dim3(g), dim3(256), 0, 0, ids, obs, pts, cam80, res, E, F_, sink, chunks, (long)kO);
  });
#define M1(V, label) run(label, rbytes + wbytes, [&] { hipLaunchKernelGGL(m1<V>, dim3(g), dim3(256), 0, 0, ids, obs, pts, cam80, res, E, F_, sink, chunks, (long)kO); });
#define M2(V, label) run(label, rbytes + wbytes, [&] { hipLaunchKernelGGL(m2<V>, dim3(g), dim3(256), 0, 0, ids, obs, pts, cam80, res, E, F_, sink, chunks, (long)kO); });
  M2(0, "m2 no partial") M2(1, "m2 lane0 partial after") M2(2, "m2 lane0 partial before")
  M2(3, "m2 wave-wide 8B store after") M2(4, "m2 lane-0 nt sc1 store after") M2(5, "m2 positive offsets") M2(0, "m2 no partial")
  M2(6, "m2 12 quads same data") M2(7, "m2 12 quads random data") M2(8, "m2 12 quads lane-uniform")
  M2(6, "m2 12 quads same data")
  M1(0, "m1 same-value")
  M1(30, "m1 same-value + partial store")
  M1(31, "m1 + 64B-line partial") M1(32, "m1 + 128B-line partial") M1(33, "m1 + 8B nt partial")
  M1(34, "m1 + 64B-line nt partial") M1(36, "m1 + partial before stores")
  run("m1 same-value, tiny kernel between", rbytes + wbytes, [&] {
    hipLaunchKernelGGL(m1<0>, dim3(g), dim3(256), 0, 0, ids, obs, pts, cam80, res, E, F_, sink, chunks, (long)kO);
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, 0, sink);
  });
  reps = 100;
  M1(0, "m1 same-value x100")
  M1(22, "m1 same-reg random x100")
  reps = 10;
  M1(20, "m1 same-reg lane-distinct") M1(21, "m1 same-reg chunk-distinct") M1(22, "m1 same-reg random")
  M1(5, "m1 int-distinct") M1(6, "m1 copies-same-value") M1(7, "m1 same-reg nonzero")
  M1(8, "m1 random-data int")
  M1(9, "m1 same + 192 indep FMA") M1(11, "m1 same + 48 indep FMA") M1(10, "m1 same + 192 int ops")
  M1(15, "m1 distinct + keep-alive") M1(16, "m1 distinct asm-block") M1(12, "m1 v_mov copies") M1(13, "m1 2-quad rotation") M1(14, "m1 4-quad rotation")
  run("wsegs one quad", wbytes, [&] { hipLaunchKernelGGL(wsegs<false>, dim3(g), dim3(256), 0, 0, res, E, F_, chunks); });
  run("wsegs 13 quads", wbytes, [&] { hipLaunchKernelGGL(wsegs<true>, dim3(g), dim3(256), 0, 0, res, E, F_, chunks); });
  run("m1 chain-values", rbytes + wbytes, [&] {
    hipLaunchKernelGGL(m1<4>, dim3(g), dim3(256), 0, 0, ids, obs, pts, cam80, res, E, F_, sink, chunks, (long)kO);
  });
  DMA(0, 1, "+segs") REG(0, 1, "+segs") DMA(1, 1, "+stage1") DMA(3, 1, "+stage1+keepalive")
  run("m1 same-value", rbytes + wbytes, [&] {
    hipLaunchKernelGGL(m1<0>, dim3(g), dim3(256), 0, 0, ids, obs, pts, cam80, res, E, F_, sink, chunks, (long)kO);
  });
  return 0;
}
