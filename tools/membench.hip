// membench.hip -- memory-path microbenchmarks for the evaluate kernel's
// access pattern on MI355X (diagnostic tool, not part of the product).
//
// Shapes are those of BAL problem-13682: O = 28,987,644 blocks, 13,682
// cameras (72 B), 4,456,117 points (24 B), per block 8 B ids + 16 B obs
// read, 16 B residuals + 48 B E cell + 144 B F cell written.
//
//   write_seq      pure 16 B/lane streaming stores of the same 6.03 GB
//   write_segs     the evaluator's three output streams per 64-block chunk
//   read_gather    ids + obs + camera gather + point reads only
//   gather_segs    both (the memory floor of the evaluator)
// Each kernel is timed with hipEvents over several launches.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

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

template <bool kNt>
__device__ __forceinline__ void st16(double* p, double a, double b) {
  if constexpr (kNt) {
    __builtin_nontemporal_store(a, p);
    __builtin_nontemporal_store(b, p + 1);
  } else {
    *reinterpret_cast<double2*>(p) = make_double2(a, b);
  }
}

template <bool kNt>
__global__ __launch_bounds__(256) void write_seq(double* out, long n2) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < n2; t += stride)
    st16<kNt>(out + 2 * t, (double)t, 1.0);
}

// One wave per 64-block chunk (grid-stride over chunks).
template <bool kNt>
__device__ __forceinline__ void write_chunk(double* res, double* E, double* F, long c, int lane,
                                            double v) {
  st16<kNt>(res + 128 * c + 2 * lane, v, v);
#pragma unroll
  for (int k = 0; k < 3; ++k) st16<kNt>(E + 384 * c + 128 * k + 2 * lane, v, v);
#pragma unroll
  for (int k = 0; k < 9; ++k) st16<kNt>(F + 1152 * c + 128 * k + 2 * lane, v, v);
}

template <bool kNt>
__global__ __launch_bounds__(256) void write_segs(double* res, double* E, double* F, long chunks) {
  const int lane = threadIdx.x & 63;
  const long stride = (long)gridDim.x * 4;
  for (long c = (long)blockIdx.x * 4 + threadIdx.x / 64; c < chunks; c += stride)
    write_chunk<kNt>(res, E, F, c, lane, (double)c);
}

__device__ __forceinline__ double gather(const int2* ids, const double2* obs, const double* state,
                                         long i) {
  const int2 id = ids[i];
  const double2 o = obs[i];
  const double* cam = state + 3L * kP + 9L * id.x;
  const double* pt = state + 3L * id.y;
  double s = o.x + o.y;
#pragma unroll
  for (int k = 0; k < 9; ++k) s += cam[k];
#pragma unroll
  for (int k = 0; k < 3; ++k) s += pt[k];
  return s;
}

// Wave-cooperative camera gather.  kPad: cameras at an 80-byte stride
// (5 x 16 B pieces, repacked table) loaded as dwordx4; otherwise the
// 72-byte state layout loaded as 9 x 8 B pieces.  Piece p of the wave's
// 64 cameras is loaded by lane p % 64 of instruction p / 64, i.e. lanes
// walk consecutive bytes of a few cameras, then the pieces are
// redistributed through LDS.
template <bool kPad>
__device__ __forceinline__ double coop_camera(const double* cams, int camid, int lane,
                                              double* lds) {
  constexpr int kPieces = kPad ? 5 : 9;
#pragma unroll
  for (int k = 0; k < kPieces; ++k) {
    const int p = k * 64 + lane;
    const int t = p / kPieces, q = p % kPieces;
    const int cid = __shfl(camid, t, 64);
    if constexpr (kPad) {
      const double2 v = *reinterpret_cast<const double2*>(cams + 10L * cid + 2 * q);
      *reinterpret_cast<double2*>(lds + t * 10 + 2 * q) = v;
    } else {
      lds[t * 9 + q] = cams[9L * cid + q];
    }
  }
  __builtin_amdgcn_wave_barrier();
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < 9; ++k) s += lds[lane * (kPad ? 10 : 9) + k];
  __builtin_amdgcn_wave_barrier();
  return s;
}

// Outputs staged through LDS exactly as the evaluator does (lane-major
// block values -> contiguous segments).
__device__ __forceinline__ void write_chunk_staged(double* res, double* E, double* F, long c,
                                                   int lane, double v, double* st) {
  auto seg = [&](double* dst, int per_lane) {
    for (int q = 0; q < per_lane; ++q) st[lane * per_lane + q] = v + q;
    __builtin_amdgcn_wave_barrier();
    for (int t = lane; t < 32 * per_lane; t += 64) {
      const double2 x = reinterpret_cast<const double2*>(st)[t];
      __builtin_nontemporal_store(x.x, dst + 2 * t);
      __builtin_nontemporal_store(x.y, dst + 2 * t + 1);
    }
    __builtin_amdgcn_wave_barrier();
  };
  seg(res + 128 * c, 2);
  seg(E + 384 * c, 6);
  seg(F + 1152 * c, 18);
}

// LDS round trip of the same volume, but the global stores do not depend
// on it (isolates LDS/VGPR-export contention from the store path).
__device__ __forceinline__ double lds_roundtrip(int lane, double v, double* st) {
  double acc = 0.0;
#pragma unroll
  for (int q = 0; q < 24; ++q) st[lane * 24 + q] = v + q;
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int q = 0; q < 24; ++q) acc += st[(q * 64 + lane) % (64 * 24)];
  __builtin_amdgcn_wave_barrier();
  return acc;
}

// Per-lane (unstaged) stores at the block stride: E 48 B, F 144 B per lane.
__device__ __forceinline__ void write_chunk_strided(double* res, double* E, double* F, long c,
                                                    int lane, double v, bool stage_f, double* st) {
  st16<true>(res + 128 * c + 2 * lane, v, v);
#pragma unroll
  for (int k = 0; k < 3; ++k) st16<true>(E + 384 * c + 6 * lane + 2 * k, v, v);
  if (stage_f) {
    for (int q = 0; q < 18; ++q) st[lane * 18 + q] = v + q;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const double2 x = reinterpret_cast<const double2*>(st)[k * 64 + lane];
      st16<true>(F + 1152 * c + 128 * k + 2 * lane, x.x, x.y);
    }
    __builtin_amdgcn_wave_barrier();
  } else {
#pragma unroll
    for (int k = 0; k < 9; ++k) st16<true>(F + 1152 * c + 18 * lane + 2 * k, v, v);
  }
}

template <bool kPad, int kWrite, int kLdsPad = 0>
__global__ __launch_bounds__(256) void coop_gather(const int2* ids, const double2* obs,
                                                   const double* state, const double* cam80,
                                                   double* res, double* E, double* F,
                                                   double* sink, long chunks, long n) {
  __shared__ double lds[4][64 * (kWrite >= 2 ? 24 : 10) + kLdsPad];
  const int lane = threadIdx.x & 63, wave = threadIdx.x / 64;
  const long stride = (long)gridDim.x * 4;
  double acc = 0.0;
  for (long c = (long)blockIdx.x * 4 + wave; c < chunks; c += stride) {
    long i = c * 64 + lane;
    if (i >= n) i = n - 1;
    const int2 id = ids[i];
    const double2 o = obs[i];
    const double* pt = state + 3L * id.y;
    double v = o.x + o.y + pt[0] + pt[1] + pt[2];
    v += kPad ? coop_camera<true>(cam80, id.x, lane, lds[wave])
              : coop_camera<false>(state + 3L * kP, id.x, lane, lds[wave]);
    if constexpr (kWrite == 1) write_chunk<true>(res, E, F, c, lane, v);
    else if constexpr (kWrite == 2) write_chunk_staged(res, E, F, c, lane, v, lds[wave]);
    else if constexpr (kWrite == 3) write_chunk<true>(res, E, F, c, lane, v + lds_roundtrip(lane, v, lds[wave]));
    else if constexpr (kWrite == 4) write_chunk_strided(res, E, F, c, lane, v, false, lds[wave]);
    else if constexpr (kWrite == 5) write_chunk_strided(res, E, F, c, lane, v, true, lds[wave]);
    else acc += v;
  }
  if (acc == 12345.678) sink[0] = acc;
}

__global__ __launch_bounds__(256) void read_gather(const int2* ids, const double2* obs,
                                                   const double* state, double* sink, long n) {
  double s = 0.0;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    s += gather(ids, obs, state, i);
  if (s == 12345.678) sink[0] = s;
}

template <bool kNt>
__global__ __launch_bounds__(256) void gather_segs(const int2* ids, const double2* obs,
                                                   const double* state, double* res, double* E,
                                                   double* F, long chunks, long n) {
  const int lane = threadIdx.x & 63;
  const long stride = (long)gridDim.x * 4;
  for (long c = (long)blockIdx.x * 4 + threadIdx.x / 64; c < chunks; c += stride) {
    long i = c * 64 + lane;
    if (i >= n) i = n - 1;
    const double v = gather(ids, obs, state, i);
    write_chunk<kNt>(res, E, F, c, lane, v);
  }
}

__global__ void init_ids(int2* ids, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // point-major: ~6.5 observations per point; cameras pseudo-random.
  const unsigned h = (unsigned)(i * 2654435761u) ^ (unsigned)(i >> 7) * 40503u;
  ids[i] = make_int2((int)(h % kC), (int)((i * (long)kP) / n));
}

int main(int argc, char** argv) {
  const int reps = 10;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const long chunks = (kO + 63) / 64;
  double *big, *res, *E, *F, *state, *sink;
  int2* ids;
  double2* obs;
  // One allocation, laid out as the evaluator's outputs: residuals, then
  // the Jacobian values (E cells, then F cells).
  CHECK(hipMalloc(&big, (128L + 384L + 1152L) * chunks * 8));
  res = big;
  E = big + 128L * chunks;
  F = E + 384L * chunks;
  CHECK(hipMalloc(&state, (3L * kP + 9L * kC) * 8));
  CHECK(hipMalloc(&ids, (long)kO * 8));
  CHECK(hipMalloc(&obs, (long)kO * 16));
  CHECK(hipMalloc(&sink, 8));
  double* cam80;
  CHECK(hipMalloc(&cam80, 10L * kC * 8));
  CHECK(hipMemset(cam80, 0, 10L * kC * 8));
  CHECK(hipMemset(state, 0, (3L * kP + 9L * kC) * 8));
  CHECK(hipMemset(obs, 0, (long)kO * 16));
  hipLaunchKernelGGL(init_ids, dim3((kO + 255) / 256), dim3(256), 0, 0, ids, (long)kO);
  CHECK(hipDeviceSynchronize());
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
    printf("%-34s %8.4f ms  %7.0f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
  };
  const long n2 = (128L + 384L + 1152L) * chunks / 2;
  for (int wpc : {0}) {
    const unsigned g = wpc ? (unsigned)(cus * wpc) : (unsigned)((chunks + 3) / 4);
    char nm[128];
    snprintf(nm, sizeof nm, "write_seq nt   grid=%u", g);
    run(nm, wbytes, [&] { hipLaunchKernelGGL(write_seq<true>, dim3(g), dim3(256), 0, 0, big, n2); });
    snprintf(nm, sizeof nm, "write_segs nt  grid=%u", g);
    run(nm, wbytes, [&] { hipLaunchKernelGGL(write_segs<true>, dim3(g), dim3(256), 0, 0, res, E, F, chunks); });
    snprintf(nm, sizeof nm, "write_segs pl  grid=%u", g);
    run(nm, wbytes, [&] { hipLaunchKernelGGL(write_segs<false>, dim3(g), dim3(256), 0, 0, res, E, F, chunks); });
    snprintf(nm, sizeof nm, "read_gather    grid=%u", g);
    run(nm, rbytes, [&] { hipLaunchKernelGGL(read_gather, dim3(g), dim3(256), 0, 0, ids, obs, state, sink, (long)kO); });
    snprintf(nm, sizeof nm, "coop72 +segs lds37K grid=%u", g);
    run(nm, rbytes + wbytes, [&] { hipLaunchKernelGGL((coop_gather<false, 1, 512>), dim3(g), dim3(256), 0, 0, ids, obs, state, cam80, res, E, F, sink, chunks, (long)kO); });
    snprintf(nm, sizeof nm, "coop72 +staged   grid=%u", g);
    run(nm, rbytes + wbytes, [&] { hipLaunchKernelGGL((coop_gather<false, 2>), dim3(g), dim3(256), 0, 0, ids, obs, state, cam80, res, E, F, sink, chunks, (long)kO); });
    snprintf(nm, sizeof nm, "coop72 +lds-indep+segs grid=%u", g);
    run(nm, rbytes + wbytes, [&] { hipLaunchKernelGGL((coop_gather<false, 3>), dim3(g), dim3(256), 0, 0, ids, obs, state, cam80, res, E, F, sink, chunks, (long)kO); });
    snprintf(nm, sizeof nm, "coop72 +strided E,F    grid=%u", g);
    run(nm, rbytes + wbytes, [&] { hipLaunchKernelGGL((coop_gather<false, 4>), dim3(g), dim3(256), 0, 0, ids, obs, state, cam80, res, E, F, sink, chunks, (long)kO); });
    snprintf(nm, sizeof nm, "coop72 +strided E, staged F grid=%u", g);
    run(nm, rbytes + wbytes, [&] { hipLaunchKernelGGL((coop_gather<false, 5>), dim3(g), dim3(256), 0, 0, ids, obs, state, cam80, res, E, F, sink, chunks, (long)kO); });
    snprintf(nm, sizeof nm, "coop72 read    grid=%u", g);
    run(nm, rbytes, [&] { hipLaunchKernelGGL((coop_gather<false, 0>), dim3(g), dim3(256), 0, 0, ids, obs, state, cam80, res, E, F, sink, chunks, (long)kO); });
    snprintf(nm, sizeof nm, "coop80 read    grid=%u", g);
    run(nm, rbytes, [&] { hipLaunchKernelGGL((coop_gather<true, 0>), dim3(g), dim3(256), 0, 0, ids, obs, state, cam80, res, E, F, sink, chunks, (long)kO); });
    snprintf(nm, sizeof nm, "coop72 +segs   grid=%u", g);
    run(nm, rbytes + wbytes, [&] { hipLaunchKernelGGL((coop_gather<false, 1>), dim3(g), dim3(256), 0, 0, ids, obs, state, cam80, res, E, F, sink, chunks, (long)kO); });
    snprintf(nm, sizeof nm, "coop80 +segs   grid=%u", g);
    run(nm, rbytes + wbytes, [&] { hipLaunchKernelGGL((coop_gather<true, 1>), dim3(g), dim3(256), 0, 0, ids, obs, state, cam80, res, E, F, sink, chunks, (long)kO); });
    snprintf(nm, sizeof nm, "gather_segs nt grid=%u", g);
    run(nm, rbytes + wbytes, [&] { hipLaunchKernelGGL(gather_segs<true>, dim3(g), dim3(256), 0, 0, ids, obs, state, res, E, F, chunks, (long)kO); });
  }
  return 0;
}
