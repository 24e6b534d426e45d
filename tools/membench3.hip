// membench3.hip -- round 4: is a persistent, same-wave double-buffered form
// of the hot kernel's memory path faster than one chunk per wave?
// (diagnostic tool, not part of the product; problem-13682 shapes.)
//
// Both forms move the evaluator's bytes: per 64-block chunk the ids (8 B a
// block), observations (16 B), points (24 B, consecutive blocks share
// them), 64 cameras by LDS-DMA from a 128-B-stride table, a fake FP64
// "functor" of kFma dependent-chain FMAs producing 26 doubles per block,
// LDS staging of the F (18) and E (6) cells, and the 13-store tail
// (global_store_dwordx4 sc1 nt) plus a lane-0 partial.
//
//   onechunk<kFma>        one chunk per wave, one-wave workgroups, 4 waves
//                         per SIMD: the shipped kernel's structure
//   persist<kFma>         persistent one-wave workgroups, 2 waves per SIMD:
//                         chunk c+1's ids/obs/points (registers) and cameras
//                         (second LDS buffer) are loaded while chunk c is
//                         computed; chunk c's stores come from a register
//                         set disjoint from chunk c-1's, so no store's
//                         VGPRs are overwritten while it may still be queued.
//                         Every vector-memory instruction is inline asm, the
//                         waits explicit (vmcnt(14) = the previous chunk's
//                         stores may stay in flight).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

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
constexpr int kRow = 16;  // doubles per repacked camera row (128 B)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef double v2d __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v4i As4(double a, double b) {
  double2 v = make_double2(a, b);
  v4i d;
  __builtin_memcpy(&d, &v, 16);
  return d;
}

template <int kOff>
__device__ __forceinline__ void St(double* p, const v4i& d) {
  asm volatile("global_store_dwordx4 %0, %1, off offset:%2 sc1 nt" ::"v"(p), "v"(d), "i"(kOff) : "memory");
}
__device__ __forceinline__ void St8(double* p, double v) {
  asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(p), "v"(v) : "memory");
}

// The fake functor: 26 outputs from 14 inputs through kFma FMAs in 26
// independent chains (bounded values).
template <int kFma>
__device__ __forceinline__ void Fake(const double* x, double* out) {
#pragma unroll
  for (int k = 0; k < 26; ++k) out[k] = x[k % 14];
#pragma unroll
  for (int it = 0; it < kFma / 26; ++it)
#pragma unroll
    for (int k = 0; k < 26; ++k) out[k] = __builtin_fma(out[k], 0.5, 0.25 * x[(k + it) % 14]);
}

// One wave's stores: F 9 pieces, E 3, residual 1 (sector-aligned chunks).
struct Set {
  v4i f[9], e[3], r;
  double *pf, *pe, *pr;
};

__device__ __forceinline__ void Stage(double* st, const double* J, int lane, Set* s) {
  // F: 18 doubles a lane, read back as 9 pieces in segment order; then E.
#pragma unroll
  for (int q = 0; q < 18; q += 2)
    *reinterpret_cast<double2*>(st + lane * 18 + q) = make_double2(J[2 + q], J[3 + q]);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const double2 v = reinterpret_cast<const double2*>(st)[k * kWave + lane];
    s->f[k] = As4(v.x, v.y);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int q = 0; q < 6; q += 2)
    *reinterpret_cast<double2*>(st + lane * 6 + q) = make_double2(J[20 + q], J[21 + q]);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double2 v = reinterpret_cast<const double2*>(st)[k * kWave + lane];
    s->e[k] = As4(v.x, v.y);
  }
  s->r = As4(J[0], J[1]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void Store13(const Set& s) {
  St<-4096>(s.pf, s.f[0]);
  St<-3072>(s.pf, s.f[1]);
  St<-2048>(s.pf, s.f[2]);
  St<-1024>(s.pf, s.f[3]);
  St<0>(s.pf, s.f[4]);
  St<1024>(s.pf, s.f[5]);
  St<2048>(s.pf, s.f[6]);
  St<3072>(s.pf, s.f[7]);
  St<0>(s.pf + 512, s.f[8]);
  St<0>(s.pe, s.e[0]);
  St<1024>(s.pe, s.e[1]);
  St<2048>(s.pe, s.e[2]);
  St<0>(s.pr, s.r);
}

__device__ __forceinline__ void Keep(const Set& s) {
#pragma unroll
  for (int k = 0; k < 9; ++k) asm volatile("" ::"v"(s.f[k]));
#pragma unroll
  for (int k = 0; k < 3; ++k) asm volatile("" ::"v"(s.e[k]));
  asm volatile("" ::"v"(s.r), "v"(s.pf), "v"(s.pe), "v"(s.pr));
}

__device__ __forceinline__ void Addr(Set* s, double* res, double* E, double* F, long c, int lane) {
  s->pr = res + 128 * c + 2 * lane;
  s->pe = E + 384 * c + 2 * lane;
  s->pf = F + 1152 * c + 2 * lane + 512;
}

// ---- one chunk per wave (the shipped structure) ----------------------------
// kLoads: 2 the evaluator's loads (ids, then the camera DMA, observations
// and point); 1 the ids only (the rest derived from them); 0 none (inputs
// derived from the block index): what the load phase costs.
template <int kFma, int kLoads = 2>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void onechunk(
    const int2* ids, const double2* obs, const double* pts, const double* cam, double* res, double* E,
    double* F, double* part, long n) {
  __shared__ alignas(16) double st[64 * 18];
  const int lane = threadIdx.x;
  const long c = blockIdx.x;
  long i = c * 64 + lane;
  if (i >= n) i = n - 1;
  double x[14];
  if constexpr (kLoads == 0) {
#pragma unroll
    for (int k = 0; k < 14; ++k) x[k] = 1.0 + 1e-3 * (double)((i + k) & 1023);
  } else {
    const long long b = __builtin_nontemporal_load(reinterpret_cast<const long long*>(ids) + i);
    const int2 id = make_int2((int)b, (int)(b >> 32));
    if constexpr (kLoads == 1) {
#pragma unroll
      for (int k = 0; k < 14; ++k) x[k] = 1.0 + 1e-3 * (double)((id.x + id.y + k) & 1023);
    } else {
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const int p = k * 64 + lane;
        const int t = p / 5, q = p - t * 5;
        const int cid = __shfl(id.x, t, 64);
        __builtin_amdgcn_global_load_lds(cam + (long)kRow * cid + 2 * q, st + 128 * k, 16, 0, 0);
      }
      x[12] = __builtin_nontemporal_load(reinterpret_cast<const double*>(obs) + 2 * i);
      x[13] = __builtin_nontemporal_load(reinterpret_cast<const double*>(obs) + 2 * i + 1);
      const double* pt = pts + 3L * id.y;
#pragma unroll
      for (int k = 0; k < 3; ++k) x[9 + k] = __builtin_nontemporal_load(pt + k);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < 9; ++k) x[k] = st[lane * 10 + k];
      __builtin_amdgcn_wave_barrier();
    }
  }
  double J[26];
  Fake<kFma>(x, J);
  double w = J[0];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) w += __shfl_xor(w, off, 64);
  Set s;
  Stage(st, J, lane, &s);
  Addr(&s, res, E, F, c, lane);
  double* pp = part + c;
  asm volatile("" : "+v"(pp), "+v"(w));
  Store13(s);
  if (lane == 0) St8(pp, w);
  Keep(s);
  asm volatile("" ::"v"(pp), "v"(w));
}

// ---- persistent, same-wave double-buffered -------------------------------
// In-flight inputs of the next chunk (registers): obs pair, point, ids of
// the chunk after it.
struct Next {
  v2d o;
  double p[3];
  long long id;  // (camera, point) of this lane's block in the chunk after
};

__device__ __forceinline__ long BlockOf(long c, int lane, long n) {
  const long i = c * 64 + lane;
  return i < n ? i : n - 1;
}

// Queue chunk cn's gather: cameras by LDS-DMA into camb (needs id = this
// lane's (camera, point) in cn), obs and point into nx, and the ids of
// chunk cnn into nx->id.  10 vector-memory instructions.
__device__ __forceinline__ void IssueGather(const int2* ids, const double2* obs, const double* pts,
                                            const double* cam, double* camb, long cn, long cnn,
                                            long long id, int lane, long n, Next* nx) {
  const int cid_own = (int)id, pid = (int)(id >> 32);
  const uint32_t lbase = (uint32_t)(uintptr_t)camb;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int p = k * 64 + lane;
    const int t = p / 5, q = p - t * 5;
    const int cid = __shfl(cid_own, t, 64);
    const double* src = cam + (long)kRow * cid + 2 * q;
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(lbase + 1024u * k);
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0)
                 : "memory", "m0");
  }
  const long i = BlockOf(cn, lane, n);
  const double* po = reinterpret_cast<const double*>(obs) + 2 * i;
  asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(nx->o) : "v"(po) : "memory");
  const double* pt = pts + 3L * pid;
  asm volatile("global_load_dwordx2 %0, %1, off nt" : "=v"(nx->p[0]) : "v"(pt) : "memory");
  asm volatile("global_load_dwordx2 %0, %1, off offset:8 nt" : "=v"(nx->p[1]) : "v"(pt) : "memory");
  asm volatile("global_load_dwordx2 %0, %1, off offset:16 nt" : "=v"(nx->p[2]) : "v"(pt) : "memory");
  const long long* pi = reinterpret_cast<const long long*>(ids) + BlockOf(cnn, lane, n);
  asm volatile("global_load_dwordx2 %0, %1, off nt" : "=v"(nx->id) : "v"(pi) : "memory");
}

// Waits for the gather queued one chunk ago (kStores: the vector-memory
// instructions issued after it: the previous chunk's stores); the loaded
// registers are marked as written by the wait so that nothing reads them
// before it.
template <int kCount>
__device__ __forceinline__ void WaitGather(Next* nx) {
  asm volatile("s_waitcnt vmcnt(%4)"
               : "+v"(nx->o), "+v"(nx->p[0]), "+v"(nx->p[1]), "+v"(nx->p[2])
               : "n"(kCount)
               : "memory");
  asm volatile("" : "+v"(nx->id));
}

constexpr int kStoreOps = 14;  // 13 stores + the lane-0 partial

template <int kFma>
__device__ __forceinline__ void Chunk(const int2* ids, const double2* obs, const double* pts,
                                      const double* cam, double* res, double* E, double* F,
                                      double* part, long n, long c, long stride, long nchunks,
                                      double* camb_cur, double* camb_nxt, double* st, Next* cur,
                                      Next* nxt, Set* mine, const Set& prev, int lane) {
  // cur: this chunk's obs/point (loaded), cur->id: the next chunk's ids.
  double x[14];
#pragma unroll
  for (int k = 0; k < 9; ++k) x[k] = camb_cur[lane * 10 + k];
  x[9] = cur->p[0];
  x[10] = cur->p[1];
  x[11] = cur->p[2];
  x[12] = cur->o.x;
  x[13] = cur->o.y;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  const long cn = c + stride;
  if (cn < nchunks)
    IssueGather(ids, obs, pts, cam, camb_nxt, cn, cn + stride, cur->id, lane, n, nxt);
  double J[26];
  Fake<kFma>(x, J);
  double w = J[0];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) w += __shfl_xor(w, off, 64);
  Stage(st, J, lane, mine);
  Addr(mine, res, E, F, c, lane);
  double* pp = part + c;
  asm volatile("" : "+v"(pp), "+v"(w));
  Store13(*mine);
  if (lane == 0) St8(pp, w);
  asm volatile("" ::"v"(pp), "v"(w));
  Keep(prev);  // the previous chunk's store registers stay untouched until here
}

template <int kFma>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void persist(
    const int2* ids, const double2* obs, const double* pts, const double* cam, double* res, double* E,
    double* F, double* part, long n) {
  __shared__ alignas(16) double camb[2][64 * 10];
  __shared__ alignas(16) double st[64 * 18];
  const int lane = threadIdx.x;
  const long nchunks = (n + 63) / 64;
  const long stride = gridDim.x;
  long c = blockIdx.x;
  if (c >= nchunks) return;
  Next A, B;
  // Prologue: chunk c's ids, then its gather (into A, camb[0]).
  long long id0;
  {
    const long long* pi = reinterpret_cast<const long long*>(ids) + BlockOf(c, lane, n);
    asm volatile("global_load_dwordx2 %0, %1, off nt\n\ts_waitcnt vmcnt(0)" : "=v"(id0) : "v"(pi) : "memory");
  }
  IssueGather(ids, obs, pts, cam, camb[0], c, c + stride, id0, lane, n, &A);
  Set S0{}, S1{};
  WaitGather<0>(&A);
  __builtin_amdgcn_wave_barrier();
  for (;;) {
    Chunk<kFma>(ids, obs, pts, cam, res, E, F, part, n, c, stride, nchunks, camb[0], camb[1], st, &A, &B,
                &S0, S1, lane);
    c += stride;
    if (c >= nchunks) break;
    WaitGather<kStoreOps>(&B);
    __builtin_amdgcn_wave_barrier();
    Chunk<kFma>(ids, obs, pts, cam, res, E, F, part, n, c, stride, nchunks, camb[1], camb[0], st, &B, &A,
                &S1, S0, lane);
    c += stride;
    if (c >= nchunks) break;
    WaitGather<kStoreOps>(&A);
    __builtin_amdgcn_wave_barrier();
  }
  Keep(S0);
  Keep(S1);
}

__global__ void init_ids(int2* ids, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned h = (unsigned)(i * 2654435761u) ^ (unsigned)(i >> 7) * 40503u;
  ids[i] = make_int2((int)(h % kC), (int)((i * (long)kP) / n));
}

__global__ void init_vals(double* p, long n, double base) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = base + 1e-3 * (double)(i % 1013);
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const long chunks = (kO + 63) / 64;
  double *res, *E, *F, *pts, *cam, *part;
  int2* ids;
  double2* obs;
  CHECK(hipMalloc(&res, 128L * chunks * 8 + 4096));
  CHECK(hipMalloc(&E, 384L * chunks * 8 + 4096));
  CHECK(hipMalloc(&F, 1152L * chunks * 8 + 8192));
  CHECK(hipMalloc(&part, chunks * 8));
  CHECK(hipMalloc(&pts, 3L * kP * 8));
  CHECK(hipMalloc(&cam, (long)kRow * kC * 8));
  CHECK(hipMalloc(&ids, (long)kO * 8));
  CHECK(hipMalloc(&obs, (long)kO * 16));
  hipLaunchKernelGGL(init_ids, dim3((kO + 255) / 256), dim3(256), 0, 0, ids, (long)kO);
  hipLaunchKernelGGL(init_vals, dim3((3L * kP + 255) / 256), dim3(256), 0, 0, pts, 3L * kP, 1.0);
  hipLaunchKernelGGL(init_vals, dim3((16L * kC + 255) / 256), dim3(256), 0, 0, cam, 16L * kC, 0.5);
  hipLaunchKernelGGL(init_vals, dim3((2L * kO + 255) / 256), dim3(256), 0, 0, (double*)obs, 2L * kO, 3.0);
  CHECK(hipDeviceSynchronize());
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  // Algorithmic bytes as the product counts them (232 per block + points + cameras).
  const double bytes = 232.0 * kO + 24.0 * kP + 72.0 * kC;
  auto run = [&](const char* name, auto launch) {
    launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("%-34s %8.4f ms  %7.0f GB/s  frac %.3f\n", name, ms, bytes / (ms * 1e-3) / 1e9,
           bytes / (ms * 1e-3) / 8e12);
    fflush(stdout);
  };
  const unsigned g1 = (unsigned)chunks;
  auto pgrid = [&](int per_cu) { return (unsigned)(cus * per_cu); };
  for (int round = 0; round < 2; ++round) {
    run("onechunk fma0", [&] { hipLaunchKernelGGL(onechunk<0>, dim3(g1), dim3(64), 0, 0, ids, obs, pts, cam, res, E, F, part, (long)kO); });
    run("onechunk fma702", [&] { hipLaunchKernelGGL(onechunk<702>, dim3(g1), dim3(64), 0, 0, ids, obs, pts, cam, res, E, F, part, (long)kO); });
    run("persist fma0 8/CU", [&] { hipLaunchKernelGGL(persist<0>, dim3(pgrid(8)), dim3(64), 0, 0, ids, obs, pts, cam, res, E, F, part, (long)kO); });
    run("persist fma702 8/CU", [&] { hipLaunchKernelGGL(persist<702>, dim3(pgrid(8)), dim3(64), 0, 0, ids, obs, pts, cam, res, E, F, part, (long)kO); });
    run("persist fma702 6/CU", [&] { hipLaunchKernelGGL(persist<702>, dim3(pgrid(6)), dim3(64), 0, 0, ids, obs, pts, cam, res, E, F, part, (long)kO); });
    run("persist fma702 4/CU", [&] { hipLaunchKernelGGL(persist<702>, dim3(pgrid(4)), dim3(64), 0, 0, ids, obs, pts, cam, res, E, F, part, (long)kO); });
    run("onechunk fma702 ids-only", [&] { hipLaunchKernelGGL((onechunk<702, 1>), dim3(g1), dim3(64), 0, 0, ids, obs, pts, cam, res, E, F, part, (long)kO); });
    run("onechunk fma702 no-loads", [&] { hipLaunchKernelGGL((onechunk<702, 0>), dim3(g1), dim3(64), 0, 0, ids, obs, pts, cam, res, E, F, part, (long)kO); });
    run("onechunk fma0 no-loads", [&] { hipLaunchKernelGGL((onechunk<0, 0>), dim3(g1), dim3(64), 0, 0, ids, obs, pts, cam, res, E, F, part, (long)kO); });
    run("onechunk fma1404", [&] { hipLaunchKernelGGL(onechunk<1404>, dim3(g1), dim3(64), 0, 0, ids, obs, pts, cam, res, E, F, part, (long)kO); });
    run("persist fma1404 8/CU", [&] { hipLaunchKernelGGL(persist<1404>, dim3(pgrid(8)), dim3(64), 0, 0, ids, obs, pts, cam, res, E, F, part, (long)kO); });
  }
  // Check: the last chunk's partial is finite, outputs were written.
  double h = 0;
  CHECK(hipMemcpy(&h, part + chunks - 1, 8, hipMemcpyDeviceToHost));
  printf("last partial %g\n", h);
  return 0;
}
