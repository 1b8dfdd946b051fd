// Microbenchmark: synchronisation inside one persistent launch for the batch-256 update.
//
// 256 workgroups of 1024 threads, one per CU (LDS-bound).  A "cohort" is a set of 32
// workgroups meant to share one XCD (blocks b with equal b % 8 under the observed round-robin
// dispatch; the placement is checked with HW_REG_XCC_ID and reported).  Per phase every
// workgroup stores its 8 KB output tile, the cohort synchronises, and every workgroup reads
// the 64 KB its 8 cohort neighbours (slots m & ~7 .. +7) stored — the hand-off of one hidden
// layer of one net at batch 256 (32 rows x 512 columns fp32 per XCD).
//
// modes:
//   0  cohort barrier, plain stores, sc1 loads (same-XCD hand-off: L2-resident)
//   1  cohort barrier, sc1 (write-through) stores, sc1 loads (placement-independent form)
//   2  cohort barrier on cohorts spread over the XCDs (b / 32), agent release + acquire fences
//   3  grid barrier (one counter, 256 arrivals), plain stores + release / acquire fences
//   4  cohort barrier only (no payload)
//   5  grid barrier only (no payload)
//
// build: hipcc -O3 --offload-arch=gfx950 tools/cohort_bench.hip -o tools/cohort_bench
// run:   tools/cohort_bench [phases]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

constexpr int kWG = 256, kThreads = 1024, kTileF = 2048;   // 8 KB tile per workgroup
constexpr long long kSpinLimit = 1ll << 26;

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }

typedef float f4 __attribute__((ext_vector_type(4)));
__device__ f4 raw_ld4(__amdgpu_buffer_rsrc_t r, int off, int soff, int aux) __asm("llvm.amdgcn.raw.ptr.buffer.load.v4f32");
__device__ void raw_st4(f4 v, __amdgpu_buffer_rsrc_t r, int off, int soff, int aux) __asm("llvm.amdgcn.raw.ptr.buffer.store.v4f32");

// arrive + wait on a counter (monotonic within the launch); returns false on timeout
__device__ bool bar(int* cnt, int target, int* err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int ok;
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    long long it = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++it > kSpinLimit) break;
    }
    ok = it <= kSpinLimit;
    if (!ok) atomicOr(err, 1);
  }
  __syncthreads();
  return ok;
}

template <int MODE>
__global__ __launch_bounds__(kThreads) void k_phases(int* cnt, float* buf, int nph, unsigned long long* t,
                                                     int* xcc_of, float* sink, int* err) {
  __shared__ float pad[24 * 1024];   // 96 KB: one workgroup per CU
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) xcc_of[b] = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xf;   // HW_REG_XCC_ID
  const bool spread = MODE == 2;
  const int c = spread ? b / 32 : b % 8, m = spread ? b % 32 : b / 8;
  const bool grid = MODE == 3 || MODE == 5;
  const bool payload = MODE <= 3;
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(buf, 0, 0x7fffffff, 0x00020000);
  pad[tid] = 0.f;
  float acc = 0.f;
  unsigned long long t0 = 0;
  for (int i = 0; i < nph; ++i) {
    if (i == 1) t0 = now();
    float* slab = buf + (size_t)((i & 1) * 8 + c) * 32 * kTileF;   // double-buffered per cohort
    if (payload) {
      // this workgroup's tile: 2048 floats, 2 per thread, as 8-byte halves of a 16-B group
      const int o = (int)(((size_t)((i & 1) * 8 + c) * 32 * kTileF + (size_t)m * kTileF) * 4) + (tid % 512) * 16;
      if (tid < 512) {
        const f4 v = {acc + i, (float)b, (float)tid, 1.f};
        if (MODE == 1) raw_st4(v, rb, o, 0, 16);          // sc1 (write-through)
        else raw_st4(v, rb, o, 0, 0);
      }
      if (MODE >= 2) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
    }
    bool ok;
    if (grid) ok = bar(cnt + 8 * 64, (i + 1) * kWG, err);
    else ok = bar(cnt + c * 64, (i + 1) * 32, err);
    if (!ok) break;
    if (payload) {
      if (MODE >= 2) {
        if (tid == 0) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
      }
      // read the 8 neighbours' tiles: 64 KB, 4 x 16 B per thread, all in flight
      const int g0 = m & ~7;
      f4 v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e = tid + q * kThreads;          // 16-B group e of 4096
        const int o = (int)((((size_t)((i & 1) * 8 + c) * 32 + g0) * kTileF) * 4) + e * 16;
        v[q] = raw_ld4(rb, o, 0, MODE >= 2 ? 0 : 16);   // sc1 loads (L1 bypass) in the fenceless modes
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) acc += v[q][0] + v[q][3];
      (void)slab;
    }
  }
  if (tid == 0 && b == 0) { t[0] = t0; t[1] = now(); }
  sink[b * kThreads + tid] = acc + pad[(tid + 1) % 1024];
}

int main(int argc, char** argv) {
  const int nph = argc > 1 ? atoi(argv[1]) : 200;
  int *cnt, *xcc, *err;
  float *buf, *sink;
  unsigned long long* t;
  CHECK(hipMalloc(&cnt, 16 * 64 * 4));
  CHECK(hipMalloc(&buf, (size_t)2 * 8 * 32 * kTileF * 4));
  CHECK(hipMalloc(&sink, (size_t)kWG * kThreads * 4));
  CHECK(hipMalloc(&t, 16));
  CHECK(hipMalloc(&xcc, kWG * 4));
  CHECK(hipMalloc(&err, 4));
  CHECK(hipMemset(buf, 0, (size_t)2 * 8 * 32 * kTileF * 4));
  const char* names[] = {"cohort, plain st + sc1 ld", "cohort, sc1 st + sc1 ld", "cohort spread over XCDs, fences",
                         "grid (256 arrivals), fences", "cohort barrier only", "grid barrier only"};
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int mode = 0; mode < 6; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      CHECK(hipMemset(cnt, 0, 16 * 64 * 4));
      CHECK(hipMemset(err, 0, 4));
      CHECK(hipEventRecord(e0, 0));
      switch (mode) {
        case 0: hipLaunchKernelGGL(k_phases<0>, dim3(kWG), dim3(kThreads), 0, 0, cnt, buf, nph, t, xcc, sink, err); break;
        case 1: hipLaunchKernelGGL(k_phases<1>, dim3(kWG), dim3(kThreads), 0, 0, cnt, buf, nph, t, xcc, sink, err); break;
        case 2: hipLaunchKernelGGL(k_phases<2>, dim3(kWG), dim3(kThreads), 0, 0, cnt, buf, nph, t, xcc, sink, err); break;
        case 3: hipLaunchKernelGGL(k_phases<3>, dim3(kWG), dim3(kThreads), 0, 0, cnt, buf, nph, t, xcc, sink, err); break;
        case 4: hipLaunchKernelGGL(k_phases<4>, dim3(kWG), dim3(kThreads), 0, 0, cnt, buf, nph, t, xcc, sink, err); break;
        case 5: hipLaunchKernelGGL(k_phases<5>, dim3(kWG), dim3(kThreads), 0, 0, cnt, buf, nph, t, xcc, sink, err); break;
      }
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      unsigned long long th[2];
      int herr = 0;
      CHECK(hipMemcpy(th, t, 16, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
      printf("mode %d %-34s phases %d: %.3f us per phase (device clock), launch %.1f us%s\n", mode, names[mode], nph,
             (double)(th[1] - th[0]) * 0.01 / (nph - 1), ms * 1e3, herr ? "  SPIN TIMEOUT" : "");
    }
  }
  std::vector<int> hx(kWG);
  CHECK(hipMemcpy(hx.data(), xcc, kWG * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int b = 0; b < kWG; ++b)
    if (hx[b] != hx[b % 8]) ++bad;
  printf("placement: block b and b %% 8 on different XCDs for %d of %d blocks; xcc of blocks 0..7:", bad, kWG);
  for (int b = 0; b < 8; ++b) printf(" %d", hx[b]);
  printf("\n");
  return 0;
}
