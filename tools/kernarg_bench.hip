// Microbenchmark: the latency of the first dependent scalar loads of a launch, by source.
//
// k_gemm's levels start with two dependent scalar round trips through their ~2 KB kernel
// argument (the descs' tile starts, then the workgroup's desc) before the first operand load;
// the phase stamps put ~0.9-1 us on the second.  This times one such load per workgroup
// (256 workgroups, one wave each) on the 100 MHz clock, from
//   karg   the kernel argument block (dynamic offset, as batch.d[p])
//   cold   a device buffer line no launch has touched before (HBM)
//   warm   a device buffer line the previous launch read (L2 / MALL)
//   prev   a device buffer line the previous launch wrote (plain stores)
// (karg: a scalar load; the buffer sources: a vector load, as the operand loads)
// launched one by one on a stream and as a captured hipGraph of 32 launches.
// build: hipcc -O3 --offload-arch=gfx950 tools/kernarg_bench.hip -o tools/kernarg_bench
#include <hip/hip_runtime.h>

#include <algorithm>
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

constexpr int kWG = 256, kLaunch = 32, kLineI = 64;   // a 256 B stride per workgroup

struct Args {
  int v[480];   // ~2 KB, as GemmBatch
};

__device__ int raw_ld(__amdgpu_buffer_rsrc_t r, int off, int soff, int aux) __asm("llvm.amdgcn.raw.ptr.buffer.load.i32");

enum Src { KARG, COLD, WARM, PREV, NSRC };

__device__ __forceinline__ unsigned opaque_zero(unsigned long long t) {
  unsigned z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z) : "s"((unsigned)t));
  return z;
}

template <int SRC>
__global__ __launch_bounds__(64) void k_lat(Args a, const int* buf, int* wr, int launch,
                                            unsigned long long* dur, int* sink) {
  const int b = blockIdx.x;
  asm volatile("s_waitcnt lgkmcnt(0)" :: "s"(buf), "s"(launch) : "memory");   // the pointer args first
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const unsigned z = opaque_zero(t0);
  int v;
  if constexpr (SRC == KARG) {
    v = a.v[(b * 7 + (int)z) % 480];
    asm volatile("" :: "s"(v));   // consumed before the second stamp
  } else {
    // cold: a line per (launch, workgroup) never read before; warm / prev: launch-independent
    const size_t line = SRC == COLD ? (size_t)(launch + 1) * kWG + b : (size_t)b;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(buf), 0, 0x7fffffff, 0x00020000);
    v = raw_ld(r, (int)((line * kLineI + z) * 4), 0, 0);
    asm volatile("" :: "v"(v));
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) {
    dur[(size_t)launch * kWG + b] = t1 - t0;
    sink[b] = v;
    if (SRC == PREV) wr[(size_t)b * kLineI] = launch;   // the next launch reads this line
  }
}

template <int S>
static void run(const char* name, bool graph, Args& a, int* buf, unsigned long long* dur, int* sink) {
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int* wr = S == PREV ? buf : sink + 4096;
  if (S == WARM || S == PREV)   // touch the warm lines once
    hipLaunchKernelGGL(k_lat<WARM>, dim3(kWG), dim3(64), 0, st, a, buf, sink + 4096, 0, dur, sink);
  if (graph) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int l = 0; l < kLaunch; ++l)
      hipLaunchKernelGGL(k_lat<S>, dim3(kWG), dim3(64), 0, st, a, buf, wr, l, dur, sink);
    CHECK(hipStreamEndCapture(st, &g));
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CHECK(hipGraphLaunch(ge, st));
    CHECK(hipStreamSynchronize(st));
    CHECK(hipGraphExecDestroy(ge));
    CHECK(hipGraphDestroy(g));
  } else {
    for (int l = 0; l < kLaunch; ++l)
      hipLaunchKernelGGL(k_lat<S>, dim3(kWG), dim3(64), 0, st, a, buf, wr, l, dur, sink);
  }
  CHECK(hipGetLastError());
  CHECK(hipStreamSynchronize(st));
  std::vector<unsigned long long> h((size_t)kLaunch * kWG);
  CHECK(hipMemcpy(h.data(), dur, h.size() * 8, hipMemcpyDeviceToHost));
  // skip the first 2 launches; median and 90th percentile over the rest
  std::vector<unsigned long long> v(h.begin() + 2 * kWG, h.end());
  std::sort(v.begin(), v.end());
  printf("%-5s %-6s median %5.2f us  p90 %5.2f us  max %5.2f us\n", name, graph ? "graph" : "stream",
         v[v.size() / 2] * 0.01, v[v.size() * 9 / 10] * 0.01, v.back() * 0.01);
  CHECK(hipStreamDestroy(st));
}

int main() {
  int *buf, *sink;
  unsigned long long* dur;
  const size_t n = (size_t)(kLaunch + 2) * kWG * kLineI * 4;   // enough cold lines
  CHECK(hipMalloc(&buf, n * sizeof(int)));
  CHECK(hipMemset(buf, 0, n * sizeof(int)));
  CHECK(hipMalloc(&sink, 8192 * sizeof(int) + (size_t)kWG * kLineI * 4));
  CHECK(hipMalloc(&dur, (size_t)kLaunch * kWG * 8));
  Args a;
  for (int i = 0; i < 480; ++i) a.v[i] = i;
  for (int graph = 0; graph < 2; ++graph) {
    run<KARG>("karg", graph, a, buf, dur, sink);
    run<COLD>("cold", graph, a, buf + (graph ? (size_t)(kLaunch + 2) * kWG * kLineI * 2 : 0), dur, sink);
    run<WARM>("warm", graph, a, buf, dur, sink);
    run<PREV>("prev", graph, a, buf, dur, sink);
  }
  return 0;
}
