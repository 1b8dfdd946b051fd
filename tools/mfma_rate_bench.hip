// Microbenchmark: how fast a k_gemm-shaped workgroup retires its fp32 MFMAs.
//
// 256 workgroups x 1024 threads (one per CU, 4 waves per SIMD), every wave runs N
// v_mfma_f32_16x16x4_f32 over 8 independent accumulators (the 32x64 tile's 2 x 4 16x16
// blocks; operands in registers, no memory) and stamps its start / end on the 100 MHz clock.
// Reported per N: the median CU's span (first wave start -> last wave end) against the
// issue-rate floor 4 waves x N x 32 cycles per SIMD, and the implied clock.
// build: hipcc -O3 --offload-arch=gfx950 tools/mfma_rate_bench.hip -o tools/mfma_rate_bench
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

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kWG = 256, kThreads = 1024;

template <int N>   // MFMAs per wave (a multiple of 8)
__global__ __launch_bounds__(kThreads) void k_mfma(const float* seed, unsigned long long* t, float* sink) {
  __shared__ float pad[36 * 1024];   // > 80 KB of LDS: one workgroup per CU
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float a[2], b[4];
#pragma unroll
  for (int i = 0; i < 2; ++i) a[i] = seed[(lane + i) & 63];
#pragma unroll
  for (int j = 0; j < 4; ++j) b[j] = seed[(lane + 2 + j) & 63];
  pad[threadIdx.x] = a[0];
  __syncthreads();
  f4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  unsigned long long t0;
  float z;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)\n\tv_mov_b32 %1, 0" : "=s"(t0), "=v"(z));
#pragma unroll
  for (int i = 0; i < 2; ++i) a[i] += z;   // the MFMAs start after the first stamp
#pragma unroll
  for (int n = 0; n < N / 8; ++n)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][3];
  unsigned long long t1;   // ... and the second waits for their results
  asm volatile("s_nop 0\n\ts_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1) : "v"(s));
  if (lane == 0) {
    t[(blockIdx.x * 16 + wave) * 2] = t0;
    t[(blockIdx.x * 16 + wave) * 2 + 1] = t1;
  }
  sink[blockIdx.x * kThreads + threadIdx.x] = s + pad[(threadIdx.x + 1) & 1023];
}

template <int N>
static void run(const float* seed, unsigned long long* t, float* sink) {
  std::vector<unsigned long long> h(kWG * 32);
  std::vector<double> spans;
  for (int rep = 0; rep < 7; ++rep) {
    hipLaunchKernelGGL(k_mfma<N>, dim3(kWG), dim3(kThreads), 0, 0, seed, t, sink);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    if (rep < 2) continue;
    CHECK(hipMemcpy(h.data(), t, h.size() * 8, hipMemcpyDeviceToHost));
    for (int b = 0; b < kWG; ++b) {
      unsigned long long lo = ~0ull, hi = 0;
      for (int w = 0; w < 16; ++w) {
        lo = std::min(lo, h[(b * 16 + w) * 2]);
        hi = std::max(hi, h[(b * 16 + w) * 2 + 1]);
      }
      spans.push_back((hi - lo) * 0.01);
    }
  }
  std::sort(spans.begin(), spans.end());
  const double us = spans[spans.size() / 2];
  const double cyc = 4.0 * N * 32;   // per SIMD
  printf("N=%4d MFMAs/wave: CU span %6.2f us (p90 %6.2f); floor %6.0f cycles/SIMD -> %5.2f GHz equivalent, %5.1f TF/s chip\n",
         N, us, spans[spans.size() * 9 / 10], cyc, cyc / us * 1e-3, 256.0 * 16 * N * 2048 / us * 1e-6);
}

int main() {
  float *seed, *sink;
  unsigned long long* t;
  CHECK(hipMalloc(&seed, 64 * 4));
  std::vector<float> hs(64);
  for (int i = 0; i < 64; ++i) hs[i] = 1e-3f * (i + 1);
  CHECK(hipMemcpy(seed, hs.data(), 256, hipMemcpyHostToDevice));
  CHECK(hipMalloc(&sink, kWG * kThreads * 4));
  CHECK(hipMalloc(&t, kWG * 32 * 8));
  run<64>(seed, t, sink);
  run<96>(seed, t, sink);
  run<256>(seed, t, sink);
  run<1024>(seed, t, sink);
  return 0;
}
