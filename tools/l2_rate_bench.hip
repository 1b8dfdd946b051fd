// Microbenchmark: the per-CU operand delivery rate of a k_gemm-like load burst by access shape.
//
// Every CU (256 workgroups of 1024 threads, one per CU) loads 192 KB — a 32x64 fp32 tile's
// A (32 x 512) and B (64 x 512) operands at batch 256 — as 16 waves x 12 vector loads of
// 16 B per lane, all issued before one wait, and stamps the burst on the 100 MHz clock.
// Shapes (one wave-instruction = 1 KB):
//   kc64    lane l -> row l & 15, bytes 16 (l >> 4): 16 rows x 64 B (k_gemm's K-contiguous form)
//   kc32x2  lane l -> row l & 15, bytes 32 (l >> 4) (+16 for the odd instruction): two
//           instructions cover 16 rows x 128 B, each touching both halves of every line
//   r128    lane l -> row l >> 3, bytes 16 (l & 7): 8 rows x 128 B
//   r256    lane l -> row l >> 4, bytes 16 (l & 15): 4 rows x 256 B
//   lin     lane l -> 16 l: 1 KB contiguous
//   mn4     dword loads, lane l -> row l >> 4, bytes 4 (l & 15): 4 rows x 64 B (k_gemm's
//           MN-contiguous fragment form: 4x as many wave-instructions of 256 B)
//   dma128  r128 through LDS-DMA (global_load_lds_dwordx4)
//   dma_lin lin through LDS-DMA
// Residency: "l2" = groups of 4 CUs of one XCD read the same 192 KB region (1.5 MB per XCD,
// warm); "mall" = every CU its own region of a 48 MB buffer (past L2, Infinity-Cache hits).
// build: hipcc -O3 --offload-arch=gfx950 tools/l2_rate_bench.hip -o tools/l2_rate_bench
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

constexpr int kWG = 256, kThreads = 1024, kInstr = 12;
constexpr int kRegion = 192 * 1024;   // bytes per CU
constexpr int kRowB = 2048;           // a 512-float row

typedef float f4 __attribute__((ext_vector_type(4)));
__device__ f4 raw_ld4(__amdgpu_buffer_rsrc_t r, int off, int soff, int aux) __asm("llvm.amdgcn.raw.ptr.buffer.load.v4f32");
__device__ float raw_ld1(__amdgpu_buffer_rsrc_t r, int off, int soff, int aux) __asm("llvm.amdgcn.raw.ptr.buffer.load.f32");

enum Shape { KC64, KC32X2, R128, R256, LIN, DMA128, DMALIN, MN4, NSHAPE };

// byte offset of lane l's 16 B in wave-instruction q of wave w (inside the CU's region)
__device__ __forceinline__ int offset(int shape, int w, int q, int l) {
  const int ins = w * kInstr + q;               // 192 instructions per CU, 1 KB each
  switch (shape) {
    case KC64: {   // rows: 96 rows of 2 KB in the region; instruction covers 16 rows x 64 B
      const int rb = (ins % 6) * 16, col = (ins / 6) * 64;   // 6 row blocks x 32 column slices
      return (rb + (l & 15)) * kRowB + col + 16 * (l >> 4);
    }
    case KC32X2: {
      const int pair = ins >> 1, half = ins & 1;
      const int rb = (pair % 6) * 16, col = (pair / 6) * 128;
      return (rb + (l & 15)) * kRowB + col + 32 * (l >> 4) + 16 * half;
    }
    case R128: case DMA128: {
      const int rb = (ins % 12) * 8, col = (ins / 12) * 128;
      return (rb + (l >> 3)) * kRowB + col + 16 * (l & 7);
    }
    case R256: {
      const int rb = (ins % 24) * 4, col = (ins / 24) * 256;
      return (rb + (l >> 4)) * kRowB + col + 16 * (l & 15);
    }
    default:
      return ins * 1024 + 16 * l;
  }
}

template <int SHAPE>
__global__ __launch_bounds__(kThreads) void k_burst(const float* buf, int mall, unsigned long long* dur, float* sink) {
  __shared__ f4 lds[kThreads * 2];   // 32 KB (DMA target, reused); + pad below
  __shared__ float pad[18 * 1024];   // total > 80 KB: one workgroup per CU
  const int b = blockIdx.x, w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int xcd = b & 7, slot = b >> 3;
  const size_t region = mall ? (size_t)b : (size_t)(xcd * 8 + (slot & 7));   // l2: 4 CUs share a region
  const char* base = reinterpret_cast<const char*>(buf) + region * kRegion;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), 0, kRegion, 0x00020000);
  pad[threadIdx.x] = 0.f;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  if constexpr (SHAPE == DMA128 || SHAPE == DMALIN) {
    // LDS-DMA: every instruction writes 1 KB at M0 + 16 * lane (wave-private 2 KB ring)
#pragma unroll
    for (int q = 0; q < kInstr; ++q) {
      const int off = offset(SHAPE, w, q, l);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(base + off),
                                       reinterpret_cast<__attribute__((address_space(3))) void*>(
                                           reinterpret_cast<uintptr_t>(&lds[w * 128 + (q & 1) * 64])),
                                       16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    acc = lds[w * 128 + l];
  } else if constexpr (SHAPE == MN4) {
    // 48 dword instructions of 4 rows x 64 B per wave (the same 12 KB): rows of a 96-row
    // region, 64-byte column slices
    float v[4 * kInstr];
#pragma unroll
    for (int q = 0; q < 4 * kInstr; ++q) {
      const int ins = w * 4 * kInstr + q;   // 768 per CU, 256 B each
      const int rb = (ins % 24) * 4, col = (ins / 24) * 64;
      v[q] = raw_ld1(r, (rb + (l >> 4)) * kRowB + col + 4 * (l & 15), 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 4 * kInstr; ++q) acc[q & 3] += v[q];
  } else {
    f4 v[kInstr];
#pragma unroll
    for (int q = 0; q < kInstr; ++q) v[q] = raw_ld4(r, offset(SHAPE, w, q, l), 0, 0);
#pragma unroll
    for (int q = 0; q < kInstr; ++q) acc += v[q];
  }
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) dur[b] = t1 - t0;
  sink[b * kThreads + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3] + pad[(threadIdx.x + 1) & 1023];
}

// a different kernel between two bursts: write-through stores of 1 KB (as the update's levels
// end), to see whether the next launch still finds the operands in L2
__global__ void k_touch(float* p) {
  __hip_atomic_store(p + threadIdx.x, 1.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
static float* g_touch = nullptr;
static int g_between = 0;   // 1: k_touch between the bursts

template <int S>
static void run(const char* name, const float* buf, unsigned long long* dur, float* sink) {
  std::vector<unsigned long long> h(kWG);
  for (int mall = 0; mall < 2; ++mall) {
    std::vector<double> med;
    for (int rep = 0; rep < 12; ++rep) {
      if (g_between) hipLaunchKernelGGL(k_touch, dim3(1), dim3(256), 0, 0, g_touch);
      hipLaunchKernelGGL(k_burst<S>, dim3(kWG), dim3(kThreads), 0, 0, buf, mall, dur, sink);
      CHECK(hipGetLastError());
      CHECK(hipDeviceSynchronize());
      if (rep < 2) continue;   // warm
      CHECK(hipMemcpy(h.data(), dur, kWG * 8, hipMemcpyDeviceToHost));
      std::sort(h.begin(), h.end());
      med.push_back(h[kWG / 2] * 0.01);
    }
    std::sort(med.begin(), med.end());
    const double us = med[med.size() / 2];
    printf("%-8s %-4s%s burst %6.2f us  -> %6.1f GB/s per CU (median CU, median of 10)\n", name, mall ? "mall" : "l2",
           g_between ? " +touch" : "", us, kRegion / us * 1e-3);
  }
}

int main() {
  float *buf, *sink;
  unsigned long long* dur;
  CHECK(hipMalloc(&buf, (size_t)kWG * kRegion));
  CHECK(hipMemset(buf, 0, (size_t)kWG * kRegion));
  CHECK(hipMalloc(&sink, (size_t)kWG * kThreads * 4));
  CHECK(hipMalloc(&dur, kWG * 8));
  CHECK(hipMalloc(&g_touch, 4096));
  for (g_between = 0; g_between < 2; ++g_between) {
    run<KC64>("kc64", buf, dur, sink);
    run<KC32X2>("kc32x2", buf, dur, sink);
    run<R128>("r128", buf, dur, sink);
    run<R256>("r256", buf, dur, sink);
    run<LIN>("lin", buf, dur, sink);
    run<DMA128>("dma128", buf, dur, sink);
    run<DMALIN>("dma_lin", buf, dur, sink);
    run<MN4>("mn4", buf, dur, sink);
  }
  return 0;
}
