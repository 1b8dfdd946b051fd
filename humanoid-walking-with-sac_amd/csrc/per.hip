// Prioritized replay (reference PrioritizedReplayBuffer, replay_buffer.py:25-90).
#include "sacmi_internal.h"

#include <cstdio>

namespace sacmi {

// push: every new row gets max(priorities[0:capacity]) (or 1.0 when the buffer was
// empty) — replay_buffer.py:38,46.  Priorities are >= 0, so the float max is the
// unsigned max of the bit patterns (order-independent => deterministic).
__global__ void k_prio_max(const float* prio, int64_t cap, unsigned int* out) {
  unsigned int m = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap;
       i += (int64_t)gridDim.x * blockDim.x)
    m = max(m, __float_as_uint(prio[i]));
  for (int o = 32; o >= 1; o >>= 1) m = max(m, (unsigned int)__shfl_xor((int)m, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

__global__ void k_prio_fill(float* prio, int64_t cap, int64_t pos, int64_t n,
                            const unsigned int* maxbits, int empty) {
  const float v = empty ? 1.0f : __uint_as_float(*maxbits);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    prio[(pos + i) % cap] = v;
}

void launch_per_push(float* prio, int64_t cap, int64_t pos, int64_t n, int empty, float* scratch,
                     hipStream_t s) {
  unsigned int* mb = reinterpret_cast<unsigned int*>(scratch);
  (void)hipMemsetAsync(mb, 0, 4, s);
  int64_t blocks = (cap + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(k_prio_max, dim3((unsigned)blocks), dim3(256), 0, s, prio, cap, mb);
  int64_t fb = (n + 255) / 256;
  if (fb > 1024) fb = 1024;
  if (fb < 1) fb = 1;
  hipLaunchKernelGGL(k_prio_fill, dim3((unsigned)fb), dim3(256), 0, s, prio, cap, pos, n, mb, empty);
}

}  // namespace sacmi
