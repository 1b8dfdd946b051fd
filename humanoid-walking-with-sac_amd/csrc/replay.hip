// Replay-side integer kernels (gfx950): bit-exact `random.sample` on the GPU.
//
// The reference draws its minibatch with CPython's random.sample(deque, B)
// (replay_buffer.py:15 -> /usr/lib/python3.10/random.py:485-504, _randbelow
// :239-249): MT19937 words, rejection sampling with getrandbits(k) = word >> (32-k),
// and either a partial Fisher-Yates over a pool (n <= setsize) or a "retry while
// already selected" loop over a set (n > setsize).
//
// Set branch, parallel and exact: every MT word w_t of the stream yields candidate
// r_t = temper(w_t) >> (32-k) accepted iff r_t < n (independent per word).  A
// candidate is SELECTED iff it is the first occurrence of its value in the
// candidate stream (an earlier equal value was selected, so the reference's retry
// loop skips it).  One workgroup processes the stream 624 words (one MT block) at a
// time: temper + accept in parallel, exclusive scan (ballot/popcount), first-
// occurrence test through an LDS hash (atomicMin of the stream sequence number),
// second scan for the selection rank; it stops at the word that yields the k-th
// selection and writes the generator back with exactly the words the reference
// would have consumed.
//
// Pool branch (small n, only while the buffer holds <= setsize rows): one lane
// runs the sequential partial Fisher-Yates in LDS.
#include "sacmi_internal.h"

#include <cstdio>

namespace sacmi {

constexpr int kMtN = 624;
constexpr int kMtM = 397;
constexpr uint32_t kMatrixA = 0x9908B0DFu;
constexpr uint32_t kUpper = 0x80000000u;
constexpr uint32_t kLower = 0x7FFFFFFFu;
constexpr uint32_t kEmpty = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9D2C5680u;
  y ^= (y << 15) & 0xEFC60000u;
  y ^= y >> 18;
  return y;
}

__device__ __forceinline__ uint32_t mt_mix(uint32_t cur, uint32_t nxt, uint32_t far) {
  const uint32_t y = (cur & kUpper) | (nxt & kLower);
  return far ^ (y >> 1) ^ ((y & 1u) ? kMatrixA : 0u);
}

// In-place twist of key[624] by the whole block (4 dependency phases).
__device__ void mt_twist_block(uint32_t* key) {
  const int t = threadIdx.x;
  uint32_t v = 0;
  // phase A: i in [0,227): all inputs old
  if (t < kMtN - kMtM) v = mt_mix(key[t], key[t + 1], key[t + kMtM]);
  __syncthreads();
  if (t < kMtN - kMtM) key[t] = v;
  __syncthreads();
  // phase B: i in [227,454): far = new key[i-227]
  int i = t + (kMtN - kMtM);
  if (t < kMtN - kMtM) v = mt_mix(key[i], key[i + 1], key[i - (kMtN - kMtM)]);
  __syncthreads();
  if (t < kMtN - kMtM) key[i] = v;
  __syncthreads();
  // phase C: i in [454,623)
  i = t + 2 * (kMtN - kMtM);
  const bool c = i < kMtN - 1;
  if (c) v = mt_mix(key[i], key[i + 1], key[i - (kMtN - kMtM)]);
  __syncthreads();
  if (c) key[i] = v;
  __syncthreads();
  // phase D: i = 623
  if (t == 0) key[kMtN - 1] = mt_mix(key[kMtN - 1], key[0], key[kMtM - 1]);
  __syncthreads();
}

__device__ void mt_twist_serial(uint32_t* key) {
  for (int i = 0; i < kMtN; ++i)
    key[i] = mt_mix(key[i], key[(i + 1) % kMtN], key[(i + kMtM) % kMtN]);
}

// Block-wide exclusive scan of a 0/1 flag; returns the rank and writes the total.
__device__ __forceinline__ int block_scan_flag(bool f, int* wave_tot, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long m = __ballot(f);
  const int in_wave = __popcll(m & ((1ull << lane) - 1ull));
  if (lane == 0) wave_tot[w] = __popcll(m);
  __syncthreads();
  int base = 0, tot = 0;
  const int nw = blockDim.x >> 6;
  for (int q = 0; q < nw; ++q) {
    const int c = wave_tot[q];
    if (q < w) base += c;
    tot += c;
  }
  *total = tot;
  __syncthreads();
  return base + in_wave;
}

__device__ __forceinline__ uint32_t hash_slot(uint32_t r, uint32_t mask) {
  return (r * 0x9E3779B1u) & mask;
}

__global__ __launch_bounds__(1024) void k_mt_sample(MtSampleArgs a, int tbl_log2) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  __shared__ uint32_t key[kMtN];
  __shared__ int wave_tot[16];
  __shared__ int s_last, s_pos;
  const int t = threadIdx.x;
  const int64_t n64 = a.sc->len;
  const uint32_t n = (uint32_t)n64;
  const int k = a.k;
  for (int i = t; i < kMtN; i += blockDim.x) key[i] = a.mt[i];
  if (t == 0) s_pos = (int)a.mt[kMtN];
  __syncthreads();
  int pos = s_pos;

  if (n64 <= (int64_t)a.setsize) {
    // ---- pool branch: sequential partial Fisher-Yates (random.py:492-499)
    int32_t* pool = reinterpret_cast<int32_t*>(smem);
    for (int i = t; i < (int)n; i += blockDim.x) pool[i] = i;
    __syncthreads();
    if (t == 0) {
      for (int i = 0; i < k; ++i) {
        const uint32_t m = n - (uint32_t)i;
        const int kb = 32 - __clz((int)m);
        uint32_t r;
        do {
          if (pos >= kMtN) { mt_twist_serial(key); pos = 0; }
          r = mt_temper(key[pos++]) >> (32 - kb);
        } while (r >= m);
        const int32_t v = pool[r];
        a.idx_out[i] = v;
        if (a.idx64_out) a.idx64_out[i] = v;
        pool[r] = pool[m - 1];
      }
      s_pos = pos;
    }
    __syncthreads();
    pos = s_pos;
  } else {
    // ---- set branch: parallel first-occurrence selection (random.py:500-504)
    const uint32_t T = 1u << tbl_log2, mask = T - 1u;
    uint32_t* hkey = smem;
    int32_t* hseq = reinterpret_cast<int32_t*>(smem + T);
    for (uint32_t i = t; i < T; i += blockDim.x) { hkey[i] = kEmpty; hseq[i] = 0x7FFFFFFF; }
    const int kb = 32 - __clz((int)n);   // bit_length(n), n < 2^31
    int count = 0, seqbase = 0;
    __syncthreads();
    for (;;) {
      if (pos >= kMtN) { mt_twist_block(key); pos = 0; }
      const int avail = kMtN - pos;
      const bool valid = t < avail;
      uint32_t r = 0;
      bool acc = false;
      if (valid) {
        r = mt_temper(key[pos + t]) >> (32 - kb);
        acc = r < n;
      }
      int ncand;
      const int crank = block_scan_flag(acc, wave_tot, &ncand);
      const int seq = seqbase + crank;
      uint32_t slot = 0;
      if (acc) {
        slot = hash_slot(r, mask);
        for (;;) {
          const uint32_t prev = atomicCAS(&hkey[slot], kEmpty, r);
          if (prev == kEmpty || prev == r) { atomicMin(&hseq[slot], seq); break; }
          slot = (slot + 1) & mask;
        }
      }
      __syncthreads();
      const bool first = acc && hseq[slot] == seq;
      int nfirst;
      const int srank = block_scan_flag(first, wave_tot, &nfirst);
      if (first && count + srank < k) {
        a.idx_out[count + srank] = (int32_t)r;
        if (a.idx64_out) a.idx64_out[count + srank] = (int64_t)r;
        if (count + srank == k - 1) s_last = t;
      }
      __syncthreads();
      if (count + nfirst >= k) { pos = pos + s_last + 1; break; }
      count += nfirst;
      seqbase += ncand;
      pos = kMtN;
      __syncthreads();
    }
  }
  __syncthreads();
  for (int i = t; i < kMtN; i += blockDim.x) a.mt[i] = key[i];
  if (t == 0) a.mt[kMtN] = (uint32_t)pos;
}

void launch_mt_sample(const MtSampleArgs& a, hipStream_t s) {
  int tl = 4;
  while ((1 << tl) < 2 * (a.k + kMtN)) ++tl;
  const size_t hash_bytes = (size_t)2 * (1u << tl) * 4;
  const size_t pool_bytes = (size_t)a.setsize * 4;
  const size_t lds = hash_bytes > pool_bytes ? hash_bytes : pool_bytes;
  static size_t attr_set = 0;
  if (lds > attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_mt_sample),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = lds;
  }
  hipLaunchKernelGGL(k_mt_sample, dim3(1), dim3(1024), lds, s, a, tl);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) fprintf(stderr, "sacmi: k_mt_sample launch failed: %s\n", hipGetErrorString(e));
}

}  // namespace sacmi
