// Prioritized replay on the GPU (reference PrioritizedReplayBuffer,
// replay_buffer.py:25-90; numpy 2.2 RandomState.choice(p=...)).
//
//   probs = prio[:len] ** alpha            float32 powf (numpy's SIMD pow is <=1 ulp
//                                          away: the one non-bit-exact step)
//   probs /= probs.sum()                   numpy's exact reduction order: 8192-element
//                                          chunks, each a pairwise tree (leaves of <=128
//                                          with 8 accumulators), chunk sums added in order
//   cdf = float64(probs).cumsum()          exact int64 fixed-point prefix in 2^-52 units:
//                                          bit-identical to the sequential float64 cumsum
//                                          whenever every nonzero prob >= 2^-29 (all
//                                          partial sums are then exact doubles); else a
//                                          sequential float64 fallback
//   cdf /= cdf[-1]; idx = cdf.searchsorted(u, 'right'), u = MT19937 53-bit doubles
//   w = (len * probs[idx]) ** -beta; w /= w.max()
#include "replay_dev.h"

#include <cstdio>

namespace sacmi {

constexpr int kChunk = 8192;     // NPY_BUFSIZE
constexpr int kLeaf = 128;       // PW_BLOCKSIZE
constexpr int kScanBlock = 1024;

// ---------------------------------------------------------------------------
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
  launch_check("PER push");
}

// ---------------------------------------------------------------------------
// 1. probs = prio ** alpha
__global__ void k_per_pow(const float* prio, int64_t len, float alpha, float* probs) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < len;
       i += (int64_t)gridDim.x * blockDim.x)
    probs[i] = powf(prio[i], alpha);
}

// numpy pairwise leaf (loops_utils.h.src, n <= 128)
__device__ float pw_leaf(const float* a, int n) {
  if (n < 8) {
    float res = -0.0f;
    for (int i = 0; i < n; ++i) res += a[i];
    return res;
  }
  float r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3], r4 = a[4], r5 = a[5], r6 = a[6], r7 = a[7];
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
    r0 += a[i + 0]; r1 += a[i + 1]; r2 += a[i + 2]; r3 += a[i + 3];
    r4 += a[i + 4]; r5 += a[i + 5]; r6 += a[i + 6]; r7 += a[i + 7];
  }
  float res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res += a[i];
  return res;
}

// 2. one workgroup per 8192-element chunk (deterministic, no contraction: plain float
// adds).  A full chunk is a perfect recursion tree — 8192 halves down to 64 leaves of
// 128 — so it is staged into LDS with float4 loads, its 64 leaves run in parallel and
// the tree combines level by level (node = left + right, the recursion's order).  The
// final partial chunk follows the recursion literally (leaves enumerated and combined
// on one lane).
__global__ __launch_bounds__(256) void k_per_chunk_sum(const float* probs, int64_t len,
                                                       float* chunk_sum) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) float buf[kChunk];
  __shared__ int leaf_off[kChunk / 64], leaf_len[kChunk / 64];
  __shared__ float leaf_val[kChunk / 64];
  __shared__ int nleaf;
  const int64_t c0 = (int64_t)blockIdx.x * kChunk;
  const int n = (int)((len - c0) < kChunk ? (len - c0) : kChunk);
  const float* a = probs + c0;
  if (n == kChunk) {
    for (int q = threadIdx.x; q < kChunk / 4; q += blockDim.x)
      reinterpret_cast<float4*>(buf)[q] = reinterpret_cast<const float4*>(a)[q];
    __syncthreads();
    constexpr int kLeaves = kChunk / kLeaf;   // 64
    if (threadIdx.x < kLeaves) leaf_val[threadIdx.x] = pw_leaf(buf + threadIdx.x * kLeaf, kLeaf);
    __syncthreads();
    for (int w = kLeaves / 2; w >= 1; w >>= 1) {
      float v = 0.f;
      if (threadIdx.x < w) v = leaf_val[2 * threadIdx.x] + leaf_val[2 * threadIdx.x + 1];
      __syncthreads();
      if (threadIdx.x < w) leaf_val[threadIdx.x] = v;
      __syncthreads();
    }
    if (threadIdx.x == 0) chunk_sum[blockIdx.x] = leaf_val[0];
    return;
  }
  if (threadIdx.x == 0) {
    // enumerate leaves in order with an explicit stack of (off, n)
    int st_off[32], st_n[32], sp = 0, k = 0;
    st_off[sp] = 0; st_n[sp] = n; ++sp;
    while (sp) {
      --sp;
      const int o = st_off[sp], m = st_n[sp];
      if (m <= kLeaf) { leaf_off[k] = o; leaf_len[k] = m; ++k; continue; }
      int m2 = m / 2;
      m2 -= m2 % 8;
      st_off[sp] = o + m2; st_n[sp] = m - m2; ++sp;   // right pushed first
      st_off[sp] = o; st_n[sp] = m2; ++sp;            // left popped first
    }
    nleaf = k;
  }
  __syncthreads();
  for (int l = threadIdx.x; l < nleaf; l += blockDim.x) leaf_val[l] = pw_leaf(a + leaf_off[l], leaf_len[l]);
  __syncthreads();
  if (threadIdx.x == 0) {
    // post-order combine: stack of partial sums mirrors the recursion
    int st_n[32], st_state[32], sp = 0, leaf = 0;
    float st_left[32];
    float result = 0.f;
    st_n[sp] = n; st_state[sp] = 0; ++sp;
    bool have = false;
    float val = 0.f;
    while (sp) {
      const int top = sp - 1;
      const int m = st_n[top];
      if (m <= kLeaf) {
        val = leaf_val[leaf++];
        have = true;
        --sp;
      } else if (st_state[top] == 0) {
        int m2 = m / 2;
        m2 -= m2 % 8;
        st_state[top] = 1;
        st_n[sp] = m2; st_state[sp] = 0; ++sp;       // left child
        continue;
      } else if (st_state[top] == 1) {
        st_left[top] = val;
        int m2 = m / 2;
        m2 -= m2 % 8;
        st_state[top] = 2;
        st_n[sp] = m - m2; st_state[sp] = 0; ++sp;   // right child
        continue;
      } else {
        val = st_left[top] + val;
        have = true;
        --sp;
      }
      if (sp == 0 && have) result = val;
    }
    chunk_sum[blockIdx.x] = (n > 0) ? result : -0.0f;
  }
}

// 3. normalise + fixed point + block-local inclusive scan
// NaN / inf / zero normaliser: np.random.choice(p=probs) raises "probabilities contain NaN"
// (replay_buffer.py:60-64; a NaN, negative or infinite priority, or none positive)
__device__ __forceinline__ bool per_total_bad(float t) { return !(t > 0.f && t <= 3.402823466e38f); }

__global__ __launch_bounds__(kScanBlock) void k_per_norm_scan(float* probs, int64_t len,
                                                              const float* chunk_sum, int nchunk,
                                                              int64_t* q, int64_t* block_sum,
                                                              int* bad, int* err) {
#pragma clang fp contract(off)
  __shared__ float s_total;
  __shared__ int64_t wsum[kScanBlock / 64];
  if (threadIdx.x == 0) {
    float t = -0.0f;
    for (int c = 0; c < nchunk; ++c) t = t + chunk_sum[c];
    s_total = t;
    if (blockIdx.x == 0 && per_total_bad(t)) {   // bad[5]: this draw's own NaN
      bad[5] = 1;
      atomicOr(err, (int)ERR_NAN_PER);
    }
  }
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kScanBlock + threadIdx.x;
  int64_t v = 0;
  if (i < len) {
    const float p = probs[i] / s_total;
    probs[i] = p;
    if (p != 0.f && !(p >= 1.862645149230957e-09f)) atomicOr(bad, 1);   // 2^-29
    v = (int64_t)((double)p * 4503599627370496.0);                    // exact when p >= 2^-29
  }
  // inclusive scan in the block
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int64_t base = 0;
  for (int k = 0; k < w; ++k) base += wsum[k];
  x += base;
  if (i < len) q[i] = x;
  if (threadIdx.x == kScanBlock - 1) block_sum[blockIdx.x] = x;
}

// 4. exclusive scan of block sums (one workgroup, sequential in chunks of 1024)
__global__ __launch_bounds__(1024) void k_per_scan_blocks(int64_t* block_sum, int nblocks) {
  __shared__ int64_t wsum[16];
  __shared__ int64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int b0 = 0; b0 < nblocks; b0 += 1024) {
    const int b = b0 + threadIdx.x;
    const int64_t v = b < nblocks ? block_sum[b] : 0;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int64_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int64_t base = carry;
    for (int k = 0; k < w; ++k) base += wsum[k];
    if (b < nblocks) block_sum[b] = base + x - v;   // exclusive
    __syncthreads();
    if (threadIdx.x == 1023) carry = base + x;
    __syncthreads();
  }
}

// 5. cdf = prefix / prefix[-1]  (or the sequential float64 fallback)
__global__ void k_per_cdf(const int64_t* q, const int64_t* block_off, const float* probs,
                          int64_t len, const int* bad, double* cdf) {
  if (*bad) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      double s = 0.0;
      for (int64_t i = 0; i < len; ++i) { s = s + (double)probs[i]; cdf[i] = s; }
      const double last = cdf[len - 1];
      for (int64_t i = 0; i < len; ++i) cdf[i] = cdf[i] / last;
    }
    return;
  }
  const int64_t nb = (len + kScanBlock - 1) / kScanBlock;
  const double last = (double)(q[len - 1] + block_off[nb - 1]);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < len;
       i += (int64_t)gridDim.x * blockDim.x)
    cdf[i] = (double)(q[i] + block_off[i / kScanBlock]) / last;
}

// 6a. k uniforms from numpy's MT19937 (random_sample: 53-bit doubles from word pairs),
// one workgroup, block-parallel twist (replay_dev.h); the generator state is written
// back with exactly the words numpy consumes.  Also beta for this draw
// (replay_buffer.py:54; -beta stored after the k uniforms) and frame += 1.
__global__ __launch_bounds__(1024) void k_per_uniforms(uint32_t* mt, int gen_u, const double* u_in,
                                                       double* u_out, int k, DevScalars* sc,
                                                       double beta_start, double beta_frames,
                                                       const int* bad, const int* err,
                                                       int skip_on_err) {
  extern __shared__ uint32_t words[];   // 2k words
  __shared__ uint32_t key[kMtN];
  const int t = threadIdx.x;
  // this draw's probabilities are NaN (bad[5]): the frame advances, the stream does not;
  // an update graph's draw after an earlier non-finite sample: nothing happens at all
  const bool own_nan = bad[5] != 0;
  if (!own_nan && skip_on_err && *err) return;
  if (gen_u && !own_nan) {
    for (int i = t; i < kMtN; i += blockDim.x) key[i] = mt[i];
    int pos = (int)mt[kMtN];
    __syncthreads();
    const int need = 2 * k;
    for (int done = 0; done < need;) {     // every thread tracks pos/done identically
      if (pos >= kMtN) { mt_twist_block(key); pos = 0; }
      const int take = min(kMtN - pos, need - done);
      for (int j = t; j < take; j += blockDim.x) words[done + j] = mt_temper(key[pos + j]);
      done += take;
      pos += take;
      __syncthreads();
    }
    for (int i = t; i < kMtN; i += blockDim.x) mt[i] = key[i];
    if (t == 0) mt[kMtN] = (uint32_t)pos;
    for (int j = t; j < k; j += blockDim.x)
      u_out[j] = ((double)(words[2 * j] >> 5) * 67108864.0 + (double)(words[2 * j + 1] >> 6)) /
                 9007199254740992.0;
  } else {
    for (int j = t; j < k; j += blockDim.x) u_out[j] = u_in[j];
  }
  if (t == 0) {
    const double fr = (double)sc->per_frame;
    double beta = beta_start + fr * (1.0 - beta_start) / beta_frames;
    if (beta > 1.0) beta = 1.0;
    u_out[k] = -beta;
    sc->per_frame += 1;
  }
}

// 6b. searchsorted(cdf, u, 'right') per draw: the block containing the answer is found
// in an LDS copy of every `stride`-th cdf value, then a binary search inside it; IS
// weight (len*P)^-beta and its maximum (weights > 0: the max of the float bits is
// order-independent, hence deterministic).
constexpr int kTopMax = 2048;
__global__ __launch_bounds__(256) void k_per_search(const double* cdf, const float* probs,
                                                    int64_t len, int64_t stride, int ntop,
                                                    const double* u, int k, int32_t* idx32,
                                                    int64_t* idx64, float* w_out,
                                                    unsigned int* wmax_bits) {
#pragma clang fp contract(off)
  __shared__ double top[kTopMax];
  for (int i = threadIdx.x; i < ntop; i += blockDim.x) {
    const int64_t e = (int64_t)(i + 1) * stride - 1;
    top[i] = cdf[e < len ? e : len - 1];
  }
  __syncthreads();
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  float pw = 0.f;
  if (j < k) {
    const double uj = u[j];
    int tlo = 0, thi = ntop;             // first top entry > u
    while (tlo < thi) {
      const int mid = (tlo + thi) >> 1;
      if (top[mid] > uj) thi = mid; else tlo = mid + 1;
    }
    int64_t lo = (int64_t)tlo * stride;
    int64_t hi = lo + stride < len ? lo + stride : len;
    if (lo > len) lo = len;
    while (lo < hi) {                    // first index with cdf > u inside the block
      const int64_t mid = (lo + hi) >> 1;
      if (cdf[mid] > uj) hi = mid; else lo = mid + 1;
    }
    if (lo > len - 1) lo = len - 1;
    idx32[j] = (int32_t)lo;
    idx64[j] = lo;
    pw = powf((float)len * probs[lo], (float)u[k]);
    w_out[j] = pw;
  }
  unsigned int m = __float_as_uint(pw);
  for (int o = 32; o >= 1; o >>= 1) m = max(m, (unsigned int)__shfl_xor((int)m, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(wmax_bits, m);
}

// 6c. w /= w.max()
__global__ void k_per_wnorm(float* w, int k, const unsigned int* wmax_bits) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < k) w[j] = w[j] / __uint_as_float(*wmax_bits);
}

// ---------------------------------------------------------------------------
// Fused PER sampling: the same arithmetic as the kernels above (bit for bit) in three
// (+1 fallback check) launches instead of nine (plus a memset):
//   F1  pow + 8192-chunk pairwise sums (one workgroup per chunk, staged in LDS) and, in
//       one extra workgroup, the numpy-MT uniforms; block 0 resets the flags/tickets
//   F2  normalise + fixed-point block scan (k_per_norm_scan's body); F2b the sequential
//       float64 cumsum fallback when a prob < 2^-29 was seen (one lane; else a no-op)
//   F3  searchsorted with the cdf formed on the fly from the block-local fixed-point
//       prefix and an LDS exclusive scan of the block totals (no cdf array), IS weights;
//       the last workgroup divides by max(w)
// Flags (PerArgs::bad): [0] fallback needed, [1] max-weight bits, [2] F2 ticket, [3] F3 ticket.
constexpr int kFusedBlocksMax = 16384;   // fixed-point blocks F3 scans in LDS (16.7 M rows)

__device__ void per_chunk_tree(float* buf, int n, float* chunk_out) {
#pragma clang fp contract(off)
  __shared__ int leaf_off[kChunk / 64], leaf_len[kChunk / 64];
  __shared__ float leaf_val[kChunk / 64];
  __shared__ int nleaf;
  if (n == kChunk) {
    constexpr int kLeaves = kChunk / kLeaf;   // 64
    if (threadIdx.x < kLeaves) leaf_val[threadIdx.x] = pw_leaf(buf + threadIdx.x * kLeaf, kLeaf);
    __syncthreads();
    for (int w = kLeaves / 2; w >= 1; w >>= 1) {
      float v = 0.f;
      if (threadIdx.x < w) v = leaf_val[2 * threadIdx.x] + leaf_val[2 * threadIdx.x + 1];
      __syncthreads();
      if (threadIdx.x < w) leaf_val[threadIdx.x] = v;
      __syncthreads();
    }
    if (threadIdx.x == 0) *chunk_out = leaf_val[0];
    return;
  }
  if (threadIdx.x == 0) {
    int st_off[32], st_n[32], sp = 0, k = 0;
    st_off[sp] = 0; st_n[sp] = n; ++sp;
    while (sp) {
      --sp;
      const int o = st_off[sp], m = st_n[sp];
      if (m <= kLeaf) { leaf_off[k] = o; leaf_len[k] = m; ++k; continue; }
      int m2 = m / 2;
      m2 -= m2 % 8;
      st_off[sp] = o + m2; st_n[sp] = m - m2; ++sp;
      st_off[sp] = o; st_n[sp] = m2; ++sp;
    }
    nleaf = k;
  }
  __syncthreads();
  for (int l = threadIdx.x; l < nleaf; l += blockDim.x) leaf_val[l] = pw_leaf(buf + leaf_off[l], leaf_len[l]);
  __syncthreads();
  if (threadIdx.x == 0) {
    int st_n[32], st_state[32], sp = 0, leaf = 0;
    float st_left[32];
    float result = 0.f;
    st_n[sp] = n; st_state[sp] = 0; ++sp;
    bool have = false;
    float val = 0.f;
    while (sp) {
      const int top = sp - 1;
      const int m = st_n[top];
      if (m <= kLeaf) {
        val = leaf_val[leaf++];
        have = true;
        --sp;
      } else if (st_state[top] == 0) {
        int m2 = m / 2;
        m2 -= m2 % 8;
        st_state[top] = 1;
        st_n[sp] = m2; st_state[sp] = 0; ++sp;
        continue;
      } else if (st_state[top] == 1) {
        st_left[top] = val;
        int m2 = m / 2;
        m2 -= m2 % 8;
        st_state[top] = 2;
        st_n[sp] = m - m2; st_state[sp] = 0; ++sp;
        continue;
      } else {
        val = st_left[top] + val;
        have = true;
        --sp;
      }
      if (sp == 0 && have) result = val;
    }
    *chunk_out = (n > 0) ? result : -0.0f;
  }
}

// The fused kernels take the fill from the device scalars (the last push published it),
// and their grids cover the capacity: workgroups past the fill return at once.
__device__ __forceinline__ int64_t per_len(const PerArgs& a) {
  return __atomic_load_n(&a.sc->len, __ATOMIC_RELAXED);
}

__global__ __launch_bounds__(256) void k_per_f1(PerArgs a, int nchunk) {
  const TlMark tl_mark(a.tl, TL_PER_F1);
  extern __shared__ __attribute__((aligned(16))) float dyn[];   // max(8192 floats, 2k words)
  if ((int)blockIdx.x == nchunk) {    // the uniforms workgroup (k_per_uniforms' body)
    __shared__ uint32_t key[kMtN];
    uint32_t* words = reinterpret_cast<uint32_t*>(dyn);
    const int t = threadIdx.x;
    // an update graph's draw after an earlier non-finite sample (ErrBits): the reference
    // never reached it — no draw, no frame step.  Otherwise the stream's words are backed up
    // (bad[4] = 1): F2 puts them back if these probabilities turn out NaN
    if (a.skip_on_err && *a.err) {
      if (t == 0) a.bad[4] = 0;
      return;
    }
    if (a.gen_u) {
      for (int i = t; i < kMtN; i += blockDim.x) key[i] = a.mt[i];
      int pos = (int)a.mt[kMtN];
      for (int i = t; i < kMtN; i += blockDim.x) a.mt_backup[i] = key[i];
      if (t == 0) a.mt_backup[kMtN] = (uint32_t)pos;
      __syncthreads();
      const int need = 2 * a.k;
      for (int done = 0; done < need;) {
        if (pos >= kMtN) { mt_twist_block(key); pos = 0; }
        const int take = min(kMtN - pos, need - done);
        for (int j = t; j < take; j += blockDim.x) words[done + j] = mt_temper(key[pos + j]);
        done += take;
        pos += take;
        __syncthreads();
      }
      for (int i = t; i < kMtN; i += blockDim.x) a.mt[i] = key[i];
      if (t == 0) a.mt[kMtN] = (uint32_t)pos;
      for (int j = t; j < a.k; j += blockDim.x)
        a.u_scratch[j] = ((double)(words[2 * j] >> 5) * 67108864.0 + (double)(words[2 * j + 1] >> 6)) /
                         9007199254740992.0;
    } else {
      for (int j = t; j < a.k; j += blockDim.x) a.u_scratch[j] = a.u[j];
    }
    if (t == 0) {
      const double fr = (double)a.sc->per_frame;
      double beta = a.beta_start + fr * (1.0 - a.beta_start) / a.beta_frames;
      if (beta > 1.0) beta = 1.0;
      a.u_scratch[a.k] = -beta;
      a.sc->per_frame += 1;
      a.bad[4] = a.gen_u ? 1 : 0;
    }
    return;
  }
  if (blockIdx.x == 0 && threadIdx.x < 4) a.bad[threadIdx.x] = 0;
  const int64_t len = per_len(a);
  const int64_t c0 = (int64_t)blockIdx.x * kChunk;
  if (c0 >= len) return;
  const int n = (int)((len - c0) < kChunk ? (len - c0) : kChunk);
  float* buf = dyn;
  if (n == kChunk) {
    for (int q = threadIdx.x; q < kChunk / 4; q += blockDim.x) {
      const float4 x = reinterpret_cast<const float4*>(a.prio + c0)[q];
      const float4 y = make_float4(powf(x.x, a.alpha), powf(x.y, a.alpha), powf(x.z, a.alpha),
                                   powf(x.w, a.alpha));
      reinterpret_cast<float4*>(a.probs + c0)[q] = y;
      reinterpret_cast<float4*>(buf)[q] = y;
    }
  } else {
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const float y = powf(a.prio[c0 + i], a.alpha);
      a.probs[c0 + i] = y;
      buf[i] = y;
    }
  }
  __syncthreads();
  per_chunk_tree(buf, n, a.chunk_sums + blockIdx.x);
}

// 256 threads per 1024-row scan block, 4 consecutive rows per thread: every block's
// workgroup is resident at once (the integer prefix is exact, so the grouping does not
// change a bit of q)
constexpr int kF2Threads = 256;
__global__ __launch_bounds__(kF2Threads) void k_per_f2(PerArgs a) {
#pragma clang fp contract(off)
  const TlMark tl_mark(a.tl, TL_PER_F2);
  __shared__ float s_total;
  __shared__ int64_t wsum[kF2Threads / 64];
  const int64_t len = per_len(a);
  if ((int64_t)blockIdx.x * kScanBlock >= len) return;
  const int nchunk = (int)((len + kChunk - 1) / kChunk);
  if (threadIdx.x < 64) {
    // the chunk sums added in chunk order (numpy): wave 0 loads 64 at a time in one
    // coalesced burst, the running sum takes them one by one with v_readlane (a scalar
    // read of lane l: no LDS round trip per element, unlike a shuffle)
    float t = -0.0f;
    for (int c0 = 0; c0 < nchunk; c0 += 64) {
      const int c = c0 + threadIdx.x;
      const float v = c < nchunk ? a.chunk_sums[c] : 0.f;
      const int m = nchunk - c0 < 64 ? nchunk - c0 : 64;
      for (int l = 0; l < m; ++l)
        t = t + __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
    }
    if (threadIdx.x == 0) s_total = t;
  }
  if (blockIdx.x == 0) {
    __syncthreads();
    if (per_total_bad(s_total)) {
      // "probabilities contain NaN": report, and give the numpy stream its words back
      if (threadIdx.x == 0) atomicOr(a.err, (int)ERR_NAN_PER);
      if (a.bad[4])
        for (int i = threadIdx.x; i <= kMtN; i += blockDim.x) a.mt[i] = a.mt_backup[i];
    }
  }
  const int64_t i0 = (int64_t)blockIdx.x * kScanBlock + 4 * threadIdx.x;
  float pin[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) pin[e] = i0 + e < len ? a.probs[i0 + e] : 0.f;
  __syncthreads();
  int64_t v[4];
  int64_t run = 0;
  bool badp = false;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = 0;
    if (i0 + e < len) {
      const float p = pin[e] / s_total;
      a.probs[i0 + e] = p;
      badp = badp || (p != 0.f && !(p >= 1.862645149230957e-09f));   // 2^-29
      v[e] = (int64_t)((double)p * 4503599627370496.0);
    }
    run += v[e];
    v[e] = run;                        // thread-local inclusive prefix
  }
  if (badp) atomicOr(a.bad, 1);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t x = run;
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int64_t base = x - run;              // exclusive prefix of this thread inside its wave
  for (int k = 0; k < w; ++k) base += wsum[k];
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (i0 + e < len) a.q[i0 + e] = base + v[e];
  if (threadIdx.x == kF2Threads - 1) a.block_sums[blockIdx.x] = base + v[3];
}

// F2b: the sequential float64 cumsum when the fixed point is not exact (a prob < 2^-29
// was seen); a no-op otherwise.  Its own launch: a last-workgroup hand-off inside F2
// would need a device-scope release per workgroup (an L2 writeback each, ~1000 of them).
__global__ void k_per_f2b(PerArgs a) {
  const TlMark tl_mark(a.tl, TL_PER_F2B);
  if (!*a.bad) return;
  const int64_t len = per_len(a);
  double sum = 0.0;
  for (int64_t j = 0; j < len; ++j) { sum = sum + (double)a.probs[j]; a.cdf[j] = sum; }
  const double last = a.cdf[len - 1];
  for (int64_t j = 0; j < len; ++j) a.cdf[j] = a.cdf[j] / last;
}

__global__ __launch_bounds__(256) void k_per_f3(PerArgs a) {
#pragma clang fp contract(off)
  const TlMark tl_mark(a.tl, TL_PER_F3);
  extern __shared__ int64_t off[];       // [nb] exclusive prefix of the block totals
  __shared__ double top[kTopMax];
  __shared__ int64_t wtot[4];
  const bool bad = __atomic_load_n(a.bad, __ATOMIC_RELAXED) != 0;
  const int64_t len = per_len(a);
  const int nb = (int)((len + kScanBlock - 1) / kScanBlock);
  int64_t stride = 1024;
  while ((len + stride - 1) / stride > kTopMax) stride *= 2;
  const int ntop = (int)((len + stride - 1) / stride);
  // exclusive scan of block_sums[0..nb) in chunks of 256 (k_per_scan_blocks' sums)
  int64_t carry = 0;
  for (int b0 = 0; b0 < nb; b0 += 256) {
    const int b = b0 + threadIdx.x;
    const int64_t v = b < nb ? a.block_sums[b] : 0;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int64_t x = v;
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wtot[w] = x;
    __syncthreads();
    int64_t base = carry;
    for (int k = 0; k < w; ++k) base += wtot[k];
    if (b < nb) off[b] = base + x - v;
    carry += wtot[0] + wtot[1] + wtot[2] + wtot[3];
    __syncthreads();
  }
  const double last = (double)(a.q[len - 1] + off[nb - 1]);
  auto cdf_at = [&](int64_t e) -> double {
    return bad ? a.cdf[e] : (double)(a.q[e] + off[e / kScanBlock]) / last;
  };
  for (int i = threadIdx.x; i < ntop; i += blockDim.x) {
    const int64_t e = (int64_t)(i + 1) * stride - 1;
    top[i] = cdf_at(e < len ? e : len - 1);
  }
  __syncthreads();
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  float pw = 0.f;
  if (j < a.k) {
    const double uj = a.u_scratch[j];
    int tlo = 0, thi = ntop;
    while (tlo < thi) {
      const int mid = (tlo + thi) >> 1;
      if (top[mid] > uj) thi = mid; else tlo = mid + 1;
    }
    int64_t lo = (int64_t)tlo * stride;
    int64_t hi = lo + stride < len ? lo + stride : len;
    if (lo > len) lo = len;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (cdf_at(mid) > uj) hi = mid; else lo = mid + 1;
    }
    if (lo > len - 1) lo = len - 1;
    a.idx32[j] = (int32_t)lo;
    a.idx_out[j] = lo;
    pw = powf((float)len * a.probs[lo], (float)a.u_scratch[a.k]);
    a.w_out[j] = pw;
  }
  unsigned int m = __float_as_uint(pw);
  for (int o = 32; o >= 1; o >>= 1) m = max(m, (unsigned int)__shfl_xor((int)m, o, 64));
  unsigned int* wmax = reinterpret_cast<unsigned int*>(a.bad + 1);
  if ((threadIdx.x & 63) == 0) atomicMax(wmax, m);
  // w /= max(w) in k_per_f4 (the kernel boundary orders the atomics; a last-workgroup
  // fence + counter here measured 5 us slower)
}

__global__ void k_per_f4(PerArgs a) {
  const TlMark tl_mark(a.tl, TL_PER_F4);
  const unsigned int* wmax = reinterpret_cast<const unsigned int*>(a.bad + 1);
  const float mx = __uint_as_float(*wmax);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < a.k) a.w_out[i] = a.w_out[i] / mx;
}

void launch_per_sample(const PerArgs& a, hipStream_t s) {
  static_assert(kPerFusedMaxRows == (int64_t)kFusedBlocksMax * kScanBlock, "fused PER bound");
  const int64_t len = a.len;
  if (a.cap <= kPerFusedMaxRows) {
    // geometry from the capacity; the kernels read the fill on the device
    const int nb0 = (int)((a.cap + kScanBlock - 1) / kScanBlock);
    const int nchunk = (int)((a.cap + kChunk - 1) / kChunk);
    size_t lds1 = (size_t)kChunk * 4;
    if ((size_t)a.k * 8 > lds1) lds1 = (size_t)a.k * 8;
    ensure_dyn_lds(reinterpret_cast<const void*>(&k_per_f1), lds1);
    // timeline slots: one per kernel, in launch order
    auto at = [&](int i) { PerArgs x = a; x.tl = a.tl ? a.tl + i * kTlWords : nullptr; return x; };
    hipLaunchKernelGGL(k_per_f1, dim3(nchunk + 1), dim3(256), lds1, s, at(0), nchunk);
    hipLaunchKernelGGL(k_per_f2, dim3(nb0), dim3(kF2Threads), 0, s, at(1));
    hipLaunchKernelGGL(k_per_f2b, dim3(1), dim3(64), 0, s, at(2));
    const size_t lds3 = (size_t)nb0 * 8;
    ensure_dyn_lds(reinterpret_cast<const void*>(&k_per_f3), lds3);
    hipLaunchKernelGGL(k_per_f3, dim3((a.k + 255) / 256), dim3(256), lds3, s, at(3));
    hipLaunchKernelGGL(k_per_f4, dim3((a.k + 255) / 256), dim3(256), 0, s, at(4));
    launch_check("PER sample (fused)");
    return;
  }
  // very large rings: the unfused sequence
  int64_t blocks = (len + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(k_per_pow, dim3((unsigned)blocks), dim3(256), 0, s, a.prio, len, a.alpha, a.probs);
  const int nchunk = (int)((len + kChunk - 1) / kChunk);
  hipLaunchKernelGGL(k_per_chunk_sum, dim3(nchunk), dim3(128), 0, s, a.probs, len, a.chunk_sums);
  const int nb = (int)((len + kScanBlock - 1) / kScanBlock);
  (void)hipMemsetAsync(a.bad, 0, 24, s);    // bad flag, max-weight bits, .., own-NaN flag
  hipLaunchKernelGGL(k_per_norm_scan, dim3(nb), dim3(kScanBlock), 0, s, a.probs, len,
                     a.chunk_sums, nchunk, a.q, a.block_sums, a.bad, a.err);
  hipLaunchKernelGGL(k_per_scan_blocks, dim3(1), dim3(1024), 0, s, a.block_sums, nb);
  hipLaunchKernelGGL(k_per_cdf, dim3((unsigned)blocks), dim3(256), 0, s, a.q, a.block_sums,
                     a.probs, len, a.bad, a.cdf);
  hipLaunchKernelGGL(k_per_uniforms, dim3(1), dim3(1024), (size_t)a.k * 8, s, a.mt, a.gen_u,
                     a.u, a.u_scratch, a.k, a.sc, a.beta_start, a.beta_frames, a.bad, a.err,
                     a.skip_on_err);
  int64_t stride = 1024;
  while ((len + stride - 1) / stride > kTopMax) stride *= 2;
  const int ntop = (int)((len + stride - 1) / stride);
  const int sg = (a.k + 255) / 256;
  unsigned int* wmax = reinterpret_cast<unsigned int*>(a.bad + 1);
  hipLaunchKernelGGL(k_per_search, dim3(sg), dim3(256), 0, s, a.cdf, a.probs, len, stride, ntop,
                     a.u_scratch, a.k, a.idx32, a.idx_out, a.w_out, wmax);
  hipLaunchKernelGGL(k_per_wnorm, dim3(sg), dim3(256), 0, s, a.w_out, a.k, wmax);
  launch_check("PER sample");
}

// update_priorities (replay_buffer.py:84-87): sequential semantics, last duplicate wins
__global__ void k_owner_claim(const int64_t* idx, int64_t n, int32_t* owner) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    atomicMax(&owner[idx[i]], (int32_t)i);
}
__global__ void k_owner_write(const int64_t* idx, const float* val, int64_t n, int32_t* owner,
                              float* prio) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    if (owner[idx[i]] == (int32_t)i) prio[idx[i]] = val[i];
}
__global__ void k_owner_reset(const int64_t* idx, int64_t n, int32_t* owner) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    owner[idx[i]] = -1;
}

void launch_per_update(float* prio, const int64_t* idx, const float* val, int64_t n,
                       int32_t* owner, hipStream_t s) {
  int64_t blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k_owner_claim, dim3((unsigned)blocks), dim3(256), 0, s, idx, n, owner);
  hipLaunchKernelGGL(k_owner_write, dim3((unsigned)blocks), dim3(256), 0, s, idx, val, n, owner, prio);
  hipLaunchKernelGGL(k_owner_reset, dim3((unsigned)blocks), dim3(256), 0, s, idx, n, owner);
  launch_check("PER update_priorities");
}

}  // namespace sacmi
