// Device bodies shared by the replay kernels and the GEMM launches they ride along
// in (multi-update graphs): bit-exact random.sample (see replay.hip) and the minibatch
// row gather.  Included by replay.hip and kernels.hip (no relocatable device code).
#pragma once
#include "sacmi_internal.h"

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

// In-place twist of key[624] by the whole block (needs >= 227 threads), two barriers.
// Word i takes key[i+1] (still old for i < 623) and key[(i+397) % 624], which is old for
// i < 227 and the NEW word i-227 after that: thread t < 227 runs the chain i = t, t+227,
// t+454 in registers from old words only; thread 0 also recomputes new[169] -> new[396]
// for word 623 (which takes new[0] and new[396]).  All reads precede the barrier, all
// writes follow it.  (Was 4 read/write phases, 7 barriers.)
__device__ void mt_twist_block(uint32_t* key) {
  constexpr int D = kMtN - kMtM;   // 227
  const int t = threadIdx.x;
  uint32_t v0 = 0, v1 = 0, v2 = 0, v3 = 0;
  if (t < D) {
    v0 = mt_mix(key[t], key[t + 1], key[t + kMtM]);
    v1 = mt_mix(key[t + D], key[t + D + 1], v0);
    if (t + 2 * D < kMtN - 1) v2 = mt_mix(key[t + 2 * D], key[t + 2 * D + 1], v1);
    if (t == 0) {
      const uint32_t a = mt_mix(key[169], key[170], key[169 + kMtM]);   // new[169]
      const uint32_t b = mt_mix(key[169 + D], key[170 + D], a);         // new[396]
      v3 = mt_mix(key[kMtN - 1], v0, b);                                // new[623]
    }
  }
  __syncthreads();
  if (t < D) {
    key[t] = v0;
    key[t + D] = v1;
    if (t + 2 * D < kMtN - 1) key[t + 2 * D] = v2;
    if (t == 0) key[kMtN - 1] = v3;
  }
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

// hash table size (log2) for k selections: >= 2 * (k + 624) slots
__host__ __device__ constexpr int mt_sample_tbl_log2(int k) {
  int tl = 4;
  while ((1 << tl) < 2 * (k + kMtN)) ++tl;
  return tl;
}

// LDS words the body needs: the hash table (set branch) or the pool, + key + scratch
__host__ __device__ constexpr size_t mt_sample_lds_words(int tbl_log2, int setsize) {
  return ((size_t)2 << tbl_log2) > (size_t)setsize ? ((size_t)2 << tbl_log2) + kMtN + 32
                                                   : (size_t)setsize + kMtN + 32;
}

// Body of the sampler for one workgroup of 1024 threads; `lds` holds
// mt_sample_lds_words(tbl_log2, setsize) words.  Used by k_mt_sample and, riding along
// in a GEMM launch, for the next update of a multi-update graph.
__device__ __forceinline__ void mt_sample_body(const MtSampleArgs& a, int tbl_log2, uint32_t* lds) {
  const size_t tbl_words = ((size_t)2 << tbl_log2) > (size_t)a.setsize ? ((size_t)2 << tbl_log2)
                                                                        : (size_t)a.setsize;
  uint32_t* smem = lds;
  uint32_t* key = lds + tbl_words;
  int* wave_tot = reinterpret_cast<int*>(key + kMtN);
  int& s_last = wave_tot[16];
  int& s_pos = wave_tot[17];
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
      // a candidate's order key is its word's position in the stream (monotone in draw
      // order, so the smallest key per value is its first occurrence): no scan needed
      const int seq = seqbase + t;
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
      seqbase += avail;
      pos = kMtN;
      // (no barrier here: the next twist reads key only after this iteration's last
      // barrier, and the scans' own barriers order every wave_tot reuse)
    }
  }
  __syncthreads();
  for (int i = t; i < kMtN; i += blockDim.x) a.mt[i] = key[i];
  if (t == 0) a.mt[kMtN] = (uint32_t)pos;
}


// One replay row b into the minibatch buffers (replay_buffer.py:13-19 stacking):
// xq[b] = [s | 1 | a], x2[b] = [s2 | 1 | .], x2[B+b] = [s | 1 | .], r[b], d[b].
// Lanes lane, lane+nl, ... of the caller share the row.
__device__ __forceinline__ void gather_row(const GatherArgs& a, int b, int lane, int nl) {
  const int64_t slot = a.by_slot ? (int64_t)a.idx[b] : (a.sc->head + (int64_t)a.idx[b]) % a.capacity;
  const float* so = a.obs + slot * a.ldo;
  const float* s2 = a.obs2 + slot * a.ldo;
  const float* ac = a.act + slot * a.lda_;
  float* xq = a.xq + (size_t)b * a.ldx;
  float* xt = a.x2 + (size_t)b * a.ldx;
  float* xa = a.x2 + (size_t)(a.B + b) * a.ldx;
  // write-through stores (sacmi_internal.h st_wt): the minibatch leaves no dirty L2 lines
  if ((a.S & 3) == 0) {
    const uint32_t oq = (uint32_t)((size_t)b * a.ldx) * 4u, ot = oq;
    const uint32_t oa = (uint32_t)((size_t)(a.B + b) * a.ldx) * 4u;
    for (int q = lane; q < a.S / 4; q += nl) {
      const float4 v = reinterpret_cast<const float4*>(so)[q];
      const float4 w = reinterpret_cast<const float4*>(s2)[q];
      st_wt4(a.xq, oq + 16u * q, v);
      st_wt4(a.x2, oa + 16u * q, v);
      st_wt4(a.x2, ot + 16u * q, w);
    }
  } else {
    for (int q = lane; q < a.S; q += nl) {
      const float v = so[q];
      st_wt(xq + q, v); st_wt(xa + q, v); st_wt(xt + q, s2[q]);
    }
  }
  for (int j = lane; j < a.A; j += nl) st_wt(xq + a.S + 1 + j, ac[j]);
  if (lane == 0) {
    st_wt(a.r + b, a.rew[slot]);
    st_wt(a.d + b, a.done[slot]);
  }
}

}  // namespace sacmi
