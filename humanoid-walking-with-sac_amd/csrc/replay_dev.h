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

__device__ __forceinline__ uint32_t hash_slot(uint32_t r, uint32_t mask) {
  return (r * 0x9E3779B1u) & mask;
}

// hash table size (log2) for k selections: >= 2 (k + 624) slots.  At most k - 1 + 624
// distinct values are ever inserted (fewer than k first occurrences before the last block
// of 624 words), so the load factor stays <= 1/2.  compact: >= 1.5 (k + 624) slots (load
// <= 2/3, a few more probes) — batch 4096 then needs 68 KB of LDS instead of 134, which
// fits k_dw_part16's LDS block (the ride-along placement B, sacmi.hip)
__host__ __device__ constexpr int mt_sample_tbl_log2(int k, bool compact = false) {
  int tl = 4;
  while ((1 << tl) < (compact ? 3 * (k + kMtN) / 2 : 2 * (k + kMtN))) ++tl;
  return tl;
}

// LDS words the body needs: the hash table (set branch) or the pool, + key + scratch
// (two 16-word rounds of wave totals, the last selector, the position)
constexpr int kMtScratch = 40;
constexpr int kMtCpt = 3;      // candidate words per thread and round at >= 256 threads
__host__ __device__ constexpr size_t mt_sample_lds_words(int tbl_log2, int setsize) {
  return ((size_t)2 << tbl_log2) > (size_t)setsize ? ((size_t)2 << tbl_log2) + kMtN + kMtScratch
                                                   : (size_t)setsize + kMtN + kMtScratch;
}

// Body of the sampler for one workgroup of 256..1024 threads; `lds` holds
// mt_sample_lds_words(tbl_log2, setsize) words.  Used by k_mt_sample and, riding along
// in a GEMM launch, for the next update of a multi-update graph.
// len_override >= 0: the population size (the mailbox rows this kernel just stored)
__device__ __forceinline__ void mt_sample_body(const MtSampleArgs& a, int tbl_log2, uint32_t* lds,
                                               int64_t len_override = -1) {
  const size_t tbl_words = ((size_t)2 << tbl_log2) > (size_t)a.setsize ? ((size_t)2 << tbl_log2)
                                                                        : (size_t)a.setsize;
  uint32_t* smem = lds;
  uint32_t* key = lds + tbl_words;
  int* wave_tot = reinterpret_cast<int*>(key + kMtN);
  int& s_last = wave_tot[32];
  int& s_pos = wave_tot[33];
  const int t = threadIdx.x;
  const int64_t n64 = len_override >= 0 ? len_override : a.sc->len;
  const uint32_t n = (uint32_t)n64;
  const int k = a.k;
  // an update graph's sampler after a non-finite policy sample / PER draw (ErrBits): the
  // reference raised and never reached this sample, so the stream is left as it is (read
  // with the key: no extra round trip; the indices it writes belong to a voided update)
  const bool keep = !(a.skip_on_err && a.sc->err);
  for (int i = t; i < kMtN; i += blockDim.x) key[i] = a.mt[i];
  if (t == 0) s_pos = (int)a.mt[kMtN];
  __syncthreads();
  int pos = s_pos;
  if (a.mt_save) {   // (unconditional: after a non-finite sample the state is kept, and so is this)
    for (int i = t; i < kMtN; i += blockDim.x) a.mt_save[i] = key[i];
    if (t == 0) a.mt_save[kMtN] = (uint32_t)pos;
  }

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
    const int lane = t & 63, w = t >> 6, nw = (int)blockDim.x >> 6;
    int count = 0, seqbase = 0;
    __syncthreads();
    // one round per block of 624 words (the rest of the current one): thread t takes the
    // cpt consecutive words t * cpt + j (cpt = 3 at 256 threads, 1 at 1024).  Two barriers a
    // round (inserts done; wave totals written): the totals alternate between two 16-word
    // halves by round, so no trailing barrier orders their reuse, and the next round's
    // inserts follow every thread's table reads of this one (before barrier 2)
    const int cpt = (kMtN + (int)blockDim.x - 1) / (int)blockDim.x;
    for (int par = 0;; par ^= 1) {
      if (pos >= kMtN) { mt_twist_block(key); pos = 0; }
      const int avail = kMtN - pos;
      uint32_t r[kMtCpt], slot[kMtCpt];
      bool first[kMtCpt];
#pragma unroll
      for (int j = 0; j < kMtCpt; ++j) {
        const int o = t * cpt + j;
        r[j] = 0; slot[j] = 0; first[j] = false;
        if (j < cpt && o < avail) {
          r[j] = mt_temper(key[pos + o]) >> (32 - kb);
          first[j] = r[j] < n;        // accepted; "first" after the table read below
        }
      }
      // a candidate's order key is its word's position in the stream (monotone in draw
      // order, so the smallest key per value is its first occurrence): no scan needed
#pragma unroll
      for (int j = 0; j < kMtCpt; ++j) {
        if (!first[j]) continue;
        uint32_t sl = hash_slot(r[j], mask);
        for (;;) {
          const uint32_t prev = atomicCAS(&hkey[sl], kEmpty, r[j]);
          if (prev == kEmpty || prev == r[j]) { atomicMin(&hseq[sl], seqbase + t * cpt + j); break; }
          sl = (sl + 1) & mask;
        }
        slot[j] = sl;
      }
      __syncthreads();
      int mine = 0;
#pragma unroll
      for (int j = 0; j < kMtCpt; ++j) {
        first[j] = first[j] && hseq[slot[j]] == seqbase + t * cpt + j;
        mine += first[j] ? 1 : 0;
      }
      // per-lane counts 0..3 as two bit planes: the wave's exclusive prefix and total
      const unsigned long long b0 = __ballot(mine & 1), b1 = __ballot(mine & 2);
      const unsigned long long below = (1ull << lane) - 1ull;
      int* wt = wave_tot + 16 * par;
      if (lane == 0) wt[w] = __popcll(b0) + 2 * __popcll(b1);
      __syncthreads();
      int base = 0, nfirst = 0;
      for (int q = 0; q < nw; ++q) {
        const int c = wt[q];
        base += q < w ? c : 0;
        nfirst += c;
      }
      int rank = count + base + __popcll(b0 & below) + 2 * __popcll(b1 & below);
#pragma unroll
      for (int j = 0; j < kMtCpt; ++j) {
        if (!first[j]) continue;
        if (rank < k) {
          a.idx_out[rank] = (int32_t)r[j];
          if (a.idx64_out) a.idx64_out[rank] = (int64_t)r[j];
          if (rank == k - 1) s_last = t * cpt + j;
        }
        ++rank;
      }
      if (count + nfirst >= k) break;    // (uniform: every thread summed the same totals)
      count += nfirst;
      seqbase += avail;
      pos = kMtN;
    }
    __syncthreads();
    pos += s_last + 1;
  }
  __syncthreads();
  if (!keep) return;
  for (int i = t; i < kMtN; i += blockDim.x) a.mt[i] = key[i];
  if (t == 0) a.mt[kMtN] = (uint32_t)pos;
}


// One replay row b into the minibatch buffers (replay_buffer.py:13-19 stacking):
// xq[b] = [s | 1 | a], x2[b] = [s2 | 1 | .], x2[B+b] = [s | 1 | .], r[b], d[b].
// Lanes lane, lane+nl, ... of the caller share the row.  x16 (act16 updates): the rows
// are bf16 (rounded once here: every consumer rounds its operands to bf16 anyway).  The
// ones column is written with the row (the two layouts share the buffers).
__device__ __forceinline__ void gather_row16(const GatherArgs& a, int64_t slot, int b, int lane, int nl) {
  const float* so = a.obs + slot * a.ldo;
  const float* s2 = a.obs2 + slot * a.ldo;
  const float* ac = a.act + slot * a.lda_;
  const uint32_t oq = (uint32_t)((size_t)b * a.ldx) * 2u, ot = oq;
  const uint32_t oa = (uint32_t)((size_t)(a.B + b) * a.ldx) * 2u;
  const int s4 = a.S >> 2;
  for (int q = lane; q < s4; q += nl) {
    const float4 v = reinterpret_cast<const float4*>(so)[q];
    const float4 w = reinterpret_cast<const float4*>(s2)[q];
    const uint32_t vl = f2bf2(v.x, v.y), vh = f2bf2(v.z, v.w);
    st_wt8(a.xq, oq + 8u * q, vl, vh);
    st_wt8(a.x2, oa + 8u * q, vl, vh);
    st_wt8(a.x2, ot + 8u * q, f2bf2(w.x, w.y), f2bf2(w.z, w.w));
  }
  for (int q = 4 * s4 + lane; q < a.S; q += nl) {
    const unsigned short v = f2bf(so[q]);
    st_wt2(a.xq, oq + 2u * q, v); st_wt2(a.x2, oa + 2u * q, v); st_wt2(a.x2, ot + 2u * q, f2bf(s2[q]));
  }
  for (int j = lane; j < a.A; j += nl) st_wt2(a.xq, oq + 2u * (a.S + 1 + j), f2bf(ac[j]));
  if (lane == 0) {
    st_wt2(a.xq, oq + 2u * a.S, kBf16One); st_wt2(a.x2, oa + 2u * a.S, kBf16One);
    st_wt2(a.x2, ot + 2u * a.S, kBf16One);
    st_wt(a.r + b, a.rew[slot]);
    st_wt(a.d + b, a.done[slot]);
  }
}

__device__ __forceinline__ void gather_row(const GatherArgs& a, int b, int lane, int nl) {
  const int64_t slot = a.by_slot ? (int64_t)a.idx[b] : (a.sc->head + (int64_t)a.idx[b]) % a.capacity;
  if (a.x16) {
    gather_row16(a, slot, b, lane, nl);
    return;
  }
  const float* so = a.obs + slot * a.ldo;
  const float* s2 = a.obs2 + slot * a.ldo;
  const float* ac = a.act + slot * a.lda_;
  float* xq = a.xq + (size_t)b * a.ldx;
  float* xt = a.x2 + (size_t)b * a.ldx;
  float* xa = a.x2 + (size_t)(a.B + b) * a.ldx;
  // write-through stores (sacmi_internal.h st_wt): the minibatch leaves no dirty L2 lines.
  // The state's whole float4s (replay rows and minibatch rows are 16-B aligned: ldo, ldx
  // multiples of 4), then its S % 4 tail (NAO-walk: S = 661)
  const uint32_t oq = (uint32_t)((size_t)b * a.ldx) * 4u, ot = oq;
  const uint32_t oa = (uint32_t)((size_t)(a.B + b) * a.ldx) * 4u;
  const int s4 = a.S >> 2;
  for (int q = lane; q < s4; q += nl) {
    const float4 v = reinterpret_cast<const float4*>(so)[q];
    const float4 w = reinterpret_cast<const float4*>(s2)[q];
    st_wt4(a.xq, oq + 16u * q, v);
    st_wt4(a.x2, oa + 16u * q, v);
    st_wt4(a.x2, ot + 16u * q, w);
  }
  for (int q = 4 * s4 + lane; q < a.S; q += nl) {
    const float v = so[q];
    st_wt(xq + q, v); st_wt(xa + q, v); st_wt(xt + q, s2[q]);
  }
  for (int j = lane; j < a.A; j += nl) st_wt(xq + a.S + 1 + j, ac[j]);
  if (lane == 0) {
    st_wt(xq + a.S, 1.f); st_wt(xa + a.S, 1.f); st_wt(xt + a.S, 1.f);
    st_wt(a.r + b, a.rew[slot]);
    st_wt(a.d + b, a.done[slot]);
  }
}

// Rows b0 + i * bstep (i < R) by one wave, every load of the R rows issued before any
// store: one latency chain for R rows instead of R (the ride-along form — a few hundred
// waves beside a level gather the whole batch).  Loads at clamped addresses, results
// discarded by predicated stores (a guarded load would drain at its guard).  States wider
// than 256 Q floats take gather_row.
template <int R, int Q>
__device__ __forceinline__ void gather_rows_wave(const GatherArgs& a, int b0, int bstep, int lane) {
  const int s4 = a.S >> 2, st = a.S & 3;
  if (s4 > 64 * Q || s4 == 0) {
    for (int i = 0; i < R; ++i)
      if (b0 + i * bstep < a.B) gather_row(a, b0 + i * bstep, lane, 64);
    return;
  }
  int64_t slot[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int b = b0 + i * bstep;
    const int32_t ix = a.idx[b < a.B ? b : 0];
    slot[i] = a.by_slot ? (int64_t)ix : (a.sc->head + (int64_t)ix) % a.capacity;
  }
  float4 v[R][Q], w[R][Q];
  float tv[R], tw[R], av[R], rv[R], dv[R];
  const int jt = 4 * s4 + (lane < st ? lane : 0), ja = lane < a.A ? lane : 0;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const float4* so = reinterpret_cast<const float4*>(a.obs + slot[i] * a.ldo);
    const float4* s2 = reinterpret_cast<const float4*>(a.obs2 + slot[i] * a.ldo);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int qq = lane + 64 * q < s4 ? lane + 64 * q : s4 - 1;
      v[i][q] = so[qq];
      w[i][q] = s2[qq];
    }
    tv[i] = a.obs[slot[i] * a.ldo + (st ? jt : 0)];
    tw[i] = a.obs2[slot[i] * a.ldo + (st ? jt : 0)];
    av[i] = a.act[slot[i] * a.lda_ + ja];
    rv[i] = a.rew[slot[i]];
    dv[i] = a.done[slot[i]];
  }
  if (a.x16) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int b = b0 + i * bstep;
      if (b >= a.B) break;
      const uint32_t oq = (uint32_t)((size_t)b * a.ldx) * 2u, ot = oq;
      const uint32_t oa = (uint32_t)((size_t)(a.B + b) * a.ldx) * 2u;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int qq = lane + 64 * q;
        if (qq < s4) {
          const uint32_t vl = f2bf2(v[i][q].x, v[i][q].y), vh = f2bf2(v[i][q].z, v[i][q].w);
          st_wt8(a.xq, oq + 8u * qq, vl, vh);
          st_wt8(a.x2, oa + 8u * qq, vl, vh);
          st_wt8(a.x2, ot + 8u * qq, f2bf2(w[i][q].x, w[i][q].y), f2bf2(w[i][q].z, w[i][q].w));
        }
      }
      if (lane < st) {
        st_wt2(a.xq, oq + 2u * jt, f2bf(tv[i])); st_wt2(a.x2, oa + 2u * jt, f2bf(tv[i]));
        st_wt2(a.x2, ot + 2u * jt, f2bf(tw[i]));
      }
      if (lane < a.A) st_wt2(a.xq, oq + 2u * (a.S + 1 + lane), f2bf(av[i]));
      if (lane == 0) {
        st_wt2(a.xq, oq + 2u * a.S, kBf16One); st_wt2(a.x2, oa + 2u * a.S, kBf16One);
        st_wt2(a.x2, ot + 2u * a.S, kBf16One);
        st_wt(a.r + b, rv[i]); st_wt(a.d + b, dv[i]);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int b = b0 + i * bstep;
    if (b >= a.B) break;
    const uint32_t oq = (uint32_t)((size_t)b * a.ldx) * 4u, ot = oq;
    const uint32_t oa = (uint32_t)((size_t)(a.B + b) * a.ldx) * 4u;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int qq = lane + 64 * q;
      if (qq < s4) {
        st_wt4(a.xq, oq + 16u * qq, v[i][q]);
        st_wt4(a.x2, oa + 16u * qq, v[i][q]);
        st_wt4(a.x2, ot + 16u * qq, w[i][q]);
      }
    }
    float* xq = a.xq + (size_t)b * a.ldx;
    float* xt = a.x2 + (size_t)b * a.ldx;
    float* xa = a.x2 + (size_t)(a.B + b) * a.ldx;
    if (lane < st) { st_wt(xq + jt, tv[i]); st_wt(xa + jt, tv[i]); st_wt(xt + jt, tw[i]); }
    if (lane < a.A) st_wt(xq + a.S + 1 + lane, av[i]);
    if (lane == 0) {
      st_wt(xq + a.S, 1.f); st_wt(xa + a.S, 1.f); st_wt(xt + a.S, 1.f);
      st_wt(a.r + b, rv[i]); st_wt(a.d + b, dv[i]);
    }
  }
}

}  // namespace sacmi
