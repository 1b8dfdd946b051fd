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
#include "replay_dev.h"

#include <cstdio>

namespace sacmi {

// The mailbox's rows into the ring slots pos0.. (k_push_rows' stores, from the packed
// host-mapped rows), then the replay's len / head; returns the new len (-1: no rows)
__device__ int64_t mailbox_scatter(const MailboxArgs& mb, DevScalars* sc) {
  __shared__ int s_n;
  __shared__ int64_t s_hdr[3];
  const int S = mb.S, A = mb.A, rowf = 2 * S + A + 2;
  // row 0 (the trainer's one row) is read together with the header: one PCIe round trip
  constexpr int kR0 = 2;
  float r0[kR0];
#pragma unroll
  for (int q = 0; q < kR0; ++q) {
    const int e = threadIdx.x + q * blockDim.x;
    r0[q] = e < rowf ? mb.rows[e] : 0.f;
  }
  if (threadIdx.x == 0) {
    const volatile PushMailbox* h = mb.hdr;
    s_n = h->n;
    s_hdr[0] = h->pos0; s_hdr[1] = h->len; s_hdr[2] = h->head;
  }
  __syncthreads();
  const int n = s_n;
  if (n <= 0) return -1;
  for (int e = threadIdx.x; e < n * rowf; e += blockDim.x) {
    const int j = e / rowf, c = e - j * rowf;
    const int64_t w = (s_hdr[0] + j) % mb.cap;
    const int q = (e - (int)threadIdx.x) / (int)blockDim.x;
    const float v = e < rowf && q < kR0 ? r0[q < kR0 ? q : 0] : mb.rows[e];
    if (c < S) mb.obs[w * mb.ldo + c] = v;
    else if (c < S + A) mb.act[w * mb.ldact + c - S] = v;
    else if (c == S + A) mb.rew[w] = v;
    else if (c < 2 * S + A + 1) mb.obs2[w * mb.ldo + c - S - A - 1] = v;
    else mb.done[w] = v;
  }
  if (threadIdx.x == 0) {
    sc->len = s_hdr[1];
    sc->head = s_hdr[2];
  }
  return s_hdr[1];
}

__global__ __launch_bounds__(1024) void k_mt_sample(MtSampleArgs a, int tbl_log2, MailboxArgs mb) {
  const TlMark tl_mark(a.tl, TL_MT_SAMPLE);
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int64_t len = mb.hdr ? mailbox_scatter(mb, const_cast<DevScalars*>(a.sc)) : -1;
  mt_sample_body(a, tbl_log2, smem, len);
}

void launch_mt_sample(const MtSampleArgs& a, hipStream_t s, const MailboxArgs* mb) {
  const int tl = mt_sample_tbl_log2(a.k);
  const size_t lds = mt_sample_lds_words(tl, a.setsize) * 4;
  ensure_dyn_lds(reinterpret_cast<const void*>(&k_mt_sample), lds);
  const MailboxArgs m = mb ? *mb : MailboxArgs{};
  hipLaunchKernelGGL(k_mt_sample, dim3(1), dim3(1024), lds, s, a, tl, m);
  launch_check("k_mt_sample");
}

// one wave per ring row (grid-stride), lanes over the row's columns; coalesced both ways
__global__ __launch_bounds__(256) void k_push_rows(PushArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const float* s = a.stage;
  const float* ac = s + a.n * a.S;
  const float* r = ac + a.n * a.A;
  const float* s2 = r + a.n;
  const float* d = s2 + a.n * a.S;
  for (int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < a.n; i += nw) {
    const int64_t w = (a.pos0 + i) % a.cap;
    for (int k = lane; k < a.S; k += 64) {
      a.obs[w * a.ldo + k] = s[i * a.S + k];
      a.obs2[w * a.ldo + k] = s2[i * a.S + k];
    }
    for (int k = lane; k < a.A; k += 64) a.act[w * a.ldact + k] = ac[i * a.A + k];
    if (lane == 0) {
      a.rew[w] = r[i];
      a.done[w] = d[i];
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.sc->len = a.len;
    a.sc->head = a.head;
  }
}

void launch_push_rows(const PushArgs& a, hipStream_t s) {
  const int64_t blocks = (a.n + 3) / 4;
  const int grid = (int)(blocks < 1024 ? (blocks > 0 ? blocks : 1) : 1024);
  hipLaunchKernelGGL(k_push_rows, dim3(grid), dim3(256), 0, s, a);
  launch_check("k_push_rows");
}

}  // namespace sacmi
