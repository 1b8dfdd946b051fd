// libsacmi host runtime: the C ABI of include/sacmi.h.
//
// Owns every device buffer of one agent (parameter arenas, replay ring, scratch),
// sequences the ~20 kernels of one SAC update on one HIP stream, and caches each
// distinct update configuration as an instantiated hipGraph so a training step is
// one graph launch (the step is launch-latency bound at batch 256: SURVEY §7).
#include "replay_dev.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

namespace sacmi {

static thread_local std::string g_last_error;

#define CHECK_HIP(expr)                                                              \
  do {                                                                               \
    hipError_t e_ = (expr);                                                          \
    if (e_ != hipSuccess)                                                            \
      throw Error{SACMI_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)}; \
  } while (0)

#define REQUIRE(cond, code, msg)           \
  do {                                     \
    if (!(cond)) throw Error{code, (msg)}; \
  } while (0)

// every device allocation of the process, for the host-side bounds validator; guarded by
// registry_mutex() (contexts may live on several host threads)
struct AllocRec { uintptr_t base; size_t bytes; };
static std::vector<AllocRec>& alloc_registry() {
  static std::vector<AllocRec> r;
  return r;
}
static std::mutex& registry_mutex() {
  static std::mutex m;
  return m;
}
static void registry_add(uintptr_t base, size_t bytes) {
  std::lock_guard<std::mutex> g(registry_mutex());
  alloc_registry().push_back({base, bytes});
}
static void registry_remove(uintptr_t base) {
  std::lock_guard<std::mutex> g(registry_mutex());
  auto& reg = alloc_registry();
  for (size_t i = 0; i < reg.size(); ++i)
    if (reg[i].base == base) { reg.erase(reg.begin() + i); break; }
}
// the validator self test checks against its own host arrays instead (this thread only)
static thread_local const std::vector<AllocRec>* g_registry_override = nullptr;

// Host-side bounds check before anything is launched: every element a kernel can touch
// (incl. the 16-byte over-read of K-contiguous GEMM fetches) must lie in ONE registered
// allocation.  GEMM levels go through validate(); every other host-launched kernel that
// writes an arena (conversions, fills, scales, column sets) through the checked launchers
// below — the bf16 shadow refresh once converted past its shadow's end (round 4).
static void check_span(const void* p, int64_t max_index, const char* what, int elem_bytes = 4) {
  if (!p) throw Error{SACMI_ESTATE, std::string("null kernel operand ") + what};
  const uintptr_t a = (uintptr_t)p, e = a + (uintptr_t)(max_index + 1) * elem_bytes;
  if (g_registry_override) {
    for (const AllocRec& r : *g_registry_override)
      if (a >= r.base && e <= r.base + r.bytes) return;
  } else {
    std::lock_guard<std::mutex> g(registry_mutex());
    for (const AllocRec& r : alloc_registry())
      if (a >= r.base && e <= r.base + r.bytes) return;
  }
  throw Error{SACMI_ESTATE, std::string("kernel operand out of bounds: ") + what};
}

// dst[0, n) = bf16(src[0, n)): both spans inside one allocation each
static void check_to_bf16(const unsigned short* dst, const float* src, int64_t n) {
  if (n <= 0) return;
  check_span(dst, n - 1, "bf16 shadow (conversion destination)", 2);
  check_span(src, n - 1, "bf16 shadow source");
}
static void to_bf16_checked(unsigned short* dst, const float* src, int64_t n, hipStream_t s) {
  check_to_bf16(dst, src, n);
  if (n > 0) launch_to_bf16(dst, src, n, s);
}
static void scale_checked(float* p, int64_t n, float f, hipStream_t s) {
  if (n <= 0) return;
  check_span(p, n - 1, "scaled range");
  launch_scale(p, n, f, s);
}
static void fill_checked(float* p, int64_t n, float v, hipStream_t s) {
  if (n <= 0) return;
  check_span(p, n - 1, "filled range");
  launch_fill(p, n, v, s);
}
static void set_column_checked(float* p, int rows, int ld, int col, float v, hipStream_t s) {
  if (rows <= 0) return;
  if (col < 0 || col >= ld) throw Error{SACMI_ESTATE, "column outside its row"};
  check_span(p, (int64_t)(rows - 1) * ld + col, "column set");
  launch_set_column(p, rows, ld, col, v, s);
}

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  void alloc(size_t count) {
    n = count;
    if (count) {
      CHECK_HIP(hipMalloc(&p, count * sizeof(T)));
      // null-stream memset: the context stream is non-blocking, so wait for the
      // zero-fill before anything is enqueued there (init writes the 1-columns).
      CHECK_HIP(hipMemset(p, 0, count * sizeof(T)));
      CHECK_HIP(hipDeviceSynchronize());
      registry_add((uintptr_t)p, count * sizeof(T));
    }
  }
  void release() {
    if (p) registry_remove((uintptr_t)p);
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

struct GraphKey {
  int batch, dev_idx, dev_eps, phase_mask, ring;
  int64_t per_len;   // PER launch geometry depends on the fill
  int reps;          // consecutive updates in one graph
  bool operator<(const GraphKey& o) const {
    return std::tie(batch, dev_idx, dev_eps, phase_mask, ring, per_len, reps) <
           std::tie(o.batch, o.dev_idx, o.dev_eps, o.phase_mask, o.ring, o.per_len, o.reps);
  }
};

}  // namespace sacmi

struct sacmi_ctx {
  sacmi_config cfg{};
  int device = 0;
  hipStream_t own_stream = nullptr;
  // multi-update graphs that cannot ride the next update's sampling along (batch-4096
  // class, prioritized replay): that sampling + gather run on this side stream, forked
  // from / joined into the capture, concurrently with the current update
  hipStream_t side_stream = nullptr;
  std::vector<hipEvent_t> side_ev;
  hipStream_t stream = nullptr;
  bool keep_grads = false;             // SACMI_S_KEEP_GRADS
  int S = 0, A = 0, H = 0, Bm = 0;
  int Kx = 0, Hd = 0, Kp1 = 0, lddh = 0;
  int nh = 2;                      // hidden layers per net (2: networks_model1, 3: model2)
  bool bf16 = false;               // bf16 MFMA operands for the MLP GEMMs
  // layout
  sacmi::Linear q_fc[2][4];        // [net][layer]: layers 0..nh-1 hidden, nh the head
  sacmi::Linear p_fc[3], p_head;   // policy hidden layers 0..nh-1, [mean | log_std]
  int64_t q_begin = 0, q_end = 0, pi_begin = 0, la_idx = 0, total = 0;
  // arenas
  sacmi::DevBuf<float> P, T, G, M, V;
  // bf16 mode: bf16 shadows of P and T (RNE, as every bf16 consumer rounds at staging),
  // kept current by every parameter store; the large-batch level kernels stage their
  // weight operands from them (half the bytes)
  sacmi::DevBuf<unsigned short> Ph, Th;
  sacmi::DevBuf<sacmi::DevScalars> sc;
  // replay
  int ldo = 0, ldact = 0;
  int64_t capacity = 0, len = 0, wpos = 0;
  sacmi::DevBuf<float> obs, act, rew, obs2, done, prio;
  sacmi::DevBuf<uint32_t> mt;      // [2][625]: random / numpy streams
  sacmi::DevBuf<uint32_t> mt_backup;   // [625]: the numpy stream before a PER draw (NaN probs)
  // scratch
  sacmi::DevBuf<int32_t> idx32, idx32b;   // b: second batch set (odd updates of a graph)
  sacmi::DevBuf<int64_t> idx64, idx64b;
  sacmi::DevBuf<float> xq, x2, r, d, eps, cache, logp;
  sacmi::DevBuf<float> xqb, x2b, rb, db;
  // hidden activations per layer: policy on [s2 ; s] (2B rows), the twin critics side by
  // side (B rows x [q1 | q2], each Hd wide with the bias-1 column at H): critic on (s, a),
  // target critics on (s2, a'), updated critics on (s, a~)
  sacmi::DevBuf<float> hp[3], hq[3], hqt[3], hqa[3];
  // backward: critic dh per hidden layer ([nh-1] = the on-the-fly head-layer rows u,
  // stored for the weight gradient), actor-pass critic dh (layers 0..nh-2), policy dh
  sacmi::DevBuf<float> dq, dq4, dhead, dhc[3], dha[3], dhp[3];
  sacmi::DevBuf<float> dotp;       // fc3 dot partials [6 slots][B][nparts]
  sacmi::DevBuf<float> pa;         // dL/da partials [2 * nparts][B][A] (L9 epilogue -> tail)
  sacmi::DevBuf<float> act_h;      // select_action's one-state hidden rows [nh][Hd] (1 at H)
  int pending_step = 0;             // batch of a sacmi_step_launch not yet waited for
  // updates enqueued since the last wait.  A synchronous step's wait (step_finish) ends when
  // the update's done word lands: the fused-Adam levels' block 0 stores it at the START of the
  // last level, behind its losses — "losses ready", NOT "update complete": that level's Adam
  // stores may still be in flight.  Safe because every reader the wait releases is either
  // stream-ordered behind the level (kernels, select_action) or synchronises the stream
  // itself (tensor / scalar / replay reads), and no host staging (push slots, mailbox) is
  // read by that level or its rides (a ride's sampler never takes the mailbox: MailboxArgs
  // go to the update's own sampler launch only)
  bool inflight = false;
  int pending_done = -1;            // the done word before that launch (step_finish)
  // The next single update's minibatch, drawn ahead: a device-sampled single update
  // (sacmi_step / _async / _launch) also runs the NEXT update's random.sample + gather as
  // ride-along workgroups (L12 / L13, as inside multi-update graphs) into the other batch
  // set, saving the MT state it started from in mt_pf.  The next such update of the same
  // batch size consumes it (no sampler / gather of its own); any other call first restores
  // the MT state (pf_settle): the stream is then exactly as if nothing had been drawn ahead.
  sacmi::DevBuf<uint32_t> mt_pf;    // [625]: the random stream before the draw ahead
  bool pf_on = true;                // SACMI_NO_PREFETCH at creation: off
  bool pf_valid = false;            // a drawn-ahead batch waits in set pf_parity
  bool pf_save = false;             // (enqueue_update: the draw ahead saves mt_pf)
  bool pf_touched = false;          // another call since the last single update: draw
                                    //   nothing ahead (a push per update would drop it)
  int pf_parity = 0, pf_B = 0;
  int act_seq = 0;                  // select_action launches (their heads' done word)
  sacmi::DevBuf<float> dw_ws;      // bf16 deep-K weight-gradient split-K partials
  int nparts = 0;
  sacmi::DevBuf<float> lpart_c, lpart_a, ring, lp_part;
  // the sharded data-parallel form's error flags (kDpFlagN): a buffer of their own, outside
  // the critic reduce-scatter's reach (the all-reduce form carries them at G + q_end)
  sacmi::DevBuf<float> dp_flags;
  int ring_slots = 0;
  // act scratch
  int act_rows = 0;
  sacmi::DevBuf<float> ax, ah1, ah2, aeps, acache, alogp, aout;
  // staging
  sacmi::DevBuf<float> stage, per_scr;
  // pinned host staging (hipHostMalloc): transition ingest slots (one in-flight H2D copy
  // each, guarded by an event), act in/out, the scalar block readback
  static constexpr int kPushSlots = 2;
  int push_rows = 0;                        // rows per ingest chunk
  float* push_host[kPushSlots] = {};
  hipEvent_t push_ev[kPushSlots] = {};
  // small pushes (the trainer's row per env step): mapped staging the scatter kernel reads
  // directly (no copy command in front of the next update)
  static constexpr int kPushZcRows = 16;
  float* push_zc_host[kPushSlots] = {};
  float* push_zc_dev[kPushSlots] = {};
  int64_t push_zc_epoch[kPushSlots] = {};  // the stream epoch that read the slot
  int push_zc_slot = 0;
  // the push mailbox (PushMailbox): rows pending for the next synchronous update's sampler
  static constexpr int kMbRows = 16;
  sacmi::PushMailbox* mb_host = nullptr;
  sacmi::PushMailbox* mb_dev = nullptr;
  int mb_pending = 0;               // rows in it
  bool mb_graph = false;            // the update being enqueued consumes them
  // stream epochs: bumped by every zero-copy push; `done_epoch` = the epoch of the last
  // completed wait (step / act / synchronize): every earlier launch that reads host staging
  // has finished (a step's wait: every launch up to its last level's start — see `inflight`),
  // so a staging slot read at an earlier epoch is free without an event (an event record is
  // one more packet between the push and the update behind it)
  int64_t epoch = 1, done_epoch = 0;
  int push_slot = 0;
  float* act_host = nullptr;                // [kActPinned][Kx] states (| 1 | 0..), then [..][A] eps / out
  float* act_host_dev = nullptr;            // the same memory, device-mapped
  int* act_nan_host = nullptr;              // select_action's Normal validation flag (mapped)
  int* act_nan_dev = nullptr;
  float* loss_host = nullptr;               // [4] losses of the last fused update (mapped),
                                            //   word 3: its ErrBits
  float* loss_host_dev = nullptr;
  sacmi::DevScalars* sc_host = nullptr;
  float* ring_host = nullptr;               // [ring_slots][3] loss readback staging
  // PER scratch (replay_kind == PER)
  sacmi::DevBuf<float> per_probs, per_chunk, per_w, per_val;
  sacmi::DevBuf<int64_t> per_q, per_blk, per_idx;
  sacmi::DevBuf<double> per_cdf, per_u, per_uin;
  sacmi::DevBuf<int32_t> per_owner, per_bad;
  std::map<sacmi::GraphKey, hipGraphExec_t> graphs;
  bool use_graphs = true;
  bool G_external = false;
  // native data parallel (sacmi_allreduce_init / sacmi_step_dp)
  ncclComm_t comm = nullptr;
  int dp_world = 0;
  int dp_rank = 0;
  bool dp_loopback = false;   // sacmi_dp_loopback_init: x world in place of the all-reduce
  // sharded optimizer step (ZeRO-1): reduce-scatter the gradients, Adam on this rank's
  // 1/world of the parameters, all-gather the parameters (enqueue_dp)
  bool dp_shard = false;
  bool dp_sharding_now = false;   // enqueue_dp is enqueueing a sharded sequence
  // a sharded step ran at world >= 2: each rank's Adam moments are current on its own chunks
  // only — reading them (tensors, checkpoints) or stepping them (any non-sharded update)
  // raises until sacmi_dp_sync_state gathers them
  bool moments_sharded = false;
  // a loopback one-rank timing run (SACMI_DP_LOOPBACK_ONE_RANK) stepped rank 0's chunks
  // only: the other chunks' moments (and parameters) were never stepped, and no collective
  // can repair that — the moments stay unreadable for the context's lifetime
  bool moments_partial = false;
  std::map<std::tuple<int, int, int64_t>, hipGraphExec_t> dp_graphs;   // (batch, n, PER fill)
  uint64_t act_calls = 0;   // gradient arena owned by the caller (sacmi_attach_grad_arena)
  // profiling (sacmi_profile_step): one event per launch site
  bool prof = false;
  bool prof_collect = false;   // record site names/FLOPs without events
  int prof_site = -1;          // >= 0: enqueue only this launch site
  int site_counter = 0;        // launch sites seen by the current enqueue_update
  std::vector<std::string> prof_names;
  std::vector<double> prof_flops, prof_bytes;
  std::vector<hipEvent_t> prof_events;
  // launch timeline (sacmi_profile_timeline): kTlPerSite * kTlWords words per launch site
  sacmi::tl_word* tl_dev = nullptr;
  int tl_cap = 0, tl_sites = 0;
  sacmi::tl_word* tl_cur = nullptr;   // the current site's slots (null: not recording)
  std::vector<std::string> tl_names;
  std::vector<double> tl_flops, tl_bytes;
};

namespace sacmi {

static void set_err(const Error& e) { g_last_error = e.msg; }

template <class F>
static int guard(F&& f) {
  try {
    f();
    return SACMI_OK;
  } catch (const Error& e) {
    set_err(e);
    return e.code;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return SACMI_EDEVICE;
  }
}

static void destroy_graphs(sacmi_ctx* c) {
  for (auto& kv : c->graphs) (void)hipGraphExecDestroy(kv.second);
  c->graphs.clear();
  for (auto& kv : c->dp_graphs) (void)hipGraphExecDestroy(kv.second);
  c->dp_graphs.clear();
}

// Capture whatever `body` enqueues on the context stream into an instantiated graph (thread-
// local capture mode)
template <class F>
static hipGraphExec_t capture_graph(sacmi_ctx* c, F&& body) {
  hipGraph_t g;
  CHECK_HIP(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
  try {
    body();
  } catch (...) {
    (void)hipStreamEndCapture(c->stream, &g);
    throw;
  }
  CHECK_HIP(hipStreamEndCapture(c->stream, &g));
  hipGraphExec_t ex;
  const hipError_t e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  CHECK_HIP(e);
  return ex;
}

// ---------------------------------------------------------------------------
static void build_layout(sacmi_ctx* c) {
  const int S = c->S, A = c->A, H = c->H;
  // bf16 mode: rows of 8-element multiples, so every bf16 activation / weight-shadow row
  // starts 16-byte aligned (k_fwd16p's LDS-DMA moves 16-byte chunks).  Contexts of the
  // batch-4096 class: whole 128-byte rows of either width (the level kernels stage 128-byte
  // row segments per slab: config 3 1,883-1,889 -> 1,912-1,924 updates/s; config 5 3,331-3,381
  // -> 3,407-3,469, the forward levels 1-2 us each faster, profiles/r06/row_pad_ab and
  // row_pad_bf16_ab); the fp32 batch-256 class takes 32-byte rows (config 2: 16-byte 8,992-9,018,
  // 32-byte 9,043-9,093, 64-byte 8,972-8,979 steps/s, profiles/r06/row_pad_small_ab; 128-byte
  // ones cost 6 %: 8,968-8,993 -> 8,420-8,435)
  const int pad = c->Bm >= 2048 ? (c->bf16 ? 64 : 32) : 8;
  c->Kx = round_up(S + 1 + A, pad);
  c->Hd = round_up(H + 1, pad);
  c->Kp1 = round_up(S + 1, pad);
  c->lddh = round_up(2 * A, 4);
  int64_t off = 0;
  auto take = [&](Linear& l, int n_out, int k_in, int ld, int bias_col, int split, bool align) {
    if (align) off = round_up64(off, 64);
    l.off = off; l.n_out = n_out; l.k_in = k_in; l.ld = ld; l.bias_col = bias_col; l.split = split;
    off += (int64_t)n_out * ld;
  };
  c->q_begin = 0;
  take(c->q_fc[0][0], H, S + A, c->Kx, S, S, true);
  take(c->q_fc[1][0], H, S + A, c->Kx, S, S, false);   // adjacent: one K=2H dL/da GEMM
  for (int l = 1; l < c->nh; ++l) {
    take(c->q_fc[0][l], H, H, c->Hd, H, H, true);
    take(c->q_fc[1][l], H, H, c->Hd, H, H, true);
  }
  take(c->q_fc[0][c->nh], 1, H, c->Hd, H, H, true);
  take(c->q_fc[1][c->nh], 1, H, c->Hd, H, H, true);
  off = round_up64(off, 64);
  c->q_end = off;
  REQUIRE((c->q_end - c->q_begin) % 4 == 0 && c->q_begin % 4 == 0, SACMI_ESTATE, "critic region not float4-aligned");
  // kShardSlack floats between the critic and the actor ranges: the data-parallel step's
  // collective over the critic range reaches past q_end (the sharded form's last chunk, and
  // the error flags of kDpFlagOff) — into this gap, never into the actor's gradients or
  // parameters.  The actor range's reach past `total` lands in the arenas' tail slack.
  off += kShardSlack;
  c->pi_begin = off;
  take(c->p_fc[0], H, S, c->Kp1, S, S, true);
  for (int l = 1; l < c->nh; ++l) take(c->p_fc[l], H, H, c->Hd, H, H, true);
  take(c->p_head, 2 * A, H, c->Hd, H, H, true);
  off = round_up64(off, 64);
  c->la_idx = off;
  c->total = off + 64;
}

static Linear head_part(const sacmi_ctx* c, int which /*0 mean 1 log_std*/) {
  Linear l = c->p_head;
  l.n_out = c->A;
  l.off = c->p_head.off + (int64_t)which * c->A * c->p_head.ld;
  return l;
}

static Linear find_linear(const sacmi_ctx* c, int net, int layer) {
  if (net == SACMI_POLICY) {
    if (layer >= 0 && layer < c->nh) return c->p_fc[layer];
    if (layer == c->nh) return head_part(c, 0);
    if (layer == c->nh + 1) return head_part(c, 1);
  } else if (net >= SACMI_Q1 && net <= SACMI_Q2_TARGET) {
    const int q = (net == SACMI_Q1 || net == SACMI_Q1_TARGET) ? 0 : 1;
    if (layer >= 0 && layer <= c->nh) return c->q_fc[q][layer];
  }
  throw Error{SACMI_EVALUE, "bad (net, layer)"};
}

static void alloc_all(sacmi_ctx* c) {
  const int Bm = c->Bm, S = c->S, A = c->A, H = c->H;
  // P and G carry kShardSlack floats past the layout: the sharded data-parallel step's
  // last chunk of the actor range (chunks of 64-float multiples) reaches past `total`
  c->P.alloc(c->total + kShardSlack); c->G.alloc(c->total + kShardSlack);
  c->M.alloc(c->total); c->V.alloc(c->total);
  c->T.alloc(c->q_end);
  // (the shadows mirror their arenas element for element, P's slack included: refresh_shadows
  // converts P.n elements — round 4 sized Ph at `total` and wrote 16 KB past it)
  if (c->bf16) { c->Ph.alloc(c->P.n); c->Th.alloc(c->T.n); }
  c->sc.alloc(1);
  c->ldo = round_up(S, 4);
  c->ldact = round_up(A, 4);
  const int64_t cap = c->capacity;
  c->obs.alloc((size_t)cap * c->ldo);
  c->obs2.alloc((size_t)cap * c->ldo);
  c->act.alloc((size_t)cap * c->ldact);
  c->rew.alloc(cap);
  c->done.alloc(cap);
  if (c->cfg.replay_kind == SACMI_REPLAY_PER) {
    c->prio.alloc(cap);
    c->per_probs.alloc(cap);
    c->per_q.alloc(cap);
    c->per_cdf.alloc(cap);
    c->per_chunk.alloc(cap / 8192 + 2);
    c->per_blk.alloc(cap / 1024 + 2);
    c->per_bad.alloc(8);
    c->mt_backup.alloc(kMtN + 1);
    c->per_owner.alloc(cap);
    CHECK_HIP(hipMemset(c->per_owner.p, 0xFF, (size_t)cap * 4));   // -1: no writer
    CHECK_HIP(hipDeviceSynchronize());
    c->per_u.alloc(c->Bm + 2);
    c->per_uin.alloc(c->Bm + 2);
    c->per_w.alloc(c->Bm + 2);
  }
  c->mt.alloc(2 * 625);
  c->mt_pf.alloc(625);
  c->pf_on = std::getenv("SACMI_NO_PREFETCH") == nullptr;
  c->per_scr.alloc(16);
  c->idx32.alloc(Bm); c->idx64.alloc(Bm); c->idx32b.alloc(Bm); c->idx64b.alloc(Bm);
  c->xq.alloc((size_t)Bm * c->Kx); c->xqb.alloc((size_t)Bm * c->Kx);
  c->x2.alloc((size_t)2 * Bm * c->Kx); c->x2b.alloc((size_t)2 * Bm * c->Kx);
  c->r.alloc(Bm); c->d.alloc(Bm); c->rb.alloc(Bm); c->db.alloc(Bm);
  const int nh = c->nh;
  for (int l = 0; l < nh; ++l) {
    c->hp[l].alloc((size_t)2 * Bm * c->Hd);
    for (auto* b : {&c->hq[l], &c->hqt[l], &c->hqa[l]}) b->alloc((size_t)Bm * 2 * c->Hd);
    c->dhc[l].alloc((size_t)Bm * 2 * H);
    c->dha[l].alloc((size_t)Bm * 2 * H);
    c->dhp[l].alloc((size_t)Bm * H);
  }
  c->eps.alloc((size_t)2 * Bm * A);
  c->act_h.alloc((size_t)nh * c->Hd);
  c->cache.alloc((size_t)2 * Bm * 3 * A);
  c->logp.alloc((size_t)2 * Bm);
  c->dq.alloc((size_t)2 * Bm + 16);   // + slack: the split-K dW kernels read 4 wide (kernels.hip)
  c->dq4.alloc((size_t)2 * Bm * 4);    // dq one value per 16-byte row (pads stay 0)
  c->nparts = (H + 31) / 32;
  // split-K dW partials (kernels.hip; bf16 only: the fp32 levels measured slower split)
  if (Bm >= 2048) c->dw_ws.alloc((size_t)16 * c->total);   // (split-K partials: bf16 and x6 levels)
  c->dotp.alloc((size_t)6 * Bm * c->nparts);
  c->pa.alloc((size_t)2 * c->nparts * Bm * A);
  c->dhead.alloc((size_t)Bm * c->lddh);
  const int nrb = (Bm + 31) / 32;    // row blocks of the L5 / L9 tiling (loss partials)
  c->lpart_c.alloc((size_t)nrb * 2); c->lpart_a.alloc(nrb);
  c->lp_part.alloc((size_t)2 * ((2 * Bm + 15) / 16) + 2);   // heads: per-workgroup logp sums
  c->dp_flags.alloc(kDpFlagN);
  hipStream_t s = c->stream;
  // constant-1 (bias) columns
  set_column_checked(c->xq.p, Bm, c->Kx, S, 1.f, s);
  set_column_checked(c->x2.p, 2 * Bm, c->Kx, S, 1.f, s);
  set_column_checked(c->xqb.p, Bm, c->Kx, S, 1.f, s);
  set_column_checked(c->x2b.p, 2 * Bm, c->Kx, S, 1.f, s);
  for (int l = 0; l < nh; ++l) {
    set_column_checked(c->hp[l].p, 2 * Bm, c->Hd, H, 1.f, s);
    set_column_checked(c->act_h.p + (size_t)l * c->Hd, 1, c->Hd, H, 1.f, s);
    for (auto* b : {&c->hq[l], &c->hqt[l], &c->hqa[l]}) {
      set_column_checked(b->p, Bm, 2 * c->Hd, H, 1.f, s);
      set_column_checked(b->p, Bm, 2 * c->Hd, c->Hd + H, 1.f, s);
    }
  }
  CHECK_HIP(hipStreamSynchronize(s));
}

static void upload_scalars(sacmi_ctx* c, const DevScalars& h) {
  *c->sc_host = h;
  CHECK_HIP(hipMemcpyAsync(c->sc.p, c->sc_host, sizeof(h), hipMemcpyHostToDevice, c->stream));
  CHECK_HIP(hipStreamSynchronize(c->stream));
}
static void mb_flush(sacmi_ctx* c);
static MailboxArgs mailbox_args(sacmi_ctx* c);
static DevScalars download_scalars(sacmi_ctx* c) {
  mb_flush(c);
  CHECK_HIP(hipMemcpyAsync(c->sc_host, c->sc.p, sizeof(DevScalars), hipMemcpyDeviceToHost, c->stream));
  CHECK_HIP(hipStreamSynchronize(c->stream));
  return *c->sc_host;
}

constexpr int kActPinned = 64;   // select_action rows served from pinned staging

static void alloc_pinned(sacmi_ctx* c) {
  const int S = c->S, A = c->A;
  c->push_rows = 1024;
  const size_t row = (size_t)2 * S + A + 2;
  for (int i = 0; i < sacmi_ctx::kPushSlots; ++i) {
    CHECK_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->push_host[i]), row * c->push_rows * 4,
                            hipHostMallocDefault));
    CHECK_HIP(hipEventCreateWithFlags(&c->push_ev[i], hipEventDisableTiming));
  }
  c->stage.alloc(row * c->push_rows);
  CHECK_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->mb_host), sizeof(PushMailbox) + row * sacmi_ctx::kMbRows * 4,
                          hipHostMallocMapped | hipHostMallocCoherent));
  CHECK_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->mb_dev), c->mb_host, 0));
  c->mb_host->n = 0;
  for (int i = 0; i < sacmi_ctx::kPushSlots; ++i) {
    CHECK_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->push_zc_host[i]), row * sacmi_ctx::kPushZcRows * 4,
                            hipHostMallocMapped | hipHostMallocCoherent));
    CHECK_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->push_zc_dev[i]), c->push_zc_host[i], 0));
  }
  // select_action staging: fine-grained (coherent) and mapped, so the kernels read the
  // states and write the actions in place (no copy commands on the env-rate path)
  // (the state rows in fc1's input layout, the ones column set here once: fc1 reads them
  // as its A operand in place)
  const size_t act_floats = (size_t)kActPinned * (c->Kx + 2 * A);
  CHECK_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->act_host), act_floats * 4 + 16,
                          hipHostMallocMapped | hipHostMallocCoherent));
  CHECK_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->act_host_dev), c->act_host, 0));
  std::memset(c->act_host, 0, act_floats * 4 + 16);
  for (int i = 0; i < kActPinned; ++i) c->act_host[(size_t)i * c->Kx + S] = 1.f;
  registry_add((uintptr_t)c->act_host_dev, act_floats * 4);
  c->act_nan_host = reinterpret_cast<int*>(c->act_host + act_floats);
  c->act_nan_dev = reinterpret_cast<int*>(c->act_host_dev + act_floats);
  c->act_nan_host[1] = 0;                        // (select_action's done word: sacmi_act)
  // update_parameters' three losses, stored here by the fused Adam levels' block 0: the
  // synchronous step reads them after the stream sync, no copy command
  CHECK_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->loss_host), 32,
                          hipHostMallocMapped | hipHostMallocCoherent));
  CHECK_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->loss_host_dev), c->loss_host, 0));
  std::memset(c->loss_host, 0, 32);             // (word 4: the done word, step_finish)
  CHECK_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->sc_host), sizeof(DevScalars),
                          hipHostMallocDefault));
  CHECK_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->ring_host), (size_t)c->ring_slots * 12,
                          hipHostMallocDefault));
}

static void free_pinned(sacmi_ctx* c) {
  for (int i = 0; i < sacmi_ctx::kPushSlots; ++i) {
    if (c->push_ev[i]) (void)hipEventDestroy(c->push_ev[i]);
    if (c->push_host[i]) (void)hipHostFree(c->push_host[i]);
    c->push_ev[i] = nullptr;
    c->push_host[i] = nullptr;
    if (c->push_zc_host[i]) (void)hipHostFree(c->push_zc_host[i]);
    if (i == 0 && c->mb_host) (void)hipHostFree(c->mb_host);
    if (i == 0) { c->mb_host = nullptr; c->mb_dev = nullptr; }
    c->push_zc_host[i] = nullptr;
    c->push_zc_dev[i] = nullptr;
  }
  if (c->act_host_dev) registry_remove((uintptr_t)c->act_host_dev);
  if (c->act_host) (void)hipHostFree(c->act_host);
  if (c->sc_host) (void)hipHostFree(c->sc_host);
  if (c->ring_host) (void)hipHostFree(c->ring_host);
  c->ring_host = nullptr;
  c->act_host = nullptr;
  c->act_host_dev = nullptr;
  c->act_nan_host = nullptr;
  c->act_nan_dev = nullptr;
  if (c->loss_host) (void)hipHostFree(c->loss_host);
  c->loss_host = nullptr;
  c->loss_host_dev = nullptr;
  c->sc_host = nullptr;
}

// ---------------------------------------------------------------------------
// one update, enqueued on c->stream.  phase_mask bit p enables phase p.
static GemmDesc gd(const float* A, int lda, int a_kc, const float* B, int ldb, int b_kc,
                   float* C, int ldc, int M, int N, int K, int epi = EPI_STORE,
                   const float* aux = nullptr, int ldaux = 0, int adam_step = 0) {
  GemmDesc d{};
  d.adam_step = adam_step;
  d.A = A; d.lda = lda; d.a_kc = a_kc;
  d.B = B; d.ldb = ldb; d.b_kc = b_kc;
  d.C = C; d.ldc = ldc; d.M = M; d.N = N; d.K = K; d.epi = epi; d.aux = aux; d.ldaux = ldaux;
  d.rs_col = -1;
  return d;
}

// forward GEMM of a hidden layer (K = H): the bias column H of W~ is added in the
// epilogue instead of riding in the K loop (keeps K = 32 chunks, balanced over 16 waves)
static GemmDesc gd_fwd_h(const float* A, int lda, const float* W, int ldw, float* C, int ldc,
                         int M, int N, int H) {
  GemmDesc d = gd(A, lda, 1, W, ldw, 1, C, ldc, M, N, H, EPI_RELU);
  d.bias = W + H;
  d.bias_ld = ldw;
  return d;
}

// weight gradient of a hidden layer: N = H columns by MFMA, the bias column (H) as the
// row sum of dY (no ninth 64-wide tile for one column)
static GemmDesc gd_dw_h(const float* dY, int ldy, const float* X, int ldx, float* C, int ldc,
                        int M, int H, int B, int epi, int step) {
  GemmDesc d = gd(dY, ldy, 0, X, ldx, 0, C, ldc, M, H, B, epi, nullptr, 0, step);
  d.rs_col = H;
  return d;
}

// Host-side bounds check of one GEMM before it is ever launched (check_span, defined with
// the allocation registry above): every element the kernel can touch (incl. the 16-byte
// over-read of K-contiguous fetches) must lie in one registered allocation, and
// vector-loaded operands must be 16-byte aligned.

static void validate(const GemmDesc& d) {
  if (d.M <= 0 || d.N <= 0 || d.K <= 0) throw Error{SACMI_ESTATE, "empty GEMM"};
  const int64_t klast = ((int64_t)(d.K - 1) / 4) * 4 + 3;
  // element bytes: bf16 activation operands (act16) are read 4 elements = 8 bytes at a time
  const int ea = d.a16 ? 2 : 4, eb = d.b16 ? 2 : 4, ec = d.c16 ? 2 : 4, ex = d.x16 ? 2 : 4;
  if (d.a_kc) {
    if (((uintptr_t)d.A & (4 * ea - 1)) || (d.lda & 3)) throw Error{SACMI_ESTATE, "A misaligned"};
    check_span(d.A, (int64_t)(d.M - 1) * d.lda + klast, "A", ea);
  } else {
    // MN-contiguous operands are read 4 columns wide from a 4-aligned start (the split-K
    // dW kernels): the span covers the last such group
    REQUIRE(!d.a16, SACMI_ESTATE, "bf16 A operands are K-contiguous");
    check_span(d.A, (int64_t)(d.K - 1) * d.lda + ((d.M - 1) & ~3) + 3, "A", ea);
  }
  if (d.b_kc) {
    REQUIRE(!d.b16, SACMI_ESTATE, "bf16 B operands are row-contiguous (weight-gradient X)");
    if (((uintptr_t)d.B & 15) || (d.ldb & 3)) throw Error{SACMI_ESTATE, "B misaligned"};
    check_span(d.B, (int64_t)(d.N - 1) * d.ldb + klast, "B");
  } else {
    if (d.b16 && (((uintptr_t)d.B & 7) || (d.ldb & 3))) throw Error{SACMI_ESTATE, "B misaligned"};
    check_span(d.B, (int64_t)(d.K - 1) * d.ldb + ((d.N - 1) & ~3) + 3, "B", eb);
  }
  if (d.c16) REQUIRE(d.rs_col < 0 && d.epi < EPI_ADAM && ((uintptr_t)d.C & 3) == 0 && d.N % 2 == 0 && d.ldc % 2 == 0,
                     SACMI_ESTATE, "bf16 C: a forward output of even width");
  if (d.C) check_span(d.C, (int64_t)(d.M - 1) * d.ldc + std::max(d.N - 1, d.rs_col), "C", ec);
  if (d.bias) check_span(d.bias, (int64_t)(d.N - 1) * d.bias_ld, "bias");
  REQUIRE(!(d.bias && d.epi == EPI_MASK), SACMI_ESTATE, "GEMM epilogue: bias and mask are exclusive");
  if (d.axk) {
    REQUIRE(d.axk == 1, SACMI_ESTATE, "unknown A transform");
    REQUIRE(d.a_kc && !d.b_kc && d.ax_w, SACMI_ESTATE, "A transform needs a K-contiguous A and w");
    check_span(d.ax_w, d.K - 1, "ax_w");
    if (d.ax_out) {
      REQUIRE(d.K % 4 == 0 && d.ax_ld % 4 == 0, SACMI_ESTATE, "ax_out rows must be float4-aligned");
      check_span(d.ax_out, (int64_t)(d.M - 1) * d.ax_ld + d.K - 1, "ax_out");
    }
  }
  if (d.a_ksc) {
    REQUIRE(!d.a_kc && d.axk != 1, SACMI_ESTATE, "a_ksc needs a row-contiguous A operand");
    check_span(d.a_ksc, d.K - 1, "a_ksc");
  }
  if (d.dotp) {
    check_span(d.dotw, d.N, "dotw");      // w3 and the head bias w3~[N]
    check_span(d.dotp, (int64_t)(d.M - 1) * d.dotp_ld + (d.N - 1) / 32, "dotp");
  }
  if (d.epi == EPI_MASK) check_span(d.aux, (int64_t)(d.M - 1) * d.ldaux + d.N - 1, "aux", ex);
  else REQUIRE(!d.x16, SACMI_ESTATE, "bf16 mask source without a mask epilogue");
}

// The level-wide operands launch_gemm may route a level's work through, checked once the
// level is complete (right before its launch):
//   * Bh, the bf16 shadow of a weight operand: k_fwd16 / k_axk16 / k_gemm<bf16> read it
//     over exactly B's element range (2 bytes per element, 8-byte vector loads);
//   * ws, the split-K partial workspace: k_dw_part16 writes and k_dw_fin reads
//     ws[0, ws_floats) at most (dw_split_plan never plans past ws_floats), so the claimed
//     capacity must lie inside one allocation.
static void validate_batch(const GemmBatch& b) {
  for (int i = 0; i < b.count; ++i) {
    const GemmDesc& d = b.d[i];
    if (!d.Bh) continue;
    REQUIRE(((uintptr_t)d.Bh & 7) == 0, SACMI_ESTATE, "Bh misaligned");
    const int64_t klast = ((int64_t)(d.K - 1) / 4) * 4 + 3;
    const int64_t last = d.b_kc ? (int64_t)(d.N - 1) * d.ldb + klast
                                : (int64_t)(d.K - 1) * d.ldb + ((d.N - 1) & ~3) + 3;
    check_span(d.Bh, last, "Bh (bf16 shadow)", 2);
  }
  if (b.ws) {
    REQUIRE(b.ws_floats > 0 && ((uintptr_t)b.ws & 15) == 0, SACMI_ESTATE, "bad split-K workspace");
    check_span(b.ws, b.ws_floats - 1, "ws (split-K workspace)");
  } else {
    REQUIRE(b.ws_floats == 0, SACMI_ESTATE, "split-K workspace capacity without a workspace");
  }
}

struct Level {
  GemmBatch b{};
  void add(const GemmDesc& d0) {
    validate(d0);
    if (b.count >= kMaxGemms) throw Error{SACMI_ESTATE, "too many GEMMs in one level"};
    if (b.count && (b.d[0].epi >= EPI_ADAM) != (d0.epi >= EPI_ADAM))
      throw Error{SACMI_ESTATE, "a GEMM level is either all fused-Adam or all plain"};
    GemmDesc d = d0;
    const int tm = (d.M + 31) / 32, tn = (d.N + 31) / 32;
    d.tiles_n = tn;
    d.tile_begin = b.total_tiles;
    b.total_tiles += tm * tn;
    b.d[b.count++] = d;
  }
};

static double level_flops(const GemmBatch& b) {
  double f = 0;
  for (int i = 0; i < b.count; ++i) {
    f += 2.0 * b.d[i].M * (double)b.d[i].N * b.d[i].K;
    if (b.d[i].pa_out) f += 2.0 * b.d[i].M * (double)b.d[i].N * b.d[i].pa_A;   // dL/da partials
  }
  return f;
}

// Algorithmic bytes of one level: each operand read once, the output written once, the
// epilogue's own operands (ReLU-mask source, bias) read once, and for a fused Adam the
// optimizer state (param, exp_avg, exp_avg_sq [+ target]) read and written once.
static double level_bytes(const GemmBatch& b) {
  double n = 0;    // bytes
  for (int i = 0; i < b.count; ++i) {
    const GemmDesc& d = b.d[i];
    const double out = (double)d.M * (d.N + (d.rs_col >= 0 ? 1 : 0));
    n += (double)d.M * d.K * (d.a16 ? 2 : 4) + (double)d.N * d.K * (d.b16 ? 2 : 4);
    if (d.epi >= EPI_ADAM) {
      n += 4.0 * (out * (d.epi == EPI_ADAM_POLYAK ? 8 : 6) + (b.adam.G ? out : 0));
    } else {
      n += out * (d.c16 ? 2 : 4) + (d.epi == EPI_MASK ? out * (d.x16 ? 2 : 4) : 0) + (d.bias ? 4.0 * d.N : 0);
    }
    if (d.pa_out) n += 4.0 * ((double)d.N * d.pa_A + (double)d.M * ((d.N + 31) / 32) * d.pa_A);
  }
  return n;
}

// profiling mark: records an event BEFORE the launch it names
// Hook in front of every launch site of the update.  Returns whether the site's
// kernels are enqueued: always, except in site-isolation mode (prof_site >= 0), where
// only site number prof_site runs (sacmi_profile_sites).
static bool mark(sacmi_ctx* c, const char* name, double flops = 0, double bytes = 0) {
  const int site = c->site_counter++;
  c->tl_cur = nullptr;
  if (c->tl_dev) {
    if (c->tl_sites >= c->tl_cap) throw Error{SACMI_ESTATE, "timeline buffer full"};
    c->tl_cur = c->tl_dev + (size_t)c->tl_sites++ * kTlPerSite * kTlWords;
    c->tl_names.push_back(name);
    c->tl_flops.push_back(flops);
    c->tl_bytes.push_back(bytes);
  }
  if (c->prof || c->prof_collect) {
    c->prof_names.push_back(name);
    c->prof_flops.push_back(flops);
    c->prof_bytes.push_back(bytes);
  }
  if (c->prof) {
    hipEvent_t e;
    CHECK_HIP(hipEventCreate(&e));
    CHECK_HIP(hipEventRecord(e, c->stream));
    c->prof_events.push_back(e);
  }
  return c->prof_site < 0 || site == c->prof_site;
}

struct BatchBufs;
static PerArgs per_args(sacmi_ctx* c, int k, int gen_u, const BatchBufs* bb = nullptr);
static PerArgs per_args_impl(sacmi_ctx* c, int k, int gen_u, int32_t* idx32, int64_t* idx64) {
  PerArgs a{};
  a.prio = c->prio.p; a.len = c->len; a.cap = c->capacity; a.alpha = (float)c->cfg.per_alpha;
  a.probs = c->per_probs.p; a.chunk_sums = c->per_chunk.p; a.q = c->per_q.p;
  a.block_sums = c->per_blk.p; a.bad = c->per_bad.p; a.cdf = c->per_cdf.p;
  a.mt = c->mt.p + 625; a.gen_u = gen_u; a.u = c->per_uin.p; a.u_scratch = c->per_u.p;
  a.k = k; a.sc = c->sc.p; a.beta_start = c->cfg.per_beta_start;
  a.beta_frames = c->cfg.per_beta_frames; a.idx32 = idx32; a.idx_out = idx64;
  a.w_out = c->per_w.p;
  a.err = &c->sc.p->err; a.mt_backup = c->mt_backup.p;
  a.skip_on_err = 1;       // update graphs; the host API (sacmi_per_sample) clears it
  return a;
}

// The minibatch buffers of one update (indices, gathered rows, r, d): set 0 is the one
// every single update and the host-side APIs use; set 1 serves the odd updates of a
// multi-update graph, so that the next update's gather can run while this one still
// reads its rows.
struct BatchBufs {
  int32_t* idx32; int64_t* idx64; float* xq; float* x2; float* r; float* d;
};
static BatchBufs batch_bufs(sacmi_ctx* c, int parity) {
  if (parity == 0) return BatchBufs{c->idx32.p, c->idx64.p, c->xq.p, c->x2.p, c->r.p, c->d.p};
  return BatchBufs{c->idx32b.p, c->idx64b.p, c->xqb.p, c->x2b.p, c->rb.p, c->db.p};
}
// the prioritized sampler writes the indices of batch set bb (set 0 by default)
static PerArgs per_args(sacmi_ctx* c, int k, int gen_u, const BatchBufs* bb) {
  return per_args_impl(c, k, gen_u, bb ? bb->idx32 : c->idx32.p, bb ? bb->idx64 : c->idx64.p);
}

static int sample_setsize(int k) {   // random.py:486-488
  int setsize = 21;
  if (k > 5) setsize += (int)std::pow(4.0, std::ceil(std::log((double)k * 3) / std::log(4.0)));
  return setsize;
}

static MtSampleArgs mt_args(sacmi_ctx* c, int B, const BatchBufs& bb) {
  MtSampleArgs m{};
  m.mt = c->mt.p; m.sc = c->sc.p; m.k = B;
  m.setsize = sample_setsize(B); m.idx_out = bb.idx32; m.idx64_out = bb.idx64;
  m.skip_on_err = 1;       // update graphs; the host API (sacmi_sample_indices) clears it
  return m;
}

// bf16 activations (act16): in bf16 mode at the batch-4096 class, every activation the
// update produces (hidden layers, minibatch rows, the sampled actions) is stored as bf16
// — every consumer rounds its MFMA operands to bf16 anyway, the ReLU masks read signs only,
// and the critic head dots use the unrounded epilogue values — halving the activation
// bytes written and staged.  Only the policy heads read values outside an MFMA operand:
// they see h rounded (the oracle's emulation rounds the same operand).  Needs every level
// on the batch-4096-class kernels (k_fwd16 / k_axk16 / k_dw_part16: launch_gemm refuses
// anything else), so batch >= 4096 and hidden a multiple of 128, >= 512.
static bool act16_on(const sacmi_ctx* c, int B) {
  return c->bf16 && B >= 4096 && c->H >= 512 && c->H % 128 == 0;
}

static GatherArgs gather_args(sacmi_ctx* c, int B, const BatchBufs& bb, bool per) {
  GatherArgs g{};
  g.idx = bb.idx32; g.obs = c->obs.p; g.act = c->act.p; g.rew = c->rew.p; g.obs2 = c->obs2.p;
  g.done = c->done.p; g.ldo = c->ldo; g.lda_ = c->ldact; g.capacity = c->capacity;
  g.sc = c->sc.p; g.S = c->S; g.A = c->A; g.B = B; g.xq = bb.xq; g.x2 = bb.x2; g.ldx = c->Kx;
  g.r = bb.r; g.d = bb.d;
  g.by_slot = per ? 1 : 0;
  g.x16 = act16_on(c, B) ? 1 : 0;
  return g;
}

// Can the next update's sampling + gather ride along in this update's launches?
static bool ride_possible(sacmi_ctx* c, int B) {
  return c->cfg.replay_kind == SACMI_REPLAY_UNIFORM &&
         mt_sample_lds_words(mt_sample_tbl_log2(B), sample_setsize(B)) * 4 <= kRideLdsBytes;
}

// ... or, in a fused multi-update graph whose batch is too large for that (the batch-4096
// class, bf16): the sampler (compact table, 256 threads) rides in L6's split-K kernel
// (k_dw_part16, 440 of 512 slots at config 5) and the gather in L12 (k_axk16, 256 of 512
// slots; a row a wave, every load before any store).  (The gather in L10 measured no
// overlap: k_gemm_sample_bwd's 1024-thread workgroups fit one per CU)
static bool ride_b_possible(sacmi_ctx* c, int B) {
  return c->cfg.replay_kind == SACMI_REPLAY_UNIFORM && c->bf16 && B >= 2048 &&
         mt_sample_lds_words(mt_sample_tbl_log2(B, true), sample_setsize(B)) * 4 <=
             (size_t)kDw16LdsBytes;
}

// One update's minibatch: device sampling (random.sample or the prioritized sampler, unless
// the indices were staged from the host) + gather, into batch set `parity`, on stream s.
// `tag` names the launch sites ("" for the update's own, "_next" on the side stream);
static void enqueue_sample_gather(sacmi_ctx* c, int B, int parity, bool dev_idx, hipStream_t s,
                                  const char* tag = "") {
  const BatchBufs bb = batch_bufs(c, parity);
  const bool per = c->cfg.replay_kind == SACMI_REPLAY_PER;
  const std::string t(tag);
  if (dev_idx && per) {
    if (mark(c, ("per_sample" + t).c_str())) {
      PerArgs pa = per_args(c, B, 1, &bb);
      pa.tl = c->tl_cur;
      launch_per_sample(pa, s);
    }
  } else if (dev_idx) {
    if (mark(c, ("mt_sample" + t).c_str())) {
      MtSampleArgs ma = mt_args(c, B, bb);
      ma.tl = c->tl_cur;
      const MailboxArgs mb = mailbox_args(c);
      launch_mt_sample(ma, s, c->mb_graph && t.empty() ? &mb : nullptr);
    }
  }
  if (mark(c, ("gather" + t).c_str())) {
    GatherArgs ga = gather_args(c, B, bb, per);
    ga.tl = c->tl_cur;
    launch_gather(ga, s);
  }
}

// The data-parallel Adam step of one range over the whole range: critic (+ Polyak, + the q
// losses) or actor (+ the alpha step, policy loss, loss ring), grad_scale = 1/world
static AdamArgs dp_adam_args(sacmi_ctx* c, bool critic, int B, float grad_scale, bool use_ring) {
  AdamArgs ad{};
  ad.p = c->P.p; ad.g = c->G.p; ad.m = c->M.p; ad.v = c->V.p;
  ad.nseg = 0;
  const int nh = c->nh, nb = (B + 31) / 32;
  auto seg = [&](const Linear& l, int idx) {
    REQUIRE(ad.nseg < kMaxAdamSegs, SACMI_ESTATE, "too many Adam segments");
    ad.seg[ad.nseg++] = AdamSeg{l.off, l.numel_padded(), idx};
  };
  if (critic) {
    for (int layer = 0; layer <= nh; ++layer)
      for (int i = 0; i < 2; ++i) seg(c->q_fc[i][layer], i == 0 ? 1 : 2);
  } else {
    for (int l = 0; l <= nh; ++l) seg(l < nh ? c->p_fc[l] : c->p_head, 0);
  }
  ad.total = 0;
  for (int i = 0; i < ad.nseg; ++i) {
    REQUIRE(ad.seg[i].n % 4 == 0 && ad.seg[i].off % 4 == 0, SACMI_ESTATE, "Adam segment not float4-aligned");
    ad.total += ad.seg[i].n;
  }
  ad.lr = (float)c->cfg.lr; ad.beta1 = 0.9f; ad.beta2 = 0.999f; ad.eps = 1e-8f; ad.grad_scale = grad_scale;
  ad.sc = c->sc.p; ad.n_part = nb; ad.loss_div = (float)B;
  // the bf16 shadows of the updated parameters / targets (read by the bf16 level kernels)
  ad.ph = c->Ph.p; ad.tgth = c->Th.p;
  if (critic) {
    ad.tgt = c->T.p; ad.tgt_base = c->q_begin;
    ad.tau = (float)c->cfg.tau; ad.step_offset = 1;
    ad.loss_part = c->lpart_c.p; ad.loss_slot0 = 0; ad.n_losses = 2;
    ad.log_alpha_idx = -1; ad.auto_entropy = 0;
    ad.err_skip = kErrSkipAll; ad.err_nopolyak = kErrActLike;
    // every rank's error flags, summed by the critic gradient collective (kDpFlagN): past the
    // critic range (all-reduce form), or in their own buffer (sharded form)
    ad.err_flags = c->dp_sharding_now ? c->dp_flags.p : c->G.p + c->q_end;
  } else {
    ad.tgt = nullptr; ad.tau = 0.f; ad.step_offset = 0;
    ad.loss_part = c->lpart_a.p; ad.loss_slot0 = 2; ad.n_losses = 1;
    ad.log_alpha_idx = c->la_idx; ad.auto_entropy = c->cfg.auto_entropy;
    ad.loss_ring = use_ring ? c->ring.p : nullptr; ad.ring = c->ring_slots;
    ad.err_skip = ~0; ad.err_nopolyak = 0;
  }
  return ad;
}

// The Adam moments are whole on this rank: every update that steps them from this rank's M, V
// (any update but the sharded data-parallel sequence) needs it.  (A loopback one-rank timing
// context, moments_partial, may go on stepping: its state is a timing artifact either way;
// reads of it raise, require_moments_readable.)
static void require_moments_whole(const sacmi_ctx* c) {
  REQUIRE(!c->moments_sharded, SACMI_ESTATE,
          "the Adam moments are sharded across the data-parallel ranks (sharded optimizer step): "
          "call sacmi_dp_sync_state on every rank before reading or writing them");
}
static void require_moments_readable(const sacmi_ctx* c) {
  REQUIRE(!c->moments_partial, SACMI_ESTATE,
          "the Adam moments of this context were left partly stepped by a loopback one-rank timing "
          "run (SACMI_DP_LOOPBACK_ONE_RANK: only rank 0's chunks were stepped); they cannot be read "
          "any more");
  require_moments_whole(c);
}

// parity: which batch buffer set this update uses; have_batch: its indices and rows
// were produced by the previous update's ride-along work; ride_next: produce the next
// update's (into the other set) inside this update's L11 / L13 launches.
static void enqueue_update(sacmi_ctx* c, int B, int dev_idx, int dev_eps, int phase_mask,
                           float grad_scale, bool use_ring, int parity = 0,
                           bool have_batch = false, bool ride_next = false) {
  hipStream_t s = c->stream;
  // every Adam step of this update but the sharded data-parallel form's own (enqueue_dp_sharded
  // steps this rank's chunks) reads and writes the whole of M, V
  if ((phase_mask & 6) && !c->dp_sharding_now) require_moments_whole(c);
  c->site_counter = 0;
  const BatchBufs bb = batch_bufs(c, parity);
  // where the next update's sampling + gather ride: L12 / L13 (placement A, batch <= ~2k,
  // any phase split) or L6 / L10 (placement B, fused updates of the batch-4096 class)
  const bool ride_b = ride_next && !ride_possible(c, B);
  REQUIRE(!ride_b || (phase_mask == 7 && ride_b_possible(c, B)), SACMI_ESTATE,
          "no ride-along placement for this batch");
  const int S = c->S, A = c->A, H = c->H, Kx = c->Kx, Hd = c->Hd;
  float* P = c->P.p;
  float* G = c->G.p;
  const float* T = c->T.p;
  const int nb = (B + 31) / 32;     // loss partials: one per 32-row block of L5 / L9
  auto W = [&](const Linear& l) { return P + l.off; };
  // fc3 dot partials: slot 0/1 q1/q2 (L2), 2/3 target q1/q2 (L4), 4/5 updated q1/q2 (L8)
  auto dotp = [&](int slot) { return c->dotp.p + (size_t)slot * B * c->nparts; };
  auto with_dot = [&](GemmDesc g, const float* w3, int slot) {
    g.dotw = w3; g.dotp = dotp(slot); g.dotp_ld = c->nparts;
    return g;
  };
  auto Wt = [&](const Linear& l) { return T + (l.off - c->q_begin); };
  auto dW = [&](const Linear& l) { return G + l.off; };
  const Linear(&q)[2][4] = c->q_fc;
  const int nh = c->nh, L = nh - 1;   // L: the last hidden layer (its head is layer nh)
  auto shadow = [&](const float* b) -> const unsigned short* {
    if (!c->Ph.p || !b) return nullptr;
    if (b >= c->P.p && b < c->P.p + c->P.n) return c->Ph.p + (b - c->P.p);
    if (b >= c->T.p && b < c->T.p + c->T.n) return c->Th.p + (b - c->T.p);
    return nullptr;
  };
  // activation buffers: element offsets in the update's activation format
  const bool act16 = act16_on(c, B);
  const int a16 = act16 ? 1 : 0;
  auto E = [&](float* base, size_t off) -> float* {
    return act16 ? reinterpret_cast<float*>(reinterpret_cast<unsigned short*>(base) + off) : base + off;
  };
  auto fw = [&](GemmDesc g) { g.a16 = a16; g.c16 = a16; return g; };        // forward level
  auto dh = [&](GemmDesc g) { g.x16 = a16; g.a16 = g.axk == 1 ? a16 : 0; return g; };   // dh level
  auto dwx = [&](GemmDesc g) { g.b16 = a16; return g; };                     // dW level (X)
  auto run = [&](Level& lv, const std::string& name) {
    lv.b.bf16 = c->bf16 ? 1 : 0;
    for (int i = 0; i < lv.b.count; ++i) lv.b.d[i].Bh = shadow(lv.b.d[i].B);
    lv.b.ws = c->dw_ws.p;
    lv.b.ws_floats = (int64_t)c->dw_ws.n;
    validate_batch(lv.b);
    if (mark(c, name.c_str(), level_flops(lv.b), level_bytes(lv.b))) {
      lv.b.tl = c->tl_cur;
      launch_gemm(lv.b, s);
    }
  };

  // fused updates whose policy dhp1 level (L12) leaves CUs idle on k_gemm: Polyak rides there
  // (data-parallel phase 1, both optimizer forms: the critic Adam before L7 leaves the
  // targets alone — sharded: enqueue_dp's chunk Adam, all-reduce: the one below)
  const bool polyak_ride = (phase_mask == 7 || (phase_mask & 2)) &&
                           !act16 && (int64_t)((B + 31) / 32) * ((H + 31) / 32) <= 192;
  if (phase_mask & 1) {
    if (!have_batch)   // (have_batch: the previous update's rides / side stream produced them)
      enqueue_sample_gather(c, B, parity, dev_idx != 0, s);

    // heads + sample for both stacks (networks_model1.py:78-99)
    HeadSampleArgs hs{};
    hs.h = c->hp[L].p; hs.Wh = W(c->p_head); hs.rows = 2 * B; hs.A = A; hs.K = H;
    hs.ldh = Hd; hs.ldw = Hd; hs.eps = c->eps.p; hs.gen_eps = dev_eps; hs.seed = c->cfg.seed;
    hs.sc = c->sc.p; hs.act = E(bb.x2, (size_t)S + 1); hs.ldact = Kx; hs.logp = c->logp.p;
    hs.h16 = a16;
    hs.cache = c->cache.p;
    hs.scale = (float)((c->cfg.action_high - c->cfg.action_low) / 2);
    hs.bias = (float)((c->cfg.action_high + c->cfg.action_low) / 2);
    hs.logp_part = c->lp_part.p; hs.split_row = B;    // sums of log pi(a~|s) for dL/dlog_alpha
    // Normal validation of policy.sample(next_state) / policy.sample(state) (sac_imp.py:89,116)
    hs.nan_flag = &c->sc.p->err; hs.nan_bit_lo = ERR_NAN_TGT; hs.nan_bit_hi = ERR_NAN_ACT;
    const bool fuse = phase_mask == 7;     // single-GPU update: Adam in the dW epilogues
    // L5: dh[L-1] = (dh[L] W[L]) * relu'(h[L-1]), with the target / critic-loss rows folded
    // in: the row prologue finishes q1, q2, qt1, qt2 from the dot partials and gives
    // dq_i = 2 (q_i - q^) / B; the A operand dh[L] = dq * w_head * [h[L] > 0] is formed
    // from h[L] on the fly (its coefficient-free rows u stored once by the column-tile-0
    // workgroups, for the weight gradient of layer L)
    Level l5;
    for (int i = 0; i < 2; ++i) {
      GemmDesc g = gd(E(c->hq[L].p, (size_t)i * Hd), 2 * Hd, 1, W(q[i][L]), Hd, 0, c->dhc[L - 1].p + i * H, 2 * H,
                      B, H, H, EPI_MASK, E(c->hq[L - 1].p, (size_t)i * Hd), 2 * Hd);
      g.axk = 1; g.ax_slot = i; g.ax_w = W(q[i][nh]); g.ax_ld = 2 * H;
      g.ax_out = c->dhc[L].p + i * H;   // the coefficient-free rows u (layer L's weight gradient)
      l5.add(dh(g));
    }
    {
      RowsFuse& rf = l5.b.rows;
      rf.kind = 1; rf.part = dotp(0); rf.nparts = c->nparts; rf.B = B;
      rf.r = bb.r; rf.d = bb.d; rf.logp = c->logp.p; rf.logp_a = c->logp.p + B;
      rf.gamma = (float)c->cfg.gamma;
      rf.sc = c->sc.p; rf.dq = c->dq.p; rf.dq4 = c->dq4.p; rf.loss_part = c->lpart_c.p;
    }
    // L1: policy fc1 on [s2 ; s] (2B rows), critic fc1 (twin) on [s|1|a]
    Level l1;
    l1.add(fw(gd(bb.x2, Kx, 1, W(c->p_fc[0]), c->p_fc[0].ld, 1, c->hp[0].p, Hd, 2 * B, H, S + 1, EPI_RELU)));
    for (int i = 0; i < 2; ++i)
      l1.add(fw(gd(bb.xq, Kx, 1, W(q[i][0]), Kx, 1, E(c->hq[0].p, (size_t)i * Hd), 2 * Hd, B, H, S + A + 1, EPI_RELU)));
    run(l1, "gemm_L1_fc1");
    // L2 (.. L2b): the remaining hidden layers (K = H, bias in the epilogue); the last one
    // also accumulates the critic head (fc3 / fc4) dot partials of q1 / q2 (slots 0 / 1)
    for (int l = 1; l < nh; ++l) {
      Level lv;
      lv.add(fw(gd_fwd_h(c->hp[l - 1].p, Hd, W(c->p_fc[l]), Hd, c->hp[l].p, Hd, 2 * B, H, H)));
      for (int i = 0; i < 2; ++i) {
        GemmDesc g = fw(gd_fwd_h(E(c->hq[l - 1].p, (size_t)i * Hd), 2 * Hd, W(q[i][l]), Hd,
                                 E(c->hq[l].p, (size_t)i * Hd), 2 * Hd, B, H, H));
        if (l == L) g = with_dot(g, W(q[i][nh]), i);
        lv.add(g);
      }
      run(lv, l == 1 ? "gemm_L2_fc2" : "gemm_L2b_fc3");
    }
    if (mark(c, "heads_sample", 2.0 * 2 * B * (2.0 * A) * H)) {
      hs.tl = c->tl_cur;
      launch_heads_sample(hs, s);
    }
    // L3/L4 (.. L4b): target critics on [s2|1|a'] (head dot partials: slots 2 / 3)
    {
      Level l3;
      for (int i = 0; i < 2; ++i)
        l3.add(fw(gd(bb.x2, Kx, 1, Wt(q[i][0]), Kx, 1, E(c->hqt[0].p, (size_t)i * Hd), 2 * Hd, B, H, S + A + 1, EPI_RELU)));
      run(l3, "gemm_L3_tgt_fc1");
    }
    for (int l = 1; l < nh; ++l) {
      Level lv;
      for (int i = 0; i < 2; ++i) {
        GemmDesc g = fw(gd_fwd_h(E(c->hqt[l - 1].p, (size_t)i * Hd), 2 * Hd, Wt(q[i][l]), Hd,
                                 E(c->hqt[l].p, (size_t)i * Hd), 2 * Hd, B, H, H));
        lv.add(l == L ? with_dot(g, Wt(q[i][nh]), 2 + i) : g);
      }
      run(lv, l == 1 ? "gemm_L4_tgt_fc2" : "gemm_L4b_tgt_fc3");
    }
    run(l5, "gemm_L5_critic_dh1");
    // L5b (3 hidden layers): dh[l-1] = (dh[l] W[l]) * relu'(h[l-1]) down to dh[0]
    for (int l = L - 1; l >= 1; --l) {
      Level lv;
      for (int i = 0; i < 2; ++i)
        lv.add(dh(gd(c->dhc[l].p + i * H, 2 * H, 1, W(q[i][l]), Hd, 0, c->dhc[l - 1].p + i * H, 2 * H,
                     B, H, H, EPI_MASK, E(c->hq[l - 1].p, (size_t)i * Hd), 2 * Hd)));
      run(lv, "gemm_L5b_critic_dh");
    }
    // L6: every critic weight gradient: into the gradient arena, or (fused) straight into
    // Adam + Polyak on the parameters.  The hidden weights are read by the dh levels
    // above, so every critic dW runs here — in both modes, so the reduction order (and
    // the bits) are the same.  Where the policy's dhp1 level (L12) leaves CUs idle and runs
    // on k_gemm (batch <= ~1k), the Polyak step rides there instead (polyak_ride): off the
    // critic Adam level, the longest of the update
    auto dst = [&](const Linear& l) { return fuse ? P + l.off : dW(l); };
    const int wepi = fuse ? (polyak_ride ? EPI_ADAM : EPI_ADAM_POLYAK) : EPI_STORE;
    Level l6;
    for (int i = 0; i < 2; ++i)
      l6.add(dwx(gd(c->dhc[0].p + i * H, 2 * H, 0, bb.xq, Kx, 0, dst(q[i][0]), Kx, H, S + A + 1, B,
                    wepi, nullptr, 0, 1 + i)));
    for (int i = 0; i < 2; ++i) {
      for (int l = 1; l < L; ++l)
        l6.add(dwx(gd_dw_h(c->dhc[l].p + i * H, 2 * H, E(c->hq[l - 1].p, (size_t)i * Hd), 2 * Hd,
                           dst(q[i][l]), Hd, H, H, B, wepi, 1 + i)));
      // L5 stored u = dh[L] / coef (the coefficient factored out of its rows): the layer-L
      // weight gradient applies coef = dL/dq_i (dq) as a per-batch-row K-scale
      GemmDesc wl = dwx(gd_dw_h(c->dhc[L].p + i * H, 2 * H, E(c->hq[L - 1].p, (size_t)i * Hd), 2 * Hd,
                                dst(q[i][L]), Hd, H, H, B, wepi, 1 + i));
      wl.a_ksc = c->dq.p + i * B;
      l6.add(wl);
      l6.add(dwx(gd_dw_h(c->dq4.p + (size_t)i * B * 4, 4, E(c->hq[L].p, (size_t)i * Hd), 2 * Hd, dst(q[i][nh]), Hd, 1, H, B,
                         wepi, 1 + i)));
    }
    if (fuse) {
      AdamFuse& f = l6.b.adam;
      l6.b.has_adam = 1;
      f.P = P; f.M = c->M.p; f.V = c->V.p; f.T = c->T.p; f.G = c->keep_grads ? G : nullptr;
      f.t_base = c->q_begin;
      f.lr = (float)c->cfg.lr; f.beta1 = 0.9f; f.beta2 = 0.999f; f.eps = 1e-8f;
      f.tau = (float)c->cfg.tau; f.step_offset = 1; f.sc = c->sc.p;
      f.loss_part = c->lpart_c.p; f.n_part = nb; f.loss_slot0 = 0; f.n_losses = 2;
      f.loss_host = c->loss_host_dev;
      f.Ph = c->Ph.p; f.Th = c->Th.p;
      f.loss_div = (float)B; f.log_alpha_idx = -1; f.auto_entropy = 0;
      f.err_skip = kErrSkipAll; f.err_nopolyak = kErrActLike;
    }
    if (ride_b) {   // the next update's random.sample rides in L6 (placement B)
      l6.b.ride.kind = 1; l6.b.ride.nblocks = 1;
      l6.b.ride.tbl_log2 = mt_sample_tbl_log2(B, true);
      l6.b.ride.mt = mt_args(c, B, batch_bufs(c, parity ^ 1));
    }
    if (!fuse) {   // data parallel: this update's error flags ride in the critic collective
      l6.b.err_flags = c->dp_sharding_now ? c->dp_flags.p : G + c->q_end;
      l6.b.err_word = &c->sc.p->err;
      check_span(l6.b.err_flags, kDpFlagN - 1, "error flags");
    }
    run(l6, fuse ? "gemm_L6_critic_dW_adam" : "gemm_L6_critic_dW1");
  }
  if (phase_mask & 2) {
   const bool fuse = phase_mask == 7;
   if (!fuse && !c->dp_sharding_now) {   // (sharded: enqueue_dp takes the critic step)
    // critic Adam (+ Polyak, + q-loss finalisation)
    AdamArgs ad = dp_adam_args(c, true, B, grad_scale, use_ring);
    if (polyak_ride) { ad.tgt = nullptr; ad.tgth = nullptr; }   // (Polyak: in L12)
    if (mark(c, polyak_ride ? "adam_critic" : "adam_critic_polyak")) {
      ad.tl = c->tl_cur;
      launch_adam(ad, s);
    }
   }
    // L7/L8 (.. L8b): updated critics on [s|1|a~] (head dot partials: slots 4 / 5)
    const float* xa = E(bb.x2, (size_t)B * Kx);
    Level l7;
    for (int i = 0; i < 2; ++i)
      l7.add(fw(gd(xa, Kx, 1, W(q[i][0]), Kx, 1, E(c->hqa[0].p, (size_t)i * Hd), 2 * Hd, B, H, S + A + 1, EPI_RELU)));
    std::vector<Level> l8s;   // L8 (.. L8b)
    for (int l = 1; l < nh; ++l) {
      Level lv;
      for (int i = 0; i < 2; ++i) {
        GemmDesc g = fw(gd_fwd_h(E(c->hqa[l - 1].p, (size_t)i * Hd), 2 * Hd, W(q[i][l]), Hd,
                                 E(c->hqa[l].p, (size_t)i * Hd), 2 * Hd, B, H, H));
        if (l == L) g = with_dot(g, W(q[i][nh]), 4 + i);
        lv.add(g);
      }
      l8s.push_back(lv);
    }
    // L9: dha[L-1] = (dha[L] W[L]) * relu'(ha[L-1]), with the actor rows folded in: the
    // prologue finishes qa1, qa2 (dot partials), min (ties 1/2 : 1/2), policy-loss
    // partials, step counters; dha[L] = dqa * w_head * [ha[L] > 0] is formed on the fly
    Level l9;
    for (int i = 0; i < 2; ++i) {
      GemmDesc g = gd(E(c->hqa[L].p, (size_t)i * Hd), 2 * Hd, 1, W(q[i][L]), Hd, 0, c->dha[L - 1].p + i * H, 2 * H,
                      B, H, H, EPI_MASK, E(c->hqa[L - 1].p, (size_t)i * Hd), 2 * Hd);
      g.axk = 1; g.ax_slot = i; g.ax_w = W(q[i][nh]);
      l9.add(dh(g));
    }
    {
      RowsFuse& rf = l9.b.rows;
      rf.kind = 2; rf.part = dotp(4); rf.nparts = c->nparts; rf.B = B;
      rf.logp = c->logp.p + B; rf.sc = c->sc.p; rf.loss_part = c->lpart_a.p;
      if (c->cfg.auto_entropy) {
        rf.alpha_grad = G + c->la_idx; rf.logp_part = c->lp_part.p;
        rf.n_lp = (2 * B + heads_rows_per_wg(2 * B) - 1) / heads_rows_per_wg(2 * B);
        rf.target_entropy = (float)(-A);
      }
    }
    // (decided on the complete level: launch_gemm picks the kernel from it)
    // 2 hidden layers: the dL/da GEMM (over both critics' dha1, K = 2H) folds into L9's
    // epilogue as per-32-column partials, and L10 shrinks to the sample-backward tail —
    // except where the level runs on k_axk16 (bf16, batch-4096 class), which keeps L10
    l9.b.bf16 = c->bf16 ? 1 : 0;
    // (batch <= 1024: the standalone L10 runs on B / 16 workgroups, too few to stream dha1;
    // at batch 4096 it fills the chip and the fold measured slower: config 3 L9 55 -> 71 us)
    // (and only where launch_gemm takes the one-wave-group tiles that form the partials:
    // batch 1024 with hidden > 512 goes to the 64-row tiles and keeps L10)
    const bool fold_dlda = nh == 2 && B <= 1024 && !std::getenv("SACMI_NO_DLDA_FOLD") &&
                           gemm_level_pa_capable(l9.b);
    if (fold_dlda) {
      for (int i = 0; i < 2; ++i) {
        GemmDesc& g = l9.b.d[i];
        g.pa_w = W(q[i][0]) + S + 1; g.pa_ld = Kx; g.pa_A = A; g.pa_base = i * c->nparts;
        g.pa_out = c->pa.p;
        check_span(g.pa_w, (int64_t)(H - 1) * Kx + A - 1, "pa_w");
        check_span(g.pa_out, ((int64_t)(g.pa_base + c->nparts) * B) * A - 1, "pa_out");
      }
    }
    std::vector<Level> l9bs;  // L9b (3 hidden layers)
    for (int l = L - 1; l >= 1; --l) {
      Level lv;
      for (int i = 0; i < 2; ++i)
        lv.add(dh(gd(c->dha[l].p + i * H, 2 * H, 1, W(q[i][l]), Hd, 0, c->dha[l - 1].p + i * H, 2 * H,
                     B, H, H, EPI_MASK, E(c->hqa[l - 1].p, (size_t)i * Hd), 2 * Hd)));
      l9bs.push_back(lv);
    }
    // L10: dL/da over both critics (K = 2H) + sample backward -> dhead
    GemmDesc da = gd(c->dha[0].p, 2 * H, 1, W(q[0][0]) + S + 1, Kx, 0, nullptr, 0, B, A, 2 * H);
    validate(da);
    // ... and, for the same rows, dhp[L] = (dhead Whead) * relu'(hp[L]) (policy heads backward)
    auto hpa = [&](int l) { return E(c->hp[l].p, (size_t)B * Hd); };   // actor rows
    SampleBwdArgs sb{};
    sb.cache = c->cache.p + (size_t)B * 3 * A; sb.eps = c->eps.p + (size_t)B * A;
    sb.dhead = c->dhead.p; sb.lddh = c->lddh; sb.A = A; sb.B = B; sb.sc = c->sc.p;
    sb.scale = (float)((c->cfg.action_high - c->cfg.action_low) / 2);
    sb.Wh = W(c->p_head); sb.ldw = Hd; sb.H = H; sb.hp2 = hpa(L); sb.ldh = Hd; sb.dhp2 = c->dhp[L].p;
    sb.hp2_16 = a16;
    check_span(sb.dhp2, (int64_t)B * H - 1, "dhp2");
    check_span(sb.Wh, (int64_t)(2 * A - 1) * Hd + H - 1, "Whead");
    // L11 (3 hidden layers) .. L12: dhp[l-1] = (dhp[l] Wpi[l]) * relu'(hp[l-1]);
    // L13: every policy dW (+ Adam, alpha step, policy loss, loss ring when fused)
    auto pdst = [&](const Linear& l) { return fuse ? P + l.off : dW(l); };
    const int pepi = fuse ? EPI_ADAM : EPI_STORE;
    std::vector<Level> l11s;
    for (int l = L; l >= 2; --l) {
      Level lv;
      lv.add(dh(gd(c->dhp[l].p, H, 1, W(c->p_fc[l]), Hd, 0, c->dhp[l - 1].p, H, B, H, H, EPI_MASK, hpa(l - 1), Hd)));
      l11s.push_back(lv);
    }
    Level l12, l13;
    l12.add(dh(gd(c->dhp[1].p, H, 1, W(c->p_fc[1]), Hd, 0, c->dhp[0].p, H, B, H, H, EPI_MASK, hpa(0), Hd)));
    if (ride_b) {   // ... and its gather in L12, two rows a wave: 256 ride workgroups at config
      // 5, the slots L12's 256 tiles leave free (512 at 2 per CU) — one round; a row a wave
      // (512 workgroups) takes a second round: 3,255 vs 3,282 updates/s
      // (profiles/r05/ride_rows_ab; the ride's 22 MB cost L12 ~8 us either way)
      const int rows_per_block = 16;   // (8 waves)
      l12.b.ride.kind = 2; l12.b.ride.nblocks = (B + rows_per_block - 1) / rows_per_block;
      l12.b.ride.ga = gather_args(c, B, batch_bufs(c, parity ^ 1), false);
    }
    // same level structure fused or not: identical reduction order
    l13.add(dwx(gd_dw_h(c->dhead.p, c->lddh, hpa(L), Hd, pdst(c->p_head), Hd, 2 * A, H, B, pepi, 0)));
    for (int l = L; l >= 1; --l)
      l13.add(dwx(gd_dw_h(c->dhp[l].p, H, hpa(l - 1), Hd, pdst(c->p_fc[l]), Hd, H, H, B, pepi, 0)));
    l13.add(dwx(gd(c->dhp[0].p, H, 0, xa, Kx, 0, pdst(c->p_fc[0]), c->p_fc[0].ld, H, S + 1, B, pepi)));
    if (fuse) {
      AdamFuse& f = l13.b.adam;
      l13.b.has_adam = 1;
      f.P = P; f.M = c->M.p; f.V = c->V.p; f.T = nullptr; f.G = c->keep_grads ? G : nullptr;
      f.t_base = 0;
      f.lr = (float)c->cfg.lr; f.beta1 = 0.9f; f.beta2 = 0.999f; f.eps = 1e-8f; f.tau = 0.f;
      f.step_offset = 0; f.sc = c->sc.p;
      f.loss_part = c->lpart_a.p; f.n_part = nb; f.loss_slot0 = 2; f.n_losses = 1;
      f.loss_host = c->loss_host_dev;
      f.Ph = c->Ph.p; f.Th = c->Th.p;
      f.loss_div = (float)B; f.log_alpha_idx = c->la_idx; f.auto_entropy = c->cfg.auto_entropy;
      f.log_alpha_grad = G + c->la_idx;
      f.loss_ring = use_ring ? c->ring.p : nullptr; f.ring = c->ring_slots;
      f.done_word = reinterpret_cast<int*>(c->loss_host_dev + 4);
      f.err_skip = ~0; f.err_nopolyak = 0;
    }
    if (polyak_ride) {   // (polyak_ride: the critic Adam above left the targets alone)
      PolyakArgs& pk = l12.b.ride.pk;
      pk.T = c->T.p; pk.P = P + c->q_begin; pk.Th = c->Th.p;
      pk.n4 = (c->q_end - c->q_begin) / 4; pk.tau = (float)c->cfg.tau; pk.sc = c->sc.p;
      l12.b.ride.pk_blocks = std::max(8, 248 - ((B + 31) / 32) * ((H + 31) / 32)) / 8 * 8;
    }
    if (ride_next && !ride_b) {
      // the next update's random.sample rides in L12 (128 tiles: idle CUs)
      const BatchBufs nb2 = batch_bufs(c, parity ^ 1);
      l12.b.ride.kind = 1; l12.b.ride.nblocks = 1;
      l12.b.ride.tbl_log2 = mt_sample_tbl_log2(B);
      l12.b.ride.mt = mt_args(c, B, nb2);
      if (c->pf_save) l12.b.ride.mt.mt_save = c->mt_pf.p;   // (a single update's draw ahead)
      // ... and its gather in L13
      l13.b.ride.kind = 2; l13.b.ride.nblocks = 16;
      l13.b.ride.ga = gather_args(c, B, nb2, false);
    }
    {
      run(l7, "gemm_L7_act_fc1");
      for (size_t i = 0; i < l8s.size(); ++i) run(l8s[i], i == 0 ? "gemm_L8_act_fc2" : "gemm_L8b_act_fc3");
      run(l9, "gemm_L9_act_dh1");
      for (Level& lv : l9bs) run(lv, "gemm_L9b_act_dh");
      if (fold_dlda) {
        if (mark(c, "sample_bwd_tail_dhp2", 2.0 * B * (2.0 * A) * H)) {
          sb.tl = c->tl_cur;
          launch_sample_bwd_tail(c->pa.p, 2 * c->nparts, sb, s);
        }
      } else if (mark(c, "gemm_L10_dlda_sample_bwd_dhp2", 2.0 * B * A * (2.0 * H) + 2.0 * B * (2.0 * A) * H)) {
        sb.tl = c->tl_cur;
        launch_gemm_sample_bwd(da, sb, s);
      }
      for (Level& lv : l11s) run(lv, "gemm_L11_pi_dhp");
      run(l12, "gemm_L12_pi_dhp1");
    }
    run(l13, fuse ? "gemm_L13_pi_dW_adam" : "gemm_L13_pi_dW1");
  }
  if ((phase_mask & 4) && phase_mask != 7) {
    AdamArgs ad = dp_adam_args(c, false, B, grad_scale, use_ring);
    if (mark(c, "adam_actor_alpha")) {
      ad.tl = c->tl_cur;
      launch_adam(ad, s);
    }
  }
}

// Explicit batch-set control for a phase-split update (the data-parallel driver's
// captured sequences): parity = this update's minibatch buffer set, have_batch = its
// indices/rows were produced by the previous update's rides, ride_next = produce the
// next update's (in the phase-1 launches).
struct PhaseRide {
  int parity = 0;
  bool have_batch = false, ride_next = false;
};

// The fill a captured update depends on: none for uniform replay and for the fused PER
// sampler (both read it from the device scalars); the unfused PER sequence of very large
// rings is sized by the host's fill.
static int64_t per_graph_len(const sacmi_ctx* c) {
  if (c->cfg.replay_kind != SACMI_REPLAY_PER || c->capacity <= kPerFusedMaxRows) return 0;
  return c->len;
}

// n consecutive fused updates (sacmi_step_many_async, the timeline's replica of it):
// the next update's sampling + gather ride along in this update's launches where they fit
// (uniform replay, batch <= ~2k), else run on the side stream concurrently with it
static void enqueue_many(sacmi_ctx* c, int B, int dev_idx, int dev_eps, bool use_ring, int reps,
                         const PhaseRide& pr = {}) {
  const bool ride = reps > 1 && dev_idx && (ride_possible(c, B) || ride_b_possible(c, B));
  // prioritized replay only: its sampler is long and mostly serial (the numpy-MT uniforms
  // of one workgroup, the 8192-row chunk trees), so overlapping it wins (config 3: 768 ->
  // 719 us per update).  The uniform batch-4096 sampler + gather on the side stream
  // measured slower, forked at the update's start (config 5: 408 -> 424 us: their
  // workgroups push level workgroups of the chip-filling levels into a second round) and
  // forked beside the levels with free slots (L6 / L12: 422 -> 430-450 us — every
  // cross-stream edge of the graph cost the main chain ~10 us); they ride (placement B)
  const bool side = reps > 1 && dev_idx && !ride &&
                    c->cfg.replay_kind == SACMI_REPLAY_PER;
  if (side) {
    if (!c->side_stream) CHECK_HIP(hipStreamCreateWithFlags(&c->side_stream, hipStreamNonBlocking));
    while ((int)c->side_ev.size() < 2 * reps) {
      hipEvent_t e;
      CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      c->side_ev.push_back(e);
    }
  }
  if (side) {
    // update r uses batch set r & 1; its successor's set is free once update r - 1 has
    // finished, i.e. at update r's start (fork); update r + 1 starts after the side
    // stream's gather (join).  The side stream's own order keeps the sampling stream's
    // state (MT / numpy MT + frame) sequential, exactly as n separate updates consume it.
    enqueue_sample_gather(c, B, 0, true, c->stream);
    for (int r = 0; r < reps; ++r) {
      if (r > 0) CHECK_HIP(hipStreamWaitEvent(c->stream, c->side_ev[2 * r + 1], 0));
      if (r + 1 < reps) {
        CHECK_HIP(hipEventRecord(c->side_ev[2 * r], c->stream));
        CHECK_HIP(hipStreamWaitEvent(c->side_stream, c->side_ev[2 * r], 0));
        enqueue_sample_gather(c, B, (r + 1) & 1, true, c->side_stream, "_next");
        CHECK_HIP(hipEventRecord(c->side_ev[2 * r + 3], c->side_stream));
      }
      enqueue_update(c, B, dev_idx, dev_eps, 7, 1.f, use_ring, r & 1, true, false);
    }
    return;
  }
  // (pr: a batch drawn ahead by the previous launch — the first update takes it, from set
  // pr.parity — and / or the next launch's drawn ahead by the last update: placement A)
  const int p0 = pr.have_batch ? pr.parity : 0;
  for (int r = 0; r < reps; ++r) {
    const bool last_ahead = r + 1 == reps && pr.ride_next;
    c->pf_save = last_ahead;
    enqueue_update(c, B, dev_idx, dev_eps, 7, 1.f, use_ring, ride || pr.have_batch ? ((p0 + r) & 1) : 0,
                   (ride && r > 0) || (r == 0 && pr.have_batch), (ride && r + 1 < reps) || last_ahead);
    c->pf_save = false;
  }
}

static void run_update(sacmi_ctx* c, int B, int dev_idx, int dev_eps, int phase_mask,
                       float grad_scale, bool use_ring, int reps = 1, PhaseRide pr = {}) {
  if (phase_mask & 6) require_moments_whole(c);   // (before any state changes; enqueue_update)
  c->pf_save = false;
  if (!c->mb_graph) mb_flush(c);   // (mb_graph: this update's sampler takes them)
  c->inflight = true;
  // consecutive fused updates hand the next update's sampling + gather to ride-along
  // workgroups of the current one
  auto enqueue_all = [&]() {
    if (phase_mask == 5) {   // phase 2 of the previous update, then phase 0 of the next
      enqueue_update(c, B, dev_idx, dev_eps, 4, grad_scale, use_ring, pr.parity ^ 1);
      enqueue_update(c, B, dev_idx, dev_eps, 1, grad_scale, use_ring, pr.parity, pr.have_batch);
      return;
    }
    if (phase_mask != 7) {   // one phase of a split update
      enqueue_update(c, B, dev_idx, dev_eps, phase_mask, grad_scale, use_ring, pr.parity,
                     pr.have_batch, pr.ride_next);
      return;
    }
    if (reps == 1 && (pr.ride_next || pr.have_batch)) {   // one fused update drawing the next one's batch ahead
      c->pf_save = true;
      enqueue_update(c, B, dev_idx, dev_eps, 7, grad_scale, use_ring, pr.parity, pr.have_batch, pr.ride_next);
      c->pf_save = false;
      return;
    }
    enqueue_many(c, B, dev_idx, dev_eps, use_ring, reps, pr);
  };
  // the caller is capturing this stream into its own graph (e.g. torch.cuda.graph around
  // a data-parallel update and its collectives): enqueue into that capture directly
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  CHECK_HIP(hipStreamIsCapturing(c->stream, &cap));
  if (!c->use_graphs || cap != hipStreamCaptureStatusNone) {
    enqueue_all();
    CHECK_HIP(hipGetLastError());
    return;
  }
  GraphKey key{B, dev_idx, dev_eps,
               phase_mask | (grad_scale != 1.f ? 8 : 0) | (c->keep_grads ? 16 : 0) |
                   (pr.parity ? 32 : 0) | (pr.have_batch ? 64 : 0) | (pr.ride_next ? 128 : 0) |
                   (c->mb_graph ? 256 : 0),
               use_ring ? c->ring_slots : 0,
               per_graph_len(c), reps};
  auto it = c->graphs.find(key);
  if (it == c->graphs.end()) it = c->graphs.emplace(key, capture_graph(c, enqueue_all)).first;
  CHECK_HIP(hipGraphLaunch(it->second, c->stream));
}

static void check_batch(sacmi_ctx* c, int B) {
  REQUIRE(B > 0 && B <= c->Bm, SACMI_EVALUE,
          "batch_size must be in [1, max_batch=" + std::to_string(c->Bm) + "]");
  REQUIRE(B <= c->len, SACMI_EVALUE, "Sample larger than population or is negative");
}

// batch of an update that samples on the device (random.sample: batch <= 4096; the PER
// sampler's uniforms workgroup holds 2 words per draw in LDS)
static void check_device_batch(sacmi_ctx* c, int B) {
  check_batch(c, B);
  REQUIRE(B <= 4096, SACMI_EVALUE, "device sampling supports batch <= 4096");
}

// ErrBits -> the ValueError text the reference raises there (SACMI_ENAN)
static std::string nan_message(const sacmi_ctx* c, int err, int B, const std::string& where) {
  const std::string shp = "(" + std::to_string(B) + ", " + std::to_string(c->A) + ")";
  const std::string normal = "Expected parameters loc / scale (Tensor of shape " + shp +
                             ") of distribution Normal to satisfy the constraints Real() / "
                             "GreaterThan(lower_bound=0.0), but found invalid values (NaN) in ";
  std::string m;
  if (err & ERR_NAN_PER) m = "probabilities contain NaN (PrioritizedReplayBuffer.sample, replay_buffer.py:64)";
  else if (err & ERR_NAN_TGT) m = normal + "policy.sample(next_state_batch) (sac_imp.py:89)";
  else if (err & (ERR_NAN_ACT | ERR_ABORT)) m = normal + "policy.sample(state_batch) (sac_imp.py:116)";
  else if (err & (ERR_REMOTE_SKIP | ERR_REMOTE_ACT))
    m = "non-finite value in another data-parallel rank's update (its update raised ValueError; "
        "this rank voided the same steps)";
  else m = "non-finite value (error bits " + std::to_string(err) + ")";
  return m + where;
}

// forget the device error bits once reported (stream-ordered: the next update starts clean)
static void clear_err(sacmi_ctx* c) {
  CHECK_HIP(hipMemsetAsync(&c->sc.p->err, 0, sizeof(int32_t), c->stream));
}

static void stage_inputs(sacmi_ctx* c, int B, const int64_t* idx, const float* eps1,
                         const float* eps2) {
  if (idx) {
    std::vector<int32_t> h(B);
    for (int i = 0; i < B; ++i) {
      REQUIRE(idx[i] >= 0 && idx[i] < c->len, SACMI_EVALUE, "index out of range");
      h[i] = (int32_t)idx[i];
    }
    CHECK_HIP(hipMemcpyAsync(c->idx32.p, h.data(), B * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    CHECK_HIP(hipStreamSynchronize(c->stream));
  }
  if (eps1 || eps2) {
    REQUIRE(eps1 && eps2, SACMI_EVALUE, "eps1 and eps2 must both be given");
    const size_t n = (size_t)B * c->A;
    CHECK_HIP(hipMemcpyAsync(c->eps.p, eps1, n * 4, hipMemcpyHostToDevice, c->stream));
    CHECK_HIP(hipMemcpyAsync(c->eps.p + n, eps2, n * 4, hipMemcpyHostToDevice, c->stream));
    CHECK_HIP(hipStreamSynchronize(c->stream));
  }
}

// ---------------------------------------------------------------------------
// RCCL, loaded at run time: a process that already holds a librccl (e.g. torch's) shares
// it — two copies of the collective runtime in one process would each own a transport —
// else $SACMI_RCCL_PATH, else the dynamic loader's librccl.so.1.
struct RcclApi {
  void* h = nullptr;
  decltype(&ncclGetUniqueId) get_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGetErrorString) err = nullptr;
};

static RcclApi& rccl() {
  static RcclApi r;
  if (r.h) return r;
  void* h = nullptr;
  for (const char* n : {"librccl.so", "librccl.so.1"}) {
    if (!h) h = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
  }
  if (!h) {
    if (const char* p = std::getenv("SACMI_RCCL_PATH")) h = dlopen(p, RTLD_NOW | RTLD_LOCAL);
  }
  for (const char* n : {"librccl.so.1", "librccl.so"}) {
    if (!h) h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
  }
  REQUIRE(h, SACMI_EDEVICE, std::string("RCCL not found (set SACMI_RCCL_PATH): ") + dlerror());
  auto sym = [&](const char* name) {
    void* f = dlsym(h, name);
    REQUIRE(f, SACMI_EDEVICE, std::string("RCCL symbol missing: ") + name);
    return f;
  };
  r.get_id = reinterpret_cast<decltype(r.get_id)>(sym("ncclGetUniqueId"));
  r.init_rank = reinterpret_cast<decltype(r.init_rank)>(sym("ncclCommInitRank"));
  r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(sym("ncclAllReduce"));
  r.reduce_scatter = reinterpret_cast<decltype(r.reduce_scatter)>(sym("ncclReduceScatter"));
  r.all_gather = reinterpret_cast<decltype(r.all_gather)>(sym("ncclAllGather"));
  r.group_start = reinterpret_cast<decltype(r.group_start)>(sym("ncclGroupStart"));
  r.group_end = reinterpret_cast<decltype(r.group_end)>(sym("ncclGroupEnd"));
  r.destroy = reinterpret_cast<decltype(r.destroy)>(sym("ncclCommDestroy"));
  r.err = reinterpret_cast<decltype(r.err)>(sym("ncclGetErrorString"));
  r.h = h;
  return r;
}

#define CHECK_RCCL(x)                                                                \
  do {                                                                               \
    ncclResult_t r_ = (x);                                                           \
    if (r_ != ncclSuccess) throw Error{SACMI_EDEVICE, std::string("RCCL: ") + rccl().err(r_)}; \
  } while (0)

// n data-parallel updates, enqueued on the context stream: the host-side driver of
// sacmi/dp.py (DataParallelUpdate over one uninterrupted sequence) with the two
// all-reduces per update issued here — sum in place on the gradient arena, 1/world
// applied by the Adam kernels.
// Sharded (ZeRO-1) form, per range [b, e) of the arena (critic, then actor): the gradients
// are reduce-scattered in place into chunk r (kShardAlign-float multiples; the last chunk may
// reach past e — into the gap between the critic and actor ranges, or into the arena's tail
// slack, never into the other range), Adam runs on chunk r of the parameters (the layer
// segments clipped to it), and the parameters are all-gathered in place.  A reduce-scatter
// does not deliver the error flags to every rank, so this form keeps them in a buffer of their
// own (dp_flags, outside the reduce-scatter's reach) and all-reduces it in the same RCCL group
// (kDpFlagN floats; the all-reduce form carries them in its critic range).  Replicas stay
// bitwise identical: every
// chunk is computed by one rank and the gather copies its bits.  Adam moments (M, V) are
// valid on each rank's own chunks only (sacmi_dp_sync_state gathers them, e.g. before a
// checkpoint).  Loopback: `world` identical ranks emulated on one GPU — the gradients x world
// in place, Adam on every rank's chunk in turn (rank 0 alone finalises the losses / ring),
// the gather an identity.
// Off by default (round 5): the sharded sequence has run only through the loopback emulation,
// never over real RCCL ranks; SACMI_DP_SHARD=1 or sacmi_dp_set_sharded selects it
#ifndef SACMI_DP_SHARD_DEFAULT
#define SACMI_DP_SHARD_DEFAULT 0
#endif
// SACMI_DP_PHASES_AT_WORLD1: a one-rank RCCL job runs the phase sequence and its collectives
// (and so the sharded form when selected) instead of the fused update
static bool dp_phases_at_world1() {
  static const bool on = std::getenv("SACMI_DP_PHASES_AT_WORLD1") != nullptr;
  return on;
}

static bool dp_shard_default(int world) {
  if (const char* e = std::getenv("SACMI_DP_SHARD")) return std::atoi(e) != 0 && world <= kMaxShardWorld;
  return SACMI_DP_SHARD_DEFAULT && world >= 2 && world <= kMaxShardWorld;
}

// The loopback's one-rank timing mode (SACMI_DP_LOOPBACK_ONE_RANK, read at each capture): the
// sequence of ONE rank of a `world`-rank job minus its collectives — the sharded Adam on rank 0's
// chunk only, and no stand-in kernels for the collectives (a real rank moves its bytes over xGMI
// instead: the driver's N > 1 lines).  Each collective then returns this rank's own gradient, so
// Adam applies no 1/world (grad_scale 1): rank 0's chunks take exactly the fused update's values
// at any world (test_dp_sharded_one_rank_chunks)
static bool loopback_one_rank(const sacmi_ctx* c) {
  return c->dp_loopback && std::getenv("SACMI_DP_LOOPBACK_ONE_RANK") != nullptr;
}

static int64_t shard_chunk(int64_t n, int world) {
  return round_up64((n + world - 1) / world, kShardAlign);
}

// Loopback stand-in for the collective over the error flags: `world` identical ranks sum to
// world x this rank's flags; SACMI_DP_LOOPBACK_REMOTE_ERR=1 (tests) adds another rank whose
// update saw a non-finite input of the skip-all class
static void loopback_flags(sacmi_ctx* c, float* f, hipStream_t s) {
  scale_checked(f, kDpFlagN, (float)c->dp_world, s);
  const char* e = std::getenv("SACMI_DP_LOOPBACK_REMOTE_ERR");
  if (e && std::atoi(e) != 0) fill_checked(f, 1, (float)c->dp_world + 1.f, s);
}

static void dp_shard_adam(sacmi_ctx* c, bool critic, int B, int r, bool use_ring) {
  const int W = c->dp_world;
  const int64_t b = critic ? c->q_begin : c->pi_begin, e = critic ? c->q_end : c->total;
  const int64_t ch = shard_chunk(e - b, W), lo = b + r * ch, hi = std::min(e, lo + ch);
  AdamArgs ad = dp_adam_args(c, critic, B, loopback_one_rank(c) ? 1.f : 1.f / (float)W, use_ring);
  ad.tgt = nullptr; ad.tgth = nullptr;   // Polyak: its own pass over the gathered critics
  const AdamArgs full = ad;
  ad.nseg = 0; ad.total = 0;
  for (int i = 0; i < full.nseg; ++i) {
    const int64_t s0 = std::max(full.seg[i].off, lo), s1 = std::min(full.seg[i].off + full.seg[i].n, hi);
    if (s1 > s0) {
      ad.seg[ad.nseg++] = AdamSeg{s0, s1 - s0, full.seg[i].step_idx};
      ad.total += s1 - s0;
    }
  }
  if (!critic && !(c->la_idx >= lo && c->la_idx < hi)) ad.log_alpha_idx = -1;   // (its owner's)
  if (r != c->dp_rank) { ad.n_losses = 0; ad.loss_ring = nullptr; }   // (loopback's other ranks)
  launch_adam(ad, c->stream);
}

static void enqueue_dp_sharded(sacmi_ctx* c, int B, int n) {
  const int W = c->dp_world;
  const bool ride = n > 1 && ride_possible(c, B);
  hipStream_t s = c->stream;
  auto range = [&](bool critic, int64_t& b, int64_t& e) {
    b = critic ? c->q_begin : c->pi_begin;
    e = critic ? c->q_end : c->total;
  };
  auto reduce_scatter = [&](bool critic) {
    int64_t b, e;
    range(critic, b, e);
    const int64_t ch = shard_chunk(e - b, W);
    float* g = c->G.p + b;
    // the critic's error flags to every rank (the reduce-scatter delivers chunk r only): an
    // all-reduce of their own buffer (disjoint from the reduce-scatter's span), in one RCCL
    // group with the reduce-scatter (one launch)
    const bool group = critic && !c->dp_loopback;
    if (group) CHECK_RCCL(rccl().group_start());
    const bool one = loopback_one_rank(c);
    if (critic) {
      (void)mark(c, "allreduce_error_flags");
      float* f = c->dp_flags.p;
      if (c->dp_loopback && !one) loopback_flags(c, f, s);
      else if (!c->dp_loopback) CHECK_RCCL(rccl().all_reduce(f, f, (size_t)kDpFlagN, ncclFloat32, ncclSum, c->comm, s));
    }
    (void)mark(c, critic ? "reduce_scatter_critic_grads" : "reduce_scatter_actor_grads");
    // (loopback: the whole span the collective covers, the last chunk's reach included)
    check_span(g, ch * W - 1, "reduce-scatter span");
    if (c->dp_loopback) {
      if (!one) scale_checked(g, ch * W, (float)W, s);
    } else {
      CHECK_RCCL(rccl().reduce_scatter(g, g + c->dp_rank * ch, (size_t)ch, ncclFloat32, ncclSum, c->comm, s));
    }
    if (group) CHECK_RCCL(rccl().group_end());
  };
  auto step = [&](bool critic) {   // Adam on the chunk(s), gather, the replicated scalars / shadows
    (void)mark(c, critic ? "adam_critic_shard" : "adam_actor_shard");
    // (SACMI_DP_LOOPBACK_ONE_RANK: timing only — rank 0's chunk alone, the per-rank work
    // of a `world`-rank run minus its collectives; the other chunks are left unstepped)
    const bool one_rank = loopback_one_rank(c);
    if (c->dp_loopback && !one_rank) {
      for (int r = 0; r < W; ++r) dp_shard_adam(c, critic, B, r, true);
    } else if (c->dp_loopback) {
      dp_shard_adam(c, critic, B, 0, true);
    } else {
      dp_shard_adam(c, critic, B, c->dp_rank, true);
    }
    int64_t b, e;
    range(critic, b, e);
    const int64_t ch = shard_chunk(e - b, W);
    (void)mark(c, critic ? "all_gather_critic_params" : "all_gather_actor_params");
    if (!c->dp_loopback) {
      float* p = c->P.p + b;
      CHECK_RCCL(rccl().all_gather(p + c->dp_rank * ch, p, (size_t)ch, ncclFloat32, c->comm, s));
    }
    if (c->Ph.p) to_bf16_checked(c->Ph.p + b, c->P.p + b, e - b, s);
    if (!critic && c->cfg.auto_entropy) launch_alpha_sync(c->sc.p, c->P.p + c->la_idx, ~0, s);
  };
  // Polyak rides in phase 1's L12 where it can (enqueue_update: polyak_ride), else its own pass
  const bool pk_ride = !act16_on(c, B) &&
                       (int64_t)((B + 31) / 32) * ((c->H + 31) / 32) <= 192;
  c->dp_sharding_now = true;
  if (!c->dp_loopback && W > 1) c->moments_sharded = true;
  if (loopback_one_rank(c) && W > 1) c->moments_partial = true;
  try {
    int parity = 0;
    bool have = false;
    for (int r = 0; r < n; ++r) {
      if (r > 0) step(false);                                             // previous actor step
      enqueue_update(c, B, 1, 1, 1, 1.f, true, parity, have);             // phase 0
      reduce_scatter(true);
      step(true);
      if (!pk_ride && mark(c, "polyak")) {
        PolyakArgs pk{};
        pk.T = c->T.p; pk.P = c->P.p + c->q_begin; pk.Th = c->Th.p;
        pk.n4 = (c->q_end - c->q_begin) / 4; pk.tau = (float)c->cfg.tau; pk.sc = c->sc.p;
        launch_polyak(pk, s);
      }
      const bool rn = ride && r + 1 < n;
      enqueue_update(c, B, 1, 1, 2, 1.f, true, parity, false, rn);        // phase 1 (no critic Adam)
      reduce_scatter(false);
      have = rn;
      parity = rn ? parity ^ 1 : 0;
    }
    step(false);
  } catch (...) {
    c->dp_sharding_now = false;
    throw;
  }
  c->dp_sharding_now = false;
}

static void enqueue_dp(sacmi_ctx* c, int B, int n) {
  if (c->dp_shard) {
    enqueue_dp_sharded(c, B, n);
    return;
  }
  const float scale = loopback_one_rank(c) ? 1.f : 1.f / (float)c->dp_world;   // (see there)
  const bool ride = n > 1 && ride_possible(c, B);
  auto allreduce = [&](int64_t begin, int64_t end) {
    const bool critic = begin == c->q_begin;
    (void)mark(c, critic ? "allreduce_critic_grads" : "allreduce_actor_grads");
    float* g = c->G.p + begin;
    if (c->dp_loopback) {   // what `world` ranks holding identical shards would all-reduce to
      if (!loopback_one_rank(c)) {
        scale_checked(g, end - begin, (float)c->dp_world, c->stream);
        if (critic) loopback_flags(c, c->G.p + c->q_end, c->stream);
      }
    } else {
      // the critic range carries the error flags past q_end (kDpFlagN)
      const int64_t n = end - begin + (critic ? kDpFlagN : 0);
      CHECK_RCCL(rccl().all_reduce(g, g, (size_t)n, ncclFloat32, ncclSum, c->comm, c->stream));
    }
  };
  int parity = 0;
  bool have = false;
  for (int r = 0; r < n; ++r) {
    if (r > 0) enqueue_update(c, B, 1, 1, 4, scale, true, parity ^ 1);   // previous phase 2
    enqueue_update(c, B, 1, 1, 1, scale, true, parity, have);            // phase 0
    allreduce(c->q_begin, c->q_end);
    const bool rn = ride && r + 1 < n;
    enqueue_update(c, B, 1, 1, 2, scale, true, parity, false, rn);        // phase 1
    allreduce(c->pi_begin, c->total);
    have = rn;
    parity = rn ? parity ^ 1 : 0;
  }
  enqueue_update(c, B, 1, 1, 4, scale, true, parity);                   // last phase 2
}

// Every rank's chunks of the Adam moments onto every rank, in place (collective; a no-op
// unless a sharded step left them valid on the rank's own chunks only).  M and V carry no
// slack: the last chunk is gathered through a bounce of the padded size
static void dp_gather_moments(sacmi_ctx* c) {
  if (c->dp_loopback) c->moments_sharded = false;   // (loopback: every chunk is on this GPU)
  if (!c->moments_sharded || c->dp_loopback || c->dp_world == 1) return;
  const int W = c->dp_world;
  for (int critic = 1; critic >= 0; --critic) {
    const int64_t b = critic ? c->q_begin : c->pi_begin, e = critic ? c->q_end : c->total;
    const int64_t ch = shard_chunk(e - b, W);
    DevBuf<float> tmp;
    tmp.alloc((size_t)ch * W);
    for (float* arena : {c->M.p, c->V.p}) {
      const int64_t lo = b + c->dp_rank * ch, hi = std::min(e, lo + ch);
      if (hi > lo) CHECK_HIP(hipMemcpyAsync(tmp.p + c->dp_rank * ch, arena + lo, (size_t)(hi - lo) * 4,
                                            hipMemcpyDeviceToDevice, c->stream));
      CHECK_RCCL(rccl().all_gather(tmp.p + c->dp_rank * ch, tmp.p, (size_t)ch, ncclFloat32, c->comm, c->stream));
      CHECK_HIP(hipMemcpyAsync(arena + b, tmp.p, (size_t)(e - b) * 4, hipMemcpyDeviceToDevice, c->stream));
    }
    CHECK_HIP(hipStreamSynchronize(c->stream));
    tmp.release();
  }
  c->moments_sharded = false;
}

}  // namespace sacmi

using namespace sacmi;

// ============================================================================
extern "C" {

// A batch drawn ahead by the previous single update is dropped by any other call: the MT
// state goes back to the save point (stream-ordered, before whatever the call enqueues), so
// the random stream is exactly as if nothing had been drawn ahead.
static void pf_settle(sacmi_ctx* c) {
  if (!c || !c->pf_valid) return;
  c->pf_valid = false;
  CHECK_HIP(hipMemcpyAsync(c->mt.p, c->mt_pf.p, 625 * 4, hipMemcpyDeviceToDevice, c->stream));
}

// Every API call other than the device-sampled updates (single or multi-update launches)
// and the read-only queries (losses, tensors, scalars, select_action)
static void pf_touch(sacmi_ctx* c) {
  if (!c) return;
  c->pf_touched = true;
  pf_settle(c);
}

int sacmi_abi_version(void) { return SACMI_ABI_VERSION; }
const char* sacmi_last_error(void) { return g_last_error.c_str(); }

int sacmi_device_count(int* n) {
  return guard([&] { CHECK_HIP(hipGetDeviceCount(n)); });
}

int sacmi_create(const sacmi_config* cfg, int device, sacmi_ctx** out) {
  return guard([&] {
    REQUIRE(cfg && out, SACMI_EVALUE, "null argument");
    REQUIRE(cfg->state_dim > 0 && cfg->action_dim > 0 && cfg->hidden_dim > 0, SACMI_EVALUE,
            "dims must be positive");
    REQUIRE(cfg->action_dim <= 32, SACMI_EVALUE, "action_dim > 32 not supported");
    REQUIRE(cfg->hidden_dim % 4 == 0, SACMI_EVALUE, "hidden_dim must be a multiple of 4");
    REQUIRE(cfg->hidden_dim <= 1020, SACMI_EVALUE, "hidden_dim must be <= 1020 (one wave holds a hidden row)");
    REQUIRE(cfg->max_batch > 0 && cfg->max_batch <= 65536, SACMI_EVALUE, "bad max_batch");
    REQUIRE(cfg->capacity > 0 && cfg->capacity < (int64_t)1 << 31, SACMI_EVALUE, "bad capacity");
    REQUIRE(cfg->n_hidden == 0 || cfg->n_hidden == 2 || cfg->n_hidden == 3, SACMI_EVALUE,
            "n_hidden must be 2 (networks_model1) or 3 (networks_model2)");
    REQUIRE(cfg->compute_dtype == SACMI_COMPUTE_FP32 || cfg->compute_dtype == SACMI_COMPUTE_BF16,
            SACMI_EVALUE, "compute_dtype must be SACMI_COMPUTE_FP32 or SACMI_COMPUTE_BF16");
    int ndev = 0;
    CHECK_HIP(hipGetDeviceCount(&ndev));
    REQUIRE(device >= 0 && device < ndev, SACMI_EDEVICE, "no such HIP device");
    CHECK_HIP(hipSetDevice(device));
    std::unique_ptr<sacmi_ctx> c(new sacmi_ctx());
    c->cfg = *cfg;
    c->device = device;
    c->S = cfg->state_dim; c->A = cfg->action_dim; c->H = cfg->hidden_dim; c->Bm = cfg->max_batch;
    c->nh = cfg->n_hidden == 0 ? 2 : cfg->n_hidden;
    c->bf16 = cfg->compute_dtype == SACMI_COMPUTE_BF16;
    c->capacity = cfg->capacity;
    CHECK_HIP(hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking));
    c->stream = c->own_stream;
    build_layout(c.get());
    alloc_all(c.get());
    c->ring_slots = 4096;
    c->ring.alloc((size_t)c->ring_slots * 3);
    alloc_pinned(c.get());
    DevScalars h{};
    h.alpha = (float)cfg->alpha;
    for (int i = 0; i < 4; ++i) { h.beta_pow[i][0] = 1.0; h.beta_pow[i][1] = 1.0; }
    h.per_frame = 1;
    upload_scalars(c.get(), h);
    // default RNG state: MT seeded with 5489 (both streams), as a fresh generator
    std::vector<uint32_t> k(625);
    k[0] = 5489u;
    for (int i = 1; i < 624; ++i) k[i] = 1812433253u * (k[i - 1] ^ (k[i - 1] >> 30)) + i;
    k[624] = 624;
    CHECK_HIP(hipMemcpy(c->mt.p, k.data(), 625 * 4, hipMemcpyHostToDevice));
    CHECK_HIP(hipMemcpy(c->mt.p + 625, k.data(), 625 * 4, hipMemcpyHostToDevice));
    const char* ng = getenv("SACMI_NO_GRAPH");
    c->use_graphs = !(ng && ng[0] == '1');
    *out = c.release();
  });
}

int sacmi_destroy(sacmi_ctx* c) {
  return guard([&] {
    if (!c) return;
    (void)hipSetDevice(c->device);
    // a fault left by the context's last work is reported by this call (SACMI_EDEVICE), after
    // the context's resources are released — not discarded
    const hipError_t sync_err = hipStreamSynchronize(c->stream);
    destroy_graphs(c);
    free_pinned(c);
    if (c->comm) (void)rccl().destroy(c->comm);
    c->comm = nullptr;
    if (c->G_external) {
      registry_remove((uintptr_t)c->G.p);
      c->G.p = nullptr;
    }
    for (auto* b : {&c->P, &c->T, &c->G, &c->M, &c->V, &c->obs, &c->act, &c->rew, &c->obs2,
                    &c->done, &c->prio, &c->xq, &c->x2, &c->r, &c->d, &c->xqb, &c->x2b, &c->rb,
                    &c->db, &c->eps,
                    &c->cache, &c->logp, &c->dq, &c->dq4, &c->dotp, &c->pa, &c->act_h, &c->dw_ws, &c->dhead, &c->lpart_c, &c->lpart_a, &c->ring, &c->lp_part, &c->dp_flags, &c->ax, &c->ah1, &c->ah2,
                    &c->aeps, &c->acache, &c->alogp, &c->aout, &c->stage, &c->per_scr, &c->per_probs,
                    &c->per_chunk, &c->per_w, &c->per_val})
      b->release();
    for (int l = 0; l < 3; ++l)
      for (auto* b : {&c->hp[l], &c->hq[l], &c->hqt[l], &c->hqa[l], &c->dhc[l], &c->dha[l], &c->dhp[l]})
        b->release();
    c->sc.release(); c->mt.release(); c->mt_backup.release(); c->mt_pf.release(); c->idx32.release(); c->idx64.release();
    c->Ph.release(); c->Th.release();
    c->idx32b.release(); c->idx64b.release();
    c->per_q.release(); c->per_blk.release(); c->per_idx.release(); c->per_cdf.release();
    c->per_u.release(); c->per_uin.release(); c->per_owner.release(); c->per_bad.release();
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    if (c->side_stream) (void)hipStreamDestroy(c->side_stream);
    for (hipEvent_t e : c->side_ev) (void)hipEventDestroy(e);
    delete c;
    if (sync_err != hipSuccess)
      throw Error{SACMI_EDEVICE, std::string("sacmi_destroy: the context's stream had failed: ") +
                                     hipGetErrorString(sync_err)};
  });
}

int sacmi_set_stream(sacmi_ctx* c, void* stream) {
  return guard([&] {
    pf_touch(c);
    REQUIRE(c, SACMI_EVALUE, "null ctx");
    CHECK_HIP(hipStreamSynchronize(c->stream));
    c->stream = stream ? (hipStream_t)stream : c->own_stream;
    destroy_graphs(c);
  });
}

int sacmi_synchronize(sacmi_ctx* c) {
  return guard([&] {
    CHECK_HIP(hipStreamSynchronize(c->stream));
    c->inflight = false;
    c->done_epoch = c->epoch;
  });
}

int sacmi_tensor_numel(sacmi_ctx* c, int net, int layer, int part, int64_t* numel) {
  return guard([&] {
    const Linear l = find_linear(c, net, layer);
    *numel = part == 0 ? (int64_t)l.n_out * l.k_in : (int64_t)l.n_out;
  });
}


static float* slot_base(sacmi_ctx* c, int slot, int net) {
  const bool target = net == SACMI_Q1_TARGET || net == SACMI_Q2_TARGET;
  if (slot == SACMI_SLOT_ADAM_M || slot == SACMI_SLOT_ADAM_V) require_moments_readable(c);
  if (target) {
    REQUIRE(slot == SACMI_SLOT_PARAM, SACMI_EVALUE, "target nets only have parameters");
    return c->T.p - c->q_begin;
  }
  switch (slot) {
    case SACMI_SLOT_PARAM: return c->P.p;
    case SACMI_SLOT_GRAD: return c->G.p;
    case SACMI_SLOT_ADAM_M: return c->M.p;
    case SACMI_SLOT_ADAM_V: return c->V.p;
  }
  throw Error{SACMI_EVALUE, "bad slot"};
}

// re-derive the bf16 shadows after a host write into the parameter / target arenas
static void refresh_shadows(sacmi_ctx* c) {
  if (!c->Ph.p) return;
  to_bf16_checked(c->Ph.p, c->P.p, (int64_t)c->P.n, c->stream);
  to_bf16_checked(c->Th.p, c->T.p, (int64_t)c->T.n, c->stream);
  CHECK_HIP(hipStreamSynchronize(c->stream));
}

static void tensor_io(sacmi_ctx* c, int slot, int net, int layer, int part, float* host,
                      const float* in, int64_t numel) {
  const Linear l = find_linear(c, net, layer);
  const int64_t want = part == 0 ? (int64_t)l.n_out * l.k_in : (int64_t)l.n_out;
  REQUIRE(part == 0 || part == 1, SACMI_EVALUE, "part must be 0 (weight) or 1 (bias)");
  REQUIRE(numel == want, SACMI_EVALUE, "tensor size mismatch");
  float* base = slot_base(c, slot, net) + l.off;
  std::vector<float> buf((size_t)l.n_out * l.ld);
  CHECK_HIP(hipStreamSynchronize(c->stream));
  CHECK_HIP(hipMemcpy(buf.data(), base, buf.size() * 4, hipMemcpyDeviceToHost));
  for (int o = 0; o < l.n_out; ++o) {
    float* row = buf.data() + (size_t)o * l.ld;
    if (part == 1) {
      if (in) row[l.bias_col] = in[o]; else host[o] = row[l.bias_col];
    } else {
      for (int k = 0; k < l.k_in; ++k) {
        const int col = k < l.split ? k : k + 1;
        if (in) row[col] = in[(size_t)o * l.k_in + k]; else host[(size_t)o * l.k_in + k] = row[col];
      }
    }
  }
  if (in) {
    CHECK_HIP(hipMemcpy(base, buf.data(), buf.size() * 4, hipMemcpyHostToDevice));
    refresh_shadows(c);
  }
}

int sacmi_set_tensor(sacmi_ctx* c, int slot, int net, int layer, int part, const float* host,
                     int64_t numel) {
  return guard([&] {
    pf_touch(c); tensor_io(c, slot, net, layer, part, nullptr, host, numel); });
}

int sacmi_get_tensor(sacmi_ctx* c, int slot, int net, int layer, int part, float* host,
                     int64_t numel) {
  return guard([&] { tensor_io(c, slot, net, layer, part, host, nullptr, numel); });
}

static void arena_scalar(sacmi_ctx* c, float* arena, int64_t idx, const double* in, double* out) {
  float v;
  CHECK_HIP(hipStreamSynchronize(c->stream));
  if (in) {
    v = (float)*in;
    CHECK_HIP(hipMemcpy(arena + idx, &v, 4, hipMemcpyHostToDevice));
  } else {
    CHECK_HIP(hipMemcpy(&v, arena + idx, 4, hipMemcpyDeviceToHost));
    *out = v;
  }
}

static void scalar_io(sacmi_ctx* c, int which, const double* in, double* out) {
  switch (which) {
    case SACMI_S_LOG_ALPHA: arena_scalar(c, c->P.p, c->la_idx, in, out); return;
    case SACMI_S_ADAM_M_LOG_ALPHA: require_moments_readable(c); arena_scalar(c, c->M.p, c->la_idx, in, out); return;
    case SACMI_S_ADAM_V_LOG_ALPHA: require_moments_readable(c); arena_scalar(c, c->V.p, c->la_idx, in, out); return;
    case SACMI_S_GRAD_LOG_ALPHA: arena_scalar(c, c->G.p, c->la_idx, in, out); return;
    case SACMI_S_GRAPH_COUNT:
      REQUIRE(!in, SACMI_EVALUE, "the graph count is read-only");
      *out = (double)(c->graphs.size() + c->dp_graphs.size());
      return;
    case SACMI_S_KEEP_GRADS:
      if (in) {
        if (c->keep_grads != (*in != 0)) destroy_graphs(c);
        c->keep_grads = *in != 0;
      } else {
        *out = c->keep_grads ? 1.0 : 0.0;
      }
      return;
    default: break;
  }
  DevScalars h = download_scalars(c);
  switch (which) {
    case SACMI_S_ALPHA: if (in) h.alpha = (float)*in; else *out = h.alpha; break;
    case SACMI_S_ALPHA_IS_TENSOR: if (in) h.alpha_is_tensor = (int)*in; else *out = h.alpha_is_tensor; break;
    case SACMI_S_STEP_POLICY: case SACMI_S_STEP_Q1: case SACMI_S_STEP_Q2: case SACMI_S_STEP_ALPHA: {
      const int k = which - SACMI_S_STEP_POLICY;
      if (in) {
        h.step[k] = *in;
        h.beta_pow[k][0] = std::pow(0.9, *in);
        h.beta_pow[k][1] = std::pow(0.999, *in);
      } else {
        *out = h.step[k];
      }
      break;
    }
    case SACMI_S_PER_FRAME: if (in) h.per_frame = (int64_t)*in; else *out = (double)h.per_frame; break;
    case SACMI_S_NOISE_COUNTER: if (in) h.noise_counter = (uint64_t)*in; else *out = (double)h.noise_counter; break;
    default: throw Error{SACMI_EVALUE, "bad scalar id"};
  }
  if (in) upload_scalars(c, h);
}

int sacmi_set_scalar(sacmi_ctx* c, int which, double value) {
  return guard([&] {
    pf_touch(c); scalar_io(c, which, &value, nullptr); });
}
int sacmi_get_scalar(sacmi_ctx* c, int which, double* value) {
  return guard([&] { scalar_io(c, which, nullptr, value); });
}

namespace sacmi {
static float* mb_rows_host(sacmi_ctx* c) { return reinterpret_cast<float*>(c->mb_host + 1); }

// The mailbox's rows through the scatter kernel (every path but the synchronous update
// that would have consumed them): staged SoA in a zero-copy slot, rows and len / head as
// the mailbox recorded them (the host's len / wpos already count them)
static void mb_flush(sacmi_ctx* c) {
  if (c->mb_pending == 0) return;
  const int S = c->S, A = c->A, m = c->mb_pending;
  const int64_t rowf = 2 * S + A + 2;
  const int k = c->push_zc_slot;
  c->push_zc_slot = (k + 1) % sacmi_ctx::kPushSlots;
  if (c->push_zc_epoch[k] > c->done_epoch) {
    CHECK_HIP(hipStreamSynchronize(c->stream));
    c->done_epoch = c->epoch;
  }
  c->push_zc_epoch[k] = ++c->epoch;
  float* h = c->push_zc_host[k];
  const float* src = mb_rows_host(c);
  for (int j = 0; j < m; ++j) {
    const float* p = src + j * rowf;
    std::memcpy(h + j * S, p, (size_t)S * 4);
    std::memcpy(h + m * S + j * A, p + S, (size_t)A * 4);
    h[m * (S + A) + j] = p[S + A];
    std::memcpy(h + m * (S + A + 1) + j * S, p + S + A + 1, (size_t)S * 4);
    h[m * (2 * S + A + 1) + j] = p[2 * S + A + 1];
  }
  PushArgs pa{};
  pa.stage = c->push_zc_dev[k];
  pa.obs = c->obs.p; pa.obs2 = c->obs2.p; pa.act = c->act.p; pa.rew = c->rew.p; pa.done = c->done.p;
  pa.S = S; pa.A = A; pa.ldo = c->ldo; pa.ldact = c->ldact;
  pa.n = m; pa.pos0 = c->mb_host->pos0; pa.cap = c->capacity;
  pa.sc = c->sc.p;
  pa.len = c->mb_host->len;
  pa.head = c->mb_host->head;
  launch_push_rows(pa, c->stream);
  CHECK_HIP(hipGetLastError());
  c->mb_pending = 0;
}

static MailboxArgs mailbox_args(sacmi_ctx* c) {
  MailboxArgs m{};
  m.hdr = c->mb_dev; m.rows = reinterpret_cast<const float*>(c->mb_dev + 1);
  m.obs = c->obs.p; m.obs2 = c->obs2.p; m.act = c->act.p; m.rew = c->rew.p; m.done = c->done.p;
  m.S = c->S; m.A = c->A; m.ldo = c->ldo; m.ldact = c->ldact; m.cap = c->capacity;
  return m;
}
}  // namespace sacmi

// Rows [n] of transitions into the ring (deque(maxlen) semantics), from either layout:
// separate arrays (packed == nullptr) or packed rows [n][2S + A + 2] = s | a | r | s2 | d.
static void push_impl(sacmi_ctx* c, const float* s, const float* a, const float* r, const float* s2,
                      const uint8_t* d, const float* packed, int64_t n) {
  REQUIRE(n >= 0, SACMI_EVALUE, "n < 0");
  if (n == 0) return;
  REQUIRE(packed || (s && a && r && s2 && d), SACMI_EVALUE, "null transition array");
  {
    // a few rows while no update is in flight: into the mailbox, for the next synchronous
    // update's sampler (uniform replay; every other path flushes them first)
    const int S = c->S, A = c->A;
    const int64_t rowf = 2 * S + A + 2;
    if (c->mb_host && !c->inflight && c->cfg.replay_kind == SACMI_REPLAY_UNIFORM &&
        c->mb_pending + n <= sacmi_ctx::kMbRows && c->mb_pending + n <= c->capacity) {
      // (rows pending beyond the capacity would map two rows onto one ring slot in the
      // sampler's scatter, stored in no fixed order: the chunked path's `skip` handles that)
      float* dst = mb_rows_host(c) + (size_t)c->mb_pending * rowf;
      for (int64_t j = 0; j < n; ++j, dst += rowf) {
        if (packed) {
          std::memcpy(dst, packed + j * rowf, (size_t)rowf * 4);
        } else {
          std::memcpy(dst, s + j * S, (size_t)S * 4);
          std::memcpy(dst + S, a + j * A, (size_t)A * 4);
          dst[S + A] = r[j];
          std::memcpy(dst + S + A + 1, s2 + j * S, (size_t)S * 4);
          dst[rowf - 1] = d[j] ? 1.f : 0.f;
        }
        dst[rowf - 1] = dst[rowf - 1] != 0.f ? 1.f : 0.f;
      }
      if (c->mb_pending == 0) c->mb_host->pos0 = c->wpos;
      c->mb_pending += (int)n;
      c->wpos = (c->wpos + n) % c->capacity;
      c->len = std::min<int64_t>(c->capacity, c->len + n);
      c->mb_host->len = c->len;
      c->mb_host->head = c->len < c->capacity ? 0 : c->wpos;
      c->mb_host->n = c->mb_pending;
      return;
    }
  }
  mb_flush(c);                     // (rows keep their order)
  // only the last `capacity` rows of a huge batch survive (deque(maxlen))
  const int64_t skip = n > c->capacity ? n - c->capacity : 0;
  const int S = c->S, A = c->A;
  const int64_t rowf = 2 * S + A + 2;
  const bool was_empty = c->len == 0;
  const int64_t cap = c->capacity;
  const int64_t pos0 = (c->wpos + skip) % cap;   // ring slot of row `skip`
  // chunks of push_rows rows: pack into a pinned slot (SoA), one async H2D copy, one
  // scatter kernel; the slot is reused once its copy has completed (event).  Chunks of at
  // most kPushZcRows rows go through mapped staging instead: the scatter kernel reads it
  for (int64_t i = skip; i < n; i += c->push_rows) {
    const int64_t m = std::min<int64_t>(c->push_rows, n - i);
    const bool zc = m <= sacmi_ctx::kPushZcRows;
    int k;
    float* h;
    if (zc) {
      k = c->push_zc_slot;
      c->push_zc_slot = (k + 1) % sacmi_ctx::kPushSlots;
      if (c->push_zc_epoch[k] > c->done_epoch) {   // its reader may still be queued
        CHECK_HIP(hipStreamSynchronize(c->stream));
        c->done_epoch = c->epoch;
      }
      c->push_zc_epoch[k] = ++c->epoch;
      h = c->push_zc_host[k];
    } else {
      k = c->push_slot;
      c->push_slot = (k + 1) % sacmi_ctx::kPushSlots;
      CHECK_HIP(hipEventSynchronize(c->push_ev[k]));
      h = c->push_host[k];
    }
    float* hd = h + m * (2 * S + A + 1);
    if (packed) {
      if (m == 1) {                    // one row: the packed layout IS the SoA layout
        std::memcpy(h, packed + i * rowf, (size_t)rowf * 4);
      } else {
        for (int64_t j = 0; j < m; ++j) {
          const float* p = packed + (i + j) * rowf;
          std::memcpy(h + j * S, p, (size_t)S * 4);
          std::memcpy(h + m * S + j * A, p + S, (size_t)A * 4);
          h[m * (S + A) + j] = p[S + A];
          std::memcpy(h + m * (S + A + 1) + j * S, p + S + A + 1, (size_t)S * 4);
          hd[j] = p[2 * S + A + 1];
        }
      }
      for (int64_t j = 0; j < m; ++j) hd[j] = hd[j] != 0.f ? 1.f : 0.f;
    } else {
      std::memcpy(h, s + i * S, (size_t)m * S * 4);
      std::memcpy(h + m * S, a + i * A, (size_t)m * A * 4);
      std::memcpy(h + m * (S + A), r + i, (size_t)m * 4);
      std::memcpy(h + m * (S + A + 1), s2 + i * S, (size_t)m * S * 4);
      for (int64_t j = 0; j < m; ++j) hd[j] = d[i + j] ? 1.f : 0.f;
    }
    if (!zc) {
      CHECK_HIP(hipMemcpyAsync(c->stage.p, h, (size_t)m * rowf * 4, hipMemcpyHostToDevice, c->stream));
      CHECK_HIP(hipEventRecord(c->push_ev[k], c->stream));
    }
    const int64_t done_rows = i + m - skip;
    PushArgs pa{};
    pa.stage = zc ? c->push_zc_dev[k] : c->stage.p;
    pa.obs = c->obs.p; pa.obs2 = c->obs2.p; pa.act = c->act.p; pa.rew = c->rew.p; pa.done = c->done.p;
    pa.S = S; pa.A = A; pa.ldo = c->ldo; pa.ldact = c->ldact;
    pa.n = m; pa.pos0 = (pos0 + (i - skip)) % cap; pa.cap = cap;
    pa.sc = c->sc.p;
    const int64_t len = std::min<int64_t>(cap, c->len + skip + done_rows);
    const int64_t wpos = (c->wpos + skip + done_rows) % cap;
    pa.len = len;
    pa.head = len < cap ? 0 : wpos;
    launch_push_rows(pa, c->stream);
    CHECK_HIP(hipGetLastError());
  }
  const int64_t added = n - skip;
  if (c->cfg.replay_kind == SACMI_REPLAY_PER) {
    launch_per_push(c->prio.p, c->capacity, pos0, added, was_empty ? 1 : 0, c->per_scr.p, c->stream);
  }
  c->wpos = (c->wpos + n) % c->capacity;
  c->len = std::min<int64_t>(c->capacity, c->len + n);
}

int sacmi_push(sacmi_ctx* c, const float* s, const float* a, const float* r, const float* s2,
               const uint8_t* d, int64_t n) {
  return guard([&] {
    pf_touch(c); push_impl(c, s, a, r, s2, d, nullptr, n); });
}

int sacmi_push_packed(sacmi_ctx* c, const float* rows, int64_t n) {
  return guard([&] {
    pf_touch(c); push_impl(c, nullptr, nullptr, nullptr, nullptr, nullptr, rows, n); });
}

int sacmi_len(sacmi_ctx* c, int64_t* n) {
  return guard([&] { *n = c->len; });
}

int sacmi_replay_clear(sacmi_ctx* c) {
  return guard([&] {
    pf_touch(c);
    REQUIRE(c, SACMI_EVALUE, "null ctx");
    DevScalars h = download_scalars(c);
    h.len = 0;
    h.head = 0;
    upload_scalars(c, h);
    c->len = 0;
    c->wpos = 0;
  });
}

int sacmi_get_rows(sacmi_ctx* c, const int64_t* idx, int64_t n, float* s, float* a, float* r,
                   float* s2, uint8_t* d) {
  return guard([&] {
    pf_touch(c);
    mb_flush(c);
    CHECK_HIP(hipStreamSynchronize(c->stream));
    const int64_t head = c->len < c->capacity ? 0 : c->wpos;
    for (int64_t i = 0; i < n; ++i) {
      REQUIRE(idx[i] >= 0 && idx[i] < c->len, SACMI_EVALUE, "index out of range");
      const int64_t sl = (head + idx[i]) % c->capacity;
      if (s) CHECK_HIP(hipMemcpy(s + i * c->S, c->obs.p + sl * c->ldo, c->S * 4, hipMemcpyDeviceToHost));
      if (s2) CHECK_HIP(hipMemcpy(s2 + i * c->S, c->obs2.p + sl * c->ldo, c->S * 4, hipMemcpyDeviceToHost));
      if (a) CHECK_HIP(hipMemcpy(a + i * c->A, c->act.p + sl * c->ldact, c->A * 4, hipMemcpyDeviceToHost));
      if (r) CHECK_HIP(hipMemcpy(r + i, c->rew.p + sl, 4, hipMemcpyDeviceToHost));
      if (d) {
        float f;
        CHECK_HIP(hipMemcpy(&f, c->done.p + sl, 4, hipMemcpyDeviceToHost));
        d[i] = f != 0.f;
      }
    }
  });
}

int sacmi_get_slots(sacmi_ctx* c, const int64_t* slots, int64_t n, float* s, float* a, float* r,
                    float* s2, uint8_t* d) {
  return guard([&] {
    pf_touch(c);
    std::vector<int64_t> pos(n);
    const int64_t head = c->len < c->capacity ? 0 : c->wpos;
    for (int64_t i = 0; i < n; ++i) {
      REQUIRE(slots[i] >= 0 && slots[i] < c->len, SACMI_EVALUE, "slot out of range");
      pos[i] = (slots[i] - head + c->capacity) % c->capacity;
    }
    const int st = sacmi_get_rows(c, pos.data(), n, s, a, r, s2, d);
    if (st != SACMI_OK) throw Error{st, g_last_error};
  });
}

int sacmi_rng_set_mt(sacmi_ctx* c, int stream, const uint32_t* key, int32_t pos) {
  return guard([&] {
    pf_touch(c);
    REQUIRE(stream == 0 || stream == 1, SACMI_EVALUE, "stream must be 0 or 1");
    REQUIRE(pos >= 0 && pos <= 624, SACMI_EVALUE, "MT position must be in [0, 624]");
    std::vector<uint32_t> k(key, key + 624);
    k.push_back((uint32_t)pos);
    CHECK_HIP(hipStreamSynchronize(c->stream));
    CHECK_HIP(hipMemcpy(c->mt.p + 625 * stream, k.data(), 625 * 4, hipMemcpyHostToDevice));
  });
}

int sacmi_rng_get_mt(sacmi_ctx* c, int stream, uint32_t* key, int32_t* pos) {
  return guard([&] {
    pf_touch(c);
    REQUIRE(stream == 0 || stream == 1, SACMI_EVALUE, "stream must be 0 or 1");
    std::vector<uint32_t> k(625);
    CHECK_HIP(hipStreamSynchronize(c->stream));
    CHECK_HIP(hipMemcpy(k.data(), c->mt.p + 625 * stream, 625 * 4, hipMemcpyDeviceToHost));
    std::memcpy(key, k.data(), 624 * 4);
    *pos = (int32_t)k[624];
  });
}

int sacmi_rng_seed_device(sacmi_ctx* c, uint64_t seed, uint64_t offset) {
  return guard([&] {
    pf_touch(c);
    CHECK_HIP(hipStreamSynchronize(c->stream));   // no graph holding the old key in flight
    destroy_graphs(c);                             // the key is a captured kernel argument
    c->cfg.seed = seed;
    double v = (double)offset;
    REQUIRE((uint64_t)v == offset, SACMI_EVALUE, "offset must be below 2^53");
    scalar_io(c, SACMI_S_NOISE_COUNTER, &v, nullptr);
  });
}

int sacmi_sample_indices(sacmi_ctx* c, int32_t batch, int64_t* idx_out) {
  return guard([&] {
    pf_touch(c);
    REQUIRE(batch >= 0 && batch <= c->len, SACMI_EVALUE, "Sample larger than population or is negative");
    REQUIRE(batch <= c->Bm, SACMI_EVALUE, "batch > max_batch");
    REQUIRE(batch <= 4096, SACMI_EVALUE, "device random.sample supports batch <= 4096");
    if (batch == 0) return;
    mb_flush(c);
    MtSampleArgs ma = mt_args(c, batch, batch_bufs(c, 0));
    ma.skip_on_err = 0;                // a host call: the reference's random.sample always runs
    launch_mt_sample(ma, c->stream);
    CHECK_HIP(hipGetLastError());
    CHECK_HIP(hipMemcpyAsync(idx_out, c->idx64.p, (size_t)batch * 8, hipMemcpyDeviceToHost, c->stream));
    CHECK_HIP(hipStreamSynchronize(c->stream));
  });
}

// A device-sampled update launch (sacmi_step / _async / _launch, and the first / last update
// of sacmi_step_many_async): it takes the batch drawn
// ahead for its batch size (no sampler / gather of its own), and draws the next one ahead
// where the ride-along fits (uniform replay, batch <= ~2k; in a graph, not under a caller's
// capture).  Anything else first settles.
static PhaseRide pf_begin(sacmi_ctx* c, int B, bool dev_idx) {
  PhaseRide pr;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  CHECK_HIP(hipStreamIsCapturing(c->stream, &cap));
  const bool graphs = c->use_graphs && cap == hipStreamCaptureStatusNone;
  // (only while single updates follow each other: the trainer's push between updates
  // would drop every batch drawn ahead, at the price of a restore each)
  const bool ahead = c->pf_on && dev_idx && graphs && !c->pf_touched && ride_possible(c, B);
  const bool use = ahead && c->pf_valid && c->pf_B == B && c->mb_pending == 0;
  if (!use) pf_settle(c);
  c->pf_valid = false;
  c->pf_touched = false;
  if (!ahead) return pr;
  pr.parity = use ? c->pf_parity : 0;
  pr.have_batch = use;
  pr.ride_next = true;
  return pr;
}
static void pf_end(sacmi_ctx* c, int B, const PhaseRide& pr, int reps = 1) {
  if (!pr.ride_next) return;
  c->pf_valid = true;
  c->pf_parity = (pr.parity + reps) & 1;    // (the set after the launch's last update)
  c->pf_B = B;
}

// A synchronous single update (sacmi_step / sacmi_step_launch): with device sampling the
// update's sampler also stores the rows waiting in the push mailbox (its graph variant)
static void run_update_mb(sacmi_ctx* c, int B, int dev_idx, int dev_eps, bool mb_ok,
                          bool use_ring = false) {
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;   // (a caller's capture would
  CHECK_HIP(hipStreamIsCapturing(c->stream, &cap));          //  replay the mailbox read)
  const PhaseRide pr = pf_begin(c, B, dev_idx != 0);
  // (a batch drawn ahead: no push since, so no mailbox rows either)
  c->mb_graph = mb_ok && dev_idx && c->mb_pending > 0 && cap == hipStreamCaptureStatusNone &&
                c->cfg.replay_kind == SACMI_REPLAY_UNIFORM && !pr.have_batch;
  try {
    run_update(c, B, dev_idx, dev_eps, 7, 1.f, use_ring, 1, pr);
    pf_end(c, B, pr);
  } catch (...) {
    c->mb_graph = false;
    throw;
  }
  if (c->mb_graph) c->mb_pending = 0;
  c->mb_graph = false;
}

// The done word's value before a synchronous step's launch: with nothing else in flight, its
// next change is that update's (step_finish polls for it); -1 otherwise (stream sync)
static int done_prev(sacmi_ctx* c) {
  if (c->inflight) return -1;
  return *reinterpret_cast<volatile int*>(c->loss_host + 4);
}

// Host wait on a word a kernel stores into host-mapped memory behind a system-scope fence
// (the update's done counter, select_action's heads).  Returns true once `done(value)` holds;
// false when the stream finished (or failed) without the store — the caller then
// synchronises the stream, which reports any error.  hipStreamQuery runs every 1024 spins.
// Done when (*w == value) == equal.
static bool poll_done(volatile int* w, hipStream_t s, int value, bool equal) {
  for (int it = 1;; ++it) {
    if ((*w == value) == equal) {
      std::atomic_thread_fence(std::memory_order_acquire);
      return true;
    }
    if ((it & 1023) == 0) {
      const hipError_t q = hipStreamQuery(s);
      if (q != hipErrorNotReady) return false;
      (void)hipGetLastError();
    }
  }
}

// the synchronous step's second half: wait, then the losses (or the error bits) the
// update's last kernels stored into host-mapped memory
// done_prev >= 0: the done word's value before the launch, with no other update in flight:
// the host polls the word the update's last level stores (host-mapped, behind a
// system-scope fence) instead of waiting for the stream's completion signal
static void step_finish(sacmi_ctx* c, int batch, float* losses_out, int done_prev = -1) {
  bool done = false;
  if (done_prev >= 0) {
    volatile int* w = reinterpret_cast<volatile int*>(c->loss_host + 4);
    done = poll_done(w, c->stream, done_prev, false);
  }
  if (!done) CHECK_HIP(hipStreamSynchronize(c->stream));
  c->inflight = false;
  c->done_epoch = c->epoch;             // (the update ran after everything enqueued before it)
  int err = 0;                                   // ErrBits the update's L6 saw
  std::memcpy(&err, c->loss_host + 3, 4);
  if (err) {
    clear_err(c);
    pf_settle(c);     // (the batch drawn ahead belongs to a voided update)
    throw Error{SACMI_ENAN, nan_message(c, err, batch, " during update_parameters")};
  }
  std::memcpy(losses_out, c->loss_host, 12);    // stored by the update's last kernels
}

int sacmi_step(sacmi_ctx* c, int32_t batch, const int64_t* idx, const float* eps1,
               const float* eps2, float* losses_out) {
  return guard([&] {
    check_batch(c, batch);
    REQUIRE(idx || batch <= 4096, SACMI_EVALUE, "device random.sample supports batch <= 4096");
    stage_inputs(c, batch, idx, eps1, eps2);
    const int prev = done_prev(c);
    run_update_mb(c, batch, idx ? 0 : 1, (eps1 || eps2) ? 0 : 1, !idx && batch <= 4096);
    if (losses_out) step_finish(c, batch, losses_out, prev);
  });
}

int sacmi_step_launch(sacmi_ctx* c, int32_t batch) {
  return guard([&] {
    REQUIRE(c->pending_step == 0, SACMI_ESTATE, "sacmi_step_launch: the previous launch was not waited for");
    check_device_batch(c, batch);
    stage_inputs(c, batch, nullptr, nullptr, nullptr);
    c->pending_done = done_prev(c);
    run_update_mb(c, batch, 1, 1, true);           // (sacmi_step's graph: the same bits)
    c->pending_step = batch;
  });
}

int sacmi_step_wait(sacmi_ctx* c, float* losses_out) {
  return guard([&] {
    REQUIRE(c->pending_step > 0, SACMI_ESTATE, "sacmi_step_wait without a launch");
    REQUIRE(losses_out, SACMI_EVALUE, "losses_out is NULL");
    const int batch = c->pending_step;
    c->pending_step = 0;
    step_finish(c, batch, losses_out, c->pending_done);
  });
}

int sacmi_step_async(sacmi_ctx* c, int32_t batch) {
  return guard([&] {
    check_device_batch(c, batch);
    run_update_mb(c, batch, 1, 1, false, true);
  });
}

int sacmi_step_many_async(sacmi_ctx* c, int32_t batch, int32_t n_updates) {
  return guard([&] {
    check_device_batch(c, batch);
    REQUIRE(n_updates >= 1 && n_updates <= 256, SACMI_EVALUE, "n_updates must be in [1, 256]");
    const PhaseRide pr = pf_begin(c, batch, true);   // (draws the next launch's batch ahead)
    run_update(c, batch, 1, 1, 7, 1.f, true, n_updates, pr);
    pf_end(c, batch, pr, n_updates);
  });
}

int sacmi_fetch_losses(sacmi_ctx* c, float* out, int32_t max_steps, int32_t* n_out) {
  return guard([&] {
    REQUIRE(max_steps >= 0 && (max_steps == 0 || out), SACMI_EVALUE, "bad output buffer");
    DevScalars h = download_scalars(c);
    const int64_t avail = std::min<int64_t>(h.loss_ring_pos, c->ring_slots);
    const int64_t n = std::min<int64_t>(avail, max_steps);
    // most recent n entries, oldest first: at most two contiguous runs of the ring,
    // copied into pinned staging with one stream sync
    const int64_t first = (h.loss_ring_pos - n) % c->ring_slots;
    const int64_t run1 = std::min<int64_t>(n, c->ring_slots - first);
    if (run1 > 0)
      CHECK_HIP(hipMemcpyAsync(c->ring_host, c->ring.p + first * 3, (size_t)run1 * 12,
                               hipMemcpyDeviceToHost, c->stream));
    if (n > run1)
      CHECK_HIP(hipMemcpyAsync(c->ring_host + run1 * 3, c->ring.p, (size_t)(n - run1) * 12,
                               hipMemcpyDeviceToHost, c->stream));
    CHECK_HIP(hipStreamSynchronize(c->stream));
    if (n > 0) std::memcpy(out, c->ring_host, (size_t)n * 12);
    *n_out = (int32_t)n;
    if (h.err) {   // the completed updates' losses are out; the first voided one is reported
      clear_err(c);
      pf_settle(c);     // (a batch drawn ahead belongs to a voided update)
      throw Error{SACMI_ENAN, nan_message(c, h.err, c->Bm, " at update #" + std::to_string(h.loss_ring_pos) +
                                                              " of this agent (0-based; later updates of that launch were skipped)")};
    }
  });
}

int sacmi_step_phase(sacmi_ctx* c, int32_t batch, int32_t phase, float grad_scale) {
  return guard([&] {
    pf_touch(c);
    REQUIRE(phase >= 0 && phase <= 3, SACMI_EVALUE, "phase must be 0, 1, 2 or 3");
    if (phase == 0 || phase == 3) check_device_batch(c, batch);
    run_update(c, batch, 1, 1, phase == 3 ? 5 : 1 << phase, grad_scale, false);
  });
}

int sacmi_step_phase_ex(sacmi_ctx* c, int32_t batch, int32_t phase, float grad_scale,
                        int32_t parity, int32_t have_batch, int32_t ride_next) {
  return guard([&] {
    pf_touch(c);
    REQUIRE(phase >= 0 && phase <= 3, SACMI_EVALUE, "phase must be 0, 1, 2 or 3");
    REQUIRE(parity == 0 || parity == 1, SACMI_EVALUE, "parity must be 0 or 1");
    if (phase == 0 || phase == 3) check_device_batch(c, batch);
    PhaseRide pr;
    pr.parity = parity;
    pr.have_batch = have_batch && (phase == 0 || phase == 3);
    pr.ride_next = ride_next && phase == 1 && ride_possible(c, batch);
    REQUIRE(!pr.have_batch || ride_possible(c, batch), SACMI_EVALUE,
            "have_batch needs uniform replay with a ride-capable batch size");
    run_update(c, batch, 1, 1, phase == 3 ? 5 : 1 << phase, grad_scale, false, 1, pr);
  });
}

int sacmi_allreduce_unique_id(void* id_out, int32_t nbytes) {
  return guard([&] {
    REQUIRE(id_out && nbytes >= (int32_t)sizeof(ncclUniqueId), SACMI_EVALUE,
            "id buffer must hold SACMI_RCCL_ID_BYTES bytes");
    static_assert(sizeof(ncclUniqueId) == SACMI_RCCL_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId id;
    CHECK_RCCL(rccl().get_id(&id));
    std::memcpy(id_out, &id, sizeof(id));
  });
}

int sacmi_allreduce_init(sacmi_ctx* c, const void* id, int32_t nbytes, int32_t rank, int32_t world) {
  return guard([&] {
    pf_touch(c);
    REQUIRE(id && nbytes == (int32_t)sizeof(ncclUniqueId), SACMI_EVALUE, "bad RCCL unique id");
    REQUIRE(world >= 1 && rank >= 0 && rank < world, SACMI_EVALUE, "bad rank / world");
    REQUIRE(!c->comm && !c->dp_loopback, SACMI_ESTATE, "communicator already initialised");
    CHECK_HIP(hipSetDevice(c->device));
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclComm_t comm;
    CHECK_RCCL(rccl().init_rank(&comm, world, uid, rank));
    c->comm = comm;
    c->dp_world = world;
    c->dp_rank = rank;
    c->dp_shard = dp_shard_default(world);
  });
}

int sacmi_dp_loopback_init(sacmi_ctx* c, int32_t world) {
  return guard([&] {
    pf_touch(c);
    REQUIRE(c, SACMI_EVALUE, "null ctx");
    REQUIRE(world >= 1 && world <= 1024, SACMI_EVALUE, "world must be in [1, 1024]");
    REQUIRE(!c->comm, SACMI_ESTATE, "communicator already initialised");
    c->dp_world = world;
    c->dp_rank = 0;
    c->dp_loopback = true;
    c->dp_shard = dp_shard_default(world);
    destroy_graphs(c);
  });
}

int sacmi_step_dp(sacmi_ctx* c, int32_t batch, int32_t n_updates) {
  return guard([&] {
    pf_touch(c);
    mb_flush(c);
    REQUIRE(c->comm || c->dp_loopback, SACMI_ESTATE, "sacmi_allreduce_init has not been called");
    check_device_batch(c, batch);
    REQUIRE(n_updates >= 1 && n_updates <= 256, SACMI_EVALUE, "n_updates must be in [1, 256]");
    // one rank: nothing to reduce — the fused update (bit-identical to the phase sequence:
    // test_dp_* world-1 and loopback tests), unless SACMI_DP_PHASES_AT_WORLD1 asks for the
    // phase sequence and its collectives anyway
    if (c->dp_world == 1 && !c->dp_loopback && !dp_phases_at_world1()) {
      run_update(c, batch, 1, 1, 7, 1.f, true, n_updates);
      return;
    }
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    CHECK_HIP(hipStreamIsCapturing(c->stream, &cap));
    if (!c->use_graphs || cap != hipStreamCaptureStatusNone) {
      enqueue_dp(c, batch, n_updates);
      CHECK_HIP(hipGetLastError());
      return;
    }
    const auto key = std::make_tuple((int)batch, (int)n_updates, per_graph_len(c));
    auto it = c->dp_graphs.find(key);
    if (it == c->dp_graphs.end())
      it = c->dp_graphs.emplace(key, capture_graph(c, [&] { enqueue_dp(c, batch, n_updates); })).first;
    CHECK_HIP(hipGraphLaunch(it->second, c->stream));
  });
}

int sacmi_dp_set_sharded(sacmi_ctx* c, int32_t on) {
  return guard([&] {
    pf_touch(c);
    REQUIRE(c->comm || c->dp_loopback, SACMI_ESTATE, "sacmi_allreduce_init has not been called");
    REQUIRE(!on || c->dp_world <= kMaxShardWorld, SACMI_EVALUE, "sharded step: world > 64");
    // leaving the sharded form: the moments whole on every rank first (the all-reduce form
    // steps every element from this rank's M, V) — a collective, like the switch itself
    if (!on) dp_gather_moments(c);
    c->dp_shard = on != 0;
    for (auto& kv : c->dp_graphs) (void)hipGraphExecDestroy(kv.second);
    c->dp_graphs.clear();
  });
}

int sacmi_dp_sharded(sacmi_ctx* c, int32_t* on) {
  return guard([&] {
    REQUIRE(c && on, SACMI_EVALUE, "null argument");
    *on = c->dp_shard && (c->dp_world > 1 || c->dp_loopback || dp_phases_at_world1()) ? 1 : 0;
  });
}

int sacmi_dp_sync_state(sacmi_ctx* c) {
  return guard([&] {
    pf_touch(c);
    REQUIRE(c->comm || c->dp_loopback, SACMI_ESTATE, "sacmi_allreduce_init has not been called");
    dp_gather_moments(c);
  });
}

int sacmi_step_act16(sacmi_ctx* c, int32_t batch, int32_t* out) {
  return guard([&] {
    pf_touch(c); *out = act16_on(c, batch) ? 1 : 0; });
}

int sacmi_read_batch(sacmi_ctx* c, int32_t batch, int64_t* idx, float* eps, int64_t eps_numel) {
  return guard([&] {
    REQUIRE(c && idx && eps, SACMI_EVALUE, "null argument");
    REQUIRE(batch >= 1 && batch <= c->Bm, SACMI_EVALUE, "bad batch");
    REQUIRE(eps_numel == (int64_t)2 * batch * c->A, SACMI_EVALUE, "eps_numel must be 2 * batch * action_dim");
    CHECK_HIP(hipStreamSynchronize(c->stream));
    CHECK_HIP(hipMemcpy(idx, c->idx64.p, (size_t)batch * 8, hipMemcpyDeviceToHost));
    CHECK_HIP(hipMemcpy(eps, c->eps.p, (size_t)eps_numel * 4, hipMemcpyDeviceToHost));
  });
}

int sacmi_read_activation(sacmi_ctx* c, int32_t pass, int32_t layer, int32_t batch, float* out,
                          int64_t numel) {
  return guard([&] {
    REQUIRE(c && out, SACMI_EVALUE, "null argument");
    REQUIRE(pass >= 0 && pass <= 3 && layer >= 0 && layer < c->nh, SACMI_EVALUE, "bad (pass, layer)");
    REQUIRE(batch >= 1 && batch <= c->Bm, SACMI_EVALUE, "bad batch");
    REQUIRE(numel == (int64_t)2 * batch * c->H, SACMI_EVALUE, "numel must be 2 * batch * hidden");
    REQUIRE(!act16_on(c, batch), SACMI_ESTATE, "activations of this batch are stored as bf16");
    CHECK_HIP(hipStreamSynchronize(c->stream));
    const size_t H4 = (size_t)c->H * 4;
    if (pass == 3) {
      CHECK_HIP(hipMemcpy2D(out, H4, c->hp[layer].p, (size_t)c->Hd * 4, H4, (size_t)2 * batch,
                            hipMemcpyDeviceToHost));
      return;
    }
    const DevBuf<float>& b = pass == 0 ? c->hq[layer] : pass == 1 ? c->hqt[layer] : c->hqa[layer];
    for (int i = 0; i < 2; ++i)
      CHECK_HIP(hipMemcpy2D(out + (size_t)i * batch * c->H, H4, b.p + (size_t)i * c->Hd, (size_t)2 * c->Hd * 4, H4,
                            (size_t)batch, hipMemcpyDeviceToHost));
  });
}

int sacmi_step_ride_possible(sacmi_ctx* c, int32_t batch, int32_t* out) {
  return guard([&] { *out = ride_possible(c, batch) ? 1 : 0; });
}

int sacmi_grad_arena_numel(sacmi_ctx* c, int64_t* numel) {
  return guard([&] { *numel = c->total + kShardSlack; });
}

int sacmi_attach_grad_arena(sacmi_ctx* c, void* ptr, int64_t numel) {
  return guard([&] {
    pf_touch(c);
    REQUIRE(ptr && numel == c->total + kShardSlack, SACMI_EVALUE, "grad arena must hold exactly grad_arena_numel floats");
    REQUIRE(((uintptr_t)ptr & 15) == 0, SACMI_EVALUE, "grad arena must be 16-byte aligned");
    CHECK_HIP(hipStreamSynchronize(c->stream));
    CHECK_HIP(hipMemset(ptr, 0, (size_t)numel * 4));
    CHECK_HIP(hipDeviceSynchronize());
    if (c->G_external) {
      // the previous arena belongs to the caller: drop its registry entry, never free it
      registry_remove((uintptr_t)c->G.p);
      c->G.p = nullptr;
      c->G.n = 0;
    } else {
      c->G.release();
    }
    c->G.p = (float*)ptr;
    c->G.n = (size_t)numel;
    c->G_external = true;
    registry_add((uintptr_t)ptr, (size_t)numel * 4);
    destroy_graphs(c);
  });
}

int sacmi_grad_buffer(sacmi_ctx* c, int which, void** ptr, int64_t* numel) {
  return guard([&] {
    pf_touch(c);
    REQUIRE(which == 0 || which == 1, SACMI_EVALUE, "which must be 0 (critic) or 1 (actor)");
    // (the critic range carries the kDpFlagN error flags past q_end: the caller's collective
    // sums them with the gradients)
    if (which == 0) { *ptr = c->G.p + c->q_begin; *numel = c->q_end - c->q_begin + kDpFlagN; }
    else { *ptr = c->G.p + c->pi_begin; *numel = c->total - c->pi_begin; }
  });
}

int sacmi_profile_step(sacmi_ctx* c, int32_t batch, int32_t iters, char* names_out,
                       float* ms_out, double* flops_out, int32_t max_sites, int32_t* n_sites) {
  return guard([&] {
    pf_touch(c);
    mb_flush(c);
    check_device_batch(c, batch);
    REQUIRE(iters > 0, SACMI_EVALUE, "iters must be > 0");
    std::vector<double> acc;
    std::vector<std::string> names;
    std::vector<double> fl;
    for (int it = 0; it < iters; ++it) {
      c->prof = true;
      c->prof_events.clear(); c->prof_names.clear(); c->prof_flops.clear(); c->prof_bytes.clear();
      try {
        enqueue_update(c, batch, 1, 1, 7, 1.f, false);
        (void)mark(c, "end");
      } catch (...) {
        c->prof = false;
        throw;
      }
      c->prof = false;
      CHECK_HIP(hipStreamSynchronize(c->stream));
      const size_t n = c->prof_events.size() - 1;
      if (acc.empty()) { acc.assign(n, 0.0); names = c->prof_names; fl = c->prof_flops; }
      for (size_t i = 0; i < n; ++i) {
        float ms = 0;
        CHECK_HIP(hipEventElapsedTime(&ms, c->prof_events[i], c->prof_events[i + 1]));
        acc[i] += ms;
      }
      for (auto e : c->prof_events) (void)hipEventDestroy(e);
      c->prof_events.clear();
    }
    const int n = (int)std::min<size_t>(acc.size(), (size_t)max_sites);
    for (int i = 0; i < n; ++i) {
      std::memset(names_out + 32 * i, 0, 32);
      std::strncpy(names_out + 32 * i, names[i].c_str(), 31);
      ms_out[i] = (float)(acc[i] / iters);
      flops_out[i] = fl[i];
    }
    *n_sites = n;
  });
}

int sacmi_profile_sites(sacmi_ctx* c, int32_t batch, int32_t reps, char* names_out,
                        float* us_out, double* flops_out, double* bytes_out, int32_t max_sites,
                        int32_t* n_sites) {
  return guard([&] {
    mb_flush(c);
    check_device_batch(c, batch);
    REQUIRE(reps > 0 && reps <= 1000, SACMI_EVALUE, "reps must be in [1, 1000]");
    // enumerate the sites of the fused single-GPU update without launching anything
    c->prof_names.clear(); c->prof_flops.clear(); c->prof_bytes.clear();
    c->prof_collect = true;
    c->prof_site = 1 << 30;
    try {
      enqueue_update(c, batch, 1, 1, 7, 1.f, false);
    } catch (...) {
      c->prof_collect = false; c->prof_site = -1;
      throw;
    }
    c->prof_collect = false;
    const std::vector<std::string> names = c->prof_names;
    const std::vector<double> fl = c->prof_flops, by = c->prof_bytes;
    c->prof_names.clear(); c->prof_flops.clear(); c->prof_bytes.clear();
    const int n = (int)std::min<size_t>(names.size(), (size_t)max_sites);
    hipEvent_t e0, e1;
    CHECK_HIP(hipEventCreate(&e0));
    CHECK_HIP(hipEventCreate(&e1));
    for (int i = 0; i < n; ++i) {
      c->prof_site = i;
      hipGraphExec_t ex;
      try {
        ex = capture_graph(c, [&] { for (int r = 0; r < reps; ++r) enqueue_update(c, batch, 1, 1, 7, 1.f, false); });
      } catch (...) {
        c->prof_site = -1;
        throw;
      }
      CHECK_HIP(hipGraphLaunch(ex, c->stream));      // warm
      CHECK_HIP(hipEventRecord(e0, c->stream));
      CHECK_HIP(hipGraphLaunch(ex, c->stream));
      CHECK_HIP(hipEventRecord(e1, c->stream));
      CHECK_HIP(hipEventSynchronize(e1));
      float ms = 0;
      CHECK_HIP(hipEventElapsedTime(&ms, e0, e1));
      CHECK_HIP(hipGraphExecDestroy(ex));
      std::memset(names_out + 32 * i, 0, 32);
      std::strncpy(names_out + 32 * i, names[i].c_str(), 31);
      us_out[i] = ms * 1000.f / reps;
      flops_out[i] = fl[i];
      if (bytes_out) bytes_out[i] = by[i];
    }
    c->prof_site = -1;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    *n_sites = n;
  });
}

// Launch timeline of whatever `enqueue` puts on the context stream, captured into one
// hipGraph with every kernel launch pointing at its own timeline slots; replayed once
// warm, then once measured between HIP events.  Sites that launch no stamping kernel (the
// RCCL all-reduces of the data-parallel sequence) leave no entry.
extern "C++" {
template <class F>
static void timeline_of(sacmi_ctx* c, int n_updates, F&& enqueue, int32_t max_kernels,
                        char* names_out, int32_t* kind_out, int32_t* grid_out, int32_t* site_out,
                        double* start_us, double* end_us, double* flops_out, double* bytes_out,
                        int32_t* n_kernels, double* graph_us) {
  REQUIRE(max_kernels > 0 && names_out && kind_out && grid_out && site_out && start_us && end_us &&
              n_kernels && graph_us, SACMI_EVALUE, "null output");
  CHECK_HIP(hipStreamSynchronize(c->stream));
  DevBuf<tl_word> buf;
  const int cap = 64 * n_updates;                // launch sites (an update has < 40)
  buf.alloc((size_t)cap * kTlPerSite * kTlWords);
  hipGraphExec_t ex = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  auto cleanup = [&]() {
    c->tl_dev = nullptr; c->tl_cur = nullptr;
    if (ex) (void)hipGraphExecDestroy(ex);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    buf.release();
  };
  try {
    c->tl_dev = buf.p; c->tl_cap = cap; c->tl_sites = 0;
    c->tl_names.clear(); c->tl_flops.clear(); c->tl_bytes.clear();
    ex = capture_graph(c, enqueue);
    c->tl_dev = nullptr; c->tl_cur = nullptr;
    CHECK_HIP(hipEventCreate(&e0));
    CHECK_HIP(hipEventCreate(&e1));
    CHECK_HIP(hipGraphLaunch(ex, c->stream));     // warm (its stamps are discarded)
    CHECK_HIP(hipMemsetAsync(buf.p, 0xFF, buf.n * sizeof(tl_word), c->stream));
    CHECK_HIP(hipEventRecord(e0, c->stream));
    CHECK_HIP(hipGraphLaunch(ex, c->stream));
    CHECK_HIP(hipEventRecord(e1, c->stream));
    CHECK_HIP(hipEventSynchronize(e1));
    float ms = 0;
    CHECK_HIP(hipEventElapsedTime(&ms, e0, e1));
    *graph_us = ms * 1000.0;
    std::vector<tl_word> h(buf.n);
    CHECK_HIP(hipMemcpy(h.data(), buf.p, buf.n * sizeof(tl_word), hipMemcpyDeviceToHost));
    if (const char* path = std::getenv("SACMI_DIAG_DUMP")) {
      // raw buffer for tools/phase_dump.py: header {sites, per-site launches, words per
      // launch, phases}, the site names (32 bytes each), then the words
      if (FILE* f = std::fopen(path, "wb")) {
        const int64_t hdr[4] = {c->tl_sites, kTlPerSite, kTlWords, kTlPhases};
        std::fwrite(hdr, sizeof(hdr), 1, f);
        for (int i = 0; i < c->tl_sites; ++i) {
          char nm[32] = {};
          std::strncpy(nm, c->tl_names[i].c_str(), 31);
          std::fwrite(nm, 32, 1, f);
        }
        std::fwrite(h.data(), sizeof(tl_word), (size_t)c->tl_sites * kTlPerSite * kTlWords, f);
        std::fclose(f);
      }
    }
    tl_word t0 = ~(tl_word)0;
    for (int sidx = 0; sidx < c->tl_sites; ++sidx)
      for (int k = 0; k < kTlPerSite; ++k) t0 = std::min(t0, h[((size_t)sidx * kTlPerSite + k) * kTlWords]);
    int n = 0;
    for (int sidx = 0; sidx < c->tl_sites; ++sidx)
      for (int k = 0; k < kTlPerSite; ++k) {
        const tl_word* w = &h[((size_t)sidx * kTlPerSite + k) * kTlWords];
        if (w[0] == ~(tl_word)0) continue;          // not launched
        REQUIRE(n < max_kernels, SACMI_EVALUE, "max_kernels too small");
        std::memset(names_out + 32 * n, 0, 32);
        std::strncpy(names_out + 32 * n, c->tl_names[sidx].c_str(), 31);
        kind_out[n] = (int32_t)w[2];
        grid_out[n] = (int32_t)w[3];
        site_out[n] = sidx;
        start_us[n] = (double)(w[0] - t0) * 0.01;   // 100 MHz ticks -> us
        tl_word end = 0;                            // the latest exit slot (all-ones: none)
        for (int x = 0; x < kTlEndSlots; ++x)
          if (w[kTlEnd + x] != ~(tl_word)0) end = std::max(end, ~w[kTlEnd + x]);
        end_us[n] = (double)(end - t0) * 0.01;
        // the site's algorithmic work, on its first kernel
        if (flops_out) flops_out[n] = k == 0 ? c->tl_flops[sidx] : 0.0;
        if (bytes_out) bytes_out[n] = k == 0 ? c->tl_bytes[sidx] : 0.0;
        ++n;
      }
    *n_kernels = n;
  } catch (...) {
    cleanup();
    throw;
  }
  cleanup();
}
}  // extern "C++"

int sacmi_profile_timeline(sacmi_ctx* c, int32_t batch, int32_t n_updates, int32_t max_kernels,
                           char* names_out, int32_t* kind_out, int32_t* grid_out, int32_t* site_out,
                           double* start_us, double* end_us, double* flops_out, double* bytes_out,
                           int32_t* n_kernels, double* graph_us) {
  return guard([&] {
    pf_touch(c);
    mb_flush(c);
    check_device_batch(c, batch);
    REQUIRE(n_updates >= 1 && n_updates <= 256, SACMI_EVALUE, "n_updates must be in [1, 256]");
    // the same update sequence sacmi_step_many_async replays
    timeline_of(c, n_updates, [&]() { enqueue_many(c, batch, 1, 1, true, n_updates); }, max_kernels, names_out, kind_out, grid_out, site_out, start_us, end_us, flops_out,
       bytes_out, n_kernels, graph_us);
  });
}

int sacmi_profile_timeline_dp(sacmi_ctx* c, int32_t batch, int32_t n_updates, int32_t max_kernels,
                              char* names_out, int32_t* kind_out, int32_t* grid_out, int32_t* site_out,
                              double* start_us, double* end_us, double* flops_out, double* bytes_out,
                              int32_t* n_kernels, double* graph_us) {
  return guard([&] {
    pf_touch(c);
    mb_flush(c);
    REQUIRE(c->comm || c->dp_loopback, SACMI_ESTATE, "sacmi_allreduce_init has not been called");
    check_device_batch(c, batch);
    REQUIRE(n_updates >= 1 && n_updates <= 256, SACMI_EVALUE, "n_updates must be in [1, 256]");
    // the sequence sacmi_step_dp replays: phases + the two RCCL all-reduces per update
    timeline_of(c, n_updates, [&]() { enqueue_dp(c, batch, n_updates); }, max_kernels,
                names_out, kind_out, grid_out, site_out, start_us, end_us, flops_out, bytes_out,
                n_kernels, graph_us);
  });
}

static void require_per(sacmi_ctx* c) {
  REQUIRE(c->cfg.replay_kind == SACMI_REPLAY_PER, SACMI_ESTATE, "context was not created with PER replay");
}

int sacmi_per_sample(sacmi_ctx* c, int32_t batch, const double* u, int64_t* idx_out,
                     float* weights_out) {
  return guard([&] {
    pf_touch(c);
    require_per(c);
    REQUIRE(c->len > 0, SACMI_EVALUE, "probabilities do not sum to 1");   // empty buffer
    REQUIRE(batch >= 0 && batch <= c->Bm, SACMI_EVALUE, "batch must be in [0, max_batch]");
    const int k = (int)std::min<int64_t>(batch, c->len);    // replay_buffer.py:50
    if (k == 0) return;
    if (u) CHECK_HIP(hipMemcpyAsync(c->per_uin.p, u, (size_t)k * 8, hipMemcpyHostToDevice, c->stream));
    PerArgs pa = per_args(c, k, u ? 0 : 1);
    pa.skip_on_err = 0;                // a host call: the reference's sample always runs
    launch_per_sample(pa, c->stream);
    CHECK_HIP(hipGetLastError());
    if (idx_out) CHECK_HIP(hipMemcpyAsync(idx_out, c->idx64.p, (size_t)k * 8, hipMemcpyDeviceToHost, c->stream));
    if (weights_out) CHECK_HIP(hipMemcpyAsync(weights_out, c->per_w.p, (size_t)k * 4, hipMemcpyDeviceToHost, c->stream));
    int32_t err = 0;
    CHECK_HIP(hipMemcpyAsync(&c->sc_host->err, &c->sc.p->err, 4, hipMemcpyDeviceToHost, c->stream));
    CHECK_HIP(hipStreamSynchronize(c->stream));
    err = c->sc_host->err;
    if (err & ERR_NAN_PER) {           // this draw's probabilities: report and forget the bit
      c->sc_host->err = err & ~ERR_NAN_PER;
      CHECK_HIP(hipMemcpyAsync(&c->sc.p->err, &c->sc_host->err, 4, hipMemcpyHostToDevice, c->stream));
      CHECK_HIP(hipStreamSynchronize(c->stream));
      throw Error{SACMI_ENAN, "probabilities contain NaN (PrioritizedReplayBuffer.sample, replay_buffer.py:64)"};
    }
  });
}

int sacmi_per_update(sacmi_ctx* c, const int64_t* idx, const float* values, int64_t n) {
  return guard([&] {
    pf_touch(c);
    require_per(c);
    if (n <= 0) return;
    for (int64_t i = 0; i < n; ++i)
      REQUIRE(idx[i] >= 0 && idx[i] < c->capacity, SACMI_EVALUE, "index out of range");
    if ((int64_t)c->per_idx.n < n) {
      c->per_idx.release(); c->per_val.release();
      c->per_idx.alloc(n); c->per_val.alloc(n);
    }
    CHECK_HIP(hipMemcpyAsync(c->per_idx.p, idx, (size_t)n * 8, hipMemcpyHostToDevice, c->stream));
    CHECK_HIP(hipMemcpyAsync(c->per_val.p, values, (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
    launch_per_update(c->prio.p, c->per_idx.p, c->per_val.p, n, c->per_owner.p, c->stream);
    CHECK_HIP(hipGetLastError());
    CHECK_HIP(hipStreamSynchronize(c->stream));
  });
}

int sacmi_per_get_priorities(sacmi_ctx* c, float* out, int64_t n) {
  return guard([&] {
    pf_touch(c);
    require_per(c);
    REQUIRE(n >= 0 && n <= c->capacity, SACMI_EVALUE, "n > capacity");
    CHECK_HIP(hipStreamSynchronize(c->stream));
    CHECK_HIP(hipMemcpy(out, c->prio.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  });
}

int sacmi_per_set_priorities(sacmi_ctx* c, const float* in, int64_t n) {
  return guard([&] {
    pf_touch(c);
    require_per(c);
    REQUIRE(n >= 0 && n <= c->capacity, SACMI_EVALUE, "n > capacity");
    CHECK_HIP(hipStreamSynchronize(c->stream));
    CHECK_HIP(hipMemcpy(c->prio.p, in, (size_t)n * 4, hipMemcpyHostToDevice));
  });
}

// select_action (sac_imp.py:54-72): the policy forward on n states through the same
// kernels as the update (rows of the step's stacked policy input are reused).
int sacmi_act(sacmi_ctx* c, const float* states, int32_t n, int32_t deterministic,
              const float* eps, float* a_out) {
  return guard([&] {
    REQUIRE(states && a_out, SACMI_EVALUE, "null argument");
    REQUIRE(n > 0 && n <= 2 * c->Bm, SACMI_EVALUE, "n must be in [1, 2*max_batch]");
    hipStream_t s = c->stream;
    const int S = c->S, A = c->A, H = c->H, Kx = c->Kx, Hd = c->Hd;
    // env-rate calls (n <= kActPinned) go through pinned staging: no pageable-copy syncs
    const bool pinned = n <= kActPinned;
    float* h_in = c->act_host;                          // [kActPinned][Kx]
    float* h_eps = c->act_host + (size_t)kActPinned * Kx;
    float* h_out = h_eps + (size_t)kActPinned * A;
    const float* src = states;
    const float* esrc = eps;
    if (pinned) {
      for (int i = 0; i < n; ++i) std::memcpy(h_in + (size_t)i * Kx, states + (size_t)i * S, (size_t)S * 4);
      src = h_in;
      if (eps && !deterministic) {
        std::memcpy(h_eps, eps, (size_t)n * A * 4);
        esrc = h_eps;
      }
    }
    // zero-copy (default for env-rate calls): fc1 reads the states from the mapped staging
    // (its A operand, the ones column in place) and the heads kernel writes the actions back
    const bool zc = pinned && c->act_host_dev;
    const bool gemv = zc && n == 1 && A <= 32;
    // every path but the one-state GEMVs writes rows of batch set 0's x2 (the states here,
    // the actions from the heads kernel): a batch drawn ahead there is given up first
    if (!gemv) pf_touch(c);
    if (!zc) {
      CHECK_HIP(hipMemcpy2DAsync(c->x2.p, (size_t)Kx * 4, src, (size_t)(pinned ? Kx : S) * 4, (size_t)S * 4, n,
                                 hipMemcpyHostToDevice, s));
      set_column_checked(c->x2.p, n, Kx, S, 1.f, s);   // (a bf16-activation update may have
    }                                                   //  overwritten the fp32 ones column)
    // one state (the env-rate call): the policy forward as GEMVs (k_act_gemv / k_act_heads:
    // a wave per output instead of 32-row level tiles that use one row), fp32, from the
    // mapped staging, the action back into it, the host polling the heads' done word
    if (gemv) {
      const float* x = c->act_host_dev;
      int K = S + 1, ldw = c->p_fc[0].ld;
      const float* Wl = c->P.p + c->p_fc[0].off;
      for (int l = 0; l < c->nh; ++l) {
        GemvArgs g{x, Wl, ldw, K, H, c->act_h.p + (size_t)l * Hd, 1};
        launch_act_gemv(g, s);
        x = g.y; K = H + 1; ldw = Hd;
        if (l + 1 < c->nh) Wl = c->P.p + c->p_fc[l + 1].off;
      }
      ActHeadsArgs ha{};
      ha.x = x; ha.Wh = c->P.p + c->p_head.off; ha.ldw = Hd; ha.K = H + 1; ha.A = A;
      ha.deterministic = deterministic ? 1 : 0; ha.gen_eps = eps ? 0 : 1;
      ha.eps = c->act_host_dev + (h_eps - c->act_host);
      ha.seed = c->cfg.seed; ha.ctr = (1ull << 63) | (++c->act_calls);   // disjoint from update noise
      ha.scale = (float)((c->cfg.action_high - c->cfg.action_low) / 2);
      ha.bias = (float)((c->cfg.action_high + c->cfg.action_low) / 2);
      ha.out = c->act_host_dev + (h_out - c->act_host);
      *c->act_nan_host = 0;
      ha.nan_flag = c->act_nan_dev;
      ha.done_word = c->act_nan_dev + 1;
      ha.done_value = ++c->act_seq;
      launch_act_heads(ha, s);
      volatile int* done_host = reinterpret_cast<volatile int*>(c->act_nan_host + 1);
      const bool done = poll_done(done_host, s, ha.done_value, true);
      if (!done) CHECK_HIP(hipStreamSynchronize(s));
      c->done_epoch = c->epoch;
      if (!deterministic && *reinterpret_cast<volatile int*>(c->act_nan_host))
        throw Error{SACMI_ENAN, "Expected parameters loc / scale (Tensor of shape (1, " + std::to_string(A) +
                                    ")) of distribution Normal to satisfy the constraints Real() / "
                                    "GreaterThan(lower_bound=0.0), but found invalid values (NaN) in "
                                    "policy.sample(state) (select_action, sac_imp.py:70)"};
      std::memcpy(a_out, h_out, (size_t)A * 4);
      return;
    }
    if (eps && !deterministic)
      CHECK_HIP(hipMemcpyAsync(c->eps.p, esrc, (size_t)n * A * 4, hipMemcpyHostToDevice, s));
    Level l1;
    l1.add(gd(zc ? c->act_host_dev : c->x2.p, Kx, 1, c->P.p + c->p_fc[0].off, c->p_fc[0].ld, 1, c->hp[0].p, Hd,
              n, H, S + 1, EPI_RELU));
    l1.b.bf16 = c->bf16;
    launch_gemm(l1.b, s);
    for (int l = 1; l < c->nh; ++l) {
      Level lv;
      lv.add(gd_fwd_h(c->hp[l - 1].p, Hd, c->P.p + c->p_fc[l].off, Hd, c->hp[l].p, Hd, n, H, H));
      lv.b.bf16 = c->bf16;
      launch_gemm(lv.b, s);
    }
    HeadSampleArgs hs{};
    hs.h = c->hp[c->nh - 1].p; hs.Wh = c->P.p + c->p_head.off; hs.rows = n; hs.A = A; hs.K = H;
    hs.ldh = Hd; hs.ldw = Hd; hs.eps = c->eps.p; hs.gen_eps = eps ? 0 : 1; hs.seed = c->cfg.seed;
    hs.sc = c->sc.p; hs.act = c->x2.p + S + 1; hs.ldact = Kx; hs.logp = c->logp.p;
    hs.cache = c->cache.p;
    hs.scale = (float)((c->cfg.action_high - c->cfg.action_low) / 2);
    hs.bias = (float)((c->cfg.action_high + c->cfg.action_low) / 2);
    hs.deterministic = deterministic ? 1 : 0;
    hs.ctr_override = (1ull << 63) | (++c->act_calls);   // disjoint from update noise
    if (zc) hs.act_host = c->act_host_dev + (h_out - c->act_host);
    // one heads workgroup: the host polls its done word instead of the stream's completion
    const bool poll_wait = zc && n <= heads_rows_per_wg(n);
    volatile int* done_host = reinterpret_cast<volatile int*>(c->act_nan_host + 1);
    if (poll_wait) {
      hs.done_word = c->act_nan_dev + 1;
      hs.done_value = ++c->act_seq;
    }
    // Normal(mean, std) validation of policy.sample (networks_model1.py:87; evaluate=True
    // takes tanh(mean) without one): a plain store into host-mapped memory
    *c->act_nan_host = 0;
    hs.nan_flag = c->act_nan_dev; hs.nan_bit_lo = hs.nan_bit_hi = 1; hs.nan_plain = 1;
    launch_heads_sample(hs, s);
    CHECK_HIP(hipGetLastError());
    if (!zc)
      CHECK_HIP(hipMemcpy2DAsync(pinned ? h_out : a_out, (size_t)A * 4, c->x2.p + S + 1, (size_t)Kx * 4,
                                 (size_t)A * 4, n, hipMemcpyDeviceToHost, s));
    bool done = false;
    if (poll_wait) done = poll_done(done_host, s, hs.done_value, true);
    if (!done) CHECK_HIP(hipStreamSynchronize(s));
    c->done_epoch = c->epoch;
    if (!deterministic && *reinterpret_cast<volatile int*>(c->act_nan_host))
      throw Error{SACMI_ENAN, "Expected parameters loc / scale (Tensor of shape (" + std::to_string(n) + ", " +
                                  std::to_string(A) + ")) of distribution Normal to satisfy the constraints "
                                  "Real() / GreaterThan(lower_bound=0.0), but found invalid values (NaN) in "
                                  "policy.sample(state) (select_action, sac_imp.py:70)"};
    if (pinned) std::memcpy(a_out, h_out, (size_t)n * A * 4);
  });
}

// Host-only self test of the launch validator (no device needed): host arrays stand in
// for registered allocations, and every case states whether validate() / validate_batch()
// must accept or reject it.
int sacmi_selftest_span_checker(int32_t* n_cases, int32_t* n_passed) {
  return guard([&] {
    REQUIRE(n_cases && n_passed, SACMI_EVALUE, "null argument");
    const int M = 64, N = 64, K = 128, ld = 132;
    std::vector<float> a((size_t)M * ld), w((size_t)N * ld), out((size_t)M * ld), ws(4096);
    std::vector<unsigned short> wh((size_t)N * ld), wh_short((size_t)N * ld - 8);
    // a registry of its own (thread-local override): the process registry, which other
    // threads' contexts may be changing, is neither read nor written
    std::vector<AllocRec> reg;
    for (auto* v : {&a, &w, &out, &ws})
      reg.push_back({(uintptr_t)v->data(), v->size() * sizeof(float)});
    for (auto* v : {&wh, &wh_short})
      reg.push_back({(uintptr_t)v->data(), v->size() * sizeof(unsigned short)});
    struct Override {
      explicit Override(const std::vector<AllocRec>* r) { g_registry_override = r; }
      ~Override() { g_registry_override = nullptr; }
    } use_local(&reg);
    struct Case { bool accept; GemmBatch b; };
    std::vector<Case> cases;
    auto base = [&]() {
      GemmBatch b{};
      b.count = 1;
      b.d[0] = gd(a.data(), ld, 1, w.data(), ld, 1, out.data(), ld, M, N, K, EPI_RELU);
      return b;
    };
    { Case k{true, base()}; cases.push_back(k); }                           // plain level
    { Case k{true, base()}; k.b.d[0].Bh = wh.data(); cases.push_back(k); }  // full shadow
    { Case k{false, base()}; k.b.d[0].Bh = wh_short.data(); cases.push_back(k); }   // short shadow
    { Case k{false, base()}; k.b.d[0].Bh = wh.data() + 8; cases.push_back(k); }     // shadow past its end
    { Case k{true, base()}; k.b.ws = ws.data(); k.b.ws_floats = 4096; cases.push_back(k); }
    { Case k{false, base()}; k.b.ws = ws.data(); k.b.ws_floats = 4097; cases.push_back(k); }  // claims more
    { Case k{false, base()}; k.b.ws = ws.data() + 4; k.b.ws_floats = 4096; cases.push_back(k); }
    { Case k{false, base()}; k.b.ws_floats = 16; cases.push_back(k); }      // capacity, no buffer
    { Case k{false, base()}; k.b.d[0].B = w.data() + 8; cases.push_back(k); }       // B past its end
    {  // MN-contiguous operand read 4 wide from a 4-aligned start: M = 62 still spans 64
      Case k{true, base()};
      k.b.d[0] = gd(a.data(), ld, 0, w.data(), ld, 0, out.data(), ld, 62, 62, 64, EPI_STORE);
      cases.push_back(k);
      Case k2{false, base()};
      k2.b.d[0] = gd(a.data() + ld * 64 - 64, ld, 0, w.data(), ld, 0, out.data(), ld, 62, 62, 64, EPI_STORE);
      cases.push_back(k2);
    }
    int pass = 0;
    for (const Case& k : cases) {
      bool ok = true;
      try {
        for (int i = 0; i < k.b.count; ++i) validate(k.b.d[i]);
        validate_batch(k.b);
      } catch (const Error&) {
        ok = false;
      }
      pass += ok == k.accept;
    }
    // the host-launched conversions (refresh_shadows / the sharded gather's shadow pass):
    // an arena of `total` floats plus the data-parallel slack and its bf16 shadow.  Round 4
    // sized the shadow at `total` and converted the whole arena: 8 KB past the shadow's end
    const int64_t total = 1000, slack = 64;
    std::vector<float> arena((size_t)(total + slack));
    std::vector<unsigned short> shadow_full((size_t)(total + slack)), shadow_short((size_t)total);
    reg.push_back({(uintptr_t)arena.data(), arena.size() * sizeof(float)});
    reg.push_back({(uintptr_t)shadow_full.data(), shadow_full.size() * sizeof(unsigned short)});
    reg.push_back({(uintptr_t)shadow_short.data(), shadow_short.size() * sizeof(unsigned short)});
    struct Conv { bool accept; unsigned short* dst; const float* src; int64_t n; };
    const Conv conv[] = {
        {true, shadow_full.data(), arena.data(), total + slack},     // the whole arena
        {true, shadow_short.data(), arena.data(), total},            // the layout only
        {false, shadow_short.data(), arena.data(), total + slack},   // round 4's overrun
        {true, shadow_full.data() + 64, arena.data() + 64, total + slack - 64},   // a chunk
        {false, shadow_full.data() + 64, arena.data() + 64, total + slack},       // past both
    };
    for (const Conv& k : conv) {
      bool ok = true;
      try {
        check_to_bf16(k.dst, k.src, k.n);
      } catch (const Error&) {
        ok = false;
      }
      pass += ok == k.accept;
    }
    *n_cases = (int32_t)(cases.size() + sizeof(conv) / sizeof(conv[0]));
    *n_passed = pass;
  });
}

}  // extern "C"
