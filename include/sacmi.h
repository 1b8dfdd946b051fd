/*
 * sacmi.h — C ABI of the MI355X-native SAC gradient-step library (libsacmi.so).
 *
 * This is the drop-in boundary for the reference's hot path
 * (FilippoCrc/Humanoid-walking-with-SAC, snapshot 2025-02-22):
 *
 *   sac_imp.SAC.__init__            sac_imp.py:9-52        -> sacmi_create
 *   sac_imp.SAC.update_parameters   sac_imp.py:74-144      -> sacmi_step / sacmi_step_async
 *   trainer updates_per_step loop   trainer.py:203-204     -> sacmi_step_many_async
 *   sac_imp.SAC._soft_update_...    sac_imp.py:146-152     -> (inside sacmi_step)
 *   sac_imp.SAC.select_action       sac_imp.py:54-72       -> sacmi_act
 *   nn.Module.state_dict / load     sac_imp.py:154-233     -> sacmi_get_tensor / sacmi_set_tensor
 *   ReplayBuffer.push / __len__     replay_buffer.py:10-11,21-22   -> sacmi_push / sacmi_len
 *   ReplayBuffer.sample (indices)   replay_buffer.py:13-19 -> sacmi_sample_indices (+ inside step)
 *   ReplayBuffer.buffer (read)      sac_imp.py:199          -> sacmi_get_rows
 *   PrioritizedReplayBuffer.sample  replay_buffer.py:48-82 -> sacmi_per_sample
 *   PrioritizedReplayBuffer.update_priorities  replay_buffer.py:84-87 -> sacmi_per_update
 *   random.getstate/setstate, np.random.get_state/set_state -> sacmi_rng_get_mt / sacmi_rng_set_mt
 *
 * Conventions
 *   - Every call returns int status: 0 = OK, otherwise an SACMI_E* code; the message
 *     is in sacmi_last_error() (thread-local).  The Python host maps codes to the
 *     reference's exceptions (ValueError for SACMI_EVALUE, RuntimeError otherwise).
 *   - One context per GPU.  All device work of a context is ordered on its HIP stream
 *     (its own, or one supplied by sacmi_set_stream).  A context is not thread-safe.
 *   - The library owns all device memory; every host pointer argument is copied in
 *     or out before the call returns (except sacmi_step_async, which writes nothing
 *     to host memory).
 *   - Plain C types only: no torch / HIP types cross this boundary.
 */
#ifndef SACMI_H_
#define SACMI_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 3 (round 6): sacmi_step_chained removed (the persistent-chain kernels are gone);
 * sacmi_grad_buffer(0)'s view documents its trailing error-flag words (kDpFlagN). */
#define SACMI_ABI_VERSION 3

enum sacmi_status {
  SACMI_OK = 0,
  SACMI_EVALUE = 1,    /* bad argument (maps to ValueError)          */
  SACMI_ESTATE = 2,    /* call not valid in the current state        */
  SACMI_EDEVICE = 3,   /* HIP runtime error / no device              */
  SACMI_ENAN = 4,      /* non-finite value surfaced (maps to ValueError, as Normal(validate_args)) */
};

enum sacmi_replay_kind { SACMI_REPLAY_UNIFORM = 0, SACMI_REPLAY_PER = 1 };

/* arithmetic of the MLP GEMMs: fp32 (exact f32 MFMA, the reference's precision) or bf16
 * (bf16 MFMA operands, fp32 accumulation; fp32 master weights, Adam, losses and row
 * algebra) — BASELINE configs[4] */
enum sacmi_compute_dtype { SACMI_COMPUTE_FP32 = 0, SACMI_COMPUTE_BF16 = 1 };

typedef struct sacmi_config {
  int32_t state_dim;          /* S  (sac_imp.py:11)                               */
  int32_t action_dim;         /* A  (sac_imp.py:12)                               */
  int32_t hidden_dim;         /* H  (sac_imp.py:13, default 256)                  */
  int32_t max_batch;          /* largest batch_size passed to step / act          */
  double gamma;               /* 0.99  (sac_imp.py:14)                            */
  double tau;                 /* 0.005 (sac_imp.py:15)                            */
  double lr;                  /* 3e-4  (sac_imp.py:16)                            */
  double alpha;               /* 0.2   (sac_imp.py:17) alpha used until the 1st update */
  int32_t auto_entropy;       /* automatic_entropy_tuning (sac_imp.py:18)          */
  int32_t replay_kind;        /* sacmi_replay_kind                                 */
  double action_low;          /* action_bounds (networks_model1.py:52-55)         */
  double action_high;
  int64_t capacity;           /* ReplayBuffer(capacity=1e6) (replay_buffer.py:7)  */
  double per_alpha;           /* 0.6   (replay_buffer.py:26)                      */
  double per_beta_start;      /* 0.4                                             */
  double per_beta_frames;     /* 1e5                                             */
  uint64_t seed;              /* Philox seed for the policy noise (perf mode)     */
  int32_t n_hidden;           /* hidden layers per net: 2 = networks_model1 (the  */
                              /* reference's SAC, sac_imp.py:4), 3 = networks_model2 */
                              /* (networks_model2.py:18-99); 0 means 2            */
  int32_t compute_dtype;      /* sacmi_compute_dtype                              */
} sacmi_config;

typedef struct sacmi_ctx sacmi_ctx;

/* Tensor ids for get/set.  Layout of every tensor is the reference nn.Linear /
 * optimizer layout: weight [out, in] row-major, bias [out]. */
enum sacmi_net { SACMI_POLICY = 0, SACMI_Q1 = 1, SACMI_Q2 = 2, SACMI_Q1_TARGET = 3,
                 SACMI_Q2_TARGET = 4 };
enum sacmi_slot { SACMI_SLOT_PARAM = 0, SACMI_SLOT_GRAD = 1, SACMI_SLOT_ADAM_M = 2,
                  SACMI_SLOT_ADAM_V = 3 };
/* layer index inside a net (n_hidden = 2): policy {0: fc1, 1: fc2, 2: mean, 3: log_std};
 * q {0: fc1, 1: fc2, 2: fc3}.  n_hidden = 3 (networks_model2): policy {0: fc1, 1: fc2,
 * 2: fc3, 3: mean, 4: log_std}; q {0: fc1, 1: fc2, 2: fc3, 3: fc4}.
 * part: 0 = weight, 1 = bias. */

/* scalar ids for get/set_scalar */
enum sacmi_scalar {
  SACMI_S_LOG_ALPHA = 0,       /* log_alpha (sac_imp.py:48)                          */
  SACMI_S_ALPHA = 1,           /* current alpha (0.2 float before the 1st update)    */
  SACMI_S_ALPHA_IS_TENSOR = 2, /* 1 once alpha = log_alpha.exp() (sac_imp.py:135)   */
  SACMI_S_STEP_POLICY = 3,     /* Adam 'step' of each optimizer                     */
  SACMI_S_STEP_Q1 = 4,
  SACMI_S_STEP_Q2 = 5,
  SACMI_S_STEP_ALPHA = 6,
  SACMI_S_ADAM_M_LOG_ALPHA = 7,
  SACMI_S_ADAM_V_LOG_ALPHA = 8,
  SACMI_S_GRAD_LOG_ALPHA = 9,
  SACMI_S_PER_FRAME = 10,      /* PrioritizedReplayBuffer.frame (replay_buffer.py:31) */
  SACMI_S_NOISE_COUNTER = 11,  /* Philox counter (updates drawn so far)             */
  SACMI_S_KEEP_GRADS = 12,     /* host flag: 1 = single-GPU updates also export the   */
                               /* gradients to the GRAD slot (param.grad after        */
                               /* backward); 0 (default) skips those stores           */
  SACMI_S_GRAPH_COUNT = 13,    /* read-only: instantiated update graphs cached by the  */
                               /* context (one per distinct update configuration)     */
  SACMI_S_COUNT = 14
};

/* ---- lifecycle ---------------------------------------------------------------- */
int sacmi_abi_version(void);
const char* sacmi_last_error(void);
int sacmi_device_count(int* n);
int sacmi_create(const sacmi_config* cfg, int device, sacmi_ctx** out);
int sacmi_destroy(sacmi_ctx* ctx);
/* Order all work on an external HIP stream (e.g. torch's current stream), passed
 * as an opaque pointer; NULL returns to the context's own stream. */
int sacmi_set_stream(sacmi_ctx* ctx, void* hip_stream);
int sacmi_synchronize(sacmi_ctx* ctx);

/* ---- parameters / optimizer state (state_dict bridge) ------------------------ */
int sacmi_tensor_numel(sacmi_ctx* ctx, int net, int layer, int part, int64_t* numel);
int sacmi_set_tensor(sacmi_ctx* ctx, int slot, int net, int layer, int part,
                     const float* host, int64_t numel);
int sacmi_get_tensor(sacmi_ctx* ctx, int slot, int net, int layer, int part,
                     float* host, int64_t numel);
int sacmi_set_scalar(sacmi_ctx* ctx, int which, double value);
int sacmi_get_scalar(sacmi_ctx* ctx, int which, double* value);

/* ---- replay (HBM ring, SoA) ----------------------------------------------------- */
/* Append n transitions (copy-in).  s,s2: [n,S] f32; a: [n,A] f32; r: [n] f32;
 * d: [n] u8.  Oldest rows are evicted past capacity (deque(maxlen)).  For PER the
 * new rows get max(priorities) (or 1.0 when empty), replay_buffer.py:36-46. */
int sacmi_push(sacmi_ctx* ctx, const float* s, const float* a, const float* r,
               const float* s2, const uint8_t* d, int64_t n);
/* The same from packed rows [n][2S + A + 2] f32: s | a | r | s2 | d (d: 0 or 1).  Up to
 * 16 rows a chunk are read by the scatter kernel straight from mapped staging (the
 * trainer's row per env step: no copy command ahead of the next update). */
int sacmi_push_packed(sacmi_ctx* ctx, const float* rows, int64_t n);
int sacmi_len(sacmi_ctx* ctx, int64_t* n);
/* Empty the replay: the assignment `replay_buffer.buffer = rows` of checkpoint loading
 * (sac_imp.py:229-230) replaces the contents, so the rows pushed next start a fresh deque.
 * PER priorities are left as they are (the reference's list assignment does not touch its
 * priority array, replay_buffer.py:28-30). */
int sacmi_replay_clear(sacmi_ctx* ctx);
/* Copy rows at deque positions idx[0..n) out (materialises ReplayBuffer.buffer). */
int sacmi_get_rows(sacmi_ctx* ctx, const int64_t* idx, int64_t n, float* s, float* a,
                   float* r, float* s2, uint8_t* d);

/* Same, addressed by ring slot (PrioritizedReplayBuffer indices are list positions
 * = ring slots, replay_buffer.py:40-44,73). */
int sacmi_get_slots(sacmi_ctx* ctx, const int64_t* slots, int64_t n, float* s, float* a,
                    float* r, float* s2, uint8_t* d);

/* ---- RNG bridges ----------------------------------------------------------------- */
/* stream 0 = CPython `random` (uniform indices), stream 1 = numpy legacy
 * RandomState (PER).  key: 624 words, pos: index 0..624. */
int sacmi_rng_set_mt(sacmi_ctx* ctx, int stream, const uint32_t* key, int32_t pos);
int sacmi_rng_get_mt(sacmi_ctx* ctx, int stream, uint32_t* key, int32_t* pos);

/* Perf-mode policy noise (eps of GaussianPolicy.sample, networks_model1.py:87-90 — the
 * reference draws it from torch's generator): Philox4x32-10 keyed by `seed`, counter
 * `offset` + one per update.  Replaces the seed given at create time; the next update
 * re-captures its graphs. */
int sacmi_rng_seed_device(sacmi_ctx* ctx, uint64_t seed, uint64_t offset);

/* random.sample(buffer, batch) positions, drawn on the GPU from stream 0 (advances it). */
int sacmi_sample_indices(sacmi_ctx* ctx, int32_t batch, int64_t* idx_out);

/* ---- the gradient step ----------------------------------------------------------- */
/* One update_parameters(batch): sample (uniform: device MT stream 0 unless idx is
 * given; PER contexts: the device PER sampler on stream 1, ring-slot indices), gather, target, twin-critic step, actor step, alpha step, Polyak.
 * idx:  NULL -> draw on device; else [batch] deque positions.
 * eps1, eps2: NULL -> on-device Philox noise; else [batch, A] standard normals
 *   (eps1 for policy.sample(next_state), eps2 for policy.sample(state)).
 * losses_out (may be NULL): {q1_loss, q2_loss, policy_loss} — synchronises. */
int sacmi_step(sacmi_ctx* ctx, int32_t batch, const int64_t* idx, const float* eps1,
               const float* eps2, float* losses_out);
/* Non-finite inputs (SACMI_ENAN -> ValueError), where the reference raises:
 *   - a NaN policy mean / log_std fed to Normal(mean, std) (networks_model1.py:87) in
 *     policy.sample(next_state) (sac_imp.py:89: the update takes no step) or in
 *     policy.sample(state) (:116: the critic step is taken, the actor / alpha / Polyak
 *     steps are not); select_action(evaluate=False) likewise (sacmi_act);
 *   - NaN PER probabilities (np.random.choice, replay_buffer.py:64: the frame advances, the
 *     numpy stream does not).
 * The device records it and every later update of the stream takes no step (a
 * multi-update launch stops where the reference's loop raised).  sacmi_step (with
 * losses_out), sacmi_fetch_losses, sacmi_per_sample and sacmi_act report it and forget it. */
/* sacmi_step(ctx, batch, NULL, NULL, NULL, losses_out) in two halves: the launch
 * (device indices + device noise; returns at once) and the wait (synchronises, writes the
 * losses, reports SACMI_ENAN like sacmi_step).  Between them the caller's thread is free
 * — the drop-in advances Python's `random` there by the reference's own random.sample
 * (sac_imp.py:75 -> replay_memory.py sample) while the GPU runs the update.  Every launch
 * is followed by exactly one wait; nothing else may be called on the context between. */
int sacmi_step_launch(sacmi_ctx* ctx, int32_t batch);
int sacmi_step_wait(sacmi_ctx* ctx, float* losses_out);
/* Same work, enqueued only (no host sync, no host writes); losses stay on device
 * in a ring of `ring` slots, fetched by sacmi_fetch_losses. */
int sacmi_step_async(sacmi_ctx* ctx, int32_t batch);
/* n_updates consecutive updates (device indices + device noise) as ONE launch: the
 * `for _ in range(updates_per_step): agent.update_parameters(batch_size)` loop of
 * trainer.py:203-204.  Identical results to n_updates sacmi_step_async calls; every
 * update's losses go to the ring.  1 <= n_updates <= 256. */
int sacmi_step_many_async(sacmi_ctx* ctx, int32_t batch, int32_t n_updates);
int sacmi_fetch_losses(sacmi_ctx* ctx, float* out, int32_t max_steps, int32_t* n_out);

/* Data-parallel split of the step (one process per GPU).  phase 0: sample, gather,
 * forward, critic backward -> critic gradient buffer; phase 1: critic Adam + Polyak,
 * actor forward/backward -> actor gradient buffer; phase 2: actor Adam + alpha;
 * phase 3: phase 2 of the previous update then phase 0 of the next, in one launch
 * (no collective sits between them).
 * Between phases the caller all-reduces (sum) the buffer named by
 * sacmi_grad_buffer(which=0 critic, 1 actor); grad_scale (1/world) is applied by the
 * Adam kernels. */
int sacmi_step_phase(sacmi_ctx* ctx, int32_t batch, int32_t phase, float grad_scale);
/* The same with the minibatch buffer sets spelled out, for a fixed sequence of split
 * updates (e.g. one captured into a graph by the caller): parity (0/1) = the buffer set
 * of the update whose phase 0 (phase 3: the NEXT update) / phase 1 runs; have_batch =
 * its indices and rows were produced by the previous update (phases 0, 3); ride_next =
 * the phase-1 launches also sample and gather the next update into set parity^1
 * (uniform replay only, sacmi_step_ride_possible).  The caller guarantees that nothing
 * changes the replay buffer or the sampling stream between a ride and its use. */
int sacmi_step_phase_ex(sacmi_ctx* ctx, int32_t batch, int32_t phase, float grad_scale,
                        int32_t parity, int32_t have_batch, int32_t ride_next);
int sacmi_step_ride_possible(sacmi_ctx* ctx, int32_t batch, int32_t* out);
/* 1 when updates of this batch store their activations as bf16 (compute_dtype bf16 at the
 * batch-4096 class: hidden layers, minibatch rows and sampled actions; the policy heads
 * then read a bf16-rounded input), else 0. */
int sacmi_step_act16(sacmi_ctx* ctx, int32_t batch, int32_t* out);
/* Test hook: the hidden activations (post-ReLU) the last update of `batch` rows left in
 * HBM, hidden layer `layer` (0-based) of pass
 *   0  the critics on (s, a)            -> [2][batch][hidden]  (q1, then q2)
 *   1  the target critics on (s', a')   -> [2][batch][hidden]
 *   2  the updated critics on (s, a~)   -> [2][batch][hidden]
 *   3  the policy on [s' ; s]           -> [2 * batch][hidden]
 * (numel = 2 * batch * hidden).  Their signs are the ReLU masks the update's backward used:
 * the parity tests recompute the fp64 gradient under the GPU's own masks.  SACMI_ESTATE for
 * bf16-stored activations (sacmi_step_act16). */
int sacmi_read_activation(sacmi_ctx* ctx, int32_t pass, int32_t layer, int32_t batch, float* out,
                          int64_t numel);
/* Test hook: the minibatch of the last device-sampled update of `batch` rows that used batch
 * set 0 (every single update, and the first of a multi-update graph): its replay indices
 * (idx[batch]: deque positions, or ring slots for PER) and the policy noise it drew
 * (eps[2 * batch * action_dim]: rows [0, batch) for policy.sample(next_state), rows [batch,
 * 2 batch) for policy.sample(state), sac_imp.py:89,116). */
int sacmi_read_batch(sacmi_ctx* ctx, int32_t batch, int64_t* idx, float* eps, int64_t eps_numel);
/* The gradient range a phase-split update's collective covers, in the gradient arena:
 * which = 0 the critic range [q1 | q2] FOLLOWED BY 4 error-flag floats (kDpFlagN: flag 0 =
 * this update saw a skip-all non-finite input, flag 1 = an actor-batch one, 2-3 zero) — they
 * travel with the critic all-reduce so that every rank voids the same steps; a grad norm or
 * clip over this view must exclude the last 4 floats.  which = 1 the actor range [policy |
 * log_alpha]. */
int sacmi_grad_buffer(sacmi_ctx* ctx, int which, void** device_ptr, int64_t* numel);
/* Gradient arena size (floats) and adoption of a caller-allocated device buffer of
 * that size (e.g. a torch tensor), so collectives run on it in place.  Must be on the
 * context's device and stay alive for the context's lifetime. */
int sacmi_grad_arena_numel(sacmi_ctx* ctx, int64_t* numel);
int sacmi_attach_grad_arena(sacmi_ctx* ctx, void* device_ptr, int64_t numel);

/* ---- native data parallel (RCCL over xGMI, no host framework) ------------------------ */
/* The same split update with the two gradient all-reduces issued by the library itself
 * (SURVEY §8(b) sacmi_allreduce_init; sac_imp.py:101-125 is the single-process update it
 * distributes).  One process per GPU: rank 0 creates the RCCL unique id
 * (sacmi_allreduce_unique_id, SACMI_RCCL_ID_BYTES bytes) and hands it to every rank by any
 * host channel; each rank then calls sacmi_allreduce_init on its context.  RCCL is loaded
 * at run time (dlopen: the process's already-loaded librccl if any, else
 * $SACMI_RCCL_PATH, else librccl.so.1): libsacmi itself has no link dependency on it. */
#define SACMI_RCCL_ID_BYTES 128
int sacmi_allreduce_unique_id(void* id_out, int32_t nbytes);
int sacmi_allreduce_init(sacmi_ctx* ctx, const void* id, int32_t nbytes, int32_t rank,
                         int32_t world);
/* n_updates complete data-parallel updates (every rank the same n): per update phase 0
 * (phase 3 after the first), all-reduce(sum) of the critic gradients, phase 1,
 * all-reduce of [actor gradients | dL/dlog_alpha], the last phase 2 at the end; updates
 * 2..n take their minibatch from the previous update's ride-along sampling/gather when
 * the replay allows it.  Captured into one hipGraph per (batch, n_updates); losses land in
 * the loss ring (sacmi_fetch_losses).  Each rank samples its own replay shard.
 * Sharded form (opt-in, 2 <= world <= 64: $SACMI_DP_SHARD=1 at sacmi_allreduce_init or
 * sacmi_dp_set_sharded): each all-reduce + Adam becomes reduce-scatter -> Adam on
 * this rank's 1/world chunk of the range -> all-gather of the parameters (ZeRO-1: the Adam
 * moments stay valid on the rank's own chunks; sacmi_dp_sync_state gathers them).
 * world == 1: the fused update (nothing to reduce; $SACMI_DP_PHASES_AT_WORLD1 forces the
 * phase sequence). */
int sacmi_step_dp(sacmi_ctx* ctx, int32_t batch, int32_t n_updates);
/* Sharded (1) or all-reduce (0) form of sacmi_step_dp; the same on every rank.  Leaving
 * the sharded form is a collective (every rank): it gathers the Adam moments first, as
 * sacmi_dp_sync_state does, since the all-reduce form steps every element from them. */
int sacmi_dp_set_sharded(sacmi_ctx* ctx, int32_t on);
int sacmi_dp_sharded(sacmi_ctx* ctx, int32_t* on);
/* Collective (every rank): all-gather the sharded Adam moments so that every rank holds
 * them whole (before sacmi_get_tensor of SACMI_SLOT_ADAM_M / _V, a checkpoint).  No-op
 * when not sharded. */
int sacmi_dp_sync_state(sacmi_ctx* ctx);
/* Test hook for the sequence above on ONE context, no RCCL: every all-reduce becomes an
 * in-place x world over the same gradient range — what `world` ranks holding identical
 * shards would reduce to — while the Adam kernels apply 1/world as in a real run.  For a
 * power-of-two world both scalings are exact, so sacmi_step_dp must equal the fused
 * updates bit for bit: every gradient element, dL/dlog_alpha included, must sit inside an
 * all-reduced range and 1/world must be applied exactly once. */
int sacmi_dp_loopback_init(sacmi_ctx* ctx, int32_t world);
/* (Sharded form under loopback: the gradients x world in place, Adam on every rank's chunk
 * in turn — rank 0's launch alone finalising the losses — and the gather an identity.) */

/* ---- prioritized replay ------------------------------------------------------------ */
/* PrioritizedReplayBuffer.sample(batch) indices + IS weights; u: NULL -> draw from
 * MT stream 1 on device, else [min(batch,len)] uniforms in [0,1).  Advances frame. */
int sacmi_per_sample(sacmi_ctx* ctx, int32_t batch, const double* u, int64_t* idx_out,
                     float* weights_out);
/* priorities[idx[i]] = values[i] in order i = 0..n-1 (last duplicate wins), where the
 * caller passes the reference's stored value float32(float(p) + 1e-6)
 * (replay_buffer.py:87; the +1e-6 is a double add, done host-side). */
int sacmi_per_update(sacmi_ctx* ctx, const int64_t* idx, const float* values, int64_t n);
int sacmi_per_get_priorities(sacmi_ctx* ctx, float* out, int64_t n);
int sacmi_per_set_priorities(sacmi_ctx* ctx, const float* in, int64_t n);

/* ---- action selection (sac_imp.py:54-72) ----------------------------------------- */
/* n states [n,S] -> actions [n,A]; deterministic: tanh(mean)*scale+bias;
 * else policy.sample with eps [n,A] (NULL -> Philox). */
int sacmi_act(sacmi_ctx* ctx, const float* s, int32_t n, int32_t deterministic,
              const float* eps, float* a_out);

/* ---- diagnostics ------------------------------------------------------------------ */
/* Run `iters` eager (non-graph) updates with a HIP event recorded on the context's
 * stream between consecutive kernel launches; returns, per launch site, its name
 * (32 bytes each, NUL-padded), the mean duration in ms and the algorithmic FLOPs of
 * one launch (GEMM sites; 0 elsewhere).  The model state advances as in sacmi_step. */
int sacmi_profile_step(sacmi_ctx* ctx, int32_t batch, int32_t iters, char* names_out,
                       float* ms_out, double* flops_out, int32_t max_sites, int32_t* n_sites);
/* Per launch site of the single-GPU update: that site's kernels alone, `reps` times
 * back to back inside one hipGraph, timed with HIP events on the context's stream;
 * us_out = mean microseconds per launch of the site (the duration the kernel has in
 * the step's graph, boundary included); flops_out / bytes_out (may be NULL) = the
 * algorithmic FLOPs / bytes of one launch (GEMM sites; 0 elsewhere).  Diagnostic:
 * every replay advances the model state again (Adam sites take `reps` extra steps). */
int sacmi_profile_sites(sacmi_ctx* ctx, int32_t batch, int32_t reps, char* names_out,
                        float* us_out, double* flops_out, double* bytes_out, int32_t max_sites,
                        int32_t* n_sites);

/* Launch timeline of the real update: n_updates consecutive updates exactly as
 * sacmi_step_many_async runs them (device sampling + noise, ride-along sampling, one
 * hipGraph), captured with every kernel stamping its first workgroup's entry and its last
 * workgroup's exit on the GPU's 100 MHz real-time clock.  Replayed once to warm up, then
 * once measured; returns per kernel launch, in launch order: the launch site's name (32
 * bytes, NUL-padded), the kernel kind (TlKind in csrc/sacmi_internal.h), its grid, the
 * site index (sites count across updates), start / end in microseconds from the first
 * kernel's start, the site's algorithmic FLOPs / bytes (GEMM sites, on the site's first
 * kernel; may be NULL); graph_us = HIP-event time of the measured replay.  Diagnostic: the model
 * state advances by 2 * n_updates updates. */
int sacmi_profile_timeline(sacmi_ctx* ctx, int32_t batch, int32_t n_updates, int32_t max_kernels,
                           char* names_out, int32_t* kind_out, int32_t* grid_out, int32_t* site_out,
                           double* start_us, double* end_us, double* flops_out, double* bytes_out,
                           int32_t* n_kernels, double* graph_us);

/* sacmi_profile_timeline over the data-parallel sequence sacmi_step_dp replays (phases +
 * the two RCCL all-reduces of every update; needs sacmi_allreduce_init, and every rank of
 * the communicator must make the same call, since the captured graph holds the
 * collectives).  The all-reduces launch no stamping kernel: their time is the gap before
 * the next kernel's start. */
int sacmi_profile_timeline_dp(sacmi_ctx* ctx, int32_t batch, int32_t n_updates, int32_t max_kernels,
                              char* names_out, int32_t* kind_out, int32_t* grid_out, int32_t* site_out,
                              double* start_us, double* end_us, double* flops_out, double* bytes_out,
                              int32_t* n_kernels, double* graph_us);

/* Host-only self test of the launch validator every GEMM level passes before it is
 * enqueued (operand spans against the registered device allocations, incl. the bf16
 * weight shadows and the split-K workspace): runs a fixed set of accept / reject cases
 * on host arrays; n_passed == n_cases when the validator decides each one correctly.
 * Needs no device. */
int sacmi_selftest_span_checker(int32_t* n_cases, int32_t* n_passed);

#ifdef __cplusplus
}
#endif
#endif /* SACMI_H_ */
