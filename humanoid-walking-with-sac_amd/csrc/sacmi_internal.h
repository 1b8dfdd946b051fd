// Internal declarations of libsacmi: device layout + kernel launchers.
//
// Data layout in HBM (fp32 unless noted) — see DESIGN.md §3:
//   * Every nn.Linear is stored "bias-folded": W~ = [W | b] with one extra input
//     column, so every activation matrix carries a constant-1 column and a single
//     MFMA GEMM produces both y = x W^T + b (forward) and [dW | db] = dY^T x~
//     (backward).  Row stride `ld` is padded to a multiple of 4 floats (16 B) and the
//     pad is kept at exactly 0.
//   * The critic input is [s | 1 | a | 0-pad] (bias column between state and
//     action) so the policy can read its input [s | 1] from the same rows.
//   * Trained parameters live in one flat arena ordered
//       [q1.fc1 q2.fc1 | q1.fc2 q2.fc2 | q1.fc3 q2.fc3 | policy.fc1 policy.fc2
//        policy.head(mean rows ; log_std rows) | log_alpha]
//     (twin fc1 adjacent so dL/da of both critics is ONE GEMM with K = 2H); the
//     gradient, Adam m and Adam v arenas mirror it, the target arena mirrors the
//     critic part.  Critic grads and actor grads are each contiguous (one
//     all-reduce each in data-parallel mode).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/sacmi.h"

namespace sacmi {

constexpr int kWave = 64;

// Errors thrown inside the library and mapped to a status code by the C ABI's guard().
struct Error {
  int code;
  std::string msg;
};

// A failed kernel launch (bad configuration, LDS over the limit, ...) is an error of the
// call that enqueued it: the launchers throw instead of printing and carrying on with
// stale outputs.
inline void launch_check(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    throw Error{SACMI_EDEVICE, std::string("kernel launch failed (") + what + "): " + hipGetErrorString(e)};
}

// hipFuncAttributeMaxDynamicSharedMemorySize is a per-device attribute: raise it once per
// (kernel, device) to the largest request seen.
void ensure_dyn_lds(const void* kernel, size_t bytes);

// Output stores of the update's kernels are write-through (sc1): a kernel then leaves no
// dirty L2 lines behind, and the end-of-kernel L2 writeback — serialised at the boundary
// to the next dependent kernel, ~B / 6 TB/s for B dirty bytes — has nothing to do (the
// Adam levels write 15-30 MB of optimizer state per update).
constexpr int kStAux = 16;   // raw buffer store cache-policy bits (16 = sc1)
// The large-batch bf16 level kernels (k_fwd16 / k_axk16 / k_dw_part16 / k_dw_fin) store
// tens of MB per launch as one dword per lane: there write-through measured slower (config
// 5: 415 -> 447 us per update, the kernel bodies grew more than the boundaries shrank), so
// they keep plain stores (st_big).
template <bool WT = true, class T>
__device__ __forceinline__ void st_wt(T* p, T v) {
  if constexpr (WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
template <class T>
__device__ __forceinline__ void st_big(T* p, T v) { st_wt<false>(p, v); }

// 16-byte write-through store at a wave-uniform base + per-lane byte offset (raw buffer
// store; the LLVM intrinsic is bound directly, see kernels.hip buf_ld4)
typedef float wt_f4 __attribute__((ext_vector_type(4)));
__device__ void llvm_raw_buffer_store_wt_v4f32(wt_f4 v, __amdgpu_buffer_rsrc_t r, int off, int soff,
                                               int aux) __asm("llvm.amdgcn.raw.ptr.buffer.store.v4f32");
__device__ __forceinline__ void st_wt4(float* base, uint32_t byte_off, float4 v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
  llvm_raw_buffer_store_wt_v4f32(wt_f4{v.x, v.y, v.z, v.w}, r, (int)byte_off, 0, kStAux);
}

// 8-byte and 2-byte write-through stores (bf16 minibatch rows under act16)
typedef int wt_i2 __attribute__((ext_vector_type(2)));
__device__ void llvm_raw_buffer_store_wt_v2i32(wt_i2 v, __amdgpu_buffer_rsrc_t r, int off, int soff,
                                               int aux) __asm("llvm.amdgcn.raw.ptr.buffer.store.v2i32");
__device__ __forceinline__ void st_wt8(void* base, uint32_t byte_off, uint32_t lo, uint32_t hi) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
  llvm_raw_buffer_store_wt_v2i32(wt_i2{(int)lo, (int)hi}, r, (int)byte_off, 0, kStAux);
}
__device__ __forceinline__ void st_wt2(void* base, uint32_t byte_off, unsigned short v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b16(v, r, (int)byte_off, 0, kStAux);
}
__device__ __forceinline__ unsigned short f2bf(float x) {   // round to nearest even
  return __builtin_bit_cast(unsigned short, (__bf16)x);
}
__device__ __forceinline__ uint32_t f2bf2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}
constexpr unsigned short kBf16One = 0x3F80;

inline int round_up(int x, int m) { return (x + m - 1) / m * m; }
inline int64_t round_up64(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// ---------------------------------------------------------------------------
// Launch timeline (sacmi_profile_timeline).  In an instrumented update graph every kernel
// launch owns kTlWords words {start, -, kind, grid, ~end[256]}: the first 8 workgroups fold
// their entry clock into `start` (atomicMin), and each of the last 4096 workgroups (every
// workgroup of the update's grids) stores its exit clock, complemented, into a slot of its
// own — no contended word (atomics of every workgroup on shared words cost ~0.4 us per
// kernel on 8 per-XCD words, ~70 us per config-5 update on 256 slots) — on the 100 MHz
// s_memrealtime clock; the buffer starts at all-ones and the host takes the latest stored
// slot as the kernel's end.
// Null pointer (every production graph): no instruction beyond the test.
typedef unsigned long long tl_word;
enum TlKind : int {
  TL_GEMM = 1, TL_FWD_X6, TL_FWD16, TL_AXK16, TL_AXK_X6, TL_DW_PART16, TL_DW_FIN, TL_HEADS,
  TL_SAMPLE_BWD, TL_MT_SAMPLE, TL_GATHER, TL_PER_F1, TL_PER_F2, TL_PER_F2B, TL_PER_F3,
  TL_PER_F4, TL_PER_UNFUSED, TL_ADAM, TL_SAMPLE_TAIL, TL_FWD16P, TL_DW_PART_X6, TL_KINDS
};
constexpr int kTlEnd = 4;            // first of the ~end slots
constexpr int kTlEndSlots = 4096;
// Diagnostic builds (-DSACMI_DIAG_PHASES, tools/build_variant.sh): the first 256 workgroups
// of a stamping kernel also record kTlPhases clocks each (SACMI_PHASE), after the end slots;
// sacmi_profile_timeline then dumps the raw buffer to $SACMI_DIAG_DUMP (tools/phase_dump.py)
#ifdef SACMI_DIAG_PHASES
constexpr int kTlPhases = 10;
#else
constexpr int kTlPhases = 0;
#endif
constexpr int kTlPhase0 = kTlEnd + kTlEndSlots;
constexpr int kTlWords = kTlPhase0 + 256 * kTlPhases;   // words per kernel launch
constexpr int kTlPerSite = 8;        // kernel launches one launch site may make
struct TlMark {
  tl_word* p;
  __device__ __forceinline__ TlMark(tl_word* q, int kind) : p(q) {
    // the first 8 workgroups (the first dispatched, one per XCD) fold in their entry.  Wave
    // 0 only, as a wave-uniform branch (a divergent single-lane branch around the atomic
    // costs the big GEMM kernels ~30 VGPRs and spills); its lanes' atomics on one address
    // with one scalar value are combined.
    if (p && blockIdx.x < 8 && __builtin_amdgcn_readfirstlane(threadIdx.x) < 64u) {
      atomicMin(p, (tl_word)wall_clock64());
      if (blockIdx.x == 0) { p[2] = (tl_word)kind; p[3] = (tl_word)gridDim.x; }
    }
  }
  __device__ __forceinline__ ~TlMark() {
    // wave 0 of each of the last kTlEndSlots (4096) workgroups — every workgroup of the
    // update's grids — stores ~clock into a slot of its own (the host takes the latest): the
    // kernel's end is the last workgroup to retire, whatever its index (the highest-numbered,
    // last dispatched workgroups alone can retire early, e.g. a grid-stride epilogue's empty
    // tail).  Plain stores: atomics from every workgroup onto shared slots cost the
    // instrumented config-5 update ~70 us (361 vs 290 us)
    if (p && blockIdx.x + kTlEndSlots >= gridDim.x && __builtin_amdgcn_readfirstlane(threadIdx.x) < 64u)
      p[kTlEnd + (blockIdx.x & (kTlEndSlots - 1))] = ~(tl_word)wall_clock64();
  }
};

#ifdef SACMI_DIAG_PHASES
#define SACMI_PHASE(tl, k)                                                                      \
  do {                                                                                         \
    if ((tl) && blockIdx.x < 256 && __builtin_amdgcn_readfirstlane(threadIdx.x) < 64u)          \
      (tl)[kTlPhase0 + blockIdx.x * kTlPhases + (k)] = (tl_word)wall_clock64();                 \
  } while (0)
// the same clock taken by the workgroup's LAST wave (slots 6 / 7: its entry and the end of
// its K loop): the dispatch skew between a workgroup's first and last waves
#define SACMI_PHASE_LAST(tl, k)                                                                 \
  do {                                                                                         \
    if ((tl) && blockIdx.x < 256 &&                                                            \
        __builtin_amdgcn_readfirstlane(threadIdx.x) >= blockDim.x - 64u)                       \
      (tl)[kTlPhase0 + blockIdx.x * kTlPhases + (k)] = (tl_word)wall_clock64();                 \
  } while (0)
#else
#define SACMI_PHASE(tl, k) do { } while (0)
#define SACMI_PHASE_LAST(tl, k) do { } while (0)
#endif

// One bias-folded linear layer inside an arena.
struct Linear {
  int64_t off = 0;   // float offset of W~ [n_out, ld]
  int n_out = 0;     // out features
  int k_in = 0;      // in features (reference)
  int ld = 0;        // row stride of W~ (>= k_in + 1, %4 == 0)
  int bias_col = 0;  // column of W~ holding the bias
  int split = 0;     // reference cols >= split sit one column to the right
  int kdim() const { return k_in + 1; }   // GEMM K including the bias column
  int64_t numel_padded() const { return (int64_t)n_out * ld; }
};

// Non-finite inputs the reference rejects with ValueError (include/sacmi.h SACMI_ENAN),
// kept as bits of DevScalars::err.  Set on the device where the reference would raise:
//   ERR_NAN_TGT  policy.sample(next_state): NaN mean / log_std (Normal(validate_args),
//                networks_model1.py:87, sac_imp.py:89) — nothing of the update has happened
//   ERR_NAN_ACT  policy.sample(state) (sac_imp.py:116) — the critic step (sac_imp.py:101-113)
//                has happened, the actor / alpha / Polyak steps have not
//   ERR_NAN_PER  np.random.choice(p=probs) with NaN probabilities (replay_buffer.py:60-64):
//                the frame has advanced, the numpy stream has not
//   ERR_ABORT    set once an ERR_NAN_ACT update has taken its critic step: every later
//                kernel of the stream skips its state writes
//   ERR_REMOTE_SKIP / ERR_REMOTE_ACT  (data-parallel updates) another rank's update saw a bit
//                of the skip-all class / ERR_NAN_ACT: every rank then voids the same steps, so
//                the replicas stay identical (the error flags travel with the critic gradient
//                collective: kDpFlagN)
// The host reports and clears them (sacmi_step / sacmi_fetch_losses / sacmi_per_sample).
enum ErrBits : int { ERR_NAN_TGT = 1, ERR_NAN_ACT = 2, ERR_NAN_PER = 4, ERR_ABORT = 8,
                     ERR_REMOTE_SKIP = 16, ERR_REMOTE_ACT = 32 };
// an update that sees any of these takes none of its steps
constexpr int kErrSkipAll = ERR_NAN_TGT | ERR_NAN_PER | ERR_ABORT | ERR_REMOTE_SKIP;
// ... and these: the critic step stands, the Polyak / actor / alpha steps do not
constexpr int kErrActLike = ERR_NAN_ACT | ERR_REMOTE_ACT;
// Data-parallel error flags: kDpFlagN floats right past the critic range of the gradient arena
// (in the gap before the actor range), inside the critic gradient collective.  The phase-0
// weight-gradient level stores flag 0 = (err & kErrSkipAll) != 0, flag 1 = (err & kErrActLike)
// != 0 (GemmBatch::err_flags); after the sum over ranks the critic Adam ORs ERR_REMOTE_* into
// the device error word where a flag is positive (AdamArgs::err_flags).  Every error source
// of an update (heads, PER sampler) runs before that level, so one exchange per update suffices.
constexpr int kDpFlagN = 4;

// Scalars shared by kernels (device resident, one struct per context).
struct DevScalars {
  float alpha;          // alpha used by this update (0.2 until the first update)
  float log_alpha_grad; // (unused slot kept for alignment)
  float losses[3];      // q1, q2, policy of the last update
  float pad0;
  double step[4];       // Adam step of policy, q1, q2, alpha optimizers
  double beta_pow[4][2];  // (beta1^step, beta2^step) per optimizer (running products)
  uint64_t noise_counter;
  int64_t len;          // replay fill
  int64_t head;         // ring slot of deque position 0
  int64_t per_frame;
  int32_t alpha_is_tensor;
  int32_t err;          // ErrBits (0: no non-finite input seen)
  int64_t loss_ring_pos;
  int32_t done_seq;     // fused updates finished (their last level's block 0 counts them)
  int32_t pad1;
};

enum Epi { EPI_STORE = 0, EPI_RELU = 1, EPI_MASK = 2,
           EPI_ADAM = 3,          // C is a parameter tensor: apply Adam with acc as the gradient
           EPI_ADAM_POLYAK = 4 }; // ... and Polyak-update its target copy

// One GEMM of a grouped launch: C[m,n] = epi( sum_k A(m,k) B(k,n) ).
//   A(m,k) = a_kc ? A[m*lda + k] : A[k*lda + m]
//   B(k,n) = b_kc ? B[n*ldb + k] : B[k*ldb + n]
//   EPI_MASK: C = acc * (aux[m*ldaux + n] > 0)   (ReLU backward)
struct GemmDesc {
  const float* A;
  const float* B;
  const unsigned short* Bh;   // bf16 mode: B's bf16 shadow (a parameter operand) or null
  float* C;
  const float* aux;
  int M, N, K;
  int lda, ldb, ldc, ldaux;
  int a_kc, b_kc, epi;
  int tiles_n, tile_begin;
  int tiles_m;         // row blocks
  int xcd_gr;          // >0: XCD-blocked tile order, gr x (8/gr) XCD grid (launch_gemm)
  // tile placement without a device-side division (assign_tiles): block t of the desc ->
  // q = t' / pl_div as mul_hi(t', pl_mag) (pl_mag 0: pl_div 1), t' = t (row-major order) or
  // t >> 3 (XCD grid: sub-grid columns pl_div, sub-grid rows pl_sr, 2^pl_gc_log2 XCD columns)
  int pl_div, pl_gc_log2, pl_sr;
  unsigned pl_mag;
  // fc3 dot partials (forward ReLU levels feeding a scalar head): for every row and
  // every 32-column block of this GEMM's output, sum_n relu(y[row][n]) * dotw[n] is
  // written to dotp[row * dotp_ld + n / 32]
  const float* dotw;
  float* dotp;
  int dotp_ld;
  // A-operand transform (the critic / actor fc3 backward folded into the next GEMM).
  // The head gradient of row b is dh2(b,k) = coef[b] * ax_w[k] * [A(b,k) > 0], and coef[b]
  // factors out of the row's dot products, so
  //   axk 1 (A K-contiguous, rows = batch): a(b,k) = A(b,k) > 0 ? ax_w[k] : 0, and the
  //         epilogue multiplies output row b by coef[b] (slot ax_slot of this workgroup's
  //         row prologue, GemmBatch.rows, which runs after the MFMAs: its loads never sit
  //         on the critical path); the column-tile-0 workgroups also store the unscaled
  //         rows u(b,k) = a(b,k) to ax_out (row stride ax_ld) — a later level applies
  //         coef with a_ksc.
  int axk, ax_slot;
  const float* ax_w;
  float* ax_out;
  int ax_ld;
  // A row-contiguous only: a(m,k) *= a_ksc[k] (per-K scale, e.g. dh2 = coef (x) u for the
  // critic fc2 weight gradient)
  const float* a_ksc;
  int adam_step;       // EPI_ADAM*: optimizer step counter index (0 pi, 1 q1, 2 q2)
  const float* bias;   // forward epilogue: C += bias[n * bias_ld] (before the ReLU)
  int bias_ld;
  int rs_col;          // >= 0 (A row-contiguous only): also produce sum_k A(m,k) — the
                       // bias gradient — into column rs_col of C (n0 == 0 tiles), with
                       // the same epilogue (store or Adam) as the tile
  // dL/da partials of the actor pass (sac_imp.py:116-125 backward through Q(s, a~)), from
  // the dha1 tile in the epilogue of the level that produces it: for every output row and
  // every 32-column block cb of this GEMM's output (hidden units of critic fc1),
  //   pa_out[((pa_base + cb) * M + row) * pa_A + j] = sum_{n in cb} C[row][n] * pa_w[n * pa_ld + j]
  // (pa_w: the fc1 weights' action columns); the sample-backward tail sums the blocks
  const float* pa_w;
  float* pa_out;
  int pa_ld, pa_A, pa_base;
  // bf16 activations (bf16 mode, batch-4096 class: sacmi.hip act16): the operand is stored
  // as bf16 at its element offsets (pointer = bf16 base reinterpreted; ld in elements).
  // a16: A (k_fwd16 input rows; k_axk16's h transform source), b16: B (k_dw_part16's X),
  // c16: C (k_fwd16 output), x16: aux (the ReLU-mask source of EPI_MASK).  launch_gemm
  // accepts them only on the kernels that read / write that form
  int a16, b16, c16, x16;
};

// Adam fused into weight-gradient epilogues (single-GPU path): the gradient tile never
// leaves the workgroup.  P/M/V/T arenas mirror each other, so the Adam state of the
// parameter at C[i] is M[C - P + i], V[...], and its target T[C - P - t_base + i].
struct AdamFuse {
  float* P; float* M; float* V; float* T;
  float* G;            // non-null: gradients are also stored (GRAD-slot export)
  int64_t t_base;
  float lr, beta1, beta2, eps, tau;
  int step_idx;        // which optimizer's step counter drives the bias corrections
  int step_offset;     // t = step + step_offset
  DevScalars* sc;
  // block 0 extras
  const float* loss_part; int n_part, loss_slot0, n_losses; float loss_div;
  int64_t log_alpha_idx; int auto_entropy;   // scalar alpha Adam (step idx 3), -1: none
  const float* log_alpha_grad;               // written by k_critic_rows
  float* loss_ring; int ring;
  float* loss_host;      // or null: the losses also stored to host-mapped memory (sync step);
                         //   block 0 stores sc->err's bits into word 3
  int* done_word;        // or null (host-mapped): the update's last level, after everything
                         //   else block 0 stores: sc->done_seq, incremented (sacmi_step's wait)
  int err_skip;          // ErrBits that void this level's stores (critic: kErrSkipAll,
  int err_nopolyak;      //   actor: every bit); ... that void only its Polyak stores (ACT)
  unsigned short* Ph;    // bf16 mode: bf16 shadows of the parameter / target arenas, kept
  unsigned short* Th;    //   in step with every parameter store (null otherwise)
};

struct GatherArgs {
  const int32_t* idx;     // deque positions [B]
  const float* obs; const float* act; const float* rew; const float* obs2; const float* done;
  int ldo, lda_;          // row strides of obs/obs2 and act in the ring
  int64_t capacity;
  const DevScalars* sc;
  int S, A, B;
  float* xq; float* x2; int ldx;   // xq [B, ldx], x2 [2B, ldx]
  float* r; float* d;
  int by_slot;            // 1: idx are ring slots (PER), 0: deque positions
  int x16;                // 1: xq / x2 rows stored as bf16 (act16 updates)
  tl_word* tl;
};
struct MtSampleArgs {
  uint32_t* mt;           // 624 key words + pos
  const DevScalars* sc;   // len
  int k;                  // batch
  int setsize;            // random.sample branch threshold (host-computed, exact)
  int32_t* idx_out;       // [k]
  int64_t* idx64_out;     // [k] or null
  int32_t* pool;          // scratch [max setsize] for the pool branch
  int skip_on_err;        // 1 (update graphs): leave the MT state untouched when sc->err is
                          // set — the reference never reaches a later update's sample
  tl_word* tl;
  uint32_t* mt_save;      // or null: the state before this draw (625 words) is stored here —
                          // the restore point of a draw made ahead for the next single update
};
// Work of the NEXT update of a multi-update graph that rides along, as extra
// workgroups, in a GEMM launch whose tiles leave CUs idle (1024-thread configs):
// its random.sample (kind 1, one workgroup) or its minibatch gather (kind 2).
// every k_gemm config launch_gemm picks has 1024 threads and a reduction buffer of at
// least 16*32*33 floats: the LDS a ride-along random.sample may use
constexpr size_t kRideLdsBytes = (size_t)16 * 32 * 33 * 4;
// k_dw_part16's LDS block (two bf16 operand slab pairs + row-sum scratch), which a
// ride-along sampler may use instead
constexpr int kDw16LdsBytes = 77824;   // 2 x 34,816 (slabs) + 16 x 128 x 4 (row sums)
// The Polyak target update (sac_imp.py:146-152), riding as extra workgroups in a level after
// the critic step: t <- t * (1 - tau) + p * tau over the critic arena, float4-wide (the
// critic region is float4-aligned), skipped after a non-finite sample (ErrBits: the
// reference raised before its Polyak step).  Targets are read only by the next update's
// target levels, so the update's critical path (the critic Adam level) does not carry it.
struct PolyakArgs {
  float* T;                 // target arena (critic part)
  const float* P;           // the critic parameters it tracks (same layout)
  unsigned short* Th;       // bf16 shadow of T or null
  int64_t n4;               // float4 groups
  float tau;
  const DevScalars* sc;
};

struct RideAlong {
  int kind;        // 0 none, 1 random.sample, 2 gather
  int nblocks;
  int tbl_log2;    // kind 1: hash table size
  MtSampleArgs mt;
  GatherArgs ga;
  int pk_blocks;   // > 0: Polyak workgroups after the kind's (k_gemm levels only)
  PolyakArgs pk;
};

// Row prologue of a level whose A operand is transformed with axk 1: per batch row,
// the fc3 heads are finished from the dot partials of the previous levels and turned
// into the coefficients of the backward (sac_imp.py:87-113 critic / 116-121 actor).
struct RowsFuse {
  int kind;                  // 0 none, 1 critic (target + MSE), 2 actor (min Q)
  const float* part;         // [nslot][B][nparts] dot partials (critic: q1 q2 qt1 qt2; actor: qa1 qa2)
  int nparts, B;
  const float* r; const float* d;
  const float* logp;         // critic: log pi(a'|s2);  actor: log pi(a~|s)
  const float* logp_a;       // critic: log pi(a~|s) for the alpha gradient
  float gamma, target_entropy;
  int auto_entropy;
  DevScalars* sc;
  float* dq;                 // [2][B] out: the per-row head gradients (read by later levels)
  float* dq4;                // [2][B][4]: the same, one per 16-byte row (column 0; the fc3
                             //   weight gradient's A operand)
  float* loss_part;          // critic [row blocks][2] squared errors; actor [row blocks]
  // actor: dL/dlog_alpha = -mean(logp_a + te) (sac_imp.py:128-133) from the heads
  // kernel's per-workgroup logp sums (slot 1 of each of n_lp workgroups)
  float* alpha_grad;
  const float* logp_part;
  int n_lp;
};

constexpr int kMaxGemms = 8;
// Sample-forward epilogue (policy heads): rows [row0, row0+M) of the stacked
// [target rows ; actor rows] matrix.
struct HeadSampleArgs {
  const float* h;        // [rows, ldh] policy hidden (h~ incl. ones col)
  int h16;               // 1: h is bf16 and the actions go to act as bf16 (act16 updates)
  const float* Wh;       // [2A, ldw] head weights (mean rows ; log_std rows)
  int rows, A, K, ldh, ldw;   // K = H: the bias (column K of Wh) is added in the epilogue
  float* eps;            // [rows, A] standard normals (read, or written when gen)
  int gen_eps;           // 1: Philox noise
  uint64_t seed;
  const DevScalars* sc;
  float* act;            // actions written to act[row*ldact + j]
  int ldact;
  float* logp;           // [rows]
  float* cache;          // [rows, 3A]: 1 - y^2 (as sech^2 x) | log_std(raw) | y
  float scale, bias;
  int deterministic;     // 1: action = tanh(mean)*scale+bias (select_action(evaluate=True))
  uint64_t ctr_override; // nonzero: Philox counter to use instead of sc->noise_counter
  float* logp_part;      // [grid][2] or null: per workgroup, sum of logp over its rows
  int split_row;         //   < split_row (slot 0) and >= split_row (slot 1)
  float* act_host;       // or null: the actions also stored [row][A] to host-mapped memory
  // Normal(mean, std) validation (networks_model1.py:87): a NaN mean or log_std of row m
  // sets bit (m < split_row ? nan_bit_lo : nan_bit_hi) of *nan_flag — by atomicOr on the
  // device scalars (update), by a plain store on host-mapped memory (select_action)
  int* nan_flag;
  int nan_bit_lo, nan_bit_hi, nan_plain;
  // or null (host-mapped; a one-workgroup launch only): done_value stored after every other
  // store of the workgroup, behind a system-scope fence (sacmi_act polls it)
  int* done_word;
  int done_value;
  tl_word* tl;
};

struct GemmBatch {
  GemmDesc d[kMaxGemms];
  int count;
  int total_tiles;
  AdamFuse adam;       // used when any desc has epi >= EPI_ADAM
  int has_adam;
  RideAlong ride;      // extra workgroups after the tiles
  RowsFuse rows;       // prologue for axk-1 descs
  int bf16;            // 1: bf16 MFMA operands (fp32 loads rounded to bf16 in registers)
  float* ws;           // bf16 deep-K weight-gradient levels: split-K partial workspace
  int64_t ws_floats;   //   (capacity; launch_gemm falls back when a level needs more)
  tl_word* tl;         // launch timeline slots of this level (kTlPerSite), or null
  int st_wt;           // k_gemm epilogue stores write-through (set by launch_gemm)
  // data-parallel phase 0's last level: block 0 stores the error flags (kDpFlagN) of
  // *err_word here, before the critic gradient collective (null: none)
  float* err_flags;
  const int* err_word;
};

// Sample-backward epilogue of the dL/da GEMM.
struct SampleBwdArgs {
  const float* cache;    // actor rows' cache [B, 3A]
  const float* eps;      // actor rows' eps [B, A]
  float* dhead;          // [B, lddh] : dmean | dlog_std
  int lddh, A, B;
  const DevScalars* sc;
  float scale;
  // dhp2 = (dhead Whead) * [hp2 > 0] for the same rows (the policy heads' backward)
  const float* Wh;       // [2A, ldw] head weights
  int ldw, H;
  const float* hp2;      // actor rows' hidden-2 [B, ldh] (ReLU mask source)
  int ldh;
  float* dhp2;           // [B, H]
  int hp2_16;            // 1: hp2 is bf16 (act16 updates; only its sign is read)
  tl_word* tl;
};

// ---------------------------------------------------------------------------
// launchers (kernels.hip)
void launch_gemm(const GemmBatch& batch, hipStream_t s);
void launch_heads_sample(const HeadSampleArgs& a, hipStream_t s);

// select_action for one state (sacmi_act, n = 1): the policy forward as GEMVs.
// y[n] = relu?(sum_{k < K} x[k] W[n * ldw + k]) (K counts the bias: x[K - 1] = 1); x and W
// are read 4-wide up to round4(K) (zeros past K in both: padded rows).
struct GemvArgs {
  const float* x;
  const float* W;
  int ldw, K, N;
  float* y;
  int relu;
};
void launch_act_gemv(const GemvArgs& a, hipStream_t s);
// ... and its heads (mean | log_std rows of Wh over x) + GaussianPolicy.sample for the row
struct ActHeadsArgs {
  const float* x;
  const float* Wh;
  int ldw, K, A;
  int deterministic, gen_eps;
  const float* eps;       // [A] (gen_eps == 0, not deterministic)
  uint64_t seed, ctr;
  float scale, bias;
  float* out;             // [A] actions (host-mapped)
  int* nan_flag;          // plain store of 1 (host-mapped)
  int* done_word;         // done_value stored last (host-mapped)
  int done_value;
};
void launch_act_heads(const ActHeadsArgs& a, hipStream_t s);
// rows per heads workgroup (and per log-prob partial): 32 from 8192 stacked rows on
inline int heads_rows_per_wg(int rows) { return rows >= 8192 ? 32 : 16; }
// dst[i] = bf16(src[i]) (round to nearest even), the parameter shadows of bf16 mode
void launch_to_bf16(unsigned short* dst, const float* src, int64_t n, hipStream_t s);
void launch_gemm_sample_bwd(const GemmDesc& d, const SampleBwdArgs& a, hipStream_t s);
// the same sample backward + dhp2 tail from the dL/da partials of the dha1 level
// (GemmDesc::pa_out): dL/da = sum over the n_pa column blocks, fixed order
void launch_sample_bwd_tail(const float* pa, int n_pa, const SampleBwdArgs& a, hipStream_t s);
// whether launch_gemm runs this level on k_axk16 (no dL/da partials there)
bool gemm_level_on_axk16(const GemmBatch& b);
// whether launch_gemm runs this axk-1 level on the tiles that compute dL/da partials
bool gemm_level_pa_capable(const GemmBatch& b);


constexpr int kMaxAdamSegs = 8;
struct AdamSeg { int64_t off, n; int step_idx; };
struct AdamArgs {
  float* p; const float* g; float* m; float* v;
  float* tgt;              // Polyak target arena (mirrors p from p_tgt_base) or null
  int64_t tgt_base;        // offset subtracted from p index to index tgt
  int nseg; AdamSeg seg[kMaxAdamSegs];
  int64_t total;           // sum of seg n (grid-stride domain)
  float lr, beta1, beta2, eps, grad_scale, tau;
  int step_offset;         // t = step[idx] + step_offset
  DevScalars* sc;
  // loss finalisation (block 0)
  const float* loss_part; int n_part; int loss_slot0; int n_losses; float loss_div;
  // alpha update: index (inside p) of log_alpha or -1
  int64_t log_alpha_idx; int auto_entropy;
  float* loss_ring;        // [ring, 3] or null
  int ring;
  unsigned short* ph;      // bf16 shadows of p / tgt (bf16 mode) or null
  unsigned short* tgth;
  int err_skip, err_nopolyak;   // as AdamFuse
  // data-parallel critic step: the error flags summed over the ranks (kDpFlagN), combined into
  // the error word before the skip test (null: the local word alone)
  const float* err_flags;
  tl_word* tl;
};
void launch_adam(const AdamArgs& a, hipStream_t s);

// Sharded data-parallel optimizer step (sacmi.hip enqueue_dp, ZeRO-1): each range (critic,
// actor) is cut into `world` chunks of a kShardAlign-float multiple; rank r reduce-scatters
// the gradients into chunk r, runs Adam on it and all-gathers the parameters.  P and G carry
// kShardSlack floats past the arena layout for the last chunk's reach.
constexpr int kShardAlign = 64;
constexpr int kMaxShardWorld = 64;
constexpr int64_t kShardSlack = (int64_t)kShardAlign * kMaxShardWorld;
// Polyak over the critic arena as its own launch (PolyakArgs: the ride-along form's body)
void launch_polyak(const PolyakArgs& a, hipStream_t s);
// alpha = exp(log_alpha) from the parameter arena after the actor all-gather (every rank:
// only the owner of log_alpha's chunk took its Adam step), unless err & err_skip
void launch_alpha_sync(DevScalars* sc, const float* log_alpha, int err_skip, hipStream_t s);

void launch_gather(const GatherArgs& a, hipStream_t s);

// Rows sacmi_push left in host-mapped staging for the next synchronous update (the
// trainer's row per env step): that update's sampler kernel scatters them into the ring
// before it draws, instead of a scatter launch of their own ahead of the update
struct PushMailbox {      // host-mapped header; rows [n][2S + A + 2] (s | a | r | s2 | d) follow
  int32_t n, pad;
  int64_t pos0, len, head;  // ring slot of row 0; the replay's len / deque head after them
};
struct MailboxArgs {
  const PushMailbox* hdr;   // null: no mailbox
  const float* rows;
  float *obs, *obs2, *act, *rew, *done;
  int S, A, ldo, ldact;
  int64_t cap;
};
void launch_mt_sample(const MtSampleArgs& a, hipStream_t s, const MailboxArgs* mb = nullptr);

// Transition ingest (replay_buffer.py:10-11 push, batched): one host->device copy of n
// packed rows [s n*S | a n*A | r n | s2 n*S | d n] (from a pinned staging slot), scattered
// into the SoA ring at slots (pos0 + i) % cap; block 0 also publishes the fill / head
// the host computed (DevScalars len, head) — no host round trip.
struct PushArgs {
  const float* stage;
  float *obs, *obs2, *act, *rew, *done;
  int S, A, ldo, ldact;
  int64_t n, pos0, cap;
  DevScalars* sc;
  int64_t len, head;
};
void launch_push_rows(const PushArgs& a, hipStream_t s);

void launch_fill(float* p, int64_t n, float v, hipStream_t s);
// p[i] *= f (the data-parallel loopback's stand-in for an all-reduce over identical ranks)
void launch_scale(float* p, int64_t n, float f, hipStream_t s);
void launch_set_column(float* p, int rows, int ld, int col, float v, hipStream_t s);
void launch_increment_steps(DevScalars* sc, hipStream_t s);

// PER (per.hip)
// Rings up to this many rows take the fused PER path, whose kernels read the fill from
// DevScalars::len (published by the last push): one captured graph serves every fill
// level.  Larger rings take the unfused sequence, sized by the host's len.
constexpr int64_t kPerFusedMaxRows = (int64_t)16384 * 1024;
struct PerArgs {
  const float* prio; int64_t len;
  int64_t cap;            // ring capacity (fused path: launch geometry)
  float alpha;
  float* probs;           // [len] scratch: prio^alpha, then normalised
  float* chunk_sums;      // [ceil(len/8192)]
  int64_t* q;             // [len] fixed-point prefix (block-local)
  int64_t* block_sums;    // [ceil(len/1024)]
  int* bad;               // 1 -> sequential float64 cumsum fallback
  double* cdf;            // [len]
  uint32_t* mt;           // numpy MT19937 stream (625 words)
  int gen_u;              // 1: draw u from mt; 0: u given in `u`
  const double* u;        // [k]
  double* u_scratch;      // [k]
  int k;
  DevScalars* sc;         // per_frame
  double beta_start, beta_frames;
  int32_t* idx32;         // [k] ring slots (feeds the update's gather)
  int64_t* idx_out;       // [k]
  float* w_out;           // [k]
  // np.random.choice's "probabilities contain NaN" (replay_buffer.py:64): the normaliser is
  // NaN / inf / 0 -> ERR_NAN_PER into *err, and the numpy stream is left as it was (the
  // draw's words are restored from mt_backup); the frame still advances (:54-55 run first)
  int* err;
  uint32_t* mt_backup;    // [625]
  int skip_on_err;        // 1 (update graphs): no draw, no frame step when *err is set
  tl_word* tl;            // kernels F1, F2, F2b, F3, F4 (or the unfused sequence) in order
};
void launch_per_sample(const PerArgs& a, hipStream_t s);
void launch_per_update(float* prio, const int64_t* idx, const float* val, int64_t n,
                       int32_t* owner, hipStream_t s);
void launch_per_push(float* prio, int64_t cap, int64_t pos, int64_t n, int empty, float* scratch,
                     hipStream_t s);

}  // namespace sacmi
