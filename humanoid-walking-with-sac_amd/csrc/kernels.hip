// HIP/CDNA4 kernels of the SAC gradient step (gfx950).
//
// GEMMs: fp32-in / fp32-accumulate MFMA (v_mfma_f32_16x16x4_f32, exact-f32 fma
// chain) — the reference computes in fp32 (sac_imp.py:81-85 FloatTensor), gfx950
// has no xf32, so this is the native full-precision matrix path.
//
// Fragment mapping of v_mfma_f32_16x16x4_f32 (cdna_hip_programming.md §3):
//   lane l supplies A[i = l&15][kk = l>>4] and B[kk = l>>4][j = l&15];
//   D[row = (l>>4)*4 + r][col = l&15] lands in accumulator register r.
// A 16-deep K chunk is consumed in 4 MFMA steps s = 0..3; lane group g = l>>4 feeds
// k = k0 + 4g + s to BOTH operands, so each lane fetches 4 consecutive k of its row
// with ONE 16-byte load when the operand is K-contiguous (nn.Linear weights,
// row-major activations) and 4 coalesced 64-byte row segments otherwise.
// Workgroups split K across their waves and reduce through LDS in a fixed wave
// order: no float atomics anywhere, results are bitwise reproducible.
#include "replay_dev.h"

#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <map>

namespace sacmi {

// Diagnostic timestamps (tools/gemm_bench.hip builds with SACMI_DIAG_STAMPS; the library
// build compiles them away): per workgroup, per wave, 100 MHz real-time counter.
#ifdef SACMI_DIAG_STAMPS
__device__ unsigned long long g_stamps[4096][40];
#define SACMI_STAMP(slot)                                                            \
  do {                                                                              \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096) {                             \
      g_stamps[blockIdx.x][slot] = __builtin_amdgcn_s_memrealtime();                \
      if ((slot) == 0)                                                              \
        g_stamps[blockIdx.x][34] =                                                  \
            ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |  \
            __builtin_amdgcn_s_getreg((31 << 11) | 4);                              \
    }                                                                               \
  } while (0)
#else
#define SACMI_STAMP(slot) do { } while (0)
#endif


typedef float f4 __attribute__((ext_vector_type(4)));


// per-(kernel, device) high-water mark of the dynamic-LDS attribute
void ensure_dyn_lds(const void* kernel, size_t bytes) {
  static std::map<std::pair<const void*, int>, size_t> seen;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  size_t& cur = seen[{kernel, dev}];
  if (bytes <= cur) return;
  const hipError_t e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e != hipSuccess)
    throw Error{SACMI_EDEVICE, std::string("dynamic LDS request of ") + std::to_string(bytes) +
                                   " bytes refused: " + hipGetErrorString(e)};
  cur = bytes;
}

#define SACMI_STR2(x) #x
#define SACMI_STR(x) SACMI_STR2(x)
#define HIP_LAUNCH_CHECK() launch_check(__FILE__ ":" SACMI_STR(__LINE__))

// ---------------------------------------------------------------------------
// Buffer-resource access (raw buffer ops): the base lives in a wave-uniform SGPR
// descriptor and each lane carries one 32-bit byte offset, shared by every array that
// is indexed alike (the Adam state) — no per-array 64-bit addresses held in VGPRs.
using rsrc_t = __amdgpu_buffer_rsrc_t;
constexpr int kBufDword3 = 0x00020000;   // gfx9-family raw buffer descriptor word 3

__device__ __forceinline__ rsrc_t make_rsrc(const float* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, (int)bytes, kBufDword3);
}
__device__ __forceinline__ float buf_ld(rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}
// ... with cache-policy bits (AUX 16 = sc1: L1 bypass, for data another workgroup of the same
// launch wrote write-through: cdna_hip_programming.md §6 Guideline 16)
template <int AUX>
__device__ __forceinline__ float buf_ld_aux(rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, AUX));
}
__device__ __forceinline__ void buf_st(rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), r, (int)off, 0, 0);
}
// the store policy a level was launched with (GemmBatch::st_wt, wave-uniform): write-through
// or plain
__device__ __forceinline__ void buf_st_pol(rsrc_t r, uint32_t off, float v, bool wt) {
  if (wt) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), r, (int)off, 0, kStAux);
  else __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), r, (int)off, 0, 0);
}
template <class T>
__device__ __forceinline__ void st_pol(T* p, T v, bool wt) {
  if (wt) st_wt<true>(p, v);
  else *p = v;
}

// 16-byte buffer load.  The LLVM intrinsic is bound directly: on this toolchain (ROCm 7.2
// hipcc) __builtin_amdgcn_raw_buffer_load_b128 lowers to a single buffer_load_dword.
__device__ f4 llvm_raw_buffer_load_v4f32(rsrc_t r, int off, int soff, int aux)
    __asm("llvm.amdgcn.raw.ptr.buffer.load.v4f32");
__device__ __forceinline__ uint2 buf_ld2(rsrc_t r, uint32_t off) {
  typedef unsigned int u2_t __attribute__((ext_vector_type(2)));
  const u2_t v = __builtin_bit_cast(u2_t, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0));
  return make_uint2(v.x, v.y);
}
__device__ __forceinline__ uint32_t buf_ld_u16(rsrc_t r, uint32_t off) {
  return (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(r, (int)off, 0, 0);
}
__device__ __forceinline__ unsigned short bf16_bits(float x) {
  return __builtin_bit_cast(unsigned short, (__bf16)x);
}
__device__ __forceinline__ float4 buf_ld4(rsrc_t r, uint32_t off) {
  const f4 v = llvm_raw_buffer_load_v4f32(r, (int)off, 0, 0);
  return float4{v[0], v[1], v[2], v[3]};
}
__device__ void llvm_raw_buffer_store_v4f32(f4 v, rsrc_t r, int off, int soff, int aux)
    __asm("llvm.amdgcn.raw.ptr.buffer.store.v4f32");
template <int AUX = 0>
__device__ __forceinline__ void buf_st4(rsrc_t r, uint32_t off, f4 v) {
  llvm_raw_buffer_store_v4f32(v, r, (int)off, 0, AUX);
}

// ---------------------------------------------------------------------------
// operand fetch: NT 16-row subtiles x 4 consecutive k (k = k0 + 4g .. +3), through one
// buffer descriptor per operand (SGPRs) and a 32-bit byte offset per subtile row:
//   KC  (K-contiguous, element (row,k) at off + 4k):       one 16-byte load
//   !KC (row-contiguous, element (row,k) at off + 4k*ld):  4 loads, each a coalesced
//        64-byte segment across the 16 lanes of a lane group.
// Branch-free: a load inside a divergent `if` (or any guarded block) is waited for at the
// end of that block, which would serialise every operand load of the burst.  Rows are
// clamped into range (row_offs) and out-of-range k reads a clamped address, zeroed by a
// select.
template <int NT>
struct OpFetch {
  rsrc_t r;
  const char* p;
  uint32_t off[NT];
#ifdef SACMI_EXP_LINFETCH
  bool lin;   // the operand has >= 16 rows: the contiguous-read experiment applies
#endif
};

#ifndef SACMI_FETCH_SADDR
#define SACMI_FETCH_SADDR 0
#endif
constexpr int kLdSc1 = 16;      // raw buffer load cache-policy bits: sc1 (coherent across XCDs)
#ifndef SACMI_A_AUX
#define SACMI_A_AUX 0           // k_gemm: cache-policy bits of the A-operand loads (experiment)
#endif
#ifndef SACMI_B_AUX
#define SACMI_B_AUX 0
#endif
#ifndef SACMI_KCONTIG
#define SACMI_KCONTIG 0         // k_gemm: contiguous K-chunk ranges per wave (experiment)
#endif
// global load with a uniform 64-bit base and a 32-bit per-lane byte offset (saddr form)
template <class T>
__device__ __forceinline__ T gld_off(const char* base, uint32_t off) {
  return *reinterpret_cast<const T*>(base + off);
}

// H16: the operand is stored as bf16 (K-contiguous only: the policy heads' input under
// act16), fetched 4 k per 8-byte load and widened exactly to fp32
template <int NT, bool KC, bool H16 = false>
__device__ __forceinline__ void row_offs(const float* P, int ld, int row0, int nrows, int lane,
                                         OpFetch<NT>& f) {
  static_assert(!H16 || KC, "bf16 operands are K-contiguous");
  f.r = make_rsrc(P, 0x7fffffffu);
  f.p = reinterpret_cast<const char*>(P);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    int row = row0 + t * 16 + (lane & 15);
    row = row < nrows ? row : nrows - 1;
    f.off[t] = KC ? (uint32_t)row * (uint32_t)ld * (H16 ? 2u : 4u) : (uint32_t)row * 4u;
#ifdef SACMI_EXP_LINFETCH
    // the 16-row block (kept inside the operand's rows), 16 B per lane
    f.lin = KC && !H16 && nrows >= 16;
    if (f.lin) {
      const int rb = row0 + t * 16 < nrows - 16 ? row0 + t * 16 : nrows - 16;
      f.off[t] = (uint32_t)rb * (uint32_t)ld * 4u + 16u * (uint32_t)(lane & 63);
    }
#endif
  }
}

__device__ __forceinline__ float bf16_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// AUX: cache-policy bits of the operand loads (SACMI_A_AUX / SACMI_B_AUX: e.g. 2 = nt)
template <int NT, bool KC, bool H16 = false, int AUX = 0>
__device__ __forceinline__ void fetch_op(const OpFetch<NT>& f, int ld, int k, int K,
                                         float (&v)[NT][4]) {
  if constexpr (H16) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const uint32_t o = f.off[t] + (uint32_t)(k < K ? k : 0) * 2u;
      const uint2 x = buf_ld2(f.r, o);
      v[t][0] = (k < K) ? bf16_lo(x.x) : 0.f;
      v[t][1] = (k + 1 < K) ? bf16_hi(x.x) : 0.f;
      v[t][2] = (k + 2 < K) ? bf16_lo(x.y) : 0.f;
      v[t][3] = (k + 3 < K) ? bf16_hi(x.y) : 0.f;
    }
    return;
  }
#ifdef SACMI_EXP_NOLOAD
  // timing experiment only: no operand loads at all (MFMA + epilogue floor)
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int s = 0; s < 4; ++s) v[t][s] = (float)(k + s + t) * 1e-3f;
  return;
#endif
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (KC) {
#ifdef SACMI_EXP_LINFETCH
      // timing experiment only (wrong values): the same 16-row block's bytes read as 1 KB
      // contiguous per wave-instruction, as an MFMA-packed operand layout would be read
      const int ch = (k >> 4) < (ld >> 4) - 1 ? (k >> 4) : (ld >> 4) - 1;
      const uint32_t o = f.lin ? f.off[t] + (uint32_t)ch * 1024u : f.off[t] + (uint32_t)(k < K ? k : 0) * 4u;
#else
      const uint32_t o = f.off[t] + (uint32_t)(k < K ? k : 0) * 4u;
#endif
      float4 x;
      if constexpr (AUX != 0) {
        const f4 y = llvm_raw_buffer_load_v4f32(f.r, (int)o, 0, AUX);
        x = float4{y[0], y[1], y[2], y[3]};
      } else {
        x = (SACMI_FETCH_SADDR & 1) ? gld_off<float4>(f.p, o) : buf_ld4(f.r, o);
      }
      v[t][0] = (k < K) ? x.x : 0.f;
      v[t][1] = (k + 1 < K) ? x.y : 0.f;
      v[t][2] = (k + 2 < K) ? x.z : 0.f;
      v[t][3] = (k + 3 < K) ? x.w : 0.f;
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int kk = (k + s < K) ? (k + s) : (K - 1);
        const uint32_t o = f.off[t] + (uint32_t)kk * (uint32_t)ld * 4u;
        const float x = AUX ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(f.r, (int)o, 0, AUX))
                            : (SACMI_FETCH_SADDR & 2) ? gld_off<float>(f.p, o) : buf_ld(f.r, o);
        v[t][s] = (k + s < K) ? x : 0.f;
      }
    }
  }
}

typedef short s4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// 4 fp32 fragment values -> 4 bf16 (round to nearest even, v_cvt_pk_bf16_f32)
__device__ __forceinline__ s4 to_bf16x4(const float (&v)[4]) {
  const bf16x4 x = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
  return __builtin_bit_cast(s4, x);
}

// One 16-deep K chunk.  fp32: 4 x v_mfma_f32_16x16x4_f32 (k-step s takes element s of
// every lane's 4).  BF16: the same 4 consecutive k per lane are exactly the operand of
// v_mfma_f32_16x16x16_bf16 (lane l holds A[l&15][4(l>>4) + j], B[4(l>>4) + j][l&15]), so
// the chunk is ONE bf16 MFMA on the rounded fragments, fp32 accumulation, same C layout.
template <int MT, int NT, bool BF16 = false>
__device__ __forceinline__ void mfma_chunk(f4 (&acc)[MT][NT], const float (&a)[MT][4],
                                           const float (&b)[NT][4]) {
#ifdef SACMI_EXP_NOMFMA
  // timing experiment only: the operands are consumed by one add, no MFMA
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j][0] += a[i][0] + b[j][0];
  return;
#endif
  if constexpr (BF16) {
    s4 ab[MT], bb[NT];
#pragma unroll
    for (int i = 0; i < MT; ++i) ab[i] = to_bf16x4(a[i]);
#pragma unroll
    for (int j = 0; j < NT; ++j) bb[j] = to_bf16x4(b[j]);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ab[i], bb[j], acc[i][j], 0, 0, 0);
  } else {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
  }
}

// ---------------------------------------------------------------------------
// fp32 GEMM on bf16 MFMA: the three-way split ("x6").  gfx950's fp32 MFMA issues at 1/16
// of the bf16 rate and has no xf32 form.  Every fp32 operand x is cut EXACTLY into three
// bf16 parts x = h + m + l by truncation (h = the top 8 significant bits, m the next 8 of
// the remainder, l the rest — at most 8 bits, so l is a bf16 with no rounding; both
// subtractions are exact in fp32).  a·b is then the 9 cross products of the parts; the
// products are exact in the fp32 accumulator (8 x 8 significant bits), and the three
// dropped ones (m·l, l·m, l·l) are below 2^-25 |a b| — under fp32's own unit roundoff, so
// the result is as accurate as the fp32 FMA chain (different rounding, not bit-identical).
// Two 16-deep fragment chunks (lane group g holds k = c0*16 + 4g .. +3 and c1*16 + 4g ..
// +3 of its row, the same for both operands) form the 8 bf16 k of one
// v_mfma_f32_16x16x32_bf16 operand; per 32 k and 16x16 block 6 MFMAs of 16 cycles
// replace 8 fp32 MFMAs of 32 cycles.  Small terms first into the accumulator.
#ifndef SACMI_X6
#define SACMI_X6 0       // measured slower at config 2 (profiles/r06/x6_ab)
#endif
#ifndef SACMI_X6_EXP
#define SACMI_X6_EXP 0   // timing builds only (wrong values): 1 no B split, 2 no split at all
#endif
typedef __bf16 x6_bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int x6_u4 __attribute__((ext_vector_type(4)));

// bf16 bits of the upper halves of (lo, hi) packed as one dword (lo in bits 0-15)
__device__ __forceinline__ uint32_t x6_pack_hi(uint32_t lo, uint32_t hi) {
  return __builtin_amdgcn_perm(hi, lo, 0x07060302u);
}
__device__ __forceinline__ void x6_split(const float (&p)[4], const float (&q)[4], x6_bf16x8& h,
                                         x6_bf16x8& m, x6_bf16x8& l, bool fake = false) {
  x6_u4 H, Mw, L;
  if (fake) {   // timing experiment (SACMI_X6_EXP): every part = the top part (finite values,
                // 4 perms instead of the split's 44 instructions)
#pragma unroll
    for (int d = 0; d < 4; ++d)
      H[d] = x6_pack_hi(__float_as_uint(d < 2 ? p[2 * d] : q[2 * d - 4]),
                        __float_as_uint(d < 2 ? p[2 * d + 1] : q[2 * d - 3]));
    h = m = l = __builtin_bit_cast(x6_bf16x8, H);
    return;
  }
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const float x0 = d < 2 ? p[2 * d] : q[2 * d - 4];
    const float x1 = d < 2 ? p[2 * d + 1] : q[2 * d - 3];
    const uint32_t u0 = __float_as_uint(x0), u1 = __float_as_uint(x1);
    H[d] = x6_pack_hi(u0, u1);
    const float r0 = x0 - __uint_as_float(u0 & 0xffff0000u);
    const float r1 = x1 - __uint_as_float(u1 & 0xffff0000u);
    const uint32_t v0 = __float_as_uint(r0), v1 = __float_as_uint(r1);
    Mw[d] = x6_pack_hi(v0, v1);
    const float s0 = r0 - __uint_as_float(v0 & 0xffff0000u);
    const float s1 = r1 - __uint_as_float(v1 & 0xffff0000u);
    L[d] = x6_pack_hi(__float_as_uint(s0), __float_as_uint(s1));
  }
  h = __builtin_bit_cast(x6_bf16x8, H);
  m = __builtin_bit_cast(x6_bf16x8, Mw);
  l = __builtin_bit_cast(x6_bf16x8, L);
}

template <int MT, int NT>
__device__ __forceinline__ void mfma_x6(f4 (&acc)[MT][NT], const float (&a0)[MT][4],
                                        const float (&b0)[NT][4], const float (&a1)[MT][4],
                                        const float (&b1)[NT][4]) {
  // the A parts of every row block first (MT <= NT), each B column block's parts split just
  // before its MFMAs: the parts of one B block live at a time (register pressure)
  x6_bf16x8 ah[MT], am[MT], al[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) x6_split(a0[i], a1[i], ah[i], am[i], al[i], SACMI_X6_EXP >= 2);
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    x6_bf16x8 bh, bm, bl;
    x6_split(b0[j], b1[j], bh, bm, bl, SACMI_X6_EXP >= 1);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      f4 c = acc[i][j];
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[i], bm, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[i], bh, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bm, c, 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh, c, 0, 0, 0);
    }
  }
}

// Each wave accumulates chunks wave, wave+KSPLIT, ... of a TM x TN tile and writes
// its partial sums to red[wave][TM][TN+1].  At batch 256 every operand read is a
// dependent L2/MALL round trip (~1-2 us), so a wave issues the loads of G chunks at
// once (with KSPLIT = 16 waves per workgroup and K <= 528 that is ALL of its chunks:
// one exposed latency per GEMM) and only then runs their MFMAs.  `pre()` runs once,
// right after the last group's loads are issued: the epilogue's own global loads go
// out there, younger than every operand load (vmcnt retires in order), so the MFMAs
// never wait for them and their latency hides under the (last) MFMA phase.
// With MG > 1 the workgroup covers MG*TM rows: wave group g = wave / KSPLIT takes rows
// m0 + g*TM .. +TM, and the K split runs inside each group.
// AXF 1: A-operand transform (GemmDesc::axk) applied to the loaded fragments before the
// MFMAs: a(b,k) = A>0 ? coef[row]*w[k] : 0 with coef in LDS (coef[tile row]); with
// store_a the transformed fragments are also written to d.ax_out.
// PIPE (G == 1, AXF == 0): software-pipelined K loop — chunk j+1's loads are in flight
// while chunk j's MFMAs run (two register buffers); the epilogue operands (pre) go out
// right behind chunk 0's loads (PIPE 1) or after the loop (PIPE 2: deep-K levels, whose
// registers then hold the second buffer instead).  Same chunk order per wave: bitwise
// identical sums.
// MIDSPLIT (k_chain's phases, one pass over K: K <= 16 KSPLIT G): every group's B operand
// (the weights) and transform weights first, then early() — the cohort barrier of the previous
// phase — then the A operands, which the previous phase wrote: the weights' latency and the
// setup overlap the barrier.  Otherwise early() runs before any load.
template <int TM, int TN, int KSPLIT, int G, bool AKC, bool BKC, bool ROWSUM, int MG = 1,
          int AXF = 0, bool BF16 = false, int PIPE = 0, bool A16 = false, int AAUX = SACMI_A_AUX,
          bool MIDSPLIT = false, class Pre, class Early = void (*)()>
__device__ __forceinline__ void gemm_core_l(const GemmDesc& d, int m0, int n0, float* red,
                                            float* rsum, Pre&& pre, bool store_a = false,
                                            Early&& early = [] {}) {
  constexpr int MT = TM / 16, NT = TN / 16;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int ks = wave % KSPLIT;
  const int mloc = (wave / KSPLIT) * TM;   // this wave group's first row in the tile
  m0 += mloc;

  SACMI_STAMP(wave);
  f4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  float rs[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) rs[i] = 0.f;
  OpFetch<MT> ra;
  OpFetch<NT> rb;
  row_offs<MT, AKC, A16>(d.A, d.lda, m0, d.M, lane, ra);
  row_offs<NT, BKC>(d.B, d.ldb, n0, d.N, lane, rb);
  const int nch = (d.K + 15) >> 4;
#if SACMI_KCONTIG
  // contiguous chunk ranges per wave (chunks ks*cpw .. +cpw-1): a wave reads whole
  // 128-byte rows of a K-contiguous operand instead of 64-byte halves shared with another wave
  const int cpw = (nch + KSPLIT - 1) / KSPLIT;
  const int nmine = nch > ks * cpw ? (nch - ks * cpw < cpw ? nch - ks * cpw : cpw) : 0;
#define SACMI_CHUNK(jj) (ks * cpw + (jj))
#else
  const int nmine = nch > ks ? (nch - ks + KSPLIT - 1) / KSPLIT : 0;
#define SACMI_CHUNK(jj) (ks + (jj) * KSPLIT)
#endif
  const int kl = 4 * (lane >> 4);
  float a[G][MT][4], b[G][NT][4];
  // per-group side operands: AXF 1 the transform weights w[k..k+3]; !AKC the A K-scale
  // (a zero-length descriptor where a desc has none: no branch around the loads)
  constexpr bool XW = AXF == 1 || !AKC;
  float xw[XW ? G : 1][4];
  const rsrc_t rxw = AXF == 1 ? make_rsrc(d.ax_w, (uint32_t)d.K * 4u)
                              : make_rsrc(d.a_ksc ? d.a_ksc : d.A, d.a_ksc ? (uint32_t)d.K * 4u : 0u);
  const bool has_ksc = AXF != 1 && d.a_ksc != nullptr;
  // AXF 1 side output: unconditional stores, dropped by a zero-length range where this
  // workgroup stores nothing (a guarded store makes the compiler's vmcnt bookkeeping
  // fall back to full drains)
  const rsrc_t rAx = make_rsrc(store_a ? d.ax_out : d.C,
                               store_a ? (uint32_t)(((size_t)(d.M - 1) * d.ax_ld + d.K) * 4) : 0u);
  if constexpr (!MIDSPLIT) early();
  if constexpr (PIPE != 0) {
    static_assert(G == 1 && AXF == 0, "pipelined K loop: one chunk per stage, no A transform");
    float a1[MT][4], b1[NT][4], xw1[4];
    auto issue = [&](int jj, float (&av)[MT][4], float (&bv)[NT][4], float (&xv)[4]) {
      jj = jj < nmine ? jj : nmine - 1;   // unconditional: past the end re-reads the last chunk
      const int k = SACMI_CHUNK(jj) * 16 + kl;
      fetch_op<MT, AKC, A16, AAUX>(ra, d.lda, k, d.K, av);
      fetch_op<NT, BKC, false, SACMI_B_AUX>(rb, d.ldb, k, d.K, bv);
      if constexpr (!AKC) {
#pragma unroll
        for (int s = 0; s < 4; ++s) xv[s] = buf_ld(rxw, (uint32_t)(k + s < d.K ? k + s : 0) * 4u);
      }
    };
    auto consume = [&](float (&av)[MT][4], const float (&bv)[NT][4], const float (&xv)[4]) {
#pragma clang fp contract(off)
      if constexpr (!AKC) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const float f = has_ksc ? xv[s] : 1.f;
#pragma unroll
          for (int i = 0; i < MT; ++i) av[i][s] *= f;
        }
      }
      mfma_chunk<MT, NT, BF16>(acc, av, bv);
      if (ROWSUM) {
#pragma unroll
        for (int i = 0; i < MT; ++i) rs[i] += (av[i][0] + av[i][1]) + (av[i][2] + av[i][3]);
      }
    };
    if (nmine == 0) {
      pre();
    } else {
      issue(0, a[0], b[0], xw[0]);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (PIPE == 1) pre();
      __builtin_amdgcn_sched_barrier(0);
      for (int j = 0; j < nmine; j += 2) {
        issue(j + 1, a1, b1, xw1);
        __builtin_amdgcn_sched_barrier(0);
        consume(a[0], b[0], xw[0]);
        __builtin_amdgcn_sched_barrier(0);
        issue(j + 2, a[0], b[0], xw[0]);
        __builtin_amdgcn_sched_barrier(0);
        if (j + 1 < nmine) consume(a1, b1, xw1);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (PIPE == 2) pre();
    }
  } else {
  if constexpr (MIDSPLIT) {
    static_assert(PIPE == 0, "MIDSPLIT: register-direct core");
    if (nmine == 0) {
      early();
      pre();
    } else {
      auto bload = [&]() {
#pragma unroll
        for (int g = 0; g < G; ++g) {   // B (and the transform weights), every group
          const int jj = g < nmine ? g : nmine - 1;
          const int k = SACMI_CHUNK(jj) * 16 + kl;
          fetch_op<NT, BKC, false, SACMI_B_AUX>(rb, d.ldb, k, d.K, b[g]);
          if constexpr (AXF == 1) {
            const float4 x = buf_ld4(rxw, (uint32_t)(k < d.K ? k : 0) * 4u);
            xw[g][0] = x.x; xw[g][1] = x.y; xw[g][2] = x.z; xw[g][3] = x.w;
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      };
      // (wave 0 polls the barrier: its weight loads deferred past the wait measured slower,
      // config 2 chain 42.4 -> 44.5 us — DESIGN.md §12a)
      bload();
      early();
#pragma unroll
      for (int g = 0; g < G; ++g) {   // A, every group
        const int jj = g < nmine ? g : nmine - 1;
        const int k = SACMI_CHUNK(jj) * 16 + kl;
        fetch_op<MT, AKC, A16, AAUX>(ra, d.lda, k, d.K, a[g]);
        if constexpr (AXF != 1 && !AKC) {
#pragma unroll
          for (int s = 0; s < 4; ++s) xw[g][s] = buf_ld(rxw, (uint32_t)(k + s < d.K ? k + s : 0) * 4u);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      pre();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (!MIDSPLIT && nmine == 0) pre();
  for (int j = 0; j < nmine; j += G) {
#pragma unroll
    for (int g = 0; g < G && !MIDSPLIT; ++g) {
      // unconditional (see fetch_op; a guard, even a wave-uniform one, makes the compiler
      // drain the loads at the end of the guarded block): a group past the wave's last
      // chunk re-reads that chunk and is skipped below
      const int jj = j + g < nmine ? j + g : nmine - 1;
      const int k = SACMI_CHUNK(jj) * 16 + kl;
      fetch_op<MT, AKC, A16, AAUX>(ra, d.lda, k, d.K, a[g]);
      fetch_op<NT, BKC, false, SACMI_B_AUX>(rb, d.ldb, k, d.K, b[g]);
      if constexpr (AXF == 1) {          // w3 rows are float4-aligned (parameter arena)
        const float4 x = buf_ld4(rxw, (uint32_t)(k < d.K ? k : 0) * 4u);
        xw[g][0] = x.x; xw[g][1] = x.y; xw[g][2] = x.z; xw[g][3] = x.w;
      } else if constexpr (!AKC) {       // per-batch-row scale: any alignment
#pragma unroll
        for (int s = 0; s < 4; ++s) xw[g][s] = buf_ld(rxw, (uint32_t)(k + s < d.K ? k + s : 0) * 4u);
      }
      // keep the issue order group by group: the first group's MFMAs then wait for it alone
      __builtin_amdgcn_sched_barrier(0);
    }
    // after the LAST operand loads (vmcnt is in order)
    if (!MIDSPLIT && j + G >= nmine) pre();
    __builtin_amdgcn_sched_barrier(0);
    // fp32 levels with chunk pairs: the x6 split form (mfma_x6) on each pair, fp32 MFMAs on an
    // unpaired last chunk; the transforms and row sums below work on the fp32 fragments
    constexpr bool X6P = SACMI_X6 && !BF16 && (G % 2 == 0);
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (j + g < nmine) {
        // no FMA contraction here: the scaled fragments feed both the MFMAs and the row
        // sums, and contracting a*f into a sum would make the row-sum bits depend on the
        // tile configuration's code generation
#pragma clang fp contract(off)
        if constexpr (AXF == 1) {
          const int k = SACMI_CHUNK(j + g) * 16 + kl;
#pragma unroll
          for (int i = 0; i < MT; ++i) {
            const int r = mloc + i * 16 + (lane & 15);
#pragma unroll
            for (int s = 0; s < 4; ++s)
              a[g][i][s] = (a[g][i][s] > 0.f && k + s < d.K) ? xw[g][s] : 0.f;
            // the rows this level's tile-0 workgroups hold in full: u for a later level
            const int rr = m0 - mloc + r;
            buf_st4(rAx, (rr < d.M && k < d.K) ? (uint32_t)(rr * d.ax_ld + k) * 4u : 0xfffffff0u,
                    f4{a[g][i][0], a[g][i][1], a[g][i][2], a[g][i][3]});
          }
        } else if constexpr (!AKC) {
          // A K-scale (selected, not branched: 1 where the desc has none)
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const float f = has_ksc ? xw[g][s] : 1.f;
#pragma unroll
            for (int i = 0; i < MT; ++i) a[g][i][s] *= f;
          }
        }
        if constexpr (!X6P) mfma_chunk<MT, NT, BF16>(acc, a[g], b[g]);
        if (ROWSUM) {
#pragma unroll
          for (int i = 0; i < MT; ++i) rs[i] += (a[g][i][0] + a[g][i][1]) + (a[g][i][2] + a[g][i][3]);
        }
      }
    if constexpr (X6P) {
#pragma unroll
      for (int g = 0; g < G; g += 2) {
        if (j + g + 1 < nmine) mfma_x6<MT, NT>(acc, a[g], b[g], a[g + 1], b[g + 1]);
        else if (j + g < nmine) mfma_chunk<MT, NT, false>(acc, a[g], b[g]);
      }
    }
  }
  }   // !PIPE
#undef SACMI_CHUNK
  SACMI_STAMP(16 + wave);
  float* my = red + wave * TM * (TN + 1);
  const int rq = (lane >> 4) * 4, cc = lane & 15;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int jj = 0; jj < NT; ++jj)
#pragma unroll
      for (int r = 0; r < 4; ++r) my[(i * 16 + rq + r) * (TN + 1) + jj * 16 + cc] = acc[i][jj][r];
  if (ROWSUM) {
    // lanes l, l+16, l+32, l+48 hold the same row: fold the 4 lane groups, fixed order
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      float v = rs[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) rsum[wave * TM + i * 16 + lane] = v;
    }
  }
}

// Tile t of a desc -> (row tile, column tile): row-major, or (xcd_gr) the XCD-blocked order
// of assign_tiles — XCD x = t & 7 owns a (tiles_m / gr) x (tiles_n / gc) sub-grid.  The
// divisors come from the host (GemmDesc::pl_*): device integer divisions cost ~0.35 us of
// dependent scalar code per level (phase stamps, profiles/r04).
__device__ __forceinline__ void place_tile(const GemmDesc& d, int t, int& tr, int& tc) {
  const uint32_t n = d.xcd_gr ? (uint32_t)t >> 3 : (uint32_t)t;
  const int q = d.pl_mag ? (int)__umulhi(n, d.pl_mag) : (int)n;
  const int r = (int)n - q * d.pl_div;
  if (d.xcd_gr) {
    const int x = t & 7;
    tr = (x >> d.pl_gc_log2) * d.pl_sr + q;
    tc = (x & ((1 << d.pl_gc_log2) - 1)) * d.pl_div + r;
  } else {
    tr = q;
    tc = r;
  }
}

// layout dispatch (wave-uniform, once per workgroup)
// AXK: whether this kernel instantiation carries the A-transform path (launch_gemm picks
// the variant from the level's descs): 1 -> axk 1 descs, 0 -> none.
// AAUX: cache-policy bits of the A-operand loads (kg_body's LDAUX); MIDSPLIT: early() is the
// mid hook of gemm_core_l (k_chain), else it runs first
template <int TM, int TN, int KSPLIT, int G, int MG, int AXK, bool BF16, int PIPE, int AAUX, bool MIDSPLIT,
          class Pre, class Early>
__device__ __forceinline__ void gemm_core(const GemmDesc& d, int m0, int n0, float* red,
                                          float* rsum, bool rowsum, Pre&& pre, Early&& early) {
  constexpr int AX = AAUX ? AAUX : SACMI_A_AUX;
  constexpr bool MS = MIDSPLIT;
  if constexpr (AXK == 1) {
    if (d.axk == 1 && !d.ax_pre) {   // fc3 backward folded into dh1 / dha1 (A = h2, B = W2)
      gemm_core_l<TM, TN, KSPLIT, G, true, false, false, MG, 1, BF16, 0, false, AX, MS>(
          d, m0, n0, red, rsum, pre, n0 == 0 && d.ax_out != nullptr, early);
      return;
    }
  }
  if (d.a_kc) {
    if (d.b_kc) gemm_core_l<TM, TN, KSPLIT, G, true, true, false, MG, 0, BF16, PIPE, false, AX, MS>(d, m0, n0, red, rsum, pre, false, early);
    else gemm_core_l<TM, TN, KSPLIT, G, true, false, false, MG, 0, BF16, PIPE, false, AX, MS>(d, m0, n0, red, rsum, pre, false, early);
  } else {
    if (d.b_kc) gemm_core_l<TM, TN, KSPLIT, G, false, true, false, MG, 0, BF16, PIPE, false, AX, MS>(d, m0, n0, red, rsum, pre, false, early);
    else if (rowsum) gemm_core_l<TM, TN, KSPLIT, G, false, false, true, MG, 0, BF16, PIPE, false, AX, MS>(d, m0, n0, red, rsum, pre, false, early);
    else gemm_core_l<TM, TN, KSPLIT, G, false, false, false, MG, 0, BF16, PIPE, false, AX, MS>(d, m0, n0, red, rsum, pre, false, early);
  }
}

// ---------------------------------------------------------------------------
// LDS-staged core (k_gemm CORE 1: the batch-256-class fp32 levels).
//
// Why: the register-direct core above reads its operands as 16 rows x 64 bytes per
// wave-instruction (the 16x16x4 fragment: 4 lane groups x 16 B of each of 16 rows).  Measured
// per CU with every CU loading at once (tools/l2_rate_bench.hip, profiles/r04/l2_rate.txt),
// that shape takes 43 GB/s from an L2-resident operand, against ~150 GB/s for 128- to 1024-byte
// row segments per instruction — the level bodies' "operand delivery" bound (round-3 phase
// stamps: the last wave's K loop 2.2-2.5x wave 0's).
//
// How: the workgroup (16 waves) streams K in slabs of BK = 16 KSP through a ring of NST LDS
// slots by LDS-DMA (global_load_lds_dwordx4: 1 KB per wave-instruction, 2-8 rows of
// 128-512 contiguous bytes), slab s + NST - 1 issued right after the barrier that retires
// slab s (counted vmcnt waits, no drain).  The tile TMW x TN is cut into NSUB sub-tiles of
// 32 x WN, and the K of each slab into KSP 16-deep parts: wave (sub, part) runs the 16x16x4
// MFMAs of its sub-tile over its part of every slab, reading fragments from LDS
// (ds_read_b128 for a K-contiguous operand, 4 x ds_read_b32 for an MN-contiguous one; 16-byte
// chunks XOR-swizzled by row on the DMA source address: conflict-free).  The KSP partial
// tiles go to `red` in k_gemm's layout ([row / TM][part][TM][TN + 1]) and k_gemm's epilogue
// (bias / ReLU / mask / fc3 dots / Adam / rowsum / dL/da partials) runs unchanged.  The ring
// aliases `red` (the partials are written after the last slab is consumed).
// Chunks past K are read from a clamped in-row address and zeroed in the fragments (last slab
// only); rows past M / N read a clamped row and are discarded by the epilogue.
typedef __attribute__((address_space(3))) void stg_lds_t;
typedef __attribute__((address_space(1))) const void stg_gbl_t;

template <int N>
__device__ __forceinline__ void stg_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
}
// s_waitcnt vmcnt(n) for a wave-uniform n (an immediate per case)
__device__ __forceinline__ void stg_vmwait_n(int n) {
  switch (n) {
    case 0: stg_vmwait<0>(); break;   case 1: stg_vmwait<1>(); break;
    case 2: stg_vmwait<2>(); break;   case 3: stg_vmwait<3>(); break;
    case 4: stg_vmwait<4>(); break;   case 5: stg_vmwait<5>(); break;
    case 6: stg_vmwait<6>(); break;   case 7: stg_vmwait<7>(); break;
    case 8: stg_vmwait<8>(); break;   case 9: stg_vmwait<9>(); break;
    case 10: stg_vmwait<10>(); break; case 11: stg_vmwait<11>(); break;
    case 12: stg_vmwait<12>(); break; case 13: stg_vmwait<13>(); break;
    case 14: stg_vmwait<14>(); break; default: stg_vmwait<15>(); break;
  }
}

constexpr int kStgKW = 1024;     // K words staged for ax_w / a_ksc (launch_gemm checks K)
constexpr int kStgRing = 144 * 1024;

// geometry of a staged tile: TMW x TN, KSP K parts, 16 waves
template <int TMW, int TN, int KSP>
struct StgGeo {
  static constexpr int NSUB = 16 / KSP, NSM = TMW / 32, NSN = NSUB / NSM;
  static constexpr int WM = 32, WN = TN / NSN, MI = WM / 16, NJ = WN / 16;
  static constexpr int BK = 16 * KSP;
  static constexpr int SLOT = (TMW + TN) * BK * 4;                 // bytes per ring slot
  static constexpr int NST = kStgRing / SLOT < 4 ? kStgRing / SLOT : 4;
  static constexpr int RING = NST * SLOT;
  static_assert(NSUB * KSP == 16 && NSM * 32 == TMW && NSN * NSM == NSUB && NJ * 16 * NSN == TN,
                "staged tile geometry");
  static_assert(NST >= 3 && SLOT % (16 * 1024) == 0, "staged ring");
};

// one operand's slab image: KC -> R rows (M or N) of BK k; MN -> BK rows (k) of R columns
template <int R, int BK, bool KC>
struct StgOp {
  static constexpr int RB = KC ? BK * 4 : R * 4;        // bytes per LDS row
  static constexpr int NR = KC ? R : BK;                 // LDS rows
  static constexpr int CPR = RB / 16;                    // 16-byte chunks per row
  static constexpr int SWZ = (CPR < 16 ? CPR : 16) - 1;  // chunk swizzle mask
  static constexpr int RPP = 1024 / RB;                  // rows per 1 KB piece
  static constexpr int BYTES = NR * RB, PIECES = BYTES / 1024;
  static_assert(RB >= 128 && RB <= 1024 && BYTES % 1024 == 0, "staged operand shape");
};

template <int TM, int TN, int KSP, int MG, bool AKC, bool BKC, bool ROWSUM, int AXF, class Pre>
__device__ __forceinline__ void gemm_core_s(const GemmDesc& d, int m0, int n0, unsigned char* ring,
                                            float* rsum, float* s_kw, Pre&& pre, bool store_a,
                                            tl_word* tl = nullptr) {
  constexpr int TMW = TM * MG;
  using G = StgGeo<TMW, TN, KSP>;
  using OA = StgOp<TMW, G::BK, AKC>;
  using OB = StgOp<TN, G::BK, BKC>;
  constexpr int BK = G::BK, NST = G::NST, SLOT = G::SLOT, MI = G::MI, NJ = G::NJ;
  constexpr int PPW = (OA::PIECES + OB::PIECES) / 16;
  static_assert(OA::PIECES + OB::PIECES == SLOT / 1024 && PPW * 16 == SLOT / 1024 && OA::PIECES % 16 == 0,
                "staged pieces: whole pieces per wave, A pieces first");
  // store_a (AXF): every workgroup issues the same number of stores per slab (zero-length
  // descriptor where it stores nothing), so the counted waits are uniform
  constexpr int SST = AXF == 1 ? (TMW * BK / 4 + 1023) / 1024 : 0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int sub = wave % G::NSUB, kp = wave / G::NSUB;
  const int wm = (sub / G::NSN) * G::WM, wn = (sub % G::NSN) * G::WN;
  const int g4 = lane >> 4, l16 = lane & 15;
  const int K = d.K;
  const int nslab = (K + BK - 1) / BK;
  // staged K vector (AXF: the fc3 weights w; !AKC: the per-k scale, where the desc has one)
  const bool has_ksc = AXF != 1 && !AKC && d.a_ksc != nullptr;
  const float* kwsrc = AXF == 1 ? d.ax_w : d.a_ksc;
  const bool has_kw = AXF == 1 || has_ksc;
  // the K vector goes global -> LDS by DMA too (a ds_write behind the slab DMAs would wait for
  // all of them: the compiler orders LDS stores after an LDS-DMA that may alias): one dword a
  // lane, 64 words a wave, zeros past K (buffer range; zero-length where the level has none)
  static_assert(kStgKW == 16 * 64, "one K-vector DMA per wave");
  {
    const rsrc_t rkw = make_rsrc(has_kw ? kwsrc : d.A, has_kw ? (uint32_t)K * 4u : 0u);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rkw, (stg_lds_t*)(s_kw + wave * 64), 4,
                                             (uint32_t)(wave * 64 + lane) * 4u, 0, 0, 0);
  }
  pre();     // the epilogue's loads: the oldest vector-memory operations of the wave
  // DMA source of each piece this wave moves: piece pc = wave + 16 q (A pieces first)
  const char* pbase[PPW];
  int kofs[PPW];
#pragma unroll
  for (int q = 0; q < PPW; ++q) {
    const int pc = wave + 16 * q;
    const bool isA = q < OA::PIECES / 16;
    const int RPP = isA ? OA::RPP : OB::RPP, CPR = isA ? OA::CPR : OB::CPR, SW = isA ? OA::SWZ : OB::SWZ;
    const bool kc = isA ? AKC : BKC;
    const int Rr = (isA ? pc : pc - OA::PIECES) * RPP + lane / CPR;   // LDS row
    const int c = (lane % CPR) ^ (Rr & SW);                           // global chunk it holds
    const float* base = isA ? d.A : d.B;
    const int ld = isA ? d.lda : d.ldb;
    const int lim = isA ? d.M : d.N;
    const int mn0 = isA ? m0 : n0;
    if (kc) {   // row mn0 + Rr (clamped), k = slab k0 + 4 c
      const int row = mn0 + Rr < lim ? mn0 + Rr : lim - 1;
      pbase[q] = reinterpret_cast<const char*>(base + (size_t)row * ld);
      kofs[q] = 4 * c;
    } else {    // k row = slab k0 + Rr (clamped), column mn0 + 4 c (clamped)
      const int col = mn0 + 4 * c < lim ? mn0 + 4 * c : 0;
      pbase[q] = reinterpret_cast<const char*>(base + col);
      kofs[q] = Rr;
    }
  }
  auto issue = [&](int sl) {
    unsigned char* dst = ring + (sl % NST) * SLOT;
    const int k0 = sl * BK;
#pragma unroll
    for (int q = 0; q < PPW; ++q) {
      const bool isA = q < OA::PIECES / 16;
      const bool kc = isA ? AKC : BKC;
      const int ld = isA ? d.lda : d.ldb;
      const char* g;
      if (kc) {
        const int k = k0 + kofs[q];
        g = pbase[q] + (size_t)(k < K ? k : 0) * 4;
      } else {
        const int k = k0 + kofs[q];
        g = pbase[q] + (size_t)(k < K ? k : K - 1) * ld * 4;
      }
      __builtin_amdgcn_global_load_lds((stg_gbl_t*)g, (stg_lds_t*)(dst + (wave + 16 * q) * 1024), 16, 0, 0);
    }
  };
#pragma unroll
  for (int sl = 0; sl < NST - 1; ++sl)
    if (sl < nslab) issue(sl);
  const rsrc_t rAx = make_rsrc(store_a ? d.ax_out : d.C,
                               store_a ? (uint32_t)(((size_t)(d.M - 1) * d.ax_ld + d.K) * 4) : 0u);
  f4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  float rs[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) rs[i] = 0.f;
  const bool rs_wave = ROWSUM && wn == 0;   // one column of sub-tiles sums the rows
  for (int sl = 0; sl < nslab; ++sl) {
    // vector-memory ops issued after slab sl's DMA: the later prologue slabs, then per
    // iteration i < sl its stores and (while slabs remain) the DMA of slab i + NST - 1
    int younger = 0;
    if (sl < NST - 1) younger += ((NST - 2 < nslab - 1 ? NST - 2 : nslab - 1) - sl) * PPW;
    for (int i = (sl - NST + 2 > 0 ? sl - NST + 2 : 0); i < sl; ++i)
      younger += SST + (i + NST - 1 < nslab ? PPW : 0);
    stg_vmwait_n(younger);
    __builtin_amdgcn_s_barrier();          // slab sl landed for every wave; slot (sl - 1) free
    asm volatile("" ::: "memory");
    if (sl == 0) SACMI_PHASE(tl, 8);
    if (sl == nslab - 1) SACMI_PHASE(tl, 9);
    (void)tl;
    const unsigned char* st = ring + (sl % NST) * SLOT;
    const int kb = sl * BK;
    if constexpr (AXF == 1) {
      // u = transformed A rows of this slab, stored by the column-tile-0 workgroups
#pragma unroll
      for (int q = 0; q < SST; ++q) {
        const int e = tid + 1024 * q, row = e / (BK / 4), c = e % (BK / 4);
        const int k = kb + 4 * c;
        f4 v = {0.f, 0.f, 0.f, 0.f};
        if (row < TMW) {
          const f4 h = *reinterpret_cast<const f4*>(st + row * OA::RB + ((c ^ (row & OA::SWZ)) << 4));
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2) v[s2] = (h[s2] > 0.f && k + s2 < K) ? s_kw[k + s2] : 0.f;
        }
        const bool ok = row < TMW && m0 + row < d.M && k < K;
        buf_st4(rAx, ok ? (uint32_t)((m0 + row) * d.ax_ld + k) * 4u : 0xfffffff0u, v);
      }
    }
    if (sl + NST - 1 < nslab) issue(sl + NST - 1);
    // this wave's 16-deep part of the slab
    float a[MI][4], b[NJ][4];
    const int kk = kp * 16 + 4 * g4;       // the lane group's first k inside the slab
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int r = wm + i * 16 + l16;
      if constexpr (AKC) {
        const int c = kk >> 2;
        const f4 x = *reinterpret_cast<const f4*>(st + r * OA::RB + ((c ^ (r & OA::SWZ)) << 4));
        a[i][0] = x[0]; a[i][1] = x[1]; a[i][2] = x[2]; a[i][3] = x[3];
      } else {
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          const int R = kk + s2;
          a[i][s2] = *reinterpret_cast<const float*>(st + R * OA::RB + ((((r >> 2) ^ (R & OA::SWZ))) << 4) + (r & 3) * 4);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = wn + j * 16 + l16;
      const unsigned char* sb = st + OA::BYTES;
      if constexpr (BKC) {
        const int c = kk >> 2;
        const f4 x = *reinterpret_cast<const f4*>(sb + n * OB::RB + ((c ^ (n & OB::SWZ)) << 4));
        b[j][0] = x[0]; b[j][1] = x[1]; b[j][2] = x[2]; b[j][3] = x[3];
      } else {
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          const int R = kk + s2;
          b[j][s2] = *reinterpret_cast<const float*>(sb + R * OB::RB + ((((n >> 2) ^ (R & OB::SWZ))) << 4) + (n & 3) * 4);
        }
      }
    }
    {
#pragma clang fp contract(off)
      const int k = kb + kk;
      if (K - kb < BK) {   // the last, partial slab: k >= K contributes nothing
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          const bool in = k + s2 < K;
#pragma unroll
          for (int i = 0; i < MI; ++i) a[i][s2] = in ? a[i][s2] : 0.f;
#pragma unroll
          for (int j = 0; j < NJ; ++j) b[j][s2] = in ? b[j][s2] : 0.f;
        }
      }
      if constexpr (AXF == 1) {
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          const float w = s_kw[k + s2 < kStgKW ? k + s2 : 0];
#pragma unroll
          for (int i = 0; i < MI; ++i) a[i][s2] = (a[i][s2] > 0.f && k + s2 < K) ? w : 0.f;
        }
      } else if constexpr (!AKC) {
        if (has_ksc) {
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2) {
            const float f = s_kw[k + s2 < kStgKW ? k + s2 : 0];
#pragma unroll
            for (int i = 0; i < MI; ++i) a[i][s2] *= f;
          }
        }
      }
      mfma_chunk<MI, NJ, false>(acc, a, b);
      if (ROWSUM && rs_wave) {
#pragma unroll
        for (int i = 0; i < MI; ++i) rs[i] += (a[i][0] + a[i][1]) + (a[i][2] + a[i][3]);
      }
    }
  }
  __syncthreads();                          // every wave is past its last ring read
  // partial tiles into red = the ring: red[((row / TM) * KSP + kp) * TM * (TN + 1) + (row % TM) * (TN + 1) + col]
  float* red = reinterpret_cast<float*>(ring);
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm + i * 16 + g4 * 4 + r, col = wn + j * 16 + l16;
        red[((row / TM) * KSP + kp) * TM * (TN + 1) + (row % TM) * (TN + 1) + col] = acc[i][j][r];
      }
  if (ROWSUM && rs_wave) {
    // lanes l, l+16, l+32, l+48 hold the same row: fold the 4 lane groups, fixed order
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      float v = rs[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const int row = wm + i * 16 + lane;
      if (lane < 16) rsum[((row / TM) * KSP + kp) * TM + row % TM] = v;
    }
  }
}

template <int TM, int TN, int KSP, int MG, int AXK, class Pre>
__device__ __forceinline__ void gemm_core_stg(const GemmDesc& d, int m0, int n0, unsigned char* ring,
                                              float* rsum, float* s_kw, bool rowsum, Pre&& pre,
                                              tl_word* tl) {
  if constexpr (AXK == 1) {
    if (d.axk == 1) {
      gemm_core_s<TM, TN, KSP, MG, true, false, false, 1>(d, m0, n0, ring, rsum, s_kw, pre,
                                                          n0 == 0 && d.ax_out != nullptr, tl);
      return;
    }
  }
  if (d.a_kc) {
    if (d.b_kc) gemm_core_s<TM, TN, KSP, MG, true, true, false, 0>(d, m0, n0, ring, rsum, s_kw, pre, false, tl);
    else gemm_core_s<TM, TN, KSP, MG, true, false, false, 0>(d, m0, n0, ring, rsum, s_kw, pre, false, tl);
  } else {
    if (d.b_kc) gemm_core_s<TM, TN, KSP, MG, false, true, false, 0>(d, m0, n0, ring, rsum, s_kw, pre, false, tl);
    else if (rowsum) gemm_core_s<TM, TN, KSP, MG, false, false, true, 0>(d, m0, n0, ring, rsum, s_kw, pre, false, tl);
    else gemm_core_s<TM, TN, KSP, MG, false, false, false, 0>(d, m0, n0, ring, rsum, s_kw, pre, false, tl);
  }
}

// DPP row rotation (within each 16-lane row) of a float
template <int CTRL>
__device__ __forceinline__ float dpp_row(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL,
                                                               0xF, 0xF, false));
}
// sum over a 16-lane row, the total in every lane of the row: row_ror 8, 4, 2, 1 (each
// step adds two equal-shaped partial sums; a + b == b + a, so every lane holds the same bits)
__device__ __forceinline__ float row16_sum(float x) {
#pragma clang fp contract(off)
  x += dpp_row<0x128>(x);
  x += dpp_row<0x124>(x);
  x += dpp_row<0x122>(x);
  x += dpp_row<0x121>(x);
  return x;
}

// Sum of the KSPLIT partials of tile element (row, col); with MG wave groups the
// tile has MG*TM rows and group g's partials sit at waves g*KSPLIT .. g*KSPLIT+KSPLIT-1.
template <int TM, int TN, int KSPLIT, int MG = 1>
__device__ __forceinline__ float reduce_partials(const float* red, int row, int col) {
  const float* base = red + (row / TM) * KSPLIT * TM * (TN + 1) + (row % TM) * (TN + 1) + col;
  float s = base[0];
#pragma unroll
  for (int w = 1; w < KSPLIT; ++w) s += base[w * TM * (TN + 1)];
  return s;
}

// ---------------------------------------------------------------------------
// Adam / Polyak element helpers (torch.optim.Adam single-tensor semantics)
struct AdamScalars { float step_size, bc2_sqrt; };

// t*(1-tau) + p*tau as three separately rounded fp32 ops, like the reference's tensor
// expression (sac_imp.py:149) — no FMA contraction, so the result is bit-exact.
__device__ __forceinline__ float polyak(float t, float p, float omtau, float tau) {
#pragma clang fp contract(off)
  const float a = t * omtau;
  const float b = p * tau;
  return a + b;
}

// bias corrections of torch Adam (bc = 1 - beta^t in double, step_size = lr/bc1),
// from the running products beta^step kept in DevScalars (no pow on the device)
__device__ __forceinline__ AdamScalars adam_scalars(const AdamArgs& a, int step_idx) {
  double p1 = a.sc->beta_pow[step_idx][0], p2 = a.sc->beta_pow[step_idx][1];
  if (a.step_offset) { p1 *= (double)a.beta1; p2 *= (double)a.beta2; }
  const double bc1 = 1.0 - p1;
  const double bc2 = 1.0 - p2;
  return AdamScalars{(float)((double)a.lr / bc1), (float)sqrt(bc2)};
}

__device__ __forceinline__ AdamScalars fuse_scalars(const AdamFuse& a, int step_idx, int offset) {
  double p1 = a.sc->beta_pow[step_idx][0], p2 = a.sc->beta_pow[step_idx][1];
  if (offset) { p1 *= (double)a.beta1; p2 *= (double)a.beta2; }
  return AdamScalars{(float)((double)a.lr / (1.0 - p1)), (float)sqrt(1.0 - p2)};
}

// Every op separately rounded (no FMA contraction): the fused-epilogue Adam and the
// stand-alone Adam kernel then produce identical bits, and the op order is torch's
// (exp_avg.lerp_, exp_avg_sq.mul_().addcmul_(), sqrt/bc2 + eps, addcdiv_).
__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, float om_b1,
                                          float b2, float om_b2, float eps, AdamScalars k) {
#pragma clang fp contract(off)
  m = m + om_b1 * (g - m);
  v = v * b2;
  v = v + om_b2 * g * g;
  const float denom = sqrtf(v) / k.bc2_sqrt + eps;
  p = p + (-k.step_size * m) / denom;
}

// Block 0 of a fused-Adam level (k_gemm / k_dw_fin): the level's losses, the scalar
// log_alpha step (alpha = exp(log_alpha), sac_imp.py:128-135) and the loss ring slot —
// none of them after a non-finite sample (the reference raised first; err: ErrBits this
// update saw) — and the error bits for the synchronous step's host-mapped readback.
// Scalar loads through a buffer descriptor (s_buffer_load): counted by lgkmcnt, so their
// wait never includes the vector stores the workgroup has in flight (vmcnt retires loads and
// stores in order: a vector load issued behind the fused-Adam epilogue's write-through
// stores waits for their acknowledgements, ~2 us).  Only for data an earlier kernel wrote
// (the scalar cache is invalidated at every kernel start, and this kernel has not stored it).
typedef int sbuf_i4 __attribute__((ext_vector_type(4)));
__device__ int llvm_s_buffer_load_i32(sbuf_i4 rsrc, int off, int aux) __asm("llvm.amdgcn.s.buffer.load.i32");
__device__ __forceinline__ sbuf_i4 s_rsrc(const void* p) {
  const uint64_t a = (uint64_t)p;
  return sbuf_i4{(int)(uint32_t)a, (int)((uint32_t)(a >> 32) & 0xffffu), 0x7fffffff, kBufDword3};
}
__device__ __forceinline__ uint32_t s_ld(sbuf_i4 r, uint32_t byte_off) {
  return (uint32_t)llvm_s_buffer_load_i32(r, (int)byte_off, 0);
}

// The fused-Adam level's scalar work (losses, the alpha step, the loss ring, the done word),
// by ONE wave, on wave-uniform values read by scalar loads (s_ld).  Every value it reads
// was written by an earlier level, and nothing of the level reads what it writes, so it
// runs at the level's start (k_gemm, GemmBatch::adam_wg -2: wave 0 of block 0 before its
// tile) — after the tile it made block 0 the level's last workgroup by 2.7-2.9 us (a chain
// of dependent round trips, then a system-scope fence; phase stamps, profiles/r04).
__device__ __forceinline__ void adam_block0_wave(const AdamFuse& af, int err, float omb1, float omb2) {
  const sbuf_i4 rLp = s_rsrc(af.loss_part), rSc = s_rsrc(af.sc);
  const bool alpha = af.log_alpha_idx >= 0 && af.auto_entropy;
  const uint32_t ao = (uint32_t)(alpha ? af.log_alpha_idx : 0) * 4u;
  float pp = __uint_as_float(s_ld(s_rsrc(af.P), ao)), mm = __uint_as_float(s_ld(s_rsrc(af.M), ao));
  float vv = __uint_as_float(s_ld(s_rsrc(af.V), ao));
  const float ga = __uint_as_float(s_ld(s_rsrc(alpha ? af.log_alpha_grad : af.P), 0u));   // (used only with alpha)
  auto s_ld64 = [&](size_t off) {
    return (uint64_t)s_ld(rSc, (uint32_t)off) | ((uint64_t)s_ld(rSc, (uint32_t)off + 4u) << 32);
  };
  double bp1 = __longlong_as_double((long long)s_ld64(offsetof(DevScalars, beta_pow) + 3 * 16));
  double bp2 = __longlong_as_double((long long)s_ld64(offsetof(DevScalars, beta_pow) + 3 * 16 + 8));
  const int64_t pos = (int64_t)s_ld64(offsetof(DevScalars, loss_ring_pos));
  float l_prev[3];
#pragma unroll
  for (int sl = 0; sl < 3; ++sl)
    l_prev[sl] = __uint_as_float(s_ld(rSc, (uint32_t)(offsetof(DevScalars, losses) + 4 * sl)));
  const int dseq = (int)s_ld(rSc, (uint32_t)offsetof(DevScalars, done_seq));
  const bool lane0 = threadIdx.x == 0;
  if (lane0 && af.loss_host) af.loss_host[3] = __int_as_float(err);
  // the level's losses: partials summed in block order (as k_adam does)
  float loss[2] = {0.f, 0.f};
#pragma unroll
  for (int l = 0; l < 2; ++l) {
    if (l >= af.n_losses) break;
    float sum = 0.f;
    for (int w = 0; w < af.n_part; ++w) sum += __uint_as_float(s_ld(rLp, (uint32_t)(w * af.n_losses + l) * 4u));
    loss[l] = sum / af.loss_div;
    if (lane0 && !err) {
      af.sc->losses[af.loss_slot0 + l] = loss[l];
      if (af.loss_host) af.loss_host[af.loss_slot0 + l] = loss[l];
    }
  }
  if (lane0 && alpha && !err) {
    if (af.step_offset) { bp1 *= (double)af.beta1; bp2 *= (double)af.beta2; }
    const AdamScalars k{(float)((double)af.lr / (1.0 - bp1)), (float)sqrt(1.0 - bp2)};
    adam_elem(pp, mm, vv, ga, omb1, af.beta2, omb2, af.eps, k);
    af.P[af.log_alpha_idx] = pp; af.M[af.log_alpha_idx] = mm; af.V[af.log_alpha_idx] = vv;
    af.sc->alpha = expf(pp);
    af.sc->alpha_is_tensor = 1;
  }
  if (lane0 && af.loss_ring && !err) {
    const int64_t q = pos % af.ring;
#pragma unroll
    for (int sl = 0; sl < 3; ++sl) {
      const int src = sl - af.loss_slot0;
      af.loss_ring[q * 3 + sl] = src == 0 ? loss[0] : src == 1 && af.n_losses > 1 ? loss[1] : l_prev[sl];
    }
    af.sc->loss_ring_pos = pos + 1;
  }
  if (lane0 && af.done_word) {   // (voided updates too: the host waits on it)
    const int v = dseq + 1;
    af.sc->done_seq = v;
    __threadfence_system();                  // the losses and error bits land first
    *reinterpret_cast<volatile int*>(af.done_word) = v;
  }
}
// ... after the block's tile (adam_wg -1, or a dedicated workgroup): wave 0
__device__ __forceinline__ void adam_block0(const AdamFuse& af, int err, float omb1, float omb2) {
  __syncthreads();
  if (threadIdx.x >= 64) return;
  adam_block0_wave(af, err, omb1, omb2);
}

// Polyak workgroup w of nw (RideAlong::pk): grid-stride float4 groups of the critic arena,
// every load of a thread's groups issued before its stores; the same three separately
// rounded fp32 ops as the Adam epilogue's form (bit-exact with the reference)
__device__ __forceinline__ void polyak_ride(const PolyakArgs& a, int w, int nw) {
  if (a.sc->err) return;   // the reference raised before sac_imp.py:138 (ErrBits)
  const float omtau = 1.f - a.tau;
  const rsrc_t rT = make_rsrc(a.T, 0x7fffffffu), rP = make_rsrc(a.P, 0x7fffffffu);
  constexpr int kPer = 2;     // groups per thread per pass
  const int64_t stride = (int64_t)nw * blockDim.x * kPer;
  for (int64_t g0 = (int64_t)w * blockDim.x * kPer + threadIdx.x; g0 < a.n4; g0 += stride) {
    float4 t[kPer], p[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int64_t g = g0 + (int64_t)k * blockDim.x;
      const uint32_t o = g < a.n4 ? (uint32_t)g * 16u : 0xfffffff0u;
      t[k] = buf_ld4(rT, o);
      p[k] = buf_ld4(rP, o);
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int64_t g = g0 + (int64_t)k * blockDim.x;
      if (g >= a.n4) break;
      const float x = polyak(t[k].x, p[k].x, omtau, a.tau), y = polyak(t[k].y, p[k].y, omtau, a.tau),
                  z = polyak(t[k].z, p[k].z, omtau, a.tau), u = polyak(t[k].w, p[k].w, omtau, a.tau);
      buf_st4<kStAux>(rT, (uint32_t)g * 16u, f4{x, y, z, u});
      if (a.Th) st_wt8(a.Th, (uint32_t)g * 8u, (uint32_t)bf16_bits(x) | ((uint32_t)bf16_bits(y) << 16),
                       (uint32_t)bf16_bits(z) | ((uint32_t)bf16_bits(u) << 16));
    }
  }
}

// ---------------------------------------------------------------------------
// grouped GEMM: one launch runs every independent GEMM of one dependency level.
// One workgroup (16 waves, K split 16 ways) per output tile, one workgroup per CU.
// Block 0 of an Adam-fused level also finalises the losses, takes the scalar
// log_alpha step (alpha = exp(log_alpha), sac_imp.py:128-135) and fills the loss ring.
// Row prologue of an axk-1 level (runs inside pre(), i.e. while the operand loads are in
// flight): four threads per batch row sum the dot partials of its heads, the row's
// thread loads r, d, logp meanwhile and turns the heads into the per-row coefficients
// of the backward —
//   critic (sac_imp.py:87-113): q^ = r + (1-d) gamma (min(qt1,qt2) - alpha logp'),
//           coef_i = dL/dq_i = 2 (q_i - q^) / B, loss partial sum (q_i - q^)^2
//   actor (sac_imp.py:116-121): coef_i = dL/dqa_i = -[i is the min]/B (ties 1/2 : 1/2),
//           loss partial sum (alpha logp - min qa)
// `writer` (one workgroup per row block) stores the coefficients and the loss partial;
// the actor's block 0 also advances the step counters and forms dL/dlog_alpha.  Every
// thread of the workgroup calls it (two barriers).
// Registers a thread carries from rows_load() (before the operand loads) to
// rows_finish() (after them).  Every prologue load is issued in rows_load() and consumed
// only in rows_finish(): vmcnt retires in order, so a value consumed before the operand
// burst would hold the burst back, and one loaded after it would wait for all of it.
constexpr int kRowsPv = 16;    // dot partials held per (row, slot) thread: H <= 512
struct RowsRegs {
  float pv[kRowsPv];          // thread (row, slot) < TMW*nslot: the row's dot partials
  float r, d, lp, alpha;      // thread row < TMW: the row's own inputs
  float lpa;                  // actor block 0, wave past the row threads: logp_part[lane]
};

template <int TMW, int NTH, int AUX = 0>
__device__ __forceinline__ void rows_load(const RowsFuse& rf, const GemmDesc& d, int m0,
                                          RowsRegs& x) {
  const int t = threadIdx.x;
  const int nslot = rf.kind == 1 ? 4 : 2;
  // unconditional buffer loads (a guarded load is drained at the end of its guard);
  // descriptors of zero length where this desc has no prologue (nothing is read), and
  // reads past a range for the threads / parts that have none (they return 0)
  const bool on = d.axk == 1;
  const uint32_t big = 0x7fffffffu, oob = 0xfffffff0u;
  const rsrc_t rPart = make_rsrc(on ? rf.part : d.C, on ? big : 0u);
  const rsrc_t rLp = make_rsrc(on ? rf.logp : d.C, on ? big : 0u);
  const rsrc_t rR = make_rsrc(on ? (rf.kind == 1 ? rf.r : rf.logp) : d.C, on ? big : 0u);
  const rsrc_t rD = make_rsrc(on ? (rf.kind == 1 ? rf.d : rf.logp) : d.C, on ? big : 0u);
  const rsrc_t rLpa = make_rsrc(on && rf.logp_part ? rf.logp_part : d.C, on && rf.logp_part ? big : 0u);
  const rsrc_t rSc = make_rsrc(on ? &rf.sc->alpha : d.C, on ? 4u : 0u);
  {
    const int row = t / nslot, sl = t % nslot;
    const bool ok = t < TMW * nslot && m0 + row < rf.B;
    const uint32_t base = (uint32_t)(((size_t)sl * rf.B + m0 + row) * rf.nparts) * 4u;
#pragma unroll
    for (int i = 0; i < kRowsPv; ++i)
      x.pv[i] = buf_ld_aux<AUX>(rPart, ok && i < rf.nparts ? base + 4u * i : oob);
  }
  const int b = m0 + t;
  const uint32_t ob = (uint32_t)((t < TMW && b < rf.B) ? b : 0) * 4u;
  x.alpha = buf_ld_aux<AUX>(rSc, 0u);
  x.lp = buf_ld_aux<AUX>(rLp, ob);
  x.r = buf_ld_aux<AUX>(rR, ob);
  x.d = buf_ld_aux<AUX>(rD, ob);
  const int lane = t - TMW * nslot;
  x.lpa = buf_ld_aux<AUX>(rLpa, (uint32_t)(2 * (lane >= 0 && lane < rf.n_lp ? lane : 0) + 1) * 4u);
}

template <int TMW, int NTH>
__device__ void rows_finish(const RowsFuse& rf, const GemmDesc& d, int m0, bool writer,
                            bool first_block, const RowsRegs& x0,
                            float (*s_q)[4], float (*s_coef)[TMW], float (*s_l)[2]) {
  const int t = threadIdx.x;
  const int nslot = rf.kind == 1 ? 4 : 2;
  // pin every prologue value to this point (after the MFMAs): without it the compiler
  // hoists cheap uses (e.g. 0 + lpa) up to the loads, and their wait then holds the
  // operand loads back
  RowsRegs x = x0;
#pragma unroll
  for (int q = 0; q < kRowsPv; ++q) asm volatile("" : "+v"(x.pv[q]));
  asm volatile("" : "+v"(x.r), "+v"(x.d), "+v"(x.lp), "+v"(x.lpa), "+v"(x.alpha));
  if (t < TMW * nslot) {
    // the row's partials summed in column order (block 0's carries the fc3 bias)
    const int row = t / nslot, sl = t % nslot;
    float acc = x.pv[0];
#pragma unroll
    for (int i = 1; i < kRowsPv; ++i)
      if (i < rf.nparts) acc += x.pv[i];
    for (int i = kRowsPv; i < rf.nparts; ++i)     // H > 512 only
      acc += rf.part[((size_t)sl * rf.B + m0 + row) * rf.nparts + i];
    s_q[row][sl] = m0 + row < rf.B ? acc : 0.f;
  }
  if (first_block && rf.kind == 2) {
    const int w0 = TMW * nslot;            // first wave past the partial-sum threads
    if (t >= w0 && t < w0 + 64) {
      // dL/dlog_alpha = -mean(logp_a + te) (sac_imp.py:128-133) from the heads kernel's
      // per-workgroup sums: strided per lane, then a fixed butterfly
      const int lane = t - w0;
      float acc = 0.f;
      if (rf.alpha_grad) {
        if (lane < rf.n_lp) acc += x.lpa;
        for (int w = lane + 64; w < rf.n_lp; w += 64) acc += rf.logp_part[2 * w + 1];
      }
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
      if (lane == 0) {
        if (rf.alpha_grad) *rf.alpha_grad = -(acc + (float)rf.B * rf.target_entropy) / (float)rf.B;
        // step counters: the critic Adam ran before this level, the actor Adam after.  After
        // a non-finite policy sample (ErrBits) only the steps the reference took advance —
        // none (target batch / PER / an earlier update), or the critics' (actor batch,
        // sac_imp.py:116 raises after the q optimizers stepped) — selected, not branched:
        // every load goes out at once
        const int err = rf.sc->err;
        const bool any = (err & kErrSkipAll) == 0;
        const bool all = any && (err & kErrActLike) == 0;
        for (int i = 0; i < 4; ++i) {
          const bool adv = all || (any && (i == 1 || i == 2));
          rf.sc->step[i] += adv ? 1.0 : 0.0;
          rf.sc->beta_pow[i][0] *= adv ? 0.9 : 1.0;   // torch Adam default betas (sac_imp.py:39-49)
          rf.sc->beta_pow[i][1] *= adv ? 0.999 : 1.0;
        }
        rf.sc->noise_counter += all ? 1 : 0;
        if (any && !all) atomicOr(&rf.sc->err, (int)ERR_ABORT);
      }
    }
  }
  __syncthreads();
  SACMI_STAMP(36);
  const int b = m0 + t;
  if (t < TMW) {
    float c0 = 0.f, c1 = 0.f, l0 = 0.f, l1 = 0.f;
    if (b < rf.B) {
      if (rf.kind == 1) {
        const float vt = fminf(s_q[t][2], s_q[t][3]) - x.alpha * x.lp;
        const float qhat = x.r + ((1.f - x.d) * rf.gamma) * vt;
        const float e1 = s_q[t][0] - qhat, e2 = s_q[t][1] - qhat;
        c0 = 2.f * e1 / (float)rf.B;
        c1 = 2.f * e2 / (float)rf.B;
        l0 = e1 * e1;
        l1 = e2 * e2;
      } else {
        const float q1 = s_q[t][0], q2 = s_q[t][1];
        l0 = x.alpha * x.lp - fminf(q1, q2);
        const float g = -1.f / (float)rf.B;
        const float w1 = q1 < q2 ? 1.f : (q1 == q2 ? 0.5f : 0.f);
        c0 = g * w1;
        c1 = g * (1.f - w1);
      }
      if (writer && rf.dq) { rf.dq[b] = c0; rf.dq[rf.B + b] = c1; }
      if (writer && rf.dq4) { rf.dq4[(size_t)b * 4] = c0; rf.dq4[((size_t)rf.B + b) * 4] = c1; }
    }
    s_coef[0][t] = c0; s_coef[1][t] = c1;
    s_l[t][0] = l0; s_l[t][1] = l1;
  }
  __syncthreads();                         // coefficients visible to the epilogue
  SACMI_STAMP(35);
}

// the row block's loss partial (fixed row order), at the very end of the kernel: a
// serial LDS chain nobody else waits for
template <int TMW>
__device__ __forceinline__ void rows_loss(const RowsFuse& rf, int m0, bool writer,
                                          const float (*s_l)[2]) {
  // one partial per 32-row block whatever the tile height: the host sizes and reduces
  // them per 32 rows, and the bits do not depend on the tile configuration
  const int t = threadIdx.x;
  const int nl = rf.kind == 1 ? 2 : 1;
  if (writer && t < nl * (TMW / 32)) {
    const int h = t / nl, l = t % nl;
    float acc = 0.f;
    for (int r = 32 * h; r < 32 * h + 32; ++r) acc += s_l[r][l];
    if (m0 + 32 * h < rf.B) rf.loss_part[(m0 / 32 + h) * nl + l] = acc;
  }
}

// LDS-staged 128x128 forward kernel for large-M levels (k_fwd) and its tile threshold
#ifndef SACMI_FWD_BIG
#define SACMI_FWD_BIG 1
#endif
#ifndef SACMI_DW_SPLIT
#define SACMI_DW_SPLIT 1
#endif
#ifndef SACMI_FWD_BF16_N64
#define SACMI_FWD_BF16_N64 1
#endif
#ifndef SACMI_FWD_BF16_ALL64
#define SACMI_FWD_BF16_ALL64 0
#endif
#ifndef SACMI_FWD_BIG_FP32
#define SACMI_FWD_BIG_FP32 0
#endif
#ifndef SACMI_FWD_BIG_MIN
#define SACMI_FWD_BIG_MIN 1      // x 256 tiles of 128x128
#endif
// K split per wave group of the batch-4096-class tile configurations (tuning knobs)
#ifndef SACMI_FWD_KS
#define SACMI_FWD_KS 4
#endif
#ifndef SACMI_AXK_KS
#define SACMI_AXK_KS 4
#endif
#ifndef SACMI_DW_KS
#define SACMI_DW_KS 8
#endif
#ifndef SACMI_PIPE
#define SACMI_PIPE 0
#endif
#ifndef SACMI_PIN_EPI
#define SACMI_PIN_EPI 1         // k_gemm: the epilogue's desc fields in the K loop's round trip
#endif
#ifndef SACMI_PIPE_DW
#define SACMI_PIPE_DW 0
#endif

// data-parallel phase 0: the update's error flags for the critic gradient collective
// (kDpFlagN; GemmBatch::err_flags).  Every error source of the update ran before this level.
__device__ __forceinline__ void store_err_flags(const GemmBatch& b) {
  if (b.err_flags && blockIdx.x == 0 && threadIdx.x == 0) {
    const int err = *b.err_word;
    b.err_flags[0] = (err & kErrSkipAll) ? 1.f : 0.f;
    b.err_flags[1] = (err & kErrActLike) ? 1.f : 0.f;
    b.err_flags[2] = 0.f;
    b.err_flags[3] = 0.f;
  }
}

// the policy heads + GaussianPolicy.sample of rows [m0, m0 + TM) (defined with k_heads_sample;
// k_gemm runs it folded into the last policy hidden layer's level, GemmBatch::heads)
// ---------------------------------------------------------------------------
// Philox4x32-10 + Box-Muller (perf-mode policy noise)
__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[0] = n0; c[1] = (uint32_t)p1; c[2] = n2; c[3] = (uint32_t)p0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}

__device__ __forceinline__ float philox_normal(uint64_t seed, uint64_t counter, uint32_t elem) {
  uint32_t c[4] = {(uint32_t)counter, (uint32_t)(counter >> 32), elem, 0x5ac3u};
  philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const float u1 = ((float)c[0] + 0.5f) * 2.3283064365386963e-10f;   // (0,1)
  const float u2 = ((float)c[1] + 0.5f) * 2.3283064365386963e-10f;
  return sqrtf(-2.f * logf(u1)) * cospif(2.f * u2);
}

constexpr float kLogSqrt2Pi = 0.91893853320467274178f;   // math.log(math.sqrt(2*pi))

// 1 - tanh(x)^2 = sech(x)^2 = 4t / (1+t)^2 with t = exp(-2|x|): the reference's
// `1 - y.pow(2)` (networks_model1.py:93) without its cancellation — for |x| ~ 4 the fp32
// difference keeps only ~12 good bits, and those few saturated elements dominate the
// policy gradient through 2y / (1 - y^2) (batch-4096 runs: 1e-4 normwise scatter between
// fp32 evaluations otherwise; this form tracks the fp64 truth)
__device__ __forceinline__ float one_minus_tanh2(float x) {
  const float t = expf(-2.f * fabsf(x));
  const float u = 1.f + t;
  return 4.f * t / (u * u);
}

// one (row m, action j) element of GaussianPolicy.sample from its head sums (bias added):
// the action, cache and noise stores and the NaN check; returns the element's log-prob term
template <bool H16, int AAUX>
__device__ __forceinline__ float heads_elem(const HeadSampleArgs& a, int m, int j, float mean, float ls_raw,
                                            float eps_in, uint64_t ctr) {
  const int A = a.A;
  const float ls = fminf(fmaxf(ls_raw, -20.f), 2.f);
  const float sd = expf(ls);
  // Normal(mean, std) argument validation (networks_model1.py:87): loc must be real (not
  // NaN) and scale positive — std = exp(clamp(log_std)) is NaN only for a NaN log_std
  // (torch.clamp keeps NaN; fmaxf above does not, hence the raw value).  evaluate=True
  // (deterministic) builds no Normal, so nothing is checked there (sac_imp.py:59-65).
#if defined(SACMI_EXP_NOMFMA) || defined(SACMI_EXP_NOLOAD) || defined(SACMI_EXP_NOADAMIO) || \
    defined(SACMI_EXP_EMPTY) || defined(SACMI_EXP_DESC) || defined(SACMI_EXP_NOSTORE)
  if (false) {   // timing experiments compute garbage: never void their updates
#else
  if (a.nan_flag && !a.deterministic && (__builtin_isnan(mean) || __builtin_isnan(ls_raw))) {
#endif
    const int bit = m < a.split_row ? a.nan_bit_lo : a.nan_bit_hi;
    if (a.nan_plain) *a.nan_flag = bit;
    else atomicOr(a.nan_flag, bit);
  }
  float eps;
  if (a.deterministic) {
    eps = 0.f;
  } else if (a.gen_eps) {
    eps = philox_normal(a.seed, ctr, (uint32_t)(m * A + j));
    a.eps[(size_t)m * A + j] = eps;
  } else {
    eps = eps_in;
  }
  const float x = a.deterministic ? mean : mean + eps * sd;
  const float y = tanhf(x);
  if constexpr (H16)
    reinterpret_cast<unsigned short*>(a.act)[(size_t)m * a.ldact + j] = bf16_bits(y * a.scale + a.bias);
  else   // (write-through where the same launch reads them back: k_chain_a's L3)
    st_pol(a.act + (size_t)m * a.ldact + j, y * a.scale + a.bias, AAUX != 0);
  if (a.act_host) a.act_host[(size_t)m * A + j] = y * a.scale + a.bias;
  const float dx = x - mean;
  float lpe = -(dx * dx) / (2.f * (sd * sd)) - logf(sd) - kLogSqrt2Pi;
  const float omy2 = one_minus_tanh2(x);
  lpe -= logf(a.scale * omy2 + 1e-6f);
  float* cr = a.cache + (size_t)m * 3 * A;
  cr[j] = omy2; cr[A + j] = ls_raw; cr[2 * A + j] = y;
  return lpe;
}

// rows [m0, m0 + TM): the log-prob row sums from lp (every thread of the workgroup calls it)
// and the row block's logp_part slot pair
template <int TM, int AAUX>
__device__ __forceinline__ void heads_logp(const HeadSampleArgs& a, int m0, int part, float (*lp)[33],
                                           float* s_lp) {
  const int A = a.A;
  __syncthreads();
  if (threadIdx.x < TM) {
    const int mm = m0 + threadIdx.x;
    float s = 0.f;
    if (mm < a.rows) {
      for (int jj = 0; jj < A; ++jj) s += lp[threadIdx.x][jj];
      st_pol(a.logp + mm, s, AAUX != 0);
    }
    s_lp[threadIdx.x] = s;
  }
  if (a.logp_part) {
    __syncthreads();
    if (threadIdx.x < 2) {    // rows below / at-or-above split_row, fixed order
      float s = 0.f;
      for (int r = 0; r < TM; ++r) {
        const int mm = m0 + r;
        if (mm < a.rows && (mm >= a.split_row) == (threadIdx.x == 1)) s += s_lp[r];
      }
      a.logp_part[2 * part + threadIdx.x] = s;
    }
  }
}

template <int TN, int KSPLIT, bool H16, int TM, int AAUX>
__device__ __forceinline__ void heads_rows(const HeadSampleArgs& a, int m0, int part, float* red,
                                           float (*lp)[33], float* s_lp);

// waves per SIMD the register allocation must allow: every wave of the workgroup
// resident at once, one workgroup per CU
template <int W>
constexpr int gemm_min_waves() { return 4; }   // 16 waves per CU: one 1024- or two 512-thread WGs

// TM x TN per wave group, MG wave groups (workgroup tile MG*TM x TN), K split KSPLIT
// ways inside each group; ADAM: fused optimizer epilogue (every desc EPI_ADAM*); BF16:
// bf16 MFMA operands (GemmBatch::bf16), everything around them fp32
// CORE 0: register-direct operand loads, K split KSPLIT ways across 64*KSPLIT*MG threads;
// CORE 1: the LDS-staged core (gemm_core_s), 1024 threads, KSPLIT = its K parts (partial tiles)
template <int KSPLIT, int MG, int CORE>
constexpr int gemm_threads() { return CORE ? 1024 : 64 * KSPLIT * MG; }
template <int CORE, int TMW, int TN, int KSP>
constexpr int stg_ring() {
  if constexpr (CORE == 1) return StgGeo<TMW, TN, KSP>::RING;
  else return 1;
}
// LDS of one k_gemm configuration (kg_body)
template <int TM, int TN, int KSPLIT, int G, int MG, bool ADAM, int AXK, bool BF16, int CORE, bool HFOLD = false>
constexpr bool kg_heads_fold() {
  // (an instantiation of its own: the fold's registers and code cost the plain levels of
  // this tile configuration ~0.6-0.8 us each when compiled in)
  return HFOLD && !ADAM && AXK == 0 && CORE == 0 && !BF16 && MG == 1 && TM == kHeadsFoldTM && TN == 64 &&
         KSPLIT == 16 && G == 2;
}
template <int TM, int TN, int KSPLIT, int G, int MG, bool ADAM, int AXK, bool BF16, int CORE, bool HFOLD = false>
struct KgSmem {
  static constexpr int TMW = TM * MG;
  static constexpr bool PA = AXK == 1 && MG == 1;
  static constexpr bool HF = kg_heads_fold<TM, TN, KSPLIT, G, MG, ADAM, AXK, BF16, CORE, HFOLD>();
  alignas(16) unsigned char ring[stg_ring<CORE, TMW, TN, KSPLIT>()];
  float red_l[CORE ? 1 : MG * KSPLIT * TM * (TN + 1)];
  float s_kw[CORE ? kStgKW : 1];
  float rsum[MG * KSPLIT * TM];
  AdamScalars s_k;
  int s_err;
  float s_q[TMW][4], s_coef[2][TMW], s_l[TMW][2], s_dotw[TN];
  float s_pa[PA ? TMW * (TN + 1) + TN * 32 : 1];
  float s_hlp[HF ? kHeadsFoldTM * (TN + 1) : 1];   // the tile's h (folded heads' partial)
  int s_hlast;
};

// The body of one k_gemm workgroup: work item `bid_in` of the level (a tile, a ride-along
// workgroup, the scalar Adam workgroup).  k_gemm runs it as blockIdx.x; the persistent chain
// kernel (k_chain) runs it for each work item of its cohort.  LDAUX: cache-policy bits of the
// loads of operands another workgroup of the SAME launch produced (the A operand, the row
// prologue's dot partials, the ReLU-mask source): sc1 (16) in k_chain, 0 in k_gemm.
// MIDSPLIT (k_chain): mid (ChainWait) — the previous phase's cohort barrier — issues its first
// poll at entry (mid.issue()) and waits (mid()) inside the K loop's load burst, after the
// weights' loads and before the A operand's (gemm_core_l), or before a return that loads
// nothing; every workgroup that calls the body with it reaches both once.
template <int TM, int TN, int KSPLIT, int G, int MG, bool ADAM, int AXK, bool BF16, int CORE, int LDAUX,
          bool MIDSPLIT = false, bool HFOLD = false, class Mid = void (*)()>
__device__ __forceinline__ void kg_body(const GemmBatch& batch, const int bid_in,
                                        KgSmem<TM, TN, KSPLIT, G, MG, ADAM, AXK, BF16, CORE, HFOLD>& sm,
                                        Mid&& mid = [] {}) {
  if constexpr (MIDSPLIT) mid.issue();   // (k_chain: the barrier's first poll, ahead of every load)
  // The scalars that locate this workgroup's work come in ONE kernarg round trip: left to
  // the compiler, each load sat behind a branch on the previous one (timeline pointer, tile
  // count, one desc's tile_begin per loop trip, then the desc's fields as they were used),
  // ~1-1.5 us of dependent scalar round trips before the first operand load of every level
  // (phase stamps, tools/phase_dump.py).  The asm pins force each value into an SGPR
  // there, so every load is issued before the one wait.
  tl_word* const tl = batch.tl;
  const int n_tiles = batch.total_tiles, n_desc = batch.count;
  int tbeg[kMaxGemms];
#pragma unroll
  for (int q = 0; q < kMaxGemms; ++q) tbeg[q] = batch.d[q].tile_begin;
  const int adam_wg = batch.adam_wg;
  // (k_chain runs several bodies in one register allocation: there the pins would keep ~40
  // SGPRs of each level live at once — spills — so it leaves the loads to the compiler)
  constexpr bool PINS = LDAUX == 0;
  if constexpr (PINS) {
    asm volatile("" :: "s"(tl), "s"(n_tiles), "s"(n_desc), "s"(adam_wg));
#pragma unroll
    for (int q = 0; q < kMaxGemms; ++q) asm volatile("" :: "s"(tbeg[q]));
  }
#if SACMI_PIN_EPI
  // ... with the level-wide epilogue scalars that do not depend on the desc (the row
  // prologue's / fused Adam's pointers): otherwise their loads sit behind the desc's
  if constexpr (!PINS) {
  } else if constexpr (AXK == 1) {
    const RowsFuse& r = batch.rows;
    asm volatile("" :: "s"(r.part), "s"(r.logp), "s"(r.r), "s"(r.d), "s"(r.kind), "s"(r.nparts),
                 "s"(r.B), "s"(r.sc), "s"(r.logp_part), "s"(r.n_lp));
  } else if constexpr (ADAM) {
    const AdamFuse& a = batch.adam;
    asm volatile("" :: "s"(a.P), "s"(a.M), "s"(a.V), "s"(a.T), "s"(a.G), "s"(a.t_base), "s"(a.sc),
                 "s"(a.step_offset));
  }
#endif
  SACMI_PHASE(tl, 0);
  SACMI_PHASE_LAST(tl, 6);
  constexpr int TMW = TM * MG;
  static_assert(!CORE || !BF16, "the staged core is fp32");
  // CORE 1: the operand ring, which the partial tiles (`red`) alias after the K loop; its
  // K vector (ax_w / a_ksc) staging
  constexpr int RING = stg_ring<CORE, TMW, TN, KSPLIT>();
  static_assert(!CORE || RING >= MG * KSPLIT * TM * (TN + 1) * 4, "staged ring holds the partial tiles");
  // LDS (KgSmem: the caller's, so that a persistent kernel can run several configurations
  // in one allocation)
  unsigned char* const ring = sm.ring;
  float* const red = CORE ? reinterpret_cast<float*>(sm.ring) : sm.red_l;
  float* const s_kw = sm.s_kw;
  float* const rsum = sm.rsum;
  AdamScalars& s_k = sm.s_k;
  int& s_err = sm.s_err;
  auto& s_q = sm.s_q;
  auto& s_coef = sm.s_coef;
  auto& s_l = sm.s_l;
  auto& s_dotw = sm.s_dotw;
  // dL/da partials (axk-1 levels of one 32-row wave group): the tile's outputs [TMW][TN+1]
  // and its fc1 action weights [TN][32]
  constexpr bool PA = AXK == 1 && MG == 1;
  float* const s_pa = sm.s_pa;
  // the policy heads folded into this level (GemmBatch::heads): the fp32 32x64 forward tiles
  constexpr bool HF = kg_heads_fold<TM, TN, KSPLIT, G, MG, ADAM, AXK, BF16, CORE, HFOLD>();
  float* const s_hlp = sm.s_hlp;
  int& s_hlast = sm.s_hlast;
  const int bid = bid_in;
#ifdef SACMI_EXP_EMPTY
  if (bid < batch.total_tiles) return;   // timing experiment only: the launch, nothing else
#endif
#ifdef SACMI_EXP_DESC
  {   // timing experiment only: the launch + this workgroup's descriptor, then out
    int pq = 0;
    for (int q = 1; q < batch.count; ++q)
      if (bid >= batch.d[q].tile_begin) pq = q;
    if (bid < batch.total_tiles && batch.d[pq].M == -7) red[threadIdx.x] = 1.f;
    if (bid < batch.total_tiles) return;
  }
#endif
  if (bid >= n_tiles && MIDSPLIT) mid();   // (k_chain: rides read nothing of the chain)
  if (bid >= n_tiles && bid == adam_wg) {
    // the level's scalar Adam work on a workgroup of its own, at once: its inputs (loss
    // partials, log_alpha's gradient, the scalars) come from earlier levels, and no tile's
    // workgroup waits behind it (block 0 did it after its tile: +2.6-3 us on the level)
    const AdamFuse& af = batch.adam;
    adam_block0(af, af.sc->err, 1.f - af.beta1, 1.f - af.beta2);
    return;
  }
  if (bid >= n_tiles) {   // ride-along workgroups (next update's replay work, Polyak)
    if constexpr (gemm_threads<KSPLIT, MG, CORE>() == 1024) {   // the host attaches rides to 1024-thread configs
      const int rb = bid - n_tiles;
      if (rb >= (batch.ride.kind ? batch.ride.nblocks : 0)) {
        polyak_ride(batch.ride.pk, rb - (batch.ride.kind ? batch.ride.nblocks : 0), batch.ride.pk_blocks);
        return;
      }
      if (batch.ride.kind == 1) {
        mt_sample_body(batch.ride.mt, batch.ride.tbl_log2, reinterpret_cast<uint32_t*>(red));
      } else {
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
        for (int b = rb * 16 + wave; b < batch.ride.ga.B; b += batch.ride.nblocks * 16)
          gather_row(batch.ride.ga, b, lane, 64);
      }
    }
    return;
  }
  int p = 0;
#pragma unroll
  for (int q = 1; q < kMaxGemms; ++q)
    if (q < n_desc && bid >= tbeg[q]) p = q;
  // the fields the K loop needs, in the second (and last) round trip before the operand
  // loads; the epilogue's fields load lazily, under the MFMAs
  const GemmDesc d = batch.d[p];
#define SACMI_DESC_PIN_K "s"(d.A), "s"(d.B), "s"(d.M), "s"(d.N), "s"(d.K), "s"(d.lda), "s"(d.ldb), \
    "s"(d.a_kc), "s"(d.b_kc), "s"(d.tiles_n), "s"(d.tiles_m), "s"(d.xcd_gr), "s"(d.pl_div), \
    "s"(d.pl_mag), "s"(d.pl_gc_log2), "s"(d.pl_sr)
#if SACMI_PIN_EPI
  // ... and, in the same round trip (one asm statement: every load issued before the one
  // wait), the fields the epilogue's buffer descriptors and scalars are formed from — the
  // compiler forms them before the K loop, behind branches on the fields: two or three more
  // dependent round trips before the first operand load otherwise (ISA)
#define SACMI_DESC_PIN_E "s"(d.C), "s"(d.aux), "s"(d.ldc), "s"(d.ldaux), "s"(d.epi), "s"(d.bias), \
    "s"(d.bias_ld), "s"(d.dotw), "s"(d.dotp), "s"(d.rs_col), "s"(d.axk), "s"(d.ax_w), "s"(d.ax_out), \
    "s"(d.ax_ld), "s"(d.a_ksc)
  if constexpr (!PINS) {
  } else if constexpr (ADAM) {
    const AdamFuse& a = batch.adam;
    asm volatile("" :: SACMI_DESC_PIN_K, SACMI_DESC_PIN_E, "s"(a.P), "s"(a.M), "s"(a.V), "s"(a.T),
                 "s"(a.G), "s"(a.t_base), "s"(a.lr), "s"(a.beta1), "s"(a.beta2), "s"(a.eps),
                 "s"(a.tau), "s"(a.step_offset), "s"(a.sc), "s"(d.adam_step));
  } else if constexpr (AXK == 1) {
    const RowsFuse& r = batch.rows;
    asm volatile("" :: SACMI_DESC_PIN_K, SACMI_DESC_PIN_E, "s"(d.pa_w), "s"(d.pa_out), "s"(d.pa_ld),
                 "s"(d.pa_A), "s"(d.pa_base), "s"(r.part), "s"(r.logp), "s"(r.r), "s"(r.d),
                 "s"(r.kind), "s"(r.nparts), "s"(r.B), "s"(r.sc), "s"(r.logp_part), "s"(r.n_lp));
  } else {
    asm volatile("" :: SACMI_DESC_PIN_K, SACMI_DESC_PIN_E);
  }
#else
  if constexpr (PINS) asm volatile("" :: SACMI_DESC_PIN_K);
#endif
  if constexpr (CORE == 0) SACMI_PHASE(batch.tl, 8);   // (diagnostic: the desc has landed)
  const int t = bid - tbeg[p];
  if (t >= d.tiles_m * d.tiles_n) {   // padding to a multiple of 8 blocks
    if constexpr (MIDSPLIT) mid();
    return;
  }
  int tr, tc;
  place_tile(d, t, tr, tc);
  const int m0 = tr * TMW, n0 = tc * TN;
  if constexpr (CORE == 0) SACMI_PHASE(batch.tl, 9);   // (diagnostic: the tile is placed)
  if constexpr (ADAM) {
    // the level's scalar Adam work first, on wave 0 of block 0 (adam_block0_wave): the
    // other waves start their K loops, wave 0 follows ~3 us later, inside the tile's time
    if (adam_wg == -2 && bid == 0 && threadIdx.x < 64) {
      const AdamFuse& a = batch.adam;
      adam_block0_wave(a, (int)s_ld(s_rsrc(a.sc), (uint32_t)offsetof(DevScalars, err)), 1.f - a.beta1,
                       1.f - a.beta2);
    }
  }
  const bool rowsum = d.rs_col >= 0 && n0 == 0;
  const AdamFuse& af = batch.adam;
  // Adam bias corrections and the error bits: thread 0 reads them in pre(), behind its
  // wave's operand loads (at the kernel's start they put a device-memory round trip in
  // front of wave 0's operand loads), into LDS for the epilogue
  // Element slots: EPT tile outputs per thread (e = tid + s*NTH) plus one slot for the
  // rowsum (bias-gradient) column.  Their epilogue operands (bias, ReLU mask, Adam
  // state) are loaded by pre() while the MFMAs run.
  constexpr int NTH = gemm_threads<KSPLIT, MG, CORE>(), EPT = TMW * TN / NTH, NS = EPT + 1;
  static_assert(TMW * TN % NTH == 0 && TMW <= NTH, "epilogue slot layout");
  const int tid = threadIdx.x;
  // slot s -> (row, col in tile, output column n, valid); recomputed where needed so
  // that only the prefetched values stay live across the MFMA phase
  auto slot = [&](int s, int& row, int& col, int& n) -> bool {
    if (s < EPT) {
      const int e = tid + s * NTH;
      row = e / TN;
      col = e % TN;
      n = n0 + col;
      return m0 + row < d.M && n < d.N;
    }
    row = tid < TMW ? tid : 0;
    col = -1;
    n = d.rs_col;
    return rowsum && tid < TMW && m0 + row < d.M;
  };
  const bool wt = SACMI_WT && batch.st_wt;   // output store policy of this level
  const bool pol = d.epi == EPI_ADAM_POLYAK;
  // byte span of this desc's output (tile rows, plus the rowsum column; the fused-Adam
  // 4-column groups reach the row's padding up to a multiple of 4: ldc is one)
  const int ncov = ADAM ? (d.N + 3) & ~3 : d.N;
  const uint32_t span = (uint32_t)(((size_t)(d.M - 1) * d.ldc + (d.rs_col >= ncov ? d.rs_col + 1 : ncov)) * 4);
  const size_t abase = ADAM ? (size_t)(d.C - af.P) : 0;
  const rsrc_t rC = make_rsrc(d.C, span);
  // u rows (GemmDesc::u_out): a zero-length range where the desc stores none
  const rsrc_t rU = make_rsrc(d.u_out ? d.u_out : d.C,
                              d.u_out ? (uint32_t)(((size_t)(d.M - 1) * d.u_ld + d.N) * 4) : 0u);
  // (unused descriptors get a zero-length range: any access through them is dropped)
  const rsrc_t rM = make_rsrc(ADAM ? af.M + abase : d.C, ADAM ? span : 0);
  const rsrc_t rV = make_rsrc(ADAM ? af.V + abase : d.C, ADAM ? span : 0);
  const rsrc_t rT = make_rsrc(ADAM && pol ? af.T + abase - af.t_base : d.C, ADAM && pol ? span : 0);
  const rsrc_t rG = make_rsrc(ADAM && af.G ? af.G + abase : d.C, ADAM && af.G ? span : 0);
  const rsrc_t rX = d.bias ? make_rsrc(d.bias, (uint32_t)(((size_t)(d.N - 1) * d.bias_ld + 1) * 4))
                  : d.epi == EPI_MASK ? make_rsrc(d.aux, (uint32_t)(((size_t)(d.M - 1) * d.ldaux + d.N) * 4))
                  : make_rsrc(d.C, 0);
  // Adam: param, exp_avg, exp_avg_sq, target; otherwise x0 = the bias or the ReLU-mask
  // source (a level has one or the other: validate())
  // Fused-Adam levels work on 4-column groups instead of single elements: their optimizer
  // state moves as 16-byte loads and write-through stores — a write-through dword store
  // is one fabric write per lane, ~6x the 16-byte form per byte (MI355X_MICROARCH.md
  // "stores of each flavour"), and these levels store 12-16 bytes of state per parameter.
  // x0..x3 then hold only the rowsum (bias-gradient) slot.
  constexpr int NG = TMW * TN / 4;                         // 4-column groups of the tile
  constexpr int EPG = ADAM ? (NG + NTH - 1) / NTH : 1;     // groups per thread
  auto group = [&](int s, int& row, int& c4, int& n) -> bool {
    const int g = tid + s * NTH;
    row = g / (TN / 4);
    c4 = (g % (TN / 4)) * 4;
    n = n0 + c4;
    return g < NG && m0 + row < d.M && n < d.N;
  };
  float4 q0[EPG], q1[EPG], q2[EPG], q3[EPG];
  float x0[ADAM ? 1 : NS], x1[1], x2[1], x3[1];
  RowsRegs rows_x{};
  // the epilogue operands (Adam state, or the bias / mask) go out under the MFMAs; the
  // fc3 dot weights of the tile go to LDS; an axk-1 level runs its row prologue
  // the fc3 dot weight of this thread's tile column, loaded up front (buffer op with a
  // zero-length range where the level has none: no branch, so nothing waits for it early)
  // (loaded in pre(), after the operand burst; staged to LDS after the MFMAs)
  float dotw_x = 0.f, dotb_x = 0.f;
  // dL/da partials (GemmDesc::pa_out, axk-1 levels only): this tile's columns of the fc1
  // action weights, loaded under the MFMAs, staged [TN][32] in LDS after them
  constexpr int PW = PA ? (TN * 32 + NTH - 1) / NTH : 1;
  float paw_x[PW];
  const bool has_pa = PA && d.pa_out != nullptr;
  // CORE 1: the Adam scalars by scalar loads into every wave (lgkmcnt: no vector-memory round
  // trip in front of the slab DMAs, and no LDS store that would wait for them)
  uint32_t skw[5] = {0u, 0u, 0u, 0u, 0u};
  // folded heads (HF): a policy tile forms its columns' share of the heads (a split-K
  // partial), so its head-weight columns come in with the epilogue operands
  const bool hf_mine = HF && batch.heads_ticket != nullptr && p >= batch.heads_desc &&
                       p < batch.heads_desc + batch.heads_ndesc;
  constexpr int HWPT = HF ? (48 * TN + NTH - 1) / NTH : 1;   // (2A <= 48)
  float hw_x[HWPT];
  auto pre = [&]() {
    if constexpr (ADAM && CORE == 1) {
      const sbuf_i4 r = s_rsrc(af.sc);
      const uint32_t o = (uint32_t)(offsetof(DevScalars, beta_pow) + d.adam_step * 16);
#pragma unroll
      for (int q = 0; q < 4; ++q) skw[q] = s_ld(r, o + 4u * q);
      skw[4] = s_ld(r, (uint32_t)offsetof(DevScalars, err));
    } else if constexpr (ADAM) {
      if (threadIdx.x == 0) {
        s_k = fuse_scalars(af, d.adam_step, af.step_offset);
        s_err = af.sc->err;
      }
    }
    if constexpr (HF) {   // zero-length range where this tile folds nothing
      const HeadSampleArgs& ha = batch.heads;
      const int n2 = 2 * ha.A;
      const rsrc_t rHW = make_rsrc(hf_mine ? ha.Wh : d.C,
                                   hf_mine ? (uint32_t)(((size_t)(n2 - 1) * ha.ldw + ha.K) * 4) : 0u);
#pragma unroll
      for (int q = 0; q < HWPT; ++q) {
        const int e = tid + q * NTH, j = e / TN, cc = e - j * TN;
        hw_x[q] = buf_ld(rHW, e < n2 * TN && n0 + cc < ha.K ? (uint32_t)(j * ha.ldw + n0 + cc) * 4u : 0xfffffff0u);
      }
    }
    // axk 1: the row prologue's loads.  Issued here, behind the operand burst, and
    // consumed after the MFMAs: anything in flight at the k-loop header is waited for by
    // the back-edge's conservative vmcnt on the first iteration.
    if constexpr (AXK == 1) rows_load<TMW, NTH, LDAUX>(batch.rows, d, m0, rows_x);   // unconditional
    if constexpr (PA) {   // zero-length range where the level has no partials
      const rsrc_t rPW = make_rsrc(has_pa ? d.pa_w : d.C,
                                   has_pa ? (uint32_t)(((size_t)(d.N - 1) * d.pa_ld + d.pa_A) * 4) : 0u);
#pragma unroll
      for (int q = 0; q < PW; ++q) {
        const int e = tid + q * NTH, c = e / 32, j = e % 32;
        const bool okw = e < TN * 32 && j < d.pa_A && n0 + c < d.N;
        paw_x[q] = buf_ld(rPW, okw ? (uint32_t)((n0 + c) * d.pa_ld + j) * 4u : 0xfffffff0u);
      }
    }
    {   // buffer ops with a zero-length range where the level has no dots: no branch
      const rsrc_t rDW = make_rsrc(d.dotp ? d.dotw : d.C, d.dotp ? (uint32_t)(d.N + 1) * 4u : 0u);
      const int nn = n0 + (tid < TN ? tid : 0);
      dotw_x = buf_ld(rDW, (uint32_t)(nn < d.N ? nn : 0) * 4u);
      dotb_x = buf_ld(rDW, (uint32_t)d.N * 4u);   // the head's bias w3~[N]
    }
    // unconditional: an empty slot reads past its descriptor's range (returns 0, no
    // access), and the level's unused operands have zero-length descriptors
    constexpr uint32_t kOob = 0xfffffff0u;
    if constexpr (ADAM) {
#pragma unroll
      for (int s = 0; s < EPG; ++s) {
        int row, c4, n;
        const bool ok = group(s, row, c4, n);
        const uint32_t o = ok ? (uint32_t)((m0 + row) * d.ldc + n) * 4u : kOob;
#ifdef SACMI_EXP_NOADAMIO
        // timing experiment only: no optimizer-state traffic
        q0[s] = q1[s] = q2[s] = q3[s] = float4{0.f, 0.f, 0.f, (float)o};
#else
        q0[s] = buf_ld4(rC, o); q1[s] = buf_ld4(rM, o); q2[s] = buf_ld4(rV, o);
        q3[s] = buf_ld4(rT, o);
#endif
      }
      int row, col, n;
      const bool ok = slot(EPT, row, col, n);      // the rowsum slot
      const uint32_t o = ok ? (uint32_t)((m0 + row) * d.ldc + n) * 4u : kOob;
      x0[0] = buf_ld(rC, o); x1[0] = buf_ld(rM, o); x2[0] = buf_ld(rV, o);
      x3[0] = buf_ld(rT, o);
    }
#pragma unroll
    for (int s = 0; s < (ADAM ? 0 : NS); ++s) {
      int row, col, n;
      const bool ok = slot(s, row, col, n);
      {
        const uint32_t o = !ok ? kOob
                         : d.bias ? (uint32_t)(n * d.bias_ld) * 4u
                                  : (uint32_t)((m0 + row) * d.ldaux + n) * 4u;
        x0[s] = buf_ld_aux<LDAUX>(rX, o);
      }
    }
  };
  // the plain (no Adam, no A transform) one-chunk-per-stage configurations pipeline their
  // K loop (register budget: the Adam and transform variants already sit near 128 VGPRs)
  constexpr int PIPE = (SACMI_PIPE && G == 1 && !ADAM && AXK == 0) ? 1
                     : (SACMI_PIPE_DW && G == 1 && ADAM && MG == 2) ? 2 : 0;
  SACMI_PHASE(batch.tl, 1);
  if constexpr (CORE == 1)
    gemm_core_stg<TM, TN, KSPLIT, MG, AXK>(d, m0, n0, ring, rsum, s_kw, rowsum, pre, batch.tl);
  else
    gemm_core<TM, TN, KSPLIT, G, MG, AXK, BF16, PIPE, LDAUX, MIDSPLIT>(d, m0, n0, red, rsum, rowsum, pre, mid);
  SACMI_PHASE(batch.tl, 2);
  SACMI_PHASE_LAST(batch.tl, 7);
  if (d.dotp && tid < TN) s_dotw[tid] = n0 + tid < d.N ? dotw_x : 0.f;
  if constexpr (PA) {
    if (has_pa) {
#pragma unroll
      for (int q = 0; q < PW; ++q) {
        const int e = tid + q * NTH;
        if (e < TN * 32) s_pa[TMW * (TN + 1) + e] = paw_x[q];
      }
    }
  }
  if constexpr (AXK == 1) {
    // the row prologue, after the MFMAs: its loads went out first and have long landed
    if (d.axk == 1)
      rows_finish<TMW, NTH>(batch.rows, d, m0, p == 0 && n0 == 0, bid == 0, rows_x,
                            s_q, s_coef, s_l);
  }
  __syncthreads();
  if (threadIdx.x < 64) SACMI_STAMP(32);
  SACMI_PHASE(batch.tl, 3);
  const float omb1 = 1.f - af.beta1, omb2 = 1.f - af.beta2, omtau = 1.f - af.tau;
  // a non-finite policy sample / PER draw of this update (ErrBits): the reference raised
  // before this step (no stores), or after the critic step but before Polyak
  int err = ADAM ? s_err : 0;
  AdamScalars k_ad = s_k;
  if constexpr (ADAM && CORE == 1) {
    double p1 = __longlong_as_double((long long)((uint64_t)skw[0] | ((uint64_t)skw[1] << 32)));
    double p2 = __longlong_as_double((long long)((uint64_t)skw[2] | ((uint64_t)skw[3] << 32)));
    if (af.step_offset) { p1 *= (double)af.beta1; p2 *= (double)af.beta2; }
    k_ad = AdamScalars{(float)((double)af.lr / (1.0 - p1)), (float)sqrt(1.0 - p2)};
    err = (int)skw[4];
  }
  const bool void_st = ADAM && (err & af.err_skip) != 0;
  const bool pol_st = pol && (err & af.err_nopolyak) == 0;
  if constexpr (ADAM) {
    // 4-column groups: the gradient of a column past N (a row pad) is taken as 0, so the
    // Adam / Polyak arithmetic leaves the pad (0) exactly 0 and the 16-byte stores rewrite it
#pragma unroll
    for (int s = 0; s < EPG; ++s) {
      int row, c4, n;
      if (!group(s, row, c4, n) || void_st) continue;
      float g[4], p[4] = {q0[s].x, q0[s].y, q0[s].z, q0[s].w}, m[4] = {q1[s].x, q1[s].y, q1[s].z, q1[s].w},
            v[4] = {q2[s].x, q2[s].y, q2[s].z, q2[s].w}, t[4] = {q3[s].x, q3[s].y, q3[s].z, q3[s].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        g[j] = n + j < d.N ? reduce_partials<TM, TN, KSPLIT, MG>(red, row, c4 + j) : 0.f;
        adam_elem(p[j], m[j], v[j], g[j], omb1, af.beta2, omb2, af.eps, k_ad);
        t[j] = polyak(t[j], p[j], omtau, af.tau);
      }
      const uint32_t o = (uint32_t)((m0 + row) * d.ldc + n) * 4u;
      auto st4 = [&](rsrc_t r, const float (&x)[4]) {
        if (wt) buf_st4<kStAux>(r, o, f4{x[0], x[1], x[2], x[3]});
        else buf_st4<0>(r, o, f4{x[0], x[1], x[2], x[3]});
      };
      auto st_bf4 = [&](unsigned short* h, const float (&x)[4]) {   // 4 bf16 shadows, 8 bytes
        const uint32_t lo = (uint32_t)bf16_bits(x[0]) | ((uint32_t)bf16_bits(x[1]) << 16);
        const uint32_t hi = (uint32_t)bf16_bits(x[2]) | ((uint32_t)bf16_bits(x[3]) << 16);
        if (wt) st_wt8(h, 0u, lo, hi);
        else *reinterpret_cast<uint2*>(h) = make_uint2(lo, hi);
      };
#ifdef SACMI_EXP_NOADAMIO
      if (p[0] + m[1] + v[2] + t[3] == 12345.f) st4(rC, p);   // (keeps the math alive)
      continue;
#endif
      if (af.G) st4(rG, g);
      st4(rC, p); st4(rM, m); st4(rV, v);
      if (af.Ph) st_bf4(af.Ph + abase + (o >> 2), p);
      if (pol_st) {
        st4(rT, t);
        if (af.Th) st_bf4(af.Th + abase - af.t_base + (o >> 2), t);
      }
    }
  }
#pragma unroll
  for (int s = ADAM ? EPT : 0; s < NS; ++s) {
    int row, col, n;
    const bool ok = slot(s, row, col, n) && !void_st;
    float v = 0.f;
    if (ok) {
      if (s < EPT) {
        v = reduce_partials<TM, TN, KSPLIT, MG>(red, row, col);
      } else {
        const float* rb = rsum + (row / TM) * KSPLIT * TM + row % TM;
        v = rb[0];
#pragma unroll
        for (int w = 1; w < KSPLIT; ++w) v += rb[w * TM];
      }
      const uint32_t o = (uint32_t)((m0 + row) * d.ldc + n) * 4u;
      if constexpr (AXK == 1) {
        if (d.axk == 1) v *= s_coef[d.ax_slot][row];   // dh = coef[b] * (u W2)
      }
      if constexpr (ADAM) {   // (the rowsum slot)
        adam_elem(x0[0], x1[0], x2[0], v, omb1, af.beta2, omb2, af.eps, k_ad);
        if (af.G) buf_st_pol(rG, o, v, wt);
        buf_st_pol(rC, o, x0[0], wt); buf_st_pol(rM, o, x1[0], wt); buf_st_pol(rV, o, x2[0], wt);
        if (af.Ph) st_pol(af.Ph + abase + (o >> 2), bf16_bits(x0[0]), wt);
        if (pol_st) {
          const float tn = polyak(x3[0], x0[0], omtau, af.tau);
          buf_st_pol(rT, o, tn, wt);
          if (af.Th) st_pol(af.Th + abase - af.t_base + (o >> 2), bf16_bits(tn), wt);
        }
      } else {
        if (d.bias) v += x0[s];
        if (d.epi == EPI_RELU) v = v <= 0.f ? 0.f : v;   // F.relu: NaN stays NaN
        else if (d.epi == EPI_MASK) v = x0[s] > 0.f ? v : 0.f;
#ifdef SACMI_EXP_NOSTORE
        if (v == 12345.f)   // timing experiment only: no output stores
#endif
        buf_st_pol(rC, o, v, wt);
        if (d.u_out && s < EPT)   // u rows (u_out)
          buf_st_pol(rU, (uint32_t)((m0 + row) * d.u_ld + n) * 4u, v > 0.f ? s_dotw[col] : 0.f, wt);
      }
    }
    if constexpr (!ADAM) {
      // fc3 dot partial of this row over its 32-column block: the 32 lanes of a half
      // wave hold one row's 32 consecutive columns (TN = 32 or 64, row-major slots)
      if (s < EPT && d.dotp) {
        float c = ok ? v * s_dotw[col] : 0.f;
        c = row16_sum(c);                 // DPP within each 16-lane row
        c += __shfl_xor(c, 16, 64);       // the two rows of the half wave
        if ((tid & 31) == 0 && m0 + row < d.M)   // block 0 adds the bias: q = sum of blocks
          st_pol(d.dotp + (size_t)(m0 + row) * d.dotp_ld + (n0 + col) / 32, n0 + col == 0 ? c + dotb_x : c, wt);
      }
    }
    if constexpr (PA) {   // every tile element, 0 outside the output
      if (has_pa && s < EPT) s_pa[row * (TN + 1) + col] = ok ? v : 0.f;
    }
    if constexpr (HF) {   // (the stored h: after the ReLU)
      if (hf_mine && s < EPT) s_hlp[row * (TN + 1) + col] = ok ? v : 0.f;
    }
  }
  if (threadIdx.x < 64) SACMI_STAMP(33);
  SACMI_PHASE(batch.tl, 4);
  if constexpr (AXK == 1) {
    if (d.axk == 1) rows_loss<TMW>(batch.rows, m0, p == 0 && n0 == 0, s_l);
  }
  if constexpr (PA) {
    if (has_pa) {
      // dL/da partial of every row over each 32-column block of this tile:
      // pa_out[((pa_base + (n0 + 32 sb) / 32) * M + row) * A + j] = sum_c C[row][c] w[c][j]
      // (outside the tile's rows / columns the stored value is the masked 0 or never read)
      const float* s_t = s_pa;
      const float* s_w = s_pa + TMW * (TN + 1);
      __syncthreads();
      const int A = d.pa_A;
      constexpr int NSB = TN / 32;
      for (int e = tid; e < TMW * NSB * A; e += NTH) {
        const int row = e / (NSB * A), rem = e - row * (NSB * A), sb = rem / A, j = rem - sb * A;
        const float* tr = s_t + row * (TN + 1) + sb * 32;
        const float* wc = s_w + sb * 32 * 32 + j;
        float acc = 0.f;
#pragma unroll 8
        for (int c = 0; c < 32; ++c) acc = fmaf(tr[c], wc[c * 32], acc);
        if (m0 + row < d.M)
          st_wt(d.pa_out + ((size_t)(d.pa_base + n0 / 32 + sb) * d.M + m0 + row) * A + j, acc);
      }
    }
  }
  if (batch.has_adam && adam_wg == -1 && bid == 0) {
    adam_block0(af, err, omb1, omb2);
  }
  store_err_flags(batch);
  if constexpr (HF) {
    // folded heads, split over the level's column tiles: each policy tile forms its TN
    // columns' share of every head output of its 32 rows (fixed column order) into
    // heads_part[row block][column tile] (write-through), acknowledged in every wave, then
    // the row block's arrival count; the last column tile to arrive sums the shares in column-
    // tile order (sc1 loads: stored from other XCDs), adds the bias and runs the sample
    // epilogue (heads_elem: k_heads_sample's per-element algebra) and the log-prob sums.
    // (the policy rows may come as heads_ndesc descs of d.M rows each, stacked in order: the
    // target and actor halves of k_chain_a's row-affine L2)
    if (hf_mine) {
      const HeadSampleArgs& ha = batch.heads;
      const int A = ha.A, n2 = 2 * A;
      const int hm0 = m0 + (p - batch.heads_desc) * d.M;   // the row in the heads' stacked rows
      const int rb = hm0 / kHeadsFoldTM, tcol = n0 / TN, ntc = d.tiles_n;
      static_assert(TMW == kHeadsFoldTM, "one 32-row block per folding tile");
      __syncthreads();                                     // s_hlp complete; red free
      float* s_w = red;                                    // [n2][TN + 1]
#pragma unroll
      for (int q = 0; q < HWPT; ++q) {
        const int e = tid + q * NTH;
        if (e < n2 * TN) s_w[(e / TN) * (TN + 1) + e % TN] = hw_x[q];
      }
      __syncthreads();
      float* part = batch.heads_part + ((size_t)rb * ntc + tcol) * (kHeadsFoldTM * n2);
      for (int e = tid; e < kHeadsFoldTM * n2; e += NTH) {
        const int row = e / n2, j = e - row * n2;
        const float* hr = s_hlp + row * (TN + 1);
        const float* wr = s_w + j * (TN + 1);
        float acc = 0.f;
#pragma unroll 16
        for (int cc = 0; cc < TN; ++cc) acc = fmaf(hr[cc], wr[cc], acc);
        st_wt(part + e, acc);
      }
      // the finishing tile's bias and noise, loaded by every folding tile before its arrival
      const int e = tid, row = e / A, j = e - (e / A) * A, m = hm0 + row;
      const bool live = e < kHeadsFoldTM * A && m < ha.rows;
      float bm = 0.f, bl = 0.f, eps_in = 0.f;
      {
        const int jj = live ? j : 0, mm = live ? m : 0;
        const rsrc_t rB = make_rsrc(ha.Wh, (uint32_t)(((size_t)(n2 - 1) * ha.ldw + ha.K + 1) * 4));
        bm = buf_ld(rB, (uint32_t)((size_t)jj * ha.ldw + ha.K) * 4u);
        bl = buf_ld(rB, (uint32_t)((size_t)(A + jj) * ha.ldw + ha.K) * 4u);
        const bool want = !ha.deterministic && !ha.gen_eps;
        eps_in = buf_ld(make_rsrc(want ? ha.eps : ha.Wh, want ? 0x7fffffffu : 0u), (uint32_t)((size_t)mm * A + jj) * 4u);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        int* tk = batch.heads_ticket + rb;
        const int old = __hip_atomic_fetch_add(tk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_hlast = old == ntc - 1;
        if (old == ntc - 1) __hip_atomic_store(tk, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      if (s_hlast) {
        float (*lp)[33] = reinterpret_cast<float (*)[33]>(red);
        float* s_lp = red + kHeadsFoldTM * 33;
        const uint64_t ctr = ha.ctr_override ? ha.ctr_override : ha.sc->noise_counter;
        if (e < kHeadsFoldTM * A) {
          float lpe = 0.f;
          if (live) {
            // (a buffer descriptor on the row block's base — uniform: a per-lane base would
            // make the compiler loop over the distinct values — and the row in the offset)
            const float* p0 = batch.heads_part + (size_t)rb * ntc * (kHeadsFoldTM * n2);
            const rsrc_t rP = make_rsrc(p0, (uint32_t)((size_t)ntc * kHeadsFoldTM * n2 * 4));
            float sm[16], sl[16];   // (ntc <= 16: H <= 1024)
#pragma unroll
            for (int t = 0; t < 16; ++t) {
              const uint32_t o = (uint32_t)((size_t)t * kHeadsFoldTM * n2 + row * n2) * 4u;
              sm[t] = buf_ld_aux<kLdSc1>(rP, t < ntc ? o + (uint32_t)j * 4u : 0xfffffff0u);
              sl[t] = buf_ld_aux<kLdSc1>(rP, t < ntc ? o + (uint32_t)(A + j) * 4u : 0xfffffff0u);
            }
            float mean = sm[0], ls_raw = sl[0];
#pragma unroll
            for (int t = 1; t < 16; ++t)
              if (t < ntc) { mean += sm[t]; ls_raw += sl[t]; }
            lpe = heads_elem<false, kLdSc1>(ha, m, j, mean + bm, ls_raw + bl, eps_in, ctr);
          }
          lp[row][j] = lpe;
        }
        heads_logp<kHeadsFoldTM, kLdSc1>(ha, hm0, rb, lp, s_lp);
      }
    }
  }
  SACMI_PHASE(batch.tl, 5);
}

template <int TM, int TN, int KSPLIT, int G, int MG, bool ADAM, int AXK = 0, bool BF16 = false, int CORE = 0,
          bool HFOLD = false>
__global__ __launch_bounds__((gemm_threads<KSPLIT, MG, CORE>()), (gemm_min_waves<KSPLIT * MG>())) void k_gemm(GemmBatch batch) {
  const TlMark tl_mark(batch.tl, TL_GEMM);
  __shared__ KgSmem<TM, TN, KSPLIT, G, MG, ADAM, AXK, BF16, CORE, HFOLD> sm;
  kg_body<TM, TN, KSPLIT, G, MG, ADAM, AXK, BF16, CORE, 0, false, HFOLD>(batch, blockIdx.x, sm);
}

// Tile order and XCD placement.  Workgroups are dealt round-robin over the 8 XCDs
// (block b -> XCD b % 8: observed dispatch behaviour, used for speed only), and each
// XCD has its own L2.  Row-major tile order puts the 8 column tiles of a row block on
// 8 different XCDs, so every XCD fetches every A row block: traffic past L2 ~ 8A + B.
// Each desc starts on a multiple of 8 blocks and, where its tile grid divides, XCD x
// gets a compact (tm/gr) x (tn/gc) sub-grid of tiles (gr*gc = 8): traffic gc*A + gr*B,
// gr chosen per desc to minimise it.
template <int TM, int TN>
static int assign_tiles(GemmBatch& b) {
  int tot = 0;
  for (int i = 0; i < b.count; ++i) {
    GemmDesc& d = b.d[i];
    d.tiles_n = (d.N + TN - 1) / TN;
    d.tiles_m = (d.M + TM - 1) / TM;
    d.tile_begin = tot;
    const double A = (double)d.M * d.K, B = (double)d.N * d.K;
    d.xcd_gr = 0;
    double best = 8 * A + B;      // row-major order
    // SACMI_XCD_GR (experiment): force the XCD grid (1: every XCD owns column tiles only)
    static const int force_gr = std::getenv("SACMI_XCD_GR") ? std::atoi(std::getenv("SACMI_XCD_GR")) : 0;
    if (force_gr > 0 && d.tiles_m % force_gr == 0 && d.tiles_n % (8 / force_gr) == 0) {
      d.xcd_gr = force_gr;
      tot += (d.tiles_m * d.tiles_n + 7) & ~7;
      continue;
    }
    for (int gr : {1, 2, 4, 8}) {
      const int gc = 8 / gr;
      if (d.tiles_m % gr || d.tiles_n % gc) continue;
      const double cost = gc * A + gr * B;
      if (cost < best) { best = cost; d.xcd_gr = gr; }
    }
    tot += (d.tiles_m * d.tiles_n + 7) & ~7;
  }
  for (int i = 0; i < b.count; ++i) {   // the placement divisor of every desc
    GemmDesc& d = b.d[i];
    const int gc = d.xcd_gr ? 8 / d.xcd_gr : 1;
    d.pl_div = d.xcd_gr ? d.tiles_n / gc : d.tiles_n;
    d.pl_gc_log2 = gc == 8 ? 3 : gc == 4 ? 2 : gc == 2 ? 1 : 0;
    d.pl_sr = d.xcd_gr ? d.tiles_m / d.xcd_gr : 0;
    // ceil(2^32 / div): mul_hi(n, mag) = n / div exactly for n, div < 2^16
    if (d.pl_div < 1 || d.pl_div >= 65536 || d.tiles_m * d.tiles_n >= 65536)
      throw Error{SACMI_ESTATE, "tile grid out of the placement range"};
    d.pl_mag = d.pl_div == 1 ? 0u : (unsigned)((((uint64_t)1 << 32) + d.pl_div - 1) / d.pl_div);
  }
  b.total_tiles = tot;
  return tot;
}

// ---------------------------------------------------------------------------
// Large-M forward levels (batch-4096 class) in bf16 mode: LDS-staged 128x128 tiles.
// C = relu(A . W^T [+ b]) with both operands K-contiguous (activations [rows][K],
// nn.Linear weights [out][K]); [+ per-32-column fc3 dot partials].  Four waves (2x2),
// each a 64x64 sub-tile over the FULL K (no K split, no partial-tile reduction): the
// workgroup stages a 32-deep K slab of its 128 A rows and 128 W rows through LDS (double
// buffered: the next slab's global loads are in flight while this slab's MFMAs run) and
// every wave reads its fragments from LDS — each operand byte crosses L2->CU once per
// workgroup instead of once per wave.  Two workgroups per CU.
constexpr int kFBM = 128, kFBK = 32, kFPad = 4, kFBN128 = 128;
#ifndef SACMI_FWD_LDS16
#define SACMI_FWD_LDS16 1       // bf16 mode: k_fwd16 (bf16 LDS slabs, 16x16x32 MFMA)
#endif

__device__ __forceinline__ float swap_adj(float x) {   // lane ^ 1's x (DPP quad_perm 1,0,3,2)
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)bf16_bits(lo) | ((uint32_t)bf16_bits(hi) << 16);
}

// k_fwd / k_fwd16 epilogue: bias, ReLU, store, per-32-column fc3 dot partials.  A wave
// owns a 64 x (16 NT) sub-tile at (r0, c0); lane holds D[row = (lane >> 4) * 4 + r]
// [col = lane & 15] of each 16x16 tile.  The operands are loaded before the K loop.
template <int NT, int MI = 4>
struct FwdEpi {
  float bias_x[NT], dotw_x[NT], dotb;
  __device__ __forceinline__ void load(const GemmDesc& d, int c0, int lane) {
    const int N = d.N;
    const bool has_bias = d.bias != nullptr, has_dot = d.dotp != nullptr;
    const rsrc_t rX = make_rsrc(has_bias ? d.bias : d.C, has_bias ? 0x7fffffffu : 0u);
    const rsrc_t rW = make_rsrc(has_dot ? d.dotw : d.C, has_dot ? (uint32_t)(N + 1) * 4u : 0u);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = c0 + j * 16 + (lane & 15);
      const int cc = col < N ? col : 0;
      bias_x[j] = buf_ld(rX, (uint32_t)(cc * d.bias_ld) * 4u);
      dotw_x[j] = col < N ? buf_ld(rW, (uint32_t)cc * 4u) : 0.f;
    }
    dotb = buf_ld(rW, (uint32_t)N * 4u);
  }
  // C16 (act16): C is bf16 — the fp32 values (the dot partials use them unrounded) are
  // rounded once, and adjacent lanes swap one value (DPP) so every lane stores a column
  // pair of one row as a 32-bit word: lane 2c row r4+rp, lane 2c+1 row r4+rp+1
  // tile (C16 only): the column-pair words go to an LDS tile image at (row - tm0, col - tn0),
  // tld words per row, instead of global memory (k_fwd16p's staged epilogue)
  template <bool C16 = false>
  __device__ __forceinline__ void store(const GemmDesc& d, f4 (&acc)[MI][NT], int r0, int c0,
                                        int lane, uint32_t* tile = nullptr, int tm0 = 0,
                                        int tn0 = 0, int tld = 0) const {
    const int M = d.M, N = d.N;
    const bool has_bias = d.bias != nullptr, has_dot = d.dotp != nullptr;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + i * 16 + (lane >> 4) * 4 + r;
        float dsum[NT / 2 > 0 ? NT / 2 : 1] = {};
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int col = c0 + j * 16 + (lane & 15);
          float v = acc[i][j][r];
          if (has_bias) v += bias_x[j];
          if (d.epi == EPI_RELU) v = v <= 0.f ? 0.f : v;   // F.relu: NaN stays NaN
          if constexpr (C16) acc[i][j][r] = v;
          else if (row < M && col < N) st_big(d.C + (size_t)row * d.ldc + col, v);
          if (has_dot) {
            // fc3 dot partial over the 32-column block (tiles j, j+1): 16 lanes per tile,
            // summed by DPP row rotations (VALU; the ds_bpermute butterfly it replaces
            // put 256 LDS-crossbar ops per lane in this epilogue)
            float c = (row < M && col < N) ? v * dotw_x[j] : 0.f;
            c = row16_sum(c);
            dsum[j >> 1] += c;
          }
        }
        if (has_dot && (lane & 15) == 0 && row < M) {
#pragma unroll
          for (int h = 0; h < NT / 2; ++h) {
            const int blk = c0 / 32 + h;
            if (blk * 32 < N)
              d.dotp[(size_t)row * d.dotp_ld + blk] = blk == 0 ? dsum[h] + dotb : dsum[h];
          }
        }
      }
    }
    if constexpr (C16) {
      unsigned short* C = reinterpret_cast<unsigned short*>(d.C);
      const bool odd = lane & 1;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int rp = 0; rp < 4; rp += 2) {
            const float a0 = acc[i][j][rp], a1 = acc[i][j][rp + 1];
            const float b0 = swap_adj(a0), b1 = swap_adj(a1);
            const int row = r0 + i * 16 + (lane >> 4) * 4 + rp + (odd ? 1 : 0);
            const int col = c0 + j * 16 + (lane & 14);
            const uint32_t w = odd ? pack_bf16x2(b1, a1) : pack_bf16x2(a0, b0);
            if (tile) tile[(row - tm0) * tld + ((col - tn0) >> 1)] = w;
            else if (row < M && col < N) st_big(reinterpret_cast<uint32_t*>(C + (size_t)row * d.ldc + col), w);
          }
    }
  }
};


template <bool BF16, int kFBN = 128>
__global__ __launch_bounds__(256, 2) void k_fwd(GemmBatch batch) {
  const TlMark tl_mark(batch.tl, TL_FWD);
  constexpr int NT = kFBN / 32;          // 16-column MFMA tiles per wave (2 x 2 waves)
  __shared__ __attribute__((aligned(16))) float sA[2][kFBM][kFBK + kFPad];
  __shared__ __attribute__((aligned(16))) float sB[2][kFBN][kFBK + kFPad];
  const int bid = blockIdx.x;
  int p = 0;
  for (int q = 1; q < batch.count; ++q)
    if (bid >= batch.d[q].tile_begin) p = q;
  const GemmDesc& d = batch.d[p];
  const int t = bid - d.tile_begin;
  if (t >= d.tiles_m * d.tiles_n) return;
  int tr, tc;
  place_tile(d, t, tr, tc);
  const int m0 = tr * kFBM, n0 = tc * kFBN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * (kFBN / 2);
  const int M = d.M, N = d.N, K = d.K;
  constexpr int NB = kFBN / 32;          // B rows staged per thread (32 rows per pass)
  // staging: thread t moves rows (t >> 3) + 32 i (i < 4) at k = 4 (t & 7) of both slabs
  const rsrc_t rA = make_rsrc(d.A, 0x7fffffffu), rB = make_rsrc(d.B, 0x7fffffffu);
  uint32_t offA[4], offB[NB];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int ra = min(m0 + (tid >> 3) + 32 * i, M - 1);
    offA[i] = (uint32_t)ra * (uint32_t)d.lda * 4u;
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int rb = min(n0 + (tid >> 3) + 32 * i, N - 1);
    offB[i] = (uint32_t)rb * (uint32_t)d.ldb * 4u;
  }
  const int kq = 4 * (tid & 7);
  float4 ga[4], gb[NB];
  auto zk = [&](float4 x, int k) {    // elements past K read the row's next columns: zeroed
    x.x = k < K ? x.x : 0.f; x.y = k + 1 < K ? x.y : 0.f; x.z = k + 2 < K ? x.z : 0.f; x.w = k + 3 < K ? x.w : 0.f;
    return x;
  };
  auto gload = [&](int k0) {
    const int k = k0 + kq;
    const uint32_t ko = (uint32_t)(k < K ? k : 0) * 4u;
#pragma unroll
    for (int i = 0; i < 4; ++i) ga[i] = zk(buf_ld4(rA, offA[i] + ko), k);
#pragma unroll
    for (int i = 0; i < NB; ++i) gb[i] = zk(buf_ld4(rB, offB[i] + ko), k);
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<float4*>(&sA[buf][(tid >> 3) + 32 * i][kq]) = ga[i];
#pragma unroll
    for (int i = 0; i < NB; ++i) *reinterpret_cast<float4*>(&sB[buf][(tid >> 3) + 32 * i][kq]) = gb[i];
  };
  f4 acc[4][NT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  // epilogue operands (bias, dot weights) issued up front: they land under the K loop
  FwdEpi<NT> ep;
  ep.load(d, n0 + wn, lane);
  gload(0);
  swrite(0);
  __syncthreads();
  const int nslab = (K + kFBK - 1) / kFBK;
  for (int sl = 0; sl < nslab; ++sl) {
    const int cur = sl & 1;
    gload((sl + 1 < nslab ? sl + 1 : sl) * kFBK);   // unconditional: the last re-reads its slab
#pragma unroll
    for (int kk = 0; kk < kFBK / 16; ++kk) {
      float a[4][4], b[NT][4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float4 x = *reinterpret_cast<const float4*>(&sA[cur][wm + i * 16 + (lane & 15)][kk * 16 + 4 * (lane >> 4)]);
        a[i][0] = x.x; a[i][1] = x.y; a[i][2] = x.z; a[i][3] = x.w;
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const float4 y = *reinterpret_cast<const float4*>(&sB[cur][wn + j * 16 + (lane & 15)][kk * 16 + 4 * (lane >> 4)]);
        b[j][0] = y.x; b[j][1] = y.y; b[j][2] = y.z; b[j][3] = y.w;
      }
      mfma_chunk<4, NT, BF16>(acc, a, b);
    }
    swrite(cur ^ 1);
    __syncthreads();
  }
  ep.store(d, acc, m0 + wm, n0 + wn, lane);
}

// bf16 mode, bf16 in LDS: the staging rounds every fp32 operand ONCE per workgroup
// (v_cvt_pk_bf16_f32) and stores [row][k] bf16 slabs 64 deep; a lane's 8 consecutive k
// of one row are one ds_read_b128 and exactly its v_mfma_f32_16x16x32_bf16 operand
// (lane l: A[l&15][8(l>>4) + j], B[8(l>>4) + j][l&15]).  Against k_fwd<true>: half the
// LDS bytes per MFMA, one conversion per element per workgroup instead of per wave, half
// the MFMA issues, and half the barriers / load round trips per K.  Same tiles, XCD
// order and epilogue as k_fwd.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u2v __attribute__((ext_vector_type(2)));
#ifndef SACMI_FWD16_BK
#define SACMI_FWD16_BK 64       // k_fwd16 slab depth (64 or 32)
#endif
#ifndef SACMI_FWD16_OCC
#define SACMI_FWD16_OCC 2       // k_fwd16 workgroups per CU the launch bounds ask for
#endif
constexpr int kHBK = SACMI_FWD16_BK, kHPad = 8;

__device__ __forceinline__ u2v pack_bf16x4(float4 v) {
  const bf16x4 x = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
  return __builtin_bit_cast(u2v, x);
}

// AH (act16): A is bf16 (4 k per 8-byte load, straight into the slab) and C is bf16.
// Waves: 2 x fwd16_wc<kFBN>() of 64 x (kFBN / wc) sub-tiles
// 8 waves (4 per SIMD at two workgroups per CU) hide each other's LDS / barrier latency
// behind MFMAs: config 5 L1 / L2 28.8 / 25.4 -> 24.8 / 21.1 us, the 64-column levels
// L3 / L4 / L7 / L8 18.9 / 16.9 -> 16.4 / 14.7 (4 waves: one wave per SIMD per workgroup)
#ifndef SACMI_FWD16_WAVES
#define SACMI_FWD16_WAVES 8     // waves per k_fwd16 workgroup at 128-column tiles (4 or 8)
#endif
#ifndef SACMI_FWD16_WAVES64
#define SACMI_FWD16_WAVES64 8   // ... at 64-column tiles (4: 2 x 2 waves of 64x32; 8: 4 x 2 of 32x32)
#endif
template <int kFBN>
__host__ __device__ constexpr int fwd16_waves() { return kFBN == 128 ? SACMI_FWD16_WAVES : SACMI_FWD16_WAVES64; }
template <int kFBN, bool BH = false, bool AH = false>
__global__ __launch_bounds__(64 * fwd16_waves<kFBN>(), SACMI_FWD16_OCC) void k_fwd16(GemmBatch batch) {
  const TlMark tl_mark(batch.tl, TL_FWD16);
  // NWV waves as WR x WC, each an MW x NW sub-tile: MI x NT 16x16 MFMA tiles
  constexpr int NWV = fwd16_waves<kFBN>(), WC = kFBN == 128 ? NWV / 2 : 2, WR = NWV / WC;
  constexpr int MW = kFBM / WR, MI = MW / 16, NW = kFBN / WC, NT = NW / 16;
  static_assert(NT >= 2 && MI >= 1, "a wave covers whole 32-column dot blocks");
  constexpr int LDR = kHBK + kHPad;      // bf16 per LDS row: 144 B at 64 deep
  constexpr int TPR = kHBK / 4;          // staging threads per row (4 k each)
  constexpr int RPP = 64 * NWV / TPR;    // rows per staging pass
  constexpr int NA = kFBM / RPP;         // A rows staged per thread
  constexpr int NB = kFBN / RPP;         // B rows staged per thread
  __shared__ __attribute__((aligned(16))) __bf16 sA[2][kFBM][LDR];
  __shared__ __attribute__((aligned(16))) __bf16 sB[2][kFBN][LDR];
  const int bid = blockIdx.x;
  int p = 0;
  for (int q = 1; q < batch.count; ++q)
    if (bid >= batch.d[q].tile_begin) p = q;
  const GemmDesc& d = batch.d[p];
  const int t = bid - d.tile_begin;
  if (t >= d.tiles_m * d.tiles_n) return;
  int tr, tc;
  place_tile(d, t, tr, tc);
  const int m0 = tr * kFBM, n0 = tc * kFBN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave / WC) * MW, wn = (wave % WC) * NW;
  const int M = d.M, N = d.N, K = d.K;
  // staging: thread t moves rows t / TPR + RPP i at k = 4 (t % TPR) of both slabs
  const rsrc_t rA = make_rsrc(d.A, 0x7fffffffu), rB = make_rsrc(d.B, 0x7fffffffu);
  uint32_t offA[NA], offB[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int ra = min(m0 + tid / TPR + RPP * i, M - 1);
    offA[i] = (uint32_t)ra * (uint32_t)d.lda * (AH ? 2u : 4u);
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int rb = min(n0 + tid / TPR + RPP * i, N - 1);
    offB[i] = (uint32_t)rb * (uint32_t)d.ldb * 4u;
  }
  const int kq = 4 * (tid % TPR);
  float4 ga[AH ? 1 : NA], gb[BH ? 1 : NB];
  uint2 gah[AH ? NA : 1];             // AH: A rows in bf16, 4 k per 8 bytes
  uint2 gh[BH ? NB : 1];              // BH: B from its bf16 shadow, 4 k per 8 bytes
  const rsrc_t rBh = make_rsrc(BH ? reinterpret_cast<const float*>(d.Bh) : d.B, 0x7fffffffu);
  auto zk = [&](float4 x, int k) {    // elements past K read the row's next columns: zeroed
    x.x = k < K ? x.x : 0.f; x.y = k + 1 < K ? x.y : 0.f; x.z = k + 2 < K ? x.z : 0.f; x.w = k + 3 < K ? x.w : 0.f;
    return x;
  };
  auto zkh = [&](uint2 x, int k) {
    x.x = (k < K ? x.x & 0xffffu : 0u) | (k + 1 < K ? x.x & 0xffff0000u : 0u);
    x.y = (k + 2 < K ? x.y & 0xffffu : 0u) | (k + 3 < K ? x.y & 0xffff0000u : 0u);
    return x;
  };
  auto gload = [&](int k0) {
    const int k = k0 + kq;
    const uint32_t ko = (uint32_t)(k < K ? k : 0) * 4u;
    if constexpr (AH) {
#pragma unroll
      for (int i = 0; i < NA; ++i) gah[i] = zkh(buf_ld2(rA, offA[i] + ko / 2u), k);
    } else {
#pragma unroll
      for (int i = 0; i < NA; ++i) ga[i] = zk(buf_ld4(rA, offA[i] + ko), k);
    }
    if constexpr (BH) {
#pragma unroll
      for (int i = 0; i < NB; ++i) gh[i] = zkh(buf_ld2(rBh, offB[i] / 2u + ko / 2u), k);
    } else {
#pragma unroll
      for (int i = 0; i < NB; ++i) gb[i] = zk(buf_ld4(rB, offB[i] + ko), k);
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      if constexpr (AH) *reinterpret_cast<u2v*>(&sA[buf][tid / TPR + RPP * i][kq]) = u2v{gah[i].x, gah[i].y};
      else *reinterpret_cast<u2v*>(&sA[buf][tid / TPR + RPP * i][kq]) = pack_bf16x4(ga[i]);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      if constexpr (BH) *reinterpret_cast<u2v*>(&sB[buf][tid / TPR + RPP * i][kq]) = u2v{gh[i].x, gh[i].y};
      else *reinterpret_cast<u2v*>(&sB[buf][tid / TPR + RPP * i][kq]) = pack_bf16x4(gb[i]);
    }
  };
  f4 acc[MI][NT];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  FwdEpi<NT, MI> ep;
  ep.load(d, n0 + wn, lane);
  gload(0);
  swrite(0);
  __syncthreads();
  const int nslab = (K + kHBK - 1) / kHBK;
  for (int sl = 0; sl < nslab; ++sl) {
    const int cur = sl & 1;
    gload((sl + 1 < nslab ? sl + 1 : sl) * kHBK);   // unconditional: the last re-reads its slab
#pragma unroll
    for (int kk = 0; kk < kHBK / 32; ++kk) {
      const int kc = kk * 32 + 8 * (lane >> 4);
      bf16x8 a[MI], b[NT];
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = *reinterpret_cast<const bf16x8*>(&sA[cur][wm + i * 16 + (lane & 15)][kc]);
#pragma unroll
      for (int j = 0; j < NT; ++j) b[j] = *reinterpret_cast<const bf16x8*>(&sB[cur][wn + j * 16 + (lane & 15)][kc]);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    swrite(cur ^ 1);
    __syncthreads();
  }
  ep.template store<AH>(d, acc, m0 + wm, n0 + wn, lane);
}

// ---------------------------------------------------------------------------
// k_fwd16p: the act16 forward levels (bf16 activations AND bf16 weight shadows) with a
// multi-slab LDS ring filled by LDS-DMA (global_load_lds_dwordx4: no VGPR per slab in
// flight).  k_fwd16 keeps one slab in flight per workgroup (its register stage), and at
// batch 4096 a slab's load round trip (~2 us under the chip-wide load) is ~5x the slab's
// MFMA time; here one workgroup per CU (1024 threads, 16 waves of (BM/4) x 32) holds
// NST = 144 KiB / stage slabs, NST - 1 of them in flight across the barriers: a counted
// `s_waitcnt vmcnt` (never 0 inside the loop) and a raw s_barrier — a __syncthreads()
// fence would drain the DMA queue (cdna_hip_programming.md, "Pipelining across barriers").
// Tiles BM x 128 (BM = 256 where that still gives a workgroup per CU, else 128), 64-deep
// slabs.  The DMA image is lane-linear (lane l of a 1 KiB piece writes bytes 16 l..), so
// the bank swizzle sits on the SOURCE address: LDS row R holds its 16-byte k-chunk c at
// position c ^ ((R >> 1) & 7) — a fragment read (16 rows at one chunk) hits 16 distinct
// 16-byte slots of a 256-byte bank row.  Chunks past K read a clamped in-row address and
// are zeroed in the fragment registers (last slab only).  Epilogue: FwdEpi (bias, ReLU,
// fc3 dot partials, bf16 column-pair stores), as k_fwd16.
#ifndef SACMI_FWD16P
#define SACMI_FWD16P 1
#endif
#ifndef SACMI_FWD16P_WAVES
#define SACMI_FWD16P_WAVES 16   // k_fwd16p waves per workgroup (8 or 16)
#endif
constexpr int kPLds = 144 * 1024;
template <int BM>
__host__ __device__ constexpr int fwd16p_stages() { return kPLds / ((BM + 128) * 128); }

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

template <int N>
__device__ __forceinline__ void vm_wait_lgkm0() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ bf16x8 zero_past(bf16x8 x, int nvalid) {   // keep elements < nvalid
  uint4 u = __builtin_bit_cast(uint4, x);
  auto m = [&](unsigned w, int e) {
    return (e < nvalid ? w & 0xffffu : 0u) | (e + 1 < nvalid ? w & 0xffff0000u : 0u);
  };
  u.x = m(u.x, 0); u.y = m(u.y, 2); u.z = m(u.z, 4); u.w = m(u.w, 6);
  return __builtin_bit_cast(bf16x8, u);
}

template <int BM, int NWV = 16>
__global__ __launch_bounds__(64 * NWV, 1) void k_fwd16p(GemmBatch batch) {
  const TlMark tl_mark(batch.tl, TL_FWD16P);
  constexpr int BN = 128, BK = 64, NST = fwd16p_stages<BM>();
  // NWV waves as WR x WC: 16 -> 4 x 4 of (BM/4) x 32; 8 -> BM 256: 4 x 2 of 64 x 64, BM 128: 2 x 4 of 64 x 32
  constexpr int WR = NWV == 16 ? 4 : (BM == 256 ? 4 : 2), WC = NWV / WR;
  constexpr int MW = BM / WR, MI = MW / 16, NW = BN / WC, NT = NW / 16;
  constexpr int ROWB = BK * 2;                       // bytes per LDS row (64 bf16)
  constexpr int STAGE = (BM + BN) * ROWB;
  constexpr int PPW = (BM + BN) / 8 / NWV;           // 1 KiB pieces per wave per slab
  constexpr int APW = BM / 8 / NWV;                  // ... of them A pieces
  static_assert(NST >= 3 && PPW * NWV * 8 == BM + BN && APW * NWV * 8 == BM, "k_fwd16p geometry");
  __shared__ __attribute__((aligned(16))) unsigned char lds[NST * STAGE];
  const int bid = blockIdx.x;
  int p = 0;
  for (int q = 1; q < batch.count; ++q)
    if (bid >= batch.d[q].tile_begin) p = q;
  const GemmDesc& d = batch.d[p];
  const int t = bid - d.tile_begin;
  if (t >= d.tiles_m * d.tiles_n) return;
  int tr, tc;
  place_tile(d, t, tr, tc);
  const int m0 = tr * BM, n0 = tc * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave / WC) * MW, wn = (wave % WC) * NW;
  const int M = d.M, N = d.N, K = d.K;
  // DMA sources: wave w moves pieces w + 16 i (A rows 8 pc.., then B rows); lane l of a
  // piece: LDS row 8 pc + (l >> 3), position l & 7, global chunk (l & 7) ^ swizzle
  const unsigned char* src[PPW];
  int cko[PPW];                                      // the lane's chunk, in bf16 elements
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int pc = wave + NWV * i;
    const bool isA = i < APW;
    const int R = (isA ? pc : pc - BM / 8) * 8 + (lane >> 3);
    const int sw = (R >> 1) & 7;
    cko[i] = 8 * ((lane & 7) ^ sw);
    if (isA) {
      const int ra = min(m0 + R, M - 1);
      src[i] = reinterpret_cast<const unsigned char*>(d.A) + (size_t)ra * d.lda * 2;
    } else {
      const int rb = min(n0 + R, N - 1);
      src[i] = reinterpret_cast<const unsigned char*>(d.Bh) + (size_t)rb * d.ldb * 2;
    }
  }
  auto issue = [&](int sl) {                         // slab sl into ring slot sl % NST
    unsigned char* dst = lds + (sl % NST) * STAGE;
    const int k0 = sl * BK;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int k = k0 + cko[i];
      const unsigned char* g = src[i] + (k < K ? k : 0) * 2;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)(dst + (wave + NWV * i) * 1024), 16, 0, 0);
    }
  };
  f4 acc[MI][NT];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  FwdEpi<NT, MI> ep;                                 // issued first: oldest on the vm queue
  ep.load(d, n0 + wn, lane);
  const int nslab = (K + BK - 1) / BK;
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nslab) issue(s);
  const int r16 = lane & 15, sx = r16 >> 1;
  for (int sl = 0; sl < nslab; ++sl) {
    // slabs sl .. min(sl + NST - 2, nslab - 1) are outstanding: retire sl only
    const int ahead = min(NST - 2, nslab - 1 - sl);
    if (ahead >= 2) vm_wait_lgkm0<2 * PPW>();
    else if (ahead == 1) vm_wait_lgkm0<PPW>();
    else vm_wait_lgkm0<0>();
    __builtin_amdgcn_s_barrier();                    // every wave's slab sl landed; slot (sl-1) free
    asm volatile("" ::: "memory");
    if (sl + NST - 1 < nslab) issue(sl + NST - 1);
    const unsigned char* st = lds + (sl % NST) * STAGE;
    const int kval = K - sl * BK;                    // valid k of this slab (>= BK but the last)
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int c = kk * 4 + (lane >> 4);
      const int off = (c ^ sx) << 4;
      bf16x8 a[MI], b[NT];
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = *reinterpret_cast<const bf16x8*>(st + (wm + i * 16 + r16) * ROWB + off);
#pragma unroll
      for (int j = 0; j < NT; ++j) b[j] = *reinterpret_cast<const bf16x8*>(st + (BM + wn + j * 16 + r16) * ROWB + off);
      if (kval < BK) {                               // the last, partial slab: zero k >= K
        const int nv = kval - 8 * c;
#pragma unroll
        for (int i = 0; i < MI; ++i) a[i] = zero_past(a[i], nv);
#pragma unroll
        for (int j = 0; j < NT; ++j) b[j] = zero_past(b[j], nv);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  // staged epilogue: the bf16 tile image in the (now idle) ring, then 16 bytes a lane per
  // store — full 128-byte lines, write-through when the level asks (batch.st_wt): the
  // kernel-end L2 writeback in front of the dependent level has less to do
  constexpr int TLD = BN / 2 + 4;                    // words per tile row (272 B: conflict-free reads)
  static_assert(BM * TLD * 4 <= NST * STAGE, "k_fwd16p epilogue tile");
  __syncthreads();                                   // every wave is past its last ring read
  uint32_t* tile = reinterpret_cast<uint32_t*>(lds);
  ep.template store<true>(d, acc, m0 + wm, n0 + wn, lane, tile, m0, n0, TLD);
  __syncthreads();
  const bool wt = batch.st_wt != 0;
  const rsrc_t rC = make_rsrc(d.C, 0x7fffffffu);
  const int ch = tid & 15;                           // 16-byte chunk of a 256-byte tile row
#pragma unroll
  for (int pass = 0; pass < BM / (4 * NWV); ++pass) {
    const int r = pass * 4 * NWV + (tid >> 4), row = m0 + r, col = n0 + 8 * ch;
    const uint4 v = *reinterpret_cast<const uint4*>(tile + r * TLD + 4 * ch);
    if (row < M && col < N) {
      const uint32_t off = (uint32_t)(((size_t)row * d.ldc + col) * 2);
      const wt_f4 x = __builtin_bit_cast(wt_f4, v);
      if (wt) llvm_raw_buffer_store_wt_v4f32(x, rC, (int)off, 0, kStAux);
      else llvm_raw_buffer_store_wt_v4f32(x, rC, (int)off, 0, 0);
    }
  }
}

// whether an act16 level can run on k_fwd16p, and its row tile (0: no).  Every operand row
// must start 16-byte aligned (the DMA moves 16-byte chunks) and hold round_up(K, 8)
// elements inside its stride (a chunk straddling K stays in its row).
static int fwd16p_plan(GemmBatch& b) {
  if (!SACMI_FWD16P || !b.bf16 || b.ride.kind) return 0;
  static const bool off = std::getenv("SACMI_NO_FWD16P") != nullptr;
  if (off) return 0;
  for (int i = 0; i < b.count; ++i) {
    const GemmDesc& d = b.d[i];
    const int k8 = (d.K + 7) & ~7;
    if (!d.a16 || !d.c16 || d.b16 || d.x16 || !d.Bh || (d.N & 1) || (d.ldc & 1)) return 0;
    if (((uintptr_t)d.A & 15) || ((uintptr_t)d.Bh & 15) || (d.lda & 7) || (d.ldb & 7)) return 0;
    if (k8 > d.lda || k8 > d.ldb || d.K < 1) return 0;
    if ((d.N & 7) || (d.ldc & 7) || ((uintptr_t)d.C & 15)) return 0;   // 16-byte epilogue stores
  }
  static const bool wt = std::getenv("SACMI_FWD16P_WT") == nullptr || std::atoi(std::getenv("SACMI_FWD16P_WT")) != 0;
  b.st_wt = wt ? 1 : 0;
  if (assign_tiles<256, 128>(b) >= 256) return 256;
  if (assign_tiles<128, 128>(b) >= 256) return 128;
  return 0;
}

// ---------------------------------------------------------------------------
// Deep-K weight-gradient levels in bf16 mode (batch 4096 class): dW = dY^T X with both
// operands row-contiguous.  k_dw_part: 128x128 output tiles, K split NS ways across
// workgroups; each workgroup stages 32-row slabs of dY (128 columns) and X (128 columns)
// through LDS (double buffered) and writes its partial tile (+ the bias-gradient row-sum
// partial) to a workspace.  k_dw_fin: one thread per output element sums the NS partials
// in fixed order and runs the epilogue (store, or Adam [+ Polyak] with the gradient export
// and block 0's loss / alpha extras) — both forms of a level take this path, so the
// fused and the data-parallel updates keep identical bits.
constexpr int kDBM = 128, kDBN = 128, kDBK = 32, kDPad = 4;
#ifndef SACMI_DW_TARGET
#define SACMI_DW_TARGET 512     // k_dw_part workgroup slots (256 CUs x 2)
#endif
constexpr int kDwMaxSplit = 16;
#ifndef SACMI_DWFIN_EPT
#define SACMI_DWFIN_EPT 1       // k_dw_fin elements per thread (1, 2, 4 measured alike)
#endif
#ifndef SACMI_DWFIN_NSL
#define SACMI_DWFIN_NSL 1       // k_dw_fin instantiated per split count (0: one 16-load form)
#endif
constexpr int kDwFinEpt = SACMI_DWFIN_EPT;
#ifndef SACMI_DW_SPLIT_FP32
#define SACMI_DW_SPLIT_FP32 0   // the split-K dW path for fp32 levels too (k_dw_part<false>)
#endif
#ifndef SACMI_AXK_LDS16
#define SACMI_AXK_LDS16 1       // bf16 mode: k_axk16 for the batch-4096-class dh levels
#endif
#ifndef SACMI_DW_LDS16
#define SACMI_DW_LDS16 1        // bf16 mode: k_dw_part16 (bf16 k-major LDS, transposed reads)
#endif

// workspace layout: partial s of desc p at ws + s * ws_stride + desc_off[p], row-major
// [M][ncols] with ncols = N (+1 for the row-sum column) rounded up to a multiple of 4: every
// partial row starts 16-byte aligned, so k_dw_fin moves 4-column groups (the pad columns are
// never written and never used)
__host__ __device__ __forceinline__ int dw_ncols_real(const GemmDesc& d) { return d.rs_col >= 0 ? d.N + 1 : d.N; }
__host__ __device__ __forceinline__ int dw_ncols(const GemmDesc& d) { return (dw_ncols_real(d) + 3) & ~3; }

// XCD placement of the split-K work (workgroup b runs on XCD b % 8): the split-major work
// list w = split * tiles + tile is dealt to the XCDs in contiguous eighths, so each XCD's
// L2 streams the rows of one or two K ranges instead of every range (SACMI_DW_XCD 0: the
// plain order).  The tile grid is padded to a multiple of 8 workgroups.
#ifndef SACMI_DW_XCD
#define SACMI_DW_XCD 1
#endif
__host__ __device__ __forceinline__ int dw_grid_tiles(int tiles, int ns) {
  return SACMI_DW_XCD ? (tiles * ns + 7) / 8 * 8 : tiles * ns;
}
__device__ __forceinline__ int dw_work_index(int b, int tiles, int ns) {
  if (!SACMI_DW_XCD) return b;
  const int W = tiles * ns, per = (W + 7) / 8;
  const int w = (b % 8) * per + b / 8;
  return w < W ? w : -1;
}

template <bool BF16>
__global__ __launch_bounds__(256, 2) void k_dw_part(GemmBatch batch, int ns, int64_t ws_stride) {
  const TlMark tl_mark(batch.tl, TL_DW_PART);
  __shared__ __attribute__((aligned(16))) float sA[2][kDBK][kDBM + kDPad];
  __shared__ __attribute__((aligned(16))) float sB[2][kDBK][kDBN + kDPad];
  const int tiles_tot = batch.total_tiles;
  const int nwg = dw_grid_tiles(tiles_tot, ns);
  if ((int)blockIdx.x >= nwg) {   // ride-along: the next update's gather
    const int rb = blockIdx.x - nwg, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int b = rb * 4 + wave; b < batch.ride.ga.B; b += batch.ride.nblocks * 4)
      gather_row(batch.ride.ga, b, lane, 64);
    return;
  }
  const int wk = dw_work_index(blockIdx.x, tiles_tot, ns);
  if (wk < 0) return;
  const int split = wk / tiles_tot, bid = wk % tiles_tot;
  int p = 0;
  for (int q = 1; q < batch.count; ++q)
    if (bid >= batch.d[q].tile_begin) p = q;
  const GemmDesc& d = batch.d[p];
  const int t = bid - d.tile_begin;
  if (t >= d.tiles_m * d.tiles_n) return;
  const int m0 = (t / d.tiles_n) * kDBM, n0 = (t % d.tiles_n) * kDBN;
  const int M = d.M, N = d.N, K = d.K;
  const int kc = ((K + ns - 1) / ns + kDBK - 1) / kDBK * kDBK;
  const int kb = split * kc, ke = min(K, kb + kc);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  // staging: thread t moves k rows (t >> 5) + 8 i (i < 4), columns 4 (t & 31) .. +3
  const int c4 = 4 * (tid & 31);
  const rsrc_t rA = make_rsrc(d.A, 0x7fffffffu), rB = make_rsrc(d.B, 0x7fffffffu);
  const rsrc_t rS = make_rsrc(d.a_ksc ? d.a_ksc : d.A, d.a_ksc ? (uint32_t)K * 4u : 0u);
  const bool has_ksc = d.a_ksc != nullptr;
  // 4-wide operand reads start at a 4-aligned column <= the last one, so they stay inside
  // a row padded to a multiple of 4; an operand narrower than 4 columns (the fc3 gradient
  // dq, lda = 1) reads up to 3 floats past its last row: dw_split_plan's caller keeps
  // that slack allocated (sacmi.hip: dq).  (A per-load scalar fallback under a branch
  // measured L6 74 -> 93 us: the guarded loads drain the load queue.)
  const int ma = min(m0 + c4, (M - 1) & ~3), nb = min(n0 + c4, (N - 1) & ~3);
  float4 ga[4], gb[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = k0 + (tid >> 5) + 8 * i;
      const bool kin = k < ke;
      const uint32_t kk = (uint32_t)(kin ? k : 0);   // row 0 always exists (a split may start past K)
      float4 x = buf_ld4(rA, (kk * (uint32_t)d.lda + (uint32_t)ma) * 4u);
      float4 y = buf_ld4(rB, (kk * (uint32_t)d.ldb + (uint32_t)nb) * 4u);
      const float f = has_ksc ? buf_ld(rS, kk * 4u) : 1.f;
      // columns past M / N (and rows past this split's K range) contribute zero
      x.x = kin && m0 + c4 < M ? x.x * f : 0.f;     x.y = kin && m0 + c4 + 1 < M ? x.y * f : 0.f;
      x.z = kin && m0 + c4 + 2 < M ? x.z * f : 0.f; x.w = kin && m0 + c4 + 3 < M ? x.w * f : 0.f;
      y.x = kin && n0 + c4 < N ? y.x : 0.f;         y.y = kin && n0 + c4 + 1 < N ? y.y : 0.f;
      y.z = kin && n0 + c4 + 2 < N ? y.z : 0.f;     y.w = kin && n0 + c4 + 3 < N ? y.w : 0.f;
      ga[i] = x; gb[i] = y;
    }
  };
  auto swrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      *reinterpret_cast<float4*>(&sA[buf][(tid >> 5) + 8 * i][c4]) = ga[i];
      *reinterpret_cast<float4*>(&sB[buf][(tid >> 5) + 8 * i][c4]) = gb[i];
    }
  };
  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  float rs = 0.f;                       // row sum of A row m0 + tid (tid < 128), this split
  const bool want_rs = d.rs_col >= 0 && n0 == 0;
  const int nslab = (ke - kb + kDBK - 1) / kDBK;
  gload(kb);
  swrite(0);
  __syncthreads();
  for (int sl = 0; sl < nslab; ++sl) {
    const int cur = sl & 1;
    gload(kb + (sl + 1 < nslab ? sl + 1 : sl) * kDBK);
#pragma unroll
    for (int kk = 0; kk < kDBK / 16; ++kk) {
      float a[4][4], b[4][4];
      const int kr = kk * 16 + 4 * (lane >> 4);
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i][s2] = sA[cur][kr + s2][wm + i * 16 + (lane & 15)];
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j][s2] = sB[cur][kr + s2][wn + j * 16 + (lane & 15)];
      }
      mfma_chunk<4, 4, BF16>(acc, a, b);
    }
    if (want_rs && tid < kDBM) {
#pragma clang fp contract(off)
      for (int r = 0; r < kDBK; ++r) rs += sA[cur][r][tid];
    }
    swrite(cur ^ 1);
    __syncthreads();
  }
  // partial tile (+ row-sum partial) to the workspace
  int64_t off = 0;
  for (int q = 0; q < p; ++q) off += (int64_t)batch.d[q].M * dw_ncols(batch.d[q]);
  float* w = batch.ws + (int64_t)split * ws_stride + off;
  const int nc = dw_ncols(d);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wm + i * 16 + (lane >> 4) * 4 + r;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + wn + j * 16 + (lane & 15);
        if (row < M && col < N) st_big(w + (int64_t)row * nc + col, acc[i][j][r]);
      }
    }
  if (want_rs && tid < kDBM && m0 + tid < M) st_big(w + (int64_t)(m0 + tid) * nc + N, rs);
}

// bf16 mode, bf16 in LDS: k_dw_part with the operands rounded once at staging and kept
// k-major ([k][128 columns] bf16, 64-deep slabs, rows padded to 272 B).  The 16x16x32
// operand (lane l: A[l&15][k = 8(l>>4) + j]) is read with two ds_read_b64_tr_b16 per
// fragment — the hardware transpose delivers 4 k of one column per lane, lane 4q+p of a
// 16-lane group addressing k row q, columns 4p..4p+3 of the block — conflict-free with
// the 68-dword row stride.  Bias-gradient row sums come from the unrounded fp32 staging
// registers: per thread over its k rows, then over the 8 threads sharing a column group
// in fixed order.
typedef short s4t __attribute__((ext_vector_type(4)));
typedef short s8t __attribute__((ext_vector_type(8)));
constexpr int kD16K = 64, kD16Pad = 8;
constexpr int kDw16OpBytes = 2 * kD16K * (kDBM + kD16Pad) * 2;      // one operand, 2 slabs
#ifndef SACMI_DW16_WAVES
#define SACMI_DW16_WAVES 8      // waves per k_dw_part16 workgroup (4: 2 x 2 of 64x64; 8: 2 x 4 of 64x32)
#endif
constexpr int kDw16Waves = SACMI_DW16_WAVES, kDw16Krp = 64 * kDw16Waves / 32;   // k rows per staging pass
static_assert(kDw16LdsBytes >= 2 * kDw16OpBytes + kDw16Krp * kDBM * 4, "k_dw_part16 LDS layout");

__device__ __forceinline__ s4t lds_tr16(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s4t*)(p));
}

// X16 (act16): the B operand (X: activations / minibatch inputs) is bf16
// AXT: the level carries a dW A transform (axk 2, opt-in): its own instantiation, so the
// plain form's staging pass issues no extra load
template <bool X16 = false, bool AXT = false>
__global__ __launch_bounds__(64 * kDw16Waves, 2) void k_dw_part16(GemmBatch batch, int ns, int64_t ws_stride) {
  const TlMark tl_mark(batch.tl, TL_DW_PART16);
  constexpr int LDR = kDBM + kD16Pad;          // bf16 per LDS k row (272 B)
  // one LDS block (kDw16LdsBytes): the two operand slabs and the row-sum scratch, or a
  // ride-along sampler's table
  __shared__ __attribute__((aligned(16))) unsigned char lds_raw[kDw16LdsBytes];
  auto& sA = *reinterpret_cast<__bf16 (*)[2][kD16K][LDR]>(lds_raw);
  auto& sB = *reinterpret_cast<__bf16 (*)[2][kD16K][LDR]>(lds_raw + kDw16OpBytes);
  auto& s_rs = *reinterpret_cast<float (*)[kDw16Krp][kDBM]>(lds_raw + 2 * kDw16OpBytes);
  constexpr int NWV = kDw16Waves, WC = NWV / 2, NJ = kDBN / WC / 16;   // 2 x WC waves of 64 x (128 / WC)
  constexpr int KRP = kDw16Krp, NI = kD16K / KRP;                       // staging: KRP k rows a pass
  const int tiles_tot = batch.total_tiles;
  const int nwg = dw_grid_tiles(tiles_tot, ns);
  if ((int)blockIdx.x >= nwg) {   // ride-along: the next update's sampling or gather
    const int rb = blockIdx.x - nwg, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (batch.ride.kind == 1) {
      if (rb == 0) mt_sample_body(batch.ride.mt, batch.ride.tbl_log2, reinterpret_cast<uint32_t*>(lds_raw));
    } else {
      for (int b = rb * NWV + wave; b < batch.ride.ga.B; b += batch.ride.nblocks * NWV)
        gather_row(batch.ride.ga, b, lane, 64);
    }
    return;
  }
  const int wk = dw_work_index(blockIdx.x, tiles_tot, ns);
  if (wk < 0) return;
  const int split = wk / tiles_tot, bid = wk % tiles_tot;
  int p = 0;
  for (int q = 1; q < batch.count; ++q)
    if (bid >= batch.d[q].tile_begin) p = q;
  const GemmDesc& d = batch.d[p];
  const int t = bid - d.tile_begin;
  if (t >= d.tiles_m * d.tiles_n) return;
  const int m0 = (t / d.tiles_n) * kDBM, n0 = (t % d.tiles_n) * kDBN;
  const int M = d.M, N = d.N, K = d.K;
  const int kc = ((K + ns - 1) / ns + kD16K - 1) / kD16K * kD16K;
  const int kb = split * kc, ke = min(K, kb + kc);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave / WC) * 64, wn = (wave % WC) * (kDBN / WC);
  // staging: thread t moves k rows (t >> 5) + KRP i (i < NI), columns 4 (t & 31) .. +3
  const int c4 = 4 * (tid & 31), kr0 = tid >> 5;
  const rsrc_t rA = make_rsrc(d.A, 0x7fffffffu), rB = make_rsrc(d.B, 0x7fffffffu);
  const rsrc_t rS = make_rsrc(d.a_ksc ? d.a_ksc : d.A, d.a_ksc ? (uint32_t)K * 4u : 0u);
  const bool has_ksc = d.a_ksc != nullptr;
  // 4-wide operand reads start at a 4-aligned column <= the last one, so they stay inside
  // a row padded to a multiple of 4; an operand narrower than 4 columns (the fc3 gradient
  // dq, lda = 1) reads up to 3 floats past its last row: dw_split_plan's caller keeps
  // that slack allocated (sacmi.hip: dq).  (A per-load scalar fallback under a branch
  // measured L6 74 -> 93 us: the guarded loads drain the load queue.)
  const int ma = min(m0 + c4, (M - 1) & ~3), nb = min(n0 + c4, (N - 1) & ~3);
  const bool want_rs = d.rs_col >= 0 && n0 == 0;
  // axk 2 (act16): A is the bf16 activation h [k][m] and the operand is u = [h > 0] w[m]
  // (w: ax_w, M % 4 == 0) — the values L5 would have stored as u rows.  Both loads are
  // issued on every pass, the unused one at an out-of-range offset: no branch around them
  const bool axt = AXT && d.axk == 2;
  const rsrc_t rAh = make_rsrc(axt ? d.A : d.C, axt ? 0x7fffffffu : 0u);
  const float4 w3v = axt ? buf_ld4(make_rsrc(d.ax_w, (uint32_t)M * 4u), (uint32_t)ma * 4u) : float4{0.f, 0.f, 0.f, 0.f};
  float4 ga[NI], gb[X16 ? 1 : NI];
  uint2 gbh[X16 ? NI : 1];
  float rs4[4] = {0.f, 0.f, 0.f, 0.f};
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int k = k0 + kr0 + KRP * i;
      const bool kin = k < ke;
      const uint32_t kk = (uint32_t)(kin ? k : 0);   // row 0 always exists (a split may start past K)
      const uint32_t ea = kk * (uint32_t)d.lda + (uint32_t)ma;
      float4 x = buf_ld4(rA, axt ? 0xfffffff0u : ea * 4u);
      if constexpr (AXT) {
        const uint2 hx = buf_ld2(rAh, axt ? ea * 2u : 0xfffffff0u);
        if (axt)
          x = make_float4(bf16_lo(hx.x) > 0.f ? w3v.x : 0.f, bf16_hi(hx.x) > 0.f ? w3v.y : 0.f,
                          bf16_lo(hx.y) > 0.f ? w3v.z : 0.f, bf16_hi(hx.y) > 0.f ? w3v.w : 0.f);
      }
      const float f = has_ksc ? buf_ld(rS, kk * 4u) : 1.f;
      // columns past M / N (and rows past this split's K range) contribute zero
      x.x = kin && m0 + c4 < M ? x.x * f : 0.f;     x.y = kin && m0 + c4 + 1 < M ? x.y * f : 0.f;
      x.z = kin && m0 + c4 + 2 < M ? x.z * f : 0.f; x.w = kin && m0 + c4 + 3 < M ? x.w * f : 0.f;
      ga[i] = x;
      if constexpr (X16) {
        uint2 h = buf_ld2(rB, (kk * (uint32_t)d.ldb + (uint32_t)nb) * 2u);
        h.x = (kin && n0 + c4 < N ? h.x & 0xffffu : 0u) | (kin && n0 + c4 + 1 < N ? h.x & 0xffff0000u : 0u);
        h.y = (kin && n0 + c4 + 2 < N ? h.y & 0xffffu : 0u) | (kin && n0 + c4 + 3 < N ? h.y & 0xffff0000u : 0u);
        gbh[i] = h;
      } else {
        float4 y = buf_ld4(rB, (kk * (uint32_t)d.ldb + (uint32_t)nb) * 4u);
        y.x = kin && n0 + c4 < N ? y.x : 0.f;         y.y = kin && n0 + c4 + 1 < N ? y.y : 0.f;
        y.z = kin && n0 + c4 + 2 < N ? y.z : 0.f;     y.w = kin && n0 + c4 + 3 < N ? y.w : 0.f;
        gb[i] = y;
      }
    }
  };
  auto swrite = [&](int buf, bool fresh) {   // fresh: a slab not staged before
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      *reinterpret_cast<u2v*>(&sA[buf][kr0 + KRP * i][c4]) = pack_bf16x4(ga[i]);
      if constexpr (X16) *reinterpret_cast<u2v*>(&sB[buf][kr0 + KRP * i][c4]) = u2v{gbh[i].x, gbh[i].y};
      else *reinterpret_cast<u2v*>(&sB[buf][kr0 + KRP * i][c4]) = pack_bf16x4(gb[i]);
    }
    if (want_rs && fresh) {
#pragma clang fp contract(off)
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        rs4[0] += ga[i].x; rs4[1] += ga[i].y; rs4[2] += ga[i].z; rs4[3] += ga[i].w;
      }
    }
  };
  f4 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const int nslab = (ke - kb + kD16K - 1) / kD16K;
  // transposed-read lane roles: group g = lane >> 4 takes k 8g..8g+7; lane 4q+p of the
  // group addresses k row q (+4 for the second half), columns 4p..4p+3 of a 16-column block
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg = lane >> 4;
  gload(kb);
  swrite(0, true);
  __syncthreads();
  for (int sl = 0; sl < nslab; ++sl) {
    const int cur = sl & 1;
    gload(kb + (sl + 1 < nslab ? sl + 1 : sl) * kD16K);
#pragma unroll
    for (int kk = 0; kk < kD16K / 32; ++kk) {
      const int kr = kk * 32 + 8 * tg + tq;
      bf16x8 a[4], b[NJ];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const s4t lo = lds_tr16(&sA[cur][kr][wm + i * 16 + 4 * tp]);
        const s4t hi = lds_tr16(&sA[cur][kr + 4][wm + i * 16 + 4 * tp]);
        const s8t v = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        a[i] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const s4t lo = lds_tr16(&sB[cur][kr][wn + j * 16 + 4 * tp]);
        const s4t hi = lds_tr16(&sB[cur][kr + 4][wn + j * 16 + 4 * tp]);
        const s8t v = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        b[j] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    swrite(cur ^ 1, sl + 1 < nslab);
    __syncthreads();
  }
  // partial tile (+ row-sum partial) to the workspace
  int64_t off = 0;
  for (int q = 0; q < p; ++q) off += (int64_t)batch.d[q].M * dw_ncols(batch.d[q]);
  float* w = batch.ws + (int64_t)split * ws_stride + off;
  const int nc = dw_ncols(d);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = m0 + wm + i * 16 + (lane >> 4) * 4 + r;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int col = n0 + wn + j * 16 + (lane & 15);
        if (row < M && col < N) st_big(w + (int64_t)row * nc + col, acc[i][j][r]);
      }
    }
  if (want_rs) {
    s_rs[kr0][c4] = rs4[0]; s_rs[kr0][c4 + 1] = rs4[1];
    s_rs[kr0][c4 + 2] = rs4[2]; s_rs[kr0][c4 + 3] = rs4[3];
    __syncthreads();
    if (tid < kDBM && m0 + tid < M) {
#pragma clang fp contract(off)
      float v = s_rs[0][tid];
      for (int g = 1; g < KRP; ++g) v += s_rs[g][tid];
      st_big(w + (int64_t)(m0 + tid) * nc + N, v);
    }
  }
}

// bf16 mode, batch-4096 class: the row-prologue dh levels (L5 / L9 and their model2
// form) on LDS-staged 64x128 tiles.  dh[b][n] = coef[b] * sum_k u[b][k] W[k][n] * [h[b][n] > 0]
// with u[b][k] = h2[b][k] > 0 ? w3[k] : 0 formed at staging (the coefficient-free rows u
// also stored, by the column-tile-0 workgroups, for the later weight gradient) and the
// per-row coefficients from the same row prologue as k_gemm's (rows_load before the K
// loop, rows_finish after it: identical values, so the losses and dq bits do not depend
// on the kernel).  A = u in [row][k] bf16 slabs (one ds_read_b128 per 16x16x32 fragment),
// B = W k-major (two ds_read_b64_tr_b16 per fragment); 2x2 waves of 32x64.
// AX = false: the same kernel for the plain dh levels (dh = (dY W) * [h > 0]: L12 and the
// model2 L5b / L9b / L11), no transform, no prologue.
constexpr int kXBM = 64, kXBN = 128, kXBK = 64;

// ACT16 (act16 updates): the ReLU-mask source (aux) is bf16, and so is A where it is the
// activation whose sign the transform reads (AX); the plain levels' A is a gradient, fp32
#ifndef SACMI_AXK16_WAVES
#define SACMI_AXK16_WAVES 8     // waves per k_axk16 workgroup (4: 2 x 2 of 32x64; 8: 2 x 4 of 32x32)
#endif
constexpr int kAxWaves = SACMI_AXK16_WAVES;
template <bool AX, bool BH = false, bool ACT16 = false>
__global__ __launch_bounds__(64 * kAxWaves, 2) void k_axk16(GemmBatch batch) {
  const TlMark tl_mark(batch.tl, TL_AXK16);
  constexpr int LDA_ = kXBK + 8;        // [row][k] bf16, 144-B rows
  constexpr int LDB_ = kXBN + 8;        // [k][n] bf16, 272-B rows
  __shared__ __attribute__((aligned(16))) __bf16 sA[2][kXBM][LDA_];
  __shared__ __attribute__((aligned(16))) __bf16 sB[2][kXBK][LDB_];
  __shared__ float s_q[kXBM][4], s_coef[2][kXBM], s_l[kXBM][2];
  constexpr int NWV = kAxWaves, NTH = 64 * NWV, WC = NWV / 2, NJ = kXBN / WC / 16;
  constexpr int ARP = NTH / 16, NAI = kXBM / ARP;   // A staging: rows a pass, passes
  constexpr int BKP = NTH / 32, NBI = kXBK / BKP;   // B staging: k rows a pass, passes
  const int bid = blockIdx.x;
  if (bid >= batch.total_tiles) {   // ride-along: the next update's gather, a row a wave
    // (one row of 3 float4 per lane: the branch's registers stay under the tiles' 128 —
    // two rows a wave took the kernel to 131 VGPRs, one 8-wave workgroup per CU)
    const int wv = (bid - batch.total_tiles) * NWV + (int)(threadIdx.x >> 6), nwv = batch.ride.nblocks * NWV;
    for (int b0 = wv; b0 < batch.ride.ga.B; b0 += nwv)
      gather_rows_wave<1, 3>(batch.ride.ga, b0, nwv, threadIdx.x & 63);
    return;
  }
  int p = 0;
  for (int q = 1; q < batch.count; ++q)
    if (bid >= batch.d[q].tile_begin) p = q;
  const GemmDesc& d = batch.d[p];
  const int t = bid - d.tile_begin;
  if (t >= d.tiles_m * d.tiles_n) return;
  int tr, tc;
  place_tile(d, t, tr, tc);
  const int m0 = tr * kXBM, n0 = tc * kXBN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave / WC) * 32, wn = (wave % WC) * (kXBN / WC);
  const int M = d.M, N = d.N, K = d.K;
  const rsrc_t rA = make_rsrc(d.A, 0x7fffffffu), rB = make_rsrc(d.B, 0x7fffffffu);
  const rsrc_t rW = make_rsrc(AX ? d.ax_w : d.A, AX ? (uint32_t)K * 4u : 0u);
  const bool store_a = AX && n0 == 0 && d.ax_out != nullptr;
  const rsrc_t rAx = make_rsrc(store_a ? d.ax_out : d.C,
                               store_a ? (uint32_t)(((size_t)(M - 1) * d.ax_ld + K) * 4) : 0u);
  // A staging: rows (t >> 4) + ARP i (i < NAI) at k = 4 (t & 15); B staging: k rows
  // (t >> 5) + BKP i (i < NBI) at columns 4 (t & 31)
  const int kq = 4 * (tid & 15), c4 = 4 * (tid & 31), kr0 = tid >> 5;
  uint32_t offA[NAI];
  constexpr bool A16 = AX && ACT16;
#pragma unroll
  for (int i = 0; i < NAI; ++i)
    offA[i] = (uint32_t)min(m0 + (tid >> 4) + ARP * i, M - 1) * (uint32_t)d.lda * (A16 ? 2u : 4u);
  const int nb = min(n0 + c4, N - 1);
  float4 ga[NAI], gb[BH ? 1 : NBI], gw;
  uint2 gh[BH ? NBI : 1];               // BH: W from its bf16 shadow
  const rsrc_t rBh = make_rsrc(BH ? reinterpret_cast<const float*>(d.Bh) : d.B, 0x7fffffffu);
  auto gload = [&](int k0) {
    const int k = k0 + kq;
    const uint32_t ko = (uint32_t)(k < K ? k : 0) * 4u;
#pragma unroll
    for (int i = 0; i < NAI; ++i) {
      if constexpr (A16) {   // (only the sign is read: exact widening)
        const uint2 h = buf_ld2(rA, offA[i] + ko / 2u);
        ga[i] = make_float4(bf16_lo(h.x), bf16_hi(h.x), bf16_lo(h.y), bf16_hi(h.y));
      } else {
        ga[i] = buf_ld4(rA, offA[i] + ko);
      }
    }
    gw = buf_ld4(rW, ko);
#pragma unroll
    for (int i = 0; i < NBI; ++i) {
      const int kb = k0 + kr0 + BKP * i;
      const bool kin = kb < K;
      const uint32_t e = (uint32_t)(kin ? kb : 0) * (uint32_t)d.ldb + (uint32_t)nb;
      if constexpr (BH) {
        uint2 h = buf_ld2(rBh, e * 2u);
        h.x = (kin && n0 + c4 < N ? h.x & 0xffffu : 0u) | (kin && n0 + c4 + 1 < N ? h.x & 0xffff0000u : 0u);
        h.y = (kin && n0 + c4 + 2 < N ? h.y & 0xffffu : 0u) | (kin && n0 + c4 + 3 < N ? h.y & 0xffff0000u : 0u);
        gh[i] = h;
      } else {
        float4 y = buf_ld4(rB, e * 4u);
        y.x = kin && n0 + c4 < N ? y.x : 0.f;         y.y = kin && n0 + c4 + 1 < N ? y.y : 0.f;
        y.z = kin && n0 + c4 + 2 < N ? y.z : 0.f;     y.w = kin && n0 + c4 + 3 < N ? y.w : 0.f;
        gb[i] = y;
      }
    }
  };
  auto swrite = [&](int buf, int k0, bool fresh) {
    const int k = k0 + kq;
#pragma unroll
    for (int i = 0; i < NAI; ++i) {
      // u = [h2 > 0] w3 (exact fp32 values: w3 or 0), rounded to bf16 for the MFMAs
      const float4 a = ga[i];
      const float4 u = AX ? make_float4(a.x > 0.f && k < K ? gw.x : 0.f, a.y > 0.f && k + 1 < K ? gw.y : 0.f,
                                        a.z > 0.f && k + 2 < K ? gw.z : 0.f, a.w > 0.f && k + 3 < K ? gw.w : 0.f)
                          : make_float4(k < K ? a.x : 0.f, k + 1 < K ? a.y : 0.f,
                                        k + 2 < K ? a.z : 0.f, k + 3 < K ? a.w : 0.f);
      const int r = (tid >> 4) + ARP * i;
      *reinterpret_cast<u2v*>(&sA[buf][r][kq]) = pack_bf16x4(u);
      if (fresh) {
        const int rr = m0 + r;
        buf_st4(rAx, (rr < M && k < K) ? (uint32_t)(rr * d.ax_ld + k) * 4u : 0xfffffff0u,
                f4{u.x, u.y, u.z, u.w});
      }
    }
#pragma unroll
    for (int i = 0; i < NBI; ++i) {
      if constexpr (BH) *reinterpret_cast<u2v*>(&sB[buf][kr0 + BKP * i][c4]) = u2v{gh[i].x, gh[i].y};
      else *reinterpret_cast<u2v*>(&sB[buf][kr0 + BKP * i][c4]) = pack_bf16x4(gb[i]);
    }
  };
  f4 acc[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  gload(0);
  // the row prologue's loads and the ReLU-mask source, behind the first slab's loads
  RowsRegs rows_x{};
  if constexpr (AX) rows_load<kXBM, NTH>(batch.rows, d, m0, rows_x);
  float hm[2][NJ][4];
  {
    constexpr uint32_t xe = ACT16 ? 2u : 4u;   // mask-source element bytes
    const rsrc_t rX = make_rsrc(d.aux, (uint32_t)(((size_t)(M - 1) * d.ldaux + N) * xe));
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + i * 16 + (lane >> 4) * 4 + r;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int col = n0 + wn + j * 16 + (lane & 15);
          const uint32_t off = row < M && col < N ? (uint32_t)(row * d.ldaux + col) * xe : 0xfffffff0u;
          hm[i][j][r] = ACT16 ? bf16_lo(buf_ld_u16(rX, off)) : buf_ld(rX, off);
        }
      }
  }
  swrite(0, 0, store_a);
  __syncthreads();
  const int nslab = (K + kXBK - 1) / kXBK;
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg = lane >> 4;
  for (int sl = 0; sl < nslab; ++sl) {
    const int cur = sl & 1;
    const int knext = (sl + 1 < nslab ? sl + 1 : sl) * kXBK;
    gload(knext);   // unconditional: the last re-reads its slab
#pragma unroll
    for (int kk = 0; kk < kXBK / 32; ++kk) {
      const int kc = kk * 32 + 8 * tg;
      bf16x8 a[2], b[NJ];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = *reinterpret_cast<const bf16x8*>(&sA[cur][wm + i * 16 + (lane & 15)][kc]);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const s4t lo = lds_tr16(&sB[cur][kc + tq][wn + j * 16 + 4 * tp]);
        const s4t hi = lds_tr16(&sB[cur][kc + tq + 4][wn + j * 16 + 4 * tp]);
        const s8t v = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        b[j] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    swrite(cur ^ 1, knext, store_a && sl + 1 < nslab);
    __syncthreads();
  }
  const bool writer = p == 0 && n0 == 0;
  if constexpr (AX) rows_finish<kXBM, NTH>(batch.rows, d, m0, writer, bid == 0, rows_x, s_q, s_coef, s_l);
  // epilogue: coefficient, ReLU-backward mask, store (k_gemm's op order)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int lr = wm + i * 16 + (lane >> 4) * 4 + r, row = m0 + lr;
      const float cf = AX ? s_coef[d.ax_slot][lr] : 1.f;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int col = n0 + wn + j * 16 + (lane & 15);
        float v = acc[i][j][r];
        if (AX) v *= cf;
        v = hm[i][j][r] > 0.f ? v : 0.f;
        if (row < M && col < N) st_big(d.C + (size_t)row * d.ldc + col, v);
      }
    }
  if constexpr (AX) rows_loss<kXBM>(batch.rows, m0, writer, s_l);
}

// whether launch_gemm may run a level on k_axk16: bf16, every desc a row-prologue dh GEMM
// (A transform, K-contiguous A, MN-contiguous 16-B aligned B, mask epilogue), no rides,
// and at least one 64x128 tile per CU
// (-1: no; 1: the row-prologue form; 0: the plain dh form)
static int axk16_ok(GemmBatch& b) {
  if (!b.bf16 || (b.ride.kind && b.ride.kind != 2)) return -1;   // (hosts the gather ride)
  const int ax = b.d[0].axk == 1 ? 1 : 0;
  if (ax != (b.rows.kind != 0 ? 1 : 0)) return -1;
  for (int i = 0; i < b.count; ++i) {
    const GemmDesc& d = b.d[i];
    if (d.axk != ax || !d.a_kc || d.b_kc || d.epi != EPI_MASK || d.bias || d.dotp || d.a_ksc ||
        d.rs_col >= 0)
      return -1;
    if (((uintptr_t)d.A & (d.a16 ? 7 : 15)) || (d.lda & 3) || ((uintptr_t)d.B & 15) || (d.ldb & 3) ||
        (ax && ((uintptr_t)d.ax_w & 15)) || (d.N & 3))
      return -1;
  }
  return assign_tiles<kXBM, kXBN>(b) >= 256 ? ax : -1;
}

// ---------------------------------------------------------------------------
// k_axk16p: the act16 batch-4096-class dh levels — k_axk16's math, dh = coef * (A W) *
// [h > 0] with A = u = [h2 > 0] w3 on the row-prologue levels (AX: L5 / L9) and A = the
// dh gradient on the plain ones (L12, model2's L5b / L9b / L11) — on k_fwd16p's multi-slab
// LDS ring: one 16-wave workgroup per CU, BM x 128 tiles, 64-deep slabs filled by LDS-DMA
// (global_load_lds_dwordx4), NST - 1 slabs in flight across raw barriers with counted
// vmcnt waits.  k_axk16 stages through registers with one slab in flight: its levels took
// ~1.6x k_fwd16p's for the same GEMM shape (config 5, round 4: L5 26 us against L4 15 us).
// Operands in the slot (the DMA image is lane-linear, so every swizzle is on the SOURCE
// address: LDS position p of row R holds the row's 16-byte chunk p ^ sw(R)):
//   A, AX: bf16 h2 rows [m][64 k] (128 B), sw = (R >> 1) & 7, read as k_fwd16p's A
//          (ds_read_b128) and transformed in registers: u = h2 > 0 ? bf16(w3[k]) : 0
//          (w3 staged in LDS once, fp32 and bf16: the bits k_axk16's staging rounds to);
//   A, !AX: fp32 gradient rows [m][64 k] (256 B), sw = R & 15, two ds_read_b128 and a
//          round to bf16 (k_axk16's pack) per fragment;
//   B: W's [k][n] rows (MN-contiguous: the layer's [out][in]), 128 bf16 columns (256 B) a
//          k row, sw = 2 (R & 3) ^ 8 ((R >> 3) & 1): conflict-free for ds_read_b64_tr_b16
//          (lane 4q + p of a 16-lane group: k row q, columns 4p..4p+3).
// The same MFMAs over the same k blocks as k_axk16 per output element: identical bits.
// AX: the column-tile-0 workgroup's wn == 0 waves also store u (fp32, ax_out) for the
// later weight gradient, as k_axk16 — those stores sit in the vmcnt count, so the counted
// waits include them.  The host runs a level here only without rides, K % 64 == 0,
// N % 8 == 0, 16-byte aligned operand rows (axk16p_plan).
#ifndef SACMI_AXK16P
#define SACMI_AXK16P 1
#endif
template <int BM, bool AX>
__host__ __device__ constexpr int axk16p_stage() { return BM * 64 * (AX ? 2 : 4) + 64 * 256; }
template <int BM, bool AX>
__host__ __device__ constexpr int axk16p_stages() { return kPLds / axk16p_stage<BM, AX>(); }

// LDS reads the compiler does not see (k_axk16p's slab reads; see there) and the tie that
// orders their consumers after an explicit lgkmcnt wait
typedef __attribute__((address_space(3))) const void lds_cvoid_t;
__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)(lds_cvoid_t*)p; }
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u4v ds_rd128(uint32_t a) {
  u4v v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
  return v;
}
__device__ __forceinline__ u2v ds_rdtr(uint32_t a) {
  u2v v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a));
  return v;
}
template <class T>
__device__ __forceinline__ void lds_tie(T& x) { asm volatile("" : "+v"(x)); }

// s_waitcnt vmcnt(ahead * PPW + sts * NS) lgkmcnt(0) for ahead < 3, sts < 4 (immediates)
template <int PPW, int NS>
__device__ __forceinline__ void axk16p_wait(int ahead, int sts) {
  switch (ahead * 4 + sts) {
    case 0: vm_wait_lgkm0<0>(); break;
    case 1: vm_wait_lgkm0<NS>(); break;
    case 2: vm_wait_lgkm0<2 * NS>(); break;
    case 3: vm_wait_lgkm0<3 * NS>(); break;
    case 4: vm_wait_lgkm0<PPW>(); break;
    case 5: vm_wait_lgkm0<PPW + NS>(); break;
    case 6: vm_wait_lgkm0<PPW + 2 * NS>(); break;
    case 7: vm_wait_lgkm0<PPW + 3 * NS>(); break;
    case 8: vm_wait_lgkm0<2 * PPW>(); break;
    case 9: vm_wait_lgkm0<2 * PPW + NS>(); break;
    case 10: vm_wait_lgkm0<2 * PPW + 2 * NS>(); break;
    default: vm_wait_lgkm0<2 * PPW + 3 * NS>(); break;
  }
}

template <int BM, bool AX>
__global__ __launch_bounds__(1024, 1) void k_axk16p(GemmBatch batch) {
  const TlMark tl_mark(batch.tl, TL_AXK16P);
  constexpr int BN = 128, BK = 64, NWV = 16, WR = 4, WC = 4;
  constexpr int MW = BM / WR, MI = MW / 16, NW = BN / WC, NT = NW / 16;
  constexpr int AROW = BK * (AX ? 2 : 4);            // bytes per A slab row
  constexpr int ABYTES = BM * AROW, STAGE = axk16p_stage<BM, AX>();
  constexpr int NST = axk16p_stages<BM, AX>();
  constexpr int APC = ABYTES / 1024, BPC = BK * 256 / 1024;   // 1 KiB pieces per slab
  constexpr int PPW = (APC + BPC) / NWV, APW = APC / NWV;
  constexpr int ALPR = AROW / 16;                     // lanes (16-byte chunks) per A row
  constexpr int NS = AX ? 2 * MI * (BK / 32) : 0;     // u stores per lane per slab
  static_assert(STAGE == ABYTES + BPC * 1024 && NST >= 3 && NST - 2 <= 2 && APC % NWV == 0 &&
                BPC % NWV == 0 && MI >= 1 && NT == 2, "k_axk16p geometry");
  // one LDS object (the ring, then w3 and the row prologue's scratch): with a second
  // __shared__ variable the compiler put a vmcnt(0) in front of the slab reads
  constexpr int XW = AX ? 512 * 4 + 512 * 2 : 0, XQ = BM * 4 * 4 + 2 * BM * 4 + BM * 2 * 4;
  __shared__ __attribute__((aligned(16))) unsigned char lds[NST * STAGE + XW + XQ];
  float* const s_w3 = reinterpret_cast<float*>(lds + NST * STAGE);
  unsigned short* const s_w3b = reinterpret_cast<unsigned short*>(lds + NST * STAGE + 512 * 4);
  auto s_q = reinterpret_cast<float (*)[4]>(lds + NST * STAGE + XW);
  auto s_coef = reinterpret_cast<float (*)[BM]>(lds + NST * STAGE + XW + BM * 16);
  auto s_l = reinterpret_cast<float (*)[2]>(lds + NST * STAGE + XW + BM * 24);
  const int bid = blockIdx.x;
  int p = 0;
  for (int q = 1; q < batch.count; ++q)
    if (bid >= batch.d[q].tile_begin) p = q;
  const GemmDesc& d = batch.d[p];
  const int t = bid - d.tile_begin;
  if (t >= d.tiles_m * d.tiles_n) return;
  int tr, tc;
  place_tile(d, t, tr, tc);
  const int m0 = tr * BM, n0 = tc * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave / WC) * MW, wn = (wave % WC) * NW;
  const int M = d.M, N = d.N, K = d.K;
  const bool store_a = AX && n0 == 0 && d.ax_out != nullptr;
  const bool stw = store_a && wn == 0;                // this wave stores u
  const rsrc_t rAx = make_rsrc(store_a ? d.ax_out : d.C,
                               store_a ? (uint32_t)(((size_t)(M - 1) * d.ax_ld + K) * 4) : 0u);
  // the row prologue's loads, the w3 vector and the ReLU-mask source go out first (oldest
  // on the vm queue: retired by the first slab's wait)
  float w3v = 0.f;
  if constexpr (AX) w3v = buf_ld(make_rsrc(d.ax_w, (uint32_t)K * 4u), (uint32_t)(tid < K ? tid : 0) * 4u);
  RowsRegs rows_x{};
  if constexpr (AX) rows_load<BM, 1024>(batch.rows, d, m0, rows_x);
  float hm[MI][NT][4];
  {
    const rsrc_t rX = make_rsrc(d.aux, (uint32_t)(((size_t)(M - 1) * d.ldaux + N) * 2));
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + i * 16 + (lane >> 4) * 4 + r;
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int col = n0 + wn + j * 16 + (lane & 15);
          const uint32_t off = row < M && col < N ? (uint32_t)(row * d.ldaux + col) * 2u : 0xfffffff0u;
          hm[i][j][r] = bf16_lo(buf_ld_u16(rX, off));
        }
      }
  }
  // DMA sources: wave w moves pieces w + 16 i (A rows first, then B k rows)
  const unsigned char* src[PPW];
  int cko[PPW];    // A: the lane's chunk byte offset in its row; B: the lane's k row in the slab
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int pc = wave + NWV * i;
    if (i < APW) {
      const int R = pc * (1024 / AROW) + lane / ALPR, pos = lane % ALPR;
      const int c = AX ? (pos ^ ((R >> 1) & 7)) : (pos ^ (R & 15));
      const int ra = min(m0 + R, M - 1);
      src[i] = reinterpret_cast<const unsigned char*>(d.A) + (size_t)ra * d.lda * (AX ? 2 : 4);
      cko[i] = c * 16;
    } else {
      const int R = (pc - APC) * 4 + (lane >> 4), pos = lane & 15;
      const int c = pos ^ (((R & 3) << 1) ^ (((R >> 3) & 1) << 3));
      const int n = min(n0 + 8 * c, N - 8);          // (N % 8 == 0: a chunk is all in or out)
      src[i] = reinterpret_cast<const unsigned char*>(d.Bh) + (size_t)n * 2;
      cko[i] = R;
    }
  }
  auto issue = [&](int sl) {                          // slab sl into ring slot sl % NST
    unsigned char* dst = lds + (sl % NST) * STAGE;
    const int k0 = sl * BK;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = wave + NWV * i;
      const unsigned char* g = i < APW ? src[i] + (size_t)k0 * (AX ? 2 : 4) + cko[i]
                                       : src[i] + (size_t)min(k0 + cko[i], K - 1) * d.ldb * 2;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)(dst + pc * 1024), 16, 0, 0);
    }
  };
  f4 acc[MI][NT];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const int nslab = K / BK;
#pragma unroll
  for (int s2 = 0; s2 < NST - 1; ++s2)
    if (s2 < nslab) issue(s2);
  if constexpr (AX) {   // (read after the first slab's barrier; asm stores: see ds_rd128)
    if (tid < K) {
      const uint32_t wb16 = __builtin_bit_cast(unsigned short, (__bf16)w3v);
      asm volatile("ds_write_b32 %0, %1" :: "v"(lds_addr(&s_w3[tid])), "v"(w3v) : "memory");
      asm volatile("ds_write_b16 %0, %1" :: "v"(lds_addr(&s_w3b[tid])), "v"(wb16) : "memory");
    }
  }
  const int r16 = lane & 15, tq = r16 >> 2, tp = lane & 3, tg = lane >> 4;
  for (int sl = 0; sl < nslab; ++sl) {
    // retire slab sl only: younger are the slabs already issued past it and the u stores
    // of the iterations since it was issued
    const int ahead = min(NST - 2, nslab - 1 - sl);
    axk16p_wait<PPW, NS>(ahead, stw ? min(sl, NST - 1) : 0);
    __builtin_amdgcn_s_barrier();                     // every wave's slab sl landed; slot (sl-1) free
    asm volatile("" ::: "memory");
    if (sl + NST - 1 < nslab) issue(sl + NST - 1);
    const unsigned char* st = lds + (sl % NST) * STAGE;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int kb = sl * BK + kk * 32 + 8 * tg;      // this lane's 8 k of the A fragment
      // every LDS read here is inline asm (ds_rd128 / ds_rdtr): a compiler-visible LDS read
      // after the slab's global_load_lds got a vmcnt(0) from the compiler (waiting for the
      // slabs just issued as well); the lgkmcnt wait is ours (lds_tie)
      u4v ar[MI][AX ? 1 : 2], wb{}, w0{}, w1{};
      u2v blo[NT], bhi[NT];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int r = wm + i * 16 + r16;
        if constexpr (AX) {
          const int c = kk * 4 + tg;
          ar[i][0] = ds_rd128(lds_addr(st + r * AROW + ((c ^ ((r >> 1) & 7)) << 4)));
        } else {
          const int c = kk * 8 + 2 * tg;
          ar[i][0] = ds_rd128(lds_addr(st + r * AROW + ((c ^ (r & 15)) << 4)));
          ar[i][1] = ds_rd128(lds_addr(st + r * AROW + (((c + 1) ^ (r & 15)) << 4)));
        }
      }
      if constexpr (AX) {
        wb = ds_rd128(lds_addr(&s_w3b[kb]));
        if (stw) {
          w0 = ds_rd128(lds_addr(&s_w3[kb]));
          w1 = ds_rd128(lds_addr(&s_w3[kb + 4]));
        }
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int cb = (wn + j * 16 + 4 * tp) >> 3, half = (tp & 1) * 8;
        const int k0r = kk * 32 + 8 * tg + tq, k1r = k0r + 4;
        const int p0 = cb ^ (((k0r & 3) << 1) ^ (((k0r >> 3) & 1) << 3));
        const int p1 = cb ^ (((k1r & 3) << 1) ^ (((k1r >> 3) & 1) << 3));
        blo[j] = ds_rdtr(lds_addr(st + ABYTES + k0r * 256 + (p0 << 4) + half));
        bhi[j] = ds_rdtr(lds_addr(st + ABYTES + k1r * 256 + (p1 << 4) + half));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int h = 0; h < (AX ? 1 : 2); ++h) lds_tie(ar[i][h]);
      lds_tie(wb); lds_tie(w0); lds_tie(w1);
#pragma unroll
      for (int j = 0; j < NT; ++j) { lds_tie(blo[j]); lds_tie(bhi[j]); }
      bf16x8 a[MI], b[NT];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        if constexpr (AX) {
          const u4v h = ar[i][0];
          auto sel = [](uint32_t hv, uint32_t wv) {   // per bf16 half: h > 0 ? w : 0
            return (bf16_lo(hv) > 0.f ? wv & 0xffffu : 0u) | (bf16_hi(hv) > 0.f ? wv & 0xffff0000u : 0u);
          };
          const uint4 u = {sel(h.x, wb.x), sel(h.y, wb.y), sel(h.z, wb.z), sel(h.w, wb.w)};
          a[i] = __builtin_bit_cast(bf16x8, u);
          if (stw) {   // u rows (fp32) for the weight gradient
            const float4 f0 = __builtin_bit_cast(float4, w0), f1 = __builtin_bit_cast(float4, w1);
            const int rr = m0 + wm + i * 16 + r16;
            const uint32_t o = rr < M ? (uint32_t)(rr * d.ax_ld + kb) * 4u : 0xfffffff0u;
            buf_st4(rAx, o, f4{bf16_lo(h.x) > 0.f ? f0.x : 0.f, bf16_hi(h.x) > 0.f ? f0.y : 0.f,
                               bf16_lo(h.y) > 0.f ? f0.z : 0.f, bf16_hi(h.y) > 0.f ? f0.w : 0.f});
            buf_st4(rAx, rr < M ? o + 16u : 0xfffffff0u,
                    f4{bf16_lo(h.z) > 0.f ? f1.x : 0.f, bf16_hi(h.z) > 0.f ? f1.y : 0.f,
                       bf16_lo(h.w) > 0.f ? f1.z : 0.f, bf16_hi(h.w) > 0.f ? f1.w : 0.f});
          }
        } else {
          const u2v lo = pack_bf16x4(__builtin_bit_cast(float4, ar[i][0]));
          const u2v hi = pack_bf16x4(__builtin_bit_cast(float4, ar[i][1]));
          const uint4 u = {lo.x, lo.y, hi.x, hi.y};
          a[i] = __builtin_bit_cast(bf16x8, u);
        }
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const uint4 v = {blo[j].x, blo[j].y, bhi[j].x, bhi[j].y};
        b[j] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  const bool writer = p == 0 && n0 == 0;
  if constexpr (AX) rows_finish<BM, 1024>(batch.rows, d, m0, writer, bid == 0, rows_x, s_q, s_coef, s_l);
  // epilogue: coefficient, ReLU-backward mask, store (k_axk16's op order)
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int lr = wm + i * 16 + (lane >> 4) * 4 + r, row = m0 + lr;
      const float cf = AX ? s_coef[d.ax_slot][lr] : 1.f;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int col = n0 + wn + j * 16 + (lane & 15);
        float v = acc[i][j][r];
        if (AX) v *= cf;
        v = hm[i][j][r] > 0.f ? v : 0.f;
        if (row < M && col < N) st_big(d.C + (size_t)row * d.ldc + col, v);
      }
    }
  if constexpr (AX) rows_loss<BM>(batch.rows, m0, writer, s_l);
}

// whether an act16 k_axk16 level (axk16_ok form `ax`) can run on k_axk16p, and its row tile
// (0: no): bf16 weight shadows, no rides, K % 64 == 0, N % 8 == 0, 16-byte operand rows,
// one workgroup per CU at least
// Opt-in (SACMI_AXK16P=1, read per enqueue): bit-identical to k_axk16 but measured slower
// (config 5, same box, alternating: L5 29.4 vs 26.3 us, L9 25.4 vs 23.2, 3,204 vs 3,268
// updates/s — profiles/r05/axk16p_ab): the dh levels are not bound by their K loop (the
// register-staged and the ring kernel take about the same time for the same tiles) but by
// what surrounds it — 32 MB of fp32 dh and u rows written per critic level
static int axk16p_plan(GemmBatch& b, int ax) {
  if (!SACMI_AXK16P || b.ride.kind || b.ride.pk_blocks) return 0;
  const char* e = std::getenv("SACMI_AXK16P");
  if (!e || std::atoi(e) == 0) return 0;
  for (int i = 0; i < b.count; ++i) {
    const GemmDesc& d = b.d[i];
    if (!d.Bh || !d.x16 || (d.K % 64) || d.K > 512 || (d.N % 8) || d.N < 8) return 0;
    if (((uintptr_t)d.A & 15) || ((uintptr_t)d.Bh & 15) || (d.ldb & 7)) return 0;
    if (ax ? (!d.a16 || (d.lda & 7) || ((uintptr_t)d.ax_w & 15) || (d.ax_out && ((d.ax_ld & 3) || ((uintptr_t)d.ax_out & 15))))
           : (d.a16 || (d.lda & 3)))
      return 0;
  }
  GemmBatch t = b;   // (b keeps k_axk16's tiles unless this kernel takes the level)
  if (assign_tiles<128, 128>(t) >= 256) { b = t; return 128; }
  t = b;
  if (!ax && assign_tiles<64, 128>(t) >= 256) { b = t; return 64; }
  return 0;
}

// NSL: the partial loads each thread issues (= ns where instantiated, else kDwMaxSplit with
// the loads past ns at an out-of-range offset): no VMEM issue slots for absent splits
template <int NSL>
__global__ __launch_bounds__(256) void k_dw_fin(GemmBatch batch, int ns, int64_t ws_stride) {
  const TlMark tl_mark(batch.tl, TL_DW_FIN);
  __shared__ AdamScalars s_k[3];
  __shared__ int s_err;
  const AdamFuse& af = batch.adam;
  const bool adam = batch.has_adam != 0;
  if (adam && threadIdx.x < 3) s_k[threadIdx.x] = fuse_scalars(af, threadIdx.x, af.step_offset);
  if (threadIdx.x == 0) s_err = adam ? af.sc->err : 0;
  __syncthreads();
  // a non-finite policy sample / PER draw of this update (ErrBits, see k_gemm)
  const bool void_st = (s_err & af.err_skip) != 0;
  const float omb1 = 1.f - af.beta1, omb2 = 1.f - af.beta2, omtau = 1.f - af.tau;
  // kDwFinEpt 4-column groups per thread (group g = block base + k * 256 + thread: 16-byte
  // loads and stores of the partials and of the optimizer state, coalesced), the workgroups
  // dealt to the descs in order: every workgroup belongs to one desc, and every load of a
  // thread's groups (partials, parameter, moments, target) is issued before any use — one
  // round trip, and all of the level's threads resident at once
  int q = -1, bstart = 0, acc = 0;
  int64_t off = 0;
  for (int qq = 0; qq < batch.count; ++qq) {
    const int n_el_q = batch.d[qq].M * dw_ncols(batch.d[qq]);
    const int nb = (n_el_q / 4 + 256 * kDwFinEpt - 1) / (256 * kDwFinEpt);
    if (q < 0 && (int)blockIdx.x < acc + nb) { q = qq; bstart = acc; }
    if (q < 0) off += n_el_q;
    acc += nb;
  }
  if (q >= 0 && !void_st) {
    const GemmDesc& d = batch.d[q];
    const int nc = dw_ncols(d), ncr = dw_ncols_real(d), gpr = nc / 4;
    const int n_gr = d.M * gpr;                 // 4-column groups (n_el < 2^31: dw_split_plan)
    const bool pol = d.epi == EPI_ADAM_POLYAK;
    const bool pol_st = pol && (s_err & af.err_nopolyak) == 0;
    const int64_t abase = adam ? (int64_t)(d.C - af.P) : 0;
    const float* wsd = batch.ws + off;
    const bool wt = batch.st_wt != 0;            // write-through parameter / state stores
    const uint32_t oob = 0xfffffff0u;
    const rsrc_t rWs = make_rsrc(wsd, (uint32_t)(((int64_t)(ns - 1) * ws_stride + (int64_t)n_gr * 4) * 4));
    const rsrc_t rTg = make_rsrc(adam && pol ? af.T + abase - af.t_base : wsd, adam && pol ? 0x7fffffffu : 0u);
    const rsrc_t rC = make_rsrc(d.C, 0x7fffffffu);
    const rsrc_t rM = make_rsrc(adam ? af.M + abase : d.C, adam ? 0x7fffffffu : 0u);
    const rsrc_t rV = make_rsrc(adam ? af.V + abase : d.C, adam ? 0x7fffffffu : 0u);
    const rsrc_t rG = make_rsrc(adam && af.G ? af.G + abase : d.C, adam && af.G ? 0x7fffffffu : 0u);
    const rsrc_t rT = make_rsrc(adam && pol ? af.T + abase - af.t_base : d.C, adam && pol ? 0x7fffffffu : 0u);
    int g[kDwFinEpt], c4[kDwFinEpt];
    uint32_t o[kDwFinEpt];
    float4 t[kDwFinEpt][NSL], pp[kDwFinEpt], mm[kDwFinEpt], vv[kDwFinEpt], tt[kDwFinEpt];
#pragma unroll
    for (int k = 0; k < kDwFinEpt; ++k) {
      g[k] = (blockIdx.x - bstart) * (256 * kDwFinEpt) + k * 256 + threadIdx.x;
      const bool live = g[k] < n_gr;
      const int row = g[k] / gpr;
      c4[k] = (g[k] - row * gpr) * 4;
      o[k] = (uint32_t)(row * d.ldc + c4[k]) * 4u;
      // all partial loads in flight at once (offsets past NS / past the desc return 0, no
      // access): no guard, so nothing drains the load queue between them
#pragma unroll
      for (int sp = 0; sp < NSL; ++sp)
        t[k][sp] = buf_ld4(rWs, live && sp < ns ? (uint32_t)((int64_t)sp * ws_stride + (int64_t)g[k] * 4) * 4u : oob);
      pp[k] = buf_ld4(rC, adam && live ? o[k] : oob);
      mm[k] = buf_ld4(rM, live ? o[k] : oob);
      vv[k] = buf_ld4(rV, live ? o[k] : oob);
      tt[k] = buf_ld4(rTg, pol && live ? o[k] : oob);
    }
#pragma unroll
    for (int k = 0; k < kDwFinEpt; ++k) {
      if (g[k] >= n_gr) continue;
      // the partial sums in split order; a column past the output (the pad of the last
      // group of a row) takes gradient 0: Adam / Polyak leave its zero parameter, moments
      // and target exactly 0, and the 16-byte stores rewrite them
      float v[4] = {t[k][0].x, t[k][0].y, t[k][0].z, t[k][0].w};
#pragma unroll
      for (int sp = 1; sp < NSL; ++sp)
        if (sp < ns) {
#pragma clang fp contract(off)
          v[0] += t[k][sp].x; v[1] += t[k][sp].y; v[2] += t[k][sp].z; v[3] += t[k][sp].w;
        }
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = c4[k] + j < ncr ? v[j] : 0.f;
      auto st4 = [&](rsrc_t r, float a0, float a1, float a2, float a3) {
        if (wt) buf_st4<kStAux>(r, o[k], f4{a0, a1, a2, a3});
        else buf_st4<0>(r, o[k], f4{a0, a1, a2, a3});
      };
      if (adam) {
        float p4[4] = {pp[k].x, pp[k].y, pp[k].z, pp[k].w}, m4[4] = {mm[k].x, mm[k].y, mm[k].z, mm[k].w};
        float v4[4] = {vv[k].x, vv[k].y, vv[k].z, vv[k].w}, t4[4] = {tt[k].x, tt[k].y, tt[k].z, tt[k].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          adam_elem(p4[j], m4[j], v4[j], v[j], omb1, af.beta2, omb2, af.eps, s_k[d.adam_step]);
          t4[j] = polyak(t4[j], p4[j], omtau, af.tau);
        }
        if (af.G) st4(rG, v[0], v[1], v[2], v[3]);
        st4(rC, p4[0], p4[1], p4[2], p4[3]);
        st4(rM, m4[0], m4[1], m4[2], m4[3]);
        st4(rV, v4[0], v4[1], v4[2], v4[3]);
        auto st_bf4 = [&](unsigned short* h, const float (&x)[4]) {   // 4 bf16 shadows, 8 bytes
          const uint32_t lo = (uint32_t)bf16_bits(x[0]) | ((uint32_t)bf16_bits(x[1]) << 16);
          const uint32_t hi = (uint32_t)bf16_bits(x[2]) | ((uint32_t)bf16_bits(x[3]) << 16);
          if (wt) st_wt8(h, 0u, lo, hi);
          else *reinterpret_cast<uint2*>(h) = make_uint2(lo, hi);
        };
        if (af.Ph) st_bf4(af.Ph + abase + o[k] / 4u, p4);
        if (pol_st) {
          st4(rT, t4[0], t4[1], t4[2], t4[3]);
          if (af.Th) st_bf4(af.Th + abase - af.t_base + o[k] / 4u, t4);
        }
      } else {
        st4(rC, v[0], v[1], v[2], v[3]);
      }
    }
  }
  if (adam && blockIdx.x == 0) adam_block0(af, s_err, omb1, omb2);
  store_err_flags(batch);
}

// k_dw_fin, pipelined (opt-in, SACMI_DWFIN_P=1 — measured slower: config 5 L6 65.8 vs 63.4 us,
// L13 42.0 vs 40.5, 3,213 vs 3,246 updates/s, profiles/r05/dwfin_p_ab): the same
// per-group arithmetic over the same virtual blocks (256 four-column groups each, dealt to
// the descs in order), but on a grid of at most kDwFinGrid workgroups that loop over them —
// the next block's loads (partials, parameter, moments, target) are issued before this
// block's stores, so the level's reads and writes overlap instead of running as one read
// phase then one write phase across the whole chip (k_dw_fin: ~2.5-2.7 TB/s at config 5,
// profiles/r05/pmc_c5.json).  Identical bits: each group's sums and updates are k_dw_fin's.
#ifndef SACMI_DWFIN_GRID
#define SACMI_DWFIN_GRID 768      // (3 resident per CU at the 11-split form's 138 VGPRs)
#endif
constexpr int kDwFinGrid = SACMI_DWFIN_GRID;

template <int NSL>
__global__ __launch_bounds__(256) void k_dw_fin_p(GemmBatch batch, int ns, int64_t ws_stride, int nvb) {
  const TlMark tl_mark(batch.tl, TL_DW_FIN_P);
  __shared__ AdamScalars s_k[3];
  __shared__ int s_err;
  const AdamFuse& af = batch.adam;
  const bool adam = batch.has_adam != 0;
  if (adam && threadIdx.x < 3) s_k[threadIdx.x] = fuse_scalars(af, threadIdx.x, af.step_offset);
  if (threadIdx.x == 0) s_err = adam ? af.sc->err : 0;
  __syncthreads();
  const bool void_st = (s_err & af.err_skip) != 0;   // (see k_dw_fin)
  const float omb1 = 1.f - af.beta1, omb2 = 1.f - af.beta2, omtau = 1.f - af.tau;
  const bool wt = batch.st_wt != 0;
  const uint32_t oob = 0xfffffff0u;
  // virtual block vb -> its desc q, the desc's first block and its partial-row offset
  auto locate = [&](int vb, int& q, int& bstart, int64_t& off) {
    q = batch.count - 1; bstart = 0; off = 0;
    int acc = 0;
    bool found = false;
    int64_t o = 0;
    for (int qq = 0; qq < batch.count; ++qq) {
      const int n_el_q = batch.d[qq].M * dw_ncols(batch.d[qq]);
      const int nb = (n_el_q / 4 + 255) / 256;
      if (!found && vb < acc + nb) { q = qq; bstart = acc; off = o; found = true; }
      o += n_el_q;
      acc += nb;
    }
  };
  struct Ld {
    float4 t[NSL], pp, mm, vv, tt;
  };
  // every load of one block's group, at once; a block past the level (vb >= nvb) or a group
  // past its desc reads at out-of-range offsets (no access)
  auto load = [&](int vb, Ld& L) {
    int q, bstart;
    int64_t off;
    locate(vb < nvb ? vb : 0, q, bstart, off);
    const GemmDesc& d = batch.d[q];
    const int nc = dw_ncols(d), gpr = nc / 4, n_gr = d.M * gpr;
    const int g = (vb - bstart) * 256 + threadIdx.x;
    const bool live = vb < nvb && g < n_gr;
    const int row = live ? g / gpr : 0, c4 = live ? (g - row * gpr) * 4 : 0;
    const uint32_t o = (uint32_t)(row * d.ldc + c4) * 4u;
    const bool pol = d.epi == EPI_ADAM_POLYAK;
    const int64_t abase = adam ? (int64_t)(d.C - af.P) : 0;
    const float* wsd = batch.ws + off;
    const rsrc_t rWs = make_rsrc(wsd, (uint32_t)(((int64_t)(ns - 1) * ws_stride + (int64_t)n_gr * 4) * 4));
    const rsrc_t rTg = make_rsrc(adam && pol ? af.T + abase - af.t_base : wsd, adam && pol ? 0x7fffffffu : 0u);
    const rsrc_t rC = make_rsrc(d.C, 0x7fffffffu);
    const rsrc_t rM = make_rsrc(adam ? af.M + abase : d.C, adam ? 0x7fffffffu : 0u);
    const rsrc_t rV = make_rsrc(adam ? af.V + abase : d.C, adam ? 0x7fffffffu : 0u);
#pragma unroll
    for (int sp = 0; sp < NSL; ++sp)
      L.t[sp] = buf_ld4(rWs, live && sp < ns ? (uint32_t)((int64_t)sp * ws_stride + (int64_t)g * 4) * 4u : oob);
    L.pp = buf_ld4(rC, adam && live ? o : oob);
    L.mm = buf_ld4(rM, live ? o : oob);
    L.vv = buf_ld4(rV, live ? o : oob);
    L.tt = buf_ld4(rTg, pol && live ? o : oob);
  };
  // k_dw_fin's arithmetic and stores for one block's group
  auto finish = [&](int vb, const Ld& L) {
    int q, bstart;
    int64_t off;
    locate(vb, q, bstart, off);
    const GemmDesc& d = batch.d[q];
    const int nc = dw_ncols(d), ncr = dw_ncols_real(d), gpr = nc / 4, n_gr = d.M * gpr;
    const int g = (vb - bstart) * 256 + threadIdx.x;
    if (g >= n_gr) return;
    const int row = g / gpr, c4 = (g - row * gpr) * 4;
    const uint32_t o = (uint32_t)(row * d.ldc + c4) * 4u;
    const bool pol = d.epi == EPI_ADAM_POLYAK;
    const bool pol_st = pol && (s_err & af.err_nopolyak) == 0;
    const int64_t abase = adam ? (int64_t)(d.C - af.P) : 0;
    const rsrc_t rC = make_rsrc(d.C, 0x7fffffffu);
    const rsrc_t rM = make_rsrc(adam ? af.M + abase : d.C, adam ? 0x7fffffffu : 0u);
    const rsrc_t rV = make_rsrc(adam ? af.V + abase : d.C, adam ? 0x7fffffffu : 0u);
    const rsrc_t rG = make_rsrc(adam && af.G ? af.G + abase : d.C, adam && af.G ? 0x7fffffffu : 0u);
    const rsrc_t rT = make_rsrc(adam && pol ? af.T + abase - af.t_base : d.C, adam && pol ? 0x7fffffffu : 0u);
    float v[4] = {L.t[0].x, L.t[0].y, L.t[0].z, L.t[0].w};
#pragma unroll
    for (int sp = 1; sp < NSL; ++sp)
      if (sp < ns) {
#pragma clang fp contract(off)
        v[0] += L.t[sp].x; v[1] += L.t[sp].y; v[2] += L.t[sp].z; v[3] += L.t[sp].w;
      }
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = c4 + j < ncr ? v[j] : 0.f;
    auto st4 = [&](rsrc_t r, float a0, float a1, float a2, float a3) {
      if (wt) buf_st4<kStAux>(r, o, f4{a0, a1, a2, a3});
      else buf_st4<0>(r, o, f4{a0, a1, a2, a3});
    };
    if (adam) {
      float p4[4] = {L.pp.x, L.pp.y, L.pp.z, L.pp.w}, m4[4] = {L.mm.x, L.mm.y, L.mm.z, L.mm.w};
      float v4[4] = {L.vv.x, L.vv.y, L.vv.z, L.vv.w}, t4[4] = {L.tt.x, L.tt.y, L.tt.z, L.tt.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        adam_elem(p4[j], m4[j], v4[j], v[j], omb1, af.beta2, omb2, af.eps, s_k[d.adam_step]);
        t4[j] = polyak(t4[j], p4[j], omtau, af.tau);
      }
      if (af.G) st4(rG, v[0], v[1], v[2], v[3]);
      st4(rC, p4[0], p4[1], p4[2], p4[3]);
      st4(rM, m4[0], m4[1], m4[2], m4[3]);
      st4(rV, v4[0], v4[1], v4[2], v4[3]);
      auto st_bf4 = [&](unsigned short* h, const float (&x)[4]) {   // 4 bf16 shadows, 8 bytes
        const uint32_t lo = (uint32_t)bf16_bits(x[0]) | ((uint32_t)bf16_bits(x[1]) << 16);
        const uint32_t hi = (uint32_t)bf16_bits(x[2]) | ((uint32_t)bf16_bits(x[3]) << 16);
        if (wt) st_wt8(h, 0u, lo, hi);
        else *reinterpret_cast<uint2*>(h) = make_uint2(lo, hi);
      };
      if (af.Ph) st_bf4(af.Ph + abase + o / 4u, p4);
      if (pol_st) {
        st4(rT, t4[0], t4[1], t4[2], t4[3]);
        if (af.Th) st_bf4(af.Th + abase - af.t_base + o / 4u, t4);
      }
    } else {
      st4(rC, v[0], v[1], v[2], v[3]);
    }
  };
  if (!void_st) {
    Ld cur, nxt;
    int vb = blockIdx.x;
    load(vb, cur);
    for (; vb < nvb; vb += gridDim.x) {
      load(vb + gridDim.x, nxt);   // (past the level: out-of-range, no access)
      finish(vb, cur);
      cur = nxt;
    }
  }
  if (adam && blockIdx.x == 0) adam_block0(af, s_err, omb1, omb2);
  store_err_flags(batch);
}

// 1 when the level carries bf16 activation operands (any GemmDesc a16 / b16 / c16 / x16);
// each kernel that takes them checks the per-desc pattern it supports
static int level_act16(const GemmBatch& b) {
  int any = 0;
  for (int i = 0; i < b.count; ++i) any |= b.d[i].a16 | b.d[i].b16 | b.d[i].c16 | b.d[i].x16;
  return any ? 1 : 0;
}

// bf16 deep-K weight-gradient levels: split count and workspace need, or 0 (old path)
static int dw_split_plan(GemmBatch& b, int64_t* stride) {
  // (rides: the gather on any split-K kernel, the sampler on k_dw_part16 only)
  if ((!b.bf16 && !SACMI_DW_SPLIT_FP32) || !b.ws || (b.ride.kind == 1 && !(b.bf16 && SACMI_DW_LDS16)))
    return 0;
  int64_t el = 0;
  int tiles = 0;
  for (int i = 0; i < b.count; ++i) {
    GemmDesc& d = b.d[i];
    if (d.a_kc || d.b_kc || d.K < 2048) return 0;
    if (d.axk && !(d.axk == 2 && b.bf16 && SACMI_DW_LDS16)) return 0;   // (axk 2: k_dw_part16 only)
    if (d.epi != EPI_STORE && d.epi < EPI_ADAM) return 0;
    // k_dw_fin's 4-column groups: the row-sum column is the bias column right after the
    // last output column, and output rows (and their Adam state) are 16-byte aligned with
    // room for a whole last group
    if ((d.rs_col >= 0 && d.rs_col != d.N) || (d.ldc & 3) || ((uintptr_t)d.C & 15) ||
        d.ldc < dw_ncols(d))
      return 0;
    if (d.epi >= EPI_ADAM && (((d.C - b.adam.P) & 3) || (b.adam.T && ((d.C - b.adam.P - b.adam.t_base) & 3))))
      return 0;
    d.tiles_m = (d.M + kDBM - 1) / kDBM;
    d.tiles_n = (d.N + kDBN - 1) / kDBN;
    d.tile_begin = tiles;
    tiles += d.tiles_m * d.tiles_n;
    el += (int64_t)d.M * dw_ncols(d);
  }
  b.total_tiles = tiles;
  if (el >= (1LL << 31)) return 0;
  // as many K splits as fit in one pass over the chip's workgroup slots (2 per CU at
  // 67 KB of LDS each): a partial second pass costs a whole slab loop (config 5: a
  // 528-workgroup L6 took 96 us, 440 workgroups 82 us)
  static const int target = std::getenv("SACMI_DW_TARGET") ? std::atoi(std::getenv("SACMI_DW_TARGET")) : SACMI_DW_TARGET;
  int ns = target / tiles;
  ns = ns < 1 ? 1 : ns > kDwMaxSplit ? kDwMaxSplit : ns;
  if ((int64_t)ns * el > b.ws_floats) return 0;
  *stride = el;
  return ns;
}

// whether launch_gemm may run a level on k_fwd: plain forward GEMMs (both operands
// K-contiguous, store / ReLU epilogue, optional bias and dot partials), no prologue,
// no rides, and enough 128x128 tiles to fill the chip
static bool fwd_big_ok(GemmBatch& b) {
  // bf16 only: with fp32 operands the 512-thread K-split tiles measured faster (config 3:
  // 1,351 vs 1,229 updates/s); with bf16 MFMAs the levels are operand-traffic bound and
  // the LDS sharing wins (config 5: 1,381 -> 1,458)
  if (b.ride.kind || (!b.bf16 && !SACMI_FWD_BIG_FP32)) return false;
  for (int i = 0; i < b.count; ++i) {
    const GemmDesc& d = b.d[i];
    if (!d.a_kc || !d.b_kc || d.axk || d.a_ksc || d.rs_col >= 0) return false;
    if (((uintptr_t)d.A & (d.a16 ? 7 : 15)) || (d.lda & 3) || ((uintptr_t)d.B & 15) || (d.ldb & 3)) return false;
    if (d.epi != EPI_RELU && d.epi != EPI_STORE) return false;
    if (d.dotp && (d.N % 32)) return false;
  }
  // 128-column tiles when they give two workgroups per CU, else 64-column ones
  if (b.bf16 && (!SACMI_FWD_BF16_N64 || (assign_tiles<kFBM, 128>(b) >= 512 && !SACMI_FWD_BF16_ALL64)))
    return assign_tiles<kFBM, 128>(b) >= 256 * SACMI_FWD_BIG_MIN;
  return assign_tiles<kFBM, 64>(b) >= 512 * SACMI_FWD_BIG_MIN;
}

// one configuration, fp32 or bf16 MFMA operands (1024 threads)
template <int TM, int TN, int KSPLIT, int G, int MG, bool ADAM, int AXK>
static void launch_k(const GemmBatch& b, int grid, hipStream_t s) {
  const dim3 blk(64 * KSPLIT * MG);
  if (b.bf16) hipLaunchKernelGGL((k_gemm<TM, TN, KSPLIT, G, MG, ADAM, AXK, true>), dim3(grid), blk, 0, s, b);
  else hipLaunchKernelGGL((k_gemm<TM, TN, KSPLIT, G, MG, ADAM, AXK, false>), dim3(grid), blk, 0, s, b);
}

// the LDS-staged core (CORE 1), 1024 threads
template <int TM, int TN, int KSP, int MG, bool ADAM, int AXK>
static void launch_ks(const GemmBatch& b, int grid, hipStream_t s) {
  hipLaunchKernelGGL((k_gemm<TM, TN, KSP, 1, MG, ADAM, AXK, false, 1>), dim3(grid), dim3(1024), 0, s, b);
}

// whether a level can take the staged core: fp32 operands, 16-byte-aligned rows, every
// 16-byte chunk a DMA lane reads inside its row (KC: ld >= round4(K); MN: ld >= round4(M|N)),
// and the K vector it stages (ax_w / a_ksc) within kStgKW
#ifndef SACMI_STAGED
#define SACMI_STAGED 0
#endif
static bool staged_ok(const GemmBatch& b) {
  // $SACMI_STAGED=0/1 overrides the build default; SACMI_NO_STAGED forces it off
  static const bool env = std::getenv("SACMI_NO_STAGED") == nullptr &&
                          (std::getenv("SACMI_STAGED") ? std::atoi(std::getenv("SACMI_STAGED")) != 0 : SACMI_STAGED != 0);
  if (!env || b.bf16) return false;
  for (int i = 0; i < b.count; ++i) {
    const GemmDesc& d = b.d[i];
    if (d.a16 || d.b16 || d.c16 || d.x16) return false;
    if (d.K < 1 || d.K > kStgKW || d.M < 1 || d.N < 1) return false;
    if (((uintptr_t)d.A & 15) || ((uintptr_t)d.B & 15) || (d.lda & 3) || (d.ldb & 3)) return false;
    if (d.lda < round_up(d.a_kc ? d.K : d.M, 4) || d.ldb < round_up(d.b_kc ? d.K : d.N, 4)) return false;
  }
  return true;
}

// every desc's B operand has a bf16 shadow (SACMI_BF16_SHADOW 0: never read them)
#ifndef SACMI_BF16_SHADOW
#define SACMI_BF16_SHADOW 1
#endif
static bool all_bh(const GemmBatch& b) {
  if (!SACMI_BF16_SHADOW) return false;
  for (int i = 0; i < b.count; ++i)
    if (!b.d[i].Bh) return false;
  return true;
}

void launch_gemm(const GemmBatch& b0, hipStream_t s) {
  if (b0.count == 0) return;
  if (b0.heads_ticket && !gemm_level_heads_fold_ok(b0, b0.heads.A))
    throw Error{SACMI_ESTATE, "policy heads folded into a level outside k_gemm's 32x64 forward tiles"};
  GemmBatch b = b0;
  // Polyak rides (RideAlong::pk) run on k_gemm's 1024-thread configurations only: a level
  // that goes to a split-K / LDS-staged kernel must not carry them
  const Error pk_err{SACMI_ESTATE, "Polyak ride on a level outside k_gemm"};
  {
    int64_t stride = 0;
    const int ns = SACMI_DW_SPLIT ? dw_split_plan(b, &stride) : 0;
    if (ns > 0) {
      if (b.ride.pk_blocks) throw pk_err;
      const int ride = b.ride.kind ? b.ride.nblocks : 0;
      if (b.ride.kind == 1 &&
          mt_sample_lds_words(b.ride.tbl_log2, b.ride.mt.setsize) * 4 > (size_t)kDw16LdsBytes)
        throw Error{SACMI_ESTATE, "ride-along sampler table exceeds k_dw_part16's LDS"};
      const int grid = dw_grid_tiles(b.total_tiles, ns) + ride;
      const int form = level_act16(b);   // act16: every X operand bf16
      for (int i = 0; i < b.count; ++i)
        if ((b.d[i].a16 && b.d[i].axk != 2) || b.d[i].c16 || b.d[i].x16 || (form && !b.d[i].b16) || form < 0)
          throw Error{SACMI_ESTATE, "split-K weight gradient: unsupported bf16 activation operand"};
      if (form && !(b.bf16 && SACMI_DW_LDS16))
        throw Error{SACMI_ESTATE, "bf16 activation operands need k_dw_part16"};
      bool axt = false;
      for (int i = 0; i < b.count; ++i) axt = axt || b.d[i].axk == 2;
      if (axt && !(b.bf16 && SACMI_DW_LDS16 && form))
        throw Error{SACMI_ESTATE, "dW A transform (axk 2) needs k_dw_part16 with bf16 X operands"};
      if (b.bf16 && SACMI_DW_LDS16 && form && axt) hipLaunchKernelGGL((k_dw_part16<true, true>), dim3(grid), dim3(64 * kDw16Waves), 0, s, b, ns, stride);
      else if (b.bf16 && SACMI_DW_LDS16 && form) hipLaunchKernelGGL(k_dw_part16<true>, dim3(grid), dim3(64 * kDw16Waves), 0, s, b, ns, stride);
      else if (b.bf16 && SACMI_DW_LDS16) hipLaunchKernelGGL(k_dw_part16<false>, dim3(grid), dim3(64 * kDw16Waves), 0, s, b, ns, stride);
      else if (b.bf16) hipLaunchKernelGGL(k_dw_part<true>, dim3(grid), dim3(256), 0, s, b, ns, stride);
      else hipLaunchKernelGGL(k_dw_part<false>, dim3(grid), dim3(256), 0, s, b, ns, stride);
      HIP_LAUNCH_CHECK();
      int fin_grid = 0;                    // k_dw_fin: kDwFinEpt 4-column groups per thread, per desc
      for (int i = 0; i < b.count; ++i)
        fin_grid += (b.d[i].M * (dw_ncols(b.d[i]) / 4) + 256 * kDwFinEpt - 1) / (256 * kDwFinEpt);
      if (b.tl) b.tl += kTlWords;          // the second kernel of the level
      const dim3 fg(fin_grid), fb(256);
      // the fin's stores: plain (SACMI_FIN_WT=1: write-through, measured slower at config 5:
      // 3,412 -> 3,357 updates/s, the boundary behind the level unchanged)
      static const bool fin_wt = std::getenv("SACMI_FIN_WT") != nullptr && std::atoi(std::getenv("SACMI_FIN_WT")) != 0;
      b.st_wt = fin_wt ? 1 : 0;
      static const bool nsl = SACMI_DWFIN_NSL && std::getenv("SACMI_NO_DWFIN_NSL") == nullptr;
      const char* fin_p = std::getenv("SACMI_DWFIN_P");   // (opt-in; read per enqueue: tests switch it)
      if (nsl && kDwFinEpt == 1 && fin_p && std::atoi(fin_p) != 0) {
        const dim3 pg(std::min(fin_grid, kDwFinGrid));
        switch (ns) {
          case 1: hipLaunchKernelGGL(k_dw_fin_p<1>, pg, fb, 0, s, b, ns, stride, fin_grid); break;
          case 2: hipLaunchKernelGGL(k_dw_fin_p<2>, pg, fb, 0, s, b, ns, stride, fin_grid); break;
          case 3: hipLaunchKernelGGL(k_dw_fin_p<3>, pg, fb, 0, s, b, ns, stride, fin_grid); break;
          case 4: hipLaunchKernelGGL(k_dw_fin_p<4>, pg, fb, 0, s, b, ns, stride, fin_grid); break;
          case 5: hipLaunchKernelGGL(k_dw_fin_p<5>, pg, fb, 0, s, b, ns, stride, fin_grid); break;
          case 6: hipLaunchKernelGGL(k_dw_fin_p<6>, pg, fb, 0, s, b, ns, stride, fin_grid); break;
          case 7: hipLaunchKernelGGL(k_dw_fin_p<7>, pg, fb, 0, s, b, ns, stride, fin_grid); break;
          case 8: hipLaunchKernelGGL(k_dw_fin_p<8>, pg, fb, 0, s, b, ns, stride, fin_grid); break;
          case 9: hipLaunchKernelGGL(k_dw_fin_p<9>, pg, fb, 0, s, b, ns, stride, fin_grid); break;
          case 10: hipLaunchKernelGGL(k_dw_fin_p<10>, pg, fb, 0, s, b, ns, stride, fin_grid); break;
          case 11: hipLaunchKernelGGL(k_dw_fin_p<11>, pg, fb, 0, s, b, ns, stride, fin_grid); break;
          case 12: hipLaunchKernelGGL(k_dw_fin_p<12>, pg, fb, 0, s, b, ns, stride, fin_grid); break;
          default: hipLaunchKernelGGL(k_dw_fin_p<kDwMaxSplit>, pg, fb, 0, s, b, ns, stride, fin_grid); break;
        }
        HIP_LAUNCH_CHECK();
        return;
      }
      switch (nsl ? ns : 0) {
        case 1: hipLaunchKernelGGL(k_dw_fin<1>, fg, fb, 0, s, b, ns, stride); break;
        case 2: hipLaunchKernelGGL(k_dw_fin<2>, fg, fb, 0, s, b, ns, stride); break;
        case 3: hipLaunchKernelGGL(k_dw_fin<3>, fg, fb, 0, s, b, ns, stride); break;
        case 4: hipLaunchKernelGGL(k_dw_fin<4>, fg, fb, 0, s, b, ns, stride); break;
        case 5: hipLaunchKernelGGL(k_dw_fin<5>, fg, fb, 0, s, b, ns, stride); break;
        case 6: hipLaunchKernelGGL(k_dw_fin<6>, fg, fb, 0, s, b, ns, stride); break;
        case 7: hipLaunchKernelGGL(k_dw_fin<7>, fg, fb, 0, s, b, ns, stride); break;
        case 8: hipLaunchKernelGGL(k_dw_fin<8>, fg, fb, 0, s, b, ns, stride); break;
        case 9: hipLaunchKernelGGL(k_dw_fin<9>, fg, fb, 0, s, b, ns, stride); break;
        case 10: hipLaunchKernelGGL(k_dw_fin<10>, fg, fb, 0, s, b, ns, stride); break;
        case 11: hipLaunchKernelGGL(k_dw_fin<11>, fg, fb, 0, s, b, ns, stride); break;
        case 12: hipLaunchKernelGGL(k_dw_fin<12>, fg, fb, 0, s, b, ns, stride); break;
        default: hipLaunchKernelGGL(k_dw_fin<kDwMaxSplit>, fg, fb, 0, s, b, ns, stride); break;
      }
      HIP_LAUNCH_CHECK();
      return;
    }
    b = b0;
    for (int i = 0; i < b.count; ++i)   // (no other kernel knows the dW A transform)
      if (b.d[i].axk == 2) throw Error{SACMI_ESTATE, "dW A transform (axk 2) outside the split-K path"};
  }
  if (SACMI_AXK_LDS16) {
    const int ax = axk16_ok(b);
    if (ax >= 0) {
      if (b.ride.pk_blocks) throw pk_err;
      for (int i = 0; i < b.count; ++i)   // k_axk16 computes no dL/da partials
        if (b.d[i].pa_out) throw Error{SACMI_ESTATE, "dL/da partials requested on a k_axk16 level"};
      const bool bh = all_bh(b);
      const dim3 grid(b.total_tiles + (b.ride.kind ? b.ride.nblocks : 0)), blk(64 * kAxWaves);
      const int form = level_act16(b);   // act16: mask sources (and AX sources) bf16
      if (form < 0) throw Error{SACMI_ESTATE, "k_axk16 level with mixed bf16 activation flags"};
      for (int i = 0; i < b.count; ++i)
        if (b.d[i].c16 || b.d[i].b16 || b.d[i].x16 != form || b.d[i].a16 != (form && b.d[i].axk == 1))
          throw Error{SACMI_ESTATE, "k_axk16: unsupported bf16 activation operand"};
      const int bm = form && bh ? axk16p_plan(b, ax) : 0;
      if (bm) {   // (axk16p_plan re-tiled the level: its grid)
        const dim3 pg(b.total_tiles);
        if (ax) hipLaunchKernelGGL((k_axk16p<128, true>), pg, dim3(1024), 0, s, b);
        else if (bm == 128) hipLaunchKernelGGL((k_axk16p<128, false>), pg, dim3(1024), 0, s, b);
        else hipLaunchKernelGGL((k_axk16p<64, false>), pg, dim3(1024), 0, s, b);
      } else if (form) {
        if (ax && bh) hipLaunchKernelGGL((k_axk16<true, true, true>), grid, blk, 0, s, b);
        else if (ax) hipLaunchKernelGGL((k_axk16<true, false, true>), grid, blk, 0, s, b);
        else if (bh) hipLaunchKernelGGL((k_axk16<false, true, true>), grid, blk, 0, s, b);
        else hipLaunchKernelGGL((k_axk16<false, false, true>), grid, blk, 0, s, b);
      } else if (ax && bh) {
        hipLaunchKernelGGL((k_axk16<true, true>), grid, blk, 0, s, b);
      } else if (ax) {
        hipLaunchKernelGGL((k_axk16<true, false>), grid, blk, 0, s, b);
      } else if (bh) {
        hipLaunchKernelGGL((k_axk16<false, true>), grid, blk, 0, s, b);
      } else {
        hipLaunchKernelGGL((k_axk16<false, false>), grid, blk, 0, s, b);
      }
      HIP_LAUNCH_CHECK();
      return;
    }
  }
  b = b0;
  static const bool fwd_big = SACMI_FWD_BIG && std::getenv("SACMI_NO_FWD_BIG") == nullptr;
  if (fwd_big && fwd_big_ok(b)) {
    if (b.ride.pk_blocks) throw pk_err;
    const bool n128 = b.d[0].tiles_n * kFBN128 >= b.d[0].N && b.d[0].tiles_n == (b.d[0].N + 127) / 128;
    const bool bh = b.bf16 && all_bh(b);
    if (level_act16(b)) {   // act16: bf16 input rows and bf16 output (k_fwd16 only)
      for (int i = 0; i < b.count; ++i)
        if (!b.d[i].a16 || !b.d[i].c16 || b.d[i].b16 || b.d[i].x16 || (b.d[i].N & 1) || (b.d[i].ldc & 1))
          throw Error{SACMI_ESTATE, "k_fwd16: unsupported bf16 activation operands"};
      if (!(b.bf16 && SACMI_FWD_LDS16)) throw Error{SACMI_ESTATE, "bf16 activations need k_fwd16"};
      if (bh) {
        GemmBatch bp = b;
        const int bm = fwd16p_plan(bp);
        if (bm) {
          static const int nwv = std::getenv("SACMI_FWD16P_WAVES") ? std::atoi(std::getenv("SACMI_FWD16P_WAVES")) : SACMI_FWD16P_WAVES;
          const dim3 g(bp.total_tiles);
          if (bm == 256 && nwv == 8) hipLaunchKernelGGL((k_fwd16p<256, 8>), g, dim3(512), 0, s, bp);
          else if (bm == 256) hipLaunchKernelGGL((k_fwd16p<256, 16>), g, dim3(1024), 0, s, bp);
          else if (nwv == 8) hipLaunchKernelGGL((k_fwd16p<128, 8>), g, dim3(512), 0, s, bp);
          else hipLaunchKernelGGL((k_fwd16p<128, 16>), g, dim3(1024), 0, s, bp);
          HIP_LAUNCH_CHECK();
          return;
        }
      }
      if (n128 && bh)hipLaunchKernelGGL((k_fwd16<128, true, true>), dim3(b.total_tiles), dim3(64 * fwd16_waves<128>()), 0, s, b);
      else if (bh) hipLaunchKernelGGL((k_fwd16<64, true, true>), dim3(b.total_tiles), dim3(64 * fwd16_waves<64>()), 0, s, b);
      else if (n128) hipLaunchKernelGGL((k_fwd16<128, false, true>), dim3(b.total_tiles), dim3(64 * fwd16_waves<128>()), 0, s, b);
      else hipLaunchKernelGGL((k_fwd16<64, false, true>), dim3(b.total_tiles), dim3(64 * fwd16_waves<64>()), 0, s, b);
      HIP_LAUNCH_CHECK();
      return;
    }
    if (b.bf16 && SACMI_FWD_LDS16 && n128 && bh) hipLaunchKernelGGL((k_fwd16<128, true>), dim3(b.total_tiles), dim3(64 * fwd16_waves<128>()), 0, s, b);
    else if (b.bf16 && SACMI_FWD_LDS16 && bh) hipLaunchKernelGGL((k_fwd16<64, true>), dim3(b.total_tiles), dim3(64 * fwd16_waves<64>()), 0, s, b);
    else if (b.bf16 && SACMI_FWD_LDS16 && n128) hipLaunchKernelGGL((k_fwd16<128>), dim3(b.total_tiles), dim3(64 * fwd16_waves<128>()), 0, s, b);
    else if (b.bf16 && SACMI_FWD_LDS16) hipLaunchKernelGGL((k_fwd16<64>), dim3(b.total_tiles), dim3(64 * fwd16_waves<64>()), 0, s, b);
    else if (b.bf16 && n128) hipLaunchKernelGGL((k_fwd<true, 128>), dim3(b.total_tiles), dim3(256), 0, s, b);
    else if (b.bf16) hipLaunchKernelGGL((k_fwd<true, 64>), dim3(b.total_tiles), dim3(256), 0, s, b);
    else hipLaunchKernelGGL((k_fwd<false, 64>), dim3(b.total_tiles), dim3(256), 0, s, b);
    HIP_LAUNCH_CHECK();
    return;
  }
  b = b0;
  if (level_act16(b))
    throw Error{SACMI_ESTATE, "bf16 activation operands on a level outside the batch-4096-class kernels"};
  const int extra0 = (b.ride.kind ? b.ride.nblocks : 0) + b.ride.pk_blocks;
  // a fused-Adam level's scalar work: by default wave 0 of block 0 before its tile (-2);
  // SACMI_B0_LATE=1: block 0 after its tile (-1, the round-3 form); SACMI_ADAM_WG=1: a
  // workgroup of its own past the tiles and rides (measured: the 257th workgroup of L6 / L13
  // waits for a free CU — L6 +0.85 us, L13 no faster)
  static const bool adam_wg_on = std::getenv("SACMI_ADAM_WG") != nullptr && std::atoi(std::getenv("SACMI_ADAM_WG")) != 0;
  static const bool b0_late = std::getenv("SACMI_B0_LATE") != nullptr && std::atoi(std::getenv("SACMI_B0_LATE")) != 0;
  const bool awg = b.has_adam && adam_wg_on;
  const int extra = extra0 + (awg ? 1 : 0);
  b.adam_wg = b0_late ? -1 : -2;
  auto set_awg = [&](int tiles) { if (awg) b.adam_wg = tiles + extra0; };
  auto grid_for = [&](int tiles) { set_awg(tiles); return tiles + extra; };
  if (b.ride.kind == 1 && mt_sample_lds_words(b.ride.tbl_log2, b.ride.mt.setsize) * 4 > kRideLdsBytes)
    throw Error{SACMI_ESTATE, "ride-along sampler table exceeds k_gemm's LDS"};
  int maxk = 0, n_adam = 0;
  int64_t outs = 0;
  for (int i = 0; i < b.count; ++i) {
    maxk = b.d[i].K > maxk ? b.d[i].K : maxk;
    n_adam += b.d[i].epi >= EPI_ADAM;
    outs += (int64_t)b.d[i].M * b.d[i].N;
  }
  // write-through epilogue stores where they shorten the boundary to the next level: the
  // Adam levels (15-30 MB of optimizer state) and the batch-256-class levels (<= 4 MB of
  // outputs: config 2 124.9 -> 121.3 us per update); the batch-4096 activation levels keep
  // plain stores (config 3: 762 -> 774 us with every level write-through)
  b.st_wt = (n_adam > 0 || outs <= (1 << 20)) ? 1 : 0;
  // (Level::add guarantees a level is all-Adam or all-plain)
  int axk = 0;
  for (int i = 0; i < b.count; ++i) axk = b.d[i].axk > axk ? b.d[i].axk : axk;
  // weight-gradient levels (both operands row-contiguous): the Adam-fused and the plain
  // (data-parallel) form of a level take the same tile geometry, so their bits agree
  bool dw = true;
  for (int i = 0; i < b.count; ++i) dw = dw && !b.d[i].a_kc && !b.d[i].b_kc;
  const int t64 = assign_tiles<32, 64>(b);
  // the batch-256 class on the LDS-staged core (same tile geometries as below)
  if (staged_ok(b) && (dw || (!n_adam && t64 <= 512))) {
    if (dw && t64 <= 256) {
      if (n_adam) launch_ks<32, 64, 8, 1, true, 0>(b, grid_for(b.total_tiles), s);
      else launch_ks<32, 64, 8, 1, false, 0>(b, grid_for(b.total_tiles), s);
    } else if (dw) {
      for (int i = 0; i < b.count; ++i)
        if (b.d[i].pa_out) throw Error{SACMI_ESTATE, "dL/da partials requested on a 64-row tile level"};
      const int g = grid_for(assign_tiles<64, 64>(b));
      if (n_adam) launch_ks<32, 64, 4, 2, true, 0>(b, g, s);
      else launch_ks<32, 64, 4, 2, false, 0>(b, g, s);
    } else if (axk == 1) {
      const int g = grid_for(assign_tiles<32, 32>(b));
      launch_ks<32, 32, 8, 1, false, 1>(b, g, s);
    } else if (t64 >= 192) {
      launch_ks<32, 64, 8, 1, false, 0>(b, grid_for(b.total_tiles), s);
    } else {
      const int g = grid_for(assign_tiles<32, 32>(b));
      launch_ks<32, 32, 8, 1, false, 0>(b, g, s);
    }
    HIP_LAUNCH_CHECK();
    return;
  }
  if (dw && t64 <= 256) {
    // one 32x64 tile per CU (policy level): 16 waves, K split 16 ways
    if (n_adam) launch_k<32, 64, 16, 1, 1, true, 0>(b, grid_for(b.total_tiles), s);
    else launch_k<32, 64, 16, 1, 1, false, 0>(b, grid_for(b.total_tiles), s);
  } else if (dw || n_adam || t64 > 512) {
    // more 32x64 tiles than CUs (the twin critic weight gradients; every level at large
    // batch): 64x64 tiles as two 32-row wave groups, each with an 8-way K split — half
    // the operand bytes per FLOP of a 32x64 tile; the epilogue state is prefetched under
    // the MFMAs
    // 16 waves per CU either as one 1024-thread workgroup (8-way K split per wave group)
    // or as several smaller ones (4- / 2-way): then one workgroup's LDS reduction and
    // epilogue overlap another's operand loads and MFMAs.  Rides attach to 1024 threads.
    const int g = grid_for(assign_tiles<64, 64>(b));
    for (int i = 0; i < b.count; ++i)   // the two-wave-group tiles compute no dL/da partials
      if (b.d[i].pa_out) throw Error{SACMI_ESTATE, "dL/da partials requested on a 64-row tile level"};
    if (n_adam) {
      if (SACMI_DW_KS == 4 && !extra0) launch_k<32, 64, 4, 1, 2, true, 0>(b, g, s);
      else launch_k<32, 64, 8, 1, 2, true, 0>(b, g, s);
    } else if (axk == 1) {
      if (SACMI_AXK_KS == 4 && !extra0) launch_k<32, 64, 4, 1, 2, false, 1>(b, g, s);
      else launch_k<32, 64, 8, 1, 2, false, 1>(b, g, s);
    } else if (dw) {
      // the plain (data-parallel) form of a weight-gradient level: the fused form's geometry
      if (SACMI_DW_KS == 4 && !extra0) launch_k<32, 64, 4, 1, 2, false, 0>(b, g, s);
      else launch_k<32, 64, 8, 1, 2, false, 0>(b, g, s);
    } else if (!extra0 && SACMI_FWD_KS == 2) {
      launch_k<32, 64, 2, 1, 2, false, 0>(b, g, s);
    } else if (!extra0 && SACMI_FWD_KS == 4) {
      launch_k<32, 64, 4, 1, 2, false, 0>(b, g, s);
    } else {
      launch_k<32, 64, 8, 1, 2, false, 0>(b, g, s);
    }
  } else if (axk == 1) {
    // dh1 / dha1 with the fc3 backward folded in (A transform, coefficient in the epilogue)
    const int g = grid_for(assign_tiles<32, 32>(b));
    launch_k<32, 32, 16, 2, 1, false, 1>(b, g, s);
  } else if (t64 >= 192) {
    // widest tile that still gives one workgroup to most CUs (the folded-heads instantiation
    // where the level carries the fold)
    if (b.heads_ticket && !b.bf16)
      hipLaunchKernelGGL((k_gemm<32, 64, 16, 2, 1, false, 0, false, 0, true>), dim3(grid_for(b.total_tiles)), dim3(1024), 0, s, b);
    else
      launch_k<32, 64, 16, 2, 1, false, 0>(b, grid_for(b.total_tiles), s);
  } else {
    const int g = grid_for(assign_tiles<32, 32>(b));
    launch_k<32, 32, 16, 2, 1, false, 0>(b, g, s);
  }
  HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
// policy heads (mean | log_std) GEMM + GaussianPolicy.sample epilogue
// (networks_model1.py:65-99, torch distributions/normal.py:83-103)
// H16 (act16 updates): h is bf16 (widened exactly; Wh fp32, fp32 MFMAs) and the actions
// go to act as bf16 (the next levels' input columns)
// TM rows per workgroup (heads_rows_per_wg: 32 at the batch-4096 class — one workgroup
// per CU covers all rows in one round and the head weights are re-read half as often)
// rows [m0, m0 + TM) by one 64 * KSPLIT-thread workgroup; part: the row block's slot pair in
// logp_part; red (KSPLIT * TM * (TN + 1) floats), lp, s_lp: LDS.  AAUX: cache-policy bits of
// the h loads (k_gemm's folded form reads h rows other workgroups of the same launch wrote:
// sc1, coherent across the XCDs' L2s)
template <int TN, int KSPLIT, bool H16, int TM, int AAUX>
__device__ __forceinline__ void heads_rows(const HeadSampleArgs& a, int m0, int part, float* red,
                                           float (*lp)[33], float* s_lp) {
  const int A = a.A;
  GemmDesc d;
  d.A = a.h; d.lda = a.ldh; d.a_kc = 1; d.M = a.rows;
  d.B = a.Wh; d.ldb = a.ldw; d.b_kc = 1; d.N = 2 * A; d.K = a.K;
  static_assert(TM * 32 <= 64 * KSPLIT, "one (row, action) element per thread (A <= 32)");
  // element e = threadIdx.x -> (row, action j); its bias values (and stored noise)
  // are loaded while the MFMAs run
  const int e = threadIdx.x;
  const int row = e / A, j = e % A, m = m0 + row;
  const bool live = e < TM * A && m < a.rows;
  float bm = 0.f, bl = 0.f, eps_in = 0.f;
  auto pre = [&]() {     // unconditional loads at clamped addresses (no guarded loads)
    const int jj = live ? j : 0, mm = live ? m : 0;
    bm = a.Wh[(size_t)jj * a.ldw + a.K];
    bl = a.Wh[(size_t)(A + jj) * a.ldw + a.K];
    const bool want = !a.deterministic && !a.gen_eps;
    eps_in = buf_ld(make_rsrc(want ? a.eps : a.Wh, want ? 0x7fffffffu : 0u),
                    (uint32_t)((size_t)mm * A + jj) * 4u);
  };
  gemm_core_l<TM, TN, KSPLIT, 2, true, true, false, 1, 0, false, 0, H16, AAUX>(d, m0, 0, red, nullptr, pre);
  __syncthreads();
  const uint64_t ctr = a.ctr_override ? a.ctr_override : a.sc->noise_counter;
  if (e < TM * A) {
    float lpe = 0.f;
    if (live) {
      const float mean = reduce_partials<TM, TN, KSPLIT>(red, row, j) + bm;
      const float ls_raw = reduce_partials<TM, TN, KSPLIT>(red, row, A + j) + bl;
      lpe = heads_elem<H16, AAUX>(a, m, j, mean, ls_raw, eps_in, ctr);
    }
    lp[row][j] = lpe;
  }
  heads_logp<TM, AAUX>(a, m0, part, lp, s_lp);
}

template <int TN, int KSPLIT, bool H16 = false, int TM = 16>
__global__ __launch_bounds__(64 * KSPLIT) void k_heads_sample(HeadSampleArgs a) {
  const TlMark tl_mark(a.tl, TL_HEADS);
  __shared__ float red[KSPLIT * TM * (TN + 1)];
  __shared__ float lp[TM][33];
  __shared__ float s_lp[TM];
  heads_rows<TN, KSPLIT, H16, TM, 0>(a, blockIdx.x * TM, blockIdx.x, red, lp, s_lp);
  if (a.done_word) {   // (one workgroup) every store above lands first
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) *reinterpret_cast<volatile int*>(a.done_word) = a.done_value;
  }
}

__global__ void k_to_bf16(unsigned short* dst, const float* src, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = bf16_bits(src[i]);
}

// ---------------------------------------------------------------------------
// select_action for one state (sacmi_act, n = 1): a 32-row level tile uses one of its rows,
// ~5-6 us a level at M = 1; here a wave per output, its lanes over K (16-byte loads of the
// weight row and of x), a fixed butterfly, 16 outputs a workgroup
__device__ __forceinline__ float gemv_dot(const float* x, const float* w, int K) {
  const int lane = threadIdx.x & 63;
  float acc = 0.f;
  for (int k = 4 * lane; k < K; k += 256) {
    const float4 wv = *reinterpret_cast<const float4*>(w + k);
    const float4 xv = *reinterpret_cast<const float4*>(x + k);
    acc = fmaf(wv.x, xv.x, acc); acc = fmaf(wv.y, xv.y, acc);
    acc = fmaf(wv.z, xv.z, acc); acc = fmaf(wv.w, xv.w, acc);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  return acc;
}

__global__ __launch_bounds__(1024) void k_act_gemv(GemvArgs a) {
  const int n = blockIdx.x * 16 + (threadIdx.x >> 6);
  if (n >= a.N) return;
  const float v = gemv_dot(a.x, a.W + (size_t)n * a.ldw, a.K);
  if ((threadIdx.x & 63) == 0) a.y[n] = a.relu ? (v <= 0.f ? 0.f : v) : v;   // F.relu keeps NaN
}

void launch_act_gemv(const GemvArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_act_gemv, dim3((a.N + 15) / 16), dim3(1024), 0, s, a);
  HIP_LAUNCH_CHECK();
}

// heads + GaussianPolicy.sample of one row (k_heads_sample's per-element algebra,
// networks_model1.py:65-99): 2A dot products over 16 waves, then thread j < A
__global__ __launch_bounds__(1024) void k_act_heads(ActHeadsArgs a) {
  __shared__ float s_h[64];
  const int wave = threadIdx.x >> 6, A = a.A;
  for (int o = wave; o < 2 * A; o += 16) {
    const float v = gemv_dot(a.x, a.Wh + (size_t)o * a.ldw, a.K);
    if ((threadIdx.x & 63) == 0) s_h[o] = v;
  }
  __syncthreads();
  const int j = threadIdx.x;
  if (j < A) {
    const float mean = s_h[j], ls_raw = s_h[A + j];
    const float ls = fminf(fmaxf(ls_raw, -20.f), 2.f);
    const float sd = expf(ls);
    if (!a.deterministic && (__builtin_isnan(mean) || __builtin_isnan(ls_raw))) *a.nan_flag = 1;
    const float eps = a.deterministic ? 0.f : a.gen_eps ? philox_normal(a.seed, a.ctr, (uint32_t)j) : a.eps[j];
    const float x = a.deterministic ? mean : mean + eps * sd;
    a.out[j] = tanhf(x) * a.scale + a.bias;
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) *reinterpret_cast<volatile int*>(a.done_word) = a.done_value;
}

void launch_act_heads(const ActHeadsArgs& a, hipStream_t s) {
  if (a.A > 32) throw Error{SACMI_EVALUE, "heads: action_dim > 32"};
  hipLaunchKernelGGL(k_act_heads, dim3(1), dim3(1024), 0, s, a);
  HIP_LAUNCH_CHECK();
}

void launch_to_bf16(unsigned short* dst, const float* src, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_to_bf16, dim3((unsigned)blocks), dim3(256), 0, s, dst, src, n);
  HIP_LAUNCH_CHECK();
}

void launch_heads_sample(const HeadSampleArgs& a, hipStream_t s) {
  const int tm = heads_rows_per_wg(a.rows);
  const int grid = (a.rows + tm - 1) / tm;
  const int n = 2 * a.A;
  if (a.A > 32) throw Error{SACMI_EVALUE, "heads: action_dim > 32"};
  if (tm == 32) {
    if (a.h16 && n <= 32) hipLaunchKernelGGL((k_heads_sample<32, 16, true, 32>), dim3(grid), dim3(1024), 0, s, a);
    else if (a.h16 && n <= 48) hipLaunchKernelGGL((k_heads_sample<48, 16, true, 32>), dim3(grid), dim3(1024), 0, s, a);
    else if (a.h16) hipLaunchKernelGGL((k_heads_sample<64, 16, true, 32>), dim3(grid), dim3(1024), 0, s, a);
    else if (n <= 32) hipLaunchKernelGGL((k_heads_sample<32, 16, false, 32>), dim3(grid), dim3(1024), 0, s, a);
    else if (n <= 48) hipLaunchKernelGGL((k_heads_sample<48, 16, false, 32>), dim3(grid), dim3(1024), 0, s, a);
    else hipLaunchKernelGGL((k_heads_sample<64, 16, false, 32>), dim3(grid), dim3(1024), 0, s, a);
  } else if (a.h16) {
    if (n <= 32) hipLaunchKernelGGL((k_heads_sample<32, 16, true>), dim3(grid), dim3(1024), 0, s, a);
    else if (n <= 48) hipLaunchKernelGGL((k_heads_sample<48, 16, true>), dim3(grid), dim3(1024), 0, s, a);
    else hipLaunchKernelGGL((k_heads_sample<64, 16, true>), dim3(grid), dim3(1024), 0, s, a);
  } else if (n <= 32) {
    hipLaunchKernelGGL((k_heads_sample<32, 16>), dim3(grid), dim3(1024), 0, s, a);
  } else if (n <= 48) {
    hipLaunchKernelGGL((k_heads_sample<48, 16>), dim3(grid), dim3(1024), 0, s, a);
  } else {
    hipLaunchKernelGGL((k_heads_sample<64, 16>), dim3(grid), dim3(1024), 0, s, a);
  }
  HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
// dL/da GEMM (both critics, K = 2H) + GaussianPolicy.sample backward epilogue.
// For L_pi = mean(alpha*logp - min Q): dL/dlogp = alpha/B.  Per element with
// u = scale*(1-y^2)+1e-6:  G = scale*dL/da + (alpha/B)*2*scale*y/u,
//   dmean = G*(1-y^2);  dlog_std = [-20<=ls<=2] * (G*(1-y^2)*eps*std - alpha/B)
// (the Normal.log_prob quadratic term's gradients w.r.t. mean and std cancel
// exactly: x - mean = eps*std).
// NST: k-steps (of 4) of the dhp2 tail's K = 2A, a compile-time bound
template <int TM, int TN, int KSPLIT, int NST, bool H16 = false>
__global__ __launch_bounds__(64 * KSPLIT) void k_gemm_sample_bwd(GemmDesc d, SampleBwdArgs a) {
  const TlMark tl_mark(a.tl, TL_SAMPLE_BWD);
  __shared__ float red[KSPLIT * TM * (TN + 1)];
  __shared__ float s_dh[TM][64 + 1];     // this workgroup's dhead rows, zero beyond 2A
  for (int i = threadIdx.x; i < TM * 65; i += 64 * KSPLIT) (&s_dh[0][0])[i] = 0.f;
  const int m0 = blockIdx.x * TM;
  static_assert(TM * TN <= 64 * KSPLIT, "one (row, action) element per thread");
  // element e = threadIdx.x -> (row, action j); the sample cache and noise are loaded
  // while the MFMAs run
  const int A = a.A;
  const int e = threadIdx.x;
  const int row = e / A, j = e % A, m = m0 + row;
  const bool live = e < TM * A && m < d.M;
  float ls_raw = 0.f, y = 0.f, eps = 0.f, omy2 = 0.f;
  // the dhp2 tail's operands for this wave's first 32-column slab: Whead fragments and
  // the ReLU-mask source, also loaded under the dL/da MFMAs
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int K2 = 2 * A, ksteps = (K2 + 3) / 4;
  float bw[2][NST], mk[2][4];
  // every load below is unconditional at a clamped address (zeroed by a select): a
  // guarded load is drained at the end of its guard, serialising the burst it sits in
  auto load_mask = [&](int n0) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = n0 + t * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int mr = m0 + (lane >> 4) * 4 + r;
        const bool ok = mr < d.M && n < a.H;
        const size_t ix = ok ? (size_t)mr * a.ldh + n : 0;
        const float x = H16 ? bf16_lo(reinterpret_cast<const unsigned short*>(a.hp2)[ix]) : a.hp2[ix];
        mk[t][r] = ok ? x : 0.f;
      }
    }
  };
  auto load_w = [&](int n0) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = n0 + t * 16 + (lane & 15);
#pragma unroll
      for (int st = 0; st < NST; ++st) {
        const int k = 4 * st + (lane >> 4);
        const bool ok = st < ksteps && k < K2 && n < a.H;
        const float x = a.Wh[ok ? (size_t)k * a.ldw + n : 0];
        bw[t][st] = ok ? x : 0.f;
      }
    }
  };
  auto pre = [&]() {
    const int mm = live ? m : 0, jj = live ? j : 0;
    const float* cr = a.cache + (size_t)mm * 3 * A;
    omy2 = cr[jj];
    ls_raw = cr[A + jj];
    y = cr[2 * A + jj];
    eps = a.eps[(size_t)mm * A + jj];
    load_mask(wave * 32);
  };
  gemm_core_l<TM, TN, KSPLIT, 2, true, false, false>(d, m0, 0, red, nullptr, pre);
  __syncthreads();
  const float glogp = a.sc->alpha / (float)a.B;
  if (live) {
    const float ga = reduce_partials<TM, TN, KSPLIT>(red, row, j);
    const float ls = fminf(fmaxf(ls_raw, -20.f), 2.f);
    const float sd = expf(ls);
    const float u = a.scale * omy2 + 1e-6f;
    const float G = a.scale * ga + glogp * (2.f * a.scale * y / u);
    const float dx = G * omy2;
    float dls = dx * eps * sd - glogp;
    if (!(ls_raw >= -20.f && ls_raw <= 2.f)) dls = 0.f;
    a.dhead[(size_t)m * a.lddh + j] = dx;
    a.dhead[(size_t)m * a.lddh + A + j] = dls;
    s_dh[row][j] = dx;
    s_dh[row][A + j] = dls;
  }
  __syncthreads();
  // dhp2[TM rows, H] = (s_dh[TM, 2A] Whead[2A, H]) * [hp2 > 0]: 16x16x4 MFMAs, A from LDS,
  // each wave a 32-column slab per pass (networks_model1.py:72-76 backward)
  for (int n0 = wave * 32; n0 < a.H; n0 += KSPLIT * 32) {
    f4 acc[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
    if (n0 != wave * 32) load_mask(n0);   // H > 512: later slabs load their mask here
    load_w(n0);
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      if (st < ksteps) {
        const float av = s_dh[lane & 15][4 * st + (lane >> 4)];
#pragma unroll
        for (int t = 0; t < 2; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bw[t][st], acc[t], 0, 0, 0);
      }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = (lane >> 4) * 4 + r, n = n0 + t * 16 + (lane & 15);
        if (m0 + rr < d.M && n < a.H)
          st_wt(a.dhp2 + (size_t)(m0 + rr) * a.H + n, mk[t][r] > 0.f ? acc[t][r] : 0.f);
      }
  }
}

void launch_gemm_sample_bwd(const GemmDesc& d, const SampleBwdArgs& a, hipStream_t s) {
  const int grid = (d.M + 15) / 16;
  const bool n10 = (2 * a.A + 3) / 4 <= 10;
  if (a.hp2_16 && n10) hipLaunchKernelGGL((k_gemm_sample_bwd<16, 32, 16, 10, true>), dim3(grid), dim3(1024), 0, s, d, a);
  else if (a.hp2_16) hipLaunchKernelGGL((k_gemm_sample_bwd<16, 32, 16, 16, true>), dim3(grid), dim3(1024), 0, s, d, a);
  else if (n10) hipLaunchKernelGGL((k_gemm_sample_bwd<16, 32, 16, 10>), dim3(grid), dim3(1024), 0, s, d, a);
  else hipLaunchKernelGGL((k_gemm_sample_bwd<16, 32, 16, 16>), dim3(grid), dim3(1024), 0, s, d, a);
  HIP_LAUNCH_CHECK();
}

constexpr int kTailRows = 8, kTailCols = 64, kTailMaxPa = 64;
struct TailSmem {
  float s_dh[kTailRows][64 + 1];       // dhead rows, zero beyond 2A
  float s_w[64][kTailCols + 1];        // Whead[k][slab columns], k < 2A
};
// One unit: rows [m0, m0 + 8) x dhp2 columns [c0, c0 + 64), by the first 256 threads of the
// workgroup (any others only join its barriers).  slab0: the unit also stores dhead.  AUX:
// cache-policy bits of the dL/da partial loads (k_chain: sc1 — L9 wrote them in the same launch)
template <int AUX, bool MIDSPLIT = false, int NPA = kTailMaxPa, class Mid = void (*)()>
__device__ __forceinline__ void tail_unit(const float* pa, int n_pa, const SampleBwdArgs& a, int m0,
                                          int c0, bool slab0, TailSmem& sm, Mid&& mid = [] {}) {
  if constexpr (MIDSPLIT) mid.issue();   // (k_chain: the barrier's first poll, as kg_body's)
  auto& s_dh = sm.s_dh;
  auto& s_w = sm.s_w;
  const int A = a.A, B = a.B, K2 = 2 * A;
  const int tid = threadIdx.x;
  const bool act = tid < 256;
  // every global load of the unit goes out first (one round trip): thread e < 8A owns
  // (row e / A, action e % A) — its partials, cache and noise; all threads stage a share
  // of the Whead slab and of the ReLU mask.  Buffer loads at out-of-range offsets return
  // 0 without an access, so no load sits behind a guard.
  const int prow = tid / A, pj = tid - prow * A, pm = m0 + prow;
  const bool own = act && tid < kTailRows * A && pm < B;
  const rsrc_t rC = make_rsrc(a.cache, (uint32_t)((size_t)B * 3 * A * 4));
  const rsrc_t rE = make_rsrc(a.eps, (uint32_t)((size_t)B * A * 4));
  const uint32_t co = own ? (uint32_t)(pm * 3 * A + pj) * 4u : 0xfffffff0u;
  constexpr int WPT = 64 * kTailCols / 256;       // Whead slab elements per thread (k < 64)
  const rsrc_t rW = make_rsrc(a.Wh, (uint32_t)(((size_t)(K2 - 1) * a.ldw + a.H) * 4));
  // the dhp2 thread layout: row tid / 32 (8 rows), 2 consecutive slab columns
  const int row = act ? tid >> 5 : 0, cq = (tid & 31) * 2, m = m0 + row;
  const rsrc_t rH = make_rsrc(a.hp2, (uint32_t)(((size_t)(B - 1) * a.ldh + a.H) * 4));
  float omy2, ls_raw, y, eps, wv[WPT], mk[2];
  auto preload = [&]() {
    omy2 = buf_ld(rC, co);
    ls_raw = buf_ld(rC, co + (uint32_t)A * 4u);
    y = buf_ld(rC, co + (uint32_t)(2 * A) * 4u);
    eps = buf_ld(rE, own ? (uint32_t)(pm * A + pj) * 4u : 0xfffffff0u);
#pragma unroll
    for (int q = 0; q < WPT; ++q) {
      const int e = tid + q * 256, k = e / kTailCols, col = c0 + (e - k * kTailCols);
      wv[q] = buf_ld(rW, act && k < K2 && col < a.H ? (uint32_t)(k * a.ldw + col) * 4u : 0xfffffff0u);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int col = c0 + cq + u;
      mk[u] = buf_ld(rH, act && m < B && col < a.H ? (uint32_t)(m * a.ldh + col) * 4u : 0xfffffff0u);
    }
  };
  // the dL/da partials the previous phase wrote: after mid() (k_chain's barrier; a no-op in
  // the standalone kernel, whose loads all went out above)
  preload();
  mid();
  const rsrc_t rP = make_rsrc(pa, (uint32_t)((size_t)n_pa * B * A * 4));
  const uint32_t pstride = (uint32_t)B * (uint32_t)A * 4u, po = (uint32_t)((own ? pm : 0) * A + pj) * 4u;
  // (NPA >= n_pa partial loads per thread: the launcher picks the smallest instantiation, so
  // no issue slots go to out-of-range loads)
  float t[NPA];
#pragma unroll
  for (int q = 0; q < NPA; ++q)
    t[q] = buf_ld_aux<AUX>(rP, own && q < n_pa ? po + (uint32_t)q * pstride : 0xfffffff0u);
  if (act) {
    for (int e = tid; e < kTailRows * 65; e += 256) (&s_dh[0][0])[e] = 0.f;
#pragma unroll
    for (int q = 0; q < WPT; ++q) {
      const int e = tid + q * 256, k = e / kTailCols;
      s_w[k][e - k * kTailCols] = wv[q];
    }
  }
  __syncthreads();
  if (own) {
    float ga = 0.f;                                 // fixed order over the column blocks
#pragma unroll
    for (int q = 0; q < NPA; ++q)
      if (q < n_pa) ga += t[q];
    const float glogp = a.sc->alpha / (float)B;
    const float ls = fminf(fmaxf(ls_raw, -20.f), 2.f);
    const float sd = expf(ls);
    const float u = a.scale * omy2 + 1e-6f;
    const float G = a.scale * ga + glogp * (2.f * a.scale * y / u);
    const float dx = G * omy2;
    float dls = dx * eps * sd - glogp;
    if (!(ls_raw >= -20.f && ls_raw <= 2.f)) dls = 0.f;
    if (slab0) {
      a.dhead[(size_t)pm * a.lddh + pj] = dx;
      a.dhead[(size_t)pm * a.lddh + A + pj] = dls;
    }
    s_dh[prow][pj] = dx;
    s_dh[prow][A + pj] = dls;
  }
  __syncthreads();
  if (act) {
    float acc[2] = {0.f, 0.f};
    for (int k = 0; k < K2; ++k) {
      const float hk = s_dh[row][k];
      acc[0] = fmaf(hk, s_w[k][cq], acc[0]);
      acc[1] = fmaf(hk, s_w[k][cq + 1], acc[1]);
    }
    if (m < B) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int col = c0 + cq + u;
        if (col < a.H) st_wt(a.dhp2 + (size_t)m * a.H + col, mk[u] > 0.f ? acc[u] : 0.f);
      }
    }
  }
}

// The sample backward + dhp2 tail of the actor pass (sac_imp.py:116-125 backward through
// GaussianPolicy.sample, networks_model1.py:78-99) from the dL/da partials the dha1 level's
// epilogue wrote (GemmDesc::pa_out): one workgroup per (8-row block, 64-column slab of
// dhp2).  dL/da = the n_pa column-block partials summed in fixed order; then the same
// per-element algebra as k_gemm_sample_bwd; the slab-0 workgroups store dhead (the heads'
// weight-gradient operand); dhp2 = (dhead Whead) * [hp2 > 0] for the slab.  Every
// workgroup of a row block recomputes the row block's dhead (a few hundred FMAs).
template <int NPA>
__global__ __launch_bounds__(256) void k_sample_bwd_tail(const float* pa, int n_pa, SampleBwdArgs a) {
  const TlMark tl_mark(a.tl, TL_SAMPLE_TAIL);
  __shared__ TailSmem sm;
  tail_unit<0, false, NPA>(pa, n_pa, a, blockIdx.x * kTailRows, blockIdx.y * kTailCols, blockIdx.y == 0, sm);
}

void launch_sample_bwd_tail(const float* pa, int n_pa, const SampleBwdArgs& a, hipStream_t s) {
  if (2 * a.A > 64 || kTailRows * a.A > 256 || n_pa > kTailMaxPa)
    throw Error{SACMI_EVALUE, "sample backward tail: unsupported action_dim / hidden_dim"};
  if (a.hp2_16) throw Error{SACMI_ESTATE, "sample backward tail: bf16 hp2 not supported"};
  const dim3 grid((a.B + kTailRows - 1) / kTailRows, (a.H + kTailCols - 1) / kTailCols);
  if (n_pa <= 16) hipLaunchKernelGGL(k_sample_bwd_tail<16>, grid, dim3(256), 0, s, pa, n_pa, a);
  else if (n_pa <= 32) hipLaunchKernelGGL(k_sample_bwd_tail<32>, grid, dim3(256), 0, s, pa, n_pa, a);
  else hipLaunchKernelGGL(k_sample_bwd_tail<kTailMaxPa>, grid, dim3(256), 0, s, pa, n_pa, a);
  HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
// k_chain: the batch-256-class actor pass as one persistent launch (sacmi_internal.h
// ChainArgs).  256 workgroups of 1024 threads, one per CU; cohort c = blockIdx % 8 owns batch
// rows [c B/8, (c+1) B/8) in every phase (row-affine tile placement: chain_assign_tiles), so
// each phase waits only for its own cohort's previous phase.
constexpr long long kChainSpinTicks = 5000000;   // 50 ms of the 100 MHz clock: a barrier timeout

// Cohort barriers (cdna_hip_programming.md §6 Guideline 16, MI355X_MICROARCH.md hand-off table
// row 1).  Per cohort, 128-byte strided words: [0, kChainBars) the arrivals at barrier b,
// kChainBars the launch ticket — monotonic and wrapping: every launch adds exactly `nmem` to
// each, so launch e's barrier b is complete once its word reaches (e + 1) nmem, e read from the
// ticket each workgroup draws at its start (nothing is ever reset).
//   chain_end   every wave's write-through stores acknowledged (vmcnt(0)), a workgroup
//               barrier, then ONE agent-scope add on the phase's barrier word (non-returning)
//   ChainWait   the next phase's wait on it: issue() — thread 0's first poll load, at the
//               very start of the phase body, ahead of its weight loads (vmcnt is in order:
//               the poll's value then does not wait for them) — and operator() after the
//               weight loads (kg_body / tail_unit MIDSPLIT hook): further polls (relaxed sc1
//               loads + s_sleep) until the cohort has arrived, then a workgroup barrier; every
//               later load of handed-off bytes is an sc1 load (LDAUX = sc1).  A bounded spin:
//               a timeout sets ERR_CHAIN_TIMEOUT (the host reports a device error) and the
//               workgroup runs on — void outputs, no hang.
__device__ __forceinline__ void chain_end(int* cnt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
struct ChainWait {
  int* cnt;
  int target;
  int* err;
  bool wait;
  tl_word* tl;
  int slot;
  int v;
  __device__ __forceinline__ void issue() {
    if (threadIdx.x == 0 && wait) v = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_sched_barrier(0);
  }
  __device__ __forceinline__ void operator()() {
    if (threadIdx.x == 0 && wait && (int)((unsigned)v - (unsigned)target) < 0) {
      const unsigned long long t0 = wall_clock64();
      while ((int)((unsigned)__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - (unsigned)target) < 0) {
        __builtin_amdgcn_s_sleep(1);
        if ((long long)(wall_clock64() - t0) > kChainSpinTicks) {
          __hip_atomic_fetch_or(err, (int)ERR_CHAIN_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __syncthreads();
    SACMI_PHASE(tl, slot);
  }
};
// the launch's completion target of every barrier word (thread 0 only: the others never wait)
__device__ __forceinline__ int chain_target(int* ticket, int nmem) {
  if (threadIdx.x != 0) return 0;
  const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return (int)(((unsigned)t & ~(unsigned)(nmem - 1)) + (unsigned)nmem);
}

using ChainKgA = KgSmem<32, 32, 16, 2, 1, false, 0, false, 0>;   // L7, L8, L12 (+ rides)
using ChainKgB = KgSmem<32, 32, 16, 2, 1, false, 1, false, 0>;   // L9 (row prologue, dL/da)
union ChainSmem {
  ChainKgA a;
  ChainKgB b;
  TailSmem t;
};

// The argument block is read through the CONSTANT address space: invariant scalar loads, as
// k_gemm's kernel argument (a generic pointer's loads behind the barriers' memory clobbers
// would be vector loads into VGPRs); the generic pointer handed to kg_body is the cast of it,
// which InferAddressSpaces folds back.  Each phase reads it through an opaque copy, so no
// phase's argument loads are hoisted into an earlier one (registers held across it: spills).
typedef __attribute__((address_space(4))) const ChainArgs ConstChainArgs;
__device__ __forceinline__ const ChainArgs* chain_args(const ChainArgs* ca) {
  ConstChainArgs* p4 = (ConstChainArgs*)ca;
  asm volatile("" : "+s"(p4));
  return (const ChainArgs*)p4;
}

// Each phase's weights (and descriptor setup) go out BEFORE the cohort barrier on the
// previous phase (kg_body / tail_unit MIDSPLIT: the barrier is their mid() hook), so their
// latency overlaps the wait.  (diagnostic builds, SACMI_DIAG_PHASES: wave 0's clock at entry
// (slot 0), at the end of phase i (slot i + 1) and right after barrier b's wait (slot 6 + b);
// tools/phase_dump.py)
__global__ __launch_bounds__(1024, 4) void k_chain(const ChainArgs* __restrict__ ca, tl_word* tl) {
  const TlMark tl_mark(tl, TL_CHAIN);
  __shared__ ChainSmem sm;
  SACMI_PHASE(tl, 0);
  const int c = blockIdx.x & (kChainCohorts - 1), bid = blockIdx.x;
  const int nmem = gridDim.x / kChainCohorts;
  int* const sync = chain_args(ca)->sync + c * (kChainBars + 1) * 32;
  int* const err = chain_args(ca)->err;
  const int target = chain_target(sync + kChainBars * 32, nmem);
  auto waiter = [&](int b, bool w) { return ChainWait{sync + b * 32, target, err, w, tl, 6 + b, 0}; };
  // L7 (updated critics fc1 on [s|1|a~])
  {
    const GemmBatch& b = chain_args(ca)->lv[0];
    if (bid < b.total_tiles) kg_body<32, 32, 16, 2, 1, false, 0, false, 0, kLdSc1>(b, bid, sm.a);
    chain_end(sync);
    SACMI_PHASE(tl, 1);
  }
  // L8 (fc2 + fc3 dot partials): barrier 0 behind its weight loads
  {
    const GemmBatch& b = chain_args(ca)->lv[1];
    if (bid < b.total_tiles) kg_body<32, 32, 16, 2, 1, false, 0, false, 0, kLdSc1, true>(b, bid, sm.a, waiter(0, true));
    chain_end(sync + 32);
    SACMI_PHASE(tl, 2);
  }
  // L9: the actor row prologue + dha1 + the dL/da partials
  {
    const GemmBatch& b = chain_args(ca)->lv[2];
    if (bid < b.total_tiles) kg_body<32, 32, 16, 2, 1, false, 1, false, 0, kLdSc1, true>(b, bid, sm.b, waiter(1, true));
    chain_end(sync + 64);
    SACMI_PHASE(tl, 3);
  }
  // the sample-backward tail: the cohort's 8-row groups x 64-column dhp2 slabs
  {
    const ChainArgs* q = chain_args(ca);
    const int ng = q->tail_groups, units = ng * q->tail_slabs;
    const int j = bid / kChainCohorts;
    if (j < units) {
      const int g = j % ng, slab = j / ng;
      tail_unit<kLdSc1, true>(q->pa, q->n_pa, q->tail, c * q->rows_per_cohort + g * kTailRows,
                              slab * kTailCols, slab == 0, sm.t, waiter(2, true));
    }
    chain_end(sync + 96);
    SACMI_PHASE(tl, 4);
  }
  // L12 (dhp1) + the level's rides (the next update's sampler, Polyak): a workgroup whose
  // item is a ride reads nothing of the chain — it does not wait
  {
    const GemmBatch& b = chain_args(ca)->lv[3];
    const int items = b.total_tiles + (b.ride.kind ? b.ride.nblocks : 0) + b.ride.pk_blocks;
    if (bid < items)
      kg_body<32, 32, 16, 2, 1, false, 0, false, 0, kLdSc1, true>(b, bid, sm.a, waiter(3, bid < b.total_tiles));
    SACMI_PHASE(tl, 5);
  }
}

// the critic pass (ChainArgs kind 1): L1 / L2 on 32x64 tiles (L2 with the policy heads
// folded in), L3 / L4 on 32x32, L5 (row prologue, A transform) on 32x32
using ChainKgW = KgSmem<32, 64, 16, 2, 1, false, 0, false, 0, true>;   // (L2 carries the heads)
union ChainSmemA {
  ChainKgW w;
  ChainKgA a;
  ChainKgB b;
};

__global__ __launch_bounds__(1024, 4) void k_chain_a(const ChainArgs* __restrict__ ca, tl_word* tl) {
  const TlMark tl_mark(tl, TL_CHAIN_A);
  __shared__ ChainSmemA sm;
  SACMI_PHASE(tl, 0);   // (diagnostic builds: as k_chain's)
  const int c = blockIdx.x & (kChainCohorts - 1), bid = blockIdx.x;
  const int nmem = gridDim.x / kChainCohorts;
  int* const sync = chain_args(ca)->sync + c * (kChainBars + 1) * 32;
  int* const err = chain_args(ca)->err;
  const int target = chain_target(sync + kChainBars * 32, nmem);
  auto waiter = [&](int b, bool w) { return ChainWait{sync + b * 32, target, err, w, tl, 6 + b, 0}; };
  // L1: 32x64 tiles
  {
    const GemmBatch& b = chain_args(ca)->lv[0];
    if (bid < b.total_tiles) kg_body<32, 64, 16, 2, 1, false, 0, false, 0, kLdSc1, false, true>(b, bid, sm.w);
    chain_end(sync);
    SACMI_PHASE(tl, 1);
  }
  // L2 (+ the heads): 32x64 tiles, barrier 0 behind its weight loads
  {
    const GemmBatch& b = chain_args(ca)->lv[1];
    if (bid < b.total_tiles) kg_body<32, 64, 16, 2, 1, false, 0, false, 0, kLdSc1, true, true>(b, bid, sm.w, waiter(0, true));
    chain_end(sync + 32);
    SACMI_PHASE(tl, 2);
  }
  // L3, L4 (target critics): 32x32 tiles
#pragma unroll 1
  for (int i = 2; i < 4; ++i) {
    const GemmBatch& b = chain_args(ca)->lv[i];
    if (bid < b.total_tiles) kg_body<32, 32, 16, 2, 1, false, 0, false, 0, kLdSc1, true>(b, bid, sm.a, waiter(i - 1, true));
    chain_end(sync + 32 * i);
    SACMI_PHASE(tl, i + 1);
  }
  // L5: the critic row prologue (targets, MSE gradients, loss partials) + dh1
  {
    const GemmBatch& b = chain_args(ca)->lv[4];
    if (bid < b.total_tiles) kg_body<32, 32, 16, 2, 1, false, 1, false, 0, kLdSc1, true>(b, bid, sm.b, waiter(3, true));
    SACMI_PHASE(tl, 5);
  }
}

// 32x32 (TN = 64: 32x64) tiles, XCD-blocked with a row grid of 8: tile t of a desc -> row
// tile (t & 7) * tm / 8 + q, so workgroup b (b & 7 = cohort) only ever touches its cohort's rows
bool chain_assign_tiles(GemmBatch& b, int tn) {
  if (tn == 64) assign_tiles<32, 64>(b);
  else assign_tiles<32, 32>(b);
  for (int i = 0; i < b.count; ++i) {
    GemmDesc& d = b.d[i];
    if (d.tiles_m % kChainCohorts || d.tile_begin % kChainCohorts) return false;
    d.xcd_gr = kChainCohorts;
    d.pl_div = d.tiles_n;
    d.pl_gc_log2 = 0;
    d.pl_sr = d.tiles_m / kChainCohorts;
    d.pl_mag = d.pl_div == 1 ? 0u : (unsigned)((((uint64_t)1 << 32) + d.pl_div - 1) / d.pl_div);
  }
  return true;
}

// The grid must be resident at once (its cohorts wait for each other): one workgroup per CU
// on at least 256 CUs
bool chain_supported() {
  static int ok_dev[64] = {};   // 0 unknown, 1 yes, 2 no
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
  if (!ok_dev[dev]) {
    hipDeviceProp_t prop;
    int per_cu = 0;
    int per_cu_a = 0;
    const bool ok = hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount >= kChainGrid &&
                    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_chain, 1024, 0) == hipSuccess &&
                    per_cu >= 1 &&
                    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_a, k_chain_a, 1024, 0) == hipSuccess &&
                    per_cu_a >= 1;
    ok_dev[dev] = ok ? 1 : 2;
  }
  return ok_dev[dev] == 1;
}

bool chain_a_l2_ok(const GemmBatch& b) {
  return gemm_level_heads_fold_ok(b, b.heads.A);
}

bool launch_chain(const ChainArgs& h, const ChainArgs* dev, tl_word* tl, hipStream_t s) {
  if (!chain_supported()) return false;
  if (h.kind == 1) {
    // the critic pass: fp32 k_gemm bodies, L1 / L2 32x64 (L2 may fold the heads), L3 / L4
    // 32x32, L5 32x32 with the critic row prologue; no Adam, rides, split-K, bf16
    for (int i = 0; i < kChainLevels; ++i) {
      const GemmBatch& b = h.lv[i];
      if (b.count < 1 || b.bf16 || b.has_adam || b.err_flags || !b.st_wt || b.ride.kind || b.ride.pk_blocks ||
          (b.heads_ticket && i != 1) || b.total_tiles > kChainGrid)
        throw Error{SACMI_ESTATE, "k_chain_a: unsupported level configuration"};
      if (b.heads_ticket && b.heads.A * 2 > 48) throw Error{SACMI_ESTATE, "k_chain_a: heads wider than 48"};
      for (int q = 0; q < b.count; ++q) {
        const GemmDesc& d = b.d[q];
        if (d.axk != (i == 4 ? 1 : 0) || d.epi >= EPI_ADAM || d.a16 || d.b16 || d.c16 || d.x16 || d.pa_out ||
            d.xcd_gr != kChainCohorts || d.tiles_m % kChainCohorts || d.M != h.rows_per_cohort * kChainCohorts)
          throw Error{SACMI_ESTATE, "k_chain_a: unsupported GEMM in a chain level"};
        if (d.K > kChainMaxK) throw Error{SACMI_ESTATE, "k_chain_a: K beyond one pass"};
        if (d.tiles_n * (i < 2 ? 64 : 32) < d.N || (i < 2 && d.tiles_n * 32 >= d.N && d.N > 32))
          throw Error{SACMI_ESTATE, "k_chain_a: a level's tiles differ from the kernel's"};
      }
    }
    hipLaunchKernelGGL(k_chain_a, dim3(kChainGrid), dim3(1024), 0, s, dev, tl);
    HIP_LAUNCH_CHECK();
    return true;
  }
  // the configuration k_chain instantiates: fp32 32x32 k_gemm tiles (L9 with the A transform
  // and the dL/da partials), no fused Adam, no split-K / bf16 activations, rides on L12 only
  if (h.kind != 0) throw Error{SACMI_ESTATE, "k_chain: unknown chain kind"};
  for (int i = 0; i < 4; ++i) {
    const GemmBatch& b = h.lv[i];
    if (b.count < 1 || b.bf16 || b.has_adam || b.heads_ticket || b.err_flags || !b.st_wt)
      throw Error{SACMI_ESTATE, "k_chain: unsupported level configuration"};
    if ((b.ride.kind || b.ride.pk_blocks) && i != 3) throw Error{SACMI_ESTATE, "k_chain: rides outside L12"};
    if (b.ride.kind == 1 && mt_sample_lds_words(b.ride.tbl_log2, b.ride.mt.setsize) * 4 > kRideLdsBytes)
      throw Error{SACMI_ESTATE, "k_chain: ride-along sampler table exceeds the LDS"};
    for (int q = 0; q < b.count; ++q) {
      const GemmDesc& d = b.d[q];
      if (d.axk != (i == 2 ? 1 : 0) || d.epi >= EPI_ADAM || d.a16 || d.b16 || d.c16 || d.x16 ||
          d.xcd_gr != kChainCohorts || d.tiles_m % kChainCohorts || (d.pa_out && i != 2))
        throw Error{SACMI_ESTATE, "k_chain: unsupported GEMM in a chain level"};
      if (d.M != h.rows_per_cohort * kChainCohorts)
        throw Error{SACMI_ESTATE, "k_chain: a level's rows differ from the chain's batch"};
      if (d.K > kChainMaxK) throw Error{SACMI_ESTATE, "k_chain: K beyond one pass"};
    }
  }
  const SampleBwdArgs& a = h.tail;
  if (2 * a.A > 64 || kTailRows * a.A > 256 || h.n_pa > kTailMaxPa || a.hp2_16 || a.B != h.rows_per_cohort * kChainCohorts ||
      h.rows_per_cohort % kTailRows || h.tail_groups != h.rows_per_cohort / kTailRows ||
      h.tail_slabs != (a.H + kTailCols - 1) / kTailCols)
    throw Error{SACMI_ESTATE, "k_chain: unsupported sample-backward tail"};
  hipLaunchKernelGGL(k_chain, dim3(kChainGrid), dim3(1024), 0, s, dev, tl);
  HIP_LAUNCH_CHECK();
  return true;
}

bool gemm_level_on_axk16(const GemmBatch& b0) {
  GemmBatch b = b0;
  return SACMI_AXK_LDS16 && axk16_ok(b) >= 0;
}

// whether launch_gemm takes this forward level on <32, 64, 16, 2, 1> fp32 tiles with
// write-through stores: the configuration that folds the policy heads (GemmBatch::heads)
bool gemm_level_heads_fold_ok(const GemmBatch& b0, int A) {
  if (b0.bf16 || b0.count < 1 || 2 * A > 48 || A < 1) return false;
  GemmBatch b = b0;
  if (staged_ok(b) || fwd_big_ok(b)) return false;
  bool dw = true;
  int axk = 0, n_adam = 0;
  int64_t outs = 0;
  for (int i = 0; i < b.count; ++i) {
    const GemmDesc& d = b.d[i];
    dw = dw && !d.a_kc && !d.b_kc;
    axk = d.axk > axk ? d.axk : axk;
    n_adam += d.epi >= EPI_ADAM;
    outs += (int64_t)d.M * d.N;
    if (d.a16 || d.b16 || d.c16 || d.x16) return false;
    if (d.N > 1024) return false;   // (at most 16 column tiles' shares per row block)
  }
  const int t64 = assign_tiles<32, 64>(b);
  // launch_gemm's <32, 64, 16, 2, 1> branch, with write-through stores (st_wt: outs <= 1 M)
  return !dw && !n_adam && !axk && t64 >= 192 && t64 <= 512 && outs <= (1 << 20);
}

// launch_gemm's own kernel choice for an axk-1 level, asked ahead of its launch: true when
// it runs on the one-wave-group k_gemm tiles (<32, 32, 16, 2, 1, false, 1>: MG == 1, AXK ==
// 1), the only form that computes dL/da partials.  Mirrors launch_gemm's order: split-K and
// the LDS-staged forward kernels never take an axk level; k_axk16 (bf16, batch-4096 class);
// then the 64-row-tile branch (more than 512 32x64 tiles, e.g. batch 1024 with hidden > 512)
bool gemm_level_pa_capable(const GemmBatch& b0) {
  if (gemm_level_on_axk16(b0)) return false;
  GemmBatch b = b0;
  bool dw = true;
  int axk = 0, n_adam = 0;
  for (int i = 0; i < b.count; ++i) {
    dw = dw && !b.d[i].a_kc && !b.d[i].b_kc;
    axk = b.d[i].axk > axk ? b.d[i].axk : axk;
    n_adam += b.d[i].epi >= EPI_ADAM;
  }
  const int t64 = assign_tiles<32, 64>(b);
  if (dw || n_adam || t64 > 512) return false;
  return axk == 1;
}

// ---------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------------------
// Adam (torch.optim.Adam single-tensor semantics, torch optim/adam.py) over the
// flat arena, 4 elements per thread-iteration (every segment is a multiple of 4 floats
// and 16-byte aligned), + optional Polyak target update (sac_imp.py:146-152) + loss
// finalisation + the scalar log_alpha step and alpha = exp(log_alpha)
// (sac_imp.py:128-135) + the loss ring slot of this update.
__global__ __launch_bounds__(256) void k_adam(AdamArgs a) {
  const TlMark tl_mark(a.tl, TL_ADAM);
  __shared__ AdamScalars s_k[kMaxAdamSegs];
  __shared__ int64_t s_prefix[kMaxAdamSegs + 1];
  __shared__ int s_err;
  if (threadIdx.x < a.nseg) s_k[threadIdx.x] = adam_scalars(a, a.seg[threadIdx.x].step_idx);
  if (threadIdx.x == 0) {
    int64_t p = 0;
    for (int i = 0; i < a.nseg; ++i) { s_prefix[i] = p; p += a.seg[i].n / 4; }
    s_prefix[a.nseg] = p;
    int err = a.sc->err;
    if (a.err_flags) {
      // the flags summed over the ranks: a rank that saw a non-finite input makes every rank
      // void the same steps (block 0 records the remote bits for the rest of the stream)
      const int rb = (a.err_flags[0] > 0.f ? (int)ERR_REMOTE_SKIP : 0) |
                     (a.err_flags[1] > 0.f ? (int)ERR_REMOTE_ACT : 0);
      if (rb && blockIdx.x == 0) atomicOr(&a.sc->err, rb);
      err |= rb;
    }
    s_err = err;
  }
  __syncthreads();
  const float om_b1 = 1.f - a.beta1, om_b2 = 1.f - a.beta2, omtau = 1.f - a.tau;
  // a non-finite policy sample / PER draw of this update (ErrBits, see k_gemm): no step,
  // or (critic, actor-batch NaN) the step without Polyak
  const int err = s_err;
  if (err & a.err_skip) return;
  const bool pol = a.tgt && (err & a.err_nopolyak) == 0;
  const int64_t total4 = s_prefix[a.nseg];
  // parameter / moment / target arenas: one descriptor each (offsets < 2 GiB: the arenas
  // hold at most a few million floats)
  const rsrc_t rP = make_rsrc(a.p, 0x7fffffffu), rM = make_rsrc(a.m, 0x7fffffffu),
               rV = make_rsrc(a.v, 0x7fffffffu),
               rT = make_rsrc(a.tgt ? a.tgt : a.p, a.tgt ? 0x7fffffffu : 0u);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total4;
       e += (int64_t)gridDim.x * blockDim.x) {
    int sg = 0;
    for (int q = 1; q < a.nseg; ++q)
      if (e >= s_prefix[q]) sg = q;
    const int64_t i = a.seg[sg].off + 4 * (e - s_prefix[sg]);
    const AdamScalars k = s_k[sg];
    float4 g = *reinterpret_cast<const float4*>(a.g + i);
    float4 p = *reinterpret_cast<const float4*>(a.p + i);
    float4 m = *reinterpret_cast<const float4*>(a.m + i);
    float4 v = *reinterpret_cast<const float4*>(a.v + i);
    // the Polyak target with the other operands (one round trip: issued after the stores it
    // would wait for them), through a zero-length range where there is none
    float4 t = buf_ld4(rT, a.tgt ? (uint32_t)(i - a.tgt_base) * 4u : 0u);
    g.x *= a.grad_scale; g.y *= a.grad_scale; g.z *= a.grad_scale; g.w *= a.grad_scale;
    adam_elem(p.x, m.x, v.x, g.x, om_b1, a.beta2, om_b2, a.eps, k);
    adam_elem(p.y, m.y, v.y, g.y, om_b1, a.beta2, om_b2, a.eps, k);
    adam_elem(p.z, m.z, v.z, g.z, om_b1, a.beta2, om_b2, a.eps, k);
    adam_elem(p.w, m.w, v.w, g.w, om_b1, a.beta2, om_b2, a.eps, k);
    buf_st4<kStAux>(rP, (uint32_t)i * 4u, f4{p.x, p.y, p.z, p.w});
    buf_st4<kStAux>(rM, (uint32_t)i * 4u, f4{m.x, m.y, m.z, m.w});
    buf_st4<kStAux>(rV, (uint32_t)i * 4u, f4{v.x, v.y, v.z, v.w});
    if (a.ph) {
      st_wt(a.ph + i, bf16_bits(p.x)); st_wt(a.ph + i + 1, bf16_bits(p.y));
      st_wt(a.ph + i + 2, bf16_bits(p.z)); st_wt(a.ph + i + 3, bf16_bits(p.w));
    }
    if (pol) {
      t.x = polyak(t.x, p.x, omtau, a.tau);
      t.y = polyak(t.y, p.y, omtau, a.tau);
      t.z = polyak(t.z, p.z, omtau, a.tau);
      t.w = polyak(t.w, p.w, omtau, a.tau);
      buf_st4<kStAux>(rT, (uint32_t)(i - a.tgt_base) * 4u, f4{t.x, t.y, t.z, t.w});
      if (a.tgth) {
        unsigned short* th = a.tgth + (i - a.tgt_base);
        st_wt(th, bf16_bits(t.x)); st_wt(th + 1, bf16_bits(t.y));
        st_wt(th + 2, bf16_bits(t.z)); st_wt(th + 3, bf16_bits(t.w));
      }
    }
  }
  if (blockIdx.x != 0 || err) return;
  if (threadIdx.x == 0 && a.log_alpha_idx >= 0 && a.auto_entropy) {
    const AdamScalars k = adam_scalars(a, 3);
    const int64_t i = a.log_alpha_idx;
    float p = a.p[i], m = a.m[i], v = a.v[i];
    adam_elem(p, m, v, a.g[i] * a.grad_scale, om_b1, a.beta2, om_b2, a.eps, k);
    a.p[i] = p; a.m[i] = m; a.v[i] = v;
    a.sc->alpha = expf(p);
    a.sc->alpha_is_tensor = 1;
  }
  if (threadIdx.x < a.n_losses) {
    float s = 0.f;
    for (int w = 0; w < a.n_part; ++w) s += a.loss_part[w * a.n_losses + threadIdx.x];
    a.sc->losses[a.loss_slot0 + threadIdx.x] = s / a.loss_div;
  }
  __syncthreads();
  if (threadIdx.x == 0 && a.loss_ring) {
    const int64_t pos = a.sc->loss_ring_pos;
    const int64_t q = pos % a.ring;
    a.loss_ring[q * 3 + 0] = a.sc->losses[0];
    a.loss_ring[q * 3 + 1] = a.sc->losses[1];
    a.loss_ring[q * 3 + 2] = a.sc->losses[2];
    a.sc->loss_ring_pos = pos + 1;
  }
}

void launch_adam(const AdamArgs& a, hipStream_t s) {
  int64_t total4 = 0;
  for (int i = 0; i < a.nseg; ++i) total4 += a.seg[i].n / 4;
  int64_t blocks = (total4 + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks), dim3(256), 0, s, a);
  HIP_LAUNCH_CHECK();
}

__global__ __launch_bounds__(256) void k_polyak(PolyakArgs a) { polyak_ride(a, blockIdx.x, gridDim.x); }
void launch_polyak(const PolyakArgs& a, hipStream_t s) {
  int64_t blocks = (a.n4 + 511) / 512;     // polyak_ride: 2 groups per thread per pass
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k_polyak, dim3((unsigned)blocks), dim3(256), 0, s, a);
  HIP_LAUNCH_CHECK();
}

// the alpha step's visible result (k_adam block 0: sac_imp.py:135) on every rank of a sharded
// data-parallel update, from the all-gathered log_alpha
__global__ void k_alpha_sync(DevScalars* sc, const float* log_alpha, int err_skip) {
  if (threadIdx.x == 0 && (sc->err & err_skip) == 0) {
    sc->alpha = expf(*log_alpha);
    sc->alpha_is_tensor = 1;
  }
}
void launch_alpha_sync(DevScalars* sc, const float* log_alpha, int err_skip, hipStream_t s) {
  hipLaunchKernelGGL(k_alpha_sync, dim3(1), dim3(64), 0, s, sc, log_alpha, err_skip);
  HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
// replay gather: deque positions -> ring slots -> critic input [s|1|a] and the
// stacked policy input [s2|1|.. ; s|1|..]  (replay_buffer.py:15-19 + sac_imp.py:81-85)
__global__ __launch_bounds__(128) void k_gather(GatherArgs a) {
  const TlMark tl_mark(a.tl, TL_GATHER);
  gather_row(a, blockIdx.x, threadIdx.x, 128);
}

void launch_gather(const GatherArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_gather, dim3(a.B), dim3(128), 0, s, a);
  HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
__global__ void k_fill(float* p, int64_t n, float v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}
void launch_fill(float* p, int64_t n, float v, hipStream_t s) {
  if (n <= 0) return;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(k_fill, dim3((unsigned)blocks), dim3(256), 0, s, p, n, v);
  HIP_LAUNCH_CHECK();
}

__global__ void k_scale(float* p, int64_t n, float f) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] *= f;
}
void launch_scale(float* p, int64_t n, float f, hipStream_t s) {
  if (n <= 0) return;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(k_scale, dim3((unsigned)blocks), dim3(256), 0, s, p, n, f);
  HIP_LAUNCH_CHECK();
}

__global__ void k_set_column(float* p, int rows, int ld, int col, float v) {
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += gridDim.x * blockDim.x)
    p[(size_t)r * ld + col] = v;
}
void launch_set_column(float* p, int rows, int ld, int col, float v, hipStream_t s) {
  if (rows <= 0) return;
  int blocks = (rows + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(k_set_column, dim3(blocks), dim3(256), 0, s, p, rows, ld, col, v);
  HIP_LAUNCH_CHECK();
}

}  // namespace sacmi
