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
  uint32_t off[NT];
};

// H16: the operand is stored as bf16 (K-contiguous only: the policy heads' input under
// act16), fetched 4 k per 8-byte load and widened exactly to fp32
template <int NT, bool KC, bool H16 = false>
__device__ __forceinline__ void row_offs(const float* P, int ld, int row0, int nrows, int lane,
                                         OpFetch<NT>& f) {
  static_assert(!H16 || KC, "bf16 operands are K-contiguous");
  f.r = make_rsrc(P, 0x7fffffffu);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    int row = row0 + t * 16 + (lane & 15);
    row = row < nrows ? row : nrows - 1;
    f.off[t] = KC ? (uint32_t)row * (uint32_t)ld * (H16 ? 2u : 4u) : (uint32_t)row * 4u;
  }
}

__device__ __forceinline__ float bf16_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

template <int NT, bool KC, bool H16 = false>
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
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (KC) {
      const float4 x = buf_ld4(f.r, f.off[t] + (uint32_t)(k < K ? k : 0) * 4u);
      v[t][0] = (k < K) ? x.x : 0.f;
      v[t][1] = (k + 1 < K) ? x.y : 0.f;
      v[t][2] = (k + 2 < K) ? x.z : 0.f;
      v[t][3] = (k + 3 < K) ? x.w : 0.f;
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int kk = (k + s < K) ? (k + s) : (K - 1);
        const float x = buf_ld(f.r, f.off[t] + (uint32_t)kk * (uint32_t)ld * 4u);
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
template <int TM, int TN, int KSPLIT, int G, bool AKC, bool BKC, bool ROWSUM, int MG = 1,
          int AXF = 0, bool BF16 = false, bool A16 = false, class Pre>
__device__ __forceinline__ void gemm_core_l(const GemmDesc& d, int m0, int n0, float* red,
                                            float* rsum, Pre&& pre, bool store_a = false) {
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
  const int nmine = nch > ks ? (nch - ks + KSPLIT - 1) / KSPLIT : 0;
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
  if (nmine == 0) pre();
  for (int j = 0; j < nmine; j += G) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      // unconditional (see fetch_op; a guard, even a wave-uniform one, makes the compiler
      // drain the loads at the end of the guarded block): a group past the wave's last
      // chunk re-reads that chunk and is skipped below
      const int jj = j + g < nmine ? j + g : nmine - 1;
      const int k = (ks + jj * KSPLIT) * 16 + kl;
      fetch_op<MT, AKC, A16>(ra, d.lda, k, d.K, a[g]);
      fetch_op<NT, BKC>(rb, d.ldb, k, d.K, b[g]);
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
    if (j + G >= nmine) pre();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (j + g < nmine) {
        // no FMA contraction here: the scaled fragments feed both the MFMAs and the row
        // sums, and contracting a*f into a sum would make the row-sum bits depend on the
        // tile configuration's code generation
#pragma clang fp contract(off)
        if constexpr (AXF == 1) {
          const int k = (ks + (j + g) * KSPLIT) * 16 + kl;
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
        mfma_chunk<MT, NT, BF16>(acc, a[g], b[g]);
        if (ROWSUM) {
#pragma unroll
          for (int i = 0; i < MT; ++i) rs[i] += (a[g][i][0] + a[g][i][1]) + (a[g][i][2] + a[g][i][3]);
        }
      }
  }
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
template <int TM, int TN, int KSPLIT, int G, int MG, int AXK, bool BF16, class Pre>
__device__ __forceinline__ void gemm_core(const GemmDesc& d, int m0, int n0, float* red,
                                          float* rsum, bool rowsum, Pre&& pre) {
  if constexpr (AXK == 1) {
    if (d.axk == 1) {   // fc3 backward folded into dh1 / dha1 (A = h2, B = W2)
      gemm_core_l<TM, TN, KSPLIT, G, true, false, false, MG, 1, BF16>(d, m0, n0, red, rsum, pre,
                                                                    n0 == 0 && d.ax_out != nullptr);
      return;
    }
  }
  if (d.a_kc) {
    if (d.b_kc) gemm_core_l<TM, TN, KSPLIT, G, true, true, false, MG, 0, BF16>(d, m0, n0, red, rsum, pre);
    else gemm_core_l<TM, TN, KSPLIT, G, true, false, false, MG, 0, BF16>(d, m0, n0, red, rsum, pre);
  } else {
    if (d.b_kc) gemm_core_l<TM, TN, KSPLIT, G, false, true, false, MG, 0, BF16>(d, m0, n0, red, rsum, pre);
    else if (rowsum) gemm_core_l<TM, TN, KSPLIT, G, false, false, true, MG, 0, BF16>(d, m0, n0, red, rsum, pre);
    else gemm_core_l<TM, TN, KSPLIT, G, false, false, false, MG, 0, BF16>(d, m0, n0, red, rsum, pre);
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
// runs at the level's start (k_gemm: wave 0 of block 0 before its tile) — after the tile it made block 0 the level's last workgroup by 2.7-2.9 us (a chain
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
// ... after the block's work (the split-K weight-gradient finish, k_dw_fin): wave 0
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

template <int TMW, int NTH>
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
      x.pv[i] = buf_ld(rPart, ok && i < rf.nparts ? base + 4u * i : oob);
  }
  const int b = m0 + t;
  const uint32_t ob = (uint32_t)((t < TMW && b < rf.B) ? b : 0) * 4u;
  x.alpha = buf_ld(rSc, 0u);
  x.lp = buf_ld(rLp, ob);
  x.r = buf_ld(rR, ob);
  x.d = buf_ld(rD, ob);
  const int lane = t - TMW * nslot;
  x.lpa = buf_ld(rLpa, (uint32_t)(2 * (lane >= 0 && lane < rf.n_lp ? lane : 0) + 1) * 4u);
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
template <bool H16>
__device__ __forceinline__ float heads_elem(const HeadSampleArgs& a, int m, int j, float mean, float ls_raw,
                                            float eps_in, uint64_t ctr) {
  const int A = a.A;
  const float ls = fminf(fmaxf(ls_raw, -20.f), 2.f);
  const float sd = expf(ls);
  // Normal(mean, std) argument validation (networks_model1.py:87): loc must be real (not
  // NaN) and scale positive — std = exp(clamp(log_std)) is NaN only for a NaN log_std
  // (torch.clamp keeps NaN; fmaxf above does not, hence the raw value).  evaluate=True
  // (deterministic) builds no Normal, so nothing is checked there (sac_imp.py:59-65).
  if (a.nan_flag && !a.deterministic && (__builtin_isnan(mean) || __builtin_isnan(ls_raw))) {
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
  else
    a.act[(size_t)m * a.ldact + j] = y * a.scale + a.bias;
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
template <int TM>
__device__ __forceinline__ void heads_logp(const HeadSampleArgs& a, int m0, int part, float (*lp)[33],
                                           float* s_lp) {
  const int A = a.A;
  __syncthreads();
  if (threadIdx.x < TM) {
    const int mm = m0 + threadIdx.x;
    float s = 0.f;
    if (mm < a.rows) {
      for (int jj = 0; jj < A; ++jj) s += lp[threadIdx.x][jj];
      a.logp[mm] = s;
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


// TM x TN per wave group, MG wave groups (workgroup tile MG*TM x TN), K split KSPLIT
// ways inside each group; ADAM: fused optimizer epilogue (every desc EPI_ADAM*); BF16:
// bf16 MFMA operands (GemmBatch::bf16), everything around them fp32.  64*KSPLIT*MG threads.
template <int KSPLIT, int MG>
constexpr int gemm_threads() { return 64 * KSPLIT * MG; }
// LDS of one k_gemm configuration (kg_body)
template <int TM, int TN, int KSPLIT, int MG, int AXK>
struct KgSmem {
  static constexpr int TMW = TM * MG;
  static constexpr bool PA = AXK == 1 && MG == 1;
  float red[MG * KSPLIT * TM * (TN + 1)];
  float rsum[MG * KSPLIT * TM];
  AdamScalars s_k;
  int s_err;
  float s_q[TMW][4], s_coef[2][TMW], s_l[TMW][2], s_dotw[TN];
  float s_pa[PA ? TMW * (TN + 1) + TN * 32 : 1];
};

// The body of one k_gemm workgroup: work item `bid` of the level (a tile, a ride-along
// workgroup, the scalar Adam workgroup).
// The scalars that locate this workgroup's work come in ONE kernarg round trip: left to
// the compiler, each load sat behind a branch on the previous one (timeline pointer, tile
// count, one desc's tile_begin per loop trip, then the desc's fields as they were used),
// ~1-1.5 us of dependent scalar round trips before the first operand load of every level
// (phase stamps, tools/phase_dump.py).  The asm pins force each value into an SGPR
// there, so every load is issued before the one wait.
template <int TM, int TN, int KSPLIT, int G, int MG, bool ADAM, int AXK, bool BF16>
__device__ __forceinline__ void kg_body(const GemmBatch& batch, const int bid,
                                        KgSmem<TM, TN, KSPLIT, MG, AXK>& sm) {
  tl_word* const tl = batch.tl;
  const int n_tiles = batch.total_tiles, n_desc = batch.count;
  int tbeg[kMaxGemms];
#pragma unroll
  for (int q = 0; q < kMaxGemms; ++q) tbeg[q] = batch.d[q].tile_begin;
  asm volatile("" :: "s"(tl), "s"(n_tiles), "s"(n_desc));
#pragma unroll
  for (int q = 0; q < kMaxGemms; ++q) asm volatile("" :: "s"(tbeg[q]));
  // ... with the level-wide epilogue scalars that do not depend on the desc (the row
  // prologue's / fused Adam's pointers): otherwise their loads sit behind the desc's
  if constexpr (AXK == 1) {
    const RowsFuse& r = batch.rows;
    asm volatile("" :: "s"(r.part), "s"(r.logp), "s"(r.r), "s"(r.d), "s"(r.kind), "s"(r.nparts),
                 "s"(r.B), "s"(r.sc), "s"(r.logp_part), "s"(r.n_lp));
  } else if constexpr (ADAM) {
    const AdamFuse& a = batch.adam;
    asm volatile("" :: "s"(a.P), "s"(a.M), "s"(a.V), "s"(a.T), "s"(a.G), "s"(a.t_base), "s"(a.sc),
                 "s"(a.step_offset));
  }
  SACMI_PHASE(tl, 0);
  SACMI_PHASE_LAST(tl, 6);
  constexpr int TMW = TM * MG;
  float* const red = sm.red;
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
  if (bid >= n_tiles) {   // ride-along workgroups (next update's replay work, Polyak)
    if constexpr (gemm_threads<KSPLIT, MG>() == 1024) {   // the host attaches rides to 1024-thread configs
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
  // ... and, in the same round trip (one asm statement: every load issued before the one
  // wait), the fields the epilogue's buffer descriptors and scalars are formed from — the
  // compiler forms them before the K loop, behind branches on the fields: two or three more
  // dependent round trips before the first operand load otherwise (ISA)
#define SACMI_DESC_PIN_E "s"(d.C), "s"(d.aux), "s"(d.ldc), "s"(d.ldaux), "s"(d.epi), "s"(d.bias), \
    "s"(d.bias_ld), "s"(d.dotw), "s"(d.dotp), "s"(d.rs_col), "s"(d.axk), "s"(d.ax_w), "s"(d.ax_out), \
    "s"(d.ax_ld), "s"(d.a_ksc)
  if constexpr (ADAM) {
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
#undef SACMI_DESC_PIN_K
#undef SACMI_DESC_PIN_E
  SACMI_PHASE(batch.tl, 8);   // (diagnostic: the desc has landed)
  const int t = bid - tbeg[p];
  if (t >= d.tiles_m * d.tiles_n) return;   // padding to a multiple of 8 blocks
  int tr, tc;
  place_tile(d, t, tr, tc);
  const int m0 = tr * TMW, n0 = tc * TN;
  SACMI_PHASE(batch.tl, 9);   // (diagnostic: the tile is placed)
  if constexpr (ADAM) {
    // the level's scalar Adam work first, on wave 0 of block 0 (adam_block0_wave): the
    // other waves start their K loops, wave 0 follows ~3 us later, inside the tile's time
    if (bid == 0 && threadIdx.x < 64) {
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
  constexpr int NTH = gemm_threads<KSPLIT, MG>(), EPT = TMW * TN / NTH, NS = EPT + 1;
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
  const bool wt = batch.st_wt != 0;   // output store policy of this level
  const bool pol = d.epi == EPI_ADAM_POLYAK;
  // byte span of this desc's output (tile rows, plus the rowsum column; the fused-Adam
  // 4-column groups reach the row's padding up to a multiple of 4: ldc is one)
  const int ncov = ADAM ? (d.N + 3) & ~3 : d.N;
  const uint32_t span = (uint32_t)(((size_t)(d.M - 1) * d.ldc + (d.rs_col >= ncov ? d.rs_col + 1 : ncov)) * 4);
  const size_t abase = ADAM ? (size_t)(d.C - af.P) : 0;
  const rsrc_t rC = make_rsrc(d.C, span);
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
  auto pre = [&]() {
    if constexpr (ADAM) {
      if (threadIdx.x == 0) {
        s_k = fuse_scalars(af, d.adam_step, af.step_offset);
        s_err = af.sc->err;
      }
    }
    // axk 1: the row prologue's loads.  Issued here, behind the operand burst, and
    // consumed after the MFMAs: anything in flight at the k-loop header is waited for by
    // the back-edge's conservative vmcnt on the first iteration.
    if constexpr (AXK == 1) rows_load<TMW, NTH>(batch.rows, d, m0, rows_x);   // unconditional
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
        q0[s] = buf_ld4(rC, o); q1[s] = buf_ld4(rM, o); q2[s] = buf_ld4(rV, o);
        q3[s] = buf_ld4(rT, o);
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
        x0[s] = buf_ld(rX, o);
      }
    }
  };
  SACMI_PHASE(batch.tl, 1);
  gemm_core<TM, TN, KSPLIT, G, MG, AXK, BF16>(d, m0, n0, red, rsum, rowsum, pre);
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
  const int err = ADAM ? s_err : 0;
  const AdamScalars k_ad = s_k;
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
        buf_st_pol(rC, o, v, wt);
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
  store_err_flags(batch);
  SACMI_PHASE(batch.tl, 5);
}

template <int TM, int TN, int KSPLIT, int G, int MG, bool ADAM, int AXK = 0, bool BF16 = false>
__global__ __launch_bounds__((gemm_threads<KSPLIT, MG>()), 4) void k_gemm(GemmBatch batch) {
  // (4 waves per SIMD: 16 waves per CU, one 1024- or two 512-thread workgroups)
  const TlMark tl_mark(batch.tl, TL_GEMM);
  __shared__ KgSmem<TM, TN, KSPLIT, MG, AXK> sm;
  kg_body<TM, TN, KSPLIT, G, MG, ADAM, AXK, BF16>(batch, blockIdx.x, sm);
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
// Large-M forward levels (batch-4096 class) in bf16 mode: LDS-staged 128-row tiles.
// C = relu(A . W^T [+ b]) with both operands K-contiguous (activations [rows][K],
// nn.Linear weights [out][K]); [+ per-32-column fc3 dot partials].  The waves cover the
// tile over the FULL K (no K split, no partial-tile reduction): the workgroup stages K
// slabs of its A rows and W rows through LDS (the next slab's global loads in flight while
// this slab's MFMAs run) and every wave reads its fragments from LDS — each operand byte
// crosses L2->CU once per workgroup instead of once per wave.
constexpr int kFBM = 128, kFBN128 = 128;

__device__ __forceinline__ float swap_adj(float x) {   // lane ^ 1's x (DPP quad_perm 1,0,3,2)
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)bf16_bits(lo) | ((uint32_t)bf16_bits(hi) << 16);
}

// k_fwd16 / k_fwd16p epilogue: bias, ReLU, store, per-32-column fc3 dot partials.  A wave
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


// bf16 mode, bf16 in LDS: the staging rounds every fp32 operand ONCE per workgroup
// (v_cvt_pk_bf16_f32) and stores [row][k] bf16 slabs 64 deep; a lane's 8 consecutive k
// of one row are one ds_read_b128 and exactly its v_mfma_f32_16x16x32_bf16 operand
// (lane l: A[l&15][8(l>>4) + j], B[8(l>>4) + j][l&15]): one conversion per element per
// workgroup instead of per wave, one 16x16x32 MFMA per 32 k.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u2v __attribute__((ext_vector_type(2)));
constexpr int kHBK = 64, kHPad = 8;   // k_fwd16 slab depth, row pad

__device__ __forceinline__ u2v pack_bf16x4(float4 v) {
  const bf16x4 x = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
  return __builtin_bit_cast(u2v, x);
}

// AH (act16): A is bf16 (4 k per 8-byte load, straight into the slab) and C is bf16.
// Waves: 2 x fwd16_wc<kFBN>() of 64 x (kFBN / wc) sub-tiles
// 8 waves (4 per SIMD at two workgroups per CU) hide each other's LDS / barrier latency
// behind MFMAs: config 5 L1 / L2 28.8 / 25.4 -> 24.8 / 21.1 us, the 64-column levels
// L3 / L4 / L7 / L8 18.9 / 16.9 -> 16.4 / 14.7 (4 waves: one wave per SIMD per workgroup)
// (8 waves at either tile width: 128 columns as 2 x 4 waves of 64x32, 64 as 4 x 2 of 32x32)
template <int kFBN>
__host__ __device__ constexpr int fwd16_waves() { return 8; }
template <int kFBN, bool BH = false, bool AH = false>
__global__ __launch_bounds__(64 * fwd16_waves<kFBN>(), 2) void k_fwd16(GemmBatch batch) {
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
// fp32 forward levels of the batch-4096 class on bf16 MFMA: the exact three-way split
// ("x6").  gfx950 has no xf32 MFMA and its fp32 MFMA issues at 1/16 of the bf16 rate.  Each
// fp32 operand x is cut EXACTLY into three bf16 parts x = h + m + l by truncation (h: the
// top 8 significant bits; m: the next 8 of the remainder; l: the rest, at most 8 bits — both
// subtractions exact in fp32), once per workgroup as the slab is staged, into three bf16 LDS
// planes per operand.  a.b is then 9 cross products of exact parts; the 6 kept (hh, hm, mh,
// mm, hl, lh) are exact in the fp32 accumulator, the 3 dropped (ml, lm, ll) are below
// 2^-25 |a b| — under fp32's own unit roundoff: the result is as accurate as the fp32 MFMA
// chain (rounded differently, not bit-identical).  Per 32 k and 16x16 block: 6
// v_mfma_f32_16x16x32_bf16 (16 cycles each) for 8 v_mfma_f32_16x16x4_f32 (32 each).
// Round 6's register-split form at batch 256 (profiles/r06/x6_ab) paid the split per wave
// per fragment; here it is paid once per staged element.
// Tiles 128 x BN (BN 128 or 64), 8 waves as 4 x 2 sub-tiles of 32 x BN/2, full K in 32-deep
// slabs; one LDS buffer (the next slab's fp32 loads in flight in registers under the MFMAs,
// two barriers a slab) so that two workgroups share a CU.  Epilogue: k_fwd16's (bias, ReLU,
// fc3 dot partials, fp32 stores).
// LDS rows (k_fwd_x6's planes and k_axk_x6's A planes): unpadded 32-bf16 rows with an XOR
// chunk swizzle (below), conflict-free for the ds_read_b128 fragment reads and the staging
// stores alike, and 20-30 % less LDS than the padded 40 / 48-bf16 rows they replace
// (profiles/r06/x6_lds_rows_ab, x6_swizzle_ab)
constexpr int kX6K = 32, kX6Waves = 8;

// the three bf16 parts of four fp32 values, each part as four packed bf16 (k order kept)
__device__ __forceinline__ void x6_split4(float4 v, u2v& h, u2v& m, u2v& l) {
  const float x[4] = {v.x, v.y, v.z, v.w};
  uint32_t ph[2], pm[2], pl[2];
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    const float x0 = x[2 * d], x1 = x[2 * d + 1];
    const uint32_t u0 = __float_as_uint(x0), u1 = __float_as_uint(x1);
    ph[d] = __builtin_amdgcn_perm(u1, u0, 0x07060302u);
    const float r0 = x0 - __uint_as_float(u0 & 0xffff0000u);
    const float r1 = x1 - __uint_as_float(u1 & 0xffff0000u);
    const uint32_t v0 = __float_as_uint(r0), v1 = __float_as_uint(r1);
    pm[d] = __builtin_amdgcn_perm(v1, v0, 0x07060302u);
    const float s0 = r0 - __uint_as_float(v0 & 0xffff0000u);
    const float s1 = r1 - __uint_as_float(v1 & 0xffff0000u);
    pl[d] = __builtin_amdgcn_perm(__float_as_uint(s1), __float_as_uint(s0), 0x07060302u);
  }
  h = u2v{ph[0], ph[1]}; m = u2v{pm[0], pm[1]}; l = u2v{pl[0], pl[1]};
}

template <int BN>
__global__ __launch_bounds__(64 * kX6Waves, 2) void k_fwd_x6(GemmBatch batch) {
  const TlMark tl_mark(batch.tl, TL_FWD_X6);
  constexpr int NWV = kX6Waves, WC = 2, WR = NWV / WC;
  constexpr int MW = kFBM / WR, MI = MW / 16, NW = BN / WC, NT = NW / 16;
  static_assert(NT >= 2 && MI >= 1, "a wave covers whole 32-column dot blocks");
  // 64-B rows, each row's 16-B k chunks stored at chunk ^ ((row >> 2) & 2): the 16 lanes of
  // every ds_read_b128 lane group on 16 distinct 4-bank slots, the two rows of each
  // ds_write_b64 lane group on all 32 banks (profiles/r06/x6_swizzle_ab)
  constexpr int LDR = kX6K;
  constexpr int TPR = kX6K / 4;          // staging threads per row (4 k each)
  constexpr int RPP = 64 * NWV / TPR;    // rows per staging pass
  constexpr int NA = kFBM / RPP, NB = BN / RPP;
  static_assert(NA >= 1 && NB >= 1, "staging passes");
  __shared__ __attribute__((aligned(16))) __bf16 sA[3][kFBM][LDR];
  __shared__ __attribute__((aligned(16))) __bf16 sB[3][BN][LDR];
  auto cw = [](int r, int k) { return (((k >> 3) ^ ((r >> 2) & 2)) << 3) | (k & 7); };
  const int bid = blockIdx.x;
  int p = 0;
  for (int q = 1; q < batch.count; ++q)
    if (bid >= batch.d[q].tile_begin) p = q;
  const GemmDesc& d = batch.d[p];
  const int t = bid - d.tile_begin;
  if (t >= d.tiles_m * d.tiles_n) return;
  int tr, tc;
  place_tile(d, t, tr, tc);
  const int m0 = tr * kFBM, n0 = tc * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave / WC) * MW, wn = (wave % WC) * NW;
  const int M = d.M, N = d.N, K = d.K;
  const rsrc_t rA = make_rsrc(d.A, 0x7fffffffu), rB = make_rsrc(d.B, 0x7fffffffu);
  uint32_t offA[NA], offB[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i)
    offA[i] = (uint32_t)min(m0 + tid / TPR + RPP * i, M - 1) * (uint32_t)d.lda * 4u;
#pragma unroll
  for (int i = 0; i < NB; ++i)
    offB[i] = (uint32_t)min(n0 + tid / TPR + RPP * i, N - 1) * (uint32_t)d.ldb * 4u;
  const int kq = 4 * (tid % TPR);
  float4 ga[NA], gb[NB];
  auto zk = [&](float4 x, int k) {    // elements past K read the row's next columns: zeroed
    x.x = k < K ? x.x : 0.f; x.y = k + 1 < K ? x.y : 0.f; x.z = k + 2 < K ? x.z : 0.f; x.w = k + 3 < K ? x.w : 0.f;
    return x;
  };
  auto gload = [&](int k0) {
    const int k = k0 + kq;
    const uint32_t ko = (uint32_t)(k < K ? k : 0) * 4u;
#pragma unroll
    for (int i = 0; i < NA; ++i) ga[i] = zk(buf_ld4(rA, offA[i] + ko), k);
#pragma unroll
    for (int i = 0; i < NB; ++i) gb[i] = zk(buf_ld4(rB, offB[i] + ko), k);
  };
  auto swrite = [&]() {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      u2v h, m, l;
      x6_split4(ga[i], h, m, l);
      const int r = tid / TPR + RPP * i, c = cw(r, kq);
      *reinterpret_cast<u2v*>(&sA[0][r][c]) = h;
      *reinterpret_cast<u2v*>(&sA[1][r][c]) = m;
      *reinterpret_cast<u2v*>(&sA[2][r][c]) = l;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      u2v h, m, l;
      x6_split4(gb[i], h, m, l);
      const int r = tid / TPR + RPP * i, c = cw(r, kq);
      *reinterpret_cast<u2v*>(&sB[0][r][c]) = h;
      *reinterpret_cast<u2v*>(&sB[1][r][c]) = m;
      *reinterpret_cast<u2v*>(&sB[2][r][c]) = l;
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
  swrite();
  __syncthreads();
  const int nslab = (K + kX6K - 1) / kX6K;
  const int kc = cw(lane & 15, 8 * (lane >> 4));   // (row blocks start at multiples of 16)
  for (int sl = 0; sl < nslab; ++sl) {
    if (sl + 1 < nslab) gload((sl + 1) * kX6K);
    // the A parts of every row block, then each B column block's parts just before its
    // MFMAs (one B block's parts live at a time); small terms first into the accumulator
    bf16x8 ah[MI], am[MI], al[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int r = wm + i * 16 + (lane & 15);
      ah[i] = *reinterpret_cast<const bf16x8*>(&sA[0][r][kc]);
      am[i] = *reinterpret_cast<const bf16x8*>(&sA[1][r][kc]);
      al[i] = *reinterpret_cast<const bf16x8*>(&sA[2][r][kc]);
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int r = wn + j * 16 + (lane & 15);
      const bf16x8 bh = *reinterpret_cast<const bf16x8*>(&sB[0][r][kc]);
      const bf16x8 bm = *reinterpret_cast<const bf16x8*>(&sB[1][r][kc]);
      const bf16x8 bl = *reinterpret_cast<const bf16x8*>(&sB[2][r][kc]);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        f4 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[i], bm, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[i], bh, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bm, c, 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh, c, 0, 0, 0);
      }
    }
    if (sl + 1 < nslab) {
      __syncthreads();   // every wave's fragment reads of this slab done
      swrite();
      __syncthreads();
    }
  }
  ep.store(d, acc, m0 + wm, n0 + wn, lane);
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

template <int BM>
__global__ __launch_bounds__(1024, 1) void k_fwd16p(GemmBatch batch) {
  constexpr int NWV = 16;
  const TlMark tl_mark(batch.tl, TL_FWD16P);
  constexpr int BN = 128, BK = 64, NST = fwd16p_stages<BM>();
  // NWV waves as WR x WC = 4 x 4 of (BM/4) x 32
  constexpr int WR = 4, WC = NWV / WR;
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
  if (!b.bf16 || b.ride.kind) return 0;
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
  b.st_wt = 1;   // write-through epilogue stores
  if (assign_tiles<256, 128>(b) >= 256) return 256;
  if (assign_tiles<128, 128>(b) >= 256) return 128;
  return 0;
}

// ---------------------------------------------------------------------------
// Deep-K weight-gradient levels in bf16 mode (batch 4096 class): dW = dY^T X with both
// operands row-contiguous.  k_dw_part16: 128x128 output tiles, K split NS ways across
// workgroups; each workgroup stages slabs of dY (128 columns) and X (128 columns)
// through LDS and writes its partial tile (+ the bias-gradient row-sum partial) to a
// workspace.  k_dw_fin: one thread per output element sums the NS partials
// in fixed order and runs the epilogue (store, or Adam [+ Polyak] with the gradient export
// and block 0's loss / alpha extras) — both forms of a level take this path, so the
// fused and the data-parallel updates keep identical bits.
constexpr int kDBM = 128, kDBN = 128;
constexpr int kDwTarget = 512;   // k_dw_part16 workgroup slots (256 CUs x 2)
constexpr int kDwMaxSplit = 16;
constexpr int kDwFinEpt = 1;     // k_dw_fin 4-column groups per thread (1, 2, 4 measured alike)

// workspace layout: partial s of desc p at ws + s * ws_stride + desc_off[p], row-major
// [M][ncols] with ncols = N (+1 for the row-sum column) rounded up to a multiple of 4: every
// partial row starts 16-byte aligned, so k_dw_fin moves 4-column groups (the pad columns are
// never written and never used)
__host__ __device__ __forceinline__ int dw_ncols_real(const GemmDesc& d) { return d.rs_col >= 0 ? d.N + 1 : d.N; }
__host__ __device__ __forceinline__ int dw_ncols(const GemmDesc& d) { return (dw_ncols_real(d) + 3) & ~3; }

// XCD placement of the split-K work (workgroup b runs on XCD b % 8): the split-major work
// list w = split * tiles + tile is dealt to the XCDs in contiguous eighths, so each XCD's
// L2 streams the rows of one or two K ranges instead of every range.  The tile grid is
// padded to a multiple of 8 workgroups.
__host__ __device__ __forceinline__ int dw_grid_tiles(int tiles, int ns) { return (tiles * ns + 7) / 8 * 8; }
__device__ __forceinline__ int dw_work_index(int b, int tiles, int ns) {
  const int W = tiles * ns, per = (W + 7) / 8;
  const int w = (b % 8) * per + b / 8;
  return w < W ? w : -1;
}

// bf16 mode, bf16 in LDS: the operands are rounded once at staging and kept
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
// waves per k_dw_part16 workgroup: 2 x 4 of 64x32 sub-tiles
constexpr int kDw16Waves = 8, kDw16Krp = 64 * kDw16Waves / 32;   // k rows per staging pass
static_assert(kDw16LdsBytes >= 2 * kDw16OpBytes + kDw16Krp * kDBM * 4, "k_dw_part16 LDS layout");

__device__ __forceinline__ s4t lds_tr16(const __bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s4t*)(p));
}

// X16 (act16): the B operand (X: activations / minibatch inputs) is bf16
template <bool X16 = false>
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
      float4 x = buf_ld4(rA, ea * 4u);
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

// fp32 mode, batch-4096 class: the deep-K weight-gradient partials on bf16 MFMA with the
// exact three-way split (k_fwd_x6's form on k_dw_part16's structure): 128x128 output tiles,
// K (the batch) split NS ways across workgroups, 32-deep slabs of dY (x the K-scale) and X
// cut once per workgroup into three bf16 planes each, [k][column] in LDS and read transposed
// (ds_read_b64_tr_b16); the bias-gradient row sums from the unrounded fp32 staging registers;
// the partial tile to the workspace for k_dw_fin.  One LDS buffer (the next slab's fp32 loads
// in registers), two workgroups per CU.
constexpr int kDX6K = 32;
__global__ __launch_bounds__(64 * kDw16Waves, 2) void k_dw_part_x6(GemmBatch batch, int ns, int64_t ws_stride) {
  const TlMark tl_mark(batch.tl, TL_DW_PART_X6);
  constexpr int LDR = kDBM + kD16Pad;          // bf16 per LDS k row (272 B)
  constexpr int PL = kDX6K * LDR;              // one plane
  __shared__ __attribute__((aligned(16))) unsigned char lds_raw[kDw16LdsBytes];
  __bf16* const sAp = reinterpret_cast<__bf16*>(lds_raw);              // [3][kDX6K][LDR]
  __bf16* const sBp = sAp + 3 * PL;
  auto& s_rs = *reinterpret_cast<float (*)[kDw16Krp][kDBM]>(lds_raw + 6 * PL * 2);
  static_assert(6 * PL * 2 + kDw16Krp * kDBM * 4 <= kDw16LdsBytes, "k_dw_part_x6 LDS layout");
  constexpr int NWV = kDw16Waves, WC = NWV / 2, NJ = kDBN / WC / 16;   // 2 x WC waves of 64 x (128 / WC)
  constexpr int KRP = kDw16Krp, NI = kDX6K / KRP;                      // staging: KRP k rows a pass
  static_assert(NI >= 1, "k_dw_part_x6 staging");
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
  // the split's K range in whole 64-deep units (k_dw_part16's ranges: the same partition)
  const int kc = ((K + ns - 1) / ns + kD16K - 1) / kD16K * kD16K;
  const int kb = split * kc, ke = min(K, kb + kc);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave / WC) * 64, wn = (wave % WC) * (kDBN / WC);
  const int c4 = 4 * (tid & 31), kr0 = tid >> 5;
  const rsrc_t rA = make_rsrc(d.A, 0x7fffffffu), rB = make_rsrc(d.B, 0x7fffffffu);
  const rsrc_t rS = make_rsrc(d.a_ksc ? d.a_ksc : d.A, d.a_ksc ? (uint32_t)K * 4u : 0u);
  const bool has_ksc = d.a_ksc != nullptr;
  const int ma = min(m0 + c4, (M - 1) & ~3), nb = min(n0 + c4, (N - 1) & ~3);
  const bool want_rs = d.rs_col >= 0 && n0 == 0;
  float4 ga[NI], gb[NI];
  float rs4[4] = {0.f, 0.f, 0.f, 0.f};
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int k = k0 + kr0 + KRP * i;
      const bool kin = k < ke;
      const uint32_t kk = (uint32_t)(kin ? k : 0);
      float4 x = buf_ld4(rA, (kk * (uint32_t)d.lda + (uint32_t)ma) * 4u);
      const float f = has_ksc ? buf_ld(rS, kk * 4u) : 1.f;
      x.x = kin && m0 + c4 < M ? x.x * f : 0.f;     x.y = kin && m0 + c4 + 1 < M ? x.y * f : 0.f;
      x.z = kin && m0 + c4 + 2 < M ? x.z * f : 0.f; x.w = kin && m0 + c4 + 3 < M ? x.w * f : 0.f;
      ga[i] = x;
      float4 y = buf_ld4(rB, (kk * (uint32_t)d.ldb + (uint32_t)nb) * 4u);
      y.x = kin && n0 + c4 < N ? y.x : 0.f;         y.y = kin && n0 + c4 + 1 < N ? y.y : 0.f;
      y.z = kin && n0 + c4 + 2 < N ? y.z : 0.f;     y.w = kin && n0 + c4 + 3 < N ? y.w : 0.f;
      gb[i] = y;
    }
  };
  auto swrite = [&]() {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int r = kr0 + KRP * i;
      u2v h, m, l;
      x6_split4(ga[i], h, m, l);
      *reinterpret_cast<u2v*>(sAp + 0 * PL + r * LDR + c4) = h;
      *reinterpret_cast<u2v*>(sAp + 1 * PL + r * LDR + c4) = m;
      *reinterpret_cast<u2v*>(sAp + 2 * PL + r * LDR + c4) = l;
      x6_split4(gb[i], h, m, l);
      *reinterpret_cast<u2v*>(sBp + 0 * PL + r * LDR + c4) = h;
      *reinterpret_cast<u2v*>(sBp + 1 * PL + r * LDR + c4) = m;
      *reinterpret_cast<u2v*>(sBp + 2 * PL + r * LDR + c4) = l;
    }
    if (want_rs) {
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
  const int nslab = (ke - kb + kDX6K - 1) / kDX6K;
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg = lane >> 4;
  const int kr = 8 * tg + tq;
  auto frag = [&](const __bf16* plane, int col) {   // transposed 16x32 fragment at column col
    const s4t lo = lds_tr16(plane + kr * LDR + col);
    const s4t hi = lds_tr16(plane + (kr + 4) * LDR + col);
    const s8t v = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    return __builtin_bit_cast(bf16x8, v);
  };
  if (nslab > 0) {
    gload(kb);
    swrite();
    __syncthreads();
  }
  for (int sl = 0; sl < nslab; ++sl) {
    if (sl + 1 < nslab) gload(kb + (sl + 1) * kDX6K);
    bf16x8 ah[4], am[4], al[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = wm + i * 16 + 4 * tp;
      ah[i] = frag(sAp, col);
      am[i] = frag(sAp + PL, col);
      al[i] = frag(sAp + 2 * PL, col);
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = wn + j * 16 + 4 * tp;
      const bf16x8 bh = frag(sBp, col), bm = frag(sBp + PL, col), bl = frag(sBp + 2 * PL, col);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        f4 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[i], bm, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[i], bh, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bm, c, 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh, c, 0, 0, 0);
      }
    }
    if (sl + 1 < nslab) {
      __syncthreads();   // every wave's fragment reads of this slab done
      swrite();
      __syncthreads();
    }
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
    __syncthreads();
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
constexpr int kAxWaves = 8;   // waves per k_axk16 workgroup: 2 x 4 of 32x32 sub-tiles
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
  // a tile wholly inside N and a slab wholly inside K stage without the edge masks (rows past
  // M read the clamped last row, as in the masked form; their outputs are never stored)
  const bool n_in = n0 + kXBN <= N;
  auto gload = [&](int k0) {
    const int k = k0 + kq;
    const uint32_t ko = (uint32_t)(k < K ? k : 0) * 4u;
    if (n_in && k0 + kXBK <= K) {
#pragma unroll
      for (int i = 0; i < NAI; ++i) {
        if constexpr (A16) {
          const uint2 h = buf_ld2(rA, offA[i] + ko / 2u);
          ga[i] = make_float4(bf16_lo(h.x), bf16_hi(h.x), bf16_lo(h.y), bf16_hi(h.y));
        } else {
          ga[i] = buf_ld4(rA, offA[i] + ko);
        }
      }
      gw = buf_ld4(rW, ko);
#pragma unroll
      for (int i = 0; i < NBI; ++i) {
        const uint32_t e = (uint32_t)(k0 + kr0 + BKP * i) * (uint32_t)d.ldb + (uint32_t)nb;
        if constexpr (BH) gh[i] = buf_ld2(rBh, e * 2u);
        else gb[i] = buf_ld4(rB, e * 4u);
      }
      return;
    }
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
    const bool k_in = k0 + kXBK <= K;
#pragma unroll
    for (int i = 0; i < NAI; ++i) {
      // u = [h2 > 0] w3 (exact fp32 values: w3 or 0), rounded to bf16 for the MFMAs
      const float4 a = ga[i];
      const float4 u = k_in ? (AX ? make_float4(a.x > 0.f ? gw.x : 0.f, a.y > 0.f ? gw.y : 0.f,
                                                a.z > 0.f ? gw.z : 0.f, a.w > 0.f ? gw.w : 0.f)
                                  : a)
                     : AX ? make_float4(a.x > 0.f && k < K ? gw.x : 0.f, a.y > 0.f && k + 1 < K ? gw.y : 0.f,
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

// fp32 dh levels of the batch-4096 class on bf16 MFMA with the exact three-way split
// (k_fwd_x6's form on k_axk16's structure): dh[b][n] = coef[b] * sum_k u[b][k] W[k][n] *
// [h[b][n] > 0] with u = [h2 > 0] w3 formed at staging (its exact fp32 rows stored by the
// column-tile-0 workgroups for the layer's weight gradient; the row prologue and coefficients
// as k_axk16 / k_gemm's, so the losses and dq bits do not depend on the kernel), or (AX =
// false) the plain dh = (dY W) * [h > 0].  64 x 128 tiles, 8 waves of 32 x 32, 32-deep slabs
// split once per workgroup into three bf16 planes per operand: A [row][k], B = W k-major
// [k][n] read transposed (ds_read_b64_tr_b16); one LDS buffer, two workgroups per CU.
// (BN: the tile width — 128, or 64 for a one-net level, which then gets two workgroups per CU)
constexpr int kXX6K = 32;
template <bool AX, int BN = kXBN>
__global__ __launch_bounds__(64 * kAxWaves, 2) void k_axk_x6(GemmBatch batch) {
  const TlMark tl_mark(batch.tl, TL_AXK_X6);
  // [row][k] bf16, 64-B rows with k_fwd_x6's chunk swizzle (profiles/r06/x6_swizzle_ab)
  constexpr int LDA_ = kXX6K;
  auto cw = [](int r, int k) { return (((k >> 3) ^ ((r >> 2) & 2)) << 3) | (k & 7); };
  constexpr int LDB_ = BN + 8;          // [k][n] bf16
  __shared__ __attribute__((aligned(16))) __bf16 sA[3][kXBM][LDA_];
  __shared__ __attribute__((aligned(16))) __bf16 sB[3][kXX6K][LDB_];
  __shared__ float s_q[kXBM][4], s_coef[2][kXBM], s_l[kXBM][2];
  constexpr int NWV = kAxWaves, NTH = 64 * NWV, WC = NWV / 2, NJ = BN / WC / 16;
  constexpr int TPRA = kXX6K / 4, ARP = NTH / TPRA, NAI = kXBM / ARP;   // A staging
  constexpr int TPRB = BN / 4, BKP = NTH / TPRB, NBI = kXX6K / BKP;     // B staging
  static_assert(NAI >= 1 && NBI >= 1 && NJ >= 1, "k_axk_x6 staging");
  const int bid = blockIdx.x;
  if (bid >= batch.total_tiles) {   // ride-along: the next update's gather, a row a wave
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
  const int m0 = tr * kXBM, n0 = tc * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave / WC) * 32, wn = (wave % WC) * (BN / WC);
  const int M = d.M, N = d.N, K = d.K;
  const rsrc_t rA = make_rsrc(d.A, 0x7fffffffu), rB = make_rsrc(d.B, 0x7fffffffu);
  const rsrc_t rW = make_rsrc(AX ? d.ax_w : d.A, AX ? (uint32_t)K * 4u : 0u);
  const bool store_a = AX && n0 == 0 && d.ax_out != nullptr;
  const rsrc_t rAx = make_rsrc(store_a ? d.ax_out : d.C,
                               store_a ? (uint32_t)(((size_t)(M - 1) * d.ax_ld + K) * 4) : 0u);
  // A staging: rows tid / TPRA + ARP i at k = 4 (tid % TPRA); B staging: k rows
  // tid / TPRB + BKP i at columns 4 (tid % TPRB)
  const int kq = 4 * (tid % TPRA), c4 = 4 * (tid % TPRB), kr0 = tid / TPRB;
  uint32_t offA[NAI];
#pragma unroll
  for (int i = 0; i < NAI; ++i)
    offA[i] = (uint32_t)min(m0 + tid / TPRA + ARP * i, M - 1) * (uint32_t)d.lda * 4u;
  const int nb = min(n0 + c4, N - 1);
  float4 ga[NAI], gb[NBI], gw;
  auto gload = [&](int k0) {
    const int k = k0 + kq;
    const uint32_t ko = (uint32_t)(k < K ? k : 0) * 4u;
#pragma unroll
    for (int i = 0; i < NAI; ++i) ga[i] = buf_ld4(rA, offA[i] + ko);
    gw = buf_ld4(rW, ko);
#pragma unroll
    for (int i = 0; i < NBI; ++i) {
      const int kb = k0 + kr0 + BKP * i;
      const bool kin = kb < K;
      float4 y = buf_ld4(rB, ((uint32_t)(kin ? kb : 0) * (uint32_t)d.ldb + (uint32_t)nb) * 4u);
      y.x = kin && n0 + c4 < N ? y.x : 0.f;         y.y = kin && n0 + c4 + 1 < N ? y.y : 0.f;
      y.z = kin && n0 + c4 + 2 < N ? y.z : 0.f;     y.w = kin && n0 + c4 + 3 < N ? y.w : 0.f;
      gb[i] = y;
    }
  };
  auto swrite = [&](int k0, bool fresh) {
    const int k = k0 + kq;
#pragma unroll
    for (int i = 0; i < NAI; ++i) {
      // u = [h2 > 0] w3 (exact fp32 values: w3 or 0)
      const float4 a = ga[i];
      const float4 u = AX ? make_float4(a.x > 0.f && k < K ? gw.x : 0.f, a.y > 0.f && k + 1 < K ? gw.y : 0.f,
                                        a.z > 0.f && k + 2 < K ? gw.z : 0.f, a.w > 0.f && k + 3 < K ? gw.w : 0.f)
                          : make_float4(k < K ? a.x : 0.f, k + 1 < K ? a.y : 0.f,
                                        k + 2 < K ? a.z : 0.f, k + 3 < K ? a.w : 0.f);
      const int r = tid / TPRA + ARP * i;
      u2v h, m, l;
      x6_split4(u, h, m, l);
      *reinterpret_cast<u2v*>(&sA[0][r][cw(r, kq)]) = h;
      *reinterpret_cast<u2v*>(&sA[1][r][cw(r, kq)]) = m;
      *reinterpret_cast<u2v*>(&sA[2][r][cw(r, kq)]) = l;
      if (fresh) {
        const int rr = m0 + r;
        buf_st4(rAx, (rr < M && k < K) ? (uint32_t)(rr * d.ax_ld + k) * 4u : 0xfffffff0u,
                f4{u.x, u.y, u.z, u.w});
      }
    }
#pragma unroll
    for (int i = 0; i < NBI; ++i) {
      u2v h, m, l;
      x6_split4(gb[i], h, m, l);
      *reinterpret_cast<u2v*>(&sB[0][kr0 + BKP * i][c4]) = h;
      *reinterpret_cast<u2v*>(&sB[1][kr0 + BKP * i][c4]) = m;
      *reinterpret_cast<u2v*>(&sB[2][kr0 + BKP * i][c4]) = l;
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
    const rsrc_t rX = make_rsrc(d.aux, (uint32_t)(((size_t)(M - 1) * d.ldaux + N) * 4u));
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + i * 16 + (lane >> 4) * 4 + r;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int col = n0 + wn + j * 16 + (lane & 15);
          hm[i][j][r] = buf_ld(rX, row < M && col < N ? (uint32_t)(row * d.ldaux + col) * 4u : 0xfffffff0u);
        }
      }
  }
  swrite(0, store_a);
  __syncthreads();
  const int nslab = (K + kXX6K - 1) / kXX6K;
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg = lane >> 4;
  const int kc = 8 * tg, kca = cw(lane & 15, kc);
  for (int sl = 0; sl < nslab; ++sl) {
    if (sl + 1 < nslab) gload((sl + 1) * kXX6K);
    bf16x8 ah[2], am[2], al[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = wm + i * 16 + (lane & 15);
      ah[i] = *reinterpret_cast<const bf16x8*>(&sA[0][r][kca]);
      am[i] = *reinterpret_cast<const bf16x8*>(&sA[1][r][kca]);
      al[i] = *reinterpret_cast<const bf16x8*>(&sA[2][r][kca]);
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      bf16x8 bp[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const s4t lo = lds_tr16(&sB[q][kc + tq][wn + j * 16 + 4 * tp]);
        const s4t hi = lds_tr16(&sB[q][kc + tq + 4][wn + j * 16 + 4 * tp]);
        const s8t v = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        bp[q] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        f4 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bp[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bp[2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[i], bp[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am[i], bp[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bp[1], c, 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bp[0], c, 0, 0, 0);
      }
    }
    if (sl + 1 < nslab) {
      __syncthreads();   // every wave's fragment reads of this slab done
      swrite((sl + 1) * kXX6K, store_a);
      __syncthreads();
    }
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

// whether launch_gemm may run an fp32 level on k_axk_x6: k_axk16's level form in fp32 mode
// (-1: no; else bit 0: the row-prologue form, bit 1: 64-wide tiles)
static int axk_x6_ok(GemmBatch& b) {
  if (b.bf16 || (b.ride.kind && b.ride.kind != 2) || b.ride.pk_blocks || b.has_adam) return -1;
  const int ax = b.d[0].axk == 1 ? 1 : 0;
  if (ax != (b.rows.kind != 0 ? 1 : 0)) return -1;
  for (int i = 0; i < b.count; ++i) {
    const GemmDesc& d = b.d[i];
    if (d.axk != ax || !d.a_kc || d.b_kc || d.epi != EPI_MASK || d.bias || d.dotp || d.a_ksc ||
        d.rs_col >= 0 || d.pa_out || d.a16 || d.b16 || d.c16 || d.x16)
      return -1;
    if (((uintptr_t)d.A & 15) || (d.lda & 3) || ((uintptr_t)d.B & 15) || (d.ldb & 3) ||
        (ax && ((uintptr_t)d.ax_w & 15)) || (d.N & 3))
      return -1;
  }
  // two workgroups per CU: 128-wide tiles where they give 512, else 64-wide ones (a one-net
  // level: the policy's dhp1; at 128 wide its 256 tiles measured slower than its k_gemm
  // form, config 3 L12 28.0-29.5 vs 27.1-27.2 us)
  if (assign_tiles<kXBM, kXBN>(b) >= 512) return ax;
  return assign_tiles<kXBM, 64>(b) >= 512 ? ax | 2 : -1;
}

static void launch_axk_x6(const GemmBatch& b, int form, hipStream_t s) {
  const dim3 grid(b.total_tiles + (b.ride.kind ? b.ride.nblocks : 0)), blk(64 * kAxWaves);
  switch (form) {
    case 0: hipLaunchKernelGGL((k_axk_x6<false>), grid, blk, 0, s, b); break;
    case 1: hipLaunchKernelGGL((k_axk_x6<true>), grid, blk, 0, s, b); break;
    case 2: hipLaunchKernelGGL((k_axk_x6<false, 64>), grid, blk, 0, s, b); break;
    default: hipLaunchKernelGGL((k_axk_x6<true, 64>), grid, blk, 0, s, b); break;
  }
  HIP_LAUNCH_CHECK();
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

// 1 when the level carries bf16 activation operands (any GemmDesc a16 / b16 / c16 / x16);
// each kernel that takes them checks the per-desc pattern it supports
static int level_act16(const GemmBatch& b) {
  int any = 0;
  for (int i = 0; i < b.count; ++i) any |= b.d[i].a16 | b.d[i].b16 | b.d[i].c16 | b.d[i].x16;
  return any ? 1 : 0;
}

// bf16 deep-K weight-gradient levels: split count and workspace need, or 0 (k_gemm)
static int dw_split_plan(GemmBatch& b, int64_t* stride) {
  if (!b.ws) return 0;   // (bf16: k_dw_part16; fp32: k_dw_part_x6)
  int64_t el = 0;
  int tiles = 0;
  for (int i = 0; i < b.count; ++i) {
    GemmDesc& d = b.d[i];
    if (d.a_kc || d.b_kc || d.K < 2048 || d.axk) return 0;
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
  int ns = kDwTarget / tiles;
  ns = ns < 1 ? 1 : ns > kDwMaxSplit ? kDwMaxSplit : ns;
  if ((int64_t)ns * el > b.ws_floats) return 0;
  *stride = el;
  return ns;
}

// whether launch_gemm may run a level on k_fwd16 / k_fwd16p: bf16 plain forward GEMMs
// (both operands K-contiguous, store / ReLU epilogue, optional bias and dot partials), no
// prologue, no rides, and enough 128-row tiles to fill the chip.  (fp32 levels: the
// 512-thread K-split k_gemm tiles measured faster — config 3: 1,351 vs 1,229 updates/s;
// with bf16 MFMAs the levels are operand-traffic bound and the LDS sharing wins — config 5:
// 1,381 -> 1,458.)
static bool fwd_big_ok(GemmBatch& b) {
  if (b.ride.kind || !b.bf16) return false;
  for (int i = 0; i < b.count; ++i) {
    const GemmDesc& d = b.d[i];
    if (!d.a_kc || !d.b_kc || d.axk || d.a_ksc || d.rs_col >= 0) return false;
    if (((uintptr_t)d.A & (d.a16 ? 7 : 15)) || (d.lda & 3) || ((uintptr_t)d.B & 15) || (d.ldb & 3)) return false;
    if (d.epi != EPI_RELU && d.epi != EPI_STORE) return false;
    if (d.dotp && (d.N % 32)) return false;
  }
  // 128-column tiles when they give two workgroups per CU, else 64-column ones
  if (assign_tiles<kFBM, 128>(b) >= 512) return true;
  return assign_tiles<kFBM, 64>(b) >= 512;
}

// one k_gemm configuration, fp32 or bf16 MFMA operands
template <int TM, int TN, int KSPLIT, int G, int MG, bool ADAM, int AXK>
static void launch_k(const GemmBatch& b, int grid, hipStream_t s) {
  const dim3 blk(64 * KSPLIT * MG);
  if (b.bf16) hipLaunchKernelGGL((k_gemm<TM, TN, KSPLIT, G, MG, ADAM, AXK, true>), dim3(grid), blk, 0, s, b);
  else hipLaunchKernelGGL((k_gemm<TM, TN, KSPLIT, G, MG, ADAM, AXK, false>), dim3(grid), blk, 0, s, b);
}

// every desc's B operand has a bf16 shadow
static bool all_bh(const GemmBatch& b) {
  for (int i = 0; i < b.count; ++i)
    if (!b.d[i].Bh) return false;
  return true;
}

// the split-K weight-gradient level: k_dw_part16 (partials) + k_dw_fin (sum + epilogue)
static void launch_dw_split(GemmBatch& b, int ns, int64_t stride, hipStream_t s) {
  if (b.ride.pk_blocks) throw Error{SACMI_ESTATE, "Polyak ride on a level outside k_gemm"};
  const int ride = b.ride.kind ? b.ride.nblocks : 0;
  if (b.ride.kind == 1 && mt_sample_lds_words(b.ride.tbl_log2, b.ride.mt.setsize) * 4 > (size_t)kDw16LdsBytes)
    throw Error{SACMI_ESTATE, "ride-along sampler table exceeds k_dw_part16's LDS"};
  const int grid = dw_grid_tiles(b.total_tiles, ns) + ride;
  const int form = level_act16(b);   // act16: every X operand bf16
  for (int i = 0; i < b.count; ++i)
    if (b.d[i].a16 || b.d[i].c16 || b.d[i].x16 || (form && !b.d[i].b16) || (!b.bf16 && b.d[i].b16))
      throw Error{SACMI_ESTATE, "split-K weight gradient: unsupported bf16 activation operand"};
  if (!b.bf16) hipLaunchKernelGGL(k_dw_part_x6, dim3(grid), dim3(64 * kDw16Waves), 0, s, b, ns, stride);
  else if (form) hipLaunchKernelGGL(k_dw_part16<true>, dim3(grid), dim3(64 * kDw16Waves), 0, s, b, ns, stride);
  else hipLaunchKernelGGL(k_dw_part16<false>, dim3(grid), dim3(64 * kDw16Waves), 0, s, b, ns, stride);
  HIP_LAUNCH_CHECK();
  int fin_grid = 0;                    // k_dw_fin: kDwFinEpt 4-column groups per thread, per desc
  for (int i = 0; i < b.count; ++i)
    fin_grid += (b.d[i].M * (dw_ncols(b.d[i]) / 4) + 256 * kDwFinEpt - 1) / (256 * kDwFinEpt);
  if (b.tl) b.tl += kTlWords;          // the second kernel of the level
  // the fin's stores are plain (write-through measured slower at config 5: 3,412 -> 3,357
  // updates/s, the boundary behind the level unchanged)
  b.st_wt = 0;
  const dim3 fg(fin_grid), fb(256);
  switch (ns) {   // one instantiation per split count: no load slots for absent splits
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
}

// the batch-4096-class dh level: k_axk16 (axk16_ok form `ax`)
static void launch_axk16(const GemmBatch& b, int ax, hipStream_t s) {
  if (b.ride.pk_blocks) throw Error{SACMI_ESTATE, "Polyak ride on a level outside k_gemm"};
  for (int i = 0; i < b.count; ++i)   // k_axk16 computes no dL/da partials
    if (b.d[i].pa_out) throw Error{SACMI_ESTATE, "dL/da partials requested on a k_axk16 level"};
  const bool bh = all_bh(b);
  const dim3 grid(b.total_tiles + (b.ride.kind ? b.ride.nblocks : 0)), blk(64 * kAxWaves);
  const int form = level_act16(b);   // act16: mask sources (and AX sources) bf16
  for (int i = 0; i < b.count; ++i)
    if (b.d[i].c16 || b.d[i].b16 || b.d[i].x16 != form || b.d[i].a16 != (form && b.d[i].axk == 1))
      throw Error{SACMI_ESTATE, "k_axk16: unsupported bf16 activation operand"};
  if (form) {
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
}

// the batch-4096-class bf16 forward level: k_fwd16p (multi-slab LDS ring) where its plan
// applies, else k_fwd16.  SACMI_NO_FWD16P (read once): k_fwd16 only — the parity test that
// holds the two kernels to the same bits (tests/test_gpu_fwd16p.py)
static void launch_fwd16(GemmBatch& b, hipStream_t s) {
  if (b.ride.pk_blocks) throw Error{SACMI_ESTATE, "Polyak ride on a level outside k_gemm"};
  const bool n128 = b.d[0].tiles_n * kFBN128 >= b.d[0].N && b.d[0].tiles_n == (b.d[0].N + 127) / 128;
  const bool bh = all_bh(b);
  const bool ah = level_act16(b) != 0;   // act16: bf16 input rows and bf16 output
  if (ah) {
    for (int i = 0; i < b.count; ++i)
      if (!b.d[i].a16 || !b.d[i].c16 || b.d[i].b16 || b.d[i].x16 || (b.d[i].N & 1) || (b.d[i].ldc & 1))
        throw Error{SACMI_ESTATE, "k_fwd16: unsupported bf16 activation operands"};
    if (bh) {
      GemmBatch bp = b;
      const int bm = fwd16p_plan(bp);
      if (bm) {
        const dim3 g(bp.total_tiles);
        if (bm == 256) hipLaunchKernelGGL((k_fwd16p<256>), g, dim3(1024), 0, s, bp);
        else hipLaunchKernelGGL((k_fwd16p<128>), g, dim3(1024), 0, s, bp);
        HIP_LAUNCH_CHECK();
        return;
      }
    }
  }
  const dim3 g(b.total_tiles), b128(64 * fwd16_waves<128>()), b64(64 * fwd16_waves<64>());
  if (ah) {
    if (n128 && bh) hipLaunchKernelGGL((k_fwd16<128, true, true>), g, b128, 0, s, b);
    else if (bh) hipLaunchKernelGGL((k_fwd16<64, true, true>), g, b64, 0, s, b);
    else if (n128) hipLaunchKernelGGL((k_fwd16<128, false, true>), g, b128, 0, s, b);
    else hipLaunchKernelGGL((k_fwd16<64, false, true>), g, b64, 0, s, b);
  } else {
    if (n128 && bh) hipLaunchKernelGGL((k_fwd16<128, true>), g, b128, 0, s, b);
    else if (bh) hipLaunchKernelGGL((k_fwd16<64, true>), g, b64, 0, s, b);
    else if (n128) hipLaunchKernelGGL((k_fwd16<128>), g, b128, 0, s, b);
    else hipLaunchKernelGGL((k_fwd16<64>), g, b64, 0, s, b);
  }
  HIP_LAUNCH_CHECK();
}

// whether launch_gemm may run an fp32 level on k_fwd_x6: plain forward GEMMs (both operands
// K-contiguous and 16-byte aligned, store / ReLU epilogue, optional bias and dot partials),
// no prologue, no rides, and two 128-row tiles per CU (128 columns wide where that gives
// them, else 64).  The tile assignment of the chosen width is left in b.
static bool fwd_x6_ok(GemmBatch& b) {
  if (b.ride.kind || b.ride.pk_blocks || b.bf16 || b.has_adam) return false;
  for (int i = 0; i < b.count; ++i) {
    const GemmDesc& d = b.d[i];
    if (!d.a_kc || !d.b_kc || d.axk || d.a_ksc || d.rs_col >= 0 || d.pa_out) return false;
    if (d.a16 || d.b16 || d.c16 || d.x16) return false;
    if (((uintptr_t)d.A & 15) || (d.lda & 3) || ((uintptr_t)d.B & 15) || (d.ldb & 3)) return false;
    if (d.epi != EPI_RELU && d.epi != EPI_STORE) return false;
    if (d.dotp && (d.N % 32)) return false;
  }
  if (assign_tiles<kFBM, 128>(b) >= 512) return true;
  return assign_tiles<kFBM, 64>(b) >= 512;
}

static void launch_fwd_x6(const GemmBatch& b, hipStream_t s) {
  const bool n128 = b.d[0].tiles_n == (b.d[0].N + 127) / 128;
  const dim3 g(b.total_tiles), blk(64 * kX6Waves);
  if (n128) hipLaunchKernelGGL(k_fwd_x6<128>, g, blk, 0, s, b);
  else hipLaunchKernelGGL(k_fwd_x6<64>, g, blk, 0, s, b);
  HIP_LAUNCH_CHECK();
}

void launch_gemm(const GemmBatch& b0, hipStream_t s) {
  if (b0.count == 0) return;
  GemmBatch b = b0;
  {
    int64_t stride = 0;
    const int ns = dw_split_plan(b, &stride);
    if (ns > 0) {
      launch_dw_split(b, ns, stride, s);
      return;
    }
  }
  b = b0;
  {
    const int ax = axk16_ok(b);
    if (ax >= 0) {
      launch_axk16(b, ax, s);
      return;
    }
  }
  b = b0;
  if (fwd_big_ok(b)) {
    launch_fwd16(b, s);
    return;
  }
  b = b0;
  if (fwd_x6_ok(b)) {
    launch_fwd_x6(b, s);
    return;
  }
  b = b0;
  {
    const int ax = axk_x6_ok(b);
    if (ax >= 0) {
      launch_axk_x6(b, ax, s);
      return;
    }
  }
  b = b0;
  if (level_act16(b))
    throw Error{SACMI_ESTATE, "bf16 activation operands on a level outside the batch-4096-class kernels"};
  // Polyak rides (RideAlong::pk) and the next update's sampler / gather run as extra
  // workgroups past the tiles, on k_gemm's 1024-thread configurations
  const int extra = (b.ride.kind ? b.ride.nblocks : 0) + b.ride.pk_blocks;
  if (b.ride.kind == 1 && mt_sample_lds_words(b.ride.tbl_log2, b.ride.mt.setsize) * 4 > kRideLdsBytes)
    throw Error{SACMI_ESTATE, "ride-along sampler table exceeds k_gemm's LDS"};
  int n_adam = 0;
  int64_t outs = 0;
  for (int i = 0; i < b.count; ++i) {
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
  if (dw && t64 <= 256) {
    // one 32x64 tile per CU (policy level): 16 waves, K split 16 ways
    if (n_adam) launch_k<32, 64, 16, 1, 1, true, 0>(b, b.total_tiles + extra, s);
    else launch_k<32, 64, 16, 1, 1, false, 0>(b, b.total_tiles + extra, s);
  } else if (dw || n_adam || t64 > 512) {
    // more 32x64 tiles than CUs (the twin critic weight gradients; every level at large
    // batch): 64x64 tiles as two 32-row wave groups, each with a K split — half the operand
    // bytes per FLOP of a 32x64 tile; the epilogue state is prefetched under the MFMAs.
    // 16 waves per CU either as one 1024-thread workgroup (8-way K split per wave group)
    // or as two 512-thread ones (4-way): then one workgroup's LDS reduction and epilogue
    // overlap the other's operand loads and MFMAs (the dh and forward levels; the
    // weight-gradient levels keep the 8-way split).  Rides attach to 1024 threads.
    const int g = assign_tiles<64, 64>(b) + extra;
    for (int i = 0; i < b.count; ++i)   // the two-wave-group tiles compute no dL/da partials
      if (b.d[i].pa_out) throw Error{SACMI_ESTATE, "dL/da partials requested on a 64-row tile level"};
    if (n_adam) launch_k<32, 64, 8, 1, 2, true, 0>(b, g, s);
    else if (dw) launch_k<32, 64, 8, 1, 2, false, 0>(b, g, s);   // the plain (data-parallel) form
    else if (axk == 1 && !extra) launch_k<32, 64, 4, 1, 2, false, 1>(b, g, s);
    else if (axk == 1) launch_k<32, 64, 8, 1, 2, false, 1>(b, g, s);
    else if (!extra) launch_k<32, 64, 4, 1, 2, false, 0>(b, g, s);
    else launch_k<32, 64, 8, 1, 2, false, 0>(b, g, s);
  } else if (axk == 1) {
    // dh1 / dha1 with the fc3 backward folded in (A transform, coefficient in the epilogue)
    launch_k<32, 32, 16, 2, 1, false, 1>(b, assign_tiles<32, 32>(b) + extra, s);
  } else if (t64 >= 192) {
    // widest tile that still gives one workgroup to most CUs
    launch_k<32, 64, 16, 2, 1, false, 0>(b, b.total_tiles + extra, s);
  } else {
    launch_k<32, 32, 16, 2, 1, false, 0>(b, assign_tiles<32, 32>(b) + extra, s);
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
// logp_part; red (KSPLIT * TM * (TN + 1) floats), lp, s_lp: LDS.
template <int TN, int KSPLIT, bool H16, int TM>
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
  gemm_core_l<TM, TN, KSPLIT, 2, true, true, false, 1, 0, false, H16>(d, m0, 0, red, nullptr, pre);
  __syncthreads();
  const uint64_t ctr = a.ctr_override ? a.ctr_override : a.sc->noise_counter;
  if (e < TM * A) {
    float lpe = 0.f;
    if (live) {
      const float mean = reduce_partials<TM, TN, KSPLIT>(red, row, j) + bm;
      const float ls_raw = reduce_partials<TM, TN, KSPLIT>(red, row, A + j) + bl;
      lpe = heads_elem<H16>(a, m, j, mean, ls_raw, eps_in, ctr);
    }
    lp[row][j] = lpe;
  }
  heads_logp<TM>(a, m0, part, lp, s_lp);
}

template <int TN, int KSPLIT, bool H16 = false, int TM = 16>
__global__ __launch_bounds__(64 * KSPLIT) void k_heads_sample(HeadSampleArgs a) {
  const TlMark tl_mark(a.tl, TL_HEADS);
  __shared__ float red[KSPLIT * TM * (TN + 1)];
  __shared__ float lp[TM][33];
  __shared__ float s_lp[TM];
  heads_rows<TN, KSPLIT, H16, TM>(a, blockIdx.x * TM, blockIdx.x, red, lp, s_lp);
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
// workgroup (any others only join its barriers).  slab0: the unit also stores dhead.
template <int NPA = kTailMaxPa>
__device__ __forceinline__ void tail_unit(const float* pa, int n_pa, const SampleBwdArgs& a, int m0,
                                          int c0, bool slab0, TailSmem& sm) {
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
  preload();
  const rsrc_t rP = make_rsrc(pa, (uint32_t)((size_t)n_pa * B * A * 4));
  const uint32_t pstride = (uint32_t)B * (uint32_t)A * 4u, po = (uint32_t)((own ? pm : 0) * A + pj) * 4u;
  // (NPA >= n_pa partial loads per thread: the launcher picks the smallest instantiation, so
  // no issue slots go to out-of-range loads)
  float t[NPA];
#pragma unroll
  for (int q = 0; q < NPA; ++q)
    t[q] = buf_ld(rP, own && q < n_pa ? po + (uint32_t)q * pstride : 0xfffffff0u);
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
  tail_unit<NPA>(pa, n_pa, a, blockIdx.x * kTailRows, blockIdx.y * kTailCols, blockIdx.y == 0, sm);
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

bool gemm_level_on_axk16(const GemmBatch& b0) {
  GemmBatch b = b0;
  return axk16_ok(b) >= 0;
}

// launch_gemm's own kernel choice for an axk-1 level, asked ahead of its launch: true when
// it runs on the one-wave-group k_gemm tiles (<32, 32, 16, 2, 1, false, 1>: MG == 1, AXK ==
// 1), the only form that computes dL/da partials.  Mirrors launch_gemm's order: the split-K
// and the bf16 forward kernels never take an axk level; k_axk16 (bf16, batch-4096 class);
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
// The scalar work runs on a workgroup of its own, the grid's last, from the kernel's start:
// its inputs (loss partials, log_alpha's gradient and state, the scalars) come from earlier
// kernels and no element reads what it writes — after block 0's elements it put a chain of
// dependent round trips at the end of the kernel (the fused levels moved it the same way,
// adam_block0_wave).  The element blocks are the grid's first gridDim.x - 1.
__device__ __forceinline__ void adam_scalar_tail(const AdamArgs& a, float om_b1, float om_b2) {
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
  const unsigned nel = gridDim.x - 1;   // element workgroups; the last one: the scalar work
  if (blockIdx.x == nel) {
    if (!err) adam_scalar_tail(a, om_b1, om_b2);
    return;
  }
  if (err & a.err_skip) return;
  const bool pol = a.tgt && (err & a.err_nopolyak) == 0;
  const int64_t total4 = s_prefix[a.nseg];
  // parameter / moment / target arenas: one descriptor each (offsets < 2 GiB: the arenas
  // hold at most a few million floats)
  const rsrc_t rP = make_rsrc(a.p, 0x7fffffffu), rM = make_rsrc(a.m, 0x7fffffffu),
               rV = make_rsrc(a.v, 0x7fffffffu),
               rT = make_rsrc(a.tgt ? a.tgt : a.p, a.tgt ? 0x7fffffffu : 0u);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total4;
       e += (int64_t)nel * blockDim.x) {
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
}

void launch_adam(const AdamArgs& a, hipStream_t s) {
  int64_t total4 = 0;
  for (int i = 0; i < a.nseg; ++i) total4 += a.seg[i].n / 4;
  int64_t blocks = (total4 + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  // + the scalar-work workgroup (the grid's last)
  hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks + 1), dim3(256), 0, s, a);
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
