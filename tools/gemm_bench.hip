// Microbenchmark for the grouped GEMM levels of the SAC step (not part of the library).
// Builds each level of the Humanoid config (S 376, A 17, H 512, B 256) with the same
// operand layouts the step uses and times every k_gemm tile/K-split variant on it,
// with the plain-store and the fused-Adam epilogues.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/gemm_bench.hip -o tools/gemm_bench
//   (add -DSACMI_DIAG_STAMPS for the per-phase stamp build: `gemm_bench stamps`)
#include "../humanoid-walking-with-sac_amd/csrc/kernels.hip"
#include <algorithm>
#include <cstring>
#include <cstdlib>
#include <map>

#include <cstdio>
#include <functional>
#include <string>
#include <vector>

using namespace sacmi;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

static float* dalloc(size_t n, float val = 0.01f) {
  float* p;
  CK(hipMalloc(&p, n * sizeof(float)));
  std::vector<float> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = val * (float)((i * 2654435761u) % 1000) / 1000.f;
  CK(hipMemcpy(p, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
  return p;
}

static GemmDesc mk(const float* A, int lda, int akc, const float* B, int ldb, int bkc, float* C,
                   int ldc, int M, int N, int K, int epi, int step = 0) {
  GemmDesc d{};
  d.A = A; d.lda = lda; d.a_kc = akc; d.B = B; d.ldb = ldb; d.b_kc = bkc;
  d.C = C; d.ldc = ldc; d.M = M; d.N = N; d.K = K; d.epi = epi; d.adam_step = step;
  d.rs_col = -1;
  return d;
}

template <int TM, int TN, int KS, int G, int MG, bool AD, int AX = 0>
static float time_cfg(GemmBatch b, int iters, hipStream_t s) {
  assign_tiles<TM * MG, TN>(b);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL((k_gemm<TM, TN, KS, G, MG, AD, AX>), dim3(b.total_tiles), dim3(64 * KS * MG), 0, s, b);
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((k_gemm<TM, TN, KS, G, MG, AD, AX>), dim3(b.total_tiles), dim3(64 * KS * MG), 0, s, b);
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipGetLastError());
  return ms * 1000.f / iters;
}

#ifdef SACMI_DIAG_STAMPS
// one launch after warm-up; per-phase breakdown from the in-kernel stamps (µs)
template <int TM, int TN, int KS, int G, int MG, bool AD, int AX = 0>
static void stamp_cfg(GemmBatch b, hipStream_t s) {
  assign_tiles<TM * MG, TN>(b);
  for (int i = 0; i < 30; ++i) hipLaunchKernelGGL((k_gemm<TM, TN, KS, G, MG, AD, AX>), dim3(b.total_tiles), dim3(64 * KS * MG), 0, s, b);
  CK(hipStreamSynchronize(s));
  static unsigned long long h[4096][40];
  memset(h, 0, sizeof(h));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), h, sizeof(h)));
  hipLaunchKernelGGL((k_gemm<TM, TN, KS, G, MG, AD, AX>), dim3(b.total_tiles), dim3(64 * KS * MG), 0, s, b);
  CK(hipStreamSynchronize(s));
  CK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_stamps), sizeof(h)));
  const int nb = std::min(b.total_tiles, 4096);
  unsigned long long t0 = ~0ull, tend = 0;
  auto live = [&](int i) { return h[i][33] != 0; };   // padding blocks exit unstamped
  for (int i = 0; i < nb; ++i) { if (!live(i)) continue; for (int w = 0; w < KS * MG; ++w) t0 = std::min(t0, h[i][w]); tend = std::max(tend, h[i][33]); }
  std::vector<double> start, core_max, core_min, syncw, epi, endt;
  for (int i = 0; i < nb; ++i) {
    if (!live(i)) continue;
    unsigned long long e0 = ~0ull, emax = 0, lmax = 0, cmax = 0, cmin = ~0ull;
    for (int w = 0; w < KS * MG; ++w) {
      e0 = std::min(e0, h[i][w]); emax = std::max(emax, h[i][w]);
      lmax = std::max(lmax, h[i][16 + w]);
      cmax = std::max(cmax, h[i][16 + w] - h[i][w]); cmin = std::min(cmin, h[i][16 + w] - h[i][w]);
    }
    start.push_back((e0 - t0) * 0.01); core_max.push_back(cmax * 0.01); core_min.push_back(cmin * 0.01);
    syncw.push_back((h[i][32] - lmax) * 0.01); epi.push_back((h[i][33] - h[i][32]) * 0.01);
    endt.push_back((h[i][33] - t0) * 0.01);
  }
  // residency census: CU identity = (xcc, se, sh, cu) from HW_ID; max WGs overlapping on one CU
  std::map<unsigned long long, std::vector<std::pair<unsigned long long, unsigned long long>>> per_cu;
  for (int i = 0; i < nb; ++i) {
    if (!live(i)) continue;
    const unsigned long long id = h[i][34];
    const unsigned long long hw = id & 0xffffffffull, xcc = (id >> 32) & 0xf;
    const unsigned long long key = (xcc << 16) | (((hw >> 8) & 0xf) << 0) | (((hw >> 12) & 0x1) << 4) | (((hw >> 13) & 0x7) << 5);
    unsigned long long e0 = ~0ull;
    for (int w = 0; w < KS * MG; ++w) e0 = std::min(e0, h[i][w]);
    per_cu[key].push_back({e0, h[i][33]});
  }
  int maxov = 0;
  for (auto& kv : per_cu) {
    for (auto& a : kv.second) {
      int ov = 0;
      for (auto& b2 : kv.second) ov += (b2.first <= a.first && a.first < b2.second);
      maxov = std::max(maxov, ov);
    }
  }
  int early = 0;
  for (double x : start) early += x < 1.0;
  printf("      CUs used %zu, max WGs co-resident on one CU %d, WGs started < 1us: %d of %d\n", per_cu.size(), maxov, early, nb);
  auto q = [](std::vector<double> v, double f) { std::sort(v.begin(), v.end()); return v[(size_t)(f * (v.size() - 1))]; };
  {
    std::vector<double> p1, p2;
    for (int i = 0; i < nb; ++i) {
      if (!live(i) || !h[i][35]) continue;
      p1.push_back((h[i][36] - h[i][0]) * 0.01);
      p2.push_back((h[i][35] - h[i][0]) * 0.01);
    }
    if (!p1.empty()) {
      auto md = [](std::vector<double>& v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
      printf("      row prologue (after the MFMAs; from wave-0 entry, medians): sum barrier %.2f | "
             "coef barrier %.2f\n", md(p1), md(p2));
    }
  }
  printf("      span %.2f | start med %.2f max %.2f | core(max wave) med %.2f max %.2f | core(min wave) med %.2f | "
         "lds+sync med %.2f | epilogue med %.2f max %.2f | end med %.2f\n",
         (tend - t0) * 0.01, q(start, .5), q(start, 1), q(core_max, .5), q(core_max, 1), q(core_min, .5),
         q(syncw, .5), q(epi, .5), q(epi, 1), q(endt, .5));
}

template <int LDSB>
__global__ __launch_bounds__(512) void k_lds_probe(float* out) {
  __shared__ float buf[LDSB / 4];
  buf[threadIdx.x] = threadIdx.x;
  __syncthreads();
  SACMI_STAMP(0);
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t < 300) { }   // hold the CU 3 us
  SACMI_STAMP(33);
  if (threadIdx.x == 0) out[blockIdx.x] = buf[(threadIdx.x + 1) % 512];
}

template <int LDSB>
static void probe(float* out, hipStream_t s) {
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_lds_probe<LDSB>, 512, 0));
  static unsigned long long h[4096][40];
  memset(h, 0, sizeof(h));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), h, sizeof(h)));
  hipLaunchKernelGGL(k_lds_probe<LDSB>, dim3(1024), dim3(512), 0, s, out);
  CK(hipStreamSynchronize(s));
  CK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_stamps), sizeof(h)));
  std::map<unsigned long long, std::vector<std::pair<unsigned long long, unsigned long long>>> per_cu;
  for (int i = 0; i < 1024; ++i) {
    const unsigned long long id = h[i][34], hw = id & 0xffffffffull, xcc = (id >> 32) & 0xf;
    const unsigned long long key = (xcc << 16) | ((hw >> 8) & 0xf) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 7) << 5);
    per_cu[key].push_back({h[i][0], h[i][33]});
  }
  int maxov = 0;
  for (auto& kv : per_cu) for (auto& a : kv.second) {
    int ov = 0;
    for (auto& b2 : kv.second) ov += (b2.first <= a.first && a.first < b2.second);
    maxov = std::max(maxov, ov);
  }
  printf("LDS probe %6d B, 512 thr: occupancy API %d, observed max co-resident %d (CUs %zu)\n", LDSB, occ, maxov, per_cu.size());
}

#endif

template <int TM, int TN, int KS, int G, int MG, bool AD>
static void occ_cfg(const char* name) {
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_gemm<TM, TN, KS, G, MG, AD>, 64 * KS, 0));
  hipFuncAttributes fa;
  CK(hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(k_gemm<TM, TN, KS, G, MG, AD>)));
  printf("%-14s occupancy API %d blocks/CU, LDS %zu, regs %d\n", name, occ, fa.sharedSizeBytes, fa.numRegs);
}

int main(int argc, char** argv) {
  const bool stamps = argc > 1 && std::string(argv[1]) == "stamps";
  const int S = 376, A = 17, H = 512;
  const int B = getenv("SACMI_BENCH_B") ? atoi(getenv("SACMI_BENCH_B")) : 256;
  const int Kx = (S + 1 + A + 3) / 4 * 4, Hd = (H + 1 + 3) / 4 * 4, Kp1 = (S + 1 + 3) / 4 * 4;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  // activations
  float* x = dalloc((size_t)B * Kx);        // critic input [B, Kx]
  float* sp = dalloc((size_t)2 * B * Kp1);  // policy input [2B, Kp1]
  float* hq1 = dalloc((size_t)B * 2 * Hd);
  float* hq2 = dalloc((size_t)B * 2 * Hd);
  float* hp1 = dalloc((size_t)2 * B * Hd);
  float* hp2 = dalloc((size_t)2 * B * Hd);
  float* dh1 = dalloc((size_t)B * 2 * H);
  float* dh2 = dalloc((size_t)B * 2 * H);
  float* dq = dalloc((size_t)2 * B);
  float* dhp2 = dalloc((size_t)B * H);
  float* dhp1 = dalloc((size_t)B * H);
  float* dhead = dalloc((size_t)B * 20);
  // parameter arena (critic: 2 x [fc1 H x Kx, fc2 H x Hd, fc3 1 x Hd], policy: fc1, fc2, head)
  const size_t q1n = (size_t)H * Kx, q2n = (size_t)H * Hd, q3n = Hd;
  const size_t qn = q1n + q2n + q3n;
  const size_t p1n = (size_t)H * Kp1, p2n = (size_t)H * Hd, phn = (size_t)2 * A * Hd;
  const size_t total = 2 * qn + p1n + p2n + phn + 64;
  float* P = dalloc(total);
  float* M = dalloc(total, 0.001f);
  float* V = dalloc(total, 0.001f);
  float* Gd = dalloc(total);
  float* T = dalloc(2 * qn);
  float* scratch = dalloc((size_t)4 * B * Hd);
  DevScalars* sc;
  CK(hipMalloc(&sc, sizeof(DevScalars)));
  DevScalars hs{};
  for (int i = 0; i < 4; ++i) { hs.beta_pow[i][0] = 0.9; hs.beta_pow[i][1] = 0.999; }
  CK(hipMemcpy(sc, &hs, sizeof(hs), hipMemcpyHostToDevice));
  AdamFuse af{};
  af.P = P; af.M = M; af.V = V; af.T = T; af.G = Gd; af.t_base = 0;
  af.lr = 3e-4f; af.beta1 = 0.9f; af.beta2 = 0.999f; af.eps = 1e-8f; af.tau = 0.005f;
  af.sc = sc; af.log_alpha_idx = -1; af.n_losses = 0;

  if (argc > 1 && std::string(argv[1]) == "occ") {
    occ_cfg<32, 64, 8, 2, 1, false>("<32,64,8,2>"); occ_cfg<32, 64, 16, 2, 1, false>("<32,64,16,2>");
    occ_cfg<32, 32, 16, 4, 1, false>("<32,32,16,4>"); occ_cfg<32, 32, 8, 2, 1, false>("<32,32,8,2>");
    occ_cfg<32, 32, 4, 4, 1, false>("<32,32,4,4>");
    return 0;
  }
  struct Level { std::string name; std::function<GemmBatch(bool)> make; };
  std::vector<Level> levels;
  levels.push_back({"L6 critic dW (K=256)", [&](bool fused) {
    GemmBatch b{};
    const int epi = fused ? EPI_ADAM_POLYAK : EPI_STORE;
    for (int i = 0; i < 2; ++i) {
      float* base = P + i * qn;
      b.d[b.count++] = mk(dh1 + i * H, 2 * H, 0, x, Kx, 0, base, Kx, H, S + 1 + A, B, epi, 1 + i);
      GemmDesc d2 = mk(dh2 + i * H, 2 * H, 0, hq1 + i * Hd, 2 * Hd, 0, base + q1n, Hd, H, H, B, epi, 1 + i);
      d2.rs_col = H; b.d[b.count++] = d2;
      GemmDesc d3 = mk(dq + i * B, 1, 0, hq2 + i * Hd, 2 * Hd, 0, base + q1n + q2n, Hd, 1, H, B, epi, 1 + i);
      d3.rs_col = H; b.d[b.count++] = d3;
    }
    b.adam = af; b.has_adam = 0;
    return b; }});
  levels.push_back({"L13 policy dW (K=256)", [&](bool fused) {
    GemmBatch b{};
    const int epi = fused ? EPI_ADAM : EPI_STORE;
    float* base = P + 2 * qn;
    b.d[b.count++] = mk(dhp1, H, 0, sp + B * Kp1, Kp1, 0, base, Kp1, H, S + 1, B, epi);
    GemmDesc d2 = mk(dhp2, H, 0, hp1 + B * Hd, Hd, 0, base + p1n, Hd, H, H, B, epi); d2.rs_col = H;
    b.d[b.count++] = d2;
    GemmDesc d3 = mk(dhead, 20, 0, hp2 + B * Hd, Hd, 0, base + p1n + p2n, Hd, 2 * A, H, B, epi); d3.rs_col = H;
    b.d[b.count++] = d3;
    b.adam = af;
    return b; }});
  levels.push_back({"L2 fwd fc2 (pi 2B + 2 q, K=512)", [&](bool) {
    GemmBatch b{};
    GemmDesc d = mk(hp1, Hd, 1, P + 2 * qn + p1n, Hd, 1, hp2, Hd, 2 * B, H, H, EPI_RELU);
    d.bias = P + 2 * qn + p1n + H; d.bias_ld = Hd; b.d[b.count++] = d;
    for (int i = 0; i < 2; ++i) {
      GemmDesc e = mk(hq1 + i * Hd, 2 * Hd, 1, P + i * qn + q1n, Hd, 1, hq2 + i * Hd, 2 * Hd, B, H, H, EPI_RELU);
      e.bias = P + i * qn + q1n + H; e.bias_ld = Hd; b.d[b.count++] = e;
    }
    return b; }});
  levels.push_back({"L1 fwd fc1 (pi 2B K=380, 2 q K=396)", [&](bool) {
    GemmBatch b{};
    b.d[b.count++] = mk(sp, Kp1, 1, P + 2 * qn, Kp1, 1, hp1, Hd, 2 * B, H, S + 1, EPI_RELU);
    for (int i = 0; i < 2; ++i)
      b.d[b.count++] = mk(x, Kx, 1, P + i * qn, Kx, 1, hq1 + i * Hd, 2 * Hd, B, H, S + 1 + A, EPI_RELU);
    return b; }});
  levels.push_back({"L5 critic dh1 (K=512, A n-contig W)", [&](bool) {
    GemmBatch b{};
    for (int i = 0; i < 2; ++i)
      b.d[b.count++] = mk(dh2 + i * H, 2 * H, 1, P + i * qn + q1n, Hd, 0, dh1 + i * H, 2 * H, B, H, H, EPI_MASK);
    b.d[0].aux = hq1; b.d[0].ldaux = 2 * Hd; b.d[1].aux = hq1 + Hd; b.d[1].ldaux = 2 * Hd;
    return b; }});
  // L5 with the critic rows folded in (row prologue from dot partials + A transform)
  float* part = dalloc((size_t)4 * B * 16, 0.1f);
  float* rvec = dalloc(B), *dvec = dalloc(B, 0.f), *lpv = dalloc(2 * B), *dqv = dalloc(2 * B);
  float* lpart = dalloc(64);
  float* dh2o = dalloc((size_t)B * 2 * H);
  levels.push_back({"L5 fused rows (K=512)", [&](bool) {
    GemmBatch b{};
    for (int i = 0; i < 2; ++i) {
      GemmDesc g = mk(hq2 + i * Hd, 2 * Hd, 1, P + i * qn + q1n, Hd, 0, dh1 + i * H, 2 * H, B, H, H, EPI_MASK);
      g.aux = hq1 + i * Hd; g.ldaux = 2 * Hd;
      g.axk = 1; g.ax_slot = i; g.ax_w = P + i * qn + q1n + q2n; g.ax_out = dh2o + i * H; g.ax_ld = 2 * H;
      b.d[b.count++] = g;
    }
    RowsFuse& rf = b.rows;
    rf.kind = 1; rf.part = part; rf.nparts = 16; rf.B = B;
    rf.r = rvec; rf.d = dvec; rf.logp = lpv; rf.gamma = 0.99f; rf.sc = sc; rf.dq = dqv;
    rf.loss_part = lpart;
    return b; }});
  (void)scratch; (void)dhp2;

  const int iters = 300;
  for (auto& L : levels) {
    for (int fused = 0; fused < 2; ++fused) {
      if (fused && L.name[1] != '6' && L.name.substr(0, 3) != "L13") continue;
      GemmBatch b = L.make(fused);
      int t32 = assign_tiles<32, 32>(b), t64 = assign_tiles<32, 64>(b), t6464 = assign_tiles<64, 64>(b);
      printf("%-40s %-6s tiles32x32=%d 32x64=%d 64x64=%d\n", L.name.c_str(), fused ? "adam" : "store", t32, t64, t6464);
      if (L.name.rfind("L5 fused", 0) == 0) {
#ifdef SACMI_DIAG_STAMPS
        if (stamps) { printf("   <32,32,16,2,axk1>\n"); stamp_cfg<32, 32, 16, 2, 1, false, 1>(b, s); continue; }
#endif
        printf("   <32,32,16,2,axk1> %7.2f us\n", time_cfg<32, 32, 16, 2, 1, false, 1>(b, iters, s));
        printf("   <32x2,64,8,1,axk1> %7.2f us\n", time_cfg<32, 64, 8, 1, 2, false, 1>(b, iters, s));
        continue;
      }
#ifdef SACMI_DIAG_STAMPS
      if (stamps) {
        if (fused) {
          printf("   <32x2,64,8,1,adam>\n"); stamp_cfg<32, 64, 8, 1, 2, true>(b, s);
          printf("   <32x2,64,8,2,adam>\n"); stamp_cfg<32, 64, 8, 2, 2, true>(b, s);
          printf("   <32,64,16,2,adam>\n"); stamp_cfg<32, 64, 16, 2, 1, true>(b, s);
          continue;
        }
        printf("   <64,64,8,2>\n"); stamp_cfg<64, 64, 8, 2, 1, false>(b, s);
        printf("   <32,64,16,2>\n"); stamp_cfg<32, 64, 16, 2, 1, false>(b, s);
        printf("   <32,32,16,4>\n"); stamp_cfg<32, 32, 16, 4, 1, false>(b, s);
        continue;
      }
#endif
      if (fused) {
        printf("   <32x2,64,8,1,adam> %7.2f us\n", time_cfg<32, 64, 8, 1, 2, true>(b, iters, s));
        printf("   <32x2,64,8,2,adam> %7.2f us\n", time_cfg<32, 64, 8, 2, 2, true>(b, iters, s));
        printf("   <64,64,8,2,adam>  %7.2f us\n", time_cfg<64, 64, 8, 2, 1, true>(b, iters, s));
        printf("   <32,64,16,2,adam> %7.2f us\n", time_cfg<32, 64, 16, 2, 1, true>(b, iters, s));
        continue;
      }
      printf("   <32x2,64,8,1> %7.2f us\n", time_cfg<32, 64, 8, 1, 2, false>(b, iters, s));
      printf("   <64,64,8,2>  %7.2f us\n", time_cfg<64, 64, 8, 2, 1, false>(b, iters, s));
      printf("   <64,64,4,4>  %7.2f us\n", time_cfg<64, 64, 4, 4, 1, false>(b, iters, s));
      printf("   <32,64,16,2> %7.2f us\n", time_cfg<32, 64, 16, 2, 1, false>(b, iters, s));
      printf("   <32,32,16,4> %7.2f us\n", time_cfg<32, 32, 16, 4, 1, false>(b, iters, s));
      printf("   <32,32,16,2> %7.2f us\n", time_cfg<32, 32, 16, 2, 1, false>(b, iters, s));
      fflush(stdout);
    }
  }
  return 0;
}
