// Phase timeline of the production GEMM from in-kernel s_memrealtime stamps (diagnostic build,
// -DGEMM_STAMPS): per workgroup, first tile: start, first k-step data landed, second k-step,
// k-loop end, epilogue end.  Prints medians / percentiles relative to the earliest start.
#define GEMM_STAMPS 1
#include "../../csrc/kernels/gemm.hip"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static unsigned short rbf(unsigned& st) {
  st = st * 1664525u + 1013904223u;
  float f = ((st >> 8) & 0xFFFF) / 32768.f - 1.f;
  unsigned u; memcpy(&u, &f, 4);
  return (unsigned short)(u >> 16);
}

int main() {
  struct Sh { int M, N, K, mode, bm; };
  std::vector<Sh> shapes = {{8192, 512, 512, 0, 64},  {8192, 512, 512, 0, 128}, {8192, 1536, 512, 0, 64},
                            {8192, 1536, 512, 0, 128}, {8192, 512, 1024, 0, 64}, {8192, 512, 512, 1, 64},
                            {8192, 512, 512, 2, 128}, {8192, 1536, 512, 2, 128}};
  const size_t maxe = (size_t)8192 * 10240;
  unsigned short *A, *B, *C;
  (void)hipMalloc(&A, maxe * 2); (void)hipMalloc(&B, maxe * 2); (void)hipMalloc(&C, maxe * 2);
  std::vector<unsigned short> h(maxe);
  unsigned st = 7;
  for (auto& x : h) x = rbf(st);
  (void)hipMemcpy(A, h.data(), maxe * 2, hipMemcpyHostToDevice);
  for (auto& x : h) x = rbf(st);
  (void)hipMemcpy(B, h.data(), maxe * 2, hipMemcpyHostToDevice);
  float* slab;
  (void)hipMalloc(&slab, (size_t)16 * 1536 * 512 * 4);
  unsigned long long* stamps;
  const int maxwg = 4096;
  (void)hipMalloc(&stamps, maxwg * 8 * 8);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_gemm_stamps), &stamps, sizeof(stamps));
  for (const Sh& sh : shapes) {
    GemmArgs g{};
    g.mode = sh.mode; g.alpha = 1.f; g.dscale = 1.f; g.splits = 1;
    g.A = A; g.lda = sh.K; g.B = B; g.ldb = sh.mode == 0 ? sh.K : sh.N; g.M = sh.M; g.N = sh.N; g.K = sh.K;
    g.C = C; g.ldc = sh.N;
    if (sh.mode == 2) {  // weight gradient dW[N,K] = dY^T X over M tokens, 16/8-way split-K into fp32 slabs
      g.A = A; g.lda = sh.N; g.B = B; g.ldb = sh.K; g.M = sh.N; g.N = sh.K; g.K = sh.M;
      g.C = slab; g.ldc = sh.K; g.out_f32 = 1; g.atomic = 0; g.splits = sh.N <= 512 ? 16 : 8;
      g.c_split_stride = (long)sh.N * sh.K;
    }
    smi_gemm_set_bm(sh.bm);
    for (int i = 0; i < 30; ++i) smi_gemm(&g, 0);  // warm, clocks up
    (void)hipMemset(stamps, 0, maxwg * 64);
    (void)hipDeviceSynchronize();
    smi_gemm(&g, 0);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> hs(maxwg * 8);
    (void)hipMemcpy(hs.data(), stamps, hs.size() * 8, hipMemcpyDeviceToHost);
    int nwg = 0;
    unsigned long long t0 = ~0ull, tend = 0;
    for (int b = 0; b < maxwg; ++b)
      if (hs[b * 8]) { ++nwg; t0 = std::min(t0, hs[b * 8]); tend = std::max(tend, hs[b * 8 + 4]); }
    printf("M%d N%d K%d mode%d bm%d: %d WGs, first-tile span %.2f us\n", sh.M, sh.N, sh.K, sh.mode, sh.bm, nwg,
           (tend - t0) / 100.0);
    const char* names[5] = {"start", "kt0 landed", "kt1 landed", "kloop end", "epi end"};
    for (int p = 0; p < 5; ++p) {
      std::vector<double> v;
      for (int b = 0; b < maxwg; ++b)
        if (hs[b * 8]) v.push_back((hs[b * 8 + p] - t0) / 100.0);
      std::sort(v.begin(), v.end());
      printf("   %-11s min %6.2f p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f us\n", names[p], v[0], v[v.size() / 10],
             v[v.size() / 2], v[v.size() * 9 / 10], v.back());
    }
    // per-phase durations
    {
      const char* en[4] = {"epi barrier", "epi lds wr", "epi math", "epi stores"};
      const int from[4] = {3, 5, 6, 7}, to[4] = {5, 6, 7, 4};
      for (int p = 0; p < 4; ++p) {
        std::vector<double> v;
        for (int b = 0; b < maxwg; ++b)
          if (hs[b * 8] && hs[b * 8 + to[p]] && hs[b * 8 + from[p]])
            v.push_back(((double)hs[b * 8 + to[p]] - (double)hs[b * 8 + from[p]]) / 100.0);
        if (v.empty()) continue;
        std::sort(v.begin(), v.end());
        printf("   dur %-11s p10 %6.2f p50 %6.2f p90 %6.2f us\n", en[p], v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10]);
      }
    }
    const char* dn[4] = {"prologue", "kstep0", "kloop rest", "epilogue"};
    for (int p = 0; p < 4; ++p) {
      std::vector<double> v;
      for (int b = 0; b < maxwg; ++b)
        if (hs[b * 8]) v.push_back(((double)hs[b * 8 + p + 1] - (double)hs[b * 8 + p]) / 100.0);
      std::sort(v.begin(), v.end());
      printf("   dur %-10s p10 %6.2f p50 %6.2f p90 %6.2f us\n", dn[p], v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10]);
    }
  }
  return 0;
}
