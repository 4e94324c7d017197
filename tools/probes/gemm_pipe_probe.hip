// A/B probe: production persistent GEMM vs the cross-tile pipelined variant (gemm_pipe_kernel)
// on the transformer shapes, in ONE process, graph-timed (20 launches per graph replay), random
// bf16 operands; checks the pipelined output bitwise against the production kernel.
#include "../../csrc/kernels/gemm.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstring>

static float graph_time(GemmArgs g, int reps = 20, int iters = 10) {
  hipStream_t s;
  (void)hipStreamCreate(&s);
  smi_gemm(&g, s);
  (void)hipStreamSynchronize(s);
  hipGraph_t gr;
  hipGraphExec_t ge;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < reps; ++i) smi_gemm(&g, s);
  (void)hipStreamEndCapture(s, &gr);
  (void)hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
  (void)hipGraphLaunch(ge, s);
  (void)hipStreamSynchronize(s);
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  (void)hipEventRecord(a, s);
  for (int i = 0; i < iters; ++i) (void)hipGraphLaunch(ge, s);
  (void)hipEventRecord(b, s);
  (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b);
  (void)hipGraphExecDestroy(ge); (void)hipGraphDestroy(gr); (void)hipStreamDestroy(s);
  return ms * 1000.f / (reps * iters);
}

static unsigned short rbf(unsigned& st) {
  st = st * 1664525u + 1013904223u;
  float f = ((st >> 8) & 0xFFFF) / 32768.f - 1.f;
  unsigned u; memcpy(&u, &f, 4);
  return (unsigned short)(u >> 16);
}

int main(int argc, char** argv) {
  struct Sh { int M, N, K, mode, bias, resid; };
  std::vector<Sh> shapes = {{8192, 512, 512, 0, 1, 0}, {8192, 1536, 512, 0, 1, 0}, {8192, 1024, 512, 0, 1, 0},
                            {8192, 512, 1024, 0, 1, 0}, {8192, 512, 512, 1, 0, 1}, {8192, 512, 1536, 1, 0, 1},
                            {8192, 512, 1024, 1, 0, 0}, {8192, 10000, 512, 0, 0, 0}};
  const size_t maxe = (size_t)8192 * 10000;
  unsigned short *A, *B, *C0, *C1, *R;
  float* bias;
  (void)hipMalloc(&A, maxe * 2); (void)hipMalloc(&B, maxe * 2); (void)hipMalloc(&R, maxe * 2);
  (void)hipMalloc(&C0, maxe * 2); (void)hipMalloc(&C1, maxe * 2); (void)hipMalloc(&bias, 16384 * 4);
  {
    std::vector<unsigned short> h(maxe);
    unsigned st = 1;
    for (auto& x : h) x = rbf(st);
    (void)hipMemcpy(A, h.data(), maxe * 2, hipMemcpyHostToDevice);
    for (auto& x : h) x = rbf(st);
    (void)hipMemcpy(B, h.data(), maxe * 2, hipMemcpyHostToDevice);
    for (auto& x : h) x = rbf(st);
    (void)hipMemcpy(R, h.data(), maxe * 2, hipMemcpyHostToDevice);
    std::vector<float> hb(16384);
    for (auto& x : hb) x = 0.01f * (float)((st = st * 1664525u + 1013904223u) >> 24);
    (void)hipMemcpy(bias, hb.data(), hb.size() * 4, hipMemcpyHostToDevice);
  }
  const int cfg[][3] = {{0, 0, 0}, {0, 0, 128}, {1, 3, 0}, {2, 3, 0}, {2, 2, 0}, {2, 4, 0}, {3, 3, 0}, {4, 3, 0}, {1, 3, 128}, {2, 3, 128}, {2, 4, 128}};
  for (const Sh& sh : shapes) {
    GemmArgs g{};
    g.mode = sh.mode; g.alpha = 1.f; g.dscale = 1.f; g.splits = 1;
    g.A = A; g.lda = sh.K; g.B = B; g.ldb = sh.mode == 0 ? sh.K : sh.N; g.M = sh.M; g.N = sh.N; g.K = sh.K;
    g.C = C0; g.ldc = sh.N;
    if (sh.bias) g.bias = bias;
    if (sh.resid) { g.resid = R; g.ldr = sh.N; }
    const double fl = 2.0 * sh.M * sh.N * sh.K;
    printf("M%d N%d K%d mode%d bias%d resid%d\n", sh.M, sh.N, sh.K, sh.mode, sh.bias, sh.resid);
    for (int round = 0; round < 2; ++round)
      for (auto& c : cfg) {
        smi_gemm_set_pipe(c[0], c[1], c[2] ? 128 : 64);
        GemmArgs gg = g;
        gg.C = c[0] ? C1 : C0;
        const float us = graph_time(gg);
        long bad = -1;
        if (c[0]) {
          std::vector<unsigned short> h0((size_t)sh.M * sh.N), h1((size_t)sh.M * sh.N);
          (void)hipMemcpy(h0.data(), C0, h0.size() * 2, hipMemcpyDeviceToHost);
          (void)hipMemcpy(h1.data(), C1, h1.size() * 2, hipMemcpyDeviceToHost);
          bad = 0;
          for (size_t i = 0; i < h0.size(); ++i) bad += h0[i] != h1[i];
        }
        printf("  r%d pipe tpw=%d ns=%d %s: %7.2f us %6.0f TF  mismatches %ld\n", round, c[0], c[1],
               c[2] ? "bm128" : "bm64 ", us, fl / us / 1e6, bad);
      }
  }
  return 0;
}
