// Phase stamps + K-scan of the split-plane fp32 GEMM forward (csrc/include/smi_gemm_sp_impl.h),
// diagnostic build (SP_STAMPS): per workgroup, s_memrealtime at kernel entry, after the first
// stage landed (prologue), after the k-loop, after the LDS epilogue staging, after the stores.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -DSP_STAMPS -Icsrc/include tools/probes/sp_probe.hip -o sp_probe
#include "smi_gemm_sp_impl.h"
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
  const int M = 8192, N = argc > 1 ? atoi(argv[1]) : 512, nw = argc > 2 ? atoi(argv[2]) : 8;
  const int Ks[] = {64, 128, 256, 512, 1024, 2048};
  const int Kmax = 2048;
  std::vector<unsigned short> h((size_t)3 * M * Kmax);
  srand(1);
  for (auto& v : h) v = (unsigned short)(0x3C00 + (rand() & 0x7FF)) ^ ((rand() & 1) << 15);  // |x| in [2^-7, 2)
  unsigned short *A, *B;
  float *C, *bias;
  CK(hipMalloc(&A, 2 * (size_t)3 * M * Kmax));
  CK(hipMalloc(&B, 2 * (size_t)3 * N * Kmax));
  CK(hipMalloc(&C, 4 * (size_t)M * N));
  CK(hipMalloc(&bias, 4 * (size_t)N));
  CK(hipMemset(bias, 0, 4 * N));
  CK(hipMemcpy(A, h.data(), 2 * (size_t)3 * M * Kmax, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data(), 2 * (size_t)3 * N * Kmax, hipMemcpyHostToDevice));
  const int nwg = (M / 128) * ((N + 127) / 128);
  unsigned long long* st;
  CK(hipMalloc(&st, 8 * 8 * (size_t)nwg));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_sp_stamps), &st, sizeof(st)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<unsigned long long> hs((size_t)nwg * 8);
  for (int K : Ks) {
    GemmSpArgs g{};
    g.mode = 0; g.A = A; g.lda = K; g.aps = (long)M * K; g.B = B; g.ldb = K; g.bps = (long)N * K;
    g.M = M; g.N = N; g.K = K; g.C = C; g.ldc = N; g.bias = bias; g.dscale = 1.f;
    g.a_bytes = 2 * ((M - 1) * K + K); g.b_bytes = 2 * ((N - 1) * K + K);
    auto launch = [&]() {
      if (nw == 8) hipLaunchKernelGGL((gemm_sp_kernel<8, false, false, SE_BIAS, SO_C>), dim3(nwg), dim3(512), 0, 0, g);
      else hipLaunchKernelGGL((gemm_sp_kernel<4, false, false, SE_BIAS, SO_C>), dim3(nwg), dim3(256), 0, 0, g);
    };
    for (int it = 0; it < 3; ++it) launch();
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0));
    for (int it = 0; it < reps; ++it) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipMemcpy(hs.data(), st, 8 * 8 * (size_t)nwg, hipMemcpyDeviceToHost));
    unsigned long long t0min = ~0ull, t4max = 0;
    double ph[4] = {0, 0, 0, 0};
    for (int b = 0; b < nwg; ++b) {
      const unsigned long long* s = &hs[(size_t)b * 8];
      if (s[0] < t0min) t0min = s[0];
      if (s[4] > t4max) t4max = s[4];
      for (int p = 0; p < 4; ++p) ph[p] += (double)(s[p + 1] - s[p]);
    }
    const double us = ms * 1000.0 / reps;
    const double fl = 2.0 * M * N * K;
    printf("waves=%d K=%5d N=%d kernel %.1f us (%.0f TF)  last launch span %.1f us | per-WG avg us: prologue %.2f  kloop %.2f "
           "(%.3f per k-step)  epi-stage %.2f  epi-store %.2f\n",
           nw, K, N, us, fl / (us * 1e-6) / 1e12, (t4max - t0min) / 100.0, ph[0] / nwg / 100.0, ph[1] / nwg / 100.0,
           ph[1] / nwg / 100.0 / (K / 32), ph[2] / nwg / 100.0, ph[3] / nwg / 100.0);
  }
  return 0;
}
