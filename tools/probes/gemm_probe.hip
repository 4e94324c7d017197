// GEMM ablation probe (8192 x 512 x 512 and friends): the production kernel vs builds without
// LDS-DMA staging (-DGEMM_PROBE_NODMA) or without MFMA (-DGEMM_PROBE_NOMFMA), HIP-event timed.
#include "../../csrc/kernels/gemm.hip"
#include <cstdio>
#include <cstdlib>

template <class F>
float timeit(F f, int it = 50) {
  for (int i = 0; i < 5; ++i) f();
  hipEvent_t s, e;
  (void)hipEventCreate(&s); (void)hipEventCreate(&e);
  (void)hipEventRecord(s);
  for (int i = 0; i < it; ++i) f();
  (void)hipEventRecord(e);
  (void)hipEventSynchronize(e);
  float ms; (void)hipEventElapsedTime(&ms, s, e);
  return ms * 1000.f / it;
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 8192, N = argc > 2 ? atoi(argv[2]) : 512, K = argc > 3 ? atoi(argv[3]) : 512;
  const int mode = argc > 4 ? atoi(argv[4]) : 0;
  unsigned short *A, *B, *C;
  float* Cf;
  (void)hipMalloc(&A, (size_t)M * K * 2 + (size_t)K * M * 2);
  (void)hipMalloc(&B, (size_t)N * K * 2 + (size_t)K * N * 2);
  (void)hipMalloc(&C, (size_t)M * N * 2);
  (void)hipMalloc(&Cf, (size_t)M * N * 4);
  (void)hipMemset(A, 0, (size_t)M * K * 4);
  (void)hipMemset(B, 0, (size_t)N * K * 4);
  GemmArgs g{};
  g.mode = mode; g.alpha = 1.f; g.dscale = 1.f; g.splits = 1;
  if (mode == 0) { g.A = A; g.lda = K; g.B = B; g.ldb = K; g.M = M; g.N = N; g.K = K; g.C = C; g.ldc = N; }
  else if (mode == 1) { g.A = A; g.lda = N; g.B = B; g.ldb = K; g.M = M; g.N = K; g.K = N; g.C = C; g.ldc = K; }
  else { g.A = A; g.lda = N; g.B = B; g.ldb = K; g.M = N; g.N = K; g.K = M; g.C = Cf; g.ldc = K; g.out_f32 = 1; g.atomic = 1;
         g.splits = argc > 5 ? atoi(argv[5]) : 8; }
  const double fl = 2.0 * M * N * K;
  const float us = timeit([&] { smi_gemm(&g, 0); });
  printf("M%d N%d K%d mode%d: %.2f us  %.0f TF\n", M, N, K, mode, us, fl / us / 1e6);
  return 0;
}
