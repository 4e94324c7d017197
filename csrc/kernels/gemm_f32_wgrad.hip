// fp32 GEMM, WGRAD instantiations (dW += dY^T . X, + bias gradient): the standalone split-K /
// accumulate launches and the grouped launch of a whole backward's weight gradients; split from
// gemm_f32.hip so the per-mode kernel sets compile in parallel (csrc/include/smi_gemm_f32_impl.h).
#include "smi_gemm_f32_impl.h"

extern "C" int smi_gemm_f32_algo(int set);

int smi_f32_launch_wgrad(const GemmF32Args& g, int fe, int algo, dim3 grid2, hipStream_t st) {
  const dim3 block(256);
#define F32PW(E)                                                                                  \
  do {                                                                                            \
    if (algo == 0) hipLaunchKernelGGL((gemm_f32_pipe_kernel<true, true, E, 0>), grid2, block, 0, st, g); \
    else hipLaunchKernelGGL((gemm_f32_pipe_kernel<true, true, E, 1>), grid2, block, 0, st, g);      \
  } while (0)
  if (fe == FE_ACC) F32PW(FE_ACC);
  else if (fe == FE_ATOMIC) F32PW(FE_ATOMIC);
  else F32PW(-1);
#undef F32PW
  SMI_CHECK_LAUNCH();
}

extern "C" int smi_gemm_f32_wgrad_group(const void* const* A, const long* lda, const void* const* B, const long* ldb,
                                        void* const* C, void* const* bias, const int* n, const int* k, const int* T,
                                        int count, hipStream_t st) {
  if (count < 1 || count > WGF_MAX) return -1;
  WgradGroupF32 gr{};
  int tot = 0;
  for (int i = 0; i < count; ++i) {
    if (T[i] < 1 || n[i] < 4 || k[i] < 4 || n[i] % 4 || k[i] % 4 || lda[i] % 4 || ldb[i] % 4) return -1;
    if (lda[i] < n[i] || ldb[i] < k[i] || lda[i] > (1L << 30) || ldb[i] > (1L << 30)) return -1;
    if ((((uintptr_t)A[i]) | ((uintptr_t)B[i])) & 15) return -1;
    gr.A[i] = (const float*)A[i]; gr.B[i] = (const float*)B[i];
    gr.C[i] = (float*)C[i]; gr.bias[i] = (float*)bias[i];
    gr.lda[i] = (int)lda[i]; gr.ldb[i] = (int)ldb[i]; gr.n[i] = n[i]; gr.k[i] = k[i]; gr.T[i] = T[i];
    gr.t0[i] = tot;
    const int nwg = ((n[i] + 127) / 128) * ((k[i] + FBN - 1) / FBN);
    tot += (nwg + 7) / 8 * 8;
  }
  gr.t0[count] = tot;
  gr.count = count;
  if (smi_gemm_f32_algo(-1) == 0) hipLaunchKernelGGL(gemm_f32_wgrad_group_kernel<0>, dim3(tot), dim3(256), 0, st, gr);
  else hipLaunchKernelGGL(gemm_f32_wgrad_group_kernel<1>, dim3(tot), dim3(256), 0, st, gr);
  SMI_CHECK_LAUNCH();
}
