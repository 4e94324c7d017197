// Split-plane fp32 GEMM, DGRAD instances (dX = dY . W with the fused residual / relu'-dropout
// epilogues; the weight is read k-major through ds_read_b64_tr_b16).  See smi_gemm_sp_impl.h.
#include "smi_gemm_sp_impl.h"

int smi_sp_launch_dgrad(const GemmSpArgs& g, int epi, int out, dim3 grid, bool t256, hipStream_t st) {
  const bool w8 = smi_sp_waves() == 8;
#define SPD(E, O)                                                                                  \
  do {                                                                                             \
    if (t256 && smi_sp_tm() == 16) hipLaunchKernelGGL((gemm_sp256m_kernel<false, true, E, O>), grid, dim3(512), 0, st, g); \
    else if (t256) hipLaunchKernelGGL((gemm_sp256_kernel<false, true, E, O>), grid, dim3(512), 0, st, g); \
    else if (w8) hipLaunchKernelGGL((gemm_sp_kernel<8, false, true, E, O>), grid, dim3(512), 0, st, g); \
    else hipLaunchKernelGGL((gemm_sp_kernel<4, false, true, E, O>), grid, dim3(256), 0, st, g);    \
  } while (0)
  if (epi == 0 && out == SO_C) SPD(0, SO_C);
  else if (epi == SE_RESID && out == SO_C) SPD(SE_RESID, SO_C);
  else if (epi == SE_DACT && out == SO_C) SPD(SE_DACT, SO_C);
  // the FFN's hidden gradient dh feeds only linear1's dgrad / wgrad: planes (+ fp32 on request)
  else if (epi == SE_DACT && out == SO_P) SPD(SE_DACT, SO_P);
  else if (epi == SE_DACT && out == (SO_C | SO_P)) SPD(SE_DACT, SO_C | SO_P);
  // the attention output's gradient dO (out-projection dgrad): planes for the attention backward
  // kernels (+ fp32 when a kernel without plane inputs reads it)
  // linear2's dgrad on the FFN hidden mask instead of the fp32 activation
  else if (epi == SE_DMASK && out == SO_P) SPD(SE_DMASK, SO_P);
  else if (epi == SE_DMASK && out == (SO_C | SO_P)) SPD(SE_DMASK, SO_C | SO_P);
  else if (epi == 0 && out == SO_P) SPD(0, SO_P);
  else if (epi == 0 && out == (SO_C | SO_P)) SPD(0, SO_C | SO_P);
  else return -1;
#undef SPD
  SMI_CHECK_LAUNCH();
}
