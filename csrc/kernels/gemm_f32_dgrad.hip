// fp32 GEMM, DGRAD instantiations (dX = dY . W, + residual / relu'-dropout mask): split from
// gemm_f32.hip so the per-mode kernel sets compile in parallel (csrc/include/smi_gemm_f32_impl.h).
#include "smi_gemm_f32_impl.h"

int smi_f32_launch_dgrad(const GemmF32Args& g, int fe, int algo, dim3 grid2, hipStream_t st) {
  const dim3 block(256);
#define F32PD(E)                                                                                  \
  do {                                                                                            \
    if (algo == 0) hipLaunchKernelGGL((gemm_f32_pipe_kernel<false, true, E, 0>), grid2, block, 0, st, g); \
    else hipLaunchKernelGGL((gemm_f32_pipe_kernel<false, true, E, 2>), grid2, block, 0, st, g);     \
  } while (0)
  switch (fe) {
    case 0: F32PD(0); break;
    case FE_RESID: F32PD(FE_RESID); break;
    case FE_DACT: F32PD(FE_DACT); break;
    default: F32PD(-1); break;
  }
#undef F32PD
  SMI_CHECK_LAUNCH();
}
