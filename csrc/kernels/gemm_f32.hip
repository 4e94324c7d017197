// fp32 GEMM on the fp32-input matrix cores (v_mfma_f32_32x32x2_f32: exact f32 products and an
// f32 fmaf accumulation chain, 64 FLOP/clk/SIMD = 157 TF dense) with the same fused epilogues as
// the bf16 GEMM — the REFERENCE-PRECISION path of every Linear of the reference models
// (transformer.py:71-72,107-117,175-176,271 run in fp32 by pytorch_machine_translator.py:120-137):
//
//   FWD   C[M,N]  = X[M,K] . W[N,K]^T  (+bias, ReLU, dropout)        A k-contig, B k-contig
//   DGRAD dX[M,K] = dY[M,N] . W[N,K]   (+residual, x relu'/dropout)  A k-contig, B k-major
//   WGRAD dW[N,K] += dY[M,N]^T . X[M,K] (+ bias grad = dY^T 1)       A k-major,  B k-major
//
// CDNA4 design.  The f32 MFMA runs at 1/16 of the bf16 rate, so this kernel is matrix-core bound
// by a wide margin (a 32-deep k-tile of a 128 x 128 tile = 64 MFMAs = 4096 cycles per
// SIMD against 32 KiB of L2 -> LDS traffic per workgroup): everything else is arranged so the
// MFMA pipe never idles —
//  * 256-thread workgroups (2 x 2 waves), BN = 128, BM = 64 or 128 (a wave owns 32*FM x 64 =
//    FM x 2 accumulators of 32 x 32), two workgroups per CU so one's barrier / epilogue overlaps
//    the other's MFMAs;
//  * register-staged double buffering: the next k-tile's float4 global loads are issued before
//    the current k-tile's MFMAs and written to the other LDS buffer after them — one barrier
//    per k-tile, global latency hidden under 2-4 k us of matrix work;
//  * k-permuted fragments: lane half h of a 32x32x2 MFMA supplies k = 16h + s at step s, so a
//    k-contiguous operand is read as four ds_read_b128 per 16 steps from an LDS image with a
//    36-float row pitch (conflict-free for the ds_read_b128 lane groups), and a k-major operand
//    as ds_read_b32 rows (32 consecutive floats per half-wave: conflict-free, no transpose);
//  * XCD-aware tile order (tiles sharing an A row-panel run on one XCD's L2).
// The accumulator layout (col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)) gives each
// store instruction two full 128-B row segments.
#include "smi_gemm_f32_impl.h"

// fp32 product algorithm: 0 = f32 MFMA (v_mfma_f32_32x32x2_f32), 6 = 3-way bf16 split, 6 terms
// (SMI_F32_ALGO; see split3_8)
int smi_f32_launch_dgrad(const GemmF32Args& g, int fe, int algo, dim3 grid2, hipStream_t st);
int smi_f32_launch_wgrad(const GemmF32Args& g, int fe, int algo, dim3 grid2, hipStream_t st);

static int g_f32_algo = -1;
static int smi_f32_algo() {
  if (g_f32_algo < 0) {
    g_f32_algo = 6;
  }
  return g_f32_algo;
}
extern "C" int smi_gemm_f32_algo(int set) {  // set < 0: query only
  if (set == 0 || set == 6) g_f32_algo = set;
  return smi_f32_algo();
}

static int f32_ok(const GemmF32Args& g) {
  if (g.M < 1 || g.N < 1 || g.K < 1) return 0;
  const bool ak = g.mode == 2, bk = g.mode != 0;
  // float4 staging granularity along each operand's contiguous dimension, 16-B aligned rows
  if ((!ak && g.K % 4) || (ak && g.M % 4) || (!bk && g.K % 4) || (bk && g.N % 4)) return 0;
  if (g.lda % 4 || g.ldb % 4) return 0;
  if (((uintptr_t)g.A | (uintptr_t)g.B) & 15) return 0;
  return 1;
}

extern "C" int smi_gemm_f32(const GemmF32Args* args, hipStream_t st) {
  GemmF32Args g = *args;
  if (!f32_ok(g) || g.mode < 0 || g.mode > 2) return -1;
  const bool ak = g.mode == 2;
  if (g.splits < 1) g.splits = 1;
  if (g.splits > 1 && !g.atomic) return -1;
  int kps = (g.K / g.splits + FBK - 1) / FBK * FBK;
  if (kps < FBK) kps = FBK;
  g.k_per_split = kps;
  g.splits = (g.K + kps - 1) / kps;
  const dim3 block(256);
  {  // the software-pipelined one-wave-per-SIMD kernel
    const int nwg128 = ((g.M + 127) / 128) * ((g.N + FBN - 1) / FBN);
    const dim3 grid2((unsigned)(nwg128 * g.splits));
    // specialised epilogues for the feature sets the models use; anything else -> generic (-1)
    int fe = 0;
    if (g.mode == 0) {
      fe = (g.bias ? FE_BIAS : 0) | (g.relu == 1 ? FE_RELU : 0) | (g.relu == 2 ? FE_SIG : 0) | (g.thresh ? FE_DROP : 0);
    } else if (g.mode == 1) {
      fe = (g.resid ? FE_RESID : 0) | (g.dact_y ? FE_DACT : 0);
    }
    fe |= (g.atomic ? FE_ATOMIC : (g.beta_acc ? FE_ACC : 0));
// split path per mode (measured, tools/f32_split_check.py): FWD and DGRAD split once at staging
// into LDS bf16 planes (XS 2; the k-major DGRAD weight through ds_read_b64_tr_b16), WGRAD splits
// the fp32 fragments per wave (XS 1: 520 vs 563 us for a decoder layer's grouped launch)
#define F32P(AKV, BKV, E)                                                                          \
  do {                                                                                             \
    if (smi_f32_algo() == 0) hipLaunchKernelGGL((gemm_f32_pipe_kernel<AKV, BKV, E, 0>), grid2, block, 0, st, g); \
    else hipLaunchKernelGGL((gemm_f32_pipe_kernel<AKV, BKV, E, (AKV ? 1 : 2)>), grid2, block, 0, st, g); \
  } while (0)
    if (g.mode == 0) {
      switch (fe) {
        case 0: F32P(false, false, 0); break;
        case FE_BIAS: F32P(false, false, FE_BIAS); break;
        case FE_BIAS | FE_RELU: F32P(false, false, FE_BIAS | FE_RELU); break;
        case FE_BIAS | FE_RELU | FE_DROP: F32P(false, false, FE_BIAS | FE_RELU | FE_DROP); break;
        default: F32P(false, false, -1); break;
      }
    } else if (g.mode == 1) {
      return smi_f32_launch_dgrad(g, fe, smi_f32_algo(), grid2, st);  // csrc/kernels/gemm_f32_dgrad.hip
    } else {
      return smi_f32_launch_wgrad(g, fe, smi_f32_algo(), grid2, st);  // csrc/kernels/gemm_f32_wgrad.hip
    }
#undef F32P
    SMI_CHECK_LAUNCH();
  }
}

