// Argument block of the fp32 (reference-precision) GEMM, csrc/kernels/gemm_f32.hip.
#pragma once
#include <stdint.h>
struct GemmF32Args {
  int mode;                 // 0 FWD (A,B k-contig), 1 DGRAD (B k-major), 2 WGRAD (A,B k-major)
  const float* A; long lda;
  const float* B; long ldb;
  int M, N, K;              // C[M,N] = sum_k A(m,k) B(k,n)
  float* C; long ldc;
  int beta_acc;             // C += result (else C = result)
  int atomic;               // split-K partial sums added with fp32 atomics (WGRAD fallback)
  const float* bias;        // [N] added in the epilogue (FWD)
  int relu;                 // FWD activation after bias: 1 relu, 2 sigmoid
  const float* resid; long ldr;    // DGRAD: + resid[M,N]
  const float* dact_y; long ldy;   // DGRAD: relu+dropout backward mask source (saved FWD output)
  const uint32_t* seedp; uint32_t salt; uint32_t thresh; float dscale;  // dropout (FWD) / mask scale (DGRAD)
  int splits, k_per_split;  // split-K (filled by the launcher)
  float* bias_grad;         // WGRAD: += row sums of A (dY^T 1 = the bias gradient)
};
