// Argument block of the split-plane fp32 GEMM (csrc/kernels/gemm_sp*.hip).
//
// An fp32 matrix X is carried as three bf16 PLANES hi / mid / lo with X = hi + mid + lo exactly
// (each plane the round-to-nearest-even bf16 of the residual left by the planes before it), so
// every product of two fp32 values is the sum of six exact bf16 slice products.  A plane tensor
// is [3][rows][ld] bf16: plane p of X starts `ps` elements after plane p - 1.
#pragma once
#include <stdint.h>

struct GemmSpArgs {
  int mode;                         // 0 FWD (A, B k-contig), 1 DGRAD (B k-major), 2 WGRAD (A, B k-major)
  const unsigned short* A; long lda; long aps;   // plane 0 of A, row stride, plane stride (elements)
  const unsigned short* B; long ldb; long bps;
  int M, N, K;                      // C[M,N] = sum_k A(m,k) B(k,n)
  int kpad;                         // k-contig operands are zero-padded to a multiple of 32 in k
  float* C; long ldc;               // fp32 output (may be null when only planes are written)
  unsigned short* P; long ldp; long pps;  // optional plane output of the epilogue's result
  int beta_acc;                     // C += result
  const float* bias;                // FWD: + bias[N]
  int relu;                         // FWD: 1 relu after bias
  const float* resid; long ldr;     // DGRAD: + resid[M,N]
  const float* dact_y; long ldy;    // DGRAD: x [dact_y > 0] * dscale (relu + dropout backward)
  const uint32_t* seedp; uint32_t salt; uint32_t thresh; float dscale;  // FWD dropout / DGRAD mask scale
  float* bias_grad;                 // WGRAD: += row sums of A (dY^T 1, the bias gradient)
  unsigned char* mask; long ldm;    // FWD (out): bit e of mask[row][col / 4] = output (col + e) > 0;
                                    // DGRAD (in): the same mask replaces dact_y (relu' x dropout)
  int a_bytes, b_bytes;             // per-plane operand extents (filled by the launcher)
};
