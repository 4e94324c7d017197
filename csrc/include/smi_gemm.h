// Argument block shared by csrc/kernels/gemm.hip and csrc/bindings.cpp.
#pragma once
#include <stdint.h>
struct GemmArgs {
  int mode;                 // 0 FWD (A k-contig, B k-contig), 1 DGRAD (B k-major), 2 WGRAD (A,B k-major)
  const unsigned short* A; long lda;
  const unsigned short* B; long ldb;
  int M, N, K;              // C[M,N] = sum_k A(m,k) B(k,n)
  void* C; long ldc;
  int out_f32, atomic, beta_acc;
  float alpha;
  const float* bias;                        // [N] fp32 (bf16-out modes)
  const unsigned short* resid; long ldr;    // [M,N] bf16 added before activation
  int act;                                  // 1 = relu
  const unsigned short* dact_y; long ldy;   // relu+dropout backward mask source (saved output)
  const uint32_t* seedp; uint32_t salt; uint32_t thresh; float dscale;  // dropout
  int splits;
  int k_per_split;          // filled by the launcher
  long a_bytes, b_bytes;    // operand extents for the buffer descriptors (filled by the launcher)
  long c_split_stride;      // split-K into slabs: split s writes C + s * c_split_stride (no atomics)
  float* bias_grad;         // WGRAD only: column sums of A (= dY^T 1, the bias gradient) computed by an
  long bias_split_stride;   // extra MFMA per fragment; slab mode writes + s*stride, atomic mode adds
};
