// Exact fp32 products on the bf16 matrix cores: x = hi + mid + lo (three bf16 slices), shared by
// the fp32 GEMM (csrc/kernels/gemm_f32.hip) and the fp32 attention (attention_f32.hip).
#pragma once
#include "smi_common.h"

struct Split3 { bf16x8_t h, m, l; };
__device__ __forceinline__ void split3_pair(float x0, float x1, uint32_t& h, uint32_t& m, uint32_t& l) {
  h = pack2bf(x0, x1);
  const float r0 = x0 - __uint_as_float(h << 16), r1 = x1 - __uint_as_float(h & 0xFFFF0000u);
  m = pack2bf(r0, r1);
  const float s0 = r0 - __uint_as_float(m << 16), s1 = r1 - __uint_as_float(m & 0xFFFF0000u);
  l = pack2bf(s0, s1);
}
// 8 consecutive fragment values f[o..o+7] -> the three bf16x8 MFMA operands
__device__ __forceinline__ Split3 split3_8(const float* f) {
  uint32_t h[4], m[4], l[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) split3_pair(f[2 * q], f[2 * q + 1], h[q], m[q], l[q]);
  Split3 r;
  r.h = __builtin_bit_cast(bf16x8_t, (uint4){h[0], h[1], h[2], h[3]});
  r.m = __builtin_bit_cast(bf16x8_t, (uint4){m[0], m[1], m[2], m[3]});
  r.l = __builtin_bit_cast(bf16x8_t, (uint4){l[0], l[1], l[2], l[3]});
  return r;
}
#define MF32X16(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16((a), (b), (c), 0, 0, 0)

// acc += x . y over a chain of T f32-MFMA steps (v_mfma_f32_32x32x2_f32 takes x[t], y[t] from lane
// half h as k = (h, t)); the split form regroups 8 consecutive steps into one 32x32x16 block
// (lane half h supplies k = 8h + e <-> step 8j + e of the same lane), six slice products per block
// summed smallest first into the same accumulator (6 roundings per 16 k vs 8 for the f32 chain).
template <int XS, int T>
__device__ __forceinline__ f32x16_t f32_chain(const float (&x)[T], const float (&y)[T], f32x16_t acc) {
  if constexpr (XS == 0) {
#pragma unroll
    for (int t = 0; t < T; ++t) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x[t], y[t], acc, 0, 0, 0);
  } else {
#pragma unroll
    for (int j = 0; j < T / 8; ++j) {
      const Split3 a = split3_8(&x[8 * j]), b = split3_8(&y[8 * j]);
      acc = MF32X16(a.l, b.h, acc);
      acc = MF32X16(a.m, b.m, acc);
      acc = MF32X16(a.h, b.l, acc);
      acc = MF32X16(a.m, b.h, acc);
      acc = MF32X16(a.h, b.m, acc);
      acc = MF32X16(a.h, b.h, acc);
    }
  }
  return acc;
}

// the same chain with y already split (an operand reused across chunks: split once per kernel)
template <int XS, int T>
struct F32Pre {
  Split3 s[XS ? T / 8 : 1];
  __device__ __forceinline__ void set(const float (&y)[T]) {
    if constexpr (XS != 0) {
#pragma unroll
      for (int j = 0; j < T / 8; ++j) s[j] = split3_8(&y[8 * j]);
    }
  }
};
template <int XS, int T>
__device__ __forceinline__ f32x16_t f32_chain_pre(const float (&x)[T], const float (&y)[T], const F32Pre<XS, T>& ys,
                                                  f32x16_t acc) {
  if constexpr (XS == 0) {
    return f32_chain<0, T>(x, y, acc);
  } else {
#pragma unroll
    for (int j = 0; j < T / 8; ++j) {
      const Split3 a = split3_8(&x[8 * j]);
      const Split3& b = ys.s[j];
      acc = MF32X16(a.l, b.h, acc);
      acc = MF32X16(a.m, b.m, acc);
      acc = MF32X16(a.h, b.l, acc);
      acc = MF32X16(a.m, b.h, acc);
      acc = MF32X16(a.h, b.m, acc);
      acc = MF32X16(a.h, b.h, acc);
    }
    return acc;
  }
}
