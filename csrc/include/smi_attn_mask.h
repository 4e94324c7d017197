// Mask / bias helpers shared by the bf16 (attention.hip) and fp32 (attention_f32.hip) attention
// kernels.  Reference semantics: transformer.py:12-25 + SURVEY.md Q6 — mode 0 none, 1 "reference"
// (+1.0 on keys strictly before the query, in log2 units LOG2E), 2 causal (-inf on later keys); an
// optional uint8 key-padding vector adds -inf.
#pragma once
#include "smi_common.h"

#define LOG2E_F 1.4426950408889634f

// Masked, biased, log2-scaled score for key kj / query qi; -inf where masked.  Specialised on
// the mask mode at compile time (the generic form was ~4x the VALU work of the softmax itself):
// `full` (uniform) = the whole key chunk is inside Sk; `kmask` = the chunk's padded keys.
template <int MODE, bool KPAD>
__device__ __forceinline__ float score_adj(float s, int qi, int kj, int kl, bool full, int Sk, unsigned long long kmask,
                                           float scale_log2) {
  float x = s * scale_log2;
  if (MODE == 1) x += (kj < qi) ? LOG2E_F : 0.f;
  if (MODE == 2) x = (kj > qi) ? -INFINITY : x;
  if (KPAD) x = ((kmask >> kl) & 1ull) ? -INFINITY : x;
  if (!full) x = (kj >= Sk) ? -INFINITY : x;
  return x;
}

// Block-vs-rows classification (wave-uniform): with keys [k0, k0+KW) and query rows [qlo, qhi],
// is the mask/bias the same for every pair?  Returns true and the common log2-domain bias (0,
// LOG2E, or -inf = all masked) when it is, so the per-element path only runs on the diagonal
// blocks and on ragged / padded ones.
template <int MODE, bool KPAD, int KW = 64>
__device__ __forceinline__ bool uniform_bias(int k0, int qlo, int qhi, bool full, float& bias) {
  if (KPAD || !full) return false;
  if (MODE == 0) { bias = 0.f; return true; }
  if (k0 + KW - 1 < qlo) { bias = (MODE == 1) ? LOG2E_F : 0.f; return true; }  // every key before every query
  if (MODE == 1 && k0 >= qhi) { bias = 0.f; return true; }                     // no key strictly before
  if (MODE == 2 && k0 > qhi) { bias = -INFINITY; return true; }                // every key after every query
  return false;
}

// bit i = key k0 + i is padded (64 keys per chunk, one per lane)
__device__ __forceinline__ unsigned long long chunk_pad_mask(const unsigned char* kp, int k0, int Sk) {
  const int k = k0 + (threadIdx.x & 63);
  return __ballot(k < Sk && kp[k] != 0);
}
