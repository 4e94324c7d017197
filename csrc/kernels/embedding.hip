// Token embedding gather fused with the sinusoidal positional-encoding add and dropout, and
// its scatter-add backward.
//
// Reference: SentenceEmbedding.forward = dropout_{0.1}(Embedding(x) + PE) (transformer.py:57-62;
// PE table transformer.py:33-42, precomputed once here instead of per forward) and
// the LSTM's plain nn.Embedding with padding_idx (distributed_lstm.py:115,128).
// Forward: one thread per 8 contiguous features (16-B loads of the bf16 table copy), bf16 out.
// Backward: fp32 atomic adds into the dense fp32 gradient table, rows == padding_idx skipped
// (that row's gradient stays zero like torch's padding_idx).  Dense semantics are kept on
// purpose: the reference's Adam decays every row.
#include "smi_common.h"

__global__ void emb_fwd_kernel(const long long* __restrict__ ids, const unsigned short* __restrict__ table,
                               const float* __restrict__ pe, unsigned short* __restrict__ out, long T, int D, int S,
                               const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale) {
  const uint32_t seed = smi_seed(seedp, salt);
  const int vpr = D / 8;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= T * vpr) return;
  const long t = i / vpr;
  const int c = (int)(i % vpr) * 8;
  const long id = ids[t];
  u16x8_t w = *(const u16x8_t*)(table + id * D + c);
  u16x8_t o;
  const float* pr = pe ? pe + (long)(t % S) * D + c : nullptr;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float x = bf2f(w[j]) + (pr ? pr[j] : 0.f);
    if (thresh) x = smi_keep(seed, (uint32_t)(t * D + c + j), thresh) ? x * dscale : 0.f;
    o[j] = f2bf(x);
  }
  *(u16x8_t*)(out + t * D + c) = o;
}

// one wave per token, lane = column (64 consecutive floats per atomic wave-instruction: the
// 256-B contiguous shape the memory-side float atomics run at full rate)
__global__ void emb_bwd_kernel(const long long* __restrict__ ids, const unsigned short* __restrict__ dout,
                               float* __restrict__ dtable, long T, int D, long long padding_idx,
                               const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale) {
  const uint32_t seed = smi_seed(seedp, salt);
  const int lane = threadIdx.x & 63;
  for (long t = (long)blockIdx.x * 4 + (threadIdx.x >> 6); t < T; t += (long)gridDim.x * 4) {
    const long long id = ids[t];
    if (id == padding_idx) continue;
    float* dst = dtable + id * D;
    for (int c = lane; c < D; c += 64) {
      float g = bf2f(dout[t * D + c]);
      if (thresh) g = smi_keep(seed, (uint32_t)(t * D + c), thresh) ? g * dscale : 0.f;
      atomicAdd(dst + c, g);
    }
  }
}

extern "C" int smi_emb_fwd(const long long* ids, const void* table, const float* pe, void* out, long T, int D, int S,
                           const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale, hipStream_t st) {
  if (D % 8) return -1;
  const long n = T * (D / 8);
  hipLaunchKernelGGL(emb_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, ids,
                     (const unsigned short*)table, pe, (unsigned short*)out, T, D, S, seedp, salt, thresh, dscale);
  SMI_CHECK_LAUNCH();
}

extern "C" int smi_emb_bwd(const long long* ids, const void* dout, float* dtable, long T, int D, long long padding_idx,
                           const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale, hipStream_t st) {
  long nb = (T + 3) / 4;
  if (nb > 4096) nb = 4096;
  hipLaunchKernelGGL(emb_bwd_kernel, dim3((unsigned)nb), dim3(256), 0, st, ids,
                     (const unsigned short*)dout, dtable, T, D, padding_idx, seedp, salt, thresh, dscale);
  SMI_CHECK_LAUNCH();
}
