// Token embedding gather fused with the sinusoidal positional-encoding add and dropout, and
// its scatter-add backward.
//
// Reference: SentenceEmbedding.forward = dropout_{0.1}(Embedding(x) + PE) (transformer.py:57-62;
// PE table transformer.py:33-42, precomputed once here instead of per forward) and
// the LSTM's plain nn.Embedding with padding_idx (distributed_lstm.py:115,128).
// Forward: one thread per 8 contiguous features (16-B loads of the bf16 table copy), bf16 out.
// Backward: fp32 atomic adds (runs of equal ids merged first) into the dense fp32 gradient
// table, rows == padding_idx skipped
// (that row's gradient stays zero like torch's padding_idx).  Dense semantics are kept on
// purpose: the reference's Adam decays every row.
#include "smi_common.h"

// T = storage of the table copy and the output: unsigned short (bf16 shadow) or float (fp32
// reference-precision path: the fp32 master table itself).
template <typename T>
__global__ void emb_fwd_kernel(const long long* __restrict__ ids, const T* __restrict__ table,
                               const float* __restrict__ pe, T* __restrict__ out, long Tn, int D, int S,
                               const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale) {
  const uint32_t seed = smi_seed(seedp, salt);
  const int vpr = D / 8;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Tn * vpr) return;
  const long t = i / vpr;
  const int c = (int)(i % vpr) * 8;
  const long id = ids[t];
  V8<T> w;
  w.load(table + id * D + c);
  float o[8];
  const float* pr = pe ? pe + (long)(t % S) * D + c : nullptr;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float x = w[j] + (pr ? pr[j] : 0.f);
    if (thresh) x = smi_keep(seed, (uint32_t)(t * D + c + j), thresh) ? x * dscale : 0.f;
    o[j] = x;
  }
  V8<T>::store(out + t * D + c, o);
}

// One wave per run of EMB_RUN consecutive tokens, lane = column (a wave-instruction covers 64
// consecutive columns: 128-B coalesced loads, and 256-B contiguous float atomics — the shape the
// memory-side atomics run at full rate).  The wave loads all its rows first, then walks them in
// order and merges consecutive tokens with the same id in registers, so a run of equal ids (the
// padding tail of every sequence: ~25 % of the reference's tokens share one id) costs one atomic
// row per wave instead of one per token (same-address float atomics serialise at the L2).
#define EMB_RUN 8
__device__ __forceinline__ float emb_ld(const unsigned short* p) { return bf2f(*p); }
__device__ __forceinline__ float emb_ld(const float* p) { return *p; }
template <typename TS>
__global__ __launch_bounds__(256) void emb_bwd_kernel(const long long* __restrict__ ids,
                                                      const TS* __restrict__ dout,
                                                      float* __restrict__ dtable, long T, int D, long long padding_idx,
                                                      const uint32_t* seedp, uint32_t salt, uint32_t thresh,
                                                      float dscale) {
  const uint32_t seed = thresh ? smi_seed(seedp, salt) : 0u;
  const int lane = threadIdx.x & 63;
  const long t0 = ((long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * EMB_RUN;
  if (t0 >= T) return;
  const int nt = (int)min((long)EMB_RUN, T - t0);
  long long id[EMB_RUN];
#pragma unroll
  for (int i = 0; i < EMB_RUN; ++i) id[i] = i < nt ? ids[t0 + i] : padding_idx;
  for (int c0 = 0; c0 < D; c0 += 512) {
    float v[EMB_RUN][8];
#pragma unroll
    for (int i = 0; i < EMB_RUN; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c0 + j * 64 + lane;
        v[i][j] = (i < nt && c < D) ? emb_ld(dout + (t0 + i) * D + c) : 0.f;
      }
    float acc[8];
    long long cur = -1;
#pragma unroll
    for (int i = 0; i <= EMB_RUN; ++i) {
      const long long nid = (i < nt) ? id[i] : -2;
      if (nid != cur) {
        if (cur >= 0 && cur != padding_idx) {
          float* dst = dtable + cur * D + c0 + lane;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (c0 + j * 64 + lane < D) atomicAdd(dst + j * 64, acc[j]);
        }
        cur = nid;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = 0.f;
      }
      if (i < nt) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float g = v[i][j];
          if (thresh) g = smi_keep(seed, (uint32_t)((t0 + i) * D + c0 + j * 64 + lane), thresh) ? g * dscale : 0.f;
          acc[j] += g;
        }
      }
    }
  }
}

extern "C" int smi_emb_fwd(const long long* ids, const void* table, const float* pe, void* out, long T, int D, int S,
                           const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale, hipStream_t st) {
  if (D % 8) return -1;
  const long n = T * (D / 8);
  hipLaunchKernelGGL(emb_fwd_kernel<unsigned short>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, ids,
                     (const unsigned short*)table, pe, (unsigned short*)out, T, D, S, seedp, salt, thresh, dscale);
  SMI_CHECK_LAUNCH();
}
extern "C" int smi_emb_fwd_f32(const long long* ids, const void* table, const float* pe, void* out, long T, int D, int S,
                               const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale, hipStream_t st) {
  if (D % 8) return -1;
  const long n = T * (D / 8);
  hipLaunchKernelGGL(emb_fwd_kernel<float>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, ids,
                     (const float*)table, pe, (float*)out, T, D, S, seedp, salt, thresh, dscale);
  SMI_CHECK_LAUNCH();
}

extern "C" int smi_emb_bwd(const long long* ids, const void* dout, float* dtable, long T, int D, long long padding_idx,
                           const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale, hipStream_t st) {
  const long waves = (T + EMB_RUN - 1) / EMB_RUN;
  hipLaunchKernelGGL(emb_bwd_kernel<unsigned short>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, ids,
                     (const unsigned short*)dout, dtable, T, D, padding_idx, seedp, salt, thresh, dscale);
  SMI_CHECK_LAUNCH();
}
extern "C" int smi_emb_bwd_f32(const long long* ids, const void* dout, float* dtable, long T, int D, long long padding_idx,
                               const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale, hipStream_t st) {
  const long waves = (T + EMB_RUN - 1) / EMB_RUN;
  hipLaunchKernelGGL(emb_bwd_kernel<float>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, ids,
                     (const float*)dout, dtable, T, D, padding_idx, seedp, salt, thresh, dscale);
  SMI_CHECK_LAUNCH();
}
