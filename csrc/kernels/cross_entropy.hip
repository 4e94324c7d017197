// Softmax cross-entropy with ignore_index and mean over non-ignored rows, bf16/fp32 logits.
//
// Reference: nn.CrossEntropyLoss(ignore_index=0, reduction='none') followed by a manual masked
// mean over non-pad targets (pytorch_machine_translator.py:125-126,182-188); with ignore=-100
// and all rows valid it is the plain mean CE of the MLP/CNN/LSTM scripts
// (distributed_cnn.py:141, distributed_lstm.py:142,189).
// Forward: one 256-thread block per row, online (max, sum) pass over V with 16-B loads (4 in
// flight per thread); stores the row logsumexp and row loss; a one-block finalize sums them.
// Backward: grad = (softmax - onehot) * dloss / count, written in place or out of place; fp32
// path: optionally also its bf16 hi/mid/lo planes [3][M][ldp] (ldp >= V, zero columns V..ldp-1),
// the dY operand of the vocab projection's split-plane dgrad / wgrad (no separate split pass).
// The valid-row count lives on the device, so the whole loss is graph-capturable.
#include "smi_common.h"
#include "smi_split3.h"

// Sums the per-row losses and counts the valid rows (one block): a single-address atomic per row
// from 8192 blocks serialises at the L2 (~120 us measured), this is one pass over 32 KiB.
__global__ __launch_bounds__(1024) void ce_finalize_kernel(const long long* __restrict__ labels,
                                                           const float* __restrict__ row_loss, int M, long long ignore,
                                                           float* __restrict__ count, float* __restrict__ loss) {
  __shared__ float pc[16], pl[16];
  float c = 0.f, l = 0.f;
  for (int i = threadIdx.x; i < M; i += blockDim.x) {
    const bool v = labels[i] != ignore;
    c += v ? 1.f : 0.f;
    l += v ? row_loss[i] : 0.f;
  }
  c = wave_sum(c);
  l = wave_sum(l);
  if ((threadIdx.x & 63) == 0) { pc[threadIdx.x >> 6] = c; pl[threadIdx.x >> 6] = l; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float tc = 0.f, tl = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { tc += pc[w]; tl += pl[w]; }
    count[0] = tc;
    loss[0] = tc > 0.f ? tl / tc : 0.f;
  }
}

template <bool BF16>
__device__ __forceinline__ void load8f(const void* p, long idx, float (&x)[8]) {
  if (BF16) {
    u16x8_t v = *(const u16x8_t*)((const unsigned short*)p + idx);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = bf2f(v[j]);
  } else {
    float4 a = *(const float4*)((const float*)p + idx);
    float4 b = *(const float4*)((const float*)p + idx + 4);
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  }
}
template <bool BF16>
__device__ __forceinline__ float load1f(const void* p, long idx) {
  return BF16 ? bf2f(((const unsigned short*)p)[idx]) : ((const float*)p)[idx];
}

template <bool BF16>
__global__ __launch_bounds__(256) void ce_fwd_kernel(const void* __restrict__ logits, const long long* __restrict__ labels,
                                                     int V, long long ignore, float* __restrict__ lse_out,
                                                     float* __restrict__ row_loss) {
  const int row = blockIdx.x;
  const long base = (long)row * V;
  float m = -INFINITY, s = 0.f;
  const int nvec = (V % 8 == 0) ? V / 8 : 0;
  // 4 vectors (32 logits) per thread per chunk: all four loads are issued before any math, so
  // each thread has 4 independent loads in flight instead of one rolled-loop latency per vector
  for (int i0 = threadIdx.x; i0 < nvec; i0 += 4 * 256) {
    float x[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * 256;
      if (i < nvec) load8f<BF16>(logits, base + (long)i * 8, x[u]);
      else {
#pragma unroll
        for (int j = 0; j < 8; ++j) x[u][j] = -INFINITY;
      }
    }
    float lm = x[0][0];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) lm = fmaxf(lm, x[u][j]);
    const float nm = fmaxf(m, lm);
    float acc = (m == -INFINITY) ? 0.f : s * __expf(m - nm);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += __expf(x[u][j] - nm);
    s = acc; m = nm;
  }
  for (int i = nvec * 8 + threadIdx.x; i < V; i += 256) {
    const float x = load1f<BF16>(logits, base + i);
    const float nm = fmaxf(m, x);
    s = s * __expf(m - nm) + __expf(x - nm);
    m = nm;
  }
  // block-wide (max, sum) merge
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    const float nm = fmaxf(m, om);
    s = (nm == -INFINITY) ? 0.f : s * __expf(m - nm) + os * __expf(om - nm);
    m = nm;
  }
  __shared__ float sm[4], ss[4];
  if ((threadIdx.x & 63) == 0) { sm[threadIdx.x >> 6] = m; ss[threadIdx.x >> 6] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M0 = sm[0], S0 = ss[0];
    for (int w = 1; w < 4; ++w) {
      const float nm = fmaxf(M0, sm[w]);
      S0 = S0 * __expf(M0 - nm) + ss[w] * __expf(sm[w] - nm);
      M0 = nm;
    }
    const float lse = M0 + __logf(S0);
    lse_out[row] = lse;
    const long long lab = labels[row];
    row_loss[row] = (lab != ignore) ? lse - load1f<BF16>(logits, base + lab) : 0.f;
  }
}

template <bool BF16>
__global__ __launch_bounds__(256) void ce_bwd_kernel(const void* __restrict__ logits, const long long* __restrict__ labels,
                                                     int V, long long ignore, const float* __restrict__ lse_in,
                                                     const float* __restrict__ count, const float* __restrict__ dloss,
                                                     void* __restrict__ grad, unsigned short* __restrict__ P, long ldp,
                                                     long pps) {
  const int row = blockIdx.x;
  const long base = (long)row * V;
  const long long lab = labels[row];
  const float c = count[0];
  const float scale = (lab == ignore || c <= 0.f) ? 0.f : dloss[0] / c;
  const float lse = lse_in[row];
  const int nvec = (V % 8 == 0) ? V / 8 : 0;
  for (int i = threadIdx.x; i < nvec; i += 256) {
    float x[8];
    load8f<BF16>(logits, base + (long)i * 8, x);
    float gq[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = i * 8 + j;
      gq[j] = (__expf(x[j] - lse) - (col == lab ? 1.f : 0.f)) * scale;
    }
    if (BF16) {
      u16x8_t o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(gq[j]);
      *(u16x8_t*)((unsigned short*)grad + base + (long)i * 8) = o;
    } else {
      if (grad) {  // null: planes only (the vocab projection's dgrad / wgrad read nothing else)
        *(float4*)((float*)grad + base + (long)i * 8) = make_float4(gq[0], gq[1], gq[2], gq[3]);
        *(float4*)((float*)grad + base + (long)i * 8 + 4) = make_float4(gq[4], gq[5], gq[6], gq[7]);
      }
      if (P) {
        uint32_t h[4], m[4], l[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) split3_pair(gq[2 * e], gq[2 * e + 1], h[e], m[e], l[e]);
        unsigned short* q = P + (long)row * ldp + (long)i * 8;
        *(uint4*)q = make_uint4(h[0], h[1], h[2], h[3]);
        *(uint4*)(q + pps) = make_uint4(m[0], m[1], m[2], m[3]);
        *(uint4*)(q + 2 * pps) = make_uint4(l[0], l[1], l[2], l[3]);
      }
    }
  }
  for (int i = nvec * 8 + threadIdx.x; i < V; i += 256) {
    const float x = load1f<BF16>(logits, base + i);
    const float gq = (__expf(x - lse) - (i == lab ? 1.f : 0.f)) * scale;
    if (BF16) ((unsigned short*)grad)[base + i] = f2bf(gq);
    else if (grad) ((float*)grad)[base + i] = gq;
    if (!BF16 && P) {
      unsigned short* q = P + (long)row * ldp + i;
      const unsigned short hb = f2bf(gq);
      const float r = gq - bf2f(hb);
      const unsigned short mb = f2bf(r);
      q[0] = hb; q[pps] = mb; q[2 * pps] = f2bf(r - bf2f(mb));
    }
  }
  if (!BF16 && P) {  // the k padding of the GEMM operand
    for (long i = V + threadIdx.x; i < ldp; i += 256) {
      unsigned short* q = P + (long)row * ldp + i;
      q[0] = 0; q[pps] = 0; q[2 * pps] = 0;
    }
  }
}

extern "C" int smi_ce_fwd(const void* logits, int is_bf16, const long long* labels, int M, int V, long long ignore,
                          float* lse, float* count, float* loss, float* row_loss, hipStream_t st) {
  if (!row_loss) return -1;
  if (is_bf16)
    hipLaunchKernelGGL(ce_fwd_kernel<true>, dim3(M), dim3(256), 0, st, logits, labels, V, ignore, lse, row_loss);
  else
    hipLaunchKernelGGL(ce_fwd_kernel<false>, dim3(M), dim3(256), 0, st, logits, labels, V, ignore, lse, row_loss);
  hipLaunchKernelGGL(ce_finalize_kernel, dim3(1), dim3(1024), 0, st, labels, row_loss, M, ignore, count, loss);
  SMI_CHECK_LAUNCH();
}

extern "C" int smi_ce_bwd(const void* logits, int is_bf16, const long long* labels, int M, int V, long long ignore,
                          const float* lse, const float* count, const float* dloss, void* grad, void* planes, long ldp,
                          long pps, hipStream_t st) {
  unsigned short* P = (unsigned short*)planes;
  if (P && (is_bf16 || ldp < V || ldp % 8 || pps < (long)M * ldp || ((uintptr_t)P & 15))) return -1;
  if (!grad && !P) return -1;  // fp32 gradient omitted only when its planes are written
  if (is_bf16)
    hipLaunchKernelGGL(ce_bwd_kernel<true>, dim3(M), dim3(256), 0, st, logits, labels, V, ignore, lse, count, dloss, grad,
                       nullptr, 0L, 0L);
  else
    hipLaunchKernelGGL(ce_bwd_kernel<false>, dim3(M), dim3(256), 0, st, logits, labels, V, ignore, lse, count, dloss, grad,
                       P, ldp, pps);
  SMI_CHECK_LAUNCH();
}
