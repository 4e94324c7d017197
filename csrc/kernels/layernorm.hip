// Fused (dropout(h) + residual) -> LayerNorm forward / backward for post-LN transformer blocks.
//
// Reference semantics: transformer.py:86-101 (LayerNormalization: biased variance, eps inside
// sqrt, gamma*y+beta) applied as norm(dropout(sublayer(x)) + x) at transformer.py:131-138 and
// :209-223. One wave64 owns one row; each lane holds 8 contiguous bf16 (16-B loads), so D=512
// is one 1-KiB wave-instruction per tensor. Statistics are fp32; the pre-norm sum is saved in
// bf16 for the backward. dgamma/dbeta are reduced per block into fp32 partial slabs and summed
// by a second kernel that accumulates into the caller's (flat) fp32 gradient buffer.
#include "smi_common.h"

template <int VPL>  // 8-element vectors per lane: D = VPL * 512
__global__ __launch_bounds__(256) void ln_fwd_kernel(
    const unsigned short* __restrict__ h, const unsigned short* __restrict__ r,
    const float* __restrict__ gamma, const float* __restrict__ beta,
    unsigned short* __restrict__ y, unsigned short* __restrict__ xsave,
    float* __restrict__ mean_out, float* __restrict__ rstd_out,
    int M, float eps, const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale) {
  const uint32_t seed = smi_seed(seedp, salt);
  constexpr int D = VPL * 512;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + wid;
  if (row >= M) return;
  float x[VPL][8];
  const size_t base = (size_t)row * D;
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int col = v * 512 + lane * 8;
    u16x8_t hv = *(const u16x8_t*)(h + base + col);
    u16x8_t rv;
    if (r) rv = *(const u16x8_t*)(r + base + col);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a = bf2f(hv[j]);
      if (thresh) a = smi_keep(seed, (uint32_t)(base + col + j), thresh) ? a * dscale : 0.f;
      x[v][j] = a + (r ? bf2f(rv[j]) : 0.f);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int v = 0; v < VPL; ++v)
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[v][j];
  const float mean = wave_sum(s) * (1.0f / D);
  float q = 0.f;
#pragma unroll
  for (int v = 0; v < VPL; ++v)
#pragma unroll
    for (int j = 0; j < 8; ++j) { float d = x[v][j] - mean; q += d * d; }
  const float var = wave_sum(q) * (1.0f / D);
  const float rstd = 1.0f / sqrtf(var + eps);
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int col = v * 512 + lane * 8;
    u16x8_t out, xs;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      out[j] = f2bf((x[v][j] - mean) * rstd * gamma[col + j] + beta[col + j]);
      xs[j] = f2bf(x[v][j]);
    }
    *(u16x8_t*)(y + base + col) = out;
    if (xsave) *(u16x8_t*)(xsave + base + col) = xs;
  }
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// Backward. grid-stride over rows, 4 waves per block; per-lane dgamma/dbeta partials for
// its 8*VPL columns accumulate in registers and are reduced across waves through LDS.
template <int VPL>
__global__ __launch_bounds__(256) void ln_bwd_kernel(
    const unsigned short* __restrict__ dy, const unsigned short* __restrict__ xs,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const float* __restrict__ gamma,
    unsigned short* __restrict__ dres, unsigned short* __restrict__ dh,
    const unsigned short* __restrict__ dres_add,
    float* __restrict__ part_g, float* __restrict__ part_b,
    int M, const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale) {
  const uint32_t seed = smi_seed(seedp, salt);
  constexpr int D = VPL * 512;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  float pg[VPL][8], pb[VPL][8];
#pragma unroll
  for (int v = 0; v < VPL; ++v)
#pragma unroll
    for (int j = 0; j < 8; ++j) { pg[v][j] = 0.f; pb[v][j] = 0.f; }
  float gam[VPL][8];
#pragma unroll
  for (int v = 0; v < VPL; ++v)
#pragma unroll
    for (int j = 0; j < 8; ++j) gam[v][j] = gamma[v * 512 + lane * 8 + j];

  for (int row = blockIdx.x * 4 + wid; row < M; row += gridDim.x * 4) {
    const size_t base = (size_t)row * D;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[VPL][8], g[VPL][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int col = v * 512 + lane * 8;
      u16x8_t dv = *(const u16x8_t*)(dy + base + col);
      u16x8_t xv = *(const u16x8_t*)(xs + base + col);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float d = bf2f(dv[j]);
        xh[v][j] = (bf2f(xv[j]) - mean) * rstd;
        g[v][j] = d * gam[v][j];
        s1 += g[v][j];
        s2 += g[v][j] * xh[v][j];
        pg[v][j] += d * xh[v][j];
        pb[v][j] += d;
      }
    }
    s1 = wave_sum(s1) * (1.0f / D);
    s2 = wave_sum(s2) * (1.0f / D);
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int col = v * 512 + lane * 8;
      u16x8_t o1, o2, ad;
      if (dres_add) ad = *(const u16x8_t*)(dres_add + base + col);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float dx = rstd * (g[v][j] - s1 - xh[v][j] * s2);
        float dr = dx + (dres_add ? bf2f(ad[j]) : 0.f);
        o1[j] = f2bf(dr);
        float dd = dx;
        if (thresh) dd = smi_keep(seed, (uint32_t)(base + col + j), thresh) ? dx * dscale : 0.f;
        o2[j] = f2bf(dd);
      }
      if (dres) *(u16x8_t*)(dres + base + col) = o1;
      if (dh) *(u16x8_t*)(dh + base + col) = o2;
    }
  }
  __shared__ float red[2][4][D];
#pragma unroll
  for (int v = 0; v < VPL; ++v)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[0][wid][v * 512 + lane * 8 + j] = pg[v][j];
      red[1][wid][v * 512 + lane * 8 + j] = pb[v][j];
    }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += 256) {
    part_g[(size_t)blockIdx.x * D + c] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
    part_b[(size_t)blockIdx.x * D + c] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
  }
}

// out[c] (+)= sum_b part[b][c]; two outputs (gamma, beta)
__global__ void colsum2_kernel(const float* __restrict__ pg, const float* __restrict__ pb, int nb, int D,
                               float* __restrict__ og, float* __restrict__ ob, int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= D) return;
  float sg = 0.f, sb = 0.f;
  for (int b = 0; b < nb; ++b) { sg += pg[(size_t)b * D + c]; sb += pb[(size_t)b * D + c]; }
  if (accumulate) { og[c] += sg; ob[c] += sb; } else { og[c] = sg; ob[c] = sb; }
}

extern "C" int smi_ln_fwd(const void* h, const void* r, const float* gamma, const float* beta, void* y,
                          void* xsave, float* mean, float* rstd, int M, int D, float eps,
                          const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale, hipStream_t st) {
  dim3 grid((M + 3) / 4), block(256);
  const auto* hh = (const unsigned short*)h; const auto* rr = (const unsigned short*)r;
  auto* yy = (unsigned short*)y; auto* xx = (unsigned short*)xsave;
  switch (D) {
    case 512: hipLaunchKernelGGL(ln_fwd_kernel<1>, grid, block, 0, st, hh, rr, gamma, beta, yy, xx, mean, rstd, M, eps, seedp, salt, thresh, dscale); break;
    case 1024: hipLaunchKernelGGL(ln_fwd_kernel<2>, grid, block, 0, st, hh, rr, gamma, beta, yy, xx, mean, rstd, M, eps, seedp, salt, thresh, dscale); break;
    case 2048: hipLaunchKernelGGL(ln_fwd_kernel<4>, grid, block, 0, st, hh, rr, gamma, beta, yy, xx, mean, rstd, M, eps, seedp, salt, thresh, dscale); break;
    default: return -1;
  }
  SMI_CHECK_LAUNCH();
}

extern "C" int smi_ln_bwd(const void* dy, const void* xs, const float* mean, const float* rstd,
                          const float* gamma, void* dres, void* dh, const void* dres_add,
                          float* part_g, float* part_b, int nblocks, float* dgamma, float* dbeta,
                          int accumulate, int M, int D, const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale,
                          hipStream_t st) {
  dim3 grid(nblocks), block(256);
  const auto* a = (const unsigned short*)dy; const auto* b = (const unsigned short*)xs;
  auto* o1 = (unsigned short*)dres; auto* o2 = (unsigned short*)dh;
  const auto* ad = (const unsigned short*)dres_add;
  switch (D) {
    case 512: hipLaunchKernelGGL(ln_bwd_kernel<1>, grid, block, 0, st, a, b, mean, rstd, gamma, o1, o2, ad, part_g, part_b, M, seedp, salt, thresh, dscale); break;
    case 1024: hipLaunchKernelGGL(ln_bwd_kernel<2>, grid, block, 0, st, a, b, mean, rstd, gamma, o1, o2, ad, part_g, part_b, M, seedp, salt, thresh, dscale); break;
    default: return -1;
  }
  hipLaunchKernelGGL(colsum2_kernel, dim3((D + 255) / 256), dim3(256), 0, st, part_g, part_b, nblocks, D, dgamma, dbeta, accumulate);
  SMI_CHECK_LAUNCH();
}
