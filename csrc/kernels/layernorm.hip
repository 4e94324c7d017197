// Fused (dropout(h) + residual) -> LayerNorm forward / backward for post-LN transformer blocks.
//
// Reference semantics: transformer.py:86-101 (LayerNormalization: biased variance, eps inside
// sqrt, gamma*y+beta) applied as norm(dropout(sublayer(x)) + x) at transformer.py:131-138 and
// :209-223. One wave64 owns one row; each lane holds 8 contiguous bf16 (16-B loads), so D=512
// is one 1-KiB wave-instruction per tensor. Statistics are fp32; the pre-norm sum is saved in
// bf16 for the backward. dgamma/dbeta are reduced per block into fp32 partial slabs and summed
// by a second kernel that accumulates into the caller's (flat) fp32 gradient buffer.
#include "smi_common.h"

template <int VPL>  // 8-element vectors per lane: D <= VPL * 512, D % 8 == 0
__global__ __launch_bounds__(256) void ln_fwd_kernel(
    const unsigned short* __restrict__ h, const unsigned short* __restrict__ r,
    const float* __restrict__ gamma, const float* __restrict__ beta,
    unsigned short* __restrict__ y, unsigned short* __restrict__ xsave,
    float* __restrict__ mean_out, float* __restrict__ rstd_out,
    int M, int D, float eps, const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale) {
  const uint32_t seed = smi_seed(seedp, salt);
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + wid;
  if (row >= M) return;
  float x[VPL][8];
  const size_t base = (size_t)row * D;
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int col = v * 512 + lane * 8;
    if (col >= D) {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[v][j] = 0.f;
      continue;
    }
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
  const float invD = 1.0f / (float)D;
  const float mean = wave_sum(s) * invD;
  float q = 0.f;
#pragma unroll
  for (int v = 0; v < VPL; ++v)
#pragma unroll
    for (int j = 0; j < 8; ++j) { float d = (v * 512 + lane * 8 < D) ? x[v][j] - mean : 0.f; q += d * d; }
  const float var = wave_sum(q) * invD;
  const float rstd = 1.0f / sqrtf(var + eps);
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int col = v * 512 + lane * 8;
    if (col >= D) continue;
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
    int M, int D, const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale) {
  const uint32_t seed = smi_seed(seedp, salt);
  const float invD = 1.0f / (float)D;
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
    for (int j = 0; j < 8; ++j) gam[v][j] = (v * 512 + lane * 8 < D) ? gamma[v * 512 + lane * 8 + j] : 0.f;

  for (int row = blockIdx.x * 4 + wid; row < M; row += gridDim.x * 4) {
    const size_t base = (size_t)row * D;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[VPL][8], g[VPL][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int col = v * 512 + lane * 8;
      if (col >= D) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { xh[v][j] = 0.f; g[v][j] = 0.f; }
        continue;
      }
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
    s1 = wave_sum(s1) * invD;
    s2 = wave_sum(s2) * invD;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int col = v * 512 + lane * 8;
      if (col >= D) continue;
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
  __shared__ float red[2][4][VPL * 512];
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

// out[c] (+)= sum_b part[b][c]; two outputs (gamma, beta).  Block: 32 columns x 8 partial-row
// phases, so the nb-long sums run 8-wide in parallel and finish through LDS.
__global__ void colsum2_kernel(const float* __restrict__ pg, const float* __restrict__ pb, int nb, int D,
                               float* __restrict__ og, float* __restrict__ ob, int accumulate) {
  const int c = blockIdx.x * 32 + (threadIdx.x & 31);
  const int ph = threadIdx.x >> 5;
  float sg = 0.f, sb = 0.f;
  if (c < D)
    for (int b = ph; b < nb; b += 8) { sg += pg[(size_t)b * D + c]; sb += pb[(size_t)b * D + c]; }
  __shared__ float rg[8][33], rb[8][33];
  rg[ph][threadIdx.x & 31] = sg;
  rb[ph][threadIdx.x & 31] = sb;
  __syncthreads();
  if (ph == 0 && c < D) {
    for (int p = 1; p < 8; ++p) { sg += rg[p][threadIdx.x]; sb += rb[p][threadIdx.x]; }
    if (accumulate) { og[c] += sg; ob[c] += sb; } else { og[c] = sg; ob[c] = sb; }
  }
}

extern "C" int smi_ln_fwd(const void* h, const void* r, const float* gamma, const float* beta, void* y,
                          void* xsave, float* mean, float* rstd, int M, int D, float eps,
                          const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale, hipStream_t st) {
  dim3 grid((M + 3) / 4), block(256);
  const auto* hh = (const unsigned short*)h; const auto* rr = (const unsigned short*)r;
  auto* yy = (unsigned short*)y; auto* xx = (unsigned short*)xsave;
  if (D % 8 || D > 4096) return -1;
  const int vpl = (D + 511) / 512;
  if (vpl == 1) hipLaunchKernelGGL(ln_fwd_kernel<1>, grid, block, 0, st, hh, rr, gamma, beta, yy, xx, mean, rstd, M, D, eps, seedp, salt, thresh, dscale);
  else if (vpl == 2) hipLaunchKernelGGL(ln_fwd_kernel<2>, grid, block, 0, st, hh, rr, gamma, beta, yy, xx, mean, rstd, M, D, eps, seedp, salt, thresh, dscale);
  else if (vpl <= 4) hipLaunchKernelGGL(ln_fwd_kernel<4>, grid, block, 0, st, hh, rr, gamma, beta, yy, xx, mean, rstd, M, D, eps, seedp, salt, thresh, dscale);
  else hipLaunchKernelGGL(ln_fwd_kernel<8>, grid, block, 0, st, hh, rr, gamma, beta, yy, xx, mean, rstd, M, D, eps, seedp, salt, thresh, dscale);
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
  if (D % 8 || D > 2048) return -1;
  const int vpl = (D + 511) / 512;
  if (vpl == 1) hipLaunchKernelGGL(ln_bwd_kernel<1>, grid, block, 0, st, a, b, mean, rstd, gamma, o1, o2, ad, part_g, part_b, M, D, seedp, salt, thresh, dscale);
  else if (vpl == 2) hipLaunchKernelGGL(ln_bwd_kernel<2>, grid, block, 0, st, a, b, mean, rstd, gamma, o1, o2, ad, part_g, part_b, M, D, seedp, salt, thresh, dscale);
  else hipLaunchKernelGGL(ln_bwd_kernel<4>, grid, block, 0, st, a, b, mean, rstd, gamma, o1, o2, ad, part_g, part_b, M, D, seedp, salt, thresh, dscale);
  hipLaunchKernelGGL(colsum2_kernel, dim3((D + 31) / 32), dim3(256), 0, st, part_g, part_b, nblocks, D, dgamma, dbeta, accumulate);
  SMI_CHECK_LAUNCH();
}
