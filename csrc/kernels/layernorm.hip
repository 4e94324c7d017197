// Fused (dropout(h) + residual) -> LayerNorm forward / backward for post-LN transformer blocks.
//
// Reference semantics: transformer.py:86-101 (LayerNormalization: biased variance, eps inside
// sqrt, gamma*y+beta) applied as norm(dropout(sublayer(x)) + x) at transformer.py:131-138 and
// :209-223. One wave64 owns one row; each lane holds 8 contiguous elements (bf16: one 16-B load,
// fp32 reference-precision path: two), so D=512 is one 1-KiB (2-KiB) wave-instruction per tensor.
// Statistics are fp32; the pre-norm sum is saved in the activation dtype for the backward. dgamma/dbeta are reduced per block into fp32 partial slabs and summed
// by a second kernel that accumulates into the caller's (flat) fp32 gradient buffer.
#include "smi_common.h"
#include "smi_split3.h"

// fp32 path: the output's bf16 hi/mid/lo planes ([3][M][D], plane stride pps) for the split-plane
// GEMM that consumes it (sparkmi/ops/planes.py), written beside the fp32 store
__device__ __forceinline__ void ln_store_planes(unsigned short* P, long pps, const float (&v)[8]) {
  uint32_t h[4], m[4], l[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) split3_pair(v[2 * e], v[2 * e + 1], h[e], m[e], l[e]);
  *(uint4*)P = make_uint4(h[0], h[1], h[2], h[3]);
  *(uint4*)(P + pps) = make_uint4(m[0], m[1], m[2], m[3]);
  *(uint4*)(P + 2 * pps) = make_uint4(l[0], l[1], l[2], l[3]);
}

// Every global load a row needs (h, r, gamma, beta; the dropout seed) is issued before the
// first reduction: a load that depends on a reduction result serialises two memory latencies
// per wave (measured: 20 us -> 8.6 us at 8192 x 512 for hoisting gamma/beta alone).
// T = activation storage: unsigned short (bf16 path) or float (fp32 reference-precision path).
template <int VPL, typename T>  // 8-element vectors per lane: D <= VPL * 512, D % 8 == 0
__global__ __launch_bounds__(256) void ln_fwd_kernel(
    const T* __restrict__ h, const T* __restrict__ r,
    const float* __restrict__ gamma, const float* __restrict__ beta,
    T* __restrict__ y, T* __restrict__ xsave,
    float* __restrict__ mean_out, float* __restrict__ rstd_out,
    int M, int D, float eps, const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale,
    unsigned short* __restrict__ yp, long pps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (row >= M) return;
  const size_t base = (size_t)row * D;
  V8<T> hv[VPL], rv[VPL];
  float4 g0[VPL], g1[VPL], b0[VPL], b1[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int col = v * 512 + lane * 8;
    if (col < D) {
      hv[v].load(h + base + col);
      if (r) rv[v].load(r + base + col);
      g0[v] = *(const float4*)(gamma + col); g1[v] = *(const float4*)(gamma + col + 4);
      b0[v] = *(const float4*)(beta + col); b1[v] = *(const float4*)(beta + col + 4);
    }
  }
  const uint32_t seed = thresh ? smi_seed(seedp, salt) : 0u;
  float x[VPL][8];
  float s = 0.f;
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int col = v * 512 + lane * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a = 0.f;
      if (col < D) {
        a = hv[v][j];
        if (thresh) a = smi_keep(seed, (uint32_t)(base + col + j), thresh) ? a * dscale : 0.f;
        if (r) a += rv[v][j];
      }
      x[v][j] = a;
      s += a;
    }
  }
  const float invD = 1.0f / (float)D;
  const float mean = wave_sum(s) * invD;
  float q = 0.f;
#pragma unroll
  for (int v = 0; v < VPL; ++v)
#pragma unroll
    for (int j = 0; j < 8; ++j) { float d = (v * 512 + lane * 8 < D) ? x[v][j] - mean : 0.f; q += d * d; }
  const float rstd = rsqrtf(wave_sum(q) * invD + eps);
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int col = v * 512 + lane * 8;
    if (col >= D) continue;
    const float gg[8] = {g0[v].x, g0[v].y, g0[v].z, g0[v].w, g1[v].x, g1[v].y, g1[v].z, g1[v].w};
    const float bb[8] = {b0[v].x, b0[v].y, b0[v].z, b0[v].w, b1[v].x, b1[v].y, b1[v].z, b1[v].w};
    float out[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = (x[v][j] - mean) * rstd * gg[j] + bb[j];
    V8<T>::store(y + base + col, out);
    if (yp) ln_store_planes(yp + base + col, pps, out);
    if (xsave) V8<T>::store(xsave + base + col, x[v]);
  }
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// Backward: each wave owns RPW consecutive rows and issues ALL their loads (dy, xs, dres_add,
// mean, rstd) up front, then runs the per-row math; dgamma/dbeta partials of the block's
// 4*RPW rows are reduced across waves through LDS into one [D] slab row per block.
template <int VPL, int RPW, typename T>
__global__ __launch_bounds__(256) void ln_bwd_kernel(
    const T* __restrict__ dy, const T* __restrict__ xs,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const float* __restrict__ gamma,
    T* __restrict__ dres, T* __restrict__ dh,
    const T* __restrict__ dres_add,
    float* __restrict__ part_g, float* __restrict__ part_b,
    int M, int D, const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale,
    unsigned short* __restrict__ dhp, long pps) {
  const float invD = 1.0f / (float)D;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int row0 = (blockIdx.x * 4 + wid) * RPW;
  V8<T> dv[RPW][VPL], xv[RPW][VPL], av[RPW][VPL];
  float mean[RPW], rstd[RPW];
  float4 ga[VPL], gb[VPL];
#pragma unroll
  for (int v = 0; v < VPL; ++v) {
    const int col = v * 512 + lane * 8;
    if (col < D) { ga[v] = *(const float4*)(gamma + col); gb[v] = *(const float4*)(gamma + col + 4); }
  }
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int row = row0 + rr;
    if (row >= M) continue;
    const size_t base = (size_t)row * D;
    mean[rr] = mean_in[row];
    rstd[rr] = rstd_in[row];
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int col = v * 512 + lane * 8;
      if (col < D) {
        dv[rr][v].load(dy + base + col);
        xv[rr][v].load(xs + base + col);
        if (dres_add) av[rr][v].load(dres_add + base + col);
      }
    }
  }
  const uint32_t seed = thresh ? smi_seed(seedp, salt) : 0u;
  float pg[VPL][8], pb[VPL][8];
#pragma unroll
  for (int v = 0; v < VPL; ++v)
#pragma unroll
    for (int j = 0; j < 8; ++j) { pg[v][j] = 0.f; pb[v][j] = 0.f; }
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int row = row0 + rr;
    if (row >= M) continue;
    const size_t base = (size_t)row * D;
    float xh[VPL][8], g[VPL][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int col = v * 512 + lane * 8;
      const float gam[8] = {ga[v].x, ga[v].y, ga[v].z, ga[v].w, gb[v].x, gb[v].y, gb[v].z, gb[v].w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (col < D) {
          const float d = dv[rr][v][j];
          xh[v][j] = (xv[rr][v][j] - mean[rr]) * rstd[rr];
          g[v][j] = d * gam[j];
          pg[v][j] += d * xh[v][j];
          pb[v][j] += d;
        } else {
          xh[v][j] = 0.f; g[v][j] = 0.f;
        }
        s1 += g[v][j];
        s2 += g[v][j] * xh[v][j];
      }
    }
    s1 = wave_sum(s1) * invD;
    s2 = wave_sum(s2) * invD;
#pragma unroll
    for (int v = 0; v < VPL; ++v) {
      const int col = v * 512 + lane * 8;
      if (col >= D) continue;
      float o1[8], o2[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float dx = rstd[rr] * (g[v][j] - s1 - xh[v][j] * s2);
        o1[j] = dx + (dres_add ? av[rr][v][j] : 0.f);
        float dd = dx;
        if (thresh) dd = smi_keep(seed, (uint32_t)(base + col + j), thresh) ? dx * dscale : 0.f;
        o2[j] = dd;
      }
      if (dres) V8<T>::store(dres + base + col, o1);
      if (dh) V8<T>::store(dh + base + col, o2);
      if (dhp) ln_store_planes(dhp + base + col, pps, o2);
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

// out[c] (+)= sum_b part[b][c] for two outputs (gamma, beta).  Grid (D/64, row groups): each
// block sums its share of the partial rows for 64 columns with 4 row phases (coalesced 256-B
// row segments, all loads of a thread independent), combines the phases in LDS and adds its
// result with one atomic per column (several row groups) or a plain store (one group).
__global__ __launch_bounds__(256) void colsum2_kernel(const float* __restrict__ pg, const float* __restrict__ pb, int nb,
                                                      int D, float* __restrict__ og, float* __restrict__ ob,
                                                      int accumulate) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int ph = threadIdx.x >> 6;
  const int rows_per = (nb + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * rows_per, r1 = min(nb, r0 + rows_per);
  float sg = 0.f, sb = 0.f;
  if (c < D) {
#pragma unroll 4
    for (int b = r0 + ph; b < r1; b += 4) { sg += pg[(size_t)b * D + c]; sb += pb[(size_t)b * D + c]; }
  }
  __shared__ float rg[4][64], rb[4][64];
  rg[ph][threadIdx.x & 63] = sg;
  rb[ph][threadIdx.x & 63] = sb;
  __syncthreads();
  if (ph == 0 && c < D) {
    sg = (rg[0][threadIdx.x] + rg[1][threadIdx.x]) + (rg[2][threadIdx.x] + rg[3][threadIdx.x]);
    sb = (rb[0][threadIdx.x] + rb[1][threadIdx.x]) + (rb[2][threadIdx.x] + rb[3][threadIdx.x]);
    if (gridDim.y > 1) { atomicAdd(og + c, sg); atomicAdd(ob + c, sb); }
    else if (accumulate) { og[c] += sg; ob[c] += sb; }
    else { og[c] = sg; ob[c] = sb; }
  }
}

template <typename T>
static int ln_fwd_launch(const void* h, const void* r, const float* gamma, const float* beta, void* y, void* xsave,
                         float* mean, float* rstd, int M, int D, float eps, const uint32_t* seedp, uint32_t salt,
                         uint32_t thresh, float dscale, void* planes, long pps, hipStream_t st) {
  dim3 grid((M + 3) / 4), block(256);
  unsigned short* yp = (unsigned short*)planes;
  const T* hh = (const T*)h; const T* rr = (const T*)r;
  T* yy = (T*)y; T* xx = (T*)xsave;
  if (D % 8 || D > 4096) return -1;
  const int vpl = (D + 511) / 512;
  if (vpl == 1) hipLaunchKernelGGL((ln_fwd_kernel<1, T>), grid, block, 0, st, hh, rr, gamma, beta, yy, xx, mean, rstd, M, D, eps, seedp, salt, thresh, dscale, yp, pps);
  else if (vpl == 2) hipLaunchKernelGGL((ln_fwd_kernel<2, T>), grid, block, 0, st, hh, rr, gamma, beta, yy, xx, mean, rstd, M, D, eps, seedp, salt, thresh, dscale, yp, pps);
  else if (vpl <= 4) hipLaunchKernelGGL((ln_fwd_kernel<4, T>), grid, block, 0, st, hh, rr, gamma, beta, yy, xx, mean, rstd, M, D, eps, seedp, salt, thresh, dscale, yp, pps);
  else hipLaunchKernelGGL((ln_fwd_kernel<8, T>), grid, block, 0, st, hh, rr, gamma, beta, yy, xx, mean, rstd, M, D, eps, seedp, salt, thresh, dscale, yp, pps);
  SMI_CHECK_LAUNCH();
}

extern "C" int smi_ln_fwd(const void* h, const void* r, const float* gamma, const float* beta, void* y,
                          void* xsave, float* mean, float* rstd, int M, int D, float eps,
                          const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale, hipStream_t st) {
  return ln_fwd_launch<unsigned short>(h, r, gamma, beta, y, xsave, mean, rstd, M, D, eps, seedp, salt, thresh, dscale,
                                       nullptr, 0, st);
}
extern "C" int smi_ln_fwd_f32(const void* h, const void* r, const float* gamma, const float* beta, void* y,
                              void* xsave, float* mean, float* rstd, int M, int D, float eps,
                              const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale, void* planes,
                              long pps, hipStream_t st) {
  // planes: [3][M][D] bf16 of y (or null); D % 8 == 0 keeps every 16-B plane store aligned
  if (planes && (((uintptr_t)planes & 15) || pps < (long)M * D)) return -1;
  return ln_fwd_launch<float>(h, r, gamma, beta, y, xsave, mean, rstd, M, D, eps, seedp, salt, thresh, dscale, planes,
                              pps, st);
}

template <typename T>
static int ln_bwd_launch(const void* dy, const void* xs, const float* mean, const float* rstd,
                         const float* gamma, void* dres, void* dh, const void* dres_add,
                         float* part_g, float* part_b, int nblocks, float* dgamma, float* dbeta,
                         int accumulate, int M, int D, const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale,
                         void* planes, long pps, hipStream_t st) {
  unsigned short* dhp = (unsigned short*)planes;
  // nblocks = capacity (rows) of the partial slabs; the kernel needs ceil(M / (4 * RPW)) of them
  const T* a = (const T*)dy; const T* b = (const T*)xs;
  T* o1 = (T*)dres; T* o2 = (T*)dh;
  const T* ad = (const T*)dres_add;
  if (D % 8 || D > 2048) return -1;
  const int vpl = (D + 511) / 512;
  const int rpw = vpl <= 2 ? 2 : 1;
  const int nb = (M + 4 * rpw - 1) / (4 * rpw);
  if (nb > nblocks) return -1;
  dim3 grid(nb), block(256);
  if (vpl == 1) hipLaunchKernelGGL((ln_bwd_kernel<1, 2, T>), grid, block, 0, st, a, b, mean, rstd, gamma, o1, o2, ad, part_g, part_b, M, D, seedp, salt, thresh, dscale, dhp, pps);
  else if (vpl == 2) hipLaunchKernelGGL((ln_bwd_kernel<2, 2, T>), grid, block, 0, st, a, b, mean, rstd, gamma, o1, o2, ad, part_g, part_b, M, D, seedp, salt, thresh, dscale, dhp, pps);
  else hipLaunchKernelGGL((ln_bwd_kernel<4, 1, T>), grid, block, 0, st, a, b, mean, rstd, gamma, o1, o2, ad, part_g, part_b, M, D, seedp, salt, thresh, dscale, dhp, pps);
  if (dgamma) {  // else the caller reduces the partials itself (smi_ln_bwd_reduce, e.g. on a side stream)
    const int groups = accumulate ? (nb >= 1024 ? 16 : (nb >= 256 ? 8 : (nb >= 64 ? 4 : 1))) : 1;
    hipLaunchKernelGGL(colsum2_kernel, dim3((D + 63) / 64, groups), dim3(256), 0, st, part_g, part_b, nb, D, dgamma, dbeta,
                       accumulate);
  }
  SMI_CHECK_LAUNCH();
}

extern "C" int smi_ln_bwd(const void* dy, const void* xs, const float* mean, const float* rstd,
                          const float* gamma, void* dres, void* dh, const void* dres_add,
                          float* part_g, float* part_b, int nblocks, float* dgamma, float* dbeta,
                          int accumulate, int M, int D, const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale,
                          hipStream_t st) {
  return ln_bwd_launch<unsigned short>(dy, xs, mean, rstd, gamma, dres, dh, dres_add, part_g, part_b, nblocks, dgamma,
                                       dbeta, accumulate, M, D, seedp, salt, thresh, dscale, nullptr, 0, st);
}
extern "C" int smi_ln_bwd_f32(const void* dy, const void* xs, const float* mean, const float* rstd,
                              const float* gamma, void* dres, void* dh, const void* dres_add,
                              float* part_g, float* part_b, int nblocks, float* dgamma, float* dbeta,
                              int accumulate, int M, int D, const uint32_t* seedp, uint32_t salt, uint32_t thresh,
                              float dscale, void* planes, long pps, hipStream_t st) {
  // planes: [3][M][D] bf16 of dh (or null)
  // dh null with planes: the sublayer's last Linear reads dh's planes only (planes-only output)
  if (planes && (((uintptr_t)planes & 15) || pps < (long)M * D)) return -1;
  if (!planes && !dh) return -1;
  return ln_bwd_launch<float>(dy, xs, mean, rstd, gamma, dres, dh, dres_add, part_g, part_b, nblocks, dgamma, dbeta,
                              accumulate, M, D, seedp, salt, thresh, dscale, planes, pps, st);
}

// dgamma/dbeta (+)= column sums of the nb partial rows written by smi_ln_bwd
extern "C" int smi_ln_bwd_reduce(const float* part_g, const float* part_b, int nb, int D, float* dgamma, float* dbeta,
                                 int accumulate, hipStream_t st) {
  const int groups = accumulate ? (nb >= 1024 ? 16 : (nb >= 256 ? 8 : (nb >= 64 ? 4 : 1))) : 1;
  hipLaunchKernelGGL(colsum2_kernel, dim3((D + 63) / 64, groups), dim3(256), 0, st, part_g, part_b, nb, D, dgamma, dbeta,
                     accumulate);
  SMI_CHECK_LAUNCH();
}

// Deferred dgamma/dbeta folds of up to 32 LayerNorm backwards in ONE launch (the per-LN colsum2
// launch is ~2 us of work and ~5 us in the step: 30 per transformer step).  blockIdx.y = LN,
// 16 row phases of 64 columns per block, fixed-order combine: deterministic.
#define LN_MULTI 32
struct Colsum2Multi {
  const float* pg[LN_MULTI]; const float* pb[LN_MULTI]; float* og[LN_MULTI]; float* ob[LN_MULTI];
  int nb[LN_MULTI]; int D[LN_MULTI]; int accumulate;
};
__global__ __launch_bounds__(1024) void colsum2_multi_kernel(Colsum2Multi a) {
  const int e = blockIdx.y;
  const int D = a.D[e], nb = a.nb[e];
  if ((int)blockIdx.x * 64 >= D) return;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int ph = threadIdx.x >> 6;  // 16 phases
  const float* pg = a.pg[e];
  const float* pb = a.pb[e];
  float sg = 0.f, sb = 0.f;
  if (c < D) {
#pragma unroll 4
    for (int b = ph; b < nb; b += 16) { sg += pg[(size_t)b * D + c]; sb += pb[(size_t)b * D + c]; }
  }
  __shared__ float rg[16][64], rb[16][64];
  rg[ph][threadIdx.x & 63] = sg;
  rb[ph][threadIdx.x & 63] = sb;
  __syncthreads();
  if (ph == 0 && c < D) {
    float tg = 0.f, tb = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) { tg += rg[i][threadIdx.x]; tb += rb[i][threadIdx.x]; }
    if (a.accumulate) { a.og[e][c] += tg; a.ob[e][c] += tb; }
    else { a.og[e][c] = tg; a.ob[e][c] = tb; }
  }
}

extern "C" int smi_ln_bwd_reduce_multi(const float* const* pg, const float* const* pb, float* const* og, float* const* ob,
                                       const int* nb, const int* D, int count, int accumulate, hipStream_t st) {
  if (count < 1 || count > LN_MULTI) return -1;
  Colsum2Multi a{};
  int maxd = 0;
  for (int i = 0; i < count; ++i) {
    a.pg[i] = pg[i]; a.pb[i] = pb[i]; a.og[i] = og[i]; a.ob[i] = ob[i]; a.nb[i] = nb[i]; a.D[i] = D[i];
    if (D[i] > maxd) maxd = D[i];
  }
  a.accumulate = accumulate;
  hipLaunchKernelGGL(colsum2_multi_kernel, dim3((maxd + 63) / 64, count), dim3(1024), 0, st, a);
  SMI_CHECK_LAUNCH();
}
