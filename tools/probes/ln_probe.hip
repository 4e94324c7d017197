// LayerNorm-forward variants at 8192 x 512 bf16: find what keeps the current kernel at ~20 us.
#include "../../csrc/kernels/layernorm.hip"
#include <cstdio>

// V: 0 = baseline structure with vector gamma/beta loads hoisted before the reductions
//    1 = + no seed load (thresh 0 path compiled out)
//    2 = + DPP-free: single-pass (sum, sumsq) reduction
template <int V>
__global__ __launch_bounds__(256) void ln2(const unsigned short* __restrict__ h, const unsigned short* __restrict__ r,
                                           const float* __restrict__ gamma, const float* __restrict__ beta,
                                           unsigned short* __restrict__ y, unsigned short* __restrict__ xsave,
                                           float* __restrict__ mean_out, float* __restrict__ rstd_out, int M, int D,
                                           float eps, const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const size_t base = (size_t)row * D;
  const int col = lane * 8;
  const u16x8_t hv = *(const u16x8_t*)(h + base + col);
  const u16x8_t rv = *(const u16x8_t*)(r + base + col);
  const float4 g0 = *(const float4*)(gamma + col), g1 = *(const float4*)(gamma + col + 4);
  const float4 b0 = *(const float4*)(beta + col), b1 = *(const float4*)(beta + col + 4);
  uint32_t seed = 0;
  if (V == 0) seed = smi_seed(seedp, salt);
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float a = bf2f(hv[j]);
    if (V == 0 && thresh) a = smi_keep(seed, (uint32_t)(base + col + j), thresh) ? a * dscale : 0.f;
    x[j] = a + bf2f(rv[j]);
  }
  float mean, rstd;
  if (V == 2) {
    float s = 0.f, q = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) { s += x[j]; q += x[j] * x[j]; }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { s += __shfl_xor(s, o, 64); q += __shfl_xor(q, o, 64); }
    mean = s / D;
    rstd = rsqrtf(fmaxf(q / D - mean * mean, 0.f) + eps);
  } else {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j];
    mean = wave_sum(s) / D;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) { const float d = x[j] - mean; q += d * d; }
    rstd = rsqrtf(wave_sum(q) / D + eps);
  }
  const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
  const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
  u16x8_t out, xs;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    out[j] = f2bf((x[j] - mean) * rstd * gg[j] + bb[j]);
    xs[j] = f2bf(x[j]);
  }
  *(u16x8_t*)(y + base + col) = out;
  *(u16x8_t*)(xsave + base + col) = xs;
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// one wave: only loads + stores + reductions, no gamma/beta
__global__ __launch_bounds__(256) void ln_nogb(const unsigned short* __restrict__ h, const unsigned short* __restrict__ r,
                                               unsigned short* __restrict__ y, unsigned short* __restrict__ xsave, int M,
                                               int D) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const size_t base = (size_t)row * D;
  const int col = lane * 8;
  const u16x8_t hv = *(const u16x8_t*)(h + base + col);
  const u16x8_t rv = *(const u16x8_t*)(r + base + col);
  float x[8], s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) { x[j] = bf2f(hv[j]) + bf2f(rv[j]); s += x[j]; }
  const float mean = wave_sum(s) / D;
  u16x8_t out, xs;
#pragma unroll
  for (int j = 0; j < 8; ++j) { out[j] = f2bf(x[j] - mean); xs[j] = f2bf(x[j]); }
  *(u16x8_t*)(y + base + col) = out;
  *(u16x8_t*)(xsave + base + col) = xs;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)
template <class F>
float timeit(F f, int it = 50) {
  for (int i = 0; i < 5; ++i) f();
  hipEvent_t s, e;
  (void)hipEventCreate(&s); (void)hipEventCreate(&e);
  (void)hipEventRecord(s);
  for (int i = 0; i < it; ++i) f();
  (void)hipEventRecord(e);
  (void)hipEventSynchronize(e);
  float ms; (void)hipEventElapsedTime(&ms, s, e);
  return ms * 1000.f / it;
}

int main() {
  const int M = 8192, D = 512;
  const size_t n = (size_t)M * D;
  unsigned short *a, *b, *c, *d;
  float *g, *be, *mean, *rstd;
  unsigned int* seed;
  CK(hipMalloc(&a, n * 2)); CK(hipMalloc(&b, n * 2)); CK(hipMalloc(&c, n * 2)); CK(hipMalloc(&d, n * 2));
  CK(hipMalloc(&g, D * 4)); CK(hipMalloc(&be, D * 4)); CK(hipMalloc(&mean, M * 4)); CK(hipMalloc(&rstd, M * 4));
  CK(hipMalloc(&seed, 4));
  CK(hipMemset(a, 0, n * 2)); CK(hipMemset(b, 0, n * 2)); CK(hipMemset(g, 0, D * 4)); CK(hipMemset(be, 0, D * 4));
  CK(hipMemset(seed, 0, 4));
  const double bytes = 4.0 * n * 2;
  auto rep = [&](const char* name, float us) { printf("%-28s %8.2f us  %7.0f GB/s\n", name, us, bytes / us / 1e3); };
  rep("ln_fwd current", timeit([&] { smi_ln_fwd(a, b, g, be, c, d, mean, rstd, M, D, 1e-5f, seed, 7, 429496730u, 1.1f, 0); }));
  rep("ln2<0> (gb hoisted, drop)", timeit([&] { ln2<0><<<M / 4, 256>>>(a, b, g, be, c, d, mean, rstd, M, D, 1e-5f, seed, 7, 429496730u, 1.1f); }));
  rep("ln2<1> (no seed/drop)", timeit([&] { ln2<1><<<M / 4, 256>>>(a, b, g, be, c, d, mean, rstd, M, D, 1e-5f, seed, 7, 0u, 1.f); }));
  rep("ln2<2> (1-pass stats)", timeit([&] { ln2<2><<<M / 4, 256>>>(a, b, g, be, c, d, mean, rstd, M, D, 1e-5f, seed, 7, 0u, 1.f); }));
  rep("ln_nogb", timeit([&] { ln_nogb<<<M / 4, 256>>>(a, b, c, d, M, D); }));
  CK(hipDeviceSynchronize());
  return 0;
}
