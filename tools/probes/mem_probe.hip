// Bandwidth probe for row-wise memory-bound kernels at the transformer's shapes (8192 x 512 bf16):
// how fast can 2-in/2-out row kernels go with one row per wave vs several rows per wave, and
// what the current LayerNorm kernels reach.  Build: hipcc -O3 --offload-arch=gfx950 -I csrc/include
#include "../../csrc/kernels/layernorm.hip"
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void copy_row(const u16x8_t* __restrict__ a, const u16x8_t* __restrict__ b,
                                                u16x8_t* __restrict__ c, u16x8_t* __restrict__ d, int rows, int vpr) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= rows) return;
  for (int v = lane; v < vpr; v += 64) {
    const size_t i = (size_t)row * vpr + v;
    u16x8_t x = a[i], y = b[i];
    c[i] = x + y;
    d[i] = x;
  }
}

template <int RPW>
__global__ __launch_bounds__(256) void copy_rows(const u16x8_t* __restrict__ a, const u16x8_t* __restrict__ b,
                                                 u16x8_t* __restrict__ c, u16x8_t* __restrict__ d, int rows, int vpr) {
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  u16x8_t x[RPW], y[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const size_t i = (size_t)(row0 + r) * vpr + lane;
    if (row0 + r < rows) { x[r] = a[i]; y[r] = b[i]; }
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const size_t i = (size_t)(row0 + r) * vpr + lane;
    if (row0 + r < rows) { c[i] = x[r] + y[r]; d[i] = x[r]; }
  }
}

__global__ __launch_bounds__(256) void copy_gs(const u16x8_t* __restrict__ a, const u16x8_t* __restrict__ b,
                                               u16x8_t* __restrict__ c, u16x8_t* __restrict__ d, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    u16x8_t x = a[i], y = b[i];
    c[i] = x + y;
    d[i] = x;
  }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

template <class F>
float timeit(F f, int it = 50) {
  for (int i = 0; i < 5; ++i) f();
  hipEvent_t s, e;
  hipEventCreate(&s); hipEventCreate(&e);
  hipEventRecord(s);
  for (int i = 0; i < it; ++i) f();
  hipEventRecord(e);
  hipEventSynchronize(e);
  float ms; hipEventElapsedTime(&ms, s, e);
  return ms * 1000.f / it;
}

int main() {
  const int M = 8192, D = 512, vpr = D / 8;
  const size_t n = (size_t)M * D;
  unsigned short *a, *b, *c, *d;
  float *g, *be, *mean, *rstd, *pg, *pb;
  unsigned int* seed;
  CK(hipMalloc(&a, n * 2)); CK(hipMalloc(&b, n * 2)); CK(hipMalloc(&c, n * 2)); CK(hipMalloc(&d, n * 2));
  CK(hipMalloc(&g, D * 4)); CK(hipMalloc(&be, D * 4)); CK(hipMalloc(&mean, M * 4)); CK(hipMalloc(&rstd, M * 4));
  CK(hipMalloc(&pg, 2048 * D * 4)); CK(hipMalloc(&pb, 2048 * D * 4)); CK(hipMalloc(&seed, 4));
  CK(hipMemset(a, 0, n * 2)); CK(hipMemset(b, 0, n * 2)); CK(hipMemset(g, 0, D * 4)); CK(hipMemset(be, 0, D * 4));
  CK(hipMemset(seed, 0, 4));
  const double bytes = 4.0 * n * 2;
  auto rep = [&](const char* name, float us) { printf("%-28s %8.2f us  %7.0f GB/s\n", name, us, bytes / us / 1e3); };
  rep("copy_row (1 row/wave)", timeit([&] { copy_row<<<M / 4, 256>>>((u16x8_t*)a, (u16x8_t*)b, (u16x8_t*)c, (u16x8_t*)d, M, vpr); }));
  rep("copy_rows<2>", timeit([&] { copy_rows<2><<<M / 8, 256>>>((u16x8_t*)a, (u16x8_t*)b, (u16x8_t*)c, (u16x8_t*)d, M, vpr); }));
  rep("copy_rows<4>", timeit([&] { copy_rows<4><<<M / 16, 256>>>((u16x8_t*)a, (u16x8_t*)b, (u16x8_t*)c, (u16x8_t*)d, M, vpr); }));
  rep("copy_rows<8>", timeit([&] { copy_rows<8><<<M / 32, 256>>>((u16x8_t*)a, (u16x8_t*)b, (u16x8_t*)c, (u16x8_t*)d, M, vpr); }));
  for (int grid : {256, 512, 1024, 2048, 4096})  {
    char nm[64]; snprintf(nm, 64, "copy_gs grid %d", grid);
    rep(nm, timeit([&] { copy_gs<<<grid, 256>>>((u16x8_t*)a, (u16x8_t*)b, (u16x8_t*)c, (u16x8_t*)d, n / 8); }));
  }
  rep("ln_fwd (drop+resid)", timeit([&] { smi_ln_fwd(a, b, g, be, c, d, mean, rstd, M, D, 1e-5f, seed, 7, 429496730u, 1.1f, 0); }));
  rep("ln_fwd (no drop)", timeit([&] { smi_ln_fwd(a, b, g, be, c, d, mean, rstd, M, D, 1e-5f, seed, 7, 0u, 1.f, 0); }));
  rep("ln_bwd (drop)", timeit([&] { smi_ln_bwd(a, b, mean, rstd, g, c, d, nullptr, pg, pb, 2048, g, be, 1, M, D, seed, 7, 429496730u, 1.1f, 0); }));
  rep("ln_bwd (no drop)", timeit([&] { smi_ln_bwd(a, b, mean, rstd, g, c, d, nullptr, pg, pb, 2048, g, be, 1, M, D, seed, 7, 0u, 1.f, 0); }));
  {
    rep("ln_bwd_kernel<1,1> only", timeit([&] { hipLaunchKernelGGL((ln_bwd_kernel<1, 1>), dim3(M / 4), dim3(256), 0, 0, a, b, mean, rstd, g, c, d, nullptr, pg, pb, M, D, seed, 7, 429496730u, 1.1f); }));
    rep("ln_bwd_kernel<1,2> only", timeit([&] { hipLaunchKernelGGL((ln_bwd_kernel<1, 2>), dim3(M / 8), dim3(256), 0, 0, a, b, mean, rstd, g, c, d, nullptr, pg, pb, M, D, seed, 7, 429496730u, 1.1f); }));
    rep("ln_bwd_kernel<1,4> only", timeit([&] { hipLaunchKernelGGL((ln_bwd_kernel<1, 4>), dim3(M / 16), dim3(256), 0, 0, a, b, mean, rstd, g, c, d, nullptr, pg, pb, M, D, seed, 7, 429496730u, 1.1f); }));
    for (int nb : {512, 1024, 2048})
      for (int gy : {1, 4, 8, 16}) {
        char nm2[80]; snprintf(nm2, 80, "colsum2 nb=%d groups %d", nb, gy);
        rep(nm2, timeit([&] { hipLaunchKernelGGL(colsum2_kernel, dim3(D / 64, gy), dim3(256), 0, 0, pg, pb, nb, D, g, be, 1); }));
      }
  }
  CK(hipDeviceSynchronize());
  return 0;
}
