// Device-resident L-BFGS (the solver of MultilayerPerceptronClassifier, mllib_multilayer_perceptron
// _classifier.py:32-35; Spark runs Breeze's LBFGS on the driver over treeAggregate'd gradients).
// Here the correction pairs (S, Y: [m, n] ring buffers), rho [m] and the ring state {head, count}
// live in HBM, and the two-loop recursion and the pair update are one workgroup-wide kernel each:
// the host only sees the line-search scalars (f, g.d).  One workgroup of 1024 threads (16 waves)
// streams the vectors; every dot product is a double-precision block reduction (wave shuffles,
// then 16 partials through LDS), so the recursion's 2m+3 dependent dots cost one barrier pair each
// instead of a kernel launch and a host round trip each.  MLlib models are small (n = 50 for the
// reference's [4,5,4,3] network), so one workgroup is the right size: the work is latency-bound.
#include <hip/hip_runtime.h>

#define LB_THREADS 1024
#define LB_MAX_M 64

__device__ __forceinline__ double lb_block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();  // red[] may still be read by the previous reduction
  if (l == 0) red[w] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int i = 0; i < LB_THREADS / 64; ++i) t += red[i];
  return t;
}

__device__ __forceinline__ double lb_dot(const float* a, const float* b, long n, double* red) {
  double s = 0.0;
  for (long i = threadIdx.x; i < n; i += LB_THREADS) s += (double)a[i] * (double)b[i];
  return lb_block_sum(s, red);
}

// d = -H g (two-loop recursion over the stored pairs, newest first),
// out = {g.d, |g|_1, |g|_2^2, pairs used}.
// reset != 0 drops the memory (d = -g).
__global__ __launch_bounds__(LB_THREADS) void lbfgs_direction_kernel(const float* __restrict__ S,
                                                                     const float* __restrict__ Y,
                                                                     const float* __restrict__ rho, int* st, int m,
                                                                     long n, const float* __restrict__ g,
                                                                     float* __restrict__ d, float* __restrict__ out,
                                                                     int reset) {
  __shared__ double red[LB_THREADS / 64];
  __shared__ double alpha[LB_MAX_M];
  const int head = st[0];
  const int count = reset ? 0 : st[1];
  for (long i = threadIdx.x; i < n; i += LB_THREADS) d[i] = g[i];
  for (int j = 0; j < count; ++j) {
    const int k = (head - 1 - j + 2 * m) % m;
    const float* s = S + (long)k * n;
    const float* y = Y + (long)k * n;
    const double a = (double)rho[k] * lb_dot(s, d, n, red);
    if (threadIdx.x == 0) alpha[j] = a;
    for (long i = threadIdx.x; i < n; i += LB_THREADS) d[i] = (float)((double)d[i] - a * (double)y[i]);
  }
  double gamma = 1.0;
  if (count > 0) {
    const int k = (head - 1 + m) % m;
    const double yy = lb_dot(Y + (long)k * n, Y + (long)k * n, n, red);
    gamma = (1.0 / (double)rho[k]) / (yy > 0.0 ? yy : 1.0);  // s.y / y.y
  }
  for (long i = threadIdx.x; i < n; i += LB_THREADS) d[i] = (float)(gamma * (double)d[i]);
  __syncthreads();  // alpha[] written by thread 0 above
  for (int j = count - 1; j >= 0; --j) {
    const int k = (head - 1 - j + 2 * m) % m;
    const float* s = S + (long)k * n;
    const float* y = Y + (long)k * n;
    const double b = (double)rho[k] * lb_dot(y, d, n, red);
    const double c = alpha[j] - b;
    for (long i = threadIdx.x; i < n; i += LB_THREADS) d[i] = (float)((double)d[i] + c * (double)s[i]);
  }
  double gd = 0.0, g1 = 0.0, g2 = 0.0;
  for (long i = threadIdx.x; i < n; i += LB_THREADS) {
    const double gi = g[i];
    const double di = -(double)d[i];
    d[i] = (float)di;
    gd += gi * di;
    g1 += fabs(gi);
    g2 += gi * gi;
  }
  gd = lb_block_sum(gd, red);
  g1 = lb_block_sum(g1, red);
  g2 = lb_block_sum(g2, red);
  if (threadIdx.x == 0) {
    out[0] = (float)gd;
    out[1] = (float)g1;
    out[2] = (float)g2;
    out[3] = (float)count;
    if (reset) st[1] = 0;
  }
}

// Accepted step t along d: x += t d; the pair s = t d, y = g_new - g_old is stored (and the ring
// advanced) when s.y > eps (curvature condition), otherwise the memory is left as it was.
__global__ __launch_bounds__(LB_THREADS) void lbfgs_update_kernel(float* __restrict__ S, float* __restrict__ Y,
                                                                  float* __restrict__ rho, int* st, int m, long n,
                                                                  const float* __restrict__ d, float t,
                                                                  const float* __restrict__ g_new,
                                                                  const float* __restrict__ g_old,
                                                                  float* __restrict__ x, float eps) {
  __shared__ double red[LB_THREADS / 64];
  double sy = 0.0;
  for (long i = threadIdx.x; i < n; i += LB_THREADS) {
    const double s = (double)t * (double)d[i];
    sy += s * ((double)g_new[i] - (double)g_old[i]);
  }
  sy = lb_block_sum(sy, red);
  const int head = st[0], count = st[1];
  if (sy > (double)eps) {
    float* s_out = S + (long)head * n;
    float* y_out = Y + (long)head * n;
    for (long i = threadIdx.x; i < n; i += LB_THREADS) {
      s_out[i] = t * d[i];
      y_out[i] = g_new[i] - g_old[i];
    }
  }
  for (long i = threadIdx.x; i < n; i += LB_THREADS) x[i] += t * d[i];
  __syncthreads();  // every thread read st[] before thread 0 advances it
  if (threadIdx.x == 0 && sy > (double)eps) {
    rho[head] = (float)(1.0 / sy);
    st[0] = (head + 1) % m;
    st[1] = count < m ? count + 1 : m;
  }
}

extern "C" int smi_lbfgs_direction(const float* S, const float* Y, const float* rho, int* st, int m, long n,
                                   const float* g, float* d, float* out, int reset, hipStream_t stream) {
  if (m < 1 || m > LB_MAX_M || n < 1) return -1;
  hipLaunchKernelGGL(lbfgs_direction_kernel, dim3(1), dim3(LB_THREADS), 0, stream, S, Y, rho, st, m, n, g, d, out,
                     reset);
  return (int)hipGetLastError();
}

extern "C" int smi_lbfgs_update(float* S, float* Y, float* rho, int* st, int m, long n, const float* d, float t,
                                const float* g_new, const float* g_old, float* x, float eps, hipStream_t stream) {
  if (m < 1 || m > LB_MAX_M || n < 1) return -1;
  hipLaunchKernelGGL(lbfgs_update_kernel, dim3(1), dim3(LB_THREADS), 0, stream, S, Y, rho, st, m, n, d, t, g_new,
                     g_old, x, eps);
  return (int)hipGetLastError();
}
