// Fused optimizers over flat fp32 parameter / gradient / state buffers.  One launch updates
// every parameter of the model (the flat layout replaces multi-tensor-apply), writes the bf16
// compute copy in the same pass and optionally zeroes the gradient for the next step.
//
// Reference: torch.optim.Adam(lr=1e-3) (pytorch_machine_translator.py:129,
// distributed_lstm.py:141) and torch.optim.SGD(lr) without momentum
// (distributed_multilayer_perceptron.py:111, distributed_cnn.py:138).  Adam follows torch's
// formula: m,v EMA; bias corrections 1-b^t; eps added after sqrt(v_hat).  The step counter and
// lr live on the device so a captured HIP graph replays correct updates every step.
#include "smi_common.h"

__global__ void step_inc_kernel(float* step) { step[0] += 1.f; }

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                                   float* __restrict__ v, unsigned short* __restrict__ pbf, long n,
                                                   const float* __restrict__ lr_p, const float* __restrict__ step_p,
                                                   float b1, float b2, float eps, float wd, float gscale, int adamw,
                                                   int zero_grad) {
  const float t = step_p[0];
  const float lr = lr_p[0];
  const float bc1 = 1.f - powf(b1, t), bc2 = 1.f - powf(b2, t);
  const float step_size = lr / bc1;
  const float rbc2 = 1.f / sqrtf(bc2);
  const long n4 = n / 4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 pp = ((float4*)p)[i], gg = ((float4*)g)[i], mm = ((float4*)m)[i], vv = ((float4*)v)[i];
    float* pa = &pp.x; float* ga = &gg.x; float* ma = &mm.x; float* va = &vv.x;
    unsigned short ob[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gr = ga[j] * gscale;
      if (wd != 0.f) {
        if (adamw) pa[j] *= (1.f - lr * wd);
        else gr += wd * pa[j];
      }
      ma[j] = b1 * ma[j] + (1.f - b1) * gr;
      va[j] = b2 * va[j] + (1.f - b2) * gr * gr;
      const float denom = sqrtf(va[j]) * rbc2 + eps;
      pa[j] -= step_size * ma[j] / denom;
      ob[j] = f2bf(pa[j]);
    }
    ((float4*)p)[i] = pp; ((float4*)m)[i] = mm; ((float4*)v)[i] = vv;
    if (zero_grad) ((float4*)g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (pbf) {
      uint2 w; w.x = ob[0] | ((unsigned)ob[1] << 16); w.y = ob[2] | ((unsigned)ob[3] << 16);
      ((uint2*)pbf)[i] = w;
    }
  }
  // tail
  if (blockIdx.x == 0) {
    for (long i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) {
      float gr = g[i] * gscale;
      if (wd != 0.f) { if (adamw) p[i] *= (1.f - lr * wd); else gr += wd * p[i]; }
      m[i] = b1 * m[i] + (1.f - b1) * gr;
      v[i] = b2 * v[i] + (1.f - b2) * gr * gr;
      p[i] -= step_size * m[i] / (sqrtf(v[i]) * rbc2 + eps);
      if (zero_grad) g[i] = 0.f;
      if (pbf) pbf[i] = f2bf(p[i]);
    }
  }
}

// p -= lr * (g*gscale + wd*p) with optional (heavy-ball, torch-style) momentum buffer
__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ buf,
                                                  unsigned short* __restrict__ pbf, long n, const float* __restrict__ lr_p,
                                                  const float* __restrict__ step_p, float momentum, float dampening,
                                                  float wd, int nesterov, float gscale, int zero_grad) {
  const float lr = lr_p[0];
  const bool first = step_p[0] <= 1.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float d = g[i] * gscale;
    if (wd != 0.f) d += wd * p[i];
    if (momentum != 0.f) {
      const float b = first ? d : momentum * buf[i] + (1.f - dampening) * d;
      buf[i] = b;
      d = nesterov ? d + momentum * b : b;
    }
    p[i] -= lr * d;
    if (zero_grad) g[i] = 0.f;
    if (pbf) pbf[i] = f2bf(p[i]);
  }
}

static inline unsigned grid_for(long n) {
  long b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (unsigned)b;
}

extern "C" int smi_step_inc(float* step, hipStream_t st) {
  hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, st, step);
  SMI_CHECK_LAUNCH();
}

extern "C" int smi_adam(float* p, float* g, float* m, float* v, void* pbf, long n, const float* lr, const float* step,
                        float b1, float b2, float eps, float wd, float gscale, int adamw, int zero_grad, hipStream_t st) {
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n / 4 + 1)), dim3(256), 0, st, p, g, m, v, (unsigned short*)pbf, n, lr,
                     step, b1, b2, eps, wd, gscale, adamw, zero_grad);
  SMI_CHECK_LAUNCH();
}

extern "C" int smi_sgd(float* p, float* g, float* buf, void* pbf, long n, const float* lr, const float* step,
                       float momentum, float dampening, float wd, int nesterov, float gscale, int zero_grad,
                       hipStream_t st) {
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(n)), dim3(256), 0, st, p, g, buf, (unsigned short*)pbf, n, lr, step,
                     momentum, dampening, wd, nesterov, gscale, zero_grad);
  SMI_CHECK_LAUNCH();
}
