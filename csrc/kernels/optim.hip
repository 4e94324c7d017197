// Fused optimizers over flat fp32 parameter / gradient / state buffers.  One launch updates
// every parameter of the model (the flat layout replaces multi-tensor-apply), writes the bf16
// compute copy in the same pass and optionally zeroes the gradient for the next step.
//
// Reference: torch.optim.Adam(lr=1e-3) (pytorch_machine_translator.py:129,
// distributed_lstm.py:141) and torch.optim.SGD(lr) without momentum
// (distributed_multilayer_perceptron.py:111, distributed_cnn.py:138).  Adam follows torch's
// formula: m,v EMA; bias corrections 1-b^t; eps added after sqrt(v_hat).  The step counter and
// lr live on the device so a captured HIP graph replays correct updates every step.
//
// The step counter advances inside the update kernel (no separate increment launch): every
// block computes t = step[0] + 1 on entry, and the last block to finish (atomic ticket on the
// `done` word) stores t and re-arms the ticket — all other blocks have read step[0] by then.
#include <stdlib.h>

#include "smi_common.h"
#include "smi_split3.h"

__global__ void step_inc_kernel(float* step) { step[0] += 1.f; }
// dropout step seed (sparkmi/ops/rng.py DropoutRNG.advance): one lane, captured in step graphs
__global__ void seed_inc_kernel(int* seed) { seed[0] += 1; }

// No __threadfence: nothing but the counter itself is published (the next launch sees it at the
// kernel boundary), and an agent-scope release on gfx950 writes back L2 — once per block that
// doubled the 47M-parameter Adam (0.27 -> 0.55 ms).  Every block has consumed its step[0] read
// (bias corrections) before its ticket, so the last block's store cannot be seen early.
// seed (optional): the model's dropout step seed (sparkmi/ops/rng.py DropoutRNG), advanced here
// for the NEXT step instead of by a separate one-lane launch at the start of every step (the
// training-step runner binds it: sparkmi/train/runner.py); no kernel of this launch reads it.
__device__ __forceinline__ void finish_step(float* step, unsigned* done, float t, int* seed) {
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(done, 1u) == gridDim.x - 1) {
    step[0] = t;
    if (seed) seed[0] += 1;
    done[0] = 0u;
  }
}

// Split planes of the updated weights (the operand format of the fp32 GEMM,
// csrc/include/smi_gemm_sp.h): hi / mid / lo at pl, pl + ps, pl + 2 ps.
__device__ __forceinline__ void store_planes4(unsigned short* __restrict__ pl, long ps, long i4, const float* pa) {
  uint32_t h0, m0, l0, h1, m1, l1;
  split3_pair(pa[0], pa[1], h0, m0, l0);
  split3_pair(pa[2], pa[3], h1, m1, l1);
  ((uint2*)pl)[i4] = make_uint2(h0, h1);
  ((uint2*)(pl + ps))[i4] = make_uint2(m0, m1);
  ((uint2*)(pl + 2 * ps))[i4] = make_uint2(l0, l1);
}
__device__ __forceinline__ void store_planes1(unsigned short* __restrict__ pl, long ps, long i, float x) {
  const unsigned short hh = f2bf(x);
  const float r = x - bf2f(hh);
  const unsigned short mm = f2bf(r);
  pl[i] = hh;
  pl[ps + i] = mm;
  pl[2 * ps + i] = f2bf(r - bf2f(mm));
}

template <int NT>
__global__ __launch_bounds__(NT) void adam_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                                   float* __restrict__ v, unsigned short* __restrict__ pbf, long n,
                                                   const float* __restrict__ lr_p, float* __restrict__ step_p,
                                                   unsigned* __restrict__ done, float b1, float b2, float eps, float wd,
                                                   float gscale, int adamw, int zero_grad, unsigned short* __restrict__ pl,
                                                   long ps, int* __restrict__ seed) {
  const float t = step_p[0] + 1.f;
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
    if (pl) store_planes4(pl, ps, i, pa);
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
      if (pl) store_planes1(pl, ps, i, p[i]);
    }
  }
  finish_step(step_p, done, t, seed);
}

// Adam over several disjoint ranges in ONE launch with ONE step advance: the ZeRO-1 update of
// a data-parallel rank, which owns one piece of every gradient bucket (sparkmi/parallel/ddp.py)
// and keeps the moments of its pieces only (compact m / v); and a step's update in parts (the
// parameters already final while the backward still runs, then the rest: sparkmi/optim/adam.py
// step_ranges).  Range e owns blocks [blk0[e], blk0[e+1]); float4 body (every piece is a multiple
// of 4 floats, 16-B aligned).  advance = 0: an early part — it reads the step counter like every
// part (same t, same bias corrections) but neither advances it nor takes a ticket.
#define ADAM_MULTI_MAX 64
struct AdamMulti {
  float* p[ADAM_MULTI_MAX]; float* g[ADAM_MULTI_MAX]; float* m[ADAM_MULTI_MAX]; float* v[ADAM_MULTI_MAX];
  unsigned short* pbf[ADAM_MULTI_MAX]; unsigned short* pl[ADAM_MULTI_MAX]; long n[ADAM_MULTI_MAX];
  int blk0[ADAM_MULTI_MAX + 1]; int count; long ps;
};
__global__ __launch_bounds__(256) void adam_multi_kernel(AdamMulti a, const float* __restrict__ lr_p,
                                                         float* __restrict__ step_p, unsigned* __restrict__ done, float b1,
                                                         float b2, float eps, float wd, float gscale, int adamw,
                                                         int zero_grad, int* __restrict__ seed, int advance) {
  const float t = step_p[0] + 1.f;
  const float lr = lr_p[0];
  const float bc1 = 1.f - powf(b1, t), bc2 = 1.f - powf(b2, t);
  const float step_size = lr / bc1;
  const float rbc2 = 1.f / sqrtf(bc2);
  int e = 0;
  while (e + 1 < a.count && (int)blockIdx.x >= a.blk0[e + 1]) ++e;  // wave-uniform scan
  const long lb = blockIdx.x - a.blk0[e], nb = a.blk0[e + 1] - a.blk0[e];
  float* p = a.p[e]; float* g = a.g[e]; float* m = a.m[e]; float* v = a.v[e]; unsigned short* pbf = a.pbf[e];
  unsigned short* pl = a.pl[e];
  const long n4 = a.n[e] / 4;
  for (long i = lb * blockDim.x + threadIdx.x; i < n4; i += nb * blockDim.x) {
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
    if (pl) store_planes4(pl, a.ps, i, pa);
  }
  if (advance) finish_step(step_p, done, t, seed);
}

// p -= lr * (g*gscale + wd*p) with optional (heavy-ball, torch-style) momentum buffer
__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ buf,
                                                  unsigned short* __restrict__ pbf, long n, const float* __restrict__ lr_p,
                                                  float* __restrict__ step_p, unsigned* __restrict__ done, float momentum,
                                                  float dampening, float wd, int nesterov, float gscale, int zero_grad,
                                                  unsigned short* __restrict__ pl, long ps, int* __restrict__ seed) {
  const float lr = lr_p[0];
  const float t = step_p[0] + 1.f;
  const bool first = t <= 1.f;
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
    if (pl) store_planes1(pl, ps, i, p[i]);
  }
  finish_step(step_p, done, t, seed);
}

static inline unsigned grid_for(long n) {
  long b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (unsigned)b;
}

extern "C" int smi_seed_inc(int* seed, hipStream_t st) {
  hipLaunchKernelGGL(seed_inc_kernel, dim3(1), dim3(1), 0, st, seed);
  return (int)hipGetLastError();
}

extern "C" int smi_step_inc(float* step, hipStream_t st) {
  hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, st, step);
  SMI_CHECK_LAUNCH();
}

// Adam launch shape: 1024-thread blocks, <= 512 of them (default) / 256-thread blocks, <= 4096
// (SMI_ADAM_WIDE=0)
static int g_adam_wide = -1;
extern "C" int smi_adam_wide(int set) {
  if (set == 0 || set == 1) g_adam_wide = set;
  if (g_adam_wide < 0) {
    g_adam_wide = 1;
  }
  return g_adam_wide;
}
static int adam_wide() { return smi_adam_wide(-1); }

extern "C" int smi_adam(float* p, float* g, float* m, float* v, void* pbf, long n, const float* lr, float* step,
                        unsigned* done, float b1, float b2, float eps, float wd, float gscale, int adamw, int zero_grad,
                        void* pl, long ps, int* seed, hipStream_t st) {
  if (pl && (((uintptr_t)pl & 7) || ps % 4 || ps < n)) return -1;
  if (adam_wide()) {
    // 1024-thread blocks, at most two per CU: every block takes one ticket on the shared `done`
    // word at its end, and same-address atomics serialise at one L2 channel (~10 ns each) — the
    // 3,000-block launch of a 3M-parameter model spent most of its 40 us in that ticket queue
    long b = (n / 4 + 1023) / 1024;
    if (b > 512) b = 512;
    if (b < 1) b = 1;
    hipLaunchKernelGGL(adam_kernel<1024>, dim3((unsigned)b), dim3(1024), 0, st, p, g, m, v, (unsigned short*)pbf, n,
                       lr, step, done, b1, b2, eps, wd, gscale, adamw, zero_grad, (unsigned short*)pl, ps, seed);
  } else {
    hipLaunchKernelGGL(adam_kernel<256>, dim3(grid_for(n / 4 + 1)), dim3(256), 0, st, p, g, m, v, (unsigned short*)pbf,
                       n, lr, step, done, b1, b2, eps, wd, gscale, adamw, zero_grad, (unsigned short*)pl, ps, seed);
  }
  SMI_CHECK_LAUNCH();
}

extern "C" int smi_adam_multi(float* const* p, float* const* g, float* const* m, float* const* v, void* const* pbf,
                              const long* n, int count, const float* lr, float* step, unsigned* done, float b1, float b2,
                              float eps, float wd, float gscale, int adamw, int zero_grad, void* const* pl, long ps,
                              int* seed, int advance, hipStream_t st) {
  if (count < 1 || count > ADAM_MULTI_MAX) return -1;
  AdamMulti a{};
  long total4 = 0;
  for (int i = 0; i < count; ++i) {
    if (n[i] % 4 || ((((uintptr_t)p[i]) | ((uintptr_t)g[i]) | ((uintptr_t)m[i]) | ((uintptr_t)v[i])) & 15)) return -1;
    total4 += n[i] / 4;
  }
  int tot = 0;
  for (int i = 0; i < count; ++i) {
    a.p[i] = p[i]; a.g[i] = g[i]; a.m[i] = m[i]; a.v[i] = v[i]; a.pbf[i] = (unsigned short*)pbf[i]; a.n[i] = n[i];
    a.pl[i] = pl ? (unsigned short*)pl[i] : nullptr;
    // blocks proportional to the range's share of a <= 4096-block launch
    long b = total4 ? (long)((double)(n[i] / 4) / (double)total4 * 4096.0) : 1;
    if (b > (n[i] / 4 + 255) / 256) b = (n[i] / 4 + 255) / 256;
    if (b < 1) b = 1;
    a.blk0[i] = tot;
    tot += (int)b;
  }
  a.blk0[count] = tot;
  a.count = count;
  a.ps = ps;
  hipLaunchKernelGGL(adam_multi_kernel, dim3((unsigned)tot), dim3(256), 0, st, a, lr, step, done, b1, b2, eps, wd, gscale,
                     adamw, zero_grad, advance ? seed : nullptr, advance);
  SMI_CHECK_LAUNCH();
}

extern "C" int smi_sgd(float* p, float* g, float* buf, void* pbf, long n, const float* lr, float* step, unsigned* done,
                       float momentum, float dampening, float wd, int nesterov, float gscale, int zero_grad, void* pl,
                       long ps, int* seed, hipStream_t st) {
  if (pl && ps < n) return -1;
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(n)), dim3(256), 0, st, p, g, buf, (unsigned short*)pbf, n, lr, step,
                     done, momentum, dampening, wd, nesterov, gscale, zero_grad, (unsigned short*)pl, ps, seed);
  SMI_CHECK_LAUNCH();
}

// Several small device-to-device copies in ONE launch (the per-step static-input refresh of a
// replayed HIP graph: one blit launch per input cost ~5 us each).  blockIdx.y = buffer.
struct MultiCopyArgs { const unsigned char* src[8]; unsigned char* dst[8]; long bytes[8]; };
__global__ __launch_bounds__(256) void multi_copy_kernel(MultiCopyArgs a) {
  const int b = blockIdx.y;
  const long n = a.bytes[b];
  const unsigned char* s = a.src[b];
  unsigned char* d = a.dst[b];
  const long stride = (long)gridDim.x * blockDim.x;
  long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if ((((unsigned long)s | (unsigned long)d) & 15) == 0) {
    const long n16 = n >> 4;
    for (long i = i0; i < n16; i += stride) ((uint4*)d)[i] = ((const uint4*)s)[i];
    for (long i = (n16 << 4) + i0; i < n; i += stride) d[i] = s[i];
  } else {
    for (long i = i0; i < n; i += stride) d[i] = s[i];
  }
}

extern "C" int smi_multi_copy(void* const* dst, const void* const* src, const long* bytes, int count, hipStream_t st) {
  if (count < 1 || count > 8) return -1;
  MultiCopyArgs a{};
  long mx = 0;
  for (int i = 0; i < count; ++i) {
    a.dst[i] = (unsigned char*)dst[i]; a.src[i] = (const unsigned char*)src[i]; a.bytes[i] = bytes[i];
    if (bytes[i] > mx) mx = bytes[i];
  }
  long blocks = (mx / 16 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(multi_copy_kernel, dim3((unsigned)blocks, (unsigned)count), dim3(256), 0, st, a);
  SMI_CHECK_LAUNCH();
}
