// Fused small-MLP forward/backward: affine -> sigmoid|relu hidden layers -> affine logits ->
// softmax cross-entropy, for the reference's 4-5-4-3 sigmoid MLP (distributed_multilayer_
// perceptron.py:44-53, pytorch_multilayer_perceptron.py:33-42) and Spark MLlib's
// MultilayerPerceptronClassifier topology (AffineLayer + Sigmoid, SoftmaxLayerWithCrossEntropy;
// SURVEY App. A.1), which is the same model.
//
// The whole network is a few dozen parameters, so the GPU cost is launch latency, not FLOPs:
// ONE kernel does a whole training step — forward, softmax-CE, backward and the SGD update
// (mode 2; the reference's optimizer.step(), distributed_multilayer_perceptron.py:108-111) — or
// forward + loss (mode 0) or forward + backward into gradient buffers (mode 1, autograd and
// data-parallel paths).  Each wave64 handles 64 rows (one row per lane); per-lane activations and
// pre-activation gradients live in LDS rows with an odd pitch (an even multiple-of-32 pitch put
// all 64 lanes on one bank: 74 us per backward at batch 30); each weight-gradient entry is summed
// over the 64 rows by one lane in row order.  Across blocks nothing is atomic but a ticket: every
// block publishes its partial gradient + loss, and the last block to arrive sums them in block
// order, so gradients are bit-reproducible run to run.  Row weights implement MLlib's per-block
// loss averaging (or 1/n for the torch-style mean).
#include "smi_common.h"

#include "smi_mlp.h"

__device__ __forceinline__ float mlp_act(float v, int act) {
  return act == 1 ? fmaxf(v, 0.f) : 1.f / (1.f + __expf(-v));
}

// forward one row; activations of every layer stored in a (lane-private) LDS slab; Wp / bp: the
// layer parameters (an LDS copy when they fit, else the global tensors)
__device__ __forceinline__ float mlp_forward_row(const MLPArgs& a, int row, float* act_s, const float* const* Wp,
                                                 const float* const* bp) {
  int off = 0;
  const int d0 = a.dims[0];
  for (int i = 0; i < d0; ++i) act_s[i] = a.x[(long)row * d0 + i];
  for (int l = 0; l < a.nlayers; ++l) {
    const int din = a.dims[l], dout = a.dims[l + 1];
    const float* in = act_s + off;
    float* out = act_s + off + din;
    const bool last = l == a.nlayers - 1;
    for (int o = 0; o < dout; ++o) {
      float s = bp[l][o];
      const float* w = Wp[l] + o * din;
      for (int i = 0; i < din; ++i) s += w[i] * in[i];
      out[o] = last ? s : mlp_act(s, a.act);
    }
    off += din;
  }
  // softmax CE on the last layer (offset `off`)
  const int C = a.dims[a.nlayers];
  const float* z = act_s + off;
  float m = z[0];
  for (int c = 1; c < C; ++c) m = fmaxf(m, z[c]);
  float se = 0.f;
  for (int c = 0; c < C; ++c) se += __expf(z[c] - m);
  const float lse = m + __logf(se);
  const long long lab = a.y ? a.y[row] : 0;
  return lse - z[lab];
}

#define MLP_ACT_LD (MLP_ACT_STRIDE + 1)        // odd LDS pitch: lane-private rows on distinct banks
#define MLP_DEL_LD (MLP_MAXW * MLP_MAXL + 1)
#define MLP_MAXT 8192                          // parameters (weights + biases)
#define MLP_WLDS 2048                          // parameters staged in LDS (fits beside the slabs)

__device__ __forceinline__ int mlp_total(const MLPArgs& a) {
  int t = 0;
  for (int l = 0; l < a.nlayers; ++l) t += a.dims[l + 1] * (a.dims[l] + 1);
  return t;
}

// Last step of every mode: the block-order sum of the per-block partials (entries 0..T-1 the
// gradient, entry T the loss) — identical bits for any run with the same grid, no float atomics
// — then the loss / gradient / SGD-updated parameters are written.  With one block the partials
// are its own LDS values.
__device__ void mlp_finalize(const MLPArgs& a, int mode, int T, const float* gacc, float lsum) {
  const int lane = threadIdx.x;
  const bool multi = gridDim.x > 1;
  const int W = T + 1;
  if (mode == 0) {
    float s = lsum;
    if (multi) {
      s = 0.f;
      for (int i = lane; i < (int)gridDim.x; i += 64)
        s += __hip_atomic_load(a.ws + (long)i * W + T, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s = wave_sum(s);
    }
    if (lane == 0 && a.loss) a.loss[0] = s;
    return;
  }
  // loss: lane 0 sums the block losses in block order
  if (lane == 0 && a.loss) {
    float s = lsum;
    if (multi) {
      s = 0.f;
      for (int i = 0; i < (int)gridDim.x; ++i)
        s += __hip_atomic_load(a.ws + (long)i * W + T, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    a.loss[0] = s;
  }
  const float lr = mode == 2 ? a.lr[0] * a.gscale : 0.f;
  for (int l = 0, base = 0; l < a.nlayers; ++l) {
    const int din = a.dims[l], dout = a.dims[l + 1], nl = dout * (din + 1);
    for (int r = lane; r < nl; r += 64) {
      float g = 0.f;
      if (multi) {
        for (int i = 0; i < (int)gridDim.x; ++i)
          g += __hip_atomic_load(a.ws + (long)i * W + base + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        g = gacc[base + r];
      }
      const bool bias = r >= dout * din;
      if (mode == 2) {
        float* p = bias ? const_cast<float*>(a.b[l]) + (r - dout * din) : const_cast<float*>(a.W[l]) + r;
        *p -= lr * g;
      } else {
        float* q = bias ? a.gb[l] + (r - dout * din) : a.gW[l] + r;
        *q = a.accumulate ? *q + g : g;
      }
    }
    base += nl;
  }
  if (mode == 2 && lane == 0 && a.step) a.step[0] += 1.f;
}

// mode 0: forward + loss (+ logits); 1: + backward, gradients to gW/gb; 2: + SGD update of W/b.
// One wave64 per block, one row per lane; the grid-level sums are deterministic (block order).
__global__ __launch_bounds__(64) void mlp_kernel(MLPArgs a, int mode) {
  __shared__ float acts[64 * MLP_ACT_LD];  // per row: layer inputs (dims[0..L-1]) + logits
  __shared__ float dls[64 * MLP_DEL_LD];   // per row: grad wrt each layer's pre-activation output
  __shared__ float gacc[MLP_MAXT];
  __shared__ float wts[MLP_WLDS];          // the parameters (layer-major), when they fit
  __shared__ int last;
  const int L = a.nlayers, lane = threadIdx.x;
  int offs[MLP_MAXL + 1];  // activation offsets (offs[l] = input of layer l)
  offs[0] = 0;
  for (int l = 0; l < L; ++l) offs[l + 1] = offs[l] + a.dims[l];
  const int T = mlp_total(a);
  // every parameter read of the row loops from LDS: one round of global loads up front instead
  // of a dependent global load per multiply-add (the kernel is latency-bound at these sizes)
  const float* Wp[MLP_MAXL];
  const float* bp[MLP_MAXL];
  const bool wl = T <= MLP_WLDS;
  for (int l = 0, base = 0; l < L; ++l) {
    const int din = a.dims[l], dout = a.dims[l + 1];
    if (wl) {
      for (int i = lane; i < dout * din; i += 64) wts[base + i] = a.W[l][i];
      for (int i = lane; i < dout; i += 64) wts[base + dout * din + i] = a.b[l][i];
      Wp[l] = wts + base;
      bp[l] = wts + base + dout * din;
    } else {
      Wp[l] = a.W[l];
      bp[l] = a.b[l];
    }
    base += dout * (din + 1);
  }
  if (wl) __syncthreads();
  if (mode > 0)
    for (int i = lane; i < T; i += 64) gacc[i] = 0.f;
  float* act_s = acts + lane * MLP_ACT_LD;
  float* del_s = dls + lane * MLP_DEL_LD;
  const float dl = a.dloss ? a.dloss[0] : 1.f;
  const int d0 = a.dims[0];
  float lsum = 0.f;
  for (int chunk = blockIdx.x * 64; chunk < a.n; chunk += gridDim.x * 64) {
    const int row = chunk + lane;
    if (row < a.n) {
      const float w = a.row_w ? a.row_w[row] : 1.f / (float)a.n;
      lsum += w * mlp_forward_row(a, row, act_s, Wp, bp);
      if (a.logits) {
        const int C = a.dims[L];
        for (int c = 0; c < C; ++c) a.logits[(long)row * C + c] = act_s[offs[L] + c];
      }
      if (mode > 0) {
        const int C = a.dims[L];
        const float* z = act_s + offs[L];
        float* dz = del_s + offs[L] - d0;
        float m = z[0];
        for (int c = 1; c < C; ++c) m = fmaxf(m, z[c]);
        float se = 0.f;
        for (int c = 0; c < C; ++c) se += __expf(z[c] - m);
        const long long lab = a.y[row];
        const float wd = w * dl;
        for (int c = 0; c < C; ++c) dz[c] = (__expf(z[c] - m) / se - (c == lab ? 1.f : 0.f)) * wd;
        for (int l = L - 1; l > 0; --l) {  // grad wrt layer l-1's pre-activation output
          const int din = a.dims[l], dout = a.dims[l + 1];
          const float* dcur = del_s + offs[l + 1] - d0;
          float* dprev = del_s + offs[l] - d0;
          const float* h = act_s + offs[l];
          for (int i = 0; i < din; ++i) {
            float s = 0.f;
            for (int o = 0; o < dout; ++o) s += Wp[l][o * din + i] * dcur[o];
            dprev[i] = a.act == 1 ? (h[i] > 0.f ? s : 0.f) : s * h[i] * (1.f - h[i]);
          }
        }
      }
    } else if (mode > 0) {  // rows past n contribute nothing
      for (int j = 0; j < offs[L] + a.dims[L] - d0; ++j) del_s[j] = 0.f;
      for (int j = 0; j < offs[L]; ++j) act_s[j] = 0.f;
    }
    if (mode == 0) continue;
    __syncthreads();
    // gradient entry e (layer-major: W[o][i] then b[o]) summed over the chunk's 64 rows, in row order
    for (int e = lane; e < T; e += 64) {
      int l = 0, base = 0;
      while (e >= base + a.dims[l + 1] * (a.dims[l] + 1)) { base += a.dims[l + 1] * (a.dims[l] + 1); ++l; }
      const int din = a.dims[l], dout = a.dims[l + 1], r = e - base;
      const bool bias = r >= dout * din;
      const int o = bias ? r - dout * din : r / din, i = bias ? 0 : r - (r / din) * din;
      const float* dp = dls + offs[l + 1] - d0 + o;
      const float* ap = acts + offs[l] + i;
      float s = 0.f;
      for (int k = 0; k < 64; ++k) s += dp[k * MLP_DEL_LD] * (bias ? 1.f : ap[k * MLP_ACT_LD]);
      gacc[e] += s;
    }
    __syncthreads();
  }
  lsum = wave_sum(lsum);
  if (gridDim.x == 1) {
    mlp_finalize(a, mode, T, gacc, lsum);
    return;
  }
  // publish this block's partials, the last block to arrive reduces them in block order
  float* part = a.ws + (long)blockIdx.x * (T + 1);
  if (mode > 0)  // write-through hand-off to the last block (smi_common.h), no L2 fences
    for (int i = lane; i < T; i += 64) smi_wt_store(part + i, gacc[i]);
  if (lane == 0) smi_wt_store(part + T, lsum);
  smi_wt_drain();
  __syncthreads();
  if (lane == 0) last = atomicAdd(a.ticket, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  mlp_finalize(a, mode, T, gacc, lsum);
  if (lane == 0) a.ticket[0] = 0u;  // re-arm for the next launch (stream-ordered)
}

// Compile-time form for the reference topology (4-5-4-3 sigmoid, batch <= 64: one wave, one row
// per lane; distributed_multilayer_perceptron.py:44-53, batch 30 at :93).  The generic kernel above
// loops over runtime dims through dynamically indexed pointer / offset arrays and LDS rows (13.7 us
// per step, latency-bound); here every activation and gradient lives in registers, the 64
// parameters are uniform (scalar) loads, and the only LDS round trip is the per-parameter row sum:
// each lane writes its row's T products, then lane e sums parameter e over the rows in row order.
// Same modes as mlp_kernel (0 loss, 1 gradients, 2 fused SGD step).
//
// Parameter q (layer-major: W[o][i] then b[o] per layer — also the gradient-row order) is read
// through an accessor P(q) with a compile-time q: the global tensors (scalar loads) in the one-step
// kernel, an LDS copy in the multi-step kernel.
template <int D0, int D1, int D2, int D3, int ACT>  // ACT: 1 relu, 2 sigmoid (compile-time: no branches)
struct Mlp43 {
  static constexpr int T1 = D1 * (D0 + 1), T2 = D2 * (D1 + 1), T3 = D3 * (D2 + 1), T = T1 + T2 + T3;
  static constexpr int PT = T + 1;  // odd pitch: the 64 lanes' product rows on distinct banks
  // the parameter (GRAD = false) or gradient (true) tensor element of entry q
  template <bool GRAD = false>
  static __device__ __forceinline__ float* addr(const MLPArgs& a, int q) {
    const int l = q < T1 ? 0 : (q < T1 + T2 ? 1 : 2);
    const int r = q - (l == 0 ? 0 : (l == 1 ? T1 : T1 + T2));
    const int din = l == 0 ? D0 : (l == 1 ? D1 : D2), dout = l == 0 ? D1 : (l == 1 ? D2 : D3);
    if (GRAD) return r >= dout * din ? a.gb[l] + (r - dout * din) : a.gW[l] + r;
    return r >= dout * din ? const_cast<float*>(a.b[l]) + (r - dout * din) : const_cast<float*>(a.W[l]) + r;
  }
  // One row (this lane's) through forward + softmax-CE (+ backward: the row's T per-parameter
  // products into the lane-private LDS row `pr`).  Returns the wave's weighted loss sum.
  template <typename PF>
  static __device__ __forceinline__ float row(PF P, const float (&x)[D0], int lab, float w, float dl, bool valid,
                                              bool bwd, float* pr, float* logits_row) {
    constexpr int act = ACT;
    float h1[D1], h2[D2], z[D3];
#pragma unroll
    for (int o = 0; o < D1; ++o) {
      float s = P(D1 * D0 + o);
#pragma unroll
      for (int i = 0; i < D0; ++i) s += P(o * D0 + i) * x[i];
      h1[o] = mlp_act(s, act);
    }
#pragma unroll
    for (int o = 0; o < D2; ++o) {
      float s = P(T1 + D2 * D1 + o);
#pragma unroll
      for (int i = 0; i < D1; ++i) s += P(T1 + o * D1 + i) * h1[i];
      h2[o] = mlp_act(s, act);
    }
#pragma unroll
    for (int o = 0; o < D3; ++o) {
      float s = P(T1 + T2 + D3 * D2 + o);
#pragma unroll
      for (int i = 0; i < D2; ++i) s += P(T1 + T2 + o * D2 + i) * h2[i];
      z[o] = s;
    }
    float m = z[0];
#pragma unroll
    for (int c = 1; c < D3; ++c) m = fmaxf(m, z[c]);
    float e[D3], se = 0.f;
#pragma unroll
    for (int c = 0; c < D3; ++c) { e[c] = __expf(z[c] - m); se += e[c]; }
    const float lse = m + __logf(se);
    float zl = z[0];
#pragma unroll
    for (int c = 1; c < D3; ++c) zl = c == lab ? z[c] : zl;
    const float lsum = wave_sum(valid ? w * (lse - zl) : 0.f);
    if (logits_row && valid) {
#pragma unroll
      for (int c = 0; c < D3; ++c) logits_row[c] = z[c];
    }
    if (!bwd) return lsum;
    // backward (rows past n: w = 0, every product 0)
    float dz[D3], d2[D2], d1[D1];
    const float inv = 1.f / se, wd = w * dl;
#pragma unroll
    for (int c = 0; c < D3; ++c) dz[c] = (e[c] * inv - (c == lab ? 1.f : 0.f)) * wd;
#pragma unroll
    for (int i = 0; i < D2; ++i) {
      float s = 0.f;
#pragma unroll
      for (int o = 0; o < D3; ++o) s += P(T1 + T2 + o * D2 + i) * dz[o];
      d2[i] = act == 1 ? (h2[i] > 0.f ? s : 0.f) : s * h2[i] * (1.f - h2[i]);
    }
#pragma unroll
    for (int i = 0; i < D1; ++i) {
      float s = 0.f;
#pragma unroll
      for (int o = 0; o < D2; ++o) s += P(T1 + o * D1 + i) * d2[o];
      d1[i] = act == 1 ? (h1[i] > 0.f ? s : 0.f) : s * h1[i] * (1.f - h1[i]);
    }
#pragma unroll
    for (int o = 0; o < D1; ++o) {
#pragma unroll
      for (int i = 0; i < D0; ++i) pr[o * D0 + i] = d1[o] * x[i];
      pr[D1 * D0 + o] = d1[o];
    }
#pragma unroll
    for (int o = 0; o < D2; ++o) {
#pragma unroll
      for (int i = 0; i < D1; ++i) pr[T1 + o * D1 + i] = d2[o] * h1[i];
      pr[T1 + D2 * D1 + o] = d2[o];
    }
#pragma unroll
    for (int o = 0; o < D3; ++o) {
#pragma unroll
      for (int i = 0; i < D2; ++i) pr[T1 + T2 + o * D2 + i] = dz[o] * h2[i];
      pr[T1 + T2 + D3 * D2 + o] = dz[o];
    }
    return lsum;
  }
  // entry q's gradient: the row-order sum of the 64 product rows
  static __device__ __forceinline__ float colsum(const float* prod, int q) {
    float g = 0.f;
#pragma unroll 16
    for (int k = 0; k < 64; ++k) g += prod[k * PT + q];
    return g;
  }
  static __device__ __forceinline__ void load_row(const float* xp, const long long* yp, int row, float (&x)[D0],
                                                  long long& lab) {
#pragma unroll
    for (int i = 0; i < D0; ++i) x[i] = xp[(long)row * D0 + i];
    lab = yp ? yp[row] : 0;
  }
  static __device__ __forceinline__ int clamp_label(long long l0) { return l0 < 0 ? 0 : (l0 >= D3 ? D3 - 1 : (int)l0); }
};

template <int D0, int D1, int D2, int D3, int ACT>
__global__ __launch_bounds__(64) void mlp_small_kernel(MLPArgs a, int mode) {
  using M = Mlp43<D0, D1, D2, D3, ACT>;
  __shared__ float prod[64 * M::PT];
  const int lane = threadIdx.x;
  const bool valid = lane < a.n;
  const int row = valid ? lane : 0;
  // parameters: uniform addresses (scalar loads, all in flight together)
  auto P = [&](int q) -> float { return *M::addr(a, q); };
  float x[D0];
  long long lab;
  M::load_row(a.x, a.y, row, x, lab);
  const float w = valid ? (a.row_w ? a.row_w[row] : 1.f / (float)a.n) : 0.f;
  const float dl = a.dloss ? a.dloss[0] : 1.f;
  const float lsum = M::row(P, x, M::clamp_label(lab), w, dl, valid, mode != 0, prod + lane * M::PT,
                            a.logits ? a.logits + (long)row * D3 : nullptr);
  if (mode == 0) {
    if (lane == 0 && a.loss) a.loss[0] = lsum;
    return;
  }
  __syncthreads();
  const float lr = mode == 2 ? a.lr[0] * a.gscale : 0.f;
  for (int q = lane; q < M::T; q += 64) {
    const float g = M::colsum(prod, q);
    if (mode == 2) {
      float* p = M::addr(a, q);
      *p -= lr * g;
    } else {
      float* gp = M::template addr<true>(a, q);
      *gp = a.accumulate ? *gp + g : g;
    }
  }
  if (lane == 0) {
    if (a.loss) a.loss[0] = lsum;
    if (mode == 2 && a.step) a.step[0] += 1.f;
  }
}

// ``s.n`` consecutive fused SGD steps (mode 2) in ONE launch: step t trains on batch (s.x[t],
// s.y[t]) and writes its loss to s.loss[t].  The parameters live in LDS between steps (lane q
// updates entry q after the row sums, a barrier, every lane reads the new values), so each step is
// bitwise the one-step kernel's step; they are written back once at the end, the step counter
// advanced by s.n.  The next step's rows are loaded while the current step computes.  A launch per
// step left the step latency-bound on launch gaps (~5 us per step inside a multi-step graph).
template <int D0, int D1, int D2, int D3, int ACT>
__global__ __launch_bounds__(64) void mlp_small_steps_kernel(MLPArgs a, MLPSteps s) {
  using M = Mlp43<D0, D1, D2, D3, ACT>;
  __shared__ float prod[64 * M::PT];
  __shared__ float pl[M::T];
  __shared__ int srcs[MLP_MAX_STEPS][64];  // index mode: every step's dataset row of each lane
  __shared__ float lsums[MLP_MAX_STEPS];    // the step losses, stored once at the end
  const int lane = threadIdx.x;
  for (int q = lane; q < M::T; q += 64) pl[q] = *M::addr(a, q);
  const bool valid = lane < a.n;
  const int row = valid ? lane : 0;
  const int c0 = s.perm ? s.cursor[0] : 0;
  if (s.perm) {  // all steps' permutation entries in flight at once, then one LDS table
    for (int t = 0; t < s.n; ++t) srcs[t][lane] = (int)s.perm[(long)(c0 + t) * s.B + row];
  }
  const float w = valid ? (a.row_w ? a.row_w[row] : 1.f / (float)a.n) : 0.f;
  const float lr = a.lr[0] * a.gscale;
  const float dl = a.dloss ? a.dloss[0] : 1.f;
  auto P = [&](int q) -> float { return pl[q]; };
  __syncthreads();
  auto src = [&](int t) -> int { return s.perm ? srcs[t][lane] : row; };
  float x[D0];
  long long lab;
  M::load_row(s.x[0], s.y[0], src(0), x, lab);
  // the first rows arrive here: no load is outstanding at the loop head, so the waitcnt pass does
  // not make every step wait for its own prefetch (the loop-head wait merges the entry path)
#pragma unroll
  for (int i = 0; i < D0; ++i) asm volatile("" : "+v"(x[i]));
  asm volatile("" : "+v"(lab));
  for (int t = 0; t < s.n; ++t) {
    // the next step's rows, loaded now: their wait sits at the end of this step (the label is
    // clamped at its use, not at the load)
    float xn[D0];
    long long ln;
    const int tn = t + 1 < s.n ? t + 1 : t;  // the last step reloads its own rows (unused)
    M::load_row(s.x[tn], s.y[tn], src(tn), xn, ln);
    const float lsum = M::row(P, x, M::clamp_label(lab), w, dl, valid, true, prod + lane * M::PT, nullptr);
    __syncthreads();
    for (int q = lane; q < M::T; q += 64) pl[q] -= lr * M::colsum(prod, q);
    // no global store inside the loop: stores share the in-order vmcnt with the prefetch loads, so
    // the step-end wait for the next rows would also wait out the store's round trip
    if (lane == 0) lsums[t] = lsum;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < D0; ++i) x[i] = xn[i];
    lab = ln;
  }
  for (int q = lane; q < M::T; q += 64) *M::addr(a, q) = pl[q];
  if (lane == 0) {
    float tot = 0.f;
    for (int t = 0; t < s.n; ++t) {
      if (s.loss[t]) s.loss[t][0] = lsums[t];
      tot += lsums[t];
    }
    if (s.loss_sum) s.loss_sum[0] = tot;
    if (a.step) a.step[0] += (float)s.n;
    if (s.perm) s.cursor[0] = c0 + s.n;
  }
}

static bool mlp_small_ok(const MLPArgs& a) {
  return a.nlayers == 3 && a.dims[0] == 4 && a.dims[1] == 5 && a.dims[2] == 4 && a.dims[3] == 3 && a.n >= 1 &&
         a.n <= 64 && (a.act == 1 || a.act == 2);
}

static int mlp_check(const MLPArgs& a) {
  if (a.nlayers < 1 || a.nlayers > MLP_MAXL) return -1;
  int total = 0;
  for (int l = 0; l <= a.nlayers; ++l) if (a.dims[l] < 1 || a.dims[l] > MLP_MAXW) return -1;
  for (int l = 0; l < a.nlayers; ++l) total += a.dims[l + 1] * (a.dims[l] + 1);
  if (total > MLP_MAXT) return -1;
  return 0;
}

extern "C" int smi_mlp_grid(int n) {
  int b = (n + 63) / 64;
  return b < 1 ? 1 : (b > MLP_MAX_GRID ? MLP_MAX_GRID : b);
}

// the compile-time 4-5-4-3 kernel for batches of <= 64 rows (1, default) or always the generic one
// (0: tests compare the two)
static int g_mlp_small = 1;
extern "C" int smi_mlp_small(int set) {
  if (set == 0 || set == 1) g_mlp_small = set;
  return g_mlp_small;
}

// mode 0 forward/loss, 1 forward+backward (gradients), 2 forward+backward+SGD (one launch per
// training step).  grid > 1 needs a.ws ([grid][total+1] floats) and a zeroed a.ticket.
extern "C" int smi_mlp(const MLPArgs* args, int mode, hipStream_t st) {
  const MLPArgs& a = *args;
  if (mlp_check(a) || mode < 0 || mode > 2) return -1;
  const int grid = smi_mlp_grid(a.n);
  if (grid > 1 && (!a.ws || !a.ticket)) return -1;
  if (mode > 0 && !a.y) return -1;
  if (mode == 1) for (int l = 0; l < a.nlayers; ++l) if (!a.gW[l] || !a.gb[l]) return -1;
  if (mode == 2 && !a.lr) return -1;
  if (mlp_small_ok(a) && g_mlp_small) {
    if (mode == 2 && !a.logits) {
      // the fused SGD step IS the multi-step kernel with one step: a step is then the same code
      // whether it runs alone or inside a multi-step launch (bitwise the same training run)
      MLPSteps s{};
      s.n = 1; s.x[0] = a.x; s.y[0] = a.y; s.loss[0] = a.loss;
      if (a.act == 1) hipLaunchKernelGGL((mlp_small_steps_kernel<4, 5, 4, 3, 1>), dim3(1), dim3(64), 0, st, a, s);
      else hipLaunchKernelGGL((mlp_small_steps_kernel<4, 5, 4, 3, 2>), dim3(1), dim3(64), 0, st, a, s);
    } else if (a.act == 1) {
      hipLaunchKernelGGL((mlp_small_kernel<4, 5, 4, 3, 1>), dim3(1), dim3(64), 0, st, a, mode);
    } else {
      hipLaunchKernelGGL((mlp_small_kernel<4, 5, 4, 3, 2>), dim3(1), dim3(64), 0, st, a, mode);
    }
  } else {
    hipLaunchKernelGGL(mlp_kernel, dim3(grid), dim3(64), 0, st, a, mode);
  }
  SMI_CHECK_LAUNCH();
}

// s.n fused SGD steps in one launch (the 4-5-4-3 kernel's shapes only: -1 otherwise, the caller
// runs one launch per step)
extern "C" int smi_mlp_steps(const MLPArgs* args, const MLPSteps* steps, hipStream_t st) {
  const MLPArgs& a = *args;
  const MLPSteps& s = *steps;
  if (mlp_check(a) || !mlp_small_ok(a) || !g_mlp_small || !a.lr || !a.y || a.logits) return -1;
  if (s.n < 1 || s.n > MLP_MAX_STEPS || (s.perm && (!s.cursor || s.B != a.n))) return -1;
  for (int t = 0; t < s.n; ++t)
    if (!s.x[t] || !s.y[t] || !s.loss[t]) return -1;
  if (a.act == 1) hipLaunchKernelGGL((mlp_small_steps_kernel<4, 5, 4, 3, 1>), dim3(1), dim3(64), 0, st, a, s);
  else hipLaunchKernelGGL((mlp_small_steps_kernel<4, 5, 4, 3, 2>), dim3(1), dim3(64), 0, st, a, s);
  SMI_CHECK_LAUNCH();
}
