// Fused small-MLP forward/backward: affine -> sigmoid|relu hidden layers -> affine logits ->
// softmax cross-entropy, for the reference's 4-5-4-3 sigmoid MLP (distributed_multilayer_
// perceptron.py:44-53, pytorch_multilayer_perceptron.py:33-42) and Spark MLlib's
// MultilayerPerceptronClassifier topology (AffineLayer + Sigmoid, SoftmaxLayerWithCrossEntropy;
// SURVEY App. A.1), which is the same model.
//
// The whole network is a few dozen parameters, so the GPU cost is launch latency, not FLOPs:
// one kernel does the full-batch (or minibatch) forward + loss, one does forward-recompute +
// backward + gradient accumulation; each wave64 handles 64 rows (one row per lane), per-lane
// activations and pre-activation gradients live in LDS rows with an odd pitch (an even
// multiple-of-32 pitch put all 64 lanes on one bank: 74 us per backward at batch 30), and each
// weight-gradient entry is summed over the 64 rows by one lane (no LDS atomics, fixed order),
// then flushed with one global atomic per parameter per block.  Row weights implement MLlib's per-block
// loss averaging (or 1/n for the torch-style mean).
#include "smi_common.h"

#include "smi_mlp.h"

__device__ __forceinline__ float mlp_act(float v, int act) {
  return act == 1 ? fmaxf(v, 0.f) : 1.f / (1.f + __expf(-v));
}

// forward one row; activations of every layer stored in a (lane-private) LDS slab
__device__ __forceinline__ float mlp_forward_row(const MLPArgs& a, int row, float* act_s) {
  int off = 0;
  const int d0 = a.dims[0];
  for (int i = 0; i < d0; ++i) act_s[i] = a.x[(long)row * d0 + i];
  for (int l = 0; l < a.nlayers; ++l) {
    const int din = a.dims[l], dout = a.dims[l + 1];
    const float* in = act_s + off;
    float* out = act_s + off + din;
    const bool last = l == a.nlayers - 1;
    for (int o = 0; o < dout; ++o) {
      float s = a.b[l][o];
      const float* w = a.W[l] + o * din;
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

__device__ unsigned mlp_loss_ticket = 0u;
__device__ float mlp_loss_part[1024];  // per-block partial losses (grid <= 1024, mlp_grid)

#define MLP_ACT_LD (MLP_ACT_STRIDE + 1)        // odd LDS pitch: lane-private rows on distinct banks
#define MLP_DEL_LD (MLP_MAXW * MLP_MAXL + 1)

__global__ __launch_bounds__(64) void mlp_fwd_kernel(MLPArgs a) {
  __shared__ float acts[64 * MLP_ACT_LD];
  float* act_s = acts + threadIdx.x * MLP_ACT_LD;
  float lsum = 0.f;
  for (int row = blockIdx.x * 64 + threadIdx.x; row < a.n; row += gridDim.x * 64) {
    const float l = mlp_forward_row(a, row, act_s);
    const float w = a.row_w ? a.row_w[row] : 1.f / (float)a.n;
    lsum += w * l;
    if (a.logits) {
      int off = 0;
      for (int k = 0; k < a.nlayers; ++k) off += a.dims[k];
      const int C = a.dims[a.nlayers];
      for (int c = 0; c < C; ++c) a.logits[(long)row * C + c] = act_s[off + c];
    }
  }
  lsum = wave_sum(lsum);
  if (!a.loss) return;
  // mean loss without a zeroed accumulator (one fill launch per step): per-block partials, the
  // last block (atomic ticket) adds them in block order and re-arms the ticket
  __shared__ int last;
  if (threadIdx.x == 0) {
    mlp_loss_part[blockIdx.x] = lsum;
    __threadfence();
    last = atomicAdd(&mlp_loss_ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (last) {
    __threadfence();
    float s = 0.f;
    for (int i = threadIdx.x; i < (int)gridDim.x; i += 64)
      s += __hip_atomic_load(mlp_loss_part + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s = wave_sum(s);
    if (threadIdx.x == 0) {
      a.loss[0] = s;
      mlp_loss_ticket = 0u;
    }
  }
}

__global__ __launch_bounds__(64) void mlp_bwd_kernel(MLPArgs a) {
  __shared__ float acts[64 * MLP_ACT_LD];  // per row: layer inputs (dims[0..L-1]) + logits
  __shared__ float dls[64 * MLP_DEL_LD];   // per row: grad wrt each layer's pre-activation output
  __shared__ float gacc[8192];
  const int L = a.nlayers, lane = threadIdx.x;
  int offs[MLP_MAXL + 1];  // activation offsets (offs[l] = input of layer l)
  offs[0] = 0;
  for (int l = 0; l < L; ++l) offs[l + 1] = offs[l] + a.dims[l];
  int total = 0;
  for (int l = 0; l < L; ++l) total += a.dims[l + 1] * (a.dims[l] + 1);
  for (int i = lane; i < total; i += 64) gacc[i] = 0.f;
  float* act_s = acts + lane * MLP_ACT_LD;
  float* del_s = dls + lane * MLP_DEL_LD;
  const float dl = a.dloss ? a.dloss[0] : 1.f;
  const int d0 = a.dims[0];
  for (int chunk = blockIdx.x * 64; chunk < a.n; chunk += gridDim.x * 64) {
    const int row = chunk + lane;
    if (row < a.n) {
      mlp_forward_row(a, row, act_s);
      const float w = (a.row_w ? a.row_w[row] : 1.f / (float)a.n) * dl;
      const int C = a.dims[L];
      const float* z = act_s + offs[L];
      float* dz = del_s + offs[L] - d0;
      float m = z[0];
      for (int c = 1; c < C; ++c) m = fmaxf(m, z[c]);
      float se = 0.f;
      for (int c = 0; c < C; ++c) se += __expf(z[c] - m);
      const long long lab = a.y[row];
      for (int c = 0; c < C; ++c) dz[c] = (__expf(z[c] - m) / se - (c == lab ? 1.f : 0.f)) * w;
      for (int l = L - 1; l > 0; --l) {  // grad wrt layer l-1's pre-activation output
        const int din = a.dims[l], dout = a.dims[l + 1];
        const float* dcur = del_s + offs[l + 1] - d0;
        float* dprev = del_s + offs[l] - d0;
        const float* h = act_s + offs[l];
        for (int i = 0; i < din; ++i) {
          float s = 0.f;
          for (int o = 0; o < dout; ++o) s += a.W[l][o * din + i] * dcur[o];
          dprev[i] = a.act == 1 ? (h[i] > 0.f ? s : 0.f) : s * h[i] * (1.f - h[i]);
        }
      }
    } else {  // rows past n contribute nothing
      for (int j = 0; j < offs[L] + a.dims[L] - d0; ++j) del_s[j] = 0.f;
      for (int j = 0; j < offs[L]; ++j) act_s[j] = 0.f;
    }
    __syncthreads();
    // gradient entry e (layer-major: W[o][i] then b[o]) summed over the chunk's 64 rows, in row order
    for (int e = lane; e < total; e += 64) {
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
  for (int l = 0, base = 0; l < L; ++l) {
    const int din = a.dims[l], dout = a.dims[l + 1];
    const float* g = gacc + base;
    for (int i = lane; i < dout * din; i += 64) atomicAdd(&a.gW[l][i], g[i]);
    for (int i = lane; i < dout; i += 64) atomicAdd(&a.gb[l][i], g[dout * din + i]);
    base += dout * (din + 1);
  }
}

static int mlp_check(const MLPArgs& a) {
  if (a.nlayers < 1 || a.nlayers > MLP_MAXL) return -1;
  int total = 0;
  for (int l = 0; l <= a.nlayers; ++l) if (a.dims[l] < 1 || a.dims[l] > MLP_MAXW) return -1;
  for (int l = 0; l < a.nlayers; ++l) total += a.dims[l + 1] * (a.dims[l] + 1);
  if (total > 8192) return -1;
  return 0;
}

static unsigned mlp_grid(int n) {
  int b = (n + 63) / 64;
  return (unsigned)(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}

extern "C" int smi_mlp_fwd(const MLPArgs* args, hipStream_t st) {
  if (mlp_check(*args)) return -1;
  hipLaunchKernelGGL(mlp_fwd_kernel, dim3(mlp_grid(args->n)), dim3(64), 0, st, *args);
  SMI_CHECK_LAUNCH();
}

extern "C" int smi_mlp_bwd(const MLPArgs* args, hipStream_t st) {
  if (mlp_check(*args)) return -1;
  hipLaunchKernelGGL(mlp_bwd_kernel, dim3(mlp_grid(args->n)), dim3(64), 0, st, *args);
  SMI_CHECK_LAUNCH();
}
