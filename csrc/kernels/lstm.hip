// Persistent multi-layer LSTM: embedding gather + L stacked LSTM layers (inter-layer dropout) +
// per-step fc head, forward and full BPTT, one workgroup per sequence.
//
// Reference: distributed_lstm.py:110-135 / pytorch_lstm.py:94-119 (nn.Embedding(V, 32,
// padding_idx) -> nn.LSTM(32, 32, num_layers=2, batch_first, dropout=0.5) -> fc_out at every
// step), trained with CE on pred[:, -1, :] (distributed_lstm.py:186-189).
//
// MI355X design: the recurrence is latency bound (T=129 dependent steps, 32 sequences per GPU),
// so every sequence gets one workgroup that keeps ALL its weights in registers for the whole
// sequence: thread (l, r) owns gate row r of layer l (its W_ih / W_hh rows, fp32) and the layers
// are software-pipelined across "ticks" (layer l works on step t = tick - l), so an L-layer
// stack costs T + L - 1 ticks, not L*T.  A tick is: gate pre-activations (row dot products
// against the LDS-broadcast input / hidden vectors) -> barrier -> cell update by H threads per
// layer -> barrier.  Gates, c and h are saved to a workspace for BPTT.
//
// Backward runs the ticks in reverse with the layers pipelined the other way (top layer
// first).  Thread (l, r) accumulates dW_ih[r,:], dW_hh[r,:] and db[r] in registers over all
// steps (no atomics inside the loop) and holds a slice of W columns for the transposed
// products dh_{t-1} = W_hh^T da and dx_t = W_ih^T da (2 or 4 threads per output, combined
// through LDS).  Layer-0 gate grads go to a scratch buffer and the embedding gradient is one
// parallel W_ih0^T * da pass at the end, scattered into the fp32 table gradient with atomics
// (rows == padding_idx skipped).  Weight gradients are added atomically into the caller's
// (flat) fp32 gradient buffers once per sequence.
#include "smi_common.h"
#include "smi_lstm.h"

__device__ __forceinline__ float smi_sigmoid(float x) { return 1.0f / (1.0f + __expf(-x)); }
__device__ __forceinline__ float smi_tanh(float x) {
  const float e = __expf(-2.0f * fabsf(x));
  const float t = (1.0f - e) / (1.0f + e);
  return copysignf(t, x);
}

__device__ __forceinline__ uint32_t lstm_drop_idx(int b, int t, int l, int j, int T, int L, int H) {
  return (uint32_t)((((size_t)b * T + t) * L + l) * H + j);
}

template <int H, int MI, int NT>  // hidden size, padded input width (>= E, >= H), block threads
__global__ __launch_bounds__(NT) void lstm_fwd_kernel(LSTMArgs a) {
  constexpr int G = 4 * H;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int L = a.L, T = a.T, E = a.E, C = a.C;
  const int l = tid / G, r = tid % G;
  const bool act = l < L;
  const int In = l == 0 ? E : H;
  __shared__ __attribute__((aligned(16))) float s_in[LSTM_MAXL][MI];
  __shared__ __attribute__((aligned(16))) float s_h[LSTM_MAXL][H];
  __shared__ float s_g[LSTM_MAXL][G];

  float wi[MI], wh[H], bias = 0.f;
#pragma unroll
  for (int i = 0; i < MI; ++i) wi[i] = (act && i < In) ? a.w_ih[l][(size_t)r * In + i] : 0.f;
#pragma unroll
  for (int i = 0; i < H; ++i) wh[i] = act ? a.w_hh[l][(size_t)r * H + i] : 0.f;
  if (act) bias = a.b_ih[l][r] + a.b_hh[l][r];
  for (int i = tid; i < LSTM_MAXL * MI; i += blockDim.x) (&s_in[0][0])[i] = 0.f;
  float c = 0.f;
  __syncthreads();
  if (act && r < H) {
    c = a.c0 ? a.c0[((size_t)l * a.B + b) * H + r] : 0.f;
    s_h[l][r] = a.h0 ? a.h0[((size_t)l * a.B + b) * H + r] : 0.f;
  }
  const long long* ids = a.ids + (size_t)b * T;
  for (int e = tid; e < E; e += blockDim.x) s_in[0][e] = a.emb[(size_t)ids[0] * E + e];
  __syncthreads();

  const uint32_t seed = smi_seed(a.seedp, a.salt);
  const int gate = r / H;  // 0 i, 1 f, 2 g, 3 o
  float* wsb = a.ws + (size_t)b * L * T * 6 * H;
  const int nt = T + L - 1;
  for (int k = 0; k < nt; ++k) {
    const int t = k - l;
    const bool on = act && t >= 0 && t < T;
    if (on) {
      float s0 = bias, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
      for (int i = 0; i < MI; i += 4) {
        const float4 x = *(const float4*)&s_in[l][i];
        s0 += wi[i] * x.x; s1 += wi[i + 1] * x.y; s2 += wi[i + 2] * x.z; s3 += wi[i + 3] * x.w;
      }
#pragma unroll
      for (int i = 0; i < H; i += 4) {
        const float4 x = *(const float4*)&s_h[l][i];
        s0 += wh[i] * x.x; s1 += wh[i + 1] * x.y; s2 += wh[i + 2] * x.z; s3 += wh[i + 3] * x.w;
      }
      const float z = (s0 + s1) + (s2 + s3);
      s_g[l][r] = gate == 2 ? smi_tanh(z) : smi_sigmoid(z);
    }
    __syncthreads();
    if (on && r < H) {
      const float ig = s_g[l][r], fg = s_g[l][H + r], gg = s_g[l][2 * H + r], og = s_g[l][3 * H + r];
      c = fg * c + ig * gg;
      const float h = og * smi_tanh(c);
      s_h[l][r] = h;
      float* w = wsb + ((size_t)l * T + t) * 6 * H;
      w[r] = ig; w[H + r] = fg; w[2 * H + r] = gg; w[3 * H + r] = og; w[4 * H + r] = c; w[5 * H + r] = h;
      if (l + 1 < L) {
        float hd = h;
        if (a.thresh) hd = smi_keep(seed, lstm_drop_idx(b, t, l, r, T, L, H), a.thresh) ? h * a.dscale : 0.f;
        s_in[l + 1][r] = hd;
      }
    }
    if (k + 1 < T)  // layer 0's input for the next tick (s_in[0] was consumed before the barrier)
      for (int e = tid; e < E; e += blockDim.x) s_in[0][e] = a.emb[(size_t)ids[k + 1] * E + e];
    __syncthreads();
  }
  if (act && r < H) {
    if (a.hn) a.hn[((size_t)l * a.B + b) * H + r] = s_h[l][r];
    if (a.cn) a.cn[((size_t)l * a.B + b) * H + r] = c;
  }
  // fc head at every step (reads this workgroup's own workspace writes, ordered by the barrier)
  const float* top = wsb + (size_t)(L - 1) * T * 6 * H + 5 * H;
  for (int o = tid; o < T * C; o += blockDim.x) {
    const int t = o / C, cc = o % C;
    float s = a.b_fc[cc];
    const float* hv = top + (size_t)t * 6 * H;
    const float* wv = a.w_fc + (size_t)cc * H;
#pragma unroll 8
    for (int j = 0; j < H; ++j) s += wv[j] * hv[j];
    a.pred[((size_t)b * T + t) * C + cc] = s;
  }
}

template <int H, int MI, int NT>
__global__ __launch_bounds__(NT) void lstm_bwd_kernel(LSTMArgs a) {
  constexpr int G = 4 * H;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int L = a.L, T = a.T, E = a.E, C = a.C;
  const int l = tid / G, r = tid % G;
  const bool act = l < L;
  const int In = l == 0 ? E : H;
  __shared__ __attribute__((aligned(16))) float s_x[LSTM_MAXL][MI];
  __shared__ __attribute__((aligned(16))) float s_hp[LSTM_MAXL][H];
  __shared__ __attribute__((aligned(16))) float s_da[LSTM_MAXL][G];
  __shared__ float s_part[LSTM_MAXL][G];
  __shared__ float s_dhr[LSTM_MAXL][H];
  __shared__ float s_dxu[LSTM_MAXL][H];

  // transposed-product assignment: l >= 1: output o = r % 2H (o < H: dh via W_hh col o, else dx
  // via W_ih col o-H) over gate rows [part*2H, part*2H+2H); l == 0: o = r % H (dh only) over
  // rows [part*H, part*H+H).
  const int nq = l == 0 ? H : 2 * H;
  const int o = r % nq, part = r / nq, row0 = part * nq;
  float wc[2 * H];
#pragma unroll
  for (int q = 0; q < 2 * H; ++q) {
    float v = 0.f;
    if (act && q < nq) {
      const int rr = row0 + q;
      v = (o < H) ? a.w_hh[l][(size_t)rr * H + o] : a.w_ih[l][(size_t)rr * H + (o - H)];
    }
    wc[q] = v;
  }
  float dWi[MI], dWh[H], db = 0.f;
#pragma unroll
  for (int i = 0; i < MI; ++i) dWi[i] = 0.f;
#pragma unroll
  for (int i = 0; i < H; ++i) dWh[i] = 0.f;

  for (int i = tid; i < LSTM_MAXL * MI; i += blockDim.x) (&s_x[0][0])[i] = 0.f;
  float dc = 0.f;
  if (act && r < H) {
    dc = a.dcn ? a.dcn[((size_t)l * a.B + b) * H + r] : 0.f;
    s_dhr[l][r] = a.dhn ? a.dhn[((size_t)l * a.B + b) * H + r] : 0.f;
    s_dxu[l][r] = 0.f;
  }
  __syncthreads();

  const uint32_t seed = smi_seed(a.seedp, a.salt);
  const long long* ids = a.ids + (size_t)b * T;
  const float* wsb = a.ws + (size_t)b * L * T * 6 * H;
  const float* dpred = a.dpred + (size_t)b * T * C;
  float* dab = a.ws_da + (size_t)b * T * G;
  const int nt = T + L - 1;
  for (int k = 0; k < nt; ++k) {
    const int t = T - 1 - k + (L - 1 - l);
    const bool on = act && t >= 0 && t < T;
    if (on && r < H) {  // cell backward for unit j = r
      const int j = r;
      const float* w = wsb + ((size_t)l * T + t) * 6 * H;
      const float ig = w[j], fg = w[H + j], gg = w[2 * H + j], og = w[3 * H + j], cc = w[4 * H + j];
      float cp, hp;
      if (t > 0) { cp = w[j + 4 * H - 6 * H]; hp = w[j + 5 * H - 6 * H]; }
      else {
        cp = a.c0 ? a.c0[((size_t)l * a.B + b) * H + j] : 0.f;
        hp = a.h0 ? a.h0[((size_t)l * a.B + b) * H + j] : 0.f;
      }
      float dh = s_dhr[l][j];
      if (l == L - 1) {
        for (int q = 0; q < C; ++q) dh += a.w_fc[(size_t)q * H + j] * dpred[(size_t)t * C + q];
      } else {
        dh += s_dxu[l][j];
      }
      const float tc = smi_tanh(cc);
      const float d_o = dh * tc;
      dc += dh * og * (1.f - tc * tc);
      s_da[l][j] = dc * gg * ig * (1.f - ig);
      s_da[l][H + j] = dc * cp * fg * (1.f - fg);
      s_da[l][2 * H + j] = dc * ig * (1.f - gg * gg);
      s_da[l][3 * H + j] = d_o * og * (1.f - og);
      dc *= fg;
      s_hp[l][j] = hp;
      if (l >= 1) {
        const float hx = wsb[((size_t)(l - 1) * T + t) * 6 * H + 5 * H + j];
        s_x[l][j] = a.thresh ? (smi_keep(seed, lstm_drop_idx(b, t, l - 1, j, T, L, H), a.thresh) ? hx * a.dscale : 0.f)
                             : hx;
      }
    }
    if (on && l == 0)
      for (int e = r; e < E; e += G) s_x[0][e] = a.emb[(size_t)ids[t] * E + e];
    __syncthreads();
    if (on) {
      const float da = s_da[l][r];
#pragma unroll
      for (int i = 0; i < MI; i += 4) {
        const float4 x = *(const float4*)&s_x[l][i];
        dWi[i] += da * x.x; dWi[i + 1] += da * x.y; dWi[i + 2] += da * x.z; dWi[i + 3] += da * x.w;
      }
#pragma unroll
      for (int i = 0; i < H; i += 4) {
        const float4 x = *(const float4*)&s_hp[l][i];
        dWh[i] += da * x.x; dWh[i + 1] += da * x.y; dWh[i + 2] += da * x.z; dWh[i + 3] += da * x.w;
      }
      db += da;
      float p0 = 0.f, p1 = 0.f;
#pragma unroll
      for (int q = 0; q < 2 * H; q += 2) {
        if (q < nq) { p0 += wc[q] * s_da[l][row0 + q]; p1 += wc[q + 1] * s_da[l][row0 + q + 1]; }
      }
      s_part[l][r] = p0 + p1;
      if (l == 0) dab[(size_t)t * G + r] = da;
    }
    __syncthreads();
    if (on && r < H) {
      const int j = r;
      if (l >= 1) {
        s_dhr[l][j] = s_part[l][j] + s_part[l][2 * H + j];
        const float dx = s_part[l][H + j] + s_part[l][3 * H + j];
        s_dxu[l - 1][j] = a.thresh ? (smi_keep(seed, lstm_drop_idx(b, t, l - 1, j, T, L, H), a.thresh) ? dx * a.dscale : 0.f)
                                   : dx;
      } else {
        s_dhr[0][j] = (s_part[0][j] + s_part[0][H + j]) + (s_part[0][2 * H + j] + s_part[0][3 * H + j]);
      }
    }
    __syncthreads();
  }
  if (act && r < H) {
    if (a.dh0) a.dh0[((size_t)l * a.B + b) * H + r] = s_dhr[l][r];
    if (a.dc0) a.dc0[((size_t)l * a.B + b) * H + r] = dc;
  }
  if (act) {
    float* gwi = a.g_w_ih[l] + (size_t)r * In;
#pragma unroll
    for (int i = 0; i < MI; ++i) if (i < In) atomicAdd(gwi + i, dWi[i]);
    float* gwh = a.g_w_hh[l] + (size_t)r * H;
#pragma unroll
    for (int i = 0; i < H; ++i) atomicAdd(gwh + i, dWh[i]);
    atomicAdd(a.g_b_ih[l] + r, db);
    atomicAdd(a.g_b_hh[l] + r, db);
  }
  // fc head grads: dW_fc[c][j] = sum_t dpred[t][c] * h_top(t)[j]; db_fc[c] = sum_t dpred[t][c]
  const float* top = wsb + (size_t)(L - 1) * T * 6 * H + 5 * H;
  for (int q = tid; q < C * (H + 1); q += blockDim.x) {
    const int cc = q / (H + 1), j = q % (H + 1);
    float s = 0.f;
    if (j < H) { for (int t = 0; t < T; ++t) s += dpred[(size_t)t * C + cc] * top[(size_t)t * 6 * H + j]; atomicAdd(a.g_w_fc + (size_t)cc * H + j, s); }
    else { for (int t = 0; t < T; ++t) s += dpred[(size_t)t * C + cc]; atomicAdd(a.g_b_fc + cc, s); }
  }
  // embedding grads: d emb[ids[t]] += W_ih0^T da0(t)   (scratch written above by this workgroup)
  if (a.g_emb) {
    for (int q = tid; q < T * E; q += blockDim.x) {
      const int t = q / E, e = q % E;
      const long long id = ids[t];
      if (id == a.pad_idx) continue;
      const float* dv = dab + (size_t)t * G;
      const float* wv = a.w_ih[0] + e;
      float s0 = 0.f, s1 = 0.f;
      for (int rr = 0; rr < G; rr += 2) { s0 += wv[(size_t)rr * E] * dv[rr]; s1 += wv[(size_t)(rr + 1) * E] * dv[rr + 1]; }
      atomicAdd(a.g_emb + (size_t)id * E + e, s0 + s1);
    }
  }
}

// 4*H*L <= 256 threads: one wave per SIMD, so the backward's register-resident gradient rows
// and W column slices get the full 512-entry (VGPR + AGPR) file.
template <int H, int MI>
static int lstm_launch(const LSTMArgs* a, int backward, hipStream_t st) {
  const int threads = ((4 * H * a->L + 63) / 64) * 64;
  if (threads <= 256) {
    if (backward) hipLaunchKernelGGL((lstm_bwd_kernel<H, MI, 256>), dim3(a->B), dim3(threads), 0, st, *a);
    else hipLaunchKernelGGL((lstm_fwd_kernel<H, MI, 256>), dim3(a->B), dim3(threads), 0, st, *a);
  } else {
    if (backward) hipLaunchKernelGGL((lstm_bwd_kernel<H, MI, 512>), dim3(a->B), dim3(threads), 0, st, *a);
    else hipLaunchKernelGGL((lstm_fwd_kernel<H, MI, 512>), dim3(a->B), dim3(threads), 0, st, *a);
  }
  return (int)hipGetLastError();
}

extern "C" int smi_lstm_supported(int E, int H, int L, int C) {
  if (L < 1 || L > LSTM_MAXL || C < 1 || C > LSTM_MAXC || E < 1) return 0;
  if (H != 16 && H != 32 && H != 64) return 0;
  if (4 * H * L > 512) return 0;
  const int mi = E <= H ? H : (E <= 2 * H ? 2 * H : 0);
  if (!mi || mi > 64) return 0;
  return 1;
}

extern "C" int smi_lstm(const LSTMArgs* a, int backward, hipStream_t st) {
  if (!smi_lstm_supported(a->E, a->H, a->L, a->C) || a->B < 1 || a->T < 1) return -1;
  const int H = a->H;
  const bool wide = a->E > H;
  if (H == 16) return wide ? lstm_launch<16, 32>(a, backward, st) : lstm_launch<16, 16>(a, backward, st);
  if (H == 32) return wide ? lstm_launch<32, 64>(a, backward, st) : lstm_launch<32, 32>(a, backward, st);
  return lstm_launch<64, 64>(a, backward, st);
}
