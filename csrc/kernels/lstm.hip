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
// first).  A tick is the recurrence only: the cell backward of unit j (H threads per layer) on
// terms prepared a tick ahead, then the transposed products dh_{t-1} = W_hh^T da and
// dx_t = W_ih^T da (thread (l, r) holds a slice of W columns; 2 or 4 threads per output,
// combined through LDS); two LDS-only barriers per tick.  No global load sits on the critical
// path: the saved gates / cell state and the head's dpred are prefetched TWO ticks ahead into
// rotating register sets.
// The BPTT kernel runs only the recurrence (cell backward + transposed products) and saves every
// layer's gate gradients; the weight gradients are then a split-K GEMM over all (b, t) with a
// fixed-order combine (lstm_wgrad_partial / _combine, 128+ workgroups), and the embedding-table
// gradient the position-ordered bucketed backward of csrc/kernels/embedding.hip over
// lstm_xe_kernel's per-token W_ih0^T da0.  No float atomics anywhere: bit-reproducible.
#include "smi_common.h"
#include "smi_lstm.h"
#include "smi_emb_pair.h"

// v_rcp_f32 (1 ulp) instead of the IEEE division sequence (~10 dependent instructions): the
// activations sit on the recurrence's serial chain three times per tick
__device__ __forceinline__ float smi_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float smi_tanh(float x) {
  const float e = __expf(-2.0f * fabsf(x));
  const float t = (1.0f - e) * __builtin_amdgcn_rcpf(1.0f + e);
  return copysignf(t, x);
}

#ifdef LSTM_STAMPS  // diagnostic build only (tools/probes/lstm_probe.hip): per-phase cycle sums
__device__ unsigned long long lstm_stamps[4][8];
__device__ unsigned long long lstm_rt[4];  // [0..1] s_memrealtime / [2..3] s_memtime around the fwd tick loop
// sums kept in registers, added to lstm_stamps once per wave at exit (a global read-modify-write
// per tick waited on its load every tick and slowed the stamped workgroup)
#define LSTAMP_DECL long long lst_[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define LSTAMP_T(v) do { (v) = clock64(); } while (0)
#define LSTAMP_ADD(slot, i, t0, t1) (lst_[i] += (t1) - (t0))
#define LSTAMP_FLUSH(slot) do { if ((threadIdx.x & 63) == 0 && blockIdx.x == 0) for (int i_ = 0; i_ < 8; ++i_) lstm_stamps[slot][i_] += lst_[i_]; } while (0)
#else
#define LSTAMP_DECL
#define LSTAMP_T(v) do {} while (0)
#define LSTAMP_ADD(slot, i, t0, t1) do {} while (0)
#define LSTAMP_FLUSH(slot) do {} while (0)
#endif


__device__ __forceinline__ uint32_t lstm_drop_idx(int b, int t, int l, int j, int T, int L, int H) {
  return (uint32_t)((((size_t)b * T + t) * L + l) * H + j);
}

// Fused CE on the last step's prediction (LSTMArgs::ce_labels; distributed_lstm.py:189
// CrossEntropyLoss(pred[:, -1, :], labels - 1) with its mean): thread 0 of sequence b's workgroup
// computes the row loss and the head gradient (softmax - onehot) / B from the logits in LDS; the
// last workgroup to finish (ticket; write-through hand-off) sums the row losses in sequence
// order.  Replaces three launches (CE forward, finalize, backward) per step.
__device__ __forceinline__ void lstm_ce_tail(const LSTMArgs& a, int b, const float* s_plast) {
  __shared__ int s_lastwg;
  __syncthreads();  // s_plast complete
  if (threadIdx.x == 0) {
    const int C = a.C;
    float m = s_plast[0];
    for (int c = 1; c < C; ++c) m = fmaxf(m, s_plast[c]);
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += __expf(s_plast[c] - m);
    const float lse = m + __logf(se);
    long long lab = a.ce_labels[b];
    lab = lab < 0 ? 0 : (lab >= C ? C - 1 : lab);  // memory safety: the host passes ids in [0, C)
    smi_wt_store(a.ce_row + b, lse - s_plast[lab]);  // read by the last workgroup (smi_common.h)
    const float inv = 1.0f / (float)a.B;
    for (int c = 0; c < C; ++c) a.ce_dlast[(size_t)b * C + c] = (__expf(s_plast[c] - lse) - (c == lab ? 1.f : 0.f)) * inv;
    smi_wt_drain();
    s_lastwg = atomicAdd(a.ce_tick, 1u) == (unsigned)a.B - 1;
  }
  __syncthreads();
  if (s_lastwg && threadIdx.x < 64) {
    float sum = 0.f;
    for (int i = threadIdx.x; i < a.B; i += 64) sum += __hip_atomic_load(a.ce_row + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sum = wave_sum(sum);
    if (threadIdx.x == 0) {
      a.ce_loss[0] = sum / (float)a.B;
      a.ce_tick[0] = 0u;
    }
  }
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
  __shared__ long long s_ids[LSTM_MAXT];
  for (int i = tid; i < T; i += blockDim.x) s_ids[i] = a.ids[(size_t)b * T + i];

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
  __syncthreads();  // s_ids
  // layer-0 input rows, prefetched two ticks ahead (thread e < E owns feature e)
  auto emb_at = [&](int t) { return (tid < E && t < T) ? a.emb[(size_t)s_ids[t] * E + tid] : 0.f; };
  if (tid < E) s_in[0][tid] = emb_at(0);
  // next-tick inputs rotate through three registers (X[(k+1)%3] is written at tick k, X[k%3]
  // reloaded): no register copies, so no wait on a load issued in the same tick
  float x0 = 0.f, x1 = emb_at(1), x2 = emb_at(2);
  __syncthreads();

  const uint32_t seed = smi_seed(a.seedp, a.salt);
  const int gate = r / H;  // 0 i, 1 f, 2 g, 3 o
  float* wsb = a.ws + (size_t)b * L * T * 6 * H;
  const int nt = T + L - 1;
  auto tick = [&](int k, float& xnext, float& xload) {
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
    smi_lds_barrier();
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
    if (tid < E) {  // layer 0's input for the next tick (s_in[0] was consumed before the barrier)
      s_in[0][tid] = xnext;
      xload = emb_at(k + 3);
    }
    smi_lds_barrier();
  };
  int k = 0;
  for (; k + 3 <= nt; k += 3) {
    tick(k, x1, x0);
    tick(k + 1, x2, x1);
    tick(k + 2, x0, x2);
  }
  if (k < nt) tick(k, x1, x0);
  if (k + 1 < nt) tick(k + 1, x2, x1);
  __syncthreads();  // ws (global) written by every cell thread is read by the fc head below
  if (act && r < H) {
    if (a.hn) a.hn[((size_t)l * a.B + b) * H + r] = s_h[l][r];
    if (a.cn) a.cn[((size_t)l * a.B + b) * H + r] = c;
  }
  // fc head at every step, from LDS-staged chunks of the top layer's h (coalesced loads, many in
  // flight; a per-output global dot product would serialise on load latency)
  {
    __shared__ float s_top[LSTM_TCH * H];
    __shared__ float s_wfc[LSTM_MAXC * H];
    __shared__ float s_plast[LSTM_MAXC];
    const float* top = wsb + (size_t)(L - 1) * T * 6 * H + 5 * H;
    for (int i = tid; i < C * H; i += blockDim.x) s_wfc[i] = a.w_fc[i];
    // pred == null (the fused-CE training step, whose loss reads the last step only): the head at
    // the last step alone (the other steps' predictions have no consumer)
    for (int t0 = a.pred ? 0 : T - 1; t0 < T; t0 += LSTM_TCH) {
      const int nc = min(LSTM_TCH, T - t0);
      __syncthreads();
      for (int i = tid; i < nc * H; i += blockDim.x) s_top[i] = top[(size_t)(t0 + i / H) * 6 * H + i % H];
      __syncthreads();
      for (int o = tid; o < nc * C; o += blockDim.x) {
        const int t = o / C, cc = o % C;
        float s0 = a.b_fc[cc], s1 = 0.f;
#pragma unroll
        for (int j = 0; j < H; j += 2) {
          s0 += s_wfc[cc * H + j] * s_top[t * H + j];
          s1 += s_wfc[cc * H + j + 1] * s_top[t * H + j + 1];
        }
        if (a.pred) a.pred[((size_t)b * T + t0 + t) * C + cc] = s0 + s1;
        if (a.pred_last && t0 + t == T - 1) a.pred_last[(size_t)b * C + cc] = s0 + s1;
        if (t0 + t == T - 1) s_plast[cc] = s0 + s1;
      }
    }
    if (a.ce_labels) lstm_ce_tail(a, b, s_plast);
  }
}

// what a cell thread consumes at one backward tick, loaded two ticks ahead (CM >= C head outputs:
// 4 for the reference's 4 classes, so three in-flight sets stay small — register pressure is
// what bounds this kernel's tick)
template <int CM>
struct LstmBwdIn {
  float ig, fg, gg, og, cc, cp;  // raw: loaded two ticks ahead
  float dp[CM];
  float A, Bo, gi, cf, ig2, fct, dm;  // derived one tick ahead (prep), off the dependent chain
};

template <int H, int MI, int NT, int CM>
__global__ __launch_bounds__(NT) void lstm_bwd_kernel(LSTMArgs a) {
  LSTAMP_DECL;
  constexpr int G = 4 * H;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int L = a.L, T = a.T, E = a.E, C = a.C;
  const int l = tid / G, r = tid % G;
  const bool act = l < L;
  const int In = l == 0 ? E : H;
  __shared__ __attribute__((aligned(16))) float s_da[LSTM_MAXL][G];
  __shared__ float s_part[LSTM_MAXL][G];
  __shared__ float s_dhr[LSTM_MAXL][H];
  __shared__ long long s_ids[LSTM_MAXT];
  for (int i = tid; i < T; i += blockDim.x) s_ids[i] = a.ids[(size_t)b * T + i];

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
  const bool cell = act && r < H, top = l == L - 1;
  float wfc[CM];  // head column j (top-layer cell threads)
#pragma unroll
  for (int q = 0; q < CM; ++q) wfc[q] = (cell && top && q < C) ? a.w_fc[(size_t)q * H + r] : 0.f;

  float dc = 0.f;
  if (cell) {
    dc = a.dcn ? a.dcn[((size_t)l * a.B + b) * H + r] : 0.f;
    s_dhr[l][r] = a.dhn ? a.dhn[((size_t)l * a.B + b) * H + r] : 0.f;
  }
  __syncthreads();  // s_ids

  const uint32_t seed = smi_seed(a.seedp, a.salt);
  const float* wsb = a.ws + (size_t)b * L * T * 6 * H;
  // dpred_last: only the last step's head gradient exists ([B][C]; the loss reads pred[:, -1])
  const float* dpred = a.dpred + (size_t)b * (a.dpred_last ? 1 : T) * C;
  const float dps = a.dpred_scale ? a.dpred_scale[0] : 1.f;
  float* dab = a.ws_da + (size_t)b * L * T * G;  // gate gradients of every layer [L][T][4H]
  const int nt = T + L - 1;
  const int tl = T - 1 + (L - 1 - l);  // this layer's step at tick k is tl - k
  auto load_in = [&](int t, LstmBwdIn<CM>& v) {
    if (!cell || t < 0 || t >= T) return;
    const int j = r;
    const float* w = wsb + ((size_t)l * T + t) * 6 * H;
    v.ig = w[j]; v.fg = w[H + j]; v.gg = w[2 * H + j]; v.og = w[3 * H + j]; v.cc = w[4 * H + j];
    v.cp = t > 0 ? w[j - 2 * H] : (a.c0 ? a.c0[((size_t)l * a.B + b) * H + j] : 0.f);
    if (top) {
#pragma unroll
      for (int q = 0; q < CM; ++q)
        v.dp[q] = (q < C && (!a.dpred_last || t == T - 1)) ? dpred[(size_t)(a.dpred_last ? 0 : t) * C + q] * dps : 0.f;
    }
  };
  // everything of step t's cell backward that does not depend on the incoming dh / dc
  auto prep = [&](int t, LstmBwdIn<CM>& v) {
    if (!cell || t < 0 || t >= T) return;
    const float tc = smi_tanh(v.cc);
    v.A = v.og * (1.f - tc * tc);
    v.Bo = tc * v.og * (1.f - v.og);
    v.gi = v.gg * v.ig * (1.f - v.ig);
    v.cf = v.cp * v.fg * (1.f - v.fg);
    v.ig2 = v.ig * (1.f - v.gg * v.gg);
    float f = 0.f;
    if (top) {
#pragma unroll
      for (int q = 0; q < CM; ++q) f += wfc[q] * v.dp[q];
    }
    v.fct = f;
    v.dm = top ? 0.f : (a.thresh ? (smi_keep(seed, lstm_drop_idx(b, t, l, r, T, L, H), a.thresh) ? a.dscale : 0.f) : 1.f);
  };
  // The tick is the recurrence only: cell backward -> da (LDS + global) -> transposed products.
  // The weight gradients dW = sum_t da_t^T [x_t | h_{t-1}] are a GEMM over the saved da after
  // the loop, off the serial critical path.  Per-tick inputs rotate through three register sets
  // (no copies, no same-tick load waits); two LDS barriers per tick, the recurrent dh and the dx
  // handed down by the layer above are read straight from s_part (the previous tick's products).
  LstmBwdIn<CM> ia{}, ib{}, ic{};
  load_in(tl, ia);
  load_in(tl - 1, ib);
  prep(tl, ia);
  auto own_dh = [&](int j) {
    return l >= 1 ? s_part[l][j] + s_part[l][2 * H + j]
                  : (s_part[0][j] + s_part[0][H + j]) + (s_part[0][2 * H + j] + s_part[0][3 * H + j]);
  };
  auto tick = [&](int k, const LstmBwdIn<CM>& cv, LstmBwdIn<CM>& pv, LstmBwdIn<CM>& nv) {
    const int t = tl - k;
    const bool on = act && t >= 0 && t < T;
    long long c_0 = 0, c_1 = 0, c_2 = 0, c_3 = 0, c_4 = 0;
    (void)c_0; (void)c_1; (void)c_2; (void)c_3; (void)c_4;
    LSTAMP_T(c_0);
    load_in(t - 2, nv);  // in flight during this tick and the next
    if (on && r < H) {  // cell backward for unit j = r: a short chain on top of prep()'d terms
      const int j = r;
      float dh = t == T - 1 ? s_dhr[l][j] : own_dh(j);
      dh += top ? cv.fct : (s_part[l + 1][H + j] + s_part[l + 1][3 * H + j]) * cv.dm;  // head / dx from above
      dc += dh * cv.A;
      const float d0 = dc * cv.gi, d1 = dc * cv.cf, d2 = dc * cv.ig2, d3 = dh * cv.Bo;
      s_da[l][j] = d0; s_da[l][H + j] = d1; s_da[l][2 * H + j] = d2; s_da[l][3 * H + j] = d3;
      float* dg = dab + ((size_t)l * T + t) * G;
      dg[j] = d0; dg[H + j] = d1; dg[2 * H + j] = d2; dg[3 * H + j] = d3;
      dc *= cv.fg;
    }
    LSTAMP_T(c_1);
    smi_lds_barrier();
    LSTAMP_T(c_2);
    prep(t - 1, pv);  // next tick's terms (loaded last tick): independent work the compiler
                      // interleaves with the transposed products below
    if (on) {  // transposed products, 8 independent partial sums (short FMA chains)
      float p[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (l == 0) {
#pragma unroll
        for (int q = 0; q < H; q += 8) {
          const float4 d4 = *(const float4*)&s_da[0][row0 + q];
          const float4 e4 = *(const float4*)&s_da[0][row0 + q + 4];
          p[0] += wc[q] * d4.x; p[1] += wc[q + 1] * d4.y; p[2] += wc[q + 2] * d4.z; p[3] += wc[q + 3] * d4.w;
          p[4] += wc[q + 4] * e4.x; p[5] += wc[q + 5] * e4.y; p[6] += wc[q + 6] * e4.z; p[7] += wc[q + 7] * e4.w;
        }
      } else {
#pragma unroll
        for (int q = 0; q < 2 * H; q += 8) {
          const float4 d4 = *(const float4*)&s_da[l][row0 + q];
          const float4 e4 = *(const float4*)&s_da[l][row0 + q + 4];
          p[0] += wc[q] * d4.x; p[1] += wc[q + 1] * d4.y; p[2] += wc[q + 2] * d4.z; p[3] += wc[q + 3] * d4.w;
          p[4] += wc[q + 4] * e4.x; p[5] += wc[q + 5] * e4.y; p[6] += wc[q + 6] * e4.z; p[7] += wc[q + 7] * e4.w;
        }
      }
      s_part[l][r] = ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
    }
    LSTAMP_T(c_3);
    smi_lds_barrier();
    LSTAMP_T(c_4);
    LSTAMP_ADD(threadIdx.x >> 6, 0, c_0, c_1);
    LSTAMP_ADD(threadIdx.x >> 6, 1, c_1, c_2);
    LSTAMP_ADD(threadIdx.x >> 6, 2, c_2, c_3);
    LSTAMP_ADD(threadIdx.x >> 6, 3, c_3, c_4);
  };
  long long cl0 = 0, cl1 = 0;
  (void)cl0; (void)cl1;
  LSTAMP_T(cl0);
  int k = 0;
  for (; k + 3 <= nt; k += 3) {
    tick(k, ia, ib, ic);
    tick(k + 1, ib, ic, ia);
    tick(k + 2, ic, ia, ib);
  }
  if (k < nt) tick(k, ia, ib, ic);
  if (k + 1 < nt) tick(k + 1, ib, ic, ia);
  __syncthreads();  // dab (global) is read across threads below
  LSTAMP_T(cl1);
  LSTAMP_ADD(threadIdx.x >> 6, 4, cl0, cl1);
  LSTAMP_FLUSH(threadIdx.x >> 6);
  if (cell) {
    if (a.dh0) a.dh0[((size_t)l * a.B + b) * H + r] = own_dh(r);  // W_hh^T da at t = 0
    if (a.dc0) a.dc0[((size_t)l * a.B + b) * H + r] = dc;
  }

}

// ---- two-wave recurrence (L * H <= 64 and In + H <= 64: the reference's H = 32, L = 2) --------
//
// The tick above costs ~2.5k cycles, almost all of it LDS round trips behind TWO workgroup
// barriers (gate exchange, then the cell update's h exchange).  Here lane (l, j) of a 64-lane
// wave owns unit j of layer l, and the workgroup is just two waves: wave w owns the gate pair
// {2w, 2w + 1} (w = 0: i, f; w = 1: g, o), i.e. 2 x (In + H) <= 128 fp32 weights per lane, held in
// VGPRs and accumulated with packed v_pk_fma_f32.  After the single barrier that exchanges the
// gate pairs BOTH waves run the (cheap) cell update redundantly and write h / the dropped-out
// layer input into their OWN LDS copy, which only the same wave reads at the next tick — in-order
// LDS within a wave needs no barrier — so a tick has exactly one barrier.  The backward is the
// same shape: both waves run the cell backward redundantly into their own da copy; wave 0 forms
// dh_{t-1} = W_hh^T da (its lane holds W_hh column j), wave 1 forms dx_t = W_ih^T da for the
// layer below (column j of W_ih), one barrier hands them over.
//
// Why not MFMA for the gate products: per tick and layer they are [32 seq x 64] x [64 x 128];
// fp32-exact through the 3-plane bf16 split that is 6 x 4 k-steps x 4 tiles = 96
// v_mfma_f32_32x32x16_bf16 per layer per tick (~1.5k cycles on one CU for the batch), while the
// same products spread over one CU per sequence are ~128 cycles of packed fp32 VALU.  The
// recurrence is a latency chain; batching it onto the matrix cores lengthens the chain.
typedef float smi_f2 __attribute__((ext_vector_type(2)));
#define SMI_WAVE_LDS_ORDER() asm volatile("" ::: "memory")  // compiler order only: LDS is in-order per wave

// Workgroups B .. of the forward launch (LSTMArgs::emb_side): the pair-compare ordering of the
// B x T ids for the embedding backward, on CUs the B recurrence workgroups leave idle (it ran
// serialised after the forward as its own launches, 24 us of the step).  Each takes a tile of 64
// tokens; the last to finish (ticket, write-through hand-off) builds the plan in LDS.
__device__ __forceinline__ void lstm_emb_side(const LSTMArgs& a) {
  __shared__ __attribute__((aligned(16))) int s_id[LSTM_EMB_MAX];
  __shared__ int s_cnt[2][64], s_min[2][64];
  __shared__ int s_f[LSTM_EMB_MAX], s_off[LSTM_EMB_MAX], s_coff[LSTM_EMB_MAX];
  __shared__ int s_wsum[2][2];
  __shared__ int s_last;
  const long T = (long)a.B * a.T;
  const EmbPair e = emb_pair_layout(a.emb_ws, T);
  const int ntile = (int)((T + 63) / 64);
  emb_pair_rank_tile<128, true>(a.ids, T, a.pad_idx, e, (blockIdx.x - a.B) * 64, s_id, s_cnt, s_min);
  smi_wt_drain();
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(a.emb_tick, 1u) == (unsigned)ntile - 1;
  __syncthreads();
  if (!s_last) return;
  emb_pair_plan_body<128, true>(T, e, s_f, s_off, s_coff, s_wsum);
  if (threadIdx.x == 0) a.emb_tick[0] = 0u;
}

template <int H, int MI>
__global__ __launch_bounds__(128) void lstm_fwd_w2_kernel(LSTMArgs a) {
  if ((int)blockIdx.x >= a.B) {  // the embedding-backward ordering workgroups (uniform)
    lstm_emb_side(a);
    return;
  }
  LSTAMP_DECL;
  const int b = blockIdx.x, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int L = a.L, T = a.T, E = a.E, C = a.C;
  const int l = lane / H, j = lane % H;
  const bool act = l < L;
  const int In = l == 0 ? E : H;
  constexpr int SI = MI + 4, SH = H + 4;  // padded rows: the L broadcast rows of a read hit distinct banks
  __shared__ __attribute__((aligned(16))) float s_in[2][2][LSTM_MAXL * SI];  // [wave][buf][layer row]
  __shared__ __attribute__((aligned(16))) float s_h[2][2][LSTM_MAXL * SH];
  __shared__ float s_g[2][LSTM_MAXL][4][H];                                // [buf][layer][gate][unit]
  __shared__ long long s_ids[LSTM_MAXT];
  // layer 0's inputs (embedding rows) for two windows of LSTM_XW ticks, refilled half a window
  // ahead: the tick loop issues no per-tick global load, so its per-tick stores of the saved
  // activations never sit in front of a load the tick waits for (gfx9 vmcnt counts both, in order)
  constexpr int XW = LSTM_XW, NX = XW * MI / 128;  // window ticks, values per thread per window
  static_assert((XW * MI) % 128 == 0, "whole window per 128 threads");
  __shared__ __attribute__((aligned(16))) float s_x[2][XW][SI];
  for (int i = tid; i < T; i += blockDim.x) s_ids[i] = a.ids[(size_t)b * T + i];

  const int g0 = 2 * w, g1 = 2 * w + 1;
  smi_f2 wi0[MI / 2], wi1[MI / 2], wh0[H / 2], wh1[H / 2];
#pragma unroll
  for (int i = 0; i < MI; i += 2) {
    const float* r0 = a.w_ih[act ? l : 0] + (size_t)(g0 * H + j) * In;
    const float* r1 = a.w_ih[act ? l : 0] + (size_t)(g1 * H + j) * In;
    wi0[i / 2] = smi_f2{(act && i < In) ? r0[i] : 0.f, (act && i + 1 < In) ? r0[i + 1] : 0.f};
    wi1[i / 2] = smi_f2{(act && i < In) ? r1[i] : 0.f, (act && i + 1 < In) ? r1[i + 1] : 0.f};
  }
#pragma unroll
  for (int i = 0; i < H; i += 2) {
    const float* r0 = a.w_hh[act ? l : 0] + (size_t)(g0 * H + j) * H;
    const float* r1 = a.w_hh[act ? l : 0] + (size_t)(g1 * H + j) * H;
    wh0[i / 2] = act ? smi_f2{r0[i], r0[i + 1]} : smi_f2{0.f, 0.f};
    wh1[i / 2] = act ? smi_f2{r1[i], r1[i + 1]} : smi_f2{0.f, 0.f};
  }
  const float bias0 = act ? a.b_ih[l][g0 * H + j] + a.b_hh[l][g0 * H + j] : 0.f;
  const float bias1 = act ? a.b_ih[l][g1 * H + j] + a.b_hh[l][g1 * H + j] : 0.f;
  for (int i = tid; i < 2 * 2 * LSTM_MAXL * SI; i += blockDim.x) (&s_in[0][0][0])[i] = 0.f;
  float c = 0.f, hl = 0.f;
  __syncthreads();
  if (act) {
    c = a.c0 ? a.c0[((size_t)l * a.B + b) * H + j] : 0.f;
    hl = a.h0 ? a.h0[((size_t)l * a.B + b) * H + j] : 0.f;
    s_h[w][0][l * SH + j] = hl;  // a layer reads h_{-1} from the buffer of its first tick: both
    s_h[w][1][l * SH + j] = hl;
  }
  __syncthreads();  // s_ids
  // window loads: unconditional (clamped) so that no select waits on them at issue; the mask
  // (columns >= E, ticks >= T) is applied when the window is written to LDS, half a window later
  float xr[NX];
  auto win_load = [&](int t0) {
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int e = (tid + 128 * i) % MI, tt = (tid + 128 * i) / MI;
      xr[i] = a.emb[(size_t)s_ids[min(t0 + tt, T - 1)] * E + min(e, E - 1)];
    }
  };
  auto win_store = [&](int t0, int buf) {
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int e = (tid + 128 * i) % MI, tt = (tid + 128 * i) / MI;
      s_x[buf][tt][e] = (e < E && t0 + tt < T) ? xr[i] : 0.f;
    }
  };
  win_load(0);
  win_store(0, 0);
  if (XW < T) win_load(XW);
  __syncthreads();

  const uint32_t seed = smi_seed(a.seedp, a.salt);
  float* wsb = a.ws + (size_t)b * L * T * 6 * H;
  const int nt = T + L - 1;
  // every prologue load (weights, h0 / c0) retired here, so the tick loop's wait counts are exact
  __builtin_amdgcn_s_waitcnt(0);
  auto tick = [&](int k) {
    const int t = k - l;
    const bool on = act && t >= 0 && t < T;
    const int rb = k & 1, wb = rb ^ 1;
    long long c_0 = 0, c_1 = 0, c_2 = 0, c_3 = 0;
    (void)c_0; (void)c_1; (void)c_2; (void)c_3;
    LSTAMP_T(c_0);
    if (on) {
      // eight independent packed-FMA chains (two per gate and input half, input rows and h rows
      // apart): four chains of 16 dependent v_pk_fma_f32 left the gate phase latency-bound
      smi_f2 p0 = {bias0, 0.f}, q0 = {0.f, 0.f}, p1 = {bias1, 0.f}, q1 = {0.f, 0.f};
      smi_f2 r0 = {0.f, 0.f}, u0 = {0.f, 0.f}, r1 = {0.f, 0.f}, u1 = {0.f, 0.f};
      const float* xin = l == 0 ? &s_x[(t / XW) & 1][t % XW][0] : &s_in[w][rb][l * SI];
      const float* hin = &s_h[w][rb][l * SH];
#pragma unroll
      for (int i = 0; i < MI; i += 4) {
        const float4 x = *(const float4*)&xin[i];
        const smi_f2 xa = {x.x, x.y}, xb = {x.z, x.w};
        p0 = __builtin_elementwise_fma(wi0[i / 2], xa, p0);
        q0 = __builtin_elementwise_fma(wi0[i / 2 + 1], xb, q0);
        p1 = __builtin_elementwise_fma(wi1[i / 2], xa, p1);
        q1 = __builtin_elementwise_fma(wi1[i / 2 + 1], xb, q1);
      }
#pragma unroll
      for (int i = 0; i < H; i += 4) {
        const float4 x = *(const float4*)&hin[i];
        const smi_f2 xa = {x.x, x.y}, xb = {x.z, x.w};
        r0 = __builtin_elementwise_fma(wh0[i / 2], xa, r0);
        u0 = __builtin_elementwise_fma(wh0[i / 2 + 1], xb, u0);
        r1 = __builtin_elementwise_fma(wh1[i / 2], xa, r1);
        u1 = __builtin_elementwise_fma(wh1[i / 2 + 1], xb, u1);
      }
      const float z0 = ((p0.x + p0.y) + (q0.x + q0.y)) + ((r0.x + r0.y) + (u0.x + u0.y));
      const float z1 = ((p1.x + p1.y) + (q1.x + q1.y)) + ((r1.x + r1.y) + (u1.x + u1.y));
      s_g[rb][l][g0][j] = w == 1 ? smi_tanh(z0) : smi_sigmoid(z0);  // gate 2 (g) is the tanh one
      s_g[rb][l][g1][j] = smi_sigmoid(z1);
    }
    LSTAMP_T(c_1);
    smi_lds_barrier();
    LSTAMP_T(c_2);
    if (on) {
      const float ig = s_g[rb][l][0][j], fg = s_g[rb][l][1][j], gg = s_g[rb][l][2][j], og = s_g[rb][l][3][j];
      c = fg * c + ig * gg;
      hl = og * smi_tanh(c);
      s_h[w][wb][l * SH + j] = hl;
      if (l + 1 < L) {
        float hd = hl;
        if (a.thresh) hd = smi_keep(seed, lstm_drop_idx(b, t, l, j, T, L, H), a.thresh) ? hl * a.dscale : 0.f;
        s_in[w][wb][(l + 1) * SI + j] = hd;
      }
      float* ws = wsb + ((size_t)l * T + t) * 6 * H;  // saved activations: i f g (wave 0), o c h (wave 1)
      if (w == 0) { ws[j] = ig; ws[H + j] = fg; ws[2 * H + j] = gg; }
      else { ws[3 * H + j] = og; ws[4 * H + j] = c; ws[5 * H + j] = hl; }
    }
    SMI_WAVE_LDS_ORDER();
    LSTAMP_T(c_3);
    LSTAMP_ADD(w, 0, c_0, c_1);  // gates: LDS reads, packed FMAs, activations
    LSTAMP_ADD(w, 1, c_1, c_2);  // the barrier
    LSTAMP_ADD(w, 2, c_2, c_3);  // cell update, LDS writes, prefetch
    long long c_4 = 0, c_5 = 0;
    (void)c_4; (void)c_5;
    LSTAMP_T(c_4);
    if (k % XW == XW / 2) {  // mid-window: window w + 1 into LDS (its buffer last held w - 1), load w + 2
      const int wn = k / XW + 1;
      if (wn * XW < T) {
        win_store(wn * XW, wn & 1);  // read from tick wn * XW on: many barriers later
        if ((wn + 1) * XW < T) win_load((wn + 1) * XW);
      }
    }
    LSTAMP_T(c_5);
    LSTAMP_ADD(w, 3, c_3, c_4);  // stamp bookkeeping
    LSTAMP_ADD(w, 4, c_4, c_5);  // window refill (every LSTM_XW ticks)
  };
  int k = 0;
#ifdef LSTM_STAMPS
  unsigned long long rt0 = __builtin_amdgcn_s_memrealtime(), ct0 = __builtin_amdgcn_s_memtime();
#endif
  for (; k < nt; ++k) tick(k);
#ifdef LSTM_STAMPS
  if (tid == 0 && b == 0) {
    lstm_rt[0] += __builtin_amdgcn_s_memrealtime() - rt0;
    lstm_rt[2] += __builtin_amdgcn_s_memtime() - ct0;
  }
#endif
  LSTAMP_FLUSH(w);
  __syncthreads();  // ws (global) written by both waves is read by the fc head below
  if (act && w == 0) {
    if (a.hn) a.hn[((size_t)l * a.B + b) * H + j] = hl;
    if (a.cn) a.cn[((size_t)l * a.B + b) * H + j] = c;
  }
  {
    __shared__ float s_top[LSTM_TCH * H];
    __shared__ float s_wfc[LSTM_MAXC * H];
    __shared__ float s_plast[LSTM_MAXC];
    const float* top = wsb + (size_t)(L - 1) * T * 6 * H + 5 * H;
    for (int i = tid; i < C * H; i += blockDim.x) s_wfc[i] = a.w_fc[i];
    // pred == null (the fused-CE training step, whose loss reads the last step only): the head at
    // the last step alone (the other steps' predictions have no consumer)
    for (int t0 = a.pred ? 0 : T - 1; t0 < T; t0 += LSTM_TCH) {
      const int nc = min(LSTM_TCH, T - t0);
      __syncthreads();
      for (int i = tid; i < nc * H; i += blockDim.x) s_top[i] = top[(size_t)(t0 + i / H) * 6 * H + i % H];
      __syncthreads();
      for (int o = tid; o < nc * C; o += blockDim.x) {
        const int t = o / C, cc = o % C;
        float s0 = a.b_fc[cc], s1 = 0.f;
#pragma unroll
        for (int q = 0; q < H; q += 2) {
          s0 += s_wfc[cc * H + q] * s_top[t * H + q];
          s1 += s_wfc[cc * H + q + 1] * s_top[t * H + q + 1];
        }
        if (a.pred) a.pred[((size_t)b * T + t0 + t) * C + cc] = s0 + s1;
        if (a.pred_last && t0 + t == T - 1) a.pred_last[(size_t)b * C + cc] = s0 + s1;
        if (t0 + t == T - 1) s_plast[cc] = s0 + s1;
      }
    }
    if (a.ce_labels) lstm_ce_tail(a, b, s_plast);
  }
}

template <int H, int MI, int CM>
__global__ __launch_bounds__(128) void lstm_bwd_w2_kernel(LSTMArgs a) {
  LSTAMP_DECL;
  constexpr int G = 4 * H;
  const int b = blockIdx.x, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int L = a.L, T = a.T, C = a.C;
  const int l = lane / H, j = lane % H;
  const bool act = l < L, top = l == L - 1;
  __shared__ __attribute__((aligned(16))) float s_da[2][LSTM_MAXL][G + 4];  // per-wave copy
  __shared__ float s_dh[2][LSTM_MAXL][H];  // [buf]: W_hh^T da (wave 0)
  __shared__ float s_dx[2][LSTM_MAXL][H];  // [buf]: W_ih^T da, the layer below's input gradient (wave 1)
  // gate gradients of the last LSTM_WCH ticks [tick % LSTM_WCH][layer][4H], burst-stored (no global
  // store inside the tick: it would share vmcnt with the prefetched workspace loads)
  __shared__ __attribute__((aligned(16))) float s_dab[LSTM_WCH][(64 / H) * G];
  // wave 0: column j of W_hh[l]; wave 1: column j of W_ih[l] (l >= 1: In = H; layer 0's input
  // gradient is lstm_xe_kernel's job after the loop)
  const bool prod = act && (w == 0 || l >= 1);
  smi_f2 wc[G / 2];
#pragma unroll
  for (int q = 0; q < G; q += 2) {
    const float* m = w == 0 ? a.w_hh[act ? l : 0] : a.w_ih[act ? l : 0];
    wc[q / 2] = prod ? smi_f2{m[(size_t)q * H + j], m[(size_t)(q + 1) * H + j]} : smi_f2{0.f, 0.f};
  }
  float wfc[CM];
#pragma unroll
  for (int q = 0; q < CM; ++q) wfc[q] = (act && top && q < C) ? a.w_fc[(size_t)q * H + j] : 0.f;
  float dc = 0.f, dhn = 0.f;
  if (act) {
    dc = a.dcn ? a.dcn[((size_t)l * a.B + b) * H + j] : 0.f;
    dhn = a.dhn ? a.dhn[((size_t)l * a.B + b) * H + j] : 0.f;
  }
  for (int i = tid; i < 2 * LSTM_MAXL * H; i += blockDim.x) (&s_dx[0][0][0])[i] = 0.f;
  __syncthreads();

  const uint32_t seed = smi_seed(a.seedp, a.salt);
  const float* wsb = a.ws + (size_t)b * L * T * 6 * H;
  const float* dpred = a.dpred + (size_t)b * (a.dpred_last ? 1 : T) * C;
  float* dab = a.ws_da + (size_t)b * L * T * G;
  const int nt = T + L - 1;
  const int tl = T - 1 + (L - 1 - l);
  const float c0v = (act && a.c0) ? a.c0[((size_t)l * a.B + b) * H + j] : 0.f;
  float dpl[CM];
  const float dps = a.dpred_scale ? a.dpred_scale[0] : 1.f;
#pragma unroll
  for (int q = 0; q < CM; ++q) dpl[q] = (a.dpred_last && top && q < C) ? dpred[min(q, C - 1)] * dps : 0.f;
  // every lane loads every value at clamped indices (no branch around a load: the compiler can
  // then count vmcnt exactly instead of waiting for everything in flight)
  auto load_in = [&](int t, LstmBwdIn<CM>& v) {
    const int tc = min(max(t, 0), T - 1);
    const float* ws = wsb + ((size_t)(act ? l : L - 1) * T + tc) * 6 * H;
    v.ig = ws[j]; v.fg = ws[H + j]; v.gg = ws[2 * H + j]; v.og = ws[3 * H + j]; v.cc = ws[4 * H + j];
    const float cpv = ws[(tc > 0 ? -2 * H : 4 * H) + j];  // c at t - 1 (t = 0: c0)
    v.cp = t > 0 ? cpv : c0v;
    if (a.dpred_last) {  // the last step's dpred only: loaded once before the loop
#pragma unroll
      for (int q = 0; q < CM; ++q) v.dp[q] = t == T - 1 ? dpl[q] : 0.f;
    } else {
#pragma unroll
      for (int q = 0; q < CM; ++q) {
        const float d = dpred[(size_t)tc * C + min(q, C - 1)] * dps;
        v.dp[q] = (top && q < C) ? d : 0.f;
      }
    }
  };
  auto prep = [&](int t, LstmBwdIn<CM>& v) {
    if (!act || t < 0 || t >= T) return;
    const float tc = smi_tanh(v.cc);
    v.A = v.og * (1.f - tc * tc);
    v.Bo = tc * v.og * (1.f - v.og);
    v.gi = v.gg * v.ig * (1.f - v.ig);
    v.cf = v.cp * v.fg * (1.f - v.fg);
    v.ig2 = v.ig * (1.f - v.gg * v.gg);
    float f = 0.f;
    if (top) {
#pragma unroll
      for (int q = 0; q < CM; ++q) f += wfc[q] * v.dp[q];
    }
    v.fct = f;
    v.dm = top ? 0.f : (a.thresh ? (smi_keep(seed, lstm_drop_idx(b, t, l, j, T, L, H), a.thresh) ? a.dscale : 0.f) : 1.f);
  };
  LstmBwdIn<CM> ia{}, ib{}, ic{};
  load_in(tl, ia);
  load_in(tl - 1, ib);
  prep(tl, ia);
  __builtin_amdgcn_s_waitcnt(0);  // prologue loads retired: exact wait counts in the tick loop
  float dh_first = 0.f;  // W_hh^T da at t = 0 (wave 0): the gradient of h0
  auto tick = [&](int k, const LstmBwdIn<CM>& cv, LstmBwdIn<CM>& pv, LstmBwdIn<CM>& nv) {
    const int t = tl - k;
    const bool on = act && t >= 0 && t < T;
    const int rb = k & 1, wb = rb ^ 1;
    long long c_0 = 0, c_1 = 0, c_2 = 0, c_3 = 0, c_4 = 0;
    (void)c_0; (void)c_1; (void)c_2; (void)c_3; (void)c_4;
    LSTAMP_T(c_0);
    load_in(t - 2, nv);
    if (on) {  // cell backward (both waves, bit-identical) on terms prep()'d a tick ahead
      float dh = t == T - 1 ? dhn : s_dh[rb][l][j];
      dh += top ? cv.fct : s_dx[rb][l + 1][j] * cv.dm;
      dc += dh * cv.A;
      const float d0 = dc * cv.gi, d1 = dc * cv.cf, d2 = dc * cv.ig2, d3 = dh * cv.Bo;
      s_da[w][l][j] = d0; s_da[w][l][H + j] = d1; s_da[w][l][2 * H + j] = d2; s_da[w][l][3 * H + j] = d3;
      float* dg = &s_dab[k & (LSTM_WCH - 1)][l * G];
      if (w == 0) { dg[j] = d0; dg[H + j] = d1; }
      else { dg[2 * H + j] = d2; dg[3 * H + j] = d3; }
      dc *= cv.fg;
    }
    SMI_WAVE_LDS_ORDER();
    LSTAMP_T(c_1);
    prep(t - 1, pv);
    if (on && prod) {  // this wave's transposed product over the layer's 4H gate gradients
      smi_f2 p0 = {0.f, 0.f}, p1 = {0.f, 0.f}, p2 = {0.f, 0.f}, p3 = {0.f, 0.f};
      const float* da = &s_da[w][l][0];
      // two rounds of G / 8 LDS reads issued back to back before their FMAs (the interleaved form
      // kept 2-3 reads in flight: ~32 exposed LDS latencies, most of the 1.3k-cycle product);
      // same accumulation order
#pragma unroll
      for (int hq = 0; hq < G; hq += G / 2) {
        float4 dv[G / 8];
#pragma unroll
        for (int i = 0; i < G / 8; ++i) dv[i] = *(const float4*)&da[hq + 4 * i];
#pragma unroll
        for (int i = 0; i < G / 8; i += 2) {
          const int q = hq + 4 * i;
          p0 = __builtin_elementwise_fma(wc[q / 2], smi_f2{dv[i].x, dv[i].y}, p0);
          p1 = __builtin_elementwise_fma(wc[q / 2 + 1], smi_f2{dv[i].z, dv[i].w}, p1);
          p2 = __builtin_elementwise_fma(wc[q / 2 + 2], smi_f2{dv[i + 1].x, dv[i + 1].y}, p2);
          p3 = __builtin_elementwise_fma(wc[q / 2 + 3], smi_f2{dv[i + 1].z, dv[i + 1].w}, p3);
        }
      }
      const float s = ((p0.x + p0.y) + (p1.x + p1.y)) + ((p2.x + p2.y) + (p3.x + p3.y));
      if (w == 0) {
        s_dh[wb][l][j] = s;
        if (t == 0) dh_first = s;
      } else {
        s_dx[wb][l][j] = s;
      }
    }
    LSTAMP_T(c_2);
    smi_lds_barrier();
    LSTAMP_T(c_3);
    if ((k & (LSTM_WCH - 1)) == LSTM_WCH - 1 || k == nt - 1) {  // burst the staged gate gradients
      const int k0 = k & ~(LSTM_WCH - 1), rows = (k - k0 + 1) * L;
      constexpr int R4 = G / 4;
      for (int e = tid; e < rows * R4; e += blockDim.x) {
        const int r = e / R4, c4 = e - r * R4, kk = k0 + r / L, ll = r % L, tt = T - 1 + (L - 1 - ll) - kk;
        if (tt >= 0 && tt < T)
          *(float4*)(dab + ((size_t)ll * T + tt) * G + 4 * c4) = *(const float4*)&s_dab[kk & (LSTM_WCH - 1)][ll * G + 4 * c4];
      }
      __syncthreads();  // the next tick overwrites slot 0
    }
    LSTAMP_T(c_4);
    LSTAMP_ADD(w, 5, c_0, c_1);  // load issue (waits on the loads of two ticks ago) + cell backward
    LSTAMP_ADD(w, 6, c_1, c_2);  // prep of the next tick + transposed product
    LSTAMP_ADD(w, 7, c_2, c_3);  // barrier
    LSTAMP_ADD(w, 3, c_3, c_4);  // burst flush (every LSTM_WCH ticks)
  };
  int k = 0;
  for (; k + 3 <= nt; k += 3) {
    tick(k, ia, ib, ic);
    tick(k + 1, ib, ic, ia);
    tick(k + 2, ic, ia, ib);
  }
  if (k < nt) tick(k, ia, ib, ic);
  if (k + 1 < nt) tick(k + 1, ib, ic, ia);
  LSTAMP_FLUSH(2 + w);
  __syncthreads();  // dab (global) is read across workgroups by the weight-gradient kernels (next launch)
  if (act && w == 0) {
    if (a.dh0) a.dh0[((size_t)l * a.B + b) * H + j] = dh_first;
    if (a.dc0) a.dc0[((size_t)l * a.B + b) * H + j] = dc;
  }
}

// ---- weight gradients, off the recurrence: for every layer l,
//   [dW_ih | dW_hh | db][r, :] = sum_{b,t} da[b,l,t,r] * [x_t | h_{t-1} | 1]
// and for the head [dW_fc | db_fc][c, :] = sum_{b,t} dpred[b,t,c] * [h_top(t) | 1].
// The B*T (b,t) reduction is split into LSTM_KS fixed chunks; workgroup (chunk, row block, layer)
// writes its partial tile, lstm_wgrad_combine sums the chunks in order (bit-reproducible) into
// the gradient buffers.  128+ workgroups instead of the recurrence kernel's 32 doing it serially.
#define LSTM_KS 64
#define LSTM_RB 32    // gate rows per workgroup
#define LSTM_WC 72    // padded columns (In + H + 1 <= 129 handled in column passes)
#define LSTM_KSUB 64  // (b,t) rows staged per LDS round

__host__ __device__ __forceinline__ int lstm_cols(const LSTMArgs& a, int l) {
  return l < a.L ? (l == 0 ? a.E : a.H) + a.H + 1 : a.H + 1;
}
__host__ __device__ __forceinline__ int lstm_rows(const LSTMArgs& a, int l) { return l < a.L ? 4 * a.H : a.C; }
// partial-tile scratch offset of (layer l, chunk s): [l][s][rows][cols]
__host__ __device__ __forceinline__ long lstm_part_off(const LSTMArgs& a, int l, int s) {
  long off = 0;
  for (int i = 0; i < l; ++i) off += (long)LSTM_KS * lstm_rows(a, i) * lstm_cols(a, i);
  return off + (long)s * lstm_rows(a, l) * lstm_cols(a, l);
}

__global__ __launch_bounds__(256) void lstm_wgrad_partial(LSTMArgs a) {
  const int s = blockIdx.x, rb = blockIdx.y, l = blockIdx.z;
  const int L = a.L, T = a.T, H = a.H, E = a.E, C = a.C, G = 4 * H;
  const int rows = lstm_rows(a, l), cols = lstm_cols(a, l);
  const int r0 = rb * LSTM_RB;
  if (r0 >= rows) return;  // uniform per workgroup
  const int nr = min(LSTM_RB, rows - r0);
  const long BT = (long)a.B * T, kc = (BT + LSTM_KS - 1) / LSTM_KS;
  const long k0 = (long)s * kc, k1 = min(BT, k0 + kc);
  __shared__ float s_d[LSTM_KSUB][LSTM_RB];
  __shared__ float s_x[LSTM_KSUB][LSTM_WC + 1];
  const int tid = threadIdx.x, ri = tid >> 3, cg = tid & 7;
  const uint32_t seed = smi_seed(a.seedp, a.salt);
  for (int c0 = 0; c0 < cols; c0 += LSTM_WC) {  // column passes of LSTM_WC
    const int ncol = min(LSTM_WC, cols - c0);
    float acc[LSTM_WC / 8];
#pragma unroll
    for (int m = 0; m < LSTM_WC / 8; ++m) acc[m] = 0.f;
    for (long kb = k0; kb < k1; kb += LSTM_KSUB) {
      const int nk = (int)min((long)LSTM_KSUB, k1 - kb);
      __syncthreads();
      for (int i = tid; i < nk * LSTM_RB; i += 256) {
        const int kk = i / LSTM_RB, rr = i % LSTM_RB;
        const long bt = kb + kk;
        const int b = (int)(bt / T), t = (int)(bt % T);
        float v = 0.f;
        if (rr < nr) {
          if (l < L) v = a.ws_da[(((size_t)b * L + l) * T + t) * G + r0 + rr];
          else if (!a.dpred_last) v = a.dpred[((size_t)b * T + t) * C + r0 + rr];
          else v = t == T - 1 ? a.dpred[(size_t)b * C + r0 + rr] : 0.f;
          if (l == L && a.dpred_scale) v *= a.dpred_scale[0];
        }
        s_d[kk][rr] = v;
      }
      for (int i = tid; i < nk * LSTM_WC; i += 256) {
        const int kk = i / LSTM_WC, cc = i % LSTM_WC, c = c0 + cc;
        const long bt = kb + kk;
        const int b = (int)(bt / T), t = (int)(bt % T);
        const float* wsb = a.ws + (size_t)b * L * T * 6 * H;
        float v = 0.f;
        if (c < cols) {
          if (l == L) {  // head: [h_top(t) | 1]
            v = c < H ? wsb[((size_t)(L - 1) * T + t) * 6 * H + 5 * H + c] : 1.f;
          } else {
            const int In = l == 0 ? E : H;
            if (c < In) {  // x_t: embedding row, or the (dropped-out) output of the layer below
              if (l == 0) v = a.emb[(size_t)a.ids[(size_t)b * T + t] * E + c];
              else {
                const float hx = wsb[((size_t)(l - 1) * T + t) * 6 * H + 5 * H + c];
                v = a.thresh ? (smi_keep(seed, lstm_drop_idx(b, t, l - 1, c, T, L, H), a.thresh) ? hx * a.dscale : 0.f)
                             : hx;
              }
            } else if (c < In + H) {  // h_{t-1}
              const int j = c - In;
              v = t > 0 ? wsb[((size_t)l * T + t - 1) * 6 * H + 5 * H + j] : (a.h0 ? a.h0[((size_t)l * a.B + b) * H + j] : 0.f);
            } else {
              v = 1.f;  // bias column
            }
          }
        }
        s_x[kk][cc] = v;
      }
      __syncthreads();
      for (int kk = 0; kk < nk; ++kk) {
        const float d = s_d[kk][ri];
#pragma unroll
        for (int m = 0; m < LSTM_WC / 8; ++m) acc[m] += d * s_x[kk][cg + 8 * m];
      }
    }
    if (ri < nr) {
      float* out = a.g_slab + lstm_part_off(a, l, s) + (size_t)(r0 + ri) * cols + c0;
#pragma unroll
      for (int m = 0; m < LSTM_WC / 8; ++m)
        if (cg + 8 * m < ncol) out[cg + 8 * m] = acc[m];
    }
  }
}

__global__ __launch_bounds__(256) void lstm_wgrad_combine(LSTMArgs a) {
  const int l = blockIdx.y;
  const int rows = lstm_rows(a, l), cols = lstm_cols(a, l);
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= (long)rows * cols) return;
  const int r = (int)(p / cols), c = (int)(p % cols);
  float v = 0.f;
  for (int s = 0; s < LSTM_KS; ++s) v += a.g_slab[lstm_part_off(a, l, s) + p];  // chunk order
  if (l == a.L) {
    if (c < a.H) a.g_w_fc[(size_t)r * a.H + c] += v;
    else a.g_b_fc[r] += v;
    return;
  }
  const int In = l == 0 ? a.E : a.H;
  if (c < In) a.g_w_ih[l][(size_t)r * In + c] += v;
  else if (c < In + a.H) a.g_w_hh[l][(size_t)r * a.H + (c - In)] += v;
  else {
    a.g_b_ih[l][r] += v;
    a.g_b_hh[l][r] += v;
  }
}

// ONE launch for every weight gradient of the stack (layers + head) AND the embedding-input
// gradients xe, on the fp32 matrix cores: v_mfma_f32_16x16x4_f32 (exact fp32 products, an fmaf
// chain per accumulator — the reference's fp32 precision).
//   dW_l[r][c] = sum over all B*T (b,t) of da_l[b,t][r] * x_l[b,t][c]   (x = [input | h_{t-1} | 1])
//   xe[b,t][e] = sum_r da_0[b,t][r] * W_ih0[r][e]
// Workgroup (chunk s, column tile ct, layer l): its (b,t) range is staged through LDS in rounds of
// LW_KR rows with every load of a round in flight at once (a per-lane gather loop was latency-
// bound: 117 us), wave w accumulates row tile w of the 16-column slice over the whole range, the
// partial tile goes to the slab, and the LAST of the nch chunk workgroups of (l, ct) — a ticket
// per column tile — sums the nch partials in chunk order (bit-reproducible, no float atomics, no
// second launch).  The (chunk, ct = 0, l = 0) workgroups also turn their staged da_0 rows into xe
// rows against W_ih0 (staged once).  Operand layouts (16x16x4 f32): lane l holds A row / B column
// l & 15 at k = l >> 4; the accumulator's register j of lane l is row 4 (l >> 4) + j, column l & 15.
#define LW_WAVES 8
#define LW_KR 64    // (b,t) rows per LDS round
#define LW_PD 144   // s_d pitch: >= 4H (128); == 16 mod 64 -> the 4 k-rows of an A read hit distinct banks
#define LW_PW 48    // s_w pitch (E <= 32)
__device__ __forceinline__ float lw_d(const LSTMArgs& a, int l, int b, int t, int r, int rows) {
  if (r >= rows) return 0.f;
  if (l < a.L) return a.ws_da[(((size_t)b * a.L + l) * a.T + t) * 4 * a.H + r];
  const float ds = a.dpred_scale ? a.dpred_scale[0] : 1.f;
  if (!a.dpred_last) return a.dpred[((size_t)b * a.T + t) * a.C + r] * ds;
  return t == a.T - 1 ? a.dpred[(size_t)b * a.C + r] * ds : 0.f;
}
__device__ __forceinline__ float lw_x(const LSTMArgs& a, int l, int b, int t, int c, int cols, uint32_t seed) {
  if (c >= cols) return 0.f;
  const int H = a.H, L = a.L, T = a.T;
  const float* wsb = a.ws + (size_t)b * L * T * 6 * H;
  if (l == L) return c < H ? wsb[((size_t)(L - 1) * T + t) * 6 * H + 5 * H + c] : 1.f;
  const int In = l == 0 ? a.E : H;
  if (c < In) {
    if (l == 0) return a.emb[(size_t)a.ids[(size_t)b * T + t] * a.E + c];
    const float hx = wsb[((size_t)(l - 1) * T + t) * 6 * H + 5 * H + c];
    return a.thresh ? (smi_keep(seed, lstm_drop_idx(b, t, l - 1, c, T, L, H), a.thresh) ? hx * a.dscale : 0.f) : hx;
  }
  if (c < In + H) {
    const int j = c - In;
    return t > 0 ? wsb[((size_t)l * T + t - 1) * 6 * H + 5 * H + j] : (a.h0 ? a.h0[((size_t)l * a.B + b) * H + j] : 0.f);
  }
  return 1.f;
}
// chunks of the (b,t) reduction: one per ~2 LDS rounds, at most LSTM_KS (the slab's capacity)
static inline int lw_chunks(const LSTMArgs& a) {
  const long BT = (long)a.B * a.T;
  const long n = (BT + 2 * LW_KR - 1) / (2 * LW_KR);
  return (int)(n < 1 ? 1 : (n > LSTM_KS ? LSTM_KS : n));
}
static inline int lw_ctiles(const LSTMArgs& a) {
  int m = 0;
  for (int l = 0; l <= a.L; ++l) m = max(m, (lstm_cols(a, l) + 15) / 16);
  return m;
}
#define LW_TICKS 8  // ticket slots per layer (column tiles; cols <= 128)
#define MF16F32(a, b, c) __builtin_amdgcn_mfma_f32_16x16x4f32((a), (b), (c), 0, 0, 0)

// two 512-thread workgroups per CU (<= 128 VGPRs, 2 x 64 KB LDS): the whole grid (33 chunks x 5
// column tiles x 3 layers at the reference shape) is resident at once
__global__ __launch_bounds__(64 * LW_WAVES, 2) void lstm_wgrad_mfma(LSTMArgs a) {
  __shared__ float s_d[LW_KR * LW_PD];
  __shared__ float s_x[LW_KR * 16];
  __shared__ float s_w[128 * LW_PW];
  __shared__ int s_last;
  const int s = blockIdx.x, ct = blockIdx.y, l = blockIdx.z;
  const int rows = lstm_rows(a, l), cols = lstm_cols(a, l);
  if (ct * 16 >= cols) return;  // uniform per workgroup; never counted by the ticket
  const int c0 = ct * 16;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int T = a.T, L = a.L, G = 4 * a.H, E = a.E;
  const int nch = gridDim.x;
  const long BT = (long)a.B * T, kc = (BT + nch - 1) / nch;
  const long kb = (long)s * kc, ke = min(BT, kb + kc);
  const int rt = (rows + 15) / 16, rp = rt * 16;  // row tiles (<= LW_WAVES), padded rows
  const uint32_t seed = smi_seed(a.seedp, a.salt);
  const bool do_xe = l == 0 && ct == 0 && a.g_xe;
  if (do_xe)
    for (int i = tid; i < G * E; i += 64 * LW_WAVES) s_w[(i / E) * LW_PW + i % E] = a.w_ih[0][i];
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  for (long k = kb; k < ke; k += LW_KR) {
    const int nk = (int)min((long)LW_KR, ke - k), nk4 = (nk + 3) & ~3;
    __syncthreads();  // the previous round's LDS reads are done
    if (l < L) {  // da rows: 16-B loads, every one of the round in flight together
      const int q4 = rp / 4;
      for (int i = tid; i < nk4 * q4; i += 64 * LW_WAVES) {
        const int kk = i / q4, q = i - kk * q4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (kk < nk) {
          const int bt = (int)k + kk;  // B * T < 2^31 (LSTM_MAXT): 32-bit division
          const int b = bt / T, t = bt - b * T;
          v = *(const float4*)(a.ws_da + (((size_t)b * L + l) * T + t) * G + 4 * q);
        }
        *(float4*)(s_d + kk * LW_PD + 4 * q) = v;
      }
    } else {
      for (int i = tid; i < nk4 * rp; i += 64 * LW_WAVES) {
        const int kk = i / rp, r = i - kk * rp;
        float v = 0.f;
        if (kk < nk) {
          const int bt = (int)k + kk;  // B * T < 2^31 (LSTM_MAXT): 32-bit division
          const int b = bt / T, t = bt - b * T;
          v = lw_d(a, l, b, t, r, rows);
        }
        s_d[kk * LW_PD + r] = v;
      }
    }
    for (int i = tid; i < nk4 * 16; i += 64 * LW_WAVES) {
      const int kk = i >> 4, cc = i & 15;
      float v = 0.f;
      if (kk < nk) {
        const int bt = (int)k + kk;
        const int b = bt / T, t = bt - b * T;
        v = lw_x(a, l, b, t, c0 + cc, cols, seed);
      }
      s_x[kk * 16 + cc] = v;
    }
    __syncthreads();
    if (w < rt) {
#pragma unroll 4
      for (int k0 = 0; k0 < nk4; k0 += 4)
        acc = MF16F32(s_d[(k0 + lk) * LW_PD + w * 16 + li], s_x[(k0 + lk) * 16 + li], acc);
    }
    if (do_xe) {  // xe rows of this round: (row tile, 16-column group) per wave
      const int et = (E + 15) / 16, xt = ((nk + 15) / 16) * et;
      for (int x = w; x < xt; x += LW_WAVES) {
        const int r16 = (x / et) * 16, e0 = (x % et) * 16;
        f32x4_t xa = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
        for (int kr = 0; kr < G; kr += 4) {
          const float av = r16 + li < nk ? s_d[(r16 + li) * LW_PD + kr + lk] : 0.f;
          xa = MF16F32(av, s_w[(kr + lk) * LW_PW + e0 + li], xa);
        }
        if (e0 + li < E) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int rr = r16 + 4 * lk + j;
            if (rr < nk) a.g_xe[(k + rr) * E + e0 + li] = xa[j];
          }
        }
      }
    }
  }
  // this chunk's partial of the slice: [rows][cols] tile s of layer l in the slab
  float* part = a.g_slab + lstm_part_off(a, l, s);
  if (w < rt && c0 + li < cols) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = w * 16 + 4 * lk + j;
      if (r < rows) smi_wt_store(part + (size_t)r * cols + c0 + li, acc[j]);  // write-through hand-off
    }
  }
  smi_wt_drain();
  __syncthreads();
  if (tid == 0) s_last = atomicAdd(a.ce_tick + l * LW_TICKS + ct, 1u) == (unsigned)nch - 1;
  __syncthreads();
  if (!s_last) return;
  const int In = l < L ? (l == 0 ? E : a.H) : 0;
  const long pstride = (long)rows * cols;  // consecutive chunks' partial tiles of layer l
  const float* pbase = a.g_slab + lstm_part_off(a, l, 0);
  for (int p = tid; p < rows * 16; p += 64 * LW_WAVES) {
    const int r = p >> 4, c = c0 + (p & 15);
    if (c >= cols) continue;
    const size_t o = (size_t)r * cols + c;
    // every chunk's load in flight at once (device-scope loads reach memory: a serial chain of
    // them made the reduction the kernel's long pole), then the fixed chunk-order sum
    float v = 0.f;
    for (int q0 = 0; q0 < nch; q0 += 16) {
      float pv[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) pv[j] = q0 + j < nch ? smi_cc_load(pbase + (q0 + j) * pstride + o) : 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (q0 + j < nch) v += pv[j];
    }
    if (l == L) {
      if (c < a.H) a.g_w_fc[(size_t)r * a.H + c] += v;
      else a.g_b_fc[r] += v;
    } else if (c < In) a.g_w_ih[l][(size_t)r * In + c] += v;
    else if (c < In + a.H) a.g_w_hh[l][(size_t)r * a.H + (c - In)] += v;
    else {
      a.g_b_ih[l][r] += v;
      a.g_b_hh[l][r] += v;
    }
  }
  if (tid == 0) a.ce_tick[l * LW_TICKS + ct] = 0u;  // re-armed for the next step (graph replay)
}

// the MFMA form's limits: 4H (and C) <= 128 rows, E <= 32, column tiles <= LW_TICKS
static bool lw_fits(const LSTMArgs& a) {
  return 4 * a.H <= 128 && a.C <= 128 && a.E <= 32 && lw_ctiles(a) <= LW_TICKS && a.ce_tick != nullptr;
}

// the MFMA weight gradient (default; 35 us for every weight gradient against 39 + 8 us for the
// VALU split-K pair, docs/PERF_NOTES.md round 4); 0: the two-launch VALU split-K reduction above
// (+ lstm_xe_kernel), still taken by the shapes outside lw_fits
static int g_lstm_wgrad_mfma = 1;
static int lstm_wgrad_mfma_enabled() { return g_lstm_wgrad_mfma; }

// per-token embedding-input gradients xe[b,t,:] = W_ih0^T da0[b,t,:] (the table gradient is their
// position-ordered per-id sum, csrc/kernels/embedding.hip)
__global__ __launch_bounds__(256) void lstm_xe_kernel(LSTMArgs a) {
  const long q = (long)blockIdx.x * 256 + threadIdx.x;
  const long BT = (long)a.B * a.T;
  if (q >= BT * a.E) return;
  const long bt = q / a.E;
  const int e = (int)(q % a.E), b = (int)(bt / a.T), t = (int)(bt % a.T), G = 4 * a.H;
  const float* d = a.ws_da + (((size_t)b * a.L) * a.T + t) * G;  // layer 0
  const float* w = a.w_ih[0] + e;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  for (int r = 0; r < G; r += 4) {
    s0 += w[(size_t)r * a.E] * d[r];
    s1 += w[(size_t)(r + 1) * a.E] * d[r + 1];
    s2 += w[(size_t)(r + 2) * a.E] * d[r + 2];
    s3 += w[(size_t)(r + 3) * a.E] * d[r + 3];
  }
  a.g_xe[q] = (s0 + s1) + (s2 + s3);
}

// 4*H*L <= 256 threads: one wave per SIMD, so the backward's register-resident gradient rows
// and W column slices get the full 512-entry (VGPR + AGPR) file.
static int lstm_w2_enabled() { return 1; }

template <int H, int MI>
static int lstm_launch(const LSTMArgs* a, int backward, hipStream_t st) {
  if constexpr (MI + H <= 64) {
    if (a->L * H <= 64 && lstm_w2_enabled()) {
      if (backward) {
        if (a->C <= 4) hipLaunchKernelGGL((lstm_bwd_w2_kernel<H, MI, 4>), dim3(a->B), dim3(128), 0, st, *a);
        else hipLaunchKernelGGL((lstm_bwd_w2_kernel<H, MI, LSTM_MAXC>), dim3(a->B), dim3(128), 0, st, *a);
      } else {
        const int side = a->emb_side == 1 ? (int)(((long)a->B * a->T + 63) / 64) : 0;
        hipLaunchKernelGGL((lstm_fwd_w2_kernel<H, MI>), dim3(a->B + side), dim3(128), 0, st, *a);
      }
      return (int)hipGetLastError();
    }
  }
  const int threads = ((4 * H * a->L + 63) / 64) * 64;
  if (threads <= 256) {
    if (backward) {
      if (a->C <= 4) hipLaunchKernelGGL((lstm_bwd_kernel<H, MI, 256, 4>), dim3(a->B), dim3(threads), 0, st, *a);
      else hipLaunchKernelGGL((lstm_bwd_kernel<H, MI, 256, LSTM_MAXC>), dim3(a->B), dim3(threads), 0, st, *a);
    }
    else hipLaunchKernelGGL((lstm_fwd_kernel<H, MI, 256>), dim3(a->B), dim3(threads), 0, st, *a);
  } else {
    if (backward) {
      if (a->C <= 4) hipLaunchKernelGGL((lstm_bwd_kernel<H, MI, 512, 4>), dim3(a->B), dim3(threads), 0, st, *a);
      else hipLaunchKernelGGL((lstm_bwd_kernel<H, MI, 512, LSTM_MAXC>), dim3(a->B), dim3(threads), 0, st, *a);
    }
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

extern "C" int smi_emb_bwd_f32(const long long* ids, const void* dout, float* dtable, long T, int D, long long padding_idx,
                               const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale, long V, void* ws,
                               hipStream_t st);
extern "C" int smi_emb_sum(int algo, int bf16, const long long* ids, const void* dout, float* dtable, long T, int D,
                           long long padding_idx, const uint32_t* seedp, uint32_t salt, uint32_t thresh, float dscale,
                           long V, void* ws, hipStream_t st);

extern "C" long smi_lstm_slab_floats(int B, int E, int H, int L, int C) {
  LSTMArgs a{};
  a.B = B; a.E = E; a.H = H; a.L = L; a.C = C;
  return lstm_part_off(a, L + 1, 0);  // partial tiles of every layer and the head
}

extern "C" int smi_emb_plan(const long long* ids, long T, long long padding_idx, long V, void* ws, hipStream_t st);
extern "C" int smi_emb_plan_algo(long T, long V);

extern "C" int smi_lstm(const LSTMArgs* args, int backward, hipStream_t st) {
  LSTMArgs ab = *args;
  const LSTMArgs* a = &ab;
  if (!smi_lstm_supported(a->E, a->H, a->L, a->C) || a->B < 1 || a->T < 1 || a->T > LSTM_MAXT) return -1;
  if (!backward && a->emb_side) {
    // order the ids for the embedding backward in this launch (pair path, w2 kernel) or, when
    // that does not apply, with the standalone ordering launches first
    const long T = (long)a->B * a->T;
    const int algo = smi_emb_plan_algo(T, a->emb_V);
    const bool w2 = a->L * a->H <= 64 && lstm_w2_enabled() && (a->H == 16 || a->H == 32) &&
                    (a->E <= a->H ? a->H : 2 * a->H) + a->H <= 64;
    if (!a->emb_ws || !a->emb_tick || algo == 0) return -1;  // the caller counts on a plan
    if (algo == 1 && T <= LSTM_EMB_MAX && w2) {
      ab.emb_side = 1;
    } else {
      if (smi_emb_plan(a->ids, T, a->pad_idx, a->emb_V, a->emb_ws, st) != algo) return -1;
      ab.emb_side = 2;  // planned already: no side workgroups
    }
  }
  if (backward && (!a->g_slab || (a->g_emb && (!a->g_xe || a->V < 1 || !a->emb_ws)))) return -1;
  const int H = a->H;
  const bool wide = a->E > H;
  int rc;
  if (H == 16) rc = wide ? lstm_launch<16, 32>(a, backward, st) : lstm_launch<16, 16>(a, backward, st);
  else if (H == 32) rc = wide ? lstm_launch<32, 64>(a, backward, st) : lstm_launch<32, 32>(a, backward, st);
  else rc = lstm_launch<64, 64>(a, backward, st);
  if (rc || !backward) return rc;
  if (lstm_wgrad_mfma_enabled() && lw_fits(*a)) {
    // ce_tick (backward): (L + 1) x LW_TICKS zeroed counters, re-armed by the kernel
    hipLaunchKernelGGL(lstm_wgrad_mfma, dim3(lw_chunks(*a), lw_ctiles(*a), a->L + 1), dim3(64 * LW_WAVES), 0, st, *a);
    if ((rc = (int)hipGetLastError())) return rc;
    if (a->g_emb && a->emb_planned)
      return smi_emb_sum(a->emb_planned, 0, a->ids, a->g_xe, a->g_emb, (long)a->B * a->T, a->E, a->pad_idx, nullptr, 0,
                         0, 1.f, a->V, a->emb_ws, st);
    if (a->g_emb)
      return smi_emb_bwd_f32(a->ids, a->g_xe, a->g_emb, (long)a->B * a->T, a->E, a->pad_idx, nullptr, 0, 0, 1.f, a->V,
                             a->emb_ws, st);
    return 0;
  }
  const int maxrows = 4 * H > a->C ? 4 * H : a->C;
  hipLaunchKernelGGL(lstm_wgrad_partial, dim3(LSTM_KS, (maxrows + LSTM_RB - 1) / LSTM_RB, a->L + 1), dim3(256), 0, st,
                     *a);
  int maxout = 0;
  for (int l = 0; l <= a->L; ++l) {
    const int n = lstm_rows(*a, l) * lstm_cols(*a, l);
    if (n > maxout) maxout = n;
  }
  hipLaunchKernelGGL(lstm_wgrad_combine, dim3((maxout + 255) / 256, a->L + 1), dim3(256), 0, st, *a);
  if ((rc = (int)hipGetLastError())) return rc;
  if (a->g_emb) {
    const long n = (long)a->B * a->T * a->E;
    hipLaunchKernelGGL(lstm_xe_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, *a);
    return smi_emb_bwd_f32(a->ids, a->g_xe, a->g_emb, (long)a->B * a->T, a->E, a->pad_idx, nullptr, 0, 0, 1.f, a->V,
                           a->emb_ws, st);
  }
  return (int)hipGetLastError();
}
