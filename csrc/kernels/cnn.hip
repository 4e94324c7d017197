// Fused FashionMNIST CNN training kernel: one workgroup = one image, the WHOLE forward
// (conv3x3+ReLU x2, maxpool, conv3x3+ReLU x2, maxpool, flatten, linear, softmax-CE) AND backward
// (CE grad, linear, unpool, ReLU', transposed convs, weight/bias gradients) in one launch,
// every activation resident in LDS (zero-halo padded planes, no bounds checks in the conv
// loops), weights read through the scalar cache (wave-uniform indices).
//
// Reference model: FashionMNISTModel (distributed_cnn.py:47-86 / pytorch_cnn.py:12-49):
// block_1 = Conv(Cin->C,3,p1) ReLU Conv(C->C,3,p1) ReLU MaxPool(2); block_2 = same at 14x14;
// classifier = Flatten (NCHW order) + Linear(C*7*7 -> classes); trained with CrossEntropyLoss
// (mean) + SGD (distributed_cnn.py:138-141).  At the reference batch (32 images/GPU) the step is
// latency-bound (6.7 MFLOP/image), so whole-step fusion beats per-layer GEMMs: one launch per
// step for fwd+bwd, one for the cross-image gradient reduction (+dloss scale), one for SGD.
// ToTensor()'s uint8 -> [0,1] scaling is fused into the image load.
//
// Per-image gradients go to a slab [B][P] (P = all parameters, packed in the order
// w1 b1 w2 b2 w3 b3 w4 b4 wfc bfc); cnn_grad_reduce sums the slab over images (fixed order:
// bit-reproducible) and accumulates into the model's gradient buffers.
#include <algorithm>

#include "smi_common.h"
#include "smi_cnn.h"
#include <type_traits>

// One workgroup per image; 1024 threads (16 waves) so every phase of the per-image pipeline has
// enough independent work items (the batch of 32 images occupies only 32 CUs)
#define CNN_THREADS 1024
#ifdef CNN_STAMPS  // diagnostic build only (tools/probes/cnn_probe.hip): per-phase s_memtime
__device__ unsigned long long cnn_stamps[256 * 32];  // image + helper workgroups
#define STAMP(i)                                                                            \
  do {                                                                                      \
    if (threadIdx.x == 0) {                                                                 \
      unsigned long long t_;                                                                \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");           \
      cnn_stamps[blockIdx.x * 32 + (i)] = t_;                                               \
    }                                                                                       \
  } while (0)
// global-clock (s_memrealtime, 100 MHz, one clock for every XCD) stamps: cross-workgroup timing
__device__ unsigned long long cnn_rstamps[256 * 8];
#define RSTAMP(i)                                                                           \
  do {                                                                                      \
    if (threadIdx.x == 0) cnn_rstamps[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define STAMP(i) do {} while (0)
#define RSTAMP(i) do {} while (0)
#endif
#define P28 30   // 28x28 plane with 1-pixel zero halo
#define P14 16   // 14x14 plane with 1-pixel zero halo
// channel-plane stride: the halo plane plus CNN_PAD floats, so the same position of consecutive
// channels lands in different LDS banks (a 16 x 16 plane is 256 floats: every channel started at
// bank 0, and the weight-gradient / MFMA operand reads of 16 channels conflicted).  Swept with
// tools/probes/cnn_probe.hip (-DCNN_PAD14 / -DCNN_PAD28): 0/0 94.8k clocks per image body, 4/8
// 85.9k (14 x 14 weight gradients 6.4k -> 4.1k), a plateau beyond.
#ifndef CNN_PAD14
#define CNN_PAD14 4
#endif
#ifndef CNN_PAD28
#define CNN_PAD28 8
#endif
#define CPL(pp) ((pp) * (pp) + ((pp) == P14 ? CNN_PAD14 : CNN_PAD28))
#ifndef CNN_CONV1_VALU_MAXC
#define CNN_CONV1_VALU_MAXC 2
#endif
#define PL28 CPL(P28)
#define PL14 CPL(P14)
// weight-gradient helper workgroups per image (CNNArgs::hand): conv4, conv3, conv2 (two halves of
// its columns)
#ifndef CNN_HELPERS
#define CNN_HELPERS 4  // >= 3: conv4, conv3, then conv2's column tiles split over the rest
#endif
static_assert(CNN_HELPERS >= 3, "conv4, conv3 and at least one conv2 helper");

__device__ __forceinline__ int i28(int c, int y, int x) { return c * PL28 + (y + 1) * P28 + (x + 1); }
__device__ __forceinline__ int i14(int c, int y, int x) { return c * PL14 + (y + 1) * P14 + (x + 1); }

// Weights and biases are read through the constant address space: every lane reads the same
// element, so these become s_load (scalar cache) operands of the FMAs instead of per-lane vector
// loads (global_load) or LDS reads — the vector form made the conv loops load-bound (~14x off).
typedef const __attribute__((address_space(4))) float* cfp;

// ticket of the in-kernel mean-loss reduction (one training step in flight per device)
__device__ unsigned cnn_loss_ticket = 0u;

// forward 3x3 conv + bias + relu over an HxH plane set; in/out padded with pitch PP.
// Work unit = (output-channel group, 64-position chunk), one per wave: at 14 x 14 (196
// positions = 4 chunks) the 16 waves split the output channels 4 ways, so every wave works
// (one lane per position computing all channels left 12 of 16 waves idle and made conv3/conv4
// as slow as the 4x larger conv2).  The group index is wave-uniform, so weights stay scalar.
// Channel groups are compile-time (CC = channel capacity of this kernel instance): the group
// loop fully unrolls, all of a step's weights are fetched as a few wide s_loads, and a group
// that runs past cout computes on clamped weights and skips the store — runtime per-channel
// guards compiled into one scalar branch + s_waitcnt lgkmcnt(0) per channel (conv2 forward
// 41k -> 19k cycles; docs/PERF_NOTES.md CNN section).
//
// Each lane computes a horizontal PAIR of output positions with packed fp32 FMAs
// (v_pk_fma_f32, scalar weight broadcast to both halves): one 3x4 window (3 aligned 8-B LDS
// reads x 2) serves both outputs, and every weight s_load and FMA issue covers two outputs.
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 pkfma(float w, f2 v, f2 acc) { return __builtin_elementwise_fma((f2)(w), v, acc); }

template <int H, int CC>
struct ConvGroups {
  static constexpr int NPAIR = H * H / 2;                // H even: pairs (y, 2i), (y, 2i+1)
  static constexpr int NCH = (NPAIR + 63) / 64;          // 64-pair chunks
  static constexpr int NW = CNN_THREADS / 64;
  static constexpr int NG0 = NW / NCH > 0 ? NW / NCH : 1;
  static constexpr int NGRP = NG0 < CC ? NG0 : CC;       // channel groups
  static constexpr int CG = (CC + NGRP - 1) / NGRP;      // channels per group
};

// 3 x 4 window at row pointer r (8-B aligned, pitch PP): per row, pairs (c0,c1), (c1,c2), (c2,c3)
template <int PP>
__device__ __forceinline__ void load_win(const float* r, f2 (&A)[3], f2 (&M)[3], f2 (&B)[3], int rstep) {
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    const f2* q = (const f2*)(r + ky * rstep);
    A[ky] = q[0];
    B[ky] = q[1];
    M[ky] = f2{A[ky].y, B[ky].x};
  }
}

template <int H, int PP, int CC, bool EX>
__device__ __forceinline__ void conv_fwd(const float* __restrict__ in, int cin, float* __restrict__ out, int cout,
                         const float* __restrict__ wg, const float* __restrict__ bg) {
  using G = ConvGroups<H, CC>;
  constexpr int HP = H / 2;
  const cfp w = (cfp)wg;
  const cfp b = (cfp)bg;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  for (int u = wv; u < G::NGRP * G::NCH; u += G::NW) {
    const int grp = u / G::NCH, chunk = u - grp * G::NCH;
    const int co0 = __builtin_amdgcn_readfirstlane(grp * G::CG);
    if (co0 >= cout) continue;
    // the last group slides back to end at cout (its overlap with the previous group is
    // recomputed, stored once); rows stay contiguous, so each is one s_load_dwordx8 + dword
    const int base = EX ? min(co0, CC - G::CG) : max(0, min(co0, cout - G::CG));
    int wrow[G::CG];
#pragma unroll
    for (int c = 0; c < G::CG; ++c) wrow[c] = EX ? base + c : min(base + c, cout - 1);
    const int q = chunk * 64 + lane;
    const bool ok = q < G::NPAIR;
    const int qq = ok ? q : 0;
    const int y = qq / HP, x0 = (qq - y * HP) * 2;
    f2 acc[G::CG];
#pragma unroll
    for (int c = 0; c < G::CG; ++c) acc[c] = (f2)(b[wrow[c]]);
#pragma unroll 1  // a full unroll (cin is compile-time with EX) hoists every weight into SGPRs and spills
    for (int ci = 0; ci < cin; ++ci) {
      f2 A[3], M[3], B[3];  // output x0 uses cols x0..x0+2, x0+1 uses x0+1..x0+3 (halo coords)
      load_win<PP>(in + ci * CPL(PP) + y * PP + x0, A, M, B, PP);
#pragma unroll
      for (int c = 0; c < G::CG; ++c) {
        const cfp wp = w + (wrow[c] * cin + ci) * 9;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          acc[c] = pkfma(wp[ky * 3 + 0], A[ky], acc[c]);
          acc[c] = pkfma(wp[ky * 3 + 1], M[ky], acc[c]);
          acc[c] = pkfma(wp[ky * 3 + 2], B[ky], acc[c]);
        }
      }
    }
    if (ok) {
#pragma unroll
      for (int c = 0; c < G::CG; ++c)
        if (base + c >= co0 && base + c < cout) {
          float* op = out + (base + c) * CPL(PP) + (y + 1) * PP + (x0 + 1);
          op[0] = fmaxf(acc[c].x, 0.f);
          op[1] = fmaxf(acc[c].y, 0.f);
        }
    }
  }
}

// 2x2/2 max pool of H x H (pitch PPI) into H/2 planes (pitch PPO, halo offset HO)
template <int H, int PPI, int PPO, int HO>
__device__ __forceinline__ void pool_fwd(const float* __restrict__ in, float* __restrict__ out, int c) {
  constexpr int Ho = H / 2;
  for (int e = threadIdx.x; e < c * Ho * Ho; e += blockDim.x) {
    const int ch = e / (Ho * Ho), r = e % (Ho * Ho), py = r / Ho, px = r % Ho;
    const float* p = in + ch * CPL(PPI) + (2 * py + 1) * PPI + (2 * px + 1);
    const float m = fmaxf(fmaxf(p[0], p[1]), fmaxf(p[PPI], p[PPI + 1]));
    out[HO ? (ch * CPL(PPO) + (py + 1) * PPO + (px + 1)) : (ch * Ho * Ho + py * Ho + px)] = m;
  }
}

// unpool the gradient g (per pooled element) into the pre-pool activation buffer a IN PLACE:
// a <- (pos == first argmax of its window && a > 0) ? g : 0   (torch max_pool2d + relu backward)
template <int H, int PPI>
__device__ __forceinline__ void unpool_relu_inplace(float* __restrict__ a, const float* __restrict__ g, int gpitch, int ghalo,
                                    int c) {
  constexpr int Ho = H / 2;
  for (int e = threadIdx.x; e < c * Ho * Ho; e += blockDim.x) {
    const int ch = e / (Ho * Ho), r = e % (Ho * Ho), py = r / Ho, px = r % Ho;
    float* p = a + ch * CPL(PPI) + (2 * py + 1) * PPI + (2 * px + 1);
    const float gv = ghalo ? g[ch * CPL(gpitch) + (py + 1) * gpitch + (px + 1)] : g[ch * Ho * Ho + py * Ho + px];
    const float v0 = p[0], v1 = p[1], v2 = p[PPI], v3 = p[PPI + 1];
    int am = 0;
    float m = v0;
    if (v1 > m) { m = v1; am = 1; }
    if (v2 > m) { m = v2; am = 2; }
    if (v3 > m) { m = v3; am = 3; }
    const float gg = m > 0.f ? gv : 0.f;
    p[0] = am == 0 ? gg : 0.f;
    p[1] = am == 1 ? gg : 0.f;
    p[PPI] = am == 2 ? gg : 0.f;
    p[PPI + 1] = am == 3 ? gg : 0.f;
  }
}

// dW[co][ci][k] = sum_pos dz[co][pos] * in[ci][pos+k-1]; db[co] = sum_pos dz[co][pos]
// as a GEMM on the fp32 matrix cores: D[co][n] = sum_p dz[co][p] * X[p][n] with n = ci*9 + k
// (im2col gathered straight from the LDS planes) and one extra all-ones column n = cin*9 for
// the bias.  v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation): A[i][k] = dz of
// output channel i (lane & 15) at position 4s + (lane >> 4), B[k][j] = im2col element of column
// j (lane & 15) at the same position; co is padded to 16, n to whole 16-column tiles.  Work
// unit = (n tile, chunk of k-steps); per-unit 16x16 tiles go to LDS scratch and a final pass
// sums the chunks of each entry in chunk order (deterministic).  The VALU version (window
// reuse across 5 output channels + a 64-value transposing wave reduction) spent 4 cycles of
// SIMD issue per FMA-equivalent and was 45 % of the fused step.
typedef float f4 __attribute__((ext_vector_type(4)));
#define WG_SCRATCH (12 * 256)  // floats: up to 12 units of one 16x16 tile

template <int H, int PP>
// [tlo, thi): the 16-column tiles to compute (a weight-gradient helper takes half of conv2's)
__device__ __forceinline__ void conv_wgrad(const float* __restrict__ dz, const float* __restrict__ in, int cin, int cout,
                           float* __restrict__ acc, float* __restrict__ scratch, int sb = -1, int tlo = 0,
                           int thi = 1 << 20) {
  // k-steps come in groups of 7 = 28 positions (one row at H = 28, two at H = 14), so a lane's
  // 7 gather offsets inside a group are fixed: per group, 14 LDS reads at precomputed addresses,
  // 14 address increments and 7 MFMAs — no per-step index math (per-step y/x updates and
  // mode selects made the VALU, not the matrix core, the bottleneck: ~240 cycles per k-step).
  constexpr int GS = 7, NG = H * H / 28, GROWS = 28 / H;
  static_assert(H * H % 28 == 0, "position groups");
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = blockDim.x >> 6;
  const int ncol = cin * 9 + 1;            // im2col columns + bias column
  const int t_hi = min(thi, (ncol + 15) >> 4), nt = t_hi - tlo;  // 16-column tiles of this call
  const int nch = max(1, min(min(nw, WG_SCRATCH / 256) / nt, NG));  // group chunks per tile
  const int units = nt * nch;
  const int i = lane & 15, kq = lane >> 4;
  const float* zero_cell = scratch + WG_SCRATCH;      // 0.f (A padding rows, B padding columns)
  const float* one_cell = scratch + WG_SCRATCH + 1;   // 1.f (bias column)
  int off[GS];
#pragma unroll
  for (int q = 0; q < GS; ++q) {
    const int pp = 4 * q + kq;
    off[q] = (pp / H) * PP + pp % H;
  }
  const bool aok = i < cout;
  const int astr = aok ? GROWS * PP : 0;
  for (int u = wv; u < units; u += nw) {
    const int t = u % nt, ch = u / nt;
    const int n = (tlo + t) * 16 + i;      // this lane's B column (j = lane & 15)
    const float* bbase;
    int bstr = 0;
    const bool bg = n < cin * 9;
    if (bg) {
      const int ci = n / 9, k = n - ci * 9;
      bbase = in + ci * CPL(PP) + (k / 3) * PP + (k % 3);
      bstr = GROWS * PP;
    } else {
      bbase = n == cin * 9 ? one_cell : zero_cell;
    }
    const int g0 = ch * NG / nch, g1 = (ch + 1) * NG / nch;
    const float* pa[GS];
    const float* pb[GS];
#pragma unroll
    for (int q = 0; q < GS; ++q) {
      pa[q] = aok ? dz + i * CPL(PP) + PP + 1 + off[q] + g0 * astr : zero_cell;  // dz at (y+1, x+1)
      pb[q] = bbase + (bg ? off[q] : 0) + g0 * bstr;
    }
    f4 d0 = {0.f, 0.f, 0.f, 0.f}, d1 = {0.f, 0.f, 0.f, 0.f};  // MFMA dependent latency 40 > issue 32
    for (int g = g0; g < g1; ++g) {
      float av[GS], bv[GS];
#pragma unroll
      for (int q = 0; q < GS; ++q) { av[q] = *pa[q]; bv[q] = *pb[q]; }
#pragma unroll
      for (int q = 0; q < GS; ++q) {
        if (q & 1) d1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q], bv[q], d1, 0, 0, 0);
        else d0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q], bv[q], d0, 0, 0, 0);
        pa[q] += astr;
        pb[q] += bstr;
      }
    }
    const f4 d = d0 + d1;
    float* row = scratch + u * 256;        // [co 16][col 16]: lane holds rows 4*(lane>>4)+r, col lane&15
#pragma unroll
    for (int r = 0; r < 4; ++r) row[(kq * 4 + r) * 16 + i] = d[r];
  }
  if (sb >= 0) STAMP(sb);      // probe build: wave 0's units done
  __syncthreads();
  if (sb >= 0) STAMP(sb + 1);  // all units done
  // combine the chunks of every entry in chunk order; weights [co][ci*9+k], then biases
  const int nwt = cout * cin * 9;
  for (int e = threadIdx.x; e < nwt + cout; e += blockDim.x) {
    const int co = e < nwt ? e / (cin * 9) : e - nwt;
    const int col = e < nwt ? e - co * cin * 9 : cin * 9;
    const int tt = (col >> 4) - tlo, j = col & 15;
    if (tt < 0 || tt >= nt) continue;  // another call's tile
    float v = 0.f;
    for (int c = 0; c < nch; ++c) v += scratch[(c * nt + tt) * 256 + co * 16 + j];
    acc[e] = v;
  }
}

// in-place transposed conv + relu': a[ci][pos] <- (a[ci][pos] > 0) ? sum_co sum_k w[co][ci][k] dz[co][pos-k+1] : 0
// (relu=false: plain write into out).  Same (input-channel group, 64-position chunk) per-wave
// units as conv_fwd: a lane loads each dz window once and applies it to every input channel of
// its group with wave-uniform (scalar) weights; the former lane-per-(ci, pos) mapping re-read the
// window per input channel and fell back to per-lane weight loads where a wave straddled two
// channels.
template <int H, int PP, int CC, bool EX>
__device__ __forceinline__ void conv_dgrad(const float* __restrict__ dz, int cout, const float* __restrict__ wg, int cin,
                           float* __restrict__ a, bool relu) {
  using G = ConvGroups<H, CC>;
  constexpr int HP = H / 2;
  const cfp w = (cfp)wg;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  for (int u = wv; u < G::NGRP * G::NCH; u += G::NW) {
    const int grp = u / G::NCH, chunk = u - grp * G::NCH;
    const int ci0 = __builtin_amdgcn_readfirstlane(grp * G::CG);  // wave-uniform (see conv_fwd)
    if (ci0 >= cin) continue;
    const int base = EX ? min(ci0, CC - G::CG) : max(0, min(ci0, cin - G::CG));
    int wcol[G::CG];
#pragma unroll
    for (int c = 0; c < G::CG; ++c) wcol[c] = EX ? base + c : min(base + c, cin - 1);
    const int q = chunk * 64 + lane;
    const bool ok = q < G::NPAIR;
    const int qq = ok ? q : 0;
    const int y = qq / HP, x0 = (qq - y * HP) * 2;
    f2 acc[G::CG];
#pragma unroll
    for (int c = 0; c < G::CG; ++c) acc[c] = f2{0.f, 0.f};
#pragma unroll 1
    for (int co = 0; co < cout; ++co) {
      // rows y+2-ky (ky = 0..2) of dz, cols x0..x0+3: output x0 takes col x0+2-kx, x0+1 takes x0+3-kx
      f2 A[3], M[3], B[3];
      load_win<PP>(dz + co * CPL(PP) + (y + 2) * PP + x0, A, M, B, -PP);
#pragma unroll
      for (int c = 0; c < G::CG; ++c) {
        const cfp wp = w + (co * cin + wcol[c]) * 9;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          acc[c] = pkfma(wp[ky * 3 + 0], B[ky], acc[c]);
          acc[c] = pkfma(wp[ky * 3 + 1], M[ky], acc[c]);
          acc[c] = pkfma(wp[ky * 3 + 2], A[ky], acc[c]);
        }
      }
    }
    if (ok) {
#pragma unroll
      for (int c = 0; c < G::CG; ++c) {
        if (base + c >= ci0 && base + c < cin) {
          float* ap = a + (base + c) * CPL(PP) + (y + 1) * PP + (x0 + 1);
          ap[0] = relu ? (ap[0] > 0.f ? acc[c].x : 0.f) : acc[c].x;
          ap[1] = relu ? (ap[1] > 0.f ? acc[c].y : 0.f) : acc[c].y;
        }
      }
    }
  }
}

// ---- bf16 matrix-core convolutions (the BASELINE CNN config's precision; fp32 accumulation) --
// A 3x3/pad-1 conv over an H x H LDS plane set is an implicit GEMM on v_mfma_f32_16x16x32_bf16:
//   forward  D[pos][co] = sum_{k = ci*9 + ky*3 + kx} in[ci][pos + (ky-1, kx-1)] * W[co][ci][ky][kx]
//   dgrad    D[pos][ci] = sum_{k = co*9 + ky*3 + kx} dz[co][pos + (1-ky, 1-kx)] * W[co][ci][ky][kx]
// M = 16 positions per tile, N = 16 channels (C <= 16), K = 9 * channels padded to 32-steps.
// Lane l gathers A[row l&15][k = 32s + 8(l>>4) + j] straight from the zero-halo fp32 planes
// (per-lane offsets precomputed once per layer, so a k-step is 8 LDS reads + 4 packs + 1 MFMA)
// and holds B[k][col l&15] = the weights for its (k, channel), converted to bf16 once per layer.
// D: col = channel l&15, rows = positions 4(l>>4) + r.  Tiles are spread over the 16 waves.

__device__ __forceinline__ bf16x8_t cnn_pack8(const float (&v)[8]) {
  const unsigned p0 = pack2bf(v[0], v[1]), p1 = pack2bf(v[2], v[3]), p2 = pack2bf(v[4], v[5]), p3 = pack2bf(v[6], v[7]);
  typedef __attribute__((ext_vector_type(4))) unsigned u4;
  return __builtin_bit_cast(bf16x8_t, (u4){p0, p1, p2, p3});
}

// DG = false: forward (+bias, ReLU) into `out`; DG = true: transposed conv into `out` in place of
// the forward activation, times relu'(out) when RELU (dz of the layer below), plain otherwise.
// `tab` (LDS scratch): the layer's k -> plane-offset table and the bf16 B fragments of every
// k-step, built once per call so the per-tile loop keeps almost nothing in registers (the
// kernel runs 16 waves: 128 VGPRs per lane).
// fragment-table entries (per layer: built once per call, or for the exact instance once per
// launch: cnn_pretab).  Entry e = k-step s (e >> 6) x lane l: 8 bf16 of B[k = 32 s + 8 (l >> 4) + j]
// [col = l & 15].  conv_mfma orders k channel-major (k = c * 9 + tap), the channels-last form
// tap-major over 16 channels (k = tap * 16 + c).
template <bool DG>
__device__ __forceinline__ bf16x8_t cnn_wtab_entry(int e, const float* __restrict__ wg, int nin, int nout) {
  const int s = e >> 6, l = e & 63, col = l & 15, K = nin * 9;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 32 * s + 8 * (l >> 4) + j;
    const int c = k / 9, kk = k - c * 9;
    v[j] = (k < K && col < nout) ? wg[DG ? (c * nout + col) * 9 + kk : (col * nin + c) * 9 + kk] : 0.f;
  }
  return cnn_pack8(v);
}
template <int PP, bool DG>
__device__ __forceinline__ int cnn_otab_entry(int k, int nin) {
  const int c = k / 9, kk = k - c * 9, ky = kk / 3, kx = kk - ky * 3;
  return k < nin * 9 ? (DG ? c * CPL(PP) + (2 - ky) * PP + (2 - kx) : c * CPL(PP) + ky * PP + kx) : -1;
}

// the per-tile loop of conv_mfma over built tables (otab: [ks * 32] plane offsets, -1 padding;
// wtab: [ks][64] B fragments; bg: the bias (forward))
template <int H, int PP, bool DG, bool RELU>
__device__ __forceinline__ void conv_mfma_tiles(const float* __restrict__ in, float* __restrict__ out, int nout,
                                                const int* __restrict__ otab, const bf16x8_t* __restrict__ wtab, int ks,
                                                const float* __restrict__ bg) {
  constexpr int NT = (H * H + 15) / 16;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int col = lane & 15, kq = lane >> 4;
  const float bias = (!DG && col < nout) ? bg[col] : 0.f;
  for (int t = wv; t < NT; t += nw) {
    const int p = t * 16 + col;  // this lane's A row (position)
    const bool pv = p < H * H;
    const int base = pv ? (p / H) * PP + (p % H) : 0;
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < ks; ++s) {
      const int4 o0 = *(const int4*)(otab + 32 * s + 8 * kq), o1 = *(const int4*)(otab + 32 * s + 8 * kq + 4);
      const int o[8] = {o0.x, o0.y, o0.z, o0.w, o1.x, o1.y, o1.z, o1.w};
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (pv && o[j] >= 0) ? in[base + o[j]] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cnn_pack8(v), wtab[s * 64 + lane], acc, 0, 0, 0);
    }
    if (col < nout) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = t * 16 + 4 * kq + r;
        if (q < H * H) {
          float* o = out + col * CPL(PP) + (q / H + 1) * PP + (q % H + 1);
          if (!DG) *o = fmaxf(acc[r] + bias, 0.f);
          else *o = RELU ? (*o > 0.f ? acc[r] : 0.f) : acc[r];
        }
      }
    }
  }
}

// DG = false: forward (+bias, ReLU) into `out`; DG = true: transposed conv into `out` in place of
// the forward activation, times relu'(out) when RELU (dz of the layer below), plain otherwise.
// `tab` (LDS scratch): the layer's k -> plane-offset table and the bf16 B fragments of every
// k-step, built once per call so the per-tile loop keeps almost nothing in registers (the
// kernel runs 16 waves: 128 VGPRs per lane).
template <int H, int PP, bool DG, bool RELU>
__device__ __forceinline__ void conv_mfma(const float* __restrict__ in, int nin, float* __restrict__ out, int nout,
                                          const float* __restrict__ wg, const float* __restrict__ bg,
                                          float* __restrict__ tab) {
  const int ks = (nin * 9 + 31) / 32;
  int* otab = (int*)tab;                          // [ks * 32] plane offsets (-1: padding k)
  bf16x8_t* wtab = (bf16x8_t*)(tab + 256);        // [ks][64 lanes] B fragments
  for (int k = threadIdx.x; k < ks * 32; k += blockDim.x) otab[k] = cnn_otab_entry<PP, DG>(k, nin);
  for (int e = threadIdx.x; e < ks * 64; e += blockDim.x) wtab[e] = cnn_wtab_entry<DG>(e, wg, nin, nout);
  __syncthreads();
  conv_mfma_tiles<H, PP, DG, RELU>(in, out, nout, otab, wtab, ks, bg);
}

// ---- 28 x 28 MFMA convolutions from a channels-last bf16 copy (the exact C = 10 instance) ----
// conv_mfma gathers each lane's 8 consecutive k of one position from the fp32 planes: 8 scalar LDS
// reads + 2 offset-table reads per k-step, LDS-issue bound (conv2's forward and dgrad were the two
// longest phases of the image).  Ordering k tap-major over 16 (padded) channels — k = tap * 16 +
// channel — makes those 8 values 8 consecutive channels of one position: with the input first
// copied to position-major bf16 rows of 16 channels, one 16-B read.  9 taps x 16 = 144 k in 5
// k-steps (vs 3 for 90 k): more MFMAs, a fifth of the LDS instructions.  Same bf16 operand values
// (round-to-nearest of the same fp32 activations and weights), fp32 accumulation.  The copy (900
// padded positions x 32 B) lives in the 14 x 14 planes' region, dead during conv2's forward and
// during its dgrad.
#define HWC_KS 5

// hw[half * ...]: row pos (padded position of the PP x PP plane) = 2 granules of 8 channels
template <int PP>
__device__ __forceinline__ void cnn_to_hwc(const float* __restrict__ in, int nin, uint4* __restrict__ hw) {
  for (int e = threadIdx.x; e < 2 * PP * PP; e += blockDim.x) {
    const int half = e >= PP * PP, pos = e - half * PP * PP, c0 = 8 * half;  // lanes: consecutive positions
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = c0 + j < nin ? in[(c0 + j) * CPL(PP) + pos] : 0.f;
    hw[2 * pos + half] = make_uint4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7]));
  }
}

// channels-last B fragments: forward W[col][c][tap]; dgrad (A offset (dy, dx) = (1 - ky, 1 - kx))
// W[c][col][8 - tap]
template <bool DG>
__device__ __forceinline__ bf16x8_t cnn_wtab_hwc_entry(int e, const float* __restrict__ wg, int nin, int nout) {
  const int s = e >> 6, l = e & 63, col = l & 15;
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 32 * s + 8 * (l >> 4) + j, tap = k >> 4, c = k & 15;
    v[j] = (tap < 9 && c < nin && col < nout) ? wg[DG ? (c * nout + col) * 9 + (8 - tap) : (col * nin + c) * 9 + tap] : 0.f;
  }
  return cnn_pack8(v);
}

template <int H, int PP, bool DG, bool RELU>
__device__ __forceinline__ void conv_hwc_tiles(const uint4* __restrict__ hw, float* __restrict__ out, int nout,
                                               const bf16x8_t* __restrict__ wtab, const float* __restrict__ bg) {
  constexpr int NT = (H * H + 15) / 16;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int col = lane & 15, half = (lane >> 4) & 1, tsel = lane >> 5;  // k = 32 s + 8 (lane >> 4) + j
  const float bias = (!DG && col < nout) ? bg[col] : 0.f;
  const bf16x8_t* hb = (const bf16x8_t*)hw;
  for (int t = wv; t < NT; t += nw) {
    const int p = t * 16 + col;  // this lane's A row (position)
    const bool pv = p < H * H;
    const int base = pv ? (p / H + 1) * PP + (p % H + 1) : PP + 1;  // padded position
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < HWC_KS; ++s) {
      const int tap = 2 * s + tsel;  // this lane's tap (dy, dx) = (tap / 3 - 1, tap % 3 - 1)
      const bf16x8_t z = {0, 0, 0, 0, 0, 0, 0, 0};
      const bf16x8_t a = (pv && tap < 9) ? hb[2 * (base + (tap / 3 - 1) * PP + (tap % 3 - 1)) + half] : z;
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wtab[s * 64 + lane], acc, 0, 0, 0);
    }
    if (col < nout) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = t * 16 + 4 * (lane >> 4) + r;
        if (q < H * H) {
          float* o = out + col * CPL(PP) + (q / H + 1) * PP + (q % H + 1);
          if (!DG) *o = fmaxf(acc[r] + bias, 0.f);
          else *o = RELU ? (*o > 0.f ? acc[r] : 0.f) : acc[r];
        }
      }
    }
  }
}

// conv_mfma's contract (DG / RELU / out / epilogue) with the input `in` given as fp32 planes and
// copied to the channels-last bf16 rows `hw` first (nin, nout <= 16); wtab: prebuilt fragments
// (cnn_pretab) or null (built here in `tab`)
template <int H, int PP, bool DG, bool RELU>
__device__ __forceinline__ void conv_mfma_hwc(const float* __restrict__ in, int nin, uint4* __restrict__ hw,
                                              float* __restrict__ out, int nout, const float* __restrict__ wg,
                                              const float* __restrict__ bg, float* __restrict__ tab,
                                              const bf16x8_t* __restrict__ wtab_pre = nullptr) {
  cnn_to_hwc<PP>(in, nin, hw);
  const bf16x8_t* wtab = wtab_pre;
  if (!wtab_pre) {
    bf16x8_t* wt = (bf16x8_t*)tab;
    for (int e = threadIdx.x; e < HWC_KS * 64; e += blockDim.x) wt[e] = cnn_wtab_hwc_entry<DG>(e, wg, nin, nout);
    wtab = wt;
  }
  __syncthreads();
  conv_hwc_tiles<H, PP, DG, RELU>(hw, out, nout, wtab, bg);
}

// ---- the exact bf16 instance's fragment tables, built once per launch (cnn_pretab) ----
// Every MFMA conv of the image then skips its table build (per call: ~1k clocks of weight reads,
// packing and a barrier); the weights are read from global memory once, while the workgroup
// clears its LDS.  Layout (16-B granules): conv2 forward / dgrad channels-last [HWC_KS][64] each,
// conv3 / conv4 forward / dgrad [3][64] each, the 14 x 14 forward / dgrad offset tables [96] ints
// each, the four conv biases [4][16].
struct CnnTabs {
  bf16x8_t *t2f, *t2d, *t3f, *t3d, *t4f, *t4d;
  int *o14f, *o14d;
  float* bias;
};
#define CNN_PRETAB_FLOATS (4 * (2 * HWC_KS * 64 + 4 * 3 * 64) + 2 * 96 + 64 + 4)
__device__ __forceinline__ CnnTabs cnn_tabs(float* at) {
  CnnTabs t;
  bf16x8_t* b = (bf16x8_t*)(((uintptr_t)at + 15) & ~(uintptr_t)15);
  t.t2f = b; t.t2d = b + HWC_KS * 64;
  t.t3f = t.t2d + HWC_KS * 64; t.t3d = t.t3f + 3 * 64; t.t4f = t.t3d + 3 * 64; t.t4d = t.t4f + 3 * 64;
  t.o14f = (int*)(t.t4d + 3 * 64); t.o14d = t.o14f + 96;
  t.bias = (float*)(t.o14d + 96);
  return t;
}
// C = nin = nout = 10 (three 32-deep k-steps of 90 channel-major k)
__device__ __forceinline__ void cnn_pretab(const CNNArgs& g, const CnnTabs& t, int C) {
  constexpr int NH = HWC_KS * 64, NO = 3 * 64;
  for (int e = threadIdx.x; e < 2 * NH + 4 * NO + 2 * 96 + 64; e += blockDim.x) {
    int r = e;
    if (r < NH) { t.t2f[r] = cnn_wtab_hwc_entry<false>(r, g.w[1], C, C); continue; }
    r -= NH;
    if (r < NH) { t.t2d[r] = cnn_wtab_hwc_entry<true>(r, g.w[1], C, C); continue; }
    r -= NH;
    if (r < NO) { t.t3f[r] = cnn_wtab_entry<false>(r, g.w[2], C, C); continue; }
    r -= NO;
    if (r < NO) { t.t3d[r] = cnn_wtab_entry<true>(r, g.w[2], C, C); continue; }
    r -= NO;
    if (r < NO) { t.t4f[r] = cnn_wtab_entry<false>(r, g.w[3], C, C); continue; }
    r -= NO;
    if (r < NO) { t.t4d[r] = cnn_wtab_entry<true>(r, g.w[3], C, C); continue; }
    r -= NO;
    if (r < 96) { t.o14f[r] = cnn_otab_entry<P14, false>(r, C); continue; }
    r -= 96;
    if (r < 96) { t.o14d[r] = cnn_otab_entry<P14, true>(r, C); continue; }
    r -= 96;
    const int l = r >> 4, c = r & 15;
    t.bias[r] = c < C ? g.b[l][c] : 0.f;
  }
}

// bf16 weight gradient (the bf16 path): the same GEMM D[co][n] = sum_pos dz[co][pos] X[pos][n] on
// v_mfma_f32_16x16x32_bf16 (fp32 accumulation), summed over the PADDED position index q (rows of
// the halo plane, halo columns included: dz is zero there), so a lane's 8 positions of a 32-deep
// k-step are 8 CONSECUTIVE floats — dz by 4 ds_read_b64, the im2col column by 8 ds_read_b32 at one
// base — instead of one scalar gather per position (the fp32 16x16x4 form: 2 gathers per 4
// positions, LDS-issue bound).  q covers [PP, PP + 32 KS) — every interior position; an im2col
// index below 0 (the first position, a halo one: dz = 0 there) is clamped to 0, indices past the
// plane read the next buffer's finite values (times dz = 0).
template <int H, int PP>
__device__ __forceinline__ void conv_wgrad_bf16(const float* __restrict__ dz, const float* __restrict__ in, int cin, int cout,
                                                float* __restrict__ acc, float* __restrict__ scratch, int tlo = 0,
                                                int thi = 1 << 20) {
  constexpr int KS = (H * PP + H - PP + 1 + 31) / 32;  // 32-position k-steps
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = blockDim.x >> 6;
  const int ncol = cin * 9 + 1;
  const int t_hi = min(thi, (ncol + 15) >> 4), nt = t_hi - tlo;  // 16-column tiles of this call
  const int nch = max(1, min(min(nw, WG_SCRATCH / 256) / nt, KS));
  const int units = nt * nch;
  const int i = lane & 15, g = lane >> 4;
  const bool aok = i < cout;
  const float* pa = dz + (aok ? i : 0) * CPL(PP);
  for (int u = wv; u < units; u += nw) {
    const int t = u % nt, ch = u / nt;
    const int n = (tlo + t) * 16 + i;  // this lane's B column
    const int mode = n < cin * 9 ? 0 : (n == cin * 9 ? 1 : 2);  // gather / bias ones / padding zeros
    int boff = 0;
    if (mode == 0) {
      const int ci = n / 9, k = n - ci * 9;
      boff = ci * CPL(PP) + (k / 3 - 1) * PP + (k % 3 - 1);
    }
    const int s0 = ch * KS / nch, s1 = (ch + 1) * KS / nch;
    f32x4_t d = {0.f, 0.f, 0.f, 0.f};
    for (int s = s0; s < s1; ++s) {
      // 28 x 28: lane group g takes positions q + g + 4 e — for one e the 64 lanes read 16
      // channels x 4 consecutive positions (distinct banks at the 908-float plane stride) instead
      // of 8-position runs (measured: conv2 / conv1 weight gradients -4 %, -5 %; at 14 x 14 the
      // runs are faster)
      constexpr int QS = H == 28 ? 4 : 1;
      const int q = PP + 32 * s + (QS == 4 ? g : 8 * g);
      float av[8], bv[8];
      if (aok) {
        if (QS == 1) {
          const f2* ap = (const f2*)(pa + q);  // q even, plane bases 8-B aligned
#pragma unroll
          for (int e = 0; e < 4; ++e) { const f2 v = ap[e]; av[2 * e] = v.x; av[2 * e + 1] = v.y; }
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) av[e] = pa[q + QS * e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) av[e] = 0.f;
      }
      if (mode == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) bv[e] = in[max(boff + q + QS * e, 0)];
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) bv[e] = mode == 1 ? 1.f : 0.f;
      }
      d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cnn_pack8(av), cnn_pack8(bv), d, 0, 0, 0);
    }
    float* row = scratch + u * 256;  // [co 16][col 16]: lane holds rows 4 g + r, column i
#pragma unroll
    for (int r = 0; r < 4; ++r) row[(g * 4 + r) * 16 + i] = d[r];
  }
  __syncthreads();
  const int nwt = cout * cin * 9;
  for (int e = threadIdx.x; e < nwt + cout; e += blockDim.x) {
    const int co = e < nwt ? e / (cin * 9) : e - nwt;
    const int col = e < nwt ? e - co * cin * 9 : cin * 9;
    const int tt = (col >> 4) - tlo, j = col & 15;
    if (tt < 0 || tt >= nt) continue;  // another call's tile
    float v = 0.f;
    for (int c = 0; c < nch; ++c) v += scratch[(c * nt + tt) * 256 + co * 16 + j];
    acc[e] = v;
  }
}

// Compact slab row (P floats, P % 4 == 0): the conv layers' gradients at their parameter offsets
// [0, off[8]), then from the 16-B aligned cnn_cs(g) the image's logit gradient dl [NC] and pooled
// activations p2 [F] in place of the NC x F fc outer product (the reducers form the batch sum of
// dl[o] * p2[i]: a third of the bytes to hand off).
__device__ __forceinline__ int cnn_cs(const CNNArgs& g) { return (g.off[8] + 3) & ~3; }

// Pin a loaded value in its register here: the compiler's wait for it happens at this point (with
// the level's other loads in flight alongside) and not in front of a later store, where its
// conservative count-to-zero wait also drains every store before (one round trip per store).
#define CNN_PIN(x) asm volatile("" : "+v"(x))

// Fused SGD tail (CNNArgs::fused): the step's remaining work without a second launch.  Every
// workgroup of the launch (images and their helpers) counts itself done on one counter; the
// workgroups of images 0 .. nsl - 1 (nsl = min(CNN_NSL, B)) are the SLICE workgroups: a slice loads
// its parameters, waits until the counter says every workgroup is done (a bounded wait: the
// slices are the first workgroups of the grid, so every workgroup they wait for is running or
// gets a CU; a time-out poisons the slice with NaN), then slice s owns the s-th part of the
// parameters: it sums every image's slab entries of its conv granules (image chunks over the
// threads, chunk partials in LDS, fixed order), stages every image's dl and its p2 columns in LDS,
// forms its fc columns' gradient as the batch sum of dl[o] * p2[i] (image chunks over lanes, a
// fixed-order butterfly), and applies torch SGD (p -= lr * g); the last slice to finish writes the
// mean loss (image order), the step counter and the index-mode cursor.  Hand-offs are write-
// through stores + device-scope loads in 16-B granules (smi_common.h), no L2 fences.
// Deterministic: every sum has a fixed order.  One level, fixed slices: the earlier two-level
// form (per-group tickets, group partial sums handed over, then 4 slices) paid two more round
// trips, and slices picked by ticket order loaded their parameters only after their ticket
// (docs/PERF_NOTES.md).
// GRADIENT mode (lr == null; the data-parallel step): the same, but the slices ADD the batch
// gradient to gw / gb (the flat fp32 gradient buffer, reduced across executors next and consumed
// by the optimizer) instead of updating the parameters: g += batch sum, written as g - (-1) * sum so
// both modes share one code path (exact), no step bump, no shadows.
__device__ __forceinline__ void cnn_fused_tail(const CNNArgs& g, float* sm, int slice) {
  __shared__ int last;
  const int nsl = min(CNN_NSL, g.B);
  const unsigned total = (g.hand ? 1u + CNN_HELPERS : 1u) * (unsigned)g.B;  // workgroups of the launch
  const int off8 = g.off[8], NC = g.classes, F = g.C * 49, nt = blockDim.x, P = g.P;
  const int cs = cnn_cs(g), n4 = cs >> 2;  // conv part in 16-B granules
  const __amdgpu_buffer_rsrc_t rslab = smi_rsrc(g.slab, g.B * P * 4);
  smi_wt_drain();  // this wave's slab stores reached the coherence point
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(g.tick, 1u);  // done
  if (slice < 0 || slice >= nsl) return;
  RSTAMP(5);
  STAMP(26);
  const bool gmode = g.lr == nullptr;
  const int ilo = slice * F / nsl, ihi = (slice + 1) * F / nsl, Fs = ihi - ilo;         // fc columns
  const int q4lo = slice * n4 / nsl, q4hi = (slice + 1) * n4 / nsl, nq = q4hi - q4lo;  // conv granules
  // the tensor the slice updates for slab segment seg: the parameter, or (gradient mode) its gradient
  auto dst_of = [&](int seg) -> float* {
    return gmode ? (seg % 2 == 0 ? g.gw[seg / 2] : g.gb[seg / 2]) : const_cast<float*>(seg % 2 == 0 ? g.w[seg / 2] : g.b[seg / 2]);
  };
  // parameter p's segment (compares against the uniform offsets), offset in it and destination (a
  // table in LDS: a lane-varying index into the argument block reads it from memory, one dependent
  // load per step, and selects over the 8 pointers spill)
  __shared__ float* seg_dst[8];
  __shared__ unsigned short* seg_sh[8];
  __shared__ int seg_off[8];
  if (threadIdx.x < 8) {
    seg_dst[threadIdx.x] = dst_of(threadIdx.x);
    seg_sh[threadIdx.x] = g.shadow[threadIdx.x];
    seg_off[threadIdx.x] = g.off[threadIdx.x];
  }
  __syncthreads();
  // (the segment's offset from the LDS table too: selecting it from the argument block compiled to
  // a global load of the selected address, whose wait also waited out every earlier store)
  auto conv_seg = [&](int p, int& seg, int& r) {
    seg = 0;
#pragma unroll
    for (int k = 1; k < 8; ++k) seg += p >= g.off[k] ? 1 : 0;
    r = p - seg_off[seg];
    return seg_dst[seg] + r;
  };
  auto shadow_of = [&](int seg) { return seg_sh[seg]; };
  // The slice's own parameters first: nothing else writes them in this launch, so their loads fly
  // during the wait.  Loads are unconditional (clamped addresses; a range-checked buffer load past
  // the end reads 0): a load under a branch makes the compiler wait for EVERY outstanding memory
  // operation, stores included, before its first use (measured: one store round trip per
  // parameter, 6 us in the fc update).
  // fc: slot = (column i, class half h: two halves of 8 classes, o4 granules ob, ob+1, when NC > 8
  // and two columns per thread fit), KCH consecutive lanes per slot, lane kc taking images kc,
  // kc + KCH, ...
  const int H = (NC > 8 && 2 * Fs <= nt) ? 2 : 1, no4 = (H == 2 || NC <= 8) ? 2 : 4, nslot = H * Fs;
  int KCH = 1;
  while (KCH < 8 && 2 * KCH * nslot <= nt) KCH *= 2;
  const int slot = (int)threadIdx.x / KCH, kc = (int)threadIdx.x - slot * KCH;
  const int h = H == 2 ? slot / Fs : 0, ob = H == 2 ? 2 * h : 0;
  const int i0 = ilo + slot - h * Fs;
  const bool fc_on = h < H && i0 < ihi;
  float* fw = dst_of(8);
  auto fc_load = [&](int i, float* pv) {
#pragma unroll
    for (int t = 0; t < 16; ++t) pv[t] = fw[min(4 * ob + t, NC - 1) * F + min(max(i, 0), F - 1)];
  };
  float pfc[16];  // the thread's first column
  fc_load(i0, pfc);
  float* fb = dst_of(9);
  const int bo = (int)threadIdx.x - (nt - 128);  // fc bias entry of this thread (wave nt / 64 - 2)
  const float pb = fb[min(max(bo, 0), NC - 1)];
  auto conv_pload = [&](int q4, float* pv) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      int seg, r;
      pv[u] = *(const __attribute__((address_space(1))) float*)conv_seg(min(max(4 * q4 + u, 0), off8 - 1), seg, r);
    }
  };
  // the conv update runs on the LAST threads (granule q = nt - 1 - threadIdx.x) and the fc update
  // on the first ones: different waves, so the two run side by side instead of one after the
  // other on wave 0
  const int cq = nt - 1 - (int)threadIdx.x;
  float pcv[4];  // granule q4lo + cq (the one-granule-per-thread case)
  conv_pload(min(q4lo + cq, q4hi - 1), pcv);
  const float lr0 = gmode ? -1.f : g.lr[0];  // (a load after the wait: one more round trip)
  // wait until every workgroup is done
  if (threadIdx.x == 0) {
    int bad = 0;
    for (int it = 0; __hip_atomic_load(g.tick, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < total; ++it) {
      if (it >= (1 << 22)) { bad = 1; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    last = bad;
  }
  __syncthreads();
  const bool poison = last != 0;
  const float lr = poison ? __builtin_nanf("") : lr0;
  RSTAMP(6);
  STAMP(28);
  // one round trip: the staging loads (every image's dl and this slice's p2 granules into R4-float
  // rows in the free activation planes), the row losses and the conv slab chunks all in flight
  const int R4 = (NC + F + 3) & ~3;
  const int ndl4 = (NC + 3) >> 2, p4lo = (NC + ilo) >> 2, np4 = ((NC + ihi + 3) >> 2) - p4lo, ng = ndl4 + np4;
  const int nst = g.B * ng;
  auto stage_j4 = [&](int e, int& im) {
    im = e / ng;
    const int jj = e - im * ng;
    return jj < ndl4 ? jj : p4lo + (jj - ndl4);
  };
  float4 sv;  // the thread's first staging granule (B <= 64: one per thread at C = 10)
  {
    int im;
    const int j4 = stage_j4(threadIdx.x, im);
    sv = smi_cc_load4(rslab, (im * P + cs + 4 * j4) * 4);  // im >= B: 0
  }
  // Straight-line loads only: a load inside a loop makes the compiler wait for every outstanding
  // load (vmcnt(0)) at the loop, which serialised the staging, row-loss and chunk round trips
  // lane i: row loss i (B <= 64; wave 0 forms the last slice's mean loss; used there only)
  const float rlv = smi_cc_load(g.row_loss + min((int)(threadIdx.x & 63), g.B - 1));
  // conv: chunk c of nch (<= 8) sums images [c B / nch, (c + 1) B / nch) of granule q in image order
  const int nch = max(1, min(min(nt / max(nq, 1), g.B), 8));
  float4* cpart = reinterpret_cast<float4*>(sm + g.B * R4);  // [nch][nq] after the staged rows
  auto chunk_sum = [&](int u, float4* v) {  // the 4 first images' loads of (chunk, granule) u
    const int c = u / nq, q4 = q4lo + (u - c * nq);
    const int lo = c * g.B / nch, hi = (c + 1) * g.B / nch;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = smi_cc_load4(rslab, ((lo + k < hi ? lo + k : g.B) * P + 4 * q4) * 4);  // B: 0
  };
  auto chunk_add = [&](int u, const float4* v) {
    const int c = u / nq, q4 = q4lo + (u - c * nq);
    const int lo = c * g.B / nch, hi = (c + 1) * g.B / nch;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < 4; ++k) acc = make_float4(acc.x + v[k].x, acc.y + v[k].y, acc.z + v[k].z, acc.w + v[k].w);
    for (int im = lo + 4; im < hi; ++im) {  // chunks past 4 images (batches above 32)
      const float4 w = smi_cc_load4(rslab, (im * P + 4 * q4) * 4);
      acc = make_float4(acc.x + w.x, acc.y + w.y, acc.z + w.z, acc.w + w.w);
    }
    return acc;
  };
  // one (chunk, granule) per thread and at most 4 images a chunk: no loop; the loads pinned here,
  // after every load of the phase is issued (the compiler otherwise sinks them into the store's
  // branch behind a vmcnt(0))
  const bool one_chunk = nch * nq <= nt && (g.B + nch - 1) / nch <= 4;
  float4 cv[4];
  chunk_sum(min((int)threadIdx.x, nch * nq - 1), cv);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    CNN_PIN(cv[k].x);
    CNN_PIN(cv[k].y);
    CNN_PIN(cv[k].z);
    CNN_PIN(cv[k].w);
  }
  if (one_chunk) {
    if ((int)threadIdx.x < nch * nq) cpart[threadIdx.x] = chunk_add(threadIdx.x, cv);
  } else {
    for (int u = threadIdx.x; u < nch * nq; u += nt) {
      chunk_sum(u, cv);
      cpart[u] = chunk_add(u, cv);
    }
  }
  {
    int im;
    const int j4 = stage_j4(threadIdx.x, im);
    if ((int)threadIdx.x < nst) reinterpret_cast<float4*>(sm + im * R4)[j4] = sv;
  }
  for (int e = threadIdx.x + nt; e < nst; e += nt) {  // past one granule per thread
    int im;
    const int j4 = stage_j4(e, im);
    reinterpret_cast<float4*>(sm + im * R4)[j4] = smi_cc_load4(rslab, (im * P + cs + 4 * j4) * 4);
  }
#pragma unroll
  for (int t = 0; t < 16; ++t) CNN_PIN(pfc[t]);
  __syncthreads();
  STAMP(21);
  // conv SGD from the chunk partials (chunk order; every LDS read issued before the adds)
  auto conv_apply = [&](int q, const float* pv) {
    float4 cp[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) cp[c] = cpart[min(c, nch - 1) * nq + q];
    float4 gs4 = cp[0];
#pragma unroll
    for (int c = 1; c < 8; ++c)
      if (c < nch) gs4 = make_float4(gs4.x + cp[c].x, gs4.y + cp[c].y, gs4.z + cp[c].z, gs4.w + cp[c].w);
    const float gv[4] = {gs4.x, gs4.y, gs4.z, gs4.w};
    float np[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      np[u] = pv[u] - lr * gv[u];
      CNN_PIN(np[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = 4 * (q4lo + q) + u;
      if (p >= off8) continue;
      int seg, r;
      // global-address-space stores: through a generic pointer (read from the LDS table) they are
      // flat stores, which also count in lgkmcnt, so the next LDS wait would wait them out
      float* dst = conv_seg(p, seg, r);
      *(__attribute__((address_space(1))) float*)dst = np[u];
      unsigned short* sh = shadow_of(seg);
      if (sh) *(__attribute__((address_space(1))) unsigned short*)(sh + r) = f2bf(np[u]);
    }
  };
  if (nq <= nt) {
    if (cq < nq) conv_apply(cq, pcv);
  } else {
    for (int q = threadIdx.x; q < nq; q += nt) {
      float pv[4];
      conv_pload(q4lo + q, pv);
      conv_apply(q, pv);
    }
  }
  STAMP(22);
  STAMP(30);
  // gW[o][i] = sum_im dl[im][o] * p2[im][i] (o = 4 * (ob + t4) + c): lane kc of the slot sums
  // images kc, kc + KCH, ... in batches of IB with every LDS read of a batch issued before the
  // FMAs (one LDS latency per batch), then the slot's lanes combine by a butterfly.
  // NO4 (compile time): the class granules of the slot's half
  auto fc_column_n = [&](auto no4c, int i, const float* pv, int k0, int kst) {
    constexpr int NO4 = decltype(no4c)::value;
    float gw[4 * NO4];
#pragma unroll
    for (int t = 0; t < 4 * NO4; ++t) gw[t] = 0.f;
    constexpr int IB = 8 / NO4;  // images per batch: 32 registers of dl granules in flight
    int im = k0;
    for (; im + (IB - 1) * kst < g.B; im += IB * kst) {
      float x[IB];
      float4 d[IB][NO4];
#pragma unroll
      for (int u = 0; u < IB; ++u) {
        const float* row = sm + (im + u * kst) * R4;
        x[u] = row[NC + i];
#pragma unroll
        for (int t4 = 0; t4 < NO4; ++t4) d[u][t4] = reinterpret_cast<const float4*>(row)[ob + t4];
      }
#pragma unroll
      for (int u = 0; u < IB; ++u)
#pragma unroll
        for (int t4 = 0; t4 < NO4; ++t4) {
          gw[4 * t4] += d[u][t4].x * x[u];
          gw[4 * t4 + 1] += d[u][t4].y * x[u];
          gw[4 * t4 + 2] += d[u][t4].z * x[u];
          gw[4 * t4 + 3] += d[u][t4].w * x[u];
        }
    }
    for (; im < g.B; im += kst) {
      const float* row = sm + im * R4;
      const float x = row[NC + i];
#pragma unroll
      for (int t4 = 0; t4 < NO4; ++t4) {
        const float4 d = reinterpret_cast<const float4*>(row)[ob + t4];
        gw[4 * t4] += d.x * x;
        gw[4 * t4 + 1] += d.y * x;
        gw[4 * t4 + 2] += d.z * x;
        gw[4 * t4 + 3] += d.w * x;
      }
    }
    // the slot's kst (1, 2, 4 or 8) aligned lanes, all active: a DPP butterfly over lane ^ 7 (half-row
    // mirror), ^ 2, ^ 1 (quad perms) — VALU exchanges, not LDS permutes; a + b == b + a, so every
    // lane of the slot holds the same sum
#pragma unroll
    for (int t = 0; t < 4 * NO4; ++t) {
      if (kst >= 8) gw[t] += smi_dpp<SMI_DPP_HMIRROR>(gw[t]);
      if (kst >= 4) gw[t] += smi_dpp<SMI_DPP_QP2301>(gw[t]);
      if (kst >= 2) gw[t] += smi_dpp<SMI_DPP_QP1032>(gw[t]);
    }
    float np[4 * NO4];
#pragma unroll
    for (int t = 0; t < 4 * NO4; ++t) {
      np[t] = pv[t] - lr * gw[t];
      CNN_PIN(np[t]);
    }
    if (k0 != 0) return;
#pragma unroll
    for (int t = 0; t < 4 * NO4; ++t) {
      const int o = 4 * ob + t;
      if (o >= NC) continue;
      fw[o * F + i] = np[t];
      if (g.shadow[8]) g.shadow[8][o * F + i] = f2bf(np[t]);
    }
  };
  auto fc_column = [&](int i, const float* pv, int k0, int kst) {
    if (no4 == 2) fc_column_n(std::integral_constant<int, 2>{}, i, pv, k0, kst);
    else fc_column_n(std::integral_constant<int, 4>{}, i, pv, k0, kst);
  };
  if (nslot * KCH <= nt) {  // one slot per lane group: no loop (a loop's loads make every store wait)
    if (fc_on) fc_column(i0, pfc, kc, KCH);
  } else {  // KCH == 1
    for (int i = i0; i < ihi; i += nt) {
      float pv[16];
      fc_load(i, pv);
      fc_column(i, pv, 0, 1);
    }
  }
  STAMP(23);
  if (slice == 0 && bo >= 0 && bo < NC) {  // the fc bias on the second-to-last wave (beside the rest)
    const int o = bo;
    float gb = 0.f;
#pragma unroll 8
    for (int im = 0; im < g.B; ++im) gb += sm[im * R4 + o];
    const float np = pb - lr * gb;
    fb[o] = np;
    if (g.shadow[9]) g.shadow[9][o] = f2bf(np);
  }
  STAMP(29);
  RSTAMP(7);
  // the last slice to finish: the mean loss (image order), the step counter, the cursor, re-arms
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(g.tick + 1, 1u) == (unsigned)(nsl - 1);
  __syncthreads();
  if (!last) return;
  if (threadIdx.x < 64) {
    const float ls = wave_sum((int)threadIdx.x < g.B ? rlv : 0.f);
    if (threadIdx.x == 0) {
      if (g.loss) g.loss[0] = ls * g.loss_scale;
      if (g.step && !gmode) g.step[0] += 1.f;
      if (g.cursor) g.cursor[0] += 1;  // index mode: every workgroup read it before its ticket
      g.tick[0] = 0u;
      g.tick[1] = 0u;
    }
  }
  // the weight-gradient helpers' hand-off flags, re-armed for the next launch (every helper read
  // its flag before its ticket; conv2's flag is read by two helpers, so none of them re-arms it)
  if (g.hflag)
    for (int i = threadIdx.x; i < 3 * g.B; i += blockDim.x)
      __hip_atomic_store(g.hflag + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- weight-gradient helpers (CNNArgs::hand): the weight gradients off the image's critical path
// The image workgroup's backward is a chain (unpool, dgrad, unpool, dgrad) with a weight gradient
// beside every dgrad; the three large ones (conv4, conv3, conv2: ~60 % of the weight-gradient
// clocks) need only the layer's dz and input planes.  The image workgroup hands those two plane
// sets over through global memory (write-through 16-B stores issued before the dgrad that
// overwrites the input in place, drained by the barrier after it; conv2's drained at once: it is
// the longest) and raises a flag; helper workgroup (image, layer) polls the flag (one lane,
// bounded: a timed-out helper writes NaN gradients instead of hanging), loads the planes into the
// same padded LDS layout, runs the same conv_wgrad, writes the layer's slab entries and joins the
// fused tail's ticket (4 arrivals per image).  Helpers are dispatched after every image workgroup
// (higher block index), so an image never waits for a slot held by a helper.
__host__ __device__ __forceinline__ int cnn_hand_f(int C) { return 2 * C * PL14 + C * PL28; }
// dz plane-set offset of helper j (0: conv4, 1: conv3, 2: conv2) in an image's hand-off area
__host__ __device__ __forceinline__ int cnn_hand_dz(int C, int j) { return j * C * PL14; }

// copy n floats (n % 4 == 0, 16-B aligned) of LDS plane sets into the hand-off area (write-through)
__device__ __forceinline__ void cnn_hand_put(__amdgpu_buffer_rsrc_t rs, int dst, const float* src, int n) {
  for (int i = threadIdx.x; i < n / 4; i += blockDim.x)
    smi_wt_store4(rs, (dst + 4 * i) * 4, reinterpret_cast<const float4*>(src)[i]);
}
__device__ __forceinline__ void cnn_hand_publish(const CNNArgs& g, int img, int j) {
  if (threadIdx.x == 0) __hip_atomic_store(g.hflag + 3 * img + j, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Helper j of image img, after recomputing its layer's input planes (the image's forward prefix, in
// the same LDS layout: bitwise the image workgroup's values) while the image workgroup works: wait
// for the flag, load dz into its plane set, the layer's weight gradient, the slab entries.
template <int H, int PP, bool BF>
__device__ __forceinline__ void cnn_helper_finish(const CNNArgs& g, int img, int j, int C, float* dz, const float* in,
                                                  float* wacc, float* wscr, int tlo = 0, int thi = 1 << 20) {
  __shared__ int s_bad;
  if (threadIdx.x == 0) {
    int bad = 0;
    for (int it = 0; __hip_atomic_load(g.hflag + 3 * img + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u; ++it) {
      if (it >= (1 << 22)) { bad = 1; break; }
      __builtin_amdgcn_s_sleep(4);
    }
    s_bad = bad;
  }
  __syncthreads();
  RSTAMP(1);
  const __amdgpu_buffer_rsrc_t rs = smi_rsrc(g.hand + (long)img * cnn_hand_f(C), cnn_hand_f(C) * 4);
  const int d0 = cnn_hand_dz(C, j), n4 = C * CPL(PP) / 4;
  for (int i = threadIdx.x; i < n4; i += blockDim.x) reinterpret_cast<float4*>(dz)[i] = smi_cc_load4(rs, (d0 + 4 * i) * 4);
  __syncthreads();
  RSTAMP(2);
  if (BF) conv_wgrad_bf16<H, PP>(dz, in, C, C, wacc, wscr, tlo, thi);
  else conv_wgrad<H, PP>(dz, in, C, C, wacc, wscr, -1, tlo, thi);
  __syncthreads();
  RSTAMP(3);
  const bool bad = s_bad != 0;
  const int ow = g.off[6 - 2 * j], ob = g.off[7 - 2 * j];  // conv4 / conv3 / conv2 weight, bias
  float* gs = g.slab + (long)img * g.P;
  for (int e = threadIdx.x; e < C * C * 9 + C; e += blockDim.x) {
    const int col = e < C * C * 9 ? e % (C * 9) : C * 9;
    if ((col >> 4) < tlo || (col >> 4) >= thi) continue;  // the other helper's columns
    smi_wt_store(gs + (e < C * C * 9 ? ow + e : ob + e - C * C * 9), bad ? __builtin_nanf("") : wacc[e]);
  }
}

// One image's forward + backward; true when the fused tail follows (training).  role >= 0: weight-
// gradient helper role (0: conv4, 1: conv3, 2: conv2) of image img — the forward prefix up to that
// layer's input, then cnn_helper_finish.  CC: channel capacity; EX: g.C == CC exactly (compile-time channel count)
template <int CC, bool EX, bool BF>
__device__ __forceinline__ bool cnn_image(const CNNArgs& g, float* sm, const int img, const int role) {
  const int C = EX ? CC : g.C, CI = g.cin, NC = g.classes;
  // the dataset row of this image (index mode: two dependent scalar loads, issued before the
  // weight staging and LDS clearing so their latency hides behind them)
  const long src = g.perm ? g.perm[(long)g.cursor[0] * g.B + img] : (long)img;
  float* xin = sm;                       // CI x 30x30
  float* a1 = xin + CI * PL28;           // C x 30x30
  float* a2 = a1 + C * PL28;             // C x 30x30
  float* p1 = a2 + C * PL28;             // C x 16x16
  float* a3 = p1 + C * PL14;             // C x 16x16
  float* a4 = a3 + C * PL14;             // C x 16x16
  // conv2's channels-last bf16 copy (conv_mfma_hwc) overlays p1 .. a4
  static_assert(!(BF && EX) || (3 * CC * PL14 * 4 >= 2 * P28 * P28 * 16 && 3 * CC * PL14 % 4 == 0),
                "conv_mfma_hwc copy exceeds the 14x14 planes");
  float* p2 = a4 + C * PL14;             // C*49 (flat, NCHW)
  float* lg = p2 + C * 49;               // logits / dlogits [16]
  float* wacc = lg + 16;                 // max(C, CI)*C*9 + C wgrad accumulators
  const int WC = C > CI ? C : CI;
  float* wscr = wacc + WC * C * 9 + C;   // conv_wgrad per-unit 16x16 partial tiles (WG_SCRATCH floats)
  // the four conv layers' weights and biases, staged once for the bf16 (MFMA) convs, whose per-
  // layer fragment tables read them element-wise (the fp32 convs keep global weights: they read
  // them through the constant address space as scalar loads)
  float* wst = wscr + WG_SCRATCH + 2;
  // the exact bf16 instance: every MFMA conv's fragment tables built once here instead (cnn_pretab)
  constexpr bool PRE = BF && EX;
  const CnnTabs tabs = cnn_tabs(wst);
  if (PRE) cnn_pretab(g, tabs, C);
  const float* lw[4] = {};
  const float* lb[4] = {};
  {
    int o = 0;
    for (int l = 0; l < 4; ++l) {
      const int n = C * (l == 0 ? CI : C) * 9;
      if (BF && !PRE && g.wstage) {
        for (int i = threadIdx.x; i < n; i += blockDim.x) wst[o + i] = g.w[l][i];
        for (int i = threadIdx.x; i < C; i += blockDim.x) wst[o + n + i] = g.b[l][i];
        lw[l] = wst + o;
        lb[l] = wst + o + n;
      } else {
        lw[l] = g.w[l];
        lb[l] = g.b[l];
      }
      o += n + C;
    }
  }
  const int total = CI * PL28 + 2 * C * PL28 + 3 * C * PL14 + C * 49 + 16 + WC * C * 9 + C;
  for (int i = threadIdx.x; i < total; i += blockDim.x) sm[i] = 0.f;
  if (threadIdx.x == 0) { wscr[WG_SCRATCH] = 0.f; wscr[WG_SCRATCH + 1] = 1.f; }  // conv_wgrad pad cells
  __syncthreads();
  STAMP(0);
  // the label (thread 0 computes the loss), loaded now so its memory round trip overlaps the
  // image load and conv1 instead of stalling the cross-entropy (measured ~2k clocks)
  int lab0 = 0;
  if (threadIdx.x == 0 && g.y && role < 0) lab0 = (int)g.y[src];
  // image load (+ ToTensor scaling)
  for (int e = threadIdx.x; e < CI * 784; e += blockDim.x) {
    const int c = e / 784, r = e % 784;
    const long gi = src * CI * 784 + e;
    const float v = g.x_u8 ? (float)((const unsigned char*)g.x)[gi] * g.x_scale : ((const float*)g.x)[gi];
    xin[i28(c, r / 28, r % 28)] = v;
  }
  __syncthreads();
  STAMP(1);
  // conv1 on the VALU in both modes when the input has one or two channels: an MFMA k-step would
  // be 9 (18) real taps of 32, and the fp32 sliding-window conv needs no fragment tables
  // (measured at 1 channel: 6.4k -> 2.9k clocks; its weight gradient stays on the bf16 MFMA path,
  // the fp32 one measured 4.7k -> 6.4k)
  if (BF && CI > CNN_CONV1_VALU_MAXC) conv_mfma<28, P28, false, false>(xin, CI, a1, C, lw[0], lb[0], wscr);
  else conv_fwd<28, P28, CC, EX>(xin, CI, a1, C, g.w[0], g.b[0]);
  __syncthreads();
  STAMP(2);
  if (role >= 2) {  // conv2's helpers (their share of its 16-column tiles): their input is a1
    const int np = CNN_HELPERS - 2, j = role - 2, nt2 = (C * 9 + 1 + 15) / 16;
    cnn_helper_finish<28, P28, BF>(g, img, 2, C, a2, a1, wacc, wscr, j * nt2 / np, j == np - 1 ? 1 << 20 : (j + 1) * nt2 / np);
    return true;
  }
  CNN_PIN(lab0);  // arrived during conv1
  if (BF && EX) {
    conv_mfma_hwc<28, P28, false, false>(a1, C, (uint4*)p1, a2, C, nullptr, tabs.bias + 16, wscr, tabs.t2f);
    __syncthreads();
    // the copy overlaid the 14 x 14 planes: their zero halos again
    for (int i = threadIdx.x; i < 3 * C * PL14 / 4; i += blockDim.x) reinterpret_cast<float4*>(p1)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  } else if (BF) {
    conv_mfma<28, P28, false, false>(a1, C, a2, C, lw[1], lb[1], wscr);
  } else {
    conv_fwd<28, P28, CC, EX>(a1, C, a2, C, g.w[1], g.b[1]);
  }
  __syncthreads();
  STAMP(3);
  pool_fwd<28, P28, P14, 1>(a2, p1, C);
  __syncthreads();
  STAMP(4);
  if (role == 1) {  // conv3's helper: its input is p1
    cnn_helper_finish<14, P14, BF>(g, img, 1, C, a3, p1, wacc, wscr);
    return true;
  }
  if (PRE) conv_mfma_tiles<14, P14, false, false>(p1, a3, C, tabs.o14f, tabs.t3f, 3, tabs.bias + 32);
  else if (BF) conv_mfma<14, P14, false, false>(p1, C, a3, C, lw[2], lb[2], wscr);
  else conv_fwd<14, P14, CC, EX>(p1, C, a3, C, g.w[2], g.b[2]);
  __syncthreads();
  STAMP(5);
  if (role == 0) {  // conv4's helper: its input is a3
    cnn_helper_finish<14, P14, BF>(g, img, 0, C, a4, a3, wacc, wscr);
    return true;
  }
  if (PRE) conv_mfma_tiles<14, P14, false, false>(a3, a4, C, tabs.o14f, tabs.t4f, 3, tabs.bias + 48);
  else if (BF) conv_mfma<14, P14, false, false>(a3, C, a4, C, lw[3], lb[3], wscr);
  else conv_fwd<14, P14, CC, EX>(a3, C, a4, C, g.w[3], g.b[3]);
  __syncthreads();
  STAMP(6);
  // classifier: wave w computes logit o = w (NC <= 16 = the waves); its weight row is loaded
  // before pool2 (its round trip overlaps the pool; an LDS-only barrier after the pool leaves it
  // in flight)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int F = C * 49;
  constexpr int FK = (CC * 49 + 63) / 64;  // lane's share of a row: i = lane + 64 k
  float fcw[FK];
  if (wv < NC) {  // (wave-uniform) every load unconditional inside: clamped addresses
    const float* wr = g.w[4] + wv * F;
#pragma unroll
    for (int k = 0; k < FK; ++k) fcw[k] = wr[min(lane + 64 * k, F - 1)];
  }
  // the fc backward's weight columns (thread i < F holds W[o][i] of every class; F <= 784 < the
  // 1024 threads), loaded now too: their round trip overlaps pool2, the classifier and the CE
  float wc[16];
  if (g.train && wv * 64 < F) {
    const int i = min((int)threadIdx.x, F - 1);
#pragma unroll
    for (int o = 0; o < 16; ++o) wc[o] = g.w[4][min(o, NC - 1) * F + i];
  }
  pool_fwd<14, P14, 7, 0>(a4, p2, C);
  smi_lds_barrier();
  STAMP(7);
  if (wv < NC) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < FK; ++k)
      if (lane + 64 * k < F) s += fcw[k] * p2[lane + 64 * k];
    s = wave_sum(s);
    if (lane == 0) lg[wv] = s + g.b[4][wv];
  }
  __syncthreads();
  STAMP(8);
  // cross-entropy on wave 0, lane o = class o (NC <= 16): max, log-sum-exp and the logit gradient
  // as DPP wave reductions, the argmax from a ballot, the label's logit by readlane (one lane
  // walking the classes through dependent LDS reads took ~3k clocks, shuffles ~2.7k)
  float row_l = 0.f;  // lane 0: this image's loss, stored after the fc backward's loads are used
  if (threadIdx.x < 64) {
    const int o = threadIdx.x;
    const float v = o < NC ? lg[o] : -INFINITY;
    const float m = wave_max(v);
    const unsigned long long top = __ballot(v == m);
    const int am = top ? __builtin_ctzll(top) : 0;  // the first maximum
    const float lse = m + __logf(wave_sum(o < NC ? __expf(v - m) : 0.f));
    const int lab = min(max(__builtin_amdgcn_readfirstlane(lab0), 0), NC - 1);
    row_l = lse - __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lab));
    if (o == 0 && g.pred) g.pred[img] = am;
    if (o < NC) {
      if (g.logits) g.logits[(long)img * NC + o] = v;
      // dlogits = (softmax - onehot) * loss_scale   (loss_scale = 1/B for a mean loss)
      if (g.train) lg[o] = (__expf(v - lse) - (o == lab ? 1.f : 0.f)) * g.loss_scale;
    }
  }
  // the row loss (thread 0) and, unfused, the mean loss without a second launch: the last
  // workgroup to get here (atomic ticket) sums row_loss in image order with wave 0 and re-arms the
  // ticket (the fused step's tail forms the mean loss instead)
  auto store_loss = [&]() {
    if (threadIdx.x == 0 && g.row_loss) smi_wt_store(g.row_loss + img, row_l);
    if (g.loss && g.row_loss && !g.fused) {
      __shared__ int cnn_last;
      smi_wt_drain();
      __syncthreads();
      if (threadIdx.x == 0) cnn_last = atomicAdd(&cnn_loss_ticket, 1u) == (unsigned)g.B - 1;
      __syncthreads();
      if (cnn_last && threadIdx.x < 64) {
        float s = 0.f;
        for (int i = threadIdx.x; i < g.B; i += 64)
          s += __hip_atomic_load(g.row_loss + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s = wave_sum(s);
        if (threadIdx.x == 0) {
          g.loss[0] = s * g.loss_scale;
          cnn_loss_ticket = 0u;
        }
      }
    }
  };
  if (!g.train) {
    store_loss();
    return false;
  }
  // LDS-only barriers from here to the dgrad chain: the row loss / slab stores stay in flight (a
  // plain __syncthreads waits for them: ~1.5k clocks each); the tail drains before its ticket
  smi_lds_barrier();
  STAMP(9);
  float* gs = g.slab + (long)img * g.P;  // this image's gradient slab
  // fc grads: the slab keeps this image's dl (NC) and p2 (F) in place of the NC x F outer product
  // gW[o][i] = dl[o] * p2[i] (gb[o] = dl[o]): the reducers form the batch sum of products (a
  // third of the bytes to reduce).  dp2[i] = sum_o W[o][i] dl[o] replaces p2[i] in place (the
  // thread that read p2[i]: no barrier between).  Every store comes after the W loads' use (a
  // wait for a load issued after a store would wait out the store too: vmcnt retires in order)
  if ((int)threadIdx.x < F) {
    const int i = threadIdx.x;
    const float pv = p2[i];
    // all 16 logit-gradient slots read unconditionally, issued together (slots >= NC hold 0 from
    // the LDS clear: their terms add +0, the sum is unchanged); a guarded loop waited per read
    float l16[16];
#pragma unroll
    for (int o = 0; o < 16; ++o) l16[o] = lg[o];
    float s = 0.f;
#pragma unroll
    for (int o = 0; o < 16; ++o) s += wc[o] * l16[o];
    p2[i] = s;  // dp2 (flat NCHW)
    smi_wt_store(gs + cnn_cs(g) + NC + i, pv);
  }
  if ((int)threadIdx.x < NC) smi_wt_store(gs + cnn_cs(g) + threadIdx.x, lg[threadIdx.x]);
  store_loss();
  smi_lds_barrier();
  STAMP(10);
  STAMP(11);
  // pool2 backward + relu'(a4): dz4 in a4
  unpool_relu_inplace<14, P14>(a4, p2, 7, 0, C);
  __syncthreads();
  STAMP(12);
  if (g.hand) {
    // conv4 / conv3 / conv2 weight gradients by the helpers (which recomputed the layers' inputs);
    // this workgroup hands over each dz and runs the dgrad chain.  dz4 / dz3 are drained by the
    // barrier after the next dgrad, conv2's (the largest weight gradient) at once
    const __amdgpu_buffer_rsrc_t rh = smi_rsrc(g.hand + (long)img * cnn_hand_f(C), cnn_hand_f(C) * 4);
    cnn_hand_put(rh, cnn_hand_dz(C, 0), a4, C * PL14);  // dz4
    if (PRE) conv_mfma_tiles<14, P14, true, true>(a4, a3, C, tabs.o14d, tabs.t4d, 3, nullptr);
    else if (BF) conv_mfma<14, P14, true, true>(a4, C, a3, C, lw[3], nullptr, wscr);
    else conv_dgrad<14, P14, CC, EX>(a4, C, g.w[3], C, a3, true);
    smi_wt_drain();
    __syncthreads();
    cnn_hand_publish(g, img, 0);
    STAMP(14);
    cnn_hand_put(rh, cnn_hand_dz(C, 1), a3, C * PL14);  // dz3
    if (PRE) conv_mfma_tiles<14, P14, true, false>(a3, p1, C, tabs.o14d, tabs.t3d, 3, nullptr);
    else if (BF) conv_mfma<14, P14, true, false>(a3, C, p1, C, lw[2], nullptr, wscr);
    else conv_dgrad<14, P14, CC, EX>(a3, C, g.w[2], C, p1, false);
    smi_wt_drain();
    __syncthreads();
    cnn_hand_publish(g, img, 1);
    STAMP(16);
    unpool_relu_inplace<28, P28>(a2, p1, P14, 1, C);
    __syncthreads();
    STAMP(17);
    cnn_hand_put(rh, cnn_hand_dz(C, 2), a2, C * PL28);  // dz2
    smi_wt_drain();
    __syncthreads();
    cnn_hand_publish(g, img, 2);
    STAMP(18);
    RSTAMP(1);
    if (BF && EX) conv_mfma_hwc<28, P28, true, true>(a2, C, (uint4*)p1, a1, C, nullptr, nullptr, wscr, tabs.t2d);
    else if (BF) conv_mfma<28, P28, true, true>(a2, C, a1, C, lw[1], nullptr, wscr);
    else conv_dgrad<28, P28, CC, EX>(a2, C, g.w[1], C, a1, true);
    __syncthreads();
    STAMP(19);
    if (BF) conv_wgrad_bf16<28, P28>(a1, xin, CI, C, wacc, wscr);
    else conv_wgrad<28, P28>(a1, xin, CI, C, wacc, wscr, 23);
    __syncthreads();
    STAMP(20);
    for (int e = threadIdx.x; e < C * CI * 9 + C; e += blockDim.x)
      smi_wt_store(gs + (e < C * CI * 9 ? g.off[0] + e : g.off[1] + e - C * CI * 9), wacc[e]);
    return true;
  }
  // conv4: dW4, db4 (from dz4, a3); then dz3 = convT(dz4) * relu'(a3) in a3
  if (BF) conv_wgrad_bf16<14, P14>(a4, a3, C, C, wacc, wscr);
  else conv_wgrad<14, P14>(a4, a3, C, C, wacc, wscr, 25);
  __syncthreads();
  STAMP(13);
  for (int e = threadIdx.x; e < C * C * 9 + C; e += blockDim.x) {
    smi_wt_store(gs + (e < C * C * 9 ? g.off[6] + e : g.off[7] + e - C * C * 9), wacc[e]);
    wacc[e] = 0.f;
  }
  if (PRE) conv_mfma_tiles<14, P14, true, true>(a4, a3, C, tabs.o14d, tabs.t4d, 3, nullptr);
  else if (BF) conv_mfma<14, P14, true, true>(a4, C, a3, C, lw[3], nullptr, wscr);
  else conv_dgrad<14, P14, CC, EX>(a4, C, g.w[3], C, a3, true);
  __syncthreads();
  STAMP(14);
  // conv3: dW3 (dz3, p1); dp1 = convT(dz3) into p1 (no relu: p1 is a pool output)
  if (BF) conv_wgrad_bf16<14, P14>(a3, p1, C, C, wacc, wscr);
  else conv_wgrad<14, P14>(a3, p1, C, C, wacc, wscr);
  __syncthreads();
  STAMP(15);
  for (int e = threadIdx.x; e < C * C * 9 + C; e += blockDim.x) {
    smi_wt_store(gs + (e < C * C * 9 ? g.off[4] + e : g.off[5] + e - C * C * 9), wacc[e]);
    wacc[e] = 0.f;
  }
  if (PRE) conv_mfma_tiles<14, P14, true, false>(a3, p1, C, tabs.o14d, tabs.t3d, 3, nullptr);
  else if (BF) conv_mfma<14, P14, true, false>(a3, C, p1, C, lw[2], nullptr, wscr);
  else conv_dgrad<14, P14, CC, EX>(a3, C, g.w[2], C, p1, false);
  __syncthreads();
  STAMP(16);
  // pool1 backward + relu'(a2): dz2 in a2
  unpool_relu_inplace<28, P28>(a2, p1, P14, 1, C);
  __syncthreads();
  STAMP(17);
  // conv2: dW2 (dz2, a1); dz1 = convT(dz2) * relu'(a1) in a1
  if (BF) conv_wgrad_bf16<28, P28>(a2, a1, C, C, wacc, wscr);
  else conv_wgrad<28, P28>(a2, a1, C, C, wacc, wscr, 21);
  __syncthreads();
  STAMP(18);
  for (int e = threadIdx.x; e < C * C * 9 + C; e += blockDim.x) {
    smi_wt_store(gs + (e < C * C * 9 ? g.off[2] + e : g.off[3] + e - C * C * 9), wacc[e]);
    wacc[e] = 0.f;
  }
  if (BF && EX) conv_mfma_hwc<28, P28, true, true>(a2, C, (uint4*)p1, a1, C, nullptr, nullptr, wscr, tabs.t2d);
  else if (BF) conv_mfma<28, P28, true, true>(a2, C, a1, C, lw[1], nullptr, wscr);
  else conv_dgrad<28, P28, CC, EX>(a2, C, g.w[1], C, a1, true);
  __syncthreads();
  STAMP(19);
  // conv1: dW1 (dz1, x)
  if (BF) conv_wgrad_bf16<28, P28>(a1, xin, CI, C, wacc, wscr);
  else conv_wgrad<28, P28>(a1, xin, CI, C, wacc, wscr, 23);
  __syncthreads();
  STAMP(20);
  for (int e = threadIdx.x; e < C * CI * 9 + C; e += blockDim.x)
    smi_wt_store(gs + (e < C * CI * 9 ? g.off[0] + e : g.off[1] + e - C * CI * 9), wacc[e]);
  return true;
}

// one workgroup per image (+ with CNNArgs::hand, three weight-gradient helpers per image after
// them); every workgroup of a fused step then joins the tail (its one call site: a second inlined
// copy of the register-heavy tail made the whole kernel spill)
template <int CC, bool EX, bool BF>
__global__ __launch_bounds__(CNN_THREADS) void cnn_kernel(CNNArgs g) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  RSTAMP(0);
  const int wg = blockIdx.x;
  const bool helper = g.hand && wg >= g.B;  // uniform per workgroup
  const int img = helper ? (wg - g.B) / CNN_HELPERS : wg;
  if (!cnn_image<CC, EX, BF>(g, sm, img, helper ? (wg - g.B) % CNN_HELPERS : -1)) return;
  RSTAMP(4);
  if (g.fused) cnn_fused_tail(g, sm, helper ? -1 : img);
}

// grad[p] (+)= dloss * sum_img slab[img][p], scattered to the 10 parameter tensors; also the mean
// loss / correct-count reductions (thread 0 of block 0)
__global__ void cnn_reduce_kernel(CNNArgs g) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const float dl = g.dloss ? g.dloss[0] : 1.f;
  if (p < g.P) {
    // the compact slab (cnn_cs): an fc weight gradient entry is the batch sum of dl[o] * p2[i]
    const int off8 = g.off[8], F = g.C * 49, cs = cnn_cs(g);
    int a = p, b = -1;  // slab entries: the value, or the product of two
    if (p >= g.off[9]) a = cs + (p - g.off[9]);
    else if (p >= off8) { const int o = (p - off8) / F; a = cs + o; b = cs + g.classes + (p - off8 - o * F); }
    // 8 independent partial sums: all 8 loads of a round are in flight together (a plain
    // serial loop waited one memory round trip per image: 10 us for 32 images), fixed order
    float q[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int i = 0;
    for (; i + 8 <= g.B; i += 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float* r = g.slab + (long)(i + j) * g.P;
        q[j] += b < 0 ? r[a] : r[a] * r[b];
      }
    }
    for (int j = 0; i < g.B; ++i, ++j) {
      const float* r = g.slab + (long)i * g.P;
      q[j] += b < 0 ? r[a] : r[a] * r[b];
    }
    const float s = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
    int seg = 0;
    while (seg < 9 && p >= g.off[seg + 1]) ++seg;
    float* dst = seg % 2 == 0 ? g.gw[seg / 2] : g.gb[seg / 2];
    dst[p - g.off[seg]] += s * dl;
  }
}

static size_t cnn_lds_bytes(const CNNArgs& g) {
  const int C = g.C, CI = g.cin;
  // + conv_wgrad scratch (WG_SCRATCH floats)
  const int WC = C > CI ? C : CI;  // wgrad accumulators hold [C][max(C, CI)*9] + C
  // + the staged conv weights and biases (C * CI * 9 + 3 * C * C * 9 + 4 * C) when wstage
  // + the launch-wide fragment tables instead (wstage 2: the exact C = 10 bf16 instance)
  return sizeof(float) * (size_t)(CI * PL28 + 2 * C * PL28 + 3 * C * PL14 + C * 49 + 16 + WC * C * 9 + C + 4 +
                                  WG_SCRATCH + 2 +
                                  (g.wstage == 2 ? CNN_PRETAB_FLOATS : g.wstage ? C * CI * 9 + 3 * C * C * 9 + 4 * C : 0));
}

// the fused tail's LDS: every image's staged dl / p2 row, then the conv chunk partials (at most 8
// chunks of a slice's granules, float4; cnn_fused_tail)
static size_t cnn_tail_lds(int C, int cin, int classes, int B) {
  const int n4 = ((C * cin * 9 + C + 3 * (C * C * 9 + C)) + 3) >> 2, nsl = B < CNN_NSL ? B : CNN_NSL;
  const int nq = (n4 + nsl - 1) / nsl;  // a slice's conv granules (at most)
  return sizeof(float) * ((size_t)B * ((classes + C * 49 + 3) & ~3) + 4 * 8 * (size_t)nq);
}

extern "C" int smi_cnn(const CNNArgs* args, hipStream_t st) {
  CNNArgs g = *args;
  if (g.fused && (g.P % 4 || g.B > CNN_MAXB || !g.tick || !g.slab || !g.row_loss || !g.train)) return -1;
  if (g.perm && (!g.fused || !g.cursor)) return -1;  // index mode: fused steps only
  if (g.hand && (!g.fused || !g.hflag)) return -1;    // helpers: fused steps only
  if (g.fused && !g.lr) {  // gradient mode: every gradient destination, no shadows
    for (int i = 0; i < 5; ++i)
      if (!g.gw[i] || !g.gb[i]) return -1;
    for (int i = 0; i < 10; ++i)
      if (g.shadow[i]) return -1;
  }
  if (g.C < 1 || g.C > CNN_MAXC || g.cin < 1 || g.cin > 4 || g.classes < 1 || g.classes > 16) return -1;
  g.wstage = g.bf16 ? (g.C == 10 ? 2 : 1) : 0;
  if (g.wstage == 1 && cnn_lds_bytes(g) > 160 * 1024) g.wstage = 0;  // the weights then stay global
  // the fused tail reuses the kernel's LDS: the allocation covers the larger of the two (the
  // body's ~125 KiB already keeps one workgroup per CU, so a few KiB more cost no occupancy)
  size_t lds = cnn_lds_bytes(g);
  if (g.fused) lds = std::max(lds, cnn_tail_lds(g.C, g.cin, g.classes, g.B));
  if (lds > 160 * 1024) return -1;
  // channel capacity 10 (the reference model's hidden_units) gets exact compile-time groups
  // (LDS residency caps C at 13 for 1-channel input, so no exact instance above 10)
  auto kern = g.bf16 ? (g.C == 10 ? cnn_kernel<10, true, true> : cnn_kernel<CNN_MAXC, false, true>)
                     : (g.C == 10 ? cnn_kernel<10, true, false> : cnn_kernel<CNN_MAXC, false, false>);
  hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3(g.hand ? (1 + CNN_HELPERS) * g.B : g.B), dim3(CNN_THREADS), lds, st, g);
  SMI_CHECK_LAUNCH();
}

// floats of one image's hand-off area for the weight-gradient helpers (0: helpers not available)
extern "C" int smi_cnn_hand_floats(int C) { return (C >= 1 && C <= CNN_MAXC) ? cnn_hand_f(C) : 0; }

// The fused step's batch limit: the counter block (CNN_MAXB) and the fused tail's LDS, which with the
// body's (dtype-dependent: the exact bf16 C = 10 instance keeps its fragment tables there, wstage 2
// — the same choice as smi_cnn) must fit one 160 KiB allocation.
extern "C" int smi_cnn_fused_ok(int C, int cin, int classes, int B, int bf16) {
  if (C < 1 || C > CNN_MAXC || cin < 1 || cin > 4 || classes < 1 || classes > 16) return 0;
  CNNArgs g{};
  g.C = C; g.cin = cin; g.classes = classes; g.bf16 = bf16;
  g.wstage = bf16 ? (C == 10 ? 2 : 1) : 0;
  if (g.wstage == 1 && cnn_lds_bytes(g) > 160 * 1024) g.wstage = 0;
  const int P = C * cin * 9 + C + 3 * (C * C * 9 + C) + classes * C * 49 + classes;
  return P % 4 == 0 && B >= 1 && B <= CNN_MAXB && std::max(cnn_lds_bytes(g), cnn_tail_lds(C, cin, classes, B)) <= 160 * 1024;
}
// the largest batch a fused step takes for this model and dtype (0: none)
extern "C" int smi_cnn_max_batch(int C, int cin, int classes, int bf16) {
  for (int B = CNN_MAXB; B >= 1; --B)
    if (smi_cnn_fused_ok(C, cin, classes, B, bf16)) return B;
  return 0;
}

extern "C" int smi_cnn_reduce(const CNNArgs* args, hipStream_t st) {
  const CNNArgs& g = *args;
  hipLaunchKernelGGL(cnn_reduce_kernel, dim3((g.P + 255) / 256), dim3(256), 0, st, g);
  SMI_CHECK_LAUNCH();
}
