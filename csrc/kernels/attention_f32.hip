// Fused scaled-dot-product attention at the REFERENCE precision: fp32 Q/K/V/O, fp32 scores,
// softmax and accumulation, exact fp32 products.  Products run on the bf16 matrix cores through
// the exact 3-way bf16 split (XS = 1, smi_split3.h: six v_mfma_f32_32x32x16_bf16 slice products
// per fp32 product; the owned rows are split once) — the default — or on the fp32-input matrix
// cores (XS = 0, v_mfma_f32_32x32x2_f32; smi_gemm_f32_algo(0)).  head_dim = 64.  Forward + dQ +
// dK/dV, no S x S tensor in HBM; outputs optionally also as split planes for the next GEMM.
//
// Reference semantics: transformer.py:12-25 (scaled_dot_product) as called by MultiHeadAttention
// (:74-83) and MultiHeadCrossAttention (:177-191), run in fp32 by pytorch_machine_translator.py
// (model built at :120 and trained at :129-196 with default fp32 modules).  Mask modes as in
// csrc/include/smi_attn_mask.h (Q6: "reference" = +1.0 on strictly-past keys).
//
// CDNA4 structure.  A 32x32x2 f32 MFMA takes 64 cycles, so the work per 32-key x 32-query block
// (64 MFMAs forward, 96 for dQ, 128 for dK/dV) dwarfs its softmax VALU (16 scores per lane) —
// the kernels are matrix-core bound and built so the MFMA stream has no bubbles:
//  * workgroup = 4 waves x 32 rows of the OWNED axis (queries: forward, dQ; keys: dK/dV); the
//    owned rows' Q (or K, V) stay in registers, lane l / l+32 hold the two 32-wide halves of row
//    l & 31 of the head dimension (k = 32h + s for step s);
//  * the STREAMED operand goes through double-buffered 32-row LDS chunks (register-staged float4
//    loads of chunk c+1 in flight under chunk c's MFMAs);
//  * scores are produced with the owned row on the lane (S^T = K Q^T in the forward), so the
//    online-softmax statistics are lane-local up to one permlane32 swap, and the accumulator of
//    the first product IS the B operand of the second: register s of the 32x32 accumulator holds
//    key (s&3) + 8(s>>2) + 4h, which is exactly the k the 32x32x2 MFMA takes from lane half h at
//    step s when the other operand is read in that key order (ds_read_b32 rows of the LDS image).
//  * outputs come out transposed (O^T = V^T P^T ...): each lane owns one row and stores 4
//    consecutive head-dim values per register group (16-B stores).
// LDS images: [32 rows][68 floats] for row-fragment (ds_read_b128, conflict-free at pitch 68)
// operands, [32][64] for column-only operands (ds_read_b32 rows, conflict-free at any pitch).
// 32-row chunks keep the staging registers at 16 per thread (64-row chunks spilled dK/dV).
#include <stdlib.h>

#include "smi_common.h"
#include "smi_attention.h"
#include "smi_attn_mask.h"
#include "smi_split3.h"

#define FCH 32    // rows per streamed chunk (= one 32-row MFMA block)
#define FPR 68    // padded pitch (floats) of row-fragment images
#define MF32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x2f32((a), (b), (c), 0, 0, 0)

struct FStage { float4 v[2]; };  // one 32 x 64 fp32 chunk = 2 float4 per thread

// Diagnostic build (-DATTN_STAMPS, tools/probes/attn_fwd_probe.hip): per-phase shader-clock sums
// of the staged forward, kept in registers and added once per wave at exit, plus each wave's
// s_memrealtime start / end (dispatch ramp and drain).
#ifdef ATTN_STAMPS
__device__ unsigned long long attn_stamps[8 * 4096];  // [wave][phase]: plain stores (same-address atomics
                                                     // from every wave queued at one L2 channel: 4x slower)
__device__ unsigned long long attn_wave_rt[2 * 4096];
#define AST_DECL long long ast_[8] = {0, 0, 0, 0, 0, 0, 0, 0}; const unsigned long long ast_rt0 = __builtin_amdgcn_s_memrealtime()
#define AST_T(v) long long v = clock64()
#define AST_ADD(i, t0, t1) (ast_[i] += (t1) - (t0))
#define AST_END()                                                                                      \
  do {                                                                                               \
    if ((threadIdx.x & 63) == 0) {                                                                   \
      const int wid_ = ((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6); \
      if (wid_ < 4096) {                                                                             \
        for (int i_ = 0; i_ < 8; ++i_) attn_stamps[8 * wid_ + i_] = (unsigned long long)ast_[i_];   \
        attn_wave_rt[2 * wid_] = ast_rt0; attn_wave_rt[2 * wid_ + 1] = __builtin_amdgcn_s_memrealtime(); \
      }                                                                                              \
    }                                                                                                \
  } while (0)
#else
#define AST_DECL
#define AST_T(v)
#define AST_ADD(i, t0, t1)
#define AST_END() do {} while (0)
#endif

__device__ __forceinline__ void fa_load_chunk(const float* __restrict__ base, long ss, int r0, int rmax, FStage& p) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = threadIdx.x + 256 * u;
    const int row = i >> 4, c = i & 15, r = r0 + row;
    p.v[u] = r < rmax ? *(const float4*)(base + (long)r * ss + c * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
template <int PITCH>
__device__ __forceinline__ void fa_store_chunk(float* img, const FStage& p) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = threadIdx.x + 256 * u;
    *(float4*)(img + (i >> 4) * PITCH + (i & 15) * 4) = p.v[u];
  }
}
// row fragment: f[s] = img[row0 + (lane & 31)][32h + s], s = 0..31 (eight ds_read_b128)
__device__ __forceinline__ void fa_rowfrag(const float* img, int row0, int lane, float (&f)[32]) {
  const float* p = img + (row0 + (lane & 31)) * FPR + 32 * (lane >> 5);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float4 t = *(const float4*)(p + 4 * q);
    f[4 * q] = t.x; f[4 * q + 1] = t.y; f[4 * q + 2] = t.z; f[4 * q + 3] = t.w;
  }
}
// column fragment in accumulator row order: f[s] = img[row0 + (s&3) + 8(s>>2) + 4h][col0 + (lane & 31)]
template <int PITCH>
__device__ __forceinline__ void fa_colfrag(const float* img, int row0, int col0, int lane, float (&f)[16]) {
  const float* p = img + (row0 + 4 * (lane >> 5)) * PITCH + col0 + (lane & 31);
#pragma unroll
  for (int s = 0; s < 16; ++s) f[s] = p[((s & 3) + 8 * (s >> 2)) * PITCH];
}
// own row of a global [rows][64] operand: f[s] = base[row][32h + s] (zero past rmax)
__device__ __forceinline__ void fa_ownrow(const float* __restrict__ base, long ss, int row, int rmax, int lane, float (&f)[32]) {
  const bool ok = row < rmax;
  const float* p = base + (long)row * ss + 32 * (lane >> 5);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float4 t = ok ? *(const float4*)(p + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
    f[4 * q] = t.x; f[4 * q + 1] = t.y; f[4 * q + 2] = t.z; f[4 * q + 3] = t.w;
  }
}
// store a transposed 32x32 accumulator tile: lane's row gets d = col0 + (r&3) + 8(r>>2) + 4h
__device__ __forceinline__ void fa_store_rowT(float* __restrict__ dst, const f32x16_t& a, int lane, float sc) {
  const int h = lane >> 5;
#pragma unroll
  for (int g = 0; g < 4; ++g)
    *(float4*)(dst + 8 * g + 4 * h) = make_float4(a[4 * g] * sc, a[4 * g + 1] * sc, a[4 * g + 2] * sc, a[4 * g + 3] * sc);
}
// the same tile as split planes (P: plane-0 element matching dst, planes ps apart)
__device__ __forceinline__ void fa_store_rowT_planes(unsigned short* __restrict__ P, long ps, const f32x16_t& a, int lane,
                                                     float sc) {
  const int h = lane >> 5;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    uint32_t h0, m0, l0, h1, m1, l1;
    split3_pair(a[4 * g] * sc, a[4 * g + 1] * sc, h0, m0, l0);
    split3_pair(a[4 * g + 2] * sc, a[4 * g + 3] * sc, h1, m1, l1);
    unsigned short* q = P + 8 * g + 4 * h;
    *(uint2*)q = make_uint2(h0, h1);
    *(uint2*)(q + ps) = make_uint2(m0, m1);
    *(uint2*)(q + 2 * ps) = make_uint2(l0, l1);
  }
}
__device__ __forceinline__ int fa_kl(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// ---------------------------------------------------------------------------------------------
// Forward: S^T = K Q^T (query on the lane), online softmax, O^T += V^T P^T.
template <int MODE, bool KPAD, int XS>
__global__ __launch_bounds__(256, 2) void attn_f32_fwd_kernel(AttnF32Args a) {
  __shared__ __attribute__((aligned(16))) float Ks[2][FCH * FPR];
  __shared__ __attribute__((aligned(16))) float Vs[2][FCH * 64];
  const int hh = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  const int qwave = blockIdx.x * 128 + w * 32;
  const int qi = qwave + (lane & 31);
  const float* Q = a.q + b * a.q_sb + hh * a.q_sh;
  const float* K = a.k + b * a.k_sb + hh * a.k_sh;
  const float* V = a.v + b * a.v_sb + hh * a.v_sh;
  const unsigned char* kp = a.kpad ? a.kpad + (long)b * a.Sk : nullptr;
  int kend = a.Sk;
  if (MODE == 2) kend = min(a.Sk, blockIdx.x * 128 + 128);
  const int nchunks = (kend + FCH - 1) / FCH;
  FStage pk, pv;
  fa_load_chunk(K, a.k_ss, 0, a.Sk, pk);
  fa_load_chunk(V, a.v_ss, 0, a.Sk, pv);
  float qf[32];
  fa_ownrow(Q, a.q_ss, qi, a.Sq, lane, qf);
  F32Pre<XS, 32> qs;  // the owned Q row split once (reused by every chunk)
  qs.set(qf);
  fa_store_chunk<FPR>(Ks[0], pk);
  fa_store_chunk<64>(Vs[0], pv);
  __syncthreads();
  float m = -INFINITY, l = 0.f;
  f32x16_t o[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1;
    const bool more = c + 1 < nchunks;
    if (more) { fa_load_chunk(K, a.k_ss, (c + 1) * FCH, a.Sk, pk); fa_load_chunk(V, a.v_ss, (c + 1) * FCH, a.Sk, pv); }
    const unsigned long long kmask = KPAD ? chunk_pad_mask(kp, c * FCH, a.Sk) : 0ull;
    do {
      const int kb = 0, k0 = c * FCH;
      float ub;
      const bool full = k0 + 32 <= a.Sk;
      const bool uni = uniform_bias<MODE, KPAD, 32>(k0, qwave, qwave + 31, full, ub);
      if (uni && ub == -INFINITY) break;  // every key of this block after every query (causal)
      f32x16_t s;
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = 0.f;
      {
        float kf[32];
        fa_rowfrag(Ks[buf], kb, lane, kf);
        s = f32_chain_pre<XS, 32>(kf, qf, qs, s);
      }
      float cmax = -INFINITY;
      if (uni) {
#pragma unroll
        for (int r = 0; r < 16; ++r) cmax = fmaxf(cmax, s[r]);
        cmax = cmax * a.scale_log2 + ub;
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kl = kb + fa_kl(r, h);
          s[r] = score_adj<MODE, KPAD>(s[r], qi, c * FCH + kl, kl, full, a.Sk, kmask, a.scale_log2);
          cmax = fmaxf(cmax, s[r]);
        }
      }
      cmax = smi_row32_swap_max(cmax);
      const float mnew = fmaxf(m, cmax);
      const float mref = (mnew == -INFINITY) ? 0.f : mnew;
      const float alpha = __builtin_amdgcn_exp2f(m - mref);
      float psum = 0.f;
      if (uni) {
        const float off = ub - mref;
#pragma unroll
        for (int r = 0; r < 16; ++r) { s[r] = __builtin_amdgcn_exp2f(fmaf(s[r], a.scale_log2, off)); psum += s[r]; }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) { s[r] = __builtin_amdgcn_exp2f(s[r] - mref); psum += s[r]; }
      }
      psum = smi_row32_swap_sum(psum);
      l = l * alpha + psum;
      m = mnew;
      float sv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) sv[r] = s[r];
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        o[dt] *= alpha;
        float vf[16];
        fa_colfrag<64>(Vs[buf], kb, dt * 32, lane, vf);
        o[dt] = f32_chain<XS, 16>(vf, sv, o[dt]);
      }
    } while (0);
    if (more) { fa_store_chunk<FPR>(Ks[buf ^ 1], pk); fa_store_chunk<64>(Vs[buf ^ 1], pv); }
    __syncthreads();
  }
  if (qi < a.Sq) {
    float* O = a.o + b * a.o_sb + hh * a.o_sh + (long)qi * a.o_ss;
    const float inv = l > 0.f ? 1.0f / l : 0.f;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) fa_store_rowT(O + dt * 32, o[dt], lane, inv);
    if (a.op) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) fa_store_rowT_planes(a.op + (O - a.o) + dt * 32, a.op_ps, o[dt], lane, inv);
    }
    if (h == 0) {
      const float mref = (m == -INFINITY) ? 0.f : m;
      a.lse[((long)b * a.H + hh) * a.Sq + qi] = l > 0.f ? mref + log2f(l) : INFINITY;
    }
  }
}

// dQ: S^T = K Q^T, dP^T = V dO^T, dS^T = P^T o (dP^T - delta), dQ^T += K^T dS^T; also writes
// delta = rowsum(dO * O) for the dK/dV kernel.
template <int MODE, bool KPAD, int XS>
__global__ __launch_bounds__(256, XS ? 1 : 2) void attn_f32_dq_kernel(AttnF32Args a) {
  __shared__ __attribute__((aligned(16))) float Ks[2][FCH * FPR];
  __shared__ __attribute__((aligned(16))) float Vs[2][FCH * FPR];
  const int hh = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  const int qwave = blockIdx.x * 128 + w * 32;
  const int qi = qwave + (lane & 31);
  const float* Q = a.q + b * a.q_sb + hh * a.q_sh;
  const float* K = a.k + b * a.k_sb + hh * a.k_sh;
  const float* V = a.v + b * a.v_sb + hh * a.v_sh;
  const float* dO = a.dout + b * a.o_sb + hh * a.o_sh;
  const float* Og = a.o + b * a.o_sb + hh * a.o_sh;
  const unsigned char* kp = a.kpad ? a.kpad + (long)b * a.Sk : nullptr;
  int kend = a.Sk;
  if (MODE == 2) kend = min(a.Sk, blockIdx.x * 128 + 128);
  const int nchunks = (kend + FCH - 1) / FCH;
  FStage pk, pv;
  fa_load_chunk(K, a.k_ss, 0, a.Sk, pk);
  fa_load_chunk(V, a.v_ss, 0, a.Sk, pv);
  float qf[32], df[32];
  fa_ownrow(Q, a.q_ss, qi, a.Sq, lane, qf);
  fa_ownrow(dO, a.o_ss, qi, a.Sq, lane, df);
  F32Pre<XS, 32> qs, ds;  // owned Q / dO rows split once
  qs.set(qf);
  ds.set(df);
  float dl;
  {
    float of[32];
    fa_ownrow(Og, a.o_ss, qi, a.Sq, lane, of);
    float sacc = 0.f;
#pragma unroll
    for (int t = 0; t < 32; ++t) sacc = fmaf(df[t], of[t], sacc);
    dl = smi_row32_swap_sum(sacc);
  }
  const long rbase = ((long)b * a.H + hh) * a.Sq;
  if (h == 0 && qi < a.Sq) a.delta[rbase + qi] = dl;
  const float lse = qi < a.Sq ? a.lse[rbase + qi] : INFINITY;
  fa_store_chunk<FPR>(Ks[0], pk);
  fa_store_chunk<FPR>(Vs[0], pv);
  __syncthreads();
  f32x16_t acc[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[dt][r] = 0.f;
  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1;
    const bool more = c + 1 < nchunks;
    if (more) { fa_load_chunk(K, a.k_ss, (c + 1) * FCH, a.Sk, pk); fa_load_chunk(V, a.v_ss, (c + 1) * FCH, a.Sk, pv); }
    const unsigned long long kmask = KPAD ? chunk_pad_mask(kp, c * FCH, a.Sk) : 0ull;
    do {
      const int kb = 0, k0 = c * FCH;
      float ub;
      const bool full = k0 + 32 <= a.Sk;
      const bool uni = uniform_bias<MODE, KPAD, 32>(k0, qwave, qwave + 31, full, ub);
      if (uni && ub == -INFINITY) break;
      f32x16_t s, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s[r] = 0.f; dp[r] = 0.f; }
      {
        float kf[32];
        fa_rowfrag(Ks[buf], kb, lane, kf);
        s = f32_chain_pre<XS, 32>(kf, qf, qs, s);
      }
      {
        float vf[32];
        fa_rowfrag(Vs[buf], kb, lane, vf);
        dp = f32_chain_pre<XS, 32>(vf, df, ds, dp);
      }
      if (uni) {
        const float off = ub - lse;
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = __builtin_amdgcn_exp2f(fmaf(s[r], a.scale_log2, off)) * (dp[r] - dl);
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kl = kb + fa_kl(r, h);
          const float x = score_adj<MODE, KPAD>(s[r], qi, c * FCH + kl, kl, full, a.Sk, kmask, a.scale_log2);
          s[r] = __builtin_amdgcn_exp2f(x - lse) * (dp[r] - dl);  // exp2(-inf) = 0 for masked entries
        }
      }
      float sv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) sv[r] = s[r];
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        float kc[16];
        fa_colfrag<FPR>(Ks[buf], kb, dt * 32, lane, kc);
        acc[dt] = f32_chain<XS, 16>(kc, sv, acc[dt]);
      }
    } while (0);
    if (more) { fa_store_chunk<FPR>(Ks[buf ^ 1], pk); fa_store_chunk<FPR>(Vs[buf ^ 1], pv); }
    __syncthreads();
  }
  if (qi < a.Sq) {
    float* dQ = a.dq + b * a.q_sb + hh * a.q_sh + (long)qi * a.q_ss;
    if (!a.no_f32_grad) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) fa_store_rowT(dQ + dt * 32, acc[dt], lane, a.scale);
    }
    if (a.dqp) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) fa_store_rowT_planes(a.dqp + (dQ - a.dq) + dt * 32, a.dq_ps, acc[dt], lane, a.scale);
    }
  }
}

// dK, dV: key on the lane.  S = Q K^T, dP = dO V^T, P = exp2(S' - lse), dS = P o (dP - delta),
// dV^T += dO^T P, dK^T += Q^T dS.
template <int MODE, bool KPAD, int XS>
__global__ __launch_bounds__(256, XS ? 1 : 2) void attn_f32_dkdv_kernel(AttnF32Args a) {
  __shared__ __attribute__((aligned(16))) float Qs[2][FCH * FPR];
  __shared__ __attribute__((aligned(16))) float Ds[2][FCH * FPR];
  __shared__ float lse_s[2][FCH], dl_s[2][FCH];
  const int hh = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  const int kwave = blockIdx.x * 128 + w * 32;
  const int kj = kwave + (lane & 31);
  const float* Q = a.q + b * a.q_sb + hh * a.q_sh;
  const float* K = a.k + b * a.k_sb + hh * a.k_sh;
  const float* V = a.v + b * a.v_sb + hh * a.v_sh;
  const float* dO = a.dout + b * a.o_sb + hh * a.o_sh;
  const long rbase = ((long)b * a.H + hh) * a.Sq;
  int qstart = 0;
  if (MODE == 2) qstart = (blockIdx.x * 128) & ~(FCH - 1);
  const int nchunks = qstart < a.Sq ? (a.Sq - qstart + FCH - 1) / FCH : 0;
  FStage pq, pd;
  float lse_r = INFINITY, dl_r = 0.f;
  if (nchunks) {
    fa_load_chunk(Q, a.q_ss, qstart, a.Sq, pq);
    fa_load_chunk(dO, a.o_ss, qstart, a.Sq, pd);
    if (threadIdx.x < FCH && qstart + (int)threadIdx.x < a.Sq) {
      lse_r = a.lse[rbase + qstart + threadIdx.x];
      dl_r = a.delta[rbase + qstart + threadIdx.x];
    }
  }
  float kf[32], vf[32];
  fa_ownrow(K, a.k_ss, kj, a.Sk, lane, kf);
  fa_ownrow(V, a.v_ss, kj, a.Sk, lane, vf);
  F32Pre<XS, 32> ks, vs;  // owned K / V rows split once
  ks.set(kf);
  vs.set(vf);
  const bool kok = kj < a.Sk && !(KPAD && a.kpad[(long)b * a.Sk + kj]);
  const float kbias = kok ? 0.f : -INFINITY;
  f32x16_t dk[2], dv[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dk[dt][r] = 0.f; dv[dt][r] = 0.f; }
  if (nchunks) {
    fa_store_chunk<FPR>(Qs[0], pq);
    fa_store_chunk<FPR>(Ds[0], pd);
    if (threadIdx.x < FCH) { lse_s[0][threadIdx.x] = lse_r; dl_s[0][threadIdx.x] = dl_r; }
  }
  __syncthreads();
  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1, q0 = qstart + c * FCH;
    const bool more = c + 1 < nchunks;
    if (more) {
      fa_load_chunk(Q, a.q_ss, q0 + FCH, a.Sq, pq);
      fa_load_chunk(dO, a.o_ss, q0 + FCH, a.Sq, pd);
      lse_r = INFINITY; dl_r = 0.f;
      if (threadIdx.x < FCH && q0 + FCH + (int)threadIdx.x < a.Sq) {
        lse_r = a.lse[rbase + q0 + FCH + threadIdx.x];
        dl_r = a.delta[rbase + q0 + FCH + threadIdx.x];
      }
    }
    do {
      const int qb = 0;
      if (MODE == 2 && q0 + 31 < kwave) break;  // every query of the block before every key
      f32x16_t s, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s[r] = 0.f; dp[r] = 0.f; }
      {
        float qr[32];
        fa_rowfrag(Qs[buf], qb, lane, qr);
        s = f32_chain_pre<XS, 32>(qr, kf, ks, s);
      }
      {
        float dr[32];
        fa_rowfrag(Ds[buf], qb, lane, dr);
        dp = f32_chain_pre<XS, 32>(dr, vf, vs, dp);
      }
      // s[r]: query q0 + qb + fa_kl(r, h), key kj.  Rows past Sq carry lse = +inf (p = 0).
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ql = qb + fa_kl(r, h);
        const int qq = q0 + ql;
        float x = fmaf(s[r], a.scale_log2, kbias);
        if (MODE == 1) x += (kj < qq) ? LOG2E_F : 0.f;
        if (MODE == 2) x = (kj > qq) ? -INFINITY : x;
        const float p = __builtin_amdgcn_exp2f(x - lse_s[buf][ql]);
        s[r] = p;
        dp[r] = p * (dp[r] - dl_s[buf][ql]);
      }
      float sv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) sv[r] = s[r];
      float dpv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) dpv[r] = dp[r];
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        float dc[16];
        fa_colfrag<FPR>(Ds[buf], qb, dt * 32, lane, dc);
        dv[dt] = f32_chain<XS, 16>(dc, sv, dv[dt]);
        float qc[16];
        fa_colfrag<FPR>(Qs[buf], qb, dt * 32, lane, qc);
        dk[dt] = f32_chain<XS, 16>(qc, dpv, dk[dt]);
      }
    } while (0);
    if (more) {
      fa_store_chunk<FPR>(Qs[buf ^ 1], pq);
      fa_store_chunk<FPR>(Ds[buf ^ 1], pd);
      if (threadIdx.x < FCH) { lse_s[buf ^ 1][threadIdx.x] = lse_r; dl_s[buf ^ 1][threadIdx.x] = dl_r; }
    }
    __syncthreads();
  }
  if (kj < a.Sk) {
    float* dK = a.dk + b * a.k_sb + hh * a.k_sh + (long)kj * a.k_ss;
    float* dV = a.dv + b * a.v_sb + hh * a.v_sh + (long)kj * a.v_ss;
    if (!a.no_f32_grad) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        fa_store_rowT(dK + dt * 32, dk[dt], lane, a.scale);
        fa_store_rowT(dV + dt * 32, dv[dt], lane, 1.0f);
      }
    }
    if (a.dkp) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        fa_store_rowT_planes(a.dkp + (dK - a.dk) + dt * 32, a.dkv_ps, dk[dt], lane, a.scale);
        fa_store_rowT_planes(a.dvp + (dV - a.dv) + dt * 32, a.dkv_ps, dv[dt], lane, 1.0f);
      }
    }
  }
}


// ---------------------------------------------------------------------------------------------
// STAGED-PLANE kernels (the default; smi_attn_f32_sp): the same three passes and accumulation
// order, but every streamed 32-row chunk is split into bf16 hi / mid / lo planes ONCE, while it
// is staged into LDS (each thread splits the 8 values it loads), instead of every wave splitting
// every fragment it reads (the XS = 1 kernels re-split each streamed value per wave and per use:
// VALU-bound at ~40 % of the split ceiling).  Fragments then come out of LDS as ready bf16
// operands: row fragments (k = head dim) by ds_read_b128, column fragments (k = the streamed
// rows) by ds_read_b64_tr_b16; six v_mfma_f32_32x32x16_bf16 per fragment pair.  Only the
// per-block P / dS values (computed in registers) are split in the loop.
//
// LDS image per operand plane: [32 rows][64] bf16, 128-B rows, 16-B chunk c stored at
// c ^ as_sw(row), as_sw(r) = ((r >> 1) & 1) << 2 | ((r >> 2) & 3): conflict-free both for the
// row-fragment reads (each 16-lane ds_read_b128 group reads one chunk of 16 rows: same-parity
// rows get 8 distinct swizzles) and for the column-fragment reads (each 32-lane transpose group
// reads 4 consecutive rows x 4 chunks: rows r and r + 2 land in opposite chunk halves).
// Column fragments take the streamed rows in the ACCUMULATOR's order: k-step t, lane half h,
// slot j <-> row 16 t + (j & 3) + 8 (j >> 2) + 4 h — the rows lane (n, h) holds in registers
// 8 t .. 8 t + 7 of a 32 x 32 accumulator — so P / dS feed the second product straight from
// registers.
#define AS_PL (32 * 64)
#define AS_OP (3 * AS_PL)
typedef __attribute__((ext_vector_type(4))) short as_s16x4_t;

__device__ __forceinline__ int as_sw(int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ int as_off(int r, int c) { return r * 64 + ((((c >> 3) ^ as_sw(r)) & 7) << 3) + (c & 7); }

struct AStage { float4 v[2]; };
// thread t (< 256) loads 8 consecutive floats: row t >> 3, columns 8 (t & 7) .. + 7 (rows >= rmax: zero)
__device__ __forceinline__ void as_load(const float* __restrict__ base, long ss, int r0, int rmax, AStage& p,
                                        int ti = -1) {
  if (ti < 0) ti = threadIdx.x;
  const int r = ti >> 3, c = (ti & 7) * 8;
  if (r0 + r < rmax) {
    const float* q = base + (long)(r0 + r) * ss + c;
    p.v[0] = *(const float4*)q;
    p.v[1] = *(const float4*)(q + 4);
  } else {
    p.v[0] = p.v[1] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
__device__ __forceinline__ void as_store(unsigned short* img, const AStage& p, int ti = -1) {
  if (ti < 0) ti = threadIdx.x;
  const int r = ti >> 3, c = (ti & 7) * 8;
  const float f[8] = {p.v[0].x, p.v[0].y, p.v[0].z, p.v[0].w, p.v[1].x, p.v[1].y, p.v[1].z, p.v[1].w};
  const Split3 sp = split3_8(f);
  const int o = as_off(r, c);
  *(bf16x8_t*)(img + o) = sp.h;
  *(bf16x8_t*)(img + AS_PL + o) = sp.m;
  *(bf16x8_t*)(img + 2 * AS_PL + o) = sp.l;
}
// one operand's fp32 source: staged loads / owned rows (split once per kernel)
struct AsSrc {
  const float* f; long ss;
  __device__ __forceinline__ void load(int r0, int rmax, AStage& st, int ti = -1) const { as_load(f, ss, r0, rmax, st, ti); }
  // the owned row as ready operands (F32Pre order: s[j] = head dims 32 h + 8 j .. + 7)
  __device__ __forceinline__ void own(int row, int rmax, int lane, F32Pre<1, 32>& o) const {
    float v[32];
    fa_ownrow(f, ss, row, rmax, lane, v);
    o.set(v);
  }
  __device__ __forceinline__ void own_f32(int row, int rmax, int lane, float (&v)[32]) const {
    fa_ownrow(f, ss, row, rmax, lane, v);
  }
};

// A operand, rows = streamed rows (lane & 31), k-step j: head dims 32 h + 8 j .. + 7 (the owned
// operand's F32Pre order)
__device__ __forceinline__ Split3 as_rowfrag(const unsigned short* img, int lane, int j) {
  const int o = as_off(lane & 31, 32 * (lane >> 5) + 8 * j);
  Split3 r;
  r.h = *(const bf16x8_t*)(img + o);
  r.m = *(const bf16x8_t*)(img + AS_PL + o);
  r.l = *(const bf16x8_t*)(img + 2 * AS_PL + o);
  return r;
}
// A operand, rows = head dims 32 dt + (lane & 31), k-step t over the streamed rows (accumulator order)
__device__ __forceinline__ Split3 as_colfrag(const unsigned short* img, int lane, int dt, int t) {
  const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4;
  const int col = 32 * dt + 16 * (g & 1) + 4 * p;
  const int r0 = 16 * t + 4 * (g >> 1) + q;
  const int o0 = as_off(r0, col), o1 = as_off(r0 + 8, col);
  Split3 r;
  bf16x8_t* outs[3] = {&r.h, &r.m, &r.l};
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) {
    const unsigned short* b = img + pl * AS_PL;
    const as_s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) as_s16x4_t*)(b + o0));
    const as_s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) as_s16x4_t*)(b + o1));
    *outs[pl] = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
  }
  return r;
}
// acc += a . b, six slice products smallest first (the XS = 1 chains' order)
__device__ __forceinline__ f32x16_t as_mma(const Split3& a, const Split3& b, f32x16_t acc) {
  acc = MF32X16(a.l, b.h, acc);
  acc = MF32X16(a.m, b.m, acc);
  acc = MF32X16(a.h, b.l, acc);
  acc = MF32X16(a.m, b.h, acc);
  acc = MF32X16(a.h, b.m, acc);
  return MF32X16(a.h, b.h, acc);
}
// rows x owned: sum over the 64 head dims of (streamed row-fragment) x (owned split row)
__device__ __forceinline__ f32x16_t as_rows_dot(const unsigned short* img, int lane, const F32Pre<1, 32>& own,
                                                f32x16_t acc) {
#pragma unroll
  for (int j = 0; j < 4; ++j) acc = as_mma(as_rowfrag(img, lane, j), own.s[j], acc);
  return acc;
}
// acc[dt] += (streamed columns)^T . v, v = the 16 per-lane accumulator values (split here)
__device__ __forceinline__ void as_cols_acc(const unsigned short* img, int lane, const float (&v)[16], f32x16_t (&acc)[2]) {
  const Split3 b0 = split3_8(&v[0]), b1 = split3_8(&v[8]);
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    acc[dt] = as_mma(as_colfrag(img, lane, dt, 0), b0, acc[dt]);
    acc[dt] = as_mma(as_colfrag(img, lane, dt, 1), b1, acc[dt]);
  }
}

// Row-coalesced epilogue (the kernels' transposed outputs O^T / dQ^T / dK^T / dV^T): lane (row
// l & 31, half h) holds head dims 32 dt + 8 g + 4 h + e in register 4 g + e of acc[dt], so a direct
// store writes one 16-B piece of 32 different rows per instruction (row stride apart: every
// store touches 32-64 cache lines, and the all-CU store burst at the end of the kernel is
// issue-bound).  Instead the wave stages its 32 x 64 tile in a private LDS image (pitch 68:
// conflict-free float4 rows) and stores whole rows: fp32 as 256-B row segments (4 rows per wave
// instruction), planes as 128-B row segments (8 rows per instruction, each lane splitting 8
// consecutive values).  Bitwise the same values as the direct stores.
#define AE_PITCH 68
#define AE_FLOATS (32 * AE_PITCH)
__device__ __forceinline__ void ae_stage(float* img, const f32x16_t (&acc)[2], int lane, float sc) {
  const int row = lane & 31, h = lane >> 5;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *(float4*)(img + row * AE_PITCH + 32 * dt + 8 * g + 4 * h) =
          make_float4(acc[dt][4 * g] * sc, acc[dt][4 * g + 1] * sc, acc[dt][4 * g + 2] * sc, acc[dt][4 * g + 3] * sc);
}
// dst / P: row 0 of the wave's 32 rows (fp32 output / plane 0, either may be null), rows ss apart
__device__ __forceinline__ void ae_store(const float* img, float* __restrict__ dst, unsigned short* __restrict__ P, long ss,
                                         long ps, int nrows, int lane) {
  if (dst) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int row = 4 * k + (lane >> 4), c = 4 * (lane & 15);
      if (row < nrows) *(float4*)(dst + (long)row * ss + c) = *(const float4*)(img + row * AE_PITCH + c);
    }
  }
  if (P) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int row = 8 * k + (lane >> 3), c = 8 * (lane & 7);
      if (row < nrows) {
        const float4 v0 = *(const float4*)(img + row * AE_PITCH + c), v1 = *(const float4*)(img + row * AE_PITCH + c + 4);
        const float f[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        const Split3 sp = split3_8(f);
        unsigned short* q = P + (long)row * ss + c;
        *(bf16x8_t*)q = sp.h;
        *(bf16x8_t*)(q + ps) = sp.m;
        *(bf16x8_t*)(q + 2 * ps) = sp.l;
      }
    }
  }
}

// operand source of batch b, head hh
#define AS_SRC(NAME, FP, SB, SH, SS) const AsSrc NAME{(FP) + b * (SB) + hh * (SH), (SS)}

// Forward: four waves of 32 queries per workgroup, two workgroups per CU; K / V streamed in
// 32-row chunks through double-buffered staged planes (an 8-wave variant with one staged chunk
// per 256 queries, and a staggered one, measured no faster in the step: round 4).
template <int MODE, bool KPAD>
__global__ __launch_bounds__(256, 2) void attn_sp_fwd4(AttnF32Args a) {
  constexpr int QW = 128;  // queries per workgroup
  __shared__ __attribute__((aligned(16))) unsigned short Ks[2][AS_OP];
  __shared__ __attribute__((aligned(16))) unsigned short Vs[2][AS_OP];
  AST_DECL;
  AST_T(tk0);
  const int hh = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  const int qwave = blockIdx.x * QW + w * 32;
  const int qi = qwave + (lane & 31);
  AS_SRC(Q, a.q, a.q_sb, a.q_sh, a.q_ss);
  AS_SRC(K, a.k, a.k_sb, a.k_sh, a.k_ss);
  AS_SRC(V, a.v, a.v_sb, a.v_sh, a.v_ss);
  const unsigned char* kp = a.kpad ? a.kpad + (long)b * a.Sk : nullptr;
  int kend = a.Sk;
  if (MODE == 2) kend = min(a.Sk, blockIdx.x * QW + QW);
  const int nchunks = (kend + FCH - 1) / FCH;
  // chunk staging: every thread stages 8 values of K and 8 of V
  AStage pk, pv;
  auto stage_load = [&](int r0) { K.load(r0, a.Sk, pk); V.load(r0, a.Sk, pv); };
  auto stage_store = [&](int bf) { as_store(Ks[bf], pk); as_store(Vs[bf], pv); };
  stage_load(0);
  F32Pre<1, 32> qs;
  Q.own(qi, a.Sq, lane, qs);
  stage_store(0);
  __syncthreads();
  AST_T(tk1);
  AST_ADD(0, tk0, tk1);  // prologue
  float m = -INFINITY, l = 0.f;
  f32x16_t o[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1;
    const bool more = c + 1 < nchunks;
    AST_T(tc0);
    if (more) stage_load((c + 1) * FCH);
    const unsigned long long kmask = KPAD ? chunk_pad_mask(kp, c * FCH, a.Sk) : 0ull;
    AST_T(tc1);
    AST_ADD(1, tc0, tc1);  // next chunk's load issue
    do {
      const int k0 = c * FCH;
      float ub;
      const bool full = k0 + 32 <= a.Sk;
      const bool uni = uniform_bias<MODE, KPAD, 32>(k0, qwave, qwave + 31, full, ub);
      if (uni && ub == -INFINITY) break;
      f32x16_t s;
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = 0.f;
      s = as_rows_dot(Ks[buf], lane, qs, s);  // S^T = K Q^T: key rows, query on the lane
      float cmax = -INFINITY;
      if (uni) {
#pragma unroll
        for (int r = 0; r < 16; ++r) cmax = fmaxf(cmax, s[r]);
        cmax = cmax * a.scale_log2 + ub;
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kl = fa_kl(r, h);
          s[r] = score_adj<MODE, KPAD>(s[r], qi, k0 + kl, kl, full, a.Sk, kmask, a.scale_log2);
          cmax = fmaxf(cmax, s[r]);
        }
      }
      cmax = smi_row32_swap_max(cmax);
      const float mnew = fmaxf(m, cmax);
      const float mref = (mnew == -INFINITY) ? 0.f : mnew;
      const float alpha = __builtin_amdgcn_exp2f(m - mref);
      float psum = 0.f;
      float pv16[16];
      if (uni) {
        const float off = ub - mref;
#pragma unroll
        for (int r = 0; r < 16; ++r) { pv16[r] = __builtin_amdgcn_exp2f(fmaf(s[r], a.scale_log2, off)); psum += pv16[r]; }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) { pv16[r] = __builtin_amdgcn_exp2f(s[r] - mref); psum += pv16[r]; }
      }
      psum = smi_row32_swap_sum(psum);
      l = l * alpha + psum;
      m = mnew;
      AST_T(tc2);
      AST_ADD(2, tc1, tc2);  // S chain + online softmax
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) o[dt] *= alpha;
      as_cols_acc(Vs[buf], lane, pv16, o);  // O^T += V^T P^T
      AST_T(tc3);
      AST_ADD(3, tc2, tc3);  // rescale (waits for the previous PV) + P split + PV issue
    } while (0);
    AST_T(tc4);
    if (more) stage_store(buf ^ 1);
    AST_T(tc5);
    AST_ADD(4, tc4, tc5);  // wait for the chunk's loads, split, LDS stores
    __syncthreads();
    AST_T(tc6);
    AST_ADD(5, tc5, tc6);  // barrier
  }
  AST_T(tk2);
  const float inv = l > 0.f ? 1.0f / l : 0.f;
  if (a.ae16) {
    // row-coalesced stores through the (now free) K / V staging buffers: 4 x 8.5 KiB of 48 KiB
    float* img = (float*)(w < 2 ? &Ks[0][0] : &Vs[0][0]) + (w & 1) * AE_FLOATS;  // 2 x 8.5 of 24 KiB each
    ae_stage(img, o, lane, inv);
    __syncthreads();
    const long r0 = (long)b * a.o_sb + hh * a.o_sh + (long)qwave * a.o_ss;
    ae_store(img, a.o + r0, a.op ? a.op + r0 : nullptr, a.o_ss, a.op_ps, a.Sq - qwave, lane);
  } else if (qi < a.Sq) {
    float* O = a.o + b * a.o_sb + hh * a.o_sh + (long)qi * a.o_ss;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) fa_store_rowT(O + dt * 32, o[dt], lane, inv);
    if (a.op) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) fa_store_rowT_planes(a.op + (O - a.o) + dt * 32, a.op_ps, o[dt], lane, inv);
    }
  }
  if (qi < a.Sq && h == 0) {
    const float mref = (m == -INFINITY) ? 0.f : m;
    a.lse[((long)b * a.H + hh) * a.Sq + qi] = l > 0.f ? mref + log2f(l) : INFINITY;
  }
  AST_T(tk3);
  AST_ADD(6, tk2, tk3);  // epilogue stores
  AST_ADD(7, tk0, tk3);  // wave lifetime
  AST_END();
}

template <int MODE, bool KPAD>
__global__ __launch_bounds__(256, 2) void attn_sp_dq_kernel(AttnF32Args a) {
  __shared__ __attribute__((aligned(16))) unsigned short Ks[2][AS_OP];
  __shared__ __attribute__((aligned(16))) unsigned short Vs[2][AS_OP];
  const int hh = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  const int qwave = blockIdx.x * 128 + w * 32;
  const int qi = qwave + (lane & 31);
  AS_SRC(Q, a.q, a.q_sb, a.q_sh, a.q_ss);
  AS_SRC(K, a.k, a.k_sb, a.k_sh, a.k_ss);
  AS_SRC(V, a.v, a.v_sb, a.v_sh, a.v_ss);
  AS_SRC(dO, a.dout, a.o_sb, a.o_sh, a.o_ss);
  const float* Og = a.o + b * a.o_sb + hh * a.o_sh;
  const unsigned char* kp = a.kpad ? a.kpad + (long)b * a.Sk : nullptr;
  int kend = a.Sk;
  if (MODE == 2) kend = min(a.Sk, blockIdx.x * 128 + 128);
  const int nchunks = (kend + FCH - 1) / FCH;
  AStage pk, pv;
  K.load(0, a.Sk, pk);
  V.load(0, a.Sk, pv);
  F32Pre<1, 32> qs, ds;
  float dl;
  {
    float df[32], of[32];
    Q.own(qi, a.Sq, lane, qs);
    dO.own(qi, a.Sq, lane, ds);
    dO.own_f32(qi, a.Sq, lane, df);
    fa_ownrow(Og, a.o_ss, qi, a.Sq, lane, of);
    float sacc = 0.f;
#pragma unroll
    for (int t = 0; t < 32; ++t) sacc = fmaf(df[t], of[t], sacc);
    dl = smi_row32_swap_sum(sacc);
  }
  const long rbase = ((long)b * a.H + hh) * a.Sq;
  if (h == 0 && qi < a.Sq) a.delta[rbase + qi] = dl;
  const float lse = qi < a.Sq ? a.lse[rbase + qi] : INFINITY;
  as_store(Ks[0], pk);
  as_store(Vs[0], pv);
  __syncthreads();
  f32x16_t acc[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[dt][r] = 0.f;
  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1;
    const bool more = c + 1 < nchunks;
    if (more) { K.load((c + 1) * FCH, a.Sk, pk); V.load((c + 1) * FCH, a.Sk, pv); }
    const unsigned long long kmask = KPAD ? chunk_pad_mask(kp, c * FCH, a.Sk) : 0ull;
    do {
      const int k0 = c * FCH;
      float ub;
      const bool full = k0 + 32 <= a.Sk;
      const bool uni = uniform_bias<MODE, KPAD, 32>(k0, qwave, qwave + 31, full, ub);
      if (uni && ub == -INFINITY) break;
      f32x16_t s, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s[r] = 0.f; dp[r] = 0.f; }
      s = as_rows_dot(Ks[buf], lane, qs, s);   // S^T = K Q^T
      dp = as_rows_dot(Vs[buf], lane, ds, dp);  // dP^T = V dO^T
      float dsv[16];
      if (uni) {
        const float off = ub - lse;
#pragma unroll
        for (int r = 0; r < 16; ++r) dsv[r] = __builtin_amdgcn_exp2f(fmaf(s[r], a.scale_log2, off)) * (dp[r] - dl);
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kl = fa_kl(r, h);
          const float x = score_adj<MODE, KPAD>(s[r], qi, k0 + kl, kl, full, a.Sk, kmask, a.scale_log2);
          dsv[r] = __builtin_amdgcn_exp2f(x - lse) * (dp[r] - dl);  // exp2(-inf) = 0 for masked entries
        }
      }
      as_cols_acc(Ks[buf], lane, dsv, acc);  // dQ^T += K^T dS^T
    } while (0);
    if (more) { as_store(Ks[buf ^ 1], pk); as_store(Vs[buf ^ 1], pv); }
    __syncthreads();
  }
  if (a.ae16) {
    // staging buffers free after the loop's last barrier: waves 0-1 in Ks, 2-3 in Vs (2 x 8.5 of 24 KiB)
    float* img = (float*)(w < 2 ? &Ks[0][0] : &Vs[0][0]) + (w & 1) * AE_FLOATS;
    ae_stage(img, acc, lane, a.scale);
    __syncthreads();
    const long r0 = (long)b * a.q_sb + hh * a.q_sh + (long)qwave * a.q_ss;
    ae_store(img, a.no_f32_grad ? nullptr : a.dq + r0, a.dqp ? a.dqp + r0 : nullptr, a.q_ss, a.dq_ps, a.Sq - qwave,
             lane);
  } else if (qi < a.Sq) {
    float* dQ = a.dq + b * a.q_sb + hh * a.q_sh + (long)qi * a.q_ss;
    if (!a.no_f32_grad) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) fa_store_rowT(dQ + dt * 32, acc[dt], lane, a.scale);
    }
    if (a.dqp) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) fa_store_rowT_planes(a.dqp + (dQ - a.dq) + dt * 32, a.dq_ps, acc[dt], lane, a.scale);
    }
  }
}

// dK / dV with EIGHT waves per workgroup (256 keys: a whole head at S = 256), two waves per SIMD.
// The 4-wave kernel above needs > 256 registers per lane (owned K and V splits, dK / dV
// accumulators, P / dS splits), so it runs one wave per SIMD with every LDS / MFMA / exp latency
// exposed, in two rounds of 256 workgroups.  Here the owned V rows live in LDS instead (a [32 keys]
// [64] plane image per wave, read back as the dP product's B fragments exactly like a staged
// chunk's row fragments: 12 extra ds_read_b128 per chunk), which fits two waves per SIMD, and each
// staged Q / dO chunk serves 256 keys instead of 128 (threads 0-255 stage Q, 256-511 dO).
// LDS: 2 x 2 x 12 KiB staging + 8 x 12 KiB owned V = 144 KiB.
#define AS_DKDV8_KEYS 256
template <int MODE, bool KPAD>
__global__ __launch_bounds__(512, 1) void attn_sp_dkdv8_kernel(AttnF32Args a) {
  __shared__ __attribute__((aligned(16))) unsigned short Qs[2][AS_OP];
  __shared__ __attribute__((aligned(16))) unsigned short Ds[2][AS_OP];
  __shared__ __attribute__((aligned(16))) unsigned short Vo[8][AS_OP];
  __shared__ float lse_s[2][FCH], dl_s[2][FCH];
  const int hh = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
  const int kb0 = blockIdx.x * AS_DKDV8_KEYS;
  const int kwave = kb0 + w * 32;
  const int kj = kwave + (lane & 31);
  const bool stq = tid < 256;  // this thread stages Q (waves 0-3) or dO (waves 4-7)
  const int ti = tid & 255;
  AS_SRC(Q, a.q, a.q_sb, a.q_sh, a.q_ss);
  AS_SRC(K, a.k, a.k_sb, a.k_sh, a.k_ss);
  AS_SRC(V, a.v, a.v_sb, a.v_sh, a.v_ss);
  AS_SRC(dO, a.dout, a.o_sb, a.o_sh, a.o_ss);
  const AsSrc& SQ = stq ? Q : dO;
  const long rbase = ((long)b * a.H + hh) * a.Sq;
  int qstart = 0;
  if (MODE == 2) qstart = kb0 & ~(FCH - 1);
  const int nchunks = qstart < a.Sq ? (a.Sq - qstart + FCH - 1) / FCH : 0;
  AStage ps;
  float lse_r = INFINITY, dl_r = 0.f;
  if (nchunks) {
    SQ.load(qstart, a.Sq, ps, ti);
    if (tid < FCH && qstart + tid < a.Sq) {
      lse_r = a.lse[rbase + qstart + tid];
      dl_r = a.delta[rbase + qstart + tid];
    }
  }
  // owned V rows of the block -> the eight per-wave plane images (four 32-row passes of 512 threads)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = tid + 512 * i, blk = idx >> 8;
    AStage pv;
    V.load(kb0 + 32 * blk, a.Sk, pv, idx & 255);
    as_store(Vo[blk], pv, idx & 255);
  }
  F32Pre<1, 32> ks;
  K.own(kj, a.Sk, lane, ks);
  const bool kok = kj < a.Sk && !(KPAD && a.kpad[(long)b * a.Sk + kj]);
  const float kbias = kok ? 0.f : -INFINITY;
  f32x16_t dk[2], dv[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dk[dt][r] = 0.f; dv[dt][r] = 0.f; }
  if (nchunks) {
    as_store(stq ? Qs[0] : Ds[0], ps, ti);
    if (tid < FCH) { lse_s[0][tid] = lse_r; dl_s[0][tid] = dl_r; }
  }
  __syncthreads();
  const unsigned short* vimg = Vo[w];
  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1, q0 = qstart + c * FCH;
    const bool more = c + 1 < nchunks;
    if (more) {
      SQ.load(q0 + FCH, a.Sq, ps, ti);
      lse_r = INFINITY; dl_r = 0.f;
      if (tid < FCH && q0 + FCH + tid < a.Sq) {
        lse_r = a.lse[rbase + q0 + FCH + tid];
        dl_r = a.delta[rbase + q0 + FCH + tid];
      }
    }
    do {
      if (MODE == 2 && q0 + 31 < kwave) break;  // every query of the chunk before every key of the wave
      f32x16_t s, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s[r] = 0.f; dp[r] = 0.f; }
      s = as_rows_dot(Qs[buf], lane, ks, s);  // S = Q K^T: query rows, key on the lane
#pragma unroll
      for (int j = 0; j < 4; ++j)  // dP = dO V^T, V's fragments from the wave's LDS image
        dp = as_mma(as_rowfrag(Ds[buf], lane, j), as_rowfrag(vimg, lane, j), dp);
      float pvv[16], dsv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ql = fa_kl(r, h);
        const int qq = q0 + ql;
        float x = fmaf(s[r], a.scale_log2, kbias);
        if (MODE == 1) x += (kj < qq) ? LOG2E_F : 0.f;
        if (MODE == 2) x = (kj > qq) ? -INFINITY : x;
        const float pr = __builtin_amdgcn_exp2f(x - lse_s[buf][ql]);  // rows past Sq: lse = +inf -> 0
        pvv[r] = pr;
        dsv[r] = pr * (dp[r] - dl_s[buf][ql]);
      }
      as_cols_acc(Ds[buf], lane, pvv, dv);  // dV^T += dO^T P
      as_cols_acc(Qs[buf], lane, dsv, dk);  // dK^T += Q^T dS
    } while (0);
    if (more) {
      as_store(stq ? Qs[buf ^ 1] : Ds[buf ^ 1], ps, ti);
      if (tid < FCH) { lse_s[buf ^ 1][tid] = lse_r; dl_s[buf ^ 1][tid] = dl_r; }
    }
    __syncthreads();
  }
  if (a.ae16) {
    // every wave's dK and dV tiles through the (free) owned-V images: 2 x 8.5 KiB of its 12 KiB
    float* img = (float*)&Vo[w][0];
    ae_stage(img, dk, lane, a.scale);
    __syncthreads();
    const long rk = (long)b * a.k_sb + hh * a.k_sh + (long)kwave * a.k_ss;
    const long rv = (long)b * a.v_sb + hh * a.v_sh + (long)kwave * a.v_ss;
    ae_store(img, a.no_f32_grad ? nullptr : a.dk + rk, a.dkp ? a.dkp + rk : nullptr, a.k_ss, a.dkv_ps, a.Sk - kwave,
             lane);
    __syncthreads();
    ae_stage(img, dv, lane, 1.0f);
    __syncthreads();
    ae_store(img, a.no_f32_grad ? nullptr : a.dv + rv, a.dvp ? a.dvp + rv : nullptr, a.v_ss, a.dkv_ps, a.Sk - kwave,
             lane);
  } else if (kj < a.Sk) {
    float* dK = a.dk + b * a.k_sb + hh * a.k_sh + (long)kj * a.k_ss;
    float* dV = a.dv + b * a.v_sb + hh * a.v_sh + (long)kj * a.v_ss;
    if (!a.no_f32_grad) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        fa_store_rowT(dK + dt * 32, dk[dt], lane, a.scale);
        fa_store_rowT(dV + dt * 32, dv[dt], lane, 1.0f);
      }
    }
    if (a.dkp) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        fa_store_rowT_planes(a.dkp + (dK - a.dk) + dt * 32, a.dkv_ps, dk[dt], lane, a.scale);
        fa_store_rowT_planes(a.dvp + (dV - a.dv) + dt * 32, a.dkv_ps, dv[dt], lane, 1.0f);
      }
    }
  }
}

// SINGLE-PASS backward (Sk <= 256: the default whenever a head's keys fit one workgroup).  The
// dQ + dK/dV pair above forms S and dP twice (once per kernel: 7 products per query-key block);
// here one 8-wave workgroup owns every key of its (batch, head), streams 32-query chunks of Q / dO
// once, forms P and dS once and finishes the chunk's dQ itself (5 products):
//  * products phase (wave w, keys 32 w .. + 31 on the lane, as attn_sp_dkdv8_kernel with the roles
//    of K and V swapped): S = Q K^T with K's B fragments read from the wave's K plane image, dP =
//    dO V^T with the owned V rows split in registers, P, dS; dV^T += dO^T P, dK^T += Q^T dS.  Each
//    wave also writes its dS tile (fp32) into a [32 queries][256 keys] LDS image — the transpose the
//    dQ product needs (its reduction index, the key, is the lane index of dS);
//  * dQ phase: dQ^T = K^T dS^T for the chunk as eight 16 x 16 tiles on v_mfma_f32_16x16x32_bf16,
//    one per wave (16 head dims x 16 queries, all 256 keys: K^T fragments by ds_read_b64_tr_b16 from
//    the eight K images, dS^T fragments read as fp32 rows and split), fixed order, no atomics; the
//    tile is stored directly (one 16-B fp32 store / three 8-B plane stores per lane).
//  * delta = rowsum(dO o O) per chunk by the threads that stage dO (no dQ kernel to hand it over).
// Per chunk: products -> barrier (dS complete, staged chunk consumed) -> dQ + store of the next
// staged chunk -> barrier.  LDS: 12 + 12 KiB staging (single buffer: the second barrier already
// separates the consumers from the next store) + 8 x 12 KiB K images + 32.5 KiB dS = 153 KiB.
#define AS_BWD8_PITCH 260  // dS image row pitch (floats): = 4 mod 64 -> conflict-free 16-row b128 reads
#define MF16X32(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)
template <int MODE, bool KPAD>
__global__ __launch_bounds__(512, 1) void attn_sp_bwd8_kernel(AttnF32Args a) {
  __shared__ __attribute__((aligned(16))) unsigned short Qs[AS_OP];
  __shared__ __attribute__((aligned(16))) unsigned short Ds[AS_OP];
  __shared__ __attribute__((aligned(16))) unsigned short Ko[8][AS_OP];
  __shared__ __attribute__((aligned(16))) float dSs[FCH * AS_BWD8_PITCH];
  __shared__ float lse_s[FCH], dl_s[FCH];
  AST_DECL;
  AST_T(tk0);
  const int hh = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
  const int kwave = w * 32;
  const int kj = kwave + (lane & 31);
  const bool stq = tid < 256;  // this thread stages Q (waves 0-3) or dO and delta (waves 4-7)
  const int ti = tid & 255;
  AS_SRC(Q, a.q, a.q_sb, a.q_sh, a.q_ss);
  AS_SRC(K, a.k, a.k_sb, a.k_sh, a.k_ss);
  AS_SRC(V, a.v, a.v_sb, a.v_sh, a.v_ss);
  AS_SRC(dO, a.dout, a.o_sb, a.o_sh, a.o_ss);
  AS_SRC(Og, a.o, a.o_sb, a.o_sh, a.o_ss);
  const AsSrc& SQ = stq ? Q : dO;
  const long rbase = ((long)b * a.H + hh) * a.Sq;
  const int nchunks = (a.Sq + FCH - 1) / FCH;
  const int nimg = (a.Sk + 31) >> 5;  // K images holding at least one key
  AStage ps, po;
  float lse_r = INFINITY;
  auto stage_load = [&](int r0) {
    SQ.load(r0, a.Sq, ps, ti);
    lse_r = (tid < FCH && r0 + tid < a.Sq) ? a.lse[rbase + r0 + tid] : INFINITY;
  };
  auto stage_store = [&]() {
    as_store(stq ? Qs : Ds, ps, ti);
    if (!stq) {  // delta of row ti >> 3: its 64 values are 8 consecutive lanes' 8 each
      float d = ps.v[0].x * po.v[0].x;
      d = fmaf(ps.v[0].y, po.v[0].y, d); d = fmaf(ps.v[0].z, po.v[0].z, d); d = fmaf(ps.v[0].w, po.v[0].w, d);
      d = fmaf(ps.v[1].x, po.v[1].x, d); d = fmaf(ps.v[1].y, po.v[1].y, d);
      d = fmaf(ps.v[1].z, po.v[1].z, d); d = fmaf(ps.v[1].w, po.v[1].w, d);
      d += smi_dpp<SMI_DPP_QP1032>(d);
      d += smi_dpp<SMI_DPP_QP2301>(d);
      d += smi_dpp<SMI_DPP_HMIRROR>(d);  // lanes 0-3 + 4-7 of each 8-lane group: the row's sum
      if ((ti & 7) == 0) dl_s[ti >> 3] = d;
    }
    if (tid < FCH) lse_s[tid] = lse_r;
  };
  if (nchunks) { stage_load(0); if (!stq) Og.load(0, a.Sq, po, ti); }
  // every wave's 32 K rows -> its plane image (four 32-row passes of 512 threads)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = tid + 512 * i, blk = idx >> 8;
    AStage pk;
    K.load(32 * blk, a.Sk, pk, idx & 255);
    as_store(Ko[blk], pk, idx & 255);
  }
  F32Pre<1, 32> vs;
  V.own(kj, a.Sk, lane, vs);
  const bool kok = kj < a.Sk && !(KPAD && a.kpad[(long)b * a.Sk + kj]);
  const float kbias = kok ? 0.f : -INFINITY;
  f32x16_t dk[2], dv[2];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) { dk[dt][r] = 0.f; dv[dt][r] = 0.f; }
  if (nchunks) stage_store();
  __syncthreads();
  AST_T(tk1);
  AST_ADD(0, tk0, tk1);  // prologue
  const unsigned short* kimg = Ko[w];
  // dQ tile of this wave: head dims 16 dtq .. + 15 x queries 16 qtq .. + 15 of each chunk
  const int dtq = w & 3, qtq = w >> 2, l16 = lane & 15, g4 = lane >> 4;
  for (int c = 0; c < nchunks; ++c) {
    const int q0 = c * FCH;
    const bool more = c + 1 < nchunks;
    AST_T(tc0);
    if (more) stage_load(q0 + FCH);
    // a wave whose keys all follow the chunk's queries (causal) or lie past Sk has P = dS = 0
    if (!(MODE == 2 && q0 + 31 < kwave) && kwave < a.Sk) {
      f32x16_t s, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s[r] = 0.f; dp[r] = 0.f; }
#pragma unroll
      for (int j = 0; j < 4; ++j)  // S = Q K^T, K's fragments from the wave's image
        s = as_mma(as_rowfrag(Qs, lane, j), as_rowfrag(kimg, lane, j), s);
      dp = as_rows_dot(Ds, lane, vs, dp);  // dP = dO V^T
      float pvv[16], dsv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ql = fa_kl(r, h);
        const int qq = q0 + ql;
        float x = fmaf(s[r], a.scale_log2, kbias);
        if (MODE == 1) x += (kj < qq) ? LOG2E_F : 0.f;
        if (MODE == 2) x = (kj > qq) ? -INFINITY : x;
        const float pr = __builtin_amdgcn_exp2f(x - lse_s[ql]);  // rows past Sq: lse = +inf -> 0
        pvv[r] = pr;
        dsv[r] = pr * (dp[r] - dl_s[ql]);
        dSs[ql * AS_BWD8_PITCH + kj] = dsv[r];
      }
      AST_T(tc1);
      AST_ADD(1, tc0, tc1);  // S, dP, P, dS (+ dS image stores)
      as_cols_acc(Ds, lane, pvv, dv);  // dV^T += dO^T P
      as_cols_acc(Qs, lane, dsv, dk);  // dK^T += Q^T dS
      AST_T(tc2);
      AST_ADD(2, tc1, tc2);  // dV, dK products issue
    }
    AST_T(tc2b);
    // O rows of the next chunk (delta) only now: held across the dQ phase, not the products
    if (more && !stq) Og.load(q0 + FCH, a.Sq, po, ti);
    smi_lds_barrier();  // dS complete; every read of the staged chunk done
    AST_T(tc3);
    AST_ADD(3, tc2b, tc3);  // first barrier (waits for the MFMAs too)
    {
      // dQ^T (16 x 16) = sum over the key images of K^T dS^T; causal: images past the chunk are 0
      const int nk = MODE == 2 ? min(nimg, c + 1) : nimg;
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
      const float* srow = dSs + (16 * qtq + l16) * AS_BWD8_PITCH + 8 * g4;
      const int o0 = as_off(8 * g4 + (l16 >> 2), 16 * dtq + 4 * (l16 & 3));
      const int o1 = as_off(8 * g4 + 4 + (l16 >> 2), 16 * dtq + 4 * (l16 & 3));
      // fully unrolled, image kw + 1's reads issued before image kw's split and MFMAs (reads past
      // nk are in bounds and unused: images past Sk are zero rows, their dS columns never read)
      Split3 kt[2];
      float4 u[2][2];
      auto ldq = [&](int kw, int sl) {
        bf16x8_t* outs[3] = {&kt[sl].h, &kt[sl].m, &kt[sl].l};
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
          const unsigned short* bp = Ko[kw] + pl * AS_PL;
          const as_s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) as_s16x4_t*)(bp + o0));
          const as_s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) as_s16x4_t*)(bp + o1));
          *outs[pl] = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
        }
        u[sl][0] = *(const float4*)(srow + 32 * kw);
        u[sl][1] = *(const float4*)(srow + 32 * kw + 4);
      };
      ldq(0, 0);
#pragma unroll
      for (int kw = 0; kw < 8; ++kw) {
        if (kw + 1 < 8) ldq(kw + 1, (kw + 1) & 1);
        if (kw < nk) {
          const int sl = kw & 1;
          const float f[8] = {u[sl][0].x, u[sl][0].y, u[sl][0].z, u[sl][0].w,
                              u[sl][1].x, u[sl][1].y, u[sl][1].z, u[sl][1].w};
          const Split3 sd = split3_8(f);
          acc = MF16X32(kt[sl].l, sd.h, acc);
          acc = MF16X32(kt[sl].m, sd.m, acc);
          acc = MF16X32(kt[sl].h, sd.l, acc);
          acc = MF16X32(kt[sl].m, sd.h, acc);
          acc = MF16X32(kt[sl].h, sd.m, acc);
          acc = MF16X32(kt[sl].h, sd.h, acc);
        }
      }
      // lane: query q0 + 16 qtq + l16, head dims 16 dtq + 4 g4 .. + 3
      const int qi = q0 + 16 * qtq + l16;
      if (qi < a.Sq) {
        const long off = (long)b * a.q_sb + hh * a.q_sh + (long)qi * a.q_ss + 16 * dtq + 4 * g4;
        const float v0 = acc[0] * a.scale, v1 = acc[1] * a.scale, v2 = acc[2] * a.scale, v3 = acc[3] * a.scale;
        if (!a.no_f32_grad) *(float4*)(a.dq + off) = make_float4(v0, v1, v2, v3);
        if (a.dqp) {
          uint32_t h0, m0, l0, h1, m1, l1;
          split3_pair(v0, v1, h0, m0, l0);
          split3_pair(v2, v3, h1, m1, l1);
          unsigned short* qp = a.dqp + off;
          *(uint2*)qp = make_uint2(h0, h1);
          *(uint2*)(qp + a.dq_ps) = make_uint2(m0, m1);
          *(uint2*)(qp + 2 * a.dq_ps) = make_uint2(l0, l1);
        }
      }
    }
    AST_T(tc4);
    AST_ADD(4, tc3, tc4);  // dQ phase + its stores
    if (more) stage_store();
    AST_T(tc5);
    AST_ADD(5, tc4, tc5);  // next chunk's stage store + delta
    smi_lds_barrier();  // next chunk staged; every dS read done before the next chunk's writes
    AST_T(tc6);
    AST_ADD(6, tc5, tc6);  // second barrier
  }
  // dK / dV through the (now free: the last barrier follows every dQ read) K images
  if (a.ae16) {
    float* img = (float*)&Ko[w][0];
    ae_stage(img, dk, lane, a.scale);
    __syncthreads();
    const long rk = (long)b * a.k_sb + hh * a.k_sh + (long)kwave * a.k_ss;
    const long rv = (long)b * a.v_sb + hh * a.v_sh + (long)kwave * a.v_ss;
    ae_store(img, a.no_f32_grad ? nullptr : a.dk + rk, a.dkp ? a.dkp + rk : nullptr, a.k_ss, a.dkv_ps, a.Sk - kwave,
             lane);
    __syncthreads();
    ae_stage(img, dv, lane, 1.0f);
    __syncthreads();
    ae_store(img, a.no_f32_grad ? nullptr : a.dv + rv, a.dvp ? a.dvp + rv : nullptr, a.v_ss, a.dkv_ps, a.Sk - kwave,
             lane);
  } else if (kj < a.Sk) {
    float* dK = a.dk + b * a.k_sb + hh * a.k_sh + (long)kj * a.k_ss;
    float* dV = a.dv + b * a.v_sb + hh * a.v_sh + (long)kj * a.v_ss;
    if (!a.no_f32_grad) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        fa_store_rowT(dK + dt * 32, dk[dt], lane, a.scale);
        fa_store_rowT(dV + dt * 32, dv[dt], lane, 1.0f);
      }
    }
    if (a.dkp) {
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        fa_store_rowT_planes(a.dkp + (dK - a.dk) + dt * 32, a.dkv_ps, dk[dt], lane, a.scale);
        fa_store_rowT_planes(a.dvp + (dV - a.dv) + dt * 32, a.dkv_ps, dv[dt], lane, 1.0f);
      }
    }
  }
  AST_T(tk3);
  AST_ADD(7, tk0, tk3);  // wave lifetime
  AST_END();
}

// Launch over the compile-time (mask mode, key padding) instances of a kernel, NT threads
#define SMI_ATTN_SP_MODES(KERNEL, GRID, NT, ARGS)                                                        \
  do {                                                                                                   \
    const bool kp_ = (ARGS).kpad != nullptr;                                                             \
    switch ((ARGS).mode) {                                                                               \
      case 0: if (kp_) hipLaunchKernelGGL((KERNEL<0, true>), GRID, dim3(NT), 0, st, ARGS);               \
              else hipLaunchKernelGGL((KERNEL<0, false>), GRID, dim3(NT), 0, st, ARGS); break;           \
      case 1: if (kp_) hipLaunchKernelGGL((KERNEL<1, true>), GRID, dim3(NT), 0, st, ARGS);               \
              else hipLaunchKernelGGL((KERNEL<1, false>), GRID, dim3(NT), 0, st, ARGS); break;           \
      case 2: if (kp_) hipLaunchKernelGGL((KERNEL<2, true>), GRID, dim3(NT), 0, st, ARGS);               \
              else hipLaunchKernelGGL((KERNEL<2, false>), GRID, dim3(NT), 0, st, ARGS); break;           \
      default: return -1;                                                                                \
    }                                                                                                    \
  } while (0)

// product algorithm shared with the fp32 GEMM (csrc/kernels/gemm_f32.hip:smi_gemm_f32_algo):
// 0 = f32 MFMA chains (the XS = 0 kernels above), otherwise the exact-product bf16 split: the
// staged-plane kernels
extern "C" int smi_gemm_f32_algo(int);
#define SMI_ATTN_F32_MODES(KERNEL, XSV, GRID, ARGS)                                                        \
  switch ((ARGS).mode) {                                                                                   \
    case 0: if (kp_) hipLaunchKernelGGL((KERNEL<0, true, XSV>), GRID, dim3(256), 0, st, ARGS);             \
            else hipLaunchKernelGGL((KERNEL<0, false, XSV>), GRID, dim3(256), 0, st, ARGS); break;         \
    case 1: if (kp_) hipLaunchKernelGGL((KERNEL<1, true, XSV>), GRID, dim3(256), 0, st, ARGS);             \
            else hipLaunchKernelGGL((KERNEL<1, false, XSV>), GRID, dim3(256), 0, st, ARGS); break;         \
    case 2: if (kp_) hipLaunchKernelGGL((KERNEL<2, true, XSV>), GRID, dim3(256), 0, st, ARGS);             \
            else hipLaunchKernelGGL((KERNEL<2, false, XSV>), GRID, dim3(256), 0, st, ARGS); break;         \
    default: return -1;                                                                                    \
  }
#define SMI_ATTN_F32_DISPATCH(KERNEL, GRID, ARGS)                                                           \
  do {                                                                                                     \
    const bool kp_ = (ARGS).kpad != nullptr;                                                               \
    if (smi_gemm_f32_algo(-1) == 0) { SMI_ATTN_F32_MODES(KERNEL, 0, GRID, ARGS) }                         \
    else { SMI_ATTN_F32_MODES(KERNEL, 1, GRID, ARGS) }                                                     \
  } while (0)

static int fa_ok(const AttnF32Args& a) {
  // float4 access to every row: 16-B aligned bases and strides that are multiples of 4 floats
  const long st[] = {a.q_ss, a.k_ss, a.v_ss, a.o_ss, a.q_sh, a.k_sh, a.v_sh, a.o_sh, a.q_sb, a.k_sb, a.v_sb, a.o_sb};
  for (long s : st)
    if (s % 4) return 0;
  if ((((uintptr_t)a.q) | ((uintptr_t)a.k) | ((uintptr_t)a.v) | ((uintptr_t)a.o)) & 15) return 0;
  // plane outputs: 8-B stores of 4 consecutive head-dim values
  if ((((uintptr_t)a.op) | ((uintptr_t)a.dqp) | ((uintptr_t)a.dkp) | ((uintptr_t)a.dvp)) & 7) return 0;
  if ((a.dkp != nullptr) != (a.dvp != nullptr)) return 0;
  return a.B > 0 && a.H > 0 && a.Sq > 0 && a.Sk > 0;
}

// whole-row 16-B stores of an output (fp32: float4 rows, already required by fa_ok) and of its
// planes (8 bf16 per store): 16-B plane base and strides that are multiples of 8 elements
static bool fa_ae16(const unsigned short* p, long sb, long sh, long ss) {
  return !p || ((((uintptr_t)p) & 15) == 0 && sb % 8 == 0 && sh % 8 == 0 && ss % 8 == 0);
}
// The row-coalesced epilogue (ae_stage / ae_store) of all three staged-plane kernels; the one A/B
// switch of this file: SMI_ATTN_AE=0 selects the per-lane transposed stores (also taken whenever an
// output's alignment rules the 16-B row stores out).  In isolation (tools/ab_attn.py:
// self-attention, compact layouts) the backward's measured +3..5 us per call, but inside the step
// the cross-attention dK / dV go to the 6-layer concatenated kv gradient (row stride 6144), where
// the per-lane stores touched 32-64 rows per instruction: dK/dV 98 -> 57 us, the fp32 step
// 15.59 -> 15.11 ms (round 4, same box).
static int g_attn_ae = -1;
extern "C" int smi_attn_ae(int set) {
  if (set == 0 || set == 1) g_attn_ae = set;
  if (g_attn_ae < 0) {
    const char* e = getenv("SMI_ATTN_AE");
    g_attn_ae = (e && e[0] == '0') ? 0 : 1;
  }
  return g_attn_ae;
}

// Single-pass backward at Sk <= 256 (attn_sp_bwd8_kernel here, attn_bwd8_kernel in attention.hip):
// 1 = on (default), 0 = the dQ + dK/dV kernel pair (SMI_ATTN_BWD1=0; A/B and tests).
static int g_attn_bwd1 = -1;
extern "C" int smi_attn_bwd1(int set) {
  if (set == 0 || set == 1) g_attn_bwd1 = set;
  if (g_attn_bwd1 < 0) {
    const char* e = getenv("SMI_ATTN_BWD1");
    g_attn_bwd1 = (e && e[0] == '0') ? 0 : 1;
  }
  return g_attn_bwd1;
}

extern "C" int smi_attn_f32_fwd(const AttnF32Args* args, hipStream_t st) {
  AttnF32Args a = *args;
  if (!fa_ok(a)) return -1;
  a.ae16 = smi_attn_ae(-1) && fa_ae16(a.op, a.o_sb, a.o_sh, a.o_ss);
  dim3 grid((a.Sq + 127) / 128, a.H, a.B);
  if (smi_gemm_f32_algo(-1) != 0) SMI_ATTN_SP_MODES(attn_sp_fwd4, grid, 256, a);
  else SMI_ATTN_F32_DISPATCH(attn_f32_fwd_kernel, grid, a);
  SMI_CHECK_LAUNCH();
}

extern "C" int smi_attn_f32_bwd(const AttnF32Args* args, hipStream_t st) {
  AttnF32Args a = *args;
  if (!fa_ok(a) || !a.dout || !a.delta || (((uintptr_t)a.dout | (uintptr_t)a.dq | (uintptr_t)a.dk | (uintptr_t)a.dv) & 15))
    return -1;
  a.ae16 = smi_attn_ae(-1) && fa_ae16(a.dqp, a.q_sb, a.q_sh, a.q_ss) && fa_ae16(a.dkp, a.k_sb, a.k_sh, a.k_ss) &&
           fa_ae16(a.dvp, a.v_sb, a.v_sh, a.v_ss);
  if (a.no_f32_grad && (!a.dqp || !a.dkp || !a.dvp)) return -1;  // planes-only needs every plane output
  if (smi_gemm_f32_algo(-1) != 0) {
    if (a.Sk <= AS_DKDV8_KEYS && smi_attn_bwd1(-1)) {
      SMI_ATTN_SP_MODES(attn_sp_bwd8_kernel, dim3(1, a.H, a.B), 512, a);
    } else {
      SMI_ATTN_SP_MODES(attn_sp_dq_kernel, dim3((a.Sq + 127) / 128, a.H, a.B), 256, a);
      SMI_ATTN_SP_MODES(attn_sp_dkdv8_kernel, dim3((a.Sk + AS_DKDV8_KEYS - 1) / AS_DKDV8_KEYS, a.H, a.B), 512, a);
    }
  } else {
    SMI_ATTN_F32_DISPATCH(attn_f32_dq_kernel, dim3((a.Sq + 127) / 128, a.H, a.B), a);
    SMI_ATTN_F32_DISPATCH(attn_f32_dkdv_kernel, dim3((a.Sk + 127) / 128, a.H, a.B), a);
  }
  SMI_CHECK_LAUNCH();
}
