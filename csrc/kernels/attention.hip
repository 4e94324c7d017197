// Fused scaled-dot-product attention, forward and backward, head_dim = 64, bf16 in/out,
// fp32 softmax/accumulation, MFMA v_mfma_f32_16x16x32_bf16.
//
// Reference semantics: transformer.py:12-25 (scaled_dot_product) as called by
// MultiHeadAttention (:74-83) and MultiHeadCrossAttention (:177-191).  The reference adds a
// *boolean* mask after a (0,1,3,2) permute; SURVEY.md Q6 shows this is a +1.0 additive bias on
// strictly-past keys for the look-ahead mask and a softmax no-op for the padding mask.
// mode: 0 = no mask, 1 = "reference" (+1 on key < query), 2 = causal (-inf on key > query);
// an optional uint8 key-padding vector adds -inf on padded keys.
//
// Layout: element (b, s, h, d) of Q/K/V/O lives at base + b*sb + s*ss + h*sh + d, so the
// kernels read q/k/v straight out of the fused qkv / kv projection outputs (per-head
// interleaved [q_h|k_h|v_h] layout of transformer.py:76-79) and write O already head-merged.
//
// Structure (MI355X): one workgroup = 4 waves = 128 rows of the "owned" axis (queries for the
// forward and dQ, keys for dK/dV), 32 per wave as two 16-row MFMA sub-tiles that share every
// LDS fragment.  The streamed operand goes through double-buffered 64-row LDS chunks (below).
// Scores are computed with the owned axis on the lane (S^T = K Q^T in the forward), so the
// online-softmax statistics and the output rescale are lane-local, and the 16x16 accumulators
// of two adjacent 16-row tiles form the bf16 operand of the second product directly (k order
// permuted identically on both operands; cdna_hip_programming.md §3).  Outputs are produced
// transposed (O^T = V^T P^T etc.), so each lane stores 4 consecutive head-dim values.
#include "smi_common.h"


#include "smi_attention.h"
#include "smi_attn_mask.h"

// ---------------------------------------------------------------------------------------------
// LDS images: 64 rows x 64 bf16 (128-B rows), 16-B chunk c of row r stored at chunk c ^ (r & 7).
// The same image serves both operand reads conflict-free:
//  * row fragments (ds_read_b128: 8 consecutive d of one row) — A operand with k = d;
//  * transposed fragments (ds_read_b64_tr_b16: one d column of 4+4 rows) — A/B operand with
//    k = row, in the permuted key order of two adjacent 16-row accumulator tiles, so a P / dS
//    tile packed straight from the accumulators multiplies it without any register shuffle.
// Chunks are double-buffered: the global loads of chunk c+1 are issued (16 B per lane, into
// registers) before chunk c's MFMAs and stored to the other buffer after them.
#define IMG_ELEMS (64 * 64)

__device__ __forceinline__ int swz(int row, int chunk) { return row * 64 + ((chunk ^ (row & 7)) << 3); }

struct Piece2 { u16x8_t v[2]; };

__device__ __forceinline__ void load_chunk(const unsigned short* __restrict__ base, long ss, int r0, int rmax, Piece2& p) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = threadIdx.x + 256 * u;
    const int row = i >> 3, c = i & 7, r = r0 + row;
    if (r < rmax) p.v[u] = *(const u16x8_t*)(base + (long)r * ss + c * 8);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) p.v[u][j] = 0;
    }
  }
}
__device__ __forceinline__ void store_chunk(unsigned short* img, const Piece2& p) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = threadIdx.x + 256 * u;
    *(u16x8_t*)(img + swz(i >> 3, i & 7)) = p.v[u];
  }
}

// row fragment: 8 bf16 of row `row`, 16-B chunk `chunk`
__device__ __forceinline__ bf16x8_t frag_row(const unsigned short* img, int row, int chunk) {
  return *(const bf16x8_t*)(img + swz(row, chunk));
}
// transposed fragment: element jj = img[krow0 + (jj < 4 ? 4g + jj : 16 + 4g + jj - 4)][col0 + (lane & 15)]
typedef __attribute__((ext_vector_type(4))) short s16x4_t;
__device__ __forceinline__ bf16x8_t frag_tr(const unsigned short* img, int krow0, int col0, int lane) {
  const int q = (lane & 15) >> 2, p = lane & 3, g = lane >> 4;
  const int col = col0 + 4 * p;
  s16x4_t v[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = krow0 + 16 * h + 4 * g + q;
    const unsigned short* addr = img + row * 64 + (((col >> 3) ^ (row & 7)) << 3) + (col & 7);
    v[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)addr);
  }
  // one vector concatenation: the two 64-bit reads can land in adjacent registers (element-wise
  // assembly costs v_mov per element, as measured in the GEMM k-loop)
  return __builtin_shufflevector(v[0], v[1], 0, 1, 2, 3, 4, 5, 6, 7);
}
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
__device__ __forceinline__ bf16x8_t pack_acc(const f32x4_t& a, const f32x4_t& b) {
  const u32x4_t w = {pack2bf(a[0], a[1]), pack2bf(a[2], a[3]), pack2bf(b[0], b[1]), pack2bf(b[2], b[3])};
  return __builtin_bit_cast(bf16x8_t, w);
}
__device__ __forceinline__ bf16x8_t load8(const unsigned short* p, bool ok) {
  bf16x8_t r;
  if (ok) r = *(const bf16x8_t*)p;
  else {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = 0;
  }
  return r;
}
__device__ __forceinline__ void store4(unsigned short* p, const f32x4_t& v, float sc) {
  uint2 pk;
  pk.x = pack2bf(v[0] * sc, v[1] * sc);
  pk.y = pack2bf(v[2] * sc, v[3] * sc);
  *(uint2*)p = pk;
}


// Reductions across the four 16-lane rows of a wave (lanes n, n+16, n+32, n+48) with the gfx950
// row-swap instructions (VALU, a few cycles) instead of __shfl_xor (ds_bpermute through the LDS
// crossbar, ~100+ cycles of latency on the softmax's critical path).  permlane16_swap(v, v)
// returns rows (R0,R0,R2,R2) and (R1,R1,R3,R3): their combination is the xor-16 reduction in
// every lane; permlane32_swap(v, v) likewise gives halves (lo,lo) and (hi,hi) for xor-32.
__device__ __forceinline__ float rows4_max(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float rows4_sum(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

#define MFMA16(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

// ---------------------------------------------------------------------------------------------
// Forward: workgroup = 4 waves x 32 queries (two 16-query sub-tiles per wave); K/V streamed in
// 64-key chunks.  S^T = K Q^T (lane owns one query column), online softmax in registers,
// O^T += V^T P^T (so O's rescale by the running max is lane-local too).
template <int MODE, bool KPAD>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(AttnFwdArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned short Ks[2][IMG_ELEMS];
  __shared__ __attribute__((aligned(16))) unsigned short Vs[2][IMG_ELEMS];
  const int h = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  const int qwave = blockIdx.x * 128 + w * 32;
  const unsigned short* Q = a.q + b * a.q_sb + h * a.q_sh;
  const unsigned short* K = a.k + b * a.k_sb + h * a.k_sh;
  const unsigned short* V = a.v + b * a.v_sb + h * a.v_sh;
  const unsigned char* kp = a.kpad ? a.kpad + (long)b * a.Sk : nullptr;
  int kend = a.Sk;
  if (MODE == 2) kend = min(a.Sk, blockIdx.x * 128 + 128);
  const int nchunks = (kend + 63) / 64;
  Piece2 pk, pv;
  load_chunk(K, a.k_ss, 0, a.Sk, pk);
  load_chunk(V, a.v_ss, 0, a.Sk, pv);
  bf16x8_t qf[2][2];
#pragma unroll
  for (int qs = 0; qs < 2; ++qs) {
    const int qi = qwave + qs * 16 + n;
    qf[qs][0] = load8(Q + (long)qi * a.q_ss + 8 * g, qi < a.Sq);
    qf[qs][1] = load8(Q + (long)qi * a.q_ss + 32 + 8 * g, qi < a.Sq);
  }
  store_chunk(Ks[0], pk);
  store_chunk(Vs[0], pv);
  __syncthreads();
  float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};
  f32x4_t o[2][4];
#pragma unroll
  for (int qs = 0; qs < 2; ++qs)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[qs][dt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1, k0 = c * 64;
    const bool more = c + 1 < nchunks;
    if (more) { load_chunk(K, a.k_ss, k0 + 64, a.Sk, pk); load_chunk(V, a.v_ss, k0 + 64, a.Sk, pv); }
    const unsigned short* ks_ = Ks[buf];
    const unsigned short* vs_ = Vs[buf];
    const bool full = k0 + 64 <= a.Sk;
    const unsigned long long kmask = KPAD ? chunk_pad_mask(kp, k0, a.Sk) : 0ull;
    f32x4_t s[2][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const bf16x8_t k0f = frag_row(ks_, t * 16 + n, g), k1f = frag_row(ks_, t * 16 + n, 4 + g);
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) {
        s[qs][t] = MFMA16(k0f, qf[qs][0], ((f32x4_t){0.f, 0.f, 0.f, 0.f}));
        s[qs][t] = MFMA16(k1f, qf[qs][1], s[qs][t]);
      }
    }
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      const int qi = qwave + qs * 16 + n;
      const int qlo = qwave + qs * 16;
      float ub;
      const bool uni = uniform_bias<MODE, KPAD>(k0, qlo, qlo + 15, full, ub);
      float cmax = -INFINITY;
      if (uni) {  // x = s*scale + ub for every entry: max on the raw scores, one FMA per exp below
        float r = -INFINITY;
#pragma unroll
        for (int t = 0; t < 4; ++t) r = fmaxf(r, fmaxf(fmaxf(s[qs][t][0], s[qs][t][1]), fmaxf(s[qs][t][2], s[qs][t][3])));
        cmax = r * a.scale_log2 + ub;
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int kl = t * 16 + 4 * g + j;
            s[qs][t][j] = score_adj<MODE, KPAD>(s[qs][t][j], qi, k0 + kl, kl, full, a.Sk, kmask, a.scale_log2);
            cmax = fmaxf(cmax, s[qs][t][j]);
          }
      }
      cmax = rows4_max(cmax);
      const float mnew = fmaxf(m[qs], cmax);
      const float mref = (mnew == -INFINITY) ? 0.f : mnew;
      const float alpha = __builtin_amdgcn_exp2f(m[qs] - mref);
      float psum = 0.f;
      if (uni) {
        const float off = ub - mref;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            s[qs][t][j] = __builtin_amdgcn_exp2f(fmaf(s[qs][t][j], a.scale_log2, off));
            psum += s[qs][t][j];
          }
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) { s[qs][t][j] = __builtin_amdgcn_exp2f(s[qs][t][j] - mref); psum += s[qs][t][j]; }
      }
      psum = rows4_sum(psum);
      l[qs] = l[qs] * alpha + psum;
      m[qs] = mnew;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[qs][dt] *= alpha;
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8_t pa0 = pack_acc(s[0][2 * s2], s[0][2 * s2 + 1]);
      const bf16x8_t pa1 = pack_acc(s[1][2 * s2], s[1][2 * s2 + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8_t vf = frag_tr(vs_, 32 * s2, dt * 16, lane);
        o[0][dt] = MFMA16(vf, pa0, o[0][dt]);
        o[1][dt] = MFMA16(vf, pa1, o[1][dt]);
      }
    }
    if (more) { store_chunk(Ks[buf ^ 1], pk); store_chunk(Vs[buf ^ 1], pv); }
    __syncthreads();
  }
  unsigned short* O = a.o + b * a.o_sb + h * a.o_sh;
  // (direct 8-B stores: a row-coalesced pass through the idle K staging measured 15.2 -> 15.7 us per
  // call — two workgroups per CU already overlap one's stores with the other's loop)
#pragma unroll
  for (int qs = 0; qs < 2; ++qs) {
    const int qi = qwave + qs * 16 + n;
    if (qi < a.Sq) {
      const float inv = l[qs] > 0.f ? 1.0f / l[qs] : 0.f;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) store4(O + (long)qi * a.o_ss + dt * 16 + 4 * g, o[qs][dt], inv);
      if (g == 0) {
        const float mref = (m[qs] == -INFINITY) ? 0.f : m[qs];
        a.lse[((long)b * a.H + h) * a.Sq + qi] = l[qs] > 0.f ? mref + log2f(l[qs]) : INFINITY;
      }
    }
  }
}

// dQ: workgroup = 4 waves x 32 queries; K/V streamed.  S^T = K Q^T, dP^T = V dO^T,
// dS^T = P^T o (dP^T - delta), dQ^T += K^T dS^T.
template <int MODE, bool KPAD>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(AttnBwdArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned short Ks[2][IMG_ELEMS];
  __shared__ __attribute__((aligned(16))) unsigned short Vs[2][IMG_ELEMS];
  const int h = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  const int qwave = blockIdx.x * 128 + w * 32;
  const unsigned short* Q = a.q + b * a.q_sb + h * a.q_sh;
  const unsigned short* K = a.k + b * a.k_sb + h * a.k_sh;
  const unsigned short* V = a.v + b * a.v_sb + h * a.v_sh;
  const unsigned short* dO = a.dout + b * a.o_sb + h * a.o_sh;
  const unsigned char* kp = a.kpad ? a.kpad + (long)b * a.Sk : nullptr;
  int kend = a.Sk;
  if (MODE == 2) kend = min(a.Sk, blockIdx.x * 128 + 128);
  const int nchunks = (kend + 63) / 64;
  Piece2 pk, pv;
  load_chunk(K, a.k_ss, 0, a.Sk, pk);
  load_chunk(V, a.v_ss, 0, a.Sk, pv);
  bf16x8_t qf[2][2], df[2][2], of[2][2];
  float lse[2], dl[2];
  const unsigned short* Og = a.o + b * a.o_sb + h * a.o_sh;
#pragma unroll
  for (int qs = 0; qs < 2; ++qs) {
    const int qi = qwave + qs * 16 + n;
    const bool ok = qi < a.Sq;
    qf[qs][0] = load8(Q + (long)qi * a.q_ss + 8 * g, ok);
    qf[qs][1] = load8(Q + (long)qi * a.q_ss + 32 + 8 * g, ok);
    df[qs][0] = load8(dO + (long)qi * a.o_ss + 8 * g, ok);
    df[qs][1] = load8(dO + (long)qi * a.o_ss + 32 + 8 * g, ok);
    of[qs][0] = load8(Og + (long)qi * a.o_ss + 8 * g, ok);
    of[qs][1] = load8(Og + (long)qi * a.o_ss + 32 + 8 * g, ok);
    lse[qs] = ok ? a.lse[((long)b * a.H + h) * a.Sq + qi] : INFINITY;
  }
  // delta = rowsum(dO * O) for this wave's queries (the four lanes n, n+16, n+32, n+48 hold a
  // row's 64 values between them); written once for the dK/dV kernel, which runs next
#pragma unroll
  for (int qs = 0; qs < 2; ++qs) {
    float sacc = 0.f;
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        sacc += bf2f((unsigned short)df[qs][u][j]) * bf2f((unsigned short)of[qs][u][j]);
    sacc = rows4_sum(sacc);
    dl[qs] = sacc;
    const int qi = qwave + qs * 16 + n;
    if (g == 0 && qi < a.Sq) a.delta_out[((long)b * a.H + h) * a.Sq + qi] = sacc;
  }
  store_chunk(Ks[0], pk);
  store_chunk(Vs[0], pv);
  __syncthreads();
  f32x4_t acc[2][4];
#pragma unroll
  for (int qs = 0; qs < 2; ++qs)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) acc[qs][dt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1, k0 = c * 64;
    const bool more = c + 1 < nchunks;
    if (more) { load_chunk(K, a.k_ss, k0 + 64, a.Sk, pk); load_chunk(V, a.v_ss, k0 + 64, a.Sk, pv); }
    const unsigned short* ks_ = Ks[buf];
    const unsigned short* vs_ = Vs[buf];
    const bool full = k0 + 64 <= a.Sk;
    const unsigned long long kmask = KPAD ? chunk_pad_mask(kp, k0, a.Sk) : 0ull;
    f32x4_t s[2][4], dp[2][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const bf16x8_t k0f = frag_row(ks_, t * 16 + n, g), k1f = frag_row(ks_, t * 16 + n, 4 + g);
      const bf16x8_t v0f = frag_row(vs_, t * 16 + n, g), v1f = frag_row(vs_, t * 16 + n, 4 + g);
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) {
        s[qs][t] = MFMA16(k0f, qf[qs][0], ((f32x4_t){0.f, 0.f, 0.f, 0.f}));
        s[qs][t] = MFMA16(k1f, qf[qs][1], s[qs][t]);
        dp[qs][t] = MFMA16(v0f, df[qs][0], ((f32x4_t){0.f, 0.f, 0.f, 0.f}));
        dp[qs][t] = MFMA16(v1f, df[qs][1], dp[qs][t]);
      }
    }
#pragma unroll
    for (int qs = 0; qs < 2; ++qs) {
      const int qi = qwave + qs * 16 + n;
      const int qlo = qwave + qs * 16;
      float ub;
      if (uniform_bias<MODE, KPAD>(k0, qlo, qlo + 15, full, ub)) {
        const float off = ub - lse[qs];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float p = __builtin_amdgcn_exp2f(fmaf(s[qs][t][j], a.scale_log2, off));
            s[qs][t][j] = p * (dp[qs][t][j] - dl[qs]);
          }
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int kl = t * 16 + 4 * g + j;
            const float x = score_adj<MODE, KPAD>(s[qs][t][j], qi, k0 + kl, kl, full, a.Sk, kmask, a.scale_log2);
            const float p = __builtin_amdgcn_exp2f(x - lse[qs]);  // exp2(-inf) = 0 for masked entries
            s[qs][t][j] = p * (dp[qs][t][j] - dl[qs]);
          }
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8_t d0 = pack_acc(s[0][2 * s2], s[0][2 * s2 + 1]);
      const bf16x8_t d1 = pack_acc(s[1][2 * s2], s[1][2 * s2 + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8_t kt = frag_tr(ks_, 32 * s2, dt * 16, lane);
        acc[0][dt] = MFMA16(kt, d0, acc[0][dt]);
        acc[1][dt] = MFMA16(kt, d1, acc[1][dt]);
      }
    }
    if (more) { store_chunk(Ks[buf ^ 1], pk); store_chunk(Vs[buf ^ 1], pv); }
    __syncthreads();
  }
  unsigned short* dQ = a.dq + b * a.q_sb + h * a.q_sh;
#pragma unroll
  for (int qs = 0; qs < 2; ++qs) {
    const int qi = qwave + qs * 16 + n;
    if (qi < a.Sq) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) store4(dQ + (long)qi * a.q_ss + dt * 16 + 4 * g, acc[qs][dt], a.scale);
    }
  }
}

// dK, dV: workgroup = 4 waves x 32 keys; Q / dO streamed.  S = Q K^T and dP = dO V^T with the
// key on the lane, P = exp2(S' - lse), dS = P o (dP - delta), dV^T += dO^T P, dK^T += Q^T dS.
template <int MODE, bool KPAD>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_kernel(AttnBwdArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned short Qs[2][IMG_ELEMS];
  __shared__ __attribute__((aligned(16))) unsigned short Ds[2][IMG_ELEMS];
  __shared__ float lse_s[2][64], dl_s[2][64];
  const int h = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  const int kwave = blockIdx.x * 128 + w * 32;
  const unsigned short* Q = a.q + b * a.q_sb + h * a.q_sh;
  const unsigned short* K = a.k + b * a.k_sb + h * a.k_sh;
  const unsigned short* V = a.v + b * a.v_sb + h * a.v_sh;
  const unsigned short* dO = a.dout + b * a.o_sb + h * a.o_sh;
  const long rowbase = ((long)b * a.H + h) * a.Sq;
  int qstart = 0;
  if (MODE == 2) qstart = (blockIdx.x * 128) & ~63;
  const int nchunks = qstart < a.Sq ? (a.Sq - qstart + 63) / 64 : 0;
  Piece2 pq, pd;
  float lse_r = INFINITY, dl_r = 0.f;
  if (nchunks) {
    load_chunk(Q, a.q_ss, qstart, a.Sq, pq);
    load_chunk(dO, a.o_ss, qstart, a.Sq, pd);
    if (threadIdx.x < 64 && qstart + (int)threadIdx.x < a.Sq) {
      lse_r = a.lse[rowbase + qstart + threadIdx.x];
      dl_r = a.delta[rowbase + qstart + threadIdx.x];
    }
  }
  bf16x8_t kf[2][2], vf[2][2];
  bool kok[2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int kj = kwave + kt * 16 + n;
    const bool ok = kj < a.Sk;
    kok[kt] = ok && !(KPAD && a.kpad[(long)b * a.Sk + kj]);
    kf[kt][0] = load8(K + (long)kj * a.k_ss + 8 * g, ok);
    kf[kt][1] = load8(K + (long)kj * a.k_ss + 32 + 8 * g, ok);
    vf[kt][0] = load8(V + (long)kj * a.v_ss + 8 * g, ok);
    vf[kt][1] = load8(V + (long)kj * a.v_ss + 32 + 8 * g, ok);
  }
  f32x4_t dk[2][4], dv[2][4];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) { dk[kt][dt] = (f32x4_t){0.f, 0.f, 0.f, 0.f}; dv[kt][dt] = dk[kt][dt]; }
  if (nchunks) {
    store_chunk(Qs[0], pq);
    store_chunk(Ds[0], pd);
    if (threadIdx.x < 64) { lse_s[0][threadIdx.x] = lse_r; dl_s[0][threadIdx.x] = dl_r; }
  }
  __syncthreads();
  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1, q0 = qstart + c * 64;
    const bool more = c + 1 < nchunks;
    if (more) {
      load_chunk(Q, a.q_ss, q0 + 64, a.Sq, pq);
      load_chunk(dO, a.o_ss, q0 + 64, a.Sq, pd);
      lse_r = INFINITY; dl_r = 0.f;
      if (threadIdx.x < 64 && q0 + 64 + (int)threadIdx.x < a.Sq) {
        lse_r = a.lse[rowbase + q0 + 64 + threadIdx.x];
        dl_r = a.delta[rowbase + q0 + 64 + threadIdx.x];
      }
    }
    const unsigned short* qs_ = Qs[buf];
    const unsigned short* ds_ = Ds[buf];
    f32x4_t s[2][4], dp[2][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const bf16x8_t q0f = frag_row(qs_, t * 16 + n, g), q1f = frag_row(qs_, t * 16 + n, 4 + g);
      const bf16x8_t d0f = frag_row(ds_, t * 16 + n, g), d1f = frag_row(ds_, t * 16 + n, 4 + g);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        s[kt][t] = MFMA16(q0f, kf[kt][0], ((f32x4_t){0.f, 0.f, 0.f, 0.f}));
        s[kt][t] = MFMA16(q1f, kf[kt][1], s[kt][t]);
        dp[kt][t] = MFMA16(d0f, vf[kt][0], ((f32x4_t){0.f, 0.f, 0.f, 0.f}));
        dp[kt][t] = MFMA16(d1f, vf[kt][1], dp[kt][t]);
      }
    }
    // s[kt][t][j]: query q0 + t*16 + 4g + j, key kwave + kt*16 + n.  Rows past Sq carry
    // lse = +inf (p = 0); a masked key lane has kok = false.
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int kj = kwave + kt * 16 + n;
      const float kbias = kok[kt] ? 0.f : -INFINITY;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ql = t * 16 + 4 * g + j;
          const int qq = q0 + ql;
          float x = fmaf(s[kt][t][j], a.scale_log2, kbias);
          if (MODE == 1) x += (kj < qq) ? LOG2E_F : 0.f;
          if (MODE == 2) x = (kj > qq) ? -INFINITY : x;
          const float p = __builtin_amdgcn_exp2f(x - lse_s[buf][ql]);
          s[kt][t][j] = p;
          dp[kt][t][j] = p * (dp[kt][t][j] - dl_s[buf][ql]);
        }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8_t p0 = pack_acc(s[0][2 * s2], s[0][2 * s2 + 1]);
      const bf16x8_t p1 = pack_acc(s[1][2 * s2], s[1][2 * s2 + 1]);
      const bf16x8_t e0 = pack_acc(dp[0][2 * s2], dp[0][2 * s2 + 1]);
      const bf16x8_t e1 = pack_acc(dp[1][2 * s2], dp[1][2 * s2 + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8_t dot = frag_tr(ds_, 32 * s2, dt * 16, lane);
        const bf16x8_t qt = frag_tr(qs_, 32 * s2, dt * 16, lane);
        dv[0][dt] = MFMA16(dot, p0, dv[0][dt]);
        dv[1][dt] = MFMA16(dot, p1, dv[1][dt]);
        dk[0][dt] = MFMA16(qt, e0, dk[0][dt]);
        dk[1][dt] = MFMA16(qt, e1, dk[1][dt]);
      }
    }
    if (more) {
      store_chunk(Qs[buf ^ 1], pq);
      store_chunk(Ds[buf ^ 1], pd);
      if (threadIdx.x < 64) { lse_s[buf ^ 1][threadIdx.x] = lse_r; dl_s[buf ^ 1][threadIdx.x] = dl_r; }
    }
    __syncthreads();
  }
  unsigned short* dK = a.dk + b * a.k_sb + h * a.k_sh;
  unsigned short* dV = a.dv + b * a.v_sb + h * a.v_sh;
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int kj = kwave + kt * 16 + n;
    if (kj < a.Sk) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        store4(dK + (long)kj * a.k_ss + dt * 16 + 4 * g, dk[kt][dt], a.scale);
        store4(dV + (long)kj * a.v_ss + dt * 16 + 4 * g, dv[kt][dt], 1.0f);
      }
    }
  }
}

// Single-pass backward (Sk <= 256, the default there): one 8-wave workgroup owns every key of its
// (batch, head) — wave w keys 32 w .. + 31, K / V in registers as in the dK/dV kernel — and streams
// 64-query chunks of Q / dO once.  Per chunk: S, dP, P, dS (keys on the lane), dV^T += dO^T P and
// dK^T += Q^T dS; every wave also writes its bf16 dS tile into a [256 keys][64 queries] LDS image
// (8-B stores of the accumulator's four consecutive queries), and after a barrier the chunk's dQ^T
// = K^T dS^T is formed as sixteen 16 x 16 tiles, two per wave (one head-dim block x two query
// blocks: the K^T fragment is shared), both operands by ds_read_b64_tr_b16 in the same permuted key
// order from the K image (all 256 keys, staged once) and the dS image; fixed order, no atomics.
// delta = rowsum(dO o O) is formed per chunk by the threads that stage dO (they load O beside it).
// 5 products per query-key block instead of the pair's 7 (S and dP formed once), one launch.
// LDS: 8 + 8 KiB staging (single buffer: the second barrier of a chunk separates its readers from
// the next store) + 32 KiB K image + 32 KiB dS image.
template <int MODE, bool KPAD>
__global__ __launch_bounds__(512, 1) void attn_bwd8_kernel(AttnBwdArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned short Qs[IMG_ELEMS];
  __shared__ __attribute__((aligned(16))) unsigned short Ds[IMG_ELEMS];
  __shared__ __attribute__((aligned(16))) unsigned short Ki[4][IMG_ELEMS];   // keys 64 i .. + 63
  __shared__ __attribute__((aligned(16))) unsigned short dSi[4][IMG_ELEMS];  // [keys 64 i ..][64 queries]
  __shared__ float lse_s[64], dl_s[64];
  const int h = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n = lane & 15, g = lane >> 4;
  const int ti = tid & 255;
  const bool stq = tid < 256;  // stages Q (waves 0-3) or dO + delta (waves 4-7)
  const int kwave = w * 32;
  const unsigned short* Q = a.q + b * a.q_sb + h * a.q_sh;
  const unsigned short* K = a.k + b * a.k_sb + h * a.k_sh;
  const unsigned short* V = a.v + b * a.v_sb + h * a.v_sh;
  const unsigned short* dO = a.dout + b * a.o_sb + h * a.o_sh;
  const unsigned short* Og = a.o + b * a.o_sb + h * a.o_sh;
  const long rowbase = ((long)b * a.H + h) * a.Sq;
  const int nchunks = (a.Sq + 63) / 64;
  const int nstep = (a.Sk + 31) >> 5;  // 32-key steps of the dQ product holding at least one key
  // thread ti stages 16-B pieces i = ti, ti + 256 of a 64 x 64 chunk: row i >> 3, chunk i & 7
  Piece2 ps, po;
  float lse_r = INFINITY;
  const unsigned short* SQ = stq ? Q : dO;
  const long sss = stq ? a.q_ss : a.o_ss;
  auto ld = [&](const unsigned short* base, long ss, int r0, int rmax, Piece2& p) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = ti + 256 * u, r = r0 + (i >> 3);
      if (r < rmax) p.v[u] = *(const u16x8_t*)(base + (long)r * ss + (i & 7) * 8);
      else {
#pragma unroll
        for (int j = 0; j < 8; ++j) p.v[u][j] = 0;
      }
    }
  };
  auto stage_load = [&](int r0) {
    ld(SQ, sss, r0, a.Sq, ps);
    lse_r = (tid < 64 && r0 + tid < a.Sq) ? a.lse[rowbase + r0 + tid] : INFINITY;
  };
  auto stage_store = [&]() {
    unsigned short* img = stq ? Qs : Ds;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = ti + 256 * u;
      *(u16x8_t*)(img + swz(i >> 3, i & 7)) = ps.v[u];
      if (!stq) {  // delta of row i >> 3: 8 consecutive lanes hold its 64 values
        float d = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) d = fmaf(bf2f(ps.v[u][j]), bf2f(po.v[u][j]), d);
        d += smi_dpp<SMI_DPP_QP1032>(d);
        d += smi_dpp<SMI_DPP_QP2301>(d);
        d += smi_dpp<SMI_DPP_HMIRROR>(d);
        if ((i & 7) == 0) dl_s[i >> 3] = d;
      }
    }
    if (tid < 64) lse_s[tid] = lse_r;
  };
  if (nchunks) { stage_load(0); if (!stq) ld(Og, a.o_ss, 0, a.Sq, po); }
  // the head's K rows -> four 64-row images (pieces of 16 B, 4 per thread)
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = tid + 512 * u, r = i >> 3;
    u16x8_t v;
    if (r < a.Sk) v = *(const u16x8_t*)(K + (long)r * a.k_ss + (i & 7) * 8);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = 0;
    }
    *(u16x8_t*)(&Ki[r >> 6][0] + swz(r & 63, i & 7)) = v;
  }
  bf16x8_t kf[2][2], vf[2][2];
  bool kok[2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int kj = kwave + kt * 16 + n;
    const bool ok = kj < a.Sk;
    kok[kt] = ok && !(KPAD && a.kpad[(long)b * a.Sk + kj]);
    kf[kt][0] = load8(K + (long)kj * a.k_ss + 8 * g, ok);
    kf[kt][1] = load8(K + (long)kj * a.k_ss + 32 + 8 * g, ok);
    vf[kt][0] = load8(V + (long)kj * a.v_ss + 8 * g, ok);
    vf[kt][1] = load8(V + (long)kj * a.v_ss + 32 + 8 * g, ok);
  }
  f32x4_t dk[2][4], dv[2][4];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) { dk[kt][dt] = (f32x4_t){0.f, 0.f, 0.f, 0.f}; dv[kt][dt] = dk[kt][dt]; }
  if (nchunks) stage_store();
  __syncthreads();
  // this wave's dQ tiles: head dims 16 dtq .. + 15 x query blocks 2 qpq, 2 qpq + 1 (16 each)
  const int dtq = w & 3, qpq = w >> 2;
  unsigned short* dQ = a.dq + b * a.q_sb + h * a.q_sh;
  unsigned short* dSw = &dSi[w >> 1][0];  // this wave's 32 key rows start at row 32 (w & 1)
  for (int c = 0; c < nchunks; ++c) {
    const int q0 = c * 64;
    const bool more = c + 1 < nchunks;
    if (more) stage_load(q0 + 64);
    if (!(MODE == 2 && q0 + 63 < kwave) && kwave < a.Sk) {  // else P = dS = 0 for every key of the wave
      f32x4_t s[2][4], dp[2][4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bf16x8_t q0f = frag_row(Qs, t * 16 + n, g), q1f = frag_row(Qs, t * 16 + n, 4 + g);
        const bf16x8_t d0f = frag_row(Ds, t * 16 + n, g), d1f = frag_row(Ds, t * 16 + n, 4 + g);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          s[kt][t] = MFMA16(q0f, kf[kt][0], ((f32x4_t){0.f, 0.f, 0.f, 0.f}));
          s[kt][t] = MFMA16(q1f, kf[kt][1], s[kt][t]);
          dp[kt][t] = MFMA16(d0f, vf[kt][0], ((f32x4_t){0.f, 0.f, 0.f, 0.f}));
          dp[kt][t] = MFMA16(d1f, vf[kt][1], dp[kt][t]);
        }
      }
      // s[kt][t][j]: query q0 + t*16 + 4g + j, key kwave + kt*16 + n
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const int kj = kwave + kt * 16 + n;
        const float kbias = kok[kt] ? 0.f : -INFINITY;
        const int krow = 32 * (w & 1) + kt * 16 + n;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int ql = t * 16 + 4 * g + j;
            const int qq = q0 + ql;
            float x = fmaf(s[kt][t][j], a.scale_log2, kbias);
            if (MODE == 1) x += (kj < qq) ? LOG2E_F : 0.f;
            if (MODE == 2) x = (kj > qq) ? -INFINITY : x;
            const float p = __builtin_amdgcn_exp2f(x - lse_s[ql]);
            s[kt][t][j] = p;
            dp[kt][t][j] = p * (dp[kt][t][j] - dl_s[ql]);
          }
          // dS row krow, queries t*16 + 4g .. + 3 (the same bf16 values the dK product takes)
          const int col = t * 16 + 4 * g;
          *(uint2*)(dSw + swz(krow, col >> 3) + (col & 7)) =
              make_uint2(pack2bf(dp[kt][t][0], dp[kt][t][1]), pack2bf(dp[kt][t][2], dp[kt][t][3]));
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8_t p0 = pack_acc(s[0][2 * s2], s[0][2 * s2 + 1]);
        const bf16x8_t p1 = pack_acc(s[1][2 * s2], s[1][2 * s2 + 1]);
        const bf16x8_t e0 = pack_acc(dp[0][2 * s2], dp[0][2 * s2 + 1]);
        const bf16x8_t e1 = pack_acc(dp[1][2 * s2], dp[1][2 * s2 + 1]);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const bf16x8_t dot = frag_tr(Ds, 32 * s2, dt * 16, lane);
          const bf16x8_t qt = frag_tr(Qs, 32 * s2, dt * 16, lane);
          dv[0][dt] = MFMA16(dot, p0, dv[0][dt]);
          dv[1][dt] = MFMA16(dot, p1, dv[1][dt]);
          dk[0][dt] = MFMA16(qt, e0, dk[0][dt]);
          dk[1][dt] = MFMA16(qt, e1, dk[1][dt]);
        }
      }
    }
    // O rows of the next chunk (delta) only now: held across the dQ phase, not the products
    if (more && !stq) ld(Og, a.o_ss, q0 + 64, a.Sq, po);
    smi_lds_barrier();  // dS image complete; every read of the staged chunk done
    {
      // dQ^T tiles = sum over 32-key steps of K^T dS^T; causal: steps past the chunk are 0
      const int ns = MODE == 2 ? min(nstep, 2 * c + 2) : nstep;
      f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
      // fully unrolled, step st8 + 1's fragments read before step st8's MFMAs (reads past ns are
      // in bounds and unused)
      bf16x8_t kt[2], d0[2], d1[2];
      auto ldq = [&](int st8, int sl) {
        const int img = st8 >> 1, kr = 32 * (st8 & 1);
        kt[sl] = frag_tr(Ki[img], kr, 16 * dtq, lane);
        d0[sl] = frag_tr(dSi[img], kr, 32 * qpq, lane);
        d1[sl] = frag_tr(dSi[img], kr, 32 * qpq + 16, lane);
      };
      ldq(0, 0);
#pragma unroll
      for (int st8 = 0; st8 < 8; ++st8) {
        if (st8 + 1 < 8) ldq(st8 + 1, (st8 + 1) & 1);
        if (st8 < ns) {
          acc0 = MFMA16(kt[st8 & 1], d0[st8 & 1], acc0);
          acc1 = MFMA16(kt[st8 & 1], d1[st8 & 1], acc1);
        }
      }
      // lane: query q0 + 32 qpq (+ 16) + n, head dims 16 dtq + 4g .. + 3
      const int qa = q0 + 32 * qpq + n, qb = qa + 16;
      if (qa < a.Sq) store4(dQ + (long)qa * a.q_ss + 16 * dtq + 4 * g, acc0, a.scale);
      if (qb < a.Sq) store4(dQ + (long)qb * a.q_ss + 16 * dtq + 4 * g, acc1, a.scale);
    }
    if (more) stage_store();
    smi_lds_barrier();  // next chunk staged; every dS read done before the next chunk's writes
  }
  unsigned short* dK = a.dk + b * a.k_sb + h * a.k_sh;
  unsigned short* dV = a.dv + b * a.v_sb + h * a.v_sh;
  if (a.k_ss % 8 == 0 && a.v_ss % 8 == 0 && !((uintptr_t)dK & 15) && !((uintptr_t)dV & 15)) {
    // row-coalesced epilogue (the fp32 kernel's ae16): the wave parks its 32 keys x 64 dims of dK
    // and dV as bf16 in its own 4 KiB of the (now idle) K and dS images — 16-B chunk c of row r at
    // c ^ (r & 7) — and stores whole 128-B rows (8 rows per wave instruction) instead of 8-B
    // pieces of 16 rows.  The loop's last barrier retired every read of those images.
    unsigned short* ik = &Ki[0][0] + w * 2048;
    unsigned short* iv = &dSi[0][0] + w * 2048;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int r = kt * 16 + n, c = dt * 16 + 4 * g;
        const int off = r * 64 + ((((c >> 3) ^ r) & 7) << 3) + (c & 7);
        store4(ik + off, dk[kt][dt], a.scale);
        store4(iv + off, dv[kt][dt], 1.0f);
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's image writes are done
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int pc = it * 64 + lane, r = pc >> 3, ch = pc & 7;
      const int off = r * 64 + (((ch ^ r) & 7) << 3);
      const u16x8_t vk = *(const u16x8_t*)(ik + off), vv = *(const u16x8_t*)(iv + off);
      const int kj = kwave + r;
      if (kj < a.Sk) {
        *(u16x8_t*)(dK + (long)kj * a.k_ss + ch * 8) = vk;
        *(u16x8_t*)(dV + (long)kj * a.v_ss + ch * 8) = vv;
      }
    }
    return;
  }
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int kj = kwave + kt * 16 + n;
    if (kj < a.Sk) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        store4(dK + (long)kj * a.k_ss + dt * 16 + 4 * g, dk[kt][dt], a.scale);
        store4(dV + (long)kj * a.v_ss + dt * 16 + 4 * g, dv[kt][dt], 1.0f);
      }
    }
  }
}

#define SMI_ATTN_DISPATCH_NT(KERNEL, GRID, NT, ARGS)                                                        \
  do {                                                                                                     \
    const bool kp_ = (ARGS).kpad != nullptr;                                                               \
    switch ((ARGS).mode) {                                                                                 \
      case 0: if (kp_) hipLaunchKernelGGL((KERNEL<0, true>), GRID, dim3(NT), 0, st, ARGS);                 \
              else hipLaunchKernelGGL((KERNEL<0, false>), GRID, dim3(NT), 0, st, ARGS); break;             \
      case 1: if (kp_) hipLaunchKernelGGL((KERNEL<1, true>), GRID, dim3(NT), 0, st, ARGS);                 \
              else hipLaunchKernelGGL((KERNEL<1, false>), GRID, dim3(NT), 0, st, ARGS); break;             \
      case 2: if (kp_) hipLaunchKernelGGL((KERNEL<2, true>), GRID, dim3(NT), 0, st, ARGS);                 \
              else hipLaunchKernelGGL((KERNEL<2, false>), GRID, dim3(NT), 0, st, ARGS); break;             \
      default: return -1;                                                                                  \
    }                                                                                                      \
  } while (0)
#define SMI_ATTN_DISPATCH(KERNEL, GRID, ARGS) SMI_ATTN_DISPATCH_NT(KERNEL, GRID, 256, ARGS)
extern "C" int smi_attn_bwd1(int);

extern "C" int smi_attn_fwd(const AttnFwdArgs* args, hipStream_t st) {
  const AttnFwdArgs& a = *args;
  dim3 grid((a.Sq + 127) / 128, a.H, a.B);
  SMI_ATTN_DISPATCH(attn_fwd_kernel, grid, a);
  SMI_CHECK_LAUNCH();
}

extern "C" int smi_attn_bwd(const AttnBwdArgs* args, const void* o, float* delta, hipStream_t st) {
  const AttnBwdArgs& a = *args;
  // delta = rowsum(dO * O) is computed inside the dQ kernel (it already holds dO's rows) and
  // handed to the dK/dV kernel through `delta` — no separate launch
  AttnBwdArgs b2 = a;
  b2.o = (const unsigned short*)o;
  b2.delta_out = delta;
  b2.delta = delta;
  if (a.Sk <= 256 && smi_attn_bwd1(-1)) {
    SMI_ATTN_DISPATCH_NT(attn_bwd8_kernel, dim3(1, a.H, a.B), 512, b2);
  } else {
    SMI_ATTN_DISPATCH(attn_bwd_dq_kernel, dim3((a.Sq + 127) / 128, a.H, a.B), b2);
    SMI_ATTN_DISPATCH(attn_bwd_dkdv_kernel, dim3((a.Sk + 127) / 128, a.H, a.B), b2);
  }
  SMI_CHECK_LAUNCH();
}
