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
// Structure (MI355X): one workgroup = 4 waves = 64 rows of the "owned" axis, 16 per wave.
// The streamed operand (64-row chunks) is staged in LDS: a row-major image with the 16-B
// chunk XOR swizzle (c ^ (row & 7)) for the ds_read_b128 A-operand reads, and a transposed
// image with a 144-B row pitch (conflict-free ds_read_b64) for the B operand of the second
// product.  S is computed transposed (K·Qᵀ) so each lane owns one query column and the
// 16x16 accumulators of two adjacent key tiles form the bf16 A operand of P·V directly
// (k order permuted identically on both operands; cdna_hip_programming.md §3).
#include "smi_common.h"

#define LOG2E_F 1.4426950408889634f

#include "smi_attention.h"

#define VT_PITCH 72  // transposed image row pitch in bf16 elements (144 B)

__device__ __forceinline__ int swz(int row, int chunk) { return row * 64 + ((chunk ^ (row & 7)) << 3); }

// Stage 64 rows x 64 d of X (row-major, swizzled) and optionally its transpose into LDS.
__device__ __forceinline__ void stage_rows(const unsigned short* __restrict__ base, long ss, int r0, int rmax,
                                           unsigned short* rowimg, unsigned short* trimg) {
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int row = i >> 3, c = i & 7, r = r0 + row;
    u16x8_t val;
    if (r < rmax) val = *(const u16x8_t*)(base + (long)r * ss + c * 8);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) val[j] = 0;
    }
    if (rowimg) *(u16x8_t*)(rowimg + swz(row, c)) = val;
    if (trimg) {
#pragma unroll
      for (int j = 0; j < 8; ++j) trimg[(c * 8 + j) * VT_PITCH + row] = val[j];
    }
  }
}

__device__ __forceinline__ bf16x8_t lds_a(const unsigned short* img, int row, int chunk) {
  return *(const bf16x8_t*)(img + swz(row, chunk));
}
// B operand of the second product: 8 values of transposed row `drow` at keys
// {32s+4g .. +3} and {32s+16+4g .. +3} (the permuted k order).
__device__ __forceinline__ bf16x8_t lds_bt(const unsigned short* tr, int drow, int s, int g) {
  const uint2 lo = *(const uint2*)(tr + drow * VT_PITCH + 32 * s + 4 * g);
  const uint2 hi = *(const uint2*)(tr + drow * VT_PITCH + 32 * s + 16 + 4 * g);
  bf16x8_t r;
  r[0] = (short)(lo.x & 0xffff); r[1] = (short)(lo.x >> 16); r[2] = (short)(lo.y & 0xffff); r[3] = (short)(lo.y >> 16);
  r[4] = (short)(hi.x & 0xffff); r[5] = (short)(hi.x >> 16); r[6] = (short)(hi.y & 0xffff); r[7] = (short)(hi.y >> 16);
  return r;
}
__device__ __forceinline__ bf16x8_t pack_acc(const f32x4_t& a, const f32x4_t& b) {
  bf16x8_t r;
#pragma unroll
  for (int j = 0; j < 4; ++j) { r[j] = (short)f2bf(a[j]); r[4 + j] = (short)f2bf(b[j]); }
  return r;
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

#define MFMA16(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

// masked, biased, log2-scaled score; returns -inf for masked-out entries
__device__ __forceinline__ float score_adj(float s, int qi, int kj, int Sk, int mode, const unsigned char* kp,
                                           float scale_log2) {
  if (kj >= Sk) return -INFINITY;
  if (mode == 2 && kj > qi) return -INFINITY;
  if (kp && kp[kj]) return -INFINITY;
  float x = s * scale_log2;
  if (mode == 1 && kj < qi) x += LOG2E_F;
  return x;
}

__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnFwdArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned short Ks[64 * 64];
  __shared__ __attribute__((aligned(16))) unsigned short Vt[64 * VT_PITCH];
  const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  const int q0 = qb * 64 + w * 16;
  const int qi = q0 + n;
  const unsigned short* Q = a.q + b * a.q_sb + h * a.q_sh;
  const unsigned short* K = a.k + b * a.k_sb + h * a.k_sh;
  const unsigned short* V = a.v + b * a.v_sb + h * a.v_sh;
  const unsigned char* kp = a.kpad ? a.kpad + (long)b * a.Sk : nullptr;
  bf16x8_t qf[2];
  qf[0] = load8(Q + (long)qi * a.q_ss + 8 * g, qi < a.Sq);
  qf[1] = load8(Q + (long)qi * a.q_ss + 32 + 8 * g, qi < a.Sq);
  float m = -INFINITY, l = 0.f;
  f32x4_t o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  int kend = a.Sk;
  if (a.mode == 2) kend = min(a.Sk, qb * 64 + 64);
  for (int k0 = 0; k0 < kend; k0 += 64) {
    __syncthreads();
    stage_rows(K, a.k_ss, k0, a.Sk, Ks, nullptr);
    stage_rows(V, a.v_ss, k0, a.Sk, nullptr, Vt);
    __syncthreads();
    f32x4_t s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) s[t] = MFMA16(lds_a(Ks, t * 16 + n, 4 * ks + g), qf[ks], s[t]);
    }
    float cmax = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kj = k0 + t * 16 + 4 * g + j;
        s[t][j] = score_adj(s[t][j], qi, kj, a.Sk, a.mode, kp, a.scale_log2);
        cmax = fmaxf(cmax, s[t][j]);
      }
    cmax = fmaxf(cmax, __shfl_xor(cmax, 16, 64));
    cmax = fmaxf(cmax, __shfl_xor(cmax, 32, 64));
    const float mnew = fmaxf(m, cmax);
    const float mref = (mnew == -INFINITY) ? 0.f : mnew;
    const float alpha = exp2f(m - mref);
    float psum = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) { s[t][j] = exp2f(s[t][j] - mref); psum += s[t][j]; }
    psum += __shfl_xor(psum, 16, 64);
    psum += __shfl_xor(psum, 32, 64);
    l = l * alpha + psum;
    m = mnew;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float aj = __shfl(alpha, 4 * g + j, 64);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt][j] *= aj;
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8_t pa = pack_acc(s[2 * s2], s[2 * s2 + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt] = MFMA16(pa, lds_bt(Vt, dt * 16 + n, s2, g), o[dt]);
    }
  }
  unsigned short* O = a.o + b * a.o_sb + h * a.o_sh;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float lj = __shfl(l, 4 * g + j, 64);
    const float inv = lj > 0.f ? 1.0f / lj : 0.f;
    const int qq = q0 + 4 * g + j;
    if (qq < a.Sq) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) O[(long)qq * a.o_ss + dt * 16 + n] = f2bf(o[dt][j] * inv);
    }
  }
  if (g == 0 && qi < a.Sq) {
    const float mref = (m == -INFINITY) ? 0.f : m;
    a.lse[((long)b * a.H + h) * a.Sq + qi] = l > 0.f ? mref + log2f(l) : INFINITY;
  }
}

// delta[b,h,q] = sum_d dO * O
__global__ void attn_delta_kernel(const unsigned short* __restrict__ o, const unsigned short* __restrict__ dout,
                                  long o_sb, long o_ss, long o_sh, float* __restrict__ delta, int B, int H, int Sq) {
  const int lane = threadIdx.x & 63;
  const long wg = (long)blockIdx.x * 4 + (threadIdx.x >> 6);  // one wave per (b, q, head-group of 8)
  const int hg_n = (H + 7) / 8;
  if (wg >= (long)B * Sq * hg_n) return;
  const int hg = wg % hg_n;
  const int q = (wg / hg_n) % Sq;
  const int b = wg / ((long)hg_n * Sq);
  const int h = hg * 8 + (lane >> 3);
  float s = 0.f;
  if (h < H) {
    const long off = b * o_sb + (long)q * o_ss + h * o_sh + (lane & 7) * 8;
    u16x8_t x = *(const u16x8_t*)(o + off);
    u16x8_t y = *(const u16x8_t*)(dout + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += bf2f(x[j]) * bf2f(y[j]);
  }
  s = group_sum<8>(s);
  if (h < H && (lane & 7) == 0) delta[((long)b * H + h) * Sq + q] = s;
}

// dQ: one workgroup per (q-block of 64, h, b); queries on lanes, keys streamed.
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(AttnBwdArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned short Ks[64 * 64];
  __shared__ __attribute__((aligned(16))) unsigned short Vs[64 * 64];
  __shared__ __attribute__((aligned(16))) unsigned short Kt[64 * VT_PITCH];
  const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  const int q0 = qb * 64 + w * 16;
  const int qi = q0 + n;
  const unsigned short* Q = a.q + b * a.q_sb + h * a.q_sh;
  const unsigned short* K = a.k + b * a.k_sb + h * a.k_sh;
  const unsigned short* V = a.v + b * a.v_sb + h * a.v_sh;
  const unsigned short* dO = a.dout + b * a.o_sb + h * a.o_sh;
  const unsigned char* kp = a.kpad ? a.kpad + (long)b * a.Sk : nullptr;
  const bool qok = qi < a.Sq;
  bf16x8_t qf[2], df[2];
  qf[0] = load8(Q + (long)qi * a.q_ss + 8 * g, qok);
  qf[1] = load8(Q + (long)qi * a.q_ss + 32 + 8 * g, qok);
  df[0] = load8(dO + (long)qi * a.o_ss + 8 * g, qok);
  df[1] = load8(dO + (long)qi * a.o_ss + 32 + 8 * g, qok);
  const long rowidx = ((long)b * a.H + h) * a.Sq + qi;
  const float lse = qok ? a.lse[rowidx] : INFINITY;
  const float dl = qok ? a.delta[rowidx] : 0.f;
  f32x4_t acc[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) acc[dt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  int kend = a.Sk;
  if (a.mode == 2) kend = min(a.Sk, qb * 64 + 64);
  for (int k0 = 0; k0 < kend; k0 += 64) {
    __syncthreads();
    stage_rows(K, a.k_ss, k0, a.Sk, Ks, Kt);
    stage_rows(V, a.v_ss, k0, a.Sk, Vs, nullptr);
    __syncthreads();
    f32x4_t s[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
      dp[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        s[t] = MFMA16(lds_a(Ks, t * 16 + n, 4 * ks + g), qf[ks], s[t]);
        dp[t] = MFMA16(lds_a(Vs, t * 16 + n, 4 * ks + g), df[ks], dp[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kj = k0 + t * 16 + 4 * g + j;
        const float x = score_adj(s[t][j], qi, kj, a.Sk, a.mode, kp, a.scale_log2);
        const float p = (x == -INFINITY) ? 0.f : exp2f(x - lse);
        s[t][j] = p * (dp[t][j] - dl);  // dS (w.r.t. the scaled score)
      }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8_t pa = pack_acc(s[2 * s2], s[2 * s2 + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) acc[dt] = MFMA16(pa, lds_bt(Kt, dt * 16 + n, s2, g), acc[dt]);
    }
  }
  unsigned short* dQ = a.dq + b * a.q_sb + h * a.q_sh;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int qq = q0 + 4 * g + j;
    if (qq < a.Sq) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dQ[(long)qq * a.q_ss + dt * 16 + n] = f2bf(acc[dt][j] * a.scale);
    }
  }
}

// dK, dV: one workgroup per (k-block of 64, h, b); keys on lanes, queries streamed.
__global__ __launch_bounds__(256) void attn_bwd_dkdv_kernel(AttnBwdArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned short Qs[64 * 64];
  __shared__ __attribute__((aligned(16))) unsigned short Ds[64 * 64];
  __shared__ __attribute__((aligned(16))) unsigned short Qt[64 * VT_PITCH];
  __shared__ __attribute__((aligned(16))) unsigned short Dt[64 * VT_PITCH];
  __shared__ float lse_s[64], dl_s[64];
  const int kb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;
  const int kw0 = kb * 64 + w * 16;
  const int kj = kw0 + n;
  const unsigned short* Q = a.q + b * a.q_sb + h * a.q_sh;
  const unsigned short* K = a.k + b * a.k_sb + h * a.k_sh;
  const unsigned short* V = a.v + b * a.v_sb + h * a.v_sh;
  const unsigned short* dO = a.dout + b * a.o_sb + h * a.o_sh;
  const bool kok = kj < a.Sk && !(a.kpad && a.kpad[(long)b * a.Sk + kj]);
  bf16x8_t kf[2], vf[2];
  kf[0] = load8(K + (long)kj * a.k_ss + 8 * g, kj < a.Sk);
  kf[1] = load8(K + (long)kj * a.k_ss + 32 + 8 * g, kj < a.Sk);
  vf[0] = load8(V + (long)kj * a.v_ss + 8 * g, kj < a.Sk);
  vf[1] = load8(V + (long)kj * a.v_ss + 32 + 8 * g, kj < a.Sk);
  f32x4_t dk[4], dv[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) { dk[dt] = (f32x4_t){0.f, 0.f, 0.f, 0.f}; dv[dt] = dk[dt]; }
  const long rowbase = ((long)b * a.H + h) * a.Sq;
  int qstart = 0;
  if (a.mode == 2) qstart = (kb * 64) & ~63;
  for (int q0 = qstart; q0 < a.Sq; q0 += 64) {
    __syncthreads();
    stage_rows(Q, a.q_ss, q0, a.Sq, Qs, Qt);
    stage_rows(dO, a.o_ss, q0, a.Sq, Ds, Dt);
    if (threadIdx.x < 64) {
      const int qq = q0 + threadIdx.x;
      lse_s[threadIdx.x] = qq < a.Sq ? a.lse[rowbase + qq] : INFINITY;
      dl_s[threadIdx.x] = qq < a.Sq ? a.delta[rowbase + qq] : 0.f;
    }
    __syncthreads();
    f32x4_t s[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
      dp[t] = s[t];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        s[t] = MFMA16(lds_a(Qs, t * 16 + n, 4 * ks + g), kf[ks], s[t]);
        dp[t] = MFMA16(lds_a(Ds, t * 16 + n, 4 * ks + g), vf[ks], dp[t]);
      }
    }
    // s[t][j] : query q0 + t*16 + 4g + j, key kj
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ql = t * 16 + 4 * g + j;
        const int qq = q0 + ql;
        float p = 0.f;
        if (kok && qq < a.Sq && !(a.mode == 2 && kj > qq)) {
          float x = s[t][j] * a.scale_log2;
          if (a.mode == 1 && kj < qq) x += LOG2E_F;
          p = exp2f(x - lse_s[ql]);
        }
        s[t][j] = p;
        dp[t][j] = p * (dp[t][j] - dl_s[ql]);
      }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const bf16x8_t pa = pack_acc(s[2 * s2], s[2 * s2 + 1]);
      const bf16x8_t da = pack_acc(dp[2 * s2], dp[2 * s2 + 1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dv[dt] = MFMA16(pa, lds_bt(Dt, dt * 16 + n, s2, g), dv[dt]);
        dk[dt] = MFMA16(da, lds_bt(Qt, dt * 16 + n, s2, g), dk[dt]);
      }
    }
  }
  unsigned short* dK = a.dk + b * a.k_sb + h * a.k_sh;
  unsigned short* dV = a.dv + b * a.v_sb + h * a.v_sh;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int kk = kw0 + 4 * g + j;
    if (kk < a.Sk) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dK[(long)kk * a.k_ss + dt * 16 + n] = f2bf(dk[dt][j] * a.scale);
        dV[(long)kk * a.v_ss + dt * 16 + n] = f2bf(dv[dt][j]);
      }
    }
  }
}

extern "C" int smi_attn_fwd(const AttnFwdArgs* args, hipStream_t st) {
  const AttnFwdArgs& a = *args;
  dim3 grid((a.Sq + 63) / 64, a.H, a.B);
  hipLaunchKernelGGL(attn_fwd_kernel, grid, dim3(256), 0, st, a);
  SMI_CHECK_LAUNCH();
}

extern "C" int smi_attn_bwd(const AttnBwdArgs* args, const void* o, float* delta, hipStream_t st) {
  const AttnBwdArgs& a = *args;
  const long waves = (long)a.B * a.Sq * ((a.H + 7) / 8);
  hipLaunchKernelGGL(attn_delta_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st,
                     (const unsigned short*)o, a.dout, a.o_sb, a.o_ss, a.o_sh, delta, a.B, a.H, a.Sq);
  AttnBwdArgs b2 = a;
  b2.delta = delta;
  hipLaunchKernelGGL(attn_bwd_dq_kernel, dim3((a.Sq + 63) / 64, a.H, a.B), dim3(256), 0, st, b2);
  hipLaunchKernelGGL(attn_bwd_dkdv_kernel, dim3((a.Sk + 63) / 64, a.H, a.B), dim3(256), 0, st, b2);
  SMI_CHECK_LAUNCH();
}
