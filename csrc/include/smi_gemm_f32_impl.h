// Shared device code of the fp32 GEMM (tiles, split-product paths, epilogues, kernel templates);
// instantiated per mode in csrc/kernels/gemm_f32{,_dgrad,_wgrad}.hip so the three translation
// units compile in parallel.
#pragma once
// fp32 GEMM on the fp32-input matrix cores (v_mfma_f32_32x32x2_f32: exact f32 products and an
// f32 fmaf accumulation chain, 64 FLOP/clk/SIMD = 157 TF dense) with the same fused epilogues as
// the bf16 GEMM — the REFERENCE-PRECISION path of every Linear of the reference models
// (transformer.py:71-72,107-117,175-176,271 run in fp32 by pytorch_machine_translator.py:120-137):
//
//   FWD   C[M,N]  = X[M,K] . W[N,K]^T  (+bias, ReLU, dropout)        A k-contig, B k-contig
//   DGRAD dX[M,K] = dY[M,N] . W[N,K]   (+residual, x relu'/dropout)  A k-contig, B k-major
//   WGRAD dW[N,K] += dY[M,N]^T . X[M,K] (+ bias grad = dY^T 1)       A k-major,  B k-major
//
// CDNA4 design.  The f32 MFMA runs at 1/16 of the bf16 rate, so this kernel is matrix-core bound
// by a wide margin (a 32-deep k-tile of a 128 x 128 tile = 64 MFMAs = 4096 cycles per
// SIMD against 32 KiB of L2 -> LDS traffic per workgroup): everything else is arranged so the
// MFMA pipe never idles —
//  * 256-thread workgroups (2 x 2 waves), BN = 128, BM = 64 or 128 (a wave owns 32*FM x 64 =
//    FM x 2 accumulators of 32 x 32), two workgroups per CU so one's barrier / epilogue overlaps
//    the other's MFMAs;
//  * register-staged double buffering: the next k-tile's float4 global loads are issued before
//    the current k-tile's MFMAs and written to the other LDS buffer after them — one barrier
//    per k-tile, global latency hidden under 2-4 k us of matrix work;
//  * k-permuted fragments: lane half h of a 32x32x2 MFMA supplies k = 16h + s at step s, so a
//    k-contiguous operand is read as four ds_read_b128 per 16 steps from an LDS image with a
//    36-float row pitch (conflict-free for the ds_read_b128 lane groups), and a k-major operand
//    as ds_read_b32 rows (32 consecutive floats per half-wave: conflict-free, no transpose);
//  * XCD-aware tile order (tiles sharing an A row-panel run on one XCD's L2).
// The accumulator layout (col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)) gives each
// store instruction two full 128-B row segments.
#include "smi_common.h"
#include "smi_gemm_f32.h"
#include "smi_split3.h"

#define FBN 128
#define FBK 32
#define KC_PITCH 36  // k-contig LDS row pitch (floats)
#define NUM_CU 256

template <bool KMAJ, int R>
struct F32Tile {
  // floats of one staged operand tile: k-contig [R rows][36], k-major [32 k][R cols]
  static constexpr int ELEMS = KMAJ ? FBK * R : R * KC_PITCH;
  static constexpr int NV = R / 32;  // float4 staging loads per thread
};

// Branch-free global -> register staging through a buffer descriptor: out-of-range rows / k read
// 0 because their offset is pushed past the descriptor's extent (the range check returns zeros),
// so a k-loop body stays ONE basic block and sched_group_barrier can interleave it.
#define F32_OOB 0x7FFFFFF0
template <bool KMAJ, int R>
__device__ __forceinline__ void f32_bload(__amdgpu_buffer_rsrc_t rs, long ld, int r0, int rlim, int k0, int klim,
                                          float4 (&v)[F32Tile<KMAJ, R>::NV], int tid) {
#pragma unroll
  for (int i = 0; i < F32Tile<KMAJ, R>::NV; ++i) {
    const int f = tid + 256 * i;
    int off;
    if (!KMAJ) {
      const int gr = r0 + (f >> 3), gk = k0 + (f & 7) * 4;
      off = (gr < rlim && gk < klim) ? (int)(((long)gr * ld + gk) * 4) : F32_OOB;
    } else {
      const int gk = k0 + f / (R / 4), gc = r0 + (f % (R / 4)) * 4;
      off = (gk < klim && gc < rlim) ? (int)(((long)gk * ld + gc) * 4) : F32_OOB;
    }
    v[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
  }
}

template <bool KMAJ, int R>
__device__ __forceinline__ void f32_lstore(float* __restrict__ lds, const float4 (&v)[F32Tile<KMAJ, R>::NV], int tid) {
#pragma unroll
  for (int i = 0; i < F32Tile<KMAJ, R>::NV; ++i) {
    const int f = tid + 256 * i;
    if (!KMAJ) *(float4*)(lds + (f >> 3) * KC_PITCH + (f & 7) * 4) = v[i];
    else *(float4*)(lds + (f / (R / 4)) * R + (f % (R / 4)) * 4) = v[i];
  }
}

// The 16 k-values (k = 16h + s, s = 0..15) this lane feeds the 32x32x2 MFMAs of one 32-row /
// 32-col fragment starting at tile row/col c0.
template <bool KMAJ, int R>
__device__ __forceinline__ void f32_frag(const float* __restrict__ lds, int c0, int lane, float (&f)[16]) {
  const int rc = c0 + (lane & 31), h = lane >> 5;
  if (!KMAJ) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 t = *(const float4*)(lds + rc * KC_PITCH + 16 * h + 4 * q);
      f[4 * q] = t.x; f[4 * q + 1] = t.y; f[4 * q + 2] = t.z; f[4 * q + 3] = t.w;
    }
  } else {
#pragma unroll
    for (int s = 0; s < 16; ++s) f[s] = lds[(16 * h + s) * R + rc];
  }
}

__device__ __forceinline__ int f32_tile_remap(int orig, int nwg) {
  // XCD-aware bijective remap: consecutive blocks land on different XCDs (b % 8); give each XCD a
  // contiguous range of tiles so tiles sharing an A row-panel share its L2
  if (nwg < 16) return orig;
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// ---- fp32 products on the bf16 matrix cores (3-way split, 6 product terms) ----
// x = hi + mid + lo exactly (three bf16 slices of 8 significant bits each, round-to-nearest-even
// at every step, so each residual is exact in fp32), and every slice product is exact in the
// fp32 accumulator.  a.b = hi.hi + (hi.mid + mid.hi + hi.lo + mid.mid + lo.hi) + O(2^-24 |a||b|):
// the dropped terms (mid.lo, lo.mid, lo.lo) are below one fp32 rounding of the product, and the
// big term is accumulated in its OWN fp32 chain (same rounding sequence as the f32 MFMA path) with
// the five correction terms in a second accumulator added once at the end.  Rate: 6 x
// v_mfma_f32_32x32x16_bf16 (32 cycles each) per 32x32x16 block vs 8 x v_mfma_f32_32x32x2_f32
// (64 cycles each) — 2.7x the f32 matrix-core rate for the same exact-product fp32 arithmetic.

// Compile-time epilogue feature set of the pipelined kernel (EPI < 0: generic runtime flags).
// Measured: the runtime-generic epilogue was ~9,700 instructions per wave (per-element mode /
// flag branches, 64-bit address math, scalar loads of the C operand) = the ~20 us fixed cost of
// every launch in the K scan (tools/f32_kscan.py); the specialised, LDS-staged one below is a
// few hundred.
enum : int { FE_BIAS = 1, FE_RELU = 2, FE_SIG = 4, FE_DROP = 8, FE_RESID = 16, FE_DACT = 32, FE_ACC = 64, FE_ATOMIC = 128 };
#define FE_PITCH 132  // LDS pitch of the staged 128 x 128 fp32 tile (conflict-free both passes)

template <int EPI>
__device__ __forceinline__ bool fe_has(const GemmF32Args& g, int f) {
  if constexpr (EPI >= 0) return (EPI & f) != 0;
  switch (f) {
    case FE_BIAS: return g.mode == 0 && g.bias;
    case FE_RELU: return g.mode == 0 && g.relu == 1;
    case FE_SIG: return g.mode == 0 && g.relu == 2;
    case FE_DROP: return g.mode == 0 && g.thresh;
    case FE_RESID: return g.mode == 1 && g.resid;
    case FE_DACT: return g.mode == 1 && g.dact_y;
    case FE_ACC: return g.beta_acc && !g.atomic;
    case FE_ATOMIC: return g.atomic;
  }
  return false;
}

// The accumulators go through LDS once ([128][132] image, 66 KiB of the idle stage ring) so each
// thread then owns 4 consecutive columns of 16 rows: float4 operand loads (bias once, residual /
// mask / C per row) and float4 stores of whole 512-B row segments, no per-element addressing.
template <bool AK, int EPI>
__device__ __forceinline__ void f32_epilogue_lds(const GemmF32Args& g, f32x16_t (&acc)[2][2], float (&bsum)[2], int m0,
                                                 int n0, int wm, int wn, int lane, bool do_bias, float* smem) {
  const int tid = threadIdx.x, h = lane >> 5;
  __syncthreads();  // every wave is done reading the k-loop's LDS stages
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        smem[(wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * FE_PITCH + wn * 64 + j * 32 + (lane & 31)] = acc[i][j][r];
  __syncthreads();
  const int c4 = (tid & 31) * 4, col = n0 + c4;
  // float4 stores / loads need 16-B aligned rows: ragged leading dimensions take the scalar path
  const bool vec = ((g.ldc | (fe_has<EPI>(g, FE_RESID) ? g.ldr : 0) | (fe_has<EPI>(g, FE_DACT) ? g.ldy : 0)) & 3) == 0;
  const bool full_cols = vec && col + 3 < g.N;
  const uint32_t seed = fe_has<EPI>(g, FE_DROP) ? smi_seed(g.seedp, g.salt) : 0u;
  float4 bia = make_float4(0.f, 0.f, 0.f, 0.f);
  if (fe_has<EPI>(g, FE_BIAS)) {
    if (full_cols) bia = *(const float4*)(g.bias + col);
    else {
      if (col < g.N) bia.x = g.bias[col];
      if (col + 1 < g.N) bia.y = g.bias[col + 1];
      if (col + 2 < g.N) bia.z = g.bias[col + 2];
      if (col + 3 < g.N) bia.w = g.bias[col + 3];
    }
  }
  const float bb[4] = {bia.x, bia.y, bia.z, bia.w};
#pragma unroll 4
  for (int q = 0; q < 16; ++q) {
    const int rl = (tid >> 5) + 8 * q, row = m0 + rl;
    if (row >= g.M || col >= g.N) continue;
    const float4 t = *(const float4*)(smem + rl * FE_PITCH + c4);
    float v[4] = {t.x, t.y, t.z, t.w};
    const long cidx = (long)row * g.ldc + col;
    if (full_cols) {
      float4 rs, dy, cc;
      if (fe_has<EPI>(g, FE_RESID)) rs = *(const float4*)(g.resid + (long)row * g.ldr + col);
      if (fe_has<EPI>(g, FE_DACT)) dy = *(const float4*)(g.dact_y + (long)row * g.ldy + col);
      if (fe_has<EPI>(g, FE_ACC)) cc = *(const float4*)(g.C + cidx);
      const float rv[4] = {rs.x, rs.y, rs.z, rs.w}, dv[4] = {dy.x, dy.y, dy.z, dy.w}, cv[4] = {cc.x, cc.y, cc.z, cc.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = v[e] + bb[e];
        if (fe_has<EPI>(g, FE_RELU)) x = fmaxf(x, 0.f);
        if (fe_has<EPI>(g, FE_SIG)) x = 1.f / (1.f + __expf(-x));
        if (fe_has<EPI>(g, FE_DROP)) x = smi_keep(seed, (uint32_t)(cidx + e), g.thresh) ? x * g.dscale : 0.f;
        if (fe_has<EPI>(g, FE_RESID)) x += rv[e];
        if (fe_has<EPI>(g, FE_DACT)) x = dv[e] > 0.f ? x * g.dscale : 0.f;
        if (fe_has<EPI>(g, FE_ACC)) x += cv[e];
        v[e] = x;
      }
      if (fe_has<EPI>(g, FE_ATOMIC)) {
#pragma unroll
        for (int e = 0; e < 4; ++e) atomicAdd(g.C + cidx + e, v[e]);
      } else {
        *(float4*)(g.C + cidx) = make_float4(v[0], v[1], v[2], v[3]);
      }
    } else {
      for (int e = 0; e < 4 && col + e < g.N; ++e) {
        float x = v[e] + bb[e];
        if (fe_has<EPI>(g, FE_RELU)) x = fmaxf(x, 0.f);
        if (fe_has<EPI>(g, FE_SIG)) x = 1.f / (1.f + __expf(-x));
        if (fe_has<EPI>(g, FE_DROP)) x = smi_keep(seed, (uint32_t)(cidx + e), g.thresh) ? x * g.dscale : 0.f;
        if (fe_has<EPI>(g, FE_RESID)) x += g.resid[(long)row * g.ldr + col + e];
        if (fe_has<EPI>(g, FE_DACT)) x = g.dact_y[(long)row * g.ldy + col + e] > 0.f ? x * g.dscale : 0.f;
        if (fe_has<EPI>(g, FE_ATOMIC)) atomicAdd(g.C + cidx + e, x);
        else g.C[cidx + e] = fe_has<EPI>(g, FE_ACC) ? g.C[cidx + e] + x : x;
      }
    }
  }
  if (AK && do_bias) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      // lanes l and l + 32 hold the two k-halves of row (l & 31)
      auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(bsum[i]), __float_as_uint(bsum[i]), false, false);
      const float tot = __uint_as_float(a[0]) + __uint_as_float(a[1]);
      const int row = m0 + wm * 64 + i * 32 + (lane & 31);
      if (h == 0 && row < g.M) {
        if (fe_has<EPI>(g, FE_ATOMIC)) atomicAdd(g.bias_grad + row, tot);
        else g.bias_grad[row] = fe_has<EPI>(g, FE_ACC) ? g.bias_grad[row] + tot : tot;
      }
    }
  }
}

// Software-pipelined form (one workgroup = one wave per SIMD, 128 x 128 tile, 3-stage LDS ring):
// measured on the two-workgroups-per-CU form, the matrix pipe idled ~37 % of the time — the two
// waves of a SIMD drift into lock-step (both in their load / barrier phase at once).  Here one
// wave per SIMD keeps the pipe busy by itself: every k-tile's 64 MFMAs are issued back to back
// while, in their shadow (an f32 32x32x2 MFMA occupies the pipe 64 cycles), the wave
//   * issues the global loads of k-tile t+3 (register set R[t&1]),
//   * reads k-tile t+1's fragments from LDS stage (t+1)%3 into the idle fragment set,
//   * writes k-tile t+2 (loaded one iteration earlier) into LDS stage (t+2)%3,
// interleaved one-per-MFMA by sched_group_barrier; one barrier per k-tile.
#define SGB(mask, n) __builtin_amdgcn_sched_group_barrier((mask), (n), 0)
#define SG_VALU 0x002  // (split paths)
#define SG_MFMA 0x008
#define SG_VMEM_RD 0x020
#define SG_DS_RD 0x100
#define SG_DS_WR 0x200
template <bool AK, bool BKM, int EPI, int XS = 0>
__device__ __forceinline__ void gemm_f32_tile_pipe(const GemmF32Args& g, int tile, int split, float* smem) {
  constexpr int FM = 2, BMT = 128;
  using TA = F32Tile<AK, BMT>;
  using TB = F32Tile<BKM, FBN>;
  constexpr int STAGE = TA::ELEMS + TB::ELEMS;
  constexpr int NRD = (AK ? 32 : 8) + (BKM ? 32 : 8);  // LDS fragment reads per k-tile per wave
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int ntn = (g.N + FBN - 1) / FBN;
  const int m0 = (tile / ntn) * BMT, n0 = (tile % ntn) * FBN;
  const int kbeg = split * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  const int nk = (kend - kbeg + FBK - 1) / FBK;
  f32x16_t acc[FM][2], cacc[FM][2];  // cacc: correction terms of the split-bf16 path (XS)
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = cacc[i][j][r] = 0.f;
  const bool do_bias = AK && g.bias_grad && n0 == 0 && wn == 0;
  float bsum[FM] = {0.f, 0.f};
  float af0[FM][16], bf0[2][16], af1[FM][16], bf1[2][16];
  float4 ra0[TA::NV], rb0[TB::NV], ra1[TA::NV], rb1[TB::NV];
  const long a_bytes = 4 * (AK ? (long)(g.K - 1) * g.lda + g.M : (long)(g.M - 1) * g.lda + g.K);
  const long b_bytes = 4 * (BKM ? (long)(g.K - 1) * g.ldb + g.N : (long)(g.N - 1) * g.ldb + g.K);
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)g.A, 0, (int)a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)g.B, 0, (int)b_bytes, 0x00020000);
  // every step is unconditional (tiles past nk load zeros into stages nobody reads): no branches
  auto ld = [&](int t, float4 (&ra)[TA::NV], float4 (&rb)[TB::NV]) {
    f32_bload<AK, BMT>(rA, g.lda, m0, g.M, kbeg + t * FBK, kend, ra, tid);
    f32_bload<BKM, FBN>(rB, g.ldb, n0, g.N, kbeg + t * FBK, kend, rb, tid);
  };
  auto st = [&](int t, const float4 (&ra)[TA::NV], const float4 (&rb)[TB::NV]) {
    float* d = smem + (t % 3) * STAGE;
    f32_lstore<AK, BMT>(d, ra, tid);
    f32_lstore<BKM, FBN>(d + TA::ELEMS, rb, tid);
  };
  auto rd = [&](int t, float (&af)[FM][16], float (&bf)[2][16]) {
    const float* ta = smem + (t % 3) * STAGE;
#pragma unroll
    for (int i = 0; i < FM; ++i) f32_frag<AK, BMT>(ta, wm * BMT / 2 + i * 32, lane, af[i]);
#pragma unroll
    for (int j = 0; j < 2; ++j) f32_frag<BKM, FBN>(ta + TA::ELEMS, wn * 64 + j * 32, lane, bf[j]);
  };
  auto mma = [&](float (&af)[FM][16], float (&bf)[2][16]) {
    if constexpr (XS == 1) {
      // k-block b of the 32-deep tile: lane half h feeds k = 16h + 8b + e (e = 0..7) — the same
      // k <-> (lane, slot) permutation for A and B, so the fp32 fragments are reused as read
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        Split3 sa[FM], sb[2];
#pragma unroll
        for (int i = 0; i < FM; ++i) sa[i] = split3_8(&af[i][8 * b]);
#pragma unroll
        for (int j = 0; j < 2; ++j) sb[j] = split3_8(&bf[j][8 * b]);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            acc[i][j] = MF32X16(sa[i].h, sb[j].h, acc[i][j]);
            cacc[i][j] = MF32X16(sa[i].l, sb[j].h, cacc[i][j]);
            cacc[i][j] = MF32X16(sa[i].m, sb[j].m, cacc[i][j]);
            cacc[i][j] = MF32X16(sa[i].h, sb[j].l, cacc[i][j]);
            cacc[i][j] = MF32X16(sa[i].m, sb[j].h, cacc[i][j]);
            cacc[i][j] = MF32X16(sa[i].h, sb[j].m, cacc[i][j]);
          }
      }
    } else {
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s2], bf[j][s2], acc[i][j], 0, 0, 0);
    }
    if constexpr (AK) {  // bias-gradient row sums (kept only by the column-block-0 waves)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2) bsum[i] += af[i][s2];
    }
  };
  // the interleave of one iteration: 8 x (MFMA, global load), reads, 8 x (MFMA, LDS write), rest
  auto schedule = [&]() {
    if constexpr (XS != 0) return;  // split path: compiler-scheduled (VALU splits between MFMAs)
#pragma unroll
    for (int i = 0; i < TA::NV + TB::NV; ++i) { SGB(SG_MFMA, 1); SGB(SG_VMEM_RD, 1); }
    if constexpr (NRD <= 40) {
#pragma unroll
      for (int i = 0; i < NRD; ++i) { SGB(SG_MFMA, 1); SGB(SG_DS_RD, 1); }
    } else {
#pragma unroll
      for (int i = 0; i < NRD / 2; ++i) { SGB(SG_MFMA, 1); SGB(SG_DS_RD, 2); }
    }
#pragma unroll
    for (int i = 0; i < TA::NV + TB::NV; ++i) { SGB(SG_MFMA, 1); SGB(SG_DS_WR, 1); }
    SGB(SG_MFMA, 64);
  };
  // prologue: k-tiles 0, 1 in LDS; k-tile 2 in R1; k-tile 0's fragments in F0
  ld(0, ra0, rb0);
  ld(1, ra1, rb1);
  st(0, ra0, rb0);
  st(1, ra1, rb1);
  ld(2, ra1, rb1);
  __syncthreads();
  rd(0, af0, bf0);
  // k-tiles in pairs with NO exit between the halves (an odd nk runs one extra all-zero k-tile:
  // tiles past nk load zeros): a mid-pair exit made the compiler keep the accumulators in two
  // register sets and copy 64 AGPRs per k-tile
  const int nk2 = (nk + 1) & ~1;
  for (int kt = 0; kt < nk2; kt += 2) {
    ld(kt + 3, ra0, rb0);
    rd(kt + 1, af1, bf1);
    st(kt + 2, ra1, rb1);
    mma(af0, bf0);
    schedule();
    __syncthreads();
    ld(kt + 4, ra1, rb1);
    rd(kt + 2, af0, bf0);
    st(kt + 3, ra0, rb0);
    mma(af1, bf1);
    schedule();
    __syncthreads();
  }
  if constexpr (XS != 0) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] += cacc[i][j];
  }
  f32_epilogue_lds<AK, EPI>(g, acc, bsum, m0, n0, wm, wn, lane, do_bias, smem);
}

// ---- split-at-stage form of the 3-way bf16 path (XS = 2) ----
// The fp32 k-tile is split ONCE, by the thread that stages it (each value once per workgroup, not
// once per reading wave), into three bf16 planes in LDS; the waves read MFMA-ready bf16x8
// fragments (one ds_read_b128 per plane per 16-deep block).  Staging thread map: each thread
// owns 4 consecutive k of a row — a float4 for a k-contiguous operand, four coalesced dword
// loads (adjacent lanes = adjacent rows) for a k-major one, so the transposition is free.
// LDS plane: [128 rows][32 k] bf16, 64-B rows, 16-B chunk index XOR-swizzled with (row >> 2) & 3
// (the 16 rows a ds_read_b128 quarter-wave touches land on 16 distinct bank quads); stage =
// 2 operands x 3 planes x 8 KiB = 48 KiB, 3 stages.
#define XS_PLANE 4096                    // bf16 per plane (128 x 32)
#define XS_OPER (3 * XS_PLANE)           // one operand's three planes
#define XS_STAGE (2 * XS_OPER)           // bf16 per stage
#define XS_SMEM_FLOATS (3 * XS_STAGE / 2)  // 3 stages, in floats (36864 = 144 KiB)

__device__ __forceinline__ int xs_off(int row, int k) {  // bf16 offset of (row, k) in a plane; k % 4 == 0
  return row * 32 + ((((k >> 3) ^ (row >> 2)) & 3) << 3) + (k & 7);
}

// k-major operand image: [32 k][128 rows] bf16 per plane (256-B k-rows), 16-B chunk ch of k-row r
// stored at chunk ch ^ (((r & 3) << 2) | ((r >> 2) & 3)) — conflict-free for both the staging
// writes and ds_read_b64_tr_b16 (cdna_hip_programming.md T10 image (b))
__device__ __forceinline__ int xs_koff(int k, int col) {  // col % 4 == 0
  return k * 128 + ((((col >> 3) ^ (((k & 3) << 2) | ((k >> 2) & 3))) & 15) << 3) + (col & 7);
}

// staging map: k-contiguous operand: thread f = tid + 256 i holds row f >> 3, k (f & 7) * 4 .. + 3
// (one float4); k-major: k-row (f >> 5), rows (f & 31) * 4 .. + 3 (one float4 of the natural layout)
template <bool KMAJ>
__device__ __forceinline__ void xs_bload(__amdgpu_buffer_rsrc_t rs, long ld, int r0, int rlim, int k0, int klim,
                                         float4 (&v)[4], int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int f = tid + 256 * i;
    int off;
    if (!KMAJ) {
      const int gr = r0 + (f >> 3), gk = k0 + (f & 7) * 4;
      off = (gr < rlim && gk < klim) ? (int)(((long)gr * ld + gk) * 4) : F32_OOB;
    } else {
      const int gk = k0 + (f >> 5), gc = r0 + (f & 31) * 4;
      off = (gk < klim && gc < rlim) ? (int)(((long)gk * ld + gc) * 4) : F32_OOB;
    }
    v[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
  }
}

// split the staged values into the three planes of one operand (dst = that operand's plane 0)
template <bool KMAJ>
__device__ __forceinline__ void xs_lstore(unsigned short* __restrict__ dst, const float4 (&v)[4], int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int f = tid + 256 * i;
    const int o = KMAJ ? xs_koff(f >> 5, (f & 31) * 4) : xs_off(f >> 3, (f & 7) * 4);
    uint32_t h0, m0, l0, h1, m1, l1;
    split3_pair(v[i].x, v[i].y, h0, m0, l0);
    split3_pair(v[i].z, v[i].w, h1, m1, l1);
    *(uint2*)(dst + o) = make_uint2(h0, h1);
    *(uint2*)(dst + XS_PLANE + o) = make_uint2(m0, m1);
    *(uint2*)(dst + 2 * XS_PLANE + o) = make_uint2(l0, l1);
  }
}

// the three bf16x8 planes of a 32-row fragment (rows c0 + (lane & 31), k = 16 b + 8 h + e)
typedef __attribute__((ext_vector_type(4))) short xs_s16x4_t;
template <bool KMAJ>
__device__ __forceinline__ Split3 xs_frag(const unsigned short* __restrict__ op, int c0, int b, int lane) {
  Split3 r;
  if (!KMAJ) {
    const int row = c0 + (lane & 31), k = 16 * b + 8 * (lane >> 5);
    const int o = xs_off(row, k);
    r.h = *(const bf16x8_t*)(op + o);
    r.m = *(const bf16x8_t*)(op + XS_PLANE + o);
    r.l = *(const bf16x8_t*)(op + 2 * XS_PLANE + o);
  } else {
    // ds_read_b64_tr_b16 per 16-lane group g: lane 4q + p addresses k-row q of the 4 x 16 block
    // (columns 4p .. 4p + 3); lane i receives column i.  Group g: rows c0 + 16 (g & 1) + i,
    // k-half h = g >> 1; two reads give k = 16 b + 8 h + 0..3 and + 4..7.
    const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4;
    const int col = c0 + 16 * (g & 1) + 4 * p;
    const int kb = 16 * b + 8 * (g >> 1) + q;
    const int o0 = xs_koff(kb, col), o1 = xs_koff(kb + 4, col);
    bf16x8_t* outs[3] = {&r.h, &r.m, &r.l};
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
      const unsigned short* base = op + pl * XS_PLANE;
      const xs_s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) xs_s16x4_t*)(base + o0));
      const xs_s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) xs_s16x4_t*)(base + o1));
      *outs[pl] = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
    }
  }
  return r;
}

template <bool AK, bool BKM, int EPI>
__device__ __forceinline__ void gemm_xs_tile(const GemmF32Args& g, int tile, int split, float* smem) {
  constexpr int FM = 2;
  unsigned short* lds = (unsigned short*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int ntn = (g.N + FBN - 1) / FBN;
  const int m0 = (tile / ntn) * 128, n0 = (tile % ntn) * FBN;
  const int kbeg = split * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  const int nk = (kend - kbeg + FBK - 1) / FBK;
  f32x16_t acc[FM][2], cacc[FM][2];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = cacc[i][j][r] = 0.f;
  const bool do_bias = AK && g.bias_grad && n0 == 0;
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};  // AK: partial row sums of A rows (tid & 31) * 4 + j
  const long a_bytes = 4 * (AK ? (long)(g.K - 1) * g.lda + g.M : (long)(g.M - 1) * g.lda + g.K);
  const long b_bytes = 4 * (BKM ? (long)(g.K - 1) * g.ldb + g.N : (long)(g.N - 1) * g.ldb + g.K);
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)g.A, 0, (int)a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)g.B, 0, (int)b_bytes, 0x00020000);
  float4 ra0[4], rb0[4], ra1[4], rb1[4];
  auto ld = [&](int t, float4 (&ra)[4], float4 (&rb)[4]) {
    xs_bload<AK>(rA, g.lda, m0, g.M, kbeg + t * FBK, kend, ra, tid);
    xs_bload<BKM>(rB, g.ldb, n0, g.N, kbeg + t * FBK, kend, rb, tid);
  };
  auto st = [&](int t, const float4 (&ra)[4], const float4 (&rb)[4]) {
    unsigned short* d = lds + (t % 3) * XS_STAGE;
    xs_lstore<AK>(d, ra, tid);
    xs_lstore<BKM>(d + XS_OPER, rb, tid);
    if constexpr (AK) {
#pragma unroll
      for (int i = 0; i < 4; ++i) { bsum[0] += ra[i].x; bsum[1] += ra[i].y; bsum[2] += ra[i].z; bsum[3] += ra[i].w; }
    }
  };
  auto rd = [&](int t, int b, Split3 (&fa)[FM], Split3 (&fb)[2]) {
    const unsigned short* d = lds + (t % 3) * XS_STAGE;
#pragma unroll
    for (int i = 0; i < FM; ++i) fa[i] = xs_frag<AK>(d, wm * 64 + i * 32, b, lane);
#pragma unroll
    for (int j = 0; j < 2; ++j) fb[j] = xs_frag<BKM>(d + XS_OPER, wn * 64 + j * 32, b, lane);
  };
  auto mma = [&](const Split3 (&sa)[FM], const Split3 (&sb)[2]) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        acc[i][j] = MF32X16(sa[i].h, sb[j].h, acc[i][j]);
        cacc[i][j] = MF32X16(sa[i].l, sb[j].h, cacc[i][j]);
        cacc[i][j] = MF32X16(sa[i].m, sb[j].m, cacc[i][j]);
        cacc[i][j] = MF32X16(sa[i].h, sb[j].l, cacc[i][j]);
        cacc[i][j] = MF32X16(sa[i].m, sb[j].h, cacc[i][j]);
        cacc[i][j] = MF32X16(sa[i].h, sb[j].m, cacc[i][j]);
      }
  };
  constexpr int NVM = (AK ? 16 : 4) + (BKM ? 16 : 4);  // global load instructions per k-tile
  // one half-iteration: [block 0 MFMAs | global loads of t+3, block-1 fragment reads, split +
  // LDS writes of t+2 (first half)] [block 1 MFMAs | split + LDS writes (second half), next
  // k-tile's block-0 fragment reads]
  auto schedule = [&]() {
#pragma unroll
    for (int i = 0; i < 24; ++i) {
      SGB(SG_MFMA, 1);
      SGB(SG_VMEM_RD, (NVM + 23) / 24);
      if (i < 12) SGB(SG_DS_RD, 1);
      SGB(SG_VALU, 4);
      if (i >= 12) SGB(SG_DS_WR, 1);
    }
#pragma unroll
    for (int i = 0; i < 24; ++i) {
      SGB(SG_MFMA, 1);
      SGB(SG_VALU, 4);
      if (i < 12) SGB(SG_DS_WR, 1);
      else SGB(SG_DS_RD, 1);
    }
  };
  Split3 pa[FM], pb[2], qa[FM], qb[2];
  // prologue: k-tiles 0, 1 split into LDS, k-tile 2 in registers, block 0 of k-tile 0 in P
  ld(0, ra0, rb0);
  ld(1, ra1, rb1);
  st(0, ra0, rb0);
  st(1, ra1, rb1);
  ld(2, ra1, rb1);
  __syncthreads();
  rd(0, 0, pa, pb);
  const int nk2 = (nk + 1) & ~1;  // pairs of k-tiles, no exit between the halves (zero tiles past nk)
  for (int kt = 0; kt < nk2; kt += 2) {
    ld(kt + 3, ra0, rb0);
    rd(kt, 1, qa, qb);
    mma(pa, pb);
    st(kt + 2, ra1, rb1);
    rd(kt + 1, 0, pa, pb);
    mma(qa, qb);
    schedule();
    __syncthreads();
    ld(kt + 4, ra1, rb1);
    rd(kt + 1, 1, qa, qb);
    mma(pa, pb);
    st(kt + 3, ra0, rb0);
    rd(kt + 2, 0, pa, pb);
    mma(qa, qb);
    schedule();
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] += cacc[i][j];
  float bias_tot = 0.f;
  if (do_bias) {  // the 8 staging threads of a row group (tid & 31) combine through LDS in order
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) smem[(tid >> 5) * 128 + (tid & 31) * 4 + j] = bsum[j];
    __syncthreads();
    if (tid < 128) {
#pragma unroll
      for (int q = 0; q < 8; ++q) bias_tot += smem[q * 128 + tid];
    }
  }
  float nob[2] = {0.f, 0.f};
  f32_epilogue_lds<AK, EPI>(g, acc, nob, m0, n0, wm, wn, lane, false, smem);
  if (do_bias && tid < 128 && m0 + tid < g.M) {
    const int row = m0 + tid;
    if (fe_has<EPI>(g, FE_ATOMIC)) atomicAdd(g.bias_grad + row, bias_tot);
    else g.bias_grad[row] = fe_has<EPI>(g, FE_ACC) ? g.bias_grad[row] + bias_tot : bias_tot;
  }
}

template <bool AK, bool BKM, int EPI, int XS>
__global__ __launch_bounds__(256, 1) void gemm_f32_pipe_kernel(GemmF32Args g) {
  __shared__ __attribute__((aligned(16)))
  float smem[XS == 2 ? XS_SMEM_FLOATS : 3 * (F32Tile<AK, 128>::ELEMS + F32Tile<BKM, FBN>::ELEMS)];
  const int nwg = ((g.M + 127) / 128) * ((g.N + FBN - 1) / FBN);
  const int split = blockIdx.x / nwg;
  const int tile = f32_tile_remap(blockIdx.x - split * nwg, nwg);
  if constexpr (XS == 2) gemm_xs_tile<AK, BKM, EPI>(g, tile, split, smem);
  else gemm_f32_tile_pipe<AK, BKM, EPI, XS>(g, tile, split, smem);
}

// Grouped weight-gradient GEMMs (fp32): gw_e[n,k] += dY_e[T,n]^T X_e[T,k] (and gb_e[n] += dY_e^T 1)
// for up to WGF_MAX problems in ONE launch, no split-K: each 128 x 128 output tile reduces all T
// tokens and adds into the fp32 gradient (deterministic, no slabs, no atomics).  Problem e's
// tiles start at t0[e], a multiple of 8 (same XCD pattern as a standalone launch).  Queued by
// sparkmi/ops/_grad.py during the backward and flushed per gradient bucket / at its end.
#define WGF_MAX 40
#ifndef WGF_PF
#define WGF_PF 1
#endif
struct WgradGroupF32 {
  const float* A[WGF_MAX]; const float* B[WGF_MAX];
  float* C[WGF_MAX]; float* bias[WGF_MAX];
  int lda[WGF_MAX], ldb[WGF_MAX], n[WGF_MAX], k[WGF_MAX], T[WGF_MAX];
  int t0[WGF_MAX + 1]; int count;
};
template <int XS>
__global__ __launch_bounds__(256, 1) void gemm_f32_wgrad_group_kernel(WgradGroupF32 gr) {
  __shared__ __attribute__((aligned(16)))
  float smem[XS == 2 ? XS_SMEM_FLOATS : 3 * (F32Tile<true, 128>::ELEMS + F32Tile<true, FBN>::ELEMS)];
  const int t = blockIdx.x;
  int e = 0;
  while (e + 1 < gr.count && t >= gr.t0[e + 1]) ++e;  // uniform scan over <= WGF_MAX entries
  GemmF32Args g{};
  g.mode = 2; g.A = gr.A[e]; g.lda = gr.lda[e]; g.B = gr.B[e]; g.ldb = gr.ldb[e];
  g.M = gr.n[e]; g.N = gr.k[e]; g.K = gr.T[e]; g.C = gr.C[e]; g.ldc = gr.k[e];
  g.beta_acc = 1; g.atomic = 0; g.dscale = 1.f; g.splits = 1; g.k_per_split = g.K;
  g.bias_grad = gr.bias[e];
  const int nwg = ((g.M + 127) / 128) * ((g.N + FBN - 1) / FBN);
  const int lt = t - gr.t0[e];
  if (lt >= nwg) return;  // padding
  if constexpr (XS == 2) gemm_xs_tile<true, true, FE_ACC>(g, f32_tile_remap(lt, nwg), 0, smem);
  else gemm_f32_tile_pipe<true, true, FE_ACC, XS>(g, f32_tile_remap(lt, nwg), 0, smem);  // lt >= nwg: padding
}

