// Split-plane fp32 GEMM: shared device code, instantiated per mode in
// csrc/kernels/gemm_sp{,_dgrad,_wgrad}.hip (the three translation units compile in parallel).
//
//   FWD   C[M,N]  = X[M,K] . W[N,K]^T  (+bias, ReLU, dropout)        A k-contig, B k-contig
//   DGRAD dX[M,K] = dY[M,N] . W[N,K]   (+residual, x relu'/dropout)  A k-contig, B k-major
//   WGRAD dW[N,K] += dY[M,N]^T . X[M,K] (+ bias grad = dY^T 1)       A k-major,  B k-major
//
// Reference precision (fp32 operands, exact products, fp32 accumulation) on the bf16 matrix
// cores.  Both operands arrive PRE-SPLIT as three bf16 planes (x = hi + mid + lo exactly, see
// smi_gemm_sp.h): the weights are split by the optimizer when it updates them
// (csrc/kernels/optim.hip), activations by the kernel that produces them (or once by
// smi_split3).  The k-loop therefore contains no splitting arithmetic at all — it is the
// structure of a bf16 GEMM that issues SIX v_mfma_f32_32x32x16_bf16 per fragment pair
// (hi.hi into the main accumulator; lo.hi, mid.mid, hi.lo, mid.hi, hi.mid into a correction
// accumulator added once at the end: the dropped mid.lo / lo.mid / lo.lo terms are below one
// fp32 rounding of the product).  Per 32-deep k-step a 128 x 128 tile issues 48 MFMAs per wave
// against 48 KiB of staged planes, 32 B/clk/CU at the matrix-core rate.
//
// CDNA4 structure: 256-thread workgroups (2 x 2 waves, a wave owns 64 x 64 = 2 x 2 accumulators
// of 32 x 32), ONE workgroup per CU (147 KiB of LDS: three stages of 2 operands x 3 planes x
// 128 x 32 bf16).  Stages are filled by buffer_load_dwordx4 ... lds (LDS-DMA, no VGPR round trip;
// per-lane source offsets computed once per tile, the k advance is the scalar soffset; one buffer
// descriptor per plane, so out-of-range rows / k read as zero through the descriptor's extent).
// The LDS images carry their XOR swizzles in the per-lane SOURCE offsets (the DMA writes
// lane-linear): k-contig planes [128 rows][32 k] (64-B rows, 16-B chunk ^ (row >> 2) & 3, conflict
// free for the 32x32x16 A/B fragment reads), k-major planes [32 k][128 cols] (256-B k-rows,
// chunk ^ ((k & 3) << 2 | (k >> 2) & 3), read as fragments by ds_read_b64_tr_b16).  Two k-steps
// stay in flight (counted vmcnt, raw s_barrier, one barrier per k-step).  XCD-aware tile order.
#pragma once
#include "smi_common.h"
#include "smi_gemm_sp.h"
#include "smi_split3.h"

#define SP_BK 32            // k-step depth
#define SP_PL 4096          // bf16 per plane tile (128 x 32)
#define SP_OP (3 * SP_PL)   // one operand's three planes
#define SP_ST (2 * SP_OP)   // one stage: A then B (48 KiB)
#define SP_NS 3
#define SP_OOB 0x7FFFFFF0u  // offset past every descriptor extent: the DMA reads zeros
#define SP_EPI_PITCH 132    // LDS pitch (floats) of the staged 128 x 128 fp32 epilogue tile
#define SP_NUM_CU 256

// Wave layout of a 128 x 128 tile: NW = 4 (2 x 2 waves of 64 x 64, one wave per SIMD) or 8 (2 x 4
// waves of 64 x 32, two per SIMD: one wave's LDS-DMA / fragment-read issue runs beside its
// partner's MFMAs — measured, one wave per SIMD stalled on issue 62 % of its cycles).
template <int NW>
struct SpCfg {
  static constexpr int NT = 64 * NW;       // threads
  static constexpr int WGN = NW / 2;       // waves along N
  static constexpr int WCOL = 128 / WGN;   // columns per wave
  static constexpr int WJ = WCOL / 32;     // 32-column accumulator blocks per wave
  static constexpr int PPW = 8 / NW;       // DMA pieces (1 KiB) per wave per plane
  static constexpr int NDMA = 6 * PPW;     // DMA pieces per wave per stage
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
};

#ifdef SP_STAMPS
// diagnostic build only (tools/probes/sp_probe.hip): s_memrealtime (100 MHz) stamps of each
// workgroup's phases, written by thread 0 to a buffer no output depends on
__device__ unsigned long long* g_sp_stamps;
#define SP_STAMP(slot)                                                                     \
  do {                                                                                     \
    if (threadIdx.x == 0) g_sp_stamps[(long)blockIdx.x * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define SP_STAMP(slot) do {} while (0)
#endif

enum : int { SE_BIAS = 1, SE_RELU = 2, SE_DROP = 8, SE_RESID = 16, SE_DACT = 32, SE_ACC = 64, SE_DMASK = 256 };
enum : int { SO_C = 1, SO_P = 2, SO_M = 4 };  // epilogue outputs: fp32 C, planes P, positivity mask

typedef __attribute__((address_space(3))) void sp_lds_void;
typedef __attribute__((ext_vector_type(4))) short sp_s16x4_t;

// k-contig plane image [128 rows][32 k] (64-B rows), 16-B chunk ^ (row >> 2) & 3: conflict-free
// for the four lane groups of a ds_read_b128 of 32x32x16 fragments (rows c0 + (lane & 31), chunk
// 2 b + (lane >> 5)).
__device__ __forceinline__ int sp_off(int row, int k) {  // k % 8 == 0
  return row * 32 + ((((k >> 3) ^ (row >> 2)) & 3) << 3) + (k & 7);
}
// k-major plane image [32 k][128 cols] (256-B k-rows), chunk ^ ((k & 3) << 2 | (k >> 2) & 3)
__device__ __forceinline__ int sp_swz(int k) { return ((k & 3) << 2) | ((k >> 2) & 3); }
__device__ __forceinline__ int sp_koff(int k, int col) {  // col % 4 == 0
  return k * 128 + ((((col >> 3) ^ sp_swz(k)) & 15) << 3) + (col & 7);
}

__device__ __forceinline__ int sp_tile_remap(int orig, int nwg) {
  // XCD-aware bijective remap (blocks b and b + 8 share an XCD): each XCD gets a contiguous range
  // of tiles, so the tiles sharing an A row-panel share its L2
  if (nwg < 16) return orig;
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// Per-lane DMA source offsets (bytes, relative to a plane base, k0 = 0) of the PPW 1-KiB pieces
// wave w stages per plane (pieces PPW w + i of the 8 that make a plane tile):
//   k-contig: a piece = 16 rows; lane L -> row 16 s + L / 4, physical chunk L & 3
//   k-major : a piece = 4 k-rows; lane L -> k-row 4 s + L / 16, physical chunk L & 15
// (the logical chunk is the physical one XOR the swizzle).
template <bool KMAJ, int PPW>
__device__ __forceinline__ void sp_voffs(long ld, int r0, int rlim, int w, int lane, uint32_t (&vo)[PPW]) {
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int s = PPW * w + i;
    if (!KMAJ) {
      const int row = 16 * s + (lane >> 2);
      const int c = (lane & 3) ^ ((row >> 2) & 3);
      vo[i] = (r0 + row < rlim) ? (uint32_t)(((long)(r0 + row) * ld + 8 * c) * 2) : SP_OOB;
    } else {
      const int kr = 4 * s + (lane >> 4);
      const int col = r0 + 8 * ((lane & 15) ^ sp_swz(kr));
      vo[i] = (col < rlim) ? (uint32_t)(((long)kr * ld + col) * 2) : SP_OOB;
    }
  }
}

// The three bf16x8 fragments of a 32-row block (rows c0 + (lane & 31), k = 16 b + 8 (lane >> 5) + e)
template <bool KMAJ>
__device__ __forceinline__ Split3 sp_frag(const unsigned short* __restrict__ op, int c0, int b, int lane) {
  Split3 r;
  if (!KMAJ) {
    const int o = sp_off(c0 + (lane & 31), 16 * b + 8 * (lane >> 5));
    r.h = *(const bf16x8_t*)(op + o);
    r.m = *(const bf16x8_t*)(op + SP_PL + o);
    r.l = *(const bf16x8_t*)(op + 2 * SP_PL + o);
  } else {
    // ds_read_b64_tr_b16 per 16-lane group g: lane 4q + p addresses k-row q of a 4 x 16 block
    // (columns 4p .. 4p + 3), lane i receives column i; group g covers columns c0 + 16 (g & 1) + i
    // and k-half g >> 1; two reads give k = 16 b + 8 h + 0..3 and + 4..7.
    const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4;
    const int col = c0 + 16 * (g & 1) + 4 * p;
    const int kb = 16 * b + 8 * (g >> 1) + q;
    const int o0 = sp_koff(kb, col), o1 = sp_koff(kb + 4, col);
    bf16x8_t* outs[3] = {&r.h, &r.m, &r.l};
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
      const unsigned short* base = op + pl * SP_PL;
      const sp_s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) sp_s16x4_t*)(base + o0));
      const sp_s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) sp_s16x4_t*)(base + o1));
      *outs[pl] = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
    }
  }
  return r;
}

// f32 value -> its three bf16 slices, stored as 4-element groups (8 B per plane)
__device__ __forceinline__ void sp_store4(unsigned short* p, long pps, const float (&v)[4]) {
  uint32_t h0, m0, l0, h1, m1, l1;
  split3_pair(v[0], v[1], h0, m0, l0);
  split3_pair(v[2], v[3], h1, m1, l1);
  *(uint2*)p = make_uint2(h0, h1);
  *(uint2*)(p + pps) = make_uint2(m0, m1);
  *(uint2*)(p + 2 * pps) = make_uint2(l0, l1);
}
__device__ __forceinline__ void sp_store1(unsigned short* p, long pps, float x) {
  const unsigned short h = f2bf(x);
  const float r = x - bf2f(h);
  const unsigned short m = f2bf(r);
  p[0] = h;
  p[pps] = m;
  p[2 * pps] = f2bf(r - bf2f(m));
}

// Epilogue, second half: the staged fp32 tile ep [TM][SP_EPI_PITCH] -> bias / activation / dropout /
// residual / relu'-mask / accumulate -> fp32 C and / or split planes P; thread t owns 4 columns
// of rows (t >> 5) + (NT / 32) q (float4 operand loads, 16-B stores of whole row segments).
template <int TM, int NT, int EPI, int OUT>
__device__ __forceinline__ void sp_store_tile(const GemmSpArgs& g, const float* ep, int m0, int n0) {
  const int tid = threadIdx.x;
  const int c4 = (tid & 31) * 4, col = n0 + c4;
  const bool hasC = (OUT & SO_C) && g.C;
  const bool vec = ((g.ldc | ((EPI & SE_RESID) ? g.ldr : 0) | ((EPI & SE_DACT) ? g.ldy : 0) |
                     ((OUT & SO_P) ? g.ldp : 0)) & 3) == 0;
  const bool full_cols = vec && col + 3 < g.N;
  const uint32_t seed = (EPI & SE_DROP) ? smi_seed(g.seedp, g.salt) : 0u;
  float bb[4] = {0.f, 0.f, 0.f, 0.f};
  if (EPI & SE_BIAS) {
    if (full_cols) {
      const float4 t = *(const float4*)(g.bias + col);
      bb[0] = t.x; bb[1] = t.y; bb[2] = t.z; bb[3] = t.w;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (col + e < g.N) bb[e] = g.bias[col + e];
    }
  }
  constexpr int RS = NT / 32;  // rows between a thread's consecutive rows
#pragma unroll 4
  for (int q = 0; q < TM / RS; ++q) {
    const int rl = (tid >> 5) + RS * q, row = m0 + rl;
    if (row >= g.M) continue;  // uniform over the 32 lanes that share the row
    if (col >= g.N) continue;
    const float4 t = *(const float4*)(ep + rl * SP_EPI_PITCH + c4);
    float v[4] = {t.x, t.y, t.z, t.w};
    const long cidx = (long)row * g.ldc + col;
    if (full_cols) {
      float4 rs = make_float4(0.f, 0.f, 0.f, 0.f), dy = rs, cc = rs;
      if (EPI & SE_RESID) rs = *(const float4*)(g.resid + (long)row * g.ldr + col);
      if (EPI & SE_DACT) dy = *(const float4*)(g.dact_y + (long)row * g.ldy + col);
      if ((EPI & SE_ACC) && hasC) cc = *(const float4*)(g.C + cidx);
      const unsigned mk = (EPI & SE_DMASK) ? g.mask[(long)row * g.ldm + (col >> 2)] : 0u;
      const float rv[4] = {rs.x, rs.y, rs.z, rs.w}, dv[4] = {dy.x, dy.y, dy.z, dy.w}, cv[4] = {cc.x, cc.y, cc.z, cc.w};
      unsigned bits = 0u;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = v[e] + bb[e];
        if (EPI & SE_RELU) x = fmaxf(x, 0.f);
        if (EPI & SE_DROP) x = smi_keep(seed, (uint32_t)(cidx + e), g.thresh) ? x * g.dscale : 0.f;
        if (EPI & SE_RESID) x += rv[e];
        if (EPI & SE_DACT) x = dv[e] > 0.f ? x * g.dscale : 0.f;
        if (EPI & SE_DMASK) x = ((mk >> e) & 1u) ? x * g.dscale : 0.f;
        if (EPI & SE_ACC) x += cv[e];
        bits |= (x > 0.f ? 1u : 0u) << e;
        v[e] = x;
      }
      if (hasC) *(float4*)(g.C + cidx) = make_float4(v[0], v[1], v[2], v[3]);
      if (OUT & SO_P) sp_store4(g.P + (long)row * g.ldp + col, g.pps, v);
      if (OUT & SO_M) g.mask[(long)row * g.ldm + (col >> 2)] = (unsigned char)bits;
    } else {
      const unsigned mk = (EPI & SE_DMASK) ? g.mask[(long)row * g.ldm + (col >> 2)] : 0u;
      unsigned bits = 0u;
      for (int e = 0; e < 4 && col + e < g.N; ++e) {
        float x = v[e] + bb[e];
        if (EPI & SE_RELU) x = fmaxf(x, 0.f);
        if (EPI & SE_DROP) x = smi_keep(seed, (uint32_t)(cidx + e), g.thresh) ? x * g.dscale : 0.f;
        if (EPI & SE_RESID) x += g.resid[(long)row * g.ldr + col + e];
        if (EPI & SE_DACT) x = g.dact_y[(long)row * g.ldy + col + e] > 0.f ? x * g.dscale : 0.f;
        if (EPI & SE_DMASK) x = ((mk >> e) & 1u) ? x * g.dscale : 0.f;
        if ((EPI & SE_ACC) && hasC) x += g.C[cidx + e];
        if (hasC) g.C[cidx + e] = x;
        if (OUT & SO_P) sp_store1(g.P + (long)row * g.ldp + col + e, g.pps, x);
        bits |= (x > 0.f ? 1u : 0u) << e;
        v[e] = x;
      }
      if (OUT & SO_M) g.mask[(long)row * g.ldm + (col >> 2)] = (unsigned char)bits;
    }
  }
}

// Bias-gradient row sums of a tile's A fragments (WGRAD, dY^T 1) on v_mfma_f32_16x16x32_bf16.
// Read as a 16x16x32 A operand, a 32x32x16 fragment (lane l: row l & 31, k-half l >> 5) puts
// tile rows r and r + 16 in different k-groups (vk = l >> 4: row vr + 16 (vk & 1), k-half
// vk >> 1), so ONE MFMA against a selector fragment that is 1.0 in column 0 for even k-groups and
// in column 1 for odd ones sums rows 0..15 into column 0 and rows 16..31 into column 1 — all 32
// row sums in 4 accumulator registers.  The hi plane uses columns 0 / 1, mid + lo columns 2 / 3:
// two exact fp32 chains (one rounding per 16 k each), added once at the end.
template <int NI = 2>
struct SpBiasSum {
  f32x4_t c[NI];         // per 32-row fragment i
  bf16x8_t sel_hi, sel_ml;
  __device__ __forceinline__ void init(int lane) {
    const int vk = (lane >> 4) & 1, col = lane & 15;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sel_hi[e] = col == vk ? (short)0x3F80 : (short)0;       // bf16 1.0
      sel_ml[e] = col == 2 + vk ? (short)0x3F80 : (short)0;
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) c[i] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  }
  __device__ __forceinline__ void add(int i, const Split3& f) {
    c[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.l, sel_ml, c[i], 0, 0, 0);
    c[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.m, sel_ml, c[i], 0, 0, 0);
    c[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.h, sel_hi, c[i], 0, 0, 0);
  }
  // lanes with column 0 / 1 own tile rows 16 col + 4 (lane >> 4) + r of fragment i (r = 0..3);
  // their mid + lo chain sits two lanes up (columns 2 / 3)
  __device__ __forceinline__ void store(const GemmSpArgs& g, int row0, int lane, bool accumulate) {
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float ml = __shfl_down(c[i][r], 2, 64);
        const int col = lane & 15;
        const int row = row0 + i * 32 + 16 * col + 4 * (lane >> 4) + r;
        if (col < 2 && row < g.M) {
          const float v = c[i][r] + ml;
          g.bias_grad[row] = accumulate ? g.bias_grad[row] + v : v;
        }
      }
  }
};

// One 128 x 128 output tile: the whole k-loop and the fused epilogue.  BIASG: this workgroup also
// reduces the bias gradient (WGRAD, column block 0; a separate instance keeps the k-loop one
// basic block for the MFMA / LDS-read / DMA interleave).
//
// Accumulation: hi.hi in its own fp32 accumulator (the rounding sequence of a plain fp32 chain,
// one rounding per 16 k), the five correction products (lo.hi, mid.mid, hi.lo, mid.hi, hi.mid) in
// a second one added at the end.  Measured: ONE accumulator for all six (six roundings per 16 k)
// let the 8192-token weight-gradient reduction drift to 1.7x the f32-MFMA kernel's error.
template <int NW, bool AK, bool BKM, int EPI, int OUT, bool BIASG = false>
__device__ __forceinline__ void gemm_sp_tile(const GemmSpArgs& g, int tile, unsigned short* lds) {
  using CF = SpCfg<NW>;
  constexpr int PPW = CF::PPW, WJ = CF::WJ, NT = CF::NT;
  SP_STAMP(0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / CF::WGN, wn = w % CF::WGN, h = lane >> 5;
  const int ntn = (g.N + 127) / 128;
  const int m0 = (tile / ntn) * 128, n0 = (tile % ntn) * 128;
  const int nk = (g.K + SP_BK - 1) / SP_BK;
  __amdgpu_buffer_rsrc_t ra[3], rb[3];
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    ra[p] = __builtin_amdgcn_make_buffer_rsrc((void*)(g.A + p * g.aps), 0, g.a_bytes, 0x00020000);
    rb[p] = __builtin_amdgcn_make_buffer_rsrc((void*)(g.B + p * g.bps), 0, g.b_bytes, 0x00020000);
  }
  uint32_t va[PPW], vb[PPW];
  sp_voffs<AK, PPW>(g.lda, m0, g.M, w, lane, va);
  sp_voffs<BKM, PPW>(g.ldb, n0, g.N, w, lane, vb);
  f32x16_t acc[2][WJ], cacc[2][WJ];
  SpBiasSum<> bsum;
  if constexpr (BIASG) bsum.init(lane);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < WJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = cacc[i][j][r] = 0.f;
  }
  // k-steps run in pairs with no exit between the halves; k-steps >= nk (the odd tail and the
  // look-ahead past the end) stage ZEROS: their soffset is pushed past every extent
  const int nk2 = (nk + 1) & ~1;
  auto issue = [&](int kt, int slot) {
#ifdef SP_PROBE_NODMA
    if (kt >= 3) return;  // diagnostic: the loop without its DMA (stale stages)
#endif
    unsigned short* st = lds + slot * SP_ST;
    const bool real = kt < nk;
    const int k0 = kt * SP_BK;
    const uint32_t sa = real ? (AK ? (uint32_t)((long)k0 * g.lda * 2) : (uint32_t)(k0 * 2)) : SP_OOB;
    const uint32_t sb = real ? (BKM ? (uint32_t)((long)k0 * g.ldb * 2) : (uint32_t)(k0 * 2)) : SP_OOB;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int i = 0; i < PPW; ++i) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra[p], (sp_lds_void*)(st + p * SP_PL + (PPW * w + i) * 512), 16, va[i],
                                                 sa, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb[p], (sp_lds_void*)(st + SP_OP + p * SP_PL + (PPW * w + i) * 512),
                                                 16, vb[i], sb, 0, 0);
      }
  };
  auto read = [&](int slot, Split3 (&fa)[2][2], Split3 (&fb)[2][WJ]) {
#ifdef SP_PROBE_NOREAD
    if (slot >= 0) return;  // diagnostic: MFMAs on stale fragments
#endif
    const unsigned short* st = lds + slot * SP_ST;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[b][i] = sp_frag<AK>(st, wm * 64 + i * 32, b, lane);
#pragma unroll
      for (int j = 0; j < WJ; ++j) fb[b][j] = sp_frag<BKM>(st + SP_OP, wn * CF::WCOL + j * 32, b, lane);
    }
  };
  auto mma = [&](const Split3 (&fa)[2][2], const Split3 (&fb)[2][WJ]) {
#if defined(SP_PROBE_NOMFMA)
    acc[0][0][0] += (float)fa[0][0].h[0] + (float)fb[1][WJ - 1].l[7];  // diagnostic: reads kept live
    return;
#endif
#pragma unroll
    for (int b = 0; b < 2; ++b) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < WJ; ++j) {
          acc[i][j] = MF32X16(fa[b][i].h, fb[b][j].h, acc[i][j]);
          cacc[i][j] = MF32X16(fa[b][i].l, fb[b][j].h, cacc[i][j]);
          cacc[i][j] = MF32X16(fa[b][i].m, fb[b][j].m, cacc[i][j]);
          cacc[i][j] = MF32X16(fa[b][i].h, fb[b][j].l, cacc[i][j]);
          cacc[i][j] = MF32X16(fa[b][i].m, fb[b][j].h, cacc[i][j]);
          cacc[i][j] = MF32X16(fa[b][i].h, fb[b][j].m, cacc[i][j]);
        }
      if constexpr (BIASG) {
#pragma unroll
        for (int i = 0; i < 2; ++i) bsum.add(i, fa[b][i]);
      }
    }
  };
  // One k-step: the fragments of stage kt are in registers (read during the previous step).
  // Wait until this wave's fragment reads and its DMA pieces of stage kt + 1 are done (stage
  // kt + 2's may still fly), barrier (every wave's pieces landed, every wave's reads of stage kt
  // retired), then: read stage kt + 1 into the other fragment set, refill stage kt's slot with
  // k-step kt + 3, and run stage kt's MFMAs — reads and DMA issues interleaved between them.
  constexpr int NRD = 2 * (2 * (AK ? 6 : 3) + WJ * (BKM ? 6 : 3));  // LDS fragment reads per k-step
  constexpr int NMF = 2 * (2 * WJ * 6 + (BIASG ? 6 : 0));            // MFMAs per k-step (incl. bias)
  constexpr int NDMA = CF::NDMA;
  Split3 f0a[2][2], f0b[2][WJ], f1a[2][2], f1b[2][WJ];
  issue(0, 0);
  issue(1, 1);
  issue(2, 2);
  if constexpr (NDMA == 6) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  SP_STAMP(1);
  read(0, f0a, f0b);
  int slot = 0;
  for (int kt = 0; kt < nk2; kt += 2) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if constexpr (NDMA == 6) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      const int nxt = slot == SP_NS - 1 ? 0 : slot + 1;
      if (half == 0) read(nxt, f1a, f1b);
      else read(nxt, f0a, f0b);
      issue(kt + half + 3, slot);
      if (half == 0) mma(f0a, f0b);
      else mma(f1a, f1b);
#ifndef SP_SCHED
#define SP_SCHED 1
#endif
      if constexpr (SP_SCHED == 1) {
        // fragment reads spread over the first MFMAs, the DMA issues after them
        constexpr int RPM = NRD <= NMF / 2 ? 1 : 2;  // reads per MFMA slot
#pragma unroll
        for (int i = 0; i < NRD / RPM; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);    // MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, RPM, 0);  // DS read
        }
#pragma unroll
        for (int i = 0; i < NDMA; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM (LDS-DMA)
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NMF, 0);
      } else if constexpr (SP_SCHED == 2) {
        // DMA issues first (one per MFMA), then the fragment reads
#pragma unroll
        for (int i = 0; i < NDMA; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
        constexpr int RPM = NRD <= (NMF - NDMA) / 2 ? 1 : 2;
#pragma unroll
        for (int i = 0; i < NRD / RPM; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, RPM, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NMF, 0);
      } else if constexpr (SP_SCHED == 3) {
        // DMA issues spread evenly: every (NMF / NDMA) MFMAs one DMA, reads in between
        constexpr int GAP = NMF / NDMA;
        constexpr int RPG = (NRD + NDMA - 1) / NDMA;  // reads per DMA group
#pragma unroll
        for (int i = 0; i < NDMA; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
#pragma unroll
          for (int j = 0; j < GAP; ++j) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            if (j < RPG) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          }
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NMF, 0);
      }
      // SP_SCHED == 0: the compiler's own order
      slot = nxt;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the zero look-ahead stages before LDS reuse
  SP_STAMP(2);

  // ---- epilogue: accumulators -> LDS [128][132] -> each thread owns 4 columns of 128/(NT/32) rows ----
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < WJ; ++j) acc[i][j] += cacc[i][j];
  __syncthreads();  // every wave is done reading the k-loop's stages
  float* ep = (float*)lds;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < WJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        ep[(wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * SP_EPI_PITCH + wn * CF::WCOL + j * 32 + (lane & 31)] =
            acc[i][j][r];
  __syncthreads();
  SP_STAMP(3);
  sp_store_tile<128, NT, EPI, OUT>(g, ep, m0, n0);
  SP_STAMP(4);
  if constexpr (BIASG) {
    if (wn == 0) bsum.store(g, m0 + wm * 64, lane, (EPI & SE_ACC) != 0);
  }
}

// 256 x 128 output tile (the N >= 1024 shapes and the weight gradients): 8 waves (4 x 2, each
// 64 x 64, two per SIMD), two 72 KiB stages.  Per 32-deep k-step a CU issues 384 MFMAs against
// 72 KiB of staged planes — a quarter fewer bytes and a third fewer LDS fragment reads per MFMA
// than the 128 x 128 tile, whose k-loop measured 1.3 us per k-step against 0.8 us for its MFMAs
// alone and 0.8 us for its DMA + LDS reads alone (tools/probes/sp_probe.hip).  Registers allow one
// fragment set: the stage a k-step reads is refilled (k-step kt + 2) after a second barrier
// that follows this step's fragment reads.
#define SP_ST256 (3 * (256 + 128) * SP_BK)  // bf16 per stage: A 3 x 256 x 32, B 3 x 128 x 32
template <bool AK, bool BKM, int EPI, int OUT, bool BIASG = false>
__device__ __forceinline__ void gemm_sp_tile256(const GemmSpArgs& g, int tile, unsigned short* lds) {
  constexpr int NT = 512, WJ = 2;
  constexpr int AOP = 3 * 256 * SP_BK;  // A planes of a stage (plane p at p * 8192)
  constexpr int APL = 256 * SP_BK;
  SP_STAMP(0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1, h = lane >> 5;
  const int ntn = (g.N + 127) / 128;
  const int m0 = (tile / ntn) * 256, n0 = (tile % ntn) * 128;
  const int nk = (g.K + SP_BK - 1) / SP_BK;
  __amdgpu_buffer_rsrc_t ra[3], rb[3];
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    ra[p] = __builtin_amdgcn_make_buffer_rsrc((void*)(g.A + p * g.aps), 0, g.a_bytes, 0x00020000);
    rb[p] = __builtin_amdgcn_make_buffer_rsrc((void*)(g.B + p * g.bps), 0, g.b_bytes, 0x00020000);
  }
  // A: 16 pieces per plane (pieces 2w, 2w + 1; k-major: 2 sub-images of [32 k][128 cols]);
  // B: 8 pieces per plane (piece w)
  uint32_t va[2], vb[1];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int s = 2 * w + i;
    if (!AK) {
      const int row = 16 * s + (lane >> 2);
      const int c = (lane & 3) ^ ((row >> 2) & 3);
      va[i] = (m0 + row < g.M) ? (uint32_t)(((long)(m0 + row) * g.lda + 8 * c) * 2) : SP_OOB;
    } else {
      const int sub = s >> 3, kr = 4 * (s & 7) + (lane >> 4);
      const int col = m0 + 128 * sub + 8 * ((lane & 15) ^ sp_swz(kr));
      va[i] = (col < g.M) ? (uint32_t)(((long)kr * g.lda + col) * 2) : SP_OOB;
    }
  }
  sp_voffs<BKM, 1>(g.ldb, n0, g.N, w, lane, vb);
  f32x16_t acc[2][WJ], cacc[2][WJ];
  SpBiasSum<> bsum;
  if constexpr (BIASG) bsum.init(lane);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < WJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = cacc[i][j][r] = 0.f;
  auto issue = [&](int kt, int slot) {
    unsigned short* st = lds + slot * SP_ST256;
    const bool real = kt < nk;
    const int k0 = kt * SP_BK;
    const uint32_t sa = real ? (AK ? (uint32_t)((long)k0 * g.lda * 2) : (uint32_t)(k0 * 2)) : SP_OOB;
    const uint32_t sb = real ? (BKM ? (uint32_t)((long)k0 * g.ldb * 2) : (uint32_t)(k0 * 2)) : SP_OOB;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra[p], (sp_lds_void*)(st + p * APL + (2 * w + i) * 512), 16, va[i],
                                                 sa, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb[p], (sp_lds_void*)(st + AOP + p * SP_PL + w * 512), 16, vb[0], sb,
                                               0, 0);
    }
  };
  // A fragment of tile rows c0 .. c0 + 31: k-contig image [256][32]; k-major: sub-image c0 / 128
  auto frag_a = [&](const unsigned short* st, int c0, int b) -> Split3 {
    if (!AK) {
      const int o = sp_off(c0 + (lane & 31), 16 * b + 8 * (lane >> 5));
      Split3 r;
      r.h = *(const bf16x8_t*)(st + o);
      r.m = *(const bf16x8_t*)(st + APL + o);
      r.l = *(const bf16x8_t*)(st + 2 * APL + o);
      return r;
    } else {
      // the k-major reader addresses planes SP_PL apart; each plane's sub-image c0 / 128 holds
      // the fragment: read the three planes through three sub-image bases
      const unsigned short* base = st + (c0 >> 7) * SP_PL;
      const int cc = c0 & 127;
      Split3 r;
      const int i = lane & 15, q = i >> 2, p = i & 3, g2 = lane >> 4;
      const int col = cc + 16 * (g2 & 1) + 4 * p;
      const int kb = 16 * b + 8 * (g2 >> 1) + q;
      const int o0 = sp_koff(kb, col), o1 = sp_koff(kb + 4, col);
      bf16x8_t* outs[3] = {&r.h, &r.m, &r.l};
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
        const unsigned short* pb = base + pl * APL;
        const sp_s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) sp_s16x4_t*)(pb + o0));
        const sp_s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) sp_s16x4_t*)(pb + o1));
        *outs[pl] = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
      }
      return r;
    }
  };
  issue(0, 0);
  issue(1, 1);
  for (int kt = 0; kt < nk; ++kt) {
    const int slot = kt & 1;
    asm volatile("s_waitcnt vmcnt(9)" ::: "memory");  // this wave's pieces of stage kt landed
    __builtin_amdgcn_s_barrier();
    const unsigned short* st = lds + slot * SP_ST256;
    Split3 fa[2][2], fb[2][WJ];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[b][i] = frag_a(st, wm * 64 + i * 32, b);
#pragma unroll
      for (int j = 0; j < WJ; ++j) fb[b][j] = sp_frag<BKM>(st + AOP, wn * 64 + j * 32, b, lane);
    }
    // every wave's reads of this stage retired -> refill it with k-step kt + 2
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue(kt + 2, slot);
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < WJ; ++j) {
          acc[i][j] = MF32X16(fa[b][i].h, fb[b][j].h, acc[i][j]);
          cacc[i][j] = MF32X16(fa[b][i].l, fb[b][j].h, cacc[i][j]);
          cacc[i][j] = MF32X16(fa[b][i].m, fb[b][j].m, cacc[i][j]);
          cacc[i][j] = MF32X16(fa[b][i].h, fb[b][j].l, cacc[i][j]);
          cacc[i][j] = MF32X16(fa[b][i].m, fb[b][j].h, cacc[i][j]);
          cacc[i][j] = MF32X16(fa[b][i].h, fb[b][j].m, cacc[i][j]);
        }
    if constexpr (BIASG) {
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 2; ++i) bsum.add(i, fa[b][i]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the zero look-ahead stages before LDS reuse
  SP_STAMP(2);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < WJ; ++j) acc[i][j] += cacc[i][j];
  __syncthreads();
  float* ep = (float*)lds;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < WJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        ep[(wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * SP_EPI_PITCH + wn * 64 + j * 32 + (lane & 31)] =
            acc[i][j][r];
  __syncthreads();
  SP_STAMP(3);
  sp_store_tile<256, NT, EPI, OUT>(g, ep, m0, n0);
  SP_STAMP(4);
  if constexpr (BIASG) {
    if (wn == 0) bsum.store(g, m0 + wm * 64, lane, (EPI & SE_ACC) != 0);
  }
}

template <int NW, bool AK, bool BKM, int EPI, int OUT>
__global__ __launch_bounds__(64 * NW, 1) void gemm_sp_kernel(GemmSpArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned short lds[SP_NS * SP_ST];
  const int nwg = ((g.M + 127) / 128) * ((g.N + 127) / 128);
  const int tile = sp_tile_remap(blockIdx.x, nwg);
  if constexpr (AK) {
    if (g.bias_grad && tile % ((g.N + 127) / 128) == 0) {
      gemm_sp_tile<NW, AK, BKM, EPI, OUT, true>(g, tile, lds);
      return;
    }
  }
  gemm_sp_tile<NW, AK, BKM, EPI, OUT, false>(g, tile, lds);
}

template <bool AK, bool BKM, int EPI, int OUT>
__global__ __launch_bounds__(512, 1) void gemm_sp256_kernel(GemmSpArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned short lds[2 * SP_ST256];
  const int nwg = ((g.M + 255) / 256) * ((g.N + 127) / 128);
  gemm_sp_tile256<AK, BKM, EPI, OUT>(g, sp_tile_remap(blockIdx.x, nwg), lds);
}


// ---------------------------------------------------------------------------------------------
// The 256 x 128 tile on v_mfma_f32_16x16x32_bf16 (gemm_sp_tm 16, the default).  Same stages, DMA, LDS bytes,
// MFMA cycles per FLOP and registers as gemm_sp_tile256 (a wave's 64 x 64 = 4 x 4 accumulators of
// 16 x 16; one k-step = one MFMA of k 32 per product), but the chip holds a higher clock on the
// 16 x 16 shape under load (docs: MI355X_MICROARCH "DVFS give-back" item 7: ~1.15x FLOP/s on
// random data).  Fragments: lane l holds row (col) l & 15 at k 8 (l >> 4) .. + 7.  k-contig images
// swizzle 16-B chunks by S[(row >> 2) & 3], S = {0, 2, 3, 1}: the four 16-lane groups of a
// ds_read_b128 ({0-3,12-15,20-27}, ...) then hit 16 distinct (row % 4, chunk) bank sets; the
// k-major images keep sp_koff (the two 32-lane groups of ds_read_b64_tr_b16 read k-rows
// {0-3, 8-11} / {16-19, 24-27}: 16 distinct physical chunks each).
__device__ __forceinline__ int sp16_swz(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }
__device__ __forceinline__ int sp16_off(int row, int k) {  // k % 8 == 0; [rows][32] image
  return row * 32 + ((((k >> 3) ^ sp16_swz(row)) & 3) << 3);
}

// the three bf16x8 plane fragments (h, m, l) of a 16-row (k-contig) / 16-column (k-major) block, k 0..31
template <bool KMAJ>
__device__ __forceinline__ Split3 sp16_frag(const unsigned short* __restrict__ img, int pl_stride, int c0, int lane) {
  Split3 r;
  if (!KMAJ) {
    const int o = sp16_off(c0 + (lane & 15), 8 * (lane >> 4));
    r.h = *(const bf16x8_t*)(img + o);
    r.m = *(const bf16x8_t*)(img + pl_stride + o);
    r.l = *(const bf16x8_t*)(img + 2 * pl_stride + o);
  } else {
    const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4;
    const int col = c0 + 4 * p;
    const int o0 = sp_koff(8 * g + q, col), o1 = sp_koff(8 * g + 4 + q, col);
    bf16x8_t* outs[3] = {&r.h, &r.m, &r.l};
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
      const unsigned short* base = img + pl * pl_stride;
      const sp_s16x4_t v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) sp_s16x4_t*)(base + o0));
      const sp_s16x4_t v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) sp_s16x4_t*)(base + o1));
      *outs[pl] = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
    }
  }
  return r;
}

// bias row sums of 16-row A fragments: one 16x16x32 MFMA against a fragment that is 1.0 in column
// 0 (hi chain) / column 1 (mid + lo chain) gives all 16 row sums
template <int NI>
struct SpBiasSum16 {
  f32x4_t c[NI];
  bf16x8_t sel_hi, sel_ml;
  __device__ __forceinline__ void init(int lane) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sel_hi[e] = (lane & 15) == 0 ? (short)0x3F80 : (short)0;
      sel_ml[e] = (lane & 15) == 1 ? (short)0x3F80 : (short)0;
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) c[i] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  }
  __device__ __forceinline__ void add(int i, const Split3& f) {
    c[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.l, sel_ml, c[i], 0, 0, 0);
    c[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.m, sel_ml, c[i], 0, 0, 0);
    c[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.h, sel_hi, c[i], 0, 0, 0);
  }
  // lanes of column 0 own rows 4 (lane >> 4) + r of fragment i; the mid + lo chain is one lane up
  __device__ __forceinline__ void store(const GemmSpArgs& g, int row0, int lane, bool accumulate) {
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float ml = __shfl_down(c[i][r], 1, 64);
        const int row = row0 + i * 16 + 4 * (lane >> 4) + r;
        if ((lane & 15) == 0 && row < g.M) {
          const float v = c[i][r] + ml;
          g.bias_grad[row] = accumulate ? g.bias_grad[row] + v : v;
        }
      }
  }
};

#define MF16(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

// fp32 operands as hi / mid / lo planes, six slice products per 32-deep k-step.
template <bool AK, bool BKM, int EPI, int OUT, bool BIASG = false>
__device__ __forceinline__ void gemm_sp_tile256m(const GemmSpArgs& g, int tile, unsigned short* lds) {
  constexpr int NT = 512, NB = 4;  // 4 x 4 blocks of 16 x 16 per wave
  constexpr int AOP = 3 * 256 * SP_BK;
  constexpr int APL = 256 * SP_BK;
  constexpr int KSTEP = SP_BK;  // k per stage
  SP_STAMP(0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int ntn = (g.N + 127) / 128;
  const int m0 = (tile / ntn) * 256, n0 = (tile % ntn) * 128;
  const int nk = (g.K + KSTEP - 1) / KSTEP;
  __amdgpu_buffer_rsrc_t ra[3], rb[3];
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    ra[p] = __builtin_amdgcn_make_buffer_rsrc((void*)(g.A + p * g.aps), 0, g.a_bytes, 0x00020000);
    rb[p] = __builtin_amdgcn_make_buffer_rsrc((void*)(g.B + p * g.bps), 0, g.b_bytes, 0x00020000);
  }
  // A: 16 pieces per plane (pieces 2w, 2w + 1), B: 8 (piece w); k-contig pieces swizzled by sp16_swz
  uint32_t va[2], vb;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int s = 2 * w + i;
    if (!AK) {
      const int row = 16 * s + (lane >> 2);
      const int c = (lane & 3) ^ sp16_swz(row);
      va[i] = (m0 + row < g.M) ? (uint32_t)(((long)(m0 + row) * g.lda + 8 * c) * 2) : SP_OOB;
    } else {
      const int sub = s >> 3, kr = 4 * (s & 7) + (lane >> 4);
      const int col = m0 + 128 * sub + 8 * ((lane & 15) ^ sp_swz(kr));
      va[i] = (col < g.M) ? (uint32_t)(((long)kr * g.lda + col) * 2) : SP_OOB;
    }
  }
  if (!BKM) {
    const int row = 16 * w + (lane >> 2);
    const int c = (lane & 3) ^ sp16_swz(row);
    vb = (n0 + row < g.N) ? (uint32_t)(((long)(n0 + row) * g.ldb + 8 * c) * 2) : SP_OOB;
  } else {
    const int kr = 4 * w + (lane >> 4);
    const int col = n0 + 8 * ((lane & 15) ^ sp_swz(kr));
    vb = (col < g.N) ? (uint32_t)(((long)kr * g.ldb + col) * 2) : SP_OOB;
  }
  f32x4_t acc[NB][NB], cacc[NB][NB];
  SpBiasSum16<NB> bsum;
  if constexpr (BIASG) bsum.init(lane);
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = cacc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  auto issue = [&](int kt, int slot) {
    unsigned short* st = lds + slot * SP_ST256;
    const bool real = kt < nk;
    const int k0 = kt * KSTEP;
    const uint32_t sa = real ? (AK ? (uint32_t)((long)k0 * g.lda * 2) : (uint32_t)(k0 * 2)) : SP_OOB;
    const uint32_t sb = real ? (BKM ? (uint32_t)((long)k0 * g.ldb * 2) : (uint32_t)(k0 * 2)) : SP_OOB;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra[p], (sp_lds_void*)(st + p * APL + (2 * w + i) * 512), 16, va[i],
                                                 sa, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb[p], (sp_lds_void*)(st + AOP + p * SP_PL + w * 512), 16, vb, sb, 0,
                                               0);
    }
  };
  auto frag_a = [&](const unsigned short* st, int c0) -> Split3 {
    // k-major A: sub-image c0 / 128 of each plane ([32][128] images SP_PL apart inside the plane)
    return AK ? sp16_frag<true>(st + (c0 >> 7) * SP_PL, APL, c0 & 127, lane)
              : sp16_frag<false>(st, APL, c0, lane);
  };
  issue(0, 0);
  issue(1, 1);
  for (int kt = 0; kt < nk; ++kt) {
    const int slot = kt & 1;
    // this wave's pieces of stage kt landed (3 DMA instructions per plane and stage; stage kt + 1's
    // still in flight)
    asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const unsigned short* st = lds + slot * SP_ST256;
    Split3 fa[NB], fb[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) fa[i] = frag_a(st, wm * 64 + i * 16);
#pragma unroll
    for (int j = 0; j < NB; ++j) fb[j] = sp16_frag<BKM>(st + AOP, SP_PL, wn * 64 + j * 16, lane);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's reads of this stage retired -> refill it
    issue(kt + 2, slot);
    // product-major: consecutive MFMAs write different accumulators
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[i][j] = MF16(fa[i].h, fb[j].h, acc[i][j]);
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        cacc[i][j] = MF16(fa[i].l, fb[j].h, cacc[i][j]);
        cacc[i][j] = MF16(fa[i].m, fb[j].m, cacc[i][j]);
        cacc[i][j] = MF16(fa[i].h, fb[j].l, cacc[i][j]);
        cacc[i][j] = MF16(fa[i].m, fb[j].h, cacc[i][j]);
        cacc[i][j] = MF16(fa[i].h, fb[j].m, cacc[i][j]);
      }
    if constexpr (BIASG) {
#pragma unroll
      for (int i = 0; i < NB; ++i) bsum.add(i, fa[i]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  SP_STAMP(2);
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] += cacc[i][j];
  __syncthreads();
  float* ep = (float*)lds;
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        ep[(wm * 64 + i * 16 + 4 * (lane >> 4) + r) * SP_EPI_PITCH + wn * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
  __syncthreads();
  SP_STAMP(3);
  sp_store_tile<256, NT, EPI, OUT>(g, ep, m0, n0);
  SP_STAMP(4);
  if constexpr (BIASG) {
    if (wn == 0) bsum.store(g, m0 + wm * 64, lane, (EPI & SE_ACC) != 0);
  }
}

template <bool AK, bool BKM, int EPI, int OUT>
__global__ __launch_bounds__(512, 1) void gemm_sp256m_kernel(GemmSpArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned short lds[2 * SP_ST256];
  const int nwg = ((g.M + 255) / 256) * ((g.N + 127) / 128);
  gemm_sp_tile256m<AK, BKM, EPI, OUT>(g, sp_tile_remap(blockIdx.x, nwg), lds);
}

// waves per workgroup of the launches (SMI_SP_WAVES = 4 | 8; default 8)
int smi_sp_waves();
// 256-row tiles where they fill the chip: SMI_SP_TM = 16 (default: 8 waves on the 16x16x32 MFMA),
// 256 (8 waves, 32x32x16), 4 (4 waves, pipelined), 128 (128-row tiles only)
int smi_sp_tm();
// 256 x 128 tiles when they fill the chip and do not lose a partial wave against 128 x 128 tiles:
// (M, N) = (8192, 1536) is 384 tiles of 256 rows (1.5 waves of 256 CUs) but 768 of 128 rows
// (3 full waves) — measured 87 vs 78 us (profiles/r3_gemm_sp_tiles_bench.log).
static inline bool sp_use256(int M, int N) {
  if (smi_sp_tm() == 128) return false;
  const long t256 = (long)((M + 255) / 256) * ((N + 127) / 128);
  const long t128 = (long)((M + 127) / 128) * ((N + 127) / 128);
  if (t256 < SP_NUM_CU) return false;
  const long w256 = (t256 + SP_NUM_CU - 1) / SP_NUM_CU, w128 = (t128 + SP_NUM_CU - 1) / SP_NUM_CU;
  return 2 * w256 <= w128 || smi_sp_tm() == 256;
}

// Host-side checks shared by the launchers: 16-B aligned plane rows, descriptor-addressable
// extents (each plane has its own descriptor), chunk (8-element) granularity of each operand's
// contiguous dimension.  k-contig operand: [rows][K]; k-major operand: [K][cols].
static inline bool sp_operand_ok(const unsigned short* p, long ld, long ps, long rows, long cols, bool kmaj, int kpad,
                                 int K, int& bytes) {
  if (!p || ((uintptr_t)p & 15) || ld % 8 || ps % 8 || rows < 1 || cols < 1 || K < 1) return false;
  long ext;
  if (!kmaj) {  // K must be a multiple of 32 or the rows zero-padded to one
    const long kp = (K + 31) / 32 * 32;
    if (K % 32 && !(kpad && ld >= kp)) return false;
    if (ld < K) return false;
    ext = 2 * ((rows - 1) * ld + kp);
  } else {      // cols a multiple of 8 (16-B chunks)
    if (cols % 8 || ld < cols) return false;
    ext = 2 * ((long)(K - 1) * ld + cols);
  }
  if (ext >= (1L << 31)) return false;
  bytes = (int)ext;
  return true;
}
