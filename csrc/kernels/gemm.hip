// bf16 GEMM on MFMA (v_mfma_f32_16x16x32_bf16) with fused epilogues, for the three GEMMs of
// every linear layer of the reference models (transformer.py Linear layers, MLP/CNN heads):
//
//   FWD   C[M,N]  = X[M,K] . W[N,K]^T  (+bias, ReLU, dropout)        A k-contig, B k-contig
//   DGRAD dX[M,K] = dY[M,N] . W[N,K]   (+residual, x relu'/dropout)  A k-contig, B k-major
//   WGRAD dW[N,K] += dY[M,N]^T . X[M,K]  (fp32, split-K atomics)     A k-major,  B k-major
//
// CDNA4 structure: PERSISTENT workgroups (one per CU: 256 threads = 4 waves 2x2, 128x128
// output tile, BK = 64, four LDS stages = 128 KiB) walk a flattened stream of (tile, k-step)
// work items, so the DMA pipeline never drains between tiles: the next tile's first k-steps are
// in flight while the current tile's epilogue stores.  Tiles are staged by
// buffer_load_dwordx4 ... lds (LDS-DMA, no VGPR round trip; per-lane offsets computed once per
// tile, the k advance is a scalar soffset, out-of-range rows read as 0 through the descriptor's
// bounds) in the operand's NATURAL global layout —
// no transpose kernels: k-contiguous tiles are read with ds_read_b128 through an XOR chunk
// swizzle (c ^ (row&7): conflict-free for the 16x16x32 operand groups), k-major tiles with the
// gfx950 transposing read ds_read_b64_tr_b16 through a pair swizzle (conflict-free per 32-lane
// half).  Swizzles are applied to the per-lane SOURCE address of the DMA (LDS image stays
// lane-linear; cdna_hip_programming.md rule 21).  Up to three k-steps stay in flight across raw
// s_barriers with counted `s_waitcnt vmcnt(N)` waits (never 0 inside the loop).
// Tile order is XCD-aware (bijective remap: tiles sharing an A row-panel run on one XCD's L2).
// bf16/plain-fp32 epilogues use the operand-swapped MFMA so each lane owns 4 consecutive output
// columns (8-/16-byte stores); the split-K fp32 atomic epilogue keeps lanes along columns
// (64-byte row segments per atomic wave-instruction).  A ragged K (multiple of 8) is handled by
// zeroing the out-of-range A columns of the last k-tile in LDS.
#include "smi_common.h"
#include "smi_gemm.h"
#include <stdlib.h>

#define BM 128
#define BN 128
#define BKK 64
#ifndef GEMM_NS
#define GEMM_NS 2
#endif
#ifdef GEMM_PROBE_NOEPI
static constexpr bool kProbeNoEpi = true;
#else
static constexpr bool kProbeNoEpi = false;
#endif
#ifdef GEMM_STAMPS
// diagnostic build only (tools/probes/gemm_stamp_probe.hip): s_memrealtime (100 MHz) stamps of
// each workgroup's phases, written by lane 0 of wave 0 to a buffer no output depends on
__device__ unsigned long long* g_gemm_stamps;
#define GSTAMP(slot)                                                                       \
  do {                                                                                     \
    if (threadIdx.x == 0 && t == (int)blockIdx.x)                                          \
      g_gemm_stamps[(long)blockIdx.x * 8 + (slot)] = __builtin_amdgcn_s_memrealtime();      \
  } while (0)
#else
#define GSTAMP(slot) do {} while (0)
#endif
#define TILE_ELEMS (BM * BKK)  // 8192 bf16 = 16 KiB per operand per stage
#define NUM_CU 256

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(4))) short s16x4_t;

// LDS-DMA through a buffer descriptor: 32-bit per-lane voffset (fixed per tile), scalar soffset
// (the k advance), out-of-range records read as 0 — no per-step address VALU, no clamping.
__device__ __forceinline__ void bdma16(__amdgpu_buffer_rsrc_t rsrc, unsigned short* lds_base, uint32_t voff,
                                       uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)lds_base, 16, voff, soff, 0, 0);
}

// pair swizzle for k-major tiles (128 cols = 16 chunks of 8 bf16 per k-row)
__device__ __forceinline__ int kmaj_s(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

// Per-lane byte offsets (relative to the operand base, k0 = 0) of the NP DMA pieces this wave
// issues for one (32*NP) x 64 k-contig tile ([rows][64 k]) or a 64 x 128 k-major tile
// ([64 k][128 cols], NP = 4).  The XOR swizzle lives in these SOURCE offsets; the LDS image is
// lane-linear (each piece = one wave-instruction = 1 KiB).
template <bool KMAJ, int NP>
__device__ __forceinline__ void tile_voffsets(long ld, int r0, int w, int lane, uint32_t (&vo)[NP]) {
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int ins = w * NP + i;
    if (!KMAJ) {
      const int row = ins * 8 + (lane >> 3);
      const int lc = (lane & 7) ^ (row & 7);
      vo[i] = (uint32_t)(((long)(r0 + row) * ld + lc * 8) * 2);
    } else {
      const int row = ins * 4 + (lane >> 4);  // k row 0..63
      const int lc = (lane & 15) ^ (kmaj_s(row) << 1);
      vo[i] = (uint32_t)(((long)row * ld + r0 + lc * 8) * 2);
    }
  }
}

// Issue the NP DMA pieces of one tile at k0 (soffset = k0 * k-stride bytes).
template <bool KMAJ, int NP>
__device__ __forceinline__ void stage_tile(__amdgpu_buffer_rsrc_t rsrc, long ld, int k0, const uint32_t (&vo)[NP],
                                           unsigned short* tile, int w) {
#ifdef GEMM_PROBE_NODMA
  return;
#endif
  const uint32_t soff = KMAJ ? (uint32_t)((long)k0 * ld * 2) : (uint32_t)(k0 * 2);
#pragma unroll
  for (int i = 0; i < NP; ++i) bdma16(rsrc, tile + (w * NP + i) * 512, vo[i], soff);
}

// zero logical k-columns >= kvalid of a staged tile (ragged-K tail); `rows` rows for k-contig
template <bool KMAJ>
__device__ __forceinline__ void zero_ktail(unsigned short* tile, int kvalid, int tid, int rows) {
  if (!KMAJ) {
    for (int e = tid; e < rows * 8; e += 256) {
      const int row = e >> 3, c = e & 7;
      if (c * 8 >= kvalid) *(uint4*)(tile + row * 64 + ((c ^ (row & 7)) << 3)) = make_uint4(0, 0, 0, 0);
      else if (c * 8 + 8 > kvalid) {
        unsigned short* p = tile + row * 64 + ((c ^ (row & 7)) << 3);
        for (int j = kvalid - c * 8; j < 8; ++j) p[j] = 0;
      }
    }
  } else {
    for (int e = tid; e < 64 * 16; e += 256) {
      const int kr = e >> 4;
      if (kr >= kvalid) *(uint4*)(tile + kr * 128 + (e & 15) * 8) = make_uint4(0, 0, 0, 0);
    }
  }
}

// A/B fragment (8 bf16) for the 16-row sub-tile starting at tile-row/col `r0`, k-step ks (0/1)
template <bool KMAJ>
__device__ __forceinline__ bf16x8_t read_frag(const unsigned short* tile, int r0, int ks, int lane) {
  if (!KMAJ) {
    const int row = r0 + (lane & 15);
    const int c = ks * 4 + (lane >> 4);
    return *(const bf16x8_t*)(tile + row * 64 + ((c ^ (row & 7)) << 3));
  } else {
    const int q = (lane & 15) >> 2, p = lane & 3, g = lane >> 4;
    const int col = r0 + 4 * p;
    s16x4_t v[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kr = ks * 32 + 8 * g + 4 * h + q;
      const int c = col >> 3;
      const int pc = c ^ (kmaj_s(kr) << 1);
      const unsigned short* addr = tile + kr * 128 + pc * 8 + (col & 7);
      v[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)addr);
    }
    // concatenate as one vector op so the two 64-bit reads can land in adjacent registers
    // (element-wise assembly left ~60 v_mov per k-step in the weight-gradient loop)
    return __builtin_shufflevector(v[0], v[1], 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

// Epilogue feature set.  EPI >= 0: a compile-time bitmask (the kernel is specialised: no
// runtime tests, no speculatively computed dropout hash per element); EPI < 0: generic (runtime
// tests on the argument block).  Measured: the generic epilogue of a 64 x 128 tile issued ~1200
// instructions per wave (if-converted dropout hash and per-element flag selects) = 2-4 us per
// tile, a third of a K = 512 GEMM (tools/probes/gemm_stamp_probe.hip).
enum : int { EPI_BIAS = 1, EPI_RESID = 2, EPI_RELU = 4, EPI_DACT = 8, EPI_DROP = 16 };
struct EpiFlags {
  bool bias, resid, relu, dact, drop;
};
template <int EPI>
__device__ __forceinline__ EpiFlags epi_flags(const GemmArgs& g) {
  if constexpr (EPI < 0) return EpiFlags{g.bias != nullptr, g.resid != nullptr, g.act == 1, g.dact_y != nullptr, g.thresh != 0};
  else return EpiFlags{(EPI & EPI_BIAS) != 0, (EPI & EPI_RESID) != 0, (EPI & EPI_RELU) != 0, (EPI & EPI_DACT) != 0,
                       (EPI & EPI_DROP) != 0};
}

// epilogue value transform for bf16 outputs
__device__ __forceinline__ float epi_val(const GemmArgs& g, const EpiFlags& f, float v, float bia, int row, int col,
                                         long cidx, uint32_t seed) {
  v = v * g.alpha + bia;
  if (f.resid) v += bf2f(g.resid[(long)row * g.ldr + col]);
  if (f.relu) v = fmaxf(v, 0.f);
  if (f.dact) {  // backward of relu+dropout: y > 0 <=> kept and positive
    v = bf2f(g.dact_y[(long)row * g.ldy + col]) > 0.f ? v * g.dscale : 0.f;
  } else if (f.drop) {
    v = smi_keep(seed, (uint32_t)cidx, g.thresh) ? v * g.dscale : 0.f;
  }
  return v;
}

struct TileInfo {
  int m0, n0, kbeg, nk, split;
};

__device__ __forceinline__ TileInfo tile_of(const GemmArgs& g, int t, int ntn, int nwg, int bm) {
  // t enumerates (split, tile); XCD-aware bijective remap inside one split's tile set
  const int split = t / nwg;
  const int orig = t - split * nwg;
  int wgid = orig;
  if (nwg >= 16) {
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  }
  TileInfo ti;
  ti.m0 = (wgid / ntn) * bm;
  ti.n0 = (wgid % ntn) * BN;
  ti.split = split;
  ti.kbeg = split * g.k_per_split;
  const int kend = min(g.K, ti.kbeg + g.k_per_split);
  ti.nk = (kend - ti.kbeg + BKK - 1) / BKK;
  return ti;
}
// One output tile (all its k-steps and the epilogue) of the problem in `g`; t = the tile
// index within that problem's (split, tile) enumeration.  `smem` = the NS-stage LDS ring.
template <bool AK, bool BKM, bool SWAP, int NS, int FM, int EPI>
__device__ __forceinline__ void gemm_tile(const GemmArgs& g, const int t, unsigned short* smem) {
  constexpr int BMT = 32 * FM;                 // tile rows (M)
  constexpr int NPA = AK ? 4 : FM;             // DMA pieces per wave per stage, A operand
  constexpr int A_ELEMS = BMT * BKK;
  constexpr int STAGE = A_ELEMS + TILE_ELEMS;  // A then B (128 rows) per stage
  constexpr int VM1 = NPA + 4;                 // vector-memory ops per wave per stage
  static_assert(!AK || FM == 4, "k-major A needs 128-wide tiles");
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int ntn = (g.N + BN - 1) / BN;
  const int ntm = (g.M + BMT - 1) / BMT;
  const int nwg = ntm * ntn;
  const bool ragged = (g.K % BKK) != 0 || (g.K % g.k_per_split) != 0;
  const uint32_t seed = smi_seed(g.seedp, g.salt);
  const EpiFlags ef = epi_flags<EPI>(g);
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)g.A, 0, (int)g.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)g.B, 0, (int)g.b_bytes, 0x00020000);

    GSTAMP(0);
    const TileInfo ti = tile_of(g, t, ntn, nwg, BMT);
    const int m0 = ti.m0, n0 = ti.n0, nk = ti.nk;
    uint32_t voA[NPA], voB[4];
    tile_voffsets<AK, NPA>(g.lda, m0, w, lane, voA);
    tile_voffsets<BKM, 4>(g.ldb, n0, w, lane, voB);
    f32x4_t acc[FM][4];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    // fused bias gradient (WGRAD): the workgroups of the first output-column block multiply
    // their A fragments by a ones fragment — one extra MFMA per A fragment, no extra loads
    const bool do_bias = AK && g.bias_grad && n0 == 0 && wn == 0;
    f32x4_t accb[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) accb[i] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s0 = 0; s0 < NS - 1; ++s0) {
      if (s0 < nk) {
        unsigned short* st = smem + s0 * STAGE;
        stage_tile<AK, NPA>(rA, g.lda, ti.kbeg + s0 * BKK, voA, st, w);
        stage_tile<BKM, 4>(rB, g.ldb, ti.kbeg + s0 * BKK, voB, st + A_ELEMS, w);
      }
    }
    int rd = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const int ahead = min(NS - 2, nk - 1 - kt);  // items staged beyond kt
      if (NS >= 4 && ahead >= 2) {
        if (VM1 == 8) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      } else if (NS >= 3 && ahead >= 1) {
        if (VM1 == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      if (kt == 0) GSTAMP(1);
      if (kt == 1) GSTAMP(2);
      if (ragged) {
        const int kv = min(g.K, ti.kbeg + g.k_per_split) - (ti.kbeg + kt * BKK);
        if (kv < BKK) {
          zero_ktail<AK>(smem + rd * STAGE, kv, tid, BMT);
          __syncthreads();
        }
      }
      // Read BOTH k-substeps' fragments of this stage before issuing the next stage's DMA:
      // hipcc orders an LDS-DMA before any later ds_read_b64_tr_b16 builtin with vmcnt(0) (it
      // cannot prove they touch different stages), which made every DGRAD / WGRAD k-step wait
      // for the DMA it had just issued.  Reads first, DMA second, MFMAs last keeps the DMA of
      // step kt+NS-1 in flight under this step's MFMAs.
      const unsigned short* ta = smem + rd * STAGE;
      const unsigned short* tb = ta + A_ELEMS;
      bf16x8_t af[2][FM], bf[2][4];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int i = 0; i < FM; ++i) af[ks][i] = read_frag<AK>(ta, wm * 16 * FM + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) bf[ks][j] = read_frag<BKM>(tb, wn * 64 + j * 16, ks, lane);
      }
      if (kt + NS - 1 < nk) {
        int ws = rd + NS - 1;
        if (ws >= NS) ws -= NS;
        unsigned short* st = smem + ws * STAGE;
        stage_tile<AK, NPA>(rA, g.lda, ti.kbeg + (kt + NS - 1) * BKK, voA, st, w);
        stage_tile<BKM, 4>(rB, g.ldb, ti.kbeg + (kt + NS - 1) * BKK, voB, st + A_ELEMS, w);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
#ifdef GEMM_PROBE_NOMFMA
            acc[i][j][0] += (float)af[ks][i][0] + (float)bf[ks][j][0];
#else
            if (SWAP) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[ks][j], af[ks][i], acc[i][j], 0, 0, 0);
            else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bf[ks][j], acc[i][j], 0, 0, 0);
#endif
          }
        if (AK && do_bias) {
          bf16x8_t ones;
#pragma unroll
          for (int e = 0; e < 8; ++e) ones[e] = (short)0x3F80;  // bf16 1.0
#pragma unroll
          for (int i = 0; i < FM; ++i) {
            if (SWAP) accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, af[ks][i], accb[i], 0, 0, 0);
            else accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], ones, accb[i], 0, 0, 0);
          }
        }
      }
      rd = (rd + 1 == NS) ? 0 : rd + 1;
    }
    GSTAMP(3);
    // ---------------- epilogue (no DMA in flight) ----------------
#ifdef GEMM_PROBE_NOEPI
    {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
      if (t == 1234.5f) ((float*)g.C)[tid] = t;
    }
    if (false) {
#else
    const bool vec8 = (g.N % 8 == 0) && (g.ldc % 8 == 0) && (!ef.resid || g.ldr % 8 == 0) && (!ef.dact || g.ldy % 8 == 0);
    if (SWAP && !g.out_f32 && vec8) {
      // LDS-staged bf16 epilogue.  Each wave parks its 64x64 fp32 sub-tile in its own 16 KiB of the
      // (now idle) staging LDS — 16-B chunk c of row r at c ^ (r & 15), conflict-free for both
      // passes — then re-reads it row-wise so every lane owns 8 consecutive columns: residual /
      // mask operands are 16-B loads and each store instruction writes 8 full 128-B row segments
      // (the direct form wrote 32-B pieces of 16 rows).
      __syncthreads();  // every wave is done reading the k-loop's staging buffers
      GSTAMP(5);
      float* ep = (float*)smem + w * (FM * 16 * 64);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = i * 16 + (lane & 15), c = j * 4 + (lane >> 4);
          *(f32x4_t*)(ep + r * 64 + ((c ^ (r & 15)) << 2)) = acc[i][j];
        }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes are done
      GSTAMP(6);
      const int q = lane & 7;               // 8-column group of this lane
      const int col = n0 + wn * 64 + q * 8;
      float bb[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) bb[e] = 0.f;
      if (ef.bias && col < g.N) {
        const float4 b0 = *(const float4*)(g.bias + col), b1 = *(const float4*)(g.bias + col + 4);
        bb[0] = b0.x; bb[1] = b0.y; bb[2] = b0.z; bb[3] = b0.w; bb[4] = b1.x; bb[5] = b1.y; bb[6] = b1.z; bb[7] = b1.w;
      }
      // two passes: every load (LDS image, residual, mask source) and all the epilogue math
      // first, then all the stores — a load issued after a store would make the wave wait for
      // that store's completion (vmcnt counts both in issue order), serialising the tile's stores
      uint4 pk[2 * FM];
      bool ok[2 * FM];
#pragma unroll
      for (int it = 0; it < 2 * FM; ++it) {
        const int r = it * 8 + (lane >> 3);
        const int row = m0 + wm * 16 * FM + r;
        const f32x4_t lo = *(const f32x4_t*)(ep + r * 64 + (((2 * q) ^ (r & 15)) << 2));
        const f32x4_t hi = *(const f32x4_t*)(ep + r * 64 + (((2 * q + 1) ^ (r & 15)) << 2));
        ok[it] = row < g.M && col < g.N;
        const int rowc = ok[it] ? row : 0, colc = ok[it] ? col : 0;
        float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const long cidx = (long)rowc * g.ldc + colc;
        u16x8_t rs, dy;
        if (ef.resid) rs = *(const u16x8_t*)(g.resid + (long)rowc * g.ldr + colc);
        if (ef.dact) dy = *(const u16x8_t*)(g.dact_y + (long)rowc * g.ldy + colc);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float x = v[e] * g.alpha + bb[e];
          if (ef.resid) x += bf2f(rs[e]);
          if (ef.relu) x = fmaxf(x, 0.f);
          if (ef.dact) x = bf2f(dy[e]) > 0.f ? x * g.dscale : 0.f;
          else if (ef.drop) x = smi_keep(seed, (uint32_t)(cidx + e), g.thresh) ? x * g.dscale : 0.f;
          v[e] = x;
        }
        pk[it].x = pack2bf(v[0], v[1]); pk[it].y = pack2bf(v[2], v[3]);
        pk[it].z = pack2bf(v[4], v[5]); pk[it].w = pack2bf(v[6], v[7]);
      }
      GSTAMP(7);
#pragma unroll
      for (int it = 0; it < 2 * FM; ++it) {
        const int row = m0 + wm * 16 * FM + it * 8 + (lane >> 3);
#if defined(GEMM_PROBE_NOSTORE)
        if (ok[it] && pk[it].x == 0x12345678u) *(uint4*)((unsigned short*)g.C + (long)row * g.ldc + col) = pk[it];
#else
        if (ok[it]) *(uint4*)((unsigned short*)g.C + (long)row * g.ldc + col) = pk[it];
#endif
      }
    } else if (SWAP) {
#endif
      // acc[i][j][r] = C[m0 + wm*64 + i*16 + (lane&15)][n0 + wn*64 + j*16 + 4*(lane>>4) + r]
      const int cl = 4 * (lane >> 4);
      const bool interior = (m0 + BMT <= g.M) && (n0 + BN <= g.N);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + wn * 64 + j * 16 + cl;
        float4 bia = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ef.bias && (interior || col + 3 < g.N)) bia = *(const float4*)(g.bias + col);
        else if (ef.bias) {
          if (col < g.N) bia.x = g.bias[col];
          if (col + 1 < g.N) bia.y = g.bias[col + 1];
          if (col + 2 < g.N) bia.z = g.bias[col + 2];
        }
        const float bb[4] = {bia.x, bia.y, bia.z, bia.w};
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int row = m0 + wm * 16 * FM + i * 16 + (lane & 15);
          const long cidx = (long)row * g.ldc + col;
          if (g.out_f32) {
            float* C = (float*)g.C + cidx + (long)ti.split * g.c_split_stride;
            float4 v = make_float4(acc[i][j][0] * g.alpha, acc[i][j][1] * g.alpha, acc[i][j][2] * g.alpha,
                                   acc[i][j][3] * g.alpha);
            if (interior || (row < g.M && col + 3 < g.N)) {
              if (g.beta_acc) { float4 o = *(float4*)C; v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w; }
              *(float4*)C = v;
            } else if (row < g.M) {
              float vv[4] = {v.x, v.y, v.z, v.w};
              for (int r = 0; r < 4; ++r)
                if (col + r < g.N) C[r] = g.beta_acc ? C[r] + vv[r] : vv[r];
            }
          } else if (interior || (row < g.M && col + 3 < g.N)) {
            float o[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = epi_val(g, ef, acc[i][j][r], bb[r], row, col + r, cidx + r, seed);
            uint2 pk;
            pk.x = pack2bf(o[0], o[1]);
            pk.y = pack2bf(o[2], o[3]);
            *(uint2*)((unsigned short*)g.C + cidx) = pk;
          } else if (row < g.M) {
            for (int r = 0; r < 4; ++r)
              if (col + r < g.N)
                ((unsigned short*)g.C)[cidx + r] = f2bf(epi_val(g, ef, acc[i][j][r], bb[r], row, col + r, cidx + r, seed));
          }
        }
      }
    } else if (!kProbeNoEpi) {
      // acc[i][j][r] = C[m0 + wm*64 + i*16 + 4*(lane>>4) + r][n0 + wn*64 + j*16 + (lane&15)]
      const int cl = lane & 15, rg = (lane >> 4) * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + wn * 64 + j * 16 + cl;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = m0 + wm * 16 * FM + i * 16 + rg + r;
            if (row < g.M && col < g.N) {
              const long cidx = (long)row * g.ldc + col;
              float* C = (float*)g.C;
              const float v = acc[i][j][r] * g.alpha;
              if (g.atomic) atomicAdd(C + cidx, v);
              else C[cidx] = g.beta_acc ? C[cidx] + v : v;
            }
          }
        }
      }
    }
    if (AK && do_bias) {
      // SWAP: lane holds sum_k A[k][c] for c = i*16 + (lane & 15) in all four registers;
      // non-SWAP: lane holds rows 4*(lane>>4) + r of fragment i in register r
      float* bdst = g.bias_grad + (g.atomic ? 0 : (long)ti.split * g.bias_split_stride);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        if (SWAP) {
          const int row = m0 + wm * 16 * FM + i * 16 + (lane & 15);
          if ((lane >> 4) == 0 && row < g.M) {
            if (g.atomic) atomicAdd(bdst + row, accb[i][0]);
            else bdst[row] = g.beta_acc ? bdst[row] + accb[i][0] : accb[i][0];
          }
        } else if ((lane & 15) == 0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = m0 + wm * 16 * FM + i * 16 + 4 * (lane >> 4) + r;
            if (row < g.M) {
              if (g.atomic) atomicAdd(bdst + row, accb[i][r]);
              else bdst[row] = g.beta_acc ? bdst[row] + accb[i][r] : accb[i][r];
            }
          }
        }
      }
    }
    GSTAMP(4);
    __syncthreads();  // every wave is done with the LDS stages before the next tile's prologue
}


// SWAP: accumulate C^T tiles (lane owns 4 consecutive output columns of one row).
// Persistent over tiles (grid = min(tiles, WG_PER_CU * 256)); per tile: NS-deep DMA prologue,
// k-loop with counted waits, drain, epilogue.  With NS = 2 (64 KiB LDS) two workgroups share a
// CU, so one's prologue/epilogue overlaps the other's MFMA loop.
// FM = 16-row A fragments per wave: 4 -> 128 x 128 tiles, 2 -> 64 x 128 tiles (twice the
// workgroups for the transformer's N = 512 GEMMs, so two tiles share a CU and one's load /
// store phases overlap the other's MFMAs).  A k-major A operand (wgrad) always uses FM = 4.
template <bool AK, bool BKM, bool SWAP, int NS, int FM, int EPI>
__global__ __launch_bounds__(256, (NS <= 2 ? (FM == 2 ? 3 : 2) : (NS == 3 && FM == 2 ? 2 : 1))) void gemm_bf16_kernel(GemmArgs g) {
  constexpr int BMT = 32 * FM;                 // tile rows (M)
  constexpr int NPA = AK ? 4 : FM;             // DMA pieces per wave per stage, A operand
  constexpr int A_ELEMS = BMT * BKK;
  constexpr int STAGE = A_ELEMS + TILE_ELEMS;  // A then B (128 rows) per stage
  __shared__ __attribute__((aligned(16))) unsigned short smem[NS * STAGE];
  const int nwg = ((g.M + BMT - 1) / BMT) * ((g.N + BN - 1) / BN);
  const int total_tiles = nwg * g.splits;
  for (int t = blockIdx.x; t < total_tiles; t += gridDim.x) gemm_tile<AK, BKM, SWAP, NS, FM, EPI>(g, t, smem);
}


static int g_bm_force = 0;
// runtime override of the tile height (64 / 128; 0 = automatic) — A/B probes in one process
extern "C" void smi_gemm_set_bm(int bm) { g_bm_force = bm; }

extern "C" int smi_gemm(const GemmArgs* args, hipStream_t st) {
  GemmArgs g = *args;
  if (g.K % 8 != 0 || g.K < 8 || g.M < 8 || g.N < 8 || (g.mode != 0 && (g.M % 8 || g.N % 8))) return -1;
  if (g.splits < 1) g.splits = 1;
  int kps = (g.K / g.splits + BKK - 1) / BKK * BKK;
  if (kps < BKK) kps = BKK;
  g.k_per_split = kps;
  g.splits = (g.K + kps - 1) / kps;
  if (g.splits > 1 && !(g.out_f32 && (g.atomic || g.c_split_stride >= (long)g.M * g.ldc))) return -1;
  // operand extents (elements -> bytes) for the DMA buffer descriptors
  const bool ak = g.mode == 2, bk = g.mode != 0;
  g.a_bytes = 2 * (ak ? (long)(g.K - 1) * g.lda + g.M : (long)(g.M - 1) * g.lda + g.K);
  g.b_bytes = 2 * (bk ? (long)(g.K - 1) * g.ldb + g.N : (long)(g.N - 1) * g.ldb + g.K);
  if (g.a_bytes >= (1L << 31) || g.b_bytes >= (1L << 31)) return -1;
  // tile height: 64 rows (up to 3 workgroups per CU whose load / MFMA / store phases overlap)
  // unless there are > 4 128-row tiles per CU anyway (the vocab projection); measured on the
  // transformer shapes (tools/probes/run_gemm_probe3.sh).
  const int tiles128 = ((g.M + 127) / 128) * ((g.N + BN - 1) / BN) * g.splits;
  int bm = (ak || tiles128 > 1024) ? 128 : 64;
  if (!ak && (g_bm_force == 64 || g_bm_force == 128)) bm = g_bm_force;
  const int ntiles = ((g.M + bm - 1) / bm) * ((g.N + BN - 1) / BN) * g.splits;
  // pipeline depth: NS=2 (two workgroups per CU) or NS=4 (one per CU, three k-steps in flight)
  // ring depth: 2 stages (2-3 WGs per CU) everywhere by default — measured: 3 or 4 stages
  // (fewer WGs per CU) were 3-5 % slower per step, for WGRAD too.
  const int ns = ak ? 2 : GEMM_NS;
  const int maxg = NUM_CU * (ns == 2 ? (bm == 64 ? 3 : 2) : (ns == 3 && bm == 64 ? 2 : 1));
  const int grid = ntiles < maxg ? ntiles : maxg;
  const bool atomic = g.out_f32 && g.atomic;


  const int epi = (g.bias ? EPI_BIAS : 0) | (g.resid ? EPI_RESID : 0) | (g.act == 1 ? EPI_RELU : 0) |
                  (g.dact_y ? EPI_DACT : 0) | (!g.dact_y && g.thresh ? EPI_DROP : 0);
#define SMI_K(MODEB, NSV, FMV, E) hipLaunchKernelGGL((gemm_bf16_kernel<false, MODEB, true, NSV, FMV, E>), dim3(grid), dim3(256), 0, st, g)
  // specialised epilogues for the feature sets the models use; anything else -> generic (-1)
#define SMI_GEMM_LAUNCH(NSV, FMV)                                                            \
  if (g.mode == 0) {                                                                         \
    switch (epi) {                                                                           \
      case 0: SMI_K(false, NSV, FMV, 0); break;                                              \
      case EPI_BIAS: SMI_K(false, NSV, FMV, EPI_BIAS); break;                                \
      case EPI_BIAS | EPI_RELU: SMI_K(false, NSV, FMV, EPI_BIAS | EPI_RELU); break;          \
      case EPI_BIAS | EPI_RELU | EPI_DROP: SMI_K(false, NSV, FMV, EPI_BIAS | EPI_RELU | EPI_DROP); break; \
      default: SMI_K(false, NSV, FMV, -1); break;                                            \
    }                                                                                        \
  } else if (g.mode == 1) {                                                                  \
    switch (epi) {                                                                           \
      case 0: SMI_K(true, NSV, FMV, 0); break;                                               \
      case EPI_RESID: SMI_K(true, NSV, FMV, EPI_RESID); break;                               \
      case EPI_DACT: SMI_K(true, NSV, FMV, EPI_DACT); break;                                 \
      default: SMI_K(true, NSV, FMV, -1); break;                                             \
    }                                                                                        \
  } else {                                                                                   \
    return -1;                                                                               \
  }
  if (g.mode == 2) {
    if (ns == 4) {
      if (atomic) hipLaunchKernelGGL((gemm_bf16_kernel<true, true, false, 4, 4, 0>), dim3(grid), dim3(256), 0, st, g);
      else hipLaunchKernelGGL((gemm_bf16_kernel<true, true, true, 4, 4, 0>), dim3(grid), dim3(256), 0, st, g);
    } else {
      if (atomic) hipLaunchKernelGGL((gemm_bf16_kernel<true, true, false, 2, 4, 0>), dim3(grid), dim3(256), 0, st, g);
      else hipLaunchKernelGGL((gemm_bf16_kernel<true, true, true, 2, 4, 0>), dim3(grid), dim3(256), 0, st, g);
    }
  } else if (ns == 4) {
    if (bm == 64) { SMI_GEMM_LAUNCH(4, 2) } else { SMI_GEMM_LAUNCH(4, 4) }
  } else if (ns == 3) {
    if (bm == 64) { SMI_GEMM_LAUNCH(3, 2) } else { SMI_GEMM_LAUNCH(3, 4) }
  } else {
    if (bm == 64) { SMI_GEMM_LAUNCH(2, 2) } else { SMI_GEMM_LAUNCH(2, 4) }
  }
#undef SMI_GEMM_LAUNCH
#undef SMI_K
  SMI_CHECK_LAUNCH();
}

// out[i] (+)= sum_s slab[s][i]: the split-K combine of a slab-mode GEMM (deterministic, no atomics).
// One launch folds BOTH the weight slabs (n elements per split) and the optional bias slabs (nb
// per split, stored after the weight slabs): the bias range is handled by the grid's tail blocks.
// Each thread owns one float4 and issues the loads of all its splits before adding (SPLITS is a
// compile-time constant, so all S loads are in flight at once — the fold is HBM/MALL-bound, not
// latency-bound); the running sum is added in split order, so the result is deterministic.
template <int SPLITS>
__device__ __forceinline__ void fold4(const float* __restrict__ slab, long stride4, long i, float4* __restrict__ out,
                                      int accumulate) {
  float4 v[SPLITS];
#pragma unroll
  for (int s = 0; s < SPLITS; ++s) v[s] = ((const float4*)slab)[(long)s * stride4 + i];
  float4 acc = accumulate ? out[i] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int s = 0; s < SPLITS; ++s) { acc.x += v[s].x; acc.y += v[s].y; acc.z += v[s].z; acc.w += v[s].w; }
  out[i] = acc;
}

template <int SPLITS>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ slab, int splits, long n,
                                                           float* __restrict__ out, long nb, float* __restrict__ bout,
                                                           int accumulate, int wblocks) {
  if ((int)blockIdx.x < wblocks) {
    const long n4 = n / 4;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)wblocks * 256) {
      if constexpr (SPLITS > 0) fold4<SPLITS>(slab, n4, i, (float4*)out, accumulate);
      else {
        float4 acc = accumulate ? ((const float4*)out)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        for (int s = 0; s < splits; ++s) {
          const float4 v = ((const float4*)(slab + (long)s * n))[i];
          acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
        ((float4*)out)[i] = acc;
      }
    }
    for (long i = n4 * 4 + (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)wblocks * 256) {
      float acc = accumulate ? out[i] : 0.f;
      for (int s = 0; s < splits; ++s) acc += slab[(long)s * n + i];
      out[i] = acc;
    }
  } else {
    const float* bslab = slab + (long)splits * n;
    for (long i = (long)(blockIdx.x - wblocks) * 256 + threadIdx.x; i < nb; i += (long)(gridDim.x - wblocks) * 256) {
      float acc = accumulate ? bout[i] : 0.f;
      for (int s = 0; s < splits; ++s) acc += bslab[(long)s * nb + i];
      bout[i] = acc;
    }
  }
}

extern "C" int smi_splitk_reduce(const float* slab, int splits, long n, float* out, long nb, float* bout,
                                 int accumulate, hipStream_t st) {
  long blocks = (n / 4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  const int bblocks = (nb > 0 && bout) ? (int)((nb + 255) / 256 < 8 ? (nb + 255) / 256 : 8) : 0;
  if (!bout) nb = 0;
  const dim3 grid((unsigned)(blocks + bblocks));
  const int wb = (int)blocks;
#define SMI_RED(S) hipLaunchKernelGGL(splitk_reduce_kernel<S>, grid, dim3(256), 0, st, slab, splits, n, out, nb, bout, accumulate, wb)
  if (n % 4 != 0) { SMI_RED(0); }
  else switch (splits) {
    case 2: SMI_RED(2); break;
    case 4: SMI_RED(4); break;
    case 8: SMI_RED(8); break;
    case 16: SMI_RED(16); break;
    default: SMI_RED(0); break;
  }
#undef SMI_RED
  SMI_CHECK_LAUNCH();
}

// Deferred split-K folds of many weight-gradient GEMMs in ONE launch (sparkmi/ops/_grad.py:
// queued during the backward, flushed by the autograd final callback).  Entry e owns blocks
// [blk0[e], blk0[e+1]): its weight float4s first (one per thread), then its bias elements.
// Outputs of one batch are distinct (the host splits batches on a repeated output).
#define FOLD_MAX 64
struct FoldBatch {
  const float* slab[FOLD_MAX]; float* out[FOLD_MAX]; float* bout[FOLD_MAX];
  long n[FOLD_MAX]; int nb[FOLD_MAX]; int splits[FOLD_MAX]; int wblk[FOLD_MAX];
  int blk0[FOLD_MAX + 1]; int count;
};
__global__ __launch_bounds__(256) void splitk_fold_multi_kernel(FoldBatch a) {
  const int b = blockIdx.x;
  int e = 0;
  while (e + 1 < a.count && b >= a.blk0[e + 1]) ++e;  // wave-uniform scan over <= 64 entries
  const int lb = b - a.blk0[e];
  const float* slab = a.slab[e];
  const long n = a.n[e];
  const int S = a.splits[e];
  if (lb < a.wblk[e]) {
    const long n4 = n / 4;
    const long i = (long)lb * 256 + threadIdx.x;
    if (i < n4) {
      float4 acc = ((const float4*)a.out[e])[i];
      if (S <= 16) {  // all split loads in flight, then summed in split order
        float4 p[16];
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2)
          if (s2 < S) p[s2] = ((const float4*)(slab + (long)s2 * n))[i];
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2)
          if (s2 < S) { acc.x += p[s2].x; acc.y += p[s2].y; acc.z += p[s2].z; acc.w += p[s2].w; }
      } else {
        for (int s2 = 0; s2 < S; ++s2) {
          const float4 v = ((const float4*)(slab + (long)s2 * n))[i];
          acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
      }
      ((float4*)a.out[e])[i] = acc;
    }
    if (lb == 0)  // n % 4 tail
      for (long t = n4 * 4 + threadIdx.x; t < n; t += 256) {
        float acc = a.out[e][t];
        for (int s2 = 0; s2 < S; ++s2) acc += slab[(long)s2 * n + t];
        a.out[e][t] = acc;
      }
  } else {
    const long i = (long)(lb - a.wblk[e]) * 256 + threadIdx.x;
    if (i < a.nb[e]) {
      const float* bslab = slab + (long)S * n;
      float acc = a.bout[e][i];
      for (int s2 = 0; s2 < S; ++s2) acc += bslab[(long)s2 * a.nb[e] + i];
      a.bout[e][i] = acc;
    }
  }
}

extern "C" int smi_splitk_fold_multi(const float* const* slab, float* const* out, float* const* bout, const long* n,
                                     const int* nb, const int* splits, int count, hipStream_t st) {
  if (count < 1 || count > FOLD_MAX) return -1;
  FoldBatch a{};
  int tot = 0;
  for (int i = 0; i < count; ++i) {
    a.slab[i] = slab[i]; a.out[i] = out[i]; a.bout[i] = bout[i]; a.n[i] = n[i];
    a.nb[i] = bout[i] ? nb[i] : 0; a.splits[i] = splits[i];
    a.wblk[i] = (int)((n[i] / 4 + 255) / 256);
    if (a.wblk[i] < 1) a.wblk[i] = 1;
    a.blk0[i] = tot;
    tot += a.wblk[i] + (a.nb[i] + 255) / 256;
  }
  a.blk0[count] = tot;
  a.count = count;
  hipLaunchKernelGGL(splitk_fold_multi_kernel, dim3((unsigned)tot), dim3(256), 0, st, a);
  SMI_CHECK_LAUNCH();
}

// Grouped weight-gradient GEMMs: gw_e[N,K] += dY_e[T,N]^T X_e[T,K] (and gb_e[N] += dY_e^T 1)
// for up to WG_MAX problems in ONE persistent launch, with no split-K (sparkmi/ops/_grad.py:
// every Linear's wgrad is queued during the backward — it is off the critical path — and the
// queue is flushed by the autograd final callback).  One launch covers ~2,000 128 x 128 output
// tiles of the whole backward, each with its FULL token reduction (T / 64 k-steps), so the
// per-tile prologue / epilogue is amortised over ~128 k-steps instead of 8-16 split-K steps, and
// the fp32 slabs (~1.4 GB written + read per transformer step) disappear: each tile owns its
// output and adds straight into gw.  Problem e's tiles start at t0[e], a multiple of 8, so the
// XCD-aware remap inside tile_of sees the same XCD pattern as a standalone launch.
#define WG_MAX 40
struct WgradGroup {
  const unsigned short* A[WG_MAX]; const unsigned short* B[WG_MAX];
  float* C[WG_MAX]; float* bias[WG_MAX];
  int lda[WG_MAX], ldb[WG_MAX], n[WG_MAX], k[WG_MAX], T[WG_MAX];
  int t0[WG_MAX + 1]; int count;
};
__global__ __launch_bounds__(256, 2) void gemm_wgrad_group_kernel(WgradGroup gr) {
  __shared__ __attribute__((aligned(16))) unsigned short smem[2 * (2 * TILE_ELEMS)];
  const int total = gr.t0[gr.count];
  for (int t = blockIdx.x; t < total; t += gridDim.x) {
    int e = 0;
    while (e + 1 < gr.count && t >= gr.t0[e + 1]) ++e;  // uniform scan over <= WG_MAX entries
    GemmArgs g{};
    g.mode = 2; g.A = gr.A[e]; g.lda = gr.lda[e]; g.B = gr.B[e]; g.ldb = gr.ldb[e];
    g.M = gr.n[e]; g.N = gr.k[e]; g.K = gr.T[e]; g.C = gr.C[e]; g.ldc = gr.k[e];
    g.out_f32 = 1; g.atomic = 0; g.beta_acc = 1; g.alpha = 1.f; g.dscale = 1.f;
    g.splits = 1; g.k_per_split = g.K;
    g.a_bytes = 2 * ((long)(g.K - 1) * g.lda + g.M);
    g.b_bytes = 2 * ((long)(g.K - 1) * g.ldb + g.N);
    g.bias_grad = gr.bias[e];
    const int lt = t - gr.t0[e];
    const int nwg = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
    if (lt < nwg) gemm_tile<true, true, true, 2, 4, 0>(g, lt, smem);  // lt >= nwg: alignment padding
  }
}

extern "C" int smi_gemm_wgrad_group(const void* const* A, const long* lda, const void* const* B, const long* ldb,
                                    void* const* C, void* const* bias, const int* n, const int* k, const int* T,
                                    int count, hipStream_t st) {
  if (count < 1 || count > WG_MAX) return -1;
  WgradGroup gr{};
  int tot = 0;
  for (int i = 0; i < count; ++i) {
    // same preconditions as smi_gemm's WGRAD path (multiples of 8, descriptor-addressable operands)
    if (T[i] < 8 || n[i] < 8 || k[i] < 8 || T[i] % 8 || n[i] % 8 || k[i] % 8) return -1;
    if (lda[i] < n[i] || ldb[i] < k[i] || lda[i] > (1L << 30) || ldb[i] > (1L << 30)) return -1;
    if (2 * ((long)(T[i] - 1) * lda[i] + n[i]) >= (1L << 31) || 2 * ((long)(T[i] - 1) * ldb[i] + k[i]) >= (1L << 31))
      return -1;
    gr.A[i] = (const unsigned short*)A[i]; gr.B[i] = (const unsigned short*)B[i];
    gr.C[i] = (float*)C[i]; gr.bias[i] = (float*)bias[i];
    gr.lda[i] = (int)lda[i]; gr.ldb[i] = (int)ldb[i]; gr.n[i] = n[i]; gr.k[i] = k[i]; gr.T[i] = T[i];
    gr.t0[i] = tot;
    const int nwg = ((n[i] + BM - 1) / BM) * ((k[i] + BN - 1) / BN);
    tot += (nwg + 7) / 8 * 8;
  }
  gr.t0[count] = tot;
  gr.count = count;
  const int grid = tot < 2 * NUM_CU ? tot : 2 * NUM_CU;
  hipLaunchKernelGGL(gemm_wgrad_group_kernel, dim3(grid), dim3(256), 0, st, gr);
  SMI_CHECK_LAUNCH();
}
