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

// Global -> registers: the operand tile at (row/col origin r0, k origin k0).  Out-of-range rows /
// columns / k read as 0 (rlim, klim exclusive; float4 granularity: klim % 4 == 0 for k-contig,
// rlim % 4 == 0 for k-major, checked by the launcher).
template <bool KMAJ, int R>
__device__ __forceinline__ void f32_gload(const float* __restrict__ base, long ld, int r0, int rlim, int k0, int klim,
                                          float4 (&v)[F32Tile<KMAJ, R>::NV], int tid) {
#pragma unroll
  for (int i = 0; i < F32Tile<KMAJ, R>::NV; ++i) {
    const int f = tid + 256 * i;
    if (!KMAJ) {
      const int row = f >> 3, gr = r0 + row, gk = k0 + (f & 7) * 4;
      v[i] = (gr < rlim && gk < klim) ? *(const float4*)(base + (long)gr * ld + gk) : make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      const int kr = f / (R / 4), gk = k0 + kr, gc = r0 + (f % (R / 4)) * 4;
      v[i] = (gk < klim && gc < rlim) ? *(const float4*)(base + (long)gk * ld + gc) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
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

// One output tile (all its k-tiles of split `split` and the epilogue).
template <bool AK, bool BKM, int FM>
__device__ __forceinline__ void gemm_f32_tile(const GemmF32Args& g, int tile, int split, float* smem) {
  constexpr int BMT = 64 * FM;
  using TA = F32Tile<AK, BMT>;
  using TB = F32Tile<BKM, FBN>;
  constexpr int STAGE = TA::ELEMS + TB::ELEMS;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int ntn = (g.N + FBN - 1) / FBN;
  const int m0 = (tile / ntn) * BMT, n0 = (tile % ntn) * FBN;
  const int kbeg = split * g.k_per_split;
  const int kend = min(g.K, kbeg + g.k_per_split);
  const int nk = (kend - kbeg + FBK - 1) / FBK;

  f32x16_t acc[FM][2];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const bool do_bias = AK && g.bias_grad && n0 == 0 && wn == 0;
  float bsum[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) bsum[i] = 0.f;

  float4 va[TA::NV], vb[TB::NV];
  f32_gload<AK, BMT>(g.A, g.lda, m0, g.M, kbeg, kend, va, tid);
  f32_gload<BKM, FBN>(g.B, g.ldb, n0, g.N, kbeg, kend, vb, tid);
  f32_lstore<AK, BMT>(smem, va, tid);
  f32_lstore<BKM, FBN>(smem + TA::ELEMS, vb, tid);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {  // next k-tile's loads fly under this k-tile's MFMAs
      f32_gload<AK, BMT>(g.A, g.lda, m0, g.M, kbeg + (kt + 1) * FBK, kend, va, tid);
      f32_gload<BKM, FBN>(g.B, g.ldb, n0, g.N, kbeg + (kt + 1) * FBK, kend, vb, tid);
    }
    const float* ta = smem + (kt & 1) * STAGE;
    const float* tb = ta + TA::ELEMS;
    float af[FM][16], bf[2][16];
#pragma unroll
    for (int i = 0; i < FM; ++i) f32_frag<AK, BMT>(ta, wm * BMT / 2 + i * 32, lane, af[i]);
#pragma unroll
    for (int j = 0; j < 2; ++j) f32_frag<BKM, FBN>(tb, wn * 64 + j * 32, lane, bf[j]);
#pragma unroll
    for (int s = 0; s < 16; ++s)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
    if (do_bias) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int s = 0; s < 16; ++s) bsum[i] += af[i][s];
    }
    if (more) {
      float* nx = smem + ((kt + 1) & 1) * STAGE;
      f32_lstore<AK, BMT>(nx, va, tid);
      f32_lstore<BKM, FBN>(nx + TA::ELEMS, vb, tid);
    }
    __syncthreads();
  }

  // ---------------- epilogue ----------------
  const uint32_t seed = g.thresh ? smi_seed(g.seedp, g.salt) : 0u;
  const int h = lane >> 5;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn * 64 + j * 32 + (lane & 31);
    const bool cok = col < g.N;
    const float bia = (g.bias && cok) ? g.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * BMT / 2 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (!cok || row >= g.M) continue;
        const long cidx = (long)row * g.ldc + col;
        float v = acc[i][j][r];
        if (g.mode == 0) {
          v += bia;
          if (g.relu == 1) v = fmaxf(v, 0.f);
          else if (g.relu == 2) v = 1.f / (1.f + __expf(-v));
          if (g.thresh) v = smi_keep(seed, (uint32_t)cidx, g.thresh) ? v * g.dscale : 0.f;
        } else if (g.mode == 1) {
          if (g.resid) v += g.resid[(long)row * g.ldr + col];
          if (g.dact_y) v = g.dact_y[(long)row * g.ldy + col] > 0.f ? v * g.dscale : 0.f;
        }
        if (g.atomic) atomicAdd(g.C + cidx, v);
        else g.C[cidx] = g.beta_acc ? g.C[cidx] + v : v;
      }
    }
  }
  if (do_bias) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      // lanes l and l + 32 hold the two k-halves of row (l & 31)
      auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(bsum[i]), __float_as_uint(bsum[i]), false, false);
      const float tot = __uint_as_float(a[0]) + __uint_as_float(a[1]);
      const int row = m0 + wm * BMT / 2 + i * 32 + (lane & 31);
      if (h == 0 && row < g.M) {
        if (g.atomic) atomicAdd(g.bias_grad + row, tot);
        else g.bias_grad[row] = g.beta_acc ? g.bias_grad[row] + tot : tot;
      }
    }
  }
}

template <bool AK, bool BKM, int FM>
__global__ __launch_bounds__(256, 2) void gemm_f32_kernel(GemmF32Args g) {
  constexpr int BMT = 64 * FM;
  __shared__ __attribute__((aligned(16))) float smem[2 * (F32Tile<AK, BMT>::ELEMS + F32Tile<BKM, FBN>::ELEMS)];
  const int nwg = ((g.M + BMT - 1) / BMT) * ((g.N + FBN - 1) / FBN);
  const int split = blockIdx.x / nwg;
  const int tile = f32_tile_remap(blockIdx.x - split * nwg, nwg);
  gemm_f32_tile<AK, BKM, FM>(g, tile, split, smem);
}

static int f32_ok(const GemmF32Args& g) {
  if (g.M < 1 || g.N < 1 || g.K < 1) return 0;
  const bool ak = g.mode == 2, bk = g.mode != 0;
  // float4 staging granularity along each operand's contiguous dimension, 16-B aligned rows
  if ((!ak && g.K % 4) || (ak && g.M % 4) || (!bk && g.K % 4) || (bk && g.N % 4)) return 0;
  if (g.lda % 4 || g.ldb % 4) return 0;
  if (((uintptr_t)g.A | (uintptr_t)g.B) & 15) return 0;
  return 1;
}

extern "C" int smi_gemm_f32(const GemmF32Args* args, hipStream_t st) {
  GemmF32Args g = *args;
  if (!f32_ok(g) || g.mode < 0 || g.mode > 2) return -1;
  const bool ak = g.mode == 2;
  static int bm_env = -1;
  if (bm_env < 0) {
    const char* e = getenv("SMI_GEMM_F32_BM");
    bm_env = e ? atoi(e) : 0;
  }
  const int t128 = ((g.M + 127) / 128) * ((g.N + FBN - 1) / FBN);
  // 64-row tiles until there are >= 2 128-row tiles per CU (two co-resident workgroups per CU)
  int bm = (ak || t128 >= 2 * NUM_CU) ? 128 : 64;
  if (!ak && (bm_env == 64 || bm_env == 128)) bm = bm_env;
  const int nwg = ((g.M + bm - 1) / bm) * ((g.N + FBN - 1) / FBN);
  if (g.splits < 1) g.splits = 1;
  if (g.splits > 1 && !g.atomic) return -1;
  int kps = (g.K / g.splits + FBK - 1) / FBK * FBK;
  if (kps < FBK) kps = FBK;
  g.k_per_split = kps;
  g.splits = (g.K + kps - 1) / kps;
  const dim3 grid((unsigned)(nwg * g.splits)), block(256);
  if (g.mode == 0) {
    if (bm == 64) hipLaunchKernelGGL((gemm_f32_kernel<false, false, 1>), grid, block, 0, st, g);
    else hipLaunchKernelGGL((gemm_f32_kernel<false, false, 2>), grid, block, 0, st, g);
  } else if (g.mode == 1) {
    if (bm == 64) hipLaunchKernelGGL((gemm_f32_kernel<false, true, 1>), grid, block, 0, st, g);
    else hipLaunchKernelGGL((gemm_f32_kernel<false, true, 2>), grid, block, 0, st, g);
  } else {
    hipLaunchKernelGGL((gemm_f32_kernel<true, true, 2>), grid, block, 0, st, g);
  }
  SMI_CHECK_LAUNCH();
}

// Grouped weight-gradient GEMMs (fp32): gw_e[n,k] += dY_e[T,n]^T X_e[T,k] (and gb_e[n] += dY_e^T 1)
// for up to WGF_MAX problems in ONE launch, no split-K: each 128 x 128 output tile reduces all T
// tokens and adds into the fp32 gradient (deterministic, no slabs, no atomics).  Problem e's
// tiles start at t0[e], a multiple of 8 (same XCD pattern as a standalone launch).  Queued by
// sparkmi/ops/_grad.py during the backward and flushed per gradient bucket / at its end.
#define WGF_MAX 40
struct WgradGroupF32 {
  const float* A[WGF_MAX]; const float* B[WGF_MAX];
  float* C[WGF_MAX]; float* bias[WGF_MAX];
  int lda[WGF_MAX], ldb[WGF_MAX], n[WGF_MAX], k[WGF_MAX], T[WGF_MAX];
  int t0[WGF_MAX + 1]; int count;
};
__global__ __launch_bounds__(256, 2) void gemm_f32_wgrad_group_kernel(WgradGroupF32 gr) {
  __shared__ __attribute__((aligned(16))) float smem[2 * (F32Tile<true, 128>::ELEMS + F32Tile<true, FBN>::ELEMS)];
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
  if (lt < nwg) gemm_f32_tile<true, true, 2>(g, f32_tile_remap(lt, nwg), 0, smem);  // lt >= nwg: padding
}

extern "C" int smi_gemm_f32_wgrad_group(const void* const* A, const long* lda, const void* const* B, const long* ldb,
                                        void* const* C, void* const* bias, const int* n, const int* k, const int* T,
                                        int count, hipStream_t st) {
  if (count < 1 || count > WGF_MAX) return -1;
  WgradGroupF32 gr{};
  int tot = 0;
  for (int i = 0; i < count; ++i) {
    if (T[i] < 1 || n[i] < 4 || k[i] < 4 || n[i] % 4 || k[i] % 4 || lda[i] % 4 || ldb[i] % 4) return -1;
    if (lda[i] < n[i] || ldb[i] < k[i] || lda[i] > (1L << 30) || ldb[i] > (1L << 30)) return -1;
    if ((((uintptr_t)A[i]) | ((uintptr_t)B[i])) & 15) return -1;
    gr.A[i] = (const float*)A[i]; gr.B[i] = (const float*)B[i];
    gr.C[i] = (float*)C[i]; gr.bias[i] = (float*)bias[i];
    gr.lda[i] = (int)lda[i]; gr.ldb[i] = (int)ldb[i]; gr.n[i] = n[i]; gr.k[i] = k[i]; gr.T[i] = T[i];
    gr.t0[i] = tot;
    const int nwg = ((n[i] + 127) / 128) * ((k[i] + FBN - 1) / FBN);
    tot += (nwg + 7) / 8 * 8;
  }
  gr.t0[count] = tot;
  gr.count = count;
  hipLaunchKernelGGL(gemm_f32_wgrad_group_kernel, dim3(tot), dim3(256), 0, st, gr);
  SMI_CHECK_LAUNCH();
}
