// bf16 GEMM on the 256 x 128, 8-wave, v_mfma_f32_16x16x32_bf16 tile of the split-plane GEMM
// (csrc/include/smi_gemm_sp_impl.h gemm_sp_tile256m with NPL = 2): the bf16 path of every
// transformer Linear whose problem fills the chip (transformer.py:71-72,107-117,175-176,271 run
// in bf16 with fp32 master weights).  A 64-deep k-step is staged as the two 32-deep "planes" of
// the fp32 tile's LDS image (plane stride 32 elements k-contig / 32 rows k-major), so the bf16 GEMM
// inherits its LDS-DMA stages, swizzles, transposing fragment reads, XCD-aware tile order and the
// row-segment epilogue (bias / ReLU / dropout / residual / relu'-mask, bf16 in and out via SE_BF;
// fp32 accumulation into the weight gradients).  Shapes it does not cover (K of a k-contiguous
// operand not a multiple of 64, fewer than one wave of 256-row tiles, unaligned operands,
// split-K / atomic / fp32-output modes) keep the 128 x 128 persistent kernel of gemm.hip.
#include "smi_gemm_sp_impl.h"
#include "smi_gemm.h"

template <bool AK, bool BKM, int EPI, int OUT>
__global__ __launch_bounds__(512, 1) void gemm_bf256_kernel(GemmSpArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned short lds[2 * SP_ST256];
  const int nwg = ((g.M + 255) / 256) * ((g.N + 127) / 128);
  gemm_sp_tile256m<AK, BKM, EPI, OUT, false, 2>(g, sp_tile_remap(blockIdx.x, nwg), lds);
}

// the 256 x 128 bf16 kernels (1) or always gemm.hip's 128 x 128 kernel (0, default).  Measured in
// the bf16 transformer step (profiles/r5_ab_gemm_bf256.log): QKV 28.3 vs 22.2 us (384 tiles = 1.5
// waves of one 8-wave WG per CU), FFN1 21.5 vs 20.4, vocab 83.6 vs 80.7, wgrad groups 0.90 vs
// 0.87 ms -- the 2-plane k-step does not hide its LDS stage the way the 6-product fp32 step does,
// so the 128 x 128 kernel (2 WGs per CU) stays the bf16 default; opt-in for tests and A/B.
static int g_bf256 = 0;
extern "C" int smi_gemm_bf256_enable(int set) {
  if (set == 0 || set == 1) g_bf256 = set;
  return g_bf256;
}

static inline bool bf_al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
static inline bool bf_al8(const void* p) { return ((uintptr_t)p & 7) == 0; }

// 1: launched, 0: not covered (the caller runs gemm.hip's kernel), < 0: launch error
extern "C" int smi_gemm_bf256(const GemmArgs* args, hipStream_t st) {
  const GemmArgs& a = *args;
  if (!g_bf256 || (a.mode != 0 && a.mode != 1) || a.out_f32 || a.atomic || a.beta_acc || a.splits > 1 ||
      a.alpha != 1.f || a.bias_grad)
    return 0;
  if (a.K % 64 || a.M < 1 || a.N < 1 || a.N % 4 || a.ldc % 4) return 0;
  if (!bf_al16(a.A) || !bf_al16(a.B) || a.lda % 8 || a.ldb % 8 || !bf_al8(a.C)) return 0;
  if (a.mode == 0 && (a.resid || a.dact_y || a.act > 1)) return 0;
  if (a.mode == 1 && (a.bias || a.act || (a.thresh && !a.dact_y))) return 0;
  if (a.resid && (!bf_al8(a.resid) || a.ldr % 4)) return 0;
  if (a.dact_y && (!bf_al8(a.dact_y) || a.ldy % 4)) return 0;
  if (a.mode == 1 && a.N % 8) return 0;  // k-major B: 16-B chunks along its columns
  const long t256 = (long)((a.M + 255) / 256) * ((a.N + 127) / 128);
  if (t256 < SP_NUM_CU) return 0;  // fewer tiles than CUs: the 64 / 128-row kernel fills the chip better
  GemmSpArgs g{};
  g.mode = a.mode;
  g.A = a.A; g.lda = a.lda; g.aps = 32;
  g.B = a.B; g.ldb = a.ldb; g.bps = a.mode == 0 ? 32 : 32 * a.ldb;
  g.M = a.M; g.N = a.N; g.K = a.K;
  g.C = (float*)a.C; g.ldc = a.ldc;  // bf16 storage (SE_BF)
  g.bias = a.bias; g.relu = a.act == 1;
  g.resid = (const float*)a.resid; g.ldr = a.ldr;  // bf16 storage (SE_BF)
  g.dact_y = (const float*)a.dact_y; g.ldy = a.ldy;
  g.seedp = a.seedp; g.salt = a.salt; g.thresh = a.thresh; g.dscale = a.dscale;
  const long ea = 2 * ((long)(a.M - 1) * a.lda + a.K);
  const long eb = a.mode == 0 ? 2 * ((long)(a.N - 1) * a.ldb + a.K) : 2 * ((long)(a.K - 1) * a.ldb + a.N);
  if (ea >= (1L << 31) || eb >= (1L << 31)) return 0;
  g.a_bytes = (int)ea; g.b_bytes = (int)eb;
  const dim3 grid((unsigned)t256);
  const int drop = a.thresh && !a.dact_y;
  if (a.mode == 0) {
    const int epi = (a.bias ? SE_BIAS : 0) | (a.act == 1 ? SE_RELU : 0) | (drop ? SE_DROP : 0);
#define BFF(E) hipLaunchKernelGGL((gemm_bf256_kernel<false, false, SE_BF | (E), SO_C>), grid, dim3(512), 0, st, g)
    switch (epi) {
      case 0: BFF(0); break;
      case SE_BIAS: BFF(SE_BIAS); break;
      case SE_BIAS | SE_RELU: BFF(SE_BIAS | SE_RELU); break;
      case SE_BIAS | SE_RELU | SE_DROP: BFF(SE_BIAS | SE_RELU | SE_DROP); break;
      default: return 0;
    }
#undef BFF
  } else {
    const int epi = (a.resid ? SE_RESID : 0) | (a.dact_y ? SE_DACT : 0);
#define BFD(E) hipLaunchKernelGGL((gemm_bf256_kernel<false, true, SE_BF | (E), SO_C>), grid, dim3(512), 0, st, g)
    switch (epi) {
      case 0: BFD(0); break;
      case SE_RESID: BFD(SE_RESID); break;
      case SE_DACT: BFD(SE_DACT); break;
      case SE_RESID | SE_DACT: BFD(SE_RESID | SE_DACT); break;
      default: return 0;
    }
#undef BFD
  }
  return hipGetLastError() == hipSuccess ? 1 : -1;
}

// Grouped bf16 weight gradients on the same tile: gw_e[n,k] += dY_e[T,n]^T X_e[T,k] (+ gb_e[n] +=
// dY_e^T 1) for up to BFG_MAX entries in one launch, every tile reducing all T tokens into the fp32
// gradient (no split-K, deterministic).  Both operands k-major (tokens = k): no T % 64 condition.
#define BFG_MAX 40
struct BfWgradGroup {
  const unsigned short* A[BFG_MAX]; const unsigned short* B[BFG_MAX];
  float* C[BFG_MAX]; float* bias[BFG_MAX];
  int lda[BFG_MAX], ldb[BFG_MAX], n[BFG_MAX], k[BFG_MAX], T[BFG_MAX], a_bytes[BFG_MAX], b_bytes[BFG_MAX];
  int t0[BFG_MAX + 1]; int count;
};
__global__ __launch_bounds__(512, 1) void gemm_bf_wgrad_group256_kernel(BfWgradGroup gr) {
  __shared__ __attribute__((aligned(16))) unsigned short lds[2 * SP_ST256];
  const int t = blockIdx.x;
  int e = 0;
  while (e + 1 < gr.count && t >= gr.t0[e + 1]) ++e;
  GemmSpArgs g{};
  g.mode = 2; g.A = gr.A[e]; g.lda = gr.lda[e]; g.aps = 32L * gr.lda[e]; g.B = gr.B[e]; g.ldb = gr.ldb[e];
  g.bps = 32L * gr.ldb[e]; g.M = gr.n[e]; g.N = gr.k[e]; g.K = gr.T[e]; g.C = gr.C[e]; g.ldc = gr.k[e];
  g.beta_acc = 1; g.dscale = 1.f; g.bias_grad = gr.bias[e];
  g.a_bytes = gr.a_bytes[e]; g.b_bytes = gr.b_bytes[e];
  const int nwg = ((g.M + 255) / 256) * ((g.N + 127) / 128);
  const int lt = t - gr.t0[e];
  if (lt >= nwg) return;  // alignment padding
  const int tile = sp_tile_remap(lt, nwg);
  if (g.bias_grad && tile % ((g.N + 127) / 128) == 0)
    gemm_sp_tile256m<true, true, SE_ACC, SO_C, true, 2>(g, tile, lds);
  else
    gemm_sp_tile256m<true, true, SE_ACC, SO_C, false, 2>(g, tile, lds);
}

// same contract as gemm.hip smi_gemm_wgrad_group; 1 launched, 0 not covered, < 0 error
extern "C" int smi_gemm_bf_wgrad_group(const void* const* A, const long* lda, const void* const* B, const long* ldb,
                                       void* const* C, void* const* bias, const int* n, const int* k, const int* T,
                                       int count, hipStream_t st) {
  if (!g_bf256 || count < 1 || count > BFG_MAX) return 0;
  BfWgradGroup gr{};
  int tot = 0;
  for (int i = 0; i < count; ++i) {
    if (!bf_al16(A[i]) || !bf_al16(B[i]) || lda[i] % 8 || ldb[i] % 8 || n[i] % 8 || k[i] % 8 || T[i] < 1 ||
        lda[i] < n[i] || ldb[i] < k[i] || !C[i] || ((uintptr_t)C[i] & 15))
      return 0;
    const long ea = 2 * ((long)(T[i] - 1) * lda[i] + n[i]), eb = 2 * ((long)(T[i] - 1) * ldb[i] + k[i]);
    if (ea >= (1L << 31) || eb >= (1L << 31) || lda[i] > (1L << 24) || ldb[i] > (1L << 24)) return 0;
    gr.A[i] = (const unsigned short*)A[i]; gr.B[i] = (const unsigned short*)B[i];
    gr.C[i] = (float*)C[i]; gr.bias[i] = (float*)bias[i];
    gr.lda[i] = (int)lda[i]; gr.ldb[i] = (int)ldb[i]; gr.n[i] = n[i]; gr.k[i] = k[i]; gr.T[i] = T[i];
    gr.a_bytes[i] = (int)ea; gr.b_bytes[i] = (int)eb;
    gr.t0[i] = tot;
    tot += (((n[i] + 255) / 256) * ((k[i] + 127) / 128) + 7) / 8 * 8;
  }
  gr.t0[count] = tot;
  gr.count = count;
  if (tot < SP_NUM_CU) return 0;
  hipLaunchKernelGGL(gemm_bf_wgrad_group256_kernel, dim3((unsigned)tot), dim3(512), 0, st, gr);
  return hipGetLastError() == hipSuccess ? 1 : -1;
}
