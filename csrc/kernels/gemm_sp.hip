// Split-plane fp32 GEMM (csrc/include/smi_gemm_sp_impl.h): FORWARD instances, the launcher, and
// the standalone plane splitter.  Reference call sites: every nn.Linear of the reference models
// in fp32 (transformer.py:71-72,107-117,175-176,271 trained by pytorch_machine_translator.py:120-137).
#include "smi_gemm_sp_impl.h"

#include <stdlib.h>

static int g_sp_waves = 8;  // waves per 128 x 128 tile (gemm_sp_waves sets 4 for A/B runs)
int smi_sp_waves() { return g_sp_waves; }
// tile form of the large problems: 16 = 256 x 128 on the 16x16x32 MFMA (default), 256 = the same
// on 32x32x16, 128 = 128 x 128 tiles (a 4-wave software-pipelined 256 x 128 form measured 157 vs
// 181-187 TF and was removed in round 5)
static int sp_tm_env() {  // SMI_SP_TM = 16 | 256 | 128 (profiling A/Bs of whole runs); default 16
  const char* e = getenv("SMI_SP_TM");
  const int v = e ? atoi(e) : 16;
  return (v == 128 || v == 256 || v == 16) ? v : 16;
}
static int g_sp_tm = sp_tm_env();
int smi_sp_tm() { return g_sp_tm; }
// set 128 / 256 / 16 for A/B runs in one process; other values query
extern "C" int smi_gemm_sp_tm(int set) {
  if (set == 128 || set == 256 || set == 16) g_sp_tm = set;
  return smi_sp_tm();
}
// the grouped weight-gradient launch's tile (gemm_sp_wg_tm = 128 | 256 | 16 | 4; default: follow
// smi_sp_tm).  Per backward the group holds every layer's weight gradients, each a long
// K = tokens reduction: fewer, larger tiles can leave CUs idle where 128-row tiles fill them.
// -1 (default): follow smi_sp_tm; 128 / 256 / 16: forced.  128-row tiles for the encoder's
// 1.5-wave group (384 tiles of 256 x 128 on 256 CUs) measured +0.18 ms per fp32 step
// (profiles/r5_ab_wgrad_group_tile.log): the 256-row tile's higher efficiency outweighs the
// half-empty second wave.
static int g_sp_wg_tm = 16;  // (16 = the default sp_tm; pinned so an sp_tm A/B leaves the group alone)
int smi_sp_wg_tm() {
  return g_sp_wg_tm > 0 ? g_sp_wg_tm : smi_sp_tm();
}
extern "C" int smi_gemm_sp_wg_tm(int set) {
  if (set == 128 || set == 256 || set == 16 || set == -1) g_sp_wg_tm = set;
  return smi_sp_wg_tm();
}
extern "C" int smi_gemm_sp_waves(int set) {  // set 4 / 8 (A/B runs in one process); other values query
  if (set == 4 || set == 8) g_sp_waves = set;
  return smi_sp_waves();
}

int smi_sp_launch_dgrad(const GemmSpArgs& g, int epi, int out, dim3 grid, bool t256, hipStream_t st);
int smi_sp_launch_wgrad(const GemmSpArgs& g, int epi, dim3 grid, hipStream_t st);

// x[rows][cols] (row stride ldx) -> planes P[3][rows][ldp] (plane stride ps); columns
// [cols, ldp) of every plane are written as zeros (the k padding of a k-contig GEMM operand).
// One thread per 4 plane columns of a row: a float4 load (scalar at a ragged edge), 3 x 8-B stores.
__global__ __launch_bounds__(256) void split3_kernel(const float* __restrict__ x, long rows, int cols, long ldx,
                                                     unsigned short* __restrict__ P, long ldp, long ps) {
  const long nch = ldp / 4;
  const long total = rows * nch;
  const bool vec = ((ldx | cols) & 3) == 0 && ((uintptr_t)x & 15) == 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / nch;
    const int c = (int)(i - r * nch) * 4;
    float v[4];
    const float* src = x + r * ldx + c;
    if (vec && c + 3 < cols) {
      const float4 t = *(const float4*)src;
      v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = c + e < cols ? src[e] : 0.f;
    }
    sp_store4(P + r * ldp + c, ps, v);
  }
}

extern "C" int smi_split3(const float* x, long rows, int cols, long ldx, void* P, long ldp, long ps, hipStream_t st) {
  if (rows < 1 || cols < 1 || ldp % 4 || ldp < cols || ps < rows * ldp || ((uintptr_t)P & 7)) return -1;
  long blocks = (rows * (ldp / 4) + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(split3_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, rows, cols, ldx,
                     (unsigned short*)P, ldp, ps);
  SMI_CHECK_LAUNCH();
}

extern "C" int smi_gemm_sp(const GemmSpArgs* args, hipStream_t st) {
  GemmSpArgs g = *args;
  if (g.mode < 0 || g.mode > 2 || g.M < 1 || g.N < 1 || g.K < 1) return -1;
  const bool ak = g.mode == 2, bk = g.mode != 0;
  if (!sp_operand_ok(g.A, g.lda, g.aps, g.M, g.M, ak, g.kpad, g.K, g.a_bytes)) return -1;
  if (!sp_operand_ok(g.B, g.ldb, g.bps, g.N, g.N, bk, g.kpad, g.K, g.b_bytes)) return -1;
  if (g.P && (((uintptr_t)g.P & 7) || g.ldp % 4 || g.pps % 4)) return -1;
  if (!g.C && !g.P) return -1;
  if (g.mode == 2 && g.P) return -1;
  const int out = (g.C ? SO_C : 0) | (g.P ? SO_P : 0) | (g.mode == 0 && g.mask ? SO_M : 0);
  if (g.mask && (g.ldm < (g.N + 3) / 4 || (g.mode == 1 && g.dact_y))) return -1;
  const bool t256 = sp_use256(g.M, g.N);
  const int nwg = t256 ? ((g.M + 255) / 256) * ((g.N + 127) / 128) : ((g.M + 127) / 128) * ((g.N + 127) / 128);
  const dim3 grid((unsigned)nwg);
  int epi = 0;
  if (g.mode == 0) epi = (g.bias ? SE_BIAS : 0) | (g.relu == 1 ? SE_RELU : 0) | (g.thresh ? SE_DROP : 0);
  else if (g.mode == 1) epi = (g.resid ? SE_RESID : 0) | (g.dact_y ? SE_DACT : 0) | (g.mask ? SE_DMASK : 0);
  if (g.beta_acc) epi |= SE_ACC;
  if (g.mode == 1) return smi_sp_launch_dgrad(g, epi, out, grid, t256, st);  // csrc/kernels/gemm_sp_dgrad.hip
  if (g.mode == 2) return smi_sp_launch_wgrad(g, epi, grid, st);       // csrc/kernels/gemm_sp_wgrad.hip
  const bool w8 = smi_sp_waves() == 8;
  // the feature sets the models use (anything else: the caller falls back to gemm_f32):
  // fp32 output, or fp32 output + planes (the FFN hidden activation, consumed by linear2)
  if (g.relu > 1 || (!g.C && out != (SO_P | SO_M))) return -1;
#define SPF(E, O)                                                                                   \
  do {                                                                                              \
    if (t256 && smi_sp_tm() == 16) hipLaunchKernelGGL((gemm_sp256m_kernel<false, false, E, O>), grid, dim3(512), 0, st, g); \
    else if (t256) hipLaunchKernelGGL((gemm_sp256_kernel<false, false, E, O>), grid, dim3(512), 0, st, g); \
    else if (w8) hipLaunchKernelGGL((gemm_sp_kernel<8, false, false, E, O>), grid, dim3(512), 0, st, g); \
    else hipLaunchKernelGGL((gemm_sp_kernel<4, false, false, E, O>), grid, dim3(256), 0, st, g);    \
  } while (0)
#define SPF_OUT(E)                  \
  do {                              \
    if (out == SO_C) SPF(E, SO_C);  \
    else if (out == (SO_C | SO_P)) SPF(E, SO_C | SO_P); \
    else return -1;                 \
  } while (0)
  // the FFN hidden activation: planes for linear2's GEMMs + the positivity mask for its dgrad
  // epilogue, no fp32 tensor (sparkmi/ops/linear.py FFNFn)
  if (out == (SO_P | SO_M)) {
    if (epi == (SE_BIAS | SE_RELU | SE_DROP)) SPF(SE_BIAS | SE_RELU | SE_DROP, SO_P | SO_M);
    else if (epi == (SE_BIAS | SE_RELU)) SPF(SE_BIAS | SE_RELU, SO_P | SO_M);
    else return -1;
    SMI_CHECK_LAUNCH();
  }
  switch (epi) {
    case 0: SPF_OUT(0); break;
    case SE_BIAS: SPF_OUT(SE_BIAS); break;
    case SE_BIAS | SE_RELU: SPF_OUT(SE_BIAS | SE_RELU); break;
    case SE_BIAS | SE_RELU | SE_DROP: SPF_OUT(SE_BIAS | SE_RELU | SE_DROP); break;
    default: return -1;
  }
#undef SPF_OUT
#undef SPF
  SMI_CHECK_LAUNCH();
}
