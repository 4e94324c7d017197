// Split-plane fp32 GEMM, WGRAD instances: gW[N,K] += dY^T X and gb[N] += dY^T 1 over all M
// tokens (both operands k-major, ds_read_b64_tr_b16 fragments; the bias row sums are extra
// MFMAs of the dY planes against a ones fragment, exact products).  See smi_gemm_sp_impl.h.
#include "smi_gemm_sp_impl.h"

int smi_sp_wg_tm();


// Grouped weight-gradient GEMMs: every Linear's wgrad of a backward in ONE launch (queued by
// sparkmi/ops/_grad.py), no split-K: each 128 x 128 output tile reduces all T tokens and adds
// into its fp32 gradient (deterministic, no slabs, no atomics).  Problem e's tiles start at
// t0[e], a multiple of 8 (the XCD pattern of a standalone launch).
#define SPG_MAX 40
struct SpWgradGroup {
  const unsigned short* A[SPG_MAX]; const unsigned short* B[SPG_MAX];
  float* C[SPG_MAX]; float* bias[SPG_MAX];
  int lda[SPG_MAX], ldb[SPG_MAX], aps[SPG_MAX], bps[SPG_MAX];
  int n[SPG_MAX], k[SPG_MAX], T[SPG_MAX], a_bytes[SPG_MAX], b_bytes[SPG_MAX];
  int cb0[SPG_MAX], ncb[SPG_MAX];  // the column blocks [cb0, cb0 + ncb) of entry e this launch covers
  int t0[SPG_MAX + 1]; int count;
};

// 128-row form (gemm_sp_tm 128).  Column block 0 of an entry with a bias also reduces dY^T 1.
template <int NW, bool BIASG>
__global__ __launch_bounds__(64 * NW, 1) void gemm_sp_wgrad_group_kernel(SpWgradGroup gr) {
  __shared__ __attribute__((aligned(16))) unsigned short lds[SP_NS * SP_ST];
  const int t = blockIdx.x;
  int e = 0;
  while (e + 1 < gr.count && t >= gr.t0[e + 1]) ++e;  // uniform scan over <= SPG_MAX entries
  GemmSpArgs g{};
  g.mode = 2; g.A = gr.A[e]; g.lda = gr.lda[e]; g.aps = gr.aps[e]; g.B = gr.B[e]; g.ldb = gr.ldb[e];
  g.bps = gr.bps[e]; g.M = gr.n[e]; g.N = gr.k[e]; g.K = gr.T[e]; g.C = gr.C[e]; g.ldc = gr.k[e];
  g.beta_acc = 1; g.dscale = 1.f; g.bias_grad = BIASG ? gr.bias[e] : nullptr;
  g.a_bytes = gr.a_bytes[e]; g.b_bytes = gr.b_bytes[e];
  const int ncb = gr.ncb[e], ntn = (g.N + 127) / 128;
  const int nwg = ((g.M + 127) / 128) * ncb;
  const int lt = t - gr.t0[e];
  if (lt >= nwg) return;  // alignment padding
  const int l2 = sp_tile_remap(lt, nwg);
  const int tile = (l2 / ncb) * ntn + gr.cb0[e] + l2 % ncb;
  if (BIASG && g.bias_grad && gr.cb0[e] + l2 % ncb == 0) gemm_sp_tile<NW, true, true, SE_ACC, SO_C, true>(g, tile, lds);
  else gemm_sp_tile<NW, true, true, SE_ACC, SO_C, false>(g, tile, lds);
}

// main (non-bias) tiles on 256 x 128 tiles: n rows of gW in 256-row blocks
__global__ __launch_bounds__(512, 1) void gemm_sp_wgrad_group256_kernel(SpWgradGroup gr) {
  __shared__ __attribute__((aligned(16))) unsigned short lds[2 * SP_ST256];
  const int t = blockIdx.x;
  int e = 0;
  while (e + 1 < gr.count && t >= gr.t0[e + 1]) ++e;
  GemmSpArgs g{};
  g.mode = 2; g.A = gr.A[e]; g.lda = gr.lda[e]; g.aps = gr.aps[e]; g.B = gr.B[e]; g.ldb = gr.ldb[e];
  g.bps = gr.bps[e]; g.M = gr.n[e]; g.N = gr.k[e]; g.K = gr.T[e]; g.C = gr.C[e]; g.ldc = gr.k[e];
  g.beta_acc = 1; g.dscale = 1.f; g.bias_grad = gr.bias[e];
  g.a_bytes = gr.a_bytes[e]; g.b_bytes = gr.b_bytes[e];
  const int ncb = gr.ncb[e], ntn = (g.N + 127) / 128;
  const int nwg = ((g.M + 255) / 256) * ncb;
  const int lt = t - gr.t0[e];
  if (lt >= nwg) return;
  const int l2 = sp_tile_remap(lt, nwg);
  const int cb = gr.cb0[e] + l2 % ncb;
  // column block 0 of an entry with a bias also reduces dY^T 1 (SpBiasSum: 16 extra registers)
  if (g.bias_grad && cb == 0) gemm_sp_tile256<true, true, SE_ACC, SO_C, true>(g, (l2 / ncb) * ntn + cb, lds);
  else gemm_sp_tile256<true, true, SE_ACC, SO_C, false>(g, (l2 / ncb) * ntn + cb, lds);
}

// the same on the 16x16x32 MFMA (gemm_sp_tm 16, gemm_sp_tile256m)
__global__ __launch_bounds__(512, 1) void gemm_sp_wgrad_group256m_kernel(SpWgradGroup gr) {
  __shared__ __attribute__((aligned(16))) unsigned short lds[2 * SP_ST256];
  const int t = blockIdx.x;
  int e = 0;
  while (e + 1 < gr.count && t >= gr.t0[e + 1]) ++e;
  GemmSpArgs g{};
  g.mode = 2; g.A = gr.A[e]; g.lda = gr.lda[e]; g.aps = gr.aps[e]; g.B = gr.B[e]; g.ldb = gr.ldb[e];
  g.bps = gr.bps[e]; g.M = gr.n[e]; g.N = gr.k[e]; g.K = gr.T[e]; g.C = gr.C[e]; g.ldc = gr.k[e];
  g.beta_acc = 1; g.dscale = 1.f; g.bias_grad = gr.bias[e];
  g.a_bytes = gr.a_bytes[e]; g.b_bytes = gr.b_bytes[e];
  const int ncb = gr.ncb[e], ntn = (g.N + 127) / 128;
  const int nwg = ((g.M + 255) / 256) * ncb;
  const int lt = t - gr.t0[e];
  if (lt >= nwg) return;
  const int l2 = sp_tile_remap(lt, nwg);
  const int cb = gr.cb0[e] + l2 % ncb;
  if (g.bias_grad && cb == 0) gemm_sp_tile256m<true, true, SE_ACC, SO_C, true>(g, (l2 / ncb) * ntn + cb, lds);
  else gemm_sp_tile256m<true, true, SE_ACC, SO_C, false>(g, (l2 / ncb) * ntn + cb, lds);
}

// A_e: dY planes [3][T][lda] (plane stride aps), B_e: X planes [3][T][ldb]; C_e = gW [n][k] (row
// stride k), bias_e = gb [n] or null.
extern "C" int smi_gemm_sp_wgrad_group(const void* const* A, const long* lda, const long* aps, const void* const* B,
                                       const long* ldb, const long* bps, void* const* C, void* const* bias,
                                       const int* n, const int* k, const int* T, int count, hipStream_t st) {
  if (count < 1 || count > SPG_MAX) return -1;
  SpWgradGroup gm{}, gb{};
  int tm = 0, tb = 0, cm = 0, cb = 0;
  const int wtm = smi_sp_wg_tm();
  const bool t16 = wtm == 16, t256 = wtm == 256 || t16;
  for (int i = 0; i < count; ++i) {
    int ab = 0, bb = 0;
    if (!sp_operand_ok((const unsigned short*)A[i], lda[i], aps[i], n[i], n[i], true, 0, T[i], ab)) return -1;
    if (!sp_operand_ok((const unsigned short*)B[i], ldb[i], bps[i], k[i], k[i], true, 0, T[i], bb)) return -1;
    if (lda[i] > (1L << 30) || ldb[i] > (1L << 30) || aps[i] > (1L << 30) || bps[i] > (1L << 30) || !C[i] ||
        (k[i] & 3) || ((uintptr_t)C[i] & 15))
      return -1;
    const int ntn = (k[i] + 127) / 128;
    auto add = [&](SpWgradGroup& gr, int& c, int& tot, int cb0, int ncb, int rows) {
      const int nrb = (n[i] + rows - 1) / rows;
      gr.A[c] = (const unsigned short*)A[i]; gr.B[c] = (const unsigned short*)B[i];
      gr.C[c] = (float*)C[i]; gr.bias[c] = (float*)bias[i];
      gr.lda[c] = (int)lda[i]; gr.ldb[c] = (int)ldb[i]; gr.aps[c] = (int)aps[i]; gr.bps[c] = (int)bps[i];
      gr.n[c] = n[i]; gr.k[c] = k[i]; gr.T[c] = T[i]; gr.a_bytes[c] = ab; gr.b_bytes[c] = bb;
      gr.cb0[c] = cb0; gr.ncb[c] = ncb;
      gr.t0[c] = tot;
      tot += (nrb * ncb + 7) / 8 * 8;
      ++c;
    };
    add(gm, cm, tm, 0, ntn, t256 ? 256 : 128);
  }
  (void)gb; (void)tb; (void)cb;
  gm.t0[cm] = tm; gm.count = cm;
  if (t16) hipLaunchKernelGGL(gemm_sp_wgrad_group256m_kernel, dim3((unsigned)tm), dim3(512), 0, st, gm);
  else if (t256) hipLaunchKernelGGL(gemm_sp_wgrad_group256_kernel, dim3((unsigned)tm), dim3(512), 0, st, gm);
  else if (smi_sp_waves() == 8) hipLaunchKernelGGL((gemm_sp_wgrad_group_kernel<8, true>), dim3((unsigned)tm), dim3(512), 0, st, gm);
  else hipLaunchKernelGGL((gemm_sp_wgrad_group_kernel<4, true>), dim3((unsigned)tm), dim3(256), 0, st, gm);
  SMI_CHECK_LAUNCH();
}

// standalone form (a one-entry group): gw[N,K] += A^T B over all M tokens (+ bias row sums)
int smi_sp_launch_wgrad(const GemmSpArgs& g, int epi, dim3, hipStream_t st) {
  if (epi != SE_ACC || !g.C || g.ldc != g.N) return -1;  // accumulate into a contiguous fp32 gradient
  const void* A = g.A; const void* B = g.B; void* C = g.C; void* bias = g.bias_grad;
  return smi_gemm_sp_wgrad_group(&A, &g.lda, &g.aps, &B, &g.ldb, &g.bps, &C, &bias, &g.M, &g.N, &g.K, 1, st);
}
