// Where the single-pass fp32 attention backward (attn_sp_bwd8_kernel) spends its time
// (-DATTN_STAMPS diagnostic build of csrc/kernels/attention_f32.hip): per-wave shader-clock sums of
// each phase of the chunk loop, averaged per wave and per chunk.  Flagship self-attention shape:
// B 32, S 256, H 8, hd 64, mode 1, packed qkv rows, gradients written as planes only (the model's
// setting).  Also times the plain kernel and the dQ + dK/dV pair with events (NO_STAMPS build).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc/include tools/probes/attn_bwd_probe.hip -o tools/probes/attn_bwd_probe
#ifndef NO_STAMPS
#define ATTN_STAMPS
#endif
#include "../../csrc/kernels/attention_f32.hip"
#include <algorithm>
#include <cstdio>
#include <vector>

extern "C" int smi_gemm_f32_algo(int) { return 1; }  // the split-product path

int main() {
  const int B = 32, S = 256, H = 8, D = 64, W = 3 * H * D;
  const size_t nq = (size_t)B * S * W, no = (size_t)B * S * H * D;
  std::vector<float> hq(nq), hd(no);
  unsigned s = 12345u;
  for (auto& x : hq) { s = s * 1664525u + 1013904223u; x = ((s >> 8) * (1.0f / 16777216.0f) - 0.5f) * 2.f; }
  for (auto& x : hd) { s = s * 1664525u + 1013904223u; x = ((s >> 8) * (1.0f / 16777216.0f) - 0.5f) * 2.f; }
  float *qkv, *o, *lse, *dout, *delta, *dqkv;
  unsigned short *op, *gp;
  (void)hipMalloc(&qkv, nq * 4);
  (void)hipMemcpy(qkv, hq.data(), nq * 4, hipMemcpyHostToDevice);
  (void)hipMalloc(&dout, no * 4);
  (void)hipMemcpy(dout, hd.data(), no * 4, hipMemcpyHostToDevice);
  (void)hipMalloc(&o, no * 4);
  (void)hipMalloc(&op, 3 * no * 2);
  (void)hipMalloc(&lse, (size_t)B * H * S * 4);
  (void)hipMalloc(&delta, (size_t)B * H * S * 4);
  (void)hipMalloc(&dqkv, nq * 4);
  (void)hipMalloc(&gp, 3 * nq * 2);
  AttnF32Args a{};
  a.q = qkv; a.k = qkv + H * D; a.v = qkv + 2 * H * D;
  a.q_ss = a.k_ss = a.v_ss = W; a.q_sh = a.k_sh = a.v_sh = D; a.q_sb = a.k_sb = a.v_sb = (long)S * W;
  a.o = o; a.o_ss = H * D; a.o_sh = D; a.o_sb = (long)S * H * D;
  a.lse = lse; a.B = B; a.H = H; a.Sq = S; a.Sk = S; a.mode = 1;
  a.scale_log2 = 1.4426950408889634f / 8.f; a.scale = 1.f / 8.f;
  a.op = op; a.op_ps = (long)no;
  if (smi_attn_f32_fwd(&a, 0)) { printf("fwd launch failed\n"); return 1; }
  a.op = nullptr;
  a.dout = dout; a.delta = delta;
  a.dq = dqkv; a.dk = dqkv + H * D; a.dv = dqkv + 2 * H * D;
  a.dqp = gp; a.dkp = gp + H * D; a.dvp = gp + 2 * H * D; a.dq_ps = a.dkv_ps = (long)nq;
  a.no_f32_grad = 1;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int pass = 0; pass < 2; ++pass) {
    smi_attn_bwd1(pass == 0 ? 1 : 0);
    for (int it = 0; it < 5; ++it) (void)smi_attn_f32_bwd(&a, 0);
    (void)hipEventRecord(e0, 0);
    const int n = 50;
    for (int it = 0; it < n; ++it) (void)smi_attn_f32_bwd(&a, 0);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%s backward: %.1f us per call\n", pass == 0 ? "single-pass" : "dQ + dK/dV pair", 1000.f * ms / n);
  }
  smi_attn_bwd1(1);
#ifdef ATTN_STAMPS
  (void)smi_attn_f32_bwd(&a, 0);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> sw(8 * 4096), st(8, 0ull);
  (void)hipMemcpyFromSymbol(sw.data(), HIP_SYMBOL(attn_stamps), 8 * 4096 * 8);
  const int waves = B * H * 8, chunks = S / 32;
  for (int wv = 0; wv < waves; ++wv)
    for (int i = 0; i < 8; ++i) st[i] += sw[8 * wv + i];
  std::vector<unsigned long long> lt(waves);
  for (int wv = 0; wv < waves; ++wv) lt[wv] = sw[8 * wv + 7];
  std::sort(lt.begin(), lt.end());
  printf("wave lifetime cycles: min %llu p50 %llu max %llu\n", lt[0], lt[waves / 2], lt[waves - 1]);
  const double pw = 1.0 / waves, pc = pw / chunks;
  const char* nm[8] = {"prologue", "S,dP,P,dS", "dV,dK issue", "barrier 1", "dQ phase", "stage store", "barrier 2",
                       "lifetime"};
  double loop = 0;
  for (int i = 0; i < 8; ++i) {
    const bool per_chunk = i >= 1 && i <= 6;
    if (per_chunk) loop += st[i] * pc;
    printf("%-12s %8.0f cycles/%s\n", nm[i], st[i] * (per_chunk ? pc : pw), per_chunk ? "chunk" : "wave ");
  }
  printf("loop per chunk %.0f cycles; epilogue ~%.0f cycles/wave\n", loop,
         st[7] * pw - st[0] * pw - loop * chunks);
#endif
  return 0;
}
