// Where the staged-plane fp32 attention forward spends its time (-DATTN_STAMPS diagnostic build of
// csrc/kernels/attention_f32.hip): per-wave shader-clock sums of each phase of the chunk loop,
// averaged per wave and per chunk, plus the s_memrealtime spread of wave starts / ends (dispatch
// ramp, drain).  Flagship self-attention shape: B 32, S 256, H 8, hd 64, mode 1, packed qkv rows,
// O written with its split planes.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc/include tools/probes/attn_fwd_probe.hip -o tools/probes/attn_fwd_probe
#ifndef NO_STAMPS
#define ATTN_STAMPS
#endif
#include "../../csrc/kernels/attention_f32.hip"
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#ifdef ATTN_STAMPS
#define STAMPED "stamped"
#else
#define STAMPED "plain"
#endif
extern "C" int smi_gemm_f32_algo(int) { return 1; }  // the split-product path

int main() {
  const int B = 32, S = 256, H = 8, D = 64, W = 3 * H * D;
  std::vector<float> hq((size_t)B * S * W);
  unsigned s = 12345u;
  for (auto& x : hq) { s = s * 1664525u + 1013904223u; x = ((s >> 8) * (1.0f / 16777216.0f) - 0.5f) * 2.f; }
  float *qkv, *o, *lse; unsigned short* op;
  (void)hipMalloc(&qkv, hq.size() * 4);
  (void)hipMemcpy(qkv, hq.data(), hq.size() * 4, hipMemcpyHostToDevice);
  (void)hipMalloc(&o, (size_t)B * S * H * D * 4);
  (void)hipMalloc(&op, (size_t)3 * B * S * H * D * 2);
  (void)hipMalloc(&lse, (size_t)B * H * S * 4);
  AttnF32Args a{};
  a.q = qkv; a.k = qkv + H * D; a.v = qkv + 2 * H * D;
  a.q_ss = a.k_ss = a.v_ss = W; a.q_sh = a.k_sh = a.v_sh = D; a.q_sb = a.k_sb = a.v_sb = (long)S * W;
  a.o = o; a.o_ss = H * D; a.o_sh = D; a.o_sb = (long)S * H * D;
  a.lse = lse; a.B = B; a.H = H; a.Sq = S; a.Sk = S; a.mode = 1;
  a.scale_log2 = 1.4426950408889634f / 8.f; a.scale = 1.f / 8.f;
  a.op = op; a.op_ps = (long)B * S * H * D;
  for (int it = 0; it < 3; ++it)
    if (smi_attn_f32_fwd(&a, 0)) { printf("launch failed\n"); return 1; }
  (void)hipDeviceSynchronize();
#ifdef ATTN_STAMPS
  const int R = 1;  // per-wave slots of the last run
  (void)smi_attn_f32_fwd(&a, 0);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> sw(8 * 4096), st(8, 0ull), rt(2 * 4096);
  (void)hipMemcpyFromSymbol(sw.data(), HIP_SYMBOL(attn_stamps), 8 * 4096 * 8);
  (void)hipMemcpyFromSymbol(rt.data(), HIP_SYMBOL(attn_wave_rt), 2 * 4096 * 8);  // last run
  const int waves = B * H * (S / 128) * 4, chunks = S / 32;
  for (int wv = 0; wv < waves; ++wv)
    for (int i = 0; i < 8; ++i) st[i] += sw[8 * wv + i];
  // lifetime distribution (shader cycles)
  std::vector<unsigned long long> lt(waves);
  for (int wv = 0; wv < waves; ++wv) lt[wv] = sw[8 * wv + 7];
  {
    double xs[8] = {0}, xe[8] = {0}, qx[2] = {0};
    for (int wv = 0; wv < waves; ++wv) {
      const int wg = wv / 4;  // linear workgroup id; blockIdx.x = wg % 2 (query half)
      xs[wg % 8] += (double)sw[8 * wv + 7] / (waves / 8);
      xe[wg % 8] += (double)(rt[2 * wv + 1] - rt[2 * wv]) / 100.0 / (waves / 8);
      qx[wg % 2] += (double)sw[8 * wv + 7] / (waves / 2);
    }
    printf("mean lifetime by XCD (wg %% 8), cycles / us:");
    for (int x = 0; x < 8; ++x) printf(" %.0f/%.1f", xs[x], xe[x]);
    printf("\nmean lifetime by query half: %.0f %.0f\n", qx[0], qx[1]);
  }
  std::sort(lt.begin(), lt.end());
  printf("wave lifetime cycles: min %llu p10 %llu p50 %llu p90 %llu max %llu\n", lt[0], lt[waves / 10], lt[waves / 2],
         lt[waves * 9 / 10], lt[waves - 1]);
  const double pw = 1.0 / ((double)R * waves), pc = pw / chunks;
  const char* nm[8] = {"prologue", "load issue", "S+softmax", "PV", "stage store", "barrier", "epilogue", "lifetime"};
  for (int i = 0; i < 8; ++i)
    printf("%-12s %8.0f cycles/%s\n", nm[i], st[i] * ((i >= 1 && i <= 5) ? pc : pw), (i >= 1 && i <= 5) ? "chunk" : "wave ");
  unsigned long long s0 = ~0ull, s1 = 0, e0 = ~0ull, e1 = 0;
  for (int i = 0; i < waves; ++i) {
    s0 = std::min(s0, rt[2 * i]); s1 = std::max(s1, rt[2 * i]);
    e0 = std::min(e0, rt[2 * i + 1]); e1 = std::max(e1, rt[2 * i + 1]);
  }
  printf("wave starts %.2f..%.2f us, ends %.2f..%.2f us (100 MHz realtime, from the first start)\n", 0.0,
         (s1 - s0) / 100.0, (e0 - s0) / 100.0, (e1 - s0) / 100.0);
#endif
  hipEvent_t v0, v1; (void)hipEventCreate(&v0); (void)hipEventCreate(&v1);
  for (int rep = 0; rep < 3; ++rep)
    for (int nw8 = 0; nw8 < 2; ++nw8) {
      smi_attn_fwd8(nw8);
      for (int it = 0; it < 3; ++it) (void)smi_attn_f32_fwd(&a, 0);
      (void)hipEventRecord(v0);
      for (int it = 0; it < 20; ++it) (void)smi_attn_f32_fwd(&a, 0);
      (void)hipEventRecord(v1); (void)hipEventSynchronize(v1);
      float ms; (void)hipEventElapsedTime(&ms, v0, v1);
      printf("fwd %d-wave (%s build): %.1f us per call\n", nw8 ? 8 : 4, STAMPED, ms * 1000 / 20);
    }
  smi_attn_fwd8(1);
  return 0;
}
