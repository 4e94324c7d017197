// Per-phase cycle sums of the two-wave LSTM forward tick (-DLSTM_STAMPS diagnostic build),
// workgroup 0, lane 0 of each wave: [0] gates (LDS reads, packed FMAs, activations), [1] the
// barrier, [2] cell update + LDS writes + prefetch; plus the tick loop's s_memtime (shader clock)
// against s_memrealtime (100 MHz): the clock the recurrence actually runs at.
// build: hipcc --offload-arch=gfx950 -O3 -I csrc/include tools/probes/lstm_fwd_probe.hip csrc/kernels/embedding.hip
#define LSTM_STAMPS
#include "../../csrc/kernels/lstm.hip"
#include <cstdio>
#include <vector>

int main() {
  const int B = 32, T = 129, E = 32, H = 32, L = 2, C = 4, V = 1000;
  LSTMArgs a{};
  a.B = B; a.T = T; a.E = E; a.H = H; a.L = L; a.C = C; a.pad_idx = -1; a.V = V;
  auto zalloc = [](size_t n) { float* p; (void)hipMalloc(&p, n * 4); (void)hipMemset(p, 0, n * 4); return p; };
  long long* ids; (void)hipMalloc(&ids, (size_t)B * T * 8); (void)hipMemset(ids, 0, (size_t)B * T * 8);
  a.ids = ids; a.emb = zalloc((size_t)V * E);
  for (int l = 0; l < L; ++l) {
    const int In = l == 0 ? E : H;
    a.w_ih[l] = zalloc(4 * H * In); a.w_hh[l] = zalloc(4 * H * H); a.b_ih[l] = zalloc(4 * H); a.b_hh[l] = zalloc(4 * H);
  }
  a.w_fc = zalloc(C * H); a.b_fc = zalloc(C);
  a.pred = zalloc((size_t)B * T * C); a.hn = zalloc(L * B * H); a.cn = zalloc(L * B * H);
  a.ws = zalloc((size_t)B * L * T * 6 * H);
  for (int it = 0; it < 3; ++it) smi_lstm(&a, 0, 0);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> z(32, 0ull);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(lstm_stamps), z.data(), 32 * 8);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(lstm_rt), z.data(), 4 * 8);
  const int R = 20;
  for (int it = 0; it < R; ++it) smi_lstm(&a, 0, 0);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> st(32), rt(4);
  (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(lstm_stamps), 32 * 8);
  (void)hipMemcpyFromSymbol(rt.data(), HIP_SYMBOL(lstm_rt), 4 * 8);
  const char* nm[5] = {"gates", "barrier", "cell+writes", "stamps", "flush"};
  for (int w = 0; w < 2; ++w) {
    printf("wave %d:", w);
    for (int i = 0; i < 5; ++i) printf("  %s %.0f", nm[i], (double)st[w * 8 + i] / R / (T + L - 1));
    printf("  (cycles per tick)\n");
  }
  const double us = (double)rt[0] / R / 100.0, cyc = (double)rt[2] / R;
  printf("tick loop: %.1f us, %.0f shader cycles -> %.2f GHz, %.0f cycles / %.3f us per tick\n", us, cyc,
         cyc / us / 1000.0, cyc / (T + L - 1), us / (T + L - 1));
  // backward recurrence kernel alone (last-step dpred), stamped: slots 2 + wave
  {
    float *dpred = zalloc((size_t)B * C), *wsda = zalloc((size_t)B * L * T * 4 * H);
    a.dpred = dpred; a.dpred_last = 1; a.ws_da = wsda;
    for (int it = 0; it < 3; ++it) hipLaunchKernelGGL((lstm_bwd_w2_kernel<32, 32, 4>), dim3(B), dim3(128), 0, 0, a);
    (void)hipDeviceSynchronize();
    (void)hipMemcpyToSymbol(HIP_SYMBOL(lstm_stamps), z.data(), 32 * 8);
    for (int it = 0; it < R; ++it) hipLaunchKernelGGL((lstm_bwd_w2_kernel<32, 32, 4>), dim3(B), dim3(128), 0, 0, a);
    (void)hipDeviceSynchronize();
    (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(lstm_stamps), 32 * 8);
    const char* bn[4] = {"flush", "load+cell", "prep+product", "barrier"};
    const int bi[4] = {3, 5, 6, 7};
    for (int w = 0; w < 2; ++w) {
      printf("bwd wave %d:", w);
      for (int i = 0; i < 4; ++i) printf("  %s %.0f", bn[i], (double)st[(2 + w) * 8 + bi[i]] / R / (T + L - 1));
      printf("  (cycles per tick)\n");
    }
    hipEvent_t f0, f1; (void)hipEventCreate(&f0); (void)hipEventCreate(&f1);
    (void)hipEventRecord(f0);
    for (int it = 0; it < 20; ++it) hipLaunchKernelGGL((lstm_bwd_w2_kernel<32, 32, 4>), dim3(B), dim3(128), 0, 0, a);
    (void)hipEventRecord(f1); (void)hipEventSynchronize(f1);
    float bms; (void)hipEventElapsedTime(&bms, f0, f1);
    printf("bwd recurrence: %.1f us per call\n", bms * 1000 / 20);
  }
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  for (int it = 0; it < 20; ++it) smi_lstm(&a, 0, 0);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  printf("fwd: %.1f us per call\n", ms * 1000 / 20);
  return 0;
}
