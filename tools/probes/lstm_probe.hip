// Per-phase cycle sums of the LSTM BPTT kernel (-DLSTM_STAMPS diagnostic build), workgroup 0,
// lane 0 of each wave: [0] cell phase, [1] barrier A wait, [2] gradient/transposed phase,
// [3] barrier B wait (summed over ticks), [4] whole tick loop, [5] tail phases.
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
    a.g_w_ih[l] = zalloc(4 * H * In); a.g_w_hh[l] = zalloc(4 * H * H); a.g_b_ih[l] = zalloc(4 * H); a.g_b_hh[l] = zalloc(4 * H);
  }
  a.w_fc = zalloc(C * H); a.b_fc = zalloc(C); a.g_w_fc = zalloc(C * H); a.g_b_fc = zalloc(C);
  a.pred = zalloc((size_t)B * T * C); a.hn = zalloc(L * B * H); a.cn = zalloc(L * B * H);
  a.ws = zalloc((size_t)B * L * T * 6 * H); a.ws_da = zalloc((size_t)B * L * T * 4 * H);
  a.dpred = zalloc((size_t)B * T * C); a.g_emb = zalloc((size_t)V * E);
  a.g_slab = zalloc((size_t)smi_lstm_slab_floats(B, E, H, L, C)); a.g_xe = zalloc((size_t)B * T * E);
  void* ews; (void)hipMalloc(&ews, 1 << 24); a.emb_ws = ews;
  for (int it = 0; it < 3; ++it) { smi_lstm(&a, 0, 0); smi_lstm(&a, 1, 0); }
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> z(32, 0ull);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(lstm_stamps), z.data(), 32 * 8);
  const int R = 5;
  for (int it = 0; it < R; ++it) smi_lstm(&a, 1, 0);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> st(32);
  (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(lstm_stamps), 32 * 8);
  const char* nm[6] = {"cell phase", "barrier A wait", "grad phase", "barrier B wait", "tick loop", "tail"};
  for (int w = 0; w < 4; ++w) {
    printf("wave %d:", w);
    for (int i = 0; i < 6; ++i) printf("  %s %.0f", nm[i], (double)st[w * 8 + i] / R);
    printf("  (cycles per call)\n");
  }
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  for (int it = 0; it < 20; ++it) smi_lstm(&a, 1, 0);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  printf("bwd (incl. reduce + emb): %.1f us per call\n", ms * 1000 / 20);
  return 0;
}
