// Per-phase timing of the fused CNN kernel (one workgroup per image): s_memtime after every
// barrier (-DCNN_STAMPS diagnostic build), averaged over images.
#ifndef CNN_PROBE_NOSTAMP  // -DCNN_PROBE_NOSTAMP: the production kernel, launch timing only
#define CNN_STAMPS
#endif
#ifndef CNN_SRC  // -DCNN_SRC='"path"': another version of the kernel (tools/cnn_ab.sh)
#define CNN_SRC "../../csrc/kernels/cnn.hip"
#endif
#include CNN_SRC
#include <cstdio>
#include <vector>

int main(int argc, char** argv) {
  const int B = 32, C = 10, CI = 1, NC = 10;
  CNNArgs g{};
  g.B = B; g.cin = CI; g.C = C; g.classes = NC; g.x_u8 = 1; g.x_scale = 1.f / 255.f; g.train = 1; g.loss_scale = 1.f / B; g.bf16 = argc > 1;
  unsigned char* x; long long* y; float *w[5], *b[5], *slab, *rl, *loss; int* pred;
  (void)hipMalloc(&x, B * 784);
  {  // random pixels and weights (zeros run at a higher clock and leave every ReLU off)
    std::vector<unsigned char> hx(B * 784);
    unsigned r = 12345u;
    for (auto& v : hx) { r = r * 1664525u + 1013904223u; v = (unsigned char)(r >> 24); }
    (void)hipMemcpy(x, hx.data(), hx.size(), hipMemcpyHostToDevice);
  }
  (void)hipMalloc(&y, B * 8); (void)hipMemset(y, 0, B * 8);
  const int sz[5] = {C * CI * 9, C * C * 9, C * C * 9, C * C * 9, NC * C * 49};
  int off = 0;
  const int bs[10] = {C * CI * 9, C, C * C * 9, C, C * C * 9, C, C * C * 9, C, NC * C * 49, NC};
  for (int i = 0; i < 10; ++i) { g.off[i] = off; off += bs[i]; }
  g.P = off;
  for (int i = 0; i < 5; ++i) {
    (void)hipMalloc(&w[i], sz[i] * 4);
    {
      std::vector<float> hw(sz[i]);
      unsigned r = 777u + i;
      for (auto& v : hw) { r = r * 1664525u + 1013904223u; v = ((float)(r >> 8) / 16777216.f - 0.5f) * 0.3f; }
      (void)hipMemcpy(w[i], hw.data(), hw.size() * 4, hipMemcpyHostToDevice);
    }
    (void)hipMalloc(&b[i], 64); (void)hipMemset(b[i], 0, 64);
    g.w[i] = w[i]; g.b[i] = b[i];
  }
  (void)hipMalloc(&slab, (size_t)B * g.P * 4); (void)hipMalloc(&rl, B * 4); (void)hipMalloc(&loss, 4); (void)hipMalloc(&pred, B * 4);
  g.x = x; g.y = y; g.slab = slab; g.row_loss = rl; g.loss = loss; g.pred = pred;
  if (argc > 2) {  // the fused single-executor SGD step (ticketed slab reduction + SGD in the tail)
    float *lr, *step; unsigned* tick;
#ifndef CNN_TICKS  // a kernel version from before the one-ticket tail (tools/cnn_ab.sh REV)
#define CNN_TICKS (CNN_GRP + 2)
    (void)hipMalloc(&g.part, (size_t)((B + CNN_GRP - 1) / CNN_GRP) * g.P * 4);
#endif
    (void)hipMalloc(&tick, (CNN_TICKS + 3 * B) * 4); (void)hipMemset(tick, 0, (CNN_TICKS + 3 * B) * 4);
    (void)hipMalloc(&lr, 4); (void)hipMemset(lr, 0, 4);
    (void)hipMalloc(&step, 4); (void)hipMemset(step, 0, 4);
    g.fused = 1; g.tick = tick; g.lr = lr; g.step = step;
    if (argc > 3) {  // the weight-gradient helper workgroups (CNNArgs::hand)
      (void)hipMalloc(&g.hand, (size_t)B * smi_cnn_hand_floats(C) * 4);
      g.hflag = tick + CNN_TICKS;
    }
  }
  printf("mode: %s%s%s\n", g.bf16 ? "bf16" : "fp32", g.fused ? " fused" : "", g.hand ? " helpers" : "");
  for (int it = 0; it < 20; ++it) smi_cnn(&g, 0);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> st(256 * 32);
#ifdef CNN_STAMPS
  (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(cnn_stamps), st.size() * 8);
#endif
  int nph = 0;
  for (int i = 0; i < 21; ++i) if (st[i]) nph = i + 1;
  printf("phases %d\n", nph);
  for (int p = 1, q = 0; p < nph; ++p) {  // consecutive stamps that were set (paths skip some)
    if (!st[p]) continue;
    double d = 0;
    for (int im = 0; im < B; ++im) d += (double)(st[im * 32 + p] - st[im * 32 + q]);
    printf("phase %2d -> %2d: %8.0f ticks\n", q, p, d / B);
    q = p;
  }
  // conv_wgrad sub-stamps (slot sb: wave 0's units done, sb+1: all units done; phase end = combine done)
  const int sub[3][3] = {{21, 17, 18}, {23, 19, 20}, {25, 12, 13}};
  const char* nm[3] = {"conv2 wgrad", "conv1 wgrad", "conv4 wgrad"};
  if (g.bf16) {  // bf16 build: slot 24 / 25 = conv2 forward / dgrad tables ready (conv_mfma sb)
    const int tb[2][3] = {{24, 2, 3}, {25, 18, 19}};
    const char* tn[2] = {"conv2 fwd", "conv2 dgrad"};
    for (int k = 0; k < 2; ++k) {
      double a = 0, b = 0;
      for (int im = 0; im < B; ++im) {
        a += (double)(st[im * 32 + tb[k][0]] - st[im * 32 + tb[k][1]]);
        b += (double)(st[im * 32 + tb[k][2]] - st[im * 32 + tb[k][0]]);
      }
      printf("%s: tables %8.0f, tiles + barrier %8.0f ticks\n", tn[k], a / B, b / B);
    }
  }
  for (int k = 0; k < 3 && !g.bf16; ++k) {
    const int sb = sub[k][0], p0 = sub[k][1], p1 = sub[k][2];
    if (!st[sb]) continue;
    double u0 = 0, ua = 0, cb = 0;
    for (int im = 0; im < B; ++im) {
      u0 += (double)(st[im * 32 + sb] - st[im * 32 + p0]);
      ua += (double)(st[im * 32 + sb + 1] - st[im * 32 + p0]);
      cb += (double)(st[im * 32 + p1] - st[im * 32 + sb + 1]);
    }
    printf("%s: wave0 units %8.0f, all units %8.0f, combine+write %8.0f ticks\n", nm[k], u0 / B, ua / B, cb / B);
  }
  // fused tail stamps (slots 26-29: group sum start / done, final start / SGD done), relative to
  // the same workgroup's body end (slot 20; s_memtime is per-XCD, so only same-WG differences)
  for (int im = 0; im < B; ++im)
    for (int k = (g.bf16 ? 21 : 26); k < 31; ++k)
      if (st[im * 32 + k]) printf("img %2d slot %d: %+8lld ticks after its body end\n", im, k,
                                  (long long)(st[im * 32 + k] - st[im * 32 + 20]));
#ifdef CNN_STAMPS
  if (g.hand) {  // global-clock timeline (10 ns ticks) from the kernel's earliest start
    std::vector<unsigned long long> rt(256 * 8);
    (void)hipMemcpyFromSymbol(rt.data(), HIP_SYMBOL(cnn_rstamps), rt.size() * 8);
    unsigned long long t0 = ~0ull;
    for (int w = 0; w < (1 + CNN_HELPERS) * B; ++w) if (rt[w * 8] && rt[w * 8] < t0) t0 = rt[w * 8];
    auto avg = [&](int w0, int w1, int step, int k) {
      double s = 0; int n = 0;
      for (int w = w0; w < w1; w += step) if (rt[w * 8 + k]) { s += (double)(rt[w * 8 + k] - t0) * 10.0 / 1000.0; ++n; }
      return n ? s / n : -1.0;
    };
    printf("image wg (us from kernel start): start %.2f, conv2 handed over %.2f, body done %.2f\n", avg(0, B, 1, 0),
           avg(0, B, 1, 1), avg(0, B, 1, 4));
    const int HW = CNN_HELPERS, NW = (1 + CNN_HELPERS) * B;
    for (int j = 0; j < HW; ++j)
      printf("helper %s %d: start %.2f, flag %.2f, loaded %.2f, wgrad %.2f, done %.2f\n", j == 0 ? "conv4" : j == 1 ? "conv3" : "conv2",
             j, avg(B + j, NW, HW, 0), avg(B + j, NW, HW, 1), avg(B + j, NW, HW, 2), avg(B + j, NW, HW, 3), avg(B + j, NW, HW, 4));
    // tail stamps of THIS launch only (earlier launches' last workgroups left older values)
    auto cur = [&](unsigned long long v) { return v >= t0 && v < t0 + 100000ull; };
    unsigned long long tl = 0;  // the last workgroup to finish its image / helper work
    for (int w = 0; w < (1 + CNN_HELPERS) * B; ++w) if (cur(rt[w * 8 + 4]) && rt[w * 8 + 4] > tl) tl = rt[w * 8 + 4];
    printf("last workgroup done: %.2f us\n", (double)(tl - t0) * 0.01);
    for (int k = 5; k < 8; ++k) {
      const char* kn = k == 5 ? "slice ticket" : (k == 6 ? "slice start" : "slice done");
      printf("tail %s:", kn);
      for (int w = 0; w < (1 + CNN_HELPERS) * B; ++w)
        if (cur(rt[w * 8 + k])) printf(" %.2f", (double)(rt[w * 8 + k] - t0) * 0.01);
      printf(" us\n");
    }
    // the level-2 slices' phases (same-workgroup s_memtime differences)
    for (int w = 0; w < (1 + CNN_HELPERS) * B; ++w) {
      if (!cur(rt[w * 8 + 6])) continue;
      const unsigned long long* q = &st[w * 32];
      printf("slice wg %3d: loads %lld, conv apply %lld, fc %lld, bias %lld ticks\n", w,
             (long long)(q[21] - q[28]), (long long)(q[22] - q[21]), (long long)(q[23] - q[30]),
             (long long)(q[29] - q[23]));
    }
  }
#endif
  double tot = 0;
  for (int im = 0; im < B; ++im) tot += (double)(st[im * 32 + nph - 1] - st[im * 32]);
  printf("total %8.0f ticks\n", tot / B);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  for (int it = 0; it < 50; ++it) smi_cnn(&g, 0);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  printf("kernel+loss: %.1f us per call\n", ms * 1000 / 50);
  // the same launches captured in one graph (the bench's replay: no host launch gaps)
  hipStream_t cs; (void)hipStreamCreateWithFlags(&cs, hipStreamNonBlocking);
  hipGraph_t gr; hipGraphExec_t ge;
  (void)hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed);
  for (int it = 0; it < 50; ++it) smi_cnn(&g, cs);
  (void)hipStreamEndCapture(cs, &gr);
  (void)hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
  // ~0.2 s of replays first: the clocks ramp up under sustained load (a cold first run reads slow)
  for (int r = 0; r < 80; ++r) (void)hipGraphLaunch(ge, cs);
  (void)hipStreamSynchronize(cs);
  float best = 1e9f;
  for (int r = 0; r < 20; ++r) {
    (void)hipEventRecord(e0, cs); (void)hipGraphLaunch(ge, cs); (void)hipEventRecord(e1, cs);
    (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  printf("graph: %.2f us per step (best of 20 x 50, after a warm-up)\n", best * 1000 / 50);
  return 0;
}
