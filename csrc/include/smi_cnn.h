// Argument block shared by csrc/kernels/cnn.hip and csrc/bindings.cpp.
#pragma once
#define CNN_MAXC 16
struct CNNArgs {
  const void* x; int x_u8; float x_scale;   // images [B, cin, 28, 28] (uint8 scaled, or fp32)
  const long long* y;                       // labels [B] (null for inference)
  int B, cin, C, classes;
  const float* w[5]; const float* b[5];     // conv1..4 [C,cin|C,3,3], fc [classes, C*49]
  float* gw[5]; float* gb[5];               // gradient destinations (reduce kernel)
  float* slab; int P; int off[10];          // per-image packed gradients [B][P]
  float* row_loss; int* pred; float* logits; float* loss;
  float loss_scale;                          // 1/B for a mean loss
  const float* dloss;                        // upstream grad of the loss (reduce kernel)
  int train;
  int bf16;                                  // convolutions on bf16 matrix cores (fp32 accumulate)
  // fused SGD step (cnn_kernel's tail, one launch per training step): the last min(CNN_NSL, B)
  // workgroups to finish (one ticket counter) become slice workgroups; the slices sum the
  // per-image slabs of their part of the parameters and apply p -= lr * g (+ the bf16 shadows);
  // the last one writes the mean loss and the step counter.  tick: CNN_TICKS zeroed counters
  // (re-armed by the kernel), owned by the model, followed by the helpers' flags (hflag).
  int fused;
  int wstage;  // set by the launcher: the bf16 convs read LDS-staged weights (when they fit)
  unsigned* tick; const float* lr; float* step;
  unsigned short* shadow[10];                // per-parameter bf16 shadows (slab order) or null
  // INDEX mode (fused steps only; sparkmi/data/dataset.py DeviceLoader fixed=True): x / y are the
  // whole HBM-resident dataset and image i of the batch is row perm[cursor[0] * B + i]; the step's
  // last workgroup advances the device cursor — the shuffled batch gather inside the step kernel
  const long long* perm; int* cursor;
  // WEIGHT-GRADIENT HELPERS (fused steps; hand != null): 3 extra workgroups per image compute the
  // conv4 / conv3 / conv2 weight gradients from (dz, input) plane sets the image's workgroup hands
  // over through `hand` ([B][cnn_hand_floats(C)]); hflag: 3 * B zeroed flags (re-armed by the
  // helpers) — the image's workgroup runs the dgrad chain meanwhile
  float* hand; unsigned* hflag;
};
#ifndef CNN_NSL
#define CNN_NSL 16  // fused tail: at most this many parameter slices (slice workgroups)
#endif
#define CNN_TICKS 2    // the tail's ticket and departure counters
#define CNN_MAXB 64    // fused steps: batch limit (the model's counter block: CNN_TICKS + 3 B <= 226)
static_assert(CNN_NSL >= 1 && CNN_TICKS + 3 * CNN_MAXB <= 226, "sparkmi/models/cnn.py owns 226 counters");
