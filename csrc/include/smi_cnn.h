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
  // fused SGD step (cnn_kernel's tail, one launch per training step): the per-image slabs are
  // summed in two ticketed levels (groups of CNN_GRP images, then the groups) and the LAST
  // workgroup applies p -= lr * g to the parameters (+ their bf16 shadows), the mean loss and the
  // step counter.  part: [ceil(B / CNN_GRP)][P] group sums; tick: CNN_GRP + 2 zeroed counters
  // (re-armed by the kernel), owned by the model.
  int fused;
  int wstage;  // set by the launcher: the bf16 convs read LDS-staged weights (when they fit)
  float* part; unsigned* tick; const float* lr; float* step;
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
#ifndef CNN_GRP
#define CNN_GRP 8
#endif
static_assert(CNN_GRP >= 1 && CNN_GRP <= 32, "the model owns CNN_GRP + 2 <= 34 tickets");
