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
};
