// Argument block shared by csrc/kernels/mlp.hip and csrc/bindings.cpp.
#pragma once
#define MLP_MAXL 6
#define MLP_MAXW 32
#define MLP_ACT_STRIDE (MLP_MAXW * (MLP_MAXL + 1))

struct MLPArgs {
  const float* x;            // [n, dims[0]] row-major
  const long long* y;        // [n] class index
  const float* row_w;        // [n] per-row loss weight or null (-> 1/n)
  int n;
  int nlayers;
  int dims[MLP_MAXL + 1];
  const float* W[MLP_MAXL];  // torch layout [out, in]
  const float* b[MLP_MAXL];
  float* gW[MLP_MAXL];
  float* gb[MLP_MAXL];
  float* logits;             // optional [n, C]
  float* loss;               // scalar, written (mean loss of the whole batch)
  const float* dloss;        // scalar upstream gradient (bwd)
  int act;                   // 1 relu, 2 sigmoid
  // deterministic cross-block reduction (grid > 1): per-block partials [grid][total + 1] and a
  // zeroed ticket word that the last block re-arms
  float* ws;
  unsigned* ticket;
  int accumulate;            // bwd: gW/gb += gradient (else =)
  // fused SGD (mode 2): params -= lr * gscale * gradient, step += 1; gradients are not stored
  const float* lr;
  float* step;
  float gscale;
};
#define MLP_MAX_GRID 256

// consecutive fused SGD steps in one launch (smi_mlp_steps): step t's batch and loss
#define MLP_MAX_STEPS 32
struct MLPSteps {
  int n;
  const float* x[MLP_MAX_STEPS];
  const long long* y[MLP_MAX_STEPS];
  float* loss[MLP_MAX_STEPS];
  float* loss_sum;  // optional: the step losses summed in step order (the metrics' group sum)
  // index mode (perm != null): x[t] / y[t] are the whole dataset and step t's row i is dataset row
  // perm[(cursor + t) * B + i] (the shuffled batch gather inside the kernel); cursor += n at the end
  const long long* perm;
  int* cursor;
  int B;
};

