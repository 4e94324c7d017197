// Argument blocks shared by csrc/kernels/attention.hip and csrc/bindings.cpp.
#pragma once
struct AttnFwdArgs {
  const unsigned short* q; const unsigned short* k; const unsigned short* v;
  long q_sb, q_ss, q_sh, k_sb, k_ss, k_sh, v_sb, v_ss, v_sh;
  unsigned short* o; long o_sb, o_ss, o_sh;
  float* lse;                 // [B,H,Sq], log2 units of the scaled+biased scores
  const unsigned char* kpad;  // [B,Sk] or null
  int B, H, Sq, Sk, mode;
  float scale_log2;           // log2(e)/sqrt(head_dim)
};
struct AttnBwdArgs {
  const unsigned short* q; const unsigned short* k; const unsigned short* v;
  long q_sb, q_ss, q_sh, k_sb, k_ss, k_sh, v_sb, v_ss, v_sh;
  const unsigned short* dout; long o_sb, o_ss, o_sh;   // dO shares O's layout
  const float* lse; const float* delta;                // [B,H,Sq]
  unsigned short* dq; unsigned short* dk; unsigned short* dv;  // same layouts as q / k / v
  const unsigned char* kpad;
  int B, H, Sq, Sk, mode;
  float scale_log2, scale;    // scale = 1/sqrt(head_dim)
  const unsigned short* o;    // forward output (O's layout): the dQ kernel computes delta = rowsum(dO*O)
  float* delta_out;           // ... and writes it here for the dK/dV kernel
};
// fp32 (reference-precision) attention, csrc/kernels/attention_f32.hip: same layouts as above
// with fp32 elements; one block serves the forward and both backward kernels.
struct AttnF32Args {
  const float* q; const float* k; const float* v;
  long q_sb, q_ss, q_sh, k_sb, k_ss, k_sh, v_sb, v_ss, v_sh;
  float* o; long o_sb, o_ss, o_sh;   // forward output / backward: the saved output (O's layout)
  const float* dout;                 // backward: dO (O's layout)
  float* lse;                        // [B,H,Sq] log2 units: written by the forward, read by the backward
  float* delta;                      // [B,H,Sq] rowsum(dO * O): written by the dQ kernel, read by dK/dV
  float* dq; float* dk; float* dv;   // same layouts as q / k / v
  const unsigned char* kpad;         // [B,Sk] or null
  int B, H, Sq, Sk, mode;
  float scale_log2, scale;           // log2(e)/sqrt(hd), 1/sqrt(hd)
  // optional bf16 hi/mid/lo planes of the outputs for the split-plane GEMMs that consume them
  // (sparkmi/ops/planes.py): same element offsets as O / dQ / dK,dV, planes op_ps / dq_ps / dkv_ps apart
  unsigned short* op; unsigned short* dqp; unsigned short* dkp; unsigned short* dvp;
  long op_ps, dq_ps, dkv_ps;
  int no_f32_grad;                   // backward: write dQ / dK / dV as planes only (dqp / dkp / dvp set)
  int ae16;                          // set by the launcher: outputs and their planes admit whole-row
                                     // 16-B stores (row-coalesced LDS epilogue, attention_f32.hip)
};
