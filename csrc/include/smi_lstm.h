// Argument block shared by csrc/kernels/lstm.hip and csrc/bindings.cpp.
#pragma once
#include <stdint.h>
#define LSTM_MAXL 4
#define LSTM_MAXC 16
struct LSTMArgs {
  const long long* ids;                    // token ids [B][T]
  int B, T, E, H, L, C;                    // batch, steps, embed dim, hidden, layers, fc outputs
  long long pad_idx;                       // embedding row that receives no gradient (-1: none)
  const float* emb;                        // [V][E]
  const float* w_ih[LSTM_MAXL];            // [4H][E | H], gate order i,f,g,o (torch nn.LSTM)
  const float* w_hh[LSTM_MAXL];            // [4H][H]
  const float* b_ih[LSTM_MAXL];
  const float* b_hh[LSTM_MAXL];
  const float* w_fc; const float* b_fc;    // [C][H], [C]
  const float* h0; const float* c0;        // [L][B][H] (null: zeros)
  float* pred;                             // [B][T][C]
  float* pred_last;                        // [B][C]: the last step's prediction again (or null)
  float* hn; float* cn;                    // [L][B][H]
  float* ws;                               // saved activations [B][L][T][6H] (i,f,g,o,c,h)
  float* ws_da;                            // gate grads [B][L][T][4H] (backward scratch)
  const uint32_t* seedp; uint32_t salt; uint32_t thresh; float dscale;  // inter-layer dropout
  // backward
  const float* dpred; const float* dhn; const float* dcn;
  int dpred_last;                          // 1: dpred is [B][C], the last step's only (others zero)
  float* g_emb; float* g_w_ih[LSTM_MAXL]; float* g_w_hh[LSTM_MAXL];
  float* g_b_ih[LSTM_MAXL]; float* g_b_hh[LSTM_MAXL];
  float* g_w_fc; float* g_b_fc;
  float* dh0; float* dc0;
  // deterministic gradient reduction (backward): per-sequence gradient slab [B][P] (P =
  // sum_l 4H*(In_l + H + 1) + C*H + C), per-token embedding-input gradients [B][T][E]; V =
  // embedding rows (bucketed table backward)
  float* g_slab; float* g_xe; long V; void* emb_ws;  // emb_ws: smi_emb_det_ws_bytes(B*T, V)
  // fused cross-entropy on the last step (forward; labels non-null): per-sequence loss, the head
  // gradient dlast = (softmax - onehot) / B, and the mean loss through a last-workgroup ticket
  // (ce_tick: one zeroed counter, re-armed by the kernel)
  // backward: ce_tick = the weight-gradient kernel's (L + 1) x 8 per-column-tile tickets (zeroed, re-armed)
  const long long* ce_labels; float* ce_row; float* ce_dlast; float* ce_loss; unsigned* ce_tick;
  const float* dpred_scale;                // backward: dpred x this device scalar (the loss's dloss)
  int emb_planned;                         // backward: emb_ws already holds the ordering of ids
                                           // (the algorithm the forward planned with): sum only
  // forward: order the ids for the embedding backward into emb_ws during this launch (pair path:
  // extra workgroups beside the recurrence's B, on CUs it leaves idle; emb_tick: one zeroed
  // counter, re-armed); else smi_emb_plan on the stream first
  int emb_side; unsigned* emb_tick; long emb_V;
};
#define LSTM_MAXT 2048
#define LSTM_TCH 64  // timesteps per LDS-staged chunk in the kernels' tail phases
#define LSTM_WCH 16  // backward: ticks of per-tick outputs staged in LDS between burst stores (power of 2)
#define LSTM_XW 64   // two-wave forward: ticks per LDS window of layer-0 inputs
#define LSTM_EMB_MAX 4608  // tokens (B x T) the forward launch orders itself (LDS-resident plan)
