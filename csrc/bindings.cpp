// pybind11 bindings for the sparkmi HIP kernel library (sparkmi._C).
// Every launcher takes raw device pointers (uintptr_t, from torch's tensor.data_ptr()) and the
// HIP stream handle (torch.cuda.current_stream().cuda_stream), so launches land on torch's
// stream and are captured by torch.cuda.graph().  Non-zero return codes raise RuntimeError.
#include <pybind11/pybind11.h>
#include <hip/hip_runtime.h>
#include <cstdint>
#include <stdexcept>
#include <string>

namespace py = pybind11;
using u = uintptr_t;
#define P(x) reinterpret_cast<void*>(x)
#define PF(x) reinterpret_cast<float*>(x)
#define S(x) reinterpret_cast<hipStream_t>(x)

#include "smi_attention.h"
#include "smi_mlp.h"
#include "smi_gemm.h"
#include "smi_gemm_f32.h"
#include "smi_gemm_sp.h"
#include "smi_cnn.h"
#include "smi_lstm.h"
#include <pybind11/stl.h>
#include <vector>

extern "C" {
int smi_ln_fwd(const void*, const void*, const float*, const float*, void*, void*, float*, float*, int, int, float,
               const uint32_t*, uint32_t, uint32_t, float, hipStream_t);
int smi_ln_bwd(const void*, const void*, const float*, const float*, const float*, void*, void*, const void*, float*,
               float*, int, float*, float*, int, int, int, const uint32_t*, uint32_t, uint32_t, float, hipStream_t);
int smi_ln_bwd_reduce(const float*, const float*, int, int, float*, float*, int, hipStream_t);
int smi_ln_bwd_reduce_multi(const float* const*, const float* const*, float* const*, float* const*, const int*, const int*,
                            int, int, hipStream_t);
int smi_ln_fwd_f32(const void*, const void*, const float*, const float*, void*, void*, float*, float*, int, int, float,
                   const uint32_t*, uint32_t, uint32_t, float, void*, long, hipStream_t);
int smi_ln_bwd_f32(const void*, const void*, const float*, const float*, const float*, void*, void*, const void*, float*,
                   float*, int, float*, float*, int, int, int, const uint32_t*, uint32_t, uint32_t, float, void*, long,
                   hipStream_t);
int smi_emb_fwd_f32(const long long*, const void*, const float*, void*, long, int, int, const uint32_t*, uint32_t, uint32_t,
                    float, void*, long, hipStream_t);
int smi_emb_bwd_f32(const long long*, const void*, float*, long, int, long long, const uint32_t*, uint32_t, uint32_t, float, long, void*,
                    hipStream_t);
int smi_attn_fwd(const AttnFwdArgs*, hipStream_t);
int smi_attn_f32_fwd(const AttnF32Args*, hipStream_t);
int smi_attn_f32_bwd(const AttnF32Args*, hipStream_t);
int smi_attn_bwd(const AttnBwdArgs*, const void*, float*, hipStream_t);
int smi_ce_fwd(const void*, int, const long long*, int, int, long long, float*, float*, float*, float*, hipStream_t);
int smi_ce_bwd(const void*, int, const long long*, int, int, long long, const float*, const float*, const float*, void*,
               void*, long, long, hipStream_t);
int smi_emb_fwd(const long long*, const void*, const float*, void*, long, int, int, const uint32_t*, uint32_t, uint32_t, float,
                hipStream_t);
int smi_emb_bwd(const long long*, const void*, float*, long, int, long long, const uint32_t*, uint32_t, uint32_t, float, long,
                void*, hipStream_t);
long smi_emb_det_ws_bytes(long, long, long);
int smi_bias_act_drop_fwd(const void*, const float*, void*, long, int, int, const uint32_t*, uint32_t, uint32_t, float, hipStream_t);
int smi_act_drop_bwd(const void*, const void*, void*, long, int, const uint32_t*, uint32_t, uint32_t, float, hipStream_t);
int smi_act_drop_bwd_f32(const float*, const float*, float*, long, int, const uint32_t*, uint32_t, uint32_t, float,
                         hipStream_t);
int smi_colsum_bf16(const void*, long, int, float*, int, float*, int, hipStream_t);
int smi_cast_f32_bf16(const float*, void*, long, hipStream_t);
int smi_add_bf16(const void*, const void*, void*, long, hipStream_t);
int smi_step_inc(float*, hipStream_t);
int smi_seed_inc(int*, hipStream_t);
int smi_lbfgs_direction(const float*, const float*, const float*, int*, int, long, const float*, float*, float*, int,
                        hipStream_t);
int smi_lbfgs_update(float*, float*, float*, int*, int, long, const float*, float, const float*, const float*, float*,
                     float, hipStream_t);
int smi_mlp(const MLPArgs*, int, hipStream_t);
int smi_mlp_grid(int);
int smi_mlp_small(int);
int smi_mlp_steps(const MLPArgs*, const MLPSteps*, hipStream_t);
int smi_gemm(const GemmArgs*, hipStream_t);
int smi_gemm_f32(const GemmF32Args*, hipStream_t);
int smi_gemm_f32_algo(int);
int smi_gemm_f32_wgrad_group(const void* const*, const long*, const void* const*, const long*, void* const*, void* const*,
                             const int*, const int*, const int*, int, hipStream_t);
int smi_gemm_sp(const GemmSpArgs*, hipStream_t);
int smi_gemm_sp_wgrad_group(const void* const*, const long*, const long*, const void* const*, const long*, const long*,
                            void* const*, void* const*, const int*, const int*, const int*, int, hipStream_t);
int smi_split3(const float*, long, int, long, void*, long, long, hipStream_t);
int smi_gemm_sp_waves(int);
int smi_gemm_sp_tm(int);
int smi_gemm_sp_wg_tm(int);
int smi_attn_ae(int);
int smi_attn_bwd1(int);
int smi_adam_wide(int);
int smi_splitk_reduce(const float*, int, long, float*, long, float*, int, hipStream_t);
int smi_splitk_fold_multi(const float* const*, float* const*, float* const*, const long*, const int*, const int*, int,
                          hipStream_t);
void smi_gemm_set_bm(int);
int smi_gemm_wgrad_group(const void* const*, const long*, const void* const*, const long*, void* const*, void* const*,
                         const int*, const int*, const int*, int, hipStream_t);
int smi_cnn(const CNNArgs*, hipStream_t);
int smi_cnn_hand_floats(int C);
int smi_cnn_fused_ok(int, int, int, int, int);
int smi_cnn_max_batch(int, int, int, int);
long smi_emb_pair_max(long);
int smi_emb_plan_algo(long, long);
int smi_emb_plan(const long long*, long, long long, long, void*, hipStream_t);
int smi_emb_sum(int, int, const long long*, const void*, float*, long, int, long long, const uint32_t*, uint32_t,
                uint32_t, float, long, void*, hipStream_t);
int smi_emb_pair(int);
int smi_cnn_reduce(const CNNArgs*, hipStream_t);
int smi_gather_rows(const void*, const long long*, void*, long, long, hipStream_t);
int smi_sparse_rank_sum(const long long*, const float*, int*, float*, int, int, int, long, hipStream_t);
int smi_gather_batch(const void* const*, void* const*, const long*, int, const long long*, int*, unsigned*, int, hipStream_t);
int smi_gather_u8_scale(const void*, const long long*, void*, long, long, float, int, hipStream_t);
int smi_lstm(const LSTMArgs*, int, hipStream_t);
int smi_lstm_supported(int, int, int, int);
long smi_lstm_slab_floats(int, int, int, int, int);
int smi_adam(float*, float*, float*, float*, void*, long, const float*, float*, unsigned*, float, float, float, float, float,
             int, int, void*, long, int*, hipStream_t);
int smi_sgd(float*, float*, float*, void*, long, const float*, float*, unsigned*, float, float, float, int, float, int,
            void*, long, int*, hipStream_t);
int smi_adam_multi(float* const*, float* const*, float* const*, float* const*, void* const*, const long*, int, const float*,
                   float*, unsigned*, float, float, float, float, float, int, int, void* const*, long, int*, int, hipStream_t);
int smi_multi_copy(void* const*, const void* const*, const long*, int, hipStream_t);
}

static void chk(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string("sparkmi._C.") + what + " failed: " +
                                        (rc > 0 ? hipGetErrorString((hipError_t)rc) : "unsupported shape"));
}

PYBIND11_MODULE(_C, m) {
  m.doc() = "sparkmi HIP/CDNA4 kernels for MI355X (gfx950)";
  m.attr("ARCH") = "gfx950";

  m.def("ln_fwd", [](u h, u r, u gamma, u beta, u y, u xsave, u mean, u rstd, int M, int D, float eps, u seedp, uint32_t salt,
                     uint32_t thresh, float dscale, u st) {
    chk(smi_ln_fwd(P(h), P(r), PF(gamma), PF(beta), P(y), P(xsave), PF(mean), PF(rstd), M, D, eps, (const uint32_t*)seedp, salt, thresh, dscale,
                   S(st)), "ln_fwd");
  });
  m.def("ln_bwd", [](u dy, u xs, u mean, u rstd, u gamma, u dres, u dh, u dres_add, u pg, u pb, int nblocks, u dgamma,
                     u dbeta, int accumulate, int M, int D, u seedp, uint32_t salt, uint32_t thresh, float dscale, u st) {
    chk(smi_ln_bwd(P(dy), P(xs), PF(mean), PF(rstd), PF(gamma), P(dres), P(dh), P(dres_add), PF(pg), PF(pb), nblocks,
                   PF(dgamma), PF(dbeta), accumulate, M, D, (const uint32_t*)seedp, salt, thresh, dscale, S(st)), "ln_bwd");
  });
  // planes / pps: optional bf16 hi/mid/lo planes [3][M][D] of the output y (fwd) / dh (bwd), 0 for none
  m.def("ln_fwd_f32", [](u h, u r, u gamma, u beta, u y, u xsave, u mean, u rstd, int M, int D, float eps, u seedp,
                         uint32_t salt, uint32_t thresh, float dscale, u planes, long pps, u st) {
    chk(smi_ln_fwd_f32(P(h), P(r), PF(gamma), PF(beta), P(y), P(xsave), PF(mean), PF(rstd), M, D, eps,
                       (const uint32_t*)seedp, salt, thresh, dscale, P(planes), pps, S(st)), "ln_fwd_f32");
  });
  m.def("ln_bwd_f32", [](u dy, u xs, u mean, u rstd, u gamma, u dres, u dh, u dres_add, u pg, u pb, int nblocks, u dgamma,
                         u dbeta, int accumulate, int M, int D, u seedp, uint32_t salt, uint32_t thresh, float dscale,
                         u planes, long pps, u st) {
    chk(smi_ln_bwd_f32(P(dy), P(xs), PF(mean), PF(rstd), PF(gamma), P(dres), P(dh), P(dres_add), PF(pg), PF(pb), nblocks,
                       PF(dgamma), PF(dbeta), accumulate, M, D, (const uint32_t*)seedp, salt, thresh, dscale, P(planes),
                       pps, S(st)),
        "ln_bwd_f32");
  });
  m.def("emb_fwd_f32", [](u ids, u table, u pe, u out, long T, int D, int Sp, u seedp, uint32_t salt, uint32_t thresh,
                          float dscale, u planes, long pps, u st) {
    chk(smi_emb_fwd_f32((const long long*)ids, P(table), PF(pe), P(out), T, D, Sp, (const uint32_t*)seedp, salt, thresh,
                        dscale, P(planes), pps, S(st)), "emb_fwd_f32");
  });
  m.def("emb_bwd_f32", [](u ids, u dout, u dtable, long T, int D, long long pad, u seedp, uint32_t salt, uint32_t thresh,
                          float dscale, long V, u ws, u st) {
    chk(smi_emb_bwd_f32((const long long*)ids, P(dout), PF(dtable), T, D, pad, (const uint32_t*)seedp, salt, thresh,
                        dscale, V, P(ws), S(st)), "emb_bwd_f32");
  });
  m.def("ln_bwd_reduce_multi", [](std::vector<u> pg, std::vector<u> pb, std::vector<u> og, std::vector<u> ob,
                                  std::vector<int> nb, std::vector<int> D, int accumulate, u st) {
    const size_t n = pg.size();
    if (pb.size() != n || og.size() != n || ob.size() != n || nb.size() != n || D.size() != n)
      throw std::runtime_error("ln_bwd_reduce_multi: list sizes differ");
    std::vector<const float*> a(n), b(n);
    std::vector<float*> c(n), d(n);
    for (size_t i = 0; i < n; ++i) { a[i] = PF(pg[i]); b[i] = PF(pb[i]); c[i] = PF(og[i]); d[i] = PF(ob[i]); }
    chk(smi_ln_bwd_reduce_multi(a.data(), b.data(), c.data(), d.data(), nb.data(), D.data(), (int)n, accumulate, S(st)),
        "ln_bwd_reduce_multi");
  });
  m.def("ln_bwd_reduce", [](u pg, u pb, int nb, int D, u dgamma, u dbeta, int accumulate, u st) {
    chk(smi_ln_bwd_reduce(PF(pg), PF(pb), nb, D, PF(dgamma), PF(dbeta), accumulate, S(st)), "ln_bwd_reduce");
  });
  m.def("attn_fwd", [](u q, u k, u v, py::tuple qs, py::tuple ks, py::tuple vs, u o, py::tuple os, u lse, u kpad, int B,
                       int H, int Sq, int Sk, int mode, float scale_log2, u st) {
    AttnFwdArgs a{};
    a.q = (const unsigned short*)q; a.k = (const unsigned short*)k; a.v = (const unsigned short*)v;
    a.q_sb = qs[0].cast<long>(); a.q_ss = qs[1].cast<long>(); a.q_sh = qs[2].cast<long>();
    a.k_sb = ks[0].cast<long>(); a.k_ss = ks[1].cast<long>(); a.k_sh = ks[2].cast<long>();
    a.v_sb = vs[0].cast<long>(); a.v_ss = vs[1].cast<long>(); a.v_sh = vs[2].cast<long>();
    a.o = (unsigned short*)o; a.o_sb = os[0].cast<long>(); a.o_ss = os[1].cast<long>(); a.o_sh = os[2].cast<long>();
    a.lse = (float*)lse; a.kpad = (const unsigned char*)kpad;
    a.B = B; a.H = H; a.Sq = Sq; a.Sk = Sk; a.mode = mode; a.scale_log2 = scale_log2;
    chk(smi_attn_fwd(&a, S(st)), "attn_fwd");
  });
  m.def("attn_bwd", [](u q, u k, u v, py::tuple qs, py::tuple ks, py::tuple vs, u o, u dout, py::tuple os, u lse,
                       u delta, u dq, u dk, u dv, u kpad, int B, int H, int Sq, int Sk, int mode, float scale_log2,
                       float scale, u st) {
    AttnBwdArgs a{};
    a.q = (const unsigned short*)q; a.k = (const unsigned short*)k; a.v = (const unsigned short*)v;
    a.q_sb = qs[0].cast<long>(); a.q_ss = qs[1].cast<long>(); a.q_sh = qs[2].cast<long>();
    a.k_sb = ks[0].cast<long>(); a.k_ss = ks[1].cast<long>(); a.k_sh = ks[2].cast<long>();
    a.v_sb = vs[0].cast<long>(); a.v_ss = vs[1].cast<long>(); a.v_sh = vs[2].cast<long>();
    a.dout = (const unsigned short*)dout;
    a.o_sb = os[0].cast<long>(); a.o_ss = os[1].cast<long>(); a.o_sh = os[2].cast<long>();
    a.lse = (const float*)lse; a.delta = (const float*)delta;
    a.dq = (unsigned short*)dq; a.dk = (unsigned short*)dk; a.dv = (unsigned short*)dv;
    a.kpad = (const unsigned char*)kpad;
    a.B = B; a.H = H; a.Sq = Sq; a.Sk = Sk; a.mode = mode; a.scale_log2 = scale_log2; a.scale = scale;
    chk(smi_attn_bwd(&a, P(o), PF(delta), S(st)), "attn_bwd");
  });
  // fp32 attention: (q, k, v) pointers + (batch, seq, head) strides; o/lse written by the forward
  // op / op_ps (fwd), dqp / dkp / dvp / dq_ps / dkv_ps (bwd): optional split planes of the outputs
  m.def("attn_f32_fwd", [](u q, u k, u v, py::tuple qs, py::tuple ks, py::tuple vs, u o, py::tuple os, u lse, u kpad,
                           int B, int H, int Sq, int Sk, int mode, float scale_log2, u op, long op_ps, u st) {
    AttnF32Args a{};
    a.q = (const float*)q; a.k = (const float*)k; a.v = (const float*)v;
    a.q_sb = qs[0].cast<long>(); a.q_ss = qs[1].cast<long>(); a.q_sh = qs[2].cast<long>();
    a.k_sb = ks[0].cast<long>(); a.k_ss = ks[1].cast<long>(); a.k_sh = ks[2].cast<long>();
    a.v_sb = vs[0].cast<long>(); a.v_ss = vs[1].cast<long>(); a.v_sh = vs[2].cast<long>();
    a.o = (float*)o; a.o_sb = os[0].cast<long>(); a.o_ss = os[1].cast<long>(); a.o_sh = os[2].cast<long>();
    a.lse = (float*)lse; a.kpad = (const unsigned char*)kpad;
    a.B = B; a.H = H; a.Sq = Sq; a.Sk = Sk; a.mode = mode; a.scale_log2 = scale_log2;
    a.op = (unsigned short*)op; a.op_ps = op_ps;
    chk(smi_attn_f32_fwd(&a, S(st)), "attn_f32_fwd");
  });
  m.def("attn_f32_bwd", [](u q, u k, u v, py::tuple qs, py::tuple ks, py::tuple vs, u o, u dout, py::tuple os, u lse,
                           u delta, u dq, u dk, u dv, u kpad, int B, int H, int Sq, int Sk, int mode, float scale_log2,
                           float scale, u dqp, u dkp, u dvp, long dq_ps, long dkv_ps, int no_f32_grad, u st) {
    AttnF32Args a{};
    a.no_f32_grad = no_f32_grad;
    a.dqp = (unsigned short*)dqp; a.dkp = (unsigned short*)dkp; a.dvp = (unsigned short*)dvp;
    a.dq_ps = dq_ps; a.dkv_ps = dkv_ps;
    a.q = (const float*)q; a.k = (const float*)k; a.v = (const float*)v;
    a.q_sb = qs[0].cast<long>(); a.q_ss = qs[1].cast<long>(); a.q_sh = qs[2].cast<long>();
    a.k_sb = ks[0].cast<long>(); a.k_ss = ks[1].cast<long>(); a.k_sh = ks[2].cast<long>();
    a.v_sb = vs[0].cast<long>(); a.v_ss = vs[1].cast<long>(); a.v_sh = vs[2].cast<long>();
    a.o = (float*)o; a.dout = (const float*)dout;
    a.o_sb = os[0].cast<long>(); a.o_ss = os[1].cast<long>(); a.o_sh = os[2].cast<long>();
    a.lse = (float*)lse; a.delta = (float*)delta;
    a.dq = (float*)dq; a.dk = (float*)dk; a.dv = (float*)dv; a.kpad = (const unsigned char*)kpad;
    a.B = B; a.H = H; a.Sq = Sq; a.Sk = Sk; a.mode = mode; a.scale_log2 = scale_log2; a.scale = scale;
    chk(smi_attn_f32_bwd(&a, S(st)), "attn_f32_bwd");
  });
  m.def("ce_fwd", [](u logits, int is_bf16, u labels, int M, int V, long long ignore, u lse, u count, u loss,
                     u row_loss, u st) {
    chk(smi_ce_fwd(P(logits), is_bf16, (const long long*)labels, M, V, ignore, PF(lse), PF(count), PF(loss),
                   PF(row_loss), S(st)), "ce_fwd");
  });
  // planes / ldp / pps: optional split planes of the fp32 gradient (0 for none)
  m.def("ce_bwd", [](u logits, int is_bf16, u labels, int M, int V, long long ignore, u lse, u count, u dloss, u grad,
                     u planes, long ldp, long pps, u st) {
    chk(smi_ce_bwd(P(logits), is_bf16, (const long long*)labels, M, V, ignore, PF(lse), PF(count), PF(dloss), P(grad),
                   P(planes), ldp, pps, S(st)), "ce_bwd");
  });
  m.def("emb_fwd", [](u ids, u table, u pe, u out, long T, int D, int Sp, u seedp, uint32_t salt, uint32_t thresh, float dscale,
                      u st) {
    chk(smi_emb_fwd((const long long*)ids, P(table), PF(pe), P(out), T, D, Sp, (const uint32_t*)seedp, salt, thresh, dscale, S(st)), "emb_fwd");
  });
  // V: table rows; ws: emb_det_ws_bytes(T, V, D) scratch -> deterministic bucketed backward (0: fp32 atomics)
  m.def("emb_det_ws_bytes", [](long T, long V, long D) { return smi_emb_det_ws_bytes(T, V, D); });
  m.def("emb_bwd", [](u ids, u dout, u dtable, long T, int D, long long pad, u seedp, uint32_t salt, uint32_t thresh,
                      float dscale, long V, u ws, u st) {
    chk(smi_emb_bwd((const long long*)ids, P(dout), PF(dtable), T, D, pad, (const uint32_t*)seedp, salt, thresh, dscale,
                    V, P(ws), S(st)), "emb_bwd");
  });
  m.def("bias_act_drop_fwd", [](u x, u bias, u y, long total, int N, int act, u seedp, uint32_t salt, uint32_t thresh,
                                float dscale, u st) {
    chk(smi_bias_act_drop_fwd(P(x), PF(bias), P(y), total, N, act, (const uint32_t*)seedp, salt, thresh, dscale, S(st)), "bias_act_drop_fwd");
  });
  m.def("act_drop_bwd", [](u dy, u y, u dx, long total, int act, u seedp, uint32_t salt, uint32_t thresh, float dscale, u st) {
    chk(smi_act_drop_bwd(P(dy), P(y), P(dx), total, act, (const uint32_t*)seedp, salt, thresh, dscale, S(st)), "act_drop_bwd");
  });
  m.def("act_drop_bwd_f32", [](u dy, u y, u dx, long total, int act, u seedp, uint32_t salt, uint32_t thresh, float dscale,
                               u st) {
    chk(smi_act_drop_bwd_f32(PF(dy), PF(y), PF(dx), total, act, (const uint32_t*)seedp, salt, thresh, dscale, S(st)),
        "act_drop_bwd_f32");
  });
  m.def("colsum_bf16", [](u x, long M, int N, u part, int rpb, u out, int acc, u st) {
    chk(smi_colsum_bf16(P(x), M, N, PF(part), rpb, PF(out), acc, S(st)), "colsum_bf16");
  });
  m.def("cast_f32_bf16", [](u x, u y, long n, u st) { chk(smi_cast_f32_bf16(PF(x), P(y), n, S(st)), "cast_f32_bf16"); });
  m.def("add_bf16", [](u a, u b, u y, long n, u st) { chk(smi_add_bf16(P(a), P(b), P(y), n, S(st)), "add_bf16"); });
  m.def("step_inc", [](u step, u st) { chk(smi_step_inc(PF(step), S(st)), "step_inc"); });
  // device L-BFGS (csrc/kernels/lbfgs.hip): st = int32 {head, count}; out = fp32 {g.d, |g|_1, |g|_2^2, pairs}
  m.def("lbfgs_direction", [](u Sm, u Ym, u rho, u st, int mm, long n, u g, u d, u out, int reset, u stream) {
    chk(smi_lbfgs_direction(PF(Sm), PF(Ym), PF(rho), reinterpret_cast<int*>(st), mm, n, PF(g), PF(d), PF(out), reset,
                            S(stream)), "lbfgs_direction");
  });
  m.def("lbfgs_update", [](u Sm, u Ym, u rho, u st, int mm, long n, u d, float t, u gn, u go, u x, float eps, u stream) {
    chk(smi_lbfgs_update(PF(Sm), PF(Ym), PF(rho), reinterpret_cast<int*>(st), mm, n, PF(d), t, PF(gn), PF(go), PF(x),
                         eps, S(stream)), "lbfgs_update");
  });
  m.def("seed_inc", [](u seed, u st) { chk(smi_seed_inc(reinterpret_cast<int*>(seed), S(st)), "seed_inc"); });
  // step: device step counter (advanced by the kernel); done: zeroed uint32 ticket word;
  // pl / ps: optional split planes of the updated weights (plane stride ps elements); seed: an
  // optional int32 dropout step seed the update kernel advances for the next step (0: none)
  m.def("adam", [](u p, u g, u mm, u v, u pbf, long n, u lr, u step, u done, float b1, float b2, float eps, float wd,
                   float gscale, int adamw, int zero_grad, u pl, long ps, u seed, u st) {
    chk(smi_adam(PF(p), PF(g), PF(mm), PF(v), P(pbf), n, PF(lr), PF(step), reinterpret_cast<unsigned*>(done), b1, b2,
                 eps, wd, gscale, adamw, zero_grad, P(pl), ps, reinterpret_cast<int*>(seed), S(st)), "adam");
  });
  // Adam over several disjoint ranges, one launch, one step advance (ZeRO-1 shard update)
  m.def("adam_multi", [](std::vector<u> p, std::vector<u> g, std::vector<u> mm, std::vector<u> v, std::vector<u> pbf,
                         std::vector<long> n, u lr, u step, u done, float b1, float b2, float eps, float wd, float gscale,
                         int adamw, int zero_grad, std::vector<u> pl, long ps, u seed, int advance, u st) {
    const size_t c = p.size();
    if (g.size() != c || mm.size() != c || v.size() != c || pbf.size() != c || n.size() != c ||
        (!pl.empty() && pl.size() != c))
      throw std::runtime_error("adam_multi: list sizes differ");
    std::vector<float*> a(c), b(c), d(c), e(c);
    std::vector<void*> f(c), q(c);
    for (size_t i = 0; i < c; ++i) {
      a[i] = PF(p[i]); b[i] = PF(g[i]); d[i] = PF(mm[i]); e[i] = PF(v[i]); f[i] = P(pbf[i]);
      q[i] = pl.empty() ? nullptr : P(pl[i]);
    }
    chk(smi_adam_multi(a.data(), b.data(), d.data(), e.data(), f.data(), n.data(), (int)c, PF(lr), PF(step),
                       reinterpret_cast<unsigned*>(done), b1, b2, eps, wd, gscale, adamw, zero_grad,
                       pl.empty() ? nullptr : q.data(), ps, reinterpret_cast<int*>(seed), advance, S(st)),
        "adam_multi");
  });
  m.def("sgd", [](u p, u g, u buf, u pbf, long n, u lr, u step, u done, float mom, float damp, float wd, int nesterov,
                  float gscale, int zero_grad, u pl, long ps, u seed, u st) {
    chk(smi_sgd(PF(p), PF(g), PF(buf), P(pbf), n, PF(lr), PF(step), reinterpret_cast<unsigned*>(done), mom, damp, wd,
                nesterov, gscale, zero_grad, P(pl), ps, reinterpret_cast<int*>(seed), S(st)), "sgd");
  });
  m.def("multi_copy", [](std::vector<u> dst, std::vector<u> src, std::vector<long> bytes, u st) {
    if (dst.size() != src.size() || dst.size() != bytes.size()) throw std::runtime_error("multi_copy: list sizes differ");
    std::vector<void*> d(dst.size());
    std::vector<const void*> s(src.size());
    for (size_t i = 0; i < dst.size(); ++i) { d[i] = P(dst[i]); s[i] = reinterpret_cast<const void*>(src[i]); }
    chk(smi_multi_copy(d.data(), s.data(), bytes.data(), (int)dst.size(), S(st)), "multi_copy");
  });

  // MLP: dims list, per-layer pointer lists (weights torch [out,in] layout, fp32)
  // mode 0 forward (+loss/logits), 1 + backward into gW/gb (accumulate or overwrite), 2 + SGD
  // update of W/b with lr (device scalar) * gscale and step += 1.  ws/ticket: grid reduction.
  m.def("mlp", [](int mode, u x, u y, u row_w, int n, std::vector<int> dims, std::vector<u> W, std::vector<u> b,
                  std::vector<u> gW, std::vector<u> gb, u logits, u loss, u dloss, int act, u ws, u ticket,
                  int accumulate, u lr, u step, float gscale, u st) {
    MLPArgs a{};
    const int L = (int)dims.size() - 1;
    if (L < 1 || L > MLP_MAXL || (int)W.size() != L || (int)b.size() != L) throw std::runtime_error("mlp: bad layer lists");
    a.x = (const float*)x; a.y = (const long long*)y; a.row_w = (const float*)row_w; a.n = n; a.nlayers = L;
    for (int i = 0; i <= L; ++i) a.dims[i] = dims[i];
    for (int l = 0; l < L; ++l) {
      a.W[l] = (const float*)W[l]; a.b[l] = (const float*)b[l];
      a.gW[l] = mode == 1 ? (float*)gW.at(l) : nullptr; a.gb[l] = mode == 1 ? (float*)gb.at(l) : nullptr;
    }
    a.logits = (float*)logits; a.loss = (float*)loss; a.dloss = (const float*)dloss; a.act = act;
    a.ws = (float*)ws; a.ticket = reinterpret_cast<unsigned*>(ticket); a.accumulate = accumulate;
    a.lr = (const float*)lr; a.step = (float*)step; a.gscale = gscale;
    chk(smi_mlp(&a, mode, S(st)), "mlp");
  });
  m.def("mlp_steps", [](std::vector<u> xs, std::vector<u> ys, std::vector<u> losses, int n, std::vector<int> dims,
                        std::vector<u> W, std::vector<u> b, int act, u lr, u step, float gscale, u perm, u cursor,
                        u loss_sum, u st) {
    MLPArgs a{};
    MLPSteps sv{};
    sv.perm = (const long long*)perm; sv.cursor = (int*)cursor; sv.B = n; sv.loss_sum = (float*)loss_sum;
    const int L = (int)dims.size() - 1;
    if (L < 1 || L > MLP_MAXL || (int)W.size() != L || (int)b.size() != L) throw std::runtime_error("mlp_steps: bad layer lists");
    if (xs.empty() || xs.size() > MLP_MAX_STEPS || ys.size() != xs.size() || losses.size() != xs.size())
      throw std::runtime_error("mlp_steps: bad step lists");
    a.n = n; a.nlayers = L; a.act = act; a.lr = (const float*)lr; a.step = (float*)step; a.gscale = gscale;
    for (int i = 0; i <= L; ++i) a.dims[i] = dims[i];
    for (int l = 0; l < L; ++l) { a.W[l] = (const float*)W[l]; a.b[l] = (const float*)b[l]; }
    a.x = (const float*)xs[0]; a.y = (const long long*)ys[0];
    sv.n = (int)xs.size();
    for (int t = 0; t < sv.n; ++t) {
      sv.x[t] = (const float*)xs[t]; sv.y[t] = (const long long*)ys[t]; sv.loss[t] = (float*)losses[t];
    }
    return smi_mlp_steps(&a, &sv, S(st)) == 0;
  }, "s fused SGD steps of the 4-5-4-3 MLP in one launch; False when the shapes are not covered");
  m.def("mlp_grid", [](int n) { return smi_mlp_grid(n); });
  m.def("mlp_small", [](int set) { return smi_mlp_small(set); },
        "MLP kernel: 1 = the compile-time 4-5-4-3 kernel for batches <= 64 (default), 0 = the generic one; -1 queries");

  m.def("gemm", [](int mode, u A, long lda, u B, long ldb, int M, int N, int K, u C, long ldc, int out_f32, int atomic,
                   int beta_acc, float alpha, u bias, u resid, long ldr, int act, u dact_y, long ldy, u seedp,
                   uint32_t salt, uint32_t thresh, float dscale, int splits, u st) {
    GemmArgs g{};
    g.mode = mode; g.A = (const unsigned short*)A; g.lda = lda; g.B = (const unsigned short*)B; g.ldb = ldb;
    g.M = M; g.N = N; g.K = K; g.C = (void*)C; g.ldc = ldc; g.out_f32 = out_f32; g.atomic = atomic;
    g.beta_acc = beta_acc; g.alpha = alpha; g.bias = (const float*)bias; g.resid = (const unsigned short*)resid;
    g.ldr = ldr; g.act = act; g.dact_y = (const unsigned short*)dact_y; g.ldy = ldy;
    g.seedp = (const uint32_t*)seedp; g.salt = salt; g.thresh = thresh; g.dscale = dscale; g.splits = splits;
    chk(smi_gemm(&g, S(st)), "gemm");
  });

  // weight-gradient GEMM in slab mode: split s of dW[N,K] = dY^T X (M split into `splits`) is
  // written (fp32, no atomics) to slab + s*N*K; splitk_reduce then folds the slabs into the grad
  // bias_slab (optional, [splits][N]) receives the per-split column sums of dY (the bias gradient)
  m.def("gemm_wgrad_slab", [](u A, long lda, u B, long ldb, int N, int K, int M, u slab, int splits, u bias_slab, u st) {
    GemmArgs g{};
    g.mode = 2; g.A = (const unsigned short*)A; g.lda = lda; g.B = (const unsigned short*)B; g.ldb = ldb;
    g.M = N; g.N = K; g.K = M; g.C = (void*)slab; g.ldc = K; g.out_f32 = 1; g.atomic = 0; g.beta_acc = 0;
    g.alpha = 1.f; g.dscale = 1.f; g.splits = splits; g.c_split_stride = (long)N * K;
    g.bias_grad = (float*)bias_slab; g.bias_split_stride = N;
    chk(smi_gemm(&g, S(st)), "gemm_wgrad_slab");
  });
  // atomic-accumulate form: gw[N,K] += dY^T X (split-K fp32 atomics), gb[N] += dY^T 1 when given
  m.def("gemm_wgrad_atomic", [](u A, long lda, u B, long ldb, int N, int K, int M, u gw, long ldgw, int splits, u gb,
                                u st) {
    GemmArgs g{};
    g.mode = 2; g.A = (const unsigned short*)A; g.lda = lda; g.B = (const unsigned short*)B; g.ldb = ldb;
    g.M = N; g.N = K; g.K = M; g.C = (void*)gw; g.ldc = ldgw; g.out_f32 = 1; g.atomic = 1; g.beta_acc = 1;
    g.alpha = 1.f; g.dscale = 1.f; g.splits = splits; g.bias_grad = (float*)gb;
    chk(smi_gemm(&g, S(st)), "gemm_wgrad_atomic");
  });
  // out[n] (+)= sum_s slab[s][:n]; with bout, also bout[nb] (+)= sum_s bias_slab[s][:nb] where the
  // bias slabs follow the weight slabs (slab + splits * n) — one launch for both
  m.def("splitk_fold_multi", [](std::vector<u> slab, std::vector<u> out, std::vector<u> bout, std::vector<long> n,
                                std::vector<int> nb, std::vector<int> splits, u st) {
    const size_t c = slab.size();
    if (out.size() != c || bout.size() != c || n.size() != c || nb.size() != c || splits.size() != c)
      throw std::runtime_error("splitk_fold_multi: list sizes differ");
    std::vector<const float*> a(c);
    std::vector<float*> o(c), bo(c);
    for (size_t i = 0; i < c; ++i) { a[i] = PF(slab[i]); o[i] = PF(out[i]); bo[i] = PF(bout[i]); }
    chk(smi_splitk_fold_multi(a.data(), o.data(), bo.data(), n.data(), nb.data(), splits.data(), (int)c, S(st)),
        "splitk_fold_multi");
  });
  // grouped no-split wgrad: gw_e[n,k] += A_e[T,n]^T B_e[T,k] (+ gb_e[n] += A_e^T 1) for every entry, one launch
  m.def("gemm_wgrad_group", [](std::vector<u> A, std::vector<long> lda, std::vector<u> B, std::vector<long> ldb,
                               std::vector<u> C, std::vector<u> bias, std::vector<int> n, std::vector<int> k,
                               std::vector<int> T, u st) {
    const size_t c = A.size();
    if (lda.size() != c || B.size() != c || ldb.size() != c || C.size() != c || bias.size() != c || n.size() != c ||
        k.size() != c || T.size() != c)
      throw std::runtime_error("gemm_wgrad_group: list sizes differ");
    std::vector<const void*> a(c), b(c);
    std::vector<void*> o(c), bo(c);
    for (size_t i = 0; i < c; ++i) { a[i] = (const void*)A[i]; b[i] = (const void*)B[i]; o[i] = (void*)C[i]; bo[i] = (void*)bias[i]; }
    chk(smi_gemm_wgrad_group(a.data(), lda.data(), b.data(), ldb.data(), o.data(), bo.data(), n.data(), k.data(),
                             T.data(), (int)c, S(st)),
        "gemm_wgrad_group");
  });
  m.def("splitk_reduce", [](u slab, int splits, long n, u out, long nb, u bout, int accumulate, u st) {
    chk(smi_splitk_reduce((const float*)slab, splits, n, (float*)out, nb, (float*)bout, accumulate, S(st)),
        "splitk_reduce");
  });
  m.def("gemm_set_bm", [](int bm) { smi_gemm_set_bm(bm); });
  // fp32 (reference-precision) GEMM on v_mfma_f32_32x32x2_f32: mode 0 FWD, 1 DGRAD, 2 WGRAD
  m.def("gemm_f32", [](int mode, u A, long lda, u B, long ldb, int M, int N, int K, u C, long ldc, int beta_acc,
                       int atomic, u bias, int relu, u resid, long ldr, u dact_y, long ldy, u seedp, uint32_t salt,
                       uint32_t thresh, float dscale, int splits, u bias_grad, u st) {
    GemmF32Args g{};
    g.mode = mode; g.A = (const float*)A; g.lda = lda; g.B = (const float*)B; g.ldb = ldb;
    g.M = M; g.N = N; g.K = K; g.C = (float*)C; g.ldc = ldc; g.beta_acc = beta_acc; g.atomic = atomic;
    g.bias = (const float*)bias; g.relu = relu; g.resid = (const float*)resid; g.ldr = ldr;
    g.dact_y = (const float*)dact_y; g.ldy = ldy; g.seedp = (const uint32_t*)seedp; g.salt = salt;
    g.thresh = thresh; g.dscale = dscale; g.splits = splits; g.bias_grad = (float*)bias_grad;
    chk(smi_gemm_f32(&g, S(st)), "gemm_f32");
  });
  // split-plane fp32 GEMM (csrc/kernels/gemm_sp*.hip): operands as bf16 planes [3][rows][ld]
  // (plane stride aps / bps), optional plane output P of the epilogue result
  m.def("gemm_sp", [](int mode, u A, long lda, long aps, u B, long ldb, long bps, int M, int N, int K, int kpad, u C,
                      long ldc, u Pp, long ldp, long pps, int beta_acc, u bias, int relu, u resid, long ldr, u dact_y,
                      long ldy, u seedp, uint32_t salt, uint32_t thresh, float dscale, u bias_grad, u mask,
                      long ldm, u st) {
    GemmSpArgs g{};
    g.mask = (unsigned char*)mask; g.ldm = ldm;
    g.mode = mode; g.A = (const unsigned short*)A; g.lda = lda; g.aps = aps;
    g.B = (const unsigned short*)B; g.ldb = ldb; g.bps = bps; g.M = M; g.N = N; g.K = K; g.kpad = kpad;
    g.C = (float*)C; g.ldc = ldc; g.P = (unsigned short*)Pp; g.ldp = ldp; g.pps = pps; g.beta_acc = beta_acc;
    g.bias = (const float*)bias; g.relu = relu; g.resid = (const float*)resid; g.ldr = ldr;
    g.dact_y = (const float*)dact_y; g.ldy = ldy; g.seedp = (const uint32_t*)seedp; g.salt = salt;
    g.thresh = thresh; g.dscale = dscale; g.bias_grad = (float*)bias_grad;
    const int rc = smi_gemm_sp(&g, S(st));  // < 0: shape / feature set not covered (caller falls back)
    if (rc > 0) chk(rc, "gemm_sp");
    return rc == 0;
  });
  m.def("gemm_sp_wgrad_group", [](std::vector<u> A, std::vector<long> lda, std::vector<long> aps, std::vector<u> B,
                                  std::vector<long> ldb, std::vector<long> bps, std::vector<u> C, std::vector<u> bias,
                                  std::vector<int> n, std::vector<int> k, std::vector<int> T, u st) {
    const size_t c = A.size();
    if (lda.size() != c || aps.size() != c || B.size() != c || ldb.size() != c || bps.size() != c || C.size() != c ||
        bias.size() != c || n.size() != c || k.size() != c || T.size() != c)
      throw std::runtime_error("gemm_sp_wgrad_group: list sizes differ");
    std::vector<const void*> a(c), b(c);
    std::vector<void*> o(c), bo(c);
    for (size_t i = 0; i < c; ++i) { a[i] = (const void*)A[i]; b[i] = (const void*)B[i]; o[i] = (void*)C[i]; bo[i] = (void*)bias[i]; }
    chk(smi_gemm_sp_wgrad_group(a.data(), lda.data(), aps.data(), b.data(), ldb.data(), bps.data(), o.data(), bo.data(),
                                n.data(), k.data(), T.data(), (int)c, S(st)),
        "gemm_sp_wgrad_group");
  });
  // x[rows][cols] fp32 -> bf16 planes P[3][rows][ldp] (x = hi + mid + lo exactly; pad columns zeroed)
  m.def("split3", [](u x, long rows, int cols, long ldx, u Pp, long ldp, long ps, u st) {
    chk(smi_split3(PF(x), rows, cols, ldx, P(Pp), ldp, ps, S(st)), "split3");
  });
  m.def("gemm_sp_waves", [](int set) { return smi_gemm_sp_waves(set); },
        "split-plane GEMM waves per 128x128 tile (4 | 8); other values query");
  m.def("gemm_sp_tm", [](int set) { return smi_gemm_sp_tm(set); },
        "split-plane GEMM tile form for large problems (16: 256x128 on 16x16x32 MFMA | 256 | 128); other values query");
  m.def("adam_wide", [](int set) { return smi_adam_wide(set); },
        "Adam launch: 1 = 1024-thread blocks, <= 512 (default), 0 = 256-thread blocks, <= 4096; other values query");
  m.def("gemm_sp_wg_tm", [](int set) { return smi_gemm_sp_wg_tm(set); },
        "tile form of the grouped weight-gradient launch (128 | 256 | 16; -1 follows gemm_sp_tm); other values query");
  m.def("gemm_f32_algo", [](int set) { return smi_gemm_f32_algo(set); },
        "fp32 GEMM product algorithm: 0 = f32 MFMA, 6 = 3-way bf16 split (6 terms); set < 0 queries");
  m.def("gemm_f32_wgrad_group", [](std::vector<u> A, std::vector<long> lda, std::vector<u> B, std::vector<long> ldb,
                                   std::vector<u> C, std::vector<u> bias, std::vector<int> n, std::vector<int> k,
                                   std::vector<int> T, u st) {
    const size_t c = A.size();
    if (lda.size() != c || B.size() != c || ldb.size() != c || C.size() != c || bias.size() != c || n.size() != c ||
        k.size() != c || T.size() != c)
      throw std::runtime_error("gemm_f32_wgrad_group: list sizes differ");
    std::vector<const void*> a(c), b(c);
    std::vector<void*> o(c), bo(c);
    for (size_t i = 0; i < c; ++i) { a[i] = (const void*)A[i]; b[i] = (const void*)B[i]; o[i] = (void*)C[i]; bo[i] = (void*)bias[i]; }
    chk(smi_gemm_f32_wgrad_group(a.data(), lda.data(), b.data(), ldb.data(), o.data(), bo.data(), n.data(), k.data(),
                                 T.data(), (int)c, S(st)),
        "gemm_f32_wgrad_group");
  });
  m.def("gather_batch", [](std::vector<u> src, std::vector<u> out, std::vector<long> row_bytes, u perm, u cursor,
                           u done, int B, u st) {
    if (src.size() != out.size() || src.size() != row_bytes.size()) throw std::runtime_error("gather_batch: sizes");
    std::vector<const void*> s(src.size());
    std::vector<void*> o(out.size());
    for (size_t i = 0; i < src.size(); ++i) { s[i] = P(src[i]); o[i] = P(out[i]); }
    chk(smi_gather_batch(s.data(), o.data(), row_bytes.data(), (int)src.size(), (const long long*)perm, (int*)cursor,
                         (unsigned*)done, B, S(st)), "gather_batch");
  }, "out_a[i] = src_a[perm[cursor * B + i]] for up to 4 arrays, then cursor += 1 (device cursor)");
  m.def("sparse_rank_sum", [](u ids, u rows, u pos, u g, int W, int k, int d, long nrow, u st) {
    chk(smi_sparse_rank_sum((const long long*)ids, (const float*)rows, (int*)pos, (float*)g, W, k, d, nrow, S(st)),
        "sparse_rank_sum");
  }, "g[v] = rank-order sum of the gathered (id, row) lists' rows of v (csrc/kernels/sparse_rows.hip)");
  m.def("gather_rows", [](u src, u idx, u out, long n, long row_bytes, u st) {
    chk(smi_gather_rows(P(src), (const long long*)idx, P(out), n, row_bytes, S(st)), "gather_rows");
  });
  m.def("gather_u8_scale", [](u src, u idx, u out, long n, long row, float scale, int bf16, u st) {
    chk(smi_gather_u8_scale(P(src), (const long long*)idx, P(out), n, row, scale, bf16, S(st)), "gather_u8_scale");
  });

  // fused CNN: phase 0 = fwd(+bwd if train), 1 = gradient reduce
  m.def("cnn", [](int phase, u x, int x_u8, float x_scale, u y, int B, int cin, int C, int classes, std::vector<u> w,
                  std::vector<u> b, std::vector<u> gw, std::vector<u> gb, u slab, u row_loss, u pred, u logits,
                  u loss, float loss_scale, u dloss, int train, int bf16, u st) {
    CNNArgs a{};
    a.bf16 = bf16;
    if (w.size() != 5 || b.size() != 5) throw std::runtime_error("cnn: need 5 weight and 5 bias pointers");
    a.x = (const void*)x; a.x_u8 = x_u8; a.x_scale = x_scale; a.y = (const long long*)y;
    a.B = B; a.cin = cin; a.C = C; a.classes = classes;
    for (int i = 0; i < 5; ++i) {
      a.w[i] = (const float*)w[i]; a.b[i] = (const float*)b[i];
      a.gw[i] = gw.size() == 5 ? (float*)gw[i] : nullptr; a.gb[i] = gb.size() == 5 ? (float*)gb[i] : nullptr;
    }
    const int sz[10] = {C * cin * 9, C, C * C * 9, C, C * C * 9, C, C * C * 9, C, classes * C * 49, classes};
    int o = 0;
    for (int i = 0; i < 10; ++i) { a.off[i] = o; o += sz[i]; }
    a.P = o; a.slab = (float*)slab; a.row_loss = (float*)row_loss; a.pred = (int*)pred; a.logits = (float*)logits;
    a.loss = (float*)loss; a.loss_scale = loss_scale; a.dloss = (const float*)dloss; a.train = train;
    chk(phase == 0 ? smi_cnn(&a, S(st)) : smi_cnn_reduce(&a, S(st)), "cnn");
  });

  // the whole single-executor CNN training step in ONE launch: forward + backward per image and
  // the fused slab reduction + SGD update in the kernel's tail (CNNArgs::fused)
  m.def("cnn_sgd_step", [](u x, int x_u8, float x_scale, u y, int B, int cin, int C, int classes, std::vector<u> w,
                           std::vector<u> b, std::vector<u> shadow, u slab, u row_loss, u loss,
                           float loss_scale, u lr, u step, u tick, int bf16, u perm, u cursor, u hand, u st) {
    CNNArgs a{};
    a.bf16 = bf16;
    if (w.size() != 5 || b.size() != 5) throw std::runtime_error("cnn_sgd_step: need 5 weight and 5 bias pointers");
    if (!shadow.empty() && shadow.size() != 10) throw std::runtime_error("cnn_sgd_step: 0 or 10 shadow pointers");
    a.x = (const void*)x; a.x_u8 = x_u8; a.x_scale = x_scale; a.y = (const long long*)y;
    a.B = B; a.cin = cin; a.C = C; a.classes = classes;
    for (int i = 0; i < 5; ++i) { a.w[i] = (const float*)w[i]; a.b[i] = (const float*)b[i]; }
    for (int i = 0; i < 10; ++i) a.shadow[i] = shadow.empty() ? nullptr : (unsigned short*)shadow[i];
    const int sz[10] = {C * cin * 9, C, C * C * 9, C, C * C * 9, C, C * C * 9, C, classes * C * 49, classes};
    int o = 0;
    for (int i = 0; i < 10; ++i) { a.off[i] = o; o += sz[i]; }
    a.P = o; a.slab = (float*)slab; a.row_loss = (float*)row_loss; a.loss = (float*)loss;
    a.loss_scale = loss_scale; a.train = 1; a.fused = 1;
    a.lr = (const float*)lr; a.step = (float*)step; a.tick = (unsigned*)tick;
    // the helpers' flags follow the tail's counters in the model's tick block
    a.hand = (float*)hand; a.hflag = hand ? a.tick + CNN_TICKS : nullptr;
    a.perm = (const long long*)perm; a.cursor = (int*)cursor;
    chk(smi_cnn(&a, S(st)), "cnn_sgd_step");
  });
  // the same launch in GRADIENT mode (the data-parallel step): the tail adds the batch gradient
  // to gw / gb (the flat gradient buffer) instead of updating the parameters
  m.def("cnn_grad_step", [](u x, int x_u8, float x_scale, u y, int B, int cin, int C, int classes, std::vector<u> w,
                            std::vector<u> b, std::vector<u> gw, std::vector<u> gb, u slab, u row_loss, u loss,
                            float loss_scale, u tick, int bf16, u perm, u cursor, u hand, u st) {
    CNNArgs a{};
    a.bf16 = bf16;
    if (w.size() != 5 || b.size() != 5 || gw.size() != 5 || gb.size() != 5)
      throw std::runtime_error("cnn_grad_step: need 5 weight, bias, weight-gradient and bias-gradient pointers");
    a.x = (const void*)x; a.x_u8 = x_u8; a.x_scale = x_scale; a.y = (const long long*)y;
    a.B = B; a.cin = cin; a.C = C; a.classes = classes;
    for (int i = 0; i < 5; ++i) {
      a.w[i] = (const float*)w[i]; a.b[i] = (const float*)b[i]; a.gw[i] = (float*)gw[i]; a.gb[i] = (float*)gb[i];
    }
    const int sz[10] = {C * cin * 9, C, C * C * 9, C, C * C * 9, C, C * C * 9, C, classes * C * 49, classes};
    int o = 0;
    for (int i = 0; i < 10; ++i) { a.off[i] = o; o += sz[i]; }
    a.P = o; a.slab = (float*)slab; a.row_loss = (float*)row_loss; a.loss = (float*)loss;
    a.loss_scale = loss_scale; a.train = 1; a.fused = 1; a.lr = nullptr; a.tick = (unsigned*)tick;
    a.hand = (float*)hand; a.hflag = hand ? a.tick + CNN_TICKS : nullptr;
    a.perm = (const long long*)perm; a.cursor = (int*)cursor;
    chk(smi_cnn(&a, S(st)), "cnn_grad_step");
  });
  m.def("attn_ae", [](int set) { return smi_attn_ae(set); },
        "fp32 attention outputs (forward and backward): 1 = whole-row stores through LDS (default), 0 = per-lane stores; -1 queries");
  m.def("attn_bwd1", [](int set) { return smi_attn_bwd1(set); },
        "attention backward at Sk <= 256 (fp32 and bf16): 1 = one single-pass kernel (default), 0 = the dQ + "
        "dK/dV pair; -1 queries");
  m.def("emb_pair_max", [](long set) { return smi_emb_pair_max(set); },
        "largest token batch the pair-compare embedding backward takes (set < 0 queries)");
  m.def("emb_plan_algo", [](long T, long V) { return smi_emb_plan_algo(T, V); },
        "the ordering algorithm emb_plan picks for T tokens over V rows (1 pair, 2 bucketed, 0 none)");
  m.def("emb_plan", [](u ids, long T, long long pad, long V, u ws, u st) {
        return smi_emb_plan((const long long*)ids, T, pad, V, (void*)ws, S(st)); },
        "ordering half of the deterministic embedding backward (ids only); returns the algorithm for emb_sum");
  m.def("emb_sum", [](int algo, int bf16, u ids, u dout, u dtable, long T, int D, long long pad, u seedp,
                      uint32_t salt, uint32_t thresh, float dscale, long V, u ws, u st) {
        chk(smi_emb_sum(algo, bf16, (const long long*)ids, (const void*)dout, (float*)dtable, T, D, pad,
                        (const uint32_t*)seedp, salt, thresh, dscale, V, (void*)ws, S(st)), "emb_sum"); },
        "summing half of the embedding backward after emb_plan");
  m.def("emb_pair", [](int set) { return smi_emb_pair(set); },
        "deterministic embedding backward: 1 = pair-compare (<= 8192 tokens), 0 = bucketed lists; -1 queries");
  m.def("cnn_fused_ok", [](int C, int cin, int classes, int B, int bf16) {
        return smi_cnn_fused_ok(C, cin, classes, B, bf16) != 0; },
        "whether a fused CNN step (one launch: forward, backward, SGD) takes batch B for this model and dtype");
  m.def("cnn_max_batch", [](int C, int cin, int classes, int bf16) { return smi_cnn_max_batch(C, cin, classes, bf16); },
        "the largest batch a fused CNN step takes for this model and dtype (the LDS of the fused tail)");
  m.def("cnn_hand_floats", [](int C) { return smi_cnn_hand_floats(C); });  // 0: weight-gradient helpers off

  m.def("lstm_supported", [](int E, int H, int L, int C) { return smi_lstm_supported(E, H, L, C) != 0; });
  m.def("lstm_slab_floats", [](int B, int E, int H, int L, int C) { return smi_lstm_slab_floats(B, E, H, L, C); });
  // LSTM: pointer lists per layer; dict-free flat signature (forward fills pred/hn/cn/ws,
  // backward reads ws + dpred/dhn/dcn and accumulates into the g_* buffers).
  m.def("lstm", [](int backward, u ids, int B, int T, int E, int H, int L, int C, long long pad_idx, u emb,
                   std::vector<u> w_ih, std::vector<u> w_hh, std::vector<u> b_ih, std::vector<u> b_hh, u w_fc, u b_fc,
                   u h0, u c0, u pred, u hn, u cn, u ws, u ws_da, u seedp, uint32_t salt, uint32_t thresh, float dscale,
                   u dpred, u dhn, u dcn, u g_emb, std::vector<u> g_w_ih, std::vector<u> g_w_hh, std::vector<u> g_b_ih,
                   std::vector<u> g_b_hh, u g_w_fc, u g_b_fc, u dh0, u dc0, u g_slab, u g_xe, long V, u emb_ws,
                   u pred_last, int dpred_last, u ce_labels, u ce_row, u ce_dlast, u ce_loss, u ce_tick,
                   u dpred_scale, int emb_planned, int emb_side, u emb_tick, u st) {
    if (L < 1 || L > LSTM_MAXL || (int)w_ih.size() != L || (int)w_hh.size() != L || (int)b_ih.size() != L ||
        (int)b_hh.size() != L)
      throw std::runtime_error("lstm: need L pointers per weight list");
    if (backward && ((int)g_w_ih.size() != L || (int)g_w_hh.size() != L || (int)g_b_ih.size() != L ||
                     (int)g_b_hh.size() != L))
      throw std::runtime_error("lstm: need L gradient pointers per list");
    LSTMArgs a{};
    a.ids = (const long long*)ids; a.B = B; a.T = T; a.E = E; a.H = H; a.L = L; a.C = C; a.pad_idx = pad_idx;
    a.emb = (const float*)emb;
    for (int i = 0; i < L; ++i) {
      a.w_ih[i] = (const float*)w_ih[i]; a.w_hh[i] = (const float*)w_hh[i];
      a.b_ih[i] = (const float*)b_ih[i]; a.b_hh[i] = (const float*)b_hh[i];
      if (backward) {
        a.g_w_ih[i] = (float*)g_w_ih[i]; a.g_w_hh[i] = (float*)g_w_hh[i];
        a.g_b_ih[i] = (float*)g_b_ih[i]; a.g_b_hh[i] = (float*)g_b_hh[i];
      }
    }
    a.w_fc = (const float*)w_fc; a.b_fc = (const float*)b_fc; a.h0 = (const float*)h0; a.c0 = (const float*)c0;
    a.pred = (float*)pred; a.hn = (float*)hn; a.cn = (float*)cn; a.ws = (float*)ws; a.ws_da = (float*)ws_da;
    a.seedp = (const uint32_t*)seedp; a.salt = salt; a.thresh = thresh; a.dscale = dscale;
    a.dpred = (const float*)dpred; a.dhn = (const float*)dhn; a.dcn = (const float*)dcn;
    a.g_emb = (float*)g_emb; a.g_w_fc = (float*)g_w_fc; a.g_b_fc = (float*)g_b_fc; a.dh0 = (float*)dh0; a.dc0 = (float*)dc0;
    a.g_slab = (float*)g_slab; a.g_xe = (float*)g_xe; a.V = V; a.emb_ws = (void*)emb_ws;
    a.pred_last = (float*)pred_last; a.dpred_last = dpred_last;
    a.ce_labels = (const long long*)ce_labels; a.ce_row = (float*)ce_row; a.ce_dlast = (float*)ce_dlast;
    a.ce_loss = (float*)ce_loss; a.ce_tick = (unsigned*)ce_tick; a.dpred_scale = (const float*)dpred_scale;
    a.emb_planned = emb_planned;
    a.emb_side = emb_side; a.emb_tick = (unsigned*)emb_tick; a.emb_V = V;
    if (a.ce_labels && (!a.ce_row || !a.ce_dlast || !a.ce_loss || !a.ce_tick || a.C > LSTM_MAXC))
      throw std::runtime_error("lstm: fused CE needs row, dlast, loss and ticket buffers");
    chk(smi_lstm(&a, backward, S(st)), "lstm");
  });
}
