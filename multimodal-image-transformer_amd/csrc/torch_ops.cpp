// torch_ops.cpp — the PyTorch-ROCm operator library over the C ABI (include/mit_hip.h):
// TORCH_LIBRARY(mit_hip) registers the train step's hot ops as dispatcher ops, so torch code, autograd
// (ops.py registers each op's backward formula with torch.library.register_autograd) and torch.cuda
// graph capture see typed operators instead of opaque ctypes calls. Every op allocates its outputs with
// torch, runs on torch's current HIP stream (c10::hip::getCurrentHIPStream) and forwards to the C entry
// point: the kernels are the ones native.py drives. Built by the Makefile into ../lib/libmit_torch_ops.so
// (linked against libmit_hip.so) and loaded by ops.load() (torch.ops.load_library).
//
// What each op replaces in the reference (file:line under /root/reference, or the torch /
// transformers code it dispatches to); bf16 or f32 operands, f32 parameters (bias, gamma, beta):
//   linear / linear_backward      F.linear (+ activation, + residual): nn.MultiheadAttention's packed
//                                 in_proj / out_proj (torch/nn/functional.py:6435, 6489), decoder.py:124,191
//                                 (fc_out), model.py:99,145 (projection), modeling_vit.py:213-254
//   ffn / ffn_backward            TransformerDecoderLayer._ff_block: linear2(dropout(relu(linear1(x))))
//                                 (torch/nn/modules/transformer.py:1197-1199)
//   layer_norm(_train/_backward)  LayerNorm(x + dropout(sublayer)) of the post-LN blocks
//                                 (transformer.py:1144-1153) and the encoder pre-LN (modeling_vit.py:274,281)
//   attention(_train/_backward)   F.scaled_dot_product_attention inside nn.MultiheadAttention with the
//                                 merged causal + key-padding mask and attention dropout
//                                 (functional.py:6370-6404, 6553-6566; utils.py:30-36, 47-70)
//   embedding / embedding_backward  dropout(Emb[tok] * sqrt(d) + PE[t]) (decoder.py:168-171, 34-47, 105)
//   cross_entropy                 nn.CrossEntropyLoss(ignore_index=PAD), mean (train.py:90,327)
//   clip_adamw_step               clip_grad_norm_ + AdamW.step over the flat f32 buffers (train.py:96-100;
//                                 torch/nn/utils/clip_grad.py:165-186, torch/optim/adam.py:419-547)
// Weights: the ops that own a trainable matrix (linear, ffn, embedding) take the f32 master tensor
// (what autograd differentiates; its gradient comes back in f32) and, in bf16 mode, its bf16 shadow
// `*_lp` that the GEMMs read (params.FlatParams keeps the two in sync).
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include <cmath>
#include <tuple>

#include "../../include/mit_hip.h"

namespace {

using OptT = c10::optional<at::Tensor>;

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

int dtype_code(const at::Tensor& t) {
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat,
              "mit_hip: operands must be bfloat16 or float32, got ", t.scalar_type());
  return t.scalar_type() == at::kBFloat16 ? MIT_BF16 : MIT_F32;
}

void check_rc(int rc, const char* op) {
  if (rc != MIT_OK) {
    const char* msg = mit_last_error();
    TORCH_CHECK(false, op, " failed (rc=", rc, "): ", msg ? msg : "");
  }
}

// every tensor operand on x's ROCm device (a CPU bias / gamma would hand the kernel a host pointer)
void check_dev(const at::Tensor& t, const at::Tensor& ref, const char* op, const char* name) {
  TORCH_CHECK(t.is_cuda(), op, ": ", name, " must be a ROCm device tensor (there is no CPU fallback)");
  TORCH_CHECK(t.device() == ref.device(), op, ": ", name, " is on ", t.device(), ", x on ", ref.device());
}
void check_opt(const OptT& t, const at::Tensor& ref, const char* op, const char* name) {
  if (t) check_dev(*t, ref, op, name);
}

// [..., K] -> rows x K with unit column stride (a view when possible)
at::Tensor rows2d(const at::Tensor& x) {
  at::Tensor c = x.stride(-1) == 1 ? x : x.contiguous();
  if (c.dim() == 2) {
    if (c.size(0) > 1 && c.stride(0) < c.size(1)) c = c.contiguous();
    return c;
  }
  return c.reshape({-1, c.size(-1)});
}

const uint64_t* seed_ptr(const OptT& seed, double p, const char* op) {
  if (p <= 0.0) return nullptr;
  TORCH_CHECK(seed && seed->is_cuda() && seed->scalar_type() == at::kLong && seed->numel() >= 1, op,
              ": dropout needs a device int64 seed tensor");
  return (const uint64_t*)seed->data_ptr<int64_t>();
}

at::Tensor f32(const at::Tensor& t) { return t.scalar_type() == at::kFloat ? t.contiguous() : t.to(at::kFloat).contiguous(); }

// the matrix the GEMM reads: the low-precision shadow when given, else the master itself
const at::Tensor& gemm_weight(const at::Tensor& w, const OptT& w_lp) { return w_lp ? *w_lp : w; }

// the compute-dtype gradient a backward GEMM reads as its A operand (an f32 upstream gradient, e.g.
// of f32 logits, is rounded once by mit_cast_f32 in bf16 mode)
at::Tensor as_compute(const at::Tensor& g, at::ScalarType dt) {
  at::Tensor c = g.stride(-1) == 1 ? g : g.contiguous();
  c = rows2d(c).contiguous();
  if (c.scalar_type() == dt) return c;
  TORCH_CHECK(c.scalar_type() == at::kFloat && dt == at::kBFloat16, "mit_hip: gradient dtype ", c.scalar_type(),
              " for a ", dt, " op");
  at::Tensor o = at::empty(c.sizes(), c.options().dtype(dt));
  check_rc(mit_cast_f32(MIT_BF16, c.numel(), c.data_ptr<float>(), o.data_ptr(), stream()), "mit_hip: cast");
  return o;
}

mit_gemm_args gemm_nt(const at::Tensor& a, const at::Tensor& b, at::Tensor& c) {
  mit_gemm_args g{};
  g.dtype = dtype_code(a);
  g.a_layout = MIT_K_CONTIG;
  g.b_layout = MIT_K_CONTIG;
  g.M = a.size(0);
  g.N = b.size(0);
  g.K = a.size(1);
  g.A = a.data_ptr();
  g.lda = a.stride(0);
  g.B = b.data_ptr();
  g.ldb = b.stride(0);
  g.C = c.data_ptr();
  g.ldc = c.stride(0);
  g.alpha = 1.0f;
  g.out_f32 = c.scalar_type() == at::kFloat;
  return g;
}

// dX [M, K] = dY [M, N] W [N, K]
at::Tensor gemm_dx(const at::Tensor& dy, const at::Tensor& w, at::ScalarType out_dt, const char* op) {
  at::Tensor dx = at::empty({dy.size(0), w.size(1)}, dy.options().dtype(out_dt));
  mit_gemm_args g{};
  g.dtype = dtype_code(dy);
  g.a_layout = MIT_K_CONTIG;
  g.b_layout = MIT_MN_CONTIG;
  g.M = dy.size(0);
  g.N = w.size(1);
  g.K = dy.size(1);
  g.A = dy.data_ptr();
  g.lda = dy.stride(0);
  g.B = w.data_ptr();
  g.ldb = w.stride(0);
  g.C = dx.data_ptr();
  g.ldc = g.N;
  g.alpha = 1.0f;
  g.out_f32 = out_dt == at::kFloat;
  check_rc(mit_gemm(&g, stream()), op);
  return dx;
}

// dW [N, K] = dY^T [N, M] X [M, K] in f32, the bias gradient (row sums of dY^T) fused in; split-K
// scratch from torch's allocator
std::tuple<at::Tensor, at::Tensor> gemm_dw(const at::Tensor& dy, const at::Tensor& x, bool want_db, const char* op) {
  const int64_t M = dy.size(0), N = dy.size(1), K = x.size(1);
  at::Tensor dw = at::empty({N, K}, dy.options().dtype(at::kFloat));
  at::Tensor db = want_db ? at::empty({N}, dy.options().dtype(at::kFloat)) : at::Tensor();
  const long wsb = mit_gemm_workspace_bytes(N, K, M);
  at::Tensor ws = wsb > 0 ? at::zeros({(wsb + 3) / 4}, dy.options().dtype(at::kFloat)) : at::Tensor();
  mit_gemm_args g{};
  g.dtype = dtype_code(dy);
  g.a_layout = MIT_MN_CONTIG;
  g.b_layout = MIT_MN_CONTIG;
  g.M = N;
  g.N = K;
  g.K = M;
  g.A = dy.data_ptr();
  g.lda = dy.stride(0);
  g.B = x.data_ptr();
  g.ldb = x.stride(0);
  g.C = dw.data_ptr();
  g.ldc = K;
  g.alpha = 1.0f;
  g.out_f32 = 1;
  g.rowsum = want_db ? db.data_ptr<float>() : nullptr;
  g.workspace = wsb > 0 ? ws.data_ptr() : nullptr;
  g.workspace_bytes = wsb;
  check_rc(mit_gemm(&g, stream()), op);
  return {dw, db};
}

// ---- linear ------------------------------------------------------------------------------------
// y = dropout(act(x W^T + bias)) + residual ; x [..., K], W [N, K] (nn.Linear layout), bias [N],
// residual [..., N] in x's dtype; out_f32: f32 output whatever the operand dtype (the f32 logits of
// decoder.py:191)
at::Tensor linear(const at::Tensor& x, const at::Tensor& w, const OptT& bias, int64_t act, const OptT& residual,
                  double drop_p, const OptT& seed, int64_t site, bool out_f32, const OptT& w_lp) {
  const char* op = "mit_hip::linear";
  check_dev(x, x, op, "x");
  check_dev(w, x, op, "weight");
  check_opt(bias, x, op, "bias");
  check_opt(residual, x, op, "residual");
  check_opt(w_lp, x, op, "weight_lp");
  const at::Tensor& wk = gemm_weight(w, w_lp);
  TORCH_CHECK(x.scalar_type() == wk.scalar_type(), op, ": x (", x.scalar_type(), ") and the GEMM weight (",
              wk.scalar_type(), ") dtypes differ");
  TORCH_CHECK(wk.dim() == 2 && x.size(-1) == wk.size(1), op, ": weight must be [N, K] with K = x.size(-1)");
  TORCH_CHECK(act >= MIT_ACT_NONE && act <= MIT_ACT_QUICK_GELU, op, ": bad activation code ", act);
  TORCH_CHECK(drop_p >= 0.0 && drop_p < 1.0, op, ": drop_p must be in [0, 1)");
  const c10::DeviceGuard guard(x.device());
  const at::Tensor a = rows2d(x), b = wk.stride(1) == 1 ? wk : wk.contiguous();
  const int64_t M = a.size(0), N = b.size(0);
  std::vector<int64_t> shape(x.sizes().begin(), x.sizes().end());
  shape.back() = N;
  at::Tensor y = at::empty(shape, x.options().dtype(out_f32 ? at::kFloat : x.scalar_type()));
  at::Tensor bias_f, res;
  if (bias) {
    bias_f = f32(*bias);
    TORCH_CHECK(bias_f.numel() == N, op, ": bias must have N elements");
  }
  if (residual) {
    TORCH_CHECK(residual->scalar_type() == y.scalar_type() && residual->size(-1) == N && residual->numel() == M * N,
                op, ": residual must be [..., N] in the output dtype");
    res = rows2d(*residual);
  }
  at::Tensor y2 = y.view({M, N});
  mit_gemm_args g = gemm_nt(a, b, y2);
  g.bias = bias ? bias_f.data_ptr<float>() : nullptr;
  g.act = (int)act;
  g.residual = residual ? res.data_ptr() : nullptr;
  g.ldr = residual ? res.stride(0) : 0;
  g.drop_p = (float)drop_p;
  g.seed = seed_ptr(seed, drop_p, op);
  g.site = (uint32_t)site;
  check_rc(mit_gemm(&g, stream()), op);
  return y;
}

// gradients of linear without activation / dropout: (dx in x's dtype, dW f32, db f32); dy [..., N]
std::tuple<at::Tensor, at::Tensor, at::Tensor> linear_backward(const at::Tensor& dy, const at::Tensor& x,
                                                               const at::Tensor& w_gemm, bool need_dx, bool need_dw,
                                                               bool need_db) {
  const char* op = "mit_hip::linear_backward";
  check_dev(dy, x, op, "grad");
  check_dev(w_gemm, x, op, "weight");
  const c10::DeviceGuard guard(x.device());
  const at::ScalarType dt = x.scalar_type();
  const at::Tensor g = as_compute(dy, dt), a = rows2d(x).contiguous();
  at::Tensor dx, dw, db;
  if (need_dx) {
    dx = gemm_dx(g, w_gemm.stride(1) == 1 ? w_gemm : w_gemm.contiguous(), dt, op);
    std::vector<int64_t> shape(x.sizes().begin(), x.sizes().end());
    dx = dx.view(shape);
  }
  if (need_dw || need_db) std::tie(dw, db) = gemm_dw(g, a, need_db, op);
  return {dx, need_dw ? dw : at::Tensor(), need_db ? db : at::Tensor()};
}

// ---- feed-forward block ------------------------------------------------------------------------
// y = W2 dropout(relu(W1 x + b1)) + b2, the hidden h = dropout(relu(.)) returned for the backward
std::tuple<at::Tensor, at::Tensor> ffn(const at::Tensor& x, const at::Tensor& w1, const at::Tensor& b1,
                                       const at::Tensor& w2, const at::Tensor& b2, double drop_p, const OptT& seed,
                                       int64_t site, const OptT& w1_lp, const OptT& w2_lp) {
  at::Tensor h = linear(x, w1, b1, MIT_ACT_RELU, c10::nullopt, drop_p, seed, site, false, w1_lp);
  at::Tensor y = linear(h, w2, b2, MIT_ACT_NONE, c10::nullopt, 0.0, c10::nullopt, 0, false, w2_lp);
  return {y, h};
}

// (dx, dW1, db1, dW2, db2): dh = (dy W2) * (h > 0) / (1 - p) (the aux-mask epilogue of the dX GEMM:
// h > 0 exactly where relu passed and dropout kept)
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> ffn_backward(
    const at::Tensor& dy, const at::Tensor& x, const at::Tensor& h, const at::Tensor& w1_gemm,
    const at::Tensor& w2_gemm, double drop_p) {
  const char* op = "mit_hip::ffn_backward";
  check_dev(dy, x, op, "grad");
  check_dev(h, x, op, "hidden");
  const c10::DeviceGuard guard(x.device());
  const at::ScalarType dt = x.scalar_type();
  const at::Tensor g = as_compute(dy, dt), a = rows2d(x).contiguous(), hh = rows2d(h).contiguous();
  const int64_t R = g.size(0), F = hh.size(1), d = a.size(1);
  at::Tensor dh = at::empty({R, F}, g.options());
  mit_gemm_args m{};
  m.dtype = dtype_code(g);
  m.a_layout = MIT_K_CONTIG;
  m.b_layout = MIT_MN_CONTIG;
  m.M = R;
  m.N = F;
  m.K = g.size(1);
  m.A = g.data_ptr();
  m.lda = g.stride(0);
  m.B = w2_gemm.data_ptr();
  m.ldb = w2_gemm.stride(0);
  m.C = dh.data_ptr();
  m.ldc = F;
  m.alpha = 1.0f;
  m.aux = hh.data_ptr();
  m.ld_aux = hh.stride(0);
  m.aux_scale = drop_p > 0.0 ? (float)(1.0 / (1.0 - drop_p)) : 1.0f;
  m.out_f32 = dt == at::kFloat;
  check_rc(mit_gemm(&m, stream()), op);
  at::Tensor dw2, db2, dw1, db1;
  std::tie(dw2, db2) = gemm_dw(g, hh, true, op);
  at::Tensor dx = gemm_dx(dh, w1_gemm, dt, op);
  std::tie(dw1, db1) = gemm_dw(dh, a, true, op);
  std::vector<int64_t> shape(x.sizes().begin(), x.sizes().end());
  (void)d;
  return {dx.view(shape), dw1, db1, dw2, db2};
}

// ---- LayerNorm ---------------------------------------------------------------------------------
// y = LN(x + dropout(residual)) over the last dim, f32 statistics; also z = x + dropout(residual)
// and the row statistics (mean, rstd) for the backward
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> layer_norm_train(const at::Tensor& x, const at::Tensor& gamma,
                                                                            const at::Tensor& beta, double eps,
                                                                            const OptT& residual, double drop_p,
                                                                            const OptT& seed, int64_t site) {
  const char* op = "mit_hip::layer_norm";
  check_dev(x, x, op, "x");
  check_dev(gamma, x, op, "gamma");
  check_dev(beta, x, op, "beta");
  check_opt(residual, x, op, "residual");
  const c10::DeviceGuard guard(x.device());
  const at::Tensor a = rows2d(x);
  const int64_t R = a.size(0), C = a.size(1);
  const at::Tensor g = f32(gamma), bt = f32(beta);
  TORCH_CHECK(g.numel() == C && bt.numel() == C, op, ": gamma / beta must have x.size(-1) elements");
  at::Tensor res;
  if (residual) {
    TORCH_CHECK(residual->scalar_type() == x.scalar_type() && residual->numel() == x.numel(), op,
                ": residual must match x");
    res = rows2d(*residual);
  }
  at::Tensor y = at::empty(x.sizes(), x.options());
  at::Tensor z = at::empty(x.sizes(), x.options());
  at::Tensor mean = at::empty({R}, x.options().dtype(at::kFloat)), rstd = at::empty({R}, x.options().dtype(at::kFloat));
  check_rc(mit_layernorm_fwd(dtype_code(x), R, C, a.data_ptr(), a.stride(0), residual ? res.data_ptr() : nullptr,
                             residual ? res.stride(0) : 0, (float)drop_p, seed_ptr(seed, drop_p, op), (uint32_t)site,
                             g.data_ptr<float>(), bt.data_ptr<float>(), (float)eps, z.data_ptr(), y.data_ptr(), C,
                             mean.data_ptr<float>(), rstd.data_ptr<float>(), stream()),
           op);
  return {y, z, mean, rstd};
}

at::Tensor layer_norm(const at::Tensor& x, const at::Tensor& gamma, const at::Tensor& beta, double eps,
                      const OptT& residual) {
  return std::get<0>(layer_norm_train(x, gamma, beta, eps, residual, 0.0, c10::nullopt, 0));
}

// (dx, dresidual, dgamma, dbeta) of layer_norm_train
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> layer_norm_backward(
    const at::Tensor& dy, const at::Tensor& z, const at::Tensor& mean, const at::Tensor& rstd, const at::Tensor& gamma,
    double drop_p, const OptT& seed, int64_t site, bool has_residual) {
  const char* op = "mit_hip::layer_norm_backward";
  check_dev(dy, z, op, "grad");
  const c10::DeviceGuard guard(z.device());
  const at::Tensor zz = rows2d(z).contiguous(), g = as_compute(dy, z.scalar_type()), gm = f32(gamma);
  const int64_t R = zz.size(0), C = zz.size(1);
  at::Tensor dx = at::empty({R, C}, zz.options());
  at::Tensor dr = has_residual ? at::empty({R, C}, zz.options()) : at::Tensor();
  at::Tensor dgamma = at::empty({C}, zz.options().dtype(at::kFloat)), dbeta = at::empty({C}, zz.options().dtype(at::kFloat));
  at::Tensor ws = at::empty({mit_layernorm_bwd_ws_floats(R, C)}, zz.options().dtype(at::kFloat));
  check_rc(mit_layernorm_bwd(dtype_code(zz), R, C, g.data_ptr(), zz.data_ptr(), mean.data_ptr<float>(),
                             rstd.data_ptr<float>(), gm.data_ptr<float>(), dx.data_ptr(),
                             has_residual ? dr.data_ptr() : nullptr, (float)drop_p, seed_ptr(seed, drop_p, op),
                             (uint32_t)site, dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), ws.data_ptr<float>(),
                             stream()),
           op);
  return {dx.view(z.sizes()), has_residual ? dr.view(z.sizes()) : dr, dgamma, dbeta};
}

// ---- attention ---------------------------------------------------------------------------------
// q [B, Lq, H*Dh], k / v [B, Lk, H*Dh]: token rows with the heads interleaved, the last dim
// contiguous, any row / batch strides (views of a packed projection). key_tokens int64 [B, Lk]: key j
// of batch b is masked where key_tokens == pad_idx.
mit_attn_args attn_args(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, at::Tensor& o, float* lse,
                        const OptT& key_tokens, int64_t pad_idx, bool causal, double scale, double drop_p,
                        const OptT& seed, int64_t site, const char* op) {
  mit_attn_args a{};
  a.q = q.data_ptr();
  a.q_row = q.stride(1);
  a.q_batch = q.stride(0);
  a.k = k.data_ptr();
  a.k_row = k.stride(1);
  a.k_batch = k.stride(0);
  a.v = v.data_ptr();
  a.v_row = v.stride(1);
  a.v_batch = v.stride(0);
  a.o = o.data_ptr();
  a.o_row = o.stride(1);
  a.o_batch = o.stride(0);
  a.lse = lse;
  if (key_tokens) {
    TORCH_CHECK(key_tokens->scalar_type() == at::kLong && key_tokens->is_contiguous() &&
                    key_tokens->numel() == k.size(0) * k.size(1), op, ": key_tokens must be contiguous int64 [B, Lk]");
    a.key_tokens = key_tokens->data_ptr<int64_t>();
    a.tok_batch = k.size(1);
  }
  a.pad_idx = (int)pad_idx;
  a.causal = causal ? 1 : 0;
  a.scale = (float)scale;
  a.drop_p = (float)drop_p;
  a.seed = seed_ptr(seed, drop_p, op);
  a.site = (uint32_t)site;
  return a;
}

void attn_check(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, int64_t heads, const OptT& key_tokens,
                const char* op) {
  check_dev(q, q, op, "q");
  check_dev(k, q, op, "k");
  check_dev(v, q, op, "v");
  check_opt(key_tokens, q, op, "key_tokens");
  TORCH_CHECK(q.dim() == 3 && k.dim() == 3 && v.dim() == 3, op, ": q, k, v must be [B, L, H*Dh]");
  TORCH_CHECK(q.scalar_type() == k.scalar_type() && q.scalar_type() == v.scalar_type(), op, ": q, k, v dtypes differ");
  TORCH_CHECK(q.stride(2) == 1 && k.stride(2) == 1 && v.stride(2) == 1, op, ": last dim must be contiguous");
  const int64_t B = q.size(0), E = q.size(2), Lk = k.size(1);
  TORCH_CHECK(heads > 0 && E % heads == 0 && k.size(2) == E && v.size(2) == E && k.size(0) == B && v.size(0) == B &&
                  v.size(1) == Lk, op, ": shape mismatch");
}

// (o [B, Lq, E], lse f32 [B*H*Lq])
std::tuple<at::Tensor, at::Tensor> attention_train(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                                   int64_t heads, bool causal, double scale, const OptT& key_tokens,
                                                   int64_t pad_idx, double drop_p, const OptT& seed, int64_t site) {
  const char* op = "mit_hip::attention";
  attn_check(q, k, v, heads, key_tokens, op);
  const c10::DeviceGuard guard(q.device());
  const int64_t B = q.size(0), Lq = q.size(1), E = q.size(2), Lk = k.size(1);
  at::Tensor o = at::empty({B, Lq, E}, q.options());
  at::Tensor lse = at::empty({B * heads * Lq}, q.options().dtype(at::kFloat));
  mit_attn_args a = attn_args(q, k, v, o, lse.data_ptr<float>(), key_tokens, pad_idx, causal, scale, drop_p, seed, site, op);
  check_rc(mit_attention_fwd(dtype_code(q), B, heads, Lq, Lk, E / heads, &a, stream()), op);
  return {o, lse};
}

at::Tensor attention(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, int64_t heads, bool causal,
                     double scale) {
  return std::get<0>(attention_train(q, k, v, heads, causal, scale, c10::nullopt, -1, 0.0, c10::nullopt, 0));
}

// (dq, dk, dv), each a new [B, L, E] tensor
std::tuple<at::Tensor, at::Tensor, at::Tensor> attention_backward(
    const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, const at::Tensor& o,
    const at::Tensor& lse, int64_t heads, bool causal, double scale, const OptT& key_tokens, int64_t pad_idx,
    double drop_p, const OptT& seed, int64_t site) {
  const char* op = "mit_hip::attention_backward";
  attn_check(q, k, v, heads, key_tokens, op);
  check_dev(dout, q, op, "grad");
  const c10::DeviceGuard guard(q.device());
  const int64_t B = q.size(0), Lq = q.size(1), E = q.size(2), Lk = k.size(1);
  at::Tensor oc = o.contiguous();
  at::Tensor dO = dout.scalar_type() == q.scalar_type() ? dout.contiguous() : as_compute(dout, q.scalar_type()).view({B, Lq, E});
  at::Tensor dq = at::empty({B, Lq, E}, q.options()), dk = at::empty({B, Lk, E}, q.options()),
             dv = at::empty({B, Lk, E}, q.options());
  at::Tensor delta = at::empty({B * heads * Lq}, q.options().dtype(at::kFloat));
  mit_attn_args a = attn_args(q, k, v, oc, (float*)lse.data_ptr<float>(), key_tokens, pad_idx, causal, scale, drop_p,
                              seed, site, op);
  mit_attn_grads g{};
  g.dout = dO.data_ptr();
  g.do_row = E;
  g.do_batch = Lq * E;
  g.dq = dq.data_ptr();
  g.dq_row = E;
  g.dq_batch = Lq * E;
  g.dk = dk.data_ptr();
  g.dk_row = E;
  g.dk_batch = Lk * E;
  g.dv = dv.data_ptr();
  g.dv_row = E;
  g.dv_batch = Lk * E;
  g.delta_ws = delta.data_ptr<float>();
  check_rc(mit_attention_bwd(dtype_code(q), B, heads, Lq, Lk, E / heads, &a, &g, stream()), op);
  return {dq, dk, dv};
}

// ---- token embedding ---------------------------------------------------------------------------
// x = dropout(table[tokens] * scale + pe[t]) ; tokens int64 [B, T], table [V, d] (the GEMM-dtype
// shadow table_lp when given), pe f32 [>= T, d]
at::Tensor embedding(const at::Tensor& tokens, const at::Tensor& table, const at::Tensor& pe, double scale, double drop_p,
                     const OptT& seed, int64_t site, const OptT& table_lp, int64_t pad_idx) {
  (void)pad_idx;  // the forward reads the row as it is (nn.Embedding(padding_idx)); the backward skips it
  const char* op = "mit_hip::embedding";
  check_dev(tokens, tokens, op, "tokens");
  check_dev(table, tokens, op, "table");
  check_dev(pe, tokens, op, "pe");
  check_opt(table_lp, tokens, op, "table_lp");
  TORCH_CHECK(tokens.dim() == 2 && tokens.scalar_type() == at::kLong && tokens.is_contiguous(), op,
              ": tokens must be contiguous int64 [B, T]");
  const at::Tensor& tb = gemm_weight(table, table_lp);
  TORCH_CHECK(tb.dim() == 2 && tb.is_contiguous(), op, ": table must be contiguous [V, d]");
  const at::Tensor pf = f32(pe);
  const int64_t B = tokens.size(0), T = tokens.size(1), d = tb.size(1);
  TORCH_CHECK(pf.dim() == 2 && pf.size(0) >= T && pf.size(1) == d, op, ": pe must be [>= T, d]");
  const c10::DeviceGuard guard(tokens.device());
  at::Tensor out = at::empty({B, T, d}, tb.options());
  check_rc(mit_embed_fwd(dtype_code(tb), B, T, d, tokens.data_ptr<int64_t>(), tb.data_ptr(), (float)scale,
                         pf.data_ptr<float>(), (float)drop_p, seed_ptr(seed, drop_p, op), (uint32_t)site, out.data_ptr(),
                         stream()),
           op);
  return out;
}

// dtable f32 [V, d]: each token row the sum of its positions' rows in position order (deterministic
// plan) when B*T <= 16384 and d % 8 == 0; the pad_idx row gets nothing
at::Tensor embedding_backward(const at::Tensor& dx, const at::Tensor& tokens, int64_t V, double scale, double drop_p,
                              const OptT& seed, int64_t site, int64_t pad_idx) {
  const char* op = "mit_hip::embedding_backward";
  check_dev(dx, tokens, op, "grad");
  const c10::DeviceGuard guard(tokens.device());
  const int64_t B = tokens.size(0), T = tokens.size(1), d = dx.size(-1);
  const at::Tensor g = dx.contiguous();
  at::Tensor dt = at::zeros({V, d}, g.options().dtype(at::kFloat));
  at::Tensor plan;
  const bool planned = B * T <= 16384 && d % 8 == 0;
  if (planned) {
    plan = at::empty({mit_embed_plan_ints(B * T)}, tokens.options().dtype(at::kInt));
    check_rc(mit_embed_plan(tokens.data_ptr<int64_t>(), B * T, plan.data_ptr<int>(), stream()), op);
  }
  check_rc(mit_embed_bwd(dtype_code(g), B, T, d, tokens.data_ptr<int64_t>(), g.data_ptr(), (float)scale, (float)drop_p,
                         seed_ptr(seed, drop_p, op), (uint32_t)site, (int)pad_idx, planned ? plan.data_ptr<int>() : nullptr,
                         dt.data_ptr<float>(), stream()),
           op);
  return dt;
}

// ---- cross-entropy -----------------------------------------------------------------------------
// (loss f32 [] = mean over the targets != ignore_index of -log_softmax(logits)[t], dlogits = its
// gradient with respect to logits [..., V], computed in the same pass)
std::tuple<at::Tensor, at::Tensor> cross_entropy(const at::Tensor& logits, const at::Tensor& targets,
                                                 int64_t ignore_index) {
  const char* op = "mit_hip::cross_entropy";
  check_dev(logits, logits, op, "logits");
  check_dev(targets, logits, op, "targets");
  const c10::DeviceGuard guard(logits.device());
  const at::Tensor t = targets.contiguous();
  TORCH_CHECK(t.scalar_type() == at::kLong, op, ": targets must be int64");
  const int64_t V = logits.size(-1), R = logits.numel() / V;
  TORCH_CHECK(t.numel() == R, op, ": targets must have logits.numel() / V elements");
  at::Tensor grad = logits.contiguous().clone().view({R, V});
  at::Tensor sc = at::zeros({3}, logits.options().dtype(at::kFloat));  // count, loss_sum, loss
  at::Tensor rows = at::empty({R}, logits.options().dtype(at::kFloat));
  float* s = sc.data_ptr<float>();
  check_rc(mit_count_targets(t.data_ptr<int64_t>(), R, (int)ignore_index, s, stream()), op);
  check_rc(mit_cross_entropy(dtype_code(grad), R, V, grad.data_ptr(), V, t.data_ptr<int64_t>(), (int)ignore_index, s,
                             s + 1, 1, rows.data_ptr<float>(), stream()),
           op);
  check_rc(mit_scalar_div(s + 1, s, s + 2, stream()), op);
  return {sc.select(0, 2), grad.view(logits.sizes())};
}

// ---- clip_grad_norm_ + AdamW -------------------------------------------------------------------
// In place over the flat f32 buffers (params.FlatParams): the total gradient norm and the clip
// coefficient (max_norm > 0) into norm_out = {total_norm, coef}, the device step counter + 1, then
// decoupled-weight-decay AdamW with bias corrections reading lr / step / coef from device memory;
// shadow (bf16, optional) is refreshed from the new parameters. ws: mit_grad_norm_ws_floats(n) f32.
void clip_adamw_step(const at::Tensor& param, const at::Tensor& grad, const at::Tensor& exp_avg,
                     const at::Tensor& exp_avg_sq, const OptT& shadow, const at::Tensor& step, const at::Tensor& lr,
                     const at::Tensor& norm_out, const at::Tensor& ws, double max_norm, double beta1, double beta2,
                     double eps, double weight_decay) {
  const char* op = "mit_hip::clip_adamw_step";
  for (auto* t : {&grad, &exp_avg, &exp_avg_sq, &lr, &norm_out, &ws}) {
    check_dev(*t, param, op, "buffer");
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), op, ": f32 contiguous buffers only");
  }
  check_dev(step, param, op, "step");
  check_opt(shadow, param, op, "shadow");
  const int64_t n = param.numel();
  TORCH_CHECK(param.scalar_type() == at::kFloat && param.is_contiguous() && grad.numel() == n && exp_avg.numel() == n &&
                  exp_avg_sq.numel() == n && norm_out.numel() >= 2 && ws.numel() >= mit_grad_norm_ws_floats(n) &&
                  step.scalar_type() == at::kLong,
              op, ": buffer sizes / dtypes");
  TORCH_CHECK(!shadow || (shadow->scalar_type() == at::kBFloat16 && shadow->numel() == n && shadow->is_contiguous()), op,
              ": shadow must be contiguous bf16 [n]");
  const c10::DeviceGuard guard(param.device());
  check_rc(mit_grad_norm(grad.data_ptr<float>(), n, (float)max_norm, ws.data_ptr<float>(), norm_out.data_ptr<float>(),
                         stream()),
           op);
  check_rc(mit_step_inc(step.data_ptr<int64_t>(), stream()), op);
  check_rc(mit_adamw(n, param.data_ptr<float>(), grad.data_ptr<float>(), exp_avg.data_ptr<float>(),
                     exp_avg_sq.data_ptr<float>(), shadow ? shadow->data_ptr() : nullptr, norm_out.data_ptr<float>(),
                     lr.data_ptr<float>(), step.data_ptr<int64_t>(), (float)beta1, (float)beta2, (float)eps,
                     (float)weight_decay, stream()),
           op);
}

}  // namespace

TORCH_LIBRARY(mit_hip, m) {
  m.def("linear(Tensor x, Tensor weight, Tensor? bias=None, int act=0, Tensor? residual=None, float drop_p=0.0, "
        "Tensor? seed=None, int site=0, bool out_f32=False, Tensor? weight_lp=None) -> Tensor");
  m.def("linear_backward(Tensor grad, Tensor x, Tensor weight, bool need_dx, bool need_dw, bool need_db) "
        "-> (Tensor, Tensor, Tensor)");
  m.def("ffn(Tensor x, Tensor w1, Tensor b1, Tensor w2, Tensor b2, float drop_p=0.0, Tensor? seed=None, int site=0, "
        "Tensor? w1_lp=None, Tensor? w2_lp=None) -> (Tensor, Tensor)");
  m.def("ffn_backward(Tensor grad, Tensor x, Tensor hidden, Tensor w1, Tensor w2, float drop_p) "
        "-> (Tensor, Tensor, Tensor, Tensor, Tensor)");
  m.def("layer_norm(Tensor x, Tensor gamma, Tensor beta, float eps, Tensor? residual=None) -> Tensor");
  m.def("layer_norm_train(Tensor x, Tensor gamma, Tensor beta, float eps, Tensor? residual=None, float drop_p=0.0, "
        "Tensor? seed=None, int site=0) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("layer_norm_backward(Tensor grad, Tensor z, Tensor mean, Tensor rstd, Tensor gamma, float drop_p, "
        "Tensor? seed, int site, bool has_residual) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("attention(Tensor q, Tensor k, Tensor v, int heads, bool causal=False, float scale=0.125) -> Tensor");
  m.def("attention_train(Tensor q, Tensor k, Tensor v, int heads, bool causal=False, float scale=0.125, "
        "Tensor? key_tokens=None, int pad_idx=-1, float drop_p=0.0, Tensor? seed=None, int site=0) -> (Tensor, Tensor)");
  m.def("attention_backward(Tensor grad, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, int heads, bool causal, "
        "float scale, Tensor? key_tokens, int pad_idx, float drop_p, Tensor? seed, int site) -> (Tensor, Tensor, Tensor)");
  m.def("embedding(Tensor tokens, Tensor table, Tensor pe, float scale, float drop_p=0.0, Tensor? seed=None, "
        "int site=0, Tensor? table_lp=None, int pad_idx=-1) -> Tensor");
  m.def("embedding_backward(Tensor grad, Tensor tokens, int V, float scale, float drop_p, Tensor? seed, int site, "
        "int pad_idx) -> Tensor");
  m.def("cross_entropy(Tensor logits, Tensor targets, int ignore_index=-100) -> (Tensor, Tensor)");
  m.def("clip_adamw_step(Tensor(a!) param, Tensor grad, Tensor(b!) exp_avg, Tensor(c!) exp_avg_sq, Tensor(d!)? shadow, "
        "Tensor(e!) step, Tensor lr, Tensor(f!) norm_out, Tensor(g!) ws, float max_norm, float beta1, float beta2, "
        "float eps, float weight_decay) -> ()");
}

// ROCm builds of torch dispatch device tensors under the CUDA key
TORCH_LIBRARY_IMPL(mit_hip, CUDA, m) {
  m.impl("linear", &linear);
  m.impl("linear_backward", &linear_backward);
  m.impl("ffn", &ffn);
  m.impl("ffn_backward", &ffn_backward);
  m.impl("layer_norm", &layer_norm);
  m.impl("layer_norm_train", &layer_norm_train);
  m.impl("layer_norm_backward", &layer_norm_backward);
  m.impl("attention", &attention);
  m.impl("attention_train", &attention_train);
  m.impl("attention_backward", &attention_backward);
  m.impl("embedding", &embedding);
  m.impl("embedding_backward", &embedding_backward);
  m.impl("cross_entropy", &cross_entropy);
  m.impl("clip_adamw_step", &clip_adamw_step);
}
