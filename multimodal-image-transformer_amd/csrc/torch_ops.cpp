// torch_ops.cpp — the PyTorch operator surface over the C ABI (include/mit_hip.h): TORCH_LIBRARY(mit_hip)
// registers the decoder layer's and the encoder's hot ops as dispatcher ops, so torch code (and
// torch.cuda.graphs capture) sees typed operators instead of opaque ctypes calls. Each op allocates its
// output with torch, takes torch's current HIP stream and forwards to the C entry point; the kernels
// are the same ones native.py drives. Built by the Makefile into ../lib/libmit_torch_ops.so (linked
// against libmit_hip.so) and loaded with torch.ops.load_library (native.load_torch_ops).
//
// What each op replaces in the reference (file:line under /root/reference or the torch / transformers
// code it dispatches to), bf16 or f32 operands, f32 parameters (bias, gamma, beta):
//   mit_hip::linear     F.linear / nn.Linear + activation + residual add: torch/nn/functional.py:6435
//                       (MHA packed in_proj), torch/nn/modules/transformer.py:1197-1199 (linear1 +
//                       ReLU, linear2), decoder.py:124 (fc_out), modeling_vit.py:213-215,233,249-254
//   mit_hip::layer_norm nn.LayerNorm of x + residual (the post-LN blocks, transformer.py:1144-1153;
//                       the ViT / CLIP pre-LN, modeling_vit.py:274,281)
//   mit_hip::attention  F.scaled_dot_product_attention inside nn.MultiheadAttention
//                       (torch/nn/functional.py:6370-6404), the decoder's causal self-attention and
//                       cross-attention (decoder.py:112-120) and the encoder MHSA (modeling_vit.py:164-189)
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "../../include/mit_hip.h"

namespace {

// torch's current stream on the current device (ROCm torch keeps device tensors under the CUDA device
// type; its HIP streams "masquerade" as CUDA ones)
hipStream_t stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

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

void check_dev(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "mit_hip: ", name, " must be a ROCm device tensor (there is no CPU fallback)");
}

// [..., K] -> rows x K with unit column stride (a view when possible)
at::Tensor rows2d(const at::Tensor& x) {
  at::Tensor c = x.stride(-1) == 1 ? x : x.contiguous();
  if (c.dim() == 2) return c;
  return c.reshape({-1, c.size(-1)});
}

// y = act(x W^T + bias) + residual ; x [..., K], W [N, K] (nn.Linear layout), bias f32 [N],
// residual [..., N] in x's dtype
at::Tensor linear(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias, int64_t act,
                  const c10::optional<at::Tensor>& residual) {
  check_dev(x, "x");
  check_dev(w, "weight");
  TORCH_CHECK(x.scalar_type() == w.scalar_type(), "mit_hip::linear: x and weight dtypes differ");
  TORCH_CHECK(w.dim() == 2 && x.size(-1) == w.size(1), "mit_hip::linear: weight must be [N, K] with K = x.size(-1)");
  TORCH_CHECK(act >= MIT_ACT_NONE && act <= MIT_ACT_QUICK_GELU, "mit_hip::linear: bad activation code ", act);
  const c10::DeviceGuard guard(x.device());
  const at::Tensor a = rows2d(x), b = w.stride(1) == 1 ? w : w.contiguous();
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  std::vector<int64_t> shape(x.sizes().begin(), x.sizes().end());
  shape.back() = N;
  at::Tensor y = at::empty(shape, x.options());
  at::Tensor bias_f, res;
  if (bias) {
    bias_f = bias->to(at::kFloat).contiguous();
    TORCH_CHECK(bias_f.numel() == N, "mit_hip::linear: bias must have N elements");
  }
  if (residual) {
    TORCH_CHECK(residual->scalar_type() == x.scalar_type() && residual->size(-1) == N &&
                    residual->numel() == M * N, "mit_hip::linear: residual must be [..., N] in x's dtype");
    res = rows2d(*residual);
  }
  mit_gemm_args g{};
  g.dtype = dtype_code(x);
  g.a_layout = MIT_K_CONTIG;
  g.b_layout = MIT_K_CONTIG;
  g.M = M;
  g.N = N;
  g.K = K;
  g.A = a.data_ptr();
  g.lda = a.stride(0);
  g.B = b.data_ptr();
  g.ldb = b.stride(0);
  g.C = y.data_ptr();
  g.ldc = N;
  g.alpha = 1.0f;
  g.bias = bias ? bias_f.data_ptr<float>() : nullptr;
  g.act = (int)act;
  g.residual = residual ? res.data_ptr() : nullptr;
  g.ldr = residual ? res.stride(0) : 0;
  g.out_f32 = g.dtype == MIT_F32;
  check_rc(mit_gemm(&g, stream()), "mit_hip::linear");
  return y;
}

// y = LN(x + residual) over the last dim, f32 statistics; gamma / beta f32 [C]
at::Tensor layer_norm(const at::Tensor& x, const at::Tensor& gamma, const at::Tensor& beta, double eps,
                      const c10::optional<at::Tensor>& residual) {
  check_dev(x, "x");
  const c10::DeviceGuard guard(x.device());
  const at::Tensor a = rows2d(x);
  const int64_t R = a.size(0), C = a.size(1);
  const at::Tensor g = gamma.to(at::kFloat).contiguous(), bt = beta.to(at::kFloat).contiguous();
  TORCH_CHECK(g.numel() == C && bt.numel() == C, "mit_hip::layer_norm: gamma / beta must have x.size(-1) elements");
  at::Tensor res;
  if (residual) {
    TORCH_CHECK(residual->scalar_type() == x.scalar_type() && residual->numel() == x.numel(),
                "mit_hip::layer_norm: residual must match x");
    res = rows2d(*residual);
  }
  at::Tensor y = at::empty(x.sizes(), x.options());
  check_rc(mit_layernorm_fwd(dtype_code(x), R, C, a.data_ptr(), a.stride(0), residual ? res.data_ptr() : nullptr,
                             residual ? res.stride(0) : 0, 0.f, nullptr, 0u, g.data_ptr<float>(), bt.data_ptr<float>(),
                             (float)eps, nullptr, y.data_ptr(), C, nullptr, nullptr,
                             stream()),
           "mit_hip::layer_norm");
  return y;
}

// o = softmax(q k^T * scale [+ causal mask]) v per head; q [B, Lq, H*Dh], k / v [B, Lk, H*Dh] (token
// rows with the heads interleaved, as nn.MultiheadAttention's packed projections leave them; the
// last dim contiguous, any row / batch strides), o [B, Lq, H*Dh]
at::Tensor attention(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, int64_t heads, bool causal,
                     double scale) {
  check_dev(q, "q");
  TORCH_CHECK(q.dim() == 3 && k.dim() == 3 && v.dim() == 3, "mit_hip::attention: q, k, v must be [B, L, H*Dh]");
  TORCH_CHECK(q.scalar_type() == k.scalar_type() && q.scalar_type() == v.scalar_type(),
              "mit_hip::attention: q, k, v dtypes differ");
  TORCH_CHECK(q.stride(2) == 1 && k.stride(2) == 1 && v.stride(2) == 1, "mit_hip::attention: last dim must be contiguous");
  const int64_t B = q.size(0), Lq = q.size(1), E = q.size(2), Lk = k.size(1);
  TORCH_CHECK(heads > 0 && E % heads == 0 && k.size(2) == E && v.size(2) == E && k.size(0) == B && v.size(0) == B &&
                  v.size(1) == Lk, "mit_hip::attention: shape mismatch");
  const c10::DeviceGuard guard(q.device());
  at::Tensor o = at::empty({B, Lq, E}, q.options());
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
  a.o_row = E;
  a.o_batch = Lq * E;
  a.causal = causal ? 1 : 0;
  a.pad_idx = -1;
  a.scale = (float)scale;
  check_rc(mit_attention_fwd(dtype_code(q), B, heads, Lq, Lk, E / heads, &a, stream()),
           "mit_hip::attention");
  return o;
}

}  // namespace

TORCH_LIBRARY(mit_hip, m) {
  m.def("linear(Tensor x, Tensor weight, Tensor? bias=None, int act=0, Tensor? residual=None) -> Tensor");
  m.def("layer_norm(Tensor x, Tensor gamma, Tensor beta, float eps, Tensor? residual=None) -> Tensor");
  m.def("attention(Tensor q, Tensor k, Tensor v, int heads, bool causal=False, float scale=0.125) -> Tensor");
}

// ROCm builds of torch dispatch device tensors under the CUDA key
TORCH_LIBRARY_IMPL(mit_hip, CUDA, m) {
  m.impl("linear", &linear);
  m.impl("layer_norm", &layer_norm);
  m.impl("attention", &attention);
}
