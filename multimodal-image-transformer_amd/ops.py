"""torch.ops.mit_hip: the PyTorch-ROCm operator library (csrc/torch_ops.cpp, TORCH_LIBRARY over the C ABI)
with its autograd formulas and fake (meta) kernels registered here through torch.library.

    import ops
    mh = ops.load()                       # torch.ops.mit_hip, autograd + fake kernels registered
    y = mh.linear(x, w, b, weight_lp=w_bf16)   # differentiable in x, w (f32 master), b

Each forward op's backward is another op of the same library (linear_backward, ffn_backward,
layer_norm_backward, attention_backward, embedding_backward), so ``loss.backward()`` through these ops
runs the same HIP kernels the fused train step does. ImageToTextModel.__call__ builds its autograd
graph from them (model.ImageToTextModel.forward -> decoder.TransformerDecoder.forward_ops): the
reference loop (train.py:80-100: model(images, tokens) -> criterion -> loss.backward()) dispatches
through torch.ops.mit_hip. The fake kernels give output shapes without running anything (torch.compile /
FakeTensor tracing).

Differentiable inputs: linear (x, weight, bias, residual; act = NONE and drop_p = 0 when a gradient is
needed), ffn (x, w1, b1, w2, b2), layer_norm_train (x, gamma, beta, residual), attention_train (q, k, v),
embedding (table), cross_entropy (logits). The extra outputs (z / mean / rstd of layer_norm_train, lse of
attention_train, the hidden of ffn, dlogits of cross_entropy) are saved state, not differentiable.
"""
from __future__ import annotations

import torch

import native

_registered = False


def _lib_ops():
    return torch.ops.mit_hip


def _gemm_w(w, w_lp):
    return w_lp if w_lp is not None else w


def _as(t, like):
    return t if t is None or t.dtype == like.dtype else t.to(like.dtype)


# ---- linear ------------------------------------------------------------------------------------------
def _linear_setup(ctx, inputs, output):
    x, w, bias, act, residual, drop_p, seed, site, out_f32, w_lp = inputs
    ctx.act, ctx.drop_p = act, drop_p
    ctx.has_bias, ctx.has_res = bias is not None, residual is not None
    ctx.save_for_backward(x, _gemm_w(w, w_lp), w)


def _linear_backward(ctx, gy):
    x, wg, w = ctx.saved_tensors
    need = ctx.needs_input_grad
    if (need[0] or need[1] or need[2]) and (ctx.act != native.ACT_NONE or ctx.drop_p > 0):
        raise NotImplementedError("mit_hip::linear: gradients through a fused activation / dropout epilogue are "
                                  "not implemented (use mit_hip::ffn for linear2(dropout(relu(linear1(x)))))")
    dx, dw, db = _lib_ops().linear_backward(gy, x, wg, bool(need[0]), bool(need[1]), bool(need[2] and ctx.has_bias))
    dres = gy if ctx.has_res and need[4] else None
    return (dx if need[0] else None, _as(dw, w) if need[1] else None, db if need[2] else None, None, dres,
            None, None, None, None, None)


# ---- feed-forward block ------------------------------------------------------------------------------
def _ffn_setup(ctx, inputs, output):
    x, w1, b1, w2, b2, drop_p, seed, site, w1_lp, w2_lp = inputs
    ctx.drop_p = drop_p
    ctx.mark_non_differentiable(output[1])
    ctx.save_for_backward(x, output[1], _gemm_w(w1, w1_lp), _gemm_w(w2, w2_lp), w1, w2)


def _ffn_backward(ctx, gy, gh):
    x, h, w1g, w2g, w1, w2 = ctx.saved_tensors
    dx, dw1, db1, dw2, db2 = _lib_ops().ffn_backward(gy, x, h, w1g, w2g, ctx.drop_p)
    return dx, _as(dw1, w1), db1, _as(dw2, w2), db2, None, None, None, None, None


# ---- LayerNorm -----------------------------------------------------------------------------------------
def _ln_setup(ctx, inputs, output):
    x, gamma, beta, eps, residual, drop_p, seed, site = inputs
    y, z, mean, rstd = output
    ctx.mark_non_differentiable(z, mean, rstd)
    ctx.drop_p, ctx.site, ctx.has_res = drop_p, site, residual is not None
    ctx.save_for_backward(z, mean, rstd, gamma, seed if seed is not None else torch.empty(0))
    ctx.has_seed = seed is not None


def _ln_backward(ctx, gy, gz, gm, gr):
    z, mean, rstd, gamma, seed = ctx.saved_tensors
    dx, dr, dgamma, dbeta = _lib_ops().layer_norm_backward(gy, z, mean, rstd, gamma, ctx.drop_p,
                                                           seed if ctx.has_seed else None, ctx.site, ctx.has_res)
    return dx, _as(dgamma, gamma), _as(dbeta, gamma), None, dr if ctx.has_res else None, None, None, None


# ---- attention -----------------------------------------------------------------------------------------
def _attn_setup(ctx, inputs, output):
    q, k, v, heads, causal, scale, key_tokens, pad_idx, drop_p, seed, site = inputs
    o, lse = output
    ctx.mark_non_differentiable(lse)
    ctx.meta = (heads, causal, scale, pad_idx, drop_p, site, key_tokens is not None, seed is not None)
    e = torch.empty(0)
    ctx.save_for_backward(q, k, v, o, lse, key_tokens if key_tokens is not None else e, seed if seed is not None else e)


def _attn_backward(ctx, go, glse):
    q, k, v, o, lse, kt, seed = ctx.saved_tensors
    heads, causal, scale, pad_idx, drop_p, site, has_kt, has_seed = ctx.meta
    dq, dk, dv = _lib_ops().attention_backward(go, q, k, v, o, lse, heads, causal, scale, kt if has_kt else None,
                                               pad_idx, drop_p, seed if has_seed else None, site)
    return dq, dk, dv, None, None, None, None, None, None, None, None


# ---- token embedding -------------------------------------------------------------------------------------
def _emb_setup(ctx, inputs, output):
    tokens, table, pe, scale, drop_p, seed, site, table_lp, pad_idx = inputs
    ctx.meta = (table.shape[0], scale, drop_p, site, pad_idx, seed is not None)
    ctx.save_for_backward(tokens, seed if seed is not None else torch.empty(0), table)


def _emb_backward(ctx, gx):
    tokens, seed, table = ctx.saved_tensors
    V, scale, drop_p, site, pad_idx, has_seed = ctx.meta
    dt = _lib_ops().embedding_backward(gx, tokens, V, scale, drop_p, seed if has_seed else None, site, pad_idx)
    return None, _as(dt, table), None, None, None, None, None, None, None


# ---- cross-entropy -----------------------------------------------------------------------------------------
def _ce_setup(ctx, inputs, output):
    loss, dlogits = output
    ctx.mark_non_differentiable(dlogits)
    ctx.save_for_backward(dlogits)


def _ce_backward(ctx, gloss, gd):
    (dl,) = ctx.saved_tensors
    return dl * gloss.to(dl.dtype), None, None


def _register():
    L = torch.library
    L.register_autograd("mit_hip::linear", _linear_backward, setup_context=_linear_setup)
    L.register_autograd("mit_hip::ffn", _ffn_backward, setup_context=_ffn_setup)
    L.register_autograd("mit_hip::layer_norm_train", _ln_backward, setup_context=_ln_setup)
    L.register_autograd("mit_hip::attention_train", _attn_backward, setup_context=_attn_setup)
    L.register_autograd("mit_hip::embedding", _emb_backward, setup_context=_emb_setup)
    L.register_autograd("mit_hip::cross_entropy", _ce_backward, setup_context=_ce_setup)

    # fake (meta) kernels: output shapes / dtypes only
    @L.register_fake("mit_hip::linear")
    def _(x, w, bias=None, act=0, residual=None, drop_p=0.0, seed=None, site=0, out_f32=False, weight_lp=None):
        return x.new_empty(x.shape[:-1] + (w.shape[0],), dtype=torch.float32 if out_f32 else x.dtype)

    @L.register_fake("mit_hip::linear_backward")
    def _(g, x, w, need_dx, need_dw, need_db):
        f = torch.float32
        return (x.new_empty(x.shape) if need_dx else None, x.new_empty(w.shape, dtype=f) if need_dw else None,
                x.new_empty((w.shape[0],), dtype=f) if need_db else None)

    @L.register_fake("mit_hip::ffn")
    def _(x, w1, b1, w2, b2, drop_p=0.0, seed=None, site=0, w1_lp=None, w2_lp=None):
        return x.new_empty(x.shape[:-1] + (w2.shape[0],)), x.new_empty(x.shape[:-1] + (w1.shape[0],))

    @L.register_fake("mit_hip::ffn_backward")
    def _(g, x, h, w1, w2, drop_p):
        f = torch.float32
        return (x.new_empty(x.shape), x.new_empty(w1.shape, dtype=f), x.new_empty((w1.shape[0],), dtype=f),
                x.new_empty(w2.shape, dtype=f), x.new_empty((w2.shape[0],), dtype=f))

    @L.register_fake("mit_hip::layer_norm")
    def _(x, gamma, beta, eps, residual=None):
        return x.new_empty(x.shape)

    @L.register_fake("mit_hip::layer_norm_train")
    def _(x, gamma, beta, eps, residual=None, drop_p=0.0, seed=None, site=0):
        R = x.numel() // x.shape[-1]
        return (x.new_empty(x.shape), x.new_empty(x.shape), x.new_empty((R,), dtype=torch.float32),
                x.new_empty((R,), dtype=torch.float32))

    @L.register_fake("mit_hip::layer_norm_backward")
    def _(g, z, mean, rstd, gamma, drop_p, seed, site, has_residual):
        C = z.shape[-1]
        return (z.new_empty(z.shape), z.new_empty(z.shape) if has_residual else None,
                z.new_empty((C,), dtype=torch.float32), z.new_empty((C,), dtype=torch.float32))

    @L.register_fake("mit_hip::attention")
    def _(q, k, v, heads, causal=False, scale=0.125):
        return q.new_empty(q.shape)

    @L.register_fake("mit_hip::attention_train")
    def _(q, k, v, heads, causal=False, scale=0.125, key_tokens=None, pad_idx=-1, drop_p=0.0, seed=None, site=0):
        return q.new_empty(q.shape), q.new_empty((q.shape[0] * heads * q.shape[1],), dtype=torch.float32)

    @L.register_fake("mit_hip::attention_backward")
    def _(g, q, k, v, o, lse, heads, causal, scale, key_tokens, pad_idx, drop_p, seed, site):
        return q.new_empty(q.shape), k.new_empty(k.shape), v.new_empty(v.shape)

    @L.register_fake("mit_hip::embedding")
    def _(tokens, table, pe, scale, drop_p=0.0, seed=None, site=0, table_lp=None, pad_idx=-1):
        t = table_lp if table_lp is not None else table
        return t.new_empty(tuple(tokens.shape) + (t.shape[1],))

    @L.register_fake("mit_hip::embedding_backward")
    def _(g, tokens, V, scale, drop_p, seed, site, pad_idx):
        return g.new_empty((V, g.shape[-1]), dtype=torch.float32)

    @L.register_fake("mit_hip::cross_entropy")
    def _(logits, targets, ignore_index=-100):
        return logits.new_empty((), dtype=torch.float32), logits.new_empty(logits.shape)

    @L.register_fake("mit_hip::clip_adamw_step")
    def _(param, grad, exp_avg, exp_avg_sq, shadow, step, lr, norm_out, ws, max_norm, beta1, beta2, eps, wd):
        return None


def load():
    """Load libmit_torch_ops.so (native.load_torch_ops) and register the autograd formulas and fake kernels
    once. Returns torch.ops.mit_hip."""
    global _registered
    mh = native.load_torch_ops()
    if not _registered:
        _register()
        _registered = True
    return mh
