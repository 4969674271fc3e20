"""CPU oracle — a plain-PyTorch fp32 functional restatement of the captioning train step.

TEST INFRASTRUCTURE ONLY. Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker / the timed CPU baseline.
The product path (``multimodal-image-transformer_amd/``) never imports it and has no CPU fallback.

Parity pinning: checked against the golden fixtures in ``tests/golden/*.safetensors``, which were
produced by running the reference's own code (model.py / decoder.py / utils.py / train.py) in this
container (``tests/golden/make_fixtures.py``); see ``tests/test_oracle.py``.

Every function below cites the reference (or the third-party code the reference calls) it follows.
Parameters are a flat ``{name: tensor}`` dict in the reference's ``state_dict`` naming:
``encoder.*`` (HF ViT / CLIP vision names, transformers 5.x), ``projection.*``, ``decoder.*``.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

Params = Dict[str, torch.Tensor]


# --------------------------------------------------------------------------------------------
# encoders (frozen, forward only)
# --------------------------------------------------------------------------------------------
def _mhsa(x: torch.Tensor, wq, bq, wk, bk, wv, bv, wo, bo, heads: int) -> torch.Tensor:
    """Bidirectional multi-head self-attention, scale head_dim**-0.5, no mask.
    tf/models/vit/modeling_vit.py:164-238 (eager_attention_forward + ViTAttention)."""
    b, n, e = x.shape
    dh = e // heads
    q = F.linear(x, wq, bq).view(b, n, heads, dh).transpose(1, 2)
    k = F.linear(x, wk, bk).view(b, n, heads, dh).transpose(1, 2)
    v = F.linear(x, wv, bv).view(b, n, heads, dh).transpose(1, 2)
    att = torch.softmax((q @ k.transpose(-1, -2)) * dh ** -0.5, dim=-1)
    o = (att @ v).transpose(1, 2).reshape(b, n, e)
    return F.linear(o, wo, bo)


def vit_forward(p: Params, images: torch.Tensor, *, heads: int, layers: int, patch: int,
                eps: float = 1e-12, prefix: str = "encoder.") -> torch.Tensor:
    """HF ViTModel.forward -> last_hidden_state (tf/models/vit/modeling_vit.py:356-389):
    Conv2d patch embed (60,69), CLS concat + position add (146-157), pre-LN layers (257-286) with
    GELU(erf) MLP (241-254), final LayerNorm (385). Pooler (386) is not observable: skipped."""
    g = lambda k: p[prefix + k]  # noqa: E731
    x = F.conv2d(images, g("embeddings.patch_embeddings.projection.weight"),
                 g("embeddings.patch_embeddings.projection.bias"), stride=patch)
    x = x.flatten(2).transpose(1, 2)
    cls = g("embeddings.cls_token").expand(x.shape[0], -1, -1)
    x = torch.cat([cls, x], dim=1) + g("embeddings.position_embeddings")
    e = x.shape[-1]
    for i in range(layers):
        L = f"layers.{i}."
        h = F.layer_norm(x, (e,), g(L + "layernorm_before.weight"), g(L + "layernorm_before.bias"), eps)
        x = x + _mhsa(h, g(L + "attention.q_proj.weight"), g(L + "attention.q_proj.bias"),
                      g(L + "attention.k_proj.weight"), g(L + "attention.k_proj.bias"),
                      g(L + "attention.v_proj.weight"), g(L + "attention.v_proj.bias"),
                      g(L + "attention.o_proj.weight"), g(L + "attention.o_proj.bias"), heads)
        h = F.layer_norm(x, (e,), g(L + "layernorm_after.weight"), g(L + "layernorm_after.bias"), eps)
        h = F.gelu(F.linear(h, g(L + "mlp.fc1.weight"), g(L + "mlp.fc1.bias")))
        x = x + F.linear(h, g(L + "mlp.fc2.weight"), g(L + "mlp.fc2.bias"))
    return F.layer_norm(x, (e,), g("layernorm.weight"), g("layernorm.bias"), eps)


def clip_vision_forward(p: Params, images: torch.Tensor, *, heads: int, layers: int, patch: int,
                        eps: float = 1e-5, prefix: str = "encoder.") -> torch.Tensor:
    """HF CLIPVisionModel.forward -> last_hidden_state (tf/models/clip/modeling_clip.py:613-657):
    bias-free conv (148-154), class_embedding + position Embedding (212-219), pre_layrnorm (642),
    pre-LN layers with quick_gelu x*sigmoid(1.702x) (tf/activations.py:117-123); the
    last_hidden_state is NOT post-LayerNormed (649)."""
    g = lambda k: p[prefix + k]  # noqa: E731
    x = F.conv2d(images, g("embeddings.patch_embedding.weight"), None, stride=patch)
    x = x.flatten(2).transpose(1, 2)
    cls = g("embeddings.class_embedding").view(1, 1, -1).expand(x.shape[0], -1, -1)
    x = torch.cat([cls, x], dim=1) + g("embeddings.position_embedding.weight").unsqueeze(0)
    e = x.shape[-1]
    x = F.layer_norm(x, (e,), g("pre_layrnorm.weight"), g("pre_layrnorm.bias"), eps)
    for i in range(layers):
        L = f"encoder.layers.{i}."
        h = F.layer_norm(x, (e,), g(L + "layer_norm1.weight"), g(L + "layer_norm1.bias"), eps)
        x = x + _mhsa(h, g(L + "self_attn.q_proj.weight"), g(L + "self_attn.q_proj.bias"),
                      g(L + "self_attn.k_proj.weight"), g(L + "self_attn.k_proj.bias"),
                      g(L + "self_attn.v_proj.weight"), g(L + "self_attn.v_proj.bias"),
                      g(L + "self_attn.out_proj.weight"), g(L + "self_attn.out_proj.bias"), heads)
        h = F.layer_norm(x, (e,), g(L + "layer_norm2.weight"), g(L + "layer_norm2.bias"), eps)
        h = F.linear(h, g(L + "mlp.fc1.weight"), g(L + "mlp.fc1.bias"))
        h = h * torch.sigmoid(1.702 * h)
        x = x + F.linear(h, g(L + "mlp.fc2.weight"), g(L + "mlp.fc2.bias"))
    return x


# --------------------------------------------------------------------------------------------
# decoder
# --------------------------------------------------------------------------------------------
def sinusoidal_pe(max_len: int, d: int) -> torch.Tensor:
    """decoder.py:34-47 (PositionalEncodingBatchFirst buffer), shape [max_len, d]."""
    pos = torch.arange(max_len).unsqueeze(1)
    div = torch.exp(torch.arange(0, d, 2) * (-math.log(10000.0) / d))
    pe = torch.zeros(max_len, d)
    pe[:, 0::2] = torch.sin(pos * div)
    pe[:, 1::2] = torch.cos(pos * div)
    return pe


def _mha(q_in, kv_in, w_in, b_in, w_out, b_out, heads, mask=None, drop=None):
    """F.multi_head_attention_forward with packed in_proj (torch/nn/functional.py:6435),
    additive float mask merged from causal + key padding (6370-6404, 6553-6566), SDPA (6629).
    ``drop``: optional pre-scaled dropout multiplier on the attention probabilities."""
    b, t, d = q_in.shape
    s = kv_in.shape[1]
    dh = d // heads
    q = F.linear(q_in, w_in[:d], b_in[:d]).view(b, t, heads, dh).transpose(1, 2)
    k = F.linear(kv_in, w_in[d:2 * d], b_in[d:2 * d]).view(b, s, heads, dh).transpose(1, 2)
    v = F.linear(kv_in, w_in[2 * d:], b_in[2 * d:]).view(b, s, heads, dh).transpose(1, 2)
    sc = (q @ k.transpose(-1, -2)) / math.sqrt(dh)
    if mask is not None:
        sc = sc + mask
    att = torch.softmax(sc, dim=-1)
    if drop is not None:
        att = att * drop
    o = (att @ v).transpose(1, 2).reshape(b, t, d)
    return F.linear(o, w_out, b_out)


def decoder_forward(p: Params, tokens: torch.Tensor, memory: torch.Tensor, *, heads: int, layers: int,
                    pad_idx: int = 0, max_len: int = 100, prefix: str = "decoder.",
                    drops: Optional[dict] = None, return_hidden: bool = False,
                    memory_padding_mask: Optional[torch.Tensor] = None):
    """decoder.TransformerDecoder.forward (decoder.py:134-193):
    causal mask (utils.py:30-36) + key-padding mask tok==PAD (utils.py:66), Emb*sqrt(d) + PE
    (decoder.py:168-171), L x nn.TransformerDecoderLayer post-LN / ReLU / eps 1e-5
    (torch/nn/modules/transformer.py:1131-1199), fc_out (decoder.py:191).
    ``drops`` (test hook): {site: multiplier tensor} pre-scaled dropout masks, keys
    'emb', f'{i}.sa', f'{i}.d1', f'{i}.ca', f'{i}.d2', f'{i}.ff', f'{i}.d3'.
    ``memory_padding_mask`` bool [B, S] (True = pad): memory_key_padding_mask of the cross-attention
    (decoder.py:179-186), a -inf additive mask on those keys."""
    g = lambda k: p[prefix + k]  # noqa: E731
    dr = drops or {}
    b, t = tokens.shape
    d = g("token_embedding.weight").shape[1]
    causal = torch.triu(torch.full((t, t), float("-inf")), diagonal=1)
    kpm = torch.zeros(b, 1, 1, t).masked_fill((tokens == pad_idx).view(b, 1, 1, t), float("-inf"))
    mask = causal.view(1, 1, t, t) + kpm
    mmask = None
    if memory_padding_mask is not None:
        mmask = torch.zeros(b, 1, 1, memory.shape[1]).masked_fill(memory_padding_mask.view(b, 1, 1, -1), float("-inf"))
    x = F.embedding(tokens, g("token_embedding.weight")) * math.sqrt(d)
    x = x + sinusoidal_pe(max_len, d)[:t].unsqueeze(0)
    if "emb" in dr:
        x = x * dr["emb"]
    for i in range(layers):
        L = f"transformer_decoder.layers.{i}."
        sa = _mha(x, x, g(L + "self_attn.in_proj_weight"), g(L + "self_attn.in_proj_bias"),
                  g(L + "self_attn.out_proj.weight"), g(L + "self_attn.out_proj.bias"), heads, mask,
                  dr.get(f"{i}.sa"))
        if f"{i}.d1" in dr:
            sa = sa * dr[f"{i}.d1"]
        x = F.layer_norm(x + sa, (d,), g(L + "norm1.weight"), g(L + "norm1.bias"), 1e-5)
        ca = _mha(x, memory, g(L + "multihead_attn.in_proj_weight"), g(L + "multihead_attn.in_proj_bias"),
                  g(L + "multihead_attn.out_proj.weight"), g(L + "multihead_attn.out_proj.bias"), heads,
                  mmask, dr.get(f"{i}.ca"))
        if f"{i}.d2" in dr:
            ca = ca * dr[f"{i}.d2"]
        x = F.layer_norm(x + ca, (d,), g(L + "norm2.weight"), g(L + "norm2.bias"), 1e-5)
        h = F.relu(F.linear(x, g(L + "linear1.weight"), g(L + "linear1.bias")))
        if f"{i}.ff" in dr:
            h = h * dr[f"{i}.ff"]
        h = F.linear(h, g(L + "linear2.weight"), g(L + "linear2.bias"))
        if f"{i}.d3" in dr:
            h = h * dr[f"{i}.d3"]
        x = F.layer_norm(x + h, (d,), g(L + "norm3.weight"), g(L + "norm3.bias"), 1e-5)
    logits = F.linear(x, g("fc_out.weight"), g("fc_out.bias"))
    return (logits, x) if return_hidden else logits


# --------------------------------------------------------------------------------------------
# composed model, loss, optimizer
# --------------------------------------------------------------------------------------------
def encode(p: Params, images: torch.Tensor, enc: dict) -> torch.Tensor:
    if enc["kind"] == "vit":
        return vit_forward(p, images, heads=enc["heads"], layers=enc["layers"], patch=enc["patch"],
                           eps=enc.get("eps", 1e-12))
    return clip_vision_forward(p, images, heads=enc["heads"], layers=enc["layers"], patch=enc["patch"],
                               eps=enc.get("eps", 1e-5))


def memory_from_features(p: Params, feats: torch.Tensor, mode: str) -> torch.Tensor:
    """model.py:141-151 (cls: CLS row only, S=1) or the full sequence (patches);
    projection = nn.Linear(e, d) when e != d else Identity (model.py:97-102)."""
    x = feats[:, :1, :] if mode == "cls" else feats
    if "projection.weight" in p:
        x = F.linear(x, p["projection.weight"], p["projection.bias"])
    return x


def model_forward(p: Params, images, tokens, enc: dict, dec: dict, mode: str, drops=None):
    """ImageToTextModel.forward (model.py:116-169): encoder under no_grad, projection, decoder."""
    with torch.no_grad():
        feats = encode(p, images, enc)
    mem = memory_from_features(p, feats, mode)
    return decoder_forward(p, tokens, mem, heads=dec["heads"], layers=dec["layers"],
                           max_len=dec.get("max_seq_len", 100), drops=drops)


def ce_loss(logits: torch.Tensor, targets: torch.Tensor, pad_idx: int = 0) -> torch.Tensor:
    """nn.CrossEntropyLoss(ignore_index=PAD), mean over non-PAD targets (train.py:90,327)."""
    return F.cross_entropy(logits.reshape(-1, logits.shape[-1]), targets.reshape(-1), ignore_index=pad_idx)


def clip_coef(grads: List[torch.Tensor], max_norm: float) -> Tuple[float, float]:
    """torch.nn.utils.clip_grad_norm_ (torch/nn/utils/clip_grad.py:165-186):
    total = ||[||g_i||]||_2 ; coef = min(1, max_norm / (total + 1e-6))."""
    total = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g) for g in grads]))
    coef = min(1.0, float(max_norm / (total + 1e-6)))
    return float(total), coef


class AdamWState:
    """torch.optim.AdamW single-tensor math (torch/optim/adam.py:419-547) with
    lr 1e-4, betas (0.9, 0.98), eps 1e-9, wd 1e-5 (train.py:319-325, config.py:80-90)."""

    def __init__(self, params: Dict[str, torch.Tensor], lr=1e-4, betas=(0.9, 0.98), eps=1e-9, wd=1e-5):
        self.lr, self.b1, self.b2, self.eps, self.wd = lr, betas[0], betas[1], eps, wd
        self.m = {k: torch.zeros_like(v) for k, v in params.items()}
        self.v = {k: torch.zeros_like(v) for k, v in params.items()}
        self.t = 0

    @torch.no_grad()
    def step(self, params: Dict[str, torch.Tensor], grads: Dict[str, torch.Tensor]):
        self.t += 1
        bc1 = 1 - self.b1 ** self.t
        bc2 = 1 - self.b2 ** self.t
        for k, pr in params.items():
            g = grads[k]
            pr.mul_(1 - self.lr * self.wd)                                   # adam.py:419
            self.m[k].lerp_(g, 1 - self.b1)                                  # adam.py:457
            self.v[k].mul_(self.b2).addcmul_(g, g, value=1 - self.b2)        # adam.py:476
            denom = (self.v[k].sqrt() / math.sqrt(bc2)).add_(self.eps)       # adam.py:542
            pr.addcdiv_(self.m[k], denom, value=-self.lr / bc1)              # adam.py:547


def train_step(p: Params, trainable: List[str], opt: AdamWState, images, dec_in, targets,
               enc: dict, dec: dict, mode: str, clip: float, drops=None):
    """One step of train.py:75-100: forward, CE(ignore PAD), backward, clip_grad_norm_, AdamW.
    Returns (loss, pre-clip total norm, post-clip grads dict)."""
    leaves = {k: p[k].detach().clone().requires_grad_(True) for k in trainable}
    q = dict(p)
    q.update(leaves)
    logits = model_forward(q, images, dec_in, enc, dec, mode, drops)
    loss = ce_loss(logits, targets)
    loss.backward()
    grads = {k: leaves[k].grad.detach().clone() for k in trainable}
    total, coef = clip_coef(list(grads.values()), clip) if clip > 0 else (float("nan"), 1.0)
    for g in grads.values():
        g.mul_(coef)
    with torch.no_grad():
        opt.step({k: p[k] for k in trainable}, grads)
    return float(loss.detach()), total, grads


@torch.no_grad()
def greedy_generate(p: Params, pixel_values: torch.Tensor, enc: dict, dec: dict, start: int, end: int,
                    max_len: int = 100, mode: str = "cls") -> List[int]:
    """ImageToTextModel.generate, method='greedy' (model.py:171-242): full-prefix recompute,
    argmax of the last position, stop when END is produced (END kept in the output)."""
    feats = encode(p, pixel_values, enc)
    mem = memory_from_features(p, feats, mode)
    ids = [start]
    for _ in range(max_len - 1):
        logits = decoder_forward(p, torch.tensor([ids]), mem, heads=dec["heads"], layers=dec["layers"],
                                 max_len=dec.get("max_seq_len", 100))
        nxt = int(logits[0, -1].argmax())
        ids.append(nxt)
        if nxt == end:
            break
    return ids


def vit_image_processor(img_hwc_uint8: torch.Tensor, size: int = 224) -> torch.Tensor:
    """ViTImageProcessor defaults (tf/models/vit/image_processing_vit.py; constants
    tf/utils/constants.py:3-4): resize to size x size (PIL bilinear), x/255, (x-0.5)/0.5 -> [1,3,H,W]."""
    from PIL import Image
    import numpy as np
    im = Image.fromarray(img_hwc_uint8.numpy()).resize((size, size), Image.BILINEAR)
    a = torch.from_numpy(np.asarray(im, dtype=np.float32)) / 255.0
    a = (a - 0.5) / 0.5
    return a.permute(2, 0, 1).unsqueeze(0).contiguous()
