"""Loading helpers for the golden fixtures (tests/golden/*.safetensors). Test infrastructure only."""
from __future__ import annotations

import json
import os
import sys
from functools import lru_cache

import torch
from safetensors import safe_open

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLDEN)
import procedural as P  # noqa: E402

# every BASELINE config is pinned by one of these: configs[0] = cfg0_b4_* (d128 / 8 heads = head_dim 16),
# configs[1] = cfg1_b2_patches, configs[2] = cfg2_b2_patches (CLIP-L/14@336, S = 577),
# configs[3] = cfg3_b2_patches (+ dp2_tiny for the data-parallel step), configs[4] = cfg1_gen_cls;
# tiny_vit_v509 has a vocabulary that is not a multiple of 8
CASES = ["tiny_vit_cls", "tiny_vit_patches", "tiny_clip336_patches", "tiny_clip336_cls", "cfg1_b2_patches",
         "cfg3_b2_patches", "cfg0_b4_cls", "cfg0_b4_patches", "cfg2_b2_patches", "tiny_vit_v509"]


@lru_cache(maxsize=None)
def load(name: str):
    path = os.path.join(GOLDEN, f"{name}.safetensors")
    with safe_open(path, "pt") as f:
        meta = json.loads(f.metadata()["meta"])
        tensors = {k: f.get_tensor(k) for k in f.keys()}
    return meta, tensors


@lru_cache(maxsize=None)
def load_dense(name: str):
    """The denser gradient pins of a fixture (tests/golden/make_grad_dense.py: 1024 elements per tensor of
    more than 4096, a superset of the fixture's 64), as {tensor name: (index LongTensor, reference values)};
    None for fixtures without them."""
    path = os.path.join(GOLDEN, f"{name}.grad_dense.safetensors")
    if not os.path.exists(path):
        return None
    with safe_open(path, "pt") as f:
        meta = json.loads(f.metadata()["meta"])
        vals = {k[len("grad1.dense."):]: f.get_tensor(k) for k in f.keys()}
    fx_meta, _ = load(name)
    numel = {n: int(torch.tensor(s).prod()) for n, s in fx_meta["spec"]}
    return {n: (P.sample_index(numel[n], meta["k"], meta["seeds"][n]), v) for n, v in vals.items()}


def enc_desc(meta) -> dict:
    """Encoder geometry from the fixture's HF config kwargs (ViTConfig()/CLIPVisionConfig() defaults)."""
    c = dict(meta["enc_cfg"])
    if meta["enc_kind"] == "vit":
        base = dict(hidden_size=768, num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072,
                    image_size=224, patch_size=16, eps=1e-12)
    else:
        base = dict(hidden_size=768, num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072,
                    image_size=224, patch_size=32, eps=1e-5)
    base.update(c)
    return {"kind": meta["enc_kind"], "hidden": base["hidden_size"], "layers": base["num_hidden_layers"],
            "heads": base["num_attention_heads"], "mlp": base["intermediate_size"],
            "image": base["image_size"], "patch": base["patch_size"], "eps": base["eps"]}


def dec_desc(meta) -> dict:
    d = meta["dec"]
    return {"vocab": d["vocab"], "d": d["embed_dim"], "heads": d["heads"], "layers": d["layers"],
            "ff": d["ff"], "max_seq_len": d.get("max_seq_len", 100)}


def state(meta):
    spec = [(n, tuple(s)) for n, s in meta["spec"]]
    st = P.make_state(spec, meta["seed"])
    chk = P.checksum(st[n] for n, _ in spec)
    assert abs(chk - meta["weights_checksum"]) <= 1e-9 * max(1.0, abs(chk)), "procedural weights drifted"
    return st


def inputs(meta, step: int = 0):
    imgs = P.make_images(meta["B"], meta["image_size"], meta["seed"] + 1)
    cap = P.make_captions(meta["B"], meta["cap_len"], meta["dec"]["vocab"], meta["seed"] + 2 + step,
                          meta["lengths"])
    return imgs, cap[:, :-1].contiguous(), cap[:, 1:].contiguous()


def logits_at(meta, T, logits):
    """The reference logits a fixture pins and ours at the same places: full [B,T,V], or the
    row-sampled positions ("fwd.logits_sel", meta["logit_sel"] = [[b, t], ...])."""
    if "fwd.logits" in T:
        return logits, T["fwd.logits"]
    sel = meta["logit_sel"]
    got = torch.stack([logits[b, t] for b, t in sel])
    return got, T["fwd.logits_sel"]


def encoder_rows(T, feats):
    """(ours, reference) pairs for the encoder's last_hidden_state entries a fixture holds."""
    if "enc.last_hidden_state" in T:
        return [(feats, T["enc.last_hidden_state"])]
    return [(feats[:, 0], T["enc.cls_rows"]), (feats[:, 17], T["enc.row17"]), (feats[:, -1], T["enc.row_last"])]


def trainable_names(meta):
    return [n for n, _ in meta["spec"] if not n.startswith("encoder.")]


def degenerate_mask(name: str, t: torch.Tensor, meta=None):
    """Elements whose reference gradient is exactly 0 in real arithmetic (so the stored value is
    rounding noise, ~1e-10, that AdamW then normalises to an arbitrary +-lr step): the KEY part of a
    packed in_proj_bias — softmax is invariant to a per-row constant, so d(loss)/d(b_k) = 0.
    Returns a bool mask of the elements that ARE pinned, or None."""
    cls_cross = meta is not None and meta.get("mode") == "cls" and "multihead_attn" in name
    if name.endswith("in_proj_bias"):
        d = t.numel() // 3
        m = torch.ones(t.numel(), dtype=torch.bool)
        m[(0 if cls_cross else d):2 * d] = False
        return m
    # cls mode: memory length S = 1 and softmax over one key == 1, so the cross-attention QUERY and
    # KEY projections get exactly-zero gradients as well
    if cls_cross and name.endswith("in_proj_weight"):
        n = t.numel()
        d = int(round((n / 3) ** 0.5))
        m = torch.ones(n, dtype=torch.bool)
        m[:2 * d * d] = False
        return m
    return None


def compare_stat(prefix, name, t, tensors, meta, rtol, atol, scale_tol=0.0, outlier_frac=0.0):
    """Compare a tensor to its fixture entry (full / sample+stats). Returns max abs err on samples.
    scale_tol: absolute tolerance as a fraction of the tensor's max |value| (sum-order noise of
    reductions is relative to the tensor's scale, not to each element)."""
    t = t.detach().float().cpu()
    if scale_tol:
        st_key = f"{prefix}.stats.{name}"
        full_key = f"{prefix}.full.{name}"
        mx = tensors[full_key].abs().max().item() if full_key in tensors else tensors[st_key][2].item()
        atol = max(atol, scale_tol * mx)
    # step-1 AdamW update = -lr * g / (|g| + 1e-9): for |g| below ~1e-8 the last-ulp differences of
    # any other summation order become visible, so such elements are not pinned by the update
    gmin = 1e-8 if prefix == "delta1" else None
    if f"{prefix}.full.{name}" in tensors:
        ref = tensors[f"{prefix}.full.{name}"]
        got = t.reshape(ref.shape)
        m = degenerate_mask(name, ref, meta) if prefix.startswith("delta") else None
        if gmin is not None and f"grad1.full.{name}" in tensors:
            gm = tensors[f"grad1.full.{name}"].flatten().abs() >= gmin
            m = gm if m is None else (m & gm)
        if m is not None:
            got, ref = got.flatten()[m], ref.flatten()[m]
        if got.numel() == 0:  # every element excluded above (degenerate / below the pinning floor)
            return 0.0
        if outlier_frac:
            _assert_close_outliers(got.flatten(), ref.flatten(), rtol, atol, outlier_frac, 10 * atol, f"{prefix} {name}")
        else:
            torch.testing.assert_close(got, ref, rtol=rtol, atol=atol, msg=lambda s: f"{prefix} {name}: {s}")
        return float((got - ref).abs().max())
    idx = torch.tensor(meta["sample_index"][name])
    ref = tensors[f"{prefix}.sample.{name}"]
    got = t.flatten()[idx]
    m = degenerate_mask(name, t.flatten(), meta) if prefix.startswith("delta") else None
    if m is not None:
        got, ref = got[m[idx]], ref[m[idx]]
    if gmin is not None and f"grad1.sample.{name}" in tensors:
        keep = tensors[f"grad1.sample.{name}"].abs() >= gmin
        if m is not None:
            keep = keep[m[idx]]
        got, ref = got[keep], ref[keep]
    if got.numel() == 0:
        return 0.0
    torch.testing.assert_close(got, ref, rtol=rtol, atol=atol, msg=lambda s: f"{prefix} {name}: {s}")
    st = tensors[f"{prefix}.stats.{name}"].double()
    flat = t.flatten().double()
    norm = flat.norm()
    if m is None:
        assert abs(norm - st[1]) <= rtol * abs(st[1]) + atol * flat.numel() ** 0.5, f"{prefix} {name} norm"
    return float((got - ref).abs().max())


def _assert_close_outliers(got, ref, rtol, atol, outlier_frac, outlier_atol, what):
    """assert_close that tolerates up to `outlier_frac` of elements beyond tolerance, each still
    within `outlier_atol` (ReLU-boundary flips: a pre-activation within an ulp of 0 gets a
    different mask under another summation order, moving one row's contribution)."""
    bad = (got - ref).abs() > atol + rtol * ref.abs()
    nbad = int(bad.sum())
    if nbad == 0:
        return
    assert nbad <= max(1, int(outlier_frac * got.numel())), f"{what}: {nbad}/{got.numel()} elements off"
    worst = float((got - ref)[bad].abs().max())
    assert worst <= outlier_atol, f"{what}: outlier error {worst:.3e} > {outlier_atol:.3e}"
