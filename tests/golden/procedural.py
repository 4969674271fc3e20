"""Procedural (seeded) inputs and weights shared by the fixture generator and the tests.

TEST INFRASTRUCTURE ONLY. Nothing in the product path imports this module.

The golden fixtures under ``tests/golden/*.safetensors`` store the reference's OUTPUTS only;
the inputs (images, captions) and every weight are regenerated here from a seed with torch's CPU
generator, which is deterministic for a given torch build (the same image runs here and on the GPU
box). Each fixture stores a checksum of the regenerated weights and inputs so that a drift in the
generator is caught before any numerics are compared.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List, Sequence, Tuple

import torch

Spec = List[Tuple[str, Tuple[int, ...]]]


def _is_norm_weight(name: str) -> bool:
    leaf = name.rsplit(".", 2)
    owner = leaf[-2] if len(leaf) >= 2 else ""
    return name.endswith(".weight") and ("norm" in owner or "layrnorm" in owner)


def make_state(spec: Spec, seed: int) -> Dict[str, torch.Tensor]:
    """Seeded weights for a list of (name, shape) pairs, in list order.

    Initialisation family per name (scales chosen so activations stay O(1) through deep stacks):
      * LayerNorm weights: 1 + 0.1 * N(0,1); biases of any kind: 0.05 * N(0,1)
      * CLS / position / class embeddings: 0.1 * N(0,1)
      * every other tensor with >= 2 dims: N(0,1) / sqrt(fan_in), fan_in = prod(shape[1:])
    """
    g = torch.Generator().manual_seed(seed)
    out: Dict[str, torch.Tensor] = {}
    for name, shape in spec:
        x = torch.randn(*shape, generator=g, dtype=torch.float32)
        if _is_norm_weight(name):
            x = 1.0 + 0.1 * x
        elif name.endswith("bias"):
            x = 0.05 * x
        elif any(k in name for k in ("cls_token", "position_embedding", "class_embedding")):
            x = 0.1 * x
        elif len(shape) >= 2:
            fan_in = 1
            for s in shape[1:]:
                fan_in *= s
            x = x / math.sqrt(fan_in)
        else:
            x = 0.05 * x
        out[name] = x
    return out


def make_images(b: int, size: int, seed: int) -> torch.Tensor:
    """'Already normalised' synthetic images, f32 NCHW."""
    g = torch.Generator().manual_seed(seed)
    return torch.randn(b, 3, size, size, generator=g, dtype=torch.float32)


def make_captions(b: int, length: int, vocab: int, seed: int, lengths: Sequence[int] | None = None,
                  start_id: int = 2, pad_id: int = 0) -> torch.Tensor:
    """Caption ids [b, length] int64: col 0 = START, body uniform in [4, vocab), PAD tails.

    ``lengths[i]`` is the number of non-PAD ids in row i (>= 2 so no decoder row is all PAD).
    """
    g = torch.Generator().manual_seed(seed)
    cap = torch.randint(4, vocab, (b, length), generator=g, dtype=torch.int64)
    cap[:, 0] = start_id
    if lengths is not None:
        for i, n in enumerate(lengths):
            cap[i, n:] = pad_id
    return cap


def checksum(tensors: Iterable[torch.Tensor]) -> float:
    """Order-sensitive float64 checksum of a sequence of tensors."""
    acc = 0.0
    for i, t in enumerate(tensors):
        t64 = t.detach().double().flatten()
        w = torch.arange(1, t64.numel() + 1, dtype=torch.float64) % 97 + 1
        acc += (i + 1) * float((t64 * w).sum())
    return acc


def sample_index(numel: int, k: int, seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    k = min(k, numel)
    return torch.randperm(numel, generator=g)[:k]


def pil_like_image(h: int, w: int, seed: int) -> torch.Tensor:
    """uint8 HWC image used for the generate() fixtures (smooth pattern + noise)."""
    g = torch.Generator().manual_seed(seed)
    yy = torch.linspace(0, 1, h).view(h, 1, 1)
    xx = torch.linspace(0, 1, w).view(1, w, 1)
    ch = torch.tensor([0.2, 0.5, 0.8]).view(1, 1, 3)
    base = 0.5 + 0.4 * torch.sin(6.0 * xx + 4.0 * yy + 3.0 * ch)
    noise = 0.08 * torch.randn(h, w, 3, generator=g)
    return ((base + noise).clamp(0, 1) * 255).round().to(torch.uint8)
