"""Mask helpers with the reference's names (utils.py:11-70).

The kernels never materialise these masks (attention computes causal and key-padding masking from
``j > i`` and ``tokens == PAD`` in-kernel); the functions are kept for API compatibility and for
tests. Unlike the reference's create_padding_mask (utils.py:70, ``.to(config.DEVICE)`` = cuda:0),
the mask stays on the input's device, which is what a multi-GPU process needs.
"""
import torch

import config


def generate_square_subsequent_mask(sz: int, device=None) -> torch.Tensor:
    """[sz, sz] f32: 0 on and below the diagonal, -inf above (utils.py:11-37)."""
    return torch.triu(torch.full((sz, sz), float("-inf"), device=device), diagonal=1)


def create_padding_mask(seq: torch.Tensor, pad_idx: int = config.PAD_TOKEN_ID) -> torch.Tensor:
    """[B, T] bool, True where seq == pad_idx (utils.py:47-70), on seq's device."""
    return seq == pad_idx
