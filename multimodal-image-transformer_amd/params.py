"""Flat parameter storage: ONE f32 master buffer, ONE f32 gradient buffer, the AdamW moments, and a
bf16 shadow copy the GEMMs read (bf16 mode). Named tensors are views into these buffers.

Entries are laid out in the order the backward FINISHES them (fc_out first, then decoder layers
top-down, the fused cross-attention K/V block, the embedding, the projection), so a data-parallel
gradient all-reduce can launch contiguous buckets while the rest of the backward still runs.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import torch

import native

ALIGN = 64  # elements: keeps every view 256-B aligned for 16-B vector access in every dtype


class FlatParams:
    def __init__(self, entries: Sequence[Tuple[str, Tuple[int, ...]]], device, compute_dtype: torch.dtype):
        self.entries: List[Tuple[str, Tuple[int, ...], int, int]] = []
        off = 0
        for name, shape in entries:
            n = 1
            for s in shape:
                n *= s
            self.entries.append((name, tuple(shape), off, n))
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        self.index: Dict[str, Tuple[Tuple[int, ...], int, int]] = {e[0]: (e[1], e[2], e[3]) for e in self.entries}
        self.device = device
        self.compute_dtype = compute_dtype
        self.master = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=device)
        if compute_dtype == torch.float32:
            self.shadow = self.master
        else:
            self.shadow = torch.zeros(self.numel, dtype=compute_dtype, device=device)
        self.exp_avg = None
        self.exp_avg_sq = None
        self._synced = self.master._version

    # views (cached: the buffers are allocated once and only ever updated in place) -------------
    def _view(self, buf, name, cache):
        v = cache.get(name)
        if v is None:
            shape, off, n = self.index[name]
            v = cache[name] = buf[off:off + n].view(shape)
        return v

    def p(self, name):
        """f32 master view."""
        return self._view(self.master, name, self.__dict__.setdefault("_pv", {}))

    def w(self, name):
        """compute-dtype view (what kernels read)."""
        return self._view(self.shadow, name, self.__dict__.setdefault("_wv", {}))

    def g(self, name):
        return self._view(self.grad, name, self.__dict__.setdefault("_gv", {}))

    def span(self, first: str, last: str):
        """[start, end) element range covering entries first..last (inclusive, layout order)."""
        s = self.index[first][1]
        _, off, n = self.index[last]
        return s, off + n

    def names(self):
        return [e[0] for e in self.entries]

    # maintenance ------------------------------------------------------------------------------
    def sync_shadow(self):
        """master -> bf16 shadow (after a load / manual edit; AdamW keeps them in sync itself)."""
        if self.shadow is not self.master:
            native.cast_f32(self.master, self.shadow)
        self._synced = self.master._version

    def ensure_shadow(self, force: bool = False):
        """Refresh the bf16 shadow from the f32 master. Without ``force`` only when torch modified the
        master through a parameter view since the last sync (in-place ops on the views, e.g.
        torch.optim.AdamW.step, bump the version counter they share with the master); the fused
        optim.AdamW writes master and shadow in one kernel (no bump, nothing to do). An edit through
        ``p.data`` (``p.data.copy_``, ...) is NOT seen by the version counter (``.data`` is a detached
        alias with its own counter): the non-fused paths (autograd forward, evaluation, generation)
        therefore refresh with ``force=True`` every call (one 1.5-byte-per-parameter cast), and the
        fused train step -- which checks the counter only -- needs ``model.sync_shadow()`` after such
        an out-of-band edit."""
        if self.shadow is not self.master and (force or self.master._version != self._synced):
            self.sync_shadow()

    def zero_grad(self):
        native.zero(self.grad)

    def ensure_optimizer_state(self):
        if self.exp_avg is None:
            self.exp_avg = torch.zeros_like(self.master)
            self.exp_avg_sq = torch.zeros_like(self.master)
