"""Data parallelism for the train step: one process per GPU, torch.distributed over RCCL (backend
"nccl" on ROCm) across xGMI. The reference has no distributed code; this is the
build's DP stack:

  * init: broadcast the flat f32 master buffer (and the frozen encoder) from rank 0;
  * loss semantics: before the backward, all-reduce the non-PAD target COUNT (one f32); each rank
    then backpropagates loss_sum_local / count_global, so the SUM of the ranks' gradients equals
    the single-process reference gradient of nn.CrossEntropyLoss(ignore_index=PAD) at the global
    batch (train.py:90) even when the ranks hold different numbers of PAD targets;
  * gradients: the flat gradient buffer is laid out in backward-completion order, so each
    ``grads_ready(first, last)`` span from the decoder's backward is one contiguous bucket
    (fc_out ~20 MB, one decoder layer ~15 MB, then cross-K/V + embedding + projection ~24 MB at
    cfg1). Each bucket is all-reduced (SUM) asynchronously as soon as it is final; RCCL runs on
    its own stream, ordered after the producing kernels, overlapping the rest of the backward.
    ``finish_backward`` joins the buckets before clip + AdamW, which then run redundantly (and
    identically) on every rank.
"""
from __future__ import annotations

import os
from typing import List

import torch
import torch.distributed as dist

import native


def init_from_env(backend: str = None):
    """torch.distributed init from RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT (torchrun)."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if backend is None:  # MIT_DIST_BACKEND=gloo: rehearse N ranks on one GPU (tools/gpu_dp_smoke.sh)
        backend = os.environ.get("MIT_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group(backend, device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return rank, world


class DataParallel:
    """Gradient synchronisation for a model whose trainable state is one FlatParams store."""

    def __init__(self, model, overlap: bool = True, group=None):
        self.model = model
        self.store = model.store
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.overlap = overlap
        self._work: List = []
        self._pending_spans = []
        self._covered = []  # the spans announced this step: every entry in exactly one (checked on 4 steps)
        self._checks_left = 4
        self._broadcast_state()

    def _broadcast_state(self):
        dist.broadcast(self.store.master, 0, group=self.group)
        self.store.sync_shadow()
        enc = getattr(self.model, "encoder", None)
        if enc is not None:
            for k in sorted(enc.w):
                dist.broadcast(enc.w[k], 0, group=self.group)
        if hasattr(self.model, "set_rank_seed"):
            self.model.set_rank_seed(self.rank)

    # hooks called by model.train_step ------------------------------------------------------------
    def all_reduce_count(self, count: torch.Tensor):
        native.host_call(lambda: dist.all_reduce(count, group=self.group))

    def grads_ready(self, first: str, last: str):
        s, e = self.store.span(first, last)
        self._covered.append((s, e))
        if self.overlap:
            self._work.append(dist.all_reduce(self.store.grad[s:e], group=self.group, async_op=True))
        else:
            self._pending_spans.append((s, e))

    def finish_backward(self, loss: torch.Tensor):
        native.host_call(lambda: self._finish(loss))

    def _finish(self, loss: torch.Tensor):
        spans, self._covered = sorted(self._covered), []
        # host-side bookkeeping only, on the first steps (the buckets are the same every step): every parameter
        # entry in exactly one bucket (a missed or doubly reduced entry would leave the ranks' gradients unequal
        # or scaled); the gaps between entries are alignment
        self._checks_left -= 1
        for name, (_, off, n) in (self.store.index.items() if self._checks_left >= 0 else ()):
            hits = sum(1 for a, b in spans if a <= off and off + n <= b)
            if hits != 1:
                raise RuntimeError(f"DataParallel: gradient entry {name} is in {hits} buckets this step ({spans})")
        if not self.overlap and self._pending_spans:
            s = min(a for a, _ in self._pending_spans)
            e = max(b for _, b in self._pending_spans)
            dist.all_reduce(self.store.grad[s:e], group=self.group)
        for w in self._work:
            w.wait()
        self._work.clear()
        self._pending_spans.clear()
        # loss = loss_sum_local / count_global on each rank -> SUM is the global mean loss
        dist.all_reduce(loss, group=self.group)
