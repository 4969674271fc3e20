"""Fused clip_grad_norm_ + AdamW over the model's flat f32 parameter buffer.

Replaces train.py:96-100 (torch.nn.utils.clip_grad_norm_(model.parameters(), GRAD_CLIP_VALUE) then
optimizer.step()) and the AdamW construction at train.py:319-325. Math is torch/optim/adam.py:419-547
(decoupled weight decay, lerp first moment, bias corrections) with the clip coefficient of
torch/nn/utils/clip_grad.py:165-186 applied to the gradient as it is read. Three launches per step:
sum-of-squares partials + norm finalisation, the step counter, the elementwise update (which also
refreshes the bf16 shadow the GEMMs read). No host synchronisation: lr, the step count and the clip
coefficient live in device memory, so the whole step can be captured in a hipGraph.
"""
from __future__ import annotations

import torch

import native
from params import FlatParams


class AdamW:
    def __init__(self, store: FlatParams, lr=1e-4, betas=(0.9, 0.98), eps=1e-9, weight_decay=1e-5):
        self.store = store
        self.betas, self.eps, self.weight_decay = betas, eps, weight_decay
        store.ensure_optimizer_state()
        dev = store.device
        self.lr_t = torch.full((1,), float(lr), dtype=torch.float32, device=dev)
        self.step_t = torch.zeros(1, dtype=torch.int64, device=dev)
        self.norm_t = torch.zeros(2, dtype=torch.float32, device=dev)  # {total_norm, clip_coef}
        self.ws = torch.empty(native.grad_norm_ws_floats(store.numel), dtype=torch.float32, device=dev)
        self.param_groups = [{"lr": float(lr), "betas": betas, "eps": eps, "weight_decay": weight_decay}]
        self._lr_host = float(lr)

    def zero_grad(self, set_to_none: bool = True):
        """No-op by design: every gradient element is written (not accumulated) by the backward."""

    def _sync_lr(self):
        lr = float(self.param_groups[0]["lr"])
        if lr != self._lr_host:
            self.lr_t.fill_(lr)
            self._lr_host = lr

    def step(self, max_norm: float = 0.0):
        """clip (max_norm > 0) + AdamW. The pre-clip total norm is left in ``self.norm_t[0]``."""
        self._sync_lr()
        st = self.store
        native.grad_norm(st.grad, max_norm if max_norm > 0 else 0.0, self.ws, self.norm_t)
        native.step_inc(self.step_t)
        shadow = st.shadow if st.shadow is not st.master else None
        native.adamw(st.master, st.grad, st.exp_avg, st.exp_avg_sq, shadow, self.norm_t, self.lr_t, self.step_t,
                     self.betas[0], self.betas[1], self.eps, self.weight_decay)

    # checkpoint I/O (train.py:422-436 stores optimizer.state_dict())
    def state_dict(self):
        return {"step": int(self.step_t.item()), "exp_avg": self.store.exp_avg.detach().cpu(),
                "exp_avg_sq": self.store.exp_avg_sq.detach().cpu(), "param_groups": self.param_groups}

    def load_state_dict(self, sd):
        self.step_t.fill_(int(sd["step"]))
        self.store.exp_avg.copy_(sd["exp_avg"])
        self.store.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.param_groups = sd["param_groups"]
        self._lr_host = None
        self._sync_lr()
