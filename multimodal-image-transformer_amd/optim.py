"""Fused clip_grad_norm_ + AdamW over the model's flat f32 parameter buffer.

Replaces train.py:96-100 (torch.nn.utils.clip_grad_norm_(model.parameters(), GRAD_CLIP_VALUE) then
optimizer.step()) and the AdamW construction at train.py:319-325. Math is torch/optim/adam.py:419-547
(decoupled weight decay, lerp first moment, bias corrections) with the clip coefficient of
torch/nn/utils/clip_grad.py:165-186 applied to the gradient as it is read. Three launches per step:
sum-of-squares partials + norm finalisation, the step counter, the elementwise update (which also
refreshes the bf16 shadow the GEMMs read). No host synchronisation: lr, the step count and the clip
coefficient live in device memory, so the whole step can be captured in a hipGraph.

Checkpoints: ``state_dict()`` / ``load_state_dict()`` use torch.optim.AdamW's format
({"state": {index: {"step", "exp_avg", "exp_avg_sq"}}, "param_groups": [...]}) with the parameter
indices of the REFERENCE model's ``model.parameters()`` (frozen encoder tensors first, then the
projection and the decoder, model.py:48-114), so a reference-written checkpoint resumes here and
vice versa (train.py:347-375, 422-436). Anything that does not match is rejected before any state
is touched.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch

import native
from params import FlatParams


class OptimizerStateError(ValueError):
    """An optimizer state_dict that does not describe this model's trainable parameters."""


def reference_trainable(layout: dict) -> List[Tuple[str, Tuple[int, ...]]]:
    """(name, shape) of the reference's trainable tensors in its named_parameters() order:
    projection (if any, model.py:97-102), decoder.token_embedding (decoder.py:105), per layer
    self_attn / multihead_attn (in_proj_weight, in_proj_bias, out_proj.weight, out_proj.bias),
    linear1, linear2, norm1..3 (torch/nn/modules/transformer.py:1030-1087), fc_out (decoder.py:124)."""
    V, d, L, F, E = layout["V"], layout["d"], layout["L"], layout["F"], layout.get("proj_in")
    out = []
    if E is not None:
        out += [("projection.weight", (d, E)), ("projection.bias", (d,))]
    out.append(("decoder.token_embedding.weight", (V, d)))
    for i in range(L):
        p = f"decoder.transformer_decoder.layers.{i}."
        for a in ("self_attn.", "multihead_attn."):
            out += [(p + a + "in_proj_weight", (3 * d, d)), (p + a + "in_proj_bias", (3 * d,)),
                    (p + a + "out_proj.weight", (d, d)), (p + a + "out_proj.bias", (d,))]
        out += [(p + "linear1.weight", (F, d)), (p + "linear1.bias", (F,)), (p + "linear2.weight", (d, F)),
                (p + "linear2.bias", (d,))]
        for k in (1, 2, 3):
            out += [(p + f"norm{k}.weight", (d,)), (p + f"norm{k}.bias", (d,))]
    out += [("decoder.fc_out.weight", (V, d)), ("decoder.fc_out.bias", (V,))]
    return out


class _BufView:
    """Duck-typed FlatParams whose .p(name) views another flat buffer (exp_avg / exp_avg_sq)."""

    def __init__(self, store: FlatParams, buf: torch.Tensor):
        self.store, self.buf, self.vocab = store, buf, getattr(store, "vocab", None)

    def p(self, name):
        shape, off, n = self.store.index[name]
        return self.buf[off:off + n].view(shape)


def _store_of(params) -> FlatParams:
    if isinstance(params, FlatParams):
        return params
    params = list(params)
    stores = {id(getattr(p, "_mit_store", None)) for p in params}
    st = getattr(params[0], "_mit_store", None) if params else None
    if st is None or len(stores) != 1 or len(params) != len(st.entries):
        raise ValueError("optim.AdamW takes the model's FlatParams store or ALL of model.parameters() "
                         "(for any other parameter list use torch.optim.AdamW: the model supports it)")
    return st


def reference_state(store: FlatParams, lay: dict, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor, step: int,
                    group: dict) -> dict:
    """torch.optim.AdamW state_dict of the REFERENCE model's parameters (frozen encoder indices first,
    then reference_trainable order) from flat moment buffers laid out like ``store``."""
    from decoder import flat_to_reference
    names = reference_trainable(lay)
    base = lay["n_encoder_params"]
    ref = {}
    for key, buf in (("exp_avg", exp_avg), ("exp_avg_sq", exp_avg_sq)):
        view = _BufView(store, buf)
        sd = flat_to_reference(view, lay["L"], lay["d"])
        if lay.get("proj_in") is not None:
            sd["projection.weight"] = view.p("projection.weight").detach().clone()
            sd["projection.bias"] = view.p("projection.bias").detach().clone()
        ref[key] = sd
    state = {}
    if step > 0:
        for i, (n, _) in enumerate(names):
            state[base + i] = {"step": torch.tensor(float(step)), "exp_avg": ref["exp_avg"][n].cpu(),
                               "exp_avg_sq": ref["exp_avg_sq"][n].cpu()}
    g = {"lr": float(group["lr"]), "betas": tuple(group["betas"]), "eps": group["eps"],
         "weight_decay": group["weight_decay"]}
    g.update(amsgrad=False, maximize=False, foreach=None, capturable=False, differentiable=False, fused=None,
             decoupled_weight_decay=True, params=list(range(base + len(names))))
    return {"state": state, "param_groups": [g]}


def flat_moments(store: FlatParams, lay: dict, sd: dict):
    """Validate a torch.optim.AdamW state_dict of the reference model and convert it -> (exp_avg,
    exp_avg_sq) flat f32 buffers laid out like ``store`` (on its device), the step count, and the
    parameter group. Raises OptimizerStateError before anything is written anywhere."""
    from decoder import reference_to_flat
    if not isinstance(sd, dict) or "state" not in sd or "param_groups" not in sd:
        raise OptimizerStateError(f"not a torch.optim.AdamW state_dict (keys: {sorted(sd) if isinstance(sd, dict) else type(sd)})")
    names = reference_trainable(lay)
    groups = sd["param_groups"]
    if len(groups) != 1:
        raise OptimizerStateError(f"{len(groups)} parameter groups; the reference builds one (train.py:319-325)")
    g0 = groups[0]
    if g0.get("amsgrad") or g0.get("maximize"):
        raise OptimizerStateError("amsgrad / maximize AdamW states are not supported")
    idx = list(g0["params"])
    if len(idx) < len(names):
        raise OptimizerStateError(f"the state covers {len(idx)} parameters, the model trains {len(names)}")
    train_idx = idx[len(idx) - len(names):]
    frozen_with_state = [i for i in idx[:len(idx) - len(names)] if i in sd["state"]]
    if frozen_with_state:
        raise OptimizerStateError(f"optimizer state for {len(frozen_with_state)} parameters that are frozen here "
                                  f"(encoder / layout mismatch)")
    steps = set()
    moments = {"exp_avg": {}, "exp_avg_sq": {}}
    for i, (n, shape) in zip(train_idx, names):
        s = sd["state"].get(i)
        if s is None:  # never stepped (no gradient yet): zero moments
            for k in moments:
                moments[k][n] = torch.zeros(shape)
            continue
        for k in moments:
            t = s.get(k)
            if t is None or tuple(t.shape) != tuple(shape):
                raise OptimizerStateError(f"{n}: {k} has shape {None if t is None else tuple(t.shape)}, "
                                          f"expected {tuple(shape)}")
            moments[k][n] = t.detach().float().cpu()
        steps.add(float(s["step"]))
    if len(steps) > 1:
        raise OptimizerStateError(f"per-parameter step counts differ ({sorted(steps)[:4]}); the flat layout "
                                  f"fuses tensors and keeps one step count")
    out = []
    for k in ("exp_avg", "exp_avg_sq"):
        flat = reference_to_flat(moments[k], lay["L"], lay["d"])
        buf = torch.zeros(store.numel, dtype=torch.float32, device=store.device)
        view = _BufView(store, buf)
        for n, t in flat.items():
            dst = view.p(n)
            dst[:t.shape[0]].copy_(t.to(dst.device).reshape((t.shape[0],) + tuple(dst.shape[1:])))
        out.append(buf)
    return out[0], out[1], int(round(steps.pop())) if steps else 0, g0


class AdamW:
    def __init__(self, params, lr=1e-4, betas=(0.9, 0.98), eps=1e-9, weight_decay=1e-5):
        store = _store_of(params)
        self.store = store
        self.betas, self.eps, self.weight_decay = tuple(betas), eps, weight_decay
        store.ensure_optimizer_state()
        dev = store.device
        self.lr_t = torch.full((1,), float(lr), dtype=torch.float32, device=dev)
        self.step_t = torch.zeros(1, dtype=torch.int64, device=dev)
        self.norm_t = torch.zeros(2, dtype=torch.float32, device=dev)  # {total_norm, clip_coef}
        self.ws = torch.empty(native.grad_norm_ws_floats(store.numel), dtype=torch.float32, device=dev)
        self.param_groups = [{"lr": float(lr), "betas": tuple(betas), "eps": eps, "weight_decay": weight_decay}]
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

    # --- checkpoint I/O in torch.optim.AdamW's format (train.py:422-436 stores optimizer.state_dict()) -----
    def _layout(self) -> dict:
        lay = getattr(self.store, "layout", None)
        if lay is None:
            raise OptimizerStateError("the parameter store has no model layout (built outside ImageToTextModel)")
        return lay

    def state_dict(self) -> dict:
        return reference_state(self.store, self._layout(), self.store.exp_avg, self.store.exp_avg_sq,
                               int(self.step_t.item()), self.param_groups[0])

    def load_state_dict(self, sd: dict):
        """torch.optim.AdamW state (reference checkpoints, or ours) -> the flat moments, the step
        count and the hyper-parameters. Validated completely before anything is written."""
        ea, eas, step, g0 = flat_moments(self.store, self._layout(), sd)
        with torch.no_grad():
            self.store.exp_avg.copy_(ea)
            self.store.exp_avg_sq.copy_(eas)
        self.step_t.fill_(step)
        self.betas = tuple(g0.get("betas", self.betas))
        self.eps = g0.get("eps", self.eps)
        self.weight_decay = g0.get("weight_decay", self.weight_decay)
        self.param_groups = [{"lr": float(g0["lr"]), "betas": self.betas, "eps": self.eps,
                              "weight_decay": self.weight_decay}]
        self._lr_host = None
        self._sync_lr()

