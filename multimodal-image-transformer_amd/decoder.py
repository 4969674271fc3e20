"""Transformer decoder (reference decoder.py:75-193) with an explicit forward/backward on the
gfx950 kernels.

Semantics reproduced exactly (post-LN nn.TransformerDecoderLayer, torch/nn/modules/transformer.py
:1131-1199, built at decoder.py:112-120):
    x  = dropout(Emb[tok] * sqrt(d) + PE[t])                                  decoder.py:168-171
    x  = LN1(x + dropout(SelfAttn(x; causal + key-padding mask, attn dropout)))
    x  = LN2(x + dropout(CrossAttn(x, memory; attn dropout)))
    x  = LN3(x + dropout(W2 dropout(relu(W1 x + b1)) + b2))
    logits = x Wfc^T + bfc                                                   decoder.py:191
MHA uses a packed in_proj (q,k,v rows), scale 1/sqrt(head_dim) (torch/nn/functional.py:6435).

MI355X-specific layout decisions:
  * the cross-attention K/V projections of ALL layers only depend on the memory, so they are one
    GEMM  kv_all[B*S, L*2d] = memory @ W_kv_all^T  (N = 6144 at cfg1) in the forward, and one
    dW GEMM + one dX GEMM in the backward (the reference issues 2 x L smaller ones);
  * the masks are never materialised (computed in-kernel from tokens == PAD and j > i);
  * dropout masks are regenerated from (seed, site, index) in the backward, never stored;
  * weight gradients are written ONCE (no zero-fill + accumulate), straight into the flat f32
    gradient buffer (params.FlatParams) in backward-completion order.
"""
from __future__ import annotations

import math
import os
from typing import Callable, Dict, List, Optional, Tuple

import torch

import native
from params import FlatParams

EMB_SITE = 4000


def sinusoidal_pe(max_len: int, d: int) -> torch.Tensor:
    """The PositionalEncodingBatchFirst buffer (decoder.py:34-47), [max_len, d] f32."""
    pos = torch.arange(max_len).unsqueeze(1)
    div = torch.exp(torch.arange(0, d, 2) * (-math.log(10000.0) / d))
    pe = torch.zeros(max_len, d)
    pe[:, 0::2] = torch.sin(pos * div)
    pe[:, 1::2] = torch.cos(pos * div)
    return pe


def padded_vocab(V: int) -> int:
    """The vocabulary head is stored with Vp = round8(V) rows: the bf16 GEMMs need the contiguous
    extent of every operand (the fc_out weight gradient has M = V, lda = V) to be a multiple of 8,
    and the reference sizes V from the trained tokenizer (tokenizer.py:200-201, any size). The pad
    rows of fc_out are zero and stay zero (their gradient is exactly 0, so AdamW never moves them);
    the pad logit columns are 0 and never reach the caller, the loss or argmax."""
    return (V + 7) // 8 * 8


def decoder_entries(V: int, d: int, L: int, F: int, proj_in: Optional[int]) -> List[Tuple[str, Tuple[int, ...]]]:
    """Flat-buffer layout in backward-completion order (see params.py)."""
    Vp = padded_vocab(V)
    e = [("fc_out.weight", (Vp, d)), ("fc_out.bias", (Vp,))]
    for i in reversed(range(L)):
        p = f"layers.{i}."
        e += [(p + "linear2.weight", (d, F)), (p + "linear2.bias", (d,)), (p + "linear1.weight", (F, d)),
              (p + "linear1.bias", (F,)), (p + "norm3.weight", (d,)), (p + "norm3.bias", (d,)),
              (p + "cross_out.weight", (d, d)), (p + "cross_out.bias", (d,)), (p + "cross_q.weight", (d, d)),
              (p + "cross_q.bias", (d,)), (p + "norm2.weight", (d,)), (p + "norm2.bias", (d,)),
              (p + "self_out.weight", (d, d)), (p + "self_out.bias", (d,)), (p + "self_in.weight", (3 * d, d)),
              (p + "self_in.bias", (3 * d,)), (p + "norm1.weight", (d,)), (p + "norm1.bias", (d,))]
    e += [("cross_kv.weight", (L * 2 * d, d)), ("cross_kv.bias", (L * 2 * d,)), ("token_embedding.weight", (V, d))]
    if proj_in is not None:
        e += [("projection.weight", (d, proj_in)), ("projection.bias", (d,))]
    return e


def reference_to_flat(sd: Dict[str, torch.Tensor], L: int, d: int, prefix: str = "decoder.") -> Dict[str, torch.Tensor]:
    """Reference state_dict names (decoder.* / projection.*) -> flat entry names."""
    out = {}
    kv_w, kv_b = [None] * L, [None] * L
    for k, v in sd.items():
        if k.startswith("projection."):
            out[k] = v
            continue
        if not k.startswith(prefix):
            continue
        k = k[len(prefix):]
        if k in ("fc_out.weight", "fc_out.bias", "token_embedding.weight"):
            out[k] = v
        elif k.startswith("transformer_decoder.layers."):
            rest = k[len("transformer_decoder.layers."):]
            i, sub = rest.split(".", 1)
            i = int(i)
            p = f"layers.{i}."
            if sub == "self_attn.in_proj_weight":
                out[p + "self_in.weight"] = v
            elif sub == "self_attn.in_proj_bias":
                out[p + "self_in.bias"] = v
            elif sub.startswith("self_attn.out_proj."):
                out[p + "self_out." + sub.rsplit(".", 1)[1]] = v
            elif sub == "multihead_attn.in_proj_weight":
                out[p + "cross_q.weight"] = v[:d]
                kv_w[i] = v[d:]
            elif sub == "multihead_attn.in_proj_bias":
                out[p + "cross_q.bias"] = v[:d]
                kv_b[i] = v[d:]
            elif sub.startswith("multihead_attn.out_proj."):
                out[p + "cross_out." + sub.rsplit(".", 1)[1]] = v
            else:  # linear1/linear2/norm1-3
                out[p + sub] = v
    if all(x is not None for x in kv_w):
        out["cross_kv.weight"] = torch.cat(kv_w, 0)
    if all(x is not None for x in kv_b):
        out["cross_kv.bias"] = torch.cat(kv_b, 0)
    return out


def flat_to_reference(store: FlatParams, L: int, d: int, prefix: str = "decoder.") -> Dict[str, torch.Tensor]:
    """Inverse of reference_to_flat: the reference's state_dict keys (§8b), f32 copies."""
    sd = {}
    p = lambda n: store.p(n).detach().clone()  # noqa: E731
    kvw, kvb = store.p("cross_kv.weight"), store.p("cross_kv.bias")
    sd[prefix + "token_embedding.weight"] = p("token_embedding.weight")
    for i in range(L):
        r, q = f"{prefix}transformer_decoder.layers.{i}.", f"layers.{i}."
        sd[r + "self_attn.in_proj_weight"] = p(q + "self_in.weight")
        sd[r + "self_attn.in_proj_bias"] = p(q + "self_in.bias")
        sd[r + "self_attn.out_proj.weight"] = p(q + "self_out.weight")
        sd[r + "self_attn.out_proj.bias"] = p(q + "self_out.bias")
        sd[r + "multihead_attn.in_proj_weight"] = torch.cat([p(q + "cross_q.weight"), kvw[i * 2 * d:(i + 1) * 2 * d]], 0)
        sd[r + "multihead_attn.in_proj_bias"] = torch.cat([p(q + "cross_q.bias"), kvb[i * 2 * d:(i + 1) * 2 * d]], 0)
        sd[r + "multihead_attn.out_proj.weight"] = p(q + "cross_out.weight")
        sd[r + "multihead_attn.out_proj.bias"] = p(q + "cross_out.bias")
        for s in ("linear1", "linear2", "norm1", "norm2", "norm3"):
            sd[r + s + ".weight"] = p(q + s + ".weight")
            sd[r + s + ".bias"] = p(q + s + ".bias")
    V = getattr(store, "vocab", None)
    sd[prefix + "fc_out.weight"] = p("fc_out.weight")[:V]
    sd[prefix + "fc_out.bias"] = p("fc_out.bias")[:V]
    return sd


class _Acts:
    """Activation arena for one (B, T, S, train) shape; allocated once, reused every step."""

    def __init__(self, B, T, S, d, F, L, V, H, dt, dev, train: bool, proj_in: Optional[int] = None):
        R = B * T
        e = lambda *s: torch.empty(*s, dtype=dt, device=dev)  # noqa: E731
        f = lambda *s: torch.empty(*s, dtype=torch.float32, device=dev)  # noqa: E731
        self.R = R
        self.x0 = e(R, d)
        self.y = e(R, d)
        self.kv = e(B * S, L * 2 * d)
        self.logits = e(R, padded_vocab(V))  # padded head columns: row stride Vp
        nl = L if train else 1  # eval keeps one set of per-layer buffers and reuses it
        self.qkv = [e(R, 3 * d) for _ in range(nl)]
        self.os = [e(R, d) for _ in range(nl)]
        self.oc = [e(R, d) for _ in range(nl)]
        self.qc = [e(R, d) for _ in range(nl)]
        self.h = [e(R, F) for _ in range(nl)]
        self.z = [[e(R, d) for _ in range(3)] for _ in range(nl)]
        self.st = [[(f(R), f(R)) for _ in range(3)] for _ in range(nl)]
        self.lse_s = [f(B * H * T) for _ in range(nl)]
        self.lse_c = [f(B * H * T) for _ in range(nl)]
        # per-layer normalised outputs x1, x2, x3 (x3 of layer l = input of layer l+1)
        self.xs = [[e(R, d) for _ in range(3)] for _ in range(L if train else 2)]
        self.count_loss = f(2)  # {non-PAD target count, CE loss sum}: one memset per step
        self.count = self.count_loss[0:1]
        self.loss_sum = self.count_loss[1:2]
        self.loss = f(1)
        self.row_loss = f(R)  # per-row CE losses (deterministic loss sum)
        # split-K scratch of the main stream: the d_model GEMMs (R x d outputs, 128 tiles at B = 64)
        # combine their K slices in-launch; weight-gradient / long-K GEMMs reduce in a second launch.
        # Zero-filled once: its first 4 KiB are tile counters the kernels leave at zero.
        E = proj_in or d
        Vp = padded_vocab(V)
        shapes = [(R, d, d), (R, d, F), (R, d, 3 * d), (R, d, Vp)]
        if train:
            shapes += [(Vp, d, R), (d, F, R), (F, d, R), (d, d, R), (3 * d, d, R), (L * 2 * d, d, B * S), (d, E, B * S),
                       (B * S, d, L * 2 * d)]
        need = max(native.gemm_workspace_bytes(m, n, k) for m, n, k in shapes)
        self.gemm_ws = torch.zeros(max(need, 4096) // 4 + 4, dtype=torch.float32, device=dev)
        if train:
            self.dx = e(R, d)
            self.dy = e(R, d)
            self.do = e(R, d)
            self.dq = e(R, d)
            self.dqkv = e(R, 3 * d)
            self.dh = e(R, F)
            self.dkv = e(B * S, L * 2 * d)
            self.dmem = e(B * S, d)
            self.delta = f(B * H * T)
            self.ln_ws = f(native.layernorm_bwd_ws_floats(R, d))
            # one column-partial buffer per LayerNorm: their dgamma/dbeta reductions run on the
            # side stream, off the dX chain (run_backward)
            self.ln_ws_side = [f(native.layernorm_bwd_ws_floats(R, d)) for _ in range(3 * L)]
            # deterministic embedding-gradient order (native.embed_plan of the step's tokens)
            self.emb_plan = torch.empty(native.embed_plan_ints(R), dtype=torch.int32, device=dev)
            # the weight-gradient GEMMs run on a side stream (_SideStream) with their own scratch
            self.gemm_ws_side = torch.zeros(max(need, 4096) // 4 + 4, dtype=torch.float32, device=dev)
            # grouped per-layer dW (TransformerDecoder.dw_grouped): the six dY operands of a layer in their own
            # buffers, two sets (layer parity) so layer l's grouped launch overlaps layer l-1's dX chain
            self.gdy = [[e(R, d) for _ in range(3)] for _ in range(2)]
            self.gdh = [e(R, F) for _ in range(2)]
            self.gdq = [e(R, d) for _ in range(2)]
            self.gdqkv = [e(R, 3 * d) for _ in range(2)]
            self.gws = None  # allocated on first use (native.gemm_grouped_ws_bytes)
            self.gws_tail = None  # the cross-K/V + projection pair
            self.gws_kv = None  # the cross-K/V weight gradient alone (TransformerDecoder.kv_dw_early)


class _SideStream:
    """Second HIP stream for the backward's weight-gradient GEMMs (dW = dY^T X). Each layer's dW
    and dX GEMMs are independent; at d = 512 a decoder GEMM fills only 128-512 of the CUs' 512
    block slots, so running the dW chain beside the main dX -> LayerNorm -> attention chain fills
    the machine. Ordering: side waits for main before each dW (its dY is final); main waits for the
    side's last reader of a gradient buffer before overwriting it (guard); join() at the end. All
    edges are HIP events, so the step still captures into ONE hipGraph (as parallel branches)."""

    def __init__(self, device, priority: int = 0):
        self.stream = torch.cuda.Stream(device=device, priority=priority)
        self.ptr = self.stream.cuda_stream
        self.events = native.HipEvents(64)  # recorded on the main stream (side waits for main)
        self.plan_events = native.HipEvents(2)  # the embedding plan (side) -> embedding backward (main)
        self.side_events = native.HipEvents(128)  # recorded on the side stream only: a recycled slot
        self.pending = {}                         # re-recorded later on the SAME stream stays a safe wait

    def run(self, fn, reads=()):
        """fn issues native launches only (routed by native.on_stream, no torch stream switch)."""
        self.events.wait_stream(self.ptr, native.stream_ptr())
        with native.on_stream(self.ptr):
            fn()
        if reads:
            ev = self.side_events.record(self.ptr)
            for t in reads:
                self.pending[t.data_ptr()] = ev

    def guard(self, t):
        """Before the main stream writes t: wait for the side-stream GEMM still reading it."""
        ev = self.pending.pop(t.data_ptr(), None)
        if ev is not None:
            native.HipEvents.wait(native.stream_ptr(), ev)

    def under(self, fn):
        """Run fn (e.g. a DP gradient-bucket all-reduce) on the side stream after everything issued
        so far on both streams (a host step of a recorded program: native.host_call)."""
        self.events.wait_stream(self.ptr, native.stream_ptr())

        def call():
            with torch.cuda.stream(self.stream):
                fn()
        native.host_call(call)

    def join(self):
        """The caller's stream waits for everything issued on the side stream."""
        native.HipEvents.wait(native.stream_ptr(), self.side_events.record(self.ptr))
        self.pending.clear()


class DecodeState:
    """Device state of a batched greedy decode (TransformerDecoder.decode_begin / decode_step):
    token ids [B, max_len] (int64; column 0 = START), the device position, per-row finished flags
    and their count, the cross-attention K/V of all layers [B*S, L*2d], per-layer self-attention
    caches [B, max_len, 2d] (K | V), and the B-row activations of one token step."""

    def __init__(self, dec: "TransformerDecoder", B: int, S: int, max_len: int, start_id: int, end_id: int):
        dev, dt = dec.device, dec.dtype
        d, F, L, V = dec.d, dec.F, dec.L, dec.V
        self.B, self.S, self.max_len, self.end_id = B, S, max_len, int(end_id)
        self.ids = torch.full((B, max_len), dec.pad_idx, dtype=torch.int64, device=dev)
        self.ids[:, 0] = int(start_id)
        self.pos = torch.zeros(1, dtype=torch.int64, device=dev)
        self.finished = torch.zeros(B, dtype=torch.int32, device=dev)
        self.n_finished = torch.zeros(1, dtype=torch.int32, device=dev)
        # per layer contiguous [L][B*S][2d] (K | V): a decode attention block (b, h) then reads its S keys
        # at a 2 KiB stride instead of the training layout's L * 2d row (12 KiB at cfg1), which left the
        # S = 197 cross attention at ~2.6 TB/s on DRAM page misses
        self.kv = torch.empty(L, B * S, 2 * d, dtype=dt, device=dev)
        self.cache = [torch.empty(B, max_len, 2 * d, dtype=dt, device=dev) for _ in range(L)]
        e = lambda n: torch.empty(B, n, dtype=dt, device=dev)  # noqa: E731
        self.x, self.x1, self.x2, self.y, self.o, self.q = e(d), e(d), e(d), e(d), e(d), e(d)
        self.qkv, self.h = e(3 * d), e(F)
        self.logits = torch.empty(B, padded_vocab(V), dtype=torch.float32, device=dev)  # f32: argmax on unrounded logits
        # bf16 step with the LayerNorms folded into the GEMMs (native.decode_gemm): the three pre-LN sums
        # of a layer in f32 and their per-64-column row statistics; the pick advances pos via `ticket`
        self.fused = dt == torch.bfloat16 and os.environ.get("MIT_DECODE_FUSED", "1") != "0"
        if self.fused:
            P = (d + 63) // 64
            self.z = [torch.empty(B, d, dtype=torch.float32, device=dev) for _ in range(3)]
            self.zst = [torch.empty(B, P, 2, dtype=torch.float32, device=dev) for _ in range(3)]
            self.ticket = torch.zeros(1, dtype=torch.int32, device=dev)
            # the head's packed argmax, ARGMAX_SLOTS per row (0 between steps)
            self.keys = torch.zeros(native.ARGMAX_SLOTS * B, dtype=torch.int64, device=dev)

    def token_lists(self) -> List[List[int]]:
        """Per row: START .. up to and including the first END (model.py:236-242), else max_len ids."""
        out = []
        for row in self.ids.cpu().tolist():
            if self.end_id in row[1:]:
                row = row[: row.index(self.end_id, 1) + 1]
            out.append(row)
        return out


class TransformerDecoder:
    """Reference-surface decoder: same constructor arguments as decoder.py:84-85.

    Parameters live in a FlatParams store (shared with the model's projection when built by
    model.ImageToTextModel). ``forward(tgt_tokens, memory, memory_padding_mask=None)`` matches
    decoder.py:134-193 and returns f32 logits [B, T, V].
    """

    def __init__(self, vocab_size: int, embed_dim: int, num_heads: int, num_layers: int, ff_dim: int,
                 max_seq_len: int, dropout: float = 0.1, pad_idx: int = 0, *, store: Optional[FlatParams] = None,
                 device=None, dtype: Optional[torch.dtype] = None):
        native.require_gpu()
        self.V, self.d, self.H, self.L, self.F = vocab_size, embed_dim, num_heads, num_layers, ff_dim
        self.Vp = padded_vocab(vocab_size)
        if embed_dim % num_heads:
            raise ValueError(f"embed_dim {embed_dim} is not divisible by num_heads {num_heads}")
        self.hd = embed_dim // num_heads
        if self.hd not in (16, 32, 64, 128):
            raise ValueError(f"head_dim {self.hd} unsupported: the attention kernels take 16, 32, 64 or 128")
        self.max_seq_len, self.dropout, self.pad_idx = max_seq_len, dropout, pad_idx
        self.embed_dim = embed_dim
        self.device = device or torch.device("cuda")
        if store is None:
            dt = dtype or torch.bfloat16
            store = FlatParams(decoder_entries(vocab_size, embed_dim, num_layers, ff_dim, None), self.device, dt)
            store.vocab = vocab_size
            self._own_store = True
        else:
            self._own_store = False
        self.store = store
        self.dtype = store.compute_dtype
        self.pe = sinusoidal_pe(max_seq_len, embed_dim).to(self.device)
        self.training = True
        self._acts: Dict[tuple, _Acts] = {}
        # weight-gradient GEMMs on a second stream; in bf16 a decoder layer's six weight gradients go out
        # as ONE grouped launch (native.gemm_grouped; fp32 parity mode: one GEMM each, as they become
        # ready); the cross-K/V weight gradient (all layers' dY final once layer 0's cross-attention
        # backward ran) goes out right then, ahead of layer 0's grouped dW
        self.dw_side_stream = True
        self.dw_grouped = True
        self.kv_dw_early = True
        self._side = None
        self.side_priority = 0
        if self._own_store:
            self.init_weights(0)

    # --- weights -----------------------------------------------------------------------------
    def init_weights(self, seed: int = 0):
        """decoder.py:128-132: xavier_uniform_ on every >=2-D weight (embedding included, so the
        PAD row is not zero); MHA in/out-proj biases 0 (torch/nn/modules/activation.py:1241-1242);
        LayerNorm 1/0; Linear biases U(-1/sqrt(fan_in), 1/sqrt(fan_in)) (nn.Linear default)."""
        g = torch.Generator().manual_seed(seed)
        d, L = self.d, self.L
        for name, shape, _, _ in self.store.entries:
            if name.startswith("projection."):
                continue
            if name == "cross_kv.weight":
                # xavier on each layer's full in_proj [3d, d] (fan_out = 3d), restricted to the kv rows
                a = math.sqrt(6.0 / (3 * d + d))
                t = (torch.rand(*shape, generator=g) * 2 - 1) * a
            elif len(shape) == 2:
                rows, fi = shape
                if name == "fc_out.weight":
                    rows = self.V  # the pad rows of the head stay 0 (padded_vocab)
                fo = 3 * d if name.endswith("cross_q.weight") else rows
                a = math.sqrt(6.0 / (fo + fi))
                t = torch.zeros(shape)
                t[:rows] = (torch.rand(rows, fi, generator=g) * 2 - 1) * a
            elif "norm" in name:
                t = torch.ones(shape) if name.endswith("weight") else torch.zeros(shape)
            elif any(s in name for s in ("self_in.bias", "self_out.bias", "cross_q.bias", "cross_out.bias",
                                          "cross_kv.bias")):
                t = torch.zeros(shape)
            else:  # linear1/linear2/fc_out biases
                fan_in = {"linear1.bias": d, "linear2.bias": self.F, "fc_out.bias": d}[name.split(".", 2)[-1]
                                                                                        if name.startswith("layers.")
                                                                                        else name]
                b = 1 / math.sqrt(fan_in)
                n = self.V if name == "fc_out.bias" else shape[0]
                t = torch.zeros(shape)
                t[:n] = (torch.rand(n, generator=g) * 2 - 1) * b
            self.store.p(name).copy_(t)
        self.store.sync_shadow()

    def train(self, mode: bool = True):
        self.training = mode
        return self

    def eval(self):
        return self.train(False)

    def _side_stream(self) -> "_SideStream":
        if self._side is None:
            self._side = _SideStream(self.device, self.side_priority)
        return self._side

    # --- forward -----------------------------------------------------------------------------
    def acts(self, B, T, S, train) -> _Acts:
        key = (B, T, S, train)
        if key not in self._acts:
            pi = self.store.index.get("projection.weight")
            self._acts[key] = _Acts(B, T, S, self.d, self.F, self.L, self.V, self.H, self.dtype, self.device, train,
                                    proj_in=pi[0][1] if pi else None)
        return self._acts[key]

    def _p(self):
        return self.dropout if self.training else 0.0

    def run_forward(self, tokens: torch.Tensor, mem: torch.Tensor, mem_ld: int, S: int, A: _Acts,
                    seed: Optional[torch.Tensor], train: bool, logits_out: Optional[torch.Tensor] = None,
                    drop_p: Optional[float] = None, mem_keys: Optional[torch.Tensor] = None,
                    tick: Optional[Callable[[], None]] = None):
        """tokens int64 [B,T] (device); mem: memory rows [B*S, d] with row stride mem_ld.
        tick: called before each layer's launches (the train step issues other work there).
        train=True keeps every layer's activations for run_backward (A must be a train arena);
        drop_p defaults to the module's dropout in train mode and 0 otherwise.
        mem_keys: optional int64 [B, S], 0 where the memory key is padding (memory_padding_mask,
        decoder.py:134-186 -> memory_key_padding_mask of nn.TransformerDecoder), else 1."""
        B, T = tokens.shape
        d, H, L, V = self.d, self.H, self.L, self.V
        st = self.store
        p = drop_p if drop_p is not None else (self._p() if train else 0.0)
        w = st.w
        R = B * T
        ws = A.gemm_ws
        # fused cross-attention K/V projection of every layer (decoder-layer independent)
        native.gemm(mem, w("cross_kv.weight"), A.kv, B * S, L * 2 * d, d, lda=mem_ld, bias=st.p("cross_kv.bias"))
        native.embed_fwd(tokens, w("token_embedding.weight"), math.sqrt(d), self.pe, A.x0, drop_p=p, seed=seed,
                         site=EMB_SITE)
        xin = A.x0
        for l in range(L):
            if tick is not None:
                tick()
            j = l if train else 0
            xs = A.xs[l] if train else A.xs[l % 2]
            z, stt = A.z[j], A.st[j]
            pre = f"layers.{l}."
            base = 64 * l
            qkv = A.qkv[j]
            native.linear(xin, w(pre + "self_in.weight"), qkv, bias=st.p(pre + "self_in.bias"))
            sa = native.attn_args(qkv, 3 * d, T * 3 * d, qkv[:, d:], 3 * d, T * 3 * d, qkv[:, 2 * d:], 3 * d, T * 3 * d,
                                  A.os[j], d, T * d, lse=A.lse_s[j], key_tokens=tokens, tok_batch=T,
                                  pad_idx=self.pad_idx, causal=True, scale=1.0 / math.sqrt(self.hd), drop_p=p, seed=seed,
                                  site=base + 0)
            native.attention_fwd(native.dtype_code(qkv), B, H, T, T, sa, Dh=self.hd)
            native.linear(A.os[j], w(pre + "self_out.weight"), A.y, bias=st.p(pre + "self_out.bias"), workspace=ws)
            native.layernorm_fwd(xin, st.p(pre + "norm1.weight"), st.p(pre + "norm1.bias"), 1e-5, xs[0], r=A.y,
                                 drop_p=p, seed=seed, site=base + 1, z=z[0], mean=stt[0][0], rstd=stt[0][1])
            native.linear(xs[0], w(pre + "cross_q.weight"), A.qc[j], bias=st.p(pre + "cross_q.bias"), workspace=ws)
            kvl = A.kv[:, l * 2 * d:]
            ca = native.attn_args(A.qc[j], d, T * d, kvl, L * 2 * d, S * L * 2 * d, kvl[:, d:], L * 2 * d,
                                  S * L * 2 * d, A.oc[j], d, T * d, lse=A.lse_c[j], scale=1.0 / math.sqrt(self.hd), drop_p=p,
                                  seed=seed, site=base + 2, key_tokens=mem_keys, tok_batch=S, pad_idx=0)
            native.attention_fwd(native.dtype_code(qkv), B, H, T, S, ca, Dh=self.hd)
            native.linear(A.oc[j], w(pre + "cross_out.weight"), A.y, bias=st.p(pre + "cross_out.bias"), workspace=ws)
            native.layernorm_fwd(xs[0], st.p(pre + "norm2.weight"), st.p(pre + "norm2.bias"), 1e-5, xs[1], r=A.y,
                                 drop_p=p, seed=seed, site=base + 3, z=z[1], mean=stt[1][0], rstd=stt[1][1])
            native.linear(xs[1], w(pre + "linear1.weight"), A.h[j], bias=st.p(pre + "linear1.bias"),
                          act=native.ACT_RELU, drop_p=p, seed=seed, site=base + 4)
            native.linear(A.h[j], w(pre + "linear2.weight"), A.y, bias=st.p(pre + "linear2.bias"), workspace=ws)
            native.layernorm_fwd(xs[1], st.p(pre + "norm3.weight"), st.p(pre + "norm3.bias"), 1e-5, xs[2], r=A.y,
                                 drop_p=p, seed=seed, site=base + 5, z=z[2], mean=stt[2][0], rstd=stt[2][1])
            xin = xs[2]
        logits = A.logits if logits_out is None else logits_out
        native.linear(xin, w("fc_out.weight"), logits, bias=st.p("fc_out.bias"))
        return logits, xin

    def run_backward(self, tokens: torch.Tensor, mem: torch.Tensor, mem_ld: int, S: int, A: _Acts,
                     seed: Optional[torch.Tensor], dlogits: torch.Tensor,
                     proj_input: Optional[Tuple[torch.Tensor, int, int]] = None,
                     grads_ready: Optional[Callable[[str, str], None]] = None,
                     mem_keys: Optional[torch.Tensor] = None, tick: Optional[Callable[[], None]] = None):
        """Backward of run_forward(train=True) given dlogits [R, V] (compute dtype); tick as in run_forward.
        proj_input = (enc_rows, ld, E): encoder features feeding the projection (for dW_proj).
        grads_ready(first, last) is called as soon as the grads of a contiguous entry span are final."""
        B, T = tokens.shape
        d, H, L, V, F = self.d, self.H, self.L, self.V, self.F
        st, p = self.store, self._p()
        w, g = st.w, st.g
        R = B * T
        MN, K = native.MN_CONTIG, native.K_CONTIG
        x_last = A.xs[L - 1][2]
        ws = A.gemm_ws
        side = self._side_stream() if self.dw_side_stream else None
        # the embedding gradient's deterministic summation order depends on the tokens only: build it
        # on the side stream now, off the dX chain
        if side is None:
            native.embed_plan(tokens, A.emb_plan)
        else:
            # the embedding plan depends on the tokens only; the table gradient's zero fill (20 MB at
            # cfg1) rides with it, off the main stream's chain (the previous AdamW, its last reader, is
            # behind the side stream's wait on main)
            side.run(lambda: (native.embed_plan(tokens, A.emb_plan), native.zero(g("token_embedding.weight"))))
            plan_ev = side.plan_events.record(side.ptr)

        def dW(dy, x, wname, bname, M, N, K, lda, ldb):
            """weight grad dY^T X (TN GEMM) with the bias grad (row sums of dY^T) fused in, split-K;
            on the side stream when enabled."""
            if side is None:
                native.gemm(dy, x, g(wname), M, N, K, a_layout=MN, b_layout=MN, lda=lda, ldb=ldb, rowsum=g(bname),
                            workspace=ws)
                return
            side.run(lambda: native.gemm(dy, x, g(wname), M, N, K, a_layout=MN, b_layout=MN, lda=lda, ldb=ldb,
                                         rowsum=g(bname), workspace=A.gemm_ws_side), reads=(dy,))

        def guard(t):
            if side is not None:
                side.guard(t)

        def ln_bwd(l, k, dx, z, stt, dr, site, defer=False):
            """LayerNorm k (1..3) of layer l backward; dgamma/dbeta reduced on the side stream (defer: the
            reduction job is returned for the layer's grouped dW launch instead)."""
            gname, bname = f"layers.{l}.norm{k}.weight", f"layers.{l}.norm{k}.bias"
            if side is None:
                native.layernorm_bwd(dx, z, stt[0], stt[1], st.p(gname), dx, g(gname), g(bname), A.ln_ws, dr=dr,
                                     drop_p=p, seed=seed, site=site)
                return None
            ws_l = A.ln_ws_side[3 * l + k - 1]
            native.layernorm_bwd(dx, z, stt[0], stt[1], st.p(gname), dx, None, None, ws_l, dr=dr, drop_p=p, seed=seed,
                                 site=site)
            if defer:
                return (R, d, ws_l, g(gname), g(bname))
            side.run(lambda: native.layernorm_param_grads(R, d, ws_l, g(gname), g(bname)))
            return None

        def ready(first, last):
            if grads_ready is None:
                return
            if side is None:  # a host step of a recorded program (replayed in place)
                native.host_call(lambda: grads_ready(first, last))
            else:
                side.under(lambda: grads_ready(first, last))

        # fc_out
        Vp = self.Vp  # dlogits [R, Vp]: the pad columns hold exactly 0 (padded_vocab)
        dW(dlogits, x_last, "fc_out.weight", "fc_out.bias", Vp, d, R, Vp, d)
        native.gemm(dlogits, w("fc_out.weight"), A.dx, R, d, Vp, b_layout=MN, ldb=d, workspace=ws)
        ready("fc_out.weight", "fc_out.bias")
        ascale = 1.0 / (1.0 - p) if p > 0 else 1.0
        grouped = side is not None and self.dw_grouped and self.dtype == torch.bfloat16
        BS = B * S
        pair = grouped and proj_input is not None
        early = pair and self.kv_dw_early
        kv_prob = (A.dkv, mem, g("cross_kv.weight"), L * 2 * d, d, BS, L * 2 * d, mem_ld, g("cross_kv.bias"))

        def kv_early():
            if not early:
                return
            if A.gws_kv is None:
                A.gws_kv = torch.empty((native.gemm_grouped_ws_bytes([kv_prob]) + 255) // 4, dtype=torch.float32,
                                       device=self.device)
            side.run(lambda: native.gemm_grouped([kv_prob], A.gws_kv), reads=(A.dkv,))
            # its own DP bucket (12.6 MB at cfg1): all-reduced under the rest of the backward instead of with
            # the embedding / projection gradients after it (exposed communication)
            ready("cross_kv.weight", "cross_kv.bias")
        for l in reversed(range(L)):
            if tick is not None:
                tick()
            pre = f"layers.{l}."
            base = 64 * l
            xs, z, stt = A.xs[l], A.z[l], A.st[l]
            xin = A.x0 if l == 0 else A.xs[l - 1][2]
            if grouped:
                self._layer_backward_grouped(l, A, tokens, seed, p, xs, z, stt, xin, S, mem_keys, g, w, ln_bwd, guard,
                                             side, after_cross=kv_early if l == 0 else None)
                ready(pre + "linear2.weight", pre + "norm1.bias")
                continue
            # LN3 -> dz3 (dx, in place) and d(ffn_out) (dy)
            guard(A.dy)
            ln_bwd(l, 3, A.dx, z[2], stt[2], A.dy, base + 5)
            # FFN
            dW(A.dy, A.h[l], pre + "linear2.weight", pre + "linear2.bias", d, F, R, d, F)
            guard(A.dh)
            native.gemm(A.dy, w(pre + "linear2.weight"), A.dh, R, F, d, b_layout=MN, ldb=F, aux=A.h[l], ld_aux=F,
                        aux_scale=ascale)
            dW(A.dh, xs[1], pre + "linear1.weight", pre + "linear1.bias", F, d, R, F, d)
            native.gemm(A.dh, w(pre + "linear1.weight"), A.dx, R, d, F, b_layout=MN, ldb=d, residual=A.dx, ldr=d,
                        workspace=ws)
            # LN2
            guard(A.dy)
            ln_bwd(l, 2, A.dx, z[1], stt[1], A.dy, base + 3)
            # cross-attention block
            dW(A.dy, A.oc[l], pre + "cross_out.weight", pre + "cross_out.bias", d, d, R, d, d)
            native.gemm(A.dy, w(pre + "cross_out.weight"), A.do, R, d, d, b_layout=MN, ldb=d, workspace=ws)
            kvl, dkvl = A.kv[:, l * 2 * d:], A.dkv[:, l * 2 * d:]
            ca = native.attn_args(A.qc[l], d, T * d, kvl, L * 2 * d, S * L * 2 * d, kvl[:, d:], L * 2 * d,
                                  S * L * 2 * d, A.oc[l], d, T * d, lse=A.lse_c[l], scale=1.0 / math.sqrt(self.hd), drop_p=p,
                                  seed=seed, site=base + 2, key_tokens=mem_keys, tok_batch=S, pad_idx=0)
            cg = native.attn_grads(A.do, d, T * d, A.dq, d, T * d, dkvl, L * 2 * d, S * L * 2 * d, dkvl[:, d:],
                                   L * 2 * d, S * L * 2 * d, A.delta)
            guard(A.dq)
            native.attention_bwd(native.dtype_code(A.dq), B, H, T, S, ca, cg, Dh=self.hd)
            dW(A.dq, xs[0], pre + "cross_q.weight", pre + "cross_q.bias", d, d, R, d, d)
            native.gemm(A.dq, w(pre + "cross_q.weight"), A.dx, R, d, d, b_layout=MN, ldb=d, residual=A.dx, ldr=d,
                        workspace=ws)
            # LN1
            guard(A.dy)
            ln_bwd(l, 1, A.dx, z[0], stt[0], A.dy, base + 1)
            # self-attention block
            dW(A.dy, A.os[l], pre + "self_out.weight", pre + "self_out.bias", d, d, R, d, d)
            native.gemm(A.dy, w(pre + "self_out.weight"), A.do, R, d, d, b_layout=MN, ldb=d, workspace=ws)
            qkv = A.qkv[l]
            sa = native.attn_args(qkv, 3 * d, T * 3 * d, qkv[:, d:], 3 * d, T * 3 * d, qkv[:, 2 * d:], 3 * d, T * 3 * d,
                                  A.os[l], d, T * d, lse=A.lse_s[l], key_tokens=tokens, tok_batch=T,
                                  pad_idx=self.pad_idx, causal=True, scale=1.0 / math.sqrt(self.hd), drop_p=p, seed=seed,
                                  site=base + 0)
            sg = native.attn_grads(A.do, d, T * d, A.dqkv, 3 * d, T * 3 * d, A.dqkv[:, d:], 3 * d, T * 3 * d,
                                   A.dqkv[:, 2 * d:], 3 * d, T * 3 * d, A.delta)
            guard(A.dqkv)
            native.attention_bwd(native.dtype_code(A.dq), B, H, T, T, sa, sg, Dh=self.hd)
            dW(A.dqkv, xin, pre + "self_in.weight", pre + "self_in.bias", 3 * d, d, R, 3 * d, d)
            native.gemm(A.dqkv, w(pre + "self_in.weight"), A.dx, R, d, 3 * d, b_layout=MN, ldb=d, residual=A.dx,
                        ldr=d, workspace=ws)
            ready(pre + "linear2.weight", pre + "norm1.bias")
        # cross K/V of all layers
        if pair:
            # the memory gradient first, then the projection weight gradient -- with the cross-K/V one
            # as a group unless that went out early (kv_early) -- the step's last GEMMs
            enc_rows, enc_ld, E = proj_input
            native.gemm(A.dkv, w("cross_kv.weight"), A.dmem, BS, d, L * 2 * d, b_layout=MN, ldb=d, workspace=ws)
            tail = ([] if early else [kv_prob]) + [
                (A.dmem, enc_rows, g("projection.weight"), d, E, BS, d, enc_ld, g("projection.bias"))]
            if A.gws_tail is None:
                A.gws_tail = torch.empty((native.gemm_grouped_ws_bytes(tail) + 255) // 4, dtype=torch.float32,
                                         device=self.device)
            side.run(lambda: native.gemm_grouped(tail, A.gws_tail), reads=(A.dkv, A.dmem))
        else:
            dW(A.dkv, mem, "cross_kv.weight", "cross_kv.bias", L * 2 * d, d, BS, L * 2 * d, mem_ld)
        # embedding (scatter-add into a zeroed table gradient; PAD row gets nothing)
        ge = g("token_embedding.weight")
        if side is not None:
            native.HipEvents.wait(native.stream_ptr(), plan_ev)  # the plan and the zeroed table
        else:
            native.zero(ge)
        native.embed_bwd(tokens, A.dx, math.sqrt(d), ge, self.pad_idx, drop_p=p, seed=seed, site=EMB_SITE,
                         plan=A.emb_plan)
        last = "token_embedding.weight"
        if pair:
            last = "projection.bias"
        elif proj_input is not None:
            enc_rows, enc_ld, E = proj_input
            native.gemm(A.dkv, w("cross_kv.weight"), A.dmem, BS, d, L * 2 * d, b_layout=MN, ldb=d, workspace=ws)
            dW(A.dmem, enc_rows, "projection.weight", "projection.bias", d, E, BS, d, enc_ld)
            last = "projection.bias"
        ready("token_embedding.weight" if early else "cross_kv.weight", last)
        if side is not None:
            side.join()

    def _layer_backward_grouped(self, l, A, tokens, seed, p, xs, z, stt, xin, S, mem_keys, g, w, ln_bwd, guard, side,
                                after_cross=None):
        """One decoder layer of run_backward with its six weight gradients issued as ONE grouped launch
        (native.gemm_grouped) on the side stream after the layer's dX chain; the dY operands live in the
        layer-parity buffers A.gdy / gdh / gdq / gdqkv until that launch has read them."""
        B, T = tokens.shape
        d, H, L, F, R = self.d, self.H, self.L, self.F, A.R
        MN = native.MN_CONTIG
        pre = f"layers.{l}."
        base = 64 * l
        sp = l % 2
        dyF, dyC, dyS = A.gdy[sp]
        dh, dq, dqkv = A.gdh[sp], A.gdq[sp], A.gdqkv[sp]
        ascale = 1.0 / (1.0 - p) if p > 0 else 1.0
        ws = A.gemm_ws
        # LN3 -> dz3 (dx, in place) and d(ffn_out)
        guard(dyF)
        j3 = ln_bwd(l, 3, A.dx, z[2], stt[2], dyF, base + 5, defer=True)
        guard(dh)
        native.gemm(dyF, w(pre + "linear2.weight"), dh, R, F, d, b_layout=MN, ldb=F, aux=A.h[l], ld_aux=F,
                    aux_scale=ascale)
        native.gemm(dh, w(pre + "linear1.weight"), A.dx, R, d, F, b_layout=MN, ldb=d, residual=A.dx, ldr=d, workspace=ws)
        guard(dyC)
        j2 = ln_bwd(l, 2, A.dx, z[1], stt[1], dyC, base + 3, defer=True)
        native.gemm(dyC, w(pre + "cross_out.weight"), A.do, R, d, d, b_layout=MN, ldb=d, workspace=ws)
        kvl, dkvl = A.kv[:, l * 2 * d:], A.dkv[:, l * 2 * d:]
        ca = native.attn_args(A.qc[l], d, T * d, kvl, L * 2 * d, S * L * 2 * d, kvl[:, d:], L * 2 * d, S * L * 2 * d,
                              A.oc[l], d, T * d, lse=A.lse_c[l], scale=1.0 / math.sqrt(self.hd), drop_p=p, seed=seed,
                              site=base + 2, key_tokens=mem_keys, tok_batch=S, pad_idx=0)
        cg = native.attn_grads(A.do, d, T * d, dq, d, T * d, dkvl, L * 2 * d, S * L * 2 * d, dkvl[:, d:], L * 2 * d,
                               S * L * 2 * d, A.delta)
        guard(dq)
        native.attention_bwd(native.dtype_code(dq), B, H, T, S, ca, cg, Dh=self.hd)
        if after_cross is not None:
            after_cross()
        native.gemm(dq, w(pre + "cross_q.weight"), A.dx, R, d, d, b_layout=MN, ldb=d, residual=A.dx, ldr=d, workspace=ws)
        guard(dyS)
        j1 = ln_bwd(l, 1, A.dx, z[0], stt[0], dyS, base + 1, defer=True)
        native.gemm(dyS, w(pre + "self_out.weight"), A.do, R, d, d, b_layout=MN, ldb=d, workspace=ws)
        qkv = A.qkv[l]
        sa = native.attn_args(qkv, 3 * d, T * 3 * d, qkv[:, d:], 3 * d, T * 3 * d, qkv[:, 2 * d:], 3 * d, T * 3 * d,
                              A.os[l], d, T * d, lse=A.lse_s[l], key_tokens=tokens, tok_batch=T, pad_idx=self.pad_idx,
                              causal=True, scale=1.0 / math.sqrt(self.hd), drop_p=p, seed=seed, site=base + 0)
        sg = native.attn_grads(A.do, d, T * d, dqkv, 3 * d, T * 3 * d, dqkv[:, d:], 3 * d, T * 3 * d, dqkv[:, 2 * d:],
                               3 * d, T * 3 * d, A.delta)
        guard(dqkv)
        native.attention_bwd(native.dtype_code(dq), B, H, T, T, sa, sg, Dh=self.hd)
        native.gemm(dqkv, w(pre + "self_in.weight"), A.dx, R, d, 3 * d, b_layout=MN, ldb=d, residual=A.dx, ldr=d,
                    workspace=ws)
        probs = [(dyF, A.h[l], g(pre + "linear2.weight"), d, F, R, d, F, g(pre + "linear2.bias")),
                 (dh, xs[1], g(pre + "linear1.weight"), F, d, R, F, d, g(pre + "linear1.bias")),
                 (dyC, A.oc[l], g(pre + "cross_out.weight"), d, d, R, d, d, g(pre + "cross_out.bias")),
                 (dq, xs[0], g(pre + "cross_q.weight"), d, d, R, d, d, g(pre + "cross_q.bias")),
                 (dyS, A.os[l], g(pre + "self_out.weight"), d, d, R, d, d, g(pre + "self_out.bias")),
                 (dqkv, xin, g(pre + "self_in.weight"), 3 * d, d, R, 3 * d, d, g(pre + "self_in.bias"))]
        if A.gws is None:
            A.gws = torch.empty((native.gemm_grouped_ws_bytes(probs) + 255) // 4, dtype=torch.float32,
                                device=self.device)
        side.run(lambda: native.gemm_grouped(probs, A.gws, ln_jobs=(j3, j2, j1)), reads=(dyF, dh, dyC, dq, dyS, dqkv))

    # --- batched greedy decoding with a KV cache (config 5) ---------------------------------------
    def decode_begin(self, mem: torch.Tensor, mem_ld: int, S: int, B: int, max_len: int, start_id: int,
                     end_id: int) -> "DecodeState":
        """Set up a batched greedy decode over B images whose memory rows are mem [B*S, d] (row
        stride mem_ld): cross-attention K/V of every layer computed once (one fused GEMM), empty
        self-attention caches, ids[:, 0] = START, position 0 on the device."""
        if max_len > self.pe.shape[0]:
            raise ValueError(f"max_len {max_len} exceeds the positional table ({self.pe.shape[0]} = "
                             f"decoder_max_seq_len; the reference's PositionalEncoding would fail too)")
        stt = DecodeState(self, B, S, max_len, start_id, end_id)
        d, L, st = self.d, self.L, self.store
        wkv, bkv = st.w("cross_kv.weight"), st.p("cross_kv.bias")
        for l in range(L):
            native.gemm(mem, wkv[l * 2 * d:], stt.kv[l], B * S, 2 * d, d, lda=mem_ld, bias=bkv[l * 2 * d:])
        return stt

    def decode_step(self, stt: "DecodeState"):
        """One greedy token for every row: position p = stt.pos (device) -> ids[:, p+1]; p += 1.
        No host synchronisation: capturable into a hipGraph."""
        if stt.fused:
            return self._decode_step_fused(stt)
        d, H, L, V = self.d, self.H, self.L, self.V
        st, w = self.store, self.store.w
        B, S, Tm = stt.B, stt.S, stt.max_len
        native.embed_decode(stt.ids, stt.pos, w("token_embedding.weight"), math.sqrt(d), self.pe, stt.x)
        x = stt.x
        for l in range(L):
            pre = f"layers.{l}."
            cache = stt.cache[l]
            native.linear(x, w(pre + "self_in.weight"), stt.qkv, bias=st.p(pre + "self_in.bias"))
            native.kv_store(stt.qkv[:, d:], 3 * d, cache, 2 * d, Tm * 2 * d, B, 2 * d, stt.pos)
            native.attention_decode(stt.qkv, 3 * d, cache, 2 * d, Tm * 2 * d, cache[:, :, d:], 2 * d, Tm * 2 * d, stt.o,
                                    d, B, H, pos=stt.pos, key_tokens=stt.ids, tok_batch=Tm, pad_idx=self.pad_idx,
                                    scale=1.0 / math.sqrt(self.hd), Dh=self.hd)
            native.linear(stt.o, w(pre + "self_out.weight"), stt.y, bias=st.p(pre + "self_out.bias"))
            native.layernorm_fwd(x, st.p(pre + "norm1.weight"), st.p(pre + "norm1.bias"), 1e-5, stt.x1, r=stt.y)
            native.linear(stt.x1, w(pre + "cross_q.weight"), stt.q, bias=st.p(pre + "cross_q.bias"))
            kvl = stt.kv[l]
            native.attention_decode(stt.q, d, kvl, 2 * d, S * 2 * d, kvl[:, d:], 2 * d, S * 2 * d,
                                    stt.o, d, B, H, Lk=S, scale=1.0 / math.sqrt(self.hd), Dh=self.hd)
            native.linear(stt.o, w(pre + "cross_out.weight"), stt.y, bias=st.p(pre + "cross_out.bias"))
            native.layernorm_fwd(stt.x1, st.p(pre + "norm2.weight"), st.p(pre + "norm2.bias"), 1e-5, stt.x2, r=stt.y)
            native.linear(stt.x2, w(pre + "linear1.weight"), stt.h, bias=st.p(pre + "linear1.bias"),
                          act=native.ACT_RELU)
            native.linear(stt.h, w(pre + "linear2.weight"), stt.y, bias=st.p(pre + "linear2.bias"))
            native.layernorm_fwd(stt.x2, st.p(pre + "norm3.weight"), st.p(pre + "norm3.bias"), 1e-5, x, r=stt.y)
        native.linear(x, w("fc_out.weight"), stt.logits, bias=st.p("fc_out.bias"))
        native.greedy_pick(stt.logits, stt.ids, stt.pos, stt.end_id, self.pad_idx, stt.finished, stt.n_finished, V=V)
        native.step_inc(stt.pos)

    def _decode_step_fused(self, stt: "DecodeState"):
        """decode_step on bf16 with 8 GEMM/attention launches per layer (was 12): every post-LN residual
        block (transformer.py:1144-1153) is z = sublayer + LN_prev(z_prev) written in f32 by the
        GEMM that produces the sublayer output, and LN(z) is applied by its consumers (the next
        GEMM's operand staging / residual epilogue); the self-attention K|V row goes straight from the
        in_proj GEMM into the cache; the vocabulary head leaves each row's argmax as a packed atomic max
        (no logits in HBM) and the pick reads it and advances the position."""
        d, H, L, V = self.d, self.H, self.L, self.V
        st, w, p = self.store, self.store.w, self.store.p
        B, S, Tm = stt.B, stt.S, stt.max_len
        z1, z2, z3 = stt.z
        s1, s2, s3 = stt.zst
        scale = 1.0 / math.sqrt(self.hd)
        native.embed_decode(stt.ids, stt.pos, w("token_embedding.weight"), math.sqrt(d), self.pe, stt.x)
        for l in range(L):
            pre = f"layers.{l}."
            cache = stt.cache[l]
            if l == 0:
                a, a_ln = stt.x, None
            else:
                q3 = f"layers.{l - 1}.norm3."
                a, a_ln = z3, (s3, p(q3 + "weight"), p(q3 + "bias"))
            ln1 = (s1, p(pre + "norm1.weight"), p(pre + "norm1.bias"))
            ln2 = (s2, p(pre + "norm2.weight"), p(pre + "norm2.bias"))
            native.decode_gemm(a, w(pre + "self_in.weight"), out=stt.qkv, bias=p(pre + "self_in.bias"), a_ln=a_ln,
                               cache=cache, c_row=2 * d, c_batch=Tm * 2 * d, kv_col0=d, pos=stt.pos)
            native.attention_decode(stt.qkv, 3 * d, cache, 2 * d, Tm * 2 * d, cache[:, :, d:], 2 * d, Tm * 2 * d, stt.o,
                                    d, B, H, pos=stt.pos, key_tokens=stt.ids, tok_batch=Tm, pad_idx=self.pad_idx,
                                    scale=scale, Dh=self.hd)
            native.decode_gemm(stt.o, w(pre + "self_out.weight"), bias=p(pre + "self_out.bias"), residual=a, r_ln=a_ln,
                               z_out=z1, stats_out=s1)
            native.decode_gemm(z1, w(pre + "cross_q.weight"), out=stt.q, bias=p(pre + "cross_q.bias"), a_ln=ln1)
            kvl = stt.kv[l]
            native.attention_decode(stt.q, d, kvl, 2 * d, S * 2 * d, kvl[:, d:], 2 * d, S * 2 * d,
                                    stt.o, d, B, H, Lk=S, scale=scale, Dh=self.hd)
            native.decode_gemm(stt.o, w(pre + "cross_out.weight"), bias=p(pre + "cross_out.bias"), residual=z1,
                               r_ln=ln1, z_out=z2, stats_out=s2)
            native.decode_gemm(z2, w(pre + "linear1.weight"), out=stt.h, bias=p(pre + "linear1.bias"),
                               act=native.ACT_RELU, a_ln=ln2)
            native.decode_gemm(stt.h, w(pre + "linear2.weight"), bias=p(pre + "linear2.bias"), residual=z2, r_ln=ln2,
                               z_out=z3, stats_out=s3)
        q3 = f"layers.{L - 1}.norm3."
        native.decode_layernorm(z3, s3, p(q3 + "weight"), p(q3 + "bias"), stt.x)
        # the head on the 128x128 GEMM with the argmax epilogue (mit_gemm argmax_keys): one round of 158 blocks,
        # ~10 us, against ~20 us for mit_decode_gemm's 628 split-K 64x64 blocks at one per CU
        # (per token step, 3 interleaved processes on one box: 667 -> 658 us, 383.7 k -> 389.0 k tokens/s)
        native.gemm(stt.x, w("fc_out.weight")[:V], None, B, V, d, bias=p("fc_out.bias")[:V], argmax_keys=stt.keys)
        native.greedy_pick_keys(stt.keys, stt.ids, stt.pos, stt.end_id, self.pad_idx, stt.finished, stt.n_finished)

    def forward_ops(self, tokens: torch.Tensor, mem: torch.Tensor, S: int, params: Dict[str, torch.Tensor],
                    seed: Optional[torch.Tensor], drop_p: float, mem_keys: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The forward of run_forward built from torch.ops.mit_hip operators (ops.py), so torch's autograd
        records it and ``loss.backward()`` runs each op's HIP backward (the reference loop, train.py:80-100).
        tokens int64 [B, T]; mem [B*S, d] memory rows (may require grad: the projection's output);
        params: the trainable f32 tensors by flat entry name (the model's nn.Parameters), whose compute-dtype
        shadows (store.w) the GEMMs read. Returns f32 logits [B, T, V]. Same kernels, dropout sites and
        seeds as run_forward: the same values."""
        import ops
        mh = ops.load()
        B, T = tokens.shape
        d, H, L = self.d, self.H, self.L
        st = self.store
        lp = (lambda n: st.w(n)) if st.shadow is not st.master else (lambda n: None)  # noqa: E731
        P = params
        sc = 1.0 / math.sqrt(self.hd)
        x = mh.embedding(tokens, P["token_embedding.weight"], self.pe, math.sqrt(d), drop_p, seed, EMB_SITE,
                         lp("token_embedding.weight"), self.pad_idx)
        kv = mh.linear(mem, P["cross_kv.weight"], P["cross_kv.bias"], weight_lp=lp("cross_kv.weight")).view(B, S, L * 2 * d)
        for l in range(L):
            q = f"layers.{l}."
            base = 64 * l

            def lin(t, n):
                return mh.linear(t, P[q + n + ".weight"], P[q + n + ".bias"], weight_lp=lp(q + n + ".weight"))

            def ln(t, r, k, site):
                return mh.layer_norm_train(t, P[q + f"norm{k}.weight"], P[q + f"norm{k}.bias"], 1e-5, r, drop_p, seed,
                                           site)[0]
            qkv = lin(x, "self_in")
            o = mh.attention_train(qkv[..., :d], qkv[..., d:2 * d], qkv[..., 2 * d:], H, True, sc, tokens,
                                   self.pad_idx, drop_p, seed, base + 0)[0]
            x1 = ln(x, lin(o, "self_out"), 1, base + 1)
            kvl = kv[..., l * 2 * d:(l + 1) * 2 * d]
            oc = mh.attention_train(lin(x1, "cross_q"), kvl[..., :d], kvl[..., d:], H, False, sc, mem_keys, 0, drop_p,
                                    seed, base + 2)[0]
            x2 = ln(x1, lin(oc, "cross_out"), 2, base + 3)
            y = mh.ffn(x2, P[q + "linear1.weight"], P[q + "linear1.bias"], P[q + "linear2.weight"],
                       P[q + "linear2.bias"], drop_p, seed, base + 4, lp(q + "linear1.weight"),
                       lp(q + "linear2.weight"))[0]
            x = ln(x2, y, 3, base + 5)
        logits = mh.linear(x, P["fc_out.weight"], P["fc_out.bias"], out_f32=True, weight_lp=lp("fc_out.weight"))
        return logits if self.Vp == self.V else logits[..., :self.V]

    def forward(self, tgt_tokens: torch.Tensor, memory: torch.Tensor, memory_padding_mask=None) -> torch.Tensor:
        """decoder.py:134-193: f32 logits [B, T, V] (no autograd; training goes through the model's
        train step). memory_padding_mask: bool [B, S], True = padded memory position, masked out of
        the cross-attention (memory_key_padding_mask, decoder.py:179-186); a query whose memory is
        all padding gets NaN, like the reference."""
        tokens = tgt_tokens.to(self.device, torch.int64).contiguous()
        B, T = tokens.shape
        S = memory.shape[1]
        self.store.ensure_shadow(force=True)
        mem = memory.to(self.device, self.dtype).reshape(B * S, self.d).contiguous()
        keys = None
        if memory_padding_mask is not None:
            if tuple(memory_padding_mask.shape) != (B, S):
                raise ValueError(f"memory_padding_mask must be [B, S] = {(B, S)}, got {tuple(memory_padding_mask.shape)}")
            keys = (~memory_padding_mask.to(self.device, torch.bool)).to(torch.int64).contiguous()
        A = self.acts(B, T, S, False)
        out = torch.empty(B * T, self.Vp, dtype=torch.float32, device=self.device)
        self.run_forward(tokens, mem, self.d, S, A, None, False, logits_out=out, mem_keys=keys)
        return self.unpad_logits(out, B, T)

    __call__ = forward

    def unpad_logits(self, out: torch.Tensor, B: int, T: int) -> torch.Tensor:
        """[B*T, Vp] head output -> [B, T, V] (a copy only when V is not a multiple of 8)."""
        if self.Vp == self.V:
            return out.view(B, T, self.V)
        return out[:, :self.V].reshape(B, T, self.V)

    def flops_per_sequence(self, T: int, S: int) -> float:
        """Algorithmic forward FLOPs for one caption (SURVEY.md §8d convention)."""
        d, F, V, L = self.d, self.F, self.V, self.L
        layer = 2 * T * 3 * d * d + 2 * T * d * d + 4 * T * T * d + 2 * T * d * d + 2 * S * 2 * d * d + 4 * T * S * d \
            + 2 * T * d * d + 2 * T * 2 * d * F
        return L * layer + 2 * T * d * V
