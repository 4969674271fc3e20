"""Frozen vision encoder (ViT / CLIP vision tower), forward only, on the gfx950 kernels.

Replaces the HF modules the reference loads in model.py:48-66 and calls at model.py:133-141:
  ViT  (tf/models/vit/modeling_vit.py:356-389): Conv2d patch embed + CLS + position embeddings,
       pre-LN layers (LN eps 1e-12, MHSA scale 1/8, GELU(erf) MLP), final LayerNorm.
  CLIP (tf/models/clip/modeling_clip.py:613-657): bias-free patch conv, class + position embeddings,
       pre_layrnorm, pre-LN layers with quick_gelu, NO post-LN on last_hidden_state.
The pooler (modeling_vit.py:386) is not observable through last_hidden_state and is not computed.

Per layer: LN -> one packed QKV GEMM (N = 3E) -> attention -> o_proj GEMM with the residual add
fused in its epilogue -> LN -> fc1 GEMM with GELU fused -> fc2 GEMM with the residual fused.
Weights live in the compute dtype (bf16 or f32); biases and LN parameters in f32.

Also the counterpart of the reference's standalone encoder.py helpers (encoder.py:65-124):
``get_encoder_output_dim`` and ``encode_image``.
"""
from __future__ import annotations

import math
import re
from typing import Dict, Optional

import torch

import config
import native


def _round8(x):
    return (x + 7) // 8 * 8


def _normalize_hf_key(k: str) -> str:
    """Map HF ViT/CLIP vision state_dict names (transformers 4.x or 5.x, with or without the
    'encoder.' / 'vision_model.' prefixes the reference's checkpoints carry) to one scheme."""
    for pre in ("encoder.vision_model.", "vision_model.", "encoder."):
        if k.startswith(pre) and not k.startswith(("encoder.layer.", "encoder.layers.")):
            k = k[len(pre):]
            break
    if k.startswith("encoder.") and k[len("encoder."):].startswith(("layer.", "layers.")):
        k = k[len("encoder."):]
    k = re.sub(r"^layer\.", "layers.", k)
    # transformers 4.x ViT
    k = k.replace("attention.attention.query", "attention.q_proj").replace("attention.attention.key", "attention.k_proj")
    k = k.replace("attention.attention.value", "attention.v_proj").replace("attention.output.dense", "attention.o_proj")
    k = k.replace("intermediate.dense", "mlp.fc1")
    k = re.sub(r"(layers\.\d+)\.output\.dense", r"\1.mlp.fc2", k)
    # CLIP names -> ViT-style names
    k = k.replace("self_attn.q_proj", "attention.q_proj").replace("self_attn.k_proj", "attention.k_proj")
    k = k.replace("self_attn.v_proj", "attention.v_proj").replace("self_attn.out_proj", "attention.o_proj")
    k = k.replace("layer_norm1", "layernorm_before").replace("layer_norm2", "layernorm_after")
    return k


_END = object()  # end-of-generator sentinel (forward_iter_groups)


def drain(it):
    """Run a launch-chunk generator (VisionEncoder.forward_iter) to its end; returns its result."""
    while True:
        try:
            next(it)
        except StopIteration as e:
            return e.value


class VisionEncoder:
    """Frozen encoder. ``spec`` = config.ENCODER_SPECS entry (kind, hidden, layers, heads, mlp, image, patch, eps)."""

    def __init__(self, spec: dict, device, dtype: torch.dtype):
        self.spec = dict(spec)
        self.kind = spec["kind"]
        self.E, self.L, self.H, self.mlp = spec["hidden"], spec["layers"], spec["heads"], spec["mlp"]
        self.image, self.patch, self.eps = spec["image"], spec["patch"], spec["eps"]
        if self.E % self.H or self.E // self.H not in (16, 32, 64, 128):
            raise ValueError(f"encoder head_dim {self.E / self.H} unsupported (kernels take 16, 32, 64, 128)")
        self.hd = self.E // self.H
        self.np = (self.image // self.patch) ** 2
        self.N = self.np + 1
        self.kin = 3 * self.patch * self.patch
        self.kpad = _round8(self.kin)
        self.device, self.dtype = device, dtype
        # bf16 stream: each pre-LN sublayer's LayerNorm folded into the GEMM that consumes it (fold_layernorm):
        # no LayerNorm launch inside the tower, the statistics come from the producing GEMM's epilogue. ViT
        # towers only: on the 2-layer CLIP-336 cls fixture the folded path's largest logit error (0.039) left
        # the asserted 1.5x of the reference's own bf16 error (0.037) while its encoder rel-L2 improved
        # (5.40e-3 vs 5.54e-3); the deep CLIP-L towers run the f32 residual stream anyway
        self._fold_ok = (dtype == torch.bfloat16 and self.E % 64 == 0 and self.kind == "vit"
                         and str(getattr(config, "ENCODER_FOLD_LN", "auto")).lower() not in ("off", "0", "false"))
        self.w: Dict[str, torch.Tensor] = {}
        self._ws = {}
        self.configure_for(None)

    def configure_for(self, memory_mode: Optional[str]):
        """Pick the residual-stream precision for the decoder memory this encoder feeds (the model calls this
        with its memory_mode). f32 residual stream (bf16 compute only): z = h + sublayer(bf16) in f32, fused
        into the next LayerNorm (mit_layernorm_fwd_x32), as autocast keeps modeling_vit.py:312-323 /
        modeling_clip.py:379-393. config.ENCODER_F32_RESIDUAL "auto" turns it on
          - for the 24-layer CLIP-L towers (configs[2] / configs[3]): a bf16 stream doubles their error;
          - in "cls" memory mode (model.py:141-151): the memory is ONE encoder row per image and the
            S = 1 cross-attention passes its error to the logits undamped (patches mode averages it over
            197 rows). tools/bf16_bisect.py on cfg0_b4_cls: logits rel-L2 9.64e-3 (1.20x the reference's
            own bf16 error) with the bf16 stream, 8.53e-3 (1.06x) with the f32 one; encoder alone 7.26e-3
            vs 6.26e-3 for the decoder alone. The bench path (patches) keeps the folded bf16 stream.
        "on" / "off" force it."""
        mode = str(getattr(config, "ENCODER_F32_RESIDUAL", "auto")).lower()
        res32 = self.dtype == torch.bfloat16 and (
            mode in ("on", "1", "true") or (mode == "auto" and (self.L >= 24 or memory_mode == "cls")))
        if getattr(self, "res32", None) != res32:
            self._ws = {}  # the arenas differ between the two streams
        self.res32 = res32
        self.fold_ln = self._fold_ok and not res32  # the folded operands exist whenever _fold_ok (load time)
        return self

    # --- weights -----------------------------------------------------------------------------
    @property
    def hidden_size(self):
        return self.E

    # tensors the reference model holds but last_hidden_state never reads (ViTModel's pooler,
    # modeling_vit.py:386; CLIPVisionTransformer's post_layernorm, modeling_clip.py:649): kept as
    # host copies so state_dict() round-trips and the parameter count matches the reference's
    def _extra_shapes(self):
        E = self.E
        if self.kind == "vit":
            return {"pooler.dense.weight": (E, E), "pooler.dense.bias": (E,)}
        return {"post_layernorm.weight": (E,), "post_layernorm.bias": (E,)}

    def num_reference_params(self) -> int:
        """len(list(encoder.parameters())) of the reference's HF module: patch/cls/pos (+ CLIP's
        pre_layrnorm), 16 per layer, ViT's final LayerNorm, and the extras above."""
        if self.kind == "vit":
            return 4 + 16 * self.L + 2 + 2
        return 3 + 2 + 16 * self.L + 2

    def _collect(self, sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        """HF-named state -> this encoder's host tensors; raises KeyError / ValueError (nothing is
        modified) when a tensor is missing or has the wrong shape."""
        n = {_normalize_hf_key(k): v.detach().float().cpu() for k, v in sd.items()}
        E, mlp = self.E, self.mlp

        def get(k, shape):
            if k not in n:
                raise KeyError(f"encoder weight '{k}' missing (have e.g. {sorted(n)[:4]})")
            t = n[k]
            if t.numel() != int(torch.tensor(shape).prod()):
                raise ValueError(f"encoder weight '{k}': {tuple(t.shape)} does not fit {shape}")
            return t.reshape(shape)

        w = {}
        if self.kind == "vit":
            pw = get("embeddings.patch_embeddings.projection.weight", (E, self.kin))
            pb = get("embeddings.patch_embeddings.projection.bias", (E,))
            cls = get("embeddings.cls_token", (E,))
            pos = get("embeddings.position_embeddings", (self.N, E))
        else:
            pw = get("embeddings.patch_embedding.weight", (E, self.kin))
            pb = torch.zeros(E)
            cls = get("embeddings.class_embedding", (E,))
            pos = get("embeddings.position_embedding.weight", (self.N, E))
            w["pre_ln.w"] = get("pre_layrnorm.weight", (E,))
            w["pre_ln.b"] = get("pre_layrnorm.bias", (E,))
        pwp = torch.zeros(E, self.kpad)
        pwp[:, :self.kin] = pw
        w["patch.w"], w["patch.b"], w["cls"], w["pos"] = pwp, pb, cls, pos
        for i in range(self.L):
            p = f"layers.{i}."
            w[f"{i}.ln1.w"], w[f"{i}.ln1.b"] = get(p + "layernorm_before.weight", (E,)), get(p + "layernorm_before.bias", (E,))
            w[f"{i}.ln2.w"], w[f"{i}.ln2.b"] = get(p + "layernorm_after.weight", (E,)), get(p + "layernorm_after.bias", (E,))
            w[f"{i}.qkv.w"] = torch.cat([get(p + f"attention.{x}_proj.weight", (E, E)) for x in "qkv"], 0)
            w[f"{i}.qkv.b"] = torch.cat([get(p + f"attention.{x}_proj.bias", (E,)) for x in "qkv"], 0)
            w[f"{i}.o.w"], w[f"{i}.o.b"] = get(p + "attention.o_proj.weight", (E, E)), get(p + "attention.o_proj.bias", (E,))
            w[f"{i}.fc1.w"], w[f"{i}.fc1.b"] = get(p + "mlp.fc1.weight", (mlp, E)), get(p + "mlp.fc1.bias", (mlp,))
            w[f"{i}.fc2.w"], w[f"{i}.fc2.b"] = get(p + "mlp.fc2.weight", (E, mlp)), get(p + "mlp.fc2.bias", (E,))
        if self.kind == "vit":
            w["final_ln.w"], w["final_ln.b"] = get("layernorm.weight", (E,)), get("layernorm.bias", (E,))
        extra = {k: get(k, shp).clone() for k, shp in self._extra_shapes().items() if k in n}
        return w, extra

    def check_hf_state_dict(self, sd: Dict[str, torch.Tensor]):
        self._collect(sd)

    def load_hf_state_dict(self, sd: Dict[str, torch.Tensor]):
        """Load HF ViTModel / CLIPVisionModel weights (any of the naming schemes above)."""
        w, extra = self._collect(sd)
        dt, dev = self.dtype, self.device
        out = {}
        for k, v in w.items():
            is_mat = k.endswith(".w") and v.dim() == 2 and not k.endswith("ln.w")
            out[k] = v.to(device=dev, dtype=dt if is_mat else torch.float32).contiguous()
        if self._fold_ok:  # from the f32 weights (one rounding of W o gamma), whichever stream runs now
            for i in range(self.L):
                for mat, ln in (("qkv", "ln1"), ("fc1", "ln2")):
                    wf, bf, sf = fold_layernorm(w[f"{i}.{mat}.w"], w[f"{i}.{mat}.b"], w[f"{i}.{ln}.w"], w[f"{i}.{ln}.b"])
                    out[f"{i}.{mat}.wf"] = wf.to(dev).contiguous()
                    out[f"{i}.{mat}.bf"] = bf.to(dev).contiguous()
                    out[f"{i}.{mat}.sf"] = sf.to(dev).contiguous()
        self.w = out
        old = getattr(self, "extra", {})
        self.extra = {k: extra.get(k, old.get(k, torch.zeros(shp))) for k, shp in self._extra_shapes().items()}
        return self

    def hf_state_dict(self) -> Dict[str, torch.Tensor]:
        """Weights back in HF transformers-5.x names (ViTModel / CLIPVisionModel), f32 CPU copies."""
        w, E = {k: v.detach().float().cpu() for k, v in self.w.items()}, self.E
        sd = {}
        pw = w["patch.w"][:, :self.kin].reshape(E, 3, self.patch, self.patch).clone()
        if self.kind == "vit":
            sd["embeddings.cls_token"] = w["cls"].view(1, 1, E)
            sd["embeddings.position_embeddings"] = w["pos"].view(1, self.N, E)
            sd["embeddings.patch_embeddings.projection.weight"] = pw
            sd["embeddings.patch_embeddings.projection.bias"] = w["patch.b"]
            lp, att, ln1, ln2 = "layers.", "attention.", "layernorm_before", "layernorm_after"
            names = dict(q="q_proj", k="k_proj", v="v_proj", o="o_proj")
        else:
            sd["embeddings.class_embedding"] = w["cls"]
            sd["embeddings.patch_embedding.weight"] = pw
            sd["embeddings.position_embedding.weight"] = w["pos"]
            sd["pre_layrnorm.weight"], sd["pre_layrnorm.bias"] = w["pre_ln.w"], w["pre_ln.b"]
            lp, att, ln1, ln2 = "encoder.layers.", "self_attn.", "layer_norm1", "layer_norm2"
            names = dict(q="q_proj", k="k_proj", v="v_proj", o="out_proj")
        for i in range(self.L):
            p = f"{lp}{i}."
            qw, qb = w[f"{i}.qkv.w"], w[f"{i}.qkv.b"]
            for j, x in enumerate("qkv"):
                sd[p + att + names[x] + ".weight"] = qw[j * E:(j + 1) * E].clone()
                sd[p + att + names[x] + ".bias"] = qb[j * E:(j + 1) * E].clone()
            sd[p + att + names["o"] + ".weight"], sd[p + att + names["o"] + ".bias"] = w[f"{i}.o.w"], w[f"{i}.o.b"]
            sd[p + ln1 + ".weight"], sd[p + ln1 + ".bias"] = w[f"{i}.ln1.w"], w[f"{i}.ln1.b"]
            sd[p + ln2 + ".weight"], sd[p + ln2 + ".bias"] = w[f"{i}.ln2.w"], w[f"{i}.ln2.b"]
            sd[p + "mlp.fc1.weight"], sd[p + "mlp.fc1.bias"] = w[f"{i}.fc1.w"], w[f"{i}.fc1.b"]
            sd[p + "mlp.fc2.weight"], sd[p + "mlp.fc2.bias"] = w[f"{i}.fc2.w"], w[f"{i}.fc2.b"]
        if self.kind == "vit":
            sd["layernorm.weight"], sd["layernorm.bias"] = w["final_ln.w"], w["final_ln.b"]
        for k, v in getattr(self, "extra", {}).items():
            sd[k] = v.clone()
        return sd

    def random_init(self, seed: int = 0):
        """Seeded random weights in HF naming (no pretrained weights offline)."""
        g = torch.Generator().manual_seed(seed)
        E, m = self.E, self.mlp

        def rnd(*s, scale):
            return torch.randn(*s, generator=g) * scale

        sd = {}
        if self.kind == "vit":
            sd["embeddings.patch_embeddings.projection.weight"] = rnd(E, 3, self.patch, self.patch, scale=self.kin ** -0.5)
            sd["embeddings.patch_embeddings.projection.bias"] = rnd(E, scale=0.02)
            sd["embeddings.cls_token"] = rnd(1, 1, E, scale=0.02)
            sd["embeddings.position_embeddings"] = rnd(1, self.N, E, scale=0.02)
            sd["layernorm.weight"] = 1 + rnd(E, scale=0.02)
            sd["layernorm.bias"] = rnd(E, scale=0.02)
            sd["pooler.dense.weight"] = rnd(E, E, scale=0.02)
            sd["pooler.dense.bias"] = torch.zeros(E)
        else:
            sd["embeddings.patch_embedding.weight"] = rnd(E, 3, self.patch, self.patch, scale=self.kin ** -0.5)
            sd["embeddings.class_embedding"] = rnd(E, scale=0.02)
            sd["embeddings.position_embedding.weight"] = rnd(self.N, E, scale=0.02)
            sd["pre_layrnorm.weight"] = 1 + rnd(E, scale=0.02)
            sd["pre_layrnorm.bias"] = rnd(E, scale=0.02)
            sd["post_layernorm.weight"] = torch.ones(E)
            sd["post_layernorm.bias"] = torch.zeros(E)
        for i in range(self.L):
            p = f"layers.{i}."
            for x in "qkvo":
                sd[p + f"attention.{x}_proj.weight"] = rnd(E, E, scale=E ** -0.5)
                sd[p + f"attention.{x}_proj.bias"] = rnd(E, scale=0.02)
            sd[p + "layernorm_before.weight"] = 1 + rnd(E, scale=0.02)
            sd[p + "layernorm_before.bias"] = rnd(E, scale=0.02)
            sd[p + "layernorm_after.weight"] = 1 + rnd(E, scale=0.02)
            sd[p + "layernorm_after.bias"] = rnd(E, scale=0.02)
            sd[p + "mlp.fc1.weight"] = rnd(m, E, scale=E ** -0.5)
            sd[p + "mlp.fc1.bias"] = rnd(m, scale=0.02)
            sd[p + "mlp.fc2.weight"] = rnd(E, m, scale=m ** -0.5)
            sd[p + "mlp.fc2.bias"] = rnd(E, scale=0.02)
        return self.load_hf_state_dict(sd)

    # --- forward -----------------------------------------------------------------------------
    def _workspace(self, B, slot=0):
        """Activation arena per (batch, slot): slot 1 is a second arena so a forward for the NEXT
        batch can run on another stream while this batch's output is still being read."""
        key = (B, slot)
        if key not in self._ws:
            R, E, dt, dev = B * self.N, self.E, self.dtype, self.device
            self._ws[key] = dict(
                cols=torch.empty(B * self.np, self.kpad, dtype=dt, device=dev),
                pt=torch.empty(B * self.np, E, dtype=dt, device=dev),
                h=torch.empty(R, E, dtype=dt, device=dev),
                a=torch.empty(R, E, dtype=dt, device=dev),
                qkv=torch.empty(R, 3 * E, dtype=dt, device=dev),
                o=torch.empty(R, E, dtype=dt, device=dev),
                m=torch.empty(R, self.mlp, dtype=dt, device=dev),
            )  # "out" (the ViT final LayerNorm / f32-stream result) is allocated on first use: _out
            if self.fold_ln:  # per-64-column (mean, M2) of the residual stream's rows
                self._ws[key]["st"] = torch.empty(R, E // 64, 2, dtype=torch.float32, device=dev)
            if self.res32:  # f32 residual stream, the bf16 sublayer output (delta) and CLIP's f32 embeddings
                ws = self._ws[key]
                ws["h32"] = torch.empty(R, E, dtype=torch.float32, device=dev)
                ws["d"] = torch.empty(R, E, dtype=dt, device=dev)
                ws["pt32"] = torch.empty(R, E, dtype=torch.float32, device=dev)
                del ws["pt"], ws["h"]
        return self._ws[key]

    def _out(self, ws):
        """The arena's result rows [B*N, E], allocated when a forward first writes them there (the grouped
        forward's per-group arenas write into the shared groups_out buffer instead and never allocate it:
        ~150 MB across its 2 slots x 2 groups at CLIP-L/14@336, B = 64)."""
        if "out" not in ws:
            ws["out"] = torch.empty(ws["qkv"].shape[0], self.E, dtype=self.dtype, device=self.device)
        return ws["out"]

    def forward(self, images: torch.Tensor, rows: str = "all", slot: int = 0) -> torch.Tensor:
        """images f32 [B,3,H,W] (already normalised) -> last_hidden_state in the compute dtype.
        rows="all": [B, N, E] ; rows="cls": only the CLS rows are finalised, returned as the
        strided view [B, E] of the [B, N, E] buffer (row stride N*E)."""
        if self.groups_for(images.shape[0], rows) == 2:
            return drain(self.forward_iter_groups(images, slot))
        return drain(self.forward_iter(images, rows, slot))

    def forward_iter(self, images: torch.Tensor, rows: str = "all", slot: int = 0, out: Optional[torch.Tensor] = None,
                     tiles: int = 0):
        """forward() as a generator of launch chunks: the patch embedding, then one chunk per layer, each
        chunk followed by a yield; the final chunk (last LayerNorm) returns forward()'s result (drain()).
        The train step issues these chunks between its decoder layers (model.prefetch_encoder_iter).
        out: [B*N, E] rows the f32-stream forward writes its result into; tiles: the f32-stream GEMMs' tile
        kernel (mit_gemm_args.tiles; both for forward_iter_groups)."""
        B = images.shape[0]
        if tuple(images.shape[1:]) != (3, self.image, self.image):
            raise ValueError(f"expected images [B,3,{self.image},{self.image}], got {tuple(images.shape)}")
        images = images.contiguous().float()
        ws, w, E = self._workspace(B, slot), self.w, self.E
        native.im2col(images, ws["cols"], self.patch, self.kpad)
        act = native.ACT_GELU if self.kind == "vit" else native.ACT_QUICK_GELU
        if self.res32:
            return (yield from self._forward_res32(B, ws, rows, act, out, tiles))
        if out is not None or tiles:
            raise ValueError("forward_iter: out= / tiles= are for the f32 residual stream")
        native.linear(ws["cols"], w["patch.w"], ws["pt"], bias=w["patch.b"])
        h = ws["h"]
        native.vit_assemble(ws["pt"], w["cls"], w["pos"], h, B, self.np, E)
        if self.kind == "clip":
            native.layernorm_fwd(h, w["pre_ln.w"], w["pre_ln.b"], self.eps, ws["a"])
            h, ws["a"] = ws["a"], h  # swap roles: the normalised tensor is the residual stream
            ws["h"] = h
        a, qkv, o, m = ws["a"], ws["qkv"], ws["o"], ws["m"]
        yield
        for i in range(self.L):
            self._layers(B, h, a, qkv, o, m, act, i, i + 1, ws)
            yield
        return self._finish(B, ws, h, rows)

    # f32-stream towers of at least this many rows run their forward as two image groups (CLIP-L/14@336 at
    # B = 64, 36,928 rows: configs[2] 1879 -> 2010 pairs/s; CLIP-L/14 at B = 64, 16,448 rows: configs[3]
    # 2975 -> 3200 pairs/s, one box each, profiles/r05_clip_groups_ab.txt). Not the ViT-B/16
    # bench path (12,608 rows, folded bf16 stream): its partial rounds already hold the decoder's kernels,
    # and two groups were 1-2 % slower there (13.0-13.2 k vs 13.3 k pairs/s, profiles/r05_decoder_experiments.txt)
    GROUP_ROWS = 16384

    def groups_for(self, B: int, rows: str = "all") -> int:
        """2 when forward_iter_groups applies (CLIP-L/14@336 at B = 64: 36,928 rows), else 1."""
        return 2 if (self.res32 and rows == "all" and B % 2 == 0 and B * self.N >= self.GROUP_ROWS) else 1

    def forward_iter_groups(self, images: torch.Tensor, slot: int = 0):
        """forward_iter(images, "all", slot) as two image groups of B / 2, one on the current stream and
        one on the encoder's second stream, issued chunk by chunk in lockstep (forward() and the model's
        prefetch take this path whenever groups_for says 2, so a batch's rows never depend on which ran). Every 256-tile GEMM grid ends in a partial
        round (CLIP-L/14@336, B = 64: fc2 580 tiles = 2.27 rounds of the 256 CUs, fc1 2320 = 9.06): the
        other group's kernels run in it. Each image goes through the same kernels either way (every op
        is row- or image-wise); the result is one [B*N, E] buffer. The cross-stream edges are
        native.HipEvents (captured by launch plans); the current stream waits for the second one before the
        result is returned."""
        B = images.shape[0]
        Bg, N, E = B // 2, self.N, self.E
        key = ("groups_out", B, slot)
        if key not in self._ws:
            self._ws[key] = torch.empty(B * N, E, dtype=self.dtype, device=self.device)
        gout = self._ws[key]
        if getattr(self, "_stream2", None) is None:
            self._stream2 = torch.cuda.Stream(device=self.device)
            self._gevents = native.HipEvents(8)
        stream2, events = self._stream2, self._gevents
        s0, s1 = native.stream_ptr(), stream2.cuda_stream
        events.wait_stream(s1, s0)  # group 1 starts behind everything issued on the current stream
        # 256 tiles for every GEMM (per shape, the half-batch o-proj / fc2 would take the 128 kernel, whose
        # cost model counts the partial round as idle: 31.3 instead of 28.2 ms, tools/enc_groups_bench.py)
        gens = [self.forward_iter(images[g * Bg:(g + 1) * Bg], "all", 16 + 2 * slot + g,
                                  out=gout[g * Bg * N:(g + 1) * Bg * N], tiles=256) for g in range(2)]
        done = [False, False]
        while True:
            for g in range(2):
                if done[g]:
                    continue
                if g == 1:
                    with torch.cuda.stream(stream2):
                        done[g] = next(gens[g], _END) is _END
                else:
                    done[g] = next(gens[g], _END) is _END
            if all(done):
                break
            yield
        events.wait_stream(s0, s1)
        return gout.view(B, N, E)

    def _attention(self, B, a, qkv, o, i, tiles=0):
        w, E, N, H = self.w, self.E, self.N, self.H
        native.linear(a, w[f"{i}.qkv.w"], qkv, bias=w[f"{i}.qkv.b"], tiles=tiles)
        args = native.attn_args(qkv, 3 * E, N * 3 * E, qkv[:, E:], 3 * E, N * 3 * E, qkv[:, 2 * E:], 3 * E,
                                N * 3 * E, o, E, N * E, scale=1.0 / math.sqrt(self.hd))
        native.attention_fwd(native.dtype_code(qkv), B, H, N, N, args, Dh=self.hd)

    def _layers(self, B, h, a, qkv, o, m, act, i0, i1, ws=None):
        w = self.w
        if self.fold_ln:
            return self._layers_folded(B, h, qkv, o, m, act, i0, i1, ws)
        for i in range(i0, i1):
            native.layernorm_fwd(h, w[f"{i}.ln1.w"], w[f"{i}.ln1.b"], self.eps, a)
            self._attention(B, a, qkv, o, i)
            native.linear(o, w[f"{i}.o.w"], h, bias=w[f"{i}.o.b"], residual=h)
            native.layernorm_fwd(h, w[f"{i}.ln2.w"], w[f"{i}.ln2.b"], self.eps, a)
            native.linear(a, w[f"{i}.fc1.w"], m, bias=w[f"{i}.fc1.b"], act=act)
            native.linear(m, w[f"{i}.fc2.w"], h, bias=w[f"{i}.fc2.b"], residual=h)

    def _layers_folded(self, B, h, qkv, o, m, act, i0, i1, ws):
        """The bf16-stream layers with every LayerNorm folded into its consumer GEMM (mit_gemm ln_stats): the
        qkv and fc1 GEMMs read the raw residual stream h and normalise in the epilogue from per-64-column
        row statistics, which the o-proj / fc2 residual GEMMs write for the h they produce (stats_out);
        layer 0's come from one mit_row_stats64 pass over the embeddings. 5 launches per layer instead of 7,
        no LayerNorm output round trip through HBM (2 x 19 MB per LayerNorm at ViT-B/16, B = 64)."""
        w, E, R = self.w, self.E, B * self.N
        st = ws["st"]
        if i0 == 0:
            native.row_stats64(h, st)
        for i in range(i0, i1):
            native.gemm(h, w[f"{i}.qkv.wf"], qkv, R, 3 * E, E, bias=w[f"{i}.qkv.bf"], ln_stats=st,
                        ln_colsum=w[f"{i}.qkv.sf"], ln_eps=self.eps)
            args = native.attn_args(qkv, 3 * E, self.N * 3 * E, qkv[:, E:], 3 * E, self.N * 3 * E, qkv[:, 2 * E:], 3 * E,
                                    self.N * 3 * E, o, E, self.N * E, scale=1.0 / math.sqrt(self.hd))
            native.attention_fwd(native.dtype_code(qkv), B, self.H, self.N, self.N, args, Dh=self.hd)
            native.gemm(o, w[f"{i}.o.w"], h, R, E, E, bias=w[f"{i}.o.b"], residual=h, stats_out=st)
            native.gemm(h, w[f"{i}.fc1.wf"], m, R, self.mlp, E, bias=w[f"{i}.fc1.bf"], act=act, ln_stats=st,
                        ln_colsum=w[f"{i}.fc1.sf"], ln_eps=self.eps)
            native.gemm(m, w[f"{i}.fc2.w"], h, R, E, self.mlp, bias=w[f"{i}.fc2.b"], residual=h, stats_out=st)

    def _forward_res32(self, B, ws, rows, act, out=None, tiles=0):
        """The same forward with the residual stream h32 in f32: every sublayer output (o-proj, fc2)
        is written in bf16 to d and added to h32 in f32 by the next LayerNorm (z = h32 + d written back,
        y = LN(z)), so the stream is never rounded to bf16 -- torch.autocast's arithmetic for the
        reference's HF layers. Patch embedding, QKV / attention / MLP operands stay bf16."""
        w, E = self.w, self.E
        h32, d, a, qkv, o, m = ws["h32"], ws["d"], ws["a"], ws["qkv"], ws["o"], ws["m"]
        if self.kind == "vit":
            native.linear(ws["cols"], w["patch.w"], ws["pt32"], bias=w["patch.b"])
            native.vit_assemble(ws["pt32"], w["cls"], w["pos"], h32, B, self.np, E)
        else:  # patch + class + positions -> pt32, pre_layrnorm (f32 out) -> the stream h32
            pt32 = ws["pt32"]
            native.linear(ws["cols"], w["patch.w"], h32[:B * self.np], bias=w["patch.b"])
            native.vit_assemble(h32[:B * self.np], w["cls"], w["pos"], pt32, B, self.np, E)
            native.layernorm_fwd_x32(pt32, w["pre_ln.w"], w["pre_ln.b"], self.eps, h32)
        yield
        pend = None
        for i in range(self.L):
            native.layernorm_fwd_x32(h32, w[f"{i}.ln1.w"], w[f"{i}.ln1.b"], self.eps, a, r=pend,
                                     z=h32 if pend is not None else None)
            self._attention(B, a, qkv, o, i, tiles)
            native.linear(o, w[f"{i}.o.w"], d, bias=w[f"{i}.o.b"], tiles=tiles)
            native.layernorm_fwd_x32(h32, w[f"{i}.ln2.w"], w[f"{i}.ln2.b"], self.eps, a, r=d, z=h32)
            native.linear(a, w[f"{i}.fc1.w"], m, bias=w[f"{i}.fc1.b"], act=act, tiles=tiles)
            native.linear(m, w[f"{i}.fc2.w"], d, bias=w[f"{i}.fc2.b"], tiles=tiles)
            pend = d
            yield
        N = self.N
        out = self._out(ws) if out is None else out
        if self.kind == "vit":
            if rows == "cls":
                native.layernorm_fwd_x32(h32, w["final_ln.w"], w["final_ln.b"], self.eps, out, r=pend, rows=B,
                                         cols=E, ldx=N * E, ldr=N * E, ldy=N * E)
                return out.view(B, N, E)[:, 0, :]
            native.layernorm_fwd_x32(h32, w["final_ln.w"], w["final_ln.b"], self.eps, out, r=pend)
            return out.view(B, N, E)
        if rows == "cls":
            native.residual_out(h32, pend, out, rows=B, cols=E, ldx=N * E, ldr=N * E, ldy=N * E)
            return out.view(B, N, E)[:, 0, :]
        native.residual_out(h32, pend, out)
        return out.view(B, N, E)

    def _finish(self, B, ws, h, rows):
        w, E, N = self.w, self.E, self.N
        if self.kind == "vit":
            out = self._out(ws)
            if rows == "cls":
                native.layernorm_fwd(h, w["final_ln.w"], w["final_ln.b"], self.eps, out, rows=B, cols=E, ldx=N * E,
                                     ldy=N * E)
                return out.view(B, N, E)[:, 0, :]
            native.layernorm_fwd(h, w["final_ln.w"], w["final_ln.b"], self.eps, out)
            return out.view(B, N, E)
        return h.view(B, N, E)[:, 0, :] if rows == "cls" else h.view(B, N, E)

    def flops_per_image(self) -> float:
        """Algorithmic forward FLOPs per image (SURVEY.md §8d convention)."""
        N, E, m = self.N, self.E, self.mlp
        per_layer = 2 * N * 4 * E * E + 2 * N * 2 * E * m + 4 * N * N * E
        return self.L * per_layer + 2 * (N - 1) * E * self.kin


def fold_layernorm(W: torch.Tensor, b: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor):
    """A pre-LN sublayer y = LN(x) W^T + b with LN(x) = (x - mean) rstd gamma + beta, rewritten for a GEMM on
    the raw rows x (mit_gemm ln_stats): y = rstd (x (W o gamma)^T - mean s) + (b + W beta), s_n = sum_k
    (W o gamma)_nk. Returns (W o gamma in bf16 -- what the GEMM reads --, the folded bias f32, s f32 summed
    from the bf16-rounded weights so the mean term cancels exactly what the GEMM accumulates). The frozen
    encoder's weights never change, so this runs once at load (encoder.py:load_hf_state_dict)."""
    W64, g64 = W.double(), gamma.double()
    wf = (W64 * g64[None, :]).to(torch.bfloat16)
    s = wf.double().sum(1).float()
    bf = (b.double() + W64 @ beta.double()).float()
    return wf, bf, s


def get_encoder_output_dim(name: Optional[str] = None) -> int:
    """encoder.py:112-124 counterpart: hidden size of the named encoder."""
    return config.ENCODER_SPECS[name or config.ENCODER_MODEL_NAME]["hidden"]


def build_encoder(name: Optional[str] = None, device=None, dtype=None, weights_path=None, seed=0) -> VisionEncoder:
    """model.py:48-66 counterpart without the network: geometry from config.ENCODER_SPECS, weights
    from a local safetensors file (HF names) if given, else seeded random init."""
    name = name or config.ENCODER_MODEL_NAME
    if name not in config.ENCODER_SPECS:
        raise ValueError(f"encoder '{name}' is not supported (have {sorted(config.ENCODER_SPECS)})")
    device = device or torch.device("cuda")
    dtype = dtype or (torch.bfloat16 if config.DTYPE == "bf16" else torch.float32)
    enc = VisionEncoder(config.ENCODER_SPECS[name], device, dtype)
    path = weights_path if weights_path is not None else config.ENCODER_WEIGHTS_PATH
    if path:
        from safetensors.torch import load_file
        enc.load_hf_state_dict(load_file(path))
    else:
        enc.random_init(seed)
    return enc
