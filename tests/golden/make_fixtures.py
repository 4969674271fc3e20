"""Generate the golden fixtures by running the REFERENCE code in this container.

TEST INFRASTRUCTURE ONLY — run here (where /root/reference exists), never on the GPU box:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_fixtures.py

What runs is the reference's own code, unmodified, imported from /root/reference:
  * ``model.ImageToTextModel.forward`` / ``.generate`` (model.py:116-169, 171-242), bound to an
    object built with ``__new__`` because ``__init__`` downloads weights (model.py:50,70 — no network);
    the encoder is a locally constructed HF ``ViTModel`` / ``CLIPVisionModel``;
  * ``decoder.TransformerDecoder`` (decoder.py:75-193) including its masks from utils.py;
  * ``train.train_one_epoch`` (train.py:62-123), extracted with ``ast`` from train.py and executed
    (``import train`` itself fails offline: wandb/torchvision/dataset download at import);
  * ``torch.optim.AdamW`` / ``nn.CrossEntropyLoss(ignore_index=PAD)`` configured as train.py:319-327.

The "patches" memory mode (north star: cross-attention over the whole patch sequence) is the
reference decoder fed ``projection(last_hidden_state)``; everything else in that
path is reference code.

Inputs and weights are regenerated from seeds (procedural.py); fixtures store outputs only, as
float32 tensors in one .safetensors per case, plus a JSON ``meta`` entry in the safetensors header.
All dropout probabilities are 0 (dropout RNG streams cannot match across implementations).
"""
from __future__ import annotations

import ast
import json
import math
import os
import sys

os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, REF)

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
from safetensors.torch import save_file  # noqa: E402
from tqdm import tqdm  # noqa: E402
from transformers import CLIPVisionConfig, CLIPVisionModel, ViTConfig, ViTModel, ViTImageProcessor  # noqa: E402
from PIL import Image  # noqa: E402

import config as ref_config  # noqa: E402  (reference config.py)
import decoder as ref_decoder  # noqa: E402
import model as ref_model  # noqa: E402
import procedural as P  # noqa: E402

torch.set_num_threads(8)


def _load_train_functions():
    """Exec train.py's train_one_epoch/evaluate (train.py:62-151) without importing train.py."""
    src = open(os.path.join(REF, "train.py")).read()
    tree = ast.parse(src)
    fns = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in ("train_one_epoch", "evaluate")]
    mod = ast.Module(body=fns, type_ignores=[])
    ns = {"torch": torch, "tqdm": tqdm, "wandb": None}
    exec(compile(mod, os.path.join(REF, "train.py"), "exec"), ns)
    return ns["train_one_epoch"], ns["evaluate"]


train_one_epoch, evaluate = _load_train_functions()

_CLIP_NORMS = []
_orig_clip = torch.nn.utils.clip_grad_norm_


def _recording_clip(*a, **k):
    """Records the pre-clip total norm clip_grad_norm_ returns (train.py:96-97 discards it)."""
    n = _orig_clip(*a, **k)
    _CLIP_NORMS.append(float(n))
    return n


torch.nn.utils.clip_grad_norm_ = _recording_clip


class _PatchesMemory(ref_model.ImageToTextModel):
    """north-star memory mode: decoder cross-attends to projection(last_hidden_state)."""

    def forward(self, image_tensors, tgt_tokens):
        with torch.no_grad():
            feats = self.encoder(pixel_values=image_tensors).last_hidden_state
        memory = self.projection(feats)
        return self.decoder(tgt_tokens=tgt_tokens, memory=memory, memory_padding_mask=None)


def build_reference(enc_kind: str, enc_cfg: dict, dec: dict, mode: str, seed: int):
    cls = ref_model.ImageToTextModel if mode == "cls" else _PatchesMemory
    m = cls.__new__(cls)
    nn.Module.__init__(m)
    if enc_kind == "vit":
        m.encoder = ViTModel(ViTConfig(**enc_cfg))
    else:
        m.encoder = CLIPVisionModel(CLIPVisionConfig(**enc_cfg))
    for p in m.encoder.parameters():
        p.requires_grad = False
    m.encoder.eval()
    m.encoder_output_dim = m.encoder.config.hidden_size
    m.image_processor = ViTImageProcessor()
    m.decoder_embed_dim = dec["embed_dim"]
    m.decoder_pad_idx = 0
    m.projection = (nn.Linear(m.encoder_output_dim, dec["embed_dim"])
                    if m.encoder_output_dim != dec["embed_dim"] else nn.Identity())
    m.decoder = ref_decoder.TransformerDecoder(
        vocab_size=dec["vocab"], embed_dim=dec["embed_dim"], num_heads=dec["heads"],
        num_layers=dec["layers"], ff_dim=dec["ff"], max_seq_len=dec.get("max_seq_len", 100),
        dropout=0.0, pad_idx=0)
    spec = [(n, tuple(p.shape)) for n, p in m.named_parameters()]
    state = P.make_state(spec, seed)
    with torch.no_grad():
        for n, p in m.named_parameters():
            p.copy_(state[n])
    return m, spec, state


def _stat_entries(prefix: str, name: str, t: torch.Tensor, out: dict, meta_idx: dict, seed: int):
    t = t.detach().float()
    if t.numel() <= 4096:
        out[f"{prefix}.full.{name}"] = t.contiguous().clone()
        return
    idx = P.sample_index(t.numel(), 64, seed)
    meta_idx[name] = idx.tolist()
    flat = t.flatten()
    out[f"{prefix}.sample.{name}"] = flat[idx].clone()
    out[f"{prefix}.stats.{name}"] = torch.tensor([flat.double().sum().item(), flat.double().norm().item(),
                                                   flat.double().abs().max().item()], dtype=torch.float32)


def trainable(m):
    return [(n, p) for n, p in m.named_parameters() if p.requires_grad]


def run_case(name, enc_kind, enc_cfg, dec, mode, *, B, cap_len, lengths, seed, image_size,
             steps=3, clip_first=5.0, clip_rest=0.1, full_logits=True, gen=False):
    torch.manual_seed(0)
    m, spec, state = build_reference(enc_kind, enc_cfg, dec, mode, seed)
    images = P.make_images(B, image_size, seed + 1)
    caps = [P.make_captions(B, cap_len, dec["vocab"], seed + 2 + s, lengths) for s in range(steps)]
    batches = [{"images": images, "decoder_input_tokens": c[:, :-1], "target_tokens": c[:, 1:]} for c in caps]
    out, meta_idx = {}, {}

    # 1. encoder output + forward logits (reference ImageToTextModel.forward, model.py:116-169)
    m.eval()
    with torch.no_grad():
        lhs = m.encoder(pixel_values=images).last_hidden_state
        logits = m(images, batches[0]["decoder_input_tokens"])
    if lhs.numel() <= 600_000:
        out["enc.last_hidden_state"] = lhs.contiguous()
    else:
        out["enc.cls_rows"] = lhs[:, 0, :].contiguous()
        out["enc.row17"] = lhs[:, 17, :].contiguous()
        out["enc.row_last"] = lhs[:, -1, :].contiguous()
    logit_sel = None
    if full_logits:
        out["fwd.logits"] = logits.contiguous()
    else:
        out["fwd.logits_pos0"] = logits[:, 0, :].contiguous()
        out["fwd.logits_poslast"] = logits[:, -1, :].contiguous()
        # row-sampled logits: 8 positions per caption (first, last, 6 seeded) pin the whole sequence
        Tt = logits.shape[1]
        logit_sel = []
        for b in range(B):
            extra = P.sample_index(Tt - 2, 6, seed + 300 + b) + 1
            logit_sel += [[b, t] for t in sorted({0, Tt - 1, *extra.tolist()})]
        out["fwd.logits_sel"] = torch.stack([logits[b, t] for b, t in logit_sel]).contiguous()
    out["fwd.argmax"] = logits.argmax(-1).to(torch.float32)
    top2 = logits.topk(2, dim=-1).values
    out["fwd.margin"] = (top2[..., 0] - top2[..., 1]).contiguous()
    crit = nn.CrossEntropyLoss(ignore_index=0)
    loss0 = crit(logits.reshape(-1, logits.size(-1)), batches[0]["target_tokens"].reshape(-1))
    out["fwd.loss"] = loss0.reshape(1).float()

    # 2. one reference training step (train.py:62-123), grads + params after it
    opt = torch.optim.AdamW(m.parameters(), lr=ref_config.LEARNING_RATE,
                            betas=(ref_config.ADAM_BETA1, ref_config.ADAM_BETA2),
                            eps=ref_config.ADAM_EPS, weight_decay=ref_config.WEIGHT_DECAY)
    p_before = {n: p.detach().clone() for n, p in trainable(m)}
    # the grad norm clip_grad_norm_ sees (train.py:96-97) — recomputed from the grads after the step
    _CLIP_NORMS.clear()
    avg1 = train_one_epoch(m, [batches[0]], opt, crit, "cpu", clip_first, None, 0, 50, None)
    out["step1.loss"] = torch.tensor([avg1], dtype=torch.float32)
    # grads left on the params are POST-clip (clip_grad_norm_ scales them in place)
    gnorm = torch.tensor(_CLIP_NORMS[0], dtype=torch.float64)
    out["step1.grad_total_norm_preclip"] = gnorm.reshape(1).float()
    for i, (n, p) in enumerate(trainable(m)):
        g = p.grad if p.grad is not None else torch.zeros_like(p)
        _stat_entries("grad1", n, g, out, meta_idx, 1000 + i)
        _stat_entries("delta1", n, p.detach() - p_before[n], out, {}, 1000 + i)
    # 3. two more steps with a small clip so clip_grad_norm_ actually scales (train.py:96-97)
    losses = []
    if steps > 1:
        _CLIP_NORMS.clear()
        avg = train_one_epoch(m, batches[1:], opt, crit, "cpu", clip_rest, None, 1, 50, None)
        losses.append(avg)
        out["step23.grad_total_norm_preclip"] = torch.tensor(_CLIP_NORMS, dtype=torch.float32)
        for i, (n, p) in enumerate(trainable(m)):
            _stat_entries("delta3", n, p.detach() - p_before[n], out, {}, 1000 + i)
        out["step3.avg_loss_23"] = torch.tensor([avg], dtype=torch.float32)
    # 4. evaluate() (train.py:125-151) on batch 0 after the steps
    out["eval.loss"] = torch.tensor([evaluate(m, [batches[0]], crit, "cpu")], dtype=torch.float32)

    gen_meta = None
    if gen:
        ids_all = []
        for k in range(2):
            img = P.pil_like_image(40 + 8 * k, 56 - 8 * k, seed + 50 + k)
            pil = Image.fromarray(img.numpy())
            pv = m.image_processor(images=pil, return_tensors="pt")["pixel_values"]
            out[f"gen.pixel_values{k}"] = pv.float().contiguous()
            ids = ref_model.ImageToTextModel.generate(m, pil, start_token_id=ref_config.START_TOKEN_ID,
                                                      end_token_id=ref_config.END_TOKEN_ID, max_len=12)
            ids_all.append(ids)
        gen_meta = {"ids": ids_all, "max_len": 12, "start": ref_config.START_TOKEN_ID,
                    "end": ref_config.END_TOKEN_ID, "image_shapes": [[40, 56], [48, 48]]}

    meta = {
        "case": name, "enc_kind": enc_kind, "enc_cfg": enc_cfg, "dec": dec, "mode": mode,
        "B": B, "cap_len": cap_len, "lengths": lengths, "seed": seed, "image_size": image_size,
        "grads_are": "post-clip (as left on .grad by train_one_epoch)",
        "steps": steps, "clip_first": clip_first, "clip_rest": clip_rest,
        "lr": ref_config.LEARNING_RATE, "betas": [ref_config.ADAM_BETA1, ref_config.ADAM_BETA2],
        "eps": ref_config.ADAM_EPS, "weight_decay": ref_config.WEIGHT_DECAY,
        "spec": [[n, list(s)] for n, s in spec],
        "weights_checksum": P.checksum(state[n] for n, _ in spec),
        "images_checksum": P.checksum([images]),
        "captions_checksum": P.checksum(caps),
        "sample_index": meta_idx, "generate": gen_meta, "logit_sel": logit_sel,
        "versions": {"torch": torch.__version__, "transformers": __import__("transformers").__version__},
    }
    path = os.path.join(HERE, f"{name}.safetensors")
    save_file({k: v.contiguous() for k, v in out.items()}, path, metadata={"meta": json.dumps(meta)})
    print(f"{name}: {os.path.getsize(path)/1e6:.2f} MB, loss0={loss0.item():.5f} "
          f"gnorm={gnorm.item():.4f}", flush=True)


def run_dp_case(name, enc_kind, enc_cfg, dec, *, B, cap_len, lengths, seed, image_size):
    """Single-process reference step at global batch B; halves have unequal PAD."""
    torch.manual_seed(0)
    m, spec, state = build_reference(enc_kind, enc_cfg, dec, "patches", seed)
    images = P.make_images(B, image_size, seed + 1)
    cap = P.make_captions(B, cap_len, dec["vocab"], seed + 2, lengths)
    batch = {"images": images, "decoder_input_tokens": cap[:, :-1], "target_tokens": cap[:, 1:]}
    crit = nn.CrossEntropyLoss(ignore_index=0)
    opt = torch.optim.AdamW(m.parameters(), lr=ref_config.LEARNING_RATE,
                            betas=(ref_config.ADAM_BETA1, ref_config.ADAM_BETA2),
                            eps=ref_config.ADAM_EPS, weight_decay=ref_config.WEIGHT_DECAY)
    p_before = {n: p.detach().clone() for n, p in trainable(m)}
    _CLIP_NORMS.clear()
    avg = train_one_epoch(m, [batch], opt, crit, "cpu", 5.0, None, 0, 50, None)
    out, meta_idx = {"loss": torch.tensor([avg], dtype=torch.float32),
                     "grad_total_norm_preclip": torch.tensor(_CLIP_NORMS, dtype=torch.float32)}, {}
    for i, (n, p) in enumerate(trainable(m)):
        _stat_entries("grad1", n, p.grad, out, meta_idx, 2000 + i)
        _stat_entries("delta1", n, p.detach() - p_before[n], out, {}, 2000 + i)
    meta = {"case": name, "enc_kind": enc_kind, "enc_cfg": enc_cfg, "dec": dec, "mode": "patches",
            "B": B, "cap_len": cap_len, "lengths": lengths, "seed": seed, "image_size": image_size,
            "spec": [[n, list(s)] for n, s in spec], "sample_index": meta_idx,
            "weights_checksum": P.checksum(state[n] for n, _ in spec),
            "lr": ref_config.LEARNING_RATE, "betas": [ref_config.ADAM_BETA1, ref_config.ADAM_BETA2],
            "eps": ref_config.ADAM_EPS, "weight_decay": ref_config.WEIGHT_DECAY, "clip": 5.0}
    path = os.path.join(HERE, f"{name}.safetensors")
    save_file({k: v.contiguous() for k, v in out.items()}, path, metadata={"meta": json.dumps(meta)})
    print(f"{name}: {os.path.getsize(path)/1e6:.2f} MB loss={avg:.5f}", flush=True)


class _TensorProcessor:
    """Stands in for the HF image processor when generate() is handed an already-normalised tensor
    (the reference's generate calls self.image_processor(images=..., return_tensors="pt"), model.py:192)."""

    class _Out(dict):
        def to(self, device):
            return self

    def __call__(self, images, return_tensors="pt"):
        return self._Out(pixel_values=images)


def run_gen_case(name, enc_kind, enc_cfg, dec, *, n_images, seed, image_size, max_len, start, end):
    """Reference greedy generate (model.py:171-242, cls memory as the reference computes it) on
    procedural images with the initial procedural weights (configs[4]: batched decode parity)."""
    torch.manual_seed(0)
    m, spec, state = build_reference(enc_kind, enc_cfg, dec, "cls", seed)
    m.image_processor = _TensorProcessor()
    images = P.make_images(n_images, image_size, seed + 7)
    ids = [ref_model.ImageToTextModel.generate(m, images[i:i + 1], start_token_id=start, end_token_id=end,
                                               max_len=max_len) for i in range(n_images)]
    # the full teacher-forced logits of each generated sequence: argmax margins for near-tie handling
    margins = []
    with torch.no_grad():
        for i, row in enumerate(ids):
            lg = m(images[i:i + 1], torch.tensor([row[:-1]]))[0]
            top2 = lg.topk(2, dim=-1).values
            margins.append((top2[:, 0] - top2[:, 1]).tolist())
    meta = {"case": name, "enc_kind": enc_kind, "enc_cfg": enc_cfg, "dec": dec, "mode": "cls", "seed": seed,
            "image_size": image_size, "n_images": n_images, "image_seed": seed + 7, "max_len": max_len,
            "start": start, "end": end, "ids": ids, "margins": margins,
            "spec": [[n, list(s)] for n, s in spec], "weights_checksum": P.checksum(state[n] for n, _ in spec),
            "images_checksum": P.checksum([images]),
            "versions": {"torch": torch.__version__, "transformers": __import__("transformers").__version__}}
    path = os.path.join(HERE, f"{name}.safetensors")
    save_file({"ids_flat": torch.tensor([t for r in ids for t in r], dtype=torch.float32)}, path,
              metadata={"meta": json.dumps(meta)})
    print(f"{name}: {[len(r) for r in ids]} ids, min margin {min(min(x) for x in margins):.4f}", flush=True)


def run_memory_mask_case(name, dec, *, B, T, S, mem_lengths, seed):
    """The reference decoder alone (decoder.TransformerDecoder.forward, decoder.py:134-193) with a
    memory_padding_mask (True = padded memory position), which model.forward never passes."""
    torch.manual_seed(0)
    m = ref_decoder.TransformerDecoder(vocab_size=dec["vocab"], embed_dim=dec["embed_dim"], num_heads=dec["heads"],
                                       num_layers=dec["layers"], ff_dim=dec["ff"], max_seq_len=100, dropout=0.0,
                                       pad_idx=0)
    spec = [("decoder." + n, tuple(p.shape)) for n, p in m.named_parameters()]
    state = P.make_state(spec, seed)
    with torch.no_grad():
        for n, p in m.named_parameters():
            p.copy_(state["decoder." + n])
    m.eval()
    g = torch.Generator().manual_seed(seed + 1)
    memory = torch.randn(B, S, dec["embed_dim"], generator=g)
    mask = torch.zeros(B, S, dtype=torch.bool)
    for i, n in enumerate(mem_lengths):
        mask[i, n:] = True
    tokens = P.make_captions(B, T, dec["vocab"], seed + 2, [T, T - 5, 3][:B])
    with torch.no_grad():
        logits = m(tokens, memory, memory_padding_mask=mask)
    meta = {"case": name, "dec": dec, "B": B, "T": T, "S": S, "mem_lengths": mem_lengths, "seed": seed,
            "spec": [[n, list(s)] for n, s in spec], "weights_checksum": P.checksum(state[n] for n, _ in spec)}
    path = os.path.join(HERE, f"{name}.safetensors")
    save_file({"logits": logits.contiguous(), "memory": memory.contiguous(), "tokens": tokens.float()}, path,
              metadata={"meta": json.dumps(meta)})
    print(f"{name}: {os.path.getsize(path) / 1e6:.2f} MB", flush=True)


TINY_VIT = dict(hidden_size=128, num_hidden_layers=2, num_attention_heads=2, intermediate_size=512,
                image_size=224, patch_size=16)
TINY_CLIP = dict(hidden_size=128, num_hidden_layers=2, num_attention_heads=2, intermediate_size=512,
                 image_size=336, patch_size=14)
TINY_DEC = dict(vocab=512, embed_dim=128, heads=2, layers=2, ff=512)
# decoder width differs from the encoder width so the projection is a real Linear (model.py:97-99)
TINY_DEC96 = dict(vocab=512, embed_dim=192, heads=3, layers=2, ff=384)
CFG1_DEC = dict(vocab=10000, embed_dim=512, heads=8, layers=6, ff=2048)
# configs[0]: 2L d128 decoder with 8 heads (head_dim 16), ff = 4d
CFG0_DEC = dict(vocab=10000, embed_dim=128, heads=8, layers=2, ff=512)
# configs[2]: CLIP ViT-L/14@336 (577 tokens) + the cfg1 decoder
CLIP_L14_336 = dict(hidden_size=1024, intermediate_size=4096, num_hidden_layers=24, num_attention_heads=16,
                    image_size=336, patch_size=14)
# a vocabulary that is not a multiple of 8 (the tokenizer decides V, tokenizer.py:200-201)
TINY_DEC509 = dict(vocab=509, embed_dim=192, heads=3, layers=2, ff=384)
# configs[3]: CLIP ViT-L/14 (224 px -> 257 tokens) + 12L d768 decoder (H = 12, ff = 4d)
CLIP_L14 = dict(hidden_size=1024, intermediate_size=4096, num_hidden_layers=24, num_attention_heads=16,
                image_size=224, patch_size=14)
CFG3_DEC = dict(vocab=10000, embed_dim=768, heads=12, layers=12, ff=3072)

if __name__ == "__main__":
    only = set(sys.argv[1:])

    def want(n):
        return not only or n in only

    L31 = [32, 27, 20, 9]
    if want("tiny_vit_cls"):
        run_case("tiny_vit_cls", "vit", TINY_VIT, TINY_DEC96, "cls", B=4, cap_len=32, lengths=L31,
                 seed=11, image_size=224, gen=True)
    if want("tiny_vit_patches"):
        run_case("tiny_vit_patches", "vit", TINY_VIT, TINY_DEC96, "patches", B=4, cap_len=32,
                 lengths=L31, seed=12, image_size=224)
    if want("tiny_clip336_patches"):
        run_case("tiny_clip336_patches", "clip", TINY_CLIP, TINY_DEC96, "patches", B=2, cap_len=24,
                 lengths=[24, 13], seed=13, image_size=336)
    if want("tiny_clip336_cls"):
        run_case("tiny_clip336_cls", "clip", TINY_CLIP, TINY_DEC, "cls", B=2, cap_len=24,
                 lengths=[24, 13], seed=14, image_size=336, steps=1)
    if want("cfg1_b2_patches"):
        # full cfg1 architecture (ViT-B/16 = ViTConfig() defaults + 6L d512 V=10000), batch 2
        run_case("cfg1_b2_patches", "vit", {}, CFG1_DEC, "patches", B=2, cap_len=64, lengths=[64, 41],
                 seed=21, image_size=224, steps=1, full_logits=False)
    if want("cfg3_b2_patches"):
        run_case("cfg3_b2_patches", "clip", CLIP_L14, CFG3_DEC, "patches", B=2, cap_len=64, lengths=[64, 37],
                 seed=41, image_size=224, steps=1, full_logits=False)
    if want("cfg0_b4_cls"):
        run_case("cfg0_b4_cls", "vit", {}, CFG0_DEC, "cls", B=4, cap_len=32, lengths=[32, 29, 20, 11],
                 seed=51, image_size=224, full_logits=False)
    if want("cfg0_b4_patches"):
        run_case("cfg0_b4_patches", "vit", {}, CFG0_DEC, "patches", B=4, cap_len=32, lengths=[32, 30, 17, 6],
                 seed=52, image_size=224, full_logits=False)
    if want("cfg2_b2_patches"):
        run_case("cfg2_b2_patches", "clip", CLIP_L14_336, CFG1_DEC, "patches", B=2, cap_len=64, lengths=[64, 45],
                 seed=61, image_size=336, steps=1, full_logits=False)
    if want("tiny_vit_v509"):
        run_case("tiny_vit_v509", "vit", TINY_VIT, TINY_DEC509, "patches", B=4, cap_len=24, lengths=[24, 19, 12, 5],
                 seed=71, image_size=224)
    if want("cfg1_gen_cls"):
        # configs[4] parity anchor: the cfg1 architecture with the cfg1_b2_patches weights (seed 21)
        run_gen_case("cfg1_gen_cls", "vit", {}, CFG1_DEC, n_images=4, seed=21, image_size=224, max_len=16,
                     start=ref_config.START_TOKEN_ID, end=ref_config.END_TOKEN_ID)
    if want("dec_memory_mask"):
        run_memory_mask_case("dec_memory_mask", TINY_DEC96, B=3, T=17, S=37, mem_lengths=[37, 20, 5], seed=81)
    if want("dp2_tiny"):
        run_dp_case("dp2_tiny", "vit", TINY_VIT, TINY_DEC96, B=8, cap_len=20,
                    lengths=[20, 20, 18, 20, 7, 9, 11, 5], seed=31, image_size=224)
