"""Where does the bf16 path's logits error come from? Per golden fixture, the logits rel-L2 against the
reference's fp32 logits with one stage at a time computed differently (VERDICT r04 "next" #1):
  bf16      the benchmarked path as shipped
  enc_f32   bf16 decoder fed the fp32 encoder's features (rounded once to bf16): the decoder's share
  dec_f32   fp32 decoder fed the bf16 encoder's features: the encoder's share
  res32     bf16 with the encoder's f32 residual stream (config.ENCODER_F32_RESIDUAL = on)
  nofold    bf16 with the encoder LayerNorms as explicit launches (config.ENCODER_FOLD_LN = off)
plus the encoder's own rel-L2 for the bf16 / res32 / nofold towers, next to the reference's bf16
(torch.autocast) error from tests/golden/bf16_reference_calibration.json.
Run on the GPU box: python tools/bf16_bisect.py [case ...]  -> gpurun_out/bf16_bisect.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "multimodal-image-transformer_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import config  # noqa: E402
import fixtures as FX  # noqa: E402
from model_util import build_model  # noqa: E402
from parity_metrics import rel  # noqa: E402


def _build(meta, dtype, res32="auto", fold="auto"):
    config.ENCODER_F32_RESIDUAL, config.ENCODER_FOLD_LN = res32, fold
    try:
        m, _ = build_model(meta, dtype)
    finally:
        config.ENCODER_F32_RESIDUAL, config.ENCODER_FOLD_LN = "auto", "auto"
    m.eval()
    return m


def _feats(m, imgs):
    with torch.no_grad():
        return m.encoder.forward(imgs.cuda(), rows="all").clone()


def _inject(m, feats):
    """m's encoder replaced by fixed features [B, N, E] (cast to m's compute dtype)."""
    B, N, E = feats.shape
    f = feats.to(m.dtype)

    def rows(images, slot=0):
        if m.memory_mode == "cls":
            return f[:, 0].contiguous(), E, 1
        return f.reshape(B * N, E).contiguous(), E, N
    m._encoder_rows = rows


def _logits_rel(meta, T, m, imgs, di):
    with torch.no_grad():
        logits = m(imgs.cuda(), di.cuda()).float().cpu()
    got, ref = FX.logits_at(meta, T, logits)
    return rel(got, ref)


def _enc_rel(T, feats):
    return max(rel(a, b) for a, b in FX.encoder_rows(T, feats.float().cpu()))


def case(name):
    meta, T = FX.load(name)
    cal = json.load(open(os.path.join(FX.GOLDEN, "bf16_reference_calibration.json")))[name]
    imgs, di, _ = FX.inputs(meta, 0)
    out = {"ref_bf16_logits": cal["logits_rel_l2"], "ref_bf16_enc": cal["enc_rel_l2"]}
    m32 = _build(meta, torch.float32)
    f32 = _feats(m32, imgs)
    m16 = _build(meta, torch.bfloat16)
    f16 = _feats(m16, imgs)
    out["bf16"] = _logits_rel(meta, T, m16, imgs, di)
    out["enc_bf16"] = _enc_rel(T, f16)
    out["fold"] = bool(m16.encoder.fold_ln)
    out["res32_default"] = bool(m16.encoder.res32)
    _inject(m16, f32)
    out["enc_f32"] = _logits_rel(meta, T, m16, imgs, di)
    _inject(m32, f16)
    out["dec_f32"] = _logits_rel(meta, T, m32, imgs, di)
    out["fp32"] = None
    del m16, m32
    for key, kw in (("res32", dict(res32="on")), ("nofold", dict(fold="off"))):
        m = _build(meta, torch.bfloat16, **kw)
        out[key] = _logits_rel(meta, T, m, imgs, di)
        out["enc_" + key] = _enc_rel(T, _feats(m, imgs))
        del m
    torch.cuda.empty_cache()
    out["ratio_bf16"] = out["bf16"] / cal["logits_rel_l2"]
    return out


def main():
    res = {}
    for name in sys.argv[1:] or FX.CASES:
        res[name] = case(name)
        r = res[name]
        print(f"{name:22s} logits rel-L2: bf16 {r['bf16']:.3e} ({r['ratio_bf16']:.2f}x ref {r['ref_bf16_logits']:.3e}) "
              f"enc_f32 {r['enc_f32']:.3e} dec_f32 {r['dec_f32']:.3e} res32 {r['res32']:.3e} nofold {r['nofold']:.3e} | "
              f"encoder: bf16 {r['enc_bf16']:.3e} res32 {r['enc_res32']:.3e} nofold {r['enc_nofold']:.3e} "
              f"ref {r['ref_bf16_enc']:.3e}", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "bf16_bisect.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
