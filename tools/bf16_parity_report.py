"""bf16 parity of the MI355X path against the reference's golden outputs, per fixture (DESIGN §6
table): encoder rows, logits (max-abs, relative L2, scale), argmax agreement, loss, one train step
(loss, pre-clip grad norm, per-tensor relative errors of the post-clip gradients and the AdamW
update). Writes gpurun_out/bf16_parity.json. Run on the GPU box: python tools/bf16_parity_report.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "multimodal-image-transformer_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import fixtures as FX  # noqa: E402
from model_util import build_model  # noqa: E402


def rel(a, b):
    return float((a - b).norm() / max(b.norm(), 1e-30))


def tensor_err(prefix, name, t, T, meta):
    """(error RMS / the reference tensor's RMS) on the entries a fixture stores for one tensor (full, or
    64 sampled elements + the tensor's [sum, norm, maxabs]), and the relative error of its L2 norm.
    RMS-normalised: a sampled element near 0 does not blow the ratio up (most embedding rows have
    exactly-zero gradients)."""
    t = t.detach().float().cpu().flatten()
    n = t.numel()
    if f"{prefix}.full.{name}" in T:
        ref = T[f"{prefix}.full.{name}"].flatten()
        rn = float(ref.norm())
        return float((t - ref).norm()) / max(rn, 1e-30), abs(float(t.norm()) - rn) / max(rn, 1e-30)
    idx = torch.tensor(meta["sample_index"][name])
    ref = T[f"{prefix}.sample.{name}"]
    rn = float(T[f"{prefix}.stats.{name}"][1])
    rms_err = float((t[idx] - ref).norm()) / len(idx) ** 0.5
    return rms_err / max(rn / n ** 0.5, 1e-30), abs(float(t.norm()) - rn) / max(rn, 1e-30)


def main():
    import optim
    from decoder import flat_to_reference
    out = {}
    cases = sys.argv[1:] or FX.CASES
    for name in cases:
        meta, T = FX.load(name)
        r = {}
        for dtype in (torch.bfloat16, torch.float32):
            tag = "bf16" if dtype == torch.bfloat16 else "fp32"
            m, _ = build_model(meta, dtype)
            imgs, di, tg = FX.inputs(meta, 0)
            m.eval()
            with torch.no_grad():
                feats = m.encoder.forward(imgs.cuda(), rows="all").float().cpu()
                logits = m(imgs.cuda(), di.cuda()).float().cpu()
            enc = [(rel(a, b), float((a - b).abs().max()), float(b.abs().max())) for a, b in FX.encoder_rows(T, feats)]
            got, ref = FX.logits_at(meta, T, logits)
            safe = T["fwd.margin"] > 5e-2
            loss = torch.nn.functional.cross_entropy(logits.reshape(-1, logits.shape[-1]), tg.reshape(-1),
                                                     ignore_index=0).item()
            r[tag] = {"enc_rel_l2": max(e[0] for e in enc), "enc_max_abs": max(e[1] for e in enc),
                      "enc_scale": max(e[2] for e in enc),
                      "logits_max_abs": float((got - ref).abs().max()), "logits_rel_l2": rel(got, ref),
                      "logits_scale": float(ref.abs().max()),
                      "logits_max_abs_over_scale": float((got - ref).abs().max() / ref.abs().max()),
                      "argmax_agree_margin_gt_5e-2": float((logits.argmax(-1).float()[safe] ==
                                                            T["fwd.argmax"][safe]).float().mean()),
                      "loss_abs_err": abs(loss - T["fwd.loss"].item())}
            m.train()
            opt = optim.AdamW(m.store, lr=meta["lr"], betas=tuple(meta["betas"]), eps=meta["eps"],
                              weight_decay=meta["weight_decay"])
            names = FX.trainable_names(meta)
            before = {k: v.clone() for k, v in m.state_dict().items() if k in names}
            l1 = m.train_step(imgs.cuda(), di.cuda(), tg.cuda()).item()
            opt.step(meta["clip_first"])
            total, coef = opt.norm_t.tolist()

            class GV:
                vocab = m.decoder.V

                def p(self, n):
                    return m.store.g(n)

            grads = flat_to_reference(GV(), m.decoder.L, m.decoder_embed_dim)
            if m.has_projection:
                grads["projection.weight"] = m.store.g("projection.weight")
                grads["projection.bias"] = m.store.g("projection.bias")
            after = m.state_dict()
            ge = {k: tensor_err("grad1", k, grads[k] * coef, T, meta) for k in names}
            gerr = {k: v[0] for k, v in ge.items()}
            gnorm = {k: v[1] for k, v in ge.items()}
            derr = {k: tensor_err("delta1", k, after[k] - before[k], T, meta)[0] for k in names
                    if not k.endswith("in_proj_bias")}
            r[tag].update({"step1_loss_abs_err": abs(l1 - T["step1.loss"].item()),
                           "grad_norm_rel_err": abs(total - T["step1.grad_total_norm_preclip"].item()) / total,
                           "grad_rel_l2_max": max(gerr.values()), "grad_rel_l2_worst": max(gerr, key=gerr.get),
                           "grad_rel_l2_median": sorted(gerr.values())[len(gerr) // 2],
                           "grad_norm_rel_err_max": max(gnorm.values()), "grad_norm_worst": max(gnorm, key=gnorm.get),
                           "delta1_rel_l2_max": max(derr.values()), "delta1_rel_l2_worst": max(derr, key=derr.get),
                           "delta1_rel_l2_median": sorted(derr.values())[len(derr) // 2]})
            del m
            torch.cuda.empty_cache()
        out[name] = r
        print(name, json.dumps(r), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "bf16_parity.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
