"""How close does the REFERENCE itself get to its fp32 outputs when run in bf16? Calibration for the
bf16 parity bounds of the MI355X path. TEST INFRASTRUCTURE ONLY — run here (where
/root/reference exists), never on the GPU box:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_bf16_calibration.py

For each golden fixture: the reference model (make_fixtures.build_reference, same procedural
weights and inputs) is run under torch.autocast("cpu", dtype=torch.bfloat16) — bf16 matmuls with
fp32 accumulation, fp32 LayerNorm / softmax / residual stream, torch's standard mixed precision — for
the forward logits and one train step (train.py:80-100), and compared with the fp32 fixture using the
same metrics tools/bf16_parity_report.py computes for the HIP path. Output:
tests/golden/bf16_reference_calibration.json (numbers only)."""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
import make_fixtures as MF  # noqa: E402  (imports the reference from /root/reference)
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

import fixtures as FX  # noqa: E402


def rms_err(prefix, name, t, T, meta):
    t = t.detach().float().flatten()
    n = t.numel()
    if f"{prefix}.full.{name}" in T:
        ref = T[f"{prefix}.full.{name}"].flatten()
        return float((t - ref).norm() / max(ref.norm(), 1e-30))
    idx = torch.tensor(meta["sample_index"][name])
    rn = float(T[f"{prefix}.stats.{name}"][1])
    return float((t[idx] - T[f"{prefix}.sample.{name}"]).norm() / len(idx) ** 0.5) / max(rn / n ** 0.5, 1e-30)


def main():
    out = {}
    for name in (sys.argv[1:] or FX.CASES):
        meta, T = FX.load(name)
        torch.manual_seed(0)
        m, spec, state = MF.build_reference(meta["enc_kind"], meta["enc_cfg"], meta["dec"], meta["mode"], meta["seed"])
        imgs, di, tg = FX.inputs(meta, 0)
        m.eval()
        with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
            feats = m.encoder(pixel_values=imgs).last_hidden_state.float()
            logits = m(imgs, di).float()
        enc = max(float((a - b).norm() / b.norm()) for a, b in FX.encoder_rows(T, feats))
        got, ref = FX.logits_at(meta, T, logits)
        r = {"enc_rel_l2": enc, "logits_max_abs": float((got - ref).abs().max()),
             "logits_rel_l2": float((got - ref).norm() / ref.norm()), "logits_scale": float(ref.abs().max())}
        m.train()
        crit = nn.CrossEntropyLoss(ignore_index=0)
        with torch.autocast("cpu", dtype=torch.bfloat16):
            lg = m(imgs, di)
            loss = crit(lg.float().reshape(-1, lg.shape[-1]), tg.reshape(-1))
        loss.backward()
        names = FX.trainable_names(meta)
        params = dict(m.named_parameters())
        grads = [params[k].grad for k in names]
        total = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g) for g in grads])).item()
        coef = min(1.0, meta["clip_first"] / (total + 1e-6))
        ge = {k: rms_err("grad1", k, params[k].grad * coef, T, meta) for k in names}
        dense = FX.load_dense(name)
        if dense is not None:  # the same metric over the denser pins (make_grad_dense.py, 1024 per tensor)
            from parity_metrics import dense_metrics
            r.update(dense_metrics(names, {k: params[k].grad * coef for k in names}, T, dense))
        r.update({"step1_loss_abs_err": abs(loss.item() - T["step1.loss"].item()),
                  "grad_norm_rel_err": abs(total - T["step1.grad_total_norm_preclip"].item()) / total,
                  "grad_rms_median": sorted(ge.values())[len(ge) // 2], "grad_rms_max": max(ge.values()),
                  "grad_rms_worst": max(ge, key=ge.get)})
        out[name] = r
        print(name, json.dumps(r), flush=True)
    path = os.path.join(HERE, "bf16_reference_calibration.json")
    old = json.load(open(path)) if os.path.exists(path) else {}
    old.update(out)
    with open(path, "w") as f:
        json.dump(old, f, indent=1)


if __name__ == "__main__":
    main()
