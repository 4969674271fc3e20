"""Parity metrics of the MI355X path against the golden fixtures, per fixture and dtype (used by
tests/test_bf16_parity_gpu.py and tools/bf16_parity_report.py). Test infrastructure."""
import torch

import fixtures as FX
from model_util import build_model


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


def dense_err(name, t, T, dense, trim=0.0):
    """tensor_err's RMS ratio over the denser pins (FX.load_dense: 1024 elements) instead of the 64; for
    tensors stored whole it is tensor_err's. trim > 0: the largest ceil(trim * pins) squared errors are left out
    first (a trimmed RMS: the per-element errors are heavy-tailed -- a bf16 ReLU-boundary flip moves a whole
    row of a linear1 weight gradient -- so the plain RMS of a sample is carried by a handful of elements,
    tools/grad_metric_report.py). Returns (ratio, per-element squared-error shares sorted descending)."""
    t = t.detach().float().cpu().flatten()
    if f"grad1.full.{name}" in T:
        ref = T[f"grad1.full.{name}"].flatten()
        rms_t = float(ref.norm()) / t.numel() ** 0.5
        e2 = (t - ref) ** 2
    else:
        idx, ref = dense[name]
        rms_t = float(T[f"grad1.stats.{name}"][1]) / t.numel() ** 0.5
        e2 = (t[idx] - ref) ** 2
    srt = e2.sort(descending=True)[0]
    share = srt / srt.sum().clamp_min(1e-30)
    if trim > 0:
        srt = srt[int(-(-trim * srt.numel() // 1)):]
    return float(srt.mean().sqrt()) / max(rms_t, 1e-30), share


def dense_metrics(names, grads, T, dense):
    """Worst / median over the tensors of dense_err: plain ("_dense") and 1 %-trimmed ("_trim")."""
    r = {}
    for tag, trim in (("dense", 0.0), ("trim", 0.01)):
        de = {k: dense_err(k, grads[k], T, dense, trim)[0] for k in names}
        r.update({f"grad_rms_max_{tag}": max(de.values()), f"grad_rms_worst_{tag}": max(de, key=de.get),
                  f"grad_rms_median_{tag}": sorted(de.values())[len(de) // 2]})
    return r


def step1(m, meta, imgs, di, tg):
    """The fixture's first train step (train.py:80-100: forward, CE, backward, clip_first, AdamW) on the HIP
    path. Returns (loss, pre-clip total norm, clip coefficient, {reference tensor name: gradient})."""
    import optim
    from decoder import flat_to_reference
    m.train()
    opt = optim.AdamW(m.store, lr=meta["lr"], betas=tuple(meta["betas"]), eps=meta["eps"],
                      weight_decay=meta["weight_decay"])
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
    return l1, total, coef, grads


def case_metrics(name, dtype):
    """encoder rows, logits, argmax, loss, and one train step (train.py:80-100) of the HIP path at
    `dtype` against the reference's fp32 outputs."""
    meta, T = FX.load(name)
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
    r = {"enc_rel_l2": max(e[0] for e in enc), "enc_max_abs": max(e[1] for e in enc),
         "enc_scale": max(e[2] for e in enc),
         "logits_max_abs": float((got - ref).abs().max()), "logits_rel_l2": rel(got, ref),
         "logits_scale": float(ref.abs().max()),
         "logits_max_abs_over_scale": float((got - ref).abs().max() / ref.abs().max()),
         "argmax_agree_margin_gt_5e-2": float((logits.argmax(-1).float()[safe] == T["fwd.argmax"][safe]).float().mean()),
         "loss_abs_err": abs(loss - T["fwd.loss"].item())}
    names = FX.trainable_names(meta)
    before = {k: v.clone() for k, v in m.state_dict().items() if k in names}
    l1, total, coef, grads = step1(m, meta, imgs, di, tg)
    after = m.state_dict()
    ge = {k: tensor_err("grad1", k, grads[k] * coef, T, meta) for k in names}
    gerr = {k: v[0] for k, v in ge.items()}
    gnorm = {k: v[1] for k, v in ge.items()}
    derr = {k: tensor_err("delta1", k, after[k] - before[k], T, meta)[0] for k in names
            if not k.endswith("in_proj_bias")}
    dense = FX.load_dense(name)
    if dense is not None:  # the same metric over 1024 pinned elements per tensor (make_grad_dense.py)
        r.update(dense_metrics(names, {k: grads[k] * coef for k in names}, T, dense))
    r.update({"step1_loss_abs_err": abs(l1 - T["step1.loss"].item()),
              "grad_norm_rel_err": abs(total - T["step1.grad_total_norm_preclip"].item()) / total,
              "grad_rms_max": max(gerr.values()), "grad_rms_worst": max(gerr, key=gerr.get),
              "grad_rms_median": sorted(gerr.values())[len(gerr) // 2],
              "grad_norm_rel_err_max": max(gnorm.values()), "grad_norm_worst": max(gnorm, key=gnorm.get),
              "delta1_rms_max": max(derr.values()), "delta1_rms_median": sorted(derr.values())[len(derr) // 2]})
    return r
