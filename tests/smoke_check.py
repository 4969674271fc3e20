"""__graft_entry__.smoke(): one tiny train step of the flagship path on cuda:0, checked against the
reference's golden outputs (tests/golden, produced by the reference code) and the CPU oracle."""
import torch

import fixtures as FX
from model_util import build_model


def run():
    if not torch.cuda.is_available():
        raise RuntimeError("smoke() needs a GPU")
    import native
    import optim
    from oracle import ref_cpu as R
    native.load_library()
    meta, T = FX.load("tiny_vit_patches")
    m, st = build_model(meta, torch.bfloat16)
    imgs, di, tg = FX.inputs(meta, 0)
    m.eval()
    with torch.no_grad():
        logits = m(imgs.cuda(), di.cuda()).float().cpu()
    err = (logits - T["fwd.logits"]).abs().max().item()
    assert err < 1e-2 * max(1.0, T["fwd.logits"].abs().max().item()), f"bf16 logits off by {err}"
    # oracle cross-check on the same inputs
    oracle_logits = R.model_forward(st, imgs, di, FX.enc_desc(meta), FX.dec_desc(meta), meta["mode"])
    assert (logits - oracle_logits).abs().max().item() < 5e-2
    m.train()
    opt = optim.AdamW(m.store, lr=meta["lr"], betas=tuple(meta["betas"]), eps=meta["eps"],
                      weight_decay=meta["weight_decay"])
    loss = m.train_step(imgs.cuda(), di.cuda(), tg.cuda())
    opt.step(meta["clip_first"])
    torch.cuda.synchronize()
    lv = loss.item()
    assert abs(lv - T["step1.loss"].item()) < 1e-2, (lv, T["step1.loss"].item())
    assert torch.isfinite(m.store.master).all()
    print(f"smoke ok: bf16 logits max err {err:.2e}, train-step loss {lv:.5f} "
          f"(reference {T['step1.loss'].item():.5f}), grad norm {opt.norm_t[0].item():.4f}")


if __name__ == "__main__":
    run()
