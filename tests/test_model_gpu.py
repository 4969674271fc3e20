"""End-to-end parity of the MI355X train path against the reference's own outputs (golden
fixtures produced by running the reference in the build container) and against the CPU oracle.

fp32 mode: logits within 1e-3 (north star), argmax bit-exact wherever the reference's top-1/top-2
margin exceeds 1e-4, loss 1e-5, grads/updates at 1e-3 relative.
bf16 mode: logits within 1e-2 relative to their scale... see per-test tolerances (north star:
logits within 1e-2 bf16); argmax exact where the reference margin exceeds 5e-2.
"""
import pytest
import torch

import fixtures as FX
from model_util import build_model

pytestmark = pytest.mark.gpu

CASES = FX.CASES


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _fwd(m, meta):
    imgs, di, tg = FX.inputs(meta, 0)
    m.eval()
    with torch.no_grad():
        return m(imgs.cuda(), di.cuda()).float().cpu(), tg


@pytest.mark.parametrize("name", CASES)
def test_forward_fp32_matches_reference(name):
    meta, T = FX.load(name)
    m, _ = build_model(meta, torch.float32)
    logits, tg = _fwd(m, meta)
    got, ref = FX.logits_at(meta, T, logits)
    torch.testing.assert_close(got, ref, rtol=0, atol=1e-3)
    safe = T["fwd.margin"] > 1e-4
    assert torch.equal(logits.argmax(-1).float()[safe], T["fwd.argmax"][safe])
    loss = torch.nn.functional.cross_entropy(logits.reshape(-1, logits.shape[-1]), tg.reshape(-1), ignore_index=0)
    assert abs(loss.item() - T["fwd.loss"].item()) < 1e-4


@pytest.mark.parametrize("name", CASES)
def test_forward_bf16_matches_reference(name):
    meta, T = FX.load(name)
    m, _ = build_model(meta, torch.bfloat16)
    logits, tg = _fwd(m, meta)
    got, ref = FX.logits_at(meta, T, logits)
    # north star: logits within 1e-2 in bf16 — relative L2 error <= 1e-2, and no element off by
    # more than 2e-2 of the logit scale (bf16 keeps 8 mantissa bits: ~4e-3 per rounding)
    rel = ((got - ref).norm() / ref.norm()).item()
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    print(f"{name}: bf16 logits rel-L2 {rel:.2e}, max abs {err:.3e} (scale {scale:.2f})")
    assert rel <= 1e-2, f"bf16 logits rel-L2 err {rel:.4f}"
    assert err <= 2e-2 * max(1.0, scale), f"bf16 logits err {err:.4f} (scale {scale:.2f})"
    safe = T["fwd.margin"] > 5e-2
    agree = (logits.argmax(-1).float()[safe] == T["fwd.argmax"][safe]).float().mean().item()
    assert agree == 1.0, f"argmax agreement {agree:.4f} on margin>5e-2 positions"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("name", CASES)
def test_encoder_matches_reference(name, dtype):
    """The frozen encoder's last_hidden_state (HF ViT / CLIP vision tower) against the reference's,
    directly (not only through the decoder): fp32 within 1e-3; bf16 relative L2 <= 1.5e-2 and max
    error <= 3e-2 of the row scale (bf16 keeps 8 mantissa bits and the residual stream is bf16: the
    measured rel-L2 is 5.6e-3 for 2 layers, 9.1e-3 for ViT-B/16's 12, 1.07e-2 for CLIP-L's 24 —
    DESIGN.md §6)."""
    meta, T = FX.load(name)
    m, _ = build_model(meta, dtype)
    imgs, _, _ = FX.inputs(meta, 0)
    with torch.no_grad():
        feats = m.encoder.forward(imgs.cuda(), rows="all").float().cpu()
    for got, ref in FX.encoder_rows(T, feats):
        if dtype == torch.float32:
            torch.testing.assert_close(got, ref, rtol=0, atol=1e-3)
        else:
            rel = ((got - ref).norm() / ref.norm()).item()
            err = (got - ref).abs().max().item()
            print(f"{name}: bf16 encoder rows rel-L2 {rel:.2e} max abs {err:.3e} (scale {ref.abs().max():.2f})")
            assert rel <= 1.5e-2 and err <= 3e-2 * ref.abs().max().item()


@pytest.mark.parametrize("name", CASES)
def test_train_steps_fp32_match_reference(name):
    """train.py:62-123 step 1 (clip 5.0) and steps 2-3 (clip 0.1): loss, pre-clip grad norm,
    post-clip grads and parameter updates vs the reference."""
    import optim
    from decoder import flat_to_reference
    meta, T = FX.load(name)
    m, st = build_model(meta, torch.float32)
    m.train()
    names = FX.trainable_names(meta)
    opt = optim.AdamW(m.store, lr=meta["lr"], betas=tuple(meta["betas"]), eps=meta["eps"],
                      weight_decay=meta["weight_decay"])
    before = {k: v.clone() for k, v in m.state_dict().items() if k in names}
    imgs, di, tg = FX.inputs(meta, 0)
    loss = m.train_step(imgs.cuda(), di.cuda(), tg.cuda())
    torch.cuda.synchronize()
    assert abs(loss.item() - T["step1.loss"].item()) < 1e-4
    opt.step(meta["clip_first"])
    total, coef = opt.norm_t.tolist()
    assert abs(total - T["step1.grad_total_norm_preclip"].item()) < 1e-3 * total
    # post-clip grads in reference naming: rebuild a reference-named dict from the flat grad buffer
    gstore = _GradView(m.store)
    grads = flat_to_reference(gstore, m.decoder.L, m.decoder_embed_dim)
    if m.has_projection:
        grads["projection.weight"] = m.store.g("projection.weight").clone()
        grads["projection.bias"] = m.store.g("projection.bias").clone()
    after = m.state_dict()
    for k in names:
        FX.compare_stat("grad1", k, grads[k].cpu() * coef, T, meta, rtol=2e-3, atol=2e-6, scale_tol=1e-3,
                        outlier_frac=2e-3)
        FX.compare_stat("delta1", k, (after[k] - before[k]).cpu(), T, meta, rtol=2e-3, atol=2e-6)
    if meta["steps"] > 1:
        losses = []
        for s in range(1, meta["steps"]):
            _, di, tg = FX.inputs(meta, s)
            losses.append(m.train_step(imgs.cuda(), di.cuda(), tg.cuda()).item())
            opt.step(meta["clip_rest"])
        assert abs(sum(losses) / len(losses) - T["step3.avg_loss_23"].item()) < 1e-4
        after = m.state_dict()
        for k in names:
            FX.compare_stat("delta3", k, (after[k] - before[k]).cpu(), T, meta, rtol=5e-3, atol=3e-6)


class _GradView:
    """Duck-typed FlatParams whose .p() returns gradient views (to reuse flat_to_reference)."""

    def __init__(self, store):
        self.s = store
        self.vocab = getattr(store, "vocab", None)

    def p(self, name):
        return self.s.g(name)


@pytest.mark.parametrize("name", ["tiny_vit_patches", "cfg1_b2_patches", "cfg3_b2_patches"])
def test_train_step_bf16_close_to_reference(name):
    import optim
    meta, T = FX.load(name)
    m, st = build_model(meta, torch.bfloat16)
    m.train()
    opt = optim.AdamW(m.store, lr=meta["lr"], betas=tuple(meta["betas"]), eps=meta["eps"],
                      weight_decay=meta["weight_decay"])
    imgs, di, tg = FX.inputs(meta, 0)
    loss = m.train_step(imgs.cuda(), di.cuda(), tg.cuda())
    opt.step(meta["clip_first"])
    assert abs(loss.item() - T["step1.loss"].item()) < 1e-2
    total = opt.norm_t[0].item()
    assert abs(total - T["step1.grad_total_norm_preclip"].item()) < 3e-2 * total


def test_generate_matches_reference():
    """model.generate greedy ids (model.py:171-242) after the fixture's 3 reference steps."""
    import optim
    meta, T = FX.load("tiny_vit_cls")
    m, st = build_model(meta, torch.float32)
    m.train()
    opt = optim.AdamW(m.store, lr=meta["lr"], betas=tuple(meta["betas"]), eps=meta["eps"],
                      weight_decay=meta["weight_decay"])
    for s in range(meta["steps"]):
        imgs, di, tg = FX.inputs(meta, s)
        m.train_step(imgs.cuda(), di.cuda(), tg.cuda())
        opt.step(meta["clip_first"] if s == 0 else meta["clip_rest"])
    g = meta["generate"]
    for k in range(2):
        ids = m.generate(T[f"gen.pixel_values{k}"], g["start"], g["end"], max_len=g["max_len"])
        assert ids == g["ids"][k]


def test_dropout_train_step_matches_oracle_with_same_masks():
    """Dropout p=0.1 everywhere: rebuild the kernels' masks (mit_dropout_mask) and feed them to the
    CPU oracle (oracle.ref_cpu.decoder_forward drops=...); loss and grads must agree."""
    import math
    import native
    from oracle import ref_cpu as R
    meta, T = FX.load("tiny_vit_patches")
    m, st = build_model(meta, torch.float32, dropout=0.1)
    m.train()
    imgs, di, tg = FX.inputs(meta, 0)
    seed_before = m.seed_t.clone()
    loss = m.train_step(imgs.cuda(), di.cuda(), tg.cuda())
    torch.cuda.synchronize()
    seed = seed_before + 1  # train_step bumps the seed once before the forward
    dec = FX.dec_desc(meta)
    B, Tt = di.shape
    d, H, L, F = dec["d"], dec["heads"], dec["layers"], dec["ff"]
    S = FX.enc_desc(meta)["image"] // FX.enc_desc(meta)["patch"]
    S = S * S + 1

    def mask(n, site):
        out = torch.empty(n, device="cuda")
        native.dropout_mask(n, 0.1, seed, site, out)
        return out.cpu()

    drops = {"emb": mask(B * Tt * d, 4000).view(B, Tt, d)}
    for l in range(L):
        b = 64 * l
        drops[f"{l}.sa"] = mask(B * H * Tt * Tt, b).view(B, H, Tt, Tt)
        drops[f"{l}.d1"] = mask(B * Tt * d, b + 1).view(B, Tt, d)
        drops[f"{l}.ca"] = mask(B * H * Tt * S, b + 2).view(B, H, Tt, S)
        drops[f"{l}.d2"] = mask(B * Tt * d, b + 3).view(B, Tt, d)
        drops[f"{l}.ff"] = mask(B * Tt * F, b + 4).view(B, Tt, F)
        drops[f"{l}.d3"] = mask(B * Tt * d, b + 5).view(B, Tt, d)
    enc, decd = FX.enc_desc(meta), FX.dec_desc(meta)
    names = FX.trainable_names(meta)
    leaves = {k: st[k].clone().requires_grad_(True) for k in names}
    q = dict(st)
    q.update(leaves)
    logits = R.model_forward(q, imgs, di, enc, decd, meta["mode"], drops=drops)
    ref_loss = R.ce_loss(logits, tg)
    ref_loss.backward()
    assert abs(loss.item() - ref_loss.item()) < 1e-4
    from decoder import flat_to_reference
    grads = flat_to_reference(_GradView(m.store), L, d)
    for k in ["decoder.fc_out.weight", "decoder.transformer_decoder.layers.0.linear1.weight",
              "decoder.transformer_decoder.layers.0.self_attn.in_proj_weight", "decoder.token_embedding.weight",
              "decoder.transformer_decoder.layers.1.multihead_attn.in_proj_weight"]:
        torch.testing.assert_close(grads[k].cpu(), leaves[k].grad, rtol=2e-3, atol=2e-5)


def test_graphed_step_matches_eager():
    """make_graphed_step (one hipGraph per step) reproduces eager steps (dropout on, bf16)."""
    import optim
    meta, T = FX.load("tiny_vit_patches")
    res = []
    for graphed in (False, True):
        m, _ = build_model(meta, torch.bfloat16, dropout=0.1)
        m.train()
        opt = optim.AdamW(m.store, lr=1e-3)
        imgs, di, tg = FX.inputs(meta, 0)
        imgs, di, tg = imgs.cuda(), di.cuda(), tg.cuda()
        losses = []
        if graphed:
            g = m.make_graphed_step(opt, imgs, di, tg, 5.0)
            for _ in range(3):
                losses.append(g().item())
        else:
            for _ in range(3):
                losses.append(m.train_step(imgs, di, tg).item())
                opt.step(5.0)
        res.append((losses, m.store.master.clone()))
    (l0, p0), (l1, p1) = res
    assert all(abs(a - b) < 1e-3 for a, b in zip(l0, l1)), (l0, l1)
    torch.testing.assert_close(p1, p0, rtol=0, atol=1e-4)


def test_encoder_prefetch_matches_inline():
    """train_step(..., next_images=...) runs the frozen encoder of the next batch one step ahead on
    a second stream (double-buffered arenas); losses and parameters equal the inline schedule,
    including when the batch changes between steps."""
    import optim
    meta, T = FX.load("tiny_vit_patches")
    batches = [[t.cuda() for t in FX.inputs(meta, s)] for s in range(3)]
    res = []
    for prefetch in (False, True):
        m, _ = build_model(meta, torch.float32, dropout=0.1)
        m.train()
        opt = optim.AdamW(m.store, lr=1e-3)
        losses = []
        for s in range(4):
            imgs, di, tg = batches[s % 3]
            nxt = batches[(s + 1) % 3][0] if prefetch else None
            losses.append(m.train_step(imgs, di, tg, next_images=nxt).item())
            opt.step(5.0)
        res.append((losses, m.store.master.clone()))
    (l0, p0), (l1, p1) = res
    # every reduction of the step sums in a fixed order (split-K slabs, LayerNorm partials, CE rows,
    # the planned embedding scatter): the two schedules are bit-identical
    assert l0 == l1, (l0, l1)
    assert torch.equal(p1, p0)


def test_checkpoint_save_resume_roundtrip(tmp_path):
    """train.save_checkpoint -> train.load_checkpoint (train.py:343-375, 412-442): a resumed model
    continues where the original left off (weights, AdamW moments, step count, scheduler);
    the .safetensors restores weights only (inference.py:66-67)."""
    import optim
    import train as TR
    meta, _ = FX.load("tiny_vit_patches")
    batches = [[t.cuda() for t in FX.inputs(meta, s)] for s in range(3)]

    def fresh():
        m, _ = build_model(meta, torch.float32)
        m.train()
        opt = optim.AdamW(m.store, lr=1e-3)
        sch = TR.LinearWarmup(opt, 2, 10)
        return m, opt, sch

    def step(m, opt, sch, b):
        loss = m.train_step(*b)
        opt.step(5.0)
        sch.step()
        return loss.item()

    m, opt, sch = fresh()
    for b in batches[:2]:
        step(m, opt, sch, b)
    name = TR.save_checkpoint(m, opt, 0, 1.2345, str(tmp_path / "ck"), sch)
    ref_next = step(m, opt, sch, batches[2])
    ref_params = m.store.master.clone()

    m2, opt2, sch2 = fresh()
    start, best = TR.load_checkpoint(m2, opt2, sch2, name + ".pt")
    assert start == 1 and abs(best - 1.2345) < 1e-9
    # deterministic step: the resumed run continues bit-identically
    assert step(m2, opt2, sch2, batches[2]) == ref_next
    assert torch.equal(m2.store.master, ref_params)

    m3, opt3, sch3 = fresh()
    assert TR.load_checkpoint(m3, opt3, sch3, name + ".safetensors") == (0, float("inf"))
    m3.eval()
    m2b, _, _ = fresh()
    TR.load_checkpoint(m2b, optim.AdamW(m2b.store, lr=1e-3), None, name + ".pt")
    m2b.eval()
    imgs, di, _ = batches[0]
    with torch.no_grad():
        torch.testing.assert_close(m3(imgs, di), m2b(imgs, di), rtol=0, atol=0)
    assert TR.load_checkpoint(m3, opt3, sch3, str(tmp_path / "missing.pt")) == (0, float("inf"))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_decoder_memory_padding_mask_matches_reference(dtype):
    """TransformerDecoder.forward(tokens, memory, memory_padding_mask) against the reference decoder
    (fixture dec_memory_mask: memory rows past each length are padding)."""
    from decoder import TransformerDecoder, reference_to_flat
    meta, T = FX.load("dec_memory_mask")
    st = FX.state(meta)
    d = meta["dec"]
    dec = TransformerDecoder(d["vocab"], d["embed_dim"], d["heads"], d["layers"], d["ff"], 100, 0.0, 0, dtype=dtype)
    flat = reference_to_flat(st, d["layers"], d["embed_dim"])
    for k, v in flat.items():
        dec.store.p(k).copy_(v.cuda())
    dec.store.sync_shadow()
    dec.eval()
    B, S = meta["B"], meta["S"]
    mask = torch.zeros(B, S, dtype=torch.bool)
    for i, n in enumerate(meta["mem_lengths"]):
        mask[i, n:] = True
    logits = dec(T["tokens"].long().cuda(), T["memory"].cuda(), memory_padding_mask=mask).cpu()
    ref = T["logits"]
    if dtype == torch.float32:
        torch.testing.assert_close(logits, ref, rtol=0, atol=1e-3)
    else:
        assert ((logits - ref).norm() / ref.norm()).item() <= 1e-2
    # the mask matters: without it the logits differ
    assert (dec(T["tokens"].long().cuda(), T["memory"].cuda()).cpu() - ref).abs().max().item() > 1e-2
