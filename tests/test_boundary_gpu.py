"""The reference's own training-loop call sequence on the MI355X model (SURVEY.md §8b boundary):

    optimizer = torch.optim.AdamW(model.parameters(), lr, betas, eps, weight_decay)   train.py:319-325
    criterion = nn.CrossEntropyLoss(ignore_index=PAD)                                  train.py:327
    optimizer.zero_grad()                                                              train.py:80
    logits = model(images, decoder_input_tokens)                                       train.py:83
    loss = criterion(logits.view(-1, V), target_tokens.view(-1))                       train.py:90
    loss.backward()                                                                    train.py:93
    torch.nn.utils.clip_grad_norm_(model.parameters(), GRAD_CLIP_VALUE)               train.py:96-97
    optimizer.step()                                                                   train.py:100

and train.train_one_epoch / train.evaluate (train.py:62-151) against the reference's outputs
(golden fixtures: step1.loss, grad1 (post-clip), delta1, step3.avg_loss_23, delta3, eval.loss),
plus resuming from a checkpoint in the reference's format (train.py:347-375, 422-436)."""
import pytest
import torch
import torch.nn as nn

import fixtures as FX
from model_util import build_model

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _named_grads(m):
    """p.grad of model.parameters() (flat entries) in the reference's names."""
    from decoder import flat_to_reference
    params = dict(m.named_parameters())

    class GV:
        vocab = m.decoder.V

        def p(self, n):
            g = params[n].grad
            return g if g is not None else torch.zeros_like(params[n])

    out = flat_to_reference(GV(), m.decoder.L, m.decoder_embed_dim)
    if m.has_projection:
        out["projection.weight"] = params["projection.weight"].grad
        out["projection.bias"] = params["projection.bias"].grad
    return out


def _reference_step(m, opt, crit, imgs, di, tg, clip):
    opt.zero_grad()
    logits = m(imgs, di)
    loss = crit(logits.view(-1, logits.size(-1)), tg.view(-1))
    loss.backward()
    torch.nn.utils.clip_grad_norm_(m.parameters(), clip)
    opt.step()
    return loss.item()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("name", ["tiny_vit_patches", "tiny_vit_v509", "cfg0_b4_cls"])
def test_reference_loop_with_torch_adamw(name, dtype):
    meta, T = FX.load(name)
    m, _ = build_model(meta, dtype)
    m.train()
    opt = torch.optim.AdamW(m.parameters(), lr=meta["lr"], betas=tuple(meta["betas"]), eps=meta["eps"],
                            weight_decay=meta["weight_decay"])
    crit = nn.CrossEntropyLoss(ignore_index=0)
    names = FX.trainable_names(meta)
    before = {k: v.clone() for k, v in m.state_dict().items() if k in names}
    imgs, di, tg = [t.cuda() for t in FX.inputs(meta, 0)]
    loss = _reference_step(m, opt, crit, imgs, di, tg, meta["clip_first"])
    after = m.state_dict()
    if dtype == torch.float32:
        assert abs(loss - T["step1.loss"].item()) < 1e-4
        grads = _named_grads(m)
        for k in names:
            FX.compare_stat("grad1", k, grads[k].cpu(), T, meta, rtol=2e-3, atol=2e-6, scale_tol=1e-3,
                            outlier_frac=2e-3)
            FX.compare_stat("delta1", k, (after[k] - before[k]).cpu(), T, meta, rtol=2e-3, atol=2e-6)
    else:  # bf16: DESIGN.md §6 tolerances (loss 5e-3, updates through the sign of near-zero grads)
        assert abs(loss - T["step1.loss"].item()) < 5e-3
    if meta["steps"] > 1:
        losses = []
        for s in range(1, meta["steps"]):
            _, di, tg = [t.cuda() for t in FX.inputs(meta, s)]
            losses.append(_reference_step(m, opt, crit, imgs, di, tg, meta["clip_rest"]))
        tol = 1e-4 if dtype == torch.float32 else 5e-3
        assert abs(sum(losses) / len(losses) - T["step3.avg_loss_23"].item()) < tol
        if dtype == torch.float32:
            after = m.state_dict()
            for k in names:
                FX.compare_stat("delta3", k, (after[k] - before[k]).cpu(), T, meta, rtol=5e-3, atol=3e-6)


@pytest.mark.parametrize("fused", [True, False])
def test_train_one_epoch_and_evaluate_match_reference(fused):
    """train.train_one_epoch over the fixture's batches exactly as make_fixtures ran the reference's
    (one epoch of batch 0 with clip 5.0, one epoch of batches 1-2 with clip 0.1), then evaluate():
    the returned averages equal step1.loss, step3.avg_loss_23 and eval.loss. fused: optim.AdamW +
    model.train_step; else torch.optim.AdamW through autograd."""
    import optim
    import train as TR
    meta, T = FX.load("tiny_vit_patches")
    m, _ = build_model(meta, torch.float32)
    kw = dict(lr=meta["lr"], betas=tuple(meta["betas"]), eps=meta["eps"], weight_decay=meta["weight_decay"])
    opt = optim.AdamW(m.parameters(), **kw) if fused else torch.optim.AdamW(m.parameters(), **kw)
    crit = nn.CrossEntropyLoss(ignore_index=0)
    batches = []
    for s in range(meta["steps"]):
        imgs, di, tg = FX.inputs(meta, s)
        batches.append({"images": imgs, "decoder_input_tokens": di, "target_tokens": tg})
    a1 = TR.train_one_epoch(m, batches[:1], opt, crit, "cuda", meta["clip_first"], None, 0, 50, None)
    assert abs(a1 - T["step1.loss"].item()) < 1e-4
    a23 = TR.train_one_epoch(m, batches[1:], opt, crit, "cuda", meta["clip_rest"], None, 1, 50, None)
    assert abs(a23 - T["step3.avg_loss_23"].item()) < 1e-4
    ev = TR.evaluate(m, batches[:1], crit, "cuda")
    assert abs(ev - T["eval.loss"].item()) < 1e-4


def test_uint8_collate_batch_equals_normalised_batch():
    """A data.collate_fn batch (uint8 HWC images, normalised on the GPU by model.image_processor)
    trains exactly like the same images normalised on the host first."""
    import numpy as np
    import data
    import optim
    import train as TR
    meta, _ = FX.load("tiny_vit_patches")
    g = torch.Generator().manual_seed(3)
    u8 = torch.randint(0, 256, (meta["B"], 224, 224, 3), generator=g, dtype=torch.uint8)
    _, di, tg = FX.inputs(meta, 0)
    items = [{"image_path": f"{i}.jpg", "image": u8[i], "caption_tokens": torch.cat([di[i, :1], tg[i]])}
             for i in range(meta["B"])]
    b_u8 = data.collate_fn(items)
    x = (u8.float().numpy() / np.float32(255.0) - np.float32(0.5)) / np.float32(0.5)
    b_f = dict(b_u8, images=torch.from_numpy(x).permute(0, 3, 1, 2).contiguous())
    res = []
    for b in (b_u8, b_f):
        m, _ = build_model(meta, torch.float32)
        opt = optim.AdamW(m.parameters(), lr=1e-3)
        res.append((TR.train_one_epoch(m, [b], opt, None, "cuda", 5.0, None, 0, 0, None), m.store.master.clone()))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])


def test_resume_from_reference_format_checkpoint(tmp_path):
    """A checkpoint written the way the reference writes it (train.py:422-436: model.state_dict()
    in the reference's keys incl. the frozen encoder, torch.optim.AdamW(model.parameters()).state_dict()
    with encoder indices first) resumes here: step 2 after the resume equals the oracle's step 2."""
    import optim
    import train as TR
    from oracle import ref_cpu as R
    meta, T = FX.load("tiny_vit_patches")
    st = FX.state(meta)
    enc, dec = FX.enc_desc(meta), FX.dec_desc(meta)
    names = FX.trainable_names(meta)
    spec_names = [n for n, _ in meta["spec"]]
    # reference: one step (oracle = pinned restatement), optimizer = torch AdamW over ALL parameters
    ref_params = {n: st[n].clone().requires_grad_(n in names) for n in spec_names}
    topt = torch.optim.AdamW([ref_params[n] for n in spec_names], lr=meta["lr"], betas=tuple(meta["betas"]),
                             eps=meta["eps"], weight_decay=meta["weight_decay"])
    imgs, di, tg = FX.inputs(meta, 0)
    logits = R.model_forward(ref_params, imgs, di, enc, dec, meta["mode"])
    R.ce_loss(logits, tg).backward()
    torch.nn.utils.clip_grad_norm_([ref_params[n] for n in names], meta["clip_first"])
    topt.step()
    ck = {"epoch": 0, "model_state_dict": {n: p.detach().clone() for n, p in ref_params.items()},
          "optimizer_state_dict": topt.state_dict(), "best_val_loss": 3.21}
    ck["model_state_dict"]["decoder.positional_encoding.pe"] = torch.zeros(1, 100, dec["d"])
    path = str(tmp_path / "ref_format.pt")
    torch.save(ck, path)
    # reference step 2
    _, di2, tg2 = FX.inputs(meta, 1)
    topt.zero_grad()
    logits = R.model_forward(ref_params, imgs, di2, enc, dec, meta["mode"])
    loss2 = R.ce_loss(logits, tg2)
    loss2.backward()
    torch.nn.utils.clip_grad_norm_([ref_params[n] for n in names], meta["clip_rest"])
    topt.step()
    # ours: fresh model (different weights), resume, step 2
    m, _ = build_model(meta, torch.float32)
    with torch.no_grad():
        m.store.master.mul_(0.5)  # make sure the resume really overwrites the weights
    opt = optim.AdamW(m.parameters(), lr=1.0)
    start, best = TR.load_checkpoint(m, opt, None, path)
    assert start == 1 and abs(best - 3.21) < 1e-9
    assert opt.param_groups[0]["lr"] == meta["lr"] and int(opt.step_t.item()) == 1
    ours = m.train_step(imgs.cuda(), di2.cuda(), tg2.cuda())
    opt.step(meta["clip_rest"])
    assert abs(ours.item() - loss2.item()) < 1e-4
    sd = m.state_dict()
    for n in names:
        got, ref = sd[n].cpu().flatten(), ref_params[n].detach().flatten()
        keep = FX.degenerate_mask(n, ref, meta)  # in_proj_bias key rows: exactly-zero true gradient
        if keep is not None:
            got, ref = got[keep], ref[keep]
        torch.testing.assert_close(got, ref, rtol=1e-4, atol=2e-6)
    # and our checkpoint's optimizer state IS torch's format: torch.optim.AdamW loads it
    name = TR.save_checkpoint(m, opt, 1, 1.0, str(tmp_path / "ours"))
    ck2 = torch.load(name + ".pt", map_location="cpu", weights_only=True)
    topt.load_state_dict(ck2["optimizer_state_dict"])
    for i, n in enumerate(spec_names):
        if n in names:
            torch.testing.assert_close(topt.state[ref_params[n]]["exp_avg"], ck2["optimizer_state_dict"]["state"][i]["exp_avg"])


def test_incompatible_checkpoint_raises(tmp_path):
    """A checkpoint that exists but does not fit raises instead of silently training from scratch."""
    import optim
    import train as TR
    meta, _ = FX.load("tiny_vit_patches")
    m, _ = build_model(meta, torch.float32)
    opt = optim.AdamW(m.parameters(), lr=1e-3)
    bad = {"epoch": 0, "model_state_dict": m.state_dict(), "optimizer_state_dict": {"step": 3}}
    torch.save(bad, str(tmp_path / "bad.pt"))
    before = m.store.master.clone()
    with pytest.raises(TR.CheckpointError):
        TR.load_checkpoint(m, opt, None, str(tmp_path / "bad.pt"))
    sd = m.state_dict()
    sd["decoder.fc_out.weight"] = sd["decoder.fc_out.weight"][:-1]
    torch.save({"epoch": 0, "model_state_dict": sd, "optimizer_state_dict": opt.state_dict()}, str(tmp_path / "b2.pt"))
    with pytest.raises(TR.CheckpointError):
        TR.load_checkpoint(m, opt, None, str(tmp_path / "b2.pt"))
    assert torch.equal(m.store.master, before)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_weight_edit_through_p_data_is_seen(dtype):
    """An out-of-band weight edit through p.data (no version-counter bump) reaches the kernels: the
    autograd forward, evaluation and generation refresh the bf16 shadow every call, and after
    model.sync_shadow() the fused train step sees it too (params.FlatParams.ensure_shadow)."""
    meta, _ = FX.load("tiny_vit_patches")
    m, _ = build_model(meta, dtype)
    ref, _ = build_model(meta, dtype)
    m.eval()
    ref.eval()
    imgs, di, tg = [t.cuda() for t in FX.inputs(meta, 0)]
    pm = dict(m.named_parameters())
    pr = dict(ref.named_parameters())
    g = torch.Generator().manual_seed(3)
    new = torch.randn(pm["fc_out.weight"].shape, generator=g).mul_(0.05).cuda()
    with torch.no_grad():
        _ = m(imgs, di)  # shadow synced once before the edit
        pm["fc_out.weight"].data.copy_(new)
        pr["fc_out.weight"].data.copy_(new)
        ref.sync_shadow()
        got, want = m(imgs, di), ref(imgs, di)
    assert torch.equal(got, want)
    m.train()
    ref.train()
    with torch.no_grad():
        pm["fc_out.bias"].data.add_(0.25)
        pr["fc_out.bias"].data.add_(0.25)
    m.sync_shadow()
    ref.sync_shadow()
    assert torch.equal(m.train_step(imgs, di, tg), ref.train_step(imgs, di, tg))


def test_torch_adamw_checkpoint_round_trip(tmp_path):
    """The autograd path's torch.optim.AdamW(model.parameters()) state is saved in the REFERENCE
    format (train.optimizer_state_reference): the reference-shaped torch.optim.AdamW loads it, and it
    resumes a fresh model's torch.optim.AdamW -- whose next step then equals the uninterrupted one."""
    import train as TR
    meta, _ = FX.load("tiny_vit_patches")
    kw = dict(lr=meta["lr"], betas=tuple(meta["betas"]), eps=meta["eps"], weight_decay=meta["weight_decay"])
    crit = nn.CrossEntropyLoss(ignore_index=0)
    m, st = build_model(meta, torch.float32)
    m.train()
    opt = torch.optim.AdamW(m.parameters(), **kw)
    imgs, di, tg = [t.cuda() for t in FX.inputs(meta, 0)]
    _reference_step(m, opt, crit, imgs, di, tg, meta["clip_first"])
    name = TR.save_checkpoint(m, opt, 0, 2.5, str(tmp_path / "tadam"))
    ck = torch.load(name + ".pt", map_location="cpu", weights_only=True)
    osd = ck["optimizer_state_dict"]
    # reference layout: encoder tensors first (no state), then reference_trainable order
    import optim
    lay = m.store.layout
    names = optim.reference_trainable(lay)
    assert len(osd["param_groups"][0]["params"]) == lay["n_encoder_params"] + len(names)
    for i, (n, shape) in enumerate(names):
        assert tuple(osd["state"][lay["n_encoder_params"] + i]["exp_avg"].shape) == shape, n
    ref_params = [torch.nn.Parameter(torch.zeros(1)) for _ in range(lay["n_encoder_params"])] + \
        [torch.nn.Parameter(torch.zeros(shape)) for _, shape in names]
    torch.optim.AdamW(ref_params, **kw).load_state_dict(osd)
    # resume into a fresh model + torch AdamW, then one more step on both
    m2, _ = build_model(meta, torch.float32)
    m2.train()
    opt2 = torch.optim.AdamW(m2.parameters(), lr=1.0)
    start, best = TR.load_checkpoint(m2, opt2, None, name + ".pt")
    assert start == 1 and abs(best - 2.5) < 1e-9 and opt2.param_groups[0]["lr"] == meta["lr"]
    _, di1, tg1 = [t.cuda() for t in FX.inputs(meta, 1)]
    l1 = _reference_step(m, opt, crit, imgs, di1, tg1, meta["clip_rest"])
    l2 = _reference_step(m2, opt2, crit, imgs, di1, tg1, meta["clip_rest"])
    assert abs(l1 - l2) < 1e-6
    torch.testing.assert_close(m2.store.master, m.store.master, rtol=1e-5, atol=1e-7)
