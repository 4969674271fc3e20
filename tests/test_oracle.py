"""Pins the CPU oracle (oracle/ref_cpu.py) to the reference's own outputs (tests/golden).

Runs on CPU only. The fixtures were produced by executing the reference code (make_fixtures.py)."""
import pytest
import torch

import fixtures as FX
from oracle import ref_cpu as R


def _run_oracle_case(name):
    meta, T = FX.load(name)
    st = FX.state(meta)
    enc, dec = FX.enc_desc(meta), FX.dec_desc(meta)
    imgs, dec_in, tgt = FX.inputs(meta, 0)
    return meta, T, st, enc, dec, imgs, dec_in, tgt


@pytest.mark.parametrize("name", FX.CASES)
def test_oracle_forward_matches_reference(name):
    meta, T, st, enc, dec, imgs, dec_in, tgt = _run_oracle_case(name)
    with torch.no_grad():
        feats = R.encode(st, imgs, enc)
        for got, ref in FX.encoder_rows(T, feats):
            torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)
        logits = R.model_forward(st, imgs, dec_in, enc, dec, meta["mode"])
    got, ref = FX.logits_at(meta, T, logits)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)
    am = logits.argmax(-1).float()
    safe = T["fwd.margin"] > 1e-4
    assert torch.equal(am[safe], T["fwd.argmax"][safe])
    loss = R.ce_loss(logits, tgt)
    assert abs(float(loss) - float(T["fwd.loss"])) < 1e-5


@pytest.mark.parametrize("name", FX.CASES)
def test_oracle_train_steps_match_reference(name):
    meta, T, st, enc, dec, imgs, dec_in, tgt = _run_oracle_case(name)
    names = FX.trainable_names(meta)
    before = {k: st[k].clone() for k in names}
    opt = R.AdamWState({k: st[k] for k in names}, lr=meta["lr"], betas=tuple(meta["betas"]),
                       eps=meta["eps"], wd=meta["weight_decay"])
    loss, total, grads = R.train_step(st, names, opt, imgs, dec_in, tgt, enc, dec, meta["mode"], meta["clip_first"])
    assert abs(loss - float(T["step1.loss"])) < 1e-5
    assert abs(total - float(T["step1.grad_total_norm_preclip"])) < 1e-4 * max(1, total)
    for k in names:
        FX.compare_stat("grad1", k, grads[k], T, meta, rtol=1e-3, atol=1e-6)
        FX.compare_stat("delta1", k, st[k] - before[k], T, meta, rtol=1e-3, atol=1e-6)
    if meta["steps"] > 1:
        losses, norms = [], []
        for s in range(1, meta["steps"]):
            _, di, tg = FX.inputs(meta, s)
            l, n, _ = R.train_step(st, names, opt, imgs, di, tg, enc, dec, meta["mode"], meta["clip_rest"])
            losses.append(l)
            norms.append(n)
        assert abs(sum(losses) / len(losses) - float(T["step3.avg_loss_23"])) < 1e-5
        torch.testing.assert_close(torch.tensor(norms), T["step23.grad_total_norm_preclip"], rtol=1e-4, atol=1e-5)
        for k in names:
            FX.compare_stat("delta3", k, st[k] - before[k], T, meta, rtol=1e-3, atol=1e-6)


def test_oracle_generate_matches_reference():
    meta, T = FX.load("tiny_vit_cls")
    st = FX.state(meta)
    enc, dec = FX.enc_desc(meta), FX.dec_desc(meta)
    # generate() in the fixture ran AFTER the 3 training steps — replay them
    names = FX.trainable_names(meta)
    opt = R.AdamWState({k: st[k] for k in names}, lr=meta["lr"], betas=tuple(meta["betas"]),
                       eps=meta["eps"], wd=meta["weight_decay"])
    for s in range(meta["steps"]):
        imgs, di, tg = FX.inputs(meta, s)
        R.train_step(st, names, opt, imgs, di, tg, enc, dec, meta["mode"],
                     meta["clip_first"] if s == 0 else meta["clip_rest"])
    g = meta["generate"]
    import procedural as P
    for k in range(2):
        h, w = g["image_shapes"][k]
        img = P.pil_like_image(h, w, meta["seed"] + 50 + k)
        pv = R.vit_image_processor(img)
        torch.testing.assert_close(pv, T[f"gen.pixel_values{k}"], rtol=0, atol=1e-5)
        ids = R.greedy_generate(st, pv, enc, dec, g["start"], g["end"], g["max_len"], meta["mode"])
        assert ids == g["ids"][k]


def test_oracle_batched_generate_fixture():
    """cfg1_gen_cls (configs[4] anchor): the oracle's greedy ids = the reference's on all 4 images."""
    import procedural as P
    meta, _ = FX.load("cfg1_gen_cls")
    st = FX.state(meta)
    enc, dec = FX.enc_desc(meta), FX.dec_desc(meta)
    imgs = P.make_images(meta["n_images"], meta["image_size"], meta["image_seed"])
    assert abs(P.checksum([imgs]) - meta["images_checksum"]) < 1e-6 * abs(meta["images_checksum"])
    torch.set_num_threads(8)
    for i in range(meta["n_images"]):
        ids = R.greedy_generate(st, imgs[i:i + 1], enc, dec, meta["start"], meta["end"], meta["max_len"], "cls")
        assert ids == meta["ids"][i]


def test_procedural_inputs_stable():
    meta, _ = FX.load("tiny_vit_cls")
    import procedural as P
    imgs, di, tg = FX.inputs(meta, 0)
    assert abs(P.checksum([imgs]) - meta["images_checksum"]) < 1e-6 * abs(meta["images_checksum"]) + 1e-6


def test_oracle_decoder_memory_padding_mask():
    """decoder.TransformerDecoder.forward(tokens, memory, memory_padding_mask) (decoder.py:134-193)."""
    meta, T = FX.load("dec_memory_mask")
    st = FX.state(meta)
    B, S = meta["B"], meta["S"]
    mask = torch.zeros(B, S, dtype=torch.bool)
    for i, n in enumerate(meta["mem_lengths"]):
        mask[i, n:] = True
    d = meta["dec"]
    with torch.no_grad():
        logits = R.decoder_forward(st, T["tokens"].long(), T["memory"], heads=d["heads"], layers=d["layers"],
                                   memory_padding_mask=mask)
    torch.testing.assert_close(logits, T["logits"], rtol=1e-4, atol=1e-4)
