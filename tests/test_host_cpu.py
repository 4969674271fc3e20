"""Host-side logic that needs no GPU: HF key normalisation, reference <-> flat state-dict mapping,
flat-buffer layout, FLOP accounting."""
import pytest
import torch

import fixtures as FX


def test_hf_key_normalisation_vit5_vit4_clip():
    from encoder import _normalize_hf_key as n
    # transformers 5.x ViT (as the fixtures / reference state_dict carry them, with 'encoder.' prefix)
    assert n("encoder.layers.3.attention.q_proj.weight") == "layers.3.attention.q_proj.weight"
    assert n("encoder.layernorm.weight") == "layernorm.weight"
    assert n("encoder.embeddings.cls_token") == "embeddings.cls_token"
    assert n("layers.0.mlp.fc1.bias") == "layers.0.mlp.fc1.bias"
    # transformers 4.x ViT: ViTModel keys ('encoder.layer.N...') with and without the model prefix
    assert n("encoder.layer.2.attention.attention.query.weight") == "layers.2.attention.q_proj.weight"
    assert n("encoder.encoder.layer.2.attention.output.dense.bias") == "layers.2.attention.o_proj.bias"
    assert n("encoder.layer.5.intermediate.dense.weight") == "layers.5.mlp.fc1.weight"
    assert n("encoder.layer.5.output.dense.weight") == "layers.5.mlp.fc2.weight"
    assert n("encoder.layer.5.layernorm_before.weight") == "layers.5.layernorm_before.weight"
    # CLIP vision (5.x CLIPVisionModel and CLIPModel.vision_model)
    assert n("encoder.encoder.layers.1.self_attn.out_proj.weight") == "layers.1.attention.o_proj.weight"
    assert n("vision_model.encoder.layers.1.layer_norm2.bias") == "layers.1.layernorm_after.bias"
    assert n("encoder.pre_layrnorm.weight") == "pre_layrnorm.weight"


@pytest.mark.parametrize("name", ["tiny_vit_cls", "cfg1_b2_patches"])
def test_reference_flat_roundtrip(name):
    """reference_to_flat / flat_to_reference are inverse on the fixture weights (CPU FlatParams)."""
    from decoder import decoder_entries, flat_to_reference, reference_to_flat
    from params import FlatParams
    meta, _ = FX.load(name)
    st = FX.state(meta)
    dec = FX.dec_desc(meta)
    E = FX.enc_desc(meta)["hidden"]
    store = FlatParams(decoder_entries(dec["vocab"], dec["d"], dec["layers"], dec["ff"],
                                       E if E != dec["d"] else None), torch.device("cpu"), torch.float32)
    flat = reference_to_flat({k: v for k, v in st.items() if not k.startswith("encoder.")}, dec["layers"], dec["d"])
    assert set(flat) == set(store.names())
    for k, v in flat.items():
        store.p(k).copy_(v)
    back = flat_to_reference(store, dec["layers"], dec["d"])
    for k, v in back.items():
        torch.testing.assert_close(v, st[k], rtol=0, atol=0)
    # layout: 256-B aligned views, ordered fc_out first, embedding/projection last
    for _, _, off, _ in store.entries:
        assert off % 64 == 0
    assert store.names()[0] == "fc_out.weight"


def test_cfg1_flop_accounting_matches_survey():
    """cfg1 patches 50.17 GFLOP/pair, cls 45.56."""
    import math
    from decoder import decoder_entries
    N, E, mlp, Lenc = 197, 768, 3072, 12
    enc = Lenc * (2 * N * 4 * E * E + 2 * N * 2 * E * mlp + 4 * N * N * E) + 2 * (N - 1) * E * 768
    T, d, F, V, L = 63, 512, 2048, 10000, 6

    def dec(S):
        layer = 2 * T * 3 * d * d + 2 * T * d * d + 4 * T * T * d + 2 * T * d * d + 2 * S * 2 * d * d \
            + 4 * T * S * d + 2 * T * d * d + 2 * T * 2 * d * F
        return L * layer + 2 * T * d * V + 2 * S * E * d
    assert abs((enc + 3 * dec(197)) / 1e9 - 50.17) < 0.05
    assert abs((enc + 3 * dec(1)) / 1e9 - 45.56) < 0.05


def test_utils_masks_match_reference_semantics():
    import utils
    m = utils.generate_square_subsequent_mask(4)
    assert m[0, 1] == float("-inf") and m[1, 0] == 0 and m[3, 3] == 0
    tok = torch.tensor([[2, 5, 0, 0]])
    assert utils.create_padding_mask(tok, 0).tolist() == [[False, False, True, True]]


def test_linear_warmup_schedule():
    import train

    class O:
        param_groups = [{"lr": 1.0}]
    o = O()
    s = train.LinearWarmup(o, 2, 10)
    assert o.param_groups[0]["lr"] == 0.0
    s.step()
    assert abs(o.param_groups[0]["lr"] - 0.5) < 1e-9
    for _ in range(9):
        s.step()
    assert o.param_groups[0]["lr"] == 0.0


def test_inference_postprocess_matches_reference_rules():
    """inference.py:98-126: cut at the first END, drop one leading START, strip UNK and whitespace."""
    from inference import clean_text, postprocess_ids
    S, E = 1, 2
    assert postprocess_ids([1, 5, 6, 2, 7, 2], S, E) == [5, 6]
    assert postprocess_ids([1, 5, 6], S, E) == [5, 6]  # no END: everything kept
    assert postprocess_ids([5, 1, 6, 2], S, E) == [5, 1, 6]  # START only dropped in front
    assert postprocess_ids([1, 1, 2], S, E) == [1]  # one START dropped, not all
    assert postprocess_ids([2, 5], S, E) == []
    assert postprocess_ids([], S, E) == []
    assert clean_text("  a <UNK> dog   on<UNK> grass ") == "a dog on grass"
    assert clean_text("<UNK>") == ""


def _cpu_store(meta, n_enc):
    from decoder import decoder_entries
    from params import FlatParams
    dec = FX.dec_desc(meta)
    E = FX.enc_desc(meta)["hidden"]
    proj = E if E != dec["d"] else None
    store = FlatParams(decoder_entries(dec["vocab"], dec["d"], dec["layers"], dec["ff"], proj), torch.device("cpu"),
                       torch.float32)
    store.vocab = dec["vocab"]
    store.layout = dict(V=dec["vocab"], d=dec["d"], L=dec["layers"], F=dec["ff"], proj_in=proj, n_encoder_params=n_enc)
    return store


@pytest.mark.parametrize("name", ["tiny_vit_patches", "tiny_vit_v509", "tiny_clip336_cls"])
def test_optimizer_state_maps_torch_adamw_format(name):
    """optim.AdamW speaks torch.optim.AdamW's state_dict in the reference's parameter order
    (train.py:319-325 builds the optimizer over model.parameters(): frozen encoder first): a state
    produced by torch over the reference-shaped parameters loads into the flat moments, and
    state_dict() gives it back; a mismatching state is rejected with nothing written."""
    import optim
    meta, _ = FX.load(name)
    spec = [(n, tuple(s)) for n, s in meta["spec"]]
    n_enc = sum(1 for n, _ in spec if n.startswith("encoder."))
    store = _cpu_store(meta, n_enc)
    assert [n for n, _ in optim.reference_trainable(store.layout)] == [n for n, _ in spec if not n.startswith("encoder.")]
    params = [torch.nn.Parameter(torch.randn(s)) for _, s in spec]
    topt = torch.optim.AdamW(params, lr=3e-4, betas=(0.9, 0.98), eps=1e-9, weight_decay=1e-5)
    for i, (n, _) in enumerate(spec):
        if not n.startswith("encoder."):
            params[i].grad = torch.randn_like(params[i])
    topt.step()
    topt.step()
    sd = topt.state_dict()
    opt = optim.AdamW(store, lr=1.0)
    opt.load_state_dict(sd)
    assert opt.param_groups[0]["lr"] == 3e-4 and int(opt.step_t.item()) == 2
    back = opt.state_dict()
    assert back["param_groups"][0]["params"] == sd["param_groups"][0]["params"]
    assert set(back["state"]) == set(sd["state"])
    for i, s in sd["state"].items():
        for k in ("exp_avg", "exp_avg_sq"):
            torch.testing.assert_close(back["state"][i][k], s[k], rtol=0, atol=0)
        assert float(back["state"][i]["step"]) == float(s["step"])
    # padded head: the pad rows of the moments stay zero
    V = store.vocab
    fo = optim._BufView(store, store.exp_avg).p("fc_out.weight")
    assert torch.count_nonzero(fo[V:]) == 0
    # mismatches raise and leave the state alone
    before = store.exp_avg.clone()
    bad = {"state": dict(sd["state"]), "param_groups": sd["param_groups"]}
    k0 = max(bad["state"])
    bad["state"][k0] = dict(bad["state"][k0], exp_avg=torch.zeros(3))
    with pytest.raises(optim.OptimizerStateError):
        opt.load_state_dict(bad)
    with pytest.raises(optim.OptimizerStateError):
        opt.load_state_dict({"step": 1, "exp_avg": before})
    assert torch.equal(store.exp_avg, before)


@pytest.mark.parametrize("dp", [False, True])
def test_train_one_epoch_non_finite_loss(dp, monkeypatch, capsys):
    """Failure detection: a NaN loss (the reference's all-PAD batch) is reported with its step
    index -- raised with config.NONFINITE_LOSS = "raise", printed once by default (the reference trains on).
    The check runs on a device flag at log points (single process) and at the end of the epoch."""
    import torch
    import config
    import train as TR

    class Tiny(torch.nn.Module):
        device = torch.device("cpu")
        decoder_pad_idx = 0

        def __init__(self):
            super().__init__()
            self.w = torch.nn.Linear(4, 5)

        def forward(self, images, tokens):
            return self.w(images.flatten(1)).unsqueeze(1).expand(-1, tokens.shape[1], -1).contiguous()

    m = Tiny()
    opt = torch.optim.SGD(m.parameters(), lr=0.1)

    def crit(logits, tgt):  # the all-PAD batch: 0 / 0
        keep = tgt != 0
        return torch.nn.functional.cross_entropy(logits[keep], tgt[keep], reduction="sum") / keep.sum()
    batches = [{"images": torch.randn(2, 4), "decoder_input_tokens": torch.ones(2, 3, dtype=torch.int64),
                "target_tokens": torch.randint(1, 5, (2, 3)) if i != 2 else torch.zeros(2, 3, dtype=torch.int64)}
               for i in range(4)]
    monkeypatch.setattr(config, "NONFINITE_LOSS", "raise")
    with pytest.raises(TR.NonFiniteLossError, match="batch 3 .step index 2"):
        TR.train_one_epoch(m, batches, opt, crit, "cpu", 1.0, None, 0, 2, None)
    assert TR.train_one_epoch(m, batches[:2], opt, crit, "cpu", 1.0, None, 0, 0, None) > 0
    monkeypatch.setattr(config, "NONFINITE_LOSS", "warn")
    capsys.readouterr()
    TR.train_one_epoch(m, batches, opt, crit, "cpu", 1.0, None, 0, 1, None)
    err = capsys.readouterr().err
    assert err.count("non-finite training loss at batch 3 (step index 2)") == 1
    if dp:  # data parallel: no mid-epoch check (only rank 0 logs), the end-of-epoch one on every rank
        calls = []
        monkeypatch.setattr(TR, "_check_finite", lambda fb, ep: calls.append(int(fb.item())))
        monkeypatch.setattr(TR, "_fused_loss_ok", lambda *a: True)

        class FakeAdamW(TR.optim.AdamW):
            param_groups = [{"lr": 0.1}]

            def __init__(self):
                pass

            def zero_grad(self):
                pass

            def step(self, clip=0.0):
                pass

        m.train_step = lambda im, di, tg, dist=None, next_images=None: crit(m(im, di), tg).reshape(1)
        TR.train_one_epoch(m, batches, FakeAdamW(), crit, "cpu", 1.0, None, 0, 1, None, dist=object())
        assert calls == [2]


def test_encoder_residual_stream_policy(monkeypatch):
    """config.ENCODER_F32_RESIDUAL "auto": the f32 residual stream for the 24-layer CLIP-L towers and for
    "cls" memory (one encoder row per image reaches the logits undamped, tools/bf16_bisect.py); the folded
    bf16 stream for ViT towers feeding patch memory (the bench path); fp32 compute never folds."""
    import torch
    import config
    from encoder import VisionEncoder
    monkeypatch.setattr(config, "ENCODER_F32_RESIDUAL", "auto")
    vit, clip_l = config.ENCODER_SPECS["google/vit-base-patch16-224-in21k"], config.ENCODER_SPECS[
        "openai/clip-vit-large-patch14-336"]
    e = VisionEncoder(vit, torch.device("cpu"), torch.bfloat16)
    assert (e.res32, e.fold_ln) == (False, True)
    assert (e.configure_for("cls").res32, e.fold_ln) == (True, False)
    assert (e.configure_for("patches").res32, e.fold_ln) == (False, True)
    c = VisionEncoder(clip_l, torch.device("cpu"), torch.bfloat16)
    assert (c.configure_for("patches").res32, c.fold_ln) == (True, False)
    f = VisionEncoder(vit, torch.device("cpu"), torch.float32)
    assert (f.configure_for("cls").res32, f.fold_ln) == (False, False)
    monkeypatch.setattr(config, "ENCODER_F32_RESIDUAL", "off")
    assert (e.configure_for("cls").res32, e.fold_ln) == (False, True)
