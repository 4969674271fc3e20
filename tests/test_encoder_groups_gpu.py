"""The f32-stream encoder forward as two image groups on two streams (encoder.forward_iter_groups: the
CLIP-L/14@336 and CLIP-L/14 forwards of configs[2] / configs[3]) against the one-stream forward on the same
256-tile GEMM kernels: bit-identical rows (every op is row- or image-wise)."""
import pytest
import torch

import encoder
import native

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    native.load_library()


@pytest.mark.parametrize("name,B", [("openai/clip-vit-large-patch14-336", 64), ("openai/clip-vit-large-patch14", 64),
                                    ("openai/clip-vit-base-patch32", 6), ("google/vit-base-patch16-224-in21k", 4)])
def test_groups_equal_one_stream(name, B):
    dev = torch.device("cuda")
    enc = encoder.build_encoder(name, dev, torch.bfloat16, seed=3)
    enc.configure_for("patches" if enc.L >= 24 else "cls")  # the f32 residual stream
    assert enc.res32
    small = B * enc.N < enc.GROUP_ROWS
    if small:
        # force the grouped path, and the 256-tile kernel for every GEMM (below 256 rows a half-batch GEMM
        # takes the 128 kernel: the same values up to the fp32 summation order)
        enc.GROUP_ROWS = B * enc.N
        native.gemm_set_variant(2)
    assert enc.groups_for(B) == 2
    try:
        g = torch.Generator().manual_seed(B)
        img = torch.randn(B, 3, enc.image, enc.image, generator=g).to(dev)
        # the one-stream forward on the groups' kernels (tiles = 256) as the reference
        ref = encoder.drain(enc.forward_iter(img, "all", 0, tiles=256)).clone()
        for slot in (0, 1):
            out = encoder.drain(enc.forward_iter_groups(img, slot)) if slot else enc.forward(img, rows="all", slot=0)
            torch.cuda.synchronize()
            assert out.shape == ref.shape
            assert torch.equal(out, ref), (out.float() - ref.float()).abs().max().item()
    finally:
        native.gemm_set_variant(0)


def test_groups_only_for_large_f32_stream():
    dev = torch.device("cuda")
    enc = encoder.build_encoder("openai/clip-vit-large-patch14-336", dev, torch.bfloat16, seed=1)
    enc.configure_for("patches")
    assert enc.groups_for(64) == 2 and enc.groups_for(32) == 2 and enc.groups_for(28) == 1 and enc.groups_for(63) == 1
    assert enc.groups_for(64, rows="cls") == 1


@pytest.mark.parametrize("workload", ["clip336", "cfg3"])
def test_bench_step_grouped_encoder_prefetch_bitwise_neutral(workload):
    """configs[2] / configs[3] as bench.py runs them (CLIP-L/14@336 + 6L d512 decoder / CLIP-L/14 + 12L d768
    decoder, patches memory, batch 64; the encoder as two image groups): steps with the prefetched encoder
    and without a prefetch give bit-identical losses and master weights, and the same steps replayed from
    recorded launch plans match them."""
    import argparse
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    a = argparse.Namespace(workload=workload, memory_mode="patches", vocab=10000, dtype="bf16", batch=64, seq_len=64)
    torch.cuda.set_device(0)
    res = []
    for mode in ("none", "prefetch", "replay"):
        m, opt = bench.build(a, 0)
        opt.param_groups[0]["lr"] = 1e-4
        m.train()
        images, di, tg = bench.synthetic_batch(a.batch, a.seq_len, a.vocab, torch.device("cuda", 0), 1000,
                                               m.encoder.image)
        assert m.encoder.groups_for(a.batch) == 2

        def step():
            loss = m.train_step(images, di, tg, next_images=None if mode == "none" else images)
            opt.step(5.0)
            return loss
        losses = [step().item() for _ in range(2)]
        if mode == "replay":
            loss_t = m.decoder.acts(64, 63, m.encoder.N, True).loss
            progs = []
            for _ in range(2):
                progs.append(native.record(step))
                losses.append(loss_t.item())
            for k in range(2):
                opt._sync_lr()
                progs[k % 2].run()
                losses.append(loss_t.item())
        else:
            losses += [step().item() for _ in range(4)]
        torch.cuda.synchronize()
        res.append((losses, m.store.master.clone()))
        del m, opt
    for losses, master in res[1:]:
        assert losses == res[0][0], (losses, res[0][0])
        assert torch.equal(master, res[0][1]), (master - res[0][1]).abs().max().item()
