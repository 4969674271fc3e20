"""Correctness gate for the exact launch sequence bench.py times (configs[1]: ViT-B/16 + 6L d512
decoder, patches memory, batch 64, seq_len 64, dropout 0.1, encoder prefetch stream, native replay).

* Replayed steps (native.record / mit_plan_run, as bench.py's timed loop runs them) equal eager
  steps bit for bit from the same state (the step is deterministic): losses and every f32 master
  weight after 2 warm-up + 2 recorded + 2 replayed steps.
* Training works at this size: on a fixed batch at lr 1e-3 the loss of 5 replayed steps is finite
  and decreasing (each step below the first, the last below all earlier ones)."""
import argparse
import math
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench_args():
    sys.path.insert(0, ROOT)
    import bench
    return bench, argparse.Namespace(workload="train", memory_mode="patches", vocab=10000, dtype="bf16", batch=64,
                                     seq_len=64)


def _model(lr):
    bench, a = _bench_args()
    torch.cuda.set_device(0)
    m, opt = bench.build(a, 0)
    opt.param_groups[0]["lr"] = lr
    m.train()
    images, di, tg = bench.synthetic_batch(a.batch, a.seq_len, a.vocab, torch.device("cuda", 0), 1000, m.encoder.image)
    return m, opt, images, di, tg


def test_bench_size_replay_equals_eager_bitwise():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import native
    res = []
    for replay in (False, True):
        m, opt, images, di, tg = _model(1e-4)

        def step():
            loss = m.train_step(images, di, tg, next_images=images)
            opt.step(5.0)
            return loss
        losses = [step().item() for _ in range(2)]
        if replay:
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
        res.append((losses, m.store.master.clone(), int(opt.step_t.item())))
        del m, opt
    (l0, p0, s0), (l1, p1, s1) = res
    assert s0 == s1 == 6
    assert l0 == l1, (l0, l1)
    assert torch.equal(p0, p1), (p0 - p1).abs().max().item()


def test_bench_size_loss_decreases():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import native
    m, opt, images, di, tg = _model(1e-3)
    loss_t = m.decoder.acts(64, 63, m.encoder.N, True).loss

    def step():
        m.train_step(images, di, tg, next_images=images)
        opt.step(5.0)
    opt._sync_lr()  # the lr lives in device memory: set it outside the recorded launches
    progs = [native.record(step) for _ in range(2)]
    losses = []
    for k in range(5):
        opt._sync_lr()
        progs[k % 2].run()
        losses.append(loss_t.item())
    assert all(math.isfinite(x) for x in losses), losses
    assert all(x < losses[0] for x in losses[1:]), losses
    assert losses[-1] < min(losses[:-1]), losses


def test_bench_size_prefetch_is_bitwise_neutral():
    """The encoder prefetch stream shares the chip with the step's decoder kernels: 3 steps with and
    without it must give bit-identical losses and master weights (a latent LDS WAR race in the 128-tile
    GEMM only showed under that concurrency, tools/diag_race.py)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = []
    for prefetch in (False, True, True):
        m, opt, images, di, tg = _model(1e-4)
        losses = []
        for _ in range(3):
            losses.append(m.train_step(images, di, tg, next_images=images if prefetch else None).item())
            opt.step(5.0)
        res.append((losses, m.store.master.clone()))
        del m, opt
    for losses, master in res[1:]:
        assert losses == res[0][0], (losses, res[0][0])
        assert torch.equal(master, res[0][1])
