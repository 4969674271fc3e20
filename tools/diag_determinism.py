"""Determinism diagnostic at the bench size (configs[1], B = 64). (1) Three freshly built models (same
seed) run 4 train steps: without the encoder prefetch, with it, with it again -- losses and master
weights must be bit-identical across all three. (2) The encoder output computed on the prefetch
stream beside a train step must equal the same encoder run alone. Usage (GPU box):
python tools/diag_determinism.py"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

A = argparse.Namespace(workload="train", memory_mode="patches", vocab=10000, dtype="bf16", batch=64, seq_len=64)


def steps(prefetch, n=4):
    m, opt = bench.build(A, 0)
    images, di, tg = bench.synthetic_batch(64, 64, 10000, torch.device("cuda", 0), 1000, m.encoder.image)
    losses = []
    for _ in range(n):
        losses.append(m.train_step(images, di, tg, next_images=images if prefetch else None).clone())
        opt.step(5.0)
    torch.cuda.synchronize()
    out = ([x.item() for x in losses], m.store.master.clone())
    del m, opt
    return out


def encoder_concurrency(rounds=4):
    m, opt = bench.build(A, 0)
    images, di, tg = bench.synthetic_batch(64, 64, 10000, torch.device("cuda", 0), 1000, m.encoder.image)
    ref = m._encoder_rows(images, 0)[0].clone()
    alone1 = m._encoder_rows(images, 1)[0].clone()
    print("encoder slot0 == slot1 (alone):", torch.equal(ref, alone1), flush=True)
    m.train_step(images, di, tg)  # arenas sized
    for r in range(rounds):
        m.train_step(images, di, tg, next_images=images)  # prefetch beside this step
        pf = m._prefetched
        torch.cuda.synchronize()
        got = pf[2][0]
        d = (got.float() - ref.float()).abs()
        print(f"round {r}: prefetched slot {pf[1]} equal={torch.equal(got, ref)} n_diff={(d > 0).sum().item()} "
              f"max={d.max().item():.3e}", flush=True)
        m._prefetched = None  # recompute inline next time
        m._enc_slot = 0


def main():
    torch.cuda.set_device(0)
    a = steps(False)
    b = steps(True)
    c = steps(True)
    print("no prefetch :", a[0])
    print("prefetch #1 :", b[0])
    print("prefetch #2 :", c[0])
    print("masters equal a/b:", torch.equal(a[1], b[1]), " b/c:", torch.equal(b[1], c[1]), flush=True)
    encoder_concurrency()


if __name__ == "__main__":
    main()
