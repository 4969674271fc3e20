"""Interleaved same-process A/B of the configs[1] train step (bench.py's replayed plan) over GEMM tile-kernel
variants (mit_gemm_set_variant: 0 = per-shape default, 1 = 128 kernel only, 2 = 256 kernel wherever split-K is
not planned) and decoder options. Each arm records its own two-step plan; rounds alternate the arms.
Usage: python tools/step_ab.py --arms 0,2 [--rounds 3] [--steps 20]
An arm is "<variant>" or "<variant>:<env>=<value>[:...]" (environment set while the arm's plan records)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multimodal-image-transformer_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", default="0,2")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    args = argparse.Namespace(workload="train", memory_mode="patches", vocab=10000, dtype="bf16", batch=64, seq_len=64)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    model, opt = bench.build(args, 0)
    model.train()
    images, di, tg = bench.synthetic_batch(args.batch, args.seq_len, args.vocab, dev, 1000, model.encoder.image)

    def step():
        model.train_step(images, di, tg, next_images=images)
        opt.step(5.0)

    arms = {}
    for arm in a.arms.split(","):
        parts = arm.split(":")
        env = dict(p.split("=", 1) for p in parts[1:])
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        native.gemm_set_variant(int(parts[0]))
        for _ in range(3):
            step()
        arms[arm] = [native.record(step) for _ in range(2)]
        native.gemm_set_variant(0)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    res = {k: [] for k in arms}
    for _ in range(a.rounds):
        for arm, progs in arms.items():
            native.gemm_set_variant(int(arm.split(":")[0]))  # mit_gemm picks its kernel at replay time too
            for i in range(4):
                progs[i % 2].run()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.steps):
                opt._sync_lr()
                progs[i % 2].run()
            torch.cuda.synchronize()
            res[arm].append(round(args.batch * a.steps / (time.perf_counter() - t0), 1))
    native.gemm_set_variant(0)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
