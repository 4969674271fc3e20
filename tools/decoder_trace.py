"""The configs[1] decoder half of the train step ALONE (the encoder's features of one batch prefetched once and
re-used: projection, decoder forward + CE + backward, clip + AdamW), replayed as bench.py replays the step, for a
rocprofv3 --kernel-trace run; analyse the CSV with tools/trace_gaps.py.
Usage: rocprofv3 --kernel-trace -d DIR -o run -- python3 tools/decoder_trace.py [--steps K]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multimodal-image-transformer_amd"))

import bench  # noqa: E402
import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    args = argparse.Namespace(workload="train", memory_mode="patches", vocab=10000, dtype="bf16", batch=64, seq_len=64)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    model, opt = bench.build(args, 0)
    model.train()
    images, di, tg = bench.synthetic_batch(args.batch, args.seq_len, args.vocab, dev, 1000, model.encoder.image)
    model.prefetch_encoder(images)
    torch.cuda.synchronize()
    pf = model._prefetched

    def dec():
        model._prefetched = pf
        model.train_step(images, di, tg)
        opt.step(5.0)
    for _ in range(2):
        dec()
    prog = native.record(dec)
    for _ in range(a.steps):
        model._prefetched = pf
        prog.run()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
