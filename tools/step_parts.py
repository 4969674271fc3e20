"""Where the train step's time goes without a profiler in the way (rocprofv3's per-dispatch callbacks
stretch the host issue and serialise the streams: a profiled step runs ~25 % longer). Times, on the bench
workload (configs[1]) with native replay, HIP events around K replays of each:

  encoder   the frozen encoder forward alone (one batch)
  decoder   the step without the encoder: the prefetched features of one batch re-used every step
            (projection, decoder forward + CE + backward, clip + AdamW)
  serial    encoder then decoder on one stream (bench.py --no-prefetch)
  step      the bench step: the next batch's encoder on its own stream beside the decoder

overlap = (encoder + decoder - step) / min(encoder, decoder): 1 = the shorter part fully hidden.
Usage: python tools/step_parts.py [--steps K]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multimodal-image-transformer_amd"))

import bench  # noqa: E402
import native  # noqa: E402


def timed(fn, steps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / steps  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    args = argparse.Namespace(workload="train", memory_mode="patches", vocab=10000, dtype="bf16", batch=64, seq_len=64)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    model, opt = bench.build(args, 0)
    model.train()
    images, di, tg = bench.synthetic_batch(args.batch, args.seq_len, args.vocab, dev, 1000, model.encoder.image)
    out = {}

    def enc():
        model.encoder.forward(images, slot=0)
    out["encoder_us"] = timed(native.record(enc).run, a.steps)

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
    out["decoder_us"] = timed(lambda: (setattr(model, "_prefetched", pf), prog.run()), a.steps)
    model._prefetched = None

    def serial():
        model.train_step(images, di, tg)
        opt.step(5.0)
    for _ in range(2):
        serial()
    prog = native.record(serial)
    out["serial_us"] = timed(prog.run, a.steps)

    def full():
        model.train_step(images, di, tg, next_images=images)
        opt.step(5.0)
    for _ in range(3):
        full()
    progs = [native.record(full) for _ in range(2)]
    it = [0]

    def run():
        progs[it[0] % 2].run()
        it[0] += 1
    out["step_us"] = timed(run, a.steps)
    e, d, s = out["encoder_us"], out["decoder_us"], out["step_us"]
    out["overlap"] = round((e + d - s) / min(e, d), 3)
    out = {k: round(v, 1) if isinstance(v, float) and k != "overlap" else v for k, v in out.items()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
