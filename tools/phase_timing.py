"""Phase timeline of the bench's train step without a profiler: device wall-clock stamps (mit_stamp)
inserted on the main stream and the encoder-prefetch stream, recorded into the same native replay
bench.py times, then read back. Prints per-phase durations (us) of the replayed steps and where the
encoder prefetch runs relative to the decoder. Usage (GPU box): python tools/phase_timing.py"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multimodal-image-transformer_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import native  # noqa: E402

NAMES = ["start", "memory ready", "decoder fwd done", "CE done", "backward issued", "opt start", "opt done",
         "enc start", "enc done"]
WALL_HZ = 100e6  # MI300/MI355X device wall clock (hipDeviceAttributeWallClockRate = 100000 kHz)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--no-prefetch", action="store_true")
    a = ap.parse_args()
    args = argparse.Namespace(memory_mode="patches", workload="train", vocab=10000, dtype="bf16", batch=64, seq_len=64)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    model, opt = bench.build(args, 0)
    model.train()
    images, di, tg = bench.synthetic_batch(64, 64, 10000, dev, 1000, model.encoder.image)
    buf = torch.zeros(4 * 16, dtype=torch.int64, device=dev)
    row = [0]

    def stamp(i, stream=None):
        native.stamp(buf[row[0] * 16:], i, stream)

    dec = model.decoder
    wrap = [(model, "_encode_memory", 0, 1), (dec, "run_forward", None, 2), (dec, "run_backward", None, 4),
            (opt, "step", 5, 6)]
    for obj, name, before, after in wrap:
        fn = getattr(obj, name)

        def w(*x, _fn=fn, _b=before, _a=after, **k):
            if _b is not None:
                stamp(_b)
            r = _fn(*x, **k)
            stamp(_a)
            return r
        setattr(obj, name, w)
    ce = native.cross_entropy

    def ce_w(*x, **k):
        r = ce(*x, **k)
        stamp(3)
        return r
    native.cross_entropy = ce_w
    enc_rows = model._encoder_rows

    def enc_w(*x, **k):  # inside prefetch_encoder: the current stream is the encoder stream
        stamp(7)
        r = enc_rows(*x, **k)
        stamp(8)
        return r
    model._encoder_rows = enc_w

    def step():
        r = model.train_step(images, di, tg, next_images=None if a.no_prefetch else images)
        opt.step(5.0)
        return r
    for _ in range(5):
        step()
    progs = []
    for i in range(2):
        row[0] = i
        progs.append(native.record(step))
    torch.cuda.synchronize()
    for i in range(a.steps):
        progs[i % 2].run()
    torch.cuda.synchronize()
    t = buf.view(4, 16).cpu().tolist()
    for p in range(2):
        s = t[p]
        base = s[0]
        print(f"program {p}: " + ", ".join(f"{NAMES[i]} {1e6 * (s[i] - base) / WALL_HZ:8.1f}" for i in range(9) if s[i]))
    # step period: program 0's start to program 1's start
    per = 1e6 * (t[1][0] - t[0][0]) / WALL_HZ
    print(f"start(p1) - start(p0): {per:.1f} us")


if __name__ == "__main__":
    main()
