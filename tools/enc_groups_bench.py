"""Encoder forward alone, one stream vs two image groups on two streams (VisionEncoder.forward_iter_groups),
CLIP-L/14@336 f32 residual stream at B = 64 (configs[2]'s encoder), eager launches: ms per forward (min of
rounds) and the max |difference| of the two outputs. Optional argv[1]: gemm variant (0 per shape, 2 = 256
tiles everywhere)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-image-transformer_amd"))
import torch  # noqa: E402

import encoder  # noqa: E402
import native  # noqa: E402


def main():
    native.load_library()
    native.gemm_set_variant(int(sys.argv[1]) if len(sys.argv) > 1 else 0)
    dev = torch.device("cuda")
    enc = encoder.build_encoder("openai/clip-vit-large-patch14-336", dev, torch.bfloat16)
    enc.configure_for("patches")
    B = 64
    img = torch.randn(B, 3, 336, 336, device=dev)
    assert enc.groups_for(B) == 2, "expected the grouped path"

    def one():  # one stream, tiles per shape
        return encoder.drain(enc.forward_iter(img, "all", 0))

    def grouped():
        return encoder.drain(enc.forward_iter_groups(img, 0))

    a = one().clone()
    b = grouped().clone()
    torch.cuda.synchronize()
    print(f"max |one - grouped| = {(a.float() - b.float()).abs().max().item():.3e}  "
          f"bitwise equal: {torch.equal(a, b)}", flush=True)
    best = {}
    for _ in range(3):
        for name, fn in (("one stream", one), ("two groups", grouped)):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                fn()
            e1.record()
            torch.cuda.synchronize()
            best[name] = min(best.get(name, 1e9), e0.elapsed_time(e1) / 3)
    for k, v in best.items():
        print(f"{k:12s} {v:8.2f} ms per forward", flush=True)


if __name__ == "__main__":
    main()
