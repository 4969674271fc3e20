"""Host-side (Python) cost of enqueueing the default bench step: cProfile over K steps on the GPU box.
    python tools/host_profile.py [steps]"""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-image-transformer_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)

    class A:
        vocab, memory_mode, dtype = 10000, "patches", "bf16"
    model, opt = bench.build(A, 0)
    model.train()
    images, di, tg = bench.synthetic_batch(64, 64, 10000, dev, 1000)

    def step():
        model.train_step(images, di, tg, next_images=images)
        opt.step(5.0)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(K):
        step()
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
