"""Decoder cross-attention (64 images x 8 heads, 63 queries over 197 patch keys, head_dim 64) forward and
backward with the K/V rows in the training layout (all layers' K|V in one [B*S, L*2d] row: 12 KiB row stride at
configs[1]) against a per-layer contiguous layout ([B*S, 2d] rows: 2 KiB stride): is the strided K/V read
costing DRAM efficiency? Usage: python tools/attn_layout_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-image-transformer_amd"))
import torch  # noqa: E402

import native as N  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    dev = torch.device("cuda")
    B, H, T, S, d, L = 64, 8, 63, 197, 512, 6
    q = torch.randn(B * T, d, device=dev).to(torch.bfloat16)
    do = torch.randn(B * T, d, device=dev).to(torch.bfloat16)
    o = torch.empty_like(q)
    dq = torch.empty_like(q)
    lse = torch.empty(B * H * T, device=dev)
    delta = torch.empty(B * H * T, device=dev)
    seed = torch.tensor([3], dtype=torch.int64, device=dev)
    res = {}
    for name, width in (("training layout (L*2d row)", L * 2 * d), ("per-layer layout (2d row)", 2 * d)):
        kv = torch.randn(B * S, width, device=dev).to(torch.bfloat16)
        dkv = torch.empty_like(kv)
        a = N.attn_args(q, d, T * d, kv, width, S * width, kv[:, d:], width, S * width, o, d, T * d, lse=lse,
                        scale=0.125, drop_p=0.1, seed=seed, site=2)
        g = N.attn_grads(do, d, T * d, dq, d, T * d, dkv, width, S * width, dkv[:, d:], width, S * width, delta)
        tf = timeit(lambda: N.attention_fwd(N.BF16, B, H, T, S, a))
        tb = timeit(lambda: N.attention_bwd(N.BF16, B, H, T, S, a, g))
        res[name] = (tf, tb)
        print(f"{name:28s} forward {tf:6.1f} us  backward {tb:6.1f} us", flush=True)


if __name__ == "__main__":
    N.load_library()
    main()
