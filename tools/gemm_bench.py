"""Micro-benchmark of mit_gemm on the train step's shapes (bf16, random operands)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-image-transformer_amd"))
import torch  # noqa: E402

import native  # noqa: E402

SHAPES = [  # name, M, N, K, a_layout, b_layout
    ("enc qkv", 12608, 2304, 768, 0, 0), ("enc o", 12608, 768, 768, 0, 0), ("enc fc1", 12608, 3072, 768, 0, 0),
    ("enc fc2", 12608, 768, 3072, 0, 0), ("dec kv_all", 12608, 6144, 512, 0, 0), ("dec ffn1", 4032, 2048, 512, 0, 0),
    ("dec fc_out", 4032, 10000, 512, 0, 0), ("dX fc_out", 4032, 512, 10000, 0, 1), ("dW fc_out", 10000, 512, 4032, 1, 1),
    ("dW kv_all", 6144, 512, 12608, 1, 1), ("dX kv_all", 12608, 512, 6144, 0, 1), ("dW ffn1", 2048, 512, 4032, 1, 1),
    ("4096^3", 4096, 4096, 4096, 0, 0),
]


def run(iters=20):
    torch.manual_seed(0)
    dev = torch.device("cuda")
    res = []
    for name, M, N, K, al, bl in SHAPES:
        A = (torch.randn(M, K) if al == 0 else torch.randn(K, M)).to(dev, torch.bfloat16)
        B = (torch.randn(N, K) if bl == 0 else torch.randn(K, N)).to(dev, torch.bfloat16)
        out_f32 = al == 1
        C = torch.empty(M, N, device=dev, dtype=torch.float32 if out_f32 else torch.bfloat16)
        for _ in range(3):
            native.gemm(A, B, C, M, N, K, a_layout=al, b_layout=bl)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            native.gemm(A, B, C, M, N, K, a_layout=al, b_layout=bl)
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / iters * 1e-3
        tf = 2 * M * N * K / t / 1e12
        res.append((name, M, N, K, t * 1e6, tf))
        print(f"{name:12s} {M:6d} {N:6d} {K:6d} {al}{bl}  {t*1e6:9.1f} us  {tf:7.1f} TFLOP/s", flush=True)
    return res


if __name__ == "__main__":
    native.load_library()
    run()
