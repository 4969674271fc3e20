"""Micro-benchmark of mit_attention_bwd on the decoder's training shapes (bf16, dropout 0.1):
self-attention (63 x 63, causal + key-PAD mask, 8 heads) and cross-attention (63 queries x 197
patches). Run under rocprofv3 --kernel-trace --stats for the dQ / dKV kernel split."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-image-transformer_amd"))
import torch  # noqa: E402

import native  # noqa: E402


def run(iters=20):
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    B, H, T, S, d = 64, 8, 63, 197, 512
    seed = torch.tensor([123], device=dev)
    tok = torch.randint(4, 1000, (B, T), generator=g).to(dev)
    for name, causal, Lk in (("self", True, T), ("cross", False, S)):
        q = torch.randn(B, T, d, generator=g).to(dev, torch.bfloat16)
        kv = torch.randn(B, Lk, 2 * d, generator=g).to(dev, torch.bfloat16)
        o = torch.empty(B, T, d, device=dev, dtype=torch.bfloat16)
        lse = torch.empty(B * H * T, device=dev)
        a = native.attn_args(q, d, T * d, kv, 2 * d, Lk * 2 * d, kv[..., d:], 2 * d, Lk * 2 * d, o, d, T * d, lse=lse,
                             key_tokens=tok if causal else None, tok_batch=T, causal=causal, scale=0.125, drop_p=0.1,
                             seed=seed, site=3)
        native.attention_fwd(native.BF16, B, H, T, Lk, a)
        do = torch.randn(B, T, d, generator=g).to(dev, torch.bfloat16)
        dq = torch.empty_like(q)
        dkv = torch.empty_like(kv)
        delta = torch.empty(B * H * T, device=dev)
        gr = native.attn_grads(do, d, T * d, dq, d, T * d, dkv, 2 * d, Lk * 2 * d, dkv[..., d:], 2 * d, Lk * 2 * d, delta)
        for _ in range(3):
            native.attention_bwd(native.BF16, B, H, T, Lk, a, gr)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            native.attention_bwd(native.BF16, B, H, T, Lk, a, gr)
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / iters * 1e-3
        fl = 8.0 * B * H * T * Lk * 64  # dS/dP (2) + dQ, dK, dV (3) ... counted as 2x the forward's 4*Lq*Lk*d
        print(f"bwd {name:6s} B={B} H={H} Lq={T} Lk={Lk}  {t * 1e6:8.1f} us  {fl / t / 1e12:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    native.load_library()
    run()
