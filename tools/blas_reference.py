"""Per-shape GEMM time: mit_gemm (our kernels) vs torch.matmul (hipBLASLt, the vendor library as a
known-good reference on the same device; guide §5.4 rule 10), bf16, random operands, interleaved
rounds in one process. Shapes = the configs[1] train step's GEMMs (encoder B*197 = 12608 rows,
decoder B*T = 4032 rows); --clip336: the configs[2] step's CLIP-L/14@336 shapes.
Usage (GPU box): python tools/blas_reference.py [--clip336]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-image-transformer_amd"))
import torch  # noqa: E402

import native  # noqa: E402

# name, M, N, K, a_layout, b_layout (0 = K-contig, 1 = MN-contig), count per step ("dec1": one
# token step of the configs[4] batched decode, B = 256 rows; not part of the train-step sum)
SHAPES = [
    ("enc qkv", 12608, 2304, 768, 0, 0, 12), ("enc o+res", 12608, 768, 768, 0, 0, 12),
    ("enc fc1+gelu", 12608, 3072, 768, 0, 0, 12), ("enc fc1 plain", 12608, 3072, 768, 0, 0, 0), ("enc fc2+res", 12608, 768, 3072, 0, 0, 12),
    ("dec kv_all", 12608, 6144, 512, 0, 0, 1), ("dec self_in", 4032, 1536, 512, 0, 0, 6),
    ("dec d-out", 4032, 512, 512, 0, 0, 18), ("dec ffn1", 4032, 2048, 512, 0, 0, 6),
    ("dec ffn2", 4032, 512, 2048, 0, 0, 6), ("dec fc_out", 4032, 10000, 512, 0, 0, 1),
    ("dX d-out", 4032, 512, 512, 0, 1, 18), ("dX ffn1", 4032, 512, 2048, 0, 1, 6),
    ("dX ffn2", 4032, 2048, 512, 0, 1, 6), ("dX self_in", 4032, 512, 1536, 0, 1, 6),
    ("dX fc_out", 4032, 512, 10000, 0, 1, 1), ("dX kv_all", 12608, 512, 6144, 0, 1, 1),
    ("dW d-d", 512, 512, 4032, 1, 1, 18), ("dW ffn1", 2048, 512, 4032, 1, 1, 6),
    ("dW ffn2", 512, 2048, 4032, 1, 1, 6), ("dW self_in", 1536, 512, 4032, 1, 1, 6),
    ("dW fc_out", 10000, 512, 4032, 1, 1, 1), ("dW kv_all", 6144, 512, 12608, 1, 1, 1),
    ("dec1 self_in", 256, 1536, 512, 0, 0, 6), ("dec1 d-out", 256, 512, 512, 0, 0, 18),
    ("dec1 ffn1", 256, 2048, 512, 0, 0, 6), ("dec1 ffn2", 256, 512, 2048, 0, 0, 6),
    ("dec1 fc_out", 256, 10000, 512, 0, 0, 1),
    ("4096^3", 4096, 4096, 4096, 0, 0, 0),
]
# configs[2]: CLIP ViT-L/14@336 (577 tokens, E = 1024, mlp 4096, 24 layers; f32 residual stream, so the
# o-proj / fc2 GEMMs write the bf16 sublayer output with a bias and no residual) + the 6L d512 decoder with
# S = 577 memory rows (B * S = 36928)
CLIP_SHAPES = [
    ("clip qkv+bias", 36928, 3072, 1024, 0, 0, 24), ("clip o+bias", 36928, 1024, 1024, 0, 0, 24),
    ("clip fc1+qgelu", 36928, 4096, 1024, 0, 0, 24), ("clip fc2+bias", 36928, 1024, 4096, 0, 0, 24),
    ("clip patch", 36864, 1024, 592, 0, 0, 1),
    ("proj 1024->512", 36928, 512, 1024, 0, 0, 1), ("dec kv_all577", 36928, 6144, 512, 0, 0, 1),
    ("dX kv_all577", 36928, 512, 6144, 0, 1, 1), ("dW kv_all577", 6144, 512, 36928, 1, 1, 1),
    ("dW proj577", 512, 1024, 36928, 1, 1, 1),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters  # us


def main():
    native.load_library()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    tot_ours = tot_blas = 0.0
    print(f"{'shape':14s} {'M':>6s} {'N':>6s} {'K':>6s}  {'ours us':>8s} {'TF':>6s}  {'hipBLASLt us':>12s} {'TF':>6s}  ratio")
    shapes = CLIP_SHAPES if "--clip336" in sys.argv else SHAPES
    for name, M, N, K, al, bl, cnt in shapes:
        A = (torch.randn(M, K) if al == 0 else torch.randn(K, M)).to(dev, torch.bfloat16)
        B = (torch.randn(N, K) if bl == 0 else torch.randn(K, N)).to(dev, torch.bfloat16)
        out_f32 = al == 1
        C = torch.empty(M, N, device=dev, dtype=torch.float32 if out_f32 else torch.bfloat16)
        ws = native.gemm_workspace(M, N, K, dev)
        kw = {}
        if "res" in name:
            kw["residual"] = torch.randn(M, N, device=dev).to(torch.bfloat16)
        if "qgelu" in name:
            kw["act"] = native.ACT_QUICK_GELU
        elif "gelu" in name:
            kw["act"] = native.ACT_GELU
        if "bias" in name or "qgelu" in name:
            kw["bias"] = torch.randn(N, device=dev)
        ours = lambda: native.gemm(A, B, C, M, N, K, a_layout=al, b_layout=bl, workspace=ws, **kw)  # noqa: E731
        At = A if al == 0 else A.t()
        Bt = B.t() if bl == 0 else B
        blas = lambda: torch.matmul(At, Bt)  # noqa: E731
        to, tb = [], []
        for _ in range(3):  # interleaved rounds
            to.append(timeit(ours))
            tb.append(timeit(blas))
        to, tb = min(to), min(tb)
        fl = 2.0 * M * N * K
        if not name.startswith("dec1"):
            tot_ours += cnt * to
            tot_blas += cnt * tb
        print(f"{name:14s} {M:6d} {N:6d} {K:6d}  {to:8.1f} {fl / to / 1e6:6.0f}  {tb:12.1f} {fl / tb / 1e6:6.0f}  {tb / to:5.2f}",
              flush=True)
    print(f"per-step GEMM sum (isolated, x count): ours {tot_ours / 1e3:.3f} ms, hipBLASLt {tot_blas / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
