"""A/B of the persistent 256x256 GEMM (gemm256p_kernel) against the one-tile-per-workgroup kernel on
the configs[1] step's 256-tile shapes (encoder B*197 = 12608 rows, decoder kv_all / fc_out), with
each launch's real epilogue, interleaved rounds in one process. Usage (GPU box):
python tools/gemm256p_ab.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-image-transformer_amd"))
import torch  # noqa: E402

import native  # noqa: E402

# name, M, N, K, b_layout, epilogue, count per step
SHAPES = [
    ("enc qkv+bias", 12608, 2304, 768, 0, "bias", 12), ("enc o+res", 12608, 768, 768, 0, "res", 12),
    ("enc fc1+gelu", 12608, 3072, 768, 0, "gelu", 12), ("enc fc2+res", 12608, 768, 3072, 0, "res", 12),
    ("dec kv_all", 12608, 6144, 512, 0, "bias", 1), ("dec fc_out", 4032, 10000, 512, 0, "bias", 1),
    ("dX kv_all", 12608, 512, 6144, 1, "plain", 1), ("4096^3", 4096, 4096, 4096, 0, "plain", 0),
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
    native.gemm_set_variant(2)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    tot = [0.0, 0.0]
    print(f"{'shape':14s} {'M':>6s} {'N':>6s} {'K':>6s}  {'1-tile us':>9s} {'TF':>6s}  {'persist us':>10s} {'TF':>6s}  speedup")
    for name, M, N, K, bl, epi, cnt in SHAPES:
        A = torch.randn(M, K, device=dev).to(torch.bfloat16)
        B = (torch.randn(N, K, device=dev) if bl == 0 else torch.randn(K, N, device=dev)).to(torch.bfloat16)
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        kw = {}
        if epi in ("bias", "gelu"):
            kw["bias"] = torch.randn(N, device=dev)
        if epi == "gelu":
            kw["act"] = native.ACT_GELU
        if epi == "res":
            kw["residual"] = torch.randn(M, N, device=dev).to(torch.bfloat16)
        fn = lambda: native.gemm(A, B, C, M, N, K, b_layout=bl, **kw)  # noqa: E731
        ts = [[], []]
        for _ in range(3):
            for p in (0, 1):
                native.gemm_set_persistent(p)
                ts[p].append(timeit(fn))
        t0, t1 = min(ts[0]), min(ts[1])
        tot[0] += cnt * t0
        tot[1] += cnt * t1
        fl = 2.0 * M * N * K
        print(f"{name:14s} {M:6d} {N:6d} {K:6d}  {t0:9.1f} {fl / t0 / 1e6:6.0f}  {t1:10.1f} {fl / t1 / 1e6:6.0f}  {t0 / t1:6.3f}",
              flush=True)
    native.gemm_set_persistent(1)
    print(f"per-step sum (isolated, x count): one-tile {tot[0] / 1e3:.3f} ms, persistent {tot[1] / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
