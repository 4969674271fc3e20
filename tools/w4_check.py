"""Prototype check: the one-wave-per-SIMD 256x256 kernel (mit_gemm_set_variant(4)) against gemm256_kernel
(variant 0, tiles=256) on the same operands -- bitwise equal outputs expected (same MFMAs, same K order) -- for
plain / bias / GELU / quick_gelu / LayerNorm-folded epilogues, ragged M / N, K tails."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-image-transformer_amd"))
import torch  # noqa: E402

import native as N  # noqa: E402


def run(M, Nn, K, kind, seed=0):
    torch.manual_seed(seed)
    dev = torch.device("cuda")
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    B = (0.05 * torch.randn(Nn, K, device=dev)).to(torch.bfloat16)
    kw = {}
    if kind != "plain":
        kw["bias"] = torch.randn(Nn, device=dev)
    if kind in ("gelu", "lngelu"):
        kw["act"] = N.ACT_GELU
    if kind == "qgelu":
        kw["act"] = N.ACT_QUICK_GELU
    if kind == "resst":  # residual + per-64-column row statistics (STG 4)
        kw["residual"] = torch.randn(M, Nn, device=dev).to(torch.bfloat16)
    if kind.startswith("ln"):
        mean = 0.1 * torch.randn(M, K // 64, device=dev)
        m2 = 64.0 * (0.5 + torch.rand(M, K // 64, device=dev))
        kw.update(ln_stats=torch.stack([mean, m2], -1).contiguous(), ln_colsum=torch.randn(Nn, device=dev), ln_eps=1e-5)
    outs, stats = [], []
    for v in (0, 4):
        N.gemm_set_variant(v)
        C = torch.full((M, Nn), float("nan"), device=dev, dtype=torch.bfloat16)
        st = torch.full((M, Nn // 64, 2), float("nan"), device=dev) if kind == "resst" else None
        N.gemm(A, B, C, M, Nn, K, tiles=256, stats_out=st, **kw)
        torch.cuda.synchronize()
        outs.append(C)
        stats.append(st)
    N.gemm_set_variant(0)
    same = torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))
    if kind == "resst":
        same = same and torch.equal(stats[0].view(torch.int32), stats[1].view(torch.int32))
    ref = (A.float() @ B.float().t())
    err = (outs[1].float() - outs[0].float()).abs().max().item()
    print(f"{M:6d} {Nn:6d} {K:6d} {kind:7s} bitwise {'EQUAL' if same else 'DIFF'} maxdiff {err:.3g} "
          f"nan {torch.isnan(outs[1].float()).sum().item()}", flush=True)
    return same


if __name__ == "__main__":
    N.load_library()
    ok = True
    for M, Nn, K, kind in [(512, 512, 256, "plain"), (4096, 4096, 4096, "plain"), (12608, 3072, 768, "gelu"),
                           (12608, 2304, 768, "bias"), (12608, 3072, 768, "lngelu"), (12608, 2304, 768, "lnbias"),
                           (1000, 776, 200, "bias"), (300, 264, 1000, "qgelu"), (12608, 6144, 512, "bias"),
                           (256, 256, 64, "plain"), (257, 512, 128, "gelu"), (12608, 768, 768, "resst"),
                           (12608, 768, 3072, "resst"), (1000, 512, 256, "resst")]:
        ok &= run(M, Nn, K, kind)
    print("ALL EQUAL" if ok else "MISMATCH")
    sys.exit(0 if ok else 1)
