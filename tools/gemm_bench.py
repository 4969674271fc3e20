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
    ("enc fc1+gelu", 12608, 3072, 768, 0, 0, "gelu"), ("enc fc2+res", 12608, 768, 3072, 0, 0, "res"),
    ("enc o+res+st", 12608, 768, 768, 0, 0, "resst"), ("enc fc2+res+st", 12608, 768, 3072, 0, 0, "resst"),
    ("enc qkv+ln", 12608, 2304, 768, 0, 0, "lnbias"), ("enc fc1+gelu+ln", 12608, 3072, 768, 0, 0, "lngelu"),
    ("enc qkv+bias", 12608, 2304, 768, 0, 0, "bias"), ("enc o+res", 12608, 768, 768, 0, 0, "res"), ("dec ffn1+relu+drop", 4032, 2048, 512, 0, 0, "reludrop"),
    # the d_model = 512 decoder GEMMs (128 output tiles)
    ("fwd out+bias", 4032, 512, 512, 0, 0, "bias"), ("fwd lin2+res", 4032, 512, 2048, 0, 0, "res"),
    ("fwd self_in+bias", 4032, 1536, 512, 0, 0, "bias"), ("fwd lin2+bias", 4032, 512, 2048, 0, 0, "bias"),
    ("dX out", 4032, 512, 512, 0, 1), ("dX q+res", 4032, 512, 512, 0, 1, "res0"),
    ("dX lin1+res", 4032, 512, 2048, 0, 1, "res0"), ("dX self_in+res", 4032, 512, 1536, 0, 1, "res0"),
    ("dX fc_out ws", 4032, 512, 10000, 0, 1, "ws"), ("dW dd ws", 512, 512, 4032, 1, 1, "ws"),
    ("dW ffn ws", 2048, 512, 4032, 1, 1, "ws"),
    # CLIP ViT-L/14 encoder shapes: configs[2] (336 px, 577 tokens) and configs[3] (224 px, 257)
    ("clip o+res", 36928, 1024, 1024, 0, 0, "res"), ("clip fc2+res", 36928, 1024, 4096, 0, 0, "res"),
    ("clip qkv", 36928, 3072, 1024, 0, 0, "bias"), ("clip fc1+gelu", 36928, 4096, 1024, 0, 0, "gelu"), ("clip fc1+qgelu", 36928, 4096, 1024, 0, 0, "qgelu"),
    ("cfg3 o+res", 16448, 1024, 1024, 0, 0, "res"), ("cfg3 fc2+res", 16448, 1024, 4096, 0, 0, "res"),
    # epilogue-concurrency probes (tools/g256_stamps.py): 8 / 64 / 128 tiles of the encoder's K = 768
    ("iso8", 2048, 256, 768, 0, 0), ("iso8 res", 2048, 256, 768, 0, 0, "res"), ("iso64", 2048, 2048, 768, 0, 0),
    ("iso128", 4096, 2048, 768, 0, 0),
]


def run(iters=20, variants=(1, 2)):
    torch.manual_seed(0)
    dev = torch.device("cuda")
    res = []
    only = os.environ.get("GEMM_SHAPES")
    for name, M, N, K, al, bl, *epi in SHAPES:
        if only and name not in only.split(",") and name.replace(" ", "_") not in only.split(","):  # "_" for " "
            continue
        epi = epi[0] if epi else ""
        A = (torch.randn(M, K) if al == 0 else torch.randn(K, M)).to(dev, torch.bfloat16)
        B = (torch.randn(N, K) if bl == 0 else torch.randn(K, N)).to(dev, torch.bfloat16)
        out_f32 = al == 1
        C = torch.empty(M, N, device=dev, dtype=torch.float32 if out_f32 else torch.bfloat16)
        kw = {}
        ws = native.gemm_workspace(M, N, K, dev)  # as the train step passes it (split-K when planned)
        if epi == "ws":
            pass
        elif epi == "res0":
            kw["residual"] = torch.randn(M, N, device=dev).to(torch.bfloat16)
        elif epi:
            kw["bias"] = torch.randn(N, device=dev)
        if epi in ("gelu", "lngelu"):
            kw["act"] = native.ACT_GELU
        if epi.startswith("ln"):  # the LayerNorm-folded encoder GEMMs (qkv, fc1): (mean, M2) per 64 columns of A
            mean = 0.1 * torch.randn(M, K // 64, device=dev)
            m2 = 64.0 * (0.5 + torch.rand(M, K // 64, device=dev))
            kw.update(ln_stats=torch.stack([mean, m2], -1).contiguous(), ln_colsum=torch.randn(N, device=dev), ln_eps=1e-5)
        if epi == "qgelu":
            kw["act"] = native.ACT_QUICK_GELU
        if epi in ("res", "resst"):
            kw["residual"] = torch.randn(M, N, device=dev).to(torch.bfloat16)
        if epi == "resst":  # + the output rows' per-64-column (mean, M2): the folded encoder's o-proj / fc2
            kw["stats_out"] = torch.empty(M, N // 64, 2, device=dev)
        if epi == "reludrop":
            kw.update(act=native.ACT_RELU, drop_p=0.1, seed=torch.tensor([7], device=dev), site=1)
        best = {}
        for rnd in range(3):  # interleaved rounds, one process (guide §5.4 rule 24)
            for v in variants:  # "<variant>" with the workspace, "<variant>n" without (no split-K)
                native.gemm_set_variant(int(v.rstrip("n")))
                kv = dict(kw, workspace=None if v.endswith("n") else ws)
                for _ in range(3):
                    native.gemm(A, B, C, M, N, K, a_layout=al, b_layout=bl, **kv)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(iters):
                    native.gemm(A, B, C, M, N, K, a_layout=al, b_layout=bl, **kv)
                e1.record()
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1) / iters * 1e-3
                best[v] = min(best.get(v, 1e9), t)
        line = f"{name:12s} {M:6d} {N:6d} {K:6d} {al}{bl}"
        for v in variants:
            t = best[v]
            tf = 2 * M * N * K / t / 1e12
            res.append((name, v, M, N, K, t * 1e6, tf))
            line += f"  v{v:3s} {t*1e6:8.1f} us {tf:7.1f} TF"
        print(line, flush=True)
    native.gemm_set_variant(0)
    return res


if __name__ == "__main__":
    native.load_library()
    vs = tuple(sys.argv[1].split(",")) if len(sys.argv) > 1 else ("1", "2")
    run(variants=vs)
