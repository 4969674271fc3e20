"""Micro-benchmark of mit_decode_gemm on the configs[4] token-step shapes (B = 256 rows, d 512, ff 2048):
per-launch time of back-to-back launches, warm (one weight matrix) and cycling through 12 weight matrices
(the 6 layers x 2 of a step: weights not L2-resident). Prints us per launch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-image-transformer_amd"))
import torch  # noqa: E402

import native  # noqa: E402


def main(iters=200):
    native.load_library()
    dev = torch.device("cuda")
    M, d, F = 256, 512, 2048
    bf = lambda *s: torch.randn(*s, device=dev).to(torch.bfloat16)  # noqa: E731
    z = torch.randn(M, d, device=dev)
    st = torch.rand(M, d // 64, 2, device=dev) + 0.5
    gam, bet = torch.ones(d, device=dev), torch.zeros(d, device=dev)
    zo = torch.empty(M, d, device=dev)
    so = torch.empty(M, d // 64, 2, device=dev)
    a16, h16 = bf(M, d), bf(M, F)
    out = {n: torch.empty(M, n, device=dev, dtype=torch.bfloat16) for n in (d, 3 * d, F)}
    shapes = {
        "out-proj +res-LN (N 512, K 512)": lambda w: native.decode_gemm(a16, w, bias=gam, residual=z, r_ln=(st, gam, bet),
                                                                         z_out=zo, stats_out=so),
        "cross-q LN-operand (N 512, K 512)": lambda w: native.decode_gemm(z, w, out=out[d], bias=gam, a_ln=(st, gam, bet)),
        "linear1 LN+relu (N 2048, K 512)": lambda w: native.decode_gemm(z, w, out=out[F], bias=torch.zeros(F, device=dev),
                                                                         act=native.ACT_RELU, a_ln=(st, gam, bet)),
        "linear2 +res-LN (N 512, K 2048)": lambda w: native.decode_gemm(h16, w, bias=gam, residual=z, r_ln=(st, gam, bet),
                                                                         z_out=zo, stats_out=so),
    }
    wshape = {"out-proj +res-LN (N 512, K 512)": (d, d), "cross-q LN-operand (N 512, K 512)": (d, d),
              "linear1 LN+relu (N 2048, K 512)": (F, d), "linear2 +res-LN (N 512, K 2048)": (d, F)}
    # the vocabulary head (V = 10000): the folded greedy argmax vs a plain bf16 output, and mit_gemm's kernel
    V = 10000
    keys = torch.zeros(native.ARGMAX_SLOTS * M, dtype=torch.int64, device=dev)
    bv = torch.zeros(V, device=dev)
    lg = torch.empty(M, V, device=dev, dtype=torch.bfloat16)
    shapes["head argmax_keys (N 10000, K 512)"] = lambda w: native.decode_gemm(a16, w, bias=bv, argmax_keys=keys)
    shapes["head bf16 out (N 10000, K 512)"] = lambda w: native.decode_gemm(a16, w, out=lg, bias=bv)
    shapes["head mit_gemm bf16 (N 10000, K 512)"] = lambda w: native.gemm(a16, w, lg, M, V, d, bias=bv)
    for k in ("head argmax_keys (N 10000, K 512)", "head bf16 out (N 10000, K 512)", "head mit_gemm bf16 (N 10000, K 512)"):
        wshape[k] = (V, d)
    only = os.environ.get("DG_SHAPES")
    for name, fn in shapes.items():
        if only and not any(o in name for o in only.split(",")):
            continue
        ws = [bf(*wshape[name]) for _ in range(12)]
        for mode in ("warm", "12 weights"):
            for i in range(10):
                fn(ws[0] if mode == "warm" else ws[i % 12])
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(iters):
                fn(ws[0] if mode == "warm" else ws[i % 12])
            e1.record()
            torch.cuda.synchronize()
            print(f"{name:36s} {mode:10s} {e0.elapsed_time(e1) / iters * 1e3:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
