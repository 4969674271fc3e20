"""Where a gemm256_kernel launch spends its time, from in-kernel clock stamps.

Needs the diagnostic build (`tools/build_variants.sh stamp -DMIT_G256_STAMP`, run with
MIT_LIB=multimodal-image-transformer_amd/lib/variants/libmit_hip_stamp.so). For each shape: warm launches, then one
stamped launch; per workgroup the shader-clock phases (prologue = entry -> first K-tile resident,
K loop, epilogue = loop end -> stores drained) and, on the 100 MHz global clock, when the tile started
and ended relative to the first workgroup's start. Prints medians / quantiles per phase and the
effective clock. Usage: python tools/g256_stamps.py [shape names as in tools/gemm_bench.py]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-image-transformer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

import native  # noqa: E402
from gemm_bench import SHAPES  # noqa: E402

SLOTS = 24


def stamped(lib, fn, nblk):
    lib.mit_g256_stamps_clear()
    torch.cuda.synchronize()
    fn()
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (nblk * SLOTS))()
    assert lib.mit_g256_stamps(buf, ctypes.c_long(nblk * SLOTS)) == 0
    return np.frombuffer(buf, dtype=np.uint64).reshape(nblk, SLOTS).astype(np.float64)


def q(x):
    return f"med {np.median(x):7.2f} p10 {np.percentile(x, 10):7.2f} p90 {np.percentile(x, 90):7.2f}"


def main(names):
    lib = native.load_library()
    lib.mit_g256_stamps.argtypes = [ctypes.c_void_p, ctypes.c_long]
    dev = torch.device("cuda")
    torch.manual_seed(0)
    native.gemm_set_variant(2)  # the 256 kernel wherever it has an instance (small probe grids too)
    for name, M, N, K, al, bl, *epi in SHAPES:
        if names and name.replace(" ", "_") not in names and name not in names:
            continue
        epi = epi[0] if epi else ""
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        kw = {}
        if epi in ("bias", "gelu"):
            kw["bias"] = torch.randn(N, device=dev)
        if epi == "gelu":
            kw["act"] = native.ACT_GELU
        if epi == "res":
            kw["residual"] = torch.randn(M, N, device=dev).to(torch.bfloat16)

        def fn():
            native.gemm(A, B, C, M, N, K, **kw)

        for _ in range(20):
            fn()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(20):
            fn()
        t1.record()
        torch.cuda.synchronize()
        ev_us = t0.elapsed_time(t1) / 20 * 1000
        nblk = ((M + 255) // 256) * ((N + 255) // 256)
        s = stamped(lib, fn, nblk)
        rt0, mt0, mt1, mt2, mt3, xcc = (s[:, i] for i in range(6))
        rt_end = s[:, 12]
        w4 = s[:, 7:11]
        ghz = (mt3 - mt0) / ((rt_end - rt0) * 10.0)  # shader cycles per ns
        clk = np.median(ghz)
        to_us = lambda cyc: cyc / clk / 1000.0  # noqa: E731
        start = (rt0 - rt0.min()) / 100.0  # us on the global clock
        end = (rt_end - rt0.min()) / 100.0
        flop = 2.0 * M * N * K
        print(f"\n== {name}: M={M} N={N} K={K} {epi or 'plain'}  blocks {nblk}  event {ev_us:.1f} us "
              f"({flop / ev_us / 1e6:.0f} TF)  stamped span {end.max():.1f} us  clock {clk:.2f} GHz")
        print(f"  prologue  (us) {q(to_us(mt1 - mt0))}")
        print(f"  K loop    (us) {q(to_us(mt2 - mt1))}  per K-step {np.median(to_us(mt2 - mt1)) / ((K + 63) // 64):.3f}")
        print(f"  epilogue  (us) {q(to_us(mt3 - mt2))}")
        print(f"  epilogue issue (loop end -> last store issued, us) {q(to_us(s[:, 13] - mt2))}  "
              f"wave4 {q(to_us(s[:, 14] - w4[:, 2]))}")
        print(f"  wave4 loop-end lag vs wave0 (us) {q(to_us(w4[:, 2] - w4[:, 0] - (mt2 - mt0)))}")
        print(f"  tile total(us) {q(end - start)}")
        if s[:, 15].any():  # LDS-staged epilogue checkpoints (wave 0)
            pts = [mt2] + [s[:, k] for k in range(15, 20)] + [s[:, 13]]
            names = ["realign", "stage0", "pass0 stores issued", "barrier", "stage1", "pass1 stores issued"]
            print("  epilogue steps (us): " + ", ".join(f"{n} {np.median(to_us(b - a)):.2f}"
                                                     for n, a, b in zip(names, pts[:-1], pts[1:])))
        order = np.argsort(start)
        rounds = int(np.ceil(nblk / 256))
        for r in range(rounds):
            idx = order[r * 256:(r + 1) * 256]
            print(f"  round {r}: {len(idx)} tiles start {start[idx].min():6.1f}..{start[idx].max():6.1f} "
                  f"end {end[idx].min():6.1f}..{end[idx].max():6.1f} us  prologue med "
                  f"{np.median(to_us(mt1 - mt0)[idx]):5.2f}  epilogue med {np.median(to_us(mt3 - mt2)[idx]):5.2f}")
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        np.savez(os.path.join(ROOT, "gpurun_out", f"stamps_{name.replace(' ', '_').replace('^', '')}.npz"), s=s)
        print(f"  xcc histogram {np.bincount(xcc.astype(int), minlength=8).tolist()}")


if __name__ == "__main__":
    main(sys.argv[1:])
