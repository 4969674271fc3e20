"""Long-dispatch clock / MFMA-busy calibration (MI355X_MICROARCH.md: GRBM_GUI_ACTIVE / 8 / wall reads high
on dispatches shorter than ~0.3 ms and is within 3 % of the in-kernel clock at >= 10 ms). Runs the
step's GEMM kernels on shapes long enough for that: the 256-tile kernel (plain NT, and the fc1+GELU
epilogue), the 128-tile kernel (variant 1) and the one-wave 256 kernel (variant 4), each dispatch ~5-15 ms, so a rocprofv3 pass with
SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES / GRBM_GUI_ACTIVE over this script gives their clock under
sustained MFMA load (tools/rocpd_summary.py --sq condenses it). Prints TFLOP/s per dispatch.
Usage: python tools/clock_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-image-transformer_amd"))
import torch  # noqa: E402

import native  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    M, N, K = 131072, 6144, 4096
    A = (torch.randn(M, K, device=dev) * 0.1).to(torch.bfloat16)
    B = (torch.randn(N, K, device=dev) * 0.1).to(torch.bfloat16)
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    bias = torch.zeros(N, device=dev)
    cases = [("256 plain", 0, {}), ("256 gelu", 0, {"bias": bias, "act": native.ACT_GELU}), ("128 plain", 1, {}),
             ("256w plain", 4, {})]  # variant 4: the one-wave-per-SIMD 256 kernel (gemm256w_kernel)
    # touch C's 1.6 GB once (the first GEMM into a fresh allocation paid its first-touch cost: round 6 read
    # 1.64 GHz for the first 256-kernel case, 1.90 once warm) and warm the chip up with hipBLASLt GEMMs (kernels
    # the pass does not summarise)
    C.zero_()
    Aw = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    for _ in range(400):
        torch.matmul(Aw, Aw)
    torch.cuda.synchronize()
    del Aw
    # run order: the 128 kernel first -- it absorbs the clock ramp of a freshly started run (the 256 kernel measured
    # first read 1.65-1.76 GHz, 1.87-1.94 once warm; interleaved A/B: profiles/r06_gemm256w_ab.txt)
    order = os.environ.get("CLOCK_CASES", "2,0,1,3")  # case indices in run order
    cases = [cases[int(i)] for i in order.split(",")]
    for name, variant, kw in cases:
        native.gemm_set_variant(variant)
        for it in range(4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            native.gemm(A, B, C, M, N, K, **kw)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if it:
                print(f"{name}: {dt * 1e3:.2f} ms {2 * M * N * K / dt / 1e12:.0f} TFLOP/s", flush=True)
    native.gemm_set_variant(0)


if __name__ == "__main__":
    main()
