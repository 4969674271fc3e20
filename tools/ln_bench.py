"""Micro-benchmark of mit_layernorm_fwd on the train step's shapes (bf16): the encoder's pre-LN
(12608 x 768, no residual) and the decoder's post-LN LN(x + dropout(r)) (4032 x 512). Prints us and
TB/s of algorithmic bytes (x [+ r] read, y [+ z] written)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-image-transformer_amd"))
import torch  # noqa: E402

import native  # noqa: E402

SHAPES = [("enc ln 768", 12608, 768, False), ("enc ln 768 +res+drop", 12608, 768, True),
          ("dec ln 512 +res+drop", 4032, 512, True), ("clip ln 1024", 36928, 1024, False), ("ln 256", 16384, 256, False)]


def run(iters=50):
    dev = torch.device("cuda")
    for name, R, C, res in SHAPES:
        x = torch.randn(R, C, device=dev).to(torch.bfloat16)
        r = torch.randn(R, C, device=dev).to(torch.bfloat16) if res else None
        y = torch.empty_like(x)
        z = torch.empty_like(x) if res else None
        g, b = torch.randn(C, device=dev), torch.randn(C, device=dev)
        seed = torch.tensor([5], dtype=torch.int64, device=dev)
        kw = dict(r=r, drop_p=0.1, seed=seed, site=3, z=z) if res else {}
        for _ in range(5):
            native.layernorm_fwd(x, g, b, 1e-5, y, **kw)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            native.layernorm_fwd(x, g, b, 1e-5, y, **kw)
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / iters * 1e-3
        nb = R * C * 2 * (4 if res else 2)
        print(f"{name:22s} {R:6d} x {C:5d}  {t * 1e6:7.2f} us  {nb / t / 1e12:5.2f} TB/s", flush=True)
        if not res:  # the same bytes as a plain device copy (x -> y), for scale
            e0.record()
            for _ in range(iters):
                y.copy_(x)
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / iters * 1e-3
            print(f"{'  copy':22s} {R:6d} x {C:5d}  {t * 1e6:7.2f} us  {nb / t / 1e12:5.2f} TB/s", flush=True)


def run_x32(iters=30):
    """mit_layernorm_fwd_x32 on the CLIP-L/14@336 residual stream (36928 x 1024: z = x + r in place, f32;
    y = LN(z) bf16): us and TB/s of x, r read + z, y written (12 B per element)."""
    dev = torch.device("cuda")
    R, C = 36928, 1024
    x = torch.randn(R, C, device=dev)
    r = torch.randn(R, C, device=dev).to(torch.bfloat16)
    y = torch.empty(R, C, device=dev, dtype=torch.bfloat16)
    g, b = torch.randn(C, device=dev), torch.randn(C, device=dev)
    for _ in range(3):
        native.layernorm_fwd_x32(x, g, b, 1e-5, y, r=r, z=x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        native.layernorm_fwd_x32(x, g, b, 1e-5, y, r=r, z=x)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / iters * 1e-3
    print(f"{'clip ln x32 1024 +res':22s} {R:6d} x {C:5d}  {t * 1e6:7.2f} us  {R * C * 12 / t / 1e12:5.2f} TB/s", flush=True)


def run_bwd(iters=50):
    """mit_layernorm_bwd on the decoder's post-LN shape (4032 x 512, residual dropout, dr written, dgamma /
    dbeta partials left for the side stream): us and TB/s of dy, z read + dx, dr written."""
    dev = torch.device("cuda")
    R, C = 4032, 512
    dy = torch.randn(R, C, device=dev).to(torch.bfloat16)
    z = torch.randn(R, C, device=dev).to(torch.bfloat16)
    dx, dr = torch.empty_like(dy), torch.empty_like(dy)
    mean, rstd = z.float().mean(1), z.float().var(1).add(1e-5).rsqrt()
    g = torch.randn(C, device=dev)
    ws = torch.empty(native.layernorm_bwd_ws_floats(R, C), device=dev)
    seed = torch.tensor([5], dtype=torch.int64, device=dev)
    fn = lambda: native.layernorm_bwd(dy, z, mean, rstd, g, dx, None, None, ws, dr=dr, drop_p=0.1, seed=seed, site=3)  # noqa: E731
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / iters * 1e-3
    print(f"{'dec ln bwd 512 +drop':22s} {R:6d} x {C:5d}  {t * 1e6:7.2f} us  {R * C * 8 / t / 1e12:5.2f} TB/s", flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "x32":
    native.load_library()
    run_x32()
elif __name__ == "__main__":
    native.load_library()
    run()
    run_bwd()
