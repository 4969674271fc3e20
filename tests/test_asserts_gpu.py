"""The diagnostic build with the kernel extent asserts compiled in (common.h MIT_DASSERT, SURVEY.md §5
"kernel bounds asserts behind a flag"; `make -C multimodal-image-transformer_amd/csrc asserts` ->
lib/diag/libmit_hip_asserts.so): every GEMM tile kernel (256, 128 + split-K, register-streaming, f32)
and the attention kernels (head-resident forward, 64-query forward, fused backward) run under it with
ragged extents and return the same results as the shipped build -- no assert fires. Runs in a child
process (the library is loaded once per process, selected by MIT_LIB)."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "multimodal-image-transformer_amd", "lib", "diag", "libmit_hip_asserts.so")

CHILD = r'''
import math, sys, torch
sys.path.insert(0, sys.argv[1])
import native as N
N.load_library()
torch.manual_seed(0)
dev = "cuda"
def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()
for (M, Nn, K, al, bl) in [(520, 776, 200, 0, 0), (1000, 520, 136, 0, 1), (264, 136, 1096, 1, 1), (4032, 512, 2048, 1, 1),
                           (250, 520, 200, 0, 0)]:
    A = torch.randn(M, K) if al == 0 else torch.randn(K, M)
    B = torch.randn(Nn, K) if bl == 0 else torch.randn(K, Nn)
    ref = (A if al == 0 else A.t()) @ (B.t() if bl == 0 else B)
    for v in (0, 1, 2, 3):
        N.gemm_set_variant(v)
        C = torch.empty(M, Nn, device=dev)
        ws = N.gemm_workspace(M, Nn, K, dev)
        N.gemm(A.to(dev, torch.bfloat16), B.to(dev, torch.bfloat16), C, M, Nn, K, a_layout=al, b_layout=bl, workspace=ws)
        assert rel(C.cpu(), ref) < 1e-2, (M, Nn, K, al, bl, v)
    C32 = torch.empty(M, Nn, device=dev)
    N.gemm(A.to(dev), B.to(dev), C32, M, Nn, K, a_layout=al, b_layout=bl)
    assert rel(C32.cpu(), ref) < 1e-5
N.gemm_set_variant(0)
for (Bb, H, Lq, Lk, causal) in [(3, 12, 197, 197, 0), (2, 8, 63, 197, 0), (4, 8, 63, 63, 1)]:
    D = 64
    q = torch.randn(Bb, Lq, H * D, device=dev).to(torch.bfloat16)
    k = torch.randn(Bb, Lk, H * D, device=dev).to(torch.bfloat16)
    v = torch.randn(Bb, Lk, H * D, device=dev).to(torch.bfloat16)
    o = torch.empty_like(q)
    lse = torch.empty(Bb * H * Lq, device=dev)
    a = N.attn_args(q, H * D, Lq * H * D, k, H * D, Lk * H * D, v, H * D, Lk * H * D, o, H * D, Lq * H * D, lse=lse,
                    causal=bool(causal), scale=1 / math.sqrt(D))
    N.attention_fwd(N.BF16, Bb, H, Lq, Lk, a)
    sh = lambda t, L: t.float().reshape(Bb, L, H, D).transpose(1, 2)
    ref = torch.nn.functional.scaled_dot_product_attention(sh(q, Lq), sh(k, Lk), sh(v, Lk), is_causal=bool(causal))
    assert rel(o.float(), ref.transpose(1, 2).reshape(Bb, Lq, H * D)) < 1e-2
    if Lq <= 64:
        do = torch.randn_like(q)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        g = N.attn_grads(do, H * D, Lq * H * D, dq, H * D, Lq * H * D, dk, H * D, Lk * H * D, dv, H * D, Lk * H * D,
                         torch.empty(Bb * H * Lq, device=dev))
        N.attention_bwd(N.BF16, Bb, H, Lq, Lk, a, g)
torch.cuda.synchronize()
print("ASSERTS_OK")
'''


def test_assert_build_runs_clean():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(LIB):
        pytest.skip("asserts build missing (make -C multimodal-image-transformer_amd/csrc asserts)")
    env = dict(os.environ, MIT_LIB=LIB)
    r = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "multimodal-image-transformer_amd")], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "ASSERTS_OK" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
