"""The 256x256 bf16 GEMM tile kernel (gemm.hip gemm256_kernel) against an fp32 torch product and the
128x128 kernel, all four operand layouts, ragged edges, odd K-tile counts, every fused epilogue, and
a race screen (a deterministic kernel must return bit-identical outputs on every repeat)."""
import pytest
import torch
import torch.nn.functional as F

import native as N

pytestmark = pytest.mark.gpu


def dev():
    return torch.device("cuda")


@pytest.fixture(autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    N.load_library()
    yield
    N.gemm_set_variant(0)


def _ops(M, Nn, K, al, bl, seed=0):
    g = torch.Generator().manual_seed(seed)
    A = torch.randn(M, K, generator=g) if al == 0 else torch.randn(K, M, generator=g)
    B = torch.randn(Nn, K, generator=g) if bl == 0 else torch.randn(K, Nn, generator=g)
    A, B = A.to(dev(), torch.bfloat16), B.to(dev(), torch.bfloat16)
    Am = A.float() if al == 0 else A.float().t()
    Bm = B.float().t() if bl == 0 else B.float()
    return A, B, Am @ Bm


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


SHAPES = [(256, 256, 64), (264, 136, 72), (520, 776, 200), (1000, 520, 136), (512, 1024, 768), (2056, 768, 1536)]


@pytest.mark.parametrize("al,bl", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,Nn,K", SHAPES)
def test_gemm256_layouts(al, bl, M, Nn, K):
    A, B, ref = _ops(M, Nn, K, al, bl)
    outs = []
    for v in (2, 1):
        N.gemm_set_variant(v)
        C = torch.empty(M, Nn, device=dev(), dtype=torch.float32)
        N.gemm(A, B, C, M, Nn, K, a_layout=al, b_layout=bl)
        outs.append(C)
    assert _rel(outs[0], ref) < 1e-5, "256 kernel vs fp32 reference"
    assert (outs[0] - outs[1]).abs().max().item() <= 1e-3 * ref.abs().max().item()


def test_gemm256_epilogues():
    M, Nn, K = 600, 520, 200
    N.gemm_set_variant(2)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(M, K, generator=g).to(dev(), torch.bfloat16)
    w = (torch.randn(Nn, K, generator=g) / 10).to(dev(), torch.bfloat16)
    bias = torch.randn(Nn, generator=g).to(dev())
    res = torch.randn(M, Nn, generator=g).to(dev(), torch.bfloat16)
    base = x.float() @ w.float().t()
    for act, fn in [(N.ACT_RELU, F.relu), (N.ACT_GELU, F.gelu), (N.ACT_QUICK_GELU, lambda t: t * torch.sigmoid(1.702 * t))]:
        out = torch.empty(M, Nn, device=dev(), dtype=torch.bfloat16)
        N.linear(x, w, out, bias=bias, act=act, residual=res)
        assert _rel(out, fn(base + bias) + res.float()) < 8e-3
    acc = torch.randn(M, Nn, generator=g).to(dev())
    ref = acc + 0.5 * base
    N.gemm(x, w, acc, M, Nn, K, alpha=0.5, accumulate=True)
    assert _rel(acc, ref) < 1e-5
    seed = torch.tensor([99], dtype=torch.int64, device=dev())
    out = torch.empty(M, Nn, device=dev(), dtype=torch.bfloat16)
    N.linear(x, w, out, bias=bias, act=N.ACT_RELU, drop_p=0.1, seed=seed, site=5)
    mk = torch.empty(M * Nn, device=dev())
    N.dropout_mask(M * Nn, 0.1, seed, 5, mk)
    assert _rel(out, F.relu(base + bias) * mk.view(M, Nn)) < 8e-3


def test_gemm256_rowsum_weight_grad():
    """dW = dY^T X with the fused bias-gradient row sums (TN layout, f32 out)."""
    R, dout, din = 1032, 520, 264
    N.gemm_set_variant(2)
    g = torch.Generator().manual_seed(2)
    dy = torch.randn(R, dout, generator=g).to(dev(), torch.bfloat16)
    x = torch.randn(R, din, generator=g).to(dev(), torch.bfloat16)
    dw = torch.empty(dout, din, device=dev())
    db = torch.empty(dout, device=dev())
    N.gemm(dy, x, dw, dout, din, R, a_layout=N.MN_CONTIG, b_layout=N.MN_CONTIG, rowsum=db)
    assert _rel(dw, dy.float().t() @ x.float()) < 1e-5
    assert _rel(db, dy.float().sum(0)) < 1e-5


@pytest.mark.parametrize("al,bl,M,Nn,K", [(0, 0, 2056, 2304, 768), (0, 1, 1288, 520, 1024), (1, 1, 520, 776, 1096)])
def test_gemm256_race_screen(al, bl, M, Nn, K):
    N.gemm_set_variant(2)
    A, B, ref = _ops(M, Nn, K, al, bl, seed=3)
    C0 = torch.empty(M, Nn, device=dev(), dtype=torch.bfloat16)
    N.gemm(A, B, C0, M, Nn, K, a_layout=al, b_layout=bl)
    assert _rel(C0, ref) < 8e-3
    C = torch.empty_like(C0)
    bad = 0
    for _ in range(30):
        C.fill_(0)
        N.gemm(A, B, C, M, Nn, K, a_layout=al, b_layout=bl)
        bad += int(not torch.equal(C, C0))
    assert bad == 0, f"{bad}/30 repeats differ bitwise (LDS race)"


def test_gemm_gelu_epilogue_accuracy():
    """bf16 GEMM, f32 output, bias + GELU: the branch-free erf of the vector epilogue (gelu_fast)
    against torch's exact-erf GELU of the same fp32 product: |err| ~1e-7 of the scale."""
    M, Nn, K = 512, 776, 256
    g = torch.Generator().manual_seed(5)
    x = torch.randn(M, K, generator=g).to(dev(), torch.bfloat16)
    w = (torch.randn(Nn, K, generator=g) / 8).to(dev(), torch.bfloat16)
    bias = torch.randn(Nn, generator=g).to(dev())
    ref = F.gelu(x.double() @ w.double().t() + bias.double())
    for v in (1, 2):
        N.gemm_set_variant(v)
        out = torch.empty(M, Nn, device=dev())
        N.gemm(x, w, out, M, Nn, K, bias=bias, act=N.ACT_GELU)
        err = (out.double() - ref).abs().max().item()
        assert err < 2e-5 * ref.abs().max().item(), (v, err)


@pytest.mark.parametrize("M,Nn,K", [(4032, 512, 512), (4032, 512, 2048), (256, 10000, 512), (250, 520, 200),
                                    (1000, 136, 1096), (64, 64, 64), (70, 2048, 72)])
def test_register_streaming_kernel(M, Nn, K):
    """The 64x64 register-streaming NT kernel (gemm_rs_kernel, variant 3) against fp32 torch and the
    128 kernel: ragged M / N / K edges, K split over the four waves, every fused epilogue."""
    A, B, ref = _ops(M, Nn, K, 0, 0, seed=M + Nn + K)
    N.gemm_set_variant(3)
    C = torch.empty(M, Nn, device=dev(), dtype=torch.float32)
    N.gemm(A, B, C, M, Nn, K)
    assert _rel(C, ref) < 1e-5
    g = torch.Generator().manual_seed(9)
    bias = torch.randn(Nn, generator=g).to(dev())
    res = torch.randn(M, Nn, generator=g).to(dev(), torch.bfloat16)
    aux = torch.randn(M, Nn, generator=g).to(dev(), torch.bfloat16)
    seed = torch.tensor([7], dtype=torch.int64, device=dev())
    cases = [dict(bias=bias, act=a, residual=res) for a in (N.ACT_RELU, N.ACT_GELU, N.ACT_QUICK_GELU)]
    cases += [dict(bias=bias, act=N.ACT_RELU, drop_p=0.1, seed=seed, site=5), dict(aux=aux, aux_scale=1.5),
              dict(residual=res, aux=aux, aux_scale=2.0)]
    for kw in cases:
        outs = []
        for v in (3, 1):
            N.gemm_set_variant(v)
            out = torch.empty(M, Nn, device=dev(), dtype=torch.bfloat16)
            N.gemm(A, B, out, M, Nn, K, **kw)
            outs.append(out.float())
        scale = outs[1].abs().max().item()
        assert (outs[0] - outs[1]).abs().max().item() <= 1e-2 * max(scale, 1.0), kw
    acc0 = torch.randn(M, Nn, generator=g).to(dev())
    N.gemm_set_variant(3)
    acc = acc0.clone()
    N.gemm(A, B, acc, M, Nn, K, alpha=0.5, accumulate=True)
    assert _rel(acc, acc0 + 0.5 * ref) < 1e-5
    C2 = torch.empty_like(C)
    N.gemm(A, B, C2, M, Nn, K)
    assert torch.equal(C, C2), "register-streaming kernel not deterministic"
