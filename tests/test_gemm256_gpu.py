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
    N.gemm_set_fused_split(0)
    N.gemm_set_persist(0)


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


@pytest.mark.parametrize("al,bl", [(0, 0), (0, 1)])
@pytest.mark.parametrize("M,Nn,K", [(4032, 512, 1536), (4032, 512, 2048), (1000, 520, 3072), (200, 136, 4096)])
@pytest.mark.parametrize("epi", ["plain", "bias_res", "relu_drop", "aux_f32acc", "gelu"])
def test_gemm_split_k_in_launch_combine(al, bl, M, Nn, K, epi):
    """Split-K with the in-launch combine (<= 128 output tiles, any epilogue): equal to the same
    GEMM without a workspace (no split) up to fp32 summation order, bit-identical over repeats
    (the combine sums slabs in slice order whatever the arrival order), counters left at zero."""
    N.gemm_set_fused_split(1)
    A, B, ref = _ops(M, Nn, K, al, bl, seed=M + K)
    g = torch.Generator().manual_seed(3)
    kw = {}
    out_dt = torch.bfloat16
    if epi == "bias_res":
        kw = dict(bias=torch.randn(Nn, generator=g).to(dev()), residual=torch.randn(M, Nn, generator=g).to(dev(), torch.bfloat16))
    elif epi == "relu_drop":
        kw = dict(act=N.ACT_RELU, drop_p=0.25, seed=torch.tensor([11], device=dev()), site=3)
    elif epi == "aux_f32acc":
        kw = dict(aux=torch.randn(M, Nn, generator=g).to(dev(), torch.bfloat16), aux_scale=1.5, accumulate=True)
        out_dt = torch.float32
    elif epi == "gelu":
        kw = dict(act=N.ACT_GELU, bias=torch.randn(Nn, generator=g).to(dev()))
    ws = N.gemm_workspace(M, Nn, K, dev())
    args = N.GemmArgs(N.BF16, al, bl, M, Nn, K, A.data_ptr(), K if al == 0 else M, B.data_ptr(),
                      K if bl == 0 else Nn, 0, Nn, 1.0, None, 0, None, Nn, None, Nn, 1.0, 0.0, None, 0, 0, 0, None,
                      ws.data_ptr(), ws.numel() * 4)
    tile, ks = N.gemm_plan(args)
    assert tile == 128 and ks >= 2, (tile, ks)
    base = torch.randn(M, Nn, generator=g).to(dev(), out_dt)
    outs = []
    for w in (None, ws, ws, ws):
        C = base.clone()
        N.gemm(A, B, C, M, Nn, K, a_layout=al, b_layout=bl, workspace=w, **kw)
        outs.append(C)
    assert torch.equal(outs[1], outs[2]) and torch.equal(outs[1], outs[3])
    assert torch.count_nonzero(ws[:1024]).item() == 0
    d = (outs[1].float() - outs[0].float()).abs().max().item()
    scale = max(outs[0].float().abs().max().item(), 1.0)
    assert d <= (2e-2 if out_dt == torch.bfloat16 else 1e-4) * scale, d



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


@pytest.mark.parametrize("M,Nn,K", [(200, 264, 72), (961, 776, 200), (1000, 768, 3072), (12608, 768, 768)])
@pytest.mark.parametrize("epi", ["plain", "bias_res", "gelu", "f32"])
def test_gemm256_short_tiles_bit_identical(M, Nn, K, epi):
    """160 / 192-row tiles (variants 5 / 6) run the same per-element MFMA K order as the 256-row tile,
    so every epilogue's output is bit-identical, ragged M included."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(M, K, generator=g).to(dev(), torch.bfloat16)
    w = (torch.randn(Nn, K, generator=g) / 10).to(dev(), torch.bfloat16)
    kw = {}
    if epi == "bias_res":
        kw = dict(bias=torch.randn(Nn, generator=g).to(dev()), residual=torch.randn(M, Nn, generator=g).to(dev(), torch.bfloat16))
    elif epi == "gelu":
        kw = dict(bias=torch.randn(Nn, generator=g).to(dev()), act=N.ACT_GELU)
    outs = {}
    for v in (2, 6, 5):
        N.gemm_set_variant(v)
        C = torch.full((M, Nn), float("nan"), device=dev(), dtype=torch.float32 if epi == "f32" else torch.bfloat16)
        N.gemm(x, w, C, M, Nn, K, **kw)
        outs[v] = C
    ref = x.float() @ w.float().t()
    if epi == "plain" or epi == "f32":
        assert _rel(outs[2], ref) < 8e-3
    for v in (6, 5):
        assert torch.equal(outs[v], outs[2]), f"variant {v}"


TALL_SHAPES = [(256, 128, 32), (264, 136, 72), (520, 776, 200), (1000, 520, 136), (2056, 768, 1536), (12608, 2304, 768)]


@pytest.mark.parametrize("M,Nn,K", TALL_SHAPES)
def test_gemm_tall_bit_identical_to_256(M, Nn, K):
    """The two-workgroup 256x128 kernel (gemm_tall_kernel, variant 7) runs every output element's MFMAs
    in the same K order as the 256x256 kernel (32-deep chunks in sequence), so NT outputs are
    bit-identical; and within the fp32 reference's tolerance."""
    A, B, ref = _ops(M, Nn, K, 0, 0, seed=4)
    g = torch.Generator().manual_seed(6)
    bias = torch.randn(Nn, generator=g).to(dev())
    res = torch.randn(M, Nn, generator=g).to(dev(), torch.bfloat16)
    seed = torch.tensor([5], dtype=torch.int64, device=dev())
    cases = [dict(f32=True), dict(bias=bias), dict(bias=bias, act=N.ACT_GELU), dict(residual=res),
             dict(bias=bias, act=N.ACT_RELU, drop_p=0.1, seed=seed, site=3), dict(bias=bias, act=N.ACT_QUICK_GELU)]
    for kw in cases:
        f32 = kw.pop("f32", False)
        outs = []
        for v in (7, 2):
            N.gemm_set_variant(v)
            C = torch.empty(M, Nn, device=dev(), dtype=torch.float32 if f32 else torch.bfloat16)
            N.gemm(A, B, C, M, Nn, K, **kw)
            outs.append(C)
        assert torch.equal(outs[0], outs[1]), (kw.keys(), (outs[0].float() - outs[1].float()).abs().max().item())
        if f32:
            assert _rel(outs[0], ref) < 1e-5


def test_gemm_tall_race_screen():
    N.gemm_set_variant(7)
    M, Nn, K = 4104, 2312, 776
    A, B, ref = _ops(M, Nn, K, 0, 0, seed=7)
    C0 = torch.empty(M, Nn, device=dev(), dtype=torch.bfloat16)
    N.gemm(A, B, C0, M, Nn, K)
    assert _rel(C0, ref) < 8e-3
    C = torch.empty_like(C0)
    bad = 0
    for _ in range(30):
        C.fill_(0)
        N.gemm(A, B, C, M, Nn, K)
        bad += int(not torch.equal(C, C0))
    assert bad == 0, f"{bad}/30 repeats differ bitwise (LDS race)"


@pytest.mark.parametrize("M,Nn,K", [(4104, 4104, 768), (4352, 4096, 200), (12608, 2304, 768)])
def test_gemm256_persistent_bit_identical(M, Nn, K):
    """Multi-round NT grids run on the persistent 256 kernel (gemm256p_kernel: the next tile's first
    K-tile loaded during this tile's two-pass staged epilogue); variant 8 forces the one-tile grid.
    Same K loop and epilogue arithmetic: outputs bit-identical for every epilogue, and repeatable."""
    A, B, ref = _ops(M, Nn, K, 0, 0, seed=8)
    g = torch.Generator().manual_seed(9)
    bias = torch.randn(Nn, generator=g).to(dev())
    res = torch.randn(M, Nn, generator=g).to(dev(), torch.bfloat16)
    seed = torch.tensor([11], dtype=torch.int64, device=dev())
    cases = [dict(), dict(bias=bias), dict(bias=bias, act=N.ACT_GELU), dict(residual=res, bias=bias),
             dict(bias=bias, act=N.ACT_RELU, drop_p=0.1, seed=seed, site=3)]
    N.gemm_set_persist(1)
    for kw in cases:
        outs = []
        for v in (0, 8, 0):
            N.gemm_set_variant(v)
            C = torch.empty(M, Nn, device=dev(), dtype=torch.bfloat16)
            N.gemm(A, B, C, M, Nn, K, **kw)
            outs.append(C)
        assert torch.equal(outs[0], outs[1]), (list(kw), (outs[0].float() - outs[1].float()).abs().max().item())
        assert torch.equal(outs[0], outs[2])
    N.gemm_set_persist(0)
    N.gemm_set_variant(0)
    C = torch.empty(M, Nn, device=dev(), dtype=torch.bfloat16)
    N.gemm(A, B, C, M, Nn, K)
    assert _rel(C, ref) < 8e-3
