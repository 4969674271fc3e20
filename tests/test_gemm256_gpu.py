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


@pytest.mark.parametrize("r", [1, 63, 64, 65, 127, 128, 129, 191, 192, 193, 255])
def test_gemm256_ragged_last_row_tile(r):
    """The last row tile with r live rows of 256 (each wave group's 64-row halves live, partly live or
    dead): every epilogue form against fp32 torch, and nothing written past row M (sentinel rows after
    the output)."""
    M, Nn, K = 256 + r, 520, 200
    N.gemm_set_variant(2)
    g = torch.Generator().manual_seed(r)
    x = torch.randn(M, K, generator=g).to(dev(), torch.bfloat16)
    w = (torch.randn(Nn, K, generator=g) / 10).to(dev(), torch.bfloat16)
    bias = torch.randn(Nn, generator=g).to(dev())
    res = torch.randn(M, Nn, generator=g).to(dev(), torch.bfloat16)
    base = x.float() @ w.float().t()
    sentinel = -12288.0  # exact in bf16

    def buf(dtype):
        b = torch.full((M + 64, Nn), sentinel, device=dev(), dtype=dtype)
        return b, b[:M]

    whole, out = buf(torch.float32)
    N.gemm(x, w, out, M, Nn, K)
    assert _rel(out, base) < 1e-5
    assert (whole[M:] == sentinel).all()
    for act, fn in [(N.ACT_GELU, F.gelu), (N.ACT_QUICK_GELU, lambda t: t * torch.sigmoid(1.702 * t))]:
        whole, out = buf(torch.bfloat16)
        N.linear(x, w, out, bias=bias, act=act)
        assert _rel(out, fn(base + bias)) < 8e-3
        assert (whole[M:].float() == sentinel).all()
    whole, out = buf(torch.bfloat16)
    N.linear(x, w, out, bias=bias, residual=res)
    assert _rel(out, base + bias + res.float()) < 8e-3
    assert (whole[M:].float() == sentinel).all()


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
    """bf16 GEMM, f32 output, bias + GELU: the one-exp GELU of the vector epilogue (gelu_fast2, relative
    error <= 6.6e-6, tools/gelu_fit.py) against torch's exact-erf GELU of the same fp32 product."""
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


def test_gemm_gelu_epilogue_extremes():
    """The one-exp GELU past its fit range (common.h gelu_fast / gelu_fast2): +inf -> +inf (not inf - inf),
    -inf and large negative -> 0 within 5.9e-9 (the correction term is capped at 6 Phi(-6), it does not grow
    with |x|), large positive -> x, NaN -> NaN. Injected through the bias columns, f32 and bf16 outputs, on
    the 128 kernel's vector epilogue (variant 1) and the 256 kernel's staged one (variant 2)."""
    M, Nn, K = 512, 776, 256
    g = torch.Generator().manual_seed(6)
    x = torch.randn(M, K, generator=g).to(dev(), torch.bfloat16)
    w = (torch.randn(Nn, K, generator=g) / 8).to(dev(), torch.bfloat16)
    special = [float("inf"), float("-inf"), float("nan"), -1000.0, 1000.0, -1e30, 1e30]
    moderate = [-7.0, 7.0, -6.0, 6.0, -6.5, 6.5]  # checked against the reference with the other columns
    bias = torch.randn(Nn, generator=g) * 0.1
    cols = list(range(3, 3 + 8 * len(special), 8))
    for c, b in zip(cols, special):
        bias[c] = b
    for i, b in enumerate(moderate):
        bias[500 + 8 * i] = b
    bias = bias.to(dev())
    rest = [c for c in range(Nn) if c not in cols]
    ref = F.gelu(x.double() @ w.double().t() + bias.double()).cpu()[:, rest]
    for v in (1, 2):
        N.gemm_set_variant(v)
        for odt in (torch.float32, torch.bfloat16):
            out = torch.empty(M, Nn, device=dev(), dtype=odt)
            N.gemm(x, w, out, M, Nn, K, bias=bias, act=N.ACT_GELU)
            o = out.double().cpu()
            for c, b in zip(cols, special):
                col = o[:, c]
                if b != b:
                    assert torch.isnan(col).all(), (v, odt, b)
                elif b == float("inf") or b == 1e30:
                    assert (col == torch.tensor(b).to(odt).double()).all(), (v, odt, b)
                elif b > 0:
                    assert ((col - b).abs() <= 16).all(), (v, odt, b)
                else:  # -inf, -1e30, -1000: GELU -> 0; the capped correction leaves at most 5.9e-9
                    assert (col.abs() <= 6e-9).all() and not torch.isnan(col).any(), (v, odt, b, col.abs().max())
            tol = 1e-2 if odt == torch.bfloat16 else 2e-5
            assert (o[:, rest] - ref).abs().max().item() < tol * ref.abs().max().item(), (v, odt)


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


def _stats64_ref(y):
    """per-64-column (mean, M2) of each row, float64"""
    R, C = y.shape
    t = y.double().view(R, C // 64, 64)
    m = t.mean(-1)
    return torch.stack([m, ((t - m[..., None]) ** 2).sum(-1)], -1)


def test_row_stats64_matches_torch():
    R, C = 1003, 768
    x = (3 * torch.randn(R, 2 * C, device=dev()) + 1).to(torch.bfloat16)
    st = torch.empty(R, C // 64, 2, device=dev())
    N.row_stats64(x, st, rows=R, cols=C, ldx=2 * C)
    ref = _stats64_ref(x[:, :C])
    assert (st.double() - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()


@pytest.mark.parametrize("act", [0, 2])
@pytest.mark.parametrize("M,Nn,K", [(1000, 2304, 768), (12608, 3072, 768), (300, 520, 256)])
def test_gemm_layernorm_fold(M, Nn, K, act):
    """LN(x) W^T + b computed as rstd (x (W o gamma)^T - mean colsum) + (b + W beta) in the 256 kernel's
    epilogue (encoder.fold_layernorm + mit_gemm ln_stats) against float64 torch; no less accurate than the
    LayerNorm kernel -> bf16 -> GEMM sequence it replaces."""
    import torch.nn.functional as F
    from encoder import fold_layernorm
    torch.manual_seed(M + Nn)
    x = (2 * torch.randn(M, K, device=dev()) + 0.5 * torch.randn(K, device=dev())).to(torch.bfloat16)
    W = torch.randn(Nn, K) / K ** 0.5
    b, gamma, beta = 0.1 * torch.randn(Nn), 1 + 0.2 * torch.randn(K), 0.1 * torch.randn(K)
    wf, bf, sf = fold_layernorm(W, b, gamma, beta)
    st = torch.empty(M, K // 64, 2, device=dev())
    N.row_stats64(x, st)
    out = torch.empty(M, Nn, device=dev(), dtype=torch.bfloat16)
    N.gemm(x, wf.to(dev()), out, M, Nn, K, bias=bf.to(dev()), act=act, ln_stats=st, ln_colsum=sf.to(dev()),
           ln_eps=1e-12)
    ln = F.layer_norm(x.double(), (K,), gamma.double().to(dev()), beta.double().to(dev()), 1e-12)
    ref = ln @ W.double().to(dev()).t() + b.double().to(dev())
    ref = F.gelu(ref) if act == 2 else ref
    # the sequence it replaces: LayerNorm kernel -> bf16 operand -> GEMM on W
    a = torch.empty_like(x)
    N.layernorm_fwd(x, gamma.to(dev()), beta.to(dev()), 1e-12, a)
    seq = torch.empty_like(out)
    N.gemm(a, W.to(dev(), torch.bfloat16), seq, M, Nn, K, bias=b.to(dev()), act=act)
    e_fold, e_seq = _rel(out.double(), ref), _rel(seq.double(), ref)
    print(f"LN fold rel-L2 {e_fold:.3e} vs LN->GEMM {e_seq:.3e}")
    assert e_fold < 8e-3 and e_fold <= 1.1 * e_seq


@pytest.mark.parametrize("M,E,F4", [(2000, 768, 3072), (300, 64, 256), (257, 192, 128)])
def test_gemm_stats_out_and_chain(M, E, F4):
    """A residual GEMM writes the per-64-column statistics of its bf16 output rows (stats_out); a
    LayerNorm-folded GEMM reading them equals LN(out) W^T + b -- the encoder's o-proj -> fc1 chain
    (E = 64 / 192: output widths narrower than the 256-column tile, whose idle waves write nothing)."""
    import torch.nn.functional as F
    from encoder import fold_layernorm
    torch.manual_seed(11)
    o = torch.randn(M, E, device=dev()).to(torch.bfloat16)
    h = (3 * torch.randn(M, E, device=dev())).to(torch.bfloat16)
    Wo = (torch.randn(E, E, device=dev()) / E ** 0.5).to(torch.bfloat16)
    bo = 0.1 * torch.randn(E, device=dev())
    st_buf = torch.full((M + 1, E // 64, 2), float("nan"), device=dev())
    st = st_buf[:M]
    h2 = h.clone()
    N.gemm(o, Wo, h2, M, E, E, bias=bo, residual=h2, stats_out=st)
    ref_h = o.float() @ Wo.float().t() + bo + h.float()
    assert _rel(h2, ref_h) < 5e-3
    ref_st = _stats64_ref(h2)
    assert (st.double() - ref_st).abs().max().item() <= 1e-4 * ref_st.abs().max().item()
    assert torch.isnan(st_buf[M]).all()  # nothing written past the last row's partials
    W1 = torch.randn(F4, E) / E ** 0.5
    b1, g, be = 0.1 * torch.randn(F4), 1 + 0.2 * torch.randn(E), 0.1 * torch.randn(E)
    wf, bf, sf = fold_layernorm(W1, b1, g, be)
    m = torch.empty(M, F4, device=dev(), dtype=torch.bfloat16)
    N.gemm(h2, wf.to(dev()), m, M, F4, E, bias=bf.to(dev()), act=N.ACT_GELU, ln_stats=st, ln_colsum=sf.to(dev()),
           ln_eps=1e-12)
    ref = F.gelu(F.layer_norm(h2.double(), (E,), g.double().to(dev()), be.double().to(dev()), 1e-12)
                 @ W1.double().to(dev()).t() + b1.double().to(dev()))
    assert _rel(m.double(), ref) < 8e-3


def test_gemm_layernorm_fold_rejects_bad_args():
    x = torch.randn(256, 200, device=dev()).to(torch.bfloat16)
    w = torch.randn(256, 200, device=dev()).to(torch.bfloat16)
    out = torch.empty(256, 256, device=dev(), dtype=torch.bfloat16)
    st = torch.zeros(256, 4, 2, device=dev())
    with pytest.raises(N.NativeError, match="ln_stats"):  # K % 64 != 0
        N.gemm(x, w, out, 256, 256, 200, ln_stats=st, ln_colsum=torch.zeros(256, device=dev()))


@pytest.mark.parametrize("M,Nn,K,kind", [(256, 256, 64, "plain"), (520, 776, 192, "bias"), (1000, 512, 256, "resst"),
                                         (2056, 768, 768, "gelu"), (1032, 2304, 768, "lnbias"),
                                         (1032, 3072, 768, "lngelu"), (300, 264, 1024, "qgelu")])
def test_gemm256w_one_wave_per_simd_bitwise(M, Nn, K, kind):
    """The opt-in one-wave-per-SIMD 256x256 kernel (mit_gemm_set_variant(4), gemm256w_kernel) sums the same
    MFMAs in the same K order as gemm256_kernel: outputs (and STG 4 row statistics) bitwise equal, for the
    plain / bias / GELU / quick_gelu / LayerNorm-folded / residual + statistics epilogues and ragged M / N."""
    torch.manual_seed(3)
    A = torch.randn(M, K, device=dev()).to(torch.bfloat16)
    B = (0.05 * torch.randn(Nn, K, device=dev())).to(torch.bfloat16)
    kw = {}
    if kind != "plain":
        kw["bias"] = torch.randn(Nn, device=dev())
    if kind in ("gelu", "lngelu"):
        kw["act"] = N.ACT_GELU
    if kind == "qgelu":
        kw["act"] = N.ACT_QUICK_GELU
    if kind == "resst":
        kw["residual"] = torch.randn(M, Nn, device=dev()).to(torch.bfloat16)
    if kind.startswith("ln"):
        mean = 0.1 * torch.randn(M, K // 64, device=dev())
        m2 = 64.0 * (0.5 + torch.rand(M, K // 64, device=dev()))
        kw.update(ln_stats=torch.stack([mean, m2], -1).contiguous(), ln_colsum=torch.randn(Nn, device=dev()), ln_eps=1e-5)
    outs = []
    for v in (0, 4):
        N.gemm_set_variant(v)
        C = torch.full((M, Nn), float("nan"), device=dev(), dtype=torch.bfloat16)
        st = torch.full((M, Nn // 64, 2), float("nan"), device=dev()) if kind == "resst" else None
        N.gemm(A, B, C, M, Nn, K, tiles=256, stats_out=st, **kw)
        torch.cuda.synchronize()
        outs.append((C, st))
    N.gemm_set_variant(0)
    assert torch.equal(outs[0][0].view(torch.int16), outs[1][0].view(torch.int16))
    if kind == "resst":
        assert torch.equal(outs[0][1].view(torch.int32), outs[1][1].view(torch.int32))
    ref = A.float() @ B.float().t()
    if kind in ("plain",):
        assert _rel(outs[1][0], ref) < 1e-2
