"""The encoder's f32 residual stream (encoder.VisionEncoder.res32: auto for the 24-layer CLIP-L towers,
ENCODER_F32_RESIDUAL=on for any tower) and its two kernels, mit_layernorm_fwd_x32 (z = x + r in f32, y =
LN(z) in bf16 or f32; z may alias x; strided rows) and mit_residual_out (y = x + r, rounded), against torch.
The encoder-level check runs the res32 path on the 2-layer ViT (the ViT branch, reached only with the flag
on) and the CLIP-336 fixtures in both memory modes (the rows="cls" strided branch), against the
reference's own last_hidden_state."""
import pytest
import torch
import torch.nn.functional as F

import fixtures as FX
import native as N
from model_util import build_model

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    N.load_library()


def _ln(z, g, b, eps):
    return F.layer_norm(z.double(), (z.shape[-1],), g.double(), b.double(), eps)


@pytest.mark.parametrize("cols", [768, 1024])
@pytest.mark.parametrize("case", ["r_z_bf16", "inplace", "no_r_f32y", "strided"])
def test_layernorm_fwd_x32_matches_torch(cols, case):
    torch.manual_seed(cols)
    R, eps = 301, 1e-5
    g, b = 1 + 0.1 * torch.randn(cols, device="cuda"), 0.1 * torch.randn(cols, device="cuda")
    r = (0.5 * torch.randn(R, cols, device="cuda")).to(torch.bfloat16)
    if case == "strided":  # rows of a wider buffer (the rows="cls" form: ldx = ldr = ldy = N * E)
        xb = 3 * torch.randn(R, 2 * cols, device="cuda")
        rb = torch.zeros(R, 2 * cols, device="cuda", dtype=torch.bfloat16)
        rb[:, :cols] = r
        yb = torch.zeros(R, 2 * cols, device="cuda", dtype=torch.bfloat16)
        x0 = xb[:, :cols].clone()
        N.layernorm_fwd_x32(xb, g, b, eps, yb, r=rb, rows=R, cols=cols, ldx=2 * cols, ldr=2 * cols, ldy=2 * cols)
        ref = _ln(x0 + r.float(), g, b, eps)
        assert (yb[:, :cols].double() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()
        assert yb[:, cols:].abs().max().item() == 0.0  # nothing written past the row's columns
        return
    x = 3 * torch.randn(R, cols, device="cuda")
    x0 = x.clone()
    rr = None if case == "no_r_f32y" else r
    z = x if case == "inplace" else (None if case == "no_r_f32y" else torch.empty_like(x))
    y = torch.empty(R, cols, device="cuda", dtype=torch.float32 if case == "no_r_f32y" else torch.bfloat16)
    N.layernorm_fwd_x32(x, g, b, eps, y, r=rr, z=z)
    zr = x0 + (rr.float() if rr is not None else 0)
    ref = _ln(zr, g, b, eps)
    tol = 1e-5 if y.dtype == torch.float32 else 2e-2
    assert (y.double() - ref).abs().max().item() <= tol * ref.abs().max().item()
    if z is not None:
        assert (z - zr).abs().max().item() <= 1e-6 * zr.abs().max().item()  # f32 add of a bf16 value: exact
    if case == "no_r_f32y":
        assert torch.equal(x, x0)


@pytest.mark.parametrize("with_r", [True, False])
def test_residual_out_matches_torch(with_r):
    R, C = 257, 1024
    xb = 2 * torch.randn(R, 2 * C, device="cuda")
    r = torch.randn(R, C, device="cuda").to(torch.bfloat16) if with_r else None
    y = torch.zeros(R, C, device="cuda", dtype=torch.bfloat16)
    N.residual_out(xb, r, y, rows=R, cols=C, ldx=2 * C)
    ref = (xb[:, :C] + (r.float() if with_r else 0)).to(torch.bfloat16)
    assert torch.equal(y, ref)


@pytest.mark.parametrize("name", ["tiny_vit_patches", "tiny_clip336_patches", "tiny_clip336_cls"])
def test_encoder_res32_matches_reference(name, monkeypatch):
    """res32 forced on: last_hidden_state within the bf16 encoder bound of test_model_gpu (rel-L2 <=
    1.5e-2, max error <= 3e-2 of the scale), and no worse than 1.1x the bf16-stream encoder's error."""
    import config
    meta, T = FX.load(name)
    errs = {}
    for mode in ("off", "on"):
        monkeypatch.setattr(config, "ENCODER_F32_RESIDUAL", mode)
        m, _ = build_model(meta, torch.bfloat16)
        assert m.encoder.res32 == (mode == "on")
        imgs, _, _ = FX.inputs(meta, 0)
        with torch.no_grad():
            feats = m.encoder.forward(imgs.cuda(), rows="all").float().cpu()
            if meta["mode"] == "cls":  # the strided CLS-rows branch against the CLS rows of the full forward
                cls = m.encoder.forward(imgs.cuda(), rows="cls").float().cpu()
                assert (cls - feats[:, 0]).abs().max().item() <= 2e-2 * feats[:, 0].abs().max().item()
        rel = []
        for got, ref in FX.encoder_rows(T, feats):
            rel.append(((got - ref).norm() / ref.norm()).item())
            assert rel[-1] <= 1.5e-2 and (got - ref).abs().max().item() <= 3e-2 * ref.abs().max().item()
        errs[mode] = max(rel)
        del m
    print(f"{name}: encoder rel-L2 bf16 stream {errs['off']:.2e}, f32 stream {errs['on']:.2e}")
    assert errs["on"] <= 1.1 * errs["off"]
