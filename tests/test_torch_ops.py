"""torch.ops.mit_hip (csrc/torch_ops.cpp, TORCH_LIBRARY over the C ABI; ops.py registers the autograd formulas
and fake kernels): the library registers its schemas and fake kernels on the CPU (no launches; CPU tensors
are refused by the dispatcher), and on the GPU every op and every backward matches the torch op it
replaces (F.linear + activation + residual, the TransformerDecoderLayer feed-forward block, F.layer_norm,
F.scaled_dot_product_attention with the causal / key-padding masks, nn.Embedding + positional encoding,
F.cross_entropy(ignore_index), clip_grad_norm_ + torch.optim.AdamW), forward and torch.autograd backward,
and the ops replay inside a torch.cuda graph."""
import math

import pytest
import torch
import torch.nn.functional as F

import native
import ops

OPS = ["linear", "linear_backward", "ffn", "ffn_backward", "layer_norm", "layer_norm_train", "layer_norm_backward",
       "attention", "attention_train", "attention_backward", "embedding", "embedding_backward", "cross_entropy",
       "clip_adamw_step"]


def test_torch_ops_register_schemas_on_cpu():
    mh = ops.load()
    for name in OPS:
        schema = str(getattr(mh, name).default._schema)
        assert schema.startswith(f"mit_hip::{name}("), schema
    assert "Tensor? weight_lp=None" in str(mh.linear.default._schema)
    assert "Tensor(a!) param" in str(mh.clip_adamw_step.default._schema)


def test_torch_ops_refuse_cpu_tensors():
    mh = ops.load()
    x, w = torch.randn(4, 8), torch.randn(16, 8)
    with pytest.raises((NotImplementedError, RuntimeError)):
        mh.linear(x, w)


def test_torch_ops_fake_kernels_give_shapes():
    """register_fake: shapes / dtypes without a kernel (torch.compile / FakeTensor tracing)."""
    mh = ops.load()
    m = dict(device="meta")
    x = torch.empty(2, 7, 64, dtype=torch.bfloat16, **m)
    w, b = torch.empty(96, 64, **m), torch.empty(96, **m)
    y = mh.linear(x, w, b, out_f32=True)
    assert y.shape == (2, 7, 96) and y.dtype == torch.float32
    yy, z, mean, rstd = mh.layer_norm_train(x, torch.empty(64, **m), torch.empty(64, **m), 1e-5, x)
    assert yy.shape == z.shape == x.shape and mean.shape == rstd.shape == (14,)
    o, lse = mh.attention_train(x, x, x, 4, True)
    assert o.shape == x.shape and lse.shape == (2 * 4 * 7,) and lse.dtype == torch.float32
    y2, h = mh.ffn(x, torch.empty(128, 64, **m), torch.empty(128, **m), torch.empty(64, 128, **m), torch.empty(64, **m))
    assert y2.shape == x.shape and h.shape == (2, 7, 128)
    tok = torch.empty(2, 7, dtype=torch.int64, **m)
    e = mh.embedding(tok, torch.empty(50, 64, **m), torch.empty(100, 64, **m), 8.0)
    assert e.shape == (2, 7, 64)
    loss, g = mh.cross_entropy(torch.empty(14, 50, **m), torch.empty(14, dtype=torch.int64, **m), 0)
    assert loss.shape == () and g.shape == (14, 50)


def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    native.load_library()
    return ops.load()


def _close(a, b, tol):
    a, b = a.float(), b.float()
    return (a - b).abs().max().item() <= tol * max(b.abs().max().item(), 1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("act", [0, 1, 2, 3])
def test_torch_linear_matches_torch(dtype, act):
    mh = _gpu()
    torch.manual_seed(0)
    x = torch.randn(3, 50, 256, device="cuda").to(dtype)
    w = (torch.randn(384, 256, device="cuda") / 16).to(dtype)
    b = torch.randn(384, device="cuda")
    r = torch.randn(3, 50, 384, device="cuda").to(dtype)
    y = mh.linear(x, w, b, act, r)
    z = F.linear(x.float(), w.float(), b)
    z = [z, F.relu(z), F.gelu(z), z * torch.sigmoid(1.702 * z)][act] + r.float()
    assert y.shape == (3, 50, 384) and y.dtype == dtype
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    assert _close(y, z, tol)
    y0 = mh.linear(x, w)  # no bias / activation / residual
    assert (y0.float() - F.linear(x.float(), w.float())).abs().max().item() <= tol * 8


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_torch_linear_backward_matches_autograd(dtype):
    """Gradients of y = x W^T + b + r with respect to x, the f32 master W (the GEMM reads its bf16 shadow),
    b and r against torch.autograd of F.linear in float64."""
    mh = _gpu()
    torch.manual_seed(1)
    x = torch.randn(2, 70, 264, device="cuda").to(dtype).requires_grad_()
    w = (torch.randn(136, 264, device="cuda") / 16).requires_grad_()
    b = torch.randn(136, device="cuda").requires_grad_()
    r = torch.randn(2, 70, 136, device="cuda").to(dtype).requires_grad_()
    lp = w.detach().to(dtype) if dtype == torch.bfloat16 else None
    y = mh.linear(x, w, b, 0, r, weight_lp=lp, out_f32=dtype == torch.float32)
    gy = torch.randn(y.shape, device="cuda").to(y.dtype)
    y.backward(gy)
    xd, wd, bd, rd = (t.detach().double().requires_grad_() for t in (x, (lp if lp is not None else w), b, r))
    (F.linear(xd, wd, bd) + rd).backward(gy.double())
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    assert w.grad.dtype == torch.float32 and b.grad.dtype == torch.float32 and x.grad.dtype == dtype
    for got, ref in ((x.grad, xd.grad), (w.grad, wd.grad), (b.grad, bd.grad), (r.grad, rd.grad)):
        assert _close(got, ref, tol)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("drop_p", [0.0, 0.2])
def test_torch_ffn_matches_autograd(dtype, drop_p):
    """linear2(dropout(relu(linear1(x)))) (transformer.py:1197-1199) and its five gradients; the dropout
    mask is the kernels' counter hash (mit_dropout_mask at the same site), fed to the torch reference."""
    mh = _gpu()
    torch.manual_seed(2)
    R, d, Fd = 130, 128, 512
    x = torch.randn(R, d, device="cuda").to(dtype).requires_grad_()
    w1 = (torch.randn(Fd, d, device="cuda") / 11).requires_grad_()
    b1 = (0.1 * torch.randn(Fd, device="cuda")).requires_grad_()
    w2 = (torch.randn(d, Fd, device="cuda") / 22).requires_grad_()
    b2 = (0.1 * torch.randn(d, device="cuda")).requires_grad_()
    seed = torch.tensor([1234], dtype=torch.int64, device="cuda")
    lp = (lambda t: t.detach().to(dtype)) if dtype == torch.bfloat16 else (lambda t: None)  # noqa: E731
    y, h = mh.ffn(x, w1, b1, w2, b2, drop_p, seed, 7, lp(w1), lp(w2))
    gy = torch.randn(y.shape, device="cuda").to(dtype)
    y.backward(gy)
    mask = torch.ones(R * Fd, device="cuda")
    if drop_p > 0:
        native.dropout_mask(R * Fd, drop_p, seed, 7, mask)
    mask = mask.view(R, Fd).double()
    ref = [t.detach().double().requires_grad_() for t in (x, lp(w1) if dtype == torch.bfloat16 else w1, b1,
                                                          lp(w2) if dtype == torch.bfloat16 else w2, b2)]
    yr = F.linear(F.relu(F.linear(ref[0], ref[1], ref[2])) * mask, ref[3], ref[4])
    yr.backward(gy.double())
    tol = 3e-2 if dtype == torch.bfloat16 else 1e-5
    assert _close(y, yr, tol)
    for got, r in zip((x.grad, w1.grad, b1.grad, w2.grad, b2.grad), ref):
        assert _close(got, r.grad, tol)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("cols", [512, 768])
def test_torch_layer_norm_matches_torch(dtype, cols):
    mh = _gpu()
    x = torch.randn(2, 99, cols, device="cuda").to(dtype)
    r = torch.randn(2, 99, cols, device="cuda").to(dtype)
    g, b = 1 + 0.1 * torch.randn(cols, device="cuda"), 0.1 * torch.randn(cols, device="cuda")
    y = mh.layer_norm(x, g, b, 1e-5, r)
    ref = F.layer_norm(x.float() + r.float(), (cols,), g, b, 1e-5)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    assert _close(y, ref, tol)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_torch_layer_norm_backward_matches_autograd(dtype):
    mh = _gpu()
    torch.manual_seed(3)
    C = 512
    x = torch.randn(3, 41, C, device="cuda").to(dtype).requires_grad_()
    r = torch.randn(3, 41, C, device="cuda").to(dtype).requires_grad_()
    g = (1 + 0.1 * torch.randn(C, device="cuda")).requires_grad_()
    b = (0.1 * torch.randn(C, device="cuda")).requires_grad_()
    y = mh.layer_norm_train(x, g, b, 1e-5, r)[0]
    gy = torch.randn(y.shape, device="cuda").to(dtype)
    y.backward(gy)
    ref = [t.detach().double().requires_grad_() for t in (x, r, g, b)]
    F.layer_norm(ref[0] + ref[1], (C,), ref[2], ref[3], 1e-5).backward(gy.double())
    tol = 3e-2 if dtype == torch.bfloat16 else 1e-5
    for got, rr in zip((x.grad, r.grad, g.grad, b.grad), ref):
        assert _close(got, rr.grad, tol)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("Lq,Lk,causal", [(197, 197, False), (63, 197, False), (64, 64, True)])
def test_torch_attention_matches_sdpa(dtype, Lq, Lk, causal):
    mh = _gpu()
    B, H, D = 2, 8, 64
    q = torch.randn(B, Lq, H * D, device="cuda").to(dtype)
    kv = torch.randn(B, Lk, 2 * H * D, device="cuda").to(dtype)
    k, v = kv[..., : H * D], kv[..., H * D:]  # strided views, as the packed projections leave them
    o = mh.attention(q, k, v, H, causal, 1 / math.sqrt(D))
    sh = lambda t, L: t.float().reshape(B, L, H, D).transpose(1, 2)  # noqa: E731
    ref = F.scaled_dot_product_attention(sh(q, Lq), sh(k, Lk), sh(v, Lk), is_causal=causal)
    ref = ref.transpose(1, 2).reshape(B, Lq, H * D)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    assert _close(o, ref, tol)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("Lq,Lk,causal", [(63, 63, True), (63, 197, False)])
def test_torch_attention_backward_matches_autograd(dtype, Lq, Lk, causal):
    """dq, dk, dv of the decoder's self-attention (causal + key padding from the tokens, functional.py
    :6370-6404) and cross-attention against torch.autograd of SDPA with the same float mask."""
    mh = _gpu()
    torch.manual_seed(4)
    B, H, D = 2, 8, 64
    qkv = torch.randn(B, max(Lq, Lk), 3 * H * D, device="cuda").to(dtype)
    q = qkv[:, :Lq, : H * D].detach().requires_grad_()
    k = qkv[:, :Lk, H * D: 2 * H * D].detach().requires_grad_()
    v = qkv[:, :Lk, 2 * H * D:].detach().requires_grad_()
    toks = None
    if causal:
        toks = torch.randint(4, 100, (B, Lk), device="cuda")
        toks[0, 50:] = 0  # padded tail of caption 0
    o = mh.attention_train(q, k, v, H, causal, 1 / math.sqrt(D), toks, 0)[0]
    go = torch.randn(o.shape, device="cuda").to(dtype)
    o.backward(go)
    sh = lambda t, L: t.detach().double().reshape(B, L, H, D).transpose(1, 2).requires_grad_()  # noqa: E731
    qd, kd, vd = sh(q, Lq), sh(k, Lk), sh(v, Lk)
    mask = torch.zeros(B, 1, Lq, Lk, dtype=torch.float64, device="cuda")
    if causal:
        mask = mask.masked_fill(torch.ones(Lq, Lk, dtype=torch.bool, device="cuda").triu(1), float("-inf"))
        mask = mask.masked_fill((toks == 0)[:, None, None, :], float("-inf"))
    ref = F.scaled_dot_product_attention(qd, kd, vd, attn_mask=mask)
    ref.backward(go.double().reshape(B, Lq, H, D).transpose(1, 2))
    un = lambda t, L: t.transpose(1, 2).reshape(B, L, H * D)  # noqa: E731
    tol = 3e-2 if dtype == torch.bfloat16 else 1e-4
    assert _close(o, un(ref, Lq), tol)
    for got, r, L in ((q.grad, qd.grad, Lq), (k.grad, kd.grad, Lk), (v.grad, vd.grad, Lk)):
        assert _close(got, un(r, L), tol)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_torch_embedding_matches_autograd(dtype):
    """dropout(Emb[tok] * sqrt(d) + PE[t]) (decoder.py:168-171) and the table gradient with
    nn.Embedding(padding_idx=PAD) semantics (the PAD row gets none), deterministic over repeats."""
    mh = _gpu()
    torch.manual_seed(5)
    V, d, B, T = 300, 128, 4, 33
    table = torch.randn(V, d, device="cuda").requires_grad_()
    pe = torch.randn(64, d, device="cuda")
    tok = torch.randint(0, V, (B, T), device="cuda")
    tok[:, -5:] = 0
    lp = table.detach().to(dtype) if dtype == torch.bfloat16 else None
    x = mh.embedding(tok, table, pe, math.sqrt(d), 0.0, None, 0, lp, 0)
    gx = torch.randn(x.shape, device="cuda").to(dtype)
    x.backward(gx)
    tr = (lp if lp is not None else table).detach().double().requires_grad_()
    xr = F.embedding(tok, tr, padding_idx=0) * math.sqrt(d) + pe[:T].double()
    xr.backward(gx.double())
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    assert _close(x, xr, tol)
    assert _close(table.grad, tr.grad, tol)
    assert table.grad[0].abs().max().item() == 0.0
    g1 = table.grad.clone()
    table.grad = None
    mh.embedding(tok, table, pe, math.sqrt(d), 0.0, None, 0, lp, 0).backward(gx)
    assert torch.equal(table.grad, g1)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_torch_cross_entropy_matches_torch(dtype):
    mh = _gpu()
    torch.manual_seed(6)
    R, V = 200, 1000
    logits = (3 * torch.randn(R, V, device="cuda")).to(dtype).requires_grad_()
    t = torch.randint(1, V, (R,), device="cuda")
    t[::7] = 0
    loss = mh.cross_entropy(logits, t, 0)[0]
    loss.backward()
    lr = logits.detach().double().requires_grad_()
    ref = F.cross_entropy(lr, t, ignore_index=0)
    ref.backward()
    assert abs(loss.item() - ref.item()) <= (5e-3 if dtype == torch.bfloat16 else 1e-5) * abs(ref.item())
    assert _close(logits.grad, lr.grad, 2e-2 if dtype == torch.bfloat16 else 1e-5)


@pytest.mark.gpu
def test_torch_clip_adamw_step_matches_torch():
    """clip_grad_norm_ + torch.optim.AdamW over one flat f32 buffer, with the bf16 shadow refreshed."""
    mh = _gpu()
    torch.manual_seed(7)
    n = 100_003
    p0 = torch.randn(n, device="cuda")
    grads = [torch.randn(n, device="cuda") * s for s in (3.0, 0.01)]
    param, ea, eas = p0.clone(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    shadow = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    step, lr = torch.zeros(1, dtype=torch.int64, device="cuda"), torch.full((1,), 1e-3, device="cuda")
    norm, ws = torch.zeros(2, device="cuda"), torch.empty(native.grad_norm_ws_floats(n), device="cuda")
    ref = p0.clone().requires_grad_()
    opt = torch.optim.AdamW([ref], lr=1e-3, betas=(0.9, 0.98), eps=1e-9, weight_decay=1e-2)
    for g in grads:
        mh.clip_adamw_step(param, g, ea, eas, shadow, step, lr, norm, ws, 5.0, 0.9, 0.98, 1e-9, 1e-2)
        ref.grad = g.clone()
        tn = torch.nn.utils.clip_grad_norm_([ref], 5.0)
        opt.step()
        assert abs(norm[0].item() - tn.item()) <= 1e-5 * tn.item()
    assert step.item() == 2
    assert (param - ref.detach()).abs().max().item() <= 1e-6
    assert torch.equal(shadow, param.to(torch.bfloat16))


@pytest.mark.gpu
def test_torch_ops_replay_in_cuda_graph():
    mh = _gpu()
    x = torch.randn(64, 512, device="cuda").to(torch.bfloat16)
    w = (torch.randn(512, 512, device="cuda") / 22).to(torch.bfloat16)
    g, b = torch.ones(512, device="cuda"), torch.zeros(512, device="cuda")
    eager = mh.layer_norm(mh.linear(x, w, None, 1), g, b, 1e-5)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        mh.layer_norm(mh.linear(x, w, None, 1), g, b, 1e-5)  # warm-up on the capture stream
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = mh.layer_norm(mh.linear(x, w, None, 1), g, b, 1e-5)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, eager)


@pytest.mark.gpu
def test_model_autograd_path_dispatches_through_torch_ops():
    """model(images, tokens) under autograd records torch.ops.mit_hip nodes (the reference loop's
    forward / backward go through the operator library), and the gradients land in the flat buffer."""
    import fixtures as FX
    from model_util import build_model
    _gpu()
    meta, _ = FX.load("tiny_vit_patches")
    m, _ = build_model(meta, torch.bfloat16)
    m.train()
    imgs, di, tg = [t.cuda() for t in FX.inputs(meta, 0)]
    seen = set()

    class Spy(torch.utils._python_dispatch.TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            if func.namespace == "mit_hip":
                seen.add(func.__name__.split(".")[0])
            return func(*args, **(kwargs or {}))
    with Spy():
        logits = m(imgs, di)
        loss = torch.nn.functional.cross_entropy(logits.reshape(-1, logits.shape[-1]), tg.reshape(-1), ignore_index=0)
        loss.backward()
    assert {"linear", "ffn", "layer_norm_train", "attention_train", "embedding"} <= seen, seen
    assert {"linear_backward", "ffn_backward", "layer_norm_backward", "attention_backward",
            "embedding_backward"} <= seen, seen
    for n, p in m.named_parameters():
        assert p.grad is not None and p.grad.data_ptr() == m.store.g(n).data_ptr(), n
