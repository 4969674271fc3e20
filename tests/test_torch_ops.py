"""torch.ops.mit_hip (csrc/torch_ops.cpp, TORCH_LIBRARY over the C ABI): the operator library loads and
registers its schemas on the CPU (no launches; CPU tensors are refused by the dispatcher), and on the
GPU each op matches the torch op it replaces (F.linear + activation + residual, F.layer_norm,
F.scaled_dot_product_attention) and replays inside a torch.cuda graph."""
import math

import pytest
import torch
import torch.nn.functional as F

import native


def test_torch_ops_register_schemas_on_cpu():
    ops = native.load_torch_ops()
    for name, arg in (("linear", "Tensor? residual=None"), ("layer_norm", "float eps"), ("attention", "bool causal=False")):
        schema = str(getattr(ops, name).default._schema)
        assert schema.startswith(f"mit_hip::{name}(") and arg in schema, schema


def test_torch_ops_refuse_cpu_tensors():
    ops = native.load_torch_ops()
    x, w = torch.randn(4, 8), torch.randn(16, 8)
    with pytest.raises((NotImplementedError, RuntimeError)):
        ops.linear(x, w)


def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    native.load_library()
    return native.load_torch_ops()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("act", [0, 1, 2, 3])
def test_torch_linear_matches_torch(dtype, act):
    ops = _gpu()
    torch.manual_seed(0)
    x = torch.randn(3, 50, 256, device="cuda").to(dtype)
    w = (torch.randn(384, 256, device="cuda") / 16).to(dtype)
    b = torch.randn(384, device="cuda")
    r = torch.randn(3, 50, 384, device="cuda").to(dtype)
    y = ops.linear(x, w, b, act, r)
    z = F.linear(x.float(), w.float(), b)
    z = [z, F.relu(z), F.gelu(z), z * torch.sigmoid(1.702 * z)][act] + r.float()
    assert y.shape == (3, 50, 384) and y.dtype == dtype
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    assert (y.float() - z).abs().max().item() <= tol * z.abs().max().item()
    y0 = ops.linear(x, w)  # no bias / activation / residual
    assert (y0.float() - F.linear(x.float(), w.float())).abs().max().item() <= tol * 8


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("cols", [512, 768])
def test_torch_layer_norm_matches_torch(dtype, cols):
    ops = _gpu()
    x = torch.randn(2, 99, cols, device="cuda").to(dtype)
    r = torch.randn(2, 99, cols, device="cuda").to(dtype)
    g, b = 1 + 0.1 * torch.randn(cols, device="cuda"), 0.1 * torch.randn(cols, device="cuda")
    y = ops.layer_norm(x, g, b, 1e-5, r)
    ref = F.layer_norm(x.float() + r.float(), (cols,), g, b, 1e-5)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-5
    assert (y.float() - ref).abs().max().item() <= tol * ref.abs().max().item()


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("Lq,Lk,causal", [(197, 197, False), (63, 197, False), (64, 64, True)])
def test_torch_attention_matches_sdpa(dtype, Lq, Lk, causal):
    ops = _gpu()
    B, H, D = 2, 8, 64
    q = torch.randn(B, Lq, H * D, device="cuda").to(dtype)
    kv = torch.randn(B, Lk, 2 * H * D, device="cuda").to(dtype)
    k, v = kv[..., : H * D], kv[..., H * D:]  # strided views, as the packed projections leave them
    o = ops.attention(q, k, v, H, causal, 1 / math.sqrt(D))
    sh = lambda t, L: t.float().reshape(B, L, H, D).transpose(1, 2)  # noqa: E731
    ref = F.scaled_dot_product_attention(sh(q, Lq), sh(k, Lk), sh(v, Lk), is_causal=causal)
    ref = ref.transpose(1, 2).reshape(B, Lq, H * D)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    assert (o.float() - ref).abs().max().item() <= tol * ref.abs().max().item()


@pytest.mark.gpu
def test_torch_ops_replay_in_cuda_graph():
    ops = _gpu()
    x = torch.randn(64, 512, device="cuda").to(torch.bfloat16)
    w = (torch.randn(512, 512, device="cuda") / 22).to(torch.bfloat16)
    g, b = torch.ones(512, device="cuda"), torch.zeros(512, device="cuda")
    eager = ops.layer_norm(ops.linear(x, w, None, 1), g, b, 1e-5)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.layer_norm(ops.linear(x, w, None, 1), g, b, 1e-5)  # warm-up on the capture stream
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = ops.layer_norm(ops.linear(x, w, None, 1), g, b, 1e-5)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, eager)
