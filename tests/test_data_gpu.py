"""GPU image normalisation (image.hip mit_image_normalize) against the HF processors' pixel_values
(tests/golden/preprocess.safetensors): bit-identical after the host resample, for ViT (mean = std =
0.5) and CLIP (OPENAI mean/std, 224 and 336); plus a synthetic batch against numpy float32."""
import json
import os

import numpy as np
import pytest
import torch
from safetensors import safe_open

import data
import native as N

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "preprocess.safetensors")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    N.load_library()


@pytest.mark.parametrize("kind,key,size", [("vit", "vit", 224), ("clip", "clip", 224), ("clip", "clip336", 336)])
def test_preprocessor_matches_hf_pixel_values(kind, key, size):
    with safe_open(GOLD, "pt") as f:
        T = {k: f.get_tensor(k) for k in f.keys()}
    ref = T[key]
    pre = data.ImagePreprocessor(kind, size)
    ims = [T[f"img{i}"].numpy() for i in range(ref.shape[0])]
    got = pre(ims)["pixel_values"]
    assert got.shape == ref.shape and got.dtype == torch.float32 and got.is_cuda
    assert torch.equal(got.cpu(), ref)


def test_normalize_kernel_batch_vs_numpy():
    g = np.random.default_rng(5)
    u8 = g.integers(0, 256, (7, 64, 36, 3), dtype=np.uint8)
    mean, std = (0.1, 0.7, 0.33), (0.2, 1.5, 0.9)
    out = torch.empty(7, 3, 64, 36, device="cuda")
    N.image_normalize(torch.from_numpy(u8).cuda(), out, mean, std)
    m, s = np.array(mean, np.float32), np.array(std, np.float32)
    ref = (((u8.astype(np.float32) / np.float32(255.0)) - m) / s).transpose(0, 3, 1, 2)
    assert np.array_equal(out.cpu().numpy(), ref)


def test_collated_batch_to_device():
    b = [{"image_path": "p", "image": torch.full((32, 32, 3), 51 * i, dtype=torch.uint8),
          "caption_tokens": torch.tensor([1, 5, 2, 0])} for i in range(3)]
    pre = data.ImagePreprocessor("vit", 32)
    out = data.to_device(data.collate_fn(b), pre)
    assert out["images"].shape == (3, 3, 32, 32) and out["images"].is_cuda
    for i in range(3):
        v = (np.float32(51 * i) / np.float32(255.0) - np.float32(0.5)) / np.float32(0.5)
        assert torch.all(out["images"][i] == float(v))
    assert out["target_tokens"].is_cuda and out["decoder_input_tokens"].tolist() == [[1, 5, 2]] * 3
