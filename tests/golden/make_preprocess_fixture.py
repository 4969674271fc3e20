"""Golden vectors for the data path: HF ViTImageProcessor() and
CLIPImageProcessor() (transformers 5.15.0, the reference's AutoImageProcessor backends; local
defaults, no hub access) applied to small seeded RGB images of odd sizes. Stores the input pixels
and the processors' pixel_values (f32). Regenerate: python tests/golden/make_preprocess_fixture.py
"""
import json
import os

import numpy as np
import torch
from PIL import Image
from safetensors.torch import save_file
from transformers import CLIPImageProcessor, ViTImageProcessor

SHAPES = [(61, 90), (150, 97)]  # (H, W): landscape and portrait, both upsampled


def images():
    rng = np.random.default_rng(1234)
    out = []
    for h, w in SHAPES:
        # smooth gradients + noise: resampling filters see structure, not just white noise
        yy, xx = np.mgrid[0:h, 0:w]
        base = np.stack([(xx * 255 // max(w - 1, 1)), (yy * 255 // max(h - 1, 1)), ((xx + yy) * 7) % 256], -1)
        noise = rng.integers(-40, 41, (h, w, 3))
        out.append(np.clip(base + noise, 0, 255).astype(np.uint8))
    return out


def main():
    ims = images()
    pil = [Image.fromarray(a) for a in ims]
    t = {}
    for i, a in enumerate(ims):
        t[f"img{i}"] = torch.from_numpy(a.copy())
    v = ViTImageProcessor()(images=pil, return_tensors="np")["pixel_values"]
    c = CLIPImageProcessor()(images=pil, return_tensors="np")["pixel_values"]
    c336 = CLIPImageProcessor(size={"shortest_edge": 336}, crop_size={"height": 336, "width": 336})(
        images=pil[:1], return_tensors="np")["pixel_values"]
    t["vit"] = torch.from_numpy(v.astype(np.float32))
    t["clip"] = torch.from_numpy(c.astype(np.float32))
    t["clip336"] = torch.from_numpy(c336.astype(np.float32))
    meta = {"shapes": SHAPES, "generator": "transformers ViTImageProcessor() / CLIPImageProcessor() defaults",
            "clip_mean": list(CLIPImageProcessor().image_mean), "clip_std": list(CLIPImageProcessor().image_std)}
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "preprocess.safetensors")
    save_file(t, out, metadata={"meta": json.dumps(meta)})
    print(out, {k: tuple(x.shape) for k, x in t.items()})


if __name__ == "__main__":
    main()
