"""Data path of the captioning train step: captions JSON -> (image, tokens)
pairs -> collated batches, with the image normalisation on the GPU.

Reference behaviour restated here (dataset.py, tokenizer.py):
  * ImageTextDataset (dataset.py:29-101): {filename: [caption, ...]} JSON; one pair per (existing
    image, string caption); missing files / non-string captions skipped; load errors yield a black
    image and an all-PAD caption (dataset.py:113-128).
  * tokenizer (tokenizer.py:276-313): ByteLevelBPE + BertProcessing(START ... END), padded to and
    truncated at config.MAX_SEQ_LEN inside encode().
  * _pad_or_truncate (dataset.py:149-171): cut to max_seq_len; a full-length sequence whose last id
    is not END gets END written over its last position -- including a PAD tail when the tokenizer
    padded to a longer MAX_SEQ_LEN (the END-overwrite quirk; kept, it changes the targets).
  * collate_fn (dataset.py:173-206): stack; decoder input = tokens[:, :-1], target = tokens[:, 1:].
  * image processor (dataset.py:135 -> AutoImageProcessor): ViT = resize to 224x224 bilinear; CLIP =
    shortest edge -> size (bicubic, long edge int(size * long / short)) + centre crop; then
    rescale 1/255 and normalise.

MI355X split: the PIL resampling stays on the host (it defines the reference's pixels); workers
hand uint8 HWC tiles to the collate, and the rescale + normalise + HWC->CHW runs as ONE HBM-bound
kernel on the batch (mit_image_normalize) when the batch reaches the GPU (to_device), bit-identical
to the processors' float32 numpy arithmetic.
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

import config
import native

VIT_MEAN = VIT_STD = (0.5, 0.5, 0.5)  # tf/utils/constants.py:3-4 (IMAGENET_STANDARD)
CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)  # tf/utils/constants.py:5-6 (OPENAI_CLIP)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


class ImagePreprocessor:
    """Host resample/crop to uint8 (`resize`) + GPU normalise (`normalize`); `__call__` does both,
    returning {"pixel_values": f32 [B,3,S,S] on `device`} like the HF processor."""

    def __init__(self, kind: str = "vit", size: int = 224, device=None):
        if kind not in ("vit", "clip"):
            raise ValueError(f"kind must be 'vit' or 'clip', got {kind}")
        self.kind, self.size = kind, size
        self.mean, self.std = (VIT_MEAN, VIT_STD) if kind == "vit" else (CLIP_MEAN, CLIP_STD)
        self.device = device

    @classmethod
    def for_encoder(cls, name: Optional[str] = None, device=None):
        spec = config.ENCODER_SPECS[name or config.ENCODER_MODEL_NAME]
        return cls("clip" if spec["kind"] == "clip" else "vit", spec["image"], device)

    def resize(self, image) -> np.ndarray:
        """PIL image (any mode) or HWC uint8 array -> uint8 [S, S, 3] (the processor's resampling)."""
        from PIL import Image
        im = image if isinstance(image, Image.Image) else Image.fromarray(np.asarray(image))
        im = im.convert("RGB")
        S = self.size
        if self.kind == "vit":
            return np.asarray(im.resize((S, S), Image.BILINEAR))
        w, h = im.size
        if w <= h:
            nw, nh = S, int(S * h / w)
        else:
            nw, nh = int(S * w / h), S
        a = np.asarray(im.resize((nw, nh), Image.BICUBIC))
        top, left = (nh - S) // 2, (nw - S) // 2
        return a[top:top + S, left:left + S]

    def normalize(self, u8: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """uint8 [B,S,S,3] (any device; moved to the GPU) -> f32 [B,3,S,S] on the GPU."""
        dev = self.device or torch.device("cuda", torch.cuda.current_device())
        u8 = u8.to(dev, non_blocking=True).contiguous()
        B, H, W, _ = u8.shape
        if out is None:
            out = torch.empty(B, 3, H, W, dtype=torch.float32, device=dev)
        native.image_normalize(u8, out, self.mean, self.std)
        return out

    def __call__(self, images, return_tensors: str = "pt"):
        ims = images if isinstance(images, (list, tuple)) else [images]
        u8 = torch.from_numpy(np.stack([self.resize(im) for im in ims]))
        return {"pixel_values": self.normalize(u8)}


def pad_or_truncate(ids: Sequence[int], max_seq_len: int, end_id: int = config.END_TOKEN_ID,
                    pad_id: int = config.PAD_TOKEN_ID) -> List[int]:
    """dataset.py:149-171, quirk included: a full-length sequence not ending in END gets END
    written over its last position."""
    out = list(ids)[:max_seq_len]
    if len(out) == max_seq_len and out[max_seq_len - 1] != end_id:
        out[max_seq_len - 1] = end_id
    if len(out) < max_seq_len:
        out.extend([pad_id] * (max_seq_len - len(out)))
    return out


def load_tokenizer(vocab_path: str = config.VOCAB_PATH, merges_path: str = config.MERGES_PATH,
                   max_len: int = config.MAX_SEQ_LEN):
    """tokenizer.py:276-313: ByteLevelBPE from vocab/merges, BertProcessing(START, END), padding to
    and truncation at max_len."""
    from tokenizers import ByteLevelBPETokenizer
    from tokenizers.processors import BertProcessing
    if not (os.path.exists(vocab_path) and os.path.exists(merges_path)):
        raise FileNotFoundError(f"Tokenizer vocabulary file ('{vocab_path}') or merges file ('{merges_path}') "
                                f"not found.")
    tok = ByteLevelBPETokenizer(vocab=vocab_path, merges=merges_path)
    s, e = tok.token_to_id(config.START_TOKEN), tok.token_to_id(config.END_TOKEN)
    if s is None or e is None:
        raise ValueError("START_TOKEN or END_TOKEN not found in tokenizer vocabulary after loading.")
    tok._tokenizer.post_processor = BertProcessing(sep=(config.END_TOKEN, e), cls=(config.START_TOKEN, s))
    pad = tok.token_to_id(config.PAD_TOKEN)
    if pad is not None:
        tok.enable_padding(pad_id=pad, pad_token=config.PAD_TOKEN, length=max_len)
    tok.enable_truncation(max_length=max_len)
    return tok


class ImageTextDataset(torch.utils.data.Dataset):
    """dataset.py:29-171 with the image left as resized uint8 HWC (normalised later on the GPU)."""

    def __init__(self, image_dir: str, captions_file: str, max_seq_len: int, tokenizer=None,
                 preprocessor: Optional[ImagePreprocessor] = None):
        self.image_dir, self.max_seq_len = image_dir, max_seq_len
        self.tokenizer = tokenizer
        self.pre = preprocessor or ImagePreprocessor.for_encoder()
        self.image_paths: List[str] = []
        self.captions: List[str] = []
        try:
            with open(captions_file, "r", encoding="utf-8") as f:
                data = json.load(f)
        except FileNotFoundError:
            print(f"Error: Captions file not found at {captions_file}. Dataset will be empty.")
            return
        except json.JSONDecodeError:
            print(f"Error: Could not decode JSON from {captions_file}. Dataset will be empty.")
            return
        if not isinstance(data, dict):
            print(f"Error: Captions data from {captions_file} is not in the expected dictionary format.")
            return
        for filename, caps in data.items():
            path = os.path.join(image_dir, filename)
            if not os.path.exists(path):
                print(f"Warning: Image file not found, but listed in captions: {path}. Skipping associated captions.")
                continue
            for c in caps:
                if isinstance(c, str):
                    self.image_paths.append(path)
                    self.captions.append(c)
                else:
                    print(f"Warning: Found non-string caption for image {filename}: {c}. Skipping this caption.")

    def __len__(self):
        return len(self.image_paths)

    def encode(self, caption: str) -> List[int]:
        if self.tokenizer is None:
            self.tokenizer = load_tokenizer()
        enc = self.tokenizer.encode(caption)
        return list(enc.ids if hasattr(enc, "ids") else enc)

    def __getitem__(self, idx: int) -> Dict[str, Any]:
        from PIL import Image
        path = self.image_paths[idx]
        try:
            image = Image.open(path).convert("RGB")
        except Exception as e:  # noqa: BLE001 -- dataset.py:116-128: a dummy item, not a crash
            print(f"Error loading image {path}: {e}. Returning a dummy item.")
            S = self.pre.size
            return {"image_path": "error_loading_image_path",
                    "image": torch.from_numpy(self.pre.resize(Image.new("RGB", (S, S))).copy()),
                    "caption_tokens": torch.full((self.max_seq_len,), config.PAD_TOKEN_ID, dtype=torch.long)}
        ids = pad_or_truncate(self.encode(self.captions[idx]), self.max_seq_len)
        return {"image_path": path, "image": torch.from_numpy(self.pre.resize(image).copy()),
                "caption_tokens": torch.tensor(ids, dtype=torch.long)}


def collate_fn(batch: List[Dict[str, Any]]) -> Dict[str, Any]:
    """dataset.py:173-206 (images stay uint8 [B,S,S,3] until to_device)."""
    caps = torch.stack([b["caption_tokens"] for b in batch])
    return {"image_paths": [b["image_path"] for b in batch], "images": torch.stack([b["image"] for b in batch]),
            "decoder_input_tokens": caps[:, :-1], "target_tokens": caps[:, 1:]}


def to_device(batch: Dict[str, Any], preprocessor: ImagePreprocessor, device=None) -> Dict[str, Any]:
    """Move a collated batch to the GPU; uint8 images are normalised there (one kernel)."""
    dev = device or torch.device("cuda", torch.cuda.current_device())
    out = dict(batch)
    imgs = batch["images"]
    out["images"] = preprocessor.normalize(imgs) if imgs.dtype == torch.uint8 else imgs.to(dev, non_blocking=True)
    out["decoder_input_tokens"] = batch["decoder_input_tokens"].to(dev, non_blocking=True)
    out["target_tokens"] = batch["target_tokens"].to(dev, non_blocking=True)
    return out


def make_dataloader(dataset: ImageTextDataset, batch_size: int = config.BATCH_SIZE, shuffle: bool = True,
                    num_workers: int = 2, seed: int = config.RANDOM_SEED):
    g = torch.Generator().manual_seed(seed)
    return torch.utils.data.DataLoader(dataset, batch_size=batch_size, shuffle=shuffle, num_workers=num_workers,
                                       collate_fn=collate_fn, pin_memory=True, generator=g, drop_last=False)
