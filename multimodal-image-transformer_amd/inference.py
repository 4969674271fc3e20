"""Caption generation from a trained checkpoint (reference inference.py), batched on the MI355X path.

The reference captions one image per call: model.generate() greedy decode with a full-prefix
recompute per token (inference.py:84-91 -> model.py:171-242), then trims the ids at the first END,
drops a leading START (inference.py:98-115) and cleans the decoded text (inference.py:116-126).
Here the same ids come from ImageToTextModel.generate_batch (KV cache, one hipGraph-replayed token
step for the whole batch, decode.hip); postprocess_ids / clean_text restate the reference's
post-processing so a batch yields the reference's caption for every image.
"""
from __future__ import annotations

import argparse
import os
from typing import Callable, List, Optional, Sequence

import torch

import config


def postprocess_ids(ids: Sequence[int], start_token_id: int, end_token_id: int) -> List[int]:
    """inference.py:98-113: keep the ids before the first END (all of them when there is none),
    then drop one leading START."""
    ids = list(ids)
    if end_token_id in ids:
        ids = ids[:ids.index(end_token_id)]
    if ids and ids[0] == start_token_id:
        ids = ids[1:]
    return ids


def clean_text(text: str, unk_token: str = config.UNK_TOKEN) -> str:
    """inference.py:120-126: remove every UNK token string, strip, collapse runs of whitespace."""
    return " ".join(text.replace(unk_token, "").strip().split())


def load_model(checkpoint_path: str, vocab_size: Optional[int] = None, device=None, dtype=None,
               memory_mode: Optional[str] = None):
    """inference.py:52-68: build ImageToTextModel with config's decoder geometry and load the weights.
    .safetensors (the reference's format) or a .pt written by train.save_checkpoint, read with
    torch.load(weights_only=True) — nothing in the file is executed."""
    from model import ImageToTextModel
    if not os.path.exists(checkpoint_path):
        raise FileNotFoundError(f"Checkpoint file not found: {checkpoint_path}")
    if checkpoint_path.endswith(".safetensors"):
        from safetensors.torch import load_file
        sd = load_file(checkpoint_path)
    else:
        ck = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        sd = ck.get("model_state_dict", ck)
    if vocab_size is None:
        vocab_size = sd["decoder.fc_out.weight"].shape[0] if "decoder.fc_out.weight" in sd else config.VOCAB_SIZE
    model = ImageToTextModel(vocab_size, config.DECODER_EMBED_DIM, config.DECODER_HEADS, config.DECODER_LAYERS,
                             config.DECODER_FF_DIM, config.MAX_SEQ_LEN, config.DECODER_DROPOUT, config.PAD_TOKEN_ID,
                             device=device, dtype=dtype, memory_mode=memory_mode)
    model.load_state_dict(sd)
    model.eval()
    return model


def generate_captions(model, images, decode: Optional[Callable[[List[int]], str]] = None,
                      start_token_id: int = config.START_TOKEN_ID, end_token_id: int = config.END_TOKEN_ID,
                      max_len: int = config.MAX_SEQ_LEN, batch_size: int = 256):
    """Captions for a list of PIL images / HWC arrays or a [B,3,H,W] pixel tensor, `batch_size` images
    per batched decode. Returns [(processed ids, text)] — text is None without a `decode` function
    (the BPE tokenizer, tokenizer.py, is a host-side library outside this path)."""
    if isinstance(images, torch.Tensor):
        pv = images if images.dim() == 4 else images.unsqueeze(0)
    else:
        pv = model.image_processor(images=list(images), return_tensors="pt")["pixel_values"]
    # at most two batches on the device: the current one and the next, whose encoder runs beside this
    # batch's token steps (generate_batch next_images); the next iteration passes that very tensor object,
    # which generate_batch recognises as prefetched
    starts = list(range(0, pv.shape[0], batch_size))

    def dev(i):
        return pv[i:i + batch_size].to(model.device).float()
    out = []
    chunk = dev(starts[0]) if starts else None
    for j in range(len(starts)):
        nxt = dev(starts[j + 1]) if j + 1 < len(starts) else None
        ids = model.generate_batch(chunk, start_token_id, end_token_id, max_len=max_len, next_images=nxt)
        chunk = nxt
        for seq in ids:
            p = postprocess_ids(seq, start_token_id, end_token_id)
            out.append((p, clean_text(decode(p)) if decode is not None else None))
    return out


def generate_caption(image, model, decode=None) -> str:
    """inference.py:17-128 for one image (path, PIL image or pixel tensor) with a loaded model."""
    if isinstance(image, str):
        if not os.path.exists(image):
            raise FileNotFoundError(f"Image file not found: {image}")
        from PIL import Image
        image = Image.open(image).convert("RGB")
    ids, text = generate_captions(model, image if isinstance(image, torch.Tensor) else [image], decode)[0]
    return text if text is not None else " ".join(map(str, ids))


def _tokenizer_decode():
    """The trained BPE tokenizer's decode when its files exist (config.VOCAB_PATH / MERGES_PATH), else None."""
    vocab, merges = getattr(config, "VOCAB_PATH", None), getattr(config, "MERGES_PATH", None)
    if not vocab or not merges or not (os.path.exists(vocab) and os.path.exists(merges)):
        return None
    from tokenizers import ByteLevelBPETokenizer
    tok = ByteLevelBPETokenizer(vocab, merges)
    return lambda ids: tok.decode(ids, skip_special_tokens=False)


def main(argv=None):
    ap = argparse.ArgumentParser(description="Generate captions for images with a trained checkpoint.")
    ap.add_argument("--image_path", nargs="+", required=True, help="one or more image files")
    ap.add_argument("--checkpoint_path", required=True, help=".safetensors or .pt checkpoint")
    ap.add_argument("--batch_size", type=int, default=256)
    args = ap.parse_args(argv)
    from PIL import Image
    model = load_model(args.checkpoint_path)
    for p in args.image_path:
        if not os.path.exists(p):
            raise FileNotFoundError(f"Image file not found: {p}")
    ims = [Image.open(p).convert("RGB") for p in args.image_path]
    for p, (ids, text) in zip(args.image_path, generate_captions(model, ims, _tokenizer_decode(),
                                                                  batch_size=args.batch_size)):
        print(f"{p}: {text if text is not None else ids}")


if __name__ == "__main__":
    main()
