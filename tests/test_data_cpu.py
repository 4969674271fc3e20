"""Data path host logic against the reference's rules (dataset.py:29-206,
tokenizer.py:276-313) and the HF processors' golden pixels (tests/golden/preprocess.safetensors,
made by tests/golden/make_preprocess_fixture.py): the uint8 resampling / crop geometry here, the GPU
normalisation in test_data_gpu.py."""
import json
import os

import numpy as np
import pytest
import torch
from PIL import Image
from safetensors import safe_open

import config
import data

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "preprocess.safetensors")


def _gold():
    with safe_open(GOLD, "pt") as f:
        return json.loads(f.metadata()["meta"]), {k: f.get_tensor(k) for k in f.keys()}


def test_pad_or_truncate_rules_and_end_overwrite_quirk():
    S, E, P = 1, 2, 0
    f = lambda ids, n: data.pad_or_truncate(ids, n, end_id=E, pad_id=P)  # noqa: E731
    assert f([S, 5, 6, E], 8) == [S, 5, 6, E, P, P, P, P]  # short: padded
    assert f([S, 5, 6, 7, 8, 9, E], 5) == [S, 5, 6, 7, E]  # truncated: last -> END
    assert f([S, 5, 6, E], 4) == [S, 5, 6, E]  # exact fit already ending in END: unchanged
    # the tokenizer pads to MAX_SEQ_LEN first; cut shorter, the PAD tail's last slot becomes END
    assert f([S, 5, E, P, P, P, P, P, P, P], 6) == [S, 5, E, P, P, E]
    assert f([], 3) == [P, P, P]


def test_collate_shifts_tokens():
    b = [{"image_path": f"p{i}", "image": torch.full((4, 4, 3), i, dtype=torch.uint8),
          "caption_tokens": torch.tensor([1, 10 + i, 11 + i, 2, 0])} for i in range(3)]
    out = data.collate_fn(b)
    assert out["images"].shape == (3, 4, 4, 3) and out["images"].dtype == torch.uint8
    assert torch.equal(out["decoder_input_tokens"], torch.tensor([[1, 10, 11, 2], [1, 11, 12, 2], [1, 12, 13, 2]]))
    assert torch.equal(out["target_tokens"], torch.tensor([[10, 11, 2, 0], [11, 12, 2, 0], [12, 13, 2, 0]]))
    assert out["image_paths"] == ["p0", "p1", "p2"]


def test_dataset_pairs_and_skips(tmp_path):
    d = tmp_path / "images"
    d.mkdir()
    Image.fromarray(np.zeros((30, 40, 3), np.uint8)).save(d / "a.png")
    Image.fromarray(np.full((50, 20, 3), 200, np.uint8)).save(d / "b.png")
    (d / "bad.png").write_bytes(b"not an image")
    caps = {"a.png": ["one", "two", 3], "b.png": ["three"], "missing.png": ["x"], "bad.png": ["y"]}
    cf = tmp_path / "captions.json"
    cf.write_text(json.dumps(caps))

    class Tok:  # stands in for the BPE tokenizer: START, one id per word, END, padded to 10
        def encode(self, s):
            ids = [config.START_TOKEN_ID] + [10 + len(w) for w in s.split()] + [config.END_TOKEN_ID]
            return ids + [config.PAD_TOKEN_ID] * (10 - len(ids))

    ds = data.ImageTextDataset(str(d), str(cf), 6, tokenizer=Tok(), preprocessor=data.ImagePreprocessor("vit", 32))
    assert len(ds) == 4  # one, two (3 skipped: not a string), three, y; missing.png skipped
    it = ds[0]
    assert it["image"].shape == (32, 32, 3) and it["image"].dtype == torch.uint8
    assert it["caption_tokens"].tolist() == [1, 13, 2, 0, 0, 2]  # END-overwrite quirk at max_seq_len 6
    bad = ds[3]
    assert bad["image_path"] == "error_loading_image_path"
    assert bad["caption_tokens"].tolist() == [config.PAD_TOKEN_ID] * 6
    empty = data.ImageTextDataset(str(d), str(tmp_path / "nope.json"), 6, tokenizer=Tok())
    assert len(empty) == 0


@pytest.mark.parametrize("kind,key,size", [("vit", "vit", 224), ("clip", "clip", 224), ("clip", "clip336", 336)])
def test_host_resample_geometry_matches_processor(kind, key, size):
    """uint8 resampling + crop, normalised in numpy float32 the way the kernel does, equals the HF
    processor's pixel_values bit for bit (so the GPU kernel only has to match this arithmetic)."""
    meta, T = _gold()
    pre = data.ImagePreprocessor(kind, size)
    ref = T[key].numpy()
    for i in range(ref.shape[0]):
        u8 = pre.resize(T[f"img{i}"].numpy())
        assert u8.shape == (size, size, 3) and u8.dtype == np.uint8
        m, s = np.array(pre.mean, np.float32), np.array(pre.std, np.float32)
        x = ((u8.astype(np.float32) / np.float32(255.0)) - m) / s
        assert np.array_equal(x.transpose(2, 0, 1), ref[i]), (key, i)
