"""Build the MI355X model from a golden fixture (same procedural weights the reference ran with).
Test infrastructure only."""
import torch

import fixtures as FX


def build_model(meta, dtype, dropout=0.0):
    import config
    from encoder import VisionEncoder
    from model import ImageToTextModel
    enc_d = FX.enc_desc(meta)
    spec = dict(kind=enc_d["kind"], hidden=enc_d["hidden"], layers=enc_d["layers"], heads=enc_d["heads"],
                mlp=enc_d["mlp"], image=enc_d["image"], patch=enc_d["patch"], eps=enc_d["eps"])
    st = FX.state(meta)
    enc = VisionEncoder(spec, torch.device("cuda"), dtype)
    enc.load_hf_state_dict({k: v for k, v in st.items() if k.startswith("encoder.")})
    dec = FX.dec_desc(meta)
    m = ImageToTextModel(dec["vocab"], dec["d"], dec["heads"], dec["layers"], dec["ff"], dec["max_seq_len"], dropout,
                         0, encoder=enc, memory_mode=meta["mode"], dtype=dtype)
    m.load_state_dict({k: v for k, v in st.items() if not k.startswith("encoder.")}, strict=True)
    return m, st
