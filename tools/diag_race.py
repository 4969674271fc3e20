"""Race bisection at the bench size: the decoder forward (train arena, dropout off) run alone and
then beside the encoder prefetch on the second stream; every saved activation of the forward is
compared bitwise with the alone run. Usage (GPU box): python tools/diag_race.py"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

A = argparse.Namespace(workload="train", memory_mode="patches", vocab=10000, dtype="bf16", batch=64, seq_len=64)


def snap(Ac, L):
    out = {"x0": Ac.x0, "kv": Ac.kv, "logits": Ac.logits}
    for l in range(L):
        out[f"qkv{l}"] = Ac.qkv[l]
        out[f"os{l}"] = Ac.os[l]
        out[f"oc{l}"] = Ac.oc[l]
        out[f"qc{l}"] = Ac.qc[l]
        out[f"h{l}"] = Ac.h[l]
        for k in range(3):
            out[f"z{l}.{k}"] = Ac.z[l][k]
            out[f"xs{l}.{k}"] = Ac.xs[l][k]
    return {k: v.clone() for k, v in out.items()}


def main():
    torch.cuda.set_device(0)
    m, opt = bench.build(A, 0)
    images, di, tg = bench.synthetic_batch(64, 64, 10000, torch.device("cuda", 0), 1000, m.encoder.image)
    m.train_step(images, di, tg)  # arenas
    dec = m.decoder
    tokens = di.to(torch.int64).contiguous()
    B, T = tokens.shape
    order = None

    def fwd(noise):
        mem, mem_ld, S, _, _ = m._encode_memory(images, refresh=False)
        if noise:
            m.prefetch_encoder(images)
        Ac = dec.acts(B, T, S, True)
        dec.run_forward(tokens, mem, mem_ld, S, Ac, m.seed_t, True, drop_p=0.0)
        torch.cuda.synchronize()
        s = snap(Ac, dec.L)
        m._prefetched = None
        m._enc_slot = 0
        return s

    ref = fwd(False)
    print("alone twice equal:", all(torch.equal(ref[k], v) for k, v in fwd(False).items()), flush=True)
    for r in range(6):
        s = fwd(True)
        bad = [k for k in ref if not torch.equal(ref[k], s[k])]
        first = bad[0] if bad else None
        extra = ""
        if first:
            d = (ref[first].float() - s[first].float()).abs()
            nz = (d > 0).nonzero()
            extra = f" first={first} n_diff={nz.shape[0]} max={d.max().item():.3e} rows={sorted(set(nz[:, 0].tolist()))[:12]}"
        print(f"round {r}: {len(bad)} tensors differ{extra}", flush=True)
        if bad:
            print("   ", bad[:40], flush=True)


if __name__ == "__main__":
    main()
