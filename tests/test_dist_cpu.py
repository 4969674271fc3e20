"""Data-parallel gradient semantics on CPU (gloo, world_size 2) against the reference.

The dp2_tiny fixture is ONE reference train step (train.py:62-123) at global batch 8 whose two
halves hold different numbers of PAD targets. Each rank here computes its half with the CPU oracle
standing in for the GPU kernels, normalises by the all-reduced GLOBAL non-PAD count through
dist.DataParallel.all_reduce_count, writes its gradients into the same flat, backward-ordered
buffer the GPU path uses, and lets DataParallel all-reduce the buckets exactly as the HIP backward
announces them (grads_ready spans). The summed gradients must equal the reference's single-process
gradients, i.e. per-rank mean-of-means (the naive DDP average) is NOT what is computed.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import fixtures as FX


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Model:
    """The pieces of ImageToTextModel that DataParallel touches (store only, no encoder)."""

    def __init__(self, store):
        self.store = store


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from decoder import decoder_entries, reference_to_flat
        from dist import DataParallel
        from oracle import ref_cpu as R
        from params import FlatParams
        torch.set_num_threads(2)
        meta, T = FX.load("dp2_tiny")
        st = FX.state(meta)
        enc, dec = FX.enc_desc(meta), FX.dec_desc(meta)
        imgs = torch.randn(0)  # placeholder for type
        import procedural as P
        imgs = P.make_images(meta["B"], meta["image_size"], meta["seed"] + 1)
        cap = P.make_captions(meta["B"], meta["cap_len"], dec["vocab"], meta["seed"] + 2, meta["lengths"])
        di, tg = cap[:, :-1], cap[:, 1:]
        half = meta["B"] // world
        sl = slice(rank * half, (rank + 1) * half)
        E = enc["hidden"]
        store = FlatParams(decoder_entries(dec["vocab"], dec["d"], dec["layers"], dec["ff"],
                                           E if E != dec["d"] else None), torch.device("cpu"), torch.float32)
        dp = DataParallel(_Model(store), overlap=True)
        names = FX.trainable_names(meta)
        leaves = {k: st[k].clone().requires_grad_(True) for k in names}
        qp = dict(st)
        qp.update(leaves)
        logits = R.model_forward(qp, imgs[sl], di[sl], enc, dec, meta["mode"])
        count = (tg[sl] != 0).sum().float().reshape(1)
        dp.all_reduce_count(count)
        loss_sum = torch.nn.functional.cross_entropy(logits.reshape(-1, logits.shape[-1]), tg[sl].reshape(-1),
                                                     ignore_index=0, reduction="sum")
        (loss_sum / count).backward()
        flat = reference_to_flat({k: v.grad for k, v in leaves.items()}, dec["layers"], dec["d"])
        for k, v in flat.items():
            store.g(k).copy_(v)
        # announce buckets in the order the HIP backward finishes them
        dp.grads_ready("fc_out.weight", "fc_out.bias")
        for l in reversed(range(dec["layers"])):
            dp.grads_ready(f"layers.{l}.linear2.weight", f"layers.{l}.norm1.bias")
        dp.grads_ready("cross_kv.weight", store.names()[-1])
        loss = (loss_sum / count).detach().reshape(1)
        dp.finish_backward(loss)
        if rank == 0:
            q.put((loss.item(), store.grad.clone(), store.names()))
    finally:
        dist.destroy_process_group()


def test_dp2_gloo_matches_single_process_reference():
    meta, T = FX.load("dp2_tiny")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    loss, grad, names = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert abs(loss - T["loss"].item()) < 1e-5
    # the reference grads are post-clip (clip 5.0): scale ours the same way
    from decoder import decoder_entries, flat_to_reference
    from params import FlatParams
    dec, enc = FX.dec_desc(meta), FX.enc_desc(meta)
    E = enc["hidden"]
    store = FlatParams(decoder_entries(dec["vocab"], dec["d"], dec["layers"], dec["ff"],
                                       E if E != dec["d"] else None), torch.device("cpu"), torch.float32)
    store.grad.copy_(grad)
    total = float(grad.double().norm())
    assert abs(total - T["grad_total_norm_preclip"].item()) < 1e-4 * total
    coef = min(1.0, 5.0 / (total + 1e-6))

    class GV:
        def p(self, n):
            return store.g(n)

    ref_named = flat_to_reference(GV(), dec["layers"], dec["d"])
    if "projection.weight" in store.index:
        ref_named["projection.weight"] = store.g("projection.weight")
        ref_named["projection.bias"] = store.g("projection.bias")
    for k in FX.trainable_names(meta):
        FX.compare_stat("grad1", k, ref_named[k] * coef, T, meta, rtol=1e-3, atol=1e-6, scale_tol=1e-4)
