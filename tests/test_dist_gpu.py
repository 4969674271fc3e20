"""The data-parallel train step through the REAL HIP path: two ranks (gloo; RCCL needs one GPU per
rank, the box has one) share cuda:0 and run ImageToTextModel.train_step(dist=DataParallel) on the two
halves of the dp2_tiny batch — the HIP backward announces its gradient buckets (grads_ready) from
the weight-gradient side stream, DataParallel all-reduces them and the global non-PAD count.
The summed gradients, the loss and the AdamW update must equal the reference's single-process
step at the global batch (tests/golden/dp2_tiny: train.py:62-123 at B = 8, unequal PAD per half)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

import fixtures as FX

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, backend="gloo"):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.join(here, "..", "multimodal-image-transformer_amd"), os.path.join(here, "golden")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    if backend == "nccl":
        torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        import fixtures as FX
        import optim
        from dist import DataParallel
        from model_util import build_model
        import procedural as P
        meta, T = FX.load("dp2_tiny")
        m, _ = build_model(meta, torch.float32)
        m.train()
        dp = DataParallel(m, overlap=True)
        imgs = P.make_images(meta["B"], meta["image_size"], meta["seed"] + 1)
        cap = P.make_captions(meta["B"], meta["cap_len"], meta["dec"]["vocab"], meta["seed"] + 2, meta["lengths"])
        half = meta["B"] // world
        sl = slice(rank * half, (rank + 1) * half)
        opt = optim.AdamW(m.store, lr=meta["lr"], betas=tuple(meta["betas"]), eps=meta["eps"],
                          weight_decay=meta["weight_decay"])
        before = m.state_dict()
        loss = m.train_step(imgs[sl].cuda(), cap[sl, :-1].cuda(), cap[sl, 1:].cuda(), dist=dp)
        torch.cuda.synchronize()
        grad = m.store.grad.clone().cpu()
        opt.step(meta["clip"])
        torch.cuda.synchronize()
        after = m.state_dict()
        if rank == 0:
            names = FX.trainable_names(meta)
            # numpy (pickled by value): the worker may exit before the parent reads the queue
            q.put((loss.item(), grad.numpy(), opt.norm_t.cpu().tolist(),
                   {k: (after[k] - before[k]).cpu().numpy() for k in names}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,backend", [(2, "gloo"), (1, "nccl")])
def test_dp2_train_step_on_hip_path_matches_reference(world, backend):
    """world 2 / gloo: the two halves on cuda:0. world 1 / nccl: ONE rank over RCCL (the backend the
    driver's multi-GPU runs use; this box has one GPU, and RCCL takes one GPU per rank) -- the same
    DataParallel path with ProcessGroupNCCL: the bucket all-reduces issued under the weight-gradient
    side stream (decoder._SideStream.under) and joined before clip + AdamW."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    meta, T = FX.load("dp2_tiny")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, backend)) for r in range(world)]
    for p in procs:
        p.start()
    loss, grad, (total, coef), deltas = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert abs(loss - T["loss"].item()) < 1e-4
    assert abs(total - T["grad_total_norm_preclip"].item()) < 1e-3 * total
    _check_against_reference(meta, T, grad, coef, {k: torch.from_numpy(v) for k, v in deltas.items()})


def _check_against_reference(meta, T, grad, coef, deltas):
    """The flat gradient (pre-clip, times the clip coefficient) and the AdamW update of every trainable
    tensor against the reference's step (dp2_tiny's grad1 / delta1 statistics)."""
    from decoder import decoder_entries, flat_to_reference
    from params import FlatParams
    dec, enc = FX.dec_desc(meta), FX.enc_desc(meta)
    E = enc["hidden"]
    store = FlatParams(decoder_entries(dec["vocab"], dec["d"], dec["layers"], dec["ff"],
                                       E if E != dec["d"] else None), torch.device("cpu"), torch.float32)
    store.grad.copy_(torch.from_numpy(grad))

    class GV:
        vocab = dec["vocab"]

        def p(self, n):
            return store.g(n)

    named = flat_to_reference(GV(), dec["layers"], dec["d"])
    if "projection.weight" in store.index:
        named["projection.weight"] = store.g("projection.weight")
        named["projection.bias"] = store.g("projection.bias")
    for k in FX.trainable_names(meta):
        FX.compare_stat("grad1", k, named[k] * coef, T, meta, rtol=2e-3, atol=2e-6, scale_tol=1e-3, outlier_frac=2e-3)
        FX.compare_stat("delta1", k, deltas[k], T, meta, rtol=2e-3, atol=2e-6)


def _train_main_worker(rank, world, port, q):
    """train.main on 2 synthetic global batches of 8 pairs (dropout off): world 1 = one process with
    the whole batch, world 2 = two gloo ranks on cuda:0 with their halves (shard_batches)."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "..", "multimodal-image-transformer_amd"))
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                          WORLD_SIZE=str(world), MIT_DIST_BACKEND="gloo")
    else:
        os.environ.pop("WORLD_SIZE", None)
    torch.cuda.set_device(0)
    import config
    config.DECODER_DROPOUT = 0.0
    config.WARMUP_STEPS = 0
    config.LOG_INTERVAL = 0
    import train
    hist = train.main(["--batches", "2", "--batch-size", "8", "--seq-len", "16", "--epochs", "1"])
    if rank == 0:
        q.put(hist)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def _run_train_main(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_train_main_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    hist = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return hist


def test_train_main_dp2_matches_one_rank_global_batch():
    """train.main (reference train.py:62-123 loop, its main's DP wiring): 2 ranks x half batches give
    the 1-rank global-batch epoch losses (train mean over the 2 batches, then validation after the
    updates). bf16 GEMMs on different M sum in different orders: 2e-3 relative."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    one = _run_train_main(1)
    two = _run_train_main(2)
    assert len(one) == len(two) == 1
    (t1, v1), (t2, v2) = one[0], two[0]
    assert abs(t1 - t2) <= 2e-3 * abs(t1), (t1, t2)
    assert abs(v1 - v2) <= 2e-3 * abs(v1), (v1, v2)


def test_bench_spawns_its_own_ranks():
    """`bench.py --gpus 2` with no launcher starts its 2 rank processes itself (gloo here: one GPU);
    the JSON line reports n_gpus 2 and the whole-job pairs/s."""
    import json
    import subprocess
    import sys
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MIT_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--batch", "8", "--no-cpu-baseline", "--no-roofline", "--no-also"],
                       env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["global_batch"] == 16 and rec["value"] > 0



def _replay_worker(port, q):
    """ONE rank over RCCL (ProcessGroupNCCL, world size 1): the launch path bench.py --gpus N takes on the
    driver's 8-GPU node -- DataParallel(overlap=True), train_step(next_images=...) with the encoder prefetch,
    steps recorded by native.record (the bucket all-reduces and the count all-reduce as recorded host steps
    between native plans) and replayed by mit_plan_run. Two models from the same weights: "eager" runs 5
    eager steps; "replay" runs step 1 eager (arenas, optimizer state and split-K scratch are set up by a real
    step first, as bench.py's warm-up does), records steps 2-3 (run for real while recording) and replays
    the two programs as steps 4-5. Reports each step's loss, the final master / AdamW moments / dropout seed
    of both, and the eager run's step-1 loss, gradient, clip norm and update (the reference comparison).
    fp32 without dropout (the reference's step) and bf16 with dropout 0.1 (the bench's arithmetic: the
    replayed steps must advance the dropout seed and the AdamW step exactly as eager steps do)."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.join(here, "..", "multimodal-image-transformer_amd"), os.path.join(here, "golden")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        import fixtures as FX
        import native
        import optim
        from dist import DataParallel
        from model_util import build_model
        import procedural as P
        meta, T = FX.load("dp2_tiny")
        imgs = P.make_images(meta["B"], meta["image_size"], meta["seed"] + 1).cuda()
        cap = P.make_captions(meta["B"], meta["cap_len"], meta["dec"]["vocab"], meta["seed"] + 2, meta["lengths"])
        di, tg = cap[:, :-1].contiguous().cuda(), cap[:, 1:].contiguous().cuda()
        names = FX.trainable_names(meta)
        out = {"backend": dist.get_backend()}
        for tag, dtype, p in (("f32", torch.float32, 0.0), ("bf16", torch.bfloat16, 0.1)):
            runs = {}
            for mode in ("eager", "replay"):
                m, _ = build_model(meta, dtype, dropout=p)
                m.train()
                dp = DataParallel(m, overlap=True)
                opt = optim.AdamW(m.store, lr=meta["lr"], betas=tuple(meta["betas"]), eps=meta["eps"],
                                  weight_decay=meta["weight_decay"])
                held = {}

                def step():
                    held["loss"] = m.train_step(imgs, di, tg, dist=dp, next_images=imgs)
                    opt.step(meta["clip"])

                # step 1, eager in both runs; the eager run keeps its gradient and update for the reference
                before = {k: v.clone() for k, v in m.state_dict().items() if k in names}
                held["loss"] = m.train_step(imgs, di, tg, dist=dp, next_images=imgs)
                torch.cuda.synchronize()
                grad1 = m.store.grad.clone().cpu().numpy()
                opt.step(meta["clip"])
                after = m.state_dict()
                first = dict(loss=held["loss"].item(), grad=grad1, norm=opt.norm_t.cpu().tolist(),
                             delta={k: (after[k] - before[k]).cpu().numpy() for k in names})
                losses = [first["loss"]]
                if mode == "eager":
                    for _ in range(4):
                        step()
                        losses.append(held["loss"].item())
                else:
                    progs = []
                    for _ in range(2):
                        progs.append(native.record(step))
                        losses.append(held["loss"].item())
                    for i in range(2):
                        opt._sync_lr()
                        progs[i].run()
                        losses.append(held["loss"].item())
                    out.setdefault("launches", progs[0].launches())
                torch.cuda.synchronize()
                st = m.store
                runs[mode] = dict(losses=losses, master=st.master.cpu().numpy(), exp_avg=st.exp_avg.cpu().numpy(),
                                  exp_avg_sq=st.exp_avg_sq.cpu().numpy(), seed=m.seed_t.cpu().numpy(),
                                  first=first if mode == "eager" else None)
                del m, dp, opt, held
                torch.cuda.synchronize()
            out[tag] = runs
        q.put(out)
    finally:
        dist.destroy_process_group()


def test_rccl_one_rank_native_replay_matches_eager_and_reference():
    """The driver's N-GPU launch path (native record / replay with the DP collectives as host steps and the
    encoder prefetch), run under RCCL at world size 1 on this one-GPU box: replayed steps bit-identical to
    eager ones (losses, master weights, AdamW moments, dropout seed), step 1 equal to the reference's
    single-process step on dp2_tiny (train.py:62-123 at B = 8)."""
    import numpy as np
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    meta, T = FX.load("dp2_tiny")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    pr = ctx.Process(target=_replay_worker, args=(port, q))
    pr.start()
    out = q.get(timeout=300)
    pr.join(timeout=60)
    assert pr.exitcode == 0
    assert out["backend"] == "nccl" and out["launches"] > 0
    for tag in ("f32", "bf16"):
        e, r = out[tag]["eager"], out[tag]["replay"]
        assert e["losses"] == r["losses"], (tag, e["losses"], r["losses"])
        assert len(set(e["losses"])) > 1, (tag, e["losses"])  # the steps did update the weights
        for k in ("master", "exp_avg", "exp_avg_sq", "seed"):
            assert np.array_equal(e[k], r[k]), (tag, k)
    f = out["f32"]["eager"]["first"]
    assert abs(f["loss"] - T["loss"].item()) < 1e-4
    total, coef = f["norm"]
    assert abs(total - T["grad_total_norm_preclip"].item()) < 1e-3 * total
    _check_against_reference(meta, T, f["grad"], coef, {k: torch.from_numpy(v) for k, v in f["delta"].items()})
