"""Training loop surface of the reference train.py, on the MI355X train step.

``train_one_epoch`` / ``evaluate`` keep the reference signatures (train.py:62, 125) and semantics:
per batch zero_grad -> forward -> criterion -> backward -> clip_grad_norm_(grad_clip_value)
-> optimizer.step() -> scheduler.step(); the epoch returns the mean batch loss. Two ways to run it:
  * the fused path (optim.AdamW + the reference criterion, train.py:319-327): forward + CE +
    backward are ONE kernel sequence (model.train_step) and clip + AdamW one more
    (optim.AdamW.step); the per-batch loss stays on the device and the reference's per-step
    ``loss.item()`` sync (train.py:109) becomes one sync per ``log_interval`` batches;
  * any other optimizer / criterion (torch.optim.AdamW(model.parameters()), label smoothing, ...):
    the reference's own call sequence through autograd (model.forward's backward is the HIP
    backward).
``main()`` runs the loop on synthetic batches (the dataset / tokenizer / W&B / Hub plumbing of the
reference main() is out of scope: SURVEY.md §2a) and writes reference-format checkpoints.
"""
from __future__ import annotations

import argparse
import math
import os
import sys
import time

import torch

import config
import optim
from model import ImageToTextModel


def _lr_of(optimizer):
    return optimizer.param_groups[0]["lr"]


def _fused_loss_ok(model, criterion) -> bool:
    """The fused step computes nn.CrossEntropyLoss(ignore_index=PAD) with mean reduction
    (train.py:327); any other criterion runs through autograd on the returned logits."""
    if criterion is None:
        return True
    return (isinstance(criterion, torch.nn.CrossEntropyLoss) and criterion.ignore_index == model.decoder_pad_idx
            and criterion.reduction == "mean" and criterion.weight is None and criterion.label_smoothing == 0.0)


def _staged(model, dataloader):
    """Batches on the device. Images go to the GPU once, so the next step can consume the encoder
    output that model.prefetch_encoder computed for this very tensor one step earlier; uint8
    batches (data.collate_fn) are normalised there by one kernel (model.image_processor)."""
    for b in dataloader:
        b = dict(b)
        if b["images"].dtype == torch.uint8:
            b["images"] = model.image_processor.normalize(b["images"])
        else:
            b["images"] = b["images"].to(model.device, non_blocking=True)
        yield b


def train_one_epoch(model, dataloader, optimizer, criterion, device, grad_clip_value, scheduler, epoch,
                    log_interval, wandb_run, dist=None):
    """train.py:62-123. Returns the average training loss of the epoch.

    With the fused optimizer (optim.AdamW) and the reference criterion, each batch is ONE kernel
    sequence (model.train_step: forward + CE + backward, no host sync) plus optimizer.step(clip).
    With any other optimizer (e.g. torch.optim.AdamW over model.parameters()) or criterion, the
    reference's own call sequence runs (train.py:80-100): zero_grad, logits = model(...),
    loss = criterion(...), loss.backward() (the HIP backward via autograd), clip_grad_norm_,
    optimizer.step()."""
    model.train()
    fused = isinstance(optimizer, optim.AdamW) and _fused_loss_ok(model, criterion)
    if dist is not None and not fused:
        raise ValueError("data-parallel training runs the fused step: pass optim.AdamW and the reference criterion")
    total = torch.zeros(1, dtype=torch.float32, device=model.device)
    # failure detection: the index of the first batch whose loss is NaN / inf, tracked on the
    # device (no per-step sync; the reference's all-PAD rows give NaN, dataset.py:116-130). Checked at the end
    # of the epoch and, single-process, at every log point. Data parallel: only at the end of the epoch, which
    # every rank reaches after the same steps (only rank 0 logs; a mid-epoch raise on one rank would leave the
    # others blocked in the next step's all-reduce). config.NONFINITE_LOSS = "warn" (default: the reference
    # trains on through a NaN loss) prints the batch index, "raise" stops with NonFiniteLossError.
    first_bad = torch.full((1,), -1, dtype=torch.int64, device=model.device)
    n = 0
    it = _staged(model, dataloader)
    batch = next(it, None)
    i = -1
    while batch is not None:
        i += 1
        nxt = next(it, None)
        if fused:
            optimizer.zero_grad()
            # the frozen encoder of the NEXT batch runs on a second stream during this step
            loss = model.train_step(batch["images"], batch["decoder_input_tokens"], batch["target_tokens"], dist=dist,
                                    next_images=nxt["images"] if nxt is not None else None)
            optimizer.step(grad_clip_value if grad_clip_value > 0 else 0.0)
        else:
            optimizer.zero_grad()
            logits = model(batch["images"], batch["decoder_input_tokens"])
            tgt = batch["target_tokens"].to(model.device)
            if _fused_loss_ok(model, criterion):  # the reference criterion: the CE row kernel (mit_hip::cross_entropy)
                import ops
                loss = ops.load().cross_entropy(logits, tgt.to(torch.int64), model.decoder_pad_idx)[0]
            else:
                loss = criterion(logits.view(-1, logits.size(-1)), tgt.reshape(-1))
            loss.backward()
            if grad_clip_value > 0:
                torch.nn.utils.clip_grad_norm_(model.parameters(), grad_clip_value)
            optimizer.step()
            loss = loss.detach().reshape(1)
        if scheduler:
            scheduler.step()
        total += loss
        bad = ~torch.isfinite(loss)
        first_bad.copy_(torch.where(bad & (first_bad < 0), torch.full_like(first_bad, i), first_bad))
        n += 1
        if log_interval and (i + 1) % log_interval == 0:
            if dist is None:
                _check_finite(first_bad, epoch)
            lv = loss.item()
            print(f"epoch {epoch + 1} batch {i + 1}: loss {lv:.4f} lr {_lr_of(optimizer):.2e}", flush=True)
            if wandb_run:
                wandb_run.log({"train_batch_loss": lv, "learning_rate": _lr_of(optimizer),
                               "global_step": epoch * max(1, len(dataloader)) + i + 1})
        batch = nxt
    _check_finite(first_bad, epoch)
    return (total / max(n, 1)).item()


class NonFiniteLossError(FloatingPointError):
    """A training batch produced a NaN / inf loss (e.g. a batch whose targets are all PAD)."""


def _check_finite(first_bad: torch.Tensor, epoch: int):
    """Report the first non-finite batch loss of the epoch: raise (config.NONFINITE_LOSS == "raise") or
    print it once (the default, "warn": training goes on as the reference's does)."""
    i = int(first_bad.item())
    if i < 0:
        return
    msg = (f"epoch {epoch + 1}: non-finite training loss at batch {i + 1} (step index {i}); "
           f"the parameters were updated with it -- check the batch (all-PAD targets give NaN)")
    if str(getattr(config, "NONFINITE_LOSS", "warn")).lower() == "raise":
        raise NonFiniteLossError(msg)
    if not getattr(first_bad, "_mit_reported", False):  # once per epoch
        print("warning: " + msg, file=sys.stderr, flush=True)
        first_bad._mit_reported = True


@torch.no_grad()
def evaluate(model, dataloader, criterion, device):
    """train.py:125-151: mean over batches of the criterion (CE(ignore PAD)), no dropout."""
    model.eval()
    total = torch.zeros(1, dtype=torch.float32, device=model.device)
    n = 0
    fused = _fused_loss_ok(model, criterion)
    for batch in _staged(model, dataloader):
        if fused:
            total += model.eval_loss(batch["images"], batch["decoder_input_tokens"], batch["target_tokens"])
        else:
            logits = model(batch["images"], batch["decoder_input_tokens"])
            tgt = batch["target_tokens"].to(model.device)
            total += criterion(logits.view(-1, logits.size(-1)), tgt.reshape(-1)).reshape(1)
        n += 1
    model.train()
    return (total / max(n, 1)).item()


class LinearWarmup:
    """transformers.get_linear_schedule_with_warmup semantics (train.py:331-341)."""

    def __init__(self, optimizer, num_warmup_steps, num_training_steps):
        self.opt, self.w, self.t, self.step_n = optimizer, num_warmup_steps, num_training_steps, 0
        self.base = _lr_of(optimizer)
        self._apply()

    def _factor(self):
        s = self.step_n
        if s < self.w:
            return s / max(1, self.w)
        return max(0.0, (self.t - s) / max(1, self.t - self.w))

    def _apply(self):
        self.opt.param_groups[0]["lr"] = self.base * self._factor()

    def step(self):
        self.step_n += 1
        self._apply()

    def get_last_lr(self):
        return [_lr_of(self.opt)]

    def state_dict(self):
        return {"step_n": self.step_n, "base": self.base, "w": self.w, "t": self.t}

    def load_state_dict(self, sd):
        self.step_n, self.base, self.w, self.t = sd["step_n"], sd["base"], sd["w"], sd["t"]
        self._apply()


def synthetic_loader(n_batches, B, seq_len, vocab, image, seed=0):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n_batches):
        cap = torch.randint(4, vocab, (B, seq_len), generator=g)
        cap[:, 0] = config.START_TOKEN_ID
        out.append({"images": torch.randn(B, 3, image, image, generator=g),
                    "decoder_input_tokens": cap[:, :-1], "target_tokens": cap[:, 1:]})
    return out


def _torch_adamw_params(model, optimizer):
    """(name, parameter) of a torch.optim.AdamW built over model.parameters() (one group, the flat
    entries in order); raises CheckpointError for any other parameter list."""
    named = list(model.named_parameters())
    g = optimizer.param_groups
    if len(g) != 1 or len(g[0]["params"]) != len(named) or any(a is not b for a, (_, b) in zip(g[0]["params"], named)):
        raise CheckpointError("checkpoints hold the reference's optimizer layout: the torch.optim.AdamW must be built "
                              "over model.parameters() as one parameter group (train.py:319-325)")
    return named


def optimizer_state_reference(model, optimizer) -> dict:
    """The optimizer's state in the REFERENCE checkpoint format: torch.optim.AdamW's state_dict with
    the reference model's parameter indices (frozen encoder first, then projection + decoder in the
    reference's tensors, train.py:422-436). optim.AdamW writes it itself; a torch.optim.AdamW over
    model.parameters() (the flat, fused entries: layers.i.cross_kv, self_in, padded fc_out, ...)
    is converted through the same flat -> reference mapping."""
    if isinstance(optimizer, optim.AdamW):
        return optimizer.state_dict()
    if not isinstance(optimizer, torch.optim.AdamW):
        raise CheckpointError(f"save_checkpoint: {type(optimizer).__name__} has no reference-format state "
                              f"(optim.AdamW or torch.optim.AdamW over model.parameters())")
    named = _torch_adamw_params(model, optimizer)
    store = model.store
    ea = torch.zeros(store.numel, dtype=torch.float32, device=store.device)
    eas = torch.zeros_like(ea)
    steps = set()
    with torch.no_grad():
        for n, p in named:
            st = optimizer.state.get(p)
            if not st:
                continue
            _, off, k = store.index[n]
            ea[off:off + k].copy_(st["exp_avg"].reshape(-1))
            eas[off:off + k].copy_(st["exp_avg_sq"].reshape(-1))
            steps.add(float(st["step"]))
    if len(steps) > 1:
        raise CheckpointError(f"per-parameter step counts differ ({sorted(steps)[:4]}): not representable in the "
                              f"reference layout, whose tensors the flat entries fuse")
    step = int(round(steps.pop())) if steps else 0
    return optim.reference_state(store, store.layout, ea, eas, step, optimizer.param_groups[0])


def load_optimizer_state_reference(model, optimizer, sd: dict):
    """Inverse of optimizer_state_reference: a reference-format AdamW state -> optim.AdamW, or -> a
    torch.optim.AdamW over model.parameters() (its per-parameter state for the flat entries).
    Validated completely before anything is written."""
    if isinstance(optimizer, optim.AdamW):
        return optimizer.load_state_dict(sd)
    if not isinstance(optimizer, torch.optim.AdamW):
        raise CheckpointError(f"load_checkpoint: {type(optimizer).__name__} cannot take a reference-format "
                              f"AdamW state (optim.AdamW or torch.optim.AdamW over model.parameters())")
    named = _torch_adamw_params(model, optimizer)
    store = model.store
    ea, eas, step, g0 = optim.flat_moments(store, store.layout, sd)
    for n, p in named:
        _, off, k = store.index[n]
        if step > 0:
            optimizer.state[p] = {"step": torch.tensor(float(step)),
                                  "exp_avg": ea[off:off + k].view(p.shape).clone(),
                                  "exp_avg_sq": eas[off:off + k].view(p.shape).clone()}
        else:
            optimizer.state.pop(p, None)
    grp = optimizer.param_groups[0]
    for key in ("lr", "betas", "eps", "weight_decay"):
        if key in g0:
            grp[key] = tuple(g0[key]) if key == "betas" else g0[key]


def save_checkpoint(model, optimizer, epoch, val_loss, path_prefix, scheduler=None):
    """train.py:412-442: a .pt dict {epoch, model_state_dict, optimizer_state_dict,
    scheduler_state_dict, best_val_loss} and a .safetensors of model.state_dict() (reference key
    names). The optimizer state is always in the reference's format (optimizer_state_reference),
    so the reference resumes it and vice versa, for optim.AdamW and torch.optim.AdamW alike."""
    from safetensors.torch import save_file
    name = f"{path_prefix}_{config.ENCODER_MODEL_NAME.replace('/', '_')}_epoch_{epoch + 1}_val_loss_{val_loss:.4f}"
    sd = {k: v.detach().cpu().contiguous() for k, v in model.state_dict().items()}
    torch.save({"epoch": epoch, "model_state_dict": sd, "optimizer_state_dict": optimizer_state_reference(model, optimizer),
                "scheduler_state_dict": scheduler.state_dict() if scheduler is not None else None,
                "best_val_loss": val_loss}, name + ".pt")
    save_file(sd, name + ".safetensors")
    return name


class CheckpointError(RuntimeError):
    """A checkpoint that exists but cannot resume this model / optimizer."""


def load_checkpoint(model, optimizer, scheduler, path):
    """train.py:343-375: resume from a .pt checkpoint (the reference's own or save_checkpoint's) ->
    (start_epoch, best_val_loss). A missing path means training from scratch (0, inf), as the
    reference does. A checkpoint that exists but does not fit (unreadable file, missing keys, shape
    or optimizer-state mismatch) raises CheckpointError BEFORE anything is loaded: the reference
    falls back to scratch on any error (train.py:362-368), possibly after loading the weights but
    not the optimizer — a silent half-resume this build refuses.
    Loaded with torch.load(weights_only=True): tensors and plain containers only, nothing in the
    file is executed (the reference uses weights_only=False). A .safetensors path
    (inference.py:66-67) restores the model weights only. The optimizer state is torch.optim.AdamW's
    over the REFERENCE model's parameters (the reference's checkpoints, and save_checkpoint's); it
    resumes optim.AdamW or a torch.optim.AdamW built over model.parameters()."""
    if not path or not os.path.exists(path):
        if path:
            print(f"Warning: checkpoint '{path}' does not exist. Starting training from scratch.")
        return 0, math.inf
    try:
        if path.endswith(".safetensors"):
            from safetensors.torch import load_file
            sd = load_file(path)
            model.check_state_dict(sd)
            model.load_state_dict(sd)
            return 0, math.inf
        ck = torch.load(path, map_location="cpu", weights_only=True)
        for k in ("model_state_dict", "optimizer_state_dict", "epoch"):
            if k not in ck:
                raise KeyError(f"checkpoint has no '{k}' (keys: {sorted(ck)})")
        model.check_state_dict(ck["model_state_dict"])
        # validates everything before it writes (all or nothing), for optim.AdamW and for a
        # torch.optim.AdamW over model.parameters()
        load_optimizer_state_reference(model, optimizer, ck["optimizer_state_dict"])
    except Exception as e:  # noqa: BLE001
        raise CheckpointError(f"cannot resume from '{path}': {e}") from e
    model.load_state_dict(ck["model_state_dict"])
    if scheduler is not None and ck.get("scheduler_state_dict"):
        scheduler.load_state_dict(ck["scheduler_state_dict"])
    start = ck["epoch"] + 1
    print(f"Successfully resumed training. Starting from epoch {start}.")
    return start, ck.get("best_val_loss", math.inf)


def shard_batches(batches, rank: int, world: int):
    """The rank's share of every global batch: rows [rank*B/world, (rank+1)*B/world) (the
    data-parallel loader; each global batch of B pairs is split evenly over the ranks)."""
    for b in batches:
        B = b["decoder_input_tokens"].shape[0]
        if B % world:
            raise ValueError(f"global batch {B} is not divisible by the {world} data-parallel ranks")
        lo, hi = rank * B // world, (rank + 1) * B // world
        yield {k: v[lo:hi] for k, v in b.items()}


def main(argv=None):
    """train.py:282-452 on synthetic batches. Data parallel when launched with WORLD_SIZE > 1
    (torchrun, one process per GPU; RCCL): every rank takes its slice of each global batch of
    --batch-size pairs (shard_batches), the decoder gradients are all-reduced by bucket during the
    backward (dist.DataParallel) with the loss normalised by the GLOBAL non-PAD count, so the step
    equals the single-process step at the global batch; validation runs the whole batch on every
    rank (identical results), and only rank 0 writes checkpoints. Returns the per-epoch
    (train, val) losses."""
    ap = argparse.ArgumentParser(description="Train the captioning model on synthetic batches (MI355X path)")
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--batch-size", type=int, default=config.BATCH_SIZE, help="global batch (all ranks)")
    ap.add_argument("--seq-len", type=int, default=64)
    ap.add_argument("--out", default=None, help="checkpoint prefix (optional)")
    ap.add_argument("--resume", default=getattr(config, "RESUME_CHECKPOINT_PATH", None),
                    help="resume from a .pt checkpoint (train.py:343-375)")
    args = ap.parse_args(argv)
    from dist import DataParallel, init_from_env
    rank, world = init_from_env()
    torch.manual_seed(config.RANDOM_SEED)
    model = ImageToTextModel(config.VOCAB_SIZE, config.DECODER_EMBED_DIM, config.DECODER_HEADS, config.DECODER_LAYERS,
                             config.DECODER_FF_DIM, config.MAX_SEQ_LEN, config.DECODER_DROPOUT, config.PAD_TOKEN_ID)
    opt = optim.AdamW(model.parameters(), lr=config.LEARNING_RATE, betas=(config.ADAM_BETA1, config.ADAM_BETA2),
                      eps=config.ADAM_EPS, weight_decay=config.WEIGHT_DECAY)
    sched = None
    if config.WARMUP_STEPS > 0:
        sched = LinearWarmup(opt, config.WARMUP_STEPS, args.batches * args.epochs)
    train = synthetic_loader(args.batches, args.batch_size, args.seq_len, config.VOCAB_SIZE, model.encoder.image, 1)
    val = synthetic_loader(2, args.batch_size, args.seq_len, config.VOCAB_SIZE, model.encoder.image, 2)
    start, best = load_checkpoint(model, opt, sched, args.resume)
    dp = None
    if world > 1:
        import torch.distributed as tdist
        dp = DataParallel(model)  # broadcasts rank 0's weights (a resumed state is identical on every rank)
        train = list(shard_batches(train, rank, world))
    history = []
    for epoch in range(start, args.epochs):
        t0 = time.time()
        tl = train_one_epoch(model, train, opt, None, "cuda", config.GRAD_CLIP_VALUE, sched, epoch,
                             config.LOG_INTERVAL if rank == 0 else 0, None, dist=dp)
        vl = evaluate(model, val, None, "cuda")
        if world > 1:
            # every rank takes rank 0's validation loss, so the best-checkpoint decision (and the barrier
            # around the save) is the same on all ranks even if their losses differ in the last ulp
            on = "cuda" if tdist.get_backend() == "nccl" else "cpu"
            t = torch.tensor([vl], dtype=torch.float64, device=on)
            tdist.broadcast(t, 0)
            vl = t.item()
        history.append((tl, vl))
        if rank == 0:
            print(f"epoch {epoch + 1}: train {tl:.4f} val {vl:.4f} ({time.time() - t0:.1f}s, {world} rank(s))", flush=True)
        if vl < best and args.out:
            best = vl
            if rank == 0:
                print("saved", save_checkpoint(model, opt, epoch, vl, args.out, sched))
        if world > 1:
            tdist.barrier()
    return history


if __name__ == "__main__":
    main()
