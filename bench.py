"""Throughput benchmark of the MI355X train step (BASELINE.json metric: image-caption pairs/sec).

Workload (BASELINE.json configs[1]): 6-layer d_model=512 decoder + ViT-B/16 encoder (197 patches,
memory_mode "patches": the decoder cross-attends to the projected patch sequence), bf16 compute
with f32 master weights / grads / AdamW state, batch 64 per GPU, 64-token captions (decoder T=63),
vocab 10000, dropout 0.1, synthetic data (randn images, random caption ids), random-init weights.
One step = encoder forward + projection + decoder forward + CE + backward + clip_grad_norm_(5.0)
+ AdamW, i.e. train.py:75-100 for one batch.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU, RCCL data parallel)

Rank 0 prints ONE JSON line. `value` = pairs processed by all ranks / max-over-ranks wall time.
`roofline` = the dominant kernel's achieved algorithmic TFLOP/s (HIP events around each of its
launches during an instrumented replay of the same steps) against the bf16 dense MFMA peak.
`cpu_baseline` = the CPU oracle (oracle/ref_cpu.py, an fp32 PyTorch restatement of the reference
path) timed on this host on a bounded sample (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "multimodal-image-transformer_amd")
# 8 hardware queues before HIP initialises (native.py explains: with HIP's default 4 the RCCL stream of the
# N-GPU path shares a queue with a compute stream, 10.0 k vs 13.6 k pairs/s for one RCCL rank)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)

import torch  # noqa: E402

MFMA_BF16_PEAK_TFLOPS = 2516.6  # 256 CU x 2.4 GHz x 4096 FLOP/clk (MI355X_MICROARCH.md, dense)
PMC_SUMMARIES = ("r06f_pmc.json", "r06_pmc.json", "r05_pmc.json", "r04_pmc.json")  # the newest committed PMC summary is used
METRIC = "image-caption pairs/sec (train step), 6L/d512 decoder + ViT-B/16, 1/2/4/8 GPU"


class HipEvent:
    """hipEvent created with hipEventDisableSystemFence: a timing-only event whose record does not
    write back / invalidate caches (a default event's system-scope fence adds ~8 us to every
    bracketed launch). Recorded on the stream the kernels are launched on (native.stream_ptr())."""
    _hip = None
    DISABLE_SYSTEM_FENCE = 0x20000000

    def __init__(self):
        import ctypes
        if HipEvent._hip is None:
            import native
            h = native.hip_runtime()  # the runtime this process already maps
            h.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
            h.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            h.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
            h.hipEventDestroy.argtypes = [ctypes.c_void_p]
            HipEvent._hip = h
        self.ev = ctypes.c_void_p()
        if HipEvent._hip.hipEventCreateWithFlags(ctypes.byref(self.ev), self.DISABLE_SYSTEM_FENCE) != 0:
            raise RuntimeError("hipEventCreateWithFlags failed")

    def record(self, stream):
        if HipEvent._hip.hipEventRecord(self.ev, stream) != 0:
            raise RuntimeError("hipEventRecord failed")

    def seconds_to(self, other):
        import ctypes
        ms = ctypes.c_float()
        if HipEvent._hip.hipEventElapsedTime(ctypes.byref(ms), self.ev, other.ev) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return ms.value * 1e-3

    def __del__(self):
        if HipEvent._hip is not None and self.ev:
            HipEvent._hip.hipEventDestroy(self.ev)


class GemmProbe:
    """Times the GEMM kernels of the eager step two ways, with fence-free HIP events on the launch
    stream: (1) an event pair around every launch in place; (2) the launches of one step replayed
    in their original order, back-to-back, `passes` times, between ONE event pair per kernel
    instance (tile kernel, a_layout, b_layout; native.gemm_plan) -- this is the per-launch kernel duration (event markers between
    kernels add a dispatch ramp that the kernel itself does not spend; rocprofv3's per-dispatch
    average, profiles/r02_bench_kernel_stats.csv, is the cross-check)."""

    def __init__(self):
        self.rec = []
        self.cur = None
        self.step = []

    def new_step(self):
        self.step = []

    def before(self, dt, al, bl, M, N, K, nbytes):
        import native
        e0 = HipEvent()
        e0.record(native.stream_ptr())
        self.cur = (e0, (al, bl), 2.0 * M * N * K, nbytes)

    @staticmethod
    def kernel_key(g, al, bl):
        """(kernel template, a_layout, b_layout) of the launch mit_gemm makes for args g."""
        import native
        tile, ks = native.gemm_plan(g)
        return ({256: "gemm256_kernel", 65: "gemm_rs_kernel"}.get(tile, "gemm_bf16_kernel"), al, bl)

    def after(self, g):
        import ctypes
        import native
        e1 = HipEvent()
        s = native.stream_ptr()
        e1.record(s)
        e0, (al, bl), fl, nb = self.cur
        key = self.kernel_key(g, al, bl)
        self.rec.append((e0, e1, key, fl, nb))
        gc = type(g)()
        ctypes.memmove(ctypes.byref(gc), ctypes.byref(g), ctypes.sizeof(g))
        self.step.append((key, lambda: native.gemm_relaunch(gc, s), s, fl, nb))

    def grouped(self, flops, nbytes, launch):
        """A grouped dW launch (native.gemm_grouped): launch() issues it on the current stream."""
        import native
        s = native.stream_ptr()
        e0, e1 = HipEvent(), HipEvent()
        e0.record(s)
        launch()
        e1.record(s)
        key = ("gemm_bf16_grouped", 1, 1)
        self.rec.append((e0, e1, key, flops, nbytes))
        self.step.append((key, launch, s, flops, nbytes))

    def summary(self):
        """{(kernel, a_layout, b_layout): [seconds, flops, launches, algorithmic bytes]} from the in-place pairs."""
        torch.cuda.synchronize()
        agg = {}
        for e0, e1, key, fl, nb in self.rec:
            t = e0.seconds_to(e1)
            a = agg.setdefault(key, [0.0, 0.0, 0, 0])
            a[0] += t
            a[1] += fl
            a[2] += 1
            a[3] += nb
        return agg

    def replay(self, passes=3):
        """{(kernel, a_layout, b_layout): [seconds, flops, launches, algorithmic bytes]} over the replays of the
        last recorded step (modifies activations/grads in place: run after everything measured)."""
        import native
        torch.cuda.synchronize()
        out = {}
        for key in sorted({k for k, *_ in self.step}):
            launches = [r for r in self.step if r[0] == key]
            s = launches[0][2]
            for _, relaunch, _, _, _ in launches:  # warm the code object / caches once
                with native.on_stream(s):
                    relaunch()
            e0, e1 = HipEvent(), HipEvent()
            e0.record(s)
            for _ in range(passes):
                for _, relaunch, _, _, _ in launches:
                    with native.on_stream(s):
                        relaunch()
            e1.record(s)
            torch.cuda.synchronize()
            n = passes * len(launches)
            out[key] = [e0.seconds_to(e1), passes * sum(r[3] for r in launches), n,
                        passes * sum(r[4] for r in launches)]
        return out


def _pmc_summary():
    for name in PMC_SUMMARIES:
        path = os.path.join(ROOT, "profiles", name)
        try:
            with open(path) as f:
                return json.load(f), f"profiles/{name}"
        except (OSError, ValueError):
            continue
    return None, None


def pmc_traffic(kernel_prefix):
    """HBM bytes per launch of a kernel (averaged over the launches of all its template instances)
    from the committed rocprofv3 PMC summary (FETCH_SIZE and WRITE_SIZE passes of
    tools/profile_round.sh over this same command, condensed by tools/rocpd_summary.py); None when no
    summary is present."""
    d, src = _pmc_summary()
    if d is None:
        return None, None
    tot, n = 0.0, 0
    for name, e in d.get("kernels", {}).items():
        if name.startswith(kernel_prefix) and "hbm_bytes_per_launch" in e:
            tot += e["hbm_bytes_per_launch"] * e["launches"]
            n += e["launches"]
    return (round(tot / n), src) if n else (None, None)


def pmc_mfma(kernel_prefix):
    """MFMA busy / peak of a kernel (SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x dispatch wall x 2.4 GHz): the
    share of the dense bf16 peak's MFMA issue kept busy), launch-weighted over its template instances, from
    the MFMA-busy pass of the committed PMC summary (tools/rocpd_summary.py)."""
    d, src = _pmc_summary()
    ks = (d or {}).get("mfma_pass", {}).get("kernels", {})
    busy, n = 0.0, 0
    for name, e in ks.items():
        if name.startswith(kernel_prefix) and "mfma_busy_of_peak" in e:
            busy += e["mfma_busy_of_peak"] * e["launches"]
            n += e["launches"]
    return (round(busy / n, 4), src) if n else (None, None)


def clock_calibration(kernel_prefix):
    """Effective engine clock (GHz) of a kernel under sustained load: GRBM_GUI_ACTIVE / 8 / wall over 5-6 ms
    dispatches of the same kernel (tools/clock_pass.sh -> profiles/*_clock_pass.json). The short in-step
    dispatches' GRBM quotient reads high (MI355X_MICROARCH.md: below ~0.3 ms), so it is not used here."""
    for name in sorted((f for f in os.listdir(os.path.join(ROOT, "profiles")) if f.endswith("_clock_pass.json")),
                       reverse=True):
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        cl = [e["eff_clock_ghz"] for k, e in d.items() if k.startswith(kernel_prefix.split("<")[0])
              and isinstance(e, dict) and "eff_clock_ghz" in e]
        if cl:
            return round(min(2.4, sum(cl) / len(cl)), 3), f"profiles/{name}"
    return None, None


# Train workloads: BASELINE.json configs[1] (the metric's config, the default) and the single-GPU
# shares of configs[2] / configs[3] (CLIP encoders; cfg3 = 64 of its global 512 pairs per GPU).
# (encoder name, decoder d, heads, layers, ff, workload label)
WORKLOADS = {
    "train": ("google/vit-base-patch16-224-in21k", 512, 8, 6, 2048,
              "configs[1]: 6L d512 decoder + ViT-B/16 (197 patches), batch 64/GPU, seq_len 64"),
    "clip336": ("openai/clip-vit-large-patch14-336", 512, 8, 6, 2048,
                "configs[2]: 6L d512 decoder + CLIP ViT-L/14@336 (577 patches), batch 64/GPU, seq_len 64"),
    "cfg3": ("openai/clip-vit-large-patch14", 768, 12, 12, 3072,
             "configs[3]: 12L d768 decoder + CLIP ViT-L/14 (257 patches), batch 64/GPU (global 512 at 8 GPUs), "
             "seq_len 64"),
}


def build(args, rank):
    import config
    from model import ImageToTextModel
    import optim
    config.MEMORY_MODE = args.memory_mode
    enc_name, d, heads, layers, ff, _ = WORKLOADS.get(args.workload, WORKLOADS["train"])
    config.ENCODER_MODEL_NAME = enc_name
    m = ImageToTextModel(args.vocab, d, heads, layers, ff, 100, 0.1, 0, memory_mode=args.memory_mode, dtype=args.dtype,
                         seed=42)
    opt = optim.AdamW(m.store, lr=1e-4, betas=(0.9, 0.98), eps=1e-9, weight_decay=1e-5)
    return m, opt


def synthetic_batch(B, seq_len, vocab, device, seed, image=224):
    g = torch.Generator().manual_seed(seed)
    images = torch.randn(B, 3, image, image, generator=g).to(device)
    cap = torch.randint(4, vocab, (B, seq_len), generator=g)
    cap[:, 0] = 2
    return images, cap[:, :-1].contiguous().to(device), cap[:, 1:].contiguous().to(device)


def _cpu_threads() -> int:
    """The threads this job may use on the host: OMP_NUM_THREADS (the GPU box sets it to the job's CPU
    share, 16 per GPU; os.cpu_count() there reports the whole machine), else every CPU."""
    try:
        return max(1, int(os.environ["OMP_NUM_THREADS"]))
    except (KeyError, ValueError):
        return os.cpu_count() or 1


def cpu_baseline(model, args):
    """The CPU oracle's train step (oracle/ref_cpu.py: fp32 torch CPU restatement of the reference
    path, pinned to the reference's outputs; dropout off) on bounded samples (SURVEY.md §8d / BASELINE.md
    §3): configs[1]'s architecture in patches mode (the metric's workload -> `value`) and cls mode,
    and configs[0] (2L d128 H8 decoder + ViT-B/16, batch 4, seq_len 32, cls = the reference's own
    path). Same ViT-B/16 weights as the GPU model; median of `cpu_steps` steps after a warm-up."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import ref_cpu as R
    import optim
    threads = _cpu_threads()
    torch.set_num_threads(threads)
    sd = {k: v.float().cpu() for k, v in model.state_dict().items()}
    enc = {"kind": "vit", "heads": 12, "layers": 12, "patch": 16, "eps": 1e-12}

    def timed(params, names, dec, mode, B, seq_len):
        images, di, tg = synthetic_batch(B, seq_len, args.vocab, "cpu", 7)
        opt = R.AdamWState({k: params[k] for k in names})
        R.train_step(params, names, opt, images, di, tg, enc, dec, mode, 5.0)  # warm-up
        times = []
        for _ in range(args.cpu_steps):
            t0 = time.perf_counter()
            R.train_step(params, names, opt, images, di, tg, enc, dec, mode, 5.0)
            times.append(time.perf_counter() - t0)
        return B / sorted(times)[len(times) // 2]

    names1 = [k for k in sd if not k.startswith("encoder.") and not k.endswith("positional_encoding.pe")]
    dec1 = {"heads": 8, "layers": 6, "max_seq_len": 100}
    B = args.cpu_batch
    v_patches = timed(dict(sd), names1, dec1, "patches", B, args.seq_len)
    v_cls = timed(dict(sd), names1, dec1, "cls", B, args.seq_len)
    # configs[0]: the same encoder + a seeded 2L d128 / 8-head decoder in the reference's tensor names
    lay0 = dict(V=args.vocab, d=128, L=2, F=512, proj_in=768)
    g = torch.Generator().manual_seed(0)
    p0 = {k: v for k, v in sd.items() if k.startswith("encoder.")}
    for n, shp in optim.reference_trainable(lay0):
        t = torch.randn(*shp, generator=g)
        p0[n] = t / (shp[1] ** 0.5) if len(shp) == 2 else 0.02 * t
    names0 = [n for n, _ in optim.reference_trainable(lay0)]
    v_cfg0 = timed(p0, names0, {"heads": 8, "layers": 2, "max_seq_len": 100}, "cls", 4, 32)
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(v_patches, 3), "unit": "pairs/s", "cores": threads, "kind": "port",
            "sample": f"oracle/ref_cpu.py fp32 train step (encoder fwd + decoder fwd/bwd + clip + AdamW), configs[1] "
                      f"architecture, patches mode, batch {B}, seq_len {args.seq_len}; median of {args.cpu_steps} steps "
                      f"after 1 warm-up, dropout off; {threads} threads = this job's CPU share (OMP_NUM_THREADS); "
                      f"cpu: {cpu_model}",
            "also": {"configs[1] cls mode (the reference's CLS-only memory)": round(v_cls, 3),
                     "configs[0] (2L d128 H8 + ViT-B/16, batch 4, seq_len 32, cls)": round(v_cfg0, 3)}}


def decode_throughput(args, launch=None):
    """configs[4]: greedy captions for a batch of images (ImageToTextModel.generate_batch). END is set
    to an id the vocabulary never produces, so every caption runs the full max_len - 1 tokens (fixed
    work per call). One call = encoder forward + cross K/V + (max_len - 1) token steps, replayed as a
    native launch plan (mit_plan_run) by default or as one hipGraph per step (launch="graph")."""
    import model as model_mod  # noqa: F401  (generate_batch reads MIT_DECODE_LAUNCH per call)
    dev = torch.device("cuda", torch.cuda.current_device())
    a = argparse.Namespace(**vars(args))
    a.memory_mode, a.workload = "patches", "train"
    model, _ = build(a, 0)
    model.eval()
    B = args.decode_batch
    images = synthetic_batch(B, 2, args.vocab, dev, 5)[0]
    never = args.vocab + 7
    old = os.environ.get("MIT_DECODE_LAUNCH")
    if launch:
        os.environ["MIT_DECODE_LAUNCH"] = launch
    try:
        # the next call's encoder runs beside this call's token steps (generate_batch next_images)
        nxt = None if getattr(args, "no_prefetch", False) else images
        for _ in range(max(1, args.warmup // 2)):
            model.generate_batch(images, 2, never, max_len=args.max_len, next_images=nxt)
        torch.cuda.synchronize()
        K = max(1, args.steps // 4)
        t0 = time.perf_counter()
        for _ in range(K):
            ids = model.generate_batch(images, 2, never, max_len=args.max_len, next_images=nxt)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    finally:
        if launch:
            if old is None:
                os.environ.pop("MIT_DECODE_LAUNCH", None)
            else:
                os.environ["MIT_DECODE_LAUNCH"] = old
    toks = B * (args.max_len - 1) * K
    return {"value": round(toks / el, 1), "unit": "tokens/s", "calls": K, "ms_per_call": round(1e3 * el / K, 3),
            "images_per_s": round(B * K / el, 2), "us_per_token_step": round(1e6 * el / K / (args.max_len - 1), 2),
            "ids_per_caption": len(ids[0]), "images": B, "max_len": args.max_len,
            "launch": launch or os.environ.get("MIT_DECODE_LAUNCH", "plan")}


DECODE_LAUNCH_NOTE = ("per-token step replayed as a native launch plan (mit_plan_run: the step's launches recorded "
                      "once, re-issued from C++); a hipGraph of the same step is the slower alternative on ROCm 7 "
                      "(graph replay issues its nodes one by one, ~8.7 us each on the host) -- both are timed in "
                      "the bench's `also` block")


def bench_decode(args):
    torch.cuda.set_device(0)
    d = decode_throughput(args)
    out = {"metric": "greedy caption tokens/sec (batched KV-cache decode, 6L/d512 decoder + ViT-B/16)",
           "value": d["value"], "unit": "tokens/s", "n_gpus": 1, "steps": d["calls"], "warmup": max(1, args.warmup // 2),
           "ms_per_step": d["ms_per_call"], "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": args.dtype, "data": "synthetic (randn 224x224 images; random-init weights)",
           "config": {"workload": "configs[4]: inference.py greedy decode, cached cross-attn K/V, the next call's "
                                      "encoder issued beside the token steps (--no-prefetch: inline), " + DECODE_LAUNCH_NOTE,
                      "images": d["images"], "max_len": args.max_len, "memory_mode": "patches"},
           "images_per_s": d["images_per_s"], "us_per_token_step": d["us_per_token_step"],
           "ids_per_caption": d["ids_per_caption"]}
    print(json.dumps(out), flush=True)


def also_block(args):
    """The other single-GPU BASELINE configs in the same run (N = 1, rank 0), after the headline line's
    measurements: configs[2] (6L d512 decoder + CLIP ViT-L/14@336, 577 patches) and one GPU's share of
    configs[3] (12L d768 decoder + CLIP ViT-L/14, 64 of the global 512 pairs) train-step pairs/s, and
    configs[4] (batched greedy decode, B = 256, max_len 100) tokens/s with the default native launch plan
    and with one hipGraph per token step. configs[2] / configs[3] run as `bench.py --workload clip336 /
    cfg3` in child processes: configs[2] built and replayed inside this process (after the headline model) it read 1.5-2 % lower than
    the same command alone (1853-1872 vs 1892-1899 pairs/s on one box), with or without the CPU baseline
    before it and with the headline model's state released (profiles/r05_decoder_experiments.txt)."""
    import subprocess
    out = {}
    t_all = time.perf_counter()
    steps = max(2, args.also_steps)
    for key, workload, metric in (
            ("configs[2]", "clip336", "image-caption pairs/sec (train step), 6L/d512 decoder + CLIP ViT-L/14@336"),
            ("configs[3]", "cfg3", "image-caption pairs/sec (train step), one GPU's 64 of the global 512 pairs, "
                                   "12L/d768 decoder + CLIP ViT-L/14")):
        cmd = [sys.executable, os.path.abspath(__file__), "--workload", workload, "--no-cpu-baseline", "--no-also",
               "--no-roofline", "--steps", str(steps), "--warmup", "3", "--batch", str(args.batch),
               "--seq-len", str(args.seq_len), "--vocab", str(args.vocab), "--dtype", args.dtype]
        # a failed, hung or unparsable child is recorded under its key; the headline line, already measured,
        # is printed either way
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
            lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
            if r.returncode != 0 or not lines:
                raise RuntimeError(f"child exited {r.returncode}: {r.stderr[-1500:]}")
            c = json.loads(lines[-1])
        except (subprocess.TimeoutExpired, RuntimeError, ValueError, OSError) as e:
            out[key] = {"metric": metric, "error": f"{type(e).__name__}: {str(e)[-1500:]}",
                        "process": "own: " + " ".join(["bench.py"] + cmd[2:])}
            continue
        out[key] = {"metric": metric, "value": c["value"], "unit": "pairs/s", "steps": c["steps"],
                    "ms_per_step": c["ms_per_step"], "batch": args.batch, "seq_len": args.seq_len, "dtype": c["dtype"],
                    "step_mfma_frac": c["step_mfma_frac"], "launch_path": c["launch_path"],
                    "process": "own: " + " ".join(["bench.py"] + cmd[2:])}
    dmetric = "greedy caption tokens/sec (batched KV-cache decode, 6L/d512 decoder + ViT-B/16)"
    try:
        d = decode_throughput(args)
        g = decode_throughput(args, "graph")
        out["configs[4]"] = dict(d, metric=dmetric, note=DECODE_LAUNCH_NOTE, graph_tokens_per_s=g["value"],
                                 graph_us_per_token_step=g["us_per_token_step"])
    except Exception as e:  # noqa: BLE001 -- recorded, the headline line still prints
        out["configs[4]"] = {"metric": dmetric, "error": f"{type(e).__name__}: {str(e)[-1500:]}"}
    out["seconds"] = round(time.perf_counter() - t_all, 1)
    return out


def spawn_ranks(args) -> int:
    """--gpus N > 1 with no launcher (WORLD_SIZE unset): start N rank processes of this script, one per
    GPU, with the torchrun environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
    MASTER_PORT). This parent makes no GPU call; rank 0 prints the JSON line. If a rank fails the
    others are terminated and the failing status is returned."""
    import socket
    import subprocess
    port = os.environ.get("MASTER_PORT")
    if not port:
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = str(sk.getsockname()[1])
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)  # 20 steps read ~0.5 % low: the first replay's enqueue latency is timed too
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="pairs per GPU")
    ap.add_argument("--seq-len", type=int, default=64)
    ap.add_argument("--vocab", type=int, default=10000)
    ap.add_argument("--memory-mode", default="patches", choices=["patches", "cls"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--cpu-batch", type=int, default=4)
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--graph", action="store_true",
                    help="replay the step as ONE hipGraph (N=1). Default: eager launches, which let the backward's "
                         "weight-gradient stream run beside the main stream (measured faster than the graph, whose "
                         "parallel branches ROCm 7 does not overlap)")
    ap.add_argument("--no-graph", action="store_true", help="(default; kept for older scripts)")
    ap.add_argument("--no-replay", action="store_true",
                    help="issue every step from Python (eager launches). Default: the step's launches are recorded "
                         "once (native.record, mit_plan_*) and replayed from C++ per step, same streams and order")
    ap.add_argument("--no-prefetch", action="store_true",
                    help="run the frozen encoder inside each step (train) / call (decode) instead of one ahead on a "
                         "second stream")
    ap.add_argument("--workload", default="train", choices=["train", "clip336", "cfg3", "decode"],
                    help="train: the BASELINE metric (default, configs[1]). clip336 / cfg3: the one-GPU share of "
                         "configs[2] / configs[3] (same step, CLIP-L encoders). decode: configs[4], batched greedy "
                         "captioning (KV cache, per-token step replayed as a native launch plan)")
    ap.add_argument("--decode-batch", type=int, default=256)
    ap.add_argument("--max-len", type=int, default=100, help="decode: ids per caption (config.MAX_SEQ_LEN)")
    ap.add_argument("--also-steps", type=int, default=10, help="timed configs[2] steps in the `also` block")
    ap.add_argument("--no-also", action="store_true",
                    help="skip the `also` block (configs[2] train step and configs[4] decode in the same run, N=1)")
    ap.add_argument("--dp", action="store_true",
                    help="N=1 only: build DataParallel over a world-size-1 torch.distributed group (RCCL, backend "
                         "\"nccl\"; MIT_DIST_BACKEND=gloo to rehearse) so the step runs the N-GPU launch path -- count "
                         "all-reduce, bucket all-reduces under the weight-gradient stream, join before clip + AdamW, "
                         "all as host steps of the replayed program -- and its collectives' cost is measured "
                         "(parallelism \"dp1-nccl\")")
    args = ap.parse_args()
    if args.workload == "decode":
        return bench_decode(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))

    from dist import DataParallel, init_from_env
    import torch.distributed as tdist
    rank, world = init_from_env()
    dp1 = None
    if args.dp and world == 1:  # a one-rank process group: the N-GPU path's collectives on this GPU
        import socket
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
        dp1 = os.environ.get("MIT_DIST_BACKEND") or "nccl"
        torch.cuda.set_device(0)
        if dp1 == "nccl":
            tdist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        else:
            tdist.init_process_group(dp1, rank=0, world_size=1)
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)", file=sys.stderr, flush=True)
        sys.exit(2)
    if world == 1:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    model, opt = build(args, rank)
    dp = DataParallel(model, overlap=not args.no_overlap) if (world > 1 or dp1) else None
    model.train()
    images, di, tg = synthetic_batch(args.batch, args.seq_len, args.vocab, dev, 1000 + rank, model.encoder.image)

    prefetch = not args.no_prefetch

    def eager_step():
        # the frozen encoder's forward for the next batch runs on a second stream beside this
        # step's decoder work (model.prefetch_encoder); one encoder forward per step either way
        return model.train_step(images, di, tg, dist=dp, next_images=images if prefetch else None)

    use_graph = world == 1 and args.graph and not args.no_graph
    replay = not args.no_replay and not use_graph
    if use_graph:
        gstep = model.make_graphed_step(opt, images, di, tg, 5.0)

        def step():
            return gstep()
    else:
        def step():
            loss = eager_step()
            opt.step(5.0)
            return loss

    def barrier():
        if world > 1 or dp1:
            tdist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    if replay:
        # two consecutive real steps recorded (the encoder prefetch alternates between two arenas),
        # then replayed alternately: one C++ call per native segment instead of a Python wrapper per launch
        import native
        progs = [native.record(step) for _ in range(2)]
        n_launch = progs[0].launches()
        out_loss = model.decoder.acts(args.batch, args.seq_len - 1, 1 if args.memory_mode == "cls" else model.encoder.N,
                                      True).loss
        it = [0]

        def step():
            opt._sync_lr()
            progs[it[0] % 2].run()
            it[0] += 1
            return out_loss
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t_enq = time.perf_counter() - t0  # host time to enqueue the K steps (launches are asynchronous)
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = t.item()
    loss = step().item()

    pairs = args.batch * world * args.steps
    value = pairs / elapsed
    flops_pair = model.flops_per_pair(args.seq_len - 1)
    out = {
        "metric": METRIC if args.workload == "train" else METRIC.replace(
            "6L/d512 decoder + ViT-B/16, 1/2/4/8 GPU", WORKLOADS[args.workload][5].split(": ")[1].split(",")[0]),
        "value": round(value, 2), "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "bf16" if args.dtype == "bf16" else "f32",
        "data": f"synthetic (randn {model.encoder.image}x{model.encoder.image} images, uniform caption ids; "
                "random-init weights)",
        "config": {"workload": WORKLOADS[args.workload][5],
                   "global_batch": args.batch * world, "seq_len": args.seq_len, "vocab": args.vocab,
                   "memory_mode": args.memory_mode, "parallelism": f"dp{world}" + (f"-{dp1}" if dp1 else ""),
                   "gflop_per_pair": round(flops_pair / 1e9, 3)},
        "step_mfma_frac": round(value / world * flops_pair / (MFMA_BF16_PEAK_TFLOPS * 1e12), 4),
        # ~ms_per_step when the host's launch path, not the GPU, paces the step
        "host_enqueue_ms_per_step": round(1e3 * t_enq / args.steps, 3),
        "launch_path": ("native replay (mit_plan_run), %d launches/step" % n_launch) if replay else
                       ("hipGraph" if use_graph else "eager (Python per launch)"),
        "final_loss": round(loss, 4),
    }
    if not args.no_roofline:
        import native
        probe = GemmProbe()
        native.set_gemm_probe(probe)
        for _ in range(min(args.steps, 5)):  # eager replay of the same step (events need eager launches)
            # park the GPU on a ~50 ms spin so the host enqueues the whole step ahead of it: the event
            # pairs then time back-to-back kernels, not the host's launch latency
            torch.cuda.synchronize()
            torch.cuda._sleep(120_000_000)
            probe.new_step()
            eager_step()
            opt.step(5.0)
        native.set_gemm_probe(None)
        inplace = probe.summary()
        agg = probe.replay()
        role = {(0, 0): "NT: forward", (0, 1): "NN: dX", (1, 1): "TN: dW", (1, 0): "TT"}

        def names(k):
            if k[0] == "gemm_bf16_grouped":
                return "gemm_bf16_grouped (TN: a decoder layer's six dW, one launch + split-K combine)"
            return f"{k[0]}<{k[1]},{k[2]}> ({role[(k[1], k[2])]})"
        key = max(agg, key=lambda k: agg[k][0])
        # achieved: the launches as they ran INSIDE the steps (an event pair around each, the other streams'
        # kernels sharing the chip) -- what rocprofv3's per-dispatch average of the same run sees; the
        # isolated back-to-back replay of the same launches is reported beside it
        t, fl, n, nb = inplace[key]
        ach = fl / t / 1e12
        tr, flr, nr, _ = agg[key]
        # the committed PMC summary was collected on configs[1]; other workloads report no traffic
        traffic, src = (pmc_traffic(f"{key[0]}<{key[1]}, {key[2]},") if args.workload == "train" else (None, None))
        busy, bsrc = (pmc_mfma(f"{key[0]}<{key[1]}, {key[2]},") if args.workload == "train" else (None, None))
        clk, csrc = clock_calibration(key[0])
        out["roofline"] = {"bound": "mfma", "kernel": names(key), "achieved": round(ach, 1),
                           "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(ach / MFMA_BF16_PEAK_TFLOPS, 4),
                           "traffic": traffic, "traffic_unit": "HBM bytes per launch (PMC)", "traffic_source": src,
                           "mfma_busy_of_peak": busy, "mfma_busy_source": bsrc,
                           "eff_clock_ghz": clk, "eff_clock_source": csrc,
                           "eff_clock_note": "long-dispatch GRBM_GUI_ACTIVE/8/wall of the same kernel (sustained MFMA load)",
                           "algorithmic_bytes_per_launch": round(nb / n), "flop_per_launch": round(fl / n),
                           "launches": n, "avg_launch_us": round(1e6 * t / n, 2),
                           "avg_launch_us_isolated_replay": round(1e6 * tr / nr, 2),
                           "achieved_isolated_replay": round(flr / tr / 1e12, 1),
                           "timing": "every launch of this kernel in the last min(steps, 5) eager steps, each between "
                                     "fence-free HIP events on its launch stream (the step's other streams running); "
                                     "isolated replay: one step's launches re-issued back-to-back, 3 passes"}
        out["gemm_breakdown"] = {names(k): {"tflops": round(v[1] / v[0] / 1e12, 1),
                                                        "ms_per_step": round(1e3 * v[0] * inplace[k][2] / v[2] / min(args.steps, 5), 3)}
                                 for k, v in agg.items()}
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload == "train":
        out["cpu_baseline"] = cpu_baseline(model, args)
    if rank == 0 and world == 1 and not args.no_also and args.workload == "train":
        out["also"] = also_block(args)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1 or dp1:
        tdist.barrier()
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
