"""ctypes binding of libmit_hip.so (the C ABI in include/mit_hip.h).

This is the only module that touches the native library. Every wrapper takes torch tensors that
live on the current HIP device, passes raw pointers / extents / the current stream, and raises
``NativeError`` with the library's message on a rejected argument or a failed launch.

There is deliberately NO fallback: if the library is missing, or no GPU is present, the first
call raises. (The CPU oracle lives in /oracle and is test infrastructure only.)
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

# Hardware queues per process (read once, when HIP initialises: set before the first HIP call). A train step
# runs on up to five streams -- main, weight-gradient side stream, encoder prefetch, the CLIP towers' second
# encoder stream, and under data parallelism RCCL's stream (ProcessGroupNCCL) -- and HIP's default of 4 queues
# makes two of them share one: a stream-wait on the shared queue then stalls the other stream's kernels too.
# Measured on one MI355X (bench.py --dp, one RCCL rank, native replay): 4 queues 10.0 k pairs/s, 8 queues
# 13.6 k, 16 queues 13.6 k; the plain one-process step 13.7 k with 4 or 8 (profiles/r06_dp1_nccl_run.json).
# The driver's multi-GPU bench runs exactly the RCCL path. An explicit setting in the environment wins.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MIT_HIP_LIB", os.path.join(_HERE, "lib", "libmit_hip.so"))
ABI_VERSION = 6  # mit_abi_version() of the library this binding matches (include/mit_hip.h)
ARGMAX_SLOTS = 16  # MIT_ARGMAX_SLOTS: slots per row of the decode head's argmax keys

F32, BF16 = 0, 1
K_CONTIG, MN_CONTIG = 0, 1
ACT_NONE, ACT_RELU, ACT_GELU, ACT_QUICK_GELU = 0, 1, 2, 3


class NativeError(RuntimeError):
    pass


_lib: Optional[ctypes.CDLL] = None

vp = ctypes.c_void_p
L = ctypes.c_long
I = ctypes.c_int
Fl = ctypes.c_float
U32 = ctypes.c_uint32


class GemmArgs(ctypes.Structure):
    _fields_ = [("dtype", I), ("a_layout", I), ("b_layout", I), ("M", L), ("N", L), ("K", L),
                ("A", vp), ("lda", L), ("B", vp), ("ldb", L), ("C", vp), ("ldc", L), ("alpha", Fl),
                ("bias", vp), ("act", I), ("residual", vp), ("ldr", L), ("aux", vp), ("ld_aux", L),
                ("aux_scale", Fl), ("drop_p", Fl), ("seed", vp), ("site", U32), ("out_f32", I),
                ("accumulate", I), ("rowsum", vp), ("workspace", vp), ("workspace_bytes", L),
                ("ln_stats", vp), ("ln_colsum", vp), ("ln_parts", I), ("ln_eps", Fl), ("stats_out", vp), ("tiles", I),
                ("argmax_keys", vp)]


class DecodeGemmArgs(ctypes.Structure):
    _fields_ = [("M", L), ("N", L), ("K", L), ("A", vp), ("lda", L), ("a_stats", vp), ("a_gamma", vp),
                ("a_beta", vp), ("B", vp), ("ldb", L), ("bias", vp), ("act", I), ("c_f32", I), ("C", vp),
                ("ldc", L), ("r_mode", I), ("r", vp), ("ldr", L), ("r_stats", vp), ("r_gamma", vp),
                ("r_beta", vp), ("eps", Fl), ("z_out", vp), ("ldz", L), ("stats_out", vp), ("cache", vp),
                ("c_row", L), ("c_batch", L), ("kv_col0", L), ("pos", vp), ("argmax_keys", vp)]


class LnGradsJob(ctypes.Structure):
    _fields_ = [("rows", L), ("cols", L), ("ws", vp), ("dgamma", vp), ("dbeta", vp)]


class AttnArgs(ctypes.Structure):
    _fields_ = [("q", vp), ("q_row", L), ("q_batch", L), ("k", vp), ("k_row", L), ("k_batch", L),
                ("v", vp), ("v_row", L), ("v_batch", L), ("o", vp), ("o_row", L), ("o_batch", L),
                ("lse", vp), ("key_tokens", vp), ("tok_batch", L), ("pad_idx", I), ("causal", I),
                ("scale", Fl), ("drop_p", Fl), ("seed", vp), ("site", U32)]


class AttnGrads(ctypes.Structure):
    _fields_ = [("dout", vp), ("do_row", L), ("do_batch", L), ("dq", vp), ("dq_row", L), ("dq_batch", L),
                ("dk", vp), ("dk_row", L), ("dk_batch", L), ("dv", vp), ("dv_row", L), ("dv_batch", L),
                ("delta_ws", vp)]


# name -> (restype, argtypes); mirrors include/mit_hip.h one to one
SIGNATURES = {
    "mit_last_error": (ctypes.c_char_p, []),
    "mit_abi_version": (I, []),
    "mit_gemm": (I, [ctypes.POINTER(GemmArgs), vp]),
    "mit_gemm_workspace_bytes": (L, [L, L, L]),
    "mit_gemm_set_variant": (I, [I]),
    "mit_gemm_plan": (I, [ctypes.POINTER(GemmArgs), ctypes.POINTER(I)]),
    "mit_gemm_grouped_ws_bytes": (L, [ctypes.POINTER(GemmArgs), I]),
    "mit_gemm_grouped": (I, [ctypes.POINTER(GemmArgs), I, ctypes.POINTER(LnGradsJob), I, vp, L, vp]),
    "mit_layernorm_fwd": (I, [I, L, L, vp, L, vp, L, Fl, vp, U32, vp, vp, Fl, vp, vp, L, vp, vp, vp]),
    "mit_layernorm_fwd_x32": (I, [L, L, vp, L, vp, L, vp, vp, vp, Fl, vp, I, L, vp]),
    "mit_residual_out": (I, [L, L, vp, L, vp, L, vp, L, vp]),
    "mit_row_stats64": (I, [L, L, vp, L, vp, vp]),
    "mit_layernorm_bwd_ws_floats": (L, [L, L]),
    "mit_layernorm_bwd": (I, [I, L, L, vp, vp, vp, vp, vp, vp, vp, Fl, vp, U32, vp, vp, vp, vp]),
    "mit_layernorm_param_grads": (I, [L, L, vp, vp, vp, vp]),
    "mit_attention_fwd": (I, [I, L, L, L, L, L, ctypes.POINTER(AttnArgs), vp]),
    "mit_attention_bwd": (I, [I, L, L, L, L, L, ctypes.POINTER(AttnArgs), ctypes.POINTER(AttnGrads), vp]),
    "mit_attention_set_index_limit": (I, [ctypes.c_double]),
    "mit_im2col": (I, [I, L, L, L, L, L, vp, vp, L, vp]),
    "mit_vit_assemble": (I, [I, L, L, L, vp, vp, vp, vp, vp]),
    "mit_embed_fwd": (I, [I, L, L, L, vp, vp, Fl, vp, Fl, vp, U32, vp, vp]),
    "mit_embed_bwd": (I, [I, L, L, L, vp, vp, Fl, Fl, vp, U32, I, vp, vp, vp]),
    "mit_embed_plan_ints": (L, [L]),
    "mit_embed_plan": (I, [vp, L, vp, vp]),
    "mit_count_targets": (I, [vp, L, I, vp, vp]),
    "mit_cross_entropy": (I, [I, L, L, vp, L, vp, I, vp, vp, I, vp, vp]),
    "mit_colsum": (I, [I, L, L, vp, L, vp, I, vp, vp]),
    "mit_colsum_ws_floats": (L, [L, L]),
    "mit_grad_norm_ws_floats": (L, [L]),
    "mit_grad_norm": (I, [vp, L, Fl, vp, vp, vp]),
    "mit_step_inc": (I, [vp, vp]),
    "mit_stamp": (I, [vp, I, vp]),
    "mit_adamw": (I, [L, vp, vp, vp, vp, vp, vp, vp, vp, Fl, Fl, Fl, Fl, vp]),
    "mit_cast_f32": (I, [I, L, vp, vp, vp]),
    "mit_zero": (I, [vp, L, vp]),
    "mit_scalar_div": (I, [vp, vp, vp, vp]),
    "mit_dropout_mask": (I, [L, Fl, vp, U32, vp, vp]),
    "mit_attention_decode": (I, [I, L, L, L, vp, L, vp, L, L, vp, L, L, vp, L, L, vp, vp, L, I, Fl, vp]),
    "mit_kv_store": (I, [I, L, L, vp, L, vp, L, L, vp, vp]),
    "mit_embed_decode": (I, [I, L, L, vp, L, vp, vp, Fl, vp, vp, vp]),
    "mit_image_normalize": (I, [L, L, L, vp, vp, ctypes.POINTER(Fl), ctypes.POINTER(Fl), vp]),
    "mit_plan_begin": (vp, []),
    "mit_plan_end": (vp, []),
    "mit_plan_size": (L, [vp]),
    "mit_plan_run": (I, [vp]),
    "mit_plan_destroy": (None, [vp]),
    "mit_event_record": (I, [vp, vp]),
    "mit_stream_wait_event": (I, [vp, vp]),
    "mit_greedy_pick": (I, [L, L, vp, L, vp, L, vp, ctypes.c_int64, ctypes.c_int64, vp, vp, vp]),
    "mit_greedy_pick_advance": (I, [L, L, vp, L, vp, L, vp, ctypes.c_int64, ctypes.c_int64, vp, vp, vp, vp]),
    "mit_greedy_pick_keys": (I, [L, vp, vp, L, vp, ctypes.c_int64, ctypes.c_int64, vp, vp, vp]),
    "mit_decode_gemm": (I, [ctypes.POINTER(DecodeGemmArgs), vp]),
    "mit_decode_layernorm": (I, [L, L, vp, L, vp, vp, vp, Fl, vp, L, vp]),
}


def load_library(path: str = None) -> ctypes.CDLL:
    """Load the HIP library and declare every signature. Raises if the file is missing.
    MIT_LIB overrides the in-tree path (A/B builds of the same sources, tools/build_variants.sh)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("MIT_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise NativeError(f"libmit_hip.so not found at {path}: build it with `python __graft_entry__.py build` "
                          f"(or `make -C multimodal-image-transformer_amd/csrc`). There is no CPU fallback.")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.mit_abi_version() != ABI_VERSION:
        raise NativeError(f"{path}: ABI version {lib.mit_abi_version()}, this binding needs {ABI_VERSION}: rebuild it")
    _lib = lib
    return lib


def lib() -> ctypes.CDLL:
    return _lib if _lib is not None else load_library()


TORCH_OPS_PATH = os.path.join(_HERE, "lib", "libmit_torch_ops.so")
_torch_ops_loaded = False


def load_torch_ops(path: str = None):
    """Register the dispatcher ops of csrc/torch_ops.cpp (TORCH_LIBRARY(mit_hip)): torch.ops.mit_hip.linear /
    layer_norm / attention over the same kernels (the library links the in-tree libmit_hip.so). Device
    tensors only: a CPU tensor has no kernel registered and the dispatcher raises. Returns torch.ops.mit_hip."""
    global _torch_ops_loaded
    if not _torch_ops_loaded:
        p = path or TORCH_OPS_PATH
        if not os.path.exists(p):
            raise NativeError(f"libmit_torch_ops.so not found at {p}: build it with `python __graft_entry__.py build`")
        torch.ops.load_library(p)
        _torch_ops_loaded = True
    return torch.ops.mit_hip


def require_gpu():
    if not torch.cuda.is_available():
        raise NativeError("multimodal-image-transformer_amd kernels need a ROCm GPU (MI355X / gfx950); none is "
                          "visible. The product path has no CPU fallback.")


def _check(rc: int, name: str):
    if rc != 0:
        msg = lib().mit_last_error()
        raise NativeError(f"{name} failed (rc={rc}): {msg.decode() if msg else ''}")


def ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


_stream_override = None


def stream_ptr():
    """The stream native launches go to: the innermost on_stream() override, else torch's current
    stream (raw lookup: torch.cuda.current_stream() costs ~8 us of Python per call)."""
    if _stream_override is not None:
        return _stream_override
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


class on_stream:
    """Route native launches (only) to the raw HIP stream `ptr` inside the block. torch ops keep
    torch's current stream: use torch.cuda.stream() around code that mixes in torch ops."""

    def __init__(self, ptr):
        self.ptr = ptr

    def __enter__(self):
        global _stream_override
        self.prev, _stream_override = _stream_override, self.ptr

    def __exit__(self, *exc):
        global _stream_override
        _stream_override = self.prev


_hip_rt = None


def hip_runtime() -> ctypes.CDLL:
    """The HIP runtime library this process already uses (torch's, or the one libmit_hip.so links):
    the libamdhip64 mapped into the process (/proc/self/maps), else the first of the usual sonames
    that loads -- never a second runtime of another ROCm major version."""
    global _hip_rt
    if _hip_rt is not None:
        return _hip_rt
    load_library()  # maps the runtime libmit_hip.so was linked against
    paths = []
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split()
                if parts and "libamdhip64.so" in parts[-1] and parts[-1] not in paths:
                    paths.append(parts[-1])
    except OSError:
        pass
    errs = []
    for name in paths + ["libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6"]:
        try:
            _hip_rt = ctypes.CDLL(name)
            return _hip_rt
        except OSError as e:
            errs.append(str(e))
    raise NativeError("cannot load the HIP runtime (libamdhip64): " + "; ".join(errs))


class HipEvents:
    """Timing-free HIP events from a recycled pool, recorded / waited on raw stream pointers
    (cross-stream edges of the step without torch.cuda.Event's Python overhead). Record and wait go
    through the library (mit_event_record / mit_stream_wait_event), so launch plans capture them."""
    _hip = None
    DISABLE_TIMING = 0x2

    def __init__(self, n=64):
        if HipEvents._hip is None:
            h = hip_runtime()
            h.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
            h.hipEventDestroy.argtypes = [vp]
            HipEvents._hip = h
        self.pool = []
        for _ in range(n):
            ev = vp()
            if HipEvents._hip.hipEventCreateWithFlags(ctypes.byref(ev), self.DISABLE_TIMING) != 0:
                raise NativeError("hipEventCreateWithFlags failed")
            self.pool.append(ev)
        self.i = 0

    def record(self, stream):
        """Record the next pool event on `stream`; returns it. A pool slot is reused after len(pool)
        records: callers wait on an event well before that (one step issues < 64)."""
        ev = self.pool[self.i]
        self.i = (self.i + 1) % len(self.pool)
        _check(lib().mit_event_record(ev, stream), "mit_event_record")
        return ev

    def record_at(self, i, stream):
        """Record pool event i (a fixed edge, e.g. one per arena slot) on `stream`; returns it."""
        _check(lib().mit_event_record(self.pool[i], stream), "mit_event_record")
        return self.pool[i]

    @staticmethod
    def wait(stream, ev):
        _check(lib().mit_stream_wait_event(stream, ev), "mit_stream_wait_event")

    def wait_stream(self, stream, other):
        """stream waits for everything issued so far on other."""
        self.wait(stream, self.record(other))


# ------------------------------------------------------------------------------------------------
# recorded programs: native launch plans (mit_plan_*) interleaved with host calls
# ------------------------------------------------------------------------------------------------
class Program:
    """One recorded run of a host function (e.g. a train step + optimizer step): its launches as
    native plans, cut wherever the function made a host call (host_call: a collective, a Python
    callback), which is re-run in place. run() replays everything in the recorded order."""

    def __init__(self):
        self.items = []  # (0, plan handle) | (1, callable)

    def run(self):
        for kind, x in self.items:
            if kind == 0:
                _check(lib().mit_plan_run(x), "mit_plan_run")
            else:
                x()

    def launches(self) -> int:
        return sum(lib().mit_plan_size(x) for k, x in self.items if k == 0)

    def __del__(self):
        if _lib is not None:
            for kind, x in self.items:
                if kind == 0 and x:
                    _lib.mit_plan_destroy(x)
        self.items = []


_recording: Optional[Program] = None
_guard_paused = 0


class _NoTorchKernels(TorchDispatchMode):
    """Active while native.record() runs fn(): a replay re-issues only the recorded NATIVE launches,
    so a torch op that would enqueue GPU work (a fill_, copy_, arithmetic on a CUDA tensor) would be
    silently dropped from every replay. Any such op raises instead. Metadata-only ops (views,
    reshapes, size queries, empty allocations) and ops on CPU tensors pass; host_call() actions (DP
    collectives, callbacks), which are recorded and re-run on replay, are exempt.
    MIT_RECORD_GUARD=0 switches the check off."""
    ALLOWED = {"view", "_unsafe_view", "as_strided", "slice", "select", "narrow", "reshape", "alias", "detach",
               "t", "transpose", "permute", "unsqueeze", "squeeze", "expand", "split", "split_with_sizes",
               "chunk", "unbind", "flatten", "contiguous", "empty", "empty_like", "empty_strided", "view_as",
               "_reshape_alias", "lift_fresh", "sym_size", "sym_stride", "sym_numel", "sym_storage_offset",
               "is_same_size", "_local_scalar_dense", "item", "record_stream", "set_"}

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        name = func.__name__.split(".")[0]
        if not _guard_paused and name not in self.ALLOWED:
            def on_gpu(x):
                return isinstance(x, torch.Tensor) and x.is_cuda
            flat = list(args) + list(kwargs.values())
            # a copy / cast ONTO the GPU (host-to-device, e.g. CPU or int32 tokens in train_step) enqueues
            # a copy kernel too: the replay would read the recording run's temporary
            to_gpu = name == "_to_copy" and torch.device(kwargs.get("device") or "cpu").type == "cuda"
            if to_gpu or any(on_gpu(x) or (isinstance(x, (list, tuple)) and any(on_gpu(y) for y in x)) for x in flat):
                raise NativeError(f"native.record: torch op {func} would enqueue GPU work while recording; a "
                                  f"replay re-issues only native launches and would drop it (do it outside the "
                                  f"recorded function, or through a native entry point / host_call)")
        return func(*args, **kwargs)


def record(fn) -> Program:
    """Run fn() once for real while recording every native launch (and host_call) into a Program.
    A torch op on a CUDA tensor inside fn() raises (see _NoTorchKernels)."""
    global _recording
    if _recording is not None:
        raise NativeError("record: already recording")
    prog = Program()
    if not lib().mit_plan_begin():
        raise NativeError(f"mit_plan_begin failed: {lib().mit_last_error().decode()}")
    _recording = prog
    guard = os.environ.get("MIT_RECORD_GUARD", "1") != "0"
    try:
        if guard:
            with _NoTorchKernels():
                fn()
        else:
            fn()
    finally:
        prog.items.append((0, lib().mit_plan_end()))
        _recording = None
    return prog


def host_call(fn):
    """Run a host-side action now; inside record(), also record it as a host step of the Program
    between two native plans (so a replay re-runs it at the same point of the launch sequence)."""
    global _guard_paused
    if _recording is not None:
        _recording.items.append((0, lib().mit_plan_end()))
        _recording.items.append((1, fn))
        _guard_paused += 1
        try:
            fn()
        finally:
            _guard_paused -= 1
            if not lib().mit_plan_begin():
                raise NativeError(f"mit_plan_begin failed: {lib().mit_last_error().decode()}")
        return
    fn()


def dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.bfloat16:
        return BF16
    if t.dtype == torch.float32:
        return F32
    raise NativeError(f"unsupported dtype {t.dtype}")


# ------------------------------------------------------------------------------------------------
# thin wrappers
# ------------------------------------------------------------------------------------------------
def gemm(A, B, C, M, N, K, *, a_layout=K_CONTIG, b_layout=K_CONTIG, lda=None, ldb=None, ldc=None, bias=None,
         act=ACT_NONE, residual=None, ldr=None, aux=None, ld_aux=None, aux_scale=1.0, alpha=1.0, drop_p=0.0,
         seed=None, site=0, accumulate=False, rowsum=None, workspace=None, ln_stats=None, ln_colsum=None, ln_eps=0.0,
         stats_out=None, tiles=0, argmax_keys=None):
    """C = epi(alpha * A(m,k) B(k,n)); see include/mit_hip.h. Output dtype = C.dtype (f32 or operand dtype).
    argmax_keys: int64 [ARGMAX_SLOTS * M] zeros <- the rows' packed argmax keys (argmax_of_keys); C may be None.
    rowsum: optional f32 [M] <- sum_k A(m,k) (fused bias gradient); workspace: split-K scratch, zero-filled
    once before first use (gemm_workspace(M, N, K)), one per stream. ln_stats / ln_colsum / ln_eps: the
    LayerNorm of A's rows folded in (B, bias already folded: encoder.fold_layernorm); stats_out: f32
    [M, N / 64, 2] <- per-64-column (mean, M2) of the output rows. tiles: 0 per shape, 256 / 128 the tile
    kernel to use where it applies (256: another stream runs beside this launch)."""
    dt = dtype_code(A)
    if B.dtype != A.dtype:
        raise NativeError("gemm: A and B dtypes differ")
    if argmax_keys is not None and argmax_keys.numel() < ARGMAX_SLOTS * M:
        raise NativeError(f"gemm: argmax_keys needs {ARGMAX_SLOTS} x M = {ARGMAX_SLOTS * M} entries")
    if C is not None and C.dtype != A.dtype and C.dtype != torch.float32:
        raise NativeError("gemm: C must be f32 or the operand dtype")
    out_f32 = 1 if C is not None and C.dtype == torch.float32 else 0
    if lda is None:
        lda = K if a_layout == K_CONTIG else M
    if ldb is None:
        ldb = K if b_layout == K_CONTIG else N
    if ldc is None:
        ldc = N
    g = GemmArgs(dt, a_layout, b_layout, M, N, K, ptr(A), lda, ptr(B), ldb, ptr(C), ldc, alpha, ptr(bias), act,
                 ptr(residual), ldr if ldr is not None else ldc, ptr(aux), ld_aux if ld_aux is not None else ldc,
                 aux_scale, drop_p, ptr(seed), site, out_f32, 1 if accumulate else 0, ptr(rowsum), ptr(workspace),
                 0 if workspace is None else workspace.numel() * workspace.element_size(), ptr(ln_stats),
                 ptr(ln_colsum), K // 64 if ln_stats is not None else 0, ln_eps, ptr(stats_out), tiles,
                 ptr(argmax_keys))
    probe = _gemm_probe
    if probe is not None:
        # algorithmic bytes: operands once, output once (+ read-back of C / residual / aux when used)
        esz = A.element_size()
        nbytes = (M * K + N * K) * esz + M * N * (C.element_size() if C is not None else 0) * (2 if accumulate else 1)
        nbytes += M * N * esz * ((residual is not None) + (aux is not None))
        probe.before(dt, a_layout, b_layout, M, N, K, nbytes)
    _check(lib().mit_gemm(ctypes.byref(g), stream_ptr()), "mit_gemm")
    if probe is not None:
        probe.after(g)


def _dw_args(problems):
    arr = (GemmArgs * len(problems))()
    for i, (A, B, C, M, N, K, lda, ldb, rowsum) in enumerate(problems):
        if A.dtype != torch.bfloat16 or B.dtype != torch.bfloat16 or C.dtype != torch.float32:
            raise NativeError("gemm_grouped: bf16 operands and f32 outputs")
        arr[i] = GemmArgs(BF16, MN_CONTIG, MN_CONTIG, M, N, K, ptr(A), lda, ptr(B), ldb, ptr(C), C.stride(0), 1.0, None,
                          ACT_NONE, None, 0, None, 0, 1.0, 0.0, None, 0, 1, 0, ptr(rowsum), None, 0)
    return arr


def gemm_grouped_ws_bytes(problems) -> int:
    return lib().mit_gemm_grouped_ws_bytes(_dw_args(problems), len(problems))


def gemm_grouped(problems, workspace, ln_jobs=()):
    """Weight gradients C_i[M_i, N_i] (f32) = A_i^T B_i of up to 8 problems in one launch
    (mit_gemm_grouped): problems = [(A [K, M] bf16 (row stride lda), B [K, N] bf16 (ldb), C, M, N, K,
    lda, ldb, rowsum f32 [M] or None)], rowsum_i = the bias gradient (row sums of A_i^T).
    ln_jobs: up to 4 (rows, cols, ws, dgamma, dbeta) LayerNorm parameter reductions of partials that
    layernorm_bwd(dgamma=None) left in ws, done by extra blocks of the same grid."""
    arr = _dw_args(problems)
    jobs = (LnGradsJob * max(1, len(ln_jobs)))()
    for i, (rows, cols, lws, dg, db) in enumerate(ln_jobs):
        jobs[i] = LnGradsJob(rows, cols, ptr(lws), ptr(dg), ptr(db))
    wsb = workspace.numel() * workspace.element_size()

    def launch():
        _check(lib().mit_gemm_grouped(arr, len(problems), jobs, len(ln_jobs), ptr(workspace), wsb, stream_ptr()),
               "mit_gemm_grouped")
    probe = _gemm_probe
    if probe is None:
        launch()
        return
    # algorithmic: operands once, f32 output once
    flops = sum(2.0 * M * N * K for _, _, _, M, N, K, _, _, _ in problems)
    nbytes = sum(2 * K * (M + N) + 4 * M * N for _, _, _, M, N, K, _, _, _ in problems)
    probe.grouped(flops, nbytes, launch)


_gemm_probe = None


def gemm_relaunch(g, stream) -> None:
    """Launch a recorded mit_gemm_args again (bench.py replays one step's GEMMs back-to-back)."""
    _check(lib().mit_gemm(ctypes.byref(g), stream), "mit_gemm")


def set_gemm_probe(probe):
    """Install an object with before(dtype, a_layout, b_layout, M, N, K, nbytes) / after(args) called around
    every GEMM launch (bench.py records HIP events there to time the GEMM kernels in place)."""
    global _gemm_probe
    _gemm_probe = probe


def attention_set_index_limit(limit: float = 0.0):
    """Test knob (mit_attention_set_index_limit): dropout attentions with B*H*Lq*Lk >= limit run the 64-bit
    mask-index kernels; 0 restores the default 2^32."""
    _check(lib().mit_attention_set_index_limit(float(limit)), "mit_attention_set_index_limit")


def gemm_set_variant(v):
    """0 = per-shape tile-kernel choice, 1 = 128x128 only, 2 = 256x256 wherever legal, 3 = 64x64
    register-streaming kernel for NT GEMMs, 4 = as 0 with the one-wave-per-SIMD 256x256 kernel for the NT
    bf16 GEMMs it covers (gemm256w_kernel: bitwise equal, measured slower in the step)."""
    _check(lib().mit_gemm_set_variant(int(v)), "mit_gemm_set_variant")


def gemm_plan(g):
    """(tile edge, split-K factor) of the launch mit_gemm would make for recorded args g."""
    ks = ctypes.c_int(1)
    tile = lib().mit_gemm_plan(ctypes.byref(g), ctypes.byref(ks))
    return tile, ks.value


def gemm_workspace_bytes(M, N, K):
    return lib().mit_gemm_workspace_bytes(M, N, K)


def gemm_workspace(M, N, K, device=None):
    """A zero-filled split-K workspace big enough for an (M, N, K) GEMM."""
    return torch.zeros(max(gemm_workspace_bytes(M, N, K), 4096) // 4 + 4, dtype=torch.float32, device=device)


def linear(x, w, out, *, bias=None, act=ACT_NONE, residual=None, drop_p=0.0, seed=None, site=0, workspace=None,
           tiles=0):
    """out[M,N] = act(x[M,K] @ w[N,K]^T + bias) (+ residual) — nn.Linear forward."""
    M, K = x.shape[0], x.shape[-1]
    N = w.shape[0]
    gemm(x, w, out, M, N, K, lda=x.stride(0), bias=bias, act=act, residual=residual, drop_p=drop_p, seed=seed,
         site=site, workspace=workspace, tiles=tiles)


def layernorm_fwd(x, gamma, beta, eps, y, *, r=None, drop_p=0.0, seed=None, site=0, z=None, mean=None, rstd=None,
                  rows=None, cols=None, ldx=None, ldy=None):
    cols = cols if cols is not None else x.shape[-1]
    rows = rows if rows is not None else x.numel() // cols
    _check(lib().mit_layernorm_fwd(dtype_code(x), rows, cols, ptr(x), ldx or cols, ptr(r), cols, drop_p, ptr(seed),
                                   site, ptr(gamma), ptr(beta), eps, ptr(z), ptr(y), ldy or cols, ptr(mean),
                                   ptr(rstd), stream_ptr()), "mit_layernorm_fwd")


def layernorm_fwd_x32(x, gamma, beta, eps, y, *, r=None, z=None, rows=None, cols=None, ldx=None, ldr=None, ldy=None):
    """z = x + r (f32; z may be x), y = LN(z) in y's dtype, for the f32 residual stream x
    (mit_layernorm_fwd_x32; r = the sublayer's bf16 output or None)."""
    if x.dtype != torch.float32 or (z is not None and z.dtype != torch.float32):
        raise NativeError("layernorm_fwd_x32: x and z must be f32")
    if r is not None and r.dtype != torch.bfloat16:
        raise NativeError("layernorm_fwd_x32: r must be bf16")
    cols = cols if cols is not None else x.shape[-1]
    rows = rows if rows is not None else x.numel() // cols
    _check(lib().mit_layernorm_fwd_x32(rows, cols, ptr(x), ldx or cols, ptr(r), ldr or cols, ptr(z), ptr(gamma), ptr(beta),
                                       eps, ptr(y), dtype_code(y), ldy or cols, stream_ptr()), "mit_layernorm_fwd_x32")


def row_stats64(x, out, *, rows=None, cols=None, ldx=None):
    """out f32 [rows, cols / 64, 2] <- per-64-column (mean, M2) of the bf16 rows of x (mit_row_stats64)."""
    cols = cols if cols is not None else x.shape[-1]
    rows = rows if rows is not None else x.numel() // cols
    _check(lib().mit_row_stats64(rows, cols, ptr(x), ldx or cols, ptr(out), stream_ptr()), "mit_row_stats64")


def residual_out(x, r, y, *, rows=None, cols=None, ldx=None, ldr=None, ldy=None):
    """y (bf16) = x (f32) + r (bf16 or None) (mit_residual_out)."""
    cols = cols if cols is not None else x.shape[-1]
    rows = rows if rows is not None else x.numel() // cols
    _check(lib().mit_residual_out(rows, cols, ptr(x), ldx or cols, ptr(r), ldr or cols, ptr(y), ldy or cols,
                                  stream_ptr()),
           "mit_residual_out")


def layernorm_bwd_ws_floats(rows, cols):
    return lib().mit_layernorm_bwd_ws_floats(rows, cols)


def layernorm_bwd(dy, z, mean, rstd, gamma, dx, dgamma, dbeta, ws, *, dr=None, drop_p=0.0, seed=None, site=0):
    """dgamma = dbeta = None: leave the column partials in ws for layernorm_param_grads."""
    cols = z.shape[-1]
    rows = z.numel() // cols
    _check(lib().mit_layernorm_bwd(dtype_code(z), rows, cols, ptr(dy), ptr(z), ptr(mean), ptr(rstd), ptr(gamma),
                                   ptr(dx), ptr(dr), drop_p, ptr(seed), site, ptr(dgamma), ptr(dbeta), ptr(ws),
                                   stream_ptr()), "mit_layernorm_bwd")


def layernorm_param_grads(rows, cols, ws, dgamma, dbeta):
    _check(lib().mit_layernorm_param_grads(rows, cols, ptr(ws), ptr(dgamma), ptr(dbeta), stream_ptr()),
           "mit_layernorm_param_grads")


def attn_args(q, q_row, q_batch, k, k_row, k_batch, v, v_row, v_batch, o, o_row, o_batch, *, lse=None,
              key_tokens=None, tok_batch=0, pad_idx=0, causal=False, scale=0.125, drop_p=0.0, seed=None, site=0):
    return AttnArgs(ptr(q), q_row, q_batch, ptr(k), k_row, k_batch, ptr(v), v_row, v_batch, ptr(o), o_row, o_batch,
                    ptr(lse), ptr(key_tokens), tok_batch, pad_idx, 1 if causal else 0, scale, drop_p, ptr(seed), site)


def attention_fwd(dtype, B, H, Lq, Lk, args: AttnArgs, Dh=64):
    _check(lib().mit_attention_fwd(dtype, B, H, Lq, Lk, Dh, ctypes.byref(args), stream_ptr()), "mit_attention_fwd")


def attention_bwd(dtype, B, H, Lq, Lk, args: AttnArgs, grads: AttnGrads, Dh=64):
    _check(lib().mit_attention_bwd(dtype, B, H, Lq, Lk, Dh, ctypes.byref(args), ctypes.byref(grads), stream_ptr()),
           "mit_attention_bwd")


def attn_grads(dout, do_row, do_batch, dq, dq_row, dq_batch, dk, dk_row, dk_batch, dv, dv_row, dv_batch, delta_ws):
    return AttnGrads(ptr(dout), do_row, do_batch, ptr(dq), dq_row, dq_batch, ptr(dk), dk_row, dk_batch, ptr(dv),
                     dv_row, dv_batch, ptr(delta_ws))


def im2col(img, out, patch, kpad):
    B, C, H, W = img.shape
    _check(lib().mit_im2col(dtype_code(out), B, C, H, W, patch, ptr(img), ptr(out), kpad, stream_ptr()), "mit_im2col")


def vit_assemble(patch_out, cls, pos, h, B, np_, E):
    _check(lib().mit_vit_assemble(dtype_code(h), B, np_, E, ptr(patch_out), ptr(cls), ptr(pos), ptr(h), stream_ptr()),
           "mit_vit_assemble")


def embed_fwd(tokens, table, scale, pe, out, *, drop_p=0.0, seed=None, site=0):
    B, T = tokens.shape
    d = table.shape[1]
    _check(lib().mit_embed_fwd(dtype_code(out), B, T, d, ptr(tokens), ptr(table), scale, ptr(pe), drop_p, ptr(seed),
                               site, ptr(out), stream_ptr()), "mit_embed_fwd")


def embed_plan_ints(n):
    return lib().mit_embed_plan_ints(n)


def embed_plan(tokens, plan):
    """plan (int32 [embed_plan_ints(tokens.numel())]) <- the deterministic scatter order of tokens."""
    _check(lib().mit_embed_plan(ptr(tokens), tokens.numel(), ptr(plan), stream_ptr()), "mit_embed_plan")


def embed_bwd(tokens, dx, scale, dtable, pad_idx, *, drop_p=0.0, seed=None, site=0, plan=None):
    """plan from embed_plan(tokens): deterministic; None: float atomics."""
    B, T = tokens.shape
    d = dtable.shape[1]
    _check(lib().mit_embed_bwd(dtype_code(dx), B, T, d, ptr(tokens), ptr(dx), scale, drop_p, ptr(seed), site,
                               pad_idx, ptr(plan), ptr(dtable), stream_ptr()), "mit_embed_bwd")


def count_targets(targets, ignore_index, count):
    _check(lib().mit_count_targets(ptr(targets), targets.numel(), ignore_index, ptr(count), stream_ptr()),
           "mit_count_targets")


def cross_entropy(logits, targets, ignore_index, count, loss_sum, want_grad, rows=None, V=None, ld=None,
                  row_loss=None):
    """loss_sum += sum of -log p[target]; if want_grad, logits <- (softmax - onehot) / count (in place).
    row_loss: optional f32 [rows] scratch -> deterministic (row-ordered) loss sum."""
    V = V if V is not None else logits.shape[-1]
    rows = rows if rows is not None else targets.numel()
    _check(lib().mit_cross_entropy(dtype_code(logits), rows, V, ptr(logits), ld or V, ptr(targets), ignore_index,
                                   ptr(count), ptr(loss_sum), 1 if want_grad else 0, ptr(row_loss), stream_ptr()),
           "mit_cross_entropy")


def scalar_div(a, b, out):
    _check(lib().mit_scalar_div(ptr(a), ptr(b), ptr(out), stream_ptr()), "mit_scalar_div")


def zero(t):
    """Zero a tensor's storage span with hipMemsetAsync (t must be contiguous)."""
    _check(lib().mit_zero(ptr(t), t.numel() * t.element_size(), stream_ptr()), "mit_zero")


def colsum_ws_floats(M, N):
    return lib().mit_colsum_ws_floats(M, N)


def colsum(dy, M, N, out, ws, *, ld=None, accumulate=False):
    _check(lib().mit_colsum(dtype_code(dy), M, N, ptr(dy), ld or N, ptr(out), 1 if accumulate else 0, ptr(ws),
                            stream_ptr()), "mit_colsum")


def grad_norm_ws_floats(n):
    return lib().mit_grad_norm_ws_floats(n)


def grad_norm(grads, max_norm, ws, norm_out):
    _check(lib().mit_grad_norm(ptr(grads), grads.numel(), max_norm, ptr(ws), ptr(norm_out), stream_ptr()),
           "mit_grad_norm")


def stamp(buf: torch.Tensor, idx: int, stream=None):
    """buf[idx] (int64 device tensor) = device wall clock when `stream` (default: current) gets here."""
    _check(lib().mit_stamp(ptr(buf), int(idx), stream if stream is not None else stream_ptr()), "mit_stamp")


def step_inc(step):
    _check(lib().mit_step_inc(ptr(step), stream_ptr()), "mit_step_inc")


def adamw(param, grad, m, v, shadow, norm_out, lr, step, beta1, beta2, eps, weight_decay):
    _check(lib().mit_adamw(param.numel(), ptr(param), ptr(grad), ptr(m), ptr(v), ptr(shadow), ptr(norm_out), ptr(lr),
                           ptr(step), beta1, beta2, eps, weight_decay, stream_ptr()), "mit_adamw")


def cast_f32(src, dst):
    _check(lib().mit_cast_f32(dtype_code(dst), src.numel(), ptr(src), ptr(dst), stream_ptr()), "mit_cast_f32")


def dropout_mask(n, p, seed, site, out):
    _check(lib().mit_dropout_mask(n, p, ptr(seed), site, ptr(out), stream_ptr()), "mit_dropout_mask")


# --- batched greedy decoding (decode.hip) -------------------------------------------------------
def attention_decode(q, q_batch, k, k_row, k_batch, v, v_row, v_batch, o, o_batch, B, H, *, Lk=0, pos=None,
                     key_tokens=None, tok_batch=0, pad_idx=0, scale=0.125, Dh=64):
    """One query per (b, h) over Lk keys (Lk = pos+1 from the device scalar when pos is given)."""
    _check(lib().mit_attention_decode(dtype_code(q), B, H, Dh, ptr(q), q_batch, ptr(k), k_row, k_batch, ptr(v), v_row,
                                      v_batch, ptr(o), o_batch, Lk, ptr(pos), ptr(key_tokens), tok_batch, pad_idx,
                                      scale, stream_ptr()), "mit_attention_decode")


def kv_store(src, s_batch, cache, c_row, c_batch, B, n, pos):
    _check(lib().mit_kv_store(dtype_code(src), B, n, ptr(src), s_batch, ptr(cache), c_row, c_batch, ptr(pos),
                              stream_ptr()), "mit_kv_store")


def embed_decode(ids, pos, table, scale, pe, out):
    B, ld = ids.shape
    _check(lib().mit_embed_decode(dtype_code(table), B, table.shape[1], ptr(ids), ld, ptr(pos), ptr(table), scale,
                                  ptr(pe), ptr(out), stream_ptr()), "mit_embed_decode")


def greedy_pick(logits, ids, pos, end_id, pad_id, finished, n_finished, V=None):
    B = logits.shape[0]
    V = V if V is not None else logits.shape[1]
    _check(lib().mit_greedy_pick(B, V, ptr(logits), logits.stride(0), ptr(ids), ids.shape[1], ptr(pos), int(end_id),
                                 int(pad_id), ptr(finished), ptr(n_finished), stream_ptr()), "mit_greedy_pick")


def greedy_pick_advance(logits, ids, pos, end_id, pad_id, finished, n_finished, ticket, V=None):
    """greedy_pick, then pos += 1 (int32 `ticket` device counter, 0 before and after)."""
    B = logits.shape[0]
    V = V if V is not None else logits.shape[1]
    _check(lib().mit_greedy_pick_advance(B, V, ptr(logits), logits.stride(0), ptr(ids), ids.shape[1], ptr(pos),
                                         int(end_id), int(pad_id), ptr(finished), ptr(n_finished), ptr(ticket),
                                         stream_ptr()), "mit_greedy_pick_advance")


def decode_gemm(a, w, *, out=None, bias=None, act=ACT_NONE, a_ln=None, residual=None, r_ln=None, eps=1e-5,
                z_out=None, stats_out=None, cache=None, c_row=0, c_batch=0, kv_col0=0, pos=None, argmax_keys=None):
    """Decode-step GEMM (mit_decode_gemm): out = act(A' w^T + bias) (+ residual), w bf16 [N, K].
    a: bf16 rows [M, K], or f32 pre-LN sums when a_ln = (stats, gamma, beta) (A' = LN(a));
    residual: bf16 rows, or f32 pre-LN sums when r_ln = (stats, gamma, beta) (+ LN(residual));
    z_out / stats_out: f32 pre-LN sum of the next LayerNorm and its per-64-column row statistics
    [M, ceil(N/64), 2]; cache: the columns >= kv_col0 also go to cache[m*c_batch + pos*c_row + n - kv_col0];
    argmax_keys: int64 [ARGMAX_SLOTS * M] zeros <- per row and slot the packed (value, first column) maximum
    of the column blocks of that slot (the greedy pick folded into the head: greedy_pick_keys, argmax_of_keys)."""
    M, K = a.shape[0], a.shape[-1]
    if argmax_keys is not None and argmax_keys.numel() < ARGMAX_SLOTS * M:
        raise NativeError(f"decode_gemm: argmax_keys needs {ARGMAX_SLOTS} x M = {ARGMAX_SLOTS * M} entries")
    N = w.shape[0]
    r_mode = 0 if residual is None else (2 if r_ln is not None else 1)
    g = DecodeGemmArgs(M, N, K, ptr(a), a.stride(0), ptr(a_ln[0]) if a_ln else None, ptr(a_ln[1]) if a_ln else None,
                       ptr(a_ln[2]) if a_ln else None, ptr(w), w.stride(0), ptr(bias), act,
                       1 if out is not None and out.dtype == torch.float32 else 0, ptr(out),
                       out.stride(0) if out is not None else 0, r_mode, ptr(residual),
                       residual.stride(0) if residual is not None else 0, ptr(r_ln[0]) if r_ln else None,
                       ptr(r_ln[1]) if r_ln else None, ptr(r_ln[2]) if r_ln else None, eps, ptr(z_out),
                       z_out.stride(0) if z_out is not None else 0, ptr(stats_out), ptr(cache), c_row, c_batch, kv_col0,
                       ptr(pos), ptr(argmax_keys))
    _check(lib().mit_decode_gemm(ctypes.byref(g), stream_ptr()), "mit_decode_gemm")


def greedy_pick_keys(keys, ids, pos, end_id, pad_id, finished, n_finished):
    """ids[:, pos + 1] <- the picks a decode_gemm(argmax_keys=keys) left (keys reset to 0), then pos += 1."""
    B = ids.shape[0]
    if keys.numel() != ARGMAX_SLOTS * B:
        raise NativeError(f"greedy_pick_keys: keys must hold {ARGMAX_SLOTS} x B = {ARGMAX_SLOTS * B} entries")
    _check(lib().mit_greedy_pick_keys(B, ptr(keys), ptr(ids), ids.shape[1], ptr(pos), int(end_id), int(pad_id),
                                      ptr(finished), ptr(n_finished), stream_ptr()), "mit_greedy_pick_keys")


def argmax_of_keys(keys, M):
    """The column each row's argmax keys (int64 [ARGMAX_SLOTS * M], unsigned packed keys) name: the largest
    key over the row's slots, unsigned order (host-side helper for tests and tools)."""
    k = keys.view(ARGMAX_SLOTS, M) ^ torch.iinfo(torch.int64).min  # unsigned order as signed order
    best = k.max(0).values ^ torch.iinfo(torch.int64).min
    return 0xFFFFFFFF - (best & 0xFFFFFFFF)


def decode_layernorm(z, stats, gamma, beta, out, eps=1e-5):
    """out (bf16 [M, W]) = LN(z) from mit_decode_gemm row statistics."""
    M, W = z.shape
    _check(lib().mit_decode_layernorm(M, W, ptr(z), z.stride(0), ptr(stats), ptr(gamma), ptr(beta), eps, ptr(out),
                                      out.stride(0), stream_ptr()), "mit_decode_layernorm")


def image_normalize(src_u8, dst, mean, std):
    """dst [B,3,H,W] f32 <- (src [B,H,W,3] uint8 / 255 - mean) / std (mit_image_normalize)."""
    B, H, W, C = src_u8.shape
    if C != 3 or src_u8.dtype != torch.uint8 or dst.dtype != torch.float32:
        raise NativeError("image_normalize: src uint8 [B,H,W,3], dst f32 [B,3,H,W]")
    m = (Fl * 3)(*[float(x) for x in mean])
    s = (Fl * 3)(*[float(x) for x in std])
    _check(lib().mit_image_normalize(B, H, W, ptr(src_u8), ptr(dst), m, s, stream_ptr()), "mit_image_normalize")
