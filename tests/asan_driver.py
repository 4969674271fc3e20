"""Host-code AddressSanitizer run of the C ABI (SURVEY.md §5 sanitizers), CPU only: loads the
ASan-instrumented libmit_hip (make -C multimodal-image-transformer_amd/csrc asan) through the same
ctypes signatures as native.py and drives every entry point's argument validation and the launch-plan
recorder (mit_plan_*) with arguments that must be rejected before any HIP call. Run by
tests/test_capi_asan.py in a child process with the ASan runtime preloaded; any ASan report aborts it.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-image-transformer_amd"))

import native  # noqa: E402

SAFE_ZERO = {  # entry points that are valid with all-zero / null arguments or only query
    "mit_last_error", "mit_abi_version", "mit_gemm_workspace_bytes", "mit_gemm_grouped_ws_bytes",
    "mit_layernorm_bwd_ws_floats", "mit_colsum_ws_floats", "mit_grad_norm_ws_floats", "mit_plan_begin",
    "mit_plan_end", "mit_plan_size", "mit_plan_destroy", "mit_gemm_set_variant",
    "mit_gemm_plan", "mit_embed_plan_ints", "mit_event_record", "mit_stream_wait_event"}


def zero_args(argtypes):
    out = []
    for t in argtypes:
        if t in (ctypes.c_float, ctypes.c_double):
            out.append(t(0.0))
        elif t in (ctypes.c_int, ctypes.c_long, ctypes.c_uint32, ctypes.c_uint, ctypes.c_ulong, ctypes.c_int64):
            out.append(t(0))
        else:
            out.append(None)  # every pointer / struct pointer: NULL
    return out


def main(path):
    lib = native.load_library(path)
    rejected = 0
    # 1. every launching entry point with all-null / zero arguments: rejected by its argument checks
    for name, (_, argtypes) in sorted(native.SIGNATURES.items()):
        if name in SAFE_ZERO:
            continue
        rc = getattr(lib, name)(*zero_args(argtypes))
        msg = lib.mit_last_error()
        if rc == 0:
            # a zero-size call may legitimately be a no-op; it must not have touched anything
            continue
        assert isinstance(msg, bytes) and len(msg) > 0, (name, rc)
        rejected += 1
    assert rejected >= 30, rejected
    # 2. mit_gemm's checks one by one (the struct the C ABI copies by value into the plan recorder)
    base = dict(dtype=native.BF16, a_layout=0, b_layout=0, M=64, N=64, K=64, lda=64, ldb=64, ldc=64)
    bufs = [ctypes.create_string_buffer(64 * 64 * 4 + 64) for _ in range(3)]
    al = [ctypes.addressof(b) + (-ctypes.addressof(b)) % 16 for b in bufs]

    def gemm(**kw):
        a = dict(base, **kw)
        g = native.GemmArgs(a["dtype"], a["a_layout"], a["b_layout"], a["M"], a["N"], a["K"], a.get("A", al[0]),
                            a["lda"], a.get("B", al[1]), a["ldb"], a.get("C", al[2]), a["ldc"], 1.0)
        return lib.mit_gemm(ctypes.byref(g), None), lib.mit_last_error()
    for kw, frag in [(dict(dtype=7), b"bad dtype"), (dict(M=-1), b"negative"), (dict(A=None), b"null operand"),
                     (dict(a_layout=5), b"a_layout"), (dict(lda=8), b"lda too small"), (dict(ldc=4), b"ldc too small"),
                     (dict(lda=66), b"multiples of 8"), (dict(A=al[0] + 2), b"aligned")]:
        rc, msg = gemm(**kw)
        assert rc != 0 and frag in msg, (kw, rc, msg)
    # 3. the plan recorder: closures copy their arguments (the GemmArgs struct dies before the replay)
    plan = lib.mit_plan_begin()
    assert plan
    assert not lib.mit_plan_begin() and b"already recording" in lib.mit_last_error()
    for _ in range(3):
        rc, _ = gemm(A=None)  # recorded, then rejected
        assert rc != 0
    g = native.GemmArgs(native.BF16, 0, 0, 8, 8, 8, None, 8, None, 8, None, 8, 1.0)
    lib.mit_gemm(ctypes.byref(g), None)
    del g
    p = lib.mit_plan_end()
    assert p and lib.mit_plan_size(p) == 4
    assert not lib.mit_plan_end() and b"not recording" in lib.mit_last_error()
    assert lib.mit_plan_run(p) != 0 and b"null operand" in lib.mit_last_error()
    assert lib.mit_plan_run(None) != 0
    lib.mit_plan_destroy(p)
    lib.mit_plan_destroy(None)
    # 4. an empty plan replays as a no-op
    p = lib.mit_plan_begin()
    p = lib.mit_plan_end()
    assert lib.mit_plan_size(p) == 0 and lib.mit_plan_run(p) == 0
    lib.mit_plan_destroy(p)
    print(f"asan driver: {rejected} entry points rejected null arguments; gemm checks and plan recorder clean",
          flush=True)


if __name__ == "__main__":
    main(sys.argv[1])
