"""The C-ABI library loads and exports exactly what include/mit_hip.h declares (CPU-only test:
dlopen + symbol lookup, no kernel launches)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mit_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mit_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_functions():
    names = declared_functions()
    assert "mit_gemm" in names and "mit_attention_bwd" in names and len(names) >= 20


def test_library_exports_every_declared_symbol():
    import native
    if not os.path.exists(native.LIB_PATH):
        pytest.fail(f"library not built: {native.LIB_PATH} (run python __graft_entry__.py build)")
    lib = ctypes.CDLL(native.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, f"missing exports: {missing}"
    assert lib.mit_abi_version() == 6


def test_python_binding_covers_header():
    import native
    assert sorted(native.SIGNATURES) == declared_functions()


def test_binding_loads_and_rejects_bad_args_without_gpu():
    import native
    lib = native.load_library()
    # argument validation happens before any launch, so this runs on a CPU-only host
    g = native.GemmArgs(native.BF16, 0, 0, 16, 16, 16, None, 16, None, 16, None, 16, 1.0)
    rc = lib.mit_gemm(ctypes.byref(g), None)
    assert rc == 1 and b"null operand" in lib.mit_last_error()
