"""SURVEY.md §5 sanitizer row: the C ABI's host code (argument validation of every entry point, the
launch-plan recorder) under AddressSanitizer, on the CPU. The instrumented library is built by
`make -C multimodal-image-transformer_amd/csrc asan` (__graft_entry__.build() runs it); the driver
(tests/asan_driver.py) runs in a child process with the compiler's ASan runtime preloaded, so any
heap / stack / use-after-free report fails the test."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_LIB = os.path.join(ROOT, "multimodal-image-transformer_amd", "lib", "asan", "libmit_hip_asan.so")


def _runtime():
    hits = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return hits[-1] if hits else None


def test_c_abi_host_code_is_asan_clean():
    rt = _runtime()
    if rt is None:
        pytest.skip("no clang ASan runtime in this image")
    if not os.path.exists(ASAN_LIB):
        pytest.skip("ASan library not built (make -C multimodal-image-transformer_amd/csrc asan)")
    env = dict(os.environ, LD_PRELOAD=":".join(x for x in (rt, os.environ.get("LD_PRELOAD", "")) if x),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1:verify_asan_link_order=0",
               HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "asan_driver.py"), ASAN_LIB], env=env,
                       capture_output=True, text=True, timeout=600)
    assert "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "plan recorder clean" in r.stdout
