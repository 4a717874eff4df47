"""The host-side C++ of libahr_hip under AddressSanitizer (sanitizer builds of the C ABI).

__graft_entry__.build_asan() compiles the library with -fsanitize=address on the host code only
(GPU ASan is not available on this pool). This test runs the no-GPU ABI tests in a child Python
with the clang ASan runtime preloaded and AHR_LIB_PATH pointing at that build; any ASan report
(heap overflow, use-after-free, ...) fails it.
"""
import os
import subprocess
import sys

from conftest import ROOT


def test_abi_host_paths_under_asan():
    sys.path.insert(0, ROOT)
    import __graft_entry__ as g
    lib = g.build_asan()
    rt = g.asan_runtime()
    assert os.path.exists(rt), rt
    env = dict(os.environ, LD_PRELOAD=rt, AHR_LIB_PATH=lib,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1")
    cmd = [sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider",
           os.path.join(ROOT, "tests", "test_abi_cpu.py"), os.path.join(ROOT, "tests", "test_abi_host_cpu.py")]
    res = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    out = res.stdout + res.stderr
    assert "AddressSanitizer" not in out, out[-4000:]
    assert res.returncode == 0, out[-4000:]
    assert " passed" in out
