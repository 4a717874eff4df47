"""Test configuration: paths, the `gpu` marker, shared fixtures.

`-m "not gpu"` runs on this CPU-only container: oracle vs golden vectors, host logic, the
C-ABI export check, gloo multi-process tests. `-m gpu` runs on an MI355X and calls the HIP
kernels through libahr_hip.so, checking them against oracle/ (never the other way round).
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ah-rag_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm) GPU and libahr_hip.so")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test started without a visible ROCm GPU")
    from ah_rag import _native
    _native.lib()  # fail loudly if the HIP library is missing
    return torch.device("cuda", 0)
