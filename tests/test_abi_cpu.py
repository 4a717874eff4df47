"""CPU checks of the boundary: the C-ABI library loads and exports every symbol include/ahr.h
declares (no compute calls), the header and the Python binding agree, and the product modules
import without a GPU."""
import ctypes
import os
import re

from conftest import ROOT


def _header_symbols():
    with open(os.path.join(ROOT, "include", "ahr.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(ahr_\w+)\(", src, flags=re.M)))


def test_header_and_binding_agree():
    from ah_rag import _native
    assert sorted(_native.EXPORTED_SYMBOLS) == _header_symbols()


def test_library_exports_every_declared_symbol():
    from ah_rag import _native
    lib = _native.lib()
    for name in _header_symbols():
        assert hasattr(lib, name), name
    assert lib.ahr_abi_version() == 1


def test_error_channel_without_gpu():
    from ah_rag import _native
    lib = _native.lib()
    # argument validation happens before any device call
    rc = lib.ahr_index_create(0, 0, 10, 0, ctypes.byref(ctypes.c_void_p()))
    assert rc == _native.AHR_EINVAL
    assert b"dim" in lib.ahr_last_error()


def test_key_decode_host_helper():
    import numpy as np
    from ah_rag import _native
    from ah_rag.embeddings import decode_keys
    lib = _native.lib()
    vals = np.array([0.5, -0.25, 1.0, -3.0], np.float32)
    rows = np.array([7, 0, 123456, 5], np.uint32)
    u = vals.view(np.uint32)
    ordv = np.where(u & 0x80000000, ~u, u | 0x80000000).astype(np.uint64)
    keys = (ordv << np.uint64(32)) | (np.uint64(0xFFFFFFFF) - rows.astype(np.uint64))
    s = np.empty(4, np.float32)
    r = np.empty(4, np.int64)
    assert lib.ahr_key_decode(keys.ctypes.data, 4, s.ctypes.data, r.ctypes.data) == 0
    np.testing.assert_array_equal(s, vals)
    np.testing.assert_array_equal(r, rows.astype(np.int64))
    s2, r2 = decode_keys(keys)
    np.testing.assert_array_equal(s2, vals)
    np.testing.assert_array_equal(r2, rows.astype(np.int64))
    # key order == (score desc, row asc)
    order = np.argsort(-keys.astype(np.float64))
    assert list(order) == [2, 0, 1, 3]


def test_product_imports_without_gpu():
    import ah_rag.agent.environment  # noqa: F401
    import ah_rag.agent.gym_env  # noqa: F401
    import ah_rag.graph.hierarchical_graph  # noqa: F401
    import ah_rag.graph_search  # noqa: F401
    import baselines.naive_rag  # noqa: F401
