"""Host-side paths of the C ABI that run without a GPU: argument validation, CSR checks and the
host image of ahr_graph_create, merge-shape checks, key decode. These are the paths the
AddressSanitizer build exercises (tests/test_asan_cpu.py runs this file under it); every call
here returns before any kernel launch."""
import ctypes

import numpy as np

P = ctypes.c_void_p


def _lib():
    from ah_rag import _native
    return _native, _native.lib()


def test_index_argument_validation():
    nat, lib = _lib()
    h = P()
    assert lib.ahr_index_create(768, 7, 10, 0, ctypes.byref(h)) == nat.AHR_EINVAL  # unknown dtype
    assert b"dtype" in lib.ahr_last_error()
    assert lib.ahr_index_create(768, 0, -1, 0, ctypes.byref(h)) == nat.AHR_EINVAL
    assert lib.ahr_index_create(768, 0, 10, 0, None) == nat.AHR_EINVAL
    n = ctypes.c_int64()
    assert lib.ahr_index_count(None, ctypes.byref(n)) == nat.AHR_EINVAL
    assert lib.ahr_index_upsert(None, None, 0, None, 0, 0, None) == nat.AHR_EINVAL
    assert lib.ahr_index_query(None, None, 1, 10, 0, None, None, None) == nat.AHR_EINVAL
    assert lib.ahr_index_set_workspace(None, 0) == nat.AHR_EINVAL
    assert lib.ahr_index_destroy(None) == nat.AHR_OK


def test_merge_shape_validation():
    nat, lib = _lib()
    assert lib.ahr_topk_merge(None, -1, 1, 1, 1, None, None, None, None) == nat.AHR_EINVAL
    assert lib.ahr_topk_merge(None, 1, 1, 1, 5000, None, None, None, None) == nat.AHR_EUNSUP
    assert lib.ahr_topk_merge(None, 0, 1, 1, 4, None, None, None, None) == nat.AHR_OK  # empty batch
    assert lib.ahr_topk_merge(None, 2, 3, 4, 4, None, None, None, None) == nat.AHR_EINVAL  # null keys


def _csr(n, edges):
    """CSR offsets/targets for n nodes from (src, dst) pairs in order."""
    off = np.zeros(n + 1, np.int64)
    tgt = []
    for u in range(n):
        vs = [v for a, v in edges if a == u]
        tgt += vs
        off[u + 1] = len(tgt)
    return off, np.asarray(tgt if tgt else [0], np.int32)


def test_graph_create_validates_csr_before_the_device():
    nat, lib = _lib()
    n = 6
    types = np.array([1, 1, 2, 2, 3, 0], np.int8)
    judge = np.full(n, np.nan)
    conf = np.full(n, np.nan)
    terms = np.zeros(n)
    good = [_csr(n, [(0, 2), (1, 3)]), _csr(n, [(2, 0), (3, 1)]), _csr(n, []), _csr(n, []),
            _csr(n, [(0, 4)]), _csr(n, [(4, 0)])]
    bad_target = list(good)
    bad_target[0] = (good[0][0], np.array([2, 99], np.int32))  # node 99 out of range
    bad_offsets = list(good)
    o = good[1][0].copy()
    o[0] = 1
    bad_offsets[1] = (o, good[1][1])
    for adj, want in ((bad_target, nat.AHR_ERANGE), (bad_offsets, nat.AHR_EINVAL)):
        offs = (P * nat.AHR_ADJ_COUNT)(*[a[0].ctypes.data for a in adj])
        tgts = (P * nat.AHR_ADJ_COUNT)(*[a[1].ctypes.data for a in adj])
        g = P()
        rc = lib.ahr_graph_create(n, types.ctypes.data, judge.ctypes.data, conf.ctypes.data, terms.ctypes.data,
                                  terms.ctypes.data, offs, tgts, 0, ctypes.byref(g))
        assert rc == want, (rc, lib.ahr_last_error())
        assert not g.value
    assert lib.ahr_graph_create(-1, None, None, None, None, None, None, None, 0, ctypes.byref(P())) == nat.AHR_EINVAL
    assert lib.ahr_graph_create(2, None, None, None, None, None, None, None, 0, ctypes.byref(P())) == nat.AHR_EINVAL
    params = nat.RerankParams()
    assert lib.ahr_graph_expand_rerank(None, None, None, 1, 1, ctypes.byref(params), 4, *([None] * 8),
                                       None) == nat.AHR_EINVAL
    assert lib.ahr_graph_expand(None, 0, None, 1, 1, 10, None, None, None) == nat.AHR_EINVAL


def test_expand_host_validation_and_workspace_size():
    """ahr_graph_expand_host's argument checks and ahr_graph_expand_ws_bytes' layout (inputs,
    out [B][max(limit, 1)], count [B], each part rounded up to 256 B): host arithmetic only."""
    nat, lib = _lib()
    n = ctypes.c_int64()
    assert lib.ahr_graph_expand_ws_bytes(1, 3, 10, ctypes.byref(n)) == nat.AHR_OK
    assert n.value == 256 * 3
    assert lib.ahr_graph_expand_ws_bytes(100, 3, 0, ctypes.byref(n)) == nat.AHR_OK
    assert n.value == 1280 + 512 + 512  # 1200 B inputs, out of width 1, 400 B counts
    assert lib.ahr_graph_expand_ws_bytes(-1, 3, 10, ctypes.byref(n)) == nat.AHR_EINVAL
    assert lib.ahr_graph_expand_ws_bytes(1, 3, 10, None) == nat.AHR_EINVAL
    buf = (ctypes.c_int32 * 64)()
    assert lib.ahr_graph_expand_host(None, 0, buf, 1, 3, 10, buf, buf, buf, 4096, None) == nat.AHR_EINVAL
    assert b"graph" in lib.ahr_last_error()


def test_key_decode_edge_values():
    nat, lib = _lib()
    from ah_rag.distributed import encode_keys_host
    vals = np.array([np.inf, -np.inf, 0.0, -0.0, 1e-38, -1e38], np.float32)
    rows = np.array([0, 1, 2, 3, 0xFFFFFFFE, 5], np.int64)
    keys = encode_keys_host(vals, rows)
    s = np.empty(len(vals), np.float32)
    r = np.empty(len(vals), np.int64)
    assert lib.ahr_key_decode(keys.ctypes.data, len(vals), s.ctypes.data, r.ctypes.data) == nat.AHR_OK
    np.testing.assert_array_equal(s, vals)
    np.testing.assert_array_equal(r, rows)
    assert lib.ahr_key_decode(None, 0, None, None) == nat.AHR_OK
    assert lib.ahr_key_decode(None, 3, None, None) == nat.AHR_EINVAL
    empty = np.zeros(2, np.uint64)  # key 0 = empty slot
    assert lib.ahr_key_decode(empty.ctypes.data, 2, s.ctypes.data, r.ctypes.data) == nat.AHR_OK
    assert np.isneginf(s[:2]).all() and (r[:2] == -1).all()
