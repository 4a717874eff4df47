"""Dense top-k oracle (test infrastructure only; see oracle/__init__.py).

Restates an exhaustive cosine query of the reference's Chroma collection
(reference src/ah_rag/graph/hierarchical_graph.py:611 space=cosine, :714 coll.query) over
L2-normalised vectors (:656, :712): top-k rows by inner product, ties by row ascending.
"""
from __future__ import annotations

import ctypes
import os
from typing import Tuple

import numpy as np

from .build import LIB, build

_lib = None


def _c():
    global _lib
    if _lib is None:
        path = LIB if os.path.exists(LIB) else build()
        _lib = ctypes.CDLL(path)
        P = ctypes.c_void_p
        _lib.ahr_oracle_dense_topk.argtypes = [P, ctypes.c_int64, P, ctypes.c_int64, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_int, P, P]
        _lib.ahr_oracle_scores.argtypes = [P, ctypes.c_int64, P, ctypes.c_int64, ctypes.c_int,
                                           ctypes.c_int, P]
        _lib.ahr_oracle_round_bf16.argtypes = [P, P, ctypes.c_int64]
        _lib.ahr_oracle_threads.restype = ctypes.c_int
    return _lib


def _f32(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.float32))


def round_to_storage(x: np.ndarray, dtype: str) -> np.ndarray:
    """fp32 values after the device's storage conversion (RNE), as fp32."""
    x = _f32(x)
    if dtype in ("f32", "fp32", "float32"):
        return x.copy()
    if dtype in ("f16", "fp16", "float16"):
        return x.astype(np.float16).astype(np.float32)
    out = np.empty_like(x)
    _c().ahr_oracle_round_bf16(x.ctypes.data, out.ctypes.data, x.size)
    return out


def normalize_rows(x: np.ndarray) -> np.ndarray:
    x = _f32(x)
    n = np.sqrt((x.astype(np.float64) ** 2).sum(axis=1, keepdims=True))
    return (x / np.maximum(n, 1e-12)).astype(np.float32)


def topk(corpus: np.ndarray, queries: np.ndarray, k: int, mode: str = "fma") -> Tuple[np.ndarray, np.ndarray]:
    """Exact top-k (scores float64 [B,k], rows int64 [B,k]).

    mode "fma": fp32 fma chain in k order (bit-exact contract of the f32 device mode).
    mode "f64": double accumulation of the given (already storage-rounded) values.
    """
    c, q = _f32(corpus), _f32(queries)
    n, d = c.shape
    B = q.shape[0]
    scores = np.empty((B, k), np.float64)
    rows = np.empty((B, k), np.int64)
    rc = _c().ahr_oracle_dense_topk(c.ctypes.data, n, q.ctypes.data, B, d, int(k),
                                    0 if mode == "fma" else 1, scores.ctypes.data, rows.ctypes.data)
    assert rc == 0
    return scores, rows


def scores_matrix(corpus: np.ndarray, queries: np.ndarray, mode: str = "fma") -> np.ndarray:
    c, q = _f32(corpus), _f32(queries)
    out = np.empty((q.shape[0], c.shape[0]), np.float32)
    _c().ahr_oracle_scores(c.ctypes.data, c.shape[0], q.ctypes.data, q.shape[0], c.shape[1],
                           0 if mode == "fma" else 1, out.ctypes.data)
    return out


def threads() -> int:
    return int(_c().ahr_oracle_threads())


def topk_numpy(corpus: np.ndarray, queries: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
    """The CPU baseline path of BASELINE.md: BLAS fp32 Q @ C.T + argpartition, tie rule
    (score desc, row asc). Returns (scores f32 [B,k], rows int64 [B,k])."""
    s = _f32(queries) @ _f32(corpus).T
    k_eff = min(k, s.shape[1])
    part = np.argpartition(-s, k_eff - 1, axis=1)[:, :k_eff]
    ps = np.take_along_axis(s, part, axis=1)
    idx = np.empty_like(part)
    for b in range(s.shape[0]):
        idx[b] = part[b][np.lexsort((part[b], -ps[b]))]
    return np.take_along_axis(s, idx, axis=1), idx.astype(np.int64)
