"""Deterministic stand-in encoder shared by the golden-fixture generator and the tests
(test infrastructure; the product's ah_rag.embeddings.HashEncoder must reproduce it bit for bit).
sha1(text)[:8] little-endian seeds numpy.default_rng; standard normal fp32; L2-normalised in fp32.
"""
from __future__ import annotations

import hashlib
from typing import Sequence, Union

import numpy as np


def hash_vec(text: str, dim: int) -> np.ndarray:
    seed = int.from_bytes(hashlib.sha1(text.encode("utf-8")).digest()[:8], "little")
    return np.random.default_rng(seed).standard_normal(dim).astype(np.float32)


def encode(texts: Union[str, Sequence[str]], dim: int, normalize: bool = True) -> np.ndarray:
    single = isinstance(texts, str)
    items = [texts] if single else list(texts)
    out = np.stack([hash_vec(t, dim) for t in items])
    if normalize:
        out = out / np.maximum(np.linalg.norm(out, axis=1, keepdims=True), 1e-12)
    out = out.astype(np.float32)
    return out[0] if single else out
