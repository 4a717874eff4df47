"""TEST INFRASTRUCTURE (oracle) — CPU restatement of the centroid cosine in
SemanticAggregator.generate_l1_relations (reference src/ah_rag/aggregate/semantic_aggregator.py:
608-613 norm(), :636-638 cosine = float(np.dot(ca, cb)) on float32 vectors, 0.0 when a centroid
is missing). Used only by tests/ as the checker of ah_rag.aggregate.relations; never shipped.
Pinned by tests/golden/relations_cases.json (the reference's own outputs).
"""
from __future__ import annotations

import numpy as np


def norm(v):
    if v is None:
        return None
    arr = np.asarray(v, dtype=np.float32)
    n = np.linalg.norm(arr)
    return arr / n if n > 0 else arr


def cosine_matrix(l1_nodes):
    """(sorted topic ids, float32 [T, T] cosine matrix) with the reference's per-pair np.dot."""
    cen = {int(n["topic_id"]): norm(n.get("centroid")) for n in l1_nodes}
    ids = sorted(cen)
    T = len(ids)
    out = np.zeros((T, T), np.float32)
    for i, a in enumerate(ids):
        for j in range(i + 1, T):
            ca, cb = cen[a], cen[ids[j]]
            out[i, j] = out[j, i] = float(np.dot(ca, cb)) if (ca is not None and cb is not None) else 0.0
    return ids, out
