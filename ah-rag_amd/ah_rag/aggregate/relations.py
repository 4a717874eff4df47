"""L1 topic relations: drop-in for
SemanticAggregator.generate_l1_relations (reference src/ah_rag/aggregate/semantic_aggregator.py:594-680).

The reference walks all T·(T−1)/2 topic pairs in Python (:620-661): member overlap and Jaccard of
the two member sets, cosine of the L2-normalised float32 centroids (np.dot, :638), an OR of three
thresholds (:640-646), weight 0.5·jaccard + 0.5·cosine (:649), rounded fields (:652-660), optional
top-k by weight (:664-665), then artifacts/l1_edges.json, a `neighbors` list on every node and
artifacts/l1_nodes.json (:667-680).

Here the O(T²·d) part is one pass of this library's fp32 tile kernel (ahr_index_scores: the
centroid cosine matrix),
member overlaps are one sparse product of the topic × member incidence matrix, and only the pairs
that pass a rule reach the host loop, which keeps the reference's arithmetic (Python floats,
round()) and pair order (sorted topic ids, row-major upper triangle).
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

ARTIFACT_DIR = "artifacts"


def _norm(v) -> Optional[np.ndarray]:
    """reference :608-613: float32, divided by its norm unless the norm is 0."""
    if v is None:
        return None
    arr = np.asarray(v, dtype=np.float32)
    n = np.linalg.norm(arr)
    return arr / n if n > 0 else arr


def _prepare(l1_nodes: Sequence[Dict[str, Any]]):
    centroids = {int(n["topic_id"]): _norm(n.get("centroid")) for n in l1_nodes}
    members = {int(n["topic_id"]): set(n.get("members", [])) for n in l1_nodes}
    confidences = {int(n["topic_id"]): float(n.get("confidence", 5.0)) for n in l1_nodes}
    return centroids, members, confidences, sorted(centroids.keys())


def overlap_matrix(topic_ids: Sequence[int], members: Dict[int, set]) -> np.ndarray:
    """|A ∩ B| for every topic pair: M·Mᵀ of the sparse topic × member incidence matrix."""
    from scipy import sparse

    T = len(topic_ids)
    codes: Dict[Any, int] = {}
    rows, cols = [], []
    for i, t in enumerate(topic_ids):
        for m in members.get(t, ()):
            rows.append(i)
            cols.append(codes.setdefault(m, len(codes)))
    M = sparse.csr_matrix((np.ones(len(rows), np.int64), (rows, cols)), shape=(T, max(1, len(codes))))
    ov = (M @ M.T).toarray()
    np.fill_diagonal(ov, 0)
    return ov


def cosine_matrix_gpu(topic_ids: Sequence[int], centroids: Dict[int, Optional[np.ndarray]],
                      device: Optional[torch.device] = None) -> np.ndarray:
    """float32 cosine of every centroid pair in one device pass: the centroids become an fp32
    DenseIndex and ahr_index_scores runs the fused tile kernel's GEMM core over them (every score
    a k-ordered fma chain). Missing centroids give 0 (reference :636-638). Raises without a GPU
    (no CPU fallback in the product path)."""
    if not torch.cuda.is_available():
        raise RuntimeError("generate_l1_relations needs a GPU (HIP device) for the centroid GEMM")
    dev = device or torch.device("cuda", torch.cuda.current_device())
    dims = {c.shape[0] for c in centroids.values() if c is not None}
    if len(dims) > 1:
        raise ValueError("centroids of different dimensions")
    d = dims.pop() if dims else 1
    X = np.zeros((len(topic_ids), d), np.float32)
    for i, t in enumerate(topic_ids):
        c = centroids.get(t)
        if c is not None:
            X[i] = c
    from ..embeddings import DenseIndex
    ix = DenseIndex(d, max(1, len(topic_ids)), dtype="f32", device=dev)
    try:
        ix.upsert(X)
        return ix.scores(X).cpu().numpy()  # fp32 tile kernel, scores mode (ahr_index_scores)
    finally:
        ix.close()


def edges_from_matrices(topic_ids: Sequence[int], members: Dict[int, set], confidences: Dict[int, float],
                        cos: np.ndarray, ov: np.ndarray, min_overlap: int, min_jaccard: float,
                        min_cosine: float) -> List[Dict[str, Any]]:
    """The reference's rule, weight and rounding (:620-661) on precomputed matrices, pairs in its
    order. Only pairs that can pass a rule are visited."""
    T = len(topic_ids)
    sizes = np.asarray([len(members.get(t, ())) for t in topic_ids], np.int64)
    iu, ju = np.triu_indices(T, 1)
    union = sizes[iu] + sizes[ju] - ov[iu, ju]
    with np.errstate(divide="ignore", invalid="ignore"):
        jac = np.where(union > 0, ov[iu, ju] / np.maximum(union, 1), 0.0)
    # screen (conservative on the float comparisons; the exact test is redone below)
    cand = (ov[iu, ju] >= min_overlap) | (jac >= min_jaccard - 1e-12) | (cos[iu, ju] >= min_cosine - 1e-6)
    cand &= (sizes[iu] > 0) | (sizes[ju] > 0)  # both member sets empty: skipped (:626-627)
    edges: List[Dict[str, Any]] = []
    for i, j in zip(iu[cand].tolist(), ju[cand].tolist()):
        a, b = topic_ids[i], topic_ids[j]
        A, B = members.get(a, set()), members.get(b, set())
        overlap = int(ov[i, j])
        un = len(A) + len(B) - overlap
        jaccard = (overlap / un) if un else 0.0
        cosine = float(cos[i, j])
        if not ((overlap >= min_overlap) or (jaccard >= min_jaccard) or (cosine >= min_cosine)):
            continue
        weight = 0.5 * jaccard + 0.5 * cosine
        conf = (confidences.get(a, 5.0) + confidences.get(b, 5.0)) / 2.0
        edges.append({"source": int(a), "target": int(b), "relation_type": "related_summary",
                      "weight": round(weight, 4), "overlap": overlap, "jaccard": round(jaccard, 4),
                      "cosine": round(cosine, 4), "confidence": round(conf, 2)})
    return edges


def finish(l1_nodes: List[Dict[str, Any]], edges: List[Dict[str, Any]], top_k: Optional[int],
           artifact_dir: str) -> List[Dict[str, Any]]:
    """top-k pruning, artifacts and node neighbour lists (reference :663-680)."""
    if top_k is not None and len(edges) > top_k:
        edges = sorted(edges, key=lambda e: e["weight"], reverse=True)[:top_k]
    os.makedirs(artifact_dir, exist_ok=True)
    with open(os.path.join(artifact_dir, "l1_edges.json"), "w", encoding="utf-8") as f:
        json.dump(edges, f, ensure_ascii=False, indent=2)
    adj: Dict[int, list] = {int(n["topic_id"]): [] for n in l1_nodes}
    for e in edges:
        adj[e["source"]].append((e["target"], e["weight"]))
        adj[e["target"]].append((e["source"], e["weight"]))
    for n in l1_nodes:
        tid = int(n["topic_id"])
        n["neighbors"] = [{"topic_id": t, "weight": w}
                          for t, w in sorted(adj.get(tid, []), key=lambda x: x[1], reverse=True)]
    with open(os.path.join(artifact_dir, "l1_nodes.json"), "w", encoding="utf-8") as f:
        json.dump(l1_nodes, f, ensure_ascii=False, indent=2)
    return edges


def generate_l1_relations(l1_nodes: List[Dict[str, Any]], min_overlap: int = 3, min_jaccard: float = 0.2,
                          min_cosine: float = 0.5, top_k: Optional[int] = None,
                          artifact_dir: str = ARTIFACT_DIR,
                          device: Optional[torch.device] = None) -> List[Dict[str, Any]]:
    """Same arguments, return value, artifacts and node mutation as the reference method."""
    if not l1_nodes:
        return []
    centroids, members, confidences, topic_ids = _prepare(l1_nodes)
    cos = cosine_matrix_gpu(topic_ids, centroids, device)
    ov = overlap_matrix(topic_ids, members)
    edges = edges_from_matrices(topic_ids, members, confidences, cos, ov, min_overlap, min_jaccard, min_cosine)
    return finish(l1_nodes, edges, top_k, artifact_dir)
