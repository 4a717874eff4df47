"""§8f row 4 measurement: L1 topic relations at C2 scale (3,000 topics, 768-d centroids,
87,000 entities with 2 topic memberships each). GPU drop-in vs the reference's
pairwise Python loop (semantic_aggregator.py:620-661, restated per pair as in the reference),
the latter timed on a sample of rows and extrapolated to all T(T-1)/2 pairs.
Usage: python tools/bench_relations.py"""
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ah-rag_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ah_rag.aggregate import relations as rel  # noqa: E402


def main():
    rng = np.random.default_rng(20251003)
    T, d, E = 3000, 768, 87_000
    cen = rng.standard_normal((T, d)).astype(np.float32)
    topic = rng.integers(0, T, E)
    second = rng.integers(0, T, E)
    mem = [[] for _ in range(T)]
    for e in range(E):
        mem[topic[e]].append(f"e{e}")
        mem[second[e]].append(f"e{e}")
    nodes = [{"topic_id": t, "members": mem[t], "centroid": cen[t].tolist(), "confidence": 7.0} for t in range(T)]
    dev = torch.device("cuda", 0)
    tmp = tempfile.mkdtemp()
    rel.generate_l1_relations([dict(n) for n in nodes[:64]], artifact_dir=tmp, device=dev)  # warm-up
    t0 = time.perf_counter()
    edges = rel.generate_l1_relations(nodes, min_overlap=1, min_jaccard=0.05, min_cosine=0.3, artifact_dir=tmp,
                                      device=dev)
    t_gpu = time.perf_counter() - t0
    # reference-shaped loop on a row sample
    cs = {t: rel._norm(nodes[t]["centroid"]) for t in range(T)}
    ms = {t: set(nodes[t]["members"]) for t in range(T)}
    rows = 20
    t1 = time.perf_counter()
    n_pairs = 0
    for a in range(rows):
        for b in range(a + 1, T):
            A, B = ms[a], ms[b]
            inter = A & B
            union = A | B
            jac = len(inter) / len(union) if union else 0.0
            cos = float(np.dot(cs[a], cs[b]))
            _ = (len(inter) >= 1) or (jac >= 0.05) or (cos >= 0.3)
            n_pairs += 1
    per_pair = (time.perf_counter() - t1) / n_pairs
    total_pairs = T * (T - 1) // 2
    print(json.dumps({"metric": "L1 topic relations wall time (s), T=3000, d=768", "topics": T, "dim": d,
                      "edges": len(edges), "gpu_dropin_s": round(t_gpu, 3),
                      "reference_loop_s_extrapolated": round(per_pair * total_pairs, 1),
                      "reference_loop_sample_pairs": n_pairs, "speedup": round(per_pair * total_pairs / t_gpu, 1)}))


if __name__ == "__main__":
    main()
