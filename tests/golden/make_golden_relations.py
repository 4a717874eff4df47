#!/usr/bin/env python3
"""Golden fixture for the L1 topic relations, from the REFERENCE's own code.

Runs SemanticAggregator.generate_l1_relations (reference
src/ah_rag/aggregate/semantic_aggregator.py:594-680) unmodified on a seeded synthetic set of L1
topic nodes and records inputs and outputs as data in tests/golden/relations_cases.json.
The module imports sentence_transformers, bertopic, umap and hdbscan at load time (:1-11), all
absent here; the method uses none of them, so empty stand-in modules are injected.

Run: python tests/golden/make_golden_relations.py   (needs /root/reference; this container only)
"""
from __future__ import annotations

import copy
import json
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"


def stub_modules():
    for name, attrs in (("sentence_transformers", ("SentenceTransformer",)), ("bertopic", ("BERTopic",)),
                        ("umap", ("UMAP",)), ("hdbscan", ("HDBSCAN",))):
        m = types.ModuleType(name)
        for a in attrs:
            setattr(m, a, type(a, (), {}))
        sys.modules[name] = m


def make_nodes(seed: int = 20251016, T: int = 100, d: int = 48):
    rng = np.random.default_rng(seed)
    groups = rng.standard_normal((10, d)).astype(np.float32)
    pool = [f"entity_{i}" for i in range(600)]
    nodes = []
    for t in range(T):
        g = int(rng.integers(0, 10))
        cen = groups[g] + 0.6 * rng.standard_normal(d).astype(np.float32)
        lo = g * 60
        n_mem = int(rng.integers(5, 16))
        mem = [pool[lo + int(x)] for x in rng.integers(0, 60, n_mem)]
        mem += [pool[int(x)] for x in rng.integers(0, 600, int(rng.integers(0, 3)))]
        node = {"topic_id": int(1000 - 3 * t), "title": f"topic {t}", "members": mem,
                "centroid": [float(x) for x in cen], "confidence": float(np.round(rng.uniform(3, 10), 3))}
        if t % 37 == 5:
            node["centroid"] = None           # missing centroid: cosine 0
        if t % 41 == 7:
            node["members"] = []              # empty member set
        if t % 29 == 3:
            del node["confidence"]            # default confidence 5.0
        if t % 31 == 11:
            node["centroid"] = [0.0] * d      # zero vector: norm() leaves it, cosine 0
        nodes.append(node)
    return nodes


def main():
    stub_modules()
    sys.path.insert(0, REF_SRC)
    from ah_rag.aggregate.semantic_aggregator import SemanticAggregator  # reference code

    nodes = make_nodes()
    cases = []
    params_list = [dict(), dict(min_overlap=1, min_jaccard=0.05, min_cosine=0.3),
                   dict(top_k=40), dict(min_overlap=10, min_jaccard=0.9, min_cosine=0.95)]
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            for params in params_list:
                work = copy.deepcopy(nodes)
                edges = SemanticAggregator.generate_l1_relations(None, work, **params)
                with open(os.path.join("artifacts", "l1_edges.json"), encoding="utf-8") as f:
                    file_edges = json.load(f)
                assert file_edges == edges
                cases.append({"params": params, "edges": edges,
                              "neighbors": {str(n["topic_id"]): n["neighbors"] for n in work}})
        finally:
            os.chdir(cwd)
    out = {"source": "reference semantic_aggregator.py:594-680 via tests/golden/make_golden_relations.py",
           "l1_nodes": nodes, "cases": cases}
    with open(os.path.join(HERE, "relations_cases.json"), "w", encoding="utf-8") as f:
        json.dump(out, f)
    print({"cases": [len(c["edges"]) for c in cases]})


if __name__ == "__main__":
    main()
