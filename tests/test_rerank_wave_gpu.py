"""GPU: the search() tail kernels (expansion + rerank, hierarchical_graph.py:726-782) against the
oracle restatement (oracle.search_ref.expand_rerank) on random graphs built to stress the dict
semantics: repeated seeds (a later seed overwrites an entry in place), seeds that are also
expansions of earlier seeds and the reverse, seeds unknown to the graph, missing hits, members
lists longer and shorter than member_top_m, equal rounded scores (stable order), every filter, and
top_k 0 .. beyond the entry count. Covers the wave-per-query kernel (k_seed <= 64) and the serial
kernel it replaced (k_seed > 64): both must give the oracle's dicts exactly.
"""
import json

import numpy as np
import pytest

from oracle import search_ref

pytestmark = pytest.mark.gpu
TYPES = ["entity", "summary", "hyperedge", None]


def random_graph(rng, n):
    import networkx as nx
    G = nx.DiGraph()
    kinds = rng.choice(4, size=n, p=[0.55, 0.3, 0.1, 0.05])
    for i in range(n):
        t = TYPES[kinds[i]]
        d = {"node_type": t, "name": f"n{i}"}
        r = rng.random()
        if r < 0.5:
            d["judge_scores"] = json.dumps({"overall": float(rng.integers(0, 100)) / 10.0})
        elif r < 0.6:
            d["judge_scores"] = "{broken"
        if rng.random() < 0.6:
            d["confidence"] = [3, 5.5, 7, 8.25, 9][int(rng.integers(0, 5))]
        G.add_node(f"x{i}", **d)
    ents = [i for i in range(n) if kinds[i] == 0]
    sums = [i for i in range(n) if kinds[i] == 1]
    for e in ents:  # 0-4 parents, random insertion order
        for s in rng.choice(sums, size=int(rng.integers(0, 5)), replace=False):
            G.add_edge(f"x{e}", f"x{int(s)}", edge_type="belongs_to")
    for s in sums[: len(sums) // 3]:  # summaries under summaries
        G.add_edge(f"x{s}", f"x{int(rng.choice(sums))}", edge_type="belongs_to")
    for _ in range(n // 4):
        a, b = rng.choice(sums, size=2)
        G.add_edge(f"x{int(a)}", f"x{int(b)}", edge_type="related_to")
    return G


@pytest.mark.parametrize("k_seed", [1, 5, 12, 40, 64, 80])
def test_rerank_kernels_match_oracle(cuda, k_seed):
    import torch

    from ah_rag.graph_search import DeviceGraph, RerankParams

    rng = np.random.default_rng(1000 + k_seed)
    n = 300
    G = random_graph(rng, n)
    dg = DeviceGraph(G, cuda)
    B = 48
    # seeds: graph nodes (with repeats), unknown ids (>= n), missing hits (-1); scores from a small
    # set of float32 values so rounded rerank scores tie often
    idx = rng.integers(0, n, size=(B, k_seed))
    idx[rng.random((B, k_seed)) < 0.15] = rng.integers(0, 20, size=1)  # repeats of a few nodes
    idx[rng.random((B, k_seed)) < 0.05] = n + 3
    idx[rng.random((B, k_seed)) < 0.05] = -1
    vals = np.float32(rng.choice([0.91, 0.8, 0.8000001, 0.55, 0.3333, 0.1], size=(B, k_seed)))
    vals = -np.sort(-vals, axis=1)  # rank order
    ids = [f"x{i}" for i in range(n)]
    for member_top_m in (0, 1, 3, 8):
        for top_k, filt in ((0, {}), (1, {}), (5, {"type_filter": ["summary"]}), (12, {"judge_min": 4.0}),
                            (500, {"confidence_min": 6.0}), (7, {"type_filter": ["entity", "summary"],
                                                                 "judge_min": 2.0})):
            p = RerankParams(alpha=0.6, beta=0.2, gamma=0.1, delta=0.1, judge_min=filt.get("judge_min"),
                             confidence_min=filt.get("confidence_min"),
                             layer_boost={"entity": 0.0, "summary": 1.0, "hyperedge": 0.0},
                             type_filter=filt.get("type_filter"), member_top_m=member_top_m, top_k=top_k)
            res = dg.expand_rerank(torch.from_numpy(idx.astype(np.int32)).to(cuda),
                                   torch.from_numpy(vals).to(cuda), p).to_host()
            op = {"alpha": 0.6, "beta": 0.2, "gamma": 0.1, "delta": 0.1, "judge_overall_min": filt.get("judge_min"),
                  "confidence_min": filt.get("confidence_min"), "member_top_m": member_top_m,
                  "type_filter": filt.get("type_filter"), "top_k": top_k,
                  "layer_boost": {"entity": 0.0, "summary": 1.0, "hyperedge": 0.0}}

            def name(i):
                return ids[i] if i < n else f"unknown{i}"
            for b in range(B):
                seeds = [{"node_id": name(int(i)), "semantic": 1.0 - float(np.float32(1.0) - v), "meta": {}}
                         for i, v in zip(idx[b], vals[b]) if i >= 0]
                want = search_ref.expand_rerank(G, seeds, op, return_cluster=True)
                e = int(res.exp_count[b])
                got_exp = [(name(int(i)), float(s)) for i, s in zip(res.exp_nodes[b, :e], res.exp_sem[b, :e])]
                assert got_exp == [(x["node_id"], x["semantic"]) for x in want["expanded"]], (k_seed, b, member_top_m)
                m = int(res.out_count[b]) if top_k > 0 else 0
                got = [(name(int(i)), float(s), float(c)) for i, s, c in
                       zip(res.out_nodes[b, :m], res.out_sem[b, :m], res.out_score[b, :m])]
                assert got == [(r["node_id"], r["semantic"], r["score"]) for r in want["reranked"]], \
                    (k_seed, b, member_top_m, top_k, filt)
    dg.close()
