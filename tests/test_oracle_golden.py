"""CPU: pin the oracle restatements against the reference's own outputs (tests/golden/).

If these pass, oracle/ reproduces what the reference computed, so the GPU parity tests that
compare libahr_hip.so with oracle/ inherit the reference as their anchor.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import dense_ref, encoder_stub, search_ref

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with open(os.path.join(GOLDEN, name), encoding="utf-8") as f:
        return json.load(f)


@pytest.fixture(scope="module")
def graph():
    G, meta = search_ref.load_graph(os.path.join(GOLDEN, "reference_graph"))
    return G, meta


def _index(G, include_hyperedges=False, dim=384, indexed_meta=None):
    ids = search_ref.indexed_nodes(G, include_hyperedges=include_hyperedges, indexed_meta=indexed_meta)
    texts, metas = zip(*[search_ref.embedding_text(G, n) for n in ids])
    vecs = encoder_stub.encode(list(texts), dim)
    return ids, vecs, list(metas)


def _oracle_search(G, meta, index, query, params, return_cluster):
    ids, vecs, metas = index
    p = search_ref.resolve_params(meta.get("search_params", {}), **params)
    q = encoder_stub.encode([query], 384)
    k = p["top_k"]
    scores, rows = dense_ref.topk(vecs, q, min(k, len(ids)), mode="fma")
    seeds = []
    for s, r in zip(scores[0], rows[0]):
        dist = float(np.float32(1.0) - np.float32(s))  # Chroma: fp32 distance
        m = dict(metas[r])
        m["updated_at"] = "<ts>"
        seeds.append({"node_id": ids[r], "semantic": 1.0 - float(dist), "meta": m})
    return search_ref.expand_rerank(G, seeds, p, return_cluster)


def test_encoder_stub_digest():
    d = _load("encoder_digest.json")
    v = encoder_stub.encode(d["texts"], d["dim"])
    assert hashlib.sha1(v.tobytes()).hexdigest() == d["sha1"]


def test_search_cases(graph):
    G, meta = graph
    cases = _load("search_cases.json")["cases"]
    idx = _index(G)
    # the second collection was built from the saved graph, whose indexed_meta already holds every
    # entity/summary key: upsert_only leaves only the hyperedges to index (reference semantics)
    idx_h = _index(G, include_hyperedges=True, indexed_meta=meta["vector_index"]["indexed_meta"])
    assert len(cases) > 50
    for c in cases:
        ix = idx_h if c.get("include_hyperedges") else idx
        got = _oracle_search(G, meta, ix, c["query"], c["params"], c["return_cluster"])
        assert search_ref.isclose_dicts(json.loads(json.dumps(got)), c["result"]), (c["query"], c["params"])


def test_search_seeds_vs_numpy_f64(graph):
    """The fixtures' dense step (R3) against an independent exhaustive scorer: numpy float64 matrix
    products over the same stub-encoded vectors, not the C oracle the stand-in collection scored
    with when the fixtures were made (tests/golden/make_golden.py), so the golden search results
    are not anchored on the oracle alone. Every dense hit the reference recorded (result["seeds"],
    return_cluster cases) must carry its f64 score within 1e-6 and lie in the f64 top-k (near-ties
    within 1e-6 may trade places); unfiltered cases must return exactly the f64 top-k."""
    G, meta = graph
    cases = [c for c in _load("search_cases.json")["cases"] if c["return_cluster"]]
    idx = _index(G)
    idx_h = _index(G, include_hyperedges=True, indexed_meta=meta["vector_index"]["indexed_meta"])
    filters = {"type_filter", "judge_overall_min", "confidence_min"}
    n_checked = 0
    for c in cases:
        ids, vecs, _ = idx_h if c.get("include_hyperedges") else idx
        if not ids:
            continue
        q = encoder_stub.encode([c["query"]], 384)[0].astype(np.float64)
        s64 = vecs.astype(np.float64) @ q
        p = search_ref.resolve_params(meta.get("search_params", {}), **c["params"])
        k = min(p["top_k"], len(ids))
        order = sorted(range(len(ids)), key=lambda i: (-s64[i], i))[:k]
        kth = s64[order[-1]]
        pos = {n: i for i, n in enumerate(ids)}
        seeds = c["result"]["seeds"]
        prev = np.inf
        for sd in seeds:
            r = pos[sd["node_id"]]
            assert abs(sd["semantic"] - s64[r]) < 1e-6, (c["query"], sd["node_id"], sd["semantic"], s64[r])
            assert s64[r] >= kth - 1e-6, (c["query"], sd["node_id"])
            assert sd["semantic"] <= prev + 1e-6
            prev = sd["semantic"]
        if not (filters & set(c["params"])):
            assert len(seeds) == k
            got = sorted(pos[sd["node_id"]] for sd in seeds)
            for r in set(got) ^ set(order):  # a row on one side only: a near-tie at the k-th score
                assert abs(s64[r] - kth) < 1e-6, (c["query"], ids[r])
        n_checked += 1
    assert n_checked > 30


def test_env_expansions(graph):
    G, _ = graph
    n = 0
    for case in _load("env_cases.json")["cases"]:
        for st in case["steps"]:
            call = st["call"]
            if call in ("expand_parents", "expand_children", "expand_related") and "obs" in st:
                action = call.split("_")[1]
                got = search_ref.env_expand(G, action, st["args"]["node_ids"], st["args"].get("limit", 10))
                want = [x["node_id"] for x in st["obs"]["selection"]]
                assert got == want, (call, st["args"])
                n += 1
            elif call == "expand_to_lca":
                if "error" in st:
                    with pytest.raises(Exception):
                        search_ref.env_lca(G, st["args"]["node_ids"], st["args"].get("max_results", 5))
                else:
                    lcas, is_dag = search_ref.env_lca(G, st["args"]["node_ids"], st["args"].get("max_results", 5))
                    assert lcas == [x["node_id"] for x in st["obs"]["selection"]]
                    assert is_dag == st["info"]["dag"]
                n += 1
    assert n > 60


def test_node_briefs(graph):
    G, _ = graph
    for case in _load("env_cases.json")["cases"]:
        for st in case["steps"]:
            for b in (st.get("obs") or {}).get("seeds", []):
                want = {k: b[k] for k in ("node_id", "node_type", "entity_type", "layer", "title", "name",
                                          "judge_overall", "confidence")}
                assert search_ref.node_brief(G, b["node_id"]) == want


def test_featurizer_and_reward():
    for ep in _load("gym_cases.json")["cases"]:
        prev = ep["reset"]["info"]["raw_obs"]
        np.testing.assert_array_equal(search_ref.featurize(prev), np.asarray(ep["reset"]["vec"], np.float32))
        last = None
        for st in ep["steps"]:
            raw = st["info"]["raw_obs"]
            np.testing.assert_array_equal(search_ref.featurize(raw), np.asarray(st["vec"], np.float32))
            if not (st["action"] == 5):
                r = search_ref.step_reward(prev, raw)
                if last is not None and st["action"] == last:
                    r -= 0.02
                assert r == st["reward"]
            last = st["action"]
            prev = raw
