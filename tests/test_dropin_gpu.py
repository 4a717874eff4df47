"""GPU parity of the drop-in HierarchicalGraph / GraphEnvironment / AHRAGGymEnv / NaiveRAG against
the reference's own outputs (tests/golden/, produced by tests/golden/make_golden.py).

Exact comparison: ids, order, node types, rounded semantic/score values, filters, env state,
observations, rewards and 84-d feature vectors must equal the reference's (timestamps and
wall-clock `time_s` excluded). The index runs in fp32 exact mode (bit-exact dense scores).
"""
import json
import os
import shutil

import numpy as np
import pytest

from oracle.search_ref import isclose_dicts

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with open(os.path.join(GOLDEN, name), encoding="utf-8") as f:
        return json.load(f)


def _norm(x):
    return json.loads(json.dumps(x, default=lambda o: o.tolist() if hasattr(o, "tolist") else str(o)))


@pytest.fixture(scope="module")
def workdir(tmp_path_factory, cuda):
    from ah_rag.graph.hierarchical_graph import HierarchicalGraph
    d = tmp_path_factory.mktemp("dropin")
    shutil.copytree(os.path.join(GOLDEN, "reference_graph"), d / "graph")
    # the settings hold for this module only (restored after it: no leak into later modules)
    with pytest.MonkeyPatch.context() as mp:
        mp.setenv("AHR_ENCODER", "hash")
        mp.setenv("AHR_INDEX_DTYPE", "f32")
        mp.chdir(d)
        hg = HierarchicalGraph.load("graph")
        # the fixture graph's meta already lists every entity/summary key (it was saved after the
        # reference built its index), so rebuild the collection without the upsert-only skip
        hg.build_vector_index(db_path="vector_db", layers={0, 1}, upsert_only=False, reset=True)
        yield d, hg


def test_hash_encoder_matches_fixture_encoder():
    import hashlib
    from ah_rag.embeddings import HashEncoder
    dg = _load("encoder_digest.json")
    v = HashEncoder("all-MiniLM-L6-v2").encode(dg["texts"], normalize_embeddings=True)
    assert hashlib.sha1(v.tobytes()).hexdigest() == dg["sha1"]


def test_search_matches_reference(workdir):
    d, hg = workdir
    from ah_rag.graph.hierarchical_graph import HierarchicalGraph
    hg2 = HierarchicalGraph.load("graph")
    hg2.build_vector_index(db_path="vector_db_h", layers={0, 1}, include_hyperedges=True, reset=True)
    n = 0
    for c in _load("search_cases.json")["cases"]:
        if c.get("include_hyperedges"):
            got = hg2.search(c["query"], return_cluster=True, db_path="vector_db_h", **c["params"])
        else:
            got = hg.search(c["query"], return_cluster=c["return_cluster"], **c["params"])
        assert isclose_dicts(_norm(got), c["result"]), (c["query"], c["params"])
        n += 1
    assert n > 80


def test_search_topk_beyond_count(workdir):
    """top_k above the index count (and above AHR_MAX_K_LARGE): Chroma returns every row, so does
    the drop-in (tests/golden/make_golden_bigk.py, the reference's own search over 313 rows)."""
    d, hg = workdir
    cases = _load("search_bigk_cases.json")["cases"]
    assert any(c["params"]["top_k"] > 4096 for c in cases)
    for c in cases:
        got = hg.search(c["query"], return_cluster=c["return_cluster"], **c["params"])
        assert isclose_dicts(_norm(got), c["result"]), (c["query"], c["params"])


def test_search_batch_equals_single(workdir):
    d, hg = workdir
    qs = [c["query"] for c in _load("search_cases.json")["cases"][:40:7]]
    batch = hg.search_batch(qs, top_k=7, return_cluster=True)
    for q, b in zip(qs, batch):
        assert isclose_dicts(_norm(b), _norm(hg.search(q, top_k=7, return_cluster=True)))


def test_environment_matches_reference(workdir):
    from ah_rag.agent.environment import GraphEnvironment
    import networkx as nx
    cases = _load("env_cases.json")["cases"]
    for case in cases:
        env = GraphEnvironment(graph_dir="graph", logging_enabled=False)
        for st in case["steps"]:
            call, args = st["call"], st["args"]
            if call == "semantic_anchor":
                env.set_filters(judge_overall_min=5.0, type_filter=["summary", "entity"])
                env.set_search_weights(alpha=0.7, delta=0.3, top_k=6)
            fn = getattr(env, call)
            if "error" in st:
                with pytest.raises(nx.NetworkXError):
                    fn(**args)
                continue
            obs, info = fn(**args)
            assert isclose_dicts(_norm(obs), st["obs"]), (case["query"], call, args)
            assert isclose_dicts({k: v for k, v in _norm(info).items() if k != "time_s"}, st["info"]), (call, args)
        cum = dict(env.stats["cumulative"])
        want = dict(case["stats_cumulative"])
        cum.pop("time_s"), want.pop("time_s", None)
        assert cum == want


def test_gym_matches_reference(workdir):
    from ah_rag.agent.gym_env import AHRAGGymEnv
    for ep in _load("gym_cases.json")["cases"]:
        genv = AHRAGGymEnv(graph_dir="graph", max_steps=6)
        vec, info = genv.reset(ep["query"])
        np.testing.assert_array_equal(vec, np.asarray(ep["reset"]["vec"], np.float32))
        assert isclose_dicts(_norm(info), ep["reset"]["info"])
        for st in ep["steps"]:
            v, r, done, inf = genv.step(st["action"])
            np.testing.assert_array_equal(v, np.asarray(st["vec"], np.float32))
            assert r == st["reward"] and done == st["done"]
            assert isclose_dicts(_norm(inf), st["info"])


def test_naive_rag_matches_reference(workdir):
    d, hg = workdir
    from baselines.naive_rag import NaiveRAG

    class EchoGen:
        def generate(self, query, context, cfg):
            return {"query": query, "context": context}
    naive = NaiveRAG(hg, EchoGen())
    for c in _load("naive_cases.json")["cases"]:
        assert _norm(naive.run(c["query"], top_k=c["top_k"])) == c["out"]


def test_incremental_reindex_matches_reference(workdir):
    """§8f row 2: build_vector_index(upsert_only=True) after editing 3 nodes and adding one writes
    only those 4 rows into the HBM-resident index (no reload of the store), with the reference's
    indexed_meta, and search() then returns the reference's results."""
    from ah_rag.graph.hierarchical_graph import HierarchicalGraph
    case = _load("upsert_cases.json")
    hg = HierarchicalGraph.load("graph")
    hg.build_vector_index(db_path="vector_db_up", layers={0, 1}, upsert_only=False, reset=True)
    assert hg.G.graph["vector_index"]["indexed_meta"] == case["indexed_meta_before"]
    for c in case["pre"]:  # first search makes the index resident (one full load)
        assert isclose_dicts(_norm(hg.search(c["query"], top_k=8, return_cluster=True, db_path="vector_db_up")),
                             c["result"])
    res = hg.resident_index("vector_db_up")
    index_obj, loads = res.index, res.full_loads
    for nid, key, val in case["edits"]:
        hg.G.nodes[nid][key] = val
    ne = case["new_entity"]
    assert hg.add_entity(name=ne["name"], description="added after the first index build",
                         entity_type="person") == ne["id"]
    hg.add_belongs_to(ne["id"], ne["summary"], prob=0.5)
    hg.build_vector_index(db_path="vector_db_up", layers={0, 1}, upsert_only=True)
    vi = hg.G.graph["vector_index"]
    assert vi["indexed_meta"] == case["indexed_meta_after"]
    assert vi["indexed_nodes"] == case["vector_index"]["indexed_nodes"]
    for c in case["post"]:
        got = hg.search(c["query"], top_k=8, return_cluster=True, db_path="vector_db_up")
        assert isclose_dicts(_norm(got), c["result"]), c["query"]
    res = hg.resident_index("vector_db_up")
    assert res.index is index_obj and res.full_loads == loads  # no reload, no reallocation
    assert res.rows_upserted == len(case["changed"]) == 4
    # the persisted store holds the same rows (a fresh process reloads them)
    hg2 = HierarchicalGraph.load("graph")
    hg2.G.graph["vector_index"] = dict(vi)
    for nid, key, val in case["edits"]:
        hg2.G.nodes[nid][key] = val
    hg2.add_entity(name=ne["name"], description="added after the first index build", entity_type="person")
    hg2.add_belongs_to(ne["id"], ne["summary"], prob=0.5)
    c = case["post"][0]
    assert isclose_dicts(_norm(hg2.search(c["query"], top_k=8, return_cluster=True, db_path="vector_db_up")),
                         c["result"])


def test_concurrent_search_threads(workdir):
    """Two threads calling search() / search_batch() on one graph at once (the GIL is released
    during the native calls): the engine's reused staging and result buffers are taken in turns, so
    every answer equals the serial one (no silent cross-talk)."""
    import threading
    d, hg = workdir
    cases = [c for c in _load("search_cases.json")["cases"] if not c.get("include_hyperedges")][:24]
    want = [_norm(hg.search(c["query"], return_cluster=c["return_cluster"], **c["params"])) for c in cases]
    errors = []

    def worker(off):
        try:
            for rep in range(6):
                for i in range(off, len(cases), 2):
                    c = cases[i]
                    if rep % 2:
                        got = hg.search_batch([c["query"], c["query"]], return_cluster=c["return_cluster"],
                                              **c["params"])[1]
                    else:
                        got = hg.search(c["query"], return_cluster=c["return_cluster"], **c["params"])
                    if _norm(got) != want[i]:
                        errors.append((off, rep, i))
        except Exception as e:  # noqa: BLE001 — reported below
            errors.append(repr(e))
    ts = [threading.Thread(target=worker, args=(o,)) for o in (0, 1)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors[:5]


def test_search_results_survive_later_calls(workdir):
    """search_batch() builds its dicts from views of the engine's reused result buffer (no copy):
    what a call returned must not change when later calls overwrite that buffer, and the arrays
    search_arrays() returns are the caller's own."""
    import copy
    d, hg = workdir
    cases = [c for c in _load("search_cases.json")["cases"] if not c.get("include_hyperedges")][:6]
    first = hg.search(cases[0]["query"], return_cluster=True, **cases[0]["params"])
    kept = copy.deepcopy(first)
    _, _, rows, scores, res = hg.search_arrays([cases[0]["query"]], **cases[0]["params"])
    kept_arrays = [a.copy() for a in (rows, scores, res.out_nodes, res.out_score, res.exp_nodes)]
    for c in cases[1:]:
        hg.search(c["query"], return_cluster=c["return_cluster"], **c["params"])
        hg.search_batch([c["query"]], return_cluster=True, **c["params"])
    assert _norm(first) == _norm(kept)
    for a, b in zip((rows, scores, res.out_nodes, res.out_score, res.exp_nodes), kept_arrays):
        assert np.array_equal(a, b)
