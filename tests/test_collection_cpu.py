"""CPU: the Chroma seam (ah_rag.collection) — its host bookkeeping, and the recorded collection
traffic of the reference (tests/golden/collection_cases.json, make_golden.py) pinned against the
oracle, so the GPU test that replays it through the device index has a checked anchor.

Reference call sites: /root/reference/src/ah_rag/graph/hierarchical_graph.py:605-611 (client,
delete / get_or_create), :660 (upsert), :714-724 (query, and the seeds the reference builds from
its answer).
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import dense_ref, encoder_stub, search_ref

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with open(os.path.join(GOLDEN, name), encoding="utf-8") as f:
        return json.load(f)


class HostCollection:
    """Chroma's upsert semantics restated on the host (update in place, append new ids)."""

    def __init__(self):
        self.ids, self.vecs, self.metas, self.docs = [], [], [], []

    def upsert(self, ids, vecs, metas, docs):
        for nid, v, m, d in zip(ids, vecs, metas, docs):
            if nid in self.ids:
                j = self.ids.index(nid)
                self.vecs[j], self.metas[j], self.docs[j] = v, m, d
            else:
                self.ids.append(nid)
                self.vecs.append(v)
                self.metas.append(m)
                self.docs.append(d)

    def query(self, q, n):
        C = np.stack(self.vecs)
        k = min(n, len(self.ids))
        s, r = dense_ref.topk(C, q, k, mode="fma")
        return {"ids": [[self.ids[j] for j in row] for row in r],
                "distances": [[float(np.float32(1.0) - np.float32(x)) for x in row] for row in s],
                "metadatas": [[self.metas[j] for j in row] for row in r],
                "documents": [[self.docs[j] for j in row] for row in r]}


def replay(calls, make):
    """Feed the recorded calls to collections made by make(); yield (call, answer) per query."""
    colls = {}
    for c in calls:
        if c["op"] == "delete":
            colls.pop(c["coll"], None)
        elif c["op"] == "create":
            colls[c["coll"]] = make(c)
        elif c["op"] == "upsert":
            vecs = encoder_stub.encode(c["documents"], c["dim"], normalize=True)
            colls[c["coll"]].upsert(c["ids"], vecs, c["metadatas"], c["documents"])
        elif c["op"] == "query":
            q = encoder_stub.encode(c["texts"], 384, normalize=True)
            yield c, colls[c["coll"]].query(q, c["n_results"])


def test_collection_fixture_vs_oracle():
    """Every raw answer the reference received equals Chroma's semantics restated over the oracle's
    fp32 fma-chain scores (ranking score desc / insertion order asc, float32 distances)."""
    calls = _load("collection_cases.json")["calls"]
    n = 0
    for c, got in replay(calls, lambda c: HostCollection()):
        exp = c["result"]
        assert got["ids"] == exp["ids"], c["texts"]
        assert got["distances"] == exp["distances"], c["texts"]
        assert got["metadatas"] == exp["metadatas"]
        assert got["documents"] == exp["documents"]
        n += 1
    assert n >= 140
    # the incremental re-index is in the log: a second upsert of existing ids on one collection
    ups = [c for c in calls if c["op"] == "upsert" and c["coll"] == "vector_db_up/nodes"]
    assert len(ups) == 2 and len(ups[1]["ids"]) == 4
    assert len(set(ups[1]["ids"]) & set(ups[0]["ids"])) == 3  # 3 edited nodes updated in place, 1 new


def seeds_from_answer(res):
    """hierarchical_graph.py:715-724: the reference's seeds from a collection answer."""
    ids = res.get("ids", [[]])[0]
    distances = res.get("distances", [[]])[0]
    metas = res.get("metadatas", [[]])[0]
    seeds = []
    for nid, dist, meta in zip(ids, distances, metas):
        if nid is None:
            continue
        seeds.append({"node_id": nid, "semantic": 1.0 - float(dist) if dist is not None else 0.0, "meta": meta})
    return seeds


def search_pairs(calls):
    """The vector_db / vector_db_h queries of the log in the order search_cases.json records the
    reference's search() calls that made them."""
    cases = _load("search_cases.json")["cases"]
    plain = [c for c in cases if not c.get("include_hyperedges")]
    hyper = [c for c in cases if c.get("include_hyperedges")]
    q_plain = [c for c in calls if c["op"] == "query" and c["coll"] == "vector_db/nodes"]
    q_hyper = [c for c in calls if c["op"] == "query" and c["coll"] == "vector_db_h/nodes"]
    assert len(q_plain) == len(plain) and len(q_hyper) == len(hyper)
    return list(zip(q_plain, plain)) + list(zip(q_hyper, hyper))


def test_raw_answers_reproduce_search_cases():
    """The reference's search() = its seeds from the raw answer + the expansion / rerank tail
    (oracle.search_ref.expand_rerank): the recorded raw answers give back search_cases.json."""
    G, meta = search_ref.load_graph(os.path.join(GOLDEN, "reference_graph"))
    calls = _load("collection_cases.json")["calls"]
    for raw, case in search_pairs(calls):
        assert raw["texts"] == [case["query"]]
        p = search_ref.resolve_params(meta.get("search_params", {}), **case["params"])
        assert raw["n_results"] == p["top_k"]
        got = search_ref.expand_rerank(G, seeds_from_answer(raw["result"]), p, case["return_cluster"])
        assert search_ref.isclose_dicts(json.loads(json.dumps(got)), case["result"]), (case["query"], case["params"])


def test_collection_host_bookkeeping(tmp_path):
    from ah_rag import _native as nat
    from ah_rag import collection as chroma

    chroma._REGISTRY.clear()
    client = chroma.PersistentClient(path=str(tmp_path / "db"), settings=chroma.Settings(allow_reset=True))
    with pytest.raises(chroma.NotFoundError):
        client.delete_collection(name="nodes")  # the reference swallows this (:607-610)
    coll = client.get_or_create_collection(name="nodes", metadata={"hnsw:space": "cosine"})
    v = encoder_stub.encode(["a", "b", "c"], 8)
    coll.upsert(ids=["a", "b", "c"], documents=["A", "B", "C"], embeddings=[x.tolist() for x in v],
                metadatas=[{"i": 0}, {"i": 1}, {"i": 2}])
    w = encoder_stub.encode(["b2", "d"], 8)
    coll.upsert(ids=["b", "d"], documents=["B2", "D"], embeddings=[x.tolist() for x in w],
                metadatas=[{"i": 10}, {"i": 3}])
    assert coll.count() == 4
    got = coll.get(include=["metadatas", "documents", "embeddings"])
    assert got["ids"] == ["a", "b", "c", "d"]  # in place, then appended
    assert got["documents"] == ["A", "B2", "C", "D"]
    assert got["metadatas"][1] == {"i": 10}
    assert np.array_equal(got["embeddings"][1], w[0])
    # search() opens a new client and gets the collection without metadata: the same one
    again = chroma.PersistentClient(path=str(tmp_path / "db")).get_or_create_collection(name="nodes")
    assert again is coll and again.metadata == {"hnsw:space": "cosine"}
    # persisted: a fresh process (registry cleared) reads it back
    chroma._REGISTRY.clear()
    back = chroma.PersistentClient(path=str(tmp_path / "db")).get_collection("nodes")
    assert back.ids == ["a", "b", "c", "d"] and back.metadata == {"hnsw:space": "cosine"}
    assert np.array_equal(back.get(ids=["d"], include=["embeddings"])["embeddings"][0], w[1])
    back.delete(["a"])
    assert back.get()["ids"] == ["b", "c", "d"]
    assert chroma.PersistentClient(path=str(tmp_path / "db")).list_collections() == ["nodes"]
    with pytest.raises(ValueError):
        chroma.PersistentClient(path=str(tmp_path / "db")).reset()  # allow_reset not set
    if not torch.cuda.is_available():  # no CPU fallback: the query needs the device index
        with pytest.raises(nat.NativeLibraryError):
            back.query(query_embeddings=[w[0].tolist()], n_results=2)
    client.delete_collection(name="nodes")
    assert client.list_collections() == []
    with pytest.raises(chroma.NotFoundError):
        client.get_collection("nodes")
    with pytest.raises(ValueError):
        client.get_or_create_collection(name="x", metadata={"hnsw:space": "manhattan"})
    chroma._REGISTRY.clear()
