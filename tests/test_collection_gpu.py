"""GPU parity of the Chroma seam (ah_rag.collection over libahr_hip.so) against the raw collection
traffic of the reference (tests/golden/collection_cases.json): the same upserts, then every query
the reference's build_vector_index / search() made must come back as the identical dict — ids,
float32 distances, metadatas, documents — and the reference's own search tail over those answers
(oracle.search_ref.expand_rerank) must give search_cases.json. fp32 storage (the default).
"""
import json
import os

import numpy as np
import pytest

from oracle import encoder_stub, search_ref
from test_collection_cpu import GOLDEN, _load, replay, search_pairs, seeds_from_answer

pytestmark = pytest.mark.gpu
KEYS = ("ids", "distances", "metadatas", "documents")


class Adapter:
    """The seam driven the way the reference drives chromadb (hierarchical_graph.py:605-611, 660, 714)."""

    def __init__(self, root, coll):
        from ah_rag import collection as chroma
        path, name = coll.split("/")
        self.client = chroma.PersistentClient(path=os.path.join(root, path), settings=chroma.Settings(allow_reset=True))
        try:
            self.client.delete_collection(name=name)
        except Exception:
            pass
        self.coll = self.client.get_or_create_collection(name=name, metadata={"hnsw:space": "cosine"})

    def upsert(self, ids, vecs, metas, docs):
        self.coll.upsert(ids=ids, documents=docs, embeddings=[e.tolist() for e in vecs], metadatas=metas)

    def query(self, q, n):
        return self.coll.query(query_embeddings=[x.tolist() for x in q], n_results=n,
                               include=["distances", "metadatas", "documents"])


def test_collection_replays_reference_traffic(tmp_path, cuda):
    from ah_rag import collection as chroma
    chroma._REGISTRY.clear()
    calls = _load("collection_cases.json")["calls"]
    answers = []
    for c, got in replay(calls, lambda c: Adapter(str(tmp_path), c["coll"])):
        for key in KEYS:
            assert got[key] == c["result"][key], (c["coll"], c["texts"], key)
        answers.append((c, got))
    assert len(answers) >= 140
    # the incremental collection holds each id once after the upsert-only re-index
    up = chroma.PersistentClient(path=str(tmp_path / "vector_db_up")).get_collection("nodes")
    assert len(set(up.ids)) == len(up.ids) == up.count()
    chroma._REGISTRY.clear()


def test_collection_answers_drive_reference_search(tmp_path, cuda):
    """The reference's search() on top of the seam: seeds from the adapter's answer (:715-724),
    expansion + rerank (:726-789, oracle restatement) == the reference's recorded search()."""
    from ah_rag import collection as chroma
    chroma._REGISTRY.clear()
    calls = _load("collection_cases.json")["calls"]
    G, meta = search_ref.load_graph(os.path.join(GOLDEN, "reference_graph"))
    got_by_id = {}
    for c, got in replay(calls, lambda c: Adapter(str(tmp_path), c["coll"])):
        got_by_id[id(c)] = got
    n = 0
    for raw, case in search_pairs(calls):
        p = search_ref.resolve_params(meta.get("search_params", {}), **case["params"])
        res = search_ref.expand_rerank(G, seeds_from_answer(got_by_id[id(raw)]), p, case["return_cluster"])
        assert search_ref.isclose_dicts(json.loads(json.dumps(res)), case["result"]), (case["query"], case["params"])
        n += 1
    assert n >= 130
    chroma._REGISTRY.clear()


def test_collection_batch_query_and_spaces(tmp_path, cuda):
    """A batch of query embeddings in one call (one device pass) equals the per-query answers; the
    ip space gives cosine's distances, l2 the float32 squared distance; n_results above the count
    returns every row; an empty collection answers empty lists."""
    from ah_rag import collection as chroma
    chroma._REGISTRY.clear()
    client = chroma.PersistentClient(path=str(tmp_path / "db"))
    texts = [f"row {i}" for i in range(300)]
    v = encoder_stub.encode(texts, 64)
    qs = encoder_stub.encode(["q0", "q1", "q2", "q3"], 64)
    for space in ("cosine", "ip", "l2"):
        coll = client.get_or_create_collection(name=space, metadata={"hnsw:space": space})
        assert coll.query(query_embeddings=[qs[0].tolist()], n_results=3)["ids"] == [[]]
        coll.upsert(ids=texts, embeddings=[x.tolist() for x in v], documents=texts)
        batch = coll.query(query_embeddings=[x.tolist() for x in qs], n_results=7)
        for b in range(len(qs)):
            one = coll.query(query_embeddings=[qs[b].tolist()], n_results=7)
            assert one["ids"][0] == batch["ids"][b] and one["distances"][0] == batch["distances"][b]
        s = v.astype(np.float64) @ qs[0].astype(np.float64)
        top = [texts[i] for i in sorted(range(len(texts)), key=lambda i: (-s[i], i))[:7]]
        assert batch["ids"][0] == top
        d0 = np.asarray(batch["distances"][0])
        if space == "l2":
            exp = np.array([np.sum((qs[0].astype(np.float64) - v[texts.index(t)]) ** 2) for t in top])
        else:
            exp = 1.0 - s[[texts.index(t) for t in top]]
        assert np.abs(d0 - exp).max() < 1e-5, space
        assert len(coll.query(query_embeddings=[qs[0].tolist()], n_results=1000)["ids"][0]) == len(texts)
    # an upsert after a query reaches the device copy (slot write, no duplicate)
    coll = client.get_collection("cosine")
    coll.upsert(ids=["row 5"], embeddings=[qs[0].tolist()], documents=["moved"])
    res = coll.query(query_embeddings=[qs[0].tolist()], n_results=2)
    assert res["ids"][0][0] == "row 5" and res["documents"][0][0] == "moved" and res["ids"][0][1] != "row 5"
    chroma._REGISTRY.clear()
