#!/usr/bin/env python3
"""Generate golden fixtures by running the REFERENCE's own Python code (this container only).

The reference (Yaron9/AH-RAG @ /root/reference, read-only) imports two third-party packages that
are absent here: `sentence_transformers` (hierarchical_graph.py:8) and `chromadb` (:12-13). This
script injects in-memory stand-ins for them and then drives the reference's unmodified
HierarchicalGraph / GraphEnvironment / AHRAGGymEnv / NaiveRAG over a seeded synthetic graph,
recording their outputs as data under tests/golden/:

  reference_graph/structure.json, meta.json   the reference's own save() output
  search_cases.json                           HierarchicalGraph.search (R3-R8)
  env_cases.json                              GraphEnvironment action scripts (R9-R11)
  gym_cases.json                              AHRAGGymEnv episodes (R10, R12)
  naive_cases.json                            NaiveRAG.run contexts (R13)
  collection_cases.json                       every raw collection upsert / query the reference's
                                              build_vector_index / search made for search_cases and
                                              upsert_cases (the Chroma seam, ah_rag.collection)

Stand-ins (test scaffolding, not product code):
  * encoder: sha1(text) seeds numpy.default_rng -> standard normal vector, L2-normalised in fp32
    (identical to ah_rag.embeddings.HashEncoder, which the tests check by digest);
  * collection: exhaustive cosine over the stored vectors. Scores are the fp32 fma chain of the
    C oracle (oracle/ahr_oracle.c, mode 0), distance = float32(1 - score) as hnswlib returns it, ranking
    (score desc, insertion order asc) — what Chroma returns when its HNSW walk is exhaustive.

Run: python tests/golden/make_golden.py   (needs /root/reference; never runs on the GPU box)
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
from oracle import dense_ref  # noqa: E402  (C oracle for the fp32 fma-chain scores)

DIMS = {"all-MiniLM-L6-v2": 384, "sentence-transformers/all-MiniLM-L6-v2": 384}


# --------------------------------------------------------------------------------------------
# stand-ins for the absent third-party packages
# --------------------------------------------------------------------------------------------
from oracle.encoder_stub import encode as stub_encode  # noqa: E402


_TEXT_OF: dict = {}  # sha1 of an encoded single-text query vector -> its text (collection_cases)


def _vsha(v) -> str:
    return hashlib.sha1(np.asarray(v, np.float32).tobytes()).hexdigest()


class StubSentenceTransformer:
    def __init__(self, model_name: str, **_):
        self.dim = DIMS.get(model_name, 384)

    def encode(self, texts, normalize_embeddings=False, show_progress_bar=False, **_):
        out = stub_encode(texts, self.dim, normalize=normalize_embeddings)
        if not isinstance(texts, str) and len(texts) == 1 and normalize_embeddings:
            _TEXT_OF[_vsha(out[0])] = texts[0]
        return out


_STORE: dict = {}
# The raw collection traffic while RECORD["on"] (collection_cases.json): the reference's own
# upsert / query arguments and the stand-in's answers, per collection (db directory name / name).
RECORD: dict = {"on": False, "calls": []}


class StubCollection:
    def __init__(self, tag="", metadata=None):
        self.ids, self.vecs, self.metas, self.docs = [], [], [], []
        self.tag, self.metadata = tag, metadata

    def upsert(self, ids, documents=None, embeddings=None, metadatas=None):
        if RECORD["on"]:
            # the vectors are the stand-in encoder's of the documents (checked): stored as text
            enc = stub_encode(list(documents), len(embeddings[0]), normalize=True)
            assert np.array_equal(enc, np.asarray(embeddings, np.float32)), "upsert vectors are not encode(documents)"
            RECORD["calls"].append({"coll": self.tag, "op": "upsert", "ids": list(ids), "documents": list(documents),
                                    "metadatas": [dict(m) for m in metadatas], "dim": len(embeddings[0])})
        for i, nid in enumerate(ids):
            vec = np.asarray(embeddings[i], np.float32)
            meta = dict(metadatas[i]) if metadatas else {}
            doc = documents[i] if documents else None
            if nid in self.ids:
                j = self.ids.index(nid)
                self.vecs[j], self.metas[j], self.docs[j] = vec, meta, doc
            else:
                self.ids.append(nid); self.vecs.append(vec); self.metas.append(meta); self.docs.append(doc)

    def query(self, query_embeddings, n_results=10, include=None):
        out = {"ids": [], "distances": [], "metadatas": [], "documents": []}
        C = np.stack(self.vecs) if self.vecs else np.zeros((0, len(query_embeddings[0])), np.float32)
        for q in query_embeddings:
            s = dense_ref.scores_matrix(C, np.asarray([q], np.float32), mode="fma")[0]
            order = sorted(range(len(s)), key=lambda i: (-float(s[i]), i))[:n_results]
            out["ids"].append([self.ids[i] for i in order])
            # hnswlib (Chroma's index) returns 1 - <q, x> as a float32 distance
            out["distances"].append([float(np.float32(1.0) - np.float32(s[i])) for i in order])
            out["metadatas"].append([self.metas[i] for i in order])
            out["documents"].append([self.docs[i] for i in order])
        if RECORD["on"]:
            RECORD["calls"].append({"coll": self.tag, "op": "query",
                                    "texts": [_TEXT_OF[_vsha(q)] for q in query_embeddings],
                                    "n_results": n_results, "include": list(include or []), "result": out})
        return out


class StubClient:
    def __init__(self, path=None, settings=None):
        self.path = os.path.abspath(path or ".")

    def delete_collection(self, name):
        if RECORD["on"]:
            RECORD["calls"].append({"coll": f"{os.path.basename(self.path)}/{name}", "op": "delete"})
        _STORE.pop((self.path, name), None)

    def get_or_create_collection(self, name, metadata=None):
        if (self.path, name) not in _STORE:
            _STORE[(self.path, name)] = StubCollection(f"{os.path.basename(self.path)}/{name}", metadata)
            if RECORD["on"]:
                RECORD["calls"].append({"coll": _STORE[(self.path, name)].tag, "op": "create", "metadata": metadata})
        return _STORE[(self.path, name)]


def install_stubs() -> None:
    st = types.ModuleType("sentence_transformers")
    st.SentenceTransformer = StubSentenceTransformer
    sys.modules["sentence_transformers"] = st
    ch = types.ModuleType("chromadb")
    ch.PersistentClient = StubClient
    cfg = types.ModuleType("chromadb.config")
    cfg.Settings = lambda **kw: kw
    ch.config = cfg
    sys.modules["chromadb"] = ch
    sys.modules["chromadb.config"] = cfg


# --------------------------------------------------------------------------------------------
# synthetic graph built through the reference's own API
# --------------------------------------------------------------------------------------------
def build_graph(HierarchicalGraph, seed: int = 20251003):
    rng = np.random.default_rng(seed)
    hg = HierarchicalGraph()
    n_sum, n_l2, n_ent, n_hedge = 48, 5, 260, 110
    sids = []
    for t in range(n_sum):
        conf = [None, 7, 6.5, 8.25, 3][t % 5]
        judge = None if t % 7 == 3 else {"overall": float(rng.integers(30, 95)) / 10.0, "coherence": 5}
        sid = hg.add_summary(topic_id=t, title=f"Topic {t} on {['film', 'music', 'science', 'sport'][t % 4]}",
                             summary_text=f"Summary of topic {t}: " + " ".join(f"w{int(x)}" for x in rng.integers(0, 500, 6)),
                             confidence=conf, top_words=[f"w{int(x)}" for x in rng.integers(0, 500, 12)],
                             judge_scores=judge)
        sids.append(sid)
    hg.G.nodes[sids[5]]["judge_scores"] = "{not json"  # parse failure -> judge None
    hg.G.nodes[sids[9]]["judge_scores"] = json.dumps({"coherence": 4})  # no "overall" -> 0.0
    l2 = []
    for j in range(n_l2):
        sid = hg.add_summary(topic_id=100 + j, title=f"Community {j}", summary_text=f"L2 community {j}",
                             confidence=9.0, top_words=["c", str(j)], judge_scores={"overall": 7.5})
        hg.G.nodes[sid]["level"] = 2
        l2.append(sid)
    for t, sid in enumerate(sids):
        hg.add_belongs_to(sid, l2[t % n_l2], prob=1.0)
    eids = []
    for i in range(n_ent):
        eid = hg.add_entity(name=f"Entity {i} {['Burton', 'Depp', 'Derrickson', 'Gunn', 'Bates'][i % 5]}",
                            description=f"Entity number {i} appears in passage {int(rng.integers(0, 25))}",
                            entity_type=["person", "film", "org"][i % 3])
        eids.append(eid)
    # belongs_to: 0-3 parents, inserted in random order (exercises [:2] and load order)
    members = {s: [] for s in sids}
    for eid in eids:
        k = int(rng.choice([0, 1, 1, 2, 2, 3]))
        for s in rng.choice(n_sum, size=k, replace=False):
            members[sids[int(s)]].append(eid)
    for s in sids:
        order = list(members[s])
        rng.shuffle(order)
        for eid in order:
            hg.add_belongs_to(eid, s, prob=float(rng.random()))
    for _ in range(70):
        a, b = rng.choice(n_sum, size=2, replace=False)
        hg.add_related(sids[int(a)], sids[int(b)], weight=float(rng.random()))
    for h in range(n_hedge):
        hid = hg.add_hyperedge(uid=f"h{h}", description=f"Relation {h} between entities",
                               relation_type=["CoOccurrence", "Mention", "Directed"][h % 3],
                               confidence_score=5.0)
        for e in rng.choice(n_ent, size=int(rng.integers(1, 6)), replace=False):
            hg.add_participation(eids[int(e)], hid, role="arg")
    return hg, sids, eids


def strip_ts(obj):
    if isinstance(obj, dict):
        return {k: ("<ts>" if k in ("updated_at", "created_at") else strip_ts(v)) for k, v in obj.items()
                if k not in ("time_s",)}
    if isinstance(obj, list):
        return [strip_ts(x) for x in obj]
    if isinstance(obj, float) and not np.isfinite(obj):
        return repr(obj)
    return obj


def jsonable(obj):
    if isinstance(obj, np.ndarray):
        return obj.tolist()
    if isinstance(obj, (np.floating,)):
        return float(obj)
    if isinstance(obj, (np.integer,)):
        return int(obj)
    if isinstance(obj, set):
        return sorted(obj)
    raise TypeError(type(obj))


def dump(name, data):
    with open(os.path.join(HERE, name), "w", encoding="utf-8") as f:
        json.dump(strip_ts(data), f, ensure_ascii=False, separators=(",", ":"), default=jsonable)


def main() -> None:
    install_stubs()
    sys.path.insert(0, os.path.join(REF, "src"))
    sys.path.insert(0, REF)
    from ah_rag.graph.hierarchical_graph import HierarchicalGraph
    from ah_rag.agent.environment import GraphEnvironment
    from ah_rag.agent.gym_env import AHRAGGymEnv
    from baselines.naive_rag import NaiveRAG

    work = tempfile.mkdtemp(prefix="ahr_golden_")
    cwd = os.getcwd()
    os.chdir(work)  # AHRAGGymEnv logs under ./artifacts
    try:
        hg, sids, eids = build_graph(HierarchicalGraph)
        gdir = os.path.join(work, "graph")
        hg.save(gdir)
        hg = HierarchicalGraph.load(gdir)  # the loaded graph is what every caller sees
        db = os.path.join(work, "vector_db")
        hg.G.graph["vector_index"]["db_path"] = db
        RECORD["on"] = True
        hg.build_vector_index(db_path=db, layers={0, 1}, reset=True)
        hg.save(gdir)
        out_graph = os.path.join(HERE, "reference_graph")
        shutil.rmtree(out_graph, ignore_errors=True)
        os.makedirs(out_graph)
        for fn in ("structure.json", "meta.json"):
            shutil.copy(os.path.join(gdir, fn), os.path.join(out_graph, fn))
        # meta.json keeps the absolute temp db_path; record the relative name instead
        with open(os.path.join(out_graph, "meta.json")) as f:
            meta = json.load(f)
        meta["vector_index"]["db_path"] = "vector_db"
        with open(os.path.join(out_graph, "meta.json"), "w") as f:
            json.dump(meta, f, ensure_ascii=False, indent=2)

        names = [hg.G.nodes[e]["name"] for e in eids[:6]]
        titles = [hg.G.nodes[s]["title"] for s in sids[:4]]
        queries = names + titles + ["Tim Burton", "a film about horror", "quantum processor release",
                                    "music producer and composer", "sports community", "Entity 17 Gunn"]
        combos = [
            {"top_k": 5},
            {"top_k": 10, "member_top_m": 3},
            {"top_k": 8, "type_filter": ["summary"]},
            {"top_k": 6, "judge_overall_min": 6.0, "confidence_min": 5.0},
            {"top_k": 7, "alpha": 0.5, "beta": 0.3, "gamma": 0.15, "delta": 0.05},
            {"top_k": 4, "member_top_m": 8},
            {"top_k": 12, "type_filter": ["entity", "summary"], "judge_overall_min": 4.0},
            {"top_k": 40, "member_top_m": 5},  # beyond the fused kernels' 32: the large-k path
        ]
        search_cases = []
        for q in queries:
            for ci, params in enumerate(combos):
                rc = ci % 2 == 0
                res = hg.search(q, return_cluster=rc, **params)
                search_cases.append({"query": q, "params": params, "return_cluster": rc, "result": res})
        # hyperedges indexed too (seeds of type hyperedge: no expansion)
        db2 = os.path.join(work, "vector_db_h")
        hg2 = HierarchicalGraph.load(gdir)
        hg2.build_vector_index(db_path=db2, layers={0, 1}, include_hyperedges=True, reset=True)
        for q in queries[:6]:
            res = hg2.search(q, top_k=8, return_cluster=True, db_path=db2)
            search_cases.append({"query": q, "params": {"top_k": 8}, "return_cluster": True,
                                 "include_hyperedges": True, "result": res})
        dump("search_cases.json", {"dim": 384, "model": "all-MiniLM-L6-v2", "cases": search_cases})

        # ---- incremental re-index after node edits (build_vector_index upsert_only, :602-673)
        hg3 = HierarchicalGraph.load(gdir)
        db3 = os.path.join(work, "vector_db_up")
        hg3.build_vector_index(db_path=db3, layers={0, 1}, upsert_only=False, reset=True)
        before = dict(hg3.G.graph["vector_index"]["indexed_meta"])
        probe = queries[:6] + ["a freshly edited description of entity three", "Topic 2 renamed"]
        pre = [hg3.search(q, top_k=8, return_cluster=True, db_path=db3) for q in probe[:2]]
        edits = [[eids[3], "description", "a freshly edited description of entity three"],
                 [eids[10], "description", "Entity number ten now appears in passage 99"],
                 [sids[2], "title", "Topic 2 renamed"]]
        for nid, key, val in edits:
            hg3.G.nodes[nid][key] = val
        new_eid = hg3.add_entity(name="Entity Brand New", description="added after the first index build",
                                 entity_type="person")
        hg3.add_belongs_to(new_eid, sids[2], prob=0.5)
        hg3.build_vector_index(db_path=db3, layers={0, 1}, upsert_only=True)
        after = dict(hg3.G.graph["vector_index"]["indexed_meta"])
        post = [{"query": q, "result": hg3.search(q, top_k=8, return_cluster=True, db_path=db3)} for q in probe]
        RECORD["on"] = False
        dump("collection_cases.json", {"dim": 384, "model": "all-MiniLM-L6-v2", "calls": RECORD["calls"]})
        dump("upsert_cases.json", {"edits": edits, "new_entity": {"name": "Entity Brand New", "id": new_eid,
                                                                  "summary": sids[2]},
                                   "indexed_meta_before": before, "indexed_meta_after": after,
                                   "changed": sorted(k for k in after if before.get(k) != after[k]),
                                   "pre": [{"query": q, "result": r} for q, r in zip(probe[:2], pre)],
                                   "post": post, "vector_index": {k: v for k, v in hg3.G.graph["vector_index"].items()
                                                                  if k != "db_path"}})

        # ---- GraphEnvironment scripts
        env_cases = []
        for q in queries[:10]:
            env = GraphEnvironment(graph_dir=gdir, logging_enabled=False)
            hg_env = env.hg
            hg_env.G.graph["vector_index"]["db_path"] = db
            steps = []
            obs, info = env.reset(seed_query=q, top_k=5)
            steps.append({"call": "reset", "args": {"seed_query": q, "top_k": 5}, "obs": obs, "info": info})
            top = [x["node_id"] for x in obs["selection"]]

            def rec(call, args, fn):
                try:
                    o, i = fn(**args)
                    steps.append({"call": call, "args": args, "obs": o, "info": i})
                except Exception as e:  # reference exceptions are part of the contract
                    steps.append({"call": call, "args": args, "error": type(e).__name__, "message": str(e)})
            rec("expand_parents", {"node_ids": top[:2]}, env.expand_parents)
            rec("expand_children", {"node_ids": top[:2]}, env.expand_children)
            rec("expand_related", {"node_ids": top[:1]}, env.expand_related)
            rec("commit_selection", {"node_ids": top[:3]}, env.commit_selection)
            if top:
                rec("query_node_details", {"node_id": top[0]}, env.query_node_details)
            rec("query_node_details", {"node_id": "nope:missing"}, env.query_node_details)
            ents = [x for x in top if x.startswith("ent:")]
            summ = [x for x in top if x.startswith("sum:")]
            rec("expand_related", {"node_ids": ents[:2] + summ[:1], "limit": 10}, env.expand_related)
            rec("expand_children", {"node_ids": summ + [sids[1], sids[2]], "limit": 7}, env.expand_children)
            rec("expand_parents", {"node_ids": [sids[0], sids[3]] + ents, "limit": 4}, env.expand_parents)
            rec("expand_to_lca", {"node_ids": ents[:2] or [eids[0], eids[1]]}, env.expand_to_lca)
            rec("expand_to_lca", {"node_ids": [sids[0], sids[1]], "max_results": 3}, env.expand_to_lca)
            env.set_filters(judge_overall_min=5.0, type_filter=["summary", "entity"])
            env.set_search_weights(alpha=0.7, delta=0.3, top_k=6)
            rec("semantic_anchor", {"query": q, "top_k": 6}, env.semantic_anchor)
            rec("expand_related", {"node_ids": [eids[3], eids[4], eids[5]], "limit": 10}, env.expand_related)
            env_cases.append({"query": q, "steps": steps, "stats_cumulative": env.stats["cumulative"]})
        dump("env_cases.json", {"cases": env_cases})

        # ---- AHRAGGymEnv episodes (featurizer + reward + action mask)
        gym_cases = []
        scripts = [[0, 1, 2, 3, 4, 5], [2, 2, 0, 3, 1, 4], [3, 3, 1, 1, 0, 2], [4, 0, 2, 1, 3, 0, 1]]
        for qi, q in enumerate(queries[:8]):
            genv = AHRAGGymEnv(graph_dir=gdir, max_steps=6)
            genv.env.hg.G.graph["vector_index"]["db_path"] = db
            vec, info = genv.reset(q)
            ep = {"query": q, "reset": {"vec": vec, "info": info}, "steps": []}
            for a in scripts[qi % len(scripts)]:
                v, r, d, inf = genv.step(a)
                ep["steps"].append({"action": a, "vec": v, "reward": r, "done": d, "info": inf})
                if d:
                    break
            gym_cases.append(ep)
        dump("gym_cases.json", {"cases": gym_cases})

        # ---- NaiveRAG contexts (answer generation stubbed: it is downstream of this path)
        class EchoGen:
            def generate(self, query, context, cfg):
                return {"query": query, "context": context}
        naive = NaiveRAG(hg, EchoGen())
        dump("naive_cases.json", {"cases": [{"query": q, "top_k": k, "out": naive.run(q, top_k=k)}
                                            for q in queries[:8] for k in (5, 10)]})
        # digest of the stand-in encoder so tests can confirm HashEncoder reproduces it
        enc = StubSentenceTransformer("all-MiniLM-L6-v2")
        probe = enc.encode(queries, normalize_embeddings=True)
        with open(os.path.join(HERE, "encoder_digest.json"), "w") as f:
            json.dump({"texts": queries, "dim": 384,
                       "sha1": hashlib.sha1(probe.tobytes()).hexdigest()}, f, indent=1)
    finally:
        os.chdir(cwd)
        shutil.rmtree(work, ignore_errors=True)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
