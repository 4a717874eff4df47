"""HierarchicalGraph — drop-in for reference src/ah_rag/graph/hierarchical_graph.py (class at :21).

The graph model (networkx DiGraph of entity / hyperedge / summary nodes, node-link JSON
persistence) keeps the reference's data format, so graphs saved by either implementation load
in the other. What changes is the retrieval core behind the same signatures:

  build_vector_index  (reference :602-673) encodes node texts once and writes an on-disk vector
                      store (`<db_path>/ahr_vectors.npy` + `ahr_rows.json`) instead of a Chroma
                      SQLite collection, with the same sha1 upsert-only bookkeeping in
                      G.graph["vector_index"]["indexed_meta"];
  search              (reference :675-789) runs dense top-k, 1-hop expansion and rerank on the
                      MI355X (ah_rag.graph_search.SearchEngine -> libahr_hip.so) and only builds
                      the result dicts on the host. search_batch() answers many queries per call.

build_from_artifacts (:241-421) assembles the graph from an artifacts directory; the offline C1
ingest (ah_rag.ingest) feeds it the deterministic extractor's extractions.json.

Caching: the device index and device graph are built on first search and reused. Mutations made
through this class's add_* methods invalidate them; after editing self.G directly, call
invalidate_device_cache().
"""
from __future__ import annotations

import copy
import datetime
import hashlib
import itertools
import json
import os
import weakref
from typing import Any, Dict, List, Optional, Sequence, Tuple

import networkx as nx
import numpy as np
import torch

from ..embeddings import DEFAULT_MODEL, DenseIndex, load_encoder
from ..graph_search import (DeviceGraph, SEARCH_DEFAULTS, SearchEngine, parse_judge,
                            resolve_search_params)
from .. import _native as nat

ARTIFACT_DIR = "artifacts"
GRAPH_DIR = "graph"
STRUCTURE_FILE = os.path.join(GRAPH_DIR, "structure.json")
META_FILE = os.path.join(GRAPH_DIR, "meta.json")

VECTORS_FILE = "ahr_vectors.npy"
ROWS_FILE = "ahr_rows.json"

# Process-wide version numbers of resident indexes: a cache keyed on one can never match a later
# index (an id() can be reused once the old object is gone, and a per-object counter restarts).
_INDEX_VERSIONS = itertools.count(1)

# Process-wide sharing of what is derived from files (the reference's PPO loop builds every
# environment with AHRAGGymEnv(graph_dir=...), each loading the graph and opening the store again,
# scripts/train_ppo.py:25-26): the HBM copy of a vector store per (store path, storage type, GPU),
# the device graph per (saved graph file, GPU) while a loaded graph is unmodified, and the loaded
# graph itself per graph directory for the environments (HierarchicalGraph.load_shared). Weak
# values: an entry lives as long as some graph object uses it.
_RESIDENT: "weakref.WeakValueDictionary" = weakref.WeakValueDictionary()
_DEVICE_GRAPHS: "weakref.WeakValueDictionary" = weakref.WeakValueDictionary()
_SHARED_GRAPHS: "weakref.WeakValueDictionary" = weakref.WeakValueDictionary()


def _abspath(path: str) -> str:
    """os.path.abspath, memoised per (working directory, path): search() resolves the same store path
    on every call."""
    cwd = os.getcwd()
    k = (cwd, path)
    a = _ABSPATHS.get(k)
    if a is None:
        if len(_ABSPATHS) > 1024:
            _ABSPATHS.clear()
        a = _ABSPATHS[k] = os.path.abspath(path)
    return a


_ABSPATHS: Dict[Tuple[str, str], str] = {}


def _file_stamp(path: str) -> Tuple:
    try:
        st = os.stat(path)
        return (st.st_mtime_ns, st.st_size)
    except OSError:
        return (0, 0)


def _sha(text: str) -> str:
    return hashlib.sha1(text.encode("utf-8")).hexdigest()


class VectorStore:
    """The persisted node-vector collection (Chroma's role): rows of (id, fp32 vector, metadata)."""

    def __init__(self, path: str) -> None:
        self.path = path
        self.ids: List[str] = []
        self.metas: List[Dict[str, Any]] = []
        self.vectors = np.zeros((0, 0), np.float32)
        self.model: Optional[str] = None
        vp, rp = os.path.join(path, VECTORS_FILE), os.path.join(path, ROWS_FILE)
        if os.path.exists(vp) and os.path.exists(rp):
            with open(rp, encoding="utf-8") as f:
                rows = json.load(f)
            self.ids, self.metas, self.model = rows["ids"], rows["metadatas"], rows.get("model")
            self.vectors = np.load(vp, allow_pickle=False)

    def clear(self) -> None:
        self.ids, self.metas = [], []
        self.vectors = np.zeros((0, 0), np.float32)

    def upsert(self, ids: Sequence[str], vectors: np.ndarray, metas: Sequence[Dict[str, Any]]) -> None:
        slot = {nid: i for i, nid in enumerate(self.ids)}
        if self.vectors.size == 0:
            self.vectors = np.zeros((0, vectors.shape[1]), np.float32)
        if vectors.shape[1] != self.vectors.shape[1]:
            raise ValueError("embedding dimension differs from the stored collection")
        new_rows = []
        for nid, v, m in zip(ids, vectors, metas):
            if nid in slot:
                self.vectors[slot[nid]] = v
                self.metas[slot[nid]] = dict(m)
            else:
                slot[nid] = len(self.ids) + len(new_rows)
                new_rows.append((nid, v, m))
        if new_rows:
            self.ids += [r[0] for r in new_rows]
            self.metas += [dict(r[2]) for r in new_rows]
            self.vectors = np.concatenate([self.vectors, np.stack([r[1] for r in new_rows])]).astype(np.float32)

    def save(self, model: str) -> None:
        os.makedirs(self.path, exist_ok=True)
        self.model = model
        np.save(os.path.join(self.path, VECTORS_FILE), self.vectors.astype(np.float32), allow_pickle=False)
        with open(os.path.join(self.path, ROWS_FILE), "w", encoding="utf-8") as f:
            json.dump({"model": model, "ids": self.ids, "metadatas": self.metas}, f, ensure_ascii=False)

    def stamp(self) -> Tuple:
        return store_stamp(self.path)


def store_stamp(path: str) -> Tuple:
    """(mtime, size) of a store's vector file: a change made by another writer forces a reload."""
    try:
        st = os.stat(os.path.join(path, VECTORS_FILE))
        return (st.st_mtime_ns, st.st_size)
    except OSError:
        return (0, 0)


class ResidentIndex:
    """The HBM copy of one vector store (Chroma's collection role): DenseIndex + row id table.

    build_vector_index writes it incrementally — rows whose sha1 key changed are upserted into
    their slots, new nodes appended (ahr_index_upsert), the reference's collection semantics
    (hierarchical_graph.py:660: existing ids updated in place, new ids appended in order) — so a
    re-index after editing a few nodes moves those rows only, never the whole store."""

    def __init__(self, path: str, device) -> None:
        self.path = path
        self.device = device
        self.dtype = os.environ.get("AHR_INDEX_DTYPE", "f32")
        self.full_loads = 0
        self.rows_upserted = 0
        self.version = 0
        self.index: Optional[DenseIndex] = None
        self.reload()

    def reload(self) -> None:
        store = VectorStore(self.path)
        n, dim = store.vectors.shape if store.vectors.size else (0, 1)
        self._alloc(dim, max(n, 1))
        if n:
            self.index.upsert(store.vectors)
        self.ids, self.metas = list(store.ids), list(store.metas)
        self.slot = {nid: i for i, nid in enumerate(self.ids)}
        self.stamp = store.stamp()
        self.full_loads += 1
        self.version = next(_INDEX_VERSIONS)

    def _alloc(self, dim: int, capacity: int) -> None:
        if self.index is not None:
            self.index.close()
        # headroom so that appended nodes rarely force a reallocation
        self.index = DenseIndex(dim, capacity + max(256, capacity // 4), dtype=self.dtype, device=self.device)

    def apply(self, ids: Sequence[str], vectors: np.ndarray, metas: Sequence[Dict[str, Any]]) -> None:
        """Upsert rows into the resident index in the store's slot order (VectorStore.upsert)."""
        if vectors.shape[1] != self.index.dim:
            self.reload()
            return
        old_i, old_s, new_i = [], [], []
        for i, nid in enumerate(ids):
            if nid in self.slot:
                old_i.append(i)
                old_s.append(self.slot[nid])
                self.metas[self.slot[nid]] = dict(metas[i])
            else:
                new_i.append(i)
        n0 = len(self.ids)
        if n0 + len(new_i) > self.index.capacity:
            self.reload()  # grow: one full upload of the (already saved) store
            return
        if old_i:
            self.index.upsert(vectors[old_i], slots=np.asarray(old_s, np.int64))
        if new_i:
            self.index.upsert(vectors[new_i], start=n0)
            for i in new_i:
                self.slot[ids[i]] = len(self.ids)
                self.ids.append(ids[i])
                self.metas.append(dict(metas[i]))
        self.rows_upserted += len(old_i) + len(new_i)
        self.stamp = store_stamp(self.path)
        self.version = next(_INDEX_VERSIONS)

    def close(self) -> None:
        if self.index is not None:
            self.index.close()


class HierarchicalGraph:
    """Unified DiGraph of L0 entities, L0 hyperedges and L1+ summaries (attributes on nodes/edges)."""

    def __init__(self) -> None:
        self.G: nx.DiGraph = nx.DiGraph()
        self.name_to_entity_id: Dict[str, str] = {}
        self.topic_to_summary_id: Dict[int, str] = {}
        self._query_embedder_name: Optional[str] = None
        self._query_embedder = None
        self.G.graph.setdefault("search_params", copy.deepcopy(SEARCH_DEFAULTS))
        self.G.graph.setdefault("dirty", False)
        self.G.graph.setdefault("vector_index", {"db_path": "vector_db", "model": DEFAULT_MODEL,
                                                 "indexed_nodes": 0, "indexed_meta": {}})
        self._version = 0
        self._source: Optional[Tuple] = None  # (saved structure file, its stamp, node count) after load()
        self._dev_graph: Optional[Tuple[Tuple, DeviceGraph]] = None
        self._indexes: Dict[str, ResidentIndex] = {}
        self._engines: Dict[str, Tuple[Tuple, SearchEngine]] = {}

    # ---- ids ---------------------------------------------------------------------------------
    @staticmethod
    def _hash(text: str, length: int = 10) -> str:
        return _sha(text)[:length]

    @staticmethod
    def make_entity_id(name: str) -> str:
        return "ent:" + HierarchicalGraph._hash(name)

    @staticmethod
    def make_hyperedge_id(uid: str) -> str:
        return "hedge:" + uid

    @staticmethod
    def make_summary_id(topic_id: int) -> str:
        return "sum:%d" % int(topic_id)

    # ---- mutation (ingest-side API the graph builders use) -----------------------------------
    def _touch(self) -> None:
        self.G.graph["dirty"] = True
        self._version += 1

    def add_entity(self, name: str, description: Optional[str] = None, entity_type: Optional[str] = None,
                   embedding_ref: Optional[Tuple[str, int]] = None,
                   l1_parents: Optional[Dict[str, float]] = None) -> str:
        nid = self.name_to_entity_id.get(name)
        parents_json = json.dumps(l1_parents) if l1_parents else None
        if nid is None:
            nid = self.make_entity_id(name)
            self.G.add_node(nid, node_type="entity", name=name, description=description,
                            entity_type=entity_type, embedding_ref=embedding_ref, l1_parents=parents_json)
            self.name_to_entity_id[name] = nid
        else:
            attrs = self.G.nodes[nid]
            if description is not None and not attrs.get("description"):
                attrs["description"] = description
            if entity_type is not None and not attrs.get("entity_type"):
                attrs["entity_type"] = entity_type
            if embedding_ref is not None:
                attrs["embedding_ref"] = embedding_ref
            if l1_parents is not None:
                attrs["l1_parents"] = json.dumps(l1_parents)
        self._touch()
        return nid

    def add_hyperedge(self, uid: str, description: str, relation_type: str,
                      confidence_score: Optional[float] = None, source_text_ref: Optional[str] = None) -> str:
        nid = self.make_hyperedge_id(uid)
        if nid not in self.G:
            self.G.add_node(nid, node_type="hyperedge", description=description, relation_type=relation_type,
                            confidence_score=confidence_score, source_text_ref=source_text_ref)
        self._touch()
        return nid

    def add_summary(self, topic_id: int, title: Optional[str] = None, summary_text: Optional[str] = None,
                    confidence: Optional[float] = None, top_words: Optional[List[str]] = None,
                    members: Optional[List[str]] = None, judge_scores: Optional[Dict[str, Any]] = None,
                    centroid: Optional[List[float]] = None) -> str:
        tid = int(topic_id)
        enc = {"top_words": json.dumps(top_words) if top_words is not None else None,
               "members": json.dumps(members) if members is not None else None,
               "judge_scores": json.dumps(judge_scores) if judge_scores is not None else None,
               "centroid": json.dumps(centroid) if centroid is not None else None}
        nid = self.topic_to_summary_id.get(tid)
        if nid is None:
            nid = self.make_summary_id(tid)
            # new nodes store falsy lists/dicts as None (the reference's `x if x else None`)
            self.G.add_node(nid, node_type="summary", topic_id=tid, title=title, summary_text=summary_text,
                            confidence=confidence,
                            top_words=enc["top_words"] if top_words else None,
                            members=enc["members"] if members else None,
                            judge_scores=enc["judge_scores"] if judge_scores else None,
                            centroid=enc["centroid"])
            self.topic_to_summary_id[tid] = nid
        else:
            attrs = self.G.nodes[nid]
            for key, val in (("title", title), ("summary_text", summary_text), ("confidence", confidence)):
                if val is not None:
                    attrs[key] = val
            for key, raw in (("top_words", top_words), ("members", members), ("judge_scores", judge_scores),
                             ("centroid", centroid)):
                if raw is not None:
                    attrs[key] = enc[key]
        self._touch()
        return nid

    def add_participation(self, entity_id: str, hyperedge_id: str, role: Optional[str] = None) -> None:
        self.G.add_edge(entity_id, hyperedge_id, edge_type="participates_in", role=role)
        self._touch()

    def add_belongs_to(self, entity_id: str, summary_id: str, prob: Optional[float] = None) -> None:
        self.G.add_edge(entity_id, summary_id, edge_type="belongs_to", prob=prob)
        self._touch()

    def add_related(self, summary_a: str, summary_b: str, weight: Optional[float] = None,
                    jaccard: Optional[float] = None, cosine: Optional[float] = None,
                    overlap: Optional[int] = None, confidence: Optional[float] = None) -> None:
        self.G.add_edge(summary_a, summary_b, edge_type="related_to", weight=weight, jaccard=jaccard,
                        cosine=cosine, overlap=overlap, confidence=confidence)
        self._touch()

    def build_from_artifacts(self, artifacts_dir: str = ARTIFACT_DIR) -> None:
        """Assemble the graph from an ingest artifacts directory (reference :241-421).

        Reads whichever of topics.json (entity_to_parents, l1_nodes), l1_nodes.json, l1_edges.json,
        l1_judge_nodes.json, l1_judge_edges.json, extractions.json, l2_nodes.json and l1_to_l2.json
        exist, in the reference's order of node and edge insertion (it fixes networkx adjacency
        order, which search()'s [:2] / [:member_top_m] truncations see). The
        offline C1 path has extractions.json only (ah_rag.extract): entities, hyperedges and
        participates_in edges."""
        def read(name: str, default):
            path = os.path.join(artifacts_dir, name)
            if not os.path.exists(path):
                return default
            with open(path, encoding="utf-8") as f:
                return json.load(f)

        topics = read("topics.json", {})
        entity_to_parents: Dict[str, List[Dict[str, Any]]] = topics.get("entity_to_parents", {}) if topics else {}
        l1_nodes = read("l1_nodes.json", topics.get("l1_nodes", []) if topics else [])
        l1_edges = read("l1_edges.json", [])
        judge_nodes = read("l1_judge_nodes.json", [])
        judge_edges = read("l1_judge_edges.json", [])
        extractions = read("extractions.json", [])
        l2_nodes = read("l2_nodes.json", [])
        l1_to_l2 = read("l1_to_l2.json", {})

        # entity facts gathered from every extraction: distinct descriptions, first-seen type
        facts: Dict[str, Dict[str, Any]] = {}
        for rec in extractions:
            for ent in rec.get("entities", []):
                name = ent.get("name")
                if not name:
                    continue
                f = facts.setdefault(name, {"descriptions": [], "entity_type": ent.get("type")})
                desc = ent.get("description")
                if desc and desc not in f["descriptions"]:
                    f["descriptions"].append(desc)

        def joined(name: str) -> Optional[str]:
            descs = facts.get(name, {}).get("descriptions", [])
            return "; ".join(descs) if descs else None

        # entities with topic parents first (their order), then the rest in extraction order
        for name, parents in entity_to_parents.items():
            self.add_entity(name=name, description=joined(name), entity_type=facts.get(name, {}).get("entity_type"),
                            embedding_ref=(os.path.join(ARTIFACT_DIR, "embeddings.npy"), -1),
                            l1_parents={str(p.get("topic_id")): p.get("prob") for p in parents})
        for name, f in facts.items():
            if name not in entity_to_parents:
                self.add_entity(name=name, description=joined(name), entity_type=f.get("entity_type"))
        for node in l1_nodes:
            self.add_summary(topic_id=int(node.get("topic_id")), title=node.get("title"),
                             summary_text=node.get("summary") or node.get("summary_text"),
                             confidence=node.get("confidence"), top_words=node.get("top_words") or [],
                             members=node.get("members") or [], centroid=node.get("centroid"))
        for name, parents in entity_to_parents.items():
            eid = self.name_to_entity_id.get(name)
            if not eid:
                continue
            for p in parents:
                sid = self.topic_to_summary_id.get(int(p.get("topic_id")))
                if sid:
                    self.add_belongs_to(eid, sid, prob=p.get("prob"))
        for e in l1_edges:
            a = self.topic_to_summary_id.get(int(e.get("source")))
            b = self.topic_to_summary_id.get(int(e.get("target")))
            if a and b:
                self.add_related(a, b, weight=e.get("weight"), jaccard=e.get("jaccard"), cosine=e.get("cosine"),
                                 overlap=e.get("overlap"), confidence=e.get("confidence"))
        for i, rec in enumerate(extractions):
            uid = rec.get("id")
            if uid is None:
                uid = "hedge_%d_%s" % (i, rec.get("relation_type", "unknown"))
            hid = self.add_hyperedge(uid=str(uid), description=rec.get("hyperedge"),
                                     relation_type=rec.get("relation_type"),
                                     confidence_score=rec.get("confidence_score"))
            for ent in rec.get("entities", []):
                eid = self.name_to_entity_id.get(ent.get("name")) if ent.get("name") else None
                if eid:
                    self.add_participation(eid, hid, role=ent.get("role") if isinstance(ent, dict) else None)
        if l2_nodes:
            for n in l2_nodes:
                sid = self.add_summary(topic_id=int(n.get("topic_id")), title=n.get("title"),
                                       summary_text=n.get("summary"), confidence=n.get("confidence"),
                                       top_words=n.get("top_words"), members=n.get("members"),
                                       centroid=n.get("centroid"))
                self.G.nodes[sid]["level"] = 2
            for l1_key, l2_tid in l1_to_l2.items():
                try:
                    l1_sid = self.topic_to_summary_id.get(int(l1_key))
                except (TypeError, ValueError):
                    continue
                l2_sid = self.topic_to_summary_id.get(int(l2_tid))
                if l1_sid and l2_sid:
                    self.add_belongs_to(l1_sid, l2_sid, prob=1.0)
        by_topic = {int(d.get("topic_id")): n for n, d in self.G.nodes(data=True) if d.get("node_type") == "summary"}
        for js in judge_nodes:
            nid = by_topic.get(int(js.get("id")))
            if nid:
                self.G.nodes[nid]["judge_scores"] = json.dumps(js)
        if judge_edges:
            self.G.graph["judge_edges"] = judge_edges

    def invalidate_device_cache(self) -> None:
        self._version += 1

    # ---- persistence (node-link JSON, reference :175-236) ------------------------------------
    def save(self, directory: str = GRAPH_DIR, meta: Optional[Dict[str, Any]] = None) -> None:
        os.makedirs(directory, exist_ok=True)
        with open(os.path.join(directory, "structure.json"), "w", encoding="utf-8") as f:
            json.dump(nx.node_link_data(self.G, edges="links"), f, ensure_ascii=False, indent=2)
        out = dict(meta or {})
        out.update({"search_params": self.G.graph.get("search_params", {}),
                    "graph_hash": self._graph_snapshot_hash(),
                    "dirty": self.G.graph.get("dirty", False),
                    "vector_index": self.G.graph.get("vector_index", {})})
        with open(os.path.join(directory, "meta.json"), "w", encoding="utf-8") as f:
            json.dump(out, f, ensure_ascii=False, indent=2)

    @classmethod
    def load_shared(cls, directory: str = GRAPH_DIR) -> "HierarchicalGraph":
        """load(directory), shared by every caller in the process while the saved files and the
        loaded graph are unchanged: GraphEnvironment / AHRAGGymEnv(graph_dir=...) use it, so the
        environments of one training loop parse the graph (seconds at 130k nodes) and build its
        device structures once. The environment API only reads the graph; a graph changed through
        add_* is not handed out again. AHR_SHARE_GRAPH=0 gives every caller its own load()."""
        if os.environ.get("AHR_SHARE_GRAPH", "1") == "0":
            return cls.load(directory)
        d = os.path.abspath(directory)
        key = (d, _file_stamp(os.path.join(d, "structure.json")), _file_stamp(os.path.join(d, "meta.json")))
        hg = _SHARED_GRAPHS.get(key)
        if hg is None or hg._version != 0 or hg._source is None or len(hg.G) != hg._source[2]:
            hg = cls.load(directory)
            _SHARED_GRAPHS[key] = hg
        return hg

    @classmethod
    def load(cls, directory: str = GRAPH_DIR) -> "HierarchicalGraph":
        spath = os.path.abspath(os.path.join(directory, "structure.json"))
        stamp = _file_stamp(spath)
        with open(os.path.join(directory, "structure.json"), encoding="utf-8") as f:
            data = json.load(f)
        hg = cls()
        hg.G = nx.node_link_graph(data, directed=True, edges="links")
        for nid, attrs in hg.G.nodes(data=True):
            kind = attrs.get("node_type")
            if kind == "entity" and attrs.get("name"):
                hg.name_to_entity_id[attrs["name"]] = nid
            elif kind == "summary" and attrs.get("topic_id") is not None:
                hg.topic_to_summary_id[int(attrs["topic_id"])] = nid
        hg.G.graph.setdefault("search_params", copy.deepcopy(SEARCH_DEFAULTS))
        hg.G.graph.setdefault("dirty", False)
        hg.G.graph.setdefault("vector_index", {"db_path": "vector_db", "model": DEFAULT_MODEL,
                                               "indexed_nodes": 0, "indexed_meta": {}})
        mp = os.path.join(directory, "meta.json")
        if os.path.exists(mp):
            try:
                with open(mp, encoding="utf-8") as f:
                    meta = json.load(f)
                if isinstance(meta.get("search_params"), dict):
                    hg.G.graph["search_params"] = {**hg.G.graph["search_params"], **meta["search_params"]}
                if isinstance(meta.get("vector_index"), dict):
                    hg.G.graph["vector_index"] = meta["vector_index"]
                if isinstance(meta.get("dirty"), bool):
                    hg.G.graph["dirty"] = meta["dirty"]
            except Exception:
                pass
        hg._source = (spath, stamp, len(hg.G))
        return hg

    def _graph_snapshot_hash(self) -> str:
        rows = sorted(((nid, d.get("node_type"), d.get("name"), d.get("title"), d.get("summary_text"),
                        d.get("description")) for nid, d in self.G.nodes(data=True)), key=lambda r: r[0])
        return _sha(json.dumps(rows, ensure_ascii=False))

    # ---- lookups (reference :426-553) --------------------------------------------------------
    def get_parents(self, node_id: str) -> List[str]:
        return list(self.G.successors(node_id))

    def get_children(self, node_id: str) -> List[str]:
        return list(self.G.predecessors(node_id))

    def find_entity(self, name: str) -> Optional[str]:
        return self.name_to_entity_id.get(name)

    def find_summary(self, topic_id: int) -> Optional[str]:
        return self.topic_to_summary_id.get(int(topic_id))

    def _neighbors_by_edge_type(self, node_id: str, direction: str, edge_type: str) -> List[str]:
        adj = self.G.succ if direction == "out" else self.G.pred
        return [nb for nb, a in adj[node_id].items() if a.get("edge_type") == edge_type]

    def get_belongs_to(self, node_id: str) -> List[str]:
        return self._neighbors_by_edge_type(node_id, "out", "belongs_to")

    def get_summary_members(self, summary_id: str) -> List[str]:
        return self._neighbors_by_edge_type(summary_id, "in", "belongs_to")

    def get_hyperedge_participants(self, hyperedge_id: str) -> List[str]:
        return self._neighbors_by_edge_type(hyperedge_id, "in", "participates_in")

    def get_entity_hyperedges(self, entity_id: str) -> List[str]:
        return self._neighbors_by_edge_type(entity_id, "out", "participates_in")

    def get_siblings(self, node_id: str) -> List[str]:
        sibs = {c for p in set(self.get_belongs_to(node_id)) for c in self.get_summary_members(p)}
        sibs.discard(node_id)
        return list(sibs)

    def search_by_name_or_title(self, q: str, limit: int = 20) -> List[Tuple[str, Dict[str, Any]]]:
        needle = q.lower()
        hits = []
        for nid, d in self.G.nodes(data=True):
            if needle in str(d.get("name") or "").lower() or needle in str(d.get("title") or "").lower():
                hits.append((nid, d))
            if len(hits) >= limit:
                break
        return hits

    def summaries_with_top_word(self, word: str, limit: int = 50) -> List[str]:
        w = word.lower()
        hits: List[str] = []
        for nid, d in self.G.nodes(data=True):
            if d.get("node_type") != "summary":
                continue
            tw = d.get("top_words")
            if tw:
                try:
                    words = json.loads(tw) if isinstance(tw, str) else tw
                except Exception:
                    words = []
                if any(w in str(x).lower() for x in words):
                    hits.append(nid)
            if len(hits) >= limit:
                break
        return hits

    def validate_belongs_to_dag(self) -> bool:
        sub = nx.DiGraph([(u, v) for u, v, a in self.G.edges(data=True) if a.get("edge_type") == "belongs_to"])
        return nx.is_directed_acyclic_graph(sub)

    def validate_required_attributes(self) -> Dict[str, List[str]]:
        bad: Dict[str, List[str]] = {"entity": [], "hyperedge": [], "summary": []}
        for nid, d in self.G.nodes(data=True):
            kind = d.get("node_type")
            if kind == "entity" and not d.get("name"):
                bad["entity"].append(nid)
            elif kind == "hyperedge" and (not d.get("description") or not d.get("relation_type")):
                bad["hyperedge"].append(nid)
            elif kind == "summary" and d.get("topic_id") is None:
                bad["summary"].append(nid)
        return bad

    def stats(self) -> Dict[str, Any]:
        nodes = {k: 0 for k in ("entity", "hyperedge", "summary")}
        edges = {k: 0 for k in ("participates_in", "belongs_to", "related_to")}
        for _, d in self.G.nodes(data=True):
            if d.get("node_type") in nodes:
                nodes[d["node_type"]] += 1
        n_edges = 0
        for _, _, a in self.G.edges(data=True):
            n_edges += 1
            if a.get("edge_type") in edges:
                edges[a["edge_type"]] += 1
        return {"nodes": nodes, "edges": edges, "n_nodes": self.G.number_of_nodes(), "n_edges": n_edges}

    # ---- vector index (reference :558-673) ---------------------------------------------------
    def _embedding_text(self, node_id: str) -> Tuple[str, Dict[str, Any]]:
        d = self.G.nodes[node_id]
        kind = d.get("node_type")
        if kind == "entity":
            text = "Entity: %s. %s" % (d.get("name") or "", d.get("description") or "")
        elif kind == "summary":
            words: List[str] = []
            if d.get("top_words"):
                try:
                    words = json.loads(d["top_words"]) if isinstance(d["top_words"], str) else d["top_words"]
                except Exception:
                    words = []
            text = "Summary: %s. %s. Keywords: %s" % (d.get("title") or "",
                                                      d.get("summary_text") or d.get("summary") or "",
                                                      ", ".join(words[:10]) if words else "")
        else:
            text = "Relation: %s. %s" % (d.get("relation_type") or "", d.get("description") or "")
        meta = {"node_id": node_id, "node_type": kind,
                "layer": 0 if kind == "entity" else (1 if kind == "summary" else 0),
                "judge_overall": parse_judge(d.get("judge_scores")), "confidence": d.get("confidence"),
                "updated_at": datetime.datetime.utcnow().isoformat() + "Z"}
        return text, meta

    @staticmethod
    def _index_key(d: Dict[str, Any]) -> str:
        return _sha("|".join([str(d.get("node_type")), str(d.get("name") or d.get("title") or ""),
                              str(d.get("summary_text") or ""), str(d.get("description") or "")]))

    def build_vector_index(self, db_path: str = "vector_db", layers: set = {0, 1}, include_hyperedges: bool = False,
                           model_name: str = DEFAULT_MODEL, upsert_only: bool = True, reset: bool = False) -> None:
        os.makedirs(db_path, exist_ok=True)
        store = VectorStore(db_path)
        if reset:
            store.clear()
        vi = self.G.graph.get("vector_index", {})
        prev = vi.get("indexed_meta") if isinstance(vi.get("indexed_meta"), dict) else {}
        todo: List[str] = []
        for nid, d in self.G.nodes(data=True):
            kind = d.get("node_type")
            wanted = (kind == "entity" and 0 in layers) or (kind == "summary" and 1 in layers) or \
                     (kind == "hyperedge" and include_hyperedges)
            if wanted and ((not upsert_only) or prev.get(nid) != self._index_key(d)):
                todo.append(nid)
        if not todo:
            return
        texts, metas = zip(*[self._embedding_text(n) for n in todo])
        vectors = np.asarray(load_encoder(model_name).encode(list(texts), show_progress_bar=False,
                                                             normalize_embeddings=True), np.float32)
        store.upsert(todo, vectors, metas)
        store.save(model_name)
        # the resident HBM copy (shared by every graph object on this store) follows the same upsert
        # (changed rows only); after a reset it is reloaded from the rewritten store
        resident = self._indexes.get(os.path.abspath(db_path)) or _RESIDENT.get(self._resident_key(db_path))
        if resident is not None:
            if reset:
                resident.reload()
            else:
                resident.apply(todo, vectors, metas)
        new_meta = dict(prev)
        for nid in todo:
            new_meta[nid] = self._index_key(self.G.nodes[nid])
        self.G.graph["vector_index"] = {"db_path": db_path, "model": model_name,
                                        "indexed_nodes": len(new_meta), "indexed_meta": new_meta}
        self.G.graph["dirty"] = False

    # ---- device caches -----------------------------------------------------------------------
    def _graph_stamp(self) -> Tuple:
        return (id(self.G), len(self.G), self._version)

    def device_graph(self) -> DeviceGraph:
        stamp = self._graph_stamp()
        if self._dev_graph is None or self._dev_graph[0] != stamp:
            dev = torch.device("cuda", torch.cuda.current_device())
            # a graph unchanged since load() shares the device graph of every other load of the same
            # saved file (same content, same networkx order)
            shared = self._source is not None and self._version == 0 and len(self.G) == self._source[2]
            key = (self._source[:2], dev.index) if shared else None
            dg = _DEVICE_GRAPHS.get(key) if shared else None
            if dg is None:
                dg = DeviceGraph(self.G, dev)
                if shared:
                    _DEVICE_GRAPHS[key] = dg
            self._dev_graph = (stamp, dg)
            self._engines.clear()
        return self._dev_graph[1]

    def _resident_key(self, db_path: str) -> Tuple:
        return (os.path.abspath(db_path), os.environ.get("AHR_INDEX_DTYPE", "f32"), torch.cuda.current_device())

    def resident_index(self, db_path: str) -> ResidentIndex:
        """The store at db_path resident in HBM (one copy per store, storage type and GPU in the
        process, shared by every graph object); reloaded whole only when another writer changed the
        file (build_vector_index keeps it current incrementally)."""
        key = _abspath(db_path)
        res = self._indexes.get(key)
        if res is None:
            rkey = self._resident_key(key)
            res = _RESIDENT.get(rkey)
            if res is None:
                res = ResidentIndex(key, self.device_graph().device)
                _RESIDENT[rkey] = res
            self._indexes[key] = res
        if res.stamp != store_stamp(key):
            res.reload()
        return res

    def search_engine(self, db_path: str) -> SearchEngine:
        graph = self.device_graph()
        key = _abspath(db_path)
        res = self.resident_index(key)
        stamp = (res.version, graph.serial)
        hit = self._engines.get(key)
        if hit is None or hit[0] != stamp:
            self._engines[key] = (stamp, SearchEngine(res.index, res.ids, res.metas, graph))
        return self._engines[key][1]

    def _encoder(self, model_name: str):
        if self._query_embedder is None or self._query_embedder_name != model_name:
            self._query_embedder = load_encoder(model_name)
            self._query_embedder_name = model_name
        return self._query_embedder

    # ---- search (reference :675-789) ---------------------------------------------------------
    def search(self, query: str, top_k: int = 5, member_top_m: int = 5,
               alpha: Optional[float] = None, beta: Optional[float] = None, gamma: Optional[float] = None,
               delta: Optional[float] = None, judge_overall_min: Optional[float] = None,
               confidence_min: Optional[float] = None, type_filter: Optional[List[str]] = None,
               return_cluster: bool = False, db_path: Optional[str] = None,
               model_name: Optional[str] = None) -> Any:
        return self.search_batch([query], top_k, member_top_m, alpha, beta, gamma, delta, judge_overall_min,
                                 confidence_min, type_filter, return_cluster, db_path, model_name)[0]

    def search_batch(self, queries: Sequence[str], top_k: int = 5, member_top_m: int = 5,
                     alpha: Optional[float] = None, beta: Optional[float] = None, gamma: Optional[float] = None,
                     delta: Optional[float] = None, judge_overall_min: Optional[float] = None,
                     confidence_min: Optional[float] = None, type_filter: Optional[List[str]] = None,
                     return_cluster: bool = False, db_path: Optional[str] = None,
                     model_name: Optional[str] = None, query_vectors: Optional[np.ndarray] = None) -> List[Any]:
        """search() over many queries with one device pass (B = len(queries))."""
        def assemble(engine, params, rows, scores, res):
            return [self._assemble(engine, rows[b], scores[b], res, b, params.top_k, return_cluster)
                    for b in range(rows.shape[0])]

        return self._search_arrays(queries, top_k, member_top_m, alpha, beta, gamma, delta, judge_overall_min,
                                   confidence_min, type_filter, db_path, model_name, query_vectors, assemble)

    def search_arrays(self, queries: Sequence[str], top_k: int = 5, member_top_m: int = 5,
                      alpha: Optional[float] = None, beta: Optional[float] = None, gamma: Optional[float] = None,
                      delta: Optional[float] = None, judge_overall_min: Optional[float] = None,
                      confidence_min: Optional[float] = None, type_filter: Optional[List[str]] = None,
                      db_path: Optional[str] = None, model_name: Optional[str] = None,
                      query_vectors: Optional[np.ndarray] = None):
        """search_batch() before the result dicts: (engine, params, dense rows [B,k], dense scores
        [B,k], host RerankResult); _assemble(engine, rows[b], scores[b], res, b, ...) turns query b
        into search()'s return value. VecAHRAGGymEnv works on these arrays directly."""
        return self._search_arrays(queries, top_k, member_top_m, alpha, beta, gamma, delta, judge_overall_min,
                                   confidence_min, type_filter, db_path, model_name, query_vectors, None)

    def _search_arrays(self, queries, top_k, member_top_m, alpha, beta, gamma, delta, judge_overall_min,
                       confidence_min, type_filter, db_path, model_name, query_vectors, consume):
        """search_arrays(); with `consume`, its result goes to consume(engine, params, rows, scores,
        res) under the engine's lock instead, as views of the engine's result buffer (no copy: a
        small host batch's arrays are overwritten by the next call), and its return value is returned."""
        params = resolve_search_params(self.G.graph.get("search_params", {}), top_k, member_top_m, alpha, beta,
                                       gamma, delta, judge_overall_min, confidence_min, type_filter)
        vi = self.G.graph.get("vector_index") if isinstance(self.G.graph.get("vector_index"), dict) else {}
        db_path = db_path or vi.get("db_path", "vector_db")
        model_name = model_name or vi.get("model", DEFAULT_MODEL)
        engine = self.search_engine(db_path)
        # Chroma answers n_results > count with every row (:714); only a dense top-k that really
        # needs more than AHR_MAX_K_LARGE rows is out of this index's range
        if min(top_k, engine.n_rows) > nat.AHR_MAX_K_LARGE:
            raise ValueError(f"top_k={top_k} exceeds the dense index limit ({nat.AHR_MAX_K_LARGE})")
        if query_vectors is None:
            enc = self._encoder(model_name)
            # a GPU encoder hands its [B, d] fp32 output over on the device (no host round trip)
            extra = {"convert_to_tensor": True} if getattr(enc, "on_device", False) else {}
            query_vectors = enc.encode(list(queries), normalize_embeddings=True, **extra)
        if isinstance(query_vectors, torch.Tensor):
            q = query_vectors.to(torch.float32)
            if q.dim() == 1:
                q = q.unsqueeze(0)
        else:  # host vectors go to the engine as numpy (its one-call path stages them itself)
            q = np.asarray(query_vectors, np.float32)
            if q.ndim == 1:
                q = q.reshape(1, -1)
        if consume is None:
            rows, scores, res = engine.run(q, params)
            return engine, params, rows, scores, res
        with engine._lock:
            rows, scores, res = engine.run(q, params, borrow=True)
            return consume(engine, params, rows, scores, res)

    def _assemble(self, engine: SearchEngine, rows, scores, res, b: int, top_k: int, return_cluster: bool):
        n_nodes = engine.graph.n_nodes
        nodes = self.G.nodes
        reranked = []
        m = int(res.out_count[b]) if top_k > 0 else 0
        # one list conversion per array row (numpy scalar indexing per element is the slow part)
        out_nodes, out_sem, out_score = res.out_nodes[b, :m].tolist(), res.out_sem[b, :m].tolist(), \
            res.out_score[b, :m].tolist()
        for idx, sem, score in zip(out_nodes, out_sem, out_score):
            nid = engine.node_id(idx)
            d = nodes[nid] if nid in self.G else {}
            kind = d.get("node_type")
            reranked.append({"node_id": nid, "node_type": kind,
                             "layer": 0 if kind == "entity" else (1 if kind == "summary" else 0),
                             "semantic": sem, "judge_overall": parse_judge(d.get("judge_scores")),
                             "confidence": d.get("confidence"), "score": score,
                             "name": d.get("name"), "title": d.get("title")})
        if not return_cluster:
            return reranked
        seeds = []
        # Chroma's cosine distance of a hit is a float32 (hnswlib: 1 - <q, x> in single precision);
        # the reference turns it into semantic = 1.0 - float(dist) in double (:719-724)
        dists = (np.float32(1.0) - np.asarray(scores, np.float32)).tolist()
        for r, dist in zip(rows.tolist(), dists):
            if r < 0:
                continue
            seeds.append({"node_id": engine.row_ids[r], "semantic": 1.0 - float(dist), "meta": engine.row_metas[r]})
        expanded = []
        e = int(res.exp_count[b])
        for idx, src, sem in zip(res.exp_nodes[b, :e].tolist(), res.exp_src[b, :e].tolist(),
                                 res.exp_sem[b, :e].tolist()):
            nid = engine.node_id(idx)
            if src >= 0:
                kind = nodes[nid].get("node_type") if idx < n_nodes else None
                expanded.append({**seeds[src], "node_type": kind})
            else:
                assumed = nat.NODE_TYPE_NAMES[-1 - src]
                expanded.append({"node_id": nid, "semantic": sem,
                                 "meta": {"expanded": True}, "node_type": assumed})
        return {"seeds": seeds, "expanded": expanded, "reranked": reranked}
