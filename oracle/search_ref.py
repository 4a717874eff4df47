"""Restatement of the reference's search tail, environment actions, featurizer and reward.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). Pinned by tests/golden/*.json, which were
produced by the reference's own code (tests/golden/make_golden.py).

Each function cites the reference lines it restates (paths relative to /root/reference):
  expand_rerank      src/ah_rag/graph/hierarchical_graph.py:719-789
  neighbors          src/ah_rag/graph/hierarchical_graph.py:441-462
  env_expand         src/ah_rag/agent/environment.py:393-480
  env_lca            src/ah_rag/agent/environment.py:243-299
  node_brief         src/ah_rag/agent/environment.py:92-116
  featurize          src/ah_rag/agent/featurizer.py:7-56
  step_reward        src/ah_rag/agent/reward.py:6-26
"""
from __future__ import annotations

import json
import math
import os
from typing import Any, Dict, List, Optional, Sequence, Tuple

import networkx as nx
import numpy as np

DEFAULT_PARAMS = {"alpha": 0.6, "beta": 0.2, "gamma": 0.1, "delta": 0.1, "judge_overall_min": None,
                  "confidence_min": None, "member_top_m": 5, "type_filter": None,
                  "layer_boost": {"entity": 0.0, "summary": 1.0, "hyperedge": 0.0}}


def load_graph(directory: str) -> Tuple[nx.DiGraph, Dict[str, Any]]:
    """structure.json (node-link, edges under "links") + meta.json, as hierarchical_graph.py:191-218."""
    with open(os.path.join(directory, "structure.json"), encoding="utf-8") as f:
        data = json.load(f)
    G = nx.node_link_graph(data, directed=True, edges="links")
    meta = {}
    mp = os.path.join(directory, "meta.json")
    if os.path.exists(mp):
        with open(mp, encoding="utf-8") as f:
            meta = json.load(f)
    return G, meta


def embedding_text(G: nx.DiGraph, nid: str) -> Tuple[str, Dict[str, Any]]:
    """Text and Chroma metadata of an indexed node (hierarchical_graph.py:558-600)."""
    d = G.nodes[nid]
    nt = d.get("node_type")
    if nt == "entity":
        text = f"Entity: {d.get('name') or ''}. {d.get('description') or ''}"
    elif nt == "summary":
        tw = d.get("top_words")
        try:
            words = (json.loads(tw) if isinstance(tw, str) else tw) if tw else []
        except Exception:
            words = []
        kw = ", ".join(words[:10]) if words else ""
        text = f"Summary: {d.get('title') or ''}. {d.get('summary_text') or d.get('summary') or ''}. Keywords: {kw}"
    else:
        text = f"Relation: {d.get('relation_type') or ''}. {d.get('description') or ''}"
    meta = {"node_id": nid, "node_type": nt, "layer": 0 if nt == "entity" else (1 if nt == "summary" else 0),
            "judge_overall": judge_of(d), "confidence": d.get("confidence")}
    return text, meta


def index_key(d: Dict[str, Any]) -> str:
    """Upsert key of a node (hierarchical_graph.py:622-625)."""
    import hashlib
    blob = (str(d.get("node_type")) + "|" + str(d.get("name") or d.get("title") or "") + "|"
            + str(d.get("summary_text") or "") + "|" + str(d.get("description") or ""))
    return hashlib.sha1(blob.encode("utf-8")).hexdigest()


def indexed_nodes(G: nx.DiGraph, layers=(0, 1), include_hyperedges: bool = False,
                  indexed_meta: Optional[Dict[str, str]] = None, upsert_only: bool = True) -> List[str]:
    """Node ids in the order build_vector_index upserts them (hierarchical_graph.py:627-649):
    with upsert_only, nodes whose key already matches the graph's indexed_meta are skipped."""
    prev = indexed_meta or {}
    out = []
    for nid, d in G.nodes(data=True):
        nt = d.get("node_type")
        if (nt == "entity" and 0 in layers) or (nt == "summary" and 1 in layers) or \
                (nt == "hyperedge" and include_hyperedges):
            if (not upsert_only) or prev.get(nid) != index_key(d):
                out.append(nid)
    return out


def judge_of(d: Dict[str, Any]) -> Optional[float]:
    raw = d.get("judge_scores")
    if not raw:
        return None
    try:
        js = json.loads(raw) if isinstance(raw, str) else raw
        return float(js.get("overall", 0.0))
    except Exception:
        return None


def neighbors(G: nx.DiGraph, node: str, direction: str, edge_type: str) -> List[str]:
    """Edge-type filtered neighbours in networkx adjacency order (hierarchical_graph.py:441-453)."""
    if direction == "out":
        return [v for _, v, a in G.out_edges(node, data=True) if a.get("edge_type") == edge_type]
    return [u for u, _, a in G.in_edges(node, data=True) if a.get("edge_type") == edge_type]


def resolve_params(meta_params: Dict[str, Any], **overrides) -> Dict[str, Any]:
    sp = {**DEFAULT_PARAMS, **(meta_params or {})}
    p = {}
    for key in ("alpha", "beta", "gamma", "delta"):
        p[key] = overrides.get(key) if overrides.get(key) is not None else sp.get(key)
    for key in ("judge_overall_min", "confidence_min"):
        p[key] = overrides.get(key) if overrides.get(key) is not None else sp.get(key)
    p["member_top_m"] = overrides.get("member_top_m") if overrides.get("member_top_m") is not None \
        else sp.get("member_top_m", 5)
    tf = overrides.get("type_filter")
    if tf is None:
        tf = sp.get("type_filter")
        if isinstance(tf, (set, tuple)):
            tf = list(tf)
    p["type_filter"] = tf
    p["layer_boost"] = sp.get("layer_boost", DEFAULT_PARAMS["layer_boost"])
    p["top_k"] = overrides.get("top_k", 5)
    return p


def expand_rerank(G: nx.DiGraph, seeds: List[Dict[str, Any]], p: Dict[str, Any], return_cluster: bool):
    """seeds: [{"node_id", "semantic", "meta"}] in rank order."""
    expanded: Dict[str, Dict[str, Any]] = {}
    for s in seeds:
        nid = s["node_id"]
        nt = G.nodes[nid].get("node_type") if nid in G else None
        expanded[nid] = {**s, "node_type": nt}
        if nt == "entity":
            for par in neighbors(G, nid, "out", "belongs_to")[:2]:
                if par not in expanded:
                    expanded[par] = {"node_id": par, "semantic": s["semantic"] * 0.9,
                                     "meta": {"expanded": True}, "node_type": "summary"}
        elif nt == "summary":
            for ch in neighbors(G, nid, "in", "belongs_to")[:p["member_top_m"]]:
                if ch not in expanded:
                    expanded[ch] = {"node_id": ch, "semantic": s["semantic"] * 0.85,
                                    "meta": {"expanded": True}, "node_type": "entity"}
    results = []
    boost = p["layer_boost"]
    for nid, info in expanded.items():
        d = G.nodes[nid] if nid in G else {}
        ntype = d.get("node_type")
        judge = judge_of(d)
        conf = d.get("confidence")
        if p["type_filter"] and ntype not in p["type_filter"]:
            continue
        if p["judge_overall_min"] is not None and (judge is None or judge < p["judge_overall_min"]):
            continue
        if p["confidence_min"] is not None and (conf is None or conf < p["confidence_min"]):
            continue
        sem = float(info.get("semantic", 0.0))
        jt = (1.0 / (1.0 + np.exp(-((judge or 0.0) / 10.0)))) if judge is not None else 0.0
        ct = float(conf) / 10.0 if conf is not None else 0.0
        score = p["alpha"] * sem + p["beta"] * jt + p["gamma"] * ct + p["delta"] * float(boost.get(ntype, 0.0))
        results.append({"node_id": nid, "node_type": ntype,
                        "layer": 0 if ntype == "entity" else (1 if ntype == "summary" else 0),
                        "semantic": round(sem, 4), "judge_overall": judge, "confidence": conf,
                        "score": round(float(score), 4), "name": d.get("name"), "title": d.get("title")})
    results.sort(key=lambda r: r["score"], reverse=True)
    top = results[:p["top_k"]]
    if return_cluster:
        return {"seeds": seeds, "expanded": list(expanded.values()), "reranked": top}
    return top


def env_expand(G: nx.DiGraph, action: str, node_ids: Sequence[str], limit: int = 10) -> List[str]:
    """expand_parents / expand_children / expand_related id lists (environment.py:393-480)."""
    raw: List[str] = []
    for nid in node_ids:
        if nid not in G:
            continue
        if action == "parents":
            raw += [v for v in G.successors(nid) if G.get_edge_data(nid, v).get("edge_type") == "belongs_to"]
        elif action == "children":
            raw += [u for u in G.predecessors(nid) if G.get_edge_data(u, nid).get("edge_type") == "belongs_to"]
        else:
            raw += [v for _, v, a in G.out_edges(nid, data=True) if a.get("edge_type") == "related_to"]
            raw += [u for u, _, a in G.in_edges(nid, data=True) if a.get("edge_type") == "related_to"]
            if G.nodes[nid].get("node_type") == "entity":
                for _, h, a in G.out_edges(nid, data=True):
                    if a.get("edge_type") == "participates_in":
                        raw.append(h)
                        raw += [u for u, _, b in G.in_edges(h, data=True)
                                if b.get("edge_type") == "participates_in" and u != nid]
        if len(raw) >= limit:
            break
    return list(dict.fromkeys(raw))[:limit]


def env_lca(G: nx.DiGraph, node_ids: Sequence[str], max_results: int = 5) -> Tuple[List[str], bool]:
    """Lowest common ancestors over belongs_to edges (environment.py:243-299)."""
    dag = nx.DiGraph()
    for u, v, a in G.edges(data=True):
        if a.get("edge_type") == "belongs_to":
            dag.add_edge(u, v)
    anc = [nx.ancestors(dag, n) | {n} for n in node_ids]
    inter = set.intersection(*anc) if anc else set()
    lcas = [n for n in inter if not (set(dag.successors(n)) & inter)]
    lcas = sorted(lcas, key=lambda x: (G.nodes[x].get("level") or 1, x))[:max_results]
    return lcas, nx.is_directed_acyclic_graph(dag)


def node_brief(G: nx.DiGraph, nid: str) -> Dict[str, Any]:
    d = G.nodes.get(nid, {})
    nt = d.get("node_type")
    return {"node_id": nid, "node_type": nt, "entity_type": d.get("entity_type"),
            "layer": 0 if nt == "entity" else (d.get("level") or (1 if nt == "summary" else 0)),
            "title": d.get("title"), "name": d.get("name"), "judge_overall": judge_of(d),
            "confidence": d.get("confidence")}


def featurize(obs: Dict[str, Any], k_nodes: int = 10) -> np.ndarray:
    """84-d float32 vector: 4 globals + k_nodes x 8 node features (featurizer.py:21-56)."""
    state = obs.get("state") or {}
    head = [float(obs.get("step") or 0), float(len(state.get("selection_ids") or [])),
            float(len(state.get("frontier_ids") or [])), float(len(obs.get("seeds") or []))]
    body = np.zeros((k_nodes, 8), np.float64)
    for i, n in enumerate((obs.get("selection") or [])[:k_nodes]):
        nt = str(n.get("node_type") or "")
        body[i] = [nt == "entity", nt == "summary", nt not in ("entity", "summary"),
                   float(n.get("layer") or 0), float(n.get("score") or 0.0), float(n.get("semantic") or 0.0),
                   float(n.get("judge_overall") or 0.0), float(n.get("confidence") or 0.0)]
    return np.asarray(head + body.ravel().tolist(), dtype=np.float32)


def step_reward(prev: Optional[Dict[str, Any]], cur: Dict[str, Any]) -> float:
    """+1 per new selection id, +0.05 per frontier growth (cap 10), -0.05 per step (reward.py:6-26)."""
    if prev is None:
        return 0.0
    ps, cs = prev.get("state") or {}, cur.get("state") or {}
    add_sel = len(set(cs.get("selection_ids") or []) - set(ps.get("selection_ids") or []))
    add_fr = max(0, len(set(cs.get("frontier_ids") or [])) - len(set(ps.get("frontier_ids") or [])))
    return float(1.0 * add_sel + 0.05 * min(add_fr, 10) - 0.05)


def py_round4(x: float) -> float:
    return round(x, 4)


def isclose_dicts(a, b, tol: float = 0.0, ignore=("updated_at",)) -> bool:
    """Structural equality with optional float tolerance (used by tests)."""
    if isinstance(a, dict) and isinstance(b, dict):
        ka = {k for k in a if k not in ignore}
        kb = {k for k in b if k not in ignore}
        return ka == kb and all(isclose_dicts(a[k], b[k], tol, ignore) for k in ka)
    if isinstance(a, (list, tuple)) and isinstance(b, (list, tuple)):
        return len(a) == len(b) and all(isclose_dicts(x, y, tol, ignore) for x, y in zip(a, b))
    if isinstance(a, float) or isinstance(b, float):
        if a is None or b is None:
            return a is b
        if isinstance(a, str) or isinstance(b, str):
            return a == b
        return a == b or (tol > 0 and math.isclose(float(a), float(b), abs_tol=tol))
    return a == b


class GymEpisode:
    """One AHRAGGymEnv episode restated on a networkx graph: the GraphEnvironment state (selection /
    frontier sets, step count), its observations and the gym's action dispatch, reward and done
    rule. Restates environment.py:118-150 (_observation), :155-241 (reset / semantic_anchor),
    :301-355 (query_node_details, commit_selection), :393-480 (expansions via env_expand) and
    gym_env.py:41-125 (reset, get_action_mask, _pick_top_ids, step). The dense search result is
    given to reset() as the search() cluster (expand_rerank of the oracle's dense top-k)."""

    TOP = {0: 2, 1: 2, 2: 1, 3: 3, 4: 1}
    EXPAND = {0: "parents", 1: "children", 2: "related"}

    def __init__(self, G: nx.DiGraph, max_steps: int = 6, repeat_penalty: float = 0.02,
                 counts_per_observation: bool = False) -> None:
        """counts_per_observation: recount the graph's nodes and edges for every observation, as the
        reference does (environment.py:136-139, an O(N) networkx walk per call; the host baseline of
        bench.py's C5 line times both forms); False: counted once (same values)."""
        self.G = G
        self._counts_once = {"n_nodes": G.number_of_nodes(), "n_edges": G.number_of_edges()}
        self.counts_per_observation = bool(counts_per_observation)
        self.max_steps = max(1, int(max_steps))
        self.repeat_penalty = float(repeat_penalty)

    @property
    def counts(self) -> Dict[str, int]:
        if self.counts_per_observation:
            return {"n_nodes": self.G.number_of_nodes(), "n_edges": self.G.number_of_edges()}
        return self._counts_once

    def _brief_scored(self, res: Dict[str, Any]) -> Dict[str, Any]:
        b = node_brief(self.G, res.get("node_id"))
        b.update({"score": res.get("score"), "semantic": res.get("semantic")})
        return b

    def _observation(self, seeds, reranked) -> Dict[str, Any]:
        return {"selection": [self._brief_scored(x) for x in reranked],
                "seeds": [self._brief_scored(x) for x in seeds],
                "state": {"selection_ids": sorted(self.selection), "frontier_ids": sorted(self.frontier)[:50]},
                "counts": dict(self.counts), "step": self.env_step}

    def mask(self) -> List[int]:
        if not (self.raw or {}).get("selection"):
            return [0, 0, 0, 0, 0, 1]
        return [1] * 6

    def reset(self, cluster: Dict[str, Any]) -> Tuple[np.ndarray, Dict[str, Any]]:
        self.selection, self.frontier = set(), set()
        self.env_step = 1  # reset -> semantic_anchor
        self.cur = 0
        self.last_action = None
        reranked = cluster.get("reranked", [])
        self.frontier = {x.get("node_id") for x in reranked if x.get("node_id")}
        self.raw = self._observation(cluster.get("seeds", []), reranked)
        return featurize(self.raw), self.raw

    def _top(self, k: int) -> List[str]:
        return [n["node_id"] for n in (self.raw.get("selection") or [])[:k] if n.get("node_id")]

    def step(self, action: int) -> Tuple[np.ndarray, float, bool, Dict[str, Any]]:
        self.cur += 1
        prev = self.raw
        done = False
        if action in self.EXPAND:
            self.env_step += 1
            ids = env_expand(self.G, self.EXPAND[action], self._top(self.TOP[action]), 10)
            obs = self._observation([{"node_id": n, "semantic": 0.0} for n in ids],
                                    [{"node_id": n, "score": 0.0, "semantic": 0.0} for n in ids])
            self.frontier.update(ids)
        elif action == 3:
            self.env_step += 1
            added = []
            for nid in self._top(3):
                if nid in self.G and nid not in self.selection:
                    self.selection.add(nid)
                    added.append(nid)
                    self.frontier.discard(nid)
            obs = self._observation([], [{"node_id": n, "score": 0.0, "semantic": 0.0} for n in added])
        elif action == 4:
            ids = self._top(1)
            if ids:
                self.env_step += 1
                d = self.G.nodes[ids[0]]
                details = {**node_brief(self.G, ids[0]), "title": d.get("title"), "name": d.get("name"),
                           "summary_text": (d.get("summary_text") or d.get("summary") or "")[:500],
                           "description": (d.get("description") or "")[:500],
                           "top_words": d.get("top_words"), "members": d.get("members")}
                obs = {"selection": [details], "seeds": [], "counts": dict(self.counts), "step": self.env_step}
            else:
                obs = prev
        else:
            done = True
            obs = prev
        r = 0.0 if done else step_reward(prev, obs)
        if not done and self.last_action is not None and action == self.last_action and self.repeat_penalty > 0:
            r -= self.repeat_penalty
        done = done or self.cur >= self.max_steps
        self.raw = obs
        self.last_action = action
        return featurize(obs), float(r), bool(done), obs
