"""GraphEnvironment — drop-in for reference src/ah_rag/agent/environment.py (class at :15).

Same constructor, actions, observation and info dicts. The differences are where the time goes:
  * neighbour expansions (expand_parents / expand_children / expand_related, reference :393-480)
    run as the batched HIP kernel ahr_graph_expand over the device CSR (B = 1 here;
    VecAHRAGGymEnv in ah_rag.agent.vec_env batches them across environments);
  * semantic_anchor goes through HierarchicalGraph.search (dense top-k + expansion + rerank on the
    GPU);
  * the node/edge counts every observation reports (reference :136-139, an O(N) networkx walk per
    step) are computed once per graph version;
  * expand_to_lca (reference :243-299, which rebuilds the belongs_to subgraph on every call) runs
    as ahr_graph_lca over the device CSR (visited set in LDS), and queries whose ancestor sets
    exceed that kernel's capacity as ahr_graph_lca_large (visited set in global memory).
"""
from __future__ import annotations

import json
import os
import time
import uuid
from collections import deque
from datetime import datetime
from typing import Any, Dict, List, Optional, Sequence, Set, Tuple

import networkx as nx
import numpy as np
import torch

from ..graph.hierarchical_graph import HierarchicalGraph
from ..graph_search import parse_judge, to_host_arrays

ADJ_BT_OUT, ADJ_BT_IN = 0, 1


class GraphEnvironment:
    """Action API over a HierarchicalGraph: reset, semantic_anchor, expansions, LCA, details,
    selection/frontier state, dynamic filters and weights, session logging."""

    def __init__(self, graph_dir: str = "graph", random_state: int = 42,
                 logging_enabled: bool = True, log_dir: str = "artifacts/phase2", session_id: Optional[str] = None,
                 debug: bool = False, log_level: str = "normal", redact: bool = True, *,
                 graph: Optional[HierarchicalGraph] = None) -> None:
        """`graph` (keyword-only, not in the reference) shares an already loaded graph, e.g. across
        the environments of a VecAHRAGGymEnv, instead of loading graph_dir again."""
        self.graph_dir = graph_dir
        self.random_state = random_state
        self.hg: Optional[HierarchicalGraph] = graph
        self.last_query: Optional[str] = None
        self.last_results: Optional[Dict[str, Any]] = None
        self.step_count = 0
        self.selection_set: Set[str] = set()
        self.frontier_set: Set[str] = set()
        self.current_filters: Dict[str, Any] = {"judge_overall_min": None, "confidence_min": None,
                                                "type_filter": None}
        self.current_weights: Dict[str, Any] = {"alpha": None, "beta": None, "gamma": None, "delta": None,
                                                "member_top_m": None, "top_k": 5}
        self.logging_enabled = logging_enabled
        self.log_dir = log_dir
        self.session_id = session_id or datetime.utcnow().strftime("%Y%m%dT%H%M%S") + "-" + uuid.uuid4().hex[:6]
        self.session_path = os.path.join(log_dir, self.session_id)
        self.debug = debug
        self.stats: Dict[str, Any] = {"actions": [], "cumulative": {"steps": 0, "queries": 0, "expansions": 0,
                                                                   "time_s": 0.0}}
        self.logger = None
        if logging_enabled:
            from ..utils.logging_init import get_logger
            self.logger = get_logger(self.session_path, self.session_id, level=log_level, redact=redact)
            try:
                with open(os.path.join(self.session_path, "session.json"), "w", encoding="utf-8") as f:
                    json.dump({"session_id": self.session_id, "created_at": datetime.utcnow().isoformat() + "Z"}, f)
            except Exception:
                pass
        self._count_cache: Optional[Tuple[Tuple, Dict[str, int]]] = None
        self._dag_cache: Optional[Tuple[Tuple, bool, Set[str]]] = None
        self._brief_cache: Dict[str, Dict[str, Any]] = {}
        self._brief_stamp: Optional[Tuple] = None
        self._ensure_graph_loaded()

    # ---- plumbing ----------------------------------------------------------------------------
    def _ensure_graph_loaded(self) -> None:
        if self.hg is None:
            # environments of one graph directory share the loaded graph and its device structures
            # (read-only here; HierarchicalGraph.load_shared, AHR_SHARE_GRAPH=0: a private load each)
            self.hg = HierarchicalGraph.load_shared(self.graph_dir)

    def _log(self, event: Dict[str, Any]) -> None:
        if self.logging_enabled and self.logger is not None:
            try:
                self.logger.info(**{**event, "step": self.step_count})
            except Exception:
                pass

    def _record(self, info: Dict[str, Any], expansion: bool = False, query_time: Optional[float] = None) -> None:
        self.stats["actions"].append(info)
        cum = self.stats["cumulative"]
        cum["steps"] += 1
        if expansion:
            cum["expansions"] += 1
        if query_time is not None:
            cum["queries"] += 1
            cum["time_s"] += query_time

    def _counts(self) -> Dict[str, int]:
        stamp = self.hg._graph_stamp()
        if self._count_cache is None or self._count_cache[0] != stamp:
            self._count_cache = (stamp, {"n_nodes": self.hg.G.number_of_nodes(),
                                         "n_edges": self.hg.G.number_of_edges()})
        return dict(self._count_cache[1])

    def _briefs(self) -> Dict[str, Dict[str, Any]]:
        """The node-brief cache of the current graph version (emptied when the graph's stamp — the
        one that invalidates the device graph — changes; attribute edits go through the graph's
        mutators, which bump it)."""
        stamp = self.hg._graph_stamp()
        if self._brief_stamp != stamp:
            self._brief_cache, self._brief_stamp = {}, stamp
        return self._brief_cache

    def _node_brief(self, node_id: str, cache: Optional[Dict[str, Dict[str, Any]]] = None) -> Dict[str, Any]:
        """The node's brief (reference :104-116) as a fresh dict; its static part built once per node
        and graph version (`cache`: the caller's _briefs(), fetched once per observation)."""
        if cache is None:
            cache = self._briefs()
        b = cache.get(node_id)
        if b is None:
            d = self.hg.G.nodes.get(node_id, {})
            kind = d.get("node_type")
            b = {"node_id": node_id, "node_type": kind, "entity_type": d.get("entity_type"),
                 "layer": 0 if kind == "entity" else (d.get("level") or (1 if kind == "summary" else 0)),
                 "title": d.get("title"), "name": d.get("name"),
                 "judge_overall": parse_judge(d.get("judge_scores")), "confidence": d.get("confidence")}
            cache[node_id] = b
        return dict(b)

    def _brief_scored(self, res: Dict[str, Any], cache: Optional[Dict[str, Dict[str, Any]]] = None) -> Dict[str, Any]:
        b = self._node_brief(res.get("node_id"), cache)
        b["score"] = res.get("score")
        b["semantic"] = res.get("semantic")
        return b

    def _observation(self, seeds: List[Dict[str, Any]], reranked: List[Dict[str, Any]]) -> Dict[str, Any]:
        return self._observation_of(seeds, reranked, self.selection_set, self.frontier_set, self.step_count)

    def _observation_of(self, seeds: List[Dict[str, Any]], reranked: List[Dict[str, Any]], selection_set,
                        frontier_set, step: int) -> Dict[str, Any]:
        """The observation dict (reference :118-150) for the given state; VecAHRAGGymEnv builds its
        environments' observations through this from their state snapshots."""
        cache = self._briefs()
        obs: Dict[str, Any] = {
            "selection": [self._brief_scored(x, cache) for x in reranked],
            "seeds": [self._brief_scored(x, cache) for x in seeds],
            "state": {"selection_ids": sorted(selection_set),
                      "frontier_ids": sorted(frontier_set)[:50]},
            "counts": self._counts(),
            "step": step,
        }
        if self.debug:
            obs["diagnostics"] = {"filters": self.current_filters, "weights": self.current_weights,
                                  "last_query": self.last_query, "frontier_size": len(self.frontier_set),
                                  "selection_size": len(self.selection_set)}
        return obs

    def _bare_observation(self, selection: List[Dict[str, Any]], step: Optional[int] = None) -> Dict[str, Any]:
        return {"selection": selection, "seeds": [], "counts": self._counts(),
                "step": self.step_count if step is None else step}

    # ---- core API ----------------------------------------------------------------------------
    def reset(self, seed_query: Optional[str] = None, top_k: int = 5) -> Tuple[Dict[str, Any], Dict[str, Any]]:
        self._ensure_graph_loaded()
        self.last_query = None
        self.last_results = None
        self.step_count = 0
        self.selection_set.clear()
        self.frontier_set.clear()
        if seed_query:
            return self.semantic_anchor(seed_query, top_k=top_k)
        self._log({"action": "reset", "message": "reset without seed_query"})
        return self._bare_observation([]), {"message": "reset without seed_query"}

    def _search_kwargs(self, top_k, member_top_m, judge_overall_min, confidence_min, type_filter):
        f, w = self.current_filters, self.current_weights
        return {"top_k": top_k, "member_top_m": member_top_m,
                "judge_overall_min": f.get("judge_overall_min") if judge_overall_min is None else judge_overall_min,
                "confidence_min": f.get("confidence_min") if confidence_min is None else confidence_min,
                "type_filter": f.get("type_filter") if type_filter is None else type_filter,
                "alpha": w.get("alpha"), "beta": w.get("beta"), "gamma": w.get("gamma"), "delta": w.get("delta")}

    def semantic_anchor(self, query: str, top_k: int = 5, member_top_m: int = 5,
                        judge_overall_min: Optional[float] = None, confidence_min: Optional[float] = None,
                        type_filter: Optional[List[str]] = None) -> Tuple[Dict[str, Any], Dict[str, Any]]:
        self._ensure_graph_loaded()
        self.step_count += 1
        self.last_query = query
        kw = self._search_kwargs(top_k, member_top_m, judge_overall_min, confidence_min, type_filter)
        t0 = time.perf_counter()
        cluster = self.hg.search(query=query, return_cluster=True, **kw)
        dur = time.perf_counter() - t0
        return self._anchor_result(query, top_k, cluster, dur)

    def _anchor_result(self, query: str, top_k: int, cluster: Dict[str, Any], dur: float):
        seeds = cluster.get("seeds", [])
        reranked = cluster.get("reranked", [])
        self.frontier_set = {x.get("node_id") for x in reranked if x.get("node_id")}
        obs = self._observation(seeds, reranked)
        info = {"action": "semantic_anchor", "query": query, "top_k": top_k, "returned": len(reranked),
                "time_s": round(dur, 4)}
        self.last_results = cluster
        self._log({**info, "filters": self.current_filters, "weights": self.current_weights})
        self._record(info, query_time=dur)
        return obs, info

    # ---- LCA over belongs_to (reference :243-299) ---------------------------------------------
    def _belongs_to_dag(self) -> Tuple[bool, Set[str]]:
        """(is_acyclic, nodes touching a belongs_to edge) — cached per graph version."""
        stamp = self.hg._graph_stamp()
        if self._dag_cache is None or self._dag_cache[0] != stamp:
            dg = self.hg.device_graph()
            n = dg.n_nodes
            out_off, out_tgt = dg._offsets[ADJ_BT_OUT], dg._targets[ADJ_BT_OUT]
            indeg = np.zeros(n, np.int64)
            members: Set[int] = set()
            for u in range(n):
                for v in out_tgt[out_off[u]:out_off[u + 1]]:
                    indeg[v] += 1
                    members.add(u)
                    members.add(int(v))
            # Kahn's algorithm restricted to nodes that carry a belongs_to edge
            queue = deque(u for u in members if indeg[u] == 0)
            seen = 0
            while queue:
                u = queue.popleft()
                seen += 1
                for v in out_tgt[out_off[u]:out_off[u + 1]]:
                    indeg[v] -= 1
                    if indeg[v] == 0:
                        queue.append(int(v))
            self._dag_cache = (stamp, seen == len(members), {dg.ids[i] for i in members})
        return self._dag_cache[1], self._dag_cache[2]

    def expand_to_lca(self, node_ids: List[str], max_results: int = 5) -> Tuple[Dict[str, Any], Dict[str, Any]]:
        self._ensure_graph_loaded()
        self.step_count += 1
        is_dag, dag_nodes = self._belongs_to_dag()
        for nid in node_ids:
            if nid not in dag_nodes:
                raise nx.NetworkXError(f"The node {nid} is not in the digraph.")
        lowest = lca_batch(self.hg, [node_ids])[0]  # ancestor sets + intersection on the device
        G = self.hg.G
        t0 = time.perf_counter()
        picked = sorted(lowest, key=lambda x: (G.nodes[x].get("level") or 1, x))[:max_results]
        obs = self._observation([{"node_id": n, "semantic": 0.0} for n in picked],
                                [{"node_id": n, "score": 0.0, "semantic": 0.0} for n in picked])
        info = {"action": "expand_to_lca", "inputs": node_ids, "lca_count": len(picked), "dag": is_dag,
                "time_s": round(time.perf_counter() - t0, 4)}
        self._log(info)
        self._record(info, expansion=True)
        return obs, info

    def query_node_details(self, node_id: str) -> Tuple[Dict[str, Any], Dict[str, Any]]:
        self._ensure_graph_loaded()
        self.step_count += 1
        if node_id not in self.hg.G:
            return self._bare_observation([]), {"error": "node_not_found", "node_id": node_id}
        info = {"action": "query_node_details", "node_id": node_id}
        self._log(info)
        self._record(info)
        return self._bare_observation([self._details(node_id)]), info

    def _details(self, node_id: str) -> Dict[str, Any]:
        """query_node_details' entry for a graph node (reference :301-325)."""
        d = self.hg.G.nodes[node_id]
        return {**self._node_brief(node_id), "title": d.get("title"), "name": d.get("name"),
                "summary_text": (d.get("summary_text") or d.get("summary") or "")[:500],
                "description": (d.get("description") or "")[:500],
                "top_words": d.get("top_words"), "members": d.get("members")}

    # ---- state & dynamic params --------------------------------------------------------------
    def commit_selection(self, node_ids: List[str]) -> Tuple[Dict[str, Any], Dict[str, Any]]:
        self._ensure_graph_loaded()
        self.step_count += 1
        added = []
        for nid in node_ids:
            if nid in self.hg.G and nid not in self.selection_set:
                self.selection_set.add(nid)
                added.append(nid)
                self.frontier_set.discard(nid)
        obs = self._observation([], [{"node_id": n, "score": 0.0, "semantic": 0.0} for n in added])
        info = {"action": "commit_selection", "added": added, "total_selection": len(self.selection_set)}
        self._log(info)
        self._record(info)
        return obs, info

    def set_filters(self, judge_overall_min: Optional[float] = None, confidence_min: Optional[float] = None,
                    type_filter: Optional[List[str]] = None) -> Dict[str, Any]:
        if judge_overall_min is not None:
            self.current_filters["judge_overall_min"] = judge_overall_min
        if confidence_min is not None:
            self.current_filters["confidence_min"] = confidence_min
        if type_filter is not None:
            self.current_filters["type_filter"] = list(type_filter)
        info = {"action": "set_filters", **self.current_filters}
        self._log(info)
        self.stats["actions"].append(info)
        return info

    def set_search_weights(self, alpha: Optional[float] = None, beta: Optional[float] = None,
                           gamma: Optional[float] = None, delta: Optional[float] = None,
                           member_top_m: Optional[int] = None, top_k: Optional[int] = None) -> Dict[str, Any]:
        for key, val in (("alpha", alpha), ("beta", beta), ("gamma", gamma), ("delta", delta),
                         ("member_top_m", member_top_m), ("top_k", top_k)):
            if val is not None:
                self.current_weights[key] = val
        info = {"action": "set_search_weights", **self.current_weights}
        self._log(info)
        self.stats["actions"].append(info)
        return info

    # ---- expansions (device kernel) ----------------------------------------------------------
    def _expand(self, action: str, node_ids: List[str], limit: int) -> Tuple[Dict[str, Any], Dict[str, Any]]:
        self._ensure_graph_loaded()
        ids = expand_batch(self.hg, action, [node_ids], limit)[0]
        return self._expand_finish(action, node_ids, ids)

    def _expand_finish(self, action: str, node_ids: List[str], ids: List[str]) -> Tuple[Dict[str, Any], Dict[str, Any]]:
        self.step_count += 1
        obs = self._observation([{"node_id": x, "semantic": 0.0} for x in ids],
                                [{"node_id": x, "score": 0.0, "semantic": 0.0} for x in ids])
        info = {"action": "expand_" + action, "inputs": node_ids, "returned": len(ids)}
        self.frontier_set.update(ids)
        self._log(info)
        self._record(info, expansion=True)
        return obs, info

    def expand_children(self, node_ids: List[str], limit: int = 10) -> Tuple[Dict[str, Any], Dict[str, Any]]:
        return self._expand("children", node_ids, limit)

    def expand_parents(self, node_ids: List[str], limit: int = 10) -> Tuple[Dict[str, Any], Dict[str, Any]]:
        return self._expand("parents", node_ids, limit)

    def expand_related(self, node_ids: List[str], limit: int = 10) -> Tuple[Dict[str, Any], Dict[str, Any]]:
        return self._expand("related", node_ids, limit)

    # ---- debug & episode end -----------------------------------------------------------------
    def set_debug(self, enabled: bool = True) -> Dict[str, Any]:
        self.debug = enabled
        info = {"action": "set_debug", "debug": self.debug}
        self._log(info)
        self.stats["actions"].append(info)
        return info

    def end_episode(self) -> Dict[str, Any]:
        summary = {"session_id": self.session_id, "created_at": datetime.utcnow().isoformat() + "Z",
                   "selection_size": len(self.selection_set), "frontier_size": len(self.frontier_set),
                   "stats": self.stats, "filters": self.current_filters, "weights": self.current_weights,
                   "last_query": self.last_query}
        try:
            with open(os.path.join(self.session_path, "summary.json"), "w", encoding="utf-8") as f:
                json.dump(summary, f, ensure_ascii=False, indent=2)
        except Exception:
            pass
        self._log({"action": "end_episode"})
        return summary


def lca_batch(hg: HierarchicalGraph, inputs: Sequence[Sequence[str]]) -> List[List[str]]:
    """Lowest common members of each input list on the belongs_to DAG, one ahr_graph_lca launch for
    the batch (environment.py:243-289 before the (level, id) sort). The ids must be DAG nodes."""
    dg = hg.device_graph()
    width = max(1, max((len(x) for x in inputs), default=1))
    idx = np.full((len(inputs), width), -1, np.int32)
    for b, ids in enumerate(inputs):
        if ids:
            idx[b, :len(ids)] = dg.node_indices(ids)
    out, cnt = dg.lca(torch.from_numpy(idx))
    out_h, cnt_h = to_host_arrays(out, cnt)
    res = [[dg.ids[i] for i in out_h[b, :cnt_h[b]]] if cnt_h[b] >= 0 else None for b in range(len(inputs))]
    over = np.nonzero(cnt_h < 0)[0]
    if len(over):
        # ancestor sets beyond the LDS kernel's capacity (4096 visited nodes, 1024 per level):
        # the global-memory form of the same walk answers those queries (ahr_graph_lca_large)
        out2, cnt2 = dg.lca_large(torch.from_numpy(idx[over]))
        out2_h, cnt2_h = to_host_arrays(out2, cnt2)
        for j, b in enumerate(over):
            if cnt2_h[j] < 0:
                raise RuntimeError("ahr_graph_lca_large reported an overflow with max_out = n_nodes")
            res[b] = [dg.ids[i] for i in out2_h[j, :cnt2_h[j]]]
    return res


def expand_batch(hg: HierarchicalGraph, action: str, inputs: Sequence[Sequence[str]], limit: int = 10
                 ) -> List[List[str]]:
    """One ahr_graph_expand launch for many environments: inputs[b] are env b's node ids."""
    dg = hg.device_graph()
    width = max(1, max((len(x) for x in inputs), default=1))
    if len(inputs) == 1:  # the single environment's call: one row, no per-row numpy writes
        get = dg.index.get
        row = [get(x, -1) for x in inputs[0]]
        idx = np.array([row + [-1] * (width - len(row))], np.int32)
    else:
        idx = np.full((len(inputs), width), -1, np.int32)
        for b, ids in enumerate(inputs):
            if ids:
                idx[b, :len(ids)] = dg.node_indices(ids)
    out_h, cnt_h = dg.expand_host(action, idx, limit)
    names = dg.ids
    return [[names[i] for i in out_h[b, :cnt_h[b]].tolist()] for b in range(len(inputs))]
