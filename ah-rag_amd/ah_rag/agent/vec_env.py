"""Batched RL environment loop (SURVEY config C5: 2-hop expand + re-score inside the env loop).

The reference steps its PPO "vectorised" environments one after another
(src/ah_rag/agent/policy_ppo.py:145,163-214), each loading its own copy of the graph
(gym_env.py:27 -> environment.py:73-77) and paying an O(N) edge count per observation.
VecAHRAGGymEnv keeps N AHRAGGymEnv-equivalent environments over ONE device graph, and keeps
their state as arrays rather than N Python environment objects:
  reset(queries)  -> one batched search (dense top-k + expansion + rerank on the GPU, the result
                     arrays taken as they come back, no result dicts built);
  step(actions)   -> environments that chose the same expansion action share one
                     ahr_graph_expand launch on the node indices of their selections; commit /
                     details / end are array updates (plus one small set update per environment);
  observations    -> the 84-d featurizer vectors as one [N, 84] array from per-node feature
                     tables (built once per graph version) and the kernels' outputs.
The per-environment dicts the gym returns (info["raw_obs"], the search cluster) are built only
when a caller reads them (LazyInfos, EnvView), through GraphEnvironment's own dict builders and
from state snapshots taken at the step, so they are exactly what N AHRAGGymEnv objects stepped
one by one would return (tests/test_vec_env_gpu.py, tests/test_c5_env_gpu.py).
The per-action stats log of GraphEnvironment (stats["actions"]) is not kept here.
"""
from __future__ import annotations

from collections.abc import Sequence as _SequenceABC
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..graph.hierarchical_graph import HierarchicalGraph
from ..graph_search import parse_judge, to_host_arrays
from .environment import GraphEnvironment
from .featurizer import NODE_FEATS, featurize_observation
from .gym_env import END_EPISODE, N_ACTIONS, TOP_IDS

EXPAND_ACTIONS = {0: "parents", 1: "children", 2: "related"}
K_NODES = 10          # featurizer nodes (featurizer.py:21) = the widest selection (expansion limit 10)
VEC_DIM = 4 + NODE_FEATS * K_NODES
OBS_RESET, OBS_EXPAND, OBS_COMMIT, OBS_DETAILS = 0, 1, 2, 3
_EMPTY = frozenset()


class _NodeTable:
    """Featurizer inputs per node over the search engine's extended index (graph nodes 0..n-1 in
    networkx order, then n + r for a store row r whose id is not a graph node): is_entity,
    is_summary, is_other, layer, judge_overall, confidence, each as featurizer.node_row computes it
    from the node brief (environment.py _node_brief). A node whose attributes the featurizer
    cannot convert is flagged; an environment showing one is featurized from its dict instead (and
    raises as the reference would)."""

    def __init__(self, hg: HierarchicalGraph, engine) -> None:
        n = engine.graph.n_nodes
        m = n + len(engine.row_ids)
        feats = np.zeros((m, 6), np.float64)
        feats[:, 2] = 1.0  # an id unknown to the graph: node_type None -> "other", the rest 0
        bad = np.zeros(m, bool)
        for i, (_, d) in enumerate(hg.G.nodes(data=True)):  # DeviceGraph.ids order
            kind = d.get("node_type")
            k = str(kind or "")
            layer = 0 if kind == "entity" else (d.get("level") or (1 if kind == "summary" else 0))
            try:
                feats[i] = (k == "entity", k == "summary", k not in ("entity", "summary"), float(layer or 0.0),
                            float(parse_judge(d.get("judge_scores")) or 0.0), float(d.get("confidence") or 0.0))
            except (TypeError, ValueError):
                bad[i] = True
        self.feats, self.bad, self.n = feats, bad, n


class _ObsBatch:
    """One observation per environment as arrays (what one reset or step produced). Selections
    hold extended node indices (-1 past sel_n); S / F are the selection / frontier sets at the
    observation (immutable: the environment replaces, never mutates, a set it changes); alias[e] =
    (batch, index) where the gym returned the previous observation object itself."""

    def __init__(self, E: int) -> None:
        self.kind = np.zeros(E, np.int8)
        self.step = np.zeros(E, np.int64)
        self.sel = np.full((E, K_NODES), -1, np.int64)
        self.sel_n = np.zeros(E, np.int64)
        self.score = np.zeros((E, K_NODES), np.float64)
        self.sem = np.zeros((E, K_NODES), np.float64)
        self.seed_n = np.zeros(E, np.int64)
        self.s_size = np.zeros(E, np.int64)
        self.f_size = np.zeros(E, np.int64)
        self.S: List[frozenset] = [_EMPTY] * E
        self.F: List[Any] = [_EMPTY] * E
        self.alias: Optional[List[Optional[Tuple["_ObsBatch", int]]]] = None
        self.cache: Dict[int, Dict[str, Any]] = {}
        self.search = None  # reset: (engine, params, rows, scores, res, seed_idx, seed_sem, seed_n)
        self.stamp = None   # the graph version the observation was taken on (HierarchicalGraph._graph_stamp)

    def copy_rows(self, src: "_ObsBatch", idx: Optional[np.ndarray] = None) -> None:
        """src's rows idx into this batch (idx None: every row)."""
        if idx is None:
            for name in ("kind", "step", "sel", "sel_n", "score", "sem", "seed_n", "s_size", "f_size"):
                getattr(self, name)[:] = getattr(src, name)
            self.S, self.F = list(src.S), list(src.F)
            return
        for name in ("kind", "step", "sel", "sel_n", "score", "sem", "seed_n", "s_size", "f_size"):
            getattr(self, name)[idx] = getattr(src, name)[idx]
        for e in idx.tolist():
            self.S[e], self.F[e] = src.S[e], src.F[e]


class LazyInfos(_SequenceABC):
    """The gym info dicts of a batch, built on first access (then cached)."""

    def __init__(self, n: int, make: Callable[[int], Dict[str, Any]]) -> None:
        self._n, self._make, self._cache = n, make, {}

    def __len__(self) -> int:
        return self._n

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(self._n))]
        if i < 0:
            i += self._n
        if not 0 <= i < self._n:
            raise IndexError(i)
        d = self._cache.get(i)
        if d is None:
            d = self._cache[i] = self._make(i)
        return d


class _GraphEnvView:
    """GraphEnvironment-shaped read access to one environment of the batch."""

    def __init__(self, venv: "VecAHRAGGymEnv", e: int) -> None:
        self._v, self._e = venv, e

    @property
    def last_results(self):
        return self._v._cluster(self._e)

    @property
    def last_query(self):
        return self._v._queries[self._e] if self._v._queries else None

    @property
    def step_count(self) -> int:
        return int(self._v._steps[self._e])

    def end_episode(self, *_, **__):
        raise NotImplementedError("VecAHRAGGymEnv keeps no per-environment GraphEnvironment: step the environment "
                                  "with action 5 (end_episode) instead")

    @property
    def stats(self):
        raise NotImplementedError("VecAHRAGGymEnv does not keep GraphEnvironment's per-action stats log")

    @property
    def session_path(self):
        raise NotImplementedError("VecAHRAGGymEnv writes no per-environment session log")

    @property
    def selection_set(self) -> set:
        return {self._v._id(i) for i in self._v._S[self._e]}

    @property
    def frontier_set(self) -> set:
        return {self._v._id(i) for i in self._v._F[self._e]}


class EnvView:
    """AHRAGGymEnv-shaped read access to environment e (get_action_mask, the last observation)."""

    def __init__(self, venv: "VecAHRAGGymEnv", e: int) -> None:
        self._v, self._e = venv, e
        self.env = _GraphEnvView(venv, e)

    @property
    def action_size(self) -> int:
        return N_ACTIONS

    def get_action_mask(self) -> List[int]:
        ob = self._v._obs
        return [0] * (N_ACTIONS - 1) + [1] if ob is None else self._v._mask_list(ob, self._e)

    @property
    def _last_raw_obs(self):
        ob = self._v._obs
        return None if ob is None else self._v._obs_dict(ob, self._e)


class VecAHRAGGymEnv:
    def __init__(self, graph_dir: str = "graph", n_envs: int = 8, max_steps: int = 6,
                 enable_action_mask: bool = True, repeat_penalty: float = 0.02,
                 graph: Optional[HierarchicalGraph] = None) -> None:
        self.hg = graph or HierarchicalGraph.load(graph_dir)
        self.max_steps = max(1, int(max_steps))
        self.enable_action_mask = bool(enable_action_mask)
        self.repeat_penalty = float(repeat_penalty)
        E = int(n_envs)
        # the dict builders (briefs, observation / details layout, counts) of one shared environment
        self._genv = GraphEnvironment(graph_dir=graph_dir, log_level="off", logging_enabled=False, graph=self.hg)
        self._steps = np.zeros(E, np.int64)         # GraphEnvironment.step_count
        self._cur = np.zeros(E, np.int64)           # AHRAGGymEnv._cur_step
        self._last_action = np.full(E, -1, np.int64)
        self._S: List[Any] = [_EMPTY] * E           # selection sets (extended node indices)
        self._F: List[Any] = [_EMPTY] * E           # frontier sets
        self._obs: Optional[_ObsBatch] = None
        self._reset_batch: Optional[_ObsBatch] = None
        self._queries: Optional[List[str]] = None
        self._engine = None
        self._table: Optional[Tuple[Any, _NodeTable]] = None
        self.envs = [EnvView(self, e) for e in range(E)]

    @property
    def n_envs(self) -> int:
        return len(self.envs)

    # ---- helpers -------------------------------------------------------------------------------
    def _id(self, idx: int) -> str:
        return self._engine.node_id(int(idx))

    def _node_table(self) -> _NodeTable:
        key = (id(self._engine), self.hg._graph_stamp())
        if self._table is None or self._table[0] != key:
            self._table = (key, _NodeTable(self.hg, self._engine))
        return self._table[1]

    def action_masks(self) -> np.ndarray:
        """[N, 6] int64: every action where the observation has a selection, else end_episode only
        (gym_env.py:54-75)."""
        m = np.zeros((self.n_envs, N_ACTIONS), np.int64)
        if self._obs is None:
            m[:, END_EPISODE] = 1
            return m
        m[self._obs.sel_n > 0] = 1
        m[:, END_EPISODE] = 1
        return m

    def _featurize(self, ob: _ObsBatch) -> np.ndarray:
        """featurize_observation for every environment at once (featurizer.py:21-56)."""
        tab = self._node_table()
        E = self.n_envs
        vec = np.zeros((E, VEC_DIM), np.float64)
        full = ob.kind != OBS_DETAILS  # a details observation has no "state" and no seeds
        vec[:, 0] = ob.step
        vec[:, 1] = np.where(full, ob.s_size, 0)
        vec[:, 2] = np.where(full, np.minimum(ob.f_size, 50), 0)
        vec[:, 3] = ob.seed_n
        valid = np.arange(K_NODES)[None, :] < ob.sel_n[:, None]
        f = tab.feats[np.where(valid, ob.sel, 0)]
        body = vec[:, 4:].reshape(E, K_NODES, NODE_FEATS)
        body[..., 0:4] = f[..., 0:4]
        body[..., 4] = ob.score
        body[..., 5] = ob.sem
        body[..., 6:8] = f[..., 4:6]
        body[~valid] = 0.0
        out = vec.astype(np.float32)
        bad = (tab.bad[np.where(valid, ob.sel, 0)] & valid).any(axis=1)
        for e in np.flatnonzero(bad).tolist():  # unconvertible attributes: the reference's path (raises)
            out[e] = featurize_observation(self._obs_dict(ob, e), K_NODES)[0]
        return out

    # ---- lazily built dicts --------------------------------------------------------------------
    def _check_stamp(self, ob: _ObsBatch) -> None:
        """A dict is built on first access from the live graph's attributes; if the graph changed
        since the step that produced the observation, it would mix two graph versions, so refuse."""
        if ob.stamp is not None and ob.stamp != self.hg._graph_stamp():
            raise RuntimeError("the graph changed after this observation was taken: its info dicts can no longer be "
                               "built as the step would have returned them (read info[i] before mutating the graph)")

    def _briefs(self, idx: np.ndarray, n: int, score, sem) -> List[Dict[str, Any]]:
        ids = [self._id(i) for i in idx[:n].tolist()]
        sc = [score] * n if not isinstance(score, np.ndarray) else score[:n].tolist()
        sm = [sem] * n if not isinstance(sem, np.ndarray) else sem[:n].tolist()
        return [{"node_id": i, "score": a, "semantic": b} for i, a, b in zip(ids, sc, sm)]

    def _obs_dict(self, ob: _ObsBatch, e: int) -> Dict[str, Any]:
        if ob.alias is not None and ob.alias[e] is not None:
            src, se = ob.alias[e]
            return self._obs_dict(src, se)
        d = ob.cache.get(e)
        if d is not None:
            return d
        self._check_stamp(ob)
        g = self._genv
        kind, n, step = int(ob.kind[e]), int(ob.sel_n[e]), int(ob.step[e])
        if kind == OBS_DETAILS:
            d = g._bare_observation([g._details(self._id(ob.sel[e, 0]))] if n else [], step=step)
        else:
            S = {self._id(i) for i in ob.S[e]}
            F = {self._id(i) for i in ob.F[e]}
            if kind == OBS_RESET:
                _, _, _, _, _, seed_idx, seed_sem, seed_n = ob.search
                seeds = self._briefs(seed_idx[e], int(seed_n[e]), None, seed_sem[e])
                sel = self._briefs(ob.sel[e], n, ob.score[e], ob.sem[e])
            elif kind == OBS_EXPAND:
                seeds = self._briefs(ob.sel[e], n, None, 0.0)
                sel = self._briefs(ob.sel[e], n, 0.0, 0.0)
            else:  # OBS_COMMIT
                seeds = []
                sel = self._briefs(ob.sel[e], n, 0.0, 0.0)
            d = g._observation_of(seeds, sel, S, F, step)
        ob.cache[e] = d
        return d

    def _cluster(self, e: int):
        """search()'s return_cluster dict of environment e's last reset (GraphEnvironment.last_results)."""
        ob = self._reset_batch
        if ob is None:
            return None
        key = ("cluster", e)
        c = ob.cache.get(key)
        if c is None:
            self._check_stamp(ob)
            engine, params, rows, scores, res = ob.search[:5]
            c = ob.cache[key] = self.hg._assemble(engine, rows[e], scores[e], res, e, params.top_k, True)
        return c

    def _aux(self, ob: _ObsBatch, e: int) -> Dict[str, Any]:
        return {"top_node_ids": [str(n.get("node_id")) for n in self._obs_dict(ob, e).get("selection")[:K_NODES]]}

    def _mask_list(self, ob: _ObsBatch, e: int) -> List[int]:
        return [1] * N_ACTIONS if ob.sel_n[e] > 0 else [0] * (N_ACTIONS - 1) + [1]

    # ---- the gym API, batched ------------------------------------------------------------------
    def reset(self, queries: Sequence[str], query_vectors: Optional[np.ndarray] = None
              ) -> Tuple[np.ndarray, LazyInfos]:
        E = self.n_envs
        if len(queries) != E:
            raise ValueError("one query per environment")
        # AHRAGGymEnv.reset -> GraphEnvironment.reset -> semantic_anchor(top_k=5) (environment.py:155-241)
        engine, params, rows, scores, res = self.hg.search_arrays(list(queries), top_k=5, member_top_m=5,
                                                                  query_vectors=query_vectors)
        self._engine = engine
        self._queries = list(queries)
        n_out = np.minimum(res.out_count.astype(np.int64), K_NODES)
        ob = _ObsBatch(E)
        ob.kind[:] = OBS_RESET
        self._steps[:] = 1
        ob.step[:] = 1
        w = min(res.out_nodes.shape[1], K_NODES)
        ob.sel[:, :w] = res.out_nodes[:, :w]
        ob.sel_n[:] = n_out
        ob.score[:, :w] = res.out_score[:, :w]
        ob.sem[:, :w] = res.out_sem[:, :w]
        ob.sel[np.arange(K_NODES)[None, :] >= n_out[:, None]] = -1
        # the dense hits (Chroma's float32 distance -> 1 - dist in double, hierarchical_graph.py:719-724)
        valid = rows >= 0
        seed_n = valid.sum(axis=1).astype(np.int64)
        seed_idx = np.where(valid, engine.row_to_node_host[np.maximum(rows, 0)], -1).astype(np.int64)
        seed_sem = 1.0 - (np.float32(1.0) - np.asarray(scores, np.float32)).astype(np.float64)
        ob.seed_n[:] = seed_n
        ob.search = (engine, params, rows, scores, res, seed_idx, seed_sem, seed_n)
        ob.stamp = self.hg._graph_stamp()
        # selection cleared; frontier = the reranked nodes
        self._S = [_EMPTY] * E
        self._F = [frozenset(r[:c]) for r, c in zip(ob.sel.tolist(), n_out.tolist())]
        ob.S = list(self._S)
        ob.F = list(self._F)
        ob.f_size[:] = [len(f) for f in self._F]
        self._cur[:] = 0
        self._last_action[:] = -1
        self._obs = self._reset_batch = ob
        vecs = self._featurize(ob)

        def info(e: int) -> Dict[str, Any]:
            d: Dict[str, Any] = {"raw_obs": self._obs_dict(ob, e), "aux": self._aux(ob, e)}
            if self.enable_action_mask:
                d["action_mask"] = self._mask_list(ob, e)
            return d
        return vecs, LazyInfos(E, info)

    def step(self, actions: Sequence[int]) -> Tuple[np.ndarray, np.ndarray, np.ndarray, LazyInfos]:
        prev = self._obs
        if prev is None:
            raise AssertionError("Call reset() first")
        E = self.n_envs
        a = np.asarray([int(x) for x in actions], np.int64)
        if a.shape != (E,):
            raise ValueError("one action per environment")
        self._cur += 1
        n_graph = self._engine.graph.n_nodes
        ob = _ObsBatch(E)
        ob.copy_rows(prev)  # the defaults: unchanged (aliased) observations
        ob.alias = [None] * E
        ob.search = prev.search
        ob.stamp = self.hg._graph_stamp()
        pos = np.arange(K_NODES)[None, :]
        top_valid = pos < prev.sel_n[:, None]

        # expansions (environment.py:393-480): one ahr_graph_expand launch per action kind, all
        # enqueued before one host copy (one stream sync per step, not one per kind)
        launched = []
        for act, name in EXPAND_ACTIONS.items():
            g = np.flatnonzero(a == act)
            if not len(g):
                continue
            t = TOP_IDS[act]
            inp = np.where(top_valid[g, :t] & (prev.sel[g, :t] < n_graph), prev.sel[g, :t], -1)
            launched.append((g, *self._engine.graph.expand(name, torch.from_numpy(inp.astype(np.int32)), K_NODES)))
        host = to_host_arrays(*[x for _, out, cnt in launched for x in (out, cnt)])
        for i, (g, _, _) in enumerate(launched):
            out_h, cnt_h = host[2 * i].astype(np.int64), host[2 * i + 1].astype(np.int64)
            self._steps[g] += 1
            ob.kind[g] = OBS_EXPAND
            ob.step[g] = self._steps[g]
            ob.sel[g] = np.where(pos < cnt_h[:, None], out_h[:, :K_NODES], -1)
            ob.sel_n[g] = cnt_h
            ob.score[g] = 0.0
            ob.sem[g] = 0.0
            ob.seed_n[g] = cnt_h
            # the observation shows the frontier before this expansion's ids join it (:292-300)
            for e, row, c in zip(g.tolist(), out_h.tolist(), cnt_h.tolist()):
                F = self._F[e]
                ob.S[e], ob.F[e] = self._S[e], F
                ob.s_size[e], ob.f_size[e] = len(self._S[e]), len(F)
                if c:
                    self._F[e] = F.union(row[:c])

        # commit_selection of the top 3 (environment.py:327-341)
        for e in np.flatnonzero(a == 3).tolist():
            S, F = self._S[e], self._F[e]
            added = []
            for x in prev.sel[e, :min(3, int(prev.sel_n[e]))].tolist():
                if x < n_graph and x not in S:
                    if not added:
                        S, F = set(S), set(F)
                    S.add(x)
                    added.append(x)
                    F.discard(x)
            self._S[e], self._F[e] = S, F
            self._steps[e] += 1
            ob.kind[e] = OBS_COMMIT
            ob.step[e] = self._steps[e]
            ob.sel[e] = -1
            ob.sel[e, :len(added)] = added
            ob.sel_n[e] = len(added)
            ob.score[e] = 0.0
            ob.sem[e] = 0.0
            ob.seed_n[e] = 0
            ob.S[e], ob.F[e] = S, F
            ob.s_size[e], ob.f_size[e] = len(S), len(F)

        # query_node_details of the top 1 (environment.py:301-325); none: the previous observation
        det = np.flatnonzero((a == 4) & (prev.sel_n > 0))
        if len(det):
            node = prev.sel[det, 0]
            in_g = node < n_graph
            self._steps[det] += 1
            ob.kind[det] = OBS_DETAILS
            ob.step[det] = self._steps[det]
            ob.sel[det] = -1
            ob.sel[det, 0] = np.where(in_g, node, -1)
            ob.sel_n[det] = in_g.astype(np.int64)
            ob.score[det] = 0.0
            ob.sem[det] = 0.0
            ob.seed_n[det] = 0
        # end_episode, and any action past the five (gym_env.py _apply's last branch): done, same observation
        ends = (a < 0) | (a > 4)
        for e in np.flatnonzero(((a == 4) & (prev.sel_n == 0)) | ends).tolist():
            ob.alias[e] = prev.alias[e] if prev.alias is not None and prev.alias[e] is not None else (prev, e)

        # rewards (reward.py:6-26 on the raw observations; a details observation has no "state")
        pf, cf = prev.kind != OBS_DETAILS, ob.kind != OBS_DETAILS
        add_sel = np.where(cf, ob.s_size - np.where(pf, prev.s_size, 0), 0)
        add_fr = np.maximum(0, np.where(cf, np.minimum(ob.f_size, 50), 0) - np.where(pf, np.minimum(prev.f_size, 50), 0))
        r = 1.0 * add_sel + 0.05 * np.minimum(add_fr, 10) - 0.05
        done = ends
        r[done] = 0.0
        rep = (~done) & (self._last_action == a) & (self._last_action >= 0)
        if self.repeat_penalty > 0:
            r[rep] -= self.repeat_penalty
        done = done | (self._cur >= self.max_steps)
        self._last_action = a
        self._obs = ob
        vecs = self._featurize(ob)
        cur = self._cur.copy()

        def info(e: int) -> Dict[str, Any]:
            d: Dict[str, Any] = {"action": int(a[e])}
            if self.enable_action_mask:
                d["action_mask"] = self._mask_list(ob, e)
            d.update({"raw_obs": self._obs_dict(ob, e), "aux": self._aux(ob, e), "step": int(cur[e])})
            return d
        return vecs, r.astype(np.float32), done, LazyInfos(E, info)
