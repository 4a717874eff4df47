"""Batched RL environment loop (SURVEY config C5: 2-hop expand + re-score inside the env loop).

The reference steps its PPO "vectorised" environments one after another
(src/ah_rag/agent/policy_ppo.py:145,163-214), each loading its own copy of the graph
(gym_env.py:27 -> environment.py:73-77) and paying an O(N) edge count per observation.
VecAHRAGGymEnv keeps N AHRAGGymEnv-equivalent environments over ONE device graph, and keeps
their state as arrays rather than N Python environment objects:
  reset(queries)  -> one batched search (dense top-k + expansion + rerank on the GPU, the result
                     arrays taken as they come back, no result dicts built);
  step(actions)   -> one ahr_graph_env_step launch for every environment: expansions, commits,
                     details and the selection / frontier sets, which live in device memory as
                     per-environment slot arrays; the state comes back in one copy and is the
                     step's snapshot (no per-environment Python on the step path);
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
        self.has_bad = bool(bad.any())  # (none: the steps skip the per-environment check)


class _ObsBatch:
    """One observation per environment as arrays (what one reset or step produced). Selections
    hold extended node indices (-1 past sel_n); the selection / frontier sets the observations show
    are rows of the state snapshot taken at the step (S_snap / F_snap); alias[e]: the gym returned
    the previous observation object itself (prev's own e-th one)."""

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
        # the selection / frontier the observation shows: rows of a state snapshot (the host copy
        # of the device state after this step; -1 = a removed frontier slot), S row[:s_size], F
        # row[:f_shown]
        self.S_snap: Optional[np.ndarray] = None
        self.F_snap: Optional[np.ndarray] = None
        self.f_shown = np.zeros(E, np.int64)
        # alias[e]: environment e's observation is the previous batch's (self.prev) own e-th one
        self.alias: Optional[np.ndarray] = None
        self.prev: Optional["_ObsBatch"] = None
        self.cache: Dict[int, Dict[str, Any]] = {}
        self.search = None  # reset: (engine, params, rows, scores, res, seed_idx, seed_sem, seed_n)
        self.stamp = None   # the graph version the observation was taken on (HierarchicalGraph._graph_stamp)

    _ROWS = ("kind", "step", "sel", "sel_n", "score", "sem", "seed_n", "s_size", "f_size", "f_shown")

    def copy_rows(self, src: "_ObsBatch") -> None:
        """src's rows into this batch (the defaults of a step: unchanged observations)."""
        for name in self._ROWS:
            getattr(self, name)[:] = getattr(src, name)

    @classmethod
    def following(cls, prev: "_ObsBatch") -> "_ObsBatch":
        """A new batch holding copies of prev's rows (= cls(E) + copy_rows(prev), one pass)."""
        ob = cls.__new__(cls)
        for name in cls._ROWS:
            setattr(ob, name, getattr(prev, name).copy())
        ob.S_snap = ob.F_snap = ob.alias = ob.prev = ob.search = ob.stamp = None
        ob.cache = {}
        return ob


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
        return {self._v._id(i) for i in self._v._state_rows("S", self._e)}

    @property
    def frontier_set(self) -> set:
        return {self._v._id(i) for i in self._v._state_rows("F", self._e)}


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
        # the environments' selection / frontier sets live in device memory (ahr_graph_env_step:
        # append-only slot arrays per environment, sized for max_steps steps after a reset and grown
        # if an environment is stepped further); self._st is the host mirror after the last step
        self._bufs = None
        self._st: Optional[np.ndarray] = None
        self._offs: Optional[List[int]] = None
        self._layout: Dict[str, Tuple[int, int]] = {}
        self._fcap = self._scap = 0
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

    # ---- device state ---------------------------------------------------------------------------
    def _part(self, st: np.ndarray, name: str) -> np.ndarray:
        """A part of an environment-state buffer (DeviceGraph.ENV_PARTS) as a numpy view."""
        o, size = self._layout[name]
        v = st[o:o + size]
        if name == "vec":
            return v.view(np.float32).reshape(self.n_envs, VEC_DIM)
        return v.reshape(self.n_envs, -1) if name in ("sel", "F", "S") else v

    def _state_rows(self, which: str, e: int) -> List[int]:
        """Environment e's current selection (S) or frontier (F) members, extended node indices."""
        if self._st is None:
            return []
        if which == "S":
            return self._part(self._st, "S")[e, :int(self._part(self._st, "S_n")[e])].tolist()
        row = self._part(self._st, "F")[e, :int(self._part(self._st, "F_end")[e])]
        return row[row >= 0].tolist()

    def _alloc_state(self, fcap: int, scap: int) -> None:
        g = self._engine.graph
        self._fcap, self._scap = fcap, scap
        self._bufs, self._st, self._offs = g.env_buffers(self.n_envs, K_NODES, fcap, scap)
        # (offset, int32 element count) of every part, resolved once per layout
        from ..graph_search import DeviceGraph
        E = self.n_envs
        sizes = {"sel": E * K_NODES, "F": E * fcap, "S": E * scap, "vec": E * VEC_DIM, "err": 1}
        self._layout = {name: (self._offs[i], sizes.get(name, E)) for i, name in enumerate(DeviceGraph.ENV_PARTS)}

    def _grow_state(self) -> None:
        """Double the frontier / selection capacity, keeping the state (an environment stepped far
        beyond max_steps without a reset)."""
        old, ofc, osc = self._st.copy(), self._fcap, self._scap
        prev_offs = self._offs
        self._alloc_state(ofc * 2, osc * 2)
        from ..graph_search import DeviceGraph
        E, K = self.n_envs, K_NODES
        for i, name in enumerate(DeviceGraph.ENV_PARTS):
            o = prev_offs[i]
            if name == "F":
                self._part(self._st, "F")[:] = -1
                self._part(self._st, "F")[:, :ofc] = old[o:o + E * ofc].reshape(E, ofc)
            elif name == "S":
                self._part(self._st, "S")[:] = -1
                self._part(self._st, "S")[:, :osc] = old[o:o + E * osc].reshape(E, osc)
            elif name == "sel":
                self._part(self._st, "sel")[:] = old[o:o + E * K].reshape(E, K)
            elif name == "vec":
                self._part(self._st, "vec")[:] = old[o:o + E * VEC_DIM].view(np.float32).reshape(E, VEC_DIM)
            elif name != "err":
                self._part(self._st, name)[:] = old[o:o + E]
        self._engine.graph.env_upload(self._bufs, self._st)

    def _node_table(self) -> _NodeTable:
        key = (id(self._engine), self.hg._graph_stamp())
        if self._table is None or self._table[0] != key:
            tab = _NodeTable(self.hg, self._engine)
            tab.dev = self._engine.graph.env_node_table(tab.feats)  # the step kernel's copy
            self._table = (key, tab)
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
        sel0 = np.where(valid, ob.sel, 0)
        f = tab.feats[sel0]
        body = vec[:, 4:].reshape(E, K_NODES, NODE_FEATS)
        body[..., 0:4] = f[..., 0:4]
        body[..., 4] = ob.score
        body[..., 5] = ob.sem
        body[..., 6:8] = f[..., 4:6]
        body[~valid] = 0.0
        out = vec.astype(np.float32)
        if tab.has_bad:
            bad = (tab.bad[sel0] & valid).any(axis=1)
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
        while ob.alias is not None and ob.alias[e]:
            ob = ob.prev
        d = ob.cache.get(e)
        if d is not None:
            return d
        self._check_stamp(ob)
        g = self._genv
        kind, n, step = int(ob.kind[e]), int(ob.sel_n[e]), int(ob.step[e])
        if kind == OBS_DETAILS:
            d = g._bare_observation([g._details(self._id(ob.sel[e, 0]))] if n else [], step=step)
        else:
            S = {self._id(i) for i in ob.S_snap[e, :int(ob.s_size[e])].tolist()}
            fr = ob.F_snap[e, :int(ob.f_shown[e])]
            F = {self._id(i) for i in fr[fr >= 0].tolist()}
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
    def reset(self, queries: Sequence[str], query_vectors=None) -> Tuple[np.ndarray, LazyInfos]:
        """Reset every environment with its query. query_vectors: [n_envs, d] host array or device
        tensor (an on-device encoder's output goes to the dense search without a host round trip);
        None encodes the queries with the graph's encoder."""
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
        # selection cleared; frontier = the reranked nodes (distinct): the device state of the batch
        fcap = K_NODES * (self.max_steps + 2)
        scap = 3 * (self.max_steps + 2)
        if self._bufs is None or self._fcap < fcap or self._scap < scap or self._bufs[0].device != engine.graph.device:
            self._alloc_state(max(fcap, 32), max(scap, 8))
        st = self._st
        self._part(st, "sel")[:] = ob.sel
        self._part(st, "sel_n")[:] = ob.sel_n
        F = self._part(st, "F")
        F[:] = -1
        F[:, :K_NODES] = ob.sel
        self._part(st, "F_end")[:] = n_out
        self._part(st, "F_n")[:] = n_out
        self._part(st, "S")[:] = -1
        self._part(st, "S_n")[:] = 0
        ob.S_snap, ob.F_snap = self._part(st, "S").copy(), F.copy()
        ob.f_shown[:] = n_out
        ob.f_size[:] = n_out
        self._cur[:] = 0
        self._last_action[:] = -1
        self._obs = self._reset_batch = ob
        vecs = self._featurize(ob)
        self._part(st, "step")[:] = 1
        self._part(st, "vec")[:] = vecs  # an unchanged observation keeps its vector on the device
        engine.graph.env_upload(self._bufs, st)

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
        if isinstance(actions, np.ndarray) and actions.ndim == 1 and (
                actions.dtype.kind in "bi" or (actions.dtype.kind == "u" and actions.dtype.itemsize < 8)):
            a = actions.astype(np.int64)  # (a policy's integer array: int() of each, without the loop)
        else:
            a = np.asarray([int(x) for x in actions], np.int64)
        if a.shape != (E,):
            raise ValueError("one action per environment")
        self._cur += 1
        ob = _ObsBatch.following(prev)  # the defaults: unchanged (aliased) observations
        ob.search = prev.search
        ob.stamp = self.hg._graph_stamp()

        # the step on the device (ahr_graph_env_step, one C call): expansions of the top 2 / 2 / 1
        # (environment.py:393-480), commits of the top 3 (:340-355), details of the top 1
        # (:301-335), the frontier / selection sets updated in device memory; the whole state comes
        # back as this step's snapshot (the observation dicts are built from it on demand)
        graph = self._engine.graph
        st = self._st
        if int(self._part(st, "F_end").max(initial=0)) + K_NODES > self._fcap or \
                int(self._part(st, "S_n").max(initial=0)) + 3 > self._scap:
            self._grow_state()
            st = self._st
        self._part(st, "actions")[:] = a
        tab = self._node_table()
        graph.env_step(self._bufs, st, E, K_NODES, self._fcap, self._scap, K_NODES, tab.dev)
        if self._part(st, "err")[0]:
            raise RuntimeError("environment state capacity exceeded (ahr_graph_env_step)")
        snap = st.copy()
        kind = self._part(snap, "kind")
        moved = kind > 0
        moved2 = moved[:, None]
        self._steps[:] = self._part(snap, "step")
        np.copyto(ob.step, self._steps, where=moved)
        # kernel kinds 1 / 2 / other -> expansion / commit / details (OBS_EXPAND / OBS_COMMIT /
        # OBS_DETAILS are 1 / 2 / 3)
        np.copyto(ob.kind, np.minimum(kind, OBS_DETAILS), where=moved, casting="unsafe")
        np.copyto(ob.sel, self._part(snap, "sel"), where=moved2)
        np.copyto(ob.sel_n, self._part(snap, "sel_n"), where=moved)
        np.copyto(ob.score, 0.0, where=moved2)
        np.copyto(ob.sem, 0.0, where=moved2)
        np.copyto(ob.seed_n, self._part(snap, "seed_n"), where=moved)
        sf = moved & (kind != 3)  # expansions and commits show the sets
        np.copyto(ob.s_size, self._part(snap, "s_size"), where=sf)
        np.copyto(ob.f_size, self._part(snap, "f_size"), where=sf)
        np.copyto(ob.f_shown, self._part(snap, "f_shown"), where=sf)
        ob.S_snap, ob.F_snap = self._part(snap, "S"), self._part(snap, "F")
        # end_episode, and any action past the five (gym_env.py _apply's last branch), and details of
        # an empty selection: the same observation
        ends = (a < 0) | (a > 4)
        ob.alias, ob.prev = ~moved, prev

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
        # the observations' vectors, written by the step kernel from the node table (an unchanged
        # observation keeps its own); environments showing a node whose attributes the featurizer
        # cannot convert take the reference's path (featurize_observation on the dict: it raises)
        vecs = self._part(snap, "vec")
        if tab.has_bad:
            valid = np.arange(K_NODES)[None, :] < ob.sel_n[:, None]
            bad = moved & (tab.bad[np.where(valid, ob.sel, 0)] & valid).any(axis=1)
            for e in np.flatnonzero(bad).tolist():
                vecs[e] = featurize_observation(self._obs_dict(ob, e), K_NODES)[0]
        cur = self._cur.copy()

        def info(e: int) -> Dict[str, Any]:
            d: Dict[str, Any] = {"action": int(a[e])}
            if self.enable_action_mask:
                d["action_mask"] = self._mask_list(ob, e)
            d.update({"raw_obs": self._obs_dict(ob, e), "aux": self._aux(ob, e), "step": int(cur[e])})
            return d
        return vecs, r.astype(np.float32), done, LazyInfos(E, info)
