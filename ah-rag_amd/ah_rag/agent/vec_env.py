"""Batched RL environment loop (SURVEY config C5: 2-hop expand + re-score inside the env loop).

The reference steps its PPO "vectorised" environments one after another
(src/ah_rag/agent/policy_ppo.py:145,163-214), each loading its own copy of the graph
(gym_env.py:27 -> environment.py:73-77) and paying an O(N) edge count per observation.
VecAHRAGGymEnv keeps N AHRAGGymEnv-equivalent environments over ONE device graph:
  reset(queries)  -> one batched search (dense top-k + expansion + rerank) for all N queries;
  step(actions)   -> environments that chose the same expansion action share one
                     ahr_graph_expand launch; commit/details/end are host bookkeeping.
Per-environment results are identical to stepping N AHRAGGymEnv objects one by one
(tests/test_vec_env_gpu.py).
"""
from __future__ import annotations

import time
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..graph.hierarchical_graph import HierarchicalGraph
from .environment import expand_batch
from .gym_env import AHRAGGymEnv, TOP_IDS, top_ids

EXPAND_ACTIONS = {0: "parents", 1: "children", 2: "related"}


class VecAHRAGGymEnv:
    def __init__(self, graph_dir: str = "graph", n_envs: int = 8, max_steps: int = 6,
                 enable_action_mask: bool = True, repeat_penalty: float = 0.02,
                 graph: Optional[HierarchicalGraph] = None) -> None:
        self.hg = graph or HierarchicalGraph.load(graph_dir)
        self.envs = [AHRAGGymEnv(graph_dir, max_steps=max_steps, enable_action_mask=enable_action_mask,
                                 repeat_penalty=repeat_penalty, graph=self.hg) for _ in range(n_envs)]
        for e in self.envs:  # per-step JSONL logging is off in the vectorised loop
            e.env.logging_enabled = False

    @property
    def n_envs(self) -> int:
        return len(self.envs)

    def reset(self, queries: Sequence[str], query_vectors: Optional[np.ndarray] = None
              ) -> Tuple[np.ndarray, List[Dict[str, Any]]]:
        if len(queries) != self.n_envs:
            raise ValueError("one query per environment")
        t0 = time.perf_counter()
        clusters = self.hg.search_batch(list(queries), top_k=5, member_top_m=5, return_cluster=True,
                                        query_vectors=query_vectors)
        dur = (time.perf_counter() - t0) / max(1, self.n_envs)
        vecs, infos = [], []
        for e, q, c in zip(self.envs, queries, clusters):
            ge = e.env
            e._query = q
            e._cur_step = 0
            ge.last_query = None
            ge.last_results = None
            ge.step_count = 0
            ge.selection_set.clear()
            ge.frontier_set.clear()
            ge.step_count += 1
            ge.last_query = q
            obs, _ = ge._anchor_result(q, 5, c, dur)
            v, info = e._finish_reset(obs)
            vecs.append(v)
            infos.append(info)
        return np.stack(vecs), infos

    def step(self, actions: Sequence[int]) -> Tuple[np.ndarray, np.ndarray, np.ndarray, List[Dict[str, Any]]]:
        actions = [int(a) for a in actions]
        prevs = [e._last_raw_obs for e in self.envs]
        if any(p is None for p in prevs):
            raise AssertionError("Call reset() first")
        for e in self.envs:
            e._cur_step += 1
        results: List[Optional[Tuple[Dict[str, Any], bool]]] = [None] * self.n_envs
        for a, name in EXPAND_ACTIONS.items():
            group = [i for i, x in enumerate(actions) if x == a]
            if not group:
                continue
            inputs = [top_ids(prevs[i], TOP_IDS[a]) for i in group]
            outs = expand_batch(self.hg, name, inputs, 10)
            for i, ids_in, ids_out in zip(group, inputs, outs):
                results[i] = (self.envs[i].env._expand_finish(name, ids_in, ids_out)[0], False)
        vecs, rews, dones, infos = [], [], [], []
        for i, e in enumerate(self.envs):
            obs, done = results[i] if results[i] is not None else e._apply(actions[i], prevs[i])
            v, r, d, info = e._finish_step(actions[i], prevs[i], obs, done)
            vecs.append(v)
            rews.append(r)
            dones.append(d)
            infos.append(info)
        return np.stack(vecs), np.asarray(rews, np.float32), np.asarray(dones), infos
