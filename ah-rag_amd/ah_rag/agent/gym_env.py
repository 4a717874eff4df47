"""AHRAGGymEnv — drop-in for reference src/ah_rag/agent/gym_env.py (class at :11).

Discrete actions: 0 expand_parents(top 2), 1 expand_children(top 2), 2 expand_related(top 1),
3 commit_top(top 3), 4 query_details_top(top 1), 5 end_episode. Observations are the 84-d
featurizer vector; dense step rewards with a repeat-action penalty.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

from .environment import GraphEnvironment
from .featurizer import featurize_observation
from .reward import step_reward

N_ACTIONS = 6
END_EPISODE = 5
TOP_IDS = {0: 2, 1: 2, 2: 1, 3: 3, 4: 1}


def top_ids(raw_obs: Dict[str, Any], k: int) -> List[str]:
    return [n["node_id"] for n in (raw_obs.get("selection") or [])[:k] if n.get("node_id")]


def action_mask(raw_obs: Optional[Dict[str, Any]]) -> List[int]:
    """Only end_episode is valid when the observation has no selection (reference :54-75)."""
    if not (raw_obs or {}).get("selection"):
        return [0] * (N_ACTIONS - 1) + [1]
    return [1] * N_ACTIONS


class AHRAGGymEnv:
    def __init__(self, graph_dir: str = "graph", max_steps: int = 6, debug: bool = False,
                 enable_action_mask: bool = True, repeat_penalty: float = 0.02, *, graph=None) -> None:
        self.env = GraphEnvironment(graph_dir=graph_dir, debug=debug, log_level="off", redact=True, graph=graph)
        self.max_steps = max(1, int(max_steps))
        self._cur_step = 0
        self._last_obs: Optional[Dict[str, Any]] = None
        self._last_raw_obs: Optional[Dict[str, Any]] = None
        self._query: Optional[str] = None
        self.enable_action_mask = bool(enable_action_mask)
        self.repeat_penalty = float(repeat_penalty)
        self._last_action: Optional[int] = None

    @property
    def action_size(self) -> int:
        return N_ACTIONS

    def get_action_mask(self) -> List[int]:
        return action_mask(self._last_raw_obs)

    def _pick_top_ids(self, raw_obs: Dict[str, Any], k: int = 2) -> List[str]:
        return top_ids(raw_obs, k)

    def reset(self, query: str) -> Tuple[Any, Dict[str, Any]]:
        self._query = query
        self._cur_step = 0
        raw_obs, _ = self.env.reset(seed_query=query)
        return self._finish_reset(raw_obs)

    def _finish_reset(self, raw_obs: Dict[str, Any]) -> Tuple[Any, Dict[str, Any]]:
        vec, aux = featurize_observation(raw_obs)
        self._last_obs = {"vec": vec, "aux": aux}
        self._last_raw_obs = raw_obs
        info: Dict[str, Any] = {"raw_obs": raw_obs, "aux": aux}
        if self.enable_action_mask:
            info["action_mask"] = self.get_action_mask()
        self._last_action = None
        return vec, info

    def _apply(self, action: int, prev_raw: Dict[str, Any]) -> Tuple[Dict[str, Any], bool]:
        ids = top_ids(prev_raw, TOP_IDS.get(action, 0))
        if action == 0:
            return self.env.expand_parents(ids)[0], False
        if action == 1:
            return self.env.expand_children(ids)[0], False
        if action == 2:
            return self.env.expand_related(ids)[0], False
        if action == 3:
            return self.env.commit_selection(ids)[0], False
        if action == 4:
            return (self.env.query_node_details(ids[0])[0] if ids else prev_raw), False
        return prev_raw, True

    def step(self, action: int) -> Tuple[Any, float, bool, Dict[str, Any]]:
        assert self._last_raw_obs is not None, "Call reset() first"
        self._cur_step += 1
        prev_raw = self._last_raw_obs
        obs, done = self._apply(int(action), prev_raw)
        return self._finish_step(int(action), prev_raw, obs, done)

    def _finish_step(self, action: int, prev_raw: Dict[str, Any], obs: Dict[str, Any], done: bool):
        r = 0.0 if done else step_reward(prev_raw, obs)
        if not done and self._last_action is not None and action == self._last_action and self.repeat_penalty > 0:
            r -= self.repeat_penalty
        done = done or self._cur_step >= self.max_steps
        vec, aux = featurize_observation(obs)
        self._last_obs = {"vec": vec, "aux": aux}
        self._last_raw_obs = obs
        info: Dict[str, Any] = {"action": action}
        if self.enable_action_mask:
            info["action_mask"] = self.get_action_mask()
        self._last_action = action
        info.update({"raw_obs": obs, "aux": aux, "step": self._cur_step})
        return vec, float(r), bool(done), info
