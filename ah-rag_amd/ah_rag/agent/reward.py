"""Dense step reward and final reward (reference src/ah_rag/agent/reward.py:6-38)."""
from __future__ import annotations

from typing import Any, Dict, Optional


def _ids(obs: Optional[Dict[str, Any]], key: str) -> set:
    return set(((obs or {}).get("state") or {}).get(key) or [])


def step_reward(prev_obs: Optional[Dict[str, Any]], cur_obs: Dict[str, Any]) -> float:
    """+1.0 per new selection id, +0.05 per frontier growth (at most 10), -0.05 per step."""
    if prev_obs is None:
        return 0.0
    gained = len(_ids(cur_obs, "selection_ids") - _ids(prev_obs, "selection_ids"))
    grown = max(0, len(_ids(cur_obs, "frontier_ids")) - len(_ids(prev_obs, "frontier_ids")))
    return float(1.0 * gained + 0.05 * min(grown, 10) - 0.05)


def final_reward(metrics: Dict[str, float]) -> float:
    w = {"f1": 0.4, "faithfulness": 0.3, "answer_relevancy": 0.2, "contextual_recall": 0.1}
    return sum(wt * float(metrics.get(k, 0.0)) for k, wt in w.items())
