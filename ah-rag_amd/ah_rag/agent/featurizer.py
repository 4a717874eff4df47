"""Observation -> fixed-length float32 vector (reference src/ah_rag/agent/featurizer.py:7-56).

Layout: [step, |selection_ids|, |frontier_ids|, |seeds|] + k_nodes blocks of
[is_entity, is_summary, is_other, layer, score, semantic, judge_overall, confidence] for the
first k_nodes entries of obs["selection"], zero padded (84 values at k_nodes = 10).
"""
from __future__ import annotations

from typing import Any, Dict, List, Sequence, Tuple

import numpy as np

NODE_FEATS = 8


def _num(x: Any) -> float:
    return float(x or 0.0)


def node_row(n: Dict[str, Any]) -> List[float]:
    kind = str(n.get("node_type") or "")
    return [float(kind == "entity"), float(kind == "summary"), float(kind not in ("entity", "summary")),
            _num(n.get("layer")), _num(n.get("score")), _num(n.get("semantic")),
            _num(n.get("judge_overall")), _num(n.get("confidence"))]


def featurize_observation(obs: Dict[str, Any], k_nodes: int = 10) -> Tuple[np.ndarray, Dict[str, Any]]:
    state = obs.get("state") or {}
    sel = (obs.get("selection") or [])[:k_nodes]
    # one Python list, one float32 conversion (each value rounded once from double, as before);
    # node_row inlined (the single environment featurizes every step)
    row = [_num(obs.get("step")), float(len(state.get("selection_ids") or [])),
           float(len(state.get("frontier_ids") or [])), float(len(obs.get("seeds") or []))]
    for n in sel:
        g = n.get
        kind = str(g("node_type") or "")
        ent, summ = kind == "entity", kind == "summary"
        row += (float(ent), float(summ), float(not (ent or summ)), float(g("layer") or 0.0),
                float(g("score") or 0.0), float(g("semantic") or 0.0), float(g("judge_overall") or 0.0),
                float(g("confidence") or 0.0))
    row.extend([0.0] * (NODE_FEATS * (k_nodes - len(sel))))
    vec = np.array(row, np.float32)
    return vec, {"top_node_ids": [str(n.get("node_id")) for n in sel]}


def featurize_batch(observations: Sequence[Dict[str, Any]], k_nodes: int = 10) -> np.ndarray:
    """[N, 4 + 8 k_nodes] float32 for a batch of environments."""
    return np.stack([featurize_observation(o, k_nodes)[0] for o in observations]) if observations else \
        np.zeros((0, 4 + NODE_FEATS * k_nodes), np.float32)
