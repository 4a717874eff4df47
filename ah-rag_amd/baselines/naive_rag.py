"""NaiveRAG — drop-in for reference baselines/naive_rag.py:7-43: flat top-K evidence from the
graph's hybrid search, packed into skeleton lines, handed to the shared answer generator."""
from __future__ import annotations

from typing import Any, Dict, List, Optional


class NaiveRAG:
    def __init__(self, hg: Any, answer_generator: Any) -> None:
        self.hg = hg
        self.answer_generator = answer_generator

    def context(self, query: str, top_k: int = 5) -> Dict[str, Any]:
        hits = self.hg.search(query, top_k=top_k, return_cluster=False) or []
        lines: List[str] = []
        used: List[str] = []
        for nid in [h.get("node_id") for h in hits if h.get("node_id")]:
            d = self.hg.G.nodes.get(nid, {})
            title = d.get("title") or d.get("name") or ""
            body = d.get("summary_text") or d.get("summary") or d.get("description") or ""
            lines.append(f"- [{nid}] {title} :: {body[:200]}")
            used.append(nid)
        return {"context_text": "\n".join(lines), "used_nodes": used, "stats": {}}

    def run(self, query: str, top_k: int = 5, gen_cfg: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
        return self.answer_generator.generate(query, self.context(query, top_k), gen_cfg or {})
