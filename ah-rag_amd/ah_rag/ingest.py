"""Offline text -> graph -> vector index pipeline (the C1 plumbing of BASELINE.json configs[0]).

Mirrors the reference's scripts/demo_cli.py:run_pipeline (:75-118) for the case it takes without
an LLM endpoint or BERTopic (neither exists offline): chunk the document (smart_chunks, :30-72),
extract hyperedges with the deterministic fallback (ah_rag.extract), write
artifacts/extractions.json (:95-97), HierarchicalGraph.build_from_artifacts + save (:109-111),
build_vector_index(layers={0, 1, 2}, reset=True) (:114). The L1/L2 aggregation step (:99-106:
BERTopic topics, LLM summaries, relations, communities) is out of scope, so the
graph is the L0 layer: entities, hyperedges, participates_in edges.
"""
from __future__ import annotations

import json
import os
from typing import Callable, List, Optional

from .extract import HypergraphExtractor
from .graph.hierarchical_graph import HierarchicalGraph


def _token_counter() -> Callable[[str], int]:
    """cl100k token count when tiktoken is importable (the reference's tokenize_len, :20-25);
    otherwise an upper-bound estimate of one token per 3 bytes (English BPE averages ~4)."""
    try:
        import tiktoken  # type: ignore
        enc = tiktoken.get_encoding("cl100k_base")
        return lambda t: len(enc.encode(t))
    except Exception:
        return lambda t: (len(t.encode("utf-8")) + 2) // 3


def smart_chunks(text: str, model_ctx: int = 8000, max_output: int = 1200, buffer: int = 400,
                 count_tokens: Optional[Callable[[str], int]] = None) -> List[str]:
    """Token-budgeted chunks (demo_cli.py:28-72): the whole text if it fits the budget, else
    blank-line paragraphs packed greedily, a paragraph over the budget split by lines."""
    count = count_tokens or _token_counter()
    limit = model_ctx - max_output - buffer
    if count(text) <= limit:
        return [text]
    chunks: List[str] = []
    cur: List[str] = []
    cur_tok = 0
    for para in (p.strip() for p in text.split("\n\n")):
        if not para:
            continue
        ptok = count(para)
        if cur_tok + ptok + 1 <= limit:
            cur.append(para)
            cur_tok += ptok + 1
            continue
        if cur:
            chunks.append("\n\n".join(cur))
        if ptok <= limit:
            cur, cur_tok = [para], ptok + 1
            continue
        buf: List[str] = []
        btok = 0
        for line in para.splitlines():
            ltok = count(line)
            if btok + ltok + 1 <= limit:
                buf.append(line)
                btok += ltok + 1
            else:
                if buf:
                    chunks.append("\n".join(buf))
                buf, btok = [line], ltok + 1
        if buf:
            chunks.append("\n".join(buf))
        cur, cur_tok = [], 0
    if cur:
        chunks.append("\n\n".join(cur))
    return chunks


def ingest_text(document: str, workdir: str = ".", source: Optional[str] = None,
                model_name: str = "all-MiniLM-L6-v2", db_path: Optional[str] = None) -> HierarchicalGraph:
    """Run the offline pipeline in `workdir` (artifacts/, graph/, vector_db/ as the reference
    lays them out) and return the indexed graph."""
    extractor = HypergraphExtractor()
    records = []
    for chunk in smart_chunks(document):
        records.extend(extractor.extract(chunk))
    art = os.path.join(workdir, "artifacts")
    os.makedirs(art, exist_ok=True)
    with open(os.path.join(art, "extractions.json"), "w", encoding="utf-8") as f:
        json.dump(records, f, ensure_ascii=False, indent=2)
    hg = HierarchicalGraph()
    hg.build_from_artifacts(art)
    hg.save(os.path.join(workdir, "graph"), meta={"source": source} if source else None)
    hg.build_vector_index(db_path=db_path or os.path.join(workdir, "vector_db"), layers={0, 1, 2},
                          model_name=model_name, reset=True)
    return hg
