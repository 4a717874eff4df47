#!/usr/bin/env python3
"""Generate the C1 fixtures (BASELINE.json configs[0]) by running the REFERENCE's own code.

C1 = baselines.naive_rag on samples/hotpotqa_mini.txt. The reference's pipeline for a text file
is scripts/demo_cli.py:run_pipeline (:75-118): chunk -> HypergraphExtractor.extract -> artifacts
-> SemanticAggregator (BERTopic) -> HierarchicalGraph.build_from_artifacts -> save ->
build_vector_index(layers={0,1,2}, reset=True). Offline, extract() ends in the deterministic
`_fallback_extract` (hypergraph_extractor.py:214-264; no LLM endpoint), and the aggregator's
BERTopic/UMAP/HDBSCAN are absent, so the graph holds the L0 layer only: entities, hyperedges,
participates_in edges — what build_from_artifacts makes from extractions.json alone
(hierarchical_graph.py:241-421). Chunking: demo_cli.smart_chunks returns the whole text as one
chunk when it is under 6,400 cl100k tokens (:30-33); tiktoken is absent here, and the 14 KB
English sample is ~3.4k tokens, so the document is one chunk.

This script (this container only; it imports /root/reference under the same in-memory stand-ins
for sentence_transformers / chromadb as make_golden.py) writes tests/golden/c1/:
  hotpotqa_mini.txt      the input document (a data file of the reference, copied as the C1 input)
  extractions.json       reference _fallback_extract output, model_dump()'d (demo_cli.py:96-97)
  structure.json, meta.json   the reference's save() of the built graph
  naive_d384.json, naive_d768.json
                         NaiveRAG.run(title, top_k=10) for the 25 passage titles, encoder stand-in
                         at d = 384 (all-MiniLM-L6-v2, the reference default) and d = 768.

Run: python tests/golden/make_golden_c1.py
"""
from __future__ import annotations

import json
import os
import re
import shutil
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
OUT = os.path.join(HERE, "c1")
sys.path.insert(0, HERE)

import make_golden as mg  # noqa: E402  (stand-ins + dump helpers)

MODELS = {384: "all-MiniLM-L6-v2", 768: "all-mpnet-base-v2"}


def titles(text: str):
    return [m.strip() for m in re.findall(r"^###\s+(.+)$", text, flags=re.M)]


def main() -> None:
    mg.DIMS["all-mpnet-base-v2"] = 768
    mg.install_stubs()
    sys.path.insert(0, os.path.join(REF, "src"))
    sys.path.insert(0, REF)
    from ah_rag.extract.hypergraph_extractor import HypergraphExtractor
    from ah_rag.graph.hierarchical_graph import HierarchicalGraph
    from baselines.naive_rag import NaiveRAG

    with open(os.path.join(REF, "samples", "hotpotqa_mini.txt"), encoding="utf-8") as f:
        doc = f.read()
    shutil.rmtree(OUT, ignore_errors=True)
    os.makedirs(OUT)
    with open(os.path.join(OUT, "hotpotqa_mini.txt"), "w", encoding="utf-8") as f:
        f.write(doc)

    work = tempfile.mkdtemp(prefix="ahr_c1_")
    cwd = os.getcwd()
    os.chdir(work)
    try:
        ex = HypergraphExtractor()._fallback_extract(doc)
        os.makedirs("artifacts", exist_ok=True)
        records = [e.model_dump() for e in ex]
        with open(os.path.join("artifacts", "extractions.json"), "w", encoding="utf-8") as f:
            json.dump(records, f, ensure_ascii=False, indent=2)
        shutil.copy(os.path.join("artifacts", "extractions.json"), os.path.join(OUT, "extractions.json"))
        hg = HierarchicalGraph()
        hg.build_from_artifacts("artifacts")
        hg.save("graph", meta={"source": "samples/hotpotqa_mini.txt"})
        for fn in ("structure.json", "meta.json"):
            shutil.copy(os.path.join("graph", fn), os.path.join(OUT, fn))

        class EchoGen:
            def generate(self, query, context, cfg):
                return {"query": query, "context": context}

        qs = titles(doc)
        for dim, model in MODELS.items():
            g = HierarchicalGraph.load("graph")
            db = os.path.join(work, f"vector_db_{dim}")
            g.build_vector_index(db_path=db, layers={0, 1, 2}, model_name=model, reset=True)
            naive = NaiveRAG(g, EchoGen())
            cases = [{"query": q, "top_k": 10, "out": naive.run(q, top_k=10)} for q in qs]
            n_idx = g.G.graph["vector_index"]["indexed_nodes"]
            with open(os.path.join(OUT, f"naive_d{dim}.json"), "w", encoding="utf-8") as f:
                json.dump(mg.strip_ts({"dim": dim, "model": model, "indexed_nodes": n_idx, "cases": cases}), f,
                          ensure_ascii=False, separators=(",", ":"), default=mg.jsonable)
        kinds = {}
        for _, d in hg.G.nodes(data=True):
            kinds[d.get("node_type")] = kinds.get(d.get("node_type"), 0) + 1
        print("C1 graph:", kinds, "edges", hg.G.number_of_edges(), "queries", len(qs))
    finally:
        os.chdir(cwd)
        shutil.rmtree(work, ignore_errors=True)
    print("C1 fixtures written to", OUT)


if __name__ == "__main__":
    main()
