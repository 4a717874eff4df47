#!/usr/bin/env python3
"""Golden cases for search(top_k > corpus rows), from the REFERENCE's own code (this container only).

Chroma answers `collection.query(n_results=N)` with N > count by returning every row (it clamps
n_results to the collection size); the stand-in collection of make_golden.py does the same (its
`sorted(...)[:n_results]`). The reference's HierarchicalGraph.search (hierarchical_graph.py:675-789)
is run unmodified on the same seeded 423-node graph as search_cases.json, with top_k = 5000 and
1000 (> AHR_MAX_K_LARGE = 4096 and > the index count), and its results are recorded in
search_bigk_cases.json for tests/test_dropin_gpu.py::test_search_topk_beyond_count.

Run: python tests/golden/make_golden_bigk.py   (needs /root/reference; never runs on the GPU box)
"""
from __future__ import annotations

import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (stand-ins, graph builder, JSON dump)


def main() -> None:
    mg.install_stubs()
    sys.path.insert(0, os.path.join(mg.REF, "src"))
    sys.path.insert(0, mg.REF)
    from ah_rag.graph.hierarchical_graph import HierarchicalGraph

    work = tempfile.mkdtemp(prefix="ahr_golden_bigk_")
    cwd = os.getcwd()
    os.chdir(work)
    try:
        hg, sids, eids = mg.build_graph(HierarchicalGraph)
        gdir = os.path.join(work, "graph")
        hg.save(gdir)
        hg = HierarchicalGraph.load(gdir)
        db = os.path.join(work, "vector_db")
        hg.G.graph["vector_index"]["db_path"] = db
        hg.build_vector_index(db_path=db, layers={0, 1}, reset=True)
        queries = [hg.G.nodes[eids[0]]["name"], hg.G.nodes[sids[1]]["title"], "a film about horror"]
        cases = []
        for q, top_k, rc in zip(queries, (5000, 1000, 5000), (True, False, False)):
            res = hg.search(q, top_k=top_k, member_top_m=2, return_cluster=rc)
            cases.append({"query": q, "params": {"top_k": top_k, "member_top_m": 2}, "return_cluster": rc,
                          "result": res})
        mg.dump("search_bigk_cases.json", {"dim": 384, "model": "all-MiniLM-L6-v2", "cases": cases})
    finally:
        os.chdir(cwd)


if __name__ == "__main__":
    main()
