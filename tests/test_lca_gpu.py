"""Device expand_to_lca (ahr_graph_lca) against the oracle's restatement of the reference
(oracle/search_ref.env_lca <- environment.py:243-299) on the reference's own saved graph, batched
over many input lists: single inputs, duplicates, summaries of both levels, entity/summary mixes,
padding; plus the capacity guard (a query beyond the kernel's LDS tables raises, never answers)."""
import os

import numpy as np
import pytest

from oracle import search_ref

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _sorted(G, ids, max_results=5):
    return sorted(ids, key=lambda x: (G.nodes[x].get("level") or 1, x))[:max_results]


def test_lca_batch_matches_oracle(cuda):
    from ah_rag.agent.environment import lca_batch
    from ah_rag.graph.hierarchical_graph import HierarchicalGraph
    hg = HierarchicalGraph.load(os.path.join(GOLDEN, "reference_graph"))
    G = hg.G
    dag_nodes = sorted({n for u, v, a in G.edges(data=True) if a.get("edge_type") == "belongs_to" for n in (u, v)})
    rng = np.random.default_rng(5)
    cases = [[n] for n in dag_nodes[:40]]
    for _ in range(300):
        m = int(rng.integers(1, 6))
        cases.append([dag_nodes[int(i)] for i in rng.integers(0, len(dag_nodes), m)])
    summaries = [n for n in dag_nodes if n.startswith("sum:")]
    cases += [[summaries[0], summaries[0]], summaries[:2], summaries[:7], [summaries[3], dag_nodes[0]]]
    got = lca_batch(hg, cases)
    for ids, g in zip(cases, got):
        want, _ = search_ref.env_lca(G, ids, max_results=10 ** 6)
        assert _sorted(G, g, 10 ** 6) == want, ids
    assert lca_batch(hg, [[]]) == [[]]


def test_lca_capacity_guard(cuda):
    """An ancestor set larger than the kernel's per-query table raises instead of truncating."""
    import networkx as nx
    from ah_rag.agent.environment import lca_batch
    from ah_rag.graph.hierarchical_graph import HierarchicalGraph
    hg = HierarchicalGraph()
    top = hg.add_summary(0, title="top")
    for i in range(5000):  # 5000 members of one summary: its ancestor set exceeds 4096 nodes
        hg.add_belongs_to(hg.add_entity(f"e{i}"), top)
    with pytest.raises(RuntimeError, match="capacity"):
        lca_batch(hg, [[top]])
    assert isinstance(hg.G, nx.DiGraph)
