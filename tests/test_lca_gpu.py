"""Device expand_to_lca (ahr_graph_lca) against the oracle's restatement of the reference
(oracle/search_ref.env_lca <- environment.py:243-299) on the reference's own saved graph, batched
over many input lists: single inputs, duplicates, summaries of both levels, entity/summary mixes,
padding; plus queries beyond the LDS kernel's tables, answered by the global-memory kernel; and
the host-to-host expansion entry (ahr_graph_expand_host) against the device one."""
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


def test_lca_large_matches_lds_kernel(cuda):
    """ahr_graph_lca_large (global-memory visited set) gives lca()'s answers on every case."""
    import torch
    from ah_rag.graph.hierarchical_graph import HierarchicalGraph
    hg = HierarchicalGraph.load(os.path.join(GOLDEN, "reference_graph"))
    dg = hg.device_graph()
    G = hg.G
    dag_nodes = sorted({n for u, v, a in G.edges(data=True) if a.get("edge_type") == "belongs_to" for n in (u, v)})
    rng = np.random.default_rng(9)
    idx = np.full((200, 5), -1, np.int32)
    for b in range(200):
        m = int(rng.integers(0, 6))
        idx[b, :m] = dg.node_indices([dag_nodes[int(i)] for i in rng.integers(0, len(dag_nodes), m)])
    o1, c1 = dg.lca(torch.from_numpy(idx))
    o2, c2 = dg.lca_large(torch.from_numpy(idx))
    o1, c1, o2, c2 = o1.cpu().numpy(), c1.cpu().numpy(), o2.cpu().numpy(), c2.cpu().numpy()
    assert (c1 >= 0).all() and np.array_equal(c1, c2)
    for b in range(200):
        assert sorted(o1[b, :c1[b]]) == sorted(o2[b, :c2[b]])


def test_lca_over_capacity_matches_oracle(cuda):
    """Ancestor sets beyond the LDS kernel's tables (4096 visited nodes, 1024 per BFS level) are
    answered by ahr_graph_lca_large, with the reference's result (it used to raise)."""
    import networkx as nx
    from ah_rag.agent.environment import GraphEnvironment, lca_batch
    from ah_rag.graph.hierarchical_graph import HierarchicalGraph
    hg = HierarchicalGraph()
    top = hg.add_summary(0, title="top")
    mids = [hg.add_summary(1 + j, title=f"mid{j}") for j in range(3)]
    ents = [hg.add_entity(f"e{i}") for i in range(5000)]
    for i, e in enumerate(ents):  # 5000 members of one summary: its ancestor set exceeds 4096 nodes
        hg.add_belongs_to(e, top)
        if i % 2 == 0:
            hg.add_belongs_to(e, mids[i % 3])
    for m in mids:
        hg.add_belongs_to(m, top)
    G = hg.G
    cases = [[top], [top, mids[0]], mids[:2], [mids[1]], [top, top], [ents[0], top], [mids[2], ents[4]]]
    got = lca_batch(hg, cases)
    for ids, g in zip(cases, got):
        want, _ = search_ref.env_lca(G, ids, max_results=10 ** 6)
        assert _sorted(G, g, 10 ** 6) == want, ids
    env = GraphEnvironment(graph=hg, logging_enabled=False)
    obs, info = env.expand_to_lca([top, mids[0]])
    want, _ = search_ref.env_lca(G, [top, mids[0]])
    assert [x["node_id"] for x in obs["selection"]] == want and info["lca_count"] == len(want)
    assert isinstance(hg.G, nx.DiGraph)


def test_expand_host_matches_device_expand(cuda):
    """ahr_graph_expand_host (host in, host out, one call; reused per-shape buffers) returns what
    ahr_graph_expand writes on the device, for every action, ragged inputs (-1 padding), limits 0,
    1, 10 and 32, batch shapes met more than once (the buffers are reused), the small-batch path
    (B * n_in <= 16: inputs as kernel arguments, results stored into the pinned buffer) and the
    copy path, and pageable host buffers (which always take the copy path)."""
    import torch
    from ah_rag.graph.hierarchical_graph import HierarchicalGraph
    hg = HierarchicalGraph.load(os.path.join(GOLDEN, "reference_graph"))
    dg = hg.device_graph()
    nodes = list(hg.G.nodes)
    rng = np.random.default_rng(11)
    for rep in range(2):
        for action in ("parents", "children", "related"):
            for B, n_in, limit in ((1, 3, 10), (1, 1, 1), (7, 5, 10), (64, 2, 0), (33, 4, 3), (4, 4, 10),
                                     (16, 1, 32), (2, 8, 5), (1, 0, 3), (3, 5, 0)):
                idx = np.full((B, n_in), -1, np.int32)
                for b in range(B):
                    m = int(rng.integers(0, n_in + 1))
                    idx[b, :m] = dg.node_indices([nodes[int(i)] for i in rng.integers(0, len(nodes), m)])
                out_h, cnt_h = dg.expand_host(action, idx, limit)
                out_d, cnt_d = dg.expand(action, torch.from_numpy(idx), limit)
                cnt_d = cnt_d.cpu().numpy()
                out_d = out_d.cpu().numpy()
                assert np.array_equal(cnt_h, cnt_d), (action, B, n_in, limit)
                for b in range(B):
                    assert np.array_equal(out_h[b, :cnt_h[b]], out_d[b, :cnt_d[b]]), (action, B, b)
                # the same call through pageable numpy buffers (direct C call)
                from ah_rag import _native as nat
                lim = max(limit, 1)
                res = np.zeros(B * lim + B, np.int32)
                x = np.ascontiguousarray(idx)
                need = nat.ctypes.c_int64()
                nat.check(nat.lib().ahr_graph_expand_ws_bytes(B, n_in, limit, nat.ctypes.byref(need)), "ws")
                ws = torch.empty(max(need.value, 8), dtype=torch.uint8, device=dg.device)
                nat.check(nat.lib().ahr_graph_expand_host(
                    dg._h, {"parents": 0, "children": 1, "related": 2}[action], x.ctypes.data, B, n_in, limit,
                    res.ctypes.data, res.ctypes.data + 4 * B * lim, ws.data_ptr(), need.value,
                    nat.stream_ptr(None, dg._dev_index)), "ahr_graph_expand_host")
                assert np.array_equal(res[B * lim:], cnt_d), (action, B, n_in, limit)
                for b in range(B):
                    assert np.array_equal(res[b * lim:b * lim + cnt_d[b]], out_d[b, :cnt_d[b]]), (action, B, b)
