"""VecAHRAGGymEnv's array state machine against the oracle's reference episode, on the CPU.

The two device passes it calls — the batched search (dense top-5 + expansion + rerank,
HierarchicalGraph.search_arrays) and the batched expansions (DeviceGraph.expand) — are replaced by
host stand-ins built from the oracle (oracle/search_ref.py: expand_rerank for
hierarchical_graph.py:719-789, env_expand for environment.py:393-480), so what is checked here is
everything the vectorised environment does on the host: selection / frontier sets, the commit /
details / end / invalid-action rules, observation dicts built lazily from state snapshots, the
batched featurizer, rewards, repeat penalty and done flags, against search_ref.GymEpisode
(environment.py:118-150, :301-355; gym_env.py:41-125; featurizer.py:21-56; reward.py:6-26).
The GPU tests (test_vec_env_gpu.py, test_c5_env_gpu.py) run the same loop on the real kernels.
"""
import json
import os
import shutil
import types

import numpy as np
import pytest
import torch

from oracle import search_ref

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _norm(x):
    return json.loads(json.dumps(x, default=lambda o: o.tolist() if hasattr(o, "tolist") else str(o)))


class _HostGraph:
    """DeviceGraph stand-in: ids / n_nodes and expand() by the oracle's env_expand."""

    def __init__(self, G):
        self.G = G
        self.ids = list(G.nodes)
        self.index = {n: i for i, n in enumerate(self.ids)}
        self.n_nodes = len(self.ids)

    # ahr_graph_env_step restated on the host over the oracle's expansions (environment.py:301-355,
    # :393-480 on the environments' slot arrays; include/ahr.h documents the kernel's contract)
    def env_buffers(self, E, K, fcap, scap):
        from ah_rag.graph_search import DeviceGraph
        offs, nbytes = DeviceGraph.env_layout(E, K, fcap, scap)
        return None, np.zeros(nbytes // 4, np.int32), offs

    def env_upload(self, bufs, host):
        pass

    def env_node_table(self, feats):
        return np.asarray(feats, np.float32)

    def env_step(self, bufs, st, E, K, fcap, scap, limit, feats=None):
        from ah_rag.graph_search import DeviceGraph
        offs, _ = DeviceGraph.env_layout(E, K, fcap, scap)
        part = {n: st[offs[i]:] for i, n in enumerate(DeviceGraph.ENV_PARTS)}
        sel, F, S = part["sel"][:E * K].reshape(E, K), part["F"][:E * fcap].reshape(E, fcap), \
            part["S"][:E * scap].reshape(E, scap)
        n_g = self.n_nodes
        for e in range(E):
            a, n = int(part["actions"][e]), int(part["sel_n"][e])
            top = [int(x) if 0 <= x < n_g else -1 for x in sel[e, :min(n, 3)]]
            fe, fn, sn = int(part["F_end"][e]), int(part["F_n"][e]), int(part["S_n"][e])
            kind = -1
            if 0 <= a <= 2:
                names = [self.ids[x] for x in top[:(2, 2, 1)[a]] if x >= 0]
                out = [self.index[i] for i in search_ref.env_expand(self.G, ("parents", "children", "related")[a],
                                                                     names, limit)]
                part["f_shown"][e], part["f_size"][e], part["s_size"][e] = fe, fn, sn
                sel[e] = -1
                sel[e, :len(out)] = out
                part["sel_n"][e] = part["seed_n"][e] = len(out)
                for v in out:
                    if v not in F[e, :fe].tolist():
                        F[e, fe] = v
                        fe += 1
                        fn += 1
                kind = 1
            elif a == 3:
                added = []
                for x in top[:3]:
                    if x >= 0 and x not in S[e, :sn].tolist():
                        S[e, sn] = x
                        sn += 1
                        added.append(x)
                        hit = np.flatnonzero(F[e, :fe] == x)
                        if len(hit):
                            F[e, hit[0]] = -1
                            fn -= 1
                sel[e] = -1
                sel[e, :len(added)] = added
                part["sel_n"][e], part["seed_n"][e] = len(added), 0
                part["f_shown"][e], part["f_size"][e], part["s_size"][e] = fe, fn, sn
                kind = 2
            elif a == 4 and n > 0:
                node = int(sel[e, 0])
                sel[e] = -1
                if node < n_g:
                    sel[e, 0] = node
                part["sel_n"][e], part["seed_n"][e] = int(node < n_g), 0
                kind = 3
            part["F_end"][e], part["F_n"][e], part["S_n"][e], part["kind"][e] = fe, fn, sn, kind
            if kind > 0 and feats is not None:  # the featurizer vector of the new observation
                part["step"][e] += 1
                vec = part["vec"][:E * (4 + 8 * K)].view(np.float32).reshape(E, 4 + 8 * K)
                full = kind != 3
                ns = int(part["sel_n"][e])
                f_obs = int(part["f_size"][e])
                row = [float(part["step"][e]), float(sn) if full else 0.0, float(min(f_obs, 50)) if full else 0.0,
                       float(part["seed_n"][e])]
                for i in range(K):
                    if i < ns:
                        f = feats[int(sel[e, i])]
                        row += [f[0], f[1], f[2], f[3], 0.0, 0.0, f[4], f[5]]
                    else:
                        row += [0.0] * 8
                vec[e] = np.asarray(row, np.float32)

    def expand(self, action, inputs, limit=10, stream=None):
        x = inputs.numpy()
        out = np.full((x.shape[0], limit), -1, np.int32)
        cnt = np.zeros(x.shape[0], np.int32)
        for b, row in enumerate(x):
            ids = search_ref.env_expand(self.G, action, [self.ids[i] for i in row if i >= 0], limit)
            out[b, :len(ids)] = [self.index[i] for i in ids]
            cnt[b] = len(ids)
        return torch.from_numpy(out), torch.from_numpy(cnt)


def _host_search(hg, graph, row_ids, vectors, metas):
    """HierarchicalGraph.search_arrays stand-in: exact fp32 top-5 + the oracle's expand_rerank,
    returned as the rerank kernel's result arrays."""
    from ah_rag import _native as nat
    from ah_rag.graph_search import RerankResult, resolve_search_params
    n = graph.n_nodes
    row_to_node = np.asarray([graph.index.get(r, n + i) for i, r in enumerate(row_ids)], np.int32)
    engine = types.SimpleNamespace(graph=graph, row_ids=row_ids, row_metas=metas, row_to_node_host=row_to_node,
                                   node_id=lambda idx: graph.ids[idx] if idx < n else row_ids[idx - n])
    ext = lambda nid: graph.index.get(nid, n + row_ids.index(nid) if nid in row_ids else -1)  # noqa: E731

    def search_arrays(queries, top_k=5, member_top_m=5, query_vectors=None, **_):
        G = hg.G
        params = resolve_search_params(G.graph.get("search_params", {}), top_k, member_top_m, None, None, None,
                                       None, None, None, None)
        p = search_ref.resolve_params(G.graph.get("search_params", {}), top_k=top_k, member_top_m=member_top_m)
        q = np.asarray(query_vectors, np.float32)
        s = q @ vectors.T
        B, k = len(q), min(top_k, len(row_ids))
        rows = np.full((B, top_k), -1, np.int32)
        scores = np.full((B, top_k), -np.inf, np.float32)
        W = k * (1 + max(2, member_top_m))
        res = RerankResult(*(np.zeros((B, W), t) for t in (np.int32, np.float64, np.int32)), np.zeros(B, np.int32),
                           *(np.zeros((B, max(top_k, 1)), t) for t in (np.int32, np.float64, np.float64)),
                           np.zeros(B, np.int32))
        for b in range(B):
            order = np.lexsort((np.arange(len(row_ids)), -s[b]))[:k]
            rows[b, :k], scores[b, :k] = order, s[b, order]
            dist = (np.float32(1.0) - scores[b, :k].astype(np.float32)).tolist()
            seeds = [{"node_id": row_ids[r], "semantic": 1.0 - float(x), "meta": metas[r]} for r, x in zip(order, dist)]
            cl = search_ref.expand_rerank(G, seeds, p, return_cluster=True)
            pos = {sd["node_id"]: i for i, sd in enumerate(seeds)}
            for j, e in enumerate(cl["expanded"]):
                res.exp_nodes[b, j] = ext(e["node_id"])
                res.exp_sem[b, j] = e["semantic"]
                src = pos.get(e["node_id"]) if not e.get("meta", {}).get("expanded") else None
                res.exp_src[b, j] = src if src is not None else -1 - nat.NODE_TYPE_CODES.get(e["node_type"], 0)
            res.exp_count[b] = len(cl["expanded"])
            for j, r in enumerate(cl["reranked"]):
                res.out_nodes[b, j] = ext(r["node_id"])
                res.out_sem[b, j] = r["semantic"]
                res.out_score[b, j] = r["score"]
            res.out_count[b] = len(cl["reranked"])
        return engine, params, rows, scores, res
    return search_arrays


@pytest.fixture(scope="module")
def env_graph(tmp_path_factory):
    from ah_rag.graph.hierarchical_graph import HierarchicalGraph
    d = tmp_path_factory.mktemp("vec_cpu") / "graph"
    shutil.copytree(os.path.join(GOLDEN, "reference_graph"), d)
    hg = HierarchicalGraph.load(str(d))
    ids = [n for n, a in hg.G.nodes(data=True) if a.get("node_type") in ("entity", "summary")]
    rng = np.random.default_rng(5)
    vec = rng.standard_normal((len(ids), 64)).astype(np.float32)
    vec /= np.linalg.norm(vec, axis=1, keepdims=True)
    metas = [hg._embedding_text(n)[1] for n in ids]
    return hg, ids, vec, metas


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_vec_env_state_machine_matches_oracle(env_graph, monkeypatch, seed):
    from ah_rag.agent import vec_env as ve
    hg, ids, vec, metas = env_graph
    G = hg.G
    graph = _HostGraph(G)
    monkeypatch.setattr(hg, "search_arrays", _host_search(hg, graph, ids, vec, metas))
    E, steps = 24, 7
    rng = np.random.default_rng(seed)
    venv = ve.VecAHRAGGymEnv(n_envs=E, max_steps=6, graph=hg)
    eps = [search_ref.GymEpisode(G, max_steps=6) for _ in range(E)]
    for episode in range(2):
        pick = rng.integers(0, len(ids), E)
        qv = vec[pick] + 0.3 * rng.standard_normal((E, vec.shape[1])).astype(np.float32)
        qv /= np.linalg.norm(qv, axis=1, keepdims=True)
        vecs, infos = venv.reset([f"q{i}" for i in range(E)], query_vectors=qv)
        for b in range(E):
            cluster = venv.envs[b].env.last_results
            v_want, raw_want = eps[b].reset(cluster)
            np.testing.assert_array_equal(vecs[b], v_want)
            assert search_ref.isclose_dicts(_norm(infos[b]["raw_obs"]), _norm(raw_want)), b
            assert infos[b]["action_mask"] == eps[b].mask() == venv.envs[b].get_action_mask()
            assert infos[b]["aux"]["top_node_ids"] == [str(n["node_id"]) for n in raw_want["selection"][:10]]
        prev_raw = [infos[b]["raw_obs"] for b in range(E)]
        for t in range(steps):
            # every action kind, invalid ones (7, -1) and repeats; masked envs mostly end
            acts = rng.choice([0, 1, 2, 3, 4, 5, 0, 2, 3, 4, 7, -1], E)
            v, r, d, inf = venv.step(acts)
            assert v.shape == (E, 84) and v.dtype == np.float32 and r.dtype == np.float32
            for b in range(E):
                v_want, r_want, d_want, raw_want = eps[b].step(int(acts[b]))
                np.testing.assert_array_equal(v[b], v_want, err_msg=f"{episode} {t} {b} {acts[b]}")
                assert r[b] == np.float32(r_want) and bool(d[b]) == d_want, (t, b, acts[b], r[b], r_want)
                assert search_ref.isclose_dicts(_norm(inf[b]["raw_obs"]), _norm(raw_want)), (t, b, acts[b])
                assert inf[b]["action_mask"] == eps[b].mask()
                assert inf[b]["action"] == int(acts[b]) and inf[b]["step"] == t + 1
            for b in range(E):  # an action that keeps the observation returns the same object (prev_raw)
                if int(acts[b]) not in (0, 1, 2, 3, 4):
                    assert inf[b]["raw_obs"] is prev_raw[b]
            prev_raw = [inf[b]["raw_obs"] for b in range(E)]
    # state views
    assert venv.envs[0].env.step_count == venv._steps[0]
    assert all(isinstance(x, str) for x in venv.envs[0].env.frontier_set)
