"""C5 (BASELINE configs[4]) at its workload: the batched RL environment loop on the HotpotQA-
distractor-shaped graph (87k entities + 3k summaries indexed, ~40k unindexed
hyperedges, ~130k nodes), 64 environments x 6 scripted steps, every reset and every step checked
against the oracle:

  reset   dense top-5 of each query = oracle/ahr_oracle.c's exact fp32 fma chain over the 90k x 768
          corpus (the fp32 index is bit-exact), then search_ref.expand_rerank (hierarchical_graph.py:
          719-789) -> the whole search() cluster, the observation and its 84-d feature vector;
  steps   search_ref.GymEpisode (environment.py:118-150, :301-355, :393-480 via env_expand;
          gym_env.py:41-125; featurizer.py:21-56; reward.py:6-26): observation dicts, feature
          vectors bit for bit, rewards and done flags.

Reference loop: /root/reference/src/ah_rag/agent/policy_ppo.py:145,163-214 over
/root/reference/src/ah_rag/agent/environment.py:393-480.
"""
import json

import numpy as np
import pytest

from oracle import dense_ref as dr
from oracle import search_ref

pytestmark = pytest.mark.gpu

N_ENVS = 64
STEPS = 6
# scripted actions per (env, step): every action kind in every position; an env whose selection
# is empty (only end_episode valid) takes 5 instead
SCRIPT = [2, 0, 3, 1, 4, 2, 2, 1, 0, 3, 5, 4]


def _norm(x):
    return json.loads(json.dumps(x, default=lambda o: o.tolist() if hasattr(o, "tolist") else str(o)))


@pytest.fixture(scope="module")
def hotpot_env(cuda, tmp_path_factory):
    import torch
    from ah_rag.synthetic import HOTPOT_90K, SyntheticCorpus, build_hotpot_graph, install_vectors
    with pytest.MonkeyPatch.context() as mp:  # module-scoped: restored after this module
        mp.setenv("AHR_INDEX_DTYPE", "f32")  # the drop-in default (exact mode)
        corpus = SyntheticCorpus(HOTPOT_90K, cuda)
        rows = corpus.rows()
        vectors = rows.cpu().numpy()
        hg, ids = build_hotpot_graph(corpus, np.random.default_rng(20251003))
        db = str(tmp_path_factory.mktemp("c5") / "vector_db")
        install_vectors(hg, ids, vectors, db)
        q, _ = corpus.queries(N_ENVS, rows, salt=3)
        torch.cuda.synchronize()
        yield hg, ids, vectors, q.cpu().numpy()


def test_c5_hotpot_graph_shape(hotpot_env):
    hg, ids, vectors, _ = hotpot_env
    G = hg.G
    kinds = {}
    for _, d in G.nodes(data=True):
        kinds[d.get("node_type")] = kinds.get(d.get("node_type"), 0) + 1
    assert kinds["entity"] == 87_000 and kinds["summary"] == 3_000 and kinds["hyperedge"] > 35_000
    assert G.number_of_nodes() > 125_000 and len(ids) == vectors.shape[0] == 90_000


def test_c5_vec_env_episodes_match_oracle(hotpot_env):
    from ah_rag.agent.vec_env import VecAHRAGGymEnv
    hg, ids, vectors, qv = hotpot_env
    G = hg.G
    queries = [f"c5 query {i}" for i in range(N_ENVS)]
    venv = VecAHRAGGymEnv(n_envs=N_ENVS, max_steps=STEPS, graph=hg)
    vecs, infos = venv.reset(queries, query_vectors=qv)

    # oracle reset: exact dense top-5 (fp32 fma chain), Chroma's float32 distance, expand + rerank
    es, er = dr.topk(vectors, qv, 5, mode="fma")
    p = search_ref.resolve_params(G.graph.get("search_params", {}), top_k=5, member_top_m=5)
    metas = {n: hg._embedding_text(n)[1] for n in set(ids[r] for r in er.ravel())}
    eps = [search_ref.GymEpisode(G, max_steps=STEPS) for _ in range(N_ENVS)]
    n_expanded = 0
    for b in range(N_ENVS):
        dist = (np.float32(1.0) - es[b].astype(np.float32)).tolist()
        seeds = [{"node_id": ids[r], "semantic": 1.0 - float(x), "meta": metas[ids[r]]} for r, x in zip(er[b], dist)]
        cluster = search_ref.expand_rerank(G, seeds, p, return_cluster=True)
        n_expanded += len(cluster["expanded"]) - len(seeds)
        v_want, raw_want = eps[b].reset(cluster)
        np.testing.assert_array_equal(vecs[b], v_want)
        assert search_ref.isclose_dicts(_norm(infos[b]["raw_obs"]), _norm(raw_want)), b
        assert infos[b]["action_mask"] == eps[b].mask()
        # the cluster behind the observation, dict for dict
        got_cluster = venv.envs[b].env.last_results
        assert search_ref.isclose_dicts(_norm(got_cluster), _norm(cluster)), b
    assert n_expanded > 0  # the 1-hop expansion contributed entries

    kinds = np.zeros(6, int)
    for t in range(STEPS):
        acts = []
        for b in range(N_ENVS):
            a = SCRIPT[(b + 3 * t) % len(SCRIPT)]
            if eps[b].mask()[a] == 0:
                a = 5
            acts.append(a)
            kinds[a] += 1
        # (a list, or a policy's integer array: int64 / int32)
        v, r, d, inf = venv.step(acts if t % 2 == 0 else np.asarray(acts, np.int64 if t % 4 == 1 else np.int32))
        for b in range(N_ENVS):
            v_want, r_want, d_want, raw_want = eps[b].step(acts[b])
            np.testing.assert_array_equal(v[b], v_want)
            assert r[b] == np.float32(r_want) and bool(d[b]) == d_want, (t, b, acts[b])
            assert search_ref.isclose_dicts(_norm(inf[b]["raw_obs"]), _norm(raw_want)), (t, b, acts[b])
            assert inf[b]["action_mask"] == eps[b].mask()
    assert (kinds[:5] > 0).all(), kinds  # every action kind was exercised
    print(f"C5: {N_ENVS} envs x {STEPS} steps on {G.number_of_nodes()} nodes match the oracle; actions {kinds.tolist()}")


def test_search_host_fused_merge_equals_device_path(hotpot_env):
    """The one-call search path (host queries, ahr_search_host) merges the small-batch plan's 256
    per-split lists inside the rerank kernel; the device-tensor path launches the merge kernel and
    then the rerank (ahr_index_query + ahr_graph_expand_rerank_rows). Same rows, scores and result
    arrays bit for bit, for every small-plan batch (B <= 4) and several top_k (fused up to
    256 x top_k <= 2,048 keys: top_k 8 is fused, 10 and 16 take the merge launch inside the call;
    a member_top_m too large for the wave kernel takes the merge launch and the serial kernel)."""
    import torch
    from ah_rag.graph_search import resolve_search_params
    hg, ids, vectors, qv = hotpot_env
    db = hg.G.graph["vector_index"]["db_path"]
    eng = hg.search_engine(db)
    for top_k, m in ((1, 5), (5, 5), (8, 5), (10, 5), (16, 5), (8, 200), (2, 600)):
        params = resolve_search_params(hg.G.graph.get("search_params", {}), top_k, m, *([None] * 7))
        for B in (1, 2, 4):
            q = np.ascontiguousarray(qv[3 * B:4 * B], np.float32)
            rows_h, scores_h, res_h = eng.run(q, params)  # host path (fused where it fits)
            rows_d, scores_d, res_d = eng.run(torch.from_numpy(q).cuda(), params)  # device path
            assert np.array_equal(rows_h, rows_d) and np.array_equal(scores_h.view(np.uint32),
                                                                      scores_d.view(np.uint32)), (top_k, m, B)
            # (the arrays are written up to each query's count; past it the buffers hold leftovers)
            assert np.array_equal(res_h.exp_count, res_d.exp_count) and np.array_equal(res_h.out_count,
                                                                                       res_d.out_count), (top_k, m, B)
            for b in range(B):
                for f, cnt in (("exp_nodes", res_h.exp_count), ("exp_sem", res_h.exp_count),
                               ("exp_src", res_h.exp_count), ("out_nodes", res_h.out_count),
                               ("out_sem", res_h.out_count), ("out_score", res_h.out_count)):
                    n = int(cnt[b])
                    a, d = np.asarray(getattr(res_h, f))[b, :n], np.asarray(getattr(res_d, f))[b, :n]
                    assert np.array_equal(a.view(np.uint8), d.view(np.uint8)), (top_k, m, B, b, f)
    plan = eng.index.plan(1, 5)
    assert plan["kernel"] == "small" and plan["n_splits"] * 5 <= 2048, plan
