"""cProfile of the drop-in single-environment loop on the C5 workload (diagnostic).

AHRAGGymEnv stepped one environment at a time (tools/bench_env.py's `single` leg: reset at B = 1
with a precomputed query vector, then random valid actions), profiled over --envs episodes after
one warm-up episode; prints the wall rate and the top functions by own and cumulative time.
usage: python tools/profile_single_env.py [--envs 64] [--steps 6] [--search]
(--search: profile HierarchicalGraph.search_batch at B = 1, return_cluster=False, instead)
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ah-rag_amd"), ROOT, os.path.join(ROOT, "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench_env  # noqa: E402
from ah_rag.agent.gym_env import AHRAGGymEnv  # noqa: E402
from ah_rag.synthetic import HOTPOT_90K, SyntheticCorpus, build_hotpot_graph, install_vectors  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--search", action="store_true")
    ap.add_argument("--reps", type=int, default=1, help="timed loops (each rate printed)")
    ap.add_argument("--no-brief-cache", action="store_true",
                    help="A/B: build every node brief from the graph (the round-5 form)")
    ap.add_argument("--raw", action="store_true",
                    help="with --search: also time SearchEngine.run and the bare ahr_search_host call (the floor)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(7)
    corpus = SyntheticCorpus(HOTPOT_90K, dev)
    vectors = corpus.rows().cpu().numpy()
    hg, ids = build_hotpot_graph(corpus, np.random.default_rng(20251003))
    install_vectors(hg, ids, vectors, os.path.join(tempfile.mkdtemp(prefix="ahr_single_"), "vector_db"))
    q, _ = corpus.queries(a.envs + 1, corpus.rows())
    qv = q.cpu().numpy()
    env = AHRAGGymEnv(max_steps=a.steps + 1, graph=hg)
    env.env.logging_enabled = False
    if a.no_brief_cache:
        from ah_rag.graph_search import parse_judge

        def brief(node_id):
            d = hg.G.nodes.get(node_id, {})
            kind = d.get("node_type")
            return {"node_id": node_id, "node_type": kind, "entity_type": d.get("entity_type"),
                    "layer": 0 if kind == "entity" else (d.get("level") or (1 if kind == "summary" else 0)),
                    "title": d.get("title"), "name": d.get("name"),
                    "judge_overall": parse_judge(d.get("judge_scores")), "confidence": d.get("confidence")}
        env.env._node_brief = brief

    def episode(i):
        if a.search:
            hg.search_batch([f"q{i}"], top_k=5, member_top_m=5, query_vectors=qv[i:i + 1])
            return
        bench_env.single_reset(env, hg, f"q{i}", qv[i:i + 1])
        for _ in range(a.steps):
            env.step(bench_env.random_actions(rng, [env.get_action_mask()])[0])

    episode(a.envs)  # warm-up
    torch.cuda.synchronize()
    for rep in range(a.reps):
        t0 = time.perf_counter()
        for i in range(a.envs):
            episode(i)
        wall = time.perf_counter() - t0
        if a.reps > 1 and not a.search:
            print(f"rep {rep}: {a.envs * (1 + a.steps) / wall:.1f} env-steps/s", flush=True)
    prof = cProfile.Profile()
    prof.enable()
    for i in range(a.envs):
        episode(i)
    prof.disable()
    if a.search:
        print(f"search_batch B = 1: {a.envs / wall:.1f} calls/s ({wall / a.envs * 1e3:.4f} ms per call)", flush=True)
        if a.raw:
            from ah_rag import _native as nat
            from ah_rag.graph_search import resolve_search_params
            eng = hg.search_engine(hg.G.graph["vector_index"]["db_path"])
            params = resolve_search_params(hg.G.graph.get("search_params", {}), 5, 5, *([None] * 7))
            qt = torch.from_numpy(qv[:1].copy())
            eng.run(qt, params)
            t0 = time.perf_counter()
            for _ in range(a.envs):
                eng.run(qt, params)
            print(f"SearchEngine.run B = 1: {(time.perf_counter() - t0) / a.envs * 1e3:.4f} ms per call", flush=True)
            (key, b), = [(k, v) for k, v in eng._hbufs.items() if k[0] == 1]
            ws, ws_bytes, q_host, q_np, out = b[:5]
            c = params.to_c_cached()
            args = (eng.index.handle, eng.graph._h, q_host.data_ptr(), 1, key[2], eng.row_to_node.data_ptr(),
                    int(eng.row_to_node.shape[0]), nat.ctypes.byref(c), key[3], ws.data_ptr(), ws_bytes,
                    out.data_ptr(), nat.stream_ptr())
            fn = nat.lib().ahr_search_host
            t0 = time.perf_counter()
            for _ in range(a.envs):
                fn(*args)
            print(f"bare ahr_search_host B = 1: {(time.perf_counter() - t0) / a.envs * 1e3:.4f} ms per call", flush=True)
    else:
        print(f"single env: {a.envs * (1 + a.steps) / wall:.1f} env-steps/s "
              f"({wall / a.envs * 1e3:.3f} ms per episode of reset + {a.steps} steps)", flush=True)
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        pstats.Stats(prof, stream=s).sort_stats(key).print_stats(30)
        print(f"==== by {key}\n" + s.getvalue()[:7000], flush=True)


if __name__ == "__main__":
    main()
