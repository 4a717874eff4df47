"""Host-time split of the drop-in search() at B = 1 (diagnostic): the C5 graph and fp32 store of
tools/bench_env.py, then per call the pieces of HierarchicalGraph.search_batch timed on their own
(argument resolution, engine lookup, the native call, the result dicts) over N calls each.
usage: python tools/search_host_split.py [--n 2000]"""
import argparse
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ah-rag_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ah_rag.graph_search import resolve_search_params  # noqa: E402
from ah_rag.synthetic import HOTPOT_90K, SyntheticCorpus, build_hotpot_graph, install_vectors  # noqa: E402


def per_call(fn, n):
    fn()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    return round((time.perf_counter() - t) / n * 1e6, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    corpus = SyntheticCorpus(HOTPOT_90K, dev)
    vectors = corpus.rows().cpu().numpy()
    hg, ids = build_hotpot_graph(corpus, np.random.default_rng(20251003))
    install_vectors(hg, ids, vectors, os.path.join(tempfile.mkdtemp(prefix="ahr_split_"), "vector_db"))
    q, _ = corpus.queries(4, corpus.rows())
    qv = q.cpu().numpy()[:1]
    qt = torch.from_numpy(qv.copy())
    sp = hg.G.graph.get("search_params", {})
    db = hg.G.graph["vector_index"]["db_path"]
    eng, params, rows, scores, res = hg.search_arrays(["q"], top_k=5, member_top_m=5, query_vectors=qv)
    out = {
        "search_batch": per_call(lambda: hg.search_batch(["q"], top_k=5, member_top_m=5, query_vectors=qv), a.n),
        "search_arrays": per_call(lambda: hg.search_arrays(["q"], top_k=5, member_top_m=5, query_vectors=qv), a.n),
        "resolve_search_params": per_call(lambda: resolve_search_params(sp, 5, 5, *([None] * 7)), a.n),
        "search_engine": per_call(lambda: hg.search_engine(db), a.n),
        "engine.run": per_call(lambda: eng.run(qt, params), a.n),
        "engine.run(numpy, borrow)": per_call(lambda: eng.run(qv, params, borrow=True), a.n),
        "_assemble": per_call(lambda: hg._assemble(eng, rows[0], scores[0], res, 0, 5, False), a.n),
        "_assemble(return_cluster)": per_call(lambda: hg._assemble(eng, rows[0], scores[0], res, 0, 5, True), a.n),
    }
    # the pieces of SearchEngine._run_host (graph_search.py) on their own
    from ah_rag import _native as nat
    from ah_rag.graph_search import _host_views
    eng.run(qt, params)
    b = next(iter(eng._hbufs.values()))
    ws, ws_bytes, q_np, ob, out_np, specs, offs, fixed, _, q_host = b
    max_exp = specs[2][0][1]
    stream = nat.stream_ptr(device_index=dev.index)
    cp = params.to_c_cached()
    lib = nat.lib()

    def bare():
        lib.ahr_search_host(eng.index.handle, *fixed, nat.ctypes.byref(cp), max_exp, ws.data_ptr(), ws_bytes,
                            ob.data_ptr(), stream)

    out["native_call"] = per_call(bare, a.n)
    out["copy+views"] = per_call(lambda: _host_views(out_np.copy(), specs, offs), a.n)
    out["stream_ptr"] = per_call(lambda: nat.stream_ptr(device_index=dev.index), a.n)
    print(out, flush=True)


if __name__ == "__main__":
    main()
