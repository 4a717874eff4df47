"""Line-level host timing of VecAHRAGGymEnv.reset / step on the C5 setup (development aid).

bench_env.py's graph, 1,024 environments, three warm-up episodes, then 20 episodes (reset + 6 steps
of random valid actions) under a line tracer over reset / step / _featurize and the search path;
prints the 40 costliest lines in microseconds per episode (the tracer inflates short lines).
usage: python tools/env_host_lines.py"""
import os, sys, time, collections, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ah-rag_amd"), ROOT, os.path.join(ROOT, "tools")]
import numpy as np, torch
from bench_env import random_actions_batch
from ah_rag.synthetic import HOTPOT_90K, SyntheticCorpus, build_hotpot_graph, install_vectors
from ah_rag.agent import vec_env as V
from ah_rag.graph import hierarchical_graph as H
from ah_rag import graph_search as GS
dev = torch.device("cuda", 0)
corpus = SyntheticCorpus(HOTPOT_90K, dev)
vectors = corpus.rows().cpu().numpy()
hg, ids = build_hotpot_graph(corpus, np.random.default_rng(20251003))
install_vectors(hg, ids, vectors, os.path.join(tempfile.mkdtemp(), "vector_db"))
q, _ = corpus.queries(1024, corpus.rows())
q = q.contiguous()
queries = [f"q{i}" for i in range(1024)]
venv = V.VecAHRAGGymEnv(n_envs=1024, max_steps=7, graph=hg)
rng = np.random.default_rng(1)
def episode():
    venv.reset(queries, query_vectors=q)
    for _ in range(6):
        venv.step(random_actions_batch(rng, venv.action_masks()))
for _ in range(3): episode()
torch.cuda.synchronize()
codes = {f.__code__: f.__qualname__ for f in (V.VecAHRAGGymEnv.reset, V.VecAHRAGGymEnv.step, V.VecAHRAGGymEnv._featurize,
         H.HierarchicalGraph._search_arrays, GS.SearchEngine._run, GS.SearchEngine.run)}
acc = collections.Counter(); st = {}
def tr(frame, ev, arg):
    c = frame.f_code
    if c not in codes: return None
    key = id(frame)
    def lt(frame, ev, arg):
        now = time.perf_counter()
        l = st.get(key)
        if l is not None: acc[(codes[c], l[0])] += now - l[1]
        if ev == "line": st[key] = (frame.f_lineno, time.perf_counter())
        else: st.pop(key, None)
        return lt
    return lt
N = 20
sys.settrace(tr)
for _ in range(N): episode()
sys.settrace(None)
src = {}
for (fn, ln), t in acc.most_common(40):
    mod = V if fn.startswith("VecAHRAGGymEnv") else (H if fn.startswith("Hier") else GS)
    lines = src.setdefault(mod, open(mod.__file__).read().split("\n"))
    print(f"{t/N*1e6:8.1f} us/episode  {fn}:{ln}: {lines[ln-1].strip()[:90]}")
