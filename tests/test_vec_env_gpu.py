"""The batched environment loop gives each environment exactly the reference episode
(tests/golden/gym_cases.json), while sharing one graph and one kernel launch per action kind."""
import json
import os
import shutil

import numpy as np
import pytest

from oracle.search_ref import isclose_dicts

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _norm(x):
    return json.loads(json.dumps(x, default=lambda o: o.tolist() if hasattr(o, "tolist") else str(o)))


def test_vec_env_matches_reference_episodes(tmp_path, cuda, monkeypatch):
    monkeypatch.setenv("AHR_ENCODER", "hash")
    monkeypatch.setenv("AHR_INDEX_DTYPE", "f32")
    from ah_rag.agent.vec_env import VecAHRAGGymEnv
    from ah_rag.graph.hierarchical_graph import HierarchicalGraph
    with open(os.path.join(GOLDEN, "gym_cases.json")) as f:
        eps = json.load(f)["cases"]
    shutil.copytree(os.path.join(GOLDEN, "reference_graph"), tmp_path / "graph")
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        hg = HierarchicalGraph.load("graph")
        hg.build_vector_index(db_path="vector_db", layers={0, 1}, upsert_only=False, reset=True)
        venv = VecAHRAGGymEnv("graph", n_envs=len(eps), graph=hg)
        vecs, infos = venv.reset([e["query"] for e in eps])
        for i, ep in enumerate(eps):
            np.testing.assert_array_equal(vecs[i], np.asarray(ep["reset"]["vec"], np.float32))
            assert isclose_dicts(_norm(infos[i]), ep["reset"]["info"])
        n_steps = max(len(ep["steps"]) for ep in eps)
        for t in range(n_steps):
            acts = [ep["steps"][t]["action"] if t < len(ep["steps"]) else 5 for ep in eps]
            v, r, d, inf = venv.step(acts)
            for i, ep in enumerate(eps):
                if t < len(ep["steps"]):
                    st = ep["steps"][t]
                    np.testing.assert_array_equal(v[i], np.asarray(st["vec"], np.float32))
                    assert r[i] == np.float32(st["reward"]) and bool(d[i]) == st["done"]
                    assert isclose_dicts(_norm(inf[i]), st["info"])
    finally:
        os.chdir(cwd)
