"""Rerank scores that sit on 4-decimal half-way points (hierarchical_graph.py:766-781).

The reference evaluates `alpha*sem + beta*jt + gamma*ct + delta*boost` in CPython float64, where
every multiply and add rounds on its own, then applies round(x, 4) and sorts on the rounded
value. A device compiler that contracts `s + gamma*ct` into one fma rounds once instead of twice;
near a half-way point (x.xxxx5) that flips round(x, 4). The cases below are constructed so the
two evaluation orders round to DIFFERENT 4-decimal values (checked on the host with exact
rational arithmetic), so the GPU test only passes if the kernel keeps CPython's order and
rounding.
"""
import math
from fractions import Fraction

import numpy as np
import pytest


def _f(x):
    return Fraction(x)


def _fma(a, b, c):
    """Correctly rounded a*b + c (Python 3.10 has no math.fma): exact rational, one rounding."""
    return float(_f(a) * _f(b) + _f(c))


def ref_score(alpha, sem, gamma, ct):
    """The reference's expression with jt = 0 (judge None) and boost 0 (entity): CPython order."""
    s = alpha * sem
    s = s + 0.2 * 0.0
    s = s + gamma * ct
    s = s + 0.1 * 0.0
    return s


def contracted_score(alpha, sem, gamma, ct):
    s = alpha * sem
    s = _fma(0.2, 0.0, s)
    s = _fma(gamma, ct, s)
    return _fma(0.1, 0.0, s)


def sem_of(score32):
    """semantic = 1.0 - float(dist), dist = Chroma's float32 distance 1 - score."""
    return 1.0 - float(np.float32(1.0) - np.float32(score32))


def halfway_cases(n_cases=48, seed=7):
    """(score32, conf) pairs whose reference and fma-contracted rerank scores round apart."""
    rng = np.random.default_rng(seed)
    alpha, gamma = 0.6, 0.1
    out = []
    while len(out) < n_cases:
        s32 = float(np.float32(rng.uniform(0.2, 0.9)))
        sem = sem_of(s32)
        a = alpha * sem
        # aim a + gamma*ct at a half-way point (2m+1)/20000 just above a
        m = math.floor(a * 10000.0) + int(rng.integers(3, 40))
        target = (2 * m + 1) / 20000.0
        conf0 = (target - a) / gamma * 10.0
        c = conf0
        for _ in range(64):
            c = math.nextafter(c, -math.inf)
        for _ in range(128):
            ct = c / 10.0
            r = round(ref_score(alpha, sem, gamma, ct), 4)
            rc = round(contracted_score(alpha, sem, gamma, ct), 4)
            if r != rc:
                out.append((s32, c))
                break
            c = math.nextafter(c, math.inf)
    return alpha, gamma, out


def test_halfway_cases_discriminate():
    """CPU: every constructed case really separates CPython's order from an fma contraction."""
    alpha, gamma, cases = halfway_cases()
    assert len(cases) == 48
    for s32, conf in cases:
        sem, ct = sem_of(s32), conf / 10.0
        assert round(ref_score(alpha, sem, gamma, ct), 4) != round(contracted_score(alpha, sem, gamma, ct), 4)


@pytest.mark.gpu
def test_rerank_halfway_matches_cpython(cuda):
    import networkx as nx
    import torch

    from ah_rag.graph_search import DeviceGraph, RerankParams

    alpha, gamma, cases = halfway_cases()
    G = nx.DiGraph()
    for i, (_, conf) in enumerate(cases):
        G.add_node(f"ent:{i}", node_type="entity", name=f"E{i}", confidence=conf)
    dg = DeviceGraph(G, cuda)
    B = len(cases)
    seeds = torch.arange(B, dtype=torch.int32, device=cuda).view(B, 1)
    sems = torch.tensor([[s] for s, _ in cases], dtype=torch.float32, device=cuda)
    p = RerankParams(alpha=alpha, beta=0.2, gamma=gamma, delta=0.1, judge_min=None, confidence_min=None,
                     layer_boost={"entity": 0.0, "summary": 1.0, "hyperedge": 0.0}, type_filter=None,
                     member_top_m=5, top_k=1)
    res = dg.expand_rerank(seeds, sems, p).to_host()
    torch.cuda.synchronize()
    for b, (s32, conf) in enumerate(cases):
        sem = sem_of(s32)
        assert res.out_count[b] == 1
        assert res.exp_sem[b, 0] == sem, "seed semantic must be 1 - float32 distance"
        want = round(ref_score(alpha, sem, gamma, conf / 10.0), 4)
        assert res.out_score[b, 0] == want, (b, s32, conf, res.out_score[b, 0], want)
        assert res.out_sem[b, 0] == round(sem, 4)
    dg.close()
