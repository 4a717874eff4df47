"""L1 topic relations — host logic against the reference's own outputs.

ah_rag.aggregate.relations computes the centroid cosine matrix on the GPU; here its host side
(overlap scatter, rules, rounding, pair order, top-k, neighbour lists, artifacts) is fed the
oracle's cosines (the reference's per-pair float32 np.dot, oracle/relations_ref.py) and must
reproduce tests/golden/relations_cases.json exactly.
"""
import copy
import json
import os

import numpy as np
import pytest

from oracle import relations_ref
from ah_rag.aggregate import relations as rel

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "relations_cases.json")


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN, encoding="utf-8") as f:
        return json.load(f)


def test_overlap_matrix_matches_sets(golden):
    _, members, _, ids = rel._prepare(golden["l1_nodes"])
    ov = rel.overlap_matrix(ids, members)
    for i in range(len(ids)):
        for j in range(len(ids)):
            want = 0 if i == j else len(members[ids[i]] & members[ids[j]])
            assert ov[i, j] == want


@pytest.mark.parametrize("case", range(4))
def test_host_logic_reproduces_reference(golden, tmp_path, case):
    c = golden["cases"][case]
    nodes = copy.deepcopy(golden["l1_nodes"])
    ids, cos = relations_ref.cosine_matrix(nodes)
    _, members, conf, ids2 = rel._prepare(nodes)
    assert ids == ids2
    p = dict(min_overlap=3, min_jaccard=0.2, min_cosine=0.5, top_k=None)
    p.update(c["params"])
    ov = rel.overlap_matrix(ids, members)
    edges = rel.edges_from_matrices(ids, members, conf, cos, ov, p["min_overlap"], p["min_jaccard"], p["min_cosine"])
    edges = rel.finish(nodes, edges, p["top_k"], str(tmp_path))
    assert edges == c["edges"]
    assert {str(n["topic_id"]): n["neighbors"] for n in nodes} == c["neighbors"]
    with open(tmp_path / "l1_edges.json", encoding="utf-8") as f:
        assert json.load(f) == c["edges"]


def test_empty_input():
    assert rel.generate_l1_relations([]) == []
