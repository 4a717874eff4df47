"""oracle/ — CPU restatement of the reference's hot-path algorithms: TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package,
and only as the checker. The product path (ah-rag_amd/) never imports it and has no CPU fallback.

Parity anchors:
  * dense top-k (ahr_oracle.c / dense_ref.py): restates an exhaustive Chroma cosine query
    (reference hierarchical_graph.py:611,714). Chroma itself is un-vendored and unpinned, so the
    dense step is pinned by known-answer properties (self-match at rank 0, tie order, shard
    invariance) and by golden outputs of the reference's own search() run under an exact stub
    collection (tests/golden/make_golden.py).
  * search tail / env / featurizer (search_ref.py): restates hierarchical_graph.py:719-789,
    environment.py:118-480, gym_env.py:85-125, featurizer.py:7-56, reward.py:6-26; pinned by the
    same golden fixtures.
"""
