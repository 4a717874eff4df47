"""Cluster-probe seeds vs the sampled pre-pass at several corpus sizes (C3 generator, f16, B = 1024).

For each row count: wall time per batch of back-to-back queries (one stream) without clusters and
with DenseIndex.build_clusters(rows / per_cluster) for each --per-cluster value, interleaved over
rounds (best round), plus the equality of the results. Sizes stand in for C4's per-rank shards
(5M / G rows on G GPUs).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ah-rag_amd"), ROOT]

import torch  # noqa: E402

from ah_rag.embeddings import DenseIndex  # noqa: E402
from ah_rag.synthetic import SYNTH_5M, SyntheticCorpus  # noqa: E402


def wall_ms(ix, q, k, steps):
    for _ in range(3):
        ix.query(q, k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ix.query(q, k)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="625000,1250000,2500000,5000000")
    ap.add_argument("--per-cluster", default="100")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    c = SyntheticCorpus(SYNTH_5M, dev)
    allrows = c.rows()
    for n in [int(x) for x in a.rows.split(",")]:
        rows = allrows[:n]
        ix = DenseIndex(rows.shape[1], n, dtype="f16", device=dev)
        for s in range(0, n, 1_000_000):
            ix.upsert(rows[s:s + 1_000_000], start=s)
        q, _ = c.queries(1024, rows)
        ref = [t.clone() for t in ix.query(q, 10)]
        line = {"rows": n}
        for pc in [int(x) for x in a.per_cluster.split(",")]:
            t0 = time.perf_counter()
            info = ix.build_clusters(max(16, n // pc))
            torch.cuda.synchronize()
            build_s = time.perf_counter() - t0
            got = ix.query(q, 10)
            same = bool(torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]))
            res = {"plain": [], "probe": []}
            cl = ix._clusters
            for _ in range(a.rounds):
                ix._clusters = None
                res["plain"].append(wall_ms(ix, q, 10, a.steps))
                ix._clusters = cl
                res["probe"].append(wall_ms(ix, q, 10, a.steps))
            ix.drop_clusters()
            line["plain_ms"] = round(min(res["plain"]), 4)
            line[f"probe_n/{pc}_ms"] = round(min(res["probe"]), 4)
            line[f"probe_n/{pc}"] = {"clusters": info["clusters"], "build_s": round(build_s, 2), "same": same}
        ix.close()
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
