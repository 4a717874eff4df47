"""C2 step with and without hipGraph replay (development aid).

The C2 bench step (query conversion, register-resident top-k, merge) issued eagerly on one stream
versus the same launches captured once into a hipGraph (torch.cuda.CUDAGraph: a graph of G steps)
and replayed. Same batch, same index, alternating variants after a clock ramp; ms per step from the
wall clock around K steps bracketed by synchronisations. One JSON line.

usage: python tools/graph_step.py [--steps 300] [--graph-steps 1,10] [--rounds 3]
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
from ah_rag.synthetic import HOTPOT_90K, SyntheticCorpus  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--graph-steps", default="1,10")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    c = SyntheticCorpus(HOTPOT_90K, dev)
    rows = c.rows()
    q, _ = c.queries(1024, rows)
    ix = DenseIndex(rows.shape[1], rows.shape[0], dtype="bf16", device=dev)
    ix.upsert(rows)
    ix.reserve(1024, 10)
    s = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize()
    graphs = {}
    for g in [int(x) for x in a.graph_steps.split(",")]:
        cg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(cg, stream=s):
            for _ in range(g):
                out = ix.query(q, 10, stream=s)
        graphs[g] = (cg, out)
    torch.cuda.synchronize()

    def eager(n):
        with torch.cuda.stream(s):
            for _ in range(n):
                ix.query(q, 10, stream=s)

    def replay(g, n):
        cg = graphs[g][0]
        with torch.cuda.stream(s):
            for _ in range(n // g):
                cg.replay()

    def timed(fn, *args):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fn(*args)
        torch.cuda.synchronize()
        return (time.perf_counter() - t) * 1e3

    eager(200)  # clock ramp
    res = {}
    for _ in range(a.rounds):
        res.setdefault("eager", []).append(round(timed(eager, a.steps) / a.steps, 4))
        for g in graphs:
            res.setdefault(f"graph{g}", []).append(round(timed(replay, g, a.steps) / (a.steps // g * g), 4))
    # the graph's results equal an eager query's
    ref = ix.query(q, 10)
    torch.cuda.synchronize()
    for g, (_, out) in graphs.items():
        graphs[g][0].replay()
        torch.cuda.synchronize()
        assert torch.equal(out[1], ref[1]) and torch.equal(out[0], ref[0]), g
    res["ms_per_step_best"] = {k: min(v) for k, v in res.items()}
    print(json.dumps(res), flush=True)
    ix.close()


if __name__ == "__main__":
    main()
