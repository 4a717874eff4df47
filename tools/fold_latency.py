"""Single-search latency with and without the small kernels' last-workgroup fold (C2 corpus).

Per storage type and batch (1, 4): wall time per call of back-to-back serial queries (one stream,
synchronised at the end), and of two batches in flight (two streams / workspaces), for the fold
(opt-in flag 8192) and the merge launch (the default), interleaved over rounds; best round reported.
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

FOLD = 8192


def timed(ix, q, k, calls, streams):
    for _ in range(10):
        ix.query(q, k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(calls):
        j = i % len(streams)
        ix.set_workspace(j)
        with torch.cuda.stream(streams[j]):
            ix.query(q, k)
    torch.cuda.synchronize()
    ix.set_workspace(0)
    return (time.perf_counter() - t0) / calls * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    c = SyntheticCorpus(HOTPOT_90K, dev)
    rows = c.rows()
    out = {}
    for dtype in ("bf16", "f32"):
        ix = DenseIndex(rows.shape[1], rows.shape[0], dtype=dtype, device=dev)
        ix.upsert(rows)
        for i in range(2):
            ix.set_workspace(i)
            ix.reserve(4, 16)
        ix.set_workspace(0)
        s2 = [torch.cuda.current_stream(dev), torch.cuda.Stream(device=dev)]
        for B in (1, 2, 4):
            q, _ = c.queries(B, rows)
            res = {}
            for _ in range(a.rounds):
                for name, flags in (("fold", FOLD), ("merge_launch", 0)):
                    ix.set_debug_flags(flags)
                    res.setdefault(name + "_serial_us", []).append(timed(ix, q, 10, a.calls, s2[:1]))
                    res.setdefault(name + "_inflight2_us", []).append(timed(ix, q, 10, a.calls, s2))
            ix.set_debug_flags(0)
            out[f"{dtype}_B{B}"] = {n: round(min(v), 2) for n, v in res.items()}
            print(json.dumps({f"{dtype}_B{B}": out[f"{dtype}_B{B}"]}), flush=True)
        ix.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
