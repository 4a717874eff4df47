"""Streaming-kernel timing for one library build (same-box A/B aid, SURVEY §8d C2 batch sweep).

Times the B <= 16 path (topk_small_kernel bf16, topk_small_f32_kernel fp32) on the C2 corpus
(90,000 x 768) with HIP events around the tile-kernel stage (DenseIndex profile), warm (corpus
Infinity-Cache resident between queries) and cold (L2 + Infinity Cache flushed by a 512 MiB write
before every query, outside the events). Prints one JSON line. Run it alternately per build:
  AHR_LIB_PATH=<lib.so> python tools/small_ab.py [--reps 50]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ah-rag_amd"), ROOT]

import torch  # noqa: E402

from ah_rag.embeddings import DenseIndex  # noqa: E402
from ah_rag.synthetic import HOTPOT_90K, SyntheticCorpus  # noqa: E402


def stage_ms(ix, q, k, reps, flush=None, mode="read"):
    ix.query(q, k)
    torch.cuda.synchronize()
    ix.profile_begin(reps)
    for _ in range(reps):
        if flush is not None:
            if mode == "read":
                flush.amax()
            else:
                flush.fill_(1.0)
        ix.query(q, k)
    torch.cuda.synchronize()
    p = ix.profile_end()
    return {s: round(v / max(1, p["calls"]) * 1e3, 2) for s, v in p["ms_sum"].items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--batches", default="1,4,16")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    corpus = SyntheticCorpus(HOTPOT_90K, dev)
    rows = corpus.rows()
    q, _ = corpus.queries(16, rows)
    flush = torch.zeros(128 << 20, dtype=torch.float32, device=dev)
    out = {"lib": os.environ.get("AHR_LIB_PATH", "in-tree")}
    for dtype in ("bf16", "f32"):
        ix = DenseIndex(768, rows.shape[0], dtype=dtype, device=dev)
        ix.upsert(rows)
        for b in [int(x) for x in a.batches.split(",")]:
            if dtype == "f32" and b > 4:
                continue
            qb = q[:b].contiguous()
            plan = ix.plan(b, 10)["kernel"]
            warm = stage_ms(ix, qb, 10, a.reps)
            cold = stage_ms(ix, qb, 10, a.reps, flush, "read")
            dirty = stage_ms(ix, qb, 10, a.reps, flush, "write")
            out[f"{dtype}_b{b}"] = {"plan": plan, "warm_us": warm, "cold_us": cold, "cold_dirty_us": dirty}
        ix.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
