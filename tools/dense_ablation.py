"""Ablation timings of the dense search stages on one GPU (interleaved variants, one process).

Variants (--variants name:sample_rows:debug_flags,...): production; pre-pass sample sizes;
no threshold pre-pass (sample 0); GEMM only (flag 2: epilogue skipped, wrong output); the
glds-ring kernel (flag 4). Prints per-stage milliseconds (HIP events on the query stream; an
empty stage reads ~5 us) per variant and batch size.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ah-rag_amd"), ROOT]

import torch  # noqa: E402

from ah_rag.embeddings import DenseIndex  # noqa: E402
from ah_rag.synthetic import HOTPOT_90K, SYNTH_5M, CorpusSpec, SyntheticCorpus  # noqa: E402


def run(ix, q, k, steps):
    for _ in range(3):
        ix.query(q, k)
    torch.cuda.synchronize()
    ix.profile_begin(steps)
    for _ in range(steps):
        ix.query(q, k)
    torch.cuda.synchronize()
    p = ix.profile_end()
    return {s: round(v / p["calls"], 4) for s, v in p["ms_sum"].items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="hotpot90k")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--rows", type=int, default=0, help="use only the first ROWS corpus rows (0 = all)")
    ap.add_argument("--batches", default="1,64,256,1024,4096")
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="prod:-1:0,tile128:-1:8,kb256:-1:131072,no_prepass:0:0,gemm_only:-1:2,max_only:-1:256")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    spec = {"hotpot90k": HOTPOT_90K, "hotpot90k_d384": CorpusSpec(dim=384), "synth5m": SYNTH_5M}[a.workload]
    c = SyntheticCorpus(spec, dev)
    rows = c.rows()
    if a.rows:
        rows = rows[:a.rows].contiguous()
    ix = DenseIndex(rows.shape[1], rows.shape[0], dtype=a.dtype, device=dev)
    for s in range(0, rows.shape[0], 1_000_000):
        ix.upsert(rows[s:s + 1_000_000], start=s)
    variants = [(n, int(sr), int(fl)) for n, sr, fl in (v.split(":") for v in a.variants.split(","))]
    out = []
    for B in [int(x) for x in a.batches.split(",")]:
        q, _ = c.queries(B, rows)
        res = {}
        for r in range(a.rounds):
            for name, sample, flags in variants:
                ix.set_sample_rows(sample)
                ix.set_debug_flags(flags)
                t = run(ix, q, a.k, a.steps)
                res.setdefault(name, []).append(t)
        ix.set_sample_rows(-1)
        ix.set_debug_flags(0)
        best = {n: min(v, key=lambda d: sum(d.values())) for n, v in res.items()}
        flops = 2.0 * B * rows.shape[0] * rows.shape[1]
        line = {"B": B, "plan": ix.plan(B, a.k)}
        for n, t in best.items():
            line[n] = t
            line[n + "_tile_TFs"] = round(flops / (t["tile_topk"] * 1e-3) / 1e12, 1)
            line[n + "_qps"] = round(B / (sum(t.values()) * 1e-3))
        out.append(line)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
