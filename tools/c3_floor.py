"""Where the C3 (synth5m) register-resident launch spends its time beyond the GEMM (diagnostic).

Alternating variants on one box: the self-seeded default, a caller-supplied perfect seed (each
query's exact k-th score: no events, the fewest survivors possible) and that seed lowered by a
margin, and — with the ablation build (AHR_LIB_PATH=.../_lib/ablation/libahr_hip.so) — the
GEMM-only switch (flag 2: no screening, wrong output). Tile-kernel stage event-timed. One JSON line.

usage: python tools/c3_floor.py [--workload synth5m] [--rounds 2] [--gemm]
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


def tile_ms(ix, q, k, steps):
    for _ in range(2):
        ix.query(q, k)
    torch.cuda.synchronize()
    ix.profile_begin(steps)
    for _ in range(steps):
        ix.query(q, k)
    torch.cuda.synchronize()
    p = ix.profile_end()
    return round(p["ms_sum"]["tile_topk"] / max(1, p["calls"]), 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="synth5m")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--margins", default="0,0.1")
    ap.add_argument("--gemm", action="store_true")
    ap.add_argument("--only", default="", help="run only this variant (self_seeded | perfect | gemm_only), for "
                                               "counter passes (rocprofv3 --pmc) of one launch kind")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    spec = {"hotpot90k": HOTPOT_90K, "hotpot90k_d384": CorpusSpec(dim=384), "synth5m": SYNTH_5M}[a.workload]
    c = SyntheticCorpus(spec, dev)
    rows = c.rows()
    q, _ = c.queries(1024, rows)
    ix = DenseIndex(rows.shape[1], rows.shape[0], dtype="f16" if a.workload == "synth5m" else "bf16", device=dev)
    for s in range(0, rows.shape[0], 1_000_000):
        ix.upsert(rows[s:s + 1_000_000], start=s)
    del rows
    s, _ = ix.query(q, 10)
    kth = s[:, 9].contiguous().clone()
    seeds = {m: (kth - float(m)).contiguous() for m in a.margins.split(",")}
    res = {}
    if a.only:
        if a.only == "perfect":
            ix.set_seed(seeds[a.margins.split(",")[0]])
        elif a.only == "gemm_only":
            ix.set_debug_flags(2)
        res[a.only] = [tile_ms(ix, q, 10, a.steps)]
        print(json.dumps(res), flush=True)
        ix.close()
        return
    for _ in range(a.rounds):
        ix.set_seed(None)
        res.setdefault("self_seeded", []).append(tile_ms(ix, q, 10, a.steps))
        for m, t in seeds.items():
            ix.set_seed(t)
            res.setdefault(f"seed_kth_minus_{m}", []).append(tile_ms(ix, q, 10, a.steps))
        ix.set_seed(None)
        if a.gemm:
            ix.set_debug_flags(2)
            res.setdefault("gemm_only", []).append(tile_ms(ix, q, 10, a.steps))
            ix.set_debug_flags(0)
    out = {kk: sorted(v) for kk, v in res.items()}
    out["workload"] = a.workload
    out["plan"] = ix.plan(1024, 10)
    out["kth_score_mean"] = round(float(kth.mean()), 4)
    ix.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
