"""How much of the register-resident kernel's time is the admission threshold (diagnostic).

Runs the C2 batch (90,000 rows, B = 1024, top-10) at d = 768 and 384 with the self-seeded default,
then with caller-supplied thresholds (ahr_index_set_seed; self-seeding off): the exact k-th best
score of each query as this kernel computes it (a perfect seed: no seeding events, no first-event
wait, the fewest survivors possible) and that score lowered by a margin (a looser, still valid
seed). The gap between the default and the perfect seed bounds what any seeding scheme can gain.
Tile-kernel stage event-timed (DenseIndex profile), alternating variants. Prints one JSON line.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ah-rag_amd"), ROOT]

import torch  # noqa: E402

from ah_rag.embeddings import DenseIndex  # noqa: E402
from ah_rag.synthetic import CorpusSpec, SyntheticCorpus  # noqa: E402


def tile_us(ix, q, k, steps=30):
    for _ in range(3):
        ix.query(q, k)
    torch.cuda.synchronize()
    ix.profile_begin(steps)
    for _ in range(steps):
        ix.query(q, k)
    torch.cuda.synchronize()
    p = ix.profile_end()
    return round(p["ms_sum"]["tile_topk"] / max(1, p["calls"]) * 1e3, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--margins", default="0,0.03,0.1,0.2,0.4")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = {}
    for dim in (768, 384):
        c = SyntheticCorpus(CorpusSpec(dim=dim), dev)
        rows = c.rows()
        q, _ = c.queries(1024, rows)
        ix = DenseIndex(dim, rows.shape[0], dtype="bf16", device=dev)
        ix.upsert(rows)
        s, _ = ix.query(q, 10)
        kth = s[:, 9].contiguous().clone()
        seeds = {m: (kth - float(m)).contiguous() for m in a.margins.split(",")}
        res = {}
        for _ in range(a.rounds):
            ix.set_seed(None)
            res.setdefault("self_seeded", []).append(tile_us(ix, q, 10))
            ix.set_debug_flags(1 << 26)  # seeded by the sampled pre-pass launch instead
            res.setdefault("prepass_seeded", []).append(tile_us(ix, q, 10))
            ix.set_debug_flags(1 << 27)  # self-seeded, the first event only
            res.setdefault("seed_first_event_only", []).append(tile_us(ix, q, 10))
            ix.set_debug_flags(1 << 23)  # qres forced: with no sample it would not be planned
            ix.set_sample_rows(0)  # no seed at all: each lane's own k-th best
            res.setdefault("unseeded", []).append(tile_us(ix, q, 10))
            ix.set_sample_rows(-1)
            ix.set_debug_flags(0)
            for m, t in seeds.items():
                ix.set_seed(t)
                res.setdefault(f"seed_kth_minus_{m}", []).append(tile_us(ix, q, 10))
            ix.set_seed(None)
        out[f"d{dim}"] = {kk: sorted(v) for kk, v in res.items()}
        # how far below the k-th best each seed sits: the pre-pass seed vs the kernel's k-th score
        out[f"d{dim}"]["kth_score_mean"] = round(float(kth.mean()), 4)
        out[f"d{dim}"]["plan"] = ix.plan(1024, 10)
        ix.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
