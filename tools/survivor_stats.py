"""Survivor statistics of the threshold pre-pass on a bench workload (diagnostic).

For B queries: the pre-pass seed (k-th largest 16-row group max over the first S rows, groups as
the tile kernels form them) and, over the whole corpus, how many rows / 16-row groups per query
reach it — the work the top-k epilogue has to do. Scores via torch.mm on the GPU (fp32 accumulate).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ah-rag_amd"), ROOT]

import torch  # noqa: E402

from ah_rag.synthetic import HOTPOT_90K, SYNTH_5M, SyntheticCorpus  # noqa: E402


def group_ids(n):
    """Kernel grouping: within each 32-row block, lane half h holds rows 4h + (r&3) + 8(r>>2)."""
    r = torch.arange(n)
    blk, off = r // 32, r % 32
    half = (off // 4) % 2
    return blk * 2 + half


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="hotpot90k")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--sample", type=int, default=8192)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    spec = HOTPOT_90K if a.workload == "hotpot90k" else SYNTH_5M
    c = SyntheticCorpus(spec, dev)
    rows = c.rows()
    q, _ = c.queries(a.batch, rows)
    C = rows.to(torch.bfloat16)
    Q = q.to(torch.bfloat16)
    S = (Q.float() @ C[: min(len(C), 200_000)].float().T)  # [B, N] fp32
    n = S.shape[1]
    g = group_ids(a.sample).to(dev)
    gm = torch.full((a.batch, a.sample // 16), -float("inf"), device=dev)
    gm.scatter_reduce_(1, g.expand(a.batch, -1), S[:, : a.sample], reduce="amax")
    thr = gm.topk(a.k, dim=1).values[:, -1:]
    above = (S >= thr)
    per_q = above.sum(1).float()
    kth_true = S.topk(a.k, dim=1).values[:, -1:]
    ga = group_ids(n).to(dev)
    ng = int(ga.max()) + 1
    gmax = torch.full((a.batch, ng), -float("inf"), device=dev)
    gmax.scatter_reduce_(1, ga.expand(a.batch, -1), S, reduce="amax")
    groups = (gmax >= thr).sum(1).float()
    out = {"workload": a.workload, "B": a.batch, "k": a.k, "sample": a.sample, "rows": n,
           "rows_above_seed_mean": per_q.mean().item(), "rows_above_seed_p50": per_q.median().item(),
           "rows_above_seed_p99": per_q.quantile(0.99).item(), "rows_above_seed_max": per_q.max().item(),
           "groups_passing_mean": groups.mean().item(), "groups_passing_max": groups.max().item(),
           "seed_minus_true_kth_mean": (thr - kth_true).mean().item(),
           "rows_above_true_kth_mean": (S >= kth_true).sum(1).float().mean().item()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
