"""Experiment: what a tighter admission threshold buys the fused tile kernel (C2 shape).

The production seed is the k-th best 16-row group maximum over the first S = 8,192 rows (a valid
lower bound that admits ~110 rows per query on this data). Here the seed comes instead from a
coarse-cluster probe computed with torch on the GPU (k-means centroids, the query's p nearest
clusters, the exact k-th best score among their members minus a rounding margin) and is handed to
the kernel through DenseIndex.set_seed (ahr_index_set_seed). Measures, per (clusters, probes):
survivors per query (rows scoring >= the seed), the tile kernel's event-timed duration, and that
the results equal the production path's. The torch probe itself is not timed (this bounds the
gain a device probe could bring). The second half times the product path (build_clusters ->
ahr_index_probe_seed -> seeded kernels) end to end, and a library GEMM + topk centroid search.
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


def tile_ms(ix, q, k, steps=20):
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
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--clusters", default="1024,4096")
    ap.add_argument("--probes", default="1,2,4")
    ap.add_argument("--probe-clusters", type=int, default=0, help="device path: nearest clusters per query (0: default)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    c = SyntheticCorpus(HOTPOT_90K, dev)
    rows = c.rows()
    N, d = rows.shape
    ix = DenseIndex(d, N, dtype="bf16", device=dev)
    ix.upsert(rows)
    q, _ = c.queries(a.batch, rows)
    k = a.k
    R = rows.to(torch.bfloat16).float()
    Q = q.to(torch.bfloat16).float()
    S = Q @ R.T  # [B, N] fp32 scores of the stored (rounded) vectors
    out = {"B": a.batch, "N": N, "k": k}
    ref = [t.clone() for t in ix.query(q, k)]
    base = tile_ms(ix, q, k)
    # production seed, restated: k-th largest 16-row group max over the first 8,192 rows
    gm = S[:, :8192].reshape(a.batch, -1, 16).amax(2)
    prod_seed = gm.topk(k, dim=1).values[:, -1]
    out["production"] = {"stages_ms": base, "survivors_per_query": float((S >= prod_seed[:, None]).sum(1).float().mean())}
    out["exact_kth_survivors"] = float((S >= S.topk(k, dim=1).values[:, -1:]).sum(1).float().mean())
    g = torch.Generator(device="cpu").manual_seed(7)
    for C in [int(x) for x in a.clusters.split(",")]:
        cent = R[torch.randperm(N, generator=g)[:C].to(dev)].clone()
        for _ in range(8):  # Lloyd iterations on the sphere
            asg = (R @ cent.T).argmax(1)
            acc = torch.zeros_like(cent).index_add_(0, asg, R)
            cnt = torch.bincount(asg, minlength=C)
            keep = cnt > 0
            cent[keep] = torch.nn.functional.normalize(acc[keep], dim=1)
        asg = (R @ cent.T).argmax(1)
        for p in [int(x) for x in a.probes.split(",")]:
            near = (Q @ cent.T).topk(p, dim=1).indices  # [B, p]
            member = (asg[None, :, None] == near[:, None, :]).any(2)  # [B, N]
            sm = S.masked_fill(~member, float("-inf"))
            kth = sm.topk(k, dim=1).values[:, -1]
            # the kernel sums the same exact bf16 products in another order: |difference| < 5e-5
            seed = torch.where(torch.isfinite(kth), kth - 1e-4 * (1 + kth.abs()), torch.full_like(kth, float("-inf")))
            seed = seed.contiguous()
            ix.set_seed(seed)
            got = ix.query(q, k)
            same = bool(torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]))
            st = tile_ms(ix, q, k)
            ix.set_seed(None)
            out[f"C{C}_p{p}"] = {"stages_ms": st, "same_results": same,
                                 "survivors_per_query": float((S >= seed[:, None]).sum(1).float().mean()),
                                 "weak_queries": int((~torch.isfinite(kth)).sum()),
                                 "probed_rows_per_query": float(member.sum(1).float().mean())}
    # the product path: DenseIndex.build_clusters -> per query batch a centroid top-8 search, the
    # probe kernel, the fused kernel seeded with its thresholds (all on the device, all timed)
    def wall(fn, steps=50):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3
    ix.drop_clusters()
    out["device_production_ms_per_batch"] = round(wall(lambda: ix.query(q, k)), 4)
    if a.probe_clusters:
        ix.PROBE_CLUSTERS = a.probe_clusters
    t0 = time.perf_counter()
    info = ix.build_clusters()
    torch.cuda.synchronize()
    out["device_clusters"] = dict(info, build_s=round(time.perf_counter() - t0, 2))
    got = ix.query(q, k)
    out["device_probe_same_results"] = bool(torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1]))
    out["device_probe_ms_per_batch"] = round(wall(lambda: ix.query(q, k)), 4)
    out["device_probe_stages_ms"] = tile_ms(ix, q, k)
    cl = ix._clusters
    out["device_centroid_search_ms"] = round(wall(lambda: cl["index"].query_keys(q, ix.PROBE_CLUSTERS)), 4)
    out["device_centroid_plus_probe_ms"] = round(wall(lambda: ix._probe_seed(q, k, False, None)), 4)
    # the centroid search seeded by its own sampled pre-pass (512 of its rows)
    cl["index"].set_sample_rows(512)
    out["device_centroid_search_prepass512_ms"] = round(wall(lambda: cl["index"].query_keys(q, ix.PROBE_CLUSTERS)), 4)
    out["device_probe_prepass512_ms_per_batch"] = round(wall(lambda: ix.query(q, k)), 4)
    cl["index"].set_sample_rows(-1)
    # a library GEMM (hipBLASLt through torch) + torch.topk for the same centroid top-P
    cent_bf = cl["index"].read().to(torch.bfloat16)
    qb = q.to(torch.bfloat16)
    out["library_centroid_gemm_topk_ms"] = round(wall(lambda: torch.topk(qb @ cent_bf.T, ix.PROBE_CLUSTERS, dim=1)), 4)
    out["library_centroid_gemm_ms"] = round(wall(lambda: qb @ cent_bf.T), 4)
    thr = ix._probe_seed(q, k, False, None)
    out["device_probe_survivors_per_query"] = float((S >= thr[:, None]).sum(1).float().mean())
    out["device_probe_weak_queries"] = int((~torch.isfinite(thr)).sum())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
