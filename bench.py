#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X dense-retrieval hot path.

Metric (BASELINE.json): queries/sec + recall@10, d=768 HotpotQA corpus, 1/2/4/8 MI355X.
Workload (default, BASELINE.json configs[1]): HotpotQA-distractor-shaped graph corpus,
90,000 rows (87k entity + 3k summary) x d=768 stored bf16 in HBM, batch of 1,024 queries,
exact top-10 by inner product of L2-normalised vectors (= cosine), fused Q.N^T + top-k kernel.
One step = one batch through ahr_index_query (query conversion, threshold pre-pass, fused tile
kernel, cross-split merge). Inputs are resident in HBM before the timed region.

--workload synth5m runs configs[2] (5M x 768 fp16). --gpus N (launched by torch.distributed.run)
runs one process per GPU: --shard queries (default) gives every rank a corpus replica and its own
query batch (weak scaling, no collective on the data path); --shard rows splits the corpus rows
across ranks and merges the per-rank top-k with an RCCL all-gather (strong scaling, configs[3]).

The data is synthetic (no dataset or encoder weights offline).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "ah-rag_amd"), ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from ah_rag.distributed import ShardedDenseIndex, all_gather_keys  # noqa: E402
from ah_rag.embeddings import DenseIndex, merge_topk_keys  # noqa: E402
from ah_rag.synthetic import HOTPOT_90K, SYNTH_5M, SyntheticCorpus  # noqa: E402

METRIC = "queries/sec + recall@10, d=768 HotpotQA corpus, 1/2/4/8 MI355X"
MFMA_PEAK_TFLOPS = {"bf16": 2500.0, "f16": 2500.0, "f32": 157.3}  # MI355X_MICROARCH.md, dense
HBM_PEAK_GBS = 8000.0


def parse_args():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", choices=["hotpot90k", "synth5m"], default="hotpot90k")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--dtype", choices=["bf16", "f16", "f32"], default=None)
    ap.add_argument("--shard", choices=["queries", "rows"], default="queries")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl = RCCL (default); gloo only to rehearse several ranks on one GPU")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (s)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--inflight", type=int, default=2,
                    help="batches in flight (one stream + index workspace each); rows-sharded runs use 1")
    ap.add_argument("--recall-queries", type=int, default=256)
    ap.add_argument("--debug-flags", type=int, default=0,
                    help="ablation/kernel-selection switches (DenseIndex.set_debug_flags); 0 in production")
    return ap.parse_args()


def recall_at_k(got: np.ndarray, exact: np.ndarray) -> float:
    k = exact.shape[1]
    hits = [len(set(g.tolist()) & set(e.tolist())) for g, e in zip(got, exact)]
    return float(np.mean(hits) / k)


def cpu_baseline(rows: np.ndarray, queries: np.ndarray, k: int, budget_s: float) -> dict:
    """The reference math on the host: fp32 BLAS Q @ C.T + argpartition top-k (oracle port)."""
    from oracle import dense_ref  # checker / baseline only

    try:
        from threadpoolctl import threadpool_info
        blas = [i for i in threadpool_info() if i.get("user_api") == "blas"]
        threads = int(blas[0]["num_threads"]) if blas else 1
        blas_name = f"{blas[0].get('internal_api')} {blas[0].get('version')}" if blas else "unknown"
    except Exception:
        threads, blas_name = int(os.environ.get("OMP_NUM_THREADS", "1")), "unknown"
    chunk = 256
    done, t0 = 0, time.perf_counter()
    i = 0
    while True:
        qs = queries[(i * chunk) % len(queries):][:chunk]
        dense_ref.topk_numpy(rows, qs, k)
        done += len(qs)
        i += 1
        if time.perf_counter() - t0 >= budget_s and done >= chunk:
            break
    dt = time.perf_counter() - t0
    return {"value": round(done / dt, 2), "unit": "queries/s", "cores": threads, "kind": "port",
            "sample": (f"{done} queries in {chunk}-query batches over the full {rows.shape[0]}x{rows.shape[1]} "
                       f"fp32 corpus, numpy BLAS ({blas_name}, {threads} threads) + argpartition top-{k}; "
                       f"{dt:.1f}s; host os.cpu_count()={os.cpu_count()}")}


def read_traffic(kernel: str, workload: str, batch: int):
    """Per-launch HBM bytes of `kernel` from the committed PMC summary (profiles/), if it was
    measured on this workload and batch (else None)."""
    paths = [os.path.join(ROOT, "profiles", "pmc_traffic.json")]
    paths += sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "*", "pmc_traffic.json")))
    for path in paths:
        try:
            with open(path) as f:
                data = json.load(f)
        except Exception:
            continue
        if data.get("_workload", "hotpot90k") != workload or data.get("_batch", 1024) != batch:
            continue
        v = data.get(kernel, {}).get("hbm_bytes_per_launch")
        if v is not None:
            return v
    return None


def main() -> None:
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run (one process per GPU)")
    dev_index = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    spec = HOTPOT_90K if args.workload == "hotpot90k" else SYNTH_5M
    dtype = args.dtype or ("bf16" if args.workload == "hotpot90k" else "f16")
    B, k = args.batch, args.k
    corpus = SyntheticCorpus(spec, dev)
    rows = corpus.rows()
    N, d = rows.shape
    sharded = args.shard == "rows" and world > 1
    if sharded:
        index = ShardedDenseIndex(d, N, dtype=dtype, device=dev)
        lo, hi = index.lo, index.hi
        for s0 in range(0, N, 1_000_000):
            index.upsert_global(s0, rows[s0:min(N, s0 + 1_000_000)])
        local = index.local
    else:
        lo, hi = 0, N
        index = local = DenseIndex(d, N, dtype=dtype, device=dev)
        for s0 in range(0, N, 1_000_000):
            local.upsert(rows[s0:min(N, s0 + 1_000_000)], start=s0)
    if args.debug_flags:
        local.set_debug_flags(args.debug_flags)
    salt = rank if args.shard == "queries" else 0
    q, src = corpus.queries(B, rows, salt=salt)
    index.reserve(B, k)
    keys = torch.empty((B, k), dtype=torch.int64, device=dev)
    # Batches in flight: batch i runs on stream i % inflight with index workspace i % inflight,
    # so the latency-bound stages of one batch (query conversion, pre-pass k-th selection, merge,
    # launch gaps) overlap the neighbouring batch's tile kernel. Every batch still runs the whole
    # path; only the order of independent batches' kernels on the GPU changes.
    inflight = 1 if sharded else max(1, args.inflight)
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(device=dev) for _ in range(inflight - 1)]
    outs = [(torch.empty((B, k), dtype=torch.float32, device=dev), torch.empty((B, k), dtype=torch.int32, device=dev))
            for _ in range(inflight)]
    for i in range(inflight):
        local.set_workspace(i)
        local.reserve(B, k)
    local.set_workspace(0)
    for st in streams[1:]:
        st.wait_stream(streams[0])  # queries and index are ready
    counter = [0]

    def step(depth: int):
        if sharded:
            index.query_keys(q, k, out=keys)
            gathered = all_gather_keys(keys)                  # RCCL all-gather over xGMI
            s_, r_, _ = merge_topk_keys(gathered.permute(1, 0, 2).contiguous(), k)
            return s_, r_
        i = counter[0] % depth
        counter[0] += 1
        local.set_workspace(i)
        with torch.cuda.stream(streams[i]):  # current stream = the batch's stream: no cross-stream wait
            return local.query(q, k, out=outs[i])

    def timed(depth: int) -> float:
        for _ in range(args.warmup):
            step(depth)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(depth)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    dt_serial = timed(1) if inflight > 1 else None
    counter[0] = 0
    dt = timed(inflight)
    local.set_workspace(0)
    res = step(1)
    torch.cuda.synchronize()
    # Stage timings (HIP events between the kernels of a step) in a separate, untimed pass: the
    # event records themselves add ~6 us of GPU-side gap per stage boundary.
    local.profile_begin(args.steps)
    for _ in range(args.steps):
        step(1)
    torch.cuda.synchronize()
    prof = local.profile_end()
    if world > 1:
        t = torch.tensor([dt, dt_serial or 0.0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t[0].item())
        dt_serial = float(t[1].item()) if dt_serial is not None else None

    q_per_step = B * world if not sharded else B
    value = q_per_step * args.steps / dt

    # ---- recall@10 against exact fp32 ground truth of the fp32 source vectors (untimed)
    got_rows = res[1].cpu().numpy().astype(np.int64)
    nq = min(args.recall_queries, B)
    if N <= 200_000:
        from oracle import dense_ref
        _, exact = dense_ref.topk_numpy(rows.cpu().numpy(), q[:nq].cpu().numpy(), k)
    else:
        gt = DenseIndex(d, N, dtype="f32", device=dev)
        for s in range(0, N, 1_000_000):
            gt.upsert(rows[s:s + 1_000_000], start=s)
        exact = gt.query(q[:nq], k)[1].cpu().numpy().astype(np.int64)
        gt.close()
    if sharded:
        got_global = got_rows[:nq]
    else:
        got_global = got_rows[:nq] + lo
    rec = recall_at_k(got_global, exact)

    if rank == 0:
        calls = max(1, prof["calls"])
        tile_ms = prof["ms_sum"]["tile_topk"] / calls
        n_local = hi - lo
        flops = 2.0 * B * n_local * d
        achieved_tf = flops / (tile_ms * 1e-3) / 1e12
        peak = MFMA_PEAK_TFLOPS[dtype]
        elem = 4 if dtype == "f32" else 2
        alg_bytes = n_local * d * elem + B * d * elem + B * k * 8
        plan = local.plan(B, k)
        kname = {"lane256": "topk_lane_kernel", "lane256x128": "topk_lane_kernel",
                 "tilelane128": "topk_tilelane_kernel", "t256": "topk_t256_kernel",
                 "small": "topk_small_f32_kernel" if dtype == "f32" else "topk_small_kernel",
                 "qkv128": "topk_qkv_kernel"}.get(plan["kernel"], "topk_tile_kernel")
        # arithmetic intensity 2*B*N*d / (N*d*elem) against the ridge (peak flops / HBM bytes):
        # small batches are bound by the corpus stream
        hbm_bound = flops / alg_bytes < peak * 1e12 / (HBM_PEAK_GBS * 1e9)
        hbm_gbs = alg_bytes / (tile_ms * 1e-3) / 1e9
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak" if not sharded else "strong",
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic (SURVEY.md §8d clustered generator, seed 20251003; no HotpotQA/encoder offline)",
            "recall_at_10": round(rec, 4),
            "config": {
                "workload": ("hotpot90k: HotpotQA-distractor-shaped corpus 87k entity + 3k summary rows"
                             if args.workload == "hotpot90k" else "synth5m: 5M-row synthetic corpus"),
                "corpus_rows": N, "dim": d, "batch": B, "top_k": k, "index_dtype": dtype,
                "parallelism": (f"rows{world}" if sharded else (f"queries{world}" if world > 1 else "single")),
                "launch": plan,
                "inflight": inflight,
                "serial_ms_per_step": round(dt_serial / args.steps * 1e3, 4) if dt_serial else None,
            },
            "stages_ms_per_step": {kk: round(v / calls, 4) for kk, v in prof["ms_sum"].items()},
            "roofline": {
                "kernel": f"{kname} (fused {'VALU fma-chain' if kname == 'topk_small_f32_kernel' else 'MFMA'} Q.N^T + top-k, {plan['kernel']})",
                "bound": "hbm" if hbm_bound else "mfma",
                "achieved": round(hbm_gbs if hbm_bound else achieved_tf, 2),
                "peak": HBM_PEAK_GBS if hbm_bound else peak,
                "unit": "GB/s" if hbm_bound else "TFLOP/s",
                "frac": round(hbm_gbs / HBM_PEAK_GBS if hbm_bound else achieved_tf / peak, 4),
                "traffic": read_traffic(kname, args.workload, B),
                "algorithmic_flops_per_launch": flops,
                "algorithmic_bytes_per_launch": alg_bytes,
                "hbm_equiv_GBs": round(alg_bytes / (tile_ms * 1e-3) / 1e9, 1),
                "avg_launch_ms": round(tile_ms, 5),
            },
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            nc = min(len(q), 1024)
            out["cpu_baseline"] = cpu_baseline(rows.cpu().numpy(), q[:nc].cpu().numpy(), k, args.cpu_seconds)
        print(json.dumps(out), flush=True)
    index.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
