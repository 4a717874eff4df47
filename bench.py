#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X dense-retrieval hot path.

Metric (BASELINE.json): queries/sec + recall@10, d=768 HotpotQA corpus, 1/2/4/8 MI355X.

N = 1 (default; BASELINE.json configs[1]): HotpotQA-distractor-shaped corpus, 90,000 rows (87k
entity + 3k summary) x d=768 stored bf16 in HBM, batches of 1,024 queries, exact top-10 by inner
product of L2-normalised vectors (= cosine). One step = one batch through ahr_index_query (query
conversion, threshold pre-pass, fused MFMA Q.N^T + top-k tile kernel, cross-split merge). Inputs
are resident in HBM before the timed region.

N > 1 (BASELINE.json configs[3]): the 5M x 768 fp16 corpus (configs[2]) row-sharded over the N
GPUs of the node, one process per GPU. One step = local fused top-k on every rank -> RCCL
all-gather of the [B, 10] packed keys over xGMI -> on-device merge, all inside the timed region
(strong scaling: the job answers B queries per step). rank 0 also times the unsharded 5M search
on its own GPU in the same run (config.n1_same_workload_qps). `--shard queries` is the replica
mode instead (every rank a full corpus and its own batches, weak scaling).

Launch: the driver's `python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`, or
plain `python bench.py --gpus N`, which spawns the N rank processes itself before any GPU call.

The data is synthetic (no dataset or encoder weights offline). recall@10 is
measured against the exact fp32 ground truth of the fp32 source vectors, computed on the host
with numpy/BLAS (the reference's numpy path), on a sample of the batch.
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

from ah_rag.distributed import ShardedDenseIndex, launch  # noqa: E402
from ah_rag.embeddings import DenseIndex  # noqa: E402
from ah_rag.synthetic import HOTPOT_90K, SYNTH_5M, CorpusSpec, SyntheticCorpus  # noqa: E402

METRIC = "queries/sec + recall@10, d=768 HotpotQA corpus, 1/2/4/8 MI355X"
HOTPOT_90K_D384 = CorpusSpec(dim=384)  # the reference's default embedding width
MFMA_PEAK_TFLOPS = {"bf16": 2500.0, "f16": 2500.0, "f32": 157.3}  # MI355X_MICROARCH.md, dense
HBM_PEAK_GBS = 8000.0
KERNEL_NAMES = {"lane256": "topk_lane_kernel", "lane256x128": "topk_lane_kernel",
                "tilelane128": "topk_tilelane_kernel", "t256": "topk_t256_kernel",
                "qkv128": "topk_qkv_kernel", "kb256": "topk_kb256_kernel",
                "kb128": "topk_kb256_kernel", "qres256": "topk_qres_kernel"}


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--workload", choices=["hotpot90k", "hotpot90k_d384", "synth5m", "env"], default=None,
                    help="default: hotpot90k at N=1, synth5m (row-sharded) at N>1; hotpot90k_d384 = the same "
                         "corpus at the reference's default width d = 384; env = configs[4], the RL "
                         "environment loop (VecAHRAGGymEnv, replicas: --envs per GPU)")
    ap.add_argument("--envs", type=int, default=1024, help="--workload env: environments per GPU")
    ap.add_argument("--episodes", type=int, default=5, help="C5 line: timed episodes after a warm-up one")
    ap.add_argument("--clock-ramp", type=int, default=200,
                    help="untimed steps before the --warmup steps of the timed pass (the GPU reaches its working "
                         "clock; reported as config.clock_ramp_steps)")
    ap.add_argument("--no-sublines", action="store_true",
                    help="N=1 hotpot90k: skip the synth5m (configs[2]) and C5 env (configs[4]) sub-lines")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--dtype", choices=["bf16", "f16", "f32"], default=None)
    ap.add_argument("--shard", choices=["queries", "rows"], default=None,
                    help="N>1: rows (default; configs[3]) or queries (replicas)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl = RCCL (default); gloo only to rehearse several ranks on one GPU")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU baseline budget per leg (s)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-n1-ref", action="store_true", help="rows mode: skip the unsharded rank-0 timing")
    ap.add_argument("--no-f32-line", action="store_true",
                    help="N=1 hotpot90k: skip the exact-mode (fp32 index) line beside the bf16 headline")
    ap.add_argument("--no-batch-sweep", action="store_true",
                    help="N=1 hotpot90k: skip the B = 1 and B = 64 lines beside the B = 1024 headline")
    ap.add_argument("--inflight", type=int, default=0,
                    help="batches in flight (one stream + index workspace each); 0 = auto: 1 for the "
                         "register-resident plan (it fills every CU and the library orders its batches), else 2")
    ap.add_argument("--recall-queries", type=int, default=256)
    ap.add_argument("--probe-seeds", action="store_true",
                    help="seed the fused kernels from a coarse-cluster probe (DenseIndex.build_clusters, built "
                         "untimed with the index) instead of the sampled pre-pass; the probe runs inside every step")
    ap.add_argument("--probe-clusters", type=int, default=0,
                    help="with --probe-seeds: number of k-means clusters (0: rows / 22)")
    ap.add_argument("--sample-rows", type=int, default=-1,
                    help="threshold pre-pass sample rows (DenseIndex.set_sample_rows; -1 = automatic)")
    ap.add_argument("--debug-flags", type=int, default=0,
                    help="ablation/kernel-selection switches (DenseIndex.set_debug_flags); 0 in production")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------------------------
# host-side numpy path (the reference's CPU math: BLAS fp32 + argpartition, tie rule score desc /
# row asc) — used for the recall ground truth and timed as the CPU baseline
# ---------------------------------------------------------------------------------------------
def numpy_topk(corpus: np.ndarray, queries: np.ndarray, k: int, row_base: int = 0):
    s = np.asarray(queries, np.float32) @ np.asarray(corpus, np.float32).T
    k_eff = min(k, s.shape[1])
    part = np.argpartition(-s, k_eff - 1, axis=1)[:, :k_eff]
    ps = np.take_along_axis(s, part, axis=1)
    idx = np.empty_like(part)
    for b in range(s.shape[0]):
        idx[b] = part[b][np.lexsort((part[b], -ps[b]))]
    return np.take_along_axis(s, idx, axis=1), idx.astype(np.int64) + row_base


def cpu_baseline_chunked(chunks, queries: np.ndarray, k: int, n_rows: int, d: int):
    """(exact top-k rows, cpu_baseline) over a corpus too large to build twice: each chunk is
    brought to host memory untimed, then the reference math (fp32 BLAS Q @ C.T + argpartition, the
    running top-k merged with the tie rule) is timed on it with all of the process's BLAS threads.
    The sample is the queries given over the whole corpus."""
    info = host_info()
    best_s = np.full((len(queries), k), -np.inf, np.float32)
    best_r = np.full((len(queries), k), -1, np.int64)
    t_cpu = 0.0
    for s0, x in chunks:
        xh = np.ascontiguousarray(x.cpu().numpy())
        t0 = time.perf_counter()
        cs, cr = numpy_topk(xh, queries, k, row_base=s0)
        alls, allr = np.concatenate([best_s, cs], 1), np.concatenate([best_r, cr], 1)
        order = np.lexsort((allr, -alls), axis=1)[:, :k]
        best_s, best_r = np.take_along_axis(alls, order, 1), np.take_along_axis(allr, order, 1)
        t_cpu += time.perf_counter() - t0
    cpu = {"value": round(len(queries) / t_cpu, 2), "unit": "queries/s", "cores": info.get("blas_threads", 1),
           "kind": "port",
           "sample": (f"{len(queries)} queries of the batch over the full {n_rows}x{d} fp32 corpus (host-resident "
                      f"chunks; only the host math timed), numpy BLAS ({info.get('blas', 'unknown')}, "
                      f"{info.get('blas_threads')} threads) + argpartition top-{k} + running merge, {t_cpu:.1f}s"),
           "host": info}
    return best_r, cpu


def numpy_topk_chunked(chunks, queries: np.ndarray, k: int):
    """Exact fp32 top-k over a corpus given as (start, device rows) chunks, never held whole."""
    best_s = np.full((len(queries), k), -np.inf, np.float32)
    best_r = np.full((len(queries), k), -1, np.int64)
    for s0, x in chunks:
        cs, cr = numpy_topk(x.cpu().numpy(), queries, k, row_base=s0)
        alls, allr = np.concatenate([best_s, cs], 1), np.concatenate([best_r, cr], 1)
        order = np.lexsort((allr, -alls), axis=1)[:, :k]
        best_s, best_r = np.take_along_axis(alls, order, 1), np.take_along_axis(allr, order, 1)
    return best_s, best_r


def recall_at_k(got: np.ndarray, exact: np.ndarray) -> float:
    k = exact.shape[1]
    hits = [len(set(g.tolist()) & set(e.tolist())) for g, e in zip(got, exact)]
    return float(np.mean(hits) / k)


def host_info() -> dict:
    info = {"os_cpu_count": os.cpu_count(), "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except Exception:
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()
        info["cgroup_cpu_quota"] = None if quota == "max" else round(int(quota) / int(period), 2)
    except Exception:
        pass
    try:
        from threadpoolctl import threadpool_info
        blas = [i for i in threadpool_info() if i.get("user_api") == "blas"]
        if blas:
            info["blas"] = f"{blas[0].get('internal_api')} {blas[0].get('version')}"
            info["blas_threads"] = int(blas[0]["num_threads"])
    except Exception:
        pass
    return info


def cpu_baseline(rows: np.ndarray, queries: np.ndarray, k: int, budget_s: float, workload: str) -> dict:
    """The reference math on the host (BASELINE.md "CPU baseline plan"): fp32 BLAS Q @ C.T +
    argpartition top-k over the full corpus on all of the process's host threads, at B = 1024 and
    B = 1, and — for the HotpotQA-shaped graph — the same B = 1024 batches followed by the
    reference 1-hop expansion + rerank (hierarchical_graph.py:726-782, restated in
    oracle/search_ref.py) per query."""
    info = host_info()
    threads = info.get("blas_threads", int(os.environ.get("OMP_NUM_THREADS", "1")))

    def timed(bsz, extra=None, budget=budget_s):
        done, i, t0 = 0, 0, time.perf_counter()
        while True:
            off = (i * bsz) % max(1, len(queries) - bsz + 1)
            qs = queries[off:off + bsz]
            s, r = numpy_topk(rows, qs, k)
            if extra is not None:
                extra(s, r)
            done += len(qs)
            i += 1
            if time.perf_counter() - t0 >= budget and done >= bsz:
                break
        return done, time.perf_counter() - t0

    n_b, t_b = timed(min(1024, len(queries)))
    by_threads = {threads: round(n_b / t_b, 2)}
    # every host thread the process may use (the box reports far more CPUs than its cgroup quota:
    # both counts are timed and the faster one is the baseline)
    n_all = info.get("affinity_cpus") or os.cpu_count() or threads
    if n_all != threads:
        try:
            from threadpoolctl import threadpool_limits
            with threadpool_limits(limits=n_all, user_api="blas"):
                n_a, t_a = timed(min(1024, len(queries)), budget=budget_s / 2)
            by_threads[n_all] = round(n_a / t_a, 2)
        except Exception as e:  # noqa: BLE001 — report, keep the quota-sized number
            by_threads[n_all] = f"unavailable: {e}"
    best_threads = max((t for t, v in by_threads.items() if isinstance(v, float)), key=lambda t: by_threads[t])
    n_1, t_1 = timed(1, budget=budget_s / 2)
    out = {"value": by_threads[best_threads], "unit": "queries/s", "cores": best_threads, "kind": "port",
           "b1_queries_per_s": round(n_1 / t_1, 2), "b1024_queries_per_s_by_blas_threads": by_threads}
    sample = (f"B=1024: {n_b} queries over the full {rows.shape[0]}x{rows.shape[1]} fp32 corpus, numpy BLAS "
              f"({info.get('blas', 'unknown')}, {threads} threads; also {n_all} threads: {by_threads.get(n_all)}) "
              f"+ argpartition top-{k}, {t_b:.1f}s; B=1: {n_1} single-query calls, {t_1:.1f}s")
    if workload == "hotpot90k":
        from oracle import search_ref  # CPU baseline leg only
        from ah_rag.synthetic import build_hotpot_graph
        corpus = SyntheticCorpus(HOTPOT_90K, torch.device("cpu"))
        hg, ids = build_hotpot_graph(corpus)
        p = search_ref.resolve_params({}, top_k=k)

        def rerank(s, r):
            for sb, rb in zip(s, r):
                dist_ = (np.float32(1.0) - sb.astype(np.float32)).tolist()
                seeds = [{"node_id": ids[j], "semantic": 1.0 - float(dd), "meta": {}} for j, dd in zip(rb, dist_)]
                search_ref.expand_rerank(hg.G, seeds, p, return_cluster=False)

        n_r, t_r = timed(min(1024, len(queries)), rerank)
        out["with_expand_rerank_queries_per_s"] = round(n_r / t_r, 2)
        sample += (f"; dense + R5/R7 expansion + rerank (synthetic {hg.G.number_of_nodes()}-node graph): "
                   f"{n_r} queries, {t_r:.1f}s")
    out["sample"] = sample + f"; host {json.dumps(info)}"
    out["host"] = info
    return out


def _dense_topk(vectors: np.ndarray, q: np.ndarray, k: int):
    """The reference's dense step on the host at B = 1 (one Chroma query per env reset,
    hierarchical_graph.py:714), restated as numpy fp32 BLAS + argpartition, ties by row."""
    s = vectors @ q
    part = np.argpartition(-s, k - 1)[:k]
    order = part[np.lexsort((part, -s[part]))]
    return s[order], order


def cpu_env_baseline(hg, ids, vectors: np.ndarray, qv: np.ndarray, steps: int, budget_s: float = 10.0,
                     seed: int = 20251003) -> dict:
    """configs[4] on the host: the reference's environment loop (policy_ppo.py:163-214: every env
    reset, then stepped one after another), restated by the oracle (oracle/search_ref.py: the
    search() tail expand_rerank of hierarchical_graph.py:719-789, GymEpisode for environment.py:
    118-150, :301-355, :393-480 and gym_env.py:41-125) over the same networkx graph, with the dense
    top-5 of each reset as numpy fp32 BLAS over the same 90k x d fp32 vectors. Random valid actions
    as in the GPU line. Timed twice for half the budget each: with the graph's node/edge counts
    computed once, and recounted for every observation as the reference does (environment.py:
    136-139). `value` is the faster (counted-once) form."""
    from oracle import search_ref  # CPU baseline leg only
    G = hg.G
    p = search_ref.resolve_params(G.graph.get("search_params", {}), top_k=5, member_top_m=5)
    metas = {}

    def meta(nid):
        m = metas.get(nid)
        if m is None:
            m = metas[nid] = hg._embedding_text(nid)[1]
        return m

    def run(per_obs: bool, budget: float):
        rng = np.random.default_rng(seed)
        # one environment object reset per episode (policy_ppo.py:145 builds the envs once)
        ep = search_ref.GymEpisode(G, max_steps=steps + 1, counts_per_observation=per_obs)
        n_steps, i, t0 = 0, 0, time.perf_counter()
        while True:
            sc, rows = _dense_topk(vectors, qv[i % len(qv)], 5)
            dist = (np.float32(1.0) - sc.astype(np.float32)).tolist()
            seeds = [{"node_id": ids[r], "semantic": 1.0 - float(x), "meta": meta(ids[r])} for r, x in zip(rows, dist)]
            ep.reset(search_ref.expand_rerank(G, seeds, p, return_cluster=True))
            n_steps += 1
            for _ in range(steps):
                ep.step(int(rng.choice(np.flatnonzero(np.asarray(ep.mask())))))
                n_steps += 1
            i += 1
            dt = time.perf_counter() - t0
            if dt >= budget:
                return n_steps, i, dt

    info = host_info()
    s_once, e_once, t_once = run(False, budget_s / 2)
    s_obs, e_obs, t_obs = run(True, budget_s / 2)
    return {"value": round(s_once / t_once, 1), "unit": "env-steps/s", "cores": info.get("blas_threads", 1),
            "kind": "port",
            "reference_counts_per_observation_env_steps_per_s": round(s_obs / t_obs, 1),
            "sample": (f"{e_once} episodes (reset + {steps} random valid steps) stepped one env after another over the "
                       f"{G.number_of_nodes()}-node networkx graph, dense top-5 by numpy fp32 BLAS "
                       f"({info.get('blas', 'unknown')}, {info.get('blas_threads')} threads; the rest single-threaded "
                       f"Python) over {vectors.shape[0]}x{vectors.shape[1]}, {t_once:.1f}s; with the reference's "
                       f"per-observation node/edge recount: {e_obs} episodes, {t_obs:.1f}s"),
            "host": info}


def auto_inflight(ix, B: int, k: int) -> int:
    """Batches in flight for --inflight 0: one for the register-resident plan (its batches fill every
    CU and the library orders them across streams, so a second gains nothing), else two."""
    return 1 if ix.plan(B, k)["kernel"] == "qres256" else 2


def time_queries(ix, q, k: int, steps: int, warmup: int, inflight: int, dev):
    """Queries/s of `ix` on batch q with `inflight` batches in flight (one stream + workspace
    each), then a serial pass with per-stage HIP events."""
    B = q.shape[0]
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(device=dev) for _ in range(inflight - 1)]
    outs = [(torch.empty((B, k), dtype=torch.float32, device=dev), torch.empty((B, k), dtype=torch.int32, device=dev))
            for _ in range(inflight)]
    for i in range(inflight):
        ix.set_workspace(i)
        ix.reserve(B, k)
    ix.set_workspace(0)
    for st in streams[1:]:
        st.wait_stream(streams[0])

    def run_n(n):
        for j in range(n):
            i = j % inflight
            ix.set_workspace(i)
            with torch.cuda.stream(streams[i]):
                ix.query(q, k, out=outs[i])

    run_n(warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_n(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ix.set_workspace(0)
    res = ix.query(q, k)
    ix.profile_begin(steps)
    for _ in range(steps):
        ix.query(q, k)
    torch.cuda.synchronize()
    return dt, ix.profile_end(), res


def cold_kernel_ms(ix, q, k: int, reps: int, dev, dirty: bool = False) -> float:
    """Average event-timed tile-kernel time of `ix.query(q, k)` with L2 and the Infinity Cache
    flushed before every query, outside the kernel's events: by a 512 MiB read (the caches then
    hold clean lines of another buffer), or with dirty=True by a 512 MiB write (the query's reads
    then also pay the write-back of up to 256 MiB of dirty lines — not the kernel's traffic)."""
    flush = torch.zeros(128 << 20, dtype=torch.float32, device=dev)
    ix.query(q, k)
    torch.cuda.synchronize()
    ix.profile_begin(reps)
    for _ in range(reps):
        if dirty:
            flush.fill_(1.0)
        else:
            flush.amax()
        ix.query(q, k)
    torch.cuda.synchronize()
    prof = ix.profile_end()
    del flush
    return prof["ms_sum"]["tile_topk"] / max(1, prof["calls"])


def read_traffic(kernel: str, workload: str, batch: int, dt: int = None):
    """(per-launch HBM bytes of `kernel`, the summary file) from the newest committed PMC summary
    (profiles/) measured on this workload, batch and storage type (dt: 0 f32, 1 f16, 2 bf16; None =
    the workload's default), else (None, None). A committed measurement, not this run's: the file is
    reported beside the value. Summaries without a recorded "_dt" (before round 6) count as the
    workload's default type, or fp32 for the fp32-only kernel."""
    default_dt = 1 if workload == "synth5m" else 2
    want = default_dt if dt is None else dt
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "*", "pmc_traffic.json")), reverse=True)
    paths.append(os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    for path in paths:
        try:
            with open(path) as f:
                data = json.load(f)
        except Exception:
            continue
        if data.get("_workload", "hotpot90k") != workload or data.get("_batch", 1024) != batch:
            continue
        file_dt = data.get("_dt", 0 if kernel == "topk_small_f32_kernel" else default_dt)
        if file_dt != want:
            continue
        v = data.get(kernel, {}).get("hbm_bytes_per_launch")
        if v is not None:
            return v, os.path.relpath(path, ROOT)
    return None, None


def roofline(plan: dict, dtype: str, B: int, n_rows: int, d: int, k: int, tile_ms: float, workload: str) -> dict:
    """Roofline of the dominant (tile) kernel: algorithmic flops = 2*B*N*d and bytes = N*d*s +
    B*d*s + B*k*8 per launch over its event-timed average launch; bound = the
    lower of the two ceilings by arithmetic intensity against the ridge."""
    flops = 2.0 * B * n_rows * d
    achieved_tf = flops / (tile_ms * 1e-3) / 1e12
    peak = MFMA_PEAK_TFLOPS[dtype]
    elem = 4 if dtype == "f32" else 2
    alg_bytes = n_rows * d * elem + B * d * elem + B * k * 8
    kname = KERNEL_NAMES.get(plan["kernel"], "topk_tile_kernel")
    if plan["kernel"] == "small":
        kname = "topk_small_f32_kernel" if dtype == "f32" else "topk_small_kernel"
    # arithmetic intensity 2*B*N*d / (N*d*elem) against the ridge (peak flops / HBM bytes):
    # small batches are bound by the corpus stream
    hbm_bound = flops / alg_bytes < peak * 1e12 / (HBM_PEAK_GBS * 1e9)
    hbm_gbs = alg_bytes / (tile_ms * 1e-3) / 1e9
    traffic, traffic_src = read_traffic(kname, workload, B, {"f32": 0, "f16": 1, "bf16": 2}[dtype])
    return {
        "kernel": f"{kname} (fused {'VALU fma-chain' if kname == 'topk_small_f32_kernel' else 'MFMA'} "
                  f"Q.N^T + top-k, {plan['kernel']})",
        "bound": "hbm" if hbm_bound else "mfma",
        "achieved": round(hbm_gbs if hbm_bound else achieved_tf, 2),
        "peak": HBM_PEAK_GBS if hbm_bound else peak,
        "unit": "GB/s" if hbm_bound else "TFLOP/s",
        "frac": round(hbm_gbs / HBM_PEAK_GBS if hbm_bound else achieved_tf / peak, 4),
        "traffic": traffic,
        "traffic_source": traffic_src,
        "algorithmic_flops_per_launch": flops,
        "algorithmic_bytes_per_launch": alg_bytes,
        "hbm_equiv_GBs": round(hbm_gbs, 1),
        "mfma_TFLOPs": round(achieved_tf, 2),
        "avg_launch_ms": round(tile_ms, 5),
    }


def sub_line(args, dev, spec, dtype: str, workload: str, label: str) -> dict:
    """A workload beside the N = 1 headline, on this GPU, timed like the headline (inflight batches,
    then a serial pass with stage events): B = --batch, top --k, recall@k on 128 queries."""
    B, k = args.batch, args.k
    corpus = SyntheticCorpus(spec, dev)
    N, d = spec.n_rows, spec.dim
    rows = corpus.rows() if spec.n_summaries else None
    chunks = (lambda: [(0, rows)]) if rows is not None else corpus.entity_chunks
    ix = DenseIndex(d, N, dtype=dtype, device=dev)
    for s0, x in chunks():
        ix.upsert(x, start=s0)
    q, _ = corpus.queries(B, rows, salt=0)
    if N > 1_000_000:  # C3: ~7 ms per step, 20 steps = 0.14 s
        steps, warm = max(3, min(args.steps, 20)), max(1, min(args.warmup, 3))
    else:  # d = 384 at C2's size: ~0.12 ms per step — a 20-step region is one hiccup away from
        # doubling, and the clock needs the headline's ramp (untimed) first
        steps, warm = max(3, min(args.steps, 200)), max(args.warmup, min(args.clock_ramp, 200))
    dt, prof, res = time_queries(ix, q, k, steps, warm, args.inflight or auto_inflight(ix, B, k), dev)
    calls = max(1, prof["calls"])
    tile_ms = prof["ms_sum"]["tile_topk"] / calls
    nq = min(128, B)
    plan = ix.plan(B, k)
    ix.close()
    cpu = None
    if rows is None and not args.no_cpu_baseline:
        # the corpus is generated chunk by chunk: the recall ground truth and the CPU baseline come
        # from one pass, with only the host work on each host-resident chunk timed
        exact, cpu = cpu_baseline_chunked(chunks(), q[:nq].cpu().numpy(), k, N, d)
    else:
        _, exact = numpy_topk_chunked(chunks(), q[:nq].cpu().numpy(), k)
        if not args.no_cpu_baseline:  # the headline's host legs (B = 1024 and B = 1) on this corpus
            cpu = cpu_baseline(rows.cpu().numpy(), q.cpu().numpy(), k, args.cpu_seconds / 2, workload)
    return {
        "workload": label,
        "value": round(B * steps / dt, 1), "unit": "queries/s", "steps": steps, "untimed_steps_before": warm,
        "ms_per_step": round(dt / steps * 1e3, 4), "recall_at_10": round(recall_at_k(
            res[1][:nq].cpu().numpy().astype(np.int64), exact), 4),
        "launch": plan,
        "stages_ms_per_step": {kk: round(v / calls, 4) for kk, v in prof["ms_sum"].items()},
        "roofline": roofline(plan, dtype, B, N, d, k, tile_ms, workload),
        "cpu_baseline": cpu,
    }


def env_line(args, dev, rank: int = 0, world: int = 1) -> dict:
    """configs[4]: the RL environment loop (tools/bench_env.py measure): VecAHRAGGymEnv over the
    130k-node HotpotQA-shaped graph, `--envs` environments per GPU, plus the drop-in single-env rate."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_env  # noqa: E402
    cpu_fn = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu_fn = lambda *x: cpu_env_baseline(*x, budget_s=max(4.0, args.cpu_seconds))  # noqa: E731
    return bench_env.measure(dev, args.envs, 6, single=64, rank=rank, world=world, total_envs=args.envs * world,
                             backend=args.backend, episodes=max(1, args.episodes), cpu_baseline_fn=cpu_fn)


def run_env(args) -> None:
    """--workload env: configs[4] as the bench line (replicas: every GPU its own graph copy and
    --envs environments, no collective on the data path; weak scaling)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local_rank % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    r = env_line(args, dev, rank, world)
    if rank == 0:
        steps = r["steps_per_episode"] + 1  # the reset counts as one env step, as in the rate
        out = {
            "metric": r["metric"], "value": r["vec_env_steps_per_s"], "unit": "env-steps/s", "n_gpus": world,
            "steps": steps * r["episodes"], "warmup": steps, "ms_per_step": round(r["episode_s"] / steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": r["data"],
            "config": {"workload": "env: BASELINE configs[4], 2-hop expand + re-score inside the RL env loop",
                       "envs_per_gpu": r["envs_per_gpu"], "parallelism": r["parallelism"], "graph": r["graph"]},
            "c5": r, "roofline": None, "cpu_baseline": r.get("cpu_baseline"),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def run(args) -> None:
    if args.workload == "env":
        run_env(args)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    workload = args.workload or ("synth5m" if world > 1 else "hotpot90k")
    shard = args.shard or ("rows" if world > 1 else "queries")
    dev_index = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    spec = {"hotpot90k": HOTPOT_90K, "hotpot90k_d384": HOTPOT_90K_D384}.get(workload, SYNTH_5M)
    dtype = args.dtype or ("f16" if workload == "synth5m" else "bf16")
    B, k = args.batch, args.k
    corpus = SyntheticCorpus(spec, dev)
    N, d = spec.n_rows, spec.dim
    # The 5M corpus (no summary rows) is generated chunk by chunk (each chunk has its own seed)
    # and never held whole: a row-sharded rank generates and stores only its own shard. The 90k
    # corpus needs all entity rows for its summary rows, and is small.
    rows = corpus.rows() if spec.n_summaries else None

    def corpus_chunks(lo: int = 0, hi: int = N):
        if rows is not None:
            for s0 in range(lo, hi, 1_000_000):
                yield s0, rows[s0:min(hi, s0 + 1_000_000)]
        else:
            yield from corpus.entity_chunks(lo=lo, hi=hi)

    sharded = shard == "rows" and world > 1
    if sharded:
        index = ShardedDenseIndex(d, N, dtype=dtype, device=dev)
        lo, hi = index.lo, index.hi
        for s0, x in corpus_chunks(lo, hi):
            index.upsert_global(s0, x)
        local = index.local
    else:
        lo, hi = 0, N
        index = local = DenseIndex(d, N, dtype=dtype, device=dev)
        for s0, x in corpus_chunks():
            local.upsert(x, start=s0)
    if args.debug_flags:
        local.set_debug_flags(args.debug_flags)
    if args.sample_rows >= 0:
        local.set_sample_rows(args.sample_rows)
    clusters = None
    if args.probe_seeds:  # index build, like the corpus upsert: outside the timed region
        t_cl = time.perf_counter()
        clusters = local.build_clusters(args.probe_clusters or None)
        torch.cuda.synchronize()
        clusters["build_s"] = round(time.perf_counter() - t_cl, 2)
    salt = rank if shard == "queries" else 0
    q, src = corpus.queries(B, rows, salt=salt)
    # Batches in flight: batch i runs on stream i % inflight with index workspace i % inflight,
    # so the latency-bound stages of one batch (query conversion, pre-pass k-th selection, merge,
    # launch gaps) overlap the neighbouring batch's tile kernel. Every batch still runs the whole
    # path; only the order of independent batches' kernels on the GPU changes.
    # Row-sharded runs pipeline the same way: batch i's RCCL all-gather and merge overlap batch
    # i + 1's local search (the collective is ordered after the work of the batch's stream).
    inflight = args.inflight if args.inflight > 0 else (1 if not sharded and auto_inflight(local, B, k) == 1 else 2)
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(device=dev) for _ in range(inflight - 1)]
    outs = [(torch.empty((B, k), dtype=torch.float32, device=dev), torch.empty((B, k), dtype=torch.int32, device=dev))
            for _ in range(inflight)]
    keys = [torch.empty((B, k), dtype=torch.int64, device=dev) for _ in range(inflight)]
    for i in range(inflight):
        local.set_workspace(i)
        local.reserve(B, k)
    local.set_workspace(0)
    for st in streams[1:]:
        st.wait_stream(streams[0])  # queries and index are ready
    counter = [0]

    def step(depth: int):
        i = counter[0] % depth
        counter[0] += 1
        local.set_workspace(i)
        with torch.cuda.stream(streams[i]):  # current stream = the batch's stream: no cross-stream wait
            if sharded:  # local top-k -> RCCL all-gather over xGMI -> device merge
                return index.query(q, k, out_keys=keys[i])
            return local.query(q, k, out=outs[i])

    def timed(depth: int, warmup: int) -> float:
        for _ in range(warmup):
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

    # (the serial pass comes first: it gets the clock ramp, so the GPU is at its working clock)
    dt_serial = timed(1, args.clock_ramp + args.warmup) if inflight > 1 else None
    counter[0] = 0
    # (one batch in flight: no serial pass before it, so the ramp precedes the --warmup steps here)
    dt = timed(inflight, args.warmup if inflight > 1 else args.clock_ramp + args.warmup)
    local.set_workspace(0)
    res = step(1)
    torch.cuda.synchronize()
    got_rows = res[1].cpu().numpy().astype(np.int64)
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

    # the same workload unsharded on rank 0's GPU, same run (the N = 1 point of the C4 curve)
    n1_qps = None
    if sharded and rank == 0 and not args.no_n1_ref:
        full = DenseIndex(d, N, dtype=dtype, device=dev)
        for s0, x in corpus_chunks():
            full.upsert(x, start=s0)
        full.reserve(B, k)
        for _ in range(max(2, args.warmup)):
            full.query(q, k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            full.query(q, k)
        torch.cuda.synchronize()
        n1_qps = B * args.steps / (time.perf_counter() - t0)
        full.close()
    if world > 1:
        dist.barrier()

    if rank == 0:
        # ---- recall@10 against exact fp32 ground truth of the fp32 source vectors (untimed)
        nq = min(args.recall_queries if N <= 200_000 else min(args.recall_queries, 128), B)
        qh = q[:nq].cpu().numpy()
        if rows is not None:
            _, exact = numpy_topk(rows.cpu().numpy(), qh, k)
        else:
            _, exact = numpy_topk_chunked(corpus_chunks(), qh, k)
        got_global = got_rows[:nq] if sharded else got_rows[:nq] + lo
        rec = recall_at_k(got_global, exact)

        calls = max(1, prof["calls"])
        tile_ms = prof["ms_sum"]["tile_topk"] / calls
        n_local = hi - lo
        plan = local.plan(B, k)
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None,
            "dtype": dtype,
            "data": "synthetic (SURVEY.md §8d clustered generator, seed 20251003; no HotpotQA/encoder offline)",
            "recall_at_10": round(rec, 4),
            "config": {
                "workload": {"hotpot90k": "hotpot90k: HotpotQA-distractor-shaped corpus 87k entity + 3k summary rows",
                             "hotpot90k_d384": "hotpot90k_d384: the hotpot90k corpus at d = 384"}.get(
                                 workload, "synth5m: 5M-row synthetic corpus"),
                "corpus_rows": N, "dim": d, "batch": B, "top_k": k, "index_dtype": dtype,
                "parallelism": (f"rows{world}" if sharded else (f"queries{world}" if world > 1 else "single")),
                "launch": plan,
                "inflight": inflight,
                # untimed steps run before the --warmup steps of a timed pass (the step is ~0.15 ms: the
                # GPU's clock settles over the first few ms of load); warmup + clock_ramp_steps ran untimed
                "clock_ramp_steps": args.clock_ramp,
                "untimed_steps_before_timed_region": args.clock_ramp + args.warmup,
                "serial_ms_per_step": round((dt_serial or dt) / args.steps * 1e3, 4),
                "recall_queries": nq,
                "threshold_seed": (f"cluster probe ({clusters['clusters']} clusters, built in {clusters['build_s']} s)"
                                   if clusters else
                                   ("self-seeded inside the register-resident kernel (published split maxima; "
                                    "no pre-pass launch)" if plan["kernel"] == "qres256"
                                    and not args.debug_flags & (1 << 26) and args.sample_rows != 0
                                    else "sampled pre-pass")),
            },
            "stages_ms_per_step": {kk: round(v / calls, 4) for kk, v in prof["ms_sum"].items()},
            "roofline": roofline(plan, dtype, B, n_local, d, k, tile_ms, workload),
            "cpu_baseline": None,
        }
        if sharded:
            out["config"]["n1_same_workload_qps"] = round(n1_qps, 1) if n1_qps else None
            out["config"]["shard_rows"] = n_local
        if world == 1 and workload == "hotpot90k" and dtype != "f32" and not args.no_f32_line:
            # the exact mode beside the headline: fp32 index (the reference's arithmetic; rows and
            # scores bit-identical to the oracle's k-ordered fma chain), same corpus, queries, k
            f32 = DenseIndex(d, N, dtype="f32", device=dev)
            f32.upsert(rows)
            f_dt, f_prof, f_res = time_queries(f32, q, k, args.steps, args.warmup,
                                               args.inflight or auto_inflight(f32, B, k), dev)
            f_tile = f_prof["ms_sum"]["tile_topk"] / max(1, f_prof["calls"])
            f_plan = f32.plan(B, k)
            out["exact_fp32"] = {
                "value": round(B * args.steps / f_dt, 1), "unit": "queries/s",
                "ms_per_step": round(f_dt / args.steps * 1e3, 4),
                "recall_at_10": round(recall_at_k(f_res[1][:nq].cpu().numpy().astype(np.int64), exact), 4),
                "launch": f_plan,
                "tile_ms": round(f_tile, 4),
                "roofline": roofline(f_plan, "f32", B, N, d, k, f_tile, workload),
            }
            if not args.no_batch_sweep:
                # B = 1 on the fp32 index: the drop-in search() / GraphEnvironment default
                # (hierarchical_graph.py:712-714 per env reset), the exact-mode streaming kernel
                q1 = q[:1].contiguous()
                b_steps = args.steps * 4
                b_dt, b_prof, _ = time_queries(f32, q1, k, b_steps, args.warmup, args.inflight or auto_inflight(f32, 1, k), dev)
                b_calls = max(1, b_prof["calls"])
                b_plan = f32.plan(1, k)
                e1 = {"batch": 1, "value": round(b_steps / b_dt, 1), "unit": "queries/s",
                      "ms_per_step": round(b_dt / b_steps * 1e3, 4), "steps": b_steps, "launch": b_plan,
                      "stages_ms_per_step": {kk: round(v / b_calls, 4) for kk, v in b_prof["ms_sum"].items()},
                      "roofline": roofline(b_plan, "f32", 1, N, d, k, b_prof["ms_sum"]["tile_topk"] / b_calls, workload)}
                e1["roofline"]["note"] = "corpus Infinity-Cache resident between queries (warm)"
                cold_ms = cold_kernel_ms(f32, q1, k, max(10, args.steps), dev)
                e1["roofline_cold_caches"] = roofline(b_plan, "f32", 1, N, d, k, cold_ms, workload)
                e1["roofline_cold_caches"]["note"] = "L2 and Infinity Cache refilled with clean lines before each query"
                out["exact_fp32"]["batch1"] = e1
            f32.close()
        if world == 1 and workload == "hotpot90k" and not args.no_batch_sweep:
            # BASELINE.md's C2 batch sweep beside the B = 1024 headline: B = 1 (the drop-in
            # search() / RL reset; streaming kernel, HBM-bound) and B = 64 (tile path), same index
            out["batch_sweep"] = []
            for b in (1, 64):
                qb = q[:b].contiguous()
                b_steps = args.steps * 4
                b_dt, b_prof, _ = time_queries(local, qb, k, b_steps, args.warmup,
                                               args.inflight or auto_inflight(local, b, k), dev)
                b_calls = max(1, b_prof["calls"])
                b_plan = local.plan(b, k)
                entry = {
                    "batch": b, "value": round(b * b_steps / b_dt, 1), "unit": "queries/s",
                    "ms_per_step": round(b_dt / b_steps * 1e3, 4), "steps": b_steps, "launch": b_plan,
                    "stages_ms_per_step": {kk: round(v / b_calls, 4) for kk, v in b_prof["ms_sum"].items()},
                    "roofline": roofline(b_plan, dtype, b, N, d, k, b_prof["ms_sum"]["tile_topk"] / b_calls,
                                         workload)}
                if b == 1:
                    # back to back, the 138 MB corpus stays in the 256 MiB Infinity Cache, so the line
                    # above is not an HBM-roofline claim; the same kernel with L2 + Infinity Cache
                    # flushed before every query (a 512 MiB write, untimed) is
                    entry["roofline"]["note"] = "corpus Infinity-Cache resident between queries (warm)"
                    cold_ms = cold_kernel_ms(local, qb, k, max(10, args.steps), dev)
                    entry["roofline_cold_caches"] = roofline(b_plan, dtype, b, N, d, k, cold_ms, workload)
                    entry["roofline_cold_caches"]["note"] = ("L2 and Infinity Cache refilled with clean lines (a 512 MiB "
                                                             "read) before each query")
                    entry["roofline_cold_caches"]["avg_launch_ms_dirty_caches"] = round(
                        cold_kernel_ms(local, qb, k, max(10, args.steps), dev, dirty=True), 5)
                out["batch_sweep"].append(entry)
        if world == 1 and workload == "hotpot90k" and not args.no_sublines:
            # configs[2] and configs[4] under the driver's clock, beside the configs[1] headline
            local.close()
            index = None
            out["synth5m"] = sub_line(args, dev, SYNTH_5M, "f16", "synth5m",
                                      "synth5m: BASELINE configs[2], 5M x 768 fp16, synthetic (SURVEY §8d generator)")
            out["hotpot90k_d384"] = sub_line(args, dev, HOTPOT_90K_D384, "bf16", "hotpot90k_d384",
                                             "hotpot90k at d = 384 (the reference's default all-MiniLM-L6-v2 "
                                             "width, hierarchical_graph.py:50), bf16")
            out["c5_env"] = env_line(args, dev)
        if world == 1 and not args.no_cpu_baseline:
            nc = min(len(q), 1024)
            if rows is not None:
                host_rows = rows.cpu().numpy()
            else:  # assembled chunk by chunk on the host
                host_rows = np.empty((N, d), np.float32)
                for s0, x in corpus_chunks():
                    host_rows[s0:s0 + x.shape[0]] = x.cpu().numpy()
            out["cpu_baseline"] = cpu_baseline(host_rows, q[:nc].cpu().numpy(), k, args.cpu_seconds, workload)
            del host_rows
        print(json.dumps(out), flush=True)
    if index is not None:
        index.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main() -> None:
    args = parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU, spawned before this process touches the GPU
        launch(args.gpus, run, (args,))
        return
    run(args)


if __name__ == "__main__":
    main()
