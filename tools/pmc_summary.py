"""Summarise rocprofv3 PMC passes (tools/profile_pmc.sh output) into profiles/pmc_traffic.json.

Per kernel and per launch (mean over launches):
  * HBM read bytes  = FETCH_SIZE (KiB) x 1024 x 2   — gfx950 FETCH_SIZE reports half the bytes of
    wide (16 B/lane) coalesced streaming reads (MI355X_MICROARCH.md §HBM); our corpus and query
    staging loads are exactly that pattern;
  * HBM write bytes = WRITE_SIZE (KiB) x 1024       — exact for 16-B stores; our partial-list stores
    are 8 B/lane (uncalibrated width, reported as measured);
  * MFMA work from SQ_INSTS_VALU_MFMA_MOPS_BF16 / _F16 (bf16 / f16 launches) and the matrix-core
    busy cycles SQ_VALU_MFMA_BUSY_CYCLES (summed over the 1024 SIMDs: 16 per 16x16x32 MFMA, 32 per
    32x32x16), as a fraction of 1024 SIMDs x the traced duration x the 2.4 GHz peak clock;
  * the kernel duration from the kernel trace.
Infinity-Cache hits are counted inside FETCH_SIZE (the counter sits on the L2's memory side), so
"HBM" here means "beyond L2".

Usage: python tools/pmc_summary.py gpurun_out/pmc5 [--out profiles/pmc_traffic.json]
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import re


def _rows(pattern: str):
    files = glob.glob(pattern)
    if not files:
        return []
    with open(files[0], newline="") as f:
        return list(csv.DictReader(f))


def _short(name: str) -> str:
    m = re.search(r"ahr::(?:dense|graph)::(?:qres::)?(\w+)(<[^>]*>)?", name)
    if not m:
        return name[:60]
    return m.group(1) + (m.group(2) or "")


def counters(pattern: str):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in _rows(pattern):
        agg[_short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def durations(pattern: str):
    out = {}
    for r in _rows(pattern):
        out[_short(r["Name"])] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--workload", default="hotpot90k", help="bench workload the passes ran (bench reads only a match)")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                   "profiles", "pmc_traffic.json"))
    ap.add_argument("--dt", type=int, default=None,
                    help="storage type of the measured launches (0 f32, 1 f16, 2 bf16; default: the workload's)")
    a = ap.parse_args()
    if a.dt is None:
        a.dt = 1 if a.workload == "synth5m" else 2
    fetch = counters(os.path.join(a.pmc_dir, "fetch", "*", "*_counter_collection.csv"))
    write = counters(os.path.join(a.pmc_dir, "write", "*", "*_counter_collection.csv"))
    sq = counters(os.path.join(a.pmc_dir, "sq", "*", "*_counter_collection.csv"))
    dur = durations(os.path.join(a.pmc_dir, "trace", "*", "*_kernel_stats.csv"))
    out = {"_method": ("FETCH_SIZE KiB x 1024 x 2 (gfx950 wide-read correction) + WRITE_SIZE KiB x 1024, "
                       "mean per launch, separate rocprofv3 --pmc passes; durations from --kernel-trace --stats"),
           "_source": a.pmc_dir, "_workload": a.workload, "_batch": a.batch, "_dt": a.dt}
    for k in sorted(set(fetch) | set(write) | set(dur)):
        base = k.split("<")[0]
        if base not in ("topk_tile_kernel", "topk_tilelane_kernel", "topk_lane_kernel", "topk_qkv_kernel", "topk_t256_kernel",
                        "topk_small_kernel", "topk_small_f32_kernel", "merge_block_kernel", "merge_lane_lists_kernel", "merge_heads_kernel",
                        "merge_kernel", "sample_kth_kernel", "convert_rows_kernel", "expand_rerank_kernel",
                        "expand_kernel", "topk_kb256_kernel", "reblock_kb_kernel", "lca_kernel",
                        "topk_qres_kernel", "topk_qres16_kernel", "convert_queries_frag_kernel"):
            continue
        rec = out.setdefault(base, {"variants": {}})
        f = fetch.get(k, {}).get("FETCH_SIZE", [])
        w = write.get(k, {}).get("WRITE_SIZE", [])
        mean = lambda c: (sum(c) / len(c)) if c else None  # noqa: E731
        mf = sq.get(k, {}).get("SQ_INSTS_VALU_MFMA_MOPS_BF16", [])
        mh = sq.get(k, {}).get("SQ_INSTS_VALU_MFMA_MOPS_F16", [])
        mb = sq.get(k, {}).get("SQ_VALU_MFMA_BUSY_CYCLES", [])
        v = {"launches": len(f) or len(w),
             "read_bytes_per_launch": (sum(f) / len(f)) * 1024 * 2 if f else None,
             "write_bytes_per_launch": (sum(w) / len(w)) * 1024 if w else None,
             "mfma_mops_bf16_per_launch": mean(mf),
             "mfma_mops_f16_per_launch": mean(mh),
             "mfma_busy_cycles_per_launch": mean(mb),
             "avg_us_trace": dur.get(k, {}).get("avg_us")}
        if v["mfma_busy_cycles_per_launch"] and v["avg_us_trace"]:
            v["mfma_busy_frac"] = round(v["mfma_busy_cycles_per_launch"] / (1024 * v["avg_us_trace"] * 1e-6 * 2.4e9), 4)
        if v["read_bytes_per_launch"] is not None and v["write_bytes_per_launch"] is not None:
            v["hbm_bytes_per_launch"] = v["read_bytes_per_launch"] + v["write_bytes_per_launch"]
        rec["variants"][k] = v
        # the workload's storage type (first template argument): bench.py's exact-fp32 line runs
        # the same kernels on an fp32 index in the same process and must not stand in for them
        same_dt = [v for n, v in rec["variants"].items() if re.match(r"\w+<%d[,>]" % a.dt, n)]
        best = max(same_dt or rec["variants"].values(), key=lambda x: x.get("avg_us_trace") or 0)
        rec["hbm_bytes_per_launch"] = best.get("hbm_bytes_per_launch")
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v.get("hbm_bytes_per_launch") for k, v in out.items() if not k.startswith("_")}))


if __name__ == "__main__":
    main()
