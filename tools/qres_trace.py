"""Per-workgroup timeline of one topk_qres_kernel launch (development aid, the ablation build).

Thread 0 of every workgroup stamps s_memrealtime (100 MHz) at entry, at loop entry, after every
stage sync (a stage = one 32-row block at d = 768, two at d = 384) and around the first seeding event, and s_memtime at entry and exit (kFlagQresTrace,
ahr_qres.hip ABL_TRACE). Prints the launch skew, the per-block interval profile over the split
(median / p90 over workgroups), the first event's parts and the shader clock.

usage: python tools/qres_trace.py [--workload hotpot90k|hotpot90k_d384|synth5m] [--batch 1024]
                                  [--flags 0] [--json out.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("AHR_LIB_PATH", os.path.join(ROOT, "ah-rag_amd", "ah_rag", "_lib", "ablation", "libahr_hip.so"))
sys.path[:0] = [os.path.join(ROOT, "ah-rag_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ah_rag.embeddings import DenseIndex  # noqa: E402
from ah_rag.synthetic import HOTPOT_90K, SYNTH_5M, CorpusSpec, SyntheticCorpus  # noqa: E402

TRACE = 1 << 29
TICK_US = 0.01  # s_memrealtime: 100 MHz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="hotpot90k")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--flags", type=lambda s: int(s, 0), default=0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    spec = {"hotpot90k": HOTPOT_90K, "hotpot90k_d384": CorpusSpec(dim=384), "synth5m": SYNTH_5M}[a.workload]
    dtype = "f16" if a.workload == "synth5m" else "bf16"
    c = SyntheticCorpus(spec, dev)
    rows = c.rows()
    ix = DenseIndex(rows.shape[1], rows.shape[0], dtype=dtype, device=dev)
    for s in range(0, rows.shape[0], 1_000_000):
        ix.upsert(rows[s:s + 1_000_000], start=s)
    q, _ = c.queries(a.batch, rows)
    plan = ix.plan(a.batch, a.k)
    assert plan["kernel"] == "qres256", plan
    grid = plan["n_splits"] * plan["qblocks"]
    trace = torch.zeros(grid * 64, dtype=torch.int64, device=dev)
    os.environ["AHR_QRES_TRACE_PTR"] = "%x" % trace.data_ptr()
    ix.set_debug_flags(TRACE | a.flags)
    out = {"workload": a.workload, "batch": a.batch, "flags": a.flags, "plan": plan, "reps": []}
    for _ in range(3):
        ix.query(q, a.k)
    torch.cuda.synchronize()
    for rep in range(a.reps):
        trace.zero_()
        ix.query(q, a.k)
        torch.cuda.synchronize()
        t = trace.view(grid, 64).cpu().numpy().astype(np.int64)
        t0 = t[:, 0].min()
        us = lambda x: (x - t0) * TICK_US  # noqa: E731
        # ring stages: a stage holds two blocks at d = 384 (kPB = 2), one at 768
        pb = 2 if a.workload == "hotpot90k_d384" else 1
        n_st = (plan["tiles_per_split"] + pb - 1) // pb
        js = min(n_st, 55)
        stage = t[:, 3:3 + js + 1]
        d = np.diff(stage, axis=1) * TICK_US  # interval j-1 -> j: block j-1's MMA + block j-2's screening (SPB 1)
        dur = (t[:, 62] - t[:, 0]) * TICK_US
        clk = (t[:, 63] - t[:, 1]) / np.maximum(dur, 1e-9)  # s_memtime ticks per us
        r = {
            "entry_skew_us": [round(float(np.percentile(us(t[:, 0]), p)), 2) for p in (50, 90, 100)],
            "loop_entry_us": [round(float(np.percentile(us(t[:, 2]), p)), 2) for p in (0, 50, 100)],
            "exit_us": [round(float(np.percentile(us(t[:, 62]), p)), 2) for p in (0, 50, 100)],
            "interval_median_us": [round(float(x), 3) for x in np.median(d, axis=0)],
            "interval_p90_us": [round(float(x), 3) for x in np.percentile(d, 90, axis=0)],
            "first_event_us": {
                "select": round(float(np.median((t[:, 60] - t[:, 59]) * TICK_US)), 3) if t[:, 59].any() else None,
                "select_max": round(float(np.max((t[:, 60] - t[:, 59]) * TICK_US)), 3) if t[:, 59].any() else None,
                "read": round(float(np.median((t[:, 61] - t[:, 60]) * TICK_US)), 3) if t[:, 59].any() else None,
                "read_max": round(float(np.max((t[:, 61] - t[:, 60]) * TICK_US)), 3) if t[:, 59].any() else None,
            },
            "tail_us": round(float(np.median(us(t[:, 62]) - us(t[:, 3 + js]))), 3),
            "memtime_ticks_per_us": round(float(np.median(clk)), 1),
        }
        # per workgroup (blockIdx order): exit relative to the first entry, for placement analyses
        r["wg_exit_us"] = [round(float(x), 2) for x in us(t[:, 62])]
        r["wg_entry_us"] = [round(float(x), 2) for x in us(t[:, 0])]
        r["wg_clk"] = [round(float(x), 1) for x in clk]  # s_memtime ticks per us, per workgroup
        x = np.arange(grid) & 7  # blockIdx -> XCD (round-robin dispatch)
        r["xcd_exit_median_us"] = [round(float(np.median(us(t[x == i, 62]))), 2) for i in range(8)]
        r["xcd_clk_median"] = [round(float(np.median(clk[x == i])), 1) for i in range(8)]
        r["xcd_steady_block_us"] = [round(float(np.median(d[x == i, -10:-2])), 3) for i in range(8)]
        out["reps"].append(r)
        print(json.dumps({kk: vv for kk, vv in r.items() if not kk.startswith("wg_")}))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
