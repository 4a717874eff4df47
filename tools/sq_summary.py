"""Per-kernel means of rocprofv3 --pmc counter passes (tools/profile_sq.sh output).

Usage: python tools/sq_summary.py gpurun_out/sq_x [--kernel topk_] -> one JSON line per kernel:
counter -> mean per launch, plus derived ratios (fractions of wave cycles parked / issue-stalled /
active, MFMA busy per CU-busy cycle, LDS bank-conflict share, L2 hit rate).
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def short(name: str) -> str:
    m = re.search(r"ahr::(?:dense|graph)::(?:qres::)?(\w+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:50]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--kernel", default="topk_")
    a = ap.parse_args()
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(a.root, "**", "*_counter_collection.csv"), recursive=True):
        with open(path, newline="") as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                if a.kernel not in k:
                    continue
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in sorted(acc.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = {}
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in m:
                    d[c + "/wave"] = round(m[c] / wc, 4)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "SQ_BUSY_CU_CYCLES" in m:
            # MFMA busy cycles summed over SIMDs vs CU-busy quad-cycles (x4) per SIMD (x4)
            d["mfma_busy/cu_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["SQ_BUSY_CU_CYCLES"] * 4 * 4), 4)
        if "SQ_LDS_BANK_CONFLICT" in m and "SQ_LDS_IDX_ACTIVE" in m:
            d["lds_conflict/lds_active"] = round(m["SQ_LDS_BANK_CONFLICT"] / max(1.0, m["SQ_LDS_IDX_ACTIVE"]), 4)
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
            d["l2_hit"] = round(m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 4)
        if "GRBM_GUI_ACTIVE" in m:
            d["gui_active"] = m["GRBM_GUI_ACTIVE"]
        print(json.dumps({"kernel": k, "launches": len(next(iter(cs.values()))), "derived": d,
                          "counters": {c: round(v, 1) for c, v in sorted(m.items())}}))


if __name__ == "__main__":
    main()
