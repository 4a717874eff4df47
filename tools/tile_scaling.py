"""Per-workgroup fixed cost vs per-tile cost of the dense kernels (diagnostic).

Times the tile stage at B queries over corpora of 32 * 128 * T rows (T tiles per split at the
B = 1024 plan of 32 splits) and fits time = fixed + per_tile * T, for the query-resident kernel
(debug flag 4096) and the lane-local tile kernel (flag 32).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ah-rag_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ah_rag.embeddings import DenseIndex  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--tiles", default="1,2,4,8,16,22")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    out = {}
    for name, flags in (("qkv", 4096), ("tilelane", 32)):
        pts = []
        for T in [int(t) for t in a.tiles.split(",")]:
            n = 32 * 128 * T
            C = torch.nn.functional.normalize(torch.randn(n, 768, device=dev, generator=g), dim=1)
            Q = torch.nn.functional.normalize(torch.randn(a.batch, 768, device=dev, generator=g), dim=1)
            ix = DenseIndex(768, n, dtype="bf16", device=dev)
            ix.upsert(C)
            ix.set_sample_rows(256)
            ix.set_debug_flags(flags)
            for _ in range(3):
                ix.query(Q, 10)
            torch.cuda.synchronize()
            ix.profile_begin(a.steps)
            for _ in range(a.steps):
                ix.query(Q, 10)
            torch.cuda.synchronize()
            p = ix.profile_end()
            ms = p["ms_sum"]["tile_topk"] / p["calls"]
            pts.append((T, ms * 1e3))
            ix.close()
        t = np.array([p[0] for p in pts], float)
        us = np.array([p[1] for p in pts], float)
        slope, icpt = np.polyfit(t, us, 1)
        out[name] = {"points_us": pts, "fixed_us": round(float(icpt), 2), "per_tile_us": round(float(slope), 3)}
        print(json.dumps({name: out[name]}), flush=True)


if __name__ == "__main__":
    main()
