"""Host cost of one C2 search call vs its GPU time (is the serial step host-bound?).

Times N back-to-back DenseIndex.query calls: the host-side enqueue time (no sync inside the loop)
and the wall time to completion, for the out= form bench.py uses.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ah-rag_amd"), ROOT]

import torch  # noqa: E402

from ah_rag.embeddings import DenseIndex  # noqa: E402
from ah_rag.synthetic import HOTPOT_90K, SyntheticCorpus  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    c = SyntheticCorpus(HOTPOT_90K, dev)
    rows = c.rows()
    ix = DenseIndex(rows.shape[1], rows.shape[0], dtype="bf16", device=dev)
    ix.upsert(rows)
    q, _ = c.queries(1024, rows)
    out = (torch.empty((1024, 10), dtype=torch.float32, device=dev), torch.empty((1024, 10), dtype=torch.int32, device=dev))
    ix.reserve(1024, 10)
    for _ in range(20):
        ix.query(q, 10, out=out)
    torch.cuda.synchronize()
    n = 200
    t0 = time.perf_counter()
    for _ in range(n):
        ix.query(q, 10, out=out)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print({"host_us_per_call": round((t1 - t0) / n * 1e6, 1), "wall_us_per_call": round((t2 - t0) / n * 1e6, 1)})


if __name__ == "__main__":
    main()
