"""world_size-2 gloo test of the row-sharded search protocol on CPU.

The device kernels cannot run here, so each rank computes its shard's top-k with the oracle and
the test exercises the product's distribution logic: shard_bounds, global row offsets, the key
packing, all_gather_keys' rank-major layout, and that merging the gathered lists by key equals
the unsharded top-k (ties included).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, result_q):
    import sys
    sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ah-rag_amd"),
                    os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ah_rag.distributed import all_gather_keys, encode_keys_host, shard_bounds
        from oracle import dense_ref
        rng = np.random.default_rng(11)
        C = dense_ref.normalize_rows(rng.standard_normal((5003, 64)))
        C[4000:4010] = C[17]          # exact duplicates across the shard boundary: tie order
        Q = dense_ref.normalize_rows(rng.standard_normal((9, 64)))
        Q[0] = C[17]
        k = 12
        lo, hi = shard_bounds(len(C), world)[rank]
        s, r = dense_ref.topk(C[lo:hi], Q, k, mode="fma")
        keys = encode_keys_host(s.astype(np.float32), np.where(r >= 0, r + lo, -1))
        g = all_gather_keys(torch.from_numpy(keys.view(np.int64)))
        merged = np.sort(g.numpy().view(np.uint64).transpose(1, 0, 2).reshape(len(Q), -1), axis=1)[:, ::-1][:, :k]
        es, er = dense_ref.topk(C, Q, k, mode="fma")
        want = encode_keys_host(es.astype(np.float32), er)
        result_q.put((rank, bool(np.array_equal(merged, want)), tuple(g.shape)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_row_sharded_gather_merge(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
    assert all(shape == (world, 9, 12) for _, _, shape in res)


def test_shard_bounds_cover_exactly():
    from ah_rag.distributed import shard_bounds
    for n in (0, 1, 7, 90000, 5_000_000):
        for g in (1, 2, 3, 8):
            b = shard_bounds(n, g)
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(g - 1))
            assert max(h - l for l, h in b) - min(h - l for l, h in b) <= 1
