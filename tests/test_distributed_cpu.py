"""world_size-2 gloo tests of the row-sharded search on CPU.

The HIP kernels cannot run here, so each rank's shard answers through a host stand-in built on
the oracle (HostShard: exact top-k -> packed keys with GLOBAL row ids, the device key format) and
the gathered lists are folded by a host key merge. Everything between is the product's own code:
the bench's rank launcher (ah_rag.distributed.launch), ShardedDenseIndex (shard bounds, global
upsert routing, row offsets) and its query() path — all_gather_keys' rank-major layout, the
[B, G, k] permute and the merge call. The result must equal the unsharded top-k, ties included.
"""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class HostShard:
    """CPU stand-in for the rank's DenseIndex (oracle top-k -> keys)."""

    def __init__(self, dim, capacity):
        self.rows = np.zeros((capacity, dim), np.float32)
        self.count = 0
        self.device = torch.device("cpu")

    def upsert(self, vectors, start=0, normalize=False):
        v = vectors.numpy() if isinstance(vectors, torch.Tensor) else np.asarray(vectors, np.float32)
        self.rows[start:start + len(v)] = v
        self.count = max(self.count, start + len(v))

    def query_keys(self, queries, k, row_base=0, out=None):
        from ah_rag.distributed import encode_keys_host
        from oracle import dense_ref
        s, r = dense_ref.topk(self.rows[:self.count], np.asarray(queries, np.float32), k, mode="fma")
        keys = encode_keys_host(s.astype(np.float32), np.where(r >= 0, r + row_base, -1))
        return torch.from_numpy(keys.view(np.int64).copy())

    def close(self):
        pass


def host_merge(keys, k):
    """[B, G, k_in] keys -> top k (scores, rows, keys): the merge rule of ahr_topk_merge."""
    from ah_rag.embeddings import decode_keys
    u = keys.numpy().view(np.uint64).reshape(keys.shape[0], -1)
    top = np.ascontiguousarray(np.sort(u, axis=1)[:, ::-1][:, :k])
    s, r = decode_keys(top)
    return torch.from_numpy(s), torch.from_numpy(r.astype(np.int32)), torch.from_numpy(top.view(np.int64))


def _rank_main(result_q):
    import torch.distributed as dist
    sys.path[:0] = [os.path.join(ROOT, "ah-rag_amd"), ROOT]
    dist.init_process_group("gloo")
    try:
        from ah_rag.distributed import ShardedDenseIndex, shard_bounds
        from oracle import dense_ref
        rank, world = dist.get_rank(), dist.get_world_size()
        rng = np.random.default_rng(11)
        C = dense_ref.normalize_rows(rng.standard_normal((5003, 64)))
        C[2495:2510] = C[17]          # exact duplicates straddling the shard boundary: tie order
        Q = dense_ref.normalize_rows(rng.standard_normal((9, 64)))
        Q[0] = C[17]
        k = 12
        lo, hi = shard_bounds(len(C), world)[rank]
        ix = ShardedDenseIndex(64, len(C), local=HostShard(64, hi - lo), merge=host_merge)
        for s0 in range(0, len(C), 1000):  # every rank is offered every chunk; keeps its own rows
            ix.upsert_global(s0, torch.from_numpy(C[s0:s0 + 1000]))
        s, r = ix.query(torch.from_numpy(Q), k)
        es, er = dense_ref.topk(C, Q, k, mode="fma")
        ok = bool(np.array_equal(r.numpy(), er) and np.array_equal(s.numpy(), es.astype(np.float32)))
        result_q.put((rank, ok, (ix.lo, ix.hi), int(ix.local.count)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_query_through_launcher(world):
    import torch.multiprocessing as mp
    sys.path[:0] = [os.path.join(ROOT, "ah-rag_amd"), ROOT]
    from ah_rag.distributed import launch
    q = mp.get_context("spawn").Queue()
    launch(world, _rank_main, (q,))
    res = sorted(q.get(timeout=60) for _ in range(world))
    assert all(ok for _, ok, _, _ in res), res
    assert [b for _, _, b, _ in res] == [(0, 2501), (2501, 5003)]
    assert [c for _, _, _, c in res] == [2501, 2502]


def test_shard_bounds_cover_exactly():
    from ah_rag.distributed import shard_bounds
    for n in (0, 1, 7, 90000, 5_000_000):
        for g in (1, 2, 3, 8):
            b = shard_bounds(n, g)
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(g - 1))
            assert max(h - l for l, h in b) - min(h - l for l, h in b) <= 1
