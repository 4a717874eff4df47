"""ah_rag.distributed — the corpus embedding matrix row-sharded across the GPUs of a node.

North star (BASELINE.json): "The corpus embedding matrix shards by rows across the 8 GPUs of one
node with an RCCL all-gather of local top-k over xGMI". One process per GPU (torch.distributed,
backend "nccl" = RCCL on ROCm). Rank g owns the contiguous rows [lo_g, hi_g); a query batch is
answered by
    local fused top-k on rank g   -> packed keys [B, k] with GLOBAL row ids (row_base = lo_g)
    RCCL all-gather               -> [G, B, k] on every rank (B*k*8 bytes per rank: 80 KB at
                                     B=1024, k=10 — latency-bound on xGMI)
    on-device k-way merge         -> top-k [B, k], identical to the unsharded result
The packed key orders (score desc, row asc), so the merge reproduces the single-GPU tie rule
bit for bit for any G (tests/test_dense_gpu.py::test_merge_matches_single_shard).

The reference has no distributed code at all (no NCCL/MPI/Gloo); this is new.
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .embeddings import DenseIndex, merge_topk_keys


def shard_bounds(n_rows: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous, balanced row blocks: rank g owns [g*n//G, (g+1)*n//G)."""
    if world <= 0:
        raise ValueError("world must be positive")
    return [(g * n_rows // world, (g + 1) * n_rows // world) for g in range(world)]


def encode_keys_host(scores: np.ndarray, rows: np.ndarray) -> np.ndarray:
    """Host packing of (fp32 score, row) into the device key format (ahr_common.h make_key)."""
    s = np.ascontiguousarray(scores, np.float32)
    u = s.view(np.uint32)
    ordv = np.where(u & np.uint32(0x80000000), ~u, u | np.uint32(0x80000000)).astype(np.uint64)
    keys = (ordv << np.uint64(32)) | (np.uint64(0xFFFFFFFF) - np.asarray(rows).astype(np.uint64))
    return np.where(np.asarray(rows) < 0, np.uint64(0), keys)


def all_gather_keys(keys: torch.Tensor, group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """[B, k] int64 keys on every rank -> [G, B, k] (rank-major). RCCL all_gather_into_tensor for
    device tensors; the list form for backends without it (gloo on CPU)."""
    world = dist.get_world_size(group)
    out = torch.empty((world,) + tuple(keys.shape), dtype=keys.dtype, device=keys.device)
    if keys.is_cuda and dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, keys.contiguous(), group=group)
    else:
        dist.all_gather(list(out.unbind(0)), keys.contiguous(), group=group)
    return out


def free_port() -> int:
    """An unused TCP port on 127.0.0.1 for the rendezvous of spawned ranks."""
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def _rank_entry(local_rank: int, world: int, port: int, target: Callable, args: tuple) -> None:
    os.environ.update({"RANK": str(local_rank), "LOCAL_RANK": str(local_rank), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this driver
    target(*args)


def launch(world: int, target: Callable, args: tuple = ()) -> None:
    """One process per rank on this node, torch.distributed.run-style environment (RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT), then target(*args) in each.

    Fresh interpreters (spawn start method): call this BEFORE anything in the parent touches the
    GPU (a process that initialised HIP must not fork or exec). Raises if any rank fails."""
    import torch.multiprocessing as mp
    mp.spawn(_rank_entry, args=(world, free_port(), target, args), nprocs=world, join=True)


class ShardedDenseIndex:
    """This rank's shard of a row-partitioned corpus + the gather/merge query path.

    `local` (default: a DenseIndex on this rank's GPU) answers the shard's top-k as packed keys
    with global row ids; `merge` (default: the on-device ahr_topk_merge) folds the gathered
    [B, G, k] lists. Both are injectable so the distribution logic runs on CPU ranks with a host
    stand-in (tests/test_distributed_cpu.py); the product path always uses the defaults."""

    def __init__(self, dim: int, n_rows: int, dtype: str = "bf16", group: Optional[dist.ProcessGroup] = None,
                 device: Optional[torch.device] = None, local=None, merge: Optional[Callable] = None) -> None:
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.n_rows = int(n_rows)
        self.lo, self.hi = shard_bounds(self.n_rows, self.world)[self.rank]
        self.local = local if local is not None else DenseIndex(dim, max(1, self.hi - self.lo), dtype=dtype,
                                                                device=device)
        self.device = self.local.device
        self._merge = merge or merge_topk_keys

    def upsert_global(self, start: int, vectors: torch.Tensor, normalize: bool = False) -> None:
        """Offer global rows [start, start + n); this rank keeps the part inside its shard."""
        n = vectors.shape[0]
        a, b = max(start, self.lo), min(start + n, self.hi)
        if a < b:
            self.local.upsert(vectors[a - start:b - start], start=a - self.lo, normalize=normalize)

    def reserve(self, max_batch: int, max_k: int) -> None:
        self.local.reserve(max_batch, max_k)

    def query_keys(self, queries: torch.Tensor, k: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        return self.local.query_keys(queries, k, row_base=self.lo, out=out)

    def query(self, queries: torch.Tensor, k: int, out_keys: Optional[torch.Tensor] = None
              ) -> Tuple[torch.Tensor, torch.Tensor]:
        """Global top-k of the batch (every rank gets the same answer): scores f32, rows int32."""
        keys = self.query_keys(queries, k, out=out_keys)
        gathered = all_gather_keys(keys, self.group)          # [G, B, k], RCCL over xGMI
        s, r, _ = self._merge(gathered.permute(1, 0, 2).contiguous(), k)
        return s, r

    def close(self) -> None:
        self.local.close()
