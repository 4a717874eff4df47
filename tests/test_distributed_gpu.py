"""The row-sharded query path over a real RCCL communicator (backend "nccl" = RCCL on ROCm).

One GPU box cannot host a multi-rank RCCL group (RCCL refuses two ranks on one device), so this
runs the product path — init_process_group("nccl", device_id=...), ShardedDenseIndex.upsert_global,
local fused top-k, all_gather_into_tensor of the packed keys, on-device merge — on a one-rank
communicator in a child process, and checks it bitwise against the unsharded DenseIndex. The
multi-rank logic itself (shard bounds, global row ids, gather layout, merge) is covered by
tests/test_distributed_cpu.py with two gloo ranks.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import os, sys
import numpy as np
import torch
import torch.distributed as dist
sys.path[:0] = [os.path.join({root!r}, "ah-rag_amd"), {root!r}]
from ah_rag.distributed import ShardedDenseIndex, all_gather_keys
from ah_rag.embeddings import DenseIndex

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
assert dist.get_backend() == "nccl"
rng = np.random.default_rng(5)
C = rng.standard_normal((20000, 768)).astype(np.float32)
C /= np.linalg.norm(C, axis=1, keepdims=True)
Q = C[:100] + 0.1 * rng.standard_normal((100, 768)).astype(np.float32)
idx = ShardedDenseIndex(768, len(C), dtype="bf16", device=dev)
assert (idx.lo, idx.hi) == (0, len(C))
for s0 in range(0, len(C), 7000):
    idx.upsert_global(s0, torch.from_numpy(C[s0:s0 + 7000]).to(dev))
s, r = idx.query(torch.from_numpy(Q).to(dev), 10)
ref = DenseIndex(768, len(C), dtype="bf16", device=dev)
ref.upsert(C)
s2, r2 = ref.query(Q, 10)
assert torch.equal(r.cpu(), r2.cpu()), "rows differ"
assert torch.equal(s.cpu(), s2.cpu()), "scores differ"
# two batches in flight (bench.py's pipelined sharded step): a stream and a workspace each, the
# collective of one batch beside the local search of the next
streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(device=dev)]
kb = [torch.empty((100, 10), dtype=torch.int64, device=dev) for _ in range(2)]
for i in range(2):
    idx.local.set_workspace(i)
    idx.reserve(100, 10)
streams[1].wait_stream(streams[0])
Qd = torch.from_numpy(Q).to(dev)
outs = []
for j in range(6):
    i = j % 2
    idx.local.set_workspace(i)
    with torch.cuda.stream(streams[i]):
        outs.append(idx.query(Qd, 10, out_keys=kb[i]))
torch.cuda.synchronize()
idx.local.set_workspace(0)
for s3, r3 in outs:
    assert torch.equal(r3.cpu(), r2.cpu()) and torch.equal(s3.cpu(), s2.cpu()), "pipelined batch differs"
g = all_gather_keys(torch.arange(12, dtype=torch.int64, device=dev).view(3, 4))
assert g.shape == (1, 3, 4) and g.is_cuda and torch.equal(g[0].cpu(), torch.arange(12).view(3, 4))
torch.cuda.synchronize()
dist.barrier()
dist.destroy_process_group()
print("RCCL_OK")
"""


@pytest.mark.gpu
def test_rccl_one_rank_sharded_query_matches_unsharded(cuda):
    from ah_rag.distributed import free_port
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, "-c", SCRIPT.format(root=ROOT, port=free_port())], env=env,
                       capture_output=True, text=True, timeout=180)
    assert p.returncode == 0 and "RCCL_OK" in p.stdout, (p.stdout[-2000:], p.stderr[-4000:])
