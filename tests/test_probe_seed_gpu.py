"""Cluster-probe seeds (DenseIndex.build_clusters -> ahr_index_probe_seed -> ahr_index_set_seed).

The seed is an admission threshold only: with it the fused kernels must return exactly what they
return with the sampled pre-pass (bitwise), including ties, ragged tiles, rows upserted or truncated
after the clusters were built, and two batches in flight. Each seed must also lower-bound the
query's k-th best score as the kernels compute it.
"""
import numpy as np
import pytest
import torch

from oracle import dense_ref as dr

pytestmark = pytest.mark.gpu


def _clustered(rng, n, d, n_centers=300, noise=0.35):
    c = dr.normalize_rows(rng.standard_normal((n_centers, d)).astype(np.float32))
    lab = rng.integers(0, n_centers, n)
    x = c[lab] + noise * rng.standard_normal((n, d)).astype(np.float32) / np.sqrt(d)
    return dr.normalize_rows(x)


def _both(ix, Q, k, **kw):
    ix.drop_clusters()
    a = [t.cpu().numpy() for t in ix.query(Q, k, **kw)]
    info = ix.build_clusters()
    b = [t.cpu().numpy() for t in ix.query(Q, k, **kw)]
    return a, b, info


@pytest.mark.parametrize("dtype,n,d,B,k,dup", [
    ("bf16", 40001, 768, 1024, 10, 1), ("f16", 33000, 384, 300, 16, 1), ("bf16", 12000, 256, 600, 1, 1),
    ("bf16", 24000, 768, 257, 10, 40), ("f16", 50000, 768, 2048, 5, 1)])
def test_probe_seed_same_results(cuda, dtype, n, d, B, k, dup):
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(300 + n + B + k)
    C = _clustered(rng, n // dup, d)
    C = np.concatenate([C] * dup)[:n] if dup > 1 else C
    Q = _clustered(rng, B, d)
    ix = DenseIndex(d, n, dtype=dtype, device=cuda)
    ix.upsert(C)
    a, b, info = _both(ix, Q, k)
    assert info["rows"] == n and info["clusters"] >= 16
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[0], b[0])
    # every seed lower-bounds the kernel's own k-th score of its query
    q = torch.from_numpy(Q).to(cuda)
    thr = ix._probe_seed(q, k, False, None).cpu().numpy()
    assert (thr <= b[0][:, k - 1]).all()
    assert np.isfinite(thr).mean() > 0.99  # the probe found >= k rows for (nearly) every query
    ix.close()


def test_probe_seed_after_upserts_and_truncate(cuda):
    """Lists built before later writes stay valid: new rows are not probed, truncated slots are
    skipped, rewritten slots are scored with their current contents."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(17)
    C = _clustered(rng, 30000, 768)
    Q = np.concatenate([C[:200] + 0.02 * rng.standard_normal((200, 768)).astype(np.float32),
                        _clustered(rng, 312, 768)])
    ix = DenseIndex(768, 40000, dtype="bf16", device=cuda)
    ix.upsert(C[:25000])
    ix.build_clusters()
    ix.upsert(C[25000:], start=25000)                   # appended after the build
    ix.upsert(C[5000:6000][::-1].copy(), start=5000)    # rewritten slots
    seeded = [t.cpu().numpy() for t in ix.query(Q, 10)]
    ix.drop_clusters()
    plain = [t.cpu().numpy() for t in ix.query(Q, 10)]
    np.testing.assert_array_equal(seeded[1], plain[1])
    np.testing.assert_array_equal(seeded[0], plain[0])
    ix.build_clusters()
    ix.truncate(20000)
    seeded = [t.cpu().numpy() for t in ix.query(Q, 10)]
    ix.drop_clusters()
    plain = [t.cpu().numpy() for t in ix.query(Q, 10)]
    np.testing.assert_array_equal(seeded[1], plain[1])
    np.testing.assert_array_equal(seeded[0], plain[0])
    assert (seeded[1] < 20000).all()
    ix.close()


def test_probe_seed_streams_and_keys(cuda):
    """Two batches in flight (two workspaces, the centroid index's too) and the keyed query."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(23)
    C = _clustered(rng, 40000, 768)
    Qs = [torch.from_numpy(_clustered(rng, B, 768)).to(cuda) for B in (1024, 700, 1024, 300)]
    ix = DenseIndex(768, len(C), dtype="bf16", device=cuda)
    ix.upsert(C)
    serial = [[t.cpu().numpy() for t in ix.query(q, 10)] for q in Qs]
    keys_plain = ix.query_keys(Qs[0], 10, row_base=77).cpu().numpy()
    ix.build_clusters()
    for i in range(2):
        ix.set_workspace(i)
        ix.reserve(1024, 10)
    ix.set_workspace(0)
    streams = [torch.cuda.current_stream(cuda), torch.cuda.Stream(device=cuda)]
    streams[1].wait_stream(streams[0])
    outs = []
    for rep in range(2):
        for i, q in enumerate(Qs):
            ix.set_workspace(i % 2)
            with torch.cuda.stream(streams[i % 2]):
                outs.append(ix.query(q, 10))
    torch.cuda.synchronize()
    ix.set_workspace(0)
    for j, (s, r) in enumerate(outs):
        np.testing.assert_array_equal(r.cpu().numpy(), serial[j % len(Qs)][1])
        np.testing.assert_array_equal(s.cpu().numpy(), serial[j % len(Qs)][0])
    np.testing.assert_array_equal(ix.query_keys(Qs[0], 10, row_base=77).cpu().numpy(), keys_plain)
    ix.close()


def test_probe_seed_rejects_f32(cuda):
    from ah_rag.embeddings import DenseIndex
    ix = DenseIndex(64, 1000, dtype="f32", device=cuda)
    ix.upsert(np.eye(64, dtype=np.float32).repeat(10, axis=0))
    with pytest.raises(ValueError):
        ix.build_clusters()
    ix.close()
