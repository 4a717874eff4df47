"""Parity of the fused HIP top-k (libahr_hip.so) against the CPU oracle (oracle/).

fp32 mode: bit-exact — rows AND fp32 scores equal the oracle's k-ordered fma chain.
bf16 / f16: scores within 1e-4 of the double-precision oracle on the same rounded inputs;
            rows equal except near-ties (a differing row's exact score is within 2e-5 of the
            oracle's score at that rank).
"""
import numpy as np
import pytest
import torch

from oracle import dense_ref as dr

pytestmark = pytest.mark.gpu


def _unit(rng, n, d):
    return dr.normalize_rows(rng.standard_normal((n, d)).astype(np.float32))


def _clustered(rng, n, d, n_centers=50, noise=0.35):
    c = _unit(rng, n_centers, d)
    lab = rng.integers(0, n_centers, n)
    x = c[lab] + noise * rng.standard_normal((n, d)).astype(np.float32) / np.sqrt(d)
    return dr.normalize_rows(x)


def _run(index_dtype, C, Q, k, cuda):
    from ah_rag.embeddings import DenseIndex
    ix = DenseIndex(C.shape[1], max(1, C.shape[0]), dtype=index_dtype, device=cuda)
    if C.shape[0]:
        ix.upsert(C)
    s, r = ix.query(Q, k)
    torch.cuda.synchronize()
    out = s.cpu().numpy(), r.cpu().numpy().astype(np.int64)
    ix.close()
    return out


@pytest.mark.parametrize("n,d,B,k", [
    (1, 768, 1, 1), (100, 768, 3, 5), (1000, 384, 7, 10), (5000, 768, 130, 10),
    (20000, 768, 64, 16), (9000, 100, 5, 32), (300, 768, 129, 8),
    (40000, 768, 200, 10), (33000, 384, 1, 32)])  # >= 8*4096 rows: threshold pre-pass path
def test_f32_bit_exact(cuda, n, d, B, k):
    rng = np.random.default_rng(1000 + n + d + B + k)
    C = _clustered(rng, n, d)
    Q = _clustered(rng, B, d)
    s, r = _run("f32", C, Q, k, cuda)
    es, er = dr.topk(C, Q, k, mode="fma")
    kk = min(k, n)
    np.testing.assert_array_equal(r[:, :kk], er[:, :kk])
    np.testing.assert_array_equal(s[:, :kk].astype(np.float32), es[:, :kk].astype(np.float32))
    if kk < k:
        assert (r[:, kk:] == -1).all() and np.isneginf(s[:, kk:]).all()


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("n,d,B,k", [(4000, 768, 17, 10), (20000, 768, 256, 10), (12000, 384, 33, 5),
                                     (50000, 768, 300, 10)])
def test_half_precision_vs_f64(cuda, dtype, n, d, B, k):
    rng = np.random.default_rng(7 + n + B)
    C = dr.round_to_storage(_clustered(rng, n, d), dtype)
    Q = dr.round_to_storage(_clustered(rng, B, d), dtype)
    s, r = _run(dtype, C, Q, k, cuda)
    es, er = dr.topk(C, Q, k, mode="f64")
    full = dr.scores_matrix(C, Q, mode="f64").astype(np.float64)
    # scores of the rows the GPU returned, recomputed exactly
    got_exact = np.take_along_axis(full, r, axis=1)
    assert np.abs(s - got_exact).max() < 1e-4
    assert np.abs(s - es).max() < 1e-4
    mism = r != er
    if mism.any():
        # every mismatch must be a near-tie: the exact score of the row returned at a rank is
        # within 2e-5 of the oracle's score at that rank (adjacent swap or k-th boundary)
        assert (np.abs(got_exact[mism] - es[mism]) < 2e-5).all()


def test_self_match_rank0(cuda):
    rng = np.random.default_rng(3)
    C = _unit(rng, 10000, 768)
    for dtype in ("f32", "bf16"):
        s, r = _run(dtype, C, C[::997], 3, cuda)
        np.testing.assert_array_equal(r[:, 0], np.arange(0, 10000, 997))
        assert np.abs(s[:, 0] - 1.0).max() < (1e-6 if dtype == "f32" else 1e-2)


def test_ties_order_by_row(cuda):
    rng = np.random.default_rng(4)
    base = _unit(rng, 1, 768)
    C = np.repeat(base, 50, axis=0)  # 50 identical rows
    C = np.concatenate([_unit(rng, 1000, 768), C])
    s, r = _run("f32", C, base, 10, cuda)
    np.testing.assert_array_equal(r[0], np.arange(1000, 1010))


def test_upsert_slots_and_truncate(cuda):
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(5)
    C = _unit(rng, 600, 384)
    ix = DenseIndex(384, 1000, dtype="f32", device=cuda)
    ix.upsert(C[:300])
    ix.upsert(C[300:], start=300)
    perm = rng.permutation(600)
    ix.upsert(C[perm], slots=perm)  # overwrite in scrambled order: same content
    assert len(ix) == 600
    back = ix.read().cpu().numpy()
    np.testing.assert_array_equal(back, C)
    s, r = ix.query(C[:4], 1)
    np.testing.assert_array_equal(r.cpu().numpy()[:, 0], np.arange(4))
    ix.truncate(2)
    s, r = ix.query(C[:4], 3)
    rr = r.cpu().numpy()
    assert set(rr[:, :2].ravel().tolist()) <= {0, 1} and (rr[:, 2] == -1).all()
    ix.close()


def test_normalize_on_upsert(cuda):
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(6)
    raw = rng.standard_normal((200, 768)).astype(np.float32) * 3.0
    ix = DenseIndex(768, 200, dtype="f32", device=cuda)
    ix.upsert(raw, normalize=True)
    back = ix.read().cpu().numpy()
    assert np.abs(np.linalg.norm(back, axis=1) - 1).max() < 1e-5
    s, r = ix.query(raw[:3], 1, normalize=True)
    np.testing.assert_array_equal(r.cpu().numpy()[:, 0], [0, 1, 2])
    ix.close()


def test_empty_index(cuda):
    from ah_rag.embeddings import DenseIndex
    ix = DenseIndex(64, 10, dtype="bf16", device=cuda)
    s, r = ix.query(np.ones((2, 64), np.float32), 4)
    assert (r.cpu().numpy() == -1).all()
    ix.close()


@pytest.mark.parametrize("k", [10, 100])
def test_merge_matches_single_shard(cuda, k):
    """Row-sharded search + key merge == unsharded search (the multi-GPU contract, on 1 GPU);
    k = 100 goes through the large-k query path and the radix key merge."""
    from ah_rag.embeddings import DenseIndex, merge_topk_keys
    rng = np.random.default_rng(8)
    C = _clustered(rng, 30000, 768)
    Q = _clustered(rng, 40, 768)
    full_s, full_r = _run("f32", C, Q, k, cuda)
    for G in (2, 3, 8):
        bounds = np.linspace(0, len(C), G + 1).astype(int)
        lists = []
        for g in range(G):
            ix = DenseIndex(768, bounds[g + 1] - bounds[g], dtype="f32", device=cuda)
            ix.upsert(C[bounds[g]:bounds[g + 1]])
            lists.append(ix.query_keys(Q, k, row_base=int(bounds[g])))
            torch.cuda.synchronize()
            ix.close()
        keys = torch.stack(lists, dim=1)  # [B, G, k]
        s, r, _ = merge_topk_keys(keys, k)
        np.testing.assert_array_equal(r.cpu().numpy(), full_r)
        np.testing.assert_array_equal(s.cpu().numpy(), full_s)


def test_prepass_disabled_same_result(cuda):
    """The threshold pre-pass only prunes work: results equal with it switched off."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(9)
    C = _clustered(rng, 40000, 768)
    Q = _clustered(rng, 100, 768)
    ix = DenseIndex(768, len(C), dtype="bf16", device=cuda)
    ix.upsert(C)
    a = [t.cpu().numpy() for t in ix.query(Q, 10)]
    ix.set_sample_rows(0)
    b = [t.cpu().numpy() for t in ix.query(Q, 10)]
    ix.set_sample_rows(256)
    c = [t.cpu().numpy() for t in ix.query(Q, 10)]
    ix.close()
    for x, y in ((a, b), (a, c)):
        np.testing.assert_array_equal(x[0], y[0])
        np.testing.assert_array_equal(x[1], y[1])


def test_many_lists_merge(cuda):
    """Small batches use hundreds of row splits: the heads merge must still be exact."""
    rng = np.random.default_rng(10)
    C = _clustered(rng, 60000, 384)
    Q = _clustered(rng, 3, 384)
    s, r = _run("f32", C, Q, 32, cuda)
    es, er = dr.topk(C, Q, 32, mode="fma")
    np.testing.assert_array_equal(r, er)
    np.testing.assert_array_equal(s, es.astype(np.float32))


# ---- lane kernels (B >= 512, k <= 16): per-lane register top-k lists --------------------------

@pytest.mark.parametrize("n,d,B,k", [(3000, 256, 6200, 10), (1001, 128, 6144, 16), (2000, 384, 6500, 5)])
def test_lane_f32_bit_exact(cuda, n, d, B, k):
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(2000 + n + B)
    C = _clustered(rng, n, d)
    Q = _clustered(rng, B, d)
    ix = DenseIndex(d, n, dtype="f32", device=cuda)
    assert ix.plan(B, k)["kernel"] == "lane256"
    ix.close()
    s, r = _run("f32", C, Q, k, cuda)
    es, er = dr.topk(C, Q, k, mode="fma")
    np.testing.assert_array_equal(r, er)
    np.testing.assert_array_equal(s, es.astype(np.float32))


def test_default_plans(cuda):
    from ah_rag.embeddings import DenseIndex
    ix = DenseIndex(768, 90000, dtype="bf16", device=cuda)
    ix.upsert(np.zeros((90000, 768), np.float32))
    assert ix.plan(1024, 10)["kernel"] == "qres256"  # tests/test_qres_gpu.py
    assert ix.plan(1024, 13)["kernel"] == "tilelane128"
    assert ix.plan(1, 16)["kernel"] == "small"
    assert ix.plan(16, 10)["kernel"] == "small"
    assert ix.plan(17, 10)["kernel"] in ("tilelane128", "lane64")
    assert ix.plan(1, 17)["kernel"] == "tile128"
    assert ix.plan(2048, 10)["kernel"] == "qres256"
    assert ix.plan(6144, 10)["kernel"] == "qres256"
    assert ix.plan(2048, 13)["kernel"] == "tilelane128"  # k beyond the register-resident kernel
    assert ix.plan(1024, 17)["kernel"] == "tile128"
    with pytest.raises(Exception):  # the 128-query-resident kernel: ablation build only
        ix.set_debug_flags(4096)
    with pytest.raises(ValueError):
        ix.set_debug_flags(1 << 32)
    with pytest.raises(ValueError):
        ix.set_debug_flags(-1)
    ix.set_debug_flags(2048)  # without the query-resident kernels
    assert ix.plan(1024, 10)["kernel"] == "tilelane128"
    assert ix.plan(6144, 10)["kernel"] == "lane256"
    ix.close()
    ix = DenseIndex(768, 400000, dtype="f16", device=cuda)  # seed samples < 1/32 of the rows
    ix.upsert(np.zeros((300000, 768), np.float32))
    assert ix.plan(4096, 10)["kernel"] == "qres256"
    assert ix.plan(4096, 13)["kernel"] == "tilelane128"
    ix.close()
    ix = DenseIndex(1024, 1000, dtype="bf16", device=cuda)  # not a query-resident dimension
    assert ix.plan(1024, 10)["kernel"] == "tilelane128"
    ix.close()
    ix = DenseIndex(384, 90000, dtype="bf16", device=cuda)  # the reference's default width
    ix.upsert(np.zeros((90000, 384), np.float32))
    assert ix.plan(1024, 10)["kernel"] == "qres256"
    assert ix.plan(511, 10)["kernel"] == "tilelane128"
    ix.close()


@pytest.mark.parametrize("k,sample", [(10, 8192), (16, 8192), (5, 0), (10, 0), (1, 8192)])
def test_lane_kernels_bitwise_equal(cuda, k, sample):
    """All kernels chain the same 16-deep MFMA steps in k order: bitwise equal results. Sample 0
    (no pre-pass) makes every score of the first tiles a candidate: full scans / overflow rounds."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(31 + k + sample)
    C = _clustered(rng, 40001, 768)   # >= 4 x 8192 rows: the pre-pass runs when sample > 0
    Q = _clustered(rng, 6150, 768)    # >= 6144: the 256x256 lane kernel is the default
    ix = DenseIndex(768, len(C), dtype="bf16", device=cuda)
    ix.upsert(C)
    ix.set_sample_rows(sample)
    ix.set_debug_flags(32)
    a = [t.cpu().numpy() for t in ix.query(Q, k)]
    # 8: 128x128 tile kernel, cooperative screening; 32: 128x128 lane-local tile kernel; 2048:
    # without the query-resident kernels (the 256x256 lane kernel at this batch); 1 << 23: the
    # 256-query register-resident kernel (k <= 12; 24 query blocks, 8 splits: not self-seeded)
    variants = [(8, "tile128"), (32, "tilelane128"), (2048, "lane256")] + ([(1 << 23, "qres256")] if k <= 12 else [])
    for flags, name in variants:
        ix.set_debug_flags(flags)
        assert ix.plan(len(Q), k)["kernel"] == name
        b = [t.cpu().numpy() for t in ix.query(Q, k)]
        np.testing.assert_array_equal(a[1], b[1], err_msg=name)
        np.testing.assert_array_equal(a[0], b[0], err_msg=name)
    ix.close()


@pytest.mark.parametrize("dtype", ["bf16", "f32"])
@pytest.mark.parametrize("B", [17, 64])
def test_prepass_wave_form_small_batch(cuda, dtype, B):
    """B <= 64 seeds from sample_groupmax_kernel (one wave per 32 rows x 32 queries, the tile
    kernel's MFMA chain): results equal the unseeded scan's, with the sampled rows repeated later
    in the corpus so the seed ties exactly with later rows' scores."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(77 + B)
    C = _clustered(rng, 40001, 768)
    C[20000:28192] = C[:8192]          # exact copies of the sampled rows: seed == later scores
    Q = C[rng.integers(0, 8192, B)] + 0.01 * rng.standard_normal((B, 768)).astype(np.float32)
    ix = DenseIndex(768, len(C), dtype=dtype, device=cuda)
    ix.upsert(C)
    assert ix.plan(B, 10)["kernel"] != "small"
    out = {}
    for sample in (8192, 0):
        ix.set_sample_rows(sample)
        out[sample] = [t.cpu().numpy() for t in ix.query(Q, 10)]
    np.testing.assert_array_equal(out[8192][1], out[0][1])
    np.testing.assert_array_equal(out[8192][0], out[0][0])
    ix.close()


LANE64_SCRIPT = r"""
import sys
sys.path[:0] = [{root!r}, {pkg!r}]
import numpy as np
from oracle import dense_ref as dr
from ah_rag.embeddings import DenseIndex
for dtype, d, B in (("bf16", 768, 64), ("bf16", 768, 17), ("f16", 384, 40), ("bf16", 100, 64)):
    rng = np.random.default_rng(91 + B + d)
    c = dr.normalize_rows(rng.standard_normal((50, d)).astype(np.float32))
    C = dr.normalize_rows(c[rng.integers(0, 50, 40001)] + 0.35 * rng.standard_normal((40001, d)).astype(np.float32) / np.sqrt(d))
    Q = dr.normalize_rows(c[rng.integers(0, 50, B)] + 0.35 * rng.standard_normal((B, d)).astype(np.float32) / np.sqrt(d))
    ix = DenseIndex(d, len(C), dtype=dtype, device="cuda:0")
    ix.upsert(C)
    assert ix.plan(B, 10)["kernel"] == "lane64", ix.plan(B, 10)
    a = [t.cpu().numpy() for t in ix.query(Q, 10)]
    ix.set_debug_flags(32)
    assert ix.plan(B, 10)["kernel"] == "tilelane128"
    b = [t.cpu().numpy() for t in ix.query(Q, 10)]
    ix.close()
    assert (a[0] == b[0]).all() and (a[1] == b[1]).all(), (dtype, d, B)
print("LANE64_OK")
"""


def test_lane64_equals_tilelane(cuda):
    """The opt-in 256 x 64 lane-local plan (AHR_LANE64=1, 17 <= B <= 64, half precision) chains the
    same k-ordered MFMA steps as the 128 x 128 one: bitwise equal results (flag 32 forces the
    128 x 128 plan). The setting is read once per process, hence one child process for all cases."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, AHR_LANE64="1")
    p = subprocess.run([sys.executable, "-c", LANE64_SCRIPT.format(root=root, pkg=os.path.join(root, "ah-rag_amd"))],
                       env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0 and "LANE64_OK" in p.stdout, (p.stdout[-2000:], p.stderr[-4000:])


def test_lane_ties_order_by_row(cuda):
    """Duplicate corpus rows tie exactly: lower row id first, across tiles and splits."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(12)
    base = _clustered(rng, 300, 256)
    C = np.concatenate([base] * 40)  # 12000 rows, each vector 40 times
    Q = base[rng.integers(0, 300, 600)]
    ix = DenseIndex(256, len(C), dtype="f32", device=cuda)
    ix.upsert(C)
    s, r = [t.cpu().numpy() for t in ix.query(Q, 16)]
    ix.close()
    es, er = dr.topk(C, Q, 16, mode="fma")
    np.testing.assert_array_equal(r, er)
    np.testing.assert_array_equal(s, es.astype(np.float32))


def test_workspaces_concurrent_streams(cuda):
    """Batches in flight on two streams with two query workspaces == the same batches run one by
    one (workspaces share nothing but the read-only corpus)."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(14)
    C = _clustered(rng, 40000, 768)
    Qs = [torch.from_numpy(_clustered(rng, B, 768)).to(cuda) for B in (1024, 700, 1024, 300)]
    ix = DenseIndex(768, len(C), dtype="bf16", device=cuda)
    ix.upsert(C)
    serial = [[t.cpu().numpy() for t in ix.query(q, 10)] for q in Qs]
    streams = [torch.cuda.current_stream(cuda), torch.cuda.Stream(device=cuda)]
    streams[1].wait_stream(streams[0])
    outs = []
    for rep in range(3):
        for i, q in enumerate(Qs):
            ix.set_workspace(i % 2)
            outs.append(ix.query(q, 10, stream=streams[i % 2]))
    torch.cuda.synchronize()
    ix.set_workspace(0)
    for j, (s, r) in enumerate(outs):
        np.testing.assert_array_equal(r.cpu().numpy(), serial[j % len(Qs)][1])
        np.testing.assert_array_equal(s.cpu().numpy(), serial[j % len(Qs)][0])
    with pytest.raises(Exception):
        ix.set_workspace(4)
    ix.close()


def _close_topk(a, b, tol=2e-6):
    """Two kernels' (scores, rows): scores within tol; a row differs only where another of the
    returned scores lies within tol of it (a near-tie reordered or swapped at the k-th place)."""
    np.testing.assert_allclose(a[0], b[0], rtol=0, atol=tol)
    mism = a[1] != b[1]
    if mism.any():
        gap = np.abs(a[0][:, :, None] - b[0][:, None, :])
        near = (gap < tol).sum(axis=2) >= 2  # a tie group inside the list (order swapped)
        near[:, -1] = True                   # or the k-th place (a tie with a row outside)
        assert near[mism].all()

# ---- k beyond the register lists (AHR_MAX_K < k <= AHR_MAX_K_LARGE): scores + radix select ----

@pytest.mark.parametrize("dtype,n,d,B,k", [
    ("f32", 5000, 384, 7, 100), ("f32", 3000, 768, 130, 500), ("f32", 700, 256, 3, 1000),
    ("f32", 50, 128, 2, 40), ("bf16", 20000, 768, 33, 64), ("f16", 9000, 384, 5, 4096)])
def test_large_k(cuda, dtype, n, d, B, k):
    """k > 32 (Chroma's n_results has no small cap): fp32 rows and scores bit-identical to the
    oracle's fma chain; bf16/f16 scores within 1e-4 of the f64 oracle on the rounded inputs,
    rows equal except near-ties; k > n pads with (-inf, -1)."""
    rng = np.random.default_rng(4000 + n + k)
    C = _clustered(rng, n, d)
    Q = _clustered(rng, B, d)
    if dtype != "f32":
        C, Q = dr.round_to_storage(C, dtype), dr.round_to_storage(Q, dtype)
    s, r = _run(dtype, C, Q, k, cuda)
    kk = min(k, n)
    if dtype == "f32":
        es, er = dr.topk(C, Q, k, mode="fma")
        np.testing.assert_array_equal(r[:, :kk], er[:, :kk])
        np.testing.assert_array_equal(s[:, :kk].astype(np.float32), es[:, :kk].astype(np.float32))
    else:
        es, er = dr.topk(C, Q, k, mode="f64")
        assert np.abs(s[:, :kk] - es[:, :kk]).max() < 1e-4
        mism = r[:, :kk] != er[:, :kk]
        if mism.any():
            full = dr.scores_matrix(C, Q, mode="f64").astype(np.float64)
            got = np.take_along_axis(full, r[:, :kk], axis=1)
            assert (np.abs(got[mism] - es[:, :kk][mism]) < 2e-5).all()
    if kk < k:
        assert (r[:, kk:] == -1).all() and np.isneginf(s[:, kk:]).all()


def test_large_k_ties_order_by_row(cuda):
    """Duplicate rows tie exactly at and across the radix-select boundary: lowest rows first."""
    rng = np.random.default_rng(15)
    base = _clustered(rng, 300, 256)
    C = np.concatenate([base] * 40)  # 12000 rows, each vector 40 times
    Q = base[rng.integers(0, 300, 40)]
    s, r = _run("f32", C, Q, 100, cuda)
    es, er = dr.topk(C, Q, 100, mode="fma")
    np.testing.assert_array_equal(r, er)
    np.testing.assert_array_equal(s, es.astype(np.float32))


# ---- 256 x 256 16x16x32 kernel (debug flag 32768 while it is not a default plan) ----------------

@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("n,d,B,k,sample", [
    (40001, 768, 1024, 10, 8192), (40001, 768, 1024, 10, 0), (33000, 384, 300, 16, 8192),
    (300, 768, 1, 1, 0), (1000, 128, 257, 8, 0), (90000, 768, 2048, 5, 8192)])
def test_t256_matches_tilelane(cuda, dtype, n, d, B, k, sample):
    """16x16x32 MFMAs sum each 32-deep slice inside one instruction: scores within 2e-6 of the
    32x32x16 chain, rows equal except near-ties; splits with no tiles, ragged blocks, no seed."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(91 + n + B + k)
    C = _clustered(rng, n, d)
    Q = _clustered(rng, B, d)
    ix = DenseIndex(d, n, dtype=dtype, device=cuda)
    ix.upsert(C)
    ix.set_sample_rows(sample)
    ix.set_debug_flags(32768)
    assert ix.plan(B, k)["kernel"] == "t256"
    a = [t.cpu().numpy() for t in ix.query(Q, k)]
    ix.set_debug_flags(32)
    b = [t.cpu().numpy() for t in ix.query(Q, k)]
    ix.close()
    _close_topk(a, b)


# ---- k-blocked 256 x 256 kernel (kb256): bitwise the t256 kernel's scores and rows ------------------------------

@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("n,d,B,k,sample", [
    (40001, 768, 1024, 10, 8192), (40001, 768, 1024, 10, 0), (33000, 384, 300, 16, 8192),
    (300, 768, 1, 1, 0), (1000, 128, 257, 8, 0), (90000, 768, 2048, 5, 8192), (5000, 100, 17, 12, 0),
    (4000, 1100, 40, 10, 0), (90000, 768, 1024, 10, 8192)])
def test_kb256_matches_t256(cuda, dtype, n, d, B, k, sample):
    """Same 16x16x32 fragment map and k order as t256 (only the staging differs: 32-deep k-blocked
    steps through a 4-stage ring): scores and rows bitwise equal; ragged last tile, splits without
    tiles, d_pad 128 / 1152, no seed."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(191 + n + B + k)
    C = _clustered(rng, n, d)
    Q = _clustered(rng, B, d)
    ix = DenseIndex(d, n, dtype=dtype, device=cuda)
    half = n // 2 + 37  # two upserts: the k-blocked copy is refreshed per written range
    ix.upsert(C[:half])
    ix.upsert(C[half:], start=half)
    ix.set_sample_rows(sample)
    ix.set_debug_flags(131072)
    assert ix.plan(B, k)["kernel"] == "kb256"
    a = [t.cpu().numpy() for t in ix.query(Q, k)]
    ix.set_debug_flags(32768)
    assert ix.plan(B, k)["kernel"] == "t256"
    b = [t.cpu().numpy() for t in ix.query(Q, k)]
    ix.close()
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[0], b[0])
    kk = min(k, n)
    Cr, Qr = dr.round_to_storage(C, dtype), dr.round_to_storage(Q, dtype)
    es, _ = dr.topk(Cr, Qr, k, mode="f64")
    assert np.abs(a[0][:, :kk] - es[:, :kk]).max() < 1e-4


@pytest.mark.parametrize("flag,name", [(131072, "kb256")])
def test_kb256_slot_upsert_and_ties(cuda, flag, name):
    """Scattered-slot upserts refresh the k-blocked copy; duplicate rows order by row id."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(23)
    base = _clustered(rng, 300, 768)
    C = np.concatenate([base] * 40)  # 12000 rows, each vector 40 times
    ix = DenseIndex(768, len(C), dtype="bf16", device=cuda)
    ix.upsert(np.zeros_like(C))
    perm = rng.permutation(len(C))
    ix.upsert(C[perm], slots=perm)
    ix.set_debug_flags(flag)
    pick = rng.integers(0, 300, 64)
    assert ix.plan(64, 16)["kernel"] == name
    s, r = [t.cpu().numpy() for t in ix.query(base[pick], 16)]
    ix.close()
    np.testing.assert_array_equal(r, pick[:, None] + 300 * np.arange(16)[None, :])
    assert (s == s[:, :1]).all()


# ---- small batches (B <= 16, bf16/f16, k <= 16): corpus-streaming 16x16x32 kernel -------------

def test_small_plans(cuda):
    from ah_rag.embeddings import DenseIndex
    ix = DenseIndex(768, 5000, dtype="f32", device=cuda)  # fp32: the VALU fma-chain stream, B <= 4
    ix.upsert(np.zeros((5000, 768), np.float32))
    assert ix.plan(1, 10)["kernel"] == "small"
    assert ix.plan(4, 16)["kernel"] == "small"
    assert ix.plan(5, 10)["kernel"] != "small"
    assert ix.plan(1, 17)["kernel"] != "small"
    ix.close()
    ix = DenseIndex(1100, 100, dtype="f32", device=cuda)  # d_pad > 1024: the tile path
    assert ix.plan(1, 10)["kernel"] != "small"
    ix.close()
    ix = DenseIndex(768, 90000, dtype="bf16", device=cuda)
    ix.upsert(np.zeros((90000, 768), np.float32))
    p = ix.plan(1, 10)
    assert p["kernel"] == "small" and p["n_splits"] == 256
    ix.set_debug_flags(32)  # an explicit kernel flag overrides the small-batch plan
    assert ix.plan(1, 10)["kernel"] == "tilelane128"
    ix.set_debug_flags(0)
    assert ix.plan(17, 10)["kernel"] in ("tilelane128", "lane64")
    ix.close()


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("n,d,B,k,norm", [
    (90000, 768, 1, 10, False), (40001, 768, 16, 16, True), (33000, 384, 7, 5, False),
    (300, 768, 1, 1, False), (17, 128, 3, 8, True), (1, 768, 2, 4, False), (5000, 100, 5, 12, True),
    (5000, 102, 4, 10, True), (4000, 1100, 9, 10, False), (2000, 1000, 16, 16, True)])
def test_small_matches_t256(cuda, dtype, n, d, B, k, norm):
    """The small-batch kernel feeds the t256 kernel's 16x16x32 fragment map in the same k order,
    and converts its queries with the convert kernel's arithmetic (in LDS; d = 102 and 1100 take
    the converted query buffer instead): scores and rows bitwise equal to the t256 kernel; k > n
    pads with (-inf, -1); splits that get fewer blocks than waves; ragged last block; a ragged
    group of 16 queries."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(500 + n + d + B + k)
    C = _clustered(rng, n, d)
    Q = _clustered(rng, B, d) * (3.0 if norm else 1.0)
    ix = DenseIndex(d, n, dtype=dtype, device=cuda)
    ix.upsert(C)
    assert ix.plan(B, k)["kernel"] == "small"
    a = [t.cpu().numpy() for t in ix.query(Q, k, normalize=norm)]
    ix.set_sample_rows(0)
    ix.set_debug_flags(32768)
    assert ix.plan(B, k)["kernel"] == "t256"
    b = [t.cpu().numpy() for t in ix.query(Q, k, normalize=norm)]
    ix.close()
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    kk = min(k, n)
    if kk < k:
        assert (a[1][:, kk:] == -1).all() and np.isneginf(a[0][:, kk:]).all()
    # and against the f64 oracle on the rounded inputs
    Qn = dr.normalize_rows(Q) if norm else Q
    es, er = dr.topk(dr.round_to_storage(C, dtype), dr.round_to_storage(Qn, dtype), k, mode="f64")
    assert np.abs(a[0][:, :kk] - es[:, :kk]).max() < 1e-4


def test_small_ties_order_by_row(cuda):
    """Duplicate rows score identically in bf16: the lowest row ids win across waves and splits."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(16)
    base = _clustered(rng, 300, 768)
    C = np.concatenate([base] * 40)  # 12000 rows, each vector 40 times
    pick = rng.integers(0, 300, 16)
    ix = DenseIndex(768, len(C), dtype="bf16", device=cuda)
    ix.upsert(C)
    assert ix.plan(16, 16)["kernel"] == "small"
    s, r = [t.cpu().numpy() for t in ix.query(base[pick], 16)]
    ix.close()
    np.testing.assert_array_equal(r, pick[:, None] + 300 * np.arange(16)[None, :])
    assert (s == s[:, :1]).all()


def test_small_sharded_keys(cuda):
    """row_base offsets and the key merge through the small-batch plan == one unsharded query."""
    from ah_rag.embeddings import DenseIndex, merge_topk_keys
    rng = np.random.default_rng(17)
    C = _clustered(rng, 20000, 384)
    Q = _clustered(rng, 5, 384)
    full = DenseIndex(384, len(C), dtype="bf16", device=cuda)
    full.upsert(C)
    fs, fr = [t.cpu().numpy() for t in full.query(Q, 10)]
    full.close()
    bounds = [0, 7001, 13000, 20000]
    lists = []
    for g in range(3):
        ix = DenseIndex(384, bounds[g + 1] - bounds[g], dtype="bf16", device=cuda)
        ix.upsert(C[bounds[g]:bounds[g + 1]])
        assert ix.plan(5, 10)["kernel"] == "small"
        lists.append(ix.query_keys(Q, 10, row_base=bounds[g]))
        torch.cuda.synchronize()
        ix.close()
    s, r, _ = merge_topk_keys(torch.stack(lists, dim=1), 10)
    np.testing.assert_array_equal(r.cpu().numpy(), fr)
    np.testing.assert_array_equal(s.cpu().numpy(), fs)


@pytest.mark.parametrize("n,d,B,k,norm", [
    (90000, 768, 1, 10, False), (40001, 768, 4, 16, True), (33000, 384, 3, 5, False), (1, 768, 1, 4, False),
    (300, 100, 2, 1, True), (65, 1000, 4, 12, False), (5000, 102, 1, 8, True)])
def test_small_f32_bit_exact(cuda, n, d, B, k, norm):
    """fp32 small batches (B <= 4): one lane runs each (row, query) fma chain in k order on the
    VALU, undoing the stored lane permutation: rows and scores bit-identical to the oracle; ragged
    64-row items, k > n, normalisation in the convert kernel."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(900 + n + d + B + k)
    C = _clustered(rng, n, d)
    Q = _clustered(rng, B, d) * (2.0 if norm else 1.0)
    ix = DenseIndex(d, n, dtype="f32", device=cuda)
    ix.upsert(C)
    assert ix.plan(B, k)["kernel"] == "small"
    s, r = [t.cpu().numpy() for t in ix.query(Q, k, normalize=norm)]
    ix.close()
    Qn = Q
    if norm:  # the device normalisation (fp32 wave reduction) is the convert kernel's, as in the tile path
        ix2 = DenseIndex(d, max(1, B), dtype="f32", device=cuda)
        ix2.upsert(Q, normalize=True)
        Qn = ix2.read(0, B).cpu().numpy()
        ix2.close()
    es, er = dr.topk(C, Qn, k, mode="fma")
    kk = min(k, n)
    np.testing.assert_array_equal(r[:, :kk], er[:, :kk])
    np.testing.assert_array_equal(s[:, :kk].astype(np.float32), es[:, :kk].astype(np.float32))
    if kk < k:
        assert (r[:, kk:] == -1).all() and np.isneginf(s[:, kk:]).all()


@pytest.mark.parametrize("dtype,n,d,B", [("f32", 3000, 768, 3000), ("f32", 517, 100, 33), ("bf16", 2000, 384, 129),
                                         ("f32", 1, 64, 1)])
def test_index_scores_matrix(cuda, dtype, n, d, B):
    """ahr_index_scores (the tile kernel's GEMM core in scores mode, used by the L1 relation
    builder): fp32 = the oracle's k-ordered fma chain bit for bit; bf16 within 1e-4 of f64."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(77 + n + B)
    C = _clustered(rng, n, d)
    Q = _clustered(rng, B, d)
    ix = DenseIndex(d, n, dtype=dtype, device=cuda)
    ix.upsert(C)
    S = ix.scores(Q).cpu().numpy()
    ix.close()
    assert S.shape == (B, n)
    if dtype == "f32":
        np.testing.assert_array_equal(S, dr.scores_matrix(C, Q, mode="fma"))
    else:
        ref = dr.scores_matrix(dr.round_to_storage(C, dtype), dr.round_to_storage(Q, dtype), mode="f64")
        assert np.abs(S - ref).max() < 1e-4
