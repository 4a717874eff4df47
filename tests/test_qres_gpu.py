"""The 256-query register-resident kernel (csrc/ahr_qres.hip) — the default B >= 512 bf16/f16 plan at
d = 768 and 384, k <= 12 (the C2 headline shape; reference src/ah_rag/graph/hierarchical_graph.py:714).

At d = 768 its block product is a chain of v_mfma_f32_16x16x32 over 32-deep steps in k order, the
chain of the 256x256 tile kernel (topk_t256_kernel); at d = 384 the 32x32x16 chain of the lane-local
tile kernel (topk_tilelane_kernel); scores AND rows must be bitwise equal to that reference (ref_of)
— with its admission threshold seeded by itself
(the default: splits publish per-query maxima, the k-th largest becomes the seed), by the sampled
pre-pass launch (flag 1 << 26), or not at all (sample rows 0: every score a candidate, the survivor
buffers' compaction path) — including ragged row and query blocks, splits with no rows, adversarial
row order (the records all in the last split, or every row a new record), exact ties (lowest row
id first), consecutive launches with changing batch shapes (stale granules of another launch) and
row-base offsets. A seed above a query's true k-th score would drop rows: the bitwise comparisons
are the validity check. Against the f64 oracle the half-precision tolerance of test_dense_gpu.py
applies.
"""
import numpy as np
import pytest
import torch

from oracle import dense_ref as dr

pytestmark = pytest.mark.gpu

QRES = 1 << 23      # plan the register-resident kernel wherever it applies
PREPASS = 1 << 26   # ... seeded by the sampled pre-pass launch instead of by itself
TILELANE = 32       # the lane-local 128x128 tile kernel at any batch
MUTE = 4            # split 0 seeds under a tag no launch has: every bounded wait on it times out
T256 = 32768        # the 256x256 16x16x32 tile kernel


def ref_of(d):
    """The bitwise reference of the register-resident kernel at width d (ahr_qres.h AHR_QRES_MMA16 = 1,
    the shipped build): at d = 768 its block product is a chain of v_mfma_f32_16x16x32 over 32-deep
    steps in k order, the t256 kernel's chain; at d = 384 the 32x32x16 chain of the tilelane kernel."""
    return (T256, "t256") if d > 384 else (TILELANE, "tilelane128")


def _clustered(rng, n, d, n_centers=50, noise=0.35):
    c = dr.normalize_rows(rng.standard_normal((n_centers, d)).astype(np.float32))
    lab = rng.integers(0, n_centers, n)
    x = c[lab] + noise * rng.standard_normal((n, d)).astype(np.float32) / np.sqrt(d)
    return dr.normalize_rows(x)


def _run(ix, Q, k, flags, kernel):
    ix.set_debug_flags(flags)
    assert ix.plan(len(Q), k)["kernel"] == kernel
    out = [t.cpu().numpy() for t in ix.query(Q, k)]
    ix.set_debug_flags(0)
    return out


def _check_forms(ix, Q, k):
    """Self-seeded and pre-pass-seeded launches against the tile kernel, bitwise; returns the
    self-seeded (default) result."""
    a = _run(ix, Q, k, QRES, "qres256")
    d = _run(ix, Q, k, *ref_of(ix.dim))
    np.testing.assert_array_equal(a[1], d[1])
    np.testing.assert_array_equal(a[0], d[0])
    e = _run(ix, Q, k, QRES | PREPASS, "qres256")
    np.testing.assert_array_equal(e[1], a[1])
    np.testing.assert_array_equal(e[0], a[0])
    return a


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
@pytest.mark.parametrize("n,B,k,sample,d", [
    (90000, 1024, 10, 8192, 768),  # the C2 shape
    (90000, 1024, 10, 8192, 384),  # ... at the reference's default width
    (40001, 512, 10, 8192, 768),   # ragged last row block; 128 splits (two granules per lane)
    (40001, 700, 1, 8192, 768),    # ragged query block (a partly live wave, whole dead waves), k = 1
    (40001, 700, 12, 8192, 384),
    (40001, 1024, 12, 0, 768),     # no seed: compaction from the first block on
    (33000, 2048, 8, 8192, 768),   # 32 splits
    (33000, 4096, 10, 8192, 384),  # 16 splits: too few to seed itself, the pre-pass seeds it
    (5000, 600, 10, 0, 768),
    (5000, 600, 10, 8192, 768),    # 157 blocks over 80 splits: too few for self-seeding
    (300, 512, 5, 0, 768),         # 10 row blocks over 8 splits, queries 300.. of the second block dead
])
def test_qres_matches_tilelane(cuda, dtype, n, B, k, sample, d):
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(501 + n + B + k + sample + d)
    C = _clustered(rng, n, d)
    Q = _clustered(rng, B, d)
    ix = DenseIndex(d, n, dtype=dtype, device=cuda)
    ix.upsert(C)
    ix.set_sample_rows(sample)
    a = _check_forms(ix, Q, k)
    ix.close()
    # and against the f64 oracle on the rounded inputs (sampled queries)
    sel = np.arange(0, B, max(1, B // 48))
    es, _ = dr.topk(dr.round_to_storage(C, dtype), dr.round_to_storage(Q[sel], dtype), k, mode="f64")
    kk = min(k, n)
    assert np.abs(a[0][sel, :kk] - es[:, :kk]).max() < 1e-4


def test_qres_default_plan(cuda):
    from ah_rag.embeddings import DenseIndex
    ix = DenseIndex(768, 90000, dtype="bf16", device=cuda)
    ix.upsert(np.zeros((90000, 768), np.float32))
    assert ix.plan(1024, 10)["kernel"] == "qres256"
    p = ix.plan(1024, 10)
    assert (p["qblocks"], p["n_splits"]) == (4, 64)
    assert ix.plan(512, 12)["kernel"] == "qres256"
    assert ix.plan(511, 10)["kernel"] == "tilelane128"
    assert ix.plan(1024, 13)["kernel"] == "tilelane128"  # k beyond the lane buffer's reach
    ix.set_debug_flags(2048)
    assert ix.plan(1024, 10)["kernel"] == "tilelane128"
    ix.close()
    ix = DenseIndex(768, 20000, dtype="bf16", device=cuda)  # no pre-pass below 4 x 8192 rows
    ix.upsert(np.zeros((20000, 768), np.float32))
    assert ix.plan(1024, 10)["kernel"] == "tilelane128"
    ix.close()
    ix = DenseIndex(384, 90000, dtype="bf16", device=cuda)  # the other resident dimension
    ix.upsert(np.zeros((90000, 384), np.float32))
    assert ix.plan(1024, 10)["kernel"] == "qres256"
    ix.close()
    ix = DenseIndex(512, 90000, dtype="bf16", device=cuda)  # not a resident dimension
    ix.upsert(np.zeros((90000, 512), np.float32))
    assert ix.plan(1024, 10)["kernel"] != "qres256"
    ix.close()
    ix = DenseIndex(768, 90000, dtype="f32", device=cuda)  # exact mode keeps the fp32 tile kernel
    ix.upsert(np.zeros((90000, 768), np.float32))
    assert ix.plan(1024, 10)["kernel"] == "tilelane128"
    ix.close()


@pytest.mark.parametrize("sample,k,order", [(8192, 10, "asc"), (0, 10, "asc"), (0, 12, "asc"), (8192, 12, "desc"),
                                            (8192, 10, "split")])
def test_qres_adversarial_order(cuda, sample, k, order):
    """asc: rows sorted so that every row beats the ones before it for query 0 (each row a new
    record of that lane: the buffer fills and compacts again and again; every published maximum is
    low until the last split's); desc: the best rows first (block 0 of split 0 holds the top k, the
    first seed is exactly the k-th score: ties with the threshold); split: query 0's 64 best rows
    all inside the last split. Other queries see the same rows in clustered order."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(61 + sample + k)
    C = _clustered(rng, 40000, 768)
    Q = _clustered(rng, 1024, 768)
    s0 = C @ Q[0]
    if order == "asc":
        C = C[np.argsort(s0)]
    elif order == "desc":
        C = C[np.argsort(-s0)]
    else:
        top = np.argsort(-s0)[:64]
        rest = np.setdiff1d(np.arange(len(C)), top)
        C = np.concatenate([C[rest], C[top]])
    ix = DenseIndex(768, len(C), dtype="bf16", device=cuda)
    ix.upsert(C)
    ix.set_sample_rows(sample)
    _check_forms(ix, Q, k)
    ix.close()


def test_qres_ties_order_by_row(cuda):
    """bf16 duplicate rows score identically: the lowest row ids win, across blocks and splits."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(19)
    base = _clustered(rng, 300, 768)
    C = np.concatenate([base] * 120)  # 36000 rows, each vector 120 times
    pick = rng.integers(0, 300, 600)
    ix = DenseIndex(768, len(C), dtype="bf16", device=cuda)
    ix.upsert(C)
    for flags, k in ((QRES, 10), (QRES, 12), (QRES | PREPASS, 12)):
        s, r = _run(ix, base[pick], k, flags, "qres256")
        np.testing.assert_array_equal(r, pick[:, None] + 300 * np.arange(k)[None, :])
        assert (s == s[:, :1]).all()
    ix.close()


def test_qres_xcd_balanced_splits(cuda):
    """XCD-balanced splits (flag 1 << 28): the split bounds move with the per-XCD weights each
    launch sets for the next; every launch must still cover every row once — bitwise the tile
    kernel's answer, launch after launch as the weights settle."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(83)
    C = _clustered(rng, 90000, 768)
    Q = _clustered(rng, 1024, 768)
    ix = DenseIndex(768, len(C), dtype="bf16", device=cuda)
    ix.upsert(C)
    ref = _run(ix, Q, 10, *ref_of(ix.dim))
    for _ in range(6):
        s, r = _run(ix, Q, 10, QRES | (1 << 28), "qres256")
        np.testing.assert_array_equal(r, ref[1])
        np.testing.assert_array_equal(s, ref[0])
    ix.close()


@pytest.mark.parametrize("prepass", [False, True])
def test_qres_compaction_below_k(cuda, prepass):
    """k = 12 and a lane buffer compacted while it holds 11 keys: a threshold taken from fewer than k
    keys would exceed the lane's k-th best and drop the 12th. Query 0's 11 best rows all sit in one
    lane's rows of one block (the lane's 16 rows of a 32-row block are block offsets 0-3, 8-11,
    16-19, 24-27; 19 and 24-27 score low, so the next quad starts with 11 buffered keys and
    compacts), its 12th best in the same lane one block later; the split's other rows score -1.
    (That is the 32x32x16 form's lane map; the 16x16x32 form's lane fh = 0 holds block offsets 0-7
    and 16-23 in quads 0-3, 4-7, 16-19, 20-23: there rows 19 and 20-23 score low.)"""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(71)
    d, n, k = 768, 40000, 12
    C = dr.normalize_rows(rng.standard_normal((n, d)).astype(np.float32))
    Q = dr.normalize_rows(rng.standard_normal((1024, d)).astype(np.float32))
    q0 = Q[0]

    def at(cos):  # a unit row with cosine `cos` to q0
        u = rng.standard_normal(d).astype(np.float32)
        u -= (u @ q0) * q0
        u /= np.linalg.norm(u)
        return cos * q0 + np.sqrt(1 - cos * cos) * u

    base = 39520  # block 5 of the last split (64 splits of 1,250 row blocks: rows 39,360..)
    C[39360:] = -q0  # nothing else of that split enters the lane's buffer
    offs = (0, 1, 2, 3, 4, 5, 6, 7, 16, 17, 18) if ref_of(d)[0] == T256 else (0, 1, 2, 3, 8, 9, 10, 11, 16, 17, 18)
    for i, off in enumerate(offs):
        C[base + off] = at(0.99 - 0.01 * i)
    C[base + 32] = at(0.85)
    ix = DenseIndex(d, n, dtype="bf16", device=cuda)
    ix.upsert(C)
    flags = QRES | (PREPASS if prepass else 0)
    s, r = _run(ix, Q, k, flags, "qres256")
    assert r[0, k - 1] == base + 32, r[0]
    d_ = _run(ix, Q, k, *ref_of(ix.dim))
    np.testing.assert_array_equal(r, d_[1])
    np.testing.assert_array_equal(s, d_[0])
    ix.close()


def test_qres_sharded_keys(cuda):
    """row_base offsets and the key merge through the register-resident plan == one unsharded query
    (the C4 shape in miniature)."""
    from ah_rag.embeddings import DenseIndex, merge_topk_keys
    rng = np.random.default_rng(23)
    C = _clustered(rng, 120000, 768)
    Q = _clustered(rng, 1024, 768)
    full = DenseIndex(768, len(C), dtype="bf16", device=cuda)
    full.upsert(C)
    assert full.plan(len(Q), 10)["kernel"] == "qres256"
    fs, fr = [t.cpu().numpy() for t in full.query(Q, 10)]
    full.close()
    bounds = [0, 40001, 80000, 120000]
    lists = []
    for g in range(3):
        ix = DenseIndex(768, bounds[g + 1] - bounds[g], dtype="bf16", device=cuda)
        ix.upsert(C[bounds[g]:bounds[g + 1]])
        assert ix.plan(len(Q), 10)["kernel"] == "qres256"
        lists.append(ix.query_keys(Q, 10, row_base=bounds[g]))
        torch.cuda.synchronize()
        ix.close()
    s, r, _ = merge_topk_keys(torch.stack(lists, dim=1), 10)
    np.testing.assert_array_equal(r.cpu().numpy(), fr)
    np.testing.assert_array_equal(s.cpu().numpy(), fs)


def test_qres_concurrent_streams(cuda):
    """Two workspaces on two streams through the register-resident plan == the batches one by one
    (the fragment-major query copy is per workspace)."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(29)
    C = _clustered(rng, 40000, 768)
    Qs = [torch.from_numpy(_clustered(rng, B, 768)).to(cuda) for B in (1024, 700, 1024, 512)]
    ix = DenseIndex(768, len(C), dtype="bf16", device=cuda)
    ix.upsert(C)
    ix.set_debug_flags(QRES)
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
    ix.close()
    for j, (s, r) in enumerate(outs):
        np.testing.assert_array_equal(r.cpu().numpy(), serial[j % len(Qs)][1])
        np.testing.assert_array_equal(s.cpu().numpy(), serial[j % len(Qs)][0])


@pytest.mark.parametrize("dim,normalize", [(766, False), (768, True), (764, True)])
def test_qres_query_conversion_paths(cuda, dim, normalize):
    """dim % 4 == 0 converts the queries and writes the kernel's fragment-major copy in one launch;
    other dims (same d_pad = 768) take the conversion kernel plus the separate fragment copy: both
    must give the tile kernel's answer, with and without query normalisation."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(41 + dim)
    C = _clustered(rng, 40000, dim)
    Q = rng.standard_normal((700, dim)).astype(np.float32) * (3.0 if normalize else 1.0)
    if not normalize:
        Q = dr.normalize_rows(Q)
    ix = DenseIndex(dim, len(C), dtype="bf16", device=cuda)
    ix.upsert(C)
    outs = []
    for flags, kernel in ((QRES, "qres256"), ref_of(ix.dim)):
        ix.set_debug_flags(flags)
        assert ix.plan(len(Q), 10)["kernel"] == kernel
        outs.append([t.cpu().numpy() for t in ix.query(Q, 10, normalize=normalize)])
    ix.close()
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    np.testing.assert_array_equal(outs[0][0], outs[1][0])


def test_qres_consecutive_launches(cuda):
    """Back-to-back self-seeded launches on one workspace with changing batch sizes (so the split
    count, and the granule layout, change between launches) and k: every launch equals the tile
    kernel. Granules left by an earlier launch carry its epoch and must not seed this one."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(37)
    C = _clustered(rng, 60000, 768)
    ix = DenseIndex(768, len(C), dtype="bf16", device=cuda)
    ix.upsert(C)
    shapes = [(1024, 10), (512, 10), (2048, 12), (700, 1), (1024, 10), (600, 8)]
    Qs = [_clustered(rng, B, 768) for B, _ in shapes]
    ix.set_debug_flags(QRES)
    got = [[t.cpu().numpy() for t in ix.query(Q, k)] for Q, (_, k) in zip(Qs, shapes)]
    ix.set_debug_flags(ref_of(ix.dim)[0])
    for Q, (_, k), a in zip(Qs, shapes, got):
        b = [t.cpu().numpy() for t in ix.query(Q, k)]
        np.testing.assert_array_equal(a[1], b[1])
        np.testing.assert_array_equal(a[0], b[0])
    ix.close()


def test_qres_reserve_allocates_nothing(cuda):
    """After reserve() the self-seeded plan's query calls allocate nothing (graph-capturable): the
    fragment-major query copy and the seeding granules are sized by reserve."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(43)
    C = _clustered(rng, 40000, 768)
    Q = torch.from_numpy(_clustered(rng, 1024, 768)).to(cuda)
    ix = DenseIndex(768, len(C), dtype="bf16", device=cuda)
    ix.upsert(C)
    ix.reserve(1024, 12)
    torch.cuda.synchronize()
    s = torch.cuda.Stream(device=cuda)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        out = ix.query(Q, 10, stream=s)
    g.replay()
    torch.cuda.synchronize()
    ref = [t.cpu().numpy() for t in ix.query(Q, 10)]
    np.testing.assert_array_equal(out[1].cpu().numpy(), ref[1])
    np.testing.assert_array_equal(out[0].cpu().numpy(), ref[0])
    ix.close()


@pytest.mark.parametrize("d,n,B,k", [(768, 90000, 1024, 10), (384, 90000, 1024, 10), (768, 40001, 2048, 12)])
def test_qres_seed_wait_timeouts(cuda, d, n, B, k):
    """The bounded waits of the self-seeding (ahr_qres.hip: the first event polls up to 10 us for
    every split's block-0 granule, then for its queries' seeds) must only weaken the seed when
    they time out. Flag 4: split 0 tags everything it publishes, and compares what it reads,
    with a tag no launch has — the other splits never see its maxima or the seeds it selects
    (their waits on them run to the limit: the first event of every query block times out),
    and split 0 never sees theirs (it runs unseeded). Results: bitwise the tile kernel's, over
    several launches, and the launch takes longer by at least one timed-out wait."""
    from ah_rag.embeddings import DenseIndex
    rng = np.random.default_rng(97 + d + B)
    C = _clustered(rng, n, d)
    Q = _clustered(rng, B, d)
    ix = DenseIndex(d, n, dtype="bf16", device=cuda)
    ix.upsert(C)
    ref = _run(ix, Q, k, *ref_of(ix.dim))
    for flags in (QRES | MUTE, QRES, QRES | MUTE, QRES | MUTE):
        s, r = _run(ix, Q, k, flags, "qres256")
        np.testing.assert_array_equal(r, ref[1])
        np.testing.assert_array_equal(s, ref[0])

    def kernel_ms(flags, reps=20):
        ix.set_debug_flags(flags)
        ix.query(Q, k)
        torch.cuda.synchronize()
        ix.profile_begin(reps)
        for _ in range(reps):
            ix.query(Q, k)
        torch.cuda.synchronize()
        prof = ix.profile_end()
        ix.set_debug_flags(0)
        return prof["ms_sum"]["tile_topk"] / max(1, prof["calls"])

    plain, muted = kernel_ms(QRES), kernel_ms(QRES | MUTE)
    ix.close()
    print(f"seed-wait timeouts d={d} n={n} B={B}: kernel {plain * 1e3:.1f} us, with split 0 muted {muted * 1e3:.1f} us")
    assert muted > plain + 0.005  # at least one 10-us wait ran out (and split 0 ran unseeded)


def test_qres_large_corpus_plan(cuda):
    """From 512k rows (the corpus streams from HBM) qres256 is planned only where it seeds itself
    (>= 32 splits: B <= 2048 at k <= 12); larger batches keep kb256."""
    from ah_rag.embeddings import DenseIndex
    ix = DenseIndex(768, 600000, dtype="f16", device=cuda)
    ix.upsert(np.zeros((600000, 768), np.float32))
    assert ix.plan(1024, 10)["kernel"] == "qres256"
    assert ix.plan(2048, 10)["kernel"] == "qres256"
    assert ix.plan(4096, 10)["kernel"] == "kb256"
    assert ix.plan(8192, 10)["kernel"] == "kb256"
    ix.set_debug_flags(QRES)
    assert ix.plan(4096, 10)["kernel"] == "qres256"  # forced
    ix.close()
