"""Parity at the exact BASELINE.json configurations, through the default plan the bench runs.

C2  hotpot90k: 90,000 x 768 (87k entity + 3k summary rows, SURVEY §8d generator), B = 1024,
    top-10. bf16 storage: scores within 1e-4 of the double-precision oracle on the same rounded
    inputs; rows equal except near-ties (a differing row's exact score is within 2e-5 of the
    oracle's score at that rank).
    fp32 exact mode: rows AND scores bit-identical to the oracle's k-ordered fma chain.
    numpy/BLAS cross-check (north_star: "outputs match the reference numpy/CPU path"): the fp32
    rows equal numpy's fp32 `Q @ C.T` + argpartition top-10 except near-ties (the two fp32
    accumulation orders differ by a few ulps; a swap is allowed only where the double-precision
    scores of the swapped rows are within 1e-5 of each other).
C2 at d = 384 (the reference's default all-MiniLM-L6-v2 width, hierarchical_graph.py:50, 603, 705):
    the same corpus generator at 90,000 x 384, B = 1024, bf16, every query against the f64 oracle
    with the C2 bf16 tolerances.
C3  synth5m: 5,000,000 x 768 fp16, B = 1024, top-10: a sampled subset of 256 queries (a quarter of
    the batch: every query block and split of the default plan) is checked against the oracle over
    the fp16-rounded corpus (chunked through host memory), same tolerances as C2 bf16.

References: the dense step replaces coll.query, /root/reference/src/ah_rag/graph/
hierarchical_graph.py:714 (exhaustive-cosine restatement: oracle/ahr_oracle.c).
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import dense_ref as dr

pytestmark = pytest.mark.gpu

K = 10
B = 1024


@pytest.fixture(scope="module")
def hotpot(cuda):
    from ah_rag.synthetic import HOTPOT_90K, SyntheticCorpus
    corpus = SyntheticCorpus(HOTPOT_90K, cuda)
    rows = corpus.rows()
    q, _ = corpus.queries(B, rows)
    return rows, q, rows.cpu().numpy(), q.cpu().numpy()


def _log_margin(name, **fields):
    """Parity margins (how many queries / rows differed and by how much) for DESIGN.md §4: printed,
    and appended to $AHR_PARITY_LOG as JSON lines when set (GPU runs keep them under profiles/)."""
    rec = {"test": name, **fields}
    print("parity-margin", json.dumps(rec))
    path = os.environ.get("AHR_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(rec) + "\n")


def _query(dtype, rows, q, cuda, expect_kernel=None):
    from ah_rag.embeddings import DenseIndex
    ix = DenseIndex(rows.shape[1], rows.shape[0], dtype=dtype, device=cuda)
    ix.upsert(rows)
    plan = ix.plan(q.shape[0], K)
    if expect_kernel is not None:
        assert plan["kernel"] == expect_kernel, plan
    s, r = ix.query(q, K)
    torch.cuda.synchronize()
    out = s.cpu().numpy(), r.cpu().numpy().astype(np.int64)
    ix.close()
    return out, plan


def _check_half(s, r, C, Q, es, er):
    """bf16/f16 contract: scores <= 1e-4 from the f64 oracle, rows equal except near-ties."""
    got_exact = np.einsum("bd,bkd->bk", Q.astype(np.float64), C[r].astype(np.float64))
    assert np.abs(s - got_exact).max() < 1e-4
    assert np.abs(s - es).max() < 1e-4
    mism = r != er
    gap = float(np.abs(got_exact[mism] - es[mism]).max()) if mism.any() else 0.0
    if mism.any():
        # a differing row is a near-tie: its exact score is within 2e-5 of the oracle's score at
        # that rank (adjacent swaps and substitutions at the k-th boundary alike)
        assert gap < 2e-5, int(mism.sum())
    return {"rows_differing": int(mism.sum()), "queries_differing": int(mism.any(axis=1).sum()),
            "max_exact_gap_at_differing_rank": gap, "max_score_err_vs_f64": float(np.abs(s - es).max())}


def test_c2_bf16_default_plan(hotpot, cuda):
    rows, q, C, Q = hotpot
    (s, r), plan = _query("bf16", rows, q, cuda)
    # the headline bench runs this exact plan (bench.py default workload)
    assert plan["kernel"] in ("qres256", "tilelane128", "t256"), plan
    Cr, Qr = dr.round_to_storage(C, "bf16"), dr.round_to_storage(Q, "bf16")
    es, er = dr.topk(Cr, Qr, K, mode="f64")
    m = _check_half(s, r, Cr, Qr, es, er)
    _log_margin("c2_bf16_default_plan", batch=B, k=K, kernel=plan["kernel"], **m)
    assert m["rows_differing"] <= B * K // 1000  # near-ties are rare (documented in DESIGN.md §4)


def test_c2_d384_bf16_default_plan(cuda):
    """The C2 workload at the reference's default embedding width (d = 384): rows and scores of
    every query against the f64 oracle on the storage-rounded inputs, the near-tie rule of
    _check_half, margins logged."""
    from ah_rag.synthetic import CorpusSpec, SyntheticCorpus
    corpus = SyntheticCorpus(CorpusSpec(dim=384), cuda)
    rows = corpus.rows()
    q, _ = corpus.queries(B, rows)
    (s, r), plan = _query("bf16", rows, q, cuda, expect_kernel="qres256")
    C, Q = rows.cpu().numpy(), q.cpu().numpy()
    Cr, Qr = dr.round_to_storage(C, "bf16"), dr.round_to_storage(Q, "bf16")
    es, er = dr.topk(Cr, Qr, K, mode="f64")
    m = _check_half(s, r, Cr, Qr, es, er)
    _log_margin("c2_d384_bf16_default_plan", batch=B, k=K, dim=384, kernel=plan["kernel"], **m)
    assert m["rows_differing"] <= B * K // 1000


def test_c2_f32_bit_exact(hotpot, cuda):
    rows, q, C, Q = hotpot
    (s, r), _ = _query("f32", rows, q, cuda)
    es, er = dr.topk(C, Q, K, mode="fma")
    np.testing.assert_array_equal(r, er)
    np.testing.assert_array_equal(s, es.astype(np.float32))


def test_c2_f32_vs_numpy_blas(hotpot, cuda):
    """fp32 rows vs numpy/BLAS fp32 (Q @ C.T + argpartition). Two fp32 accumulation orders of a
    d-term dot product each err by at most ~d * 2^-24 * sum|q_i x_i| (the standard forward bound),
    so rows a and b can trade places between the two paths only if their exact (double) scores are
    within the sum of those bounds for both rows and both paths; every difference must be such a
    pair, and the counts are recorded."""
    rows, q, C, Q = hotpot
    (s, r), _ = _query("f32", rows, q, cuda)
    _, nr = dr.topk_numpy(C, Q, K)  # the CPU baseline path: BLAS fp32 + argpartition
    Q64, C64 = Q.astype(np.float64), C.astype(np.float64)
    exact = lambda idx: np.einsum("bd,bkd->bk", Q64, C64[idx])
    absdot = lambda idx: np.einsum("bd,bkd->bk", np.abs(Q64), np.abs(C64[idx]))
    d = C.shape[1]
    u = 2.0 ** -24
    e_gpu, e_np = exact(r), exact(nr)
    a_gpu, a_np = absdot(r), absdot(nr)
    diff_q, diff_rows, worst_ratio = 0, 0, 0.0
    for b in range(B):
        if np.array_equal(r[b], nr[b]):
            continue
        diff_q += 1
        for i in range(K):
            if r[b, i] == nr[b, i]:
                continue
            diff_rows += 1
            # the two rows at rank i: their exact gap against the rounding bound of both paths
            bound = d * u * (a_gpu[b, i] + a_np[b, i])
            gap = abs(e_gpu[b, i] - e_np[b, i])
            worst_ratio = max(worst_ratio, gap / bound)
            assert gap <= bound, (b, i, r[b], nr[b], gap, bound)
    _log_margin("c2_f32_vs_numpy_blas", batch=B, k=K, queries_differing=diff_q, rows_differing=diff_rows,
                worst_gap_over_fp32_bound=worst_ratio)
    assert diff_q <= B // 50


def test_c2_bf16_b1_and_b16_small_kernel(hotpot, cuda):
    """The single-query / RL-env batch sizes at C2 take the streaming kernel."""
    rows, q, C, Q = hotpot
    Cr = dr.round_to_storage(C, "bf16")
    for b in (1, 16):
        (s, r), plan = _query("bf16", rows, q[:b], cuda)
        assert plan["kernel"] == "small", plan
        Qr = dr.round_to_storage(Q[:b], "bf16")
        es, er = dr.topk(Cr, Qr, K, mode="f64")
        m = _check_half(s, r, Cr, Qr, es, er)
        _log_margin(f"c2_bf16_b{b}", batch=b, k=K, kernel=plan["kernel"], **m)


def test_c2_bf16_b64(hotpot, cuda):
    """BASELINE.md's C2 batch sweep middle point, B = 64 (the 128-query tile path + pre-pass)."""
    rows, q, C, Q = hotpot
    Cr = dr.round_to_storage(C, "bf16")
    (s, r), plan = _query("bf16", rows, q[:64], cuda)
    assert plan["kernel"] != "small", plan
    Qr = dr.round_to_storage(Q[:64], "bf16")
    es, er = dr.topk(Cr, Qr, K, mode="f64")
    m = _check_half(s, r, Cr, Qr, es, er)
    _log_margin("c2_bf16_b64", batch=64, k=K, kernel=plan["kernel"], **m)


def test_c3_synth5m_f16_sampled(cuda):
    from ah_rag.embeddings import DenseIndex
    from ah_rag.synthetic import SYNTH_5M, SyntheticCorpus
    corpus = SyntheticCorpus(SYNTH_5M, cuda)
    N, d = SYNTH_5M.n_rows, SYNTH_5M.dim
    ix = DenseIndex(d, N, dtype="f16", device=cuda)
    chunks = []
    for start, x in corpus.entity_chunks():  # the bench's chunking (chunk seeds depend on it)
        ix.upsert(x, start=start)
        chunks.append((start, x.to(torch.float16).cpu()))  # host copy in storage precision
    # queries: the generator's scheme over the same rows (perturbed rows need the row values)
    g = torch.Generator(device="cpu").manual_seed(SYNTH_5M.seed + 7919)
    src = torch.randint(0, N, (B // 2,), generator=g)
    t = torch.randint(0, SYNTH_5M.n_centroids, (B - B // 2,), generator=g)
    eps = torch.randn(B, d, generator=g) / np.sqrt(d)
    base_rows = torch.empty(B // 2, d)
    for start, x in chunks:
        m = (src >= start) & (src < start + x.shape[0])
        if m.any():
            base_rows[m] = x[src[m] - start].float()
    base = torch.cat([base_rows, corpus.centroids[t.to(cuda)].cpu()])
    scale = torch.cat([torch.full((B // 2, 1), 0.2), torch.full((B - B // 2, 1), SYNTH_5M.noise)])
    qh = base + scale * eps
    qh = qh / qh.norm(dim=1, keepdim=True)
    q = qh.to(cuda)
    plan = ix.plan(B, K)
    s, r = ix.query(q, K)
    torch.cuda.synchronize()
    s, r = s.cpu().numpy(), r.cpu().numpy().astype(np.int64)
    ix.close()
    assert plan["kernel"] in ("qres256", "kb256"), plan  # the defaults at 5M rows (B >= 512 / below)
    pick = np.sort(np.random.default_rng(11).choice(B, 256, replace=False))
    Qr = dr.round_to_storage(qh.numpy()[pick], "f16")
    # oracle over the whole corpus, chunk by chunk (top-k of the union = top-k of chunk top-ks)
    best_s = np.full((len(pick), K), -np.inf)
    best_r = np.full((len(pick), K), -1, np.int64)
    for start, x in chunks:
        cs, cr = dr.topk(x.float().numpy(), Qr, K, mode="f64")
        alls = np.concatenate([best_s, cs], axis=1)
        allr = np.concatenate([best_r, cr + start], axis=1)
        order = np.lexsort((allr, -alls), axis=1)[:, :K]
        best_s, best_r = np.take_along_axis(alls, order, 1), np.take_along_axis(allr, order, 1)
    got_s, got_r = s[pick], r[pick]
    assert np.abs(got_s - best_s).max() < 1e-4
    mism = got_r != best_r
    if mism.any():
        # recompute the exact scores of the GPU's rows for the near-tie rule
        rows_h = {}
        for start, x in chunks:
            sel = np.unique(got_r[(got_r >= start) & (got_r < start + x.shape[0])])
            for rr in sel:
                rows_h[int(rr)] = x[rr - start].float().numpy().astype(np.float64)
        ex = np.array([[Qr[i].astype(np.float64) @ rows_h[int(got_r[i, j])] for j in range(K)]
                       for i in range(len(pick))])
        assert (np.abs(ex[mism] - best_s[mism]) < 2e-5).all()
    gap = float(np.abs(ex[mism] - best_s[mism]).max()) if mism.any() else 0.0
    _log_margin("c3_synth5m_f16_sampled", batch=B, k=K, sampled_queries=len(pick), kernel=plan["kernel"],
                rows_differing=int(mism.sum()), queries_differing=int(mism.any(axis=1).sum()),
                max_exact_gap_at_differing_rank=gap, max_score_err_vs_f64=float(np.abs(got_s - best_s).max()))
    # known-answer half: perturbed corpus rows should mostly find their source row
    hits = [int(src[i]) in set(r[i].tolist()) for i in range(B // 2)]
    assert np.mean(hits) > 0.95


@pytest.mark.parametrize("G", [2, 4, 8])
def test_c4_synth5m_row_shards_bitwise(cuda, G):
    """C4 (BASELINE configs[3]): the 5M x 768 f16 corpus row-sharded G ways exactly as
    ShardedDenseIndex shards it (rank g owns [g*N/G, (g+1)*N/G), row_base = lo_g), every shard
    answered by its own DenseIndex in this process (2.5M / 1.25M / 625k rows: the self-seeded qres256
    plan at B = 1024), the
    [B, G, k] key lists merged on the device (ahr_topk_merge, what follows the RCCL all-gather):
    the merged keys must equal the unsharded 5M answer bit for bit (scores, rows, tie order). The
    unsharded answer itself is checked against the oracle by test_c3_synth5m_f16_sampled."""
    from ah_rag.distributed import shard_bounds
    from ah_rag.embeddings import DenseIndex, decode_keys, merge_topk_keys
    from ah_rag.synthetic import SYNTH_5M, SyntheticCorpus
    corpus = SyntheticCorpus(SYNTH_5M, cuda)
    rows = corpus.rows()
    N, d = rows.shape
    q, _ = corpus.queries(B, rows)
    full = DenseIndex(d, N, dtype="f16", device=cuda)
    for s0 in range(0, N, 1_000_000):
        full.upsert(rows[s0:s0 + 1_000_000], start=s0)
    assert full.plan(B, K)["kernel"] in ("qres256", "kb256")
    want = full.query_keys(q, K).cpu().numpy()
    full.close()
    lists = []
    for lo, hi in shard_bounds(N, G):
        ix = DenseIndex(d, hi - lo, dtype="f16", device=cuda)
        for s0 in range(lo, hi, 1_000_000):
            ix.upsert(rows[s0:min(hi, s0 + 1_000_000)], start=s0 - lo)
        assert ix.plan(B, K)["kernel"] in ("qres256", "kb256"), (G, lo, hi, ix.plan(B, K))
        lists.append(ix.query_keys(q, K, row_base=lo))
        torch.cuda.synchronize()
        ix.close()
    gathered = torch.stack(lists, dim=1)  # [B, G, k], the all-gather's layout after the permute
    s, r, keys = merge_topk_keys(gathered, K)
    got = keys.cpu().numpy()
    np.testing.assert_array_equal(got, want)
    ws, wr = decode_keys(want)
    np.testing.assert_array_equal(r.cpu().numpy().astype(np.int64), wr)
    np.testing.assert_array_equal(s.cpu().numpy(), ws)
    print(f"C4 G={G}: {B}x{K} merged keys bitwise equal to the unsharded 5M answer")

