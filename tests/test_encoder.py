"""The GPU sentence encoder (ah_rag.encoder.TorchEncoder): the reference's
SentenceTransformer.encode seam (hierarchical_graph.py:655-656, :709-712) as a batched bf16 PyTorch
forward of the model's architecture on the MI355X.

No checkpoint exists offline, so weights are seeded random and the vectors are parity unpinned
against the pretrained model; these tests pin the encode contract instead: shapes, dtype,
normalisation, determinism, invariance to input order and batch size (bf16 tolerance: cosine
>= 0.999), and self-retrieval through the drop-in index and search path.
"""
import json
import os

import numpy as np
import pytest

C1 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c1")


def _texts(n=200, seed=3):
    rng = np.random.default_rng(seed)
    words = ["film", "director", "Tim", "Burton", "river", "city", "album", "band", "war", "novel",
             "Paris", "bridge", "1984", "station", "king", "queen", "of", "the", "and", "in"]
    return ["Entity: " + " ".join(rng.choice(words, size=int(rng.integers(1, 60)))) + "." for _ in range(n)]


def test_hash_tokenizer_contract():
    from ah_rag.encoder import CLS_ID, SEP_ID, FIRST_WORD_ID, HashTokenizer
    tok = HashTokenizer(30522, 16)
    a = tok(["Tim Burton, director.", "tim burton , DIRECTOR ."])
    assert a[0] == a[1]  # lower-cased, punctuation split off
    assert a[0][0] == CLS_ID and a[0][-1] == SEP_ID and len(a[0]) == 2 + 5
    assert all(FIRST_WORD_ID <= i < 30522 for i in a[0][1:-1])
    long = tok([" ".join(f"w{i}" for i in range(100))])[0]
    assert len(long) == 16 and long[-1] == SEP_ID  # truncated to max_seq_length
    assert HashTokenizer(30522, 16)(["Paris"]) == tok(["Paris"])  # deterministic across instances


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["all-MiniLM-L6-v2", "all-mpnet-base-v2"])
def test_torch_encoder_contract(cuda, model):
    import torch
    from ah_rag.encoder import TorchEncoder
    texts = _texts()
    enc = TorchEncoder(model, cuda)
    d = enc.get_sentence_embedding_dimension()
    assert d == (384 if "MiniLM" in model else 768) and not enc.pretrained
    v = enc.encode(texts, normalize_embeddings=True)
    assert v.shape == (len(texts), d) and v.dtype == np.float32 and np.isfinite(v).all()
    assert np.abs(np.linalg.norm(v, axis=1) - 1).max() < 1e-5
    # deterministic: a second instance (same seeded weights) gives the same vectors
    v2 = TorchEncoder(model, cuda).encode(texts, normalize_embeddings=True)
    np.testing.assert_allclose(v, v2, rtol=0, atol=1e-6)
    # order and batch size only regroup the padded batches: bf16 rounding differences at most
    rev = enc.encode(texts[::-1], normalize_embeddings=True)[::-1]
    one = enc.encode(texts[:40], normalize_embeddings=True, batch_size=1)
    assert (np.sum(v * rev, axis=1) > 0.999).all()
    assert (np.sum(v[:40] * one, axis=1) > 0.999).all()
    # device output and the single-string form
    t = enc.encode(texts[:8], normalize_embeddings=True, convert_to_tensor=True)
    assert isinstance(t, torch.Tensor) and t.device.type == "cuda" and t.shape == (8, d)
    s = enc.encode(texts[0], normalize_embeddings=True)
    assert s.shape == (d,) and float(np.dot(s, v[0])) > 0.999
    # unnormalised output is the mean-pooled hidden state (norm not 1)
    u = enc.encode(texts[:4])
    assert np.abs(np.linalg.norm(u, axis=1) - 1).max() > 1e-3


@pytest.mark.gpu
def test_torch_encoder_self_retrieval(cuda, tmp_path, monkeypatch):
    """The C1 graph indexed with the GPU encoder: each entity's own embedding text, searched
    through the drop-in HierarchicalGraph.search, returns that entity (or a node with the very
    same text) first."""
    import shutil
    monkeypatch.setenv("AHR_ENCODER", "torch")
    from ah_rag.graph.hierarchical_graph import HierarchicalGraph
    art = tmp_path / "artifacts"
    art.mkdir()
    shutil.copy(os.path.join(C1, "extractions.json"), art / "extractions.json")
    hg = HierarchicalGraph()
    hg.build_from_artifacts(str(art))
    hg.build_vector_index(db_path=str(tmp_path / "vdb"), layers={0, 1}, model_name="all-MiniLM-L6-v2", reset=True)
    ents = [n for n, d in hg.G.nodes(data=True) if d.get("node_type") == "entity"]
    texts = {n: hg._embedding_text(n)[0] for n in ents}
    by_text = {}
    for n, t in texts.items():
        by_text.setdefault(t, set()).add(n)
    sample = ents[::7]
    res = hg.search_batch([texts[n] for n in sample], top_k=1, return_cluster=True)
    for n, r in zip(sample, res):
        top = r["seeds"][0]
        assert top["node_id"] in by_text[texts[n]], n
        assert top["semantic"] > 0.999
    json.dumps(res)  # plain JSON-able result dicts, as the reference returns


@pytest.mark.gpu
def test_torch_encoder_rejects_unknown_names(cuda):
    """Unknown model names raise instead of silently becoming MiniLM with random weights."""
    from ah_rag.encoder import TorchEncoder
    with pytest.raises(ValueError, match="known architecture"):
        TorchEncoder("my-org/not-a-model", cuda)
