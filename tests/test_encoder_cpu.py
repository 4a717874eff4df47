"""Encoder selection is explicit: the reference imports sentence_transformers
at module load and fails loudly without it (/root/reference/src/ah_rag/graph/hierarchical_graph.py:
8); load_encoder must raise, never hand back stand-in vectors silently."""
import pytest


def test_default_encoder_raises_without_sentence_transformers(monkeypatch):
    pytest.importorskip("numpy")
    try:
        import sentence_transformers  # noqa: F401
        pytest.skip("sentence-transformers is installed here")
    except ImportError:
        pass
    from ah_rag.embeddings import EncoderUnavailableError, load_encoder
    monkeypatch.delenv("AHR_ENCODER", raising=False)
    with pytest.raises(EncoderUnavailableError, match="AHR_ENCODER"):
        load_encoder("all-MiniLM-L6-v2")
    monkeypatch.setenv("AHR_ENCODER", "sentence-transformers")
    with pytest.raises(EncoderUnavailableError):
        load_encoder("all-MiniLM-L6-v2")


def test_explicit_stand_in_and_bad_mode(monkeypatch):
    from ah_rag.embeddings import HashEncoder, load_encoder
    monkeypatch.setenv("AHR_ENCODER", "hash")
    enc = load_encoder("all-MiniLM-L6-v2")
    assert isinstance(enc, HashEncoder) and enc.get_sentence_embedding_dimension() == 384
    monkeypatch.setenv("AHR_ENCODER", "bogus")
    with pytest.raises(ValueError, match="AHR_ENCODER"):
        load_encoder("all-MiniLM-L6-v2")

