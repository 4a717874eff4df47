"""ah_rag.encoder — the sentence encoder as a thin PyTorch-ROCm forward on the GPU.

Reference seams: SentenceTransformer(model_name).encode(texts, normalize_embeddings=True) for the
corpus (src/ah_rag/graph/hierarchical_graph.py:655-656) and the query (:709-712), and the entity
encode of the aggregator (src/ah_rag/aggregate/semantic_aggregator.py:71-74). The north star keeps
the encoder "a thin PyTorch-ROCm call, not re-implemented": this module is exactly that — a
transformers BertModel of the named model's architecture, batched on the GPU in bf16, mean-pooled
over the attention mask and L2-normalised (what sentence-transformers does for all-MiniLM-L6-v2:
Transformer -> Pooling(mean) -> Normalize).

Weights. Neither sentence-transformers nor any checkpoint is present in this image or on the GPU
box (no network). So:
  * if `model_name` is a local directory holding a Hugging Face checkpoint (config.json +
    weights, tokenizer.json), that checkpoint and its tokenizer are loaded through AutoModel
    (local files only; BERT for MiniLM, MPNet for all-mpnet-base-v2);
  * otherwise, for a model name in the architecture table below, a BERT of that size is built
    with seeded random weights and a deterministic hash tokenizer (words -> ids by sha1); any
    other name raises. The forward pass is the real one
    (same layers, widths, sequence lengths, so the same GPU work and the same throughput); the
    vectors are not the pretrained model's and are labelled as such (`pretrained = False`).
The reference's own CPU path cannot run here either, so encoder outputs are parity
unpinned; what the tests pin is the encode contract (shapes, normalisation, determinism, order
and batch invariance, self-retrieval through the index).
"""
from __future__ import annotations

import hashlib
import os
import re
import threading
from typing import Dict, List, Optional, Sequence, Union

import numpy as np
import torch

# architecture of the reference's model names (hierarchical_graph.py:50,603,705: all-MiniLM-L6-v2;
# the north-star d = 768 is served by the BERT-base-sized mpnet entry: 12 layers x 768)
ARCHS: Dict[str, dict] = {
    "all-MiniLM-L6-v2": dict(hidden_size=384, num_hidden_layers=6, num_attention_heads=12,
                             intermediate_size=1536, vocab_size=30522, max_seq_length=256),
    "all-mpnet-base-v2": dict(hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                              intermediate_size=3072, vocab_size=30527, max_seq_length=384),
}
ARCHS["sentence-transformers/all-MiniLM-L6-v2"] = ARCHS["all-MiniLM-L6-v2"]
ARCHS["sentence-transformers/all-mpnet-base-v2"] = ARCHS["all-mpnet-base-v2"]

CLS_ID, SEP_ID, PAD_ID, FIRST_WORD_ID = 101, 102, 0, 1000
_WORD = re.compile(r"\w+|[^\w\s]", re.UNICODE)


class HashTokenizer:
    """Deterministic stand-in for the WordPiece tokenizer: lower-cased words and punctuation, each
    mapped to an id by sha1, framed as [CLS] ... [SEP] and truncated to max_seq_length."""

    def __init__(self, vocab_size: int, max_seq_length: int) -> None:
        self.vocab_size = int(vocab_size)
        self.max_seq_length = int(max_seq_length)
        self._cache: Dict[str, int] = {}

    def _id(self, w: str) -> int:
        i = self._cache.get(w)
        if i is None:
            h = int.from_bytes(hashlib.sha1(w.encode("utf-8")).digest()[:4], "little")
            i = self._cache[w] = FIRST_WORD_ID + h % (self.vocab_size - FIRST_WORD_ID)
        return i

    def __call__(self, texts: Sequence[str]) -> List[List[int]]:
        n = self.max_seq_length - 2
        return [[CLS_ID] + [self._id(w) for w in _WORD.findall(t.lower())[:n]] + [SEP_ID] for t in texts]


class _HFTokenizer:
    """A checkpoint's own tokenizer.json (tokenizers library), same call shape as HashTokenizer."""

    def __init__(self, path: str, max_seq_length: int) -> None:
        from tokenizers import Tokenizer
        self.tok = Tokenizer.from_file(path)
        self.tok.enable_truncation(max_seq_length)
        self.max_seq_length = max_seq_length

    def __call__(self, texts: Sequence[str]) -> List[List[int]]:
        return [e.ids for e in self.tok.encode_batch(list(texts))]


class TorchEncoder:
    """SentenceTransformer-shaped encoder: `encode(texts, normalize_embeddings, batch_size,
    convert_to_tensor)` -> float32 [n, d] (numpy, or a device tensor with convert_to_tensor)."""

    on_device = True  # search_batch asks for the device tensor

    def __init__(self, model_name: str = "all-MiniLM-L6-v2", device: Optional[Union[str, torch.device]] = None,
                 dtype: torch.dtype = torch.bfloat16, seed: int = 20251003) -> None:
        from transformers import AutoConfig, AutoModel, BertConfig, BertModel
        if not torch.cuda.is_available():
            raise RuntimeError("TorchEncoder runs the encoder forward on a ROCm GPU")
        self.model_name = model_name
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.dtype = dtype
        local = os.path.isdir(model_name) and os.path.exists(os.path.join(model_name, "config.json"))
        if local:  # a real checkpoint on local disk (never fetched), whatever its architecture
            cfg = AutoConfig.from_pretrained(model_name, local_files_only=True)
            extra = {"add_pooling_layer": False} if cfg.model_type in ("bert", "mpnet", "roberta",
                                                                        "xlm-roberta") else {}
            self.model = AutoModel.from_pretrained(model_name, local_files_only=True, attn_implementation="sdpa",
                                                   **extra)
            self.max_seq_length = min(512, int(getattr(self.model.config, "max_position_embeddings", 512)))
            tok_json = os.path.join(model_name, "tokenizer.json")
            self.tokenizer = _HFTokenizer(tok_json, self.max_seq_length) if os.path.exists(tok_json) else \
                HashTokenizer(self.model.config.vocab_size, self.max_seq_length)
            self.pretrained = True
        else:
            if model_name not in ARCHS:
                raise ValueError(f"TorchEncoder: {model_name!r} is neither a local checkpoint directory nor a "
                                 f"known architecture ({', '.join(sorted(ARCHS))})")
            arch = dict(ARCHS[model_name])
            self.max_seq_length = arch.pop("max_seq_length")
            cfg = BertConfig(max_position_embeddings=512, attn_implementation="sdpa", **arch)
            gen_state = torch.random.get_rng_state()
            torch.manual_seed(seed)  # the same random weights in every process
            self.model = BertModel(cfg, add_pooling_layer=False)
            torch.random.set_rng_state(gen_state)
            self.tokenizer = HashTokenizer(cfg.vocab_size, self.max_seq_length)
            self.pretrained = False
        self.model = self.model.to(device=self.device, dtype=dtype).eval()
        self.dim = int(self.model.config.hidden_size)
        # the checkpoint's own pad id (MPNet / RoBERTa vocabularies pad with 1: their id 0 is the
        # <s> token every sequence starts with); BERT and the seeded stand-in pad with 0
        pad = getattr(self.model.config, "pad_token_id", None)
        self.pad_id = int(pad) if pad is not None else PAD_ID

    def get_sentence_embedding_dimension(self) -> int:
        return self.dim

    @torch.inference_mode()
    def encode(self, texts: Union[str, Sequence[str]], normalize_embeddings: bool = False,
               show_progress_bar: bool = False, batch_size: int = 256, convert_to_tensor: bool = False,
               convert_to_numpy: bool = True, **_: object):
        single = isinstance(texts, str)
        items = [texts] if single else list(texts)
        out = torch.empty((len(items), self.dim), dtype=torch.float32, device=self.device)
        if items:
            ids = self.tokenizer(items)
            # longest first (as sentence-transformers does): batches of similar length, little padding
            order = sorted(range(len(ids)), key=lambda i: -len(ids[i]))
            for s in range(0, len(order), batch_size):
                sel = order[s:s + batch_size]
                L = max(len(ids[i]) for i in sel)
                tok = np.full((len(sel), L), self.pad_id, np.int64)
                for j, i in enumerate(sel):
                    tok[j, :len(ids[i])] = ids[i]
                tok_t = torch.from_numpy(tok).to(self.device, non_blocking=True)
                # the mask from the sequence lengths, not from token values (a real token may
                # share the pad id)
                lens = torch.as_tensor([len(ids[i]) for i in sel], device=self.device)
                mask = torch.arange(L, device=self.device).unsqueeze(0) < lens.unsqueeze(1)
                h = self.model(input_ids=tok_t, attention_mask=mask.to(torch.long)).last_hidden_state
                m = mask.unsqueeze(-1).to(torch.float32)
                pooled = (h.float() * m).sum(1) / m.sum(1).clamp_min(1e-9)  # mean pooling in fp32
                if normalize_embeddings:
                    pooled = torch.nn.functional.normalize(pooled, p=2.0, dim=1)
                out[torch.as_tensor(sel, device=self.device)] = pooled
        if convert_to_tensor:
            return out[0] if single else out
        arr = out.cpu().numpy()
        return arr[0] if single else arr


_CACHE: Dict[tuple, TorchEncoder] = {}
_LOCK = threading.Lock()


def torch_encoder(model_name: str, device: Optional[Union[str, torch.device]] = None) -> TorchEncoder:
    """One TorchEncoder per (model, device) per process (the reference caches its query encoder
    per graph, hierarchical_graph.py:709-711; corpus builds re-load it, here they reuse it)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    key = (model_name, str(dev))
    with _LOCK:
        enc = _CACHE.get(key)
        if enc is None:
            enc = _CACHE[key] = TorchEncoder(model_name, dev)
    return enc
