"""Synthetic HotpotQA-shaped corpora: no dataset or encoder weights are
reachable offline, so the benchmark corpora are generated with a fixed seed.

C2  N = 90,000 rows = 87,000 entity + 3,000 summary, d = 768:
    entity row  = normalize(c[topic] + 0.35 * eps), eps ~ N(0, I/d), 3,000 unit centroids;
    summary row = normalize(mean of its member entity rows) (semantic_aggregator.py:194 analogue).
C3  N = 5,000,000 rows, same generator with 50,000 centroids, generated in chunks on the GPU.
Queries: half perturbed corpus rows normalize(x_r + 0.2 eps) (known source row), half fresh
cluster draws normalize(c[t] + 0.35 eps).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterator, Optional, Tuple

import numpy as np
import torch

SEED = 20251003


def _normalize(x: torch.Tensor) -> torch.Tensor:
    return x / x.norm(dim=1, keepdim=True).clamp_min(1e-12)


@dataclass
class CorpusSpec:
    n_entities: int = 87_000
    n_summaries: int = 3_000
    dim: int = 768
    n_centroids: int = 3_000
    noise: float = 0.35
    seed: int = SEED

    @property
    def n_rows(self) -> int:
        return self.n_entities + self.n_summaries


HOTPOT_90K = CorpusSpec()
SYNTH_5M = CorpusSpec(n_entities=5_000_000, n_summaries=0, n_centroids=50_000)


class SyntheticCorpus:
    """Deterministic corpus: rows are produced chunk by chunk on `device` (torch Generator)."""

    def __init__(self, spec: CorpusSpec = HOTPOT_90K, device: Optional[torch.device] = None) -> None:
        self.spec = spec
        self.device = device or torch.device("cpu")
        g = torch.Generator(device="cpu").manual_seed(spec.seed)
        self.centroids = _normalize(torch.randn(spec.n_centroids, spec.dim, generator=g)).to(self.device)
        self.topics = torch.randint(0, spec.n_centroids, (spec.n_entities,), generator=g)

    def entity_chunks(self, chunk: int = 100_000, lo: int = 0, hi: Optional[int] = None
                      ) -> Iterator[Tuple[int, torch.Tensor]]:
        """(start, rows) chunks of the entity rows; chunks entirely outside [lo, hi) are skipped
        without being generated (each chunk has its own seed, so any subset is reproducible)."""
        s = self.spec
        hi = s.n_entities if hi is None else hi
        for start in range(0, s.n_entities, chunk):
            n = min(chunk, s.n_entities - start)
            if start + n <= lo or start >= hi:
                continue
            g = torch.Generator(device=self.device).manual_seed(s.seed + 1 + start // chunk)
            eps = torch.randn(n, s.dim, generator=g, device=self.device) / np.sqrt(s.dim)
            t = self.topics[start:start + n].to(self.device)
            yield start, _normalize(self.centroids[t] + s.noise * eps)

    def rows(self) -> torch.Tensor:
        """All rows [n_rows, dim] fp32 on `device` (entities first, then summaries)."""
        s = self.spec
        out = torch.empty(s.n_rows, s.dim, dtype=torch.float32, device=self.device)
        for start, x in self.entity_chunks():
            out[start:start + x.shape[0]] = x
        if s.n_summaries:
            ent = out[:s.n_entities]
            topic = self.topics.to(self.device)
            # summaries = normalized member means over the first n_summaries topics
            sums = torch.zeros(s.n_centroids, s.dim, device=self.device)
            sums.index_add_(0, topic, ent)
            out[s.n_entities:] = _normalize(sums[:s.n_summaries] + 1e-6 * self.centroids[:s.n_summaries])
        return out

    def rows_at(self, idx: torch.Tensor) -> torch.Tensor:
        """rows()[idx] without materialising the corpus: the chunks holding idx are regenerated
        one at a time (a sharded rank never holds the other ranks' rows)."""
        s = self.spec
        idx = idx.to(torch.int64).cpu()
        if s.n_summaries and bool((idx >= s.n_entities).any()):
            return self.rows()[idx.to(self.device)]
        out = torch.empty(len(idx), s.dim, dtype=torch.float32, device=self.device)
        for start, x in self.entity_chunks():
            m = (idx >= start) & (idx < start + x.shape[0])
            if bool(m.any()):
                out[m.nonzero().squeeze(1).to(self.device)] = x[(idx[m] - start).to(self.device)]
        return out

    def queries(self, batch: int, rows: Optional[torch.Tensor] = None, salt: int = 0
                ) -> Tuple[torch.Tensor, torch.Tensor]:
        """(queries fp32 [batch, dim], source_row int64 [batch] or -1 for fresh draws). Without
        `rows`, the source rows are regenerated chunk by chunk (rows_at)."""
        s = self.spec
        g = torch.Generator(device="cpu").manual_seed(s.seed + 7919 * (salt + 1))
        half = batch // 2
        n_rows = rows.shape[0] if rows is not None else s.n_rows  # rows may be a truncated corpus
        src = torch.randint(0, n_rows, (half,), generator=g)
        t = torch.randint(0, s.n_centroids, (batch - half,), generator=g)
        eps = torch.randn(batch, s.dim, generator=g) / np.sqrt(s.dim)
        eps = eps.to(self.device)
        src_rows = rows[src.to(rows.device)].to(self.device) if rows is not None else self.rows_at(src)
        base = torch.cat([src_rows, self.centroids[t.to(self.device)]])
        scale = torch.cat([torch.full((half, 1), 0.2), torch.full((batch - half, 1), s.noise)]).to(self.device)
        q = _normalize(base + scale * eps)
        source = torch.cat([src, torch.full((batch - half,), -1, dtype=torch.int64)])
        return q, source


def build_hotpot_graph(corpus: SyntheticCorpus, rng: Optional[np.random.Generator] = None,
                       n_hyper: int = 40_000):
    """HotpotQA-distractor-shaped HierarchicalGraph over the corpus rows: one summary
    per topic (the first n_summaries topics), 1-2 belongs_to parents per entity, ~2 related_to per
    summary, n_hyper unindexed hyperedges of 2-5 same-topic participants. Returns (graph, ids),
    ids[r] = node id of corpus row r (entities first, then summaries, the rows() order)."""
    from .graph.hierarchical_graph import HierarchicalGraph
    rng = rng if rng is not None else np.random.default_rng(SEED)
    s = corpus.spec
    topics = corpus.topics.numpy()
    hg = HierarchicalGraph()
    sids = [hg.add_summary(t, title=f"Topic {t}", summary_text=f"summary of topic {t}",
                           confidence=float(rng.uniform(5, 10)), top_words=[f"w{t}", f"v{t}"],
                           judge_scores={"overall": float(rng.uniform(0, 10))}) for t in range(s.n_summaries)]
    eids = [hg.add_entity(f"entity {i}", description=f"entity {i} of topic {topics[i]}", entity_type="thing")
            for i in range(s.n_entities)]
    second = rng.integers(0, s.n_summaries, s.n_entities)
    for i, e in enumerate(eids):
        hg.add_belongs_to(e, sids[topics[i] % s.n_summaries], prob=0.9)
        if second[i] != topics[i] % s.n_summaries:
            hg.add_belongs_to(e, sids[second[i]], prob=0.1)
    for t in range(s.n_summaries):
        for u in rng.integers(0, s.n_summaries, 2):
            if u != t:
                hg.add_related(sids[t], sids[u], weight=0.5)
    by_topic: dict = {}
    for i, t in enumerate(topics):
        by_topic.setdefault(int(t), []).append(i)
    for h in range(n_hyper):
        pool = by_topic.get(int(rng.integers(0, s.n_centroids)))
        if not pool:
            continue
        k = min(len(pool), int(rng.integers(2, 6)))  # mean ~3.5-3.8 participants
        hid = hg.add_hyperedge(f"h{h}", description=f"relation {h}", relation_type="rel",
                               confidence_score=float(rng.uniform(0, 1)))
        for i in rng.choice(pool, k, replace=False):
            hg.add_participation(eids[int(i)], hid)
    return hg, eids + sids


def install_vectors(hg, ids, vectors: np.ndarray, db_path: str, model: str = "synthetic") -> None:
    """What build_vector_index (hierarchical_graph.py:602-673) stores for the nodes `ids`, with
    given corpus vectors instead of an encoder's (no weights offline): the on-disk vector store and
    G.graph["vector_index"] with its sha1 indexed_meta."""
    from .graph.hierarchical_graph import VectorStore
    store = VectorStore(db_path)
    store.clear()
    metas = [hg._embedding_text(n)[1] for n in ids]
    store.upsert(ids, np.asarray(vectors, np.float32), metas)
    store.save(model)
    hg.G.graph["vector_index"] = {"db_path": db_path, "model": model, "indexed_nodes": len(ids),
                                  "indexed_meta": {n: hg._index_key(hg.G.nodes[n]) for n in ids}}
    hg.G.graph["dirty"] = False
