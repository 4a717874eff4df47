"""Deterministic offline ingest for the C1 plumbing path (BASELINE.json configs[0]).

Restates the reference's no-LLM extraction, HypergraphExtractor._fallback_extract and its helpers
(/root/reference/src/ah_rag/extract/hypergraph_extractor.py:214-264 and :325-336). The LLM
extraction itself (:71-187) is out of scope: without an endpoint the reference
ends in this fallback too (:80-82, :96-97), so for offline ingest the two agree.

Records are plain dicts in the key order of the reference's pydantic model_dump()
(hypergraph_schema.py:9-13): {"hyperedge", "relation_type", "entities": [{"name", "type",
"description"}], "confidence_score"} — exactly what demo_cli.py:96-97 writes to
artifacts/extractions.json and HierarchicalGraph.build_from_artifacts reads back.
"""
from __future__ import annotations

import re
from typing import Any, Dict, List

# sentence boundary: whitespace after a CJK or ASCII terminal mark (:217)
_SENTENCE_SPLIT = re.compile(r"(?<=[。！？.!?])\s+")
# one capitalised word, or a run of capitalised words separated by whitespace (:242)
_NAME = re.compile(r"(?:[A-Z][a-z]+(?:\s+[A-Z][a-z]+)+|[A-Z][a-z]+)")

# keyword groups of _infer_entity_type (:325-336), checked in this order
_WORK_CUES = (" film", " movie", " drama", "comedy")
_PERSON_CUES = (" director", " actor", "actress", "singer", "writer", "woman", "man", "person")
_PLACE_CUES = (" city", "neighborhood", "country", "state", "province")
_ROLE_CUES = (" government", "office", "position", "chief")

MAX_TEXT = 240  # hyperedge text / entity description cut (:225, :250)


def infer_entity_type(name: str, sentence: str) -> str:
    """Coarse type of a capitalised name from cue words in its sentence (:325-336)."""
    ctx = sentence.lower()
    if any(c in ctx for c in _WORK_CUES) and name.lower() in ctx:
        return "film"
    for cues, label in ((_PERSON_CUES, "person"), (_PLACE_CUES, "location"), (_ROLE_CUES, "role")):
        if any(c in ctx for c in cues):
            return label
    return "entity"


def sentence_entities(sentence: str) -> List[Dict[str, str]]:
    """Distinct capitalised names of a sentence, first occurrence order (:241-264)."""
    names = list(dict.fromkeys(_NAME.findall(sentence)))
    return [{"name": n, "type": infer_entity_type(n, sentence), "description": sentence[:MAX_TEXT]}
            for n in names]


def fallback_extract(text: str) -> List[Dict[str, Any]]:
    """One hyperedge per sentence that names at least one entity; a single DocumentSummary
    record when none does (:214-239)."""
    out: List[Dict[str, Any]] = []
    for sent in (s.strip() for s in _SENTENCE_SPLIT.split(text)):
        if not sent:
            continue
        ents = sentence_entities(sent)
        if ents:
            out.append({"hyperedge": sent[:MAX_TEXT],
                        "relation_type": "CoOccurrence" if len(ents) > 1 else "Mention",
                        "entities": ents, "confidence_score": 5.0})
    if not out:
        out.append({"hyperedge": text[:MAX_TEXT], "relation_type": "DocumentSummary",
                    "entities": [{"name": "Document", "type": "text", "description": text[:MAX_TEXT]}],
                    "confidence_score": 3.0})
    return out


class HypergraphExtractor:
    """Call shape of the reference class (hypergraph_extractor.py:10): extract(chunk) -> records.
    Offline-only: always the deterministic fallback."""

    def __init__(self, granularity: str = "fine") -> None:
        self.granularity = granularity

    def extract(self, text_chunk: str) -> List[Dict[str, Any]]:
        return fallback_extract(text_chunk)
