"""Ingest-side aggregation ops on the GPU: L1 topic relations."""
from .relations import generate_l1_relations

__all__ = ["generate_l1_relations"]
