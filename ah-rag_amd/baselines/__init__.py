"""Comparator RAG systems (reference baselines/)."""
