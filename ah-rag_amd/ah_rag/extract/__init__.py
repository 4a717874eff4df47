from .fallback import HypergraphExtractor, fallback_extract

__all__ = ["HypergraphExtractor", "fallback_extract"]
