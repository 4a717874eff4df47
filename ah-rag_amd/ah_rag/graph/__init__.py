from .hierarchical_graph import HierarchicalGraph

__all__ = ["HierarchicalGraph"]
