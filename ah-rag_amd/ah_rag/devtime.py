"""Device-time accounting for host loops (the C5 bench's device/host split).

`recording()` turns on span recording for the block it wraps: every device pass that the search
pipeline and the environment expansions issue (SearchEngine.run's dense top-k + gather +
expansion/rerank, DeviceGraph.expand / lca) records a HIP event pair around its launches on the
stream they go to. `total_ms()` synchronises and sums the pairs: the GPU time of those passes
(each pass is followed by a host read of its results, so the spans do not overlap). Wall time
minus that sum is the host's share. Off by default: no events are recorded outside recording().
"""
from __future__ import annotations

import contextlib
from typing import List, Optional, Tuple

import torch

_pairs: Optional[List[Tuple[torch.cuda.Event, torch.cuda.Event]]] = None


@contextlib.contextmanager
def recording():
    """Record device spans inside the block; yields the list the spans go to."""
    global _pairs
    prev, _pairs = _pairs, []
    try:
        yield _pairs
    finally:
        _pairs = prev


def active() -> bool:
    """Whether spans are being recorded (callers on a hot path skip span() when not)."""
    return _pairs is not None


@contextlib.contextmanager
def span(stream: Optional[torch.cuda.Stream] = None, device: Optional[torch.device] = None):
    """A HIP event pair around the launches issued inside the block (on `stream`, or the
    device's current stream), when recording() is active; nothing otherwise."""
    pairs = _pairs
    if pairs is None:
        yield
        return
    s = stream if stream is not None else torch.cuda.current_stream(device)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    try:
        yield
    finally:
        b.record(s)
        pairs.append((a, b))


def total_ms(pairs: List[Tuple[torch.cuda.Event, torch.cuda.Event]]) -> float:
    """Sum of the recorded spans (synchronises on the last event)."""
    if not pairs:
        return 0.0
    pairs[-1][1].synchronize()
    return float(sum(a.elapsed_time(b) for a, b in pairs))
