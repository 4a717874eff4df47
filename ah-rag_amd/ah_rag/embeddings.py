"""ah_rag.embeddings — text encoders and the HBM-resident dense index.

Reference seams this module replaces (Yaron9/AH-RAG):
  * the SentenceTransformer encode calls, src/ah_rag/graph/hierarchical_graph.py:655-656 (corpus,
    normalize_embeddings=True) and :709-712 (query, cached per graph), and
    src/ah_rag/aggregate/semantic_aggregator.py:47,71-74;
  * the Chroma collection that stores the embeddings, hierarchical_graph.py:605-611 / :660 / :714.

The encoder stays a thin PyTorch call (north star: "not re-implemented"). sentence-transformers
is the default, as in the reference; this image has neither the package nor weights, so a run
here must choose another encoder explicitly (AHR_ENCODER=hash: deterministic, L2-normalised
stand-in vectors; AHR_ENCODER=torch: the model's architecture on the GPU). Nothing falls back
silently.

DenseIndex is the device half: fp32 vectors go in, the index keeps them row-major in HBM as
bf16 / f16 / f32 and answers batched top-k queries through libahr_hip.so. Nothing here falls
back to the CPU.
"""
from __future__ import annotations

import hashlib
import json
import os
from typing import Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import _native as nat

ArrayLike = Union[np.ndarray, torch.Tensor, Sequence[Sequence[float]]]

DEFAULT_MODEL = "all-MiniLM-L6-v2"  # hierarchical_graph.py:50,603,705
MODEL_DIMS = {"all-MiniLM-L6-v2": 384, "sentence-transformers/all-MiniLM-L6-v2": 384,
              "all-mpnet-base-v2": 768, "sentence-transformers/all-mpnet-base-v2": 768}


# ----------------------------------------------------------------------------------------------
# Encoders
# ----------------------------------------------------------------------------------------------
class HashEncoder:
    """Deterministic stand-in encoder: sha1(text) seeds a Gaussian vector, L2-normalised.

    Same call shape as SentenceTransformer.encode. Identical texts give identical vectors, so
    self-similarity is exactly 1 (the property test/test_embeddings.py:10-17 checks).
    """

    def __init__(self, model_name: str = DEFAULT_MODEL, dim: Optional[int] = None) -> None:
        self.model_name = model_name
        self.dim = int(dim or MODEL_DIMS.get(model_name, 384))

    def get_sentence_embedding_dimension(self) -> int:
        return self.dim

    def _one(self, text: str) -> np.ndarray:
        seed = int.from_bytes(hashlib.sha1(text.encode("utf-8")).digest()[:8], "little")
        return np.random.default_rng(seed).standard_normal(self.dim).astype(np.float32)

    def encode(self, texts: Union[str, Sequence[str]], normalize_embeddings: bool = False,
               show_progress_bar: bool = False, batch_size: int = 32, **_: object) -> np.ndarray:
        single = isinstance(texts, str)
        items = [texts] if single else list(texts)
        out = np.stack([self._one(t) for t in items]) if items else np.zeros((0, self.dim), np.float32)
        if normalize_embeddings and len(items):
            out = out / np.maximum(np.linalg.norm(out, axis=1, keepdims=True), 1e-12)
        out = out.astype(np.float32)
        return out[0] if single else out


class EncoderUnavailableError(RuntimeError):
    """The requested sentence encoder cannot be loaded (and no stand-in was asked for)."""


ENCODER_MODES = ("", "sentence-transformers", "hash", "torch")


def load_encoder(model_name: str = DEFAULT_MODEL, dim: Optional[int] = None):
    """The query / corpus encoder, chosen by AHR_ENCODER:

      unset or "sentence-transformers": SentenceTransformer(model_name), as the reference does
          (hierarchical_graph.py:8 imports it at module load, :655 / :709-711 construct it). If the
          package or the model cannot be loaded this raises EncoderUnavailableError — it never
          silently degrades to stand-in vectors (a broken model load would otherwise turn search()
          into hash-random retrieval with no signal);
      "hash": HashEncoder, the deterministic stand-in (tests and synthetic benchmarks);
      "torch": the model's architecture as a batched bf16 PyTorch forward on the GPU
          (ah_rag.encoder.TorchEncoder: a local checkpoint directory if `model_name` is one, else
          seeded random weights for a known architecture).
    """
    mode = os.environ.get("AHR_ENCODER", "").lower()
    if mode not in ENCODER_MODES:
        raise ValueError(f"AHR_ENCODER={mode!r}: expected one of {', '.join(repr(m) for m in ENCODER_MODES)}")
    if mode == "torch":
        from .encoder import torch_encoder
        return torch_encoder(model_name)
    if mode == "hash":
        return HashEncoder(model_name, dim)
    try:
        from sentence_transformers import SentenceTransformer  # type: ignore
    except ImportError as e:
        raise EncoderUnavailableError(
            "sentence-transformers is not installed; set AHR_ENCODER=torch (GPU forward of the model's "
            "architecture) or AHR_ENCODER=hash (deterministic stand-in vectors) to choose another encoder") from e
    device = "cuda" if torch.cuda.is_available() else "cpu"
    try:
        return SentenceTransformer(model_name, device=device)
    except Exception as e:
        raise EncoderUnavailableError(f"SentenceTransformer({model_name!r}) failed to load: {e}") from e


# ----------------------------------------------------------------------------------------------
# Dense index (device)
# ----------------------------------------------------------------------------------------------
def _as_f32_device(x: ArrayLike, device: torch.device) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        t = x.detach()
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(x, dtype=np.float32)))
    if t.dim() == 1:
        t = t.unsqueeze(0)
    if t.device.type == "cpu" and device.type == "cuda" and t.numel() <= (1 << 16):
        # a small host batch (the drop-in B = 1 search): staged in pinned memory and copied
        # asynchronously on the current stream, not a pageable copy that blocks the caller
        return t.to(torch.float32).contiguous().pin_memory().to(device, non_blocking=True)
    return t.to(device=device, dtype=torch.float32).contiguous()


class DenseIndex:
    """Row-major [capacity, dim] embedding matrix in HBM + exact batched top-k.

    Rows are identified by slot numbers 0..count-1 (the caller keeps the id table).
    dtype: "bf16" (default, north-star config), "f16", or "f32" (exact mode: every score is a
    k-ordered fp32 fma chain, bit-exact against oracle/ahr_oracle.c).
    """

    def __init__(self, dim: int, capacity: int, dtype: str = "bf16",
                 device: Optional[Union[int, str, torch.device]] = None) -> None:
        if not torch.cuda.is_available():
            raise nat.NativeLibraryError("DenseIndex needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.dim = int(dim)
        self.capacity = int(capacity)
        self.dtype = dtype
        if device is None:
            device = torch.cuda.current_device()
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        code = nat.DTYPE_CODES[dtype]
        h = nat.ctypes.c_void_p()
        nat.check(nat.lib().ahr_index_create(self.dim, code, self.capacity, self.device.index,
                                             nat.ctypes.byref(h)), "ahr_index_create")
        self._h = h
        self._seed = None       # caller's admission thresholds (set_seed)
        self._clusters = None   # cluster-probe seeding state (build_clusters)

    # -- lifecycle ---------------------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_clusters", None) is not None:
            self._clusters["index"].close()
            self._clusters = None
        if getattr(self, "_h", None) is not None and self._h.value:
            nat.lib().ahr_index_destroy(self._h)
            self._h = nat.ctypes.c_void_p()

    def __del__(self) -> None:
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self) -> nat.ctypes.c_void_p:
        return self._h

    def __len__(self) -> int:
        n = nat.ctypes.c_int64()
        nat.check(nat.lib().ahr_index_count(self._h, nat.ctypes.byref(n)), "ahr_index_count")
        return int(n.value)

    def info(self) -> dict:
        d, dt, pd = nat.ctypes.c_int(), nat.ctypes.c_int(), nat.ctypes.c_int()
        cap, rb = nat.ctypes.c_int64(), nat.ctypes.c_int64()
        nat.check(nat.lib().ahr_index_info(self._h, nat.ctypes.byref(d), nat.ctypes.byref(dt),
                                           nat.ctypes.byref(cap), nat.ctypes.byref(pd),
                                           nat.ctypes.byref(rb)), "ahr_index_info")
        return {"dim": d.value, "dtype": dt.value, "capacity": cap.value, "padded_dim": pd.value,
                "row_bytes": rb.value, "count": len(self)}

    # -- writes (hierarchical_graph.py:660) ----------------------------------------------------
    def upsert(self, vectors: ArrayLike, slots: Optional[ArrayLike] = None, start: int = 0,
               normalize: bool = False, stream: Optional[torch.cuda.Stream] = None) -> None:
        v = _as_f32_device(vectors, self.device)
        if v.shape[1] != self.dim:
            raise ValueError(f"vectors have dim {v.shape[1]}, index dim is {self.dim}")
        sl = None
        if slots is not None:
            sl = torch.as_tensor(np.asarray(slots, dtype=np.int64) if not isinstance(slots, torch.Tensor)
                                 else slots, dtype=torch.int64).to(self.device).contiguous()
            if sl.numel() != v.shape[0]:
                raise ValueError("one slot per vector")
        with torch.cuda.device(self.device):
            nat.check(nat.lib().ahr_index_upsert(self._h, nat.ptr(v), v.shape[0], nat.ptr(sl), int(start),
                                                 int(bool(normalize)), nat.stream_ptr(stream)),
                      "ahr_index_upsert")
            # keep the sources alive until the conversion kernel has consumed them
            (stream or torch.cuda.current_stream()).synchronize()

    def append(self, vectors: ArrayLike, normalize: bool = False) -> Tuple[int, int]:
        n0 = len(self)
        v = _as_f32_device(vectors, self.device)
        self.upsert(v, start=n0, normalize=normalize)
        return n0, n0 + v.shape[0]

    def truncate(self, count: int = 0) -> None:
        nat.check(nat.lib().ahr_index_truncate(self._h, int(count)), "ahr_index_truncate")

    def set_workspace(self, slot: int) -> None:
        """Query workspace (0..3) for the following queries: batches in flight on different
        streams must use different workspaces (include/ahr.h ahr_index_set_workspace)."""
        nat.check(nat.lib().ahr_index_set_workspace(self._h, int(slot)), "ahr_index_set_workspace")
        if self._clusters is not None:  # the centroid search runs inside every seeded query
            self._clusters["index"].set_workspace(slot)

    def reserve(self, max_batch: int, max_k: int = nat.AHR_MAX_K) -> None:
        with torch.cuda.device(self.device):
            nat.check(nat.lib().ahr_index_reserve(self._h, int(max_batch), int(max_k)), "ahr_index_reserve")
        if self._clusters is not None:
            self._clusters["index"].reserve(max_batch, self.PROBE_CLUSTERS)

    # -- cluster-probe seeds (the tile kernels' admission threshold) --------------------------
    PROBE_CLUSTERS = 8  # nearest clusters offered to the probe per query
    PROBE_MIN_ROWS = 64  # the probe stops walking clusters once it holds this many rows

    def build_clusters(self, n_clusters: Optional[int] = None, iters: int = 4, seed: int = 7) -> dict:
        """Coarse clusters of the stored rows, so that query() (B > 16, k <= 16, bf16/f16) seeds the
        fused kernels from each query's nearest clusters (ahr_index_probe_seed: the exact k-th best
        over those rows, less a rounding bound) instead of the sampled pre-pass. Spherical k-means:
        random member rows as initial centroids, assignment by this library's fused top-1 against
        a centroid index of the same dtype, centroids = normalised member means. Upserts and
        truncation after the build leave every seed valid (new rows are simply not probed); call
        again to refresh. Returns {"clusters", "rows", "empty"}."""
        if self.dtype == "f32":
            raise ValueError("cluster-probe seeds need a bf16 / f16 index")
        n = len(self)
        C = int(n_clusters or max(16, n // 22))
        if n < 2 * C:
            raise ValueError("too few rows for that many clusters")
        X = self.read()
        g = torch.Generator(device="cpu").manual_seed(seed)
        cent = torch.nn.functional.normalize(X[torch.randperm(n, generator=g)[:C].to(self.device)], dim=1)
        cidx = DenseIndex(self.dim, C, dtype=self.dtype, device=self.device)
        asg = torch.empty(n, dtype=torch.int64, device=self.device)
        for it in range(iters + 1):
            cidx.upsert(cent, start=0)
            for s0 in range(0, n, 1 << 18):
                asg[s0:s0 + (1 << 18)] = cidx.query(X[s0:s0 + (1 << 18)], 1)[1][:, 0].long()
            if it == iters:
                break
            acc = torch.zeros_like(cent).index_add_(0, asg, X)
            cnt = torch.bincount(asg, minlength=C)
            keep = cnt > 0
            cent[keep] = torch.nn.functional.normalize(acc[keep], dim=1)
        cnt = torch.bincount(asg, minlength=C)
        off = torch.zeros(C + 1, dtype=torch.int64, device=self.device)
        off[1:] = torch.cumsum(cnt, 0)
        rows = torch.argsort(asg, stable=True).to(torch.int32).contiguous()
        if self._clusters is not None:
            self._clusters["index"].close()
        self._clusters = {"index": cidx, "off": off, "rows": rows, "C": C}
        del X
        return {"clusters": C, "rows": n, "empty": int((cnt == 0).sum())}

    def drop_clusters(self) -> None:
        if self._clusters is not None:
            self._clusters["index"].close()
        self._clusters = None

    def _probe_seed(self, q: torch.Tensor, k: int, normalize: bool, stream) -> Optional[torch.Tensor]:
        """Device thresholds [B] from the query's nearest clusters (None: this call takes the
        sampled pre-pass: no clusters, the small-batch kernels, k > 16)."""
        c = self._clusters
        B = q.shape[0]
        if c is None or B <= 16 or k > 16:
            return None
        keys = c["index"].query_keys(q, self.PROBE_CLUSTERS, normalize=normalize, stream=stream)
        thr = torch.empty((B,), dtype=torch.float32, device=self.device)
        _on_stream(stream, self.device, thr)
        with torch.cuda.device(self.device):
            nat.check(nat.lib().ahr_index_probe_seed(self._h, nat.ptr(q), B, int(k), int(bool(normalize)),
                                                     nat.ptr(keys), self.PROBE_CLUSTERS, nat.ptr(c["off"]),
                                                     nat.ptr(c["rows"]), self.PROBE_MIN_ROWS, nat.ptr(thr),
                                                     nat.stream_ptr(stream)), "ahr_index_probe_seed")
        if stream is not None:
            keys.record_stream(stream)
        return thr

    def _seeded(self, q: torch.Tensor, k: int, normalize: bool, stream, launch) -> None:
        thr = self._probe_seed(q, k, normalize, stream)
        if thr is None:
            launch()
            return
        nat.check(nat.lib().ahr_index_set_seed(self._h, nat.ptr(thr)), "ahr_index_set_seed")
        try:
            launch()
        finally:  # back to the caller's seed (or the pre-pass)
            nat.check(nat.lib().ahr_index_set_seed(self._h, nat.ptr(self._seed)), "ahr_index_set_seed")

    def read(self, start: int = 0, n: Optional[int] = None) -> torch.Tensor:
        """Stored rows decoded to fp32 [n, dim] on the device (after dtype rounding)."""
        total = len(self)
        n = total - start if n is None else n
        out = torch.empty((n, self.dim), dtype=torch.float32, device=self.device)
        with torch.cuda.device(self.device):
            nat.check(nat.lib().ahr_index_read(self._h, int(start), int(n), nat.ptr(out), nat.stream_ptr()),
                      "ahr_index_read")
        return out

    # -- diagnostics --------------------------------------------------------------------------
    def set_sample_rows(self, rows: int) -> None:
        """Rows scored by the threshold pre-pass (0 disables it)."""
        nat.check(nat.lib().ahr_index_set_sample_rows(self._h, int(rows)), "ahr_index_set_sample_rows")

    def set_seed(self, thr: Optional[torch.Tensor]) -> None:
        """Admission thresholds for the next queries (device fp32 [>= B], one valid lower bound of
        each query's k-th best score), replacing the sampled pre-pass; None restores it. The
        tensor must stay alive while queries use it."""
        if thr is not None:
            if not (thr.is_cuda and thr.dtype == torch.float32 and thr.is_contiguous()):
                raise ValueError("seed must be a contiguous float32 device tensor")
        self._seed = thr
        nat.check(nat.lib().ahr_index_set_seed(self._h, nat.ptr(thr)), "ahr_index_set_seed")

    def set_debug_flags(self, flags: int) -> None:
        """Plan / A/B switches (include/ahr.h; a 32-bit unsigned word, unknown bits refused):
        4 = the register-resident kernel's split 0 seeds under a tag no launch has (its bounded
        waits time out; results unchanged: a test of that path), 8 = 128x128 tile kernel
        (cooperative), 32 = 128x128 lane-local kernel at any batch, 2048 = plan without the
        query-resident kernels, 4096 = the 128-query-resident (qkv) kernel wherever it applies (the
        ablation build only), 16384 = tilelane without the cross-tile prefetch, 32768 = the 256x256
        16x16x32 kernel (bf16/f16, k <= 16), 131072 / 262144 = always / never the k-blocked kernel,
        8192 = small batches (B <= 4) merged by the kernel's last workgroup (the fold) instead of
        the merge launch (the default), 1 << 22 = the merge launch even with 8192,
        1 << 23 = the 256-query register-resident kernel wherever it applies (bf16/f16, d 384/768,
        k <= 12), 1 << 26 = that kernel seeded by the sampled pre-pass instead of seeding itself, 1 << 27 = its
        self-seeding with the first event only, 1 << 28 / 1 << 19 = its splits XCD-balanced at any corpus
        size / never (default: from 256 row blocks per split).
        Garbage-result cost-split switches (2, 256, 512, 1024, 1 << 20, 1 << 21, 1 << 24, 1 << 25,
        1 << 29 .. 1 << 31) need the ablation build. Values outside [0, 2**32) raise ValueError."""
        flags = int(flags)
        if not 0 <= flags < 1 << 32:
            raise ValueError(f"debug flags must fit an unsigned 32-bit word, got {flags}")
        nat.check(nat.lib().ahr_index_set_debug_flags(self._h, flags), "ahr_index_set_debug_flags")

    _KERNELS = ("tile128", "lane256", "(retired)", "tilelane128", "(retired)", "qkv128", "t256", "small", "kb256",
                "(retired)", "qres256", "lane64")

    def plan(self, batch: int, k: int = 10) -> dict:
        """Launch geometry of a query of this batch size and top-k (diagnostics)."""
        kern, a, b, c = (nat.ctypes.c_int() for _ in range(4))
        nat.check(nat.lib().ahr_index_plan(self._h, int(batch), int(k), nat.ctypes.byref(kern), nat.ctypes.byref(a),
                                           nat.ctypes.byref(b), nat.ctypes.byref(c)), "ahr_index_plan")
        return {"kernel": self._KERNELS[kern.value], "n_splits": a.value, "tiles_per_split": b.value,
                "qblocks": c.value}

    def profile_begin(self, max_calls: int) -> None:
        """Record HIP events around each query stage for the next max_calls calls."""
        with torch.cuda.device(self.device):
            nat.check(nat.lib().ahr_index_profile_begin(self._h, int(max_calls)), "ahr_index_profile_begin")

    STAGES = ("convert", "threshold_prepass", "tile_topk", "merge")

    def profile_end(self) -> dict:
        """Per-stage summed milliseconds and the number of recorded calls."""
        arr = (nat.ctypes.c_float * 4)()
        n = nat.ctypes.c_int()
        with torch.cuda.device(self.device):
            nat.check(nat.lib().ahr_index_profile_end(self._h, arr, nat.ctypes.byref(n)), "ahr_index_profile_end")
        return {"calls": n.value, "ms_sum": {name: float(arr[i]) for i, name in enumerate(self.STAGES)}}

    # -- reads (hierarchical_graph.py:714) -----------------------------------------------------
    def query(self, queries: ArrayLike, k: int, normalize: bool = False,
              stream: Optional[torch.cuda.Stream] = None,
              out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """Exact top-k: (scores f32 [B,k] descending, rows int32 [B,k]) on the device.

        Ties order by row ascending; missing hits are (-inf, -1).
        """
        q = _as_f32_device(queries, self.device)
        if q.shape[1] != self.dim:
            raise ValueError(f"queries have dim {q.shape[1]}, index dim is {self.dim}")
        B = q.shape[0]
        if out is None:
            scores = torch.empty((B, k), dtype=torch.float32, device=self.device)
            rows = torch.empty((B, k), dtype=torch.int32, device=self.device)
        else:
            scores, rows = out
        _on_stream(stream, self.device, q, scores, rows)
        with torch.cuda.device(self.device):
            self._seeded(q, k, normalize, stream, lambda: nat.check(
                nat.lib().ahr_index_query(self._h, nat.ptr(q), B, int(k), int(bool(normalize)), nat.ptr(scores),
                                          nat.ptr(rows), nat.stream_ptr(stream)), "ahr_index_query"))
        return scores, rows

    def scores(self, queries: ArrayLike, normalize: bool = False,
               stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
        """Every score [B, count] fp32 on the device (ahr_index_scores: the tile kernel's GEMM core
        in scores mode; fp32 index = k-ordered fma chains)."""
        q = _as_f32_device(queries, self.device)
        n = len(self)
        out = torch.empty((q.shape[0], max(n, 1)), dtype=torch.float32, device=self.device)
        _on_stream(stream, self.device, q, out)
        with torch.cuda.device(self.device):
            nat.check(nat.lib().ahr_index_scores(self._h, nat.ptr(q), q.shape[0], int(bool(normalize)), nat.ptr(out),
                                                 out.shape[1], nat.stream_ptr(stream)), "ahr_index_scores")
        return out[:, :n]

    def query_keys(self, queries: ArrayLike, k: int, row_base: int = 0, normalize: bool = False,
                   stream: Optional[torch.cuda.Stream] = None,
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Packed uint64 keys [B,k] (as int64 tensor) for cross-shard merging."""
        q = _as_f32_device(queries, self.device)
        B = q.shape[0]
        keys = out if out is not None else torch.empty((B, k), dtype=torch.int64, device=self.device)
        _on_stream(stream, self.device, q, keys)
        with torch.cuda.device(self.device):
            self._seeded(q, k, normalize, stream, lambda: nat.check(
                nat.lib().ahr_index_query_keys(self._h, nat.ptr(q), B, int(k), int(bool(normalize)), int(row_base),
                                               nat.ptr(keys), nat.stream_ptr(stream)), "ahr_index_query_keys"))
        return keys


def _on_stream(stream: Optional[torch.cuda.Stream], device: torch.device, *tensors: torch.Tensor) -> None:
    """Before a launch on a non-current `stream`: order it after the current stream (which made
    the inputs and allocated the outputs) and tell the caching allocator that `stream` uses
    these blocks, so none is recycled before the kernel has consumed or written it."""
    if stream is None:
        return
    cur = torch.cuda.current_stream(device)
    if stream == cur:
        return
    stream.wait_stream(cur)
    for t in tensors:
        if t is not None and t.is_cuda:
            t.record_stream(stream)


def merge_topk_keys(keys: torch.Tensor, k: int, stream: Optional[torch.cuda.Stream] = None
                    ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Merge per-shard key lists [n_lists, B, k_in] (or [B, n_lists, k_in]) into the top k.

    Returns (scores f32 [B,k], rows int32 [B,k], keys int64 [B,k]) — the on-device merge that
    follows the RCCL all-gather of shard results.
    """
    if keys.dim() != 3:
        raise ValueError("keys must be [B, n_lists, k_in]")
    keys = keys.contiguous()
    B, n_lists, k_in = keys.shape
    dev = keys.device
    scores = torch.empty((B, k), dtype=torch.float32, device=dev)
    rows = torch.empty((B, k), dtype=torch.int32, device=dev)
    kout = torch.empty((B, k), dtype=torch.int64, device=dev)
    _on_stream(stream, dev, keys, scores, rows, kout)
    with torch.cuda.device(dev):
        nat.check(nat.lib().ahr_topk_merge(nat.ptr(keys), B, n_lists, k_in, int(k), nat.ptr(scores),
                                           nat.ptr(rows), nat.ptr(kout), nat.stream_ptr(stream)),
                  "ahr_topk_merge")
    return scores, rows, kout


def decode_keys(keys: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Host decode of packed keys (mirrors ahr_common.h)."""
    k = np.asarray(keys).astype(np.uint64)
    hi = (k >> np.uint64(32)).astype(np.uint32)
    lo = (k & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    u = np.where(hi & np.uint32(0x80000000), hi & np.uint32(0x7FFFFFFF), ~hi).astype(np.uint32)
    scores = u.view(np.float32).copy()
    rows = (np.uint32(0xFFFFFFFF) - lo).astype(np.int64)
    empty = k == 0
    scores[empty] = -np.inf
    rows[empty] = -1
    return scores, rows
