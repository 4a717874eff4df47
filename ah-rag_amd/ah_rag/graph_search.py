"""ah_rag.graph_search — the device graph and the batched search pipeline.

Reference behaviour reproduced (paths relative to Yaron9/AH-RAG):
  * HierarchicalGraph.search, src/ah_rag/graph/hierarchical_graph.py:675-789: dense top-k of the
    query against the node index (Chroma query :714), distance -> similarity (:719-724), 1-hop
    expansion (:726-740), rerank + 4-decimal rounding + stable sort (:742-782), return shapes
    (:783-789);
  * GraphEnvironment.expand_{parents,children,related}, src/ah_rag/agent/environment.py:393-480.

Everything after the query embedding runs on the GPU through libahr_hip.so:
  dense top-k  (ahr_index_query)  ->  row -> node map (one gather)  ->  expansion + rerank
  (ahr_graph_expand_rerank), batched over B queries, one stream, one host sync per batch.
The host only turns the small result arrays into the reference's dicts.

DeviceGraph mirrors the networkx graph as per-edge-type CSR lists in the exact order networkx
iterates neighbours (G.succ / G.pred), so the reference's [:2] / [:member_top_m] truncations and
the environment's limit/break rules see the same neighbour sequence.
"""
from __future__ import annotations

import functools
import itertools
import json
import math
import threading
from dataclasses import dataclass
from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple

import networkx as nx
import numpy as np
import torch

from . import _native as nat
from . import devtime
from .embeddings import _on_stream

EDGE_TYPES = ("belongs_to", "related_to", "participates_in")
# CSR list order of include/ahr.h: belongs_to out/in, related_to out/in, participates_in out/in
ADJ_SPECS = (("belongs_to", "out"), ("belongs_to", "in"), ("related_to", "out"),
             ("related_to", "in"), ("participates_in", "out"), ("participates_in", "in"))
ACTIONS = {"parents": 0, "children": 1, "related": 2}
_GRAPH_SERIALS = itertools.count(1)  # process-wide: caches key on it instead of id()

SEARCH_DEFAULTS = {  # hierarchical_graph.py:37-47
    "alpha": 0.6, "beta": 0.2, "gamma": 0.1, "delta": 0.1,
    "judge_overall_min": None, "confidence_min": None, "member_top_m": 5, "type_filter": None,
    "layer_boost": {"entity": 0.0, "summary": 1.0, "hyperedge": 0.0},
}


def _parse_judge_obj(obj: Any) -> Optional[float]:
    try:
        return float(obj.get("overall", 0.0))
    except Exception:
        return None


@functools.lru_cache(maxsize=1 << 16)
def _parse_judge_str(raw: str) -> Optional[float]:
    try:
        return _parse_judge_obj(json.loads(raw))
    except Exception:
        return None


def parse_judge(raw: Any) -> Optional[float]:
    """`overall` of a node's judge_scores (JSON string or dict); None when absent or unparsable.
    A string's value is a pure function of the string, so it is memoised (the batched search and
    the environments parse the same few thousand strings over and over)."""
    if not raw:
        return None
    if isinstance(raw, str):
        return _parse_judge_str(raw)
    return _parse_judge_obj(raw)


def _as_float(x: Any) -> float:
    if x is None:
        return math.nan
    try:
        return float(x)
    except (TypeError, ValueError):
        return math.nan


class DeviceGraph:
    """HBM copy of a networkx graph: node attribute table + 6 CSR adjacency lists."""

    def __init__(self, G: nx.DiGraph, device: Optional[torch.device] = None) -> None:
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        _d = torch.device(self.device)
        self._dev_index = _d.index if _d.index is not None else torch.cuda.current_device()
        self._xbufs: Dict[Tuple[int, int, int], Tuple] = {}  # expand_host's buffers per shape
        self._xlock = threading.Lock()  # expand_host: one caller at a time on the reused buffers
        self.serial = next(_GRAPH_SERIALS)
        self.ids: List[str] = list(G.nodes)
        self.index: Dict[str, int] = {nid: i for i, nid in enumerate(self.ids)}
        n = len(self.ids)
        self.n_nodes = n
        self.n_edges = G.number_of_edges()
        types = np.zeros(n, np.int8)
        judge = np.full(n, np.nan)
        conf = np.full(n, np.nan)
        for i, (nid, d) in enumerate(G.nodes(data=True)):
            types[i] = nat.NODE_TYPE_CODES.get(d.get("node_type"), nat.NODE_OTHER)
            j = parse_judge(d.get("judge_scores"))
            judge[i] = math.nan if j is None else j
            conf[i] = _as_float(d.get("confidence"))
        # Rerank terms with the reference's own float64 arithmetic (hierarchical_graph.py:766-767),
        # so the device score is bit-identical: 1/(1+np.exp(-(judge/10))) and conf/10.
        with np.errstate(over="ignore", invalid="ignore"):
            judge_term = np.array([1.0 / (1.0 + np.exp(-((j if j == j else 0.0) / 10.0))) for j in judge])
        conf_term = np.array([(c / 10.0) if c == c else 0.0 for c in conf])
        self.node_type = types
        self.judge = judge
        self.conf = conf
        offsets, targets = [], []
        for etype, direction in ADJ_SPECS:
            adj = G.succ if direction == "out" else G.pred
            off = np.zeros(n + 1, np.int64)
            tgt: List[int] = []
            for i, nid in enumerate(self.ids):
                for nb, attrs in adj[nid].items():
                    if attrs.get("edge_type") == etype:
                        tgt.append(self.index[nb])
                off[i + 1] = len(tgt)
            offsets.append(off)
            targets.append(np.asarray(tgt, np.int32) if tgt else np.zeros(1, np.int32))
        self._offsets, self._targets = offsets, targets  # host copies (env LCA / tests)
        off_ptrs = (nat.ctypes.c_void_p * nat.AHR_ADJ_COUNT)(*[o.ctypes.data for o in offsets])
        tgt_ptrs = (nat.ctypes.c_void_p * nat.AHR_ADJ_COUNT)(*[t.ctypes.data for t in targets])
        h = nat.ctypes.c_void_p()
        with torch.cuda.device(self.device):
            nat.check(nat.lib().ahr_graph_create(
                n, types.ctypes.data, judge.ctypes.data, conf.ctypes.data, judge_term.ctypes.data,
                conf_term.ctypes.data, off_ptrs, tgt_ptrs, self.device.index, nat.ctypes.byref(h)),
                "ahr_graph_create")
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            nat.lib().ahr_graph_destroy(self._h)
            self._h = nat.ctypes.c_void_p()

    def __del__(self) -> None:
        try:
            self.close()
        except Exception:
            pass

    # -- host helpers over the CSR mirror ------------------------------------------------------
    def neighbors(self, node: int, adj: int) -> np.ndarray:
        o = self._offsets[adj]
        return self._targets[adj][o[node]:o[node + 1]]

    def node_indices(self, ids: Sequence[str]) -> np.ndarray:
        return np.asarray([self.index.get(x, -1) for x in ids], np.int32)

    # -- device passes -------------------------------------------------------------------------
    def expand_rerank(self, seed_nodes: torch.Tensor, seed_sem: torch.Tensor, params: "RerankParams",
                      stream: Optional[torch.cuda.Stream] = None) -> "RerankResult":
        """seed_nodes int32 [B,k] (-1 absent; >= n_nodes = id unknown to the graph), seed_sem f32 [B,k]."""
        B, k = seed_nodes.shape
        dev = self.device
        fan = max(2, params.member_top_m)
        max_exp = max(1, k * (1 + fan))
        top_k = max(params.top_k, 0)
        kk = max(top_k, 1)
        # the eight outputs as views of one device arena: one host copy brings them all back
        arena, (en, es, ex, ec, on, osem, osc, oc) = _arena(dev, [
            ((B, max_exp), torch.int32), ((B, max_exp), torch.float64), ((B, max_exp), torch.int32),
            ((B,), torch.int32), ((B, kk), torch.int32), ((B, kk), torch.float64), ((B, kk), torch.float64),
            ((B,), torch.int32)])
        c = params.to_c()
        sn = seed_nodes.to(device=dev, dtype=torch.int32).contiguous()
        ss = seed_sem.to(device=dev, dtype=torch.float32).contiguous()
        _on_stream(stream, dev, sn, ss, arena)
        with torch.cuda.device(dev):
            nat.check(nat.lib().ahr_graph_expand_rerank(
                self._h, nat.ptr(sn), nat.ptr(ss), B, k, nat.ctypes.byref(c), max_exp,
                nat.ptr(en), nat.ptr(es), nat.ptr(ex), nat.ptr(ec), nat.ptr(on), nat.ptr(osem),
                nat.ptr(osc), nat.ptr(oc), nat.stream_ptr(stream)), "ahr_graph_expand_rerank")
        return RerankResult(en, es, ex, ec, on, osem, osc, oc, arena)

    def rerank_specs(self, B: int, k: int, params: "RerankParams"):
        """(shape, dtype) of expand_rerank's eight outputs for B queries of k seeds (_arena order)."""
        fan = max(2, params.member_top_m)
        max_exp = max(1, k * (1 + fan))
        kk = max(max(params.top_k, 0), 1)
        return [((B, max_exp), torch.int32), ((B, max_exp), torch.float64), ((B, max_exp), torch.int32),
                ((B,), torch.int32), ((B, kk), torch.int32), ((B, kk), torch.float64), ((B, kk), torch.float64),
                ((B,), torch.int32)]

    def expand_rerank_rows(self, rows: torch.Tensor, scores: torch.Tensor, row_to_node: torch.Tensor,
                           params: "RerankParams", max_exp: int, out_ptrs: Sequence[int], arena: torch.Tensor,
                           stream: Optional[torch.cuda.Stream] = None) -> None:
        """expand_rerank fed by the dense step's rows directly (ahr_graph_expand_rerank_rows: the
        row -> node gather inside the kernel); `out_ptrs` = device addresses of the eight outputs
        inside `arena`, laid out by rerank_specs (no tensor views: the caller reads them on the
        host only)."""
        B, k = rows.shape
        c = params.to_c()
        _on_stream(stream, self.device, rows, scores, row_to_node, arena)
        with torch.cuda.device(self.device):
            nat.check(nat.lib().ahr_graph_expand_rerank_rows(
                self._h, nat.ptr(rows), nat.ptr(row_to_node), int(row_to_node.shape[0]), nat.ptr(scores), B, k,
                nat.ctypes.byref(c), int(max_exp), *out_ptrs, nat.stream_ptr(stream)),
                "ahr_graph_expand_rerank_rows")

    def lca(self, inputs: torch.Tensor, max_out: int = 1024,
            stream: Optional[torch.cuda.Stream] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """Batched expand_to_lca core (ahr_graph_lca): inputs int32 [B, n_in] node indices ->
        (out int32 [B, max_out] unordered lowest common members, count int32 [B]; -1 = over the
        kernel's per-query capacity)."""
        B, n_in = inputs.shape
        dev = self.device
        out = torch.empty((B, max(max_out, 1)), dtype=torch.int32, device=dev)
        cnt = torch.empty((B,), dtype=torch.int32, device=dev)
        x = inputs.to(device=dev, dtype=torch.int32).contiguous()
        _on_stream(stream, dev, x, out, cnt)
        with torch.cuda.device(dev), devtime.span(stream, dev):
            nat.check(nat.lib().ahr_graph_lca(self._h, nat.ptr(x), B, n_in, int(max_out), nat.ptr(out), nat.ptr(cnt),
                                              nat.stream_ptr(stream)), "ahr_graph_lca")
        return out, cnt

    def lca_large(self, inputs: torch.Tensor, stream: Optional[torch.cuda.Stream] = None
                  ) -> Tuple[torch.Tensor, torch.Tensor]:
        """ahr_graph_lca_large: the same result as lca() without its per-query capacity (the
        visited set lives in a global-memory workspace of 5 * n_nodes int32 per query), for the
        queries lca() reported as over capacity. Chunked so the workspace stays <= 256 MiB."""
        B, n_in = inputs.shape
        dev = self.device
        n = max(self.n_nodes, 1)
        chunk = max(1, min(B, (256 << 20) // (20 * n)))
        outs, cnts = [], []
        x_all = inputs.to(device=dev, dtype=torch.int32).contiguous()
        for b0 in range(0, B, chunk):
            x = x_all[b0:b0 + chunk].contiguous()
            nb = x.shape[0]
            need = nat.ctypes.c_int64()
            nat.check(nat.lib().ahr_graph_lca_workspace(self._h, nb, nat.ctypes.byref(need)),
                      "ahr_graph_lca_workspace")
            ws = torch.empty((max(need.value // 4, 1),), dtype=torch.int32, device=dev)
            out = torch.empty((nb, n), dtype=torch.int32, device=dev)
            cnt = torch.empty((nb,), dtype=torch.int32, device=dev)
            _on_stream(stream, dev, x, ws, out, cnt)
            with torch.cuda.device(dev):
                nat.check(nat.lib().ahr_graph_lca_large(self._h, nat.ptr(x), nb, n_in, n, nat.ptr(out), nat.ptr(cnt),
                                                        nat.ptr(ws), need.value, nat.stream_ptr(stream)),
                          "ahr_graph_lca_large")
            outs.append(out)
            cnts.append(cnt)
        return torch.cat(outs), torch.cat(cnts)

    def expand(self, action: str, inputs: torch.Tensor, limit: int = 10,
               stream: Optional[torch.cuda.Stream] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """Batched environment expansion: inputs int32 [B, n_in] node indices (-1 = skip)."""
        B, n_in = inputs.shape
        dev = self.device
        arena, (out, cnt) = _arena(dev, [((B, max(limit, 1)), torch.int32), ((B,), torch.int32)])
        x = inputs.to(device=dev, dtype=torch.int32).contiguous()
        _on_stream(stream, dev, x, arena)
        with torch.cuda.device(dev), devtime.span(stream, dev):
            nat.check(nat.lib().ahr_graph_expand(self._h, ACTIONS[action], nat.ptr(x), B, n_in, int(limit),
                                                 nat.ptr(out), nat.ptr(cnt), nat.stream_ptr(stream)),
                      "ahr_graph_expand")
        return out, cnt

    def expand_host(self, action: str, idx: np.ndarray, limit: int = 10) -> Tuple[np.ndarray, np.ndarray]:
        """expand() of host node indices (int32 [B, n_in], -1 = skip) with host results (out
        [B, max(limit, 1)], count [B]) through ahr_graph_expand_host: one C call copies the inputs
        in, expands, copies both outputs back and waits. Pinned host buffers and the device
        workspace are kept per shape and reused; a lock makes concurrent callers (threads sharing
        one graph) take turns, so none overwrites another's staged inputs or results."""
        with self._xlock:
            return self._expand_host(action, idx, limit)

    def _expand_host(self, action: str, idx: np.ndarray, limit: int) -> Tuple[np.ndarray, np.ndarray]:
        B, n_in = idx.shape
        lim = max(limit, 1)
        key = (B, n_in, lim)
        b = self._xbufs.get(key)
        if b is None:
            if len(self._xbufs) >= 8:
                self._xbufs.clear()
            need = nat.ctypes.c_int64()
            nat.check(nat.lib().ahr_graph_expand_ws_bytes(B, n_in, int(limit), nat.ctypes.byref(need)),
                      "ahr_graph_expand_ws_bytes")
            ws_bytes = need.value
            ws = torch.empty(max(ws_bytes, 8), dtype=torch.uint8, device=self.device)
            x_host = torch.empty((B, n_in), dtype=torch.int32, pin_memory=True)
            res = torch.empty(B * lim + B, dtype=torch.int32, pin_memory=True)  # out [B][lim], then count [B]
            # (tensors kept alive by the tuple; their addresses resolved once)
            b = (ws, x_host, res, x_host.numpy(), res.numpy(),
                 (nat.ptr(x_host), B, n_in, int(limit), nat.ptr(res), nat.ptr(res) + 4 * B * lim, nat.ptr(ws),
                  ws_bytes))
            self._xbufs[key] = b
        x_np, res_np, args = b[3], b[4], b[5]
        np.copyto(x_np, idx, casting="same_kind")
        # (small batches: the library passes the inputs as kernel arguments and the kernel stores the
        # results straight into the pinned buffer, ahr_graph_expand_host)
        if devtime._pairs is None:
            st = nat.lib().ahr_graph_expand_host(self._h, ACTIONS[action], *args,
                                                 nat.stream_ptr(None, self._dev_index))
        else:
            with devtime.span(None, self.device):
                st = nat.lib().ahr_graph_expand_host(self._h, ACTIONS[action], *args,
                                                     nat.stream_ptr(None, self._dev_index))
        nat.check(st, "ahr_graph_expand_host")
        return res_np[:B * lim].reshape(B, lim).copy(), res_np[B * lim:].copy()

    # -- vectorised environment state (VecAHRAGGymEnv) -----------------------------------------
    ENV_PARTS = ("actions", "sel", "sel_n", "F", "F_end", "F_n", "S", "S_n", "kind", "seed_n", "f_shown", "f_size",
                 "s_size", "step", "vec", "err")

    @staticmethod
    def env_layout(E: int, K: int, fcap: int, scap: int) -> Tuple[List[int], int]:
        """(int32 element offsets of ahr_graph_env_layout's parts, total bytes)."""
        offs = (nat.ctypes.c_int64 * 16)()
        nbytes = nat.ctypes.c_int64()
        nat.check(nat.lib().ahr_graph_env_layout(E, K, fcap, scap, offs, nat.ctypes.byref(nbytes)),
                  "ahr_graph_env_layout")
        return list(offs), nbytes.value

    def env_buffers(self, E: int, K: int, fcap: int, scap: int):
        """(device workspace, pinned host mirror as an int32 numpy array, element offsets) of one
        environment batch's state (ahr_graph_env_step)."""
        offs, nbytes = self.env_layout(E, K, fcap, scap)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        host = torch.zeros(nbytes // 4, dtype=torch.int32, pin_memory=True)
        return (ws, host), host.numpy(), offs

    def env_node_table(self, feats: np.ndarray) -> torch.Tensor:
        """The featurizer's node table [m][6] (float64 on the host) as the fp32 device table
        ahr_graph_env_step reads (each value rounded once, as featurize_observation does)."""
        return torch.from_numpy(np.ascontiguousarray(feats, np.float32)).to(self.device)

    def env_upload(self, bufs, host_np: np.ndarray) -> None:
        """The host mirror's state -> the device workspace (after a reset)."""
        ws, host = bufs
        with torch.cuda.device(self.device):
            ws.view(torch.int32).copy_(host, non_blocking=True)

    def env_step(self, bufs, host_np: np.ndarray, E: int, K: int, fcap: int, scap: int, limit: int,
                 feats: Optional[torch.Tensor] = None) -> None:
        """One step of the environments whose actions sit in host_np's actions part: the kernel
        updates the device state (and, given the device node table `feats` [m][6] fp32, writes the
        new observations' featurizer vectors), and the whole workspace comes back into host_np (one
        C call)."""
        ws, host = bufs
        with devtime.span(None, self.device):
            nat.check(nat.lib().ahr_graph_env_step_host(
                self._h, E, K, fcap, scap, limit, nat.ptr(feats), 0 if feats is None else int(feats.shape[0]),
                host.data_ptr(), ws.data_ptr(), ws.numel(), host.data_ptr(),
                nat.stream_ptr(device_index=self.device.index)), "ahr_graph_env_step_host")


@dataclass
class RerankParams:
    alpha: float
    beta: float
    gamma: float
    delta: float
    judge_min: Optional[float]
    confidence_min: Optional[float]
    layer_boost: Dict[Any, float]
    type_filter: Optional[Iterable[str]]
    member_top_m: int
    top_k: int

    def key(self) -> Tuple:
        boost = self.layer_boost or {}
        tf = None if not self.type_filter else tuple(self.type_filter)
        return (self.alpha, self.beta, self.gamma, self.delta, self.judge_min, self.confidence_min,
                tuple(sorted(((str(k), k is None), float(v)) for k, v in boost.items())), tf,
                int(self.member_top_m), int(max(self.top_k, 0)))

    def to_c_cached(self) -> nat.RerankParams:
        """to_c() of these values, built once per distinct parameter set (the drop-in search resolves
        the same defaults on every call). The struct is shared: callers must not modify it."""
        k = self.key()
        c = _C_PARAMS.get(k)
        if c is None:
            if len(_C_PARAMS) >= 256:
                _C_PARAMS.clear()
            c = _C_PARAMS[k] = self.to_c()
        return c

    def to_c(self) -> nat.RerankParams:
        c = nat.RerankParams()
        c.alpha, c.beta, c.gamma, c.delta = (float(self.alpha), float(self.beta), float(self.gamma),
                                            float(self.delta))
        c.judge_min = math.nan if self.judge_min is None else float(self.judge_min)
        c.confidence_min = math.nan if self.confidence_min is None else float(self.confidence_min)
        boost = self.layer_boost or {}
        c.layer_boost[nat.NODE_OTHER] = float(boost.get(None, 0.0))
        for name, code in nat.NODE_TYPE_CODES.items():
            c.layer_boost[code] = float(boost.get(name, 0.0))
        mask = 0
        if self.type_filter:
            for t in self.type_filter:
                mask |= 1 << nat.NODE_TYPE_CODES.get(t, nat.NODE_OTHER) if t is not None else 1
        c.type_mask = mask
        c.member_top_m = int(self.member_top_m)
        c.top_k = int(max(self.top_k, 0))
        return c


_C_PARAMS: Dict[Tuple, nat.RerankParams] = {}


@dataclass
class RerankResult:
    exp_nodes: torch.Tensor
    exp_sem: torch.Tensor
    exp_src: torch.Tensor
    exp_count: torch.Tensor
    out_nodes: torch.Tensor
    out_sem: torch.Tensor
    out_score: torch.Tensor
    out_count: torch.Tensor
    arena: Optional[torch.Tensor] = None  # the device buffer the eight outputs are views of

    def to_host(self, *extra: torch.Tensor):
        """The result as host arrays (and `extra` tensors after it), one stream sync for all."""
        arrs = to_host_arrays(self.exp_nodes, self.exp_sem, self.exp_src, self.exp_count, self.out_nodes,
                              self.out_sem, self.out_score, self.out_count, *extra)
        res = RerankResult(*arrs[:8])
        return (res, *arrs[8:]) if extra else res


_ELEM = {torch.int32: (4, np.int32), torch.float64: (8, np.float64), torch.float32: (4, np.float32),
         torch.int64: (8, np.int64), torch.uint8: (1, np.uint8)}


def _layout(specs: Sequence[Tuple[Tuple[int, ...], torch.dtype]]) -> Tuple[List[int], int]:
    """8-byte aligned offsets of tensors of the given (shape, dtype)s in one buffer, and its size."""
    offs, total = [], 0
    for shape, dt in specs:
        offs.append(total)
        total += (math.prod(shape) * _ELEM[dt][0] + 7) // 8 * 8
    return offs, max(total, 8)


def _arena(dev: torch.device, specs: Sequence[Tuple[Tuple[int, ...], torch.dtype]], first: Optional[int] = None):
    """One uninitialised device buffer holding tensors of the given (shape, dtype)s (_layout):
    (buffer, views). With `first`, views of the first `first` only, and the offsets of all:
    (buffer, views, offsets) — the rest are passed to a kernel as addresses and read back with
    _host_views (a tensor view costs a few torch dispatches each)."""
    offs, total = _layout(specs)
    buf = torch.empty(total, dtype=torch.uint8, device=dev)
    views = []
    for (shape, dt), o in zip(specs[:first], offs):
        v = buf[o:o + math.prod(shape) * _ELEM[dt][0]].view(dt).view(shape)
        v._ahr_arena = (buf, o)  # (a dtype view is not tracked as a view of buf: to_host_arrays)
        views.append(v)
    return (buf, views) if first is None else (buf, views, offs)


def _host_views(host: np.ndarray, specs: Sequence[Tuple[Tuple[int, ...], torch.dtype]],
                offs: Sequence[int]) -> List[np.ndarray]:
    """numpy views of a host copy (uint8) of an _arena buffer, one per spec."""
    out = []
    for (shape, dt), o in zip(specs, offs):
        esz, npt = _ELEM[dt]
        out.append(host[o:o + math.prod(shape) * esz].view(npt).reshape(shape))
    return out


def to_host_arrays(*tensors: torch.Tensor) -> List[np.ndarray]:
    """Device tensors -> numpy with one synchronisation: asynchronous copies into pinned host
    memory on the current stream, then one wait (a .cpu() per tensor waits once per tensor; the
    single-environment loop made ~14 such round trips per episode). Views of one _arena buffer
    come back with one copy of that buffer."""
    if not tensors:
        return []
    dev = tensors[0].device
    if dev.type != "cuda":
        return [t.numpy() for t in tensors]
    srcs: Dict[int, torch.Tensor] = {}
    plan = []
    for t in tensors:
        ar = getattr(t, "_ahr_arena", None)
        if ar is not None:
            base, o = ar
            srcs.setdefault(id(base), base)
            plan.append((id(base), (o, t)))
        else:
            srcs[id(t)] = t
            plan.append((id(t), None))
    host = {k: v.to("cpu", non_blocking=True) for k, v in srcs.items()}
    torch.cuda.current_stream(dev).synchronize()
    host = {k: v.numpy() for k, v in host.items()}
    out = []
    for key, view in plan:
        if view is None:
            out.append(host[key])
            continue
        o, t = view
        esz, npt = _ELEM[t.dtype]
        out.append(host[key][o:o + t.numel() * esz].view(npt).reshape(tuple(t.shape)))
    return out


def resolve_search_params(stored: Dict[str, Any], top_k: int, member_top_m: Optional[int],
                          alpha, beta, gamma, delta, judge_overall_min, confidence_min,
                          type_filter) -> RerankParams:
    """Argument resolution of hierarchical_graph.py:682-699 (explicit value > graph meta > default)."""
    sp = {**SEARCH_DEFAULTS, **(stored or {})}

    def pick(v, key):
        return v if v is not None else sp.get(key)

    if type_filter is None:
        tf = sp.get("type_filter")
        type_filter = list(tf) if isinstance(tf, (set, tuple)) else tf
    return RerankParams(
        alpha=pick(alpha, "alpha"), beta=pick(beta, "beta"), gamma=pick(gamma, "gamma"),
        delta=pick(delta, "delta"), judge_min=pick(judge_overall_min, "judge_overall_min"),
        confidence_min=pick(confidence_min, "confidence_min"),
        layer_boost=sp.get("layer_boost", SEARCH_DEFAULTS["layer_boost"]), type_filter=type_filter,
        member_top_m=member_top_m if member_top_m is not None else sp.get("member_top_m", 5),
        top_k=top_k)


def _index_lock(index) -> threading.Lock:
    """One lock per DenseIndex (its query workspaces and the engines' reused buffers)."""
    lk = getattr(index, "_ahr_engine_lock", None)
    if lk is None:
        lk = threading.RLock()
        try:
            index._ahr_engine_lock = lk
        except AttributeError:
            pass
    return lk


class SearchEngine:
    """DenseIndex (node vectors) + row->node map + DeviceGraph: the batched search pipeline."""

    def __init__(self, index, row_ids: Sequence[str], row_metas: Sequence[Dict[str, Any]],
                 graph: DeviceGraph) -> None:
        self.index = index
        self.row_ids = list(row_ids)
        self.row_metas = list(row_metas)
        self.graph = graph
        n = graph.n_nodes
        rows = np.asarray([graph.index.get(r, n + i) for i, r in enumerate(self.row_ids)], np.int32)
        self.row_to_node_host = rows if len(rows) else np.zeros(1, np.int32)
        self.row_to_node = torch.from_numpy(self.row_to_node_host).to(graph.device)
        self.n_rows = len(self.row_ids)  # the index's row count when the engine was built (its version)
        self._bufs: Dict[Tuple, Tuple] = {}
        self._hbufs: Dict[Tuple, Tuple] = {}
        # the staging / result buffers are reused across calls: one caller at a time per index
        # (engines over the same index share its workspaces too), concurrent callers take turns
        self._lock = _index_lock(index)

    _BUF_SHAPES = 8  # result-buffer sets kept (one per batch shape / search parameter shape)

    def _buffers(self, specs, B: int, dim: int):
        """The device buffer of a search's outputs (dense scores / rows + the eight rerank arrays),
        its pinned host copy and a pinned + device query staging pair, per shape, reused across
        calls: run() synchronises before it returns, so no call touches a buffer a previous one
        still uses (one caller at a time per engine, like the reference's search())."""
        key = (tuple(specs), dim)
        b = self._bufs.get(key)
        if b is None:
            if len(self._bufs) >= self._BUF_SHAPES:
                self._bufs.clear()
            dev = self.graph.device
            arena, (scores, rows), offs = _arena(dev, specs, first=2)
            host = torch.empty(arena.numel(), dtype=torch.uint8, pin_memory=True)
            q_host = torch.empty((B, dim), dtype=torch.float32, pin_memory=True)
            q_dev = torch.empty((B, dim), dtype=torch.float32, device=dev)
            b = (arena, scores, rows, offs, [arena.data_ptr() + o for o in offs[2:]], host, host.numpy(),
                 q_host, q_host.numpy(), q_dev)
            self._bufs[key] = b
        return b

    def node_id(self, idx: int) -> str:
        n = self.graph.n_nodes
        return self.graph.ids[idx] if idx < n else self.row_ids[idx - n]

    HOST_PATH_MAX_B = 64  # host query batches up to this size take ahr_search_host (one C call)

    def run(self, query_vectors, params: RerankParams, stream: Optional[torch.cuda.Stream] = None,
            borrow: bool = False) -> Tuple[np.ndarray, np.ndarray, RerankResult]:
        """Dense top_k -> expansion -> rerank for a batch (a torch tensor, or a host numpy array).
        Returns host (rows, scores, result). borrow=True (the caller holds self._lock until it has
        read them): a small host batch's arrays are views of the engine's pinned result buffer,
        which the next call overwrites — no copy (search_batch assembles its dicts under the lock)."""
        with self._lock:
            if isinstance(query_vectors, np.ndarray):
                B = int(query_vectors.shape[0]) if query_vectors.ndim > 1 else 1
                if stream is None and 1 <= B <= self.HOST_PATH_MAX_B:
                    return self._run_host(query_vectors, params, borrow)
                query_vectors = torch.from_numpy(np.ascontiguousarray(query_vectors, np.float32))
            if stream is None and query_vectors.device.type == "cpu" and \
                    1 <= (query_vectors.shape[0] if query_vectors.dim() > 1 else 1) <= self.HOST_PATH_MAX_B:
                return self._run_host(query_vectors.numpy(), params, borrow)
            return self._run(query_vectors, params, stream)

    def _run_host(self, query_vectors: np.ndarray, params: RerankParams, borrow: bool = False
                  ) -> Tuple[np.ndarray, np.ndarray, RerankResult]:
        """A small host batch through ahr_search_host: query copy, dense top-k, expansion + rerank,
        result copy and stream wait in one C call, on the current stream (the drop-in search())."""
        B = int(query_vectors.shape[0]) if query_vectors.ndim > 1 else 1
        dim = int(query_vectors.shape[-1])
        k_dense = min(max(1, params.top_k), max(1, self.n_rows), nat.AHR_MAX_K_LARGE)
        max_exp = max(1, k_dense * (1 + max(2, params.member_top_m)))
        kk = max(max(params.top_k, 0), 1)
        key = (B, dim, k_dense, max_exp, kk)
        b = self._hbufs.get(key)
        if b is None:
            if len(self._hbufs) >= self._BUF_SHAPES:
                self._hbufs.clear()
            offs = (nat.ctypes.c_int64 * 10)()
            ws_b, ar_b = nat.ctypes.c_int64(), nat.ctypes.c_int64()
            nat.check(nat.lib().ahr_search_layout(B, dim, k_dense, max_exp, kk, offs, nat.ctypes.byref(ws_b),
                                                  nat.ctypes.byref(ar_b)), "ahr_search_layout")
            ws = torch.empty(ws_b.value, dtype=torch.uint8, device=self.graph.device)
            q_host = torch.empty((B, dim), dtype=torch.float32, pin_memory=True)
            out = torch.empty(ar_b.value, dtype=torch.uint8, pin_memory=True)
            specs = [((B, k_dense), torch.float32), ((B, k_dense), torch.int32)] + self.graph.rerank_specs(
                B, k_dense, params)
            out_np = out.numpy()
            scores_b, rows_b, *outs_b = _host_views(out_np, specs, list(offs))
            # (the fixed arguments of the C call, resolved once per buffer set)
            fixed = (self.graph._h, q_host.data_ptr(), B, k_dense, self.row_to_node.data_ptr(),
                     int(self.row_to_node.shape[0]))
            b = self._hbufs[key] = (ws, ws_b.value, q_host.numpy(), out, out_np, specs, list(offs), fixed,
                                    (rows_b, scores_b, RerankResult(*outs_b)), q_host)
        ws, ws_bytes, q_np, out, out_np, specs, offs, fixed, borrowed, _ = b
        np.copyto(q_np, query_vectors.reshape(B, dim), casting="same_kind")
        dev = self.graph.device
        args = (self.index.handle, *fixed, nat.ctypes.byref(params.to_c_cached()), max_exp, ws.data_ptr(), ws_bytes, out.data_ptr(),
                nat.stream_ptr(device_index=dev.index))
        if devtime.active():
            with devtime.span(None, dev):
                st = nat.lib().ahr_search_host(*args)
        else:
            st = nat.lib().ahr_search_host(*args)
        nat.check(st, "ahr_search_host")
        if borrow:  # views of the pinned buffer: valid until the next call (the caller holds the lock)
            return borrowed
        # one copy of the whole result buffer (the pinned one is the next call's), views into it
        scores_h, rows_h, *outs = _host_views(out_np.copy(), specs, offs)
        return rows_h, scores_h, RerankResult(*outs)

    def _run(self, query_vectors: torch.Tensor, params: RerankParams,
             stream: Optional[torch.cuda.Stream] = None) -> Tuple[np.ndarray, np.ndarray, RerankResult]:
        k = max(1, params.top_k)
        # rows past the index count come back as -1 anyway: ask for at most count (Chroma's
        # n_results clamp), so a small corpus answers any top_k
        k_dense = min(k, max(1, len(self.index)), nat.AHR_MAX_K_LARGE)
        B = int(query_vectors.shape[0]) if query_vectors.dim() > 1 else 1
        # the dense scores / rows and the eight rerank outputs in one device buffer: one host copy
        dev = self.graph.device
        specs = [((B, k_dense), torch.float32), ((B, k_dense), torch.int32)] + self.graph.rerank_specs(
            B, k_dense, params)
        dim = int(query_vectors.shape[-1])
        arena, scores, rows, offs, out_ptrs, host_t, host_np, q_host, q_host_np, q_dev = self._buffers(specs, B, dim)
        if query_vectors.device.type == "cpu":  # staged in pinned memory, copied on the current stream
            np.copyto(q_host_np, query_vectors.reshape(B, dim).numpy(), casting="same_kind")
            q_dev.copy_(q_host, non_blocking=True)
            query_vectors = q_dev
        with devtime.span(None, dev):  # (recorded on the current stream, after the waits)
            self.index.query(query_vectors, k_dense, stream=stream, out=(scores, rows))
            max_exp = specs[2][0][1]  # rerank_specs: exp_nodes is [B, max_exp]
            self.graph.expand_rerank_rows(rows, scores, self.row_to_node, params, max_exp, out_ptrs, arena,
                                          stream=stream)
            if stream is not None:  # the host copy runs on the current stream
                torch.cuda.current_stream(dev).wait_stream(stream)
        host_t.copy_(arena, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
        # (copies: the host buffer is the next call's)
        scores_h, rows_h, *outs = [v.copy() for v in _host_views(host_np, specs, offs)]
        host = RerankResult(*outs)
        return rows_h, scores_h, host
