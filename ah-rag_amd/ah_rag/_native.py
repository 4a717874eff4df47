"""ctypes binding of libahr_hip.so (C ABI declared in include/ahr.h).

This is the only door into the MI355X kernels. There is no CPU fallback: if the shared library
is missing or does not load, every entry point raises NativeLibraryError.

torch is imported before the library is opened so that both share one HIP runtime
(torch's bundled libamdhip64.so.7 satisfies the library's DT_NEEDED entry).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch  # noqa: F401  (must precede the dlopen below; see module docstring)

LIB_NAME = "libahr_hip.so"
LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
LIB_PATH = os.environ.get("AHR_LIB_PATH", os.path.join(LIB_DIR, LIB_NAME))

# Status codes (include/ahr.h enum ahr_status)
AHR_OK = 0
AHR_EINVAL = -1
AHR_ENOMEM = -2
AHR_EHIP = -3
AHR_EUNSUP = -4
AHR_ERANGE = -5

# dtypes (enum ahr_dtype)
AHR_F32 = 0
AHR_F16 = 1
AHR_BF16 = 2
DTYPE_CODES = {"f32": AHR_F32, "fp32": AHR_F32, "float32": AHR_F32,
               "f16": AHR_F16, "fp16": AHR_F16, "float16": AHR_F16,
               "bf16": AHR_BF16, "bfloat16": AHR_BF16}

# node types (enum ahr_node_type)
NODE_OTHER, NODE_ENTITY, NODE_SUMMARY, NODE_HYPEREDGE = 0, 1, 2, 3
NODE_TYPE_CODES = {"entity": NODE_ENTITY, "summary": NODE_SUMMARY, "hyperedge": NODE_HYPEREDGE}
NODE_TYPE_NAMES = {NODE_ENTITY: "entity", NODE_SUMMARY: "summary", NODE_HYPEREDGE: "hyperedge",
                   NODE_OTHER: None}

AHR_MAX_K = 32          # fused kernels (and ahr_topk_merge)
AHR_MAX_K_LARGE = 4096  # ahr_index_query / _query_keys (scores + radix select beyond AHR_MAX_K)
AHR_ADJ_COUNT = 6

# Every symbol include/ahr.h declares (tests check the library exports all of them).
EXPORTED_SYMBOLS = (
    "ahr_abi_version", "ahr_last_error", "ahr_device_count",
    "ahr_index_create", "ahr_index_destroy", "ahr_index_upsert", "ahr_index_truncate",
    "ahr_index_count", "ahr_index_info", "ahr_index_rows", "ahr_index_read", "ahr_index_reserve",
    "ahr_index_profile_begin", "ahr_index_profile_end", "ahr_index_set_sample_rows", "ahr_index_set_seed", "ahr_index_probe_seed", "ahr_index_plan",
    "ahr_index_set_debug_flags", "ahr_index_set_workspace",
    "ahr_index_query", "ahr_index_query_keys", "ahr_index_scores", "ahr_topk_merge", "ahr_key_decode",
    "ahr_graph_create", "ahr_graph_destroy", "ahr_graph_expand_rerank", "ahr_graph_expand_rerank_rows",
    "ahr_graph_expand", "ahr_graph_expand_ws_bytes", "ahr_graph_expand_host",
    "ahr_graph_lca", "ahr_graph_lca_workspace", "ahr_graph_lca_large", "ahr_graph_info",
    "ahr_search_layout", "ahr_search_host", "ahr_graph_env_layout", "ahr_graph_env_step",
    "ahr_graph_env_step_host",
)


class NativeLibraryError(RuntimeError):
    """libahr_hip.so is missing, failed to load, or a call returned an error status."""


class RerankParams(ctypes.Structure):
    """struct ahr_rerank_params (include/ahr.h)."""
    _fields_ = [
        ("alpha", ctypes.c_double), ("beta", ctypes.c_double),
        ("gamma", ctypes.c_double), ("delta", ctypes.c_double),
        ("judge_min", ctypes.c_double), ("confidence_min", ctypes.c_double),
        ("layer_boost", ctypes.c_double * 4),
        ("type_mask", ctypes.c_int), ("member_top_m", ctypes.c_int), ("top_k", ctypes.c_int),
    ]


_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_int64


def _declare(lib: ctypes.CDLL) -> None:
    sig = {
        "ahr_abi_version": ([], _I),
        "ahr_last_error": ([], ctypes.c_char_p),
        "ahr_device_count": ([_P], _I),
        "ahr_index_create": ([_I, _I, _L, _I, _P], _I),
        "ahr_index_destroy": ([_P], _I),
        "ahr_index_upsert": ([_P, _P, _L, _P, _L, _I, _P], _I),
        "ahr_index_truncate": ([_P, _L], _I),
        "ahr_index_count": ([_P, _P], _I),
        "ahr_index_info": ([_P, _P, _P, _P, _P, _P], _I),
        "ahr_index_rows": ([_P, _P], _I),
        "ahr_index_read": ([_P, _L, _L, _P, _P], _I),
        "ahr_index_reserve": ([_P, _I, _I], _I),
        "ahr_index_profile_begin": ([_P, _I], _I),
        "ahr_index_profile_end": ([_P, _P, _P], _I),
        "ahr_index_set_sample_rows": ([_P, _I], _I),
        "ahr_index_set_seed": ([_P, _P], _I),
        "ahr_index_probe_seed": ([_P, _P, _I, _I, _I, _P, _I, _P, _P, _I, _P, _P], _I),
        "ahr_index_plan": ([_P, _I, _I, _P, _P, _P, _P], _I),
        "ahr_index_set_workspace": ([_P, _I], _I),
        "ahr_index_set_debug_flags": ([_P, ctypes.c_uint32], _I),
        "ahr_index_query": ([_P, _P, _I, _I, _I, _P, _P, _P], _I),
        "ahr_index_query_keys": ([_P, _P, _I, _I, _I, _L, _P, _P], _I),
        "ahr_index_scores": ([_P, _P, _I, _I, _P, _L, _P], _I),
        "ahr_topk_merge": ([_P, _I, _I, _I, _I, _P, _P, _P, _P], _I),
        "ahr_key_decode": ([_P, _L, _P, _P], _I),
        "ahr_graph_create": ([_L, _P, _P, _P, _P, _P, _P, _P, _I, _P], _I),
        "ahr_graph_destroy": ([_P], _I),
        "ahr_graph_expand_rerank": ([_P, _P, _P, _I, _I, ctypes.POINTER(RerankParams), _I,
                                     _P, _P, _P, _P, _P, _P, _P, _P, _P], _I),
        "ahr_graph_expand_rerank_rows": ([_P, _P, _P, _L, _P, _I, _I, ctypes.POINTER(RerankParams), _I,
                                          _P, _P, _P, _P, _P, _P, _P, _P, _P], _I),
        "ahr_graph_expand": ([_P, _I, _P, _I, _I, _I, _P, _P, _P], _I),
        "ahr_graph_expand_ws_bytes": ([_I, _I, _I, _P], _I),
        "ahr_graph_expand_host": ([_P, _I, _P, _I, _I, _I, _P, _P, _P, _L, _P], _I),
        "ahr_graph_lca": ([_P, _P, _I, _I, _I, _P, _P, _P], _I),
        "ahr_graph_lca_workspace": ([_P, _I, _P], _I),
        "ahr_graph_lca_large": ([_P, _P, _I, _I, _I, _P, _P, _P, _L, _P], _I),
        "ahr_graph_info": ([_P, _P, _P], _I),
        "ahr_search_layout": ([_I, _I, _I, _I, _I, _P, _P, _P], _I),
        "ahr_graph_env_layout": ([_I, _I, _I, _I, _P, _P], _I),
        "ahr_graph_env_step": ([_P, _I, _I, _I, _I, _I, _P, _L, _P, _L, _P], _I),
        "ahr_graph_env_step_host": ([_P, _I, _I, _I, _I, _I, _P, _L, _P, _P, _L, _P, _P], _I),
        "ahr_search_host": ([_P, _P, _P, _I, _I, _P, _L, ctypes.POINTER(RerankParams), _I, _P, _L, _P, _P], _I),
    }
    for name, (args, res) in sig.items():
        if not hasattr(lib, name):  # reported by the export test, not here
            continue
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res


def lib() -> ctypes.CDLL:
    """Load (once) and return the native library; raise NativeLibraryError if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise NativeLibraryError(
                    f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                    " (hipcc --offload-arch=gfx950). There is no CPU fallback.")
            try:
                handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            except OSError as e:
                raise NativeLibraryError(f"failed to load {LIB_PATH}: {e}") from e
            _declare(handle)
            _lib = handle
    return _lib


def available() -> bool:
    try:
        lib()
        return True
    except NativeLibraryError:
        return False


def check(status: int, what: str = "") -> None:
    if status != AHR_OK:
        msg = lib().ahr_last_error().decode("utf-8", "replace")
        raise NativeLibraryError(f"{what or 'ahr call'} failed with status {status}: {msg}")


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(stream: Optional["torch.cuda.Stream"] = None, device_index: Optional[int] = None) -> int:
    """hipStream_t of the given (or current) torch stream, as an integer for ctypes. With a
    device index and no stream: the current stream's handle without building a Stream object
    (a few microseconds per call on the B = 1 search path)."""
    if stream is None:
        if device_index is not None and _raw_stream is not None:
            return int(_raw_stream(device_index))
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream)


def ptr(t: Optional["torch.Tensor"]) -> Optional[int]:
    if t is None:
        return None
    return int(t.data_ptr())
