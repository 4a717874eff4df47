// Error channel and process-level queries of the C ABI (include/ahr.h).
#include "ahr_common.h"
#include "ahr_internal.h"
#include "ahr.h"

#include <stdlib.h>

#include <string>

namespace ahr {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return AHR_EHIP;
}

}  // namespace ahr

extern "C" {

int ahr_abi_version(void) { return AHR_ABI_VERSION; }

const char* ahr_last_error(void) { return ahr::g_last_error.c_str(); }

int ahr_device_count(int* n) {
  if (!n) return ahr::fail(AHR_EINVAL, "null out pointer");
  AHR_HIP(hipGetDeviceCount(n));
  return AHR_OK;
}

// ---- the drop-in search() in one call (include/ahr.h ahr_search_host) ----------------------
int ahr_search_layout(int B, int dim, int k_dense, int max_exp, int kk, int64_t offsets[10], int64_t* ws_bytes,
                      int64_t* arena_bytes) {
  if (!offsets || !ws_bytes || !arena_bytes) return ahr::fail(AHR_EINVAL, "null output");
  if (B < 1 || dim < 1 || k_dense < 1 || max_exp < 1 || kk < 1) return ahr::fail(AHR_EINVAL, "sizes must be >= 1");
  const int64_t b = B;
  const int64_t part[10] = {b * k_dense * 4, b * k_dense * 4, b * max_exp * 4, b * max_exp * 8, b * max_exp * 4,
                            b * 4,           b * kk * 4,      b * kk * 8,      b * kk * 8,      b * 4};
  int64_t o = 0;
  for (int i = 0; i < 10; ++i) {
    offsets[i] = o;
    o += (part[i] + 7) / 8 * 8;
  }
  *arena_bytes = o;
  *ws_bytes = (b * dim * 4 + 255) / 256 * 256 + o;
  return AHR_OK;
}

int ahr_search_host(ahr_index* ix, ahr_graph* g, const float* host_q, int B, int k_dense,
                    const int32_t* row_to_node, int64_t n_rows, const ahr_rerank_params* params, int max_exp,
                    void* ws, int64_t ws_bytes, void* host_out, void* stream) {
  if (!ix || !g || !params) return ahr::fail(AHR_EINVAL, "null index, graph or params");
  if (!host_q || !row_to_node || !ws || !host_out) return ahr::fail(AHR_EINVAL, "null buffer");
  int dim = 0, dt = 0, pd = 0;
  int64_t cap = 0, rb = 0;
  int st = ahr_index_info(ix, &dim, &dt, &cap, &pd, &rb);
  if (st != AHR_OK) return st;
  const int kk = params->top_k > 0 ? params->top_k : 1;
  int64_t off[10], need = 0, arena = 0;
  st = ahr_search_layout(B, dim, k_dense, max_exp, kk, off, &need, &arena);
  if (st != AHR_OK) return st;
  if (ws_bytes < need) return ahr::fail(AHR_EINVAL, "workspace smaller than ahr_search_layout's ws_bytes");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  char* q = static_cast<char*>(ws);
  char* a = q + ((int64_t)B * dim * 4 + 255) / 256 * 256;
  // AHR_SEARCH_SKIP (diagnostic cost split, wrong results): bit 0 skips the query copy, bit 1 the
  // result copy, bit 2 the rerank launch
  static const int skip = [] {
    const char* e = getenv("AHR_SEARCH_SKIP");
    return e ? atoi(e) : 0;
  }();
  if (!(skip & 1)) AHR_HIP(hipMemcpyAsync(q, host_q, (size_t)B * dim * 4, hipMemcpyHostToDevice, s));
  float* scores = reinterpret_cast<float*>(a + off[0]);
  int32_t* rows = reinterpret_cast<int32_t*>(a + off[1]);
  // the small-batch plan's per-split lists are merged by the rerank kernel itself (one launch and
  // its gap fewer) when that kernel is the wave one; AHR_SEARCH_FUSE=0 keeps the merge launch (A/B,
  // bitwise equal)
  static const bool fuse = [] {
    const char* e = getenv("AHR_SEARCH_FUSE");
    return !(e && atoi(e) == 0);
  }();
  const uint64_t* lists = nullptr;
  int n_lists = 0;
  if (fuse && !(skip & 4) && ahr::graph_rerank_fusable(k_dense, params))
    st = ahr::dense_query_lists(ix, reinterpret_cast<const float*>(q), B, k_dense, 0, scores, rows, stream, &lists,
                                &n_lists);
  else
    st = ahr_index_query(ix, reinterpret_cast<const float*>(q), B, k_dense, 0, scores, rows, stream);
  if (st != AHR_OK) return st;
  // With the fused merge every output of the rerank kernel — the merged dense rows / scores too — is
  // written once and never read back, so when host_out is pinned (device-visible) host memory the
  // kernel writes the results there directly: no result copy (AHR_SEARCH_ZC=0 keeps the copy). (The
  // round-5 zero-copy form also had the rerank kernel read the dense results from host memory: slower.)
  static const bool zc = [] {
    const char* e = getenv("AHR_SEARCH_ZC");
    return !(e && atoi(e) == 0);
  }();
  char* o = a;
  if (lists && zc && !(skip & 2)) {
    // checked on every call (a cached answer could outlive the buffer: a pageable buffer at a freed
    // pinned one's address would take device writes)
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, host_out) == hipSuccess && at.type == hipMemoryTypeHost && at.devicePointer)
      o = static_cast<char*>(at.devicePointer);
    else
      (void)hipGetLastError();  // (a pageable buffer's lookup error is not the call's)
  }
  if (o != a) {
    scores = reinterpret_cast<float*>(o + off[0]);
    rows = reinterpret_cast<int32_t*>(o + off[1]);
  }
  int32_t* o2 = reinterpret_cast<int32_t*>(o + off[2]);
  double* o3 = reinterpret_cast<double*>(o + off[3]);
  int32_t* o4 = reinterpret_cast<int32_t*>(o + off[4]);
  int32_t* o5 = reinterpret_cast<int32_t*>(o + off[5]);
  int32_t* o6 = reinterpret_cast<int32_t*>(o + off[6]);
  double* o7 = reinterpret_cast<double*>(o + off[7]);
  double* o8 = reinterpret_cast<double*>(o + off[8]);
  int32_t* o9 = reinterpret_cast<int32_t*>(o + off[9]);
  if (lists)
    st = ahr::graph_rerank_lists(g, lists, n_lists, rows, row_to_node, n_rows, scores, B, k_dense, params, max_exp, o2,
                                 o3, o4, o5, o6, o7, o8, o9, stream);
  else if (!(skip & 4))
    st = ahr_graph_expand_rerank_rows(g, rows, row_to_node, n_rows, scores, B, k_dense, params, max_exp, o2, o3, o4,
                                      o5, o6, o7, o8, o9, stream);
  if (st != AHR_OK) return st;
  if (o == a && !(skip & 2)) AHR_HIP(hipMemcpyAsync(host_out, a, (size_t)arena, hipMemcpyDeviceToHost, s));
  AHR_HIP(hipStreamSynchronize(s));
  return AHR_OK;
}

}  // extern "C"
