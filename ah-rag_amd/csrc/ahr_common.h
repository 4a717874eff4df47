// Shared host/device helpers for libahr_hip.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <atomic>
#include <string>

namespace ahr {

// Thread-local error channel behind ahr_last_error().
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

#define AHR_HIP(call)                                   \
  do {                                                  \
    hipError_t e_ = (call);                             \
    if (e_ != hipSuccess) return ::ahr::hip_fail(e_, #call); \
  } while (0)

// Opt a kernel into more than 64 KiB of dynamic LDS on the CURRENT device. The attribute is per
// (function, device), so `done` keeps one bit per device; the atomic makes concurrent first
// launches from several host threads safe (a duplicate set is harmless).
inline void ensure_lds_attr(std::atomic<uint64_t>& done, const void* fn, int bytes) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  const uint64_t bit = 1ull << (dev & 63);
  if (done.load(std::memory_order_acquire) & bit) return;
  // a refused opt-in must not surface as the next call's hipGetLastError(): a launch that needs
  // more LDS than the default then fails on its own and reports that
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess) (void)hipGetLastError();
  done.fetch_or(bit, std::memory_order_acq_rel);
}

// ---- packed sort keys --------------------------------------------------------------------
// key = ord(score) << 32 | (0xFFFFFFFF - row): a larger key is a better hit, i.e. the order
// (score desc, row asc) that SURVEY §7 fixes as the tie rule. Key 0 = empty slot.
__host__ __device__ __forceinline__ uint32_t ord_f32(float f) {
  uint32_t u;
#ifdef __HIP_DEVICE_COMPILE__
  u = __float_as_uint(f);
#else
  __builtin_memcpy(&u, &f, 4);
#endif
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__host__ __device__ __forceinline__ float unord_f32(uint32_t o) {
  uint32_t u = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
  float f;
#ifdef __HIP_DEVICE_COMPILE__
  f = __uint_as_float(u);
#else
  __builtin_memcpy(&f, &u, 4);
#endif
  return f;
}

__host__ __device__ __forceinline__ uint64_t make_key(float s, uint32_t row) {
  return ((uint64_t)ord_f32(s) << 32) | (uint64_t)(0xFFFFFFFFu - row);
}

__host__ __device__ __forceinline__ uint32_t key_row(uint64_t key) {
  return 0xFFFFFFFFu - (uint32_t)key;
}

__host__ __device__ __forceinline__ float key_score(uint64_t key) {
  return unord_f32((uint32_t)(key >> 32));
}

// The drop-in search's one-call path (ahr_search_host): the rerank wave kernel merges the dense
// stage's per-(query, split) lists itself while a query's lists hold at most this many keys
// (ahr_graph.hip expand_rerank_wave_kernel<true>; 256 splits x top_k 5 = 1,280 for search()).
constexpr int kRerankFuseKeys = 2048;

}  // namespace ahr
