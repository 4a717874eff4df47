// Device helpers shared by the dense-search translation units of libahr_hip.so (gfx950):
// fragment types, LDS swizzles, register top-k lists, DPP reductions, buffer LDS-DMA,
// MFMA steps and the ablation / plan flag bits.
#pragma once

#include "ahr_common.h"
#include "ahr.h"

namespace ahr {
namespace dense {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

enum { DT_F32 = AHR_F32, DT_F16 = AHR_F16, DT_BF16 = AHR_BF16 };

constexpr int kThreads = 256;
constexpr int kTileRows = 128;
constexpr int kTileQ = 128;
constexpr int kRowBytes = 128;  // one k-tile of one row: 8 chunks of 16 B
constexpr int kBufBytes = (kTileRows + kTileQ) * kRowBytes;  // 32 KiB: A tile, then B tile
constexpr int kProdCap = 8;  // candidate slots per (query, producer lane); 4 producers per query

// LDS map (bytes). The candidate lists overlay the two staging buffers: they are only live
// between the last k-tile of a corpus tile and the first k-tile of the next one.
constexpr int kOffBuf0 = 0;
constexpr int kOffBuf1 = kBufBytes;
constexpr int kOffCand = 0;
constexpr int kCandBytes = kTileQ * 4 * kProdCap * 8;   // 32 KiB
constexpr int kOffScratch = kOffCand + kCandBytes;         // 4 waves x 64 lanes x 32 floats
constexpr int kScratchBytes = 4 * 64 * 32 * 4;             // 32 KiB
constexpr int kOffThrKey = 2 * kBufBytes;
constexpr int kOffThrScore = kOffThrKey + kTileQ * 8;
constexpr int kOffCnt = kOffThrScore + kTileQ * 4;
constexpr int kOffFlag = kOffCnt + kTileQ * 4 * 4;
constexpr int kLdsBytes = kOffFlag + 16;
static_assert(kCandBytes + kScratchBytes <= 2 * kBufBytes, "epilogue overlay must fit the staging buffers");
static_assert(kLdsBytes % 16 == 0, "LDS carve must stay 16-B aligned");

// XOR swizzle of 16-B chunks inside a 128-B row: a ds_read_b128 lane group (rows
// {0-3,12-15,20-27} or {4-11,16-19,28-31} of a 32-row fragment, same chunk) then covers all
// 16 slots of a 256-B bank row (conflict-free).
__device__ __forceinline__ int swz(int row, int chunk) {
  return row * kRowBytes + ((chunk ^ ((row >> 1) & 7)) << 4);
}
// 64-B rows (half k-tiles): a 256-B bank row holds 4 rows; XOR the chunk with bits 2-3 of the
// row so the 16 rows of a ds_read_b128 lane group hit 16 distinct 16-B slots.
__device__ __forceinline__ int swz64(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4); }

// Sorted (descending) register list of packed keys; drops the smallest on insert.
template <int KCAP>
__device__ __forceinline__ void list_insert(uint64_t (&L)[KCAP], uint64_t key) {
  if (key <= L[KCAP - 1]) return;
#pragma unroll
  for (int j = KCAP - 1; j > 0; --j) {
    const uint64_t prev = L[j - 1];
    L[j] = (prev < key) ? prev : ((L[j] < key) ? key : L[j]);
  }
  L[0] = (L[0] < key) ? key : L[0];
}

// Wave64 max of packed keys with DPP row shifts + row broadcasts (gfx9 family): no LDS
// round trips, unlike __shfl_xor (ds_bpermute). Returns the max in every lane.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t x) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, CTRL, ROW_MASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), CTRL, ROW_MASK, 0xf, false);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

__device__ __forceinline__ uint64_t max_u64(uint64_t a, uint64_t b) { return a > b ? a : b; }

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t x) {
  x = max_u64(x, dpp_u64<0x111, 0xf>(x));  // row_shr:1
  x = max_u64(x, dpp_u64<0x112, 0xf>(x));  // row_shr:2
  x = max_u64(x, dpp_u64<0x114, 0xf>(x));  // row_shr:4
  x = max_u64(x, dpp_u64<0x118, 0xf>(x));  // row_shr:8  -> lane 15 of each row: row max
  x = max_u64(x, dpp_u64<0x142, 0xa>(x));  // row_bcast:15 -> lane 31, 63: max of row pairs
  x = max_u64(x, dpp_u64<0x143, 0xc>(x));  // row_bcast:31 -> lane 63: wave max
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), 63);
  return ((uint64_t)hi << 32) | lo;
}

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROW_MASK, 0xf, false);
}
// wave64 max of u32 values (the DPP sequence of wave_max_u64), in every lane
__device__ __forceinline__ uint32_t dpp_max_u32(uint32_t x) {
  x = max(x, dpp_u32<0x111, 0xf>(x));  // row_shr:1
  x = max(x, dpp_u32<0x112, 0xf>(x));  // row_shr:2
  x = max(x, dpp_u32<0x114, 0xf>(x));  // row_shr:4
  x = max(x, dpp_u32<0x118, 0xf>(x));  // row_shr:8
  x = max(x, dpp_u32<0x142, 0xa>(x));  // row_bcast:15
  x = max(x, dpp_u32<0x143, 0xc>(x));  // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

__device__ __forceinline__ uint64_t readlane_u64(uint64_t x, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  const uint32_t lo = __shfl_xor((uint32_t)v, m, 64);
  const uint32_t hi = __shfl_xor((uint32_t)(v >> 32), m, 64);
  return ((uint64_t)hi << 32) | lo;
}

// LDS-DMA through a buffer descriptor (MUBUF `buffer_load ... lds`). Unlike the FLAT-encoded
// global_load_lds, LLVM does not count it as a possibly out-of-order LDS access, so the
// fragment reads that follow keep counted lgkmcnt(N) waits. The descriptor covers one tile
// (32-bit offsets, whatever the corpus size) and must be built from wave-uniform values.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

// tile_rsrc from a base the compiler cannot prove uniform (it then wraps every load in a
// readfirstlane waterfall loop): the halves are made uniform explicitly (callers guarantee it)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc_u(const void* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
  const uint32_t n = (uint32_t)__builtin_amdgcn_readfirstlane((int)bytes);
  return tile_rsrc(reinterpret_cast<const void*>(((uint64_t)hi << 32) | lo), n);
}

__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, uint32_t voff, void* lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff, 0,
                                           0, 0);
}

// with a cache policy: sc1 (16) reads past the CU's L1 (what another CU wrote with sc1 stores)
__device__ __forceinline__ void blds16_pol(__amdgpu_buffer_rsrc_t r, uint32_t voff, void* lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff, 0, 0,
                                           16);
}

// the same with a wave-uniform byte offset added to the global address only, through soffset (an
// SGPR; the instruction's immediate offset would also shift the LDS destination)
__device__ __forceinline__ void blds16_soff(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, void* lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff, soff, 0,
                                           0);
}

// The register-resident plan's self-seeding tag: the query conversion before each launch advances
// it on the device (one thread), so every launch — a replayed hipGraph's too — gets its own; 0 is
// never used (zeroed granule buffers hold tag 0).
__device__ __forceinline__ void advance_epoch(uint32_t* e) {
  const uint32_t v = *e + 1u;
  *e = v ? v : 1u;
}

// Per-XCD row weights of the register-resident plan (XCD-balanced splits): the XCDs of one device
// hold different clocks under this load (measured 1.93-2.01 GHz within one launch), so each launch's
// splits get rows in proportion to the speed its XCD showed in the previous launch. w[0..7]: weights
// (1024 = 1.0, 0 = not yet measured), w[8..15]: the previous launch's summed workgroup durations per
// XCD (s_memrealtime ticks). Updated by the one thread that advances the launch tag, before the launch.
constexpr uint32_t kXcdW = 1024, kXcdWMin = 820, kXcdWMax = 1280;
__device__ __forceinline__ void rebalance_xcds(uint32_t* w) {
  uint32_t* t = w + 8;
  bool all = true;
  float mean = 0.f;
#pragma unroll
  for (int x = 0; x < 8; ++x) {
    all = all && t[x] != 0u;
    mean += (float)t[x] * 0.125f;
  }
  if (all) {  // new weight ~ old weight x (mean duration / own duration), renormalised to 1024 on average
    float v[8], sum = 0.f;
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      v[x] = (float)(w[x] ? w[x] : kXcdW) * mean / (float)t[x];
      sum += v[x];
    }
#pragma unroll
    for (int x = 0; x < 8; ++x)
      w[x] = (uint32_t)fminf(fmaxf(v[x] * (8.f * kXcdW) / sum, (float)kXcdWMin), (float)kXcdWMax);
  }
#pragma unroll
  for (int x = 0; x < 8; ++x) t[x] = 0u;
}
// the tag advance of a register-resident launch; its weights sit 8 u64 before the tag
__device__ __forceinline__ void advance_epoch_rebalance(uint32_t* e) {
  advance_epoch(e);
  rebalance_xcds(reinterpret_cast<uint32_t*>(reinterpret_cast<uint64_t*>(e) - 8));
}

// Workgroup barrier that waits for this wave's LDS traffic but leaves global_load_lds in flight
// (__syncthreads() would emit vmcnt(0) and drain the ring).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int DT>
__device__ __forceinline__ void mfma_step(const u32x4& a, const u32x4& b, f32x16& acc) {
  if constexpr (DT == DT_BF16) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                  __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
  } else if constexpr (DT == DT_F16) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                 __builtin_bit_cast(f16x8, b), acc, 0, 0, 0);
  } else {
    // fp32: the chunk holds k = 8g + 2m + h for m = 0..3 (storage permutation), so four
    // k-ordered 32x32x2 steps extend one fma chain in increasing k (exact-mode contract).
    const f32x4 af = __builtin_bit_cast(f32x4, a);
    const f32x4 bf = __builtin_bit_cast(f32x4, b);
#pragma unroll
    for (int m = 0; m < 4; ++m) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af[m], bf[m], acc, 0, 0, 0);
  }
}

// one v_mfma_f32_16x16x32 (bf16 / f16) step: acc + a . b (the t256 / small kernels' fragment map)
template <int DT>
__device__ __forceinline__ f32x4 mfma16_step(const u32x4& a, const u32x4& b, const f32x4& acc) {
  if constexpr (DT == DT_BF16)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc,
                                                   0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), acc,
                                                  0, 0, 0);
}

// Runtime-indexed read of a register list without scratch: a select chain. The opaque copy
// of j stops LLVM from folding the chain back into an indexed load (which would demote the
// whole list to scratch memory).
template <int KCAP>
__device__ __forceinline__ uint64_t list_at(const uint64_t (&L)[KCAP], int idx) {
  uint64_t v = L[0];
#pragma unroll
  for (int j = 1; j < KCAP; ++j) {
    int jj = j;
    asm volatile("" : "+s"(jj));
    v = (jj == idx) ? L[j] : v;
  }
  return v;
}

enum { MODE_TOPK = 0, MODE_GROUPMAX = 1, MODE_SCORES = 2 };
// Plan / ablation flag bits: a uint32_t word (ahr_index_set_debug_flags).
enum : uint32_t {
  kFlagXcdRemap = 1,
  kFlagSkipEpilogue = 2,  // GEMM only: the top-k epilogue is skipped (wrong results)
  kFlagQresMute = 4,      // qres self-seeding: split 0's seeding traffic carries another launch's tag, so every
                          // bounded wait on it times out (a test of the timeout path; results unchanged)
  kFlagTile128 = 8,       // the 128x128 tile kernel with cooperative screening, any k
  kFlagTileLane = 32,     // the 128x128 lane-local kernel at any batch (k <= 16)
  kFlagMaxOnly = 256,     // lane kernel: group maxima only, no scan (wrong results)
  kFlagNoLoads = 512,     // tile kernel: operands loaded for the first tile only (wrong results)
  kFlagNoWait = 1024,     // tilelane kernel: loads issued but never waited for (wrong results)
  kFlagNoQres = 2048,     // plan without the query-resident kernels (qkv and qres)
  kFlagQkv = 4096,        // the 128-query-resident kernel wherever it applies (ablation build only)
  kFlagNoTilePrefetch = 16384,  // tilelane: each tile's k-tile 0 issued at the tile start (ablation)
  kFlagT256 = 32768,      // the 256x256 16x16x32 kernel wherever it applies (bf16/f16, k <= 16)
  kFlagKB256 = 131072,    // the k-blocked 256x256 kernel wherever it applies (bf16/f16, k <= 16)
  kFlagNoKB256 = 262144,  // plan without the k-blocked kernel
  kFlagTileZero = 1u << 20,   // k-blocked kernel: every tile's operands read from tile 0 (L2-resident; wrong results)
  kFlagTileFirst = 1u << 21,  // k-blocked kernel: every tile read from the split's first tile (wrong results)
  kFlagNoFold = 1u << 22,     // small kernels: merge launch (the default since round 5; kept accepted)
  kFlagFold = 8192,           // small kernels: the last-workgroup fold instead of the merge launch (A/B)
  kFlagQres = 1u << 23,       // the 256-query register-resident kernel wherever it applies (bf16/f16, d 384/768, k <= 12)
  kFlagNoBarrier = 1u << 24,  // qres kernel: no stage barriers (wrong results)
  kFlagNoLdsRead = 1u << 25,  // qres kernel: MFMAs on a register fragment, no LDS reads (wrong results)
  kFlagQresPrepass = 1u << 26,   // qres kernel seeded by the sampled pre-pass launch, not by itself (A/B)
  kFlagQresSeedOnce = 1u << 27,  // qres self-seeding: the first event only, no later rounds (A/B)
  kFlagXcdBalance = 1u << 28,    // qres: XCD-balanced splits at any corpus size (default from 256 row blocks per split)
  kFlagNoXcdBalance = 1u << 19,  // qres: equal splits at any corpus size (A/B)
  kFlagQresTrace = 1u << 29,  // qres kernel: per-workgroup timestamps into AHR_QRES_TRACE_PTR (ablation build)
  kFlagQresEvNoSel = 1u << 30,   // qres seeding events without the selection (wrong seeds: ablation build)
  kFlagQresEvNoIssue = 1u << 31, // qres seeding events without the landing reads (ablation build)
  // internal (set by the library on a launch, never accepted from a caller): the qres kernel ends
  // each (query, split) list at its first empty slot, for the lane-list merge, which stops there
  kFlagShortLists = 65536,
};
#ifdef AHR_ABLATION
constexpr bool kAblation = true;  // the profiling build: cost-split switches compiled in
#else
constexpr bool kAblation = false;
#endif
constexpr uint32_t kKernelFlags =
    kFlagTile128 | kFlagTileLane | kFlagNoQres | kFlagQkv | kFlagT256 | kFlagKB256 | kFlagNoKB256 | kFlagQres;
// the flags that request a kernel (the kFlagNo* ones only take one out of the plan)
constexpr uint32_t kForceFlags = kKernelFlags & ~(kFlagNoQres | kFlagNoKB256);
// every flag ahr_index_set_debug_flags accepts; those that give wrong results need the ablation build
constexpr uint32_t kWrongResultFlags = kFlagSkipEpilogue | kFlagMaxOnly | kFlagNoLoads | kFlagNoWait | kFlagTileZero |
                                       kFlagTileFirst | kFlagNoBarrier | kFlagNoLdsRead | kFlagQresTrace |
                                       kFlagQresEvNoSel | kFlagQresEvNoIssue;
// (the 128-query-resident kernel, kFlagQkv, is compiled into the ablation build only)
constexpr uint32_t kKnownFlags = (kKernelFlags & (kAblation ? ~0u : ~(uint32_t)kFlagQkv)) | kWrongResultFlags |
                                 kFlagNoTilePrefetch | kFlagNoFold | kFlagFold | kFlagQresPrepass | kFlagQresSeedOnce |
                                 kFlagXcdBalance | kFlagNoXcdBalance | kFlagQresMute;
// every flag but kFlagXcdRemap is an ablation switch (ahr_index_set_debug_flags)

// One wave merges n_lists (<= 512) sorted lists of k_in keys held in LDS: k rounds of a DPP wave
// max over the list heads (lane l owns lists l + 64 u), a head advancing by an LDS read, no
// barrier per output; output j goes to o0 + j (merge_block_kernel, the small kernels' fold and
// the drop-in search's fused rerank, ahr_graph.hip).
// Returns, for k <= 64, output j in lane j (0 past k).
__device__ __forceinline__ uint64_t walk_lists_lds(const uint64_t* kb, int n_lists, int k_in, int k, int64_t o0,
                                                   float* __restrict__ scores, int32_t* __restrict__ rows,
                                                   uint64_t* __restrict__ keys_out) {
  const int lane = threadIdx.x & 63;
  constexpr int kH = 8;  // n_lists <= 512
  int ptr[kH];
  uint64_t head[kH];
#pragma unroll
  for (int u = 0; u < kH; ++u) {
    const int l = lane + 64 * u;
    ptr[u] = 0;
    head[u] = (l < n_lists && k_in > 0) ? kb[l * k_in] : 0;
  }
  uint64_t mine = 0;  // lane j % 64 keeps the j-th winner; flushed in windows of 64 outputs
  for (int j = 0; j < k; ++j) {
    uint64_t m = head[0];
#pragma unroll
    for (int u = 1; u < kH; ++u) m = max_u64(m, head[u]);
    const uint64_t best = wave_max_u64(m);
    if (best != 0 && m == best) {
#pragma unroll
      for (int u = 0; u < kH; ++u) {
        if (head[u] == best) {
          const int l = lane + 64 * u;
          ++ptr[u];
          head[u] = ptr[u] < k_in ? kb[l * k_in + ptr[u]] : 0;
        }
      }
    }
    if (lane == (j & 63)) mine = best;
    if ((j & 63) == 63 || j == k - 1) {
      const int j0 = j & ~63;
      if (j0 + lane <= j) {
        const int64_t o = o0 + j0 + lane;
        if (scores) scores[o] = mine ? key_score(mine) : -INFINITY;
        if (rows) rows[o] = mine ? (int32_t)key_row(mine) : -1;
        if (keys_out) keys_out[o] = mine;
      }
    }
  }
  return k <= 64 ? mine : 0;
}

}  // namespace dense
}  // namespace ahr
