// Launch interface of the query-resident dense top-k kernel (ahr_qres.hip), called by the search
// planner in ahr_dense.hip. Plain pointers and sizes; the kernel itself is described in ahr_qres.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ahr {
namespace dense {
namespace qres {

// The MFMA shape of the kernel's block product (AHR_QRES_MMA16, a build switch for A/B):
// 16x16x32 — per 32-deep step two 16-row corpus fragments, each read once from LDS and multiplied
//     by the wave's two 16-query tiles (the same LDS bytes and registers per FLOP), scores bitwise
//     those of topk_t256_kernel's k-ordered 16x16x32 chain;
// 32x32x16 (rounds 3-5) — scores bitwise those of topk_tilelane_kernel.
// AHR_QRES_MMA16 = 1 (default): 16x16x32 at d_pad 768, 32x32x16 at 384 (same box, round 6: C2
// 142.1 -> 137.4 us, C3 7.17 -> 6.83 ms, but d = 384 95.8 -> 100.8 us); 0: 32x32x16 everywhere;
// 2: 16x16x32 everywhere. The fragment-major query copy follows the form (frag_chunk / frag_elem).
#ifndef AHR_QRES_MMA16
#define AHR_QRES_MMA16 1
#endif
// ns = d_pad / 16 (48 at d_pad 768, 24 at 384)
__host__ __device__ constexpr bool mma16_for(int ns) { return AHR_QRES_MMA16 == 2 || (AHR_QRES_MMA16 == 1 && ns == 48); }

constexpr int kTQ = 256;     // queries per workgroup: 8 waves x 32
constexpr int kTR = 32;      // corpus rows per block
constexpr int kBufCap = 14;  // per-lane survivor buffer (keys) in LDS
constexpr int kPark = kBufCap - 8;  // self-seeding: block 0's raw scores wait in entries kPark .. kBufCap - 1

// Whether a launch seeds itself: every split has its first two blocks, the splits fit one wave's
// selection (<= 128), pair up in the landing zone (even), and are many enough for the k-th largest
// of their maxima to be a useful bound (>= 32 and >= 2k: at 16 splits, B = 4096, the self-seeded
// kernel measured 599 vs 493 us with the pre-pass; at 8 < k splits no seed exists at all).
// Otherwise the caller seeds it (the pre-pass) or it runs unseeded.
__host__ __device__ inline bool self_seeds(int64_t n_rows, int n_splits, int k) {
  return n_splits >= 32 && n_splits >= 2 * k && n_splits <= 128 && n_splits % 2 == 0 &&
         (n_rows + kTR - 1) / kTR >= 2 * (int64_t)n_splits;
}

// bf16 / f16 rows of d_pad_bytes = 1536 or 768 (d_pad = 768 or 384), k <= 12: what the kernel is built for.
bool supported(int dtype, int d_pad_bytes, int k);

// The fragment-major query copy the kernel reads, one contiguous KiB per wave B operand:
// [B/32][ns = d_pad/16 fragments][64 lanes][16 B]. 32x32x16: fragment S = k16 step S, lane l:
// query 32g + l%32, elements [16 S + 8 (l/32), +8). 16x16x32: fragment S = (k32 step S/2, query
// tile S%2), lane l: query 32g + 16 (S%2) + l%16, elements [32 (S/2) + 8 (l/16), +8). frag_chunk:
// the 16-B chunk holding element j of query q (j % 8 == 0 .. 7 inside it); frag_elem: the query and
// first element of chunk i. The buffer is padded to whole 256-query blocks.
__host__ __device__ inline int64_t frag_chunk(int64_t q, int j, int ns) {
  if (mma16_for(ns))
    return ((q >> 5) * ns + 2 * (j >> 5) + ((q >> 4) & 1)) * 64 + (q & 15) + 16 * ((j >> 3) & 3);
  return ((q >> 5) * ns + (j >> 4)) * 64 + (q & 31) + 32 * ((j >> 3) & 1);
}
__host__ __device__ inline void frag_elem(int64_t i, int ns, int64_t* q, int* j0) {
  const int l = (int)(i & 63);
  const int64_t gs = i >> 6;
  const int S = (int)(gs % ns);
  const int64_t g = gs / ns;
  if (mma16_for(ns)) {
    *q = g * 32 + 16 * (S & 1) + (l & 15);
    *j0 = 32 * (S >> 1) + 8 * (l >> 4);
  } else {
    *q = g * 32 + (l & 31);
    *j0 = 16 * S + 8 * (l >> 5);
  }
}

// Query rows [B][row_stride] (the convert kernel's storage rows) -> the fragment-major copy.
// epoch (optional): the self-seeding tag this launch advances (see launch).
void launch_frag(const uint8_t* qbuf, int64_t row_stride, int B, int d_pad_bytes, uint8_t* qfrag, uint32_t* epoch,
                 hipStream_t s);

// One fused launch: part_keys [B][n_splits][k] (the merge kernels' input), thr [B] optional
// admission seeds. grid = n_splits * qblocks; n_splits % 8 == 0 when flags has the XCD remap bit.
// pub: the self-seeding buffer, nullptr for none: pub[-9 .. -2] = the per-XCD row weights and
// duration sums (rebalance_xcds), pub[-1] = the launch's tag (low 32 bits), which
// the query conversion stream-ordered before this launch advanced (no earlier launch on these
// buffers used it); then [256 qblocks][n_splits] published maxima, then [256 qblocks] seeds.
// pub_mask / ev_mask: the self-seeding schedule over a split's block index (bit bi: publish the
// running maxima after block bi / a seeding event at the end of block bi; block 0's publication and
// the first event at block 1 are always there).
void launch(int dtype, int k, const uint8_t* rows, const uint8_t* qfrag, int64_t row_stride, int d_pad_bytes,
            int n_rows, int B, uint32_t row_base, uint64_t* part_keys, const float* thr, int n_splits, int qblocks,
            int flags, uint64_t* pub, uint64_t pub_mask, uint64_t ev_mask, hipStream_t s);

}  // namespace qres
}  // namespace dense
}  // namespace ahr
