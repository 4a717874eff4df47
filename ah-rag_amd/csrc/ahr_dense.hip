// ahr_dense.hip — fused query x corpus inner product + exact top-k for gfx950 (MI355X).
//
// Replaces the ChromaDB collection behind HierarchicalGraph.search / build_vector_index
// (reference src/ah_rag/graph/hierarchical_graph.py:605-611 create, :660 upsert, :714 query).
// Chroma answers with an approximate HNSW walk; this kernel answers the exact question
// (what Chroma returns when its HNSW is exhaustive), batched over B queries.
//
// Data layout in HBM (owned by ahr_index):
//   corpus  [cap_pad][d_pad] row-major, dtype bf16 | f16 | f32, cap_pad % 256 == 0,
//           rows 16-B aligned, zero padding dim..d_pad. fp32 rows are stored with each group
//           of 8 lanes permuted to (evens | odds) so one 16-B LDS read feeds four consecutive
//           v_mfma_f32_32x32x2_f32 k-steps (see frag_f32 below).
//   queries [q_cap][d_pad] same format, converted from fp32 on every call.
//   partial keys [B][n_splits][k] uint64 (ahr_common.h key format), merged by merge_kernel.
//
// Kernels (both keep the score tile in MFMA accumulators, never in memory; corpus rows are the
// A operand and queries the B operand of 32x32 MFMAs, so each lane's accumulator column is ONE
// query and its registers are corpus rows of it):
//  * topk_lane_kernel (B >= 6144, k <= 16): a workgroup of 8 waves owns a 256-query
//    block and a contiguous range of 256-row corpus tiles; each wave covers all 256 rows for its
//    32 queries, so every lane keeps its query's partial top-k list in registers and screens its
//    own scores (16-row group maxima against its threshold, scan of the rare passing groups):
//    no candidate buffers, atomics or barriers in the epilogue. Operands stream through a
//    4-stage buffer LDS-DMA ring. The two half-wave lists merge at the end.
//  * topk_tile_kernel (default up to B < 6144, every k, and the threshold pre-pass): 4 waves
//    (2 along rows x 2 along queries), 128-query block x 128-row tiles, two workgroups per CU.
//    k <= 16: the same lane-local epilogue (each lane holds two query columns, so two lists;
//    the 4 partial lists of a query merge at the end). k > 16: survivors are screened
//    cooperatively into per-query LDS candidate lists that one owner thread per query folds.
// The pre-pass (first 8192 rows, 16-row group maxima, k-th largest per query) seeds every
// query's threshold with a valid lower bound of its final k-th best score.
#include "ahr_common.h"
#include "ahr.h"
#include "ahr_dense_common.h"
#include "ahr_qres.h"
#include "ahr_internal.h"

#include <algorithm>
#include <cstring>
#include <type_traits>
#include <math.h>
#include <vector>

namespace ahr {
namespace dense {


// MODE_TOPK : per-(query, split) top-k lists into part_keys [n_q][n_splits][k_out].
//             thr_init (optional, [n_q]) seeds each query's threshold with a score that is a
//             valid lower bound of its final k-th best (from the sampled pre-pass).
// MODE_GROUPMAX: 16-row group maxima of the scores into score_out [n_q][score_ld] (pre-pass).
// MODE_SCORES  : every score into score_out [n_q][score_ld], row-indexed (top-k beyond the
//                register lists, k > AHR_MAX_K: radix_topk_kernel selects from them).
template <int DT, int KCAP, int MODE>
__global__ __launch_bounds__(kThreads, 2) void topk_tile_kernel(
    const uint8_t* __restrict__ corpus, const uint8_t* __restrict__ queries, int64_t row_stride,
    int n_rows, int n_q, int n_ktiles, int tiles_per_split, int n_row_tiles, uint32_t row_base,
    int k_out, uint64_t* __restrict__ part_keys, const float* __restrict__ thr_init,
    float* __restrict__ score_out, int64_t score_ld, int n_splits, int qblocks, int flags) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 1;  // wave's 64-row half of the tile
  const int wq = wave & 1;   // wave's 64-query half of the block
  const int fr = lane & 31;
  const int fh = lane >> 5;
  // 1-D grid. With kFlagXcdRemap, the qblocks workgroups that stream the same corpus rows
  // (one split) get ids that are equal mod 8 and adjacent in dispatch order: the dispatcher
  // deals ids round-robin over the 8 XCDs, so they share one L2 and read each corpus tile from
  // HBM once (placement is a speed hint only; any placement gives the same result).
  int split, qb;
  if (flags & kFlagXcdRemap) {
    const int x = blockIdx.x & 7;
    const int i = blockIdx.x >> 3;
    split = (i / qblocks) * 8 + x;
    qb = i % qblocks;
  } else {
    split = blockIdx.x % n_splits;
    qb = blockIdx.x / n_splits;
  }
  const int q0 = qb * kTileQ;
  // contiguous, balanced tile ranges (sizes differ by at most one tile)
  const int t_begin = (int)((int64_t)split * n_row_tiles / n_splits);
  const int t_end = (int)((int64_t)(split + 1) * n_row_tiles / n_splits);
  (void)tiles_per_split;

  uint64_t* thr_key = reinterpret_cast<uint64_t*>(smem + kOffThrKey);
  float* thr_score = reinterpret_cast<float*>(smem + kOffThrScore);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(smem + kOffCnt);
  int* flag = reinterpret_cast<int*>(smem + kOffFlag);
  uint64_t* cand = reinterpret_cast<uint64_t*>(smem + kOffCand);

  // Cooperative screening into per-query LDS candidate lists folded by one owner thread per
  // query (k > 16; k <= 16 has the lane-local topk_tilelane_kernel).
  uint64_t L[KCAP];
#pragma unroll
  for (int j = 0; j < KCAP; ++j) L[j] = 0;
  if (tid < kTileQ) {
    // A row whose score equals the seed may still win on the row tie-break: the seed key is
    // the smallest key with that score, minus one.
    const float seed = (thr_init && q0 + tid < n_q) ? thr_init[q0 + tid] : -INFINITY;
    thr_score[tid] = seed;
    thr_key[tid] = seed == -INFINITY ? 0 : (((uint64_t)ord_f32(seed) << 32) - 1);
  }
  if (tid < 2) flag[tid] = 0;

  // Staging by global_load_lds (no staging registers): wave w fills rows [32w, 32w+32) of both
  // tiles, 8 rows (1 KiB) per instruction; lane l lands at (row 8j + l/8, physical chunk l%8) and
  // therefore loads logical chunk (l%8) ^ swz(row): the XOR swizzle moves to the source address.
  const int ld_row = lane >> 3;
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  int round_id = 0;
  const uint32_t tile_bytes = (uint32_t)(kTileRows * row_stride);
  const __amdgpu_buffer_rsrc_t q_rsrc = tile_rsrc(queries + (int64_t)q0 * row_stride, tile_bytes);
  uint32_t ld_off[4];  // this lane's byte offset inside a tile, k-tile 0
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = wave_u * 32 + 8 * j + ld_row;
    ld_off[j] = (uint32_t)(row * row_stride) + (((lane & 7) ^ ((row >> 1) & 7)) << 4);
  }

  for (int t = t_begin; t < t_end; ++t) {
    const int64_t r0 = (int64_t)t * kTileRows;
    const __amdgpu_buffer_rsrc_t c_rsrc = tile_rsrc(corpus + r0 * row_stride, tile_bytes);
    auto stage = [&](int kt, unsigned char* buf) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t off = ld_off[j] + kt * kRowBytes;
        blds16(c_rsrc, off, buf + (wave_u * 32 + 8 * j) * kRowBytes);
        blds16(q_rsrc, off, buf + kTileRows * kRowBytes + (wave_u * 32 + 8 * j) * kRowBytes);
      }
    };
    const bool load = !(flags & kFlagNoLoads) || t == t_begin;  // ablation: LDS + MFMA ceiling
    if (load) stage(0, smem + kOffBuf0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();

    f32x16 acc[2][2];
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int bj = 0; bj < 2; ++bj)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[bi][bj][r] = 0.f;

    for (int kt = 0; kt < n_ktiles; ++kt) {
      if (kt + 1 < n_ktiles && load) stage(kt + 1, smem + (((kt + 1) & 1) ? kOffBuf1 : kOffBuf0));
      const unsigned char* buf = smem + ((kt & 1) ? kOffBuf1 : kOffBuf0);
      // Two fragment register sets, order pinned with sched_barrier: the LDS reads of step g+1
      // are in flight while the MFMAs of step g run.
      u32x4 fa0[2], fb0[2], fa1[2], fb1[2];
      auto frag_load = [&](int g, u32x4 (&a)[2], u32x4 (&b)[2]) {
        const int ch = 2 * g + fh;
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
          a[bi] = *reinterpret_cast<const u32x4*>(buf + swz(wr * 64 + bi * 32 + fr, ch));
#pragma unroll
        for (int bj = 0; bj < 2; ++bj)
          b[bj] = *reinterpret_cast<const u32x4*>(buf + kTileRows * kRowBytes + swz(wq * 64 + bj * 32 + fr, ch));
      };
      auto frag_mma = [&](const u32x4 (&a)[2], const u32x4 (&b)[2]) {
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
          for (int bj = 0; bj < 2; ++bj) mfma_step<DT>(a[bi], b[bj], acc[bi][bj]);
      };
      frag_load(0, fa0, fb0);
      frag_load(1, fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
      frag_mma(fa0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      frag_load(2, fa0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      frag_mma(fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
      frag_load(3, fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
      frag_mma(fa0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      frag_mma(fa1, fb1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stage kt+1 landed (this wave's part)
      lds_barrier();                                    // ... everyone's; everyone done with kt
    }

    if constexpr (MODE == MODE_SCORES) {
      // lane: query column fr of block bj, rows 4 fh + (r & 3) + 8 (r >> 2) of block bi
#pragma unroll
      for (int bj = 0; bj < 2; ++bj) {
        const int q = q0 + wq * 64 + bj * 32 + fr;
        if (q >= n_q) continue;
        float* dst = score_out + (int64_t)q * score_ld;
#pragma unroll
        for (int bi = 0; bi < 2; ++bi) {
          const int rb = r0 + wr * 64 + bi * 32 + 4 * fh;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = rb + (r & 3) + 8 * (r >> 2);
            if (row < n_rows) dst[row] = acc[bi][bj][r];
          }
        }
      }
      __syncthreads();
      continue;
    }
    if constexpr (MODE == MODE_GROUPMAX) {
      // Threshold pre-pass: per query, the max of each 16-row group (one lane's 16 registers of
      // one 32x32 block). The k-th largest group max is a valid lower bound of the k-th best
      // score: each group max is a distinct corpus row.
#pragma unroll
      for (int bj = 0; bj < 2; ++bj) {
        const int q = q0 + wq * 64 + bj * 32 + fr;
#pragma unroll
        for (int bi = 0; bi < 2; ++bi) {
          float gm = acc[bi][bj][0];
#pragma unroll
          for (int r = 1; r < 16; ++r) gm = fmaxf(gm, acc[bi][bj][r]);
          const int64_t g = (int64_t)t * 8 + wr * 4 + bi * 2 + fh;
          if (q < n_q) score_out[(int64_t)q * score_ld + g] = gm;
        }
      }
      __syncthreads();
      continue;
    }

    if (flags & kFlagSkipEpilogue) {  // ablation: GEMM only, keep acc live, no top-k
      float sink = 0.f;
#pragma unroll
      for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj)
#pragma unroll
          for (int r = 0; r < 16; ++r) sink += acc[bi][bj][r];
      if (sink == 1234.5678f) part_keys[0] = 1;
      continue;
    }

    // ---- epilogue: threshold filter -> LDS candidates -> owner merge (repeat on overflow).
    // Each query's 128 tile scores sit in 4 producer lanes (2 row-waves x 2 lane halves) as 32
    // registers each. A lane whose 32-score max beats its query's threshold is "flagged" and
    // spills its 32 scores to a per-wave LDS scratch; the whole wave then screens two flagged
    // lanes per pass (one score per lane), compacts survivors with a ballot and appends them to
    // the flagged lane's private kProdCap-slot buffer. No per-element branches, no atomics.
    uint64_t consumed = 0;  // bit (bj * 32 + v): score v of column bj already handed over
    const int pid = wr * 2 + fh;
    float* scr = reinterpret_cast<float*>(smem + kOffScratch) + wave * 64 * 32;
    for (;;) {
      ++round_id;
#pragma unroll
      for (int bj = 0; bj < 2; ++bj) {
        const int ql = wq * 64 + bj * 32 + fr;
        const float ths = (q0 + ql < n_q) ? thr_score[ql] : INFINITY;
        const uint64_t thk = thr_key[ql];
        float m = acc[0][bj][0];
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
#pragma unroll
          for (int r = 0; r < 16; ++r) m = fmaxf(m, acc[bi][bj][r]);
        int c = 0;  // this lane's fill of its producer buffer for column bj, this round
        uint64_t flagged = __ballot(m >= ths);
        if (flagged) {
          if (m >= ths) {
#pragma unroll
            for (int bi = 0; bi < 2; ++bi)
#pragma unroll
              for (int c4 = 0; c4 < 4; ++c4) {
                f32x4 v4 = {acc[bi][bj][4 * c4], acc[bi][bj][4 * c4 + 1], acc[bi][bj][4 * c4 + 2],
                            acc[bi][bj][4 * c4 + 3]};
                *reinterpret_cast<f32x4*>(scr + lane * 32 + bi * 16 + 4 * c4) = v4;
              }
          }
          __builtin_amdgcn_wave_barrier();
          const uint32_t cons_bj = (uint32_t)(consumed >> (bj * 32));
          const float ths_b = ths;
          const uint32_t thk_lo = (uint32_t)thk, thk_hi = (uint32_t)(thk >> 32);
          const int v = lane & 31;
          const int row_v = (v >> 4) * 32 + (v & 3) + 8 * ((v >> 2) & 3);
          while (flagged) {
            const int fA = __builtin_ctzll(flagged);
            flagged &= flagged - 1;
            const int fB = flagged ? __builtin_ctzll(flagged) : fA;
            const bool hasB = flagged != 0;
            if (hasB) flagged &= flagged - 1;
            const bool upper = lane >= 32;
            const bool active = !upper || hasB;
            const int f = upper ? fB : fA;
            // the flagged lanes' own state, broadcast through scalar reads
            const float tsA = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ths_b), fA));
            const float tsB = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ths_b), fB));
            const uint64_t tkA = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)thk_hi, fA) << 32) |
                                 (uint32_t)__builtin_amdgcn_readlane((int)thk_lo, fA);
            const uint64_t tkB = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)thk_hi, fB) << 32) |
                                 (uint32_t)__builtin_amdgcn_readlane((int)thk_lo, fB);
            const uint32_t csA = (uint32_t)__builtin_amdgcn_readlane((int)cons_bj, fA);
            const uint32_t csB = (uint32_t)__builtin_amdgcn_readlane((int)cons_bj, fB);
            const int cA = __builtin_amdgcn_readlane(c, fA);
            const int cB = __builtin_amdgcn_readlane(c, fB);
            const float ts = upper ? tsB : tsA;
            const uint64_t tk = upper ? tkB : tkA;
            const uint32_t cs = upper ? csB : csA;
            const int cf = upper ? cB : cA;
            const float val = scr[f * 32 + v];
            const int row = (int)r0 + wr * 64 + 4 * (f >> 5) + row_v;
            bool pass = active && val >= ts && !((cs >> v) & 1u) && row < n_rows;
            uint64_t key = 0;
            if (pass) {
              key = make_key(val, row_base + (uint32_t)row);
              pass = key > tk;
            }
            const uint64_t bal = __ballot(pass);
            const uint32_t half = upper ? (uint32_t)(bal >> 32) : (uint32_t)bal;
            const int rank = __builtin_popcount(half & ((1u << v) - 1u));
            const int total = __builtin_popcount(half);
            const bool store = pass && cf + rank < kProdCap;
            if (store) {
              const int qf = wq * 64 + bj * 32 + (f & 31);
              const int pf = wr * 2 + (f >> 5);
              cand[(qf * 4 + pf) * kProdCap + cf + rank] = key;
            }
            const uint64_t sbal = __ballot(store);
            const int totA = __builtin_popcount((uint32_t)bal);
            const int totB = __builtin_popcount((uint32_t)(bal >> 32));
            if (cA + totA > kProdCap || (hasB && cB + totB > kProdCap)) flag[round_id & 1] = round_id;
            (void)total;
            if (lane == fA) {
              c = min(cA + totA, kProdCap);
              consumed |= (uint64_t)(uint32_t)sbal << (bj * 32);
            }
            if (hasB && lane == fB) {
              c = min(cB + totB, kProdCap);
              consumed |= (uint64_t)(uint32_t)(sbal >> 32) << (bj * 32);
            }
          }
        }
        cnt[ql * 4 + pid] = c;
      }
      __syncthreads();
      if (tid < kTileQ) {
        bool changed = false;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int n = cnt[tid * 4 + u];
          const uint64_t* src = cand + (tid * 4 + u) * kProdCap;
          for (int i = 0; i < n; ++i) list_insert<KCAP>(L, src[i]);
          changed |= n > 0;
        }
        if (changed) {
          const uint64_t kth = list_at<KCAP>(L, k_out - 1);
          if (kth > thr_key[tid]) {
            thr_key[tid] = kth;
            thr_score[tid] = key_score(kth);
          }
        }
      }
      __syncthreads();
      // Parity slots: a round-R overflow write can never race a slower thread's read of the
      // round R-1 decision (those read the other slot).
      if (flag[round_id & 1] != round_id) break;
    }
  }

  if (MODE == MODE_TOPK && tid < kTileQ && q0 + tid < n_q) {
    uint64_t* dst = part_keys + ((int64_t)(q0 + tid) * n_splits + split) * k_out;
#pragma unroll
    for (int j = 0; j < KCAP; ++j)
      if (j < k_out) dst[j] = L[j];
  }
}

// =============================================================================================
// topk_tilelane_kernel (default for B < 6144, k <= 16): the 128x128 tile, 2x2 waves and K-loop
// of topk_tile_kernel with a lane-local top-k. Each lane holds two query columns x 32 rows of a
// tile; it keeps one sorted register list and one threshold per column (the pre-pass seed, then
// the list's k-th key). At a tile's end: 16-row group maxima against the thresholds; lanes with
// a passing group stage it into a private 64-B LDS slot (the second staging buffer is idle
// there) and insert its passing scores, one list_insert per set bit of a pass mask in a
// divergent loop. No candidate buffers, atomics or barriers; the other workgroup on the CU keeps
// the MFMA pipe busy meanwhile. At the end the 4 partial lists of a query (2 row-waves x 2 lane
// halves) merge through LDS.
// (Measured and dropped: deferring the screening into the next tile's K-steps, with one
// pending group or a second accumulator set, cost more in the K-loop than it hid.)
// =============================================================================================
template <int DT, int KCAP>
__global__ __launch_bounds__(kThreads, 2) void topk_tilelane_kernel(
    const uint8_t* __restrict__ corpus, const uint8_t* __restrict__ queries, int64_t row_stride,
    int n_rows, int n_q, int n_ktiles, int n_row_tiles, uint32_t row_base, int k_out,
    uint64_t* __restrict__ part_keys, const float* __restrict__ thr_init, int n_splits, int qblocks,
    int flags) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 1;
  const int wq = wave & 1;
  const int fr = lane & 31;
  const int fh = lane >> 5;
  int split, qb;
  if (flags & kFlagXcdRemap) {
    const int x = blockIdx.x & 7;
    const int i = blockIdx.x >> 3;
    split = (i / qblocks) * 8 + x;
    qb = i % qblocks;
  } else {
    split = blockIdx.x % n_splits;
    qb = blockIdx.x / n_splits;
  }
  const int q0 = qb * kTileQ;
  const int t_begin = (int)((int64_t)split * n_row_tiles / n_splits);
  const int t_end = (int)((int64_t)(split + 1) * n_row_tiles / n_splits);

  uint64_t L[2][KCAP];
  float thr[2];
  uint64_t thk[2];
#pragma unroll
  for (int bj = 0; bj < 2; ++bj) {
#pragma unroll
    for (int j = 0; j < KCAP; ++j) L[bj][j] = 0;
    const int q = q0 + wq * 64 + bj * 32 + fr;
    thr[bj] = q < n_q ? (thr_init ? thr_init[q] : -INFINITY) : INFINITY;
    thk[bj] = (q < n_q && thr[bj] != -INFINITY) ? (((uint64_t)ord_f32(thr[bj]) << 32) - 1) : 0;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // thr_init reads retired before the ring counts

  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const uint32_t tile_bytes = (uint32_t)(kTileRows * row_stride);
  const __amdgpu_buffer_rsrc_t q_rsrc = tile_rsrc(queries + (int64_t)q0 * row_stride, tile_bytes);
  const bool screen = !(flags & kFlagSkipEpilogue);

  f32x16 acc[2][2];
  // one k16 step: the wave's 2x2 MFMA blocks
  auto frag_mma = [&](const u32x4 (&a)[2], const u32x4 (&b)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int bj = 0; bj < 2; ++bj) mfma_step<DT>(a[bi], b[bj], acc[bi][bj]);
  };
  // a tile's first k16 step: accumulate onto 0 (an inline constant, no register zeroing)
  auto frag_mma_first = [&](const u32x4 (&a)[2], const u32x4 (&b)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int bj = 0; bj < 2; ++bj) {
        f32x16 z = {};
        mfma_step<DT>(a[bi], b[bj], z);
        acc[bi][bj] = z;
      }
  };

  // Survivor stash: a passing score's key is appended to a 4-entry register stash of its
  // column (a few instructions); the sorted list absorbs the stash only when it fills (and at
  // the end), which is also when the list can raise the column's threshold. Survivors are rare
  // once the pre-pass seeds the thresholds (~0.4 per lane and column over a whole split on the
  // C2 data), so the common path never runs the list insert or the k-th select.
  constexpr int kStash = 4;
  uint64_t S0[kStash], S1[kStash];
  int n0 = 0, n1 = 0;
  auto flush0 = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < kStash; ++c)
      if (c < n0) list_insert<KCAP>(L[0], S0[c]);
    n0 = 0;
    const uint64_t kth = list_at<KCAP>(L[0], k_out - 1);
    if (kth > thk[0]) {
      thk[0] = kth;
      thr[0] = key_score(kth);
    }
  };
  auto flush1 = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < kStash; ++c)
      if (c < n1) list_insert<KCAP>(L[1], S1[c]);
    n1 = 0;
    const uint64_t kth = list_at<KCAP>(L[1], k_out - 1);
    if (kth > thk[1]) {
      thk[1] = kth;
      thr[1] = key_score(kth);
    }
  };

  // ---- tile end: groups (bi, bj) whose max reaches the threshold of column bj; one passing group
  // per lane per round is staged in the lane's private 64-B LDS slot, and its passing scores go
  // to the column's stash, one per set bit of a pass mask in a divergent loop.
  float* slot = reinterpret_cast<float*>(smem + kOffBuf1) + tid * 16;
  auto screen_tile = [&](int r0) __attribute__((always_inline)) {
    const bool full = r0 + kTileRows <= n_rows;  // wave-uniform: row bound tests only on a ragged tile
    uint32_t gmask = 0;
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int bi = 0; bi < 2; ++bi) {
        float m0 = acc[bi][bj][0], m1 = acc[bi][bj][1];
#pragma unroll
        for (int r = 2; r < 16; r += 2) {
          m0 = fmaxf(m0, acc[bi][bj][r]);
          m1 = fmaxf(m1, acc[bi][bj][r + 1]);
        }
        gmask |= (fmaxf(m0, m1) >= thr[bj] ? 1u : 0u) << (bj * 2 + bi);
      }
    if (flags & kFlagMaxOnly) {  // ablation: group maxima only (wrong results)
      if (gmask == 0xFu && thr[0] == 1234.5f) part_keys[0] = 1;
      return;
    }
    while (__ballot(gmask != 0)) {
      const int sel = gmask ? __builtin_ctz(gmask) : -1;
      gmask &= gmask - 1;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if (sel == g) {  // static branch per group, taken only where some lane selected it
#pragma unroll
          for (int c4 = 0; c4 < 4; ++c4) {
            f32x4 v4 = {acc[g & 1][g >> 1][4 * c4], acc[g & 1][g >> 1][4 * c4 + 1], acc[g & 1][g >> 1][4 * c4 + 2],
                        acc[g & 1][g >> 1][4 * c4 + 3]};
            *reinterpret_cast<f32x4*>(slot + 4 * c4) = v4;
          }
        }
      }
      if (sel >= 0) {
        const int bjs = sel >> 1;
        const int rb = r0 + wr * 64 + (sel & 1) * 32 + 4 * fh;
        const float th = bjs ? thr[1] : thr[0];
        const uint64_t tk = bjs ? thk[1] : thk[0];
        uint32_t pm = 0;
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
          const f32x4 v4 = *reinterpret_cast<const f32x4*>(slot + 4 * c4);
#pragma unroll
          for (int e = 0; e < 4; ++e) pm |= (v4[e] >= th ? 1u : 0u) << (4 * c4 + e);
        }
        if (!full) {  // the ragged last tile only: drop rows past the corpus end
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (rb + (r & 3) + 8 * (r >> 2) >= n_rows) pm &= ~(1u << r);
        }
        while (pm) {
          const int r = __builtin_ctz(pm);
          pm &= pm - 1;
          const uint64_t key = make_key(slot[r], row_base + (uint32_t)(rb + (r & 3) + 8 * (r >> 2)));
          if (key > tk) {
            if (bjs == 0) {
#pragma unroll
              for (int c = 0; c < kStash; ++c)
                if (n0 == c) S0[c] = key;
              if (++n0 == kStash) flush0();
            } else {
#pragma unroll
              for (int c = 0; c < kStash; ++c)
                if (n1 == c) S1[c] = key;
              if (++n1 == kStash) flush1();
            }
          }
        }
      }
    }
  };

  // Two 128-B k-tile buffers: tile kt+1 streams in (buffer LDS-DMA) while kt is multiplied.
  // Wave w fills rows [32w, 32w+32) of both tiles, 8 rows (1 KiB) per instruction; lane l lands
  // at (row 8j + l/8, physical chunk l%8) and loads logical chunk (l%8) ^ swz(row).
  const int ld_row = lane >> 3;
  uint32_t ld_off[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = wave_u * 32 + 8 * j + ld_row;
    ld_off[j] = (uint32_t)(row * row_stride) + (((lane & 7) ^ ((row >> 1) & 7)) << 4);
  }
  auto stage_t = [&](int t, int kt, unsigned char* buf) __attribute__((always_inline)) {
    const __amdgpu_buffer_rsrc_t c_rsrc = tile_rsrc(corpus + (int64_t)t * kTileRows * row_stride, tile_bytes);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t off = ld_off[j] + kt * kRowBytes;
      blds16(c_rsrc, off, buf + (wave_u * 32 + 8 * j) * kRowBytes);
      blds16(q_rsrc, off, buf + kTileRows * kRowBytes + (wave_u * 32 + 8 * j) * kRowBytes);
    }
  };
  // k-tile 0 of the first tile; every later tile's k-tile 0 streams in under the previous tile's
  // last k-tile and epilogue (into buffer 0, which the last k-tile does not use when n_ktiles is
  // even), so no tile start waits a full DMA latency
  const bool even_k = (n_ktiles & 1) == 0 && !(flags & kFlagNoTilePrefetch);
  stage_t(t_begin, 0, smem + kOffBuf0);
  for (int t = t_begin; t < t_end; ++t) {
    const int r0 = t * kTileRows;
    const bool load = !(flags & kFlagNoLoads) || t == t_begin;  // ablation: LDS + MFMA ceiling
    if (!even_k && t > t_begin && load) stage_t(t, 0, smem + kOffBuf0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();  // also: every wave is past the previous tile's epilogue (slot reuse below)
    for (int kt = 0; kt < n_ktiles; ++kt) {
      if (kt + 1 < n_ktiles && load) stage_t(t, kt + 1, smem + (((kt + 1) & 1) ? kOffBuf1 : kOffBuf0));
      if (kt + 1 == n_ktiles && even_k && t + 1 < t_end && !(flags & kFlagNoLoads)) stage_t(t + 1, 0, smem + kOffBuf0);
      const unsigned char* buf = smem + ((kt & 1) ? kOffBuf1 : kOffBuf0);
      // two fragment register sets, order pinned with sched_barrier: the LDS reads of step g+1
      // are in flight while the MFMAs of step g run
      u32x4 fa0[2], fb0[2], fa1[2], fb1[2];
      auto frag_load = [&](int g, u32x4 (&a)[2], u32x4 (&b)[2]) __attribute__((always_inline)) {
        const int ch = 2 * g + fh;
#pragma unroll
        for (int bi = 0; bi < 2; ++bi)
          a[bi] = *reinterpret_cast<const u32x4*>(buf + swz(wr * 64 + bi * 32 + fr, ch));
#pragma unroll
        for (int bj = 0; bj < 2; ++bj)
          b[bj] = *reinterpret_cast<const u32x4*>(buf + kTileRows * kRowBytes + swz(wq * 64 + bj * 32 + fr, ch));
      };
      frag_load(0, fa0, fb0);
      frag_load(1, fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
      if (kt == 0)
        frag_mma_first(fa0, fb0);
      else
        frag_mma(fa0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      frag_load(2, fa0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      frag_mma(fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
      frag_load(3, fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
      frag_mma(fa0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      frag_mma(fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
      // stage kt+1 landed (the last k-tile waits for nothing: the next tile's k-tile 0 may still
      // be in flight, the tile start waits for it after the epilogue)
      if (!(flags & kFlagNoWait) && kt + 1 < n_ktiles) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();  // ... everyone's; everyone done with kt
    }
    if (screen) screen_tile(r0);
  }
  if (!screen) {  // ablation: GEMM only, keep acc live, no top-k
    float sink = 0.f;
#pragma unroll
    for (int bi = 0; bi < 2; ++bi)
#pragma unroll
      for (int bj = 0; bj < 2; ++bj)
#pragma unroll
        for (int r = 0; r < 16; ++r) sink += acc[bi][bj][r];
    if (sink == 1234.5678f) part_keys[0] = 1;
    return;
  }

  if (n0) flush0();
  if (n1) flush1();
  // merge the 4 partial lists of each query (2 row-waves x 2 lane halves) through LDS
  __syncthreads();
  uint64_t* xl = reinterpret_cast<uint64_t*>(smem);
  const int part = wr * 2 + fh;
#pragma unroll
  for (int bj = 0; bj < 2; ++bj) {
    const int ql = wq * 64 + bj * 32 + fr;
#pragma unroll
    for (int j = 0; j < KCAP; ++j) xl[(ql * 4 + part) * KCAP + j] = L[bj][j];
  }
  __syncthreads();
  if (tid < kTileQ && q0 + tid < n_q) {
    uint64_t M[KCAP];
#pragma unroll
    for (int j = 0; j < KCAP; ++j) M[j] = xl[(tid * 4) * KCAP + j];
    for (int u = 1; u < 4; ++u) {
      const uint64_t* src = xl + (tid * 4 + u) * KCAP;
      for (int j = 0; j < KCAP; ++j) {
        const uint64_t kk = src[j];
        if (kk <= M[KCAP - 1]) break;  // sorted: nothing further can enter
        list_insert<KCAP>(M, kk);
      }
    }
    uint64_t* dst = part_keys + ((int64_t)(q0 + tid) * n_splits + split) * k_out;
#pragma unroll
    for (int j = 0; j < KCAP; ++j)
      if (j < k_out) dst[j] = M[j];
  }
}

// =============================================================================================
// topk_qkv_kernel (default for bf16/f16 with d_pad = 64 * NKT, k <= 16): the query-resident
// scheme at two waves per SIMD. A workgroup of 8 waves owns 128 queries (one workgroup per CU);
// waves w and w + 4 hold the same 32 queries but opposite halves of the dimension, so each keeps
// only half of the B fragments in registers (96 VGPRs at d = 768). A ring slot ("phase") holds
// k-step j of the tile for the first half and k-step j + NKT/2 for the second. At a tile's end
// the two partial accumulators of a pair meet through LDS (each wave sends the two 32-row blocks
// the other one screens; partial(half 0) + partial(half 1)), and each wave screens its two
// blocks: 16-row group maxima against the query's threshold, passing groups to the candidate
// buffer (a list in private memory takes over when it is full). After the K-loop each lane folds
// its candidate groups (read back from its own buffer, L2-resident) into a register top-k list,
// so the sorted inserts never stall the MFMA pipe; the lists of (query, split, half) go to the
// lane-list merge. Per corpus byte brought in from L2: 128 queries x 2 flops (the two-operand
// 128 x 128 tile kernels: 64). (Measured and dropped: all 32 queries' fragments in registers at
// one wave per SIMD — LDS latency, DMA issue and the screening were exposed.)
// =============================================================================================
namespace qkv {
constexpr int kTR = 128;
constexpr int kHalfBytes = kTR * kRowBytes;         // one 64-deep k-step of 128 rows: 16 KiB
constexpr int kSlotBytes = 2 * kHalfBytes;          // a phase: the k-steps of both halves
constexpr int kXBytes = 4 * 2 * 2 * 4 * 64 * 16;    // exchange [group][from half][block][c4][lane] x 16 B
template <int ST>
struct Cfg {
  static constexpr int kOffX = ST * kSlotBytes;
  static constexpr int kLds = kOffX + kXBytes;
  static_assert(kLds <= 160 * 1024, "qkv LDS exceeds 160 KiB");
};
}  // namespace qkv

template <int DT, int NKT, int ST, int KCAP>
__global__ __launch_bounds__(512, 1) void topk_qkv_kernel(
    const uint8_t* __restrict__ corpus, const uint8_t* __restrict__ queries, int64_t row_stride,
    int n_rows, int n_q, int n_row_tiles, uint32_t row_base, int k_out,
    uint64_t* __restrict__ part_keys, const float* __restrict__ thr_init, int n_splits, int qblocks,
    int flags, uint64_t* __restrict__ cand_keys, int cand_cap) {
  static_assert(DT != DT_F32, "fp32 keeps the two-operand tile kernels (exact fma-chain contract)");
  constexpr int NH = NKT / 2;  // k-steps per half
  static_assert(NKT % 2 == 0 && NH % ST == 0 && ST >= 3, "ring slots must divide the phases of a tile");
  using C = qkv::Cfg<ST>;
  constexpr int TR = qkv::kTR;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int qg = wave & 3;
  const int kh = wave >> 2;
  const int fr = lane & 31;
  const int fh = lane >> 5;
  int split, qb;
  if (flags & kFlagXcdRemap) {
    const int x = blockIdx.x & 7;
    const int i = blockIdx.x >> 3;
    split = (i / qblocks) * 8 + x;
    qb = i % qblocks;
  } else {
    split = blockIdx.x % n_splits;
    qb = blockIdx.x / n_splits;
  }
  const int q = qb * kTileQ + qg * 32 + fr;
  const int t_begin = (int)((int64_t)split * n_row_tiles / n_splits);
  const int t_end = (int)((int64_t)(split + 1) * n_row_tiles / n_splits);

  // B fragments of this lane's query over this wave's half: k16 group i of the half covers
  // elements kh * 64 NH + [16i, 16i + 16); lane half fh holds 8 of them.
  u32x4 Bq[4 * NH];
  {
    const uint8_t* qrow = queries + (int64_t)q * row_stride + kh * NH * kRowBytes + fh * 16;
#pragma unroll
    for (int i = 0; i < 4 * NH; ++i) Bq[i] = *reinterpret_cast<const u32x4*>(qrow + i * 32);
  }
  float thr = q < n_q ? (thr_init ? thr_init[q] : -INFINITY) : INFINITY;
  uint64_t thk = (q < n_q && thr != -INFINITY) ? (((uint64_t)ord_f32(thr) << 32) - 1) : 0;
  // Fallback list (sorted, descending): private memory, touched only when the lane's candidate
  // buffer is full, so it costs no registers in the K-loop.
  volatile uint64_t Ls[KCAP];  // volatile: kept in scratch, not promoted to registers
#pragma unroll 1
  for (int j = 0; j < KCAP; ++j) Ls[j] = 0;
  // candidate key buffer of producer (query q, split, half kh, lane half fh)
  const int64_t cbase = ((int64_t)q * (4 * n_splits) + 4 * split + 2 * kh + fh) * cand_cap;
  int nc = 0;

  if (t_begin < t_end) {
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    const uint32_t tile_bytes = (uint32_t)(TR * row_stride);
    // DMA fill: wave w fills half w / 4, rows [32 (w % 4), +32) of a phase slot, 8 rows per
    // instruction; lane l lands at (row 8j + l/8, physical chunk l%8), logical chunk (l%8) ^ swz.
    // rows 8j and 8j + 16 share the swizzle: two lane offsets, the +16 rows via soffset
    uint32_t ld_off[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = (wave_u & 3) * 32 + 8 * j + (lane >> 3);
      ld_off[j] = (uint32_t)(row * row_stride) + (((lane & 7) ^ ((row >> 1) & 7)) << 4);
    }
    const uint32_t off16 = (uint32_t)(16 * row_stride);
    auto issue = [&](int tile, int ph, int slot) __attribute__((always_inline)) {
      tile = tile < t_end ? tile : t_end - 1;  // past the split: a harmless refill of a dead slot
      const __amdgpu_buffer_rsrc_t r = tile_rsrc(corpus + (int64_t)tile * TR * row_stride, tile_bytes);
      unsigned char* dst = smem + slot * qkv::kSlotBytes + (wave_u >> 2) * qkv::kHalfBytes + (wave_u & 3) * 32 * kRowBytes;
      const int kstep = (wave_u >> 2) * NH + ph;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(dst + j * 8 * kRowBytes),
                                                 16, ld_off[j & 1], kstep * kRowBytes + (j >> 1) * off16, 0, 0);
    };
    uint32_t fo[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) fo[g] = (uint32_t)(kh * qkv::kHalfBytes + swz(fr, 2 * g + fh));
    auto frag_read = [&](int slot, int g, u32x4 (&F)[4]) __attribute__((always_inline)) {
      const unsigned char* base = smem + slot * qkv::kSlotBytes + fo[g];
#pragma unroll
      for (int b = 0; b < 4; ++b) F[b] = *reinterpret_cast<const u32x4*>(base + b * 32 * kRowBytes);
    };

    f32x16 acc[4];
    // One fragment set: block b's fragment of the next k16 group is read right after block b's
    // MFMA of this group has issued, 4 MFMAs (128 cycles) before it is used (16 VGPRs, not 32).
    u32x4 F[4];
    auto mma_read = [&](int bi, bool first, int rslot, int rg) __attribute__((always_inline)) {
      const unsigned char* base = smem + rslot * qkv::kSlotBytes + fo[rg];
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        if (first) {
          f32x16 z = {};
          mfma_step<DT>(F[b], Bq[bi], z);
          acc[b] = z;
        } else {
          mfma_step<DT>(F[b], Bq[bi], acc[b]);
        }
        F[b] = *reinterpret_cast<const u32x4*>(base + b * 32 * kRowBytes);
        __builtin_amdgcn_sched_barrier(0);
      }
    };

    // exchange regions: this wave writes X[qg][kh] and reads X[qg][1 - kh]; the one it read is
    // then its private 64-B-per-lane staging slot for the list fallback
    f32x4* xw = reinterpret_cast<f32x4*>(smem + C::kOffX + (qg * 2 + kh) * 8192) + lane;
    const f32x4* xr = reinterpret_cast<const f32x4*>(smem + C::kOffX + (qg * 2 + (1 - kh)) * 8192) + lane;
    float* slot = reinterpret_cast<float*>(smem + C::kOffX + (qg * 2 + (1 - kh)) * 8192) + lane * 16;

    auto screen_blocks = [&](int r0, int b0) __attribute__((always_inline)) {
      // b0: first of the two blocks this wave screens (compile-time at each call site)
      uint32_t gmask = 0;
#pragma unroll
      for (int bb = 0; bb < 2; ++bb) {
        const int b = b0 + bb;
        float m0 = acc[b][0], m1 = acc[b][1];
#pragma unroll
        for (int r = 2; r < 16; r += 2) {
          m0 = fmaxf(m0, acc[b][r]);
          m1 = fmaxf(m1, acc[b][r + 1]);
        }
        gmask |= (fmaxf(m0, m1) >= thr ? 1u : 0u) << b;
      }
      if (flags & kFlagMaxOnly) {  // ablation: group maxima only (wrong results)
        if (gmask == 0xFu && thr == 1234.5f) part_keys[0] = 1;
        return;
      }
      while (__ballot(gmask != 0)) {
        const int sel = gmask ? __builtin_ctz(gmask) : -1;
        gmask &= gmask - 1;
        // the group's 16 scores go through the lane's 64-B LDS slot; each score that beats the
        // admission key is appended to the lane's candidate key buffer (one 8-B store), or, once
        // that is full, inserted into the private fallback list (which raises the threshold)
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
          const int b = b0 + bb;
          if (sel == b) {
#pragma unroll
            for (int c4 = 0; c4 < 4; ++c4)
              *reinterpret_cast<f32x4*>(slot + 4 * c4) =
                  f32x4{acc[b][4 * c4], acc[b][4 * c4 + 1], acc[b][4 * c4 + 2], acc[b][4 * c4 + 3]};
          }
        }
        if (sel >= 0) {
          const int rb = r0 + sel * 32 + 4 * fh;
          uint32_t pm = 0;
#pragma unroll
          for (int c4 = 0; c4 < 4; ++c4) {
            const f32x4 v4 = *reinterpret_cast<const f32x4*>(slot + 4 * c4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int r = 4 * c4 + e;
              pm |= (v4[e] >= thr && rb + (r & 3) + 8 * (r >> 2) < n_rows ? 1u : 0u) << r;
            }
          }
          while (pm) {
            const int r = __builtin_ctz(pm);
            pm &= pm - 1;
            const uint64_t key = make_key(slot[r], row_base + (uint32_t)(rb + (r & 3) + 8 * (r >> 2)));
            if (key > thk) {
              if (nc < cand_cap) {
                cand_keys[cbase + nc] = key;
                ++nc;
              } else {  // thk >= the list's k-th >= its last: key enters, the last drops
                int j = KCAP - 1;
#pragma unroll 1
                while (j > 0 && Ls[j - 1] < key) {
                  Ls[j] = Ls[j - 1];
                  --j;
                }
                Ls[j] = key;
                const uint64_t kth = Ls[k_out - 1];
                if (kth > thk) {
                  thk = kth;
                  thr = key_score(kth);
                }
              }
            }
          }
        }
      }
    };
    auto tile_end = [&](int r0) __attribute__((always_inline)) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (kh == h) {  // wave-uniform; compile-time block indices inside
#pragma unroll
          for (int bb = 0; bb < 2; ++bb) {
            const int b = (h == 0 ? 2 : 0) + bb;  // the partner's blocks
#pragma unroll
            for (int c4 = 0; c4 < 4; ++c4)
              xw[(bb * 4 + c4) * 64] = f32x4{acc[b][4 * c4], acc[b][4 * c4 + 1], acc[b][4 * c4 + 2], acc[b][4 * c4 + 3]};
          }
        }
      }
      lds_barrier();
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (kh == h) {
#pragma unroll
          for (int bb = 0; bb < 2; ++bb) {
            const int b = (h == 0 ? 0 : 2) + bb;  // own blocks: partial(half 0) + partial(half 1)
#pragma unroll
            for (int c4 = 0; c4 < 4; ++c4) {
              const f32x4 v = xr[(bb * 4 + c4) * 64];
#pragma unroll
              for (int e = 0; e < 4; ++e) acc[b][4 * c4 + e] = acc[b][4 * c4 + e] + v[e];
            }
          }
          if (!(flags & kFlagSkipEpilogue)) screen_blocks(r0, h == 0 ? 0 : 2);
        }
      }
    };

    // Ring of ST phase slots. Before phase j's data is used, barrier B(j): this wave's DMA of phase
    // j landed (vmcnt leaves the ST-2 younger phases in flight), lgkmcnt(0) (every wave's reads
    // of phase j-1 are done), s_barrier; then phase j+ST-1 is issued into slot (j-1) % ST. B(j+1)
    // sits inside phase j, after its last fragment reads, so phase j+1's first reads overlap
    // phase j's last MFMAs.
    constexpr int kVm = 4 * (ST - 2);
#pragma unroll
    for (int c = 0; c < ST - 1; ++c) issue(t_begin, c, c);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kVm) : "memory");
    lds_barrier();
    issue(t_begin, ST - 1, ST - 1);
    frag_read(0, 0, F);
    for (int t = t_begin; t < t_end; ++t) {
#pragma unroll
      for (int ph = 0; ph < NH; ++ph) {
        const int sl = ph % ST;
        __builtin_amdgcn_sched_barrier(0);
        mma_read(4 * ph + 0, ph == 0, sl, 1);
        mma_read(4 * ph + 1, false, sl, 2);
        mma_read(4 * ph + 2, false, sl, 3);
        if (!(flags & kFlagNoWait)) {
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kVm) : "memory");
          lds_barrier();
        }
        if (!(flags & kFlagNoLoads)) issue(t + (ph + ST) / NH, (ph + ST) % NH, sl);
        __builtin_amdgcn_sched_barrier(0);
        mma_read(4 * ph + 3, false, (ph + 1) % ST, 0);
      }
      tile_end(t * TR);
    }
    if (flags & kFlagSkipEpilogue) {
      float sink = 0.f;
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) sink += acc[b][r];
      if (sink == 1234.5678f) part_keys[0] = 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the workgroup ends
  }

  // Fold the candidate keys into a register list (candidate rows and the fallback list's rows are
  // disjoint), merge lanes l and l ^ 32 (disjoint rows of one query) and write one list per
  // (query, split, half).
  uint64_t L[KCAP];
#pragma unroll
  for (int j = 0; j < KCAP; ++j) L[j] = Ls[j];
  for (int g0 = 0; g0 < nc; g0 += 8) {  // 8 loads in flight, then the inserts
    uint64_t c8[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) c8[u] = g0 + u < nc ? cand_keys[cbase + g0 + u] : 0;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (c8[u]) list_insert<KCAP>(L, c8[u]);
  }
  uint64_t P[KCAP];
#pragma unroll
  for (int j = 0; j < KCAP; ++j) P[j] = shfl_xor_u64(L[j], 32);
  if (fh == 0 && q < n_q) {
#pragma unroll
    for (int j = 0; j < KCAP; ++j) list_insert<KCAP>(L, P[j]);
    uint64_t* dst = part_keys + ((int64_t)q * (2 * n_splits) + 2 * split + kh) * k_out;
#pragma unroll
    for (int j = 0; j < KCAP; ++j)
      if (j < k_out) dst[j] = L[j];
  }
}

// =============================================================================================
// topk_t256_kernel (bf16/f16, k <= 16): 256 corpus rows x 256 queries per workgroup tile, 8 waves
// (2 along rows x 4 along queries), each wave a 128 x 64 block of v_mfma_f32_16x16x32 (32
// accumulator blocks = 128 VGPRs), one workgroup per CU, 64-deep k-steps through a 2-stage
// 128-KiB buffer LDS-DMA ring that runs across tile boundaries. Against the 128 x 128 kernels:
// 2x the MFMAs per staged byte and per LDS-read byte, and a k-step of 64 MFMAs per wave between
// barriers instead of 16 (cdna_hip_programming.md: the 128^2 two-barrier structure tops out near
// 0.9 PF/s; 256^2 tiles at one workgroup per CU are what go past it). Epilogue per tile: each
// lane holds 4 query columns x 32 rows; per (query, 16-row group) the max against the query's
// threshold; passing groups are scanned straight from the accumulators, passing scores into a
// per-(query, split, row half, lane quarter) candidate key buffer (a full buffer falls back to a
// sorted list in private memory that raises the threshold). After the last tile each lane folds
// its keys into a register list per query; the 4 lane quarters of a query merge by shuffles.
// =============================================================================================
namespace t256 {
constexpr int kTR = 256, kTQ = 256;
constexpr int kStage = (kTR + kTQ) * kRowBytes;  // 64 KiB: A (corpus) rows, then B (queries) rows
constexpr int kLds = 2 * kStage;                 // 128 KiB
static_assert(kLds <= 160 * 1024, "t256 LDS exceeds 160 KiB");
}  // namespace t256

__device__ __forceinline__ void mfma16(const u32x4& a, const u32x4& b, f32x4& acc, int dt) {
  if (dt == DT_BF16)
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc, 0,
                                                  0, 0);
  else
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), acc, 0, 0,
                                                 0);
}

template <int DT, int KCAP>
__global__ __launch_bounds__(512, 1) void topk_t256_kernel(
    const uint8_t* __restrict__ corpus, const uint8_t* __restrict__ queries, int64_t row_stride, int n_rows,
    int n_q, int n_ktiles, int n_row_tiles, uint32_t row_base, int k_out, uint64_t* __restrict__ part_keys,
    const float* __restrict__ thr_init, int n_splits, int qblocks, int flags, uint64_t* __restrict__ cand_keys,
    int cand_cap) {
  static_assert(DT != DT_F32, "fp32 keeps the exact single-chain kernels");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 2;  // 128-row half of the tile
  const int wn = wave & 3;   // 64-query quarter of the block
  const int fr = lane & 15;
  const int fq = lane >> 4;
  int split, qb;
  if (flags & kFlagXcdRemap) {
    const int x = blockIdx.x & 7;
    const int i = blockIdx.x >> 3;
    split = (i / qblocks) * 8 + x;
    qb = i % qblocks;
  } else {
    split = blockIdx.x % n_splits;
    qb = blockIdx.x / n_splits;
  }
  const int q0 = qb * t256::kTQ;
  const int t_begin = (int)((int64_t)split * n_row_tiles / n_splits);
  const int t_end = (int)((int64_t)(split + 1) * n_row_tiles / n_splits);

  float thr[4];
  uint64_t thk[4];
  int nc[4];
  // one register stash key per query slot: the first survivor of a query slot stays in a register,
  // later ones go to the candidate buffer in memory; a store at a tile end would otherwise hold
  // the next k-step's vmcnt(0) wait for its write acknowledgment
  uint64_t stash[4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const int q = q0 + wn * 64 + nb * 16 + fr;
    thr[nb] = q < n_q ? (thr_init ? thr_init[q] : -INFINITY) : INFINITY;
    thk[nb] = (q < n_q && thr[nb] != -INFINITY) ? (((uint64_t)ord_f32(thr[nb]) << 32) - 1) : 0;
    nc[nb] = 0;
    stash[nb] = 0;
  }
  // producer of query slot nb: (query, split, row half wm, lane quarter fq)
  auto cbase = [&](int nb) __attribute__((always_inline)) {
    const int q = q0 + wn * 64 + nb * 16 + fr;
    return ((int64_t)q * (8 * n_splits) + 8 * split + 4 * wm + fq) * cand_cap;
  };
  volatile uint64_t Ls[4][KCAP];  // private memory: touched only when a candidate buffer is full
#pragma unroll 1
  for (int j = 0; j < 4 * KCAP; ++j) Ls[j / KCAP][j % KCAP] = 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // thr_init reads retired before the ring counts

  if (t_begin < t_end) {
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    const uint32_t tile_bytes = (uint32_t)(t256::kTR * row_stride);
    const __amdgpu_buffer_rsrc_t q_rsrc = tile_rsrc(queries + (int64_t)q0 * row_stride, tile_bytes);
    // DMA: wave w fills rows [32w, 32w + 32) of both the A and the B image, 8 rows per
    // instruction; lane l lands at (row 8j + l/8, physical chunk l%8), loads logical chunk
    // (l%8) ^ ((row >> 1) & 7). Rows 8j and 8j + 16 share the swizzle (soffset adds 16 rows).
    uint32_t ld_off[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = wave_u * 32 + 8 * j + (lane >> 3);
      ld_off[j] = (uint32_t)(row * row_stride) + (((lane & 7) ^ ((row >> 1) & 7)) << 4);
    }
    const uint32_t off16 = (uint32_t)(16 * row_stride);
    auto issue = [&](int tile, int kt, int stage) __attribute__((always_inline)) {
      const __amdgpu_buffer_rsrc_t c_rsrc = tile_rsrc(corpus + (int64_t)tile * t256::kTR * row_stride, tile_bytes);
      unsigned char* dst = smem + stage * t256::kStage + wave_u * 32 * kRowBytes;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t so = kt * kRowBytes + (j >> 1) * off16;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(c_rsrc, (__attribute__((address_space(3))) void*)(dst + j * 8 * kRowBytes),
                                                 16, ld_off[j & 1], so, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            q_rsrc, (__attribute__((address_space(3))) void*)(dst + t256::kTR * kRowBytes + j * 8 * kRowBytes), 16,
            ld_off[j & 1], so, 0, 0);
      }
    };
    // fragment reads (16x16x32: lane l reads row l & 15, 16-B chunk 4s + l / 16 of the 64-deep
    // k-step, XOR-swizzled by bits 1-3 of the row)
    const int x = (fr >> 1) & 7;
    const uint32_t fo0 = (uint32_t)(fr * kRowBytes + (((0 + fq) ^ x) << 4));
    const uint32_t fo1 = (uint32_t)(fr * kRowBytes + (((4 + fq) ^ x) << 4));

    f32x4 acc[8][4];

    auto list_push = [&](int nb, uint64_t key) {
      int j = KCAP - 1;
#pragma unroll 1
      while (j > 0 && Ls[nb][j - 1] < key) {
        Ls[nb][j] = Ls[nb][j - 1];
        --j;
      }
      Ls[nb][j] = key;
      const uint64_t kth = Ls[nb][k_out - 1];
      if (kth > thk[nb]) {
        thk[nb] = kth;
        thr[nb] = key_score(kth);
      }
    };

    issue(t_begin, 0, 0);
    int c = 0;  // global k-step counter (stage = c & 1)
    for (int t = t_begin; t < t_end; ++t) {
#pragma unroll
      for (int mb = 0; mb < 8; ++mb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) acc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int kt = 0; kt < n_ktiles; ++kt, ++c) {
        // top of step c: this wave's DMA of step c landed (the only one in flight), then the
        // barrier: everyone's landed, everyone is done reading step c - 1's stage
        if (!(flags & kFlagNoWait)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
        if (!(flags & kFlagNoLoads)) {
          if (kt + 1 < n_ktiles)
            issue(t, kt + 1, (c + 1) & 1);
          else if (t + 1 < t_end)
            issue(t + 1, 0, (c + 1) & 1);
        }
        const unsigned char* st = smem + (c & 1) * t256::kStage;
        const unsigned char* abase = st + (wm * 128) * kRowBytes;
        const unsigned char* bbase = st + (t256::kTR + wn * 64) * kRowBytes;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const uint32_t fo = s ? fo1 : fo0;
          u32x4 b[4];
#pragma unroll
          for (int nb = 0; nb < 4; ++nb) b[nb] = *reinterpret_cast<const u32x4*>(bbase + nb * 16 * kRowBytes + fo);
#pragma unroll
          for (int mb = 0; mb < 8; ++mb) {
            const u32x4 a = *reinterpret_cast<const u32x4*>(abase + mb * 16 * kRowBytes + fo);
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) mfma16(a, b[nb], acc[mb][nb], DT);
          }
        }
      }
      if (flags & kFlagSkipEpilogue) continue;
      // ---- tile end: (query slot nb, row half mh) groups = acc[4 mh .. 4 mh + 3][nb], 16 rows
      const int r0 = t * t256::kTR + wm * 128;
      uint32_t gmask = 0;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int mh = 0; mh < 2; ++mh) {
          float m = acc[4 * mh][nb][0];
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int i = 0; i < 4; ++i) m = fmaxf(m, acc[4 * mh + u][nb][i]);
          gmask |= (m >= thr[nb] ? 1u : 0u) << (nb * 2 + mh);
        }
      if (flags & kFlagMaxOnly) {  // ablation: group maxima only (wrong results)
        if (gmask == 0xFFu && thr[0] == 1234.5f) part_keys[0] = 1;
        continue;
      }
      // passing groups, one static group at a time (skipped unless some lane passes it): the
      // pass mask and the passing values come straight from the accumulators (select chain), no
      // LDS round trip
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        const int nb = g >> 1, mh = g & 1;
        if (!__ballot((gmask >> g) & 1u)) continue;
        if ((gmask >> g) & 1u) {
          const int rb = r0 + mh * 64 + fq * 4;  // value 4u + i: row rb + 16u + i
          uint32_t pm = 0;
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              pm |= (acc[4 * mh + u][nb][i] >= thr[nb] && rb + 16 * u + i < n_rows ? 1u : 0u) << (4 * u + i);
          while (pm) {
            const int r = __builtin_ctz(pm);
            pm &= pm - 1;
            float v = acc[4 * mh][nb][0];
#pragma unroll
            for (int rr = 1; rr < 16; ++rr) v = (r == rr) ? acc[4 * mh + (rr >> 2)][nb][rr & 3] : v;
            const uint64_t key = make_key(v, row_base + (uint32_t)(rb + 16 * (r >> 2) + (r & 3)));
            if (key > thk[nb]) {
              if (stash[nb] == 0) {
                stash[nb] = key;
              } else if (nc[nb] < cand_cap) {
                cand_keys[cbase(nb) + nc[nb]] = key;
                ++nc[nb];
              } else {
                list_push(nb, key);
              }
            }
          }
        }
      }
    }
    if (flags & kFlagSkipEpilogue) {
      float sink = 0.f;
#pragma unroll
      for (int mb = 0; mb < 8; ++mb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) sink += acc[mb][nb][0] + acc[mb][nb][3];
      if (sink == 1234.5678f) part_keys[0] = 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the workgroup ends
  }

  // per query slot: fold the candidate keys into a register list, merge the 4 lane quarters
  // (lanes fr, fr + 16, fr + 32, fr + 48: disjoint rows of one query), write one list per
  // (query, split, row half)
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const int q = q0 + wn * 64 + nb * 16 + fr;
    uint64_t L[KCAP];
#pragma unroll
    for (int j = 0; j < KCAP; ++j) L[j] = Ls[nb][j];
    if (stash[nb]) list_insert<KCAP>(L, stash[nb]);
    const int n = nc[nb];
    const int64_t cb = q < n_q ? cbase(nb) : 0;
    for (int g0 = 0; g0 < n; g0 += 8) {
      uint64_t c8[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) c8[u] = g0 + u < n ? cand_keys[cb + g0 + u] : 0;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (c8[u]) list_insert<KCAP>(L, c8[u]);
    }
#pragma unroll
    for (int m = 16; m <= 32; m <<= 1) {
      uint64_t P[KCAP];
#pragma unroll
      for (int j = 0; j < KCAP; ++j) P[j] = shfl_xor_u64(L[j], m);
#pragma unroll
      for (int j = 0; j < KCAP; ++j) list_insert<KCAP>(L, P[j]);
    }
    if (fq == 0 && q < n_q) {
      uint64_t* dst = part_keys + ((int64_t)q * (2 * n_splits) + 2 * split + wm) * k_out;
#pragma unroll
      for (int j = 0; j < KCAP; ++j)
        if (j < k_out) dst[j] = L[j];
    }
  }
}

// =============================================================================================
// topk_kb256_kernel (bf16/f16, k <= 16; the default from B = 17): the t256 tile (256 corpus rows x
// 256 queries, 8 waves = 2 along rows x 4 along queries, a 128 x 64 block of 16x16x32 MFMAs per
// wave, 128 accumulator VGPRs, one workgroup per CU) fed from a K-BLOCKED copy of the corpus and
// of the queries: [tile of 256 rows][32-deep k-block][256 rows][64 B].
// A 32-deep k-step of a tile
// is then one contiguous 16-KiB block whose 128-B lines are whole (row pairs), so the k-steps can
// be 32 deep without splitting lines between two requests (the cost that sank 64-B half rows in
// the row-major kernels), and 32-KiB stages leave room for a 4-stage ring: each k-step issues the
// step 3 ahead (96 KiB in flight) right after its barrier and waits, with a counted vmcnt, only
// for its own step — the t256 kernel's 64-deep 2-stage ring waited for the step it had just
// issued. Bytes per MFMA are the t256 tile's (half the 128 x 128 kernels'). One barrier per 32
// MFMAs per wave. The epilogue (group maxima, register stash, candidate buffer, fallback list,
// end-of-kernel fold and lane-quarter merge) and the fragment map and k order are t256's, so the
// scores and rows are bitwise those of t256 and of the small-batch kernel.
// =============================================================================================
namespace kb256 {
constexpr int kTR = 256, kTQ = 256;
constexpr int kKB = 64;                          // bytes of one row in one 32-deep k-block
constexpr int kBlock = kTR * kKB;                // 16 KiB: one operand's k-step
constexpr int kStage = 2 * kBlock;               // A (corpus) block, then B (queries) block
constexpr int kStages = 4;
constexpr int kLds = kStages * kStage;           // 128 KiB
static_assert(kLds <= 160 * 1024, "kb256 LDS exceeds 160 KiB");
// block index of k-block kb of tile t
__host__ __device__ __forceinline__ int64_t block(int64_t t, int kb, int n_kb) { return t * n_kb + kb; }
// byte offset of (row, k-block) in a k-blocked buffer of n_kb k-blocks
__host__ __device__ __forceinline__ int64_t offset(int64_t row, int kb, int n_kb) {
  return (block(row >> 8, kb, n_kb) * kTR + (row & 255)) * kKB;
}
// LDS image of a 64-B row: logical 16-B chunk c of row r sits in physical slot c ^ h(r), h(r) =
// (-(r >> 2)) & 3. A 256-B bank row holds 4 rows; a ds_read_b128 lane group of the 16x16x32
// fragment reads rows 0-3 and 12-15 at chunk q and rows 4-11 at chunk q ^ 1 (lanes {0-3, 12-15,
// 20-27}), so the rows r = i, i + 4, i + 8, i + 12 of a group need distinct slots: h(0..3) =
// 0, 3, 2, 1 makes {h0, 1 ^ h1, 1 ^ h2, h3} = {0, 2, 3, 1} (and its XOR with 1, 2, 3 for the
// other groups) a permutation: conflict-free. (The plain c ^ ((r >> 2) & 3) is 2-way.)
__host__ __device__ __forceinline__ int phys(int chunk, int row) { return chunk ^ ((-(row >> 2)) & 3); }
}  // namespace kb256

// row-major storage rows [row0, row0 + n) -> k-blocked copy (one thread per 16-B chunk)
__global__ __launch_bounds__(256) void reblock_kb_kernel(const uint8_t* __restrict__ src, int64_t row_stride,
                                                         int64_t row0, int64_t n, int n_kb,
                                                         uint8_t* __restrict__ dst) {
  const int per_row = n_kb * 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n * per_row) return;
  const int64_t row = row0 + i / per_row;
  const int ch = (int)(i % per_row);
  const u32x4 v = *reinterpret_cast<const u32x4*>(src + row * row_stride + (int64_t)ch * 16);
  *reinterpret_cast<u32x4*>(dst + kb256::offset(row, ch >> 2, n_kb) + (ch & 3) * 16) = v;
}

// The same kernel with WN = 2 waves along queries ("kb128": 256 rows x 128 queries, 4 waves, two
// workgroups per CU, a 3-stage ring of 24-KiB steps, 72 KiB of LDS): the wave tile, fragment map,
// k order and epilogue are unchanged, so scores and rows are bitwise kb256's; two independent
// workgroups per CU cover each other's barriers, fragment-read latency and epilogue, which eight
// waves in lock-step (one workgroup per CU) do not.
template <int WN>
struct KbCfg {
  static constexpr int kWaves = 2 * WN;
  static constexpr int kThreads = 64 * kWaves;
  static constexpr int kTQ = 64 * WN;                        // queries per workgroup
  static constexpr int kBBlock = kTQ * kb256::kKB;           // one k-step of the query block
  static constexpr int kStageBytes = kb256::kBlock + kBBlock;
  static constexpr int kStages = WN == 4 ? 4 : 3;
  static constexpr int kLds = kStages * kStageBytes;
  static constexpr int kAPieces = 16 / kWaves;               // 1-KiB DMA pieces per wave and k-step
  static constexpr int kBPieces = kTQ / 16 / kWaves;
  static constexpr int kPieces = kAPieces + kBPieces;
  static constexpr int kMinBlocks = WN == 4 ? 1 : 2;
  static_assert(kLds * kMinBlocks <= 160 * 1024, "k-blocked kernel LDS exceeds 160 KiB per CU");
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int DT, int KCAP, int WN>
__global__ __launch_bounds__(KbCfg<WN>::kThreads, KbCfg<WN>::kMinBlocks) void topk_kb256_kernel(
    const uint8_t* __restrict__ corpus_kb, const uint8_t* __restrict__ queries_kb, int n_kb, int n_rows, int n_q,
    int n_row_tiles, uint32_t row_base, int k_out, uint64_t* __restrict__ part_keys,
    const float* __restrict__ thr_init, int n_splits, int qblocks, int flags, uint64_t* __restrict__ cand_keys,
    int cand_cap) {
  static_assert(DT != DT_F32, "fp32 keeps the exact single-chain kernels");
  using C = KbCfg<WN>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN;  // 128-row half of the tile
  const int wn = wave % WN;  // 64-query block of the workgroup's queries
  const int fr = lane & 15;
  const int fq = lane >> 4;
  int split, qb;
  if (flags & kFlagXcdRemap) {
    const int x = blockIdx.x & 7;
    const int i = blockIdx.x >> 3;
    split = (i / qblocks) * 8 + x;
    qb = i % qblocks;
  } else {
    split = blockIdx.x % n_splits;
    qb = blockIdx.x / n_splits;
  }
  const int q0 = qb * C::kTQ;
  const int t_begin = (int)((int64_t)split * n_row_tiles / n_splits);
  const int t_end = (int)((int64_t)(split + 1) * n_row_tiles / n_splits);

  // Per query slot: the admission threshold (a score: every score >= it is a candidate; the seed
  // is a lower bound of the final k-th best), the first survivor in a register (a store would hold
  // the next vmcnt wait) and the candidate-buffer fill, 8 bits per slot in one register.
  float thr[4];
  uint64_t stash[4];
  uint32_t ncp = 0;
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const int q = q0 + wn * 64 + nb * 16 + fr;
    thr[nb] = q < n_q ? (thr_init ? thr_init[q] : -INFINITY) : INFINITY;
    stash[nb] = 0;
  }
  auto cbase = [&](int nb) __attribute__((always_inline)) {
    const int q = q0 + wn * 64 + nb * 16 + fr;
    return ((int64_t)q * (8 * n_splits) + 8 * split + 4 * wm + fq) * cand_cap;
  };
  volatile uint64_t Ls[4][KCAP];  // private memory: touched only when a candidate buffer is full
#pragma unroll 1
  for (int j = 0; j < 4 * KCAP; ++j) Ls[j / KCAP][j % KCAP] = 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // thr_init reads retired before the ring counts

  const int total = (t_end - t_begin) * n_kb;  // k-steps of this workgroup
  if (total > 0) {
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    // DMA: per block, wave w fills the 16-row pieces w, w + waves, w + 2 waves, ... (1 KiB each),
    // lane l at (row 16w + l/4, physical slot l%4), loading the logical chunk whose kb256::phys is
    // l%4 (phys is an involution in the chunk, and rows 16 apart share it): every ds_read_b128
    // lane group hits 16 distinct 16-B bank slots
    constexpr int kPieceStride = C::kWaves * 16 * kb256::kKB;
    const int lrow = wave_u * 16 + (lane >> 2);
    const uint32_t voff = (uint32_t)(lrow * kb256::kKB + (kb256::phys(lane & 3, lrow) << 4));
    // the workgroup's queries: rows (q0 & 255) .. + kTQ of each k-block of their 256-query tile
    const uint8_t* qblk = queries_kb + (q0 & 255) * kb256::kKB;
    auto issue = [&](int c, int stage) __attribute__((always_inline)) {
      int t = t_begin + c / n_kb;
      if (flags & kFlagTileZero) t = 0;
      if (flags & kFlagTileFirst) t = t_begin;
      const int kb = c % n_kb;
      const __amdgpu_buffer_rsrc_t a_rsrc =
          tile_rsrc(corpus_kb + kb256::block(t, kb, n_kb) * kb256::kBlock, kb256::kBlock);
      const __amdgpu_buffer_rsrc_t b_rsrc =
          tile_rsrc(qblk + kb256::block(q0 >> 8, kb, n_kb) * kb256::kBlock, C::kBBlock);
      unsigned char* dst = smem + stage * C::kStageBytes + wave_u * 16 * kb256::kKB;
#pragma unroll
      for (int j = 0; j < C::kAPieces; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            a_rsrc, (__attribute__((address_space(3))) void*)(dst + j * kPieceStride), 16, voff, j * kPieceStride, 0, 0);
#pragma unroll
      for (int j = 0; j < C::kBPieces; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            b_rsrc, (__attribute__((address_space(3))) void*)(dst + kb256::kBlock + j * kPieceStride), 16, voff,
            j * kPieceStride, 0, 0);
    };
    // fragment reads: lane l reads row l & 15, logical chunk l / 16 (k 8(l/16) .. +8 of the step)
    const uint32_t fo = (uint32_t)(fr * kb256::kKB + (kb256::phys(fq, fr) << 4));

    f32x4 acc[8][4];

    auto list_push = [&](int nb, uint64_t key) {
      int j = KCAP - 1;
#pragma unroll 1
      while (j > 0 && Ls[nb][j - 1] < key) {
        Ls[nb][j] = Ls[nb][j - 1];
        --j;
      }
      Ls[nb][j] = key;
      const uint64_t kth = Ls[nb][k_out - 1];
      if (kth) thr[nb] = fmaxf(thr[nb], key_score(kth));
    };

    constexpr int kAhead = C::kStages - 1;  // k-steps in flight ahead of the one being multiplied
    const int pro = total < kAhead ? total : kAhead;
    for (int c = 0; c < pro; ++c) issue(c, c);
    int t = t_begin;
    int kb = 0;
    int st_c = 0;                 // stage of step c
    int st_i = kAhead % C::kStages;  // stage of step c + kAhead (= step c - 1's)
    for (int c = 0; c < total; ++c) {
      // this wave's DMA of step c landed: leave the steps issued after it (up to kAhead - 1) in flight
      const int ahead = total - 1 - c;
      if (!(flags & kFlagNoWait)) {
        if constexpr (kAhead == 3) {
          if (ahead >= 2)
            wait_vmcnt<2 * C::kPieces>();
          else if (ahead == 1)
            wait_vmcnt<C::kPieces>();
          else
            wait_vmcnt<0>();
        } else {
          if (ahead >= 1)
            wait_vmcnt<C::kPieces>();
          else
            wait_vmcnt<0>();
        }
      }
      lds_barrier();  // everyone's step c landed; everyone finished reading step c - 1
      if (c + kAhead < total && !((flags & kFlagNoLoads) && c >= 1)) issue(c + kAhead, st_i);  // into step c - 1's stage
      const unsigned char* st = smem + st_c * C::kStageBytes;
      st_c = st_c + 1 == C::kStages ? 0 : st_c + 1;
      st_i = st_i + 1 == C::kStages ? 0 : st_i + 1;
      const unsigned char* abase = st + (wm * 128) * kb256::kKB + fo;
      const unsigned char* bbase = st + kb256::kBlock + (wn * 64) * kb256::kKB + fo;
      u32x4 b[4];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) b[nb] = *reinterpret_cast<const u32x4*>(bbase + nb * 16 * kb256::kKB);
      if (kb == 0) {  // a tile's first k-step accumulates onto an inline-constant 0 (no register zeroing)
#pragma unroll
        for (int mb = 0; mb < 8; ++mb) {
          const u32x4 a = *reinterpret_cast<const u32x4*>(abase + mb * 16 * kb256::kKB);
#pragma unroll
          for (int nb = 0; nb < 4; ++nb) {
            f32x4 z = {0.f, 0.f, 0.f, 0.f};
            mfma16(a, b[nb], z, DT);
            acc[mb][nb] = z;
          }
        }
      } else {
#pragma unroll
        for (int mb = 0; mb < 8; ++mb) {
          const u32x4 a = *reinterpret_cast<const u32x4*>(abase + mb * 16 * kb256::kKB);
#pragma unroll
          for (int nb = 0; nb < 4; ++nb) mfma16(a, b[nb], acc[mb][nb], DT);
        }
      }
      if (++kb < n_kb) continue;
      kb = 0;
      const int tile = t++;
      if (flags & kFlagSkipEpilogue) continue;
      // ---- tile end: (query slot nb, row half mh) groups = acc[4 mh .. 4 mh + 3][nb], 16 rows
      const int r0 = tile * kb256::kTR + wm * 128;
      const bool full = tile * kb256::kTR + kb256::kTR <= n_rows;  // row bound tests only on a ragged tile
      uint32_t gmask = 0;
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int mh = 0; mh < 2; ++mh) {
          float m = acc[4 * mh][nb][0];
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int i = 0; i < 4; ++i) m = fmaxf(m, acc[4 * mh + u][nb][i]);
          gmask |= (m >= thr[nb] ? 1u : 0u) << (nb * 2 + mh);
        }
      if (flags & kFlagMaxOnly) {  // ablation: group maxima only (wrong results)
        if (gmask == 0xFFu && thr[0] == 1234.5f) part_keys[0] = 1;
        continue;
      }
#pragma unroll
      for (int g = 0; g < 8; ++g) {
        const int nb = g >> 1, mh = g & 1;
        if (!__ballot((gmask >> g) & 1u)) continue;
        if ((gmask >> g) & 1u) {
          const int rb = r0 + mh * 64 + fq * 4;  // value 4u + i: row rb + 16u + i
          uint32_t pm = 0;
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int i = 0; i < 4; ++i) pm |= (acc[4 * mh + u][nb][i] >= thr[nb] ? 1u : 0u) << (4 * u + i);
          if (!full) {  // the ragged last tile only
#pragma unroll
            for (int r = 0; r < 16; ++r)
              if (rb + 16 * (r >> 2) + (r & 3) >= n_rows) pm &= ~(1u << r);
          }
          while (pm) {
            const int r = __builtin_ctz(pm);
            pm &= pm - 1;
            float v = acc[4 * mh][nb][0];
#pragma unroll
            for (int rr = 1; rr < 16; ++rr) v = (r == rr) ? acc[4 * mh + (rr >> 2)][nb][rr & 3] : v;
            const uint64_t key = make_key(v, row_base + (uint32_t)(rb + 16 * (r >> 2) + (r & 3)));
            const int n = (ncp >> (8 * nb)) & 255;
            if (stash[nb] == 0) {
              stash[nb] = key;
            } else if (n < cand_cap) {
              cand_keys[cbase(nb) + n] = key;
              ncp += 1u << (8 * nb);
            } else {
              list_push(nb, key);
            }
          }
        }
      }
    }
    if (flags & kFlagSkipEpilogue) {
      float sink = 0.f;
#pragma unroll
      for (int mb = 0; mb < 8; ++mb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) sink += acc[mb][nb][0] + acc[mb][nb][3];
      if (sink == 1234.5678f) part_keys[0] = 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the workgroup ends
  }

  // per query slot: fold the candidate keys into a register list, merge the 4 lane quarters
  // (lanes fr, fr + 16, fr + 32, fr + 48: disjoint rows of one query), write one list per
  // (query, split, row half)
#pragma unroll
  for (int nb = 0; nb < 4; ++nb) {
    const int q = q0 + wn * 64 + nb * 16 + fr;
    uint64_t L[KCAP];
#pragma unroll
    for (int j = 0; j < KCAP; ++j) L[j] = Ls[nb][j];
    if (stash[nb]) list_insert<KCAP>(L, stash[nb]);
    const int n = (ncp >> (8 * nb)) & 255;
    const int64_t cb = q < n_q ? cbase(nb) : 0;
    for (int g0 = 0; g0 < n; g0 += 8) {
      uint64_t c8[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) c8[u] = g0 + u < n ? cand_keys[cb + g0 + u] : 0;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (c8[u]) list_insert<KCAP>(L, c8[u]);
    }
#pragma unroll
    for (int m = 16; m <= 32; m <<= 1) {
      uint64_t P[KCAP];
#pragma unroll
      for (int j = 0; j < KCAP; ++j) P[j] = shfl_xor_u64(L[j], m);
#pragma unroll
      for (int j = 0; j < KCAP; ++j) list_insert<KCAP>(L, P[j]);
    }
    if (fq == 0 && q < n_q) {
      uint64_t* dst = part_keys + ((int64_t)q * (2 * n_splits) + 2 * split + wm) * k_out;
#pragma unroll
      for (int j = 0; j < KCAP; ++j)
        if (j < k_out) dst[j] = L[j];
    }
  }
}

// =============================================================================================
// lane kernel: waves arranged WR (along corpus rows) x WQ (along queries); each wave owns NB
// 32-row blocks x BJ 32-query blocks of the workgroup tile (MFMA 32x32: corpus rows are the A
// operand, queries B), so every lane's accumulator columns are BJ queries and the lane keeps
// one partial top-k list per query in registers. The epilogue is lane-local: per 16-row group a
// max and a compare with the lane's threshold for that query; only groups that reach it are
// scanned (staged through a per-lane LDS slot) and inserted. No candidate buffers, atomics or
// barriers, so nothing in the epilogue waits on another wave, and with two workgroups per CU
// one workgroup's epilogue runs beside the other's MFMAs. The 2 * WR partial lists of a query
// (row-waves x lane halves hold disjoint rows) merge once, at the end.
// Operands stream through a buffer LDS-DMA ring of STAGES 32-deep K-steps (64 B per row) that
// runs ahead across corpus-tile boundaries.
// =============================================================================================
namespace lanek {
constexpr int kRowBytes = 64;  // one k-tile of one row: 4 chunks of 16 B

template <int NB, int BJ, int WR, int WQ, int STAGES>
struct Cfg {
  static constexpr int kWaves = WR * WQ;
  static constexpr int kThreads = kWaves * 64;
  static constexpr int kTileRows = 32 * NB * WR;
  static constexpr int kTileQ = 32 * BJ * WQ;
  static constexpr int kParts = 2 * WR;  // partial lists per query
  static constexpr int kStageBytes = (kTileRows + kTileQ) * kRowBytes;
  static constexpr int kLoadsPerWave = (kTileRows + kTileQ) / 16 / kWaves;  // 1-KiB DMA instructions
  static constexpr int kLdsBytes = STAGES * kStageBytes;          // operand ring
  static constexpr int kLdsTotal = kLdsBytes + kThreads * 64;     // + one 16-score slot per lane
  static_assert((kTileRows + kTileQ) % (16 * kWaves) == 0, "tile rows must split evenly over waves");
  static_assert(kLdsTotal <= 160 * 1024, "lane kernel LDS exceeds 160 KiB");
  static_assert(kTileQ * kParts * 16 * 8 <= kLdsTotal, "final list exchange (KCAP <= 16) must fit");
  static_assert(NB * BJ <= 32, "group mask is 32 bits");
};

// 64-B rows: a 256-B bank row holds 4 rows; XOR the chunk with bits 2-3 of the row so the 16
// rows of a ds_read_b128 lane group ({0-3,12-15,20-27} / {4-11,16-19,28-31}) hit 16 distinct
// 16-B slots.
__device__ __forceinline__ int swz(int row, int chunk) { return swz64(row, chunk); }
}  // namespace lanek

template <int DT, int KCAP, int NB, int BJ, int WR, int WQ, int STAGES, int MINB>
__global__ __launch_bounds__(WR * WQ * 64, MINB) void topk_lane_kernel(
    const uint8_t* __restrict__ corpus, const uint8_t* __restrict__ queries, int64_t row_stride,
    int n_rows, int n_q, int n_ktiles, int n_splits, int n_row_tiles, uint32_t row_base, int k_out,
    uint64_t* __restrict__ part_keys, const float* __restrict__ thr_init, int qblocks, int flags) {
  using C = lanek::Cfg<NB, BJ, WR, WQ, STAGES>;
  using lanek::kRowBytes;
  using lanek::swz;
  constexpr int TR = C::kTileRows;
  constexpr int TQ = C::kTileQ;
  constexpr int LPW = C::kLoadsPerWave;
  constexpr int P = C::kParts;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave % WR;
  const int wq = wave / WR;
  const int fr = lane & 31;
  const int fh = lane >> 5;
  int split, qb;
  if (flags & kFlagXcdRemap) {
    const int x = blockIdx.x & 7;
    const int i = blockIdx.x >> 3;
    split = (i / qblocks) * 8 + x;
    qb = i % qblocks;
  } else {
    split = blockIdx.x % n_splits;
    qb = blockIdx.x / n_splits;
  }
  const int q0 = qb * TQ;
  const int t_begin = (int)((int64_t)split * n_row_tiles / n_splits);
  const int t_end = (int)((int64_t)(split + 1) * n_row_tiles / n_splits);
  const int total = (t_end - t_begin) * n_ktiles;

  // this lane's BJ queries, their thresholds (pre-pass seed, then the list's k-th key) and lists
  float thr[BJ];
  uint64_t thk[BJ];
  uint64_t L[BJ][KCAP];
#pragma unroll
  for (int bj = 0; bj < BJ; ++bj) {
    const int q = q0 + wq * BJ * 32 + bj * 32 + fr;
    thr[bj] = q < n_q ? (thr_init ? thr_init[q] : -INFINITY) : INFINITY;
    thk[bj] = (q < n_q && thr[bj] != -INFINITY) ? (((uint64_t)ord_f32(thr[bj]) << 32) - 1) : 0;
#pragma unroll
    for (int j = 0; j < KCAP; ++j) L[bj][j] = 0;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // thr_init reads retired before the ring counts

  // ---- operand ring: the workgroup's (TR + TQ) / 16 1-KiB pieces per K-step, LPW per wave;
  // corpus pieces first (LDS rows 0..TR-1), then query pieces; lane l of a piece lands at
  // (row 16p + l/4, physical chunk l%4) and loads the logical chunk (l%4) ^ swz(row).
  const int ld_row = lane >> 2;
  const uint32_t c_bytes = (uint32_t)(TR * row_stride);
  const __amdgpu_buffer_rsrc_t q_rsrc = tile_rsrc(queries + (int64_t)q0 * row_stride, (uint32_t)(TQ * row_stride));
  uint32_t ld_off[LPW];
#pragma unroll
  for (int j = 0; j < LPW; ++j) {
    const int piece = wave * LPW + j;
    const int row = ((piece < TR / 16) ? piece * 16 : (piece - TR / 16) * 16) + ld_row;
    ld_off[j] = (uint32_t)(row * row_stride) + (((lane & 3) ^ ((row >> 2) & 3)) << 4);
  }
  auto issue = [&](int s) {
    const int t = t_begin + s / n_ktiles;
    const int kt = s - (s / n_ktiles) * n_ktiles;
    unsigned char* buf = smem + (s % STAGES) * C::kStageBytes;
    const __amdgpu_buffer_rsrc_t c_rsrc = tile_rsrc(corpus + (int64_t)t * TR * row_stride, c_bytes);
#pragma unroll
    for (int j = 0; j < LPW; ++j) {
      const int piece = wave * LPW + j;
      blds16(piece < TR / 16 ? c_rsrc : q_rsrc, ld_off[j] + kt * kRowBytes, buf + piece * 16 * kRowBytes);
    }
  };
#pragma unroll
  for (int i = 0; i < STAGES - 1; ++i)
    if (i < total) issue(i);

  f32x16 acc[NB][BJ];
  const int row_w = wr * NB * 32 + 4 * fh;  // + bi*32 + (r&3) + 8*(r>>2)
  // per-lane 64-B slot after the operand ring: a passing 16-row group is staged here so the scan
  // reads its scores with lane-varying LDS addresses instead of register select chains
  float* slot = reinterpret_cast<float*>(smem + C::kLdsBytes) + tid * 16;

  const bool skip_epilogue = (flags & kFlagSkipEpilogue) != 0;
  for (int s = 0; s < total; ++s) {
    // stage s landed; the LPW loads of each later stage already issued may still fly
    if constexpr (STAGES >= 4) {
      if (s + 2 < total) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LPW) : "memory");
      } else if (s + 1 < total) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPW) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else if constexpr (STAGES == 3) {
      if (s + 1 < total) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPW) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    lds_barrier();  // every wave's stage-s data visible; every wave done reading stage s-1
    if (s + STAGES - 1 < total) issue(s + STAGES - 1);
    const int tk = s / n_ktiles;
    const int kt = s - tk * n_ktiles;
    if (kt == 0) {
#pragma unroll
      for (int bi = 0; bi < NB; ++bi)
#pragma unroll
        for (int bj = 0; bj < BJ; ++bj)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[bi][bj][r] = 0.f;
    }
    const unsigned char* buf = smem + (s % STAGES) * C::kStageBytes;
    // Fragment schedule: the NB + BJ reads of k16 step 0, then step 0's MFMAs interleaved with
    // the reads of step 1, then step 1's MFMAs. Reads stay ahead of their MFMAs (counted lgkmcnt
    // waits, at most 15 outstanding: the counter's width) instead of the compiler's
    // register-saving order, where every MFMA waits out an LDS latency.
    u32x4 fa[2][NB], fb[2][BJ];
    auto frag_reads = [&](int g) __attribute__((always_inline)) {
      const int ch = 2 * g + fh;
#pragma unroll
      for (int bj = 0; bj < BJ; ++bj)
        fb[g][bj] = *reinterpret_cast<const u32x4*>(buf + TR * kRowBytes + swz(wq * BJ * 32 + bj * 32 + fr, ch));
#pragma unroll
      for (int bi = 0; bi < NB; ++bi)
        fa[g][bi] = *reinterpret_cast<const u32x4*>(buf + swz(wr * NB * 32 + bi * 32 + fr, ch));
    };
    frag_reads(0);
    __builtin_amdgcn_sched_barrier(0);
    frag_reads(1);
#pragma unroll
    for (int bi = 0; bi < NB; ++bi)
#pragma unroll
      for (int bj = 0; bj < BJ; ++bj) mfma_step<DT>(fa[0][bi], fb[0][bj], acc[bi][bj]);
    if constexpr (DT != DT_F32) {  // f32 steps are 4 MFMAs each: leave those to the scheduler
#pragma unroll
      for (int i = 0; i < (NB * BJ > NB + BJ ? NB * BJ : NB + BJ); ++i) {
        if (i < NB * BJ) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
        if (i < NB + BJ) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // one LDS read
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int bi = 0; bi < NB; ++bi)
#pragma unroll
      for (int bj = 0; bj < BJ; ++bj) mfma_step<DT>(fa[1][bi], fb[1][bj], acc[bi][bj]);
    __builtin_amdgcn_sched_barrier(0);
    if (kt != n_ktiles - 1 || skip_epilogue) continue;

    const int r0 = (t_begin + tk) * TR;
    // ---- lane-local epilogue of corpus tile t_begin + tk: groups (bi, bj) whose max reaches
    // the threshold of query bj
    uint32_t gmask = 0;
#pragma unroll
    for (int bj = 0; bj < BJ; ++bj)
#pragma unroll
      for (int bi = 0; bi < NB; ++bi) {
        float m0 = acc[bi][bj][0], m1 = acc[bi][bj][1];
#pragma unroll
        for (int r = 2; r < 16; r += 2) {
          m0 = fmaxf(m0, acc[bi][bj][r]);
          m1 = fmaxf(m1, acc[bi][bj][r + 1]);
        }
        gmask |= (fmaxf(m0, m1) >= thr[bj] ? 1u : 0u) << (bj * NB + bi);
      }
    if (flags & kFlagMaxOnly) {
      if (gmask == 0xFFFFFFFFu) part_keys[0] = 1;  // keep the maxima live
      continue;
    }
    // One passing group per lane per round: stage it (a static branch per group, taken only
    // where some lane selected it), build its pass mask, then one list_insert per passing
    // score in a divergent loop: the wave pays max-survivors-per-lane inserts.
    while (__ballot(gmask != 0)) {
      const int sel = gmask ? __builtin_ctz(gmask) : -1;
      gmask &= gmask - 1;
#pragma unroll
      for (int bj = 0; bj < BJ; ++bj)
#pragma unroll
        for (int bi = 0; bi < NB; ++bi) {
          if (sel == bj * NB + bi) {
#pragma unroll
            for (int c4 = 0; c4 < 4; ++c4) {
              f32x4 v4 = {acc[bi][bj][4 * c4], acc[bi][bj][4 * c4 + 1], acc[bi][bj][4 * c4 + 2],
                          acc[bi][bj][4 * c4 + 3]};
              *reinterpret_cast<f32x4*>(slot + 4 * c4) = v4;
            }
          }
        }
      if (sel >= 0) {
        const int bjs = sel / NB;
        const int rb = r0 + row_w + (sel - bjs * NB) * 32;
#pragma unroll
        for (int bj = 0; bj < BJ; ++bj) {
          if (bjs != bj) continue;
          uint32_t pm = 0;
#pragma unroll
          for (int c4 = 0; c4 < 4; ++c4) {
            const f32x4 v4 = *reinterpret_cast<const f32x4*>(slot + 4 * c4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int r = 4 * c4 + e;
              pm |= (v4[e] >= thr[bj] && rb + (r & 3) + 8 * (r >> 2) < n_rows ? 1u : 0u) << r;
            }
          }
          bool ins = false;
          while (pm) {
            const int r = __builtin_ctz(pm);
            pm &= pm - 1;
            const uint64_t key = make_key(slot[r], row_base + (uint32_t)(rb + (r & 3) + 8 * (r >> 2)));
            if (key > thk[bj]) {
              list_insert<KCAP>(L[bj], key);
              ins = true;
            }
          }
          if (ins) {
            const uint64_t kth = list_at<KCAP>(L[bj], k_out - 1);
            if (kth > thk[bj]) {
              thk[bj] = kth;
              thr[bj] = key_score(kth);
            }
          }
        }
      }
    }
  }
  if (skip_epilogue) {
    float sink = 0.f;
#pragma unroll
    for (int bi = 0; bi < NB; ++bi)
#pragma unroll
      for (int bj = 0; bj < BJ; ++bj)
#pragma unroll
        for (int r = 0; r < 16; ++r) sink += acc[bi][bj][r];
    if (sink == 1234.5678f) part_keys[0] = 1;
    return;
  }

  // ---- merge the P partial lists of each query (row-waves x lane halves) through LDS
  __syncthreads();  // every wave is done with the operand ring (all DMA retired at the last step)
  uint64_t* xl = reinterpret_cast<uint64_t*>(smem);
  const int part = wr * 2 + fh;
#pragma unroll
  for (int bj = 0; bj < BJ; ++bj) {
    const int ql = wq * BJ * 32 + bj * 32 + fr;
#pragma unroll
    for (int j = 0; j < KCAP; ++j) xl[(ql * P + part) * KCAP + j] = L[bj][j];
  }
  __syncthreads();
  if (tid < TQ && q0 + tid < n_q) {
    uint64_t M[KCAP];
#pragma unroll
    for (int j = 0; j < KCAP; ++j) M[j] = xl[(tid * P) * KCAP + j];
    for (int u = 1; u < P; ++u) {
      const uint64_t* src = xl + (tid * P + u) * KCAP;
      for (int j = 0; j < KCAP; ++j) {
        const uint64_t kk = src[j];
        if (kk <= M[KCAP - 1]) break;  // sorted: nothing further can enter
        list_insert<KCAP>(M, kk);
      }
    }
    uint64_t* dst = part_keys + ((int64_t)(q0 + tid) * n_splits + split) * k_out;
#pragma unroll
    for (int j = 0; j < KCAP; ++j)
      if (j < k_out) dst[j] = M[j];
  }
}

// Merge n_lists sorted key lists per query into the top k. One wave per query: every lane
// folds a strided share into a register list, then k rounds of a wave-wide max pick winners.
template <int KCAP>
__global__ __launch_bounds__(64) void merge_kernel(const uint64_t* __restrict__ in, int n_lists,
                                                   int k_in, int k, float* __restrict__ scores,
                                                   int32_t* __restrict__ rows,
                                                   uint64_t* __restrict__ keys_out) {
  const int q = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t n = (int64_t)n_lists * k_in;
  const uint64_t* src = in + (int64_t)q * n;
  uint64_t L[KCAP];
#pragma unroll
  for (int j = 0; j < KCAP; ++j) L[j] = 0;
  for (int64_t i = lane; i < n; i += 64) list_insert<KCAP>(L, src[i]);
  // lane j keeps output j (k <= 64): one coalesced store per output array at the end instead of a
  // lane-0 store per round
  uint64_t mine = 0;
  for (int j = 0; j < k; ++j) {
    const uint64_t best = wave_max_u64(L[0]);
    if (best != 0 && L[0] == best) {
#pragma unroll
      for (int t = 0; t < KCAP - 1; ++t) L[t] = L[t + 1];
      L[KCAP - 1] = 0;
    }
    mine = lane == j ? best : mine;
  }
  if (lane < k) {
    const int64_t o = (int64_t)q * k + lane;
    if (scores) scores[o] = mine ? key_score(mine) : -INFINITY;
    if (rows) rows[o] = mine ? (int32_t)key_row(mine) : -1;
    if (keys_out) keys_out[o] = mine;
  }
}

// Threshold seed: k-th largest of the G sampled group maxima of each query. Group maxima are
// scores of distinct corpus rows, so the result is a valid lower bound of the query's final
// k-th best score.
constexpr int kSampleMax = 65536;              // sampled rows
constexpr int kGroupMax = kSampleMax / 16;        // group maxima per query

// One wave per query: the k-th largest ordered value is found bit by bit from the MSB
// (largest t with #{v >= t} >= k), one counting pass per bit over NJ values per lane (S <= 64 NJ
// group maxima; the launch picks the smallest NJ: register arrays sized for the largest sample
// made the S = 512 case of the 90k corpus pay 64 guarded loads and ballots per bit, 39 vs 24 us
// for the pre-pass stage at C2).
template <int NJ>
__global__ __launch_bounds__(64) void sample_kth_kernel(const float* __restrict__ scores, int S,
                                                        int k, float* __restrict__ thr) {
  const int q = blockIdx.x;
  const int lane = threadIdx.x;
  const float* src = scores + (int64_t)q * S;
  // all loads in flight at once (clamped addresses, masked after): a per-lane guard around each
  // load serialised them, one memory latency per 64 values
  float raw[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int i = lane + 64 * j;
    raw[j] = src[i < S ? i : S - 1];
  }
  uint32_t v[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) v[j] = lane + 64 * j < S ? ord_f32(raw[j]) : 0u;
  // 20 bits from the MSB (sign, exponent, 11 mantissa bits): ans is the largest 20-bit prefix
  // with #{v >= ans} >= k, so ans <= the k-th largest value: a valid, ~5e-4-relative bound.
  uint32_t ans = 0;
  for (int b = 31; b >= 12; --b) {
    const uint32_t cand = ans | (1u << b);
    // count over the wave with ballots: scalar popcounts, no cross-lane data movement
    int c = 0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) c += __builtin_popcountll(__ballot(v[j] >= cand));
    if (c >= k) ans = cand;
  }
  if (lane == 0) thr[q] = unord_f32(ans);
}

void launch_sample_kth(const float* scores, int B, int G, int k, float* thr, hipStream_t s) {
  if (G <= 8 * 64)
    hipLaunchKernelGGL(sample_kth_kernel<8>, dim3(B), dim3(64), 0, s, scores, G, k, thr);
  else if (G <= 16 * 64)
    hipLaunchKernelGGL(sample_kth_kernel<16>, dim3(B), dim3(64), 0, s, scores, G, k, thr);
  else if (G <= 32 * 64)
    hipLaunchKernelGGL(sample_kth_kernel<32>, dim3(B), dim3(64), 0, s, scores, G, k, thr);
  else
    hipLaunchKernelGGL(sample_kth_kernel<kGroupMax / 64>, dim3(B), dim3(64), 0, s, scores, G, k, thr);
}

// Group maxima of the sampled rows for batches that fill few 128 x 128 tiles (B = 64: 64 tile
// workgroups on 256 CUs, each a 12-k-tile LDS pipeline, 11 us). One wave per (32-row block,
// 32-query block) takes its fragments straight from global memory, NKT k-tiles with six in
// flight, and runs the tile kernel's MFMA chain (same fragments, same k order): its group maxima
// are bitwise topk_tile_kernel<MODE_GROUPMAX>'s, written to the same slots (group 2 rb + fh).
template <int DT, int NKT>
__global__ __launch_bounds__(64) void sample_groupmax_kernel(const uint8_t* __restrict__ corpus,
                                                            const uint8_t* __restrict__ queries,
                                                            int64_t row_stride, int n_q, int n_rb,
                                                            float* __restrict__ score_out, int64_t score_ld) {
  constexpr int kD = NKT < 6 ? NKT : 6;  // k-tiles in flight (a latency-bound wave: 2 in flight per CU at B = 64)
  const int lane = threadIdx.x;
  const int fr = lane & 31;
  const int fh = lane >> 5;
  // ids rb and rb + n_rb (n_rb a multiple of 8) stream the same rows on one XCD
  const int rb = blockIdx.x % n_rb;
  const int qb = blockIdx.x / n_rb;
  const int q = qb * 32 + fr;
  const uint8_t* a_src = corpus + (int64_t)(rb * 32 + fr) * row_stride + fh * 16;
  const uint8_t* b_src = queries + (int64_t)(q < n_q ? q : n_q - 1) * row_stride + fh * 16;
  u32x4 fa[kD][4], fb[kD][4];
  auto load = [&](int slot, int kt) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      fa[slot][g] = *reinterpret_cast<const u32x4*>(a_src + kt * kRowBytes + 32 * g);
      fb[slot][g] = *reinterpret_cast<const u32x4*>(b_src + kt * kRowBytes + 32 * g);
    }
  };
#pragma unroll
  for (int s = 0; s < kD; ++s) load(s, s);
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    const int s = kt % kD;
#pragma unroll
    for (int g = 0; g < 4; ++g) mfma_step<DT>(fa[s][g], fb[s][g], acc);
    if (kt + kD < NKT) load(s, kt + kD);
  }
  float gm = acc[0];
#pragma unroll
  for (int r = 1; r < 16; ++r) gm = fmaxf(gm, acc[r]);
  if (q < n_q) score_out[(int64_t)q * score_ld + 2 * rb + fh] = gm;
}

// true when the wave form took the pre-pass (S rows, a multiple of 256; k-tiles of a built width)
template <int DT>
bool launch_sample_groupmax(const uint8_t* corpus, const uint8_t* queries, int64_t row_stride, int n_ktiles,
                            int S, int B, float* scores, int64_t score_ld, hipStream_t s) {
  static const bool tile_only = [] {  // A/B: AHR_PREPASS_TILE=1 keeps the 128 x 128 tile pre-pass
    const char* e = getenv("AHR_PREPASS_TILE");
    return e && atoi(e) != 0;
  }();
  if (tile_only || S % 256 != 0) return false;
  const int n_rb = S / 32;
  const dim3 grid((unsigned)(n_rb * ((B + 31) / 32)));
  switch (n_ktiles) {
#define AHR_GM_CASE(N)                                                                                            \
  case N:                                                                                                        \
    hipLaunchKernelGGL((sample_groupmax_kernel<DT, N>), grid, dim3(64), 0, s, corpus, queries, row_stride, B, n_rb, \
                       scores, score_ld);                                                                        \
    return true;
    AHR_GM_CASE(4)
    AHR_GM_CASE(6)
    AHR_GM_CASE(8)
    AHR_GM_CASE(12)
    AHR_GM_CASE(16)
    AHR_GM_CASE(24)
#undef AHR_GM_CASE
    default:
      return false;
  }
}

// k-way merge when each lane holds one whole list in registers (n_lists <= 64, k_in <= KCAP):
// no dependent global loads inside the k rounds. One wave per query, 4 queries per 256-thread
// workgroup (B = 1024: 256 workgroups, not 1024 single-wave ones); a list comes in as 16-B loads
// when k_in is even and the input 16-B aligned. A round's wave max runs on the keys' upper halves (the ordered scores: 32-bit
// DPP max) and, only on a tie, on the lower halves of the tied lanes (keys are unique: distinct rows).
template <int KCAP>
__global__ __launch_bounds__(256) void merge_lane_lists_kernel(const uint64_t* __restrict__ in, int n_q,
                                                               int n_lists, int k_in, int k, int vec16,
                                                               float* __restrict__ scores,
                                                               int32_t* __restrict__ rows,
                                                               uint64_t* __restrict__ keys_out) {
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (q >= n_q) return;  // wave-uniform
  const uint64_t* src = in + ((int64_t)q * n_lists + lane) * k_in;
  uint64_t L[KCAP];
  // a list ends at its first empty slot (key 0): the register-resident kernel writes only its kept
  // keys and one terminating 0 (kFlagShortLists), so the slots after it hold another launch's keys
  if (vec16) {  // k_in even, 16-B aligned input
#pragma unroll
    for (int j = 0; j < KCAP; j += 2) {
      u32x4 v = {0u, 0u, 0u, 0u};
      if (lane < n_lists && j < k_in) v = *reinterpret_cast<const u32x4*>(src + j);
      L[j] = ((uint64_t)v[1] << 32) | v[0];
      L[j + 1] = ((uint64_t)v[3] << 32) | v[2];
    }
  } else {
#pragma unroll
    for (int j = 0; j < KCAP; ++j) L[j] = (lane < n_lists && j < k_in) ? src[j] : 0;
  }
  bool end = false;
#pragma unroll
  for (int j = 0; j < KCAP; ++j) {
    end = end || L[j] == 0;
    L[j] = end ? 0 : L[j];
  }
  // lane j keeps output j (k <= 64): one coalesced store per output array at the end instead of a
  // lane-0 store per round
  uint64_t mine = 0;
  for (int j = 0; j < k; ++j) {
    const uint32_t hi = (uint32_t)(L[0] >> 32);
    const uint32_t mh = dpp_max_u32(hi);
    const uint64_t tied = __ballot(hi == mh);
    uint64_t best;
    if (__popcll(tied) == 1) {  // wave-uniform
      best = readlane_u64(L[0], __ffsll((unsigned long long)tied) - 1);
    } else {
      const uint32_t ml = dpp_max_u32(hi == mh ? (uint32_t)L[0] : 0u);
      best = ((uint64_t)mh << 32) | ml;
    }
    if (best != 0 && L[0] == best) {
#pragma unroll
      for (int t = 0; t < KCAP - 1; ++t) L[t] = L[t + 1];
      L[KCAP - 1] = 0;
    }
    mine = lane == j ? best : mine;
  }
  if (lane < k) {
    const int64_t o = (int64_t)q * k + lane;
    if (scores) scores[o] = mine ? key_score(mine) : -INFINITY;
    if (rows) rows[o] = mine ? (int32_t)key_row(mine) : -1;
    if (keys_out) keys_out[o] = mine;
  }
}

// k-way merge of up to 64*kHeadSlots sorted lists: lane l owns lists l, l+64, ...; each round
// the lane offers the best of its list heads, the wave max wins and the owning list advances.
constexpr int kHeadSlots = 8;

__global__ __launch_bounds__(64) void merge_heads_kernel(const uint64_t* __restrict__ in, int n_lists,
                                                         int k_in, int k, float* __restrict__ scores,
                                                         int32_t* __restrict__ rows,
                                                         uint64_t* __restrict__ keys_out) {
  const int q = blockIdx.x;
  const int lane = threadIdx.x;
  const uint64_t* base = in + (int64_t)q * n_lists * k_in;
  uint64_t head[kHeadSlots];
  int ptr[kHeadSlots];
#pragma unroll
  for (int u = 0; u < kHeadSlots; ++u) {
    const int l = lane + 64 * u;
    ptr[u] = 0;
    head[u] = (l < n_lists && k_in > 0) ? base[(int64_t)l * k_in] : 0;
  }
  for (int j = 0; j < k; ++j) {
    uint64_t mine = head[0];
#pragma unroll
    for (int u = 1; u < kHeadSlots; ++u) mine = head[u] > mine ? head[u] : mine;
    const uint64_t best = wave_max_u64(mine);
    if (best != 0 && mine == best) {
#pragma unroll
      for (int u = 0; u < kHeadSlots; ++u) {
        if (head[u] == best) {
          const int l = lane + 64 * u;
          ++ptr[u];
          head[u] = ptr[u] < k_in ? base[(int64_t)l * k_in + ptr[u]] : 0;
        }
      }
    }
    if (lane == 0) {
      const int64_t o = (int64_t)q * k + j;
      if (scores) scores[o] = best ? key_score(best) : -INFINITY;
      if (rows) rows[o] = best ? (int32_t)key_row(best) : -1;
      if (keys_out) keys_out[o] = best;
    }
  }
}

// Exact top-k for k beyond the register lists (AHR_MAX_K < k <= AHR_MAX_K_LARGE) from a score
// row [n] of one query (MODE_SCORES output): one workgroup per query. (1) The k-th largest
// ordered score T by 4 passes of 8-bit radix histograms in LDS, MSB first. (2) One pass in row
// order keeps every score above T and, of those equal to T, the lowest rows (a block-wide
// ordered count), as packed keys. (3) Bitonic sort of the k keys in LDS (score desc, row asc).
constexpr int kLargeK = 4096;

__global__ __launch_bounds__(256) void radix_topk_kernel(const float* __restrict__ scores, int64_t ld, int n,
                                                         int k, uint32_t row_base, float* __restrict__ out_s,
                                                         int32_t* __restrict__ out_r,
                                                         uint64_t* __restrict__ out_keys, int64_t out_q0) {
  __shared__ uint32_t hist[256];
  __shared__ uint64_t sel[kLargeK];
  __shared__ int sh_b, sh_k, sh_eq_seen, sh_n;
  __shared__ int wsum[4];
  const int q = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const float* src = scores + (int64_t)q * ld;
  const int kk0 = k < n ? k : n;
  uint32_t prefix = 0, mask = 0;
  int kk = kk0;  // rank still to be found inside the current prefix bucket (1-based)
  for (int pass = 0; pass < 4 && kk0 > 0; ++pass) {
    const int shift = 24 - 8 * pass;
    hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += 256) {
      const uint32_t u = ord_f32(src[i]);
      if ((u & mask) == prefix) atomicAdd(&hist[(u >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      int cum = 0, b = 255;
      for (; b > 0; --b) {
        if (cum + (int)hist[b] >= kk) break;
        cum += (int)hist[b];
      }
      sh_b = b;
      sh_k = kk - cum;
    }
    __syncthreads();
    prefix |= (uint32_t)sh_b << shift;
    mask |= 255u << shift;
    kk = sh_k;
    __syncthreads();
  }
  // (2) prefix = T (the k-th largest ordered score); kk = how many entries equal to T to keep
  if (tid == 0) {
    sh_eq_seen = 0;
    sh_n = 0;
  }
  __syncthreads();
  for (int base = 0; base < n && kk0 > 0; base += 256) {
    const int i = base + tid;
    uint32_t u = 0;
    float v = 0.f;
    if (i < n) {
      v = src[i];
      u = ord_f32(v);
    }
    const bool eq = i < n && u == prefix;
    // ordered rank of this equal entry among this chunk's equal entries
    const uint64_t bal = __ballot(eq);
    const int wrank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
    if (lane == 0) wsum[wave] = __popcll(bal);
    __syncthreads();
    int before = sh_eq_seen;
    for (int w = 0; w < wave; ++w) before += wsum[w];
    const bool take = (i < n && u > prefix) || (eq && before + wrank < kk);
    if (take) {
      const int pos = atomicAdd(&sh_n, 1);
      sel[pos] = make_key(v, row_base + (uint32_t)i);
    }
    __syncthreads();
    if (tid == 0) sh_eq_seen += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
  // (3) bitonic sort, descending, over the next power of two (zero keys pad at the end)
  int np2 = 1;
  while (np2 < kk0) np2 <<= 1;
  for (int i = kk0 + tid; i < np2; i += 256) sel[i] = 0;
  __syncthreads();
  for (int size = 2; size <= np2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < np2; i += 256) {
        const int j = i ^ stride;
        if (j > i) {
          const uint64_t a = sel[i], b = sel[j];
          const bool desc = (i & size) == 0;
          if (desc ? a < b : a > b) {
            sel[i] = b;
            sel[j] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int j = tid; j < k; j += 256) {
    const uint64_t key = j < kk0 ? sel[j] : 0;
    const int64_t o = (out_q0 + q) * k + j;
    if (out_s) out_s[o] = key ? key_score(key) : -INFINITY;
    if (out_r) out_r[o] = key ? (int32_t)key_row(key) : -1;
    if (out_keys) out_keys[o] = key;
  }
}

// Top-k of packed keys (cross-shard merge for k > AHR_MAX_K): keys are unique (row ids differ),
// so the k-th largest key by 8 passes of 8-bit radix histograms is an exact cut; every key at or
// above it is kept, then bitonic-sorted in LDS. keys_in [B][n] (0 = empty slot).
__global__ __launch_bounds__(256) void radix_topk_keys_kernel(const uint64_t* __restrict__ keys_in, int n, int k,
                                                              float* __restrict__ out_s,
                                                              int32_t* __restrict__ out_r,
                                                              uint64_t* __restrict__ out_keys) {
  __shared__ uint32_t hist[256];
  __shared__ uint64_t sel[kLargeK];
  __shared__ int sh_b, sh_k, sh_n, sh_live;
  const int q = blockIdx.x;
  const int tid = threadIdx.x;
  const uint64_t* src = keys_in + (int64_t)q * n;
  if (tid == 0) {
    sh_live = 0;
    sh_n = 0;
  }
  __syncthreads();
  int live = 0;
  for (int i = tid; i < n; i += 256) live += src[i] != 0;
  atomicAdd(&sh_live, live);
  __syncthreads();
  const int kk0 = k < sh_live ? k : sh_live;
  uint64_t prefix = 0, mask = 0;
  int kk = kk0;
  for (int pass = 0; pass < 8 && kk0 > 0; ++pass) {
    const int shift = 56 - 8 * pass;
    hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += 256) {
      const uint64_t u = src[i];
      if (u && (u & mask) == prefix) atomicAdd(&hist[(u >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      int cum = 0, b = 255;
      for (; b > 0; --b) {
        if (cum + (int)hist[b] >= kk) break;
        cum += (int)hist[b];
      }
      sh_b = b;
      sh_k = kk - cum;
    }
    __syncthreads();
    prefix |= (uint64_t)sh_b << shift;
    mask |= (uint64_t)255 << shift;
    kk = sh_k;
    __syncthreads();
  }
  for (int i = tid; i < n && kk0 > 0; i += 256) {
    const uint64_t u = src[i];
    if (u && u >= prefix) sel[atomicAdd(&sh_n, 1)] = u;
  }
  int np2 = 1;
  while (np2 < kk0) np2 <<= 1;
  __syncthreads();
  for (int i = kk0 + tid; i < np2; i += 256) sel[i] = 0;
  __syncthreads();
  for (int size = 2; size <= np2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < np2; i += 256) {
        const int j = i ^ stride;
        if (j > i) {
          const uint64_t a = sel[i], b = sel[j];
          const bool desc = (i & size) == 0;
          if (desc ? a < b : a > b) {
            sel[i] = b;
            sel[j] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int j = tid; j < k; j += 256) {
    const uint64_t key = j < kk0 ? sel[j] : 0;
    const int64_t o = (int64_t)q * k + j;
    if (out_s) out_s[o] = key ? key_score(key) : -INFINITY;
    if (out_r) out_r[o] = key ? (int32_t)key_row(key) : -1;
    if (out_keys) out_keys[o] = key;
  }
}

__device__ __forceinline__ uint16_t f32_to_bf16_rne(float v) {
  uint32_t u = __float_as_uint(v);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// fp32 storage permutation inside each group of 8: position of logical lane j.
__device__ __forceinline__ int f32_perm(int j) { return (j & ~7) | ((j & 1) << 2) | ((j >> 1) & 3); }

// Fast path of convert_rows_kernel (bf16/f16 rows up to 1024 wide, dim % 4 == 0), one wave per
// row: the whole row in flight at once (clamped addresses, masked after); the general loop waits
// on each 1-KiB piece in turn. Same arithmetic and order as the loop: the per-lane fma chain in j
// order, then the butterfly. `row` may be global or LDS (topk_small_kernel converts its queries
// in place); [0, d_pad) is written in full, zeros past dim.
// frag (optional): also write the register-resident kernel's fragment-major query copy (ahr_qres.h
// launch_frag's layout) for query q.
__device__ __forceinline__ void convert_row_fast(const float* __restrict__ x, int dim, int normalize,
                                                 uint8_t* row, int d_pad, int dt, int lane, uint8_t* frag = nullptr,
                                                 int64_t q = 0) {
  f32x4 v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int j = 4 * lane + 256 * u;
    v[u] = *reinterpret_cast<const f32x4*>(x + (j < dim ? j : dim - 4));
    if (j >= dim) v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float nrm = 1.f;
  if (normalize) {
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      s = fmaf(v[u][0], v[u][0], s); s = fmaf(v[u][1], v[u][1], s);
      s = fmaf(v[u][2], v[u][2], s); s = fmaf(v[u][3], v[u][3], s);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
    nrm = fmaxf(sqrtf(s), 1e-12f);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int j = 4 * lane + 256 * u;
    if (j >= d_pad) break;
    f32x4 w4 = v[u];
    if (normalize) {
#pragma unroll
      for (int e = 0; e < 4; ++e) w4[e] = w4[e] / nrm;
    }
    uint2 w;
    if (dt == DT_BF16) {
      w.x = (uint32_t)f32_to_bf16_rne(w4[0]) | ((uint32_t)f32_to_bf16_rne(w4[1]) << 16);
      w.y = (uint32_t)f32_to_bf16_rne(w4[2]) | ((uint32_t)f32_to_bf16_rne(w4[3]) << 16);
    } else {
      w.x = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)w4[0]) |
            ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)w4[1]) << 16);
      w.y = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)w4[2]) |
            ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)w4[3]) << 16);
    }
    *reinterpret_cast<uint2*>(row + 2 * (int64_t)j) = w;
    if (frag) {  // the 4 elements stay inside one 16-B chunk of the fragment-major copy
      const int64_t o = qres::frag_chunk(q, j, d_pad >> 4) * 16 + (j & 7) * 2;
      *reinterpret_cast<uint2*>(frag + o) = w;
    }
  }
}

// Query conversion for the register-resident plan: the convert kernel's rows (the pre-pass reads
// them) plus the fragment-major copy the qres kernel loads, in one launch (bf16/f16, dim % 4 == 0,
// d_pad <= 1024: convert_row_fast's shape).
__global__ __launch_bounds__(256) void convert_queries_frag_kernel(const float* __restrict__ src, int64_t n, int dim,
                                                                   int normalize, uint8_t* __restrict__ dst,
                                                                   int64_t row_stride, int d_pad, int dt,
                                                                   uint8_t* __restrict__ frag, uint32_t* __restrict__ epoch) {
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + wave;
  if (blockIdx.x == 0 && threadIdx.x == 0 && epoch) advance_epoch_rebalance(epoch);  // the next qres launch's tag
  if (i >= n) return;
  convert_row_fast(src + i * dim, dim, normalize, dst + i * row_stride, d_pad, dt, lane, frag, i);
}

// The register-resident plan's fragment-major query copy straight from the fp32 queries, when
// nothing else reads the row-major copy (self-seeded launches: no pre-pass) and the rows need no
// normalisation: one thread per 16-B chunk of the copy (qres::frag_elem: its query and 8 elements,
// the convert kernel's rounding), so a wave writes one contiguous KiB. The row-major
// convert wrote each 16-B chunk as two 8-B pieces 1 KiB apart, plus the unused rows.
__global__ __launch_bounds__(256) void frag_from_f32_kernel(const float* __restrict__ src, int64_t n, int dim, int d_pad,
                                                            int dt, int64_t n16, uint8_t* __restrict__ frag,
                                                            uint32_t* __restrict__ epoch) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i == 0 && epoch) advance_epoch_rebalance(epoch);  // the next qres launch's tag
  if (i >= n16) return;
  int64_t q;
  int j0;
  qres::frag_elem(i, d_pad >> 4, &q, &j0);
  float v[8];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    f32x4 w = {0.f, 0.f, 0.f, 0.f};
    if (q < n && j0 + 4 * h < dim) w = *reinterpret_cast<const f32x4*>(src + q * dim + j0 + 4 * h);  // dim % 4 == 0
#pragma unroll
    for (int e = 0; e < 4; ++e) v[4 * h + e] = w[e];
  }
  u32x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (dt == DT_BF16)
      o[e] = (uint32_t)f32_to_bf16_rne(v[2 * e]) | ((uint32_t)f32_to_bf16_rne(v[2 * e + 1]) << 16);
    else
      o[e] = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)v[2 * e]) |
             ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)v[2 * e + 1]) << 16);
  }
  *reinterpret_cast<u32x4*>(frag + i * 16) = o;
}

// fp32 rows -> storage rows (one wave per row): optional L2 normalisation, dtype conversion,
// zero padding to d_pad, fp32 lane permutation. Lanes move 4 consecutive elements at a time.
__global__ __launch_bounds__(256) void convert_rows_kernel(const float* __restrict__ src, int64_t n,
                                                           int dim, const int64_t* __restrict__ slots,
                                                           int64_t start, int normalize,
                                                           uint8_t* __restrict__ dst, int64_t row_stride,
                                                           int d_pad, int dt) {
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + wave;
  if (i >= n) return;
  const float* x = src + i * dim;
  const bool vec = (dim & 3) == 0;
  if (vec && d_pad <= 1024 && dt != DT_F32) {
    const int64_t slot = slots ? slots[i] : start + i;
    convert_row_fast(x, dim, normalize, dst + slot * row_stride, d_pad, dt, lane);
    return;
  }
  float nrm = 1.f;
  if (normalize) {
    float s = 0.f;
    if (vec) {
      for (int j = 4 * lane; j < dim; j += 256) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(x + j);
        s = fmaf(v[0], v[0], s); s = fmaf(v[1], v[1], s); s = fmaf(v[2], v[2], s); s = fmaf(v[3], v[3], s);
      }
    } else {
      for (int j = lane; j < dim; j += 64) s = fmaf(x[j], x[j], s);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
    nrm = fmaxf(sqrtf(s), 1e-12f);
  }
  const int64_t slot = slots ? slots[i] : start + i;
  uint8_t* row = dst + slot * row_stride;
  for (int j = 4 * lane; j < d_pad; j += 256) {
    f32x4 v;
    if (vec && j + 3 < dim) {
      v = *reinterpret_cast<const f32x4*>(x + j);
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = (j + u < dim) ? x[j + u] : 0.f;
    }
    if (normalize) {
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = v[u] / nrm;
    }
    if (dt == DT_BF16) {
      uint2 w;
      w.x = (uint32_t)f32_to_bf16_rne(v[0]) | ((uint32_t)f32_to_bf16_rne(v[1]) << 16);
      w.y = (uint32_t)f32_to_bf16_rne(v[2]) | ((uint32_t)f32_to_bf16_rne(v[3]) << 16);
      *reinterpret_cast<uint2*>(row + 2 * (int64_t)j) = w;
    } else if (dt == DT_F16) {
      _Float16* o = reinterpret_cast<_Float16*>(row) + j;
#pragma unroll
      for (int u = 0; u < 4; ++u) o[u] = (_Float16)v[u];
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) reinterpret_cast<float*>(row)[f32_perm(j + u)] = v[u];
    }
  }
}

// Storage rows -> fp32 (inverse of convert_rows_kernel without the normalisation).
__global__ __launch_bounds__(256) void read_rows_kernel(const uint8_t* __restrict__ src, int64_t start,
                                                        int64_t n, int dim, int64_t row_stride, int dt,
                                                        float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const uint8_t* row = src + (start + i) * row_stride;
  for (int j = threadIdx.x & 63; j < dim; j += 64) {
    float v;
    if (dt == DT_BF16) {
      v = __uint_as_float((uint32_t)reinterpret_cast<const uint16_t*>(row)[j] << 16);
    } else if (dt == DT_F16) {
      v = (float)reinterpret_cast<const _Float16*>(row)[j];
    } else {
      v = reinterpret_cast<const float*>(row)[f32_perm(j)];
    }
    out[i * dim + j] = v;
  }
}


// Small-batch fold (B <= kFoldMaxQ): every workgroup of a small-batch launch publishes its
// per-(query, split) lists and arrives on a counter in the query workspace; the LAST to arrive
// merges the n_splits lists of each query (walk_lists_lds) and writes the outputs, so a single
// search() is one launch instead of search + merge_block_kernel (the merge launch and its gap
// were ~7 of ~35 us at B = 1). The counter is reset by that workgroup for the next launch on the
// workspace. lds: n_q * n_splits * k_out keys, then the arrival flag (<= kFoldMaxLds in all; no static LDS: the small
// kernel opts in to 160 KiB of dynamic LDS, which leaves none). Nothing waits: no workgroup depends on another's
// progress, so there is no residency requirement.
constexpr int kFoldMaxQ = 4;
// all queries' lists in LDS at once; beyond 64 KiB the small kernel's workgroups could no longer
// share a CU with the other batch in flight
constexpr int kFoldMaxLds = 64 * 1024;
__device__ __forceinline__ void fold_last_arrival(const uint64_t* part_keys, int n_q, int n_splits, int k_out,
                                                  uint32_t* fold_ctr, float* __restrict__ out_s,
                                                  int32_t* __restrict__ out_r, uint64_t* __restrict__ out_keys,
                                                  uint64_t* lds, int* sh_last) {
  // The lists were stored write-through (agent-scope relaxed stores: past this XCD's L2); each
  // wave waits for its stores' acknowledgement before the barrier, so they are device-visible
  // before the arrival. (An agent-scope fence instead writes back and invalidates the whole L2 in
  // every workgroup: measured 62 vs 35 us per B = 1 search.)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    *sh_last = __hip_atomic_fetch_add(fold_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               (uint32_t)(gridDim.x - 1);
  __syncthreads();
  // sh_last sits past every query's lists (the fill below must not overwrite it while a lagging
  // wave has yet to test it)
  if (!*sh_last) return;
  // Only the last workgroup acquires: one agent-scope acquire fence (cache invalidate) per search,
  // not the release write-back in every workgroup that cost 62 vs 35 us; the lists themselves were
  // written through with agent-scope stores whose acknowledgements were waited for above.
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  // every query's lists at once (read past L2 too: agent scope), then wave q walks query q
  const int n = n_splits * k_out;
  for (int i = threadIdx.x; i < n_q * n; i += blockDim.x)
    lds[i] = __hip_atomic_load(part_keys + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int wave = threadIdx.x >> 6;
  if (wave < n_q) walk_lists_lds(lds + wave * n, n_splits, k_out, k_out, (int64_t)wave * k_out, out_s, out_r, out_keys);
  if (threadIdx.x == 0) __hip_atomic_store(fold_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// =============================================================================================
// topk_small_kernel (B <= 64, bf16/f16, k <= 16): every corpus row is read once and scored
// against at most 64 queries, so the launch is bound by the corpus stream (HBM / MALL), not by
// MFMA (intensity 2 B flop per corpus byte, below the ~315 flop/B ridge), and a 128-query tile
// wastes most of its work. No threshold pre-pass and no LDS staging of the corpus: the query rows
// are converted from fp32 straight into LDS by the workgroup (convert_row_fast: the convert
// kernel's arithmetic, so the same rounded queries), and each wave streams 16-row corpus blocks
// straight into registers as the A operand of v_mfma_f32_16x16x32 (lane l: row l & 15, 16-B chunk
// l / 16 of each 32-deep step, the t256 kernel's fragment map, so the scores are bitwise those of
// its k-ordered chain), one MFMA per 16-query group (NG = 1, 2, 4) per loaded fragment.
// A wave's work is a sequence of (block, 8 k-steps) items in two register sets: the next item's
// loads (the first one before the query staging) fly under the current item's MFMAs and the
// block epilogue; 8 waves per workgroup keep 128 KiB of loads in flight, and two workgroups
// (two batches in flight) fit on a CU.
// Epilogue: lane l holds queries (l & 15) + 16 g at rows 4 (l / 16) + i of the block and keeps a
// register list per query (its k-th key is the threshold); at the end the 4 W lists of each
// query (W waves x 4 lane quarters) merge through LDS, one wave per query, into one list per
// (query, split).
// =============================================================================================
#ifndef AHR_SMALL_WAVES
#define AHR_SMALL_WAVES 8  // waves per workgroup with one query group (A/B builds override)
#endif
#ifndef AHR_SMALL_KC
#define AHR_SMALL_KC 8
#endif
namespace small {
constexpr int kMaxQ = 16;      // one group of 16 queries (the kernel is written for NG groups; only NG = 1 is built)
constexpr int kKC = AHR_SMALL_KC;  // 32-deep k-steps per work item (one register set)
constexpr int kPitchPad = 16;  // query rows in LDS: pitch = row bytes + 16 (conflict-free reads)
// waves per workgroup: 8 (A/B at B = 1 / 16, two batches in flight: 45.1 k / 594 k queries/s
// with 8 waves, 42.9 k / 516 k with 12, 38.2 k / 471 k with 16 — a 16-wave workgroup fills a CU's
// VGPRs, so the other batch's kernel cannot co-reside; serial latency 8 % higher with 8)
__host__ __device__ constexpr int waves(int ng) { return ng == 1 ? AHR_SMALL_WAVES : 8; }
// LDS: the NG * 16 query rows (then, in the DMA form, the line ring: W waves x 2 slots x 8 KiB),
// later overlaid by one group's lane lists (16 x 4 W x KCAP keys)
__host__ __device__ inline int q_region(int64_t row_stride, int ng) {
  return (int)(((int64_t)16 * ng * (row_stride + kPitchPad) + 15) & ~(int64_t)15);
}
inline int lds_bytes(int64_t row_stride, int kcap, int ng, bool dma = false) {
  const int64_t q = q_region(row_stride, ng) + (dma ? (int64_t)waves(ng) * 2 * 8192 : 0);
  const int64_t l = (int64_t)16 * 4 * waves(ng) * kcap * 8;
  return (int)(q > l ? q : l);
}
// the DMA form (A/B: AHR_SMALL_DMA=1, the ablation build only: not the default, so not shipped)
// where it fits 160 KiB of LDS
inline bool use_dma(int64_t row_stride, int ng) {
  if (!kAblation) return false;
  static const bool on = [] {
    const char* e = getenv("AHR_SMALL_DMA");
    return e && atoi(e) != 0;
  }();
  return on && ng == 1 && q_region(row_stride, ng) + waves(ng) * 2 * 8192 <= 160 * 1024;
}
}  // namespace small

template <int DT, int KCAP, int NG, bool DMA>
__global__ __launch_bounds__(small::waves(NG) * 64, 1) void topk_small_kernel(
    const uint8_t* __restrict__ corpus, const float* __restrict__ qsrc, int dim, int normalize,
    const uint8_t* __restrict__ qconv, int64_t row_stride, int d_pad, int n_rows, int n_q, int n_steps,
    int n_splits, uint32_t row_base, int k_out, uint64_t* __restrict__ part_keys, uint32_t* __restrict__ fold_ctr,
    float* __restrict__ out_s, int32_t* __restrict__ out_r, uint64_t* __restrict__ out_keys) {
  static_assert(DT != DT_F32, "fp32 keeps the exact single-chain kernels");
  constexpr int W = small::waves(NG);
  constexpr int kThreads = W * 64;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int fr = lane & 15;
  const int fq = lane >> 4;
  const int split = blockIdx.x;
  const int pitch = (int)row_stride + small::kPitchPad;

  // the split's rows [r_begin, r_end): an equal share of the corpus, in 16-row blocks from r_begin
  // (the last one may be partial: its rows past the split load the split's last row, unused)
  const int r_begin = (int)((int64_t)split * n_rows / n_splits);
  const int r_end = (int)((int64_t)(split + 1) * n_rows / n_splits);
  const int b_end = (r_end - r_begin + 15) >> 4;
  // the wave's work is a sequence of items (16-row block, 8 k-steps); two register sets keep the
  // next item's loads in flight under the current item's MFMAs, across block boundaries
  // Every load is unconditional (steps past the row clamp to its last step; a finished wave
  // re-reads its current item, an L2 hit) so that every path through the loop issues the same
  // loads: with a conditional load the compiler's waitcnt placement must assume the younger item
  // may not be in flight and waits vmcnt(0) before each MFMA, i.e. for the NEXT item's loads too,
  // which serialises the stream on one memory latency per item.
  // DMA form (AHR_SMALL_DMA=1, one workgroup per CU): an item (16 rows x 8 steps x 64 B) comes in
  // by LDS-DMA as 8 wave-instructions of 2 rows x 512 B each into a two-slot per-wave ring after
  // the query rows (row-major, 16-B chunk c of a row at position c ^ (row & 15): the fragment
  // reads below are conflict-free); the register form's loads touch 16 half-lines per instruction.
  unsigned char* ring = smem + small::q_region(row_stride, NG) + wave * (2 * 8192);
  auto dma_item = [&](int sl, int blk, int s0) __attribute__((always_inline)) {
    const int r0 = r_begin + blk * 16;
    const int rows_here = min(16, r_end - r0);  // rows past the split read as zeros
    const __amdgpu_buffer_rsrc_t r = tile_rsrc_u(corpus + (int64_t)r0 * row_stride, (uint32_t)(rows_here * row_stride));
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = 2 * j + (lane >> 5);
      const uint32_t off = (uint32_t)(row * row_stride) + s0 * 64 + (((lane & 31) ^ (row & 15)) << 4);
      blds16(r, off, ring + sl * 8192 + j * 1024);
    }
  };
  int slot = 0;
  auto load_item = [&](u32x4 (&A)[small::kKC], int blk, int s0) __attribute__((always_inline)) {
    const uint8_t* arow = corpus + (int64_t)min(r_begin + blk * 16 + fr, r_end - 1) * row_stride + fq * 16;
#pragma unroll
    for (int j = 0; j < small::kKC; ++j) {
      const int st = s0 + j < n_steps ? s0 + j : n_steps - 1;
      A[j] = *reinterpret_cast<const u32x4*>(arow + st * 64);
    }
  };
  u32x4 A0[small::kKC], A1[small::kKC];
  int cb = wave, cs = 0;
  if (cb < b_end) {  // in flight while the queries are staged
    if constexpr (DMA)
      dma_item(0, cb, 0);
    else
      load_item(A0, cb, 0);
  }

  // queries into LDS: converted from fp32 here (wave w: queries w, w + W, ...), or copied from
  // the query buffer
  if (qsrc) {
    for (int r = wave; r < n_q; r += W)
      convert_row_fast(qsrc + (int64_t)r * dim, dim, normalize, smem + r * pitch, d_pad, DT, lane);
  } else {
    const int chunks = (int)(row_stride >> 4);
    for (int i = tid; i < n_q * chunks; i += kThreads) {
      const int r = i / chunks;
      const int c = i - r * chunks;
      *reinterpret_cast<u32x4*>(smem + r * pitch + c * 16) =
          *reinterpret_cast<const u32x4*>(qconv + (int64_t)r * row_stride + c * 16);
    }
  }
  __syncthreads();

  // lane: queries fr + 16 g (g < NG), rows 4 fq + i of each block
  uint64_t L[NG][KCAP];
  uint64_t thk[NG];  // the list's k-th key (0 while it holds fewer than k)
  float thr[NG];
  f32x4 acc[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
#pragma unroll
    for (int j = 0; j < KCAP; ++j) L[g][j] = 0;
    thk[g] = 0;
    thr[g] = fr + 16 * g < n_q ? -INFINITY : INFINITY;  // columns past n_q never pass
    acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const unsigned char* qrow = smem + fr * pitch + fq * 16;
  // one item: issue the next item's loads into N, MFMAs over C, the block's epilogue after its
  // last item; returns false when the wave is done
  auto step = [&](u32x4 (&C)[small::kKC], u32x4 (&N)[small::kKC]) __attribute__((always_inline)) {
    int nb = cb, ns = cs + small::kKC;
    if (ns >= n_steps) {
      ns = 0;
      nb += W;
    }
    {
      const bool more = nb < b_end;
      if constexpr (DMA) {
        asm volatile("" ::: "memory");  // the slot's reads of the previous step are consumed
        dma_item(slot ^ 1, more ? nb : cb, more ? ns : cs);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this slot landed, the next one in flight
        const unsigned char* src = ring + slot * 8192 + fr * 512;
#pragma unroll
        for (int j = 0; j < small::kKC; ++j) C[j] = *reinterpret_cast<const u32x4*>(src + (((j * 4 + fq) ^ fr) << 4));
      } else {
        load_item(N, more ? nb : cb, more ? ns : cs);
      }
    }
#pragma unroll
    for (int j = 0; j < small::kKC; ++j) {
      // steps past the row: a zero operand (mask, not a branch) against a valid query step
      const uint32_t m = cs + j < n_steps ? 0xFFFFFFFFu : 0u;
      const int st = cs + j < n_steps ? cs + j : n_steps - 1;
      const u32x4 a = {C[j][0] & m, C[j][1] & m, C[j][2] & m, C[j][3] & m};
#pragma unroll
      for (int g = 0; g < NG; ++g)
        mfma16(a, *reinterpret_cast<const u32x4*>(qrow + 16 * g * pitch + st * 64), acc[g], DT);
    }
    if (ns == 0) {
      const int r0 = r_begin + cb * 16 + 4 * fq;
#pragma unroll
      for (int g = 0; g < NG; ++g) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (acc[g][i] >= thr[g] && r0 + i < r_end) {
            const uint64_t key = make_key(acc[g][i], row_base + (uint32_t)(r0 + i));
            if (key > thk[g]) {
              list_insert<KCAP>(L[g], key);
              thk[g] = list_at<KCAP>(L[g], k_out - 1);
              thr[g] = thk[g] ? key_score(thk[g]) : -INFINITY;
            }
          }
        }
        acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    cb = nb;
    cs = ns;
    slot ^= 1;
    return cb < b_end;
  };
  if (cb < b_end) {
    if constexpr (DMA) {
      while (step(A0, A0)) {
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the finished wave's redundant item
    } else {
      while (step(A0, A1) && step(A1, A0)) {
      }
    }
  }

  // per group: 4 W lists per query -> LDS [query][wave * 4 + quarter][KCAP] -> one wave per
  // query merges them (k rounds of a DPP wave max) into one list per (query, split)
  uint64_t* lists = reinterpret_cast<uint64_t*>(smem);
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    if (16 * g >= n_q) break;  // uniform
    __syncthreads();  // queries (g = 0) or the previous group's lists are no longer read
    if (fr + 16 * g < n_q) {
      uint64_t* dst = lists + ((int64_t)fr * (4 * W) + wave * 4 + fq) * KCAP;
#pragma unroll
      for (int j = 0; j < KCAP; ++j) dst[j] = L[g][j];
    }
    __syncthreads();
    for (int ql = wave; ql < 16; ql += W) {
      const int q = 16 * g + ql;
      if (q >= n_q) break;
      uint64_t M[KCAP];
#pragma unroll
      for (int j = 0; j < KCAP; ++j) M[j] = lane < 4 * W ? lists[((int64_t)ql * (4 * W) + lane) * KCAP + j] : 0;
      uint64_t mine = 0;  // lane j keeps the j-th winner
      for (int j = 0; j < k_out; ++j) {
        const uint64_t best = wave_max_u64(M[0]);
        if (best != 0 && M[0] == best) {
#pragma unroll
          for (int t = 0; t < KCAP - 1; ++t) M[t] = M[t + 1];
          M[KCAP - 1] = 0;
        }
        if (lane == j) mine = best;
      }
      if (lane < k_out)  // write-through: the fold's last workgroup may read it
        __hip_atomic_store(part_keys + ((int64_t)q * n_splits + split) * k_out + lane, mine, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (fold_ctr)  // B <= kFoldMaxQ: the last workgroup merges the splits (no merge launch)
    fold_last_arrival(part_keys, n_q, n_splits, k_out, fold_ctr, out_s, out_r, out_keys, lists,
                      reinterpret_cast<int*>(lists + (int64_t)n_q * n_splits * k_out));
}

// topk_small_f32_kernel (fp32 exact mode, B <= 4, k <= 16): the small-batch stream for the
// drop-in search's fp32 index. The exact-mode contract is one fmaf chain per (row, query) in
// increasing k, so one lane owns one corpus row of a 64-row item and runs the chain on the VALU
// (B <= 4 queries: <= 4 fmas per loaded float, far below the stream's cost); the stored (evens |
// odds) permutation of each group of 8 is undone by the order of the fmas. Loads: a step is one
// 128-B line of the item's 64 rows, brought in by LDS-DMA as whole lines (8 rows per
// wave-instruction) into a two-slot per-wave ring, the next step's line in flight under the
// current fmas; each lane then reads its own row's line from the slot (swizzled, conflict-free).
// The round-1 form (per-lane 16-B register loads: 64 lines per instruction) stays behind
// AHR_F32_SLOTS=0 for A/B. One workgroup per CU (up to 256 splits; ~5.5 items per split at C2).
// Queries (the convert kernel's permuted fp32 rows) are broadcast reads from LDS. Each lane keeps
// a register list per query; at the end every wave reduces its 64 lane lists (k rounds of a DPP
// wave max) and one wave merges the 8 wave lists through LDS into one list per (query, split).
namespace smallf32 {
constexpr int kWaves = 8;
constexpr int kMaxQ = 4;
// lines of the ring per wave: 0 = per-lane register loads (two register sets), 2 = LDS-DMA slots
// of one 64-row x 128-B line image each (8 KiB). (3 slots, 6 waves: measured equal to 2 at B = 1;
// the kernel is written for any depth, only 0 and 2 are built.)
__host__ __device__ constexpr int waves_for(int slots) { return slots == 3 ? 6 : kWaves; }
__host__ __device__ constexpr int ring_bytes(int slots) { return slots ? waves_for(slots) * slots * 8192 : 0; }
// A/B knobs: AHR_F32_SLOTS (0 or 2), AHR_F32_WPS = busy waves per workgroup the split count aims at
// (1: up to 256 workgroups, one per CU; 8: the round-1 geometry)
inline int env_int(const char* name, int dflt, int lo, int hi) {
  const char* e = getenv(name);
  return e ? std::max(lo, std::min(hi, atoi(e))) : dflt;
}
inline int slots() {  // (the register form, 0, is compiled into the ablation build only)
  static const int v = env_int("AHR_F32_SLOTS", 2, 0, 2);
  return kAblation && v == 0 ? 0 : 2;
}
inline int waves_per_split() {
  static const int w = env_int("AHR_F32_WPS", 1, 1, kWaves);
  return w;
}
}  // namespace smallf32

template <int KCAP, int NQ, int SLOTS>
__global__ __launch_bounds__(smallf32::waves_for(SLOTS) * 64, 1) void topk_small_f32_kernel(
    const uint8_t* __restrict__ corpus, const float* __restrict__ qsrc, int dim, int normalize,
    const uint8_t* __restrict__ qconv, int64_t row_stride, int n_rows, int n_q,
    int n_lines, int n_splits, uint32_t row_base, int k_out, uint64_t* __restrict__ part_keys,
    uint32_t* __restrict__ fold_ctr, float* __restrict__ out_s, int32_t* __restrict__ out_r,
    uint64_t* __restrict__ out_keys) {
  constexpr int W = smallf32::waves_for(SLOTS);
  constexpr bool DMA = SLOTS != 0;
  __shared__ __attribute__((aligned(16))) float qs[NQ * 1024];  // d_pad <= 1024
  __shared__ uint64_t wl[NQ][W][KCAP];
  // DMA form: the line ring (W waves x SLOTS x 8 KiB), later overlaid by the fold's lists
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int split = blockIdx.x;
  // the split's rows [r_begin, r_end): an equal share of the corpus (not whole 64-row items, so
  // every CU streams the same bytes; the split's last item may be partial); items are local
  const int r_begin = (int)((int64_t)split * n_rows / n_splits);
  const int r_end = (int)((int64_t)(split + 1) * n_rows / n_splits);
  const int i_end = (r_end - r_begin + 63) >> 6;
  const int d_pad = (int)(row_stride >> 2);

  u32x4 A0[8], A1[8];
  int ci = wave, cl = 0;  // current item, current 128-B line of the row
  auto load_line = [&](u32x4 (&A)[8], int item, int line) __attribute__((always_inline)) {
    const int row = min(r_begin + item * 64 + lane, r_end - 1);  // past the split: its last row, unused
    const u32x4* src = reinterpret_cast<const u32x4*>(corpus + (int64_t)row * row_stride + line * 128);
#pragma unroll
    for (int j = 0; j < 8; ++j) A[j] = src[j];
  };
  // DMA form: a line of the item's 64 rows comes in as 8 wave-instructions of 8 whole 128-B lines
  // each (lane 8a + b of instruction j: row 8j + a, 16-B chunk b ^ s(row), s(r) = (r >> 1) & 7),
  // landing row-major in the wave's slot; lane r then reads its row's chunk c at position c ^ s(r),
  // conflict-free (each 16-lane ds_read_b128 group covers 16 distinct 16-B bank slots). Per-lane
  // register loads touch 64 lines per instruction, 16 B each, and need every line to stay in L1
  // across the 8 instructions of a step.
  unsigned char* ring = dyn_smem + wave * (SLOTS * 8192);
  auto dma_line = [&](int slot, int item, int line) __attribute__((always_inline)) {
    const int r0 = r_begin + item * 64;
    const int rows_here = min(64, r_end - r0);  // rows past the split read as zeros
    const __amdgpu_buffer_rsrc_t r =
        tile_rsrc_u(corpus + (int64_t)r0 * row_stride, (uint32_t)(rows_here * row_stride));
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = 8 * j + (lane >> 3);
      const uint32_t off = (uint32_t)(row * row_stride) + line * 128 + (((lane & 7) ^ ((row >> 1) & 7)) << 4);
      blds16(r, off, ring + slot * 8192 + j * 1024);
    }
  };
  // DMA: the fetch cursor runs SLOTS - 1 lines ahead of the current line; past the wave's last
  // item it re-fetches the current line (every step issues the same 8 DMAs: counted vmcnt waits)
  int slot = 0, fi = ci, fl = 0;
  auto advance = [&](int& i, int& l) __attribute__((always_inline)) {
    if (++l >= n_lines) {
      l = 0;
      i += W;
    }
  };
  if (ci < i_end) {
    if constexpr (DMA) {
#pragma unroll
      for (int t = 0; t < SLOTS - 1; ++t) {
        const bool ok = fi < i_end;
        dma_line(t, ok ? fi : ci, ok ? fl : 0);
        advance(fi, fl);
      }
    } else {
      load_line(A0, ci, 0);
    }
  }
  if (qsrc) {  // queries converted here (wave r: query r), convert_rows_kernel's fp32 arithmetic
    for (int r = wave; r < n_q; r += W) {
      const float* x = qsrc + (int64_t)r * dim;
      const bool vec = (dim & 3) == 0;
      float nrm = 1.f;
      if (normalize) {
        float sq = 0.f;
        if (vec) {
          for (int j = 4 * lane; j < dim; j += 256) {
            const f32x4 v = *reinterpret_cast<const f32x4*>(x + j);
            sq = fmaf(v[0], v[0], sq); sq = fmaf(v[1], v[1], sq); sq = fmaf(v[2], v[2], sq); sq = fmaf(v[3], v[3], sq);
          }
        } else {
          for (int j = lane; j < dim; j += 64) sq = fmaf(x[j], x[j], sq);
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) sq += __shfl_xor(sq, off, 64);
        nrm = fmaxf(sqrtf(sq), 1e-12f);
      }
      for (int j = 4 * lane; j < d_pad; j += 256) {
        f32x4 v;
        if (vec && j + 3 < dim) {
          v = *reinterpret_cast<const f32x4*>(x + j);
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u) v[u] = (j + u < dim) ? x[j + u] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) qs[r * 1024 + f32_perm(j + u)] = normalize ? v[u] / nrm : v[u];
      }
    }
  } else {
    for (int i = tid; i < n_q * d_pad / 4; i += W * 64) {
      const int r = i / (d_pad / 4);
      const int c = i - r * (d_pad / 4);
      reinterpret_cast<f32x4*>(qs)[r * 256 + c] = *reinterpret_cast<const f32x4*>(qconv + (int64_t)r * row_stride + c * 16);
    }
  }
  __syncthreads();

  uint64_t L[NQ][KCAP];
  uint64_t thk[NQ];
  float acc[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
#pragma unroll
    for (int j = 0; j < KCAP; ++j) L[q][j] = 0;
    thk[q] = 0;
    acc[q] = 0.f;
  }
  auto step = [&](u32x4 (&C)[8], u32x4 (&N)[8]) __attribute__((always_inline)) {
    int ni = ci, nl = cl + 1;
    if (nl >= n_lines) {
      nl = 0;
      ni += W;
    }
    {  // unconditional (a finished wave re-reads its current line): see topk_small_kernel
      const bool more = ni < i_end;
      if constexpr (DMA) {
        asm volatile("" ::: "memory");  // the slot's reads of the previous step are consumed
        const bool ok = fi < i_end;
        int ws = slot + SLOTS - 1;
        ws = ws >= SLOTS ? ws - SLOTS : ws;
        dma_line(ws, ok ? fi : ci, ok ? fl : cl);
        advance(fi, fl);
        // this slot's 8 landed, the younger 8 (SLOTS - 1) in flight
        if constexpr (SLOTS == 2)
          asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        const unsigned char* src = ring + slot * 8192 + lane * 128;
        const int sw = (lane >> 1) & 7;
#pragma unroll
        for (int c = 0; c < 8; ++c) C[c] = *reinterpret_cast<const u32x4*>(src + ((c ^ sw) << 4));
      } else {
        load_line(N, more ? ni : ci, more ? nl : cl);
      }
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {  // 4 groups of 8 per line
      const f32x4 lo = __builtin_bit_cast(f32x4, C[2 * g]);
      const f32x4 hi = __builtin_bit_cast(f32x4, C[2 * g + 1]);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        if (q < n_q) {
          const float* qp = qs + q * 1024 + cl * 32 + g * 8;
          const f32x4 qlo = *reinterpret_cast<const f32x4*>(qp);
          const f32x4 qhi = *reinterpret_cast<const f32x4*>(qp + 4);
          // logical k order 8g + 0..7 = stored positions 0, 4, 1, 5, 2, 6, 3, 7
          float a = acc[q];
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            a = fmaf(lo[m], qlo[m], a);
            a = fmaf(hi[m], qhi[m], a);
          }
          acc[q] = a;
        }
      }
    }
    if (nl == 0) {
      const int row = r_begin + ci * 64 + lane;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        if (q < n_q && row < r_end) {
          const uint64_t key = make_key(acc[q], row_base + (uint32_t)row);
          if (key > thk[q]) {
            list_insert<KCAP>(L[q], key);
            thk[q] = list_at<KCAP>(L[q], k_out - 1);
          }
        }
        acc[q] = 0.f;
      }
    }
    ci = ni;
    cl = nl;
    slot = slot + 1 == SLOTS ? 0 : slot + 1;
    return ci < i_end;
  };
  if (ci < i_end) {
    if constexpr (DMA) {
      while (step(A0, A0)) {
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the finished wave's redundant line
    } else {
      while (step(A0, A1) && step(A1, A0)) {
      }
    }
  }
  // per query: the wave's 64 lane lists -> one list (k rounds of a wave max) -> LDS; wave 0
  // merges the W wave lists
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    if (q >= n_q) break;
    uint64_t mine = 0;
    for (int j = 0; j < k_out; ++j) {
      const uint64_t best = wave_max_u64(L[q][0]);
      if (best != 0 && L[q][0] == best) {
#pragma unroll
        for (int t = 0; t < KCAP - 1; ++t) L[q][t] = L[q][t + 1];
        L[q][KCAP - 1] = 0;
      }
      if (lane == j) mine = best;
    }
    if (lane < KCAP) wl[q][wave][lane] = lane < k_out ? mine : 0;
  }
  __syncthreads();
  if (wave == 0) {
    for (int q = 0; q < n_q; ++q) {
      uint64_t M[KCAP];
#pragma unroll
      for (int j = 0; j < KCAP; ++j) M[j] = lane < W ? wl[q][lane][j] : 0;
      uint64_t mine = 0;
      for (int j = 0; j < k_out; ++j) {
        const uint64_t best = wave_max_u64(M[0]);
        if (best != 0 && M[0] == best) {
#pragma unroll
          for (int t = 0; t < KCAP - 1; ++t) M[t] = M[t + 1];
          M[KCAP - 1] = 0;
        }
        if (lane == j) mine = best;
      }
      if (lane < k_out)  // write-through: the fold's last workgroup may read it
        __hip_atomic_store(part_keys + ((int64_t)q * n_splits + split) * k_out + lane, mine, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (fold_ctr) {  // the last workgroup merges the splits (no merge launch)
    uint64_t* fl = reinterpret_cast<uint64_t*>(dyn_smem);
    fold_last_arrival(part_keys, n_q, n_splits, k_out, fold_ctr, out_s, out_r, out_keys, fl,
                      reinterpret_cast<int*>(fl + (int64_t)n_q * n_splits * k_out));
  }
}

// k-way merge of up to 512 sorted lists per query (n_lists * k_in <= 8192), one 256-thread
// workgroup per query: every key comes into LDS with coalesced loads in one go (a head-advancing
// merge over global memory pays one dependent L2 latency per output), then one wave takes k
// rounds of a DPP wave max over the list heads held in registers (lane l owns lists l + 64 u),
// advancing a head with an LDS read: no barrier per output.
constexpr int kMergeBlockKeys = 8192;
__global__ __launch_bounds__(256) void merge_block_kernel(const uint64_t* __restrict__ in, int n_lists, int k_in,
                                                          int k, float* __restrict__ scores,
                                                          int32_t* __restrict__ rows,
                                                          uint64_t* __restrict__ keys_out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint64_t* kb = reinterpret_cast<uint64_t*>(smem);
  const int q = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int n = n_lists * k_in;
  const uint64_t* src = in + (int64_t)q * n;
  // all loads in flight at once: a load -> LDS store loop waits one L2 latency per iteration
  constexpr int kPer = kMergeBlockKeys / 256;
  uint64_t v[kPer];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int i = tid + 256 * u;
    if (256 * u < n) v[u] = src[i < n ? i : n - 1];  // 256 u < n is block-uniform
  }
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int i = tid + 256 * u;
    if (i < n) kb[i] = v[u];
  }
  __syncthreads();
  if (wave != 0) return;
  walk_lists_lds(kb, n_lists, k_in, k, (int64_t)q * k, scores, rows, keys_out);
}

// Cluster-probe seed (ahr_index_probe_seed): per query, the exact scores of the rows of its
// nearest clusters (cluster ids from a centroid search, packed keys [B][P]), walked in order until
// at least min_rows rows are gathered; the seed is the k-th largest per-row LOWER BOUND of the
// score the fused kernels compute for that row: score - err, err = sum |q_i c_i| * (2^-8 for bf16
// storage / 2^-10 for f16: the kernels score the storage-rounded query, this kernel the fp32 one;
// + dim * 2^-23: two fp32 summation orders). Any k real rows give a valid lower bound of the final
// k-th best, so the seed admits every true top-k row; with clusters that hold the query's
// neighbours it sits just under the k-th best (~18 survivors per query at C2 instead of ~110 from
// the sampled pre-pass). Fewer than k rows gathered: -inf (no pruning for that query).
// One 256-thread workgroup per query; every wave holds the fp32 query in registers (lane: dims
// 4 lane + 256 u) and scores a quarter of the rows, kProbeBatch rows' loads in flight at once.
constexpr int kProbeMaxRows = 256;
constexpr int kProbeMaxDim = 1024;
constexpr int kProbeBatch = 8;

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_f32(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, ROW_MASK, 0xf, false));
}
// wave64 sum by DPP row shifts + row broadcasts (as wave_max_u64); the result in every lane
__device__ __forceinline__ float wave_sum_f32(float x) {
  x += dpp_f32<0x111, 0xf>(x);
  x += dpp_f32<0x112, 0xf>(x);
  x += dpp_f32<0x114, 0xf>(x);
  x += dpp_f32<0x118, 0xf>(x);
  x += dpp_f32<0x142, 0xa>(x);
  x += dpp_f32<0x143, 0xc>(x);
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
}

__global__ __launch_bounds__(256, 2) void probe_seed_kernel(const uint8_t* __restrict__ corpus, int64_t row_stride,
                                                            int dt, int dim, int64_t n_rows,
                                                            const float* __restrict__ qsrc, int normalize,
                                                            const uint64_t* __restrict__ ckeys, int P,
                                                            const int64_t* __restrict__ list_off,
                                                            const int32_t* __restrict__ list_rows, int min_rows,
                                                            int k, float* __restrict__ thr) {
  __shared__ int32_t cand[kProbeMaxRows];
  __shared__ float lb[kProbeMaxRows];
  __shared__ int64_t cl_off[64];
  __shared__ int cl_start[65];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  // the query, whole, in every wave's registers
  const float* x = qsrc + (int64_t)b * dim;
  float qv[4][4];
  float ss = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int j = 4 * lane + 256 * u + e;
      qv[u][e] = j < dim ? x[j] : 0.f;
      ss = fmaf(qv[u][e], qv[u][e], ss);
    }
  // the nearest clusters' list ranges (wave 0, lane j = cluster j; P <= 64), taken in order while
  // fewer than min_rows rows are held
  if (wave == 0) {
    int64_t o0 = 0;
    int nj = 0;
    if (lane < P) {
      const uint64_t key = ckeys[(int64_t)b * P + lane];
      if (key) {
        const int c = (int)key_row(key);
        o0 = list_off[c];
        nj = (int)(list_off[c + 1] - o0);
      }
    }
    int incl = nj;  // inclusive prefix sum over the lanes
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int v = __shfl_up(incl, off, 64);
      if (lane >= off) incl += v;
    }
    const int excl = incl - nj;
    const bool take = lane < P && excl < min_rows;
    cl_off[lane] = o0;
    cl_start[lane] = take ? (excl < kProbeMaxRows ? excl : kProbeMaxRows) : kProbeMaxRows;
    const uint64_t tk = __ballot(take);
    const int last = tk ? 63 - __builtin_clzll(tk) : -1;
    const int total = last >= 0 ? __shfl(incl, last, 64) : 0;
    if (lane == 0) cl_start[64] = total < kProbeMaxRows ? total : kProbeMaxRows;
  }
  if (normalize) {
    const float inv = 1.0f / fmaxf(sqrtf(wave_sum_f32(ss)), 1e-12f);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) qv[u][e] *= inv;
  }
  __syncthreads();
  const int n = cl_start[64];
  for (int i = tid; i < n; i += 256) {
    int j = 0;
    while (j + 1 < 64 && cl_start[j + 1] <= i) ++j;  // clusters are few and in order
    const int32_t r = list_rows[cl_off[j] + (i - cl_start[j])];
    cand[i] = (r >= 0 && r < n_rows) ? r : -1;
  }
  __syncthreads();
  const float rel = (dt == DT_BF16 ? 0x1p-8f : 0x1p-10f) + (float)dim * 0x1p-23f;
  const int w_begin = wave * n / 4, w_end = (wave + 1) * n / 4;
  for (int i0 = w_begin; i0 < w_end; i0 += kProbeBatch) {
    uint2 raw[kProbeBatch][4];
#pragma unroll
    for (int rr = 0; rr < kProbeBatch; ++rr) {
      const int i = i0 + rr < w_end ? i0 + rr : i0;
      const int32_t r = cand[i];
      const uint8_t* row = corpus + (int64_t)(r < 0 ? 0 : r) * row_stride;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int j = 4 * lane + 256 * u;
        raw[rr][u] = j < dim ? *reinterpret_cast<const uint2*>(row + 2 * j) : make_uint2(0, 0);
      }
    }
#pragma unroll
    for (int rr = 0; rr < kProbeBatch; ++rr) {
      float sc = 0.f, ab = 0.f;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t w[2] = {raw[rr][u].x, raw[rr][u].y};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint16_t h = (uint16_t)(w[e >> 1] >> (16 * (e & 1)));
          const float c = dt == DT_BF16 ? __uint_as_float((uint32_t)h << 16)
                                        : (float)__builtin_bit_cast(_Float16, h);
          sc = fmaf(qv[u][e], c, sc);
          ab = fmaf(fabsf(qv[u][e]), fabsf(c), ab);
        }
      }
      sc = wave_sum_f32(sc);
      ab = wave_sum_f32(ab);
      if (lane == 0 && i0 + rr < w_end) lb[i0 + rr] = cand[i0 + rr] < 0 ? -INFINITY : sc - ab * rel;
    }
  }
  __syncthreads();
  if (wave != 0) return;
  if (n < k) {
    if (lane == 0) thr[b] = -INFINITY;
    return;
  }
  // k-th largest lower bound: the largest 20-bit ordered prefix with >= k values at or above it
  uint32_t v[kProbeMaxRows / 64];
#pragma unroll
  for (int u = 0; u < kProbeMaxRows / 64; ++u) {
    const int i = lane + 64 * u;
    v[u] = i < n ? ord_f32(lb[i]) : 0u;
  }
  uint32_t ans = 0;
  for (int bit = 31; bit >= 12; --bit) {
    const uint32_t cand_v = ans | (1u << bit);
    int c = 0;
#pragma unroll
    for (int u = 0; u < kProbeMaxRows / 64; ++u) c += __builtin_popcountll(__ballot(v[u] >= cand_v));
    if (c >= k) ans = cand_v;
  }
  if (lane == 0) thr[b] = unord_f32(ans);
}

}  // namespace dense
}  // namespace ahr

// =============================================================================================
// Host side: the index handle and the C ABI.
// =============================================================================================
using namespace ahr;
using namespace ahr::dense;

// One query workspace: converted queries, per-split partial lists, pre-pass scores/thresholds.
struct ahr_query_ws {
  uint8_t* qbuf = nullptr;
  uint8_t* qbuf_kb = nullptr;  // k-blocked copy of qbuf (half types: the kb256 kernel's B operand)
  int64_t q_cap = 0;
  uint64_t* part = nullptr;
  int64_t part_cap = 0;
  float* sample = nullptr;
  int64_t sample_cap = 0;
  uint8_t* cand = nullptr;
  int64_t cand_cap = 0;
  uint64_t* ss = nullptr;  // register-resident plan: self-seeding tag + granules (published maxima, seeds)
  int64_t ss_cap = 0;
};
constexpr int kMaxWorkspaces = 4;

struct ahr_index {
  int dim = 0;
  int dtype = 0;
  int elem = 0;
  int d_pad = 0;
  int device = 0;
  int64_t capacity = 0;
  int64_t cap_pad = 0;
  int64_t row_stride = 0;
  int64_t count = 0;
  uint8_t* rows = nullptr;
  uint8_t* rows_kb = nullptr;  // half types, once the kb256 plan ran: k-blocked copy of rows (kb256::offset)
  uint8_t* qbuf = nullptr;
  uint8_t* qbuf_kb = nullptr;
  int64_t q_cap = 0;  // rows in qbuf (multiple of kRowPad)
  uint64_t* part = nullptr;
  int64_t part_cap = 0;  // uint64 elements (+ 8: the small kernels' fold counter; + 128: kb256 pacing)
  float* sample = nullptr;  // pre-pass scores [B][S] then thresholds [B]
  int64_t sample_cap = 0;   // floats
  uint8_t* cand = nullptr;  // query-resident kernel: candidate groups (counts, row bases, scores)
  int64_t cand_cap = 0;     // bytes
  uint64_t* ss = nullptr;   // register-resident plan: [1] launch tag, [q_cap][kQresMaxSplits] published maxima, [q_cap] seeds
  int64_t ss_cap = 0;       // uint64 elements
  int sample_rows = -1;     // S; 0 disables the threshold pre-pass, -1 = sample_rows_for(count)
  const float* seed = nullptr;  // caller-supplied admission thresholds [B] (device), replace the pre-pass
  // The fields above (qbuf .. ss_cap) are the ACTIVE query workspace; the others are parked
  // here (ahr_index_set_workspace swaps them) so batches on different streams never share one.
  ahr_query_ws parked[kMaxWorkspaces];
  int cur_ws = 0;
  uint32_t debug_flags = 0;  // ablation / plan flags (kFlag*); 0 in production
  // Optional stage timing: a ring of HIP events, kStages+1 per query call, recorded on the
  // call's stream (ahr_index_profile_begin / _end).
  std::vector<hipEvent_t> prof_events;
  int prof_max_calls = 0;
  // The register-resident kernel fills every CU and its first seeding event waits (bounded) for
  // every split: a batch's kernel of this plan on one workspace's stream starts after the previous
  // one's kernel on another (its completion event; AHR_QRES_CHAIN=merge: after its merge), so no
  // workgroup of another batch delays its start.
  // The event is recorded only once batches of this plan have come on two streams (qres_multi): on
  // one stream the order is the stream's own, and the record after the merge cost the serial C2
  // step 4.7 us (merge stage 14.0 vs 9.3 us, profiles/r04/ab_endphase). (Two batches in flight
  // lose to one: 0.154-0.168 vs 0.152-0.153 ms per C2 step, the kernel runs ~5 us slower beside
  // the other batch's merge, profiles/r05/negative/chain_ab; bench.py runs this plan with one.)
  hipEvent_t qres_done = nullptr;
  hipStream_t qres_stream = nullptr;
  bool qres_multi = false;
  int prof_calls = 0;
  uint32_t* fold_ctr() const { return reinterpret_cast<uint32_t*>(part + part_cap); }
};

namespace {

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Register-resident batches of different streams (ahr_index::qres_done): a batch of this plan waits
// for the previous one of another stream, so its first seeding event finds every split resident.
// AHR_QRES_CHAIN=merge orders the whole batches (the conversion waits for the other batch's merge);
// =kernel only the kernels (the wait right before the launch, the record right after it).
inline bool qres_chain_at_kernel() {
  static const bool at_kernel = [] {
    const char* e = getenv("AHR_QRES_CHAIN");
    return !(e && strcmp(e, "merge") == 0);
  }();
  return at_kernel;
}
inline int qres_chain_wait(ahr_index* ix, hipStream_t s) {
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(s, &cap);
  if (cap == hipStreamCaptureStatusNone && ix->qres_stream && ix->qres_stream != s) {
    if (ix->qres_multi) AHR_HIP(hipStreamWaitEvent(s, ix->qres_done, 0));
    ix->qres_multi = true;  // from the next batch on (this one's predecessor recorded nothing)
  }
  return AHR_OK;
}
inline int qres_chain_record(ahr_index* ix, hipStream_t s) {
  if (!ix->qres_done) return AHR_OK;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(s, &cap);
  if (cap == hipStreamCaptureStatusNone) {
    if (ix->qres_multi) AHR_HIP(hipEventRecord(ix->qres_done, s));
    ix->qres_stream = s;
  }
  return AHR_OK;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

int kcap_for(int k) { return k <= 8 ? 8 : (k <= 16 ? 16 : 32); }

constexpr int kStages = 4;  // convert, threshold pre-pass, tile kernel, merge

inline void prof_mark(ahr_index* ix, int stage, hipStream_t s) {
  if (ix->prof_calls < ix->prof_max_calls)
    (void)hipEventRecord(ix->prof_events[(size_t)ix->prof_calls * (kStages + 1) + stage], s);
}

// ahr_index_plan kernel ids: 0 = 128x128 tile kernel, 1 = lane 256x256, 3 = 128x128 lane-local tile
// kernel, 5 = query-resident kernel (dimension halves over wave pairs), 6 = 256x256 16x16x32 kernel
// (opt-in), 7 = small-batch streaming kernel (B <= 16), 8 = k-blocked 256x256 kernel, 10 = 256-query
// register-resident kernel (ahr_qres.hip). Ids 2, 4 and 9 were measured-slower variants (lane
// 256x128, a one-wave-per-SIMD query-resident kernel, k-blocked 256x128): removed.
enum { KERNEL_TILE128 = 0, KERNEL_LANE256 = 1, KERNEL_TILELANE = 3, KERNEL_QKV = 5, KERNEL_T256 = 6,
       KERNEL_SMALL = 7, KERNEL_KB256 = 8, KERNEL_QRES = 10, KERNEL_LANE64 = 11 };
// 256 x 64 lane-local tiles for 17 <= B <= 64 (bf16 / f16): the 128-query tile would multiply
// half padding (A/B: AHR_LANE64)
inline bool lane64_on() {
  static const bool on = [] {
    const char* e = getenv("AHR_LANE64");
    return e && atoi(e) != 0;
  }();
  return on;
}

struct SearchPlan {
  int kernel;
  int qblocks, n_row_tiles, n_splits, tiles_per_split;
  bool xcd_remap;
};

// Corpus and query buffers are padded to whole 256-row tiles (the wide kernel's tile).
constexpr int64_t kRowPad = 256;
// The 256x256 lane kernel from this batch on; below it the 128x128 lane-local tile kernel is as
// fast or faster (MI355X, hotpot90k).
constexpr int kWideMinBatch = 6144;

// Resident workgroups of the 128x128 tile kernel: 2 per CU (VGPR/LDS limited).
constexpr int kResidentSlots128 = 256 * 2;
inline int env_int_clamped(const char* name, int dflt, int lo, int hi) {
  const char* e = getenv(name);
  return e ? std::max(lo, std::min(hi, atoi(e))) : dflt;
}

// The query-resident kernel keeps a 128-query block's fragments in registers: bf16/f16 and the
// dimensions it is instantiated for (d_pad = 384, 768). Its admission threshold is the pre-pass
// seed (raised only by the fallback list), so it is planned where the seed samples at least 1/32
// of the corpus, and from B = 2048 on, where it measured ahead of the lane-local tile kernel
// (hotpot90k: 276 vs 282 us at B = 2048, 531 vs 581 us at 4096; behind at 1024, 153 vs 147, and
// at 5M rows, 11.2 vs 9.1 ms; a seed from 1/350 of random data: 1.5 ms vs 0.39 ms — a full
// candidate buffer's fallback list lives in private memory, and folding the buffer into it to
// raise the threshold made the normal case slower, 591 vs 531 us at 4096). Debug flag kFlagQkv
// plans it at any size.
// Rows scored by the threshold pre-pass. The seed admits ~k * N / S candidates per query, so a
// larger corpus wants a larger sample: S = 16384 from 512k rows on (5M x 768: tile kernel 8.87 vs
// 9.10 ms at S = 8192, the pre-pass 49 vs 30 us; 625k: kb256 1.03 vs 1.06 ms, 312k: a wash),
// 8192 below (C2, 90k rows: 16384 measured +12 us end to end).
// From 2M rows S = 32768 (5M x 768, kb256: 7.41 vs 7.63 ms per batch; 2.5M: 3.80 vs 3.87 ms;
// 65536: the pre-pass grows to 173 us and eats the gain; 1.25M and 625k: 16384 stays ahead).
inline int sample_rows_for(const ahr_index* ix) {
  if (ix->sample_rows >= 0) return ix->sample_rows;
  return ix->count >= (1 << 21) ? 32768 : (ix->count >= (1 << 19) ? 16384 : 8192);
}

bool qkv_ok(const ahr_index* ix, int B, int k) {
  if (!kAblation) return false;  // compiled into the ablation build only (round 5)
  const int nkt = ix->d_pad * ix->elem / kRowBytes;
  if (k > 16 || ix->dtype == AHR_F32 || !(nkt == 6 || nkt == 12)) return false;
  if (ix->debug_flags & (kFlagTile128 | kFlagTileLane | kFlagNoQres)) return false;
  // opt-in only: the 256-query register-resident kernel covers its batches (B >= 512, k <= 12)
  return (ix->debug_flags & kFlagQkv) != 0;
}

// The small-batch streaming kernel: B <= 16, bf16/f16, k <= 16, the
// query rows (or one group's lane lists of the end merge) within LDS; not under a kernel flag.
bool small_ok(const ahr_index* ix, int B, int k) {
  if (ix->dtype == AHR_F32)  // exact mode: the VALU fma-chain stream (topk_small_f32_kernel)
    return B <= smallf32::kMaxQ && k <= 16 && ix->d_pad <= 1024 && !(ix->debug_flags & kForceFlags);
  // B <= 16: one group of 16 queries. (2 and 4 groups, B <= 64, measured slower than the 128x128
  // lane-local kernel with its pre-pass — 51 us at B = 32, 81 us at B = 64 vs ~40 us: removed.)
  if (B > small::kMaxQ || k > 16) return false;
  if (ix->debug_flags & kForceFlags) return false;
  return small::lds_bytes(ix->row_stride, 16, 1) <= 160 * 1024;
}

// The k-blocked 256x256 kernel (bf16/f16, k <= 16) from kKB256MinRows corpus rows on, below the
// register-resident kernel's batch range (or k in 13..16): there the
// corpus streams from HBM and its 3-step-deep ring beats the 128x128 kernel's 1-step one (5M
// rows, B = 1024: 8.11 vs 9.04 ms; 1.25M: 1.97 vs 2.31 ms; 625k: 1.03 vs 1.17 ms; 312k: equal;
// at 90k, L2/MALL-resident, the 128x128 kernel is ahead, 152 vs 209 us). Debug flags force it
// (kFlagKB256) or keep it out (kFlagNoKB256).
constexpr int64_t kKB256MinRows = 1 << 19;
bool kb256_ok(const ahr_index* ix, int B, int k) {
  if (k > 16 || ix->dtype == AHR_F32 || B <= 0) return false;
  if (ix->debug_flags & kFlagNoKB256) return false;
  if (ix->debug_flags & kFlagKB256) return true;
  if (ix->debug_flags & kForceFlags) return false;  // another kernel explicitly requested
  return ix->count >= kKB256MinRows;
}


// The 256-query register-resident kernel (ahr_qres.hip): bf16/f16 at d_pad = 768 or 384, k <= 12,
// from kQresMinBatch queries and kQresMinRows rows on (every split then has the blocks its
// self-seeding needs), while admission seeding is on (sample rows != 0). Debug flags force it
// (kFlagQres) or keep it out (kFlagNoQres, or any other kernel flag).
constexpr int kQresMinBatch = 512;
constexpr int64_t kQresMinRows = 32768;
// the register-resident plan's splits: one wave of 256 workgroups; a multiple of 8 with the XCD remap
// (>= 8 splits), else every split the grid has room for (fewer than 8 never seed themselves anyway)
inline int qres_splits(int64_t count, int B) {
  int want = std::max(1, 256 / (int)cdiv(B, qres::kTQ));
  want = (int)std::min<int64_t>(want, std::max<int64_t>(1, cdiv(count, qres::kTR)));
  return want >= 8 ? want / 8 * 8 : want;
}
bool qres_ok(const ahr_index* ix, int B, int k) {
  if (!qres::supported(ix->dtype, ix->d_pad * ix->elem, k) || B <= 0) return false;
  if (ix->debug_flags & kFlagNoQres) return false;
  if (ix->debug_flags & kFlagQres) return true;
  if (ix->debug_flags & kForceFlags) return false;  // another kernel explicitly requested
  if (B < kQresMinBatch || sample_rows_for(ix) <= 0 || ix->count < kQresMinRows) return false;
  // Past kKB256MinRows (the corpus streams from HBM) only where the launch seeds itself: 5M x 768
  // f16, B = 1024, self-seeded qres256 6.96 ms vs kb256 7.45 ms per launch on the same box
  // (profiles/r04/ab_sched/c3); the pre-pass-seeded form (B >= 4096: <= 16 splits) was measured
  // behind kb256 (round 3 at B = 1024: 7.71 vs 7.49 ms), so those batches keep kb256.
  return ix->count < kKB256MinRows || qres::self_seeds(ix->count, qres_splits(ix->count, B), k);
}

// Self-seeding buffer of the register-resident plan (ahr_qres.hip): the per-XCD row weights and
// duration sums (kQresTagOff words), the launch tag (advanced on the device by each query
// conversion), then per query slot of the padded batch one published maximum
// per split (at most kQresMaxSplits), then one seed (and, past the seeds, the spare slots a
// selection with no seed writes to; the kernel uses at most 128 splits, so they fit). Zeroed when allocated (tag 0 is never a
// launch's), so a granule is only ever this workspace's own.
constexpr int64_t kQresMaxSplits = 256;
// ss[0..7]: the per-XCD row weights and duration sums (rebalance_xcds), ss[8]: the launch tag
constexpr int64_t kQresTagOff = 8;
int ensure_ss(ahr_index* ix, hipStream_t s) {
  if (!ix->qres_done) AHR_HIP(hipEventCreateWithFlags(&ix->qres_done, hipEventDisableTiming));
  const int64_t need = kQresTagOff + 1 + ix->q_cap * (kQresMaxSplits + 1);
  if (need <= ix->ss_cap) return AHR_OK;
  if (ix->ss) AHR_HIP(hipFree(ix->ss));
  ix->ss = nullptr;
  ix->ss_cap = 0;
  if (hipMalloc(&ix->ss, need * sizeof(uint64_t)) != hipSuccess)
    return fail(AHR_ENOMEM, "self-seeding workspace allocation failed");
  AHR_HIP(hipMemsetAsync(ix->ss, 0, need * sizeof(uint64_t), s));
  ix->ss_cap = need;
  return AHR_OK;
}

// The register-resident kernel's self-seeding schedule over a split's block index: publications
// after blocks 0, 2, 4, 6 and then every 4th to 30, seeding events at the ends of blocks 1 (the
// first, waiting), 3, 5, 7 and every 4th to 31 (then every 8 blocks: ahr_qres.hip). A later event
// selects from the granules the previous one read and applies the seeds it read, so a seed lags its
// publication by two events; dense early events make up for that while the threshold is loose.
// AHR_QRES_PUB / AHR_QRES_EV (hex bit masks) override it for tuning.
struct QresSchedule {
  uint64_t pub, ev;
};
inline QresSchedule qres_schedule() {
  static const QresSchedule sch = [] {
    QresSchedule d{0x44444455ull, 0x888888a8ull};
    if (const char* e = getenv("AHR_QRES_PUB")) d.pub = strtoull(e, nullptr, 16);
    if (const char* e = getenv("AHR_QRES_EV")) d.ev = strtoull(e, nullptr, 16);
    return d;
  }();
  return sch;
}

// The register-resident kernel seeds itself (no pre-pass launch) unless kFlagQresPrepass asks for
// the sampled pre-pass (A/B) or the caller supplies seeds.
inline bool qres_self_seeded(const ahr_index* ix, const SearchPlan& p, int k) {
  return p.kernel == KERNEL_QRES && sample_rows_for(ix) > 0 && !ix->seed && !(ix->debug_flags & kFlagQresPrepass) &&
         qres::self_seeds(ix->count, p.n_splits, k);
}

// the second query buffer (the register-resident plan's fragment-major copy, or the k-blocked
// copy of the kb256 plan), zeroed on the caller's stream when allocated
int ensure_qbuf_kb(ahr_index* ix, hipStream_t s) {
  if (ix->qbuf_kb) return AHR_OK;
  if (hipMalloc(&ix->qbuf_kb, ix->q_cap * ix->row_stride) != hipSuccess)
    return fail(AHR_ENOMEM, "query workspace allocation failed");
  AHR_HIP(hipMemsetAsync(ix->qbuf_kb, 0, ix->q_cap * ix->row_stride, s));
  return AHR_OK;
}

// Workgroup cap of the 128 x 128 plans. Two per CU serve one batch at a time best; when the
// caller keeps batches in flight on several query workspaces (ahr_index_set_workspace: another
// slot holds a reserved one), one per CU lets two batches' workgroups co-reside: B = 64 / 128 /
// 256 two in flight 0.0388 / 0.0428 / 0.0594 -> 0.0374 / 0.0401 / 0.0545 ms per step, while one
// at a time would lose 5 / 1 / 16 % (profiles/r06/slots/); B = 384: 0.0768 -> 0.0721 ms
// (profiles/r06/inflight/). Up to 3 query blocks (B <= 384): at B = 1024 fp32 (8 blocks) one per
// CU measured 0.4 % slower (profiles/r06/slots_f32/). AHR_TILE_SLOTS (8..512) fixes the cap.
// true when another query workspace slot holds a reserved workspace: the caller keeps batches in
// flight on several streams
inline bool concurrent_workspaces(const ahr_index* ix) {
  for (int w = 0; w < kMaxWorkspaces; ++w)
    if (w != ix->cur_ws && ix->parked[w].part_cap > 0) return true;
  return false;
}
inline int tile_slots(const ahr_index* ix, int qblocks) {
  static const int fixed = env_int_clamped("AHR_TILE_SLOTS", 0, 0, kResidentSlots128);
  if (fixed) return std::max(8, fixed);
  if (qblocks > 3) return kResidentSlots128;
  // fp32, one query block (17 <= B <= 128): one per CU wins one at a time too (B = 64: 0.1965 vs
  // 0.2325 ms serial; two in flight 0.1637 vs 0.1700; B = 256 two in flight 0.3166 vs 0.3546 ms:
  // profiles/r06/slots_f32b/)
  if (ix->dtype == AHR_F32 && qblocks == 1) return kResidentSlots128 / 2;
  return concurrent_workspaces(ix) ? kResidentSlots128 / 2 : kResidentSlots128;
}

SearchPlan plan_search(const ahr_index* ix, int B, int k) {
  SearchPlan p;
  p.kernel = KERNEL_TILE128;
  if (!small_ok(ix, B, k) && qres_ok(ix, B, k)) {
    // one workgroup of 8 waves per CU, 256 queries each: one wave of 256 workgroups
    p.kernel = KERNEL_QRES;
    p.qblocks = (int)cdiv(B, qres::kTQ);
    p.n_row_tiles = (int)cdiv(ix->count, qres::kTR);
    p.n_splits = qres_splits(ix->count, B);
    p.xcd_remap = p.n_splits >= 8;
    p.tiles_per_split = (int)cdiv(p.n_row_tiles, p.n_splits);
    return p;
  }
  if (small_ok(ix, B, k)) {
    // one workgroup per CU, at least one 16-row block per wave
    p.kernel = KERNEL_SMALL;
    p.qblocks = 1;
    const bool f32 = ix->dtype == AHR_F32;  // 64-row items (a row per lane) vs 16-row blocks
    p.n_row_tiles = (int)cdiv(ix->count, f32 ? 64 : 16);
    // AHR_SMALL_SPLITS (A/B): workgroups per launch, up to 512 (two per CU co-reside: <= 128 VGPRs).
    // Unset: 256, or 128 with batches in flight on several workspaces at fp32 B = 4 / half B = 16
    // (two in flight 0.0672 -> 0.0500 / 0.0352 -> 0.0336 ms per step; one at a time they would
    // lose 0.075 -> 0.095 / 0.045 -> 0.054 ms; at B = 1 256 stays best: profiles/r06/small_splits/)
    static const int split_env = env_int_clamped("AHR_SMALL_SPLITS", 0, 0, 512);
    const int splits = split_env ? split_env
                                 : (B >= (f32 ? 4 : 16) && concurrent_workspaces(ix) ? 128 : 256);
    p.n_splits = (int)std::max<int64_t>(
        1, std::min<int64_t>(splits, cdiv(p.n_row_tiles, f32 ? smallf32::waves_per_split() : small::waves(1))));
    p.tiles_per_split = (int)cdiv(p.n_row_tiles, p.n_splits);
    p.xcd_remap = false;
    return p;
  }
  if (k <= 16 && ix->dtype != AHR_F32 && (ix->debug_flags & kFlagT256)) {
    // 256x256 tiles, one workgroup per CU: one wave of 256 workgroups
    p.kernel = KERNEL_T256;
    p.qblocks = (int)cdiv(B, t256::kTQ);
    p.n_row_tiles = (int)cdiv(ix->count, t256::kTR);
    int want = std::max(1, 256 / p.qblocks);
    want = std::min(want, std::max(1, p.n_row_tiles));
    p.xcd_remap = want >= 8;
    p.n_splits = p.xcd_remap ? want / 8 * 8 : want;
    p.tiles_per_split = (int)cdiv(p.n_row_tiles, p.n_splits);
    return p;
  }
  if (kb256_ok(ix, B, k)) {
    // 256x256 tiles, one workgroup per CU: one wave of workgroups
    p.kernel = KERNEL_KB256;
    p.qblocks = (int)cdiv(B, KbCfg<4>::kTQ);
    p.n_row_tiles = (int)cdiv(ix->count, kb256::kTR);
    int want = std::max(1, 256 / p.qblocks);
    want = std::min(want, std::max(1, p.n_row_tiles));
    p.xcd_remap = want >= 8;
    p.n_splits = p.xcd_remap ? want / 8 * 8 : want;
    p.tiles_per_split = (int)cdiv(p.n_row_tiles, p.n_splits);
    return p;
  }
  if (qkv_ok(ix, B, k)) {
    // one workgroup per CU (512 VGPRs per lane): one wave of 256 workgroups
    p.kernel = KERNEL_QKV;
    p.qblocks = (int)cdiv(B, kTileQ);
    p.n_row_tiles = (int)cdiv(ix->count, qkv::kTR);
    int want = std::max(1, 256 / p.qblocks);
    want = std::min(want, std::max(1, p.n_row_tiles));
    p.xcd_remap = want >= 8;
    p.n_splits = p.xcd_remap ? want / 8 * 8 : want;
    p.tiles_per_split = (int)cdiv(p.n_row_tiles, p.n_splits);
    return p;
  }
  if (k <= 16 && !(ix->debug_flags & kFlagTile128)) {
    if (B >= kWideMinBatch && !(ix->debug_flags & kFlagTileLane))
      p.kernel = KERNEL_LANE256;
    else if (B <= 64 && ix->dtype != DT_F32 && !(ix->debug_flags & kFlagTileLane) && lane64_on())
      p.kernel = KERNEL_LANE64;
    else
      p.kernel = KERNEL_TILELANE;
  }
  if (p.kernel == KERNEL_LANE64) {
    p.qblocks = (int)cdiv(B, 64);
    p.n_row_tiles = (int)cdiv(ix->count, 256);
    int want = std::max(1, tile_slots(ix, p.qblocks) / p.qblocks);
    want = std::min(want, std::max(1, p.n_row_tiles));
    p.xcd_remap = want >= 8;
    p.n_splits = p.xcd_remap ? want / 8 * 8 : want;
    p.tiles_per_split = (int)cdiv(p.n_row_tiles, p.n_splits);
    return p;
  }
  if (p.kernel == KERNEL_LANE256) {
    // 256 x 256 tiles, one resident workgroup per CU. One wave of workgroups; splits a multiple of
    // 8 (rounded down: an extra workgroup would run as a second wave) so the XCD remap keeps a
    // split's query blocks on one XCD.
    p.qblocks = (int)cdiv(B, 256);
    p.n_row_tiles = (int)cdiv(ix->count, 256);
    int want = std::max(1, 256 / p.qblocks);
    want = std::min(want, std::max(1, p.n_row_tiles));
    p.xcd_remap = want >= 8;
    p.n_splits = p.xcd_remap ? want / 8 * 8 : want;
    p.tiles_per_split = (int)cdiv(p.n_row_tiles, p.n_splits);
    return p;
  }
  p.qblocks = (int)cdiv(B, kTileQ);
  p.n_row_tiles = (int)cdiv(ix->count, kTileRows);
  // One wave of workgroups: at most the resident slots, splits rounded DOWN to a multiple of 8
  // (an extra workgroup would run as a second wave) so the XCD remap keeps a split's query
  // blocks on one XCD; the kernel balances tile ranges over the splits.
  int want = std::max(1, tile_slots(ix, p.qblocks) / p.qblocks);
  want = std::min(want, std::max(1, p.n_row_tiles));
  p.xcd_remap = want >= 8;
  p.n_splits = p.xcd_remap ? want / 8 * 8 : want;
  p.tiles_per_split = (int)cdiv(p.n_row_tiles, p.n_splits);
  return p;
}

// Grows the active workspace. A new query buffer is zeroed on the caller's stream: a blocking
// null-stream memset is not ordered against non-blocking streams and could land after the
// conversion kernel of the first batch on this workspace.
int ensure_query_ws(ahr_index* ix, int B, int k, hipStream_t s) {
  const int64_t q_need = cdiv(B, kRowPad) * kRowPad;
  if (q_need > ix->q_cap) {
    if (ix->qbuf) AHR_HIP(hipFree(ix->qbuf));
    if (ix->qbuf_kb) AHR_HIP(hipFree(ix->qbuf_kb));
    ix->qbuf = ix->qbuf_kb = nullptr;
    ix->q_cap = 0;  // (the self-seeding granules are sized by q_cap: ensure_ss regrows them)
    if (hipMalloc(&ix->qbuf, q_need * ix->row_stride) != hipSuccess)
      return fail(AHR_ENOMEM, "query workspace allocation failed");
    AHR_HIP(hipMemsetAsync(ix->qbuf, 0, q_need * ix->row_stride, s));
    ix->q_cap = q_need;
  }
  // Partial lists: B x n_splits x k, sized for the worst case split count at this capacity.
  const int64_t qblocks = cdiv(B, kTileQ);
  const int64_t max_splits = cdiv(std::max<int64_t>(1, cdiv(kResidentSlots128, qblocks)), 8) * 8;
  const int64_t wide_splits = std::max<int64_t>(1, 512 / cdiv(B, 128));  // >= any plan's
  const int64_t t256_lists = 2 * std::max<int64_t>(1, 512 / cdiv(B, 128));  // (split, row half) lists of t256 / kb256
  const int64_t p_need = (int64_t)B *
                         std::max<int64_t>(std::max(std::max(max_splits, wide_splits), t256_lists), kSampleMax / kTileRows) *
                         k;
  if (p_need > ix->part_cap) {
    if (ix->part) AHR_HIP(hipFree(ix->part));
    ix->part = nullptr;
    ix->part_cap = 0;
    if (hipMalloc(&ix->part, (p_need + 8) * sizeof(uint64_t)) != hipSuccess)
      return fail(AHR_ENOMEM, "partial top-k workspace allocation failed");
    ix->part_cap = p_need;
    AHR_HIP(hipMemsetAsync(ix->part + p_need, 0, 8 * sizeof(uint64_t), s));  // the small kernels' fold counter
  }
  const int64_t s_need = (int64_t)B * (kGroupMax + 1);
  if (s_need > ix->sample_cap) {
    if (ix->sample) AHR_HIP(hipFree(ix->sample));
    ix->sample = nullptr;
    ix->sample_cap = 0;
    if (hipMalloc(&ix->sample, s_need * sizeof(float)) != hipSuccess)
      return fail(AHR_ENOMEM, "sample workspace allocation failed");
    ix->sample_cap = s_need;
  }
  return AHR_OK;
}

template <int DT, int KCAP, int MODE>
void launch_tile(const ahr_index* ix, int n_splits, int qblocks, int tiles_per_split,
                 int n_row_tiles, int n_rows, int B, int k, uint32_t row_base, const float* thr,
                 float* score_out, int64_t score_ld, int flags, hipStream_t s) {
  static std::atomic<uint64_t> lds_attr{0};  // > 64 KiB dynamic LDS: opt in per device
  ensure_lds_attr(lds_attr, reinterpret_cast<const void*>(&topk_tile_kernel<DT, KCAP, MODE>), kLdsBytes);
  dim3 grid((unsigned)(n_splits * qblocks));
  hipLaunchKernelGGL((topk_tile_kernel<DT, KCAP, MODE>), grid, dim3(kThreads), kLdsBytes, s,
                     ix->rows, ix->qbuf, ix->row_stride, n_rows, B, ix->d_pad * ix->elem / kRowBytes,
                     tiles_per_split, n_row_tiles, row_base, k, ix->part, thr, score_out, score_ld,
                     n_splits, qblocks, flags);
}

template <int DT, int KCAP, int NB, int BJ, int WR, int WQ, int STAGES, int MINB>
void launch_lane(const ahr_index* ix, const SearchPlan& p, int n_rows, int B, int k, uint32_t row_base,
                 const float* thr, int flags, hipStream_t s) {
  using C = lanek::Cfg<NB, BJ, WR, WQ, STAGES>;
  constexpr auto kern = &topk_lane_kernel<DT, KCAP, NB, BJ, WR, WQ, STAGES, MINB>;
  static std::atomic<uint64_t> lds_attr{0};  // > 64 KiB dynamic LDS: opt in per device
  ensure_lds_attr(lds_attr, reinterpret_cast<const void*>(kern), C::kLdsTotal);
  hipLaunchKernelGGL(kern, dim3((unsigned)(p.n_splits * p.qblocks)), dim3(C::kThreads), C::kLdsTotal, s, ix->rows,
                     ix->qbuf, ix->row_stride, n_rows, B, ix->d_pad * ix->elem / lanek::kRowBytes, p.n_splits,
                     p.n_row_tiles, row_base, k, ix->part, thr, p.qblocks, flags);
}

// lane lists sized to k: 8, 12 or 16 keys (insert and select cost scale with the size)
template <int DT, int KCAP>
void launch_tilelane(const ahr_index* ix, const SearchPlan& p, int n_rows, int B, int k, uint32_t row_base,
                     const float* thr, int flags, hipStream_t s) {
  constexpr int lds = 2 * kBufBytes;  // the staging double buffer (also the end-merge exchange)
  static_assert(kTileQ * 4 * KCAP * 8 <= lds, "end merge exchange must fit");
  static_assert(2 * lds <= 160 * 1024, "two workgroups per CU");
  constexpr auto kern = &topk_tilelane_kernel<DT, KCAP>;
  static std::atomic<uint64_t> lds_attr{0};  // > 64 KiB dynamic LDS: opt in per device
  ensure_lds_attr(lds_attr, reinterpret_cast<const void*>(kern), lds);
  hipLaunchKernelGGL(kern, dim3((unsigned)(p.n_splits * p.qblocks)), dim3(kThreads), lds, s, ix->rows, ix->qbuf,
                     ix->row_stride, n_rows, B, ix->d_pad * ix->elem / kRowBytes, p.n_row_tiles, row_base, k,
                     ix->part, thr, p.n_splits, p.qblocks, flags);
}

// Candidate keys per producer (query, split, half, lane half): one per tile of the split covers
// the C2 survivor rate (~1 row per producer) many times over; a full buffer falls back to the
// lane's private list inside the kernel, so the cap only trades memory for speed.
inline int qkv_cand_cap(const SearchPlan& p) { return (int)std::min(64, std::max(16, p.tiles_per_split)); }
inline int64_t cand_bytes(int B, const SearchPlan& p) {
  const int64_t prod = (p.kernel == KERNEL_T256 || p.kernel == KERNEL_KB256) ? 8 : 4;  // producers per (query, split)
  return (int64_t)B * prod * p.n_splits * qkv_cand_cap(p) * 8;
}

int ensure_cand(ahr_index* ix, int64_t bytes) {
  if (bytes <= ix->cand_cap) return AHR_OK;
  if (ix->cand) AHR_HIP(hipFree(ix->cand));
  ix->cand = nullptr;
  ix->cand_cap = 0;
  if (hipMalloc(&ix->cand, bytes) != hipSuccess) return fail(AHR_ENOMEM, "candidate workspace allocation failed");
  ix->cand_cap = bytes;
  return AHR_OK;
}

template <int DT, int NKT, int ST, int KCAP>
void launch_qkv(const ahr_index* ix, const SearchPlan& p, int n_rows, int B, int k, uint32_t row_base,
                const float* thr, int flags, hipStream_t s) {
  constexpr int lds = qkv::Cfg<ST>::kLds;
  constexpr auto kern = &topk_qkv_kernel<DT, NKT, ST, KCAP>;
  static std::atomic<uint64_t> lds_attr{0};  // > 64 KiB dynamic LDS: opt in per device
  ensure_lds_attr(lds_attr, reinterpret_cast<const void*>(kern), lds);
  hipLaunchKernelGGL(kern, dim3((unsigned)(p.n_splits * p.qblocks)), dim3(512), lds, s, ix->rows, ix->qbuf,
                     ix->row_stride, n_rows, B, p.n_row_tiles, row_base, k, ix->part, thr, p.n_splits, p.qblocks,
                     flags, reinterpret_cast<uint64_t*>(ix->cand), qkv_cand_cap(p));
}

template <int DT, int KCAP>
void launch_t256(const ahr_index* ix, const SearchPlan& p, int n_rows, int B, int k, uint32_t row_base,
                 const float* thr, int flags, hipStream_t s) {
  constexpr auto kern = &topk_t256_kernel<DT, KCAP>;
  static std::atomic<uint64_t> lds_attr{0};  // > 64 KiB dynamic LDS: opt in per device
  ensure_lds_attr(lds_attr, reinterpret_cast<const void*>(kern), t256::kLds);
  hipLaunchKernelGGL(kern, dim3((unsigned)(p.n_splits * p.qblocks)), dim3(512), t256::kLds, s, ix->rows, ix->qbuf,
                     ix->row_stride, n_rows, B, ix->d_pad * ix->elem / kRowBytes, p.n_row_tiles, row_base, k, ix->part,
                     thr, p.n_splits, p.qblocks, flags, reinterpret_cast<uint64_t*>(ix->cand), qkv_cand_cap(p));
}

template <int DT, int KCAP, int WN>
void launch_kb256(const ahr_index* ix, const SearchPlan& p, int n_rows, int B, int k, uint32_t row_base,
                  const float* thr, int flags, hipStream_t s) {
  using C = KbCfg<WN>;
  constexpr auto kern = &topk_kb256_kernel<DT, KCAP, WN>;
  static std::atomic<uint64_t> lds_attr{0};  // > 64 KiB dynamic LDS: opt in per device
  ensure_lds_attr(lds_attr, reinterpret_cast<const void*>(kern), C::kLds);
  hipLaunchKernelGGL(kern, dim3((unsigned)(p.n_splits * p.qblocks)), dim3(C::kThreads), C::kLds, s, ix->rows_kb,
                     ix->qbuf_kb, ix->d_pad * ix->elem / kb256::kKB, n_rows, B, p.n_row_tiles, row_base, k, ix->part,
                     thr, p.n_splits, p.qblocks, flags, reinterpret_cast<uint64_t*>(ix->cand), qkv_cand_cap(p));
}

template <int DT, int NKT>
void launch_qkv_k(const ahr_index* ix, const SearchPlan& p, int n_rows, int B, int k, uint32_t row_base,
                  const float* thr, int flags, hipStream_t s) {
  constexpr int ST = 3;  // phase slots of 32 KiB (+ 64 KiB exchange) in 160 KiB
  if (k <= 8)
    launch_qkv<DT, NKT, ST, 8>(ix, p, n_rows, B, k, row_base, thr, flags, s);
  else if (k <= 12)
    launch_qkv<DT, NKT, ST, 12>(ix, p, n_rows, B, k, row_base, thr, flags, s);
  else
    launch_qkv<DT, NKT, ST, 16>(ix, p, n_rows, B, k, row_base, thr, flags, s);
}

template <int DT, int NB, int BJ, int WR, int WQ, int STAGES, int MINB>
void launch_lane_k(const ahr_index* ix, const SearchPlan& p, int n_rows, int B, int k, uint32_t row_base,
                   const float* thr, int flags, hipStream_t s) {
  if (k <= 8)
    launch_lane<DT, 8, NB, BJ, WR, WQ, STAGES, MINB>(ix, p, n_rows, B, k, row_base, thr, flags, s);
  else if (k <= 12)
    launch_lane<DT, 12, NB, BJ, WR, WQ, STAGES, MINB>(ix, p, n_rows, B, k, row_base, thr, flags, s);
  else
    launch_lane<DT, 16, NB, BJ, WR, WQ, STAGES, MINB>(ix, p, n_rows, B, k, row_base, thr, flags, s);
}

// fold != nullptr: the small kernels merge the splits themselves (B <= kFoldMaxQ, fold_ok())
struct FoldOut {
  uint32_t* ctr;
  float* scores;
  int32_t* rows;
  uint64_t* keys;
};

template <int DT, int KCAP, int NG>
void launch_small(const ahr_index* ix, const SearchPlan& p, const float* q, int normalize_q, int B, int k,
                  uint32_t row_base, const FoldOut* fold, hipStream_t s) {
  const bool dma = small::use_dma(ix->row_stride, NG);
  int lds = small::lds_bytes(ix->row_stride, KCAP, NG, dma);
  if (fold) lds = std::max(lds, B * p.n_splits * k * 8 + 16);
  auto go = [&](auto kern, std::atomic<uint64_t>& attr) {
    ensure_lds_attr(attr, reinterpret_cast<const void*>(kern), 160 * 1024);  // > 64 KiB: opt in per device
    hipLaunchKernelGGL(kern, dim3((unsigned)p.n_splits), dim3(small::waves(NG) * 64), lds, s, ix->rows, q, ix->dim,
                       normalize_q, ix->qbuf, ix->row_stride, ix->d_pad, (int)ix->count, B,
                       (int)(ix->d_pad * ix->elem / 64), p.n_splits, row_base, k, ix->part,
                       fold ? fold->ctr : nullptr, fold ? fold->scores : nullptr, fold ? fold->rows : nullptr,
                       fold ? fold->keys : nullptr);
  };
  static std::atomic<uint64_t> a_reg{0}, a_dma{0};
#ifdef AHR_ABLATION
  if constexpr (NG == 1) {
    if (dma) {
      go(&topk_small_kernel<DT, KCAP, NG, true>, a_dma);
      return;
    }
  }
#endif
  (void)a_dma;
  go(&topk_small_kernel<DT, KCAP, NG, false>, a_reg);
}

template <int DT, int NG>
void launch_small_k(const ahr_index* ix, const SearchPlan& p, const float* q, int normalize_q, int B, int k,
                    uint32_t row_base, const FoldOut* fold, hipStream_t s) {
  if (k <= 8)
    launch_small<DT, 8, NG>(ix, p, q, normalize_q, B, k, row_base, fold, s);
  else if (k <= 12)
    launch_small<DT, 12, NG>(ix, p, q, normalize_q, B, k, row_base, fold, s);
  else
    launch_small<DT, 16, NG>(ix, p, q, normalize_q, B, k, row_base, fold, s);
}

// queries converted inside topk_small_kernel (convert_row_fast's shape) instead of by the convert kernel
inline bool small_fuses_convert(const ahr_index* ix) {
  return ix->dtype != AHR_F32 && (ix->dim & 3) == 0 && ix->d_pad <= 1024;
}
// fp32: topk_small_f32_kernel always converts its queries itself (convert_rows_kernel's arithmetic)
inline bool small_plan_fuses_convert(const ahr_index* ix) { return ix->dtype == AHR_F32 || small_fuses_convert(ix); }

template <int KCAP>
void launch_small_f32_k(const ahr_index* ix, const SearchPlan& p, int B, int k, uint32_t row_base, const float* q,
                        int normalize_q, const FoldOut* fold, hipStream_t s) {
  const int n_lines = (int)(ix->row_stride / 128);
  const size_t fold_lds = fold ? (size_t)B * p.n_splits * k * 8 + 16 : 0;
  const int slots = smallf32::slots();
  const size_t lds = std::max<size_t>(fold_lds, smallf32::ring_bytes(slots));
  uint32_t* fc = fold ? fold->ctr : nullptr;
  float* fs = fold ? fold->scores : nullptr;
  int32_t* fr = fold ? fold->rows : nullptr;
  uint64_t* fk = fold ? fold->keys : nullptr;
  auto go = [&](auto kern, std::atomic<uint64_t>& attr) {
    if (lds > 64 * 1024) ensure_lds_attr(attr, reinterpret_cast<const void*>(kern), (int)lds);
    hipLaunchKernelGGL(kern, dim3((unsigned)p.n_splits), dim3(smallf32::waves_for(slots) * 64), lds, s, ix->rows, q,
                       ix->dim, normalize_q, ix->qbuf, ix->row_stride, (int)ix->count, B, n_lines, p.n_splits, row_base,
                       k, ix->part, fc, fs, fr, fk);
  };
  static std::atomic<uint64_t> a12{0}, a42{0};  // per instantiation
#ifdef AHR_ABLATION
  static std::atomic<uint64_t> a10{0}, a40{0};
  if (slots == 0) {
    if (B == 1)
      go(topk_small_f32_kernel<KCAP, 1, 0>, a10);
    else
      go(topk_small_f32_kernel<KCAP, 4, 0>, a40);
    return;
  }
#endif
  if (B == 1)
    go(topk_small_f32_kernel<KCAP, 1, 2>, a12);
  else
    go(topk_small_f32_kernel<KCAP, 4, 2>, a42);
}

template <int DT>
void launch_search(ahr_index* ix, const SearchPlan& p, int B, int k, uint32_t row_base, const float* q,
                   int normalize_q, const FoldOut* fold, hipStream_t s) {
  const float* thr = nullptr;
  prof_mark(ix, 1, s);
  if constexpr (DT == DT_F32) {
    if (p.kernel == KERNEL_SMALL) {
      prof_mark(ix, 2, s);
      if (k <= 8)
        launch_small_f32_k<8>(ix, p, B, k, row_base, q, normalize_q, fold, s);
      else if (k <= 12)
        launch_small_f32_k<12>(ix, p, B, k, row_base, q, normalize_q, fold, s);
      else
        launch_small_f32_k<16>(ix, p, B, k, row_base, q, normalize_q, fold, s);
      return;
    }
  } else {
    if (p.kernel == KERNEL_SMALL) {
      prof_mark(ix, 2, s);
      const float* qs = small_fuses_convert(ix) ? q : nullptr;
      launch_small_k<DT, 1>(ix, p, qs, normalize_q, B, k, row_base, fold, s);
      return;
    }
  }
  const int S = sample_rows_for(ix);
  const bool self_seed = qres_self_seeded(ix, p, k);
  if (ix->seed) {
    thr = ix->seed;  // the caller's valid lower bounds of each query's k-th best score
  } else if (!self_seed && S > 0 && ix->count >= 4 * (int64_t)S && k * 16 <= S) {
    // Threshold pre-pass: score the first S rows, take each query's k-th best.
    float* scores = ix->sample;
    float* t = ix->sample + (int64_t)B * (S / 16);
    const int G = S / 16;  // 16-row groups
    // batches up to 64 queries take the wave form (same group maxima; B = 64: 8.6 vs 11.0 us; at
    // B = 128 / 256 its per-wave fragment loads re-read the rows 4 / 8 times and it loses: 20.5 /
    // 32.8 vs 19.4 / 19.8 us for the pre-pass stage, profiles/r06/prepass/)
    // (A/B: AHR_PREPASS_WAVE_B; two in flight the wave form loses at B = 96 / 128 too: 0.0392 /
    // 0.0432 vs 0.0385 / 0.0404 ms per step, profiles/r06/inflight/)
    static const int wave_max_b = env_int_clamped("AHR_PREPASS_WAVE_B", 64, 0, 256);
    const bool wave_form = B <= wave_max_b &&
                           launch_sample_groupmax<DT>(ix->rows, ix->qbuf, ix->row_stride,
                                                      ix->d_pad * ix->elem / kRowBytes, S, B, scores, G, s);
    if (!wave_form)
      launch_tile<DT, 8, MODE_GROUPMAX>(ix, S / kTileRows, (int)cdiv(B, kTileQ), 1, S / kTileRows, S, B, k, 0,
                                        nullptr, scores, G, 0, s);
    launch_sample_kth(scores, B, G, k, t, s);
    thr = t;
  }
  prof_mark(ix, 2, s);
  const int n = (int)ix->count;
  // XCD-balanced splits on the register-resident plan from 256 row blocks per split (C3: 5M rows,
  // 2,442 per split: 7.11-7.24 vs 7.35-7.50 ms per launch, same box; at C2's 44 no gain, the spread
  // inside an XCD dominates there: profiles/r04/xcd_balance/)
  const bool xcd_bal = p.kernel == KERNEL_QRES && p.xcd_remap && !(ix->debug_flags & kFlagNoXcdBalance) &&
                       cdiv(ix->count, qres::kTR) >= 256 * (int64_t)p.n_splits;
  const uint32_t flags = (p.xcd_remap ? kFlagXcdRemap : 0u) | (xcd_bal ? kFlagXcdBalance : 0u) | ix->debug_flags;
  if constexpr (DT != DT_F32) {
    if (p.kernel == KERNEL_QRES) {
      // self-seeding buffer: the per-XCD weights and duration sums (ss[0..7]), the tag (ss[8]), then
      // [256 qblocks][n_splits] maxima and [256 qblocks] seeds
      const QresSchedule sch = qres_schedule();
      const bool once = (flags & kFlagQresSeedOnce) != 0;
      // (<= 64 splits: the lane-list merge follows, which stops at a list's first empty slot)
      const uint32_t qflags = flags | (p.n_splits <= 64 ? kFlagShortLists : 0u);
      qres::launch(DT, k, ix->rows, ix->qbuf_kb, ix->row_stride, ix->d_pad * ix->elem, n, B, row_base, ix->part, thr,
                   p.n_splits, p.qblocks, (int)qflags, self_seed ? ix->ss + kQresTagOff + 1 : nullptr, once ? 1 : sch.pub,
                   once ? 0 : sch.ev, s);
      return;
    }
    if (p.kernel == KERNEL_KB256) {
      if (k <= 8)
        launch_kb256<DT, 8, 4>(ix, p, n, B, k, row_base, thr, flags, s);
      else if (k <= 12)
        launch_kb256<DT, 12, 4>(ix, p, n, B, k, row_base, thr, flags, s);
      else
        launch_kb256<DT, 16, 4>(ix, p, n, B, k, row_base, thr, flags, s);
      return;
    }
    if (p.kernel == KERNEL_T256) {
      if (k <= 8)
        launch_t256<DT, 8>(ix, p, n, B, k, row_base, thr, flags, s);
      else if (k <= 12)
        launch_t256<DT, 12>(ix, p, n, B, k, row_base, thr, flags, s);
      else
        launch_t256<DT, 16>(ix, p, n, B, k, row_base, thr, flags, s);
      return;
    }
#ifdef AHR_ABLATION
    if (p.kernel == KERNEL_QKV) {  // (the ablation build only: qkv_ok plans it nowhere else)
      if (ix->d_pad * ix->elem / kRowBytes == 12)
        launch_qkv_k<DT, 12>(ix, p, n, B, k, row_base, thr, flags, s);
      else
        launch_qkv_k<DT, 6>(ix, p, n, B, k, row_base, thr, flags, s);
      return;
    }
#endif
  }
  if (p.kernel == KERNEL_TILELANE) {
    switch (k <= 8 ? 8 : (k <= 12 ? 12 : 16)) {  // lists sized to k
      case 8: launch_tilelane<DT, 8>(ix, p, n, B, k, row_base, thr, flags, s); break;
      case 12: launch_tilelane<DT, 12>(ix, p, n, B, k, row_base, thr, flags, s); break;
      default: launch_tilelane<DT, 16>(ix, p, n, B, k, row_base, thr, flags, s); break;
    }
    return;
  }
  if (p.kernel == KERNEL_LANE256) {
    launch_lane_k<DT, 8, 1, 1, 8, 4, 1>(ix, p, n, B, k, row_base, thr, flags, s);
    return;
  }
  if constexpr (DT != DT_F32) {
    if (p.kernel == KERNEL_LANE64) {  // NB 4, BJ 1, WR 2, WQ 2: 256 rows x 64 queries, 4 waves, 3 stages
      launch_lane_k<DT, 4, 1, 2, 2, 3, 2>(ix, p, n, B, k, row_base, thr, flags, s);
      return;
    }
  }
  switch (k <= 8 ? 8 : (k <= 12 ? 12 : (k <= 16 ? 16 : 32))) {  // lists sized to k
    case 8: launch_tile<DT, 8, MODE_TOPK>(ix, p.n_splits, p.qblocks, p.tiles_per_split, p.n_row_tiles, n, B, k, row_base, thr, nullptr, 0, flags, s); break;
    case 12: launch_tile<DT, 12, MODE_TOPK>(ix, p.n_splits, p.qblocks, p.tiles_per_split, p.n_row_tiles, n, B, k, row_base, thr, nullptr, 0, flags, s); break;
    case 16: launch_tile<DT, 16, MODE_TOPK>(ix, p.n_splits, p.qblocks, p.tiles_per_split, p.n_row_tiles, n, B, k, row_base, thr, nullptr, 0, flags, s); break;
    default: launch_tile<DT, 32, MODE_TOPK>(ix, p.n_splits, p.qblocks, p.tiles_per_split, p.n_row_tiles, n, B, k, row_base, thr, nullptr, 0, flags, s); break;
  }
}

void launch_merge(const uint64_t* in, int B, int n_lists, int k_in, int k, float* scores,
                  int32_t* rows, uint64_t* keys_out, hipStream_t s) {
  if (n_lists <= 64 && k_in <= 32) {
    const int kc = kcap_for(k_in);
    const int vec16 = (k_in % 2 == 0 && (reinterpret_cast<uintptr_t>(in) & 15) == 0) ? 1 : 0;
    if (kc == 8)
      hipLaunchKernelGGL((merge_lane_lists_kernel<8>), dim3((unsigned)cdiv(B, 4)), dim3(256), 0, s, in, B, n_lists, k_in, k, vec16, scores, rows, keys_out);
    else if (kc == 16)
      hipLaunchKernelGGL((merge_lane_lists_kernel<16>), dim3((unsigned)cdiv(B, 4)), dim3(256), 0, s, in, B, n_lists, k_in, k, vec16, scores, rows, keys_out);
    else
      hipLaunchKernelGGL((merge_lane_lists_kernel<32>), dim3((unsigned)cdiv(B, 4)), dim3(256), 0, s, in, B, n_lists, k_in, k, vec16, scores, rows, keys_out);
    return;
  }
  if (n_lists <= 512 && n_lists * k_in <= kMergeBlockKeys) {
    static std::atomic<uint64_t> lds_attr{0};  // > 64 KiB dynamic LDS: opt in per device
    ensure_lds_attr(lds_attr, reinterpret_cast<const void*>(&merge_block_kernel), kMergeBlockKeys * 8);
    hipLaunchKernelGGL(merge_block_kernel, dim3(B), dim3(256), (size_t)n_lists * k_in * 8, s, in, n_lists, k_in,
                       k, scores, rows, keys_out);
    return;
  }
  if (n_lists <= 64 * kHeadSlots) {
    hipLaunchKernelGGL(merge_heads_kernel, dim3(B), dim3(64), 0, s, in, n_lists, k_in, k, scores, rows, keys_out);
    return;
  }
  switch (kcap_for(k)) {
    case 8:
      hipLaunchKernelGGL((merge_kernel<8>), dim3(B), dim3(64), 0, s, in, n_lists, k_in, k, scores, rows, keys_out);
      break;
    case 16:
      hipLaunchKernelGGL((merge_kernel<16>), dim3(B), dim3(64), 0, s, in, n_lists, k_in, k, scores, rows, keys_out);
      break;
    default:
      hipLaunchKernelGGL((merge_kernel<32>), dim3(B), dim3(64), 0, s, in, n_lists, k_in, k, scores, rows, keys_out);
      break;
  }
}

// k > AHR_MAX_K: every score of a chunk of queries (the 128x128 tile kernel in MODE_SCORES, into
// the candidate workspace), then radix_topk_kernel per query. Chunks bound the score buffer to
// 1 GiB.
template <int DT>
int run_query_large_k(ahr_index* ix, int B, int k, uint32_t row_base, float* scores, int32_t* rows,
                      uint64_t* keys, hipStream_t s) {
  const int64_t n = ix->count;
  const int64_t ld = cdiv(std::max<int64_t>(n, 1), 64) * 64;
  int64_t chunk = std::max<int64_t>(kTileQ, ((int64_t)1 << 28) / ld / kTileQ * kTileQ);
  chunk = std::min<int64_t>(chunk, cdiv(B, kTileQ) * kTileQ);
  int st = ensure_cand(ix, chunk * ld * (int64_t)sizeof(float));
  if (st) return st;
  float* sc = reinterpret_cast<float*>(ix->cand);
  static std::atomic<uint64_t> lds_attr{0};  // > 64 KiB dynamic LDS: opt in per device
  ensure_lds_attr(lds_attr, reinterpret_cast<const void*>(&topk_tile_kernel<DT, 8, MODE_SCORES>), kLdsBytes);
  const int n_row_tiles = (int)cdiv(n, kTileRows);
  prof_mark(ix, 1, s);
  prof_mark(ix, 2, s);
  for (int64_t c0 = 0; c0 < B; c0 += chunk) {
    const int nq = (int)std::min<int64_t>(chunk, B - c0);
    const int qblocks = (int)cdiv(nq, kTileQ);
    const int n_splits = std::max(1, std::min(n_row_tiles, kResidentSlots128 / qblocks));
    if (n > 0) {
      hipLaunchKernelGGL((topk_tile_kernel<DT, 8, MODE_SCORES>), dim3((unsigned)(n_splits * qblocks)), dim3(kThreads),
                         kLdsBytes, s, ix->rows, ix->qbuf + c0 * ix->row_stride, ix->row_stride, (int)n, nq,
                         ix->d_pad * ix->elem / kRowBytes, 1, n_row_tiles, row_base, k, (uint64_t*)nullptr,
                         (const float*)nullptr, sc, ld, n_splits, qblocks, 0);
    }
    hipLaunchKernelGGL(radix_topk_kernel, dim3((unsigned)nq), dim3(256), 0, s, sc, ld, (int)n, k, row_base, scores,
                       rows, keys, c0);
  }
  prof_mark(ix, 3, s);
  prof_mark(ix, 4, s);
  if (ix->prof_calls < ix->prof_max_calls) ++ix->prof_calls;
  AHR_HIP(hipGetLastError());
  return AHR_OK;
}

int run_query(ahr_index* ix, const float* q, int B, int k, int normalize_q, int64_t row_base,
              float* scores, int32_t* rows, uint64_t* keys, void* stream, const uint64_t** lists_out = nullptr,
              int* n_lists_out = nullptr) {
  if (lists_out) *lists_out = nullptr;
  if (!ix) return fail(AHR_EINVAL, "null index");
  if (B < 0 || k <= 0) return fail(AHR_EINVAL, "B must be >= 0 and k > 0");
  if (k > AHR_MAX_K_LARGE) return fail(AHR_EUNSUP, "k exceeds AHR_MAX_K_LARGE (4096)");
  if (B == 0) return AHR_OK;
  if (!q) return fail(AHR_EINVAL, "null query pointer");
  if (row_base < 0 || row_base + ix->count > 0xFFFFFFFFll)
    return fail(AHR_ERANGE, "row ids must fit in 32 bits");
  DeviceGuard dg(ix->device);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int st = ensure_query_ws(ix, B, k, s);
  if (st) return st;
  prof_mark(ix, 0, s);
  const int pre_kernel = k <= AHR_MAX_K && ix->count > 0 ? plan_search(ix, B, k).kernel : -1;
  const bool small_plan = pre_kernel == KERNEL_SMALL;
  // the register-resident plan's fragment-major query copy (qbuf_kb: the k-blocked copy's buffer)
  bool frag_done = false;
  if (pre_kernel == KERNEL_QRES) {
    if ((st = ensure_qbuf_kb(ix, s)) || (st = ensure_ss(ix, s))) return st;
    // the whole batch after the previous register-resident batch of another stream (ahr_index::qres_done)
    if (!qres_chain_at_kernel() && (st = qres_chain_wait(ix, s))) return st;
    if (small_fuses_convert(ix) && !normalize_q && qres_self_seeded(ix, plan_search(ix, B, k), k)) {
      // only the fragment-major copy: the self-seeded launch reads nothing else
      const int64_t n16 = cdiv(B, 32) * (ix->d_pad / 16) * 64;
      hipLaunchKernelGGL(frag_from_f32_kernel, dim3((unsigned)cdiv(n16, 256)), dim3(256), 0, s, q, (int64_t)B, ix->dim,
                         ix->d_pad, ix->dtype, n16, ix->qbuf_kb, reinterpret_cast<uint32_t*>(ix->ss + kQresTagOff));
      frag_done = true;
    } else if (small_fuses_convert(ix)) {  // one launch: rows + fragments
      hipLaunchKernelGGL(convert_queries_frag_kernel, dim3((unsigned)cdiv(B, 4)), dim3(256), 0, s, q, (int64_t)B,
                         ix->dim, normalize_q, ix->qbuf, ix->row_stride, ix->d_pad, ix->dtype, ix->qbuf_kb,
                         reinterpret_cast<uint32_t*>(ix->ss + kQresTagOff));
      frag_done = true;
    }
  }
  if (!frag_done && !(small_plan && small_plan_fuses_convert(ix)))
    hipLaunchKernelGGL(convert_rows_kernel, dim3((unsigned)cdiv(B, 4)), dim3(256), 0, s, q,
                       (int64_t)B, ix->dim, (const int64_t*)nullptr, (int64_t)0, normalize_q, ix->qbuf,
                       ix->row_stride, ix->d_pad, ix->dtype);
  if (pre_kernel == KERNEL_QRES && !frag_done)
    qres::launch_frag(ix->qbuf, ix->row_stride, B, ix->d_pad * ix->elem, ix->qbuf_kb,
                      reinterpret_cast<uint32_t*>(ix->ss + kQresTagOff), s);
  if (k > AHR_MAX_K) {
    switch (ix->dtype) {
      case AHR_BF16: return run_query_large_k<DT_BF16>(ix, B, k, (uint32_t)row_base, scores, rows, keys, s);
      case AHR_F16: return run_query_large_k<DT_F16>(ix, B, k, (uint32_t)row_base, scores, rows, keys, s);
      default: return run_query_large_k<DT_F32>(ix, B, k, (uint32_t)row_base, scores, rows, keys, s);
    }
  }
  SearchPlan p = plan_search(ix, B, k);
  const bool kb_plan = p.kernel == KERNEL_KB256;
  const bool cand_plan = p.kernel == KERNEL_QKV || p.kernel == KERNEL_T256 || kb_plan;
  if (cand_plan && ix->count > 0) {
    st = ensure_cand(ix, cand_bytes(B, p));
    if (st) return st;
  }
  if (kb_plan && ix->count > 0) {
    // the k-blocked copies exist only once the kb256 plan is used (opt-in): built here, on this
    // stream, the first time; upserts keep the corpus copy in step afterwards
    const int n_kb = ix->d_pad * ix->elem / kb256::kKB;
    if (!ix->rows_kb) {
      if (hipMalloc(&ix->rows_kb, ix->cap_pad * ix->row_stride) != hipSuccess)
        return fail(AHR_ENOMEM, "k-blocked corpus allocation failed");
      AHR_HIP(hipMemsetAsync(ix->rows_kb, 0, ix->cap_pad * ix->row_stride, s));
      const int64_t all = ix->count * n_kb * 4;
      hipLaunchKernelGGL(reblock_kb_kernel, dim3((unsigned)cdiv(all, 256)), dim3(256), 0, s, ix->rows,
                         ix->row_stride, (int64_t)0, ix->count, n_kb, ix->rows_kb);
    }
    if ((st = ensure_qbuf_kb(ix, s))) return st;
    const int64_t chunks = (int64_t)B * n_kb * 4;
    hipLaunchKernelGGL(reblock_kb_kernel, dim3((unsigned)cdiv(chunks, 256)), dim3(256), 0, s, ix->qbuf,
                       ix->row_stride, (int64_t)0, (int64_t)B, n_kb, ix->qbuf_kb);
  }
  // single searches (the drop-in's search() and environment resets): the small kernels merge the
  // splits in their last workgroup, no merge launch
  // The last-workgroup fold is opt-in (kFlagFold): the merge launch measured faster from round 5
  // (fp32 B = 1 two in flight 25.2-25.7 k vs 21.6-22.0 k queries/s, bf16 41.9-42.0 k vs 36.9-37.3 k,
  // serial equal: the next batch's stream overlaps the merge, while the fold's tail holds the kernel)
  const bool fold = ix->count > 0 && p.kernel == KERNEL_SMALL && B <= kFoldMaxQ &&
                    (int64_t)B * p.n_splits * k * 8 + 16 <= kFoldMaxLds && p.n_splits <= 512 &&
                    (ix->debug_flags & kFlagFold) && !(ix->debug_flags & kFlagNoFold);
  const FoldOut fo{ix->fold_ctr(), scores, rows, keys};
  // (AHR_QRES_CHAIN=kernel: only the kernels of two streams' register-resident batches are ordered,
  // so one batch's merge and the next one's query conversion overlap the other's kernel)
  const bool chain_k = p.kernel == KERNEL_QRES && qres_chain_at_kernel();
  if (chain_k && (st = qres_chain_wait(ix, s))) return st;
  if (ix->count > 0) {
    switch (ix->dtype) {
      case AHR_BF16: launch_search<DT_BF16>(ix, p, B, k, (uint32_t)row_base, q, normalize_q, fold ? &fo : nullptr, s); break;
      case AHR_F16: launch_search<DT_F16>(ix, p, B, k, (uint32_t)row_base, q, normalize_q, fold ? &fo : nullptr, s); break;
      default: launch_search<DT_F32>(ix, p, B, k, (uint32_t)row_base, q, normalize_q, fold ? &fo : nullptr, s); break;
    }
  } else {
    prof_mark(ix, 1, s);
    prof_mark(ix, 2, s);
  }
  if (chain_k && (st = qres_chain_record(ix, s))) return st;
  prof_mark(ix, 3, s);
  if (!fold) {
    // qkv: one list per (split, dimension half); t256 / kb256: one per (split, row half)
    const int lists = (cand_plan ? 2 : 1) *
                      p.n_splits;
    // (dense_query_lists: a small-batch plan's lists go to the caller's fused merge instead; not
    // while stage events are being recorded, whose merge stage would be empty)
    if (lists_out && ix->count > 0 && p.kernel == KERNEL_SMALL && row_base == 0 &&
        (int64_t)lists * k <= kRerankFuseKeys && lists <= 512 && ix->prof_calls >= ix->prof_max_calls) {
      *lists_out = ix->part;
      *n_lists_out = lists;
    } else {
      launch_merge(ix->part, B, ix->count > 0 ? lists : 0, k, k, scores, rows, keys, s);
    }
  }
  // the next register-resident launch of another stream waits for this batch's merge
  if (p.kernel == KERNEL_QRES && !qres_chain_at_kernel() && (st = qres_chain_record(ix, s))) return st;
  prof_mark(ix, 4, s);
  if (ix->prof_calls < ix->prof_max_calls) ++ix->prof_calls;
  AHR_HIP(hipGetLastError());
  return AHR_OK;
}

}  // namespace

namespace ahr {

int dense_query_lists(ahr_index* ix, const float* q, int B, int k, int normalize_q, float* scores, int32_t* rows,
                      void* stream, const uint64_t** lists, int* n_lists) {
  if (!scores || !rows || !lists || !n_lists) return fail(AHR_EINVAL, "null output");
  return run_query(ix, q, B, k, normalize_q, 0, scores, rows, nullptr, stream, lists, n_lists);
}

}  // namespace ahr

extern "C" {

int ahr_index_create(int dim, int dtype, int64_t capacity, int device, ahr_index** out) {
  if (!out) return fail(AHR_EINVAL, "null out pointer");
  *out = nullptr;
  if (dim <= 0 || capacity < 0) return fail(AHR_EINVAL, "dim must be > 0 and capacity >= 0");
  if (dtype != AHR_F32 && dtype != AHR_F16 && dtype != AHR_BF16) return fail(AHR_EINVAL, "unknown dtype");
  DeviceGuard dg(device);
  ahr_index* ix = new ahr_index();
  ix->dim = dim;
  ix->dtype = dtype;
  ix->elem = dtype == AHR_F32 ? 4 : 2;
  // A k-tile is 128 B of a row: 64 half-precision or 32 fp32 lanes.
  const int lanes_per_ktile = kRowBytes / ix->elem;
  ix->d_pad = (int)cdiv(dim, lanes_per_ktile) * lanes_per_ktile;
  ix->device = device;
  ix->capacity = capacity;
  ix->cap_pad = std::max<int64_t>(kRowPad, cdiv(capacity, kRowPad) * kRowPad);
  ix->row_stride = (int64_t)ix->d_pad * ix->elem;
  if (hipMalloc(&ix->rows, ix->cap_pad * ix->row_stride) != hipSuccess) {
    delete ix;
    return fail(AHR_ENOMEM, "corpus allocation failed");
  }
  // zeroed before any stream (also non-blocking ones) writes rows into it
  if (hipMemset(ix->rows, 0, ix->cap_pad * ix->row_stride) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    (void)hipFree(ix->rows);
    delete ix;
    return fail(AHR_EHIP, "corpus memset failed");
  }
  *out = ix;
  return AHR_OK;
}

int ahr_index_destroy(ahr_index* ix) {
  if (!ix) return AHR_OK;
  DeviceGuard dg(ix->device);
  if (ix->rows) (void)hipFree(ix->rows);
  if (ix->rows_kb) (void)hipFree(ix->rows_kb);
  if (ix->qbuf) (void)hipFree(ix->qbuf);
  if (ix->qbuf_kb) (void)hipFree(ix->qbuf_kb);
  if (ix->part) (void)hipFree(ix->part);
  if (ix->sample) (void)hipFree(ix->sample);
  if (ix->cand) (void)hipFree(ix->cand);
  if (ix->ss) (void)hipFree(ix->ss);
  for (int w = 0; w < kMaxWorkspaces; ++w) {
    if (w == ix->cur_ws) continue;
    if (ix->parked[w].qbuf) (void)hipFree(ix->parked[w].qbuf);
    if (ix->parked[w].qbuf_kb) (void)hipFree(ix->parked[w].qbuf_kb);
    if (ix->parked[w].part) (void)hipFree(ix->parked[w].part);
    if (ix->parked[w].sample) (void)hipFree(ix->parked[w].sample);
    if (ix->parked[w].cand) (void)hipFree(ix->parked[w].cand);
    if (ix->parked[w].ss) (void)hipFree(ix->parked[w].ss);
  }
  for (hipEvent_t e : ix->prof_events) (void)hipEventDestroy(e);
  if (ix->qres_done) (void)hipEventDestroy(ix->qres_done);
  delete ix;
  return AHR_OK;
}

int ahr_index_upsert(ahr_index* ix, const float* vecs, int64_t n, const int64_t* slots,
                     int64_t start_slot, int normalize, void* stream) {
  if (!ix) return fail(AHR_EINVAL, "null index");
  if (n < 0) return fail(AHR_EINVAL, "n must be >= 0");
  if (n == 0) return AHR_OK;
  if (!vecs) return fail(AHR_EINVAL, "null vectors");
  DeviceGuard dg(ix->device);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int64_t hi = start_slot + n;
  if (slots) {
    // Slots are device data; the caller guarantees range. We need the max for `count`:
    // read back (synchronous on this stream) — upsert is the ingest path, not the query path.
    int64_t* hslots = new int64_t[n];
    hipError_t e = hipMemcpyAsync(hslots, slots, n * sizeof(int64_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
      delete[] hslots;
      return hip_fail(e, "slot readback");
    }
    hi = 0;
    for (int64_t i = 0; i < n; ++i) {
      if (hslots[i] < 0 || hslots[i] >= ix->capacity) {
        delete[] hslots;
        return fail(AHR_ERANGE, "slot out of range");
      }
      hi = std::max(hi, hslots[i] + 1);
    }
    delete[] hslots;
  } else if (start_slot < 0 || hi > ix->capacity) {
    return fail(AHR_ERANGE, "slot range exceeds capacity");
  }
  hipLaunchKernelGGL(convert_rows_kernel, dim3((unsigned)cdiv(n, 4)), dim3(256), 0, s, vecs, n,
                     ix->dim, slots, start_slot, normalize, ix->rows, ix->row_stride, ix->d_pad,
                     ix->dtype);
  if (ix->rows_kb) {
    // the k-blocked copy of the rows just written (scattered slots: every row below the highest)
    const int64_t lo = slots ? 0 : start_slot;
    const int n_kb = ix->d_pad * ix->elem / kb256::kKB;
    const int64_t chunks = (hi - lo) * n_kb * 4;
    hipLaunchKernelGGL(reblock_kb_kernel, dim3((unsigned)cdiv(chunks, 256)), dim3(256), 0, s, ix->rows,
                       ix->row_stride, lo, hi - lo, n_kb, ix->rows_kb);
  }
  AHR_HIP(hipGetLastError());
  ix->count = std::max(ix->count, hi);
  return AHR_OK;
}

int ahr_index_truncate(ahr_index* ix, int64_t new_count) {
  if (!ix) return fail(AHR_EINVAL, "null index");
  if (new_count < 0 || new_count > ix->capacity) return fail(AHR_ERANGE, "count out of range");
  ix->count = new_count;
  return AHR_OK;
}

int ahr_index_count(const ahr_index* ix, int64_t* count) {
  if (!ix || !count) return fail(AHR_EINVAL, "null argument");
  *count = ix->count;
  return AHR_OK;
}

int ahr_index_info(const ahr_index* ix, int* dim, int* dtype, int64_t* capacity, int* padded_dim,
                   int64_t* row_bytes) {
  if (!ix) return fail(AHR_EINVAL, "null index");
  if (dim) *dim = ix->dim;
  if (dtype) *dtype = ix->dtype;
  if (capacity) *capacity = ix->capacity;
  if (padded_dim) *padded_dim = ix->d_pad;
  if (row_bytes) *row_bytes = ix->row_stride;
  return AHR_OK;
}

int ahr_index_rows(const ahr_index* ix, const void** dev_rows) {
  if (!ix || !dev_rows) return fail(AHR_EINVAL, "null argument");
  *dev_rows = ix->rows;
  return AHR_OK;
}

int ahr_index_read(const ahr_index* ix, int64_t start, int64_t n, float* out, void* stream) {
  if (!ix || (n > 0 && !out)) return fail(AHR_EINVAL, "null argument");
  if (start < 0 || n < 0 || start + n > ix->count) return fail(AHR_ERANGE, "read range outside live rows");
  if (n == 0) return AHR_OK;
  DeviceGuard dg(ix->device);
  hipLaunchKernelGGL(read_rows_kernel, dim3((unsigned)cdiv(n, 4)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), ix->rows, start, n, ix->dim,
                     ix->row_stride, ix->dtype, out);
  AHR_HIP(hipGetLastError());
  return AHR_OK;
}

int ahr_index_profile_begin(ahr_index* ix, int max_calls) {
  if (!ix || max_calls < 0) return fail(AHR_EINVAL, "bad profile request");
  DeviceGuard dg(ix->device);
  for (hipEvent_t e : ix->prof_events) (void)hipEventDestroy(e);
  ix->prof_events.clear();
  ix->prof_events.resize((size_t)max_calls * (kStages + 1));
  for (auto& e : ix->prof_events) AHR_HIP(hipEventCreate(&e));
  ix->prof_max_calls = max_calls;
  ix->prof_calls = 0;
  return AHR_OK;
}

int ahr_index_profile_end(ahr_index* ix, float* stage_ms_sum, int* n_calls) {
  if (!ix) return fail(AHR_EINVAL, "null index");
  DeviceGuard dg(ix->device);
  float sum[kStages] = {0, 0, 0, 0};
  for (int c = 0; c < ix->prof_calls; ++c) {
    hipEvent_t* ev = &ix->prof_events[(size_t)c * (kStages + 1)];
    AHR_HIP(hipEventSynchronize(ev[kStages]));
    for (int st = 0; st < kStages; ++st) {
      float ms = 0.f;
      AHR_HIP(hipEventElapsedTime(&ms, ev[st], ev[st + 1]));
      sum[st] += ms;
    }
  }
  if (stage_ms_sum)
    for (int st = 0; st < kStages; ++st) stage_ms_sum[st] = sum[st];
  if (n_calls) *n_calls = ix->prof_calls;
  for (hipEvent_t e : ix->prof_events) (void)hipEventDestroy(e);
  ix->prof_events.clear();
  ix->prof_max_calls = 0;
  ix->prof_calls = 0;
  return AHR_OK;
}

int ahr_index_set_sample_rows(ahr_index* ix, int rows) {
  if (!ix) return fail(AHR_EINVAL, "null index");
  if (rows < -1 || rows > kSampleMax || (rows > 0 && ((rows & (rows - 1)) || rows < 256)))
    return fail(AHR_EINVAL, "sample rows must be -1 (automatic), 0 or a power of two in [256, 65536]");
  ix->sample_rows = rows;
  return AHR_OK;
}

int ahr_index_probe_seed(ahr_index* ix, const float* q, int B, int k, int normalize_q, const uint64_t* cluster_keys,
                         int P, const int64_t* list_off, const int32_t* list_rows, int min_rows, float* thr,
                         void* stream) {
  if (!ix) return fail(AHR_EINVAL, "null index");
  if (B < 0 || k <= 0 || P <= 0 || min_rows <= 0) return fail(AHR_EINVAL, "B >= 0, k, P, min_rows > 0 required");
  if (ix->dtype == AHR_F32) return fail(AHR_EUNSUP, "cluster probe seeds: bf16 / f16 indexes");
  if (ix->dim > kProbeMaxDim || k > kProbeMaxRows || P > 64)
    return fail(AHR_EUNSUP, "dim <= 1024, k <= 256 and P <= 64 (one lane per offered cluster)");
  if (B == 0) return AHR_OK;
  if (!q || !cluster_keys || !list_off || !list_rows || !thr) return fail(AHR_EINVAL, "null buffer");
  DeviceGuard dg(ix->device);
  hipLaunchKernelGGL(probe_seed_kernel, dim3((unsigned)B), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     ix->rows, ix->row_stride, ix->dtype, ix->dim, ix->count, q, normalize_q, cluster_keys, P,
                     list_off, list_rows, std::min(min_rows, kProbeMaxRows), k, thr);
  AHR_HIP(hipGetLastError());
  return AHR_OK;
}

int ahr_index_set_seed(ahr_index* ix, const float* thr) {
  if (!ix) return fail(AHR_EINVAL, "null index");
  ix->seed = thr;
  return AHR_OK;
}

int ahr_index_set_debug_flags(ahr_index* ix, uint32_t flags) {
  if (!ix) return fail(AHR_EINVAL, "null index");
  if (flags & ~(kKnownFlags | kFlagXcdRemap)) return fail(AHR_EINVAL, "unknown debug flag bits");
  // The cost-split switches give wrong results by design; only the ablation build
  // (__graft_entry__.build_ablation, -DAHR_ABLATION) accepts them, the shipped library refuses.
#ifndef AHR_ABLATION
  if (flags & kWrongResultFlags)
    return fail(AHR_EUNSUP, "result-corrupting ablation flags need the AHR_ABLATION build");
#endif
  ix->debug_flags = flags & kKnownFlags;
  return AHR_OK;
}

int ahr_index_set_workspace(ahr_index* ix, int slot) {
  if (!ix) return fail(AHR_EINVAL, "null index");
  if (slot < 0 || slot >= kMaxWorkspaces) return fail(AHR_EINVAL, "workspace slot out of range");
  if (slot == ix->cur_ws) return AHR_OK;
  ahr_query_ws& out = ix->parked[ix->cur_ws];
  out.qbuf = ix->qbuf;
  out.qbuf_kb = ix->qbuf_kb;
  out.q_cap = ix->q_cap;
  out.part = ix->part;
  out.part_cap = ix->part_cap;
  out.sample = ix->sample;
  out.sample_cap = ix->sample_cap;
  out.cand = ix->cand;
  out.cand_cap = ix->cand_cap;
  out.ss = ix->ss;
  out.ss_cap = ix->ss_cap;
  ahr_query_ws& in = ix->parked[slot];
  ix->qbuf = in.qbuf;
  ix->qbuf_kb = in.qbuf_kb;
  ix->q_cap = in.q_cap;
  ix->part = in.part;
  ix->part_cap = in.part_cap;
  ix->sample = in.sample;
  ix->sample_cap = in.sample_cap;
  ix->cand = in.cand;
  ix->cand_cap = in.cand_cap;
  ix->ss = in.ss;
  ix->ss_cap = in.ss_cap;
  in = ahr_query_ws{};
  ix->cur_ws = slot;
  return AHR_OK;
}

int ahr_index_plan(const ahr_index* ix, int B, int k, int* kernel, int* n_splits, int* tiles_per_split,
                   int* qblocks) {
  if (!ix || B <= 0 || k <= 0 || k > AHR_MAX_K) return fail(AHR_EINVAL, "bad plan request");
  SearchPlan p = plan_search(ix, B, k);
  if (kernel) *kernel = p.kernel;
  if (n_splits) *n_splits = p.n_splits;
  if (tiles_per_split) *tiles_per_split = p.tiles_per_split;
  if (qblocks) *qblocks = p.qblocks;
  return AHR_OK;
}

int ahr_index_reserve(ahr_index* ix, int max_batch, int max_k) {
  if (!ix) return fail(AHR_EINVAL, "null index");
  if (max_batch <= 0 || max_k <= 0 || max_k > AHR_MAX_K) return fail(AHR_EINVAL, "bad reserve sizes");
  DeviceGuard dg(ix->device);
  int st = ensure_query_ws(ix, max_batch, max_k, nullptr);
  if (st) return st;
  // the plan-specific buffers at the current corpus size: candidate groups (qkv, t256, kb256), the
  // second query buffer (kb256, qres256) and the self-seeding granules (qres256)
  for (int kk = 1; kk <= max_k; kk = kk < 8 ? 8 : kk + 8) {
    const SearchPlan p = plan_search(ix, max_batch, kk);
    if (p.kernel == KERNEL_QKV || p.kernel == KERNEL_T256 || p.kernel == KERNEL_KB256) {
      st = ensure_cand(ix, cand_bytes(max_batch, p));
      if (st) return st;
    }
    if (p.kernel == KERNEL_KB256 || p.kernel == KERNEL_QRES) {
      if ((st = ensure_qbuf_kb(ix, nullptr))) return st;
    }
    if (p.kernel == KERNEL_QRES) {
      if ((st = ensure_ss(ix, nullptr))) return st;
    }
  }
  AHR_HIP(hipDeviceSynchronize());  // zeroing done before any stream uses the workspace
  return AHR_OK;
}

int ahr_index_query(ahr_index* ix, const float* q, int B, int k, int normalize_q, float* scores,
                    int32_t* rows, void* stream) {
  if (!scores || !rows) return fail(AHR_EINVAL, "null output");
  return run_query(ix, q, B, k, normalize_q, 0, scores, rows, nullptr, stream);
}

int ahr_index_query_keys(ahr_index* ix, const float* q, int B, int k, int normalize_q,
                         int64_t row_base, uint64_t* keys, void* stream) {
  if (!keys) return fail(AHR_EINVAL, "null output");
  return run_query(ix, q, B, k, normalize_q, row_base, nullptr, nullptr, keys, stream);
}

int ahr_index_scores(ahr_index* ix, const float* q, int B, int normalize_q, float* out, int64_t ld, void* stream) {
  if (!ix) return fail(AHR_EINVAL, "null index");
  if (B < 0) return fail(AHR_EINVAL, "B must be >= 0");
  if (ld < ix->count) return fail(AHR_EINVAL, "ld must be >= the row count");
  if (B == 0 || ix->count == 0) return AHR_OK;
  if (!q || !out) return fail(AHR_EINVAL, "null buffer");
  DeviceGuard dg(ix->device);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int st = ensure_query_ws(ix, B, 1, s);
  if (st) return st;
  hipLaunchKernelGGL(convert_rows_kernel, dim3((unsigned)cdiv(B, 4)), dim3(256), 0, s, q, (int64_t)B, ix->dim,
                     (const int64_t*)nullptr, (int64_t)0, normalize_q, ix->qbuf, ix->row_stride, ix->d_pad,
                     ix->dtype);
  const int n = (int)ix->count;
  const int n_row_tiles = (int)cdiv(n, kTileRows);
  const int qblocks = (int)cdiv(B, kTileQ);
  const int n_splits = std::max(1, std::min(n_row_tiles, kResidentSlots128 / qblocks));
  switch (ix->dtype) {
    case AHR_BF16:
      launch_tile<DT_BF16, 8, MODE_SCORES>(ix, n_splits, qblocks, 1, n_row_tiles, n, B, 1, 0, nullptr, out, ld, 0, s);
      break;
    case AHR_F16:
      launch_tile<DT_F16, 8, MODE_SCORES>(ix, n_splits, qblocks, 1, n_row_tiles, n, B, 1, 0, nullptr, out, ld, 0, s);
      break;
    default:
      launch_tile<DT_F32, 8, MODE_SCORES>(ix, n_splits, qblocks, 1, n_row_tiles, n, B, 1, 0, nullptr, out, ld, 0, s);
      break;
  }
  AHR_HIP(hipGetLastError());
  return AHR_OK;
}

int ahr_topk_merge(const uint64_t* keys_in, int B, int n_lists, int k_in, int k, float* scores,
                   int32_t* rows, uint64_t* keys_out, void* stream) {
  if (B < 0 || n_lists < 0 || k_in < 0 || k <= 0) return fail(AHR_EINVAL, "bad merge shape");
  if (k > AHR_MAX_K_LARGE) return fail(AHR_EUNSUP, "k exceeds AHR_MAX_K_LARGE (4096)");
  if (B == 0) return AHR_OK;
  if (!keys_in && n_lists * k_in > 0) return fail(AHR_EINVAL, "null keys");
  if (k > AHR_MAX_K || k_in > AHR_MAX_K)
    hipLaunchKernelGGL(radix_topk_keys_kernel, dim3((unsigned)B), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       keys_in, n_lists * k_in, k, scores, rows, keys_out);
  else
    launch_merge(keys_in, B, n_lists, k_in, k, scores, rows, keys_out, reinterpret_cast<hipStream_t>(stream));
  AHR_HIP(hipGetLastError());
  return AHR_OK;
}

int ahr_key_decode(const uint64_t* keys, int64_t n, float* scores, int64_t* rows) {
  if (n < 0 || (n > 0 && !keys)) return fail(AHR_EINVAL, "bad decode args");
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t k = keys[i];
    if (scores) scores[i] = k ? key_score(k) : -INFINITY;
    if (rows) rows[i] = k ? (int64_t)key_row(k) : -1;
  }
  return AHR_OK;
}

}  // extern "C"
