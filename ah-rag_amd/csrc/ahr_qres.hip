// ahr_qres.hip — query-resident fused Q·Nᵀ + exact top-k for gfx950 (MI355X): the B ≥ 512 bf16/f16
// path behind HierarchicalGraph.search_batch / the C2 headline (reference
// src/ah_rag/graph/hierarchical_graph.py:714, Chroma `collection.query`).
//
// Why this shape. The 128 x 128 two-operand tile kernels stream 1 byte into LDS per 64 flops;
// at C2 that is ~8.6 MB per CU per launch, which the per-CU L2 -> LDS delivery (~69 GB/s
// measured) cannot feed faster than ~124 us (the GEMM-only time of topk_tilelane_kernel). Here
// a workgroup keeps 256 queries resident in VGPRs for the whole launch — wave w holds the B
// fragments of queries 32w .. 32w + 31 over the WHOLE dimension (48 x 16 B per lane at
// d = 768, 192 VGPRs) — and only the corpus streams: 1 byte per 256 flops, 4x fewer than the
// tile kernels. Every wave multiplies every 32-row corpus block (the A operand, read from LDS)
// against its own queries with one v_mfma_f32_32x32x16 chain per block (48 steps), so a corpus
// byte brought in is used by 8 waves.
//
// * Corpus: 32-row blocks, each split into two stages of 6 k-tiles (64-deep, 128 B per row:
//   24 KiB); a 4-slot ring filled by buffer LDS-DMA three stages ahead (1-KiB pieces of 8 whole
//   128-B rows, 3 per wave per stage), the XOR chunk swizzle of the tile kernels (conflict-free
//   ds_read_b128). One barrier per stage.
// * Scores: the k-order, fragment map and accumulation chain of topk_tilelane_kernel (step s of
//   a row covers k = [16 s, 16 s + 16), lane half fh holding 8 of them; the chain starts from 0),
//   so every score is bitwise the tile kernel's.
// * Top-k: a lane holds one query column x 16 rows of each block. Its 16 scores are screened
//   against the lane's threshold (the pre-pass seed, then the lane's own k-th best): the block
//   max in the common case, and for the rare passing scores one 8-B append to the lane's
//   16-entry LDS buffer. A full buffer is compacted in place to its k best, which raises the
//   threshold. At the end each lane sorts its buffer into a register list (the query registers
//   are dead by then) and the two lanes of a query merge: one list per (query, split).
// * Query fragments come from a fragment-major copy of the converted queries (launch_frag):
//   one coalesced 1-KiB load per wave per k16 step.
// * Budget: 192 query VGPRs + 16 accumulators + fragments in flight <= 256 (two waves per SIMD,
//   one workgroup of 8 waves per CU); LDS 96 KiB ring + 64 KiB lane buffers = 160 KiB.
#include "ahr_dense_common.h"
#include "ahr_qres.h"

#include <atomic>
#include <math.h>
#include <type_traits>

namespace ahr {
namespace dense {
namespace qres {

constexpr int kWaves = 8;
constexpr int kThreads = kWaves * 64;
constexpr int kKt = kTR * kRowBytes;  // 4 KiB: one 64-deep k-tile of a 32-row block
constexpr int kSlots = 4;             // ring stages: the one multiplied + 3 in flight

template <int NKT>
struct Cfg {
  static_assert(NKT % 2 == 0, "two stages per block");
  static constexpr int kSK = NKT / 2;          // k-tiles per stage
  static constexpr int kStage = kSK * kKt;     // 24 KiB at d_pad = 768
  static constexpr int kPieces = kSK * 4;      // 1-KiB DMA pieces per stage (8 rows x 128 B)
  static_assert(kPieces % kWaves == 0, "equal DMA share per wave");
  static constexpr int kPPW = kPieces / kWaves;  // pieces per wave per stage
  static constexpr int kNS = NKT * 4;          // k16 steps = query fragments per lane
  static constexpr int kSS = kSK * 4;          // k16 steps per stage
  static constexpr int kOffBuf = kSlots * kStage;
  static constexpr int kLds = kOffBuf + kBufCap * kThreads * 8;
};
static_assert(Cfg<12>::kLds <= 160 * 1024, "LDS budget: one workgroup per CU");

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__global__ __launch_bounds__(256) void frag_kernel(const uint8_t* __restrict__ qbuf, int64_t row_stride, int64_t n16,
                                                   int ns, uint8_t* __restrict__ qfrag) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // one 16-B chunk of the output
  if (i >= n16) return;
  const int l = (int)(i & 63);
  const int64_t gs = i >> 6;
  const int S = (int)(gs % ns);
  const int64_t q = (gs / ns) * 32 + (l & 31);
  const u32x4 v = *reinterpret_cast<const u32x4*>(qbuf + q * row_stride + S * 32 + (l >> 5) * 16);
  *reinterpret_cast<u32x4*>(qfrag + i * 16) = v;
}

// ABL: cost-split switches of the ablation build (always 0 in the shipped library): 1 = no top-k
// screening, 2 = no corpus DMA after the first stages, 4 = no DMA waits, 8 = no stage barriers,
// 16 = no LDS fragment reads (a register stands in). Compile-time, so the production code path is
// the ABL = 0 instantiation untouched. Every nonzero combination gives wrong results.
enum { ABL_NOSCREEN = 1, ABL_NOLOADS = 2, ABL_NOWAIT = 4, ABL_NOBARRIER = 8, ABL_NOREAD = 16 };

template <int DT, int NKT, int KCAP, bool STAGGER, int SCR, int ABL>
__global__ __launch_bounds__(kThreads, 2) void topk_qres_kernel(
    const uint8_t* __restrict__ corpus, const uint8_t* __restrict__ qfrag, int64_t row_stride, int n_rows, int n_q,
    uint32_t row_base, int k_out, uint64_t* __restrict__ part_keys, const float* __restrict__ thr_init, int n_splits,
    int qblocks, int flags) {
  using C = Cfg<NKT>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int fr = lane & 31;
  const int fh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int split, qb;
  if (flags & kFlagXcdRemap) {  // the query blocks of a split on one XCD: its corpus comes from HBM once
    const int x = blockIdx.x & 7;
    const int i = blockIdx.x >> 3;
    split = (i / qblocks) * 8 + x;
    qb = i % qblocks;
  } else {
    split = blockIdx.x % n_splits;
    qb = blockIdx.x / n_splits;
  }
  const int n_blocks = (n_rows + kTR - 1) / kTR;
  const int b_begin = (int)((int64_t)split * n_blocks / n_splits);
  const int b_end = (int)((int64_t)(split + 1) * n_blocks / n_splits);
  const int n_st = 2 * (b_end - b_begin);
  const int qw0 = qb * kTQ + wave * 32;
  const bool live = qw0 < n_q;  // wave-uniform: a wave past the batch only stages and syncs
  const int q = qw0 + fr;

  float thr = q < n_q ? (thr_init ? thr_init[q] : -INFINITY) : INFINITY;

  // DMA: piece p = wave + 8 i of a stage is k-tile p / 4, rows 8 (p % 4) .. +8; lane l lands at
  // (row 8 (p % 4) + l / 8, physical chunk l % 8) and loads logical chunk (l % 8) ^ swz(row)
  uint32_t src_off[C::kPPW];
  int dst_off[C::kPPW];
#pragma unroll
  for (int i = 0; i < C::kPPW; ++i) {
    const int p = wave + kWaves * i;
    const int row = 8 * (p & 3) + (lane >> 3);
    src_off[i] = (uint32_t)(row * row_stride) + (p >> 2) * kRowBytes + ((((lane & 7) ^ ((row >> 1) & 7))) << 4);
    dst_off[i] = (p >> 2) * kKt + (p & 3) * 1024;
  }
  const uint32_t blk_bytes = (uint32_t)(kTR * row_stride);
  auto issue = [&](int st) __attribute__((always_inline)) {
    const int b = b_begin + (st >> 1);
    const __amdgpu_buffer_rsrc_t r =
        tile_rsrc(corpus + (int64_t)b * kTR * row_stride + (st & 1) * C::kSK * kRowBytes, blk_bytes);
    unsigned char* slot = smem + (st & (kSlots - 1)) * C::kStage;
#pragma unroll
    for (int i = 0; i < C::kPPW; ++i) blds16(r, src_off[i], slot + dst_off[i]);
  };
  if (n_st > 0) issue(0);
  if (n_st > 1) issue(1);

  // resident B fragments: step S of query q = bytes [32 S + 16 fh, +16) of its row
  u32x4 qf[C::kNS];
  {
    const uint8_t* src = qfrag + (int64_t)(qb * kWaves + wave) * C::kNS * 1024 + lane * 16;
#pragma unroll
    for (int S = 0; S < C::kNS; ++S) qf[S] = *reinterpret_cast<const u32x4*>(src + S * 1024);
  }
  // The fragments and the seed are consumed here (one wait, behind the prologue DMA, both needed
  // before the first MFMA anyway), so the loop never waits on them: a use inside the loop would
  // make the waitcnt pass count the ring's in-flight pieces against them every stage.
#pragma unroll
  for (int S = 0; S < C::kNS; ++S) asm volatile("" : "+v"(qf[S]));
  asm volatile("" : "+v"(thr));
  uint64_t thk = (q < n_q && thr != -INFINITY) ? (((uint64_t)ord_f32(thr) << 32) - 1) : 0;

  // lane survivor buffer: entry c at lbuf[c * kThreads] (a wave's 64 lanes hit 64 consecutive u64)
  uint64_t* lbuf = reinterpret_cast<uint64_t*>(smem + C::kOffBuf) + tid;
  int nb = 0;
  // keep the k_out best buffered keys; the smallest kept is the lane's k-th best: new threshold
  auto compact = [&]() {
#pragma unroll 1
    while (nb > k_out) {
      int mi = 0;
      uint64_t mv = lbuf[0];
#pragma unroll 1
      for (int c = 1; c < nb; ++c) {
        const uint64_t v = lbuf[c * kThreads];
        if (v < mv) {
          mv = v;
          mi = c;
        }
      }
      lbuf[mi * kThreads] = lbuf[(nb - 1) * kThreads];
      --nb;
    }
    uint64_t mn = lbuf[0];
#pragma unroll 1
    for (int c = 1; c < nb; ++c) {
      const uint64_t v = lbuf[c * kThreads];
      mn = v < mn ? v : mn;
    }
    if (mn > thk) {
      thk = mn;
      thr = key_score(mn);
    }
  };
  // a block's 16 scores of this lane: rows r0 + 8 (j / 4) + 4 fh + j % 4.
  // SCR = 1 (default): quad maxima (the 4 rows of a register quad), then exec-masked tests of the
  // passing quads' scores, each passing score one append; a quad compacts first when its 4
  // possible appends might not fit. SCR = 0: a pass mask and a select chain per passing score.
  auto screen_quads = [&](const f32x16& acc, int r0) __attribute__((always_inline)) {
    float qm[4];
#pragma unroll
    for (int qd = 0; qd < 4; ++qd)
      qm[qd] = fmaxf(fmaxf(acc[4 * qd], acc[4 * qd + 1]), fmaxf(acc[4 * qd + 2], acc[4 * qd + 3]));
    if (fmaxf(fmaxf(qm[0], qm[1]), fmaxf(qm[2], qm[3])) < thr) return;
    const bool ragged = r0 + kTR > n_rows;  // wave-uniform: the last block only
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) {
      if (qm[qd] >= thr) {
        if (nb + 4 > kBufCap) compact();
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = acc[4 * qd + e];
          const uint32_t row = (uint32_t)(r0 + 8 * qd + 4 * fh + e);
          if (v >= thr && (!ragged || row < (uint32_t)n_rows)) {
            const uint64_t key = make_key(v, row_base + row);
            if (key > thk) {
              lbuf[nb * kThreads] = key;
              ++nb;
            }
          }
        }
      }
    }
  };
  auto screen_loop = [&](const f32x16& acc, int r0) __attribute__((always_inline)) {
    float m = fmaxf(acc[0], acc[1]);
#pragma unroll
    for (int j = 2; j < 16; ++j) m = fmaxf(m, acc[j]);
    if (m >= thr) {
      uint32_t pm = 0;
#pragma unroll
      for (int j = 0; j < 16; ++j) pm |= (acc[j] >= thr ? 1u : 0u) << j;
      if (r0 + kTR > n_rows) {  // the ragged last block only
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (r0 + 8 * (j >> 2) + 4 * fh + (j & 3) >= n_rows) pm &= ~(1u << j);
      }
      while (pm) {
        const int j = __builtin_ctz(pm);
        pm &= pm - 1;
        float v = acc[0];
#pragma unroll
        for (int jj = 1; jj < 16; ++jj) {
          int jx = jj;
          asm volatile("" : "+s"(jx));  // keep the select chain (an indexed read would go to scratch)
          v = (jx == j) ? acc[jj] : v;
        }
        const uint32_t row = (uint32_t)(r0 + 8 * (j >> 2) + 4 * fh + (j & 3));
        const uint64_t key = make_key(v, row_base + row);
        if (key > thk) {
          lbuf[nb * kThreads] = key;
          if (++nb == kBufCap) compact();
        }
      }
    }
  };

  // Waves 4-7 (the second wave of every SIMD) run one stage behind waves 0-3, so the two waves of a
  // SIMD never reach a block end together: a wave screens a finished block at the start of the
  // next interval, before its next MFMA, while its partner's MFMAs keep the SIMD's matrix pipe busy
  // (in lock-step both would stop the pipe for the screening at every block end).
  // Interval j (after sync j): waves 0-3 multiply stage j, waves 4-7 stage j - 1.
  // Sync j: this wave's pieces of stage j landed (stage j + 1 may stay in flight), then the
  // barrier: everyone's stage j landed, and everyone is done with stage j - 2 (waves 4-7 finished
  // it in interval j - 1), whose slot takes stage j + 2. A stage is issued two intervals ahead.
  auto stage_sync = [&](int j) __attribute__((always_inline)) {
    if (!(ABL & ABL_NOWAIT)) {
      if (j + 1 < n_st)
        wait_vm<C::kPPW>();
      else
        wait_vm<0>();
    }
    if (!(ABL & ABL_NOBARRIER)) lds_barrier();
    if (j + 2 < n_st && !((ABL & ABL_NOLOADS) && j >= 2)) issue(j + 2);
  };
  // A fragment of k16 step s of stage st: k-tile s / 4, chunk 2 (s % 4) + fh of row fr
  const int a_row = fr * kRowBytes;
  const int a_x = (fr >> 1) & 7;
  auto frag = [&](int st, int s) __attribute__((always_inline)) {
    if constexpr ((ABL & ABL_NOREAD) != 0) return qf[(s + 5) % C::kNS];  // MFMA + issue only
    const unsigned char* slot = smem + (st & (kSlots - 1)) * C::kStage;
    return *reinterpret_cast<const u32x4*>(slot + (s >> 2) * kKt + a_row + (((2 * (s & 3) + fh) ^ a_x) << 4));
  };
  static_assert(C::kSS % 3 == 0, "three fragment registers rotate evenly over a stage");
  const int lag = (STAGGER && wave >= 4) ? 1 : 0;
  constexpr bool skip_screen = (ABL & ABL_NOSCREEN) != 0;
  f32x16 acc;
  u32x4 fa[3];
  // the stage's 24 steps: step t prefetches step t + 2 and multiplies step t; H = block half
  auto stage_mma = [&](auto H, int st) __attribute__((always_inline)) {
    constexpr int h = decltype(H)::value;
#pragma unroll
    for (int t = 0; t < C::kSS; ++t) {
      if (t + 2 < C::kSS) fa[(t + 2) % 3] = frag(st, t + 2);
      __builtin_amdgcn_sched_barrier(0);
      if (h == 0 && t == 0) {
        f32x16 z = {};
        mfma_step<DT>(fa[0], qf[0], z);
        acc = z;
      } else {
        mfma_step<DT>(fa[t % 3], qf[h * C::kSS + t], acc);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto finish_block = [&](int st_done) __attribute__((always_inline)) {  // st_done: the block's 2nd stage
    if constexpr (skip_screen) {  // GEMM only: the chain kept live (rule 17), no top-k
      asm volatile("" ::"v"(acc));
      return;
    }
    if constexpr (SCR == 1)
      screen_quads(acc, (b_begin + (st_done >> 1)) * kTR);
    else
      screen_loop(acc, (b_begin + (st_done >> 1)) * kTR);
  };
#pragma unroll 1
  for (int j = 0; j <= n_st; ++j) {
    stage_sync(j);
    const int st = j - lag;
    if (!live) continue;
    const bool mma = st >= 0 && st < n_st;
    if (mma) {  // the stage's first fragments: in flight under the screening below
      fa[0] = frag(st, 0);
      fa[1] = frag(st, 1);
    }
    if (st >= 2 && !(st & 1)) finish_block(st - 1);  // the block that ended with stage st - 1
    if (mma) {
      if (st & 1)
        stage_mma(std::integral_constant<int, 1>{}, st);
      else
        stage_mma(std::integral_constant<int, 0>{}, st);
    }
  }
  if (live && lag && n_st > 0) finish_block(n_st - 1);  // waves 4-7: their last block

  // this lane's buffered keys, sorted (the query registers are dead from here on)
  uint64_t L[KCAP];
#pragma unroll
  for (int j = 0; j < KCAP; ++j) L[j] = 0;
#pragma unroll 1
  for (int c = 0; c < nb; ++c) list_insert<KCAP>(L, lbuf[c * kThreads]);
  // lane fr + 32 hands its list to lane fr through the (idle) ring
  __syncthreads();
  uint64_t* xch = reinterpret_cast<uint64_t*>(smem) + (wave * 32 + fr) * KCAP;
  if (fh) {
#pragma unroll
    for (int j = 0; j < KCAP; ++j) xch[j] = L[j];
  }
  __syncthreads();
  if (!fh && q < n_q) {
#pragma unroll 1
    for (int j = 0; j < k_out; ++j) {
      const uint64_t v = xch[j];
      if (v <= L[KCAP - 1]) break;  // sorted: nothing further can enter
      list_insert<KCAP>(L, v);
    }
    uint64_t* dst = part_keys + ((int64_t)q * n_splits + split) * k_out;
#pragma unroll
    for (int j = 0; j < KCAP; ++j)
      if (j < k_out) dst[j] = L[j];
  }
}

// =============================================================================================
// topk_qres16_kernel: the same structure with v_mfma_f32_16x16x32 (opt-in, kFlagQres16). MI355X holds a
// higher clock under 16x16x32 than under 32x32x16 on random operands (tools/mfma_probe.hip: 1.81-1.91
// vs 1.43-1.64 PFLOP/s at full issue), at the same operand bytes and registers: a wave's 32 queries
// are two 16-query groups (B fragments of k32 step s: query 16g + l % 16, bytes [64 s + 16 (l / 16),
// +16)), a block's 32 rows two 16-row halves (A fragment: row 16 rh + l % 16, 16-B chunk
// 4 (s % 2) + l / 16 of its 64-deep k-tile), 4 MFMAs per k32 step into acc[rh][g]. Step order,
// fragment map and the chain from 0 are topk_t256_kernel's / topk_kb256_kernel's, so the scores
// are bitwise theirs.
// A lane holds 2 queries (g) x 8 rows of each block (rows 16 rh + 4 (l / 16) + r) and keeps one
// survivor buffer per query in LDS (kLaneCap keys); a full buffer is compacted to its k best, which
// raises that lane's threshold for the query. At the end each lane sorts its two buffers into
// register lists and the 4 lanes of a query (lane quarters) merge theirs.
// Ring: 3 slots (the stage multiplied, the next in flight, the one after issued at the stage's
// start): 72 KiB, and 88 KiB of lane buffers.
// =============================================================================================
constexpr int kLaneCap = 11;  // keys per (lane, query): k <= 10 leaves one free slot after a compaction
constexpr int kSlots16 = 3;

template <int NKT>
struct Cfg16 {
  static constexpr int kSK = NKT / 2;           // k-tiles per stage
  static constexpr int kStage = kSK * kKt;      // 24 KiB at d_pad = 768
  static constexpr int kPieces = kSK * 4;
  static_assert(kPieces % kWaves == 0, "equal DMA share per wave");
  static constexpr int kPPW = kPieces / kWaves;
  static constexpr int kNS = NKT * 2;           // k32 steps
  static constexpr int kSS = kSK * 2;           // k32 steps per stage
  static constexpr int kOffBuf = kSlots16 * kStage;  // [g][kLaneCap][512 lanes] u64
  static constexpr int kLds = kOffBuf + 2 * kLaneCap * kThreads * 8;
};
static_assert(Cfg16<12>::kLds <= 160 * 1024, "LDS budget: one workgroup per CU");

template <int DT>
__device__ __forceinline__ void mfma16(const u32x4& a, const u32x4& b, f32x4& acc) {
  if constexpr (DT == DT_BF16)
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc, 0,
                                                  0, 0);
  else
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), acc, 0, 0,
                                                 0);
}

template <int N, typename F, int I = 0>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, F, I + 1>(static_cast<F&&>(f));
  }
}

__global__ __launch_bounds__(256) void frag16_kernel(const uint8_t* __restrict__ qbuf, int64_t row_stride, int64_t n16,
                                                     int ns, uint8_t* __restrict__ qfrag) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // one 16-B chunk of the output
  if (i >= n16) return;
  const int l = (int)(i & 63);
  const int64_t gs = i >> 6;
  const int S = (int)(gs % ns);
  const int64_t q = (gs / ns) * 16 + (l & 15);
  const u32x4 v = *reinterpret_cast<const u32x4*>(qbuf + q * row_stride + S * 64 + (l >> 4) * 16);
  *reinterpret_cast<u32x4*>(qfrag + i * 16) = v;
}

template <int DT, int NKT, int KCAP, int ABL>
__global__ __launch_bounds__(kThreads, 2) void topk_qres16_kernel(
    const uint8_t* __restrict__ corpus, const uint8_t* __restrict__ qfrag, int64_t row_stride, int n_rows, int n_q,
    uint32_t row_base, int k_out, uint64_t* __restrict__ part_keys, const float* __restrict__ thr_init, int n_splits,
    int qblocks, int flags) {
  using C = Cfg16<NKT>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int fr = lane & 15;
  const int fq = lane >> 4;  // lane quarter
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int split, qb;
  if (flags & kFlagXcdRemap) {  // the query blocks of a split on one XCD: its corpus comes from HBM once
    const int x = blockIdx.x & 7;
    const int i = blockIdx.x >> 3;
    split = (i / qblocks) * 8 + x;
    qb = i % qblocks;
  } else {
    split = blockIdx.x % n_splits;
    qb = blockIdx.x / n_splits;
  }
  const int n_blocks = (n_rows + kTR - 1) / kTR;
  const int b_begin = (int)((int64_t)split * n_blocks / n_splits);
  const int b_end = (int)((int64_t)(split + 1) * n_blocks / n_splits);
  const int n_st = 2 * (b_end - b_begin);
  const int qw0 = qb * kTQ + wave * 32;
  const bool live = qw0 < n_q;  // wave-uniform: a wave past the batch only stages and syncs
  float thr[2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int q = qw0 + 16 * g + fr;
    thr[g] = q < n_q ? (thr_init ? thr_init[q] : -INFINITY) : INFINITY;
  }

  // DMA (the 32x32 kernel's stages): piece p = wave + 8 i is k-tile p / 4 = wave / 4 + 2 i, rows
  // 8 (wave % 4) .. +8: the pieces of a wave differ by 2 k-tiles (256 B: the immediate offset)
  static_assert(C::kPPW * 2 * kRowBytes < 4096, "piece offsets fit the immediate");
  const int d_row = 8 * (wave & 3) + (lane >> 3);
  const uint32_t src_off = (uint32_t)(d_row * row_stride) + (wave >> 2) * kRowBytes +
                           ((((lane & 7) ^ ((d_row >> 1) & 7))) << 4);
  const int dst_off = (wave >> 2) * kKt + (wave & 3) * 1024;
  const uint32_t blk_bytes = (uint32_t)(kTR * row_stride);
  auto slot_of = [&](int st) __attribute__((always_inline)) { return smem + (st % kSlots16) * C::kStage; };
  auto issue = [&](int st) __attribute__((always_inline)) {
    const int b = b_begin + (st >> 1);
    const __amdgpu_buffer_rsrc_t r =
        tile_rsrc(corpus + (int64_t)b * kTR * row_stride + (st & 1) * C::kSK * kRowBytes, blk_bytes);
    unsigned char* slot = slot_of(st) + dst_off;
    static_for<C::kPPW>([&](auto I) { blds16_imm<decltype(I)::value * 2 * kRowBytes>(r, src_off, slot + decltype(I)::value * 2 * kKt); });
  };
  if (n_st > 0) issue(0);
  if (n_st > 1) issue(1);

  // resident B fragments: k32 step S of query group g
  u32x4 qf[C::kNS][2];
  {
    const uint8_t* src = qfrag + (int64_t)(qb * 16 + wave * 2) * C::kNS * 1024 + lane * 16;
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int S = 0; S < C::kNS; ++S) qf[S][g] = *reinterpret_cast<const u32x4*>(src + (g * C::kNS + S) * 1024);
  }
  // consumed here, behind the prologue DMA (see topk_qres_kernel)
#pragma unroll
  for (int S = 0; S < C::kNS; ++S) {
    asm volatile("" : "+v"(qf[S][0]));
    asm volatile("" : "+v"(qf[S][1]));
  }
  asm volatile("" : "+v"(thr[0]), "+v"(thr[1]));
  // Admission is by score alone (score >= thr): a score equal to the threshold whose row would lose
  // the tie is buffered too and dropped by the next compaction or the final sort (no key threshold
  // in registers: the VGPR budget is spent on the resident queries).

  // lane buffers: entry c of query g at lb[(g * kLaneCap + c) * kThreads] (64 lanes, 64 consecutive u64)
  uint64_t* lb = reinterpret_cast<uint64_t*>(smem + C::kOffBuf) + tid;
  int nb[2] = {0, 0};
  // keep the k_out best keys of buffer g; the smallest kept is the lane's k-th best: new threshold
  auto compact = [&](int g) {
    uint64_t* b = lb + g * kLaneCap * kThreads;
    int n = nb[g];
#pragma unroll 1
    while (n > k_out) {
      int mi = 0;
      uint64_t mv = b[0];
#pragma unroll 1
      for (int c = 1; c < n; ++c) {
        const uint64_t v = b[c * kThreads];
        if (v < mv) {
          mv = v;
          mi = c;
        }
      }
      b[mi * kThreads] = b[(n - 1) * kThreads];
      --n;
    }
    uint64_t mn = b[0];
#pragma unroll 1
    for (int c = 1; c < n; ++c) {
      const uint64_t v = b[c * kThreads];
      mn = v < mn ? v : mn;
    }
    nb[g] = n;
    if (n >= k_out) thr[g] = fmaxf(thr[g], key_score(mn));
  };
  // a finished block: per query group g the lane's 8 scores acc[rh][g][r], rows r0 + 16 rh + 4 fq + r
  auto screen = [&](const f32x4 (&acc)[2][2], int r0) __attribute__((always_inline)) {
    bool pass[2];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const float m = fmaxf(fmaxf(fmaxf(acc[0][g][0], acc[0][g][1]), fmaxf(acc[0][g][2], acc[0][g][3])),
                            fmaxf(fmaxf(acc[1][g][0], acc[1][g][1]), fmaxf(acc[1][g][2], acc[1][g][3])));
      pass[g] = m >= thr[g];
    }
    if (!__builtin_amdgcn_ballot_w64(pass[0] || pass[1])) return;  // wave-uniform: the common case
    const bool ragged = r0 + kTR > n_rows;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      if (pass[g]) {
#pragma unroll
        for (int rh = 0; rh < 2; ++rh)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = acc[rh][g][r];
            const uint32_t row = (uint32_t)(r0 + 16 * rh + 4 * fq + r);
            if (v >= thr[g] && (!ragged || row < (uint32_t)n_rows)) {
              lb[(g * kLaneCap + nb[g]) * kThreads] = make_key(v, row_base + row);
              if (++nb[g] == kLaneCap) compact(g);
            }
          }
      }
    }
  };

  // Sync at the start of stage st: this wave's pieces of stage st landed (st + 1 may stay in
  // flight), barrier: everyone's landed, everyone is done with stage st - 1, whose slot takes st + 2.
  auto stage_sync = [&](int st) __attribute__((always_inline)) {
    if (!(ABL & ABL_NOWAIT)) {
      if (st + 1 < n_st)
        wait_vm<C::kPPW>();
      else
        wait_vm<0>();
    }
    if (!(ABL & ABL_NOBARRIER)) lds_barrier();
    if (st + 2 < n_st && !((ABL & ABL_NOLOADS) && st >= 1)) issue(st + 2);
  };
  // A fragment (row half rh, k32 step s of a stage): k-tile s / 2, chunk 4 (s % 2) + fq of row
  // 16 rh + fr; the swizzle (row >> 1) & 7 is the same for both row halves (16 rows apart), so rh
  // is an immediate 2 KiB
  int a_off[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) a_off[h] = fr * kRowBytes + (((4 * h + fq) ^ ((fr >> 1) & 7)) << 4);
  auto frag = [&](const unsigned char* slot, int s, int rh) __attribute__((always_inline)) {
    if constexpr ((ABL & ABL_NOREAD) != 0) return qf[(s + 5) % C::kNS][rh];
    return *reinterpret_cast<const u32x4*>(slot + (s >> 1) * kKt + rh * 16 * kRowBytes + a_off[s & 1]);
  };
  u32x4 fa[2][2];  // [buffer][rh]: step t + 1 in flight while step t multiplies
  f32x4 acc[2][2];
  // one stage: 12 k32 steps, step t prefetches step t + 1 of the same stage; `pre` (the previous
  // block's screening: acc is overwritten only by the first MFMA) runs first
  auto stage = [&](auto H, int st, auto&& pre) __attribute__((always_inline)) {
    constexpr int h = decltype(H)::value;
    const unsigned char* slot = slot_of(st);
    pre();
#pragma unroll
    for (int rh = 0; rh < 2; ++rh) fa[0][rh] = frag(slot, 0, rh);
#pragma unroll
    for (int t = 0; t < C::kSS; ++t) {
      if (t + 1 < C::kSS) {
#pragma unroll
        for (int rh = 0; rh < 2; ++rh) fa[(t + 1) & 1][rh] = frag(slot, t + 1, rh);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int rh = 0; rh < 2; ++rh)
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          if (h == 0 && t == 0) {
            f32x4 z = {};
            mfma16<DT>(fa[0][rh], qf[0][g], z);
            acc[rh][g] = z;
          } else {
            mfma16<DT>(fa[t & 1][rh], qf[h * C::kSS + t][g], acc[rh][g]);
          }
        }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // a finished block's top-k screening, run after the NEXT block's first barrier, so no wave waits
  // at a barrier for another wave's survivors (the partner wave's MFMAs fill the SIMD meanwhile)
  auto finish = [&](int b) __attribute__((always_inline)) {
    if constexpr ((ABL & ABL_NOSCREEN) != 0) {  // GEMM only: every chain kept live (rule 17), no top-k
#pragma unroll
      for (int rh = 0; rh < 2; ++rh)
#pragma unroll
        for (int g = 0; g < 2; ++g) asm volatile("" ::"v"(acc[rh][g]));
    } else {
      screen(acc, b * kTR);
    }
  };
  auto nothing = []() {};
#pragma unroll 1
  for (int b = b_begin; b < b_end; ++b) {
    const int st0 = 2 * (b - b_begin);
    stage_sync(st0);
    if (live) {
      if (b > b_begin)
        stage(std::integral_constant<int, 0>{}, st0, [&]() { finish(b - 1); });
      else
        stage(std::integral_constant<int, 0>{}, st0, nothing);
    }
    stage_sync(st0 + 1);
    if (live) stage(std::integral_constant<int, 1>{}, st0 + 1, nothing);
  }
  if (live && b_end > b_begin) finish(b_end - 1);

  // each lane sorts its two buffers (the query registers are dead by now); per query the 4 lane
  // quarters' lists meet in the idle ring, quarter 0 merges them and writes the (query, split) list
  uint64_t* xch = reinterpret_cast<uint64_t*>(smem);  // [quarter 1..3][query-local 256][KCAP]
#pragma unroll 1
  for (int g = 0; g < 2; ++g) {
    uint64_t L[KCAP];
#pragma unroll
    for (int j = 0; j < KCAP; ++j) L[j] = 0;
#pragma unroll 1
    for (int c = 0; c < nb[g]; ++c) list_insert<KCAP>(L, lb[(g * kLaneCap + c) * kThreads]);
    const int qlx = wave * 32 + 16 * g + fr;
    __syncthreads();  // the ring (and, for g = 1, the previous exchange) is free
    if (fq) {
#pragma unroll
      for (int j = 0; j < KCAP; ++j) xch[((fq - 1) * kTQ + qlx) * KCAP + j] = L[j];
    }
    __syncthreads();
    const int q = qb * kTQ + qlx;
    if (!fq && q < n_q) {
#pragma unroll 1
      for (int u = 0; u < 3; ++u) {
#pragma unroll 1
        for (int j = 0; j < k_out; ++j) {
          const uint64_t v = xch[(u * kTQ + qlx) * KCAP + j];
          if (v <= L[KCAP - 1]) break;  // sorted: nothing further can enter
          list_insert<KCAP>(L, v);
        }
      }
      uint64_t* dst = part_keys + ((int64_t)q * n_splits + split) * k_out;
#pragma unroll
      for (int j = 0; j < KCAP; ++j)
        if (j < k_out) dst[j] = L[j];
    }
  }
}

bool supported(int dtype, int d_pad_bytes, int k) {
  return (dtype == AHR_BF16 || dtype == AHR_F16) && d_pad_bytes == 12 * kRowBytes && k >= 1 && k <= 12 &&
         k < kBufCap;
}

// the 16x16x32 form on request (k <= 10: its lane buffers); the 32x32x16 form by default
inline bool use16(int k, int flags) { return k < kLaneCap && (flags & kFlagQres16); }

void launch_frag(const uint8_t* qbuf, int64_t row_stride, int B, int d_pad_bytes, int k, uint8_t* qfrag, int flags,
                 hipStream_t s) {
  if (!use16(k, flags)) {  // the 32x32x16 kernel's layout: 32-query groups, k16 steps
    const int ns = d_pad_bytes / 32;
    const int64_t n16 = (int64_t)((B + 31) / 32) * ns * 64;
    hipLaunchKernelGGL(frag_kernel, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, s, qbuf, row_stride, n16, ns,
                       qfrag);
    return;
  }
  const int ns = d_pad_bytes / 64;  // 16-query groups, k32 steps
  const int64_t n16 = (int64_t)((B + 15) / 16) * ns * 64;
  hipLaunchKernelGGL(frag16_kernel, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, s, qbuf, row_stride, n16, ns,
                     qfrag);
}

template <int DT, int KCAP, int ABL = 0>
void launch16(const uint8_t* rows, const uint8_t* qfrag, int64_t row_stride, int n_rows, int B, uint32_t row_base,
              int k, uint64_t* part_keys, const float* thr, int n_splits, int qblocks, int flags, hipStream_t s) {
  if constexpr (kAblation && ABL == 0 && DT == DT_BF16) {  // the profiling build: cost-split variants
    const int abl = ((flags & kFlagSkipEpilogue) ? ABL_NOSCREEN : 0) | ((flags & kFlagNoLoads) ? ABL_NOLOADS : 0) |
                    ((flags & kFlagNoWait) ? ABL_NOWAIT : 0) | ((flags & kFlagNoBarrier) ? ABL_NOBARRIER : 0) |
                    ((flags & kFlagNoLdsRead) ? ABL_NOREAD : 0);
#define AHR_QRES_ABL(V) \
  case V: launch16<DT, KCAP, V>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags, s); return;
    switch (abl) {
      AHR_QRES_ABL(1) AHR_QRES_ABL(3) AHR_QRES_ABL(5) AHR_QRES_ABL(13) AHR_QRES_ABL(17) AHR_QRES_ABL(31)
      default: break;
    }
#undef AHR_QRES_ABL
  }
  constexpr auto kern = &topk_qres16_kernel<DT, 12, KCAP, ABL>;
  static_assert(3 * kTQ * KCAP * 8 <= kSlots16 * Cfg16<12>::kStage, "end exchange must fit the ring");
  static std::atomic<uint64_t> lds_attr{0};  // > 64 KiB dynamic LDS: opt in per device
  ensure_lds_attr(lds_attr, reinterpret_cast<const void*>(kern), Cfg16<12>::kLds);
  hipLaunchKernelGGL(kern, dim3((unsigned)(n_splits * qblocks)), dim3(kThreads), Cfg16<12>::kLds, s, rows, qfrag,
                     row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags);
}

template <int DT, int KCAP, bool STAGGER, int SCR, int ABL = 0>
void launch_t(const uint8_t* rows, const uint8_t* qfrag, int64_t row_stride, int n_rows, int B, uint32_t row_base,
              int k, uint64_t* part_keys, const float* thr, int n_splits, int qblocks, int flags, hipStream_t s) {
  if constexpr (kAblation && ABL == 0 && DT == DT_BF16) {  // the profiling build: cost-split variants
    const int abl = ((flags & kFlagSkipEpilogue) ? ABL_NOSCREEN : 0) | ((flags & kFlagNoLoads) ? ABL_NOLOADS : 0) |
                    ((flags & kFlagNoWait) ? ABL_NOWAIT : 0) | ((flags & kFlagNoBarrier) ? ABL_NOBARRIER : 0) |
                    ((flags & kFlagNoLdsRead) ? ABL_NOREAD : 0);
#define AHR_QRES_ABL(V) \
  case V: launch_t<DT, KCAP, STAGGER, SCR, V>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags, s); return;
    switch (abl) {
      AHR_QRES_ABL(1) AHR_QRES_ABL(3) AHR_QRES_ABL(5) AHR_QRES_ABL(13) AHR_QRES_ABL(17) AHR_QRES_ABL(31)
      default: break;
    }
#undef AHR_QRES_ABL
  }
  constexpr auto kern = &topk_qres_kernel<DT, 12, KCAP, STAGGER, SCR, ABL>;
  static std::atomic<uint64_t> lds_attr{0};  // > 64 KiB dynamic LDS: opt in per device
  ensure_lds_attr(lds_attr, reinterpret_cast<const void*>(kern), Cfg<12>::kLds);
  hipLaunchKernelGGL(kern, dim3((unsigned)(n_splits * qblocks)), dim3(kThreads), Cfg<12>::kLds, s, rows, qfrag,
                     row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags);
}

template <int DT, int KCAP>
void launch_s(const uint8_t* rows, const uint8_t* qfrag, int64_t row_stride, int n_rows, int B, uint32_t row_base,
              int k, uint64_t* part_keys, const float* thr, int n_splits, int qblocks, int flags, hipStream_t s) {
  if (use16(k, flags))
    launch16<DT, KCAP>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags, s);
  else if (flags & kFlagQresStagger)
    launch_t<DT, KCAP, true, 1>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags, s);
  else if (flags & kFlagQresScreenLoop)
    launch_t<DT, KCAP, false, 0>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags, s);
  else
    launch_t<DT, KCAP, false, 1>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags, s);
}

void launch(int dtype, int k, const uint8_t* rows, const uint8_t* qfrag, int64_t row_stride, int n_rows, int B,
            uint32_t row_base, uint64_t* part_keys, const float* thr, int n_splits, int qblocks, int flags,
            hipStream_t s) {
  if (dtype == AHR_BF16) {
    if (k <= 8)
      launch_s<DT_BF16, 8>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags, s);
    else
      launch_s<DT_BF16, 12>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags, s);
  } else {
    if (k <= 8)
      launch_s<DT_F16, 8>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags, s);
    else
      launch_s<DT_F16, 12>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags, s);
  }
}

}  // namespace qres
}  // namespace dense
}  // namespace ahr
