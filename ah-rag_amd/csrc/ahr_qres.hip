// ahr_qres.hip — query-resident fused Q·Nᵀ + exact top-k for gfx950 (MI355X): the B ≥ 512 bf16/f16
// path behind HierarchicalGraph.search_batch / the C2 headline (reference
// src/ah_rag/graph/hierarchical_graph.py:714, Chroma `collection.query`).
//
// Why this shape. The 128 x 128 two-operand tile kernels stream 1 byte into LDS per 64 flops;
// at C2 that is ~8.6 MB per CU per launch, which the per-CU L2 -> LDS delivery (~69 GB/s
// measured) cannot feed faster than ~124 us (the GEMM-only time of topk_tilelane_kernel). Here
// a workgroup keeps 256 queries resident in VGPRs for the whole launch — wave w holds the B
// fragments of queries 32w .. 32w + 31 over the WHOLE dimension (NKT * 4 x 16 B per lane: 192
// VGPRs at d = 768, 96 at d = 384) — and only the corpus streams: 1 byte per 256 flops, 4x fewer
// than the tile kernels. Every wave multiplies every 32-row corpus block (the A operand, read
// from LDS) against its own queries with one v_mfma_f32_32x32x16 chain per block, so a corpus
// byte brought in is used by 8 waves.
//
// * Corpus: 32-row blocks. At d_pad = 768 one 48-KiB stage per block in a 2-slot ring issued a
//   whole block ahead (two 24-KiB stages per block in a 3-slot ring measured 9 us slower at C2); at
//   384 (round 5) two blocks per 48-KiB stage in a 2-slot ring, one barrier per two blocks (one
//   24-KiB stage per block in a 3-slot ring: 113-114 vs 108 us at d = 384, same box). Buffer
//   LDS-DMA of 1-KiB pieces (8 whole 128-B rows), the XOR chunk swizzle of the tile kernels
//   (conflict-free ds_read_b128). One barrier per stage.
// * Scores: the k-order, fragment map and accumulation chain of topk_tilelane_kernel (step s of
//   a row covers k = [16 s, 16 s + 16), lane half fh holding 8 of them; the chain starts from 0),
//   so every score is bitwise the tile kernel's.
// * Top-k: a lane holds one query column x 16 rows of each block. Its 16 scores are screened
//   against the lane's threshold: the block max in the common case, and for the rare passing
//   scores one 8-B append to the lane's 14-entry LDS buffer. A full buffer is compacted in place
//   to its k best, which raises the threshold. At the end each lane sorts its buffer into a
//   register list (the query registers are dead by then) and the two lanes of a query merge:
//   one list per (query, split).
// * Admission threshold, self-seeded (no pre-pass launch): the 64 splits of a query block share
//   a rising lower bound of each query's k-th best score through memory. A split publishes, per
//   query, the max score of the rows it has scored so far (one 8-B {epoch, ord(score)} granule,
//   write-through); the split that owns query j (j mod n_splits) takes the k-th largest of the
//   published maxima — k distinct rows score at least that much, so it is a valid lower bound of
//   the k-th best — and publishes it as the query's seed, which every split reads. First round:
//   maxima of each split's first block (a 2,048-row sample at C2), the block's raw scores parked
//   in the lane buffer meanwhile and screened against the seed once it is there (a short bounded
//   wait at the end of block 1); later rounds (maxima over 3, 7, 15, ... blocks) tighten it and
//   never wait: their reads land in a per-wave LDS zone by buffer LDS-DMA and are consumed by the
//   next round. Granules carry the launch's epoch, so a stale or absent one only weakens the seed,
//   never invalidates it; every wait is bounded, so nothing assumes co-residency.
// * Query fragments come from a fragment-major copy of the converted queries (launch_frag):
//   one coalesced 1-KiB load per wave per k16 step.
// * Budget: NKT*16 query VGPRs + 16 accumulators + fragments in flight <= 256 (two waves per SIMD,
//   one workgroup of 8 waves per CU); LDS at d_pad 768: 96 KiB ring + 56 KiB lane buffers + 6 KiB
//   landing zones + 2 KiB event table = 160 KiB.
#include "ahr_qres_common.h"

namespace ahr {
namespace dense {
namespace qres {

// NKT 64-deep k-tiles per row (12 at d_pad 768, 6 at 384); a ring stage is kPB whole 32-row blocks
// (48 KiB: one block at 768, two at 384; AHR_QRES_PB6=1 builds the round-4 one-block 24-KiB stages,
// a 3-slot ring issued two blocks ahead), 48-KiB stages a 2-slot ring issued one stage ahead.
constexpr int kLandBytes = 768;

// Issue priority (A/B build switch): 0 none; 1 static s_setprio 1 for waves 4-7 (the younger half,
// the VALU-arbitration loser) before the main loop; 2 s_setprio 1 around every block's MFMA chain.
#ifndef AHR_QRES_PRIO
#define AHR_QRES_PRIO 0
#endif

static_assert(kPark >= 6, "the replay of a parked block never overtakes its unread quads");

#ifndef AHR_QRES_PB6
#define AHR_QRES_PB6 2  // 32-row blocks per ring stage at d_pad 384 (A/B builds: 1)
#endif
template <int NKT>
struct Cfg {
  static_assert(NKT == 6 || NKT == 12, "d_pad 384 or 768");
  static constexpr int kPB = NKT == 6 ? AHR_QRES_PB6 : 1;  // 32-row blocks per stage
  static constexpr int kSK = NKT;                 // k-tiles per block row
  static constexpr int kStage = kPB * kSK * kKt;  // 48 KiB (d 768; d 384 with two blocks) or 24 KiB
  static constexpr int kSlots = kPB * kSK == 12 ? 2 : 3;
  static constexpr int kAhead = kSlots - 1;       // stages in flight beyond the one multiplied
  static constexpr int kPieces = kPB * kSK * 4;   // 1-KiB DMA pieces per stage (8 rows x 128 B)
  static_assert(kPieces % kWaves == 0, "equal DMA share per wave");
  static constexpr int kPPW = kPieces / kWaves;   // pieces per wave per stage
  static constexpr int kNS = NKT * 4;             // k16 steps = query fragments per lane
  static constexpr bool kMma16 = mma16_for(kNS);  // the block product's MFMA shape (ahr_qres.h)
  static constexpr int kSS = kSK * 4;             // k16 steps per block
  // LDS: the ring, the lane buffers, the landing zones, the event table
  static constexpr int kOffBuf = kSlots * kStage;
  // the seeding events' landing zone, per wave: 64 published maxima (512 B), 32 seeds (256 B)
  static constexpr int kOffLand = kOffBuf + kBufCap * kThreads * 8;
  // the seeding events' per-lane table (see event_site): 4 B per lane
  static constexpr int kOffTab = kOffLand + kWaves * kLandBytes;
  static constexpr int kLds = kOffTab + kThreads * 4;
};
static_assert(Cfg<12>::kLds <= 160 * 1024 && Cfg<6>::kLds <= 160 * 1024,
              "LDS budget: one workgroup per CU");

// Self-seeding schedule (uniform, over a split's block index; the host passes it, publications in
// the low 32 bits, events in the high): after block bi < 32 with its publication bit set, a split
// publishes its running per-query maxima; at the end of block bi with its event bit set, a seeding
// event: the selecting splits take the k-th largest published maxima (landed since the previous
// event) as seeds, every split applies the seeds that landed, and both reads are issued again. The
// first event (block 1, after the block-0 publication) waits, bounded, for every granule and seed.
// From block 32 on (large corpora) the schedule continues every 8 blocks to block 127, then every
// 128: a publication after block 8m - 2 (128m - 2) and an event at the end of block 8m - 1.
constexpr uint32_t kSeedWaitTicks = 1000;  // s_memrealtime ticks (100 MHz): a 10-us bound per wait
#ifndef AHR_QRES_LATE
#define AHR_QRES_LATE 128  // the event period from block 128 on (A/B build switch, a power of two)
#endif
__device__ __forceinline__ bool in_sched(uint32_t mask, int bi, int off) {
  return bi < 32 ? ((mask >> bi) & 1) != 0 : (bi + off) % (bi < 128 ? 8 : AHR_QRES_LATE) == 0;
}

// k-th largest of the wave's nonzero values (lane l holds v0, v1); 0 if fewer than k are nonzero.
// k rounds of a wave max, each removing one instance (the lowest lane holding it).
__device__ __forceinline__ uint32_t wave_kth(uint32_t v0, uint32_t v1, int k, int lane) {
  uint32_t m = 0;
#pragma unroll 1
  for (int r = 0; r < k; ++r) {
    const uint32_t lm = max(v0, v1);
    m = dpp_max_u32(lm);
    if (m == 0) return 0;
    const int first = __builtin_ctzll(__ballot(lm == m));
    if (lane == first) {
      if (v0 == m)
        v0 = 0;
      else
        v1 = 0;
    }
  }
  return m;
}

// An admissible k-th largest of the wave's nonzero values (lane l holds v0, v1): the largest t on a
// grid of 2^12 with at least k values >= t. Never above the exact k-th largest, so still a valid
// lower bound (ord space: at most 2^-11 of the score below it); 0 if fewer than k are nonzero. 20
// ballot rounds, scalar between them: ~4x fewer instructions than k rounds of wave_kth.
__device__ __forceinline__ uint32_t wave_kth_grid(uint32_t v0, uint32_t v1, int k) {
  uint32_t t = 0;
#pragma unroll
  for (int b = 31; b >= 12; --b) {
    const uint32_t c = t | (1u << b);
    const int n = __popcll(__ballot(v0 >= c)) + __popcll(__ballot(v1 >= c));
    t = n >= k ? c : t;
  }
  return t;
}

// the per-lane sorted list of the end phase (k <= 12; a 16-wide bitonic network in registers
// measured 2.4 us slower at C2 than these insertions, which stop early on the partner's list)
constexpr int kListCap = 12;

__device__ __forceinline__ uint64_t granule_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1: not from L1
}
__device__ __forceinline__ void granule_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1: write-through
}
__global__ __launch_bounds__(256) void frag_kernel(const uint8_t* __restrict__ qbuf, int64_t row_stride, int64_t n16,
                                                   int ns, uint8_t* __restrict__ qfrag, uint32_t* __restrict__ epoch) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // one 16-B chunk of the output
  if (i == 0 && epoch) advance_epoch_rebalance(epoch);
  if (i >= n16) return;
  int64_t q;
  int j0;
  frag_elem(i, ns, &q, &j0);  // (2-byte elements)
  const u32x4 v = *reinterpret_cast<const u32x4*>(qbuf + q * row_stride + 2 * j0);
  *reinterpret_cast<u32x4*>(qfrag + i * 16) = v;
}


// pub: the self-seeding buffer (nullptr: no self-seeding; thr_init, if any, is the admission
// threshold): pub[-1] holds this launch's tag (low 32 bits), advanced on the device by the query
// conversion launched before it, so a replayed hipGraph gets a fresh one; then [256 qblocks]
// [n_splits] published maxima, then [256 qblocks] seeds.
template <int DT, int NKT, int ABL>
__global__ __launch_bounds__(kThreads, 2) void topk_qres_kernel(
    const uint8_t* __restrict__ corpus, const uint8_t* __restrict__ qfrag, int64_t row_stride, int n_rows, int n_q,
    uint32_t row_base, int k_out, uint64_t* __restrict__ part_keys, const float* __restrict__ thr_init, int n_splits,
    int qblocks, int flags, uint64_t* __restrict__ pub, uint64_t sched) {
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
  const int qw0 = qb * kTQ + wave * 32;
  const bool live = qw0 < n_q;  // wave-uniform: a wave past the batch only stages and syncs
  const int q = qw0 + fr;
  const bool ss = pub != nullptr && (ABL & ABL_NOSCREEN) == 0 && self_seeds(n_rows, n_splits, k_out);
  // XCD-balanced splits (kFlagXcdBalance, self-seeding launches with the XCD remap: split s runs on
  // XCD s mod 8): the splits of XCD x get rows in proportion to its weight (rebalance_xcds, set from
  // the previous launch's durations before this one); the bounds stay a partition of the blocks,
  // >= 2 blocks per split (weights within 0.64x-1.56x of each other, >= 4 blocks per split on average)
  uint32_t* const xcdw = ss ? reinterpret_cast<uint32_t*>(pub - 9) : nullptr;
  const bool bal = ss && (flags & kFlagXcdRemap) && (flags & kFlagXcdBalance) && n_splits % 8 == 0 &&
                   n_blocks >= 4 * n_splits;
  // (64-bit divisions run on the VALU: readfirstlane keeps the loop bounds, the stage index and the
  // control flow built on them scalar)
  int b_begin, b_end;
  if (bal) {
    int64_t W = 0, pre = 0, own = 0;
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      const int64_t w = xcdw[x] ? xcdw[x] : kXcdW;
      W += w;
      pre += x < (split & 7) ? w : 0;
      own = x == (split & 7) ? w : own;
    }
    const int64_t c0 = (int64_t)(split >> 3) * W + pre, tot = (int64_t)(n_splits >> 3) * W;
    b_begin = __builtin_amdgcn_readfirstlane((int)(c0 * n_blocks / tot));
    b_end = __builtin_amdgcn_readfirstlane((int)((c0 + own) * n_blocks / tot));
  } else {
    b_begin = __builtin_amdgcn_readfirstlane((int)((int64_t)split * n_blocks / n_splits));
    b_end = __builtin_amdgcn_readfirstlane((int)((int64_t)(split + 1) * n_blocks / n_splits));
  }
  const int n_bl = b_end - b_begin;                  // the split's blocks
  const int n_st = (n_bl + C::kPB - 1) / C::kPB;     // ring stages
  // ABL_TRACE (the profiling build only): thread 0 of each workgroup stamps into the buffer passed
  // as thr_init, 64 u64 per workgroup: [0] s_memrealtime at entry, [1] s_memtime at entry, [2] loop
  // entry, [3 + j] after stage j's sync (j <= 55), [59] first event entered, [60] selection done,
  // [61] seed read, [62] s_memrealtime at exit, [63] s_memtime at exit.
  constexpr bool kTrace = (ABL & ABL_TRACE) != 0;
  auto stamp = [&](int i, bool core_clock = false) __attribute__((always_inline)) {
    if constexpr (kTrace) {
      if (tid == 0)
        reinterpret_cast<uint64_t*>(const_cast<float*>(thr_init))[(int64_t)blockIdx.x * 64 + i] =
            core_clock ? __builtin_amdgcn_s_memtime() : __builtin_amdgcn_s_memrealtime();
    }
  };
  stamp(0);
  stamp(1, true);

  float thr = q < n_q ? (thr_init && !kTrace ? thr_init[q] : -INFINITY) : INFINITY;
  // (kFlagQresMute, a test switch: split 0 tags its granules and compares what it reads with a tag no
  // launch has, so its maxima and seeds never count for the others and theirs never for it — every
  // bounded wait on it runs to its time limit, and the results must not change)
  const uint32_t epoch = pub ? (uint32_t)pub[-1] ^ ((flags & kFlagQresMute) && split == 0 ? 0x40000000u : 0u) : 0u;
  // (the seed array's address is recomputed at each use from laundered operands: a live 64-bit
  // pointer costs two SGPRs the loop does not have)
  auto seeds_at = [&](int64_t qq) __attribute__((always_inline)) {
    int qbk = qblocks, ns = n_splits;
    asm volatile("" : "+s"(qbk), "+s"(ns));
    return pub + (int64_t)qbk * kTQ * ns + qq;
  };

  // DMA: piece p = wave + 8 i of a stage is k-tile p / 4, rows 8 (p % 4) .. +8; lane l lands at
  // (row 8 (p % 4) + l / 8, physical chunk l % 8) and loads logical chunk (l % 8) ^ swz(row)
  // (the per-lane source offsets are recomputed at each issue: a few VALU per stage, and three
  // registers the main loop cannot spare)
  const uint32_t blk_bytes = (uint32_t)(kTR * row_stride);
  auto slot_of = [&](int st) __attribute__((always_inline)) { return smem + (st % C::kSlots) * C::kStage; };
  // (kPB = 2: pieces 0 .. 4 kSK - 1 are the stage's first block, the rest its second, laid out after
  // it in the slot; a stage with one block left reads zeros for the second: out of the descriptor)
  auto issue = [&](int st) __attribute__((always_inline)) {
    const int b = b_begin + st * C::kPB;
    const int nbs = C::kPB == 1 ? 1 : min(C::kPB, b_end - b);
    const __amdgpu_buffer_rsrc_t r =
        tile_rsrc(corpus + (int64_t)b * kTR * row_stride, blk_bytes * (uint32_t)nbs);
    unsigned char* slot = slot_of(st);
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int i = 0; i < C::kPPW; ++i) {
      // piece wave + 8 i: block h = 8 i / (4 kSK) of the stage (wave < 8 and 4 kSK a multiple of 8:
      // a compile-time split of the unrolled pieces)
      constexpr int kPiecesPerBlock = C::kSK * 4;
      static_assert(kPiecesPerBlock % kWaves == 0, "a wave's pieces split evenly over the blocks");
      const int h = (kWaves * i) / kPiecesPerBlock;
      const int p = wave + kWaves * i - h * kPiecesPerBlock;
      const int row = 8 * (p & 3) + (ln >> 3);
      const uint32_t src_off = (uint32_t)((h * kTR + row) * row_stride) + (p >> 2) * kRowBytes +
                               ((((ln & 7) ^ ((row >> 1) & 7))) << 4);
      blds16(r, src_off, slot + (h * C::kSK + (p >> 2)) * kKt + (p & 3) * 1024);
    }
  };
#pragma unroll
  // the prologue fills every ring slot (stages 0 .. kAhead): the peeled first iteration then issues
  // nothing, and block 0's chain waits on no stage but its own
  for (int st = 0; st < C::kSlots; ++st)
    if (st < n_st) issue(st);

  // resident B fragments: step S of query q = bytes [32 S + 16 fh, +16) of its row
  u32x4 qf[C::kNS];
  {
    const uint8_t* src = qfrag + (int64_t)(qb * kWaves + wave) * C::kNS * 1024 + lane * 16;
#pragma unroll
    for (int S = 0; S < C::kNS; ++S) {
      qf[S] = *reinterpret_cast<const u32x4*>(src + S * 1024);
      __builtin_amdgcn_sched_barrier(0);  // in step order: block 0's step S waits for fragment S only
    }
  }
  // The fragments stream in behind the prologue DMA and are consumed by block 0's chain, each
  // waited for as its step needs it (the peeled first iteration below); after it an empty asm
  // "consumes" them all, so the main loop never waits on them (a use inside the loop would make the
  // waitcnt pass count the ring's in-flight pieces against them every stage).
  asm volatile("" : "+v"(thr));
  // (a score threshold only, no key: a score equal to it always passes, so exact ties may be
  // appended and cut again — correct, and the registers go to the resident fragments)

  // lane survivor buffer: entry c at lbuf[c * kThreads] (a wave's 64 lanes hit 64 consecutive u64)
  uint64_t* const lbuf0 = reinterpret_cast<uint64_t*>(smem + C::kOffBuf);
  auto lb = [&]() __attribute__((always_inline)) {  // recomputed at each use: not a live register
    int t = tid;
    asm volatile("" : "+v"(t));
    return lbuf0 + t;
  };
  int nb = 0;
  // keep the k_out best buffered keys at or above the threshold (seeds may have raised it since an
  // entry was appended: those entries go in one pass); the smallest of k_out kept ones is the lane's
  // k-th best: new threshold (fewer than k_out kept — k_out = 12 with 11 buffered, or after the
  // pass — bound nothing)
  auto compact = [&]() {
    uint64_t* const lbuf = lb();
    int nk = 0;
#pragma unroll 1
    for (int c = 0; c < nb; ++c) {
      const uint64_t v = lbuf[c * kThreads];
      if (key_score(v) >= thr) lbuf[nk++ * kThreads] = v;
    }
    nb = nk;
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
    if (nb < k_out) return;
    uint64_t mn = lbuf[0];
#pragma unroll 1
    for (int c = 1; c < nb; ++c) {
      const uint64_t v = lbuf[c * kThreads];
      mn = v < mn ? v : mn;
    }
    thr = fmaxf(thr, key_score(mn));
  };
  // the block row of score e of quad qd (acc[4 qd + e]): quad_row(qd) + e
  auto quad_row = [&](int qd) __attribute__((always_inline)) {
    return C::kMma16 ? 16 * (qd >> 1) + 8 * fh + 4 * (qd & 1) : 8 * qd + 4 * fh;
  };
  // the rows of score e of quad qd: r0 + quad_row(qd) + e. A passing quad's scores are tested one by
  // one, each passing score one append; a quad compacts first when its 4 possible appends might
  // not fit.
  auto screen_quad = [&](float v0, float v1, float v2, float v3, int qrow, bool ragged) __attribute__((always_inline)) {
    if (nb + 4 > kBufCap) compact();
    uint64_t* const lbuf = lb();
    const float vv[4] = {v0, v1, v2, v3};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t row = (uint32_t)(qrow + e);
      if (vv[e] >= thr && (!ragged || row < (uint32_t)n_rows)) {
        if (nb == kBufCap) compact();  // k_out + 4 > kBufCap (k = 12): one more cut mid-quad
        lbuf[nb * kThreads] = make_key(vv[e], row_base + row);
        ++nb;
      }
    }
  };
  // self-seeding: max score of this lane's rows so far, as its ordered bits with bit 0 set while it
  // has risen since the last publication (ord(-inf) is odd: the first publication always writes)
  uint32_t rmo = ord_f32(-INFINITY) | 1u;
  // a block's 16 scores of this lane: quad maxima, then the passing quads
  auto screen_quads = [&](const f32x16& acc, int r0) __attribute__((always_inline)) {
    float qm[4];
#pragma unroll
    for (int qd = 0; qd < 4; ++qd)
      qm[qd] = fmaxf(fmaxf(acc[4 * qd], acc[4 * qd + 1]), fmaxf(acc[4 * qd + 2], acc[4 * qd + 3]));
    const float m = fmaxf(fmaxf(qm[0], qm[1]), fmaxf(qm[2], qm[3]));
    const bool ragged = r0 + kTR > n_rows;  // wave-uniform: the last block only
    if (ss) {
      float bm = m;
      if (ragged) {
        bm = -INFINITY;
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (r0 + quad_row(j >> 2) + (j & 3) < n_rows) bm = fmaxf(bm, acc[j]);
      }
      rmo = max(rmo, ord_f32(bm) | 1u);  // a new maximum is marked risen
    }
    if (m < thr) return;
#pragma unroll
    for (int qd = 0; qd < 4; ++qd)
      if (qm[qd] >= thr) screen_quad(acc[4 * qd], acc[4 * qd + 1], acc[4 * qd + 2], acc[4 * qd + 3],
                                     r0 + quad_row(qd), ragged);
  };

  // ---- self-seeding (see the header) ----
  // (the seeding paths launder the lane's query index through an empty asm: otherwise LLVM hoists
  // their 64-bit granule addresses out of the main loop, and the extra registers spill the
  // resident fragments)
  // Vector-memory operations this wave issued after its ring pieces in the current iteration (the
  // publication store, the event's seed stores and landing loads), counted exactly: the next stage
  // sync waits for all but these (vmcnt counts in issue order), so a write-through store or a
  // cross-XCD read never holds up the ring. Each counted site issues exactly one instruction per
  // wave (some lane is always active there).
  int young = 0;
  // (the per-lane event table, built below: see event_site)
  uint32_t* const tab = reinterpret_cast<uint32_t*>(smem + C::kOffTab) + wave * 64;
  // A publication writes only the maxima that rose since the split's previous one (the others'
  // granules still hold this launch's current values): one buffer store per wave whatever the
  // lanes' state — a lane with nothing to write gets an out-of-range offset, which the buffer
  // unit drops — so the count of younger operations stays exact (round 5: WRITE per C2 launch
  // 29.7 MB -> see DESIGN §3.0). The published value is the maximum with bit 0 cleared, at most
  // one ulp below it: still a lower bound.
  auto publish = [&]() __attribute__((always_inline)) {
    const uint32_t pm = max(rmo, (uint32_t)__shfl_xor((int)rmo, 32, 64));  // the query's max over this split's rows
    int qq = q;
    asm volatile("" : "+v"(qq));
    const uint32_t off = !fh && qq < n_q && (pm & 1u) ? (uint32_t)(qq * n_splits + split) * 8u : 0xFFFFFFF0u;
    const u32x4 uni = *reinterpret_cast<const u32x4*>(tab + 48);  // (the buffer size: see the event table)
    const __amdgpu_buffer_rsrc_t r = tile_rsrc(pub, (uint32_t)__builtin_amdgcn_readfirstlane((int)uni[2]));
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{pm & ~1u, epoch}, r, (int)off, 0, 16);  // sc1: write-through
    rmo &= ~1u;
    ++young;
  };
  auto apply_seed = [&](uint64_t g) __attribute__((always_inline)) {  // a seed granule of this launch raises thr
    if (q < n_q && (uint32_t)(g >> 32) == epoch && (uint32_t)g != 0)
      thr = fmaxf(thr, key_score((uint64_t)(uint32_t)g << 32));
  };
  // Seeding events. Granule and seed reads go through the wave's LDS landing zone by buffer
  // LDS-DMA (sc1), so no register is held between two events: a later event consumes what the
  // previous one's loads landed (a landing not complete yet only leaves an earlier round's — still
  // valid — or zeroed granules) and issues the next, never waiting; the first polls (bounded) until
  // every split's block-0 granule, then every seed, of this launch is there. Granules: lane l < 32
  // of a selecting wave loads maxima 2p, 2p + 1 of its selected query i = l / np (p = l % np,
  // np = n_splits / 2; past 64 splits only the first 64: a subset, a weaker still valid bound);
  // seeds: lane l < 16 loads the seeds of the wave's queries 2l, 2l + 1. One code site serves
  // every event (two would not fit the register budget).
  unsigned char* const land = smem + C::kOffLand + wave * kLandBytes;
  if (tid % 64 < kLandBytes / 16) *reinterpret_cast<u32x4*>(land + lane * 16) = u32x4{0, 0, 0, 0};
  // The split selects for the queries j = split + m n_splits of its query block; the m-th goes to
  // wave {0, 3, 5, 6, 1, 2, 4, 7}[m % 8], so any four consecutive ones sit on four different SIMDs
  // whether a SIMD's two waves are w, w + 4 or 2s, 2s + 1 (measured: a selection still costs its
  // block ~0.5 us, not hidden by the other wave's MFMA chain).
  // Per-lane table, built once (the divisions stay out of the loop): lane l < 32 of a wave, its
  // granule read (bit 31: a selecting lane; bits 24..29: its query i, the wave's i-th; bits 0..23:
  // the byte offset in the self-seeding buffer); lanes 48..52 the wave's count of selected queries,
  // the first one's index in the query block, the buffer's byte size, the offset of the wave's
  // seeds and the index step between its selected queries.
  if (ss) {
    const int ns = n_splits;
    const int np = ns >= 128 ? 32 : ns / 2;  // lanes per selected query
    const int j0 = split + ((0x73261540 >> (4 * wave)) & 7) * ns;  // m = {0, 4, 5, 1, 6, 2, 3, 7}[wave]
    int cnt = 0;
    for (int j = j0; j < kTQ && (int64_t)qb * kTQ + j < n_q; j += kWaves * ns) ++cnt;
    uint32_t e = 0;
    if (lane < 32) {
      const int i = lane / np;
      const int64_t qq = (int64_t)qb * kTQ + j0 + i * kWaves * ns;
      e = i < cnt ? 0x80000000u | ((uint32_t)i << 24) | (uint32_t)((qq * ns + 2 * (lane - i * np)) * 8) : 0u;
    } else if (lane == 48) {
      e = (uint32_t)cnt;
    } else if (lane == 49) {
      e = (uint32_t)j0;
    } else if (lane == 52) {
      e = (uint32_t)(kWaves * ns);
    } else if (lane == 50) {
      e = (uint32_t)((int64_t)qblocks * kTQ * (ns + 1) * 8);
    } else if (lane == 51) {
      e = (uint32_t)(((int64_t)qblocks * kTQ * ns + (int64_t)qb * kTQ + wave * 32) * 8);
    }
    tab[lane] = e;
  }
  // this workgroup's start, for its XCD's duration sum (lane 60 of wave 0's table row is spare)
  if (bal && tid == 0) tab[60] = (uint32_t)__builtin_amdgcn_s_memrealtime();
  auto event_site = [&](bool first) __attribute__((always_inline)) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const uint32_t e = tab[ln];
    const u32x4 uni = *reinterpret_cast<const u32x4*>(tab + 48);
    const int jstep = __builtin_amdgcn_readfirstlane((int)tab[52]);
    const int cnt = __builtin_amdgcn_readfirstlane((int)uni[0]);
    const int j0 = __builtin_amdgcn_readfirstlane((int)uni[1]);
    const __amdgpu_buffer_rsrc_t r = tile_rsrc(pub, (uint32_t)__builtin_amdgcn_readfirstlane((int)uni[2]));
    const uint32_t seed_off = (uint32_t)__builtin_amdgcn_readfirstlane((int)uni[3]);
    const bool sel_lane = (e >> 31) != 0;
    const int my_i = (int)((e >> 24) & 63);
    auto issue_granules = [&]() __attribute__((always_inline)) {  // lanes past the selection read zeros (out of range)
      if (ln < 32) blds16_pol(r, sel_lane ? (e & 0xffffffu) : 0x7ffffff0u, land);
    };
    auto issue_seeds = [&]() __attribute__((always_inline)) {
      if (ln < 16) blds16_pol(r, seed_off + 16 * ln, land + 512);
    };
    auto landed = [&](bool seeds_part) __attribute__((always_inline)) {  // bounded poll (first event)
      const uint32_t t0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
#pragma unroll 1
      for (;;) {
        if (seeds_part)
          issue_seeds();
        else
          issue_granules();
        wait_vm<0>();
        asm volatile("" ::: "memory");
        bool ok;
        if (seeds_part) {
          ok = q >= n_q || *reinterpret_cast<const uint32_t*>(land + 512 + fr * 8 + 4) == epoch;
        } else {
          const u32x4 g = *reinterpret_cast<const u32x4*>(land + ln * 16);
          ok = !sel_lane || (g[1] == epoch && g[3] == epoch);
        }
        if (__ballot(!ok) == 0 || (uint32_t)__builtin_amdgcn_s_memrealtime() - t0 > kSeedWaitTicks) break;
        __builtin_amdgcn_s_sleep(2);
      }
    };
    if (first) {
      stamp(59);
      landed(false);
      young = 0;  // everything this wave issued so far has completed
    }
    if ((first || !(ABL & ABL_EV_NOSEL)) && cnt > 0) {  // the k-th largest of each selected query's published maxima
      const u32x4 g = *reinterpret_cast<const u32x4*>(land + ln * 16);
      const uint32_t v0 = sel_lane && g[1] == epoch ? g[0] : 0u;
      const uint32_t v1 = sel_lane && g[3] == epoch ? g[2] : 0u;
#pragma unroll 1
      for (int i = 0; i < cnt; ++i) {
        const int64_t qq = (int64_t)qb * kTQ + j0 + i * jstep;
        const uint32_t m = wave_kth_grid(my_i == i ? v0 : 0u, my_i == i ? v1 : 0u, k_out);
        // (no seed: the store goes to the spare slot past the seeds, keeping the count exact)
        if (ln == 0) granule_store(seeds_at(qq) + (m != 0 ? 0 : (int64_t)qblocks * kTQ), ((uint64_t)epoch << 32) | m);
        ++young;
      }
    }
    if (first) {
      stamp(60);
      landed(true);
      stamp(61);
      young = 0;
    }
    apply_seed(*reinterpret_cast<const uint64_t*>(land + 512 + fr * 8));
    if constexpr (!(ABL & ABL_EV_NOISSUE)) {
      issue_granules();  // for the next event (its seeds are read one block later: seed_read)
      ++young;
    }
  };
  // The seed read of an event, one block after it: by then every selector of the query block has
  // stored this round's seeds (read in the event itself, most would still be the previous round's).
  auto seed_read = [&]() __attribute__((always_inline)) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const u32x4 uni = *reinterpret_cast<const u32x4*>(tab + 48);
    const __amdgpu_buffer_rsrc_t r = tile_rsrc(pub, (uint32_t)__builtin_amdgcn_readfirstlane((int)uni[2]));
    const uint32_t seed_off = (uint32_t)__builtin_amdgcn_readfirstlane((int)uni[3]);
    if constexpr (!(ABL & ABL_EV_NOISSUE)) {
      if (ln < 16) blds16_pol(r, seed_off + 16 * ln, land + 512);
      ++young;
    }
  };
  // block 0's raw scores parked in the top of the lane buffer (entries kPark .. kPark + 7, two floats
  // each) until the first seed; replayed quad by quad from the bottom while the appends fill the
  // buffer from entry 0: after quad qd at most 4 (qd + 1) keys, below entry kPark + 2 (qd + 1)
  // (kPark >= 6) — the appends never reach a quad not yet read.
  auto park = [&](const f32x16& acc) __attribute__((always_inline)) {
    uint64_t* const lbuf = lb();
#pragma unroll
    for (int e = 0; e < 8; ++e)
      lbuf[(kPark + e) * kThreads] = ((uint64_t)__float_as_uint(acc[2 * e + 1]) << 32) | __float_as_uint(acc[2 * e]);
  };
  auto replay = [&](int r0) __attribute__((always_inline)) {
    asm volatile("" : "+s"(r0));  // (not loop-invariant to LLVM: it would hoist all 16 row keys and spill them)
    const bool ragged = r0 + kTR > n_rows;
    uint64_t* const lbuf = lb();
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) {
      const uint64_t a = lbuf[(kPark + 2 * qd) * kThreads], b = lbuf[(kPark + 1 + 2 * qd) * kThreads];
      const float v0 = __uint_as_float((uint32_t)a), v1 = __uint_as_float((uint32_t)(a >> 32));
      const float v2 = __uint_as_float((uint32_t)b), v3 = __uint_as_float((uint32_t)(b >> 32));
      if (fmaxf(fmaxf(v0, v1), fmaxf(v2, v3)) >= thr) screen_quad(v0, v1, v2, v3, r0 + quad_row(qd), ragged);
    }
  };

  // Sync j: this wave's pieces of stage j landed (with a 3-slot ring stage j + 1 may stay in
  // flight), then the barrier: everyone's stage j landed, and everyone is done with stage j - 1,
  // whose slot takes stage j + kAhead.
  auto stage_sync = [&](int j, int y) __attribute__((always_inline)) {
    if (!(ABL & ABL_NOWAIT)) wait_vm_dyn((C::kAhead == 2 && j + 1 < n_st ? C::kPPW : 0) + __builtin_amdgcn_readfirstlane(y));
    if (!(ABL & ABL_NOBARRIER)) lds_barrier();
  };
  // A fragment of k16 step s of stage st: k-tile s / 4, logical chunk 2 (s % 4) + fh of row fr,
  // stored at physical chunk (2 (s % 4) + fh) ^ ((fr >> 1) & 7) = 2 ((s % 4) ^ h) + (fh ^ a0),
  // h = (fr >> 2) & 3, a0 = (fr >> 1) & 1. The byte offset is one v_xad_u32 per read from two
  // per-lane values (the four precomputed offsets would cost two more live registers).
  // The four per-lane chunk offsets (s % 4 = m: a_row + 32 (m ^ h) + 16 (fh ^ a0)) are kept in
  // registers, so a read costs one v_add (the slot base) and an immediate k-tile offset.
  // 16x16x32 (kMma16): fragment m = 2 s2 + r of a k-tile is the 32-deep step s2's row subtile r:
  // row 16 r + l % 16, logical chunk 4 s2 + l / 16 (the same 16 B per lane and instruction).
  int a_off[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    if constexpr (C::kMma16) {
      const int row = 16 * (m & 1) + (lane & 15);
      a_off[m] = row * kRowBytes + (((4 * (m >> 1) + (lane >> 4)) ^ ((row >> 1) & 7)) << 4);
    } else {
      a_off[m] = fr * kRowBytes + ((((2 * m + fh) ^ ((fr >> 1) & 7))) << 4);
    }
    asm volatile("" : "+v"(a_off[m]));  // materialized once, here
  }
  auto frag = [&](int st, int s, int h = 0) __attribute__((always_inline)) {  // h: the stage's block
    if constexpr ((ABL & ABL_NOREAD) != 0) return qf[(s + 5) % C::kNS];  // MFMA + issue only
    const unsigned char* slot = slot_of(st);
    return *reinterpret_cast<const u32x4*>(slot + (h * C::kSK + (s >> 2)) * kKt + a_off[s & 3]);
  };
  static_assert(C::kSS % 3 == 0, "three fragment registers rotate evenly over a stage");
  constexpr bool skip_screen = (ABL & ABL_NOSCREEN) != 0;
  f32x16 acc;
  u32x4 fa[3];
  // a block's kSS fragments: fragment t prefetches fragment t + 2 and is multiplied.
  // 32x32x16: fragment t = k16 step t, one MFMA. 16x16x32: fragment t = (32-deep step t / 2, row
  // subtile r = t % 2), two MFMAs (query tiles 0 and 1: c[2 r] and c[2 r + 1]); after the chain one
  // v_permlane16_swap per register pair gives each lane the 32x32 form's share — one query (lane %
  // 32) and 16 rows — so the screening below is the same code (quad rows: quad_row).
  auto stage_mma = [&](int st, int h = 0) __attribute__((always_inline)) {
    if constexpr (AHR_QRES_PRIO == 2) __builtin_amdgcn_s_setprio(1);
    if constexpr (C::kMma16) {
      f32x4 c[4];
#pragma unroll
      for (int t = 0; t < C::kSS; ++t) {
        if (t + 2 < C::kSS) fa[(t + 2) % 3] = frag(st, t + 2, h);
        __builtin_amdgcn_sched_barrier(0);
        const int r = t & 1;
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          const f32x4 prev = t < 2 ? f32x4{} : c[2 * r + qt];
          c[2 * r + qt] = mfma16_step<DT>(fa[t % 3], qf[2 * (t >> 1) + qt], prev);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      // lane (R = l / 16, c = l % 16) held query c (c[2 r]) and 16 + c (c[2 r + 1]), rows 16 r + 4 R
      // + e; the swap moves query 16 + c to the odd rows R and query c to the even ones, so lane l
      // holds query l % 32: c[2 r] rows 16 r + 8 (l / 32) + e, c[2 r + 1] the 4 rows after them
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const auto w = __builtin_amdgcn_permlane16_swap(__float_as_uint(c[2 * r][e]),
                                                          __float_as_uint(c[2 * r + 1][e]), false, false);
          c[2 * r][e] = __uint_as_float(w[0]);
          c[2 * r + 1][e] = __uint_as_float(w[1]);
        }
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = c[i >> 2][i & 3];
    } else {
#pragma unroll
      for (int t = 0; t < C::kSS; ++t) {
        if (t + 2 < C::kSS) fa[(t + 2) % 3] = frag(st, t + 2, h);
        __builtin_amdgcn_sched_barrier(0);
        if (t == 0) {
          f32x16 z = {};
          mfma_step<DT>(fa[0], qf[0], z);
          acc = z;
        } else {
          mfma_step<DT>(fa[t % 3], qf[t], acc);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (AHR_QRES_PRIO == 2) __builtin_amdgcn_s_setprio(0);
  };
  auto finish_block = [&](int bi) __attribute__((always_inline)) {  // bi: the block just multiplied
    if constexpr (skip_screen) {  // GEMM only: the chain kept live (rule 17), no top-k
      asm volatile("" ::"v"(acc));
      return;
    }
    const int r0 = (b_begin + bi) * kTR;
    if (ss && bi == 0) {  // the first event's sample: park the scores, publish the maxima
      park(acc);
      float bm = -INFINITY;
#pragma unroll
      for (int j = 0; j < 16; ++j)  // block 0 is never ragged (>= 2 blocks per split) but check anyway
        if (r0 + quad_row(j >> 2) + (j & 3) < n_rows) bm = fmaxf(bm, acc[j]);
      rmo = max(rmo, ord_f32(bm) | 1u);
      publish();
      return;
    }
    screen_quads(acc, r0);
    if (ss && in_sched((uint32_t)sched, bi, 2)) publish();
  };
  if constexpr (AHR_QRES_PRIO == 1) {
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);  // wave: readfirstlane, so a scalar branch
  }
  stamp(2);
  {  // iteration 0, peeled: the sync waits only for stage 0's pieces (the fragments are younger)
    if (!(ABL & ABL_NOWAIT)) {  // younger than stage 0's pieces: the other prologue stages', the fragments
      if (n_st >= 3 && C::kSlots == 3)
        wait_vm<2 * C::kPPW + C::kNS>();
      else if (n_st >= 2)
        wait_vm<C::kPPW + C::kNS>();
      else
        wait_vm<C::kNS>();
    }
    if (!(ABL & ABL_NOBARRIER)) lds_barrier();
    stamp(3);
    if (live && n_st > 0) {
      fa[0] = frag(0, 0);
      fa[1] = frag(0, 1);
      stage_mma(0);
    }
#pragma unroll
    for (int S = 0; S < C::kNS; ++S) asm volatile("" : "+v"(qf[S]));
  }
  if constexpr (C::kPB == 1) {
  #pragma unroll 1
    for (int j = 1; j <= n_st; ++j) {
      stage_sync(j, young);
      young = 0;
      if (j <= 55) stamp(3 + j);
      const int bi = j - 1;  // the block that ended with stage j - 1
      const bool first = ss && j == 2;  // uniform
      // (at the first event the next stage is issued after it: its bounded polls then wait for their
      // own reads only, not for a stage in flight)
      const bool ring = j + C::kAhead < n_st && !((ABL & ABL_NOLOADS) && j >= 2);  // (j >= 1: the prologue issued up to kAhead)
      if (ring && !(first && live)) issue(j + C::kAhead);
      if (!live) continue;
      const bool mma = j < n_st;
      if (mma) {  // the stage's first fragments: in flight under the screening below
        fa[0] = frag(j, 0);
        fa[1] = frag(j, 1);
      }
      // block bi's screening, then a seeding event (the first one before block 1's screening, which
      // then runs with the first seed after block 0's parked scores)
      if (!first) finish_block(bi);
      if (ss && (first || in_sched((uint32_t)(sched >> 32), bi, 1))) event_site(first);
      if (ss && bi >= 3 && in_sched((uint32_t)(sched >> 32), bi - 1, 1)) seed_read();
      if (first) {
        if (ring) {
          issue(j + C::kAhead);
          young = 0;  // the ring's pieces are the youngest now: the next sync waits for everything
        }
        replay(b_begin * kTR);
        finish_block(bi);
      }
      if (mma) stage_mma(j);
    }
  } else {
    // One iteration per block bl: at a stage's first block the stage sync and the ring's next issue,
    // then block bl - 1's screening and seeding steps, then block bl's chain. (kPB = 2: the second
    // block of a stage runs without a sync: one barrier per two blocks.)
  #pragma unroll 1
    for (int bl = 1; bl <= n_bl; ++bl) {
      const int j = bl / C::kPB;                            // the stage holding block bl
      const bool at_stage = C::kPB == 1 || (bl & 1) == 0;   // uniform
      const int bi = bl - 1;                                // the block whose chain just ended
      const bool first = ss && bi == 1;                     // uniform
      bool ring = false;
      if (at_stage) {
        stage_sync(j, young);
        young = 0;
        if (j <= 55) stamp(3 + j);
        // (at the first event the next stage is issued after it: its bounded polls then wait for
        // their own reads only, not for a stage in flight)
        ring = j + C::kAhead < n_st && !((ABL & ABL_NOLOADS) && j >= 2);  // (the prologue issued up to kAhead)
        if (ring && !(first && live)) issue(j + C::kAhead);
      }
      if (!live) continue;
      const bool mma = bl < n_bl;
      const int h = C::kPB == 1 ? 0 : (bl & 1);  // block bl's place in its stage
      if (mma) {  // the block's first fragments: in flight under the screening below
        fa[0] = frag(j, 0, h);
        fa[1] = frag(j, 1, h);
      }
      // block bi's screening, then a seeding event (the first one before block 1's screening, which
      // then runs with the first seed after block 0's parked scores)
      if (!first) finish_block(bi);
      if (ss && (first || in_sched((uint32_t)(sched >> 32), bi, 1))) event_site(first);
      if (ss && bi >= 3 && in_sched((uint32_t)(sched >> 32), bi - 1, 1)) seed_read();
      if (first) {
        if (ring) {
          issue(j + C::kAhead);
          young = 0;  // the ring's pieces are the youngest now: the next sync waits for everything
        }
        replay(b_begin * kTR);
        finish_block(bi);
      }
      if (mma) stage_mma(j, h);
    }
  }

  // this lane's buffered keys at or above its final threshold, sorted (the query registers are dead
  // from here on). Entries appended while the seed was still loose stay buffered until a compaction;
  // those below the final threshold (the last seed — read one block after the last event and not
  // applied yet — or the lane's own k-th best) cannot be in the query's top k, since the threshold
  // never exceeds the k-th best score. Dropping them first leaves a few inserts per lane instead of
  // up to kBufCap (a wave runs as many as its fullest lane).
  if (ss) {
    wait_vm<0>();
    asm volatile("" ::: "memory");
    apply_seed(*reinterpret_cast<const uint64_t*>(land + 512 + fr * 8));
  }
  uint64_t L[kListCap];
#pragma unroll
  for (int j = 0; j < kListCap; ++j) L[j] = 0;
  uint64_t* const lbuf = lb();
  int nk = 0;
#pragma unroll 1
  for (int c = 0; c < nb; ++c) {
    const uint64_t v = lbuf[c * kThreads];
    if (key_score(v) >= thr) lbuf[nk++ * kThreads] = v;
  }
#pragma unroll 1
  for (int c = 0; c < nk; ++c) list_insert<kListCap>(L, lbuf[c * kThreads]);
  // lane fr + 32 hands its list to lane fr through the (idle) ring
  __syncthreads();
  uint64_t* xch = reinterpret_cast<uint64_t*>(smem) + (wave * 32 + fr) * kListCap;
  if (fh) {
#pragma unroll
    for (int j = 0; j < kListCap; ++j) xch[j] = L[j];
  }
  __syncthreads();
  if (!fh && q < n_q) {
#pragma unroll 1
    for (int j = 0; j < k_out; ++j) {
      const uint64_t v = xch[j];
      if (v <= L[kListCap - 1]) break;  // sorted: nothing further can enter
      list_insert<kListCap>(L, v);
    }
    uint64_t* dst = part_keys + ((int64_t)q * n_splits + split) * k_out;
    // kFlagShortLists (the merge that follows stops at a list's first empty slot): the kept keys
    // and one terminating 0, not the whole k slots (most (query, split) lists hold 0-2 keys above
    // the final threshold)
    const bool short_lists = (flags & kFlagShortLists) != 0;
#pragma unroll
    for (int j = 0; j < kListCap; ++j)
      if (j < k_out && (!short_lists || j == 0 || L[j - 1] != 0)) dst[j] = L[j];
  }
  if (bal && tid == 0)
    __hip_atomic_fetch_add(xcdw + 8 + (split & 7), (uint32_t)__builtin_amdgcn_s_memrealtime() - tab[60],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  stamp(62);
  stamp(63, true);
}

bool supported(int dtype, int d_pad_bytes, int k) {
  return (dtype == AHR_BF16 || dtype == AHR_F16) && (d_pad_bytes == 12 * kRowBytes || d_pad_bytes == 6 * kRowBytes) &&
         k >= 1 && k <= 12 && k < kBufCap;
}

void launch_frag(const uint8_t* qbuf, int64_t row_stride, int B, int d_pad_bytes, uint8_t* qfrag, uint32_t* epoch,
                 hipStream_t s) {
  const int ns = d_pad_bytes / 32;
  const int64_t n16 = (int64_t)((B + 31) / 32) * ns * 64;
  hipLaunchKernelGGL(frag_kernel, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, s, qbuf, row_stride, n16, ns,
                     qfrag, epoch);
}

template <int DT, int NKT, int ABL = 0>
void launch_t(const uint8_t* rows, const uint8_t* qfrag, int64_t row_stride, int n_rows, int B, uint32_t row_base,
              int k, uint64_t* part_keys, const float* thr, int n_splits, int qblocks, int flags, uint64_t* pub,
              uint64_t pub_mask, uint64_t ev_mask, hipStream_t s) {
  if constexpr (kAblation && ABL == 0) {  // the profiling build: cost-split variants
    const int abl = ((flags & kFlagSkipEpilogue) ? ABL_NOSCREEN : 0) | ((flags & kFlagNoLoads) ? ABL_NOLOADS : 0) |
                    ((flags & kFlagNoWait) ? ABL_NOWAIT : 0) | ((flags & kFlagNoBarrier) ? ABL_NOBARRIER : 0) |
                    ((flags & kFlagNoLdsRead) ? ABL_NOREAD : 0) | ((flags & kFlagQresTrace) ? ABL_TRACE : 0) |
                    ((flags & kFlagQresEvNoSel) ? ABL_EV_NOSEL : 0) | ((flags & kFlagQresEvNoIssue) ? ABL_EV_NOISSUE : 0);
    if (abl & ABL_TRACE) {  // the stamps go to the buffer AHR_QRES_TRACE_PTR names (device address)
      const char* e = getenv("AHR_QRES_TRACE_PTR");
      if (!e) return;
      thr = reinterpret_cast<const float*>((uintptr_t)strtoull(e, nullptr, 16));
    }
#define AHR_QRES_ABL(V) \
  case V: launch_t<DT, NKT, V>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags, pub, pub_mask, ev_mask, s); return;
    switch (abl) {
      AHR_QRES_ABL(1) AHR_QRES_ABL(3) AHR_QRES_ABL(5) AHR_QRES_ABL(13) AHR_QRES_ABL(17) AHR_QRES_ABL(31)
      AHR_QRES_ABL(32) AHR_QRES_ABL(64) AHR_QRES_ABL(128) AHR_QRES_ABL(192) AHR_QRES_ABL(96) AHR_QRES_ABL(160)
      AHR_QRES_ABL(224) AHR_QRES_ABL(2) AHR_QRES_ABL(8) AHR_QRES_ABL(16) AHR_QRES_ABL(12)
      default: break;
    }
#undef AHR_QRES_ABL
  }
  constexpr auto kern = &topk_qres_kernel<DT, NKT, ABL>;
  static std::atomic<uint64_t> lds_attr{0};  // > 64 KiB dynamic LDS: opt in per device
  constexpr int lds = Cfg<NKT>::kLds;
  ensure_lds_attr(lds_attr, reinterpret_cast<const void*>(kern), lds);
  hipLaunchKernelGGL(kern, dim3((unsigned)(n_splits * qblocks)), dim3(kThreads), lds, s, rows, qfrag,
                     row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags, pub,
                     (pub_mask & 0xffffffffull) | (ev_mask << 32));
}

void launch(int dtype, int k, const uint8_t* rows, const uint8_t* qfrag, int64_t row_stride, int d_pad_bytes,
            int n_rows, int B, uint32_t row_base, uint64_t* part_keys, const float* thr, int n_splits, int qblocks,
            int flags, uint64_t* pub, uint64_t pub_mask, uint64_t ev_mask, hipStream_t s) {
  const bool wide = d_pad_bytes == 12 * kRowBytes;
  pub_mask |= 1;  // block 0's maxima: the first event's sample
#define AHR_QRES_L(D, N) \
  launch_t<D, N>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags, pub, \
                 pub_mask, ev_mask, s)
  if (dtype == AHR_BF16) {
    if (wide)
      AHR_QRES_L(DT_BF16, 12);
    else
      AHR_QRES_L(DT_BF16, 6);
  } else {
    if (wide)
      AHR_QRES_L(DT_F16, 12);
    else
      AHR_QRES_L(DT_F16, 6);
  }
#undef AHR_QRES_L
}

}  // namespace qres
}  // namespace dense
}  // namespace ahr
