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
#include "ahr_qres_common.h"

namespace ahr {
namespace dense {
namespace qres {


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


// SYNC: 0 = a workgroup barrier per stage (default), 1 = the same with waves 4-7 one stage
// behind (A/B), 2 = one barrier per block (A/B).
template <int DT, int NKT, int KCAP, int SYNC, int SCR, int ABL>
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
  // (64-bit divisions run on the VALU: readfirstlane keeps the loop bounds, the stage index and the
  // control flow built on them scalar)
  const int b_begin = __builtin_amdgcn_readfirstlane((int)((int64_t)split * n_blocks / n_splits));
  const int b_end = __builtin_amdgcn_readfirstlane((int)((int64_t)(split + 1) * n_blocks / n_splits));
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
              if (nb == kBufCap) compact();  // k_out + 4 > kBufCap (k = 12): one more cut mid-quad
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
  // SYNC = 2: one barrier per 32-row block instead of one per stage. At a block's first stage e
  // a wave waits for ALL its pieces in flight (stages e and e + 1: vmcnt(0)), then the barrier:
  // everyone's e and e + 1 landed and everyone finished stage e - 1, so e + 2 may take stage
  // e - 2's slot now and e + 3 stage e - 1's at the block's second stage, which needs neither a
  // wait nor a barrier. The block's screening (after the barrier) then has two stages of MFMAs,
  // not one, to even out between the waves before the next barrier; the price is waiting for
  // stage e + 1 one stage after its issue instead of two.
  auto stage_sync_blk = [&](int j) __attribute__((always_inline)) {
    if (!(j & 1)) {
      wait_vm<0>();
      lds_barrier();
    }
    if (j + 2 < n_st) issue(j + 2);
  };
  auto stage_sync = [&](int j) __attribute__((always_inline)) {
    if constexpr (SYNC == 2) {
      stage_sync_blk(j);
      return;
    }
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
  const int lag = (SYNC == 1 && wave >= 4) ? 1 : 0;
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

bool supported(int dtype, int d_pad_bytes, int k) {
  return (dtype == AHR_BF16 || dtype == AHR_F16) && d_pad_bytes == 12 * kRowBytes && k >= 1 && k <= 12 &&
         k < kBufCap;
}


int frag_mode(int k, int flags) { return use16(k, flags) ? 16 : 32; }

void launch_frag(const uint8_t* qbuf, int64_t row_stride, int B, int d_pad_bytes, int k, uint8_t* qfrag, int flags,
                 hipStream_t s) {
  if (!use16(k, flags)) {  // the 32x32x16 kernel's layout: 32-query groups, k16 steps
    const int ns = d_pad_bytes / 32;
    const int64_t n16 = (int64_t)((B + 31) / 32) * ns * 64;
    hipLaunchKernelGGL(frag_kernel, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, s, qbuf, row_stride, n16, ns,
                       qfrag);
    return;
  }
  launch_frag16(qbuf, row_stride, B, d_pad_bytes, qfrag, s);
}

template <int DT, int KCAP, int SYNC, int SCR, int ABL = 0>
void launch_t(const uint8_t* rows, const uint8_t* qfrag, int64_t row_stride, int n_rows, int B, uint32_t row_base,
              int k, uint64_t* part_keys, const float* thr, int n_splits, int qblocks, int flags, hipStream_t s) {
  if constexpr (kAblation && ABL == 0 && DT == DT_BF16) {  // the profiling build: cost-split variants
    const int abl = ((flags & kFlagSkipEpilogue) ? ABL_NOSCREEN : 0) | ((flags & kFlagNoLoads) ? ABL_NOLOADS : 0) |
                    ((flags & kFlagNoWait) ? ABL_NOWAIT : 0) | ((flags & kFlagNoBarrier) ? ABL_NOBARRIER : 0) |
                    ((flags & kFlagNoLdsRead) ? ABL_NOREAD : 0);
#define AHR_QRES_ABL(V) \
  case V: launch_t<DT, KCAP, SYNC, SCR, V>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags, s); return;
    switch (abl) {
      AHR_QRES_ABL(1) AHR_QRES_ABL(3) AHR_QRES_ABL(5) AHR_QRES_ABL(13) AHR_QRES_ABL(17) AHR_QRES_ABL(31)
      default: break;
    }
#undef AHR_QRES_ABL
  }
  constexpr auto kern = &topk_qres_kernel<DT, 12, KCAP, SYNC, SCR, ABL>;
  static std::atomic<uint64_t> lds_attr{0};  // > 64 KiB dynamic LDS: opt in per device
  ensure_lds_attr(lds_attr, reinterpret_cast<const void*>(kern), Cfg<12>::kLds);
  hipLaunchKernelGGL(kern, dim3((unsigned)(n_splits * qblocks)), dim3(kThreads), Cfg<12>::kLds, s, rows, qfrag,
                     row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags);
}

template <int DT, int KCAP>
void launch_s(const uint8_t* rows, const uint8_t* qfrag, int64_t row_stride, int n_rows, int B, uint32_t row_base,
              int k, uint64_t* part_keys, const float* thr, int n_splits, int qblocks, int flags, hipStream_t s) {
  if (flags & kFlagQresStagger)
    launch_t<DT, KCAP, 1, 1>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags, s);
  else if (flags & kFlagQresBlkSync)
    launch_t<DT, KCAP, 2, 1>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags, s);
  else if (flags & kFlagQresScreenLoop)
    launch_t<DT, KCAP, 0, 0>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags, s);
  else
    launch_t<DT, KCAP, 0, 1>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags, s);
}

void launch(int dtype, int k, const uint8_t* rows, const uint8_t* qfrag, int64_t row_stride, int n_rows, int B,
            uint32_t row_base, uint64_t* part_keys, const float* thr, int n_splits, int qblocks, int flags,
            hipStream_t s) {
  if (use16(k, flags)) {
    launch16(dtype, k, rows, qfrag, row_stride, n_rows, B, row_base, part_keys, thr, n_splits, qblocks, flags, s);
    return;
  }
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
