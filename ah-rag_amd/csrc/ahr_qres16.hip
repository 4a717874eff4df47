// ahr_qres16.hip — the register-resident dense top-k kernel in its v_mfma_f32_16x16x32 form
// (see ahr_qres.hip for the structure; opt-in, kFlagQres16). Its own translation unit: built
// without IEEE NaN quieting (-fno-honor-nans -mno-amdgpu-ieee), so the fmax trees of its
// screening are plain v_max3 chains; the scores it compares are never NaN.
#include "ahr_qres_common.h"

namespace ahr {
namespace dense {
namespace qres {

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
constexpr int kSlots16 = 3;
#ifndef AHR_QRES_PRE4
#define AHR_QRES_PRE4 1
#endif
constexpr int kPre4 = AHR_QRES_PRE4;  // G = 4: the k32 step the previous block's screening precedes

template <int NKT, int W>
struct Cfg16 {
  static constexpr int kSK = NKT / 2;           // k-tiles per stage
  static constexpr int kStage = kSK * kKt;      // 24 KiB at d_pad = 768
  static constexpr int kPieces = kSK * 4;
  static_assert(kPieces % W == 0, "equal DMA share per wave");
  static constexpr int kPPW = kPieces / W;
  static constexpr int kNS = NKT * 2;           // k32 steps
  static constexpr int kSS = kSK * 2;           // k32 steps per stage
  static constexpr int kOffBuf = kSlots16 * kStage;  // [g][kLaneCap][64 W lanes] u64, G * W = 16
  static constexpr int kLds = kOffBuf + kLaneCap * 16 * 64 * 8;
};
static_assert(Cfg16<12, 8>::kLds <= 160 * 1024, "LDS budget: one workgroup per CU");

template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

template <int DT>
__device__ __forceinline__ void mfma16(const u32x4& a, const u32x4& b, f32x4& acc) {
  if constexpr (DT == DT_BF16)
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc, 0,
                                                  0, 0);
  else
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), acc, 0, 0,
                                                 0);
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

// G query groups of 16 per wave: G = 2 (8 waves, 2 per SIMD, 256 VGPRs each) or G = 4 (4 waves,
// 1 per SIMD with 512 registers: 64 resident queries, each A fragment read from LDS feeds 8 MFMAs
// instead of 4, and the previous block's screening runs inside the next block's MFMA stream).
template <int DT, int NKT, int KCAP, int ABL, int G>
__global__ __launch_bounds__(64 * (16 / G)) __attribute__((amdgpu_waves_per_eu(4 / G, 4 / G))) void topk_qres16_kernel(
    const uint8_t* __restrict__ corpus, const uint8_t* __restrict__ qfrag, int64_t row_stride, int n_rows, int n_q,
    uint32_t row_base, int k_out, uint64_t* __restrict__ part_keys, const float* __restrict__ thr_init, int n_splits,
    int qblocks, int flags) {
  constexpr int W = 16 / G;      // waves
  constexpr int NT = 64 * W;     // threads
  using C = Cfg16<NKT, W>;
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
  // (64-bit divisions run on the VALU: readfirstlane keeps the loop bounds, the stage index and the
  // control flow built on them scalar)
  const int b_begin = __builtin_amdgcn_readfirstlane((int)((int64_t)split * n_blocks / n_splits));
  const int b_end = __builtin_amdgcn_readfirstlane((int)((int64_t)(split + 1) * n_blocks / n_splits));
  const int n_st = 2 * (b_end - b_begin);
  const int qw0 = qb * kTQ + wave * 16 * G;
  const bool live = qw0 < n_q;  // wave-uniform: a wave past the batch only stages and syncs
  float thr[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int q = qw0 + 16 * g + fr;
    thr[g] = q < n_q ? (thr_init ? thr_init[q] : -INFINITY) : INFINITY;
  }

  // DMA (the 32x32 kernel's stages): piece p = wave + W i is k-tile p / 4 = wave / 4 + (W / 4) i,
  // rows 8 (wave % 4) .. +8: the pieces of a wave differ by W / 4 k-tiles (soffset, no extra VGPR)
  const int d_row = 8 * (wave & 3) + (lane >> 3);
  const uint32_t src_off = (uint32_t)(d_row * row_stride) + (wave >> 2) * kRowBytes +
                           ((((lane & 7) ^ ((d_row >> 1) & 7))) << 4);
  const int dst_off = (wave >> 2) * kKt + (wave & 3) * 1024;
  const uint32_t blk_bytes = (uint32_t)(kTR * row_stride);
  auto slot_of = [&](int st) __attribute__((always_inline)) { return smem + (st % kSlots16) * C::kStage; };
  auto issue = [&](int st) __attribute__((always_inline)) {
    const int b = b_begin + (st >> 1);
    const __amdgpu_buffer_rsrc_t r =
        tile_rsrc_u(corpus + (int64_t)b * kTR * row_stride + (st & 1) * C::kSK * kRowBytes, blk_bytes);
    unsigned char* slot = slot_of(st) + dst_off;
#pragma unroll
    for (int i = 0; i < C::kPPW; ++i)
      blds16_soff(r, src_off, i * (W / 4) * kRowBytes, slot + i * (W / 4) * kKt);
  };
  if (n_st > 0) issue(0);
  if (n_st > 1) issue(1);

  // resident B fragments: k32 step S of query group g
  // (two arrays of 2 groups: SROA leaves a single [24][4] array of 1.5 KiB in private memory)
  u32x4 qf01[C::kNS][2];
  u32x4 qf23[C::kNS][G == 4 ? 2 : 1];
#define QF(S, g) (*((g) < 2 ? &qf01[S][(g) & 1] : &qf23[S][((g) & 1) % (G == 4 ? 2 : 1)]))
  {
    const uint8_t* src = qfrag + (int64_t)(qb * 16 + wave * G) * C::kNS * 1024 + lane * 16;
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int S = 0; S < C::kNS; ++S) QF(S, g) = *reinterpret_cast<const u32x4*>(src + (g * C::kNS + S) * 1024);
  }
  // consumed here, behind the prologue DMA (see topk_qres_kernel)
#pragma unroll
  for (int S = 0; S < C::kNS; ++S)
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (g < 2)
        asm volatile("" : "+v"(QF(S, g)));
      else  // G = 4: query groups 2, 3 in AGPRs (MFMA B operands read them directly)
        asm volatile("" : "+a"(QF(S, g)));
    }
#pragma unroll
  for (int g = 0; g < G; ++g) asm volatile("" : "+v"(thr[g]));
  auto thr_at = [&](int g) __attribute__((always_inline)) {  // runtime g (thr[g] would go to scratch)
    float t = thr[0];
#pragma unroll
    for (int j = 1; j < G; ++j) {
      float tj = thr[j];
      asm volatile("" : "+v"(tj));  // a select of values, not of addresses (InstCombine would fold it)
      t = g == j ? tj : t;
    }
    return t;
  };
  // Admission is by score alone (score >= thr): a score equal to the threshold whose row would lose
  // the tie is buffered too and dropped by the next compaction or the final sort (no key threshold
  // in registers: the VGPR budget is spent on the resident queries).

  // Per (lane, query group g) LDS area of kLaneCap 8-B slots, slot c at lb[(g * kLaneCap + c) * NT]
  // (a wave's 64 lanes hit 64 consecutive u64). The split's first passing block of a lane-query is
  // staged raw — its 8 scores in slots 0-3 (2 per slot), its first row in slot 4 — with 5 stores and
  // no per-score work; a staged score leaves the candidates through a dead bit. Scores of later
  // passing blocks become keys, growing down from slot 10 (key i in slot 10 - i): up to kStageKeys
  // next to a staged block, kLaneCap once the staged survivors are keys too (key mode). A full
  // buffer is cut to the k best candidates, whose k-th score becomes the lane's threshold.
  // At C2 (seed from 8,192 rows) a lane-query sees ~0.43 passing blocks per split and 7 % see a
  // second: a wave runs the per-score path on a fifth of its blocks, the staging stores on most.
  uint64_t* lb = reinterpret_cast<uint64_t*>(smem + C::kOffBuf) + tid;
  constexpr int kStageKeys = kLaneCap - 5;
  static_assert(kLaneCap - 1 - kStageKeys == 4 && kLaneCap - 1 <= 10,
                "key mode: at most k_out <= 10 keys, the staged survivors land in slots 4..1");
  // per-lane state (the VGPR budget is the resident queries'): stg bit g: block staged, bits
  // [4 + 4 g, +4): keys; dead staged scores in 8 bits per g: stg bits [16 + 8 g) at G = 2, dm at G = 4
  uint32_t stg = 0;
  uint32_t dm = 0;
  constexpr int kDeadSh = G == 2 ? 16 : 0;
  auto nk = [&](int g) __attribute__((always_inline)) { return (int)((stg >> (4 + 4 * g)) & 0xF); };
  auto dead_of = [&](int g) __attribute__((always_inline)) {
    return ((G == 2 ? stg : dm) >> (kDeadSh + 8 * g)) & 0xFFu;
  };
  auto set_dead = [&](int g, uint32_t d) __attribute__((always_inline)) {
    uint32_t& r = G == 2 ? stg : dm;
    r = (r & ~(0xFFu << (kDeadSh + 8 * g))) | (d << (kDeadSh + 8 * g));
  };
  auto slot = [&](int g, int c) __attribute__((always_inline)) { return lb + (g * kLaneCap + c) * NT; };
  auto key_slot = [&](int g, int i) __attribute__((always_inline)) { return slot(g, kLaneCap - 1 - i); };
  // row of staged score j (slot j / 2, half j % 2) = acc[rh][g][r] with rh = j / 4, r = j % 4
  auto row_of = [&](int r0, int j) __attribute__((always_inline)) {
    return (uint32_t)(r0 + 16 * (j >> 2) + 4 * fq + (j & 3));
  };
  auto staged = [&](int g, int j) __attribute__((always_inline)) {
    const uint64_t u = *slot(g, j >> 1);
    return __uint_as_float((uint32_t)((j & 1) ? (u >> 32) : u));
  };
  // A full buffer (nk == kStageKeys next to a staged block, kLaneCap in key mode; rare): the
  // candidates (live staged scores, keys) are cut to the k_out best, the k_out-th best raises the
  // threshold. A staged block still holding live scores with the keys full has at most
  // k_out - kStageKeys <= 4 of them (k_out <= 10): they become keys 6.. in slots 4, 3, .. — read in
  // pair order 3, 2, 1, 0, a slot is only overwritten once its pair is read or holds no live score.
  auto overflow = [&](int g) __attribute__((always_inline)) {
    const bool stgd = stg & (1u << g);
    int n = nk(g);
    uint32_t dead = stgd ? dead_of(g) : 0xFFu;
    const int r0s = stgd ? (int)(uint32_t)*slot(g, 4) : 0;
    const float t = thr[g];
#pragma unroll 1
    for (int j = 0; j < 8; ++j)
      if (!((dead >> j) & 1) && staged(g, j) < t) dead |= 1u << j;
    int total = __builtin_popcount(~dead & 0xFF) + n;
    uint64_t mv = 0;
#pragma unroll 1
    while (total >= k_out) {  // remove minima until k_out are left; the last one found is the k-th
      int mi = -1;
      mv = ~0ull;
#pragma unroll 1
      for (int j = 0; j < 8; ++j) {
        if ((dead >> j) & 1) continue;
        const uint64_t kk = make_key(staged(g, j), row_base + row_of(r0s, j));
        if (kk < mv) {
          mv = kk;
          mi = j;
        }
      }
#pragma unroll 1
      for (int c = 0; c < n; ++c) {
        const uint64_t kk = *key_slot(g, c);
        if (kk < mv) {
          mv = kk;
          mi = 8 + c;
        }
      }
      if (total == k_out) break;
      if (mi < 8) {
        dead |= 1u << mi;
      } else {
        *key_slot(g, mi - 8) = *key_slot(g, n - 1);
        --n;
      }
      --total;
    }
    if (total == k_out && k_out > 0) thr[g] = fmaxf(thr[g], key_score(mv));
    if (stgd && n == kStageKeys) {  // no room left next to the staged block: its survivors become keys
#pragma unroll 1
      for (int c = 3; c >= 0; --c) {
        const uint64_t u = *slot(g, c);
#pragma unroll 1
        for (int h = 0; h < 2; ++h) {
          const int j = 2 * c + h;
          if (!((dead >> j) & 1)) {
            *key_slot(g, n) = make_key(__uint_as_float((uint32_t)(h ? (u >> 32) : u)), row_base + row_of(r0s, j));
            ++n;
          }
        }
      }
      stg &= ~(1u << g);
      dead = 0xFF;
    }
    stg = (stg & ~(0xFu << (4 + 4 * g))) | ((uint32_t)n << (4 + 4 * g));
    set_dead(g, (stg & (1u << g)) ? dead : 0u);
  };
  // a finished block: per query group g the lane's 8 scores acc[rh][g][r], rows r0 + 16 rh + 4 fq + r
  auto screen = [&](const f32x4 (&acc)[2][G], int r0) __attribute__((always_inline)) {
    bool pass[G];
    bool any = false;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float m = fmaxf(fmaxf(fmaxf(acc[0][g][0], acc[0][g][1]), fmaxf(acc[0][g][2], acc[0][g][3])),
                            fmaxf(fmaxf(acc[1][g][0], acc[1][g][1]), fmaxf(acc[1][g][2], acc[1][g][3])));
      pass[g] = m >= thr[g];
      any = any || pass[g];
    }
    if (!__builtin_amdgcn_ballot_w64(any)) return;  // wave-uniform: the common case
    if constexpr ((ABL & ABL_MAXONLY) != 0) {  // cost split: the maxima and the ballot only
      asm volatile("" ::"v"(thr[0]));
      return;
    }
    // (compile-time g: a loop this large is not unrolled, and thr would be indexed at run time)
    static_for<0, G>([&](auto GI) __attribute__((always_inline)) {
      constexpr int g = decltype(GI)::value;
      if (pass[g]) {
        if (!(stg & (1u << g)) && nk(g) == 0) {  // the split's first passing block: stage it raw
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const int rh = c >> 1, r = 2 * (c & 1);
            *slot(g, c) = ((uint64_t)__float_as_uint(acc[rh][g][r + 1]) << 32) | __float_as_uint(acc[rh][g][r]);
          }
          *slot(g, 4) = (uint32_t)r0;
          uint32_t dead = 0;
          if (r0 + kTR > n_rows) {  // ragged last block: rows past the corpus are dead from the start
#pragma unroll 1
            for (int j = 0; j < 8; ++j)
              if (row_of(r0, j) >= (uint32_t)n_rows) dead |= 1u << j;
          }
          stg |= 1u << g;
          set_dead(g, dead);
        } else {  // rare: keys for the passing scores only (one loop trip per passing score)
          if constexpr ((ABL & ABL_STAGEONLY) != 0) return;
          uint32_t pm = 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) pm |= (acc[j >> 2][g][j & 3] >= thr[g] ? 1u : 0u) << j;
#pragma unroll 1
          while (pm) {
            const int jj = __builtin_ctz(pm);
            pm &= pm - 1;
            float v = acc[0][g][0];
#pragma unroll
            for (int j2 = 1; j2 < 8; ++j2) v = (jj == j2) ? acc[j2 >> 2][g][j2 & 3] : v;
            const uint32_t row = row_of(r0, jj);
            if (v >= thr[g] && row < (uint32_t)n_rows) {  // (thr may have risen in this loop)
              *key_slot(g, nk(g)) = make_key(v, row_base + row);
              stg += 1u << (4 + 4 * g);
              if (nk(g) == ((stg & (1u << g)) ? kStageKeys : kLaneCap)) overflow(g);
            }
          }
        }
      }
    });
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
    if constexpr ((ABL & ABL_NOREAD) != 0) return QF((s + 5) % C::kNS, rh);
    return *reinterpret_cast<const u32x4*>(slot + (s >> 1) * kKt + rh * 16 * kRowBytes + a_off[s & 1]);
  };
  u32x4 fa[2][2];  // [buffer][rh]: step t + 1 in flight while step t multiplies
  f32x4 acc[2][G];
  f32x4 accp[2][G];  // the previous block's scores while its screening runs (G = 4)
  // one stage: 12 k32 steps, step t prefetches step t + 1 of the same stage; `pre` (the previous
  // block's screening) runs before step kPre: at G = 2 first (acc is overwritten only by the first
  // MFMA, no second register set), at G = 4 behind the first steps' MFMAs, which it overlaps
  constexpr int kPre = G == 4 ? kPre4 : 0;
  auto stage = [&](auto H, int st, auto&& pre) __attribute__((always_inline)) {
    constexpr int h = decltype(H)::value;
    const unsigned char* slot = slot_of(st);
    if (kPre == 0) pre();
#pragma unroll
    for (int rh = 0; rh < 2; ++rh) fa[0][rh] = frag(slot, 0, rh);
    auto step = [&](auto T) __attribute__((always_inline)) {
      constexpr int t = decltype(T)::value;
      if constexpr (t + 1 < C::kSS && (kPre == 0 || t + 1 != kPre)) {
#pragma unroll
        for (int rh = 0; rh < 2; ++rh) fa[(t + 1) & 1][rh] = frag(slot, t + 1, rh);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int rh = 0; rh < 2; ++rh)
#pragma unroll
        for (int g = 0; g < G; ++g) {
          if constexpr (h == 0 && t == 0) {
            f32x4 z = {};
            mfma16<DT>(fa[0][rh], QF(0, g), z);
            acc[rh][g] = z;
          } else {
            mfma16<DT>(fa[t & 1][rh], QF(h * C::kSS + t, g), acc[rh][g]);
          }
        }
      __builtin_amdgcn_sched_barrier(0);
    };
    // (compile-time steps: a loop holding the screening would not be unrolled, and the resident
    // fragments would be indexed at run time, from private memory)
    static_for<0, kPre>(step);
    if constexpr (kPre > 0) {  // (step kPre's fragments are read after it: 8 registers fewer live)
      pre();
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int rh = 0; rh < 2; ++rh) fa[kPre & 1][rh] = frag(slot, kPre, rh);
    }
    static_for<kPre, C::kSS>(step);
  };
  // a finished block's top-k screening, run after the NEXT block's first barrier, so no wave waits
  // at a barrier for another wave's survivors (the partner wave's MFMAs fill the SIMD meanwhile)
  auto finish = [&](const f32x4 (&a)[2][G], int b) __attribute__((always_inline)) {
    if constexpr ((ABL & ABL_NOSCREEN) != 0) {  // GEMM only: every chain kept live (rule 17), no top-k
#pragma unroll
      for (int rh = 0; rh < 2; ++rh)
#pragma unroll
        for (int g = 0; g < G; ++g) asm volatile("" ::"v"(a[rh][g]));
    } else {
      screen(a, b * kTR);
    }
  };
  auto nothing = []() __attribute__((always_inline)) {};
#pragma unroll 1
  for (int b = b_begin; b < b_end; ++b) {
    const int st0 = 2 * (b - b_begin);
    stage_sync(st0);
    if (live) {
      if (b > b_begin) {
#pragma unroll
        for (int rh = 0; rh < 2; ++rh)
#pragma unroll
          for (int g = 0; g < G; ++g) accp[rh][g] = acc[rh][g];
        stage(std::integral_constant<int, 0>{}, st0, [&]() __attribute__((always_inline)) { finish(accp, b - 1); });
      } else
        stage(std::integral_constant<int, 0>{}, st0, nothing);
    }
    stage_sync(st0 + 1);
    if (live) stage(std::integral_constant<int, 1>{}, st0 + 1, nothing);
  }
  if (live && b_end > b_begin) finish(acc, b_end - 1);

  // each lane sorts its two areas (the query registers are dead by now): keys plus a staged block's
  // scores at or above the threshold; per query the 4 lane quarters' lists meet in the idle ring,
  // quarter 0 merges them and writes the (query, split) list
  uint64_t* xch = reinterpret_cast<uint64_t*>(smem);  // [quarter 1..3][query-local 256][KCAP]
#pragma unroll 1
  for (int g = 0; g < G; ++g) {
    uint64_t L[KCAP];
#pragma unroll
    for (int j = 0; j < KCAP; ++j) L[j] = 0;
#pragma unroll 1
    for (int c = 0; c < nk(g); ++c) list_insert<KCAP>(L, *key_slot(g, c));
    if (stg & (1u << g)) {
      const float tg = thr_at(g);
      const uint32_t dead = dead_of(g);
      const int r0s = (int)(uint32_t)*slot(g, 4);
#pragma unroll 1
      for (int jj = 0; jj < 8; ++jj) {
        const float v = staged(g, jj);
        if (!((dead >> jj) & 1) && v >= tg) list_insert<KCAP>(L, make_key(v, row_base + row_of(r0s, jj)));
      }
    }
    const int qlx = wave * 16 * G + 16 * g + fr;
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

#undef QF

template <int DT, int KCAP, int G, int ABL = 0>
void launch16_t(const uint8_t* rows, const uint8_t* qfrag, int64_t row_stride, int n_rows, int B, uint32_t row_base,
              int k, uint64_t* part_keys, const float* thr, int n_splits, int qblocks, int flags, hipStream_t s) {
  if constexpr (kAblation && ABL == 0 && DT == DT_BF16) {  // the profiling build: cost-split variants
    const int abl = ((flags & kFlagSkipEpilogue) ? ABL_NOSCREEN : 0) | ((flags & kFlagNoLoads) ? ABL_NOLOADS : 0) |
                    ((flags & kFlagNoWait) ? ABL_NOWAIT : 0) | ((flags & kFlagNoBarrier) ? ABL_NOBARRIER : 0) |
                    ((flags & kFlagNoLdsRead) ? ABL_NOREAD : 0) | ((flags & kFlagMaxOnly) ? ABL_MAXONLY : 0) |
                    ((flags & kFlagQresScreenLoop) ? ABL_STAGEONLY : 0);  // (the switch is the 32x32 form's A/B)
#define AHR_QRES_ABL(V) \
  case V: launch16_t<DT, KCAP, G, V>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags, s); return;
    switch (abl) {
      AHR_QRES_ABL(1) AHR_QRES_ABL(3) AHR_QRES_ABL(5) AHR_QRES_ABL(13) AHR_QRES_ABL(17) AHR_QRES_ABL(31)
      AHR_QRES_ABL(32) AHR_QRES_ABL(64)
      default: break;
    }
#undef AHR_QRES_ABL
  }
  using C = Cfg16<12, 16 / G>;
  constexpr auto kern = &topk_qres16_kernel<DT, 12, KCAP, ABL, G>;
  static_assert(3 * kTQ * KCAP * 8 <= kSlots16 * C::kStage, "end exchange must fit the ring");
  static std::atomic<uint64_t> lds_attr{0};  // > 64 KiB dynamic LDS: opt in per device
  ensure_lds_attr(lds_attr, reinterpret_cast<const void*>(kern), C::kLds);
  hipLaunchKernelGGL(kern, dim3((unsigned)(n_splits * qblocks)), dim3(64 * (16 / G)), C::kLds, s, rows, qfrag,
                     row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks, flags);
}

void launch_frag16(const uint8_t* qbuf, int64_t row_stride, int B, int d_pad_bytes, uint8_t* qfrag, hipStream_t s) {
  const int ns = d_pad_bytes / 64;  // 16-query groups, k32 steps
  const int64_t n16 = (int64_t)((B + 15) / 16) * ns * 64;
  hipLaunchKernelGGL(frag16_kernel, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, s, qbuf, row_stride, n16, ns,
                     qfrag);
}

void launch16(int dtype, int k, const uint8_t* rows, const uint8_t* qfrag, int64_t row_stride, int n_rows, int B,
              uint32_t row_base, uint64_t* part_keys, const float* thr, int n_splits, int qblocks, int flags,
              hipStream_t s) {
  const bool w4 = flags & kFlagQres4w;
#define AHR_QRES16_GO(DT, KC)                                                                                        \
  (w4 ? launch16_t<DT, KC, 4>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks,    \
                              flags, s)                                                                              \
      : launch16_t<DT, KC, 2>(rows, qfrag, row_stride, n_rows, B, row_base, k, part_keys, thr, n_splits, qblocks,    \
                              flags, s))
  if (dtype == AHR_BF16) {
    if (k <= 8)
      AHR_QRES16_GO(DT_BF16, 8);
    else
      AHR_QRES16_GO(DT_BF16, 12);
  } else {
    if (k <= 8)
      AHR_QRES16_GO(DT_F16, 8);
    else
      AHR_QRES16_GO(DT_F16, 12);
  }
#undef AHR_QRES16_GO
}

}  // namespace qres
}  // namespace dense
}  // namespace ahr
