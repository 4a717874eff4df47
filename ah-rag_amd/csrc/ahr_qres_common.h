// Device-side pieces shared by the register-resident kernel translation units (ahr_qres.hip:
// 32x32x16 form and launchers; ahr_qres16.hip: 16x16x32 form).
#pragma once

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

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ABL: cost-split switches of the ablation build (always 0 in the shipped library): 1 = no top-k
// screening, 2 = no corpus DMA after the first stages, 4 = no DMA waits, 8 = no stage barriers,
// 16 = no LDS fragment reads (a register stands in). Compile-time, so the production code path is
// the ABL = 0 instantiation untouched. Every nonzero combination gives wrong results.
enum { ABL_NOSCREEN = 1, ABL_NOLOADS = 2, ABL_NOWAIT = 4, ABL_NOBARRIER = 8, ABL_NOREAD = 16, ABL_MAXONLY = 32,
       ABL_STAGEONLY = 64 /* 16x16 form: first-pass staging only, later passing blocks dropped */ };

constexpr int kLaneCap = 11;  // 16x16x32 form: keys per (lane, query); k <= 10 leaves one free slot

// the 16x16x32 forms on request (k <= 10: their lane buffers); the 32x32x16 form by default
inline bool use16(int k, int flags) { return k < kLaneCap && (flags & (kFlagQres16 | kFlagQres4w)); }

// ahr_qres16.hip
void launch_frag16(const uint8_t* qbuf, int64_t row_stride, int B, int d_pad_bytes, uint8_t* qfrag, hipStream_t s);
void launch16(int dtype, int k, const uint8_t* rows, const uint8_t* qfrag, int64_t row_stride, int n_rows, int B,
              uint32_t row_base, uint64_t* part_keys, const float* thr, int n_splits, int qblocks, int flags,
              hipStream_t s);

}  // namespace qres
}  // namespace dense
}  // namespace ahr
