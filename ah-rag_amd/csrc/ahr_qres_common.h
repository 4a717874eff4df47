// Device-side pieces of the register-resident kernel translation unit (ahr_qres.hip).
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
constexpr int kSlots = 3;             // ring stages: the one multiplied + 2 in flight

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// the same for a count known only at run time (wave-uniform, clamped to 15: waiting for more of
// the youngest operations is always safe)
__device__ __forceinline__ void wait_vm_dyn(int n) {
  switch (n < 15 ? n : 15) {
#define AHR_WVM(N) \
  case N: wait_vm<N>(); break;
    AHR_WVM(0) AHR_WVM(1) AHR_WVM(2) AHR_WVM(3) AHR_WVM(4) AHR_WVM(5) AHR_WVM(6) AHR_WVM(7)
    AHR_WVM(8) AHR_WVM(9) AHR_WVM(10) AHR_WVM(11) AHR_WVM(12) AHR_WVM(13) AHR_WVM(14)
#undef AHR_WVM
    default: wait_vm<15>(); break;
  }
}

// ABL: cost-split switches of the ablation build (always 0 in the shipped library): 1 = no top-k
// screening, 2 = no corpus DMA after the first stages, 4 = no DMA waits, 8 = no stage barriers,
// 16 = no LDS fragment reads (a register stands in). Compile-time, so the production code path is
// the ABL = 0 instantiation untouched. Every nonzero combination gives wrong results.
enum { ABL_NOSCREEN = 1, ABL_NOLOADS = 2, ABL_NOWAIT = 4, ABL_NOBARRIER = 8, ABL_NOREAD = 16, ABL_TRACE = 32, ABL_EV_NOSEL = 64,
       ABL_EV_NOISSUE = 128 };

}  // namespace qres
}  // namespace dense
}  // namespace ahr
