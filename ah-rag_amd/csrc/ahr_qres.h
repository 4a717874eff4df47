// Launch interface of the query-resident dense top-k kernel (ahr_qres.hip), called by the search
// planner in ahr_dense.hip. Plain pointers and sizes; the kernel itself is described in ahr_qres.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ahr {
namespace dense {
namespace qres {

constexpr int kTQ = 256;     // queries per workgroup: 8 waves x 32
constexpr int kTR = 32;      // corpus rows per block
constexpr int kBufCap = 16;  // per-lane survivor buffer (keys) in LDS

// bf16 / f16 rows of d_pad_bytes = 1536 (d_pad = 768), k <= 12: what the kernel is built for.
bool supported(int dtype, int d_pad_bytes, int k);

// Query rows [B][row_stride] (the convert kernel's storage rows) -> the fragment-major copy the
// planned form reads, one contiguous KiB per wave B operand: 16x16x32 form [B/16 groups][d_pad/32
// k32 steps][64 lanes][16 B] (lane l: query 16g + l%16, bytes [64 S + 16 (l/16), +16)); 32x32x16
// form [B/32][d_pad/16 k16 steps][64][16 B] (lane l: query 32g + l%32, bytes [32 S + 16 (l/32), +16)).
// The buffers are padded to whole 256-query blocks.
void launch_frag(const uint8_t* qbuf, int64_t row_stride, int B, int d_pad_bytes, int k, uint8_t* qfrag, int flags,
                 hipStream_t s);

// The fragment layout the planned form reads: 16 (16x16x32 form) or 32 (32x32x16 form), for the
// fused conversion (convert_queries_frag_kernel) that writes it directly.
int frag_mode(int k, int flags);

// One fused launch: part_keys [B][n_splits][k] (the merge kernels' input), thr [B] optional
// admission seeds. grid = n_splits * qblocks; n_splits % 8 == 0 when flags has the XCD remap bit.
void launch(int dtype, int k, const uint8_t* rows, const uint8_t* qfrag, int64_t row_stride, int n_rows, int B,
            uint32_t row_base, uint64_t* part_keys, const float* thr, int n_splits, int qblocks, int flags,
            hipStream_t s);

}  // namespace qres
}  // namespace dense
}  // namespace ahr
