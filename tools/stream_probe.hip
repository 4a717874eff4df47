// stream_probe.hip — how fast a corpus stream reads on gfx950 as a function of the piece shape
// (development aid for the small-batch stream kernels, not product code).
//
// The stream of topk_small_f32_kernel: one workgroup of 8 waves per CU (256 splits of the rows),
// each wave takes items of R = 8192 / P consecutive rows (round robin over the split's items) and
// reads an item as row_bytes / P steps, step s = bytes [s P, s P + P) of each of its R rows, 8 KiB
// per step by 8 LDS-DMA wave-instructions of 1 KiB into a per-wave ring of S slots (S - 1 steps in
// flight under the current one), then consumes its slot (one ds_read_b128 per lane, summed).
// P = 128 is the shipped fp32 kernel's shape (64-row items, one 128-B line per row per step).
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/stream_probe tools/stream_probe.hip
// usage: tools/stream_probe [n_rows] [reps]   (prints one line per (row_bytes, P, S))
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
  const uint32_t n = (uint32_t)__builtin_amdgcn_readfirstlane((int)bytes);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, (int)n, 0x00020000);
}

template <int P, int S>
__global__ __launch_bounds__(512, 1) void stream_kernel(const uint8_t* __restrict__ corpus, int64_t row_bytes,
                                                        int n_rows, int n_splits, uint32_t* __restrict__ sink) {
  constexpr int R = 8192 / P;      // rows per item
  constexpr int RPI = 1024 / P;    // rows per wave-instruction
  constexpr int CPR = P / 16;      // 16-B chunks per row piece
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int split = blockIdx.x;
  const int r_begin = (int)((int64_t)split * n_rows / n_splits);
  const int r_end = (int)((int64_t)(split + 1) * n_rows / n_splits);
  const int n_items = (r_end - r_begin + R - 1) / R;
  const int n_steps = (int)(row_bytes / P);
  unsigned char* ring = smem + wave * S * 8192;
  const int total = ((n_items - wave + 7) / 8) * n_steps;  // this wave's steps
  if (wave >= n_items) return;
  auto issue = [&](int g, int slot) __attribute__((always_inline)) {  // g: the wave's step index
    const int gi = g < total ? g : total - 1;
    const int item = wave + 8 * (gi / n_steps);
    const int st = gi % n_steps;
    const int r0 = r_begin + item * R;
    const int rows_here = min(R, r_end - r0);
    const __amdgpu_buffer_rsrc_t r = rsrc(corpus + (int64_t)r0 * row_bytes, (uint32_t)(rows_here * row_bytes));
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = j * RPI + lane / CPR;
      const uint32_t off = (uint32_t)(row * row_bytes) + st * P + (lane % CPR) * 16;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(ring + slot * 8192 + j * 1024),
                                               16, off, 0, 0, 0);
    }
  };
#pragma unroll
  for (int t = 0; t < S - 1; ++t) issue(t, t);
  uint32_t acc = 0;
  for (int g = 0; g < total; ++g) {
    const int slot = g % S;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    issue(g + S - 1, (g + S - 1) % S);
    if constexpr (S == 2)
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (S == 3)
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    const u32x4 v = *reinterpret_cast<const u32x4*>(ring + slot * 8192 + lane * 16);
    acc += v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;  // keep the reads
}

template <int P, int S>
double run(const uint8_t* d, int64_t row_bytes, int n_rows, uint32_t* sink, int reps) {
  const int lds = 8 * S * 8192;
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&stream_kernel<P, S>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int i = 0; i < 5; ++i)
    hipLaunchKernelGGL((stream_kernel<P, S>), dim3(256), dim3(512), lds, 0, d, row_bytes, n_rows, 256, sink);
  CHECK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((stream_kernel<P, S>), dim3(256), dim3(512), lds, 0, d, row_bytes, n_rows, 256, sink);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3 / reps;
}

int main(int argc, char** argv) {
  const int n_rows = argc > 1 ? atoi(argv[1]) : 90000;
  const int reps = argc > 2 ? atoi(argv[2]) : 200;
  uint8_t* d;
  uint32_t* sink;
  const int64_t max_bytes = (int64_t)n_rows * 3072;
  CHECK(hipMalloc(&d, max_bytes));
  CHECK(hipMalloc(&sink, 4096));
  CHECK(hipMemset(d, 1, max_bytes));
  for (int64_t rb : {3072, 1536}) {
    const double gb = (double)n_rows * rb / 1e9;
#define RUN(P, S)                                                                                     \
  {                                                                                                   \
    const double us = run<P, S>(d, rb, n_rows, sink, reps);                                           \
    printf("row_bytes %lld P %4d S %d: %7.2f us  %5.2f TB/s\n", (long long)rb, P, S, us, gb * 1e3 / us); \
  }
    RUN(128, 2) RUN(256, 2) RUN(512, 2) RUN(1024, 2) RUN(128, 3) RUN(256, 3) RUN(512, 3) RUN(1024, 3)
#undef RUN
  }
  return 0;
}
