// MFMA issue-rate probe (development aid, not part of the library): how fast one SIMD retires bf16
// MFMA chains on random register operands, for the shapes and wave layouts the dense kernels use.
// Each workgroup runs ITER x UNROLL MFMAs per chain; the kernel stamps s_memtime / s_memrealtime so the
// in-kernel clock and cycles per MFMA can be read beside the wall time.
//   build: hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o build/mfma_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int CHAINS, bool S16, int THREADS>
__global__ __launch_bounds__(THREADS) void probe(const uint32_t* seed, int iters, float* out, uint64_t* stamps) {
  const int t = threadIdx.x;
  bf16x8 a, b;
  uint32_t x = seed[(blockIdx.x * THREADS + t) & 4095];
  for (int i = 0; i < 8; ++i) {
    x = x * 1664525u + 1013904223u;
    uint16_t va = (uint16_t)((x >> 16) & 0xBFFF);
    x = x * 1664525u + 1013904223u;
    uint16_t vb = (uint16_t)((x >> 16) & 0xBFFF);
    a[i] = __builtin_bit_cast(__bf16, va);
    b[i] = __builtin_bit_cast(__bf16, vb);
  }
  f32x16 acc[CHAINS];
  f32x4 acc4[CHAINS * 4];
  for (int c = 0; c < CHAINS; ++c) acc[c] = f32x16{};
  for (int c = 0; c < CHAINS * 4; ++c) acc4[c] = f32x4{};
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
#pragma unroll
      for (int c = 0; c < CHAINS; ++c) {
        if constexpr (S16) {
          // the same FLOPs as one 32x32x16 step: four 16x16x32 MFMAs (independent accumulators)
#pragma unroll
          for (int q = 0; q < 2; ++q)
            acc4[c * 4 + q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc4[c * 4 + q], 0, 0, 0);
        } else {
          acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[c], 0, 0, 0);
        }
      }
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int c = 0; c < CHAINS; ++c)
    for (int j = 0; j < 16; ++j) s += acc[c][j];
  for (int c = 0; c < CHAINS * 4; ++c)
    for (int j = 0; j < 4; ++j) s += acc4[c][j];
  out[blockIdx.x * THREADS + t] = s;
  if (t == 0) {
    stamps[blockIdx.x * 2] = t1 - t0;
    stamps[blockIdx.x * 2 + 1] = r1 - r0;
  }
}

template <int CHAINS, bool S16, int THREADS>
void run(const char* name, const uint32_t* seed, float* out, uint64_t* stamps, int iters) {
  const int blocks = 256;
  hipLaunchKernelGGL((probe<CHAINS, S16, THREADS>), dim3(blocks), dim3(THREADS), 0, 0, seed, iters, out, stamps);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int reps = 5;
  hipEventRecord(e0);
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((probe<CHAINS, S16, THREADS>), dim3(blocks), dim3(THREADS), 0, 0, seed, iters, out, stamps);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= reps;
  std::vector<uint64_t> st(blocks * 2);
  hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost);
  double cyc = 0, rt = 0;
  for (int i = 0; i < blocks; ++i) {
    cyc += st[2 * i];
    rt += st[2 * i + 1];
  }
  cyc /= blocks;
  rt /= blocks;
  const double waves = blocks * (THREADS / 64.0);
  // flops per MFMA-equivalent step: 32*32*16*2 = 32768 (S16: 2 x 16x16x32 = 2 x 16384)
  const double mfma_eq = (double)iters * 16 * CHAINS * (S16 ? 1.0 : 1.0);
  const double flops = waves * mfma_eq * 32768.0 * (S16 ? 1.0 : 1.0);
  const double clock_ghz = cyc / (rt / 100.0) / 1000.0;  // memrealtime ticks at 100 MHz
  const double waves_per_simd = THREADS / 256.0;
  printf("%-28s %8.3f ms  %7.1f TFLOP/s  clock %.2f GHz  cycles per 32x32x16-equivalent per SIMD %.1f\n", name, ms,
         flops / (ms * 1e-3) / 1e12, clock_ghz, cyc / (mfma_eq * waves_per_simd));
}

int main() {
  uint32_t* seed;
  float* out;
  uint64_t* stamps;
  hipMalloc(&seed, 4096 * 4);
  std::vector<uint32_t> h(4096);
  for (int i = 0; i < 4096; ++i) h[i] = 0x9E3779B9u * (i + 1);
  hipMemcpy(seed, h.data(), 4096 * 4, hipMemcpyHostToDevice);
  hipMalloc(&out, 256 * 512 * 4);
  hipMalloc(&stamps, 256 * 2 * 8);
  const int iters = 2000;
  run<1, false, 512>("32x32x16 1 chain, 2 w/SIMD", seed, out, stamps, iters);
  run<2, false, 512>("32x32x16 2 chains, 2 w/SIMD", seed, out, stamps, iters / 2);
  run<1, false, 256>("32x32x16 1 chain, 1 w/SIMD", seed, out, stamps, iters);
  run<2, false, 256>("32x32x16 2 chains, 1 w/SIMD", seed, out, stamps, iters / 2);
  run<1, true, 512>("16x16x32 2 chains, 2 w/SIMD", seed, out, stamps, iters);
  run<1, true, 256>("16x16x32 2 chains, 1 w/SIMD", seed, out, stamps, iters);
  run<1, false, 512>("32x32x16 1 chain, 2 w/SIMD", seed, out, stamps, iters);
  return 0;
}
