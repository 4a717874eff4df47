// v_permlane16_swap_b32 semantics probe (development aid): lane l of x holds 1000 + l, of y 2000 + l;
// prints which source each lane of both results holds after __builtin_amdgcn_permlane16_swap(x, y).
//   build: hipcc --offload-arch=gfx950 -O2 tools/permlane_probe.hip -o tools/permlane_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* a, unsigned* b) {
  const unsigned x = 1000 + threadIdx.x, y = 2000 + threadIdx.x;
  auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  a[threadIdx.x] = r[0];
  b[threadIdx.x] = r[1];
}
int main() {
  unsigned *a, *b, ha[64], hb[64];
  hipMalloc(&a, 256);
  hipMalloc(&b, 256);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, a, b);
  hipMemcpy(ha, a, 256, hipMemcpyDeviceToHost);
  hipMemcpy(hb, b, 256, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; l += 8) printf("lane %2d: x' = %u  y' = %u\n", l, ha[l], hb[l]);
  return 0;
}
