// Which SIMD does each wave of a 768-thread workgroup land on? (s_getreg HW_ID)
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void __launch_bounds__(768, 3) k(int* out) {
  const int w = threadIdx.x >> 6;
  // HW_REG_HW_ID (4): SIMD_ID = bits [5:4], CU_ID = bits [11:8]
  const unsigned hw = __builtin_amdgcn_s_getreg((1 << 11) | (4 << 6) | 4);   // 2 bits at offset 4
  const unsigned cu = __builtin_amdgcn_s_getreg((3 << 11) | (8 << 6) | 4);   // 4 bits at offset 8
  if ((threadIdx.x & 63) == 0) { out[blockIdx.x * 24 + w * 2] = hw; out[blockIdx.x * 24 + w * 2 + 1] = cu; }
}
int main() {
  int* d; hipMalloc(&d, 8 * 24 * 4);
  hipLaunchKernelGGL(k, dim3(8), dim3(768), 100000, 0, d);   // big LDS: one WG per CU
  int h[8 * 24]; hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  for (int b = 0; b < 8; ++b) { printf("block %d:", b); for (int w = 0; w < 12; ++w) printf(" w%d:s%d", w, h[b * 24 + w * 2]); printf("\n"); }
  return 0;
}
