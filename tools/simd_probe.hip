// Which SIMD does each wave of a 768-thread, 1-workgroup-per-CU launch land on?
// (diagnostic for the Winograd conv's role split; reads HW_ID, writes one int per wave)
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(768) void probe(int* out) {
  extern __shared__ float sm[];
  unsigned hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  if ((threadIdx.x & 63) == 0) {
    sm[threadIdx.x >> 6] = 0.f;
    out[blockIdx.x * 12 + (threadIdx.x >> 6)] = (int)hw;
  }
}
int main() {
  int* d;
  hipMalloc(&d, 64 * 12 * sizeof(int));
  hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
  probe<<<64, 768, 131072>>>(d);
  int h[64 * 12];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int b = 0; b < 4; ++b) {
    printf("wg %d:", b);
    for (int w = 0; w < 12; ++w) printf(" w%d->simd%d", w, (h[b * 12 + w] >> 4) & 3);
    printf("  (cu %d)\n", (h[b * 12] >> 8) & 15);
  }
  return 0;
}
