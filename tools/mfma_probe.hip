// fp32 MFMA issue-rate microbenchmark (diagnostic): v_mfma_f32_32x32x2_f32 on
// 8 accumulators per wave, NW waves per workgroup of which NM issue MFMAs,
// a workgroup barrier every PER MFMAs per wave, LDS-limited to 1 WG per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
using f32x16 = __attribute__((ext_vector_type(16))) float;

template <int NW, int NM, int PER, bool BAR>
__global__ __launch_bounds__(NW * 64) void k(float* out, int iters) {
  extern __shared__ float sm[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  f32x16 acc[8];
  for (int x = 0; x < 8; ++x) acc[x] = f32x16{};
  float a = (float)lane, b = (float)(lane + 1);
  for (int it = 0; it < iters; ++it) {
    if (wave < NM) {
#pragma unroll
      for (int m = 0; m < PER / 8; ++m)
#pragma unroll
        for (int x = 0; x < 8; ++x) acc[x] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[x], 0, 0, 0);
#pragma unroll
      for (int x = 0; x < 8; ++x) asm volatile("" : "+v"(acc[x]));
    }
    if (BAR) __syncthreads();
  }
  float s = 0.f;
  for (int x = 0; x < 8; ++x) s += acc[x][0];
  if (s == 12345.f) out[threadIdx.x] = s + sm[0];
}

template <int NW, int NM, int PER, bool BAR>
void run(const char* name, float* d, int iters, int grid) {
  hipFuncSetAttribute((const void*)k<NW, NM, PER, BAR>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
  k<NW, NM, PER, BAR><<<grid, NW * 64, 131072>>>(d, iters);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  k<NW, NM, PER, BAR><<<grid, NW * 64, 131072>>>(d, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double fl = (double)grid * NM * iters * PER * 2.0 * 32 * 32 * 2;
  printf("%-34s %8.1f us  %6.1f TF (%4.1f%% of 157.3)\n", name, ms * 1e3, fl / ms / 1e9, fl / ms / 1e9 / 157.3 * 100);
}

int main() {
  float* d; (void)hipMalloc(&d, 4096 * 4);
  const int grid = 1024, iters = 8;
  run<12, 8, 32, true>("12w 8mfma 32/barrier", d, iters, grid);
  run<12, 8, 32, false>("12w 8mfma 32 no barrier", d, iters, grid);
  run<8, 8, 32, true>("8w 8mfma 32/barrier", d, iters, grid);
  run<12, 8, 128, true>("12w 8mfma 128/barrier", d, iters / 4, grid);
  run<4, 4, 64, true>("4w 4mfma 64/barrier", d, iters, grid);
  run<8, 8, 256, false>("8w 8mfma 256 nobar", d, 1, grid);
  return 0;
}
