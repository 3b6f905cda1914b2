// Diagnostic microbenchmark: does fp32 MFMA (v_mfma_f32_16x16x4_f32) on one
// wave overlap with VALU work of another wave on the same SIMD?
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_valu_probe.hip -o tools/mfma_valu_probe
// One 512-thread workgroup per CU: waves 0-3 (one per SIMD) run the MFMA loop,
// waves 4-7 (the partner on each SIMD) run NV independent VALU ops per
// iteration (fma, packed fma, or exp).  Cycles per iteration (s_memtime) for
// each role, median over workgroups.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>
#include <algorithm>

using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x2 = __attribute__((ext_vector_type(2))) float;

constexpr int ITERS = 256;

// mode: bit 0 = MFMA waves active, bit 1 = VALU waves active;
// kind: 0 fma, 1 pk_fma, 2 exp, 3 bf16 MFMA (32x32x16) instead of f32 MFMA
template <int NV, int KIND>
__global__ __launch_bounds__(512) void probe(int mode, unsigned long long* out, float* sink) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  float keep = 0.f;
  if (wave < 4) {
    if (mode & 1) {
      if constexpr (KIND == 3) {
        using b16x8 = __attribute__((ext_vector_type(8))) __bf16;
        using f32x16 = __attribute__((ext_vector_type(16))) float;
        f32x16 acc[4] = {};
        b16x8 a, b;
        for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(lane * 0.01f + i); b[i] = (__bf16)(i - lane * 0.02f); }
        for (int it = 0; it < ITERS; ++it) {
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j], 0, 0, 0);
        }
        for (int j = 0; j < 4; ++j) keep += acc[j][0];
      } else {
        f32x4 acc[8] = {};
        float a = lane * 0.001f, b = 1.0f - lane * 0.002f;
        for (int it = 0; it < ITERS; ++it) {
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
        }
        for (int j = 0; j < 8; ++j) keep += acc[j][0];
      }
    }
  } else {
    if (mode & 2) {
      float v[16];
      for (int i = 0; i < 16; ++i) v[i] = lane * 0.001f + i;
      for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          if constexpr (KIND == 2) {
            v[j & 15] = __builtin_amdgcn_exp2f(v[j & 15]) * 0.5f;
          } else if constexpr (KIND == 1) {
            f32x2 p{v[j & 15], v[(j + 1) & 15]};
            p = __builtin_elementwise_fma(p, f32x2{0.999f, 0.998f}, f32x2{0.001f, 0.002f});
            v[j & 15] = p.x;
            v[(j + 1) & 15] = p.y;
          } else {
            v[j & 15] = __builtin_fmaf(v[j & 15], 0.999f, 0.001f);
          }
        }
        asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
      }
      for (int i = 0; i < 16; ++i) keep += v[i];
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[blockIdx.x * 8 + wave] = t1 - t0;
  if (keep == 12345.f) sink[threadIdx.x] = keep;
}

template <int NV, int KIND>
void run(const char* name, int mode, unsigned long long* d, float* sink, int ncu) {
  hipLaunchKernelGGL((probe<NV, KIND>), dim3(ncu), dim3(512), 0, 0, mode, d, sink);
  hipLaunchKernelGGL((probe<NV, KIND>), dim3(ncu), dim3(512), 0, 0, mode, d, sink);
  std::vector<unsigned long long> h(ncu * 8);
  hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
  std::vector<double> m, v;
  for (int b = 0; b < ncu; ++b)
    for (int w = 0; w < 8; ++w) (w < 4 ? m : v).push_back((double)h[b * 8 + w] / ITERS);
  std::sort(m.begin(), m.end());
  std::sort(v.begin(), v.end());
  printf("%-28s mode %d: MFMA waves %7.1f cyc/iter, VALU waves %7.1f cyc/iter\n", name, mode,
         m[m.size() / 2], v[v.size() / 2]);
}

template <int NV, int KIND>
void trio(const char* name, unsigned long long* d, float* sink, int ncu) {
  run<NV, KIND>(name, 1, d, sink, ncu);
  run<NV, KIND>(name, 2, d, sink, ncu);
  run<NV, KIND>(name, 3, d, sink, ncu);
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  unsigned long long* d;
  float* sink;
  hipMalloc(&d, ncu * 8 * 8);
  hipMalloc(&sink, 4096);
  printf("%d CUs; per iteration the MFMA waves issue 8 x f32 16x16x4 (256 cyc at 32/MFMA) "
         "or 4 x bf16 32x32x16 (128 cyc)\n", ncu);
  trio<16, 0>("f32 MFMA + 16 fma", d, sink, ncu);
  trio<32, 0>("f32 MFMA + 32 fma", d, sink, ncu);
  trio<64, 0>("f32 MFMA + 64 fma", d, sink, ncu);
  trio<32, 1>("f32 MFMA + 32 pk_fma", d, sink, ncu);
  trio<16, 2>("f32 MFMA + 16 exp", d, sink, ncu);
  trio<32, 0>("bf16 MFMA + 32 fma", d, sink, ncu);
  hipFree(d);
  hipFree(sink);
  return 0;
}
