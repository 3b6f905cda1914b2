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
template <int NV, int KIND, int PRIO = 0>
__global__ __launch_bounds__(512) void probe(int mode, unsigned long long* out, float* sink) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (PRIO && wave >= 4) __builtin_amdgcn_s_setprio(PRIO);
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
      } else if constexpr (KIND == 4 || KIND == 5) {
        // the MFMA wave itself interleaves NV fma (KIND 4) / exp (KIND 5)
        // fillers per MFMA (independent chains), no partner wave
        f32x4 acc[8] = {};
        float a = lane * 0.001f, b = 1.0f - lane * 0.002f;
        float v[16];
        for (int i = 0; i < 16; ++i) v[i] = lane * 0.001f + i;
        for (int it = 0; it < ITERS; ++it) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
#pragma unroll
            for (int f = 0; f < NV; ++f) {
              const int q = (j * NV + f) & 15;
              if constexpr (KIND == 5) v[q] = __builtin_amdgcn_exp2f(v[q]) * 0.5f;
              else v[q] = __builtin_fmaf(v[q], 0.999f, 0.001f);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, NV * (KIND == 5 ? 2 : 1), 0);
          }
          asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
        }
        for (int j = 0; j < 8; ++j) keep += acc[j][0];
        for (int i = 0; i < 16; ++i) keep += v[i];
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
          } else if constexpr (KIND == 6) {
            v[j & 15] = __builtin_amdgcn_exp2f(v[j & 15]);
          } else if constexpr (KIND == 7) {
            v[j & 15] = __builtin_amdgcn_rcpf(v[j & 15]);
          } else if constexpr (KIND == 8) {   // independent pairs, packed mul
            const int k = 2 * (j & 7);
            f32x2 p{v[k], v[k + 1]};
            p = p * f32x2{0.999f, 0.998f};
            v[k] = p.x;
            v[k + 1] = p.y;
          } else if constexpr (KIND == 1) {   // independent pairs (v[2k], v[2k+1]), k = j % 8
            const int k = 2 * (j & 7);
            f32x2 p{v[k], v[k + 1]};
            p = __builtin_elementwise_fma(p, f32x2{0.999f, 0.998f}, f32x2{0.001f, 0.002f});
            v[k] = p.x;
            v[k + 1] = p.y;
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

template <int NV, int KIND, int PRIO = 0>
void run(const char* name, int mode, unsigned long long* d, float* sink, int ncu) {
  hipLaunchKernelGGL((probe<NV, KIND, PRIO>), dim3(ncu), dim3(512), 0, 0, mode, d, sink);
  hipLaunchKernelGGL((probe<NV, KIND, PRIO>), dim3(ncu), dim3(512), 0, 0, mode, d, sink);
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

template <int NV, int KIND, int PRIO = 0>
void trio(const char* name, unsigned long long* d, float* sink, int ncu) {
  run<NV, KIND, PRIO>(name, 1, d, sink, ncu);
  run<NV, KIND, PRIO>(name, 2, d, sink, ncu);
  run<NV, KIND, PRIO>(name, 3, d, sink, ncu);
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
  trio<32, 0>("f32 MFMA + 32 fma", d, sink, ncu);
  trio<32, 3>("bf16 MFMA + 32 fma", d, sink, ncu);
  // same-wave fillers: 2, 4, 6, 8 fma or 2, 4 exp per MFMA (mode 1 = MFMA waves only;
  // mode 3 adds the partner VALU wave with 32 fma per iteration)
  run<2, 4>("f32 MFMA w/ 2 fma fillers", 1, d, sink, ncu);
  run<4, 4>("f32 MFMA w/ 4 fma fillers", 1, d, sink, ncu);
  run<6, 4>("f32 MFMA w/ 6 fma fillers", 1, d, sink, ncu);
  run<8, 4>("f32 MFMA w/ 8 fma fillers", 1, d, sink, ncu);
  run<12, 4>("f32 MFMA w/ 12 fma fillers", 1, d, sink, ncu);
  run<2, 5>("f32 MFMA w/ 2 exp fillers", 1, d, sink, ncu);
  run<4, 5>("f32 MFMA w/ 4 exp fillers", 1, d, sink, ncu);
  run<4, 4>("f32 MFMA w/ 4 fma + partner", 3, d, sink, ncu);
  // round 4: partner-wave costs of packed fp32, bare transcendentals
  trio<32, 1>("f32 MFMA + 32 pk_fma", d, sink, ncu);
  trio<32, 8>("f32 MFMA + 32 pk_mul", d, sink, ncu);
  trio<32, 6>("f32 MFMA + 32 exp", d, sink, ncu);
  trio<32, 7>("f32 MFMA + 32 rcp", d, sink, ncu);
  trio<64, 0>("f32 MFMA + 64 fma", d, sink, ncu);
  trio<64, 1>("f32 MFMA + 64 pk_fma", d, sink, ncu);
  hipFree(d);
  hipFree(sink);
  return 0;
}
