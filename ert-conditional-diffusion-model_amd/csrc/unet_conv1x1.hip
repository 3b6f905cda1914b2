// 1x1 convolution (the ResBlock skip projections) as a plain GEMM per sample on
// fp32 MFMA (v_mfma_f32_16x16x4_f32):  out[b][co][p] = bias[co] + sum_ci W[co][ci] x[b][ci][p]
//
// Work item = (co group of 64, P consecutive output pixels: one sample's, or
// two samples' 256-pixel planes at 16x16).  4 waves, wave w = 16 co; the A
// operand is the pixel side (16 px x 4 ci fragments read from LDS), the B
// operand the weights (4 ci x 16 co), so the accumulators hold 4 consecutive
// pixels of one channel per lane (one float4 store per fragment).
//   * the input is LDS-DMA'd in 8-channel chunks ([ci 8][P px], 1 KB per
//     (sample, channel, 256 px) piece, no VALU) together with the chunk's weight
//     slice (gathered per lane from the direct packing, 2 KB), one chunk ahead
//     into a 2-slot ring -- the only vector memory operations of the K loop,
//     counted by hand;
//   * per k-step (4 channels) a wave issues P/16 + 1 ds_reads and P/16 MFMAs.
// The old implicit-GEMM kernel (conv_kernel<1, ...>: register staging, one
// launch of short K loops per 256-px tile) ran the U2 skips at 30-57 % of the
// fp32 peak.  Exact fp32 products, k-ordered accumulation per output.
#include <cstdlib>

#include "unet.h"
#include "unet_pack.h"

namespace ertd {
namespace unet {

namespace {

constexpr int NW = 4;
constexpr int T1 = 64 * NW;
using f32x4 = __attribute__((ext_vector_type(4))) float;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned;

__device__ __forceinline__ unsigned lds_u32(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// one 1-KB LDS-DMA: 16 B per lane from the lane's own src (a gather) to dst + 16 B * lane
__device__ __forceinline__ void dma1k(const float* src, float* dst) {
  const unsigned d = __builtin_amdgcn_readfirstlane(lds_u32(dst));
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(d)
      : "memory");
}

template <int P, int CCH>
__global__ __launch_bounds__(T1, 2) void conv1x1_kernel(ConvArgs a, int HW, int npb) {
  constexpr int PF = P / 16;                    // pixel fragments per wave
  constexpr int XCH = CCH * P;                  // X floats per chunk (CCH input channels)
  constexpr int WCH = 64 * CCH;                 // the chunk's weight slice (64 co x CCH ci)
  constexpr int SLOT = XCH + WCH;
  constexpr int CPW = CCH / NW;                 // channels whose pieces a wave DMAs
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int Cin = a.Cin, Ca = a.Ca;
  const int nc32 = (Cin + 31) / 32;             // the packing's 32-channel chunks
  const int tid = threadIdx.x, lane = tid & 63;
  const int cb = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int it = blockIdx.x;
  const int cog = it / npb, pb = it - cog * npb;
  const int ups = HW / 256;                     // 256-px units per sample
  const int nchunk = Cin / CCH;

  // chunk g -> ring slot: X pieces (channel c, 256-px unit u), wave cb issues
  // c = 2 cb, 2 cb + 1; waves 0 / 1 also gather the weight slice: W[co][ci] of
  // the chunk's 8 channels sits in the direct packing's (tile, 32-ch chunk)
  // block as 4 step-pair rows x 64 floats (one lane half), per tile
  // (pack_conv_elem: ci % 32 = 16 hh + 2 sp + e, lane = 32 hh + co % 32);
  // LDS slice [tile 2][sp 4][64]
  auto dma_chunk = [&](int g, float* dst) {
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int c = CPW * cb + j;
      const int cg = g * CCH + c;
#pragma unroll
      for (int u = 0; u < P / 256; ++u) {
        const int q = pb * (P / 256) + u;       // global 256-px unit
        const int smp = q / ups, off = (q - smp * ups) * 256;
        const float* src = cg < Ca ? a.srcA + ((size_t)smp * Ca + cg) * HW + off
                                   : a.srcB + ((size_t)smp * a.Cb + (cg - Ca)) * HW + off;
        dma1k(src + lane * 4, dst + c * P + u * 256);
      }
    }
    // the slice: per tile CCH / 2 step-pair rows of 64 floats (CCH / 8 KB)
    constexpr int NWD = 2 * CCH / 8;            // 1-KB pieces
    if (cb < NWD) {
      const int t = cb / (NWD / 2), pc = cb % (NWD / 2);
      const int rem = pc * 256 + lane * 4;      // float of the tile's CCH * 32
      const int spl = rem >> 6, w64 = rem & 63;
      const int ci0 = g * CCH;                  // first channel of the chunk
      const int k32 = ci0 >> 5, cil = ci0 & 31, hh = cil >> 4, sp = ((cil & 15) >> 1) + spl;
      const float* src = a.wpk + (((size_t)(2 * cog + t) * nc32 + k32) * 8 + sp) * 128 + hh * 64 + w64;
      dma1k(src, dst + XCH + t * (WCH / 2) + pc * 256);
    }
  };
  dma_chunk(0, smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // per-lane LDS offsets: A = X[ci = 4 st + (l >> 4)][16 f + (l & 15)];
  // B = the slice's W[co = 64 cog + 16 cb + (l & 15)][ci = 4 st + (l >> 4)]:
  // tile cb >> 1, step-pair row 2 st + (l >> 5), float (16 (cb & 1) + (l & 15)) * 2 + ((l >> 4) & 1)
  const int xoff = (lane >> 4) * P + (lane & 15);
  const int woff = XCH + (cb >> 1) * (WCH / 2) + (lane >> 5) * 64 + (16 * (cb & 1) + (lane & 15)) * 2 +
                   ((lane >> 4) & 1);
  f32x4 acc[PF];
#pragma unroll
  for (int f = 0; f < PF; ++f) acc[f] = f32x4{};
  for (int g = 0; g < nchunk; ++g) {
    const float* sb = smem + (g & 1) * SLOT;
    if (g + 1 < nchunk) dma_chunk(g + 1, smem + ((g + 1) & 1) * SLOT);
#pragma unroll
    for (int st = 0; st < CCH / 4; ++st) {
      const float bw = sb[woff + st * 128];
      const float* xs = sb + st * 4 * P + xoff;
      constexpr int RA = 4;                     // A-fragment read-ahead
      float av[RA + 1];
#pragma unroll
      for (int f = 0; f < RA; ++f) av[f] = xs[16 * f];
#pragma unroll
      for (int f = 0; f < PF; ++f) {
        if (f + RA < PF) av[(f + RA) % (RA + 1)] = xs[16 * (f + RA)];
        acc[f] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[f % (RA + 1)], bw, acc[f], 0, 0, 0);
        if (f + RA < PF) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                      // MFMA
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: lane holds px 16 f + 4 (l >> 4) + i of channel co, + bias
  const int co = cog * 64 + 16 * cb + (lane & 15);
  const float bias = a.bias ? a.bias[co] : 0.f;
#pragma unroll
  for (int f = 0; f < PF; ++f) {
    const int q = pb * (P / 256) + (16 * f) / 256;
    const int smp = q / ups, off = (q - smp * ups) * 256 + (16 * f) % 256 + 4 * (lane >> 4);
    f32x4 v = acc[f] + bias;
    *reinterpret_cast<f32x4*>(a.out + ((size_t)smp * a.Cout + co) * HW + off) = v;
  }
}

template <int P, int CCH>
hipError_t launch_p1(const ConvArgs& a, int B, hipStream_t s) {
  const int HW = a.Wo * a.Wo;
  const int npb = B * HW / P;
  const int nitems = npb * (a.Cout / 64);
  const size_t lds = (size_t)2 * (CCH * P + 64 * CCH) * sizeof(float);
  static std::atomic<unsigned long long> attr{0};
  set_max_lds_once((const void*)conv1x1_kernel<P, CCH>, (int)lds, attr);
  conv1x1_kernel<P, CCH><<<nitems, T1, lds, s>>>(a, HW, npb);
  return hipGetLastError();
}

}  // namespace

// ERTD_CONV1X1=0 keeps the implicit-GEMM kernel for the 1x1 convs, 2 = 8-channel
// chunks, 3 = at every eligible size (A/B)
bool conv1x1_ok(const ConvArgs& a, int act, int B) {
  static const int env = [] {
    return ERTD_KNOB("CONV1X1", 1);
  }();
  if (!env || act != ACT_NONE || a.res || a.ebias || a.gnp) return false;
  const int HW = a.Wo * a.Wo;
  if (a.Cin % 16 || a.Ca % 2 || a.Cout % 64 || HW % 256 || a.Ho != a.Hs || (B * HW) % 512) return false;
  // measured (U2 B=64, same box): faster than the implicit-GEMM kernel at 64x64
  // (u0 skips 90 / 67 / 67 -> 72 / 52 / 52 us), slower at 16x16 with K = 384-512
  // (one 4-wave workgroup per CU: 54 -> 64 us), equal at 32x32 -- taken at >= 64x64
  return HW >= 4096 || env == 3;
}

hipError_t launch_conv1x1(const ConvArgs& a, int B, hipStream_t s) {
  const int HW = a.Wo * a.Wo;
  // 512-px items where they fill the CUs, else 256
  const long long items512 = (long long)B * HW / 512 * (a.Cout / 64);
  static const int env = [] {
    return ERTD_KNOB("CONV1X1", 1);
  }();
  if (env == 2) {
    if (items512 >= device_cu_count()) return launch_p1<512, 8>(a, B, s);
    return launch_p1<256, 8>(a, B, s);
  }
  if (items512 >= device_cu_count()) return launch_p1<512, 16>(a, B, s);
  return launch_p1<256, 16>(a, B, s);
}

}  // namespace unet
}  // namespace ertd
